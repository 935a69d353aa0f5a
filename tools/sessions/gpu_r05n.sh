#!/bin/bash
# r05: bf16 warp-specialised tiles' consumers at priority 1 (release variant) against the default,
# R18 and R50 bf16
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
LIBS="libeosv.so libeosv_bprio1.so" ROUNDS=3 ARGS="--dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh 2>&1 | tail -6 || exit 1
LIBS="libeosv.so libeosv_bprio1.so" ROUNDS=2 ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh 2>&1 | tail -4 || exit 1
echo done
