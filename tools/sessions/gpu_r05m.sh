#!/bin/bash
# r05: f32 WS consumer priority (release variants -DEOSV_F32_PRIO_DEF=1 / 2) against the default
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
LIBS="libeosv.so libeosv_prio1.so libeosv_prio2.so" ROUNDS=3 ARGS="--secondary-dtype none" timeout -k 10 1000 bash tools/ab_release.sh 2>&1 | tail -9 || exit 1
echo done
