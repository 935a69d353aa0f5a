#!/bin/bash
# C4 traffic for all three dtypes on the current digest (part C's C4 line before it named f32x3)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
C4="--arch resnet50 --n-way 14 --k-shot 1 --segments 16 --list tests/golden/unreal14.list --episodes-per-step 40 --max-frames 2048 --config-label 'BASELINE configs[3]'"
TAG=r05_c4 ARGS="$C4" timeout -k 10 900 bash tools/gpu_traffic.sh bf16 f32 f32x3 2>&1 | tail -4 || exit 1
mkdir -p gpurun_out/r05c4t && cp profiles/r05_c4_traffic.json gpurun_out/r05c4t/
echo done
