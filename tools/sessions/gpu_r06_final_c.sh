#!/bin/bash
# r06 final tree, part C (first: the traffic files of this digest land in profiles/ on the box, and
# part A's bench line then carries them): PMC traffic of every config line,
# profiles/r06_c{2,3,4,5}_traffic.json.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
TAG=r06_c2 timeout -k 10 900 bash tools/gpu_traffic.sh f32 bf16 f32x3 2>&1 | tail -4 || exit 1
TAG=r06_c3 SCRIPT=tools/bench_configs.py ARGS="--config 3 --cpu-episodes 0" timeout -k 10 600 bash tools/gpu_traffic.sh bf16 2>&1 | tail -3 || exit 1
C4="--arch resnet50 --n-way 14 --k-shot 1 --segments 16 --list tests/golden/unreal14.list --episodes-per-step 40 --max-frames 2048 --config-label 'BASELINE configs[3]'"
TAG=r06_c4 ARGS="$C4" timeout -k 10 900 bash tools/gpu_traffic.sh bf16 f32 f32x3 2>&1 | tail -4 || exit 1
C5="--arch resnet101 --n-way 5 --k-shot 5 --segments 32 --res 256 --episodes-per-step 8 --max-frames 2048 --config-label 'BASELINE configs[4]'"
TAG=r06_c5 ARGS="$C5" timeout -k 10 600 bash tools/gpu_traffic.sh bf16 2>&1 | tail -3 || exit 1
mkdir -p gpurun_out/r06final && cp profiles/r06_c*_traffic.json gpurun_out/r06final/
echo done_c
