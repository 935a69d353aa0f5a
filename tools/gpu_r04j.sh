#!/bin/bash
# r04j (final tree, stem staging two ahead): final-tree PMC: like-for-like conv-family traffic for config 2 (f32 / bf16 / f32x3, one
# dtype per pass pair) and configs 3 / 4 / 5 (bf16), then SQ counter summaries of R50 and R18 bf16.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
TAG=r04j_c2 timeout -k 10 600 bash tools/gpu_traffic.sh f32 bf16 f32x3 || exit 1
TAG=r04j_c3 SCRIPT=tools/bench_configs.py ARGS="--config 3 --episodes 64 --cpu-episodes 0" timeout -k 10 400 bash tools/gpu_traffic.sh bf16 || exit 1
TAG=r04j_c4 ARGS="--arch resnet50 --n-way 14 --k-shot 1 --segments 16 --list tests/golden/unreal14.list --episodes-per-step 20 --max-frames 2048 --config-label 'BASELINE configs[3]'" \
  timeout -k 10 400 bash tools/gpu_traffic.sh bf16 || exit 1
TAG=r04j_c5 ARGS="--arch resnet101 --n-way 5 --k-shot 5 --segments 32 --res 256 --episodes-per-step 4 --max-frames 2048 --config-label 'BASELINE configs[4]'" \
  timeout -k 10 400 bash tools/gpu_traffic.sh bf16 || exit 1
BENCH_ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none --no-cpu-baseline --steps 1 --warmup 1" timeout -k 10 200 bash tools/pmc_sq.sh > gpurun_out/sq_j_r50_bf16.txt 2>&1 || exit 1
BENCH_ARGS="--dtype bf16 --secondary-dtype none --no-cpu-baseline --steps 1 --warmup 1" timeout -k 10 200 bash tools/pmc_sq.sh > gpurun_out/sq_j_r18_bf16.txt 2>&1 || exit 1
BENCH_ARGS="--secondary-dtype none --no-cpu-baseline --steps 1 --warmup 1" timeout -k 10 200 bash tools/pmc_sq.sh > gpurun_out/sq_j_r18_f32.txt 2>&1 || exit 1
head -12 gpurun_out/sq_j_r50_bf16.txt; head -8 gpurun_out/sq_j_r18_f32.txt
