#!/bin/bash
# C4 (R50 14-way 1-shot, T 32) traffic for all three dtypes (f32x3 had none measured), then the
# C4 f32x3 config line again so that it carries it (>= 20 oracle episodes)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
C4="--arch resnet50 --n-way 14 --k-shot 1 --segments 16 --list tests/golden/unreal14.list --episodes-per-step 40 --max-frames 2048 --config-label 'BASELINE configs[3]'"
TAG=r05_c4 ARGS="$C4" timeout -k 10 900 bash tools/gpu_traffic.sh bf16 f32 f32x3 2>&1 | tail -4 || exit 1
O=gpurun_out/r05c4x3; mkdir -p $O
cp profiles/r05_c4_traffic.json $O/
timeout -k 10 600 python -u tools/bench_configs.py --config 4 --dtype f32x3 --cpu-sec 170 > $O/c4_f32x3.log 2>&1 || { tail -5 $O/c4_f32x3.log; exit 1; }
grep "^{" $O/c4_f32x3.log > $O/c4_f32x3.json
echo done
