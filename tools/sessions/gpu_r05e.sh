#!/bin/bash
# r05: validate the window-marker traffic pipeline (C2 bf16) and a C4 f32 config line with a
# 20-episode cpu_parity; GEMM tests + training bench after the two-ahead GEMM prefetch
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out/r05e
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q -k "sgemm or conv_forward" --timeout 280 --timeout-method thread 2>&1 | tail -2 || exit $?
timeout -k 10 200 python tools/bench_train.py 2>&1 | grep "^{" || exit $?
TAG=r05e_c2 timeout -k 10 400 bash tools/gpu_traffic.sh bf16 2>&1 | tail -3 || exit $?
timeout -k 10 600 python tools/bench_configs.py --config 4 --dtype f32 --cpu-sec 150 > gpurun_out/r05e/c4_f32.log 2>&1 || { tail -5 gpurun_out/r05e/c4_f32.log; exit 1; }
grep "^{" gpurun_out/r05e/c4_f32.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d.get('cpu_baseline'), d.get('cpu_parity'))"
echo done
