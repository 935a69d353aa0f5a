#!/bin/bash
# r05: f32 WS tile without the consumer-loop spills: parity tests, f32 bench with per-layer times
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out/r05j
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 380 --timeout-method thread > gpurun_out/r05j/parity.log 2>&1 || { tail -30 gpurun_out/r05j/parity.log; exit 1; }
tail -1 gpurun_out/r05j/parity.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --dtype f32 --secondary-dtype none --no-cpu-baseline --steps 5 --warmup 1 --layers > gpurun_out/r05j/f32_$i.log 2>&1 || { tail -5 gpurun_out/r05j/f32_$i.log; exit 1; }
  grep -o '"value": [0-9.]*\|"frac": [0-9.]*' gpurun_out/r05j/f32_$i.log | head -2 | tr '\n' ' '; echo
done
grep "layer" gpurun_out/r05j/f32_2.log
echo done
