#!/bin/bash
# fused bottleneck pair: native check, R50 parity tests, per-layer bf16 timings
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 tests/native/conv_check > gpurun_out/conv_check.log 2>&1; rc=$?
grep -E "pair|failures" gpurun_out/conv_check.log; grep FAIL gpurun_out/conv_check.log
[ $rc -eq 0 ] || { echo "conv_check rc=$rc"; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_layers.py tests/test_gpu_configs.py > gpurun_out/pytest_pair.log 2>&1 || { tail -30 gpurun_out/pytest_pair.log; exit 1; }
tail -3 gpurun_out/pytest_pair.log
bash tools/layers_bf16.sh
