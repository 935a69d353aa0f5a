#!/bin/bash
# iteration loop: conv_check, per-layer bf16 timings (ARCHS), then a pytest subset (PYK)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
ARCHS=${ARCHS:-resnet50} bash tools/gpu_layers.sh || exit $?
if [ -n "$PYK" ]; then
  timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "$PYK" > gpurun_out/pytest_iter.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_iter.log; exit $rc
fi
