#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_poison.py -x -q -k S2ROWS --timeout 280 --timeout-method thread > gpurun_out/r05g.log 2>&1
grep -E "stage|frame|passed|failed" gpurun_out/r05g.log | head -30
