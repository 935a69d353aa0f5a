#!/bin/bash
# pytest -m gpu + the default bench line; stops at the first crash / timeout
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?; tail -c 3000 gpurun_out/bench.log; exit $rc
