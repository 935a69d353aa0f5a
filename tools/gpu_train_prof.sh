#!/bin/bash
# training step (R50, the reference's batch 6 x 16 frames x 224^2): bench line (+ 1 torch-CPU step
# as the CPU baseline), then rocprofv3 --kernel-trace --stats of the same command
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r03t}
mkdir -p gpurun_out/prof
timeout -k 10 600 python tools/bench_train.py --cpu-steps 1 > gpurun_out/train_bench.log 2>&1 || { tail -5 gpurun_out/train_bench.log; exit 1; }
tail -1 gpurun_out/train_bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/train -o $TAG -- \
  python tools/bench_train.py > gpurun_out/train_trace.log 2>&1 || { tail -5 gpurun_out/train_trace.log; exit 1; }
tail -1 gpurun_out/train_trace.log
