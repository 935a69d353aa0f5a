#!/bin/bash
# r05v: stride-1 1x1 weight gradients on wgrad_f32_kernel (EOSV_TRAIN_WGRAD_1X1=1) vs the split-K
# in-tree GEMM (default): training bench, three interleaved rounds, then a kernel trace of each
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
for round in 1 2 3; do
  for v in 0 1; do
    EOSV_TRAIN_WGRAD_1X1=$v timeout -k 10 300 python tools/bench_train.py --steps 10 > gpurun_out/r05v_$v.$round.log 2>&1 || { tail -5 gpurun_out/r05v_$v.$round.log; exit 1; }
    echo "wgrad_1x1=$v round $round: $(tail -1 gpurun_out/r05v_$v.$round.log | grep -o '"clips_per_s": [0-9.]*')"
  done
done
for v in 0 1; do
  EOSV_TRAIN_WGRAD_1X1=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/train -o r05v_$v -- \
    python tools/bench_train.py --steps 5 > gpurun_out/r05v_trace_$v.log 2>&1 || { tail -5 gpurun_out/r05v_trace_$v.log; exit 1; }
done
echo done
