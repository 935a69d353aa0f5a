#!/bin/bash
# Config 3 (aug_seg_T, R50, drop-in TestNetwork): JSON line with roofline + CPU baseline, then a
# rocprofv3 --kernel-trace --stats pass of the same command (no CPU leg) for the per-kernel split.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r02c3}
mkdir -p gpurun_out/prof
timeout -k 10 600 python tools/bench_configs.py --config 3 --dtype bf16 --episodes 128 --cpu-episodes 2 \
  > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
grep "^{" gpurun_out/${TAG}_bench.log
for DT in f32x3 f32; do
  timeout -k 10 600 python tools/bench_configs.py --config 3 --dtype $DT --episodes 64 > gpurun_out/${TAG}_bench_$DT.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_bench_$DT.log; exit 1; }
  grep "^{" gpurun_out/${TAG}_bench_$DT.log
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o $TAG -- \
  python tools/bench_configs.py --config 3 --dtype bf16 --episodes 128 > gpurun_out/${TAG}_trace.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_trace.log; exit 1; }
echo done
