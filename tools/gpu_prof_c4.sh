#!/bin/bash
# Config-4 shape (R50 14w1s T=32, bf16) under rocprofv3: bench line, kernel trace + stats, PMC
# FETCH/WRITE passes; summarise with: python tools/prof_summary.py $TAG gpurun_out/c4 profiles
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r02c4x}
O=gpurun_out/c4
mkdir -p $O/prof
ARGS="--arch resnet50 --n-way 14 --k-shot 1 --segments 16 --list tests/golden/unreal14.list --dtype bf16 --secondary-dtype none --max-frames 2048 --episodes-per-step 20 --no-cpu-baseline"
timeout -k 10 300 python bench.py $ARGS --steps 3 > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof/trace -o $TAG -- python bench.py $ARGS --steps 3 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/prof/pmc_$C -o $TAG -- python bench.py $ARGS --steps 2 > $O/pmc_$C.log 2>&1 || { tail $O/pmc_$C.log; exit 1; }
done
grep '^{' $O/bench.log | cut -c1-300
