#!/bin/bash
# rocprofv3 kernel-trace + stats of the default bench command, then separate PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
TAG=${1:-r01}
BENCH_ARGS=${BENCH_ARGS:-"--no-cpu-baseline"}
set -o pipefail
echo "== trace"; date
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o $TAG -- \
  python bench.py $BENCH_ARGS > gpurun_out/prof/trace_bench.log 2>&1 || { echo "trace rc=$?"; tail -20 gpurun_out/prof/trace_bench.log; exit 1; }
tail -3 gpurun_out/prof/trace_bench.log
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $C"; date
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d gpurun_out/prof/pmc_$C -o $TAG -- \
    python bench.py --steps 1 --warmup 1 --episodes-per-step 20 --no-cpu-baseline > gpurun_out/prof/pmc_$C.log 2>&1 || { echo "pmc rc=$?"; tail -20 gpurun_out/prof/pmc_$C.log; exit 1; }
done
find gpurun_out/prof -name "*.csv" | head -20
