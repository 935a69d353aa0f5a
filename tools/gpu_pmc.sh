#!/bin/bash
# PMC counter passes (one counter group per pass) on a small bench run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
TAG=${TAG:-pmc}
ARGS=${BENCH_ARGS:-"--steps 1 --warmup 1 --episodes-per-step 20 --no-cpu-baseline"}
i=0
for GROUP in "$@"; do
  i=$((i+1))
  echo "== pass $i: $GROUP"
  timeout -k 10 600 rocprofv3 --pmc $GROUP --output-format csv -d gpurun_out/pmc/p$i -o $TAG -- \
    python bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
done
