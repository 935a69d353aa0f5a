#!/bin/bash
# Full GPU session: gpu tests, smoke, default bench (JSON), rocprof trace+stats of the same
# command, PMC traffic passes.  Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
TAG=${TAG:-r01}
step() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n ${TAILN:-6} "gpurun_out/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP $name rc=$rc"; exit $rc; fi; return $rc; }
[ -z "$SKIP_PYTEST" ] && step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 900 python bench.py
step trace 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o $TAG -- python bench.py --no-cpu-baseline
for C in FETCH_SIZE WRITE_SIZE; do
  step pmc_$C 900 rocprofv3 --pmc $C --output-format csv -d gpurun_out/prof/pmc_$C -o $TAG -- python bench.py --no-cpu-baseline --steps 2
done
echo done
