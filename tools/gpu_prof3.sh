#!/bin/bash
# r03 measurement, part A: parity diagnostics (-s), the default bench line, rocprofv3 kernel trace
# + stats of the same command, FETCH_SIZE / WRITE_SIZE passes.  TAG names the profile set.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r03a}
mkdir -p gpurun_out/prof
step() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n ${TAILN:-4} "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; exit $rc; fi; }
if [ -z "$SKIP_PARITY" ]; then
  step parity 600 python -u -m pytest tests -q -s -m gpu --timeout 300 --timeout-method thread \
    -k "wide_fixture or eight_reference or reference_shape or fast_legs or thousand"
  grep -E "^\[" gpurun_out/parity.log > gpurun_out/parity_lines.txt
fi
step bench 600 python bench.py
step trace 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o $TAG -- python bench.py --no-cpu-baseline
for C in FETCH_SIZE WRITE_SIZE; do
  step pmc_$C 600 rocprofv3 --pmc $C --output-format csv -d gpurun_out/prof/pmc_$C -o $TAG -- python bench.py --no-cpu-baseline --steps 2
done
echo done
