#!/bin/bash
# One GPU session: parity tests, smoke, short bench with per-layer timing.
# Stops at the first step that crashes / times out (exit codes other than 0/1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" ; date
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run pytest_gpu 900 python -m pytest tests -x -q -m gpu
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps 3 --warmup 1 --episodes-per-step 50 --layers --cpu-baseline-sec 10
