#!/bin/bash
# r04d: state of the tree at the start of the round's second session: gpu suite, smoke,
# default bench, rocprofv3 stats of the bench, configs 3-5 in bf16.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
TAG=${TAG:-r04d}
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && { [ $rc -ne 1 ] || [ "$name" != pytest_gpu ]; }; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ -z "$SKIP_PYTEST" ] && run pytest_gpu 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py
run trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o $TAG -- python bench.py --no-cpu-baseline
SPECS="${SPECS:-3 bf16 512;4 bf16 100;5 bf16 20}" timeout -k 10 1200 bash tools/gpu_configs.sh
run layers_r50 300 python bench.py --arch resnet50 --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 3
run layers_r18 300 python bench.py --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 3
