#!/bin/bash
# r06 final tree, part A: gpu tests, smoke, default bench (JSON), rocprofv3 kernel trace + stats of
# the same command, per-layer tables (R18 bf16 / f32, R50 bf16), SQ summaries, the training
# fixture test's bound use.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r06final; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; tail -n ${TAILN:-4} "$O/$name.log"; if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; exit $rc; fi; }
step pytest_gpu 1100 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread
step train_margin 300 python -u -m pytest tests/test_gpu_train.py -q -s -k reference_fixture --timeout 250 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
step trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o r06 -- python bench.py --no-cpu-baseline
step layers_r18_bf16 300 python bench.py --dtype bf16 --secondary-dtype none --no-cpu-baseline --steps 3 --warmup 1 --layers
step layers_r18_f32 300 python bench.py --dtype f32 --secondary-dtype none --no-cpu-baseline --steps 3 --warmup 1 --layers
step layers_r50_bf16 300 python bench.py --arch resnet50 --dtype bf16 --secondary-dtype none --no-cpu-baseline --steps 3 --warmup 1 --layers
for A in "resnet18 bf16" "resnet18 f32" "resnet50 bf16"; do
  set -- $A
  BENCH_ARGS="--arch $1 --dtype $2 --secondary-dtype none --no-cpu-baseline --steps 1 --warmup 1" timeout -k 10 200 bash tools/pmc_sq.sh > $O/sq_$1_$2.txt 2>&1 || { echo "sq $A failed"; tail -3 $O/sq_$1_$2.txt; exit 1; }
done
echo done_a
