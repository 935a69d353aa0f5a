#!/bin/bash
# r05 first GPU pass: the in-tree training GEMMs (tests, training bench, rocprof stats of the
# training step), the pair determinism / poison tests, one headline bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; tail -n ${TAILN:-4} "$O/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP $name rc=$rc"; exit $rc; fi; return $rc; }
step train_tests 500 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread
step det_tests 400 python -u -m pytest tests/test_gpu_parity.py -x -v -k "determinism or batch_invariance" --timeout 300 --timeout-method thread
step poison 300 python -u -m pytest tests/test_gpu_poison.py -x -v --timeout 280 --timeout-method thread
step train_bench 300 python tools/bench_train.py
step train_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train_prof -o t -- python tools/bench_train.py
step bench 400 python bench.py --no-cpu-baseline
echo done
