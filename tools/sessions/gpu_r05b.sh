#!/bin/bash
# r05: stem v5 (native checks, bitwise A/B vs r04, poison), parity subset, training GEMM re-measure,
# per-layer bench of the bf16 leg
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05b}
mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; tail -n ${TAILN:-4} "$O/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP $name rc=$rc"; exit $rc; fi; return $rc; }
step native 300 python -u -m pytest tests/test_gpu_native.py -x -v --timeout 280 --timeout-method thread
grep -E "stem_pool|FAIL" $O/native.log | head -20
step stem_ab 500 python -u -m pytest tests/test_gpu_poison.py -x -v --timeout 450 --timeout-method thread
step parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layers.py -x -v --timeout 300 --timeout-method thread
step train_bench 300 python tools/bench_train.py
step bench 400 python bench.py --no-cpu-baseline --layers --secondary-dtype bf16
grep -E "layer   0|layer   5" $O/bench.log
echo "== A/B stem v5 (bf16)"
VAR=EOSV_STEM_V5 VALS="0 1" DTYPE=bf16 ROUNDS=2 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | tail -22 || exit $?
echo "== A/B f32 register epilogue"
VAR=EOSV_F32_EPD VALS="0 1" DTYPE=f32 ROUNDS=2 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | tail -22 || exit $?
echo done
