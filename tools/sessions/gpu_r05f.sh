#!/bin/bash
# r05: stride-2 entry row kernel (s2rows), register-weight row kernels (rowsr), stem staging pairs:
# native check, bitwise A/B vs the kernels they replace, timing A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 280 --timeout-method thread 2>&1 | tail -2 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_poison.py -q --timeout 580 --timeout-method thread > gpurun_out/r05f_poison.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|stage .* differ|frame" gpurun_out/r05f_poison.log | head -40
[ $rc -gt 1 ] && { echo "poison rc=$rc"; exit $rc; }
echo "== A/B s2rows (bf16)"
VAR=EOSV_BF16_S2ROWS VALS="0 1" DTYPE=bf16 ROUNDS=1 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | tail -20 || exit 1
echo "== A/B rowsr (bf16 R18)"
VAR=EOSV_BF16_ROWSR VALS="0 1" DTYPE=bf16 ROUNDS=2 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | tail -22 || exit 1
echo "== A/B rowsr (bf16 R50)"
VAR=EOSV_BF16_ROWSR VALS="0 1" DTYPE=bf16 ARCH=resnet50 ROUNDS=1 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | grep -E "ROWSR|^layer" || exit 1
echo "== A/B rowsr (bf16 R101 256)"
VAR=EOSV_BF16_ROWSR VALS="0 1" DTYPE=bf16 ARCH=resnet101 BENCH_EXTRA="--res 256" ROUNDS=1 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | grep -E "ROWSR|^layer +([0-9]|1[0-9]|2[0-4]):" || exit 1
echo done
