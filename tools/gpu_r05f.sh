#!/bin/bash
# r05: stride-2 entry row kernel (s2rows) and the register-weight stage-1 row kernel (rowsr):
# native check, bitwise A/B vs the kernels they replace, timing A/B; f32 WS and bf16 ablations
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 280 --timeout-method thread 2>&1 | tail -2 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_poison.py -q --timeout 480 --timeout-method thread > gpurun_out/r05f_poison.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|stage .* differ|frame" gpurun_out/r05f_poison.log | head -40
[ $rc -gt 1 ] && { echo "poison rc=$rc"; exit $rc; }
echo "== A/B s2rows (bf16)"
VAR=EOSV_BF16_S2ROWS VALS="0 1" DTYPE=bf16 ROUNDS=2 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | tail -22 || exit 1
echo "== A/B rowsr (bf16 R18)"
VAR=EOSV_BF16_ROWSR VALS="0 1" DTYPE=bf16 ROUNDS=2 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | tail -22 || exit 1
echo "== A/B rowsr (bf16 R50)"
VAR=EOSV_BF16_ROWSR VALS="0 1" DTYPE=bf16 ARCH=resnet50 ROUNDS=1 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | grep -E "ROWSR|layer +[0-9]:" || exit 1
echo "== f32 WS ablations (64 no epilogue, 32 no MFMA, 128 no staging, 512 dispatch only; 2048 / 4096 consumer priority)"
VAR=EOSV_CONV_ABL VALS="0 64 32 128 512 2048 4096" DTYPE=f32 ROUNDS=1 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | tail -24 || exit 1
echo done
