#!/bin/bash
# r05: stride-2 entry row kernel: native check, bitwise A/B vs the 512x128 tile, timing A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 280 --timeout-method thread 2>&1 | tail -2 || { grep -E "FAIL" gpurun_out/*.log; exit 1; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_poison.py -x -q --timeout 480 --timeout-method thread > gpurun_out/r05f_poison.log 2>&1 || { grep -E "stage|frame|FAIL|cmp" gpurun_out/r05f_poison.log | head -40; exit 1; }
tail -3 gpurun_out/r05f_poison.log
echo "== A/B s2rows (bf16)"
VAR=EOSV_BF16_S2ROWS VALS="0 1" DTYPE=bf16 ROUNDS=2 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | tail -22 || exit 1
echo done
