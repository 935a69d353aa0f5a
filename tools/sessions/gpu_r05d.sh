#!/bin/bash
# r05: stem (3-ahead staging) bitwise A/B test + timing A/B + SQ
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_poison.py -x -q --timeout 380 --timeout-method thread 2>&1 | tail -3 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 280 --timeout-method thread 2>&1 | tail -2 || exit $?
echo "== A/B stem v5 (bf16)"
VAR=EOSV_STEM_V5 VALS="0 1" DTYPE=bf16 ROUNDS=2 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | tail -22 | head -6 || exit $?
echo "== SQ bf16"
timeout -k 10 200 bash tools/pmc_sq.sh 2>&1 | grep stem
echo done
