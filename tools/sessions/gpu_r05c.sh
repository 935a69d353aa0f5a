#!/bin/bash
# r05: stem A/B (r04 vs r05) + SQ counters of the bf16 leg
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
echo "== A/B stem v5 (bf16)"
VAR=EOSV_STEM_V5 VALS="0 1" DTYPE=bf16 ROUNDS=2 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | tail -22 | head -6 || exit $?
echo "== SQ bf16"
timeout -k 10 200 bash tools/pmc_sq.sh 2>&1 | tail -12
echo done
