#!/bin/bash
# r05: f32 WS ablations and consumer priority (EOSV_CONV_ABL bits: 64 no epilogue, 32 no MFMA,
# 128 no staging, 512 dispatch only; 2048 / 4096 consumer priority)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
VAR=EOSV_CONV_ABL VALS="0 64 32 128 512 2048 4096" DTYPE=f32 ROUNDS=1 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | tail -24 || exit 1
VAR=EOSV_CONV_ABL VALS="0 2048 4096" DTYPE=f32 ROUNDS=1 timeout -k 10 300 bash tools/ab_env.sh 2>&1 | head -3 || exit 1
echo done
