#!/bin/bash
# r05: tap-shift tile with the weights two stages ahead (EOSV_BF16_TS_WS=2): bitwise A/B, timing A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_poison.py -q -k TS_WS --timeout 380 --timeout-method thread > gpurun_out/r05k_poison.log 2>&1
rc=$?; tail -3 gpurun_out/r05k_poison.log; [ $rc -ne 0 ] && { grep -E "stage|frame" gpurun_out/r05k_poison.log | head; exit $rc; }
VAR=EOSV_BF16_TS_WS VALS="1 2" DTYPE=bf16 ROUNDS=2 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | tail -22 || exit 1
VAR=EOSV_BF16_TS_WS VALS="1 2" DTYPE=bf16 ARCH=resnet50 ROUNDS=1 timeout -k 10 400 bash tools/ab_env.sh 2>&1 | grep -E "TS_WS|^layer +(1[0-9]|2[0-3]):" || exit 1
echo done
