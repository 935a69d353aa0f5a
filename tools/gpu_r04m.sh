#!/bin/bash
# r04m: warp-specialised tap-shift tile (EOSV_BF16_TS_WS, profiling build): conv_check, bitwise
# equality of the R18 / R50 stage outputs against the plain tap-shift kernel, layer A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
EOSV_BF16_TS_WS=1 timeout -k 10 240 tests/native/conv_check_prof > gpurun_out/conv_check_tsws.log 2>&1
rc=$?; echo "conv_check tsws rc=$rc"; grep -E "FAIL|failures" gpurun_out/conv_check_tsws.log | head; [ $rc -ne 0 ] && exit $rc
for A in resnet18 resnet50; do
  for T in 0 1; do
    EOSV_BF16_TS_WS=$T timeout -k 10 120 python tools/ws_diff.py save /tmp/tsws_${A}_$T.pt $A > gpurun_out/tsws_save.log 2>&1 || { tail -5 gpurun_out/tsws_save.log; exit 1; }
  done
  echo "== $A ts_ws 0 vs 1"; python tools/ws_diff.py cmp /tmp/tsws_${A}_0.pt /tmp/tsws_${A}_1.pt
done
ARCH=resnet18 LAYERS="5|6|8|9" SETS="EOSV_BF16_TS_WS=0;EOSV_BF16_TS_WS=1;EOSV_BF16_TS_WS=0;EOSV_BF16_TS_WS=1" timeout -k 10 600 bash tools/ab_sets.sh
ARCH=resnet50 LAYERS="12|16|19|22" SETS="EOSV_BF16_TS_WS=0;EOSV_BF16_TS_WS=1;EOSV_BF16_TS_WS=0;EOSV_BF16_TS_WS=1" timeout -k 10 600 bash tools/ab_sets.sh
