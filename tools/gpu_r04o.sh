#!/bin/bash
# r04o: f32 WS with 2 producer waves (EOSV_F32_WS=3) vs 4 (=2): conv_check, bitwise stages, A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
EOSV_F32_WS=3 timeout -k 10 240 tests/native/conv_check_prof > gpurun_out/conv_check_f32ws3.log 2>&1
rc=$?; echo "conv_check f32ws3 rc=$rc"; grep -E "FAIL|failures" gpurun_out/conv_check_f32ws3.log | head; [ $rc -ne 0 ] && exit $rc
for W in 0 3; do
  EOSV_F32_WS=$W timeout -k 10 120 python tools/ws_diff.py save /tmp/f32ws3_$W.pt resnet18 f32 > gpurun_out/f32ws_save.log 2>&1 || { tail -5 gpurun_out/f32ws_save.log; exit 1; }
done
echo "== resnet18 f32 ws 0 vs 3"; python tools/ws_diff.py cmp /tmp/f32ws3_0.pt /tmp/f32ws3_3.pt
ARCH=resnet18 DTYPE=f32 LAYERS="5|6|8|10|11|13|15|16|18" SETS="EOSV_F32_WS=2;EOSV_F32_WS=3;EOSV_F32_WS=0;EOSV_F32_WS=2;EOSV_F32_WS=3;EOSV_F32_WS=0" \
  timeout -k 10 900 bash tools/ab_sets.sh
ARCH=resnet50 DTYPE=f32 LAYERS="12|13|25|26|29|43|44|45|48" SETS="EOSV_F32_WS=0;EOSV_F32_WS=3" STEPS=2 timeout -k 10 600 bash tools/ab_sets.sh
