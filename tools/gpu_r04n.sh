#!/bin/bash
# r04n: warp-specialised f32 tiles (EOSV_F32_WS 1 / 2, profiling build): conv_check, bitwise
# stage equality vs conv_f32_dma_kernel (R18 / R50 f32), layer A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
for W in 1 2; do
  EOSV_F32_WS=$W timeout -k 10 240 tests/native/conv_check_prof > gpurun_out/conv_check_f32ws$W.log 2>&1
  rc=$?; echo "conv_check f32ws$W rc=$rc"; grep -E "FAIL|failures" gpurun_out/conv_check_f32ws$W.log | head; [ $rc -ne 0 ] && exit $rc
done
for A in resnet18 resnet50; do
  for W in 0 1 2; do
    EOSV_F32_WS=$W timeout -k 10 120 python tools/ws_diff.py save /tmp/f32ws_${A}_$W.pt $A f32 > gpurun_out/f32ws_save.log 2>&1 || { tail -5 gpurun_out/f32ws_save.log; exit 1; }
  done
  for W in 1 2; do echo "== $A f32 ws 0 vs $W"; python tools/ws_diff.py cmp /tmp/f32ws_${A}_0.pt /tmp/f32ws_${A}_$W.pt; done
done
ARCH=resnet18 DTYPE=f32 LAYERS="5|6|8|10|11|13|15|16|18" SETS="EOSV_F32_WS=0;EOSV_F32_WS=1;EOSV_F32_WS=2;EOSV_F32_WS=0;EOSV_F32_WS=1;EOSV_F32_WS=2" \
  timeout -k 10 900 bash tools/ab_sets.sh
