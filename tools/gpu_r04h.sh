#!/bin/bash
# r04h: WS classes (EOSV_BF16_WS bits 1 / 2 / 4) and the f32 K chunk (EOSV_F32_KCM 0 / 32 / 64 / 128):
# conv_check (release defaults, and the profiling build with every WS class), then A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 240 tests/native/conv_check > gpurun_out/conv_check_rel.log 2>&1
rc=$?; echo "conv_check release rc=$rc"; grep -E "FAIL|failures" gpurun_out/conv_check_rel.log | head; [ $rc -ne 0 ] && exit $rc
EOSV_BF16_WS=7 timeout -k 10 240 tests/native/conv_check_prof > gpurun_out/conv_check_ws7.log 2>&1
rc=$?; echo "conv_check ws7 rc=$rc"; grep -E "FAIL|failures" gpurun_out/conv_check_ws7.log | head; [ $rc -ne 0 ] && exit $rc
ARCH=resnet50 LAYERS="12|13|25|26|28|29|42|43|44|45|47|48|49" SETS="EOSV_BF16_WS=1;EOSV_BF16_WS=3;EOSV_BF16_WS=7;EOSV_BF16_WS=1;EOSV_BF16_WS=3;EOSV_BF16_WS=7" \
  timeout -k 10 600 bash tools/ab_sets.sh
ARCH=resnet18 LAYERS="5|6|10|11|13|15|16|18" SETS="EOSV_BF16_WS=1;EOSV_BF16_WS=3;EOSV_BF16_WS=7;EOSV_BF16_WS=1;EOSV_BF16_WS=3;EOSV_BF16_WS=7" \
  timeout -k 10 600 bash tools/ab_sets.sh
ARCH=resnet18 DTYPE=f32 LAYERS="5|6|8|10|11|13|15|16|18" SETS="EOSV_F32_KCM=0;EOSV_F32_KCM=32;EOSV_F32_KCM=64;EOSV_F32_KCM=128;EOSV_F32_KCM=0;EOSV_F32_KCM=32;EOSV_F32_KCM=64;EOSV_F32_KCM=128" \
  timeout -k 10 900 bash tools/ab_sets.sh
