#!/bin/bash
# r04g: warp-specialised 256x256 bf16 tile (EOSV_BF16_WS=1 one ring, 2 split rings; profiling
# build): conv_check under each, then R50 / R18 layer A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for WS in 1 2; do
  EOSV_BF16_WS=$WS timeout -k 10 240 tests/native/conv_check_prof > gpurun_out/conv_check_ws$WS.log 2>&1
  rc=$?; echo "conv_check ws$WS rc=$rc"; grep -E "FAIL|failures" gpurun_out/conv_check_ws$WS.log | head -20
  [ $rc -ne 0 ] && exit $rc
done
ARCH=resnet50 LAYERS="16|19|22|29|32|35|38|41|48|51" SETS="EOSV_BF16_WS=0;EOSV_BF16_WS=1;EOSV_BF16_WS=2;EOSV_BF16_WS=0;EOSV_BF16_WS=1;EOSV_BF16_WS=2" \
  timeout -k 10 600 bash tools/ab_sets.sh
ARCH=resnet18 LAYERS="13|14|16|18|19" SETS="EOSV_BF16_WS=0;EOSV_BF16_WS=1;EOSV_BF16_WS=2;EOSV_BF16_WS=0;EOSV_BF16_WS=1;EOSV_BF16_WS=2" \
  timeout -k 10 600 bash tools/ab_sets.sh
