#!/bin/bash
# r04r: stage-1 pair with pixels per wave (EOSV_PAIR_R, profiling build): conv_check, bitwise
# stages of R50 bf16 vs pair1x1_bf16, layer A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
EOSV_PAIR_R=1 timeout -k 10 240 tests/native/conv_check_prof > gpurun_out/conv_check_pr.log 2>&1
rc=$?; echo "conv_check pair_r rc=$rc"; grep -E "FAIL|failures|pair" gpurun_out/conv_check_pr.log | head -12; [ $rc -ne 0 ] && exit $rc
for P in 0 1; do
  EOSV_PAIR_R=$P timeout -k 10 120 python tools/ws_diff.py save /tmp/pr_$P.pt resnet50 > gpurun_out/pr_save.log 2>&1 || { tail -5 gpurun_out/pr_save.log; exit 1; }
done
echo "== resnet50 bf16 pair_r 0 vs 1"; python tools/ws_diff.py cmp /tmp/pr_0.pt /tmp/pr_1.pt
ARCH=resnet50 LAYERS="1|2|3|6|7|9|10" SETS="EOSV_PAIR_R=0;EOSV_PAIR_R=1;EOSV_PAIR_R=0;EOSV_PAIR_R=1" timeout -k 10 600 bash tools/ab_sets.sh
