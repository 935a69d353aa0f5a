#!/bin/bash
# r04s: the residual c1-64 stage-1 pair on 128-pixel rounds (EOSV_PAIR_R_NPT1, profiling build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
EOSV_PAIR_R_NPT1=1 timeout -k 10 240 tests/native/conv_check_prof > gpurun_out/conv_check_pr1.log 2>&1
rc=$?; echo "conv_check npt1 rc=$rc"; grep -E "FAIL|failures|pair1x1" gpurun_out/conv_check_pr1.log | head; [ $rc -ne 0 ] && exit $rc
ARCH=resnet50 LAYERS="3|6|7|9|10" SETS="EOSV_PAIR_R_NPT1=0;EOSV_PAIR_R_NPT1=1;EOSV_PAIR_R_NPT1=0;EOSV_PAIR_R_NPT1=1" timeout -k 10 600 bash tools/ab_sets.sh
