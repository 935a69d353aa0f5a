#!/bin/bash
# r04l: run-to-run determinism of R50 bf16 at a C4-sized batch (1024 frames), default switches,
# then with the WS tiles off and the stage-2 pair on 128-pixel rounds (profiling build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
for set in "EOSV_BF16_WS=7" "EOSV_BF16_WS=0" "EOSV_PAIRW_NPT2=0"; do
  echo "== $set"
  env $set timeout -k 10 300 python tools/race_probe.py resnet50 bf16 8 1024 > gpurun_out/race_$set.log 2>&1; rc=$?
  cat gpurun_out/race_$set.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
done
