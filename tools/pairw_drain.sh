#!/bin/bash
# the 256-pixel stage-2 pair's race against full drains at two places (profiling build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
for d in 0 1 2 3; do
  echo "== EOSV_PAIRW_NPT2=1 EOSV_PAIRW_DRAIN=$d"
  EOSV_PAIRW_NPT2=1 EOSV_PAIRW_DRAIN=$d timeout -k 10 200 python -u tools/race_modes.py resnet50 bf16 64,130 0,1 4 2>&1 | grep -v amdgpu.ids | grep -v variant
done
