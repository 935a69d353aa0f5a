#!/bin/bash
# every fused pair run twice inside the backbone (EOSV_POISON=8, profiling build): do its outputs differ?
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
for npt in 1 0; do
  echo "== EOSV_PAIRW_NPT2=$npt"
  EOSV_PAIRW_NPT2=$npt timeout -k 10 200 python -u tools/race_modes.py resnet50 bf16 64,130 8 2 2>&1 | grep -v amdgpu.ids | grep -v "differs 0 (first px -1 ch -1), z 0" | head -40
done
