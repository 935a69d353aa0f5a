#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
set -o pipefail
timeout -k 10 200 python -u tools/race_modes.py resnet50 bf16 64,130,257 0,4,1 4 2>&1 | grep -v amdgpu.ids || exit $?
timeout -k 10 200 python -u tools/race_modes.py resnet50 bf16 64,130 0,4,1 4 2>&1 | grep -v amdgpu.ids
