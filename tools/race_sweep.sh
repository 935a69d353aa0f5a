#!/bin/bash
# One sweep of run-to-run determinism (plain repeats, stream-synchronised repeats, poisoned buffers)
# over archs, dtypes and chunk sizes: tools/race_modes.py
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
set -o pipefail
for a in resnet50 resnet101 resnet18; do
  timeout -k 10 240 python -u tools/race_modes.py $a bf16 1,17,64,130,257,601 0,4,1 3 2>&1 | grep -v amdgpu.ids || exit $?
done
timeout -k 10 240 python -u tools/race_modes.py resnet50 f32x3 17,64,130 0,4,1 3 2>&1 | grep -v amdgpu.ids || exit $?
timeout -k 10 240 python -u tools/race_modes.py resnet18 f32 17,64,130 0,4,1 3 2>&1 | grep -v amdgpu.ids || exit $?
timeout -k 10 200 tests/native/conv_check pairw_stress | tail -1
