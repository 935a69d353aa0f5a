#!/bin/bash
# pairw NPT 2 under poisoning with the stream synchronised between launches (EOSV_POISON bit 4)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
for m in 5 7 4 1; do
  echo "== mode $m"
  env POISON_MODE=$m timeout -k 10 150 python -u tools/poison_check.py resnet50,resnet101 bf16 64,130 2>&1 | grep -v amdgpu.ids | grep -v "^poison_check"
  rc=${PIPESTATUS[0]}
  [ $rc -gt 1 ] && { echo "rc=$rc: stop"; exit $rc; }
done
exit 0
