#!/bin/bash
# pairw NPT 2 under poisoning: the chunk-wait rule (EOSV_PAIRW_CS=0: loads only) against the default
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
for m in 1 2 3; do
  for sw in EOSV_PAIRW_CS=0 EOSV_PAIRW_CS=1; do
    echo "== mode $m $sw"
    env POISON_MODE=$m $sw timeout -k 10 120 python -u tools/poison_check.py resnet50,resnet101 bf16 64,130 2>&1 | grep -v amdgpu.ids | grep -v "^poison_check"
    rc=${PIPESTATUS[0]}
    [ $rc -gt 1 ] && { echo "rc=$rc: stop"; exit $rc; }
  done
done
exit 0
