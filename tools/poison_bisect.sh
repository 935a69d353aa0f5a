#!/bin/bash
# Which kernel reads what it did not write: tools/poison_check.py on the failing R50 bf16 sizes under
# each poison mode (1 buffers, 2 LDS) and with one kernel family switched off at a time.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
mkdir -p gpurun_out
for m in 1 2; do
  for sw in "" EOSV_PAIR_R=0 EOSV_BF16_TS_WS=0 EOSV_BF16_WS=0 EOSV_PAIRW=0 EOSV_PAIR=0 EOSV_BF16_TS=0; do
    echo "== mode $m ${sw:-default}"
    env POISON_MODE=$m $sw timeout -k 10 120 python -u tools/poison_check.py resnet50 bf16 64,130 2>&1 | grep -v amdgpu.ids | grep -v "^poison_check"
    rc=${PIPESTATUS[0]}
    [ $rc -gt 1 ] && { echo "rc=$rc: stop"; exit $rc; }
  done
done
exit 0
