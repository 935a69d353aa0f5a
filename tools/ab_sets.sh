#!/bin/bash
# A/B sets of env assignments on the bench (per-layer times of layers $LAYERS):
# (A/B switches exist only in the profiling build: `make -C embodied-one-shot-video-recognition_amd/csrc prof`)
export EOSV_LIBRARY="${EOSV_LIBRARY:-$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so}"
#   SETS="EOSV_A=1 EOSV_B=2;EOSV_A=0" [DTYPE=bf16] [CHECK=1: run tests/native/conv_check under each set first]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
IFS=';' read -ra sets <<< "${SETS:?SETS required}"
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  if [ -n "$CHECK" ]; then
    env $set timeout -k 10 120 tests/native/conv_check > gpurun_out/ab_sets_check_$i.log 2>&1 || { echo "conv_check failed under [$set]"; grep -E "FAIL|failures" gpurun_out/ab_sets_check_$i.log | head; exit 1; }
  fi
  env $set timeout -k 10 200 python bench.py --arch ${ARCH:-resnet18} --dtype ${DTYPE:-bf16} --secondary-dtype none --no-cpu-baseline --layers --steps ${STEPS:-3} \
    > gpurun_out/ab_sets_$i.json 2> gpurun_out/ab_sets_$i.err || { tail gpurun_out/ab_sets_$i.err; exit 1; }
  echo "[$set] $(python -c "import json;d=json.load(open('gpurun_out/ab_sets_$i.json'));print(d['value'], d['roofline']['achieved'])")"
  grep -E "layer +(${LAYERS:-0|1|5|6|8|9|10|11|13|14|15|16|18|19}):" gpurun_out/ab_sets_$i.err | awk '{printf "%s%s ", $3, $4} END {print ""}'
done
