#!/bin/bash
# A/B two builds of libeosv.so on the bench (interleaved): tools/ablib/libeosv_base.so vs the tree's build.
# [DTYPE=bf16] [LAYERS=regex] [CHECK=1: conv_check with the new build first]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
LIB=embodied-one-shot-video-recognition_amd/libeosv.so
cp $LIB /tmp/libeosv_new.so
if [ -n "$CHECK" ]; then
  timeout -k 10 120 tests/native/conv_check > gpurun_out/ab_lib_check.log 2>&1 || { grep -E "FAIL|failures" gpurun_out/ab_lib_check.log | head; exit 1; }
  grep failures gpurun_out/ab_lib_check.log
fi
for arm in base new base new; do
  if [ $arm = base ]; then cp tools/ablib/libeosv_base.so $LIB; else cp /tmp/libeosv_new.so $LIB; fi
  timeout -k 10 200 python bench.py --arch ${ARCH:-resnet18} --dtype ${DTYPE:-bf16} --secondary-dtype none --no-cpu-baseline --layers --steps ${STEPS:-3} \
    > gpurun_out/ab_lib.json 2> gpurun_out/ab_lib_$arm.err || { tail gpurun_out/ab_lib_$arm.err; cp /tmp/libeosv_new.so $LIB; exit 1; }
  echo "[$arm] $(python -c "import json;d=json.load(open('gpurun_out/ab_lib.json'));print(d['value'], d['roofline']['achieved'])")"
  grep -E "layer +(${LAYERS:-0|1|5|6|8|9|10|11|13|14|15|16|18|19}):" gpurun_out/ab_lib_$arm.err | awk '{printf "%s%s ", $3, $4} END {print ""}'
done
cp /tmp/libeosv_new.so $LIB
