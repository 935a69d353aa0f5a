#!/bin/bash
# Interleaved A/B/C... of several builds of libeosv.so on the bench: VARIANTS="base a b" names
# tools/ablib/libeosv_<name>.so; two passes in round-robin order.  [ARCH] [DTYPE] [LAYERS=regex]
# [CHECK=1: conv_check with every variant first]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
LIB=embodied-one-shot-video-recognition_amd/libeosv.so
cp $LIB /tmp/libeosv_tree.so
if [ -n "$CHECK" ]; then
  for v in $VARIANTS; do
    cp tools/ablib/libeosv_$v.so $LIB
    timeout -k 10 120 tests/native/conv_check > gpurun_out/ab_multi_check_$v.log 2>&1; rc=$?
    # a numeric mismatch (rc 1) is reported and the A/B goes on; a fault, abort or timeout ends the call
    [ $rc -gt 1 ] && { echo "[$v] conv_check rc=$rc"; cp /tmp/libeosv_tree.so $LIB; exit 1; }
    grep -E "^FAIL" gpurun_out/ab_multi_check_$v.log | head -3 | cut -c1-200
    echo "[$v] $(grep failures gpurun_out/ab_multi_check_$v.log)"
    timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k batch_invariance > gpurun_out/ab_multi_bi_$v.log 2>&1 || tail -3 gpurun_out/ab_multi_bi_$v.log
    echo "[$v] $(tail -1 gpurun_out/ab_multi_bi_$v.log)"
  done
fi
for pass in 1 2; do
  for v in $VARIANTS; do
    cp tools/ablib/libeosv_$v.so $LIB
    timeout -k 10 200 python bench.py --arch ${ARCH:-resnet50} --dtype ${DTYPE:-bf16} --secondary-dtype none --no-cpu-baseline --layers --steps ${STEPS:-3} \
      > gpurun_out/ab_multi.json 2> gpurun_out/ab_multi_$v.err || { tail gpurun_out/ab_multi_$v.err; cp /tmp/libeosv_tree.so $LIB; exit 1; }
    echo "[$v] $(python -c "import json;d=json.load(open('gpurun_out/ab_multi.json'));print(d['value'], d['roofline']['achieved'])")"
    grep -E "layer +(${LAYERS:-3|7|10|13}):" gpurun_out/ab_multi_$v.err | awk '{printf "%s%s ", $3, $4} END {print ""}'
  done
done
cp /tmp/libeosv_tree.so $LIB
