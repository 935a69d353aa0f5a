#!/bin/bash
# conv_check REPS times with each build VARIANTS="a b ..." (tools/ablib/libeosv_<name>.so): failures per run
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
LIB=embodied-one-shot-video-recognition_amd/libeosv.so
cp $LIB /tmp/libeosv_tree.so
for v in $VARIANTS; do
  cp tools/ablib/libeosv_$v.so $LIB
  for i in $(seq ${REPS:-3}); do
    timeout -k 10 120 tests/native/conv_check > gpurun_out/cm_${v}_$i.log 2>&1; rc=$?
    echo "[$v #$i] rc=$rc $(grep failures gpurun_out/cm_${v}_$i.log)"; grep "^FAIL" gpurun_out/cm_${v}_$i.log | cut -c1-200
    [ $rc -gt 1 ] && { cp /tmp/libeosv_tree.so $LIB; exit 1; }
  done
done
cp /tmp/libeosv_tree.so $LIB
