#!/bin/bash
# tools/race_probe.py with each build VARIANTS="base a ..." (tools/ablib/libeosv_<name>.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
LIB=embodied-one-shot-video-recognition_amd/libeosv.so
cp $LIB /tmp/libeosv_tree.so
for v in $VARIANTS; do
  cp tools/ablib/libeosv_$v.so $LIB
  for A in ${ARCHS:-resnet50}; do
    echo "[$v]"
    timeout -k 10 200 python -u tools/race_probe.py $A ${DTYPE:-bf16} ${REPS:-12} || { cp /tmp/libeosv_tree.so $LIB; exit 1; }
  done
done
cp /tmp/libeosv_tree.so $LIB
