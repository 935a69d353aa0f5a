#!/bin/bash
# r06 session K: what bounds the fused stage-1 kernel -- per-layer times of R50 bf16 (profiling
# build) under EOSV_BNECK_ABL ablations (bneck_bf16.hip: 1 conv1, 2 conv2, 4 conv3/NEXT MFMAs off,
# 8 no HBM reads, 16 no stores, 32 no barriers; results wrong when set).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06k; mkdir -p $O
L=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
for abl in 0 1 2 4 7 8 16 24 32 31 63; do
  EOSV_LIBRARY=$L EOSV_BNECK=1 EOSV_BNECK_TAIL=0 EOSV_BNECK_ABL=$abl timeout -k 10 300 python bench.py --arch resnet50 \
    --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 2 --warmup 1 > $O/abl$abl.log 2>&1 || { tail -5 $O/abl$abl.log; exit 1; }
  echo "abl $abl: $(grep -E 'layer +(1|5):' $O/abl$abl.log | tr -s ' ' | cut -d' ' -f3,4 | paste -sd' ')"
done
