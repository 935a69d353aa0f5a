#!/bin/bash
# r06 session Z: bblock2 timing ablations (release variants -DEOSV_BB2_ABL=1 no MFMAs, 2 no fragment
# reads after the first, 4 no phase barriers; results wrong): ms per launch of the two stage-1 blocks
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06z; mkdir -p $O
P=$PWD/embodied-one-shot-video-recognition_amd
for L in libeosv libeosv_abl1 libeosv_abl2 libeosv_abl4 libeosv; do
  EOSV_LIBRARY=$P/$L.so timeout -k 10 200 python bench.py --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 2 > $O/$L.log 2>&1 || { tail -5 $O/$L.log; exit 1; }
  echo "$L $(grep -E 'layer +(1|3):' $O/$L.log | awk '{printf "%s ", $4}')"
done
