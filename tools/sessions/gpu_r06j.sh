#!/bin/bash
# r06 session J: which stage-1 blocks the fused kernels should take -- per-layer times (profiling
# build) for R50 at the C2 shape and R101 at 256 (config 5's shape) under the EOSV_BNECK modes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06j; mkdir -p $O
L=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
run() {  # tag bneck tail args...
  local t=$1 b=$2 tl=$3; shift 3
  EOSV_LIBRARY=$L EOSV_BNECK=$b EOSV_BNECK_TAIL=$tl timeout -k 10 300 python bench.py --dtype bf16 --secondary-dtype none \
    --no-cpu-baseline --layers --steps 3 "$@" > $O/$t.log 2>&1 || { tail -5 $O/$t.log; exit 1; }
  echo "$t $(grep '^{' $O/$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run r50_00 0 0 --arch resnet50
run r50_10 1 0 --arch resnet50
run r50_11 1 1 --arch resnet50
run r50_30 3 0 --arch resnet50
run r50_20 2 0 --arch resnet50
A="--arch resnet101 --n-way 5 --k-shot 5 --segments 32 --res 256 --episodes-per-step 2 --max-frames 2048"
run r101_00 0 0 $A
run r101_10 1 0 $A
run r101_11 1 1 $A
