#!/bin/bash
# r06 session T: the fused stage-1 kernels without the empty-asm address pins (libeosv_nolb.so,
# bneck_bf16.hip without asm volatile("" : "+v"(lb))) against the shipping build (libeosv_lb.so):
# stage maps bitwise equal, repeated-forward determinism, release A/B on R50 and R101.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06t; mkdir -p $O
P=$PWD/embodied-one-shot-video-recognition_amd
for N in resnet50 resnet50:224:601 resnet101:256:300; do
  for L in lb nolb; do
    EOSV_LIBRARY=$P/libeosv_$L.so timeout -k 10 200 python tools/ws_diff.py save $O/$L.pt $N bf16 > $O/save_$L.log 2>&1 || { tail -5 $O/save_$L.log; exit 1; }
  done
  echo "== $N"; timeout -k 10 100 python tools/ws_diff.py cmp $O/lb.pt $O/nolb.pt || exit 1
done
EOSV_LIBRARY=$P/libeosv_nolb.so timeout -k 10 300 python tools/race_modes.py resnet50 bf16 64,130 0 4 > $O/race.log 2>&1 || { tail -5 $O/race.log; exit 1; }
grep -v amdgpu.ids $O/race.log
ROUNDS=2 LIBS="libeosv_lb.so libeosv_nolb.so" ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none" timeout -k 10 900 bash tools/ab_release.sh > $O/ab_r50.log 2>&1 || { cat $O/ab_r50.log; exit 1; }
cat $O/ab_r50.log
ROUNDS=2 LIBS="libeosv_lb.so libeosv_nolb.so" ARGS="--arch resnet101 --n-way 5 --k-shot 5 --segments 32 --res 256 --episodes-per-step 2 --max-frames 2048 --dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh > $O/ab_r101.log 2>&1 || { cat $O/ab_r101.log; exit 1; }
cat $O/ab_r101.log
