#!/bin/bash
# r06 session L: packed epilogues in the fused stage-1 kernels -- native check, bitwise tests,
# per-layer times, release A/B against r05 (R50 at the C2 shape and R101 at config 5's shape).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 400 tests/native/bneck_check 3 > $O/bneck_check.log 2>&1 || { cat $O/bneck_check.log; exit 1; }
tail -2 $O/bneck_check.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_poison.py -k "bneck or poison" > $O/poison.log 2>&1 || { tail -15 $O/poison.log; exit 1; }
tail -1 $O/poison.log
L=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
for s in 1 0; do
  EOSV_LIBRARY=$L EOSV_BNECK=$s EOSV_BNECK_TAIL=$s timeout -k 10 300 python bench.py --arch resnet50 --dtype bf16 \
    --secondary-dtype none --no-cpu-baseline --layers --steps 3 > $O/layers_r50_$s.log 2>&1 || { tail -5 $O/layers_r50_$s.log; exit 1; }
  echo "r50 bneck=$s: $(grep -E 'layer +(1|2|3|5|6|7|9|10):' $O/layers_r50_$s.log | tr -s ' ' | cut -d' ' -f3,4 | paste -sd' ')"
done
ROUNDS=2 LIBS="libeosv_r05.so libeosv.so" ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh > $O/ab_r50.log 2>&1 || { cat $O/ab_r50.log; exit 1; }
cat $O/ab_r50.log
ROUNDS=1 LIBS="libeosv_r05.so libeosv.so" ARGS="--arch resnet101 --n-way 5 --k-shot 5 --segments 32 --res 256 --episodes-per-step 2 --max-frames 2048 --dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh > $O/ab_r101.log 2>&1 || { cat $O/ab_r101.log; exit 1; }
cat $O/ab_r101.log
