#!/bin/bash
# r06 session H: the native bneck check (CPU reference + repeat launches compared bitwise).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 400 tests/native/bneck_check 4 > $O/bneck_check.log 2>&1; rc=$?
cat $O/bneck_check.log
echo "rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_poison.py -k "bneck or poison" > $O/poison.log 2>&1; rc=$?
tail -15 $O/poison.log
echo "rc=$rc"
[ $rc -eq 0 ] || exit $rc
# layer timings: stage-1 convs of R50 bf16 fused vs the r05 path (profiling build, switch off)
for s in 1 0; do
  EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so EOSV_BNECK=$s EOSV_BNECK_TAIL=$s \
    timeout -k 10 300 python bench.py --arch resnet50 --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 3 > $O/layers_r50_bneck$s.log 2>&1 || { tail -5 $O/layers_r50_bneck$s.log; exit 1; }
done
ROUNDS=2 LIBS="libeosv_r05.so libeosv.so" ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh > $O/ab_r50.log 2>&1; rc=$?
cat $O/ab_r50.log
echo "rc=$rc"
