#!/bin/bash
# r06 session O: the r04/r05 "NPT 2 pair race" pinned to the store-data hazard -- repeated plain
# forwards (tools/race_modes.py, mode 0) of R50 / R101 bf16 at 64 and 130 frames per chunk under a
# build without the store guard (14 hazard pairs, the NPT 2 stage-2 pair among them) and under
# the shipping build (0); then the GPU determinism / poison tests and the release A/B of NPT 2.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06o; mkdir -p $O
P=$PWD/embodied-one-shot-video-recognition_amd
for L in libeosv_noguard.so libeosv.so; do
  for A in resnet50 resnet101; do
    EOSV_LIBRARY=$P/$L timeout -k 10 300 python tools/race_modes.py $A bf16 64,130 0 6 > $O/race_${A}_$L.log 2>&1 || { tail -5 $O/race_${A}_$L.log; exit 1; }
    echo "== $L $A"; cat $O/race_${A}_$L.log | tail -6
  done
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py -k "determinism_over_chunk_sizes or batch_invariance" tests/test_gpu_poison.py > $O/tests.log 2>&1 || { tail -15 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ROUNDS=2 LIBS="libeosv_r05.so libeosv_npt1.so libeosv.so" ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none" timeout -k 10 900 bash tools/ab_release.sh > $O/ab_r50.log 2>&1 || { cat $O/ab_r50.log; exit 1; }
cat $O/ab_r50.log
ROUNDS=1 LIBS="libeosv_r05.so libeosv_npt1.so libeosv.so" ARGS="--arch resnet101 --n-way 5 --k-shot 5 --segments 32 --res 256 --episodes-per-step 2 --max-frames 2048 --dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh > $O/ab_r101.log 2>&1 || { cat $O/ab_r101.log; exit 1; }
cat $O/ab_r101.log
