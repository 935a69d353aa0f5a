#!/bin/bash
# r06 session N: packed epilogues in the 1x1 pair kernels (pair1x1r_bf16, pairw_bf16) -- bitwise
# tests, release A/B: r05, this tree without the pair packing (nopairpk), this tree.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_poison.py > $O/poison.log 2>&1 || { tail -15 $O/poison.log; exit 1; }
tail -1 $O/poison.log
ROUNDS=2 LIBS="libeosv_r05.so libeosv_nopairpk.so libeosv.so" ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none" timeout -k 10 900 bash tools/ab_release.sh > $O/ab_r50.log 2>&1 || { cat $O/ab_r50.log; exit 1; }
cat $O/ab_r50.log
ROUNDS=1 LIBS="libeosv_r05.so libeosv_nopairpk.so libeosv.so" ARGS="--arch resnet101 --n-way 5 --k-shot 5 --segments 32 --res 256 --episodes-per-step 2 --max-frames 2048 --dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh > $O/ab_r101.log 2>&1 || { cat $O/ab_r101.log; exit 1; }
cat $O/ab_r101.log
EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so timeout -k 10 300 python bench.py --arch resnet50 --dtype bf16 \
    --secondary-dtype none --no-cpu-baseline --layers --steps 3 > $O/layers_r50.log 2>&1 || { tail -5 $O/layers_r50.log; exit 1; }
grep -E "layer +[0-9]+:" $O/layers_r50.log | head -40
