#!/bin/bash
# r06 session S: bneck_bf16 / bneck_tail_bf16 conv2 with double-buffered B fragments (shared
# conv2_ring) -- native check, bitwise tests, release A/B against the single-buffered form (bb1)
# and r05 on R50 (C2 shape) and R101 (256, config 5's shape).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 400 tests/native/bneck_check 3 > $O/bneck_check.log 2>&1 || { cat $O/bneck_check.log; exit 1; }
tail -2 $O/bneck_check.log
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_poison.py -k "bneck" > $O/tests.log 2>&1 || { tail -25 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ROUNDS=2 LIBS="libeosv_r05.so libeosv_bb1.so libeosv.so" ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none" timeout -k 10 900 bash tools/ab_release.sh > $O/ab_r50.log 2>&1 || { cat $O/ab_r50.log; exit 1; }
cat $O/ab_r50.log
ROUNDS=1 LIBS="libeosv_r05.so libeosv_bb1.so libeosv.so" ARGS="--arch resnet101 --n-way 5 --k-shot 5 --segments 32 --res 256 --episodes-per-step 2 --max-frames 2048 --dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh > $O/ab_r101.log 2>&1 || { cat $O/ab_r101.log; exit 1; }
cat $O/ab_r101.log
