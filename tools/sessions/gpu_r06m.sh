#!/bin/bash
# r06 session M: store guard without sched_barriers (data kept live through the s_nop) -- native
# check, bitwise tests, release A/B against the sched_barrier guard and r05.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 400 tests/native/bneck_check 3 > $O/bneck_check.log 2>&1 || { cat $O/bneck_check.log; exit 1; }
tail -2 $O/bneck_check.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_poison.py -k "bneck or poison" > $O/poison.log 2>&1 || { tail -15 $O/poison.log; exit 1; }
tail -1 $O/poison.log
ROUNDS=2 LIBS="libeosv_r05.so libeosv_sbguard.so libeosv.so" ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none" timeout -k 10 900 bash tools/ab_release.sh > $O/ab_r50.log 2>&1 || { cat $O/ab_r50.log; exit 1; }
cat $O/ab_r50.log
ROUNDS=1 LIBS="libeosv_r05.so libeosv_sbguard.so libeosv.so" ARGS="--arch resnet101 --n-way 5 --k-shot 5 --segments 32 --res 256 --episodes-per-step 2 --max-frames 2048 --dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh > $O/ab_r101.log 2>&1 || { cat $O/ab_r101.log; exit 1; }
cat $O/ab_r101.log
