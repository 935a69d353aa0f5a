#!/bin/bash
# r06 session A: the row kernels without inline-asm loads (conv_rows_bf16 / _x3 / _f32) against
# the r05 library: conv_check, stage maps bitwise (R18 / R50 in f32, bf16, f32x3), a release A/B
# of bench.py, then the GPU suite.  Stops at the first crash or timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06a; mkdir -p $O
P=$PWD/embodied-one-shot-video-recognition_amd
step() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; tail -n ${TAILN:-4} "$O/$name.log"; if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; exit $rc; fi; }
step conv_check 240 tests/native/conv_check
for a in resnet18 resnet50; do
  for d in f32 bf16 f32x3; do
    step save_old_${a}_$d 200 env EOSV_LIBRARY=$P/libeosv_r05.so python tools/ws_diff.py save $O/old_${a}_$d.pt $a $d
    step save_new_${a}_$d 200 env EOSV_LIBRARY=$P/libeosv.so python tools/ws_diff.py save $O/new_${a}_$d.pt $a $d
    TAILN=6 step cmp_${a}_$d 100 python tools/ws_diff.py cmp $O/old_${a}_$d.pt $O/new_${a}_$d.pt
  done
done
rm -f $O/*.pt
LIBS="libeosv_r05.so libeosv.so" ROUNDS=2 step ab 900 bash tools/ab_release.sh
TAILN=8 step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
echo done_r06a
