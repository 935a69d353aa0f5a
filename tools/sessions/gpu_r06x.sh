#!/bin/bash
# r06 session X: bblock2 (split-conv R18 stage-1 basic block, bblock_bf16.hip) -- native check
# against the CPU reference (in place / out of place, repeats), stage maps bitwise against the
# one-wave-both-convs kernel (libeosv_bb1.so: -DEOSV_BBLOCK2_DEF=0), the bitwise / poison tests,
# then the interleaved release A/B on R18 bf16.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06x; mkdir -p $O
P=$PWD/embodied-one-shot-video-recognition_amd
timeout -k 10 300 tests/native/bneck_check 2 > $O/bneck_check.log 2>&1; rc=$?
cat $O/bneck_check.log; [ $rc = 0 ] || exit 1
for N in resnet18:224:601 resnet18:256:300; do
  for L in libeosv libeosv_bb1; do
    EOSV_LIBRARY=$P/$L.so timeout -k 10 200 python tools/ws_diff.py save $O/$L.pt $N bf16 > $O/save_$L.log 2>&1 || { tail -5 $O/save_$L.log; exit 1; }
  done
  echo "== $N"; timeout -k 10 100 python tools/ws_diff.py cmp $O/libeosv.pt $O/libeosv_bb1.pt || exit 1
done
rm -f $O/*.pt
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_poison.py > $O/poison.log 2>&1 || { tail -15 $O/poison.log; exit 1; }
tail -1 $O/poison.log
ROUNDS=2 LIBS="libeosv_bb1.so libeosv.so" ARGS="--dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh > $O/ab_r18.log 2>&1 || { cat $O/ab_r18.log; exit 1; }
cat $O/ab_r18.log
