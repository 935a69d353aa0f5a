#!/bin/bash
# r06 session AB: read-first group schedule in the bf16 WS / tap-shift tiles (libeosv_rfirst.so,
# -DEOSV_BF16_RFIRST=1) against the release build: stage maps bitwise, release A/B on R18 and R50
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06ab; mkdir -p $O
P=$PWD/embodied-one-shot-video-recognition_amd
for N in resnet18:224:301 resnet50:224:301; do
  for L in libeosv libeosv_rfirst; do
    EOSV_LIBRARY=$P/$L.so timeout -k 10 200 python tools/ws_diff.py save $O/$L.pt $N bf16 > $O/save_$L.log 2>&1 || { tail -5 $O/save_$L.log; exit 1; }
  done
  echo "== $N"; timeout -k 10 100 python tools/ws_diff.py cmp $O/libeosv.pt $O/libeosv_rfirst.pt || exit 1
done
rm -f $O/*.pt
ROUNDS=2 LIBS="libeosv.so libeosv_rfirst.so" ARGS="--dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh > $O/ab_r18.log 2>&1 || { cat $O/ab_r18.log; exit 1; }
cat $O/ab_r18.log
ROUNDS=2 LIBS="libeosv.so libeosv_rfirst.so" ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none" timeout -k 10 900 bash tools/ab_release.sh > $O/ab_r50.log 2>&1 || { cat $O/ab_r50.log; exit 1; }
cat $O/ab_r50.log
