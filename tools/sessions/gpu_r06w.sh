#!/bin/bash
# r06 session W: fragment-read lead in three bf16 kernels (release variants, tools/build_variant.sh):
#   fd3    pairw_bf16 NPT 1 with two fragment groups read ahead (EOSV_PAIRW_FD=3)
#   bearly conv_bf16_ws / conv_bf16_ts_ws read the next slice's / tap's B fragments behind the
#          MFMAs of the last group (EOSV_BF16_WS_BEARLY=1, EOSV_BF16_TS_BEARLY=1)
#   all3   both
# Stage maps bitwise against the release build (R50, R18, R101 at 256), then interleaved release A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06w; mkdir -p $O
P=$PWD/embodied-one-shot-video-recognition_amd
for N in resnet50 resnet18 resnet101:256:40; do
  for L in libeosv libeosv_all3; do
    EOSV_LIBRARY=$P/$L.so timeout -k 10 200 python tools/ws_diff.py save $O/$L.pt $N bf16 > $O/save_$L.log 2>&1 || { tail -5 $O/save_$L.log; exit 1; }
  done
  echo "== $N"; timeout -k 10 100 python tools/ws_diff.py cmp $O/libeosv.pt $O/libeosv_all3.pt || exit 1
done
ROUNDS=2 LIBS="libeosv.so libeosv_fd3.so libeosv_bearly.so libeosv_all3.so" ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none" timeout -k 10 900 bash tools/ab_release.sh > $O/ab_r50.log 2>&1 || { cat $O/ab_r50.log; exit 1; }
cat $O/ab_r50.log
ROUNDS=2 LIBS="libeosv.so libeosv_bearly.so" ARGS="--dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh > $O/ab_r18.log 2>&1 || { cat $O/ab_r18.log; exit 1; }
cat $O/ab_r18.log
