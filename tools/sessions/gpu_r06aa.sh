#!/bin/bash
# r06 session AA: the rolling fragment lead in bblock2 (EOSV_BB2_LEAD) and in the fused bottleneck's
# conv2 (EOSV_BNECK_LEAD), both default on -- native check, stage maps bitwise against the kernels
# without it (libeosv_lead0.so) and against bblock_bf16 (libeosv_bb1.so), release A/B, layer times
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06aa; mkdir -p $O
P=$PWD/embodied-one-shot-video-recognition_amd
timeout -k 10 300 tests/native/bneck_check 2 > $O/bneck_check.log 2>&1; rc=$?
grep -c "^ok" $O/bneck_check.log; grep -E "FAIL|failures" $O/bneck_check.log; [ $rc = 0 ] || exit 1
for N in resnet18:224:601 resnet18:256:300 resnet50:224:601 resnet101:256:300; do
  for L in libeosv libeosv_lead0 libeosv_bb1; do
    EOSV_LIBRARY=$P/$L.so timeout -k 10 200 python tools/ws_diff.py save $O/$L.pt $N bf16 > $O/save_$L.log 2>&1 || { tail -5 $O/save_$L.log; exit 1; }
  done
  echo "== $N vs lead0"; timeout -k 10 100 python tools/ws_diff.py cmp $O/libeosv.pt $O/libeosv_lead0.pt || exit 1
  echo "== $N vs bb1"; timeout -k 10 100 python tools/ws_diff.py cmp $O/libeosv.pt $O/libeosv_bb1.pt | grep -v " 0/" ; true
done
rm -f $O/*.pt
ROUNDS=2 LIBS="libeosv_lead0.so libeosv.so" ARGS="--dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh > $O/ab_r18.log 2>&1 || { cat $O/ab_r18.log; exit 1; }
cat $O/ab_r18.log
ROUNDS=2 LIBS="libeosv_lead0.so libeosv.so" ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none" timeout -k 10 900 bash tools/ab_release.sh > $O/ab_r50.log 2>&1 || { cat $O/ab_r50.log; exit 1; }
cat $O/ab_r50.log
for L in libeosv_lead0 libeosv; do
  EOSV_LIBRARY=$P/$L.so timeout -k 10 200 python bench.py --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 2 > $O/layers_$L.log 2>&1 || { tail -5 $O/layers_$L.log; exit 1; }
  echo "R18 $L $(grep -E 'layer +(1|3):' $O/layers_$L.log | awk '{printf "%s ", $4}')"
  EOSV_LIBRARY=$P/$L.so timeout -k 10 200 python bench.py --arch resnet50 --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 2 > $O/layers50_$L.log 2>&1 || { tail -5 $O/layers50_$L.log; exit 1; }
  echo "R50 $L $(grep -E 'layer +(1|5):' $O/layers50_$L.log | awk '{printf "%s ", $4}')"
done
