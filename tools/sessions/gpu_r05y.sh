#!/bin/bash
# r05y: the training convs' split-K sizing (EOSV_KS_WPC 2, EOSV_KS_MIN 32, EOSV_KS_MAX 8) as
# release variants: training bench, three interleaved rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=$PWD/embodied-one-shot-video-recognition_amd
for round in 1 2 3; do
  for L in libeosv.so libeosv_k1.so libeosv_k3.so libeosv_k4.so libeosv_k4m16.so; do
    EOSV_LIBRARY=$P/$L timeout -k 10 300 python tools/bench_train.py --steps 10 > gpurun_out/r05y_$L.$round.log 2>&1 || { tail -5 gpurun_out/r05y_$L.$round.log; exit 1; }
    echo "$L round $round: $(tail -1 gpurun_out/r05y_$L.$round.log | grep -o '"clips_per_s": [0-9.]*')"
  done
done
echo done
