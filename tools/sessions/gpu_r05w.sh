#!/bin/bash
# r05w: the KxK weight-gradient split target (EOSV_WGRAD_TARGET x CUs workgroups; default 4) as
# release variants: training bench, three interleaved rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=$PWD/embodied-one-shot-video-recognition_amd
for round in 1 2 3; do
  for L in libeosv.so libeosv_wt2.so libeosv_wt8.so libeosv_wt12.so; do
    EOSV_LIBRARY=$P/$L timeout -k 10 300 python tools/bench_train.py --steps 10 > gpurun_out/r05w_$L.$round.log 2>&1 || { tail -5 gpurun_out/r05w_$L.$round.log; exit 1; }
    echo "$L round $round: $(tail -1 gpurun_out/r05w_$L.$round.log | grep -o '"clips_per_s": [0-9.]*')"
  done
done
echo done
