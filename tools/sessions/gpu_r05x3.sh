#!/bin/bash
# r05x: BN statistics block target (EOSV_BN_BLOCKS, 2048) and elementwise grid cap (EOSV_BN_EW_GRID, 4096) as
# release variants: training bench, three interleaved rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
P=$PWD/embodied-one-shot-video-recognition_amd
for round in 1 2 3; do
  for L in libeosv.so libeosv_g256.so libeosv_g512.so libeosv_g768.so libeosv_g1k.so; do
    EOSV_LIBRARY=$P/$L timeout -k 10 300 python tools/bench_train.py --steps 10 > gpurun_out/r05x3_$L.$round.log 2>&1 || { tail -5 gpurun_out/r05x3_$L.$round.log; exit 1; }
    echo "$L round $round: $(tail -1 gpurun_out/r05x3_$L.$round.log | grep -o '"clips_per_s": [0-9.]*')"
  done
done
echo done
