#!/bin/bash
# A/B an environment switch on the bench: VAR=<env var> VALS="<v1> <v2> ..." [DTYPE=bf16] [ARCH=resnet18]
# (A/B switches exist only in the profiling build: `make -C embodied-one-shot-video-recognition_amd/csrc prof`)
export EOSV_LIBRARY="${EOSV_LIBRARY:-$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so}"
# [ROUNDS=2] [BENCH_EXTRA=...]. Interleaved rounds; per-layer timings of the last round printed side by side.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
VAR=${VAR:?VAR required}
VALS=${VALS:?VALS required}
DTYPE=${DTYPE:-bf16}
ARCH=${ARCH:-resnet18}
for round in $(seq ${ROUNDS:-2}); do
  for v in $VALS; do
    log=gpurun_out/ab_${VAR}_$v.log
    env "$VAR=$v" timeout -k 10 300 python bench.py --arch $ARCH --dtype $DTYPE --secondary-dtype none --steps 3 --warmup 1 \
      --no-cpu-baseline --layers ${BENCH_EXTRA:-} > $log 2>&1 || { echo "bench $VAR=$v failed"; tail $log; exit 1; }
    echo "$VAR=$v: $(grep -o '"value": [0-9.]*' $log) $(grep -o '"achieved": [0-9.]*' $log) $(grep -o '"episode_acc": [0-9.]*' $log)"
  done
done
set -- $VALS
paste $(for v in $VALS; do echo gpurun_out/ab_${VAR}_$v.log; done) 2>/dev/null | grep "] layer" | \
  awk -F'\t' '{split($1, h, " "); printf "layer %3s", h[3]; for (i = 1; i <= NF; ++i) { split($i, f, " "); printf "  %8s ms %8s TF", f[4], f[6] } printf "\n"}'
