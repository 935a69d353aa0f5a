#!/bin/bash
# A/B conv implementations (EOSV_CONV_IMPL) on the default bench, interleaved rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
IMPLS=${IMPLS:-"1 2"}
ROUNDS=${ROUNDS:-2}
for impl in $IMPLS; do
  EOSV_CONV_IMPL=$impl timeout -k 10 120 ./tests/native/conv_check > gpurun_out/cc_$impl.log 2>&1 || { echo "conv_check impl $impl FAILED"; tail gpurun_out/cc_$impl.log; exit 1; }
done
echo "conv_check ok for $IMPLS"
for r in $(seq $ROUNDS); do
for impl in $IMPLS; do
  EOSV_CONV_IMPL=$impl timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --layers ${BENCH_EXTRA:-} > gpurun_out/ab_$impl.log 2>&1 || { echo "bench impl $impl failed"; tail gpurun_out/ab_$impl.log; exit 1; }
  echo "impl $impl: $(grep -o '"value": [0-9.]*' gpurun_out/ab_$impl.log) $(grep -o '"achieved": [0-9.]*' gpurun_out/ab_$impl.log)"
done
done
for impl in $IMPLS; do echo "-- impl $impl"; grep layer gpurun_out/ab_$impl.log | head -8; done
