#!/bin/bash
# r06 session I: stage-2 entry pairing restored behind the fused stage 1; layer timings, release A/B
# against r05, SQ counters of the R50 bf16 kernels.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06i; mkdir -p $O
for s in 1 0; do
  EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so EOSV_BNECK=$s EOSV_BNECK_TAIL=$s \
    timeout -k 10 300 python bench.py --arch resnet50 --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 3 > $O/layers_r50_bneck$s.log 2>&1 || { tail -5 $O/layers_r50_bneck$s.log; exit 1; }
done
ROUNDS=2 LIBS="libeosv_r05.so libeosv.so" ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh > $O/ab_r50.log 2>&1 || { cat $O/ab_r50.log; exit 1; }
cat $O/ab_r50.log
BENCH_ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none --no-cpu-baseline --steps 1 --warmup 1" timeout -k 10 200 bash tools/pmc_sq.sh > $O/pmc_sq.log 2>&1; rc=$?
cat $O/pmc_sq.log | head -40
echo "rc=$rc"
