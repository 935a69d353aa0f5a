#!/bin/bash
# r05p: batch-norm pass variants (tools/build_variant.sh): kernel-trace stats of the training bench
# per variant, then the training bench itself, interleaved twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
V="libeosv.so libeosv_bnu1.so libeosv_ew1.so libeosv_ew1m16.so libeosv_ew1m16p2.so libeosv_ew2m16.so"
for L in $V; do
  EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d gpurun_out/prof/bnv -o ${L%.so} -- python tools/bench_train.py --steps 5 \
    > gpurun_out/r05p_trace_$L.log 2>&1 || { tail -5 gpurun_out/r05p_trace_$L.log; exit 1; }
  echo "traced $L"
done
for round in 1 2; do
  for L in $V; do
    EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/$L timeout -k 10 300 python tools/bench_train.py --steps 10 \
      > gpurun_out/r05p_$L.$round.log 2>&1 || { tail -5 gpurun_out/r05p_$L.$round.log; exit 1; }
    echo "$L round $round: $(tail -1 gpurun_out/r05p_$L.$round.log | grep -o '"clips_per_s": [0-9.]*')"
  done
done
echo done
