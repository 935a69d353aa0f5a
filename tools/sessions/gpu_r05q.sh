#!/bin/bash
# r05q: batch-norm statistics chunk floor (EOSV_BN_MINROWS 16 in libeosv.so; 4 / 32 / 64 variants;
# bnu1 = the r04 passes): GPU training tests first, then kernel-trace stats of the training bench per
# variant, then the training bench itself, interleaved twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py \
  > gpurun_out/r05q_tests.txt 2>&1 || { tail -30 gpurun_out/r05q_tests.txt; exit 1; }
tail -2 gpurun_out/r05q_tests.txt
V="libeosv.so libeosv_m4.so libeosv_m32.so libeosv_m64.so libeosv_bnu1.so"
for L in $V; do
  EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d gpurun_out/prof/bnv -o ${L%.so} -- python tools/bench_train.py --steps 5 \
    > gpurun_out/r05q_trace_$L.log 2>&1 || { tail -5 gpurun_out/r05q_trace_$L.log; exit 1; }
  echo "traced $L"
done
for round in 1 2; do
  for L in $V; do
    EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/$L timeout -k 10 300 python tools/bench_train.py --steps 10 \
      > gpurun_out/r05q_$L.$round.log 2>&1 || { tail -5 gpurun_out/r05q_$L.$round.log; exit 1; }
    echo "$L round $round: $(tail -1 gpurun_out/r05q_$L.$round.log | grep -o '"clips_per_s": [0-9.]*')"
  done
done
echo done
