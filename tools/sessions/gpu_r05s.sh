#!/bin/bash
# r05s: BN backward's ReLU mask from 1-byte forward masks (EOSV_TRAIN_RELU_MASK) and dx from the
# written residual gradient (EOSV_BN_GIN): GPU training tests, then the training bench A/B
# (libeosv.so with masks = the new default; libeosv_nogin.so with EOSV_TRAIN_RELU_MASK=0 = r05r),
# three interleaved rounds, then a kernel-trace profile of the default
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py \
  > gpurun_out/r05s_tests.txt 2>&1 || { tail -30 gpurun_out/r05s_tests.txt; exit 1; }
tail -2 gpurun_out/r05s_tests.txt
P=$PWD/embodied-one-shot-video-recognition_amd
for round in 1 2 3; do
  EOSV_LIBRARY=$P/libeosv.so timeout -k 10 300 python tools/bench_train.py --steps 10 > gpurun_out/r05s_new.$round.log 2>&1 || { tail -5 gpurun_out/r05s_new.$round.log; exit 1; }
  echo "new round $round: $(tail -1 gpurun_out/r05s_new.$round.log | grep -o '"clips_per_s": [0-9.]*')"
  EOSV_TRAIN_RELU_MASK=0 EOSV_LIBRARY=$P/libeosv_nogin.so timeout -k 10 300 python tools/bench_train.py --steps 10 > gpurun_out/r05s_old.$round.log 2>&1 || { tail -5 gpurun_out/r05s_old.$round.log; exit 1; }
  echo "r05r round $round: $(tail -1 gpurun_out/r05s_old.$round.log | grep -o '"clips_per_s": [0-9.]*')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/train -o r05s -- \
  python tools/bench_train.py --steps 5 > gpurun_out/r05s_trace.log 2>&1 || { tail -5 gpurun_out/r05s_trace.log; exit 1; }
echo done
