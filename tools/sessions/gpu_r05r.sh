#!/bin/bash
# r05r: the r05 training passes (batch-norm statistics rows ahead and 16-row chunk floor, im2col /
# col2im vectorised, the stem's im2col reused by its weight gradient): GPU training tests, then the
# training bench A/B against libeosv_r04t.so (-DEOSV_TRAIN_R04_DEF=1 -DEOSV_BN_MINROWS=4) twice,
# then a kernel-trace profile of the shipped build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py \
  > gpurun_out/r05r_tests.txt 2>&1 || { tail -30 gpurun_out/r05r_tests.txt; exit 1; }
tail -2 gpurun_out/r05r_tests.txt
for round in 1 2; do
  for L in libeosv.so libeosv_r04t.so; do
    EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/$L timeout -k 10 300 python tools/bench_train.py --steps 10 \
      > gpurun_out/r05r_$L.$round.log 2>&1 || { tail -5 gpurun_out/r05r_$L.$round.log; exit 1; }
    echo "$L round $round: $(tail -1 gpurun_out/r05r_$L.$round.log | grep -o '"clips_per_s": [0-9.]*')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/train -o r05r -- \
  python tools/bench_train.py --steps 5 > gpurun_out/r05r_trace.log 2>&1 || { tail -5 gpurun_out/r05r_trace.log; exit 1; }
echo done
