#!/bin/bash
# r05o: batch-norm passes with 4 rows per lane loaded ahead.  BN tests (torch f64 + bitwise vs the
# one-row loops), then the training bench A/B (release libeosv.so vs libeosv_bnu1.so =
# -DEOSV_BN_UNROLL_DEF=1, since renamed -DEOSV_TRAIN_R04_DEF=1; three interleaved rounds), then a kernel-trace profile of the new tree.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_train.py -k "batchnorm" \
  > gpurun_out/r05o_tests.txt 2>&1 || { tail -30 gpurun_out/r05o_tests.txt; exit 1; }
tail -3 gpurun_out/r05o_tests.txt
for round in 1 2 3; do
  for L in libeosv.so libeosv_bnu1.so; do
    EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/$L timeout -k 10 300 python tools/bench_train.py --steps 10 \
      > gpurun_out/r05o_$L.$round.log 2>&1 || { tail -5 gpurun_out/r05o_$L.$round.log; exit 1; }
    echo "$L round $round: $(tail -1 gpurun_out/r05o_$L.$round.log | cut -c1-200)"
  done
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/train -o r05o -- \
  python tools/bench_train.py > gpurun_out/r05o_trace.log 2>&1 || { tail -5 gpurun_out/r05o_trace.log; exit 1; }
echo done
