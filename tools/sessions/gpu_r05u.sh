#!/bin/bash
# r05u: the training convs (workspace, split-K) on the warp-specialised f32 tiles: GPU training
# tests (incl. the bitwise check against conv_f32_dma_kernel), the f32 conv unit tests, then the
# training bench A/B (libeosv.so vs libeosv_wstr0.so = -DEOSV_F32_WS_TRAIN_DEF=0), three
# interleaved rounds, then a kernel-trace profile of the default
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py \
  > gpurun_out/r05u_tests.txt 2>&1 || { tail -30 gpurun_out/r05u_tests.txt; exit 1; }
tail -2 gpurun_out/r05u_tests.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_native.py \
  > gpurun_out/r05u_native.txt 2>&1 || { tail -30 gpurun_out/r05u_native.txt; exit 1; }
tail -1 gpurun_out/r05u_native.txt
P=$PWD/embodied-one-shot-video-recognition_amd
for round in 1 2 3; do
  EOSV_LIBRARY=$P/libeosv.so timeout -k 10 300 python tools/bench_train.py --steps 10 > gpurun_out/r05u_new.$round.log 2>&1 || { tail -5 gpurun_out/r05u_new.$round.log; exit 1; }
  echo "new round $round: $(tail -1 gpurun_out/r05u_new.$round.log | grep -o '"clips_per_s": [0-9.]*')"
  EOSV_LIBRARY=$P/libeosv_wstr0.so timeout -k 10 300 python tools/bench_train.py --steps 10 > gpurun_out/r05u_old.$round.log 2>&1 || { tail -5 gpurun_out/r05u_old.$round.log; exit 1; }
  echo "dma round $round: $(tail -1 gpurun_out/r05u_old.$round.log | grep -o '"clips_per_s": [0-9.]*')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/train -o r05u -- \
  python tools/bench_train.py --steps 5 > gpurun_out/r05u_trace.log 2>&1 || { tail -5 gpurun_out/r05u_trace.log; exit 1; }
echo done
