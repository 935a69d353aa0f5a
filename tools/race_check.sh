#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
LIB=embodied-one-shot-video-recognition_amd/libeosv.so
cp $LIB /tmp/tree.so
for v in base fix; do
  cp tools/ablib/libeosv_$v.so $LIB
  timeout -k 10 150 tests/native/conv_check > gpurun_out/rc_$v.log 2>&1; echo "[$v] conv_check rc=$? $(grep -c '^FAIL\|FAIL' gpurun_out/rc_$v.log) $(grep failures gpurun_out/rc_$v.log)"
  grep -i "fail" gpurun_out/rc_$v.log | head -5
  timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "batch_invariance" > gpurun_out/rc_bi_$v.log 2>&1; echo "[$v] batch_invariance rc=$?"; tail -2 gpurun_out/rc_bi_$v.log
done
cp /tmp/tree.so $LIB
