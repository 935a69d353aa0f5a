#!/bin/bash
# f32x3 split-bf16 stem: native checks + f32x3 parity tests, then stem A/B (EOSV_X3_STEM)
# (A/B switches exist only in the profiling build: `make -C embodied-one-shot-video-recognition_amd/csrc prof`)
export EOSV_LIBRARY="${EOSV_LIBRARY:-$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so}"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 120 tests/native/conv_check > gpurun_out/conv_check.log 2>&1; rc=$?
grep -E "stem_pool|failures" gpurun_out/conv_check.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread \
  -k "f32x3 or bf16" > gpurun_out/ab_x3s_tests.log 2>&1 || { tail -30 gpurun_out/ab_x3s_tests.log; exit 1; }
tail -2 gpurun_out/ab_x3s_tests.log
for v in 0 1; do
  EOSV_X3_STEM=$v timeout -k 10 200 python bench.py --dtype f32x3 --secondary-dtype none --no-cpu-baseline --layers --steps 2 \
    > gpurun_out/ab_x3s_$v.json 2> gpurun_out/ab_x3s_$v.err || exit 1
  echo "X3_STEM=$v $(python -c "import json;d=json.load(open('gpurun_out/ab_x3s_$v.json'));print(d['value'], d['roofline']['achieved'])") $(grep 'layer   0' gpurun_out/ab_x3s_$v.err)"
done
