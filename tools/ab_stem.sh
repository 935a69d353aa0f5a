#!/bin/bash
# bf16 stem: column-blocked vs full-width workgroups (EOSV_STEM_CB) + stem / bf16 parity tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_native.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread \
  -k "conv_check or bf16 or batch_invariance" > gpurun_out/ab_stem_tests.log 2>&1 || { tail -30 gpurun_out/ab_stem_tests.log; exit 1; }
tail -2 gpurun_out/ab_stem_tests.log
for cb in 0 1; do
  EOSV_STEM_CB=$cb timeout -k 10 200 python bench.py --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 3 \
    > gpurun_out/ab_stem_cb$cb.json 2> gpurun_out/ab_stem_cb$cb.err || exit 1
  echo "CB=$cb $(python -c "import json;d=json.load(open('gpurun_out/ab_stem_cb$cb.json'));print(d['value'], d['roofline']['achieved'])") $(grep 'layer   0' gpurun_out/ab_stem_cb$cb.err)"
done
