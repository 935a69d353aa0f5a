#!/bin/bash
# p8 pipeline A/B (EOSV_P8_PIPE / EOSV_P8_PRIO / EOSV_BF16_P8) after the conv checks + bf16 parity tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_native.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread \
  -k "conv_check or bf16 or batch_invariance or f32x3" > gpurun_out/ab_p8_tests.log 2>&1 || { tail -30 gpurun_out/ab_p8_tests.log; exit 1; }
tail -2 gpurun_out/ab_p8_tests.log
for v in "EOSV_P8_PIPE=0 EOSV_P8_PRIO=0" "EOSV_P8_PIPE=1 EOSV_P8_PRIO=0" "EOSV_P8_PIPE=0 EOSV_P8_PRIO=1" "EOSV_P8_PIPE=1 EOSV_P8_PRIO=1" "EOSV_BF16_P8=2" ${EXTRA:-}; do
  env $v timeout -k 10 200 python bench.py --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 3 \
    > gpurun_out/ab_p8.json 2> "gpurun_out/ab_p8_$v.err" || exit 1
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/ab_p8.json'));print(d['value'], d['roofline']['achieved'])")"
  grep -E "layer +(5|6|8|9|11|13|14|16|18|19):" "gpurun_out/ab_p8_$v.err" | awk '{printf "%s%s ", $3, $4} END {print ""}'
done
