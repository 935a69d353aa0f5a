#!/bin/bash
# A/B one environment switch of the same build on the bench (interleaved arms 0 1 0 1).
# VAR=<name> [DTYPE=f32] [ARCH=resnet18] [LAYERS=regex] [CHECK=1: conv_check with VAR=1 first]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -n "$CHECK" ]; then
  env $VAR=1 timeout -k 10 300 tests/native/conv_check > gpurun_out/ab_env_check.log 2>&1 || { grep -E "FAIL|failures" gpurun_out/ab_env_check.log | head; exit 1; }
  grep failures gpurun_out/ab_env_check.log
fi
for arm in 0 1 0 1; do
  env $VAR=$arm timeout -k 10 200 python bench.py --arch ${ARCH:-resnet18} --dtype ${DTYPE:-f32} --secondary-dtype none --no-cpu-baseline --layers --steps ${STEPS:-3} \
    > gpurun_out/ab_env.json 2> gpurun_out/ab_env_$arm.err || { tail gpurun_out/ab_env_$arm.err; exit 1; }
  echo "[$VAR=$arm] $(python -c "import json;d=json.load(open('gpurun_out/ab_env.json'));print(d['value'], d['roofline']['achieved'], d['roofline']['frac'])")"
  grep -E "layer +(${LAYERS:-0|1|5|6|8|9|10|11|13|14|15|16|18|19}):" gpurun_out/ab_env_$arm.err | awk '{printf "%s%s ", $3, $4} END {print ""}'
done
