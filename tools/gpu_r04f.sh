#!/bin/bash
# r04f: f32 chunk-major K order (EOSV_F32_KCM): conv_check, f32 R18 layer A/B (profiling build),
# FETCH_SIZE of the f32 leg under both orders
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run conv_check 240 tests/native/conv_check
grep -E "kcm1|FAIL" gpurun_out/conv_check.log | grep " f32 " | head -20
ARCH=resnet18 DTYPE=f32 LAYERS="5|6|8|9|10|11|13|14|15|16|18|19" SETS="EOSV_F32_KCM=0;EOSV_F32_KCM=1;EOSV_F32_KCM=0;EOSV_F32_KCM=1" \
  timeout -k 10 900 bash tools/ab_sets.sh
for K in 0 1; do
  EOSV_F32_KCM=$K EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/kcm_fetch_$K -o t -- \
    python bench.py --secondary-dtype none --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/kcm_fetch_$K.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/kcm_fetch_$K.log; exit 1; }
done
python tools/pmc_kernels.py $(find gpurun_out/kcm_fetch_0 gpurun_out/kcm_fetch_1 -name "*counter_collection.csv") 2>&1
