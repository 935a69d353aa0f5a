#!/bin/bash
# r04 first session: the pair fixes (wait rule, empty-record prefetch), RCCL at world size 1,
# determinism, and the A/B of the pairw wait counting stores (profiling build).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 12 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run conv_check 180 tests/native/conv_check
run rccl 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_multirank.py -k rccl
run determinism 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "determinism or batch_invariance"
run race_r101 300 python tools/race_probe.py resnet101 bf16 8
ARCH=resnet50 LAYERS="3|7|10|13|17|20|23|30|33|36|39" SETS="EOSV_PAIRW_CS=0;EOSV_PAIRW_CS=1;EOSV_PAIRW_CS=0;EOSV_PAIRW_CS=1" \
  timeout -k 10 600 bash tools/ab_sets.sh
# row-strip 3x3 (conv_strip_bf16) vs the previous kernels: 0 off, 1 W >= 14, 2 also 7x7
ARCH=resnet18 LAYERS="6|8|9|11|13|14|16|18|19" SETS="EOSV_BF16_STRIP=0;EOSV_BF16_STRIP=1;EOSV_BF16_STRIP=2;EOSV_BF16_STRIP=0;EOSV_BF16_STRIP=1;EOSV_BF16_STRIP=2" \
  timeout -k 10 600 bash tools/ab_sets.sh
ARCH=resnet50 LAYERS="16|19|22|29|32|35|38|41|48|51" SETS="EOSV_BF16_STRIP=0;EOSV_BF16_STRIP=1;EOSV_BF16_STRIP=2;EOSV_BF16_STRIP=0;EOSV_BF16_STRIP=1;EOSV_BF16_STRIP=2" \
  timeout -k 10 600 bash tools/ab_sets.sh
