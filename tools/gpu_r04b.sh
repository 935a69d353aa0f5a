#!/bin/bash
# r04b: strip v2 (weights in registers, one barrier per chunk): correctness, then A/B vs off / v1
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
grep strip gpurun_out/conv_check.log
ARCH=resnet18 LAYERS="6|8|9|11|13|14|16|18|19" SETS="EOSV_BF16_STRIP=0;EOSV_BF16_STRIP=1;EOSV_BF16_STRIP=2;EOSV_BF16_STRIP=1 EOSV_STRIP_FORM=1;EOSV_BF16_STRIP=0;EOSV_BF16_STRIP=1;EOSV_BF16_STRIP=2" \
  timeout -k 10 600 bash tools/ab_sets.sh
ARCH=resnet50 LAYERS="16|19|22|29|32|35|38|41|48|51" SETS="EOSV_BF16_STRIP=0;EOSV_BF16_STRIP=1;EOSV_BF16_STRIP=2;EOSV_BF16_STRIP=0;EOSV_BF16_STRIP=1;EOSV_BF16_STRIP=2" \
  timeout -k 10 600 bash tools/ab_sets.sh
