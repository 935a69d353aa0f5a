#!/bin/bash
# r04c: stage-2 wide pair on 256-pixel rounds (NPT 2): correctness, determinism, A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run conv_check 180 tests/native/conv_check
grep pairw gpurun_out/conv_check.log
run determinism 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "determinism or batch_invariance"
ARCH=resnet50 LAYERS="3|7|10|13|17|20|23|30|33|36|39" SETS="EOSV_PAIRW_NPT2=0;EOSV_PAIRW_NPT2=1;EOSV_PAIRW_NPT2=0;EOSV_PAIRW_NPT2=1" \
  timeout -k 10 600 bash tools/ab_sets.sh
