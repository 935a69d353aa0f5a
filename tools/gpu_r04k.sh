#!/bin/bash
# r04k: bisect the C4 bf16 embedding error (test_shaped_baseline_fast_legs[c4 bf16]) over the r04
# switches (profiling build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T='tests/test_gpu_configs.py::test_shaped_baseline_fast_legs[c4_r50_14w1s_t32_seed7-bf16]'
one() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 200 python -u -m pytest -x -q --timeout 180 --timeout-method thread "$T" > gpurun_out/bis_$label.log 2>&1
  echo "$label rc=$? $(grep -o 'assert [0-9.e-]* < 0.01' gpurun_out/bis_$label.log | head -1)"
}
one release
P=EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
one prof_default $P
one ws0 $P EOSV_BF16_WS=0
one npt1 $P EOSV_PAIRW_NPT2=0
one ws0_npt1 $P EOSV_BF16_WS=0 EOSV_PAIRW_NPT2=0
one nopairw $P EOSV_PAIRW=0
