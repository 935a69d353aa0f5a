#!/bin/bash
# A/B of the training GEMM knobs on the profiling build (tools/bench_gemm.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
for cfg in "EOSV_GEMM_AHEAD=1 EOSV_GEMM_WPC=8" "EOSV_GEMM_AHEAD=2 EOSV_GEMM_WPC=8" "EOSV_GEMM_AHEAD=2 EOSV_GEMM_WPC=4" "EOSV_GEMM_AHEAD=1 EOSV_GEMM_WPC=16" "EOSV_GEMM_AHEAD=2 EOSV_GEMM_WPC=16"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python tools/bench_gemm.py || exit $?
done
