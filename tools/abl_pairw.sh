#!/bin/bash
# R50 bf16 per-layer times of the wide pairs (pairw_bf16) under the profiling build's ablations
# (EOSV_CONV_ABL bits: 1 no weight DMA, 2 no residual loads, 4 no Y stores, 8 no MFMAs, 16 no
# chunk barriers, 32 no Z stores, 64 no X loads; results are wrong when set, timing only).  The
# bits also reach the conv kernels' own ablations, so only the pair layers are printed.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
mkdir -p gpurun_out
for v in ${ABLS:-0 1 2 4 8 16 32 64 38 103 111}; do
  EOSV_CONV_ABL=$v timeout -k 10 200 python bench.py --arch resnet50 --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 2 > gpurun_out/abl_pairw.json 2> gpurun_out/abl_pairw_$v.err || { tail gpurun_out/abl_pairw_$v.err; exit 1; }
  echo "[ABL=$v] $(grep -E 'layer +(13|17|20|23|30|33|36):' gpurun_out/abl_pairw_$v.err | awk '{printf "%s%s ", $3, $4}')"
done
