#!/bin/bash
# R50 bf16 per-layer times under the profiling build's ablations (EOSV_CONV_ABL: 0 full, 64 no
# epilogue, 1024 no K loop, 512 dispatch only); results are wrong when set, timing only
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
mkdir -p gpurun_out
for v in ${ABLS:-0 64 1024 512}; do
  EOSV_CONV_ABL=$v timeout -k 10 200 python bench.py --arch resnet50 --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 2 > gpurun_out/abl_r50.json 2> gpurun_out/abl_r50_$v.err || { tail gpurun_out/abl_r50_$v.err; exit 1; }
  echo "[ABL=$v] $(grep -E 'layer +(13|15|17|24|26|28|30|43|45|47|49|25|29):' gpurun_out/abl_r50_$v.err | awk '{printf "%s%s ", $3, $4}')"
done
