#!/bin/bash
# GPU-side (rocprofv3) durations of ablated bf16 conv kernels: EOSV_CONV_ABL values in $ABLS
# (A/B switches exist only in the profiling build: `make -C embodied-one-shot-video-recognition_amd/csrc prof`)
export EOSV_LIBRARY="${EOSV_LIBRARY:-$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so}"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for A in ${ABLS:-113}; do
  rm -rf gpurun_out/prof_abl
  mkdir -p gpurun_out/prof_abl
  EOSV_CONV_ABL=$A timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_abl -o run -- python bench.py --dtype bf16 --secondary-dtype none --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/prof_abl/bench.log 2>&1 || { tail -20 gpurun_out/prof_abl/bench.log; exit 1; }
  f=$(find gpurun_out/prof_abl -name "*kernel_stats.csv" | head -1)
  cp "$f" "gpurun_out/prof_abl_$A.csv"
  echo "== ABL=$A"; grep "conv_bf16_kernel<256, 256\|conv_bf16_kernel<128" "gpurun_out/prof_abl_$A.csv" | cut -d, -f1-4 | cut -c1-160
done
