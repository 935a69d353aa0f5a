#!/bin/bash
# bf16 conv ablations (EOSV_CONV_ABL, results wrong when set): 1 no main-loop DMA, 2 no stores, 16 no ds_reads,
# 32 no MFMAs, 64 no epilogue (conv_bf16_kernel), 256 no epilogue (p8)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in ${VARIANTS:-0 33 49 113 369 1 2}; do
  EOSV_CONV_ABL=$v timeout -k 10 200 python bench.py --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 2 \
    > gpurun_out/abl_p8.json 2> "gpurun_out/abl_p8_$v.err" || exit 1
  echo "ABL=$v $(grep -E "layer +(5|6|8|9|11|13|14|16|18|19):" "gpurun_out/abl_p8_$v.err" | awk '{printf "%s%s ", $3, $4}')"
done
