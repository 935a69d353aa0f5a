#!/bin/bash
# bf16 conv ablations (EOSV_CONV_ABL bits: 1 no main-loop loads, 4 no A, 8 no B, 2 no stores).
# (A/B switches exist only in the profiling build: `make -C embodied-one-shot-video-recognition_amd/csrc prof`)
export EOSV_LIBRARY="${EOSV_LIBRARY:-$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so}"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for abl in ${ABLS:-0 1 4 8 2}; do
  EOSV_CONV_ABL=$abl timeout -k 10 300 python bench.py --arch ${ARCH:-resnet18} --dtype bf16 --secondary-dtype none --steps 3 --warmup 1 \
    --no-cpu-baseline --layers > gpurun_out/ablb_$abl.log 2>&1 || { tail gpurun_out/ablb_$abl.log; exit 1; }
  echo "abl $abl: $(grep -o '"achieved": [0-9.]*' gpurun_out/ablb_$abl.log)"
done
paste $(for a in ${ABLS:-0 1 4 8 2}; do echo gpurun_out/ablb_$a.log; done) | grep "^layer" | \
  awk -F'\t' '{printf "%s", substr($1, 1, 10); for (i = 1; i <= NF; ++i) { split($i, f, " "); printf " %7s", f[5] } printf "\n"}'
