#!/bin/bash
# bf16 fused-stem ablations (EOSV_STEM_ABL, results wrong when set): stem layer time per variant
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in "EOSV_STEM_ABL=0" "EOSV_STEM_ABL=1" "EOSV_STEM_ABL=2" "EOSV_STEM_ABL=4" "EOSV_STEM_ABL=7" "EOSV_STEM_ABL=6" ${EXTRA:-}; do
  env $v timeout -k 10 200 python bench.py --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 2 \
    > gpurun_out/abl_stem.json 2> gpurun_out/abl_stem.err || { tail gpurun_out/abl_stem.err; exit 1; }
  echo "$v $(grep 'layer   0' gpurun_out/abl_stem.err)"
done
