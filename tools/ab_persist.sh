#!/bin/bash
# r02 experiment record: A/B of a persistent 256x256 bf16 conv selected by
# EOSV_BF16_PERSIST in a build that had it; the variant was not kept, so on the current tree the
# switch is ignored and both arms run the same kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
# 1. regression: the restructured default kernel vs the committed build (R50 bf16, R18 bf16)
DTYPE=bf16 LAYERS="10|11|13|14|15|16|18|19" bash tools/ab_lib.sh || exit 1
# 2. persistent 256x256 on the 1x1s (1) and on every Cout >= 256 conv (2), R50 bf16
EOSV_BF16_PERSIST=1 timeout -k 10 300 tests/native/conv_check > gpurun_out/pc1.log 2>&1 || { grep -E "FAIL|failures" gpurun_out/pc1.log | head; exit 1; }
EOSV_BF16_PERSIST=2 timeout -k 10 300 tests/native/conv_check > gpurun_out/pc2.log 2>&1 || { grep -E "FAIL|failures" gpurun_out/pc2.log | head; exit 1; }
grep failures gpurun_out/pc1.log gpurun_out/pc2.log
for v in 0 1 2 0 1 2; do
  EOSV_BF16_PERSIST=$v timeout -k 10 200 python bench.py --arch resnet50 --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 3 > gpurun_out/pr.json 2> gpurun_out/pr_$v.err || { tail gpurun_out/pr_$v.err; exit 1; }
  echo "[PERSIST=$v] $(python -c "import json;d=json.load(open('gpurun_out/pr.json'));print(d['value'], d['roofline']['frac'])")"
  grep -E "layer +(13|17|24|25|26|28|29|30|45|49):" gpurun_out/pr_$v.err | awk '{printf "%s%s ", $3, $4} END {print ""}'
done
