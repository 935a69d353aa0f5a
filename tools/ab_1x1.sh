#!/bin/bash
# r02 experiment record: 128x128 tiles for the R50 bf16 1x1 convs, selected by
# EOSV_BF16_1X1 in a build that had it; not kept, so on the current tree the switch is ignored.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in 0 1 2 0 1 2; do
  EOSV_BF16_1X1=$v timeout -k 10 200 python bench.py --arch resnet50 --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 3 > gpurun_out/ab11.json 2> gpurun_out/ab11_$v.err || { tail gpurun_out/ab11_$v.err; exit 1; }
  echo "[1X1=$v] $(python -c "import json;d=json.load(open('gpurun_out/ab11.json'));print(d['value'], d['roofline']['frac'])")"
  grep -E "layer +(13|15|17|24|26|28|30|43|45|47|49):" gpurun_out/ab11_$v.err | awk '{printf "%s%s ", $3, $4} END {print ""}'
done
