#!/bin/bash
# per-layer bf16 timings of ResNet-50 (config-4 shape) and ResNet-101 @256 (config-5 shape)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --arch resnet50 --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 2 --episodes-per-step 40 \
  > gpurun_out/l50.json 2> gpurun_out/l50.err || { tail gpurun_out/l50.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/l50.json'));print('R50', d['value'], d['roofline']['achieved'])"
grep "layer" gpurun_out/l50.err | awk '{printf "%s%s/%s ", $3, $4, $6} END {print ""}'
