#!/bin/bash
# per-layer bf16 conv timings (HIP events per launch) of R18 (C2 shape) and R50 (C4 shape)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for A in resnet18 resnet50; do
  timeout -k 10 300 python bench.py --arch $A --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 3 \
    > gpurun_out/layers_$A.json 2> gpurun_out/layers_$A.err || { tail gpurun_out/layers_$A.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/layers_$A.json'));print('$A', d['value'], d['roofline'])"
  grep "layer" gpurun_out/layers_$A.err
done
