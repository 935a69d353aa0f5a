#!/bin/bash
# per-layer f32 conv timings of ResNet-50 (config-4 frame shape)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --arch resnet50 --dtype f32 --secondary-dtype none --no-cpu-baseline --layers --steps 2 --episodes-per-step 60 \
    > gpurun_out/l50f.json 2> gpurun_out/l50f.err || { tail gpurun_out/l50f.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/l50f.json'));print('R50 f32', d['value'], d['roofline']['frac'], d['roofline']['per_layer_bound'])"
grep layer gpurun_out/l50f.err
