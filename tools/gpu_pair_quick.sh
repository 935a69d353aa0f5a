#!/bin/bash
# fused bottleneck pair: native check + R50 bf16 per-layer timings
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 tests/native/conv_check > gpurun_out/conv_check.log 2>&1; rc=$?
grep -E "pair|failures" gpurun_out/conv_check.log; grep FAIL gpurun_out/conv_check.log
[ $rc -eq 0 ] || { echo "conv_check rc=$rc"; exit 1; }
timeout -k 10 300 python bench.py --arch resnet50 --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 3 \
    > gpurun_out/layers_resnet50.json 2> gpurun_out/layers_resnet50.err || { tail gpurun_out/layers_resnet50.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/layers_resnet50.json'));print('R50', d['value'], d['roofline']['frac'], d['roofline']['per_layer_bound']['frac'])"
grep -E "layer +(1|2|3|6|7|9|10|12|13):" gpurun_out/layers_resnet50.err
