#!/bin/bash
# conv_check, then per-layer bf16 timings of R18 (C2 shape) and R50 (C2 episode shape) + bench lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/layers
timeout -k 10 180 tests/native/conv_check > gpurun_out/layers/conv_check.log 2>&1 || { grep -v "^ok" gpurun_out/layers/conv_check.log | tail -20; exit 1; }
grep -c "^ok" gpurun_out/layers/conv_check.log
for A in ${ARCHS:-resnet18 resnet50}; do
  timeout -k 10 200 python bench.py --arch $A --dtype bf16 --secondary-dtype ${SEC:-none} --no-cpu-baseline --layers --steps 3 --episodes-per-step 100 \
    > gpurun_out/layers/$A.json 2> gpurun_out/layers/$A.err || { tail gpurun_out/layers/$A.err; exit 1; }
  python - "$A" <<'PY'
import json, sys
a = sys.argv[1]
d = json.load(open(f"gpurun_out/layers/{a}.json"))
print(a, d["value"], "clips/s", d["roofline"]["achieved"], "TF/s frac", d["roofline"]["frac"], "per-layer", d["roofline"]["per_layer_bound"]["frac"])
for k in [k for k in d if k.startswith("secondary")]:
    s = d[k]; print("  ", s["dtype"], s["value"], s["roofline"]["frac"])
PY
  grep "layer" gpurun_out/layers/$A.err | awk '{printf "%s:%s ", $3, $4} END {print ""}'
done
