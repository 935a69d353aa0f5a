#!/bin/bash
# Like-for-like A/B of release builds (tools/build_variant.sh): bench.py under each library,
# interleaved ROUNDS times; prints the f32 / bf16 / f32x3 leg values and conv fractions.
#   LIBS="libeosv.so libeosv_f32ws0.so" [ARGS="--arch resnet50"] bash tools/ab_release.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
P=$PWD/embodied-one-shot-video-recognition_amd
for r in $(seq ${ROUNDS:-2}); do
  for L in ${LIBS:?LIBS required}; do
    EOSV_LIBRARY=$P/$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-5} ${ARGS} > gpurun_out/abr_$L.json 2> gpurun_out/abr_$L.err || { tail -5 gpurun_out/abr_$L.err; exit 1; }
    python -c "
import json; d = json.loads([l for l in open('gpurun_out/abr_$L.json') if l.startswith('{')][0])
s = [d] + [d[k] for k in ('secondary', 'secondary_f32x3') if k in d]
print('$L', ' '.join(f\"{x['dtype']} {x['value']} ({x['roofline']['frac']})\" for x in s))"
  done
done
