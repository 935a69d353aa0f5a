#!/bin/bash
# bench.py --max-frames A/B for the f32 headline (r04: 3200 / 4096 / 8192 within 0.5 %, profiles/r04x_ab_max_frames.txt)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do for mf in 4096 8192 3200; do
  timeout -k 10 300 python bench.py --secondary-dtype none --no-cpu-baseline --max-frames $mf --steps 5 > gpurun_out/mf_$mf.json 2>/dev/null || { echo fail $mf; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/mf_$mf.json').read().strip().splitlines()[-1]); print('$mf', d['value'], d['roofline']['frac'], d['ms_per_step'])"
done; done
