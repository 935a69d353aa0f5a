#!/bin/bash
# r06 session P: fused stage-1 modes after the packed epilogues and NPT 2 -- per-layer times
# (profiling build) and values for R50 at the C2 shape and R101 at 256 (config 5's shape):
# EOSV_BNECK / EOSV_BNECK_TAIL = 1/1, 1/0, 0/0.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06p; mkdir -p $O
L=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
run() {  # tag bneck tail args...
  local t=$1 b=$2 tl=$3; shift 3
  EOSV_LIBRARY=$L EOSV_BNECK=$b EOSV_BNECK_TAIL=$tl timeout -k 10 300 python bench.py --dtype bf16 --secondary-dtype none \
    --no-cpu-baseline --layers --steps 3 "$@" > $O/$t.log 2>&1 || { tail -5 $O/$t.log; exit 1; }
  python - $O/$t.log <<'PY'
import sys, re, json
d = {}; v = None
for l in open(sys.argv[1]):
    m = re.search(r'layer +(\d+): +([\d.]+) ms', l)
    if m: d[int(m.group(1))] = float(m.group(2))
    if l.startswith('{'): v = json.loads(l)
s1 = sum(t for k, t in d.items() if k <= 10)
print(sys.argv[1].split('/')[-1], v['value'], 'total', round(sum(d.values()), 3), 'stage1', round(s1, 3), {k: t for k, t in d.items() if k <= 10})
PY
}
for r in 1 2; do
  run r50_11_$r 1 1 --arch resnet50
  run r50_10_$r 1 0 --arch resnet50
  run r50_00_$r 0 0 --arch resnet50
done
A="--arch resnet101 --n-way 5 --k-shot 5 --segments 32 --res 256 --episodes-per-step 2 --max-frames 2048"
run r101_11 1 1 $A
run r101_10 1 0 $A
run r101_00 0 0 $A
