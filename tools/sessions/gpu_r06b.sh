#!/bin/bash
# r06 session B: the whole-block stage-1 kernel (bneck_bf16): bitwise against the r05 path and
# poisoned runs, then R50 bf16 per-layer timings and a release A/B against the r05 library.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06b; mkdir -p $O
P=$PWD/embodied-one-shot-video-recognition_amd
step() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; tail -n ${TAILN:-4} "$O/$name.log"; if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; exit $rc; fi; }
TAILN=12 step bitwise 600 python -u -m pytest tests/test_gpu_poison.py -x -v --timeout 280 --timeout-method thread -k "bneck or poisoned"
for A in resnet50; do
  step layers_$A 300 python bench.py --arch $A --dtype bf16 --secondary-dtype none --no-cpu-baseline --layers --steps 3
  grep layer $O/layers_$A.log | head -60
  grep '^{' $O/layers_$A.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['frac'], r['per_layer_bound']['frac'], r['traffic_algorithmic'])"
done
LIBS="libeosv_r05.so libeosv.so" ROUNDS=2 ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none" step ab_r50 600 bash tools/ab_release.sh
cat $O/ab_r50.log
echo done_r06b
