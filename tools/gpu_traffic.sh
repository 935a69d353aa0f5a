#!/bin/bash
# PMC traffic of the conv family, like for like with bench.py's traffic_algorithmic: for each
# dtype, two rocprofv3 passes (--pmc FETCH_SIZE, --pmc WRITE_SIZE) of the same bench command with
# the secondary legs off, then tools/traffic_json.py -> profiles/${TAG}_traffic.json.
#   TAG=r04x SCRIPT=bench.py ARGS="--arch resnet50 ..." bash tools/gpu_traffic.sh f32 bf16 f32x3
# (SCRIPT=tools/bench_configs.py ARGS="--config 3 ..." for config 3: --dtype is passed the same way)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/traffic_${TAG:?TAG required}
rm -rf $O; mkdir -p $O
SCRIPT=${SCRIPT:-bench.py}
EXTRA=""
[ "$SCRIPT" = bench.py ] && EXTRA="--secondary-dtype none --no-cpu-baseline --steps ${STEPS:-2} --warmup 1"
eval "ARR=($ARGS)"  # ARGS may hold quoted words (--config-label "BASELINE configs[3]")
for D in "$@"; do
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "== $D $C $(date +%T)"
    timeout -s KILL ${PMC_TIMEOUT:-300} rocprofv3 --pmc $C --output-format csv -d $O/${D}_$C -o t -- \
      python $SCRIPT "${ARR[@]}" --dtype $D $EXTRA > $O/${D}_$C.log 2>&1 || { echo "rc=$?"; tail -5 $O/${D}_$C.log; exit 1; }
  done
done
python tools/traffic_json.py profiles/${TAG}_traffic.json $O "$@"
