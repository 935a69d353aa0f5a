#!/bin/bash
# r03 measurement, part B: BASELINE configs 3-5 lines in their three dtypes (tools/bench_configs.py),
# config-3 FETCH_SIZE / WRITE_SIZE passes (bf16), SQ counters of ResNet-50 bf16 (the pairs)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r03b}
mkdir -p gpurun_out/cfg gpurun_out/prof
step() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "gpurun_out/cfg/$name.log" 2>&1; local rc=$?; grep "^{" "gpurun_out/cfg/$name.log" | cut -c1-400; if [ $rc -ne 0 ]; then tail -5 "gpurun_out/cfg/$name.log"; echo "STOP $name rc=$rc"; exit $rc; fi; }
IFS=';' read -ra LIST <<< "${SPECS:-3 bf16 512;3 f32 128;3 f32x3 256;4 bf16 0;4 f32 0;4 f32x3 0;5 bf16 0;5 f32 0;5 f32x3 0}"
for spec in "${LIST[@]}"; do
  set -- $spec
  EP=""; [ "$3" != "0" ] && EP="--episodes $3"
  CPU=""; [ "$1" = "3" ] && [ "$2" != "bf16" ] && CPU="--cpu-episodes 0"
  step c$1_$2 900 python tools/bench_configs.py --config $1 --dtype $2 $EP $CPU
done
[ -n "$SKIP_PMC" ] && exit 0
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== c3 pmc $C $(date +%T)"
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d gpurun_out/prof/c3_$C -o $TAG -- \
    python tools/bench_configs.py --config 3 --dtype bf16 --episodes 64 --cpu-episodes 0 > gpurun_out/cfg/c3_pmc_$C.log 2>&1 \
    || { tail -5 gpurun_out/cfg/c3_pmc_$C.log; exit 1; }
done
echo "== sq r50 $(date +%T)"
BENCH_ARGS="--arch resnet50 --dtype bf16 --secondary-dtype none --no-cpu-baseline --steps 1 --warmup 1" bash tools/pmc_sq.sh > gpurun_out/cfg/sq_r50_bf16.txt 2>&1 || { tail gpurun_out/cfg/sq_r50_bf16.txt; exit 1; }
head -20 gpurun_out/cfg/sq_r50_bf16.txt
echo done
