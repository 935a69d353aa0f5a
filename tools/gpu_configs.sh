#!/bin/bash
# Throughput of BASELINE configs 3/4/5 (tools/bench_configs.py).  SPECS="cfg dtype episodes;..."
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
IFS=';' read -ra LIST <<< "${SPECS:-3 bf16 512;3 f32 128;4 bf16 20;4 f32 10;5 bf16 4}"
for spec in "${LIST[@]}"; do
  set -- $spec
  echo "== config $1 $2"
  timeout -k 10 600 python tools/bench_configs.py --config $1 --dtype $2 --episodes $3 > gpurun_out/cfg_$1_$2.log 2>&1 || { tail -20 gpurun_out/cfg_$1_$2.log; exit 1; }
  grep "^{" gpurun_out/cfg_$1_$2.log | cut -c1-700
done
