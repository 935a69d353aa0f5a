#!/bin/bash
# r06 final tree, part B1: config lines (C3 bf16 with 20 oracle episodes, C4 bf16 / f32 / f32x3, C5
# bf16 with a parity dump for tools/offline_parity.py), training step bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r06final; mkdir -p $O
cfg() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 900 python -u tools/bench_configs.py "$@" > $O/$name.log 2>&1 || { echo "STOP $name"; tail -5 $O/$name.log; exit 1; }; grep "^{" $O/$name.log >> $O/configs.jsonl; grep "^{" $O/$name.log | cut -c1-300; }
cfg c3_bf16 --config 3 --dtype bf16 --cpu-episodes 20
cfg c4_bf16 --config 4 --dtype bf16 --cpu-sec 150
echo done_b1
