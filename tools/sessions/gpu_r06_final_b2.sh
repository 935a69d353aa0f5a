#!/bin/bash
# r06 final tree, part B2: config lines (C3 bf16 with 20 oracle episodes, C4 bf16 / f32 / f32x3, C5
# bf16 with a parity dump for tools/offline_parity.py), training step bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r06final; mkdir -p $O
cfg() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 900 python -u tools/bench_configs.py "$@" > $O/$name.log 2>&1 || { echo "STOP $name"; tail -5 $O/$name.log; exit 1; }; grep "^{" $O/$name.log >> $O/configs.jsonl; grep "^{" $O/$name.log | cut -c1-300; }
cfg c4_f32 --config 4 --dtype f32 --cpu-sec 170
cfg c4_f32x3 --config 4 --dtype f32x3 --cpu-sec 170
cfg c5_bf16 --config 5 --dtype bf16 --cpu-sec 60 --parity-dump $O/c5_dump.npz
timeout -k 10 300 python tools/bench_train.py > $O/train.log 2>&1 || { echo "train failed"; tail -5 $O/train.log; exit 1; }
grep "^{" $O/train.log
echo done_b2
