#!/bin/bash
# r05 final tree, part B1: the bf16 config lines again, after the traffic profiles exist (so their
# roofline.traffic is attached): C3 with 20 oracle episodes, C4, C5
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r05final_b1; rm -rf $O; mkdir -p $O
cfg() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 900 python -u tools/bench_configs.py "$@" > $O/$name.log 2>&1 || { echo "STOP $name"; tail -5 $O/$name.log; exit 1; }; grep "^{" $O/$name.log >> $O/configs.jsonl; }
cfg c3_bf16 --config 3 --dtype bf16 --cpu-episodes 20
cfg c4_bf16 --config 4 --dtype bf16 --cpu-sec 150
cfg c5_bf16 --config 5 --dtype bf16 --cpu-sec 60
echo done
