#!/bin/bash
# r05 final tree: config-4 bf16 line with >= 20 oracle episodes and traffic attached
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05final_b2; rm -rf $O; mkdir -p $O
timeout -k 10 700 python -u tools/bench_configs.py --config 4 --dtype bf16 --cpu-sec 220 > $O/c4_bf16.log 2>&1 || { tail -5 $O/c4_bf16.log; exit 1; }
grep "^{" $O/c4_bf16.log > $O/configs.jsonl
echo done
