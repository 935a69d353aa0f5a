#!/bin/bash
# r05 final tree, part D: config-4 lines at the reference's precision with >= 20 oracle episodes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r05final_d; rm -rf $O; mkdir -p $O
for D in f32 f32x3; do
  echo "== c4 $D $(date +%T)"
  timeout -k 10 600 python -u tools/bench_configs.py --config 4 --dtype $D --cpu-sec 170 > $O/c4_$D.log 2>&1 || { tail -5 $O/c4_$D.log; exit 1; }
  grep "^{" $O/c4_$D.log >> $O/configs.jsonl
done
echo done
