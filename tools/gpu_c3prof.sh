#!/bin/bash
# rocprofv3 kernel stats of the config-3 line in one dtype (DTYPE, default f32): where the
# non-conv wall time goes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c3prof
D=${DTYPE:-f32}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3prof/$D -o c3 -- \
  python tools/bench_configs.py --config 3 --dtype $D --episodes ${EP:-64} --cpu-episodes 0 > gpurun_out/c3prof/$D.log 2>&1 \
  || { tail -5 gpurun_out/c3prof/$D.log; exit 1; }
grep "^{" gpurun_out/c3prof/$D.log | cut -c1-300
python - gpurun_out/c3prof/$D/c3_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:30]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):6d} {float(r['TotalDurationNs'])/1e6:9.2f} ms {100*float(r['TotalDurationNs'])/tot:5.1f} %")
PY
