cd "${GRAFT_REPO_ROOT:-/root/repo}"
EOSV_SUB_FRAMES=5 timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_sub5.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_sub5.log; [ $rc -le 1 ] || exit $rc
for sub in ${SUBS:-0 64 128 256}; do
  EOSV_SUB_FRAMES=$sub timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline $EXTRA > gpurun_out/sub_$sub.log 2>&1 || { tail -5 gpurun_out/sub_$sub.log; exit 1; }
  python - "$sub" <<'PY'
import json,sys
d=[json.loads(l) for l in open(f"gpurun_out/sub_{sys.argv[1]}.log") if l.startswith("{")][0]
s=d.get("secondary") or {"value":0,"roofline":{"achieved":0}}
print("sub", sys.argv[1], d["dtype"], d["value"], d["roofline"]["achieved"], s.get("dtype"), s["value"], s["roofline"]["achieved"])
PY
done
