cd "${GRAFT_REPO_ROOT:-/root/repo}"
for mf in ${MFS:-256 512 1024 2048}; do
  timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --max-frames $mf > gpurun_out/mf_$mf.log 2>&1 || { tail -5 gpurun_out/mf_$mf.log; exit 1; }
  python - "$mf" <<'PY'
import json,sys
d=[json.loads(l) for l in open(f"gpurun_out/mf_{sys.argv[1]}.log") if l.startswith("{")][0]
print("max_frames", sys.argv[1], "f32", d["value"], d["roofline"]["achieved"], "bf16", d["secondary"]["value"], d["secondary"]["roofline"]["achieved"])
PY
done
