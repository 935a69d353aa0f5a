cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for spec in "3 1024" "3 4096" "4 2048" "4 4096" "3 1024" "3 4096"; do
  set -- $spec
  timeout -k 10 300 python tools/bench_configs.py --config $1 --dtype bf16 --episodes $([ $1 = 3 ] && echo 256 || echo 20) --max-frames $2 > gpurun_out/mfc.log 2>&1 || { tail gpurun_out/mfc.log; exit 1; }
  python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/mfc.log') if l.startswith('{')][0]
print('config $1 max_frames $2', d.get('episodes_per_s', d.get('value')), d['roofline']['frac'])"
done
