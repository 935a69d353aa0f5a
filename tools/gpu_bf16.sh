cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -k "bf16" > gpurun_out/pytest_bf16.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_bf16.log
[ $rc -le 1 ] || exit $rc
for t in 1 2; do
  EOSV_BF16_TILE=$t timeout -k 10 300 python bench.py --dtype bf16 --steps 3 --warmup 1 --no-cpu-baseline --layers > gpurun_out/bf16_$t.log 2>&1 || { tail gpurun_out/bf16_$t.log; exit 1; }
  echo "tile $t: $(grep -o '"value": [0-9.]*' gpurun_out/bf16_$t.log) $(grep -o '"achieved": [0-9.]*' gpurun_out/bf16_$t.log) $(grep -o '"episode_acc": [0-9.]*' gpurun_out/bf16_$t.log)"
  grep layer gpurun_out/bf16_$t.log
done
