cd "${GRAFT_REPO_ROOT:-/root/repo}"
for cfg in "EOSV_BF16_TILE=3" "EOSV_BF16_TILE=2" "EOSV_BF16_P8=2" "EOSV_BF16_TILE=9"; do
  env $cfg timeout -k 10 200 python bench.py --dtype f32x3 --secondary-dtype none --no-cpu-baseline --layers --steps 2 > gpurun_out/ab_$cfg.json 2> gpurun_out/ab_$cfg.err || exit 1
  echo "$cfg $(python -c "import json;d=json.load(open('gpurun_out/ab_$cfg.json'));print(d['value'], d['roofline']['achieved'])")"
done
