cd "${GRAFT_REPO_ROOT:-/root/repo}"
export EOSV_CONV_IMPL=5
for abl in 0 1 2 3; do
  EOSV_CONV_ABL=$abl timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --layers > gpurun_out/abl_$abl.log 2>&1 || { tail gpurun_out/abl_$abl.log; exit 1; }
  echo "abl $abl: $(grep -o '"achieved": [0-9.]*' gpurun_out/abl_$abl.log)"; grep -E "layer +(0|1|5|6|7|13):" gpurun_out/abl_$abl.log
done
