#!/bin/bash
# r04j: which WS class changes R50 bf16 outputs (profiling build; every class is meant to be bitwise
# equal to conv_bf16_kernel)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
for WS in 0 1 2 4 7; do
  EOSV_BF16_WS=$WS timeout -k 10 120 python tools/ws_diff.py save gpurun_out/ws$WS.pt resnet50 > gpurun_out/ws_save_$WS.log 2>&1 || { echo "save $WS failed"; tail -5 gpurun_out/ws_save_$WS.log; exit 1; }
done
for WS in 1 2 4 7; do echo "== ws0 vs ws$WS"; python tools/ws_diff.py cmp gpurun_out/ws0.pt gpurun_out/ws$WS.pt; done
EOSV_BF16_WS=7 timeout -k 10 120 python tools/ws_diff.py save gpurun_out/ws7b.pt resnet50 > /dev/null 2>&1 && { echo "== ws7 vs ws7 (rerun)"; python tools/ws_diff.py cmp gpurun_out/ws7.pt gpurun_out/ws7b.pt; }
