#!/bin/bash
# bf16 stem staging two steps ahead (EOSV_STEM_AHEAD 2) against one (r02): bitwise per stage,
# determinism, per-layer A/B (profiling build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
mkdir -p gpurun_out
set -o pipefail
for a in resnet18 resnet50; do
  EOSV_STEM_AHEAD=1 timeout -k 10 120 python tools/ws_diff.py save /tmp/st1_$a.pt $a bf16 2>/dev/null || exit 1
  EOSV_STEM_AHEAD=2 timeout -k 10 120 python tools/ws_diff.py save /tmp/st2_$a.pt $a bf16 2>/dev/null || exit 1
  echo "== $a bf16 stages, AHEAD 1 vs 2"; python tools/ws_diff.py cmp /tmp/st1_$a.pt /tmp/st2_$a.pt
done
timeout -k 10 200 python -u tools/race_modes.py resnet50 bf16 17,64,130 0,4,1 3 2>&1 | grep -v amdgpu.ids || exit 1
VAR=EOSV_STEM_AHEAD VALS="1 2" ARCH=resnet18 DTYPE=bf16 timeout -k 10 600 bash tools/ab_env.sh 2>&1 | head -12
