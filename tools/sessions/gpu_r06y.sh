#!/bin/bash
# r06 session Y: per-layer times of R18 bf16 with bblock2 (profiling build, EOSV_BBLOCK2=1 / 0)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06y; mkdir -p $O
for v in 1 0; do
  EOSV_BBLOCK2=$v EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so timeout -k 10 300 python bench.py --dtype bf16 \
      --secondary-dtype none --no-cpu-baseline --layers --steps 3 > $O/layers_$v.log 2>&1 || { tail -5 $O/layers_$v.log; exit 1; }
  echo "== EOSV_BBLOCK2=$v"; grep -E "layer +[0-9]+:" $O/layers_$v.log | head -8
done
