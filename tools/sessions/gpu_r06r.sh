#!/bin/bash
# r06 session R: bblock_bf16 with double-buffered B fragments -- bitwise tests, determinism,
# per-layer times, release A/B against the single-buffered form (bb1) and r05 (R18 bf16, C2 shape).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06r; mkdir -p $O
P=$PWD/embodied-one-shot-video-recognition_amd
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_poison.py -k "bblock or poisoned" > $O/tests.log 2>&1 || { tail -25 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/race_modes.py resnet18 bf16 37,64,130 0 4 > $O/race_r18.log 2>&1 || { tail -5 $O/race_r18.log; exit 1; }
grep -v amdgpu.ids $O/race_r18.log
EOSV_LIBRARY=$P/libeosv_prof.so timeout -k 10 300 python bench.py --dtype bf16 --secondary-dtype none \
    --no-cpu-baseline --layers --steps 3 > $O/layers_r18.log 2>&1 || { tail -5 $O/layers_r18.log; exit 1; }
echo "layers: $(grep -E 'layer +[0-9]:' $O/layers_r18.log | tr -s ' ' | cut -d' ' -f3,4 | paste -sd' ')"
ROUNDS=2 LIBS="libeosv_r05.so libeosv_bb1.so libeosv.so" ARGS="--dtype bf16 --secondary-dtype none" timeout -k 10 900 bash tools/ab_release.sh > $O/ab_r18.log 2>&1 || { cat $O/ab_r18.log; exit 1; }
cat $O/ab_r18.log
