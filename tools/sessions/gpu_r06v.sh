#!/bin/bash
# r06 session V: bblock_bf16 over an even share of all images' steps per workgroup (warm-up steps at
# range starts, out of place) -- native check, bitwise tests, determinism, per-layer times, release
# A/B against the whole-images form (libeosv_bbimg.so) on R18 bf16 at the C2 shape.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06v; mkdir -p $O
P=$PWD/embodied-one-shot-video-recognition_amd
timeout -k 10 500 tests/native/bneck_check 3 > $O/bneck_check.log 2>&1 || { cat $O/bneck_check.log; exit 1; }
grep -E "bblock|failures" $O/bneck_check.log
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_poison.py -k "bblock or poisoned" > $O/tests.log 2>&1 || { tail -25 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/race_modes.py resnet18 bf16 37,64,130,601 0 4 > $O/race_r18.log 2>&1 || { tail -5 $O/race_r18.log; exit 1; }
grep -v amdgpu.ids $O/race_r18.log
EOSV_LIBRARY=$P/libeosv_prof.so timeout -k 10 300 python bench.py --dtype bf16 --secondary-dtype none \
    --no-cpu-baseline --layers --steps 3 > $O/layers_r18.log 2>&1 || { tail -5 $O/layers_r18.log; exit 1; }
echo "layers: $(grep -E 'layer +[0-9]:' $O/layers_r18.log | tr -s ' ' | cut -d' ' -f3,4 | paste -sd' ')"
ROUNDS=3 LIBS="libeosv_bbimg.so libeosv.so" ARGS="--dtype bf16 --secondary-dtype none" timeout -k 10 900 bash tools/ab_release.sh > $O/ab_r18.log 2>&1 || { cat $O/ab_r18.log; exit 1; }
cat $O/ab_r18.log
