#!/bin/bash
# r04i: FETCH_SIZE of the f32 leg at K chunk 0 / 64 / 128 (profiling build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for K in 0 64 128; do
  EOSV_F32_KCM=$K EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/kcm_fetch_$K -o t -- \
    python bench.py --secondary-dtype none --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/kcm_fetch_$K.log 2>&1 || { echo "pmc rc=$?"; tail -5 gpurun_out/kcm_fetch_$K.log; exit 1; }
done
python tools/pmc_kernels.py $(find gpurun_out/kcm_fetch_0 gpurun_out/kcm_fetch_64 gpurun_out/kcm_fetch_128 -name "*counter_collection.csv") 2>&1
