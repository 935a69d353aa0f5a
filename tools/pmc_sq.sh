#!/bin/bash
# SQ cycle buckets + MFMA busy + effective clock per kernel (one PMC pass) on a short bench run
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_sq; mkdir -p gpurun_out/pmc_sq
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_sq -o sq -- python bench.py ${BENCH_ARGS:---dtype bf16 --secondary-dtype none --no-cpu-baseline --steps 1 --warmup 1} \
  > gpurun_out/pmc_sq/bench.log 2>&1 || { tail -5 gpurun_out/pmc_sq/bench.log; exit 1; }
f=$(find gpurun_out/pmc_sq -name "*counter_collection.csv" | head -1)
python tools/pmc_kernels.py "$f"
