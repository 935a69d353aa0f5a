#!/bin/bash
# LDS conflict / alignment stalls + MFMA busy + clock per kernel (one PMC pass) on a short bench run
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_lds; mkdir -p gpurun_out/pmc_lds
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_lds -o lds -- python bench.py ${BENCH_ARGS:---dtype f32x3 --secondary-dtype none --no-cpu-baseline --steps 1 --warmup 1} \
  > gpurun_out/pmc_lds/bench.log 2>&1 || { tail -5 gpurun_out/pmc_lds/bench.log; exit 1; }
f=$(find gpurun_out/pmc_lds -name "*counter_collection.csv" | head -1)
python tools/pmc_kernels.py "$f"
