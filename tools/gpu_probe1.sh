#!/bin/bash
# r03: LDS-DMA row-gather rates (tests/native/l2dma_probe) + per-kernel L2 hit rates of the bf16
# convs (R18 C2 shape and R50 C4 frame shape), one PMC pass each
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/probe1
timeout -k 10 120 tests/native/l2dma_probe > gpurun_out/probe1/l2dma.txt 2>&1 || { cat gpurun_out/probe1/l2dma.txt; exit 1; }
cat gpurun_out/probe1/l2dma.txt
for A in resnet18 resnet50; do
  timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/probe1/tcc_$A -o tcc -- \
    python bench.py --arch $A --dtype bf16 --secondary-dtype none --no-cpu-baseline --steps 1 --warmup 1 --episodes-per-step 40 \
    > gpurun_out/probe1/tcc_$A.log 2>&1 || { tail -5 gpurun_out/probe1/tcc_$A.log; exit 1; }
done
python tools/pmc_kernels.py $(find gpurun_out/probe1 -name '*counter_collection.csv') > gpurun_out/probe1/tcc_summary.txt 2>&1; head -60 gpurun_out/probe1/tcc_summary.txt
