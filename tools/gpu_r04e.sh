#!/bin/bash
# r04e: LDS-DMA rate probe (sync vs ring) and 256x256 bf16 conv ablations (profiling build):
# which part of the K-step bounds the 3x3s.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 240 tests/native/l2dma_probe > gpurun_out/l2dma.log 2>&1 || { echo "probe rc=$?"; tail gpurun_out/l2dma.log; exit 1; }
cat gpurun_out/l2dma.log
# 0 full, 48 no ds_reads + no MFMAs (DMA + barriers only), 1 no main-loop DMA, 32 no MFMAs, 17 no DMA no ds_read
ARCH=resnet50 ABLS="0 48 1 32 17" timeout -k 10 900 bash tools/abl_bf16.sh
