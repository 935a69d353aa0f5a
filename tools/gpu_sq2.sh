cd "${GRAFT_REPO_ROOT:-/root/repo}"
BENCH_ARGS="--dtype f32 --secondary-dtype none --no-cpu-baseline --steps 1 --warmup 1" bash tools/pmc_sq.sh > gpurun_out/sq_f32.txt 2>&1 || { tail gpurun_out/sq_f32.txt; exit 1; }
BENCH_ARGS="--dtype bf16 --secondary-dtype none --no-cpu-baseline --steps 1 --warmup 1" bash tools/pmc_sq.sh > gpurun_out/sq_bf16.txt 2>&1 || { tail gpurun_out/sq_bf16.txt; exit 1; }
head -30 gpurun_out/sq_f32.txt; head -30 gpurun_out/sq_bf16.txt
