#!/bin/bash
# r05: native conv check output (which case fails)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 240 tests/native/conv_check > gpurun_out/conv_check_r05i.log 2>&1
echo "rc=$?"
grep -n -E "FAIL|fail|bf16" gpurun_out/conv_check_r05i.log | head -60
