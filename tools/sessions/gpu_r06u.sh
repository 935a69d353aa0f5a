#!/bin/bash
# r06 session U: the native check of the fused kernels, bblock_bf16 included (CPU reference over the
# first images, in place and out of place, repeat launches compared bitwise).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06u; mkdir -p $O
timeout -k 10 500 tests/native/bneck_check 3 > $O/bneck_check.log 2>&1; rc=$?
cat $O/bneck_check.log
echo "rc=$rc"
