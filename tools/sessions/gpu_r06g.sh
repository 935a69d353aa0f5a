#!/bin/bash
# r06 session G: the native bneck check (CPU reference + repeat launches compared bitwise).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 400 tests/native/bneck_check 4 > $O/bneck_check.log 2>&1; rc=$?
cat $O/bneck_check.log
echo "rc=$rc"
