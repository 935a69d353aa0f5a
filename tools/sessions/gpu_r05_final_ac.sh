#!/bin/bash
# r05 final tree (after the f32 K-order default): part A then part C
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r05_final_a.sh || exit $?
bash tools/gpu_r05_final_c.sh || exit $?
echo done_ac
