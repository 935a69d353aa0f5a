#!/bin/bash
# r05 final tree (after the training-pass change in train.hip, which moves the library digest):
# part C first (the traffic files of this digest land in profiles/ on the box), then part A, whose
# bench line then carries them; the traffic JSONs are copied under gpurun_out/ to come back.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r05_final_c.sh || exit $?
bash tools/gpu_r05_final_a.sh || exit $?
cp profiles/r05_c*_traffic.json gpurun_out/r05final/
echo done_ca
