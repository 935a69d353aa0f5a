#!/bin/bash
# tools/race_probe.py on the profiling build under several A/B switch settings: SETS="A=1,B=0 ..."
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
for set in ${SETS:-none}; do
  echo "[$set]"
  env $(echo $set | tr ',' ' ' | sed 's/none//') timeout -k 10 200 python -u tools/race_probe.py ${ARCH:-resnet50} ${DTYPE:-bf16} ${REPS:-8} || exit 1
done
