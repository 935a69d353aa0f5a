#!/bin/bash
# r05z: split-K accuracy of the training convs, r04 sizing (libeosv.so) vs k4m16 (libeosv_k4m16.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
P=$PWD/embodied-one-shot-video-recognition_amd
for L in libeosv.so libeosv_k4m16.so; do
  echo "== $L"
  EOSV_LIBRARY=$P/$L timeout -k 10 300 python tools/ksplit_accuracy.py || exit 1
done
