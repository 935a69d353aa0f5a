#!/bin/bash
# r05: f32 chunk-major K (release variant -DEOSV_F32_KCM_DEF=64) against tap-major: speed
# (release libraries, interleaved) and the variant's f32 FETCH / WRITE traffic
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
set -o pipefail
LIBS="libeosv.so libeosv_kcm64.so" ROUNDS=3 timeout -k 10 900 bash tools/ab_release.sh 2>&1 | tail -6 || exit 1
EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_kcm64.so TAG=r05l_kcm64 timeout -k 10 400 bash tools/gpu_traffic.sh f32 2>&1 | tail -2 || exit 1
echo done
