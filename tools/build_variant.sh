#!/bin/bash
# Build a release-build variant of libeosv.so with extra compile-time defaults (-D...), for
# like-for-like A/B of the r04 switch defaults (the profiling build's runtime switches add
# branches of their own to some kernels, e.g. EOSV_ABL checks in conv_f32_dma_kernel):
#   tools/build_variant.sh NAME -DEOSV_F32_WS_DEF=0 ...   ->   embodied-one-shot-video-recognition_amd/libeosv_NAME.so
set -e
cd "$(dirname "$0")/../embodied-one-shot-video-recognition_amd/csrc"
name=$1; shift
make -j8 > /dev/null   # the release objects
out=build_var_$name
mkdir -p $out
for f in *.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -Wall -Wno-unused-result "$@" \
    $( [ "$f" = stem_pool_bf16.hip ] && echo -fno-honor-nans ) -c $f -o $out/${f%.hip}.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libeosv_$name.so $out/*.o
echo "built libeosv_$name.so"
