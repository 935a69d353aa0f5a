// Frame ingest: decoded uint8 RGB frames -> crop (centre, or the clip's random
// window + flip in train mode) -> ToTensor -> Normalize,
// written straight into the [F,3,crop,crop] f32 NCHW layout the backbone takes.
//
// Reference (utils.py:80-91, test mode): CenterCrop(224) -> ToTensor (x / 255) ->
// Normalize(mean, std) ((x - mean) / std), all f32.  Same operations and order here
// (correctly rounded f32 division, no FMA contraction), so the output is bit-identical to
// torchvision's on the same decoded pixels.  JPEG decode itself stays on the host.
#include "common.h"

namespace eosv {

// flip: horizontal mirror of the cropped window (torchvision hflip before ToTensor, train mode)
__global__ void normalize_frames_kernel(const unsigned char* __restrict__ rgb, int H, int W, int crop, int top,
                                        int left, int flip, float m0, float m1, float m2, float s0, float s1,
                                        float s2, float* __restrict__ out) {
  const int f = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int cc = crop * crop;
  if (p >= cc) return;
  const int y = p / crop, x = p - (p / crop) * crop;
  const int sx = flip ? crop - 1 - x : x;
  const unsigned char* px = rgb + ((long long)f * H * W + (long long)(top + y) * W + (left + sx)) * 3;
  float* o = out + (long long)f * 3 * cc + p;
  const float mean[3] = {m0, m1, m2}, sd[3] = {s0, s1, s2};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v = __fdiv_rn((float)px[c], 255.0f);
    o[(long long)c * cc] = __fdiv_rn(__fsub_rn(v, mean[c]), sd[c]);
  }
}

}  // namespace eosv

using namespace eosv;

extern "C" int eosv_crop_normalize_frames(const uint8_t* d_rgb, int n_frames, int H, int W, int crop, int top,
                                          int left, int flip, const float* mean, const float* std, float* d_out,
                                          eosv_stream_t stream) {
  if (n_frames < 0 || crop <= 0 || top < 0 || left < 0 || top + crop > H || left + crop > W || !mean || !std ||
      (n_frames && (!d_rgb || !d_out)) || n_frames > 65535) {
    set_error("eosv_crop_normalize_frames: bad argument (window inside H x W; n_frames <= 65535)");
    return EOSV_ERR_ARG;
  }
  if (n_frames == 0) return EOSV_OK;
  dim3 grid((crop * crop + 255) / 256, n_frames);
  hipLaunchKernelGGL(normalize_frames_kernel, grid, dim3(256), 0, (hipStream_t)stream, d_rgb, H, W, crop, top, left,
                     flip ? 1 : 0, mean[0], mean[1], mean[2], std[0], std[1], std[2], d_out);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

extern "C" int eosv_normalize_frames(const uint8_t* d_rgb, int n_frames, int H, int W, int crop, const float* mean,
                                     const float* std, float* d_out, eosv_stream_t stream) {
  if (crop <= 0 || H < crop || W < crop) {
    set_error("eosv_normalize_frames: bad argument (H, W >= crop; n_frames <= 65535)");
    return EOSV_ERR_ARG;
  }
  // torchvision CenterCrop: top = int(round((H - crop) / 2.0)), left likewise (round half to even)
  const int top = (int)nearbyint((H - crop) / 2.0), left = (int)nearbyint((W - crop) / 2.0);
  return eosv_crop_normalize_frames(d_rgb, n_frames, H, W, crop, top, left, 0, mean, std, d_out, stream);
}
