// Layout + pooling kernels around the conv stack (all HBM-bound byte movers).
//
//  pack_rgb_pad    : the caller's [B,3,H,W] f32 frames (what network_test.py:58 hands
//                    to self.mymodel) -> dense padded RGB [B][H+2p][Wp][3] (f32 or bf16),
//                    the layout the 7x7 stem reads (conv_f32_dma.hip / conv_bf16.hip).
//  maxpool3x3s2    : torchvision conv1 -> bn1 -> relu -> maxpool(3,2,1) (convnet.3).
//  avgpool         : AdaptiveAvgPool2d(1) + view(B,-1) (convnet.8, models.py:19-20):
//                    sequential f32 sum over the HxW positions, then / (H*W).
#include <hip/hip_bf16.h>

#include "common.h"

namespace eosv {

__device__ __forceinline__ float bf2f(unsigned short v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) {
  return __bfloat16_as_ushort(__float2bfloat16(f));  // RNE, NaN-preserving
}

// one thread = one interior pixel; the zero borders of the padded image are written once
// (eosv_create memsets the buffer) and never touched again
template <typename T>
__global__ void pack_rgb_pad_kernel(const float* __restrict__ x, long long npix, int H, int W, int pad, int Wp,
                                    T* __restrict__ y) {
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const int HW = H * W;
  const long long b = p / HW;
  const int hw = (int)(p - b * HW);
  const int yy = hw / W, xx = hw - (hw / W) * W;
  const float* src = x + b * 3 * HW + hw;
  T* dst = y + ((b * (H + 2 * pad) + yy + pad) * Wp + xx + pad) * 3;
  if constexpr (sizeof(T) == 4) {
    dst[0] = src[0];
    dst[1] = src[HW];
    dst[2] = src[2 * HW];
  } else {
    dst[0] = f2bf(src[0]);
    dst[1] = f2bf(src[HW]);
    dst[2] = f2bf(src[2 * HW]);
  }
}

int launch_pack_rgb_pad(const float* x, int B, int H, int W, int pad, void* y, int bf16, hipStream_t s) {
  const long long npix = (long long)B * H * W;
  const unsigned grid = (unsigned)((npix + 255) / 256);
  const int Wp = stem_row_pixels(W, pad);
  if (bf16)
    hipLaunchKernelGGL(pack_rgb_pad_kernel<unsigned short>, dim3(grid), dim3(256), 0, s, x, npix, H, W, pad, Wp,
                       (unsigned short*)y);
  else
    hipLaunchKernelGGL(pack_rgb_pad_kernel<float>, dim3(grid), dim3(256), 0, s, x, npix, H, W, pad, Wp, (float*)y);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

// one thread = 4 channels of one output pixel
__global__ void maxpool_f32_kernel(const float4* __restrict__ x, int B, int H, int W, int C4,
                                   float4* __restrict__ y, int Ho, int Wo) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)B * Ho * Wo * C4;
  if (t >= total) return;
  const int c = (int)(t % C4);
  long long p = t / C4;
  const int ow = (int)(p % Wo);
  p /= Wo;
  const int oh = (int)(p % Ho);
  const long long b = p / Ho;
  float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
  for (int dh = 0; dh < 3; ++dh) {
    const int ih = oh * 2 - 1 + dh;
    if ((unsigned)ih >= (unsigned)H) continue;
    for (int dw = 0; dw < 3; ++dw) {
      const int iw = ow * 2 - 1 + dw;
      if ((unsigned)iw >= (unsigned)W) continue;
      const float4 v = x[((b * H + ih) * W + iw) * C4 + c];
      m.x = fmaxf(m.x, v.x);
      m.y = fmaxf(m.y, v.y);
      m.z = fmaxf(m.z, v.z);
      m.w = fmaxf(m.w, v.w);
    }
  }
  y[t] = m;
}

// bf16: one thread = 8 channels (16 B)
__global__ void maxpool_bf16_kernel(const uint4* __restrict__ x, int B, int H, int W, int C8,
                                    uint4* __restrict__ y, int Ho, int Wo) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long total = (long long)B * Ho * Wo * C8;
  if (t >= total) return;
  const int c = (int)(t % C8);
  long long p = t / C8;
  const int ow = (int)(p % Wo);
  p /= Wo;
  const int oh = (int)(p % Ho);
  const long long b = p / Ho;
  float m[8];
  for (int k = 0; k < 8; ++k) m[k] = -INFINITY;
  for (int dh = 0; dh < 3; ++dh) {
    const int ih = oh * 2 - 1 + dh;
    if ((unsigned)ih >= (unsigned)H) continue;
    for (int dw = 0; dw < 3; ++dw) {
      const int iw = ow * 2 - 1 + dw;
      if ((unsigned)iw >= (unsigned)W) continue;
      const uint4 v = x[((b * H + ih) * W + iw) * C8 + c];
      const unsigned u[4] = {v.x, v.y, v.z, v.w};
      for (int k = 0; k < 4; ++k) {
        m[2 * k] = fmaxf(m[2 * k], bf2f((unsigned short)(u[k] & 0xffff)));
        m[2 * k + 1] = fmaxf(m[2 * k + 1], bf2f((unsigned short)(u[k] >> 16)));
      }
    }
  }
  uint4 o;
  o.x = (unsigned)f2bf(m[0]) | ((unsigned)f2bf(m[1]) << 16);
  o.y = (unsigned)f2bf(m[2]) | ((unsigned)f2bf(m[3]) << 16);
  o.z = (unsigned)f2bf(m[4]) | ((unsigned)f2bf(m[5]) << 16);
  o.w = (unsigned)f2bf(m[6]) | ((unsigned)f2bf(m[7]) << 16);
  y[t] = o;
}

int launch_maxpool3x3s2(const void* x, int B, int H, int W, int C, void* y, int Ho, int Wo, int bf16,
                        hipStream_t s) {
  if (bf16) {
    if (C % 8) return set_error("maxpool: C % 8"), EOSV_ERR_UNSUPPORTED;
    const long long total = (long long)B * Ho * Wo * (C / 8);
    hipLaunchKernelGGL(maxpool_bf16_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       (const uint4*)x, B, H, W, C / 8, (uint4*)y, Ho, Wo);
  } else {
    if (C % 4) return set_error("maxpool: C % 4"), EOSV_ERR_UNSUPPORTED;
    const long long total = (long long)B * Ho * Wo * (C / 4);
    hipLaunchKernelGGL(maxpool_f32_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       (const float4*)x, B, H, W, C / 4, (float4*)y, Ho, Wo);
  }
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

// one thread = one (frame, channel); consecutive threads = consecutive channels (coalesced)
template <bool BF16, bool SPLIT = false>
__global__ void avgpool_kernel(const void* __restrict__ xv, int B, int HW, int C, float* __restrict__ y) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)B * C) return;
  const long long b = t / C;
  const int c = (int)(t - b * C);
  float s = 0.f;
  if constexpr (SPLIT) {
    // EOSV_F32X3 layout [pixel][hi C | lo C]: value = hi + lo (exact in f32)
    const unsigned short* x = (const unsigned short*)xv + b * HW * 2 * C + c;
    for (int p = 0; p < HW; ++p) s += bf2f(x[(long long)p * 2 * C]) + bf2f(x[(long long)p * 2 * C + C]);
  } else if constexpr (BF16) {
    const unsigned short* x = (const unsigned short*)xv + b * HW * C + c;
    for (int p = 0; p < HW; ++p) s += bf2f(x[(long long)p * C]);
  } else {
    const float* x = (const float*)xv + b * HW * C + c;
    for (int p = 0; p < HW; ++p) s += x[(long long)p * C];
  }
  y[t] = s / (float)HW;
}

// activation map -> f32, same NHWC order (eosv_backbone_probe); mode as launch_avgpool's bf16
__global__ void act_to_f32_kernel(const void* __restrict__ xv, long long n, int C, int mode, float* __restrict__ y) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (mode == 2) {
    const unsigned short* x = (const unsigned short*)xv;
    const long long p = i / C;
    const int c = (int)(i - p * C);
    y[i] = bf2f(x[p * 2 * C + c]) + bf2f(x[p * 2 * C + C + c]);
  } else if (mode == 1) {
    y[i] = bf2f(((const unsigned short*)xv)[i]);
  } else {
    y[i] = ((const float*)xv)[i];
  }
}

int launch_act_to_f32(const void* x, long long n, int C, int mode, float* y, hipStream_t s) {
  if (n <= 0) return EOSV_OK;
  hipLaunchKernelGGL(act_to_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, n, C, mode, y);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int launch_avgpool(const void* x, int B, int HW, int C, float* y, int bf16, hipStream_t s) {
  const long long total = (long long)B * C;
  const unsigned grid = (unsigned)((total + 255) / 256);
  if (bf16 == 2)
    hipLaunchKernelGGL((avgpool_kernel<true, true>), dim3(grid), dim3(256), 0, s, x, B, HW, C, y);
  else if (bf16)
    hipLaunchKernelGGL(avgpool_kernel<true>, dim3(grid), dim3(256), 0, s, x, B, HW, C, y);
  else
    hipLaunchKernelGGL(avgpool_kernel<false>, dim3(grid), dim3(256), 0, s, x, B, HW, C, y);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

}  // namespace eosv
