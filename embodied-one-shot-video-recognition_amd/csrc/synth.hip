// Deterministic synthetic frames on the device, bit-identical to eosv/synth.py.
//
// The reference decodes JPEGs (utils.py:96-136); offline there are none, so benches
// and GPU parity tests generate frames in HBM from the episode plan.  Every step is
// integer arithmetic or one correctly rounded f32 op (__fmul_rn/__fadd_rn: no FMA
// contraction), so frames equal the numpy generator's bit for bit.
#include "common.h"

namespace eosv {

constexpr unsigned long long GOLDEN = 0x9E3779B97F4A7C15ull;
constexpr int GRID = 14;

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float gauss_at(unsigned long long seed, unsigned long long idx) {
  const unsigned long long z = mix64(seed + (idx + 1ull) * GOLDEN);
  const long long s = (long long)((z & 0xffff) + ((z >> 16) & 0xffff) + ((z >> 32) & 0xffff) + (z >> 48));
  return __fmul_rn((float)(s - 131070), __uint_as_float(0x37ddb3d8u));  // * GAUSS_SCALE
}

// params[f] = {class_seed, video_seed, noise_seed, frame_id}; frame_id 0 -> zero frame
__global__ void synth_frames_kernel(const unsigned long long* __restrict__ params, int H, int W,
                                    float a_cls, float a_vid, float a_noise, float* __restrict__ out) {
  const int f = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int HW = H * W;
  if (p >= HW) return;
  const unsigned long long cs = params[4 * f + 0];
  const unsigned long long vs = params[4 * f + 1];
  const unsigned long long ns = params[4 * f + 2];
  const unsigned long long fid = params[4 * f + 3];
  float* o = out + (long long)f * 3 * HW + p;
  if (fid == 0) {
    o[0] = 0.f;
    o[HW] = 0.f;
    o[2 * HW] = 0.f;
    return;
  }
  const int y = p / W, x = p - (p / W) * W;
  const int gy = (y * GRID) / H;
  const int gx = (x * GRID) / W;
  const int gxv = (gx + (int)(fid / 4)) % GRID;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float cls = __fmul_rn(gauss_at(cs, (unsigned long long)(c * GRID * GRID + gy * GRID + gx)), a_cls);
    const float vid = __fmul_rn(gauss_at(vs, (unsigned long long)(c * GRID * GRID + gy * GRID + gxv)), a_vid);
    const float nz = __fmul_rn(gauss_at(ns, (unsigned long long)c * HW + p), a_noise);
    o[(long long)c * HW] = __fadd_rn(__fadd_rn(cls, vid), nz);
  }
}

}  // namespace eosv

using namespace eosv;

extern "C" int eosv_synth_frames(const uint64_t* d_params, int n_frames, int H, int W, float* d_frames,
                                 eosv_stream_t stream) {
  if (n_frames < 0 || H <= 0 || W <= 0 || n_frames > 65535 * 64) {
    set_error("eosv_synth_frames: bad argument");
    return EOSV_ERR_ARG;
  }
  if (n_frames == 0) return EOSV_OK;
  if (!d_params || !d_frames) {
    set_error("eosv_synth_frames: null pointer");
    return EOSV_ERR_ARG;
  }
  // amplitudes mirror eosv/synth.py A_CLS, A_VID, A_NOISE
  const float a_cls = 1.0f, a_vid = 1.0f, a_noise = 0.5f;
  int done = 0;
  while (done < n_frames) {  // grid.y <= 65535
    const int nf = n_frames - done < 65535 ? n_frames - done : 65535;
    dim3 grid((H * W + 255) / 256, nf);
    hipLaunchKernelGGL(synth_frames_kernel, grid, dim3(256), 0, (hipStream_t)stream,
                       (const unsigned long long*)d_params + 4ll * done, H, W, a_cls, a_vid, a_noise,
                       d_frames + (long long)done * 3 * H * W);
    EOSV_LAUNCH_CHECK();
    done += nf;
  }
  return EOSV_OK;
}
