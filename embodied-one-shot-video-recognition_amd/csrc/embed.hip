// Clip embedding: per-frame L2 normalisation + temporal mean (wavefront reductions).
//
// Reference (network_test.py:62-65):
//     feature = F.normalize(feature, p=2, dim=1)        # x / max(||x||_2, 1e-12)
//     feature = np.mean(feature.numpy(), axis=0)        # sequential f32 row sum / T
// One 256-thread block per clip; each thread owns D/256 channels of the running sum,
// frames are folded in order (bit-equal to numpy's axis-0 reduction order); the
// squared norm of each frame is a fixed-order wave + LDS tree (deterministic).
#include "common.h"

namespace eosv {

constexpr int EMB_THREADS = 256;
constexpr int EMB_MAXV = 8;  // D <= 2048

__device__ __forceinline__ float block_sum_256(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int wid = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wid] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(EMB_THREADS) void clip_embed_kernel(
    const float* __restrict__ feat, const int* __restrict__ offsets, const int* __restrict__ counts,
    int D, int l2, float* __restrict__ emb) {
  __shared__ float red[4];
  const int c = blockIdx.x;
  const int off = offsets[c];
  const int T = counts[c];
  const int tid = threadIdx.x;
  float acc[EMB_MAXV];
#pragma unroll
  for (int j = 0; j < EMB_MAXV; ++j) acc[j] = 0.f;
  for (int t = 0; t < T; ++t) {
    const float* row = feat + (long long)(off + t) * D;
    float v[EMB_MAXV];
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < EMB_MAXV; ++j) {
      const int d = tid + EMB_THREADS * j;
      v[j] = (d < D) ? row[d] : 0.f;
      ss += v[j] * v[j];
    }
    if (l2) {
      const float nrm = fmaxf(sqrtf(block_sum_256(ss, red)), 1e-12f);
#pragma unroll
      for (int j = 0; j < EMB_MAXV; ++j) acc[j] += v[j] / nrm;
    } else {
#pragma unroll
      for (int j = 0; j < EMB_MAXV; ++j) acc[j] += v[j];
    }
  }
  const float fT = (float)T;
#pragma unroll
  for (int j = 0; j < EMB_MAXV; ++j) {
    const int d = tid + EMB_THREADS * j;
    if (d < D) emb[(long long)c * D + d] = acc[j] / fT;
  }
}

__global__ void segment_mean_kernel(const float* __restrict__ feat, int n_seg, int seg_len, int D,
                                    float* __restrict__ seg) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)n_seg * D) return;
  const long long s = t / D;
  const int d = (int)(t - s * D);
  float acc = 0.f;
  for (int k = 0; k < seg_len; ++k) acc += feat[(s * seg_len + k) * D + d];
  seg[t] = acc / (float)seg_len;
}

}  // namespace eosv

using namespace eosv;

extern "C" int eosv_clip_embed(const float* d_feat, const int32_t* d_offsets, const int32_t* d_counts,
                               int n_clips, int D, int l2, float* d_emb, eosv_stream_t stream) {
  if (n_clips < 0 || D <= 0 || D > EMB_THREADS * EMB_MAXV || (!d_feat && n_clips) ||
      (n_clips && (!d_offsets || !d_counts || !d_emb))) {
    set_error("eosv_clip_embed: bad argument (D must be in 1..2048)");
    return EOSV_ERR_ARG;
  }
  if (n_clips == 0) return EOSV_OK;
  hipLaunchKernelGGL(clip_embed_kernel, dim3(n_clips), dim3(EMB_THREADS), 0, (hipStream_t)stream,
                     d_feat, d_offsets, d_counts, D, l2, d_emb);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

extern "C" int eosv_segment_mean(const float* d_feat, int n_seg, int seg_len, int D, float* d_seg,
                                 eosv_stream_t stream) {
  if (n_seg < 0 || seg_len <= 0 || D <= 0 || (n_seg && (!d_feat || !d_seg))) {
    set_error("eosv_segment_mean: bad argument");
    return EOSV_ERR_ARG;
  }
  if (n_seg == 0) return EOSV_OK;
  const long long total = (long long)n_seg * D;
  hipLaunchKernelGGL(segment_mean_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, d_feat, n_seg, seg_len, D, d_seg);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}
