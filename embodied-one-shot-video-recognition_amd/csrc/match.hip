// One-shot matching kernels (the hot-path sink, reference classifier.py / network_test.py).
//
//  match_protonet : classifier.py:9-40 + 43-90 -- per-label prototype = sequential f32
//                   mean in first-appearance order; scipy cdist 'euclidean' in f64 on the
//                   f32 inputs; torch.FloatTensor (f64->f32); softmax(-d) over the
//                   prototypes (max-subtract, exp, 1/sum, scale); np.argmax (first max).
//  match_cosine   : classifier.py:117-120 -- sklearn cosine_similarity (rows divided by
//                   their f32 L2 norm, zero norm -> 1) then argsort(-s)[:,0] = first max.
//  segment_match  : network_test.py:207-214 + models.py:42-56 -- cdist(seg, gallery) f64
//                   -> f32 -> 3-tap [l1,l2,l1] conv along the flattened segment axis with
//                   zero padding -> first argmin over the gallery.
// One block per episode (matching is < 1% of the path's time); all reductions are
// fixed-order trees, so results are run-to-run deterministic.
#include <cfloat>

#include "common.h"

namespace eosv {

constexpr int MT = 256;
constexpr int MAXV = 8;  // D <= 2048
constexpr int MAXP = 64;

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(MT) void match_protonet_kernel(
    const float* __restrict__ query, const float* __restrict__ sup, const int* __restrict__ sup_off,
    const int* __restrict__ sup_slot, const int* __restrict__ n_proto, int D, long long* __restrict__ pred,
    float* __restrict__ score) {
  __shared__ double red[4];
  __shared__ float dist[MAXP];
  const int e = blockIdx.x;
  const int s0 = sup_off[e], s1 = sup_off[e + 1];
  const int P = n_proto[e];
  const int tid = threadIdx.x;
  float q[MAXV];
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int d = tid + MT * j;
    q[j] = d < D ? query[(long long)e * D + d] : 0.f;
  }
  for (int p = 0; p < P; ++p) {
    float acc[MAXV];
#pragma unroll
    for (int j = 0; j < MAXV; ++j) acc[j] = 0.f;
    int cnt = 0;
    for (int s = s0; s < s1; ++s) {
      if (sup_slot[s] != p) continue;
      ++cnt;
      const float* row = sup + (long long)s * D;
#pragma unroll
      for (int j = 0; j < MAXV; ++j) {
        const int d = tid + MT * j;
        if (d < D) acc[j] += row[d];
      }
    }
    double part = 0.0;
    const float fc = (float)cnt;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      const int d = tid + MT * j;
      if (d < D) {
        const double diff = (double)q[j] - (double)(acc[j] / fc);
        part += diff * diff;
      }
    }
    const double ss = block_sum(part, red);
    if (tid == 0) dist[p] = (float)sqrt(ss);
  }
  __syncthreads();
  if (tid == 0) {
    // softmax(-d) as torch-CPU computes it, then np.argmax (first maximum)
    float mx = -INFINITY;
    for (int p = 0; p < P; ++p) mx = fmaxf(mx, -dist[p]);
    float ex[MAXP];
    float sum = 0.f;
    for (int p = 0; p < P; ++p) {
      ex[p] = expf(-dist[p] - mx);
      sum += ex[p];
    }
    const float inv = 1.f / sum;
    int best = 0;
    float bv = -INFINITY;
    for (int p = 0; p < P; ++p) {
      const float pr = ex[p] * inv;
      if (pr > bv) {
        bv = pr;
        best = p;
      }
    }
    pred[e] = best;
    if (score) {
      for (int p = 0; p < MAXP; ++p) score[(long long)e * MAXP + p] = p < P ? dist[p] : 0.f;
    }
  }
}

__global__ __launch_bounds__(MT) void match_cosine_kernel(const float* __restrict__ query,
                                                          const float* __restrict__ sup,
                                                          const int* __restrict__ sup_off, int D,
                                                          long long* __restrict__ pred,
                                                          float* __restrict__ score) {
  __shared__ float red[4];
  __shared__ float sims[MAXP];
  const int e = blockIdx.x;
  const int s0 = sup_off[e], s1 = sup_off[e + 1];
  const int tid = threadIdx.x;
  float q[MAXV];
  float qs = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int d = tid + MT * j;
    q[j] = d < D ? query[(long long)e * D + d] : 0.f;
    qs += q[j] * q[j];
  }
  float qn = sqrtf(block_sum(qs, red));
  if (qn == 0.f) qn = 1.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) q[j] = q[j] / qn;
  int best = 0;
  float bv = -INFINITY;
  for (int s = s0; s < s1; ++s) {
    const float* row = sup + (long long)s * D;
    float v[MAXV];
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      const int d = tid + MT * j;
      v[j] = d < D ? row[d] : 0.f;
      ss += v[j] * v[j];
    }
    float sn = sqrtf(block_sum(ss, red));
    if (sn == 0.f) sn = 1.f;
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) dot += q[j] * (v[j] / sn);
    const float sim = block_sum(dot, red);
    if (sim > bv) {  // every thread sees the same sim: first maximum wins
      bv = sim;
      best = s - s0;
    }
    if (tid == 0 && s - s0 < MAXP) sims[s - s0] = sim;
  }
  __syncthreads();
  if (tid == 0) {
    pred[e] = best;
    if (score)
      for (int p = 0; p < MAXP; ++p) score[(long long)e * MAXP + p] = p < (s1 - s0) ? sims[p] : 0.f;
  }
}

// ---------------------------------------------------------------- segment matching
// dist[s][g] = sqrt(sum_d (seg[s][d] - gal[g][d])^2) in f64, stored f32.
// Block: 64 gallery rows x up to 64 segment rows, D staged through LDS in chunks of 32.
constexpr int SG_G = 64, SG_S = 64, SG_DK = 32;

__global__ __launch_bounds__(256) void seg_dist_kernel(const float* __restrict__ seg, int S,
                                                       const float* __restrict__ gal, int G, int D,
                                                       float* __restrict__ dist) {
  __shared__ float gs[SG_G][SG_DK + 1];
  __shared__ float ss[SG_S][SG_DK + 1];
  const int g0 = blockIdx.x * SG_G;
  const int sb = blockIdx.y * SG_S;
  const int tid = threadIdx.x;
  const int gl = tid & 63;
  const int sgrp = tid >> 6;  // 4 groups, thread owns s = sgrp + 4*i
  double acc[SG_S / 4];
#pragma unroll
  for (int i = 0; i < SG_S / 4; ++i) acc[i] = 0.0;
  for (int d0 = 0; d0 < D; d0 += SG_DK) {
    for (int t = tid; t < SG_G * SG_DK; t += 256) {
      const int r = t / SG_DK, c = t % SG_DK;
      const int g = g0 + r, d = d0 + c;
      gs[r][c] = (g < G && d < D) ? gal[(long long)g * D + d] : 0.f;
      const int s = sb + r;
      ss[r][c] = (s < S && d < D) ? seg[(long long)s * D + d] : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int c = 0; c < SG_DK; ++c) {
      const double gv = (double)gs[gl][c];
#pragma unroll
      for (int i = 0; i < SG_S / 4; ++i) {
        const double df = (double)ss[sgrp + 4 * i][c] - gv;
        acc[i] += df * df;
      }
    }
    __syncthreads();
  }
  const int g = g0 + gl;
  if (g < G) {
#pragma unroll
    for (int i = 0; i < SG_S / 4; ++i) {
      const int s = sb + sgrp + 4 * i;
      if (s < S) dist[(long long)s * G + g] = (float)sqrt(acc[i]);
    }
  }
}

// smoothed[s][g] = l1*d[s-1][g] + l2*d[s][g] + l1*d[s+1][g] (zero padded at the ends of each
// episode's S rows), argmin over g; one block per row of the n_episodes*S rows
__global__ __launch_bounds__(256) void seg_smooth_argmin_kernel(const float* __restrict__ dist, int S,
                                                                int G, float l1, float l2,
                                                                long long* __restrict__ ids,
                                                                float* __restrict__ out) {
  __shared__ float bvs[4];
  __shared__ int bis[4];
  const int s = blockIdx.x;
  const int sl = s % S;  // row within its episode
  float bv = INFINITY;
  int bi = 0x7fffffff;
  for (int g = threadIdx.x; g < G; g += 256) {
    const float dm = sl > 0 ? dist[(long long)(s - 1) * G + g] : 0.f;
    const float d0 = dist[(long long)s * G + g];
    const float dp = sl + 1 < S ? dist[(long long)(s + 1) * G + g] : 0.f;
    const float v = fmaf(l1, dp, fmaf(l2, d0, l1 * dm));
    if (out) out[(long long)s * G + g] = v;
    if (v < bv) {  // g increases per thread, so '<' keeps the first minimum
      bv = v;
      bi = g;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov < bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  }
  if ((threadIdx.x & 63) == 0) {
    bvs[threadIdx.x >> 6] = bv;
    bis[threadIdx.x >> 6] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w)
      if (bvs[w] < bv || (bvs[w] == bv && bis[w] < bi)) {
        bv = bvs[w];
        bi = bis[w];
      }
    ids[s] = bi;
  }
}

__global__ void temporal_smooth_kernel(const float* __restrict__ x, int rows, int cols, float l1, float l2,
                                       float* __restrict__ y) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)rows * cols) return;
  const int c = (int)(t % cols);
  const float xm = c > 0 ? x[t - 1] : 0.f;
  const float xp = c + 1 < cols ? x[t + 1] : 0.f;
  y[t] = fmaf(l1, xp, fmaf(l2, x[t], l1 * xm));
}

}  // namespace eosv

using namespace eosv;

extern "C" int eosv_temporal_smooth(const float* d_x, int rows, int cols, float lamda1, float lamda2, float* d_y,
                                    eosv_stream_t stream) {
  if (rows < 0 || cols < 0 || ((long long)rows * cols > 0 && (!d_x || !d_y)) || d_x == d_y) {
    set_error("eosv_temporal_smooth: bad argument (in-place not supported)");
    return EOSV_ERR_ARG;
  }
  const long long total = (long long)rows * cols;
  if (total == 0) return EOSV_OK;
  hipLaunchKernelGGL(temporal_smooth_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, d_x, rows, cols, lamda1, lamda2, d_y);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

extern "C" int eosv_match(const float* d_query, const float* d_support, const int32_t* d_sup_off,
                          const int32_t* d_sup_slot, const int32_t* d_n_proto, int n_episodes, int D,
                          int kind, int64_t* d_pred, float* d_score, eosv_stream_t stream) {
  if (n_episodes < 0 || D <= 0 || D > MT * MAXV) {
    set_error("eosv_match: bad n_episodes or D (D must be in 1..2048)");
    return EOSV_ERR_ARG;
  }
  if (n_episodes == 0) return EOSV_OK;
  if (!d_query || !d_support || !d_sup_off || !d_pred) {
    set_error("eosv_match: null pointer");
    return EOSV_ERR_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  if (kind == EOSV_MATCH_PROTONET) {
    if (!d_sup_slot || !d_n_proto) {
      set_error("eosv_match: protonet needs d_sup_slot and d_n_proto");
      return EOSV_ERR_ARG;
    }
    hipLaunchKernelGGL(match_protonet_kernel, dim3(n_episodes), dim3(MT), 0, s, d_query, d_support,
                       d_sup_off, d_sup_slot, d_n_proto, D, (long long*)d_pred, d_score);
  } else if (kind == EOSV_MATCH_COSINE) {
    hipLaunchKernelGGL(match_cosine_kernel, dim3(n_episodes), dim3(MT), 0, s, d_query, d_support,
                       d_sup_off, D, (long long*)d_pred, d_score);
  } else {
    set_error("eosv_match: unknown kind");
    return EOSV_ERR_ARG;
  }
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

extern "C" int eosv_segment_match_episodes(const float* d_seg, int n_episodes, int S, const float* d_gallery,
                                           int G, int D, float lamda1, float lamda2, int64_t* d_ids,
                                           float* d_dist, eosv_stream_t stream) {
  if (n_episodes <= 0 || S <= 0 || G <= 0 || D <= 0 || !d_seg || !d_gallery || !d_ids ||
      (long long)n_episodes * S > 0x7fffffffLL) {
    set_error("eosv_segment_match: bad argument");
    return EOSV_ERR_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  const int R = n_episodes * S;  // all episodes' rows against the one gallery: a grid that fills the chip
  float* raw = nullptr;
  EOSV_HIP_CHECK(hipMallocAsync((void**)&raw, sizeof(float) * (size_t)R * G, s));
  dim3 grid((G + SG_G - 1) / SG_G, (R + SG_S - 1) / SG_S);
  hipLaunchKernelGGL(seg_dist_kernel, grid, dim3(256), 0, s, d_seg, R, d_gallery, G, D, raw);
  hipLaunchKernelGGL(seg_smooth_argmin_kernel, dim3(R), dim3(256), 0, s, raw, S, G, lamda1, lamda2,
                     (long long*)d_ids, d_dist);
  const hipError_t le = hipGetLastError();
  EOSV_HIP_CHECK(hipFreeAsync(raw, s));
  if (le != hipSuccess) {
    set_error(std::string("eosv_segment_match launch: ") + hipGetErrorString(le));
    return EOSV_ERR_HIP;
  }
  return EOSV_OK;
}

extern "C" int eosv_segment_match(const float* d_seg, int S, const float* d_gallery, int G, int D,
                                  float lamda1, float lamda2, int64_t* d_ids, float* d_dist,
                                  eosv_stream_t stream) {
  return eosv_segment_match_episodes(d_seg, 1, S, d_gallery, G, D, lamda1, lamda2, d_ids, d_dist, stream);
}
