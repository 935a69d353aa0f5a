// One-shot matching kernels (the hot-path sink, reference classifier.py / network_test.py).
//
//  match_protonet : classifier.py:9-40 + 43-90 -- per-label prototype = sequential f32
//                   mean in first-appearance order (np.mean over axis 0); scipy cdist
//                   'euclidean' on the f32 inputs: f64 differences, squared and summed
//                   SEQUENTIALLY over d = 0..D-1 with separate multiply and add (scipy's loop;
//                   checked bit-exact, tests/test_cpu_host.py), sqrt, torch.FloatTensor
//                   (f64 -> f32); softmax(-d) over the prototypes (max-subtract, exp, 1/sum,
//                   scale); np.argmax (first max).
//  match_cosine   : classifier.py:117-120 -- sklearn cosine_similarity (rows divided by
//                   their f32 L2 norm, zero norm -> 1) then argsort(-s)[:,0] = first max.
//  segment_match  : network_test.py:207-214 + models.py:42-56 -- cdist(seg, gallery) f64
//                   (sequential, as above) -> f32 -> 3-tap [l1,l2,l1] conv along the flattened
//                   segment axis with zero padding (torch-CPU's k-ordered FMA chain) -> first
//                   argmin over the gallery.
// hipcc contracts a * b + c into an FMA by default (even through __dmul_rn / __dadd_rn): this
// file turns contraction off, so every product scipy rounds separately is rounded here too;
// the smoothing's FMAs are explicit fmaf calls (torch-CPU's conv arithmetic).
// Matching is < 1 % of the path's time; all reductions have a fixed order, so results are
// run-to-run deterministic.
#include <cfloat>

#include "common.h"

#pragma clang fp contract(off)

namespace eosv {

constexpr int MT = 256;
constexpr int MAXV = 8;  // D <= 2048
constexpr int MAXP = 64;
constexpr int PG = 8;    // prototypes per LDS group (8 x 2048 f32 = 64 KiB)

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// One block per episode.  Prototype means are built in parallel (one thread per dimension,
// sequential over the support rows) into LDS, PG prototypes at a time; then lane p of wave 0
// runs prototype p's distance as ONE sequential f64 chain over d, exactly scipy's order.
__global__ __launch_bounds__(MT) void match_protonet_kernel(
    const float* __restrict__ query, const float* __restrict__ sup, const int* __restrict__ sup_off,
    const int* __restrict__ sup_slot, const int* __restrict__ n_proto, int D, long long* __restrict__ pred,
    float* __restrict__ score) {
  __shared__ float qs[MT * MAXV];
  __shared__ float ps[PG][MT * MAXV];
  __shared__ float dist[MAXP];
  const int e = blockIdx.x;
  const int s0 = sup_off[e], s1 = sup_off[e + 1];
  const int P = min(n_proto[e], MAXP);  // eosv_match documents n_way <= 64
  const int tid = threadIdx.x;
  for (int d = tid; d < D; d += MT) qs[d] = query[(long long)e * D + d];
  for (int p0 = 0; p0 < P; p0 += PG) {
    const int np = min(PG, P - p0);
    for (int g = 0; g < np; ++g) {
      float acc[MAXV];
#pragma unroll
      for (int j = 0; j < MAXV; ++j) acc[j] = 0.f;
      int cnt = 0;
      for (int s = s0; s < s1; ++s) {
        if (sup_slot[s] != p0 + g) continue;
        const float* row = sup + (long long)s * D;
        // np.mean(axis=0): the first row is copied, the others added in order
#pragma unroll
        for (int j = 0; j < MAXV; ++j) {
          const int d = tid + MT * j;
          if (d < D) acc[j] = cnt ? acc[j] + row[d] : row[d];
        }
        ++cnt;
      }
      const float fc = (float)cnt;
#pragma unroll
      for (int j = 0; j < MAXV; ++j) {
        const int d = tid + MT * j;
        if (d < D) ps[g][d] = acc[j] / fc;
      }
    }
    __syncthreads();
    if (tid < np) {
      double ss = 0.0;
      for (int d = 0; d < D; ++d) {
        const double diff = (double)qs[d] - (double)ps[tid][d];
        ss = ss + diff * diff;
      }
      dist[p0 + tid] = (float)sqrt(ss);
    }
    __syncthreads();
  }
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
// Fused: distances, smoothing and the first argmin in one pass, no [rows, G] scratch.
// A block owns SG_G gallery columns x SG_S output rows and also computes the rows just above
// and below (the smoothing halo, recomputed by the neighbouring blocks: +3 %).
// dist[s][g] = sqrt(sum_d (seg[s][d] - gal[g][d])^2) in f64, summed sequentially over d
// (d-chunks of SG_DK staged through LDS in order), stored f32; smoothed[s][g] =
// fma(l1, d[s+1][g], fma(l2, d[s][g], l1 * d[s-1][g])) with zeros outside the row's episode;
// per row the (value, column) minimum of the block's columns is merged into ids[s] by a 64-bit
// atomic min on (ordered float key << 32 | g): the key maps the float's bits to an unsigned
// value that orders like the float for either sign (NaN after +inf, as argsort puts it), and
// equal values resolve to the smaller g (np.argsort(...)[:, 0] on ties).
constexpr int SG_G = 64, SG_S = 64, SG_DK = 32;
constexpr int SG_R = SG_S + 2;             // computed rows (halo included)
constexpr int SG_RPT = (SG_R + 3) / 4;     // rows per thread (4 row groups of 64 threads)

__global__ __launch_bounds__(256) void seg_match_kernel(const float* __restrict__ seg, int R, int S,
                                                        const float* __restrict__ gal, int G, int D, float l1,
                                                        float l2, unsigned long long* __restrict__ best,
                                                        float* __restrict__ out) {
  __shared__ float gs[SG_G][SG_DK + 1];
  __shared__ float ss[SG_RPT * 4][SG_DK + 1];
  __shared__ float dl[SG_RPT * 4][SG_G + 1];
  const int g0 = blockIdx.x * SG_G;
  const int r0 = blockIdx.y * SG_S - 1;  // local row 0 = global row r0 (the upper halo)
  const int tid = threadIdx.x;
  const int gl = tid & 63;
  const int rg = tid >> 6;  // thread owns local rows rg + 4 i
  double acc[SG_RPT];
#pragma unroll
  for (int i = 0; i < SG_RPT; ++i) acc[i] = 0.0;
  for (int d0 = 0; d0 < D; d0 += SG_DK) {
    for (int t = tid; t < SG_G * SG_DK; t += 256) {
      const int r = t / SG_DK, c = t % SG_DK;
      const int g = g0 + r, d = d0 + c;
      gs[r][c] = (g < G && d < D) ? gal[(long long)g * D + d] : 0.f;
    }
    for (int t = tid; t < SG_RPT * 4 * SG_DK; t += 256) {
      const int r = t / SG_DK, c = t % SG_DK;
      const int row = r0 + r, d = d0 + c;
      ss[r][c] = (row >= 0 && row < R && d < D) ? seg[(long long)row * D + d] : 0.f;
    }
    __syncthreads();
    const int dn = min(SG_DK, D - d0);
    for (int c = 0; c < dn; ++c) {
      const double gv = (double)gs[gl][c];
#pragma unroll
      for (int i = 0; i < SG_RPT; ++i) {
        const double df = (double)ss[rg + 4 * i][c] - gv;
        acc[i] = acc[i] + df * df;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < SG_RPT; ++i) dl[rg + 4 * i][gl] = (float)sqrt(acc[i]);
  __syncthreads();
  const int g = g0 + gl;
#pragma unroll
  for (int i = 0; i < SG_RPT; ++i) {
    const int lr = rg + 4 * i;  // output local rows 1 .. SG_S
    const int row = r0 + lr;
    if (lr < 1 || lr > SG_S || row >= R) continue;  // wave-uniform
    const int sl = row % S;  // row within its episode
    const float dm = sl > 0 ? dl[lr - 1][gl] : 0.f;
    const float dp = sl + 1 < S ? dl[lr + 1][gl] : 0.f;
    const float v = fmaf(l1, dp, fmaf(l2, dl[lr][gl], l1 * dm));
    if (out && g < G) out[(long long)row * G + g] = v;
    // order-preserving key of the float (negative values, e.g. from lamda1/lamda2 < 0 set in
    // utils, flip all bits; the others get the sign bit), -0 folded into +0 as argsort ties them,
    // and every NaN canonicalised to +qNaN first, so that it keys above +inf whatever its sign
    // (np.argsort puts NaNs last; a negative NaN would otherwise flip below -inf)
    const float vc = v != v ? __uint_as_float(0x7fc00000u) : v;
    const unsigned vb = __float_as_uint(vc == 0.f ? 0.f : vc);
    const unsigned ob = (vb & 0x80000000u) ? ~vb : (vb | 0x80000000u);
    unsigned long long key = g < G ? ((unsigned long long)ob << 32) | (unsigned)g : ~0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long ok = __shfl_xor(key, o, 64);
      key = ok < key ? ok : key;
    }
    if (gl == 0) atomicMin(best + row, key);
  }
}

__global__ void seg_ids_init_kernel(unsigned long long* __restrict__ best, int R) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < R) best[t] = ~0ull;
}

__global__ void seg_ids_final_kernel(unsigned long long* __restrict__ best, int R) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < R) best[t] &= 0xffffffffull;  // keep the column: ids[s] as int64
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
    // n_proto[e] <= 64 (MAXP) is documented in eosv.h; the kernel clamps, it is device data
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
  unsigned long long* best = (unsigned long long*)d_ids;  // the (value, column) keys live in d_ids
  const unsigned nb = (unsigned)((R + 255) / 256);
  hipLaunchKernelGGL(seg_ids_init_kernel, dim3(nb), dim3(256), 0, s, best, R);
  dim3 grid((G + SG_G - 1) / SG_G, (R + SG_S - 1) / SG_S);
  hipLaunchKernelGGL(seg_match_kernel, grid, dim3(256), 0, s, d_seg, R, S, d_gallery, G, D, lamda1, lamda2, best,
                     d_dist);
  hipLaunchKernelGGL(seg_ids_final_kernel, dim3(nb), dim3(256), 0, s, best, R);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

extern "C" int eosv_segment_match(const float* d_seg, int S, const float* d_gallery, int G, int D,
                                  float lamda1, float lamda2, int64_t* d_ids, float* d_dist,
                                  eosv_stream_t stream) {
  return eosv_segment_match_episodes(d_seg, 1, S, d_gallery, G, D, lamda1, lamda2, d_ids, d_dist, stream);
}
