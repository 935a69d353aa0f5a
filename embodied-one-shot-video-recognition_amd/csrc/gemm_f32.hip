// Plain f32 GEMMs of the training step on exact-f32 MFMA (the GEMM parts of
// model(video) in train mode and of loss.backward(), reference network_train.py:98-116), in
// place of the rocBLAS sgemm the round-2..4 library linked:
//   * stem forward       Y[P][64]      = Xcol[P][147] . W[64][147]^T             (NT)
//   * strided-conv dgrad dXcol[P][K]   = dY[P][Cout] . W[Cout][K]                (NN, then col2im)
//   * 1x1 / stem wgrad   dW[Cout][K]   = dY[P][Cout]^T . Xcol[P][K]              (TN, split over P)
//   * fc                 logits = F W^T (NT), dW = dlogits^T F (TN), dF = dlogits W (NN)
//
//   C[m][n] = alpha * sum_k opA(m, k) opB(k, n) + beta * C[m][n]       (row-major, beta 0: C unread)
//   opA(m, k) = TA ? A[k][m] : A[m][k],  opB(k, n) = TB ? B[n][k] : B[k][n]
//
// One workgroup computes a BM x BN tile (WM x WN waves of 64 x 64) over a slice of the reduction;
// a k-step stages 16 reduction rows of both operands through registers into a double-buffered
// LDS tile stored k-major ([16][BM] and [16][BN]; the operand whose k is contiguous in memory is
// transposed on the way in), one barrier per step, and the next step's global loads are in flight
// while the current one feeds the MFMAs.  v_mfma_f32_16x16x4_f32 with k as the reduction index:
// lane l's A element is opA(64 wm + 4 (l % 16) + i, 4 s + l / 16) for block i of its 4 m-blocks,
// and likewise for B, so ONE ds_read_b128 per operand feeds the 16 MFMAs of a sub-step and the
// epilogue writes runs of 4 consecutive n (the wgrad_f32 layout).  Split-K: slice s writes its raw
// partial tile to a workspace, summed afterwards in slice order with the alpha / beta epilogue
// (deterministic, no atomics).  Every k is summed in increasing order within a slice.
#include "common.h"

#include <algorithm>

namespace eosv {

namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifndef EOSV_GEMM_AHEAD_DEF
#define EOSV_GEMM_AHEAD_DEF 1
#endif
constexpr int GB_K = 16;    // reduction rows per k-step
constexpr int GB_PAD = 16;  // floats of LDS row padding

struct GemmArgs {
  const float* a;
  const float* b;
  float* c;      // C, or the [slices][m][n] partials when slices > 1
  long long lda, ldb, ldc;
  int m, n, k;
  int kps;       // reduction rows per slice (multiple of GB_K unless one slice)
  int mt, nt;    // tiles along m and n
  float alpha, beta;
  int va, vb, vc;  // float4 access allowed on A / B / C (leading dimension % 4 == 0, 16-B aligned)
  int partial;     // 1: raw partial sums to c[slice][m][n], no epilogue
};

// 4 consecutive elements of a row-major operand starting at (r, c) of a rows x cols view (zeros
// outside); vec: one 16-byte load when all 4 are inside
__device__ __forceinline__ f32x4 load4(const float* __restrict__ p, long long ld, long long r, long long c, long long rows,
                                       long long cols, bool vec) {
  if (r >= rows) return f32x4{0.f, 0.f, 0.f, 0.f};
  const float* q = p + r * ld + c;
  if (vec && c + 3 < cols) return *(const f32x4*)q;
  f32x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = c + i < cols ? q[i] : 0.f;
  return v;
}

template <int WM, int WN, bool TA, bool TB, int AHEAD>
__global__ __launch_bounds__(64 * WM * WN) void gemm_f32_kernel(GemmArgs g) {
  constexpr int NT = 64 * WM * WN, BM = 64 * WM, BN = 64 * WN;
  constexpr int LA = BM + GB_PAD, LB = BN + GB_PAD;
  constexpr int P4A = GB_K * BM / 4, P4B = GB_K * BN / 4;  // float4 pieces per step
  constexpr int AS = (P4A + NT - 1) / NT, BS = (P4B + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) float lds[2][GB_K * (LA + LB)];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - WN * (wave / WN);
  const int tile = blockIdx.x;
  const int tn = tile % g.nt, tm = tile / g.nt;
  const long long m0 = (long long)tm * BM, n0 = (long long)tn * BN;
  const long long k0 = (long long)blockIdx.y * g.kps;
  const long long k1 = min((long long)g.k, k0 + g.kps);
  const int steps = (int)((k1 - k0 + GB_K - 1) / GB_K);

  // piece -> (row, float4 column) of the operand as stored: TA: A rows are k (BM / 4 pieces per
  // row), else A rows are m (GB_K / 4 pieces per row); B likewise (TB: rows are n)
  // AHEAD register sets: a step's operands are loaded AHEAD k-steps before it runs.  1 (default):
  // 2 was 10 % slower over the R50 finetune shapes (tools/bench_gemm.py, r05: 3.54 vs 3.91 ms; its
  // second register set costs occupancy), with 8 waves per CU of split-K workgroups hiding the latency
  static_assert(AHEAD == 1 || AHEAD == 2, "prefetch depth");
  f32x4 ra2[AHEAD][AS], rb2[AHEAD][BS];
  auto load = [&](int step, int set) {
    f32x4 (&ra)[AS] = ra2[set];
    f32x4 (&rb)[BS] = rb2[set];
    const long long kb = k0 + (long long)step * GB_K;
#pragma unroll
    for (int s = 0; s < AS; ++s) {
      const int idx = tid + s * NT;
      ra[s] = f32x4{0.f, 0.f, 0.f, 0.f};
      if ((s + 1) * NT <= P4A || idx < P4A) {
        if (TA) {  // A [k][m]: row kb + r, columns m0 + 4 c ..
          const int r = idx / (BM / 4), c = idx - (BM / 4) * r;
          ra[s] = load4(g.a, g.lda, kb + r, m0 + 4 * c, k1, g.m, g.va);
        } else {  // A [m][k]: row m0 + r, columns kb + 4 c ..
          const int r = idx / (GB_K / 4), c = idx - (GB_K / 4) * r;
          ra[s] = load4(g.a, g.lda, m0 + r, kb + 4 * c, g.m, k1, g.va);
        }
      }
    }
#pragma unroll
    for (int s = 0; s < BS; ++s) {
      const int idx = tid + s * NT;
      rb[s] = f32x4{0.f, 0.f, 0.f, 0.f};
      if ((s + 1) * NT <= P4B || idx < P4B) {
        if (!TB) {  // B [k][n]
          const int r = idx / (BN / 4), c = idx - (BN / 4) * r;
          rb[s] = load4(g.b, g.ldb, kb + r, n0 + 4 * c, k1, g.n, g.vb);
        } else {  // B [n][k]
          const int r = idx / (GB_K / 4), c = idx - (GB_K / 4) * r;
          rb[s] = load4(g.b, g.ldb, n0 + r, kb + 4 * c, g.n, k1, g.vb);
        }
      }
    }
  };
  auto store = [&](int buf, int set) {
    const f32x4 (&ra)[AS] = ra2[set];
    const f32x4 (&rb)[BS] = rb2[set];
    float* LAp = lds[buf];
    float* LBp = lds[buf] + GB_K * LA;
#pragma unroll
    for (int s = 0; s < AS; ++s) {
      const int idx = tid + s * NT;
      if ((s + 1) * NT <= P4A || idx < P4A) {
        if (TA) {
          const int r = idx / (BM / 4), c = idx - (BM / 4) * r;
          *(f32x4*)(LAp + r * LA + 4 * c) = ra[s];
        } else {  // transpose: element i is k = 4 c + i of row m = r
          const int r = idx / (GB_K / 4), c = idx - (GB_K / 4) * r;
#pragma unroll
          for (int i = 0; i < 4; ++i) LAp[(4 * c + i) * LA + r] = ra[s][i];
        }
      }
    }
#pragma unroll
    for (int s = 0; s < BS; ++s) {
      const int idx = tid + s * NT;
      if ((s + 1) * NT <= P4B || idx < P4B) {
        if (!TB) {
          const int r = idx / (BN / 4), c = idx - (BN / 4) * r;
          *(f32x4*)(LBp + r * LB + 4 * c) = rb[s];
        } else {
          const int r = idx / (GB_K / 4), c = idx - (GB_K / 4) * r;
#pragma unroll
          for (int i = 0; i < 4; ++i) LBp[(4 * c + i) * LB + r] = rb[s][i];
        }
      }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int q = lane >> 4, c = lane & 15;
  if (steps > 0) {
    load(0, 0);
    store(0, 0);
    if (steps > 1) load(1, AHEAD - 1);
    if (AHEAD == 2 && steps > 2) load(2, 0);
    __syncthreads();
  }
  for (int step = 0; step < steps; ++step) {
    const int cur = step & 1;
    const float* LAp = lds[cur];
    const float* LBp = lds[cur] + GB_K * LA;
#pragma unroll
    for (int ss = 0; ss < GB_K / 4; ++ss) {
      const int r = 4 * ss + q;
      const f32x4 av = *(const f32x4*)(LAp + r * LA + 64 * wm + 4 * c);
      const f32x4 bv = *(const f32x4*)(LBp + r * LB + 64 * wn + 4 * c);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    // step + 1's operands (loaded AHEAD - 1 steps ago, or in the prologue) -> the other LDS
    // buffer; their register set then takes step + 1 + AHEAD's
    const int set = AHEAD == 2 ? (cur ^ 1) : 0;
    if (step + 1 < steps) store(cur ^ 1, set);
    if (step + 1 + AHEAD < steps) load(step + 1 + AHEAD, set);
    __syncthreads();
  }

  // lane holds D[4q + rr][c] of block (i, j): m = m0 + 64 wm + 4 (4q + rr) + i, n = n0 + 64 wn + 4c + j
  const long long nb = n0 + 64 * wn + 4 * c;
  float* out = g.partial ? g.c + (long long)blockIdx.y * g.m * g.n : g.c;
  const long long ldo = g.partial ? g.n : g.ldc;
  const bool vec = (g.partial ? (g.n & 3) == 0 : g.vc != 0) && nb + 3 < g.n;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long long m = m0 + 64 * wm + 4 * (4 * q + rr) + i;
      if (m >= g.m) continue;
      float* o = out + m * ldo + nb;
      f32x4 v{acc[i][0][rr], acc[i][1][rr], acc[i][2][rr], acc[i][3][rr]};
      if (!g.partial) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] *= g.alpha;
          if (g.beta != 0.f && nb + j < g.n) v[j] += g.beta * o[j];
        }
      }
      if (vec) {
        *(f32x4*)o = v;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (nb + j < g.n) o[j] = v[j];
      }
    }
}

// C[m][n] = alpha * sum over slices (in slice order) of w[s][m][n] + beta * C; 4 consecutive
// elements per thread (n % 4 == 0: one float4 per slice), 8 slices' loads in flight before their
// adds (the adds stay in slice order)
template <bool V4>
__global__ void gemm_slice_sum_kernel(const float* __restrict__ w, int slices, int m, int n, float alpha, float beta,
                                      float* __restrict__ c, long long ldc) {
  const long long mn = (long long)m * n;
  for (long long i = 4 * (blockIdx.x * (long long)blockDim.x + threadIdx.x); i < mn;
       i += 4 * (long long)gridDim.x * blockDim.x) {
    f32x4 s{0.f, 0.f, 0.f, 0.f};
    int j = 0;
    for (; j + 8 <= slices; j += 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float* p = w + (j + u) * mn + i;
        if (V4) {
          v[u] = *(const f32x4*)p;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[u][e] = i + e < mn ? p[e] : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; j < slices; ++j) {
      const float* p = w + j * mn + i;
      if (V4) {
        s += *(const f32x4*)p;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) s[e] += i + e < mn ? p[e] : 0.f;
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (i + e >= mn) break;
      const long long r = (i + e) / n, col = (i + e) - r * n;
      float* o = c + r * ldc + col;
      *o = beta != 0.f ? alpha * s[e] + beta * *o : alpha * s[e];
    }
  }
}

struct GemmPlan {
  int wm, wn, mt, nt, slices, kps;
};

// tile: 128 x 128 (2 x 2 waves) when both dimensions reach 128, else the 64-wide side where one
// is short (64 x 128, 128 x 64, 64 x 64); split-K (when allowed) so that tiles x slices is about 2
// workgroups per CU with at least 1024 reduction rows per slice and at most 256 slices (the
// slice sum re-reads slices x m x n floats)
GemmPlan gemm_plan(int m, int n, int k, bool split) {
  GemmPlan p{};
  p.wm = m > 64 ? 2 : 1;
  p.wn = n > 64 ? 2 : 1;
  p.mt = (m + 64 * p.wm - 1) / (64 * p.wm);
  p.nt = (n + 64 * p.wn - 1) / (64 * p.wn);
  const long long tiles = (long long)p.mt * p.nt;
  long long s = 1;
  if (split) {
    // enough workgroups for `wpc` waves per CU (latency hiding: a 64-wide tile has 2 waves), at least
    // `minrows` reduction rows per slice, at most 1024 slices (the slice sum re-reads slices x m x n)
    static const int wpc = env_switch("EOSV_GEMM_WPC", 8);
    static const int minrows = env_switch("EOSV_GEMM_MINROWS", 256);
    const long long target = (long long)wpc * device_cu_count() / (p.wm * p.wn);
    s = std::max(1LL, std::min((target + tiles - 1) / tiles, (long long)k / minrows));
    s = std::min<long long>(s, 1024);
  }
  long long kps = (k + s - 1) / s;
  if (s > 1) kps = (kps + GB_K - 1) / GB_K * GB_K;
  p.kps = (int)std::max(1LL, kps);
  p.slices = (int)((k + p.kps - 1) / p.kps);
  if (p.slices < 1) p.slices = 1;
  return p;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

int launch_gemm(bool ta, bool tb, int m, int n, int k, float alpha, const float* a, long long lda, const float* b,
                long long ldb, float beta, float* c, long long ldc, float* work, long long work_bytes, bool split,
                hipStream_t s) {
  GemmPlan p = gemm_plan(m, n, k, split);
  if (p.slices > 1 && (!work || work_bytes < (long long)p.slices * m * n * (long long)sizeof(float) || !aligned16(work)))
    p = gemm_plan(m, n, k, false);
  if ((long long)p.mt * p.nt > 0x7fffffffLL || p.slices > 65535)
    return set_error("eosv_sgemm: grid too large"), EOSV_ERR_UNSUPPORTED;
  GemmArgs g{};
  g.a = a, g.b = b, g.lda = lda, g.ldb = ldb, g.ldc = ldc;
  g.m = m, g.n = n, g.k = k, g.kps = p.kps, g.mt = p.mt, g.nt = p.nt;
  g.alpha = alpha, g.beta = beta;
  g.va = (lda % 4 == 0) && aligned16(a);
  g.vb = (ldb % 4 == 0) && aligned16(b);
  g.vc = (ldc % 4 == 0) && aligned16(c);
  g.partial = p.slices > 1;
  g.c = g.partial ? work : c;
  const dim3 grid((unsigned)(p.mt * p.nt), (unsigned)p.slices), blk(64 * p.wm * p.wn);
  static const int ahead = env_switch("EOSV_GEMM_AHEAD", EOSV_GEMM_AHEAD_DEF) == 1 ? 1 : 2;  // (A/B switch)
  const int sel = ((p.wm * 2 + p.wn) * 4 + (ta ? 2 : 0) + (tb ? 1 : 0)) * 2 + (ahead - 1);
#define EOSV_GEMM_CASE1(WM, WN, TA, TB, AH)                                                   \
  case (((WM * 2 + WN) * 4 + (TA ? 2 : 0) + (TB ? 1 : 0)) * 2 + AH - 1):                     \
    hipLaunchKernelGGL((gemm_f32_kernel<WM, WN, TA, TB, AH>), grid, blk, 0, s, g);           \
    break;
#define EOSV_GEMM_CASE(WM, WN, TA, TB) EOSV_GEMM_CASE1(WM, WN, TA, TB, 1) EOSV_GEMM_CASE1(WM, WN, TA, TB, 2)
#define EOSV_GEMM_TILE(WM, WN) \
  EOSV_GEMM_CASE(WM, WN, false, false) EOSV_GEMM_CASE(WM, WN, false, true) EOSV_GEMM_CASE(WM, WN, true, false) \
  EOSV_GEMM_CASE(WM, WN, true, true)
  switch (sel) {
    EOSV_GEMM_TILE(1, 1)
    EOSV_GEMM_TILE(1, 2)
    EOSV_GEMM_TILE(2, 1)
    EOSV_GEMM_TILE(2, 2)
    default: return set_error("eosv_sgemm: no tile"), EOSV_ERR_UNSUPPORTED;
  }
#undef EOSV_GEMM_TILE
#undef EOSV_GEMM_CASE
#undef EOSV_GEMM_CASE1
  EOSV_LAUNCH_CHECK();
  if (g.partial) {
    const long long mn = (long long)m * n;
    const dim3 sg((unsigned)std::min<long long>((mn / 4 + 255) / 256 + 1, 1 << 16));
    if (n % 4 == 0)
      hipLaunchKernelGGL(gemm_slice_sum_kernel<true>, sg, dim3(256), 0, s, work, p.slices, m, n, alpha, beta, c, ldc);
    else
      hipLaunchKernelGGL(gemm_slice_sum_kernel<false>, sg, dim3(256), 0, s, work, p.slices, m, n, alpha, beta, c, ldc);
    EOSV_LAUNCH_CHECK();
  }
  return EOSV_OK;
}
}  // namespace

}  // namespace eosv

using namespace eosv;

extern "C" {

int eosv_sgemm(int trans_a, int trans_b, int m, int n, int k, float alpha, const float* d_a, int lda,
               const float* d_b, int ldb, float beta, float* d_c, int ldc, eosv_stream_t stream) {
  if (m < 0 || n < 0 || k < 0 || !d_c || (k > 0 && (!d_a || !d_b)) || lda <= 0 || ldb <= 0 || ldc < n ||
      lda < (trans_a ? m : k) || ldb < (trans_b ? k : n))
    return set_error("eosv_sgemm: bad argument"), EOSV_ERR_ARG;
  if (m == 0 || n == 0) return EOSV_OK;
  return launch_gemm(trans_a != 0, trans_b != 0, m, n, k, alpha, d_a, lda, d_b, ldb, beta, d_c, ldc, nullptr, 0, false,
                     (hipStream_t)stream);
}

int64_t eosv_sgemm_tn_splitk_workspace(int m, int n, int k) {
  if (m <= 0 || n <= 0 || k <= 0) return 0;
  const GemmPlan p = gemm_plan(m, n, k, true);
  return p.slices > 1 ? (int64_t)p.slices * m * n * (int64_t)sizeof(float) : 0;
}

int eosv_sgemm_tn_splitk(int m, int n, int k, const float* d_a, int lda, const float* d_b, int ldb, float* d_c,
                         int ldc, float* d_work, int64_t work_bytes, eosv_stream_t stream) {
  if (m <= 0 || n <= 0 || k <= 0 || !d_a || !d_b || !d_c || lda < m || ldb < n || ldc != n)
    return set_error("eosv_sgemm_tn_splitk: bad argument"), EOSV_ERR_ARG;
  return launch_gemm(true, false, m, n, k, 1.f, d_a, lda, d_b, ldb, 0.f, d_c, ldc, d_work, work_bytes, true,
                     (hipStream_t)stream);
}

}  // extern "C"
