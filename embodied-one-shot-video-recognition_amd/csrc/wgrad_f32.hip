// Weight gradient of a KxK convolution (training path, SURVEY 8(f) f4: the conv part of
// loss.backward(), reference network_train.py:114) as an implicit GEMM, without the im2col
// buffer:
//
//   dW[co][(kh, kw, ci)] = sum over pixels p of dY[p][co] * X[in(p, kh, kw)][ci]
//
// (NHWC activations, P = N*Ho*Wo output pixels, zero outside the input).  The pixel reduction
// is split into slices so that (Cout / BM) x (K / BN) tiles x slices fill the chip; each slice
// writes its partial tile to a workspace, summed afterwards in slice order (deterministic).
//
// Per workgroup: a BM (co) x BN (k) tile, WM x WN waves of 64 x 64.  A k-step stages 16 pixels:
// dY [16][BM] (contiguous rows) and the gathered X [16][BN] (row p, column k -> input pixel
// (oh*s - pad + kh, ow*s - pad + kw), channel ci; zero when outside) through registers into a
// double-buffered LDS tile, one barrier per step.  MFMA v_mfma_f32_16x16x4_f32 with the pixel
// as the reduction index: lane l's A element is dY[p = 4s + l/16][co] and its B element
// X[p][k].  Block i of the wave's 4 co-blocks takes co = 4m + i (m = l % 16) and block j of its
// 4 k-blocks k = 4n + j, so ONE ds_read_b128 per operand feeds all 16 MFMAs of a sub-step, and
// the epilogue stores float4 runs of 4 consecutive k.
#include "common.h"

#include <algorithm>

namespace eosv {

namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int WG_BP = 16;   // pixels per k-step
constexpr int WG_PAD = 16;  // floats of LDS row padding (row groups on distinct banks)

struct WgradArgs {
  const float* x;   // [N][H][W][Cin]
  const float* dy;  // [P][Cout]
  float* out;       // [slices][Cout][K]
  int N, H, W, Cin, Ho, Wo, Cout, KW, stride, pad, K;
  long long P, rows_per_slice;  // rows_per_slice % WG_BP == 0
  int co_tiles, k_tiles;
};

template <int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void wgrad_f32_kernel(WgradArgs a) {
  constexpr int NT = 64 * WM * WN, BM = 64 * WM, BN = 64 * WN;
  constexpr int LA = BM + WG_PAD, LB = BN + WG_PAD;
  constexpr int A4 = WG_BP * BM / 4, B4 = WG_BP * BN / 4;  // float4 pieces per step
  constexpr int AS = (A4 + NT - 1) / NT, BS = (B4 + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) float lds[2][WG_BP * (LA + LB)];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - WN * (wave / WN);
  // block -> (slice, co tile, k tile); tiles vary fastest, so co-resident blocks share a slice
  int b = blockIdx.x;
  const int kt = b % a.k_tiles;
  b /= a.k_tiles;
  const int ct = b % a.co_tiles;
  const long long slice = b / a.co_tiles;
  const int co0 = ct * BM, k0 = kt * BN;
  const long long p0 = slice * a.rows_per_slice;
  const long long p1 = min(a.P, p0 + a.rows_per_slice);
  const int steps = (int)((p1 - p0 + WG_BP - 1) / WG_BP);

  // A pieces: row r, float4 column c of dY
  int ar[AS], ac[AS];
#pragma unroll
  for (int s = 0; s < AS; ++s) {
    const int idx = tid + s * NT;
    ar[s] = idx / (BM / 4);
    ac[s] = idx - (BM / 4) * ar[s];
  }
  // B pieces: row r (its pixel tracked incrementally), tap and channel of its 4 columns
  int br[BS], bkh[BS], bkw[BS], bci[BS], bimg[BS], boh[BS], bow[BS];
#pragma unroll
  for (int s = 0; s < BS; ++s) {
    const int idx = tid + s * NT;
    br[s] = idx / (BN / 4);
    const int k = k0 + 4 * (idx - (BN / 4) * br[s]);
    const int t = k / a.Cin;
    bci[s] = k - t * a.Cin;
    bkh[s] = t / a.KW;
    bkw[s] = t - a.KW * bkh[s];
    const long long p = p0 + br[s];
    const long long hw = (long long)a.Ho * a.Wo;
    bimg[s] = (int)(p / hw);
    const int rem = (int)(p - hw * bimg[s]);
    boh[s] = rem / a.Wo;
    bow[s] = rem - a.Wo * boh[s];
  }

  f32x4 ra[AS], rb[BS];
  auto load = [&](int step) {
    const long long pb = p0 + (long long)step * WG_BP;
#pragma unroll
    for (int s = 0; s < AS; ++s) {
      const long long p = pb + ar[s];
      ra[s] = f32x4{0.f, 0.f, 0.f, 0.f};
      if ((s + 1) * NT <= A4 || tid + s * NT < A4)
        if (p < p1) ra[s] = *(const f32x4*)(a.dy + p * a.Cout + co0 + 4 * ac[s]);
    }
#pragma unroll
    for (int s = 0; s < BS; ++s) {
      rb[s] = f32x4{0.f, 0.f, 0.f, 0.f};
      if ((s + 1) * NT <= B4 || tid + s * NT < B4) {
        const int ih = boh[s] * a.stride - a.pad + bkh[s], iw = bow[s] * a.stride - a.pad + bkw[s];
        if (pb + br[s] < p1 && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
          rb[s] = *(const f32x4*)(a.x + (((long long)bimg[s] * a.H + ih) * a.W + iw) * a.Cin + bci[s]);
        // next step: 16 pixels on
        int ow = bow[s] + WG_BP, oh = boh[s], img = bimg[s];
        while (ow >= a.Wo) {
          ow -= a.Wo;
          if (++oh == a.Ho) oh = 0, ++img;
        }
        bow[s] = ow, boh[s] = oh, bimg[s] = img;
      }
    }
  };
  auto store = [&](int buf) {
    float* L = lds[buf];
#pragma unroll
    for (int s = 0; s < AS; ++s)
      if ((s + 1) * NT <= A4 || tid + s * NT < A4) *(f32x4*)(L + ar[s] * LA + 4 * ac[s]) = ra[s];
#pragma unroll
    for (int s = 0; s < BS; ++s)
      if ((s + 1) * NT <= B4 || tid + s * NT < B4) *(f32x4*)(L + WG_BP * LA + br[s] * LB + 4 * (tid + s * NT - (BN / 4) * br[s])) = rb[s];
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int q = lane >> 4, c = lane & 15;
  if (steps > 0) {
    load(0);
    store(0);
    __syncthreads();
  }
  for (int step = 0; step < steps; ++step) {
    const int cur = step & 1;
    if (step + 1 < steps) load(step + 1);
    const float* L = lds[cur];
#pragma unroll
    for (int ss = 0; ss < WG_BP / 4; ++ss) {
      const int r = 4 * ss + q;
      const f32x4 av = *(const f32x4*)(L + r * LA + 64 * wm + 4 * c);
      const f32x4 bv = *(const f32x4*)(L + WG_BP * LA + r * LB + 64 * wn + 4 * c);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (step + 1 < steps) store(cur ^ 1);
    __syncthreads();
  }

  // lane holds D[m = 4q + rr][n = c] of block (i, j): co = co0 + 64 wm + 4 m + i, k = k0 + 64 wn + 4 n + j
  float* o = a.out + slice * (long long)a.Cout * a.K;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = co0 + 64 * wm + 4 * (4 * q + rr) + i;
      const int k = k0 + 64 * wn + 4 * c;
      *(float4*)(o + (long long)co * a.K + k) = make_float4(acc[i][0][rr], acc[i][1][rr], acc[i][2][rr], acc[i][3][rr]);
    }
}

struct WgradPlan {
  int wm, wn, co_tiles, k_tiles;
  long long slices, rows;
};

// tile: the first of 128 x 128 (2 x 2 waves), 64 x 256, 64 x 192, 128 x 64, 64 x 128, 64 x 64 that
// divides (Cout, K); slices so that tiles x slices is ~4 blocks per CU, at least 256 pixel rows each
bool wgrad_plan(int Cout, int K, long long P, WgradPlan* pl) {
  static const int cand[][2] = {{2, 2}, {1, 4}, {1, 3}, {2, 1}, {1, 2}, {1, 1}};
  bool ok = false;
  for (const auto& c : cand)
    if (Cout % (64 * c[0]) == 0 && K % (64 * c[1]) == 0) {
      pl->wm = c[0], pl->wn = c[1];
      ok = true;
      break;
    }
  if (!ok) return false;
  pl->co_tiles = Cout / (64 * pl->wm);
  pl->k_tiles = K / (64 * pl->wn);
  const long long tiles = (long long)pl->co_tiles * pl->k_tiles;
  const long long target = 4LL * device_cu_count();
  long long s = (target + tiles - 1) / tiles;
  s = std::max(1LL, std::min(s, P / 256));
  long long rows = (P + s - 1) / s;
  rows = (rows + WG_BP - 1) / WG_BP * WG_BP;
  pl->rows = rows;
  pl->slices = (P + rows - 1) / rows;
  return true;
}

__global__ void wgrad_sum_kernel(const float* __restrict__ w, long long slices, long long mn, float* __restrict__ c) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < mn; i += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (long long j = 0; j < slices; ++j) s += w[j * mn + i];
    c[i] = s;
  }
}
}  // namespace

}  // namespace eosv

using namespace eosv;

extern "C" {

int64_t eosv_conv_wgrad_f32_workspace(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad) {
  if (N <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0 || KH <= 0 || KW <= 0 || stride <= 0 || pad < 0) return 0;
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  if (Ho <= 0 || Wo <= 0 || Cin % 4) return 0;
  WgradPlan pl;
  if (!wgrad_plan(Cout, KH * KW * Cin, (long long)N * Ho * Wo, &pl)) return 0;
  return pl.slices > 1 ? pl.slices * (int64_t)Cout * KH * KW * Cin * (int64_t)sizeof(float) : 0;
}

int eosv_conv_wgrad_f32(const float* d_x, int N, int H, int W, int Cin, const float* d_dy, int Cout, int KH, int KW,
                        int stride, int pad, float* d_dw, float* d_work, int64_t work_bytes, eosv_stream_t stream) {
  if (!d_x || !d_dy || !d_dw || N <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0 || KH <= 0 || KW <= 0 ||
      stride <= 0 || pad < 0)
    return set_error("eosv_conv_wgrad_f32: bad argument"), EOSV_ERR_ARG;
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  if (Ho <= 0 || Wo <= 0) return set_error("eosv_conv_wgrad_f32: empty output"), EOSV_ERR_ARG;
  const int K = KH * KW * Cin;
  WgradPlan pl;
  if (Cin % 4 || ((uintptr_t)d_x | (uintptr_t)d_dy | (uintptr_t)d_dw) & 15 || !wgrad_plan(Cout, K, (long long)N * Ho * Wo, &pl))
    return set_error("eosv_conv_wgrad_f32: needs Cin % 4 == 0, 16-byte aligned operands, Cout % 64 == 0 and "
                     "K % 64 == 0"),
           EOSV_ERR_UNSUPPORTED;
  const int64_t need = eosv_conv_wgrad_f32_workspace(N, H, W, Cin, Cout, KH, KW, stride, pad);
  if (need > 0 && (!d_work || work_bytes < need || ((uintptr_t)d_work & 15)))
    return set_error("eosv_conv_wgrad_f32: workspace too small"), EOSV_ERR_ARG;
  WgradArgs a{};
  a.x = d_x, a.dy = d_dy, a.out = pl.slices > 1 ? d_work : d_dw;
  a.N = N, a.H = H, a.W = W, a.Cin = Cin, a.Ho = Ho, a.Wo = Wo, a.Cout = Cout, a.KW = KW, a.stride = stride,
  a.pad = pad, a.K = K;
  a.P = (long long)N * Ho * Wo, a.rows_per_slice = pl.rows, a.co_tiles = pl.co_tiles, a.k_tiles = pl.k_tiles;
  const long long blocks = pl.slices * pl.co_tiles * pl.k_tiles;
  if (blocks > 0x7fffffffLL) return set_error("eosv_conv_wgrad_f32: grid too large"), EOSV_ERR_UNSUPPORTED;
  const hipStream_t s = (hipStream_t)stream;
  const dim3 g((unsigned)blocks), b(64 * pl.wm * pl.wn);
  switch (pl.wm * 10 + pl.wn) {
    case 22: hipLaunchKernelGGL((wgrad_f32_kernel<2, 2>), g, b, 0, s, a); break;
    case 14: hipLaunchKernelGGL((wgrad_f32_kernel<1, 4>), g, b, 0, s, a); break;
    case 13: hipLaunchKernelGGL((wgrad_f32_kernel<1, 3>), g, b, 0, s, a); break;
    case 21: hipLaunchKernelGGL((wgrad_f32_kernel<2, 1>), g, b, 0, s, a); break;
    case 12: hipLaunchKernelGGL((wgrad_f32_kernel<1, 2>), g, b, 0, s, a); break;
    default: hipLaunchKernelGGL((wgrad_f32_kernel<1, 1>), g, b, 0, s, a); break;
  }
  EOSV_LAUNCH_CHECK();
  if (pl.slices > 1) {
    const long long mn = (long long)Cout * K;
    hipLaunchKernelGGL(wgrad_sum_kernel, dim3((unsigned)std::min<long long>((mn + 255) / 256, 1 << 20)), dim3(256), 0, s,
                       d_work, pl.slices, mn, d_dw);
    EOSV_LAUNCH_CHECK();
  }
  return EOSV_OK;
}

}  // extern "C"
