// Phased implicit-GEMM conv on bf16 MFMA for the large-tile layers (Cout >= 128, K >= 128):
// ResNet layer2-4 3x3 convs, their stride-2 entries and 1x1 downsamples, R50 bottleneck 1x1s.
//
// Same GEMM view and LDS image as conv_bf16.hip (M = output pixels, N = Cout, K = (kh, kw, cin);
// im2col never materialised; A and B rows of BK = 64 bf16 = 128 B, 16-B chunk c of row r stored
// at c ^ ((r >> 1) & 7), the XOR applied on the LDS-DMA source address).  What differs is the
// schedule, which follows the staggered 8-wave template of cdna_hip_programming.md §5 ("The 256²
// 8-phase template"):
//   * 8 waves, each owning a 128 x 64 output tile (8 x 4 tiles of v_mfma_f32_16x16x32_bf16);
//     a 256 x 256 block (Cout >= 256) or a 512 x 128 block (Cout = 128: all 160 KiB of LDS).
//   * each K-tile is 4 phases; a phase = LOAD segment (ds_read the fragments one C-quadrant
//     needs, issue a share of the next K-tile's LDS-DMA, lgkmcnt(0)) | s_barrier | MFMA
//     segment (16 MFMAs) | s_barrier.  Quadrants in the order (A0-3,B0-1) (B2-3) (A4-7) (B0-1)
//     reuse the registers already loaded: 12, 4, 8, 4 ds_read_b128 per phase.
//   * waves 4-7 (the SIMD partners of waves 0-3) run one barrier behind, so on every SIMD one
//     wave is in its MFMA segment while its partner reads LDS and issues DMA.
//   * 2 LDS buffers, each K-tile staged as 4 half-tiles: A-top (the A0-3 rows of every wave
//     row), B-left (B0-1), B-right (B2-3), A-bottom (A4-7); every wave issues the same number of
//     DMA pieces of each.  K-tile t+1's half-tiles go out one per phase of K-tile t, in the order
//     its phases consume them, and each is retired by a COUNTED vmcnt one phase before its first
//     reader (3 half-tiles stay in flight across the barriers, cdna_hip_programming.md T3+T4):
//     a half-tile gets ~4 phases of MFMA time to land instead of ~2.5 with the former
//     "all of t+1 in phases 0-1, vmcnt(0) in phase 3" (EOSV_P8_PIPE=0 keeps that for A/B).
//     WAR: a region of buffer (t+1)&1 is re-staged 3+ barriers after its last LOAD segment in
//     K-tile t-1 (waves 4-7 trail by one); RAW: each wait sits before a barrier that every
//     reader passes before its first ds_read of the region.
//   * s_setprio(1) around each MFMA segment (T5; EOSV_P8_PRIO=0 drops it).
// Epilogue as conv_bf16.hip: bias (+ residual) (+ ReLU) through an LDS-staged f32 tile so that
// residual loads and output stores are 16 B per lane.
#include <hip/hip_bf16.h>

#include "common.h"

namespace eosv {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __bfloat16_as_ushort(__float2bfloat16(f)); }
}  // namespace

// SPLIT: EOSV_F32X3 epilogue (ConvArgs::split), as in conv_bf16.hip
template <int BM, int BN, int WM, int WN, bool DS, bool SPLIT = false>
__global__ __launch_bounds__(512) void conv_bf16_p8_kernel(ConvArgs a) {
  constexpr int BK = 64;
  constexpr int NW = 8;
  static_assert(WM * WN == NW && BM / WM == 128 && BN / WN == 64, "8 waves of 128 x 64");
  constexpr int AI = BM / (8 * NW);  // A DMA instructions per wave per K-tile
  constexpr int BI = BN / (8 * NW);
  constexpr int STAGE = (BM + BN) * BK;  // bf16 elements per buffer
  static_assert(2 * STAGE * 2 <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) u16 smem[2 * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: DMA bases stay scalar
  const int half = wid >> 2;  // waves w and w + 4 share a SIMD
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int HoWo = a.Ho * a.Wo;
  const int M = a.N * HoWo;
  const int nN = (a.Cout + BN - 1) / BN;
  const int bt = xcd_tile(blockIdx.x, gridDim.x, a.xcd);
  const int mt = bt / nN;
  const int nt = bt - mt * nN;
  const int m0 = mt * BM, n0 = nt * BN;
  const u16* __restrict__ x = (const u16*)a.x;
  const u16* __restrict__ w = (const u16*)a.w;
  const u16* zero = (const u16*)a.zero;  // B rows past Cout

  // A rows by buffer loads: one descriptor over the images this M-tile touches, a 32-bit
  // byte offset per row, and a 9-bit mask of the taps that fall inside the map (an invalid tap
  // gets an out-of-range offset, which the buffer unit reads as zeros: the conv's zero padding)
  const int lr = lane >> 3;
  const int pc = lane & 7;
  const int img0 = m0 / HoWo;
  const int img1 = min(M - 1, m0 + BM - 1) / HoWo;
  const long long img_bytes = (long long)a.H * a.W * a.Cin * 2;
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(x + (long long)img0 * a.H * a.W * a.Cin), (short)0, (int)((img1 - img0 + 1) * img_bytes), 0x00020000);
  int aoffs[AI];
  unsigned amask[AI];
  // DS: the fused 1x1 downsample's input rows (K columns [K1, K)), same image range
  __amdgpu_buffer_rsrc_t xr2 = xr;
  int aoffs2[DS ? AI : 1];
  if constexpr (DS)
    xr2 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const u16*)a.x2 + (long long)img0 * a.H2 * a.W2 * a.Cin2), (short)0,
        (int)((long long)(img1 - img0 + 1) * a.H2 * a.W2 * a.Cin2 * 2), 0x00020000);
  // A piece j: half h = j / (AI/2) (0: rows 0-63 of each 128-row wave strip = A0-3, 1: rows
  // 64-127 = A4-7), 8 consecutive rows of that half; arow0[j] = the piece's first LDS row
  int arow0[AI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int h = j / (AI / 2), jj = j % (AI / 2);
    const int idx0 = wid * (BM / 2 / NW) + 8 * jj;  // in the half's row list (64 per strip)
    arow0[j] = (idx0 / 64) * 128 + h * 64 + idx0 % 64;
    const int row = arow0[j] + lr;
    const int lc = pc ^ ((row >> 1) & 7);
    const int m = m0 + row;
    amask[j] = 0;
    aoffs[j] = 0;
    if constexpr (DS) aoffs2[j] = -1;
    if (m < M) {
      const int img = m / HoWo;
      const int rem = m - img * HoWo;
      const int oh = rem / a.Wo;
      const int ow = rem - oh * a.Wo;
      const int ih = oh * a.stride - a.pad, iw = ow * a.stride - a.pad;
      aoffs[j] = (((img - img0) * a.H + ih) * a.W + iw) * a.Cin * 2 + lc * 16;
      if constexpr (DS)
        aoffs2[j] = (((img - img0) * a.H2 + oh * a.stride2) * a.W2 + ow * a.stride2) * a.Cin2 * 2 + lc * 16;
      for (int kh = 0; kh < a.KH; ++kh)
        for (int kw = 0; kw < a.KW; ++kw)
          if ((unsigned)(ih + kh) < (unsigned)a.H && (unsigned)(iw + kw) < (unsigned)a.W) amask[j] |= 1u << (kh * a.KW + kw);
    }
  }
  // B piece j: half h = j / (BI/2) (0: cols 0-31 of each 64-col wave strip = B0-1, 1: 32-63 = B2-3)
  const u16* brow[BI];
  int brow0[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int h = j / (BI / 2), jj = j % (BI / 2);
    const int idx0 = wid * (BN / 2 / NW) + 8 * jj;  // in the half's row list (32 per strip)
    brow0[j] = (idx0 / 32) * 64 + h * 32 + idx0 % 32;
    const int row = brow0[j] + lr;
    const int lc = pc ^ ((row >> 1) & 7);
    const int n = n0 + row;
    brow[j] = n < a.Cout ? w + (long long)n * a.K + lc * 8 : nullptr;
  }
  // K walk kept incrementally: tap index (kh * KW + kw), kw, channel offset c0 and the tap's
  // byte offset; K order (kh, kw, cin) or, with a.kcm, (cin / 64, kh, kw, cin % 64)
  int tap = 0, toff = 0, kwc = 0, c0 = 0, kk = 0;
  const int taps = a.KH * a.KW;
  const int row_step = (a.W - a.KW) * a.Cin * 2;  // bytes from tap (kh, KW-1) + Cin to (kh+1, 0)
  auto next_tap = [&]() {
    ++tap;
    toff += a.Cin * 2;
    if (++kwc == a.KW) {
      kwc = 0;
      toff += row_step;
    }
  };
  auto advance = [&]() {
    kk += BK;
    if (a.kcm) {
      next_tap();
      if (tap == taps) {
        tap = 0;
        kwc = 0;
        c0 += BK;
        toff = c0 * 2;
      }
    } else {
      c0 += BK;
      toff += BK * 2;
      if (c0 == a.Cin) {
        c0 = 0;
        toff -= a.Cin * 2;
        next_tap();
      }
    }
  };
  // stage half h of A (B) of the K-tile the walk state points at into As (Bs)
  auto stage_a = [&](u16* As, int h) {
    if (DS && kk >= a.K1) {
      const int d = (kk - a.K1) * 2;
#pragma unroll
      for (int j = h * (AI / 2); j < (h + 1) * (AI / 2); ++j) {
        const int voff = aoffs2[DS ? j : 0] >= 0 ? aoffs2[DS ? j : 0] + d : (int)0x80000000;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xr2, (__attribute__((address_space(3))) void*)(As + arow0[j] * BK), 16,
                                                 voff, 0, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int j = h * (AI / 2); j < (h + 1) * (AI / 2); ++j) {
      const int voff = ((amask[j] >> tap) & 1) ? aoffs[j] + toff : (int)0x80000000;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)(As + arow0[j] * BK), 16, voff,
                                               0, 0, 0);
    }
  };
  auto stage_b = [&](int k0, u16* Bs, int h) {
#pragma unroll
    for (int j = h * (BI / 2); j < (h + 1) * (BI / 2); ++j) {
      const u16* src = brow[j] ? brow[j] + k0 : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(Bs + brow0[j] * BK), 16,
                                       0, 0);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment lane map (16x16x32): row r = lane % 16, chunk q = lane / 16 of the 32-k slice
  const int r = lane & 15;
  const int q = lane >> 4;
  const int sw = (r >> 1) & 7;
  const int ch0 = ((0 * 4 + q) ^ sw) * 8;  // k-half 0 of the 64-wide K-tile
  const int ch1 = ((1 * 4 + q) ^ sw) * 8;  // k-half 1
  const int aoff = (wm * 128 + r) * BK;
  const int boff = BM * BK + (wn * 64 + r) * BK;
  bf16x8 af[4][2] = {}, bfr[2][2] = {};
  // a.abl (profiling-only ablations, results wrong when set): 1 no main-loop DMA,
  // 16 no main-loop ds_reads, 32 no MFMAs, 256 no epilogue
  auto read_a = [&](const u16* S, int i0) {
    if (a.abl & 16) return;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i][0] = *(const bf16x8*)(S + aoff + (i0 + i) * 16 * BK + ch0);
      af[i][1] = *(const bf16x8*)(S + aoff + (i0 + i) * 16 * BK + ch1);
    }
  };
  auto read_b = [&](const u16* S, int j0) {
    if (a.abl & 16) return;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bfr[j][0] = *(const bf16x8*)(S + boff + (j0 + j) * 16 * BK + ch0);
      bfr[j][1] = *(const bf16x8*)(S + boff + (j0 + j) * 16 * BK + ch1);
    }
  };
  auto mfma = [&](int i0, int j0) {
    if (a.abl & 32) {
      asm volatile("" ::"v"(af[0][0]), "v"(bfr[0][0]));
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s)
          acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][s], bfr[j][s], acc[i0 + i][j0 + j], 0, 0, 0);
  };
  // end of a LOAD segment: own LDS reads retired (WAR safety for the next re-stage), then
  // the barrier that opens the MFMA segment; the MFMA segment ends with another barrier
  const bool nobar = a.abl & 128;
  const bool prio = a.p8prio;
#define P8_LOAD_END()                                   \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    \
  if (!nobar) __builtin_amdgcn_s_barrier();             \
  __builtin_amdgcn_sched_barrier(0);                    \
  if (prio) __builtin_amdgcn_s_setprio(1)
#define P8_MFMA_END()                       \
  __builtin_amdgcn_sched_barrier(0);        \
  if (prio) __builtin_amdgcn_s_setprio(0);  \
  if (!nobar) __builtin_amdgcn_s_barrier(); \
  __builtin_amdgcn_sched_barrier(0)
#define P8_VMCNT(N) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory")
  constexpr int HA = AI / 2, HB = BI / 2;  // DMA instructions per half-tile per wave

  const int nk = a.K / BK;
  stage_a(smem, 0);
  stage_a(smem, 1);
  stage_b(0, smem + BM * BK, 0);
  stage_b(0, smem + BM * BK, 1);
  advance();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (half) __builtin_amdgcn_s_barrier();  // stagger: waves 4-7 one barrier behind
  __builtin_amdgcn_sched_barrier(0);
  if (a.p8pipe) {
    for (int t = 0; t < nk; ++t) {
      const u16* S = smem + (t & 1) * STAGE;
      u16* Nx = smem + ((t & 1) ^ 1) * STAGE;
      const bool more = t + 1 < nk && !(a.abl & 1);
      // phase 0: A0-3, B0-1; issue A-top(t+1); retire B-right(t) (younger: A-bottom(t), A-top(t+1))
      read_a(S, 0);
      read_b(S, 0);
      if (more) {
        stage_a(Nx, 0);
        P8_VMCNT(2 * HA);
      } else {
        P8_VMCNT(HA);
      }
      P8_LOAD_END();
      mfma(0, 0);
      P8_MFMA_END();
      // phase 1: B2-3; issue B-left(t+1); retire A-bottom(t) (younger: A-top(t+1), B-left(t+1))
      read_b(S, 2);
      if (more) {
        stage_b((t + 1) * BK, Nx + BM * BK, 0);
        P8_VMCNT(HA + HB);
      } else {
        P8_VMCNT(0);
      }
      P8_LOAD_END();
      mfma(0, 2);
      P8_MFMA_END();
      // phase 2: A4-7; issue B-right(t+1)
      read_a(S, 4);
      if (more) stage_b((t + 1) * BK, Nx + BM * BK, 1);
      P8_LOAD_END();
      mfma(4, 2);
      P8_MFMA_END();
      // phase 3: B0-1; issue A-bottom(t+1); retire A-top(t+1), B-left(t+1) (younger: B-right(t+1),
      // A-bottom(t+1)) before the barrier that K-tile t+1's phase-0 readers pass
      read_b(S, 0);
      if (more) {
        stage_a(Nx, 1);
        P8_VMCNT(HB + HA);
      }
      advance();
      P8_LOAD_END();
      mfma(4, 0);
      P8_MFMA_END();
    }
  } else {
    for (int t = 0; t < nk; ++t) {
      const u16* S = smem + (t & 1) * STAGE;
      u16* Nx = smem + ((t & 1) ^ 1) * STAGE;
      const bool more = t + 1 < nk && !(a.abl & 1);
      read_a(S, 0);
      read_b(S, 0);
      if (more && !(a.abl & 512)) {
        stage_a(Nx, 0);
        stage_a(Nx, 1);
      }
      advance();
      P8_LOAD_END();
      mfma(0, 0);
      P8_MFMA_END();
      read_b(S, 2);
      if (more && !(a.abl & 1024)) {
        stage_b((t + 1) * BK, Nx + BM * BK, 0);
        stage_b((t + 1) * BK, Nx + BM * BK, 1);
      }
      P8_LOAD_END();
      mfma(0, 2);
      P8_MFMA_END();
      read_a(S, 4);
      P8_LOAD_END();
      mfma(4, 2);
      P8_MFMA_END();
      read_b(S, 0);
      if (more && !(a.abl & 64)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      P8_LOAD_END();
      mfma(4, 0);
      P8_MFMA_END();
    }
  }
  if (!half) __builtin_amdgcn_s_barrier();  // re-align the halves
#undef P8_LOAD_END
#undef P8_MFMA_END
#undef P8_VMCNT
  __syncthreads();

  if (a.abl & 256) {  // profiling-only: no epilogue
    asm volatile("" ::"v"(acc[0][0][0]));
    return;
  }
  u16* __restrict__ y = (u16*)a.y;
  const u16* __restrict__ res = (const u16*)a.res;
  // Epilogue staged through LDS (the buffers are free now): pass i moves the i-th 32-row
  // M-subtile of every wave (WM*32 rows x BN cols, f32, rows padded by 4).
  constexpr int EPR = WM * 32;
  constexpr int EPS = BN + 4;
  static_assert(EPR * EPS * 4 <= 2 * STAGE * 2, "epilogue tile must fit the buffers");
  float* ep = (float*)smem;
  float bcol[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + r;
    bcol[j] = (a.bias && n < a.Cout) ? a.bias[n] : 0.f;
  }
  constexpr int NPASS = 128 / 32;
  constexpr int IPT = EPR * (BN / 8) / (64 * NW);  // 16-B output chunks per thread per pass
  static_assert(IPT * 64 * NW == EPR * (BN / 8), "epilogue work divides evenly");
  uint4 rv[2][IPT];
  uint4 rl[2][SPLIT ? IPT : 1];  // SPLIT: the residual's lo block
  const long long ostr = SPLIT ? 3LL * a.Cout : a.Cout;  // output / residual pixel stride
  auto chunk = [&](int i, int t, int& lrow, int& c8, long long& o) {
    const int idx = tid + t * 64 * NW;
    lrow = idx / (BN / 8);
    c8 = idx - lrow * (BN / 8);
    const int m = m0 + (lrow >> 5) * 128 + i * 32 + (lrow & 31);
    const int n = n0 + c8 * 8;
    o = (m < M && n < a.Cout) ? (long long)m * ostr + n : -1;
  };
  auto load_res = [&](int i) {
#pragma unroll
    for (int t = 0; t < IPT; ++t) {
      int lrow, c8;
      long long o;
      chunk(i, t, lrow, c8, o);
      if (o >= 0) {
        rv[i & 1][t] = *(const uint4*)(res + o);
        if constexpr (SPLIT) rl[i & 1][SPLIT ? t : 0] = *(const uint4*)(res + o + a.Cout);
      }
    }
  };
  if (res) load_res(0);
#pragma unroll
  for (int i = 0; i < NPASS; ++i) {
    if (res && i + 1 < NPASS) load_res(i + 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          // 16x16 C/D map: row 4 * (lane / 16) + e, column lane % 16
          const int lrow = wm * 32 + t * 16 + 4 * q + e;
          ep[lrow * EPS + wn * 64 + j * 16 + r] = acc[i * 2 + t][j][e] + bcol[j];
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int t = 0; t < IPT; ++t) {
      int lrow, c8;
      long long o;
      chunk(i, t, lrow, c8, o);
      if (o < 0) continue;
      const float4 v0 = *(const float4*)(ep + lrow * EPS + c8 * 8);
      const float4 v1 = *(const float4*)(ep + lrow * EPS + c8 * 8 + 4);
      float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      if (res) {
        const uint4 r4 = rv[i & 1][t];
        const unsigned ru[4] = {r4.x, r4.y, r4.z, r4.w};
        if constexpr (SPLIT) {
          const uint4 l4 = rl[i & 1][SPLIT ? t : 0];
          const unsigned rlo[4] = {l4.x, l4.y, l4.z, l4.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {  // hi + lo is exact in f32
            v[2 * k] += bf2f((u16)(ru[k] & 0xffff)) + bf2f((u16)(rlo[k] & 0xffff));
            v[2 * k + 1] += bf2f((u16)(ru[k] >> 16)) + bf2f((u16)(rlo[k] >> 16));
          }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            v[2 * k] += bf2f((u16)(ru[k] & 0xffff));
            v[2 * k + 1] += bf2f((u16)(ru[k] >> 16));
          }
        }
      }
      unsigned pk[4], pl[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float lo = v[2 * k], hi = v[2 * k + 1];
        if (a.relu) {
          lo = fmaxf(lo, 0.f);
          hi = fmaxf(hi, 0.f);
        }
        const u16 blo = f2bf(lo), bhi = f2bf(hi);
        pk[k] = (unsigned)blo | ((unsigned)bhi << 16);
        if constexpr (SPLIT)  // residual parts (exact differences)
          pl[k] = (unsigned)f2bf(lo - bf2f(blo)) | ((unsigned)f2bf(hi - bf2f(bhi)) << 16);
      }
      if (a.abl & 2) {
        asm volatile("" ::"v"(pk[0]), "v"(pk[1]), "v"(pk[2]), "v"(pk[3]));
      } else {
        *(uint4*)(y + o) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        if constexpr (SPLIT) {
          *(uint4*)(y + o + a.Cout) = make_uint4(pl[0], pl[1], pl[2], pl[3]);
          *(uint4*)(y + o + 2 * a.Cout) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        }
      }
    }
  }
}

bool conv_bf16_p8_ok(const ConvArgs& a) {
  return a.Cin != 3 && a.Cin % 64 == 0 && a.K % 64 == 0 && a.K >= 128 && (a.Cout == 128 || a.Cout % 256 == 0);
}

// where the phased kernel is the default (r01 A/B on R18, tools/ab_env.sh EOSV_BF16_P8): the
// stride-1 Cout = 128 convs (+1-3 %); at Cout >= 256 it ties conv_bf16_kernel's 256x256 tile and
// on the stride-2 / 1x1 entries it is 5-10 % slower.  EOSV_BF16_P8=2 routes every eligible conv.
// r01g: nowhere -- conv_bf16_kernel's 512x128 tile replaced it on the Cout = 128 convs (conv_bf16.hip);
// EOSV_BF16_P8=2 still routes every eligible conv here for A/B
bool conv_bf16_p8_default(const ConvArgs& a) {
  (void)a;
  return false;
}
// (with a fused downsample, a.K includes its Cin2 columns; the shape test above is unchanged)

static int p8_env(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

int launch_conv_bf16_p8(const ConvArgs& a0, hipStream_t s) {
  static const int pipe = p8_env("EOSV_P8_PIPE", 1), prio = p8_env("EOSV_P8_PRIO", 1);  // A/B switches
  ConvArgs a = a0;
  a.p8pipe = pipe;
  a.p8prio = prio;
  if (!conv_bf16_p8_ok(a)) return set_error("conv_bf16_p8: unsupported shape"), EOSV_ERR_UNSUPPORTED;
  const long long M = (long long)a.N * a.Ho * a.Wo;
  const int BM = a.Cout == 128 ? 512 : 256;
  const int BN = a.Cout == 128 ? 128 : 256;
  const long long nb = ((M + BM - 1) / BM) * ((a.Cout + BN - 1) / BN);
  if (nb > 0x7fffffffLL) return set_error("conv_bf16_p8: grid too large"), EOSV_ERR_UNSUPPORTED;
  if (a.x2 && (a.K1 % 64 || a.Cin2 % 64)) return set_error("conv_bf16_p8: fused downsample shape"), EOSV_ERR_UNSUPPORTED;
  if (a.split) {
#define P8_SPLIT(BM_, BN_, WM_, WN_)                                                                          \
  if (a.x2)                                                                                                 \
    hipLaunchKernelGGL((conv_bf16_p8_kernel<BM_, BN_, WM_, WN_, true, true>), dim3((unsigned)nb), dim3(512), 0, s, a); \
  else                                                                                                      \
    hipLaunchKernelGGL((conv_bf16_p8_kernel<BM_, BN_, WM_, WN_, false, true>), dim3((unsigned)nb), dim3(512), 0, s, a);
    if (a.Cout == 128) {
      P8_SPLIT(512, 128, 4, 2)
    } else {
      P8_SPLIT(256, 256, 2, 4)
    }
#undef P8_SPLIT
  } else if (a.Cout == 128) {
    if (a.x2)
      hipLaunchKernelGGL((conv_bf16_p8_kernel<512, 128, 4, 2, true>), dim3((unsigned)nb), dim3(512), 0, s, a);
    else
      hipLaunchKernelGGL((conv_bf16_p8_kernel<512, 128, 4, 2, false>), dim3((unsigned)nb), dim3(512), 0, s, a);
  } else {
    if (a.x2)
      hipLaunchKernelGGL((conv_bf16_p8_kernel<256, 256, 2, 4, true>), dim3((unsigned)nb), dim3(512), 0, s, a);
    else
      hipLaunchKernelGGL((conv_bf16_p8_kernel<256, 256, 2, 4, false>), dim3((unsigned)nb), dim3(512), 0, s, a);
  }
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

}  // namespace eosv
