// Tap-shift implicit GEMM for the stride-1 3x3 convs on bf16 MFMA (ResNet stages 2-4 and the
// R50 bottleneck 3x3s; bf16 and the EOSV_F32X3 split layout).
//
// conv_bf16_kernel stages one im2col A row per output pixel per tap, so every input pixel
// crosses L2 -> LDS 9 times, and its LDS-DMA feed (not the MFMA pipe) bounds it (DESIGN.md
// section 3).  Here a stage is (32-channel slice, kernel row kh): the A tile holds the input
// row oh + kh - 1 of the BM + 2 consecutive output pixels m0 - 1 .. m0 + BM (each at its own
// column), and the three taps kw = 0, 1, 2 of that kernel row read it at row offsets 0, 1, 2:
// output pixel m0 + r at tap kw needs input column ow + kw - 1, which is where pixel
// m0 + r + kw - 1 sits -- unless ow + kw - 1 leaves the row, and those A fragments (ow = 0 at
// kw = 0, ow = W - 1 at kw = 2: the conv's zero padding) are zeroed in registers.  A is staged
// once per kernel row instead of once per tap (3x fewer A bytes); B holds the 3 taps' weights.
//
// Staged bytes per stage, 512 x 128 tile: A 528 x 64 B + B 3 x 128 x 64 B = 58 KiB for
// 12.6 MFLOP (216 FLOP/B; the im2col tile: 105); 256 x 256: 65 KiB for 12.6 MFLOP (194; was 128).
// LDS rows are 64 B (BK = 32: one v_mfma_f32_16x16x32_bf16 k-step); 16-B chunk c of row R sits
// at c ^ ((R >> 1) & 3), applied on the DMA source: conflict-free ds_read_b128 for the fragment
// rows at any row offset (checked for every base offset against the b128 lane groups of
// MI355X_MICROARCH.md, LDS).  Ring, barriers and epilogue as conv_bf16_kernel.
#include <hip/hip_bf16.h>

#include "common.h"

namespace eosv {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __bfloat16_as_ushort(__float2bfloat16(f)); }
__device__ __forceinline__ void dma16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}
}  // namespace

// DMA stagger of the upper half of the waves: they issue the stage's DMA after tap kw = TS_STAG - 1
// (r03: 1, i.e. after the first tap; 0 = no stagger)
constexpr int TS_STAG = 1;

template <int BM, int BN, int WM, int WN, bool SPLIT>
__global__ __launch_bounds__(64 * WM * WN) void conv_bf16_ts_kernel(ConvArgs a) {
  constexpr int BK = 32;                        // channels per stage
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  constexpr int AR = (BM + 2 + 15) / 16 * 16;   // staged A rows (output pixels m0 - 1 .. m0 + BM)
  constexpr int AP = AR / 16;                   // A DMA pieces (16 rows x 64 B = 1 KiB)
  constexpr int APW = (AP + NW - 1) / NW;       // A pieces per wave (the last ones partial)
  constexpr int BP = 3 * BN / 16;               // B DMA pieces (3 taps x BN rows)
  constexpr int BPW = (BP + NW - 1) / NW;       // B pieces per wave (the last ones partial)
  constexpr int STAGE = (AR + 3 * BN) * BK;     // bf16 elements per ring slot
  __shared__ __attribute__((aligned(16))) u16 smem[2 * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int HW = a.H * a.W;
  const int M = a.N * HW;
  const int nN = a.Cout / BN;
  const int bt = xcd_tile(blockIdx.x, gridDim.x, a.xcd);
  const int mt = bt / nN;
  const int nt = bt - mt * nN;
  const int m0 = mt * BM, n0 = nt * BN;
  const u16* __restrict__ x = (const u16*)a.x;
  const u16* __restrict__ w = (const u16*)a.w;
  const u16* zero = (const u16*)a.zero;

  // A pieces: lane -> staged row 16 * piece + (lane >> 2), LDS chunk slot lane & 3 (source chunk
  // slot ^ swizzle); apix = the row's pixel at its own position, amask bit kh = input row
  // oh + kh - 1 inside the image
  const int lr = lane >> 2, sl = lane & 3;
  const u16* apix[APW];
  unsigned amask[APW];
#pragma unroll
  for (int t = 0; t < APW; ++t) {
    const int piece = wid + NW * t;
    const int row = piece * 16 + lr;
    const int p = m0 - 1 + row;
    apix[t] = zero;
    amask[t] = 0;
    if (piece < AP && row <= BM + 1 && p >= 0 && p < M) {
      const int rem = p % HW;
      const int oh = rem / a.W;
      apix[t] = x + (long long)p * a.xs + (sl ^ ((row >> 1) & 3)) * 8;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
        if ((unsigned)(oh + kh - 1) < (unsigned)a.H) amask[t] |= 1u << kh;
    }
  }
  // DS (fused 1x1 downsample, ConvArgs::x2): the same rows' pixels in x2 at (oh s2, ow s2);
  // staged rows 1 .. BM only (a DS stage is read at tap offset 1)
  const u16* apix2[APW];
  const u16* x2 = (const u16*)a.x2;
#pragma unroll
  for (int t = 0; t < APW; ++t) {
    const int piece = wid + NW * t;
    const int row = piece * 16 + lr;
    const int p = m0 - 1 + row;
    apix2[t] = zero;
    if (x2 && piece < AP && row >= 1 && row <= BM && p < M) {
      const int img = p / HW, rem = p - img * HW;
      const int oh = rem / a.W, ow = rem - oh * a.W;
      apix2[t] = x2 + (((long long)img * a.H2 + oh * a.stride2) * a.W2 + ow * a.stride2) * a.x2s +
                 (sl ^ ((row >> 1) & 3)) * 8;
    }
  }
  // B pieces: staged row kw * BN + (output channel - n0)
  const u16* bsrc[BPW];
  int btap[BPW];
#pragma unroll
  for (int t = 0; t < BPW; ++t) {
    const int row = min((wid + NW * t) * 16, BP * 16 - 16) + lr;  // pieces past BP: never issued
    const int kw = row / BN;
    btap[t] = kw;
    bsrc[t] = w + (long long)(n0 + row - kw * BN) * a.K + (sl ^ ((row >> 1) & 3)) * 8;
  }
  const long long rowoff = (long long)a.W * a.xs;  // elements from input row oh to oh + 1
  auto kidx = [&](int kh, int kw, int c) -> int {   // K column of tap (kh, kw), channel c (32-aligned)
    return a.kcm ? (((c >> 6) * 9 + kh * 3 + kw) << 6) + (c & 63) : (kh * 3 + kw) * a.Cin + c;
  };
  const int nst3 = 3 * (a.Cin / BK);  // 3x3 stages; then Cin2 / BK fused-downsample stages
  auto stage = [&](int st, int slot) {
    u16* As = smem + slot * STAGE;
    u16* Bs = As + AR * BK;
    if (st >= nst3) {  // DS stage: A = x2 pixels, B = the 1x1 weights (K columns K1 + c) in tap slot 1
      const int c0 = (st - nst3) * BK;
#pragma unroll
      for (int t = 0; t < APW; ++t) {
        const int piece = wid + NW * t;
        if (piece < AP)
          dma16(apix2[t] + (apix2[t] != zero ? (SPLIT ? split_chan(c0, a.Cin2) : c0) : 0), As + piece * 16 * BK);
      }
#pragma unroll
      for (int t = 0; t < BPW; ++t)
        if (wid + NW * t < BP && btap[t] == 1) dma16(bsrc[t] + a.K1 + c0, Bs + (wid + NW * t) * 16 * BK);
      return;
    }
    const int cs = st / 3, kh = st - 3 * cs, c0 = cs * BK;
    const long long aoff = (long long)(kh - 1) * rowoff + (SPLIT ? split_chan(c0, a.Cin) : c0);
#pragma unroll
    for (int t = 0; t < APW; ++t) {
      const int piece = wid + NW * t;
      if (piece < AP) {
        const u16* src = ((amask[t] >> kh) & 1) ? apix[t] + aoff : zero;
        dma16(src, As + piece * 16 * BK);
      }
    }
#pragma unroll
    for (int t = 0; t < BPW; ++t)
      if (wid + NW * t < BP) dma16(bsrc[t] + kidx(kh, btap[t], c0), Bs + (wid + NW * t) * 16 * BK);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int r = lane & 15;
  const int q = lane >> 4;
  // image-column edges of this lane's output rows: bit 2i = ow 0 (tap kw 0 reads padding),
  // bit 2i + 1 = ow W - 1 (kw 2)
  unsigned emask = 0;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * (BM / WM) + i * 16 + r;
    const int ow = (m % HW) % a.W;
    if (ow == 0) emask |= 1u << (2 * i);
    if (ow == a.W - 1) emask |= 2u << (2 * i);
  }

  const int nst = nst3 + (x2 ? a.Cin2 / BK : 0);
  // TS_STAG k > 0: the upper half of the waves (the partners w + NW/2 of a SIMD's pairs)
  // issues its next-stage DMA after tap kw = k - 1 instead of at the stage's start (as
  // conv_bf16_kernel's stagger: one wave's DMA issue beside the other's MFMAs).  r03, R50 bf16
  // stage-2 3x3s per 3200 frames: k = 1 0.81-0.86 -> 0.77-0.82 ms (4-5 %), k = 2 1-2 %.
  const int lkw = (TS_STAG > 0 && wid >= NW / 2) ? TS_STAG - 1 : -1;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");  // s_barrier is no compiler-level memory barrier
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    if (st + 1 < nst && lkw < 0) stage(st + 1, cur ^ 1);
    const u16* As = smem + cur * STAGE;
    const u16* Bs = As + AR * BK;
    const bool ds = st >= nst3;  // a DS stage is read at offset 1 only (no taps, no edges)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      if (kw > 0 && kw - 1 == lkw && st + 1 < nst) stage(st + 1, cur ^ 1);
      if (ds && kw != 1) continue;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * (BM / WM) + i * 16 + r + kw;  // pixel m0 + (row - kw) at tap kw
        af[i] = *(const bf16x8*)(As + row * BK + ((q ^ ((row >> 1) & 3)) * 8));
        if (kw != 1 && ((emask >> (2 * i + (kw >> 1))) & 1)) af[i] = bf16x8{};  // (never in a DS stage)
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = kw * BN + wn * (BN / WN) + j * 16 + r;
        bfr[j] = *(const bf16x8*)(Bs + row * BK + ((q ^ ((row >> 1) & 3)) * 8));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // Epilogue as conv_bf16_kernel's (LDS-staged 16-B rows, buffer resources, branch-free)
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the asm waits above are invisible to the compiler
  u16* __restrict__ y = (u16*)a.y;
  const u16* __restrict__ res = (const u16*)a.res;
  constexpr int EPR = WM * 32;
  constexpr int EPS = BN + 4;
  static_assert(EPR * EPS * 4 <= 2 * STAGE * 2, "epilogue tile must fit the ring");
  float* ep = (float*)smem;
  float bcol[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / WN) + j * 16 + r;
    bcol[j] = a.bias ? a.bias[n] : 0.f;
  }
  const int nthreads = 64 * NW;
  constexpr int NPASS = BM / WM / 32;
  constexpr int IPT = EPR * (BN / 8) / (64 * NW);
  static_assert(IPT * 64 * NW == EPR * (BN / 8), "epilogue work divides evenly");
  const long long ostr = SPLIT ? 2LL * a.Cout : a.Cout;
  const long long tile_bytes = (long long)min(BM, M - m0) * ostr * 2;
  const int nrec = (int)min(tile_bytes, 0x7fffffffLL);
  const __amdgpu_buffer_rsrc_t yr =
      __builtin_amdgcn_make_buffer_rsrc((void*)(y + (long long)m0 * ostr), (short)0, nrec, 0x00020000);
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(res ? res + (long long)m0 * ostr : zero), (short)0, res ? nrec : 0, 0x00020000);
  v4u rv[2][IPT];
  v4u rl[2][SPLIT ? IPT : 1];
  auto chunk = [&](int i, int t, int& lrow, int& c8, int& voff) {
    const int idx = tid + t * nthreads;
    lrow = idx / (BN / 8);
    c8 = idx - lrow * (BN / 8);
    const int ml = (lrow >> 5) * (BM / WM) + i * 32 + (lrow & 31);
    voff = (int)(((long long)ml * ostr + n0 + c8 * 8) * 2);
  };
  auto load_res = [&](int i) {
#pragma unroll
    for (int t = 0; t < IPT; ++t) {
      int lrow, c8, voff;
      chunk(i, t, lrow, c8, voff);
      rv[i & 1][t] = __builtin_amdgcn_raw_buffer_load_b128(rr, voff, 0, 0);
      if constexpr (SPLIT) rl[i & 1][SPLIT ? t : 0] = __builtin_amdgcn_raw_buffer_load_b128(rr, voff + 2 * a.Cout, 0, 0);
    }
  };
  load_res(0);
  const float rlow = a.relu ? 0.f : -INFINITY;
#pragma unroll
  for (int i = 0; i < NPASS; ++i) {
    if (i + 1 < NPASS) load_res(i + 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int lrow = wm * 32 + t * 16 + 4 * q + e;  // 16x16 C/D map: row 4(lane/16) + e
          ep[lrow * EPS + wn * (BN / WN) + j * 16 + r] = acc[i * 2 + t][j][e] + bcol[j];
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int t = 0; t < IPT; ++t) {
      int lrow, c8, voff;
      chunk(i, t, lrow, c8, voff);
      const float4 v0 = *(const float4*)(ep + lrow * EPS + c8 * 8);
      const float4 v1 = *(const float4*)(ep + lrow * EPS + c8 * 8 + 4);
      float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      const v4u r4 = rv[i & 1][t];
      const unsigned ru[4] = {r4.x, r4.y, r4.z, r4.w};
      if constexpr (SPLIT) {
        const v4u l4 = rl[i & 1][SPLIT ? t : 0];
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
      v4u pk, pl;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float lo = fmaxf(v[2 * k], rlow), hi = fmaxf(v[2 * k + 1], rlow);
        const u16 blo = f2bf(lo), bhi = f2bf(hi);
        pk[k] = (unsigned)blo | ((unsigned)bhi << 16);
        if constexpr (SPLIT)
          pl[k] = (unsigned)f2bf(lo - bf2f(blo)) | ((unsigned)f2bf(hi - bf2f(bhi)) << 16);
      }
      __builtin_amdgcn_raw_buffer_store_b128(pk, yr, voff, 0, 0);
      if constexpr (SPLIT) __builtin_amdgcn_raw_buffer_store_b128(pl, yr, voff + 2 * a.Cout, 0, 0);
    }
  }
}

// Warp-specialised tap-shift tile (r04, EOSV_BF16_TS_WS; bf16 layout): NW consumer waves (LDS
// fragments + MFMAs only) and NP producer waves (LDS-DMA only), as conv_bf16_ws_kernel, on split
// rings: 3 A slots (the stage's input row, two stages ahead) and 2 B slots (its 3 taps' weights,
// one ahead), 147 KiB at 512 x 128.  Same stages, taps, MFMA order and epilogue as
// conv_bf16_ts_kernel: bit-identical outputs.
#ifndef EOSV_BF16_TS_BEARLY
#define EOSV_BF16_TS_BEARLY 1
#endif
template <int BM, int BN, int WM, int WN, int NP>
__global__ __launch_bounds__(64 * (WM * WN + NP)) void conv_bf16_ts_ws_kernel(ConvArgs a) {
  constexpr int BK = 32, NW = WM * WN, TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int AR = (BM + 2 + 15) / 16 * 16, AP = AR / 16, APW = (AP + NP - 1) / NP;
  constexpr int BP = 3 * BN / 16, BPW = (BP + NP - 1) / NP;
  constexpr int AS = AR * BK, BS = 3 * BN * BK;  // bf16 elements per A / B slot
  constexpr int SMEM = 3 * AS + 2 * BS;
  __shared__ __attribute__((aligned(16))) u16 smem[SMEM];
  auto a_slot = [&](int st) { return smem + (st % 3) * AS; };
  auto b_slot = [&](int st) { return smem + 3 * AS + (st & 1) * BS; };

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int HW = a.H * a.W;
  const int M = a.N * HW;
  const int nN = a.Cout / BN;
  const int bt = xcd_tile(blockIdx.x, gridDim.x, a.xcd);
  const int mt = bt / nN;
  const int nt = bt - mt * nN;
  const int m0 = mt * BM, n0 = nt * BN;
  const u16* zero = (const u16*)a.zero;
  const int nst3 = 3 * (a.Cin / BK);
  const int nst = nst3 + (a.x2 ? a.Cin2 / BK : 0);

  if (wid >= NW) {  // ---------------------------------------------------------------- producer
    const int pw = wid - NW;
    const u16* __restrict__ x = (const u16*)a.x;
    const u16* __restrict__ w = (const u16*)a.w;
    const u16* x2 = (const u16*)a.x2;
    const int lr = lane >> 2, sl = lane & 3;
    const u16* apix[APW];
    const u16* apix2[APW];
    unsigned amask[APW];
#pragma unroll
    for (int t = 0; t < APW; ++t) {
      const int piece = pw + NP * t;
      const int row = piece * 16 + lr;
      const int p = m0 - 1 + row;
      apix[t] = zero;
      apix2[t] = zero;
      amask[t] = 0;
      if (piece < AP && row <= BM + 1 && p >= 0 && p < M) {
        const int img = p / HW, rem = p - img * HW;
        const int oh = rem / a.W, ow = rem - oh * a.W;
        apix[t] = x + (long long)p * a.xs + (sl ^ ((row >> 1) & 3)) * 8;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
          if ((unsigned)(oh + kh - 1) < (unsigned)a.H) amask[t] |= 1u << kh;
        if (x2 && row >= 1 && row <= BM)
          apix2[t] = x2 + (((long long)img * a.H2 + oh * a.stride2) * a.W2 + ow * a.stride2) * a.x2s +
                     (sl ^ ((row >> 1) & 3)) * 8;
      }
    }
    const u16* bsrc[BPW];
    int btap[BPW];
#pragma unroll
    for (int t = 0; t < BPW; ++t) {
      const int row = min((pw + NP * t) * 16, BP * 16 - 16) + lr;  // pieces past BP: never issued
      const int kw = row / BN;
      btap[t] = kw;
      bsrc[t] = w + (long long)(n0 + row - kw * BN) * a.K + (sl ^ ((row >> 1) & 3)) * 8;
    }
    const long long rowoff = (long long)a.W * a.xs;
    auto kidx = [&](int kh, int kw, int c) -> int {
      return a.kcm ? (((c >> 6) * 9 + kh * 3 + kw) << 6) + (c & 63) : (kh * 3 + kw) * a.Cin + c;
    };
    auto stage_a = [&](int st) {
      u16* As = a_slot(st);
      if (st >= nst3) {  // DS stage: the x2 pixels (read at tap offset 1)
        const int c0 = (st - nst3) * BK;
#pragma unroll
        for (int t = 0; t < APW; ++t)
          if (pw + NP * t < AP) dma16(apix2[t] + (apix2[t] != zero ? c0 : 0), As + (pw + NP * t) * 16 * BK);
        return;
      }
      const int cs = st / 3, kh = st - 3 * cs, c0 = cs * BK;
      const long long aoff = (long long)(kh - 1) * rowoff + c0;
#pragma unroll
      for (int t = 0; t < APW; ++t)
        if (pw + NP * t < AP) dma16(((amask[t] >> kh) & 1) ? apix[t] + aoff : zero, As + (pw + NP * t) * 16 * BK);
    };
    auto stage_b = [&](int st) {
      u16* Bs = b_slot(st);
      if (st >= nst3) {  // the 1x1 downsample's weights (K columns K1 + c) in tap slot 1
        const int c0 = (st - nst3) * BK;
#pragma unroll
        for (int t = 0; t < BPW; ++t)
          if (pw + NP * t < BP && btap[t] == 1) dma16(bsrc[t] + a.K1 + c0, Bs + (pw + NP * t) * 16 * BK);
        return;
      }
      const int cs = st / 3, kh = st - 3 * cs, c0 = cs * BK;
#pragma unroll
      for (int t = 0; t < BPW; ++t)
        if (pw + NP * t < BP) dma16(bsrc[t] + kidx(kh, btap[t], c0), Bs + (pw + NP * t) * 16 * BK);
    };
    // this wave's A pieces per stage (the last piece index goes to the first AP % NP waves)
    const bool big = pw < AP - (APW - 1) * NP;
    auto wait_a = [&]() {  // all but this wave's A pieces of the newest stage
      if (big)
        vm_wait<APW>();
      else
        vm_wait<APW - 1>();
    };
    if (nst > 0) {
      stage_a(0);
      stage_b(0);
    }
    if (nst > 1) {
      stage_a(1);
      wait_a();
    } else {
      vm_wait<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int st = 0; st < nst; ++st) {  // B(st + 1), then A(st + 2); B(st + 1) and A(st + 1) land, A(st + 2) may fly
      if (st + 1 < nst) stage_b(st + 1);
      if (st + 2 < nst) {
        stage_a(st + 2);
        wait_a();
      } else {
        vm_wait<0>();
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    return;
  }

  // ------------------------------------------------------------------------------------ consumer
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int r = lane & 15;
  const int q = lane >> 4;
  unsigned emask = 0;  // bit 2i: ow 0 (tap kw 0 reads padding), bit 2i + 1: ow W - 1 (kw 2)
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * (BM / WM) + i * 16 + r;
    const int ow = (m % HW) % a.W;
    if (ow == 0) emask |= 1u << (2 * i);
    if (ow == a.W - 1) emask |= 2u << (2 * i);
  }
  __builtin_amdgcn_s_barrier();  // stage 0 has landed
  asm volatile("" ::: "memory");
  for (int st = 0; st < nst; ++st) {
    const u16* As = a_slot(st);
    const u16* Bs = b_slot(st);
    const bool ds = st >= nst3;  // a DS stage is read at offset 1 only (no taps, no edges)
#if EOSV_BF16_TS_BEARLY
    // BEARLY (r06 A/B): taps 1 and 2 of a 3x3 stage get their B fragments and first A fragment in
    // the previous tap's last group, fragment j right behind the MFMA that last reads the previous
    // tap's fragment j.  A DS stage runs its one tap (offset 1) as iteration 0, so the reads at an
    // iteration's start stay unconditional (a runtime branch around them spilled the tile)
    bf16x8 bfr[TN], afr[2];
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      if (ds && kw != 0) continue;
      const int tap = ds ? 1 : kw;
      auto rdB = [&](int tp, int j) {
        const int row = tp * BN + wn * (BN / WN) + j * 16 + r;
        return *(const bf16x8*)(Bs + row * BK + ((q ^ ((row >> 1) & 3)) * 8));
      };
      auto rdAt = [&](int tp, int i) {
        const int row = wm * (BM / WM) + i * 16 + r + tp;  // pixel m0 + (row - tp) at tap tp
        bf16x8 f = *(const bf16x8*)(As + row * BK + ((q ^ ((row >> 1) & 3)) * 8));
        if (tp != 1 && ((emask >> (2 * i + (tp >> 1))) & 1)) f = bf16x8{};
        return f;
      };
      auto rdA = [&](int i) { return rdAt(tap, i); };
      if (kw == 0) {
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = rdB(tap, j);
        afr[0] = rdA(0);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (kw < 2 && i == TM - 1) {  // (a DS stage reads tap 1's fragments here and never uses them)
          static_assert(TM % 2 == 0, "the next tap's first A fragment goes into the free slot 0");
          afr[0] = rdAt(kw + 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[1], bfr[j], acc[i][j], 0, 0, 0);
            bfr[j] = rdB(kw + 1, j);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
          continue;
        }
#else
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      if (ds && kw != 1) continue;
      bf16x8 bfr[TN], afr[2];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = kw * BN + wn * (BN / WN) + j * 16 + r;
        bfr[j] = *(const bf16x8*)(Bs + row * BK + ((q ^ ((row >> 1) & 3)) * 8));
      }
      auto rdA = [&](int i) {
        const int row = wm * (BM / WM) + i * 16 + r + kw;  // pixel m0 + (row - kw) at tap kw
        bf16x8 f = *(const bf16x8*)(As + row * BK + ((q ^ ((row >> 1) & 3)) * 8));
        if (kw != 1 && ((emask >> (2 * i + (kw >> 1))) & 1)) f = bf16x8{};
        return f;
      };
      afr[0] = rdA(0);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#endif
        if (i + 1 < TM) afr[(i + 1) & 1] = rdA(i + 1);
        if constexpr (EOSV_BF16_RFIRST) {  // r06 A/B: the next A fragment's read ahead of all TN MFMAs
          if (i + 1 < TM) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, TN, 0);
        } else {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if (i + 1 < TM) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, TN - 1, 0);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[i & 1], bfr[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // epilogue (conv_bf16_ts_kernel's, consumer waves only, bf16 layout)
  u16* __restrict__ y = (u16*)a.y;
  const u16* __restrict__ res = (const u16*)a.res;
  constexpr int EPR = WM * 32, EPS = BN + 4;
  static_assert(EPR * EPS * 4 <= SMEM * 2, "epilogue tile must fit the ring");
  float* ep = (float*)smem;
  float bcol[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) bcol[j] = a.bias ? a.bias[n0 + wn * (BN / WN) + j * 16 + r] : 0.f;
  constexpr int nthreads = 64 * NW;
  constexpr int NPASS = BM / WM / 32;
  constexpr int IPT = EPR * (BN / 8) / (64 * NW);
  static_assert(IPT * 64 * NW == EPR * (BN / 8), "epilogue work divides evenly");
  const long long ostr = a.Cout;
  const long long tile_bytes = (long long)min(BM, M - m0) * ostr * 2;
  const int nrec = (int)min(tile_bytes, 0x7fffffffLL);
  const __amdgpu_buffer_rsrc_t yr =
      __builtin_amdgcn_make_buffer_rsrc((void*)(y + (long long)m0 * ostr), (short)0, nrec, 0x00020000);
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(res ? res + (long long)m0 * ostr : zero), (short)0, res ? nrec : 0, 0x00020000);
  v4u rv[IPT];  // one residual set (two spilled at 168 VGPRs): pass i's load under its LDS write
  auto chunk = [&](int i, int t, int& lrow, int& c8, int& voff) {
    const int idx = tid + t * nthreads;
    lrow = idx / (BN / 8);
    c8 = idx - lrow * (BN / 8);
    const int ml = (lrow >> 5) * (BM / WM) + i * 32 + (lrow & 31);
    voff = (int)(((long long)ml * ostr + n0 + c8 * 8) * 2);
  };
  auto load_res = [&](int i) {
#pragma unroll
    for (int t = 0; t < IPT; ++t) {
      int lrow, c8, voff;
      chunk(i, t, lrow, c8, voff);
      rv[t] = __builtin_amdgcn_raw_buffer_load_b128(rr, voff, 0, 0);
    }
  };
  const float rlow = a.relu ? 0.f : -INFINITY;
#pragma unroll
  for (int i = 0; i < NPASS; ++i) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    load_res(i);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int lrow = wm * 32 + t * 16 + 4 * q + e;
          ep[lrow * EPS + wn * (BN / WN) + j * 16 + r] = acc[i * 2 + t][j][e] + bcol[j];
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int t = 0; t < IPT; ++t) {
      int lrow, c8, voff;
      chunk(i, t, lrow, c8, voff);
      const float4 v0 = *(const float4*)(ep + lrow * EPS + c8 * 8);
      const float4 v1 = *(const float4*)(ep + lrow * EPS + c8 * 8 + 4);
      float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      const v4u r4 = rv[t];
      const unsigned ru[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[2 * k] += bf2f((u16)(ru[k] & 0xffff));
        v[2 * k + 1] += bf2f((u16)(ru[k] >> 16));
      }
      v4u pk;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        pk[k] = (unsigned)f2bf(fmaxf(v[2 * k], rlow)) | ((unsigned)f2bf(fmaxf(v[2 * k + 1], rlow)) << 16);
      __builtin_amdgcn_raw_buffer_store_b128(pk, yr, voff, 0, 0);
    }
  }
}

// shapes this kernel takes: stride-1 pad-1 3x3, Cin % 32, Cout 64 (512 x 64 tiles), 128 (512 x 128)
// or a multiple of 256 (256 x 256), optionally a fused 1x1 downsample (Cin2 % 32), no stem
bool conv_bf16_ts_ok(const ConvArgs& a) {
  const bool ds_ok = !a.x2 ? a.K == 9 * a.Cin : (a.K1 == 9 * a.Cin && a.K == a.K1 + a.Cin2 && a.Cin2 % 32 == 0);
  return a.Cin != 3 && a.KH == 3 && a.KW == 3 && a.KWp == 3 && a.stride == 1 && a.pad == 1 && a.Ho == a.H &&
         a.Wo == a.W && a.Cin % 32 == 0 && ds_ok && (a.Cout == 64 || a.Cout == 128 || a.Cout % 256 == 0) && a.zero;
}

#ifndef EOSV_BF16_TS_WS_DEF
#define EOSV_BF16_TS_WS_DEF 1
#endif

int launch_conv_bf16_ts(const ConvArgs& a, hipStream_t s) {
  if (!conv_bf16_ts_ok(a)) return set_error("conv_bf16_ts: unsupported shape"), EOSV_ERR_UNSUPPORTED;
  const long long M = (long long)a.N * a.Ho * a.Wo;
  const int BM = a.Cout <= 128 ? 512 : 256, BN = a.Cout <= 128 ? a.Cout : 256;
  const long long nb = ((M + BM - 1) / BM) * (a.Cout / BN);
  if (nb > 0x7fffffffLL) return set_error("conv_bf16_ts: grid too large"), EOSV_ERR_UNSUPPORTED;
#define TS_LAUNCH(BM_, BN_, WM_, WN_)                                                                             \
  if (a.plan) {                                                                                                  \
    static const int occ = kernel_occupancy((const void*)conv_bf16_ts_kernel<BM_, BN_, WM_, WN_, false>,           \
                                            64 * WM_ * WN_);                                                     \
    return record_launch(a.plan, nb, occ);                                                                       \
  }                                                                                                              \
  if (a.split)                                                                                                   \
    hipLaunchKernelGGL((conv_bf16_ts_kernel<BM_, BN_, WM_, WN_, true>), dim3((unsigned)nb), dim3(64 * WM_ * WN_), 0, \
                       s, a);                                                                                    \
  else                                                                                                           \
    hipLaunchKernelGGL((conv_bf16_ts_kernel<BM_, BN_, WM_, WN_, false>), dim3((unsigned)nb), dim3(64 * WM_ * WN_), \
                       0, s, a);
  static const int tsws = env_switch("EOSV_BF16_TS_WS", EOSV_BF16_TS_WS_DEF);  // 1: warp-specialised 512 x 128 tile (A/B switch; r04: R18 layer-2 3x3s 7-10 %, R50 stage-2 3x3s 4-7 % faster)
  if (tsws && !a.split && a.Cout == 128) {
    constexpr int NT = 64 * (4 * 2 + 4);
    if (a.plan) {
      static const int occ = kernel_occupancy((const void*)conv_bf16_ts_ws_kernel<512, 128, 4, 2, 4>, NT);
      return record_launch(a.plan, nb, occ);
    }
    hipLaunchKernelGGL((conv_bf16_ts_ws_kernel<512, 128, 4, 2, 4>), dim3((unsigned)nb), dim3(NT), 0, s, a);
    EOSV_LAUNCH_CHECK();
    return EOSV_OK;
  }
  if (a.Cout == 64) {
    TS_LAUNCH(512, 64, 8, 1)
  } else if (a.Cout == 128) {
    TS_LAUNCH(512, 128, 4, 2)
  } else {
    TS_LAUNCH(256, 256, 2, 4)
  }
#undef TS_LAUNCH
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

}  // namespace eosv
