// Implicit-GEMM conv, exact-f32 MFMA, LDS-DMA staging (v2 of conv_f32.hip).
//
// Same GEMM view as conv_f32.hip (M = N*Ho*Wo, N = Cout, K = taps x Cin, B = [Cout][K]),
// but the A/B tiles move HBM/L2 -> LDS with global_load_lds_dwordx4 into a 2-deep LDS
// ring: no staging registers, ONE barrier per K-step, the next tile's DMA in flight
// while the current one feeds the MFMAs.
//
// LDS image: each DMA wave-instruction writes 1 KiB linearly (lane*16 B), i.e. 1024/(4*BK)
// whole rows, so rows are unpadded.  Bank spread comes from an XOR swizzle applied on
// the SOURCE address: physical 16-B chunk c' of row r holds logical chunk c' ^ f(r),
// f(r) = (r / (64/BK)) & (BK/4 - 1).  For the MFMA fragment reads (lane -> row lane&31,
// chunk h*BK/8 + g) every ds_read_b128 lane group then touches 16 distinct bank slots.
// Out-of-bounds im2col taps (zero padding, M/N tails) read a zeroed 16-B line (a.zero).
//
// Addressing is hoisted: each lane keeps, per staged row, the pointer of its (ih0, iw0)
// pixel and the validity window; per K-step only a wave-uniform tap offset is added.
//
// Stem (Cin 3): the input is dense padded RGB, [N][H+2p][Wp][3] (Wp = W+2p rounded up to
// even) with zero borders, and
// K is laid out [kh][24] (kw*3 + c, 21 real + 3 zero weights) = 42 16-B chunks, padded to
// 176 = 11 K-steps of 16: 84 % of the MFMA work is real (NHWC4 with kw padded to 8: 66 %).
// A lane's chunk g = 4*kt + lc is kernel row g / 6, floats 4*(g % 6) .. +3 of that row's
// 21-float tap run; the 16-B DMA source is then only 4-B aligned, which LDS-DMA accepts
// (tests/native/dma_probe.cpp).  No bounds checks: the borders are real zeros.
#include "common.h"

#include <algorithm>

namespace eosv {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int BM, int BN, int BK, int WM, int WN, bool STEM, int NS, bool EPI_LDS, bool DS>
__global__ __launch_bounds__(64 * WM * WN) void conv_f32_dma_kernel(ConvArgs a) {
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  constexpr int CPR = BK / 4;         // 16-B chunks per row
  constexpr int RPI = 64 / CPR;       // rows per DMA instruction
  constexpr int RPB = 64 / BK;        // rows per 256-B bank row
  constexpr int AI = BM / (RPI * NW);  // DMA instructions per wave (A)
  constexpr int BI = BN / (RPI * NW);
  constexpr int STAGE = (BM + BN) * BK;
  static_assert(AI >= 1 && BI >= 1 && TM >= 1 && TN >= 1, "tile shape");
  static_assert(!STEM || BK == 16, "stem chunk mapping assumes 4 chunks per K-step");
  __shared__ __attribute__((aligned(16))) float smem[NS * STAGE];
  static_assert(NS == 2 || NS == 3, "ring depth");

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int HoWo = a.Ho * a.Wo;
  const int M = a.N * HoWo;
  const int nN = (a.Cout + BN - 1) / BN;
  const int bt = xcd_tile(blockIdx.x, gridDim.x, a.xcd);
  const int mt = bt / nN;
  const int nt = bt - mt * nN;
  const int m0 = mt * BM, n0 = nt * BN;
  const float* __restrict__ x = (const float*)a.x;
  const float* __restrict__ w = (const float*)a.w;
  const float* zero = (const float*)a.zero;

  const int lr = lane / CPR;
  const int pc = lane % CPR;
  // per staged A row: pointer at pixel (ih0, iw0) + this lane's logical chunk, and ih0/iw0
  const float* arow[AI];
  const float* arow2[DS ? AI : 1];  // DS: the fused downsample's input pixel (always in bounds)
  int aih[AI], aiw[AI];
  const int xrow = ((a.W + 2 * a.pad + 1) & ~1) * 3;  // STEM: floats per padded input row
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int row = wid * (BM / NW) + RPI * j + lr;
    const int lc = pc ^ ((row / RPB) & (CPR - 1));
    const int m = m0 + row;
    if (m < M) {
      const int img = m / HoWo;
      const int rem = m - img * HoWo;
      const int oh = rem / a.Wo;
      const int ow = rem - oh * a.Wo;
      aih[j] = oh * a.stride - a.pad;
      aiw[j] = ow * a.stride - a.pad;
      if constexpr (STEM) {
        // padded coordinates of tap (0, 0) are (oh*stride, ow*stride); aiw holds the chunk
        aiw[j] = lc;
        arow[j] = x + ((long long)img * (a.H + 2 * a.pad) + oh * a.stride) * xrow + (long long)ow * a.stride * 3;
      } else {
        arow[j] = x + (((long long)img * a.H + aih[j]) * a.W + aiw[j]) * a.Cin + lc * 4;
        if constexpr (DS)
          arow2[j] = (const float*)a.x2 +
                     (((long long)img * a.H2 + oh * a.stride2) * a.W2 + ow * a.stride2) * a.Cin2 + lc * 4;
      }
    } else {
      aih[j] = -(1 << 28);
      aiw[j] = 0;
      arow[j] = x;
      if constexpr (DS) arow2[j] = nullptr;
    }
  }
  const float* brow[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int row = wid * (BN / NW) + RPI * j + lr;
    const int lc = pc ^ ((row / RPB) & (CPR - 1));
    const int n = n0 + row;
    brow[j] = n < a.Cout ? w + (long long)n * a.K + lc * 4 : nullptr;
  }

  // tap of the next A stage, advanced per stage call (k0 grows by BK; Cin % BK == 0): no
  // per-K-step divisions by Cin and KW.  K order (kh, kw, cin), or with a.kcm (r04: weights
  // stored that way) chunk-major (cin / KC, kh, kw, cin % KC): a pixel's next tap is read
  // KC / BK K-steps later instead of Cin / BK, while its rows are still in L2
  const int KC = a.kcm;  // channel chunk (a power of two, a multiple of BK: the launcher checks)
  const bool kcm = KC != 0;
  int nc0 = 0, nkw = 0, nkh = 0;
  auto stage = [&](int k0, int slot) {
    float* As = smem + slot * STAGE;
    float* Bs = As + BM * BK;
    if constexpr (STEM) {
#pragma unroll
      for (int j = 0; j < AI; ++j) {
        const int g = (k0 >> 2) + aiw[j];
        const int kh = g / 6;
        const bool ok = aih[j] > -(1 << 27) && kh < a.KH;
        const float* src = ok ? arow[j] + kh * xrow + (g - 6 * kh) * 4 : zero;
        float* dst = As + (wid * (BM / NW) + RPI * j) * BK;
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      }
    } else if (DS && k0 >= a.K1) {
#pragma unroll
      for (int j = 0; j < (DS ? AI : 1); ++j) {
        const float* src = arow2[j] ? arow2[j] + (k0 - a.K1) : zero;
        float* dst = As + (wid * (BM / NW) + RPI * j) * BK;
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      }
    } else {
      const int kh = nkh, kw = nkw;
      const long long toff = ((long long)kh * a.W + kw) * a.Cin + nc0;  // wave-uniform
      nc0 += BK;
      if (kcm) {
        if ((nc0 & (KC - 1)) == 0) {  // chunk done for this tap: next tap, same chunk
          nc0 -= KC;
          if (++nkw == a.KW) {
            nkw = 0;
            if (++nkh == a.KH) nkh = 0, nc0 += KC;  // all taps done: next chunk
          }
        }
      } else if (nc0 == a.Cin) {
        nc0 = 0;
        if (++nkw == a.KW) nkw = 0, ++nkh;
      }
#pragma unroll
      for (int j = 0; j < ((EOSV_ABL(a) & 8) ? 0 : AI); ++j) {  // profiling: 8 = no A-tile DMA
        const int ih = aih[j] + kh, iw = aiw[j] + kw;
        const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const float* src = ok ? arow[j] + toff : zero;
        float* dst = As + (wid * (BM / NW) + RPI * j) * BK;
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < ((EOSV_ABL(a) & 16) ? 0 : BI); ++j) {  // profiling: 16 = no B-tile DMA
      const float* src = brow[j] ? brow[j] + k0 : zero;
      float* dst = Bs + (wid * (BN / NW) + RPI * j) * BK;
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  const int h = lane >> 5;
  const int r = lane & 31;
  const int sw = (r / RPB) & (CPR - 1);
  // K-step range: all of K, or slice blockIdx.y of gridDim.y (split-K, raw partials)
  const int nkt = a.K / BK;
  const int kb = (int)((long long)nkt * blockIdx.y / gridDim.y);
  const int nk = (int)((long long)nkt * (blockIdx.y + 1) / gridDim.y) - kb;
  if (kb > 0 && !STEM) {  // the tap counters of K column kb * BK
    const int k = kb * BK;
    int t;
    if (kcm) {
      const int per = KC * a.KH * a.KW, ch = k / per, rem = k - ch * per;
      t = rem / KC;
      nc0 = ch * KC + (rem - t * KC);
    } else {
      t = k / a.Cin;
      nc0 = k - t * a.Cin;
    }
    nkh = t / a.KW;
    nkw = t - nkh * a.KW;
  }
  constexpr int PER = AI + BI;  // DMA instructions per stage per wave
  for (int p = 0; p < NS - 1 && p < nk; ++p) stage((kb + p) * BK, p);
  if (NS == 3 && nk > 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PER) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  int slot = 0, wslot = NS - 1;
  for (int kt = 0; kt < nk; ++kt) {
    const bool issue = kt + NS - 1 < nk;
    if (issue && !(EOSV_ABL(a) & 1)) stage((kb + kt + NS - 1) * BK, wslot);
    const float* As = smem + slot * STAGE;
    const float* Bs = As + BM * BK;
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      const int pch = ((h * (BK / 8) + g) ^ sw) * 4;
      f32x4 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *(const f32x4*)(As + (wm * (BM / WM) + i * 32 + r) * BK + pch);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = *(const f32x4*)(Bs + (wn * (BN / WN) + j * 32 + r) * BK + pch);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
    }
    // the next slot's DMA must have landed (leave the newest stage in flight when NS == 3),
    // and every wave's reads of this slot must be done before anyone refills it
    if (EOSV_ABL(a) & 4) {
      // profiling: DMA issued but not waited for (results wrong)
    } else if (NS == 3 && issue) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PER) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    slot = slot + 1 == NS ? 0 : slot + 1;
    wslot = wslot + 1 == NS ? 0 : wslot + 1;
  }

  const bool part = gridDim.y > 1;  // split-K: raw partial sums, epilogue in the slice sum
  float* __restrict__ y = part ? a.kws + (long long)blockIdx.y * M * a.Cout : (float*)a.y;
  const float* __restrict__ res = part ? nullptr : (const float*)a.res;
  const int relu = part ? 0 : a.relu;
  float bcol[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / WN) + j * 32 + r;
    bcol[j] = (!part && a.bias && n < a.Cout) ? a.bias[n] : 0.f;
  }
  if constexpr (EPI_LDS) {
    // Epilogue staged through LDS (the ring is free): pass (i, wsel) moves the 32 x BN rows
    // of M-subtile i of the waves with wm == wsel, so residual loads / output stores are
    // 16 B per lane over whole 128-B lines.
    constexpr int EPS = BN + 4;
    static_assert(32 * EPS <= NS * STAGE, "epilogue slab must fit the ring");
    float* ep = smem;
    const int nthreads = 64 * NW;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      for (int wsel = 0; wsel < WM; ++wsel) {
        __syncthreads();
        if (wm == wsel) {
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q)
              ep[((q & 3) + 8 * (q >> 2) + 4 * h) * EPS + wn * (BN / WN) + j * 32 + r] = acc[i][j][q] + bcol[j];
        }
        __syncthreads();
        for (int idx = tid; idx < 32 * (BN / 4); idx += nthreads) {
          const int lrow = idx / (BN / 4);
          const int c4 = idx - lrow * (BN / 4);
          const int m = m0 + wsel * (BM / WM) + i * 32 + lrow;
          const int n = n0 + c4 * 4;
          if (m >= M || n >= a.Cout) continue;
          float4 v = *(const float4*)(ep + lrow * EPS + c4 * 4);
          const long long o = (long long)m * a.Cout + n;
          if (res) {
            const float4 rv = *(const float4*)(res + o);
            v.x += rv.x;
            v.y += rv.y;
            v.z += rv.z;
            v.w += rv.w;
          }
          if (relu) {
            v.x = fmaxf(v.x, 0.f);
            v.y = fmaxf(v.y, 0.f);
            v.z = fmaxf(v.z, 0.f);
            v.w = fmaxf(v.w, 0.f);
          }
          if (EOSV_ABL(a) & 2)
            asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
          else
            *(float4*)(y + o) = v;
        }
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / WN) + j * 32 + r;
    if (n >= a.Cout) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + wm * (BM / WM) + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (m < M) {
          const long long o = (long long)m * a.Cout + n;
          float v = acc[i][j][q] + bcol[j];
          if (res) v += res[o];
          if (relu) v = fmaxf(v, 0.f);
          if (EOSV_ABL(a) & 2) asm volatile("" ::"v"(v)); else y[o] = v;
        }
      }
    }
  }
}

// Warp-specialised f32 tile (r04, EOSV_F32_WS): NW = WM x WN consumer waves that only read LDS
// fragments and issue v_mfma_f32_32x32x2_f32, and NP producer waves that only stage A (im2col)
// and B rows by LDS-DMA (each DMA piece costs its wave 60-185 cycles of issue, MI355X_MICROARCH.md;
// in conv_f32_dma_kernel both waves of a SIMD issue theirs at the K-step's start).  Split rings:
// 3 A slots (two K-steps ahead) and 2 B slots (one ahead); one barrier per K-step; producers
// leave after the K loop.  Same K order, MFMA order and LDS-staged epilogue as conv_f32_dma_kernel
// (EPI_LDS): bit-identical outputs.  Inference only (no split-K), tap-major or chunk-major K.
// OCC: workgroups per CU the register budget is sized for (2 at NP 4: <= 80 VGPRs, 6 waves per SIMD;
// 2 at NP 2: <= 96)
// EPD (r05 A/B, EOSV_F32_EPD): the epilogue straight from the accumulators, no LDS staging and no
// barriers: a 32 x 32 accumulator register is 2 rows x 32 consecutive channels, i.e. two whole
// 128-B lines per wave instruction for the residual load and the store.
#ifndef EOSV_F32_PRIO_DEF
#define EOSV_F32_PRIO_DEF 1  // r05 release A/B (profiles/r05m_ab_f32_prio.txt): 1 +0.26 %, 2 +0.17 % over 0
#endif
template <int BM, int BN, int WM, int WN, int NP, bool DS, int OCC, bool EPD = false>
__global__ __launch_bounds__(64 * (WM * WN + NP), (OCC * (WM * WN + NP) + 3) / 4) void conv_f32_ws_kernel(ConvArgs a) {
  constexpr int BK = 16, CPR = BK / 4, RPI = 64 / CPR, RPB = 64 / BK;
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int AI = BM / (RPI * NP), BI = BN / (RPI * NP);  // DMA pieces per producer wave
  static_assert(AI >= 1 && BI >= 1 && AI * RPI * NP == BM && BI * RPI * NP == BN, "tile shape");
  constexpr int AS = BM * BK, BS = BN * BK;  // floats per A / B slot
  constexpr int EPS = BN + 4;
  constexpr int SMEM = 3 * AS + 2 * BS > 32 * EPS ? 3 * AS + 2 * BS : 32 * EPS;
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  auto a_slot = [&](int kt) { return smem + (kt % 3) * AS; };
  auto b_slot = [&](int kt) { return smem + 3 * AS + (kt & 1) * BS; };

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int HoWo = a.Ho * a.Wo;
  const int M = a.N * HoWo;
  const int nN = (a.Cout + BN - 1) / BN;
  const int bt = xcd_tile(blockIdx.x, gridDim.x, a.xcd);
  const int mt = bt / nN;
  const int nt = bt - mt * nN;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nk = a.K / BK;

  if (wid >= NW) {  // ---------------------------------------------------------------- producer
    const int pw = wid - NW;
    const float* __restrict__ x = (const float*)a.x;
    const float* __restrict__ w = (const float*)a.w;
    const float* zero = (const float*)a.zero;
    const int lr = lane / CPR, pc = lane % CPR;
    const float* arow[AI];
    const float* arow2[DS ? AI : 1];
    int aih[AI], aiw[AI];
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int row = pw * (BM / NP) + RPI * j + lr;
      const int lc = pc ^ ((row / RPB) & (CPR - 1));
      const int m = m0 + row;
      if (m < M) {
        const int img = m / HoWo, rem = m - img * HoWo, oh = rem / a.Wo, ow = rem - oh * a.Wo;
        aih[j] = oh * a.stride - a.pad;
        aiw[j] = ow * a.stride - a.pad;
        arow[j] = x + (((long long)img * a.H + aih[j]) * a.W + aiw[j]) * a.Cin + lc * 4;
        if constexpr (DS)
          arow2[j] = (const float*)a.x2 + (((long long)img * a.H2 + oh * a.stride2) * a.W2 + ow * a.stride2) * a.Cin2 + lc * 4;
      } else {
        aih[j] = -(1 << 28);
        aiw[j] = 0;
        arow[j] = x;
        if constexpr (DS) arow2[j] = nullptr;
      }
    }
    const float* brow[BI];
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const int row = pw * (BN / NP) + RPI * j + lr;
      const int lc = pc ^ ((row / RPB) & (CPR - 1));
      const int n = n0 + row;
      brow[j] = n < a.Cout ? w + (long long)n * a.K + lc * 4 : nullptr;
    }
    // tap counters of the next A stage (A stages are issued in K order)
    const int KC = a.kcm;
    int nc0 = 0, nkw = 0, nkh = 0;
    auto stage_a = [&](int kt) {
      float* As = a_slot(kt);
      const int k0 = kt * BK;
      if (DS && k0 >= a.K1) {
#pragma unroll
        for (int j = 0; j < (DS ? AI : 1); ++j) {
          const float* src = arow2[j] ? arow2[j] + (k0 - a.K1) : zero;
          __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(As + (pw * (BM / NP) + RPI * j) * BK), 16, 0, 0);
        }
        return;
      }
      const int kh = nkh, kw = nkw;
      const long long toff = ((long long)kh * a.W + kw) * a.Cin + nc0;
      nc0 += BK;
      if (KC) {
        if ((nc0 & (KC - 1)) == 0) {
          nc0 -= KC;
          if (++nkw == a.KW) {
            nkw = 0;
            if (++nkh == a.KH) nkh = 0, nc0 += KC;
          }
        }
      } else if (nc0 == a.Cin) {
        nc0 = 0;
        if (++nkw == a.KW) nkw = 0, ++nkh;
      }
#pragma unroll
      for (int j = 0; j < AI; ++j) {
        const int ih = aih[j] + kh, iw = aiw[j] + kw;
        const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const float* src = ok ? arow[j] + toff : zero;
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(As + (pw * (BM / NP) + RPI * j) * BK), 16, 0, 0);
      }
    };
    auto stage_b = [&](int kt) {
      float* Bs = b_slot(kt);
#pragma unroll
      for (int j = 0; j < BI; ++j) {
        const float* src = brow[j] ? brow[j] + kt * BK : zero;
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(Bs + (pw * (BN / NP) + RPI * j) * BK), 16, 0, 0);
      }
    };
    if (nk > 0) {
      stage_a(0);
      stage_b(0);
    }
    if (nk > 1) {
      stage_a(1);
      vm_wait<AI>();
    } else {
      vm_wait<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int kt = 0; kt < nk; ++kt) {  // B(kt + 1), then A(kt + 2); B(kt + 1) and A(kt + 1) land
      if (kt + 1 < nk) stage_b(kt + 1);
      if (kt + 2 < nk) {
        stage_a(kt + 2);
        vm_wait<AI>();
      } else {
        vm_wait<0>();
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    return;
  }

  // ------------------------------------------------------------------------------------ consumer
  // EOSV_F32_PRIO (release-variant A/B, tools/build_variant.sh): 1 = every consumer wave at
  // priority 1 (the producers' DMA issue then yields the SIMD to MFMA issue), 2 = the second half
  // of the consumers only (MI355X_MICROARCH.md, "Two waves per SIMD", item 4)
  if constexpr (EOSV_F32_PRIO_DEF == 1) __builtin_amdgcn_s_setprio(1);
  if constexpr (EOSV_F32_PRIO_DEF == 2)
    if (wid >= NW / 2) __builtin_amdgcn_s_setprio(1);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  const int h = lane >> 5;
  const int r = lane & 31;
  const int sw = (r / RPB) & (CPR - 1);
  __builtin_amdgcn_s_barrier();  // stage 0 has landed
  asm volatile("" ::: "memory");
  // Fragment addressing (r05): the 80-VGPR budget of the OCC 2 / NP 4 tile holds the 64
  // accumulators, the fragments and almost nothing else.  hipcc turned the slot offsets (kt % 3,
  // kt & 1) into per-lane induction variables and spilled two of them: two scratch reloads with a
  // vmcnt(0) wait in every K-step.  Now: one lane offset lg0 (chunk g = 1 flips bit 4 of it:
  // ((2h + 1) ^ sw) = ((2h) ^ sw) ^ 1), the wave-uniform slot offsets through readfirstlane (opaque:
  // no induction variables), and the A fragment read per row tile (12 fragment VGPRs live, not 16).
  // The same MFMAs in the same per-accumulator order: bit-identical.
  const int lg0 = (r * BK + ((h * (BK / 8)) ^ sw) * 4) * 4;
  const unsigned char* sbase = (const unsigned char*)smem;
  for (int kt = 0; kt < nk; ++kt) {
    const int aoff = __builtin_amdgcn_readfirstlane((kt % 3) * AS * 4 + wm * (BM / WM) * BK * 4);
    const int boff = __builtin_amdgcn_readfirstlane(3 * AS * 4 + (kt & 1) * BS * 4 + wn * (BN / WN) * BK * 4);
#pragma unroll
    for (int g = 0; g < BK / 8; ++g) {
      const int lo = g ? (lg0 ^ 16) : lg0;
      f32x4 bf[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = *(const f32x4*)(sbase + boff + lo + j * 32 * BK * 4);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const f32x4 af = *(const f32x4*)(sbase + aoff + lo + i * 32 * BK * 4);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s4], bf[j][s4], acc[i][j], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // epilogue (conv_f32_dma_kernel's EPI_LDS one; consumer waves only)
  float* __restrict__ y = (float*)a.y;
  const float* __restrict__ res = (const float*)a.res;
  float bcol[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / WN) + j * 32 + r;
    bcol[j] = (a.bias && n < a.Cout) ? a.bias[n] : 0.f;
  }
  if constexpr (EPD) {
    // same arithmetic order as the staged epilogue: (acc + bias) + residual, then ReLU
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * (BN / WN) + j * 32 + r;
        if (n >= a.Cout) continue;
        float rv[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int m = m0 + wm * (BM / WM) + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
          rv[q] = (res && m < M) ? res[(long long)m * a.Cout + n] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int m = m0 + wm * (BM / WM) + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
          if (m >= M) continue;
          float v = acc[i][j][q] + bcol[j];
          if (res) v += rv[q];
          if (a.relu) v = fmaxf(v, 0.f);
          y[(long long)m * a.Cout + n] = v;
        }
      }
    return;
  }
  float* ep = smem;
  constexpr int nthreads = 64 * NW;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    for (int wsel = 0; wsel < WM; ++wsel) {
      __syncthreads();
      if (wm == wsel) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int q = 0; q < 16; ++q)
            ep[((q & 3) + 8 * (q >> 2) + 4 * h) * EPS + wn * (BN / WN) + j * 32 + r] = acc[i][j][q] + bcol[j];
      }
      __syncthreads();
      for (int idx = tid; idx < 32 * (BN / 4); idx += nthreads) {
        const int lrow = idx / (BN / 4);
        const int c4 = idx - lrow * (BN / 4);
        const int m = m0 + wsel * (BM / WM) + i * 32 + lrow;
        const int n = n0 + c4 * 4;
        if (m >= M || n >= a.Cout) continue;
        float4 v = *(const float4*)(ep + lrow * EPS + c4 * 4);
        const long long o = (long long)m * a.Cout + n;
        if (res) {
          const float4 rv = *(const float4*)(res + o);
          v.x += rv.x;
          v.y += rv.y;
          v.z += rv.z;
          v.w += rv.w;
        }
        if (a.relu) {
          v.x = fmaxf(v.x, 0.f);
          v.y = fmaxf(v.y, 0.f);
          v.z = fmaxf(v.z, 0.f);
          v.w = fmaxf(v.w, 0.f);
        }
        *(float4*)(y + o) = v;
      }
    }
  }
}

// split-K (training entry only): enough slices to put ~2 workgroups on every CU, each slice at
// least 32 K-steps, at most 8
static int ksplit_count(long long blocks, int ksteps) {
  const long long want = (2LL * device_cu_count() + blocks - 1) / blocks;
  return (int)std::max(1LL, std::min({want, (long long)ksteps / 32, 8LL}));
}

// split-K epilogue: y = relu(sum over slices (in order) + bias + residual), float4 over Cout
__global__ void ksplit_sum_kernel(const float4* __restrict__ ws, int ks, long long mc4, int C4,
                                  const float* __restrict__ bias, const float4* __restrict__ res, int relu,
                                  float4* __restrict__ y) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < mc4; i += (long long)gridDim.x * blockDim.x) {
    float4 v = ws[i];
    for (int z = 1; z < ks; ++z) {
      const float4 u = ws[z * mc4 + i];
      v.x += u.x, v.y += u.y, v.z += u.z, v.w += u.w;
    }
    if (bias) {
      const float4 b = reinterpret_cast<const float4*>(bias)[i % C4];
      v.x += b.x, v.y += b.y, v.z += b.z, v.w += b.w;
    }
    if (res) {
      const float4 q = res[i];
      v.x += q.x, v.y += q.y, v.z += q.z, v.w += q.w;
    }
    if (relu) v.x = fmaxf(v.x, 0.f), v.y = fmaxf(v.y, 0.f), v.z = fmaxf(v.z, 0.f), v.w = fmaxf(v.w, 0.f);
    y[i] = v;
  }
}

static int launch_ksplit_sum(const ConvArgs& a, int ks, long long M, hipStream_t s) {
  const long long mc4 = M * a.Cout / 4;
  hipLaunchKernelGGL(ksplit_sum_kernel, dim3((unsigned)std::min<long long>((mc4 + 255) / 256, 1 << 20)), dim3(256), 0,
                     s, (const float4*)a.kws, ks, mc4, a.Cout / 4, a.bias, (const float4*)a.res, a.relu,
                     (float4*)a.y);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

template <int BM, int BN, int BK, int WM, int WN, bool STEM, int NS = 2, bool EPI = true>
static int launch_dma(const ConvArgs& a, hipStream_t s) {
  const long long M = (long long)a.N * a.Ho * a.Wo;
  const long long nb = ((M + BM - 1) / BM) * ((a.Cout + BN - 1) / BN);
  if (nb > 0x7fffffffLL) return set_error("conv: grid too large"), EOSV_ERR_UNSUPPORTED;
  if (a.plan) {
    static const int occ = kernel_occupancy(
        (const void*)conv_f32_dma_kernel<BM, BN, BK, WM, WN, false, NS, EPI, false>, 64 * WM * WN);
    return record_launch(a.plan, nb, occ);
  }
  int ks = 1;
  if (a.kws && !STEM && !a.x2 && EPI) {
    ks = ksplit_count(nb, a.K / BK);
    if ((long long)ks * M * a.Cout * (long long)sizeof(float) > a.kws_bytes) ks = 1;
  }
  if (a.x2) {
    if (STEM || a.K1 % BK || a.Cin2 % BK) return set_error("conv_f32: fused downsample shape"), EOSV_ERR_UNSUPPORTED;
    hipLaunchKernelGGL((conv_f32_dma_kernel<BM, BN, BK, WM, WN, false, NS, EPI, true>), dim3((unsigned)nb),
                       dim3(64 * WM * WN), 0, s, a);
  } else {
    hipLaunchKernelGGL((conv_f32_dma_kernel<BM, BN, BK, WM, WN, STEM, NS, EPI, false>), dim3((unsigned)nb, ks),
                       dim3(64 * WM * WN), 0, s, a);
  }
  EOSV_LAUNCH_CHECK();
  if (ks > 1) return launch_ksplit_sum(a, ks, M, s);
  return EOSV_OK;
}

// EOSV_F32_WS (r04): the warp-specialised tiles for the Cout >= 128 implicit-GEMM convs of the
// inference path (no split-K workspace): 1 one workgroup per CU (90 VGPRs), 2 two (80 VGPRs), 3 two
// workgroups of 2 producer waves each (96 VGPRs).
#ifndef EOSV_F32_WS_DEF
#define EOSV_F32_WS_DEF 2
#endif
static int f32_ws() {
  static const int v = env_switch("EOSV_F32_WS", EOSV_F32_WS_DEF);  // (A/B switch; r04: 2 is 4 % faster than 0 on R18 f32, 3 is 5 % slower than 0)
  return v;
}

template <int BM, int BN, int WM, int WN, int OCC, int NP = 4>
static int launch_ws(const ConvArgs& a, hipStream_t s) {
  constexpr int NT = 64 * (WM * WN + NP);
  const long long M = (long long)a.N * a.Ho * a.Wo;
  const long long nb = ((M + BM - 1) / BM) * ((a.Cout + BN - 1) / BN);
  if (nb > 0x7fffffffLL) return set_error("conv: grid too large"), EOSV_ERR_UNSUPPORTED;
  if (a.plan) {
    static const int occ = kernel_occupancy((const void*)conv_f32_ws_kernel<BM, BN, WM, WN, NP, false, OCC>, NT);
    return record_launch(a.plan, nb, occ);
  }
#ifdef EOSV_PROFILING
  static const int epd = env_switch("EOSV_F32_EPD", 0);  // 1: epilogue from registers (A/B)
  if (epd) {
    if (a.x2) {
      if (a.K1 % 16 || a.Cin2 % 16) return set_error("conv_f32: fused downsample shape"), EOSV_ERR_UNSUPPORTED;
      hipLaunchKernelGGL((conv_f32_ws_kernel<BM, BN, WM, WN, NP, true, OCC, true>), dim3((unsigned)nb), dim3(NT), 0, s, a);
    } else {
      hipLaunchKernelGGL((conv_f32_ws_kernel<BM, BN, WM, WN, NP, false, OCC, true>), dim3((unsigned)nb), dim3(NT), 0, s, a);
    }
    EOSV_LAUNCH_CHECK();
    return EOSV_OK;
  }
#endif
  if (a.x2) {
    if (a.K1 % 16 || a.Cin2 % 16) return set_error("conv_f32: fused downsample shape"), EOSV_ERR_UNSUPPORTED;
    hipLaunchKernelGGL((conv_f32_ws_kernel<BM, BN, WM, WN, NP, true, OCC>), dim3((unsigned)nb), dim3(NT), 0, s, a);
  } else {
    hipLaunchKernelGGL((conv_f32_ws_kernel<BM, BN, WM, WN, NP, false, OCC>), dim3((unsigned)nb), dim3(NT), 0, s, a);
  }
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

// Cout > 64 tiles: small batches (the training step: 96 frames) give grids below the chip's CU
// count, so the tile shrinks (same BK, same k-order per output: bit-identical results).
// 1 = 256x128, 2 = 128x128, 3 = 128x64.
static int f32_tile(const ConvArgs& a) {
  const long long M = (long long)a.N * a.Ho * a.Wo, cus = device_cu_count();
  auto blocks = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((a.Cout + bn - 1) / bn); };
  if (a.Cout <= 256 && blocks(256, 128) >= cus) return 1;
  if (blocks(128, 128) >= cus) return 2;
  return 3;
}

// Tile per layer (r01 / r01l A/B): 256x64 (4 waves of 64x64) for Cout 64, 256x128
// (8 waves) for Cout 128 / 256, 128x128 for Cout >= 512, all BK 16 with a 2-deep ring; 128x128 /
// 128x64 when the grid would not cover the CUs (small batches).  The fc
// head (M = frames, Cout = num_classes) runs here too: when Cout % 4 != 0 its rows are not 16-B
// aligned, so it takes the per-element epilogue instead of the LDS-staged float4 one.
int launch_conv_f32(const ConvArgs& a0, hipStream_t s) {
  ConvArgs a = a0;
  a.abl = env_switch("EOSV_CONV_ABL", 0);  // profiling build only: ablations, results are wrong when set
  const bool stem = (a.Cin == 3);
  if (!a.zero || (stem && (a.KWp != 8 || a.KW != 7 || a.K != (a.KH * 24 + 15) / 16 * 16)) ||
      (!stem && (a.K % 32 != 0 || a.Cin % 32 != 0))) {
    set_error("conv_f32: unsupported shape (K % 32, Cin % 32 or stem layout)");
    return EOSV_ERR_UNSUPPORTED;
  }
  if (stem) return launch_dma<128, 64, 16, 2, 2, true>(a, s);
  if (a.kcm && (a.kcm < 32 || (a.kcm & (a.kcm - 1)) || a.Cin % a.kcm))
    return set_error("conv_f32: chunk-major K needs a power-of-two chunk >= 32 dividing Cin"), EOSV_ERR_UNSUPPORTED;
  // stage-1 3x3 64->64 convs: row-strip direct conv (input staged once per strip, not per tap)
  static const int rows = env_switch("EOSV_F32_ROWS", 1);  // 0 = implicit GEMM (A/B switch)
  if (rows && !a.kcm && conv_rows_f32_ok(a)) return launch_conv_rows_f32(a, s);
  if (a.Cout % 4) {
    if (a.x2) return set_error("conv_f32: fused downsample needs Cout % 4 == 0"), EOSV_ERR_UNSUPPORTED;
    return launch_dma<128, 64, 16, 2, 2, false, 2, false>(a, s);
  }
  if (a.Cout <= 64) return launch_dma<256, 64, 16, 4, 1, false>(a, s);
#ifdef EOSV_PROFILING
  // A/B of the Cout >= 128 tiles: 1 BK 32, 2 three-deep ring, 3 128x128 everywhere, 4 256x256 at Cout >= 256
  static const int tile = env_switch("EOSV_F32_TILE", 0);
  if (tile == 1) return a.Cout <= 256 ? launch_dma<256, 128, 32, 4, 2, false>(a, s) : launch_dma<128, 128, 32, 2, 2, false>(a, s);
  if (tile == 2) return a.Cout <= 256 ? launch_dma<256, 128, 16, 4, 2, false, 3>(a, s) : launch_dma<128, 128, 16, 2, 2, false, 3>(a, s);
  if (tile == 3) return launch_dma<128, 128, 16, 2, 2, false>(a, s);
  if (tile == 4 && a.Cout >= 256) return launch_dma<256, 256, 16, 4, 2, false>(a, s);
  if (tile == 5) return launch_dma<512, 128, 16, 4, 2, false>(a, s);  // 8 waves of 128x64
  if (tile == 6 && a.Cout <= 256) return launch_dma<512, 128, 16, 4, 2, false>(a, s);
#endif
  if (f32_ws() && !a.kws) {
    const int t = f32_tile(a);
    if (t == 1) {
      if (f32_ws() == 3) return launch_ws<256, 128, 4, 2, 2, 2>(a, s);
      return f32_ws() == 2 ? launch_ws<256, 128, 4, 2, 2>(a, s) : launch_ws<256, 128, 4, 2, 1>(a, s);
    }
    if (t == 2) {
      if (f32_ws() == 3) return launch_ws<128, 128, 2, 2, 2, 2>(a, s);
      return f32_ws() == 2 ? launch_ws<128, 128, 2, 2, 2>(a, s) : launch_ws<128, 128, 2, 2, 1>(a, s);
    }
  }
  switch (f32_tile(a)) {
    case 1: return launch_dma<256, 128, 16, 4, 2, false>(a, s);
    case 2: return launch_dma<128, 128, 16, 2, 2, false>(a, s);
    default: return launch_dma<128, 64, 16, 2, 2, false>(a, s);
  }
}

int conv_f32_ksplit_slices(const ConvArgs& a) {
  if (a.Cin == 3 || a.x2 || a.Cout % 4 || a.Cout <= 64 || a.K % 32 || a.Cin % 32) return 1;
  if (env_switch("EOSV_F32_ROWS", 1) && conv_rows_f32_ok(a)) return 1;
  static const int bm[] = {0, 256, 128, 128}, bn[] = {0, 128, 128, 64};
  const int t = f32_tile(a);
  const long long M = (long long)a.N * a.Ho * a.Wo;
  return ksplit_count(((M + bm[t] - 1) / bm[t]) * ((a.Cout + bn[t] - 1) / bn[t]), a.K / 16);
}

}  // namespace eosv
