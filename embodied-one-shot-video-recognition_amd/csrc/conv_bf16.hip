// Implicit-GEMM conv on bf16 MFMA (v_mfma_f32_32x32x16_bf16), NHWC bf16 activations,
// f32 accumulation, folded BN + ReLU + residual in the epilogue, bf16 out.
//
// Same structure as conv_f32_dma.hip: A (im2col rows) and B ([Cout][K] weights) move by
// global_load_lds_dwordx4 into a 2-deep LDS ring, one barrier per K-step.  BK = 64 bf16
// = 128-B rows (8 x 16-B chunks), XOR swizzle chunk' = chunk ^ ((row >> 1) & 7) applied
// on the DMA source address.  One 16-B chunk = the 8 consecutive k a lane feeds one MFMA:
// in MFMA step s of a K-step, lane half h reads chunk 2s + h (k = 16s + 8h .. +7).
//
// Stem (Cin 3): dense padded RGB input [N][H+2p][Wp][3] bf16 (Wp = W+2p rounded up to even)
// with zero borders; K laid
// out [kh][24] (kw*3 + c: 21 real + 3 zero weights) = 21 16-B chunks, padded to 192 = 3
// K-steps (77 % of the MFMA work real; NHWC4 with kw padded to 8 and K 256: 57 %).  Chunk
// g = 8*kt + lc is kernel row g / 3, elements 8*(g % 3) .. +7 of that row's tap run; the
// 16-B DMA source is only 4-B aligned there (even padded row width, even stride; LDS-DMA
// accepts that: tests/native/dma_probe.cpp).
#include <hip/hip_bf16.h>

#include "common.h"

namespace eosv {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16;

__device__ __forceinline__ float bf_to_f(u16 v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ u16 f_to_bf(float f) { return __bfloat16_as_ushort(__float2bfloat16(f)); }

// MF = MFMA tile edge: 32 (v_mfma_f32_32x32x16_bf16) or 16 (v_mfma_f32_16x16x32_bf16; same
// cycles per FLOP, but the chip holds a higher clock on it with random operands)
// SPLIT: EOSV_F32X3 (ConvArgs::split): A reads virtual channel blocks (hi, lo, hi) of the stored
// (hi, lo) pixels; epilogue residual = hi + lo, output stored as (hi, lo)
// Tap order of a stride-2 3x3 conv's K loop (r03).  Its taps fall into four classes by the
// parity of (kh, kw): (0|2, 0|2), (0|2, 1), (1, 0|2), (1, 1) read disjoint input pixels, and
// the taps of one class read (nearly) the same pixels: kh = 0 and 2 are one input row apart,
// i.e. the next output row's kh = 0.  K-steps walk the taps class by class, so a pixel line's
// re-reads come one K-step apart and hit L2 (in (kh, kw) order they came 2-3 K-steps apart,
// when 32 CUs' staging had turned the XCD's L2 over: L2 hit rate 0.32-0.41, PMC r03).  Weights
// and pixels are indexed by the same tap, so only the accumulation order changes.
__device__ __forceinline__ int tap_order(const ConvArgs& a, int t) {
  constexpr unsigned long long PERM9 = 0x453718620ull;  // t -> tap: 0 2 6 8 1 7 3 5 4
  return (a.stride == 2 && a.KH == 3 && a.KW == 3) ? (int)((PERM9 >> (4 * t)) & 15) : t;
}
// (tap, first channel) of the K-step starting at k0 in the stored K order: k0 is a multiple of
// the kernel's BK (64 or 32); Cin is a multiple of 64, so a K-step never straddles a tap
__device__ __forceinline__ void ktap(const ConvArgs& a, int k0, int& tap, int& c0) {
  const int taps = a.KH * a.KW;
  if (a.kcm) {  // K = (cin / 64, kh, kw, cin % 64)
    const int chunk = k0 / (64 * taps);
    const int kk = k0 - chunk * 64 * taps;
    tap = tap_order(a, kk >> 6);
    c0 = chunk * 64 + (kk & 63);
  } else {
    tap = k0 / a.Cin;
    c0 = k0 - tap * a.Cin;
    tap = tap_order(a, tap);
  }
}
// weight column (the stored K order) of the K-step starting at k0 of the kernel's K loop
__device__ __forceinline__ int wcol(const ConvArgs& a, int k0) {
  if (a.x2 && k0 >= a.K1) return k0;  // folded downsample columns
  const int taps = a.KH * a.KW;
  if (taps == 1) return k0;
  int tap, c0;
  ktap(a, k0, tap, c0);
  return a.kcm ? (c0 >> 6) * 64 * taps + tap * 64 + (c0 & 63) : tap * a.Cin + c0;
}

#ifndef EOSV_BF16_STAG
#define EOSV_BF16_STAG 1
#endif

// BK: K per ring slot, 64 (128-B rows) or 32 (64-B rows: half the bytes per slot, so a 4-deep
// ring -- three K-steps in flight -- fits where the 64-deep slots allowed two).
// NSA > 0: separate rings, NSA slots for A (the im2col rows, loaded two K-steps ahead) and NS for
// B (the weights, one K-step ahead; every workgroup reads the same weights, so they come from L2)
template <int BM, int BN, int WM, int WN, bool STEM, int MF, int NS, bool DS, bool SPLIT = false, int BK = 64,
          int NSA = 0>
__global__ __launch_bounds__(64 * WM * WN) void conv_bf16_kernel(ConvArgs a) {
  static_assert(BK == 64 || (BK == 32 && !STEM && MF == 16), "BK 32: 16x16x32 MFMAs, no stem");
  constexpr int CPR = BK / 8;    // 16-B chunks per LDS row
  constexpr int RPP = 64 / CPR;  // rows per 1-KiB DMA piece (one wave-instruction)
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / MF;
  constexpr int TN = BN / WN / MF;
  constexpr int ACC = MF * MF / 64;  // f32 accumulator elements per lane per tile
  constexpr int AI = BM / (RPP * NW);
  constexpr int BI = BN / (RPP * NW);
  constexpr int STAGE = (BM + BN) * BK;  // bf16 elements per ring slot
  static_assert(AI >= 1 && BI >= 1 && TM >= 1 && TN >= 1, "tile shape");
  static_assert(NS >= 2 && NS <= 5, "ring depth");
  static_assert(NSA == 0 || (NSA == 3 && NS == 2 && !STEM), "split rings: 3 A slots, 2 B slots");
  constexpr int SMEM = NSA ? NSA * BM * BK + NS * BN * BK : NS * STAGE;
  __shared__ __attribute__((aligned(16))) u16 smem[SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int HoWo = a.Ho * a.Wo;
  const int M = a.N * HoWo;
  const int nN = (a.Cout + BN - 1) / BN;
  const int bt = xcd_tile(blockIdx.x, gridDim.x, a.xcd);
  if (EOSV_ABL(a) & 512) return;  // profiling-only: dispatch cost alone
  const int mt = bt / nN;
  const int nt = bt - mt * nN;
  const int m0 = mt * BM, n0 = nt * BN;
  const u16* __restrict__ x = (const u16*)a.x;
  const u16* __restrict__ w = (const u16*)a.w;
  const u16* zero = (const u16*)a.zero;

  const int lr = lane / CPR;
  const int pc = lane & (CPR - 1);
  const int xrow = ((a.W + 2 * a.pad + 1) & ~1) * 3;  // STEM: elements per padded input row
  const u16* arow[AI];
  const u16* arow2[DS ? AI : 1];  // DS: the fused downsample's input pixel (always in bounds)
  int aih[AI], aiw[AI], alc[AI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int row = wid * (BM / NW) + RPP * j + lr;
    const int lc = pc ^ ((row >> 1) & (CPR - 1));
    alc[j] = lc;
    const int m = m0 + row;
    if (m < M) {
      const int img = m / HoWo;
      const int rem = m - img * HoWo;
      const int oh = rem / a.Wo;
      const int ow = rem - oh * a.Wo;
      aih[j] = oh * a.stride - a.pad;
      aiw[j] = ow * a.stride - a.pad;
      if constexpr (STEM) {
        // padded coordinates of tap (0, 0) are (oh*stride, ow*stride)
        arow[j] = x + ((long long)img * (a.H + 2 * a.pad) + oh * a.stride) * xrow + (long long)ow * a.stride * 3;
      } else {
        arow[j] = x + (((long long)img * a.H + aih[j]) * a.W + aiw[j]) * a.xs + lc * 8;
        if constexpr (DS)
          arow2[j] = (const u16*)a.x2 +
                     (((long long)img * a.H2 + oh * a.stride2) * a.W2 + ow * a.stride2) * a.x2s + lc * 8;
      }
    } else {
      aih[j] = -(1 << 28);
      aiw[j] = 0;
      arow[j] = x;
      if constexpr (DS) arow2[j] = nullptr;
    }
  }
  const u16* brow[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int row = wid * (BN / NW) + RPP * j + lr;
    const int lc = pc ^ ((row >> 1) & (CPR - 1));
    const int n = n0 + row;
    brow[j] = n < a.Cout ? w + (long long)n * a.K + lc * 8 : nullptr;
  }

  // A into A slot aslot, B into B slot bslot (one ring: both the same slot); skip 4: no A, 8: no B
  auto stage = [&](int k0, int aslot, int bslot, int skip) {
    u16* As = NSA ? smem + aslot * BM * BK : smem + aslot * STAGE;
    u16* Bs = NSA ? smem + NSA * BM * BK + bslot * BN * BK : smem + bslot * STAGE + BM * BK;
    if (skip & 4) {
    } else if (DS && k0 >= a.K1) {
#pragma unroll
      for (int j = 0; j < (DS ? AI : 1); ++j) {
        const u16* src = arow2[j] ? arow2[j] + (SPLIT ? split_chan(k0 - a.K1, a.Cin2) : k0 - a.K1) : zero;
        u16* dst = As + (wid * (BM / NW) + RPP * j) * BK;
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      }
    } else if constexpr (STEM) {
#pragma unroll
      for (int j = 0; j < AI; ++j) {
        const int g = (k0 >> 3) + alc[j];
        const int kh = g / 3;
        const bool ok = aih[j] > -(1 << 27) && kh < a.KH;
        const u16* src = ok ? arow[j] + kh * xrow + (g - 3 * kh) * 8 : zero;
        u16* dst = As + (wid * (BM / NW) + RPP * j) * BK;
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      }
    } else {
      int tap, c0;
      ktap(a, k0, tap, c0);
      const int kh = tap / a.KW;
      const int kw = tap - kh * a.KW;
      const long long toff = ((long long)kh * a.W + kw) * a.xs + (SPLIT ? split_chan(c0, a.Cin) : c0);
#pragma unroll
      for (int j = 0; j < AI; ++j) {
        const int ih = aih[j] + kh, iw = aiw[j] + kw;
        const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const u16* src = ok ? arow[j] + toff : zero;
        u16* dst = As + (wid * (BM / NW) + RPP * j) * BK;
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      }
    }
    if (skip & 8) return;
    const int kb = STEM ? k0 : wcol(a, k0);
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const u16* src = brow[j] ? brow[j] + kb : zero;
      u16* dst = Bs + (wid * (BN / NW) + RPP * j) * BK;
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };

  typedef float accv __attribute__((ext_vector_type(ACC)));
  accv acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < ACC; ++q) acc[i][j][q] = 0.f;

  // fragment lane map: row r = lane % MF, 16-B chunk q = lane / MF of the MFMA's k-slice
  const int r = lane & (MF - 1);
  const int q = lane / MF;
  const int sw = (r >> 1) & (CPR - 1);  // tile bases are multiples of 16 rows: the swizzle depends on r only
  const int nk = (EOSV_ABL(a) & 1024) ? 0 : a.K / BK;  // 1024 (profiling-only): no K-loop
  // NS-deep ring: NS-1 stages in flight; the wait before each barrier is a counted vmcnt (the
  // newer stages stay in flight across it) and barriers are raw s_barrier (__syncthreads would
  // drain them with vmcnt(0)).  wait_stages(n): all but the wave's n newest stages have landed.
  constexpr int PER = AI + BI;  // DMA instructions per stage per wave
  auto wait_stages = [&](int n) {
    if (NS >= 5 && n >= 3)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(3 * PER) : "memory");
    else if (NS >= 4 && n >= 2)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * PER) : "memory");
    else if (NS >= 3 && n >= 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PER) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  if constexpr (NSA > 0) {  // B(0), A(0), A(1); A(1) may stay in flight
    if (nk > 0) {
      stage(0, 0, 0, 4);
      stage(0, 0, 0, 8);
    }
    if (nk > 1) {
      stage(BK, 1, 0, 8);
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(AI) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else {
    for (int p = 0; p < NS - 1 && p < nk; ++p) stage(p * BK, p, p, 0);
    wait_stages(min(NS - 2, nk - 1));
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");  // s_barrier is no compiler-level memory barrier
  int cur = 0, wslot = NS - 1;
  // The two waves of a SIMD are w and w + NW/2.  EOSV_BF16_STAG bit 0 (default): the upper half
  // issues its DMA in the middle of the K-step (after half of its MFMA groups) instead of at its
  // start, so that each SIMD pairs one wave's DMA issue with the other's MFMAs (r03, R50 bf16 per
  // 3200 frames: 3x3 convs 4-7 % faster, 1x1s unchanged, the 1x1 + folded-downsample convs 6-8 %
  // slower, so those keep the plain order unless bit 2); bit 1 (profiling build only): s_setprio 1
  // for the upper half (measured slower).
  const bool late = (EOSV_BF16_STAG & 1) && MF == 16 && (!DS || a.KH > 1 || (EOSV_BF16_STAG & 4)) && wid >= NW / 2;
#ifdef EOSV_PROFILING
  if ((EOSV_BF16_STAG & 2) && wid >= NW / 2) __builtin_amdgcn_s_setprio(1);
#endif
  // the K-step's DMA: one ring: stage kt + NS - 1 into slot wslot; split rings: B(kt + 1) then
  // A(kt + 2) (in this order: the end-of-step wait leaves only A(kt + 2) in flight)
  auto issue_step = [&](int kt) {
    if (EOSV_ABL(a) & 1) return;
    if constexpr (NSA > 0) {
      if (kt + 1 < nk) stage((kt + 1) * BK, 0, (kt + 1) & 1, 4 | EOSV_ABL(a));
      if (kt + 2 < nk) stage((kt + 2) * BK, (kt + 2) % NSA, 0, 8 | EOSV_ABL(a));
    } else if (kt + NS - 1 < nk) {
      stage((kt + NS - 1) * BK, wslot, wslot, EOSV_ABL(a));
    }
  };
  for (int kt = 0; kt < nk; ++kt) {
    // EOSV_ABL(a) (profiling-only ablations, results wrong when set): 1 no main-loop loads,
    // 4 no A loads, 8 no B loads, 16 no ds_reads, 32 no MFMAs, 64 no epilogue
    if (!late) issue_step(kt);
    const u16* As = NSA ? smem + (kt % (NSA ? NSA : 1)) * BM * BK : smem + cur * STAGE;
    const u16* Bs = NSA ? smem + NSA * BM * BK + (kt & 1) * BN * BK : As + BM * BK;
    constexpr int KS = MF == 32 ? 16 : 32;  // k per MFMA
    if constexpr (MF == 16) {
      if (!(EOSV_ABL(a) & (16 | 32))) {
        // Software-pipelined fragment reads (r03): the K-step's MFMAs go in groups (slice s, A row
        // tile i) of TN MFMAs; the next group's A fragment (and at a slice boundary the next
        // slice's TN B fragments) are read from LDS while this group's MFMAs run, instead of
        // waiting lgkmcnt(0) on fresh reads before every group (SQ_WAIT_INST_ANY 0.36 on the
        // 256x256 tile, r02z).  Same MFMAs in the same per-accumulator order: bit-identical.
        constexpr int NSL = BK / KS, NG = NSL * TM;
        bf16x8 bfr[2][TN], afr[2];
        auto rdA = [&](int g) {
          const int s = g / TM, i = g - (g / TM) * TM;
          return *(const bf16x8*)(As + (wm * (BM / WM) + i * MF + r) * BK + ((s * (KS / 8) + q) ^ sw) * 8);
        };
        auto rdB = [&](int s, bf16x8* f) {
#pragma unroll
          for (int j = 0; j < TN; ++j)
            f[j] = *(const bf16x8*)(Bs + (wn * (BN / WN) + j * MF + r) * BK + ((s * (KS / 8) + q) ^ sw) * 8);
        };
        rdB(0, bfr[0]);
        afr[0] = rdA(0);
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          const int s = g / TM, i = g - (g / TM) * TM;
          int nrd = 0;
          if (g + 1 < NG) {
            if ((g + 1) % TM == 0) {
              rdB((g + 1) / TM, bfr[((g + 1) / TM) & 1]);
              nrd += TN;
            }
            afr[(g + 1) & 1] = rdA(g + 1);
            nrd += 1;
          }
          // order: this group's first MFMA (hipcc's lgkmcnt wait for this group's fragments goes
          // before it), then the next group's reads, then the other MFMAs: the reads are not
          // covered by that wait and overlap this group's MFMAs
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if (nrd == TN + 1) __builtin_amdgcn_sched_group_barrier(0x100, TN + 1, 0);
          if (nrd == 1) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, TN - 1, 0);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[g & 1], bfr[s & 1][j], acc[i][j], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          if (late && g == NG / 2 - 1) {
            issue_step(kt);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
    } else
#pragma unroll
    for (int s = 0; s < BK / KS; ++s) {
      const int pch = ((s * (KS / 8) + q) ^ sw) * 8;
      bf16x8 af[TM], bf[TN];
      if (EOSV_ABL(a) & 16) {  // profiling-only: no ds_reads (operands stay whatever the registers hold)
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = bf16x8{};
#pragma unroll
        for (int j = 0; j < TN; ++j) bf[j] = bf16x8{};
      } else {
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = *(const bf16x8*)(As + (wm * (BM / WM) + i * MF + r) * BK + pch);
#pragma unroll
        for (int j = 0; j < TN; ++j) bf[j] = *(const bf16x8*)(Bs + (wn * (BN / WN) + j * MF + r) * BK + pch);
      }
      if (EOSV_ABL(a) & 32) {  // profiling-only: no MFMAs
        asm volatile("" ::"v"(af[0]), "v"(bf[0]));
        continue;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (MF == 32)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
    }
    // stage kt + 1 must have landed; the ones issued after it (up to kt + NS - 1) may fly on
    // (split rings: A(kt + 2), when issued)
    if constexpr (NSA > 0) {
      if (kt + 2 < nk)
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(AI) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      wait_stages(min(NS - 2, nk - 2 - kt));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    cur = cur + 1 == NS ? 0 : cur + 1;
    wslot = wslot + 1 == NS ? 0 : wslot + 1;
  }

  if (EOSV_ABL(a) & 64) {  // profiling-only: no epilogue
    asm volatile("" ::"v"(acc[0][0][0]));
    return;
  }
  // The last K-step's vmcnt(0) is inline asm, invisible to the compiler: tell it, or it waits
  // again (for the residual loads too) before the first LDS write below.
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  u16* __restrict__ y = (u16*)a.y;
  const u16* __restrict__ res = (const u16*)a.res;
  // Epilogue staged through LDS (the ring is free now): pass i moves the i-th 32-row
  // M-subtile of every wave (WM*32 rows x BN cols, f32, rows padded by 4) so that the
  // residual loads and output stores are 16 B (8 bf16) per lane, whole 128-B lines.
  // Output and residual go through buffer resources based at the tile's first row: rows past
  // M lie beyond num_records and columns past Cout get an out-of-range offset, so such loads
  // return 0 and such stores are dropped, without a branch.  Straight-line code lets the
  // compiler count vmcnt exactly; the former per-chunk `if (m < M)` form made it wait
  // vmcnt(0) -- for every earlier store -- before each residual use (r01g: the epilogue was
  // 5-25 % of a layer).
  constexpr int EPR = WM * 32;   // rows per pass
  constexpr int EPS = BN + 4;    // f32 row stride
  static_assert(EPR * EPS * 4 <= SMEM * 2, "epilogue tile must fit the ring");
  float* ep = (float*)smem;
  float bcol[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / WN) + j * MF + r;
    bcol[j] = (a.bias && n < a.Cout) ? a.bias[n] : 0.f;
  }
  const int nthreads = 64 * NW;
  constexpr int TPP = 32 / MF;                      // MFMA row-tiles per 32-row pass
  constexpr int NPASS = BM / WM / 32;
  constexpr int IPT = EPR * (BN / 8) / (64 * NW);   // 16-B output chunks per thread per pass
  static_assert(IPT * 64 * NW == EPR * (BN / 8), "epilogue work divides evenly");
  const long long ostr = SPLIT ? 2LL * a.Cout : a.Cout;  // output / residual pixel stride
  const long long tile_bytes = (long long)min(BM, M - m0) * ostr * 2;
  const int nrec = (int)min(tile_bytes, 0x7fffffffLL);
  const __amdgpu_buffer_rsrc_t yr =
      __builtin_amdgcn_make_buffer_rsrc((void*)(y + (long long)m0 * ostr), (short)0, nrec, 0x00020000);
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(res ? res + (long long)m0 * ostr : (const u16*)a.zero), (short)0, res ? nrec : 0, 0x00020000);
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  // v4u rv[2][IPT]: residual chunks of pass i, loaded one pass ahead (pass 0's right after the
  // K-loop) so that their latency overlaps the LDS staging instead of stalling each store
  v4u rv[2][IPT];
  v4u rl[2][SPLIT ? IPT : 1];  // SPLIT: the residual's lo block
  auto chunk = [&](int i, int t, int& lrow, int& c8, int& voff) {
    const int idx = tid + t * nthreads;
    lrow = idx / (BN / 8);
    c8 = idx - lrow * (BN / 8);
    const int ml = (lrow >> 5) * (BM / WM) + i * 32 + (lrow & 31);  // row within the tile
    const int n = n0 + c8 * 8;
    voff = n < a.Cout ? (int)(((long long)ml * ostr + n) * 2) : (int)0x80000000;
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
  // unconditional (no residual: rr has num_records 0, the loads return 0) and branch-free below
  load_res(0);
  const float rlow = a.relu ? 0.f : -INFINITY;  // ReLU as max(v, rlow)
#pragma unroll
  for (int i = 0; i < NPASS; ++i) {
    if (i + 1 < NPASS) load_res(i + 1);
    // raw barriers in the epilogue: only the LDS staging needs ordering, and a
    // __syncthreads() fence would also wait for the residual prefetch and the stores
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int t = 0; t < TPP; ++t)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < ACC; ++e) {
          // C/D maps: 32x32 row = (e&3) + 8(e>>2) + 4(lane>>5); 16x16 row = 4(lane>>4) + e
          const int crow = MF == 32 ? (e & 3) + 8 * (e >> 2) + 4 * q : 4 * q + e;
          const int lrow = wm * 32 + t * MF + crow;
          ep[lrow * EPS + wn * (BN / WN) + j * MF + r] = acc[i * TPP + t][j][e] + bcol[j];
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
      {
        const v4u r4 = rv[i & 1][t];
        const unsigned ru[4] = {r4.x, r4.y, r4.z, r4.w};
        if constexpr (SPLIT) {
          const v4u l4 = rl[i & 1][SPLIT ? t : 0];
          const unsigned rlo[4] = {l4.x, l4.y, l4.z, l4.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {  // hi + lo is exact in f32
            v[2 * k] += bf_to_f((u16)(ru[k] & 0xffff)) + bf_to_f((u16)(rlo[k] & 0xffff));
            v[2 * k + 1] += bf_to_f((u16)(ru[k] >> 16)) + bf_to_f((u16)(rlo[k] >> 16));
          }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            v[2 * k] += bf_to_f((u16)(ru[k] & 0xffff));
            v[2 * k + 1] += bf_to_f((u16)(ru[k] >> 16));
          }
        }
      }
      v4u pk, pl;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float lo = fmaxf(v[2 * k], rlow), hi = fmaxf(v[2 * k + 1], rlow);
        const u16 blo = f_to_bf(lo), bhi = f_to_bf(hi);
        pk[k] = (unsigned)blo | ((unsigned)bhi << 16);
        if constexpr (SPLIT)  // residual parts (exact differences)
          pl[k] = (unsigned)f_to_bf(lo - bf_to_f(blo)) | ((unsigned)f_to_bf(hi - bf_to_f(bhi)) << 16);
      }
      __builtin_amdgcn_raw_buffer_store_b128(pk, yr, voff, 0, 0);
      if constexpr (SPLIT) __builtin_amdgcn_raw_buffer_store_b128(pl, yr, voff + 2 * a.Cout, 0, 0);
    }
  }
}

// Warp-specialised 256x256 tile (r04, EOSV_BF16_WS): NW = WM x WN consumer waves that only read
// LDS fragments and issue MFMAs, plus NP producer waves that only stage the A (im2col) and B rows
// by LDS-DMA, so no consumer wave ever issues a DMA piece (60-185 cycles of the issuing wave each,
// MI355X_MICROARCH.md) or waits on vmcnt.  Same 2-slot ring, same K order, same MFMAs in the same
// per-accumulator order and the same epilogue as conv_bf16_kernel: bit-identical outputs.
// One barrier per K-step serves both directions: the producers' stage kt + 1 (into the slot
// consumed in step kt - 1) has landed (their vmcnt(0) before it), and the consumers are done with
// slot kt.  12 waves = 3 per SIMD: every wave gets <= 168 VGPRs, so the consumers keep one set of
// B fragments (the 256x256 kernel's double-buffered B set alone is 32 VGPRs more).  Producers
// leave after the K loop (s_barrier then waits only for the surviving consumer waves).
// NSA = 3: split rings as conv_bf16_kernel's NSA: 3 A slots (the im2col rows, staged two K-steps
// ahead) and 2 B slots (the weights, one ahead), 160 KiB (256x256 tiles; r04 A/B on the stride-1
// 3x3s: one ring 6-7 %, split rings 13 % faster than conv_bf16_kernel's one ring).  DS / SPLIT as in
// conv_bf16_kernel (the folded downsample's K columns; the f32x3 split layout).
#ifndef EOSV_BF16_WS_BEARLY
#define EOSV_BF16_WS_BEARLY 1
#endif
template <int BM, int BN, int WM, int WN, int NP, int NSA, bool DS, bool SPLIT>
__global__ __launch_bounds__(64 * (WM * WN + NP)) void conv_bf16_ws_kernel(ConvArgs a) {
  constexpr int BK = 64, CPR = 8, RPP = 8, MF = 16, KS = 32;
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / MF, TN = BN / WN / MF;
  constexpr int AI = BM / (RPP * NP), BI = BN / (RPP * NP);  // DMA pieces per producer wave per stage
  constexpr int STAGE = (BM + BN) * BK;
  static_assert(AI >= 1 && BI >= 1, "tile shape");
  static_assert(NSA == 0 || NSA == 3, "one ring, or 3 A + 2 B slots");
  constexpr int SMEM = NSA ? NSA * BM * BK + 2 * BN * BK : 2 * STAGE;
  __shared__ __attribute__((aligned(16))) u16 smem[SMEM];
  // A slot of K-step kt, B slot of K-step kt
  auto a_slot = [&](int kt) { return NSA ? smem + (kt % (NSA ? NSA : 1)) * BM * BK : smem + (kt & 1) * STAGE; };
  auto b_slot = [&](int kt) { return NSA ? smem + NSA * BM * BK + (kt & 1) * BN * BK : smem + (kt & 1) * STAGE + BM * BK; };

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
  const int nk = (EOSV_ABL(a) & 1024) ? 0 : a.K / BK;

  if (wid >= NW) {  // ---------------------------------------------------------------- producer
    const int pw = wid - NW;
    const u16* __restrict__ x = (const u16*)a.x;
    const u16* __restrict__ w = (const u16*)a.w;
    const u16* zero = (const u16*)a.zero;
    const int lr = lane / CPR, pc = lane & (CPR - 1);
    const u16* arow[AI];
    const u16* arow2[DS ? AI : 1];  // DS: the fused downsample's input pixel (always in bounds)
    int aih[AI], aiw[AI];
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int row = pw * (BM / NP) + RPP * j + lr;
      const int lc = pc ^ ((row >> 1) & (CPR - 1));
      const int m = m0 + row;
      if (m < M) {
        const int img = m / HoWo, rem = m - img * HoWo, oh = rem / a.Wo, ow = rem - oh * a.Wo;
        aih[j] = oh * a.stride - a.pad;
        aiw[j] = ow * a.stride - a.pad;
        arow[j] = x + (((long long)img * a.H + aih[j]) * a.W + aiw[j]) * a.xs + lc * 8;
        if constexpr (DS)
          arow2[j] = (const u16*)a.x2 + (((long long)img * a.H2 + oh * a.stride2) * a.W2 + ow * a.stride2) * a.x2s + lc * 8;
      } else {
        aih[j] = -(1 << 28);
        aiw[j] = 0;
        arow[j] = x;
        if constexpr (DS) arow2[j] = nullptr;
      }
    }
    const u16* brow[BI];
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const int row = pw * (BN / NP) + RPP * j + lr;
      const int lc = pc ^ ((row >> 1) & (CPR - 1));
      const int n = n0 + row;
      brow[j] = n < a.Cout ? w + (long long)n * a.K + lc * 8 : nullptr;
    }
    // skip 4: no A rows, 8: no B rows
    auto stage = [&](int kt, int skip) {
      const int k0 = kt * BK;
      u16* As = a_slot(kt);
      u16* Bs = b_slot(kt);
      if (skip & 4) {
      } else if (DS && k0 >= a.K1) {
#pragma unroll
        for (int j = 0; j < (DS ? AI : 1); ++j) {
          const u16* src = arow2[j] ? arow2[j] + (SPLIT ? split_chan(k0 - a.K1, a.Cin2) : k0 - a.K1) : zero;
          u16* dst = As + (pw * (BM / NP) + RPP * j) * BK;
          __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
        }
      } else {
        int tap, c0;
        ktap(a, k0, tap, c0);
        const int kh = tap / a.KW, kw = tap - (tap / a.KW) * a.KW;
        const long long toff = ((long long)kh * a.W + kw) * a.xs + (SPLIT ? split_chan(c0, a.Cin) : c0);
#pragma unroll
        for (int j = 0; j < AI; ++j) {
          const int ih = aih[j] + kh, iw = aiw[j] + kw;
          const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
          const u16* src = ok ? arow[j] + toff : zero;
          u16* dst = As + (pw * (BM / NP) + RPP * j) * BK;
          __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
        }
      }
      if (skip & 8) return;
      const int kb = wcol(a, k0);
#pragma unroll
      for (int j = 0; j < BI; ++j) {
        const u16* src = brow[j] ? brow[j] + kb : zero;
        u16* dst = Bs + (pw * (BN / NP) + RPP * j) * BK;
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      }
    };
    if constexpr (NSA) {  // B(0), A(0), then A(1) may stay in flight
      if (nk > 0) stage(0, 0);
      if (nk > 1) {
        stage(1, 8);
        vm_wait<AI>();
      } else {
        vm_wait<0>();
      }
    } else {
      if (nk > 0) stage(0, 0);
      vm_wait<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int kt = 0; kt < nk; ++kt) {
      if constexpr (NSA) {  // B(kt + 1), then A(kt + 2); B(kt + 1) and A(kt + 1) must land, A(kt + 2) may fly
        if (!(EOSV_ABL(a) & 1)) {
          if (kt + 1 < nk) stage(kt + 1, 4);
          if (kt + 2 < nk) stage(kt + 2, 8);
        }
        if (kt + 2 < nk)
          vm_wait<AI>();
        else
          vm_wait<0>();
      } else {
        if (kt + 1 < nk && !(EOSV_ABL(a) & 1)) stage(kt + 1, 0);
        vm_wait<0>();
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");  // no next-step DMA (an LDS write) moves above the barrier
    }
    return;
  }

  // ------------------------------------------------------------------------------------ consumer
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  typedef float accv __attribute__((ext_vector_type(4)));
  accv acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = accv{0.f, 0.f, 0.f, 0.f};
  const int r = lane & (MF - 1);
  const int q = lane / MF;
  const int sw = (r >> 1) & (CPR - 1);
  __builtin_amdgcn_s_barrier();  // stage 0 has landed
  asm volatile("" ::: "memory");
  for (int kt = 0; kt < nk; ++kt) {
    const u16* As = a_slot(kt);
    const u16* Bs = b_slot(kt);
    if (!(EOSV_ABL(a) & (16 | 32))) {
      // groups (slice s, A row tile i) of TN MFMAs; the next group's A fragment is read while this
      // group's MFMAs run, the slice's B fragments at its first group
      constexpr int NSL = BK / KS, NG = NSL * TM;
      bf16x8 bfr[TN], afr[2];
      auto rdA = [&](int g) {
        const int s = g / TM, i = g - (g / TM) * TM;
        return *(const bf16x8*)(As + (wm * (BM / WM) + i * MF + r) * BK + ((s * (KS / 8) + q) ^ sw) * 8);
      };
      auto rdB = [&](int s) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[j] = *(const bf16x8*)(Bs + (wn * (BN / WN) + j * MF + r) * BK + ((s * (KS / 8) + q) ^ sw) * 8);
      };
      rdB(0);
      afr[0] = rdA(0);
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int i = g - (g / TM) * TM;
        if constexpr (EOSV_BF16_WS_BEARLY) {
          if (g % TM == TM - 1 && g + 1 < NG) {
            // a slice's last group: B fragment j of the next slice is read right behind the MFMA
            // that last uses fragment j of this slice (the slice-boundary read then has three
            // MFMAs of lead instead of none)
            afr[(g + 1) & 1] = rdA(g + 1);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[g & 1], bfr[j], acc[i][j], 0, 0, 0);
              const int s1 = g / TM + 1;
              bfr[j] = *(const bf16x8*)(Bs + (wn * (BN / WN) + j * MF + r) * BK + ((s1 * (KS / 8) + q) ^ sw) * 8);
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
              __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            continue;
          }
        }
        if (!EOSV_BF16_WS_BEARLY && g > 0 && g % TM == 0) rdB(g / TM);  // slice boundary: this slice's B (not overlapped)
        if (g + 1 < NG) afr[(g + 1) & 1] = rdA(g + 1);
        if constexpr (EOSV_BF16_RFIRST) {  // r06 A/B: the next A fragment's read ahead of all TN MFMAs
          if (g + 1 < NG) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, TN, 0);
        } else {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if (g + 1 < NG) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, TN - 1, 0);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[g & 1], bfr[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  if (EOSV_ABL(a) & 64) {  // profiling-only: no epilogue
    asm volatile("" ::"v"(acc[0][0][0]));
    return;
  }

  // epilogue (the 256x256 kernel's, consumer waves only): staged through the free ring
  u16* __restrict__ y = (u16*)a.y;
  const u16* __restrict__ res = (const u16*)a.res;
  constexpr int EPR = WM * 32, EPS = BN + 4;
  static_assert(EPR * EPS * 4 <= SMEM * 2, "epilogue tile must fit the ring");
  float* ep = (float*)smem;
  float bcol[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / WN) + j * MF + r;
    bcol[j] = (a.bias && n < a.Cout) ? a.bias[n] : 0.f;
  }
  constexpr int nthreads = 64 * NW;
  constexpr int TPP = 32 / MF, NPASS = BM / WM / 32;
  constexpr int IPT = EPR * (BN / 8) / (64 * NW);
  static_assert(IPT * 64 * NW == EPR * (BN / 8), "epilogue work divides evenly");
  const long long ostr = SPLIT ? 2LL * a.Cout : a.Cout;  // output / residual pixel stride
  const long long tile_bytes = (long long)min(BM, M - m0) * ostr * 2;
  const int nrec = (int)min(tile_bytes, 0x7fffffffLL);
  const __amdgpu_buffer_rsrc_t yr =
      __builtin_amdgcn_make_buffer_rsrc((void*)(y + (long long)m0 * ostr), (short)0, nrec, 0x00020000);
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(res ? res + (long long)m0 * ostr : (const u16*)a.zero), (short)0, res ? nrec : 0, 0x00020000);
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  // residual sets: two (pass i + 1's loads in flight during pass i), one with SPLIT (its lo block
  // doubles them: two sets spilled 38 VGPRs; pass i's then load at its start, under the LDS write)
  constexpr int NRB = SPLIT ? 1 : 2;
  v4u rv[NRB][IPT];
  v4u rl[NRB][SPLIT ? IPT : 1];  // SPLIT: the residual's lo block
  auto chunk = [&](int i, int t, int& lrow, int& c8, int& voff) {
    const int idx = tid + t * nthreads;
    lrow = idx / (BN / 8);
    c8 = idx - lrow * (BN / 8);
    const int ml = (lrow >> 5) * (BM / WM) + i * 32 + (lrow & 31);
    const int n = n0 + c8 * 8;
    voff = n < a.Cout ? (int)(((long long)ml * ostr + n) * 2) : (int)0x80000000;
  };
  auto load_res = [&](int i) {
#pragma unroll
    for (int t = 0; t < IPT; ++t) {
      int lrow, c8, voff;
      chunk(i, t, lrow, c8, voff);
      rv[i % NRB][t] = __builtin_amdgcn_raw_buffer_load_b128(rr, voff, 0, 0);
      if constexpr (SPLIT) rl[i % NRB][SPLIT ? t : 0] = __builtin_amdgcn_raw_buffer_load_b128(rr, voff + 2 * a.Cout, 0, 0);
    }
  };
  // the residual of pass i + 1 is loaded once pass i's accumulators are in LDS (their registers
  // are dead by then): with the 168-VGPR budget of 12 waves, holding two residual sets beside all
  // 128 accumulators spilled
  if constexpr (!SPLIT) load_res(0);
  const float rlow = a.relu ? 0.f : -INFINITY;
#pragma unroll
  for (int i = 0; i < NPASS; ++i) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if constexpr (SPLIT) load_res(i);
#pragma unroll
    for (int t = 0; t < TPP; ++t)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int lrow = wm * 32 + t * MF + 4 * q + e;
          ep[lrow * EPS + wn * (BN / WN) + j * MF + r] = acc[i * TPP + t][j][e] + bcol[j];
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (!SPLIT && i + 1 < NPASS) load_res(i + 1);
#pragma unroll
    for (int t = 0; t < IPT; ++t) {
      int lrow, c8, voff;
      chunk(i, t, lrow, c8, voff);
      const float4 v0 = *(const float4*)(ep + lrow * EPS + c8 * 8);
      const float4 v1 = *(const float4*)(ep + lrow * EPS + c8 * 8 + 4);
      float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      const v4u r4 = rv[i % NRB][t];
      const unsigned ru[4] = {r4.x, r4.y, r4.z, r4.w};
      if constexpr (SPLIT) {
        const v4u l4 = rl[i % NRB][SPLIT ? t : 0];
        const unsigned rlo[4] = {l4.x, l4.y, l4.z, l4.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // hi + lo is exact in f32
          v[2 * k] += bf_to_f((u16)(ru[k] & 0xffff)) + bf_to_f((u16)(rlo[k] & 0xffff));
          v[2 * k + 1] += bf_to_f((u16)(ru[k] >> 16)) + bf_to_f((u16)(rlo[k] >> 16));
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[2 * k] += bf_to_f((u16)(ru[k] & 0xffff));
          v[2 * k + 1] += bf_to_f((u16)(ru[k] >> 16));
        }
      }
      v4u pk, pl;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float lo = fmaxf(v[2 * k], rlow), hi = fmaxf(v[2 * k + 1], rlow);
        const u16 blo = f_to_bf(lo), bhi = f_to_bf(hi);
        pk[k] = (unsigned)blo | ((unsigned)bhi << 16);
        if constexpr (SPLIT)  // residual parts (exact differences)
          pl[k] = (unsigned)f_to_bf(lo - bf_to_f(blo)) | ((unsigned)f_to_bf(hi - bf_to_f(bhi)) << 16);
      }
      __builtin_amdgcn_raw_buffer_store_b128(pk, yr, voff, 0, 0);
      if constexpr (SPLIT) __builtin_amdgcn_raw_buffer_store_b128(pl, yr, voff + 2 * a.Cout, 0, 0);
    }
  }
}

// EOSV_BF16_WS bits (bf16 layout only): 1 stride-1 multi-tap convs on 256x256 tiles (split
// rings), 2 the other 256x256 convs (1x1, stride 2, folded downsample; split rings), 4 the 512x128
// tiles (one ring).
#ifndef EOSV_BF16_WS_DEF
#define EOSV_BF16_WS_DEF 7
#endif
static int bf16_ws() {
  static const int v = env_switch("EOSV_BF16_WS", EOSV_BF16_WS_DEF);  // (A/B switch)
  return v;
}

template <int BM, int BN, int WM, int WN, int NSA>
static int launch_bf16_ws(const ConvArgs& a, hipStream_t s) {
  constexpr int NP = 4, NT = 64 * (WM * WN + NP);
  const long long M = (long long)a.N * a.Ho * a.Wo;
  const long long nb = ((M + BM - 1) / BM) * ((a.Cout + BN - 1) / BN);
  if (nb > 0x7fffffffLL) return set_error("conv: grid too large"), EOSV_ERR_UNSUPPORTED;
  if (a.plan) {
    static const int occ = kernel_occupancy((const void*)conv_bf16_ws_kernel<BM, BN, WM, WN, NP, NSA, false, false>, NT);
    return record_launch(a.plan, nb, occ);
  }
  if (a.x2 && (a.K1 % 64 || a.Cin2 % 64)) return set_error("conv_bf16: fused downsample shape"), EOSV_ERR_UNSUPPORTED;
  // f32x3 (split layout) stays on conv_bf16_kernel: its two residual blocks beside the 128
  // accumulators spill 13-18 VGPRs at the 168 of 12 waves
  if (a.split) return set_error("conv_bf16_ws: split layout"), EOSV_ERR_UNSUPPORTED;
  const dim3 g((unsigned)nb), b(NT);
  if (a.x2) {
    hipLaunchKernelGGL((conv_bf16_ws_kernel<BM, BN, WM, WN, NP, NSA, true, false>), g, b, 0, s, a);
  } else {
    hipLaunchKernelGGL((conv_bf16_ws_kernel<BM, BN, WM, WN, NP, NSA, false, false>), g, b, 0, s, a);
  }
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

// 256x256 tiles with split rings (3 A slots, 2 B slots: A two K-steps ahead), all of the LDS:
// 1 (default) for the convs that gain (below), 2 for every 256x256 conv, 0 never.  (Rejected in r03
// and removed from the source: 32-deep K-steps in 4/5-slot rings, 12-20 % slower on every 3x3; the
// Cout-128 stride-2 convs on 256x128 split-ring tiles, 10-17 % slower)
#ifndef EOSV_BF16_ARING
#define EOSV_BF16_ARING 1
#endif

#ifndef EOSV_BF16_ROWSR_DEF
#define EOSV_BF16_ROWSR_DEF 2
#endif

static int bf16_rows() {
  static int v = env_switch("EOSV_BF16_ROWS", 1);  // 0 = stage-1 3x3 convs on the implicit GEMM (A/B switch)
  return v;
}

template <int BM, int BN, int WM, int WN, bool STEM, int NS = 2, int BK = 64, int NSA = 0>
static int launch_bf16(const ConvArgs& a, hipStream_t s) {
  const long long M = (long long)a.N * a.Ho * a.Wo;
  const long long nb = ((M + BM - 1) / BM) * ((a.Cout + BN - 1) / BN);
  if (nb > 0x7fffffffLL) return set_error("conv: grid too large"), EOSV_ERR_UNSUPPORTED;
  if (a.plan) {
    static const int occ =
        kernel_occupancy((const void*)conv_bf16_kernel<BM, BN, WM, WN, false, 16, NS, false, false, BK, NSA>, 64 * WM * WN);
    return record_launch(a.plan, nb, occ);
  }
  if (a.split) {
    if (STEM || (a.x2 && (a.K1 % 64 || a.Cin2 % 64)))
      return set_error("conv_bf16: split layout shape"), EOSV_ERR_UNSUPPORTED;
    if (a.x2)
      hipLaunchKernelGGL((conv_bf16_kernel<BM, BN, WM, WN, false, 16, NS, true, true, BK, NSA>), dim3((unsigned)nb),
                         dim3(64 * WM * WN), 0, s, a);
    else
      hipLaunchKernelGGL((conv_bf16_kernel<BM, BN, WM, WN, false, 16, NS, false, true, BK, NSA>), dim3((unsigned)nb),
                         dim3(64 * WM * WN), 0, s, a);
  } else if (a.x2) {
    if (STEM || a.K1 % 64 || a.Cin2 % 64) return set_error("conv_bf16: fused downsample shape"), EOSV_ERR_UNSUPPORTED;
    hipLaunchKernelGGL((conv_bf16_kernel<BM, BN, WM, WN, false, 16, NS, true, false, BK, NSA>), dim3((unsigned)nb),
                       dim3(64 * WM * WN), 0, s, a);
  } else {
    hipLaunchKernelGGL((conv_bf16_kernel<BM, BN, WM, WN, STEM, 16, NS, false, false, BK, NSA>), dim3((unsigned)nb),
                       dim3(64 * WM * WN), 0, s, a);
  }
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int launch_conv_bf16(const ConvArgs& a0, hipStream_t s) {
  static const int abl = env_switch("EOSV_CONV_ABL", 0);  // profiling-only ablations; results are wrong when set
  ConvArgs a = a0;
  a.abl = abl;
  conv_pixel_strides(a);
  const bool stem = (a.Cin == 3);
  if (!a.zero || a.K % 64 != 0 || (!stem && a.Cin % 64 != 0) ||
      (stem && (a.KWp != 8 || a.KW != 7 || a.stride % 2 != 0 || a.K != (a.KH * 24 + 63) / 64 * 64))) {
    set_error("conv_bf16: unsupported shape (K % 64, Cin % 64, or stem layout)");
    return EOSV_ERR_UNSUPPORTED;
  }
  if (stem) return launch_bf16<128, 64, 2, 2, true>(a, s);
  if (bf16_rows() && !a.x2 && !a.split) {
    // r05: the weights in registers, three strip buffers (conv_rowsr_bf16.hip).  A/B (r05f, ms per
    // ~3122-frame launch): C 64 at 64x64 (R101 at 256: the 128x64 implicit GEMM before) 1.57-1.63
    // -> 0.92-0.98; C 64 at 56x56 0.69 / 0.85 (residual) -> 0.97 / 1.59 against conv_rows_bf16, C 128
    // at 28x28 / 32x32 0.71-0.78 -> 1.07-1.27 against the tap-shift tile: one wave per SIMD leaves
    // the LDS-DMA issue and fragment-read latency exposed.  2 (default): only C 64 at 64x64; 1: every
    // rowsr shape; 0: none (A/B switch)
    static const int rowsr = env_switch("EOSV_BF16_ROWSR", EOSV_BF16_ROWSR_DEF);
    if (rowsr && conv_rowsr_bf16_ok(a) && (rowsr == 1 || (a.Cin == 64 && a.W == 64))) return launch_conv_rowsr_bf16(a, s);
    if (conv_rows_bf16_ok(a)) return launch_conv_rows_bf16(a, s);
  }
  // R18 stage-2 entry (3x3/2 64 -> 128 at 56x56): row strips with the weights in registers (r05)
  static const int s2rows = env_switch("EOSV_BF16_S2ROWS", 1);  // 0 = the 512x128 implicit GEMM (A/B switch)
  if (s2rows && conv_s2rows_bf16_ok(a)) return launch_conv_s2rows_bf16(a, s);
  static const int x3rows = env_switch("EOSV_X3_ROWS", 1);  // 0 = f32x3 stage-1 3x3 convs on the tap-shift kernel (A/B switch)
  if (x3rows && conv_rows_x3_ok(a)) return launch_conv_rows_x3(a, s);
  // tap-shift kernel (conv_bf16_ts.hip) for the stride-1 3x3 convs with Cout = 128 (r01g A/B: 5-6 %
  // faster) and the f32x3 Cout = 64 convs (512x64: 10-12 % faster than 256x64); at Cout >= 256
  // its 64-B rows lost 2-8 % to the 256x256 im2col tile
  static const int ts = env_switch("EOSV_BF16_TS", 1);  // 0 never, 1 default shapes, 2 every eligible shape (A/B switch)
  if (ts && conv_bf16_ts_ok(a) && (ts == 2 || a.Cout == 128 || (a.Cout == 64 && a.split)))
    return launch_conv_bf16_ts(a, s);
  // r01 A/B: 256x128 tiles for Cout 128 and 128x128 / 128x256 tiles for the
  // K = 64 1x1 convs all measured slower than this choice.
  // f32x3 (K tripled): 256x64 tiles for the Cout-64 convs, +7 % over 128x64 (tools/ab_x3.sh)
  if (a.split && a.Cout <= 64) return launch_bf16<256, 64, 4, 1, false>(a, s);
  // Cout 128 (ResNet stage 2, R50 bottleneck 1x1s, stride-2 entries and the fused downsample):
  // 512x128 tiles (160 KiB, 8 waves of 128x64), the one-barrier-per-K-step loop of the 256x256
  // tile.  r01 A/B (tools/ab_sets.sh): 12-15 % faster than a phased 8-wave 512x128 kernel (whose 8
  // barriers per K-tile cost more than its overlap gains: SQ MFMA-busy 0.29 vs 0.42) and 5 %
  // faster than 128x128 on the stride-2 entry.
#ifdef EOSV_PROFILING
  // A/B of the Cout-128 tile for the stride-2 entries / 1x1s (not the tap-shift convs):
  // 1 256x128 (8 waves), 2 128x128 (4 waves), 3 256x128 (4 waves); bit 4: f32x3 (split) only
  static const int s2t = env_switch("EOSV_BF16_C128_TILE", 0);
  if (a.Cout == 128 && (s2t & 3) && (!(s2t & 4) || a.split)) {
    if ((s2t & 3) == 1) return launch_bf16<256, 128, 4, 2, false>(a, s);
    if ((s2t & 3) == 2) return launch_bf16<128, 128, 2, 2, false>(a, s);
    return launch_bf16<256, 128, 2, 2, false>(a, s);
  }
#endif
  const int ws = a.split ? 0 : bf16_ws();  // WS classes for this conv
  if (a.Cout == 128) {
    if (ws & 4) return launch_bf16_ws<512, 128, 4, 2, 0>(a, s);
    return launch_bf16<512, 128, 4, 2, false>(a, s);
  }
  if (a.Cout >= 256) {
    const bool s1 = a.KH * a.KW > 1 && a.stride == 1 && !a.x2;  // stride-1 multi-tap: one ring below
    if ((ws & 1) && s1) return launch_bf16_ws<256, 256, 2, 4, 3>(a, s);
    if ((ws & 2) && !s1) return launch_bf16_ws<256, 256, 2, 4, 3>(a, s);
    // split rings (A two K-steps ahead) for the 1x1s, the stride-2 3x3s and the fused-downsample
    // convs; the stride-1 3x3s keep the one ring (r03 A/B, ms per 3200 frames, R50: 1x1s 6-11 %
    // faster, e.g. stage-4 conv1 0.33 -> 0.29, 1x1 + downsample 1.15 -> 1.08, stride-2 3x3 0.67 ->
    // 0.64; stride-1 3x3s 2-4 % slower with them)
    if constexpr (EOSV_BF16_ARING != 0)
      if (EOSV_BF16_ARING == 2 || a.KH * a.KW == 1 || a.stride != 1 || a.x2)
        return launch_bf16<256, 256, 2, 4, false, 2, 64, 3>(a, s);
    return launch_bf16<256, 256, 2, 4, false>(a, s);
  }
  return launch_bf16<128, 64, 2, 2, false>(a, s);
}

}  // namespace eosv
