// Halo-staged 3x3 conv for bf16 (stride 1, pad 1, Cout a multiple of 256) on small maps:
// ResNet stages 3-4 (14x14 / 7x7 maps at 224x224 input, 16x16 / 8x8 at 256x256).
//
// The implicit GEMM (conv_bf16.hip) stages every tap's A rows afresh: per 64-channel chunk of
// a 256x256 tile, 9 x 32 KiB of pixels -- the same pixels nine times -- beside 9 x 32 KiB of
// weights, and at one workgroup per CU that staging rate (~30 GB/s per CU) is what bounds it
// (DESIGN.md section 8).  Here the tile stages, per 32-channel chunk, the padded input rows
// its 256 output pixels touch (the halo: at most 512 slots of 64 B) once, and the 9 taps read
// their A fragments from it; only the weights (16 KiB per tap and chunk) move per K-step.
// Staged bytes per 64 channels and tile: <= 64 + 288 KiB instead of 288 + 288.
//
// K order (32-channel chunk, tap) over the chunk-major weights (ConvArgs::kcm): the per-
// accumulator sums run chunk by chunk, tap by tap -- the implicit GEMM's order is (64-channel
// chunk, tap, 32-channel half), so results equal it up to f32 summation order.
//
// Halo of the tile starting at output pixel m0: padded row p = img * (H + 2) + iy + 1 (iy = -1
// and iy = H are zero rows), rows from p_lo = (padded row of m0's output row) onward, slot
// s = (p - p_lo) * (W + 2) + ix + 1.  Output pixel (img, oy, ox) and tap (kh, kw) read slot
// (img * (H + 2) + oy - p_lo + kh) * (W + 2) + ox + kw.  LDS rows are 64 B (four 16-B chunks),
// chunk c of slot s stored at position c ^ ((s >> 2) & 3) (XOR applied on the DMA source), so
// the 16 consecutive slots of one MFMA fragment read conflict-free; the weight rows (couts)
// the same way.
//
// LDS (112 KiB, one workgroup per CU): two halo buffers (chunk kc + 1 loads during chunk kc)
// and a 3-slot weight ring (B two K-steps ahead).  At the end of K-step kt, B(kt + 1) -- and
// before a chunk's first tap that chunk's halo, issued 9 K-steps earlier -- must have landed;
// younger than B(kt + 1) are this step's halo (tap 0) and B(kt + 2): counted vmcnt, raw
// barriers.  Epilogue as conv_bf16's: staged through LDS, shift + residual + ReLU, 16-B stores.
#include <hip/hip_bf16.h>

#include "common.h"

#ifndef EOSV_HALO_STAG
#define EOSV_HALO_STAG 0
#endif

namespace eosv {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

constexpr int BM = 256, BN = 256, WM = 2, WN = 4, NW = WM * WN, MF = 16;
constexpr int TM = BM / WM / MF;     // 8 pixel tiles per wave
constexpr int TN = BN / WN / MF;     // 4 cout tiles per wave
constexpr int BK = 32;               // channels per chunk (64-B rows)
constexpr int HS = 512;              // halo slots per buffer (32 KiB)
constexpr int HP = HS / 16 / NW;     // halo DMA pieces per wave: 4
constexpr int NSB = 3;               // weight ring
constexpr int BI = BN / 16 / NW;     // weight DMA pieces per wave per K-step: 2
constexpr int SMEM = 2 * HS * BK + NSB * BN * BK;  // u16 elements: 112 KiB

__device__ __forceinline__ float bf_to_f(u16 v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ u16 f_to_bf(float f) { return __bfloat16_as_ushort(__float2bfloat16(f)); }

__device__ __forceinline__ void dma16(const void* src, u16* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// halo rows a 256-pixel tile can touch on an H x W map (any start pixel): host-side bound
int halo_rows_max(int H, int W) {
  const int HW = H * W;
  int worst = 0;
  for (int r0 = 0; r0 < HW; ++r0) {
    const int m1 = r0 + BM - 1;
    const int img1 = m1 / HW, oy1 = (m1 - img1 * HW) / W;
    const int rows = img1 * (H + 2) + oy1 + 2 - r0 / W + 1;
    worst = rows > worst ? rows : worst;
  }
  return worst;
}
}  // namespace

__global__ __launch_bounds__(64 * NW) void conv_halo_bf16_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) u16 smem[SMEM];
  u16* Hb = smem;                 // [2][HS][BK]
  u16* Bb = smem + 2 * HS * BK;   // [NSB][BN][BK]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int H = a.H, W = a.W, HW = H * W, PW = W + 2, PH = H + 2;
  const int M = a.N * HW;
  const int nN = a.Cout / BN;
  const int bt = xcd_tile(blockIdx.x, gridDim.x, a.xcd);
  const int mt = bt / nN;
  const int nt = bt - mt * nN;
  const int m0 = mt * BM, n0 = nt * BN;
  const u16* __restrict__ x = (const u16*)a.x;
  const u16* __restrict__ w = (const u16*)a.w;
  const u16* zero = (const u16*)a.zero;

  // the tile's halo rows: p_lo .. p_hi
  const int img0 = m0 / HW;
  const int p_lo = img0 * PH + (m0 - img0 * HW) / W;
  const int m1 = min(m0 + BM, M) - 1;
  const int img1 = m1 / HW;
  const int p_hi = img1 * PH + (m1 - img1 * HW) / W + 2;
  const int nslots = (p_hi - p_lo + 1) * PW;

  // halo DMA sources: piece j of this wave = slots (j * NW + wid) * 16 .. +15, lane: slot +
  // lane / 4, chunk position lane % 4 (holding chunk (lane % 4) ^ ((slot >> 2) & 3))
  const u16* hsrc[HP];
#pragma unroll
  for (int j = 0; j < HP; ++j) {
    const int s = (j * NW + wid) * 16 + (lane >> 2);
    const int pr = s / PW;
    const int p = p_lo + pr;
    const int ix = s - pr * PW - 1;
    const int img = p / PH;
    const int iy = p - img * PH - 1;
    const bool ok = s < nslots && img < a.N && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    const int lc = (lane & 3) ^ ((s >> 2) & 3);
    hsrc[j] = ok ? x + (((long long)img * H + iy) * W + ix) * a.xs + lc * 8 : nullptr;
  }
  // weight DMA sources: piece j = cout rows (wid * BI + j) * 16 .. +15 of the tile
  const u16* bsrc[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int row = (wid * BI + j) * 16 + (lane >> 2);
    const int lc = (lane & 3) ^ ((row >> 2) & 3);
    bsrc[j] = w + (long long)(n0 + row) * a.K + lc * 8;
  }
  auto stage_halo = [&](int kc) {
    u16* dst = Hb + (kc & 1) * HS * BK;
#pragma unroll
    for (int j = 0; j < HP; ++j) dma16(hsrc[j] ? hsrc[j] + kc * BK : zero, dst + (j * NW + wid) * 16 * BK);
  };
  auto stage_b = [&](int kt) {
    const int kc = kt / 9, tap = kt - (kt / 9) * 9;
    const int col = (kc >> 1) * 576 + tap * 64 + (kc & 1) * 32;  // chunk-major K: (cin / 64, tap, cin % 64)
    u16* dst = Bb + (kt % NSB) * BN * BK;
#pragma unroll
    for (int j = 0; j < BI; ++j) dma16(bsrc[j] + col, dst + (wid * BI + j) * 16 * BK);
  };

  // fragment lanes: row r = lane % 16, 16-B chunk q = lane / 16 of the 32-channel slice
  const int r = lane & 15;
  const int q = lane >> 4;
  int sb[TM];  // halo slot of each pixel tile's row r at tap (0, 0)
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * (BM / WM) + i * MF + r;
    if (m < M) {
      const int img = m / HW;
      const int rem = m - img * HW;
      const int oy = rem / W;
      sb[i] = (img * PH + oy - p_lo) * PW + rem - oy * W;
    } else {
      sb[i] = 0;  // result dropped by the store's bounds
    }
  }
  const int bsw = (q ^ ((r >> 2) & 3)) * 8;  // B rows wn * 64 + j * 16 + r: swizzle of r alone

  typedef float accv __attribute__((ext_vector_type(4)));
  accv acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = accv{0.f, 0.f, 0.f, 0.f};

  const int nkc = a.Cin / BK;
  const int nk = nkc * 9;
  stage_halo(0);
  stage_b(0);
  if (nk > 1) {
    stage_b(1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(BI) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // EOSV_HALO_STAG: the upper half of the waves (the SIMD partners of the lower half) issue
  // their DMA after half of the K-step's MFMA groups, as conv_bf16's stagger
  const bool late = EOSV_HALO_STAG && wid >= NW / 2;
  for (int kt = 0; kt < nk; ++kt) {
    const int kc = kt / 9;
    const int tap = kt - kc * 9;
    const bool hnext = tap == 0 && kc + 1 < nkc;
    const bool bnext = kt + 2 < nk;
    auto issue = [&]() {
      if (hnext) stage_halo(kc + 1);
      if (bnext) stage_b(kt + 2);
    };
    if (!late) issue();
    const u16* Ha = Hb + (kc & 1) * HS * BK;
    const u16* Bs = Bb + (kt % NSB) * BN * BK;
    const int kh = tap / 3;
    const int toff = kh * PW + tap - kh * 3;
    auto rdA = [&](int i) {
      const int s = sb[i] + toff;
      return *(const bf16x8*)(Ha + s * BK + ((q ^ ((s >> 2) & 3)) * 8));
    };
    bf16x8 bfr[TN], afr[2];
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = *(const bf16x8*)(Bs + (wn * (BN / WN) + j * MF + r) * BK + bsw);
    afr[0] = rdA(0);
#pragma unroll
    for (int g = 0; g < TM; ++g) {
      if (g + 1 < TM) afr[(g + 1) & 1] = rdA(g + 1);
      // this group's first MFMA (hipcc's lgkmcnt wait for its fragments goes before it), then
      // the next group's A read, then the other MFMAs (as in conv_bf16)
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if (g + 1 < TM) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, TN - 1, 0);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[g][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[g & 1], bfr[j], acc[g][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (late && g == TM / 2 - 1) {
        issue();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // B(kt + 1) (and the next chunk's halo, older) landed; this step's halo and B(kt + 2) may fly
    if (hnext && bnext)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(HP + BI) : "memory");
    else if (hnext)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(HP) : "memory");
    else if (bnext)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(BI) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // the K-loop's last wait is inline asm, invisible to the compiler: tell it (else it waits
  // again, for the residual loads too, before the first LDS write below)
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  u16* __restrict__ y = (u16*)a.y;
  const u16* __restrict__ res = (const u16*)a.res;
  // epilogue through LDS (conv_bf16's): pass i moves the i-th 32-row M-subtile of every wave
  constexpr int EPR = WM * 32;
  constexpr int EPS = BN + 4;
  static_assert(EPR * EPS * 4 <= SMEM * 2, "epilogue tile must fit");
  float* ep = (float*)smem;
  float bcol[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) bcol[j] = a.bias ? a.bias[n0 + wn * (BN / WN) + j * MF + r] : 0.f;
  constexpr int TPP = 32 / MF;
  constexpr int NPASS = BM / WM / 32;
  constexpr int IPT = EPR * (BN / 8) / (64 * NW);
  static_assert(IPT * 64 * NW == EPR * (BN / 8), "epilogue work divides evenly");
  const long long ostr = a.Cout;
  const long long tile_bytes = (long long)min(BM, M - m0) * ostr * 2;
  const int nrec = (int)min(tile_bytes, 0x7fffffffLL);
  const __amdgpu_buffer_rsrc_t yr =
      __builtin_amdgcn_make_buffer_rsrc((void*)(y + (long long)m0 * ostr), (short)0, nrec, 0x00020000);
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(res ? res + (long long)m0 * ostr : (const u16*)a.zero), (short)0, res ? nrec : 0, 0x00020000);
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  v4u rv[2][IPT];
  auto chunk = [&](int i, int t, int& lrow, int& c8, int& voff) {
    const int idx = tid + t * 64 * NW;
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
    for (int t = 0; t < TPP; ++t)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int lrow = wm * 32 + t * MF + 4 * q + e;  // 16x16 C/D map: row 4 (lane / 16) + e
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
      const v4u r4 = rv[i & 1][t];
      const unsigned ru[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[2 * k] += bf_to_f((u16)(ru[k] & 0xffff));
        v[2 * k + 1] += bf_to_f((u16)(ru[k] >> 16));
      }
      v4u pk;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        pk[k] = (unsigned)f_to_bf(fmaxf(v[2 * k], rlow)) | ((unsigned)f_to_bf(fmaxf(v[2 * k + 1], rlow)) << 16);
      __builtin_amdgcn_raw_buffer_store_b128(pk, yr, voff, 0, 0);
    }
  }
}

bool conv_halo_bf16_ok(const ConvArgs& a) {
  if (a.split || a.x2 || !a.zero || !a.kcm || a.Cin == 3) return false;
  if (a.KH != 3 || a.KW != 3 || a.KWp != 3 || a.stride != 1 || a.pad != 1 || a.Ho != a.H || a.Wo != a.W) return false;
  if (a.Cin % 64 || a.Cout % BN || a.K != 9 * a.Cin) return false;
  return halo_rows_max(a.H, a.W) * (a.W + 2) <= HS;
}

int launch_conv_halo_bf16(const ConvArgs& a, hipStream_t s) {
  if (!conv_halo_bf16_ok(a)) return set_error("conv_halo_bf16: unsupported shape"), EOSV_ERR_UNSUPPORTED;
  const long long M = (long long)a.N * a.H * a.W;
  const long long nb = ((M + BM - 1) / BM) * (a.Cout / BN);
  if (nb > 0x7fffffffLL) return set_error("conv_halo_bf16: grid too large"), EOSV_ERR_UNSUPPORTED;
  if (a.plan) {
    static const int occ = kernel_occupancy((const void*)conv_halo_bf16_kernel, 64 * NW);
    return record_launch(a.plan, nb, occ);
  }
  hipLaunchKernelGGL(conv_halo_bf16_kernel, dim3((unsigned)nb), dim3(64 * NW), 0, s, a);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

}  // namespace eosv
