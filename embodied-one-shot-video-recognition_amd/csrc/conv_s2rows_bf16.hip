// Row-strip direct 3x3 / stride-2 conv for the ResNet-18 stage-2 entry (bf16): layer2.0.conv1,
// Cin 64 -> Cout 128, 56 x 56 -> 28 x 28, pad 1, folded BN + ReLU, no residual (reference
// models.py:19 via self.convnet; torchvision BasicBlock.conv1 with stride 2).
//
// Why: on the 512 x 128 implicit-GEMM tile this conv stages every input pixel once per tap
// (1152 B of im2col rows + 288 B of weights per output pixel) through the L2 -> LDS path and ran
// at ~24 % of the bf16 MFMA peak with MFMA-busy 0.29 (profiles/r04j_sq_r18_bf16.txt, r05 SQ).
// Here a persistent workgroup (one per CU, 4 waves) keeps ALL 128 x 576 folded weights in
// registers -- wave w owns couts 32 w .. 32 w + 31: 2 tiles x 18 k-slices = 36 A fragments, 144
// VGPRs (one wave per SIMD: the unified 512-entry file) -- and streams strips of 4 output rows:
// the 9 input rows they need are LDS-DMA'd once (76 KiB, double-buffered), 576 B staged per
// output pixel for all 128 couts, and every tap's B fragment is read from the staged rows.
//
// LDS image of a staged strip: row r (input row 2 oy0 - 1 + r, 0..8) x slot p (input column p - 1,
// 60 slots, slot 0 = the left zero pad, slots past 56 zero) x 9 16-B chunks (8 channel chunks + 1
// zero pad): chunk index (r * 60 + p) * 9 + c.  With 144-B slots and 60-slot rows, the B-fragment
// reads (lane (r16, q) of pixel tile t reads chunk ((2 oy + dy) * 60 + 2 ox + dx) * 9 + 4 h + q)
// are conflict-free for every tap, k half and tile of the strip (a small simulator of the
// ds_read_b128 lane groups; 128-B slots were 2- to 8-way).  Out-of-frame rows and the pad chunks
// read a zeroed 16-B line (a.zero).
//
// MFMA v_mfma_f32_16x16x32_bf16, D = W . X^T: a lane ends with 4 adjacent couts of one pixel, so
// the epilogue (shift, ReLU, bf16) stores 8 B per lane straight from registers.  K order per
// output: the implicit GEMM's stride-2 tap order (tap_order in conv_bf16.hip: 0 2 6 8 1 7 3 5 4),
// 32-channel slices ascending within a tap, and its epilogue arithmetic (shift, + 0 residual,
// max), so the result equals it bit for bit (tests/test_gpu_poison.py A/B).
// Per strip: the next strip's 76 DMA pieces go out one or two per k-slice among the MFMAs
// (an LDS-DMA issue costs its wave 60-185 cycles), the next k-slice's 7 B fragments are read
// while the current one's 14 MFMAs run, one barrier per strip.
#include <hip/hip_bf16.h>

#include "common.h"

#include <algorithm>

namespace eosv {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

constexpr int S2_H = 56, S2_W = 56, S2_HO = 28, S2_WO = 28;
constexpr int S2_CIN = 64, S2_COUT = 128;
constexpr int S2_TR = 4;                              // output rows per strip
constexpr int S2_ROWS = 2 * S2_TR + 1;                // staged input rows
constexpr int S2_SLOTS = 60;                          // slots per staged row (57 used)
constexpr int S2_CPS = 9;                             // 16-B chunks per slot (8 + 1 pad)
constexpr int S2_CHUNKS = S2_ROWS * S2_SLOTS * S2_CPS;  // 4860
constexpr int S2_PIECES = (S2_CHUNKS + 63) / 64;        // 76 DMA pieces of 1 KiB
constexpr int S2_BUF = S2_PIECES * 1024;                // bytes per buffer
constexpr int S2_NW = 4;                                // waves
constexpr int S2_PPW = S2_PIECES / S2_NW;               // 19 pieces per wave
constexpr int S2_TILES = S2_TR * S2_WO / 16;            // 7 pixel tiles of 16 per strip
constexpr int S2_KS = 18;                               // k-slices: 9 taps x 2 halves of 32 channels
// k-slice ks -> tap: the implicit GEMM's stride-2 order (conv_bf16.hip tap_order)
__host__ __device__ constexpr int s2_tap(int ks) { return (int)((0x453718620ull >> (4 * (ks >> 1))) & 15); }
static_assert(S2_PIECES % S2_NW == 0 && 2 * S2_BUF <= 163840, "LDS budget");
static_assert(S2_TR * S2_WO == 16 * S2_TILES, "whole pixel tiles");

__device__ __forceinline__ void dma16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}
__device__ __forceinline__ unsigned pack_bf2(float lo, float hi) {
  typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
  typedef float f32x2v __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2v){lo, hi}, bf16x2v));
}
}  // namespace

__global__ __launch_bounds__(64 * S2_NW, 1) void conv_s2rows_bf16_kernel(ConvArgs a, int nstrips) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * S2_BUF];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, q = lane >> 4;
  const u16* __restrict__ x = (const u16*)a.x;
  const u16* __restrict__ w = (const u16*)a.w;
  const u16* zero = (const u16*)a.zero;
  constexpr int SPI = S2_HO / S2_TR;  // strips per image

  // ---- weights: couts 32 wid + 16 j + r16, k-slice t = (tap, half): k = 64 tap + 32 half + 8 q ..
  bf16x8 wf[2][S2_KS];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < S2_KS; ++t)
      wf[j][t] = *(const bf16x8*)(w + (long long)(32 * wid + 16 * j + r16) * a.K + 64 * s2_tap(t) + 32 * (t & 1) +
                                  8 * q);
  f32x4 bias[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    bias[j] = a.bias ? *(const f32x4*)(a.bias + 32 * wid + 16 * j + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- DMA map of this lane's pieces (the same for every strip): LDS chunk id -> (row, slot, c)
  int goff[S2_PPW], grow[S2_PPW];
#pragma unroll
  for (int i = 0; i < S2_PPW; ++i) {
    const int id = (wid + S2_NW * i) * 64 + lane;
    const int r = id / (S2_SLOTS * S2_CPS);
    const int rem = id - r * (S2_SLOTS * S2_CPS);
    const int p = rem / S2_CPS, c = rem - p * S2_CPS;
    const bool ok = id < S2_CHUNKS && c < 8 && p >= 1 && p <= S2_W;
    goff[i] = ((r - 1) * S2_W + (p - 1)) * S2_CIN + 8 * c;  // elements from pixel (2 oy0, 0) of the image
    grow[i] = ok ? r : -1000;
  }
  auto piece = [&](int i, int strip, int buf) {
    const int img = strip / SPI;
    const int oy0 = (strip - img * SPI) * S2_TR;
    const int iy0 = 2 * oy0;  // input row of staged row 1
    const bool ok = (unsigned)(iy0 - 1 + grow[i]) < (unsigned)S2_H;
    const u16* src = ok ? x + ((long long)img * S2_H + iy0) * S2_W * S2_CIN + goff[i] : zero;
    dma16(src, smem + buf * S2_BUF + (wid + S2_NW * i) * 1024);
  };

  // ---- B-fragment addresses: pixel tile t, lane pixel o = 16 t + r16 -> (oy, ox); tap (dy, dx),
  // half h: chunk ((2 oy + dy) * 60 + 2 ox + dx) * 9 + 4 h + q
  int bbase[S2_TILES];
#pragma unroll
  for (int t = 0; t < S2_TILES; ++t) {
    const int o = 16 * t + r16;
    const int oy = o / S2_WO, ox = o - (o / S2_WO) * S2_WO;
    bbase[t] = ((2 * oy * S2_SLOTS + 2 * ox) * S2_CPS + q) * 16;
  }

  u16* __restrict__ y = (u16*)a.y;
  int strip = xcd_tile(blockIdx.x, gridDim.x, 1);
  if (strip < nstrips) {
#pragma unroll
    for (int i = 0; i < S2_PPW; ++i) piece(i, strip, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  for (int k = 0; strip < nstrips; ++k, strip += gridDim.x) {
    const int cur = k & 1;
    const int next = strip + gridDim.x;
    const unsigned char* Ib = smem + cur * S2_BUF;
    f32x4 acc[2][S2_TILES];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int t = 0; t < S2_TILES; ++t) acc[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 bf[2][S2_TILES];
    auto frags = [&](int ks, int b) {
      const int tap = s2_tap(ks), h = ks & 1;
      const int dy = tap / 3, dx = tap - 3 * (tap / 3);
      const int off = ((dy * S2_SLOTS + dx) * S2_CPS + 4 * h) * 16;
#pragma unroll
      for (int t = 0; t < S2_TILES; ++t) bf[b][t] = *(const bf16x8*)(Ib + bbase[t] + off);
    };
    frags(0, 0);
#pragma unroll
    for (int ks = 0; ks < S2_KS; ++ks) {
      // the next strip's staging: pieces 0 .. 18 over k-slices 0 .. 17 (k-slice 0 takes two)
      if (next < nstrips) {
        if (ks == 0) piece(0, next, cur ^ 1);
        piece(ks + 1, next, cur ^ 1);
      }
      if (ks + 1 < S2_KS) frags(ks + 1, (ks + 1) & 1);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < S2_TILES; ++t)
          acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][ks], bf[ks & 1][t], acc[j][t], 0, 0, 0);
    }
    // epilogue straight from registers: + shift, ReLU, bf16, 8-B stores (4 couts of one pixel)
    asm volatile("" ::: "memory");  // the stores stay after this strip's DMA pieces (vm_wait below)
    const int img = strip / SPI;
    const int oy0 = (strip - img * SPI) * S2_TR;
    const long long pbase = ((long long)img * S2_HO + oy0) * S2_WO;  // strip's first output pixel
#pragma unroll
    for (int t = 0; t < S2_TILES; ++t)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[j][t][e] + bias[j][e];
          v[e] += 0.f;  // the implicit GEMM's (absent) residual: -0 -> +0 as there
          if (a.relu) v[e] = fmaxf(v[e], 0.f);
        }
        *(uint2*)(y + (pbase + 16 * t + r16) * S2_COUT + 32 * wid + 16 * j + 4 * q) =
            make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
      }
    // every wave's pieces of the next strip have landed (younger than them: this strip's 14
    // stores) and its reads of buffer cur are done before the next strip refills it
    vm_wait<2 * S2_TILES>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

bool conv_s2rows_bf16_ok(const ConvArgs& a) {
  return a.Cin == S2_CIN && a.Cout == S2_COUT && a.KH == 3 && a.KW == 3 && a.stride == 2 && a.pad == 1 &&
         a.H == S2_H && a.W == S2_W && a.Ho == S2_HO && a.Wo == S2_WO && a.K == 9 * S2_CIN && !a.res && !a.x2 &&
         !a.split && !a.kcm && a.xs == S2_CIN && a.zero && a.N > 0;
}

int launch_conv_s2rows_bf16(const ConvArgs& a, hipStream_t s) {
  const long long nstrips = (long long)a.N * (S2_HO / S2_TR);
  if (nstrips > 0x7fffffffLL) return set_error("conv_s2rows: too many strips"), EOSV_ERR_UNSUPPORTED;
  if (a.plan) return record_launch(a.plan, nstrips, 1);  // persistent: one workgroup per CU walks strips
  const unsigned grid = (unsigned)std::min<long long>(nstrips, device_cu_count());
  hipLaunchKernelGGL(conv_s2rows_bf16_kernel, dim3(grid), dim3(64 * S2_NW), 0, s, a, (int)nstrips);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

}  // namespace eosv
