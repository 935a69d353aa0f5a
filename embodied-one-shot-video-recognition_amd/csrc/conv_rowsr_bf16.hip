// Row-strip direct 3x3 / stride-1 conv for ResNet stage 1 (bf16) with the weights in registers:
// Cin = Cout = 64, pad 1, 56-wide NHWC maps, folded BN (+ residual) + ReLU (reference models.py:19
// via self.convnet: torchvision BasicBlock / Bottleneck 3x3 convs of layer1 at 224 x 224).
//
// r05 successor of conv_rows_bf16.hip (same strips, same K order, same MFMA operand roles, same
// epilogue arithmetic: bitwise equal outputs).  That kernel keeps the 9 x 64 x 64 weights in LDS
// (72 KiB), so only two strip buffers fit, the next strip's DMA had one strip of MFMA time to land,
// 4 of a k-step's 6 fragment reads were weights, and its 7 waves load the 4 SIMDs 2-2-2-1
// (SQ r05: MFMA-busy 0.44).  Here, as in conv_s2rows_bf16.hip, a persistent workgroup of 4 waves
// (one per SIMD) keeps all weights in registers -- wave w owns couts 32 (w & 1) .. +31 (2 tiles x 18
// k-slices = 36 A fragments, 144 VGPRs) and pixel tiles 7 (w >> 1) .. +6 of the strip's 14 -- so
// LDS holds only input rows: THREE strip buffers (6 staged rows x 58 slots x 128 B each), the
// strip two ahead is DMA'd while this one computes, and a strip's 14 MFMAs per k-slice per wave
// need 7 fragment reads.
//
// LDS image of a staged strip (as conv_rows_bf16): row r (input row y0 - 1 + r, 0..5) x slot p
// (input column p - 1; slots 0 and 57 are the zero pad) x 8 16-B chunks, chunk c of slot p stored at
// c ^ (p & 7) (XOR applied on the DMA source): conflict-free B-fragment reads for every tap.
// Out-of-frame rows and the pad slots read a zeroed 16-B line (a.zero).
//
// Per strip k (buffer k % 3): residual loads of strip k; k-slices 0..10 each issue one DMA piece of
// strip k + 2 (buffer (k + 2) % 3, read last in strip k - 1, before the barrier that ended it);
// the next k-slice's 7 fragments are read while this one's 14 MFMAs run; before the epilogue each
// wave waits for everything but strip k + 2's pieces (vmcnt counts loads, stores and LDS-DMA
// together in issue order, MI355X_MICROARCH.md): its residual and its pieces of strip k + 1;
// epilogue from registers (8-B stores, left in flight); lgkmcnt(0) + one barrier.
#include <hip/hip_bf16.h>

#include "common.h"

#include <algorithm>

namespace eosv {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

constexpr int R1_W = 56;                                // map width
constexpr int R1_C = 64;                                // channels in and out
constexpr int R1_TR = 4;                                // output rows per strip
constexpr int R1_ROWS = R1_TR + 2;                      // staged input rows
constexpr int R1_SLOTS = R1_W + 2;                      // slots per staged row
constexpr int R1_CHUNKS = R1_ROWS * R1_SLOTS * 8;       // 2784 16-B chunks
constexpr int R1_NW = 4;                                // waves
constexpr int R1_PPW = 11;                              // DMA pieces per wave
constexpr int R1_PIECES = R1_NW * R1_PPW;               // 44 pieces of 1 KiB
constexpr int R1_BUF = R1_PIECES * 1024;                // bytes per strip buffer
constexpr int R1_NBUF = 3;
constexpr int R1_WT = R1_TR * R1_W / 16 / 2;            // 7 pixel tiles per wave
constexpr int R1_KS = 18;                               // k-slices: 9 taps x 2 halves of 32 channels
static_assert(R1_PIECES * 64 >= R1_CHUNKS && (R1_PIECES - 1) * 64 < R1_CHUNKS, "pieces tile the strip");
static_assert(R1_NBUF * R1_BUF <= 163840, "LDS budget");
static_assert(2 * R1_WT * 16 == R1_TR * R1_W, "whole pixel tiles");
static_assert(R1_PPW <= R1_KS, "one piece per k-slice");

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __bfloat16_as_ushort(__float2bfloat16(f)); }
__device__ __forceinline__ void dma16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}
}  // namespace

__global__ __launch_bounds__(64 * R1_NW, 1) void conv_rowsr_bf16_kernel(ConvArgs a, int nstrips) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[R1_NBUF * R1_BUF];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = wid & 1, pg = wid >> 1;
  const int r16 = lane & 15, q = lane >> 4;
  const int H = a.H;
  const int spi = H / R1_TR;  // strips per image
  const u16* __restrict__ x = (const u16*)a.x;
  const u16* __restrict__ w = (const u16*)a.w;
  const u16* zero = (const u16*)a.zero;

  // ---- weights: couts 32 cg + 16 j + r16, k-slice t = (tap t / 2, half t % 2): k = 32 t + 8 q ..
  bf16x8 wf[2][R1_KS];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int t = 0; t < R1_KS; ++t)
      wf[j][t] = *(const bf16x8*)(w + (long long)(32 * cg + 16 * j + r16) * a.K + 32 * t + 8 * q);
  f32x4 bias[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    bias[j] = a.bias ? *(const f32x4*)(a.bias + 32 * cg + 16 * j + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- DMA map of this lane's pieces (the same for every strip): LDS chunk id -> (row, slot, chunk)
  int goff[R1_PPW], grow[R1_PPW];
#pragma unroll
  for (int i = 0; i < R1_PPW; ++i) {
    const int id = (wid + R1_NW * i) * 64 + lane;
    const int r = id / (R1_SLOTS * 8);
    const int rem = id - r * (R1_SLOTS * 8);
    const int p = rem >> 3;
    const int lc = (rem & 7) ^ (p & 7);
    const bool ok = id < R1_CHUNKS && p >= 1 && p <= R1_W;
    goff[i] = ((r - 1) * R1_W + (p - 1)) * R1_C + 8 * lc;  // elements from pixel (y0, 0) of the image
    grow[i] = ok ? r : -1000;
  }
  // a strip's staging source: its first output row's pixel 0 and that row's index
  auto strip_src = [&](int strip, const u16*& base, int& y0) {
    const int img = strip / spi;
    y0 = (strip - img * spi) * R1_TR;
    base = x + ((long long)img * H + y0) * R1_W * R1_C;
  };
  auto piece = [&](int i, const u16* base, int y0, int buf) {
    const bool ok = (unsigned)(y0 - 1 + grow[i]) < (unsigned)H;
    dma16(ok ? base + goff[i] : zero, smem + buf * R1_BUF + (wid + R1_NW * i) * 1024);
  };

  // ---- B-fragment byte offsets: pixel tile t of this wave, lane pixel o -> (oy, ox); tap (dy, dx),
  // half h: slot (oy + dy, ox + dx), chunk (4 h + q) ^ ((ox + dx) & 7) = ((q ^ ((ox + dx) & 7)) ^ 4 h)
  int pb[R1_WT], ob[R1_WT];
#pragma unroll
  for (int t = 0; t < R1_WT; ++t) {
    const int o = 16 * (R1_WT * pg + t) + r16;
    const int oy = o / R1_W, ox = o - (o / R1_W) * R1_W;
    pb[t] = (oy * R1_SLOTS + ox) * 128;
    ob[t] = ox;
  }

  u16* __restrict__ y = (u16*)a.y;
  const u16* __restrict__ res = (const u16*)a.res;
  const int G = gridDim.x;
  int strip = xcd_tile(blockIdx.x, G, 1);
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    if (strip + b * G < nstrips) {
      const u16* base;
      int sy0;
      strip_src(strip + b * G, base, sy0);
#pragma unroll
      for (int i = 0; i < R1_PPW; ++i) piece(i, base, sy0, b);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  for (int k = 0; strip < nstrips; ++k, strip += G) {
    const int cur = k % R1_NBUF;
    const int ahead = strip + 2 * G;
    const bool issue = ahead < nstrips;
    const int abuf = (k + 2) % R1_NBUF;
    const u16* abase = x;
    int ay0 = 0;
    if (issue) strip_src(ahead, abase, ay0);
    const unsigned char* Ib = smem + cur * R1_BUF;
    const int img = strip / spi;
    const int y0 = (strip - img * spi) * R1_TR;
    const long long obase = ((long long)img * H + y0) * R1_W;  // strip's first output pixel

    // residual of this strip's pixels, loaded now so the k-loop hides its latency (inline asm: an
    // ordinary load's use would make hipcc wait vmcnt(0), draining the DMA pieces in flight)
    uint2 rv[R1_WT][2];
    if (res) {
#pragma unroll
      for (int t = 0; t < R1_WT; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const u16* src = res + (obase + 16 * (R1_WT * pg + t) + r16) * R1_C + 32 * cg + 16 * j + 4 * q;
          asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(rv[t][j]) : "v"(src) : "memory");
        }
    }

    f32x4 acc[2][R1_WT];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int t = 0; t < R1_WT; ++t) acc[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 bf[2][R1_WT];
    auto frags = [&](int ks, int b) {
      const int tap = ks >> 1, h = ks & 1;
      const int dy = tap / 3, dx = tap - 3 * (tap / 3);
#pragma unroll
      for (int t = 0; t < R1_WT; ++t) {
        const int ch = (q ^ ((ob[t] + dx) & 7)) ^ (4 * h);
        bf[b][t] = *(const bf16x8*)(Ib + pb[t] + (dy * R1_SLOTS + dx) * 128 + ch * 16);
      }
    };
    frags(0, 0);
#pragma unroll
    for (int ks = 0; ks < R1_KS; ++ks) {
      if (ks < R1_PPW && issue) piece(ks, abase, ay0, abuf);
      if (ks + 1 < R1_KS) frags(ks + 1, (ks + 1) & 1);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < R1_WT; ++t)
          acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][ks], bf[ks & 1][t], acc[j][t], 0, 0, 0);
    }
    // everything but strip k + 2's pieces has landed: this strip's residual and this wave's pieces
    // of strip k + 1 (issued a strip earlier)
    if (issue)
      vm_wait<R1_PPW>();
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);  // keep the uses of rv below the wait
    // epilogue from registers (conv_rows_bf16's arithmetic): + shift (+ residual), ReLU, bf16
#pragma unroll
    for (int t = 0; t < R1_WT; ++t)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[j][t][e] + bias[j][e];
        if (res) {
          v[0] += bf2f((u16)(rv[t][j].x & 0xffff));
          v[1] += bf2f((u16)(rv[t][j].x >> 16));
          v[2] += bf2f((u16)(rv[t][j].y & 0xffff));
          v[3] += bf2f((u16)(rv[t][j].y >> 16));
        }
        if (a.relu)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        const unsigned lo = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
        const unsigned hi = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
        *(uint2*)(y + (obase + 16 * (R1_WT * pg + t) + r16) * R1_C + 32 * cg + 16 * j + 4 * q) = make_uint2(lo, hi);
      }
    // every wave's reads of buffer cur are done (and its pieces of strip k + 1 have landed) before
    // strip k + 3's pieces refill buffer cur, issued after this barrier; the stores stay in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

bool conv_rowsr_bf16_ok(const ConvArgs& a) {
  return a.Cin == R1_C && a.Cout == R1_C && a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 &&
         a.W == R1_W && a.H % R1_TR == 0 && a.Ho == a.H && a.Wo == a.W && a.K == 9 * R1_C && !a.x2 && !a.split &&
         !a.kcm && a.xs == R1_C && a.zero && a.N > 0;
}

int launch_conv_rowsr_bf16(const ConvArgs& a, hipStream_t s) {
  const long long nstrips = (long long)a.N * (a.H / R1_TR);
  if (nstrips > 0x7fffffffLL) return set_error("conv_rowsr: too many strips"), EOSV_ERR_UNSUPPORTED;
  if (a.plan) return record_launch(a.plan, nstrips, 1);  // persistent: one workgroup per CU walks strips
  const unsigned grid = (unsigned)std::min<long long>(nstrips, device_cu_count());
  hipLaunchKernelGGL(conv_rowsr_bf16_kernel, dim3(grid), dim3(64 * R1_NW), 0, s, a, (int)nstrips);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

}  // namespace eosv
