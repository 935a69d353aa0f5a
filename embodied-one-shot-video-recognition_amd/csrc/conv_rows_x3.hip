// Row-strip direct 3x3 conv for ResNet stage 1 in the f32x3 (split-bf16) mode: 64 -> 64
// channels, stride 1, pad 1, 56-wide maps (R18 layer1, R50 layer1 c2 at 224x224).
//
// f32x3 activations are stored [pixel][128] bf16 = (hi, lo) blocks of 64 channels and a conv
// sums hi.w_hi + lo.w_hi + hi.w_lo (ConvArgs::split).  On the implicit GEMM that is K = 1728
// over the virtual (hi, lo, hi) channels, the hi block staged twice; stage 1 (Cout 64) ran there at ~29 % of the bf16 MFMA rate and was
// a third of the f32x3 forward.  Here, as in conv_rows_bf16.hip, a persistent workgroup per CU
// streams input strips through LDS and reads the A fragments straight from the staged rows,
// but the weights (w_hi and w_lo: 2 x 72 KiB) cannot share the LDS with the strips, so they
// live in registers:
//  * 4 waves, wave g computes couts 16g .. 16g+15 of every pixel of the strip; its 36 weight
//    fragments (w_hi and w_lo, 18 k-steps of 32) are loaded once per kernel;
//  * a strip is TR = 2 output rows (112 pixels = 7 tiles of 16); LDS holds its 4 padded input
//    rows as two planes (hi, lo) of [4 rows][58 slots][64 ch], double-buffered (120 KiB);
//  * per k-step a wave reads 14 pixel fragments (hi and lo of 7 tiles) and issues 21 MFMAs
//    (w_hi.hi, w_lo.hi, w_hi.lo per tile): 0.67 KiB of LDS reads per MFMA;
//  * epilogue from registers: acc + shift + (res_hi + res_lo), ReLU, split into
//    hi = bf16(v), lo = bf16(v - hi), stored as (hi, lo) -- the same arithmetic as the
//    implicit GEMM's split epilogue (conv_bf16.hip).
// Same staged layout and swizzle as conv_rows_bf16.hip (16-B chunk c of slot p at c ^ (p & 7));
// strips are dealt XCD-contiguously so that neighbouring strips (which share 2 input rows)
// run on the same L2.
#include <hip/hip_bf16.h>

#include "common.h"

namespace eosv {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

constexpr int RW = 56;
constexpr int SLOTS = RW + 2;
constexpr int TR = 2;
constexpr int ROW_CHUNKS = SLOTS * 8;                          // 16-B chunks per staged row
constexpr int PLANE_CHUNKS = (TR + 2) * ROW_CHUNKS;            // 1856
constexpr int PLANE_PIECES = (PLANE_CHUNKS + 63) / 64;         // 29 DMA pieces of 1 KiB
constexpr int PLANE_BYTES = PLANE_PIECES * 1024;
constexpr int NW = 4;
constexpr int NT = 64 * NW;
constexpr int PIECES = 60;                                     // 2 planes, padded to 4 waves x 15
constexpr int PPW = PIECES / NW;
constexpr int BUF = PIECES * 512;                              // bf16 elements per buffer (60 KiB)
constexpr int TILES = TR * RW / 16;                            // 7
constexpr int C = 64;                                          // logical channels
constexpr int PIX = 2 * C;                                     // stored split pixel stride (hi, lo)
constexpr int VC = 3 * C;                                      // virtual input channels (hi, lo, hi)
static_assert(TR * RW == TILES * 16, "strip = 7 pixel tiles");
static_assert(2 * PLANE_PIECES <= PIECES && PIECES % NW == 0, "DMA pieces");
static_assert(2 * BUF * 2 + NW * TILES * 1024 <= 163840, "LDS budget");

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __bfloat16_as_ushort(__float2bfloat16(f)); }

__device__ __forceinline__ void dma16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}
}  // namespace

// ABL (profiling-only instance, EOSV_CONV_ABL bits, results wrong): 1 no prefetch DMA, 2 no residual
// loads, 16 no ds_reads, 32 no MFMAs, 64 no stores
template <bool RES, bool ABL>
__global__ __launch_bounds__(NT) void conv_rows_x3_kernel(ConvArgs a, int nstrips) {
  // residual (r06): behind the two strip buffers each wave DMAs the hi and lo halves of its 16
  // couts of the strip's pixels into a region of its own, [pixel][hi 8 | hi 8 | lo 8 | lo 8]
  // (64 B), so the epilogue waits only for this wave's vmcnt and no register holds an in-flight
  // load across the k-loop.  (One array: a DMA into a second __shared__ array made hipcc wait
  // vmcnt(0) before the strip's first fragment read.)
  __shared__ __attribute__((aligned(16))) u16 In[2 * BUF + (RES ? NW * TILES * 512 : 0)];
  unsigned char* const Rs = (unsigned char*)(In + 2 * BUF);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int g = tid >> 6;  // cout group
  const int r16 = lane & 15;
  const int q = lane >> 4;
  const int H = a.H;
  const int spi = H / TR;
  const u16* __restrict__ x = (const u16*)a.x;
  const u16* __restrict__ w = (const u16*)a.w;
  const u16* zero = (const u16*)a.zero;

  // weight fragments: cout 16g + r16, k-step t = (tap t/2, 32-channel half t&1), chunk q.
  // K order (kh, kw, cin of 192) or, with a.kcm, (cin / 64, kh, kw, cin % 64)
  bf16x8 whi[18], wlo[18];
  {
    const u16* wr = w + (long long)(16 * g + r16) * a.K;
#pragma unroll
    for (int t = 0; t < 18; ++t) {
      const int tap = t >> 1, c = (4 * (t & 1) + q) * 8;
      const int khi = a.kcm ? tap * 64 + c : tap * VC + c;
      const int klo = a.kcm ? (18 + tap) * 64 + c : tap * VC + 2 * C + c;
      whi[t] = *(const bf16x8*)(wr + khi);
      wlo[t] = *(const bf16x8*)(wr + klo);
    }
  }
  const f32x4 bias = a.bias ? *(const f32x4*)(a.bias + 16 * g + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};

  // DMA map (same for every strip): piece p < 29 plane hi, 29..57 plane lo, 58, 59 padding
  int goff[PPW], grow[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int p = g + NW * i;
    const int plane = p >= PLANE_PIECES;
    const int id = (p - plane * PLANE_PIECES) * 64 + lane;
    const int r = id / ROW_CHUNKS;
    const int rem = id - r * ROW_CHUNKS;
    const int slot = rem >> 3;
    const int lc = (rem & 7) ^ (slot & 7);
    const bool ok = p < 2 * PLANE_PIECES && id < PLANE_CHUNKS && slot >= 1 && slot <= RW;
    goff[i] = ((r - 1) * RW + (slot - 1)) * PIX + plane * C + lc * 8;
    grow[i] = ok ? r : -1000;
  }
  auto stage = [&](int strip, int buf) {
    const int img = strip / spi;
    const int y0 = (strip - img * spi) * TR;
    const u16* xs = x + ((long long)img * H + y0) * RW * PIX;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const bool ok = (unsigned)(y0 - 1 + grow[i]) < (unsigned)H;
      dma16(ok ? xs + goff[i] : zero, In + buf * BUF + (g + NW * i) * 512);
    }
  };

  // tiles start at multiples of 16 pixels and 56 = 7 x 8: slot (ox + dx) & 7 = (r16 + dx) & 7,
  // so the swizzled chunk depends on (dx, half) only and the staged pixel on the tile only
  int pb[TILES];
#pragma unroll
  for (int i = 0; i < TILES; ++i) {
    const int o = i * 16 + r16;
    pb[i] = ((o / RW) * SLOTS + o % RW) * 128;
  }

  // strips dealt XCD-contiguously: logical block L of the XCD's range takes strips L, L + G, ...
  const int G = gridDim.x;
  int strip = xcd_tile(blockIdx.x, G, 1);
  if (strip < nstrips) stage(strip, 0);
  asm volatile("" ::: "memory");  // neither builtin is a compiler-level memory barrier: no LDS access or DMA crosses it
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): weights, bias, first strip
  __builtin_amdgcn_s_barrier();

  u16* __restrict__ y = (u16*)a.y;
  const u16* __restrict__ res = (const u16*)a.res;
  const float rlow = a.relu ? 0.f : -INFINITY;
  int cur = 0;
  for (; strip < nstrips; strip += G) {
    const int next = strip + G;
    const int abl = ABL ? a.abl : 0;
    if (next < nstrips && !(abl & 1)) stage(next, cur ^ 1);
    const int img = strip / spi;
    const int y0 = (strip - img * spi) * TR;
    const long long obase = ((long long)img * H + y0) * RW * PIX;
    // residual, DMA'd now so the k-loop hides its latency (r06; it was inline-asm register loads,
    // whose asynchronous register write hipcc cannot see -- the r05 conv_rowsr_bf16 fault -- and
    // plain register loads get a vmcnt(0) before the first MFMA at this kernel's register
    // pressure).  Piece i: pixels 16 i + lane / 4, 16-B part lane & 3 (hi 0-7, hi 8-15, lo 0-7,
    // lo 8-15 of couts 16 g ..).
    const bool has_res = RES && (!ABL || (res && !(abl & 2)));  // the ABL instance runs every layer, res or not
    unsigned char* rw = Rs + (RES ? g * TILES * 1024 : 0);
    if (has_res) {
#pragma unroll
      for (int i = 0; i < TILES; ++i) {
        const int part = lane & 3;
        dma16(res + obase + (long long)(i * 16 + (lane >> 2)) * PIX + (part >> 1) * C + 16 * g + 8 * (part & 1), rw + i * 1024);
      }
    }
    const unsigned char* Ib = (const unsigned char*)(In + cur * BUF);
    unsigned xr[9][2];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        xr[tap][h] = ((tap / 3) * SLOTS + tap % 3) * 128 + (((4 * h + q) ^ ((r16 + tap % 3) & 7)) << 4);

    f32x4 acc[TILES];
#pragma unroll
    for (int i = 0; i < TILES; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 xh[2][TILES] = {}, xl[2][TILES] = {};
    // plain LDS loads (r06, formerly one inline asm per tile): the tile's offset goes through an
    // empty asm, so hipcc re-adds it per read instead of hoisting the 126 summed addresses out of
    // the unrolled k-loop (register pressure), and the lo plane is the read's immediate offset
    auto frags = [&](int t, int b) {
      if (abl & 16) return;
#pragma unroll
      for (int i = 0; i < TILES; ++i) {
        unsigned o = pb[i];
        asm volatile("" : "+v"(o));
        const unsigned char* pp = Ib + (o + xr[t >> 1][t & 1]);
        xh[b][i] = *(const bf16x8*)pp;
        xl[b][i] = *(const bf16x8*)(pp + PLANE_BYTES);
      }
    };
    frags(0, 0);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 18; ++t) {
      if (t + 1 < 18) frags(t + 1, (t + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
      const int b = t & 1;
      if (!(abl & 32)) {
#pragma unroll
        for (int i = 0; i < TILES; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(whi[t], xh[b][i], acc[i], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < TILES; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wlo[t], xh[b][i], acc[i], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < TILES; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(whi[t], xl[b][i], acc[i], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the next step's reads
      __builtin_amdgcn_sched_barrier(0);
    }

    // this wave's residual DMA and next-strip DMA have landed: vmcnt(0) before the stores, so it
    // waits for nothing else (as the builtin: hipcc's tracking sees it)
    asm volatile("" ::: "memory");  // neither builtin is a compiler-level memory barrier: no LDS access or DMA crosses it
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");  // the residual's LDS reads stay below the wait
#pragma unroll
    for (int i = 0; i < TILES; ++i) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][e] + bias[e];
      if constexpr (RES) {  // hi + lo is exact in f32
        uint2 rh = {0, 0}, rl = {0, 0};
        if (has_res) {
          rh = *(const uint2*)(rw + i * 1024 + r16 * 64 + 8 * q);
          rl = *(const uint2*)(rw + i * 1024 + r16 * 64 + 32 + 8 * q);
        }
        v[0] += bf2f((u16)(rh.x & 0xffff)) + bf2f((u16)(rl.x & 0xffff));
        v[1] += bf2f((u16)(rh.x >> 16)) + bf2f((u16)(rl.x >> 16));
        v[2] += bf2f((u16)(rh.y & 0xffff)) + bf2f((u16)(rl.y & 0xffff));
        v[3] += bf2f((u16)(rh.y >> 16)) + bf2f((u16)(rl.y >> 16));
      }
      u16 hb[4], lb[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float f = fmaxf(v[e], rlow);
        hb[e] = f2bf(f);
        lb[e] = f2bf(f - bf2f(hb[e]));
      }
      const uint2 hv = make_uint2((unsigned)hb[0] | ((unsigned)hb[1] << 16), (unsigned)hb[2] | ((unsigned)hb[3] << 16));
      const uint2 lv = make_uint2((unsigned)lb[0] | ((unsigned)lb[1] << 16), (unsigned)lb[2] | ((unsigned)lb[3] << 16));
      u16* dst = y + obase + (long long)(i * 16 + r16) * PIX + 16 * g + 4 * q;
      if (abl & 64) continue;
      *(uint2*)dst = hv;  // compiler-visible stores (r06): hipcc's hazard recognizer guards their data VGPRs
      *(uint2*)(dst + 64) = lv;
    }
    // every wave's next-strip DMA has landed (the wait above) and its reads of buffer cur are
    // done (lgkmcnt(0) ends the k-loop) before it is refilled; the stores stay in flight
    asm volatile("" ::: "memory");  // neither builtin is a compiler-level memory barrier: no LDS access or DMA crosses it
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // s_barrier is no compiler-level memory barrier
    cur ^= 1;
  }
  asm volatile("" ::: "memory");  // neither builtin is a compiler-level memory barrier: no LDS access or DMA crosses it
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
}

bool conv_rows_x3_ok(const ConvArgs& a) {
  return a.split && a.Cin == VC && a.xs == PIX && a.Cout == C && a.KH == 3 && a.KW == 3 && a.KWp == 3 && a.stride == 1 &&
         a.pad == 1 && a.W == RW && a.H % TR == 0 && a.Ho == a.H && a.Wo == a.W && a.K == 9 * VC && !a.x2 &&
         a.zero;
}

int launch_conv_rows_x3(const ConvArgs& a, hipStream_t s) {
  static int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev))
      return 256;
    return n > 0 ? n : 256;
  }();
  if (!conv_rows_x3_ok(a)) return set_error("conv_rows_x3: unsupported shape"), EOSV_ERR_UNSUPPORTED;
  const long long nstrips = (long long)a.N * (a.H / TR);
  if (nstrips <= 0) return EOSV_OK;
  if (nstrips > 0x7fffffffLL) return set_error("conv_rows_x3: too many strips"), EOSV_ERR_UNSUPPORTED;
  const unsigned grid = (unsigned)std::min<long long>(nstrips, ncu);
  if (a.plan) return record_launch(a.plan, nstrips, 1);  // persistent: one workgroup per CU walks strips
#ifdef EOSV_PROFILING
  if (a.abl)
    hipLaunchKernelGGL((conv_rows_x3_kernel<true, true>), dim3(grid), dim3(NT), 0, s, a, (int)nstrips);
  else
#endif
  if (a.res)
    hipLaunchKernelGGL((conv_rows_x3_kernel<true, false>), dim3(grid), dim3(NT), 0, s, a, (int)nstrips);
  else
    hipLaunchKernelGGL((conv_rows_x3_kernel<false, false>), dim3(grid), dim3(NT), 0, s, a, (int)nstrips);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

}  // namespace eosv
