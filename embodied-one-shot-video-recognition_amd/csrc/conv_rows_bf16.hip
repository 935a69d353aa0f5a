// Row-strip direct 3x3 conv for ResNet stage 1 (bf16): Cin = Cout = 64, stride 1, pad 1,
// 56-wide NHWC maps (every 3x3 conv of layer1 of ResNet-18/50 at 224x224 input).
//
// Why a second conv kernel: the implicit GEMM (conv_bf16.hip) re-reads every input pixel
// from L2 once per tap (9x) and, with Cout = 64, its 128x64 tiles run at ~43 FLOP per byte
// staged -- layer1 was 32 % of the bf16 forward at ~520 TF/s.  Here a persistent workgroup
// (one per CU) keeps all 9 x 64 x 64 folded weights resident in LDS (72 KiB) and streams
// the input as strips: the 6 padded input rows (58 x 64 ch) a strip of TR = 4 output rows
// needs, double-buffered, so a strip's MFMA work (224 x 64 x 576) reads 44 KiB: ~370 FLOP
// per staged byte.  A fragments are read straight from the staged rows: output pixel
// (oy, ox) and tap (dy, dx) read staged row oy + dy, slot ox + dx.
//
// LDS (exactly 160 KiB): W [9 taps][64 cout][64 cin] | In[2][6 rows][58 slots][64 ch] (each
// buffer padded to 44 KiB so the DMA pieces tile it).  128-B pixel / weight rows; 16-B chunk
// c of input slot p stored at c ^ (p & 7), of weight row cout at c ^ ((cout >> 1) & 7) (XOR
// applied on the DMA source).  Both make every ds_read_b128 fragment read conflict-free for
// this kernel's pixel tiles, any tap (an input swizzle on p >> 1 cost 1.7x on the A reads).
// 7 waves: wave w owns output-pixel tiles 2w, 2w+1 (16 px each, 224 per strip) x all 64
// channels, v_mfma_f32_16x16x32_bf16 computing D = W . X^T so that a lane ends up holding 4
// adjacent channels of one pixel.  Epilogue from registers: acc + folded-BN shift
// (+ residual) + ReLU, 8-B stores; no LDS staging, no epilogue barriers.
//
// Pipeline per strip: issue next strip's DMA (buffer cur^1) and this strip's residual loads
// -> MFMAs on buffer cur -> vmcnt(0) (the DMA, issued a strip earlier) -> epilogue (8 global
// stores per lane, left in flight) -> barrier.
#include <hip/hip_bf16.h>

#include "common.h"

namespace eosv {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

constexpr int RW = 56;            // map width
constexpr int TR = 4;             // output rows per strip
constexpr int SLOTS = RW + 2;     // padded input row
constexpr int NWAVE = 7;
constexpr int NT = 64 * NWAVE;    // 448 threads
constexpr int ROW_CHUNKS = SLOTS * 8;                   // 16-B chunks per staged row
constexpr int IN_CHUNKS = (TR + 2) * ROW_CHUNKS;        // 2784
constexpr int IN_PIECES = (IN_CHUNKS + 63) / 64;        // 44 DMA pieces of 1 KiB
constexpr int IN_ELEMS = IN_PIECES * 512;               // bf16 elements per buffer (44 KiB)
constexpr int W_ELEMS = 9 * 64 * 64;                    // 72 KiB
constexpr int W_PIECES = W_ELEMS / 512;                 // 72
static_assert(W_ELEMS + 2 * IN_ELEMS == 163840 / 2, "LDS budget");
static_assert(TR * RW == NWAVE * 2 * 16, "strip = 7 waves x 2 pixel tiles");

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __bfloat16_as_ushort(__float2bfloat16(f)); }

__device__ __forceinline__ void dma16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}
}  // namespace

template <bool ABL>
__global__ __launch_bounds__(NT) void conv_rows_bf16_kernel(ConvArgs a, int nstrips) {
  __shared__ __attribute__((aligned(16))) u16 smem[W_ELEMS + 2 * IN_ELEMS];
  u16* Ws = smem;
  u16* In = smem + W_ELEMS;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int H = a.H;
  const int spi = H / TR;  // strips per image
  const u16* __restrict__ x = (const u16*)a.x;
  const u16* __restrict__ w = (const u16*)a.w;
  const u16* zero = (const u16*)a.zero;

  // resident weights: global [cout][tap*64 + c] -> LDS [tap][cout][chunk ^ swz(cout)]
  for (int p = wid; p < W_PIECES; p += NWAVE) {
    const int id = p * 64 + lane;  // 16-B chunk id in LDS order
    const int row = id >> 3;       // tap * 64 + cout
    const int tap = row >> 6, co = row & 63;
    const int lc = (id & 7) ^ ((co >> 1) & 7);
    dma16(w + (long long)co * a.K + tap * 64 + lc * 8, Ws + p * 512);
  }
  // Input strip rows (y0-1 .. y0+4) -> In[buf]; out-of-image rows / pad columns read zero.
  // The chunk -> (staged row, source offset) map is the same for every strip: precomputed.
  constexpr int PPW = (IN_PIECES + NWAVE - 1) / NWAVE;  // DMA pieces per wave (6 or 7)
  int goff[PPW], grow[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int id = (wid + NWAVE * i) * 64 + lane;
    const int r = id / ROW_CHUNKS;
    const int rem = id - r * ROW_CHUNKS;
    const int slot = rem >> 3;
    const int lc = (rem & 7) ^ (slot & 7);
    const bool colok = id < IN_CHUNKS && slot >= 1 && slot <= RW;
    goff[i] = ((r - 1) * RW + (slot - 1)) * 64 + lc * 8;  // from pixel (y0, 0)
    grow[i] = colok ? r : -1000;
  }
  auto stage = [&](int strip, int buf) {
    const int img = strip / spi;
    const int y0 = (strip - img * spi) * TR;
    const u16* xs = x + ((long long)img * H + y0) * RW * 64;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = wid + NWAVE * i;
      if (p < IN_PIECES) {
        const bool ok = (unsigned)(y0 - 1 + grow[i]) < (unsigned)H;
        dma16(ok ? xs + goff[i] : zero, In + buf * IN_ELEMS + p * 512);
      }
    }
  };

  const int r16 = lane & 15;
  const int q = lane >> 4;
  // this lane's A-fragment pixels (one per pixel tile): staged (row oy, slot ox) at tap (0, 0)
  int apix[2], aslot[2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const int o = (2 * wid + mi) * 16 + r16;
    const int oy = o / RW, ox = o - (o / RW) * RW;
    apix[mi] = oy * SLOTS + ox;
    aslot[mi] = ox;
  }
  // D = W . X^T per tile: a lane's 4 accumulators are couts j*16 + 4q .. +3 of pixel r16
  f32x4 bias[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bias[j] = a.bias ? *(const f32x4*)(a.bias + j * 16 + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};

  // strips dealt XCD-contiguously (as conv_rows_f32): at each step the 32 workgroups of an XCD
  // walk 32 consecutive strips, so the 2 halo rows a strip shares with its neighbour are read
  // from that XCD's L2 instead of another XCD's (round-robin placement put neighbours on
  // different XCDs)
  int strip = xcd_tile(blockIdx.x, gridDim.x, 1);
  if (strip < nstrips) stage(strip, 0);
  // vmcnt(0) as the builtin (not asm) so the compiler's wait tracking knows the bias loads
  // have landed and does not re-wait for them (draining the in-flight DMA) inside the loop
  asm volatile("" ::: "memory");  // neither builtin is a compiler-level memory barrier: no LDS access or DMA crosses it
  __builtin_amdgcn_s_waitcnt(0x0f70);
  __builtin_amdgcn_s_barrier();

  u16* __restrict__ y = (u16*)a.y;
  const u16* __restrict__ res = (const u16*)a.res;
  for (int k = 0; strip < nstrips; ++k, strip += gridDim.x) {
    const int cur = k & 1;
    const int next = strip + gridDim.x;
    // a.abl (EOSV_CONV_ABL, profiling-only, results wrong): 1 no prefetch DMA, 2 no residual
    // loads, 16 no ds_reads, 32 no MFMAs, 64 no epilogue stores
    const int abl = ABL ? a.abl : 0;  // the default instance compiles without the ablation branches
    if (next < nstrips && !(abl & 1)) stage(next, cur ^ 1);
    const u16* Ib = In + cur * IN_ELEMS;
    const int img = strip / spi;
    const int y0 = (strip - img * spi) * TR;
    const long long obase = ((long long)img * H + y0) * RW * 64;  // strip's first output pixel
    // Residual for the epilogue, loaded now so the MFMA phase hides its latency.  Plain loads
    // (r06): hipcc counts them, and the DMA pieces issued before them, in its own vmcnt tracking,
    // and their first use is behind the epilogue's vmcnt(0) below, so no wait lands in the k-loop.
    // (Inline-asm loads hide the asynchronous register write from the compiler, which may then
    // copy or reuse the destination before the data lands: the r05 conv_rowsr_bf16 fault.)
    uint2 rv[2][4] = {};
    if (res && !(abl & 2)) {
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          rv[mi][j] = *(const uint2*)(res + obase + ((2 * wid + mi) * 16 + r16) * 64 + j * 16 + 4 * q);
    }

    f32x4 acc[2][4];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[mi][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // 18 k-steps (9 taps x two 32-deep slices).  Fragments double-buffered in registers: the
    // next step's 6 ds_reads go out ahead of this step's 8 MFMAs (sched_barrier keeps each step's
    // reads and MFMAs in place), and one lgkmcnt(0) after them retires the next step's reads.
    // Plain LDS loads and the s_waitcnt builtin (r06, formerly inline asm): hipcc sees both, so
    // no fragment register can be touched before its read has landed.  (Left to itself hipcc
    // waited lgkmcnt(0) right after issuing every second step's reads.)
    bf16x8 af[2][2] = {}, bf[2][4] = {};
    auto frags = [&](int t, int b) {
      const int tap = t >> 1, dy = tap / 3, dx = tap - (tap / 3) * 3;
      const int lc = 4 * (t & 1) + q;  // this lane's 16-B chunk of the 32-deep k-slice
      if (abl & 16) return;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        const int pix = apix[mi] + dy * SLOTS + dx;
        af[b][mi] = *(const bf16x8*)(Ib + pix * 64 + ((lc ^ ((aslot[mi] + dx) & 7)) * 8));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = j * 16 + r16;
        bf[b][j] = *(const bf16x8*)(Ws + (tap * 64 + co) * 64 + ((lc ^ ((co >> 1) & 7)) * 8));
      }
    };
    frags(0, 0);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 18; ++t) {
      if (t + 1 < 18) frags(t + 1, (t + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);  // the reads go out before this step's MFMAs
      if (!(abl & 32))
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[mi][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[t & 1][j], af[t & 1][mi], acc[mi][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);  // ... and the wait after all of them
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      __builtin_amdgcn_sched_barrier(0);
    }

    // Epilogue straight from registers: per (pixel tile, cout tile) a lane owns 4 adjacent
    // channels of one pixel -> one 8-B store (16 lanes x 32 B per pixel row per instruction).
    // The next strip's DMA and the residual loads above have landed: vmcnt(0) here, before the
    // stores, so the wait covers nothing but them (as the builtin: hipcc's tracking sees it and
    // adds no wait of its own before the uses of rv).
    asm volatile("" ::: "memory");  // neither builtin is a compiler-level memory barrier: no LDS access or DMA crosses it
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
    __builtin_amdgcn_sched_barrier(0);  // keep the uses of rv below the wait
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[mi][j][e] + bias[j][e];
        if (res) {
          v[0] += bf2f((u16)(rv[mi][j].x & 0xffff));
          v[1] += bf2f((u16)(rv[mi][j].x >> 16));
          v[2] += bf2f((u16)(rv[mi][j].y & 0xffff));
          v[3] += bf2f((u16)(rv[mi][j].y >> 16));
        }
        if (a.relu)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        const unsigned lo = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
        const unsigned hi = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
        if (!(abl & 64)) *(uint2*)(y + obase + ((2 * wid + mi) * 16 + r16) * 64 + j * 16 + 4 * q) = make_uint2(lo, hi);
      }
    // every wave's next-strip DMA has landed (its wait above) and its reads of buffer cur are done
    // (lgkmcnt(0) ends the k-loop) before buffer cur is refilled; the stores stay in flight
    asm volatile("" ::: "memory");  // neither builtin is a compiler-level memory barrier: no LDS access or DMA crosses it
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // s_barrier is no compiler-level memory barrier: no read of buffer cur^1 above it
  }
  asm volatile("" ::: "memory");  // neither builtin is a compiler-level memory barrier: no LDS access or DMA crosses it
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the stores have left before the workgroup ends
}

// shapes this kernel takes (everything else stays on the implicit GEMM)
bool conv_rows_bf16_ok(const ConvArgs& a) {
  return a.Cin == 64 && a.Cout == 64 && a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && a.W == RW &&
         a.H % TR == 0 && a.Ho == a.H && a.Wo == a.W && a.K == 9 * 64 && a.zero;
}

int launch_conv_rows_bf16(const ConvArgs& a, hipStream_t s) {
  static int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev))
      return 256;
    return n > 0 ? n : 256;
  }();
  const long long nstrips = (long long)a.N * (a.H / TR);
  if (nstrips <= 0) return EOSV_OK;
  if (nstrips > 0x7fffffffLL) return set_error("conv_rows: too many strips"), EOSV_ERR_UNSUPPORTED;
  const unsigned grid = (unsigned)std::min<long long>(nstrips, ncu);
  if (a.plan) return record_launch(a.plan, nstrips, 1);  // persistent: one workgroup per CU walks strips
#ifdef EOSV_PROFILING
  if (a.abl)
    hipLaunchKernelGGL(conv_rows_bf16_kernel<true>, dim3(grid), dim3(NT), 0, s, a, (int)nstrips);
  else
#endif
    hipLaunchKernelGGL(conv_rows_bf16_kernel<false>, dim3(grid), dim3(NT), 0, s, a, (int)nstrips);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

}  // namespace eosv
