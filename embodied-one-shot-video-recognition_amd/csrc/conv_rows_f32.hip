// Row-strip direct 3x3 conv for ResNet stage 1 in exact f32: 64 -> 64 channels, stride 1, pad 1,
// 56- or 64-wide maps (R18 layer1 and R50 layer1 c2 at 224x224 / 256x256; models.py:19).
//
// On the implicit GEMM (conv_f32_dma.hip, 256x64 tiles) these convs ran at ~115 TF/s against
// ~130 for stages 2-4: every k-step restaged an im2col A tile, i.e. each input pixel went
// through the L2 -> LDS path 9 times, and without that DMA the same tiles ran at 139 TF/s
// (DESIGN 8).  Here, as in conv_rows_x3.hip, a persistent workgroup per CU streams input
// strips through LDS once and the 9 taps read the staged rows in place:
//  * 4 waves, wave g computes couts 16g .. 16g+15 of every pixel of the strip with
//    v_mfma_f32_16x16x4_f32 (exact f32, D = W . X^T); its 16 x 576 weights (144 VGPRs) are
//    loaded once per kernel;
//  * a strip is TR = 2 output rows (RW / 8 pixel tiles of 16); LDS holds its 4 padded input rows
//    [4][RW + 2 slots][64 ch], double-buffered;
//  * a slot is 17 chunks of 16 B (64 floats + 16 B of padding), so that the 16 pixels of a tile
//    fall on 16 different bank groups at every tap and channel offset while every address is
//    a per-tile base plus an immediate; the DMA fills the padding chunk from the zero page;
//  * K per wave: tap (9) x 16-channel group j (4) x step e (4): lane q's k-element of step
//    (tap, j, e) is channel 16j + 4q + e, so one ds_read_b128 gives a lane the B values of 4
//    steps and one float4 of weights their A values; 28 MFMAs (7 tiles x 4 steps, RW 56) per
//    7 reads;
//  * epilogue from registers: acc + shift (+ residual), ReLU, float4 stores (lane = 4
//    consecutive couts of one pixel).
// Strips are dealt XCD-contiguously so that neighbouring strips (which share 2 input rows)
// run on the same L2.
#include <utility>

#include "common.h"

namespace eosv {

namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TR = 2;
constexpr int C = 64;
constexpr int SLOT_CHUNKS = 17;  // 16 data chunks + 1 padding chunk per staged pixel
constexpr int SLOT_BYTES = SLOT_CHUNKS * 16;
constexpr int NW = 4;
constexpr int NT = 64 * NW;

template <int RW>
struct Geo {
  static constexpr int SLOTS = RW + 2;
  static constexpr int ROW_CHUNKS = SLOTS * SLOT_CHUNKS;
  static constexpr int BUF_CHUNKS = (TR + 2) * ROW_CHUNKS;
  static constexpr int PIECES = ((BUF_CHUNKS + 64 * NW - 1) / (64 * NW)) * NW;  // 1-KiB DMA pieces
  static constexpr int PPW = PIECES / NW;
  static constexpr int BUF_BYTES = PIECES * 1024;
  static constexpr int TILES = TR * RW / 16;
  static constexpr int RES_WAVE_BYTES = TILES * 1024;  // a wave's residual: 16 couts of the strip
  static constexpr int LDS_RES = 2 * BUF_BYTES + NW * RES_WAVE_BYTES;
  static_assert(TR * RW == TILES * 16, "strip = whole pixel tiles");
  static_assert(2 * BUF_BYTES <= 163840, "LDS budget");
};

__device__ __forceinline__ void dma16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// f(integral_constant<int, 0>) .. f(integral_constant<int, N - 1>), in order (compile-time
// step index: register-array indices and ds_read immediates)
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
}  // namespace

// ABL (profiling-only instance, EOSV_CONV_ABL bits, results wrong): 1 no prefetch DMA, 2 no residual
// loads, 16 no ds_reads, 32 no MFMAs, 64 no stores
template <int RW, bool RES, bool ABL>
__global__ __launch_bounds__(NT) void conv_rows_f32_kernel(ConvArgs a, int nstrips) {
  using G_ = Geo<RW>;
  constexpr int SLOTS = G_::SLOTS, TILES = G_::TILES, PPW = G_::PPW;
  extern __shared__ __attribute__((aligned(16))) unsigned char crf_smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int g = tid >> 6;  // cout group
  const int r16 = lane & 15;
  const int q = lane >> 4;
  const int H = a.H;
  const int spi = H / TR;
  const float* __restrict__ x = (const float*)a.x;
  const float* zero = (const float*)a.zero;

  // weights: cout 16g + r16, (tap, j): channels 16j + 4q .. +3, K order (kh, kw, cin)
  f32x4 w[36];
  {
    const float* wr = (const float*)a.w + (long long)(16 * g + r16) * a.K + 4 * q;
#pragma unroll
    for (int t = 0; t < 36; ++t) w[t] = *(const f32x4*)(wr + (t >> 2) * C + 16 * (t & 3));
  }
  const f32x4 bias = a.bias ? *(const f32x4*)(a.bias + 16 * g + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};

  // DMA of strip -> buffer: chunk id of the buffer = (row, slot, chunk); slots 0 and RW + 1, the
  // padding chunk and rows outside the map come from the zero page
  auto stage = [&](int strip, int buf) {
    const int img = strip / spi;
    const int y0 = (strip - img * spi) * TR;
    const float* xs = x + ((long long)img * H + y0 - 1) * RW * C;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = g + NW * i;
      const int id = p * 64 + lane;
      const int r = id / G_::ROW_CHUNKS;
      const int rem = id - r * G_::ROW_CHUNKS;
      const int slot = rem / SLOT_CHUNKS;
      const int c = rem - slot * SLOT_CHUNKS;
      const bool ok = id < G_::BUF_CHUNKS && c < 16 && slot >= 1 && slot <= RW && (unsigned)(y0 - 1 + r) < (unsigned)H;
      dma16(ok ? xs + ((long long)r * RW + slot - 1) * C + 4 * c : zero,
            crf_smem + buf * G_::BUF_BYTES + p * 1024);
    }
  };

  // lane's staged pixel of tile i at tap (0, 0), plus its channel quad
  int pb[TILES];
#pragma unroll
  for (int i = 0; i < TILES; ++i) {
    const int o = i * 16 + r16;
    pb[i] = ((o / RW) * SLOTS + o % RW) * SLOT_BYTES + 16 * q;
  }

  const int G = gridDim.x;
  int strip = xcd_tile(blockIdx.x, G, 1);
  if (strip < nstrips) stage(strip, 0);
  asm volatile("" ::: "memory");  // neither builtin is a compiler-level memory barrier: no LDS access or DMA crosses it
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): weights, bias, first strip
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");  // s_barrier is no compiler-level memory barrier

  float* __restrict__ y = (float*)a.y;
  const float* __restrict__ res = (const float*)a.res;
  const float rlow = a.relu ? 0.f : -INFINITY;
  int cur = 0;
  for (; strip < nstrips; strip += G) {
    const int next = strip + G;
    const int abl = ABL ? a.abl : 0;
    if (next < nstrips && !(abl & 1)) stage(next, cur ^ 1);
    const int img = strip / spi;
    const int y0 = (strip - img * spi) * TR;
    const long long obase = ((long long)img * H + y0) * RW * C + 16 * g + 4 * q;
    // residual: each wave DMAs the 64 B per pixel it adds (pixel k * 16 + lane / 4, quad lane % 4)
    // into its own LDS region (in the same array as the strips: a DMA into a second __shared__
    // array makes hipcc wait vmcnt(0) before the next fragment read), so the epilogue needs only
    // this wave's vmcnt.  (Register loads would be live through the k-loop at 256 VGPRs: an asm
    // load's destination may then be copied before the data lands, and a compiler-visible one is
    // waited for before the first MFMA.)
    const bool has_res = RES && (!ABL || (res && !(abl & 2)));  // the ABL instance runs every layer
    unsigned char* rl = crf_smem + 2 * G_::BUF_BYTES + g * G_::RES_WAVE_BYTES;
    if (has_res) {
#pragma unroll
      for (int k = 0; k < TILES; ++k)
        dma16(res + obase - 4 * q + (long long)(k * 16 + (lane >> 2)) * C + 4 * (lane & 3), rl + k * 1024);
    }
    const unsigned char* base[TILES];
#pragma unroll
    for (int i = 0; i < TILES; ++i) base[i] = crf_smem + cur * G_::BUF_BYTES + pb[i];

    f32x4 acc[TILES];
#pragma unroll
    for (int i = 0; i < TILES; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 xb[2][TILES];
    // B fragments of step group t = (tap t / 4, channel group t % 4): immediate offsets only.
    // Plain LDS loads and the s_waitcnt builtin (r06, formerly inline asm, whose asynchronous
    // register write hipcc cannot see): one lgkmcnt(0) per step group retires the next group's
    // reads, and hipcc knows it.
    auto frags_ = [](auto tc, int b, f32x4(&xb)[2][TILES], const unsigned char* const(&base)[TILES], int abl) {
      constexpr int t = decltype(tc)::value;
      constexpr int off = ((t >> 2) / 3 * SLOTS + (t >> 2) % 3) * SLOT_BYTES + 64 * (t & 3);
      if (abl & 16) return;
#pragma unroll
      for (int i = 0; i < TILES; ++i) xb[b][i] = *(const f32x4*)(base[i] + off);
    };
    auto frags = [&](auto tc, int b) { frags_(tc, b, xb, base, abl); };
    frags(std::integral_constant<int, 0>{}, 0);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_sched_barrier(0);
    static_for<36>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      if constexpr (t + 1 < 36) frags(std::integral_constant<int, t + 1>{}, (t + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
      if (!(abl & 32)) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < TILES; ++i)
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[t][e], xb[t & 1][i][e], acc[i], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      __builtin_amdgcn_sched_barrier(0);
    });

    // this wave's residual DMA and next-strip prefetch have landed: vmcnt(0) before the stores, so
    // it waits for nothing else
    asm volatile("" ::: "memory");  // neither builtin is a compiler-level memory barrier: no LDS access or DMA crosses it
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");  // the residual's LDS reads stay below the wait
#pragma unroll
    for (int i = 0; i < TILES; ++i) {
      f32x4 rv = {0.f, 0.f, 0.f, 0.f};
      if (has_res) rv = *(const f32x4*)(rl + i * 1024 + r16 * 64 + q * 16);
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = acc[i][e] + bias[e];
        if constexpr (RES) t += rv[e];
        v[e] = fmaxf(t, rlow);
      }
      float* dst = y + obase + (long long)(i * 16 + r16) * C;
      if (abl & 64) continue;
      // a compiler-visible store: a 16-B store's data VGPRs need a wait state before they are
      // rewritten, which only the compiler's hazard recognizer inserts
      *(f32x4*)dst = v;
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

bool conv_rows_f32_ok(const ConvArgs& a) {
  // 64-wide maps with a residual exceed the LDS (2 x 72 KiB of input + 32 KiB of residual)
  return !a.split && a.Cin == C && a.Cout == C && a.KH == 3 && a.KW == 3 && a.KWp == 3 && a.stride == 1 &&
         a.pad == 1 && (a.W == 56 || (a.W == 64 && !a.res)) && a.H % TR == 0 && a.Ho == a.H && a.Wo == a.W && a.K == 9 * C &&
         !a.x2 && a.zero && (a.xs == 0 || a.xs == C);
}

template <int RW>
static void launch_rw(const ConvArgs& a, int grid, int nstrips, hipStream_t s) {
  const size_t lds = a.res || a.abl ? Geo<RW>::LDS_RES : 2 * Geo<RW>::BUF_BYTES;
#ifdef EOSV_PROFILING
  if constexpr (Geo<RW>::LDS_RES <= 163840) {
    if (a.abl) {
      hipLaunchKernelGGL((conv_rows_f32_kernel<RW, true, true>), dim3(grid), dim3(NT), lds, s, a, nstrips);
      return;
    }
  }
#endif
  if constexpr (Geo<RW>::LDS_RES <= 163840) {
    if (a.res) {
      hipLaunchKernelGGL((conv_rows_f32_kernel<RW, true, false>), dim3(grid), dim3(NT), lds, s, a, nstrips);
      return;
    }
  }
  hipLaunchKernelGGL((conv_rows_f32_kernel<RW, false, false>), dim3(grid), dim3(NT), lds, s, a, nstrips);
}

int launch_conv_rows_f32(const ConvArgs& a, hipStream_t s) {
  if (!conv_rows_f32_ok(a)) return set_error("conv_rows_f32: unsupported shape"), EOSV_ERR_UNSUPPORTED;
  const long long nstrips = (long long)a.N * (a.H / TR);
  if (nstrips <= 0) return EOSV_OK;
  if (nstrips > 0x7fffffffLL) return set_error("conv_rows_f32: too many strips"), EOSV_ERR_UNSUPPORTED;
  if (a.plan) return record_launch(a.plan, nstrips, 1);  // persistent: one workgroup per CU walks strips
  const int grid = (int)std::min<long long>(nstrips, device_cu_count());
  if (a.W == 56)
    launch_rw<56>(a, grid, (int)nstrips, s);
  else
    launch_rw<64>(a, grid, (int)nstrips, s);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

}  // namespace eosv
