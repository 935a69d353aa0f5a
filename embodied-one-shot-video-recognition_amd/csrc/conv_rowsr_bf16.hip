// Row-strip direct 3x3 / stride-1 convs (bf16) with the weights in registers, for the two map
// shapes where all of a conv's folded weights fit one CU's register file (reference models.py:19
// via self.convnet: torchvision BasicBlock / Bottleneck 3x3 convs at 224 x 224 input):
//  * C = 64, 56 x 56 (layer1 of ResNet-18/50): r05 successor of conv_rows_bf16.hip;
//  * C = 64, 64 x 64 (layer1 at 256 x 256, config 5's R101): replaces the 128x64 implicit GEMM;
//  * C = 128, 28 x 28 / 32 x 32 (layer2's stride-1 3x3s, no fused downsample): replaces the tap-shift
//    tile (conv_bf16_ts.hip); their weights are in the chunk-major K order (ConvArgs::kcm).
// Each matches the kernel it replaces bit for bit: the same K order per output (C 64: taps
// ascending, 32-channel halves inside; C 128: the tap-shift order, 32-channel slice outer, kernel
// row, kernel column), the same MFMA per k-slice and the same epilogue arithmetic
// (tests/test_gpu_poison.py A/B).
//
// conv_rows_bf16 kept the 9 x 64 x 64 weights in LDS (72 KiB), so only two strip buffers fit, the
// next strip's DMA had one strip of MFMA time to land, 4 of a k-step's 6 fragment reads were
// weights, and its 7 waves loaded the 4 SIMDs 2-2-2-1 (SQ r05: MFMA-busy 0.44).  Here a persistent
// workgroup of 4 waves (one per SIMD) keeps every weight in registers -- wave w owns couts
// 32 (w % CG) .. +31, CG = C / 32 (2 tiles x KS k-slices: 36 A fragments at C 64 (144 VGPRs), 72 at
// C 128 (288)) and pixel tiles 7 (w / CG) .. +6 of a strip's 4 rows -- so LDS holds only input rows:
// THREE strip buffers (6 staged rows x (W + 2) slots x 2C bytes), the strip two ahead is DMA'd while
// this one computes, and a k-slice's 14 MFMAs per wave need 7 fragment reads.
//
// LDS image of a staged strip: row r (input row y0 - 1 + r, 0..5) x slot p (input column p - 1;
// slots 0 and W + 1 are the zero pad) x C / 8 16-B chunks, logical chunk c of (r, p) stored at
// c ^ swz(p, r) (the XOR applied on the DMA source): swz = p & 7 at C 64 (conv_rows_bf16's),
// (2 p + 8 r) & 15 at C 128 -- both make every B-fragment ds_read_b128 conflict-free for every
// tile, tap and k-slice (tools/lds_sim.py, a simulator of the b128 lane groups of
// MI355X_MICROARCH.md, LDS; the C 64 swizzle at 256-B slots: 2.4 LDS cycles per group on average,
// up to 4-way).  Out-of-frame rows and the pad slots read a zeroed
// 16-B line (a.zero).
//
// Per strip k (buffer k % 3): residual loads of strip k; k-slices 0 .. PPW - 1 each issue one DMA
// piece of strip k + 2 (buffer (k + 2) % 3, read last in strip k - 1, before the barrier that ended
// it; zero lines past the last strip, so the count never changes); the next k-slice's 7 fragments
// are read while this one's 14 MFMAs run; before the epilogue each wave waits for everything but
// strip k + 2's pieces (vmcnt counts loads, stores and LDS-DMA together in issue order,
// MI355X_MICROARCH.md): its residual and its pieces of strip k + 1; epilogue from registers (8-B
// stores, left in flight); lgkmcnt(0) + one barrier.  The waits are the s_waitcnt builtin and the
// residual / ReLU choices compile-time or branch-free, so hipcc's own wait insertion agrees with
// them (r05 ISA: no vmcnt wait inside the k-loop or between the epilogue's stores).
#include <hip/hip_bf16.h>

#include "common.h"

#include <algorithm>

namespace eosv {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

constexpr int R1_TR = 4;   // output rows per strip
constexpr int R1_NW = 4;   // waves
constexpr int R1_NBUF = 3;  // strip buffers

template <int C, int W>
struct RowsR {
  static constexpr int CG = C / 32;                        // cout groups (waves per pixel group)
  static constexpr int PG = R1_NW / CG;                    // pixel groups
  static constexpr int ROWS = R1_TR + 2;                   // staged input rows
  static constexpr int SLOTS = W + 2;                      // slots per staged row
  static constexpr int CPS = C / 8;                        // 16-B chunks per slot
  static constexpr int SB = C * 2;                         // bytes per slot
  static constexpr int CHUNKS = ROWS * SLOTS * CPS;
  static constexpr int PPW = (CHUNKS + 64 * R1_NW - 1) / (64 * R1_NW);  // DMA pieces per wave
  static constexpr int BUF = PPW * R1_NW * 1024;           // bytes per strip buffer
  static constexpr int WT = R1_TR * W / 16 / PG;           // pixel tiles per wave
  static constexpr int NPH = C == 64 ? 1 : 2;              // passes over a strip's tiles (registers)
  static constexpr int TPP = (WT + NPH - 1) / NPH;          // pixel tiles per pass (the last: the rest)
  static constexpr int KQ = C / 32;                        // k-slices per tap
  static constexpr int KS = 9 * KQ;                        // k-slices
  static_assert(R1_NW % CG == 0 && WT * 16 * PG == R1_TR * W, "whole pixel tiles per wave");
  static_assert(R1_NBUF * BUF <= 163840, "LDS budget");
  static_assert(PPW <= KS, "one piece per k-slice");
  // XOR mask of the 16-B chunks of staged (row r, slot p)
  __device__ static __forceinline__ int swz(int p, int r) { return C == 64 ? (p & 7) : ((2 * p + 8 * r) & 15); }
  // k-slice ks -> (tap, 32-channel slice) in the order of the kernel this one replaces
  __host__ __device__ static constexpr int tap(int ks) { return C == 64 ? ks / KQ : ks % 9; }
  __host__ __device__ static constexpr int cslice(int ks) { return C == 64 ? ks % KQ : ks / 9; }
};

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __bfloat16_as_ushort(__float2bfloat16(f)); }
__device__ __forceinline__ void dma16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}
}  // namespace

// RES: the conv adds a residual map (a compile-time branch: the epilogue stays one basic block, so
// hipcc's vmcnt tracking follows the counted waits below and adds none of its own)
template <int C, int W, bool RES>
__global__ __launch_bounds__(64 * R1_NW, 1) void conv_rowsr_bf16_kernel(ConvArgs a, int nstrips) {
  using P = RowsR<C, W>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[R1_NBUF * P::BUF];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = wid % P::CG, pg = wid / P::CG;
  const int r16 = lane & 15, q = lane >> 4;
  const int H = a.H;
  const int spi = H / R1_TR;  // strips per image
  const u16* __restrict__ x = (const u16*)a.x;
  const u16* __restrict__ w = (const u16*)a.w;
  const u16* zero = (const u16*)a.zero;

  // ---- weights: couts 32 cg + 16 j + r16, k-slice ks: channels c0 = 32 cslice + 8 q .. of its tap,
  // K column tap * C + c0, or in the chunk-major order (a.kcm, C >= 128 in bf16: 64-channel chunks)
  // ((c0 / 64) * 9 + tap) * 64 + c0 % 64
  bf16x8 wf[2][P::KS];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int ks = 0; ks < P::KS; ++ks) {
      const int c0 = 32 * P::cslice(ks);
      const int kc = a.kcm ? ((c0 / 64) * 9 + P::tap(ks)) * 64 + c0 % 64 : P::tap(ks) * C + c0;
      wf[j][ks] = *(const bf16x8*)(w + (long long)(32 * cg + 16 * j + r16) * a.K + kc + 8 * q);
    }
  f32x4 bias[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    bias[j] = a.bias ? *(const f32x4*)(a.bias + 32 * cg + 16 * j + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- DMA piece i of a strip: LDS chunk id -> (row, slot, chunk) (the same for every strip)
  auto piece_map = [&](int i, int& goff, int& grow) {
    const int id = (wid + R1_NW * i) * 64 + lane;
    const int r = id / (P::SLOTS * P::CPS);
    const int rem = id - r * (P::SLOTS * P::CPS);
    const int p = rem / P::CPS;
    const int lc = (rem % P::CPS) ^ P::swz(p, r);
    const bool ok = id < P::CHUNKS && p >= 1 && p <= W;
    goff = ((r - 1) * W + (p - 1)) * C + 8 * lc;  // elements from pixel (y0, 0) of the image
    grow = ok ? r : -1000;
  };
  // a strip's staging source: its first output row's pixel 0 and that row's index
  auto strip_src = [&](int strip, const u16*& base, int& y0) {
    const int img = strip / spi;
    y0 = (strip - img * spi) * R1_TR;
    base = x + ((long long)img * H + y0) * W * C;
  };
  auto piece = [&](int i, const u16* base, int y0, int buf) {
    int goff, grow;
    piece_map(i, goff, grow);
    const bool ok = (unsigned)(y0 - 1 + grow) < (unsigned)H;
    dma16(ok ? base + goff : zero, smem + buf * P::BUF + (wid + R1_NW * i) * 1024);
  };

  // ---- B-fragment addresses: pixel tile t of this wave, lane pixel o -> (oy, ox); tap (dy, dx),
  // slice s: staged (row oy + dy, slot ox + dx), chunk (4 s + q) ^ swz
  // pb: byte offset of (oy, ox) at tap (0, 0); sw: its swizzle term (C 64: ox; C 128: 2 ox + 8 oy),
  // to which a tap adds dx (C 64) or 2 dx + 8 dy (C 128) before the mask
  int pb[P::WT], sw[P::WT];
#pragma unroll
  for (int t = 0; t < P::WT; ++t) {
    const int o = 16 * (P::WT * pg + t) + r16;
    const int oy = o / W, ox = o - (o / W) * W;
    pb[t] = (oy * P::SLOTS + ox) * P::SB;
    sw[t] = C == 64 ? ox : 2 * ox + 8 * oy;
  }
  constexpr int RV = P::TPP;  // residual registers: one pass's tiles

  u16* __restrict__ y = (u16*)a.y;
  const u16* __restrict__ res = (const u16*)a.res;  // RES only
  const int G = gridDim.x;
  int strip = xcd_tile(blockIdx.x, G, 1);
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    if (strip + b * G < nstrips) {
      const u16* base;
      int sy0;
      strip_src(strip + b * G, base, sy0);
#pragma unroll
      for (int i = 0; i < P::PPW; ++i) piece(i, base, sy0, b);
    }
  }
  // waits as the builtin (not inline asm), so that hipcc's own vmcnt tracking sees them
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): weights, bias and the first two strips
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  const float rlow = a.relu ? 0.f : -INFINITY;  // ReLU as max(v, rlow): no branch in the epilogue

  for (int k = 0; strip < nstrips; ++k, strip += G) {
    const int cur = k % R1_NBUF;
    const int ahead = strip + 2 * G;
    const int abuf = (k + 2) % R1_NBUF;
    // strip k + 2's pieces; past the last strip every piece reads the zero line into that buffer
    // (buffer (k - 1) % 3, never read again), so every strip issues exactly PPW pieces
    const u16* abase;
    int ay0;
    strip_src(ahead < nstrips ? ahead : 0, abase, ay0);
    if (ahead >= nstrips) ay0 = -(1 << 20);
    const unsigned char* Ib = smem + cur * P::BUF;
    const int img = strip / spi;
    const int y0 = (strip - img * spi) * R1_TR;
    const long long obase = ((long long)img * H + y0) * W;  // strip's first output pixel

#pragma unroll
    for (int ph = 0; ph < P::NPH; ++ph) {
      const int t0 = ph * P::TPP;                                   // this pass's first tile
      const int nt = ph + 1 < P::NPH ? P::TPP : P::WT - t0;         // and its tile count
      // residual of this pass's pixels, loaded now so the k-loop hides its latency.  Plain loads:
      // hipcc counts them (and the LDS-DMA pieces issued after them) in its vmcnt before the first
      // use.  (Inline-asm loads, as conv_rows_bf16 had them until r06, hide the asynchronous register write
      // from the compiler: here it copied the not-yet-loaded values out right after the asm and
      // reused a load's destination pair as the next address -- a memory fault, r05.)
      uint2 rv[RV][2];
      if constexpr (RES) {
#pragma unroll
        for (int u = 0; u < RV; ++u)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            if (u >= nt) continue;
            rv[u][j] = *(const uint2*)(res + (obase + 16 * (P::WT * pg + t0 + u) + r16) * C + 32 * cg + 16 * j + 4 * q);
          }
      }
      f32x4 acc[2][RV];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int u = 0; u < RV; ++u) acc[j][u] = f32x4{0.f, 0.f, 0.f, 0.f};
      bf16x8 bf[2][RV];
      auto frags = [&](int ks, int b) {
        const int tp = P::tap(ks), s = P::cslice(ks);
        const int dy = tp / 3, dx = tp - 3 * (tp / 3);
#pragma unroll
        for (int u = 0; u < RV; ++u) {
          if (u >= nt) continue;
          const int t = t0 + u;
          // recomputed per read (a few VALU under the MFMAs): hipcc would otherwise keep every
          // (tile, tap) address live across the unrolled k-slices (C 128: 4 slices apart) and spill
          int pt = pb[t], st = sw[t];
          asm volatile("" : "+v"(pt), "+v"(st));
          const int m = C == 64 ? ((st + dx) & 7) : ((st + 2 * dx + 8 * dy) & 15);
          bf[b][u] = *(const bf16x8*)(Ib + pt + (dy * P::SLOTS + dx) * P::SB + (((4 * s + q) ^ m) << 4));
        }
      };
      frags(0, 0);
#pragma unroll
      for (int ks = 0; ks < P::KS; ++ks) {
        if (ph == 0 && ks < P::PPW) piece(ks, abase, ay0, abuf);
        if (ks + 1 < P::KS) frags(ks + 1, (ks + 1) & 1);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int u = 0; u < RV; ++u)
            if (u < nt)
              acc[j][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][ks], bf[ks & 1][u], acc[j][u], 0, 0, 0);
      }
      // pass 0: everything but strip k + 2's pieces has landed (this pass's residual and this wave's
      // pieces of strip k + 1, issued a strip earlier); later passes: their residual, the youngest
      if (ph == 0)
        __builtin_amdgcn_s_waitcnt(0x0f70 | (P::PPW & 15) | ((P::PPW >> 4) << 14));  // vmcnt(PPW)
      else
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
      __builtin_amdgcn_sched_barrier(0);  // keep the uses of rv below the wait
      // epilogue from registers, the replaced kernel's arithmetic: + shift, + residual (the tap-shift
      // tile adds its zero-filled residual when there is none: -0 -> +0), ReLU, bf16
#pragma unroll
      for (int u = 0; u < RV; ++u)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (u >= nt) continue;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[j][u][e] + bias[j][e];
            if constexpr (RES) {
            v[0] += bf2f((u16)(rv[u][j].x & 0xffff));
            v[1] += bf2f((u16)(rv[u][j].x >> 16));
            v[2] += bf2f((u16)(rv[u][j].y & 0xffff));
            v[3] += bf2f((u16)(rv[u][j].y >> 16));
          } else if constexpr (!(C == 64 && W == 56)) {  // the implicit GEMM tiles' zero residual (conv_rows_bf16: none)
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += 0.f;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], rlow);
          const unsigned lo = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
          const unsigned hi = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
          *(uint2*)(y + (obase + 16 * (P::WT * pg + t0 + u) + r16) * C + 32 * cg + 16 * j + 4 * q) =
              make_uint2(lo, hi);
        }
    }
    // every wave's reads of buffer cur are done (and its pieces of strip k + 1 have landed) before
    // strip k + 3's pieces refill buffer cur, issued after this barrier; the stores stay in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): every piece has landed before the workgroup ends
}

// 0: not a rowsr shape, else the channel count of the instance that takes it
// 0: not a rowsr shape, else 1 + the instance index (<64, 56>, <64, 64>, <128, 28>, <128, 32>)
static int rowsr_shape(const ConvArgs& a) {
  const int C = a.Cin;
  int inst = 0;
  if (C == 64 && a.W == 56) inst = 1;
  if (C == 64 && a.W == 64) inst = 2;
  if (C == 128 && a.W == 28) inst = 3;
  if (C == 128 && a.W == 32) inst = 4;
  const bool kcm_ok = !a.kcm || (C == 128 && a.kcm == 1);  // bf16 kcm: 64-channel chunks
  return inst && a.Cout == C && a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && a.H % R1_TR == 0 &&
                 a.Ho == a.H && a.Wo == a.W && a.K == 9 * C && !a.x2 && !a.split && kcm_ok && a.xs == C && a.zero &&
                 a.N > 0
             ? inst
             : 0;
}

bool conv_rowsr_bf16_ok(const ConvArgs& a) { return rowsr_shape(a) != 0; }

int launch_conv_rowsr_bf16(const ConvArgs& a, hipStream_t s) {
  const long long nstrips = (long long)a.N * (a.H / R1_TR);
  if (nstrips > 0x7fffffffLL) return set_error("conv_rowsr: too many strips"), EOSV_ERR_UNSUPPORTED;
  const int inst = rowsr_shape(a);
  if (!inst) return set_error("conv_rowsr: unsupported shape"), EOSV_ERR_UNSUPPORTED;
  if (a.plan) return record_launch(a.plan, nstrips, 1);  // persistent: one workgroup per CU walks strips
  const unsigned grid = (unsigned)std::min<long long>(nstrips, device_cu_count());
  const dim3 g(grid), b(64 * R1_NW);
  const bool r = a.res != nullptr;
  using K = void (*)(ConvArgs, int);
  K kern = nullptr;
  if (inst == 1) kern = r ? (K)conv_rowsr_bf16_kernel<64, 56, true> : (K)conv_rowsr_bf16_kernel<64, 56, false>;
  if (inst == 2) kern = r ? (K)conv_rowsr_bf16_kernel<64, 64, true> : (K)conv_rowsr_bf16_kernel<64, 64, false>;
  if (inst == 3) kern = r ? (K)conv_rowsr_bf16_kernel<128, 28, true> : (K)conv_rowsr_bf16_kernel<128, 28, false>;
  if (inst == 4) kern = r ? (K)conv_rowsr_bf16_kernel<128, 32, true> : (K)conv_rowsr_bf16_kernel<128, 32, false>;
  hipLaunchKernelGGL(kern, g, b, 0, s, a, (int)nstrips);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

}  // namespace eosv
