// Whole basic-block fusion for the bf16 ResNet-18 stage 1 (r06): one persistent launch runs a
// block's conv1 (3x3 64 -> 64, ReLU) -> conv2 (3x3 64 -> 64, + the block input, ReLU) --
// torchvision BasicBlock.forward, reached from the reference's models.py:18-19 (model_resnet18 ..
// self.convnet) via network_test.py:186-187, 202-203, 241.
//
// Why: unfused (conv_rows_bf16 twice) a block moves ~1.0 KB per pixel -- x in (1.5x for the strip
// halo) and T out for conv1, T in, x again as the residual and y out for conv2.  Here the conv1
// output T never leaves the CU and the residual is read from the same staged rows conv1 uses:
// 128 B in, 128 B out per pixel.
//
// Shape of the work: the stream of two-row steps of bneck_bf16_kernel (bneck_bf16.hip), one 8-wave
// workgroup per CU walking whole images, a zero step between images.  Per step g:
//   X rows of step g + 2 (register fragments loaded a step earlier) -> X ring in LDS (8 rows of
//   W + 2 slots, pad slots zero); step g + 3's loads go out
//   | barrier |
//   conv1 of step g + 1 from the X ring -> T ring (5 rows), bias + ReLU; a zero step writes zero rows
//   | barrier |
//   conv2 of step g from the T ring, + bias + the residual (X ring) + ReLU -> y
// Wave w owns cout tile w & 3 (16 couts) of the 4 pixel tiles of step row w >> 2 in both convs,
// with both convs' 16 x 576 weights in registers (2 x 18 fragments).  Ring rows: X row R at R & 7
// (written two steps ahead, last read two steps later: no extra barrier), T row R at R % 5.
//
// Arithmetic: both convs as conv_rows_bf16 (v_mfma_f32_16x16x32_bf16, D = W . X^T, 18 k-steps
// tap-major with two 32-channel halves per tap, epilogue + shift (+ residual), ReLU, bf16), so y is
// bitwise that of the unfused path (tests/test_gpu_poison.py: test_bblock_bitwise_equal_unfused).
// In place (y = x, as the engine runs stage 1) is safe: a pixel's input is loaded two steps before
// its output is stored, and a workgroup owns whole images.
#include <hip/hip_bf16.h>

#include <utility>

#include "common.h"

namespace eosv {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned short u16;
using epi::bf2_f;
using epi::relu_bf2;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t bb_rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0,
                                           (int)(bytes > 0x7fffffffLL ? 0x7fffffffLL : (bytes < 0 ? 0 : bytes)), 0x00020000);
}
}  // namespace

constexpr int BB_NW = 8;  // waves per workgroup (two per SIMD)

template <int W>
struct BbGeo {
  static constexpr int SP = 2 * W;           // pixels per step
  static constexpr int SLOTS = W + 2;        // ring row: pad slot, W pixels, pad slot
  static constexpr int ROWB = SLOTS * 128;   // bytes per ring row (64 bf16 per slot)
  static constexpr int XR = 8, TR = 5;       // ring rows
  static constexpr int B_OFF = 0;            // b1[64] b2[64]
  static constexpr int PAD = 1024;            // idle lanes of the last tile read up to 8 slots past a row
  static constexpr int X_OFF = 512;
  static constexpr int T_OFF = X_OFF + XR * ROWB + PAD;
  static constexpr int LDS = T_OFF + TR * ROWB + PAD;
  static_assert(W > 48 && W <= 64, "four 16-column tiles per row");
  static_assert(LDS <= 163840, "LDS budget");
};

template <int W>
__global__ __launch_bounds__(64 * BB_NW) void bblock_bf16_kernel(BneckArgs a) {
  using G = BbGeo<W>;
  constexpr int SP = G::SP, ROWB = G::ROWB;
  __shared__ __attribute__((aligned(16))) unsigned char smem[G::LDS];
  float* const b1s = (float*)(smem + G::B_OFF);
  float* const b2s = b1s + 64;
  unsigned char* const XR = smem + G::X_OFF;
  unsigned char* const TRg = smem + G::T_OFF;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  const int cw = w & 3;  // both convs: this wave's cout tile (couts 16 cw ..) and step row w >> 2
  // loads: this wave's pixel tile (row w >> 2, columns 16 (w & 3) + r); idle lanes (ox >= W) use
  // pixel SP, just past every step resource
  const int oy = w >> 2, ox = 16 * (w & 3) + r;
  const bool live = ox < W;
  const int poff = live ? oy * W + ox : SP;
  const int H = a.H;
  const int NS = H / 2 + 1;  // row pairs and the zero step
  const int GR = gridDim.x;
  const int nimg = (a.N - (int)blockIdx.x + GR - 1) / GR;  // this workgroup's images (grid <= N)
  const int total = nimg * NS;
  auto is_zero = [&](int g) { return g % NS == NS - 1; };
  auto step_res = [&](const void* base, int g) {
    const int img = (int)blockIdx.x + (g / NS) * GR;
    const int k = g - (g / NS) * NS;
    const long long p0 = ((long long)img * H + 2 * k) * W;
    return bb_rsrc((const u16*)base + p0 * 64, g < total && k < NS - 1 ? (long long)SP * 128 : 0);
  };

  // once per launch: shifts -> LDS, both rings zeroed (row -1 of the first image and every pad
  // slot), this wave's 16 couts x 576 K of both convs into registers
  for (int i = tid; i < 128; i += 64 * BB_NW) b1s[i] = i < 64 ? a.b1[i] : a.b2[i - 64];
  for (int i = tid; i < (G::LDS - G::X_OFF) / 16; i += 64 * BB_NW) *(v4u*)(XR + 16 * i) = v4u{0, 0, 0, 0};
  bf16x8 w1f[18], w2f[18];
  {
    const u16* w1 = (const u16*)a.w1 + (long long)(16 * cw + r) * 576 + 8 * q;
    const u16* w2 = (const u16*)a.w2 + (long long)(16 * cw + r) * 576 + 8 * q;
#pragma unroll
    for (int t = 0; t < 18; ++t) {
      w1f[t] = *(const bf16x8*)(w1 + (t >> 1) * 64 + 32 * (t & 1));
      w2f[t] = *(const bf16x8*)(w2 + (t >> 1) * 64 + 32 * (t & 1));
    }
  }

  typedef v4u XSet[2];  // the lane's input pixel: channels 32 s + 8q .. (s = 0, 1)
  auto load_x = [&](int g, XSet& X) {
    const __amdgpu_buffer_rsrc_t rx = step_res(a.x, g);
#pragma unroll
    for (int s = 0; s < 2; ++s) X[s] = __builtin_amdgcn_raw_buffer_load_b128(rx, (poff * 64 + 8 * q) * 2, 64 * s, 0);
  };
  // X rows of step g -> X ring rows 2g, 2g + 1 (& 7); zeros for a zero step (all threads: idle
  // columns included)
  auto put_x = [&](int g, const XSet& X) __attribute__((always_inline)) {
    if (is_zero(g)) {
      for (int i = tid; i < 2 * W * 8; i += 64 * BB_NW) {
        const int ry = i >= W * 8 ? 1 : 0, j = i - ry * W * 8;
        *(v4u*)(XR + ((2 * g + ry) & 7) * ROWB + 128 + 16 * j) = v4u{0, 0, 0, 0};
      }
      return;
    }
    if (live) {
      unsigned char* dst = XR + ((2 * g + oy) & 7) * ROWB + (ox + 1) * 128;
#pragma unroll
      for (int s = 0; s < 2; ++s) *(v4u*)(dst + (((4 * s + q) ^ ((ox + 1) & 7)) << 4)) = X[s];
    }
  };

  // 3x3 conv of step g, step row OY, this wave's cout tile, from a ring of RING rows (stream row R
  // at R mod RING): as conv_rows_bf16 / bneck_bf16's conv2.
  auto conv3x3 = [&](auto second, int g, auto oyc, f32x4(&acc)[4]) {
    constexpr bool C2 = decltype(second)::value;  // conv2: T ring, w2f; conv1: X ring, w1f
    constexpr int RING = C2 ? G::TR : G::XR;
    constexpr int OY = decltype(oyc)::value;
    const unsigned char* ring = C2 ? TRg : XR;
    int rowb[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) rowb[j] = __builtin_amdgcn_readfirstlane(((2 * g + OY + j - 1 + RING) % RING) * ROWB);
    // lane (q, r) of tile u reads slot 16u + r + dx, chunk q (^ 4 for the second half) swizzled by
    // the slot: (16u + r + dx) & 7 = (r + dx) & 7, so the per-lane part is one offset per dx and the
    // tile is a compile-time 2048 u.  Idle lanes (16u + r >= W) read past their row: ring pad.
    int e[3];
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) e[dx] = (r + dx) * 128 + ((q ^ ((r + dx) & 7)) << 4);
    auto rd = [&](int t2, bf16x8(&bf)[4]) __attribute__((always_inline)) {
      const int tap = t2 >> 1, dy = tap / 3, dx = tap - 3 * (tap / 3);
      const unsigned char* base = ring + rowb[dy] + ((t2 & 1) ? (e[dx] ^ 64) : e[dx]);
#pragma unroll
      for (int u = 0; u < 4; ++u) bf[u] = *(const bf16x8*)(base + 2048 * u);
    };
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    // B fragments double-buffered (as conv_rows_bf16): step t2 + 1's reads go out before step t2's
    // MFMAs, one lgkmcnt(0) after them
    bf16x8 bf[2][4];
    rd(0, bf[0]);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t2 = 0; t2 < 18; ++t2) {
      if (t2 + 1 < 18) rd(t2 + 1, bf[(t2 + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(C2 ? w2f[t2] : w1f[t2], bf[t2 & 1][u], acc[u], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // conv1 of step g -> T ring rows 2g, 2g + 1 (% 5); zeros for a zero step
  auto conv1_body = [&](int g, auto oyc) {
    constexpr int OY = decltype(oyc)::value;
    f32x4 acc[4];
    conv3x3(std::false_type{}, g, oyc, acc);
    const f32x4 bias = *(const f32x4*)(b1s + 16 * cw + 4 * q);
    unsigned char* trow = TRg + ((2 * g + OY) % 5) * ROWB;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (16 * u + r >= W) continue;
      const int s = 16 * u + r + 1;
      const uint2 pk = make_uint2(relu_bf2(acc[u].lo + bias.lo), relu_bf2(acc[u].hi + bias.hi));
      *(uint2*)(trow + s * 128 + (((2 * cw + (q >> 1)) ^ (s & 7)) << 4) + 8 * (q & 1)) = pk;
    }
  };
  auto conv1 = [&](int g) __attribute__((always_inline)) {
    if (is_zero(g)) {
      for (int i = tid; i < 2 * W * 8; i += 64 * BB_NW) {
        const int ry = i >= W * 8 ? 1 : 0, j = i - ry * W * 8;
        *(v4u*)(TRg + ((2 * g + ry) % 5) * ROWB + 128 + 16 * j) = v4u{0, 0, 0, 0};
      }
      return;
    }
    if (oy == 0)
      conv1_body(g, std::integral_constant<int, 0>{});
    else
      conv1_body(g, std::integral_constant<int, 1>{});
  };

  // conv2 of step g + the residual (X ring rows 2g, 2g + 1) -> y (8 B per lane and pixel tile;
  // idle lanes store past the step resource, zero steps into an empty one).  Only the MFMAs are
  // per step row; the epilogue and its stores are common code, so every wave issues the same store
  // sequence outside any branch (a branch around them made hipcc merge its wait state and drain
  // vmcnt(0) at the next step's start).
  auto conv2 = [&](int g) __attribute__((always_inline)) {
    f32x4 acc[4];
    if (oy == 0)
      conv3x3(std::true_type{}, g, std::integral_constant<int, 0>{}, acc);
    else
      conv3x3(std::true_type{}, g, std::integral_constant<int, 1>{}, acc);
    const __amdgpu_buffer_rsrc_t ry = step_res(a.y, g);
    const f32x4 bias = *(const f32x4*)(b2s + 16 * cw + 4 * q);
    const unsigned char* xrow = XR + ((2 * g + oy) & 7) * ROWB;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int col = 16 * u + r;
      const int s = (col < W ? col : W - 1) + 1;
      const uint2 rv = *(const uint2*)(xrow + s * 128 + (((2 * cw + (q >> 1)) ^ (s & 7)) << 4) + 8 * (q & 1));
      const uint2 pk = make_uint2(relu_bf2(acc[u].lo + bias.lo + bf2_f(rv.x)), relu_bf2(acc[u].hi + bias.hi + bf2_f(rv.y)));
      const int p = col < W ? oy * W + col : SP;
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, pk), ry,
                                            (p * 64 + 16 * cw + 4 * q) * 2, 0, 0);
    }
  };

  // Workgroup barrier for the LDS hand-offs (as bneck_bf16_kernel): the builtins are no compiler
  // memory barriers, so an empty asm with a memory clobber fences each side
  auto lds_barrier = [] {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // VMEM per wave and step, in issue order: step g + 3's 2 loads, then conv2's 4 stores
  constexpr int NST = 4;

  XSet S0, S1;
  load_x(0, S0);
  load_x(1, S1);
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): weights, shifts, the first two steps' rows
  __syncthreads();                     // rings zeroed, shifts visible
  put_x(0, S0);
  put_x(1, S1);
  load_x(2, S0);
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): X(2) (step 0's counted wait sees no stores before it)
  lds_barrier();
  conv1(0);
  // step g: X(g + 2) (in set A, loaded a step ago) -> ring, X(g + 3) -> set B (X(g + 1)'s, put a
  // step ago), conv1 of g + 1, conv2 of g.  Every step issues the same VMEM sequence (empty
  // resources past the end), so the counted wait below is the only one.
  auto step = [&](int g, XSet& A, XSet& B) __attribute__((always_inline)) {
    vm_wait<NST>();  // A has landed: younger are only step g - 1's stores
    put_x(g + 2, A);
    load_x(g + 3, B);
    lds_barrier();  // X rows of g + 2 in the ring; every wave's reads of T rows 2g - 3 .. done
    if (g + 1 < total) conv1(g + 1);
    lds_barrier();  // T rows of g + 1 written
    conv2(g);
  };
  for (int g = 0; g < total; g += 2) {
    step(g, S0, S1);
    if (g + 1 >= total) break;
    step(g + 1, S1, S0);
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the last stores (and empty prefetches) have left
}

// ---------------------------------------------------------------------------------------------
// Split-conv form (r06, bblock2): the same stream of two-row steps, but each wave runs ONE of the
// two convs for 32 couts (two 16-cout tiles) of one step row: waves 0-3 conv1, waves 4-7 conv2
// (a workgroup's waves fill the SIMDs cyclically, so every SIMD holds one of each).  Why: in
// bblock_bf16_kernel every wave reads each B fragment for ONE 16-cout tile, so per step the CU
// reads 1152 KiB of fragments from LDS -- 4608 LDS cycles at 256 B/clk, exactly the 4608 MFMA
// cycles per SIMD: the kernel is co-bound by the LDS and the MFMA pipe (MFMA-busy 0.54).  Here a
// fragment feeds two MFMAs (576 KiB per step), the weights of one conv (2 x 18 fragments, 144
// VGPRs) fit where both convs' 16-cout halves did, and the two convs run in the same phase on
// different steps, so one barrier per step instead of two:
//   phase g:  X rows of step g + 3 -> X ring (10 rows), step g + 4's loads go out
//             conv1 waves: conv1 of step g + 1 (X rows 2g + 1 .. 2g + 4) -> T ring (7 rows)
//             conv2 waves: conv2 of step g - 1 (T rows 2g - 3 .. 2g) + residual (X ring) -> y
//             | barrier |
// Ring rows written in phase g (X 2g + 6, 2g + 7; T 2g + 2, 2g + 3) take the slots of rows last
// read in phase g - 1.  Per accumulator the MFMAs are those of bblock_bf16_kernel in the same K
// order, and the epilogues are the same: bitwise equal.
template <int W>
struct Bb2Geo {
  static constexpr int SP = 2 * W;
  // ring rows of 66 slots at W 56 too: the idle lanes of the last pixel tile (columns W .. 63)
  // write zeros into slots W + 1 .. 64 (the right pad slot W + 1 must stay zero, and does), so no
  // lane needs its own branch or address clamp
  static constexpr int SLOTS = 66;
  static constexpr int ROWB = SLOTS * 128;
  static constexpr int XR = 10, TR = 7;      // ring rows
  static constexpr int PAD = 1024;
  static constexpr int X_OFF = 512;          // b1[64] b2[64] before it
  static constexpr int T_OFF = X_OFF + XR * ROWB + PAD;
  static constexpr int LDS = T_OFF + TR * ROWB + PAD;
  static_assert(W > 48 && W <= 64, "four 16-column tiles per row");
  static_assert(LDS <= 163840, "LDS budget");
};

// timing-only ablations of release variants (results wrong): 1 no MFMAs, 2 no fragment reads after
// the first, 4 no phase barriers
#ifndef EOSV_BB2_PRIO
#define EOSV_BB2_PRIO 0
#endif
#ifndef EOSV_BB2_LEAD
#define EOSV_BB2_LEAD 1
#endif
#ifndef EOSV_BB2_ABL
#define EOSV_BB2_ABL 0
#endif
template <int W>
__global__ __launch_bounds__(64 * BB_NW) void bblock2_bf16_kernel(BneckArgs a) {
  using G = Bb2Geo<W>;
  constexpr int SP = G::SP, ROWB = G::ROWB, XRN = G::XR, TRN = G::TR;
  __shared__ __attribute__((aligned(16))) unsigned char smem[G::LDS];
  float* const b1s = (float*)smem;
  float* const b2s = b1s + 64;
  unsigned char* const XR = smem + G::X_OFF;
  unsigned char* const TRg = smem + G::T_OFF;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  const int grp = w >> 2;         // 0: conv1 waves, 1: conv2 waves
  const int cy = (w >> 1) & 1;    // the conv's step row
  const int ch = w & 1;           // its cout half: tiles 2 ch, 2 ch + 1 (couts 32 ch ..)
  // loads (every wave, as bblock_bf16_kernel): pixel tile w & 3 of step row w >> 2
  const int oy = w >> 2, ox = 16 * (w & 3) + r;
  const int poff = ox < W ? oy * W + ox : SP;  // idle lanes: pixel SP, past every step resource
  const int H = a.H;
  const int NS = H / 2 + 1;
  const int GR = gridDim.x;
  const int nimg = (a.N - (int)blockIdx.x + GR - 1) / GR;
  const int total = nimg * NS;
  auto is_zero = [&](int g) { return g % NS == NS - 1; };
  auto step_res = [&](const void* base, int g) {
    const int img = (int)blockIdx.x + (g / NS) * GR;
    const int k = g - (g / NS) * NS;
    const long long p0 = ((long long)img * H + 2 * k) * W;
    return bb_rsrc((const u16*)base + p0 * 64, g >= 0 && g < total && k < NS - 1 ? (long long)SP * 128 : 0);
  };

  for (int i = tid; i < 128; i += 64 * BB_NW) b1s[i] = i < 64 ? a.b1[i] : a.b2[i - 64];
  for (int i = tid; i < (G::LDS - G::X_OFF) / 16; i += 64 * BB_NW) *(v4u*)(XR + 16 * i) = v4u{0, 0, 0, 0};
  // this wave's conv: 32 couts x 576 K (tile t: couts 16 (2 ch + t) + r)
  bf16x8 wf[2][18];
  {
    const u16* wsrc = (const u16*)(grp ? a.w2 : a.w1);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const u16* wr = wsrc + (long long)(16 * (2 * ch + t) + r) * 576 + 8 * q;
#pragma unroll
      for (int k = 0; k < 18; ++k) wf[t][k] = *(const bf16x8*)(wr + (k >> 1) * 64 + 32 * (k & 1));
    }
  }

  typedef v4u XSet[2];
  auto load_x = [&](int g, XSet& X) {
    const __amdgpu_buffer_rsrc_t rx = step_res(a.x, g);
#pragma unroll
    for (int s = 0; s < 2; ++s) X[s] = __builtin_amdgcn_raw_buffer_load_b128(rx, (poff * 64 + 8 * q) * 2, 64 * s, 0);
  };
  const int xlo = (ox + 1) * 128 + ((q ^ ((ox + 1) & 7)) << 4);
  auto put_x = [&](int g, const XSet& X) __attribute__((always_inline)) {
    if (is_zero(g)) {
      for (int i = tid; i < 2 * W * 8; i += 64 * BB_NW) {
        const int ry = i >= W * 8 ? 1 : 0, j = i - ry * W * 8;
        *(v4u*)(XR + ((2 * g + ry) % XRN) * ROWB + 128 + 16 * j) = v4u{0, 0, 0, 0};
      }
      return;
    }
    {  // idle lanes (ox >= W) loaded zeros past the step resource and write them.  The row base
      // is scalar, the lane part one VGPR (chunk 4 + q of the slot is chunk q's address ^ 64)
      const int o0 = __builtin_amdgcn_readfirstlane(((2 * g + oy) % XRN) * ROWB) + xlo;
      *(v4u*)(XR + o0) = X[0];
      *(v4u*)(XR + (o0 ^ 64)) = X[1];  // (XR and the rows are 128-B aligned)
    }
  };

  // 3x3 conv of step g, step row OY, this wave's two cout tiles: acc[t][u] (tile t, pixel tile u)
  auto conv3x3 = [&](auto second, int g, f32x4(&acc)[2][4]) {
    constexpr bool C2 = decltype(second)::value;
    constexpr int RING = C2 ? TRN : XRN;
    const int OY = cy;
    const unsigned char* ring = C2 ? TRg : XR;
    int rowb[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) rowb[j] = __builtin_amdgcn_readfirstlane(((2 * g + OY + j - 1 + 2 * RING) % RING) * ROWB);
    int e[3];
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) e[dx] = (r + dx) * 128 + ((q ^ ((r + dx) & 7)) << 4);
    auto rd = [&](int t2, bf16x8(&bf)[4]) __attribute__((always_inline)) {
      const int tap = t2 >> 1, dy = tap / 3, dx = tap - 3 * (tap / 3);
      const unsigned char* base = ring + rowb[dy] + ((t2 & 1) ? (e[dx] ^ 64) : e[dx]);
#pragma unroll
      for (int u = 0; u < 4; ++u) bf[u] = *(const bf16x8*)(base + 2048 * u);
    };
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 bf[2][4];
#if EOSV_BB2_LEAD
    // Fragment (t2 + 2, u) is read into the slot of (t2, u) right behind the two MFMAs that last read
    // it: every read has ~1.75 k-steps (7 reads) of lead, in the same 8 fragment registers, and hipcc
    // waits lgkmcnt(7) per pixel tile instead of lgkmcnt(0) per k-step (the skeleton of LDS latency
    // waits, 0.87 of the 1.42 ms per launch without MFMAs, no longer runs beside them but under them)
    auto rd1 = [&](int t2, int u) __attribute__((always_inline)) {
      const int tap = t2 >> 1, dy = tap / 3, dx = tap - 3 * (tap / 3);
      // the second channel half is the first's address ^ 64 (ring rows are 128-B aligned)
      const int a0 = rowb[dy] + e[dx];
      return *(const bf16x8*)(ring + ((t2 & 1) ? (a0 ^ 64) : a0) + 2048 * u);
    };
#pragma unroll
    for (int u = 0; u < 4; ++u) bf[0][u] = rd1(0, u);
#pragma unroll
    for (int u = 0; u < 4; ++u) bf[1][u] = rd1(1, u);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t2 = 0; t2 < 18; ++t2) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
          if constexpr (EOSV_BB2_ABL & 1) asm volatile("" ::"v"(bf[t2 & 1][u])); else  // (timing ablation)
          acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t][t2], bf[t2 & 1][u], acc[t][u], 0, 0, 0);
        if (t2 + 2 < 18) bf[t2 & 1][u] = rd1(t2 + 2, u);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        if (t2 + 2 < 18) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    return;
#endif
    rd(0, bf[0]);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t2 = 0; t2 < 18; ++t2) {
      if (t2 + 1 < 18 && !(EOSV_BB2_ABL & 2)) rd(t2 + 1, bf[(t2 + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if constexpr (EOSV_BB2_ABL & 1) asm volatile("" ::"v"(bf[t2 & 1][u])); else  // (timing ablation)
          acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t][t2], bf[t2 & 1][u], acc[t][u], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // conv1 of step g -> T ring rows 2g, 2g + 1 (% 7); a zero step writes zero rows (conv1 waves)
  auto conv1 = [&](int g) __attribute__((always_inline)) {
    if (is_zero(g)) {
      for (int i = tid; i < 2 * W * 8; i += 64 * 4) {
        const int ry = i >= W * 8 ? 1 : 0, j = i - ry * W * 8;
        *(v4u*)(TRg + ((2 * g + ry) % TRN) * ROWB + 128 + 16 * j) = v4u{0, 0, 0, 0};
      }
      return;
    }
    f32x4 acc[2][4];
    conv3x3(std::false_type{}, g, acc);
    unsigned char* trow = TRg + ((2 * g + cy) % TRN) * ROWB;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int cw = 2 * ch + t;
      const f32x4 bias = *(const f32x4*)(b1s + 16 * cw + 4 * q);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int s = 16 * u + r + 1;
        uint2 pk = make_uint2(relu_bf2(acc[t][u].lo + bias.lo), relu_bf2(acc[t][u].hi + bias.hi));
        if (16 * u + r >= W) pk = make_uint2(0u, 0u);  // idle column: a zero slot
        *(uint2*)(trow + s * 128 + (((2 * cw + (q >> 1)) ^ (s & 7)) << 4) + 8 * (q & 1)) = pk;
      }
    }
  };
  // conv2 of step g + the residual (X ring rows 2g, 2g + 1): the 8 packed results and their store
  // offsets (idle lanes: offsets past the step resource); the stores themselves are common code
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  auto conv2 = [&](int g, u32x2(&spk)[8], int(&svo)[8]) __attribute__((always_inline)) {
    f32x4 acc[2][4];
    conv3x3(std::true_type{}, g, acc);
    const unsigned char* xrow = XR + ((2 * g + cy + XRN) % XRN) * ROWB;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int cw = 2 * ch + t;
      const f32x4 bias = *(const f32x4*)(b2s + 16 * cw + 4 * q);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int col = 16 * u + r;
        const int s = col + 1;  // (idle columns: a zero slot, their store is dropped)
        const uint2 rv = *(const uint2*)(xrow + s * 128 + (((2 * cw + (q >> 1)) ^ (s & 7)) << 4) + 8 * (q & 1));
        spk[4 * t + u] = u32x2{relu_bf2(acc[t][u].lo + bias.lo + bf2_f(rv.x)),
                               relu_bf2(acc[t][u].hi + bias.hi + bf2_f(rv.y))};
        const int p = col < W ? cy * W + col : SP;
        svo[4 * t + u] = (p * 64 + 16 * cw + 4 * q) * 2;
      }
    }
  };

  auto lds_barrier = [] {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // prologue: steps 0-2 in the ring, step 3 in flight, conv1 of step 0.  One register set for the
  // X loads: a phase puts the set it waited for, then reloads it (the ring writes read their data at
  // issue, before any load can return into it)
  XSet S;
  load_x(0, S);
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): weights, shifts, step 0's rows
  __syncthreads();                     // rings zeroed, shifts visible
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    if (g) __builtin_amdgcn_s_waitcnt(0x0f70);
    put_x(g, S);
    load_x(g + 1, S);
  }
  lds_barrier();
  if (grp == 0) conv1(0);
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): X(3) too (phase 0's counted wait sees no stores before it)
  lds_barrier();
  // phase g: X(g + 3) (loaded in phase g - 1) -> ring, X(g + 4) into the same registers, then
  // conv1 of step g + 1 or conv2 of step g - 1.  VMEM per wave and phase in issue order: 2 loads,
  // then (conv2 waves) 8 stores -- also in phase 0, whose conv2 of step -1 stores into an empty
  // resource -- so the counted wait below is the only one.
  // Both groups issue the same 8 stores after the branch (the conv1 waves' into an empty resource,
  // dropped without memory traffic): one VMEM sequence per phase on every path, so hipcc's own wait
  // before the ring writes is the counted vmcnt(8) -- stores inside the conv2 branch gave it a path
  // without them, and a vmcnt(0) at the top of every phase (as bblock_bf16_kernel's note says)
  const __amdgpu_buffer_rsrc_t nowhere = bb_rsrc(a.y, 0);
  if constexpr (EOSV_BB2_PRIO == 1) {  // r06 A/B: the conv2 waves first at the SIMD's issue
    if (grp) __builtin_amdgcn_s_setprio(1);
  } else if constexpr (EOSV_BB2_PRIO == 2) {  // ... or the conv1 waves
    if (!grp) __builtin_amdgcn_s_setprio(1);
  }
  for (int g = 0; g <= total; ++g) {
    vm_wait<8>();  // S has landed: younger are only the previous phase's stores
    put_x(g + 3, S);
    load_x(g + 4, S);
    u32x2 spk[8];
    int svo[8];
    __amdgpu_buffer_rsrc_t srs = nowhere;
    if (grp == 0) {
      if (g + 1 < total) conv1(g + 1);
#pragma unroll
      for (int k = 0; k < 8; ++k) spk[k] = u32x2{0u, 0u}, svo[k] = 16 * k;
    } else {
      conv2(g - 1, spk, svo);
      srs = step_res(a.y, g - 1);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) __builtin_amdgcn_raw_buffer_store_b64(spk[k], srs, svo[k], 0, 0);
    if (!(EOSV_BB2_ABL & 4)) lds_barrier();
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the last stores (and empty prefetches) have left
}

bool bblock_bf16_ok(int W, int H) { return (W == 56 || W == 64) && H >= 2 && H % 2 == 0; }

#ifndef EOSV_BBLOCK2_DEF
#define EOSV_BBLOCK2_DEF 1
#endif

template <int W>
static int launch_bb(const BneckArgs& a, hipStream_t s) {
  if (a.plan) return record_launch(a.plan, a.N, 1);
  const int grid = std::min(a.N, device_cu_count());
  static const int v2 = env_switch("EOSV_BBLOCK2", EOSV_BBLOCK2_DEF);  // 0: the r06 one-wave-both-convs kernel (A/B)
  if (v2)
    hipLaunchKernelGGL((bblock2_bf16_kernel<W>), dim3(grid), dim3(64 * BB_NW), 0, s, a);
  else
    hipLaunchKernelGGL((bblock_bf16_kernel<W>), dim3(grid), dim3(64 * BB_NW), 0, s, a);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int launch_bblock_bf16(const BneckArgs& a, hipStream_t s) {
  if (a.N <= 0 || !bblock_bf16_ok(a.W, a.H) || a.cin != 64 || !a.x || !a.w1 || !a.b1 || !a.w2 || !a.b2 || !a.y)
    return set_error("bblock_bf16: unsupported shape"), EOSV_ERR_UNSUPPORTED;
  return a.W == 56 ? launch_bb<56>(a, s) : launch_bb<64>(a, s);
}

}  // namespace eosv
