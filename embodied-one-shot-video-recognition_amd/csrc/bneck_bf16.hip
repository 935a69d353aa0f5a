// Whole-bottleneck fusion for the bf16 ResNet stage 1 (r06): one persistent launch runs a block's
// conv1 (1x1 CIN -> 64) -> conv2 (3x3 64 -> 64) -> conv3 (1x1 64 -> 256, + residual or + the folded
// stride-1 downsample, ReLU), and optionally (NEXT) the following block's conv1 (1x1 256 -> 64) on
// the block output -- torchvision Bottleneck.forward, reached from the reference's
// models.py:33-37 (model_resnet50 .. self.convnet) via network_test.py:186-187, 202-203, 241.
//
// Why: stage 1 is HBM-bound.  Unfused (conv_rows_bf16 for the 3x3, pair1x1r_bf16 for conv3 + the
// next conv1) a residual block moves ~1.55 KB per pixel (its 64-channel maps T1 and T2 each written
// and read back); here T1 and T2 never leave the CU: the block reads its input once (512 B per
// pixel, 128 B for block 0) and writes its output (512 B, + 128 B for NEXT's Z).
//
// Shape of the work.  A workgroup (8 waves, two per SIMD, <= 256 VGPRs each; up to 155 KiB of
// LDS, so one per CU) walks whole images, two rows per step (a "step" = 2W pixels = 8 row-aligned
// pixel tiles of 16), as one continuous stream over its images:
//   step g:  conv1 of step g + 1 (input pixel fragments in registers, loaded two steps ahead)
//            -> T1 ring in LDS (5 rows of W + 2 slots; the two pad slots stay zero)
//            | barrier |
//            conv2 of step g: wave w one 16-cout tile (w & 3) of the 4 pixel tiles of row w >> 2,
//            its 18 weight fragments resident in registers, the B fragments read from the T1 ring
//            (rows outside the image read a zero pad slot) -> T2 (LDS)
//            | barrier |
//            conv3 of step g (+ NEXT): wave w its pixel tile w, W3 / Wn fragments from LDS,
//            residual = the same input fragments conv1 used (still in registers) -> Y (and Z)
// The input fragments rotate through three register sets (step g's residual, step g + 1's conv1
// input, step g + 2's loads in flight), so a step's HBM reads are issued a full step before use.
// At W 56 the last tile of each row has 8 idle lanes: their loads and stores fall outside the
// step's buffer resource (read 0 / dropped), so every wave issues the same VMEM count and the
// counted waits are compile-time.  Stores go through store_b128_guarded (common.h, a gfx950
// store-data hazard hipcc does not pad).
//
// Arithmetic: every conv keeps the unfused kernels' MFMA shape (v_mfma_f32_16x16x32_bf16,
// D = W . X^T), K order and epilogue order: conv1 as pair1x1r_bf16's GEMM2 (k-slices 0 .. CIN/32 - 1),
// conv2 as conv_rows_bf16 (18 k-steps: tap-major, two 32-channel slices per tap), conv3 as
// pair1x1r_bf16's GEMM1 (the folded downsample's slices after conv3's), NEXT as its GEMM2; each
// epilogue + shift (+ residual), ReLU, bf16.  So Y and Z are bitwise those of the unfused path
// (tests/test_gpu_poison.py: test_bneck_bitwise_equal_unfused).
#include <hip/hip_bf16.h>

#include <utility>

#include "common.h"

namespace eosv {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

__device__ __forceinline__ int swz(int row, int chunk) { return (chunk ^ (row & 7)) * 8; }
using epi::bf2_f;
using epi::f32x2;
using epi::pair_of;
using epi::relu_bf2;
// The 1x1 convs read their weight rows in pair1x1r_bf16's permuted order: MFMA tile i, row t (0..15)
// is channel permrow(i, t) = 32 (i >> 1) + 8 (t >> 2) + 4 (i & 1) + (t & 3) of a 64-channel group, so
// a lane ends up with channels 8q .. 8q + 7 (tiles 0, 1) and 32 + 8q .. + 7 (tiles 2, 3) of its
// pixel (see the lane-base form in the kernel).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(bytes > 0x7fffffffLL ? 0x7fffffffLL : (bytes < 0 ? 0 : bytes)),
                                           0x00020000);
}
}  // namespace

// conv2: 18 k-steps (tap-major, two 32-channel halves per tap) of one 16-cout tile over the four
// 16-pixel tiles of a step row, B fragments from the T1 ring (rowb: the three input rows' byte
// offsets).  Lane (q, r) of tile u reads slot 16u + r + dx, chunk q (^ 4 for the second half),
// swizzled by the slot: (16u + r + dx) & 7 = (r + dx) & 7, so the per-lane part is one offset per dx
// and the tile a compile-time 2048 u (idle lanes of W 56 read past their row: the next ring row or
// T2, harmless).  Fragments double-buffered: step t + 1's reads go out before step t's MFMAs, one
// lgkmcnt(0) after them (as conv_rows_bf16).
#ifndef EOSV_BNECK_LEAD
#define EOSV_BNECK_LEAD 0  // r06 A/B: bitwise equal, R50 neutral (profiles/r06aa_fragment_lead.txt)
#endif
__device__ __forceinline__ void conv2_ring(const unsigned char* T1, const int (&rowb)[3], int r, int q,
                                           const bf16x8 (&wf)[18], f32x4 (&acc)[4], bool skip) {
  int e[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) e[dx] = (r + dx) * 128 + ((q ^ ((r + dx) & 7)) << 4);
  auto rd = [&](int t2, bf16x8(&bf)[4]) __attribute__((always_inline)) {
    const int tap = t2 >> 1, dy = tap / 3, dx = tap - 3 * (tap / 3);
    const unsigned char* base = T1 + rowb[dy] + ((t2 & 1) ? (e[dx] ^ 64) : e[dx]);
#pragma unroll
    for (int u = 0; u < 4; ++u) bf[u] = *(const bf16x8*)(base + 2048 * u);
  };
#pragma unroll
  for (int u = 0; u < 4; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (skip) return;
  bf16x8 bf[2][4];
#if EOSV_BNECK_LEAD
  // r06: fragment (t2 + 2, u) is read into the slot of (t2, u) right behind the MFMA that last reads
  // it, so every read has 7 reads of lead and hipcc waits lgkmcnt(7) per MFMA instead of lgkmcnt(0)
  // per k-step (as bblock2_bf16_kernel; same registers, same MFMAs per accumulator in the same order)
  auto rd1 = [&](int t2, int u) __attribute__((always_inline)) {
    const int tap = t2 >> 1, dy = tap / 3, dx = tap - 3 * (tap / 3);
    return *(const bf16x8*)(T1 + rowb[dy] + ((t2 & 1) ? (e[dx] ^ 64) : e[dx]) + 2048 * u);
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
      acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t2], bf[t2 & 1][u], acc[u], 0, 0, 0);
      if (t2 + 2 < 18) bf[t2 & 1][u] = rd1(t2 + 2, u);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
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
    if (t2 + 1 < 18) rd(t2 + 1, bf[(t2 + 1) & 1]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t2], bf[t2 & 1][u], acc[u], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_sched_barrier(0);
  }
}

constexpr int BN_NW = 8;  // waves per workgroup (two per SIMD; <= 256 VGPRs each)

// Geometry of a step (two image rows): pixel tile t (0..7) is row t >> 2, columns 16 (t & 3) ..
// + 15 -- row-aligned, so no tile straddles the two rows; at W 56 the last tile of each row has 8
// valid columns (lanes r >= 8 of tiles 3 and 7 are idle: loads read 0, stores are dropped, LDS
// writes are skipped).
template <int W, int CIN, bool NEXT>
struct BnGeo {
  static constexpr bool DS = CIN == 64;       // block 0: conv3 carries the stride-1 downsample
  static constexpr int K3 = DS ? 128 : 64;     // conv3's K
  static constexpr int CS = CIN / 32;          // k-slices of an input pixel fragment set
  static constexpr int SP = 2 * W;             // pixels per step
  static constexpr int SLOTS = W + 2;          // T1 row: pad slot, W pixels, pad slot
  static constexpr int ROWB = SLOTS * 128;     // bytes per T1 row (64 bf16 per slot)
  // LDS byte offsets
  static constexpr int W1_OFF = 0;
  static constexpr int W3_OFF = W1_OFF + 64 * CIN * 2;
  static constexpr int WN_OFF = W3_OFF + 256 * K3 * 2;
  static constexpr int B_OFF = WN_OFF + (NEXT ? 64 * 256 * 2 : 0);  // b1[64] b2[64] b3[256] bn[64]
  static constexpr int T1_OFF = B_OFF + 448 * 4;
  static constexpr int T2_OFF = T1_OFF + 5 * ROWB;
  static constexpr int LDS = T2_OFF + SP * 128;
  static_assert(W > 48 && W <= 64, "four 16-column tiles per row");
  static_assert(LDS <= 163840, "LDS budget");
};

template <int W, int CIN, bool NEXT>
__global__ __launch_bounds__(64 * BN_NW) void bneck_bf16_kernel(BneckArgs a) {
  using G = BnGeo<W, CIN, NEXT>;
  constexpr bool DS = G::DS;
  constexpr int K3 = G::K3, CS = G::CS, SP = G::SP, ROWB = G::ROWB;
  __shared__ __attribute__((aligned(16))) unsigned char smem[G::LDS];
  u16* const W1s = (u16*)(smem + G::W1_OFF);
  u16* const W3s = (u16*)(smem + G::W3_OFF);
  u16* const Wns = (u16*)(smem + G::WN_OFF);
  float* const b1s = (float*)(smem + G::B_OFF);
  float* const b2s = b1s + 64;
  float* const b3s = b2s + 64;
  float* const bns = b3s + 256;
  unsigned char* const T1 = smem + G::T1_OFF;
  unsigned char* const T2 = smem + G::T2_OFF;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  // A-fragment reads of the resident 1x1 weights: row permrow(i, r) (+ 64 ch), 16-B chunk c stored at
  // c ^ (row & 7) = c ^ (4 (i & 1) + (r & 3)), which for c = 4s + q is 4 (s ^ (i & 1)) + (q ^ (r & 3)):
  // one per-lane byte offset per matrix plus a compile-time immediate per (i, s, ch)
  const int rl = 8 * (r >> 2) + (r & 3);  // the lane's part of permrow
  const int ql = (q ^ (r & 3)) << 4;      // the lane's part of the chunk swizzle
  // the 1x1 phases: this wave's pixel tile t = w, the lane's pixel (oy, ox), step pixel pp; idle
  // lanes (ox >= W) get an offset beyond every step resource
  const int oy = w >> 2, ox = 16 * (w & 3) + r;
  const bool live = ox < W;
  const int pp = oy * W + ox;
  // pixel index for global offsets: idle lanes use pixel SP, just past every step resource (a far
  // larger index overflowed the 32-bit byte offset at 256 channels and wrapped into the step)
  const int poff = live ? pp : SP;
  const int pt2 = live ? pp : 0;            // pixel index for T2 reads (idle: any valid pixel)
  const int H = a.H;
  // profiling-build ablations (EOSV_BNECK_ABL; results wrong): 1 no conv1 MFMAs, 2 no conv2, 4 no
  // conv3 / NEXT, 8 loads from empty resources (no HBM reads), 16 stores dropped, 32 no barriers
  const int abl = EOSV_ABL(a);
  // steps per image: H / 2 row pairs and a zero step, whose conv1 writes two zero rows into the T1
  // ring (the bottom pad row of this image and the top one of the next); a zero step runs the
  // other phases on empty resources (below)
  const int NS = H / 2 + 1;
  const int GR = gridDim.x;
  const int nimg = (a.N - (int)blockIdx.x + GR - 1) / GR;  // this workgroup's images (grid <= N)
  const int total = nimg * NS;                             // its stream steps
  auto is_zero = [&](int g) { return g % NS == NS - 1; };

  // ---- once per launch: weights and shifts -> LDS (16-B chunks of a row swizzled by the row),
  // the T1 ring zeroed (row -1 of the first image and every pad slot), this wave's 16 conv2 couts
  // x 576 K into registers
  {
    const u16* w1 = (const u16*)a.w1;
    for (int idx = tid; idx < 64 * (CIN / 8); idx += 64 * BN_NW) {
      const int row = idx / (CIN / 8), c = idx - row * (CIN / 8);
      *(v4u*)(W1s + row * CIN + swz(row, c)) = *(const v4u*)(w1 + (long long)row * CIN + c * 8);
    }
    const u16* w3 = (const u16*)a.w3;
    for (int idx = tid; idx < 256 * (K3 / 8); idx += 64 * BN_NW) {
      const int row = idx / (K3 / 8), c = idx - row * (K3 / 8);
      *(v4u*)(W3s + row * K3 + swz(row, c)) = *(const v4u*)(w3 + (long long)row * K3 + c * 8);
    }
    if constexpr (NEXT) {
      const u16* wn = (const u16*)a.wn;
      for (int idx = tid; idx < 64 * 32; idx += 64 * BN_NW) {
        const int row = idx >> 5, c = idx & 31;
        *(v4u*)(Wns + row * 256 + swz(row, c)) = *(const v4u*)(wn + (long long)row * 256 + c * 8);
      }
    }
    for (int i = tid; i < 448; i += 64 * BN_NW) {
      float v = 0.f;
      if (i < 64) v = a.b1[i];
      else if (i < 128) v = a.b2[i - 64];
      else if (i < 384) v = a.b3[i - 128];
      else if (NEXT) v = a.bn[i - 384];
      b1s[i] = v;
    }
    for (int i = tid; i < 5 * ROWB / 16; i += 64 * BN_NW) *(v4u*)(T1 + 16 * i) = v4u{0, 0, 0, 0};
  }
  const int cw = w & 3;  // conv2: this wave's cout tile (couts 16 cw ..) and pixel row w >> 2
  bf16x8 w2f[18];  // A fragments of conv2: couts 16 cw + r, k-step t = (tap t / 2, 32-channel half t & 1)
  {
    const u16* w2 = (const u16*)a.w2 + (long long)(16 * cw + r) * 576 + 8 * q;
#pragma unroll
    for (int t = 0; t < 18; ++t) w2f[t] = *(const bf16x8*)(w2 + (t >> 1) * 64 + 32 * (t & 1));
  }

  // stream step g's pixels of a [N][H][W][C] tensor: the buffer resource of its 2W pixels (an empty
  // one for a zero step or past this workgroup's last step: loads read 0, stores are dropped)
  auto step_res = [&](const void* base, int C, int g, bool off = false) {
    const int img = (int)blockIdx.x + (g / NS) * GR;
    const int k = g - (g / NS) * NS;
    const long long p0 = ((long long)img * H + 2 * k) * W;
    return rsrc((const u16*)base + p0 * C, g < total && k < NS - 1 && !off ? (long long)SP * C * 2 : 0);
  };
  // input fragments of step g: the wave's tile (k-slice s: channels 32 s + 8q .. of the lane's pixel)
  typedef v4u FragSet[CS];
  auto load_set = [&](int g, FragSet& L) {
    const __amdgpu_buffer_rsrc_t rx = step_res(a.x, CIN, g, abl & 8);
#pragma unroll
    for (int s = 0; s < CS; ++s) L[s] = __builtin_amdgcn_raw_buffer_load_b128(rx, (poff * CIN + 8 * q) * 2, 64 * s, 0);
  };

  // conv1 of stream step g (its fragments L) -> T1 ring rows 2g, 2g + 1 (mod 5); zeros for a zero step
  auto conv1 = [&](int g, const FragSet& L) {
    if (is_zero(g)) {
      for (int i = tid; i < 2 * W * 8; i += 64 * BN_NW) {  // the two rows' W pixel slots (the pad slots stay zero)
        const int ry = i >= W * 8 ? 1 : 0, j = i - ry * W * 8;
        *(v4u*)(T1 + ((2 * g + ry) % 5) * ROWB + 128 + 16 * j) = v4u{0, 0, 0, 0};
      }
      return;
    }
    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < CS; ++s) {
      if (abl & 1) break;
      bf16x8 af[4];
      {
        int lb = G::W1_OFF + rl * CIN * 2 + ql;
        asm volatile("" : "+v"(lb));  // one base per read group: hipcc would keep every (i, s) address live
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[i] = *(const bf16x8*)(smem + lb + (32 * (i >> 1) + 4 * (i & 1)) * CIN * 2 + 64 * (s ^ (i & 1)));
      }
      const bf16x8 bx = __builtin_bit_cast(bf16x8, L[s]);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bx, acc[i], 0, 0, 0);
    }
    if (live) {
      unsigned char* dst = T1 + ((2 * g + oy) % 5) * ROWB + (ox + 1) * 128;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int c0 = 32 * hh + 8 * q;
        const f32x4 bA = *(const f32x4*)(b1s + c0), bB = *(const f32x4*)(b1s + c0 + 4);
        v4u pk;
#pragma unroll
        for (int k = 0; k < 4; ++k) pk[k] = relu_bf2(pair_of(acc[2 * hh], acc[2 * hh + 1], k) + pair_of(bA, bB, k));
        *(v4u*)(dst + (((4 * hh + q) ^ ((ox + 1) & 7)) << 4)) = pk;
      }
    }
  };

  // conv2 of stream step g: wave w's 16 couts (cout tile cw) of the four pixel tiles of step row
  // w >> 2 -> T2.  Stream row R = 2g + oy + dy - 1 lives in T1 ring row R mod 5 (the zero step
  // between images makes rows -1 and H zero rows).  Idle lanes read column W - 1, write nothing.
  auto conv2_body = [&](int g, auto oyc) {
    constexpr int OY = decltype(oyc)::value;  // the step row, compile-time (two instances)
    int rowb[3];  // byte offsets of T1 ring rows 2g + OY - 1 .. + 1 (wave-uniform)
#pragma unroll
    for (int j = 0; j < 3; ++j) rowb[j] = __builtin_amdgcn_readfirstlane(((2 * g + OY + j + 4) % 5) * ROWB);
    f32x4 acc[4];
    conv2_ring(T1, rowb, r, q, w2f, acc, abl & 2);
    // epilogue: couts 16 cw + 4q .. + 3 of column 16u + r: + shift, ReLU, bf16 -> T2 (8 B, chunk
    // 2 cw + q / 2 of the pixel's 8, swizzled by the pixel)
    const f32x4 bias = *(const f32x4*)(b2s + 16 * cw + 4 * q);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (16 * u + r >= W) continue;
      const int p = OY * W + 16 * u + r;
      const uint2 pk = make_uint2(relu_bf2(acc[u].lo + bias.lo), relu_bf2(acc[u].hi + bias.hi));
      *(uint2*)(T2 + p * 128 + (((2 * cw + (q >> 1)) ^ (p & 7)) << 4) + 8 * (q & 1)) = pk;
    }
  };
  auto conv2 = [&](int g) {
    if (oy == 0)
      conv2_body(g, std::integral_constant<int, 0>{});
    else
      conv2_body(g, std::integral_constant<int, 1>{});
  };

  // conv3 of step g (+ NEXT) on the wave's pixel tile, L = step g's input fragments (the residual, or
  // the downsample's input) -> Y (and Z)
  auto conv3 = [&](int g, const FragSet& L) {
    const __amdgpu_buffer_rsrc_t ry = step_res(a.y, 256, g, abl & 16);
    const __amdgpu_buffer_rsrc_t rz = step_res(a.z, 64, g, abl & 16);
    f32x4 accn[4];
    if constexpr (NEXT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) accn[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int ch = 0; ch < 4; ++ch) {
      // T2 B fragments (read per chunk: not held across the chunks)
      bf16x8 t2f[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) t2f[s] = *(const bf16x8*)(T2 + pt2 * 128 + (((4 * s + q) ^ (pt2 & 7)) << 4));
      // per 32-channel half hh of the chunk: its two MFMA tiles (i = 2 hh, 2 hh + 1: channels
      // 64 ch + 32 hh + 8q ..), the epilogue, then the NEXT GEMM's k-slice (ch, hh) -- per
      // accumulator the order of pair1x1r_bf16
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int s = 0; s < K3 / 32; ++s) {
          if (abl & 4) break;
          bf16x8 af[2];
          {
            int lb = G::W3_OFF + rl * K3 * 2 + ql;
            asm volatile("" : "+v"(lb));
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const int i = 2 * hh + j;
              af[j] = *(const bf16x8*)(smem + lb + (64 * ch + 32 * (i >> 1) + 4 * (i & 1)) * K3 * 2 + 64 * (s ^ (i & 1)));
            }
          }
          const bf16x8 bx = s < 2 ? t2f[s & 1] : __builtin_bit_cast(bf16x8, L[s >= 2 ? s - 2 : 0]);
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[j], bx, acc[j], 0, 0, 0);
        }
        // epilogue: + shift (+ residual), ReLU, bf16 -> Y, and the NEXT GEMM's B fragment
        const int c0 = 64 * ch + 32 * hh + 8 * q;
        const f32x4 bA = *(const f32x4*)(b3s + c0), bB = *(const f32x4*)(b3s + c0 + 4);
        const v4u rv = DS ? v4u{0, 0, 0, 0} : L[2 * ch + hh];
        v4u pk;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          f32x2 v = pair_of(acc[0], acc[1], k) + pair_of(bA, bB, k);
          if constexpr (!DS) v += bf2_f(rv[k]);
          pk[k] = relu_bf2(v);
        }
        store_b128_guarded(pk, ry, (poff * 256 + 8 * q) * 2, (ch * 64 + 32 * hh) * 2);
        if (NEXT && !(abl & 4)) {
          const bf16x8 yf = __builtin_bit_cast(bf16x8, pk);
          bf16x8 aw[4];
          {
            int lb = G::WN_OFF + rl * 512 + ql;
            asm volatile("" : "+v"(lb));
#pragma unroll
            for (int i = 0; i < 4; ++i)
              aw[i] = *(const bf16x8*)(smem + lb + (32 * (i >> 1) + 4 * (i & 1)) * 512 + 16 * (8 * ch + 4 * (hh ^ (i & 1))));
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) accn[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[i], yf, accn[i], 0, 0, 0);
        }
      }
    }
    if constexpr (NEXT) {  // + shift, ReLU, bf16 -> Z
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int c0 = 32 * hh + 8 * q;
        const f32x4 bA = *(const f32x4*)(bns + c0), bB = *(const f32x4*)(bns + c0 + 4);
        v4u pk;
#pragma unroll
        for (int k = 0; k < 4; ++k) pk[k] = relu_bf2(pair_of(accn[2 * hh], accn[2 * hh + 1], k) + pair_of(bA, bB, k));
        store_b128_guarded(pk, rz, (poff * 64 + 8 * q) * 2, 32 * hh * 2);
      }
    }
  };

  // Workgroup barrier for the LDS hand-offs: neither s_waitcnt nor s_barrier (as builtins) is a
  // compiler-level memory barrier -- hipcc may sink an LDS store below both (r06: a T2 store landed
  // after the barrier at W 64, a race that changed 14 of 37 images) -- so an empty asm with a
  // memory clobber fences each side.  lgkmcnt(0): this wave's LDS reads and writes have completed.
  auto lds_barrier = [&] {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xc07f);
    if (!(abl & 32)) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // VMEM instructions per wave and step: NL loads (one fragment set), NST stores (Y, and Z)
  constexpr int NL = CS;
  constexpr int NST = 8 + (NEXT ? 2 : 0);
  static_assert(NL + NST < 64, "vmcnt range");

  FragSet L0, L1, L2;
  load_set(0, L0);
  load_set(1, L1);
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): weights, shifts, conv2 fragments, the first two sets
  __syncthreads();                     // LDS weights and the zeroed ring visible
  conv1(0, L0);

  // one stream step: conv1 of g + 1 (set Ln), conv2 and conv3 of g (set Lc); set Lf (step g - 1's,
  // dead since conv3 of g - 1) receives step g + 2's loads right after conv1, whose temporaries use
  // its registers meanwhile.  A zero step runs conv2 and conv3 too, on its empty resources (stores
  // dropped): every step then issues the same VMEM sequence, so hipcc's own wait analysis agrees
  // with the counted wait below and adds none (with a branch around them it merged the paths and
  // waited for the previous step's stores).  Branches are workgroup-uniform.
  auto step = [&](int g, FragSet& Lc, FragSet& Ln, FragSet& Lf) {
    // Ln (issued a step ago, after that step's conv1) has landed: younger are only step g - 1's
    // stores (at g = 0 none: the prologue drained)
    vm_wait<NST>();
    if (g + 1 < total) conv1(g + 1, Ln);
    load_set(g + 2, Lf);
    lds_barrier();  // T1 rows of g + 1 written (and every wave's reads of T2 done)
    conv2(g);
    lds_barrier();  // T2 written (and every wave's reads of T1 rows 2g - 1 .. done)
    conv3(g, Lc);
  };
  // three steps per iteration, so that every fragment set has a compile-time register home
  for (int g = 0; g < total; g += 3) {
    step(g, L0, L1, L2);
    if (g + 1 >= total) break;
    step(g + 1, L1, L2, L0);
    if (g + 2 >= total) break;
    step(g + 2, L2, L0, L1);
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the last stores (and empty prefetches) have left
}

// ---------------------------------------------------------------------------------------------
// The stage's last block (r06, "tail"): its conv1 output Z (64 channels) was written by the previous
// block's launch (NEXT), and its output feeds the next stage's block 0, whose conv1 (1x1 256 -> 128)
// runs here too -- the r05 path's conv_rows_bf16 + pair1x1r_bf16<128> in one launch, without the
// conv2 output's HBM round trip (1664 -> 1408 B per pixel).  Same stream of two-row steps as
// bneck_bf16_kernel; per step g: the Z rows of step g + 1 (register fragments, two steps ahead) ->
// T1 ring | barrier | conv2 -> T2 | barrier | conv3 + residual (loaded at the step's start: the
// residual is needed only once, at the end of the same step) -> Y, and the next conv1 -> Z'.
// Bitwise equal to the r05 path (conv2 as conv_rows_bf16, conv3 and the next conv1 as
// pair1x1r_bf16<128>'s GEMM1 / GEMM2, per accumulator in the same k order).
template <int W>
struct BtGeo {
  static constexpr int SP = 2 * W;
  static constexpr int SLOTS = W + 2;
  static constexpr int ROWB = SLOTS * 128;
  static constexpr int W3_OFF = 0;                        // [256][64]
  static constexpr int WN_OFF = W3_OFF + 256 * 64 * 2;    // [128][256]
  static constexpr int B_OFF = WN_OFF + 128 * 256 * 2;    // b2[64] b3[256] bn[128]
  static constexpr int T1_OFF = B_OFF + 448 * 4;
  static constexpr int T2_OFF = T1_OFF + 5 * ROWB;
  static constexpr int LDS = T2_OFF + SP * 128;
  static_assert(W > 48 && W <= 64, "four 16-column tiles per row");
  static_assert(LDS <= 163840, "LDS budget");
};

template <int W>
__global__ __launch_bounds__(64 * BN_NW) void bneck_tail_bf16_kernel(BneckArgs a) {
  using G = BtGeo<W>;
  constexpr int SP = G::SP, ROWB = G::ROWB;
  __shared__ __attribute__((aligned(16))) unsigned char smem[G::LDS];
  u16* const W3s = (u16*)(smem + G::W3_OFF);
  u16* const Wns = (u16*)(smem + G::WN_OFF);
  float* const b2s = (float*)(smem + G::B_OFF);
  float* const b3s = b2s + 64;
  float* const bns = b3s + 256;
  unsigned char* const T1 = smem + G::T1_OFF;
  unsigned char* const T2 = smem + G::T2_OFF;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  const int rl = 8 * (r >> 2) + (r & 3);  // the lane's part of permrow (bneck_bf16_kernel)
  const int ql = (q ^ (r & 3)) << 4;      // the lane's part of the chunk swizzle
  const int oy = w >> 2, ox = 16 * (w & 3) + r;
  const bool live = ox < W;
  const int pp = oy * W + ox;
  const int poff = live ? pp : SP;  // idle lanes: just past every step resource
  const int pt2 = live ? pp : 0;
  const int H = a.H;
  const int NS = H / 2 + 1;  // row pairs and the zero step
  const int GR = gridDim.x;
  const int nimg = (a.N - (int)blockIdx.x + GR - 1) / GR;
  const int total = nimg * NS;
  auto is_zero = [&](int g) { return g % NS == NS - 1; };

  {
    const u16* w3 = (const u16*)a.w3;
    for (int idx = tid; idx < 256 * 8; idx += 64 * BN_NW) {
      const int row = idx >> 3, c = idx & 7;
      *(v4u*)(W3s + row * 64 + swz(row, c)) = *(const v4u*)(w3 + (long long)row * 64 + c * 8);
    }
    const u16* wn = (const u16*)a.wn;
    for (int idx = tid; idx < 128 * 32; idx += 64 * BN_NW) {
      const int row = idx >> 5, c = idx & 31;
      *(v4u*)(Wns + row * 256 + swz(row, c)) = *(const v4u*)(wn + (long long)row * 256 + c * 8);
    }
    for (int i = tid; i < 448; i += 64 * BN_NW) b2s[i] = i < 64 ? a.b2[i] : i < 320 ? a.b3[i - 64] : a.bn[i - 320];
    for (int i = tid; i < 5 * ROWB / 16; i += 64 * BN_NW) *(v4u*)(T1 + 16 * i) = v4u{0, 0, 0, 0};
  }
  const int cw = w & 3;
  bf16x8 w2f[18];
  {
    const u16* w2 = (const u16*)a.w2 + (long long)(16 * cw + r) * 576 + 8 * q;
#pragma unroll
    for (int t = 0; t < 18; ++t) w2f[t] = *(const bf16x8*)(w2 + (t >> 1) * 64 + 32 * (t & 1));
  }

  auto step_res = [&](const void* base, int C, int g) {
    const int img = (int)blockIdx.x + (g / NS) * GR;
    const int k = g - (g / NS) * NS;
    const long long p0 = ((long long)img * H + 2 * k) * W;
    return rsrc((const u16*)base + p0 * C, g < total && k < NS - 1 ? (long long)SP * C * 2 : 0);
  };
  typedef v4u ZSet[2];  // the lane's Z pixel: channels 32 s + 8q .. (s = 0, 1)
  auto load_z = [&](int g, ZSet& Z) {
    const __amdgpu_buffer_rsrc_t rx = step_res(a.x, 64, g);
#pragma unroll
    for (int s = 0; s < 2; ++s) Z[s] = __builtin_amdgcn_raw_buffer_load_b128(rx, (poff * 64 + 8 * q) * 2, 64 * s, 0);
  };
  // Z of stream step g -> T1 ring rows 2g, 2g + 1; zeros for a zero step (its Z reads returned 0,
  // but every lane of the rows must be written, idle columns included: all threads write them)
  auto put_z = [&](int g, const ZSet& Z) {
    if (is_zero(g)) {
      for (int i = tid; i < 2 * W * 8; i += 64 * BN_NW) {
        const int ry = i >= W * 8 ? 1 : 0, j = i - ry * W * 8;
        *(v4u*)(T1 + ((2 * g + ry) % 5) * ROWB + 128 + 16 * j) = v4u{0, 0, 0, 0};
      }
      return;
    }
    if (live) {
      unsigned char* dst = T1 + ((2 * g + oy) % 5) * ROWB + (ox + 1) * 128;
#pragma unroll
      for (int s = 0; s < 2; ++s) *(v4u*)(dst + (((4 * s + q) ^ ((ox + 1) & 7)) << 4)) = Z[s];
    }
  };

  auto conv2_body = [&](int g, auto oyc) {  // as bneck_bf16_kernel
    constexpr int OY = decltype(oyc)::value;
    int rowb[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) rowb[j] = __builtin_amdgcn_readfirstlane(((2 * g + OY + j + 4) % 5) * ROWB);
    f32x4 acc[4];
    conv2_ring(T1, rowb, r, q, w2f, acc, false);
    const f32x4 bias = *(const f32x4*)(b2s + 16 * cw + 4 * q);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (16 * u + r >= W) continue;
      const int p = OY * W + 16 * u + r;
      const uint2 pk = make_uint2(relu_bf2(acc[u].lo + bias.lo), relu_bf2(acc[u].hi + bias.hi));
      *(uint2*)(T2 + p * 128 + (((2 * cw + (q >> 1)) ^ (p & 7)) << 4) + 8 * (q & 1)) = pk;
    }
  };
  auto conv2 = [&](int g) {
    if (oy == 0)
      conv2_body(g, std::integral_constant<int, 0>{});
    else
      conv2_body(g, std::integral_constant<int, 1>{});
  };

  // conv3 + residual -> Y, and the next stage's conv1 (two 64-cout groups) -> Z'
  auto conv3 = [&](int g, const v4u (&R)[8]) {
    const __amdgpu_buffer_rsrc_t ry = step_res(a.y, 256, g);
    const __amdgpu_buffer_rsrc_t rz = step_res(a.z, 128, g);
    f32x4 accn[2][4];
#pragma unroll
    for (int g2 = 0; g2 < 2; ++g2)
#pragma unroll
      for (int i = 0; i < 4; ++i) accn[g2][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < 4; ++ch) {
      bf16x8 t2f[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) t2f[s] = *(const bf16x8*)(T2 + pt2 * 128 + (((4 * s + q) ^ (pt2 & 7)) << 4));
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 af[2];
          {
            int lb = G::W3_OFF + rl * 128 + ql;
            asm volatile("" : "+v"(lb));
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const int i = 2 * hh + j;
              af[j] = *(const bf16x8*)(smem + lb + (64 * ch + 32 * (i >> 1) + 4 * (i & 1)) * 128 + 64 * (s ^ (i & 1)));
            }
          }
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[j], t2f[s], acc[j], 0, 0, 0);
        }
        const int c0 = 64 * ch + 32 * hh + 8 * q;
        const f32x4 bA = *(const f32x4*)(b3s + c0), bB = *(const f32x4*)(b3s + c0 + 4);
        const v4u rv = R[2 * ch + hh];
        v4u pk;
#pragma unroll
        for (int k = 0; k < 4; ++k) pk[k] = relu_bf2(pair_of(acc[0], acc[1], k) + pair_of(bA, bB, k) + bf2_f(rv[k]));
        store_b128_guarded(pk, ry, (poff * 256 + 8 * q) * 2, (ch * 64 + 32 * hh) * 2);
        const bf16x8 yf = __builtin_bit_cast(bf16x8, pk);
#pragma unroll
        for (int g2 = 0; g2 < 2; ++g2) {
          bf16x8 aw[4];
          {
            int lb = G::WN_OFF + rl * 512 + ql;
            asm volatile("" : "+v"(lb));
#pragma unroll
            for (int i = 0; i < 4; ++i)
              aw[i] = *(const bf16x8*)(smem + lb + (64 * g2 + 32 * (i >> 1) + 4 * (i & 1)) * 512 + 16 * (8 * ch + 4 * (hh ^ (i & 1))));
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) accn[g2][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[i], yf, accn[g2][i], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int g2 = 0; g2 < 2; ++g2)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int c0 = 64 * g2 + 32 * hh + 8 * q;
        const f32x4 bA = *(const f32x4*)(bns + c0), bB = *(const f32x4*)(bns + c0 + 4);
        v4u pk;
#pragma unroll
        for (int k = 0; k < 4; ++k) pk[k] = relu_bf2(pair_of(accn[g2][2 * hh], accn[g2][2 * hh + 1], k) + pair_of(bA, bB, k));
        store_b128_guarded(pk, rz, (poff * 128 + 8 * q) * 2, (64 * g2 + 32 * hh) * 2);
      }
  };

  auto lds_barrier = [] {  // as bneck_bf16_kernel
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // VMEM per wave and step, in issue order: the residual (8 loads), Z of g + 2 (2), Y (8) and Z' (4) stores
  constexpr int NZ = 2, NST = 8 + 4;
  ZSet Z0, Z1, Z2;
  load_z(0, Z0);
  load_z(1, Z1);
  __builtin_amdgcn_s_waitcnt(0x0f70);
  __syncthreads();
  put_z(0, Z0);
  auto step = [&](int g, ZSet& Zn, ZSet& Zf) {
    vm_wait<NST>();  // Zn (issued a step ago, before that step's stores) has landed
    if (g + 1 < total) put_z(g + 1, Zn);
    v4u R[8];  // the residual of step g, consumed at this step's end
    {
      const __amdgpu_buffer_rsrc_t rr = step_res(a.res, 256, g);
#pragma unroll
      for (int s = 0; s < 8; ++s) R[s] = __builtin_amdgcn_raw_buffer_load_b128(rr, (poff * 256 + 8 * q) * 2, 64 * s, 0);
    }
    load_z(g + 2, Zf);
    lds_barrier();
    conv2(g);
    lds_barrier();
    vm_wait<NZ>();  // the residual has landed (Zf's loads may still fly)
    conv3(g, R);
  };
  for (int g = 0; g < total; g += 3) {
    step(g, Z1, Z2);
    if (g + 1 >= total) break;
    step(g + 1, Z2, Z0);
    if (g + 2 >= total) break;
    step(g + 2, Z0, Z1);
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);
}

bool bneck_tail_bf16_ok(int W, int H) { return (W == 56 || W == 64) && H >= 2 && H % 2 == 0; }

template <int W>
static int launch_bt(const BneckArgs& a, hipStream_t s) {
  if (a.plan) return record_launch(a.plan, a.N, 1);
  const int grid = std::min(a.N, device_cu_count());
  hipLaunchKernelGGL((bneck_tail_bf16_kernel<W>), dim3(grid), dim3(64 * BN_NW), 0, s, a);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int launch_bneck_tail_bf16(const BneckArgs& a, hipStream_t s) {
  if (a.N <= 0 || !bneck_tail_bf16_ok(a.W, a.H) || a.cin != 64 || !a.x || !a.res || !a.w2 || !a.b2 || !a.w3 ||
      !a.b3 || !a.wn || !a.bn || !a.y || !a.z)
    return set_error("bneck_tail_bf16: unsupported shape"), EOSV_ERR_UNSUPPORTED;
  return a.W == 56 ? launch_bt<56>(a, s) : launch_bt<64>(a, s);
}

// the stage-1 block shapes this kernel takes: bf16 NHWC, 64 mid channels, 256 out, stride 1,
// 56- or 64-wide maps with an even height; CIN 64 (block 0, folded stride-1 downsample) or 256
bool bneck_bf16_ok(int cin, int W, int H, int next) {
  return (cin == 64 || cin == 256) && (W == 56 || W == 64) && H >= 2 && H % 2 == 0 && !(next && cin != 256);
}

template <int W, int CIN, bool NEXT>
static int launch_bn(const BneckArgs& a, hipStream_t s) {
  if (a.plan) return record_launch(a.plan, a.N, 1);  // persistent: one workgroup per CU walks images
  const int grid = std::min(a.N, device_cu_count());
  hipLaunchKernelGGL((bneck_bf16_kernel<W, CIN, NEXT>), dim3(grid), dim3(64 * BN_NW), 0, s, a);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int launch_bneck_bf16(const BneckArgs& a, hipStream_t s) {
  const bool next = a.wn != nullptr;
  if (a.N <= 0 || !bneck_bf16_ok(a.cin, a.W, a.H, next) || !a.x || !a.w1 || !a.b1 || !a.w2 || !a.b2 || !a.w3 ||
      !a.b3 || !a.y || (next && (!a.bn || !a.z)))
    return set_error("bneck_bf16: unsupported shape"), EOSV_ERR_UNSUPPORTED;
  BneckArgs b = a;
  b.abl = env_switch("EOSV_BNECK_ABL", 0);  // profiling build only (results wrong when set)
  if (b.cin == 64) return b.W == 56 ? launch_bn<56, 64, false>(b, s) : launch_bn<64, 64, false>(b, s);
  if (next) return b.W == 56 ? launch_bn<56, 256, true>(b, s) : launch_bn<64, 256, true>(b, s);
  return b.W == 56 ? launch_bn<56, 256, false>(b, s) : launch_bn<64, 256, false>(b, s);
}

}  // namespace eosv
