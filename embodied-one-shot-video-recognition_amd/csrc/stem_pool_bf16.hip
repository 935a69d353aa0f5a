// Fused ResNet stem for bf16: conv 7x7/2 p3 (3 -> 64, folded BN) + ReLU + maxpool 3x3/2 p1,
// torchvision's convnet.0-3 (reference models.py:19 via self.convnet).
//
// The unfused pair wrote the 112 x 112 x 64 stem map (1.6 MB per frame) to HBM and read it
// back for the pool; with K = 147 the stem itself is a short-K implicit GEMM that ran at
// ~280 TF/s.  Here one workgroup walks one image top to bottom:
//  * wave t owns pooled columns 7t .. 7t+6, i.e. the 16 stem columns 14t-1 .. 14t+14 (one
//    MFMA pixel tile; column 14t+14 is computed and dropped);
//  * all 64 x 192 folded stem weights live in registers (24 A fragments per lane), so the
//    k-loop only reads input pixels from LDS;
//  * per pooled row py the wave computes stem rows 2py and 2py+1 (row 2py-1 is kept from the
//    previous step), takes the row max and then the column max (DPP row shifts) of the raw
//    accumulators, and only then adds the BN shift, applies ReLU and rounds to bf16 for the
//    7 pooled pixels x 64 channels it stores (all three are monotone, so they commute with
//    max: the same values as stem conv -> bf16 -> maxpool up to f32 summation order).
//
// MFMA: v_mfma_f32_16x16x32_bf16 with D = W . X^T (rows = output channels, columns = stem
// pixels), K = [kh 8][24] (kw*3 + c, 21 real; kh 7 and the 3 spare k of each row carry zero
// weights), 6 k-slices of 32.  A B-fragment chunk (8 consecutive k of one kernel row) is 8
// consecutive bf16 of a padded input row starting at byte 12*sx + 16*c: only 4-B aligned,
// so LDS holds every input row 4 times, copy m shifted by 4m bytes so that the
// lanes with sx = m (mod 4) read it with an aligned ds_read_b128.
//
// LDS: a ring of 16 padded input rows x 4 copies (row r in slot (r + 3) & 15, so the 4 rows
// a step prefetches are contiguous); LDS-DMA from the dense padded RGB pack (4-B aligned
// sources).  Step py needs input rows 4py .. 4py+8 and prefetches 4py+9 .. 4py+12.
//
// DIRECT (default): no pack kernel.  The rows come straight from the caller's f32 NCHW frames:
// a step LDS-DMAs the 4 rows it prefetches as 12 f32 plane rows into a staging area (issued
// before the MFMAs), and after them a thread reads the R, G, B values of 2 padded columns from
// the staging, rounds them to bf16 and writes the 12 interleaved bytes into all 4 shifted
// copies (3 ds_write_b32 each); zero padding is written as zeros.  Saves the pack's 317 KB per
// frame write + read.  (Plain per-lane global loads of the same values instead of the staging
// DMA made the stem 45 % slower: 8-B lane stride, half-used lines.)
#include <hip/hip_bf16.h>

#include "common.h"

#include <type_traits>

namespace eosv {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

constexpr int MAX_TILES = 8;                         // pooled width <= 56 (input width <= 224): 2 waves/SIMD
constexpr int KSTEM = 192;                           // [kh 8][24]
constexpr int RING = 16;

__host__ __device__ constexpr int copy_chunks(int ntiles) {
  // bytes a copy must hold: 12 * (largest sx + 1) + 12 (shift) + 48 (3 chunks of a kernel row)
  return (12 * (14 * ntiles) + 12 + 48 + 15) / 16;
}
constexpr int LDS_BYTES = RING * 4 * copy_chunks(MAX_TILES) * 16;
constexpr int STG_ROW = 256;                          // f32 per staged plane row (W <= 256)
constexpr int STG_BYTES = 4 * 3 * STG_ROW * 4;        // DIRECT: 4 rows x 3 planes

__device__ __forceinline__ u16 f2bf(float f) { return __bfloat16_as_ushort(__float2bfloat16(f)); }

__device__ __forceinline__ void dma16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// value of the lane `sh` positions up within its 16-lane row (DPP row_shl); 0 past the row end
__device__ __forceinline__ float row_shl(float v, int sh) {
  const int iv = __float_as_int(v);
  const int r = sh == 1 ? __builtin_amdgcn_update_dpp(0, iv, 0x101, 0xf, 0xf, false)
                        : __builtin_amdgcn_update_dpp(0, iv, 0x102, 0xf, 0xf, false);
  return __int_as_float(r);
}
// value of the lane `sh` positions up within its 16-lane row; 0 past the row end (bound_ctrl),
// so the compiler can fold it into the consuming v_max_f32 as a DPP source
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
// (lo, hi) -> one v_cvt_pk_bf16_f32 (round to nearest even)
__device__ __forceinline__ unsigned pack_bf2(float lo, float hi) {
  const bf16x2v p = __builtin_convertvector((f32x2v){lo, hi}, bf16x2v);
  return __builtin_bit_cast(unsigned, p);
}

template <int SH>
__device__ __forceinline__ float shl_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x100 + SH, 0xf, 0xf, true));
}
}  // namespace

// x: padded bf16 RGB [N][H+6][Wp][3] (stem_row_pixels), w: [64][192] bf16, bias [64] f32,
// y: [N][Hq][Wq][64] bf16 (pooled).  Grid = N images, block = 64 * ntiles threads.
template <bool DIRECT>
__global__ __launch_bounds__(64 * MAX_TILES) void stem_pool_bf16_kernel(const u16* __restrict__ x,
                                                                       const float* __restrict__ fx,
                                                                       const u16* __restrict__ w,
                                                                       const float* __restrict__ bias, u16* y,
                                                                       int H, int W, int Hs, int Ws, int Hq, int Wq) {
  __shared__ __attribute__((aligned(16))) unsigned char ring[LDS_BYTES + (DIRECT ? STG_BYTES : 0)];
  float* stg = (float*)(ring + LDS_BYTES);  // DIRECT staging: [row 4][plane 3][STG_ROW]
  const int ntiles = blockDim.x >> 6;
  const int CH = copy_chunks(ntiles);  // 16-B chunks per copy
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int r16 = lane & 15;
  const int q = lane >> 4;
  const int img = blockIdx.x;
  const int Wp = stem_row_pixels(W, 3);
  const int rowbytes = Wp * 6;
  const int Hpad = H + 6;
  const unsigned char* ximg = DIRECT ? nullptr : (const unsigned char*)(x + (long long)img * Hpad * Wp * 3);
  const float* fimg = DIRECT ? fx + (long long)img * 3 * H * W : nullptr;
  // DIRECT: task = (padded row, column pair g); row bytes 12g .. 12g+11 = R G B of columns 2g, 2g+1
  const int GP = Wp / 2;  // column pairs per padded row (Wp is even)
  auto direct_load = [&](int prow, int g, float (&v)[6]) {
    const int yy = prow - 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int xx = 2 * g + h - 3;
      const bool ok = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
      const float* src = fimg + (ok ? (long long)yy * W + xx : 0);  // always a valid address
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float t = src[(long long)c * H * W];
        v[3 * h + c] = ok ? t : 0.f;
      }
    }
  };
  // DIRECT: 4 rows [r0, r0 + 4) x 3 planes -> staging (12 pieces of W floats, one per plane row)
  auto stage_f32 = [&](int r0) {
    for (int p = wid; p < 12; p += ntiles) {
      const int rr = p / 3, c = p - 3 * (p / 3);
      const int yy = min(max(r0 + rr - 3, 0), H - 1);  // out-of-image rows: zeroed at conversion
      if (4 * lane < W)
        dma16(fimg + ((long long)c * H + yy) * W + 4 * lane, stg + (rr * 3 + c) * STG_ROW);
    }
  };
  auto staged_load = [&](int prow, int rr, int g, float (&v)[6]) {
    const int yy = prow - 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int xx = 2 * g + h - 3;
      const bool ok = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
      const int xc = ok ? xx : 0;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float t = stg[(rr * 3 + c) * STG_ROW + xc];
        v[3 * h + c] = ok ? t : 0.f;
      }
    }
  };
  auto direct_store = [&](int prow, int g, const float (&v)[6]) {
    const unsigned d0 = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
    const unsigned d1 = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
    const unsigned d2 = (unsigned)f2bf(v[4]) | ((unsigned)f2bf(v[5]) << 16);
    unsigned char* slot = ring + (size_t)(((prow + 3) & (RING - 1)) * 4) * CH * 16;
#pragma unroll
    for (int m = 0; m < 4; ++m) {  // copy m holds the row shifted by 4m bytes
      unsigned* d = (unsigned*)(slot + (size_t)m * CH * 16 + 12 * g + 4 * m);
      d[0] = d0;
      d[1] = d1;
      d[2] = d2;
    }
  };

  // weights -> registers: A fragment (j, s) = couts j*16 + r16, k = 32s + 8q .. +7
  bf16x8 wf[4][6];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int s = 0; s < 6; ++s) wf[j][s] = *(const bf16x8*)(w + (j * 16 + r16) * KSTEM + 32 * s + 8 * q);
  f32x4 bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bv[j] = *(const f32x4*)(bias + j * 16 + 4 * q);

  // DMA of input rows [r0, r0 + nrows) (nrows * 4 copies * CH chunks, lane-linear from the
  // ring slot of r0); rows past the padded image are clamped (their results are discarded)
  auto stage = [&](int r0, int nrows) {
    const int total = nrows * 4 * CH;
    unsigned char* dst0 = ring + (size_t)(((r0 + 3) & (RING - 1)) * 4) * CH * 16;
    for (int p = wid; p * 64 < total; p += ntiles) {
      const int id = p * 64 + lane;
      const int rr = id / (4 * CH);
      const int rem = id - rr * 4 * CH;
      const int m = rem / CH;
      const int c = rem - m * CH;
      const int row = min(r0 + rr, Hpad - 1);
      const unsigned char* src = ximg + (long long)row * rowbytes + 16 * c - ((4 * m) & 15);
      if (id < total) dma16(src, dst0 + (size_t)p * 1024);  // EXEC-masked: no write past the region
    }
  };

  // this lane's stem column and its copy / byte offset inside a ring row
  const int sx = 14 * wid - 1 + r16;
  const int m = sx & 3;
  const bool colok = sx >= 0 && sx < Ws;
  // 16-B chunk index of this lane's pixel in its copy (12*sx + shift is a multiple of 16);
  // indexing whole chunks lets the compiler emit ds_read_b128 (a byte offset it cannot
  // prove aligned becomes 2 x ds_read2_b32)
  const int xchunk = m * CH + (12 * sx + ((4 * m) & 15)) / 16;

  auto stem_row = [&](int sy, f32x4 (&acc)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const int g = 4 * s + q;        // chunk of the [kh][24] K layout
      const int kh = min(g / 3, 6);   // kh 7: zero weights, any finite pixel
      const int c = g - 3 * (g / 3);
      const int slot = (2 * sy + kh + 3) & (RING - 1);
      const bf16x8 xf = ((const bf16x8*)ring)[slot * 4 * CH + xchunk + c];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][s], xf, acc[j], 0, 0, 0);
    }
  };
  // Per step a wave DMAs its share of 4 rows x 4 copies (pieces p = wid + ntiles*i of the
  // step's contiguous ring region); the chunk -> (row, source offset) map is fixed: precomputed.
  constexpr int PPW = 4;  // >= ceil(16 * CH / 64 / ntiles) for every ntiles <= MAX_TILES
  int prr[PPW], pcoff[PPW];
  const int step_chunks = 16 * CH;
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int id = (wid + ntiles * i) * 64 + lane;
    const int rr = id / (4 * CH);
    const int rem = id - rr * 4 * CH;
    const int mm = rem / CH;
    const int c = rem - mm * CH;
    prr[i] = id < step_chunks ? rr : -1;
    pcoff[i] = 16 * c - ((4 * mm) & 15);
  }
  auto stage4 = [&](int r0) {
    unsigned char* dst0 = ring + (size_t)(((r0 + 3) & (RING - 1)) * 4) * CH * 16;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int p = wid + ntiles * i;
      if (prr[i] >= 0) {  // EXEC-masked: no write past the region
        const int row = min(r0 + prr[i], Hpad - 1);
        dma16(ximg + (long long)row * rowbytes + pcoff[i], dst0 + (size_t)p * 1024);
      }
    }
  };

  if constexpr (DIRECT) {
    for (int t = tid; t < 13 * GP; t += blockDim.x) {
      float v[6];
      direct_load(t / GP, t % GP, v);
      direct_store(t / GP, t % GP, v);
    }
    __syncthreads();
  } else {
    stage(0, 13);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  // The pool runs on the raw accumulators: max over the window commutes with + shift, ReLU and
  // the bf16 rounding (all monotone), so only the 7 pooled values per channel get them.
  // Stem pixels outside the map enter as -inf (maxpool's padding).
  const float NEG = -INFINITY;
  f32x4 prev[4];  // stem row 2py - 1
#pragma unroll
  for (int j = 0; j < 4; ++j) prev[j] = f32x4{NEG, NEG, NEG, NEG};
  u16* yimg = y + (long long)img * Hq * Wq * 64;
  const int px = 7 * wid + (r16 >> 1);  // pooled column this lane writes (even r16 <= 12)
  const bool writer = !(r16 & 1) && r16 <= 12 && px < Wq;

  // DIRECT: this thread's task of the 4 rows a step prefetches (4 * GP tasks <= blockDim)
  const bool dtask = DIRECT && tid < 4 * GP;
  const int drow = tid / GP, dg = tid - (tid / GP) * GP;
  for (int py = 0; py < Hq; ++py) {
    if constexpr (DIRECT) {
      if (py + 1 < Hq) stage_f32(4 * py + 9);
    } else {
      if (py + 1 < Hq) stage4(4 * py + 9);
    }
    f32x4 a1[4], a2[4];
    stem_row(2 * py, a1);
    stem_row(2 * py + 1, a2);
    const bool ok1 = colok && 2 * py < Hs, ok2 = colok && 2 * py + 1 < Hs;
    // !DIRECT: the next step's rows (staged at this step's start) have landed before this step's
    // stores go out -- vmcnt(0) here rather than a count past the stores: a wave with no writer
    // lanes issues no stores at all, so the number of younger operations is not a constant.
    // (Loads, stores and LDS-DMA retire in issue order, MI355X_MICROARCH.md; r06 corrects the
    // earlier reason given here, that a store could retire ahead of an older load.)
    if constexpr (!DIRECT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned pk4[4][2];  // pooled bf16 pairs, stored after the DIRECT conversion
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      unsigned(&pk)[2] = pk4[j];
#pragma unroll
      for (int e2 = 0; e2 < 2; ++e2) {
        float o[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = 2 * e2 + h;
          const float v2 = ok2 ? a2[j][e] : NEG;
          const float v = fmaxf(fmaxf(prev[j][e], ok1 ? a1[j][e] : NEG), v2);  // row max
          prev[j][e] = v2;
          // column max: pooled column i of this tile = stem columns r16 = 2i, 2i+1, 2i+2
          const float c = fmaxf(fmaxf(v, row_shl(v, 1)), row_shl(v, 2));
          o[h] = fmaxf(c + bv[j][e], 0.f);
        }
        pk[e2] = (unsigned)f2bf(o[0]) | ((unsigned)f2bf(o[1]) << 16);
      }
      if (!DIRECT && writer)
        *(uint2*)(yimg + ((long long)py * Wq + px) * 64 + j * 16 + 4 * q) = make_uint2(pk[0], pk[1]);
    }
    if constexpr (DIRECT) {
      // staging landed (own DMA + barrier for the other waves'; the previous step's stores are
      // a whole step old), then convert the next step's rows into slots this step does not read
      if (py + 1 < Hq) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (dtask) {
          float dv[6];
          staged_load(4 * py + 9 + drow, drow, dg, dv);
          direct_store(4 * py + 9 + drow, dg, dv);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (writer) *(uint2*)(yimg + ((long long)py * Wq + px) * 64 + j * 16 + 4 * q) = make_uint2(pk4[j][0], pk4[j][1]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
      // every wave's next-step rows have landed (the wait above) and it is done reading the
      // slots the step after will overwrite
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// Column-blocked DIRECT variant (the default for W % 4 == 0): a workgroup of CB_TILES = 4 waves
// owns the pooled columns 28c .. 28c + 27 of one image (c = blockIdx.y), so two workgroups share
// a CU (54 KiB LDS, <= 256 VGPRs = 2 waves per SIMD).  That alone did not speed it up (r01g: the
// SIMDs were issue-bound, ~290 VALU instructions per wave-step against 48 MFMAs); the VALU-lean
// pool below did (1.56 -> 1.28 ms per 3200 frames).  No width limit: the
// column blocks tile any W (ResNet-101 at 256 x 256 too).
// Ring row of block c = padded-row bytes from 6 * pc0, pc0 = 28 * 4c - 2 (stem column 56c - 1
// is its first: the left edge of pooled column 28c's window); a lane's k = its stem column
// relative to that, + 1, so byte 12k of the row starts the lane's 7-pixel run, as before.
constexpr int CB_TILES = 4;
// 16-B chunks per ring copy: 51, not the 47 the row needs.  Lane k (stem column, k = 4a + m)
// reads chunk m * CB_CH + 3a + m (+ c): with CB_CH = 47 that is 48m + 3a + c, the same bank
// group for the 4 lanes of one a (SQ_LDS_BANK_CONFLICT at 40 % of the stem's CU cycles, r02);
// CB_CH + 1 = 52 = 4 (mod 16) spreads the 16 lanes of a row over all 16 bank groups.
constexpr int CB_CH = 51;
static_assert((CB_CH + 1) % 16 == 4 && CB_CH * 16 >= 168 * CB_TILES + 72, "conflict-free B-fragment reads");
constexpr int CB_GP = 14 * CB_TILES + 5;               // column pairs per ring row (61)
constexpr int CB_STG = 128;                             // f32 per staged plane row (32 lanes x 4)
constexpr int CB_LDS = RING * 4 * CB_CH * 16;
static_assert(12 * (CB_GP - 1) + 12 + 12 <= CB_CH * 16, "ring copy holds every pair at every shift");
static_assert(2 * (CB_GP - 1) + 1 + 3 < CB_STG, "staged row covers every pair");
static_assert(4 * CB_GP <= 64 * CB_TILES, "one conversion task per thread");

// AHEAD (r04): the f32 rows of step py + AHEAD are staged at step py.  With AHEAD 1 (r02) every
// step waited for the HBM round trip of the rows it had staged at its own start (a step's 48
// MFMAs per wave take ~0.7 us, less than that latency); AHEAD 2 stages into two buffers and
// waits for the rows staged a step earlier.
template <int AHEAD>
__global__ __launch_bounds__(64 * CB_TILES, 2) void stem_pool_bf16_cb_kernel(const float* __restrict__ fx,
                                                                        const u16* __restrict__ w,
                                                                        const float* __restrict__ bias, u16* y,
                                                                        int H, int W, int Hs, int Ws, int Hq, int Wq) {
  static_assert(AHEAD == 1 || AHEAD == 2, "staging depth");
  __shared__ __attribute__((aligned(16))) unsigned char ring[CB_LDS + AHEAD * 12 * CB_STG * 4];
  float* const stg0 = (float*)(ring + CB_LDS);  // [buffer AHEAD][row 4][plane 3][CB_STG]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: piece addressing on the SALU
  const int r16 = lane & 15;
  const int q = lane >> 4;
  const int img = blockIdx.x;
  const int t0 = blockIdx.y * CB_TILES;  // first 16-column MFMA tile of the block
  const int pc0 = 28 * t0 - 2;           // padded column of ring pair 0
  const int xs0 = 28 * t0 - 8;           // input column of staged element 0 (16-B aligned: W % 4 == 0)
  const float* fimg = fx + (long long)img * 3 * H * W;

  auto direct_load = [&](int prow, int g, float (&v)[6]) {
    const int yy = prow - 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int xx = pc0 + 2 * g + h - 3;
      const bool ok = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
      const float* src = fimg + (ok ? (long long)yy * W + xx : 0);  // always a valid address
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float t = src[(long long)c * H * W];
        v[3 * h + c] = ok ? t : 0.f;
      }
    }
  };
  // 4 rows [r0, r0 + 4) x 3 planes -> staging: 12 pieces of 128 floats from column xs0, 3 per
  // wave; 16-B pieces wholly outside the row read column 0 instead (never used: zero padding)
  auto stage_f32 = [&](int r0, int buf) {
    float* const stg = stg0 + buf * 12 * CB_STG;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int p = wid + CB_TILES * i;
      const int rr = p / 3, c = p - 3 * (p / 3);
      const int yy = min(max(r0 + rr - 3, 0), H - 1);  // out-of-image rows: zeroed at conversion
      const int xp = xs0 + 4 * lane;
      const bool ok = xp >= 0 && xp + 4 <= W;
      if (lane < CB_STG / 4)
        dma16(fimg + ((long long)c * H + yy) * W + (ok ? xp : 0), stg + (rr * 3 + c) * CB_STG);
    }
  };
  auto staged_load = [&](int prow, int rr, int g, int buf, float (&v)[6]) {
    const float* const stg = stg0 + buf * 12 * CB_STG;
    const int yy = prow - 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int xx = pc0 + 2 * g + h - 3;
      const bool ok = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float t = stg[(rr * 3 + c) * CB_STG + 2 * g + h + 3];  // xx - xs0
        v[3 * h + c] = ok ? t : 0.f;
      }
    }
  };
  auto direct_store = [&](int prow, int g, const float (&v)[6]) {
    const unsigned d0 = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
    const unsigned d1 = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
    const unsigned d2 = (unsigned)f2bf(v[4]) | ((unsigned)f2bf(v[5]) << 16);
    unsigned char* slot = ring + (size_t)(((prow + 3) & (RING - 1)) * 4) * CB_CH * 16;
#pragma unroll
    for (int m = 0; m < 4; ++m) {  // copy m holds the row shifted by 4m bytes
      unsigned* d = (unsigned*)(slot + (size_t)m * CB_CH * 16 + 12 * g + 4 * m);
      d[0] = d0;
      d[1] = d1;
      d[2] = d2;
    }
  };

  bf16x8 wf[4][6];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int s = 0; s < 6; ++s) wf[j][s] = *(const bf16x8*)(w + (j * 16 + r16) * KSTEM + 32 * s + 8 * q);
  const int k = 14 * wid + r16;  // ring-relative stem column + 1
  const int m = k & 3;
  const int sx = 14 * (t0 + wid) - 1 + r16;
  // the accumulators start from the BN shift, or -inf for stem columns outside the map: such a
  // column then pools as -inf with no per-step mask (the products are finite)
  const float cmask = (sx >= 0 && sx < Ws) ? 0.f : -INFINITY;
  f32x4 bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bv[j] = *(const f32x4*)(bias + j * 16 + 4 * q) + cmask;
  const int xchunk = m * CB_CH + (12 * k + 4 * m) / 16;

  auto stem_row = [&](int sy, f32x4 (&acc)[4]) {
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const int g = 4 * s + q;
      const int kh = min(g / 3, 6);  // kh 7: zero weights, any finite pixel
      const int c = g - 3 * (g / 3);
      const int slot = (2 * sy + kh + 3) & (RING - 1);
      const bf16x8 xf = ((const bf16x8*)ring)[slot * 4 * CB_CH + xchunk + c];
#pragma unroll
      for (int j = 0; j < 4; ++j)  // s = 0 accumulates onto the BN shift (no per-step zeroing, no shift add)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][s], xf, s ? acc[j] : bv[j], 0, 0, 0);
    }
  };

  for (int t = tid; t < 13 * CB_GP; t += 64 * CB_TILES) {
    float v[6];
    direct_load(t / CB_GP, t % CB_GP, v);
    direct_store(t / CB_GP, t % CB_GP, v);
  }
  __syncthreads();

  const float NEG = -INFINITY;
  u16* yimg = y + (long long)img * Hq * Wq * 64;
  const int px = 7 * (t0 + wid) + (r16 >> 1);
  const bool writer = !(r16 & 1) && r16 <= 12 && px < Wq;
  const bool dtask = tid < 4 * CB_GP;
  const int drow = tid / CB_GP, dg = tid - (tid / CB_GP) * CB_GP;
  // one pooled row: stem rows 2py (into a1) and 2py + 1 (into a2), pooled with `prev` (stem row
  // 2py - 1); the caller rotates the three arrays (no per-step copy of a2 into prev)
  auto step = [&](int py, const f32x4 (&prev)[4], f32x4 (&a1)[4], f32x4 (&a2)[4]) {
    // rows 4 py + 9 .. + 12 are step py + 1's new ones; with AHEAD 2 they were staged at step
    // py - 1 (step 0: loaded with the first 13 rows) and this step stages step py + 2's
    if (AHEAD == 1 && py + 1 < Hq) stage_f32(4 * py + 9, 0);
    if (AHEAD == 2 && py + 2 < Hq) stage_f32(4 * py + 13, py & 1);
    stem_row(2 * py, a1);
    stem_row(2 * py + 1, a2);
    // Pool on the accumulators, which start from the BN shift (max commutes with ReLU and the bf16
    // rounding, both monotone) or -inf (columns outside the map).  VALU-lean: the SIMD's vector
    // issue, not the MFMA pipe, bounded this loop (r01: ~290 VALU per wave-step against 48
    // MFMAs): Hs is even (launcher), so no stem row is past the map; the column max takes its
    // neighbours by DPP (bound_ctrl: lanes past the 16-lane row read 0, they are not writers);
    // the file is built with -fno-honor-nans (no canonicalising max per DPP value).
    unsigned pk4[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int e2 = 0; e2 < 2; ++e2) {
        float o[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = 2 * e2 + h;
          const float v = fmaxf(fmaxf(prev[j][e], a1[j][e]), a2[j][e]);  // row max
          const float c = fmaxf(fmaxf(v, shl_dpp<1>(v)), shl_dpp<2>(v));
          o[h] = fmaxf(c, 0.f);  // the shift is in the accumulators
        }
        pk4[j][e2] = pack_bf2(o[0], o[1]);
      }
    }
    if (py + 1 < Hq && (AHEAD == 1 || py >= 1)) {
      if (AHEAD == 2 && py + 2 < Hq)
        vm_wait<3>();  // all but this step's 3 staging pieces: the rows staged a step ago have landed
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (dtask) {
        float dv[6];
        staged_load(4 * py + 9 + drow, drow, dg, AHEAD == 2 ? (py - 1) & 1 : 0, dv);
        direct_store(4 * py + 9 + drow, dg, dv);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (writer)
        *(uint2*)(yimg + ((long long)py * Wq + px) * 64 + j * 16 + 4 * q) = make_uint2(pk4[j][0], pk4[j][1]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  f32x4 ra[4], rb[4], rc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) ra[j] = f32x4{NEG, NEG, NEG, NEG};
  // rows rotate ra -> (rb, rc) -> (ra, rb) -> (rc, ra): three steps per iteration, each reading
  // the previous step's second row as its `prev`
  int py = 0;
  for (; py + 3 <= Hq; py += 3) {
    step(py, ra, rb, rc);
    step(py + 1, rc, ra, rb);
    step(py + 2, rb, rc, ra);
  }
  if (py < Hq) step(py, ra, rb, rc);
  if (py + 1 < Hq) step(py + 1, rc, ra, rb);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// r05 form of the column-blocked DIRECT kernel (default; EOSV_STEM_V5=0 selects the r04 one):
// the same tiles, ring, staging and arithmetic (bitwise equal outputs), with the per-step issue
// cost cut, since the SIMD's vector issue -- not the MFMA pipe -- bounded the r04 loop (SQ:
// MFMA-busy 0.39, ~155 VALU + 48 MFMA per wave-step, r04j_sq_r18_bf16.txt):
//  * ONE barrier per step, at its top: it covers the previous step's ring writes (lgkmcnt(0)) and
//    the previous step's staging DMA (each wave waits for its own pieces with vmcnt(4): the step's
//    4 output stores are the only younger memory ops, and every wave issues exactly 4 -- buffer
//    stores, non-writers out of range -- so the count holds for every wave), and it orders the
//    previous step's ring / staging reads before this step's overwrites;
//  * the step loop is unrolled by 12 (the ring's 4-step period x the 3-way accumulator rotation),
//    so every ring address is a per-lane register + a compile-time offset: no VALU address math
//    (36 VALU per wave-step in r04).  The ring wrap inside a step's 9-row window is a second
//    per-lane register (for the k-slices whose two kernel rows straddle slot 15 -> 0);
//  * out-of-frame staging pieces (frame edges, rows past the bottom) come from a zeroed device
//    line, so the conversion needs no per-value selects;
//  * output stores are buffer stores with the step in the scalar offset;
//  * column max by DPP (2 VALU per value), ReLU as one packed integer max on the two bf16 values
//    (bf16 bit patterns order as signed 16-bit integers for finite values: max(x, 0) = ReLU).
__device__ __attribute__((aligned(16))) float stem_zero_line[4] = {0.f, 0.f, 0.f, 0.f};
// c[e] = max(v[e] of lanes l, l + 1, l + 2 of the lane's 16-lane row) for 4 values: 8 VOP2 DPP
// maxes.  The s_nop 1 gives the 2 wait states a DPP read needs after the VALU write of its source
// (the asm is opaque to the compiler's hazard recognizer); the second max of each value reads the
// first's result as its plain operand.
__device__ __forceinline__ void colmax4(const f32x4& v, f32x4& c) {
  float c0, c1, c2, c3;
  asm("s_nop 1\n\t"
      "v_max_f32_dpp %0, %4, %4 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_max_f32_dpp %1, %5, %5 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_max_f32_dpp %2, %6, %6 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_max_f32_dpp %3, %7, %7 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_max_f32_dpp %0, %4, %0 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_max_f32_dpp %1, %5, %1 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_max_f32_dpp %2, %6, %2 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_max_f32_dpp %3, %7, %3 row_shl:2 row_mask:0xf bank_mask:0xf bound_ctrl:1"
      : "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3)
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
  c = f32x4{c0, c1, c2, c3};
}
constexpr int CB_ROWB = 4 * CB_CH * 16;  // bytes per ring row (4 shifted copies)

__global__ __launch_bounds__(64 * CB_TILES, 2) void stem_pool_bf16_cb5_kernel(const float* __restrict__ fx,
                                                                         const u16* __restrict__ w,
                                                                         const float* __restrict__ bias, u16* y,
                                                                         int H, int W, int Hs, int Ws, int Hq, int Wq) {
  // + 1 KiB: the destination of the two waves' spare staging instruction (zero lines)
  __shared__ __attribute__((aligned(16))) unsigned char ring[CB_LDS + 3 * 12 * CB_STG * 4 + 1024];
  float* const stg0 = (float*)(ring + CB_LDS);  // [buffer 3][row 4][plane 3][CB_STG]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15;
  const int q = lane >> 4;
  const int img = blockIdx.x;
  const int t0 = blockIdx.y * CB_TILES;
  const int pc0 = 28 * t0 - 2;
  const int xs0 = 28 * t0 - 8;
  const float* fimg = fx + (long long)img * 3 * H * W;

  // ---- weights (registers) and BN shift (+ -inf for stem columns outside the map)
  bf16x8 wf[4][6];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int s = 0; s < 6; ++s) wf[j][s] = *(const bf16x8*)(w + (j * 16 + r16) * KSTEM + 32 * s + 8 * q);
  const int k = 14 * wid + r16;
  const int m = k & 3;
  const int sx = 14 * (t0 + wid) - 1 + r16;
  const float cmask = (sx >= 0 && sx < Ws) ? 0.f : -INFINITY;
  f32x4 bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bv[j] = *(const f32x4*)(bias + j * 16 + 4 * q) + cmask;
  const int xchunk = m * CB_CH + (12 * k + 4 * m) / 16;

  // ---- B-fragment addresses: k-slice s, lane q reads kernel row kh = min((4s + q) / 3, 6), chunk
  // c = (4s + q) % 3.  kh = k0[s] + d (d = 0 / 1 by lane); at a step whose compile-time slot of
  // kh = k0[s] is D = (C + k0[s]) & 15, the read is at D * ROWB + va[s] (D < 15) or vb[s] (D = 15:
  // the d = 1 lanes wrap to slot 0)
  constexpr int K0[6] = {0, 1, 2, 4, 5, 6};
  int va[6], vb[6];
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const int g = 4 * s + q;
    const int kh = min(g / 3, 6), c = g - 3 * (g / 3);
    const int d = kh - K0[s];
    const int lc = (xchunk + c) * 16;
    va[s] = d * CB_ROWB + lc;
    vb[s] = d ? lc : 15 * CB_ROWB + lc;
  }

  // ---- staging (f32 plane rows by LDS-DMA; pieces outside the frame read the zero line).  A step
  // stages 12 plane rows (staged row p = 3 rr + c: padded row r0 + rr, plane c) of CB_STG = 32 lanes
  // x 16 B each, so one DMA instruction carries two consecutive rows: lanes 0-31 row 2 e, lanes 32-63
  // row 2 e + 1 (the lane's LDS slot is the row base + 16 lane).  Wave w issues pairs e = w and
  // e = w + 4; waves 2 and 3 have no second pair and DMA zero lines into a spare 1 KiB, so every
  // wave issues two pieces per step (the counted waits below).  Per lane: its two source rows'
  // pointers at r0 = 0 and the column-window test, fixed for the kernel; a step adds r0 rows.
  // (r04: 3 pieces per wave, 30 of 64 lanes active, each piece's address rebuilt in scalar code.)
  const float* zl = stem_zero_line;
  asm volatile("" : "+v"(zl));  // one copy held in registers (hipcc rematerialised its address per use)
  const float* sbase[2];
  int srr[2];
  bool scol[2];
  int sdst[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = wid + 4 * i;  // row pair
    const int pr = 2 * e + (lane >> 5), rr = pr / 3, c = pr - 3 * (pr / 3);
    const int xp = xs0 + 4 * (lane & 31);
    scol[i] = e < 6 && xp >= 0 && xp + 4 <= W;
    srr[i] = e < 6 ? rr - 3 : -(1 << 20);
    sbase[i] = fimg + ((long long)c * H + (rr - 3)) * W + xp;
    sdst[i] = e < 6 ? 2 * e * CB_STG * 4 : 3 * 12 * CB_STG * 4;  // byte offset from stg0 (spare: past buffer 2)
  }
  auto stage_f32 = [&](int r0, int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool ok = scol[i] && (unsigned)(r0 + srr[i]) < (unsigned)H;
      const int boff = sdst[i] < 3 * 12 * CB_STG * 4 ? buf * 12 * CB_STG * 4 : 0;
      dma16(ok ? sbase[i] + (long long)r0 * W : zl, (unsigned char*)stg0 + sdst[i] + boff);
    }
  };
  // conversion task of this thread: ring row drow (0..3) of a step's 4 new rows, column pair dg
  const bool dtask = tid < 4 * CB_GP;
  const int drow = dtask ? tid / CB_GP : 0, dg = dtask ? tid - (tid / CB_GP) * CB_GP : 0;
  const int cst = (drow * 3 * CB_STG + 2 * dg + 3) * 4;  // staging byte offset of (row, plane 0, pair)
  const int cwr = drow * CB_ROWB + 12 * dg;              // ring byte offset of (row, pair) in copy 0

  // ---- prologue: the staging of the rows steps 0 and 1 convert (padded rows 9 .. 12 -> buffer 1,
  // 13 .. 16 -> buffer 2), then padded rows 0 .. 8 straight from the frame (global loads,
  // bounds-checked; all of a thread's loads issued before any conversion), one drain
  stage_f32(9, 1);
  stage_f32(13, 2);
  {
    constexpr int NPRO = (9 * CB_GP + 64 * CB_TILES - 1) / (64 * CB_TILES);
    float v[NPRO][6];
#pragma unroll
    for (int i = 0; i < NPRO; ++i) {
      const int t = tid + i * 64 * CB_TILES;
      const int prow = t / CB_GP, g = t % CB_GP;
      const int yy = prow - 3;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int xx = pc0 + 2 * g + h - 3;
        const bool ok = t < 9 * CB_GP && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
        const float* src = fimg + (ok ? (long long)yy * W + xx : 0);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float tv = src[(long long)c * H * W];
          v[i][3 * h + c] = ok ? tv : 0.f;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NPRO; ++i) {
      const int t = tid + i * 64 * CB_TILES;
      if (t >= 9 * CB_GP) break;
      const int prow = t / CB_GP, g = t % CB_GP;
      const unsigned d0 = pack_bf2(v[i][0], v[i][1]), d1 = pack_bf2(v[i][2], v[i][3]), d2 = pack_bf2(v[i][4], v[i][5]);
      unsigned char* slot = ring + (size_t)((prow + 3) & (RING - 1)) * CB_ROWB + 12 * g;
#pragma unroll
      for (int mm = 0; mm < 4; ++mm) {
        unsigned* d = (unsigned*)(slot + mm * (CB_CH * 16 + 4));
        d[0] = d0;
        d[1] = d1;
        d[2] = d2;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the prologue's staging has landed
  __syncthreads();

  // ---- output: buffer stores, lane offset fixed, the pooled row in the scalar offset
  u16* yimg = y + (long long)img * Hq * Wq * 64;
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(yimg, (short)0, Hq * Wq * 128, 0x00020000);
  const int px = 7 * (t0 + wid) + (r16 >> 1);
  const bool writer = !(r16 & 1) && r16 <= 12 && px < Wq;
  const int yvo = writer ? (px * 64 + 4 * q) * 2 : 0x40000000;  // non-writers: out of range, dropped

  const float NEG = -INFINITY;
  // step py (py = 12 i + U): stem rows 2py (a1) and 2py + 1 (a2), pooled with prev (row 2py - 1)
  auto step = [&](auto U_, int py, const f32x4 (&prev)[4], f32x4 (&a1)[4], f32x4 (&a2)[4]) {
    constexpr int U = decltype(U_)::value;
    // top: the previous step's ring writes are complete for every wave (lgkmcnt(0) + barrier), and
    // so is the staging DMA of step py - 2, which this step converts: younger than its 2 pieces are
    // that step's 4 output stores and step py - 1's 2 pieces + 4 stores (every step issues exactly
    // these; steps 0 and 1 convert the prologue's staging, drained before the loop)
    vm_wait<10>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // rows 4 py + 17 .. + 20 (converted at step py + 2) into buffer py % 3 (read by step py - 1's
    // conversion: done); past the frame's last rows the pieces read the zero line, so the count of
    // pieces per step never changes
    stage_f32(4 * py + 17, U % 3);
    // B fragments of stem row 2 py + R: all 6 k-slices read up front (the r04 loop read one,
    // waited for it and ran its 4 MFMAs, so every k-slice exposed an LDS round trip)
    auto frags = [&](auto R_, bf16x8 (&xf)[6]) {
      constexpr int R = decltype(R_)::value;
      constexpr int C = 4 * (U % 4) + 2 * R + 3;  // slot of kernel row 0 = (prow + 3) & 15, prow = 4 py + 2 R
#pragma unroll
      for (int s = 0; s < 6; ++s) {
        const int D = (C + K0[s]) & 15;
        const unsigned char* a = D == 15 ? ring + vb[s] : ring + D * CB_ROWB + va[s];
        xf[s] = *(const bf16x8*)a;
      }
    };
    auto stem_row = [&](const bf16x8 (&xf)[6], f32x4 (&acc)[4]) {
#pragma unroll
      for (int s = 0; s < 6; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][s], xf[s], s ? acc[j] : bv[j], 0, 0, 0);
    };
    bf16x8 x1[6], x2[6];
    frags(std::integral_constant<int, 0>{}, x1);
    frags(std::integral_constant<int, 1>{}, x2);
    stem_row(x1, a1);
    // convert the staged rows 4 py + 9 .. + 12 (step py + 1's new rows; staged at step py - 2 into
    // buffer (py - 2) % 3 = (U + 1) % 3, or by the prologue)
    // into ring slots (4 py + 12 + drow) & 15 = 4 ((U + 3) % 4) + drow: no wrap
    if (py + 1 < Hq && dtask) {
      const float* st = (const float*)((const unsigned char*)stg0 + ((U + 1) % 3) * 12 * CB_STG * 4 + cst);
      float v[6];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int c = 0; c < 3; ++c) v[3 * h + c] = st[c * CB_STG + h];
      const unsigned d0 = pack_bf2(v[0], v[1]), d1 = pack_bf2(v[2], v[3]), d2 = pack_bf2(v[4], v[5]);
      unsigned char* slot = ring + 4 * ((U + 3) % 4) * CB_ROWB + cwr;
#pragma unroll
      for (int mm = 0; mm < 4; ++mm) {
        unsigned* d = (unsigned*)(slot + mm * (CB_CH * 16 + 4));
        d[0] = d0;
        d[1] = d1;
        d[2] = d2;
      }
    }
    stem_row(x2, a2);
    // pool: row max (v_max3), column max over lanes r16, r16 + 1, r16 + 2 of the 16-lane row as two
    // DPP maxes (the compiler's form was two DPP moves + a v_max3; bound_ctrl reads 0 past the row
    // end: those lanes are not writers), bf16, ReLU on the packed pair
    asm volatile("" ::: "memory");  // the stores below stay after this step's staging DMA (the vm_wait count above)
    unsigned pk4[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 v, c;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(fmaxf(prev[j][e], a1[j][e]), a2[j][e]);
      colmax4(v, c);
#pragma unroll
      for (int e2 = 0; e2 < 2; ++e2) {
        typedef short s16x2 __attribute__((ext_vector_type(2)));
        const s16x2 p = __builtin_bit_cast(s16x2, pack_bf2(c[2 * e2], c[2 * e2 + 1]));
        pk4[j][e2] = __builtin_bit_cast(unsigned, __builtin_elementwise_max(p, (s16x2){0, 0}));
      }
    }
    const int so = py * Wq * 128;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, make_uint2(pk4[j][0], pk4[j][1])), yr, yvo + 32 * j,
                                            so, 0);
    }
  };
  f32x4 ra[4], rb[4], rc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) ra[j] = f32x4{NEG, NEG, NEG, NEG};
  // 12 steps per iteration (a uniform exit test after each), rows rotating ra -> (rb, rc) -> (ra, rb)
  // -> (rc, ra)
#define EOSV_STEM5_STEP(U, P, A, B)                                        \
  step(std::integral_constant<int, U>{}, py + U, P, A, B);                 \
  if (py + U + 1 >= Hq) break;
  for (int py = 0;; py += 12) {
    EOSV_STEM5_STEP(0, ra, rb, rc)
    EOSV_STEM5_STEP(1, rc, ra, rb)
    EOSV_STEM5_STEP(2, rb, rc, ra)
    EOSV_STEM5_STEP(3, ra, rb, rc)
    EOSV_STEM5_STEP(4, rc, ra, rb)
    EOSV_STEM5_STEP(5, rb, rc, ra)
    EOSV_STEM5_STEP(6, ra, rb, rc)
    EOSV_STEM5_STEP(7, rc, ra, rb)
    EOSV_STEM5_STEP(8, rb, rc, ra)
    EOSV_STEM5_STEP(9, ra, rb, rc)
    EOSV_STEM5_STEP(10, rc, ra, rb)
    EOSV_STEM5_STEP(11, rb, rc, ra)
  }
#undef EOSV_STEM5_STEP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// EOSV_F32X3 stem (column-blocked, DIRECT frames): the same fused stem conv + ReLU + maxpool in
// split-bf16 arithmetic.  Frames are split as x = x_hi + x_lo and the folded weights as
// w = w_hi + w_lo (each part bf16, round to nearest), and every MFMA k-slice accumulates
// w_hi.x_hi + w_hi.x_lo + w_lo.x_hi in f32 (the x_lo.w_lo term, ~2^-16 relative, is dropped, as
// in the split convs; tests/test_gpu_parity.py bounds the features at 1e-4 of the f32 oracle).
// Replaces the exact-f32 MFMA stem (v_mfma_f32_16x16x4_f32: 16x fewer FLOP/clk than bf16).
// Output: pooled map in the split layout [pixel][hi 64 | lo 64].
// LDS (56 KiB -> 2 workgroups per CU): w_lo [64][192] (16-B chunk c of row r at
// (c & ~7) | ((c ^ (r >> 1)) & 7): conflict-free A-fragment reads); x_hi and x_lo rings, ONE copy
// each (16 rows x 736 B), read as 4 dwords per B fragment (4-B aligned sources: no shifted
// copies); the f32 staging of the DIRECT kernel.  w_hi stays in registers.
constexpr int X3_ROWB = 736;  // bytes per ring row: 12 * CB_GP = 732, rounded up to 16
static_assert(12 * CB_GP <= X3_ROWB, "x3 ring row");
constexpr int X3_RING = RING * X3_ROWB;                 // bytes per ring (hi or lo)
constexpr int X3_WLO = 64 * KSTEM * 2;                  // bytes of w_lo

__global__ __launch_bounds__(64 * CB_TILES, 2) void stem_pool_x3_cb_kernel(const float* __restrict__ fx,
                                                                          const u16* __restrict__ w,
                                                                          const float* __restrict__ bias, u16* y,
                                                                          int H, int W, int Hs, int Ws, int Hq, int Wq) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[X3_WLO + 2 * X3_RING + 12 * CB_STG * 4];
  u16* wlo_s = (u16*)lds;
  unsigned char* rh = lds + X3_WLO;           // x_hi ring
  unsigned char* rl = rh + X3_RING;           // x_lo ring
  float* stg = (float*)(rl + X3_RING);        // [row 4][plane 3][CB_STG]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15;
  const int q = lane >> 4;
  const int img = blockIdx.x;
  const int t0 = blockIdx.y * CB_TILES;
  const int pc0 = 28 * t0 - 2;
  const int xs0 = 28 * t0 - 8;
  const float* fimg = fx + (long long)img * 3 * H * W;

  // w_lo -> LDS (swizzled 16-B chunks), w_hi -> registers
  for (int i = tid; i < 64 * (KSTEM / 8); i += 64 * CB_TILES) {
    const int r = i / (KSTEM / 8), c = i - r * (KSTEM / 8);
    const int cs = (c & ~7) | ((c ^ (r >> 1)) & 7);
    *(uint4*)(wlo_s + r * KSTEM + cs * 8) = *(const uint4*)(w + 64 * KSTEM + r * KSTEM + c * 8);
  }
  bf16x8 wf[4][6];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int s = 0; s < 6; ++s) wf[j][s] = *(const bf16x8*)(w + (j * 16 + r16) * KSTEM + 32 * s + 8 * q);
  f32x4 bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bv[j] = *(const f32x4*)(bias + j * 16 + 4 * q);

  auto direct_load = [&](int prow, int g, float (&v)[6]) {
    const int yy = prow - 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int xx = pc0 + 2 * g + h - 3;
      const bool ok = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
      const float* src = fimg + (ok ? (long long)yy * W + xx : 0);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float t = src[(long long)c * H * W];
        v[3 * h + c] = ok ? t : 0.f;
      }
    }
  };
  auto stage_f32 = [&](int r0) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int p = wid + CB_TILES * i;
      const int rr = p / 3, c = p - 3 * (p / 3);
      const int yy = min(max(r0 + rr - 3, 0), H - 1);
      const int xp = xs0 + 4 * lane;
      const bool ok = xp >= 0 && xp + 4 <= W;
      if (lane < CB_STG / 4)
        dma16(fimg + ((long long)c * H + yy) * W + (ok ? xp : 0), stg + (rr * 3 + c) * CB_STG);
    }
  };
  auto staged_load = [&](int prow, int rr, int g, float (&v)[6]) {
    const int yy = prow - 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int xx = pc0 + 2 * g + h - 3;
      const bool ok = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float t = stg[(rr * 3 + c) * CB_STG + 2 * g + h + 3];
        v[3 * h + c] = ok ? t : 0.f;
      }
    }
  };
  // pair g of padded row prow -> 12 B of the hi ring row and 12 B of the lo ring row
  auto direct_store = [&](int prow, int g, const float (&v)[6]) {
    unsigned hi[3], lo[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const unsigned ph = pack_bf2(v[2 * i], v[2 * i + 1]);
      hi[i] = ph;
      lo[i] = pack_bf2(v[2 * i] - __uint_as_float(ph << 16), v[2 * i + 1] - __uint_as_float(ph & 0xffff0000u));
    }
    const int off = ((prow + 3) & (RING - 1)) * X3_ROWB + 12 * g;
    unsigned* dh = (unsigned*)(rh + off);
    unsigned* dl = (unsigned*)(rl + off);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      dh[i] = hi[i];
      dl[i] = lo[i];
    }
  };

  const int k = 14 * wid + r16;  // ring-relative stem column + 1
  const int sx = 14 * (t0 + wid) - 1 + r16;
  const float cmask = (sx >= 0 && sx < Ws) ? 0.f : -INFINITY;
  // per k-slice s: this lane's B-fragment byte offset in a ring row, and its w_lo A-fragment chunk
  int xoff[6], khs[6];
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const int g = 4 * s + q;
    khs[s] = min(g / 3, 6);  // kh 7: zero weights, any finite pixel
    xoff[s] = 12 * k + 16 * (g - 3 * (g / 3));
  }
  auto ldx = [&](const unsigned char* ring, int row, int s) {
    const unsigned* p = (const unsigned*)(ring + ((row + khs[s] + 3) & (RING - 1)) * X3_ROWB + xoff[s]);
    unsigned v[4] = {p[0], p[1], p[2], p[3]};
    return __builtin_bit_cast(bf16x8, v);
  };
  auto stem_rows = [&](int sy0, f32x4 (&a1)[4], f32x4 (&a2)[4]) {
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      bf16x8 wl[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = j * 16 + r16, c = 4 * s + q;
        wl[j] = *(const bf16x8*)(wlo_s + r * KSTEM + ((c & ~7) | ((c ^ (r >> 1)) & 7)) * 8);
      }
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        f32x4(&acc)[4] = rr ? a2 : a1;
        const int row = 2 * (sy0 + rr);
        const bf16x8 xh = ldx(rh, row, s), xl = ldx(rl, row, s);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][s], xh, s ? acc[j] : bv[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][s], xl, acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[j], xh, acc[j], 0, 0, 0);
        }
      }
    }
  };

  for (int t = tid; t < 13 * CB_GP; t += 64 * CB_TILES) {
    float v[6];
    direct_load(t / CB_GP, t % CB_GP, v);
    direct_store(t / CB_GP, t % CB_GP, v);
  }
  __syncthreads();

  const float NEG = -INFINITY;
  f32x4 prev[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) prev[j] = f32x4{NEG, NEG, NEG, NEG};
  u16* yimg = y + (long long)img * Hq * Wq * 128;
  const int px = 7 * (t0 + wid) + (r16 >> 1);
  const bool writer = !(r16 & 1) && r16 <= 12 && px < Wq;
  const bool dtask = tid < 4 * CB_GP;
  const int drow = tid / CB_GP, dg = tid - (tid / CB_GP) * CB_GP;
  for (int py = 0; py < Hq; ++py) {
    if (py + 1 < Hq) stage_f32(4 * py + 9);
    f32x4 a1[4], a2[4];
    stem_rows(2 * py, a1, a2);
    // pool as stem_pool_bf16_cb_kernel (Hs even: no stem row past the map), then split the
    // pooled f32 value into hi + lo
    uint2 ph[4], pl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = fmaxf(fmaxf(prev[j][e], a1[j][e]), a2[j][e]) + cmask;
        prev[j][e] = a2[j][e];
        const float c = fmaxf(fmaxf(v, shl_dpp<1>(v)), shl_dpp<2>(v));
        o[e] = fmaxf(c, 0.f);
      }
      const unsigned h0 = pack_bf2(o[0], o[1]), h1 = pack_bf2(o[2], o[3]);
      ph[j] = make_uint2(h0, h1);
      pl[j] = make_uint2(pack_bf2(o[0] - __uint_as_float(h0 << 16), o[1] - __uint_as_float(h0 & 0xffff0000u)),
                         pack_bf2(o[2] - __uint_as_float(h1 << 16), o[3] - __uint_as_float(h1 & 0xffff0000u)));
    }
    if (py + 1 < Hq) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (dtask) {
        float dv[6];
        staged_load(4 * py + 9 + drow, drow, dg, dv);
        direct_store(4 * py + 9 + drow, dg, dv);
      }
    }
    if (writer) {
      u16* o = yimg + ((long long)py * Wq + px) * 128 + 4 * q;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        *(uint2*)(o + j * 16) = ph[j];
        *(uint2*)(o + 64 + j * 16) = pl[j];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

bool stem_pool_x3_ok(int H, int W) {
  const int Hs = (H + 6 - 7) / 2 + 1;
  return H >= 8 && W >= 8 && W % 4 == 0 && Hs % 2 == 0;
}

// w: [hi 64 x 192 | lo 64 x 192] bf16 (stem K layout [kh 8][24]), bias f32 [64], frames f32 NCHW,
// y: split layout [N][Hq][Wq][128] (hi 64 | lo 64)
int launch_stem_pool_x3(const float* frames, int B, int H, int W, const void* w, const float* bias, void* y,
                        hipStream_t s, LaunchInfo* info) {
  if (!stem_pool_x3_ok(H, W)) return set_error("stem_pool_x3: unsupported frame shape"), EOSV_ERR_UNSUPPORTED;
  if (B <= 0) return EOSV_OK;
  const int Hs = (H + 6 - 7) / 2 + 1, Ws = (W + 6 - 7) / 2 + 1;
  const int Hq = (Hs + 2 - 3) / 2 + 1, Wq = (Ws + 2 - 3) / 2 + 1;
  const int ncb = ((Wq + 6) / 7 + CB_TILES - 1) / CB_TILES;
  if (info) {
    static const int occ = kernel_occupancy((const void*)stem_pool_x3_cb_kernel, 64 * CB_TILES);
    return record_launch(info, (long long)B * ncb, occ);
  }
  hipLaunchKernelGGL(stem_pool_x3_cb_kernel, dim3(B, ncb), dim3(64 * CB_TILES), 0, s, frames, (const u16*)w, bias,
                     (u16*)y, H, W, Hs, Ws, Hq, Wq);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

#ifndef EOSV_STEM_AHEAD_DEF
#define EOSV_STEM_AHEAD_DEF 2
#endif
static int stem_ahead() {
  static const int v = env_switch("EOSV_STEM_AHEAD", EOSV_STEM_AHEAD_DEF);  // 1 = the r02 one-step staging (A/B switch)
  return v == 1 ? 1 : 2;
}

static bool stem_v5() {
  static const bool v = env_switch("EOSV_STEM_V5", 1) != 0;  // 0 = the r04 column-blocked kernel (A/B switch)
  return v;
}

static bool stem_cb() {
  static const bool v = env_switch("EOSV_STEM_CB", 1) != 0;  // 0 = full-width workgroups (A/B switch)
  return v;
}

// direct: the caller passes the f32 NCHW frames (no pack)
bool stem_pool_bf16_ok(int H, int W, bool direct) {
  const int Hs = (H + 6 - 7) / 2 + 1, Ws = (W + 6 - 7) / 2 + 1;
  const int Wq = (Ws + 2 - 3) / 2 + 1;
  if (H < 8 || W < 8) return false;
  return (direct && stem_cb() && W % 4 == 0 && Hs % 2 == 0) || (Wq + 6) / 7 <= MAX_TILES;
}

// pack: padded bf16 RGB rows (pack_rgb_pad), or nullptr with `frames` = the f32 NCHW input
int launch_stem_pool_bf16(const void* pack, int B, int H, int W, const void* w, const float* bias, void* y,
                          hipStream_t s, const float* frames, LaunchInfo* info) {
  const int Hs = (H + 6 - 7) / 2 + 1, Ws = (W + 6 - 7) / 2 + 1;
  const int Hq = (Hs + 2 - 3) / 2 + 1, Wq = (Ws + 2 - 3) / 2 + 1;
  const int ntiles = (Wq + 6) / 7;
  if (frames && stem_cb() && W % 4 == 0 && Hs % 2 == 0) {
    if (B <= 0) return EOSV_OK;
    const int ncb = (ntiles + CB_TILES - 1) / CB_TILES;
    if (info) {
      static const int occ = kernel_occupancy((const void*)stem_pool_bf16_cb5_kernel, 64 * CB_TILES);
      return record_launch(info, (long long)B * ncb, occ);
    }
    if (stem_v5())
      hipLaunchKernelGGL(stem_pool_bf16_cb5_kernel, dim3(B, ncb), dim3(64 * CB_TILES), 0, s, frames, (const u16*)w,
                         bias, (u16*)y, H, W, Hs, Ws, Hq, Wq);
    else if (stem_ahead() == 1)
      hipLaunchKernelGGL(stem_pool_bf16_cb_kernel<1>, dim3(B, ncb), dim3(64 * CB_TILES), 0, s, frames, (const u16*)w,
                         bias, (u16*)y, H, W, Hs, Ws, Hq, Wq);
    else
      hipLaunchKernelGGL(stem_pool_bf16_cb_kernel<2>, dim3(B, ncb), dim3(64 * CB_TILES), 0, s, frames, (const u16*)w,
                         bias, (u16*)y, H, W, Hs, Ws, Hq, Wq);
    EOSV_LAUNCH_CHECK();
    return EOSV_OK;
  }
  if (ntiles > MAX_TILES || B <= 0) return B <= 0 ? EOSV_OK : (set_error("stem_pool: too wide"), EOSV_ERR_UNSUPPORTED);
  if (info) return record_launch(info, B, 1);  // one image per workgroup, LDS-bound to 1 per CU
  const int Wp = stem_row_pixels(W, 3);
  if (frames) {
    if (4 * (Wp / 2) > 64 * ntiles) return set_error("stem_pool: direct rows need more threads"), EOSV_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(stem_pool_bf16_kernel<true>, dim3(B), dim3(64 * ntiles), 0, s, nullptr, frames, (const u16*)w,
                       bias, (u16*)y, H, W, Hs, Ws, Hq, Wq);
  } else {
    hipLaunchKernelGGL(stem_pool_bf16_kernel<false>, dim3(B), dim3(64 * ntiles), 0, s, (const u16*)pack, nullptr,
                       (const u16*)w, bias, (u16*)y, H, W, Hs, Ws, Hq, Wq);
  }
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

}  // namespace eosv
