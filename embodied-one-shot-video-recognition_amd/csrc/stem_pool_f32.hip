// Fused ResNet stem for f32: conv 7x7/2 p3 (3 -> 64, folded BN) + ReLU + maxpool 3x3/2 p1,
// torchvision's convnet.0-3 (reference models.py:19 via self.convnet); the f32 sibling of
// stem_pool_bf16.hip.
//
// The unfused f32 pair wrote the 112 x 112 x 64 f32 stem map (3.2 MB per frame) and read it back
// in the pool.  Here one workgroup walks one image top to bottom:
//  * 4 waves, wave g computes output channels 16g .. 16g+15 of every stem column: NT tiles of
//    16 columns (tile k = stem columns 16k .. 16k+15, NT = ceil(Ws / 16): 7 at 224, 8 at 256),
//    so no column is computed twice.  (r01/r02: waves over 7 pooled columns each computed 16
//    stem columns for 14 new ones.)  Its 16 x 148 weights (37 VGPRs) stay in registers;
//  * per pooled row py it computes stem rows 2py and 2py+1 (2py-1 is kept from the previous
//    step), takes the row max and then the column max of the raw accumulators -- pooled
//    column 8k + i sits on lane 2i of tile k and takes lanes 2i-1 .. 2i+1, lane -1 being lane
//    15 of tile k-1 (DPP row_shr:1 with a row_ror:1 of the previous tile as the fill value) --
//    and only then adds the BN shift and applies ReLU.  fl(a + b) is monotone in a and ReLU
//    commutes with max, so this is bit-identical to stem conv -> shift -> ReLU -> maxpool on
//    the same accumulators.
//
// MFMA: v_mfma_f32_16x16x4_f32 (exact f32, a k-ordered fma chain) with D = W . X^T (rows =
// output channels, columns = stem pixels), dense K = [kh 7][21] (kw*3 + c) + 1 zero = 148 = 37
// k-steps of 4.  Element k of lane q's step reads input row 2*sy + k/21, element 6*sx + k%21:
// a step whose 4 k straddle two kernel rows picks the row base per lane (one v_cndmask
// between two wave-uniform bases), so it is one ds_read_b32 per lane and tile.
//
// Row bands: a workgroup computes pooled rows [py0, py1) of one image (grid = images x bands),
// starting with stem row 2 py0 - 1 -- one stem row recomputed per band.  One workgroup per image
// left the last wave of a launch mostly empty (~2400 frames on 768 slots: 3.1 rounds -> 4);
// the launcher picks the band count that minimises rounds x rows per band.
//
// LDS: a ring of 13 input rows (row r in slot r % 13; a step needs rows 4py .. 4py+8 and
// prefetches 4py+9 .. 4py+12), each row Wp * 3 floats padded to 16 B, filled by LDS-DMA from
// the dense padded RGB pack (8-B aligned sources): ~36 KiB at 224, so several workgroups share
// a CU.  Columns past the map read whatever follows in the ring (finite or not): their
// accumulators are replaced by -inf with a select before the pool.
#include <hip/hip_bf16.h>

#include "common.h"

namespace eosv {

namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int SPF_MAX_TILES = 8;  // stem width <= 128 (input <= 256)
constexpr int SPF_K = 147;        // real K: 7 kernel rows x 21 (kw*3 + c)
constexpr int SPF_STEPS = 37;     // k-steps of 4 over dense K = 148
constexpr int SPF_KW = 176;       // uploaded f32 stem weight row ([kh][24] + 8 zero)
constexpr int SPF_RING = 13;
constexpr int SPF_NT = 256;       // 4 waves
constexpr int SPF_SLACK = 128;    // floats past the ring: reads of columns past the map

__host__ __device__ constexpr int spf_row_floats(int Wp) { return (Wp * 3 + 3) & ~3; }

__device__ __forceinline__ void dma16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// DPP within 16-lane rows: lane c <- lane c + 1 (shl), c - 1 (shr, lane 0 keeps `old`),
// c - 1 mod 16 (ror)
__device__ __forceinline__ float row_shl1(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x101, 0xf, 0xf, false));
}
__device__ __forceinline__ float row_shr1(float v, float old) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), 0x111, 0xf, 0xf, false));
}
__device__ __forceinline__ float row_ror1(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xf, 0xf, false));
}
}  // namespace

// x: padded f32 RGB [N][H+6][Wp][3] (stem_row_pixels), w: [64][176] f32, bias [64] f32,
// y: [N][Hq][Wq][64] f32 (pooled).  Grid = N images, block = 256 threads, NT = ceil(Ws / 16).
// SPLIT (EOSV_F32X3): y is [N][Hq][Wq][128] bf16, (hi, lo) of each pooled f32 value.
// DIRECT: x is the caller's f32 NCHW frames [N][3][H][W] (W % 4 == 0, W <= 256) instead of the
// padded pack: step py LDS-DMAs the input rows of step py + 2's prefetch as 12 plane rows into a
// staging area (wave g: row g's 3 planes), and wave g interleaves its row into the ring at the
// start of step py + 1, zero padding included (the pack's layout, the same f32 values:
// bit-identical results); the first rows are loaded directly.  No pack pass: its 602 KB read +
// 635 KB write per frame are gone.
constexpr int SPF_SROW = 264;  // staged plane row (floats): 3 + one 1-KiB DMA piece (W <= 256), 16-B rows

template <bool SPLIT, int NT, bool DIRECT = false>
__global__ __launch_bounds__(SPF_NT, 3) void stem_pool_f32_kernel(const float* __restrict__ x,
                                                                 const float* __restrict__ w,
                                                                 const float* __restrict__ bias, void* y, int H,
                                                                 int W, int Hs, int Ws, int Hq, int Wq, int bands) {
  extern __shared__ __attribute__((aligned(16))) float spf_smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int g = tid >> 6;  // output-channel group
  const int r16 = lane & 15;
  const int q = lane >> 4;
  const int img = blockIdx.x / bands, band = blockIdx.x - bands * img;
  const int rpb = (Hq + bands - 1) / bands;  // pooled rows per band
  const int py0 = band * rpb, py1 = min(Hq, py0 + rpb);
  if (py0 >= py1) return;
  const int Wp = stem_row_pixels(W, 3);
  const int RF = spf_row_floats(Wp);  // ring row stride (floats)
  const int Hpad = H + 6;
  float* ring = spf_smem;
  const float* ximg = x + (long long)img * (DIRECT ? 3LL * H * W : (long long)Hpad * Wp * 3);
  float* stg = spf_smem + SPF_RING * RF + SPF_SLACK;  // DIRECT: [row 4][plane 3][SPF_SROW]

  // A fragments: W[16g + r16][k = 4s + q], dense k -> uploaded [kh][24] column
  float wa[SPF_STEPS];
#pragma unroll
  for (int s = 0; s < SPF_STEPS; ++s) {
    const int k = 4 * s + q;
    wa[s] = k < SPF_K ? w[(16 * g + r16) * SPF_KW + 24 * (k / 21) + k % 21] : 0.f;
  }
  const f32x4 bv = *(const f32x4*)(bias + 16 * g + 4 * q);

  // DMA of input rows [r0, r0 + nrows): ppr 1-KiB pieces per row (16-B chunks c < RF / 4), rows
  // past the padded image are clamped (their results are discarded)
  const int row_chunks = RF / 4;
  const int ppr = (row_chunks + 63) / 64;
  // DIRECT: padded input row pr -> ring slot pr % 13, interleaved RGB, zero padding
  auto direct_rows = [&](int r0, int nrows) {
    for (int t = tid; t < nrows * Wp; t += SPF_NT) {
      const int rr = t / Wp, pp = t - Wp * (t / Wp);
      const int yy = r0 + rr - 3, xx = pp - 3;
      const bool ok = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
      float* d = ring + ((r0 + rr) % SPF_RING) * RF + 3 * pp;
#pragma unroll
      for (int c = 0; c < 3; ++c) d[c] = ok ? ximg[((long long)c * H + yy) * W + xx] : 0.f;
    }
  };
  // wave g stages padded row r0 + g (its 3 plane rows) and later converts that row itself: the
  // staging never crosses waves, so a wave waits only for its own DMA (no extra barrier).  A plane
  // row lands 3 floats in, so staged index = padded column: lane k converts padded columns
  // 4k .. 4k + 3 with 3 aligned 16-B reads and 3 16-B ring writes (12 interleaved floats).
  auto stage_direct = [&](int r0) {
    const int yy = min(max(r0 + g - 3, 0), H - 1);  // out-of-image rows: zeroed at conversion
#pragma unroll
    for (int c = 0; c < 3; ++c)
      if (lane < W / 4) dma16(ximg + ((long long)c * H + yy) * W + 4 * lane, stg + (g * 3 + c) * SPF_SROW + 3);
  };
  auto convert = [&](int r0) {
    const bool rowin = (unsigned)(r0 + g - 3) < (unsigned)H;
    float* d0 = ring + ((r0 + g) % SPF_RING) * RF;
    for (int k = lane; 4 * k < Wp; k += 64) {
      f32x4 v[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = *(const f32x4*)(stg + (g * 3 + c) * SPF_SROW + 4 * k);
      float o[12];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool ok = rowin && (unsigned)(4 * k + e - 3) < (unsigned)W;  // padding columns: 0
#pragma unroll
        for (int c = 0; c < 3; ++c) o[3 * e + c] = ok ? v[c][e] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (12 * k + 4 * i < RF)  // the last group's tail past the row is not written
          *(f32x4*)(d0 + 12 * k + 4 * i) = f32x4{o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]};
    }
  };
  auto stage = [&](int r0, int nrows) {
    for (int p = g; p < nrows * ppr; p += 4) {
      const int rr = p / ppr, pc = p - ppr * (p / ppr);
      const int c = pc * 64 + lane;
      const int row = min(r0 + rr, Hpad - 1);
      if (c < row_chunks)  // EXEC-masked: no write into the next ring row
        dma16(ximg + (long long)row * Wp * 3 + 4 * c, ring + ((r0 + rr) % SPF_RING) * RF + pc * 256);
    }
  };

  // tile k, this lane: stem column 16k + r16 (element 6 * column of a ring row)
  const int xoff = 6 * r16 + q;
  bool colok[NT];
#pragma unroll
  for (int k = 0; k < NT; ++k) colok[k] = 16 * k + r16 < Ws;

  auto stem_row = [&](int sy, f32x4 (&acc)[NT]) {
#pragma unroll
    for (int k = 0; k < NT; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    int rowb[7];  // ring offsets of input rows 2sy .. 2sy + 6 (wave-uniform)
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) rowb[kh] = ((2 * sy + kh) % SPF_RING) * RF;
#pragma unroll
    for (int s = 0; s < SPF_STEPS; ++s) {
      // k = 4s + q lies in kernel row kh0 for q < qs, else kh0 + 1 (the zero-weight k = 147
      // stays in row 6 and reads a real element)
      const int kh0 = (4 * s) / 21;
      const int qs = kh0 < 6 ? 21 * (kh0 + 1) - 4 * s : 4;
      const int b0 = rowb[kh0] + 4 * s - 21 * kh0;
      int off = b0;
      if (qs < 4) off = q < qs ? b0 : rowb[kh0 + 1] + 4 * s - 21 * (kh0 + 1);
      off += (kh0 == 6 && s == SPF_STEPS - 1 && q == 3) ? xoff - 1 : xoff;
#pragma unroll
      for (int k = 0; k < NT; ++k)
        acc[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[s], ring[off + 96 * k], acc[k], 0, 0, 0);
    }
  };

  const float NEG = -INFINITY;
  f32x4 prev[NT];  // stem row 2py - 1
#pragma unroll
  for (int k = 0; k < NT; ++k) prev[k] = f32x4{NEG, NEG, NEG, NEG};
  if (py0 == 0) {
    if constexpr (DIRECT)
      direct_rows(0, SPF_RING);
    else
      stage(0, SPF_RING);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
    // a band below the top starts with stem row 2 py0 - 1 (input rows 4 py0 - 2 .. 4 py0 + 4);
    // rows up to 4 py0 + 8 are the first step's
    if constexpr (DIRECT)
      direct_rows(4 * py0 - 2, 11);
    else
      stage(4 * py0 - 2, 11);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    f32x4 a0[NT];
    stem_row(2 * py0 - 1, a0);
    const bool ok0 = 2 * py0 - 1 < Hs;
#pragma unroll
    for (int k = 0; k < NT; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) prev[k][e] = ok0 && colok[k] ? a0[k][e] : NEG;
    // every wave is done with rows 4 py0 - 2, 4 py0 - 1 before the first step's DMA reuses their slots
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    // DIRECT: the first step's prefetch rows 4 py0 + 9 .. + 12 directly (read from step py0 + 1 on,
    // after that step's barrier)
    if constexpr (DIRECT)
      if (py0 + 1 < py1) direct_rows(4 * py0 + 9, 4);
  }
  // Output by buffer stores (r05): the resource (this image's pooled map) and the row / tile part of
  // the offset are wave-uniform (SGPRs), the lane part one VGPR.  The per-tile 64-bit pointers of the
  // plain stores were 14 VGPRs, two of them spilled: two scratch reloads per step, each waiting
  // (vmcnt(0)) for the step's stores issued before it.
  // bytes per pooled pixel: 64 f32, or (SPLIT) 64 bf16 hi + 64 bf16 lo -- the same 256 B
  constexpr int obytes = 256;
  static_assert(64 * 4 == 2 * 64 * 2, "the f32 and split pooled pixels have one size");
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
      (unsigned char*)y + (long long)img * Hq * Wq * obytes, (short)0, Hq * Wq * obytes, 0x00020000);
  const int yvo = (r16 >> 1) * obytes + (SPLIT ? 2 : 4) * (16 * g + 4 * q);  // lane part
  const bool even = !(r16 & 1);

  for (int py = py0; py < py1; ++py) {
    if constexpr (DIRECT) {
      // rows 4py + 9 .. + 12 (read from step py + 1 on): staged during step py - 1 and landed by
      // its end-of-step wait; step py0's came directly in the prologue.  Then this wave's staging
      // slot takes the next step's row.
      if (py > py0 && py + 1 < py1) convert(4 * py + 9);
      if (py + 2 < py1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own staging reads done before the DMA rewrites it
        stage_direct(4 * py + 13);
      }
    } else if (py + 1 < py1) {
      stage(4 * py + 9, 4);
    }
    f32x4 a1[NT], a2[NT];
    stem_row(2 * py, a1);
    stem_row(2 * py + 1, a2);
    const bool ok1 = 2 * py < Hs, ok2 = 2 * py + 1 < Hs;
    f32x4 v[NT];
#pragma unroll
    for (int k = 0; k < NT; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v2 = ok2 && colok[k] ? a2[k][e] : NEG;  // select: past-the-map columns may be NaN
        v[k][e] = fmaxf(fmaxf(prev[k][e], ok1 && colok[k] ? a1[k][e] : NEG), v2);  // row max
        prev[k][e] = v2;
      }
    // the next step's rows (staged at this step's start) have landed: waited for before the
    // stores, not by a count of younger stores after them (a store whose lanes are all past the
    // map may not be issued at all, so that count is not a constant; loads, stores and LDS-DMA
    // retire in issue order, MI355X_MICROARCH.md)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      const int px = 8 * k + (r16 >> 1);
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // column max: pooled column 8k + i = stem columns 16k + 2i - 1 .. 16k + 2i + 1
        const float left = row_shr1(v[k][e], k ? row_ror1(v[k - 1][e]) : NEG);
        const float c = fmaxf(fmaxf(left, v[k][e]), row_shl1(v[k][e]));
        o[e] = fmaxf(c + bv[e], 0.f);
      }
      if (!even || px >= Wq) continue;
      const int so = (py * Wq + 8 * k) * obytes;  // wave-uniform: pooled row py, tile k
      if constexpr (SPLIT) {
        unsigned hi[2], lo[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const unsigned short h0 = __bfloat16_as_ushort(__float2bfloat16(o[2 * h]));
          const unsigned short h1 = __bfloat16_as_ushort(__float2bfloat16(o[2 * h + 1]));
          const float r0 = o[2 * h] - __uint_as_float((unsigned)h0 << 16);  // exact
          const float r1 = o[2 * h + 1] - __uint_as_float((unsigned)h1 << 16);
          hi[h] = (unsigned)h0 | ((unsigned)h1 << 16);
          lo[h] = (unsigned)__bfloat16_as_ushort(__float2bfloat16(r0)) |
                  ((unsigned)__bfloat16_as_ushort(__float2bfloat16(r1)) << 16);
        }
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64((u32x2){hi[0], hi[1]}, yr, yvo, so, 0);
        __builtin_amdgcn_raw_buffer_store_b64((u32x2){lo[0], lo[1]}, yr, yvo + 128, so, 0);
      } else {
        typedef float f32x4v __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned,
                                                                  (f32x4v){o[0], o[1], o[2], o[3]}),
                                               yr, yvo, so, 0);
      }
    }
    // every wave's next-step rows have landed (the wait above) and it is done reading the slots
    // the step after will overwrite; the stores stay in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// bands per image: fewest (rounds of the grid over the chip's slots) x (stem rows per band)
static int spf_bands(int B, int Hq, int occ) {
  static const int forced = env_switch("EOSV_STEM_BANDS", 0);  // profiling build: fixed band count
  if (forced > 0) return forced;
  const long long slots = (long long)std::max(occ, 1) * device_cu_count();
  int best = 1;
  long long best_cost = -1;
  for (int b = 1; b <= 8 && b <= Hq; ++b) {
    const int rpb = (Hq + b - 1) / b;
    const long long rounds = ((long long)B * b + slots - 1) / slots;
    const long long cost = rounds * (2LL * rpb + (b > 1));
    if (best_cost < 0 || cost < best_cost) best = b, best_cost = cost;
  }
  return best;
}

bool stem_pool_f32_ok(int H, int W) {
  const int Ws = (W + 6 - 7) / 2 + 1;
  return H >= 8 && W >= 8 && (Ws + 15) / 16 <= SPF_MAX_TILES;
}

template <bool SPLIT, int NT, bool DIRECT>
static void launch_nt(const void* x, int B, int H, int W, const void* w, const float* bias, void* y,
                      hipStream_t s, size_t lds, int Hs, int Ws, int Hq, int Wq, int bands) {
  hipLaunchKernelGGL((stem_pool_f32_kernel<SPLIT, NT, DIRECT>), dim3(B * bands), dim3(SPF_NT), lds, s, (const float*)x,
                     (const float*)w, bias, y, H, W, Hs, Ws, Hq, Wq, bands);
}

template <bool SPLIT, bool DIRECT>
static void launch_split(int nt, const void* x, int B, int H, int W, const void* w, const float* bias, void* y,
                         hipStream_t s, size_t lds, int Hs, int Ws, int Hq, int Wq, int bands) {
  switch (nt) {
#define EOSV_SPF_NT(n) \
  case n:              \
    return launch_nt<SPLIT, n, DIRECT>(x, B, H, W, w, bias, y, s, lds, Hs, Ws, Hq, Wq, bands);
    EOSV_SPF_NT(1) EOSV_SPF_NT(2) EOSV_SPF_NT(3) EOSV_SPF_NT(4) EOSV_SPF_NT(5) EOSV_SPF_NT(6) EOSV_SPF_NT(7)
    EOSV_SPF_NT(8)
#undef EOSV_SPF_NT
  }
}

bool stem_pool_f32_direct_ok(int H, int W) { return stem_pool_f32_ok(H, W) && W % 4 == 0 && W <= 256; }

// pack: the padded RGB rows (pack_rgb_pad), or nullptr with `frames` = the f32 NCHW input (DIRECT)
int launch_stem_pool_f32(const void* pack, int B, int H, int W, const void* w, const float* bias, void* y,
                         hipStream_t s, bool split, LaunchInfo* info, const float* frames) {
  const int Hs = (H + 6 - 7) / 2 + 1, Ws = (W + 6 - 7) / 2 + 1;
  const int Hq = (Hs + 2 - 3) / 2 + 1, Wq = (Ws + 2 - 3) / 2 + 1;
  const int nt = (Ws + 15) / 16;
  if (B <= 0) return EOSV_OK;
  if (!stem_pool_f32_ok(H, W) || (frames && !stem_pool_f32_direct_ok(H, W)))
    return set_error("stem_pool_f32: unsupported frame size"), EOSV_ERR_UNSUPPORTED;
  const size_t lds = (size_t)(SPF_RING * spf_row_floats(stem_row_pixels(W, 3)) + SPF_SLACK +
                              (frames ? 12 * SPF_SROW : 0)) * 4;
  if (lds > 163840) return set_error("stem_pool_f32: rows too wide for LDS"), EOSV_ERR_UNSUPPORTED;
  static const int occ_pack = kernel_occupancy((const void*)stem_pool_f32_kernel<false, 7>, SPF_NT, lds);
  static const int occ_direct = kernel_occupancy((const void*)stem_pool_f32_kernel<false, 7, true>, SPF_NT, lds);
  const int occ = frames ? occ_direct : occ_pack;
  const int bands = spf_bands(B, Hq, occ);
  if (info) return record_launch(info, B * bands, occ);
  const void* x = frames ? (const void*)frames : pack;
  if (split && frames)
    launch_split<true, true>(nt, x, B, H, W, w, bias, y, s, lds, Hs, Ws, Hq, Wq, bands);
  else if (split)
    launch_split<true, false>(nt, x, B, H, W, w, bias, y, s, lds, Hs, Ws, Hq, Wq, bands);
  else if (frames)
    launch_split<false, true>(nt, x, B, H, W, w, bias, y, s, lds, Hs, Ws, Hq, Wq, bands);
  else
    launch_split<false, false>(nt, x, B, H, W, w, bias, y, s, lds, Hs, Ws, Hq, Wq, bands);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

}  // namespace eosv
