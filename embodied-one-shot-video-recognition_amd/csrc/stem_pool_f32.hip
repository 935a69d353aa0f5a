// Fused ResNet stem for f32: conv 7x7/2 p3 (3 -> 64, folded BN) + ReLU + maxpool 3x3/2 p1,
// torchvision's convnet.0-3 (reference models.py:19 via self.convnet); the f32 sibling of
// stem_pool_bf16.hip.
//
// The unfused f32 pair wrote the 112 x 112 x 64 f32 stem map (3.2 MB per frame) and read it back
// in the pool (8.2 + 2.5 ms per 3200-frame chunk).  Here one workgroup walks one image top to
// bottom, as in the bf16 kernel:
//  * wave t owns pooled columns 7t .. 7t+6, i.e. the 16 stem columns 14t-1 .. 14t+14;
//  * per pooled row py it computes stem rows 2py and 2py+1 (2py-1 is kept from the previous
//    step), takes the row max and then the column max (DPP row shifts) of the raw accumulators,
//    and only then adds the BN shift and applies ReLU for the 7 pooled pixels x 64 channels it
//    stores.  fl(a + b) is monotone in a and ReLU commutes with max, so this is bit-identical
//    to stem conv -> shift -> ReLU -> maxpool on the same accumulators.
//
// MFMA: v_mfma_f32_16x16x4_f32 (exact f32, a k-ordered fma chain) with D = W . X^T (rows =
// output channels, columns = stem pixels), dense K = [kh 7][21] (kw*3 + c) + 1 zero = 148 = 37
// k-steps of 4 (the padded [kh][24] layout took 42).  Element k of lane q's step reads input
// row 2*sy + k/21, element 6*sx + k%21: a step whose 4 k straddle two kernel rows picks the
// row base per lane (one v_cndmask between two wave-uniform bases), so it is still one
// ds_read_b32 per lane.  Weights live in LDS permuted so that one ds_read_b128 gives a lane
// its A values for 4 consecutive steps: Wl[j][t][r16][q][i] = W[16j + r16][16t + 4i + q].
//
// LDS: weights 40 KiB | a ring of 13 input rows (row r in slot r % 13; a step needs rows
// 4py .. 4py+8 and prefetches 4py+9 .. 4py+12), each row Wp * 3 floats padded to 16 B,
// filled by LDS-DMA from the dense padded RGB pack (8-B aligned sources).  ~80 KiB: two
// workgroups (16 waves) per CU.
#include <hip/hip_bf16.h>

#include "common.h"

namespace eosv {

namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int SPF_MAX_TILES = 8;   // pooled width <= 56
constexpr int SPF_K = 147;         // real K: 7 kernel rows x 21 (kw*3 + c)
constexpr int SPF_STEPS = 37;      // k-steps of 4 over dense K = 148
constexpr int SPF_GROUPS = 10;     // b128 weight groups of 4 steps (40 steps, the last 3 zero)
constexpr int SPF_KW = 176;        // uploaded f32 stem weight row ([kh][24] + 8 zero)
constexpr int SPF_RING = 13;
constexpr int SPF_W_FLOATS = 4 * SPF_GROUPS * 16 * 16;  // 10240 floats = 40 KiB

__host__ __device__ constexpr int spf_row_floats(int Wp) { return (Wp * 3 + 3) & ~3; }

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
}  // namespace

// x: padded f32 RGB [N][H+6][Wp][3] (stem_row_pixels), w: [64][176] f32, bias [64] f32,
// y: [N][Hq][Wq][64] f32 (pooled).  Grid = N images, block = 64 * ntiles threads.
// SPLIT (EOSV_F32X3): y is [N][Hq][Wq][128] bf16, (hi, lo) of each pooled f32 value.
template <bool SPLIT>
__global__ __launch_bounds__(64 * SPF_MAX_TILES, 2) void stem_pool_f32_kernel(const float* __restrict__ x,
                                                                             const float* __restrict__ w,
                                                                             const float* __restrict__ bias, void* y,
                                                                             int H, int W, int Hs, int Ws, int Hq,
                                                                             int Wq) {
  extern __shared__ __attribute__((aligned(16))) float spf_smem[];
  const int ntiles = blockDim.x >> 6;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int r16 = lane & 15;
  const int q = lane >> 4;
  const int img = blockIdx.x;
  const int Wp = stem_row_pixels(W, 3);
  const int RF = spf_row_floats(Wp);  // ring row stride (floats)
  const int Hpad = H + 6;
  float* Wl = spf_smem;
  float* ring = spf_smem + SPF_W_FLOATS;
  const float* ximg = x + (long long)img * Hpad * Wp * 3;

  // weights -> LDS, permuted (see header); plain loads, once per image
  for (int e = tid; e < SPF_W_FLOATS; e += blockDim.x) {
    const int i = e & 3, qq = (e >> 2) & 3, rr = (e >> 4) & 15, t = (e >> 8) % SPF_GROUPS, j = e / (256 * SPF_GROUPS);
    const int k = 16 * t + 4 * i + qq;  // dense k -> uploaded [kh][24] column
    Wl[e] = k < SPF_K ? w[(j * 16 + rr) * SPF_KW + 24 * (k / 21) + k % 21] : 0.f;
  }
  f32x4 bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bv[j] = *(const f32x4*)(bias + j * 16 + 4 * q);

  // DMA of input rows [r0, r0 + nrows): 3 pieces per row (16-B chunks c < RF / 4), rows past
  // the padded image are clamped (their results are discarded)
  const int row_chunks = RF / 4;
  auto stage = [&](int r0, int nrows) {
    for (int p = wid; p < nrows * 3; p += ntiles) {
      const int rr = p / 3, pc = p - 3 * (p / 3);
      const int c = pc * 64 + lane;
      const int row = min(r0 + rr, Hpad - 1);
      if (c < row_chunks)  // EXEC-masked: no write into the next ring row
        dma16(ximg + (long long)row * Wp * 3 + 4 * c, ring + ((r0 + rr) % SPF_RING) * RF + pc * 256);
    }
  };

  // this lane's stem column; columns outside the map enter the pool as -inf (clamped read)
  const int sx = 14 * wid - 1 + r16;
  const bool colok = sx >= 0 && sx < Ws;
  const int xoff = 6 * max(sx, 0) + q;  // + ring row base + 4s - 21 kh per step

  auto stem_row = [&](int sy, f32x4 (&acc)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int rowb[7];  // ring offsets of input rows 2sy .. 2sy + 6 (wave-uniform)
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) rowb[kh] = ((2 * sy + kh) % SPF_RING) * RF;
#pragma unroll
    for (int t = 0; t < SPF_GROUPS; ++t) {
      f32x4 wa[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) wa[j] = *(const f32x4*)(Wl + (((j * SPF_GROUPS + t) * 16 + r16) * 4 + q) * 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int s = 4 * t + i;
        if (s >= SPF_STEPS) break;
        // k = 4s + q lies in kernel row kh0 for q < qs, else kh0 + 1 (the zero-weight k = 147
        // stays in row 6 and reads a real element)
        const int kh0 = (4 * s) / 21;
        const int qs = kh0 < 6 ? 21 * (kh0 + 1) - 4 * s : 4;
        const int b0 = rowb[kh0] + 4 * s - 21 * kh0;
        int off = b0;
        if (qs < 4) off = q < qs ? b0 : rowb[kh0 + 1] + 4 * s - 21 * (kh0 + 1);
        const float xb = ring[off + (kh0 == 6 && s == SPF_STEPS - 1 && q == 3 ? xoff - 1 : xoff)];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[j][i], xb, acc[j], 0, 0, 0);
      }
    }
  };

  stage(0, SPF_RING);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // weights (plain LDS stores) and the first rows

  const float NEG = -INFINITY;
  f32x4 prev[4];  // stem row 2py - 1
#pragma unroll
  for (int j = 0; j < 4; ++j) prev[j] = f32x4{NEG, NEG, NEG, NEG};
  float* yimg = (float*)y + (long long)img * Hq * Wq * 64;
  unsigned short* ysp = (unsigned short*)y + (long long)img * Hq * Wq * 128;
  const int px = 7 * wid + (r16 >> 1);  // pooled column this lane writes (even r16 <= 12)
  const bool writer = !(r16 & 1) && r16 <= 12 && px < Wq;

  for (int py = 0; py < Hq; ++py) {
    if (py + 1 < Hq) stage(4 * py + 9, 4);
    f32x4 a1[4], a2[4];
    stem_row(2 * py, a1);
    stem_row(2 * py + 1, a2);
    const bool ok1 = colok && 2 * py < Hs, ok2 = colok && 2 * py + 1 < Hs;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v2 = ok2 ? a2[j][e] : NEG;
        const float v = fmaxf(fmaxf(prev[j][e], ok1 ? a1[j][e] : NEG), v2);  // row max
        prev[j][e] = v2;
        // column max: pooled column i of this tile = stem columns r16 = 2i, 2i+1, 2i+2
        const float c = fmaxf(fmaxf(v, row_shl(v, 1)), row_shl(v, 2));
        o[e] = fmaxf(c + bv[j][e], 0.f);
      }
      if (!writer) continue;
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
        unsigned short* d = ysp + ((long long)py * Wq + px) * 128 + j * 16 + 4 * q;
        *(uint2*)d = make_uint2(hi[0], hi[1]);
        *(uint2*)(d + 64) = make_uint2(lo[0], lo[1]);
      } else {
        *(float4*)(yimg + ((long long)py * Wq + px) * 64 + j * 16 + 4 * q) = make_float4(o[0], o[1], o[2], o[3]);
      }
    }
    // next step's rows have landed (their DMA is older than this step's 4 stores) and every
    // wave is done reading the slots the step after will overwrite
    asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

bool stem_pool_f32_ok(int H, int W) {
  const int Ws = (W + 6 - 7) / 2 + 1;
  const int Wq = (Ws + 2 - 3) / 2 + 1;
  return H >= 8 && W >= 8 && (Wq + 6) / 7 <= SPF_MAX_TILES;
}

int launch_stem_pool_f32(const void* pack, int B, int H, int W, const void* w, const float* bias, void* y,
                         hipStream_t s, bool split, LaunchInfo* info) {
  const int Hs = (H + 6 - 7) / 2 + 1, Ws = (W + 6 - 7) / 2 + 1;
  const int Hq = (Hs + 2 - 3) / 2 + 1, Wq = (Ws + 2 - 3) / 2 + 1;
  const int ntiles = (Wq + 6) / 7;
  if (B <= 0) return EOSV_OK;
  if (ntiles > SPF_MAX_TILES) return set_error("stem_pool_f32: too wide"), EOSV_ERR_UNSUPPORTED;
  const size_t lds = (size_t)(SPF_W_FLOATS + SPF_RING * spf_row_floats(stem_row_pixels(W, 3))) * 4;
  if (lds > 163840) return set_error("stem_pool_f32: rows too wide for LDS"), EOSV_ERR_UNSUPPORTED;
  if (info) {
    static const int occ = kernel_occupancy((const void*)stem_pool_f32_kernel<false>, 64 * ntiles, lds);
    return record_launch(info, B, occ);
  }
  if (split)
    hipLaunchKernelGGL(stem_pool_f32_kernel<true>, dim3(B), dim3(64 * ntiles), lds, s, (const float*)pack,
                       (const float*)w, bias, y, H, W, Hs, Ws, Hq, Wq);
  else
    hipLaunchKernelGGL(stem_pool_f32_kernel<false>, dim3(B), dim3(64 * ntiles), lds, s, (const float*)pack,
                       (const float*)w, bias, y, H, W, Hs, Ws, Hq, Wq);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

}  // namespace eosv
