// Fused 1x1 pair for the bf16 bottleneck stage 1 with the pixels owned per wave (r04,
// EOSV_PAIR_R): block b's conv3 (1x1 64 -> 256, folded BN, + residual or + the folded stride-1
// downsample, ReLU) and block b+1's conv1 (1x1 256 -> C1, folded BN, ReLU), as pair1x1_bf16
// (reference models.py:19 via self.convnet; torchvision Bottleneck.forward).
//
// pair1x1_bf16 splits GEMM1 by output channels and GEMM2 by pixels over its 4 waves, so Y goes
// through an LDS tile, two barriers per 64-pixel tile, and each wave holds the next tile's X and
// residual in registers: ~40 KiB of loads in flight per CU, the pair at 4.5-5.2 TB/s of its
// algorithmic bytes.  Here, as in pairw_bf16, a wave owns 16 NPT pixels for both GEMMs:
//   * both folded weight matrices stay in LDS for the whole launch (64-96 KiB, read-only after
//     the first barrier: no ring, no barrier in the pixel loop);
//   * GEMM1 per 64-channel chunk of Y: D1[64 cout][16 px] = W3c . X^T with the weight rows read in
//     the permuted order of pairw_bf16 (tile i, row 4q + e -> cout 32(i >> 1) + 8q + 4(i & 1) + e),
//     so a lane ends up with channels 8q .. 8q + 7 and 32 + 8q .. + 7 of its pixel: 16-B residual
//     loads and Y stores, and after bias + residual + ReLU + bf16 exactly the GEMM2 B fragments
//     of the chunk's two k-slices;
//   * GEMM2 accumulates D2[C1][16 px] += W1c . Ychunk^T over the 4 chunks, then bias + ReLU -> Z;
//   * 8 waves (two per SIMD), each with its own loads in flight: the residual of chunk ch + RD
//     and the next round's X (during the last chunk), so a CU keeps ~100 KiB of loads in flight.
// K orders and epilogue orders are the unfused kernels': outputs bit-identical to conv3 -> conv1
// (tests/native/conv_check.cpp).  Loads and stores go through buffer resources bounded at M, so
// the tail round's missing pixels read 0 and are not stored.
#include <hip/hip_bf16.h>

#include "common.h"

namespace eosv {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

__device__ __forceinline__ int swz(int row, int chunk) { return (chunk ^ (row & 7)) * 8; }
// MFMA tile i, row t (0..15) -> channel within the 64-channel group
__device__ __forceinline__ int permrow(int i, int t) { return 32 * (i >> 1) + 8 * (t >> 2) + 4 * (i & 1) + (t & 3); }
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(bytes > 0x7fffffffLL ? 0x7fffffffLL : (bytes < 0 ? 0 : bytes)),
                                           0x00020000);
}
}  // namespace

constexpr int PR_NW = 8;  // waves per workgroup

template <int C1, bool DS, int NPT>
__global__ __launch_bounds__(64 * PR_NW) void pair1x1r_bf16_kernel(Pair1x1Args a) {
  constexpr int K3 = DS ? 128 : 64;   // conv3's K (+ the downsample's 64 input channels)
  constexpr int XS = K3 / 32;         // X k-slices per pixel tile
  constexpr int G2 = C1 / 64;         // 64-cout groups of GEMM2
  constexpr int NCH = 4;              // 64-channel chunks of Y (256)
  constexpr int PX = 16 * NPT;        // pixels per wave per round
  constexpr int TILE = PX * PR_NW;    // pixels per round
  constexpr int RD = NPT == 1 && C1 == 64 ? 2 : 1;  // residual chunks loaded ahead (2 spilled 5-6 VGPRs at NPT 2 or C1 128)
  constexpr int NRS = 4;              // residual register sets: a ring of NCH, so a chunk's set is the same in every round
  __shared__ __attribute__((aligned(16))) u16 smem[256 * K3 + C1 * 256 + 2 * (256 + C1)];
  u16* const W3s = smem;
  u16* const W1s = W3s + 256 * K3;
  float* const b3s = (float*)(W1s + C1 * 256);
  float* const b1s = b3s + 256;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  const long long M = a.M;
  const long long nrounds = (M + TILE - 1) / TILE;
  long long rt = blockIdx.x;  // launch: gridDim.x <= nrounds

  // weights and shifts -> LDS once (rows of K3 / 256 bf16, 16-B chunks swizzled)
  {
    const u16* w3 = (const u16*)a.w3;
    for (int idx = tid; idx < 256 * (K3 / 8); idx += 64 * PR_NW) {
      const int row = idx / (K3 / 8), c = idx - row * (K3 / 8);
      *(v4u*)(W3s + row * K3 + swz(row, c)) = *(const v4u*)(w3 + (long long)row * K3 + c * 8);
    }
    const u16* w1 = (const u16*)a.w1;
    for (int idx = tid; idx < C1 * 32; idx += 64 * PR_NW) {
      const int row = idx >> 5, c = idx & 31;
      *(v4u*)(W1s + row * 256 + swz(row, c)) = *(const v4u*)(w1 + (long long)row * 256 + c * 8);
    }
    for (int i = tid; i < 256; i += 64 * PR_NW) b3s[i] = a.b3[i];
    for (int i = tid; i < C1; i += 64 * PR_NW) b1s[i] = a.b1[i];
  }
  __syncthreads();

  // per-round buffer resources based at the round's first pixel, bounded at M (the tail round's
  // missing pixels read 0, their stores are dropped; a round past the last one: empty records)
  struct RoundRes {
    __amdgpu_buffer_rsrc_t x, x2, res, y, z;
  };
  auto round_res = [&](long long t) {
    RoundRes rr;
    const long long p0 = t * TILE;
    const long long n = t < nrounds ? (M - p0 < TILE ? M - p0 : TILE) : 0;
    rr.x = rsrc((const u16*)a.x + p0 * 64, n * 64 * 2);
    rr.x2 = rsrc((const u16*)(DS ? a.x2 : a.x) + p0 * 64, n * 64 * 2);
    rr.res = rsrc((const u16*)(DS ? a.x : a.res) + p0 * 256, DS ? 0 : n * 256 * 2);
    rr.y = rsrc((u16*)a.y + p0 * 256, n * 256 * 2);
    rr.z = rsrc((u16*)a.z + p0 * C1, n * C1 * 2);
    return rr;
  };
  const int pw = PX * w + r;  // the lane's pixel of tile tt within the round: pw + 16 tt
  auto load_x = [&](const RoundRes& rr, v4u (*xf)[XS]) {
#pragma unroll
    for (int tt = 0; tt < NPT; ++tt)
#pragma unroll
      for (int s = 0; s < XS; ++s)
        xf[tt][s] = __builtin_amdgcn_raw_buffer_load_b128(s < 2 ? rr.x : rr.x2, ((pw + 16 * tt) * 64 + 8 * q) * 2,
                                                          64 * (s & 1), 0);
  };
  auto load_r = [&](const RoundRes& rr, int ch, v4u (*rv)[2]) {
#pragma unroll
    for (int tt = 0; tt < NPT; ++tt)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
        rv[tt][hh] = __builtin_amdgcn_raw_buffer_load_b128(rr.res, ((pw + 16 * tt) * 256 + 8 * q) * 2,
                                                           (ch * 64 + 32 * hh) * 2, 0);
  };

  RoundRes cur = round_res(rt);
  v4u xf[NPT][XS], rres[NRS][NPT][2];
  load_x(cur, xf);
  if constexpr (!DS) {
#pragma unroll
    for (int c = 0; c < RD; ++c) load_r(cur, c, rres[c]);
  }

  for (; rt < nrounds; rt += gridDim.x) {
    // the weight fragments are the same every round: without this compiler barrier they were
    // hoisted out of the round loop (all 4 chunks' fragments live at once: 232-328 VGPRs spilled)
    asm volatile("" ::: "memory");
    const RoundRes nxt = round_res(rt + gridDim.x);
    f32x4 acc2[NPT][G2][4];
#pragma unroll
    for (int tt = 0; tt < NPT; ++tt)
#pragma unroll
      for (int g = 0; g < G2; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc2[tt][g][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the 4 chunks fully unrolled: every residual register set is compile-time per chunk
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      asm volatile("" ::: "memory");  // (the same per chunk: fragments read where they are used)
      if constexpr (!DS) {  // residual of chunk ch + RD (the next round's first chunks in the last ones)
        const bool here = ch + RD < NCH;
        RoundRes rr;
        rr.res = here ? cur.res : nxt.res;
        load_r(rr, here ? ch + RD : ch + RD - NCH, rres[(ch + RD) % NRS]);
      }
      // GEMM1: D1[64 chunk couts (permuted tiles i)][16 px] over the XS k-slices
      f32x4 acc1[NPT][4];
#pragma unroll
      for (int tt = 0; tt < NPT; ++tt)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc1[tt][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < XS; ++s) {
        bf16x8 af[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 64 * ch + permrow(i, r);
          af[i] = *(const bf16x8*)(W3s + row * K3 + swz(row, 4 * s + q));
        }
#pragma unroll
        for (int tt = 0; tt < NPT; ++tt) {
          const bf16x8 bx = __builtin_bit_cast(bf16x8, xf[tt][s]);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc1[tt][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bx, acc1[tt][i], 0, 0, 0);
        }
      }
      if (ch == NCH - 1) load_x(nxt, xf);  // the round's X is dead: the next round's goes into the same registers
      // epilogue 1: + shift (+ residual), ReLU, bf16 -> Y (global) and the GEMM2 B fragments
      bf16x8 yf[NPT][2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int c0 = 64 * ch + 32 * hh + 8 * q;
        const f32x4 bA = *(const f32x4*)(b3s + c0), bB = *(const f32x4*)(b3s + c0 + 4);
#pragma unroll
        for (int tt = 0; tt < NPT; ++tt) {
          const v4u rv = DS ? v4u{0, 0, 0, 0} : rres[ch % NRS][tt][hh];
          v4u pk;
#pragma unroll
          for (int k = 0; k < 4; ++k) {  // packed (common.h, epi): bitwise the scalar form
            epi::f32x2 v = epi::pair_of(acc1[tt][2 * hh], acc1[tt][2 * hh + 1], k) + epi::pair_of(bA, bB, k);
            if constexpr (!DS) v += epi::bf2_f(rv[k]);
            pk[k] = epi::relu_bf2(v);
          }
          store_b128_guarded(pk, cur.y, ((pw + 16 * tt) * 256 + 8 * q) * 2, (ch * 64 + 32 * hh) * 2);
          yf[tt][hh] = __builtin_bit_cast(bf16x8, pk);
        }
      }
      // GEMM2: D2[64g + permuted rows][px] += W1[.., k-slice s2 of the chunk] . Ychunk
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int g = 0; g < G2; ++g) {
          bf16x8 aw[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = 64 * g + permrow(i, r);
            aw[i] = *(const bf16x8*)(W1s + row * 256 + swz(row, 8 * ch + 4 * s2 + q));
          }
#pragma unroll
          for (int tt = 0; tt < NPT; ++tt)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              acc2[tt][g][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[i], yf[tt][s2], acc2[tt][g][i], 0, 0, 0);
        }
    }
    // epilogue 2: + shift, ReLU, bf16 -> Z
#pragma unroll
    for (int tt = 0; tt < NPT; ++tt)
#pragma unroll
      for (int g = 0; g < G2; ++g)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int c0 = 64 * g + 32 * hh + 8 * q;
          const f32x4 bA = *(const f32x4*)(b1s + c0), bB = *(const f32x4*)(b1s + c0 + 4);
          v4u pk;
#pragma unroll
          for (int k = 0; k < 4; ++k)
            pk[k] = epi::relu_bf2(epi::pair_of(acc2[tt][g][2 * hh], acc2[tt][g][2 * hh + 1], k) + epi::pair_of(bA, bB, k));
          store_b128_guarded(pk, cur.z, ((pw + 16 * tt) * C1 + 8 * q) * 2, (64 * g + 32 * hh) * 2);
        }
    cur = nxt;
  }
}

template <int C1, bool DS, int NPT>
static int launch_pr(const Pair1x1Args& a, hipStream_t s) {
  constexpr int TILE = 16 * NPT * PR_NW;
  static const int occ = kernel_occupancy((const void*)pair1x1r_bf16_kernel<C1, DS, NPT>, 64 * PR_NW);
  const long long nrounds = (a.M + TILE - 1) / TILE;
  if (a.plan) return record_launch(a.plan, nrounds, occ);
  const long long grid = std::min<long long>(nrounds, (long long)occ * device_cu_count());
  hipLaunchKernelGGL((pair1x1r_bf16_kernel<C1, DS, NPT>), dim3((unsigned)grid), dim3(64 * PR_NW), 0, s, a);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

// the stage-1 pair shapes pair1x1_bf16 takes (cmid 64, cexp 256, c1 64 / 128, the stride-1
// downsample only with c1 64), any M
int launch_pair1x1r_bf16(const Pair1x1Args& a, hipStream_t s) {
  if (a.M <= 0 || !(a.c1 == 64 || a.c1 == 128) || !(a.cds == 0 || (a.cds == 64 && a.c1 == 64)) || !a.x || !a.w3 ||
      !a.b3 || !a.w1 || !a.b1 || !a.y || !a.z || (a.cds ? !a.x2 : !a.res))
    return set_error("pair1x1r_bf16: unsupported shape"), EOSV_ERR_UNSUPPORTED;
  if (a.cds) return launch_pr<64, true, 2>(a, s);
  static const int npt1 = env_switch("EOSV_PAIR_R_NPT1", 0);  // 1: the residual c1-64 pair on 128-pixel rounds (A/B switch)
  if (a.c1 == 64) return npt1 ? launch_pr<64, false, 1>(a, s) : launch_pr<64, false, 2>(a, s);
  return launch_pr<128, false, 1>(a, s);
}

}  // namespace eosv
