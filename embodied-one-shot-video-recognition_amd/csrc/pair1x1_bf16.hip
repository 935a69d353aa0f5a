// Fused 1x1 pair for the bf16 bottleneck stage 1 (ResNet-50/101 layer1, 56x56 or 64x64 maps):
// block b's conv3 (1x1 64 -> 256, folded BN, + residual or + the folded 1x1 downsample, ReLU)
// and block b+1's conv1 (1x1 256 -> C1, folded BN, ReLU) in one pass over the pixels
// (torchvision Bottleneck.forward: conv3 -> bn3 -> += identity -> relu, then the next block's
// conv1 -> bn1 -> relu; reference models.py:19 via self.convnet).
//
// Unfused, the 256-channel map Y that conv3 writes is read straight back by the next conv1:
// per pixel X 128 B + R 512 B -> Y 512 B, then Y 512 B -> Z 128 B.  Both 1x1s run at K <= 256
// and are HBM-bound (5.6 TB/s at ~160-290 TF/s).  Here a tile of 64 pixels
// computes Y, stores it (it is block b+1's residual) and keeps it in LDS as the B operand of the
// second GEMM: the Y read (28 % of the pair's bytes) disappears.
//
// Persistent workgroups (one per CU: 104-144 KiB of LDS), 4 waves.  Both folded weight matrices
// stay in LDS for the whole launch; the next tile's X (and residual) are loaded into registers
// while the current one computes, so a CU keeps ~40-50 KiB of reads in flight.
//   GEMM1: D1[256 cout][64 px] = W3 . X^T, wave w owns couts 64w .. 64w + 63 (4 x 4 MFMA tiles)
//   GEMM2: D2[C1 cout][64 px] = W1 . Y^T, wave w owns pixels 16w .. 16w + 15 (C1 / 16 tiles)
// v_mfma_f32_16x16x32_bf16 with the weights as the A operand; weight rows are permuted so that
// MFMA tile i, output row 4q + e holds cout 32(i >> 1) + 8q + 4(i & 1) + e of the wave's 64: a
// lane ends up with channels 8q .. 8q + 7 and 32 + 8q .. 32 + 8q + 7 of one pixel, so each of
// its two 16-B residual loads / output stores per 64 couts covers, with the lane's 3 quad
// neighbours, 64 contiguous bytes of the pixel's row.  K is walked in
// the order of the unfused kernels (32-wide slices, the downsample's columns after conv3's),
// bias then residual then ReLU then round-to-nearest bf16, as their epilogues do: the outputs
// equal the unfused conv3 -> conv1 pair's (tests/native/conv_check.cpp checks both maps).
// LDS rows hold 16-B chunks swizzled chunk ^ (row & 7).
#include <hip/hip_bf16.h>

#include "common.h"

namespace eosv {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

__device__ __forceinline__ float bf2f(u16 v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ u16 f2bf(float f) { return __bfloat16_as_ushort(__float2bfloat16(f)); }
__device__ __forceinline__ int swz(int row, int chunk) { return (chunk ^ (row & 7)) * 8; }
// a tile's buffer resource: num_records 0 past the last tile, so the final prefetch reads zeros
// without touching memory (as pairw_bf16's rounds)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
}
}  // namespace

constexpr int PAIR_BM = 64;  // pixels per tile

template <int C1, bool DS>
__global__ __launch_bounds__(256) void pair1x1_bf16_kernel(Pair1x1Args a) {
  constexpr int K3 = DS ? 128 : 64;  // conv3's K (+ the downsample's 64 input channels)
  constexpr int BM = PAIR_BM;
  constexpr int W3E = 256 * K3, W1E = C1 * 256, XE = BM * K3, YE = BM * 256;
  constexpr int G2 = C1 / 64;  // 64-cout groups of GEMM2
  constexpr int XL = K3 / 32;  // 16-B X chunks per thread per tile
  __shared__ __attribute__((aligned(16))) u16 smem[W3E + W1E + XE + YE];
  u16* const W3s = smem;
  u16* const W1s = W3s + W3E;
  u16* const Xs = W1s + W1E;
  u16* const Ys = Xs + XE;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  const long long ntiles = a.M / BM;
  long long t = blockIdx.x;
  if (t >= ntiles) return;  // the whole workgroup leaves together

  const u16* __restrict__ x = (const u16*)a.x;
  const u16* __restrict__ x2 = (const u16*)a.x2;
  const u16* __restrict__ res = (const u16*)a.res;
  u16* __restrict__ y = (u16*)a.y;
  u16* __restrict__ z = (u16*)a.z;

  // folded-BN shifts of this lane's channels (loaded first: the weight copy's waits retire them,
  // so none is left to wait for inside the tile loop): element k <-> channel 32(k >> 3) + 8q + (k & 7) of
  // the 64-cout group (conv3: group w, conv1: group g)
  float b3v[16], b1v[G2][16];
#pragma unroll
  for (int k = 0; k < 16; ++k) b3v[k] = a.b3[64 * w + 32 * (k >> 3) + 8 * q + (k & 7)];
#pragma unroll
  for (int g = 0; g < G2; ++g)
#pragma unroll
    for (int k = 0; k < 16; ++k) b1v[g][k] = a.b1[64 * g + 32 * (k >> 3) + 8 * q + (k & 7)];

  // weights -> LDS once (rows of K3 / 256 bf16, 16-B chunks swizzled)
  {
    const u16* w3 = (const u16*)a.w3;
    for (int idx = tid; idx < 256 * (K3 / 8); idx += 256) {
      const int row = idx / (K3 / 8), c = idx - row * (K3 / 8);
      *(v4u*)(W3s + row * K3 + swz(row, c)) = *(const v4u*)(w3 + (long long)row * K3 + c * 8);
    }
    const u16* w1 = (const u16*)a.w1;
    for (int idx = tid; idx < C1 * 32; idx += 256) {
      const int row = idx >> 5, c = idx & 31;
      *(v4u*)(W1s + row * 256 + swz(row, c)) = *(const v4u*)(w1 + (long long)row * 256 + c * 8);
    }
  }
  // X (and the downsample's input) of tile t: thread chunk k -> pixel (tid + 256k) / 8 mod 64.
  // Loads go through per-tile buffer resources with empty records past the last tile: the
  // branch-free prefetch of the loop's last iteration then reads nothing.  (It used to re-read
  // tile ntiles - 1, whose residual lines another workgroup is rewriting in place, y = res.)
  v4u xr[XL];
  auto load_x = [&](long long tt) {
    const long long p0 = tt * BM;
    const int nb = tt < ntiles ? BM * 64 * 2 : 0;
    const __amdgpu_buffer_rsrc_t rx = tile_rsrc(x + p0 * 64, nb);
    const __amdgpu_buffer_rsrc_t rx2 = tile_rsrc((DS ? x2 : x) + p0 * 64, nb);
#pragma unroll
    for (int k = 0; k < XL; ++k) {
      const int idx = tid + 256 * (k & 1);
      const int px = idx >> 3, c = idx & 7;
      xr[k] = __builtin_amdgcn_raw_buffer_load_b128((DS && k >= 2) ? rx2 : rx, (px * 64 + c * 8) * 2, 0, 0);
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int k = 0; k < XL; ++k) {
      const int idx = tid + 256 * (k & 1);
      const int px = idx >> 3, c = (idx & 7) + ((DS && k >= 2) ? 8 : 0);
      *(v4u*)(Xs + px * K3 + swz(px, c)) = xr[k];
    }
  };
  // residual of tile t for this lane: pixel 16j + r, channels 64w + 32hh + 8q .. + 7
  v4u rr[DS ? 1 : 8];
  auto load_r = [&](long long tt) {
    if constexpr (!DS) {
      const long long p0 = tt * BM;
      const __amdgpu_buffer_rsrc_t rres = tile_rsrc(res + p0 * 256, tt < ntiles ? BM * 256 * 2 : 0);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
          rr[2 * j + hh] = __builtin_amdgcn_raw_buffer_load_b128(rres, ((16 * j + r) * 256 + 8 * q) * 2,
                                                                 (64 * w + 32 * hh) * 2, 0);
    }
  };
  load_x(t);
  load_r(t);
  store_x();
  const float rlow = 0.f;  // both convs end in ReLU

  for (; t < ntiles; t += gridDim.x) {
    const long long p0 = t * BM;
    // the next tile (past the end: empty records, branch-free, so the compiler counts the loads
    // in flight instead of draining them at the join)
    const long long tn = t + gridDim.x;
    // (A): X tile (and, first time round, the weights) in LDS; the previous tile's GEMM2 is done with Ys
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    load_x(tn);
    __builtin_amdgcn_sched_barrier(0);  // issued here, not sunk below GEMM1

    // GEMM1: wave w, couts 64w + (tile i, row 4q' + e -> 32(i >> 1) + 8q' + 4(i & 1) + e), pixels 16j + r
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < K3 / 32; ++s) {
      bf16x8 af[4], bx[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = 64 * w + 32 * (i >> 1) + 8 * (r >> 2) + 4 * (i & 1) + (r & 3);
        af[i] = *(const bf16x8*)(W3s + row * K3 + swz(row, 4 * s + q));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = 16 * j + r;
        bx[j] = *(const bf16x8*)(Xs + row * K3 + swz(row, 4 * s + q));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bx[j], acc[i][j], 0, 0, 0);
    }
    // epilogue 1: + shift (+ residual), ReLU, bf16 -> Y (global: block b+1's residual) and Ys
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int prow = 16 * j + r;
      const int c0 = 64 * w + 8 * q;  // + 32hh
      float v[16];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * i + e] = acc[i][j][e] + b3v[4 * i + e];
      if constexpr (!DS) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const v4u r4 = rr[2 * j + hh];
          const unsigned ru[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            v[8 * hh + 2 * k] += bf2f((u16)(ru[k] & 0xffff));
            v[8 * hh + 2 * k + 1] += bf2f((u16)(ru[k] >> 16));
          }
        }
      }
      v4u pk[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const u16 lo = f2bf(fmaxf(v[8 * hh + 2 * k], rlow)), hi = f2bf(fmaxf(v[8 * hh + 2 * k + 1], rlow));
          pk[hh][k] = (unsigned)lo | ((unsigned)hi << 16);
        }
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        *(v4u*)(y + (p0 + prow) * 256 + c0 + 32 * hh) = pk[hh];
        *(v4u*)(Ys + prow * 256 + swz(prow, c0 / 8 + 4 * hh)) = pk[hh];
      }
    }
    load_r(tn);
    // (B): Ys complete; every wave is done reading Xs
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    // GEMM2: wave w, pixels 16w + r, couts 64g + (tile i, row 4q' + e -> 32(i >> 1) + 8q' + 4(i & 1) + e)
    f32x4 acc2[G2][4];
#pragma unroll
    for (int g = 0; g < G2; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc2[g][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int prow = 16 * w + r;
      const bf16x8 by = *(const bf16x8*)(Ys + prow * 256 + swz(prow, 4 * s + q));
#pragma unroll
      for (int g = 0; g < G2; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 64 * g + 32 * (i >> 1) + 8 * (r >> 2) + 4 * (i & 1) + (r & 3);
          const bf16x8 aw = *(const bf16x8*)(W1s + row * 256 + swz(row, 4 * s + q));
          acc2[g][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw, by, acc2[g][i], 0, 0, 0);
        }
    }
    // the next X tile -> Xs (free since (B)), here rather than at the loop head: hipcc counts only
    // loads in vmcnt, so at the head its wait for X also drained this tile's Z stores
    __builtin_amdgcn_sched_barrier(0);
    store_x();
    __builtin_amdgcn_sched_barrier(0);
    // epilogue 2: + shift, ReLU, bf16 -> Z
    {
      const long long p = p0 + 16 * w + r;
#pragma unroll
      for (int g = 0; g < G2; ++g) {
        const int c0 = 64 * g + 8 * q;  // + 32hh
        v4u pk[2];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            // element 8hh + 2k of the lane's 16 channels = tile i = (8hh + 2k) / 4, row e = (8hh + 2k) % 4
            const int c = 8 * hh + 2 * k;
            const float v0 = acc2[g][c >> 2][c & 3] + b1v[g][c];
            const float v1 = acc2[g][(c + 1) >> 2][(c + 1) & 3] + b1v[g][c + 1];
            pk[hh][k] = (unsigned)f2bf(fmaxf(v0, rlow)) | ((unsigned)f2bf(fmaxf(v1, rlow)) << 16);
          }
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) *(v4u*)(z + p * C1 + c0 + 32 * hh) = pk[hh];
      }
    }
  }
}

bool pair1x1_bf16_ok(int cmid, int cexp, int c1, int cds, long long M) {
  return cmid == 64 && cexp == 256 && (c1 == 64 || c1 == 128) && (cds == 0 || cds == 64) && !(cds && c1 == 128) &&
         M > 0 && M % PAIR_BM == 0;
}

template <int C1, bool DS>
static int launch_pair(const Pair1x1Args& a, long long ntiles, hipStream_t s) {
  static const int occ = kernel_occupancy((const void*)pair1x1_bf16_kernel<C1, DS>, 256);
  if (a.plan) return record_launch(a.plan, ntiles, occ);
  const long long grid = std::min<long long>(ntiles, (long long)occ * device_cu_count());
  hipLaunchKernelGGL((pair1x1_bf16_kernel<C1, DS>), dim3((unsigned)grid), dim3(256), 0, s, a);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

#ifndef EOSV_PAIR_R_DEF
#define EOSV_PAIR_R_DEF 1
#endif

int launch_pair1x1_bf16(const Pair1x1Args& a, hipStream_t s) {
  if (!pair1x1_bf16_ok(64, 256, a.c1, a.cds, a.M) || !a.x || !a.w3 || !a.b3 || !a.w1 || !a.b1 || !a.y || !a.z ||
      (a.cds ? !a.x2 : !a.res))
    return set_error("pair1x1_bf16: unsupported shape"), EOSV_ERR_UNSUPPORTED;
  // 1: pair1x1r_bf16 (pixels per wave; A/B switch; r04: R50 layer1.0 pair 1.96 -> 1.64 ms, layer1.2
  // pair 2.83 -> 2.50, layer1.1 pair 2.34 -> 2.33, bit-identical)
  static const int pr = env_switch("EOSV_PAIR_R", EOSV_PAIR_R_DEF);
  if (pr) return launch_pair1x1r_bf16(a, s);
  const long long ntiles = a.M / PAIR_BM;
  if (a.cds) return launch_pair<64, true>(a, ntiles, s);
  if (a.c1 == 64) return launch_pair<64, false>(a, ntiles, s);
  return launch_pair<128, false>(a, ntiles, s);
}

}  // namespace eosv
