// Row-strip 3x3 conv for bf16 (stride 1, pad 1, Cin a multiple of 64 above 64, Cout a multiple
// of 128): the stride-1 3x3 convs of ResNet stages 2-4 (28x28 / 14x14 / 7x7 maps at 224x224,
// 32 / 16 / 8 at 256x256), torchvision BasicBlock / Bottleneck conv2 (reference models.py:19 via
// self.convnet, driven from network_test.py:59 and :79).
//
// Why: the implicit GEMM (conv_bf16.hip, 256x256 tile) stages 64 KiB per
// 64-deep K-step -- 32 KiB of im2col rows (the same input pixels again for each of the 9 taps)
// and 32 KiB of weights -- and runs at ~15 B/clk of staging with the MFMAs and the staging adding
// up rather than overlapping (0.65 ms per 3200-frame stage-3 conv, MFMA-busy 0.46).  Here a
// workgroup stages, per 64-channel chunk, the input rows of its strip ONCE (the halo) and only
// the weights move per tap: 16 KiB + 1/9 of the halo per tap, 2.4x fewer staged bytes per FLOP.
//
// Slot space.  The maps are laid out as one tall image: row g = img * (H + 1) + ih + 1 holds
// input row ih of image img (g = img * (H + 1), i.e. ih = -1, is a zero row shared with the
// previous image's ih = H), and each row has RW = W + 1 slots, slot 0 the zero column shared by
// the row's left and the previous row's right padding.  Output pixel (img, oh, ow) is output
// slot o = (img * (H + 1) + oh) * RW + ow, and tap (kh, kw) reads input slot o + kh * RW + kw:
// every tap of a 16-slot MFMA tile is 16 consecutive slots.  Output slots with ow = W, or on the
// separator row (oh = H), are computed and dropped (14x14 maps: 13 % of the slots).
//
// Tile: R = floor(448 / RW) output rows of the slot space (448 slots = 28 MFMA tiles, the last
// 448 - R * RW dropped) x 128 couts.  8 waves: wave (wm, wn) owns slots 112 wm .. + 111 (7
// tiles) x couts 64 wn .. + 63 (4 tiles).  D = W . X^T on v_mfma_f32_16x16x32_bf16 (weights the
// A operand, with pairw_bf16's permuted rows: a lane ends up with 8 + 8 consecutive couts of one
// pixel, so the epilogue stores 16 B per lane straight from registers).
//
// K loop: per 64-channel chunk c, the taps t = 0..8 (the stored chunk-major K order,
// ConvArgs::kcm: (cin / 64, kh, kw, cin % 64)), two 32-wide k-slices per tap: the accumulation
// order of the implicit GEMM's kcm path.  LDS (160 KiB, one workgroup per CU): two halo buffers
// of 512 slots x 128 B (chunk c + 1's halo is DMA'd one piece per wave per tap during chunk c's
// taps 0..7) and a 2-slot weight ring (tap t + 1's 16 KiB during tap t).  One barrier per tap;
// at its end the next tap's weights (and at a chunk's last tap the next halo) must have landed:
// the wait counts only this tap's halo piece as younger.  16-B chunks of a 128-B slot / weight
// row are stored at position chunk ^ (row & 7) (XOR on the DMA source address): the 16
// consecutive slots of a fragment read hit 8 distinct positions for every tap offset.
#include <hip/hip_bf16.h>

#include "common.h"

namespace eosv {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned short u16;
typedef __attribute__((address_space(3))) void lds_t;

constexpr int WM = 4, WN = 2, NW = WM * WN;
constexpr int TP = 7;                // 16-slot pixel tiles per wave
constexpr int TC = 4;                // 16-cout tiles per wave
constexpr int BM = WM * TP * 16;     // 448 output slots per tile
constexpr int BN = WN * TC * 16;     // 128 couts per tile
constexpr int HSLOTS = 512;          // halo slots per buffer (128 B each: 64 KiB)
constexpr int HBYTES = HSLOTS * 128;
constexpr int BBYTES = BN * 128;     // one tap's weights: 16 KiB
constexpr int SMEM = 2 * HBYTES + 2 * BBYTES;  // 160 KiB
constexpr int HPW = HSLOTS / 8 / NW;  // halo DMA pieces (8 slots each) per wave: 8

__device__ __forceinline__ float bf_to_f(unsigned v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ unsigned f_to_bf(float f) { return (unsigned)__bfloat16_as_ushort(__float2bfloat16(f)); }
__device__ __forceinline__ void dma16(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(src, (lds_t*)lds, 16, 0, 0);
}
// MFMA tile i, row t -> cout within the wave's 64 (pairw_bf16's permutation)
__device__ __forceinline__ int permrow(int i, int t) { return 32 * (i >> 1) + 8 * (t >> 2) + 4 * (i & 1) + (t & 3); }
}  // namespace

// strip rows of a map of width W (slot rows of RW = W + 1 slots), 0 if the halo does not fit
static int strip_rows(int W) {
  const int RW = W + 1;
  // the 448 - R RW padding slots read up to 2 RW + 2 slots past the strip's end: keep that inside
  // the LDS allocation (dropped outputs only read there)
  if (RW > 64) return 0;
  const int R = BM / RW;
  return R >= 1 && (R + 2) * RW + 2 <= HSLOTS ? R : 0;
}

__global__ __launch_bounds__(64 * NW, 1) void conv_strip_bf16_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
  unsigned char* const hbuf = smem;                // [2][HSLOTS][128 B]
  unsigned char* const bbuf = smem + 2 * HBYTES;   // [2][BN][128 B]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid - (wid / WN) * WN;
  const int r = lane & 15, q = lane >> 4;
  const int H = a.H, W = a.W, RW = W + 1, PH = H + 1;
  const int R = BM / RW;             // launcher: strip_rows(W) > 0
  const int nN = a.Cout / BN;
  const int bt = xcd_tile(blockIdx.x, gridDim.x, a.xcd);
  const int st = bt / nN;            // strip: output slot rows r0 .. r0 + R - 1
  const int n0 = (bt - st * nN) * BN;
  const int r0 = st * R;
  const int AS = (R + 2) * RW + 2;   // halo slots of the strip (input slot rows r0 .. r0 + R + 1)
  const int nchunks = a.Cin >> 6;
  const long long K = a.K;
  const u16* __restrict__ x = (const u16*)a.x;
  const u16* __restrict__ w = (const u16*)a.w;

  // ---- halo DMA sources: piece j of this wave = slots (8 (j NW + wid) .. + 7), lane: slot + lane / 8,
  // LDS position lane % 8 holding 16-B chunk (lane % 8) ^ (slot & 7); -1 = the zero line
  int hoff[HPW];
#pragma unroll
  for (int j = 0; j < HPW; ++j) {
    const int s = 8 * (j * NW + wid) + (lane >> 3);
    const int g = r0 + s / RW;           // slot row of the tall map
    const int col = s - (s / RW) * RW;
    const int img = g / PH;
    const int ih = g - img * PH - 1, iw = col - 1;
    const int cc = (lane & 7) ^ (s & 7);
    hoff[j] = (s < AS && ih >= 0 && iw >= 0 && img < a.N) ? ((img * H + ih) * W + iw) * a.xs + cc * 8 : -1;
  }
  const int hpieces = (AS + 7) >> 3;  // pieces that hold halo slots
  auto halo_piece = [&](int j, int c, int buf) {
    const int p = j * NW + wid;  // wave-uniform
    if (p >= hpieces) return false;
    const u16* src = hoff[j] >= 0 ? x + hoff[j] + c * 64 : (const u16*)a.zero;
    dma16(src, hbuf + buf * HBYTES + p * 1024);
    return true;
  };
  // ---- weight DMA sources: pieces wid and wid + NW of a tap = ring rows 8 p .. 8 p + 7; ring row
  // RR = 64 wn' + 16 i + t holds cout n0 + 64 wn' + permrow(i, t), position lane % 8 holding chunk
  // (lane % 8) ^ (RR & 7)
  long long woff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int RR = 8 * (wid + j * NW) + (lane >> 3);
    const int co = n0 + 64 * (RR >> 6) + permrow((RR >> 4) & 3, RR & 15);
    woff[j] = (long long)co * K + (((lane & 7) ^ (RR & 7)) << 3);
  }
  auto wtap = [&](int kstep, int buf) {  // kstep = c * 9 + tap: K columns kstep * 64 .. + 63
#pragma unroll
    for (int j = 0; j < 2; ++j) dma16(w + woff[j] + kstep * 64, bbuf + buf * BBYTES + (wid + j * NW) * 1024);
  };

  f32x4 acc[TC][TP];
#pragma unroll
  for (int i = 0; i < TC; ++i)
#pragma unroll
    for (int jj = 0; jj < TP; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: chunk 0's halo and tap 0's weights
#pragma unroll
  for (int j = 0; j < HPW; ++j) halo_piece(j, 0, 0);
  wtap(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  const int ksteps = nchunks * 9;
  // fragment addressing: pixel tile jj of the wave, tap offset d: slot sl = d + 112 wm + 16 jj + r,
  // position ((4 s + q) ^ (sl & 7)) (16 jj leaves sl & 7 unchanged); weights: ring row 64 wn + 16 i + r
  const int wrow = (64 * wn + r) * 128;
  const int wpos0 = ((q) ^ (r & 7)) << 4, wpos1 = ((4 + q) ^ (r & 7)) << 4;
  int kstep = 0;
  for (int c = 0; c < nchunks; ++c) {
    const unsigned char* hb = hbuf + (c & 1) * HBYTES;
#pragma unroll 1
    for (int t = 0; t < 9; ++t, ++kstep) {
      const int kh = t / 3, kw = t - (t / 3) * 3;
      // this tap's DMA: the next tap's weights, then (taps 0..7) one piece of the next chunk's halo
      if (!(EOSV_ABL(a) & 1) && kstep + 1 < ksteps) wtap(kstep + 1, (kstep + 1) & 1);
      bool hp = false;
      if (!(EOSV_ABL(a) & 1) && c + 1 < nchunks && t < HPW) hp = halo_piece(t, c + 1, (c + 1) & 1);
      const unsigned char* wb = bbuf + (kstep & 1) * BBYTES + wrow;
      const int sl = kh * RW + kw + 112 * wm + r;
      const unsigned char* xb = hb + sl * 128;
      const int x7 = sl & 7;
      const int xpos0 = ((q) ^ x7) << 4, xpos1 = ((4 + q) ^ x7) << 4;
      if (!(EOSV_ABL(a) & 32)) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 wf[TC];
#pragma unroll
          for (int i = 0; i < TC; ++i) wf[i] = *(const bf16x8*)(wb + i * 2048 + (s ? wpos1 : wpos0));
#pragma unroll
          for (int jj = 0; jj < TP; ++jj) {
            const bf16x8 xf = *(const bf16x8*)(xb + jj * 2048 + (s ? xpos1 : xpos0));
#pragma unroll
            for (int i = 0; i < TC; ++i) acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], xf, acc[i][jj], 0, 0, 0);
          }
        }
      }
      // the next tap's weights (and after tap 7 the next halo's last piece) have landed; this
      // tap's halo piece, the only younger op, may stay in flight except before a chunk change
      if (hp && t < 8)
        asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }
  // the K loop's last wait is inline asm: tell hipcc so it does not drain again before the stores
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  if (EOSV_ABL(a) & 64) {
    asm volatile("" ::"v"(acc[0][0][0]));
    return;
  }

  // ---- epilogue from registers: lane (r, q) of tile (i, jj) holds couts 64 wn + permrow(i, 4q + e)
  // of slot 112 wm + 16 jj + r: couts 8q .. 8q + 7 (tiles 0, 1) and 32 + 8q .. (tiles 2, 3)
  const int cb = n0 + 64 * wn + 8 * q;
  float bl[16];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bl[e] = a.bias[cb + e];
    bl[8 + e] = a.bias[cb + 32 + e];
  }
  // the strip's output pixels: first real pixel p_first; stores through a buffer resource based
  // there (invalid slots get an out-of-range offset: loads return 0, stores are dropped)
  const int img_f = r0 / PH, oh_f = r0 - img_f * PH;
  const long long p_first = ((long long)img_f * H + (oh_f < H ? oh_f : H)) * W;
  const long long total = (long long)a.N * H * W;
  const long long rec = p_first < total ? (total - p_first) * a.Cout * 2 : 0;
  const int nrec = (int)(rec < 0x7fffffffLL ? rec : 0x7fffffffLL);
  u16* __restrict__ y = (u16*)a.y;
  const u16* __restrict__ res = (const u16*)a.res;
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)(y + p_first * a.Cout), (short)0, nrec, 0x00020000);
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(res ? res + p_first * a.Cout : (const u16*)a.zero), (short)0, res ? nrec : 0, 0x00020000);
  const float rlow = a.relu ? 0.f : -INFINITY;
#pragma unroll
  for (int jj = 0; jj < TP; ++jj) {
    const int o = 112 * wm + 16 * jj + r;  // output slot within the strip
    const int g = r0 + o / RW, ow = o - (o / RW) * RW;
    const int img = g / PH, oh = g - img * PH;
    const bool ok = o < R * RW && ow < W && oh < H && img < a.N;
    const long long p = ((long long)img * H + oh) * W + ow - p_first;
    const int voff = ok ? (int)((p * a.Cout + cb) * 2) : (int)0x80000000;
    const v4u ra = __builtin_amdgcn_raw_buffer_load_b128(rr, voff, 0, 0);
    const v4u rb = __builtin_amdgcn_raw_buffer_load_b128(rr, voff, 64, 0);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const v4u rv = hh ? rb : ra;
      v4u pk;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e0 = 2 * k, e1 = 2 * k + 1;  // couts 8q + e (tile 2 hh + (e >> 2), row 4q + (e & 3))
        float v0 = acc[2 * hh + (e0 >> 2)][jj][e0 & 3] + bl[8 * hh + e0];
        float v1 = acc[2 * hh + (e1 >> 2)][jj][e1 & 3] + bl[8 * hh + e1];
        v0 += bf_to_f(rv[k] & 0xffffu);
        v1 += bf_to_f(rv[k] >> 16);
        pk[k] = f_to_bf(fmaxf(v0, rlow)) | (f_to_bf(fmaxf(v1, rlow)) << 16);
      }
      __builtin_amdgcn_raw_buffer_store_b128(pk, yr, voff, hh * 64, 0);
    }
  }
}

bool conv_strip_bf16_ok(const ConvArgs& a) {
  return !a.split && !a.x2 && a.kcm && a.KH == 3 && a.KW == 3 && a.KWp == 3 && a.stride == 1 && a.pad == 1 &&
         a.Cin % 64 == 0 && a.Cin > 64 && a.Cout % BN == 0 && a.K == 9 * a.Cin && a.Ho == a.H && a.Wo == a.W &&
         strip_rows(a.W) > 0 && (a.xs == 0 || a.xs == a.Cin) &&
         // element offsets of the halo sources and the epilogue's byte offsets stay in 31 bits
         (long long)a.N * a.H * a.W * a.Cin < (1LL << 31) && (long long)a.N * a.H * a.W * a.Cout * 2 < (1LL << 31);
}

int launch_conv_strip_bf16(const ConvArgs& a0, hipStream_t s) {
  ConvArgs a = a0;
  conv_pixel_strides(a);
  if (!conv_strip_bf16_ok(a) || !a.zero || !a.bias) return set_error("conv_strip_bf16: unsupported shape"), EOSV_ERR_UNSUPPORTED;
  const int R = strip_rows(a.W);
  const long long strips = ((long long)a.N * (a.H + 1) + R - 1) / R;
  const long long nb = strips * (a.Cout / BN);
  if (nb > 0x7fffffffLL) return set_error("conv_strip_bf16: grid too large"), EOSV_ERR_UNSUPPORTED;
  if (a.plan) {
    static const int occ = kernel_occupancy((const void*)conv_strip_bf16_kernel, 64 * NW);
    return record_launch(a.plan, nb, occ);
  }
  hipLaunchKernelGGL(conv_strip_bf16_kernel, dim3((unsigned)nb), dim3(64 * NW), 0, s, a);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

}  // namespace eosv
