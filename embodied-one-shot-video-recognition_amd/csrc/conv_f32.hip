// Implicit-GEMM convolution, exact-f32 MFMA (v_mfma_f32_32x32x2_f32), NHWC.
//
// Replaces the cuDNN conv2d + BN(eval) + ReLU (+ residual add) that torchvision's
// ResNet issues inside self.convnet(x) (reference models.py:19 / 34).
//
// GEMM view: M = N*Ho*Wo output pixels, N = Cout, K = KH*KWp*Cin (tap-major,
// channel-minor, zero-padded to a multiple of BK).  A[m][k] is gathered from the
// NHWC input on the fly (im2col never materialised), B[n][k] is the BN-folded weight
// stored [Cout][K] (K contiguous), so both LDS tiles are K-contiguous rows.
//
// Block = 256 threads = 4 waves in a 2x2 grid; block tile BM x BN x BK(32);
// each wave owns (BM/2) x (BN/2) as TM x TN tiles of 32x32.  MFMA k-assignment:
// in step s of a BK chunk, lane half h supplies logical k = 16h + s, so every lane
// reads 4 consecutive k of its row with one ds_read_b128 (rows padded to 36 floats:
// conflict-free for the b128 lane groups).  Staging is register-prefetched (issue
// the next chunk's global loads before the MFMAs of the current one).
// f32 MFMA = a k-ordered fmaf chain per accumulator (exact f32, no xf32 on gfx950).
#include "common.h"

namespace eosv {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int BM, int BN>
__global__ __launch_bounds__(256) void conv_f32_kernel(ConvArgs a) {
  constexpr int BK = 32;
  constexpr int LDK = BK + 4;
  constexpr int TM = BM / 64;
  constexpr int TN = BN / 64;
  constexpr int AR = BM / 32;  // A rows staged per thread
  constexpr int BR = BN / 32;
  __shared__ __attribute__((aligned(16))) float smem[(BM + BN) * LDK];
  float* As = smem;
  float* Bs = smem + BM * LDK;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int HoWo = a.Ho * a.Wo;
  const int M = a.N * HoWo;
  const int nN = (a.Cout + BN - 1) / BN;
  const int mt = blockIdx.x / nN;
  const int nt = blockIdx.x - mt * nN;
  const int m0 = mt * BM, n0 = nt * BN;

  const int kq = tid & 7;
  const int rr = tid >> 3;
  const float* __restrict__ x = (const float*)a.x;
  const float* __restrict__ w = (const float*)a.w;

  long long abase[AR];
  int aih[AR], aiw[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = m0 + rr + 32 * i;
    if (m < M) {
      const int img = m / HoWo;
      const int rem = m - img * HoWo;
      const int oh = rem / a.Wo;
      const int ow = rem - oh * a.Wo;
      abase[i] = (long long)img * a.H * a.W * a.Cin;
      aih[i] = oh * a.stride - a.pad;
      aiw[i] = ow * a.stride - a.pad;
    } else {
      abase[i] = 0;
      aih[i] = -(1 << 28);  // forces the bounds check to fail
      aiw[i] = 0;
    }
  }

  f32x4 ra[AR], rb[BR];
  auto load = [&](int k0) {
    const int tap = k0 / a.Cin;
    const int c0 = k0 - tap * a.Cin + kq * 4;
    const int kh = tap / a.KW;
    const int kw = tap - kh * a.KW;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int ih = aih[i] + kh;
      const int iw = aiw[i] + kw;
      const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      if (ok) {
        ra[i] = *(const f32x4*)(x + abase[i] + ((long long)ih * a.W + iw) * a.Cin + c0);
      } else {
        ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int j = 0; j < BR; ++j) {
      const int n = n0 + rr + 32 * j;
      if (n < a.Cout) {
        rb[j] = *(const f32x4*)(w + (long long)n * a.K + k0 + kq * 4);
      } else {
        rb[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < AR; ++i) *(f32x4*)(As + (rr + 32 * i) * LDK + kq * 4) = ra[i];
#pragma unroll
    for (int j = 0; j < BR; ++j) *(f32x4*)(Bs + (rr + 32 * j) * LDK + kq * 4) = rb[j];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int h = lane >> 5;
  const int r = lane & 31;
  const int nk = a.K / BK;
  load(0);
  store();
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load((kt + 1) * BK);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *(const f32x4*)(As + (wm * (BM / 2) + i * 32 + r) * LDK + 16 * h + 4 * g);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bf[j] = *(const f32x4*)(Bs + (wn * (BN / 2) + j * 32 + r) * LDK + 16 * h + 4 * g);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (kt + 1 < nk) {
      store();
      __syncthreads();
    }
  }

  // epilogue: C/D map of the 32x32 MFMA: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*h
  float* __restrict__ y = (float*)a.y;
  const float* __restrict__ res = (const float*)a.res;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / 2) + j * 32 + r;
    if (n >= a.Cout) continue;
    const float b = a.bias ? a.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = m0 + wm * (BM / 2) + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (m < M) {
          const long long o = (long long)m * a.Cout + n;
          float v = acc[i][j][q] + b;
          if (res) v += res[o];
          if (a.relu) v = fmaxf(v, 0.f);
          y[o] = v;
        }
      }
    }
  }
}

template <int BM, int BN>
static int launch_v1(const ConvArgs& a, hipStream_t s) {
  const long long M = (long long)a.N * a.Ho * a.Wo;
  const long long nb = ((M + BM - 1) / BM) * ((a.Cout + BN - 1) / BN);
  if (nb > 0x7fffffffLL) return set_error("conv: grid too large"), EOSV_ERR_UNSUPPORTED;
  hipLaunchKernelGGL((conv_f32_kernel<BM, BN>), dim3((unsigned)nb), dim3(256), 0, s, a);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

static int conv_impl() {
  static int v = [] {
    const char* e = getenv("EOSV_CONV_IMPL");
    return e ? atoi(e) : 11;
  }();
  return v;
}

int launch_conv_f32(const ConvArgs& a, hipStream_t s) {
  // stem: dense padded RGB, see conv_f32_dma.hip (the only kernel that reads that layout)
  const bool stem = (a.Cin == 3);
  if ((stem && (!a.zero || a.KWp != 8 || a.KW != 7 || a.K != (a.KH * 24 + 15) / 16 * 16)) ||
      (!stem && (a.K % 32 != 0 || a.Cin % 32 != 0))) {
    set_error("conv_f32: unsupported shape (K % 32, Cin % 32 or stem layout)");
    return EOSV_ERR_UNSUPPORTED;
  }
  const int impl = a.zero ? conv_impl() : 1;
  if (a.x2 && impl == 1) return set_error("conv_f32: fused downsample needs the DMA kernel"), EOSV_ERR_UNSUPPORTED;
  if (impl == 1 && !stem) {
    if (a.Cout <= 64) return launch_v1<128, 64>(a, s);
    return launch_v1<128, 128>(a, s);
  }
  return launch_conv_f32_dma(a, s, impl);
}

}  // namespace eosv
