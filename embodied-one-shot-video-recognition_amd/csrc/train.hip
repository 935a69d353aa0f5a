// Training path: the pieces TrainNetwork.finetune_model needs on top of the
// inference kernels (reference network_train.py:52-131: ResNet in train mode, batch-statistics
// BN, fc + CrossEntropyLoss, loss.backward(), SGD with momentum on convnet and fc).
//
// The conv GEMMs of a training step that are not the inference conv kernels' shape (the stem's
// forward over an explicit im2col buffer -- 288 GB of HBM holds the largest, R50 stem at 96
// frames: 0.8 GB --, strided-conv input gradients dXcol = dY . W, 1x1 / stem weight gradients
// dW = dY^T . Xcol, the fc) are plain f32 GEMMs on the in-tree exact-f32 MFMA kernel
// (gemm_f32.hip, deterministic split-K; rocBLAS until r04).  Everything around them is here: im2col / col2im (gather,
// deterministic), batch-norm forward with batch statistics and running-stat update, its
// backward with the ReLU mask and the residual branch fused, max-pool with argmax indices and
// its gather backward, average pool, softmax cross-entropy, SGD with momentum.
// Layouts: activations NHWC f32 ([P][C] rows, P = N*H*W), conv weights [Cout][KH][KW][Cin].

#include <climits>
#include <mutex>

#include "common.h"

namespace eosv {
namespace {

constexpr int BN_CHUNKS = 1024;  // row chunks of the two-stage per-channel reductions
#ifndef EOSV_TRAIN_R04_DEF
#define EOSV_TRAIN_R04_DEF 0  // 1: the r04 passes by default (A/B builds)
#endif
// rows per lane loaded ahead in the batch-norm statistics passes (r05; release A/B variants via
// tools/build_variant.sh): forward / backward statistics and the finalize's chunks; and the
// minimum rows per lane of a statistics chunk (r04: 4; 16 since r05: a quarter of the partial-sum
// bytes written and re-read by the finalize on the narrow-P, wide-C layers)
#ifndef EOSV_BN_UP0
#define EOSV_BN_UP0 4
#endif
#ifndef EOSV_BN_UP1
#define EOSV_BN_UP1 4
#endif
#ifndef EOSV_BN_UF
#define EOSV_BN_UF 4
#endif
#ifndef EOSV_BN_MINROWS
#define EOSV_BN_MINROWS 16
#endif
// release A/B knobs (profiles/r05x_ab_bn_grids.txt): workgroups the statistics passes aim for, and
// the grid cap of the elementwise apply / dx passes (r04: 4096; 1024 since r05, +0.9-1.3 % per
// training step: each lane's per-channel operands serve more rows; 512 and below lose)
#ifndef EOSV_BN_BLOCKS
#define EOSV_BN_BLOCKS 2048
#endif
#ifndef EOSV_BN_EW_GRID
#define EOSV_BN_EW_GRID 1024
#endif
#ifndef EOSV_BN_GIN
#define EOSV_BN_GIN 1  // backward dx from the written residual gradient (r05; 0 = from dy and the mask / y)
#endif
// EOSV_TRAIN_R04=1 selects the r04 passes (one row per iteration in the batch-norm statistics,
// scalar im2col / col2im); read per call in the profiling build (A/B and the bitwise test flip it
// between calls)
bool train_r05_passes() { return env_switch("EOSV_TRAIN_R04", EOSV_TRAIN_R04_DEF) == 0; }

int grid_for(long long n, int block = 256) {
  const long long g = (n + block - 1) / block;
  return (int)std::min<long long>(std::max<long long>(g, 1), 1 << 20);
}

__global__ void im2col_kernel(const float* __restrict__ x, int N, int H, int W, int C, int KH, int KW, int stride,
                              int pad, int Ho, int Wo, float* __restrict__ col) {
  const long long K = (long long)KH * KW * C;
  const long long total = (long long)N * Ho * Wo * K;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long p = i / K;
    const int k = (int)(i - p * K);
    const int c = k % C, t = k / C, kw = t % KW, kh = t / KW;
    const int ow = (int)(p % Wo);
    const long long r = p / Wo;
    const int oh = (int)(r % Ho), n = (int)(r / Ho);
    const int ih = oh * stride - pad + kh, iw = ow * stride - pad + kw;
    col[i] = ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
                 ? x[(((long long)n * H + ih) * W + iw) * C + c]
                 : 0.f;
  }
}

// dx[n][ih][iw][c] = sum over the taps that read it of dcol[(n, oh, ow)][(kh, kw, c)]
__global__ void col2im_kernel(const float* __restrict__ col, int N, int H, int W, int C, int KH, int KW, int stride,
                              int pad, int Ho, int Wo, float* __restrict__ dx) {
  const long long K = (long long)KH * KW * C;
  const long long total = (long long)N * H * W * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long r = i / C;
    const int iw = (int)(r % W);
    const long long r2 = r / W;
    const int ih = (int)(r2 % H), n = (int)(r2 / H);
    float s = 0.f;
    for (int kh = 0; kh < KH; ++kh) {
      const int th = ih + pad - kh;
      if (th < 0 || th % stride) continue;
      const int oh = th / stride;
      if (oh >= Ho) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int tw = iw + pad - kw;
        if (tw < 0 || tw % stride) continue;
        const int ow = tw / stride;
        if (ow >= Wo) continue;
        s += col[(((long long)n * Ho + oh) * Wo + ow) * K + ((long long)kh * KW + kw) * C + c];
      }
    }
    dx[i] = s;
  }
}

// r05: four consecutive col elements per lane and one 16-byte store; the first element's (pixel,
// tap, channel) comes from divisions, the next three by carrying the counters.  Bitwise the gather
// of im2col_kernel (the R50 stem's 0.71 GB col at 96 frames ran at ~1.1 TB/s there: 64-bit
// divisions per element).  I = int when every index fits, else long long.
template <typename I>
__global__ __launch_bounds__(256) void im2col4_kernel(const float* __restrict__ x, int H, int W, int C, int KH,
                                                      int KW, int stride, int pad, int Ho, int Wo, I total,
                                                      float* __restrict__ col) {
  const I K = (I)KH * KW * C, quads = (total + 3) / 4;
  for (I q = (I)blockIdx.x * blockDim.x + threadIdx.x; q < quads; q += (I)gridDim.x * blockDim.x) {
    const I i0 = q * 4, p = i0 / K;
    const int k = (int)(i0 - p * K);
    int c = k % C, kw = (k / C) % KW, kh = k / C / KW;
    int ow = (int)(p % Wo), oh = (int)(p / Wo % Ho);
    I n = p / Wo / Ho;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ih = oh * stride - pad + kh, iw = ow * stride - pad + kw;
      v[j] = (i0 + j < total && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
                 ? x[((n * H + ih) * W + iw) * C + c]
                 : 0.f;
      if (++c == C) {
        c = 0;
        if (++kw == KW) {
          kw = 0;
          if (++kh == KH) {
            kh = 0;
            if (++ow == Wo) {
              ow = 0;
              if (++oh == Ho) oh = 0, ++n;
            }
          }
        }
      }
    }
    if (i0 + 3 < total)
      *reinterpret_cast<float4*>(col + i0) = make_float4(v[0], v[1], v[2], v[3]);
    else
      for (int j = 0; j < 4 && i0 + j < total; ++j) col[i0 + j] = v[j];
  }
}

// r05: col2im_kernel over four channels per lane (C % 4 == 0, 16-byte aligned): float4 loads of
// dcol and one division chain per four outputs; same taps in the same order, so bitwise equal
template <typename I>
__global__ __launch_bounds__(256) void col2im4_kernel(const float4* __restrict__ col, int H, int W, int C4, int KH,
                                                      int KW, int stride, int pad, int Ho, int Wo, I total4,
                                                      float4* __restrict__ dx) {
  const I K4 = (I)KH * KW * C4;
  for (I i = (I)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += (I)gridDim.x * blockDim.x) {
    const int c4 = (int)(i % C4);
    const I r = i / C4;
    const int iw = (int)(r % W), ih = (int)(r / W % H);
    const I n = r / W / H;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int kh = 0; kh < KH; ++kh) {
      const int th = ih + pad - kh;
      if (th < 0 || th % stride) continue;
      const int oh = th / stride;
      if (oh >= Ho) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int tw = iw + pad - kw;
        if (tw < 0 || tw % stride) continue;
        const int ow = tw / stride;
        if (ow >= Wo) continue;
        const float4 v = col[((n * Ho + oh) * Wo + ow) * K4 + (I)(kh * KW + kw) * C4 + c4];
        s.x += v.x, s.y += v.y, s.z += v.z, s.w += v.w;
      }
    }
    dx[i] = s;
  }
}

// V consecutive floats (V = 4: one 16-byte access)
template <int V>
__device__ inline void ldv(const float* __restrict__ p, long long i, float (&o)[V]) {
  if constexpr (V == 4) {
    const float4 v = *reinterpret_cast<const float4*>(p + i);
    o[0] = v.x, o[1] = v.y, o[2] = v.z, o[3] = v.w;
  } else {
    for (int j = 0; j < V; ++j) o[j] = p[i + j];
  }
}
template <int V>
__device__ inline void stv(float* __restrict__ p, long long i, const float (&o)[V]) {
  if constexpr (V == 4) {
    *reinterpret_cast<float4*>(p + i) = make_float4(o[0], o[1], o[2], o[3]);
  } else {
    for (int j = 0; j < V; ++j) p[i + j] = o[j];
  }
}

// V ReLU-mask bytes (1 = the forward's output > 0; V = 4: one 4-byte access) as "keep" flags
template <int V>
__device__ inline void ldm(const uint8_t* __restrict__ p, long long i, bool (&o)[V]) {
  if constexpr (V == 4) {
    const unsigned w = *reinterpret_cast<const unsigned*>(p + i);
    for (int j = 0; j < V; ++j) o[j] = (w >> (8 * j)) & 0xffu;
  } else {
    for (int j = 0; j < V; ++j) o[j] = p[i + j] != 0;
  }
}

// per (row chunk, channel): partial sums in double.  MODE 0: x, x^2.  MODE 1 (backward): g, g*xhat
// with g = dy masked by y > 0 when relu (from the forward's mask bytes mk when given, r05, else
// from y; and written to dres when given).  A block is TC lanes of V
// channels x (256 / TC) row lanes (TC = min(C / V, 256) rounded to a power of two), reduced in
// LDS, so narrow layers (C = 64) keep every lane busy.  V = 4 when C % 4 == 0 and the operands
// are 16-byte aligned.  U rows per lane are loaded before any is summed (r05: U = 4 keeps four
// 16-byte loads per operand in flight; U = 1 is the r04 loop); each lane still sums its rows in
// row order, so the partials are bitwise those of U = 1.
template <int MODE, int V, int U>
__global__ __launch_bounds__(256) void bn_partials_kernel(const float* __restrict__ a, const float* __restrict__ dy,
                                                          const float* __restrict__ y,
                                                          const uint8_t* __restrict__ mk, int relu, long long P,
                                                          int C, int tc, const float* __restrict__ mean,
                                                          const float* __restrict__ invstd, float* __restrict__ dres,
                                                          int chunks, double* __restrict__ part) {
  __shared__ double red[2 * V][256];
  const int chunk = blockIdx.y;
  const long long rows = (P + chunks - 1) / chunks;
  const long long r0 = chunk * rows, r1 = min(P, r0 + rows);
  const int lc = threadIdx.x % tc, lr = threadIdx.x / tc, nr = blockDim.x / tc;
  const int c = (blockIdx.x * tc + lc) * V;
  double s0[V], s1[V];
  for (int j = 0; j < V; ++j) s0[j] = s1[j] = 0.0;
  if (c < C) {
    if (MODE == 0) {
      for (long long r = r0 + lr; r < r1; r += (long long)U * nr) {
        float v[U][V];
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (r + (long long)u * nr < r1) ldv<V>(a, (r + (long long)u * nr) * C + c, v[u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (r + (long long)u * nr < r1)
            for (int j = 0; j < V; ++j) {
              s0[j] += (double)v[u][j];
              s1[j] += (double)v[u][j] * (double)v[u][j];
            }
      }
    } else {
      float m[V], is[V];
      ldv<V>(mean, c, m);
      ldv<V>(invstd, c, is);
      for (long long r = r0 + lr; r < r1; r += (long long)U * nr) {
        float g[U][V], x[U][V];
        bool keep[U][V];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long i = (r + (long long)u * nr) * C + c;
          if (r + (long long)u * nr < r1) {
            ldv<V>(dy, i, g[u]);
            ldv<V>(a, i, x[u]);
            if (relu && mk) {
              ldm<V>(mk, i, keep[u]);
            } else if (relu) {
              float yy[V];
              ldv<V>(y, i, yy);
              for (int j = 0; j < V; ++j) keep[u][j] = yy[j] > 0.f;
            }
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (!(r + (long long)u * nr < r1)) continue;
          if (relu)
            for (int j = 0; j < V; ++j)
              if (!keep[u][j]) g[u][j] = 0.f;
          if (dres) stv<V>(dres, (r + (long long)u * nr) * C + c, g[u]);
          for (int j = 0; j < V; ++j) {
            s0[j] += g[u][j];
            s1[j] += (double)g[u][j] * (double)((x[u][j] - m[j]) * is[j]);
          }
        }
      }
    }
  }
  for (int j = 0; j < V; ++j) {
    red[2 * j][threadIdx.x] = s0[j];
    red[2 * j + 1][threadIdx.x] = s1[j];
  }
  __syncthreads();
  if (lr == 0 && c < C) {
    for (int k = 1; k < nr; ++k)
      for (int j = 0; j < V; ++j) {
        s0[j] += red[2 * j][k * tc + lc];
        s1[j] += red[2 * j + 1][k * tc + lc];
      }
    for (int j = 0; j < V; ++j) {
      part[(long long)chunk * 2 * C + c + j] = s0[j];
      part[(long long)chunk * 2 * C + C + c + j] = s1[j];
    }
  }
}

int bn_lanes(int C) {
  int t = 1;
  while (t < C && t < 256) t <<= 1;
  return t;
}

// row chunks of the two-stage reductions: enough blocks to fill the chip, at least EOSV_BN_MINROWS
// rows per lane
int bn_chunks(long long P, int C, int V) {
  const int tc = bn_lanes(C / V), nr = 256 / tc, cblocks = (C / V + tc - 1) / tc;
  long long k = (EOSV_BN_BLOCKS + cblocks - 1) / cblocks;
  k = std::min<long long>(k, std::max<long long>(1, P / ((long long)EOSV_BN_MINROWS * nr)));
  return (int)std::max<long long>(1, std::min<long long>(k, BN_CHUNKS));
}

// the second stage: 8 channel lanes x 32 chunk lanes per block (fixed order, deterministic), then
// MODE 0 the batch statistics and running estimates, MODE 1 dgamma / dbeta and the sums for dx
template <int MODE, int U>
__global__ __launch_bounds__(256) void bn_finalize_kernel(const double* __restrict__ part, int chunks, long long P,
                                                          int C, float eps, float momentum, float* __restrict__ rmean,
                                                          float* __restrict__ rvar, float* __restrict__ out0,
                                                          float* __restrict__ out1, double* __restrict__ sums) {
  __shared__ double red[2][32][9];
  const int lc = threadIdx.x & 7, lk = threadIdx.x >> 3;
  const int c = blockIdx.x * 8 + lc;
  double s0 = 0.0, s1 = 0.0;
  if (c < C)
    for (int k = lk; k < chunks; k += 32 * U) {
      double p0[U], p1[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (k + 32 * u < chunks) {
          p0[u] = part[(long long)(k + 32 * u) * 2 * C + c];
          p1[u] = part[(long long)(k + 32 * u) * 2 * C + C + c];
        }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (k + 32 * u < chunks) s0 += p0[u], s1 += p1[u];
    }
  red[0][lk][lc] = s0;
  red[1][lk][lc] = s1;
  __syncthreads();
  if (lk != 0 || c >= C) return;
  for (int j = 1; j < 32; ++j) {
    s0 += red[0][j][lc];
    s1 += red[1][j][lc];
  }
  if (MODE == 0) {
    const double m = s0 / (double)P;
    const double var = fmax(s1 / (double)P - m * m, 0.0);  // biased: used to normalise
    out0[c] = (float)m;
    out1[c] = (float)(1.0 / sqrt(var + (double)eps));
    if (rmean) {
      const double unb = P > 1 ? var * (double)P / (double)(P - 1) : var;  // unbiased: running estimate
      rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * m);
      rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unb);
    }
  } else {
    out0[c] = (float)s1;  // dgamma
    out1[c] = (float)s0;  // dbeta
    sums[c] = s0;
    sums[C + c] = s1;
  }
}

// elementwise passes: C/4 float4 channel lanes x row lanes per block, per-channel operands held
// in registers across the rows (C % 4 == 0 and 16-byte aligned operands; else the scalar kernels)
__device__ inline float4 ld4(const float* p, int c4) { return reinterpret_cast<const float4*>(p)[c4]; }

__global__ __launch_bounds__(256) void bn_apply4_kernel(const float4* __restrict__ x, long long P, int C4,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ invstd,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta,
                                                        const float4* __restrict__ res, int relu,
                                                        float4* __restrict__ y, unsigned* __restrict__ mk) {
  const int lanes = min(C4, 256), nr = 256 / lanes;
  const int lc = threadIdx.x % lanes, lr = threadIdx.x / lanes;
  if (lr >= nr) return;
  for (int c4 = lc; c4 < C4; c4 += lanes) {
    const float4 m = ld4(mean, c4), is = ld4(invstd, c4), g = ld4(gamma, c4), b = ld4(beta, c4);
    for (long long r = (long long)blockIdx.x * nr + lr; r < P; r += (long long)gridDim.x * nr) {
      const long long i = r * C4 + c4;
      const float4 v = x[i];
      float4 o;
      o.x = (v.x - m.x) * is.x * g.x + b.x;
      o.y = (v.y - m.y) * is.y * g.y + b.y;
      o.z = (v.z - m.z) * is.z * g.z + b.z;
      o.w = (v.w - m.w) * is.w * g.w + b.w;
      if (res) {
        const float4 q = res[i];
        o.x += q.x, o.y += q.y, o.z += q.z, o.w += q.w;
      }
      if (relu) o.x = fmaxf(o.x, 0.f), o.y = fmaxf(o.y, 0.f), o.z = fmaxf(o.z, 0.f), o.w = fmaxf(o.w, 0.f);
      y[i] = o;
      if (mk)  // the backward's ReLU mask: 1 byte per element instead of re-reading y (r05)
        mk[i] = (unsigned)(o.x > 0.f) | (unsigned)(o.y > 0.f) << 8 | (unsigned)(o.z > 0.f) << 16 |
                (unsigned)(o.w > 0.f) << 24;
    }
  }
}

__device__ inline float bn_dx1(float dy, float y, int relu, float x, float m, float is, float g, float mg,
                               float mgx) {
  if (relu && !(y > 0.f)) dy = 0.f;
  const float xhat = (x - m) * is;
  return g * is * (dy - mg - xhat * mgx);
}

__global__ __launch_bounds__(256) void bn_dx4_kernel(const float4* __restrict__ dy, const float4* __restrict__ y,
                                                     const unsigned* __restrict__ mk, int relu,
                                                     const float4* __restrict__ x, long long P, int C4,
                                                     const float* __restrict__ gamma, const float* __restrict__ mean,
                                                     const float* __restrict__ invstd,
                                                     const double* __restrict__ sums, float4* __restrict__ dx) {
  const int lanes = min(C4, 256), nr = 256 / lanes;
  const int lc = threadIdx.x % lanes, lr = threadIdx.x / lanes;
  if (lr >= nr) return;
  const int C = 4 * C4;
  for (int c4 = lc; c4 < C4; c4 += lanes) {
    const float4 m = ld4(mean, c4), is = ld4(invstd, c4), g = ld4(gamma, c4);
    float mg[4], mgx[4];
    for (int j = 0; j < 4; ++j) {
      mg[j] = (float)(sums[4 * c4 + j] / (double)P);
      mgx[j] = (float)(sums[C + 4 * c4 + j] / (double)P);
    }
    for (long long r = (long long)blockIdx.x * nr + lr; r < P; r += (long long)gridDim.x * nr) {
      const long long i = r * C4 + c4;
      const float4 d = dy[i], v = x[i];
      float4 yy = make_float4(1.f, 1.f, 1.f, 1.f);  // relu: only y > 0 matters (bn_dx1)
      if (relu && mk) {
        const unsigned w = mk[i];
        yy = make_float4(w & 0xffu ? 1.f : 0.f, w & 0xff00u ? 1.f : 0.f, w & 0xff0000u ? 1.f : 0.f,
                         w & 0xff000000u ? 1.f : 0.f);
      } else if (relu) {
        yy = y[i];
      }
      float4 o;
      o.x = bn_dx1(d.x, yy.x, relu, v.x, m.x, is.x, g.x, mg[0], mgx[0]);
      o.y = bn_dx1(d.y, yy.y, relu, v.y, m.y, is.y, g.y, mg[1], mgx[1]);
      o.z = bn_dx1(d.z, yy.z, relu, v.z, m.z, is.z, g.z, mg[2], mgx[2]);
      o.w = bn_dx1(d.w, yy.w, relu, v.w, m.w, is.w, g.w, mg[3], mgx[3]);
      dx[i] = o;
    }
  }
}

__global__ void bn_apply_kernel(const float* __restrict__ x, long long P, int C, const float* __restrict__ mean,
                                const float* __restrict__ invstd, const float* __restrict__ gamma,
                                const float* __restrict__ beta, const float* __restrict__ res, int relu,
                                float* __restrict__ y, uint8_t* __restrict__ mk) {
  const long long total = P * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    float v = (x[i] - mean[c]) * invstd[c] * gamma[c] + beta[c];
    if (res) v += res[i];
    if (relu) v = fmaxf(v, 0.f);
    y[i] = v;
    if (mk) mk[i] = v > 0.f;
  }
}

// dx = gamma * invstd * (g - sum(g) / P - xhat * sum(g * xhat) / P)
__global__ void bn_dx_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                             const uint8_t* __restrict__ mk, int relu,
                             const float* __restrict__ x, long long P, int C, const float* __restrict__ gamma,
                             const float* __restrict__ mean, const float* __restrict__ invstd,
                             const double* __restrict__ sums, float* __restrict__ dx) {
  const long long total = P * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const float yv = !relu ? 1.f : mk ? (mk[i] ? 1.f : 0.f) : y[i];
    dx[i] = bn_dx1(dy[i], yv, relu, x[i], mean[c], invstd[c], gamma[c], (float)(sums[c] / (double)P),
                   (float)(sums[C + c] / (double)P));
  }
}

bool al16(const void* p) { return p == nullptr || ((uintptr_t)p & 15) == 0; }
bool al4(const void* p) { return ((uintptr_t)p & 3) == 0; }  // nullptr passes

int rows_grid(long long P, int C) {
  const int nr = 256 / std::min(C / 4, 256);
  return (int)std::min<long long>((P + nr - 1) / nr, EOSV_BN_EW_GRID);
}

// 3x3 / 2, pad 1 (torchvision's maxpool); argmax = first maximum in (kh, kw) order, as torch CPU
__global__ void maxpool_fwd_kernel(const float* __restrict__ x, int N, int H, int W, int C, int Ho, int Wo,
                                   float* __restrict__ y, int* __restrict__ idx) {
  const long long total = (long long)N * Ho * Wo * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long r = i / C;
    const int ow = (int)(r % Wo);
    const long long r2 = r / Wo;
    const int oh = (int)(r2 % Ho), n = (int)(r2 / Ho);
    float m = -INFINITY;
    int arg = -1;
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * oh - 1 + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = 2 * ow - 1 + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        const float v = x[(((long long)n * H + ih) * W + iw) * C + c];
        if (v > m || arg < 0) m = v, arg = ih * W + iw;
      }
    }
    y[i] = m;
    idx[i] = arg;
  }
}

__global__ void maxpool_bwd_kernel(const float* __restrict__ dy, const int* __restrict__ idx, int N, int H, int W,
                                   int C, int Ho, int Wo, float* __restrict__ dx) {
  const long long total = (long long)N * H * W * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long r = i / C;
    const int iw = (int)(r % W);
    const long long r2 = r / W;
    const int ih = (int)(r2 % H), n = (int)(r2 / H);
    const int me = ih * W + iw;
    float s = 0.f;
    for (int kh = 0; kh < 3; ++kh) {
      const int th = ih + 1 - kh;
      if (th < 0 || (th & 1)) continue;
      const int oh = th >> 1;
      if (oh >= Ho) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int tw = iw + 1 - kw;
        if (tw < 0 || (tw & 1)) continue;
        const int ow = tw >> 1;
        if (ow >= Wo) continue;
        const long long o = (((long long)n * Ho + oh) * Wo + ow) * C + c;
        if (idx[o] == me) s += dy[o];
      }
    }
    dx[i] = s;
  }
}

// the same two passes over 4 channels per thread (C % 4 == 0, 16-byte aligned): one pixel's
// window / pooled neighbours as float4 and int4 accesses, 32-bit pixel indexing
__global__ void maxpool_fwd4_kernel(const float4* __restrict__ x, int NP, int H, int W, int C4, int Ho, int Wo,
                                    float4* __restrict__ y, int4* __restrict__ idx) {
  const long long total = (long long)NP * C4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c4 = (int)(i % C4);
    const int r = (int)(i / C4);
    const int ow = r % Wo, r2 = r / Wo;
    const int oh = r2 % Ho, n = r2 / Ho;
    float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int arg[4] = {-1, -1, -1, -1};
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * oh - 1 + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = 2 * ow - 1 + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        const float4 v = x[((long long)(n * H + ih) * W + iw) * C4 + c4];
        const float vv[4] = {v.x, v.y, v.z, v.w};
        for (int j = 0; j < 4; ++j)
          if (vv[j] > m[j] || arg[j] < 0) m[j] = vv[j], arg[j] = ih * W + iw;
      }
    }
    y[i] = make_float4(m[0], m[1], m[2], m[3]);
    idx[i] = make_int4(arg[0], arg[1], arg[2], arg[3]);
  }
}

__global__ void maxpool_bwd4_kernel(const float4* __restrict__ dy, const int4* __restrict__ idx, int NP, int H, int W,
                                    int C4, int Ho, int Wo, float4* __restrict__ dx) {
  const long long total = (long long)NP * C4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c4 = (int)(i % C4);
    const int r = (int)(i / C4);
    const int iw = r % W, r2 = r / W;
    const int ih = r2 % H, n = r2 / H;
    const int me = ih * W + iw;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int kh = 0; kh < 3; ++kh) {
      const int th = ih + 1 - kh;
      if (th < 0 || (th & 1)) continue;
      const int oh = th >> 1;
      if (oh >= Ho) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int tw = iw + 1 - kw;
        if (tw < 0 || (tw & 1)) continue;
        const int ow = tw >> 1;
        if (ow >= Wo) continue;
        const long long o = ((long long)(n * Ho + oh) * Wo + ow) * C4 + c4;
        const int4 a = idx[o];
        const float4 d = dy[o];
        if (a.x == me) s[0] += d.x;
        if (a.y == me) s[1] += d.y;
        if (a.z == me) s[2] += d.z;
        if (a.w == me) s[3] += d.w;
      }
    }
    dx[i] = make_float4(s[0], s[1], s[2], s[3]);
  }
}

// y[n][c] = mean over HW of x[n][hw][c] (sequential); backward dx = dy / HW
__global__ void avgpool_fwd_kernel(const float* __restrict__ x, int N, int HW, int C, float* __restrict__ y) {
  const long long total = (long long)N * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long n = i / C;
    float s = 0.f;
    for (int t = 0; t < HW; ++t) s += x[(n * HW + t) * C + c];
    y[i] = s / (float)HW;
  }
}

// dx[(n, t)][c] = dy[n][c] * scale (average pool over HW, or the clip mean over T frames)
__global__ void broadcast_rows_kernel(const float* __restrict__ dy, int N, int T, int C, float scale,
                                      float* __restrict__ dx) {
  const long long total = (long long)N * T * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long n = i / ((long long)T * C);
    dx[i] = dy[n * C + c] * scale;
  }
}

// CrossEntropyLoss (mean over the batch): loss += (logsumexp - logit[label]) / B,
// dlogits = (softmax - onehot) / B.  One block per row.
__global__ void softmax_xent_kernel(const float* __restrict__ logits, const int* __restrict__ labels, int B, int C,
                                    float* __restrict__ row_loss, float* __restrict__ dlogits) {
  const int b = blockIdx.x;
  const float* l = logits + (long long)b * C;
  __shared__ float red[256];
  float m = -INFINITY;
  for (int c = threadIdx.x; c < C; c += blockDim.x) m = fmaxf(m, l[c]);
  red[threadIdx.x] = m;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  m = red[0];
  __syncthreads();
  float se = 0.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) se += expf(l[c] - m);
  red[threadIdx.x] = se;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  se = red[0];
  const int lab = labels[b];
  if ((unsigned)lab >= (unsigned)C) {
    // nn.CrossEntropyLoss raises 'Target out of bounds'; the host checks first
    // (NativeTrainer.step), and a label that gets here anyway yields a NaN loss and a zero
    // gradient for its row instead of an out-of-bounds read
    for (int c = threadIdx.x; c < C; c += blockDim.x) dlogits[(long long)b * C + c] = 0.f;
    if (threadIdx.x == 0) row_loss[b] = __int_as_float(0x7fc00000);
    return;
  }
  for (int c = threadIdx.x; c < C; c += blockDim.x)
    dlogits[(long long)b * C + c] = (expf(l[c] - m) / se - (c == lab ? 1.f : 0.f)) / (float)B;
  if (threadIdx.x == 0) row_loss[b] = (logf(se) + m - l[lab]) / (float)B;
}

__global__ void sum_rows_kernel(const float* __restrict__ x, int rows, int C, float* __restrict__ y, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int r = 0; r < rows; ++r) s += x[(long long)r * C + c];
  y[c] = accumulate ? y[c] + s : s;
}

// C[i] = sum over the slices of W (fixed slice order: deterministic)

__global__ void add_bias_kernel(float* __restrict__ y, int rows, int C, const float* __restrict__ b) {
  const long long total = (long long)rows * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x)
    y[i] += b[i % C];
}

// torch.optim.SGD (momentum, dampening 0, no weight decay): buf = g on the first step, else
// momentum * buf + g; p -= lr * buf
__global__ void sgd_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ buf, long long n,
                           float lr, float momentum, int first) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float b = first ? g[i] : momentum * buf[i] + g[i];
    buf[i] = b;
    p[i] -= lr * b;
  }
}

__global__ void axpy_kernel(float* __restrict__ y, const float* __restrict__ x, long long n, float alpha) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    y[i] += alpha * x[i];
}

// W[cout][kh][kw][cin] -> Wf[cin][KH-1-kh][KW-1-kw][cout]: the stride-1 input gradient is the
// convolution of dY with these weights (same padding for odd square kernels)
__global__ void flip_weights_kernel(const float* __restrict__ w, int Cout, int KH, int KW, int Cin,
                                    float* __restrict__ wf) {
  const long long total = (long long)Cout * KH * KW * Cin;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % Cin);
    const long long r = i / Cin;
    const int kw = (int)(r % KW);
    const long long r2 = r / KW;
    const int kh = (int)(r2 % KH), co = (int)(r2 / KH);
    wf[(((long long)ci * KH + (KH - 1 - kh)) * KW + (KW - 1 - kw)) * Cout + co] = w[i];
  }
}

// 64 zero bytes per device: the DMA target of the conv kernels' out-of-bounds taps
const void* zero_page(int dev) {
  static std::mutex mu;
  static void* pages[64] = {};
  std::lock_guard<std::mutex> lk(mu);
  if (dev < 0 || dev >= 64) return nullptr;
  if (!pages[dev]) {
    void* p = nullptr;
    if (hipMalloc(&p, 256) != hipSuccess || hipMemset(p, 0, 256) != hipSuccess) return nullptr;
    pages[dev] = p;
  }
  return pages[dev];
}

__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, int N, int C, int HW, float* __restrict__ y) {
  const long long total = (long long)N * C * HW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long long r = i / C;
    const int t = (int)(r % HW);
    const long long n = r / HW;
    y[i] = x[(n * C + c) * HW + t];
  }
}

bool pos(long long v) { return v > 0; }
}  // namespace
}  // namespace eosv

using namespace eosv;

extern "C" {

int eosv_im2col(const float* d_x, int N, int H, int W, int C, int KH, int KW, int stride, int pad, float* d_col,
                eosv_stream_t stream) {
  if (!d_x || !d_col || N <= 0 || H <= 0 || W <= 0 || C <= 0 || KH <= 0 || KW <= 0 || stride <= 0 || pad < 0)
    return set_error("eosv_im2col: bad argument"), EOSV_ERR_ARG;
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  if (Ho <= 0 || Wo <= 0) return set_error("eosv_im2col: empty output"), EOSV_ERR_ARG;
  const hipStream_t s = (hipStream_t)stream;
  const long long total = (long long)N * Ho * Wo * KH * KW * C;
  if (!train_r05_passes() || !al16(d_col))
    hipLaunchKernelGGL(im2col_kernel, dim3(grid_for(total)), dim3(256), 0, s, d_x, N, H, W, C, KH, KW, stride, pad,
                       Ho, Wo, d_col);
  else if (total < INT_MAX - 4 && (long long)N * H * W * C < INT_MAX)
    hipLaunchKernelGGL(im2col4_kernel<int>, dim3(grid_for((total + 3) / 4)), dim3(256), 0, s, d_x, H, W, C, KH, KW,
                       stride, pad, Ho, Wo, (int)total, d_col);
  else
    hipLaunchKernelGGL(im2col4_kernel<long long>, dim3(grid_for((total + 3) / 4)), dim3(256), 0, s, d_x, H, W, C, KH,
                       KW, stride, pad, Ho, Wo, total, d_col);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int eosv_col2im(const float* d_col, int N, int H, int W, int C, int KH, int KW, int stride, int pad, float* d_x,
                eosv_stream_t stream) {
  if (!d_x || !d_col || N <= 0 || H <= 0 || W <= 0 || C <= 0 || KH <= 0 || KW <= 0 || stride <= 0 || pad < 0)
    return set_error("eosv_col2im: bad argument"), EOSV_ERR_ARG;
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  if (Ho <= 0 || Wo <= 0) return set_error("eosv_col2im: empty output"), EOSV_ERR_ARG;
  const hipStream_t s = (hipStream_t)stream;
  const long long total4 = (long long)N * H * W * C / 4, colsz = (long long)N * Ho * Wo * KH * KW * C;
  if (!train_r05_passes() || C % 4 || !al16(d_col) || !al16(d_x))
    hipLaunchKernelGGL(col2im_kernel, dim3(grid_for((long long)N * H * W * C)), dim3(256), 0, s, d_col, N, H, W, C,
                       KH, KW, stride, pad, Ho, Wo, d_x);
  else if (colsz < INT_MAX && 4 * total4 < INT_MAX)
    hipLaunchKernelGGL(col2im4_kernel<int>, dim3(grid_for(total4)), dim3(256), 0, s, (const float4*)d_col, H, W,
                       C / 4, KH, KW, stride, pad, Ho, Wo, (int)total4, (float4*)d_x);
  else
    hipLaunchKernelGGL(col2im4_kernel<long long>, dim3(grid_for(total4)), dim3(256), 0, s, (const float4*)d_col, H,
                       W, C / 4, KH, KW, stride, pad, Ho, Wo, total4, (float4*)d_x);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int64_t eosv_bn_workspace_bytes(int C) { return C > 0 ? (int64_t)(2 * BN_CHUNKS + 2) * C * 8 : 0; }

int eosv_bn_train_forward(const float* d_x, int64_t P, int C, const float* d_gamma, const float* d_beta, float eps,
                          float momentum, float* d_running_mean, float* d_running_var, const float* d_residual,
                          int relu, float* d_y, uint8_t* d_mask, float* d_save_mean, float* d_save_invstd,
                          void* d_work, eosv_stream_t stream) {
  if (!d_x || !d_y || !d_gamma || !d_beta || !d_save_mean || !d_save_invstd || !d_work || !pos(P) || C <= 0 ||
      (!d_running_mean) != (!d_running_var) || !(eps > 0.f))
    return set_error("eosv_bn_train_forward: bad argument"), EOSV_ERR_ARG;
  const hipStream_t s = (hipStream_t)stream;
  double* part = (double*)d_work;
  const int V = C % 4 == 0 && al16(d_x) ? 4 : 1;
  const int tc = bn_lanes(C / V), chunks = bn_chunks(P, C, V);
  const dim3 pg((C / V + tc - 1) / tc, chunks);
  const bool un = train_r05_passes();
  auto partials = V == 4 ? (un ? bn_partials_kernel<0, 4, EOSV_BN_UP0> : bn_partials_kernel<0, 4, 1>)
                         : (un ? bn_partials_kernel<0, 1, EOSV_BN_UP0> : bn_partials_kernel<0, 1, 1>);
  hipLaunchKernelGGL(partials, pg, dim3(256), 0, s, d_x, nullptr, nullptr, nullptr, 0, (long long)P, C, tc, nullptr,
                     nullptr, nullptr, chunks, part);
  auto finalize = un ? bn_finalize_kernel<0, EOSV_BN_UF> : bn_finalize_kernel<0, 1>;
  hipLaunchKernelGGL(finalize, dim3((C + 7) / 8), dim3(256), 0, s, part, chunks, (long long)P, C, eps, momentum,
                     d_running_mean, d_running_var, d_save_mean, d_save_invstd, nullptr);
  uint8_t* mk = relu ? d_mask : nullptr;  // the ReLU mask for the backward (optional)
  if (C % 4 == 0 && al16(d_x) && al16(d_y) && al16(d_residual) && al16(d_save_mean) && al16(d_save_invstd) &&
      al16(d_gamma) && al16(d_beta) && al4(mk))
    hipLaunchKernelGGL(bn_apply4_kernel, dim3(rows_grid(P, C)), dim3(256), 0, s, (const float4*)d_x, (long long)P,
                       C / 4, d_save_mean, d_save_invstd, d_gamma, d_beta, (const float4*)d_residual, relu,
                       (float4*)d_y, (unsigned*)mk);
  else
    hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_for((long long)P * C)), dim3(256), 0, s, d_x, (long long)P, C,
                       d_save_mean, d_save_invstd, d_gamma, d_beta, d_residual, relu, d_y, mk);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int eosv_bn_train_backward(const float* d_dy, const float* d_y, const uint8_t* d_mask, int relu, const float* d_x,
                           int64_t P, int C,
                           const float* d_gamma, const float* d_save_mean, const float* d_save_invstd, float* d_dx,
                           float* d_dgamma, float* d_dbeta, float* d_dres, void* d_work, eosv_stream_t stream) {
  if (!d_dy || !d_x || !d_gamma || !d_save_mean || !d_save_invstd || !d_dx || !d_dgamma || !d_dbeta || !d_work ||
      !pos(P) || C <= 0 || (relu && !d_y && !d_mask))
    return set_error("eosv_bn_train_backward: bad argument"), EOSV_ERR_ARG;
  // the ReLU mask from the forward's bytes when given (r05: 1 byte per element, not y's 4)
  const uint8_t* mk = relu ? d_mask : nullptr;
  const float* yv = mk ? nullptr : d_y;
  const hipStream_t s = (hipStream_t)stream;
  double* part = (double*)d_work;
  double* sums = part + (long long)2 * BN_CHUNKS * C;
  const int V = C % 4 == 0 && al16(d_x) && al16(d_dy) && al16(yv) && al4(mk) && al16(d_dres) && al16(d_save_mean) &&
                        al16(d_save_invstd)
                    ? 4
                    : 1;
  const int tc = bn_lanes(C / V), chunks = bn_chunks(P, C, V);
  const dim3 pg((C / V + tc - 1) / tc, chunks);
  const bool un = train_r05_passes();
  auto partials = V == 4 ? (un ? bn_partials_kernel<1, 4, EOSV_BN_UP1> : bn_partials_kernel<1, 4, 1>)
                         : (un ? bn_partials_kernel<1, 1, EOSV_BN_UP1> : bn_partials_kernel<1, 1, 1>);
  hipLaunchKernelGGL(partials, pg, dim3(256), 0, s, d_x, d_dy, yv, mk, relu, (long long)P, C, tc, d_save_mean,
                     d_save_invstd, d_dres, chunks, part);
  auto finalize = un ? bn_finalize_kernel<1, EOSV_BN_UF> : bn_finalize_kernel<1, 1>;
  hipLaunchKernelGGL(finalize, dim3((C + 7) / 8), dim3(256), 0, s, part, chunks, (long long)P, C, 0.f, 0.f, nullptr,
                     nullptr, d_dgamma, d_dbeta, sums);
  // r05: with the residual gradient written, it is dy already masked: dx reads it alone (4 bytes per
  // element instead of dy and the mask / y; bn_dx1 then masks nothing, the same values)
  const bool g_in = EOSV_BN_GIN && un && d_dres;
  const float* gdy = g_in ? d_dres : d_dy;
  const float* gy = g_in ? nullptr : yv;
  const uint8_t* gmk = g_in ? nullptr : mk;
  const int grelu = g_in ? 0 : relu;
  if (C % 4 == 0 && al16(gdy) && al16(gy) && al4(gmk) && al16(d_x) && al16(d_dx) && al16(d_gamma) &&
      al16(d_save_mean) && al16(d_save_invstd))
    hipLaunchKernelGGL(bn_dx4_kernel, dim3(rows_grid(P, C)), dim3(256), 0, s, (const float4*)gdy, (const float4*)gy,
                       (const unsigned*)gmk, grelu, (const float4*)d_x, (long long)P, C / 4, d_gamma, d_save_mean,
                       d_save_invstd, sums, (float4*)d_dx);
  else
    hipLaunchKernelGGL(bn_dx_kernel, dim3(grid_for((long long)P * C)), dim3(256), 0, s, gdy, gy, gmk, grelu, d_x,
                       (long long)P, C, d_gamma, d_save_mean, d_save_invstd, sums, d_dx);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int eosv_maxpool_forward(const float* d_x, int N, int H, int W, int C, float* d_y, int32_t* d_idx,
                         eosv_stream_t stream) {
  if (!d_x || !d_y || !d_idx || N <= 0 || H <= 0 || W <= 0 || C <= 0)
    return set_error("eosv_maxpool_forward: bad argument"), EOSV_ERR_ARG;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  if (C % 4 == 0 && al16(d_x) && al16(d_y) && al16(d_idx) && (long long)N * H * W < (1LL << 31))
    hipLaunchKernelGGL(maxpool_fwd4_kernel, dim3(grid_for((long long)N * Ho * Wo * C / 4)), dim3(256), 0,
                       (hipStream_t)stream, (const float4*)d_x, N * Ho * Wo, H, W, C / 4, Ho, Wo, (float4*)d_y,
                       (int4*)d_idx);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for((long long)N * Ho * Wo * C)), dim3(256), 0,
                       (hipStream_t)stream, d_x, N, H, W, C, Ho, Wo, d_y, d_idx);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int eosv_maxpool_backward(const float* d_dy, const int32_t* d_idx, int N, int H, int W, int C, float* d_dx,
                          eosv_stream_t stream) {
  if (!d_dy || !d_idx || !d_dx || N <= 0 || H <= 0 || W <= 0 || C <= 0)
    return set_error("eosv_maxpool_backward: bad argument"), EOSV_ERR_ARG;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  if (C % 4 == 0 && al16(d_dy) && al16(d_idx) && al16(d_dx) && (long long)N * H * W < (1LL << 31))
    hipLaunchKernelGGL(maxpool_bwd4_kernel, dim3(grid_for((long long)N * H * W * C / 4)), dim3(256), 0,
                       (hipStream_t)stream, (const float4*)d_dy, (const int4*)d_idx, N * H * W, H, W, C / 4, Ho, Wo,
                       (float4*)d_dx);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for((long long)N * H * W * C)), dim3(256), 0, (hipStream_t)stream,
                       d_dy, d_idx, N, H, W, C, Ho, Wo, d_dx);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int eosv_avgpool_forward(const float* d_x, int N, int HW, int C, float* d_y, eosv_stream_t stream) {
  if (!d_x || !d_y || N <= 0 || HW <= 0 || C <= 0) return set_error("eosv_avgpool_forward: bad argument"), EOSV_ERR_ARG;
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(grid_for((long long)N * C)), dim3(256), 0, (hipStream_t)stream, d_x, N,
                     HW, C, d_y);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int eosv_broadcast_rows(const float* d_dy, int N, int T, int C, float scale, float* d_dx, eosv_stream_t stream) {
  if (!d_dy || !d_dx || N <= 0 || T <= 0 || C <= 0) return set_error("eosv_broadcast_rows: bad argument"), EOSV_ERR_ARG;
  hipLaunchKernelGGL(broadcast_rows_kernel, dim3(grid_for((long long)N * T * C)), dim3(256), 0, (hipStream_t)stream,
                     d_dy, N, T, C, scale, d_dx);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int eosv_softmax_xent(const float* d_logits, const int32_t* d_labels, int B, int C, float* d_row_loss,
                      float* d_dlogits, eosv_stream_t stream) {
  if (!d_logits || !d_labels || !d_row_loss || !d_dlogits || B <= 0 || C <= 0)
    return set_error("eosv_softmax_xent: bad argument"), EOSV_ERR_ARG;
  hipLaunchKernelGGL(softmax_xent_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, d_logits, d_labels, B, C,
                     d_row_loss, d_dlogits);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int eosv_sum_rows(const float* d_x, int rows, int C, float* d_y, int accumulate, eosv_stream_t stream) {
  if (!d_x || !d_y || rows <= 0 || C <= 0) return set_error("eosv_sum_rows: bad argument"), EOSV_ERR_ARG;
  hipLaunchKernelGGL(sum_rows_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, d_x, rows, C, d_y,
                     accumulate);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int eosv_add_bias(float* d_y, int rows, int C, const float* d_bias, eosv_stream_t stream) {
  if (!d_y || !d_bias || rows <= 0 || C <= 0) return set_error("eosv_add_bias: bad argument"), EOSV_ERR_ARG;
  hipLaunchKernelGGL(add_bias_kernel, dim3(grid_for((long long)rows * C)), dim3(256), 0, (hipStream_t)stream, d_y,
                     rows, C, d_bias);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int eosv_sgd_momentum(float* d_p, const float* d_g, float* d_buf, int64_t n, float lr, float momentum, int first,
                      eosv_stream_t stream) {
  if (!d_p || !d_g || !d_buf || n <= 0) return set_error("eosv_sgd_momentum: bad argument"), EOSV_ERR_ARG;
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, d_p, d_g, d_buf, (long long)n,
                     lr, momentum, first);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int eosv_axpy(float* d_y, const float* d_x, int64_t n, float alpha, eosv_stream_t stream) {
  if (!d_y || !d_x || n <= 0) return set_error("eosv_axpy: bad argument"), EOSV_ERR_ARG;
  hipLaunchKernelGGL(axpy_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, d_y, d_x, (long long)n, alpha);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

static ConvArgs conv2d_args(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad) {
  ConvArgs a{};
  a.N = N, a.H = H, a.W = W, a.Cin = Cin;
  a.Ho = (H + 2 * pad - KH) / stride + 1, a.Wo = (W + 2 * pad - KW) / stride + 1, a.Cout = Cout;
  a.KH = KH, a.KW = KW, a.KWp = KW, a.stride = stride, a.pad = pad;
  a.K = KH * KW * Cin;
  a.xcd = 1;
  return a;
}

int64_t eosv_conv2d_f32_workspace(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad) {
  if (N <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0 || KH <= 0 || KW <= 0 || stride <= 0 || pad < 0) return 0;
  const ConvArgs a = conv2d_args(N, H, W, Cin, Cout, KH, KW, stride, pad);
  if (a.Ho <= 0 || a.Wo <= 0) return 0;
  const int ks = conv_f32_ksplit_slices(a);  // the slices the launch will use (1: no workspace)
  return ks > 1 ? (int64_t)ks * N * a.Ho * a.Wo * Cout * (int64_t)sizeof(float) : 0;
}

int eosv_conv2d_f32(const float* d_x, int N, int H, int W, int Cin, const float* d_w, int Cout, int KH, int KW,
                    int stride, int pad, const float* d_bias, const float* d_res, int relu, float* d_y, float* d_work,
                    int64_t work_bytes, eosv_stream_t stream) {
  if (!d_x || !d_w || !d_y || N <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0 || KH <= 0 || KW <= 0 ||
      stride <= 0 || pad < 0)
    return set_error("eosv_conv2d_f32: bad argument"), EOSV_ERR_ARG;
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  if (Ho <= 0 || Wo <= 0) return set_error("eosv_conv2d_f32: empty output"), EOSV_ERR_ARG;
  if (Cin == 3 || Cin % 32 || (KH * KW * Cin) % 32)
    return set_error("eosv_conv2d_f32: needs Cin % 32 == 0 (the stem goes through im2col + eosv_sgemm)"),
           EOSV_ERR_UNSUPPORTED;
  int dev = 0;
  EOSV_HIP_CHECK(hipGetDevice(&dev));
  ConvArgs a = conv2d_args(N, H, W, Cin, Cout, KH, KW, stride, pad);
  a.x = d_x;
  a.w = d_w;
  a.bias = d_bias;
  a.res = d_res;
  a.y = d_y;
  a.relu = relu;
  a.zero = zero_page(dev);
  // split-K over the workspace when one is given (small grids: the training batch)
  if (d_work && work_bytes > 0 && !((uintptr_t)d_work & 15)) a.kws = d_work, a.kws_bytes = work_bytes;
  if (!a.zero) return set_error("eosv_conv2d_f32: zero page allocation failed"), EOSV_ERR_OOM;
  return launch_conv_f32(a, (hipStream_t)stream);
}

int eosv_flip_weights(const float* d_w, int Cout, int KH, int KW, int Cin, float* d_wf, eosv_stream_t stream) {
  if (!d_w || !d_wf || Cout <= 0 || KH <= 0 || KW <= 0 || Cin <= 0)
    return set_error("eosv_flip_weights: bad argument"), EOSV_ERR_ARG;
  hipLaunchKernelGGL(flip_weights_kernel, dim3(grid_for((long long)Cout * KH * KW * Cin)), dim3(256), 0,
                     (hipStream_t)stream, d_w, Cout, KH, KW, Cin, d_wf);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

int eosv_nchw_to_nhwc(const float* d_x, int N, int C, int H, int W, float* d_y, eosv_stream_t stream) {
  if (!d_x || !d_y || N <= 0 || C <= 0 || H <= 0 || W <= 0)
    return set_error("eosv_nchw_to_nhwc: bad argument"), EOSV_ERR_ARG;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for((long long)N * C * H * W)), dim3(256), 0, (hipStream_t)stream,
                     d_x, N, C, H * W, d_y);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

}  // extern "C"
