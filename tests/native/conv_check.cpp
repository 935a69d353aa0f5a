// Layer-level check of the implicit-GEMM conv against a naive CPU conv (double accum).
// Build: hipcc --offload-arch=gfx950 -O2 -I include -I <pkg>/csrc conv_check.cpp -L<pkg> -leosv
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "common.h"

using namespace eosv;

static float frand(unsigned& s) { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xffff) / 32768.f - 1.f; }

// ds_cin > 0: a fused 1x1 stride-2 downsample (ConvArgs::x2) reads x2 [N][2H][2W][ds_cin] into K
// columns [K1, K1 + ds_cin).  tol: bound on |err| / (1 + sum of |terms|) -- f32 rounding of a
// K-term dot product grows with the magnitudes summed, not with the (cancelling) result.
// kcm: device weights in the chunk-major K order (cin / 32, kh, kw, cin % 32) (ConvArgs::kcm, f32)
static int check(int N, int H, int W, int Cin, int Cout, int K, int stride, int pad, bool stem, bool res, bool relu,
                 int ds_cin = 0, double tol = 1e-5, bool kcm = false) {
  // stem: dense padded RGB input [N][H+2p][Wp][3] (zero borders), K = [kh][24] padded to 16
  const int KWp = stem ? 8 : K, Cinp = Cin;
  const int Ho = (H + 2 * pad - K) / stride + 1, Wo = (W + 2 * pad - K) / stride + 1;
  const int K1 = stem ? (K * 24 + 15) / 16 * 16 : K * KWp * Cinp;
  const int Kd = K1 + ds_cin;
  const int H2 = 2 * Ho, W2 = 2 * Wo;
  const int Hx = stem ? H + 2 * pad : H, Wx = stem ? stem_row_pixels(W, pad) : W, off = stem ? pad : 0;
  unsigned s = 12345;
  std::vector<float> x(stem ? stem_input_elems(N, H, W, pad) : (size_t)N * H * W * Cinp, 0.f),
      w((size_t)Cout * Kd, 0.f), b(Cout), r((size_t)N * Ho * Wo * Cout);
  for (int n = 0; n < N; ++n)
    for (int i = 0; i < H; ++i)
      for (int j = 0; j < W; ++j)
        for (int c = 0; c < Cin; ++c) x[(((size_t)n * Hx + i + off) * Wx + j + off) * Cinp + c] = frand(s);
  for (int o = 0; o < Cout; ++o)
    for (int kh = 0; kh < K; ++kh)
      for (int kw = 0; kw < K; ++kw)
        for (int c = 0; c < Cin; ++c) w[(size_t)o * Kd + (kh * KWp + kw) * Cinp + c] = frand(s);
  for (auto& v : b) v = frand(s);
  for (auto& v : r) v = frand(s);
  std::vector<float> x2((size_t)N * H2 * W2 * ds_cin);
  for (auto& v : x2) v = frand(s);
  for (int o = 0; o < Cout; ++o)
    for (int c = 0; c < ds_cin; ++c) w[(size_t)o * Kd + K1 + c] = frand(s);
  float* dx2 = nullptr;
  if (ds_cin) {
    hipMalloc(&dx2, x2.size() * 4);
    hipMemcpy(dx2, x2.data(), x2.size() * 4, hipMemcpyHostToDevice);
  }
  float *dx, *dw, *db, *dr, *dy;
  hipMalloc(&dx, x.size() * 4); hipMalloc(&dw, w.size() * 4); hipMalloc(&db, b.size() * 4);
  hipMalloc(&dr, r.size() * 4); hipMalloc(&dy, r.size() * 4);
  hipMemcpy(dx, x.data(), x.size() * 4, hipMemcpyHostToDevice);
  std::vector<float> wd = w;
  if (kcm)
    for (int o = 0; o < Cout; ++o)
      for (int t = 0; t < K * K; ++t)
        for (int c = 0; c < Cin; ++c)
          wd[(size_t)o * Kd + ((c / 32) * K * K + t) * 32 + c % 32] = w[(size_t)o * Kd + t * Cinp + c];
  hipMemcpy(dw, wd.data(), wd.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), b.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dr, r.data(), r.size() * 4, hipMemcpyHostToDevice);
  ConvArgs a{};
  a.kcm = kcm ? 32 : 0;
  a.x = dx; a.w = dw; a.bias = db; a.res = res ? dr : nullptr; a.y = dy;
  a.N = N; a.H = H; a.W = W; a.Cin = Cinp; a.Ho = Ho; a.Wo = Wo; a.Cout = Cout;
  a.KH = K; a.KW = K; a.KWp = KWp; a.stride = stride; a.pad = pad; a.K = Kd; a.relu = relu;
  void* dz; hipMalloc(&dz, 256); hipMemset(dz, 0, 256); a.zero = dz;
  if (ds_cin) {
    a.x2 = dx2; a.H2 = H2; a.W2 = W2; a.Cin2 = ds_cin; a.stride2 = 2; a.K1 = K1;
  }
  int rc = launch_conv_f32(a, 0);
  hipDeviceSynchronize();
  std::vector<float> y(r.size());
  hipMemcpy(y.data(), dy, y.size() * 4, hipMemcpyDeviceToHost);
  double maxerr = 0, maxref = 0; long bad = 0;
  for (int n = 0; n < N; ++n)
    for (int oh = 0; oh < Ho; ++oh)
      for (int ow = 0; ow < Wo; ++ow)
        for (int o = 0; o < Cout; ++o) {
          double acc = b[o], sabs = fabs(b[o]);
          for (int kh = 0; kh < K; ++kh)
            for (int kw = 0; kw < K; ++kw) {
              int ih = oh * stride - pad + kh, iw = ow * stride - pad + kw;
              if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
              for (int c = 0; c < Cin; ++c) {
                const double t = (double)x[(((size_t)n * Hx + ih + off) * Wx + iw + off) * Cinp + c] *
                                 w[(size_t)o * Kd + (kh * KWp + kw) * Cinp + c];
                acc += t;
                sabs += fabs(t);
              }
            }
          for (int c = 0; c < ds_cin; ++c) {
            const double t = (double)x2[(((size_t)n * H2 + 2 * oh) * W2 + 2 * ow) * ds_cin + c] * w[(size_t)o * Kd + K1 + c];
            acc += t;
            sabs += fabs(t);
          }
          size_t oi = (((size_t)n * Ho + oh) * Wo + ow) * Cout + o;
          if (res) acc += r[oi], sabs += fabs(r[oi]);
          if (relu && acc < 0) acc = 0;
          double e = fabs(acc - y[oi]);
          if (!(e <= tol * (1 + sabs))) { if (bad < 5) printf("  bad n%d oh%d ow%d o%d ref %f got %f\n", n, oh, ow, o, acc, y[oi]); ++bad; }
          maxerr = fmax(maxerr, e); maxref = fmax(maxref, fabs(acc));
        }
  printf("%s f32 N%d H%d W%d Cin%d Cout%d K%d s%d p%d res%d relu%d ds%d kcm%d rc=%d maxerr %.3e (maxref %.3e) bad %ld\n",
         bad || rc ? "FAIL" : "ok  ", N, H, W, Cin, Cout, K, stride, pad, res, relu, ds_cin, kcm, rc, maxerr, maxref, bad);
  hipFree(dx); hipFree(dw); hipFree(db); hipFree(dr); hipFree(dy);
  if (dx2) hipFree(dx2);
  hipFree(dz);
  return bad || rc ? 1 : 0;
}

static unsigned short f2bf(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}
static float bf2f(unsigned short v) {
  unsigned u = (unsigned)v << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// bf16 conv through launch_conv_bf16 (stage-1 3x3 shapes take the row-strip kernel, Cout >= 128
// the phased 8-wave kernel); reference in double on the bf16-rounded operands, checked on images
// `checked` only
// the launcher check_bf16 goes through: launch_conv_bf16 (its default dispatch), or one kernel directly
static int (*g_bf16_launch)(const ConvArgs&, hipStream_t) = launch_conv_bf16;
static int check_bf16(int N, int H, int W, int Cin, int Cout, int k, int stride, int pad, bool res, bool relu,
                      bool kcm = false) {
  const int K = k * k * Cin;
  const int Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  unsigned s = 777;
  std::vector<unsigned short> x((size_t)N * H * W * Cin), w((size_t)Cout * K), r((size_t)N * Ho * Wo * Cout);
  std::vector<float> b(Cout);
  for (auto& v : x) v = f2bf(frand(s));
  for (auto& v : w) v = f2bf(frand(s) * 0.1f);
  for (auto& v : r) v = f2bf(frand(s));
  for (auto& v : b) v = frand(s);
  unsigned short *dx, *dw, *dr, *dy;
  float* db;
  void* dz;
  hipMalloc(&dx, x.size() * 2); hipMalloc(&dw, w.size() * 2); hipMalloc(&dr, r.size() * 2);
  hipMalloc(&dy, r.size() * 2); hipMalloc(&db, Cout * 4); hipMalloc(&dz, 256); hipMemset(dz, 0, 256);
  hipMemcpy(dx, x.data(), x.size() * 2, hipMemcpyHostToDevice);
  {
    // kcm: device weights in K order (cin / 64, kh, kw, cin % 64) (ConvArgs::kcm)
    std::vector<unsigned short> wd(w.size());
    for (int o = 0; o < Cout; ++o)
      for (int t = 0; t < k * k; ++t)
        for (int c = 0; c < Cin; ++c)
          wd[(size_t)o * K + (kcm ? ((c / 64) * k * k + t) * 64 + c % 64 : t * Cin + c)] = w[(size_t)o * K + t * Cin + c];
    hipMemcpy(dw, wd.data(), wd.size() * 2, hipMemcpyHostToDevice);
  }
  hipMemcpy(dr, r.data(), r.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), Cout * 4, hipMemcpyHostToDevice);
  hipMemset(dy, 0xff, r.size() * 2);
  ConvArgs a{};
  a.x = dx; a.w = dw; a.bias = db; a.res = res ? dr : nullptr; a.y = dy;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Ho = Ho; a.Wo = Wo; a.Cout = Cout;
  a.KH = k; a.KW = k; a.KWp = k; a.stride = stride; a.pad = pad; a.K = K; a.relu = relu; a.zero = dz;
  a.xcd = 1;
  a.kcm = kcm;
  a.xs = Cin;  // dense pixels (launch_conv_bf16 sets it itself)
  const int rc = g_bf16_launch(a, 0);
  hipDeviceSynchronize();
  std::vector<unsigned short> y(r.size());
  hipMemcpy(y.data(), dy, y.size() * 2, hipMemcpyDeviceToHost);
  const int checked[4] = {0, N > 1 ? 1 : 0, N > 2 ? N - 2 : 0, N - 1};
  double maxerr = 0;
  long bad = 0;
  for (int ci = 0; ci < 4; ++ci) {
    const int n = checked[ci];
    if (ci > 0 && n == checked[ci - 1]) continue;
    for (int oh = 0; oh < Ho; ++oh)
      for (int ow = 0; ow < Wo; ++ow)
        for (int o = 0; o < Cout; ++o) {
          double acc = b[o];
          for (int kh = 0; kh < k; ++kh)
            for (int kw = 0; kw < k; ++kw) {
              const int ih = oh * stride - pad + kh, iw = ow * stride - pad + kw;
              if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
              for (int c = 0; c < Cin; ++c)
                acc += (double)bf2f(x[(((size_t)n * H + ih) * W + iw) * Cin + c]) *
                       bf2f(w[(size_t)o * K + (kh * k + kw) * Cin + c]);
            }
          const size_t oi = (((size_t)n * Ho + oh) * Wo + ow) * Cout + o;
          if (res) acc += bf2f(r[oi]);
          if (relu && acc < 0) acc = 0;
          const double e = fabs(acc - bf2f(y[oi]));
          if (!(e <= 1e-2 * (1 + fabs(acc)))) {
            if (bad < 5) printf("  bad n%d oh%d ow%d o%d ref %f got %f\n", n, oh, ow, o, acc, bf2f(y[oi]));
            ++bad;
          }
          maxerr = fmax(maxerr, e);
        }
  }
  printf("%s bf16 N%d H%d W%d Cin%d Cout%d k%d s%d p%d res%d relu%d kcm%d rc=%d maxerr %.3e bad %ld\n",
         bad ? "FAIL" : "ok  ", N, H, W, Cin, Cout, k, stride, pad, res, relu, kcm, rc, maxerr, bad);
  hipFree(dx); hipFree(dw); hipFree(dr); hipFree(dy); hipFree(db); hipFree(dz);
  return bad || rc ? 1 : 0;
}

// fused bf16 stem (7x7/2 p3, 3 -> 64) + bias + ReLU + maxpool 3x3/2 p1 vs a double reference
// on the same bf16 operands (bf16 rounding of the stem output before the pool, as the kernel)
static int check_stem_pool(int N, int H, int W, bool direct = false) {
  const int pad = 3, Wp = stem_row_pixels(W, pad), Hp = H + 2 * pad;
  const int Hs = (H + 6 - 7) / 2 + 1, Ws = (W + 6 - 7) / 2 + 1;
  const int Hq = (Hs - 1) / 2 + 1, Wq = (Ws - 1) / 2 + 1;
  unsigned s = 4242;
  std::vector<unsigned short> x(stem_input_elems(N, H, W, pad) + 256, 0), w(64 * 192, 0);
  std::vector<float> b(64);
  for (int n = 0; n < N; ++n)
    for (int i = 0; i < H; ++i)
      for (int j = 0; j < W; ++j)
        for (int c = 0; c < 3; ++c) x[128 / 2 + (((size_t)n * Hp + i + pad) * Wp + j + pad) * 3 + c] = f2bf(frand(s));
  for (int o = 0; o < 64; ++o)
    for (int kh = 0; kh < 7; ++kh)
      for (int kw = 0; kw < 7; ++kw)
        for (int c = 0; c < 3; ++c) w[o * 192 + kh * 24 + kw * 3 + c] = f2bf(frand(s) * 0.2f);
  for (auto& v : b) v = frand(s) * 0.5f;
  unsigned short *dx, *dw, *dy;
  float* db;
  const size_t ny = (size_t)N * Hq * Wq * 64;
  hipMalloc(&dx, x.size() * 2); hipMalloc(&dw, w.size() * 2); hipMalloc(&dy, ny * 2); hipMalloc(&db, 64 * 4);
  hipMemcpy(dx, x.data(), x.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dw, w.data(), w.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), 64 * 4, hipMemcpyHostToDevice);
  hipMemset(dy, 0xff, ny * 2);
  // direct: the kernel reads f32 NCHW frames (the same values, exactly representable in bf16)
  std::vector<float> fr((size_t)N * 3 * H * W);
  for (int n = 0; n < N; ++n)
    for (int i = 0; i < H; ++i)
      for (int j = 0; j < W; ++j)
        for (int c = 0; c < 3; ++c)
          fr[(((size_t)n * 3 + c) * H + i) * W + j] = bf2f(x[128 / 2 + (((size_t)n * Hp + i + pad) * Wp + j + pad) * 3 + c]);
  float* dfr;
  hipMalloc(&dfr, fr.size() * 4);
  hipMemcpy(dfr, fr.data(), fr.size() * 4, hipMemcpyHostToDevice);
  const int rc = direct ? launch_stem_pool_bf16(nullptr, N, H, W, dw, db, dy, 0, dfr)
                        : launch_stem_pool_bf16(dx + 64, N, H, W, dw, db, dy, 0);  // 128 B front slack
  hipDeviceSynchronize();
  std::vector<unsigned short> y(ny);
  hipMemcpy(y.data(), dy, ny * 2, hipMemcpyDeviceToHost);
  std::vector<float> st((size_t)Hs * Ws * 64);
  long bad = 0;
  double maxerr = 0;
  for (int n = 0; n < N; ++n) {
    for (int sy = 0; sy < Hs; ++sy)
      for (int sx = 0; sx < Ws; ++sx)
        for (int o = 0; o < 64; ++o) {
          double acc = b[o];
          for (int kh = 0; kh < 7; ++kh)
            for (int kw = 0; kw < 7; ++kw)
              for (int c = 0; c < 3; ++c)
                acc += (double)bf2f(x[64 + (((size_t)n * Hp + 2 * sy + kh) * Wp + 2 * sx + kw) * 3 + c]) *
                       bf2f(w[o * 192 + kh * 24 + kw * 3 + c]);
          st[((size_t)sy * Ws + sx) * 64 + o] = bf2f(f2bf((float)(acc > 0 ? acc : 0)));
        }
    for (int py = 0; py < Hq; ++py)
      for (int px = 0; px < Wq; ++px)
        for (int o = 0; o < 64; ++o) {
          float m = -INFINITY;
          for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
              const int sy = 2 * py + dy, sx = 2 * px + dx;
              if (sy >= 0 && sy < Hs && sx >= 0 && sx < Ws) m = fmaxf(m, st[((size_t)sy * Ws + sx) * 64 + o]);
            }
          const float got = bf2f(y[(((size_t)n * Hq + py) * Wq + px) * 64 + o]);
          const double e = fabs(got - m);
          if (e > 1e-2 * (1 + fabs(m))) {
            if (bad < 5) printf("  bad n%d py%d px%d o%d ref %f got %f\n", n, py, px, o, m, got);
            ++bad;
          }
          maxerr = fmax(maxerr, e);
        }
  }
  printf("%s stem_pool bf16%s N%d H%d W%d rc=%d maxerr %.3e bad %ld\n", bad ? "FAIL" : "ok  ", direct ? " direct" : "",
         N, H, W, rc, maxerr, bad);
  hipFree(dx); hipFree(dw); hipFree(dy); hipFree(db); hipFree(dfr);
  return bad || rc ? 1 : 0;
}


// EOSV_F32X3 split-bf16 fused stem vs a double reference on the f32 operands: the kernel splits
// frames and weights into bf16 hi + lo and drops lo.lo, so hi + lo of its output must be within
// ~1e-4 relative of the exact value (the north star's f32 bound)
static int check_stem_pool_x3(int N, int H, int W) {
  const int Hs = (H + 6 - 7) / 2 + 1, Ws = (W + 6 - 7) / 2 + 1;
  const int Hq = (Hs - 1) / 2 + 1, Wq = (Ws - 1) / 2 + 1;
  unsigned s = 777;
  std::vector<float> fr((size_t)N * 3 * H * W), wf(64 * 192, 0.f), b(64);
  for (auto& v : fr) v = frand(s) * 2.f;
  for (int o = 0; o < 64; ++o)
    for (int kh = 0; kh < 7; ++kh)
      for (int kw = 0; kw < 7; ++kw)
        for (int c = 0; c < 3; ++c) wf[o * 192 + kh * 24 + kw * 3 + c] = frand(s) * 0.2f;
  for (auto& v : b) v = frand(s) * 0.5f;
  std::vector<unsigned short> w2(2 * 64 * 192);
  for (int i = 0; i < 64 * 192; ++i) {
    w2[i] = f2bf(wf[i]);
    w2[64 * 192 + i] = f2bf(wf[i] - bf2f(w2[i]));
  }
  float *dfr, *db;
  unsigned short *dw, *dy;
  const size_t ny = (size_t)N * Hq * Wq * 128;  // split layout: (hi 64 | lo 64) per pixel
  hipMalloc(&dfr, fr.size() * 4); hipMalloc(&dw, w2.size() * 2); hipMalloc(&dy, ny * 2); hipMalloc(&db, 64 * 4);
  hipMemcpy(dfr, fr.data(), fr.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dw, w2.data(), w2.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), 64 * 4, hipMemcpyHostToDevice);
  hipMemset(dy, 0xff, ny * 2);
  const int rc = launch_stem_pool_x3(dfr, N, H, W, dw, db, dy, 0);
  hipDeviceSynchronize();
  std::vector<unsigned short> y(ny);
  hipMemcpy(y.data(), dy, ny * 2, hipMemcpyDeviceToHost);
  std::vector<double> st((size_t)Hs * Ws * 64);
  long bad = 0;
  double maxerr = 0, maxref = 0;
  for (int n = 0; n < N; ++n) {
    for (int sy = 0; sy < Hs; ++sy)
      for (int sx = 0; sx < Ws; ++sx)
        for (int o = 0; o < 64; ++o) {
          double acc = b[o];
          for (int kh = 0; kh < 7; ++kh)
            for (int kw = 0; kw < 7; ++kw) {
              const int iy = 2 * sy + kh - 3, ix = 2 * sx + kw - 3;
              if (iy < 0 || iy >= H || ix < 0 || ix >= W) continue;
              for (int c = 0; c < 3; ++c)
                acc += (double)fr[(((size_t)n * 3 + c) * H + iy) * W + ix] * wf[o * 192 + kh * 24 + kw * 3 + c];
            }
          st[((size_t)sy * Ws + sx) * 64 + o] = acc > 0 ? acc : 0;
        }
    for (int py = 0; py < Hq; ++py)
      for (int px = 0; px < Wq; ++px)
        for (int o = 0; o < 64; ++o) {
          double m = -INFINITY;
          for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
              const int sy = 2 * py + dy, sx = 2 * px + dx;
              if (sy >= 0 && sy < Hs && sx >= 0 && sx < Ws) m = fmax(m, st[((size_t)sy * Ws + sx) * 64 + o]);
            }
          const size_t base = (((size_t)n * Hq + py) * Wq + px) * 128 + o;
          const double got = (double)bf2f(y[base]) + bf2f(y[base + 64]);
          // lo is the rounding residual of hi: at most half an ulp of hi (2^-9 relative)
          const bool dup = fabs(bf2f(y[base + 64])) <= fabs(bf2f(y[base])) * (1.0 / 256);
          const double e = fabs(got - m);
          maxref = fmax(maxref, fabs(m));
          if (e > 1e-4 * (1 + fabs(m)) || !dup) {
            if (bad < 5) printf("  bad n%d py%d px%d o%d ref %f got %f dup %d\n", n, py, px, o, m, got, (int)dup);
            ++bad;
          }
          maxerr = fmax(maxerr, e);
        }
  }
  printf("%s stem_pool x3 N%d H%d W%d rc=%d maxerr %.3e (maxref %.3e) bad %ld\n", bad ? "FAIL" : "ok  ", N, H, W, rc,
         maxerr, maxref, bad);
  hipFree(dfr); hipFree(dw); hipFree(dy); hipFree(db);
  return bad || rc ? 1 : 0;
}

// fused f32 stem + shift + ReLU + maxpool vs a double reference on the same f32 operands
// (weights in the uploaded [64][176] = [kh 7][24] + 8 layout)
static int check_stem_pool_f32(int N, int H, int W, int every = 1) {
  const int pad = 3, Wp = stem_row_pixels(W, pad), Hp = H + 2 * pad;
  const int Hs = (H + 6 - 7) / 2 + 1, Ws = (W + 6 - 7) / 2 + 1;
  const int Hq = (Hs - 1) / 2 + 1, Wq = (Ws - 1) / 2 + 1;
  unsigned s = 5151;
  std::vector<float> x(stem_input_elems(N, H, W, pad) + 64, 0.f), w(64 * 176, 0.f), b(64);
  for (int n = 0; n < N; ++n)
    for (int i = 0; i < H; ++i)
      for (int j = 0; j < W; ++j)
        for (int c = 0; c < 3; ++c) x[(((size_t)n * Hp + i + pad) * Wp + j + pad) * 3 + c] = frand(s);
  for (int o = 0; o < 64; ++o)
    for (int kh = 0; kh < 7; ++kh)
      for (int kw = 0; kw < 7; ++kw)
        for (int c = 0; c < 3; ++c) w[o * 176 + kh * 24 + kw * 3 + c] = frand(s) * 0.2f;
  for (auto& v : b) v = frand(s) * 0.5f;
  float *dx, *dw, *dy, *db;
  const size_t ny = (size_t)N * Hq * Wq * 64;
  hipMalloc(&dx, x.size() * 4); hipMalloc(&dw, w.size() * 4); hipMalloc(&dy, ny * 4); hipMalloc(&db, 64 * 4);
  hipMemcpy(dx, x.data(), x.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), 64 * 4, hipMemcpyHostToDevice);
  hipMemset(dy, 0xff, ny * 4);
  const int rc = launch_stem_pool_f32(dx, N, H, W, dw, db, dy, 0);
  hipDeviceSynchronize();
  std::vector<float> y(ny);
  hipMemcpy(y.data(), dy, ny * 4, hipMemcpyDeviceToHost);
  std::vector<double> st((size_t)Hs * Ws * 64);
  long bad = 0;
  double maxerr = 0;
  for (int n = 0; n < N; ++n) {
    if (n % every && n != N - 1) continue;  // large N: a sample of the images (every band count)
    for (int sy = 0; sy < Hs; ++sy)
      for (int sx = 0; sx < Ws; ++sx)
        for (int o = 0; o < 64; ++o) {
          double acc = b[o];
          for (int kh = 0; kh < 7; ++kh)
            for (int kw = 0; kw < 7; ++kw)
              for (int c = 0; c < 3; ++c)
                acc += (double)x[(((size_t)n * Hp + 2 * sy + kh) * Wp + 2 * sx + kw) * 3 + c] * w[o * 176 + kh * 24 + kw * 3 + c];
          st[((size_t)sy * Ws + sx) * 64 + o] = acc > 0 ? acc : 0;
        }
    for (int py = 0; py < Hq; ++py)
      for (int px = 0; px < Wq; ++px)
        for (int o = 0; o < 64; ++o) {
          double m = -INFINITY;
          for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
              const int sy = 2 * py + dy, sx = 2 * px + dx;
              if (sy >= 0 && sy < Hs && sx >= 0 && sx < Ws) m = fmax(m, st[((size_t)sy * Ws + sx) * 64 + o]);
            }
          const float got = y[(((size_t)n * Hq + py) * Wq + px) * 64 + o];
          const double e = fabs(got - m);
          if (!(e <= 1e-5 * (1 + fabs(m)))) {
            if (bad < 5) printf("  bad n%d py%d px%d o%d ref %f got %f\n", n, py, px, o, m, got);
            ++bad;
          }
          maxerr = fmax(maxerr, e);
        }
  }
  // DIRECT (the f32 NCHW frames, no pack): the same values, so bit-identical to the pack run
  long dbad = 0;
  int rc2 = 0;
  const bool direct = stem_pool_f32_direct_ok(H, W);
  if (direct) {
    std::vector<float> fr((size_t)N * 3 * H * W);
    for (int n = 0; n < N; ++n)
      for (int c = 0; c < 3; ++c)
        for (int i = 0; i < H; ++i)
          for (int j = 0; j < W; ++j)
            fr[(((size_t)n * 3 + c) * H + i) * W + j] = x[(((size_t)n * Hp + i + pad) * Wp + j + pad) * 3 + c];
    float *dfr, *dy2;
    hipMalloc(&dfr, fr.size() * 4); hipMalloc(&dy2, ny * 4);
    hipMemcpy(dfr, fr.data(), fr.size() * 4, hipMemcpyHostToDevice);
    hipMemset(dy2, 0xff, ny * 4);
    rc2 = launch_stem_pool_f32(nullptr, N, H, W, dw, db, dy2, 0, false, nullptr, dfr);
    hipDeviceSynchronize();
    std::vector<float> y2(ny);
    hipMemcpy(y2.data(), dy2, ny * 4, hipMemcpyDeviceToHost);
    for (size_t i = 0; i < ny; ++i) dbad += memcmp(&y[i], &y2[i], 4) != 0;
    hipFree(dfr); hipFree(dy2);
  }
  printf("%s stem_pool f32 N%d H%d W%d rc=%d maxerr %.3e bad %ld%s\n", bad || dbad || rc2 ? "FAIL" : "ok  ", N, H, W,
         rc, maxerr, bad, direct ? (dbad || rc2 ? " direct differs" : " direct identical") : "");
  hipFree(dx); hipFree(dw); hipFree(dy); hipFree(db);
  return bad || rc || dbad || rc2 ? 1 : 0;
}

// bottleneck 1x1 pair (pair1x1_bf16.hip) vs the unfused pair through launch_conv_bf16: conv3
// (1x1 64 -> 256, + residual or + a folded stride-1 downsample) then the next block's conv1
// (1x1 256 -> c1), both with folded-BN shifts and ReLU.  Same K order, same epilogue order:
// both maps must be bit-identical.
static int check_pair(int N, int H, int W, int c1, bool ds) {
  const long long M = (long long)N * H * W;
  const int K3 = ds ? 128 : 64;
  unsigned s = 777;
  auto fill = [&](std::vector<unsigned short>& v, float scale) {
    for (auto& e : v) e = f2bf(frand(s) * scale);
  };
  std::vector<unsigned short> x(M * 64), x2(ds ? M * 64 : 1), res(M * 256), w3(256 * K3), w1((size_t)c1 * 256);
  fill(x, 1.f); fill(x2, 1.f); fill(res, 1.f); fill(w3, 0.125f); fill(w1, 0.0625f);
  std::vector<float> b3(256), b1(c1);
  for (auto& v : b3) v = frand(s) * 0.5f;
  for (auto& v : b1) v = frand(s) * 0.5f;
  auto up = [](const void* p, size_t n) { void* d; hipMalloc(&d, n); hipMemcpy(d, p, n, hipMemcpyHostToDevice); return d; };
  void *dx = up(x.data(), x.size() * 2), *dx2 = up(x2.data(), x2.size() * 2), *dr = up(res.data(), res.size() * 2);
  void *dw3 = up(w3.data(), w3.size() * 2), *dw1 = up(w1.data(), w1.size() * 2);
  float *db3 = (float*)up(b3.data(), b3.size() * 4), *db1 = (float*)up(b1.data(), b1.size() * 4);
  void *y0, *z0, *y1, *z1, *dz;
  hipMalloc(&y0, M * 512); hipMalloc(&y1, M * 512); hipMalloc(&z0, M * c1 * 2); hipMalloc(&z1, M * c1 * 2);
  hipMalloc(&dz, 256); hipMemset(dz, 0, 256);
  // unfused: conv3 (+ residual | + downsample K columns), then conv1
  ConvArgs a{};
  a.x = dx; a.w = dw3; a.bias = db3; a.res = ds ? nullptr : dr; a.y = y0;
  a.N = N; a.H = H; a.W = W; a.Cin = 64; a.Ho = H; a.Wo = W; a.Cout = 256;
  a.KH = a.KW = a.KWp = 1; a.stride = 1; a.pad = 0; a.K = K3; a.relu = 1; a.zero = dz; a.xcd = 1;
  if (ds) { a.x2 = dx2; a.H2 = H; a.W2 = W; a.Cin2 = 64; a.stride2 = 1; a.K1 = 64; }
  int rc = launch_conv_bf16(a, 0);
  ConvArgs b{};
  b.x = y0; b.w = dw1; b.bias = db1; b.res = nullptr; b.y = z0;
  b.N = N; b.H = H; b.W = W; b.Cin = 256; b.Ho = H; b.Wo = W; b.Cout = c1;
  b.KH = b.KW = b.KWp = 1; b.stride = 1; b.pad = 0; b.K = 256; b.relu = 1; b.zero = dz; b.xcd = 1;
  rc |= launch_conv_bf16(b, 0);
  Pair1x1Args p{};
  p.x = dx; p.x2 = ds ? dx2 : nullptr; p.res = ds ? nullptr : dr; p.w3 = dw3; p.b3 = db3; p.w1 = dw1; p.b1 = db1;
  p.y = y1; p.z = z1; p.M = M; p.c1 = c1; p.cds = ds ? 64 : 0;
  rc |= launch_pair1x1_bf16(p, 0);
  hipDeviceSynchronize();
  std::vector<unsigned short> hy0(M * 256), hy1(M * 256), hz0(M * c1), hz1(M * c1);
  hipMemcpy(hy0.data(), y0, M * 512, hipMemcpyDeviceToHost); hipMemcpy(hy1.data(), y1, M * 512, hipMemcpyDeviceToHost);
  hipMemcpy(hz0.data(), z0, M * c1 * 2, hipMemcpyDeviceToHost); hipMemcpy(hz1.data(), z1, M * c1 * 2, hipMemcpyDeviceToHost);
  long bady = 0, badz = 0;
  double maxd = 0;
  for (size_t i = 0; i < hy0.size(); ++i)
    if (hy0[i] != hy1[i]) ++bady, maxd = std::max(maxd, (double)fabs(bf2f(hy0[i]) - bf2f(hy1[i])));
  for (size_t i = 0; i < hz0.size(); ++i)
    if (hz0[i] != hz1[i]) ++badz, maxd = std::max(maxd, (double)fabs(bf2f(hz0[i]) - bf2f(hz1[i])));
  // the unfused maps themselves against double on the bf16 operands (a few pixels)
  double maxerr = 0;
  for (long long m = 0; m < M; m += M / 7 + 1)
    for (int o = 0; o < 256; o += 5) {
      double acc = b3[o];
      for (int k = 0; k < 64; ++k) acc += (double)bf2f(x[m * 64 + k]) * bf2f(w3[o * K3 + k]);
      if (ds) for (int k = 0; k < 64; ++k) acc += (double)bf2f(x2[m * 64 + k]) * bf2f(w3[o * K3 + 64 + k]);
      else acc += bf2f(res[m * 256 + o]);
      acc = std::max(acc, 0.0);
      maxerr = std::max(maxerr, fabs(acc - bf2f(hy0[m * 256 + o])) / (1.0 + fabs(acc)));
    }
  const bool fail = rc || bady || badz || maxerr > 1e-2;
  printf("%s pair1x1 bf16 N%d H%d W%d c1 %d ds%d rc=%d differing y %ld z %ld (max %.3e) unfused maxerr %.3e\n",
         fail ? "FAIL" : "ok  ", N, H, W, c1, ds ? 1 : 0, rc, bady, badz, maxd, maxerr);
  for (void* q : {dx, dx2, dr, dw3, dw1, (void*)db3, (void*)db1, y0, y1, z0, z1, dz}) hipFree(q);
  return fail ? 1 : 0;
}

// wide bottleneck pair (pairw_bf16.hip, stages 2-3) vs the unfused conv3 (1x1 cmid -> cexp +
// residual) -> conv1 (1x1 cexp -> c1) through launch_conv_bf16: both maps bit-identical.  M
// need not be a multiple of the 128-pixel round: the tail round runs on the buffers' padding
// (filled with NaN here: no valid output may depend on it), and it is repeated REPS times (its
// results changed from run to run while it masked the padding with out-of-range buffer ops).
// every CU's LDS filled with 0xff (NaN in bf16): a kernel reading LDS words it did not write
__global__ __launch_bounds__(256) void lds_poison_k() {
  __shared__ unsigned lds[160 * 1024 / 4];
  volatile unsigned* q = lds;
  for (int i = threadIdx.x; i < 160 * 1024 / 4; i += 256) q[i] = 0xffffffffu;
}

// inplace: y = res (as the engine runs the pair: Y lands in the residual's buffer); stress: before
// every repetition 1 GiB is written (cold caches) and the LDS poisoned
static int check_pairw(int N, int H, int W, int cmid, int cexp, int c1, int cds = 0, bool inplace = false,
                       bool stress = false, int reps = 0) {
  // cds > 0: block 0 of a stage, conv3 + the folded stride-2 downsample reading x2 [N][2H][2W][cds]
  // (ragged: 2H - 1 when odd sizes are asked for through H2/W2 below), no residual
  const long long M = (long long)N * H * W;
  const int H2 = 2 * H, W2 = 2 * W;
  const int K3 = cmid + cds;
  unsigned s = 4242 + cmid + c1;
  auto fill = [&](std::vector<unsigned short>& v, float scale) {
    for (auto& e : v) e = f2bf(frand(s) * scale);
  };
  const long long tile = pairw_tile(cmid, c1, cds);  // 128 pixels per round
  const long long Mp = (M + tile - 1) / tile * tile;  // padded to whole rounds
  std::vector<unsigned short> x(Mp * cmid, 0x7fc0), res(Mp * cexp, 0x7fc0), w3((size_t)cexp * K3), w1((size_t)c1 * cexp);
  std::vector<unsigned short> x2(cds ? (size_t)N * H2 * W2 * cds : 1);
  {
    std::vector<unsigned short> xv(M * cmid), rv(M * cexp);
    fill(xv, 1.f); fill(rv, 1.f);
    std::copy(xv.begin(), xv.end(), x.begin());
    std::copy(rv.begin(), rv.end(), res.begin());
  }
  fill(w3, 0.125f); fill(w1, 0.0625f); fill(x2, 1.f);
  std::vector<float> b3(cexp), b1(c1);
  for (auto& v : b3) v = frand(s) * 0.5f;
  for (auto& v : b1) v = frand(s) * 0.5f;
  auto up = [](const void* p, size_t n) { void* d; hipMalloc(&d, n); hipMemcpy(d, p, n, hipMemcpyHostToDevice); return d; };
  void *dx = up(x.data(), x.size() * 2), *dr = up(res.data(), res.size() * 2), *dx2 = up(x2.data(), x2.size() * 2);
  void *dw3 = up(w3.data(), w3.size() * 2), *dw1 = up(w1.data(), w1.size() * 2);
  float *db3 = (float*)up(b3.data(), b3.size() * 4), *db1 = (float*)up(b1.data(), b1.size() * 4);
  void *y0, *z0, *y1, *z1, *dz;
  hipMalloc(&y0, M * cexp * 2); hipMalloc(&y1, Mp * cexp * 2); hipMalloc(&z0, M * c1 * 2); hipMalloc(&z1, Mp * c1 * 2);
  hipMalloc(&dz, 256); hipMemset(dz, 0, 256);
  ConvArgs a{};
  a.x = dx; a.w = dw3; a.bias = db3; a.res = cds ? nullptr : dr; a.y = y0;
  a.N = N; a.H = H; a.W = W; a.Cin = cmid; a.Ho = H; a.Wo = W; a.Cout = cexp;
  a.KH = a.KW = a.KWp = 1; a.stride = 1; a.pad = 0; a.K = K3; a.relu = 1; a.zero = dz; a.xcd = 1;
  if (cds) { a.x2 = dx2; a.H2 = H2; a.W2 = W2; a.Cin2 = cds; a.stride2 = 2; a.K1 = cmid; }
  int rc = launch_conv_bf16(a, 0);
  ConvArgs b{};
  b.x = y0; b.w = dw1; b.bias = db1; b.res = nullptr; b.y = z0;
  b.N = N; b.H = H; b.W = W; b.Cin = cexp; b.Ho = H; b.Wo = W; b.Cout = c1;
  b.KH = b.KW = b.KWp = 1; b.stride = 1; b.pad = 0; b.K = cexp; b.relu = 1; b.zero = dz; b.xcd = 1;
  rc |= launch_conv_bf16(b, 0);
  Pair1x1Args p{};
  p.x = dx; p.res = cds ? nullptr : dr; p.w3 = dw3; p.b3 = db3; p.w1 = dw1; p.b1 = db1;
  p.y = y1; p.z = z1; p.M = M; p.c1 = c1; p.cmid = cmid; p.cexp = cexp;
  if (cds) { p.x2 = dx2; p.cds = cds; p.Ho = H; p.Wo = W; p.H2 = H2; p.W2 = W2; }
  p.cap_elems = Mp * std::max(cmid, std::max(cexp, c1));
  std::vector<unsigned short> hy0(M * cexp), hy1(M * cexp), hz0(M * c1), hz1(M * c1);
  hipMemcpy(hy0.data(), y0, M * cexp * 2, hipMemcpyDeviceToHost);
  hipMemcpy(hz0.data(), z0, M * c1 * 2, hipMemcpyDeviceToHost);
  long bady = 0, badz = 0;
  double maxd = 0;
  int rcp = 0;
  const int REPS = reps ? reps : M % tile ? 8 : 1;
  void* flush = nullptr;
  if (stress) hipMalloc(&flush, 1LL << 30);
  if (inplace && !cds) p.res = y1;
  for (int rep = 0; rep < REPS; ++rep) {
    hipMemset(y1, 0xff, Mp * cexp * 2); hipMemset(z1, 0xff, Mp * c1 * 2);
    if (inplace && !cds) hipMemcpy(y1, dr, M * cexp * 2, hipMemcpyDeviceToDevice);
    if (stress) {
      hipMemset(flush, rep, 1LL << 30);
      hipLaunchKernelGGL(lds_poison_k, dim3(1024), dim3(256), 0, 0);
    }
    rcp |= launch_pairw_bf16(p, 0);
    hipDeviceSynchronize();
    hipMemcpy(hy1.data(), y1, M * cexp * 2, hipMemcpyDeviceToHost);
    hipMemcpy(hz1.data(), z1, M * c1 * 2, hipMemcpyDeviceToHost);
    for (size_t i = 0; i < hy0.size(); ++i)
      if (hy0[i] != hy1[i]) ++bady, maxd = std::max(maxd, (double)fabs(bf2f(hy0[i]) - bf2f(hy1[i])));
    for (size_t i = 0; i < hz0.size(); ++i)
      if (hz0[i] != hz1[i]) ++badz, maxd = std::max(maxd, (double)fabs(bf2f(hz0[i]) - bf2f(hz1[i])));
  }
  double maxerr = 0;  // the unfused conv3 itself against double on the bf16 operands (a few pixels)
  for (long long m = 0; m < M; m += M / 7 + 1)
    for (int o = 0; o < cexp; o += 7) {
      double acc = b3[o];
      for (int k = 0; k < cmid; ++k) acc += (double)bf2f(x[m * cmid + k]) * bf2f(w3[(size_t)o * K3 + k]);
      if (cds) {
        const long long n = m / (H * W), rem = m % (H * W), oh = rem / W, ow = rem % W;
        const size_t p2 = (size_t)((n * H2 + 2 * oh) * W2 + 2 * ow) * cds;
        for (int k = 0; k < cds; ++k) acc += (double)bf2f(x2[p2 + k]) * bf2f(w3[(size_t)o * K3 + cmid + k]);
      } else {
        acc += bf2f(res[m * cexp + o]);
      }
      acc = std::max(acc, 0.0);
      maxerr = std::max(maxerr, fabs(acc - bf2f(hy0[m * cexp + o])) / (1.0 + fabs(acc)));
    }
  const bool fail = rc || rcp || bady || badz || maxerr > 1e-2;
  printf("%s pairw bf16 N%d H%d W%d %d(+ds %d)->%d->%d M%lld rc=%d/%d differing y %ld z %ld (max %.3e) unfused maxerr %.3e\n",
         fail ? "FAIL" : "ok  ", N, H, W, cmid, cds, cexp, c1, M, rc, rcp, bady, badz, maxd, maxerr);
  for (void* q : {dx, dr, dx2, dw3, dw1, (void*)db3, (void*)db1, y0, y1, z0, z1, dz, flush}) hipFree(q);
  return fail ? 1 : 0;
}

int main(int argc, char** argv) {
  int fails = 0;
  if (argc > 1 && !strcmp(argv[1], "pairw_stress")) {  // the engine's in-place pairs at C2/C3 chunk sizes
    for (int n : {64, 130, 43, 257})
      for (int c1 : {128, 256}) fails += check_pairw(n, 28, 28, 128, 512, c1, 0, true, true, 4);
    fails += check_pairw(64, 14, 14, 256, 1024, 256, 0, true, true, 4);
    fails += check_pairw(64, 28, 28, 128, 512, 128, 256, false, true, 4);
    printf("%d failures\n", fails);
    return fails ? 1 : 0;
  }
  // R50 layer2 / layer3 wide pairs: within a stage (c1 = cmid) and into the next stage; many rounds
  // per workgroup (300 x 784 = 1838 rounds), ragged M (3 x 196 = 588: 4.6 rounds), tiny M
  fails += check_pairw(300, 28, 28, 128, 512, 128);
  fails += check_pairw(3, 28, 28, 128, 512, 256);
  fails += check_pairw(3, 14, 14, 256, 1024, 256);
  fails += check_pairw(200, 14, 14, 256, 1024, 256);
  fails += check_pairw(1, 7, 5, 128, 512, 128);
  // stage-2 block 0: conv3 + the folded stride-2 downsample (x2 = the 56x56x256 stage-1 output)
  fails += check_pairw(40, 28, 28, 128, 512, 128, 256);
  fails += check_pairw(3, 7, 5, 128, 512, 128, 256);
  // R50 layer1 pairs: block 1/2 (residual, c1 64), block 0 (downsample), layer1 -> layer2 (c1 128);
  // 700 images = 34300 tiles (~134 per workgroup), 64-wide maps (R101 @ 256)
  fails += check_pair(700, 56, 56, 64, false);
  fails += check_pair(9, 56, 56, 64, true);
  fails += check_pair(9, 56, 56, 128, false);
  fails += check_pair(5, 64, 64, 64, false);
  fails += check_pair(1, 8, 8, 64, true);  // one tile: the grid is smaller than the CU count
  fails += check_stem_pool(2, 224, 224);
  fails += check_stem_pool(3, 100, 86);  // ragged: partial last column tile, odd pooled sizes
  fails += check_stem_pool(2, 64, 48);
  fails += check_stem_pool(2, 224, 224, true);
  fails += check_stem_pool(3, 100, 86, true);
  fails += check_stem_pool(2, 64, 48, true);
  // column-blocked direct kernel (W % 4 == 0): ResNet-101's 256 x 256 (3 column blocks, the last
  // half idle), a ragged last block, a single partial block
  if (stem_pool_bf16_ok(256, 256, true)) fails += check_stem_pool(2, 256, 256, true);  // (EOSV_STEM_CB=0: unfused)
  fails += check_stem_pool(3, 100, 88, true);
  fails += check_stem_pool(2, 60, 36, true);
  fails += check_stem_pool_x3(2, 224, 224);
  fails += check_stem_pool_x3(2, 256, 256);
  fails += check_stem_pool_x3(3, 60, 36);
  fails += check_stem_pool_f32(2, 224, 224);
  fails += check_stem_pool_f32(3, 100, 86);
  fails += check_stem_pool_f32(2, 64, 48);
  fails += check_stem_pool_f32(2, 40, 200);  // Ws 100: a partial last column tile
  fails += check_stem_pool_f32(2, 256, 256);  // 8 column tiles
  // row bands (one workgroup per band of pooled rows): 8 bands at small N, 3 at 1000, 7-8 at 2400
  fails += check_stem_pool_f32(1000, 224, 224, 333);
  fails += check_stem_pool_f32(2400, 224, 224, 797);
  // stage-1 shape (row-strip kernel): 300 images = 4200 strips, several strips per workgroup
  fails += check_bf16(300, 56, 56, 64, 64, 3, 1, 1, true, true);
  fails += check_bf16(3, 56, 56, 64, 64, 3, 1, 1, false, true);
  // phased 8-wave kernel: 512x128 (Cout 128) and 256x256 tiles, strided entries, 1x1s, M tails
  fails += check_bf16(40, 28, 28, 128, 128, 3, 1, 1, true, true);
  fails += check_bf16(40, 28, 28, 128, 128, 3, 1, 1, true, true, true);
  fails += check_bf16(30, 14, 14, 256, 256, 3, 1, 1, true, true, true);
  fails += check_bf16(9, 28, 28, 128, 256, 3, 2, 1, false, true, true);
  fails += check_bf16(3, 7, 7, 512, 512, 3, 1, 1, false, true, true);
  fails += check_bf16(2, 9, 11, 128, 128, 3, 1, 1, true, false, true);
  fails += check_bf16(7, 56, 56, 64, 128, 3, 2, 1, false, true);
  // r05 register-weight row strips (conv_rowsr_bf16.hip) called directly: C 64 at 56x56, C 128 at 28x28
  g_bf16_launch = launch_conv_rowsr_bf16;
  fails += check_bf16(300, 56, 56, 64, 64, 3, 1, 1, true, true);
  fails += check_bf16(37, 56, 56, 64, 64, 3, 1, 1, false, true);
  fails += check_bf16(3, 56, 56, 64, 64, 3, 1, 1, true, false);
  fails += check_bf16(300, 28, 28, 128, 128, 3, 1, 1, true, true);
  fails += check_bf16(41, 28, 28, 128, 128, 3, 1, 1, false, true);
  fails += check_bf16(2, 28, 28, 128, 128, 3, 1, 1, true, false);
  fails += check_bf16(40, 28, 28, 128, 128, 3, 1, 1, true, true, true);   // chunk-major K weights
  fails += check_bf16(45, 64, 64, 64, 64, 3, 1, 1, true, true);
  fails += check_bf16(7, 64, 64, 64, 64, 3, 1, 1, false, true);
  fails += check_bf16(33, 32, 32, 128, 128, 3, 1, 1, true, true, true);
  fails += check_bf16(6, 32, 32, 128, 128, 3, 1, 1, false, true, true);
  g_bf16_launch = launch_conv_bf16;
  fails += check_bf16(300, 56, 56, 64, 128, 3, 2, 1, false, true);   // stride-2 entry row strips: several per workgroup
  fails += check_bf16(37, 56, 56, 64, 128, 3, 2, 1, false, false);   // ... without ReLU, ragged strip count
  fails += check_bf16(5, 56, 56, 128, 128, 3, 2, 1, false, true, true);  // R50 layer2.0.conv2 (kcm)
  fails += check_bf16(3, 13, 11, 64, 128, 3, 2, 1, false, true);         // ragged stride-2 entry, M tail
  fails += check_bf16(7, 56, 56, 64, 128, 1, 2, 0, false, false);
  fails += check_bf16(30, 14, 14, 256, 256, 3, 1, 1, true, true);
  fails += check_bf16(9, 28, 28, 128, 256, 3, 2, 1, false, true);
  fails += check_bf16(20, 7, 7, 512, 512, 3, 1, 1, true, true);
  fails += check_bf16(3, 7, 7, 512, 512, 3, 1, 1, false, true);  // M = 147 < one 256-row tile
  fails += check_bf16(5, 14, 14, 1024, 256, 1, 1, 0, false, true);
  fails += check_bf16(5, 14, 14, 256, 1024, 1, 1, 0, true, true);
  fails += check_bf16(2, 9, 11, 128, 128, 3, 1, 1, true, false);  // ragged map, M = 198
  // halo-staged stride-1 3x3s (conv_halo_bf16, kcm weights, Cout % 256 == 0): 16x16 / 8x8 maps
  // (256x256 input), a ragged map with an M tail, Cout 512 (two cout tiles)
  fails += check_bf16(7, 16, 16, 256, 256, 3, 1, 1, true, true, true);
  fails += check_bf16(5, 8, 8, 512, 512, 3, 1, 1, false, true, true);
  fails += check_bf16(3, 10, 12, 128, 256, 3, 1, 1, true, false, true);
  fails += check_bf16(11, 7, 7, 256, 512, 3, 1, 1, true, true, true);
  fails += check(1, 8, 8, 32, 64, 1, 1, 0, false, false, false);
  fails += check(2, 9, 7, 64, 64, 3, 1, 1, false, false, false);
  fails += check(2, 14, 14, 64, 128, 3, 2, 1, false, true, true);
  fails += check(3, 7, 7, 256, 512, 1, 2, 0, false, false, false);
  fails += check(1, 7, 7, 512, 512, 3, 1, 1, false, true, true);
  fails += check(2, 30, 30, 3, 64, 7, 2, 3, true, false, true);
  fails += check(3, 37, 33, 3, 64, 7, 2, 3, true, false, true);  // odd sizes: row-width rounding, M tail
  fails += check(5, 1, 1, 512, 64, 1, 1, 0, false, false, false);
  // f32 stride-1 3x3 convs at the stage shapes of R18/R50, the fused downsample (K columns
  // [K1, K) from x2), ragged maps and M tails; exact-f32 products, so a tight bound
  fails += check(12, 56, 56, 64, 64, 3, 1, 1, false, true, true, 0, 2e-6);
  // f32 stage-1 row-strip kernel (conv_rows_f32.hip): 560 strips (2-3 per workgroup), R50's
  // residual-free conv, 64-wide maps (256x256 input), no ReLU
  fails += check(20, 56, 56, 64, 64, 3, 1, 1, false, true, true, 0, 2e-6);
  fails += check(3, 56, 56, 64, 64, 3, 1, 1, false, false, true, 0, 2e-6);
  fails += check(4, 64, 64, 64, 64, 3, 1, 1, false, true, true, 0, 2e-6);
  fails += check(2, 64, 64, 64, 64, 3, 1, 1, false, false, false, 0, 2e-6);
  fails += check(5, 28, 28, 128, 128, 3, 1, 1, false, false, true, 64, 2e-6);
  fails += check(6, 14, 14, 256, 256, 3, 1, 1, false, true, true, 0, 2e-6);
  fails += check(4, 14, 14, 256, 256, 3, 1, 1, false, false, true, 128, 2e-6);
  fails += check(3, 7, 7, 512, 512, 3, 1, 1, false, false, true, 256, 2e-6);
  // chunk-major K order (r04, the library's f32 weights at Cin >= 128): the R18 / R50 stage-2..4
  // 3x3s at grids that take every tile (256x128, 128x128, 128x64), stride 2, the fused downsample
  fails += check(50, 28, 28, 128, 128, 3, 1, 1, false, true, true, 0, 2e-6, true);
  fails += check(40, 28, 28, 128, 128, 3, 1, 1, false, false, true, 64, 2e-6, true);
  fails += check(60, 14, 14, 256, 256, 3, 1, 1, false, true, true, 0, 2e-6, true);
  fails += check(30, 28, 28, 128, 256, 3, 2, 1, false, false, true, 0, 2e-6, true);
  fails += check(40, 7, 7, 512, 512, 3, 1, 1, false, true, true, 0, 2e-6, true);
  fails += check(4, 14, 14, 256, 256, 3, 1, 1, false, false, true, 128, 2e-6, true);
  fails += check(3, 9, 11, 160, 96, 3, 1, 1, false, true, false, 0, 2e-6, true);
  // grids at / above the CU count: the large 256x128 and 128x128 tiles (small N takes 128x64)
  fails += check(21, 56, 56, 32, 128, 3, 1, 1, false, true, true, 0, 2e-6);
  fails += check(11, 28, 28, 32, 512, 1, 1, 0, false, false, true, 0, 2e-6);
  fails += check(3, 9, 11, 32, 64, 3, 1, 1, false, true, false, 0, 2e-6);
  fails += check(2, 5, 3, 32, 128, 3, 1, 1, false, true, true, 32, 2e-6);
  printf("%d failures\n", fails);
  return fails;
}
