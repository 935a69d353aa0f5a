// Layer-level check of bneck_bf16 (the r06 whole-block stage-1 kernel), bneck_tail_bf16 and bblock_bf16: seeded
// random bf16 operands, every output checked against a CPU reference (f32 accumulation, bf16 rounding
// between the convs as the kernels do; tolerance for the summation order), and REPEAT launches on
// the same inputs compared bitwise -- a race shows as run-to-run differences, reported with its
// first (image, row, column, channel).
// Build: hipcc --offload-arch=gfx950 -O2 -I include -I <pkg>/csrc bneck_check.cpp -L<pkg> -leosv
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.h"

using namespace eosv;
typedef unsigned short u16;

static float frand(unsigned& s) {
  s = s * 1664525u + 1013904223u;
  return ((s >> 8) & 0xffff) / 32768.f - 1.f;
}
static u16 f2bf(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (u16)(u >> 16);
}
static float bf2f(u16 v) {
  unsigned u = (unsigned)v << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static float rb(float f) { return bf2f(f2bf(f)); }

struct Dev {
  void* p = nullptr;
  explicit Dev(size_t bytes) { hipMalloc(&p, bytes); }
  ~Dev() { hipFree(p); }
};
template <class T>
static void up(Dev& d, const std::vector<T>& v) { hipMemcpy(d.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice); }

// tail = false: block with conv1 (cin 64 + downsample, or 256 [+ next 64]); tail = true: from Z
static int check(int N, int H, int W, int cin, bool next, bool tail, int reps) {
  unsigned s = 777u + 31u * (unsigned)(N * 131 + H * 17 + cin + next * 7 + tail * 3);
  const int M = N * H * W, K3 = cin == 64 && !tail ? 128 : 64, cn = tail ? 128 : 64;
  const int cx = tail ? 64 : cin;  // channels of the kernel's x
  std::vector<u16> x((size_t)M * cx), res(tail ? (size_t)M * 256 : 0), w1((size_t)64 * cin), w2((size_t)64 * 576),
      w3((size_t)256 * K3), wn((size_t)cn * 256);
  std::vector<float> b1(64), b2(64), b3(256), bn(cn);
  auto fill = [&](std::vector<u16>& v, float sc) {
    for (auto& e : v) e = f2bf(frand(s) * sc);
  };
  fill(x, 1.f);
  fill(res, 1.f);
  fill(w1, 0.15f);
  fill(w2, 0.05f);
  fill(w3, 0.15f);
  fill(wn, 0.08f);
  for (auto* b : {&b1, &b2, &b3, &bn})
    for (auto& e : *b) e = frand(s) * 0.1f;
  // CPU reference over the first NR images (the rest: repeat comparisons only)
  const int NR = N < 3 ? N : 3, MR = NR * H * W;
  std::vector<float> t1((size_t)MR * 64), t2((size_t)MR * 64), y((size_t)MR * 256), z((size_t)MR * cn);
  for (int p = 0; p < MR; ++p)
    for (int o = 0; o < 64; ++o) {
      if (tail) {
        t1[(size_t)p * 64 + o] = bf2f(x[(size_t)p * 64 + o]);
        continue;
      }
      float a = 0.f;
      for (int c = 0; c < cin; ++c) a += bf2f(w1[(size_t)o * cin + c]) * bf2f(x[(size_t)p * cin + c]);
      t1[(size_t)p * 64 + o] = rb(fmaxf(a + b1[o], 0.f));
    }
  for (int n = 0; n < NR; ++n)
    for (int i = 0; i < H; ++i)
      for (int j = 0; j < W; ++j)
        for (int o = 0; o < 64; ++o) {
          float a = 0.f;
          for (int dy = 0; dy < 3; ++dy)
            for (int dx = 0; dx < 3; ++dx) {
              const int ii = i + dy - 1, jj = j + dx - 1;
              if (ii < 0 || ii >= H || jj < 0 || jj >= W) continue;
              const float* tp = &t1[(((size_t)n * H + ii) * W + jj) * 64];
              const u16* wp = &w2[(size_t)o * 576 + (dy * 3 + dx) * 64];
              for (int c = 0; c < 64; ++c) a += bf2f(wp[c]) * tp[c];
            }
          t2[(((size_t)n * H + i) * W + j) * 64 + o] = rb(fmaxf(a + b2[o], 0.f));
        }
  for (int p = 0; p < MR; ++p) {
    for (int o = 0; o < 256; ++o) {
      float a = 0.f;
      for (int c = 0; c < 64; ++c) a += bf2f(w3[(size_t)o * K3 + c]) * t2[(size_t)p * 64 + c];
      if (K3 == 128)
        for (int c = 0; c < 64; ++c) a += bf2f(w3[(size_t)o * K3 + 64 + c]) * bf2f(x[(size_t)p * 64 + c]);
      float v = a + b3[o];
      if (tail) v += bf2f(res[(size_t)p * 256 + o]);
      else if (cin == 256) v += bf2f(x[(size_t)p * 256 + o]);
      y[(size_t)p * 256 + o] = rb(fmaxf(v, 0.f));
    }
    if (next || tail)
      for (int o = 0; o < cn; ++o) {
        float a = 0.f;
        for (int c = 0; c < 256; ++c) a += bf2f(wn[(size_t)o * 256 + c]) * y[(size_t)p * 256 + c];
        z[(size_t)p * cn + o] = rb(fmaxf(a + bn[o], 0.f));
      }
  }
  Dev dx(x.size() * 2), dres(res.size() * 2 + 16), dw1(w1.size() * 2), dw2(w2.size() * 2), dw3(w3.size() * 2),
      dwn(wn.size() * 2), db1(256), db2(256), db3(1024), dbn(512), dy((size_t)M * 512), dz((size_t)M * cn * 2 + 16);
  up(dx, x);
  if (tail) up(dres, res);
  up(dw1, w1);
  up(dw2, w2);
  up(dw3, w3);
  up(dwn, wn);
  up(db1, b1);
  up(db2, b2);
  up(db3, b3);
  up(dbn, bn);
  BneckArgs a{};
  a.x = dx.p;
  a.res = tail ? dres.p : nullptr;
  a.w1 = dw1.p;
  a.b1 = (const float*)db1.p;
  a.w2 = dw2.p;
  a.b2 = (const float*)db2.p;
  a.w3 = dw3.p;
  a.b3 = (const float*)db3.p;
  a.wn = next || tail ? dwn.p : nullptr;
  a.bn = next || tail ? (const float*)dbn.p : nullptr;
  a.y = dy.p;
  a.z = next || tail ? dz.p : nullptr;
  a.N = N;
  a.H = H;
  a.W = W;
  a.cin = tail ? 64 : cin;
  std::vector<u16> y0((size_t)M * 256), z0((size_t)M * cn), y1(y0.size()), z1(z0.size());
  int bad = 0, racy = 0;
  double maxerr = 0.0;
  for (int rep = 0; rep < reps; ++rep) {
    hipMemset(dy.p, 0xff, (size_t)M * 512);
    if (next || tail) hipMemset(dz.p, 0xff, (size_t)M * cn * 2);
    const int rc = tail ? launch_bneck_tail_bf16(a, nullptr) : launch_bneck_bf16(a, nullptr);
    if (rc || hipDeviceSynchronize() != hipSuccess) {
      printf("FAIL launch rc=%d %s\n", rc, eosv_last_error());
      return 1;
    }
    hipMemcpy(rep ? y1.data() : y0.data(), dy.p, y0.size() * 2, hipMemcpyDeviceToHost);
    if (next || tail) hipMemcpy(rep ? z1.data() : z0.data(), dz.p, z0.size() * 2, hipMemcpyDeviceToHost);
    if (rep) {
      for (size_t i = 0; i < y0.size(); ++i)
        if (y0[i] != y1[i]) {
          if (racy++ < 4) {
            const size_t p = i / 256;
            printf("  race Y rep %d: image %zu row %zu col %zu ch %zu: %g vs %g\n", rep, p / (H * W), (p / W) % H, p % W,
                   i % 256, bf2f(y0[i]), bf2f(y1[i]));
          }
        }
      if (next || tail)
        for (size_t i = 0; i < z0.size(); ++i)
          if (z0[i] != z1[i] && racy++ < 8) {
            const size_t p = i / cn;
            printf("  race Z rep %d: image %zu row %zu col %zu ch %zu\n", rep, p / (H * W), (p / W) % H, p % W, i % cn);
          }
    }
  }
  auto cmp = [&](const std::vector<u16>& g, const std::vector<float>& r, int C, const char* nm) {
    for (size_t i = 0; i < r.size(); ++i) {
      const double e = fabs((double)bf2f(g[i]) - r[i]);
      maxerr = fmax(maxerr, e);
      if (e > 0.05 + 0.02 * fabs(r[i]) && bad++ < 4) {
        const size_t p = i / C;
        printf("  bad %s image %zu row %zu col %zu ch %zu: got %g ref %g\n", nm, p / (H * W), (p / W) % H, p % W,
               i % C, bf2f(g[i]), r[i]);
      }
    }
  };
  cmp(y0, y, 256, "Y");
  if (next || tail) cmp(z0, z, cn, "Z");
  printf("%s %s N%d H%d W%d cin%d next%d reps %d: maxerr %.3g bad %d racy %d\n", bad || racy ? "FAIL" : "ok  ",
         tail ? "tail " : "bneck", N, H, W, cin, (int)next, reps, maxerr, bad, racy);
  return bad || racy ? 1 : 0;
}

// bblock_bf16 (the fused R18 stage-1 basic block): y = relu(conv2(relu(conv1(x) + b1)) + b2 + x),
// checked like the bottleneck kernels (CPU reference over the first images + repeat launches), in
// place (y = x, as the engine runs it) when inplace is set
static int check_bblock(int N, int H, int W, bool inplace, int reps) {
  unsigned s = 4242u + 17u * (unsigned)(N * 7 + H + inplace);
  const int M = N * H * W;
  std::vector<u16> x((size_t)M * 64), w1((size_t)64 * 576), w2((size_t)64 * 576);
  std::vector<float> b1(64), b2(64);
  for (auto& e : x) e = f2bf(frand(s));
  for (auto& e : w1) e = f2bf(frand(s) * 0.05f);
  for (auto& e : w2) e = f2bf(frand(s) * 0.05f);
  for (auto& e : b1) e = frand(s) * 0.1f;
  for (auto& e : b2) e = frand(s) * 0.1f;
  const int NR = N < 3 ? N : 3;
  auto conv = [&](const std::vector<float>& in, const std::vector<u16>& w, std::vector<float>& out) {
    for (int n = 0; n < NR; ++n)
      for (int i = 0; i < H; ++i)
        for (int j = 0; j < W; ++j)
          for (int o = 0; o < 64; ++o) {
            float a = 0.f;
            for (int dy = 0; dy < 3; ++dy)
              for (int dx = 0; dx < 3; ++dx) {
                const int ii = i + dy - 1, jj = j + dx - 1;
                if (ii < 0 || ii >= H || jj < 0 || jj >= W) continue;
                const float* tp = &in[(((size_t)n * H + ii) * W + jj) * 64];
                const u16* wp = &w[(size_t)o * 576 + (dy * 3 + dx) * 64];
                for (int c = 0; c < 64; ++c) a += bf2f(wp[c]) * tp[c];
              }
            out[(((size_t)n * H + i) * W + j) * 64 + o] = a;
          }
  };
  const size_t MR = (size_t)NR * H * W;
  std::vector<float> xf(MR * 64), t(MR * 64), y(MR * 64);
  for (size_t i = 0; i < MR * 64; ++i) xf[i] = bf2f(x[i]);
  conv(xf, w1, t);
  for (size_t i = 0; i < MR * 64; ++i) t[i] = rb(fmaxf(t[i] + b1[i % 64], 0.f));
  conv(t, w2, y);
  for (size_t i = 0; i < MR * 64; ++i) y[i] = rb(fmaxf(y[i] + b2[i % 64] + xf[i], 0.f));
  Dev dx(x.size() * 2), dy(x.size() * 2), dw1(w1.size() * 2), dw2(w2.size() * 2), db1(256), db2(256);
  up(dw1, w1);
  up(dw2, w2);
  up(db1, b1);
  up(db2, b2);
  BneckArgs a{};
  a.x = dx.p;
  a.w1 = dw1.p;
  a.b1 = (const float*)db1.p;
  a.w2 = dw2.p;
  a.b2 = (const float*)db2.p;
  a.y = inplace ? dx.p : dy.p;
  a.N = N;
  a.H = H;
  a.W = W;
  a.cin = 64;
  std::vector<u16> y0(x.size()), y1(x.size());
  int bad = 0, racy = 0;
  double maxerr = 0.0;
  for (int rep = 0; rep < reps; ++rep) {
    up(dx, x);  // in place overwrites the input: restore it every launch
    if (!inplace) hipMemset(dy.p, 0xff, x.size() * 2);
    if (launch_bblock_bf16(a, nullptr) || hipDeviceSynchronize() != hipSuccess) {
      printf("FAIL launch %s\n", eosv_last_error());
      return 1;
    }
    hipMemcpy(rep ? y1.data() : y0.data(), a.y, x.size() * 2, hipMemcpyDeviceToHost);
    if (rep)
      for (size_t i = 0; i < y0.size(); ++i)
        if (y0[i] != y1[i] && racy++ < 4) {
          const size_t p = i / 64;
          printf("  race Y rep %d: image %zu row %zu col %zu ch %zu\n", rep, p / (H * W), (p / W) % H, p % W, i % 64);
        }
  }
  for (size_t i = 0; i < MR * 64; ++i) {
    const double e = fabs((double)bf2f(y0[i]) - y[i]);
    maxerr = fmax(maxerr, e);
    if (e > 0.05 + 0.02 * fabs(y[i]) && bad++ < 4) {
      const size_t p = i / 64;
      printf("  bad Y image %zu row %zu col %zu ch %zu: got %g ref %g\n", p / (H * W), (p / W) % H, p % W, i % 64,
             bf2f(y0[i]), y[i]);
    }
  }
  printf("%s bblock N%d H%d W%d %s reps %d: maxerr %.3g bad %d racy %d\n", bad || racy ? "FAIL" : "ok  ", N, H, W,
         inplace ? "in place" : "out of place", reps, maxerr, bad, racy);
  return bad || racy ? 1 : 0;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 4;
  int fails = 0;
  // one image per workgroup (N < CUs) and several (N > CUs: the stream crosses images)
  for (int W : {56, 64}) {
    fails += check(37, W, W, 64, false, false, reps);
    fails += check(37, W, W, 256, true, false, reps);
    fails += check(37, W, W, 256, false, false, reps);
    fails += check(37, W, W, 64, false, true, reps);
    fails += check(300, W, W, 64, false, false, 2);
    fails += check(300, W, W, 256, true, false, 2);
    fails += check(300, W, W, 64, false, true, 2);
  }
  for (int W : {56, 64}) {
    fails += check_bblock(37, W, W, true, reps);
    fails += check_bblock(300, W, W, false, 2);
  }
  printf("\n%d failures\n", fails);
  return fails ? 1 : 0;
}
