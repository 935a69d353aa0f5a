// eosv C ABI: handle lifecycle, weight folding and the backbone layer plan.
//
// The native runtime owns what torchvision/cuDNN owned in the reference
// (models.py:9-37): the ResNet layer plan (built from the arch id, torchvision v1.5
// structure), BN folded into conv weights at load time, NHWC workspaces sized for
// max_frames, and the per-chunk launch sequence
//   pack NCHW->padded RGB -> stem conv (+BN+ReLU) -> maxpool -> blocks (conv+BN[+ReLU],
//   residual add + ReLU fused into the last conv's epilogue) -> avgpool.
#include <hip/hip_bf16.h>

#include <cmath>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.h"

#ifndef EOSV_F32_KCM_DEF
#define EOSV_F32_KCM_DEF 64  // release default of the f32 K order: 64-channel chunk-major (r05), 0 = tap-major
#endif

namespace eosv {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

int device_cu_count() {
  static const int n = [] {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) ||
        c <= 0)
      return 256;
    return c;
  }();
  return n;
}

int kernel_occupancy(const void* kernel, int threads, size_t dyn_lds) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, threads, dyn_lds) != hipSuccess || n < 1) n = 1;
  return n;
}

#ifdef EOSV_PROFILING
int env_switch(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
#endif

struct Conv {
  int cin = 0, cout = 0, kh = 1, kw = 1, kwp = 1, cinp = 0, stride = 1, pad = 0, K = 0;
  bool stem = false;
  bool kcm = false;           // weights in chunk-major K order (ConvArgs::kcm), chunks of kcmc channels
  int kcmc = 64;
  int kds = 0;                // fused downsample: extra K columns (its Cin) after this conv's K
  int id = 0;                 // layer id for profiling (plan order)
  std::string wname, bnname;  // state_dict prefixes
  void* w = nullptr;          // [cout][K] (f32 or bf16)
  float* b = nullptr;         // [cout]
  size_t wbytes = 0;          // size of the w allocation (reused by a reload of the same shape)
};

struct Block {
  bool bottleneck = false, has_ds = false;
  bool fuse_ds = false;  // downsample folded into the last conv's K (ConvArgs::x2), no ds launch
  Conv c1, c2, c3, ds;
};

}  // namespace eosv

struct eosv_handle {
  eosv_desc d{};
  int D = 0;
  int hs = 0, ws = 0, hp = 0, wp = 0;  // stem / maxpool output sizes
  eosv::Conv stem, fc;
  eosv::Conv stem_x3;  // EOSV_F32X3 split-bf16 stem: w = [hi | lo] [64][192] bf16 (stem_pool_bf16.hip)
  std::vector<eosv::Block> blocks;
  bool loaded = false;
  size_t act_elems = 0;  // per-frame max activation elements
  void* pack = nullptr;
  void* zero = nullptr;  // 256 zeroed bytes: DMA source for out-of-bounds conv taps
  void* buf[4] = {nullptr, nullptr, nullptr, nullptr};
  void* sbuf[4] = {nullptr, nullptr, nullptr, nullptr};  // sub-chunk scratch for the front stages
  int sub_frames = 0;          // front-stage sub-chunk (0 = off)
  size_t n_front = 0;          // blocks in the front phase (layer1)
  size_t stage_end[4] = {0, 0, 0, 0};  // blocks of layer1 .. layerN (cumulative)
  int stage_hwc[5][3] = {};            // output (h, w, channels) of the stem + maxpool and each layer
  size_t front_out_elems = 0;  // per-frame elements of the layer1 output
  int front_hw[2] = {0, 0};
  std::vector<void*> allocs;
  int64_t bytes = 0;
  int n_layers = 0;
  // profiling (eosv_profile_enable/read)
  struct Rec {
    int id;
    hipEvent_t a, b;
    double flops;
  };
  bool prof = false;
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  size_t pool_used = 0;
  // chunk planner (eosv_backbone_forward): a dry run of forward_chunk prices a chunk size
  bool planning = false;
  double plan_cost = 0.0;
  std::vector<double> chunk_cost;                          // by chunk size, filled on first use
  std::unordered_map<int, std::vector<int>> chunk_plans;   // by frame count
};

namespace eosv {

static int conv_out(int h, int k, int s, int p) { return (h + 2 * p - k) / s + 1; }

// empty marker dispatches bracketing a profiling window (eosv_profile_enable)
__global__ void profile_window_begin_kernel() {}
__global__ void profile_window_end_kernel() {}

// dtype roles: the residual-block convs run on the bf16 kernels for EOSV_BF16 and EOSV_F32X3;
// the stem is bf16 only for EOSV_BF16 (EOSV_F32X3 keeps it exact f32, split output)
static bool x3(const eosv_handle* h) { return h->d.dtype == EOSV_F32X3; }
static bool conv_bf(const eosv_handle* h) { return h->d.dtype != EOSV_F32; }
static bool stem_bf(const eosv_handle* h) { return h->d.dtype == EOSV_BF16; }
// bytes per activation element: f32 4, bf16 2, split (hi, lo) 4
static size_t act_bytes(const eosv_handle* h) { return x3(h) ? 4 : conv_bf(h) ? 2 : 4; }

static Conv make_conv(int cin, int cout, int k, int stride, int pad, const std::string& wname,
                      const std::string& bnname) {
  Conv c;
  c.cin = cin;
  c.cout = cout;
  c.kh = c.kw = c.kwp = k;
  c.cinp = cin;
  c.stride = stride;
  c.pad = pad;
  c.K = k * k * cin;
  c.wname = wname;
  c.bnname = bnname;
  return c;
}

// The block shortcut's 1x1 downsample conv (+ its folded BN) becomes extra K columns of the
// block's last conv: out = relu(W_last . h + W_ds . x_strided + b_last + b_ds), one launch
// instead of two and no residual round trip through HBM.  EOSV_FUSE_DS=0: separate launch.
static bool fuse_ds_enabled() {
  static const bool v = env_switch("EOSV_FUSE_DS", 1) != 0;
  return v;
}

static int build_plan(eosv_handle* h) {
  const int arch = h->d.arch;
  int layers[4];
  bool bottleneck;
  if (arch == EOSV_ARCH_R18) {
    bottleneck = false;
    int l[4] = {2, 2, 2, 2};
    memcpy(layers, l, sizeof l);
  } else if (arch == EOSV_ARCH_R50) {
    bottleneck = true;
    int l[4] = {3, 4, 6, 3};
    memcpy(layers, l, sizeof l);
  } else if (arch == EOSV_ARCH_R101) {
    bottleneck = true;
    int l[4] = {3, 4, 23, 3};
    memcpy(layers, l, sizeof l);
  } else {
    set_error("eosv_create: unsupported arch (18, 50, 101)");
    return EOSV_ERR_UNSUPPORTED;
  }
  const int exp = bottleneck ? 4 : 1;
  h->D = 512 * exp;
  // stem: 7x7/2 p3 on dense padded RGB; K = [kh 7][24] (kw*3 + c, 3 zero weights per kh)
  // padded to the kernel's K-step: f32 176 (BK 16), bf16 192 (BK 64)
  Conv st = make_conv(3, 64, 7, 2, 3, "convnet.0.weight", "convnet.1");
  st.stem = true;
  st.kwp = 8;
  st.cinp = 3;
  st.K = h->d.dtype == EOSV_BF16 ? 192 : 176;
  h->stem = st;
  h->hs = conv_out(h->d.height, 7, 2, 3);
  h->ws = conv_out(h->d.width, 7, 2, 3);
  h->hp = conv_out(h->hs, 3, 2, 1);
  h->wp = conv_out(h->ws, 3, 2, 1);
  size_t act = (size_t)h->hs * h->ws * 64;
  int hh = h->hp, ww = h->wp, inpl = 64;
  for (int li = 0; li < 4; ++li) {
    const int planes = 64 << li;
    for (int bi = 0; bi < layers[li]; ++bi) {
      const int s = (li > 0 && bi == 0) ? 2 : 1;
      const std::string p = "convnet." + std::to_string(4 + li) + "." + std::to_string(bi);
      Block b;
      b.bottleneck = bottleneck;
      const int cout = planes * exp;
      const int ho = conv_out(hh, 3, s, 1), wo = conv_out(ww, 3, s, 1);
      if (!bottleneck) {
        b.c1 = make_conv(inpl, planes, 3, s, 1, p + ".conv1.weight", p + ".bn1");
        b.c2 = make_conv(planes, planes, 3, 1, 1, p + ".conv2.weight", p + ".bn2");
        act = std::max(act, (size_t)ho * wo * planes);
      } else {
        b.c1 = make_conv(inpl, planes, 1, 1, 0, p + ".conv1.weight", p + ".bn1");
        b.c2 = make_conv(planes, planes, 3, s, 1, p + ".conv2.weight", p + ".bn2");
        b.c3 = make_conv(planes, cout, 1, 1, 0, p + ".conv3.weight", p + ".bn3");
        act = std::max(act, (size_t)hh * ww * planes);
        act = std::max(act, (size_t)ho * wo * cout);
      }
      if (bi == 0 && (s != 1 || inpl != cout)) {
        b.has_ds = true;
        b.ds = make_conv(inpl, cout, 1, s, 0, p + ".downsample.0.weight", p + ".downsample.1");
        b.fuse_ds = fuse_ds_enabled();
        if (b.fuse_ds) (bottleneck ? b.c3 : b.c2).kds = inpl;
      }
      h->blocks.push_back(b);
      hh = ho;
      ww = wo;
      inpl = cout;
      if (li == 0) {
        h->n_front = h->blocks.size();
        h->front_out_elems = (size_t)hh * ww * cout;
        h->front_hw[0] = hh;
        h->front_hw[1] = ww;
      }
    }
    h->stage_end[li] = h->blocks.size();
    h->stage_hwc[li + 1][0] = hh;
    h->stage_hwc[li + 1][1] = ww;
    h->stage_hwc[li + 1][2] = inpl;
  }
  h->stage_hwc[0][0] = h->hp;
  h->stage_hwc[0][1] = h->wp;
  h->stage_hwc[0][2] = 64;
  h->act_elems = act;
  Conv fc = make_conv(h->D, h->d.num_classes, 1, 1, 0, "fc.weight", "");
  h->fc = fc;
  int id = 0;
  h->stem.id = id++;
  for (Block& b : h->blocks) {
    b.c1.id = id++;
    b.c2.id = id++;
    if (b.bottleneck) b.c3.id = id++;
    if (b.has_ds) b.ds.id = id++;
  }
  h->fc.id = id++;
  h->n_layers = id;
  if (x3(h)) {
    // split layout: every block conv reads 3 * cin virtual channels (hi, lo, hi) of the stored
    // (hi, lo) pixels
    auto widen = [](Conv& c) {
      c.cinp = 3 * c.cin;
      c.K = c.kh * c.kw * c.cinp;
      c.kds *= 3;
    };
    for (Block& b : h->blocks) {
      widen(b.c1);
      widen(b.c2);
      if (b.bottleneck) widen(b.c3);
      if (b.has_ds) widen(b.ds);
    }
  }
  return EOSV_OK;
}

static int dmalloc(eosv_handle* h, void** p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    set_error("hipMalloc(" + std::to_string(bytes) + "): " + hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? EOSV_ERR_OOM : EOSV_ERR_HIP;
  }
  h->allocs.push_back(*p);
  h->bytes += (int64_t)bytes;
  return EOSV_OK;
}

// Copy host bytes into a weight buffer.  The handle's layer shapes are fixed, so a reload
// (eosv_load_weights called again) overwrites the previous allocation in place instead of
// allocating a new one: device memory stays constant across reloads.
static int upload_bytes(eosv_handle* h, void** dst, size_t* cap, const void* src, size_t bytes) {
  int rc;
  if (!*dst || *cap != bytes) {
    if ((rc = dmalloc(h, dst, bytes))) return rc;
    *cap = bytes;
  }
  EOSV_HIP_CHECK(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
  return EOSV_OK;
}

static unsigned short f2bf_host(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

struct Tensors {
  std::unordered_map<std::string, std::pair<const float*, int64_t>> m;
  const float* get(const std::string& n, int64_t numel) const {
    auto it = m.find(n);
    if (it == m.end()) {
      set_error("eosv_load_weights: missing tensor '" + n + "'");
      return nullptr;
    }
    if (it->second.second != numel) {
      set_error("eosv_load_weights: tensor '" + n + "' has " + std::to_string(it->second.second) +
                " elements, expected " + std::to_string(numel));
      return nullptr;
    }
    return it->second.first;
  }
};

// fold BN (eval) into the conv: host [cout][K] weights (K order as the kernels read it) and
// [cout] shift.  False (error set) on a missing tensor.
static float bf_round_host(float f) {
  const unsigned u = (unsigned)f2bf_host(f) << 16;
  float r;
  memcpy(&r, &u, 4);
  return r;
}

// split (EOSV_F32X3): c.cinp = 3 * c.cin virtual input channels; folded weight v goes to
// channels i and cin + i as hi = bf16(v) and to 2 cin + i as lo = bf16(v - hi), so the
// (hi, lo, hi) activation blocks give hi.hi + lo.hi + hi.lo
static bool fold_conv(Conv& c, const Tensors& t, bool bf16, bool has_bn, std::vector<float>& wf,
                      std::vector<float>& beta, bool split = false) {
  const float* w = t.get(c.wname, (int64_t)c.cout * c.cin * c.kh * c.kw);
  if (!w) return false;
  std::vector<float> alpha(c.cout, 1.f);
  beta.assign(c.cout, 0.f);
  if (has_bn) {
    const float* g = t.get(c.bnname + ".weight", c.cout);
    const float* bb = t.get(c.bnname + ".bias", c.cout);
    const float* mu = t.get(c.bnname + ".running_mean", c.cout);
    const float* var = t.get(c.bnname + ".running_var", c.cout);
    if (!g || !bb || !mu || !var) return false;
    for (int o = 0; o < c.cout; ++o) {
      // same arithmetic as torch's CPU BN inference: alpha = gamma / sqrt(var + eps)
      alpha[o] = (1.f / std::sqrt(var[o] + 1e-5f)) * g[o];
      beta[o] = bb[o] - mu[o] * alpha[o];
    }
  } else if (!c.bnname.empty()) {
    const float* bias = t.get(c.bnname, c.cout);
    if (!bias) return false;
    for (int o = 0; o < c.cout; ++o) beta[o] = bias[o];
  }
  // bf16 multi-tap convs with Cin > 64: K chunk-major, (cin / 64, kh, kw, cin % 64), so that a
  // conv's K walk visits all taps of one 64-channel slice of the input before the next slice.
  // f32 multi-tap convs with Cin >= 128 (the implicit GEMM's; stage 1 takes the row kernel) can
  // take (cin / C, kh, kw, cin % C) too (EOSV_F32_KCM = C, profiling build): in tap-major order a
  // pixel's next tap comes Cin / 16 K-steps later, when the XCD's 64 workgroups have staged ~8 MB
  // and L2 (4 MB) has turned over, so the tap re-reads come from beyond L2.  r04 (PMC, R18 f32):
  // C = 32 cuts the 256x128 tiles' FETCH_SIZE 3.0x and the fused-downsample ones' 5x, C = 64 2x,
  // C = 128 1.1x, but the release kernels ran 2-4 % slower with C = 32 (profiling-build A/B:
  // 0.3-0.5 %, C = 64 / 128 0.1-0.3 %): these convs are MFMA-bound with the DMA hidden.  r05
  // release A/B (profiles/r05l_ab_f32_kcm64.txt, three interleaved rounds): C = 64 costs the R18
  // f32 line 0.2-0.3 % (2,322-2,325 -> 2,315-2,320 clips/s) and takes its conv traffic from 2.21x to
  // 1.39x the algorithmic bytes (6.82 -> 4.30 GB per launch): the default since r05, the re-reads
  // beyond L2 being bytes every other tenant of the HBM pays for too
  static const int f32kcm = env_switch("EOSV_F32_KCM", EOSV_F32_KCM_DEF);  // f32 channel chunk (32, 64, 128); 0 = tap-major (A/B switch)
  c.kcmc = bf16 ? 64 : f32kcm;
  c.kcm = !c.stem && c.kcmc > 0 && c.cinp % c.kcmc == 0 && c.kh * c.kw > 1 && c.kwp == c.kw &&
          (bf16 ? c.cinp > 64 : c.cinp >= 128);
  wf.assign((size_t)c.cout * c.K, 0.f);
  if (split && c.cinp != 3 * c.cin) return set_error("fold_conv: split layout needs 3 * cin channels"), false;
  auto kidx = [&](int i, int y, int x) {
    return c.kcm ? ((size_t)(i / c.kcmc) * c.kh * c.kw + y * c.kw + x) * c.kcmc + i % c.kcmc
                 : ((size_t)y * c.kwp + x) * c.cinp + i;
  };
  for (int o = 0; o < c.cout; ++o)
    for (int i = 0; i < c.cin; ++i)
      for (int y = 0; y < c.kh; ++y)
        for (int x = 0; x < c.kw; ++x) {
          const float v = w[(((size_t)o * c.cin + i) * c.kh + y) * c.kw + x] * alpha[o];
          float* row = wf.data() + (size_t)o * c.K;
          if (!split) {
            row[kidx(i, y, x)] = v;
          } else {
            const float hi = bf_round_host(v);
            row[kidx(i, y, x)] = hi;
            row[kidx(c.cin + i, y, x)] = hi;
            row[kidx(2 * c.cin + i, y, x)] = bf_round_host(v - hi);
          }
        }
  return true;
}

// upload [cout][K (+ ds K)] weights + [cout] bias; with `ds`, the downsample's folded 1x1
// weights are appended as K columns [c.K, c.K + ds.cin) and its shift is added to the bias
static int upload_conv(eosv_handle* h, Conv& c, const Tensors& t, bool bf16, bool has_bn, Conv* ds = nullptr,
                       bool split = false) {
  std::vector<float> wf, beta;
  if (!fold_conv(c, t, bf16, has_bn, wf, beta, split)) return EOSV_ERR_ARG;
  if (ds) {
    std::vector<float> wd, bd;
    if (!fold_conv(*ds, t, bf16, true, wd, bd, split)) return EOSV_ERR_ARG;
    if (ds->cout != c.cout || ds->kh != 1 || ds->K != c.kds) return set_error("fused downsample shape"), EOSV_ERR_ARG;
    const int Kt = c.K + c.kds;
    std::vector<float> wc((size_t)c.cout * Kt);
    for (int o = 0; o < c.cout; ++o) {
      std::copy(wf.begin() + (size_t)o * c.K, wf.begin() + (size_t)(o + 1) * c.K, wc.begin() + (size_t)o * Kt);
      std::copy(wd.begin() + (size_t)o * c.kds, wd.begin() + (size_t)(o + 1) * c.kds, wc.begin() + (size_t)o * Kt + c.K);
      beta[o] += bd[o];
    }
    wf.swap(wc);
  }
  int rc;
  if (bf16) {
    std::vector<unsigned short> wb(wf.size());
    for (size_t i = 0; i < wf.size(); ++i) wb[i] = f2bf_host(wf[i]);
    if ((rc = upload_bytes(h, &c.w, &c.wbytes, wb.data(), wb.size() * 2))) return rc;
  } else {
    if ((rc = upload_bytes(h, &c.w, &c.wbytes, wf.data(), wf.size() * 4))) return rc;
  }
  size_t bcap = c.b ? (size_t)c.cout * 4 : 0;
  return upload_bytes(h, (void**)&c.b, &bcap, beta.data(), (size_t)c.cout * 4);
}

static hipEvent_t prof_event(eosv_handle* h) {
  if (h->pool_used == h->pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    h->pool.push_back(e);
  }
  return h->pool[h->pool_used++];
}

// planning: a launch of `flops` algorithmic FLOPs on `li`'s grid costs flops / wave efficiency,
// the efficiency being blocks / (slots x rounds): a grid of 4.67 waves runs 5
static void add_plan_cost(eosv_handle* h, const LaunchInfo& li, double flops) {
  if (li.blocks <= 0 || li.slots <= 0) return;
  const double rounds = (double)((li.blocks + li.slots - 1) / li.slots);
  h->plan_cost += flops * rounds * (double)li.slots / (double)li.blocks;
}

#ifdef EOSV_PROFILING
// Poisoning (profiling build, EOSV_POISON bits, read per call): 1 fills the activation buffers with
// 0xff bytes (NaN in bf16 and f32) at every chunk's start, 2 fills every CU's LDS with 0xff before
// every launch, 4 synchronises the stream before (and after) that.  A kernel whose valid outputs depend on an activation row or an LDS word that it
// (or the layer before) did not write then yields NaN or different features, in the first run:
// tools/poison_check.py compares poisoned and plain forwards bit for bit.
__global__ __launch_bounds__(256) void lds_poison_kernel() {
  __shared__ unsigned lds[160 * 1024 / 4];
  volatile unsigned* p = lds;
  for (int i = threadIdx.x; i < 160 * 1024 / 4; i += 256) p[i] = 0xffffffffu;
}
static int poison_mode() { return env_switch("EOSV_POISON", 0); }
static void poison_lds(hipStream_t s) {
  if (poison_mode() & 4) (void)hipStreamSynchronize(s);  // 4: the previous launch has drained
  if (poison_mode() & 2) hipLaunchKernelGGL(lds_poison_kernel, dim3(4 * device_cu_count()), dim3(256), 0, s);
  if (poison_mode() & 4) (void)hipStreamSynchronize(s);
}
static int poison_bufs(eosv_handle* h, hipStream_t s) {
  if (!(poison_mode() & 1)) return EOSV_OK;
  const size_t elt = act_bytes(h);
  for (void* p : h->buf) EOSV_HIP_CHECK(hipMemsetAsync(p, 0xff, (size_t)h->d.max_frames * h->act_elems * elt, s));
  for (void* p : h->sbuf)
    if (p) EOSV_HIP_CHECK(hipMemsetAsync(p, 0xff, (size_t)h->sub_frames * h->act_elems * elt, s));
  return EOSV_OK;
}
#else
static void poison_lds(hipStream_t) {}
static int poison_bufs(eosv_handle*, hipStream_t) { return EOSV_OK; }
#endif

static int run_conv(eosv_handle* h, const Conv& c, const void* x, int N, int H, int W, const void* res,
                    void* y, bool relu, bool bf16, hipStream_t s, const void* x2 = nullptr, int H2 = 0,
                    int W2 = 0, int stride2 = 1) {
  ConvArgs a{};
  a.x = x;
  a.w = c.w;
  a.bias = c.b;
  a.res = res;
  a.y = y;
  a.N = N;
  a.H = H;
  a.W = W;
  a.Cin = c.cinp;
  a.Ho = conv_out(H, c.kh, c.stride, c.pad);
  a.Wo = conv_out(W, c.kw, c.stride, c.pad);
  a.Cout = c.cout;
  a.KH = c.kh;
  a.KW = c.kw;
  a.KWp = c.kwp;
  a.stride = c.stride;
  a.pad = c.pad;
  a.K = c.K + (x2 ? c.kds : 0);
  a.relu = relu ? 1 : 0;
  if (x2) {  // fused downsample: K columns [c.K, c.K + kds) read x2 (1x1, stride2)
    a.x2 = x2;
    a.H2 = H2;
    a.W2 = W2;
    a.Cin2 = c.kds;
    a.stride2 = stride2;
    a.K1 = c.K;
  }
  a.zero = h->zero;
  static const int xcd = env_switch("EOSV_XCD", 1);  // 0 = plain blockIdx order (A/B switch)
  a.xcd = xcd;
  a.kcm = c.kcm ? (bf16 ? 1 : c.kcmc) : 0;  // bf16 kernels: a flag (64-channel chunks); f32: the chunk
  a.split = (bf16 && x3(h)) ? 1 : 0;
  a.xs = a.split ? 2 * c.cin : c.cinp;  // physical pixel strides (the split layout stores hi, lo)
  a.x2s = x2 ? (a.split ? 2 * (c.kds / 3) : c.kds) : 0;
  // algorithmic FLOPs: logical channels (the split layout's 3x virtual K is not counted)
  const double flops = 2.0 * N * a.Ho * a.Wo * c.cout *
                       ((double)c.kh * c.kw * c.cin + (x2 ? c.kds / (a.split ? 3 : 1) : 0));
  if (h->planning) {
    LaunchInfo li{};
    a.plan = &li;
    const int prc = bf16 ? launch_conv_bf16(a, s) : launch_conv_f32(a, s);
    if (prc == EOSV_OK) add_plan_cost(h, li, flops);
    return prc;
  }
  poison_lds(s);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (h->prof) {
    e0 = prof_event(h);
    e1 = prof_event(h);
    if (!e0 || !e1) return set_error("profiling: hipEventCreate failed"), EOSV_ERR_HIP;
    EOSV_HIP_CHECK(hipEventRecord(e0, s));
  }
  const int rc = bf16 ? launch_conv_bf16(a, s) : launch_conv_f32(a, s);
  if (h->prof && rc == EOSV_OK) {
    EOSV_HIP_CHECK(hipEventRecord(e1, s));
    h->recs.push_back({c.id, e0, e1, flops});
  }
  return rc;
}

// bf16 bottleneck stage 1: block b's conv3 fused with block b+1's conv1 (pair1x1_bf16.hip) when
// the shapes allow it.  EOSV_PAIR=0 (profiling build): unfused.
static bool pair_enabled() {
  static const bool v = env_switch("EOSV_PAIR", 1) != 0;
  return v;
}

// ... and in the wider stages 2-3 (pairw_bf16.hip).  EOSV_PAIRW=0 (profiling build): unfused there.
static bool pairw_enabled() {
  static const bool v = env_switch("EOSV_PAIRW", 1) != 0;
  return v;
}

// elements every activation buffer holds (the sub-chunk scratch, when on, is the smaller one)
static long long act_buffer_elems(const eosv_handle* h) {
  const long long f = h->sub_frames > 0 ? std::min(h->sub_frames, h->d.max_frames) : h->d.max_frames;
  return f * (long long)h->act_elems;
}

static bool pair_ok(const eosv_handle* h, const Block& b, const Block* nb, long long M) {
  if (!pair_enabled() || !conv_bf(h) || x3(h) || !b.bottleneck || !nb || !nb->bottleneck) return false;
  const Conv &c3 = b.c3, &n1 = nb->c1;
  if (c3.kh != 1 || n1.kh != 1 || n1.stride != 1 || n1.cin != c3.cout) return false;
  if (c3.cin != 64) {
    // the stage's block 0: conv3 + the folded stride-2 downsample (a fused-ds block whose 3x3 has
    // stride 2), or a plain residual block
    const bool ds = b.has_ds && b.fuse_ds && b.ds.stride == 2 && b.c2.stride == 2;
    if (!pairw_enabled() || (b.has_ds && !ds)) return false;
    return pairw_bf16_ok(c3.cin, c3.cout, n1.cout, ds ? c3.kds : 0, M, act_buffer_elems(h));
  }
  if (b.c2.stride != 1 || (b.has_ds && !(b.fuse_ds && b.ds.stride == 1))) return false;
  return pair1x1_bf16_ok(c3.cin, c3.cout, n1.cout, b.has_ds ? c3.kds : 0, M);
}

// conv3 of `b` (+ residual `res` or the folded downsample reading x2) -> y, and the next block's
// conv1 on y -> z, in one launch; profiled as conv3's layer with both convs' FLOPs
static int run_pair(eosv_handle* h, const Block& b, const Block& nb, const void* x, const void* x2, const void* res,
                    void* y, void* z, long long M, hipStream_t s, int ho = 0, int wo = 0, int hin = 0, int win = 0) {
  Pair1x1Args p{};
  p.x = x;
  p.x2 = x2;
  p.res = res;
  p.w3 = b.c3.w;
  p.b3 = b.c3.b;
  p.w1 = nb.c1.w;
  p.b1 = nb.c1.b;
  p.y = y;
  p.z = z;
  p.M = M;
  p.c1 = nb.c1.cout;
  p.cds = x2 ? b.c3.kds : 0;
  p.cmid = b.c3.cin;
  p.cexp = b.c3.cout;
  p.Ho = ho;
  p.Wo = wo;
  p.H2 = hin;
  p.W2 = win;
  p.cap_elems = act_buffer_elems(h);
  const bool wide = p.cmid != 64;
  const double flops = 2.0 * M * ((double)b.c3.cout * (b.c3.cin + p.cds) + (double)nb.c1.cout * nb.c1.cin);
  if (h->planning) {
    LaunchInfo li{};
    p.plan = &li;
    const int prc = wide ? launch_pairw_bf16(p, s) : launch_pair1x1_bf16(p, s);
    if (prc == EOSV_OK) add_plan_cost(h, li, flops);
    return prc;
  }
  poison_lds(s);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (h->prof) {
    e0 = prof_event(h);
    e1 = prof_event(h);
    if (!e0 || !e1) return set_error("profiling: hipEventCreate failed"), EOSV_ERR_HIP;
    EOSV_HIP_CHECK(hipEventRecord(e0, s));
  }
#ifdef EOSV_PROFILING
  // EOSV_POISON bit 8: every pair runs a second time out of place (residual copied first) into
  // scratch, and both outputs are compared bytewise on the host (stderr): does the pair's own
  // output change between two runs on the same inputs inside the backbone?
  static void* scr[3] = {nullptr, nullptr, nullptr};
  static size_t scr_b = 0;  // bytes each scratch buffer holds (grown for a larger handle / pair)
  const bool selfcheck = (poison_mode() & 8) != 0;
  const size_t cap_b = (size_t)p.cap_elems * 2;
  if (selfcheck) {
    if (cap_b > scr_b) {
      for (auto& q : scr) {
        if (q) EOSV_HIP_CHECK(hipFree(q));
        q = nullptr;
        EOSV_HIP_CHECK(hipMalloc(&q, cap_b));
      }
      scr_b = cap_b;
    }
    if (res) EOSV_HIP_CHECK(hipMemcpyAsync(scr[0], res, cap_b, hipMemcpyDeviceToDevice, s));
  }
#endif
  const int rc = wide ? launch_pairw_bf16(p, s) : launch_pair1x1_bf16(p, s);
  if (h->prof && rc == EOSV_OK) {
    EOSV_HIP_CHECK(hipEventRecord(e1, s));
    h->recs.push_back({b.c3.id, e0, e1, flops});
  }
#ifdef EOSV_PROFILING
  if (selfcheck && rc == EOSV_OK) {
    Pair1x1Args q = p;
    if (res) q.res = scr[0];
    q.y = scr[1];
    q.z = scr[2];
    const int rc2 = wide ? launch_pairw_bf16(q, s) : launch_pair1x1_bf16(q, s);
    EOSV_HIP_CHECK(hipStreamSynchronize(s));
    const size_t ny = (size_t)M * p.cexp, nz = (size_t)M * p.c1;
    std::vector<unsigned short> a(ny), c(ny);
    long long dy = 0, dz = 0, fy = -1, fz = -1;
    EOSV_HIP_CHECK(hipMemcpy(a.data(), y, ny * 2, hipMemcpyDeviceToHost));
    EOSV_HIP_CHECK(hipMemcpy(c.data(), scr[1], ny * 2, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < ny; ++i)
      if (a[i] != c[i] && dy++ == 0) fy = (long long)i;
    a.resize(nz);
    c.resize(nz);
    EOSV_HIP_CHECK(hipMemcpy(a.data(), z, nz * 2, hipMemcpyDeviceToHost));
    EOSV_HIP_CHECK(hipMemcpy(c.data(), scr[2], nz * 2, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < nz; ++i)
      if (a[i] != c[i] && dz++ == 0) fz = (long long)i;
    fprintf(stderr, "pair selfcheck layer %d %s cmid %d c1 %d cds %d M %lld rc %d/%d: y differs %lld (first px %lld ch %lld), z %lld (first px %lld ch %lld)\n",
            b.c3.id, wide ? "pairw" : "pair1x1", p.cmid, p.c1, p.cds, M, rc, rc2, dy, fy < 0 ? -1 : fy / p.cexp,
            fy < 0 ? -1 : fy % p.cexp, dz, fz < 0 ? -1 : fz / p.c1, fz < 0 ? -1 : fz % p.c1);
  }
#endif
  return rc;
}

// bf16 stage-1 bottleneck blocks as one launch each (bneck_bf16.hip, r06): conv1 -> conv2 -> conv3
// with the 64-channel maps kept on the CU.  EOSV_BNECK=0 (profiling build): the r05 path.
static bool bneck_enabled() {
  static const bool v = env_switch("EOSV_BNECK", 1) != 0;
  return v;
}

static bool bneck_eligible(const eosv_handle* h, const Block& b, int hh, int ww) {
  if (!bneck_enabled() || !conv_bf(h) || x3(h) || !b.bottleneck) return false;
  // profiling-build diagnosis switch: EOSV_BNECK=2 fuses only the 256-channel-input blocks, 3 only
  // block 0 (the 64-channel input with the folded downsample)
  static const int mode = env_switch("EOSV_BNECK", 1);
  if ((mode == 2 && b.c1.cin != 256) || (mode == 3 && b.c1.cin != 64)) return false;
  const Conv &c1 = b.c1, &c2 = b.c2, &c3 = b.c3;
  if (c1.kh != 1 || c1.stride != 1 || c1.cout != 64 || c2.kh != 3 || c2.stride != 1 || c2.cin != 64 ||
      c2.cout != 64 || c2.kcm || c3.kh != 1 || c3.cin != 64 || c3.cout != 256)
    return false;
  if (b.has_ds ? !(b.fuse_ds && b.ds.stride == 1 && c1.cin == 64 && c3.kds == 64) : c1.cin != 256) return false;
  return bneck_bf16_ok(c1.cin, ww, hh, 0);
}

// block bi is its stage's last block (stage_end holds the cumulative block counts)
static bool last_in_stage(const eosv_handle* h, size_t bi) {
  for (size_t li = 0; li < 4; ++li)
    if (bi + 1 == h->stage_end[li]) return true;
  return false;
}

// block b as one bneck_bf16 launch: x -> y, and with nb the next block's conv1 on y -> z
static int run_bneck(eosv_handle* h, const Block& b, const Block* nb, const void* x, void* y, void* z, int B, int hh,
                     int ww, hipStream_t s) {
  BneckArgs a{};
  a.x = x;
  a.w1 = b.c1.w;
  a.b1 = b.c1.b;
  a.w2 = b.c2.w;
  a.b2 = b.c2.b;
  a.w3 = b.c3.w;
  a.b3 = b.c3.b;
  a.wn = nb ? nb->c1.w : nullptr;
  a.bn = nb ? nb->c1.b : nullptr;
  a.y = y;
  a.z = z;
  a.N = B;
  a.H = hh;
  a.W = ww;
  a.cin = b.c1.cin;
  const double M = (double)B * hh * ww;
  const double flops = 2.0 * M * (64.0 * b.c1.cin + 9.0 * 64 * 64 + 256.0 * (64 + b.c3.kds) + (nb ? 64.0 * 256 : 0.0));
  if (h->planning) {
    LaunchInfo li{};
    a.plan = &li;
    const int prc = launch_bneck_bf16(a, s);
    if (prc == EOSV_OK) add_plan_cost(h, li, flops);
    return prc;
  }
  poison_lds(s);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (h->prof) {
    e0 = prof_event(h);
    e1 = prof_event(h);
    if (!e0 || !e1) return set_error("profiling: hipEventCreate failed"), EOSV_ERR_HIP;
    EOSV_HIP_CHECK(hipEventRecord(e0, s));
  }
  const int rc = launch_bneck_bf16(a, s);
  if (h->prof && rc == EOSV_OK) {
    EOSV_HIP_CHECK(hipEventRecord(e1, s));
    h->recs.push_back({b.c1.id, e0, e1, flops});  // profiled as the block's conv1 layer, with every conv's FLOPs
  }
  return rc;
}

// the stage's last bf16 stage-1 block, whose conv1 output a bneck_bf16 NEXT launch wrote, with the
// next stage's conv1 (1x1 256 -> 128): bneck_tail_bf16 (r06).  Default only at 64x64 maps (R101 at
// 256: stage 1 4.54 -> 4.47 ms per chunk); at 56x56 the two-launch path (conv_rows_bf16 +
// pair1x1r_bf16) is faster (R50 at the C2 shape: 10.00 vs 10.21-10.28 ms, 6,147-6,161 vs
// 6,090-6,110 clips/s; tools/sessions/gpu_r06p.sh).  EOSV_BNECK_TAIL (profiling build): 0 never,
// 1 always, 2 only at W 64.
static bool bneck_tail_eligible(const eosv_handle* h, const Block& b, const Block& nb, int hh, int ww) {
  static const int mode = env_switch("EOSV_BNECK_TAIL", 2);
  if (!mode || (mode == 2 && ww != 64)) return false;
  if (!bneck_enabled() || !conv_bf(h) || x3(h) || !b.bottleneck || b.has_ds || !nb.bottleneck) return false;
  const Conv &c2 = b.c2, &c3 = b.c3, &n1 = nb.c1;
  return c2.kh == 3 && c2.stride == 1 && c2.cin == 64 && c2.cout == 64 && !c2.kcm && c3.kh == 1 && c3.cin == 64 &&
         c3.cout == 256 && b.c1.cout == 64 && n1.kh == 1 && n1.stride == 1 && n1.cin == 256 && n1.cout == 128 &&
         bneck_tail_bf16_ok(ww, hh);
}

static int run_bneck_tail(eosv_handle* h, const Block& b, const Block& nb, const void* t1, const void* x, void* y,
                          void* z, int B, int hh, int ww, hipStream_t s) {
  BneckArgs a{};
  a.x = t1;
  a.res = x;
  a.w2 = b.c2.w;
  a.b2 = b.c2.b;
  a.w3 = b.c3.w;
  a.b3 = b.c3.b;
  a.wn = nb.c1.w;
  a.bn = nb.c1.b;
  a.y = y;
  a.z = z;
  a.N = B;
  a.H = hh;
  a.W = ww;
  a.cin = 64;
  const double M = (double)B * hh * ww;
  const double flops = 2.0 * M * (9.0 * 64 * 64 + 256.0 * 64 + 128.0 * 256);
  if (h->planning) {
    LaunchInfo li{};
    a.plan = &li;
    const int prc = launch_bneck_tail_bf16(a, s);
    if (prc == EOSV_OK) add_plan_cost(h, li, flops);
    return prc;
  }
  poison_lds(s);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (h->prof) {
    e0 = prof_event(h);
    e1 = prof_event(h);
    if (!e0 || !e1) return set_error("profiling: hipEventCreate failed"), EOSV_ERR_HIP;
    EOSV_HIP_CHECK(hipEventRecord(e0, s));
  }
  const int rc = launch_bneck_tail_bf16(a, s);
  if (h->prof && rc == EOSV_OK) {
    EOSV_HIP_CHECK(hipEventRecord(e1, s));
    h->recs.push_back({b.c2.id, e0, e1, flops});  // profiled as the block's conv2 layer, with conv2, conv3 and the next conv1
  }
  return rc;
}

// bf16 ResNet-18 stage-1 basic blocks as one launch each (bblock_bf16.hip, r06): conv1 -> conv2 + x
// with conv1's output kept on the CU.  EOSV_BBLOCK=0 (profiling build): conv_rows_bf16 twice.
static bool bblock_eligible(const eosv_handle* h, const Block& b, int hh, int ww) {
#ifndef EOSV_BBLOCK_DEF
#define EOSV_BBLOCK_DEF 1  // release A/B: tools/build_variant.sh nobb -DEOSV_BBLOCK_DEF=0
#endif
  static const bool on = env_switch("EOSV_BBLOCK", EOSV_BBLOCK_DEF) != 0;
  if (!on || !conv_bf(h) || x3(h) || b.bottleneck || b.has_ds) return false;
  const Conv &c1 = b.c1, &c2 = b.c2;
  return c1.kh == 3 && c1.stride == 1 && c1.cin == 64 && c1.cout == 64 && !c1.kcm && c2.kh == 3 && c2.stride == 1 &&
         c2.cin == 64 && c2.cout == 64 && !c2.kcm && bblock_bf16_ok(ww, hh);
}

static int run_bblock(eosv_handle* h, const Block& b, const void* x, void* y, int B, int hh, int ww, hipStream_t s) {
  BneckArgs a{};
  a.x = x;
  a.w1 = b.c1.w;
  a.b1 = b.c1.b;
  a.w2 = b.c2.w;
  a.b2 = b.c2.b;
  a.y = y;
  a.N = B;
  a.H = hh;
  a.W = ww;
  a.cin = 64;
  const double flops = 2.0 * B * hh * ww * 2.0 * 9 * 64 * 64;
  if (h->planning) {
    LaunchInfo li{};
    a.plan = &li;
    const int prc = launch_bblock_bf16(a, s);
    if (prc == EOSV_OK) add_plan_cost(h, li, flops);
    return prc;
  }
  poison_lds(s);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (h->prof) {
    e0 = prof_event(h);
    e1 = prof_event(h);
    if (!e0 || !e1) return set_error("profiling: hipEventCreate failed"), EOSV_ERR_HIP;
    EOSV_HIP_CHECK(hipEventRecord(e0, s));
  }
  const int rc = launch_bblock_bf16(a, s);
  if (h->prof && rc == EOSV_OK) {
    EOSV_HIP_CHECK(hipEventRecord(e1, s));
    h->recs.push_back({b.c1.id, e0, e1, flops});  // profiled as the block's conv1 layer, with both convs' FLOPs
  }
  return rc;
}

// Residual blocks [b0, b1) on x (B frames, hh x ww) using the 4-buffer set `bufs`.  The
// output of each block lands in place of its residual buffer; when `dst` is given, the last
// block writes there instead (its residual still comes from `bufs`).
static int run_blocks(eosv_handle* h, size_t b0, size_t b1, void* x, void* const* bufs, int B, int& hh,
                      int& ww, void* dst, void** xout, bool bf, hipStream_t s) {
  int rc;
  bool c1_done = false;    // this block's conv1 output is already in c1buf (fused into the previous launch)
  void* c1buf = nullptr;
  for (size_t bi = b0; bi < b1; ++bi) {
    const Block& b = h->blocks[bi];
    void* fr[3];
    int nf = 0;
    for (int k = 0; k < 4; ++k)
      if (bufs[k] != x) fr[nf++] = bufs[k];
    const int st = b.bottleneck ? b.c2.stride : b.c1.stride;  // torchvision: stride on the 3x3
    const int ho = conv_out(hh, 3, st, 1), wo = conv_out(ww, 3, st, 1);
    void* r = x;  // residual: the block input, or the downsample's output
    if (b.has_ds && !b.fuse_ds) {
      r = fr[2];
      if ((rc = run_conv(h, b.ds, x, B, hh, ww, nullptr, r, false, bf, s))) return rc;
    }
    void* y = (dst && bi + 1 == b1) ? dst : (b.has_ds ? fr[2] : r);
    // fused downsample: the last conv reads x (strided) as extra K columns, no residual
    const void* res = b.fuse_ds ? nullptr : r;
    const void* x2 = b.fuse_ds ? x : nullptr;
    const int s2 = b.has_ds ? b.ds.stride : 1;
    // the first buffer that is not `a` (and not `c`): where a next block's conv1 output goes
    auto first_not = [&](const void* a, const void* c, const void* d = nullptr) {
      for (int k = 0; k < 4; ++k)
        if (bufs[k] != a && bufs[k] != c && bufs[k] != d) return bufs[k];
      return (void*)nullptr;
    };
    const Block* nb = bi + 1 < b1 ? &h->blocks[bi + 1] : nullptr;
    if (!b.bottleneck && bblock_eligible(h, b, hh, ww)) {
      if ((rc = run_bblock(h, b, x, y, B, hh, ww, s))) return rc;  // y = x in place, or dst
    } else if (!b.bottleneck) {
      if ((rc = run_conv(h, b.c1, x, B, hh, ww, nullptr, fr[0], true, bf, s))) return rc;
      if ((rc = run_conv(h, b.c2, fr[0], B, ho, wo, res, y, true, bf, s, x2, hh, ww, s2))) return rc;
    } else if (!c1_done && nb && !last_in_stage(h, bi) && bneck_eligible(h, b, hh, ww)) {
      // the whole block in one launch (not the stage's last block: that one takes the tail kernel
      // or conv2 + the pair with the next stage's conv1); when the next block is that last one,
      // its conv1 too (into the first buffer that is not y: x itself only for a downsample block,
      // whose 64-channel input pixels are each read before their z is written)
      const bool next = last_in_stage(h, bi + 1) && nb->bottleneck && nb->c1.kh == 1 && nb->c1.cin == 256 &&
                        nb->c1.cout == 64 && nb->c1.stride == 1;
      void* z = next ? first_not(y, nullptr) : nullptr;
      if ((rc = run_bneck(h, b, next ? nb : nullptr, x, y, z, B, hh, ww, s))) return rc;
      c1_done = next;
      c1buf = z;
    } else if (c1_done && nb && last_in_stage(h, bi) && y == x && bneck_tail_eligible(h, b, *nb, hh, ww)) {
      // the stage's last block from its conv1 output: conv2 -> conv3 (+ x) -> y = x in place, and the
      // next stage's conv1 -> a buffer that is neither y nor the conv1 output being read
      void* z = first_not(y, c1buf);
      if ((rc = run_bneck_tail(h, b, *nb, c1buf, x, y, z, B, hh, ww, s))) return rc;
      c1buf = z;  // c1_done stays true
    } else {
      void* t1 = c1_done ? c1buf : fr[0];  // conv1 output
      if (!c1_done && (rc = run_conv(h, b.c1, x, B, hh, ww, nullptr, t1, true, bf, s))) return rc;
      void* t2 = t1 == fr[0] ? fr[1] : fr[0];  // conv2 output: a buffer that is neither x nor t1
      if ((rc = run_conv(h, b.c2, t1, B, hh, ww, nullptr, t2, true, bf, s))) return rc;
      // the next block's conv1 lands in the first buffer that the pair does not read (x, t2) or write
      // (y); t1 was consumed by conv2.  (Until r06: the first buffer that is not y, so with conv1
      // outputs placed by the fused stage-1 launches the stage-2 entry pair found x there and fell
      // back to two launches.)
      void* z = first_not(y, x, t2);
      const long long M = (long long)B * ho * wo;
      c1_done = z && pair_ok(h, b, nb, M) && y != dst && z != x && z != t2;
      if (c1_done) {
        if ((rc = run_pair(h, b, *nb, t2, x2, res, y, z, M, s, ho, wo, hh, ww))) return rc;
        c1buf = z;
      } else if ((rc = run_conv(h, b.c3, t2, B, ho, wo, res, y, true, bf, s, x2, hh, ww, s2))) {
        return rc;
      }
    }
    x = y;
    hh = ho;
    ww = wo;
  }
  *xout = x;
  return EOSV_OK;
}

static bool stem_pool_fused(bool bf) {
  static const bool vb = env_switch("EOSV_BF16_STEMPOOL", 1) != 0;  // 0 = separate stem conv + maxpool (A/B switch)
  static const bool vf = env_switch("EOSV_F32_STEMPOOL", 1) != 0;  // 0 = separate stem conv + maxpool (A/B switch)
  return bf ? vb : vf;
}

// Whether the stem path launches pack_rgb_pad (run_stem's decision): only then does eosv_create
// size the padded-RGB pack buffer for max_frames (2.6 GB f32 / 1.3 GB bf16 at 4096 frames of 224²)
static bool stem_needs_pack(const eosv_handle* h) {
  const int H = h->d.height, W = h->d.width;
  static const bool direct = env_switch("EOSV_STEM_DIRECT", 1) != 0;
  const bool sbf = stem_bf(h);
  const bool fused = stem_pool_fused(sbf) && (sbf ? stem_pool_bf16_ok(H, W, direct) : stem_pool_f32_ok(H, W));
  return !(fused && direct && (sbf || stem_pool_f32_direct_ok(H, W)));
}

// stem -> maxpool for frames [0, B) of `frames`, output into bufs[1]
static int run_stem(eosv_handle* h, const float* frames, int B, void* const* bufs, bool bf, hipStream_t s) {
  const int H = h->d.height, W = h->d.width;
  int rc;
  static const bool direct = env_switch("EOSV_STEM_DIRECT", 1) != 0;  // 0 = pack kernel + LDS-DMA rows (A/B switch)
  static const bool x3_split_stem = env_switch("EOSV_X3_STEM", 1) != 0;  // 0 = exact-f32 MFMA stem for EOSV_F32X3 (A/B switch)
  const bool sbf = stem_bf(h);  // EOSV_F32X3: split-bf16 (or exact-f32) stem with split output, bf16 blocks
  // EOSV_F32X3: the split-bf16 fused stem reads the f32 frames directly
  const bool x3stem = x3(h) && direct && x3_split_stem && h->stem_x3.w && stem_pool_x3_ok(H, W);
  const bool fused = stem_pool_fused(sbf) && (sbf ? stem_pool_bf16_ok(H, W, direct) : stem_pool_f32_ok(H, W));
  if (x3(h) && !fused && !x3stem) return set_error("f32x3: needs the fused stem + maxpool (frame width)"), EOSV_ERR_UNSUPPORTED;
  if (!h->planning) poison_lds(s);
  // the bf16 and f32 fused stems read the f32 NCHW frames themselves (no pack pass)
  const bool direct_bf = fused && sbf && direct;
  const bool direct_f32 = fused && !sbf && direct && stem_pool_f32_direct_ok(H, W);
  // (direct_bf || direct_f32) == !stem_needs_pack(h): otherwise the pack buffer is a stub
  if (!direct_bf && !direct_f32 && !x3stem && !h->planning &&
      (rc = launch_pack_rgb_pad(frames, B, H, W, h->stem.pad, h->pack, sbf, s)))
    return rc;
  if (h->planning && (fused || x3stem)) {
    LaunchInfo li{};
    if ((rc = x3stem ? launch_stem_pool_x3(frames, B, H, W, h->stem_x3.w, h->stem_x3.b, bufs[1], s, &li)
              : sbf  ? launch_stem_pool_bf16(direct_bf ? nullptr : h->pack, B, H, W, h->stem.w, h->stem.b, bufs[1], s,
                                             direct_bf ? frames : nullptr, &li)
                     : launch_stem_pool_f32(direct_f32 ? nullptr : h->pack, B, H, W, h->stem.w, h->stem.b, bufs[1], s,
                                            x3(h), &li, direct_f32 ? frames : nullptr)))
      return rc;
    add_plan_cost(h, li, 2.0 * B * h->hs * h->ws * 64 * 147);
  } else if (fused || x3stem) {
    // fused stem conv + ReLU + maxpool (profiled as the stem layer)
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (h->prof) {
      e0 = prof_event(h);
      e1 = prof_event(h);
      if (!e0 || !e1) return set_error("profiling: hipEventCreate failed"), EOSV_ERR_HIP;
      EOSV_HIP_CHECK(hipEventRecord(e0, s));
    }
    if ((rc = x3stem ? launch_stem_pool_x3(frames, B, H, W, h->stem_x3.w, h->stem_x3.b, bufs[1], s)
              : sbf  ? launch_stem_pool_bf16(direct_bf ? nullptr : h->pack, B, H, W, h->stem.w, h->stem.b, bufs[1], s,
                                             direct_bf ? frames : nullptr)
                     : launch_stem_pool_f32(direct_f32 ? nullptr : h->pack, B, H, W, h->stem.w, h->stem.b, bufs[1], s,
                                            x3(h), nullptr, direct_f32 ? frames : nullptr)))
      return rc;
    if (h->prof) {
      EOSV_HIP_CHECK(hipEventRecord(e1, s));
      h->recs.push_back({h->stem.id, e0, e1, 2.0 * B * h->hs * h->ws * 64 * 147});
    }
  } else {
    if ((rc = run_conv(h, h->stem, h->pack, B, H, W, nullptr, bufs[0], true, bf, s))) return rc;
    if (!h->planning && (rc = launch_maxpool3x3s2(bufs[0], B, h->hs, h->ws, 64, bufs[1], h->hp, h->wp, bf, s)))
      return rc;
  }
  return EOSV_OK;
}

// stem -> maxpool -> stage-0 blocks for frames [0, B) of `frames`, output into `dst`
static int run_front(eosv_handle* h, const float* frames, int B, void* const* bufs, void* dst, void** xout,
                     bool bf, hipStream_t s) {
  int rc;
  if ((rc = run_stem(h, frames, B, bufs, bf, s))) return rc;
  int hh = h->hp, ww = h->wp;
  return run_blocks(h, 0, h->n_front, bufs[1], bufs, B, hh, ww, dst, xout, bf, s);
}

static int forward_chunk(eosv_handle* h, const float* frames, int B, float* feat, hipStream_t s) {
  const bool bf = conv_bf(h);
  const size_t elt = act_bytes(h);
  int rc;
  void* x;
  int hh = h->hp, ww = h->wp;
  if (!h->planning && (rc = poison_bufs(h, s))) return rc;
  if (h->sub_frames > 0 && h->sub_frames < B) {
    // Front stages (stem, maxpool, layer1: the largest activations) run on sub-chunks whose
    // working set stays in the 256 MiB Infinity Cache; each sub-chunk's layer1 output lands
    // in the full-size buffer buf[1], from which layer2..4 run on the whole chunk.
    const size_t fstride = (size_t)3 * h->d.height * h->d.width;
    for (int s0 = 0; s0 < B; s0 += h->sub_frames) {
      const int nb = std::min(h->sub_frames, B - s0);
      void* dst = (char*)h->buf[1] + (size_t)s0 * h->front_out_elems * elt;
      if ((rc = run_front(h, frames + s0 * fstride, nb, h->sbuf, dst, &x, bf, s))) return rc;
    }
    x = h->buf[1];
    hh = h->front_hw[0];
    ww = h->front_hw[1];
    if ((rc = run_blocks(h, h->n_front, h->blocks.size(), x, h->buf, B, hh, ww, nullptr, &x, bf, s))) return rc;
  } else {
    // every block in one pass, so that layer1's last conv3 can pair with layer2's first conv1
    if ((rc = run_stem(h, frames, B, h->buf, bf, s))) return rc;
    if ((rc = run_blocks(h, 0, h->blocks.size(), h->buf[1], h->buf, B, hh, ww, nullptr, &x, bf, s))) return rc;
  }
  if (h->planning) return EOSV_OK;
  poison_lds(s);
  return launch_avgpool(x, B, hh * ww, h->D, feat, x3(h) ? 2 : bf ? 1 : 0, s);
}

// Chunk planner.  A launch's grid runs in whole waves of `slots` workgroups, so a chunk whose
// grids end in a part-full wave pays for the empty slots (R18 layer 4 at 3122 frames: 1196
// blocks of 256 x 256 = 4.67 waves of 256 -> 93 %).  The price of a chunk of F frames is the
// dry-run forward's FLOPs divided by each launch's wave efficiency (add_plan_cost); B frames are
// split into n - 1 chunks of c frames and a last one (n = the fewest chunks max_frames allows,
// or one more), choosing c by that price.  Prices are computed once per handle for every chunk
// size the planner tries (lazily), plans once per frame count.  EOSV_CHUNK_PLAN=0 (profiling build): equal chunks.
static double price_chunk(eosv_handle* h, int F) {
  // priced lazily, one dry run per chunk size the planner asks for (-1 = not yet priced)
  if (h->chunk_cost.empty()) h->chunk_cost.assign((size_t)h->d.max_frames + 1, -1.0);
  double& c = h->chunk_cost[F];
  if (c < 0.0) {
    h->planning = true;
    h->plan_cost = 0.0;
    // any non-null frame pointer: the launchers choose their kernel by it and record the grid
    const int rc = forward_chunk(h, (const float*)h->zero, F, nullptr, nullptr);
    h->planning = false;
    c = rc ? 1e300 : h->plan_cost;
  }
  return c;
}

static const std::vector<int>& plan_chunks(eosv_handle* h, int B) {
  auto it = h->chunk_plans.find(B);
  if (it != h->chunk_plans.end()) return it->second;
  const int mf = h->d.max_frames;
  const int nmin = (B + mf - 1) / mf;
  std::vector<int> best;
  {  // equal chunks (the plan before the planner)
    const int csz = (B + nmin - 1) / nmin;
    for (int b0 = 0; b0 < B; b0 += csz) best.push_back(std::min(csz, B - b0));
  }
  static const int on = env_switch("EOSV_CHUNK_PLAN", 1);
  if (on) {
    double bc = 0.0;
    for (int nb : best) bc += price_chunk(h, nb);
    for (int n = nmin; n <= nmin + 1; ++n) {
      const int lo = (B + n - 1) / n;  // the largest chunk holds at least this
      for (int c = lo; c <= std::min(mf, B); ++c) {
        const int last = B - (n - 1) * c;
        if (last <= 0) break;
        if (last > c) continue;
        const double cost = (n - 1) * price_chunk(h, c) + price_chunk(h, last);
        if (cost < bc * (1.0 - 1e-9)) {
          bc = cost;
          best.assign((size_t)(n - 1), c);
          best.push_back(last);
        }
      }
    }
  }
  return h->chunk_plans.emplace(B, std::move(best)).first->second;
}

}  // namespace eosv

using namespace eosv;

extern "C" {

const char* eosv_last_error(void) { return g_err.c_str(); }

int eosv_create(const eosv_desc* desc, eosv_handle** out) {
  if (!desc || !out) {
    set_error("eosv_create: null argument");
    return EOSV_ERR_ARG;
  }
  *out = nullptr;
  if (desc->height < 32 || desc->width < 32 || desc->max_frames <= 0 || desc->num_classes <= 0 ||
      (desc->dtype != EOSV_F32 && desc->dtype != EOSV_BF16 && desc->dtype != EOSV_F32X3)) {
    set_error("eosv_create: bad desc (height/width >= 32, max_frames > 0, dtype f32|bf16|f32x3)");
    return EOSV_ERR_ARG;
  }
  EOSV_HIP_CHECK(hipSetDevice(desc->device));
  eosv_handle* h = new eosv_handle();
  h->d = *desc;
  int rc = build_plan(h);
  const size_t elt = act_bytes(h);
  const size_t F = (size_t)desc->max_frames;
  // + 256 B: the fused bf16 stem's DMA reads up to 12 B before a row (stem_pool_bf16.hip)
  const size_t pack_bytes =
      rc || !stem_needs_pack(h) ? 256
                                : stem_input_elems((int)F, desc->height, desc->width, h->stem.pad) * (stem_bf(h) ? 2 : 4) + 256;
  void* pack_base = nullptr;
  if (!rc) rc = dmalloc(h, &pack_base, pack_bytes);
  // zero borders of the padded stem input: written once here, the packer only fills interiors
  if (!rc && hipMemset(pack_base, 0, pack_bytes) != hipSuccess) rc = (set_error("hipMemset pack"), EOSV_ERR_HIP);
  if (!rc) h->pack = (char*)pack_base + 128;
  if (!rc) rc = dmalloc(h, &h->zero, 256);
  if (!rc && hipMemset(h->zero, 0, 256) != hipSuccess) rc = (set_error("hipMemset zero"), EOSV_ERR_HIP);
  for (int i = 0; i < 4 && !rc; ++i) rc = dmalloc(h, &h->buf[i], F * h->act_elems * elt);
  {
    // front-stage sub-chunk: keeps stem/layer1 activations Infinity-Cache resident
    int sub = env_switch("EOSV_SUB_FRAMES", 0);  // measured: no gain at 64..256 (R18 f32/bf16, R50 bf16)
    if (sub > 0 && sub < desc->max_frames) {
      h->sub_frames = sub;
      for (int i = 0; i < 4 && !rc; ++i) rc = dmalloc(h, &h->sbuf[i], (size_t)sub * h->act_elems * elt);
    }
  }
  if (rc) {
    eosv_destroy(h);
    return rc;
  }
  *out = h;
  return EOSV_OK;
}

int eosv_load_weights(eosv_handle* h, const char* const* names, const void* const* host_ptrs,
                      const int64_t* numel, int n) {
  if (!h || (n > 0 && (!names || !host_ptrs || !numel)) || n < 0) {
    set_error("eosv_load_weights: bad argument");
    return EOSV_ERR_ARG;
  }
  EOSV_HIP_CHECK(hipSetDevice(h->d.device));
  Tensors t;
  for (int i = 0; i < n; ++i) {
    if (!names[i]) continue;
    t.m[names[i]] = {(const float*)host_ptrs[i], numel[i]};
  }
  const bool bf = conv_bf(h), sp = x3(h);
  int rc;
  // a reload overwrites the weight buffers in place: let every queued forward finish first
  if (h->loaded) EOSV_HIP_CHECK(hipDeviceSynchronize());
  h->loaded = false;
  if ((rc = upload_conv(h, h->stem, t, stem_bf(h), true))) return rc;
  if (sp) {  // split-bf16 stem weights: the bf16 stem layout (K 192), as hi and lo = bf16(w - hi)
    Conv c = h->stem;
    c.K = 192;
    std::vector<float> wf, beta;
    if (!fold_conv(c, t, true, true, wf, beta)) return EOSV_ERR_ARG;
    std::vector<unsigned short> wb(2 * wf.size());
    for (size_t i = 0; i < wf.size(); ++i) {
      const float hi = bf_round_host(wf[i]);
      wb[i] = f2bf_host(hi);
      wb[wf.size() + i] = f2bf_host(wf[i] - hi);
    }
    c.w = h->stem_x3.w;
    c.b = h->stem_x3.b;
    c.wbytes = h->stem_x3.wbytes;
    if ((rc = upload_bytes(h, &c.w, &c.wbytes, wb.data(), wb.size() * 2))) return rc;
    size_t bcap = c.b ? (size_t)c.cout * 4 : 0;
    if ((rc = upload_bytes(h, (void**)&c.b, &bcap, beta.data(), (size_t)c.cout * 4))) return rc;
    h->stem_x3 = c;
  }
  for (Block& b : h->blocks) {
    if ((rc = upload_conv(h, b.c1, t, bf, true, nullptr, sp))) return rc;
    Conv* fds = b.fuse_ds ? &b.ds : nullptr;
    if ((rc = upload_conv(h, b.c2, t, bf, true, b.bottleneck ? nullptr : fds, sp))) return rc;
    if (b.bottleneck && (rc = upload_conv(h, b.c3, t, bf, true, fds, sp))) return rc;
    if (b.has_ds && !b.fuse_ds && (rc = upload_conv(h, b.ds, t, bf, true, nullptr, sp))) return rc;
  }
  Conv& fc = h->fc;
  fc.bnname = "fc.bias";
  if ((rc = upload_conv(h, fc, t, false, false))) return rc;
  h->loaded = true;
  return EOSV_OK;
}

int eosv_backbone_forward(eosv_handle* h, const float* d_frames, int B, float* d_feat,
                          eosv_stream_t stream) {
  if (!h || B < 0 || (B > 0 && (!d_frames || !d_feat))) {
    set_error("eosv_backbone_forward: bad argument");
    return EOSV_ERR_ARG;
  }
  if (!h->loaded) {
    set_error("eosv_backbone_forward: weights not loaded");
    return EOSV_ERR_STATE;
  }
  const size_t fstride = (size_t)3 * h->d.height * h->d.width;
  if (B == 0) return EOSV_OK;
  int b0 = 0;
  for (const int nb : plan_chunks(h, B)) {
    int rc = forward_chunk(h, d_frames + b0 * fstride, nb, d_feat + (size_t)b0 * h->D, (hipStream_t)stream);
    if (rc) return rc;
    b0 += nb;
  }
  return EOSV_OK;
}

int eosv_backbone_probe(eosv_handle* h, const float* d_frames, int B, int stage, float* d_out,
                        eosv_stream_t stream) {
  if (!h || B < 1 || B > h->d.max_frames || stage < 0 || stage > 4 || !d_frames || !d_out) {
    set_error("eosv_backbone_probe: bad argument (1 <= B <= max_frames, 0 <= stage <= 4)");
    return EOSV_ERR_ARG;
  }
  if (!h->loaded) {
    set_error("eosv_backbone_probe: weights not loaded");
    return EOSV_ERR_STATE;
  }
  const bool bf = conv_bf(h);
  const hipStream_t s = (hipStream_t)stream;
  int rc;
  if ((rc = poison_bufs(h, s))) return rc;
  if ((rc = run_stem(h, d_frames, B, h->buf, bf, s))) return rc;
  void* x = h->buf[1];
  int hh = h->hp, ww = h->wp;
  if (stage > 0 && (rc = run_blocks(h, 0, h->stage_end[stage - 1], x, h->buf, B, hh, ww, nullptr, &x, bf, s)))
    return rc;
  const int* hwc = h->stage_hwc[stage];
  const long long per_frame = (long long)hwc[0] * hwc[1] * hwc[2];
  if ((rc = launch_act_to_f32(x, per_frame * B, hwc[2], x3(h) ? 2 : bf ? 1 : 0, d_out, s))) return rc;
  return (int)per_frame;
}

int eosv_fc_forward(eosv_handle* h, const float* d_feat, int B, float* d_logits, eosv_stream_t stream) {
  if (!h || B < 0 || (B > 0 && (!d_feat || !d_logits))) {
    set_error("eosv_fc_forward: bad argument");
    return EOSV_ERR_ARG;
  }
  if (!h->loaded) {
    set_error("eosv_fc_forward: weights not loaded");
    return EOSV_ERR_STATE;
  }
  if (B == 0) return EOSV_OK;
  return run_conv(h, h->fc, d_feat, B, 1, 1, nullptr, d_logits, false, false, (hipStream_t)stream);
}

int eosv_feature_dim(const eosv_handle* h) { return h ? h->D : EOSV_ERR_ARG; }

int64_t eosv_device_bytes(const eosv_handle* h) { return h ? h->bytes : EOSV_ERR_ARG; }

int eosv_profile_enable(eosv_handle* h, int enable) {
  if (!h) return set_error("eosv_profile_enable: null handle"), EOSV_ERR_ARG;
  // the window's first / last dispatch (null stream, one wave, no memory access): a kernel trace or
  // PMC pass of the same command finds exactly the profiled launches between the two markers
  // (tools/traffic_json.py), instead of counting dispatches back from the end of the run.  On the
  // handle's device (its null stream), as every other entry point that launches
  EOSV_HIP_CHECK(hipSetDevice(h->d.device));
  if (enable && !h->prof) {
    hipLaunchKernelGGL(profile_window_begin_kernel, dim3(1), dim3(64), 0, (hipStream_t)0);
    EOSV_LAUNCH_CHECK();
  } else if (!enable && h->prof) {
    hipLaunchKernelGGL(profile_window_end_kernel, dim3(1), dim3(64), 0, (hipStream_t)0);
    EOSV_LAUNCH_CHECK();
  }
  h->prof = enable != 0;
  h->recs.clear();
  h->pool_used = 0;
  return EOSV_OK;
}

int eosv_profile_read(eosv_handle* h, double* ms, double* flops, int64_t* launches, int max_layers) {
  if (!h || max_layers < 0 || (max_layers > 0 && (!ms || !flops || !launches)))
    return set_error("eosv_profile_read: bad argument"), EOSV_ERR_ARG;
  for (int i = 0; i < max_layers; ++i) {
    ms[i] = 0;
    flops[i] = 0;
    launches[i] = 0;
  }
  for (const auto& r : h->recs) {
    EOSV_HIP_CHECK(hipEventSynchronize(r.b));
    float t = 0;
    EOSV_HIP_CHECK(hipEventElapsedTime(&t, r.a, r.b));
    if (r.id < max_layers) {
      ms[r.id] += t;
      flops[r.id] += r.flops;
      launches[r.id] += 1;
    }
  }
  return h->n_layers;
}

void eosv_destroy(eosv_handle* h) {
  if (!h) return;
  for (hipEvent_t e : h->pool) (void)hipEventDestroy(e);
  for (void* p : h->allocs) (void)hipFree(p);
  delete h;
}

}  // extern "C"
