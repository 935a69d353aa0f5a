// Internal helpers shared by the eosv HIP translation units (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>

#include "eosv.h"

#include <cstdint>
#include <string>

namespace eosv {

// r06 A/B (release variants): the bf16 WS / tap-shift tiles issue a group's next A fragment read
// ahead of all of the group's MFMAs (1, r06 default: R18 +0.4 %, R50 neutral, bitwise equal;
// profiles/r06ab_rfirst.txt) or after its first (0, r04-r06)
#ifndef EOSV_BF16_RFIRST
#define EOSV_BF16_RFIRST 1
#endif

// s_waitcnt vmcnt(N) (gfx9 encoding: vmcnt split over bits 3:0 and 15:14, expcnt / lgkmcnt left
// at their "no wait" maxima).  Through the builtin, not inline asm, so that hipcc's waitcnt pass
// sees it and knows which loads it retired: after an asm wait hipcc still waited for them itself,
// and while an LDS-DMA is in flight it does so with vmcnt(0).
// The empty asm after it is the compiler-level memory barrier the builtin is not: without it,
// LDS reads of a ring slot could be scheduled above the wait (and the s_barrier after it) that
// makes the slot's DMA complete -- a race (r03: wrong bf16 features one run in several).
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
  asm volatile("" ::: "memory");
}

// 128-bit buffer store with an SGPR soffset, then one wait state before its data VGPRs can be
// rewritten.  A VMEM store wider than 64 bits reads its data VGPRs after issue; hipcc pads a VALU
// write of them right behind the store only when soffset is an inline constant.  With an SGPR
// soffset it emits nothing, and on gfx950 that write can win: bneck_bf16_kernel<64,64,false> stored
// the LDS base a following v_mov put in v152 into one dword of lanes 12/13
// (tests/native/bneck_check.cpp; tools/isa_scan.py checks every store of the library, in the CPU
// suite).  Folding the soffset into the voffset instead costs the 256-channel fused kernels 24-48
// B/lane of scratch; a bare s_nop after the store is not enough (the scheduler moved the v_mov
// above it), sched_barriers around the store cost the epilogue its overlap with the next MFMAs.
template <class V>
__device__ __forceinline__ void store_b128_guarded(V v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
#ifdef EOSV_STORE_GUARD_SB  // r06 first form (A/B only: tools/build_variant.sh sbguard -DEOSV_STORE_GUARD_SB)
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, 0);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 0");
  __builtin_amdgcn_sched_barrier(0);
#elif defined(EOSV_STORE_GUARD_OFF)  // negative control for the race tests only (tools/build_variant.sh)
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, 0);
#else
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, 0);
  asm volatile("s_nop 0" ::"v"(v));  // "uses" the data: nothing rewrites its VGPRs before the nop
#endif
}

// Packed epilogue arithmetic (r06) for the kernels that keep D = W . X^T accumulators with 8
// consecutive channels per lane (the fused 1x1 pairs and bneck_bf16): the shift and residual adds as
// v_pk_add_f32 on (even, odd) channel pairs, bf16(max(v, 0)) as one v_cvt_pk_bf16_f32 and one
// v_pk_max_i16 with 0 (a bf16 with its sign bit set is a negative int16, so negative values and -0
// become +0).  Bit for bit the scalar form `bf16(fmaxf(v, 0))` per element (NaN aside), in about
// half the VALU instructions: that form compiled to one conversion per element plus a shift and an
// or per pair.
namespace epi {
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned relu_bf2(f32x2 v) {
  const s16x2 h = __builtin_bit_cast(s16x2, __builtin_convertvector(v, bf16x2));
  return __builtin_bit_cast(unsigned, __builtin_elementwise_max(h, (s16x2){0, 0}));
}
// a bf16x2 word (lo = the even channel) as f32
__device__ __forceinline__ f32x2 bf2_f(unsigned u) {
  return (f32x2){__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}
// pair k (channels 2k, 2k + 1 of the lane's 8) of the two accumulators (or shift vectors) A, B
__device__ __forceinline__ f32x2 pair_of(const f32x4& A, const f32x4& B, int k) {
  const f32x4 X = k >> 1 ? B : A;
  return k & 1 ? X.hi : X.lo;
}
}  // namespace epi

void set_error(const std::string& msg);

// A/B switches and profiling ablations exist only in the profiling build (`make prof` ->
// libeosv_prof.so, -DEOSV_PROFILING; tools/ select it with EOSV_LIBRARY).  In the release
// library every switch is its compile-time default and no environment variable is read.
#ifdef EOSV_PROFILING
int env_switch(const char* name, int dflt);
#define EOSV_ABL(a) ((a).abl)
#else
constexpr int env_switch(const char*, int dflt) { return dflt; }
#define EOSV_ABL(a) 0
#endif

#define EOSV_HIP_CHECK(expr)                                                               \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess) {                                                                \
      ::eosv::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));               \
      return EOSV_ERR_HIP;                                                                 \
    }                                                                                      \
  } while (0)

#define EOSV_LAUNCH_CHECK()                                                                \
  do {                                                                                     \
    hipError_t _e = hipGetLastError();                                                     \
    if (_e != hipSuccess) {                                                                \
      ::eosv::set_error(std::string("kernel launch: ") + hipGetErrorString(_e));          \
      return EOSV_ERR_HIP;                                                                 \
    }                                                                                      \
  } while (0)

// ------------------------------------------------------------------ launch planning
// A launcher given a LaunchInfo (ConvArgs::plan, or the stems' `info` argument) records its grid
// instead of launching: the workgroups (persistent kernels: work items, e.g. row strips) and how
// many of them the GPU runs at once.  The chunk planner (eosv_api.hip) prices a chunk size by
// the wave quantisation this implies.
struct LaunchInfo {
  long long blocks;
  long long slots;
};
int device_cu_count();  // CUs of the current device (cached; 256 on MI355X)
// workgroups of `kernel` resident per CU (hipOccupancyMaxActiveBlocksPerMultiprocessor), >= 1
int kernel_occupancy(const void* kernel, int threads, size_t dyn_lds = 0);
inline int record_launch(LaunchInfo* info, long long blocks, long long per_cu) {
  info->blocks = blocks;
  info->slots = per_cu * device_cu_count();
  return EOSV_OK;
}

// ------------------------------------------------------------------ conv
struct ConvArgs {
  const void* x;      // NHWC input [N,H,W,Cin]  (stem, Cin = 3: padded [N][H+2p][Wp][3])
  const void* w;      // [Cout][K]: K ordered (kh, kw_padded, cin); stem (kh, kw*3 + c) 24 per kh
  const float* bias;  // [Cout] folded BN shift
  const void* res;    // NHWC residual [N,Ho,Wo,Cout] or nullptr
  void* y;            // NHWC output [N,Ho,Wo,Cout]
  int N, H, W, Cin;
  int Ho, Wo, Cout;
  int KH, KW, KWp, stride, pad;
  int K;              // padded reduction length, multiple of the kernel's BK
  int relu;
  const void* zero;   // >= 64 zeroed bytes (DMA target for out-of-bounds taps)
  int abl;            // ablation bits for profiling builds (0 = normal)
  int xcd;            // 1: XCD-aware block order (each XCD walks a contiguous range of tiles)
  int kcm;            // K chunk-major instead of (kh, kw, cin): bf16 nonzero = (cin/64, kh, kw, cin%64);
                      // f32 = the chunk C, (cin/C, kh, kw, cin%C)
  // fused 1x1 downsample (ResNet block shortcut): K columns [K1, K) read x2 at output pixel
  // (oh, ow) -> x2 pixel (oh * stride2, ow * stride2), channel k - K1; nullptr = none
  const void* x2;     // NHWC [N, H2, W2, Cin2]
  int H2, W2, Cin2, stride2, K1;
  // bf16 kernels, EOSV_F32X3: activations are stored [pixel][2 * C] bf16 = (hi, lo) blocks of C
  // channels and read as 3C virtual input channels (hi, lo, hi): Cin / Cin2 / K count those
  // (weights (w_hi, w_hi, w_lo)), virtual channel c >= 2C is physical channel c - 2C
  // (split_chan), Cout is the logical C.  The epilogue reads the residual as hi + lo and stores
  // hi, lo.
  int split;
  // physical pixel strides (elements) of x and x2: Cin / Cin2, or 2/3 of them when split
  // (0 = derive; conv_pixel_strides)
  int xs, x2s;
  LaunchInfo* plan;   // host-side: non-null = record the grid (record_launch), launch nothing
  // f32 implicit GEMM only (the training entry eosv_conv2d_f32): with a workspace, a small grid
  // splits the K loop over gridDim.y slices writing raw partial sums to kws ([slices][M][Cout],
  // kws_bytes large enough, else no split); the launcher then sums them in slice order with the
  // bias / residual / ReLU epilogue.
  float* kws;
  long long kws_bytes;
};
// the K-slice count launch_conv_f32 would use for `a` given a large enough workspace (1 = none)
int conv_f32_ksplit_slices(const ConvArgs& a);

__host__ __device__ inline int split_chan(int c, int cin3) {
  const int c2 = 2 * (cin3 / 3);
  return c >= c2 ? c - c2 : c;
}
inline void conv_pixel_strides(ConvArgs& a) {
  if (!a.xs) a.xs = a.split ? 2 * (a.Cin / 3) : a.Cin;
  if (!a.x2s) a.x2s = a.split ? 2 * (a.Cin2 / 3) : a.Cin2;
}

// Workgroups are dealt round-robin over the 8 XCDs (b and b + 8 share one L2;
// MI355X_MICROARCH.md, Workgroup dispatch).  Remap so that XCD x processes the contiguous
// logical tiles [x*q + min(x, r), ...): neighbouring M-tiles (which share input halo rows)
// and the N-tiles of one M-tile (which share the A rows) then hit the same L2.  Bijective
// on [0, nb) for any nb; placement is a speed hint only, never a correctness assumption.
__device__ __forceinline__ int xcd_tile(int b, int nb, int on) {
  if (!on) return b;
  const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return x * q + (x < r ? x : r) + i;
}

int launch_conv_f32(const ConvArgs& a, hipStream_t s);
int launch_conv_bf16(const ConvArgs& a, hipStream_t s);
bool conv_bf16_ts_ok(const ConvArgs& a);  // conv_bf16_ts.hip: tap-shift stride-1 3x3 convs
int launch_conv_bf16_ts(const ConvArgs& a, hipStream_t s);
bool stem_pool_bf16_ok(int H, int W, bool direct);  // stem_pool_bf16.hip: fused stem conv + ReLU + maxpool
int launch_stem_pool_bf16(const void* pack, int B, int H, int W, const void* w, const float* bias, void* y,
                          hipStream_t s, const float* frames = nullptr, LaunchInfo* info = nullptr);
bool stem_pool_x3_ok(int H, int W);  // stem_pool_bf16.hip: EOSV_F32X3 split-bf16 fused stem
int launch_stem_pool_x3(const float* frames, int B, int H, int W, const void* w, const float* bias, void* y,
                        hipStream_t s, LaunchInfo* info = nullptr);
bool stem_pool_f32_ok(int H, int W);  // stem_pool_f32.hip: the same for f32
bool stem_pool_f32_direct_ok(int H, int W);  // ... reading the f32 NCHW frames (W % 4 == 0, W <= 256)
int launch_stem_pool_f32(const void* pack, int B, int H, int W, const void* w, const float* bias, void* y,
                         hipStream_t s, bool split = false,  // split: y in the EOSV_F32X3 (hi, lo) layout
                         LaunchInfo* info = nullptr,
                         const float* frames = nullptr);  // non-null: DIRECT (pack unused, may be null)
bool conv_rows_bf16_ok(const ConvArgs& a);  // conv_rows_bf16.hip: stage-1 3x3 64->64 direct conv
int launch_conv_rows_bf16(const ConvArgs& a, hipStream_t s);
bool conv_rowsr_bf16_ok(const ConvArgs& a);  // conv_rowsr_bf16.hip: stage-1 3x3 64->64, weights in registers
int launch_conv_rowsr_bf16(const ConvArgs& a, hipStream_t s);
bool conv_s2rows_bf16_ok(const ConvArgs& a);  // conv_s2rows_bf16.hip: R18 stage-2 entry 3x3/2 64->128 row strips
int launch_conv_s2rows_bf16(const ConvArgs& a, hipStream_t s);

// pair1x1_bf16.hip: a bottleneck's conv3 (1x1 64 -> 256 + residual, or + a folded stride-1
// downsample reading x2 [M][64]) fused with the next block's conv1 (1x1 256 -> c1), bf16 NHWC
struct Pair1x1Args {
  const void* x;     // [M][64]   conv3 input
  const void* x2;    // [M][cds]  downsample input (cds = 64) or nullptr
  const void* res;   // [M][256]  residual (nullptr with the downsample)
  const void* w3;    // [256][64 + cds] folded conv3 (+ downsample) weights
  const float* b3;   // [256]
  const void* w1;    // [c1][256] folded next conv1 weights
  const float* b1;   // [c1]
  void* y;           // [M][256]  conv3 output (the next block's residual)
  void* z;           // [M][c1]   next conv1 output
  long long M;       // pixels, a multiple of 64 (pair1x1); any (pairw)
  int c1, cds;
  LaunchInfo* plan;  // non-null: record the grid only
  int cmid, cexp;    // pairw_bf16: conv3 is 1x1 cmid -> cexp, the next conv1 cexp -> c1
  // pairw_bf16 with the downsample (cds > 0): x2 is [N][H2][W2][cds], read at (2 oh, 2 ow) of
  // output pixel (n, oh, ow) of the Ho x Wo map
  int Ho, Wo, H2, W2;
  int abl;  // profiling-build ablation bits (EOSV_CONV_ABL), 0 otherwise
  // pairw_bf16: elements each of x, res / y and z holds (it runs on whole pairw_tile()-pixel rounds)
  long long cap_elems;
};
bool pair1x1_bf16_ok(int cmid, int cexp, int c1, int cds, long long M);
int launch_pair1x1_bf16(const Pair1x1Args& a, hipStream_t s);
// pair1x1r_bf16.hip (r04): the same pair with each wave owning its pixels for both GEMMs
int launch_pair1x1r_bf16(const Pair1x1Args& a, hipStream_t s);
// pairw_bf16.hip: the same pair for the wide stages (cmid 128 / 256, cexp 512 / 1024): weights
// streamed through an LDS ring by 64-channel chunks, Y kept in registers; residual blocks only
int pairw_tile(int cmid, int c1, int cds);  // pixels per pairw round of that shape (128, or 256 at NPT 2)
bool pairw_bf16_ok(int cmid, int cexp, int c1, int cds, long long M, long long cap_elems);
int launch_pairw_bf16(const Pair1x1Args& a, hipStream_t s);
// bneck_bf16.hip (r06): a whole bf16 stage-1 bottleneck block in one launch -- conv1 (1x1 cin -> 64)
// -> conv2 (3x3 64 -> 64) -> conv3 (1x1 64 -> 256 + residual, or + the folded stride-1 downsample
// of the block input when cin = 64), and with wn the next block's conv1 (1x1 256 -> 64) -> z
struct BneckArgs {
  const void* x;                    // [N][H][W][cin] block input (and residual / downsample input)
  const void* w1; const float* b1;  // [64][cin] folded conv1
  const void* w2; const float* b2;  // [64][9 * 64] folded conv2, K (kh, kw, cin)
  const void* w3; const float* b3;  // [256][64 (+ 64: the downsample)] folded conv3
  const void* wn; const float* bn;  // [64][256] the next block's folded conv1, or nullptr
  void* y;                          // [N][H][W][256] block output (may be x itself: in place)
  void* z;                          // [N][H][W][64] next conv1 output (wn only)
  int N, H, W, cin;
  LaunchInfo* plan;                 // non-null: record the grid only
  const void* res;                  // tail: [N][H][W][256] the residual (the block input)
  int abl;                          // profiling-build ablations (EOSV_BNECK_ABL), 0 otherwise
};
bool bneck_bf16_ok(int cin, int W, int H, int next);
int launch_bneck_bf16(const BneckArgs& a, hipStream_t s);
// the stage's last block from its conv1 output (x = [N][H][W][64], cin 64, w1 unused): conv2 ->
// conv3 + res -> y, and the next stage's conv1 (wn [128][256]) -> z [N][H][W][128]
bool bneck_tail_bf16_ok(int W, int H);
int launch_bneck_tail_bf16(const BneckArgs& a, hipStream_t s);
// a bf16 ResNet-18 stage-1 basic block (conv1 3x3 64 -> 64 + ReLU, conv2 3x3 + x + ReLU) in one
// launch (bblock_bf16.hip, r06): x, w1 / b1, w2 / b2, y (may be x), N, H, W (56 or 64), cin 64
bool bblock_bf16_ok(int W, int H);
int launch_bblock_bf16(const BneckArgs& a, hipStream_t s);
bool conv_rows_f32_ok(const ConvArgs& a);  // conv_rows_f32.hip: f32 stage-1 3x3 64->64 direct conv
int launch_conv_rows_f32(const ConvArgs& a, hipStream_t s);
bool conv_rows_x3_ok(const ConvArgs& a);  // conv_rows_x3.hip: f32x3 stage-1 3x3 64->64 direct conv
int launch_conv_rows_x3(const ConvArgs& a, hipStream_t s);

// ------------------------------------------------------------------ layout / pooling
// stem input layout: zero-bordered RGB rows of stem_row_pixels(W, pad) pixels (even, so the
// stem's bf16 DMA sources stay 4-B aligned)
__host__ __device__ inline int stem_row_pixels(int W, int pad) { return (W + 2 * pad + 1) & ~1; }
inline size_t stem_input_elems(int B, int H, int W, int pad) {
  return (size_t)B * (H + 2 * pad) * stem_row_pixels(W, pad) * 3 + 64;  // + over-read slack
}
int launch_pack_rgb_pad(const float* x, int B, int H, int W, int pad, void* y, int bf16, hipStream_t s);
int launch_maxpool3x3s2(const void* x, int B, int H, int W, int C, void* y, int Ho, int Wo,
                        int bf16, hipStream_t s);
// bf16: 0 f32 input, 1 bf16, 2 the EOSV_F32X3 split layout (value = hi + lo)
int launch_avgpool(const void* x, int B, int HW, int C, float* y, int bf16, hipStream_t s);
int launch_act_to_f32(const void* x, long long n, int C, int mode, float* y, hipStream_t s);

}  // namespace eosv
