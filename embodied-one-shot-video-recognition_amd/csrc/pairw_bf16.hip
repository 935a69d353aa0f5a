// Fused 1x1 pair for the bf16 bottleneck stages 2-3 (ResNet-50/101 layer2 / layer3): block b's
// conv3 (1x1 CMID -> CEXP, folded BN, + residual, ReLU) and block b+1's conv1 (1x1 CEXP -> C1,
// folded BN, ReLU) in one pass over the pixels (torchvision Bottleneck.forward: conv3 -> bn3 ->
// += identity -> relu, then the next block's conv1 -> bn1 -> relu; reference models.py:19 via
// self.convnet, driven from network_test.py:59).
//
// Unfused, the CEXP-channel map Y that conv3 writes is read straight back by the next conv1.
// Both 1x1s are HBM-bound (conv3 at 57-114 FLOP/B, conv1 at 102-205 FLOP/B against the bf16
// ridge of 315), so the pair's floor is its bytes: per pixel X (CMID) + R (CEXP) -> Y (CEXP) +
// Z (C1), without the second read of Y (stage 2: 2.5 KB instead of 3.5 KB per pixel).
//
// The stage-1 pair (pair1x1_bf16.hip) keeps both weight matrices in LDS; here they are 128 KB
// to 512 KB each, so they stream through LDS instead and Y never leaves registers:
//   * persistent workgroups of 8 waves (one per CU); a round is 128 pixels, 16 per wave;
//   * the CEXP channels go in chunks of 64: an LDS ring holds a chunk's W3 rows (64 x CMID) and
//     W1 columns (C1 x 64), filled by LDS-DMA two chunks ahead in 3 slots where they fit (stage
//     2: 100 / 146 KiB), else one chunk ahead in 2, one barrier per chunk; every wave reads the
//     same slot for its own 16 pixels;
//   * GEMM1 per chunk: D1[64 cout][16 px] = W3c . X^T on v_mfma_f32_16x16x32_bf16, the X
//     fragments of the wave's pixels held in registers for the whole round; W3 rows are permuted
//     (MFMA tile i, row 4q + e holds cout 32(i >> 1) + 8q + 4(i & 1) + e, as in pair1x1_bf16) so
//     a lane ends up with couts 8q .. 8q + 7 and 32 + 8q .. 32 + 8q + 7 of pixel r: 16-B residual
//     loads and Y stores, and after bias + residual + ReLU + bf16 exactly the B fragments of the
//     chunk's two 32-wide k-slices of GEMM2;
//   * GEMM2 accumulates D2[C1][16 px] += W1c . Ychunk^T chunk by chunk, then bias + ReLU -> Z.
// K is walked in the unfused kernels' order (32-wide slices, increasing k), bias then residual
// then ReLU then round-to-nearest bf16: both maps equal the unfused conv3 -> conv1 pair's bit for
// bit (tests/native/conv_check.cpp).  The residual of chunk ch + 3 is loaded while chunk ch
// computes, the next round's X during the round's last chunk; loads / stores use buffer resources
// based at the round's first pixel (per-lane part the VGPR offset, chunk / channel-group part the
// scalar offset), over whole 128-pixel tiles: the tail round runs on the buffers' padding.
#include <hip/hip_bf16.h>

#include "common.h"

namespace eosv {

namespace {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_t;

// MFMA tile i, row t (0..15) -> channel within the 64-channel group
__device__ __forceinline__ int permrow(int i, int t) { return 32 * (i >> 1) + 8 * (t >> 2) + 4 * (i & 1) + (t & 3); }
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(bytes > 0x7fffffffLL ? 0x7fffffffLL : bytes),
                                           0x00020000);
}
// one 1-KiB LDS-DMA piece (a free function: the builtin inside a lambda drops the kernel's host
// stub).  global_load_lds, not buffer_load ... lds: after the buffer form hipcc waited vmcnt(0)
// before the next LDS read (for every DMA in flight, the next chunk's included)
__device__ __forceinline__ void dma16(const unsigned char* src, void* lds) {
  __builtin_amdgcn_global_load_lds((const void*)src, (lds_t*)lds, 16, 0, 0);
}
}  // namespace

// NPT: 16-pixel tiles per wave, 8 waves (two per SIMD); a round is 128 NPT pixels.  The LDS feeds
// one 1-KiB weight fragment per MFMA at NPT = 1: per 64-channel chunk the 8 waves read 256 KiB
// (stage 2) / 512 KiB (stage 3) against 1024 / 2048 MFMA cycles per SIMD, i.e. the LDS read
// rate, not HBM, bounds the pair.  NPT = 2 (r04, restored r06: the stage-2 pair with C1 = 128 on
// 256-pixel rounds, ~240 VGPRs) reads each fragment once for two pixel tiles.
// DSC > 0 (block 0 of a stage, r03): conv3's K also holds the folded stride-2 1x1 downsample, DSC
// more columns read from the previous stage's output x2 at pixel (2 oh, 2 ow) (ConvArgs::x2 of
// the unfused conv), and there is no residual.
template <int CMID, int CEXP, int C1, int NPT, int DSC = 0>
struct PairW {
  static constexpr int K3 = CMID + DSC;                // conv3's K
  static constexpr int NW = 8;                         // waves per workgroup
  static constexpr int PX = 16 * NPT;                  // pixels per wave
  static constexpr int TILE = PX * NW;                 // pixels per round
  static constexpr int W3B = 64 * K3 * 2;  // a chunk's W3 rows (64 couts x K3), bytes
  static constexpr int W1B = C1 * 64 * 2;    // a chunk's W1 columns (C1 x 64 k), bytes
  static constexpr int STAGE_W = W3B + W1B;
  // + the chunk's 64 conv3 BN shifts (256 B, DMA'd with the weights: an LDS read outside the ring
  // slots made hipcc wait vmcnt(0), i.e. for the in-flight DMA, before it)
  static constexpr int STAGE = STAGE_W + 256;
  static constexpr int PPW = STAGE_W / 1024 / NW;  // 1-KiB DMA pieces per wave per chunk
  static constexpr int NCH = CEXP / 64;
  static constexpr int XS = K3 / 32;    // X fragments (k-slices of GEMM1) per lane
  static constexpr int XSM = CMID / 32;  // ... of them from x (the rest from x2)
  static constexpr int G2 = C1 / 64;    // 64-cout groups of GEMM2
  // weight ring: 3 slots (DMA two chunks ahead) where they fit beside the conv1 shifts, else 2
  static constexpr int NSLOT = 3 * STAGE + C1 * 4 <= 163840 ? 3 : 2;
  static constexpr int LDS = NSLOT * STAGE + C1 * 4;
  static_assert(STAGE_W % (1024 * NW) == 0 && W3B % 1024 == 0 && PPW >= 2, "DMA pieces");
  static_assert(NCH % 4 == 0, "ring slots / residual ring");
  static_assert(PPW < XS + 2 * G2, "DMA pieces go out one per fragment group, the residual loads after them");
  static_assert(NPT == 1 || (NPT == 2 && DSC == 0 && C1 == 128), "pairw_bf16: NPT 2 only for the stage-2 pair");
};

// ABL (profiling-only instance, EOSV_CONV_ABL bits; results wrong): 1 no weight DMA, 2 no
// residual loads, 4 no Y stores, 8 no MFMAs, 16 no chunk barriers, 32 no Z stores, 64 no X loads.
// CS: the chunk waits count the Y / Z stores issued after a slot's last DMA piece among the younger
// ops (vmcnt retires loads, stores and LDS-DMA together in issue order, MI355X_MICROARCH.md), so
// they do not drain the residual prefetch; without CS they count loads only (r03), which is
// stricter whenever a store is still in flight.
#ifndef EOSV_PAIRW_FD
#define EOSV_PAIRW_FD 2
#endif
template <int CMID, int CEXP, int C1, int NPT, int DSC, bool CS, bool ABL = false>
__global__ __launch_bounds__(512, 1) void pairw_bf16_kernel(Pair1x1Args a) {
  using P = PairW<CMID, CEXP, C1, NPT, DSC>;
  constexpr int FD = NPT == 1 ? EOSV_PAIRW_FD : 2;
  const int abl = ABL ? a.abl : 0;
  constexpr int K3 = P::K3, XSM = P::XSM;
  constexpr int NCH = P::NCH, XS = P::XS, G2 = P::G2, PPW = P::PPW, NT = 64 * P::NW;
  __shared__ __attribute__((aligned(16))) unsigned char smem[P::LDS];
  constexpr int NSLOT = P::NSLOT;
  float* const b1s = (float*)(smem + NSLOT * P::STAGE);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  const long long M = a.M;
  constexpr int PW_TILE = P::TILE;
  const long long nrounds = (M + PW_TILE - 1) / PW_TILE;
  long long rt = blockIdx.x;  // launch: gridDim.x <= nrounds

  for (int i = tid; i < C1; i += NT) b1s[i] = a.b1[i];

  // ---- weight DMA: piece j of this wave covers stage bytes [o, o + 1024), lane 16 B of it.
  // Per lane the source offset within a chunk is fixed (vrel); the chunk moves it by a scalar.
  const unsigned char* w3b = (const unsigned char*)a.w3;
  const unsigned char* w1b = (const unsigned char*)a.w1;
  int vrel[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int o = (w * PPW + j) * 1024 + lane * 16;
    if (o < P::W3B) {  // W3 row R (tile R >> 4, row R & 15), 16-B chunk c' = c ^ (R & 15)
      const int R = o / (K3 * 2), cs = (o % (K3 * 2)) / 16;
      const int c = cs ^ (R & 15);
      vrel[j] = (permrow(R >> 4, R & 15) * K3 + 8 * c) * 2;
    } else {  // W1 row RR (group RR >> 6, tile (RR >> 4) & 3, row RR & 15), c' = c ^ ((RR >> 1) & 7)
      const int o1 = o - P::W3B;
      const int RR = o1 / 128, cs = (o1 % 128) / 16;
      const int c = cs ^ ((RR >> 1) & 7);
      vrel[j] = ((64 * (RR >> 6) + permrow((RR >> 4) & 3, RR & 15)) * CEXP + 8 * c) * 2;
    }
  }
  auto dma_piece = [&](int j, int ch, int slot) {
    const int o = (w * PPW + j) * 1024;  // wave-uniform
    unsigned char* dst = smem + slot * P::STAGE + o;
    if (o < P::W3B)
      dma16(w3b + (long long)ch * 64 * K3 * 2 + vrel[j], dst);
    else
      dma16(w1b + ch * 128 + vrel[j], dst);
    if (j == 0 && w == 0 && lane < 16)  // the chunk's conv3 shifts: 16 lanes x 16 B
      dma16((const unsigned char*)(a.b3 + ch * 64) + lane * 16, smem + slot * P::STAGE + P::STAGE_W);
  };

  // ---- per-round resources, based at the round's first pixel and always a whole 128-pixel tile:
  // the tail round (M % 128) reads and writes its padding pixels p >= M like any others (garbage
  // in, garbage out, never read: every output pixel depends on its own input pixel only; the
  // launcher checks that the buffers hold the padded tile).  Masking them instead, with buffer
  // records ending at M, made the tail round's loads / stores partly out of range, and the tail
  // round's features then changed from run to run (r03, tools/race_probe.py).  A round past the
  // last one (the final round's prefetch) gets empty records: its loads return 0 without touching
  // memory.  (Re-reading the last round there instead -- lines another workgroup is rewriting in
  // place, y = res -- made features of other frames change from run to run in later launches.)
  struct RoundRes {
    __amdgpu_buffer_rsrc_t x, res, y, z;
  };
  auto round_res = [&](long long t) {
    RoundRes rr;
    const long long p0 = t * PW_TILE;
    const long long n = t < nrounds ? PW_TILE : 0;
    rr.x = rsrc((const unsigned short*)a.x + p0 * CMID, n * CMID * 2);
    rr.res = rsrc((const unsigned short*)a.res + p0 * CEXP, n * CEXP * 2);
    rr.y = rsrc((unsigned short*)a.y + p0 * CEXP, n * CEXP * 2);
    rr.z = rsrc((unsigned short*)a.z + p0 * C1, n * C1 * 2);
    return rr;
  };
  // the lane's pixels within a round: 16 t + r of the wave's block, t < NPT
  const int pw = P::PX * w + r;
  // DSC: x2 pixel (img, 2 oh, 2 ow) of the lane's pixel p of round t (tails: pixel 0, never stored)
  auto x2pix = [&](long long t, int tt) {
    long long p = t * PW_TILE + pw + 16 * tt;
    if (p >= M) p = 0;
    const long long hw = (long long)a.Ho * a.Wo;
    const long long img = p / hw;
    const int rem = (int)(p - img * hw), oh = rem / a.Wo, ow = rem - (rem / a.Wo) * a.Wo;
    return (const unsigned short*)a.x2 + ((img * a.H2 + 2 * oh) * a.W2 + 2 * ow) * DSC + 8 * q;
  };
  auto load_x = [&](const RoundRes& rr, long long t, v4u (*xf)[XS]) {
#pragma unroll
    for (int tt = 0; tt < NPT; ++tt) {
#pragma unroll
      for (int s = 0; s < XSM; ++s)
        xf[tt][s] = __builtin_amdgcn_raw_buffer_load_b128(rr.x, ((pw + 16 * tt) * CMID + 8 * q) * 2, 64 * s, 0);
      if constexpr (DSC > 0) {
        const unsigned short* p2 = x2pix(t, tt);
#pragma unroll
        for (int s = XSM; s < XS; ++s) xf[tt][s] = *(const v4u*)(p2 + 32 * (s - XSM));
      }
    }
  };
  auto load_r = [&](const RoundRes& rr, int ch, v4u (*rv)[2]) {
#pragma unroll
    for (int t = 0; t < NPT; ++t)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
        rv[t][hh] = __builtin_amdgcn_raw_buffer_load_b128(rr.res, ((pw + 16 * t) * CEXP + 8 * q) * 2,
                                                          (ch * 64 + 32 * hh) * 2, 0);
  };

  // the residual of chunk ch is loaded RD chunks ahead (HBM latency under load is several chunks
  // of this loop: with one chunk of lead the epilogue waited on it), into a ring of 4 register sets
  constexpr int RD = XS >= 8 ? 2 : 3;  // (CMID 256: one set fewer keeps the wave within 256 VGPRs)
  constexpr int NRES = DSC ? 0 : 2 * NPT;  // residual loads per chunk
  RoundRes cur = round_res(rt);
  v4u xf[NPT][XS], rres[4][NPT][2];
  int rslot = 0;  // NSLOT 3: ring slot of the current chunk (chunk count mod 3)
#pragma unroll
  for (int j = 0; j < PPW; ++j) dma_piece(j, 0, 0);
  if constexpr (NSLOT == 3) {  // chunk 1 too (the ring runs two chunks ahead)
#pragma unroll
    for (int j = 0; j < PPW; ++j) dma_piece(j, 1 % NCH, 1);
  }
  load_x(cur, rt, xf);
  if constexpr (!DSC) {
#pragma unroll
    for (int c = 0; c < RD; ++c) load_r(cur, c, rres[c]);
  }

  for (; rt < nrounds; rt += gridDim.x) {
    const RoundRes nxt = round_res(rt + gridDim.x);
    f32x4 acc2[NPT][G2][4];
#pragma unroll
    for (int t = 0; t < NPT; ++t)
#pragma unroll
      for (int g = 0; g < G2; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc2[t][g][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    // chunk quads: the residual register set (and with 2 slots the ring slot) are compile-time
    // per step; with 3 slots the slot of chunk ch is the workgroup's chunk count mod 3 (rslot),
    // and chunk ch + 2 goes into rslot + 2 mod 3 (the slot chunk ch - 1 was read from)
#pragma unroll 1
    for (int cp = 0; cp < NCH; cp += 4)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ch = cp + u;
      const int slot = NSLOT == 3 ? rslot : u & 1;
      const int wslot = NSLOT == 3 ? (rslot == 0 ? 2 : rslot - 1) : slot ^ 1;
      // This wave's DMA of chunk ch is done, then every wave's (barrier): the slot is complete,
      // and slot ^ 1 (chunk ch - 1) is free for the next chunk's DMA.  In chunk ch - 1 the DMA
      // pieces went out with its first PPW fragment groups (one per group: an LDS-DMA issue costs
      // the wave ~60-185 cycles, so all of them at once idled the SIMD's MFMA pipe); the loads
      // issued after the last piece (order pinned by the sched_barriers) may stay in flight:
      // 2 NPT residual loads (group PPW) and, in the round's last chunk, the next round's XS NPT
      // X loads when the epilogue (after group XS - 1) follows the last piece; before the loop:
      // XS NPT X loads + 2 RD NPT residual loads after the pieces.  The default rule (CS, r04)
      // counts the Y / Z stores issued after the last piece too: vmcnt retires loads, stores and
      // LDS-DMA in issue order (MI355X_MICROARCH.md), and the r03 failures that had been blamed on
      // counted stores came from the cp != 0 hole described below.  The r03 loads-only rule
      // survives only as the CS = 0 A/B instance (EOSV_PAIRW_CS=0, profiling build): a store still
      // in flight there makes the wait stricter (stage-2 pairs 1.43 -> 1.55 ms, stage-3 0.81 ->
      // 0.87 per 3200 frames).
      // 3 slots: chunk ch's pieces went out two chunks ago; younger than them are at least that
      // chunk's residual loads and the last chunk's pieces and residual loads (the first two
      // chunks of the launch have more: the prologue's X and residual loads), so the wait no
      // longer depends on the stores issued since
      // 2 slots, the rule (r04): the count may include the round's X loads only where chunk ch - 1
      // issued them, i.e. at the round's first chunk (cp == 0: ch - 1 was the previous round's
      // last chunk, or the prologue ran).  Until r04 every u == 0 chunk used that count, also at
      // cp = 4, 8, 12 where chunk ch - 1 (u == 3 of the previous quad) issued only its NRES residual
      // loads after its pieces: stage 3 then waited vmcnt(10) with PPW = 8 pieces + 2 residual
      // loads younger than the slot's oldest piece, i.e. for none of them, and the barrier let the
      // waves read a slot still being filled (the stage-2 DSC pair: vmcnt(12) against 8 pieces).
      // That hole explains every recorded failure (r03): the stage-2 pair of conv_check on 2 slots
      // (NCH 8, the hole at cp = 4) one run in three, R50 / R101 stage 3 (NCH 16: cp = 4, 8, 12)
      // in the race probes, and why vmcnt_probe -- which waited correctly -- found nothing.
      // With CS the 2 NPT Y stores of a chunk count too when its epilogue (after group XS - 1)
      // follows its last piece, and the round's 2 G2 NPT Z stores at a round's first chunk.
      constexpr int YS = CS && XS >= PPW ? 2 * NPT : 0;
      constexpr int YOUNG = NRES + YS;
      constexpr int YOUNG_LAST = YOUNG + (XS >= PPW ? XS * NPT : 0) + (CS ? 2 * G2 * NPT : 0);
      constexpr int YOUNG_PRO = XS * NPT + (DSC ? 0 : 2 * RD * NPT);
      static_assert(YOUNG_LAST < 64 && PPW + 2 * NRES + 2 * YS < 64, "vmcnt range");
      if constexpr (NSLOT == 3)  // younger: chunk ch - 2's residual loads (+ Y), chunk ch - 1's pieces, residual loads (+ Y)
        vm_wait<PPW + 2 * NRES + 2 * YS>();
      else if (u == 0 && cp == 0)  // scalar branch (cp is the unroll-1 loop's counter)
        vm_wait<(YOUNG_PRO < YOUNG_LAST ? YOUNG_PRO : YOUNG_LAST)>();
      else
        vm_wait<YOUNG>();
      if (!(abl & 16)) __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");  // no LDS read of the slot moves above the barrier (s_barrier is not a compiler memory barrier)
      __builtin_amdgcn_sched_barrier(0);
      // the chunk whose weights this one prefetches (the round's last one(s): the next round's first)
      const int nch = NSLOT == 3 ? (ch + 2 < NCH ? ch + 2 : ch + 2 - NCH) : (ch + 1 < NCH ? ch + 1 : 0);

      const unsigned char* ws = smem + slot * P::STAGE;
      // The chunk's A fragments come in NG groups of 4 (GEMM1 slices s = 0 .. XS - 1: W3 tiles
      // i = 0..3; then GEMM2 (k-slice s2, cout group g): W1 tiles i = 0..3), software-pipelined:
      // group gi + 1 is read from LDS while group gi's MFMAs run (sched_barriers keep the order and
      // two groups of fragments live at most: two waves per SIMD, <= 256 VGPRs).
      const unsigned char* w1s = ws + P::W3B;
      constexpr int NG = XS + 2 * G2;
      auto frags = [&](int gi, bf16x8* f) {
        if (gi < XS) {
#pragma unroll
          for (int i = 0; i < 4; ++i) f[i] = *(const bf16x8*)(ws + (16 * i + r) * (K3 * 2) + (((4 * gi + q) ^ r) << 4));
        } else {
          const int s2 = (gi - XS) / G2, g = (gi - XS) % G2;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int RR = 64 * g + 16 * i + r;
            f[i] = *(const bf16x8*)(w1s + RR * 128 + (((4 * s2 + q) ^ ((RR >> 1) & 7)) << 4));
          }
        }
      };
      // FD fragment groups in flight (r06: FD 3 = two groups read ahead where the registers allow)
      bf16x8 fr[FD][4];
      frags(0, fr[0]);
      if constexpr (FD == 3) frags(1, fr[1]);
      f32x4 acc1[NPT][4];
#pragma unroll
      for (int t = 0; t < NPT; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc1[t][i] = f32x4{0.f, 0.f, 0.f, 0.f};
      bf16x8 yf[NPT][2];
#pragma unroll
      for (int gi = 0; gi < NG; ++gi) {
        if (gi < PPW && !(abl & 1)) dma_piece(gi, nch, wslot);
        if (!DSC && gi == PPW && !(abl & 2)) {  // branch-free (scalar selects): a branch here made hipcc wait vmcnt(0) at the join
          const bool here = ch + RD < NCH;
          RoundRes rr;
          rr.res = here ? cur.res : nxt.res;
          load_r(rr, here ? ch + RD : ch + RD - NCH, rres[(u + RD) & 3]);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (gi + FD - 1 < NG) frags(gi + FD - 1, fr[(gi + FD - 1) % FD]);
        // the next group's (FD 3: the one after next) 4 LDS reads issue before this group's 4 MFMAs
        if (gi + FD - 1 < NG) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4 * NPT, 0);
        if (abl & 8) {
        } else if (gi < XS) {  // GEMM1: chunk couts, tiles i = 0..3 of 16 permuted rows
#pragma unroll
          for (int t = 0; t < NPT; ++t) {
            const bf16x8 bx = __builtin_bit_cast(bf16x8, xf[t][gi]);
#pragma unroll
            for (int i = 0; i < 4; ++i)
              acc1[t][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[gi % FD][i], bx, acc1[t][i], 0, 0, 0);
          }
        } else {  // GEMM2: D2[64g + permuted rows][px] += W1[.., k-slice s2 of the chunk] . Ychunk
          const int s2 = (gi - XS) / G2, g = (gi - XS) % G2;
#pragma unroll
          for (int t = 0; t < NPT; ++t)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              acc2[t][g][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[gi % FD][i], yf[t][s2], acc2[t][g][i], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (gi == XS - 1) {
          if (u == 3 && cp + 4 == NCH) {  // the round's X is dead: the next round's goes into the same registers
            if (!(abl & 64)) load_x(nxt, rt + gridDim.x, xf);
            __builtin_amdgcn_sched_barrier(0);
          }
          // epilogue 1: + shift, + residual, ReLU, bf16 -> Y (global) and the GEMM2 B fragments
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            // read as the fragments are (bf16x8 through the slot pointer): a float4 read here got a
            // vmcnt(0) from hipcc, as if it could alias the DMA in flight
            const unsigned char* b3c = ws + P::STAGE_W + (32 * hh + 8 * q) * 4;
            const f32x4 bA = __builtin_bit_cast(f32x4, *(const bf16x8*)b3c);
            const f32x4 bB = __builtin_bit_cast(f32x4, *(const bf16x8*)(b3c + 16));
#pragma unroll
            for (int t = 0; t < NPT; ++t) {
              const v4u rv = DSC ? v4u{0, 0, 0, 0} : rres[u][t][hh];  // ring slot ch & 3 (no residual with DSC)
              v4u pk;
#pragma unroll
              for (int k = 0; k < 4; ++k) {  // pairs of the lane's 8 couts, packed (common.h, epi): bitwise the scalar form
                epi::f32x2 v = epi::pair_of(acc1[t][2 * hh], acc1[t][2 * hh + 1], k) + epi::pair_of(bA, bB, k);
                if constexpr (!DSC) v += epi::bf2_f(rv[k]);
                pk[k] = epi::relu_bf2(v);
              }
              if (!(abl & 4))
                store_b128_guarded(pk, cur.y, ((pw + 16 * t) * CEXP + 8 * q) * 2, (ch * 64 + 32 * hh) * 2);
              yf[t][hh] = __builtin_bit_cast(bf16x8, pk);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if constexpr (NSLOT == 3) rslot = rslot == 2 ? 0 : rslot + 1;
    }
    // epilogue 2: + shift, ReLU, bf16 -> Z
#pragma unroll
    for (int t = 0; t < NPT; ++t)
#pragma unroll
      for (int g = 0; g < G2; ++g)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int c0 = 64 * g + 32 * hh + 8 * q;
          v4u pk;
#pragma unroll
          for (int k = 0; k < 4; ++k)
            pk[k] = epi::relu_bf2(epi::pair_of(acc2[t][g][2 * hh], acc2[t][g][2 * hh + 1], k) +
                                  (epi::f32x2){b1s[c0 + 2 * k], b1s[c0 + 2 * k + 1]});
          if (!(abl & 32)) store_b128_guarded(pk, cur.z, ((pw + 16 * t) * C1 + 8 * q) * 2, (64 * g + 32 * hh) * 2);
        }
    cur = nxt;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (unused) chunk-0 prefetch has landed
}

#ifndef EOSV_PAIRW_CS
#define EOSV_PAIRW_CS 1
#endif

template <int CMID, int CEXP, int C1, int NPT, int DSC = 0>
static int launch_pairw(const Pair1x1Args& a, hipStream_t s) {
  constexpr bool CS = EOSV_PAIRW_CS;
  constexpr int TILE = PairW<CMID, CEXP, C1, NPT, DSC>::TILE;
  static const int occ = kernel_occupancy((const void*)pairw_bf16_kernel<CMID, CEXP, C1, NPT, DSC, CS>, 512);
  const long long nrounds = (a.M + TILE - 1) / TILE;
  if (a.plan) return record_launch(a.plan, nrounds, occ);
  const long long grid = std::min<long long>(nrounds, (long long)occ * device_cu_count());
#ifdef EOSV_PROFILING
  static const int abl = env_switch("EOSV_CONV_ABL", 0);
  static const int cs = env_switch("EOSV_PAIRW_CS", CS);  // A/B of the wait rule
  if (abl) {
    Pair1x1Args b = a;
    b.abl = abl;
    hipLaunchKernelGGL((pairw_bf16_kernel<CMID, CEXP, C1, NPT, DSC, CS, true>), dim3((unsigned)grid), dim3(512), 0, s, b);
  } else if (cs != CS) {
    hipLaunchKernelGGL((pairw_bf16_kernel<CMID, CEXP, C1, NPT, DSC, !CS>), dim3((unsigned)grid), dim3(512), 0, s, a);
  } else
#endif
  hipLaunchKernelGGL((pairw_bf16_kernel<CMID, CEXP, C1, NPT, DSC, CS>), dim3((unsigned)grid), dim3(512), 0, s, a);
  EOSV_LAUNCH_CHECK();
  return EOSV_OK;
}

// 16-pixel tiles per wave of the pair for this shape: NPT 2 (256-pixel rounds) for the stage-2 pair
// with C1 = 128 (r04: 1.45 -> 1.34 ms per launch), NPT 1 elsewhere.  r04 / r05: NPT 2 gave
// run-to-run different R50 / R101 features inside the backbone and was removed, cause unpinned.
// r06 pinned it: the r04 build of pairw_bf16_kernel<128, 512, 128, 2> -- and no NPT 1 instance --
// holds one Y store (buffer_store_dwordx4, SGPR soffset) directly followed by a v_add_f32 that
// rewrites one of its data VGPRs (tools/isa_scan.py on the r04 sources), the gfx950 store-data
// hazard hipcc does not pad (common.h, store_b128_guarded).  Whether the store has read its data
// by then depends on how busy the memory pipeline is, hence "only inside the backbone".  The
// stores go through the guard now and the library scan is clean.  EOSV_PAIRW_NPT2=0 (profiling
// build): NPT 1 everywhere.
#ifndef EOSV_PAIRW_NPT2_DEF
#define EOSV_PAIRW_NPT2_DEF 1  // release A/B: tools/build_variant.sh npt1 -DEOSV_PAIRW_NPT2_DEF=0
#endif
static int pairw_npt(int cmid, int c1, int cds) {
  static const int npt2 = env_switch("EOSV_PAIRW_NPT2", EOSV_PAIRW_NPT2_DEF);
  return npt2 && cmid == 128 && c1 == 128 && cds == 0 ? 2 : 1;
}

int pairw_tile(int cmid, int c1, int cds) { return 128 * pairw_npt(cmid, c1, cds); }

bool pairw_bf16_ok(int cmid, int cexp, int c1, int cds, long long M, long long cap_elems) {
  if (M <= 0) return false;
  // the tail round reads and writes whole tiles: x, res / y and z must hold the padded pixel count
  const long long tile = pairw_tile(cmid, c1, cds);
  const long long padded = (M + tile - 1) / tile * tile;
  if (padded * std::max(cmid, std::max(cexp, c1)) > cap_elems) return false;
  if (cds) return cmid == 128 && cexp == 512 && c1 == 128 && cds == 256;  // stage-2 block 0
  return (cmid == 128 && cexp == 512 && (c1 == 128 || c1 == 256)) || (cmid == 256 && cexp == 1024 && c1 == 256);
}

int launch_pairw_bf16(const Pair1x1Args& a, hipStream_t s) {
  if (!pairw_bf16_ok(a.cmid, a.cexp, a.c1, a.cds, a.M, a.cap_elems) || !a.x || !a.w3 || !a.b3 || !a.w1 || !a.b1 || !a.y || !a.z ||
      (a.cds ? (!a.x2 || a.res || a.Ho <= 0 || a.Wo <= 0 || a.H2 < 2 * a.Ho - 1 || a.W2 < 2 * a.Wo - 1) : (!a.res || a.x2)))
    return set_error("pairw_bf16: unsupported shape"), EOSV_ERR_UNSUPPORTED;
  if (a.cds) return launch_pairw<128, 512, 128, 1, 256>(a, s);
  if (a.cmid == 128 && a.c1 == 128)
    return pairw_npt(128, 128, 0) == 2 ? launch_pairw<128, 512, 128, 2>(a, s) : launch_pairw<128, 512, 128, 1>(a, s);
  if (a.cmid == 128) return launch_pairw<128, 512, 256, 1>(a, s);
  return launch_pairw<256, 1024, 256, 1>(a, s);
}

}  // namespace eosv
