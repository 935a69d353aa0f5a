// Microbenchmark: f32 MFMA issue rate under the conv kernel's inner-loop shapes.
//   mode 0: MFMA only (operands in registers), 4 independent 32x32 accumulators
//   mode 1: + ds_read_b128 fragment reads per 16 MFMAs (as in conv_f32)
//   mode 2: + one __syncthreads per 64 MFMAs
//   mode 3: 16x16x4 f32 MFMA, 4 accumulators, registers only
// Prints TF/s for 1..4 blocks of 256 threads per CU.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ __launch_bounds__(256) void probe(float* out, int iters, const float* src, long long src_floats) {
  __shared__ __attribute__((aligned(16))) float lds[128 * 36 * 2];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 128 * 36 * 2; i += 256) lds[i] = (float)(i % 7) * 0.125f;
  __syncthreads();
  f32x16 acc[4];
  for (int t = 0; t < 4; ++t)
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  f32x4 acc4[4];
  for (int t = 0; t < 4; ++t) acc4[t] = f32x4{0, 0, 0, 0};
  f32x4 a0 = {1.f, 2.f, 3.f, 4.f}, a1 = {0.5f, 0.25f, 1.5f, 2.5f};
  f32x4 b0 = {1.f, 1.f, 2.f, 2.f}, b1 = {3.f, 0.5f, 0.75f, 1.f};
  const int r = lane & 31, h = lane >> 5;
  f32x4 ld[8];
  long long cursor = ((long long)blockIdx.x * 4096 + (threadIdx.x >> 3) * 32 + (threadIdx.x & 7) * 4) % src_floats;
  for (int it = 0; it < iters; ++it) {
    if (MODE >= 4) {  // 8 x 16-B loads per lane per iteration (rows of 128 B), like one conv K-step
#pragma unroll
      for (int j = 0; j < 8; ++j) ld[j] = *(const f32x4*)(src + (cursor + j * 1024) % src_floats);
      cursor = (cursor + 8 * 1024 * 37) % src_floats;
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (MODE == 1 || MODE == 2 || MODE >= 4) {
        a0 = *(const f32x4*)(lds + r * 36 + 16 * h + 4 * g);
        a1 = *(const f32x4*)(lds + (r + 32) * 36 + 16 * h + 4 * g);
        b0 = *(const f32x4*)(lds + 128 * 36 + r * 36 + 16 * h + 4 * g);
        b1 = *(const f32x4*)(lds + 128 * 36 + (r + 32) * 36 + 16 * h + 4 * g);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (MODE == 3) {
          acc4[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s], b0[s], acc4[0], 0, 0, 0);
          acc4[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s], b1[s], acc4[1], 0, 0, 0);
          acc4[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[s], b0[s], acc4[2], 0, 0, 0);
          acc4[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[s], b1[s], acc4[3], 0, 0, 0);
        } else {
          acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b0[s], acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b1[s], acc[1], 0, 0, 0);
          acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b0[s], acc[2], 0, 0, 0);
          acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b1[s], acc[3], 0, 0, 0);
        }
      }
    }
    if (MODE >= 4) {
#pragma unroll
      for (int j = 0; j < 8; ++j) *(f32x4*)(lds + 128 * 36 + (threadIdx.x & 127) * 36 + (j & 3) * 4) = ld[j];
    }
    if (MODE == 2 || MODE >= 4) __syncthreads();
  }
  float s = 0;
  for (int t = 0; t < 4; ++t) {
    for (int q = 0; q < 16; ++q) s += acc[t][q];
    for (int q = 0; q < 4; ++q) s += acc4[t][q];
  }
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

static float* g_src;
static long long g_src_floats;

template <int MODE>
static void run(int per_cu) {
  const int blocks = 256 * per_cu, iters = 2000;
  float* out;
  hipMalloc(&out, blocks * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  probe<MODE><<<blocks, 256>>>(out, 10, g_src, MODE == 5 ? g_src_floats : (1 << 20));
  hipDeviceSynchronize();
  hipEventRecord(e0);
  probe<MODE><<<blocks, 256>>>(out, iters, g_src, MODE == 5 ? g_src_floats : (1 << 20));
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops_per_mfma = MODE == 3 ? 2.0 * 16 * 16 * 4 : 2.0 * 32 * 32 * 2;
  const double flops = (double)blocks * 4 /*waves*/ * iters * 64 /*mfma per iter*/ * flops_per_mfma;
  printf("mode %d  blocks/CU %d  %.1f TF/s\n", MODE, per_cu, flops / ms / 1e9);
  hipFree(out);
}

int main() {
  g_src_floats = 1ll << 28;  // 1 GiB
  hipMalloc(&g_src, g_src_floats * 4);
  hipMemset(g_src, 0, g_src_floats * 4);
  for (int pc = 1; pc <= 4; ++pc) {
    run<0>(pc);
    run<2>(pc);
    run<4>(pc);  // + loads from a 4 MiB (L2-resident) buffer
    run<5>(pc);  // + loads streaming a 1 GiB buffer
  }
  return 0;
}
