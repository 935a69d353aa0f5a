// Microbenchmark: cycles per v_mfma_f32_16x16x32_bf16 in the f32x3 stage-1 row kernel's k-loop
// shape (conv_rows_x3.hip): one wave per SIMD, 21 MFMAs per k-step (w_hi.x_hi, w_lo.x_hi,
// w_hi.x_lo over 7 pixel tiles), 18 k-steps per strip, random bf16 operands.
//   mode 0: 36 weight fragments (w_hi, w_lo per k-step) held in registers, pixel fragments fixed
//   mode 1: 2 weight fragments reused every k-step (low register pressure), pixel fragments fixed
//   mode 2: mode 0 + the 14 ds_read_b128 pixel-fragment reads per k-step, double-buffered
//   mode 3: mode 1 + the ds_reads of mode 2
// Cycles from s_memtime (shader clock) around the loop, per wave; clock = cycles / s_memrealtime.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned hash(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352d;
  x ^= x >> 15;
  x *= 0x846ca68b;
  return x ^ (x >> 16);
}

template <int MODE>
__global__ __launch_bounds__(256) void probe(float* out, long long* cyc, int strips) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[2][16 * 1024];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < 2 * 16 * 1024; i += 256) (&lds[0][0])[i] = (unsigned short)(0x3c00 + (hash(i) & 0x3ff));
  bf16x8 w[MODE == 0 || MODE == 2 ? 36 : 2];
  constexpr int NW = MODE == 0 || MODE == 2 ? 36 : 2;
#pragma unroll
  for (int t = 0; t < NW; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) w[t][e] = (__bf16)((float)(hash(lane * 977 + t * 31 + e + blockIdx.x) & 255) / 256.f - 0.5f);
  bf16x8 xh[2][7], xl[2][7];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int i = 0; i < 7; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xh[b][i][e] = (__bf16)((float)(hash(lane * 131 + i * 7 + e) & 255) / 256.f - 0.5f);
        xl[b][i][e] = (__bf16)((float)(hash(lane * 71 + i * 5 + e) & 255) / 65536.f);
      }
  __syncthreads();
  f32x4 acc[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) unsigned short*)&lds[0][0];
  const long long t0 = __builtin_amdgcn_s_memtime();
  const long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int s = 0; s < strips; ++s) {
#pragma unroll
    for (int t = 0; t < 18; ++t) {
      const int b = t & 1;
      if (MODE >= 2 && t + 1 < 18) {
#pragma unroll
        for (int i = 0; i < 7; ++i) {
          const unsigned a = base + (((lane + i * 64 + t * 448) * 16) & 0x7fff);
          asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16384"
                       : "=v"(xh[b ^ 1][i]), "=v"(xl[b ^ 1][i]) : "v"(a));
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      const bf16x8 wh = w[NW == 36 ? t : 0], wl = w[NW == 36 ? 18 + t : 1];
#pragma unroll
      for (int i = 0; i < 7; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xh[b][i], acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 7; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, xh[b][i], acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 7; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xl[b][i], acc[i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (MODE >= 2) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  const long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 7; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + tid] = s;
  if (lane == 0) {
    cyc[(blockIdx.x * 4 + (tid >> 6)) * 2] = t1 - t0;
    cyc[(blockIdx.x * 4 + (tid >> 6)) * 2 + 1] = r1 - r0;
  }
}

template <int MODE>
static void run(int ncu) {
  const int strips = 200;
  float* out;
  long long* cyc;
  hipMalloc(&out, ncu * 256 * 4);
  hipMalloc(&cyc, ncu * 8 * 8);
  hipLaunchKernelGGL(probe<MODE>, dim3(ncu), dim3(256), 0, 0, out, cyc, 10);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(probe<MODE>, dim3(ncu), dim3(256), 0, 0, out, cyc, strips);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> c(ncu * 8);
  hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
  double cs = 0, rs = 0;
  for (int i = 0; i < ncu * 4; ++i) cs += c[2 * i], rs += c[2 * i + 1];
  const double mfmas = (double)strips * 18 * 21;
  const double cpm = cs / (ncu * 4) / mfmas;
  const double ghz = cs / rs * 0.1;
  const double tf = (double)ncu * 4 * mfmas * 2 * 16 * 16 * 32 / (ms * 1e-3) / 1e12;
  printf("mode %d: %.1f cycles per MFMA, clock %.2f GHz, %.0f TF/s (%.3f ms)\n", MODE, cpm, ghz, tf, ms);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  int n = 0;
  hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, 0);
  run<0>(n);
  run<1>(n);
  run<2>(n);
  run<3>(n);
  run<0>(n);
  return 0;
}
