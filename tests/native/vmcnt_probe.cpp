// Does `s_waitcnt vmcnt(K)` -- K = the number of vector-memory ops a wave issued after its
// LDS-DMA pieces -- guarantee that those pieces have landed in LDS, whatever the younger ops are?
// (The persistent kernels' rings rely on it: pairw_bf16.hip, conv_rows_*.hip, the stems.)
//
// Every iteration each wave LDS-DMAs P 1-KiB pieces of a 1 GiB source (streamed, so mostly HBM
// misses) into its own LDS region, then issues K younger ops of one kind, waits vmcnt(K), meets
// the other waves at a barrier, and every lane checks 16 B of every wave's region against the
// source's known contents (src[i] = hash(i)).  Mismatches are counted per kind:
//   0 none (vmcnt(0))            1 K VGPR loads of an L2-hot word    2 K stores to a scratch line
//   3 K stores out of range (empty buffer record: dropped)           4 K more LDS-DMA pieces
//   5 K VGPR loads out of range (empty record)
// usage: vmcnt_probe [iterations]   (prints one line per kind; exit 1 if kind 0 or 4 mismatches)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                      \
      exit(2);                                                                    \
    }                                                                             \
  } while (0)

constexpr int P = 6;        // DMA pieces per wave per iteration
constexpr int K = 4;        // younger ops
constexpr int NW = 4;       // waves per workgroup
constexpr long long SRC_WORDS = 1LL << 28;  // 1 GiB of u32

__device__ __host__ inline unsigned hsh(unsigned i) {
  i ^= i >> 16; i *= 0x7feb352dU; i ^= i >> 15; i *= 0x846ca68bU; i ^= i >> 16;
  return i;
}

__global__ void fill(unsigned* s, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    s[i] = hsh((unsigned)i);
}

template <int KIND>
__global__ __launch_bounds__(64 * NW) void probe(const unsigned* src, unsigned* hot, unsigned* scratch, int iters,
                                                 unsigned long long* bad) {
  __shared__ __attribute__((aligned(16))) unsigned lds[NW * (P + K) * 256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const __amdgpu_buffer_rsrc_t empty = __builtin_amdgcn_make_buffer_rsrc(scratch, (short)0, 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(scratch, (short)0, 1 << 20, 0x00020000);
  const unsigned lds0 = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) unsigned*)lds;
  unsigned nbad = 0, sink = 0;
  for (int it = 0; it < iters; ++it) {
    // this wave's pieces: different lines every iteration and workgroup
    const long long base = (((long long)it * gridDim.x + blockIdx.x) * NW + w) * (P + K) * 256 % (SRC_WORDS - 4096);
#pragma unroll
    for (int p = 0; p < P; ++p)
      __builtin_amdgcn_global_load_lds(src + base + p * 256 + lane * 4,
                                       (__attribute__((address_space(3))) void*)(lds + (w * P + p) * 256), 16, 0, 0);
    unsigned v[K];
    // the younger ops (inline asm / builtins whose results nothing uses before the iteration's
    // final vmcnt(0): hipcc inserts no wait of its own between them and the check)
    if constexpr (KIND == 1 || KIND == 5) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if constexpr (KIND == 1)
          asm volatile("global_load_dword %0, %1, off" : "=v"(v[k]) : "v"(hot + k * 64 + lane) : "memory");
        else
          asm volatile("buffer_load_dword %0, %1, %2, 0 offen" : "=v"(v[k]) : "v"(threadIdx.x * 4 + k * 4096), "s"(empty) : "memory");
      }
    }
    if constexpr (KIND == 2 || KIND == 3) {
#pragma unroll
      for (int k = 0; k < K; ++k)
        __builtin_amdgcn_raw_buffer_store_b32(it + k, KIND == 2 ? sr : empty, (blockIdx.x * 256 + threadIdx.x) * 4 + k * 4096, 0, 0);
    }
    if constexpr (KIND == 4) {
#pragma unroll
      for (int k = 0; k < K; ++k)
        __builtin_amdgcn_global_load_lds(src + base + (P + k) * 256 + lane * 4,
                                         (__attribute__((address_space(3))) void*)(lds + (NW * P + w * K + k) * 256), 16, 0, 0);
    }
    if constexpr (KIND == 0)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(K) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // check every wave's first P pieces (inline-asm LDS reads: hipcc cannot see that they alias
    // the DMA and insert a wait of its own)
    for (int ww = 0; ww < NW; ++ww) {
      const long long b2 = (((long long)it * gridDim.x + blockIdx.x) * NW + ww) * (P + K) * 256 % (SRC_WORDS - 4096);
#pragma unroll
      for (int p = 0; p < P; ++p) {
        uint4 got;
        asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(got) : "v"(lds0 + ((ww * P + p) * 256 + lane * 4) * 4) : "memory");
        const unsigned i0 = (unsigned)(b2 + p * 256 + lane * 4);
        nbad += (got.x != hsh(i0)) + (got.y != hsh(i0 + 1)) + (got.z != hsh(i0 + 2)) + (got.w != hsh(i0 + 3));
      }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if constexpr (KIND == 1 || KIND == 5) {
#pragma unroll
      for (int k = 0; k < K; ++k) sink += v[k];
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  if (nbad) atomicAdd(bad + KIND, (unsigned long long)nbad);
  if (sink == 0x12345678u) hot[1000] = sink;  // keeps the loads
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  unsigned *src, *hot, *scratch;
  unsigned long long* bad;
  CHECK(hipMalloc(&src, SRC_WORDS * 4));
  CHECK(hipMalloc(&hot, 1 << 16));
  CHECK(hipMalloc(&scratch, (1 << 20) + 4096 * 8));
  CHECK(hipMalloc(&bad, 8 * sizeof(unsigned long long)));
  CHECK(hipMemset(hot, 0, 1 << 16));
  CHECK(hipMemset(bad, 0, 8 * sizeof(unsigned long long)));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, src, SRC_WORDS);
  CHECK(hipDeviceSynchronize());
  const dim3 grid(256 * 4), block(64 * NW);
  hipLaunchKernelGGL(probe<0>, grid, block, 0, 0, src, hot, scratch, iters, bad);
  hipLaunchKernelGGL(probe<1>, grid, block, 0, 0, src, hot, scratch, iters, bad);
  hipLaunchKernelGGL(probe<2>, grid, block, 0, 0, src, hot, scratch, iters, bad);
  hipLaunchKernelGGL(probe<3>, grid, block, 0, 0, src, hot, scratch, iters, bad);
  hipLaunchKernelGGL(probe<4>, grid, block, 0, 0, src, hot, scratch, iters, bad);
  hipLaunchKernelGGL(probe<5>, grid, block, 0, 0, src, hot, scratch, iters, bad);
  CHECK(hipDeviceSynchronize());
  unsigned long long h[8];
  CHECK(hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost));
  const char* names[6] = {"none, vmcnt(0)", "VGPR loads (L2-hot)", "stores", "out-of-range stores", "LDS-DMA pieces",
                          "out-of-range loads"};
  const double checked = (double)iters * grid.x * 64 * NW * NW * P * 4;
  for (int k = 0; k < 6; ++k)
    printf("younger ops: %-22s mismatching words %llu of %.3g\n", names[k], h[k], checked);
  return (h[0] || h[4]) ? 1 : 0;
}
