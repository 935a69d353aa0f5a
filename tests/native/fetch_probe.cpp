// Calibration probe for the FETCH_SIZE counter (rocprofv3 --pmc FETCH_SIZE) on the access
// pattern of conv_f32_dma_kernel: global_load_lds of 16 B per lane in 64-B row pieces
// (BK = 16 floats), the 4 pieces of a 256-B pixel row read by 4 different instructions.
// Each kernel reads every byte of a 2 GiB buffer exactly once (beyond the 256 MiB
// Infinity Cache), so FETCH_SIZE x 1024 / 2 GiB is the counter's scale for that pattern:
//   wide      : each wave instruction reads 1 KiB contiguous (the guide's calibrated case)
//   piece<S>  : 16 rows of stride S bytes per instruction, 64 B of each row; instruction i of
//               a group reads piece i of the same 16 rows (S = 128, 256, 512: Cin 32/64/128)
// Run: rocprofv3 --pmc FETCH_SIZE -- tests/native/fetch_probe   (the kernel names tell which)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((address_space(3))) void lds_t;

__device__ __forceinline__ void dma16(const char* src, lds_t* dst) {
  __builtin_amdgcn_global_load_lds((const void*)src, dst, 16, 0, 0);
}

__global__ __launch_bounds__(256) void fetch_wide(const char* buf, long long bytes) {
  __shared__ __attribute__((aligned(16))) char lds[4 * 1024];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  lds_t* dst = (lds_t*)(lds + wid * 1024);
  const long long nunits = bytes / 1024;
  for (long long u = (long long)blockIdx.x * 4 + wid; u < nunits; u += (long long)gridDim.x * 4)
    dma16(buf + u * 1024 + lane * 16, dst);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int S>
__global__ __launch_bounds__(256) void fetch_piece(const char* buf, long long bytes) {
  __shared__ __attribute__((aligned(16))) char lds[4 * 1024];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  lds_t* dst = (lds_t*)(lds + wid * 1024);
  constexpr int GROUP = 16 * S;  // 16 rows of S bytes
  const long long ngroups = bytes / GROUP;
  const int row = lane >> 2, chunk = lane & 3;
  for (long long g = (long long)blockIdx.x * 4 + wid; g < ngroups; g += (long long)gridDim.x * 4) {
    const char* base = buf + g * GROUP + row * S + chunk * 16;
#pragma unroll
    for (int i = 0; i < S / 64; ++i) dma16(base + i * 64, dst);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int main() {
  const long long bytes = 2LL << 30;
  char* buf = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess) return 2;
  if (hipMemset(buf, 0, bytes) != hipSuccess) return 2;
  const dim3 grid(256 * 8), block(256);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(fetch_wide, grid, block, 0, 0, buf, bytes);
    hipLaunchKernelGGL(fetch_piece<128>, grid, block, 0, 0, buf, bytes);
    hipLaunchKernelGGL(fetch_piece<256>, grid, block, 0, 0, buf, bytes);
    hipLaunchKernelGGL(fetch_piece<512>, grid, block, 0, 0, buf, bytes);
  }
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("fetch_probe: kernel failed\n");
    return 1;
  }
  printf("fetch_probe ok: %lld bytes read once per dispatch\n", bytes);
  (void)hipFree(buf);
  return 0;
}
