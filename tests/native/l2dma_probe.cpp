// Per-CU LDS-DMA (global_load_lds_dwordx4) throughput for the row-gather shape of the bf16
// implicit-GEMM A/B stages: a wave instruction moves 8 rows x 128 B, rows `stride` bytes
// apart (NHWC bf16: stride = 2 x Cin; 128 = a contiguous channel-chunk plane), `pieces`
// instructions per wave per stage, 8 waves per workgroup, one workgroup per CU.
//   sync  : issue a stage, s_waitcnt vmcnt(0), barrier (the conv K-loop with no MFMAs)
//   ring  : up to 3 stages in flight per wave (throughput, not latency)
// rows = distinct rows read (rows x 128 B of data, spread over rows x stride of address
// space); every workgroup walks all of them from its own start, so the data set is
// L2-resident when rows x 128 B is well under 4 MiB.
// Output: GB/s per CU and B/clk/CU at 2.1 GHz per (mode, stride, rows).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __attribute__((address_space(3))) void lds_t;

template <bool RING>
__global__ __launch_bounds__(512) void dma_rows(const char* __restrict__ buf, long long stride, int rows, int pieces,
                                                int iters, unsigned* sink) {
  __shared__ __attribute__((aligned(16))) char lds[2][8][8 * 1024];  // [slot][wave][piece KiB] (slots may be overwritten in flight: a rate probe)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r8 = lane >> 3, c = lane & 7;
  int q = (blockIdx.x * 977 + wid * 8 * pieces) % rows;
  for (int it = 0; it < iters; ++it) {
    const int slot = it & 1;
    for (int p = 0; p < pieces; ++p) {
      int row = q + p * 8 + r8;
      if (row >= rows) row -= rows;
      const char* src = buf + (long long)row * stride + ((c ^ (row & 7)) << 4);
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_t*)&lds[slot][wid][p * 1024], 16, 0, 0);
    }
    q += 8 * 8 * pieces;
    while (q >= rows) q -= rows;
    if (RING) {
      // keep (up to) 2 older stages in flight: wait for all but this and the previous stage
      if (pieces == 4)
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = lds[0][0][lane];
}

int main(int argc, char** argv) {
  const int iters = 2000;
  const int grid = argc > 1 ? atoi(argv[1]) : 256;
  const long long max_bytes = 1LL << 31;
  char* buf = nullptr;
  unsigned* sink = nullptr;
  if (hipMalloc(&buf, max_bytes) != hipSuccess || hipMalloc(&sink, 4096 * 4) != hipSuccess) return 2;
  if (hipMemset(buf, 1, max_bytes) != hipSuccess) return 2;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const long long strides[] = {128, 256, 512, 1024, 2048, 4096};
  const int rowss[] = {4096, 16384, 262144};
  printf("mode stride rows pieces  GB/s/CU  B/clk@2.1GHz\n");
  for (int mode = 0; mode < 2; ++mode)
    for (int pieces : {4, 8})
      for (int rows : rowss)
        for (long long s : strides) {
          if ((long long)rows * s > max_bytes) continue;
          for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(e0);
            if (mode)
              hipLaunchKernelGGL(dma_rows<true>, dim3(grid), dim3(512), 0, 0, buf, s, rows, pieces, iters, sink);
            else
              hipLaunchKernelGGL(dma_rows<false>, dim3(grid), dim3(512), 0, 0, buf, s, rows, pieces, iters, sink);
            (void)hipEventRecord(e1);
            if (hipEventSynchronize(e1) != hipSuccess) {
              printf("l2dma_probe: kernel failed\n");
              return 1;
            }
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep) {
              const double bytes = (double)grid * iters * 8 * pieces * 1024;
              const double per_cu = bytes / (ms * 1e-3) / (grid < 256 ? grid : 256) / 1e9;
              printf("%s %5lld %7d %d %8.1f %8.1f\n", mode ? "ring" : "sync", s, rows, pieces, per_cu, per_cu / 2.1);
            }
          }
        }
  (void)hipFree(buf);
  (void)hipFree(sink);
  return 0;
}
