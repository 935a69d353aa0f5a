// Probe: does global_load_lds (16 B per lane) accept sources that are only 4-B aligned?
// The dense-RGB stem (3 floats / 3 bf16 per pixel) needs that.  Each lane l loads 16 B
// from src + 4*(3*l + shift) bytes into LDS (lane-linear), the kernel copies LDS out, and
// the host compares against the expected floats.  Prints "dma_probe ok" or the mismatches.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void probe(const float* src, float* out, int shift) {
  __shared__ __attribute__((aligned(16))) float lds[64 * 4];
  const int lane = threadIdx.x;
  const float* p = src + 3 * lane + shift;
  __builtin_amdgcn_global_load_lds((const void*)p, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = 0; i < 4; ++i) out[lane * 4 + i] = lds[lane * 4 + i];
}

int main() {
  const int n = 64 * 3 + 16;
  std::vector<float> h(n);
  for (int i = 0; i < n; ++i) h[i] = (float)i + 0.5f;
  float *d, *o;
  if (hipMalloc(&d, n * 4) || hipMalloc(&o, 256 * 4)) return 2;
  hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
  int bad = 0;
  for (int shift = 0; shift < 4; ++shift) {
    hipMemset(o, 0, 256 * 4);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, o, shift);
    if (hipDeviceSynchronize() != hipSuccess) {
      printf("dma_probe: kernel failed at shift %d\n", shift);
      return 1;
    }
    std::vector<float> r(256);
    hipMemcpy(r.data(), o, 256 * 4, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l)
      for (int i = 0; i < 4; ++i) {
        const float want = h[3 * l + shift + i];
        if (r[l * 4 + i] != want) {
          if (bad < 8) printf("shift %d lane %d elt %d: got %g want %g\n", shift, l, i, r[l * 4 + i], want);
          ++bad;
        }
      }
  }
  printf(bad ? "dma_probe MISMATCH %d\n" : "dma_probe ok\n", bad);
  return bad ? 1 : 0;
}
