// Launch / completion round-trip calibration (gfx950): what a small window (config 5,
// 2^16 edges) pays besides the fold itself. Per window, one tiny kernel then:
//   sync      hipStreamSynchronize
//   query     hipStreamQuery spin
//   flag      host spin on a host-mapped word the kernel stores (system scope)
//   two+sync  two back-to-back kernels, then hipStreamSynchronize
// Build: hipcc -O3 --offload-arch=gfx950 calib_launch.hip -o bin/calib_launch
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_tiny(unsigned long long* host_word, unsigned long long seq, int* scratch) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    scratch[0] += 1;
    if (host_word) __hip_atomic_store(host_word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  unsigned long long* hw = nullptr;
  CK(hipHostMalloc((void**)&hw, 64, hipHostMallocMapped | hipHostMallocCoherent));
  *hw = 0;
  unsigned long long* dw = nullptr;
  CK(hipHostGetDevicePointer((void**)&dw, hw, 0));
  int* scratch;
  CK(hipMalloc(&scratch, 256));
  const int iters = 2000;
  const char* names[] = {"sync", "query", "flag", "two+sync", "256blk+sync"};
  for (int mode = 0; mode < 5; ++mode) {
    std::vector<double> lat;
    for (int i = 0; i < iters; ++i) {
      const unsigned long long seq = (unsigned long long)mode * 1000000 + i + 1;
      const auto t0 = std::chrono::steady_clock::now();
      if (mode == 4)
        hipLaunchKernelGGL(k_tiny, dim3(256), dim3(256), 0, st, nullptr, seq, scratch);
      else
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, st, mode == 2 ? dw : nullptr, seq, scratch);
      if (mode == 3) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, st, nullptr, seq, scratch);
      if (mode == 0 || mode == 3 || mode == 4) {
        CK(hipStreamSynchronize(st));
      } else if (mode == 1) {
        while (hipStreamQuery(st) == hipErrorNotReady) {
        }
      } else {
        while (__atomic_load_n(hw, __ATOMIC_ACQUIRE) != seq) {
        }
      }
      lat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    if (mode == 2) CK(hipStreamSynchronize(st));
    std::sort(lat.begin() + 100, lat.end());
    const size_t m = lat.size() - 100;
    printf("%-12s p50 %6.2f us  p99 %6.2f us\n", names[mode], lat[100 + m / 2], lat[100 + m * 99 / 100]);
  }
  return 0;
}
