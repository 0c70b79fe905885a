// Cross-queue hand-off latency on one device: a kernel on stream A spins ~T us and stamps its
// end (wall clock, 100 MHz); a one-wave kernel on stream B, ordered behind it by one of the
// hand-off forms below, stamps its start. Prints the median / p90 gap in us per form.
//   event  : hipEventRecord(A) + hipStreamWaitEvent(B)
//   value  : hipStreamWriteValue64(A) + hipStreamWaitValue64(B, >=)
//   same   : both kernels on stream A (the in-queue dispatch gap, for scale)
// Build: hipcc --offload-arch=gfx950 -O2 tools/xq_probe.hip -o tools/xq_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

__global__ void k_spin(unsigned long long* stamp, unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  unsigned long long t = t0;
  while (t - t0 < ticks) t = wall_clock64();  // bounded: ticks of a 100 MHz clock
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) stamp[0] = wall_clock64();
}

__global__ void k_stamp(unsigned long long* stamp) {
  if (threadIdx.x == 0) stamp[1] = wall_clock64();
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 200;
  const unsigned long long ticks = 2000;  // 20 us of spinning in A
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  unsigned long long* st = nullptr;
  CK(hipMalloc(&st, 2 * sizeof(unsigned long long)));
  void* sig = nullptr;
  CK(hipExtMallocWithFlags(&sig, 8, hipMallocSignalMemory));  // (signal memory: 8 B per allocation)
  CK(hipMemset(sig, 0, 8));
  CK(hipDeviceSynchronize());
  const char* names[] = {"same", "event", "value"};
  unsigned long long seq = 0;
  for (int form = 0; form < 3; ++form) {
    std::vector<double> gaps;
    for (int r = 0; r < reps + 10; ++r) {
      hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), 0, a, st, ticks);
      hipStream_t sb = b;
      if (form == 0) {
        sb = a;
      } else if (form == 1) {
        CK(hipEventRecord(ev, a));
        CK(hipStreamWaitEvent(b, ev, 0));
      } else {
        ++seq;
        CK(hipStreamWriteValue64(a, sig, seq, 0));
        CK(hipStreamWaitValue64(b, sig, seq, hipStreamWaitValueGte, ~0ull));
      }
      hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, sb, st);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      unsigned long long h[2];
      CK(hipMemcpy(h, st, sizeof h, hipMemcpyDeviceToHost));
      if (r >= 10) gaps.push_back(((double)(long long)(h[1] - h[0])) / 100.0);
    }
    std::sort(gaps.begin(), gaps.end());
    std::printf("%-6s gap us: p10 %.2f  median %.2f  p90 %.2f  (n=%zu)\n", names[form], gaps[gaps.size() / 10],
                gaps[gaps.size() / 2], gaps[gaps.size() * 9 / 10], gaps.size());
    std::fflush(stdout);
  }
  CK(hipFree(sig));
  CK(hipFree(st));
  return 0;
}
