// Dev tool: host cost of a kernel launch (hipLaunchKernelGGL) with the filter kernels' 256-byte
// argument block, on a plain non-blocking stream and on a CU-masked stream (the chain / bulk
// streams of a <= 32-filter handle), with and without the GPU falling behind.
// Build: hipcc --offload-arch=gfx950 -O3 tools/launch_rate.hip -o tools/launch_rate
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

struct Big { double v[32]; };  // 256 bytes, as PassArgs

__global__ void k_empty(Big b, int* out) {
  if (threadIdx.x == 0 && b.v[0] == 12345.0) out[0] = 1;
}
__global__ void k_spin(int* out, long n) {  // keeps the queue busy for a while
  long s = 0;
  for (long i = 0; i < n; ++i) s += i ^ threadIdx.x;
  if (s == 42) out[0] = 2;
}

double rate(hipStream_t st, int* out, int n, bool busy) {
  Big b{};
  if (busy) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, st, out, 50000000L);
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_empty, dim3(4), dim3(256), 0, st, b, out);
  auto t1 = std::chrono::steady_clock::now();
  hipStreamSynchronize(st);
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
  int* out;
  hipMalloc(&out, 16);
  hipStream_t plain, masked;
  hipStreamCreateWithFlags(&plain, hipStreamNonBlocking);
  std::vector<uint32_t> m(8, 0);
  for (int b = 32; b < 256; ++b) m[b / 32] |= 1u << (b % 32);
  hipExtStreamCreateWithCUMask(&masked, 8, m.data());
  for (int rep = 0; rep < 2; ++rep) {
    printf("plain  idle %.2f us/launch, busy %.2f us/launch\n", rate(plain, out, 500, false),
           rate(plain, out, 500, true));
    printf("masked idle %.2f us/launch, busy %.2f us/launch\n", rate(masked, out, 500, false),
           rate(masked, out, 500, true));
  }
  return 0;
}
