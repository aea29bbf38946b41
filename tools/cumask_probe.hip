// Dev tool (not shipped): which CUs a CU-masked stream's workgroups land on.
// Build: hipcc -O3 --offload-arch=gfx950 cumask_probe.hip -o cumask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

__global__ void k_where(unsigned* out) {
  if (threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
    const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));
    out[blockIdx.x] = ((xcc & 0xf) << 16) | (((hw >> 13) & 7) << 8) | ((hw >> 8) & 15);
    __builtin_amdgcn_s_sleep(100);
  }
}

static void probe(const char* name, const std::vector<int>& bits) {
  std::vector<uint32_t> mask(8, 0);
  for (int b : bits) mask[b / 32] |= 1u << (b % 32);
  hipStream_t s;
  CK(hipExtStreamCreateWithCUMask(&s, 8, mask.data()));
  const int nb = 2048;
  unsigned* d;
  CK(hipMalloc(&d, nb * sizeof(unsigned)));
  hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, s, d);
  CK(hipStreamSynchronize(s));
  std::vector<unsigned> h(nb);
  CK(hipMemcpy(h.data(), d, nb * sizeof(unsigned), hipMemcpyDeviceToHost));
  std::set<unsigned> cus;
  for (unsigned v : h) cus.insert(v);
  printf("%-22s bits=%zu -> %zu distinct CUs:", name, bits.size(), cus.size());
  int k = 0;
  for (unsigned v : cus) {
    if (k++ < 24) printf(" x%u.se%u.cu%u", v >> 16, (v >> 8) & 0xff, v & 0xff);
  }
  printf("\n");
  CK(hipFree(d));
  CK(hipStreamDestroy(s));
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  printf("CUs %d\n", p.multiProcessorCount);
  std::vector<int> b;
  b = {0}; probe("bit0", b);
  b = {1}; probe("bit1", b);
  b = {0, 1, 2, 3, 4, 5, 6, 7}; probe("bits0-7", b);
  b = {0, 8, 16, 24, 32, 40, 48, 56}; probe("bits0,8,..56", b);
  b.clear(); for (int i = 0; i < 32; ++i) b.push_back(i); probe("bits0-31", b);
  b.clear(); for (int i = 32; i < 256; ++i) b.push_back(i); probe("bits32-255", b);
  b.clear(); for (int i = 0; i < 256; ++i) b.push_back(i); probe("all", b);
  return 0;
}
