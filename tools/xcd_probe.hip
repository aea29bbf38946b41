// dev probe: (1) which XCD (HW_REG_XCC_ID) and CU each block of a 1-D grid lands on; (2) whether a
// plain store from one CU is seen by a load with sc0 (or sc1) polling on another CU of the same
// XCD, and how long the hand-off takes (s_memrealtime, 100 MHz).
// hipcc -O3 --offload-arch=gfx950 tools/xcd_probe.hip -o tools/xcd_probe && ./tools/xcd_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_where(unsigned* out) {
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));
    out[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
  }
}

typedef __attribute__((address_space(1))) unsigned long long gu64;
template <int AUX>
__device__ unsigned long long ld(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(unsigned long long, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, AUX));
}

// block pairs (p, p + 8·S) ping-pong a counter R rounds: the even one stores v, the odd one polls
// until it sees v and stores v + 1, ... ; MODE 0: plain stores + sc0 loads, 1: agent stores + sc1
template <int MODE>
__global__ void k_pingpong(unsigned long long* buf, unsigned long long* res, int R, int S) {
  const int b = blockIdx.x;
  const int pair = b % (8 * S), side = b / (8 * S);  // side 0 or 1 (grid = 16·S)
  if (threadIdx.x != 0) return;
  unsigned long long* cell = buf + pair * 16;
  const auto r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 1 << 20, 0x00020000);
  const unsigned off = pair * 16 * 8;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long fails = 0;
  for (int i = 0; i < R; ++i) {
    const unsigned long long want = 2 * i + side;  // side 0 waits for even values
    unsigned spins = 0;
    for (;;) {
      const unsigned long long v = MODE == 0 ? ld<1>(r, off) : ld<16>(r, off);
      if (v >= want) break;
      if (++spins > (1u << 16)) { ++fails; break; }
    }
    if (fails) break;  // (a lost hand-off: stop, the partner times out as well)
    if (MODE == 0) __hip_atomic_store((gu64*)cell, want + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else __hip_atomic_store((gu64*)cell, want + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  res[2 * b] = t1 - t0;
  res[2 * b + 1] = fails;
}

int main() {
  const int nb = 64;
  unsigned* d;
  hipMalloc(&d, nb * 2 * sizeof(unsigned));
  hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, 0, d);
  std::vector<unsigned> h(nb * 2);
  hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  printf("block: xcc_id hw_id(cu=bits 8-11, sh 12, se 13-15)\n");
  for (int b = 0; b < nb; ++b) printf("%d:%u/%u%s", b, h[2 * b], (h[2 * b + 1] >> 8) & 15, b % 8 == 7 ? "\n" : "  ");
  const int S = 1, R = 2000;
  unsigned long long *buf, *res;
  hipMalloc(&buf, 1 << 20);
  hipMalloc(&res, 16 * S * 2 * 8);
  for (int mode = 0; mode < 2; ++mode) {
    hipMemset(buf, 0, 1 << 20);
    if (mode == 0) hipLaunchKernelGGL(k_pingpong<0>, dim3(16 * S), dim3(64), 0, 0, buf, res, R, S);
    else hipLaunchKernelGGL(k_pingpong<1>, dim3(16 * S), dim3(64), 0, 0, buf, res, R, S);
    hipDeviceSynchronize();
    std::vector<unsigned long long> hr(16 * S * 2);
    hipMemcpy(hr.data(), res, hr.size() * 8, hipMemcpyDeviceToHost);
    printf("mode %s: per block (ticks of 10 ns for %d round trips, fails):", mode == 0 ? "plain+sc0" : "agent+sc1", R);
    for (int b = 0; b < 16 * S; ++b) printf(" %d:%llu/%llu", b, hr[2 * b], hr[2 * b + 1]);
    printf("\n");
  }
  return 0;
}
