// dev probe: (1) which XCD (HW_REG_XCC_ID) each block of a 1-D grid lands on; (2) which cache
// policies make a store from one CU visible to a polling load on another CU of the same XCD (and
// of another XCD), and the hand-off latency (s_memrealtime, 100 MHz).
// hipcc -O3 --offload-arch=gfx950 tools/xcd_probe.hip -o tools/xcd_probe && ./tools/xcd_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_where(unsigned* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));
}

// block pairs (p, p + D) ping-pong a counter R rounds. SA / LA: buffer cache-policy bits of the
// store / the polling load (1 = sc0, 2 = nt, 16 = sc1); INV: buffer_inv sc0 before each poll load
template <int SA, int LA, int INV>
__global__ void k_pingpong(unsigned long long* buf, unsigned long long* res, int R, int D) {
  const int b = blockIdx.x;
  const int pair = b % D, side = b / D;  // grid = 2·D
  if (threadIdx.x != 0) return;
  const auto r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 1 << 20, 0x00020000);
  const unsigned off = pair * 16 * 8;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long fails = 0;
  int i = 0;
  for (; i < R; ++i) {
    const unsigned long long want = 2 * i + side;
    unsigned spins = 0;
    for (;;) {
      asm volatile("" ::: "memory");
      if (INV) asm volatile("buffer_inv sc0" ::: "memory");
      const unsigned long long v =
          __builtin_bit_cast(unsigned long long, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, LA));
      if (v >= want) break;
      if (++spins > (1u << 16)) { ++fails; break; }
    }
    if (fails) break;
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, want + 1), r, off, 0, SA);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  res[3 * b] = t1 - t0;
  res[3 * b + 1] = fails;
  res[3 * b + 2] = i;
}

template <int SA, int LA, int INV>
void run(const char* name, unsigned long long* buf, unsigned long long* res, int D) {
  const int R = 2000;
  hipMemset(buf, 0, 1 << 20);
  hipLaunchKernelGGL((k_pingpong<SA, LA, INV>), dim3(2 * D), dim3(64), 0, 0, buf, res, R, D);
  hipDeviceSynchronize();
  std::vector<unsigned long long> hr(2 * D * 3);
  hipMemcpy(hr.data(), res, hr.size() * 8, hipMemcpyDeviceToHost);
  double ns = 0;
  int ok = 0, fails = 0;
  for (int b = 0; b < 2 * D; ++b) {
    fails += hr[3 * b + 1] ? 1 : 0;
    if (!hr[3 * b + 1]) { ns += 10.0 * hr[3 * b] / (2.0 * R); ++ok; }
  }
  printf("%-34s pairs %s-XCD: %2d/%2d blocks ok, %7.1f ns per one-way hand-off\n", name,
         D % 8 == 0 ? "same" : "cross", ok, 2 * D, ok ? ns / ok : 0.0);
}

int main() {
  const int nb = 32;
  unsigned* d;
  (void)hipMalloc(&d, nb * sizeof(unsigned));
  hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, 0, d);
  std::vector<unsigned> h(nb);
  (void)hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  printf("xcc of blocks 0..31:");
  for (int b = 0; b < nb; ++b) printf(" %u", h[b]);
  printf("\n");
  unsigned long long *buf, *res;
  (void)hipMalloc(&buf, 1 << 20);
  (void)hipMalloc(&res, 64 * 3 * 8);
  for (int D : {8, 1}) {  // D = 8: partner on the same XCD (round robin); D = 1: the next XCD
    run<0, 0, 0>("store plain, load plain", buf, res, D);
    run<1, 1, 0>("store sc0, load sc0", buf, res, D);
    run<0, 1, 1>("store plain, inv sc0 + load sc0", buf, res, D);
    run<0, 0, 1>("store plain, inv sc0 + load plain", buf, res, D);
    run<0, 16, 0>("store plain, load sc1", buf, res, D);
    run<16, 1, 0>("store sc1, load sc0", buf, res, D);
    run<16, 16, 0>("store sc1, load sc1", buf, res, D);
    run<17, 17, 0>("store sc0|sc1, load sc0|sc1", buf, res, D);
  }
  return 0;
}
