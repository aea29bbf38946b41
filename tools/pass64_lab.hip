// Dev tool (not shipped): the swarm's fp64 Σ pass (512 filters, N = 256: n = 515, 2.2 GB of Σ per
// message) A/B'd standalone against the product's k_sigma_pass<double, true> on the same buffers,
// outputs (Σ_out and the kRowsOut rows) compared bit for bit. Since round 4 the product is the
// symmetric pass (k_sym here is its prototype; the ablations are of the full pass's tile).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include -I../ekf-slam_amd/csrc pass64_lab.hip -o pass64_lab
#include "../ekf-slam_amd/csrc/ekf_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace ekfslam;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

// the product's wide tile with ablations: MODE 1 = no MFMA (a VALU product keeps the operands
// live), 2 = no operand loads (constants), both = Σ_in → Σ_out only
enum { kNoMfma = 1, kNoOps = 2 };
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_ablate(PassArgs<double> A, int tcols, int xcd_b, int nf) {
  const int L = blockIdx.x, j = L >> 3;
  const int fb = (L & 7) + 8 * (j / xcd_b), bx = j % xcd_b;
  if (fb >= nf) return;
  const MsgDesc& d = A.desc[fb];
  const int lane = threadIdx.x & 63;
  const int trows = (A.n + 31) / 32;
  const int t = __builtin_amdgcn_readfirstlane(bx * 4 + (threadIdx.x >> 6));
  if (t >= trows * tcols || !(d.flags & kActive)) return;
  const int R0 = (t / tcols) * 32, C0 = (t % tcols) * 64;
  const int f = A.f0 + fb;
  const int n = A.n, ld = A.ld, ldk = A.ldk;
  const double* Sin = A.sig[d.parity] + f * A.sig_stride;
  double* Sout = A.sig[d.parity ^ 1] + f * A.sig_stride;
  const double* kc = A.kcat + f * A.km_stride;
  const double* mc = A.mcat + f * A.km_stride;
  constexpr int TJ = 4;
  const int kr = lane >> 4, kcol = lane & 15;
  const size_t pbase = static_cast<size_t>(R0) * ld;
  const unsigned sbytes = static_cast<unsigned>(min(n - R0, 32)) * ld * 8u;
  const unsigned kbytes = static_cast<unsigned>(kMaxKW) * ldk * 8u;
  const auto rin = buf_rsrc(Sin + pbase, sbytes), rout = buf_rsrc(Sout + pbase, sbytes);
  const auto rk = buf_rsrc(kc, kbytes), rm = buf_rsrc(mc, kbytes);
  double a[2][9], b[TJ][9], sv[2][TJ][4];
  const unsigned ko = static_cast<unsigned>(kr * ldk + R0 + kcol) * 8u;
  unsigned mo[TJ], so[TJ];
  const unsigned rstride = static_cast<unsigned>(ld) * 8u;
#pragma unroll
  for (int tj = 0; tj < TJ; ++tj) {
    const int col = C0 + 16 * tj + kcol;
    mo[tj] = static_cast<unsigned>(kr * ldk + min(col, n - 1)) * 8u;
    so[tj] = col < n ? static_cast<unsigned>(kr * ld + col) * 8u : kOOB;
  }
  const unsigned kstep = 4u * ldk * 8u;
  if (MODE & kNoOps) {
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      a[0][s] = 1e-3 * (s + 1);
      a[1][s] = 2e-3 * (s + 1);
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) b[tj][s] = 1e-3 * (tj + s);
    }
  } else {
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      a[0][s] = ld_f64(rk, ko, s * kstep);
      a[1][s] = ld_f64(rk, ko + 16 * 8, s * kstep);
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) b[tj][s] = ld_f64(rm, mo[tj], s * kstep);
    }
  }
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sv[ti][tj][r] = __builtin_bit_cast(
            double, __builtin_amdgcn_raw_buffer_load_b64(rin, so[tj] + (16 * ti + 4 * r) * rstride, 0, 2));
  d4 acc[2][TJ];
  if (MODE & kNoMfma) {
    double s0 = 0.0;
#pragma unroll
    for (int s = 0; s < 9; ++s) s0 += a[0][s] * a[1][s] + b[0][s] * b[1][s] + b[2][s] * b[3][s];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) acc[ti][tj] = d4{s0, s0, s0, s0};
  } else {
    const int kw = ((2 + 2 * d.m + 3) / 4) * 4;
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) acc[ti][tj] = d4{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      const bool live = 4 * s < kw;
#pragma unroll
      for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < TJ; ++tj)
          acc[ti][tj] = mfma_f64(live ? a[ti][s] : 0.0, live ? b[tj][s] : 0.0, acc[ti][tj]);
    }
  }
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double v = sv[ti][tj][r] - acc[ti][tj][r];
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), rout,
                                              so[tj] + (16 * ti + 4 * r) * rstride, 0, 2);
      }
}


// ---- measured, not kept (profiles/r4/stream_pass_notkept): 529 µs against the tile grid's 475 ----
// ---- swarm Σ pass (fp64, ≥ 16 filters): persistent, Σ_in double-buffered through LDS-DMA ---------
// The tile grid's waves (2 per SIMD, registers) each load, multiply, then store: with 2.2 GB of Σ
// streaming through HBM per message the MFMA phases leave the memory system idle (0.56 of the
// float4 copy's rate standalone). Here each wave keeps its NEXT tile's Σ_in (LDS-DMA) and operands
// (registers freed k-step by k-step behind the MFMAs) in flight while it multiplies and stores the
// current one. One workgroup of 4 waves per CU (128 KiB of LDS: two 16 KiB 32 × 64 images per
// wave); XCD x (blocks L ≡ x mod 8) walks the tiles of filters x, x+8, … in order, wave by wave
// (the filter's Kcat / Mcat stay in that XCD's L2). Same tile (32 × 64, SigmaTile64<4>), same MFMA
// order: bit-identical to k_sigma_pass. Per tile t (next tn):
//   1. wait for t's operands (a use of the newest one: the compiler's count, exact — the DMA below is
//      issued after it; t's Σ_in DMA is older, so complete too)
//   2. Σ_in(tn) → the other LDS image: 16 buffer_load_dwordx4 … lds in inline asm (invisible to the
//      compiler's wait counting: a visible LDS-DMA makes it wait vmcnt(0) at every later load use)
//   3. the 72 MFMAs of t, tn's operand loads issued step by step behind them (registers freed)
//   4. Σ_in(t) from LDS in the MFMA layout, Σ_out = Σ_in − K·M (+ Q̄), stores (+ kRowsOut rows)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
struct StreamTile {
  int fb, R0, C0, par, kw, flags;
  bool live;
};
__device__ __forceinline__ StreamTile stream_tile(const PassArgs<double>& A, int x, int t, int T,
                                                  int tpf, int tcols) {
  StreamTile s;
  s.live = t < T;
  const int tt = s.live ? t : 0, k = tt / tpf, r = tt - k * tpf;
  s.fb = x + 8 * k;
  // (through the constant address space: scalar loads, no vmcnt)
  const __attribute__((address_space(4))) MsgDesc& d = ((const __attribute__((address_space(4))) MsgDesc*)A.desc)[s.fb];
  s.flags = s.live ? d.flags : 0;
  s.live = s.live && (s.flags & kActive);
  s.par = d.parity;
  s.kw = ((2 + ((s.flags & kJoseph) ? 4 : 2) * d.m + 3) / 4) * 4;
  s.R0 = (r / tcols) * 32;
  s.C0 = (r % tcols) * 64;
  return s;
}
__device__ __forceinline__ void stream_dma(const PassArgs<double>& A, const StreamTile& s,
                                           unsigned lds_base, int lane) {
  const int n = A.n, ld = A.ld;
  const size_t fo = static_cast<size_t>(A.f0 + s.fb) * A.sig_stride;
  const double* S = A.sig[s.par] + fo + static_cast<size_t>(s.R0) * ld;
  const unsigned bytes = s.live ? static_cast<unsigned>(min(n - s.R0, 32)) * ld * 8u : 0u;
  const auto r = buf_rsrc(S, bytes);
  const int c = s.C0 + 2 * (lane & 31);
  const unsigned vo = c < n ? static_cast<unsigned>((lane >> 5) * ld + c) * 8u : kOOB;
  const unsigned rs = 2u * ld * 8u;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen nt lds"
                 : : "s"(__builtin_amdgcn_readfirstlane(lds_base + 1024u * i)), "v"(vo), "s"(r),
                     "s"(__builtin_amdgcn_readfirstlane(rs * i)) : "memory");
}
__device__ __forceinline__ void stream_ops_step(const PassArgs<double>& A, const StreamTile& s, int st,
                                                double (&a)[2][9], double (&b)[4][9], int lane) {
  const int n = A.n, ldk = A.ldk;
  const size_t fo = static_cast<size_t>(A.f0 + s.fb) * A.km_stride;
  const unsigned kbytes = s.live ? static_cast<unsigned>(kMaxKW) * ldk * 8u : 0u;
  const auto rk = buf_rsrc(A.kcat + fo, kbytes), rm = buf_rsrc(A.mcat + fo, kbytes);
  const int kr = lane >> 4, kcol = lane & 15;
  const unsigned ko = static_cast<unsigned>(kr * ldk + s.R0 + kcol) * 8u;
  const unsigned kstep = 4u * ldk * 8u;
  a[0][st] = ld_f64(rk, ko, st * kstep);
  a[1][st] = ld_f64(rk, ko + 16 * 8, st * kstep);
#pragma unroll
  for (int tj = 0; tj < 4; ++tj) {
    const unsigned mo = static_cast<unsigned>(kr * ldk + min(s.C0 + 16 * tj + kcol, n - 1)) * 8u;
    b[tj][st] = ld_f64(rm, mo, st * kstep);
  }
}
__global__ __launch_bounds__(256) void k_sigma_stream(PassArgs<double> A, int tcols, int tpf, int nf) {
  __shared__ double img[4][2][32 * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int x = blockIdx.x & 7;
  const int nfx = (nf - x + 7) / 8;  // filters x, x+8, … < nf
  const int T = nfx * tpf;
  const int W = static_cast<int>(gridDim.x >> 3) * 4;
  int t = __builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x >> 3) * 4 + wv);
  if (t >= T) return;
  typedef __attribute__((address_space(3))) double lds_d;
  const unsigned base0 = static_cast<unsigned>(reinterpret_cast<size_t>((lds_d*)&img[wv][0][0]));
  const unsigned base1 = static_cast<unsigned>(reinterpret_cast<size_t>((lds_d*)&img[wv][1][0]));
  const int n = A.n, ld = A.ld, ldk = A.ldk;
  const int kr = lane >> 4, kcol = lane & 15;
  const double q = A.q;
  StreamTile cur = stream_tile(A, x, t, T, tpf, tcols);
  double a[2][9], b[4][9];
  stream_dma(A, cur, base0, lane);
#pragma unroll
  for (int st = 0; st < 9; ++st) stream_ops_step(A, cur, st, a, b, lane);
  {  // 48 out-of-range stores: the loop's entry looks like its back edge to the compiler's wait
     // counting (48 stores behind the operands), so the first wait is vmcnt(48) there as well
    const auto none = buf_rsrc(A.rows, 0u);
#pragma unroll
    for (int i = 0; i < 48; ++i) __builtin_amdgcn_raw_buffer_store_b64(u2v{0u, 0u}, none, kOOB + 8u * i, 0, 0);
  }
  const __attribute__((address_space(4))) MsgDesc* cdesc = (const __attribute__((address_space(4))) MsgDesc*)A.desc;
  int buf = 0;
  for (;;) {
    const int tn = t + W;
    const StreamTile nxt = stream_tile(A, x, tn, T, tpf, tcols);
    // 1. t's operands (and, older, its Σ_in DMA) have landed
    asm volatile("" : : "v"(a[0][0]), "v"(a[0][1]), "v"(a[0][2]), "v"(a[0][3]), "v"(a[0][4]), "v"(a[0][5]),
                 "v"(a[0][6]), "v"(a[0][7]), "v"(a[0][8]), "v"(a[1][0]), "v"(a[1][1]), "v"(a[1][2]),
                 "v"(a[1][3]), "v"(a[1][4]), "v"(a[1][5]), "v"(a[1][6]), "v"(a[1][7]), "v"(a[1][8]));
#pragma unroll
    for (int tj = 0; tj < 4; ++tj)
      asm volatile("" : : "v"(b[tj][0]), "v"(b[tj][1]), "v"(b[tj][2]), "v"(b[tj][3]), "v"(b[tj][4]),
                   "v"(b[tj][5]), "v"(b[tj][6]), "v"(b[tj][7]), "v"(b[tj][8]));
    __builtin_amdgcn_sched_barrier(0);
    // 2. tn's Σ_in into the other image (a dummy, out of range, past the last tile)
    stream_dma(A, nxt, buf ? base0 : base1, lane);
    __builtin_amdgcn_sched_barrier(0);
    // 3. the MFMAs of t, tn's operands behind each k-step
    d4 acc[2][4];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < 4; ++tj) acc[ti][tj] = d4{0, 0, 0, 0};
#pragma unroll
    for (int st = 0; st < 9; ++st) {
      const bool live = 4 * st < cur.kw;
#pragma unroll
      for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 4; ++tj)
          acc[ti][tj] = mfma_f64(live ? a[ti][st] : 0.0, live ? b[tj][st] : 0.0, acc[ti][tj]);
      stream_ops_step(A, nxt, st, a, b, lane);
      asm volatile("" ::: "memory");      // (tn's loads stay among t's MFMAs: not sunk below,
      __builtin_amdgcn_sched_barrier(0);  //  not scheduled past)
    }
    // 4. Σ_in(t) from LDS (MFMA layout), Σ_out = Σ_in − K·M (+ Q̄) back into the image (columns
    //    ≥ n as 0: the padding stays zero), the kRowsOut rows from registers; 5. the image row by
    //    row, 16 × dwordx4 (2 rows × 512 B each). Every store is issued whatever the tile (dummy
    //    tiles and columns outside U_next go out of range): a fixed 48 VMEM stores per tile, so the
    //    compiler's wait for the next operands is an exact vmcnt(48)
    {
      const size_t fo = static_cast<size_t>(A.f0 + cur.fb) * A.sig_stride;
      double* So = A.sig[cur.par ^ 1] + fo + static_cast<size_t>(cur.R0) * ld;
      const auto rout = buf_rsrc(So, cur.live ? static_cast<unsigned>(min(n - cur.R0, 32)) * ld * 8u : 0u);
      const bool first = (cur.flags & kFirst) != 0;
      lds_d* im = (lds_d*)&img[wv][buf][0];
      int bpos[4] = {-1, -1, -1, -1};
      const bool rows_out = cur.live && (cur.flags & kRowsOut) != 0;
      if (rows_out) {  // first position in U_next of each column (scalar scan, lowest b first)
        const int nu = cdesc[cur.fb].nxt_nu;
        for (int bb = 0; bb < nu; ++bb) {
          const int dc = cdesc[cur.fb].nxt_u[bb] - cur.C0;
          if (dc >= 0 && dc < 64) {
#pragma unroll
            for (int tj = 0; tj < 4; ++tj)
              if (bpos[tj] < 0 && 16 * tj + kcol == dc) bpos[tj] = bb;
          }
        }
      }
      const auto rrows = buf_rsrc(A.rows + static_cast<size_t>(A.f0 + cur.fb) * A.rows_stride,
                                  rows_out ? static_cast<unsigned>(kRowW) * ldk * 8u : 0u);
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) {
        double sv[4][4];  // a half tile's LDS reads first (one wait)
#pragma unroll
        for (int tj = 0; tj < 4; ++tj)
#pragma unroll
          for (int r = 0; r < 4; ++r) sv[tj][r] = im[(16 * ti + kr + 4 * r) * 64 + 16 * tj + kcol];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int tj = 0; tj < 4; ++tj)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int rl = 16 * ti + kr + 4 * r, col = cur.C0 + 16 * tj + kcol, row = cur.R0 + rl;
            double v = sv[tj][r] - acc[ti][tj][r];
            if (first && row == col && row < 3) v += q;
            v = col < n ? v : 0.0;
            im[rl * 64 + 16 * tj + kcol] = v;
            const unsigned ro = bpos[tj] >= 0 && row < n
                                    ? static_cast<unsigned>(bpos[tj] * ldk + row) * 8u : kOOB;
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), rrows, ro, 0, 0);
          }
      }
      __builtin_amdgcn_sched_barrier(0);
      const int c = cur.C0 + 2 * (lane & 31);
      const unsigned vo = c < n ? static_cast<unsigned>((lane >> 5) * ld + c) * 8u : kOOB;
      const unsigned rs = 2u * ld * 8u;
      typedef double d2 __attribute__((ext_vector_type(2)));
      typedef int i4 __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const d2 w = *(const __attribute__((address_space(3))) d2*)&im[(2 * i + (lane >> 5)) * 64 + 2 * (lane & 31)];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i4, w), rout, vo, rs * i, 2);
      }
    }
    if (tn >= T) break;
    cur = nxt;
    t = tn;
    buf ^= 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the last dummy DMA out of the LDS's way)
}
#pragma clang diagnostic pop

// ---- symmetric pass: only the tiles holding an element on or above the diagonal -----------------
// Σ_out is symmetric, so element (r, c), r > c, is the mirror of (c, r): a tile computes as the
// product's does, stores its elements with c ≥ r in place and those with c > r mirrored to (c, r)
// (16 rows × 32 B per store instruction, four instructions fill 128 B of each mirrored row).
// Σ_in is read in the upper tiles only, the MFMA work of the strictly-lower tiles is skipped.
// kRowsOut: (i, u) for u ∈ U_next comes from the upper element (min, max), so a tile also hands
// off its rows that are in U_next, at the columns right of the diagonal.
__device__ __forceinline__ void sym_tile(int t, int trows, int tcols, int& tr, int& tc, bool& ok) {
  tr = 0;
  int base = 0;
  for (; tr < trows; ++tr) {
    const int c = tcols - tr / 2;
    if (t < base + c) break;
    base += c;
  }
  ok = tr < trows;
  tc = tr / 2 + (t - base);
}
// (transposed tile row stride: ekfslam::kTS)
template <int MIR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_sym(PassArgs<double> A, int tcols, int xcd_b, int nf) {
  const int L = blockIdx.x, j = L >> 3;
  const int fb = (L & 7) + 8 * (j / xcd_b), bx = j % xcd_b;
  if (fb >= nf) return;
  const MsgDesc& d = A.desc[fb];
  __shared__ int cmap[4][64], rmap[4][32];
  __shared__ double tT[MIR ? 4 : 1][MIR ? 64 * kTS : 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int trows = (A.n + 31) / 32;
  const int t = __builtin_amdgcn_readfirstlane(bx * 4 + wv);
  int tr, tc;
  bool ok;
  sym_tile(t, trows, tcols, tr, tc, ok);
  if (!ok || !(d.flags & kActive)) return;
  const int R0 = tr * 32, C0 = tc * 64;
  const int f = A.f0 + fb;
  const int n = A.n, ld = A.ld, ldk = A.ldk;
  const double* Sin = A.sig[d.parity] + f * A.sig_stride;
  double* Sout = A.sig[d.parity ^ 1] + f * A.sig_stride;
  const double* kc = A.kcat + f * A.km_stride;
  const double* mc = A.mcat + f * A.km_stride;
  constexpr int TJ = 4;
  const int kr = lane >> 4, kcol = lane & 15;
  const size_t pbase = static_cast<size_t>(R0) * ld;
  const unsigned sbytes = static_cast<unsigned>(min(n - R0, 32)) * ld * 8u;
  const unsigned kbytes = static_cast<unsigned>(kMaxKW) * ldk * 8u;
  const auto rin = buf_rsrc(Sin + pbase, sbytes), rout = buf_rsrc(Sout + pbase, sbytes);
  // the mirror: rows C0 … C0+63 of Σ_out, columns R0 …
  const size_t mbase = static_cast<size_t>(C0) * ld + R0;
  const unsigned mbytes = static_cast<unsigned>(min(n - C0, 64)) * ld * 8u;
  const auto rmir = buf_rsrc(Sout + mbase, mbytes);
  const auto rk = buf_rsrc(kc, kbytes), rm = buf_rsrc(mc, kbytes);
  double a[2][9], b[TJ][9], sv[2][TJ][4];
  const bool rows_on = (d.flags & kRowsOut) != 0;
  const int uk = rows_on ? d.nxt_u[min(lane, kMaxU)] : 0;
  const unsigned ko = static_cast<unsigned>(kr * ldk + R0 + kcol) * 8u;
  unsigned mo[TJ], so[TJ];
  const unsigned rstride = static_cast<unsigned>(ld) * 8u;
#pragma unroll
  for (int tj = 0; tj < TJ; ++tj) {
    const int col = C0 + 16 * tj + kcol;
    mo[tj] = static_cast<unsigned>(kr * ldk + min(col, n - 1)) * 8u;
    so[tj] = col < n ? static_cast<unsigned>(kr * ld + col) * 8u : kOOB;
  }
  const unsigned kstep = 4u * ldk * 8u;
#pragma unroll
  for (int s = 0; s < 9; ++s) {
    a[0][s] = ld_f64(rk, ko, s * kstep);
    a[1][s] = ld_f64(rk, ko + 16 * 8, s * kstep);
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj) b[tj][s] = ld_f64(rm, mo[tj], s * kstep);
  }
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sv[ti][tj][r] = __builtin_bit_cast(
            double, __builtin_amdgcn_raw_buffer_load_b64(rin, so[tj] + (16 * ti + 4 * r) * rstride, 0, 2));
  d4 acc[2][TJ];
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj) acc[ti][tj] = d4{0, 0, 0, 0};
  const int kw = ((2 + ((d.flags & kJoseph) ? 4 : 2) * d.m + 3) / 4) * 4;
#pragma unroll
  for (int s = 0; s < 9; ++s) {
    const bool live = 4 * s < kw;
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj)
        acc[ti][tj] = mfma_f64(live ? a[ti][s] : 0.0, live ? b[tj][s] : 0.0, acc[ti][tj]);
  }
  int bpos[TJ], rpos[2][4];
#pragma unroll
  for (int tj = 0; tj < TJ; ++tj) bpos[tj] = -1;
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int r = 0; r < 4; ++r) rpos[ti][r] = -1;
  if (rows_on) {
    int* map = cmap[wv];
    int* rmp = rmap[wv];
    map[lane] = kMaxU + 1;
    if (lane < 32) rmp[lane] = kMaxU + 1;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int nnu = d.nxt_nu;
    if (lane < nnu && uk >= C0 && uk < C0 + 64) atomicMin(&map[uk - C0], lane);
    if (lane < nnu && uk >= R0 && uk < R0 + 32) atomicMin(&rmp[uk - R0], lane);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj) {
      const int bb = map[16 * tj + kcol];
      bpos[tj] = bb <= kMaxU ? bb : -1;
    }
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int bb = rmp[16 * ti + kr + 4 * r];
        rpos[ti][r] = bb <= kMaxU ? bb : -1;
      }
  }
  const bool first = (d.flags & kFirst) != 0;
  const double q = A.q;
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = 16 * ti + kr + 4 * r, cl = 16 * tj + kcol;
        const int row = R0 + rl, col = C0 + cl;
        double v = sv[ti][tj][r] - acc[ti][tj][r];
        if (first && row == col && row < 3) v += q;
        const u2v w = __builtin_bit_cast(u2v, v);
        __builtin_amdgcn_raw_buffer_store_b64(w, rout, col >= row ? so[tj] + (16 * ti + 4 * r) * rstride : kOOB, 0, 2);
        if (MIR) {
          tT[wv][cl * kTS + rl] = v;
        } else {
          const unsigned mo2 = col > row && col < n ? static_cast<unsigned>(cl * ld + rl) * 8u : kOOB;
          __builtin_amdgcn_raw_buffer_store_b64(w, rmir, mo2, 0, 2);
        }
        if (col >= row && row < n && col < n) {
          if (bpos[tj] >= 0) A.rows[f * A.rows_stride + static_cast<size_t>(bpos[tj]) * ldk + row] = v;
          if (col > row && rpos[ti][r] >= 0) A.rows[f * A.rows_stride + static_cast<size_t>(rpos[ti][r]) * ldk + col] = v;
        }
      }
  if (MIR) {  // the mirror: row cl of the transposed tile → Σ_out row C0 + cl, columns R0 …, 2 rows per store
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int rl = lane & 31;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int cl = 2 * i + (lane >> 5);
      const double v = tT[wv][cl * kTS + rl];
      const int row = R0 + rl, col = C0 + cl;
      const unsigned mo2 = col > row && col < n ? static_cast<unsigned>(cl * ld + rl) * 8u : kOOB;
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), rmir, mo2, 0, 2);
    }
  }
}

// ---- symmetric pass, two vertically adjacent tiles per wave (the M operand loaded once) -------
// Column-major over the upper tiles: column tc holds tile rows 0 … min(trows, 2·tc + 2) − 1, in
// pairs (2j, 2j + 1); the wave loads the column's M operand once and runs the two tiles in turn.
__device__ __forceinline__ bool pair_slot(int t, int trows, int tcols, int& tc, int& r0, int& cnt) {
  int base = 0;
  for (tc = 0; tc < tcols; ++tc) {
    cnt = min(trows, 2 * tc + 2);
    const int p = (cnt + 1) / 2;
    if (t < base + p) break;
    base += p;
  }
  r0 = 2 * (t - base);
  return tc < tcols;
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_sym_pair(PassArgs<double> A, int tcols, int xcd_b, int nf) {
  const int L = blockIdx.x, j = L >> 3;
  const int fb = (L & 7) + 8 * (j / xcd_b), bx = j % xcd_b;
  if (fb >= nf) return;
  const MsgDesc& d = A.desc[fb];
  __shared__ double tTs[4][64 * kTS];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int trows = (A.n + 31) / 32;
  const int t = __builtin_amdgcn_readfirstlane(bx * 4 + wv);
  int tc, r0, cnt;
  if (!pair_slot(t, trows, tcols, tc, r0, cnt) || !(d.flags & kActive)) return;
  const int C0 = tc * 64;
  const int f = A.f0 + fb;
  const int n = A.n, ld = A.ld, ldk = A.ldk;
  const double* Sin = A.sig[d.parity] + f * A.sig_stride;
  double* Sout = A.sig[d.parity ^ 1] + f * A.sig_stride;
  constexpr int TJ = 4;
  const int kr = lane >> 4, kcol = lane & 15;
  const unsigned kbytes = static_cast<unsigned>(kMaxKW) * ldk * 8u;
  const auto rk = buf_rsrc(A.kcat + f * A.km_stride, kbytes), rm = buf_rsrc(A.mcat + f * A.km_stride, kbytes);
  const auto rmir = buf_rsrc(Sout + static_cast<size_t>(C0) * ld, static_cast<unsigned>(min(n - C0, 64)) * ld * 8u);
  double b[TJ][9];
  unsigned so[TJ];
  const unsigned kstep = 4u * ldk * 8u;
#pragma unroll
  for (int tj = 0; tj < TJ; ++tj) {
    const int col = C0 + 16 * tj + kcol;
    const unsigned mo = static_cast<unsigned>(kr * ldk + min(col, n - 1)) * 8u;
    so[tj] = col < n ? static_cast<unsigned>(kr * ld + col) * 8u : kOOB;
#pragma unroll
    for (int s = 0; s < 9; ++s) b[tj][s] = ld_f64(rm, mo, s * kstep);
  }
  const int kw = ((2 + ((d.flags & kJoseph) ? 4 : 2) * d.m + 3) / 4) * 4;
  const bool first = (d.flags & kFirst) != 0;
  const double q = A.q;
  const unsigned rstride = static_cast<unsigned>(ld) * 8u;
  double* tT = tTs[wv];
  for (int h = 0; h < 2; ++h) {
    const int tr = r0 + h;
    if (tr >= cnt) break;
    const int R0 = tr * 32;
    const auto rin = buf_rsrc(Sin + static_cast<size_t>(R0) * ld, static_cast<unsigned>(min(n - R0, 32)) * ld * 8u);
    const auto rout = buf_rsrc(Sout + static_cast<size_t>(R0) * ld, static_cast<unsigned>(min(n - R0, 32)) * ld * 8u);
    double a[2][9], sv[2][TJ][4];
    const unsigned ko = static_cast<unsigned>(kr * ldk + R0 + kcol) * 8u;
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      a[0][s] = ld_f64(rk, ko, s * kstep);
      a[1][s] = ld_f64(rk, ko + 16 * 8, s * kstep);
    }
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          sv[ti][tj][r] = __builtin_bit_cast(
              double, __builtin_amdgcn_raw_buffer_load_b64(rin, so[tj] + (16 * ti + 4 * r) * rstride, 0, 2));
    d4 acc[2][TJ];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) acc[ti][tj] = d4{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      const bool live = 4 * s < kw;
#pragma unroll
      for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < TJ; ++tj)
          acc[ti][tj] = mfma_f64(live ? a[ti][s] : 0.0, live ? b[tj][s] : 0.0, acc[ti][tj]);
    }
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rl = 16 * ti + kr + 4 * r, cl = 16 * tj + kcol;
          const int row = R0 + rl, col = C0 + cl;
          double v = sv[ti][tj][r] - acc[ti][tj][r];
          if (first && row == col && row < 3) v += q;
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), rout,
                                                col >= row ? so[tj] + (16 * ti + 4 * r) * rstride : kOOB, 0, 2);
          tT[cl * kTS + rl] = v;
        }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int rl = lane & 31;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int cl = 2 * i + (lane >> 5);
      const double v = tT[cl * kTS + rl];
      const int row = R0 + rl, col = C0 + cl;
      const unsigned mo2 = col > row && col < n ? static_cast<unsigned>(cl * ld + R0 + rl) * 8u : kOOB;
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), rmir, mo2, 0, 2);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
}

template <typename V>
__global__ void k_copy(const V* __restrict__ in, V* __restrict__ out, size_t nv) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += gridDim.x * blockDim.x) out[i] = in[i];
}

int main(int argc, char** argv) {
  const int F = argc > 1 ? atoi(argv[1]) : 512, reps = argc > 2 ? atoi(argv[2]) : 20;
  const int N = 256, n = 3 + 2 * N, ld = (n + 15) / 16 * 16, ldk = (n + 63) / 64 * 64;
  const size_t stride = static_cast<size_t>(n) * ld, km = static_cast<size_t>(kMaxKW) * ldk;
  double *S0, *S1, *kc, *mc, *rows;
  CK(hipMalloc(&S0, stride * F * 8));
  CK(hipMalloc(&S1, stride * F * 8));
  CK(hipMalloc(&kc, km * F * 8));
  CK(hipMalloc(&mc, km * F * 8));
  CK(hipMalloc(&rows, static_cast<size_t>(kRowW) * ldk * F * 8));
  {
    std::vector<double> h(stride * F);
    srand(7);
    for (auto& v : h) v = (rand() % 100000) * 1e-3;
    CK(hipMemcpy(S0, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    std::vector<double> k(km * F);
    for (auto& v : k) v = (rand() % 2000 - 1000) * 1e-4;
    CK(hipMemcpy(kc, k.data(), k.size() * 8, hipMemcpyHostToDevice));
    for (auto& v : k) v = (rand() % 2000 - 1000) * 1e-4;
    CK(hipMemcpy(mc, k.data(), k.size() * 8, hipMemcpyHostToDevice));
  }
  std::vector<MsgDesc> hd(F);
  for (int f = 0; f < F; ++f) {
    MsgDesc& d = hd[f];
    std::memset(&d, 0, sizeof d);
    d.m = 16;
    d.flags = kActive | kFirst | ((f % 3) ? kRowsOut : 0);
    d.parity = 0;
    d.nxt_nu = 35;
    for (int b = 0; b <= kMaxU; ++b) d.nxt_u[b] = b < 3 ? b : 3 + ((f * 37 + b * 11) % (n - 3));
  }
  MsgDesc* dd;
  CK(hipMalloc(&dd, sizeof(MsgDesc) * F));
  CK(hipMemcpy(dd, hd.data(), sizeof(MsgDesc) * F, hipMemcpyHostToDevice));
  PassArgs<double> a{};
  a.sig[0] = S0; a.sig[1] = S1; a.sig_stride = stride;
  a.kcat = kc; a.mcat = mc; a.km_stride = km; a.ldk = ldk;
  a.rows = rows; a.rows_stride = static_cast<size_t>(kRowW) * ldk;
  a.desc = dd; a.n = n; a.ld = ld; a.N = N; a.q = 1e-2;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = 2.0 * n * n * 8 * F;
  std::vector<double> ref(stride * F), out(stride * F), rref(a.rows_stride * F), rout(a.rows_stride * F);
  const int trows = (n + 31) / 32, tcols = (n + 63) / 64, per_filter = (trows * tcols + 3) / 4;
  // the product's pass is symmetric since round 4: its grid covers the upper tiles only
  const int prod_pf = (sym_tiles<64>(trows, tcols) + 3) / 4;
  auto prod = [&](hipStream_t st) {
    hipLaunchKernelGGL((k_sigma_pass<double, true>), dim3(8 * ((F + 7) / 8) * prod_pf), dim3(256), 0, st,
                       a, tcols, prod_pf, F);
  };
  auto time_it = [&](const char* name, auto&& fn, bool check_rows) {
    CK(hipMemset(S1, 0, stride * F * 8));
    CK(hipMemset(rows, 0, a.rows_stride * F * 8));
    for (int i = 0; i < 3; ++i) fn(s);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(out.data(), S1, stride * F * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rout.data(), rows, a.rows_stride * F * 8, hipMemcpyDeviceToHost));
    float best = 1e30f, sum = 0;
    for (int rep = 0; rep < 3; ++rep) {
      float ms;
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < reps; ++i) fn(s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
      sum += ms;
    }
    size_t bad = 0, rbad = 0;
    for (int f = 0; f < F; ++f)
      for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) {
          const size_t o = f * stride + static_cast<size_t>(r) * ld + c;
          if (std::memcmp(&out[o], &ref[o], 8)) ++bad;
        }
    if (check_rows)
      for (int f = 0; f < F; ++f)
        for (int b = 0; b < kMaxU; ++b)
          for (int r = 0; r < n; ++r) {
            const size_t o = f * a.rows_stride + static_cast<size_t>(b) * ldk + r;
            if (std::memcmp(&rout[o], &rref[o], 8)) ++rbad;
          }
    printf("%-26s %8.2f us (best of 3; mean %8.2f)  %6.0f GB/s  frac %.3f  mismatches %zu rows %zu\n", name,
           best * 1e3 / reps, sum / 3 * 1e3 / reps, bytes / (best / reps * 1e-3) / 1e9,
           bytes / (best / reps * 1e-3) / 8e12, bad, rbad);
    fflush(stdout);
  };
  CK(hipMemset(rows, 0, a.rows_stride * F * 8));
  prod(s);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(ref.data(), S1, stride * F * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(rref.data(), rows, a.rows_stride * F * 8, hipMemcpyDeviceToHost));
  {
    using F4 = float4;
    const size_t nv = stride * F * 8 / sizeof(F4);
    time_it("copy float4", [&](hipStream_t st) {
      hipLaunchKernelGGL(k_copy<F4>, dim3(8192), dim3(256), 0, st, (const F4*)S0, (F4*)S1, nv);
    }, false);
  }
  auto abl = [&](auto kern) {
    return [&, kern](hipStream_t st) {
      hipLaunchKernelGGL(kern, dim3(8 * ((F + 7) / 8) * per_filter), dim3(256), 0, st, a, tcols, per_filter, F);
    };
  };
  int dev_cus = 0;
  CK(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, 0));
  auto stream = [&](int blocks) {
    return [&, blocks](hipStream_t st) {
      hipLaunchKernelGGL(k_sigma_stream, dim3(blocks), dim3(256), 0, st, a, tcols, trows * tcols, F);
    };
  };
  int sym_tiles = 0;
  for (int tr = 0; tr < trows; ++tr) sym_tiles += tcols - tr / 2;
  const int sym_pf = (sym_tiles + 3) / 4;
  auto sym = [&](hipStream_t st) {
    constexpr int MIRV = 1;
    hipLaunchKernelGGL(k_sym<MIRV>, dim3(8 * ((F + 7) / 8) * sym_pf), dim3(256), 0, st, a, tcols, sym_pf, F);
  };
  auto sym_check = [&]() {  // Σ_out(r, c) = product's (min, max); rows(b, i) = product's (min(i, u), max)
    size_t bad = 0, rbad = 0;
    for (int f = 0; f < F; ++f) {
      for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) {
          const size_t o = f * stride + static_cast<size_t>(r) * ld + c;
          const size_t oe = f * stride + static_cast<size_t>(std::min(r, c)) * ld + std::max(r, c);
          if (std::memcmp(&out[o], &ref[oe], 8)) ++bad;
        }
      if (hd[f].flags & kRowsOut)
        for (int bb = 0; bb < hd[f].nxt_nu; ++bb) {
          bool firstpos = true;
          for (int k = 0; k < bb; ++k) firstpos = firstpos && hd[f].nxt_u[k] != hd[f].nxt_u[bb];
          if (!firstpos) continue;
          const int u = hd[f].nxt_u[bb];
          for (int i = 0; i < n; ++i) {
            const size_t o = f * a.rows_stride + static_cast<size_t>(bb) * ldk + i;
            const size_t oe = f * stride + static_cast<size_t>(std::min(i, u)) * ld + std::max(i, u);
            if (std::memcmp(&rout[o], &ref[oe], 8)) ++rbad;
          }
        }
    }
    printf("  symmetric check vs product's upper triangle: mismatches %zu rows %zu (%d of %d tiles)\n", bad, rbad,
           sym_tiles, trows * tcols);
  };
  int pairs = 0;
  for (int tc = 0; tc < tcols; ++tc) pairs += (std::min(trows, 2 * tc + 2) + 1) / 2;
  const int pair_pf = (pairs + 3) / 4;
  auto sym_pair = [&](hipStream_t st) {
    hipLaunchKernelGGL(k_sym_pair, dim3(8 * ((F + 7) / 8) * pair_pf), dim3(256), 0, st, a, tcols, pair_pf, F);
  };
  for (int round = 0; round < 2; ++round) {
    time_it("symmetric, 2 tiles per wave", sym_pair, false);
    sym_check();
    time_it("symmetric k_sym (LDS transpose)", sym, false);
    sym_check();
    time_it("product k_sigma_pass", prod, true);
    time_it("ablate: copy of product", abl(k_ablate<0>), false);
    time_it("ablate: no mfma", abl(k_ablate<kNoMfma>), false);
    time_it("ablate: sigma only", abl(k_ablate<kNoMfma | kNoOps>), false);
  }
  return 0;
}
