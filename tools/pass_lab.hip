// Dev tool (not shipped): Σ-pass variants A/B'd standalone against the product's k_sigma_pass on the
// same buffers (N = 1024 fp32, the headline's pass), outputs compared bit for bit.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include -I../ekf-slam_amd/csrc pass_lab.hip -o pass_lab
#include "../ekf-slam_amd/csrc/ekf_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace ekfslam;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

// the product's region mapping (k_sigma_pass, xcd_b = −1) for WPB waves per workgroup. MODE bits:
// 1 Σ buffers chosen by the descriptor's parity (as the product: every load waits for it),
// 2 no MFMA (one VALU product keeps the operand loads live), 4 constant operands (no operand loads),
// 8 issue priority 2 once the MFMAs are done, 16 Σ_in loads issued before the operand loads
enum { kDesc = 1, kNoMfma = 2, kNoOps = 4, kPrio = 8, kSigFirst = 16, kStag1 = 32, kStag2 = 64, kStagW = 128 };
template <int WPB, int MODE>
__global__ __launch_bounds__(64 * WPB) void k_lab_region(PassArgs<float> A, int tcols) {
  using Tile = SigmaTile<float>;
  const MsgDesc& d = A.desc[0];
  const int lane = threadIdx.x & 63;
  const int trows = (A.n + Tile::kRows - 1) / Tile::kRows;
  const int x = blockIdx.x & 7, w = (blockIdx.x >> 3) * WPB + (threadIdx.x >> 6);
  const int hx = x / kRegCols, qx = x % kRegCols;
  const int r0 = hx * trows / kRegRows, r1 = (hx + 1) * trows / kRegRows;
  const int c0 = qx * tcols / kRegCols, c1 = (qx + 1) * tcols / kRegCols;
  const int cw = c1 - c0;
  const int tt = __builtin_amdgcn_readfirstlane(w);
  if (tt >= (r1 - r0) * cw) return;
  const int tr = r0 + tt / cw, tc = c0 + tt % cw;
  const int R0 = tr * 32, C0 = tc * 32;
  // stagger: odd workgroup rounds (or odd wave slots) start ≈ 0.5 / 1 µs late
  if ((MODE & (kStag1 | kStag2)) && (((MODE & kStagW) ? (threadIdx.x >> 6) : (blockIdx.x >> 3)) & 1)) {
    if (MODE & kStag1) __builtin_amdgcn_s_sleep(20);
    else { __builtin_amdgcn_s_sleep(38); }
  }
  int par = 0;
  if (MODE & kDesc) {
    if (!(d.flags & kActive)) return;
    par = d.parity;
  }
  const float* Sin = A.sig[par];
  float* Sout = A.sig[par ^ 1];
  F32TileRegs g;
  if (MODE & kSigFirst) {
    Tile::load_sig(g, Sin, A.n, A.ld, R0, C0, lane);
    __builtin_amdgcn_sched_barrier(0);
    if (!(MODE & kNoOps)) Tile::load_ops(g, A.kcat, A.mcat, A.n, A.ldk, R0, C0, lane);
  } else {
    if (!(MODE & kNoOps)) Tile::load_ops(g, A.kcat, A.mcat, A.n, A.ldk, R0, C0, lane);
    __builtin_amdgcn_sched_barrier(0);
    Tile::load_sig(g, Sin, A.n, A.ld, R0, C0, lane);
  }
  if (MODE & kNoOps)
    for (int s2 = 0; s2 < kSteps; ++s2) g.a[s2] = g.b[s2] = 1e-3f * (s2 + 1);
  const int kw = ((2 + 2 * d.m + 3) / 4) * 4;
  const bool first = (d.flags & kFirst) != 0;
  const int kr = lane >> 5, col = C0 + (lane & 31);
  const auto rout = Tile::panel(Sout, A.n, A.ld, R0);
  const unsigned so = Tile::soff(A.n, A.ld, C0, lane);
  const unsigned rstride = static_cast<unsigned>(A.ld) * 4u;
  f16v acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  if (MODE & kNoMfma) {
    float t = 0.0f;
#pragma unroll
    for (int s2 = 0; s2 < kSteps; ++s2) t += g.a[s2] * g.b[s2];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = t;
  } else {
#pragma unroll
    for (int s2 = 0; s2 < kSteps; ++s2) {
      const bool live = 2 * s2 < kw;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(live ? g.a[s2] : 0.0f, live ? g.b[s2] : 0.0f, acc, 0, 0, 0);
    }
  }
  if (MODE & kPrio) __builtin_amdgcn_s_setprio(2);
  const float q = static_cast<float>(A.q);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = R0 + (r & 3) + 8 * (r >> 2) + 4 * kr;
    float v = g.sv[r] - acc[r];
    if (first && row == col && row < 3) v += q;
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rout,
                                          so + ((r & 3) + 8 * (r >> 2)) * rstride, 0, 0);
  }
}

// LDS-shared operands: a workgroup's 4 waves take the 2 × 2 tiles of a 64 × 64 block; the block's
// K rows (34 × 64) and M columns (34 × 64) are loaded once (17 dword loads per lane instead of 34),
// staged in LDS, and every wave reads its 34 operands from there. The Σ_in loads are issued before
// the barrier (an LDS-only barrier keeps them in flight). Blocks dealt over XCD regions of the
// block grid as the product's tiles are.
template <int MODE>
__global__ __launch_bounds__(256) void k_lab_lds(PassArgs<float> A, int bcols) {
  using Tile = SigmaTile<float>;
  __shared__ float ko[kSteps * 2][64], mo[kSteps * 2][64];
  const MsgDesc& d = A.desc[0];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n = A.n, ld = A.ld, ldk = A.ldk;
  const int brows = (n + 63) / 64;
  const int x = blockIdx.x & 7, bb = blockIdx.x >> 3;
  const int hx = x / kRegCols, qx = x % kRegCols;
  const int r0 = hx * brows / kRegRows, r1 = (hx + 1) * brows / kRegRows;
  const int c0 = qx * bcols / kRegCols, c1 = (qx + 1) * bcols / kRegCols;
  const int cw = c1 - c0;
  if (bb >= (r1 - r0) * cw) return;
  const int br = r0 + bb / cw, bc = c0 + bb % cw;
  const int B0 = br * 64, D0 = bc * 64;
  const int R0 = B0 + 32 * (wv >> 1), C0 = D0 + 32 * (wv & 1);
  const bool live_tile = R0 < n && C0 < n;
  // operands: thread t loads k-rows (t >> 6) + 4i of the block's K and M slices
  const unsigned kbytes = static_cast<unsigned>(kMaxKW) * ldk * 4u;
  const auto rk = buf_rsrc(A.kcat, kbytes), rm = buf_rsrc(A.mcat, kbytes);
  float kv[9], mv[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int k = wv + 4 * i;  // 0..35, rows ≥ 34 unused
    const int kk = k < 2 * kSteps ? k : 0;
    kv[i] = ld_f32(rk, static_cast<unsigned>(kk * ldk + min(B0 + lane, ldk - 1)) * 4u, 0);
    mv[i] = ld_f32(rm, static_cast<unsigned>(kk * ldk + min(D0 + lane, n - 1)) * 4u, 0);
  }
  F32TileRegs g;
  __builtin_amdgcn_sched_barrier(0);
  if (live_tile) Tile::load_sig(g, A.sig[0], n, ld, R0, C0, lane);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int k = wv + 4 * i;
    if (k < 2 * kSteps) {
      ko[k][lane] = kv[i];
      mo[k][lane] = mv[i];
    }
  }
  lds_barrier();
  if (!live_tile) return;
  const int h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int s2 = 0; s2 < kSteps; ++s2) {
    g.a[s2] = ko[2 * s2 + h][32 * (wv >> 1) + l32];
    g.b[s2] = mo[2 * s2 + h][32 * (wv & 1) + l32];
  }
  const int kw = ((2 + 2 * d.m + 3) / 4) * 4;
  Tile::finish(g, A.sig[1], n, ld, kw, (d.flags & kFirst) != 0, A.q, R0, C0, lane);
}
void launch_lds(const PassArgs<float>& a, hipStream_t s) {
  const int b = (a.n + 63) / 64;
  hipLaunchKernelGGL((k_lab_lds<0>), dim3(8 * region_tiles(b, b)), dim3(256), 0, s, a, b);
}

// 2 × 2 tile blocks per workgroup (wave w: tile (2·br + (w >> 1), 2·bc + (w & 1))): each K slice
// is read by two waves of one CU and each M slice by two (L1 reuse) instead of one K slice by four
// waves and four M slices. BAR: an LDS-only barrier between the operand loads and the Σ_in loads,
// so the workgroup's operand requests go out ahead of its Σ traffic.
template <bool BAR>
__global__ __launch_bounds__(256) void k_lab_2x2(PassArgs<float> A, int bcols) {
  using Tile = SigmaTile<float>;
  const MsgDesc& d = A.desc[0];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n = A.n;
  const int brows = (n + 63) / 64;
  const int x = blockIdx.x & 7, bb = blockIdx.x >> 3;
  const int hx = x / kRegCols, qx = x % kRegCols;
  const int r0 = hx * brows / kRegRows, r1 = (hx + 1) * brows / kRegRows;
  const int c0 = qx * bcols / kRegCols, c1 = (qx + 1) * bcols / kRegCols;
  const int cw = c1 - c0;
  if (bb >= (r1 - r0) * cw) return;
  const int br = r0 + bb / cw, bc = c0 + bb % cw;
  const int R0 = br * 64 + 32 * (wv >> 1), C0 = bc * 64 + 32 * (wv & 1);
  const bool live = R0 < n && C0 < n;
  F32TileRegs g;
  if (live) Tile::load_ops(g, A.kcat, A.mcat, n, A.ldk, R0, C0, lane);
  if (BAR) lds_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (!live) return;
  Tile::load_sig(g, A.sig[0], n, A.ld, R0, C0, lane);
  const int kw = ((2 + 2 * d.m + 3) / 4) * 4;
  Tile::finish(g, A.sig[1], n, A.ld, kw, (d.flags & kFirst) != 0, A.q, R0, C0, lane);
}
template <bool BAR>
void launch_2x2(const PassArgs<float>& a, hipStream_t s) {
  const int b = (a.n + 63) / 64;
  hipLaunchKernelGGL((k_lab_2x2<BAR>), dim3(8 * region_tiles(b, b)), dim3(256), 0, s, a, b);
}

// Generic tile placement: a wave computes a 32 × 32·TJ block (TJ accumulators sharing the K
// operand); a workgroup's WPB waves are placed WR tile-rows × (WPB / WR) block-columns; workgroups
// dealt over the product's 2 × 4 XCD regions of the workgroup grid.
template <int TJ, int WPB, int WR>
__global__ __launch_bounds__(64 * WPB) void k_lab_gen(PassArgs<float> A, int gcols) {
  using Tile = SigmaTile<float>;
  constexpr int WC = WPB / WR;
  const MsgDesc& d = A.desc[0];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n = A.n, ld = A.ld, ldk = A.ldk;
  const int grows = (n + 32 * WR - 1) / (32 * WR);
  const int x = blockIdx.x & 7, bb = blockIdx.x >> 3;
  const int hx = x / kRegCols, qx = x % kRegCols;
  const int r0 = hx * grows / kRegRows, r1 = (hx + 1) * grows / kRegRows;
  const int c0 = qx * gcols / kRegCols, c1 = (qx + 1) * gcols / kRegCols;
  const int cw = c1 - c0;
  if (bb >= (r1 - r0) * cw) return;
  const int gr = r0 + bb / cw, gc = c0 + bb % cw;
  const int R0 = gr * 32 * WR + 32 * (wv / WC), Cb = gc * 32 * TJ * WC + 32 * TJ * (wv % WC);
  if (R0 >= n || Cb >= n) return;
  const int kw = ((2 + 2 * d.m + 3) / 4) * 4;
  const bool first = (d.flags & kFirst) != 0;
  const int kr = lane >> 5, kcol = lane & 31;
  const unsigned kbytes = static_cast<unsigned>(kMaxKW) * ldk * 4u;
  const auto rk = buf_rsrc(A.kcat, kbytes), rm = buf_rsrc(A.mcat, kbytes);
  const unsigned ko = static_cast<unsigned>(kr * ldk + R0 + kcol) * 4u;
  const unsigned kstep = 2u * ldk * 4u;
  float a[kSteps], b[TJ][kSteps], sv[TJ][16];
#pragma unroll
  for (int s2 = 0; s2 < kSteps; ++s2) a[s2] = ld_f32(rk, ko, s2 * kstep);
#pragma unroll
  for (int tj = 0; tj < TJ; ++tj) {
    const unsigned mo = static_cast<unsigned>(kr * ldk + min(Cb + 32 * tj + kcol, n - 1)) * 4u;
#pragma unroll
    for (int s2 = 0; s2 < kSteps; ++s2) b[tj][s2] = ld_f32(rm, mo, s2 * kstep);
  }
  __builtin_amdgcn_sched_barrier(0);
  const auto rin = Tile::panel(A.sig[0], n, ld, R0), rout = Tile::panel(A.sig[1], n, ld, R0);
  const unsigned rstride = static_cast<unsigned>(ld) * 4u;
  unsigned so[TJ];
#pragma unroll
  for (int tj = 0; tj < TJ; ++tj) {
    so[tj] = Tile::soff(n, ld, Cb + 32 * tj, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) sv[tj][r] = ld_f32(rin, so[tj] + ((r & 3) + 8 * (r >> 2)) * rstride, 0);
  }
  const float q = static_cast<float>(A.q);
#pragma unroll
  for (int tj = 0; tj < TJ; ++tj) {
    f16v acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
    for (int s2 = 0; s2 < kSteps; ++s2) {
      const bool live = 2 * s2 < kw;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(live ? a[s2] : 0.0f, live ? b[tj][s2] : 0.0f, acc, 0, 0, 0);
    }
    const int col = Cb + 32 * tj + kcol;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = R0 + (r & 3) + 8 * (r >> 2) + 4 * kr;
      float v = sv[tj][r] - acc[r];
      if (first && row == col && row < 3) v += q;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rout,
                                            so[tj] + ((r & 3) + 8 * (r >> 2)) * rstride, 0, 0);
    }
  }
}
template <int TJ, int WPB, int WR>
void launch_gen(const PassArgs<float>& a, hipStream_t s) {
  constexpr int WC = WPB / WR;
  const int grows = (a.n + 32 * WR - 1) / (32 * WR), gcols = (a.n + 32 * TJ * WC - 1) / (32 * TJ * WC);
  hipLaunchKernelGGL((k_lab_gen<TJ, WPB, WR>), dim3(8 * region_tiles(grows, gcols)), dim3(64 * WPB), 0, s, a, gcols);
}

// XCD row bands: XCD x (blocks L ≡ x mod 8) takes tiles [x·T/8, (x+1)·T/8) of the row-major tile
// grid, WPB consecutive tiles per workgroup: every XCD gets the same tile count (±1), its L2 holds
// Mcat whole and an eighth of Kcat.
template <int WPB>
__global__ __launch_bounds__(64 * WPB) void k_lab_band(PassArgs<float> A, int tcols) {
  using Tile = SigmaTile<float>;
  const MsgDesc& d = A.desc[0];
  const int lane = threadIdx.x & 63;
  const int trows = (A.n + 31) / 32, T = trows * tcols;
  const int x = blockIdx.x & 7;
  const int t0 = x * T / 8, t1 = (x + 1) * T / 8;
  const int t = __builtin_amdgcn_readfirstlane(t0 + (blockIdx.x >> 3) * WPB + (threadIdx.x >> 6));
  if (t >= t1) return;
  const int tr = t / tcols, tc = t - tr * tcols;
  const int kw = ((2 + 2 * d.m + 3) / 4) * 4;
  F32TileRegs g;
  Tile::load(g, A.sig[0], A.kcat, A.mcat, A.n, A.ld, A.ldk, tr * 32, tc * 32, lane);
  Tile::finish(g, A.sig[1], A.n, A.ld, kw, (d.flags & kFirst) != 0, A.q, tr * 32, tc * 32, lane);
}
template <int WPB>
void launch_band(const PassArgs<float>& a, hipStream_t s) {
  const int tr = (a.n + 31) / 32, T = tr * tr;
  const int per = (T + 7) / 8;
  hipLaunchKernelGGL((k_lab_band<WPB>), dim3(8 * ((per + WPB - 1) / WPB)), dim3(64 * WPB), 0, s, a, tr);
}

// 4 × 4 transpose of v[0..3] across each lane quad: afterwards lane j of a quad holds in v[i] what
// lane i held in v[j] (two butterfly stages, one DPP move and three selects per register pair)
__device__ __forceinline__ float dpp_q(float x, int ctrl_sel) {
  const int xi = __builtin_bit_cast(int, x);
  return __builtin_bit_cast(float, ctrl_sel == 1 ? __builtin_amdgcn_mov_dpp(xi, 0xB1, 0xF, 0xF, false)
                                                 : __builtin_amdgcn_mov_dpp(xi, 0x4E, 0xF, 0xF, false));
}
__device__ __forceinline__ void quad_transpose(float (&v)[4], int lane) {
  const bool o1 = lane & 1, o2 = lane & 2;
#pragma unroll
  for (int k = 0; k < 4; k += 2) {  // lane bit 0 ↔ register bit 0
    const float a = v[k], b = v[k + 1];
    const float r = dpp_q(o1 ? a : b, 1);
    v[k] = o1 ? r : a;
    v[k + 1] = o1 ? b : r;
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // lane bit 1 ↔ register bit 1
    const float a = v[k], b = v[k + 2];
    const float r = dpp_q(o2 ? a : b, 2);
    v[k] = o2 ? r : a;
    v[k + 2] = o2 ? b : r;
  }
}

// fp32 tile with row-contiguous Σ access: the MFMA product (lane: column lane & 31, rows
// (r & 3) + 8 (r >> 2) + 4 (lane >> 5)) transposed within lane quads, so lane (q, j, h) holds
// row 8g + 4h + j, columns 4q..4q+3 of each group g: Σ moves as 4 dwordx4 per lane (8 rows × 128 B
// per instruction) instead of 16 dwords. LOADX4: Σ_in loaded the same way (else dword loads in the
// MFMA layout, subtracted before the transpose).
template <bool LOADX4>
__device__ __forceinline__ void tile_x4(const float* Sin, float* Sout, const float* kc, const float* mc,
                                        int n, int ld, int ldk, int kw, bool first, double qd, int R0,
                                        int C0, int lane) {
  using Tile = SigmaTile<float>;
  const int h = lane >> 5, q = (lane & 31) >> 2, j = lane & 3;
  F32TileRegs g0;
  Tile::load_ops(g0, kc, mc, n, ldk, R0, C0, lane);
  const float* a = g0.a;
  const float* b = g0.b;
  const auto rin = Tile::panel(Sin, n, ld, R0), rout = Tile::panel(Sout, n, ld, R0);
  const unsigned rstride = static_cast<unsigned>(ld) * 4u;
  // lane's row-contiguous offset: row 4h + j of group 0, columns C0 + 4q.. (a quad past n reads /
  // writes the padding columns < ld; a quad at or past ld is out of the descriptor's columns)
  const int c4 = C0 + 4 * q;
  const unsigned o4 = c4 < n ? static_cast<unsigned>((4 * h + j) * ld + c4) * 4u : kOOB;
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 s4[4];
  float sv[16];
  if (LOADX4) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
      s4[g] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rin, o4 + 8 * g * rstride, 0, 0));
  } else {
    const unsigned so = Tile::soff(n, ld, C0, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) sv[r] = ld_f32(rin, so + ((r & 3) + 8 * (r >> 2)) * rstride, 0);
  }
  f16v acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
  for (int s = 0; s < kSteps; ++s) {
    const bool live = 2 * s < kw;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(live ? a[s] : 0.0f, live ? b[s] : 0.0f, acc, 0, 0, 0);
  }
  const float qf = static_cast<float>(qd);
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    float v[4];
    if (LOADX4) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = acc[4 * g + i];
      quad_transpose(v, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = s4[g][i] - v[i];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = sv[4 * g + i] - acc[4 * g + i];
      quad_transpose(v, lane);
    }
    const int row = R0 + 8 * g + 4 * h + j;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (first && row == c4 + i && row < 3) v[i] += qf;
    f4 o = {v[0], v[1], v[2], v[3]};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(int __attribute__((ext_vector_type(4))), o),
                                           rout, o4 + 8 * g * rstride, 0, 0);
  }
}

template <int WPB, bool LOADX4>
__global__ __launch_bounds__(64 * WPB) void k_lab_x4(PassArgs<float> A, int tcols) {
  const MsgDesc& d = A.desc[0];
  const int lane = threadIdx.x & 63;
  const int trows = (A.n + 31) / 32;
  const int x = blockIdx.x & 7, w = (blockIdx.x >> 3) * WPB + (threadIdx.x >> 6);
  const int hx = x / kRegCols, qx = x % kRegCols;
  const int r0 = hx * trows / kRegRows, r1 = (hx + 1) * trows / kRegRows;
  const int c0 = qx * tcols / kRegCols, c1 = (qx + 1) * tcols / kRegCols;
  const int cw = c1 - c0;
  const int tt = __builtin_amdgcn_readfirstlane(w);
  if (tt >= (r1 - r0) * cw) return;
  const int tr = r0 + tt / cw, tc = c0 + tt % cw;
  const int kw = ((2 + 2 * d.m + 3) / 4) * 4;
  tile_x4<LOADX4>(A.sig[0], A.sig[1], A.kcat, A.mcat, A.n, A.ld, A.ldk, kw, (d.flags & kFirst) != 0,
                  A.q, tr * 32, tc * 32, lane);
}
template <int WPB, bool LOADX4>
void launch_x4(const PassArgs<float>& a, hipStream_t s) {
  const int trows = (a.n + 31) / 32, tcols = trows;
  hipLaunchKernelGGL((k_lab_x4<WPB, LOADX4>), dim3(8 * ((region_tiles(trows, tcols) + WPB - 1) / WPB)),
                     dim3(64 * WPB), 0, s, a, tcols);
}

// Operands through LDS-DMA: the wave's K rows (34 × 128 B at R0) and M rows (34 × 128 B at C0)
// land in its LDS image by 4 buffer_load_dwordx4 … lds + 1 buffer_load_dword … lds each (10 VMEM
// instructions instead of 34 dword loads), read back as the MFMA operands by ds_read_b32. SIG:
// Σ_in as the product (16 dword loads into registers, issued after the DMA so the operand
// reads wait for vmcnt(16), not vmcnt(0)); else Σ_in also by LDS-DMA (4 dwordx4) into a
// lane-linear 32 × 32 image, read back in the MFMA layout.
typedef __attribute__((address_space(3))) void lds_void;
template <int WPB, bool SIG_REGS>
__global__ __launch_bounds__(64 * WPB) void k_lab_glds(PassArgs<float> A, int tcols) {
  using Tile = SigmaTile<float>;
  constexpr int kImg = 34 * 32;  // floats per operand image
  __shared__ float lds[WPB][2 * kImg + (SIG_REGS ? 0 : 32 * 32)];
  const MsgDesc& d = A.desc[0];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n = A.n, ld = A.ld, ldk = A.ldk;
  const int trows = (n + 31) / 32;
  const int x = blockIdx.x & 7, w = (blockIdx.x >> 3) * WPB + wv;
  const int hx = x / kRegCols, qx = x % kRegCols;
  const int r0 = hx * trows / kRegRows, r1 = (hx + 1) * trows / kRegRows;
  const int c0 = qx * tcols / kRegCols, c1 = (qx + 1) * tcols / kRegCols;
  const int cw = c1 - c0;
  const int tt = __builtin_amdgcn_readfirstlane(w);
  if (tt >= (r1 - r0) * cw) return;
  const int tr = r0 + tt / cw, tc = c0 + tt % cw;
  const int R0 = tr * 32, C0 = tc * 32;
  // descriptor read before the DMA: a use of a vector load issued later would wait for vmcnt(0)
  const int kw = __builtin_amdgcn_readfirstlane(((2 + 2 * d.m + 3) / 4) * 4);
  const bool first = (__builtin_amdgcn_readfirstlane(d.flags) & kFirst) != 0;
  float* Ki = lds[wv];
  float* Mi = Ki + kImg;
  float* Si = Mi + kImg;
  const unsigned kbytes = static_cast<unsigned>(kMaxKW) * ldk * 4u;
  const auto rk = buf_rsrc(A.kcat, kbytes), rm = buf_rsrc(A.mcat, kbytes);
  {
    const unsigned o16 = static_cast<unsigned>((lane >> 3) * ldk + 4 * (lane & 7)) * 4u;
    const unsigned o4 = static_cast<unsigned>((32 + (lane >> 5)) * ldk + (lane & 31)) * 4u;
    const unsigned kr0 = static_cast<unsigned>(R0) * 4u, mc0 = static_cast<unsigned>(C0) * 4u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (lds_void*)(Ki + 256 * i), 16, o16 + kr0, i * 8 * ldk * 4, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rm, (lds_void*)(Mi + 256 * i), 16, o16 + mc0, i * 8 * ldk * 4, 0, 0);
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (lds_void*)(Ki + 1024), 4, o4 + kr0, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rm, (lds_void*)(Mi + 1024), 4, o4 + mc0, 0, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  const auto rin = Tile::panel(A.sig[0], n, ld, R0);
  const unsigned rstride = static_cast<unsigned>(ld) * 4u;
  const unsigned so = Tile::soff(n, ld, C0, lane);
  float sv[16];
  if (SIG_REGS) {
#pragma unroll
    for (int r = 0; r < 16; ++r) sv[r] = ld_f32(rin, so + ((r & 3) + 8 * (r >> 2)) * rstride, 0);
  } else {
    // lane l: row 8i + (l >> 3), columns 4(l & 7)..+3 (columns ≥ ld lie in the next row: unused)
    const unsigned s16 = static_cast<unsigned>((lane >> 3) * ld + C0 + 4 * (lane & 7)) * 4u;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rin, (lds_void*)(Si + 256 * i), 16, s16, i * 8 * rstride, 0, 0);
  }
  // the compiler does not order LDS reads after an LDS-DMA: counted waits by hand
  __builtin_amdgcn_sched_barrier(0);
  if (SIG_REGS) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  const int kr = lane >> 5, kcol = lane & 31;
  f16v acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  // operand reads in inline asm: the compiler's own wait for them would be vmcnt(0) (it cannot
  // tell the operand images from the Σ DMA still in flight)
  float av[kSteps], bv[kSteps];
  {
    typedef __attribute__((address_space(3))) float lds_f;
    const unsigned ka = static_cast<unsigned>(reinterpret_cast<size_t>((lds_f*)(Ki + kr * 32 + kcol)));
    const unsigned ma = static_cast<unsigned>(reinterpret_cast<size_t>((lds_f*)(Mi + kr * 32 + kcol)));
#pragma unroll
    for (int s2 = 0; s2 < kSteps; ++s2) {
      asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(av[s2]) : "v"(ka), "i"(256 * s2));
      asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(bv[s2]) : "v"(ma), "i"(256 * s2));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s2 = 0; s2 < kSteps; ++s2) {
    const bool live = 2 * s2 < kw;
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(live ? av[s2] : 0.0f, live ? bv[s2] : 0.0f, acc, 0, 0, 0);
  }
  if (!SIG_REGS) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < 16; ++r) sv[r] = Si[((r & 3) + 8 * (r >> 2) + 4 * kr) * 32 + kcol];
  }
  const auto rout = Tile::panel(A.sig[1], n, ld, R0);
  const float q = static_cast<float>(A.q);
  const int col = C0 + kcol;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = R0 + (r & 3) + 8 * (r >> 2) + 4 * kr;
    float v = sv[r] - acc[r];
    if (first && row == col && row < 3) v += q;
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rout,
                                          so + ((r & 3) + 8 * (r >> 2)) * rstride, 0, 0);
  }
}
template <int WPB, bool SIG_REGS>
void launch_glds(const PassArgs<float>& a, hipStream_t s) {
  const int trows = (a.n + 31) / 32, tcols = trows;
  hipLaunchKernelGGL((k_lab_glds<WPB, SIG_REGS>), dim3(8 * ((region_tiles(trows, tcols) + WPB - 1) / WPB)),
                     dim3(64 * WPB), 0, s, a, tcols);
}

template <int WPB, int PRIO>
void launch_region(const PassArgs<float>& a, hipStream_t s) {
  const int trows = (a.n + 31) / 32, tcols = (a.n + 31) / 32;
  hipLaunchKernelGGL((k_lab_region<WPB, PRIO>), dim3(8 * ((region_tiles(trows, tcols) + WPB - 1) / WPB)),
                     dim3(64 * WPB), 0, s, a, tcols);
}

template <typename V>
__global__ void k_copy(const V* __restrict__ in, V* __restrict__ out, size_t nv) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += gridDim.x * blockDim.x) out[i] = in[i];
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 1024, reps = argc > 2 ? atoi(argv[2]) : 200;
  const int n = 3 + 2 * N, ld = (n + 31) / 32 * 32, ldk = (n + 63) / 64 * 64;
  const size_t stride = static_cast<size_t>(n) * ld;
  float *S0, *S1, *kc, *mc;
  CK(hipMalloc(&S0, stride * 4));
  CK(hipMalloc(&S1, stride * 4));
  CK(hipMalloc(&kc, static_cast<size_t>(kMaxKW) * ldk * 4));
  CK(hipMalloc(&mc, static_cast<size_t>(kMaxKW) * ldk * 4));
  {
    std::vector<float> h(stride);
    srand(7);
    for (auto& v : h) v = (rand() % 100000) * 1e-3f;
    CK(hipMemcpy(S0, h.data(), stride * 4, hipMemcpyHostToDevice));
    std::vector<float> k(static_cast<size_t>(kMaxKW) * ldk);
    for (auto& v : k) v = (rand() % 2000 - 1000) * 1e-4f;
    CK(hipMemcpy(kc, k.data(), k.size() * 4, hipMemcpyHostToDevice));
    for (auto& v : k) v = (rand() % 2000 - 1000) * 1e-4f;
    CK(hipMemcpy(mc, k.data(), k.size() * 4, hipMemcpyHostToDevice));
  }
  MsgDesc hd;
  std::memset(&hd, 0, sizeof hd);
  hd.m = 16;
  hd.flags = kActive | kFirst;
  MsgDesc* dd;
  CK(hipMalloc(&dd, sizeof(MsgDesc)));
  CK(hipMemcpy(dd, &hd, sizeof hd, hipMemcpyHostToDevice));
  PassArgs<float> a{};
  a.sig[0] = S0; a.sig[1] = S1; a.sig_stride = stride;
  a.kcat = kc; a.mcat = mc; a.km_stride = static_cast<size_t>(kMaxKW) * ldk; a.ldk = ldk;
  a.desc = dd; a.n = n; a.ld = ld; a.N = N; a.q = 1e-2;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = 2.0 * n * n * 4;
  std::vector<float> ref(stride), out(stride);
  auto prod = [&](hipStream_t st) {
    const int trows = (n + 31) / 32, tcols = trows;
    hipLaunchKernelGGL((k_sigma_pass<float, false>), dim3(8 * ((region_tiles(trows, tcols) + 3) / 4), 1),
                       dim3(256), 0, st, a, tcols, -1, 1);
  };
  struct V { const char* name; void (*fn)(const PassArgs<float>&, hipStream_t); };
  auto time_it = [&](const char* name, auto&& fn) {
    CK(hipMemset(S1, 0, stride * 4));
    for (int i = 0; i < 5; ++i) fn(s);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(out.data(), S1, stride * 4, hipMemcpyDeviceToHost));
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
    size_t bad = 0;
    for (int r = 0; r < n; ++r)
      for (int c = 0; c < n; ++c)
        if (std::memcmp(&out[static_cast<size_t>(r) * ld + c], &ref[static_cast<size_t>(r) * ld + c], 4)) ++bad;
    printf("%-22s %7.2f us (best of 3; mean %7.2f)  %6.0f GB/s  frac %.3f  mismatches %zu\n", name,
           best * 1e3 / reps, sum / 3 * 1e3 / reps, bytes / (best / reps * 1e-3) / 1e9,
           bytes / (best / reps * 1e-3) / 8e12, bad);
  };
  // reference output
  prod(s);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(ref.data(), S1, stride * 4, hipMemcpyDeviceToHost));
  {
    using F4 = float4;
    const size_t nv = stride * 4 / sizeof(F4);
    time_it("copy float4", [&](hipStream_t st) {
      hipLaunchKernelGGL(k_copy<F4>, dim3(4096), dim3(256), 0, st, (const F4*)S0, (F4*)S1, nv);
    });
  }
  for (int round = 0; round < 2; ++round) {
    time_it("product k_sigma_pass", prod);
    time_it("region wpb4", [&](hipStream_t st) { launch_region<4, 0>(a, st); });
    time_it("glds ops, sig regs", [&](hipStream_t st) { launch_glds<4, true>(a, st); });
    time_it("glds ops + sig", [&](hipStream_t st) { launch_glds<4, false>(a, st); });
    time_it("glds ops, sig regs w2", [&](hipStream_t st) { launch_glds<2, true>(a, st); });
    time_it("glds ops + sig w2", [&](hipStream_t st) { launch_glds<2, false>(a, st); });
  }
  return 0;
}
