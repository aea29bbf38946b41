// Device helpers shared by the filter kernels (ekf_kernels.hip, ekf_assoc.hip): the cross-queue /
// inter-workgroup hand-off protocol and buffer-descriptor loads. Included inside namespace ekfslam.
#pragma once

// ---- cross-queue hand-offs (chain on the main stream, factors + Σ pass on the bulk stream) ----
// Protocol of cdna_hip_programming.md §6 Guideline 16: the producer stores its payload write-through
// (sc1), every storing wave drains (s_waitcnt vmcnt(0)), a workgroup barrier, then ONE lane stores
// or adds to an agent-scope epoch word; the consumer polls that word relaxed, takes ONE agent
// acquire, drains, barriers, then loads plainly. Polls are bounded (EKF_FLAG_TIMEOUT).
#define EKF_FLAG_TIMEOUT_D 4u
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

__device__ __forceinline__ unsigned epoch_load(const unsigned* p) {
  return __hip_atomic_load((const gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void epoch_store(unsigned* p, unsigned v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// One lane: wait until the epoch word reaches v (wrap-safe), then acquire. false on timeout.
__device__ __noinline__ bool epoch_wait_acquire(const unsigned* p, unsigned v) {
  bool ok = false;
  for (unsigned i = 0; i < (1u << 22); ++i) {
    if (static_cast<int>(epoch_load(p) - v) >= 0) {
      ok = true;
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return ok;
}
// A poll that timed out leaves the filter's state undefined (a hand-off was not seen): its status
// gets EKF_FLAG_TIMEOUT and the handle's host-mapped fatal word is set, which the host reports as
// EKF_E_TIMEOUT at its next synchronising call (a vector store of a constant to system scope: no RMW
// across PCIe).
__device__ __forceinline__ void flag_timeout(unsigned* status, unsigned* fatal) {
  atomicOr(status, EKF_FLAG_TIMEOUT_D);
  if (fatal) __hip_atomic_store(fatal, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// write-through stores of hand-off payload
__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store((gu64*)p, static_cast<unsigned long long>(__double_as_longlong(v)),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store((gu32*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-byte write-through store (buffer store, cache policy sc1) at byte offset `off` of `r`
__device__ __forceinline__ void st_wt2(__amdgpu_buffer_rsrc_t r, int off, double a, double b) {
  typedef int i4 __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i4, make_double2(a, b)), r, off, 0, 16);
}
__device__ __forceinline__ void st_wt(int* p, int v) {
  __hip_atomic_store((gu32*)p, static_cast<unsigned>(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// Buffer loads (32-bit offsets; a load past the descriptor's size returns 0 and touches nothing)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
__device__ __forceinline__ float ld_f32(__amdgpu_buffer_rsrc_t r, unsigned vo, unsigned so) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
}
typedef unsigned u2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double ld_f64(__amdgpu_buffer_rsrc_t r, unsigned vo, unsigned so) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0));
}
__device__ __forceinline__ float ld_t(__amdgpu_buffer_rsrc_t r, unsigned vo, float) {
  return ld_f32(r, vo, 0);
}
__device__ __forceinline__ double ld_t(__amdgpu_buffer_rsrc_t r, unsigned vo, double) {
  return ld_f64(r, vo, 0);
}

