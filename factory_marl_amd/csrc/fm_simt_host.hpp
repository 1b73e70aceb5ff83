// fm_simt_host.hpp -- the host side of the CPU backend (fm_create(..., device = -1)): the env-step kernel's own
// sources (fm_device.hpp) compiled for the host, with the wave they were written for emulated.
//
// One arena is one 64-lane wavefront.  On the host each lane is a fiber with its own stack; the lanes of a wave run
// one after another until each reaches the next cross-lane point -- a wave barrier (SYNC / FULL_SYNC), a DPP move,
// v_readlane, ds_bpermute, a ballot, an MFMA -- where the emulator resolves the operation over the 64 deposited
// operands and resumes lane 0.  Between two such points a lane's memory effects are complete before the next lane
// runs, which is the ordering the kernel's SYNC() contract gives on the GPU (lanes hand data to each other only at
// those points).  Every lane of a wave must reach the same cross-lane operation (the kernel calls them with the
// full wave active); a mismatch is reported and aborts, as a divergent DPP or ballot would be undefined on the GPU.
// Lanes that have returned take no part (a ballot sees 0 from them).  LDS is one per-thread buffer; LDS atomics
// are plain read-modify-writes (one lane runs at a time).  Arenas are independent: fm_cpu.cpp spreads them over
// host threads.
#pragma once
#ifndef FM_HOST_SIMT
#error "fm_simt_host.hpp is the host emulation layer (compile with -DFM_HOST_SIMT)"
#endif
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __noinline__ __attribute__((noinline))
#define __launch_bounds__(...)
#define __shared__

namespace fm_simt {

constexpr int W = 64;
struct Dim3 {
  unsigned x, y, z;
};

// cross-lane operations
enum Op : int { OP_BARRIER = 1, OP_READLANE, OP_READFIRST, OP_DPP, OP_BPERMUTE, OP_BALLOT, OP_MFMA };

struct Wave {
  void* sp[W];       // saved stack pointers of the lane fibers
  void* sched_sp;    // the scheduler's
  char* stacks;      // W fiber stacks
  size_t stack_bytes;
  int lane;          // the running lane
  bool done[W];
  int op[W];
  int64_t a0[W];     // per-lane operand (32 or 64 bits)
  int64_t a1[W];     // per-lane second operand (DPP old value, bpermute address, readlane lane)
  int ctrl[W];       // DPP control / readlane lane (must agree over the wave)
  int line[W];       // source line of the operation (diagnostics)
  float mf_a[W], mf_b[W], mf_c[W][4], mf_d[W][4];
  int64_t out[W];
  void (*entry)(void*);
  void* entry_arg;
  const void* kernarg;  // StepParams of the launch (kparams)
  Dim3 block, grid;
  char* lds;
  size_t lds_bytes;
  unsigned epoch;  // cross-lane rendezvous count of the running block (the race detector's phases)
};

Wave& wave();
int64_t cross(int op, int64_t a0, int64_t a1, int ctrl, int line = 0);  // deposit, rendezvous, result
void mfma_16x16x4(float a, float b, const float* c, float* d);
// a grid of `grid` emulated workgroups (fm_cpu.cpp), each lane running body(kernarg): the launch entry of the
// compile-time scene objects (fm_cpu_fixed.cpp)
void launch_kernel(unsigned grid, size_t lds_bytes, const void* kernarg, void (*body)(const void*));

inline int lane() { return wave().lane; }
inline Dim3 thread_idx() { return Dim3{(unsigned)lane(), 0u, 0u}; }

inline int readlane_i(int v, int l, int line = 0) { return (int)cross(OP_READLANE, (int64_t)(uint32_t)v, 0, l, line); }
// v_readfirstlane: the kernel applies it only to values uniform over the wave (the arena index, tree masks read from
// LDS), also inside lane-divergent code -- the lane's own copy is the value, no rendezvous
inline int readfirst_i(int v, int line = 0) {
  (void)line;
  return v;
}
inline int dpp_i(int old, int src, int ctrl) {
  return (int)cross(OP_DPP, (int64_t)(uint32_t)src, (int64_t)(uint32_t)old, ctrl);
}
inline int bpermute_i(int addr, int src) { return (int)cross(OP_BPERMUTE, (int64_t)(uint32_t)src, addr, 0); }
inline unsigned long long ballot(bool p, int line = 0) {
  return (unsigned long long)cross(OP_BALLOT, p ? 1 : 0, 0, 0, line);
}
inline void barrier(int line = 0) { (void)cross(OP_BARRIER, 0, 0, 0, line); }

inline unsigned long long wall_clock() {
  return (unsigned long long)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

}  // namespace fm_simt

#define threadIdx (::fm_simt::thread_idx())
#define blockIdx (::fm_simt::wave().block)
#define gridDim (::fm_simt::wave().grid)

// the AMDGPU builtins the kernel uses
#define __builtin_amdgcn_readlane(v, l) ::fm_simt::readlane_i((v), (l), __LINE__)
#define __builtin_amdgcn_readfirstlane(v) ::fm_simt::readfirst_i((v), __LINE__)
#define __builtin_amdgcn_update_dpp(old, src, ctrl, rm, bm, bc) ::fm_simt::dpp_i((old), (src), (ctrl))
#define __builtin_amdgcn_ds_bpermute(addr, src) ::fm_simt::bpermute_i((addr), (src))
#define __builtin_amdgcn_wave_barrier() ::fm_simt::barrier(__LINE__)
#define __builtin_amdgcn_fence(order, scope) ((void)0)
#define __builtin_amdgcn_kernarg_segment_ptr() (::fm_simt::wave().kernarg)
#define __builtin_amdgcn_mbcnt_lo(m, acc)                                                                   \
  ((unsigned)(acc) + (unsigned)__builtin_popcount((unsigned)(m) & (::fm_simt::lane() >= 32 ? 0xffffffffu   \
                                                                  : ((1u << ::fm_simt::lane()) - 1u))))
#define __builtin_amdgcn_mbcnt_hi(m, acc)                                                                   \
  ((unsigned)(acc) + (unsigned)__builtin_popcount((unsigned)(m) & (::fm_simt::lane() < 32 ? 0u              \
                                                                  : ((1u << (::fm_simt::lane() - 32)) - 1u))))

#define __syncthreads() ::fm_simt::barrier(__LINE__)
inline unsigned long long wall_clock64() { return ::fm_simt::wall_clock(); }

// HIP device helpers
inline int __float_as_int(float x) {
  int i;
  std::memcpy(&i, &x, 4);
  return i;
}
inline float __int_as_float(int i) {
  float x;
  std::memcpy(&x, &i, 4);
  return x;
}
inline long long __double_as_longlong(double x) {
  long long i;
  std::memcpy(&i, &x, 8);
  return i;
}
inline double __longlong_as_double(long long i) {
  double x;
  std::memcpy(&x, &i, 8);
  return x;
}
inline int __popc(unsigned x) { return __builtin_popcount(x); }
inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
inline int __ffsll(unsigned long long x) { return __builtin_ffsll((long long)x); }
inline int __ffsll(long long x) { return __builtin_ffsll(x); }
inline unsigned long long __umul64hi(unsigned long long a, unsigned long long b) {
  return (unsigned long long)(((unsigned __int128)a * b) >> 64);
}
#define __ballot(p) ::fm_simt::ballot((p) != 0, __LINE__)

inline int __shfl(int v, int l, int width = 64) {
  (void)width;
  return ::fm_simt::bpermute_i((l & 63) << 2, v);
}
inline unsigned __shfl(unsigned v, int l, int width = 64) { return (unsigned)__shfl((int)v, l, width); }
inline float __shfl(float v, int l, int width = 64) { return __int_as_float(__shfl(__float_as_int(v), l, width)); }
inline double __shfl(double v, int l, int width = 64) {
  const long long b = __double_as_longlong(v);
  const int lo = __shfl((int)(b & 0xffffffffll), l, width), hi = __shfl((int)(b >> 32), l, width);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
inline long long __shfl(long long v, int l, int width = 64) {
  const int lo = __shfl((int)(v & 0xffffffffll), l, width), hi = __shfl((int)(v >> 32), l, width);
  return ((long long)hi << 32) | (unsigned)lo;
}
inline unsigned long long __shfl(unsigned long long v, int l, int width = 64) {
  return (unsigned long long)__shfl((long long)v, l, width);
}
template <typename X>
inline X __shfl_xor(X v, int m, int width = 64) {
  return __shfl(v, ::fm_simt::lane() ^ m, width);
}

// atomics: one lane runs at a time (and one wave per host thread), so a read-modify-write is atomic (and exempt from
// the LDS race detector, FM_RACE_DETECT)
#define FM_NO_TSAN __attribute__((no_sanitize("thread")))
template <typename X, typename Y>
FM_NO_TSAN inline X atomicAdd(X* p, Y v) {
  const X o = *p;
  *p = (X)(o + (X)v);
  return o;
}
template <typename X, typename Y>
FM_NO_TSAN inline X atomicMax(X* p, Y v) {
  const X o = *p;
  if ((X)v > o) *p = (X)v;
  return o;
}
template <typename X, typename Y>
FM_NO_TSAN inline X atomicOr(X* p, Y v) {
  const X o = *p;
  *p = (X)(o | (X)v);
  return o;
}

// the MFMA builtin: v_mfma_f32_16x16x4_f32 over the wave (A: lane l gives A[l % 16][l / 16]; B: B[l / 16][l % 16];
// C / D: lane l holds rows 4 (l / 16) .. + 3 of column l % 16)
typedef float fm_host_f32x4 __attribute__((ext_vector_type(4)));
inline fm_host_f32x4 fm_host_mfma(float a, float b, fm_host_f32x4 c) {
  float cc[4] = {c[0], c[1], c[2], c[3]}, dd[4];
  ::fm_simt::mfma_16x16x4(a, b, cc, dd);
  fm_host_f32x4 d = {dd[0], dd[1], dd[2], dd[3]};
  return d;
}
#define __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, x, y, z) fm_host_mfma((a), (b), (c))

// HIP vector types the kernel uses
struct uint4 {
  unsigned x, y, z, w;
};
inline uint4 make_uint4(unsigned a, unsigned b, unsigned c, unsigned d) { return uint4{a, b, c, d}; }
