// fm_device.hpp -- the MI355X env-step pipeline (device code; kernels instantiated by fm_api.hip for
// runtime dims and by fm_fixed.hip once per compile-time scene): one workgroup (= one 64-lane wavefront) per arena.
//
// One launch advances every arena by one env-step of the reference
// (FactoryManipulationEnv.step -> BaseEnv.step_sim, environments.py:151-202, base_env.py:240-282):
//   AllFullRL action transform (environments.py:84-102, 481-495) and ctrl clipping (base_env.py:255-262)
//   frame_skip (=100) x [ low-pass ctrl target (base_env.py:209-215) ; dm_control legacy physics.step()
//                         = mj_step2 (actuation, smooth acceleration, Newton constraint solve, implicitfast
//                           integration) ; mj_step1 (FK, inertia, collision, constraints, bias forces) ]
//   contact-force termination (base_env.py:225-236), TaskManager.step (task_utils.py:131-144),
//   speed / spawn-rate updates (base_env.py:266-270), progress or score reward (environments.py:129-149,
//   342-383), observation (environments.py:55-82), SB3-style auto-reset (reset_sim, base_env.py:177-198).
// The arena's whole working set (state, body poses, contacts, Jacobian blocks, Newton Hessian) lives in
// LDS for the duration of the env-step; HBM is touched only for the per-arena state record, the
// action / observation rows and the (L2-resident) scene tables.
//
// Lane mapping: sequential chains run on few lanes (one lane per arm for FK + RNE, lane 0 for the task
// layer); everything with natural width runs across the wave (geoms, broadphase pairs, narrowphase,
// contact rows, Hessian entries, Cholesky trailing updates, line-search reductions).
#pragma once
#ifndef FM_HOST_SIMT
#include <hip/hip_runtime.h>
#endif

#include <cmath>
#include <type_traits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/factorysim.h"
#include "fm_dev.hpp"
#include "fm_scene.hpp"
#include "fm_arm_table.hpp"  // generated (gen_tables.cpp)
#include "fm_ik.hpp"

#ifndef FM_WS_RUNTIME_LAYOUT
#define FM_WS_RUNTIME_LAYOUT 0
#endif

namespace fm {

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E) -- every index is a constant in the body
// (a register array indexed through it stays in registers however large the body)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// The lane index, opaque at each use: lane-derived values (per-lane LDS offsets, lane masks, LANE / 3, LANE % 9, ...)
// are recomputed where they are used instead of being hoisted out of the substep loop by the compiler -- hoisted,
// the (2,4) kernel held ~65 of them live across the whole env-step and spilled them to scratch at two waves per
// SIMD (a scratch reload per use instead of one VALU op).  FM_OPAQUE_LANE=0: the plain threadIdx.x.
#ifndef FM_OPAQUE_LANE
#define FM_OPAQUE_LANE 1
#endif
// a uniform int the compiler must re-read at each use (not hoisted: see the record macros of step_arena)
__device__ __forceinline__ int opaque_uniform(int x) {
  x = __builtin_amdgcn_readfirstlane(x);  // uniform by contract (one arena per wave)
  FM_OPAQUE_S(x);
  return x;
}
__device__ __forceinline__ int lane_id() {
  int t = (int)threadIdx.x;
#if FM_OPAQUE_LANE
  FM_OPAQUE_V(t);
#endif
  return t;
}
#define LANE (::fm::lane_id())
// A workgroup is exactly one wave.  Lanes hand data to each other through LDS at SYNC(): a
// wavefront-scope release fence, the wave barrier, a wavefront-scope acquire fence.  The fences order
// every memory access before the barrier ahead of every access after it (the compiler may not move LDS
// or global accesses across them, nor forward a stored value past them); at wavefront scope they need no
// s_waitcnt and no s_barrier, since a wave's LDS instructions execute in issue order.
// FULL_SYNC() (a real workgroup barrier with memory fences) is kept where lanes hand data to each
// other through GLOBAL memory: the lane-0 task layer's records read back by the observation writer.
#define SYNC()                                              \
  do {                                                      \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  \
    __builtin_amdgcn_wave_barrier();                        \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  \
  } while (0)
#define FULL_SYNC() __syncthreads()

template <typename T, typename DIM>
struct Ws {
  char* base;
  const Lay* L;
  char* gbase = nullptr;  // DimsSpill: this arena's global scratch block (H, contact records)
  __device__ __forceinline__ T* q() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.q);
    } else {
      return (T*)(base + L->q);
    }
  }
  __device__ __forceinline__ T* v() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.v);
    } else {
      return (T*)(base + L->v);
    }
  }
  __device__ __forceinline__ double* a() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (double*)(base + c.a);
    } else {
      return (double*)(base + L->a);
    }
  }
  __device__ __forceinline__ T* as() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.as);
    } else {
      return (T*)(base + L->as);
    }
  }
  __device__ __forceinline__ T* fs() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.fs);
    } else {
      return (T*)(base + L->fs);
    }
  }
  __device__ __forceinline__ T* fc() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.fc);
    } else {
      return (T*)(base + L->fc);
    }
  }
  __device__ __forceinline__ T* pb() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.pb);
    } else {
      return (T*)(base + L->pb);
    }
  }
  __device__ __forceinline__ double* g() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (double*)(base + c.g);
    } else {
      return (double*)(base + L->g);
    }
  }
  __device__ __forceinline__ T* dir() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.dir);
    } else {
      return (T*)(base + L->dir);
    }
  }
  __device__ __forceinline__ double* Ma() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (double*)(base + c.Ma);
    } else {
      return (double*)(base + L->Ma);
    }
  }
  __device__ __forceinline__ double* tmp() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (double*)(base + c.tmp);
    } else {
      return (double*)(base + L->tmp);
    }
  }
  __device__ __forceinline__ T* tblk() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.tblk);
    } else {
      return (T*)(base + L->tblk);
    }
  }
  // the tree-block solve's coupled system (LDS after the per-tree blocks, or the arena's global block: gl_tbr)
  __device__ __forceinline__ T* tbr() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      if constexpr (DIM::template gl_tbr<sizeof(T)>())
        return (T*)(gbase + c.tbr);
      else
        return (T*)(base + c.tblk) + tb_rest(DIM::ntree);
    } else {
      return (T*)(base + L->tblk);  // runtime dims have no tree-block solve (never called)
    }
  }
  __device__ __forceinline__ T* fa() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.fa);
    } else {
      return (T*)(base + L->fa);
    }
  }
  __device__ __forceinline__ double* ctrl() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (double*)(base + c.ctrl);
    } else {
      return (double*)(base + L->ctrl);
    }
  }
  __device__ __forceinline__ double* qd() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (double*)(base + c.qd);
    } else {
      return (double*)(base + L->qd);
    }
  }
  __device__ __forceinline__ double* bposd() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (double*)((DIM::f64gl ? gbase : base) + c.bposd);
    } else {
      return (double*)(base + L->bposd);
    }
  }
  __device__ __forceinline__ double* bRd() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (double*)((DIM::f64gl ? gbase : base) + c.bRd);
    } else {
      return (double*)(base + L->bRd);
    }
  }
  __device__ __forceinline__ double* vd() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (double*)(base + c.vd);
    } else {
      return (double*)(base + L->vd);
    }
  }
  __device__ __forceinline__ T* aforce() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.aforce);
    } else {
      return (T*)(base + L->aforce);
    }
  }
  __device__ __forceinline__ T* bpos() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.bpos);
    } else {
      return (T*)(base + L->bpos);
    }
  }
  __device__ __forceinline__ T* bR() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.bR);
    } else {
      return (T*)(base + L->bR);
    }
  }
  __device__ __forceinline__ T* bcom() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.bcom);
    } else {
      return (T*)(base + L->bcom);
    }
  }
  __device__ __forceinline__ T* bIw() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.bIw);
    } else {
      return (T*)(base + L->bIw);
    }
  }
  __device__ __forceinline__ T* bF() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.bF);
    } else {
      return (T*)(base + L->bF);
    }
  }
  __device__ __forceinline__ T* bN() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.bN);
    } else {
      return (T*)(base + L->bN);
    }
  }
  __device__ __forceinline__ T* dax() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.dax);
    } else {
      return (T*)(base + L->dax);
    }
  }
  __device__ __forceinline__ T* danc() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.danc);
    } else {
      return (T*)(base + L->danc);
    }
  }
  __device__ __forceinline__ T* site() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.site);
    } else {
      return (T*)(base + L->site);
    }
  }
  __device__ __forceinline__ T* cR() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.cR);
    } else {
      return (T*)(base + L->cR);
    }
  }
  __device__ __forceinline__ T* Marm() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.Marm);
    } else {
      return (T*)(base + L->Marm);
    }
  }
  __device__ __forceinline__ uint32_t* mcache() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (uint32_t*)(base + c.mcache);
    } else {
      return (uint32_t*)(base + L->mcache);
    }
  }
  __device__ __forceinline__ T* mpos() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.mpos);
    } else {
      return (T*)(base + L->mpos);
    }
  }
  __device__ __forceinline__ T* gx() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)((DIM::template gl_gx<sizeof(T)>() ? gbase : base) + c.gx);
    } else {
      return (T*)(base + L->gx);
    }
  }
  __device__ __forceinline__ int* ginfo() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (int*)(base + c.ginfo);
    } else {
      return (int*)(base + L->ginfo);
    }
  }
  __device__ __forceinline__ int* cbi() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (int*)(base + c.cbi);
    } else {
      return (int*)(base + L->cbi);
    }
  }
  __device__ __forceinline__ T* cbw() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.cbw);
    } else {
      return (T*)(base + L->cbw);
    }
  }
  __device__ __forceinline__ uint16_t* cbg() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (uint16_t*)(base + c.cbg);
    } else {
      return (uint16_t*)(base + L->cbg);
    }
  }
  __device__ __forceinline__ uint32_t* sp() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (uint32_t*)((DIM::template gl_sp<sizeof(T)>() ? gbase : base) + c.sp);
    } else {
      return (uint32_t*)(base + L->sp);
    }
  }
  __device__ __forceinline__ uint32_t* gsurv() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (uint32_t*)(base + c.gsurv);
    } else {
      return (uint32_t*)(base + L->gsurv);
    }
  }
  __device__ __forceinline__ T* stage() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)((DIM::template gl_coll<sizeof(T)>() ? gbase : base) + c.stage);
    } else {
      return (T*)(base + L->stage);
    }
  }
  __device__ __forceinline__ int* skey() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (int*)((DIM::template gl_coll<sizeof(T)>() ? gbase : base) + c.skey);
    } else {
      return (int*)(base + L->skey);
    }
  }
  __device__ __forceinline__ uint32_t* spw() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (uint32_t*)((DIM::template gl_coll<sizeof(T)>() ? gbase : base) + c.spw);
    } else {
      return (uint32_t*)(base + L->spw);
    }
  }
  __device__ __forceinline__ T* cube() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.cube);
    } else {
      return (T*)(base + L->cube);
    }
  }
  __device__ __forceinline__ T* H() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)((DIM::spill ? gbase : base) + c.H);
    } else if constexpr (DIM::spill) {
      return (T*)(gbase + L->H);
    } else {
      return (T*)(base + L->H);
    }
  }
  __device__ __forceinline__ int* ci() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (int*)(base + c.c_i);
    } else {
      return (int*)(base + L->c_i);
    }
  }
  __device__ __forceinline__ T* cr() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)((DIM::spill ? gbase : base) + c.c_r);
    } else if constexpr (DIM::spill) {
      return (T*)(gbase + L->c_r);
    } else {
      return (T*)(base + L->c_r);
    }
  }
  __device__ __forceinline__ int* ri() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (int*)(base + c.r_i);
    } else {
      return (int*)(base + L->r_i);
    }
  }
  __device__ __forceinline__ T* rr() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.r_r);
    } else {
      return (T*)(base + L->r_r);
    }
  }
  __device__ __forceinline__ uint64_t* tmask() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (uint64_t*)(base + c.tmask);
    } else {
      return (uint64_t*)(base + L->tmask);
    }
  }
  __device__ __forceinline__ int* misc() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (int*)(base + c.misc);
    } else {
      return (int*)(base + L->misc);
    }
  }
  __device__ __forceinline__ int* sortidx() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (int*)(base + c.sort);
    } else {
      return (int*)(base + L->sort);
    }
  }
  __device__ __forceinline__ double* uctl() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (double*)(base + c.uctl);
    } else {
      return (double*)(base + L->uctl);
    }
  }
  __device__ __forceinline__ double* scal() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (double*)(base + c.scal);
    } else {
      return (double*)(base + L->scal);
    }
  }
  __device__ __forceinline__ T* bc() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (T*)(base + c.bc);
    } else {
      return (T*)(base + L->bc);
    }
  }
  __device__ __forceinline__ unsigned long long* prof() const {
    if constexpr (DIM::fixed && !FM_WS_RUNTIME_LAYOUT) {
      constexpr Lay c = DIM::template layout<sizeof(T)>();
      return (unsigned long long*)((DIM::template gl_coll<sizeof(T)>() && DIM::A == 4 ? gbase : base) + c.prof);
    } else {
      return (unsigned long long*)(base + L->prof);
    }
  }
};

// optional phase profile: lane 0 charges the wall-clock time since the previous mark to phase k
#define PMARK(k)                                                   \
  do {                                                             \
    if (M.prof) {                                                  \
      SYNC();                                                      \
      if (LANE == 0) {                                             \
        unsigned long long _n = wall_clock64();                    \
        unsigned long long* _p = w.prof();                         \
        _p[k] += _n - _p[PH_LAST];                                 \
        _p[PH_LAST] = _n;                                          \
      }                                                            \
    }                                                              \
  } while (0)
template <typename T, typename DIM>
__device__ constexpr bool dense_mfma_chol();
// narrowphase split of the compile-time scenes without the dense Cholesky (whose sub-phase slots it borrows):
// PH_CHDIAG = geom-pair expansion, PH_CHPANEL = sphere / plane pairs, PH_CHTRAIL = box-box pairs
#ifndef FM_PROF_SPLIT
#define FM_PROF_SPLIT 0  // experiment builds only: 1 / 2 lend the narrowphase slots to sub-phases of rows + setup /
                         // gradient + line search (SPLITMARK below)
#endif
#define NPMARK(k)                                                                         \
  do {                                                                                    \
    if constexpr (FM_PROF_SPLIT == 0 && DIM::fixed && !dense_mfma_chol<T, DIM>()) PMARK(k); \
  } while (0)
#define SPLITMARK(v, k)                                                               \
  do {                                                                                \
    if constexpr (FM_PROF_SPLIT == (v) && DIM::fixed && !dense_mfma_chol<T, DIM>()) PMARK(k); \
  } while (0)

// ------------------------------------------------------------------------------------------------
// tree / dof helpers
// ------------------------------------------------------------------------------------------------
template <typename DD>
__device__ __forceinline__ int tree_dof(const DD& d, int t) {
  return t == 0 ? 0 : (t <= d.K ? 1 + 6 * (t - 1) : 1 + 6 * d.K + 9 * (t - 1 - d.K));
}
template <typename DD>
__device__ __forceinline__ int tree_nd(const DD& d, int t) { return t == 0 ? 1 : (t <= d.K ? 6 : 9); }
template <typename DD>
__device__ __forceinline__ int kbody_tree(const DD& d, int kb) {
  if (kb == 0) return -1;
  if (kb == 1) return 0;
  if (kb < 2 + d.K) return kb - 1;
  return 1 + d.K + (kb - 2 - d.K) / 10;
}
template <typename DD>
__device__ __forceinline__ int dof_tree(const DD& d, int i) {
  if (i == 0) return 0;
  if (i < 1 + 6 * d.K) return 1 + (i - 1) / 6;
  return 1 + d.K + (i - 1 - 6 * d.K) / 9;
}

// ------------------------------------------------------------------------------------------------
// impedance / reference acceleration parameters (MuJoCo getimpedance, getKBIP with refsafe)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void sincos_t(float x, float* s, float* c) { sincosf(x, s, c); }
__device__ __forceinline__ void sincos_t(double x, double* s, double* c) { sincos(x, s, c); }

// 1 / sqrt(s) in float64 for a pivot: v_rsq_f64 refined by two Newton steps (~1 ulp) -- a dependent chain of 7
// operations where sqrt() then a division is ~20 (both expand to refinement sequences)
__device__ __forceinline__ double rsqrt_f64(double s) {
#ifdef FM_HOST_SIMT
  return 1.0 / sqrt(s);
#else
  double y = __builtin_amdgcn_rsq(s);
  const double h = 0.5 * s;
  y = fma(y, fma(-h * y, y, 0.5), y);
  y = fma(y, fma(-h * y, y, 0.5), y);
  return y;
#endif
}
__device__ __forceinline__ float rsqrt_f64(float s) { return 1.0f / sqrtf(s); }
// a pivot's reciprocal square root in the factor's precision
template <typename T>
__device__ __forceinline__ T rsqrt_div(T d) {
  if constexpr (sizeof(T) == 4)
    return 1.0f / sqrtf(d);
  else
    return rsqrt_f64(d);
}

template <typename T>
__device__ __forceinline__ T impedance(const T* si, T x) {
  T dmin = si[0], dmax = si[1], width = si[2], mid = si[3], power = si[4];
  const T lo = T(0.0001), hi = T(0.9999);
  dmin = dmin < lo ? lo : (dmin > hi ? hi : dmin);
  dmax = dmax < lo ? lo : (dmax > hi ? hi : dmax);
  if (dmin == dmax || width <= T(1e-15)) return T(0.5) * (dmin + dmax);
  const T ax = fabs(x);
  if (power == T(2)) {  // every contact class of this scene (solimp power 2): x = |d| / width folded into one division
    if (ax >= width) return dmax;
    if (ax <= T(0)) return dmin;
    const T r = width - ax;
    const T y = ax <= mid * width ? ax * ax / (width * width * mid) : T(1) - r * r / (width * width * (T(1) - mid));
    return dmin + y * (dmax - dmin);
  }
  x = ax / width;
  if (x >= T(1)) return dmax;
  if (x <= T(0)) return dmin;
  T y;
  if (power == T(1))
    y = x;
  else if (x <= mid)
    y = pow(x, power) / pow(mid, power - T(1));
  else
    y = T(1) - pow(T(1) - x, power) / pow(T(1) - mid, power - T(1));
  return dmin + y * (dmax - dmin);
}

template <typename T>
__device__ __forceinline__ void kb_params(T dt, const T* solref, const T* solimp, T& K, T& B) {
  T tc = solref[0], dr = solref[1];
  T dmax = solimp[1];
  dmax = dmax < T(0.0001) ? T(0.0001) : (dmax > T(0.9999) ? T(0.9999) : dmax);
  if (tc > T(0)) {
    if (tc < T(2) * dt) tc = T(2) * dt;
    T k = dmax * dmax * tc * tc * dr * dr;
    T b = dmax * tc;
    K = T(1) / (k > T(1e-15) ? k : T(1e-15));
    B = T(2) / (b > T(1e-15) ? b : T(1e-15));
  } else {
    K = -tc / (dmax * dmax);
    B = -dr / dmax;
  }
}

// ------------------------------------------------------------------------------------------------
// narrowphase (definitions identical to oracle/collide.c; normal from geom1 to geom2)
// ------------------------------------------------------------------------------------------------
// Contacts are emitted straight into the LDS staging area (slot = LDS atomic), tagged with a key
// (canonical geom pair << 3 | index within the pair); collide() sorts them by key afterwards, so the
// contact order equals the oracle's pair order whatever order the lanes emitted in.
template <typename T>
struct Emit {
  T* st;         // staging [cap][8]: dist pos(3) n(3); pos relative to the pair's anchor (contact_anchor)
  int* keys;     // [cap]
  uint32_t* pw;  // [cap] type-ordered pair word (c1 | c2 << 12 | param << 24)
  int* cnt;
  int cap;
  int key;
  uint32_t pair;
  int sub;
  double o[3];   // the anchor in the kernel frame
  template <typename X>
  __device__ void operator()(X dist, X p0, X p1, X p2, X n0, X n1, X n2) {
    if (sub >= MAXPC) return;
    int s = atomicAdd(cnt, 1);
    if (s < cap) {
      T* r = st + 8 * s;
      r[0] = (T)dist;
      r[1] = (T)((double)p0 - o[0]);
      r[2] = (T)((double)p1 - o[1]);
      r[3] = (T)((double)p2 - o[2]);
      r[4] = (T)n0;
      r[5] = (T)n1;
      r[6] = (T)n2;
      keys[s] = key | sub;
      pw[s] = pair;
    }
    sub++;
  }
};

template <typename T, typename E>
__device__ __forceinline__ void np_plane_sphere(const T* c, T r, E& emit, T zs) {
  // floor plane: world origin (z = -zs in the kernel frame, zs = the build's zshift), normal +z (scene.xml:21)
  T dist = c[2] + zs - r;
  if (dist > T(0)) return;
  emit(dist, c[0], c[1], c[2] - (r + dist / T(2)), T(0), T(0), T(1));
}

template <typename T, typename E>
__device__ __forceinline__ void np_plane_box(const T* p, const T* R, const T* h, E& emit, T zs) {
  T dist = p[2] + zs;
  int cnt = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    T cl[3] = {(i & 1) ? h[0] : -h[0], (i & 2) ? h[1] : -h[1], (i & 4) ? h[2] : -h[2]};
    T cw[3];
    matvec3(R, cl, cw);
    T ld = cw[2];
    if (dist + ld > T(0) || ld > T(0) || cnt >= 4) continue;
    T cd = dist + ld;
    emit(cd, cw[0] + p[0], cw[1] + p[1], cw[2] + p[2] - cd / T(2), T(0), T(0), T(1));
    cnt++;
  }
}

template <typename T, typename E>
__device__ __forceinline__ void np_sphere_sphere(const T* c1, T r1, const T* c2, T r2, E& emit) {
  T n[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
  T len = sqrt(dot3(n, n));
  T dist = len - r1 - r2;
  if (dist > T(0)) return;
  if (len < T(1e-15)) {
    n[0] = 1;
    n[1] = n[2] = 0;
  } else {
    for (int k = 0; k < 3; k++) n[k] /= len;
  }
  T s = r1 + dist / T(2);
  emit(dist, c1[0] + n[0] * s, c1[1] + n[1] * s, c1[2] + n[2] * s, n[0], n[1], n[2]);
}

template <typename T, typename E>
__device__ __forceinline__ void np_sphere_box(const T* c, T r, const T* p, const T* R, const T* h, E& emit) {
  T d[3] = {c[0] - p[0], c[1] - p[1], c[2] - p[2]};
  T pl[3];
  mattvec3(R, d, pl);
  T q[3];
  bool inside = true;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    q[k] = pl[k] < -h[k] ? -h[k] : (pl[k] > h[k] ? h[k] : pl[k]);
    if (q[k] != pl[k]) inside = false;
  }
  T nl[3], dist;
  if (!inside) {
    T dl[3] = {q[0] - pl[0], q[1] - pl[1], q[2] - pl[2]};
    T len = sqrt(dot3(dl, dl));
    dist = len - r;
    if (dist > T(0)) return;
    for (int k = 0; k < 3; k++) nl[k] = dl[k] / len;
  } else {
    T a0 = h[0] - fabs(pl[0]), a1 = h[1] - fabs(pl[1]), a2 = h[2] - fabs(pl[2]);
    int best = 0;
    T bd = a0;
    if (a1 < bd) {
      bd = a1;
      best = 1;
    }
    if (a2 < bd) {
      bd = a2;
      best = 2;
    }
    T pb = best == 0 ? pl[0] : (best == 1 ? pl[1] : pl[2]);
    T sg = pb >= T(0) ? T(-1) : T(1);
    nl[0] = best == 0 ? sg : T(0);
    nl[1] = best == 1 ? sg : T(0);
    nl[2] = best == 2 ? sg : T(0);
    dist = -bd - r;
  }
  T n[3];
  matvec3(R, nl, n);
  T s = r + dist / T(2);
  emit(dist, c[0] + n[0] * s, c[1] + n[1] * s, c[2] + n[2] * s, n[0], n[1], n[2]);
}

// small register-resident 3-vectors (all selections by runtime index go through selects, never
// through indexed arrays, so nothing lands in scratch)
template <typename T>
struct V3 {
  T x, y, z;
};
template <typename T>
__device__ __forceinline__ V3<T> vcol(const T* R, int k) {
  return V3<T>{R[k], R[3 + k], R[6 + k]};
}
template <typename T>
__device__ __forceinline__ T vdot(const V3<T>& a, const V3<T>& b) {
  return a.x * b.x + a.y * b.y + a.z * b.z;
}
template <typename T>
__device__ __forceinline__ V3<T> vcross(const V3<T>& a, const V3<T>& b) {
  return V3<T>{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
template <typename T>
__device__ __forceinline__ V3<T> vsel(bool c, const V3<T>& a, const V3<T>& b) {
  return V3<T>{c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z};
}
template <typename T>
__device__ __forceinline__ V3<T> vpick(int i, const V3<T>& a, const V3<T>& b, const V3<T>& c) {
  return vsel(i == 0, a, vsel(i == 1, b, c));
}
template <typename T>
__device__ __forceinline__ T spick(int i, T a, T b, T c) {
  return i == 0 ? a : (i == 1 ? b : c);
}

// box1 vs box2: SAT over 15 axes; edge-edge -> one point; face -> the vertices of the intersection of
// the incident face with the reference face, enumerated as (1) incident vertices inside the reference
// rectangle, (2) reference corners inside the incident quad, (3) proper edge/side crossings, each kept
// if it penetrates (same definition as oracle/collide.c).  Normal from box1 to box2.
// one separating axis of the box-box SAT (ax 0-2: box1's axes, 3-5: box2's, 6-14: edge crossings A_i x B_j,
// normalised; false for a near-parallel edge pair): overlap ov and signed centre distance sd along u
template <typename T>
__device__ __forceinline__ bool bb_axis(int ax, const V3<T> (&A)[3], const V3<T> (&B)[3], const T* h1, const T* h2,
                                        const V3<T>& d, V3<T>& u, T& ov, T& sd) {
  if (ax < 3) {
    u = vpick(ax, A[0], A[1], A[2]);
  } else if (ax < 6) {
    u = vpick(ax - 3, B[0], B[1], B[2]);
  } else {
    const int i = (ax - 6) / 3, j = (ax - 6) % 3;
    u = vcross(vpick(i, A[0], A[1], A[2]), vpick(j, B[0], B[1], B[2]));
    const T n2 = vdot(u, u);
    if (n2 < T(1e-12)) return false;  // |u| < 1e-6
    const T ri = rsqrt_f64(n2);       // one reciprocal square root instead of a square root and three divisions
    u = V3<T>{u.x * ri, u.y * ri, u.z * ri};
  }
  T ra = h1[0] * fabs(vdot(u, A[0])) + h1[1] * fabs(vdot(u, A[1])) + h1[2] * fabs(vdot(u, A[2]));
  T rb = h2[0] * fabs(vdot(u, B[0])) + h2[1] * fabs(vdot(u, B[1])) + h2[2] * fabs(vdot(u, B[2]));
  sd = vdot(u, d);
  ov = ra + rb - fabs(sd);
  return true;
}

// the SAT's outcome: the best face axis (0-5) and the best edge axis (6-14, or -1)
template <typename T>
struct BBSat {
  int face_id, edge_id;
  V3<T> face_u, edge_u;
  T face_s, edge_s, best_face, best_edge;
};

// face contact of a box pair: the reference box owns the best face axis, the incident box's face most
// anti-parallel to it is clipped against the reference rectangle.  Setup (frames, the incident quad in reference
// coordinates u, v, w) and the 24 candidate points in the serial order: (1) incident vertices inside the rectangle
// (c 0-3), (2) reference corners inside the incident quad (c 4-7), (3) proper crossings of incident edge m with side sd
// (c = 8 + 4 m + sd).  A candidate that exists and penetrates (w <= 0) is a contact.
template <typename T>
struct BBFace {
  V3<T> n, nref, fc, ta, tb;
  T e1, e2, cu, cv, cw, det, ia, ib;
  T U[4], V[4], W[4];
};
template <typename T>
__device__ __forceinline__ T pick4(int k, const T (&x)[4]) {
  return k == 0 ? x[0] : (k == 1 ? x[1] : (k == 2 ? x[2] : x[3]));
}
template <typename T>
__device__ __forceinline__ BBFace<T> bb_face_setup(const T* p1, const T* R1, const T* h1, const T* p2, const T* R2,
                                                   const T* h2, const BBSat<T>& sat) {
  BBFace<T> F;
  const V3<T> A[3] = {vcol(R1, 0), vcol(R1, 1), vcol(R1, 2)};
  const V3<T> B[3] = {vcol(R2, 0), vcol(R2, 1), vcol(R2, 2)};
  const V3<T> P1{p1[0], p1[1], p1[2]}, P2{p2[0], p2[1], p2[2]};
  const int face_id = sat.face_id;
  const V3<T> face_u = sat.face_u;
  const T sg = sat.face_s >= T(0) ? T(1) : T(-1);
  const V3<T> n{face_u.x * sg, face_u.y * sg, face_u.z * sg};
  const bool ref1 = face_id < 3;
  const int kr = ref1 ? face_id : face_id - 3;
  const V3<T> Rr0 = vsel(ref1, A[0], B[0]), Rr1 = vsel(ref1, A[1], B[1]), Rr2 = vsel(ref1, A[2], B[2]);
  const V3<T> Ri0 = vsel(ref1, B[0], A[0]), Ri1 = vsel(ref1, B[1], A[1]), Ri2 = vsel(ref1, B[2], A[2]);
  const T hr0 = ref1 ? h1[0] : h2[0], hr1 = ref1 ? h1[1] : h2[1], hr2 = ref1 ? h1[2] : h2[2];
  const T hi0 = ref1 ? h2[0] : h1[0], hi1 = ref1 ? h2[1] : h1[1], hi2 = ref1 ? h2[2] : h1[2];
  const V3<T> pr = vsel(ref1, P1, P2), pi = vsel(ref1, P2, P1);
  const V3<T> nref = ref1 ? n : V3<T>{-n.x, -n.y, -n.z};
  const int t1 = (kr + 1) % 3, t2 = (kr + 2) % 3;
  const T hrk = spick(kr, hr0, hr1, hr2);
  const V3<T> fc{pr.x + nref.x * hrk, pr.y + nref.y * hrk, pr.z + nref.z * hrk};
  const V3<T> ta = vpick(t1, Rr0, Rr1, Rr2), tb = vpick(t2, Rr0, Rr1, Rr2);
  const T e1 = spick(t1, hr0, hr1, hr2), e2 = spick(t2, hr0, hr1, hr2);
  // incident face: the incident box axis most anti-parallel to nref
  const T dk0 = vdot(nref, Ri0), dk1 = vdot(nref, Ri1), dk2 = vdot(nref, Ri2);
  int mi = 0;
  T bestdot = fabs(dk0), dmi = dk0;
  if (fabs(dk1) > bestdot) {
    bestdot = fabs(dk1);
    mi = 1;
    dmi = dk1;
  }
  if (fabs(dk2) > bestdot) {
    mi = 2;
    dmi = dk2;
  }
  const T sgn = dmi > T(0) ? T(-1) : T(1);
  const int u1 = (mi + 1) % 3, u2 = (mi + 2) % 3;
  const T him = spick(mi, hi0, hi1, hi2), hu1 = spick(u1, hi0, hi1, hi2), hu2 = spick(u2, hi0, hi1, hi2);
  const V3<T> am = vpick(mi, Ri0, Ri1, Ri2), a1 = vpick(u1, Ri0, Ri1, Ri2), a2 = vpick(u2, Ri0, Ri1, Ri2);
  // incident face centre relative to the reference face centre, in reference coordinates (u, v, w)
  const V3<T> icr{pi.x + sgn * him * am.x - fc.x, pi.y + sgn * him * am.y - fc.y, pi.z + sgn * him * am.z - fc.z};
  const T cu = vdot(icr, ta), cv = vdot(icr, tb), cw = vdot(icr, nref);
  const T a1u = hu1 * vdot(a1, ta), a1v = hu1 * vdot(a1, tb), a1w = hu1 * vdot(a1, nref);
  const T a2u = hu2 * vdot(a2, ta), a2v = hu2 * vdot(a2, tb), a2w = hu2 * vdot(a2, nref);
  const T sx[4] = {1, -1, -1, 1}, sy[4] = {1, 1, -1, -1};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    F.U[k] = cu + sx[k] * a1u + sy[k] * a2u;
    F.V[k] = cv + sx[k] * a1v + sy[k] * a2v;
    F.W[k] = cw + sx[k] * a1w + sy[k] * a2w;
  }
  F.n = n;
  F.nref = nref;
  F.fc = fc;
  F.ta = ta;
  F.tb = tb;
  F.e1 = e1;
  F.e2 = e2;
  F.cu = cu;
  F.cv = cv;
  F.cw = cw;
  F.det = a1u * a2v - a2u * a1v;
  F.ia = a1w * a2v - a2w * a1v;
  F.ib = a1u * a2w - a2u * a1w;
  return F;
}
template <typename T>
__device__ __forceinline__ bool bb_face_candidate(const BBFace<T>& F, int c, T& u, T& v, T& w) {
  if (c < 4) {  // (1) incident vertex c
    u = pick4(c, F.U);
    v = pick4(c, F.V);
    w = pick4(c, F.W);
    return fabs(u) <= F.e1 && fabs(v) <= F.e2;
  }
  if (c < 8) {  // (2) reference corner c - 4, w on the incident plane
    const int k = c - 4;
    const T cu_ = (k == 0 || k == 3) ? F.e1 : -F.e1, cv_ = k < 2 ? F.e2 : -F.e2;
    bool in = F.det != T(0);
#pragma unroll
    for (int m = 0; m < 4; m++) {
      const int m1 = (m + 1) & 3;
      T cr = (F.U[m1] - F.U[m]) * (cv_ - F.V[m]) - (F.V[m1] - F.V[m]) * (cu_ - F.U[m]);
      in = in && (F.det >= T(0) ? cr > T(0) : cr < T(0));
    }
    u = cu_;
    v = cv_;
    w = F.cw + (F.ia * (cu_ - F.cu) + F.ib * (cv_ - F.cv)) / F.det;
    return in;
  }
  // (3) incident edge m (vertex m -> m + 1) crossing rectangle side sd (u = +e1, -e1, v = +e2, -e2)
  const int m = (c - 8) >> 2, sd = (c - 8) & 3, m1 = (m + 1) & 3;
  const bool onu = sd < 2;
  const T ss = (sd & 1) ? T(-1) : T(1);
  const T e = onu ? F.e1 : F.e2;
  const T Um = pick4(m, F.U), Um1 = pick4(m1, F.U), Vm = pick4(m, F.V), Vm1 = pick4(m1, F.V);
  const T Wm = pick4(m, F.W), Wm1 = pick4(m1, F.W);
  const T dp = e - ss * (onu ? Um : Vm);
  const T dq = e - ss * (onu ? Um1 : Vm1);
  if (!((dp > T(0) && dq < T(0)) || (dp < T(0) && dq > T(0)))) return false;
  const T f = dp / (dp - dq);
  u = Um + (Um1 - Um) * f;
  v = Vm + (Vm1 - Vm) * f;
  w = Wm + (Wm1 - Wm) * f;
  return onu ? fabs(v) <= F.e2 : fabs(u) < F.e1;
}
template <typename T, typename E>
__device__ __forceinline__ void bb_face_emit(const BBFace<T>& F, T u, T v, T w, E& emit) {
  const T hw = T(0.5) * w;
  emit(w, F.fc.x + u * F.ta.x + v * F.tb.x + hw * F.nref.x, F.fc.y + u * F.ta.y + v * F.tb.y + hw * F.nref.y,
       F.fc.z + u * F.ta.z + v * F.tb.z + hw * F.nref.z, F.n.x, F.n.y, F.n.z);
}

template <typename T, typename E>
__device__ __forceinline__ void np_box_box_finish(const T* p1, const T* R1, const T* h1, const T* p2, const T* R2,
                                                  const T* h2, const BBSat<T>& sat, E& emit);

template <typename T, typename E>
__device__ __forceinline__ void np_box_box(const T* p1, const T* R1, const T* h1, const T* p2, const T* R2,
                                           const T* h2, E& emit) {
  const V3<T> A[3] = {vcol(R1, 0), vcol(R1, 1), vcol(R1, 2)};
  const V3<T> B[3] = {vcol(R2, 0), vcol(R2, 1), vcol(R2, 2)};
  const V3<T> d{p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  BBSat<T> sat{-1, -1, V3<T>{0, 0, 0}, V3<T>{0, 0, 0}, T(0), T(0), T(1e30), T(1e30)};
#pragma unroll
  for (int ax = 0; ax < 15; ax++) {
    V3<T> u;
    T ov, sd;
    if (!bb_axis(ax, A, B, h1, h2, d, u, ov, sd)) continue;
    if (ov < T(0)) return;
    if (ax < 6) {
      if (ov < sat.best_face) {
        sat.best_face = ov;
        sat.face_id = ax;
        sat.face_u = u;
        sat.face_s = sd;
      }
    } else if (ov < sat.best_edge) {
      sat.best_edge = ov;
      sat.edge_id = ax;
      sat.edge_u = u;
      sat.edge_s = sd;
    }
  }
  np_box_box_finish(p1, R1, h1, p2, R2, h2, sat, emit);
}

template <typename T, typename E>
__device__ __forceinline__ void np_box_box_finish(const T* p1, const T* R1, const T* h1, const T* p2, const T* R2,
                                                  const T* h2, const BBSat<T>& sat, E& emit) {
  const V3<T> A[3] = {vcol(R1, 0), vcol(R1, 1), vcol(R1, 2)};
  const V3<T> B[3] = {vcol(R2, 0), vcol(R2, 1), vcol(R2, 2)};
  const V3<T> P1{p1[0], p1[1], p1[2]}, P2{p2[0], p2[1], p2[2]};
  const int face_id = sat.face_id, edge_id = sat.edge_id;
  const T best_face = sat.best_face, best_edge = sat.best_edge;
  const V3<T> face_u = sat.face_u, edge_u = sat.edge_u;
  const T face_s = sat.face_s, edge_s = sat.edge_s;
  if (edge_id >= 0 && best_edge < T(0.95) * best_face) {
    T sg = edge_s >= T(0) ? T(1) : T(-1);
    V3<T> n{edge_u.x * sg, edge_u.y * sg, edge_u.z * sg};
    const int i = (edge_id - 6) / 3, j = (edge_id - 6) % 3;
    V3<T> e1 = P1, e2 = P2;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      T s1 = k == i ? T(0) : (vdot(n, A[k]) >= T(0) ? h1[k] : -h1[k]);
      T s2 = k == j ? T(0) : (vdot(n, B[k]) >= T(0) ? -h2[k] : h2[k]);
      e1 = V3<T>{e1.x + s1 * A[k].x, e1.y + s1 * A[k].y, e1.z + s1 * A[k].z};
      e2 = V3<T>{e2.x + s2 * B[k].x, e2.y + s2 * B[k].y, e2.z + s2 * B[k].z};
    }
    const V3<T> ai = vpick(i, A[0], A[1], A[2]), bj = vpick(j, B[0], B[1], B[2]);
    const V3<T> wv{e1.x - e2.x, e1.y - e2.y, e1.z - e2.z};
    T bbv = vdot(ai, bj), dd = vdot(ai, wv), ee = vdot(bj, wv);
    T den = T(1) - bbv * bbv;
    T s = 0, t = 0;
    if (den > T(1e-12)) {
      s = (bbv * ee - dd) / den;
      t = (ee - bbv * dd) / den;
    }
    T hi_ = spick(i, h1[0], h1[1], h1[2]);
    T hj_ = spick(j, h2[0], h2[1], h2[2]);
    s = s < -hi_ ? -hi_ : (s > hi_ ? hi_ : s);
    t = t < -hj_ ? -hj_ : (t > hj_ ? hj_ : t);
    emit(-best_edge, T(0.5) * (e1.x + s * ai.x + e2.x + t * bj.x), T(0.5) * (e1.y + s * ai.y + e2.y + t * bj.y),
         T(0.5) * (e1.z + s * ai.z + e2.z + t * bj.z), n.x, n.y, n.z);
    return;
  }
  // ---- face contact: the candidates in the serial order (incident vertices, reference corners, crossings)
  const BBFace<T> F = bb_face_setup(p1, R1, h1, p2, R2, h2, sat);
#pragma unroll
  for (int c = 0; c < 24; c++) {
    T u, v, w;
    if (bb_face_candidate(F, c, u, v, w) && !(w > T(0))) bb_face_emit(F, u, v, w, emit);
  }
}

// ------------------------------------------------------------------------------------------------
// collision (mj_collision): two-level broadphase + narrowphase
//   1. world centres of the moving geoms (gx[g] = centre, rbound)
//   2. bounds of the collision bodies (moving bodies: sphere about the body origin; static groups and
//      the belt: AABBs; the floor: half-space) and a test of every body pair MuJoCo's filters allow
//   3. expansion of the surviving body pairs into geom pairs + MuJoCo's bounding-sphere test
//   4. narrowphase per geom pair (one pair per lane), contacts staged with LDS atomics
//   5. staged contacts sorted by (geom pair, index) into the contact slots
// ------------------------------------------------------------------------------------------------
template <typename T, typename DIM>
__device__ __forceinline__ void geom_frame(const Model<T>& M, const Ws<T, DIM>& w, int g, int kb, T* R, T* h) {
  const DIM dm(M.dm);
  const T* gg = M.geom + 16 * g;
  if (kb >= 2 && kb < 2 + dm.K) {
    const T* c = w.cR() + 9 * (kb - 2);
#pragma unroll
    for (int k = 0; k < 9; k++) R[k] = c[k];
    T hh = w.cube()[4 * (kb - 2)];
    h[0] = h[1] = h[2] = hh;
    return;
  }
  h[0] = gg[12];
  h[1] = gg[13];
  h[2] = gg[14];
  if (kb == 0) {
#pragma unroll
    for (int k = 0; k < 9; k++) R[k] = gg[3 + k];
  } else if (kb == 1) {
#pragma unroll
    for (int k = 0; k < 9; k++) R[k] = (k % 4 == 0) ? T(1) : T(0);
  } else {
    int arm = (kb - 2 - dm.K) / 10, b = (kb - 2 - dm.K) % 10;
    matmul3(w.bR() + 90 * arm + 9 * b, gg + 3, R);
  }
}

// fp32 build: the narrowphase in float64 from the float64 master state (cube centres and quaternions, belt slide),
// the float64 geom table and the cubes' exact half sizes; the arm geoms' poses come from the float kinematics.
// A contact's depth is a difference of coordinates ~0.1 m apart: in float it keeps ~1e-8 m of a 2.3e-6 m resting
// depth (0.4 %), which the contact's stiffness turns into reference-acceleration errors of ~1e-4 per env-step
#ifndef FM_NP_F64
#define FM_NP_F64 1
#endif
template <typename T, typename DIM>
__device__ __forceinline__ void geom_pose_f64(const Model<T>& M, const Ws<T, DIM>& w, int g, int kb, double* p, double* R,
                                              double* h) {
  const DIM dm(M.dm);
  const double* gg = M.geomd + 16 * g;
  constexpr double zs = zshift<T>();
  h[0] = gg[12];
  h[1] = gg[13];
  h[2] = gg[14];
  if (kb == 0) {
#pragma unroll
    for (int k = 0; k < 3; k++) p[k] = gg[k];
#pragma unroll
    for (int k = 0; k < 9; k++) R[k] = gg[3 + k];
  } else if (kb == 1) {
    p[0] = 0.0;
    p[1] = w.qd()[0];
    p[2] = 1.05 - zs;
#pragma unroll
    for (int k = 0; k < 9; k++) R[k] = (k % 4 == 0) ? 1.0 : 0.0;
  } else if (kb < 2 + dm.K) {
    const int k = kb - 2;
    const double* c = w.qd() + 1 + 7 * k;
    p[0] = c[0];
    p[1] = c[1];
    p[2] = c[2] - zs;
    double qu[4] = {c[3], c[4], c[5], c[6]};
    const double n = sqrt(qu[0] * qu[0] + qu[1] * qu[1] + qu[2] * qu[2] + qu[3] * qu[3]);
    if (n < 1e-15) {
      qu[0] = 1.0;
      qu[1] = qu[2] = qu[3] = 0.0;
    } else if (fabs(n - 1.0) > 1e-15) {
      for (int e = 0; e < 4; e++) qu[e] /= n;
    }
    const double ww = qu[0], x = qu[1], y = qu[2], z = qu[3];
    R[0] = ww * ww + x * x - y * y - z * z;
    R[1] = 2.0 * (x * y - ww * z);
    R[2] = 2.0 * (x * z + ww * y);
    R[3] = 2.0 * (x * y + ww * z);
    R[4] = ww * ww - x * x + y * y - z * z;
    R[5] = 2.0 * (y * z - ww * x);
    R[6] = 2.0 * (x * z - ww * y);
    R[7] = 2.0 * (y * z + ww * x);
    R[8] = ww * ww - x * x - y * y + z * z;
    const T* cb = w.cube() + 4 * k;
    h[0] = h[1] = h[2] = (double)cb[0] + (double)cb[3];
  } else if constexpr (DIM::f64arms) {
    // the arm body's float64 pose (arm_pose_f64) and the geom's float64 local frame
    const int arm = (kb - 2 - dm.K) / 10, b = (kb - 2 - dm.K) % 10;
    const double* bp = w.bposd() + 30 * arm + 3 * b;
    const double* bR = w.bRd() + 90 * arm + 9 * b;
#pragma unroll
    for (int r = 0; r < 3; r++) {
      p[r] = bp[r] + bR[3 * r] * gg[0] + bR[3 * r + 1] * gg[1] + bR[3 * r + 2] * gg[2];
#pragma unroll
      for (int c = 0; c < 3; c++)
        R[3 * r + c] = bR[3 * r] * gg[3 + c] + bR[3 * r + 1] * gg[6 + c] + bR[3 * r + 2] * gg[9 + c];
    }
  } else {
    const T* x = w.gx() + 4 * g;
    p[0] = x[0];
    p[1] = x[1];
    p[2] = x[2];
    const int arm = (kb - 2 - dm.K) / 10, b = (kb - 2 - dm.K) % 10;
    T Rf[9];
    matmul3(w.bR() + 90 * arm + 9 * b, M.geom + 16 * g + 3, Rf);
#pragma unroll
    for (int k = 0; k < 9; k++) R[k] = Rf[k];
  }
}

// float64 poses of arm `arm`'s ten bodies (the fp32 build's DIM::f64arms scenes, for the narrowphase): the serial
// chain of arm_chain (iiwa14.xml:55-147, gripper.xml:4-44) from the float64 master state, the float64 base frame and
// the arm template's float64 constants, in the kernel frame (z - zshift)
template <typename T, typename DIM>
__device__ __forceinline__ void arm_pose_f64(const Model<T>& M, const Ws<T, DIM>& w, int arm) {
  const DIM dm(M.dm);
  const double* qa = w.qd() + 1 + 7 * dm.K + 9 * arm;
  const double* base = M.arm_base_w + 12 * arm;
  double* bpos = w.bposd() + 30 * arm;
  double* bR = w.bRd() + 90 * arm;
  double Pp[3] = {base[0], base[1], base[2] - zshift<T>()}, PR[9];
#pragma unroll
  for (int k = 0; k < 9; k++) PR[k] = base[3 + k];
  double Gp[3], GR[9];
#pragma unroll
  for (int b = 0; b < 10; b++) {
    const double* bl = ARM_BODY[b];
    if (b >= 8) {  // both plates hang off the gripper base
#pragma unroll
      for (int k = 0; k < 3; k++) Pp[k] = Gp[k];
#pragma unroll
      for (int k = 0; k < 9; k++) PR[k] = GR[k];
    }
    double o[3], Rpre[9], R[9];
#pragma unroll
    for (int r = 0; r < 3; r++) {
      o[r] = Pp[r] + PR[3 * r] * bl[0] + PR[3 * r + 1] * bl[1] + PR[3 * r + 2] * bl[2];
#pragma unroll
      for (int c = 0; c < 3; c++)
        Rpre[3 * r + c] = PR[3 * r] * bl[3 + c] + PR[3 * r + 1] * bl[6 + c] + PR[3 * r + 2] * bl[9 + c];
    }
    if (b < 7) {
      double sn, cs;
      sincos(qa[b], &sn, &cs);
#pragma unroll
      for (int r = 0; r < 3; r++) {
        R[3 * r + 0] = Rpre[3 * r + 0] * cs + Rpre[3 * r + 1] * sn;
        R[3 * r + 1] = -Rpre[3 * r + 0] * sn + Rpre[3 * r + 1] * cs;
        R[3 * r + 2] = Rpre[3 * r + 2];
      }
    } else {
#pragma unroll
      for (int k = 0; k < 9; k++) R[k] = Rpre[k];
      if (b >= 8) {
#pragma unroll
        for (int k = 0; k < 3; k++) o[k] += Rpre[3 * k] * qa[b - 1];  // slide along the plate's local x
      }
    }
#pragma unroll
    for (int k = 0; k < 3; k++) bpos[3 * b + k] = o[k];
#pragma unroll
    for (int k = 0; k < 9; k++) bR[9 * b + k] = R[k];
#pragma unroll
    for (int k = 0; k < 3; k++) Pp[k] = o[k];
#pragma unroll
    for (int k = 0; k < 9; k++) PR[k] = R[k];
    if (b == 7) {
#pragma unroll
      for (int k = 0; k < 3; k++) Gp[k] = o[k];
#pragma unroll
      for (int k = 0; k < 9; k++) GR[k] = R[k];
    }
  }
}

// A contact's position is stored relative to its pair's anchor: the centre of the pair's cube (geom 2's body if it
// is a cube, else geom 1's), otherwise the kernel-frame origin.  The point and the cube's lever arm p - c then keep
// float precision wherever the cube sits: at the parking spots x = 4..5 m (task_utils.py:31-36, 115-129) float
// coordinates are 4.8e-7 m apart against 2.3e-6 m resting depths, which turned into spin noise of parked cubes
template <typename DD>
__device__ __forceinline__ int anchor_cube(const DD& dm, int kb1, int kb2) {
  if (kb2 >= 2 && kb2 < 2 + dm.K) return kb2 - 2;
  if (kb1 >= 2 && kb1 < 2 + dm.K) return kb1 - 2;
  return -1;
}
template <typename T, typename DIM>
__device__ __forceinline__ void contact_anchor(const Ws<T, DIM>& w, int ak, double* o) {
  if (ak < 0) {
    o[0] = o[1] = o[2] = 0.0;
    return;
  }
  const double* c = w.qd() + 1 + 7 * ak;
  o[0] = c[0];
  o[1] = c[1];
  o[2] = c[2] - zshift<T>();
}
template <typename T, typename DIM, typename E>
__device__ __forceinline__ void set_anchor(const Ws<T, DIM>& w, const DIM& dm, int kb1, int kb2, E& emit) {
  contact_anchor(w, anchor_cube(dm, kb1, kb2), emit.o);
}

template <typename T, typename DIM>
__device__ __forceinline__ void narrow_batch(const Model<T>& M, const Ws<T, DIM>& w, const uint32_t* list, int n) {
  const DIM dm(M.dm);
  if (LANE >= n) return;
  if constexpr (sizeof(T) == 4 && FM_NP_F64) {
    const uint32_t pwd = list[LANE];
    const int c1 = pwd & 4095, c2 = (pwd >> 12) & 4095;
    const int gi1 = w.ginfo()[c1], gi2 = w.ginfo()[c2];
    const int t1 = gi1 & 3, t2 = gi2 & 3;
    const int kb1 = (gi1 >> 8) & 255, kb2 = (gi2 >> 8) & 255;
    const int lo = c1 < c2 ? c1 : c2, hi = c1 < c2 ? c2 : c1;
    Emit<T> emit{w.stage(), w.skey(), w.spw(), w.misc() + MISC_NSTAGE, dm.maxcon, (lo << 15) | (hi << 3), pwd, 0};
    double p1[3], R1[9], h1[3], p2[3], R2[9], h2[3];
    geom_pose_f64(M, w, c2, kb2, p2, R2, h2);
    const int ak = anchor_cube(dm, kb1, kb2);
    // the anchor (contact_anchor) is the cube's centre, i.e. its geom's pose
    if (ak < 0 || ak != kb2 - 2) contact_anchor(w, ak, emit.o);
    else
      for (int k = 0; k < 3; k++) emit.o[k] = p2[k];
    if (t1 == GC_PLANE) {
      if (t2 == GC_SPHERE)
        np_plane_sphere(p2, M.geomd[16 * c2 + 15], emit, zshift<T>());
      else
        np_plane_box(p2, R2, h2, emit, zshift<T>());
      return;
    }
    geom_pose_f64(M, w, c1, kb1, p1, R1, h1);
    if (t1 == GC_SPHERE) {
      if (t2 == GC_SPHERE)
        np_sphere_sphere(p1, M.geomd[16 * c1 + 15], p2, M.geomd[16 * c2 + 15], emit);
      else
        np_sphere_box(p1, M.geomd[16 * c1 + 15], p2, R2, h2, emit);
    } else {
      np_box_box(p1, R1, h1, p2, R2, h2, emit);
    }
    return;
  }
  uint32_t pwd = list[LANE];
  int c1 = pwd & 4095, c2 = (pwd >> 12) & 4095;
  const int gi1 = w.ginfo()[c1], gi2 = w.ginfo()[c2];
  const int t1 = gi1 & 3, t2 = gi2 & 3;
  const int kb1 = (gi1 >> 8) & 255, kb2 = (gi2 >> 8) & 255;
  const T* x1 = w.gx() + 4 * c1;
  const T* x2 = w.gx() + 4 * c2;
  int lo = c1 < c2 ? c1 : c2, hi = c1 < c2 ? c2 : c1;
  Emit<T> emit{w.stage(), w.skey(), w.spw(), w.misc() + MISC_NSTAGE, dm.maxcon, (lo << 15) | (hi << 3), pwd, 0};
  set_anchor(w, dm, kb1, kb2, emit);
  T p1[3] = {x1[0], x1[1], x1[2]}, p2[3] = {x2[0], x2[1], x2[2]};
  if (t1 == GC_PLANE) {
    if (t2 == GC_SPHERE) {
      np_plane_sphere(p2, x2[3], emit, T(zshift<T>()));
    } else {
      T R[9], h[3];
      geom_frame(M, w, c2, kb2, R, h);
      np_plane_box(p2, R, h, emit, T(zshift<T>()));
    }
  } else if (t1 == GC_SPHERE) {
    if (t2 == GC_SPHERE) {
      np_sphere_sphere(p1, x1[3], p2, x2[3], emit);
    } else {
      T R[9], h[3];
      geom_frame(M, w, c2, kb2, R, h);
      np_sphere_box(p1, x1[3], p2, R, h, emit);
    }
  } else {
    T Ra[9], ha[3], Rb[9], hb[3];
    geom_frame(M, w, c1, kb1, Ra, ha);
    geom_frame(M, w, c2, kb2, Rb, hb);
    np_box_box(p1, Ra, ha, p2, Rb, hb, emit);
  }
}

// box-box pairs with the SAT spread over the wave: 4 pairs per pass, lanes 16 p .. 16 p + 14 evaluate axis
// LANE & 15 of pair p (bb_axis: the serial loop's arithmetic), the group's separation test by ballot, the best
// face / edge axis by a DPP row minimum (first axis on ties, as the serial strict '<' keeps), the winner's axis and
// distance fetched by ds_bpermute; then a face contact's 24 clipping candidates are spread over the pair's 16 lanes
// (bb_face_candidate, numbered by a ballot prefix) and an edge contact is built on lane 16 p.  A pass costs one
// axis and two candidates per lane instead of 15 axes and 24 candidates on one lane.
template <int CTRL>
__device__ __forceinline__ double dpp_row(double x) {
  return dpp_f64<CTRL>(x, x);
}
template <int CTRL>
__device__ __forceinline__ float dpp_row(float x) {
  return dpp_f32<CTRL>(x, x);
}
template <typename NP, typename T, typename DIM>
__device__ __forceinline__ void geom_pose_np(const Model<T>& M, const Ws<T, DIM>& w, int g, int kb, NP* p, NP* R,
                                             NP* h) {
  if constexpr (sizeof(T) == 4 && FM_NP_F64) {
    geom_pose_f64(M, w, g, kb, p, R, h);
  } else {
    const T* x = w.gx() + 4 * g;
    p[0] = x[0];
    p[1] = x[1];
    p[2] = x[2];
    geom_frame(M, w, g, kb, R, h);
  }
}
template <typename T, typename DIM>
__device__ __forceinline__ void narrow_bb_parallel(const Model<T>& M, const Ws<T, DIM>& w, const uint32_t* list,
                                                   int n) {
  using NP = std::conditional_t<(sizeof(T) == 4 && FM_NP_F64 != 0), double, T>;
  const DIM dm(M.dm);
  const int grp = LANE >> 4, ax = LANE & 15;
  const uint64_t gm = 0xFFFFull << (16 * grp);
  for (int p0 = 0; p0 < n; p0 += 4) {
    const int pi = p0 + grp;
    const bool live = pi < n;
    const uint32_t pwd = list[live ? pi : 0];
    const int c1 = pwd & 4095, c2 = (pwd >> 12) & 4095;
    const int kb1 = (w.ginfo()[c1] >> 8) & 255, kb2 = (w.ginfo()[c2] >> 8) & 255;
    NP p1[3], R1[9], h1[3], p2[3], R2[9], h2[3];
    geom_pose_np<NP>(M, w, c1, kb1, p1, R1, h1);
    geom_pose_np<NP>(M, w, c2, kb2, p2, R2, h2);
    const V3<NP> A[3] = {vcol(R1, 0), vcol(R1, 1), vcol(R1, 2)};
    const V3<NP> B[3] = {vcol(R2, 0), vcol(R2, 1), vcol(R2, 2)};
    const V3<NP> d{p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    V3<NP> u{0, 0, 0};
    NP ov = 0, sd = 0;
    bool valid = false;
    if (live && ax < 15) valid = bb_axis(ax, A, B, h1, h2, d, u, ov, sd);
    const bool sep = (__ballot(valid && ov < NP(0)) & gm) != 0ull;
    const bool isf = valid && ax < 6, ise = valid && ax >= 6;
    NP fo = isf ? ov : NP(1e30), eo = ise ? ov : NP(1e30);
    fo = fmin(fo, dpp_row<0x121>(fo));  // row_ror:1, 2, 4, 8: every lane of the row holds the row minimum
    fo = fmin(fo, dpp_row<0x122>(fo));
    fo = fmin(fo, dpp_row<0x124>(fo));
    fo = fmin(fo, dpp_row<0x128>(fo));
    eo = fmin(eo, dpp_row<0x121>(eo));
    eo = fmin(eo, dpp_row<0x122>(eo));
    eo = fmin(eo, dpp_row<0x124>(eo));
    eo = fmin(eo, dpp_row<0x128>(eo));
    const uint64_t fb = __ballot(isf && ov == fo) & gm;
    const uint64_t eb = __ballot(ise && ov == eo) & gm;
    const int fl = fb ? __builtin_ctzll(fb) : 16 * grp;
    const int el = eb ? __builtin_ctzll(eb) : 16 * grp;
    BBSat<NP> sat;
    sat.face_id = fl & 15;
    sat.face_u = V3<NP>{__shfl(u.x, fl), __shfl(u.y, fl), __shfl(u.z, fl)};
    sat.face_s = __shfl(sd, fl);
    sat.best_face = fo;
    sat.edge_id = eb ? (el & 15) : -1;
    sat.edge_u = V3<NP>{__shfl(u.x, el), __shfl(u.y, el), __shfl(u.z, el)};
    sat.edge_s = __shfl(sd, el);
    sat.best_edge = eo;
    const int lo = c1 < c2 ? c1 : c2, hi = c1 < c2 ? c2 : c1;
    Emit<T> emit{w.stage(), w.skey(), w.spw(), w.misc() + MISC_NSTAGE, dm.maxcon, (lo << 15) | (hi << 3), pwd, 0};
    set_anchor(w, dm, kb1, kb2, emit);
    const bool edge =sat.edge_id >= 0 && sat.best_edge < NP(0.95) * sat.best_face;
    if (live && !sep && edge && ax == 0) np_box_box_finish(p1, R1, h1, p2, R2, h2, sat, emit);  // one point
    // face contact: candidates c = ax and 16 + ax (ax < 8) of the serial order on the pair's 16 lanes; the k-th
    // contact in that order (rank by ballot prefix) takes index k within the pair, as the serial loop numbers them
    bool f0 = false, f1 = false;
    NP u0 = 0, v0 = 0, w0 = 0, u1 = 0, v1 = 0, w1 = 0;
    BBFace<NP> F;
    if (live && !sep && !edge) {
      F = bb_face_setup(p1, R1, h1, p2, R2, h2, sat);
      f0 = bb_face_candidate(F, ax, u0, v0, w0) && !(w0 > NP(0));
      f1 = ax < 8 && bb_face_candidate(F, 16 + ax, u1, v1, w1) && !(w1 > NP(0));
    }
    const uint32_t g0 = (uint32_t)(__ballot(f0) >> (16 * grp)) & 0xFFFFu;
    const uint32_t g1 = (uint32_t)(__ballot(f1) >> (16 * grp)) & 0xFFu;
    const uint32_t mk = g0 | (g1 << 16);
    if (f0) {
      emit.sub = __popc(mk & ((1u << ax) - 1u));
      bb_face_emit(F, u0, v0, w0, emit);
    }
    if (f1) {
      emit.sub = __popc(mk & ((1u << (16 + ax)) - 1u));
      bb_face_emit(F, u1, v1, w1, emit);
    }
  }
}

// midphase passes of 64 body pairs that cover every possible pair of a compile-time scene
template <typename DIM>
__device__ constexpr int body_pair_passes() {
  if constexpr (DIM::fixed)
    return (DIM::ncb * (DIM::ncb - 1) / 2 + WAVE - 1) / WAVE;
  else
    return 1;
}

template <typename T, typename DIM>
__device__ __forceinline__ void collide(const Model<T>& M, const Ws<T, DIM>& w, int arena, int64_t* ctr) {
  const DIM dm(M.dm);
  const int K = dm.K;
  const T* q = w.q();
  T* gx = w.gx();
  const int* gin = w.ginfo();
  const int* cbi = w.cbi();
  int* misc = w.misc();
  const uint64_t below = (1ull << LANE) - 1ull;
  // compile-time scene: the allowed body pairs (a scene constant in global memory) are all requested up front,
  // so their latency hides behind the geom / bound passes
  constexpr int NPP = body_pair_passes<DIM>();
  uint32_t bpr[NPP];
  if constexpr (DIM::fixed) {
#pragma unroll
    for (int k = 0; k < NPP; k++) bpr[k] = k * WAVE + LANE < dm.ncbp ? M.cbp[k * WAVE + LANE] : 0u;
  }
  // 1. geom centres + rbound (the buffer is phase-local, so static geoms are rewritten too); unrolled so the
  // scene-table loads of every pass issue together
#pragma unroll
  for (int g = LANE; g < dm.ngc; g += WAVE) {
    const int kb = (gin[g] >> 8) & 255;
    const T* gg = M.geom + 16 * g;
    T* o = gx + 4 * g;
    o[3] = gg[15];
    if (kb == 0) {
      o[0] = gg[0];
      o[1] = gg[1];
      o[2] = gg[2];
    } else if (kb == 1) {
      o[0] = 0;
      o[1] = q[0];
      o[2] = T(1.05 - zshift<T>());
    } else if (kb < 2 + K) {
      const T* c = q + 1 + 7 * (kb - 2);
      o[0] = c[0];
      o[1] = c[1];
      o[2] = c[2];
    } else {
      int arm = (kb - 2 - K) / 10, b = (kb - 2 - K) % 10;
      const T* bp = w.bpos() + 30 * arm + 3 * b;
      const T* bR = w.bR() + 90 * arm + 9 * b;
      T off[3];
      matvec3(bR, gg, off);
      o[0] = bp[0] + off[0];
      o[1] = bp[1] + off[1];
      o[2] = bp[2] + off[2];
    }
  }
  // 2. collision-body bounds
#pragma unroll
  for (int b = LANE; b < dm.ncb; b += WAVE) {
    const int kb = cbi[4 * b], fl = cbi[4 * b + 1];
    T* o = w.cbw() + 8 * b;
    const T* cs = M.cbs + 8 * b;
#pragma unroll
    for (int k = 0; k < 7; k++) o[k] = cs[k];
    if (fl & CB_STATIC) {
    } else if (kb == 1) {
      o[0] = T(0);
      o[1] = q[0];
      o[2] = T(1.05 - zshift<T>());
    } else if (kb < 2 + K) {
      const T* c = q + 1 + 7 * (kb - 2);
      o[0] = c[0];
      o[1] = c[1];
      o[2] = c[2];
    } else {
      const T* bp = w.bpos() + 30 * ((kb - 2 - K) / 10) + 3 * ((kb - 2 - K) % 10);
      o[0] = bp[0];
      o[1] = bp[1];
      o[2] = bp[2];
    }
  }
  if (LANE == 0) misc[MISC_NSTAGE] = 0;
  SYNC();
  PMARK(PH_CBOUND);
  // 3. midphase: every allowed body pair's bounding test; the hits are compacted into sp[] (body pair | first
  // geom-pair index << 16) in one sweep, so the geom-pair expansion below runs over all of them at once.
  // DIM::midcache: the list of an inflated test (every bound + MC_MARGIN) is kept and reused while no moving
  // body has moved MC_HALF since it was built -- a pair outside the inflated test then cannot pass the exact one,
  // and the geom-pair test and narrowphase below decide the contacts as before (so the contact set is unchanged)
  // the list is built in w.sp() (the arena's global block with DIM::gl_sp, else LDS) and read back from there or,
  // when the cached list is reused, from w.mcache() (LDS; w.sp() itself when that is global): reads go through
  // address-space-typed pointers chosen per access, never through one pointer selected between the two (that would
  // be generic: FLAT instructions)
  uint32_t* const sp = w.sp();
  constexpr int SPAS = DIM::template gl_sp<sizeof(T)>() ? AS_GLOBAL : AS_LDS;
  int nsp = 0, total = 0;
  bool reuse = false;
  T infl = T(0);
  if constexpr (DIM::midcache) {
    bool moved = false;
    const int ok = misc[MISC_MC_OK] && !(FM_XF(M) & 8);  // FM_NO_MIDCACHE=1: rebuild every substep
    for (int b = LANE; b < dm.ncb; b += WAVE) {
      const T* o = w.cbw() + 8 * b;
      const T* p0 = w.mpos() + 3 * b;
      const T dx = fabs(o[0] - p0[0]), dy = fabs(o[1] - p0[1]), dz = fabs(o[2] - p0[2]);
      const T dmax = dx > dy ? (dx > dz ? dx : dz) : (dy > dz ? dy : dz);
      moved = moved || !(dmax <= T(MC_HALF));
    }
    reuse = ok && __ballot(moved) == 0ull;
    if (reuse) {
      nsp = misc[MISC_MC_N];
      total = misc[MISC_MC_TOT];
    } else {
      infl = T(MC_MARGIN);
    }
  }
  auto sweep = [&](uint32_t bpw, int pidx) {
    // branch-free: both records and both flag words are read unconditionally (a lane past the list reads body
    // 0's), so each pass is one batch of LDS reads
    const int b1 = bpw & 255, b2 = (bpw >> 8) & 255;
    const T* X = w.cbw() + 8 * b1;
    const T* Y = w.cbw() + 8 * b2;
    const int f1 = cbi[4 * b1 + 1], f2 = cbi[4 * b2 + 1], n1 = cbi[4 * b1 + 3], n2 = cbi[4 * b2 + 3];
    T d0 = fabs(X[0] - Y[0]) - X[4] - Y[4];
    T d1 = fabs(X[1] - Y[1]) - X[5] - Y[5];
    T d2 = fabs(X[2] - Y[2]) - X[6] - Y[6];
    d0 = d0 > T(0) ? d0 : T(0);
    d1 = d1 > T(0) ? d1 : T(0);
    d2 = d2 > T(0) ? d2 : T(0);
    const T rr = X[3] + Y[3] + infl;
    const bool hs = d0 * d0 + d1 * d1 + d2 * d2 <= rr * rr;
    const T zf = T(-zshift<T>()) + infl;  // the floor's height in the kernel frame (+ the cache margin)
    const bool hp1 = Y[2] - Y[6] - Y[3] <= zf, hp2 = X[2] - X[6] - X[3] <= zf;
    const bool hit = pidx < dm.ncbp && ((f1 & CB_PLANE) ? hp1 : ((f2 & CB_PLANE) ? hp2 : hs));
    const int ncomb = hit ? n1 * n2 : 0;
    const uint64_t bal = __ballot(hit);
    const int incl = wave_incl_scan(ncomb);
    if (hit)
      ((uint32_t FM_AS(SPAS)*)sp)[nsp + __popcll(bal & below)] =
          (bpw & 0xFFFFu) | ((uint32_t)(total + incl - ncomb) << 16);
    nsp += __popcll(bal);
    total += __builtin_amdgcn_readlane(incl, WAVE - 1);
  };
  if constexpr (DIM::fixed) {
    if (!reuse) {
#pragma unroll
      for (int k = 0; k < NPP; k++)
        if (k * WAVE < dm.ncbp) sweep(bpr[k], k * WAVE + LANE);
      if constexpr (DIM::midcache) {
        // keep the inflated list (when it fits) and the positions it was built at.  A list built in the global
        // block stays there (nothing else writes w.sp() until the next rebuild): it is its own cache
        const bool fits = SPAS == AS_GLOBAL || nsp <= mc_cap(DIM::nv);
        if constexpr (SPAS != AS_GLOBAL)
          for (int e = LANE; e < nsp && fits; e += WAVE) w.mcache()[e] = ((const uint32_t FM_AS(SPAS)*)sp)[e];
        for (int b = LANE; b < dm.ncb; b += WAVE) {
          const T* o = w.cbw() + 8 * b;
          T* p0 = w.mpos() + 3 * b;
          p0[0] = o[0];
          p0[1] = o[1];
          p0[2] = o[2];
        }
        if (LANE == 0) {
          misc[MISC_MC_OK] = fits ? 1 : 0;
          misc[MISC_MC_N] = nsp;
          misc[MISC_MC_TOT] = total;
        }
      }
    }
  } else {
    // allowed body pairs are fetched one pass ahead (the global load overlaps the current pass)
    uint32_t bpw_next = LANE < dm.ncbp ? M.cbp[LANE] : 0u;
    for (int p0 = 0; p0 < dm.ncbp; p0 += WAVE) {
      const uint32_t bpw = bpw_next;
      bpw_next = p0 + WAVE + LANE < dm.ncbp ? M.cbp[p0 + WAVE + LANE] : 0u;
      sweep(bpw, p0 + LANE);
    }
  }
  // pair-class -> params table, one entry per lane (read back with ds_bpermute, no memory access)
  const int ptab_l = LANE < 25 ? M.ptab[LANE] : 0;
  SYNC();
  PMARK(PH_CMID);
  // 4. geom pairs of the hit body pairs, 64 per pass: bounding-sphere test, then binned by narrowphase cost:
  // box-box pairs (SAT + face clipping) in gsb, everything else (sphere-box, sphere-sphere, plane-*) in gs,
  // so a batch of 64 lanes runs one code path instead of the union of all of them
  uint32_t* gs = w.gsurv();
  uint32_t* gsb = gs + 2 * WAVE;
  int nsurv = 0, nbb = 0;
  // the hit entry owning geom pair e (the last entry whose first index is <= e): entries starting in the pass mark
  // their lane, an inclusive prefix maximum over the wave fills the lanes in between (starts are strictly
  // increasing: every hit pair expands to >= 1 geom pair), and the pass's last owner carries into the next
  int* mark = misc + 16;  // [64] scratch of the collision phase
  int carry = 0;
  auto sp_at = [&](int i) -> uint32_t {
    if (DIM::midcache && SPAS != AS_GLOBAL && reuse) return ((const uint32_t FM_AS(AS_LDS)*)w.mcache())[i];
    return ((const uint32_t FM_AS(SPAS)*)sp)[i];
  };
  for (int e0 = 0; e0 < total; e0 += WAVE) {
    const int e = e0 + LANE;
    bool ok = false;
    uint32_t pk = 0;
    int pc = 0;
    mark[LANE] = -1;
    SYNC();
    for (int q = LANE; q < nsp; q += WAVE) {
      const int st = (int)(sp_at(q) >> 16);
      if (st >= e0 && st < e0 + WAVE) mark[st - e0] = q;
    }
    SYNC();
    int own = wave_incl_max(mark[LANE]);
    own = own > carry ? own : carry;
    carry = __builtin_amdgcn_readlane(own, WAVE - 1);
    if (e < total) {
      const uint32_t bp = sp_at(own);
      const int x = bp & 255, y = (bp >> 8) & 255;
      const int r = e - (int)(bp >> 16);
      const int ngy = cbi[4 * y + 3];
      const int i = r / ngy, j = r - i * ngy;
      int ga = w.cbg()[cbi[4 * x + 2] + i], gb = w.cbg()[cbi[4 * y + 2] + j];
      const T* xa = gx + 4 * ga;
      const T* xb = gx + 4 * gb;
      ok = true;
      if (xa[3] > T(0) && xb[3] > T(0)) {
        T d0 = xa[0] - xb[0], d1 = xa[1] - xb[1], d2 = xa[2] - xb[2];
        T rs = xa[3] + xb[3];
        ok = sqrt(d0 * d0 + d1 * d1 + d2 * d2) <= rs;
      }
      if (ok) {
        int c1 = ga < gb ? ga : gb, c2 = ga < gb ? gb : ga;
        if ((gin[c1] & 3) > (gin[c2] & 3)) {
          int t = c1;
          c1 = c2;
          c2 = t;
        }
        pc = 5 * ((gin[c1] >> GI_PC) & 7) + ((gin[c2] >> GI_PC) & 7);
        pk = (uint32_t)c1 | ((uint32_t)c2 << 12);
      }
    }
    pk |= (uint32_t)__builtin_amdgcn_ds_bpermute(pc << 2, ptab_l) << 24;
    const bool isbb = ok && (gin[pk & 4095] & 3) == GC_BOX;  // type-ordered: c1 box => both boxes
    const uint64_t b2m = __ballot(ok && !isbb);
    const uint64_t bbm = __ballot(isbb);
    if (ok && !isbb) gs[nsurv + __popcll(b2m & below)] = pk;
    if (isbb) gsb[nbb + __popcll(bbm & below)] = pk;
    nsurv += __popcll(b2m);
    nbb += __popcll(bbm);
    SYNC();
    NPMARK(PH_CHDIAG);  // geom-pair expansion
    if (nsurv >= WAVE) {
      narrow_batch(M, w, gs, WAVE);
      NPMARK(PH_CHPANEL);
      const bool mv = LANE + WAVE < nsurv;
      uint32_t t = mv ? gs[LANE + WAVE] : 0u;
      SYNC();
      if (mv) gs[LANE] = t;
      nsurv -= WAVE;
      SYNC();
    }
    if (nbb >= WAVE) {
      narrow_batch(M, w, gsb, WAVE);
      NPMARK(PH_CHTRAIL);
      const bool mv = LANE + WAVE < nbb;
      uint32_t t = mv ? gsb[LANE + WAVE] : 0u;
      SYNC();
      if (mv) gsb[LANE] = t;
      nbb -= WAVE;
      SYNC();
    }
  }
  NPMARK(PH_CHDIAG);
  if (nsurv > 0) narrow_batch(M, w, gs, nsurv);
  NPMARK(PH_CHPANEL);
  if (nbb > 0) {
    if (nbb <= 8 && !(FM_XF(M) & 4))  // FM_SERIAL_BOXBOX=1: one lane per pair throughout
      narrow_bb_parallel(M, w, gsb, nbb);
    else
      narrow_batch(M, w, gsb, nbb);
  }
  NPMARK(PH_CHTRAIL);
  SYNC();
  PMARK(PH_CNARROW);
  // 5. sort the staged contacts by key into the contact slots
  const int nst = misc[MISC_NSTAGE];
  const int ncon = nst < dm.maxcon ? nst : dm.maxcon;
  // above capacity: the excess is counted as dropped, unless the env-step will be abandoned and rerun at the wide
  // capacity (the benchmark scene, M.ovf_abort; the kernel reads MISC_OVF after the stage)
  if (LANE == 0) {
    misc[MISC_OVF] = nst > dm.maxcon ? nst - dm.maxcon : 0;
    if (nst > dm.maxcon && !M.ovf_abort) ctr[0] += nst - dm.maxcon;
  }
  // rank of each staged contact among the staged keys: contacts c = LANE + 64 h (h < DIM::MAXC / 64), the keys
  // broadcast by v_readlane
  constexpr int NHC = DIM::MAXC / WAVE;
  int mykey[NHC], myrank[NHC];
#pragma unroll
  for (int h = 0; h < NHC; h++) {
    mykey[h] = LANE + WAVE * h < ncon ? w.skey()[LANE + WAVE * h] : 0x7fffffff;
    myrank[h] = 0;
  }
#pragma unroll
  for (int hs = 0; hs < NHC; hs++) {
    const int tn = ncon - WAVE * hs < WAVE ? ncon - WAVE * hs : WAVE;
    for (int t = 0; t < tn; t++) {
      const int k = __builtin_amdgcn_readlane(mykey[hs], t);
#pragma unroll
      for (int h = 0; h < NHC; h++) myrank[h] += k < mykey[h] ? 1 : 0;
    }
  }
#pragma unroll
  for (int h = 0; h < NHC; h++) {
    const int s = LANE + WAVE * h;
    if (s >= ncon) continue;
    const int rank = myrank[h];
    const T* st = w.stage() + 8 * s;
    int* ci = w.ci() + 4 * rank;
    T* cr = w.cr() + CR_N * rank;
    const uint32_t pwd = w.spw()[s];
    ci[0] = (int)(pwd & 0xFFFFFF);
    ci[3] = (int)(pwd >> 24);
    cr[CR_DIST] = st[0];
    cr[CR_POS] = st[1];
    cr[CR_POS + 1] = st[2];
    cr[CR_POS + 2] = st[3];
    cr[CR_FR] = st[4];
    cr[CR_FR + 1] = st[5];
    cr[CR_FR + 2] = st[6];
  }
  if (LANE == 0) {
    misc[MISC_NCON] = ncon;
    misc[MISC_NROW] = 0;
    misc[MISC_CSUM] += nst;  // contact demand of this stage (before any capacity cut), for the counters
    misc[MISC_CMAX] = nst > misc[MISC_CMAX] ? nst : misc[MISC_CMAX];
  }
  SYNC();
}

// ------------------------------------------------------------------------------------------------
// stage (mj_step1): kinematics, inertia, bias forces, collision, constraint rows, efc velocities
// ------------------------------------------------------------------------------------------------
// ---- arm template constants (fm_arm_table.hpp, generated from fm_scene.cpp): with the body loop unrolled
// every table entry is an immediate; products with an exact 0 drop out and products with an exact +-1
// become copies (the same value the full product gives), so the chain carries only the real arithmetic
template <typename T>
__device__ __forceinline__ T cmul(T x, double c) {
  return c == 0.0 ? T(-0.0) : (T(c) == T(1) ? x : (T(c) == T(-1) ? -x : x * T(c)));
}
// r = R v, R a runtime matrix, v a constant vector
template <typename T>
__device__ __forceinline__ void matvec3_c(const T* R, const double* v, T* r) {
#pragma unroll
  for (int i = 0; i < 3; i++) r[i] = cmul(R[3 * i], v[0]) + cmul(R[3 * i + 1], v[1]) + cmul(R[3 * i + 2], v[2]);
}
// C = A B, A runtime, B constant
template <typename T>
__device__ __forceinline__ void matmul3_c(const T* A, const double* B, T* C) {
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++)
      C[3 * i + j] = cmul(A[3 * i], B[j]) + cmul(A[3 * i + 1], B[3 + j]) + cmul(A[3 * i + 2], B[6 + j]);
}

// sin / cos of the 7 hinge angles of every arm, one lane per hinge, ahead of the serial chain (the Hessian
// region is free during kinematics and holds nv^2 >= 104 A reals: arm_body_post's 90 per arm, then these 14)
template <typename T, typename DIM>
__device__ __forceinline__ T* arm_hinge_sc(const Ws<T, DIM>& w, int A, int arm) {
  return w.H() + 90 * A + 14 * arm;
}
template <typename T, typename DIM>
__device__ __forceinline__ void arm_hinge_sincos(const Model<T>& M, const Ws<T, DIM>& w) {
  const DIM dm(M.dm);
  for (int e = LANE; e < 7 * dm.A; e += WAVE) {
    const int arm = e / 7, j = e - 7 * arm;
    T* sc = arm_hinge_sc(w, dm.A, arm) + 2 * j;
    sincos_t(w.q()[1 + 7 * dm.K + 9 * arm + j], sc, sc + 1);
  }
}

// Forward kinematics (+ RNE when DYN) of one arm on one lane: link1..7 (hinges about local z), the gripper
// base (welded), the two plates (slides along local x) -- iiwa14.xml:62-139, gripper.xml:9-42.  Body poses,
// joint axes/anchors, coms, world inertias, gripper site to LDS; DYN adds the RNE bias forces (qacc = 0)
// of the arm's 9 dofs (MuJoCo mj_rne with flg_acc = 0: cvel / cacc recursion then the backward sum).
template <typename T, typename DIM, bool DYN>
__device__ __forceinline__ void arm_chain(const Model<T>& M, const Ws<T, DIM>& w, int arm) {
  const DIM dm(M.dm);
  const T* qa = w.q() + 1 + 7 * dm.K + 9 * arm;
  const T* va = w.v() + 1 + 6 * dm.K + 9 * arm;
  const T* hsc = arm_hinge_sc(w, dm.A, arm);
  T q[9], qd[9];
#pragma unroll
  for (int k = 0; k < 9; k++) {
    q[k] = qa[k];
    qd[k] = DYN ? va[k] : T(0);
  }
  const T* base = M.arm_base + 12 * arm;
  T* bpos = w.bpos() + 30 * arm;
  T* bR = w.bR() + 90 * arm;
  T* dax = w.dax() + 27 * arm;
  T* danc = w.danc() + 27 * arm;
  const T p0[3] = {base[0], base[1], base[2]};
  T Pp[3] = {base[0], base[1], base[2]}, PR[9];
#pragma unroll
  for (int k = 0; k < 9; k++) PR[k] = base[3 + k];
  T Pw[3] = {0, 0, 0}, Pal[3] = {0, 0, 0}, Pvo[3] = {0, 0, 0}, Pao[3] = {0, 0, 0};
  T Gp[3], GR[9], Gw[3], Gal[3], Gvo[3], Gao[3];
#pragma unroll
  for (int b = 0; b < 10; b++) {
    const double* bl = ARM_BODY[b];
    if (b >= 8) {  // both plates hang off the gripper base
#pragma unroll
      for (int k = 0; k < 3; k++) {
        Pp[k] = Gp[k];
        Pw[k] = Gw[k];
        Pal[k] = Gal[k];
        Pvo[k] = Gvo[k];
        Pao[k] = Gao[k];
      }
#pragma unroll
      for (int k = 0; k < 9; k++) PR[k] = GR[k];
    }
    T off[3], Rpre[9];
    matvec3_c(PR, bl, off);
    matmul3_c(PR, bl + 3, Rpre);
    T o[3] = {Pp[0] + off[0], Pp[1] + off[1], Pp[2] + off[2]};
    T R[9];
    T wv[3] = {Pw[0], Pw[1], Pw[2]}, al[3] = {Pal[0], Pal[1], Pal[2]};
    T vo[3] = {0, 0, 0}, ao[3] = {0, 0, 0};
    T r[3], t1[3], t2[3], t3[3];
    if (DYN) {
#pragma unroll
      for (int k = 0; k < 3; k++) r[k] = o[k] - Pp[k];
      cross3(Pw, r, t1);
      cross3(Pal, r, t2);
      cross3(Pw, t1, t3);
    }
    if (b < 7) {
      const T ax[3] = {Rpre[2], Rpre[5], Rpre[8]};
#pragma unroll
      for (int k = 0; k < 3; k++) {
        dax[3 * b + k] = ax[k];
        danc[3 * b + k] = o[k];
      }
      const T sn = hsc[2 * b], cs = hsc[2 * b + 1];
#pragma unroll
      for (int rr = 0; rr < 3; rr++) {
        R[3 * rr + 0] = Rpre[3 * rr + 0] * cs + Rpre[3 * rr + 1] * sn;
        R[3 * rr + 1] = -Rpre[3 * rr + 0] * sn + Rpre[3 * rr + 1] * cs;
        R[3 * rr + 2] = Rpre[3 * rr + 2];
      }
      if (DYN) {
        T wa[3];
        cross3(Pw, ax, wa);
#pragma unroll
        for (int k = 0; k < 3; k++) {
          vo[k] = Pvo[k] + t1[k];
          ao[k] = Pao[k] + t2[k] + t3[k];
          al[k] += wa[k] * qd[b];
          wv[k] += ax[k] * qd[b];
        }
      }
    } else if (b == 7) {
#pragma unroll
      for (int k = 0; k < 9; k++) R[k] = Rpre[k];
      if (DYN) {
#pragma unroll
        for (int k = 0; k < 3; k++) {
          vo[k] = Pvo[k] + t1[k];
          ao[k] = Pao[k] + t2[k] + t3[k];
        }
      }
    } else {
      const int d = b - 1;  // dof 7 (left plate, body 8) / 8 (right plate, body 9)
      const T ax[3] = {Rpre[0], Rpre[3], Rpre[6]};
#pragma unroll
      for (int k = 0; k < 3; k++) {
        o[k] += ax[k] * q[d];
        dax[3 * d + k] = ax[k];
        danc[3 * d + k] = o[k];
      }
#pragma unroll
      for (int k = 0; k < 9; k++) R[k] = Rpre[k];
      if (DYN) {
        // r includes the slide displacement
#pragma unroll
        for (int k = 0; k < 3; k++) r[k] = o[k] - Pp[k];
        cross3(Pw, r, t1);
        cross3(Pal, r, t2);
        cross3(Pw, t1, t3);
        T wa[3];
        cross3(Pw, ax, wa);
#pragma unroll
        for (int k = 0; k < 3; k++) {
          vo[k] = Pvo[k] + t1[k] + ax[k] * qd[d];
          ao[k] = Pao[k] + t2[k] + t3[k] + T(2) * wa[k] * qd[d];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 3; k++) bpos[3 * b + k] = o[k];
#pragma unroll
    for (int k = 0; k < 9; k++) bR[9 * b + k] = R[k];
    if (DYN) {
      // the body's angular velocity / acceleration and origin acceleration for the per-body pass
      // (arm_body_post); the Hessian region is free during kinematics
      T* sc = w.H() + 90 * arm + 9 * b;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        sc[k] = wv[k];
        sc[3 + k] = al[k];
        sc[6 + k] = ao[k];
      }
    }
    // advance the chain
#pragma unroll
    for (int k = 0; k < 3; k++) Pp[k] = o[k];
#pragma unroll
    for (int k = 0; k < 9; k++) PR[k] = R[k];
    if (DYN) {
#pragma unroll
      for (int k = 0; k < 3; k++) {
        Pw[k] = wv[k];
        Pal[k] = al[k];
        Pvo[k] = vo[k];
        Pao[k] = ao[k];
      }
    }
    if (b == 7) {
#pragma unroll
      for (int k = 0; k < 3; k++) {
        Gp[k] = o[k];
        Gw[k] = Pw[k];
        Gal[k] = Pal[k];
        Gvo[k] = Pvo[k];
        Gao[k] = Pao[k];
      }
#pragma unroll
      for (int k = 0; k < 9; k++) GR[k] = R[k];
      // between_gripper_plates site (gripper.xml:43)
      T sp[3];
      matvec3_c(R, ARM_GRIP_SITE, sp);
#pragma unroll
      for (int k = 0; k < 3; k++) w.site()[3 * arm + k] = o[k] + sp[k];
    }
  }
}

// Per-body part of the arm kinematics, one lane per (arm, body) after arm_chain: com, world inertia and, with
// DYN, the RNE body force / moment about the arm base (MuJoCo mj_rne, flg_acc = 0).  The same expressions the
// chain lane evaluated before (body constants now from the scene table, the chain's outputs from LDS).
template <typename T, typename DIM, bool DYN>
__device__ __forceinline__ void arm_body_post(const Model<T>& M, const Ws<T, DIM>& w, int arm, int b) {
  const T* bl = M.body + 32 * b;
  const T* base = M.arm_base + 12 * arm;
  const T* o = w.bpos() + 30 * arm + 3 * b;
  const T* R = w.bR() + 90 * arm + 9 * b;
  T Rr[9];
#pragma unroll
  for (int k = 0; k < 9; k++) Rr[k] = R[k];
  T ci[3];
  matvec3(Rr, bl + 13, ci);
  const T com[3] = {o[0] + ci[0], o[1] + ci[1], o[2] + ci[2]};
  T* bcom = w.bcom() + 30 * arm + 3 * b;
#pragma unroll
  for (int k = 0; k < 3; k++) bcom[k] = com[k];
  T Ri[9];
  matmul3(Rr, bl + 16, Ri);
  const T* I = bl + 25;
  T Iw[6];
  Iw[0] = Ri[0] * Ri[0] * I[0] + Ri[1] * Ri[1] * I[1] + Ri[2] * Ri[2] * I[2];
  Iw[1] = Ri[3] * Ri[3] * I[0] + Ri[4] * Ri[4] * I[1] + Ri[5] * Ri[5] * I[2];
  Iw[2] = Ri[6] * Ri[6] * I[0] + Ri[7] * Ri[7] * I[1] + Ri[8] * Ri[8] * I[2];
  Iw[3] = Ri[0] * Ri[3] * I[0] + Ri[1] * Ri[4] * I[1] + Ri[2] * Ri[5] * I[2];
  Iw[4] = Ri[0] * Ri[6] * I[0] + Ri[1] * Ri[7] * I[1] + Ri[2] * Ri[8] * I[2];
  Iw[5] = Ri[3] * Ri[6] * I[0] + Ri[4] * Ri[7] * I[1] + Ri[5] * Ri[8] * I[2];
  T* bIw = w.bIw() + 60 * arm + 6 * b;
#pragma unroll
  for (int k = 0; k < 6; k++) bIw[k] = Iw[k];
  if (DYN) {
    const T* sc = w.H() + 90 * arm + 9 * b;
    const T wv[3] = {sc[0], sc[1], sc[2]}, al[3] = {sc[3], sc[4], sc[5]}, ao[3] = {sc[6], sc[7], sc[8]};
    const T mass = bl[12];
    const T rc[3] = {com[0] - o[0], com[1] - o[1], com[2] - o[2]};
    T u1[3], u2[3], u3[3];
    cross3(al, rc, u1);
    cross3(wv, rc, u2);
    cross3(wv, u2, u3);
    T F[3];
#pragma unroll
    for (int k = 0; k < 3; k++) F[k] = (ao[k] + u1[k] + u3[k]) * mass;
    F[2] += mass * M.grav;
    T Iwv[3] = {Iw[0] * wv[0] + Iw[3] * wv[1] + Iw[4] * wv[2], Iw[3] * wv[0] + Iw[1] * wv[1] + Iw[5] * wv[2],
                Iw[4] * wv[0] + Iw[5] * wv[1] + Iw[2] * wv[2]};
    T Ial[3] = {Iw[0] * al[0] + Iw[3] * al[1] + Iw[4] * al[2], Iw[3] * al[0] + Iw[1] * al[1] + Iw[5] * al[2],
                Iw[4] * al[0] + Iw[5] * al[1] + Iw[2] * al[2]};
    T gy[3];
    cross3(wv, Iwv, gy);
    T cr[3] = {com[0] - base[0], com[1] - base[1], com[2] - base[2]}, mo[3];
    cross3(cr, F, mo);
    T* bF = w.bF() + 30 * arm + 3 * b;
    T* bN = w.bN() + 30 * arm + 3 * b;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      bF[k] = F[k];
      bN[k] = mo[k] + Ial[k] + gy[k];
    }
  }
}

// RNE backward pass of one arm (one lane per arm, after arm_body_post): generalized bias forces of the arm's
// 9 dofs (qacc = 0); the per-body records come back from LDS in one batch of independent reads
template <typename T, typename DIM>
__device__ __forceinline__ void arm_rne_back(const Model<T>& M, const Ws<T, DIM>& w, int arm) {
  const DIM dm(M.dm);
  const T* base = M.arm_base + 12 * arm;
  const T p0[3] = {base[0], base[1], base[2]};
  const T* bF = w.bF() + 30 * arm;
  const T* bN = w.bN() + 30 * arm;
  const T* dax = w.dax() + 27 * arm;
  const T* danc = w.danc() + 27 * arm;
  T* pb = w.pb() + 1 + 6 * dm.K + 9 * arm;
  pb[7] = -(dax[21] * bF[24] + dax[22] * bF[25] + dax[23] * bF[26]);
  pb[8] = -(dax[24] * bF[27] + dax[25] * bF[28] + dax[26] * bF[29]);
  T ft[3] = {0, 0, 0}, nt[3] = {0, 0, 0};
#pragma unroll
  for (int b = 9; b >= 0; b--) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      ft[k] += bF[3 * b + k];
      nt[k] += bN[3 * b + k];
    }
    if (b <= 6) {
      T ar[3] = {danc[3 * b] - p0[0], danc[3 * b + 1] - p0[1], danc[3 * b + 2] - p0[2]}, af[3];
      cross3(ar, ft, af);
      T tn[3] = {nt[0] - af[0], nt[1] - af[1], nt[2] - af[2]};
      pb[b] = -dot3(dax + 3 * b, tn);
    }
  }
}

// DPP moves inside rows of 16 lanes (dpp_row): row_shr:n (lane l reads lane l - n) and row_shl:n (lane l reads
// l + n); a lane whose source lies outside its row keeps its own value.  Full wave active at every call site.
enum { DPP_SHR = 0x110, DPP_SHL = 0x100 };

// Arm kinematics + RNE of the physics substep (arm_chain<DYN> + arm_body_post<DYN> + arm_rne_back) as scans
// over the kinematic chain instead of one serial lane per arm: arm a's body b on lane 16 a + b (one DPP row per
// arm, A <= 4).  The chain link1..7, gripper base, left plate occupies lanes b = 0..8 (each body's parent is the
// lane before); the right plate (b = 9) hangs off the gripper base (b = 7) and joins after each scan.
//  * poses: every lane builds its body's transform relative to its parent (hinge: R_body Rz(q); plate: the slide
//    along the local x axis), then a Hillis-Steele scan of rigid-transform products over row_shr 1, 2, 4, 8 gives
//    the pose relative to the arm base; one product with the base gives the world pose (a reassociation of the
//    serial chain's products);
//  * velocities (flg_acc = 0): angular velocity, angular acceleration and origin acceleration are sums along the
//    chain of per-body terms (a hinge adds axis * qdot to w and (w_parent x axis) qdot to the angular
//    acceleration; every body adds alpha_parent x r + w_parent x (w_parent x r), a plate also
//    2 (w_parent x axis) qdot), each a prefix-sum scan once its terms' parent values are known;
//  * the per-body com / world inertia / RNE force and moment of arm_body_post on the same lane, then the RNE
//    backward sums over the subtrees (both plates folded into the gripper base, a row_shl suffix scan) and the
//    bias forces of the 9 dofs.
// Outputs to LDS as the serial path: body poses, joint axes / anchors, site, coms, world inertias, qfrc_bias.
template <typename T, typename DIM>
__device__ __forceinline__ void arm_fk_scan(const Model<T>& M, const Ws<T, DIM>& w) {
  const DIM dm(M.dm);
  const int A = dm.A, K = dm.K;
  const int arm = LANE >> 4, b = LANE & 15;
  const bool on = arm < A && b < 10;
  const int bb = on ? b : 0, aa = on ? arm : 0;  // clamped for the table loads
  const T* bl = M.body + 32 * bb;
  const T* base = M.arm_base + 12 * aa;
  const int d = bb < 7 ? bb : (bb == 7 ? -1 : bb - 1);  // the body's joint: hinge b, none, slide dof 7 / 8
  const T qj = d >= 0 ? w.q()[1 + 7 * K + 9 * aa + d] : T(0);
  const T vj = d >= 0 ? w.v()[1 + 6 * K + 9 * aa + d] : T(0);
  T R[9], p[3];
  {
    T BR[9], lp[3];
#pragma unroll
    for (int k = 0; k < 9; k++) BR[k] = bl[3 + k];
#pragma unroll
    for (int k = 0; k < 3; k++) lp[k] = bl[k];
    T sn, cs;
    sincos_t(bb < 7 ? qj : T(0), &sn, &cs);
    const bool hinge = bb < 7, slide = bb >= 8;
#pragma unroll
    for (int r = 0; r < 3; r++) {
      R[3 * r + 0] = hinge ? BR[3 * r + 0] * cs + BR[3 * r + 1] * sn : BR[3 * r + 0];
      R[3 * r + 1] = hinge ? -BR[3 * r + 0] * sn + BR[3 * r + 1] * cs : BR[3 * r + 1];
      R[3 * r + 2] = BR[3 * r + 2];
      p[r] = slide ? lp[r] + BR[3 * r] * qj : lp[r];
    }
  }
  // X = (Ra, pa) o X
  auto compose = [&](const T* Ra, const T* pa) {
    T Rn[9], pn[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
#pragma unroll
      for (int j = 0; j < 3; j++) Rn[3 * i + j] = Ra[3 * i] * R[j] + Ra[3 * i + 1] * R[3 + j] + Ra[3 * i + 2] * R[6 + j];
      pn[i] = pa[i] + Ra[3 * i] * p[0] + Ra[3 * i + 1] * p[1] + Ra[3 * i + 2] * p[2];
    }
#pragma unroll
    for (int k = 0; k < 9; k++) R[k] = Rn[k];
#pragma unroll
    for (int k = 0; k < 3; k++) p[k] = pn[k];
  };
  static_for<0, 4>([&](auto rc) {
    constexpr int s = 1 << decltype(rc)::value;
    T Ra[9], pa[3];
#pragma unroll
    for (int k = 0; k < 9; k++) Ra[k] = dpp_row<DPP_SHR | s>(R[k]);
#pragma unroll
    for (int k = 0; k < 3; k++) pa[k] = dpp_row<DPP_SHR | s>(p[k]);
    if (b >= s && b <= 8) compose(Ra, pa);
  });
  {
    T Ra[9], pa[3];
#pragma unroll
    for (int k = 0; k < 9; k++) Ra[k] = dpp_row<DPP_SHR | 2>(R[k]);
#pragma unroll
    for (int k = 0; k < 3; k++) pa[k] = dpp_row<DPP_SHR | 2>(p[k]);
    if (b == 9) compose(Ra, pa);  // right plate: gripper base o right plate
  }
  const T p0[3] = {base[0], base[1], base[2]};
  {
    T Rb[9];
#pragma unroll
    for (int k = 0; k < 9; k++) Rb[k] = base[3 + k];
    compose(Rb, p0);
  }
  // joint axis (hinge: local z; slide: local x) and anchor
  const T ax[3] = {bb < 7 ? R[2] : (bb >= 8 ? R[0] : T(0)), bb < 7 ? R[5] : (bb >= 8 ? R[3] : T(0)),
                   bb < 7 ? R[8] : (bb >= 8 ? R[6] : T(0))};
  if (on) {
    T* bpos = w.bpos() + 30 * arm + 3 * b;
    T* bR = w.bR() + 90 * arm + 9 * b;
#pragma unroll
    for (int k = 0; k < 3; k++) bpos[k] = p[k];
#pragma unroll
    for (int k = 0; k < 9; k++) bR[k] = R[k];
    if (d >= 0) {
#pragma unroll
      for (int k = 0; k < 3; k++) {
        w.dax()[27 * arm + 3 * d + k] = ax[k];
        w.danc()[27 * arm + 3 * d + k] = p[k];
      }
    }
    if (b == 7) {  // between_gripper_plates site (gripper.xml:43)
      T sp[3];
      matvec3_c(R, ARM_GRIP_SITE, sp);
#pragma unroll
      for (int k = 0; k < 3; k++) w.site()[3 * arm + k] = p[k] + sp[k];
    }
  }
  // prefix sums along the chain (lanes 0..8), the right plate takes the gripper base's value plus its own term
  auto chain_sum = [&](T* x) {
    static_for<0, 4>([&](auto rc) {
      constexpr int s = 1 << decltype(rc)::value;
      T t[3];
#pragma unroll
      for (int k = 0; k < 3; k++) t[k] = dpp_row<DPP_SHR | s>(x[k]);
      if (b >= s && b <= 8) {
#pragma unroll
        for (int k = 0; k < 3; k++) x[k] += t[k];
      }
    });
    T t[3];
#pragma unroll
    for (int k = 0; k < 3; k++) t[k] = dpp_row<DPP_SHR | 2>(x[k]);
    if (b == 9) {
#pragma unroll
      for (int k = 0; k < 3; k++) x[k] += t[k];
    }
  };
  // the parent's value of x (the arm base's `root` for b = 0)
  auto parent = [&](const T* x, const T* root, T* out) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const T t1 = dpp_row<DPP_SHR | 1>(x[k]), t2 = dpp_row<DPP_SHR | 2>(x[k]);
      out[k] = b == 0 ? root[k] : (b == 9 ? t2 : t1);
    }
  };
  const T zero3[3] = {T(0), T(0), T(0)};
  T wv[3] = {bb < 7 ? ax[0] * vj : T(0), bb < 7 ? ax[1] * vj : T(0), bb < 7 ? ax[2] * vj : T(0)};
  chain_sum(wv);
  T wp[3];
  parent(wv, zero3, wp);
  T wa[3];  // w_parent x axis
  cross3(wp, ax, wa);
  T al[3] = {bb < 7 ? wa[0] * vj : T(0), bb < 7 ? wa[1] * vj : T(0), bb < 7 ? wa[2] * vj : T(0)};
  chain_sum(al);
  T alp[3], op[3];
  parent(al, zero3, alp);
  parent(p, p0, op);
  T ao[3];
  {
    const T r[3] = {p[0] - op[0], p[1] - op[1], p[2] - op[2]};
    T t1[3], t2[3], t3[3];
    cross3(wp, r, t1);
    cross3(alp, r, t2);
    cross3(wp, t1, t3);
#pragma unroll
    for (int k = 0; k < 3; k++) ao[k] = t2[k] + t3[k] + (bb >= 8 ? T(2) * wa[k] * vj : T(0));
  }
  chain_sum(ao);
  // arm_body_post on this lane: com, world inertia, RNE body force / moment about the arm base
  T F[3], N[3];
  {
    T ci[3];
    matvec3(R, bl + 13, ci);
    const T com[3] = {p[0] + ci[0], p[1] + ci[1], p[2] + ci[2]};
    T Ri[9];
    matmul3(R, bl + 16, Ri);
    const T I0 = bl[25], I1 = bl[26], I2 = bl[27];
    T Iw[6];
    Iw[0] = Ri[0] * Ri[0] * I0 + Ri[1] * Ri[1] * I1 + Ri[2] * Ri[2] * I2;
    Iw[1] = Ri[3] * Ri[3] * I0 + Ri[4] * Ri[4] * I1 + Ri[5] * Ri[5] * I2;
    Iw[2] = Ri[6] * Ri[6] * I0 + Ri[7] * Ri[7] * I1 + Ri[8] * Ri[8] * I2;
    Iw[3] = Ri[0] * Ri[3] * I0 + Ri[1] * Ri[4] * I1 + Ri[2] * Ri[5] * I2;
    Iw[4] = Ri[0] * Ri[6] * I0 + Ri[1] * Ri[7] * I1 + Ri[2] * Ri[8] * I2;
    Iw[5] = Ri[3] * Ri[6] * I0 + Ri[4] * Ri[7] * I1 + Ri[5] * Ri[8] * I2;
    if (on) {
      T* bcom = w.bcom() + 30 * arm + 3 * b;
      T* bIw = w.bIw() + 60 * arm + 6 * b;
#pragma unroll
      for (int k = 0; k < 3; k++) bcom[k] = com[k];
#pragma unroll
      for (int k = 0; k < 6; k++) bIw[k] = Iw[k];
    }
    const T mass = bl[12];
    const T rc[3] = {com[0] - p[0], com[1] - p[1], com[2] - p[2]};
    T u1[3], u2[3], u3[3];
    cross3(al, rc, u1);
    cross3(wv, rc, u2);
    cross3(wv, u2, u3);
#pragma unroll
    for (int k = 0; k < 3; k++) F[k] = (ao[k] + u1[k] + u3[k]) * mass;
    F[2] += mass * M.grav;
    const T Iwv[3] = {Iw[0] * wv[0] + Iw[3] * wv[1] + Iw[4] * wv[2], Iw[3] * wv[0] + Iw[1] * wv[1] + Iw[5] * wv[2],
                      Iw[4] * wv[0] + Iw[5] * wv[1] + Iw[2] * wv[2]};
    const T Ial[3] = {Iw[0] * al[0] + Iw[3] * al[1] + Iw[4] * al[2], Iw[3] * al[0] + Iw[1] * al[1] + Iw[5] * al[2],
                      Iw[4] * al[0] + Iw[5] * al[1] + Iw[2] * al[2]};
    T gy[3];
    cross3(wv, Iwv, gy);
    const T cr[3] = {com[0] - p0[0], com[1] - p0[1], com[2] - p0[2]};
    T mo[3];
    cross3(cr, F, mo);
#pragma unroll
    for (int k = 0; k < 3; k++) N[k] = mo[k] + Ial[k] + gy[k];
  }
  // RNE backward: subtree sums of (F, N); the plates fold into the gripper base, then a suffix scan over b <= 7
  T X[6] = {F[0], F[1], F[2], N[0], N[1], N[2]};
  {
    T t1[6], t2[6];
#pragma unroll
    for (int k = 0; k < 6; k++) {
      t1[k] = dpp_row<DPP_SHL | 1>(X[k]);
      t2[k] = dpp_row<DPP_SHL | 2>(X[k]);
    }
    if (b == 7) {
#pragma unroll
      for (int k = 0; k < 6; k++) X[k] += t1[k] + t2[k];
    }
  }
  static_for<0, 3>([&](auto rc) {
    constexpr int s = 1 << decltype(rc)::value;
    T t[6];
#pragma unroll
    for (int k = 0; k < 6; k++) t[k] = dpp_row<DPP_SHL | s>(X[k]);
    if (b + s <= 7) {
#pragma unroll
      for (int k = 0; k < 6; k++) X[k] += t[k];
    }
  });
  if (on && d >= 0) {
    T tq;
    if (b < 7) {
      const T ar[3] = {p[0] - p0[0], p[1] - p0[1], p[2] - p0[2]};
      T af[3];
      cross3(ar, X, af);
      const T tn[3] = {X[3] - af[0], X[4] - af[1], X[5] - af[2]};
      tq = -dot3(ax, tn);
    } else {
      tq = -(ax[0] * F[0] + ax[1] * F[1] + ax[2] * F[2]);
    }
    w.pb()[1 + 6 * K + 9 * arm + d] = tq;
  }
}

// column of the translational Jacobian of point p on arm body b for arm dof d (0 if not in chain)
template <typename T, typename DIM>
__device__ __forceinline__ void arm_jac_col(const Ws<T, DIM>& w, int arm, int b, int d, const T* p, T* col) {
  const T* ax = w.dax() + 27 * arm + 3 * d;
  bool in = d < 7 ? (b >= 7 || d <= b) : ((d == 7 && b == 8) || (d == 8 && b == 9));
  if (!in) {
    col[0] = col[1] = col[2] = 0;
    return;
  }
  if (d < 7) {
    const T* an = w.danc() + 27 * arm + 3 * d;
    T rel[3] = {p[0] - an[0], p[1] - an[1], p[2] - an[2]};
    cross3(ax, rel, col);
  } else {
    col[0] = ax[0];
    col[1] = ax[1];
    col[2] = ax[2];
  }
}

// the point a contact's Jacobian columns on kernel body kb need (p = the contact point relative to its anchor o,
// contact_anchor): a cube's lever arm p - c formed as p + (o - c) with o - c in float64 (exactly 0 for the anchor
// cube itself); an arm body's point in the kernel frame
template <typename T, typename DIM>
__device__ __forceinline__ void body_jac_point(const Model<T>& M, const Ws<T, DIM>& w, int kb, const T* p,
                                               const double* o, int ak, T* pt) {
  const DIM dm(M.dm);
  if (kb - 2 == ak) {  // the anchor cube itself: the stored point is its lever arm
    pt[0] = p[0];
    pt[1] = p[1];
    pt[2] = p[2];
  } else if (kb >= 2 && kb < 2 + dm.K) {
    const double* c = w.qd() + 1 + 7 * (kb - 2);
    pt[0] = p[0] + (T)(o[0] - c[0]);
    pt[1] = p[1] + (T)(o[1] - c[1]);
    pt[2] = p[2] + (T)(o[2] - (c[2] - zshift<T>()));
  } else {
    pt[0] = (T)(o[0] + (double)p[0]);
    pt[1] = (T)(o[1] + (double)p[1]);
    pt[2] = (T)(o[2] + (double)p[2]);
  }
}

// translational Jacobian column j (tree-local) on kernel body kb in its tree; pt from body_jac_point (a cube's lever
// arm, an arm body's point)
template <typename T, typename DIM>
__device__ __forceinline__ void body_jac_col(const Model<T>& M, const Ws<T, DIM>& w, int kb, int j, const T* pt, T* col) {
  const DIM dm(M.dm);
  if (kb == 1) {
    col[0] = 0;
    col[1] = 1;
    col[2] = 0;
  } else if (kb < 2 + dm.K) {
    int k = kb - 2;
    if (j < 3) {
      col[0] = col[1] = col[2] = 0;
      col[j] = 1;
    } else {
      const T* R = w.cR() + 9 * k;
      T ax[3] = {R[j - 3], R[3 + j - 3], R[6 + j - 3]};
      cross3(ax, pt, col);
    }
  } else {
    const T* p = pt;
    int arm = (kb - 2 - dm.K) / 10, b = (kb - 2 - dm.K) % 10;
    arm_jac_col(w, arm, b, j, p, col);
  }
}

template <typename O, typename T, typename DIM, typename X>
__device__ __forceinline__ void contact_jx(const Model<T>& M, const Ws<T, DIM>& w, const X* x, int ncon, int slot);

template <typename T, typename DIM>
__device__ __forceinline__ void stage(const Model<T>& M, const Ws<T, DIM>& w, int arena, int64_t* ctr) {
  const DIM dm(M.dm);
  const int A = dm.A, K = dm.K, nv = dm.nv;
  T* q = w.q();
  T* v = w.v();
  // ---- kinematics + RNE: scans over each arm's chain (arm_fk_scan, A <= 4; more arms: one lane per arm), cubes (one
  // lane per cube)
  const bool fk_scan = dm.A <= 4;
  if (fk_scan) {
    arm_fk_scan(M, w);
  } else {
    arm_hinge_sincos(M, w);
    SYNC();
    if (LANE < A) arm_chain<T, DIM, true>(M, w, LANE);
  }
  for (int k = LANE; k < K; k += WAVE) {
    T* qq = q + 1 + 7 * k;
    T qu[4] = {qq[3], qq[4], qq[5], qq[6]};
    T n = sqrt(qu[0] * qu[0] + qu[1] * qu[1] + qu[2] * qu[2] + qu[3] * qu[3]);
    if (n < T(1e-15)) {
      qu[0] = 1;
      qu[1] = qu[2] = qu[3] = 0;
    } else if (fabs(n - T(1)) > T(1e-15)) {
      for (int c = 0; c < 4; c++) qu[c] /= n;
    }
    T* R = w.cR() + 9 * k;
    T ww = qu[0], x = qu[1], y = qu[2], z = qu[3];
    R[0] = ww * ww + x * x - y * y - z * z;
    R[1] = T(2) * (x * y - ww * z);
    R[2] = T(2) * (x * z + ww * y);
    R[3] = T(2) * (x * y + ww * z);
    R[4] = ww * ww - x * x + y * y - z * z;
    R[5] = T(2) * (y * z - ww * x);
    R[6] = T(2) * (x * z - ww * y);
    R[7] = T(2) * (y * z + ww * x);
    R[8] = ww * ww - x * x - y * y + z * z;
    // passive - bias of the free joint: gravity only (com at the body origin, isotropic inertia)
    T* pb = w.pb() + 1 + 6 * k;
    T m = w.cube()[4 * k + 1];
    pb[0] = 0;
    pb[1] = 0;
    pb[2] = -m * M.grav;
    pb[3] = pb[4] = pb[5] = 0;
  }
  if (LANE == 0) w.pb()[0] = -M.belt_damp * v[0];  // belt: damping, no gravity along y
  if constexpr (DIM::f64arms && sizeof(T) == 4) {
    if (LANE < A) arm_pose_f64(M, w, LANE);
  }
  SYNC();
  if (!fk_scan) {
    // per-body com / inertia / RNE forces one lane per (arm, body), then the RNE backward sum one lane per arm
    for (int e = LANE; e < 10 * A; e += WAVE) arm_body_post<T, DIM, true>(M, w, e / 10, e % 10);
    SYNC();
    if (LANE < A) arm_rne_back(M, w, LANE);
    SYNC();
  }
  PMARK(PH_FK);
  // ---- arm mass-matrix blocks, composite-rigid-body style.  Hinge i moves the bodies b >= i; about its anchor
  // p_i their composite mass moment h_i = sum m r and inertia J_i = sum Iw + m (|r|^2 1 - r r'), r = com - p_i
  // (one lane per hinge; the Hessian region is free before the collision).  Then one entry (i >= j) per lane:
  //   hinges i >= j:  M_ij = a_i' J_i a_j + (a_i x h_i) . (a_j x (p_i - p_j))
  //   slide i (its plate only):  M_ij = m (a_i . c_j), c_j = a_j x (com - p_j) for a hinge j, a_i for j = i.
  // Same sums as sum_{b in desc} m Jc_i.Jc_j + Jr_i' Iw Jr_j, regrouped per subtree.
  for (int e = LANE; e < 7 * A; e += WAVE) {
    const int arm = e / 7, i = e - 7 * arm;
    const T* danc = w.danc() + 27 * arm;
    const T* bcom = w.bcom() + 30 * arm;
    const T* bIw = w.bIw() + 60 * arm;
    const T pi[3] = {danc[3 * i], danc[3 * i + 1], danc[3 * i + 2]};
    T mh[3] = {0, 0, 0}, J[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < 10; b++) {
      const T* com = bcom + 3 * b;
      const T* Iw = bIw + 6 * b;
      const T m = T(ARM_BODY[b][12]);
      const T r[3] = {com[0] - pi[0], com[1] - pi[1], com[2] - pi[2]};
      const T mr[3] = {m * r[0], m * r[1], m * r[2]};
      const T rr = r[0] * mr[0] + r[1] * mr[1] + r[2] * mr[2];
      const T t[6] = {Iw[0] + rr - r[0] * mr[0], Iw[1] + rr - r[1] * mr[1], Iw[2] + rr - r[2] * mr[2],
                      Iw[3] - r[0] * mr[1], Iw[4] - r[0] * mr[2], Iw[5] - r[1] * mr[2]};
      const bool in = b >= i;
#pragma unroll
      for (int k = 0; k < 3; k++) mh[k] += in ? mr[k] : T(0);
#pragma unroll
      for (int k = 0; k < 6; k++) J[k] += in ? t[k] : T(0);
    }
    T* sc = w.H() + 9 * (7 * arm + i);
#pragma unroll
    for (int k = 0; k < 3; k++) sc[k] = mh[k];
#pragma unroll
    for (int k = 0; k < 6; k++) sc[3 + k] = J[k];
  }
  SYNC();
  for (int e = LANE; e < 45 * A; e += WAVE) {
    const int arm = e / 45;
    const int t = e - 45 * arm;
    int i = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);  // packed lower-triangle index -> (i, j)
    if ((i + 1) * (i + 2) / 2 <= t) i++;
    if (i * (i + 1) / 2 > t) i--;
    const int j = t - i * (i + 1) / 2;
    const T* dax = w.dax() + 27 * arm;
    const T* danc = w.danc() + 27 * arm;
    const T ai[3] = {dax[3 * i], dax[3 * i + 1], dax[3 * i + 2]}, aj[3] = {dax[3 * j], dax[3 * j + 1], dax[3 * j + 2]};
    const T pj[3] = {danc[3 * j], danc[3 * j + 1], danc[3 * j + 2]};
    T s;
    if (i <= 6) {
      const T* sc = w.H() + 9 * (7 * arm + i);
      const T pi[3] = {danc[3 * i], danc[3 * i + 1], danc[3 * i + 2]};
      const T Ja[3] = {sc[3] * aj[0] + sc[6] * aj[1] + sc[7] * aj[2], sc[6] * aj[0] + sc[4] * aj[1] + sc[8] * aj[2],
                       sc[7] * aj[0] + sc[8] * aj[1] + sc[5] * aj[2]};
      const T h[3] = {sc[0], sc[1], sc[2]}, d[3] = {pi[0] - pj[0], pi[1] - pj[1], pi[2] - pj[2]};
      T ah[3], ad[3];
      cross3(ai, h, ah);
      cross3(aj, d, ad);
      s = dot3(ai, Ja) + dot3(ah, ad);
    } else {
      const int b = i + 1;  // the plate
      const T* com = w.bcom() + 30 * arm + 3 * b;
      T cj[3];
      if (j <= 6) {
        const T rj[3] = {com[0] - pj[0], com[1] - pj[1], com[2] - pj[2]};
        cross3(aj, rj, cj);
      } else {
        cj[0] = j == i ? aj[0] : T(0);
        cj[1] = j == i ? aj[1] : T(0);
        cj[2] = j == i ? aj[2] : T(0);
      }
      static_assert(ARM_BODY[8][12] == ARM_BODY[9][12], "the two plates are assumed to weigh the same");
      s = T(ARM_BODY[8][12]) * dot3(ai, cj);
    }
    T* Ma = w.Marm() + 81 * arm;
    Ma[9 * i + j] = s;
    Ma[9 * j + i] = s;
  }
  SYNC();  // collide's geom centres (gx) reuse the H scratch the loop above reads
  PMARK(PH_GEOM);
  collide(M, w, arena, ctr);
  int* misc = w.misc();
  PMARK(PH_COLL);
  const int ncon = misc[MISC_NCON];
  if (M.prof && LANE == 0) w.prof()[PH_NCON] += ncon;
  // ---- contact rows: frame, Jacobian blocks, impedance, D, reference-acceleration terms (one lane per contact;
  // round 4 measured one lane per (contact, column) slower: rows 5.3 -> 7.5 us per arena-substep, the frame and
  // point reloads of every column outweigh the shorter chain)
  for (int c = LANE; c < ncon; c += WAVE) {
    int* ci = w.ci() + 4 * c;
    T* cr = w.cr() + CR_N * c;
    int c1 = ci[0] & 4095, c2 = (ci[0] >> 12) & 4095;
    int pidx = ci[3];
    const int gi1 = w.ginfo()[c1], gi2 = w.ginfo()[c2];
    int kb1 = (gi1 >> 8) & 255, kb2 = (gi2 >> 8) & 255;
    int tr1 = kbody_tree(dm, kb1), tr2 = kbody_tree(dm, kb2);
    int armflag = ((gi1 | gi2) >> GI_ARM) & 1;
    // frame (mju_makeFrame), built in registers and stored once
    T f[9];
    {
      T* fs = cr + CR_FR;
      T n0 = fs[0], n1 = fs[1], n2 = fs[2];
      const T nn = sqrt(n0 * n0 + n1 * n1 + n2 * n2);
      if (nn < T(1e-15)) {
        n0 = 1;
        n1 = n2 = 0;
      } else {
        n0 /= nn;
        n1 /= nn;
        n2 /= nn;
      }
      T t0 = 0, t1 = 0, t2 = 0;
      if (n1 < T(0.5) && n1 > T(-0.5))
        t1 = 1;
      else
        t2 = 1;
      const T tt = n0 * t0 + n1 * t1 + n2 * t2;
      t0 -= tt * n0;
      t1 -= tt * n1;
      t2 -= tt * n2;
      const T m = sqrt(t0 * t0 + t1 * t1 + t2 * t2);
      if (m < T(1e-15)) {
        t0 = 1;
        t1 = t2 = 0;
      } else {
        t0 /= m;
        t1 /= m;
        t2 /= m;
      }
      f[0] = n0;
      f[1] = n1;
      f[2] = n2;
      f[3] = t0;
      f[4] = t1;
      f[5] = t2;
      cross3(f, f + 3, f + 6);
#pragma unroll
      for (int k = 0; k < 9; k++) fs[k] = f[k];
    }
    // Jacobian blocks B = frame * (J(body2) - J(body1)) on the contact point
    int ta = -1, tb = -1;
    if (tr1 >= 0) ta = tr1;
    if (tr2 >= 0) {
      if (ta < 0)
        ta = tr2;
      else if (tr2 != ta)
        tb = tr2;
    }
    int nda = ta >= 0 ? tree_nd(dm, ta) : 0;
    int ndb = tb >= 0 ? tree_nd(dm, tb) : 0;
    const T p[3] = {cr[CR_POS], cr[CR_POS + 1], cr[CR_POS + 2]};
    double o[3];
    const int ak = anchor_cube(dm, kb1, kb2);
    contact_anchor(w, ak, o);
    T pt1[3], pt2[3];
    body_jac_point(M, w, kb1, p, o, ak, pt1);
    body_jac_point(M, w, kb2, p, o, ak, pt2);
    T* J = cr + CR_J;
    for (int blk = 0; blk < 2; blk++) {
      int t = blk == 0 ? ta : tb;
      if (t < 0) continue;
      int nd = blk == 0 ? nda : ndb;
      int col0 = blk == 0 ? 0 : nda;
      for (int j = 0; j < nd; j++) {
        T col[3] = {0, 0, 0};
        if (tr2 == t) {
          T c2v[3];
          body_jac_col(M, w, kb2, j, pt2, c2v);
          for (int k = 0; k < 3; k++) col[k] += c2v[k];
        }
        if (tr1 == t) {
          T c1v[3];
          body_jac_col(M, w, kb1, j, pt1, c1v);
          for (int k = 0; k < 3; k++) col[k] -= c1v[k];
        }
        for (int r = 0; r < 3; r++) J[r * CJ + col0 + j] = dot3(f + 3 * r, col);
      }
    }
    ci[1] = ta;
    ci[2] = tb;
    ci[3] = pidx | (armflag << 16) | (nda << 20) | (ndb << 24);
    // parameters
    // impedance, R and the reference acceleration's gains in float64 in both builds: near solimp's dmax = 0.9999
    // the factor (1 - imp) of R keeps 4 significant digits in float (and 0.9999 itself rounds by 1.7e-4 of it)
    const double* prm = M.param + 8 * pidx;
    const double mu = prm[0];
    const double dist = (double)cr[CR_DIST];
    const double imp = impedance(prm + 3, dist);
    double Kk, Bb;
    kb_params(M.timestep, prm + 1, prm + 3, Kk, Bb);
    auto invw_t = [&](int kb) -> double {
      if (kb == 0) return 0.0;
      if (kb == 1) return (double)M.belt_invw_t;
      if (kb < 2 + K) return 1.0 / (double)w.cube()[4 * (kb - 2) + 1];
      return (double)M.body[32 * ((kb - 2 - K) % 10) + 28];
    };
    const double tran = invw_t(kb1) + invw_t(kb2);
    const double diag = tran + mu * mu * tran;
    // D = 1 / max(R, 1e-15), R = (1 - imp) diag / imp: one division on the lane's chain instead of two
    const double D = imp / ((1.0 - imp) * diag);
    cr[CR_MU] = (T)mu;
    cr[CR_D] = (T)(D < 1e15 ? D : 1e15);
    // pyramid edges: the position term of aref with K / (4 mu^2), pinned by MuJoCo's resting equilibria and
    // belt-carried velocities in the reference runs (oracle/solver.c, tests/test_physics_pins.py)
    cr[CR_KD] = (T)(Kk * imp * dist / (4.0 * mu * mu));
    cr[CR_BD] = (T)Bb;
  }
  SYNC();
  SPLITMARK(1, PH_CHDIAG);
  // efc velocity in the contact frame
  contact_jx<T>(M, w, v, ncon, CR_VEL);
  SPLITMARK(1, PH_CHPANEL);
  // ---- generic rows: gripper joint equality + active joint limits.  One candidate row per lane in the
  // reference's order (per arm: the equality, then each dof's lower and upper limit), compacted by ballot
  {
    constexpr int PER = 19;
    const uint64_t below = (1ull << LANE) - 1ull;
    int nr = 0;
    for (int c00 = 0; c00 < PER * A; c00 += WAVE) {
      const int cand = c00 + LANE;
      bool act = false, eq = false;
      int d0 = 0, d1 = -1;
      T c0 = 0, c1 = 0, diag = 0;
      // the constraint violation from the float64 master state and float64 limits: the plates' equality is a
      // difference of two ~0.06 m slides (a float difference keeps ~7e-9 m of a ~1e-7 m violation)
      double pos = 0.0;
      const double* qd = w.qd();
      if (cand < PER * A) {
        const int arm = cand / PER, k = cand - PER * arm;
        const int qa = 1 + 7 * K + 9 * arm, va = 1 + 6 * K + 9 * arm;
        if (k == 0) {  // gripper plates: q_left - q_right = 0 (gripper.xml:46-49)
          act = eq = true;
          d0 = va + 7;
          d1 = va + 8;
          c0 = T(1);
          c1 = T(-1);
          pos = qd[qa + 7] - qd[qa + 8];
          diag = M.dof[4 * 7 + 2] + M.dof[4 * 8 + 2];
        } else {
          const int d = (k - 1) >> 1;
          const bool upper = (k - 1) & 1;
          const double qv = qd[qa + d];
          pos = upper ? M.dofd[4 * d + 1] - qv : qv - M.dofd[4 * d];
          c0 = upper ? T(-1) : T(1);
          act = pos < 0.0;
          d0 = va + d;
          diag = M.dof[4 * d + 2];
        }
      }
      const uint64_t bal = __ballot(act);
      const int slot = nr + __popcll(bal & below);
      if (act && slot < dm.maxrow) {
        const double sr[2] = {eq ? 0.002 : 0.02, 1.0};
        const double si[5] = {eq ? 0.98 : 0.9, eq ? 0.9999 : 0.95, 0.001, 0.5, 2.0};
        int* ri = w.ri() + 4 * slot;
        T* rr = w.rr() + RR_N * slot;
        ri[0] = d0;
        ri[1] = d1;
        ri[2] = eq ? 0 : 1;  // 0 equality, 1 inequality
        rr[RR_C0] = c0;
        rr[RR_C1] = c1;
        rr[RR_POS] = (T)pos;
        const double imp = impedance(si, pos);
        double Kk, Bb;
        kb_params(M.timestep, sr, si, Kk, Bb);
        const double D = imp / ((1.0 - imp) * (double)diag);  // 1 / max(R, 1e-15), one division
        rr[RR_D] = (T)(D < 1e15 ? D : 1e15);
        const double* vd = w.vd();
        const double vel = (double)c0 * vd[d0] + (d1 >= 0 ? (double)c1 * vd[d1] : 0.0);
        rr[RR_AREF] = (T)(-Bb * vel - Kk * imp * pos);
      }
      nr += __popcll(bal);
    }
    if (LANE == 0) misc[MISC_NROW] = nr < dm.maxrow ? nr : dm.maxrow;
  }
  SYNC();
  SPLITMARK(1, PH_CHTRAIL);
  // ---- tree -> contact masks: one ballot per tree and 64-contact word (word h holds contacts 64 h .. 64 h + 63)
  {
    const int nh = DIM::MAXC == WAVE ? 1 : (dm.maxcon + WAVE - 1) / WAVE;
#pragma unroll
    for (int h = 0; h < DIM::MAXC / WAVE; h++) {
      if (h >= nh) {  // words past the scene's contact capacity hold no contact (readers scan all MAXC / 64)
        for (int t = LANE; t < dm.ntree; t += WAVE) w.tmask()[h * dm.ntree + t] = 0ull;
        continue;
      }
      int ta = -2, tb = -2;
      if (LANE + WAVE * h < ncon) {
        ta = w.ci()[4 * (LANE + WAVE * h) + 1];
        tb = w.ci()[4 * (LANE + WAVE * h) + 2];
      }
      for (int t = 0; t < dm.ntree; t++) {
        const uint64_t mk = __ballot(ta == t || tb == t);
        if (LANE == 0) w.tmask()[h * dm.ntree + t] = mk;
      }
    }
  }
  (void)nv;
  SYNC();
  PMARK(PH_ROWS);
}

// ------------------------------------------------------------------------------------------------
// block-diagonal M products and solves (belt scalar, cubes diagonal, arm 9x9 blocks)
// ------------------------------------------------------------------------------------------------
template <typename T, typename DIM>
__device__ __forceinline__ T Mdiag(const Model<T>& M, const Ws<T, DIM>& w, int i) {
  // both loads unconditional and the select on the values: with `if (i == 0) return M.belt_mass;` the compiler
  // merged the kernarg load and the LDS load into one load through a selected generic pointer (a FLAT instruction,
  // tools/isa_flat.py)
  const T bm = M.belt_mass;
  const int ii = i > 0 ? i - 1 : 0, k = ii / 6, r = ii - 6 * k;
  const T cv = w.cube()[4 * k + (r < 3 ? 1 : 2)];
  return i == 0 ? bm : cv;
}

// out = M x   (lanes over dofs), accumulated in out's type (the solver's float64 vectors: M's float entries
// times float or double operands)
template <typename T, typename DIM, typename X, typename O>
__device__ __forceinline__ void mmul(const Model<T>& M, const Ws<T, DIM>& w, int arena, const X* x, O* out) {
  const DIM dm(M.dm);
  int a0 = 1 + 6 * dm.K;
  for (int i = LANE; i < dm.nv; i += WAVE) {
    if (i < a0) {
      out[i] = (O)Mdiag(M, w, i) * (O)x[i];
    } else {
      int arm = (i - a0) / 9, r = (i - a0) % 9;
      const T* Mb = w.Marm() + 81 * arm + 9 * r;
      const X* xa = x + a0 + 9 * arm;
      O s = 0;
      for (int j = 0; j < 9; j++) s += (O)Mb[j] * (O)xa[j];
      out[i] = s;
    }
  }
}


// 9x9 SPD solve A x = b on one lane with A's lower triangle (packed row-major, P9(i,j) = i(i+1)/2 + j)
// held in registers (right-looking factor, then forward and backward substitution)
__host__ __device__ constexpr int P9(int i, int j) { return i * (i + 1) / 2 + j; }
template <typename T>
__device__ __forceinline__ void spd9_solve(T (&A)[45], T (&x)[9]) {
  // the pivots' reciprocal square roots and multiplications instead of a square root and a division per column and a
  // division per entry: a float64 division or square root is a ~10-instruction dependent sequence, and the
  // substitutions below were a chain of 18 divisions (integration 6.1 -> 4.7, smooth 5.8 -> 4.4 us per arena-substep
  // for the reciprocal alone, profiles/r05i_phase_fp32.json)
  T inv[9];
#pragma unroll
  for (int j = 0; j < 9; j++) {
    T s = A[P9(j, j)];
#pragma unroll
    for (int k = 0; k < j; k++) s -= A[P9(j, k)] * A[P9(j, k)];
    inv[j] = rsqrt_f64(s > T(1e-300) ? s : T(1e-300));
#pragma unroll
    for (int i = j + 1; i < 9; i++) {
      T t = A[P9(i, j)];
#pragma unroll
      for (int k = 0; k < j; k++) t -= A[P9(i, k)] * A[P9(j, k)];
      A[P9(i, j)] = t * inv[j];
    }
  }
#pragma unroll
  for (int i = 0; i < 9; i++) {
    T t = x[i];
#pragma unroll
    for (int k = 0; k < i; k++) t -= A[P9(i, k)] * x[k];
    x[i] = t * inv[i];
  }
#pragma unroll
  for (int i = 8; i >= 0; i--) {
    T t = x[i];
#pragma unroll
    for (int k = i + 1; k < 9; k++) t -= A[P9(k, i)] * x[k];
    x[i] = t * inv[i];
  }
}

// ------------------------------------------------------------------------------------------------
// register-resident dense Cholesky + solve of H dir = -g for nv <= NVM (lane j holds column j of the
// symmetric matrix in NVM registers; pivots and multipliers are broadcast with v_readlane)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float readlane(float x, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}
__device__ __forceinline__ double readlane(double x, int l) {
  long long b = __double_as_longlong(x);
  int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
  int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ float lane_bcast(float x, int l) { return readlane(x, l); }
// fp64 broadcast: ds_bpermute (__shfl) by default; FM_F64_READLANE=1 uses the split 64-bit v_readlane.
// Both pass the fp64 parity tests since SYNC() became a real wave barrier + fences (round 2): the earlier
// "miscompile" of the readlane form was the compiler-only barrier letting LDS traffic move across it.
#ifndef FM_F64_READLANE
#define FM_F64_READLANE 0
#endif
__device__ __forceinline__ double lane_bcast(double x, int l) {
#if FM_F64_READLANE
  return readlane(x, l);
#else
  return __shfl(x, l);
#endif
}

template <typename T>
__device__ __forceinline__ T edge_val(const T* x3, T mu, int e);

// K_c = sum over the active pyramid edges e of D c_e c_e' (3x3 in contact-frame coordinates, edge directions
// c_e = (1, +-mu, 0) / (1, 0, +-mu)), one contact per lane, stored 00 11 22 01 02 12 in CR_K
template <typename T, typename DIM>
__device__ __forceinline__ void contact_K(const Ws<T, DIM>& w, int ncon) {
  for (int c = LANE; c < ncon; c += WAVE) {
    T* cr = w.cr() + CR_N * c;
    const T mu = cr[CR_MU], D = cr[CR_D], bd = cr[CR_BD], kd = cr[CR_KD];
    T Kc[6] = {0, 0, 0, 0, 0, 0};
    const double* ja = dslot(cr, CR_JA);
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const T aref = -bd * edge_val(cr + CR_VEL, mu, e) - kd;
      const double jar = edge_val(ja, (double)mu, e) - (double)aref;  // the active set of the float64 cost
      if (jar < 0.0) {
        const T sg = (e & 1) ? -mu : mu;
        Kc[0] += D;
        if (e < 2) {
          Kc[1] += D * sg * sg;
          Kc[3] += D * sg;
        } else {
          Kc[2] += D * sg * sg;
          Kc[4] += D * sg;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 6; k++) cr[CR_K + k] = Kc[k];
  }
}

__device__ __forceinline__ int rfl(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ float rfl(float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); }

// compile-time scene (fp32 and fp64): Cholesky factor and solve of the Newton Hessian (assembled in LDS) for
// dir = -H^-1 g, in registers (lane j owns column j; pivots and trailing operands broadcast by v_readlane).
//  * Elimination order: cubes, arms, belt last (position p = dof - 1, the belt at NV - 1).  The belt touches
//    every cube resting on it; eliminated last it is a border row instead of coupling all those cubes.
//  * Tree-block sparsity: H couples two trees only through a contact between them.  The coupling graph (plus
//    the fill-in of this elimination order) comes from the tree->contact masks; a pivot updates only the row
//    blocks of trees coupled to its own.  Skipped entries are exact zeros of the dense factorization.
//  * Arrowhead fast path (chol_arrow_rl): when no contact couples two trees other than the belt -- the common
//    substep -- H in this order is block diagonal with a belt border, and the tree blocks factor independently.
template <typename T, typename DIM, bool ASM>
__device__ __forceinline__ void chol_arrow_rl(const Model<T>& M, const Ws<T, DIM>& w, const T* H, const double* g,
                                              T* dir, int ncon, int nrow);

// scenes with the register Cholesky on one 64-contact tree-mask word ((2,4), fp32 and fp64)
template <typename T, typename DIM>
__device__ constexpr bool arrow_scene() {
  if constexpr (DIM::fixed)
    return DIM::MAXC == WAVE && DIM::nv <= 48;
  else
    return false;
}
// arrowhead test: no contact shared by two trees other than the belt (tree 0); uniform, a scalar branch
template <typename T, typename DIM>
__device__ __forceinline__ bool arrow_substep(const Model<T>& M, const Ws<T, DIM>& w) {
  if (FM_XF(M) & 16) return false;  // FM_NO_ARROW=1: the general factors
  uint64_t both = 0;
#pragma unroll
  for (int h = 0; h < DIM::MAXC / WAVE; h++) {  // tree-mask words (contacts 64 h .. 64 h + 63)
    uint64_t any = 0;
#pragma unroll
    for (int t = 1; t < DIM::ntree; t++) {
      const uint64_t m = w.tmask()[h * DIM::ntree + t];
      const uint64_t mt = ((uint64_t)(unsigned)rfl((int)(m >> 32)) << 32) | (unsigned)rfl((int)(m & 0xffffffffu));
      both |= any & mt;
      any |= mt;
    }
  }
  return both == 0;
}

template <typename T, typename DIM>
__device__ __forceinline__ void chol_sparse_rl(const Model<T>& M, const Ws<T, DIM>& w, const T* H, const double* g,
                                               T* dir) {
  constexpr int NV = DIM::nv, KK = DIM::K, AA = DIM::A, NT = DIM::ntree, A0 = 1 + 6 * DIM::K;
  if (arrow_substep(M, w)) {
    chol_arrow_rl<T, DIM, false>(M, w, H, g, dir, 0, 0);
    return;
  }
  const int j = LANE;
  const int jo = j == NV - 1 ? 0 : j + 1;  // lane j's dof (original numbering)
  T col[NV];
  // ---- H (assembled in LDS, row-major, original numbering) -> lane j holds column jo in elimination order
#pragma unroll
  for (int i = 0; i < NV; i++) {
    const int io = i == NV - 1 ? 0 : i + 1;
    col[i] = j < NV ? H[io * NV + jo] : T(0);
  }
  SYNC();
  // ---- tree coupling graph + fill-in of the elimination order (trees by rank: cubes, arms, belt)
  unsigned adj[NT];
  {
    uint64_t tm[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) {
      const uint64_t m = w.tmask()[t];
      tm[t] = ((uint64_t)(unsigned)rfl((int)(m >> 32)) << 32) | (unsigned)rfl((int)(m & 0xffffffffu));
    }
#pragma unroll
    for (int t = 0; t < NT; t++) {
      unsigned a = 0;
#pragma unroll
      for (int u = 0; u < NT; u++)
        if (u != t && (tm[t] & tm[u])) a |= 1u << u;
      adj[t] = a;
    }
    auto rank = [](int t) { return t == 0 ? NT - 1 : t - 1; };
#pragma unroll
    for (int r = 0; r < NT; r++) {
      const int t = r == NT - 1 ? 0 : r + 1;
      unsigned later = 0;
#pragma unroll
      for (int u = 0; u < NT; u++)
        if (rank(u) > r) later |= 1u << u;
      const unsigned nb = adj[t] & later;
#pragma unroll
      for (int u = 0; u < NT; u++)
        if (nb & (1u << u)) adj[u] |= nb & ~(1u << u);
    }
  }
  // ---- factor (right-looking, pivots and trailing operands broadcast by v_readlane), coupled blocks only
  const T tiny = sizeof(T) == 8 ? T(1e-300) : T(1e-37);
  T dinv = T(1);
  static_for<0, NV>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int tk = k == NV - 1 ? 0 : (k < A0 - 1 ? 1 + k / 6 : 1 + KK + (k - (A0 - 1)) / 9);
    T d = readlane(col[k], k);
    d = d > tiny ? d : tiny;
    const T ri = rsqrt_div(d);
    const T lj = col[k] * ri;
    if (j == k) dinv = ri;
    if (j >= k) col[k] = lj;
    const unsigned ak = adj[tk];
    static_for<0, NT>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      constexpr int ps = u == 0 ? NV - 1 : (u <= KK ? 6 * (u - 1) : A0 - 1 + 9 * (u - 1 - KK));
      constexpr int pn = u == 0 ? 1 : (u <= KK ? 6 : 9);
      if constexpr (ps + pn > k + 1) {                 // block not entirely at or above the pivot
        if (u == tk || (ak & (1u << u))) {             // coupled to the pivot's tree (uniform)
          // the block's operands are broadcast first (uniform control flow: every cross-lane operation runs on the
          // whole wave), then used by the lanes below the pivot: the v_readlane -> VALU hazard is paid once per
          // block instead of once per entry
          T lv[pn];
#pragma unroll
          for (int ii = 0; ii < pn; ii++) lv[ii] = ps + ii > k ? readlane(lj, ps + ii) : T(0);
          if (j > k) {
#pragma unroll
            for (int ii = 0; ii < pn; ii++) {
              const int i = ps + ii;
              if (i > k) col[i] -= lv[ii] * lj;
            }
          }
        }
      }
    });
  });
  T acc = j < NV ? (T)-g[jo] : T(0);
  T y = T(0);
#pragma unroll
  for (int k = 0; k < NV; k++) {
    const T yk = readlane(acc * dinv, k);
    if (j == k) y = yk;
    if (j > k) acc -= col[k] * yk;
  }
  T acc2 = y, x = T(0);
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) {
    const T xk = readlane(acc2 * dinv, k);
    if (j == k) x = xk;
    if (j < k) acc2 -= col[k] * dinv * xk;
  }
  if (j < NV) dir[jo] = x;
  SYNC();
}

// Arrowhead Cholesky (chol_sparse_rl's fast path).  No contact couples two trees other than the belt, so in the
// elimination order (cubes, arms, belt last) H is block diagonal -- one 6x6 block per cube, one 9x9 per arm --
// plus the belt's border row, and there is no fill-in outside the blocks and the border.  All blocks take their
// s-th pivot in the same step: 9 pivot steps instead of NV - 1, and 9 + 9 substitution steps instead of 2 NV.
//  * Lane j (position j, j < NV - 1) keeps its column's rows of its own block (local index, so every lane uses
//    the same registers) and its belt row `bel` (= H[belt][j] by symmetry); the pivot and the multipliers of its
//    block come from the block's lanes by ds_bpermute.
//  * The belt lane takes no part in the block steps: its column is the other lanes' `bel`; its diagonal and its
//    forward-substitution row are accumulated afterwards in pivot order by a v_readlane chain.
// Every entry sees the operations of chol_sparse_rl in the same order (the updates it skips are products with
// exact zeros), so the factor and the direction are bit-identical to it.
// ASM = true: H is not read from LDS but assembled straight into these registers (newton() skips the LDS
// assembly on arrowhead substeps): lane j sums its column's M entries, the contacts of its own tree (K_c from
// contact_K in CR_K: B_t' K_c B_t on its block rows, B_belt' K_c B_t on its belt row when the partner is the
// belt) and the generic rows of its dof; the belt lane sums its diagonal over the belt's contacts.  Same terms
// as the LDS assembly, summed per lane in contact order instead of by atomics (not bit-identical to it).
template <typename T, typename DIM, bool ASM>
__device__ __forceinline__ void chol_arrow_rl(const Model<T>& M, const Ws<T, DIM>& w, const T* H, const double* g,
                                              T* dir, int ncon, int nrow) {
  constexpr int NV = DIM::nv, A0 = 1 + 6 * DIM::K, NB = NV - 1;
  static_assert(NV <= WAVE, "one lane per position");
  const int j = LANE;
  const bool blk = j < NB;                   // a block lane (not the belt, not idle)
  const int jo = j == NV - 1 ? 0 : j + 1;    // lane j's dof (original numbering)
  const int ps = j < A0 - 1 ? (j / 6) * 6 : A0 - 1 + ((j - (A0 - 1)) / 9) * 9;  // own block's first position
  const int pn = j < A0 - 1 ? 6 : 9;         // own block's size
  const int jl = j - ps;                     // local index
  T loc[9], bel = T(0), hbb;
  if constexpr (!ASM) {
#pragma unroll
    for (int ii = 0; ii < 9; ii++) loc[ii] = (blk && ii < pn) ? H[(ps + ii + 1) * NV + jo] : T(0);
    bel = blk ? H[jo] : T(0);  // row 0 (the belt) of column jo
    hbb = H[0];
    SYNC();
  } else {
    // the belt lane assembles its diagonal as a block of one (tree 0, local index 0)
    const bool bl = j == NV - 1;
    const int t = bl ? 0 : (j < A0 - 1 ? 1 + j / 6 : 1 + DIM::K + (j - (A0 - 1)) / 9);
    const int an = bl ? 1 : pn, al = bl ? 0 : jl;
    if (blk && j >= A0 - 1) {
      const T* Ma = w.Marm() + 81 * ((j - (A0 - 1)) / 9) + jl;
#pragma unroll
      for (int ii = 0; ii < 9; ii++) loc[ii] = Ma[9 * ii];
    } else {
      const T md = (blk || bl) ? Mdiag(M, w, jo) : T(0);
#pragma unroll
      for (int ii = 0; ii < 9; ii++) loc[ii] = ii == al ? md : T(0);
    }
    // the belt's diagonal: one lane per contact (B_belt' K_c B_belt of the contacts on the belt), then a wave sum
    // -- the belt lane would otherwise walk every belt contact while a cube lane walks four
    {
      T hb = T(0);
      if (j < ncon) {
        const int* ci = w.ci() + 4 * j;
        const int ta = ci[1], tb = ci[2], nda = (ci[3] >> 20) & 15;
        if (ta == 0 || tb == 0) {
          const T* cr = w.cr() + CR_N * j;
          const T* Kc = cr + CR_K;
          const int cb = ta == 0 ? 0 : nda;
          const T b0 = cr[CR_J + cb], b1 = cr[CR_J + CJ + cb], b2 = cr[CR_J + 2 * CJ + cb];
          hb = b0 * (Kc[0] * b0 + Kc[3] * b1 + Kc[4] * b2) + b1 * (Kc[3] * b0 + Kc[1] * b1 + Kc[5] * b2) +
               b2 * (Kc[4] * b0 + Kc[5] * b1 + Kc[2] * b2);
        }
      }
      hb = wave_sum(hb);
      if (bl) loc[0] += hb;
    }
    if (blk) {
      uint64_t mk = w.tmask()[t];
      while (mk) {
        const int c = __ffsll((unsigned long long)mk) - 1;
        mk &= mk - 1;
        const int* ci = w.ci() + 4 * c;
        const T* cr = w.cr() + CR_N * c;
        const T* Kc = cr + CR_K;
        const int ta = ci[1], tb = ci[2], nda = (ci[3] >> 20) & 15;
        const bool first = ta == t;
        const int off = first ? 0 : nda;        // own tree's first column in the record
        const int ob = first ? nda : 0;         // the partner's first column
        const T* J = cr + CR_J;
        const T k0 = Kc[0], k1 = Kc[1], k2 = Kc[2], k3 = Kc[3], k4 = Kc[4], k5 = Kc[5];
        const T b0 = J[off + al], b1 = J[CJ + off + al], b2 = J[2 * CJ + off + al];
        const T q0 = k0 * b0 + k3 * b1 + k4 * b2;
        const T q1 = k3 * b0 + k1 * b1 + k5 * b2;
        const T q2 = k4 * b0 + k5 * b1 + k2 * b2;
        T jr0[9], jr1[9], jr2[9];
#pragma unroll
        for (int ii = 0; ii < 9; ii++) {
          jr0[ii] = J[off + ii];
          jr1[ii] = J[CJ + off + ii];
          jr2[ii] = J[2 * CJ + off + ii];
        }
#pragma unroll
        for (int ii = 0; ii < 9; ii++)
          if (ii < an) loc[ii] += q0 * jr0[ii] + q1 * jr1[ii] + q2 * jr2[ii];
        if ((first ? tb : ta) == 0) bel += q0 * J[ob] + q1 * J[CJ + ob] + q2 * J[2 * CJ + ob];
      }
      // generic rows (gripper equality, joint limits: both dofs in one arm) touching this dof
      for (int r = 0; r < nrow; r++) {
        const int* ri = w.ri() + 4 * r;
        const T* rr = w.rr() + RR_N * r;
        const int d0 = ri[0], d1 = ri[1];
        if (d0 != jo && d1 != jo) continue;
        if (!(ri[2] == 0 || *dslot(rr, RR_JAR) < 0.0)) continue;
        const T D = rr[RR_D], c0 = rr[RR_C0], c1 = rr[RR_C1];
        const T cj = d0 == jo ? c0 : c1;
#pragma unroll
        for (int ii = 0; ii < 9; ii++) {
          const int d = ps + ii + 1;
          if (d == d0) loc[ii] += D * c0 * cj;
          if (d1 >= 0 && d == d1) loc[ii] += D * c1 * cj;
        }
      }
    }
    hbb = readlane(loc[0], NV - 1);
    if (!blk) {
#pragma unroll
      for (int ii = 0; ii < 9; ii++) loc[ii] = T(0);
    }
    PMARK(PH_NHESS);
  }
  const T tiny = sizeof(T) == 8 ? T(1e-300) : T(1e-37);
  T dinv = T(1), lbelt = T(0);
  static_for<0, 9>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    const bool act = blk && s < pn;  // the block has a pivot in this step
    const int p = (ps + s) & (WAVE - 1);
    T d = __shfl(loc[s], p);
    d = d > tiny ? d : tiny;
    const T ri = rsqrt_div(d);
    const T lj = loc[s] * ri;           // L[j][k] (j >= k)
    const T lb = __shfl(bel, p) * ri;   // L[belt][k]
    if (act && jl == s) {
      dinv = ri;
      lbelt = lb;
    }
    if (act && jl >= s) loc[s] = lj;
    T lv[9];
#pragma unroll
    for (int ii = s + 1; ii < 9; ii++) lv[ii] = __shfl(lj, (ps + ii) & (WAVE - 1));  // L[i][k], i in the block
    if (act && jl > s) {
#pragma unroll
      for (int ii = s + 1; ii < 9; ii++)
        if (ii < pn) loc[ii] -= lv[ii] * lj;
      bel -= lb * lj;
    }
  });
  // belt pivot: its diagonal minus its row of L, in pivot order
  T db = hbb;
#pragma unroll
  for (int k = 0; k < NB; k++) {
    const T x = readlane(lbelt, k);
    db -= x * x;
  }
  db = db > tiny ? db : tiny;
  const T rib = rsqrt_div(db);
  // forward: L y = -g
  T acc = blk ? (T)-g[jo] : T(0);
  T y = T(0);
  static_for<0, 9>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    const bool act = blk && s < pn;
    const T yk = __shfl(acc * dinv, (ps + s) & (WAVE - 1));
    if (act && jl == s) y = yk;
    if (act && jl > s) acc -= loc[s] * yk;
  });
  T accb = (T)-g[0];
#pragma unroll
  for (int k = 0; k < NB; k++) accb -= readlane(lbelt, k) * readlane(y, k);
  const T yb = accb * rib;
  // backward: L' x = y, the belt first
  const T xb = yb * rib;
  T acc2 = y;
  if (blk) acc2 -= bel * dinv * xb;
  T x = T(0);
  static_for<0, 9>([&](auto sc) {
    constexpr int s = 8 - decltype(sc)::value;
    const bool act = blk && s < pn;
    const T xk = __shfl(acc2 * dinv, (ps + s) & (WAVE - 1));
    if (act && jl == s) x = xk;
    if (act && jl < s) acc2 -= loc[s] * dinv * xk;
  });
  if (blk) dir[jo] = x;
  if (j == NV - 1) dir[0] = xb;
  SYNC();
}

// Arrowhead Cholesky of the bordered scenes ((2,8), (2,10): 64 < nv <= 80, LDS-assembled Hessian): the block
// positions do not fit one lane each, so chol_arrow_rl's block steps run in two passes of whole blocks -- positions
// [0, SPLIT) on lanes 0.., [SPLIT, nv - 1) on lanes 0.. again (SPLIT = the last block boundary <= 64) -- with one
// register set per pass; the belt's diagonal and forward row are v_readlane chains over both passes in pivot
// order.  Used when no contact couples two trees other than the belt, instead of the bordered register factor.
template <typename T, typename DIM>
__device__ constexpr int arrow_split() {
  constexpr int A0 = 1 + 6 * DIM::K;
  int sp = 0;
  for (int c = 0; c <= DIM::K; c++)
    if (6 * c <= WAVE) sp = 6 * c;
  for (int a = 0; a <= DIM::A; a++)
    if (A0 - 1 + 9 * a <= WAVE) sp = A0 - 1 + 9 * a;
  return sp;
}
template <typename T, typename DIM>
__device__ __forceinline__ void chol_arrow2_rl(const T* H, const double* g, T* dir) {
  constexpr int NV = DIM::nv, A0 = 1 + 6 * DIM::K, NB = NV - 1, SPLIT = arrow_split<T, DIM>();
  static_assert(SPLIT <= WAVE && NB - SPLIT <= WAVE && NB > WAVE, "two passes of whole blocks");
  const int j = LANE;
  bool blk[2];
  int ps[2], pn[2], jl[2], jo[2];
  T loc[2][9], bel[2], dinv[2], lbelt[2];
#pragma unroll
  for (int P = 0; P < 2; P++) {
    const int base = P ? SPLIT : 0, end = P ? NB : SPLIT;
    const int p = base + j;
    blk[P] = p < end;
    const int pa = p < A0 - 1 ? (p / 6) * 6 : A0 - 1 + ((p - (A0 - 1)) / 9) * 9;  // block start (position)
    pn[P] = p < A0 - 1 ? 6 : 9;
    jl[P] = p - pa;
    ps[P] = pa - base;  // block start (lane)
    jo[P] = p + 1;
#pragma unroll
    for (int ii = 0; ii < 9; ii++) loc[P][ii] = (blk[P] && ii < pn[P]) ? H[(pa + ii + 1) * NV + jo[P]] : T(0);
    bel[P] = blk[P] ? H[jo[P]] : T(0);
    dinv[P] = T(1);
    lbelt[P] = T(0);
  }
  const T hbb = H[0];
  SYNC();
  const T tiny = sizeof(T) == 8 ? T(1e-300) : T(1e-37);
#pragma unroll
  for (int P = 0; P < 2; P++) {
    static_for<0, 9>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      const bool act = blk[P] && s < pn[P];
      const int p = (ps[P] + s) & (WAVE - 1);
      T d = __shfl(loc[P][s], p);
      d = d > tiny ? d : tiny;
      const T ri = rsqrt_div(d);
      const T lj = loc[P][s] * ri;
      const T lb = __shfl(bel[P], p) * ri;
      if (act && jl[P] == s) {
        dinv[P] = ri;
        lbelt[P] = lb;
      }
      if (act && jl[P] >= s) loc[P][s] = lj;
      T lv[9];
#pragma unroll
      for (int ii = s + 1; ii < 9; ii++) lv[ii] = __shfl(lj, (ps[P] + ii) & (WAVE - 1));
      if (act && jl[P] > s) {
#pragma unroll
        for (int ii = s + 1; ii < 9; ii++)
          if (ii < pn[P]) loc[P][ii] -= lv[ii] * lj;
        bel[P] -= lb * lj;
      }
    });
  }
  T db = hbb;
#pragma unroll
  for (int k = 0; k < SPLIT; k++) {
    const T x = readlane(lbelt[0], k);
    db -= x * x;
  }
#pragma unroll
  for (int k = 0; k < NB - SPLIT; k++) {
    const T x = readlane(lbelt[1], k);
    db -= x * x;
  }
  db = db > tiny ? db : tiny;
  const T rib = rsqrt_div(db);
  T y[2];
  T accb = (T)-g[0];
#pragma unroll
  for (int P = 0; P < 2; P++) {
    T acc = blk[P] ? (T)-g[jo[P]] : T(0);
    y[P] = T(0);
    static_for<0, 9>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      const bool act = blk[P] && s < pn[P];
      const T yk = __shfl(acc * dinv[P], (ps[P] + s) & (WAVE - 1));
      if (act && jl[P] == s) y[P] = yk;
      if (act && jl[P] > s) acc -= loc[P][s] * yk;
    });
  }
#pragma unroll
  for (int k = 0; k < SPLIT; k++) accb -= readlane(lbelt[0], k) * readlane(y[0], k);
#pragma unroll
  for (int k = 0; k < NB - SPLIT; k++) accb -= readlane(lbelt[1], k) * readlane(y[1], k);
  const T xb = (accb * rib) * rib;
#pragma unroll
  for (int P = 0; P < 2; P++) {
    T acc2 = y[P];
    if (blk[P]) acc2 -= bel[P] * dinv[P] * xb;
    T x = T(0);
    static_for<0, 9>([&](auto sc) {
      constexpr int s = 8 - decltype(sc)::value;
      const bool act = blk[P] && s < pn[P];
      const T xk = __shfl(acc2 * dinv[P], (ps[P] + s) & (WAVE - 1));
      if (act && jl[P] == s) x = xk;
      if (act && jl[P] < s) acc2 -= loc[P][s] * dinv[P] * xk;
    });
    if (blk[P]) dir[jo[P]] = x;
  }
  if (j == 0) dir[0] = xb;
  SYNC();
}

// fp32, compile-time scene with 64 < nv <= 80 ((2,8), (2,10)): the same register Cholesky for the 64 leading
// positions (lane j owns position j; cubes, then arms) with the remaining nv - 64 positions (the last arm dofs and
// the belt) as a border:
//  * the head pivots update the border rows of their own columns as usual (L[64+i][k] is lane k's entry, read
//    with v_readlane from the pivot lane instead of from a row lane that does not exist);
//  * the border's Schur complement S = H_BB - L_B L_B' (L_B = the border rows of L, 16 x 64 padded) is one
//    16x16x64 product on the matrix cores: 16 chained v_mfma_f32_16x16x4_f32 whose A and B operands are the same
//    LDS element per lane (A[i][k] = B[k][i] = L_B[i][k]);
//  * S is factored densely on the first nv - 64 lanes; the solves run head forward, border forward (the border
//    rows' sums over the head read from LDS), border backward, head backward.
template <typename T, typename DIM>
__device__ constexpr bool border_chol() {
  if constexpr (sizeof(T) == 4 && DIM::fixed)
    return DIM::nv > WAVE && DIM::nv <= WAVE + 16;
  else
    return false;
}
typedef float fm_f32x4 __attribute__((ext_vector_type(4)));
template <typename DIM>
__device__ __forceinline__ void chol_sparse_border(const Model<float>& M, const Ws<float, DIM>& w, float* H,
                                                   const double* g, float* dir) {
  constexpr int NV = DIM::nv, KK = DIM::K, NT = DIM::ntree, A0 = 1 + 6 * DIM::K;
  constexpr int NH = WAVE, NB = NV - WAVE, NW = (DIM::MAXC + 63) / 64;
  static_assert(NB > 0 && NB <= 16, "border of at most 16 positions");
  const int j = LANE;
  const int jo = j + 1;  // head positions are never the belt (position NV - 1)
  auto dof_of = [](int p) { return p == NV - 1 ? 0 : p + 1; };
  float col[NV];
#pragma unroll
  for (int i = 0; i < NV; i++) col[i] = H[dof_of(i) * NV + jo];
  float cs[NB];  // lanes j < NB: border column NH + j, rows NH .. NV - 1
#pragma unroll
  for (int i = 0; i < NB; i++) cs[i] = j < NB ? H[dof_of(NH + i) * NV + dof_of(NH + (j < NB ? j : 0))] : 0.0f;
  // ---- tree coupling graph + fill-in (as chol_sparse_rl, tree masks of NW words)
  unsigned adj[NT];
  {
    uint64_t tm[NW][NT];
#pragma unroll
    for (int h = 0; h < NW; h++)
#pragma unroll
      for (int t = 0; t < NT; t++) {
        const uint64_t m = w.tmask()[h * NT + t];
        tm[h][t] = ((uint64_t)(unsigned)rfl((int)(m >> 32)) << 32) | (unsigned)rfl((int)(m & 0xffffffffu));
      }
#pragma unroll
    for (int t = 0; t < NT; t++) {
      unsigned a = 0;
#pragma unroll
      for (int u = 0; u < NT; u++) {
        uint64_t o = 0;
#pragma unroll
        for (int h = 0; h < NW; h++) o |= tm[h][t] & tm[h][u];
        if (u != t && o) a |= 1u << u;
      }
      adj[t] = a;
    }
    auto rank = [](int t) { return t == 0 ? NT - 1 : t - 1; };
#pragma unroll
    for (int r = 0; r < NT; r++) {
      const int t = r == NT - 1 ? 0 : r + 1;
      unsigned later = 0;
#pragma unroll
      for (int u = 0; u < NT; u++)
        if (rank(u) > r) later |= 1u << u;
      const unsigned nb = adj[t] & later;
#pragma unroll
      for (int u = 0; u < NT; u++)
        if (nb & (1u << u)) adj[u] |= nb & ~(1u << u);
    }
  }
  SYNC();  // every lane has its columns: H is scratch from here on
  // ---- head factor (coupled blocks only; border rows read from the pivot lane)
  const float tiny = 1e-37f;
  float dinv = 1.0f;
  static_for<0, NH>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int tk = k < A0 - 1 ? 1 + k / 6 : 1 + KK + (k - (A0 - 1)) / 9;
    float d = readlane(col[k], k);
    d = d > tiny ? d : tiny;
    const float ri = 1.0f / sqrtf(d);
    const float lj = col[k] * ri;
    if (j == k) dinv = ri;
    if (j >= k) col[k] = lj;
    const unsigned ak = adj[tk];
    if (j > k) {
      static_for<0, NT>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        constexpr int ps = u == 0 ? NV - 1 : (u <= KK ? 6 * (u - 1) : A0 - 1 + 9 * (u - 1 - KK));
        constexpr int pn = u == 0 ? 1 : (u <= KK ? 6 : 9);
        if constexpr (ps + pn > k + 1) {
          if (u == tk || (ak & (1u << u))) {
            float lv[pn];
#pragma unroll
            for (int ii = 0; ii < pn; ii++) {
              const int i = ps + ii;
              lv[ii] = i <= k ? 0.0f : (i < NH ? readlane(lj, i < NH ? i : 0) : readlane(col[i], k) * ri);
            }
#pragma unroll
            for (int ii = 0; ii < pn; ii++) {
              const int i = ps + ii;
              if (i > k) col[i] -= lv[ii] * lj;
            }
          }
        }
      });
    }
  });
  // ---- border Schur complement on the matrix cores: S -= L_B L_B'
  float* LB = H;              // [64 lanes][16]: L[NH + i][lane]
  float* SC = H + 16 * WAVE;  // [16][16]
#pragma unroll
  for (int i = 0; i < 16; i++) LB[16 * j + i] = i < NB ? col[NH + (i < NB ? i : 0)] * dinv : 0.0f;
  SYNC();
  fm_f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 16; s += 2) {  // two accumulators: the 40-cycle dependent latency overlaps
    const float a0 = LB[16 * (4 * s + (j >> 4)) + (j & 15)];
    const float a1 = LB[16 * (4 * (s + 1) + (j >> 4)) + (j & 15)];
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, a0, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, a1, acc1, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; r++) SC[16 * (4 * (j >> 4) + r) + (j & 15)] = acc0[r] + acc1[r];
  SYNC();
  if (j < NB) {
#pragma unroll
    for (int i = 0; i < NB; i++) cs[i] -= SC[16 * i + j];
  }
  // ---- dense factor of S on lanes j < NB
  float dinvb = 1.0f;
#pragma unroll
  for (int k = 0; k < NB; k++) {
    float d = readlane(cs[k], k);
    d = d > tiny ? d : tiny;
    const float ri = 1.0f / sqrtf(d);
    const float lj = cs[k] * ri;
    if (j == k) dinvb = ri;
    if (j >= k) cs[k] = lj;
    if (j > k && j < NB) {
      float lv[NB];
#pragma unroll
      for (int i = 0; i < NB; i++) lv[i] = i > k ? readlane(lj, i) : 0.0f;
#pragma unroll
      for (int i = 0; i < NB; i++)
        if (i > k) cs[i] -= lv[i] * lj;
    }
  }
  // ---- forward: head, then the border rows (their sums over the head columns from LDS)
  float acc = (float)-g[jo];
  float y = 0.0f;
#pragma unroll
  for (int k = 0; k < NH; k++) {
    const float yk = readlane(acc * dinv, k);
    if (j == k) y = yk;
    if (j > k) acc -= col[k] * yk;
  }
  float* ys = SC;  // SC was consumed into cs before the border factor
  SYNC();
  ys[j] = y;
  SYNC();
  float accb = 0.0f;
  if (j < NB) {
    float sum = 0.0f;
#pragma unroll 16
    for (int k = 0; k < NH; k++) sum += LB[16 * k + j] * ys[k];
    accb = (float)-g[dof_of(NH + j)] - sum;
  }
  float yb = 0.0f;
#pragma unroll
  for (int k = 0; k < NB; k++) {
    const float yk = readlane(accb * dinvb, k);
    if (j == k) yb = yk;
    if (j > k && j < NB) accb -= cs[k] * yk;
  }
  // ---- backward: border, then the head (border columns folded in first)
  float acc2b = yb, xb = 0.0f;
#pragma unroll
  for (int k = NB - 1; k >= 0; k--) {
    const float xk = readlane(acc2b * dinvb, k);
    if (j == k) xb = xk;
    if (j < k) acc2b -= cs[k] * dinvb * xk;
  }
  float acc2 = y;
#pragma unroll
  for (int i = 0; i < NB; i++) acc2 -= col[NH + i] * dinv * readlane(xb, i);
  float x = 0.0f;
#pragma unroll
  for (int k = NH - 1; k >= 0; k--) {
    const float xk = readlane(acc2 * dinv, k);
    if (j == k) x = xk;
    if (j < k) acc2 -= col[k] * dinv * xk;
  }
  SYNC();
  dir[jo] = x;
  if (j < NB) dir[dof_of(NH + j)] = xb;
  SYNC();
}

// Sparse LDS Cholesky + solve for the scenes without a register path (runtime-dims scenes such as (4,16); fp64
// above nv = 64): chol_sparse_rl's elimination order (cubes, arms, belt last) and tree-block sparsity with the
// trailing matrix in LDS (lower triangle in elimination order, entry (i, c) at H[dof(i) * nv + dof(c)]).  Per
// pivot the rows it touches -- later positions of its own tree and of the trees coupled to it, fill-in included --
// are compacted by ballot; the column is scaled one row per lane, then one lane per column of that row set updates
// its column.  The substitutions walk the same row sets.  Returns false (nothing written) when the scene has more
// trees than a 32-bit coupling mask holds.
template <typename T, typename DIM>
__device__ __forceinline__ bool chol_sparse_lds(const Model<T>& M, const Ws<T, DIM>& w, T* H, const double* g, T* dir) {
  const DIM dm(M.dm);
  const int NV = dm.nv, K = dm.K, NT = dm.ntree, A0 = 1 + 6 * K;
  const int HS = hstride(sizeof(T), NV);  // the Hessian's row stride
  if (NT > 32) return false;
  const int NW = (dm.maxcon + 63) / 64;
  T* dinv = (T*)w.tmp();      // quad()'s scratch, dead until the line search
  int* list = (int*)w.fa();   // actuator forces, consumed by smooth_acc
  auto dof = [=](int p) { return p == NV - 1 ? 0 : p + 1; };
  auto tree_of = [=](int p) { return p == NV - 1 ? 0 : (p < A0 - 1 ? 1 + p / 6 : 1 + K + (p - (A0 - 1)) / 9); };
  // tree coupling graph (lane t: trees coupled to tree t), then the fill-in of the elimination order
  unsigned adj = 0;
  if (LANE < NT) {
    for (int u = 0; u < NT; u++) {
      uint64_t o = 0;
      for (int h = 0; h < NW; h++) o |= w.tmask()[h * NT + LANE] & w.tmask()[h * NT + u];
      if (u != LANE && o) adj |= 1u << u;
    }
  }
  const unsigned all = NT < 32 ? (1u << NT) - 1u : ~0u;
  for (int r = 0; r < NT; r++) {
    const int t = r == NT - 1 ? 0 : r + 1;                                    // tree of rank r
    unsigned later = (r + 2 < 32 ? (~0u << (r + 2)) : 0u) & all;            // trees u >= 1 of rank u - 1 > r
    if (r < NT - 1) later |= 1u;                                             // the belt ranks last
    const unsigned nb = (unsigned)__builtin_amdgcn_readlane((int)adj, t) & later;
    if (LANE < NT && ((nb >> LANE) & 1u)) adj |= nb & ~(1u << LANE);
  }
  const T tiny = sizeof(T) == 8 ? T(1e-300) : T(1e-37);
  for (int k = 0; k < NV; k++) {
    const int tk = tree_of(k), dk = dof(k);
    const unsigned ak = (unsigned)__builtin_amdgcn_readlane((int)adj, tk) | (1u << tk);
    T d = H[dk * HS + dk];
    d = d > tiny ? d : tiny;
    const T ri = rsqrt_div(d);
    int m = 0;
    for (int p0 = k + 1; p0 < NV; p0 += WAVE) {
      const int p = p0 + LANE;
      const bool in = p < NV && ((ak >> tree_of(p)) & 1u);
      const uint64_t bal = __ballot(in);
      const int below = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
      if (in) list[m + below] = p;
      m += __popcll(bal);
    }
    if (LANE == 0) dinv[k] = ri;
    SYNC();
    for (int e = LANE; e < m; e += WAVE) H[dof(list[e]) * HS + dk] *= ri;  // L[i][k]
    SYNC();
    // trailing update of the row set's lower triangle, one (row, column) pair per lane: the m (m + 1) / 2 pairs
    // are spread over the wave (a pair's entry is written by that lane only; column dk is read-only here)
    const int npair = m * (m + 1) / 2;
    for (int e = LANE; e < npair; e += WAVE) {
      int a = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);  // e -> (a >= b), packed lower triangle
      if ((a + 1) * (a + 2) / 2 <= e) a++;
      if (a * (a + 1) / 2 > e) a--;
      const int b = e - a * (a + 1) / 2;
      const int di = dof(list[a]), dc = dof(list[b]);
      H[di * HS + dc] -= H[di * HS + dk] * H[dc * HS + dk];
    }
    SYNC();
  }
  // substitutions: the forward pass reads dir as the running right-hand side and writes y to yv (the row list's
  // array, free now), the backward pass runs on yv and writes x to dir -- one wave barrier per pivot
  T* yv = (T*)w.fa();
  for (int p = LANE; p < NV; p += WAVE) dir[dof(p)] = (T)-g[dof(p)];
  SYNC();
  for (int k = 0; k < NV; k++) {  // L y = -g, column by column over the pivot's row set
    const int tk = tree_of(k), dk = dof(k);
    const unsigned ak = (unsigned)__builtin_amdgcn_readlane((int)adj, tk) | (1u << tk);
    const T yk = dir[dk] * dinv[k];
    if (LANE == 0) yv[dk] = yk;
    for (int p = k + 1 + LANE; p < NV; p += WAVE)
      if ((ak >> tree_of(p)) & 1u) dir[dof(p)] -= H[dof(p) * HS + dk] * yk;
    SYNC();
  }
  for (int k = NV - 1; k >= 0; k--) {  // L' x = y
    const int tk = tree_of(k), dk = dof(k);
    const unsigned ak = (unsigned)__builtin_amdgcn_readlane((int)adj, tk) | (1u << tk);
    const T xk = yv[dk] * dinv[k];
    if (LANE == 0) dir[dk] = xk;
    for (int p = LANE; p < k; p += WAVE)
      if ((ak >> tree_of(p)) & 1u) yv[dof(p)] -= H[dk * HS + dof(p)] * xk;
    SYNC();
  }
  return true;
}

// fp32 scenes above 80 dofs ((4,16): 133; compile-time or runtime dims): dense right-looking Cholesky over
// 16-wide column blocks of H (LDS, row stride hs = nv rounded up to 16, padding an identity block; only the lower
// triangle is read), everything but the 16-step pivot chains on the matrix cores.  Per block b (columns c0..c0+15):
//  * the diagonal block is factored in registers (lane j < 16 owns row j; pivots broadcast by v_readlane) and
//    inverted (lane j forms column j of L_bb^-1 by substitution; the entries of L_bb arrive by v_readlane);
//  * the panel below it, P = H_panel L_bb^-T, one 16 x 16 tile = 4 chained v_mfma_f32_16x16x4_f32
//    (A = H_panel, B = (L_bb^-1)^T);
//  * the trailing lower triangle H -= P P' tile by tile, 4 MFMAs per tile (A[i][k] = P[16I + i][k],
//    B[k][j] = P[16J + j][k]); diagonal tiles are written whole (their upper halves are never read).
// The substitutions run blockwise: the 16-step chain on lanes 0..15, then one row per lane over the rest with the
// block's solution broadcast by v_readlane.  Row / column operands are read unconditionally (the padding makes
// every block whole), so the loads of a tile issue together.
template <typename T, typename DIM>
__device__ constexpr bool dense_mfma_chol() {
  if constexpr (sizeof(T) == 4 && DIM::fixed)
    return DIM::nv > WAVE + 16;  // compile-time scenes above the bordered register factor ((4,16))
  else
    return sizeof(T) == 4 && !DIM::fixed;
}
template <typename DIM>
__device__ __forceinline__ void chol_dense_mfma(const Model<float>& M, const Ws<float, DIM>& w, float* H, const int nv,
                                                const double* g, float* dir) {
  const int hs = hstride(4, nv);
  const int nb = hs >> 4;
  const int j = LANE, j16 = j & 15, q4 = j >> 4;
  float* dinv = (float*)w.tmp();  // [hs] 1 / L_kk (quad()'s scratch, dead until the line search)
  float* IL = H + hs * hs;        // [16][16] L_bb^-1 of the current block (hextra)
  uint64_t* nzs = (uint64_t*)w.bc();  // [nb] nonzero panel tiles of each block (bc: unused above 64 dofs)
  const float tiny = 1e-37f;
  for (int b = 0; b < nb; b++) {
    const int c0 = 16 * b;
    // ---- diagonal block: lane j16 holds row c0 + j16 (lower entries read at (max, min))
    float col[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const int hi = i > j16 ? i : j16, lo = i > j16 ? j16 : i;
      col[i] = H[(c0 + hi) * hs + c0 + lo];
    }
    float di = 1.0f;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      float d = readlane(col[k], k);
      d = d > tiny ? d : tiny;
      const float ri = 1.0f / sqrtf(d);
      const float lj = col[k] * ri;  // lane j16 > k: L[j16][k]; lane k: L[k][k]
      if (j16 == k) di = ri;
      if (j16 >= k) col[k] = lj;
      float lv[16];
#pragma unroll
      for (int i = 0; i < 16; i++) lv[i] = i > k ? readlane(lj, i) : 0.0f;
      if (j16 > k) {
#pragma unroll
        for (int i = 0; i < 16; i++)
          if (i > k) col[i] -= lv[i] * lj;
      }
    }
    // ---- L_bb^-1, column j16 on lane j16: z_i = (delta_ij - sum_{m<i} L[i][m] z_m) / L_ii
    float z[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      float sacc = i == j16 ? 1.0f : 0.0f;
#pragma unroll
      for (int m = 0; m < i; m++) sacc -= readlane(col[m], i) * z[m];
      z[i] = sacc * readlane(di, i);
    }
    SYNC();  // every lane has read its block
    if (j < 16) {
#pragma unroll
      for (int k = 0; k < 16; k++)
        if (k <= j) H[(c0 + j) * hs + c0 + k] = col[k];
#pragma unroll
      for (int i = 0; i < 16; i++) IL[16 * i + j] = z[i];
      dinv[c0 + j] = di;
    }
    SYNC();
    PMARK(PH_CHDIAG);
    // ---- panel: P = H_panel L_bb^-T, tile rows below the block.  H is block-sparse (trees couple only through
    // contacts; most cubes of a (4,16) arena rest alone): a tile whose H_panel is all zero has P = 0 and
    // contributes nothing below, so it is skipped here and in the trailing update (bit t of nz: tile row t)
    uint64_t nz = 0;
    {
      float bo[4];
#pragma unroll
      for (int s = 0; s < 4; s++) bo[s] = IL[16 * j16 + 4 * s + q4];  // B[k][jj] = L^-1[jj][k]
      for (int rI = c0 + 16; rI < hs; rI += 16) {
        float a[4];
#pragma unroll
        for (int s = 0; s < 4; s++) a[s] = H[(rI + j16) * hs + c0 + 4 * s + q4];
        if (__ballot(a[0] != 0.0f || a[1] != 0.0f || a[2] != 0.0f || a[3] != 0.0f) == 0ull) continue;
        nz |= 1ull << (rI >> 4);
        fm_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; s++) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], bo[s], acc, 0, 0, 0);
        SYNC();  // the tile's reads before its writes (other lanes read the same rows)
#pragma unroll
        for (int r = 0; r < 4; r++) H[(rI + 4 * q4 + r) * hs + c0 + j16] = acc[r];
      }
    }
    if (LANE == 0) nzs[b] = nz;
    SYNC();
    PMARK(PH_CHPANEL);
    // ---- trailing update of the lower-triangle tiles (I >= J) whose panel tiles are both nonzero, two tiles
    // per pass (pairs walked over the set bits of nz: I ascending, J <= I)
    if (nz) {
      int I = __builtin_ctzll(nz), J = I;
      bool more = true;
      auto advance = [&]() {
        const uint64_t after = J < 63 ? nz & (~0ull << (J + 1)) : 0ull;
        if (after && __builtin_ctzll(after) <= I) {
          J = __builtin_ctzll(after);
        } else {
          const uint64_t nextI = I < 63 ? nz & (~0ull << (I + 1)) : 0ull;
          if (!nextI) {
            more = false;
          } else {
            I = __builtin_ctzll(nextI);
            J = __builtin_ctzll(nz);
          }
        }
      };
      while (more) {
        const int I1 = I, J1 = J;
        advance();
        const bool two = more;
        const int I2 = two ? I : I1, J2 = two ? J : J1;
        if (two) advance();
        const int rI1 = 16 * I1, rJ1 = 16 * J1, rI2 = 16 * I2, rJ2 = 16 * J2;
        float a1[4], b1[4], a2[4], b2[4];
#pragma unroll
        for (int s = 0; s < 4; s++) {
          const int c = c0 + 4 * s + q4;
          a1[s] = H[(rI1 + j16) * hs + c];
          b1[s] = H[(rJ1 + j16) * hs + c];
          a2[s] = H[(rI2 + j16) * hs + c];
          b2[s] = H[(rJ2 + j16) * hs + c];
        }
        float c1[4], c2[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
          c1[r] = H[(rI1 + 4 * q4 + r) * hs + rJ1 + j16];
          c2[r] = H[(rI2 + 4 * q4 + r) * hs + rJ2 + j16];
        }
        fm_f32x4 acc1 = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; s++) {
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[s], b1[s], acc1, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[s], b2[s], acc2, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; r++) H[(rI1 + 4 * q4 + r) * hs + rJ1 + j16] = c1[r] - acc1[r];
        if (two) {
#pragma unroll
          for (int r = 0; r < 4; r++) H[(rI2 + 4 * q4 + r) * hs + rJ2 + j16] = c2[r] - acc2[r];
        }
      }
    }
    SYNC();
    PMARK(PH_CHTRAIL);
  }
  // ---- forward substitution L y = -g (y in dir; padded rows stay 0 and are never stored)
  for (int r = j; r < nv; r += WAVE) dir[r] = (float)-g[r];
  SYNC();
  for (int b = 0; b < nb; b++) {
    const int c0 = 16 * b;
    float lrow[16];
#pragma unroll
    for (int k = 0; k < 16; k++) lrow[k] = H[(c0 + j16) * hs + c0 + k];
    const bool own = j < 16 && c0 + j < nv;
    float acc = own ? dir[c0 + j] : 0.0f;
    const float dj = dinv[c0 + j16];
    float y = 0.0f;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const float yk = readlane(acc * dj, k);
      if (j16 == k) y = yk;
      if (j16 > k) acc -= lrow[k] * yk;
    }
    float yb[16];
#pragma unroll
    for (int k = 0; k < 16; k++) yb[k] = readlane(y, k);
    SYNC();
    if (own) dir[c0 + j] = y;
    const uint64_t nzb = nzs[b];
    for (int r = c0 + 16 + j; r < nv; r += WAVE) {
      if (!((nzb >> (r >> 4)) & 1ull)) continue;  // a zero panel tile: nothing to subtract
      float lr[16];
#pragma unroll
      for (int k = 0; k < 16; k++) lr[k] = H[r * hs + c0 + k];
      float s = 0.0f;
#pragma unroll
      for (int k = 0; k < 16; k++) s += lr[k] * yb[k];
      dir[r] -= s;
    }
    SYNC();
  }
  // ---- backward substitution L' x = y, last block first
  for (int b = nb - 1; b >= 0; b--) {
    const int c0 = 16 * b;
    float lcol[16];
#pragma unroll
    for (int k = 0; k < 16; k++) lcol[k] = H[(c0 + (k > j16 ? k : j16)) * hs + c0 + (k > j16 ? j16 : k)];
    const bool own = j < 16 && c0 + j < nv;
    float acc = own ? dir[c0 + j] : 0.0f;
    const float dj = dinv[c0 + j16];
    float x = 0.0f;
#pragma unroll
    for (int k = 15; k >= 0; k--) {
      const float xk = readlane(acc * dj, k);
      if (j16 == k) x = xk;
      if (j16 < k) acc -= lcol[k] * xk;
    }
    float xb[16];
#pragma unroll
    for (int k = 0; k < 16; k++) xb[k] = readlane(x, k);
    SYNC();
    if (own) dir[c0 + j] = x;
    for (int r = j; r < c0; r += WAVE) {
      if (!((nzs[r >> 4] >> b) & 1ull)) continue;  // L[c0 .. c0 + 15][r] lies in a zero panel tile of block r / 16
      float lc[16];
#pragma unroll
      for (int k = 0; k < 16; k++) lc[k] = H[(c0 + k) * hs + r];
      float s = 0.0f;
#pragma unroll
      for (int k = 0; k < 16; k++) s += lc[k] * xb[k];
      dir[r] -= s;
    }
    SYNC();
  }
  PMARK(PH_CHSOLVE);
}

template <typename T, int NVM>
__device__ __forceinline__ void chol_solve_reg(const T* H, T* bc, int nv, const double* g, T* dir) {
  const int j = LANE;
  const T tiny = sizeof(T) == 8 ? T(1e-300) : T(1e-37);
  T col[NVM];
#pragma unroll
  for (int i = 0; i < NVM; i++) col[i] = (i < nv && j < nv) ? H[i * nv + j] : T(0);
  SYNC();
  T dinv = T(1);
  // factor: after step k lane j (> k) holds L[j][k] in col[k]; lane k holds L[k][k]; lane j's entries
  // col[i], i > j, keep L[i][j] * L[j][j].  Rows >= nv are zero, so updates need no row guard.
#pragma unroll
  for (int k = 0; k < NVM; k++) {
    if (k < nv) {
      bc[j] = col[k];  // row k of the trailing matrix (= column k by symmetry)
      SYNC();
      T d = bc[k];
      d = d > tiny ? d : tiny;
      const T ri = rsqrt_div(d);
      const T lj = col[k] * ri;
      if (j == k) dinv = ri;
      if (j >= k) col[k] = lj;
      if (j > k) {
        const T s = lj * ri;
#pragma unroll
        for (int i = k + 1; i < NVM; i++) col[i] -= bc[i] * s;
      }
      SYNC();
    }
  }
  // forward: L y = -g ; y_k is formed on lane k and broadcast (v_readlane for fp32; ds_bpermute for
  // fp64, whose split 64-bit v_readlane miscompiles in the fully unrolled fixed-size kernel)
  T acc = j < nv ? (T)-g[j] : T(0);
  T y = T(0);
#pragma unroll
  for (int k = 0; k < NVM; k++) {
    if (k < nv) {
      const T yk = lane_bcast(acc * dinv, k);
      if (j == k) y = yk;
      if (j > k) acc -= col[k] * yk;
    }
  }
  // backward: L' x = y
  T acc2 = y, x = T(0);
#pragma unroll
  for (int k = NVM - 1; k >= 0; k--) {
    if (k < nv) {
      const T xk = lane_bcast(acc2 * dinv, k);
      if (j == k) x = xk;
      if (j < k) acc2 -= col[k] * dinv * xk;
    }
  }
  if (j < nv) dir[j] = x;
  SYNC();
}

// chol_solve_reg for the tree-block solve's small coupled system (fp32, n <= NVM): the same factor, but the pivot
// column reaches the other lanes by v_readlane (lane i holds L[i][k] after the scaling) instead of an LDS row and two
// wave barriers per pivot -- the system is one small dense block solved once per Newton iteration
// (T = double: the fp64 tree-block solve; the pivot broadcasts go through lane_bcast, ds_bpermute for 64-bit values
// -- see the 64-bit cross-lane hazard)
template <int NVM, typename T = float>
__device__ __forceinline__ void chol_solve_rl(const T* H, int nv, const double* g, T* dir) {
  const int j = LANE;
  const T tiny = sizeof(T) == 4 ? T(1e-37f) : T(1e-300);
  T col[NVM];
#pragma unroll
  for (int i = 0; i < NVM; i++) col[i] = (i < nv && j < nv) ? H[i * nv + j] : T(0);
  SYNC();
  T dinv = T(1);
#pragma unroll
  for (int k = 0; k < NVM; k++) {
    if (k < nv) {
      T d = lane_bcast(col[k], k);
      d = d > tiny ? d : tiny;
      const T ri = rsqrt_div(d);
      const T lj = col[k] * ri;  // lane j > k: L[j][k]; lane k: L[k][k]
      if (j == k) dinv = ri;
      if (j >= k) col[k] = lj;
      T lv[NVM];
#pragma unroll
      for (int i = k + 1; i < NVM; i++) lv[i] = lane_bcast(lj, i);
      if (j > k) {
#pragma unroll
        for (int i = k + 1; i < NVM; i++) col[i] -= lv[i] * lj;
      }
    }
  }
  T acc = j < nv ? (T)-g[j] : T(0);
  T y = T(0);
#pragma unroll
  for (int k = 0; k < NVM; k++) {
    if (k < nv) {
      const T yk = lane_bcast(acc * dinv, k);
      if (j == k) y = yk;
      if (j > k) acc -= col[k] * yk;
    }
  }
  T acc2 = y, x = T(0);
#pragma unroll
  for (int k = NVM - 1; k >= 0; k--) {
    if (k < nv) {
      const T xk = lane_bcast(acc2 * dinv, k);
      if (j == k) x = xk;
      if (j < k) acc2 -= col[k] * dinv * xk;
    }
  }
  if (j < nv) dir[j] = x;
  SYNC();
}

// ------------------------------------------------------------------------------------------------
// Newton solver on the primal cost (see oracle/solver.c for the definition)
// ------------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T edge_val(const T* x3, T mu, int e) {
  return x3[0] + ((e & 1) ? -mu : mu) * x3[1 + (e >> 1)];
}

// contact-frame products B x for every contact: one lane per (contact, frame row), the <= 9 + 9 columns
// unrolled with unconditional loads (x[o + j] stays inside the nv vector for every tree; columns past the
// contact's own are selected away, never multiplied), accumulated in O and stored as O at the record's slot
// (O = T for the velocity products of the rows' reference accelerations; O = double for the Newton iterate's
// products JA / JD, whose float-by-float terms are exact in double)
#ifndef FM_JX_UNROLL
#define FM_JX_UNROLL 2
#endif
// rounds of (contact, row) items per pass of contact_jx / rows_eval2 in the scenes whose contact capacity exceeds the
// wave (their records live in the arena's global scratch block: the rounds' record loads issue together).  A round
// past the last item reads record 0 (always valid when the loop runs) and stores nothing: no load indexes a slot at
// or beyond ncon, whose records hold stale data of an earlier stage.
template <typename DIM>
__host__ __device__ constexpr int jx_rounds() {
  return DIM::MAXC > WAVE ? FM_JX_UNROLL : 1;
}
template <typename O, typename T, typename DIM, typename X>
__device__ __forceinline__ void contact_jx(const Model<T>& M, const Ws<T, DIM>& w, const X* x, int ncon, int slot) {
  const DIM dm(M.dm);
  constexpr int U = jx_rounds<DIM>();
  const int ne = 3 * ncon;
  for (int e0 = LANE; e0 < ne; e0 += U * WAVE) {
    O s[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int e = e0 + u * WAVE < ne ? e0 + u * WAVE : 0;
      const int c = e / 3, r = e - 3 * c;
      const int* ci = w.ci() + 4 * c;
      const T* cr = w.cr() + CR_N * c;
      const int ta = ci[1], tb = ci[2], nda = (ci[3] >> 20) & 15, ndb = (ci[3] >> 24) & 15;
      const int oa = ta >= 0 ? tree_dof(dm, ta) : 0, ob = tb >= 0 ? tree_dof(dm, tb) : 0;
      const T* J = cr + CR_J + r * CJ;
      const T* Jb = J + nda;
      O acc = 0;
#pragma unroll
      for (int j = 0; j < 9; j++) {
        const T ja = J[j];
        const X xa = x[oa + j];
        acc += (j < nda ? (O)ja : O(0)) * (O)xa;
      }
#pragma unroll
      for (int j = 0; j < 9; j++) {
        const T jb = Jb[j];
        const X xb = x[ob + j];
        acc += (j < ndb ? (O)jb : O(0)) * (O)xb;
      }
      s[u] = acc;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int e = e0 + u * WAVE;
      if (e < ne) {
        const int c = e / 3, r = e - 3 * c;
        ((O*)(w.cr() + CR_N * c + slot))[r] = s[u];
      }
    }
  }
}

// The solver's precision split (both builds): the problem data -- J, D, aref, M, qacc_smooth -- are the build's
// reals; the iterate a, its products J a / M (a - as) / J dir / M dir, the gradient, the cost and the line
// search are float64, so the iteration converges to the optimum of the rounded problem instead of stalling at the
// float cost's resolution (sqrt(eps) in the argmin).  The Hessian and its Cholesky factor stay in the build's
// precision: an approximate Newton direction only slows the convergence (iterative refinement), it does not move
// the optimum.

// constraint part of the primal cost at the current CR_JA / RR_JAR: sum of 1/2 D jar^2 over active rows
template <typename T, typename DIM>
__device__ __forceinline__ double rows_cost(const Ws<T, DIM>& w, int ncon, int nrow, int cslot = CR_JA,
                                            int rslot = RR_JAR) {
  double cst = 0;
  for (int c = LANE; c < ncon; c += WAVE) {
    const T* cr = w.cr() + CR_N * c;
    const T mu = cr[CR_MU], D = cr[CR_D], bd = cr[CR_BD], kd = cr[CR_KD];
    const double* ja = dslot(cr, cslot);
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const T aref = -bd * edge_val(cr + CR_VEL, mu, e) - kd;
      const double jar = edge_val(ja, (double)mu, e) - (double)aref;
      if (jar < 0.0) cst += 0.5 * (double)D * jar * jar;
    }
  }
  for (int r = LANE; r < nrow; r += WAVE) {
    const int* ri = w.ri() + 4 * r;
    const T* rr = w.rr() + RR_N * r;
    const double jar = *dslot(rr, rslot);
    if (ri[2] == 0 || jar < 0.0) cst += 0.5 * (double)rr[RR_D] * jar * jar;
  }
  return wave_sum(cst);
}

// Newton warmstart (newton()): both candidates' row products in one pass -- B qacc_smooth into the line search's
// JD slots (free until then), B qacc_warmstart into JA; generic rows likewise (RR_JD / RR_JAR, minus aref).  The
// same products rows_eval forms, one J load for both.
template <typename T, typename DIM>
__device__ __forceinline__ void rows_eval2(const Model<T>& M, const Ws<T, DIM>& w, const T* xs, const double* xw,
                                           int ncon, int nrow) {
  const DIM dm(M.dm);
  constexpr int U = jx_rounds<DIM>();
  const int ne = 3 * ncon;
  for (int e0 = LANE; e0 < ne; e0 += U * WAVE) {
    double s1[U], s2[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int e = e0 + u * WAVE < ne ? e0 + u * WAVE : 0;  // past the last item: record 0, result unused
      const int c = e / 3, r = e - 3 * c;
      const int* ci = w.ci() + 4 * c;
      const T* cr = w.cr() + CR_N * c;
      const int ta = ci[1], tb = ci[2], nda = (ci[3] >> 20) & 15, ndb = (ci[3] >> 24) & 15;
      const int oa = ta >= 0 ? tree_dof(dm, ta) : 0, ob = tb >= 0 ? tree_dof(dm, tb) : 0;
      const T* J = cr + CR_J + r * CJ;
      const T* Jb = J + nda;
      double a1 = 0, a2 = 0;
#pragma unroll
      for (int j = 0; j < 9; j++) {
        const double ja = j < nda ? (double)J[j] : 0.0;
        a1 += ja * (double)xs[oa + j];
        a2 += ja * xw[oa + j];
      }
#pragma unroll
      for (int j = 0; j < 9; j++) {
        const double jb = j < ndb ? (double)Jb[j] : 0.0;
        a1 += jb * (double)xs[ob + j];
        a2 += jb * xw[ob + j];
      }
      s1[u] = a1;
      s2[u] = a2;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int e = e0 + u * WAVE;
      if (e < ne) {
        const int c = e / 3, r = e - 3 * c;
        T* cr = w.cr() + CR_N * c;
        dslot(cr, CR_JD)[r] = s1[u];
        dslot(cr, CR_JA)[r] = s2[u];
      }
    }
  }
  for (int r = LANE; r < nrow; r += WAVE) {
    const int* ri = w.ri() + 4 * r;
    T* rr = w.rr() + RR_N * r;
    *dslot(rr, RR_JD) = (double)rr[RR_C0] * (double)xs[ri[0]] +
                        (ri[1] >= 0 ? (double)rr[RR_C1] * (double)xs[ri[1]] : 0.0) - (double)rr[RR_AREF];
    *dslot(rr, RR_JAR) = (double)rr[RR_C0] * xw[ri[0]] + (ri[1] >= 0 ? (double)rr[RR_C1] * xw[ri[1]] : 0.0) -
                         (double)rr[RR_AREF];
  }
}

// f3 (per contact, float64 in CR_F3) = D * sum_active jar_e c_e, the frame force of the gradient; the edge forces
// -D jar_e (active edges) in CR_F
template <typename T, typename DIM>
__device__ __forceinline__ void contact_f3(const Ws<T, DIM>& w, int ncon) {
  for (int c = LANE; c < ncon; c += WAVE) {
    T* cr = w.cr() + CR_N * c;
    const T mu = cr[CR_MU], D = cr[CR_D];
    const double* ja = dslot(cr, CR_JA);
    double f0 = 0, f1 = 0, f2 = 0;
    T fe[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const T aref = -cr[CR_BD] * edge_val(cr + CR_VEL, mu, e) - cr[CR_KD];
      const double jar = edge_val(ja, (double)mu, e) - (double)aref;
      fe[e] = T(0);
      if (jar < 0.0) {
        const double s = (double)D * jar;
        f0 += s;
        if (e < 2)
          f1 += ((e & 1) ? -(double)mu : (double)mu) * s;
        else
          f2 += ((e & 1) ? -(double)mu : (double)mu) * s;
        fe[e] = (T)(-s);
      }
    }
    double* f3 = dslot(cr, CR_F3);
    f3[0] = f0;
    f3[1] = f1;
    f3[2] = f2;
#pragma unroll
    for (int e = 0; e < 4; e++) cr[CR_F + e] = fe[e];
  }
}

// out_i = sum over rows of J_ri * (D jar)_r for active rows  (constraint part of the gradient), accumulated in
// float64 and stored as O (double: the gradient; T: the constraint force qfrc_constraint)
template <typename T, typename DIM, typename O>
__device__ __forceinline__ void gather_JtF(const Model<T>& M, const Ws<T, DIM>& w, int ncon, int nrow, O* out, bool add) {
  const DIM dm(M.dm);
  for (int i = LANE; i < dm.nv; i += WAVE) {
    int t = dof_tree(dm, i);
    int jl = i - tree_dof(dm, t);
    double s = 0;
    const int nh = DIM::MAXC == WAVE ? 1 : (dm.maxcon + WAVE - 1) / WAVE;
    for (int h = 0; h < nh; h++) {
    uint64_t mk = w.tmask()[h * dm.ntree + t];
    while (mk) {
      int c = WAVE * h + __ffsll((unsigned long long)mk) - 1;
      mk &= mk - 1;
      const int* ci = w.ci() + 4 * c;
      const T* cr = w.cr() + CR_N * c;
      int nda = (ci[3] >> 20) & 15;
      int col = ci[1] == t ? jl : nda + jl;
      const T* J = cr + CR_J;
      const double* f3 = dslot(cr, CR_F3);
      s += (double)J[col] * f3[0] + (double)J[CJ + col] * f3[1] + (double)J[2 * CJ + col] * f3[2];
    }
    }
    for (int r = 0; r < nrow; r++) {
      const int* ri = w.ri() + 4 * r;
      const T* rr = w.rr() + RR_N * r;
      const double jar = *dslot(rr, RR_JAR);
      if (!(ri[2] == 0 || jar < 0.0)) continue;
      const double fr = (double)rr[RR_D] * jar;
      if (ri[0] == i) s += (double)rr[RR_C0] * fr;
      if (ri[1] == i) s += (double)rr[RR_C1] * fr;
    }
    out[i] = add ? (O)((double)out[i] + s) : (O)s;
  }
}

// gather_JtF by scatter ((2,4) scene): one lane per (contact, Jacobian column) adds its column's product with the
// contact's frame force into a float64 accumulator by LDS atomics (one wave: a fixed order), one lane per generic
// row likewise; the per-dof loop above is a chain of dependent LDS reads on the belt's lane, which carries every
// belt contact.  (Round 4: reducing the belt's column by a wave sum instead of its same-address atomics was measured
// slower -- gradient 5.22 -> 5.70 us per arena-substep -- and left the LDS bank-conflict rate unchanged.)  acc: nv
// doubles of scratch (the solver's tmp, dead at the gradient and at the final forces).
template <typename T, typename DIM, typename O>
__device__ __forceinline__ void gather_JtF_sc(const Model<T>& M, const Ws<T, DIM>& w, int ncon, int nrow, O* out,
                                              double* acc) {
  const DIM dm(M.dm);
  for (int i = LANE; i < dm.nv; i += WAVE) acc[i] = 0.0;
  SYNC();
#ifndef FM_SC_UNROLL
#define FM_SC_UNROLL 2
#endif
  // FM_SC_UNROLL rounds of (contact, column) pairs per pass: their record loads (the arena's global block) issue
  // together before the atomics, in the same atomic order as one round per pass (round 4, one box, two runs each:
  // config 2 187.8k -> 190.0k with 2 rounds, 184.3k with 4 -- the registers they hold, profiles/r04s_*)
  for (int e0 = LANE; e0 < CJ * ncon; e0 += FM_SC_UNROLL * WAVE) {
    double v[FM_SC_UNROLL];
    int gi[FM_SC_UNROLL];
    bool ok[FM_SC_UNROLL];
#pragma unroll
    for (int u = 0; u < FM_SC_UNROLL; u++) {
      const int e = e0 + u * WAVE;
      const int c = e < CJ * ncon ? e / CJ : 0, ii = e < CJ * ncon ? e - CJ * c : CJ;
      const int* ci = w.ci() + 4 * c;
      const int ta = ci[1], tb = ci[2], nda = (ci[3] >> 20) & 15, ndb = (ci[3] >> 24) & 15;
      const T* cr = w.cr() + CR_N * c;
      const T* J = cr + CR_J;
      const double* f3 = dslot(cr, CR_F3);
      const int iic = ii < CJ ? ii : 0;
      v[u] = (double)J[iic] * f3[0] + (double)J[CJ + iic] * f3[1] + (double)J[2 * CJ + iic] * f3[2];
      gi[u] = ii < nda ? tree_dof(dm, ta) + ii : tree_dof(dm, tb >= 0 ? tb : 0) + ii - nda;
      ok[u] = ii < nda + ndb;
    }
#pragma unroll
    for (int u = 0; u < FM_SC_UNROLL; u++)
      if (ok[u]) atomicAdd(acc + gi[u], v[u]);
  }
  for (int r = LANE; r < nrow; r += WAVE) {
    const int* ri = w.ri() + 4 * r;
    const T* rr = w.rr() + RR_N * r;
    const double jar = *dslot(rr, RR_JAR);
    if (!(ri[2] == 0 || jar < 0.0)) continue;
    const double fr = (double)rr[RR_D] * jar;
    atomicAdd(acc + ri[0], (double)rr[RR_C0] * fr);
    if (ri[1] >= 0) atomicAdd(acc + ri[1], (double)rr[RR_C1] * fr);
  }
  SYNC();
  for (int i = LANE; i < dm.nv; i += WAVE) out[i] = (O)acc[i];
}

// ------------------------------------------------------------------------------------------------
// Tree-block Newton solve of the fp32 scenes with spilled records ((2,8), (2,10): configs 3 / 4; (4,16): config 5):
// H dir = -g without the dense Hessian.
// H couples two trees only through a contact between them (mass matrix: belt scalar, cubes diagonal, arm 9 x 9
// blocks; generic rows stay inside one arm).  Elimination order: the single trees (no contact with another moving
// tree except the belt), then the coupled trees, the belt last.  In that order H is block diagonal over the singles
// with the coupled trees' block and a belt border, so
//  * every single tree's 9 x 9 block (cubes padded with an identity) is factored on its own lane, serially in
//    registers, together with its belt row l_t = L_t^-1 h_bt and its forward solve y_t = L_t^-1 (-g_t);
//  * the rest -- the coupled trees (an arm grasping a cube, two cubes touching: 15-24 dofs measured on the oracle's
//    PauseIKToggle trajectories) plus the belt, with the singles' Schur terms sum l_t'l_t and sum l_t'y_t folded into
//    the belt's diagonal and right-hand side -- is one small dense system for the register Cholesky
//    (chol_solve_rl<TB_MAXR>: pivots by v_readlane; the LDS-broadcast chol_solve_reg measured 4.6 % slower);
//  * the singles' backward solves take the belt's solution from it.
// The blocks are assembled in LDS (the Newton phase's share of the collision scratch): one lane per contact adds
// B_a'K B_a, B_b'K B_b and the cross term B_a'K B_b (a belt row, the coupled system, or -- a contact inside one
// tree -- the tree's own block) by LDS atomics; one lane per generic row likewise.  The same terms as the dense
// assembly, summed in another order (fp32 rounding differs from the dense path; both are held to the oracle).
// Returns false (nothing written but K_c) when more than TB_MAXR positions are coupled or a generic row couples two
// trees: the caller runs the scene's dense path.  Replaces the dense assembly (global atomics: the Hessian lives in
// the arena's global block) and the dense factors: (4,16) Hessian + Cholesky 44 + 117 -> 16 + 15 us of 273 -> 138 us
// per arena-substep (round 4, profiles/r04h_phase_fp32_4x16_treeblk.json).
// gather_JtF by per-contact scatter (the compile-time scenes whose contact records live in the arena's global block:
// (2,8), (2,10), (4,16)): one lane per contact adds its <= 18 column products J_c' f_c into the float64 accumulator by
// LDS atomics, one lane per generic row likewise -- one round of record loads for up to 64 contacts, where the per-dof
// walk over a tree's contacts is a chain of global-latency loads (the belt's lane walks every belt contact)
template <typename T, typename DIM, typename O>
__device__ __forceinline__ void gather_JtF_pc(const Model<T>& M, const Ws<T, DIM>& w, int ncon, int nrow, O* out,
                                              double* acc) {
  const DIM dm(M.dm);
  for (int i = LANE; i < dm.nv; i += WAVE) acc[i] = 0.0;
  SYNC();
  for (int c = LANE; c < ncon; c += WAVE) {
    const int* ci = w.ci() + 4 * c;
    const int ta = ci[1], tb = ci[2], nda = (ci[3] >> 20) & 15, ndb = (ci[3] >> 24) & 15;
    const T* cr = w.cr() + CR_N * c;
    const T* J = cr + CR_J;
    const double* f3 = dslot(cr, CR_F3);
    const double f0 = f3[0], f1 = f3[1], f2 = f3[2];
    const int oa = ta >= 0 ? tree_dof(dm, ta) : 0, ob = (tb >= 0 ? tree_dof(dm, tb) : 0) - nda;
    double v[CJ];
#pragma unroll
    for (int ii = 0; ii < CJ; ii++) v[ii] = (double)J[ii] * f0 + (double)J[CJ + ii] * f1 + (double)J[2 * CJ + ii] * f2;
#pragma unroll
    for (int ii = 0; ii < CJ; ii++)
      if (ii < nda + ndb) atomicAdd(acc + (ii < nda ? oa : ob) + ii, v[ii]);
  }
  for (int r = LANE; r < nrow; r += WAVE) {
    const int* ri = w.ri() + 4 * r;
    const T* rr = w.rr() + RR_N * r;
    const double jar = *dslot(rr, RR_JAR);
    if (!(ri[2] == 0 || jar < 0.0)) continue;
    const double fr = (double)rr[RR_D] * jar;
    atomicAdd(acc + ri[0], (double)rr[RR_C0] * fr);
    if (ri[1] >= 0) atomicAdd(acc + ri[1], (double)rr[RR_C1] * fr);
  }
  SYNC();
  for (int i = LANE; i < dm.nv; i += WAVE) out[i] = (O)acc[i];
}
template <typename T, typename DIM>
__device__ constexpr bool pc_scene() {
  if constexpr (DIM::fixed)
    return (DIM::spill || DIM::rerun) && !(DIM::MAXC == WAVE && DIM::nv <= 48);  // not the (2,4) 64-contact scene
  else
    return false;
}

template <typename T, typename DIM>
__device__ constexpr bool treeblk_scene() {
  if constexpr (DIM::fixed)
    return DIM::template treeblk_for<sizeof(T)>();
  else
    return false;
}
__device__ __forceinline__ unsigned wave_or_u32(unsigned x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x |= (unsigned)__shfl_xor((int)x, o);
  return x;
}
template <typename T, typename DIM>
__device__ __forceinline__ bool newton_treeblk(const Model<T>& M, const Ws<T, DIM>& w, const double* g, T* dir,
                                               int ncon, int nrow) {
  constexpr int NT = DIM::ntree, KK = DIM::K;
  static_assert(NT <= 32 && DIM::nv <= 1 + 9 * (NT - 1), "one 32-bit tree mask; trees of <= 9 dofs");
  const DIM dm(M.dm);
  contact_K(w, ncon);
  SYNC();
  // ---- coupled trees: both moving trees (not the belt, not the world) of a contact with an active edge
  unsigned cm = 0;
  bool rowx = false;
  for (int c = LANE; c < ncon; c += WAVE) {
    const int* ci = w.ci() + 4 * c;
    const int ta = ci[1], tb = ci[2];
    if (ta > 0 && tb > 0 && ta != tb && w.cr()[CR_N * c + CR_K] != 0.0f) cm |= (1u << ta) | (1u << tb);
  }
  for (int r = LANE; r < nrow; r += WAVE) {
    const int* ri = w.ri() + 4 * r;
    if (ri[1] >= 0 && dof_tree(dm, ri[0]) != dof_tree(dm, ri[1])) rowx = true;
  }
  cm = wave_or_u32(cm);
  constexpr unsigned CUBES = ((1u << KK) - 1u) << 1;
  const int m = 6 * __popc(cm & CUBES) + 9 * __popc(cm & ~CUBES);  // coupled positions (the belt excluded)
  if (m + 1 > TB_MAXR || __ballot(rowx) != 0ull) return false;
  const int n = m + 1;
  // position of tree t's first dof in the coupled system (trees in index order: cubes, then arms)
  auto cbase = [&](int t) {
    const unsigned below = cm & ((1u << t) - 1u);
    return 6 * __popc(below & CUBES) + 9 * __popc(below & ~CUBES);
  };
  T* const tbw = w.tblk();
  constexpr bool GR = DIM::template gl_tbr<sizeof(T)>();
  T* const R = w.tbr();
  int* const cmap = (int*)(tbw + tb_map(NT, GR));
  // ---- zero the blocks, belt rows and the coupled system; the coupled system's position map
  for (int e = LANE; e < TB_BLK * NT; e += WAVE) tbw[e] = 0.0f;
  for (int e = LANE; e < n * n; e += WAVE) R[e] = 0.0f;
  if (LANE > 0 && LANE < NT && ((cm >> LANE) & 1u)) {
    const int b = cbase(LANE), nd = LANE <= KK ? 6 : 9;
    for (int k = 0; k < nd; k++) cmap[b + k] = (LANE << 4) | k;
  }
  SYNC();
  // ---- mass matrix: belt and cube diagonals, arm blocks (lower triangles)
  for (int d = LANE; d < dm.nv; d += WAVE) {
    const int t = dof_tree(dm, d), i = d - tree_dof(dm, t);
    T* B = tbw + TB_BLK * t;
    if (t <= KK) {
      B[P9(i, i)] = Mdiag(M, w, d);
    } else {
      const T* Mr = w.Marm() + 81 * (t - 1 - KK) + 9 * i;
      for (int j = 0; j <= i; j++) B[P9(i, j)] = Mr[j];
    }
  }
  SYNC();
  // ---- contacts: one lane per contact
  for (int c = LANE; c < ncon; c += WAVE) {
    const int* ci = w.ci() + 4 * c;
    const T* cr = w.cr() + CR_N * c;
    const T* Kc = cr + CR_K;
    const T k0 = Kc[0], k1 = Kc[1], k2 = Kc[2], k3 = Kc[3], k4 = Kc[4], k5 = Kc[5];
    if (k0 == T(0)) continue;  // no active pyramid edge: no Hessian term
    const int ta = ci[1], tb = ci[2], nda = (ci[3] >> 20) & 15, ndb = (ci[3] >> 24) & 15;
    const T* J = cr + CR_J;
    T ja[3][9], jb[3][9], qa[3][9], qb[3][9];
#pragma unroll
    for (int i = 0; i < 9; i++) {
#pragma unroll
      for (int r = 0; r < 3; r++) {
        ja[r][i] = J[r * CJ + i];
        jb[r][i] = J[r * CJ + nda + i];  // nda + i <= 17 < CJ: inside the record
      }
      qa[0][i] = k0 * ja[0][i] + k3 * ja[1][i] + k4 * ja[2][i];
      qa[1][i] = k3 * ja[0][i] + k1 * ja[1][i] + k5 * ja[2][i];
      qa[2][i] = k4 * ja[0][i] + k5 * ja[1][i] + k2 * ja[2][i];
      qb[0][i] = k0 * jb[0][i] + k3 * jb[1][i] + k4 * jb[2][i];
      qb[1][i] = k3 * jb[0][i] + k1 * jb[1][i] + k5 * jb[2][i];
      qb[2][i] = k4 * jb[0][i] + k5 * jb[1][i] + k2 * jb[2][i];
    }
    // own blocks of the two trees (a tree < 0 is the world: no columns)
    if (ta >= 0) {
      T* B = tbw + TB_BLK * ta;
#pragma unroll
      for (int i = 0; i < 9; i++)
#pragma unroll
        for (int j = 0; j <= i; j++)
          if (i < nda) atomicAdd(B + P9(i, j), qa[0][i] * ja[0][j] + qa[1][i] * ja[1][j] + qa[2][i] * ja[2][j]);
    }
    if (tb >= 0) {
      T* B = tbw + TB_BLK * tb;
#pragma unroll
      for (int i = 0; i < 9; i++)
#pragma unroll
        for (int j = 0; j <= i; j++)
          if (i < ndb) atomicAdd(B + P9(i, j), qb[0][i] * jb[0][j] + qb[1][i] * jb[1][j] + qb[2][i] * jb[2][j]);
    }
    if (ta < 0 || tb < 0) continue;
    // cross term B_a' K B_b: a belt row, a contact inside one tree, or an entry pair of the coupled system
    if (tb == 0 || ta == 0) {
      const bool bb = tb == 0;  // the belt is tree b: tree a's belt row, else tree b's
      T* Bl = tbw + TB_BLK * (bb ? ta : tb) + 45;
#pragma unroll
      for (int i = 0; i < 9; i++) {
        const T v = bb ? qa[0][i] * jb[0][0] + qa[1][i] * jb[1][0] + qa[2][i] * jb[2][0]
                           : qb[0][i] * ja[0][0] + qb[1][i] * ja[1][0] + qb[2][i] * ja[2][0];
        if (i < (bb ? nda : ndb)) atomicAdd(Bl + i, v);
      }
    } else if (ta == tb) {
      T* B = tbw + TB_BLK * ta;
#pragma unroll
      for (int i = 0; i < 9; i++)
#pragma unroll
        for (int k = 0; k < 9; k++) {
          const T v = qa[0][i] * jb[0][k] + qa[1][i] * jb[1][k] + qa[2][i] * jb[2][k];
          if (i < nda && k < ndb) atomicAdd(B + (i >= k ? P9(i, k) : P9(k, i)), i == k ? T(2) * v : v);
        }
    } else {
      const int ca = cbase(ta), cb = cbase(tb);
#pragma unroll
      for (int i = 0; i < 9; i++)
#pragma unroll
        for (int k = 0; k < 9; k++) {
          const T v = qa[0][i] * jb[0][k] + qa[1][i] * jb[1][k] + qa[2][i] * jb[2][k];
          if (i < nda && k < ndb) {
            atomicAdd(R + (ca + i) * n + cb + k, v);
            atomicAdd(R + (cb + k) * n + ca + i, v);
          }
        }
    }
  }
  // ---- generic rows (gripper equality, joint limits: inside one tree), one lane per row
  for (int r = LANE; r < nrow; r += WAVE) {
    const int* ri = w.ri() + 4 * r;
    const T* rr = w.rr() + RR_N * r;
    if (!(ri[2] == 0 || *dslot(rr, RR_JAR) < 0.0)) continue;
    const T D = rr[RR_D], c0 = rr[RR_C0], c1 = rr[RR_C1];
    const int d0 = ri[0], d1 = ri[1], t = dof_tree(dm, d0), o = tree_dof(dm, t);
    T* B = tbw + TB_BLK * t;
    const int l0 = d0 - o;
    atomicAdd(B + P9(l0, l0), D * c0 * c0);
    if (d1 >= 0) {
      const int l1 = d1 - o;
      atomicAdd(B + P9(l1, l1), D * c1 * c1);
      atomicAdd(B + (l0 >= l1 ? P9(l0, l1) : P9(l1, l0)), (l0 == l1 ? T(2) : T(1)) * D * c0 * c1);
    }
  }
  SYNC();
  PMARK(PH_NHESS);
  // ---- single trees: lane t factors its block, its belt row and its forward solve in registers
  const T tiny = sizeof(T) == 4 ? T(1e-37f) : T(1e-300);
  const int t = LANE;
  const bool single = t > 0 && t < NT && !((cm >> t) & 1u);
  const bool cube = t <= KK;
  const int d0 = t < NT ? tree_dof(dm, t) : 0;
  T Lb[45], dv[9], lb[9], y[9];
  T s_t = T(0), ly_t = T(0);
  if (single) {
    const T* B = tbw + TB_BLK * t;
#pragma unroll
    for (int k = 0; k < 45; k++) Lb[k] = B[k];
#pragma unroll
    for (int k = 0; k < 9; k++) lb[k] = B[45 + k];
    if (cube) {  // identity padding of the cube's 6 x 6 block (its rows 6..8 and belt entries 6..8 are zero)
      Lb[P9(6, 6)] = T(1);
      Lb[P9(7, 7)] = T(1);
      Lb[P9(8, 8)] = T(1);
    }
#pragma unroll
    for (int k = 0; k < 9; k++) {
      T d = Lb[P9(k, k)];
      d = d > tiny ? d : tiny;
      const T ri = rsqrt_div(d);
      dv[k] = ri;
#pragma unroll
      for (int i = k + 1; i < 9; i++) Lb[P9(i, k)] *= ri;
#pragma unroll
      for (int i = k + 1; i < 9; i++)
#pragma unroll
        for (int j = k + 1; j <= i; j++) Lb[P9(i, j)] -= Lb[P9(i, k)] * Lb[P9(j, k)];
    }
#pragma unroll
    for (int i = 0; i < 9; i++) {
      T a = lb[i], b = (cube && i >= 6) ? T(0) : (T)-g[d0 + (i < 9 ? i : 0)];
#pragma unroll
      for (int k = 0; k < i; k++) {
        a -= Lb[P9(i, k)] * lb[k];
        b -= Lb[P9(i, k)] * y[k];
      }
      lb[i] = a * dv[i];
      y[i] = b * dv[i];
      s_t += lb[i] * lb[i];
      ly_t += lb[i] * y[i];
    }
  }
  const T S = wave_sum(s_t), LY = wave_sum(ly_t);
  // ---- the coupled system + belt (position m), in LDS with row stride n
  double* const grest = (double*)(tbw + tb_rhs(NT, GR));  // right-hand side (chol_solve_reg negates it)
  T* const xr = tbw + tb_sol(NT, GR);                  // its solution
  for (int e = LANE; e < n * n; e += WAVE) {
    const int i = e / n, j = e - n * (e / n);
    if (i < m && j < m) {
      const int ti = cmap[i] >> 4, li = cmap[i] & 15, tj = cmap[j] >> 4, lj = cmap[j] & 15;
      if (ti == tj) R[e] = tbw[TB_BLK * ti + (li >= lj ? P9(li, lj) : P9(lj, li))];
    } else if (i == m && j == m) {
      R[e] = tbw[0] - S;  // the belt's diagonal (block of tree 0) minus the singles' Schur terms
    } else {
      const int p = i == m ? j : i;
      R[e] = tbw[TB_BLK * (cmap[p] >> 4) + 45 + (cmap[p] & 15)];
    }
  }
  for (int i = LANE; i < n; i += WAVE)
    grest[i] = i < m ? g[tree_dof(dm, cmap[i] >> 4) + (cmap[i] & 15)] : g[0] + (double)LY;
  SYNC();
  chol_solve_rl<TB_MAXR, T>(R, n, grest, xr);
  // ---- back substitution: the coupled positions and the belt from the dense solve, the singles on their lanes
  const T xb = xr[m];
  for (int i = LANE; i < m; i += WAVE) dir[tree_dof(dm, cmap[i] >> 4) + (cmap[i] & 15)] = xr[i];
  if (LANE == 0) dir[0] = xb;
  if (single) {
    T x[9];
#pragma unroll
    for (int i = 8; i >= 0; i--) {
      T a = y[i] - lb[i] * xb;
#pragma unroll
      for (int k = i + 1; k < 9; k++) a -= Lb[P9(k, i)] * x[k];
      x[i] = a * dv[i];
    }
#pragma unroll
    for (int i = 0; i < 9; i++)
      if (i < (cube ? 6 : 9)) dir[d0 + i] = x[i];
  }
  SYNC();
  return true;
}

template <typename T, typename DIM>
__device__ __forceinline__ void newton(const Model<T>& M, const Ws<T, DIM>& w, int arena, int64_t* ctr) {
  const DIM dm(M.dm);
  const int nv = dm.nv;
  const int ncon = w.misc()[MISC_NCON], nrow = w.misc()[MISC_NROW];
  double* a = w.a();
  const T* as = w.as();
  double* g = w.g();
  T* dir = w.dir();
  double* Ma = w.Ma();
  double* tmp = w.tmp();
  T* H = w.H();
  const int hs = hstride(sizeof(T), nv);  // == nv except for the dense blocked Cholesky's scenes
  const double scale = 1.0 / ((double)M.meaninertia[arena] * (double)(nv > 1 ? nv : 1));
  const double tol = M.solver_tol;
  // quadratic part helper: returns 1/2 (x-as)' M (x-as), leaves M(x-as) in Ma
  auto quad = [&](const double* x) -> double {
    for (int i = LANE; i < nv; i += WAVE) tmp[i] = x[i] - (double)as[i];
    SYNC();
    mmul(M, w, arena, tmp, Ma);
    SYNC();
    double s = 0;
    for (int i = LANE; i < nv; i += WAVE) s += 0.5 * tmp[i] * Ma[i];
    return wave_sum(s);
  };
  // warmstart: the cheaper of qacc_warmstart and qacc_smooth.  The smooth candidate is evaluated first (its
  // quadratic part is zero), so in the common case (the warmstart wins) the row products and M(a - as) left
  // behind are already those of the chosen start and need no third evaluation
  double qc, cost;
  {
    // both candidates' row products in one pass (rows_eval2); the smooth candidate's land in the JD slots
    rows_eval2(M, w, as, a, ncon, nrow);
    SYNC();
    const double c_sm = rows_cost(w, ncon, nrow, CR_JD, RR_JD);
    const double c_ws = rows_cost(w, ncon, nrow);
    SPLITMARK(1, PH_CHSOLVE);
    qc = quad(a);
    cost = qc + c_ws;
    SYNC();
    if (!(cost < c_sm)) {
      // the smooth candidate wins: a = qacc_smooth, its products move into JA (its quadratic part is zero)
      for (int i = LANE; i < nv; i += WAVE) a[i] = (double)as[i];
      for (int e = LANE; e < 3 * ncon; e += WAVE) {
        T* cr = w.cr() + CR_N * (e / 3);
        dslot(cr, CR_JA)[e % 3] = dslot(cr, CR_JD)[e % 3];
      }
      for (int r = LANE; r < nrow; r += WAVE) {
        T* rr = w.rr() + RR_N * r;
        *dslot(rr, RR_JAR) = *dslot(rr, RR_JD);
      }
      SYNC();
      qc = quad(a);
      cost = qc + c_sm;
      SYNC();
    }
  }
  PMARK(PH_NSETUP);
  int it;
  const int maxit = M.solver_iter;
  constexpr bool scatter = arrow_scene<T, DIM>();  // gather_JtF_sc
  const int ntri = nv * (nv + 1) / 2;
  for (it = 0; it < maxit; it++) {
    // gradient g = M(a - as) + J' D jar (active)
    contact_f3(w, ncon);
    SYNC();
    SPLITMARK(2, PH_CHDIAG);
    if constexpr (scatter)
      gather_JtF_sc(M, w, ncon, nrow, g, tmp);
    else if constexpr (pc_scene<T, DIM>())
      gather_JtF_pc(M, w, ncon, nrow, g, tmp);
    else
      gather_JtF(M, w, ncon, nrow, g, false);
    SYNC();
    SPLITMARK(2, PH_CHPANEL);
    double gn = 0;
    for (int i = LANE; i < nv; i += WAVE) {
      g[i] += Ma[i];
      gn += g[i] * g[i];
    }
    gn = wave_sum(gn);
    PMARK(PH_NGRAD);
    if (scale * scale * gn < tol * tol) break;  // scale |g| < tol without the float64 square root on the chain
    // arrowhead substeps of the (2,4) scene (no contact couples two trees other than the belt: nearly every
    // substep): H is assembled straight into the block-parallel factor's registers, no LDS Hessian
    bool solved = false;
    if constexpr (arrow_scene<T, DIM>()) {
      if (arrow_substep(M, w)) {
        contact_K(w, ncon);
        SYNC();
        chol_arrow_rl<T, DIM, true>(M, w, H, g, dir, ncon, nrow);
        PMARK(PH_NCHOL);
        solved = true;
      }
    }
    if constexpr (treeblk_scene<T, DIM>()) {
      // FM_NO_TREEBLK=1 / FM_CHOL_LDS=2: the dense Hessian and its factors (the equivalence tests' reference forms)
      if (!solved && !(FM_XF(M) & (2048 | 2)) && newton_treeblk<T, DIM>(M, w, g, dir, ncon, nrow)) {
        PMARK(PH_NCHOL);
        solved = true;
      }
    }
    if (!solved) {
    // Hessian H = M + sum_c B_c' K_c B_c + generic rows
    {
      // zero fill in 16-byte stores (the region is 16-byte aligned), then the tail
      constexpr int PER16 = 16 / sizeof(T);
      const int n16 = hs * hs / PER16;
      uint4* H16 = (uint4*)H;
      for (int e = LANE; e < n16; e += WAVE) H16[e] = make_uint4(0u, 0u, 0u, 0u);
      for (int e = n16 * PER16 + LANE; e < hs * hs; e += WAVE) H[e] = T(0);
    }
    SYNC();
    {
      int a0 = 1 + 6 * dm.K;
      for (int i = LANE; i < hs; i += WAVE) {
        if (i >= nv) {
          H[i * hs + i] = T(1);  // padding (dense blocked Cholesky): an identity block
        } else if (i < a0) {
          H[i * hs + i] = Mdiag(M, w, i);
        } else {
          int arm = (i - a0) / 9, r = (i - a0) % 9;
          for (int j = 0; j < 9; j++) H[i * hs + a0 + 9 * arm + j] = w.Marm()[81 * arm + 9 * r + j];
        }
      }
    }
    SYNC();
    // contact blocks B_c' K_c B_c: K_c (3x3, from the active pyramid edges) for every contact at once, then
    // one lane per (contact, block column ii) in fixed slots of CJ, adding its whole block column with LDS
    // atomics (one wave: deterministic order).  The column's operands are read unconditionally (all inside the
    // record), so the loads issue as one batch; only the atomics are predicated on the contact's column count.
    // (Summing consecutive contacts between the same two trees on one lane before the atomics was slower: the
    // serial per-lane chain costs more than the atomics it saves.)
    contact_K(w, ncon);
    SYNC();
    for (int e = LANE; e < CJ * ncon; e += WAVE) {
      const int c = e / CJ, ii = e - CJ * c;
      const int* ci = w.ci() + 4 * c;
      const T* cr = w.cr() + CR_N * c;
      const int ta = ci[1], tb = ci[2], nda = (ci[3] >> 20) & 15, ndb = (ci[3] >> 24) & 15;
      const int ncol = nda + ndb;
      const T* Kc = cr + CR_K;
      if (ii >= ncol || Kc[0] == T(0)) continue;
      const T* J = cr + CR_J;
      const T b0 = J[ii], b1 = J[CJ + ii], b2 = J[2 * CJ + ii];
      const T q0 = Kc[0] * b0 + Kc[3] * b1 + Kc[4] * b2;
      const T q1 = Kc[3] * b0 + Kc[1] * b1 + Kc[5] * b2;
      const T q2 = Kc[4] * b0 + Kc[5] * b1 + Kc[2] * b2;
      const int oa = ta >= 0 ? tree_dof(dm, ta) : 0, ob = tb >= 0 ? tree_dof(dm, tb) : 0;
      const int gi = ii < nda ? oa + ii : ob + ii - nda;
      T* Hrow = H + gi * hs;
      T jr0[CJ], jr1[CJ], jr2[CJ];
#pragma unroll
      for (int jj = 0; jj < CJ; jj++) {
        jr0[jj] = J[jj];
        jr1[jj] = J[CJ + jj];
        jr2[jj] = J[2 * CJ + jj];
      }
#pragma unroll
      for (int jj = 0; jj < CJ; jj++) {
        const int gj = jj < nda ? oa + jj : ob + jj - nda;
        const T val = q0 * jr0[jj] + q1 * jr1[jj] + q2 * jr2[jj];
        if (jj < ncol) atomicAdd(Hrow + gj, val);
      }
    }
    SYNC();
    // generic rows, one per lane (rows may share a dof: atomics)
    for (int r = LANE; r < nrow; r += WAVE) {
      const int* ri = w.ri() + 4 * r;
      const T* rr = w.rr() + RR_N * r;
      if (!(ri[2] == 0 || *dslot(rr, RR_JAR) < 0.0)) continue;
      const T D = rr[RR_D];
      const int d0 = ri[0], d1 = ri[1];
      atomicAdd(H + d0 * hs + d0, D * rr[RR_C0] * rr[RR_C0]);
      if (d1 >= 0) {
        atomicAdd(H + d1 * hs + d1, D * rr[RR_C1] * rr[RR_C1]);
        atomicAdd(H + d0 * hs + d1, D * rr[RR_C0] * rr[RR_C1]);
        atomicAdd(H + d1 * hs + d0, D * rr[RR_C0] * rr[RR_C1]);
      }
    }
    SYNC();
    PMARK(PH_NHESS);
    if (nv <= 48) {
      if constexpr (DIM::fixed && DIM::MAXC == WAVE)  // tree masks of one word
        chol_sparse_rl<T, DIM>(M, w, H, g, dir);
      else
        chol_solve_reg<T, 48>(H, w.bc(), nv, g, dir);
      PMARK(PH_NCHOL);
    } else if (nv <= 64) {
      chol_solve_reg<T, 64>(H, w.bc(), nv, g, dir);
      PMARK(PH_NCHOL);
    } else if (border_chol<T, DIM>()) {
      if constexpr (border_chol<T, DIM>()) {
        if (arrow_substep(M, w))
          chol_arrow2_rl<T, DIM>(H, g, dir);
        else
          chol_sparse_border<DIM>(M, w, H, g, dir);
      }
      PMARK(PH_NCHOL);
    } else if (dense_mfma_chol<T, DIM>() && nv > 80 && !(FM_XF(M) & 2)) {  // hstride() pads these; FM_CHOL_LDS=2: the sparse LDS factor
      if constexpr (dense_mfma_chol<T, DIM>()) chol_dense_mfma<DIM>(M, w, H, nv, g, dir);
      PMARK(PH_NCHOL);
    } else if (chol_sparse_lds(M, w, H, g, dir)) {
      PMARK(PH_NCHOL);
    } else {
      // dense Cholesky (right-looking over the column-major lower-triangle table)
      int colstart = 0;
      for (int k = 0; k < nv; k++) {
        if (LANE == 0) {
          T s = H[k * hs + k];
          H[k * hs + k] = sqrt(s > T(1e-300) ? s : T(1e-300));
        }
        SYNC();
        T lkk = H[k * hs + k];
        for (int i = k + 1 + LANE; i < nv; i += WAVE) H[i * hs + k] /= lkk;
        SYNC();
        colstart += nv - k;  // start of column k+1 in the table
        for (int e = colstart + LANE; e < ntri; e += WAVE) {
          uint32_t ij = M.tri[e];
          int i = ij & 0xFFFF, j = ij >> 16;
          H[i * hs + j] -= H[i * hs + k] * H[j * hs + k];
        }
        SYNC();
      }
      PMARK(PH_NCHOL);
      // dir = -H^-1 g  (column-oriented substitutions)
      for (int i = LANE; i < nv; i += WAVE) dir[i] = (T)-g[i];
      SYNC();
      for (int k = 0; k < nv; k++) {
        T xk = dir[k] / H[k * hs + k];
        SYNC();
        if (LANE == 0) dir[k] = xk;
        for (int i = k + 1 + LANE; i < nv; i += WAVE) dir[i] -= H[i * hs + k] * xk;
        SYNC();
      }
      for (int k = nv - 1; k >= 0; k--) {
        T xk = dir[k] / H[k * hs + k];
        SYNC();
        if (LANE == 0) dir[k] = xk;
        for (int i = LANE; i < k; i += WAVE) dir[i] -= H[k * hs + i] * xk;
        SYNC();
      }
    }
    }  // !solved
    PMARK(PH_NSOLVE);
    // exact line search along dir (segment walking over the breakpoints of the inequality rows)
    // Jd per contact (frame components) and per generic row
    contact_jx<double>(M, w, dir, ncon, CR_JD);
    for (int r = LANE; r < nrow; r += WAVE) {
      const int* ri = w.ri() + 4 * r;
      T* rr = w.rr() + RR_N * r;
      *dslot(rr, RR_JD) = (double)rr[RR_C0] * (double)dir[ri[0]] +
                          (ri[1] >= 0 ? (double)rr[RR_C1] * (double)dir[ri[1]] : 0.0);
    }
    mmul(M, w, arena, dir, tmp);
    SYNC();
    double dMd = 0, dMa = 0;
    for (int i = LANE; i < nv; i += WAVE) {
      dMd += (double)dir[i] * tmp[i];
      dMa += (double)dir[i] * Ma[i];
    }
    dMd = wave_sum(dMd);
    dMa = wave_sum(dMa);
    SPLITMARK(2, PH_CHTRAIL);
    // the walk's per-row data is loop-invariant: the contacts (4 pyramid edges each; contact LANE + 64 h) and
    // one generic row per lane (nrow <= 64) held in registers; padding slots carry jd = 0, D = 0 and contribute
    // nothing
    constexpr int NHC = DIM::MAXC / WAVE;
    double ejar[4 * NHC], ejd[4 * NHC], ete[4 * NHC];
    T eD[NHC];
    double gjar = 0, gjd = 0, gte = 0;
    T gD = T(0);
    bool geq = false;
#pragma unroll
    for (int h = 0; h < NHC; h++) {
      eD[h] = T(0);
      if (LANE + WAVE * h < ncon) {
        const T* cr = w.cr() + CR_N * (LANE + WAVE * h);
        const T mu = cr[CR_MU], bd = cr[CR_BD], kd = cr[CR_KD];
        const double* ja = dslot(cr, CR_JA);
        const double* jd = dslot(cr, CR_JD);
        eD[h] = cr[CR_D];
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const T aref = -bd * edge_val(cr + CR_VEL, mu, e) - kd;
          ejar[4 * h + e] = edge_val(ja, (double)mu, e) - (double)aref;
          ejd[4 * h + e] = edge_val(jd, (double)mu, e);
          ete[4 * h + e] = ejd[4 * h + e] != 0.0 ? -ejar[4 * h + e] / ejd[4 * h + e] : 0.0;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; e++) {
          ejar[4 * h + e] = 1.0;
          ejd[4 * h + e] = 0.0;
          ete[4 * h + e] = 0.0;
        }
      }
    }
    if (LANE < nrow) {
      const T* rr = w.rr() + RR_N * LANE;
      geq = w.ri()[4 * LANE + 2] == 0;
      gjar = *dslot(rr, RR_JAR);
      gjd = *dslot(rr, RR_JD);
      gD = rr[RR_D];
      gte = gjd != 0.0 ? -gjar / gjd : 0.0;
    }
    double alpha = 0;
    for (int ls = 0; ls < 4 * (4 * ncon + nrow) + 4; ls++) {
      double c0 = 0, c1 = 0, tn = 1.0e300;
#pragma unroll
      for (int e = 0; e < 4 * NHC; e++) {
        const double jar = ejar[e], jd = ejd[e], te = ete[e];
        bool act;
        if (jd != 0.0) {
          act = jd < 0.0 ? te <= alpha : alpha < te;
          if (te > alpha && te < tn) tn = te;
        } else {
          act = jar < 0.0;
        }
        if (act) {
          const double De = (double)eD[e / 4];
          c0 += De * (jar + alpha * jd) * jd;
          c1 += De * jd * jd;
        }
      }
      {
        bool act;
        if (geq) {
          act = true;
        } else if (gjd != 0.0) {
          act = gjd < 0.0 ? gte <= alpha : alpha < gte;
          if (gte > alpha && gte < tn) tn = gte;
        } else {
          act = gjar < 0.0;
        }
        if (act) {
          c0 += (double)gD * (gjar + alpha * gjd) * gjd;
          c1 += (double)gD * gjd * gjd;
        }
      }
      c0 = wave_sum(c0) + dMa + alpha * dMd;
      c1 = wave_sum(c1) + dMd;
      tn = wave_min(tn);
      if (c0 >= 0.0) break;
      const double astar = alpha - c0 / c1;
      if (astar <= tn) {
        alpha = astar;
        break;
      }
      alpha = tn;
    }
    SPLITMARK(2, PH_CHSOLVE);
    // step: a, M (a - as) and the row products all move along dir (MuJoCo's Newton updates Jaref and Ma
    // the same way instead of recomputing them); the quadratic part of the cost follows exactly
    for (int i = LANE; i < nv; i += WAVE) {
      a[i] += alpha * (double)dir[i];
      Ma[i] += alpha * tmp[i];
    }
    for (int e = LANE; e < 3 * ncon; e += WAVE) {
      T* cr = w.cr() + CR_N * (e / 3);
      dslot(cr, CR_JA)[e % 3] += alpha * dslot(cr, CR_JD)[e % 3];
    }
    for (int r = LANE; r < nrow; r += WAVE) {
      T* rr = w.rr() + RR_N * r;
      *dslot(rr, RR_JAR) += alpha * *dslot(rr, RR_JD);
    }
    SYNC();
    qc += alpha * dMa + 0.5 * alpha * alpha * dMd;
    const double newcost = qc + rows_cost(w, ncon, nrow);
    SYNC();
    PMARK(PH_NLS);
    const double improvement = scale * (cost - newcost);
    cost = newcost;
    if (improvement < tol) {
      it++;
      break;
    }
  }
  if (it >= maxit && LANE == 0) ctr[2] += 1;
  if (LANE == 0) ctr[1] += it;
  // final constraint forces at a
  contact_f3(w, ncon);
  SYNC();
  if constexpr (scatter)
    gather_JtF_sc(M, w, ncon, nrow, w.fc(), tmp);
  else if constexpr (pc_scene<T, DIM>())
    gather_JtF_pc(M, w, ncon, nrow, w.fc(), tmp);
  else
    gather_JtF(M, w, ncon, nrow, w.fc(), false);
  SYNC();
  for (int i = LANE; i < nv; i += WAVE) w.fc()[i] = -w.fc()[i];
  for (int r = LANE; r < nrow; r += WAVE) {
    const int* ri = w.ri() + 4 * r;
    T* rr = w.rr() + RR_N * r;
    const double jar = *dslot(rr, RR_JAR);
    rr[RR_F] = (ri[2] == 0 || jar < 0.0) ? (T)(-(double)rr[RR_D] * jar) : T(0);
  }
  SYNC();
  PMARK(PH_NFINAL);
}

// ------------------------------------------------------------------------------------------------
// step2: actuation, smooth acceleration, constraint solve, implicitfast integration
// ------------------------------------------------------------------------------------------------
template <typename T, typename DIM>
__device__ __forceinline__ void smooth_acc(const Model<T>& M, const Ws<T, DIM>& w, int arena, bool actuation) {
  const DIM dm(M.dm);
  const int K = dm.K, nv = dm.nv;
  T* fa = w.fa();
  for (int i = LANE; i < nv; i += WAVE) fa[i] = T(0);
  SYNC();
  if (actuation) {
    // actuator forces in float64 (MuJoCo's gain * ctrl + bias, base_env.py:217 ctrl is float64): the PD
    // difference ctrl - length is exact, only the force is rounded to the build's precision
    for (int u = LANE; u < dm.nu; u += WAVE) {
      double c = w.ctrl()[u];
      const double lo = M.ctrlrange_d[2 * u], hi = M.ctrlrange_d[2 * u + 1];
      c = c < lo ? lo : (c > hi ? hi : c);
      // transmission (actuator length / velocity) from the float64 master state: the belt and arm dofs it
      // reads are the stage state's (the TaskManager's teleports only move cubes)
      double L, V;
      if (u == 0) {
        L = w.qd()[0];
        V = w.vd()[0];
      } else {
        const int qa = 1 + 7 * K + 9 * ((u - 1) / 8), va = 1 + 6 * K + 9 * ((u - 1) / 8), jj = (u - 1) % 8;
        if (jj < 7) {
          L = w.qd()[qa + jj];
          V = w.vd()[va + jj];
        } else {
          L = 0.5 * w.qd()[qa + 7] + 0.5 * w.qd()[qa + 8];
          V = 0.5 * w.vd()[va + 7] + 0.5 * w.vd()[va + 8];
        }
      }
      if (u == 0) {
        const double kv = (double)M.belt_kv;
        const T f = (T)(kv * c - kv * V);
        w.aforce()[u] = f;
        fa[0] = f;
      } else {
        int arm = (u - 1) / 8, j = (u - 1) % 8;
        int va = 1 + 6 * K + 9 * arm;
        if (j < 7) {
          const T f = (T)(2000.0 * c + -2000.0 * L + -200.0 * V);
          w.aforce()[u] = f;
          fa[va + j] = f;
        } else {
          double f = 100.0 * c + -100.0 * L + -10.0 * V;
          f = f < -100.0 ? -100.0 : (f > 100.0 ? 100.0 : f);
          w.aforce()[u] = (T)f;
          fa[va + 7] = (T)(0.5 * f);
          fa[va + 8] = (T)(0.5 * f);
        }
      }
    }
  }
  SYNC();
  for (int i = LANE; i < nv; i += WAVE) w.fs()[i] = w.pb()[i] + fa[i];
  SYNC();
  // qacc_smooth = M^-1 qfrc_smooth
  int a0 = 1 + 6 * K;
  for (int i = LANE; i < a0; i += WAVE) w.as()[i] = w.fs()[i] / Mdiag(M, w, i);
  if (LANE < dm.A) {
    // the arm block in float64 (both builds): with the gripper plates' small masses in it the block's Cholesky loses
    // ~4 digits in float (qacc_smooth of the plate dofs off by 2e-4 relative, tools/miss_probe.py), and qacc_smooth
    // sets the solver's optimum through the cost's M-norm term
    const T* Mb = w.Marm() + 81 * LANE;
    double Lp[45], x[9];
#pragma unroll
    for (int i = 0; i < 9; i++) {
#pragma unroll
      for (int j = 0; j <= i; j++) Lp[P9(i, j)] = (double)Mb[9 * i + j];
      x[i] = (double)w.fs()[a0 + 9 * LANE + i];
    }
    spd9_solve(Lp, x);
#pragma unroll
    for (int k = 0; k < 9; k++) w.as()[a0 + 9 * LANE + k] = (T)x[k];
  }
  SYNC();
}

#ifndef FM_INT_F64
#define FM_INT_F64 1  // the implicitfast acceleration solve in float64 in the fp32 build (the arm blocks' plates, as in smooth_acc)
#endif
template <typename T, typename DIM>
__device__ __forceinline__ void implicit_integrate(const Model<T>& M, const Ws<T, DIM>& w, int arena, bool actuation) {
  using IT = std::conditional_t<FM_INT_F64 != 0, double, T>;
  const DIM dm(M.dm);
  const int K = dm.K, nv = dm.nv;
  const IT dt = (IT)M.dt;
  T* q = w.q();
  T* v = w.v();
  IT* acc = (IT*)w.tmp();  // the solver's float64 scratch
  int a0 = 1 + 6 * K;
  // belt: M + dt*(kv + damping); cubes: M
  if (LANE == 0) {
    IT mb = (IT)M.belt_mass + dt * (IT)M.belt_damp + (actuation ? dt * (IT)M.belt_kv : IT(0));
    acc[0] = ((IT)w.fs()[0] + (IT)w.fc()[0]) / mb;
  }
  // cubes: the smooth force is gravity alone (stage(): (0, 0, -m g, 0, 0, 0)), so the acceleration is
  // qfrc_constraint / m - g with g in float64 -- through the float force -m g it is off by a float rounding of g, which
  // 0.4 s of free fall turn into more than a float32 ulp of the velocity the reference's obs hold (tests/
  // test_physics_pins.py)
  for (int i = 1 + LANE; i < a0; i += WAVE) {
    IT ai = (IT)w.fc()[i] / (IT)Mdiag(M, w, i);
    if ((i - 1) % 6 == 2) ai -= (IT)M.grav_d;
    acc[i] = ai;
  }
  if (LANE < dm.A) {
    const T* Mb = w.Marm() + 81 * LANE;
    IT Lp[45], x[9];
#pragma unroll
    for (int i = 0; i < 9; i++) {
#pragma unroll
      for (int j = 0; j <= i; j++) Lp[P9(i, j)] = (IT)Mb[9 * i + j];
      x[i] = (IT)w.fs()[a0 + 9 * LANE + i] + (IT)w.fc()[a0 + 9 * LANE + i];
    }
    if (actuation) {
#pragma unroll
      for (int j = 0; j < 7; j++) Lp[P9(j, j)] += dt * IT(200);
      T fg = w.aforce()[1 + 8 * LANE + 7];
      if (fg > T(-100) && fg < T(100)) {
        IT d = dt * IT(10) * IT(0.25);
        Lp[P9(7, 7)] += d;
        Lp[P9(8, 8)] += d;
        Lp[P9(8, 7)] += d;
      }
    }
    spd9_solve(Lp, x);
#pragma unroll
    for (int k = 0; k < 9; k++) acc[a0 + 9 * LANE + k] = x[k];
  }
  SYNC();
  // velocities and positions accumulate in the float64 master state (mj_integratePos); the float copies
  // the fp32 physics reads are refreshed from it
  double* qd = w.qd();
  double* vd = w.vd();
  const double h = 0.001;  // model.opt.timestep (base_env.py:207-210), exact in float64
  for (int i = LANE; i < nv; i += WAVE) {
    vd[i] += h * (double)acc[i];
    if constexpr (sizeof(T) != 8) v[i] = (T)vd[i];
  }
  SYNC();
  if (LANE == 0) {
    qd[0] += h * vd[0];
    if constexpr (sizeof(T) != 8) q[0] = (T)qd[0];
  }
  for (int k = LANE; k < K; k += WAVE) {
    double* qq = qd + 1 + 7 * k;
    const double* vv = vd + 1 + 6 * k;
    for (int c = 0; c < 3; c++) qq[c] += h * vv[c];
    double ax[3] = {vv[3], vv[4], vv[5]};
    double nrm = sqrt(dot3(ax, ax));
    if (nrm < 1e-15) {
      ax[0] = 1;
      ax[1] = ax[2] = 0;
    } else {
      for (int c = 0; c < 3; c++) ax[c] /= nrm;
    }
    double ang = h * nrm;
    double qr[4];
    if (ang == 0.0) {
      qr[0] = 1;
      qr[1] = qr[2] = qr[3] = 0;
    } else {
      double s = sin(ang * 0.5);
      qr[0] = cos(ang * 0.5);
      qr[1] = ax[0] * s;
      qr[2] = ax[1] * s;
      qr[3] = ax[2] * s;
    }
    double qu[4] = {qq[3], qq[4], qq[5], qq[6]};
    double n = sqrt(qu[0] * qu[0] + qu[1] * qu[1] + qu[2] * qu[2] + qu[3] * qu[3]);
    if (n < 1e-15) {
      qu[0] = 1;
      qu[1] = qu[2] = qu[3] = 0;
    } else if (fabs(n - 1.0) > 1e-15) {
      for (int c = 0; c < 4; c++) qu[c] /= n;
    }
    qq[3] = qu[0] * qr[0] - qu[1] * qr[1] - qu[2] * qr[2] - qu[3] * qr[3];
    qq[4] = qu[0] * qr[1] + qu[1] * qr[0] + qu[2] * qr[3] - qu[3] * qr[2];
    qq[5] = qu[0] * qr[2] - qu[1] * qr[3] + qu[2] * qr[0] + qu[3] * qr[1];
    qq[6] = qu[0] * qr[3] + qu[1] * qr[2] - qu[2] * qr[1] + qu[3] * qr[0];
    if constexpr (sizeof(T) != 8)
      for (int c = 0; c < 7; c++) q[1 + 7 * k + c] = (T)(c == 2 ? qq[c] - zshift<T>() : qq[c]);
  }
  int qa0 = 1 + 7 * K;
  for (int i = LANE; i < 9 * dm.A; i += WAVE) {
    qd[qa0 + i] += h * vd[a0 + i];
    if constexpr (sizeof(T) != 8) q[qa0 + i] = (T)qd[qa0 + i];
  }
  SYNC();
  PMARK(PH_INT);
}

// ------------------------------------------------------------------------------------------------
// task layer (lane 0 unless noted; float64 like the reference's Python)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t pcg_next(uint64_t* st) {
  const uint64_t MH = 0x2360ED051FC65DA4ULL, ML = 0x4385DF649FCCF645ULL;
  uint64_t sh = st[0], sl = st[1];
  uint64_t lo = sl * ML;
  uint64_t hi = __umul64hi(sl, ML) + sl * MH + sh * ML;
  uint64_t lo2 = lo + st[3];
  uint64_t carry = lo2 < lo ? 1ull : 0ull;
  uint64_t hi2 = hi + st[2] + carry;
  st[0] = hi2;
  st[1] = lo2;
  uint64_t x = hi2 ^ lo2;
  unsigned rot = (unsigned)(hi2 >> 58);
  return (x >> rot) | (x << ((-rot) & 63));
}
__device__ __forceinline__ double pcg_double(uint64_t* st) {
  return (double)(pcg_next(st) >> 11) * (1.0 / 9007199254740992.0);
}

template <typename DD>
__device__ __forceinline__ void hide_cube(const DD& dm, double* q, double* v, int32_t* ti, int obj) {
  ti[dm.K + ti[2 * dm.K + I_NOUT]] = obj;
  ti[2 * dm.K + I_NOUT]++;
  double* qq = q + 1 + 7 * obj;
  qq[0] = 4.0 + 1.0;
  qq[1] = ti[2 * dm.K + I_HIDDEN] * 0.2;
  qq[2] = 1.0;
  qq[3] = 1.0;
  qq[4] = qq[5] = qq[6] = 0.0;
  double* vv = v + 1 + 6 * obj;
  for (int k = 0; k < 6; k++) vv[k] = 0.0;
  ti[2 * dm.K + I_HIDDEN]++;
}

__device__ __forceinline__ void pop_at(int32_t* list, int32_t* n, int idx) {
  for (int i = idx; i < *n - 1; i++) list[i] = list[i + 1];
  (*n)--;
  list[*n] = -1;
}

// TaskManager.reset (task_utils.py:146-156) + BaseEnv.reset_sim bits (base_env.py:184-190)
template <typename T, typename DIM>
__device__ __forceinline__ void task_reset(const Model<T>& M, double* q, double* v, int32_t* ti, double* td, double* ctrl) {
  const DIM dm(M.dm);
  const int K = dm.K;
  for (int k = 0; k < K; k++) {
    double* qq = q + 1 + 7 * k;
    qq[0] = 4.0;
    qq[1] = 0.0 + k * 0.2;
    qq[2] = 1.0;
    qq[3] = 1.0;
    qq[4] = qq[5] = qq[6] = 0.0;
    double* vv = v + 1 + 6 * k;
    for (int c = 0; c < 6; c++) vv[c] = 0.0;
    ti[K + k] = k;
    ti[k] = -1;
  }
  int32_t* ts = ti + 2 * K;
  ts[I_NIN] = 0;
  ts[I_NOUT] = K;
  ts[I_STEP] = ts[I_SINCE] = ts[I_FAIL] = ts[I_HIDDEN] = 0;
  ts[I_S0] = ts[I_S1] = 0;
  ts[I_LS0] = ts[I_LS1] = 0;
  for (int u = 0; u < dm.nu; u++) ctrl[u] = 0.0;
  // FactoryManipulationEnv.reset -> IKPolicy.reset -> idle_ctrl (environments.py:243-244, ik_policy.py:120-127);
  // ignore maps, move_start and PauseIKToggleEnv.last_arm_actions persist
  for (int i = 0; i < dm.A; i++) {
    const IkArm p = ik_arm(dm, ti, td, i);
    p.s[0] = IK_IDLE;
    p.s[1] = 0;
    p.s[2] = -1;
    for (int j = 0; j < 8; j++) p.last_ctrl()[j] = IK_DEFAULT_POSE[j];
  }
  td[0] = M.spawn_freq0;  // spawn_freq
  td[1] = M.init_speed;   // conveyor speed
  td[2] = 0.0;            // play_time
}

template <typename T, typename DIM>
__device__ __forceinline__ int task_step(const Model<T>& M, double* q, double* v, int32_t* ti, double* td, uint64_t* rng, int64_t* ctr,
                                         int* orig) {
  const DIM dm(M.dm);
  const int K = dm.K;
  int32_t* ins = ti;
  int32_t* outs = ti + K;
  int32_t* ts = ti + 2 * K;
  int spawn_steps = (int)(1.0 / (0.1 * td[0]));
  if (ts[I_STEP] == 0 || ts[I_SINCE] >= spawn_steps) {
    if (ts[I_NOUT] > 0) {
      int obj = outs[0];
      pop_at(outs, &ts[I_NOUT], 0);
      double* qq = q + 1 + 7 * obj;
      qq[0] = 0.0;
      qq[1] = 1.0;
      qq[2] = 2.0;
      for (int k = 0; k < 4; k++) qq[3 + k] = 0.0 + 1.0 * pcg_double(rng);
      ins[ts[I_NIN]++] = obj;
    }
    ts[I_SINCE] = 0;
  }
  if (ts[I_NIN] > 0) {
    // out of bounds (task_utils.py:84-94): popping index i only shifts the entries above i, which the
    // descending walk has already visited, so each test reads the position it would have read up front
    for (int i = ts[I_NIN] - 1; i >= 0; i--) {
      const double* qq = q + 1 + 7 * ins[i];
      const double x = qq[0], y = qq[1], z = qq[2];
      if (!(fabs(x) > 1.2 || y < -1.5 || z < 0.9)) continue;
      int obj = ins[i];
      pop_at(ins, &ts[I_NIN], i);
      hide_cube(dm, q, v, ti, obj);
      ts[I_FAIL]++;
    }
    if (ts[I_NIN] > 0) {
      // buckets (task_utils.py:99-113): positions are captured once for both buckets (obj_pos), indices
      // into the shrinking list are reused.  orig[] keeps the captured order; a cube popped for bucket 0
      // is parked at x = 5 and lay inside bucket 0 before, so its current and captured positions both
      // fail bucket 1's test
      const int n2 = ts[I_NIN];
      for (int i = 0; i < n2; i++) orig[i] = ins[i];
      for (int b = 0; b < 2; b++) {
        double bx = b == 0 ? M.bucket_x0 : M.bucket_x1, by = M.bucket_y, bz = M.bucket_z;
        for (int i = n2 - 1; i >= 0; i--) {
          const double* qq = q + 1 + 7 * orig[i];
          bool in_x = fabs(qq[0] - bx) <= 0.6 * 0.29;
          bool in_y = fabs(qq[1] - by) <= 0.6 * 0.29;
          bool in_z = qq[2] - bz - 0.02 / 2 <= 0.07;
          if (!(in_x && in_y && in_z)) continue;
          if (i >= ts[I_NIN]) {  // reference: IndexError (task_utils.py:103-113 index reuse)
            ctr[3] += 1;
            continue;
          }
          int obj = ins[i];
          pop_at(ins, &ts[I_NIN], i);
          hide_cube(dm, q, v, ti, obj);
          ts[b == 0 ? I_S0 : I_S1]++;
        }
      }
    }
  }
  ts[I_STEP]++;
  ts[I_SINCE]++;
  return ts[I_FAIL] > 0;
}

// observation row (environments.py:55-82 over base_env.py:149-175): arms (q[8], qd[8], ctrl[8]) then
// in-scene cubes sorted by x (stable), zero padded: poses K x 7, velocities K x 6
// lane 0: TaskManager.step, BaseEnv.step_sim bookkeeping (base_env.py:266-270), progress / score reward
// (environments.py:129-149, 342-383), Monitor episode return; results in w.scal()
template <typename T, typename DIM>
__device__ __forceinline__ void task_tail(const Model<T>& M, const Ws<T, DIM>& w, int32_t* ti, double* td, uint64_t* rng,
                                       int64_t* ctr, const float* act) {
  const DIM dm(M.dm);
  const int A = dm.A, K = dm.K;
  double* sc = w.scal();
  int fail = task_step<T, DIM>(M, w.qd(), w.vd(), ti, td, rng, ctr, w.sortidx());
  double dt_env = 0.001 * dm.frame_skip;
  td[2] += dt_env;
  td[1] += M.accel * dt_env;
  td[0] *= M.spawn_inc;
  int32_t* ts = ti + 2 * K;
  int sd = (ts[I_S0] + ts[I_S1]) - (ts[I_LS0] + ts[I_LS1]);
  double rew;
  if (env_score_reward(M.env_class)) {
    rew = sd;
  } else {
    double gc = 0, bc = 0;
    double* lg = td + 3;
    double* lb = td + 3 + A;
    for (int i = 0; i < A; i++) {
      const T* gp = w.site() + 3 * i;
      double best = 0;
      int bi = -1;
      const int32_t* ign = ik_arm(dm, ti, td, i).s + 3;  // candidates skip the IK policy's ignore map
      for (int c = 0; c < ts[I_NIN]; c++) {
        bool skip = false;
        for (int o = 0; o < A; o++) skip |= ign[o] == ti[c];
        if (skip) continue;
        const double* qq = w.qd() + 1 + 7 * ti[c];
        double dx = qq[0] - (double)gp[0], dy = qq[1] - (double)gp[1], dz = qq[2] - ((double)gp[2] + zshift<T>());
        double dd = sqrt(dx * dx + dy * dy + dz * dz);
        if (bi < 0 || dd < best) {
          best = dd;
          bi = c;
        }
      }
      if (bi < 0) continue;  // no candidate: (None, last distance, 0) (environments.py:306-307, 334-335)
      gc += lg[i] - best;
      lg[i] = best;
      // closest cube to this arm's bucket
      const double* qq = w.qd() + 1 + 7 * ti[bi];
      double bx = (i % 2) == 0 ? M.bucket_x0 : M.bucket_x1;
      double dx = qq[0] - bx, dy = qq[1] - M.bucket_y, dz = qq[2] - M.bucket_z;
      double db = sqrt(dx * dx + dy * dy + dz * dz);
      bc += lb[i] - db;
      lb[i] = db;
    }
    float ss = 0.0f;
    for (int i = 0; i < dm.act_dim; i++)
      if (i % 8 != 7) ss += act[i] * act[i];
    float an = expf(-sqrtf(ss));
    double prog = M.base_reward + M.w_grip * gc + M.w_bucket * bc + M.w_action * (double)an;
    rew = sd > 0 ? (double)sd : prog;
  }
  ts[I_LS0] = ts[I_S0];
  ts[I_LS1] = ts[I_S1];
  sc[0] = rew;
  sc[1] = (fail || sc[3] != 0.0) ? 1.0 : 0.0;
  sc[2] = fail ? 1.0 : 0.0;
  td[3 + 2 * A] += rew;  // Monitor episode return
  ts[I_EPLEN]++;
}

template <typename T, typename DIM>
// obs: float32 rows, or float64 rows when M.obs64 (the toggle classes' observation is float64 in the reference: the
// float32 state block concatenated with the float64 IK proposals, environments.py:576 -- numpy widens the float32
// columns exactly, and the proposals keep all their bits)
__device__ __forceinline__ void write_obs(const Model<T>& M, const Ws<T, DIM>& w, int32_t* ti, double* td, float* obs) {
  const DIM dm(M.dm);
  const int A = dm.A, K = dm.K;
  const double* q = w.qd();  // float64 state cast to float32 (base_env.py:92-109)
  const double* v = w.vd();
  int* idx = w.sortidx();
  if (LANE == 0) {
    int n = ti[2 * K + I_NIN];
    for (int i = 0; i < n; i++) idx[i] = ti[i];
    for (int i = 1; i < n; i++) {
      int vi = idx[i];
      double x = q[1 + 7 * vi];
      int j = i - 1;
      while (j >= 0 && q[1 + 7 * idx[j]] > x) {
        idx[j + 1] = idx[j];
        j--;
      }
      idx[j + 1] = vi;
    }
  }
  SYNC();
  int n = ti[2 * K + I_NIN];
  for (int e = LANE; e < dm.obs_dim; e += WAVE) {
    float val;
    if (e < 24 * A) {
      int arm = e / 24, r = e % 24;
      if (r < 8)
        val = (float)q[1 + 7 * K + 9 * arm + r];
      else if (r < 16)
        val = (float)v[1 + 6 * K + 9 * arm + r - 8];
      else
        val = (float)w.ctrl()[1 + 8 * arm + r - 16];
    } else if (e < 24 * A + 7 * K) {
      int k = (e - 24 * A) / 7, c = (e - 24 * A) % 7;
      val = k < n ? (float)q[1 + 7 * idx[k] + c] : 0.0f;
    } else if (e < 24 * A + 13 * K) {
      int k = (e - 24 * A - 7 * K) / 6, c = (e - 24 * A - 7 * K) % 6;
      val = k < n ? (float)v[1 + 6 * idx[k] + c] : 0.0f;
    } else {  // IKTogglingEnv: the IK proposals (environments.py:576)
      const int r = e - 24 * A - 13 * K;
      const double pv = ik_arm(dm, ti, td, r / 8).ik_actions()[r % 8];
      if (M.obs64) {
        ((double*)obs)[e] = pv;
        continue;
      }
      val = (float)pv;
    }
    if (M.obs64)
      ((double*)obs)[e] = (double)val;
    else
      obs[e] = val;
  }
}

// ------------------------------------------------------------------------------------------------
// IK base policy of one arena (fm_ik.hpp): FactoryManipulationEnv._compose_control
// ------------------------------------------------------------------------------------------------
// every arm's proposal (IKPolicy.act() clipped to actuator_ctrlrange[1:9]) into prop[8A], FSM state / ignore
// maps / last_ctrl / move_start updated in the arena's IK block.  Reads the float64 master state; uses the
// phase-local H region as scratch (free outside a substep's stage / solve).  Not inlined (it runs a few times
// per env-step): every pointer it receives is global or LDS -- none into a caller's private frame, which a
// callee could only reach through the flat scratch aperture.  Every pointer parameter carries its address space
// (scene tables constant, master state LDS, task records global, scratch SAS = LDS or the arena's global block):
// through a generic parameter each access would be a FLAT instruction.
template <int SAS>
__device__ __noinline__ void ik_compose_raw(const double FM_AS(4)* arm_base_g, const double FM_AS(4)* ctrlrange_g,
                                            IkTiming tm, int A, int K, const double FM_AS(3)* qd_, const double FM_AS(3)* vd_,
                                            int32_t FM_AS(1)* ti_, double FM_AS(1)* td_, int int_base, int dbl_base,
                                            double FM_AS(SAS)* scr_, double FM_AS(SAS)* prop_) {
  const double* arm_base_w = (const double*)arm_base_g;
  const double* ctrlrange_d = (const double*)ctrlrange_g;
  const double* qd = (const double*)qd_;
  const double* vd = (const double*)vd_;
  int32_t* ti = (int32_t*)ti_;
  double* td = (double*)td_;
  double* scr = (double*)scr_;
  double* prop = (double*)prop_;
  // scr per arm (24): grip 3 | tpos 3 | tquat 4 | need | close | pad 2 | q 7 | pad 3
  struct D {
    int A, K;
  } dm{A, K};
  (void)int_base;
  (void)dbl_base;
  if (LANE < A) {
    double q[7], sR[9];
    for (int j = 0; j < 7; j++) q[j] = qd[1 + 7 * K + 9 * LANE + j];
    double sp[3];
    ik_fk(arm_base_w + 12 * LANE, q, sp, sR, nullptr, nullptr);
    for (int k = 0; k < 3; k++) scr[24 * LANE + k] = sp[k];
  }
  SYNC();
  if (LANE == 0) {  // act() in arm order: each arm's target selection sees the ignore maps written before it
    const int n_in = ti[2 * K + I_NIN];
    for (int i = 0; i < A; i++) {
      const IkArm p = ik_arm(dm, ti, td, i);
      double* sc = scr + 24 * i;
      int cl = 0;
      double g[3] = {sc[0], sc[1], sc[2]}, tp[3] = {0, 0, 0}, tq[4] = {1, 0, 0, 0};
      sc[10] = ik_plan(A, i, p, ti, n_in, qd, vd, K, g, arm_base_w + 12 * i, tm, tp, tq, &cl);
      for (int k = 0; k < 3; k++) sc[3 + k] = tp[k];
      for (int k = 0; k < 4; k++) sc[6 + k] = tq[k];
      sc[11] = cl;
      const int tgt = p.s[2];
      for (int j = 0; j < A; j++)
        if (j != i) ik_arm(dm, ti, td, j).s[3 + i] = tgt;  // ik_policies[j].ignore(target, owner i)
    }
  }
  FULL_SYNC();
  if (LANE < A) {
    const IkArm p = ik_arm(dm, ti, td, LANE);
    double* sc = scr + 24 * LANE;
    double ctrl[8];
    bool ok = false;
    if (sc[10] != 0.0) {
      double* q = sc + 14;  // the arm's private copy of its hinges (qpos_from_site_pose, inplace=False), in LDS
      for (int j = 0; j < 7; j++) q[j] = qd[1 + 7 * K + 9 * LANE + j];
      ok = ik_solve<SAS>(arm_base_g + 12 * LANE, scr_ + 24 * LANE + 14, scr_ + 24 * LANE + 3, scr_ + 24 * LANE + 6) != 0;
      if (ok) {
        for (int j = 0; j < 7; j++) ctrl[j] = q[j];
        ctrl[7] = sc[11] != 0.0 ? 0.0 : 2.0;
        for (int j = 0; j < 8; j++) p.last_ctrl()[j] = ctrl[j];
      }
    }
    if (!ok)
      for (int j = 0; j < 8; j++) ctrl[j] = p.last_ctrl()[j];
    for (int j = 0; j < 8; j++) {
      const double lo = ctrlrange_d[2 * (1 + j)], hi = ctrlrange_d[2 * (1 + j) + 1];
      prop[8 * LANE + j] = ctrl[j] < lo ? lo : (ctrl[j] > hi ? hi : ctrl[j]);
    }
  }
  FULL_SYNC();
}

template <typename T, typename DIM>
__device__ __forceinline__ void ik_compose(const Model<T>& M, const Ws<T, DIM>& w, int32_t* ti, double* td, double* prop) {
  const DIM dm(M.dm);
  constexpr int SAS = DIM::spill ? AS_GLOBAL : AS_LDS;  // where w.H() (the compose scratch) lives
  ik_compose_raw<SAS>((const double FM_AS(4)*)(const double*)M.arm_base_w,
                      (const double FM_AS(4)*)(const double*)M.ctrlrange_d, M.ik_time, dm.A, dm.K,
                      (const double FM_AS(3)*)w.qd(), (const double FM_AS(3)*)w.vd(), (int32_t FM_AS(1)*)ti,
                      (double FM_AS(1)*)td, 0, 0, (double FM_AS(SAS)*)w.H(), (double FM_AS(SAS)*)prop);
}

// IKTogglingEnv._process_observation (environments.py:560-577): fresh proposals, kept for the next step's
// composition and appended to the observation
template <typename T, typename DIM>
__device__ __forceinline__ void ik_proposals(const Model<T>& M, const Ws<T, DIM>& w, int32_t* ti, double* td) {
  const DIM dm(M.dm);
  double* prop = (double*)w.H() + 24 * dm.A;
  ik_compose(M, w, ti, td, prop);
  for (int e = LANE; e < 8 * dm.A; e += WAVE) ik_arm(dm, ti, td, e / 8).ik_actions()[e % 8] = prop[e];
  FULL_SYNC();
}

// _process_action of one entry (environments.py:84-102): float32 tanh, float64 range
template <typename T>
__device__ __forceinline__ double process_action(const Model<T>& M, float a, int j) {
  const float th = (float)tanh((double)a);  // correctly rounded float32 tanh (np.tanh on float32)
  const float s = (th + 1.0f) * 0.5f;
  const double lo = M.ctrlrange_d[2 * (1 + j)], hi = M.ctrlrange_d[2 * (1 + j) + 1];
  return lo + (double)s * (hi - lo);
}

// ------------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------------
// float copies of the float64 master state (fp32 build; in fp64 they are the same arrays)
template <typename T, typename DIM>
__device__ __forceinline__ void refresh_copies(const Model<T>& M, const Ws<T, DIM>& w) {
  if constexpr (sizeof(T) != 8) {
    const DIM dm(M.dm);
    for (int i = LANE; i < dm.nq; i += WAVE) {
      const bool cz = i >= 1 && i < 1 + 7 * dm.K && (i - 1) % 7 == 2;  // cube z in the kernel frame
      w.q()[i] = (T)(cz ? w.qd()[i] - zshift<T>() : w.qd()[i]);
    }
    for (int i = LANE; i < dm.nv; i += WAVE) w.v()[i] = (T)w.vd()[i];
  }
}

template <typename T, typename DIM>
__device__ __forceinline__ void load_state(const Model<T>& M, const State<T>& S, const Ws<T, DIM>& w, int arena, bool stage_copy) {
  const DIM dm(M.dm);
  const double* ph = S.phys + (size_t)arena * dm.phys_stride;
  const double* src_q = ph + (stage_copy ? dm.nq + dm.nv : 0);
  const double* src_v = ph + dm.nq + (stage_copy ? dm.nq + dm.nv : 0);
  for (int i = LANE; i < dm.nq; i += WAVE) w.qd()[i] = src_q[i];
  for (int i = LANE; i < dm.nv; i += WAVE) w.vd()[i] = src_v[i];
  refresh_copies(M, w);
}

// per-launch LDS setup: geom / collision-body tables, static geom centres, body bounds, cube sizes
template <typename T, typename DIM>
__device__ __forceinline__ void init_arena(const Model<T>& M, const Ws<T, DIM>& w, int arena) {
  const DIM dm(M.dm);
  for (int g = LANE; g < dm.ngc; g += WAVE) {
    w.ginfo()[g] = M.ginfo[g];
    w.cbg()[g] = M.cbg[g];
  }
  for (int i = LANE; i < 4 * dm.ncb; i += WAVE) w.cbi()[i] = M.cbi[i];
  for (int i = LANE; i < 4 * dm.K; i += WAVE) w.cube()[i] = M.cube[(size_t)arena * dm.K * 4 + i];
}

// physics.reset() + TaskManager.reset() + after_reset forward (actuation disabled) -> warmstart
template <typename T, typename DIM>
__device__ __forceinline__ void arena_reset(const Model<T>& M, const Ws<T, DIM>& w, int arena, int32_t* ti, double* td, int64_t* ctr) {
  const DIM dm(M.dm);
  double* q = w.qd();
  double* v = w.vd();
  for (int i = LANE; i < dm.nq; i += WAVE) q[i] = 0.0;
  for (int i = LANE; i < dm.nv; i += WAVE) {
    v[i] = 0.0;
    w.a()[i] = 0.0;
  }
  SYNC();
  if (LANE == 0) task_reset<T, DIM>(M, q, v, ti, td, w.ctrl());
  FULL_SYNC();
  SYNC();
  refresh_copies(M, w);
  SYNC();
  stage(M, w, arena, ctr);
  smooth_acc(M, w, arena, false);
  if (w.misc()[MISC_NCON] + w.misc()[MISC_NROW] > 0) {
    newton(M, w, arena, ctr);
  } else {
    for (int i = LANE; i < dm.nv; i += WAVE) w.a()[i] = w.as()[i];
    SYNC();
  }
}

template <typename T, typename DIM>
__device__ __forceinline__ void store_state(const Model<T>& M, const State<T>& S, const Ws<T, DIM>& w, int arena) {
  const DIM dm(M.dm);
  double* ph = S.phys + (size_t)arena * dm.phys_stride;
  for (int i = LANE; i < dm.nq; i += WAVE) ph[i] = w.qd()[i];
  for (int i = LANE; i < dm.nv; i += WAVE) ph[dm.nq + i] = w.vd()[i];
  for (int i = LANE; i < dm.nv; i += WAVE) ph[2 * dm.nq + 2 * dm.nv + i] = w.a()[i];
  double* db = S.dbl + (size_t)arena * dm.dbl_stride;
  for (int u = LANE; u < dm.nu; u += WAVE) db[u] = w.ctrl()[u];
}

template <typename T, typename DIM>
__global__ void __launch_bounds__(64) reset_kernel(Model<T> M, State<T> S, Lay L, float* obs, const uint8_t* mask) {
  FM_SMEM_DECL(smem);
  const int arena = blockIdx.x;
  const DIM dm(M.dm);
  if (mask && !mask[arena]) return;
  Ws<T, DIM> w{lds_base(smem), &L, spill_base<DIM>(S, arena)};
  int32_t* ti = S.ints + (size_t)arena * dm.int_stride;
  double* td = S.dbl + (size_t)arena * dm.dbl_stride + dm.nu;
  int64_t* ctr = S.counters + FM_NCTR * (size_t)arena;
  init_arena(M, w, arena);
  SYNC();
  arena_reset(M, w, arena, ti, td, ctr);
  // stage state = reset state
  double* ph = S.phys + (size_t)arena * dm.phys_stride;
  for (int i = LANE; i < dm.nq; i += WAVE) ph[dm.nq + dm.nv + i] = w.qd()[i];
  for (int i = LANE; i < dm.nv; i += WAVE) ph[2 * dm.nq + dm.nv + i] = w.vd()[i];
  store_state(M, S, w, arena);
  if (LANE == 0) {
    td[2 * dm.A + 3] = 0.0;  // episode return
    ti[2 * dm.K + I_EPLEN] = 0;
  }
  SYNC();
  FULL_SYNC();
  if (env_toggle(M.env_class)) ik_proposals(M, w, ti, td);  // reset()'s observation (environments.py:245)
  if (obs) write_obs(M, w, ti, td, obs + (size_t)arena * dm.obs_dim * (M.obs64 ? 2 : 1));
}

// IK: the env class may compose IK proposals (every class but AllFullRL); the AllFullRL instantiation carries
// none of the IK code (and none of its register demand)
#ifndef FM_WAVES_PER_EU
#define FM_WAVES_PER_EU 0  // the minimum waves per SIMD the register allocation must allow (0: no constraint)
#endif
#ifndef FM_WAVES_PER_EU_IK
#define FM_WAVES_PER_EU_IK FM_WAVES_PER_EU  // the same for the IK-class instantiation (step_kernel<T, DIM, true>)
#endif
#if defined(FM_HOST_SIMT) || (FM_WAVES_PER_EU == 0 && FM_WAVES_PER_EU_IK == 0)
#define FM_STEP_ATTR
#else
#define FM_STEP_ATTR                                                                                    \
  __attribute__((amdgpu_waves_per_eu(IK ? (FM_WAVES_PER_EU_IK > 0 ? FM_WAVES_PER_EU_IK : 1)           \
                                        : (FM_WAVES_PER_EU > 0 ? FM_WAVES_PER_EU : 1))))
#endif
// one env-step of one arena on the calling wave (the body of step_kernel)
template <typename T, typename DIM, bool IK>
__device__ __forceinline__ void step_arena(char* smem, const int arena) {
  // All launch parameters are read through an opaque pointer to the kernarg segment at each use, so the
  // compiler cannot hoist the ~50 scalar values out of the substep loop and run out of SGPRs.
  // The pointer stays in the constant address space (scalar loads, no FLAT instructions).
#define M (kparams<StepParams<T>>().M)
#define S (kparams<StepParams<T>>().S)
#define io (kparams<StepParams<T>>().io)
#define L (kparams<StepParams<T>>().L)
  const unsigned long long t_begin = wall_clock64();
  const DIM dm(M.dm);
  const int A = dm.A, K = dm.K, nu = dm.nu;
  // abandon the env-step at a stage above the contact capacity (benchmark scene with a rerun list): the arena's
  // records stay as the step found them and the wide kernel (FixedDims<2, 4, true>) steps it again after this launch
  constexpr bool can_abandon = DIM::fixed && !DIM::rerun && DIM::MAXC == WAVE;
  // a fresh opaque LDS base per use: workspace addresses are recomputed inside each phase instead of
  // being hoisted out of the substep loop (which would keep every phase's addresses live everywhere)
#define w (Ws<T, DIM>{lds_base(smem), &L, spill_base<DIM>(S, arena)})
  if (M.prof && LANE < FM_NPROF) w.prof()[LANE] = LANE == PH_LAST ? wall_clock64() : 0ull;
  if (LANE == 0) {
    w.misc()[MISC_CSUM] = 0;
    w.misc()[MISC_CMAX] = 0;
    w.misc()[MISC_MC_OK] = 0;  // the cached midphase list is rebuilt at the first substep of every launch
  }
  // the arena's record addresses, recomputed at each use from an opaque copy of the arena index (hoisted, the 64-bit
  // offsets stay live across the substep loop and spill)
#define ARENA_ (::fm::opaque_uniform(arena))
#define ti (S.ints + (size_t)ARENA_ * dm.int_stride)
#define td (S.dbl + (size_t)ARENA_ * dm.dbl_stride + nu)  // spawn_freq, speed, play_time, grip[A], bucket[A], ret
#define rng (S.rng + 4 * (size_t)ARENA_)
#define ctr (S.counters + FM_NCTR * (size_t)ARENA_)
#define act (io.actions + (size_t)ARENA_ * dm.act_dim)
  // the wide rerun kernel resumes an env-step the 64-contact kernel abandoned after substep 0 (State::resume): the
  // IK compose, the clipped control target and substeps 0 .. t0-1 are already done (their task-record writes stand)
  int t0 = 0;
  if constexpr (DIM::rerun) {
    const double* const rs = S.resume;
    if (rs) t0 = (int)rs[(size_t)ARENA_ * resume_stride(dm.nq, dm.nv, nu)];
  }
  if constexpr (IK && (can_abandon || DIM::rerun)) {
    // the IK compose below writes the FSM / last-action blocks of the task records: keep the step's starting
    // records for a rerun (the rerun restores them first)
    char* const bk = S.bak;
    if (bk && t0 == 0) {
      double* bd = (double*)(bk + (size_t)arena * (8 * dm.dbl_stride + 4 * dm.int_stride));
      int32_t* bi = (int32_t*)(bd + dm.dbl_stride);
      double* dd = S.dbl + (size_t)arena * dm.dbl_stride;
      for (int i = LANE; i < dm.dbl_stride; i += WAVE) {
        if (DIM::rerun)
          dd[i] = bd[i];
        else
          bd[i] = dd[i];
      }
      for (int i = LANE; i < dm.int_stride; i += WAVE) {
        if (DIM::rerun)
          ti[i] = bi[i];
        else
          bi[i] = ti[i];
      }
      FULL_SYNC();
    }
  }
  if constexpr (DIM::rerun) {
    if (LANE == 0) ctr[8] += 1;
  }
  // ---- ctrl_target (double) and the env class's control (environments.py _compose_control, base_env.py:255-262)
#define ctrl_ (w.ctrl())
  const double* dsrc = S.dbl + (size_t)arena * dm.dbl_stride;
  for (int u = LANE; u < nu; u += WAVE) ctrl_[u] = dsrc[u];
  const double speed0 = td[1];
  const int ec = M.env_class;
  double* prop = (double*)w.H() + 24 * A;  // IK proposals of this step's compose (phase-local scratch)
  if (t0 == 0) {
  if (IK && env_ik_at_step(ec)) {  // IKPolicy.act() on the state the step starts from
    load_state(M, S, w, arena, false);
    SYNC();
    ik_compose(M, w, ti, td, prop);
  }
#define uctl_ (w.uctl())
  for (int u = LANE; u < nu; u += WAVE) {
    double c;
    if (u == 0) {
      c = speed0;
    } else {
      const int arm = (u - 1) / 8, j = (u - 1) % 8;
      switch (IK ? ec : FM_ENV_ALLFULLRL_PROGRESS) {
        case FM_ENV_ALLFULLRL_PROGRESS:
          c = process_action(M, act[u - 1], j);
          break;
        case FM_ENV_SINGLEFULLRL_PROGRESS:
          c = arm == 0 ? process_action(M, act[j], j) : prop[u - 1];
          break;
        case FM_ENV_SINGLEDELTA_PROGRESS:
          c = prop[u - 1];
          if (arm == 0 && ik_arm(dm, ti, td, 0).s[0] != IK_IDLE) c += 0.5 * process_action(M, act[j], j);
          break;
        case FM_ENV_ALLDELTA_PROGRESS:
          c = prop[u - 1];
          if (ik_arm(dm, ti, td, arm).s[0] != IK_IDLE) c += 0.5 * process_action(M, act[u - 1], j);
          break;
        case FM_ENV_PAUSE_IK_TOGGLE: {
          const IkArm p = ik_arm(dm, ti, td, arm);
          c = act[arm] == 1.0f ? p.ik_actions()[j] : p.pause_last()[j];
          p.pause_last()[j] = c;  // last_arm_actions = arm_actions (environments.py:608-611)
          break;
        }
        case FM_ENV_BACKUP_IK_TOGGLE: {
          // values selected, not pointers (a select of the global record and the constant table is a FLAT load)
          const double ia = ik_arm(dm, ti, td, arm).ik_actions()[j], dp = IK_DEFAULT_POSE[j];
          c = act[arm] == 1.0f ? ia : dp;
          break;
        }
        default:  // FM_ENV_FACTORY
          c = prop[u - 1];
      }
    }
    const double lo = M.ctrlrange_d[2 * u], hi = M.ctrlrange_d[2 * u + 1];
    uctl_[u] = c < lo ? lo : (c > hi ? hi : c);
  }
  init_arena(M, w, arena);
  // warmstart
  const double* ph = S.phys + (size_t)arena * dm.phys_stride;
  for (int i = LANE; i < dm.nv; i += WAVE) w.a()[i] = ph[2 * dm.nq + 2 * dm.nv + i];
  SYNC();
  // stage (mj_step1) at the state of the last mj_step1 (pre-teleport), then integrate the current state
  load_state(M, S, w, arena, true);
  SYNC();
  } else if constexpr (DIM::rerun) {
    // resume: the substep state the 64-contact kernel saved when its stage t0 exceeded 64 contacts
    const double* r = (const double*)S.resume + (size_t)ARENA_ * resume_stride(dm.nq, dm.nv, nu);
    if (LANE == 0) {
      w.misc()[MISC_CSUM] = (int)r[1];
      w.misc()[MISC_CMAX] = (int)r[2];
    }
    r += 3;
    for (int i = LANE; i < dm.nq; i += WAVE) w.qd()[i] = r[i];
    r += dm.nq;
    for (int i = LANE; i < dm.nv; i += WAVE) {
      w.vd()[i] = r[i];
      w.a()[i] = r[dm.nv + i];
    }
    r += 2 * dm.nv;
    for (int u = LANE; u < nu; u += WAVE) {
      ctrl_[u] = r[u];
      uctl_[u] = r[nu + u];
    }
    init_arena(M, w, arena);
    SYNC();
    refresh_copies(M, w);
    SYNC();
  }
#define lp (0.001 / (0.001 + M.pt_time))
#define phw (S.phys + (size_t)ARENA_ * dm.phys_stride)
#define sc_ (w.scal())  // [0] reward, [1] terminated, [2] out_of_reach, [3] force_terminate
  bool reset_pass = false;
  // Every physics phase has exactly one call site (the kernel is one loop), which keeps the code that a
  // substep walks through small enough for the instruction cache:
  //   t = 0..frame_skip-1:  mj_step1 (stage) ; ctrl low-pass ; mj_step2 (smooth acc, solve, integrate)
  //   then the task layer; on termination one more pass = reset_sim's forward (stage, smooth, solve).
  for (int t = t0;; t++) {
    stage(M, w, arena, ctr);
    if constexpr (can_abandon) {
      // uniform (LDS scalar); the experiment build's test hooks: FM_FORCE_RERUN=1 (512), every env-step goes to the
      // wide kernel; FM_RERUN_AT_50=1 (16384), every env-step abandoned at substep 50 (the resume path's parity test)
      if (S.rerun && (w.misc()[MISC_OVF] > 0 || (FM_XF(M) & 512) || ((FM_XF(M) & 16384) && t == 50))) {
        if (!reset_pass) {
          double* const rs = S.resume;
          if (rs) {
            // the substep state for the wide kernel to resume from (substeps 0 .. t-1 done; stage t is redone there)
            double* r = rs + (size_t)ARENA_ * resume_stride(dm.nq, dm.nv, nu);
            if (LANE == 0) {
              // the contact demand of the stages before t: stage t is redone (and counted) by the wide kernel
              r[0] = (double)t;
              r[1] = (double)(w.misc()[MISC_CSUM] - w.misc()[MISC_NSTAGE]);
              r[2] = (double)w.misc()[MISC_CMAX];
            }
            r += 3;
            for (int i = LANE; i < dm.nq; i += WAVE) r[i] = w.qd()[i];
            r += dm.nq;
            for (int i = LANE; i < dm.nv; i += WAVE) {
              r[i] = w.vd()[i];
              r[dm.nv + i] = w.a()[i];
            }
            r += 2 * dm.nv;
            for (int u = LANE; u < nu; u += WAVE) {
              r[u] = ctrl_[u];
              r[nu + u] = uctl_[u];
            }
          }
          if (LANE == 0) {
            // the wide kernel reads the list after this launch has ended (kernel boundary: no fence needed)
            int32_t* const rr = S.rerun;
            const int slot = atomicAdd(rr, 1);
            rr[1 + slot] = arena + 1;
          }
          return;
        }
        // the reset pass's forward (after the task layer wrote the records) cannot be abandoned: cut and count
        if (LANE == 0) ctr[0] += w.misc()[MISC_OVF];
      }
    }
    if (t == 0 && !reset_pass) {
      load_state(M, S, w, arena, false);
      SYNC();
    }
    if (!reset_pass) {
      for (int u = LANE; u < nu; u += WAVE) {
        double ct = ctrl_[u] + (uctl_[u] - ctrl_[u]) * lp;
        ctrl_[u] = u == 0 ? -td[1] : ct;
      }
      SYNC();
    }
    smooth_acc(M, w, arena, !reset_pass);
    PMARK(PH_SMOOTH);
    if (w.misc()[MISC_NCON] + w.misc()[MISC_NROW] > 0) {
      newton(M, w, arena, ctr);
    } else {
      for (int i = LANE; i < dm.nv; i += WAVE) {
        w.a()[i] = w.as()[i];
        w.fc()[i] = T(0);
      }
      SYNC();
    }
    if (reset_pass) break;
    implicit_integrate(M, w, arena, true);
    if (t < dm.frame_skip - 1) continue;
    // ---- end of the env-step: contact-force termination on the contacts + forces of the final solve
    {
      int ncon = w.misc()[MISC_NCON];
      bool hit = false;
      for (int c = LANE; c < ncon; c += WAVE) {
        const int* ci = w.ci() + 4 * c;
        if (!((ci[3] >> 16) & 1)) continue;
        const T* cr = w.cr() + CR_N * c;
        const T* f = cr + CR_F;
        T fn = f[0] + f[1] + f[2] + f[3];
        T f1 = (f[0] - f[1]) * cr[CR_MU], f2 = (f[2] - f[3]) * cr[CR_MU];
        T mx = fabs(fn);
        mx = fabs(f1) > mx ? fabs(f1) : mx;
        mx = fabs(f2) > mx ? fabs(f2) : mx;
        if ((double)mx > M.force_thr) hit = true;
      }
      // the ballot runs on the whole wave (inside `if (LANE == 0)` it would only see lane 0's contacts)
      const bool any_hit = __ballot(hit) != 0ull;
      if (LANE == 0) sc_[3] = any_hit ? 1.0 : 0.0;
    }
    // gripper sites at the final state (the last mj_step1's site_xpos)
    arm_hinge_sincos(M, w);
    SYNC();
    if (LANE < A) arm_chain<T, DIM, false>(M, w, LANE);
    SYNC();
    for (int e = LANE; e < 10 * A; e += WAVE) arm_body_post<T, DIM, false>(M, w, e / 10, e % 10);
    SYNC();
    if (LANE == 0) task_tail(M, w, ti, td, rng, ctr, act);
    FULL_SYNC();
    SYNC();
    refresh_copies(M, w);  // the TaskManager's teleports wrote the master state
    // stage state for the next env-step = the state after the TaskManager's teleports: MuJoCo's own outputs in
    // the reference show a cube spawned from rest falling freely from its first substep (tests/test_physics_pins.py)
    for (int i = LANE; i < dm.nq; i += WAVE) phw[dm.nq + dm.nv + i] = w.qd()[i];
    for (int i = LANE; i < dm.nv; i += WAVE) phw[2 * dm.nq + dm.nv + i] = w.vd()[i];
    SYNC();
    if (IK && env_toggle(ec)) ik_proposals(M, w, ti, td);  // the step's observation (environments.py:197, 560-577)
    const int term = sc_[1] != 0.0;
    if (LANE == 0) {
      const int s_fail = sc_[2] != 0.0;
      const bool force_term = sc_[3] != 0.0;
      int32_t* ts = ti + 2 * K;
      if (io.reward) io.reward[arena] = (float)sc_[0];
      if (io.terminated) io.terminated[arena] = (uint8_t)term;
      if (io.truncated) io.truncated[arena] = 0;
      if (io.scores) {
        io.scores[2 * arena] = ts[I_S0];
        io.scores[2 * arena + 1] = ts[I_S1];
      }
      if (io.num_obj) io.num_obj[arena] = ts[I_NIN];
      // episode-mix counters (fm_get_counters): contacts per stage, objects in scene, episodes ended
      ctr[4] += w.misc()[MISC_CSUM];
      ctr[5] = w.misc()[MISC_CMAX] > ctr[5] ? w.misc()[MISC_CMAX] : ctr[5];
      ctr[6] += ts[I_NIN];
      ctr[7] += term;
      if (io.play_time) io.play_time[arena] = td[2];
      if (io.conveyor_speed) io.conveyor_speed[arena] = td[1];
      if (io.out_of_reach) io.out_of_reach[arena] = (uint8_t)s_fail;
      if (io.force_terminate) io.force_terminate[arena] = (uint8_t)force_term;
      if (term) {
        if (io.ep_return) io.ep_return[arena] = td[3 + 2 * A];
        if (io.ep_len) io.ep_len[arena] = ts[I_EPLEN];
        if (io.terminal_scores) {
          io.terminal_scores[2 * arena] = ts[I_S0];
          io.terminal_scores[2 * arena + 1] = ts[I_S1];
        }
      }
    }
    if (!term) break;
    // ---- auto-reset (reset_sim, base_env.py:177-198): terminal obs, zero state, TaskManager.reset,
    // then one more pass of this loop = the forward at the reset state that leaves qacc_warmstart
    FULL_SYNC();
    if (io.terminal_obs) write_obs(M, w, ti, td, io.terminal_obs + (size_t)arena * dm.obs_dim * (M.obs64 ? 2 : 1));
    SYNC();
    for (int i = LANE; i < dm.nq; i += WAVE) w.qd()[i] = 0.0;
    for (int i = LANE; i < dm.nv; i += WAVE) {
      w.vd()[i] = 0.0;
      w.a()[i] = 0.0;
    }
    SYNC();
    if (LANE == 0) {
      task_reset<T, DIM>(M, w.qd(), w.vd(), ti, td, w.ctrl());
      td[3 + 2 * A] = 0.0;
      ti[2 * K + I_EPLEN] = 0;
    }
    SYNC();
    refresh_copies(M, w);
    for (int i = LANE; i < dm.nq; i += WAVE) phw[dm.nq + dm.nv + i] = w.qd()[i];
    for (int i = LANE; i < dm.nv; i += WAVE) phw[2 * dm.nq + dm.nv + i] = w.vd()[i];
    SYNC();  // the reset pass's stage reads the float copies other lanes just wrote (tools/lds_race_check.py)
    reset_pass = true;
  }
  store_state(M, S, w, arena);
  FULL_SYNC();
  if (IK && reset_pass && env_toggle(ec)) ik_proposals(M, w, ti, td);  // reset()'s observation after the auto-reset
  if (io.obs) write_obs(M, w, ti, td, io.obs + (size_t)arena * dm.obs_dim * (M.obs64 ? 2 : 1));
  PMARK(PH_TAIL);
  if (M.prof && LANE < PH_LAST) atomicAdd(M.prof + LANE, w.prof()[LANE]);
  {
    uint32_t* const cost_ = S.cost;
    if (cost_ && LANE == 0) cost_[arena] = (uint32_t)(wall_clock64() - t_begin);
  }
#undef ctrl_
#undef uctl_
#undef sc_
#undef w
#undef M
#undef S
#undef io
#undef L
#undef ti
#undef td
#undef rng
#undef ctr
#undef act
#undef phw
#undef lp
#undef ARENA_
}

template <typename T, typename DIM, bool IK>
__global__ void __launch_bounds__(64) FM_STEP_ATTR step_kernel(StepParams<T> params) {
  FM_SMEM_DECL(smem);
  (void)params;
  if constexpr (DIM::rerun) {
    // the wide-capacity rerun: the arenas the 64-contact launch abandoned, S.rerun[1 + i] - 1 for i < S.rerun[0],
    // over the launch's workgroups (a small grid: the list is short, usually empty; it runs after the 64-contact launch
    // on the same stream)
    const int32_t* const rr = kparams<StepParams<T>>().S.rerun;
    const int n = rr[0];
    for (int i = (int)blockIdx.x; i < n; i += (int)gridDim.x) {
      step_arena<T, DIM, IK>(smem, rr[1 + i] - 1);
      FULL_SYNC();
    }
  } else {
    // longest-processing-time-first dispatch: the host orders the arenas by their last env-step's duration, so the
    // expensive ones start in the first wave of workgroups and the cheap ones fill the tail (results do not depend
    // on which workgroup steps an arena)
    const int32_t* const order_ = kparams<StepParams<T>>().S.order;
    step_arena<T, DIM, IK>(smem, order_ ? order_[blockIdx.x] : (int)blockIdx.x);
  }
}


// diagnostic: run one mj_step1 + acceleration stage on arena `arena` at its stored state and dump
// internals (float64) for comparison with the oracle.  Layout (see fm_debug_dump in the C ABI):
// [0] ncon [1] nrow | Marm A*81 | pb nv | as nv | a nv | fc nv | site 3A | bpos 30A | bcom 30A |
// dax 27A | contacts 64 x (g1 g2 dist pos3 frame9 mu D) | rows 20A x (d0 d1 pos D aref f)
template <typename T, typename DIM>
__global__ void __launch_bounds__(64) debug_kernel(Model<T> M, State<T> S, Lay L, int arena, int actuated,
                                                   double* out) {
  FM_SMEM_DECL(smem);
  const DIM dm(M.dm);
  Ws<T, DIM> w{lds_base(smem), &L, spill_base<DIM>(S, arena)};
  int64_t* ctr = S.counters + FM_NCTR * (size_t)arena;
  const double* ph = S.phys + (size_t)arena * dm.phys_stride;
  const double* dsrc = S.dbl + (size_t)arena * dm.dbl_stride;
  for (int u = LANE; u < dm.nu; u += WAVE) w.ctrl()[u] = dsrc[u];
  for (int i = LANE; i < dm.nv; i += WAVE) w.a()[i] = ph[2 * dm.nq + 2 * dm.nv + i];
  init_arena(M, w, arena);
  SYNC();
  load_state(M, S, w, arena, true);
  SYNC();
  stage(M, w, arena, ctr);
  smooth_acc(M, w, arena, actuated != 0);
  const int A = dm.A, nv = dm.nv;
  int ncon = w.misc()[MISC_NCON], nrow = w.misc()[MISC_NROW];
  const double zs = zshift<T>();
  // the contacts' geometry first: the solver reuses those record slots for its float64 row products
  {
    double* oc = out + 2 + 81 * A + 4 * nv + 3 * A + 60 * A + 27 * A;
    for (int c = LANE; c < 64; c += WAVE) {
      double* r = oc + 17 * c;
      if (c < ncon) {
        const int* ci = w.ci() + 4 * c;
        const T* cr = w.cr() + CR_N * c;
        r[0] = M.geom_i[4 * (ci[0] & 4095)];
        r[1] = M.geom_i[4 * ((ci[0] >> 12) & 4095)];
        r[2] = cr[CR_DIST];
        double o[3];
        contact_anchor(w, anchor_cube(dm, (w.ginfo()[ci[0] & 4095] >> 8) & 255, (w.ginfo()[(ci[0] >> 12) & 4095] >> 8) & 255),
                       o);
        for (int k = 0; k < 3; k++) r[3 + k] = o[k] + (double)cr[CR_POS + k] + (k == 2 ? zs : 0.0);
        for (int k = 0; k < 9; k++) r[6 + k] = cr[CR_FR + k];
        r[15] = cr[CR_MU];
        r[16] = cr[CR_D];
      } else {
        for (int k = 0; k < 17; k++) r[k] = 0;
      }
    }
  }
  SYNC();
  if (ncon + nrow > 0) newton(M, w, arena, ctr);
  SYNC();
  double* o = out;
  if (LANE == 0) {
    o[0] = ncon;
    o[1] = nrow;
  }
  o += 2;
  for (int i = LANE; i < 81 * A; i += WAVE) o[i] = (double)w.Marm()[i];
  o += 81 * A;
  for (int i = LANE; i < nv; i += WAVE) {
    o[i] = (double)w.pb()[i];
    o[nv + i] = (double)w.as()[i];
    o[2 * nv + i] = (double)w.a()[i];
    o[3 * nv + i] = (double)w.fc()[i];
  }
  o += 4 * nv;
  // positions back in the world frame (zshift)
  for (int i = LANE; i < 3 * A; i += WAVE) o[i] = (double)w.site()[i] + (i % 3 == 2 ? zs : 0.0);
  o += 3 * A;
  for (int i = LANE; i < 30 * A; i += WAVE) {
    o[i] = (double)w.bpos()[i] + (i % 3 == 2 ? zs : 0.0);
    o[30 * A + i] = (double)w.bcom()[i] + (i % 3 == 2 ? zs : 0.0);
  }
  o += 60 * A;
  for (int i = LANE; i < 27 * A; i += WAVE) o[i] = (double)w.dax()[i];
  o += 27 * A;
  o += 17 * 64;
  for (int r = LANE; r < 20 * A; r += WAVE) {
    double* x = o + 6 * r;
    if (r < nrow) {
      const int* ri = w.ri() + 4 * r;
      const T* rr = w.rr() + RR_N * r;
      x[0] = ri[0];
      x[1] = ri[1];
      x[2] = rr[RR_POS];
      x[3] = rr[RR_D];
      x[4] = rr[RR_AREF];
      x[5] = rr[RR_F];
    } else {
      for (int k = 0; k < 6; k++) x[k] = 0;
    }
  }
}

}  // namespace fm

