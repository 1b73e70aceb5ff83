// fm_dev.hpp -- device-side data structures and small math helpers for the env-step kernel.
#pragma once
#ifdef FM_HOST_SIMT
#include "fm_simt_host.hpp"  // the CPU backend: this code compiled for the host, the wave emulated (fm_cpu.cpp)
#else
#include <hip/hip_runtime.h>
#endif

#include <cstdint>

namespace fm {

// Address-space-tagged device pointers.  Launch parameters reach the kernel through an opaque kernarg
// pointer (see step_kernel), which hides from the compiler where the pointers stored in them point; a
// plain pointer would then be accessed with FLAT instructions (which count against both vmcnt and
// lgkmcnt, so every table read also drains the wave's LDS traffic).  cptr<X> (read-only scene tables,
// actions) round-trips through the constant address space -> scalar loads for uniform indices and
// global_load otherwise; gptr<X> (state, outputs) through the global address space -> global_load/store.
#if defined(__HIP_DEVICE_COMPILE__)
#define FM_AS_CONST __attribute__((address_space(4)))
#define FM_AS_GLOBAL __attribute__((address_space(1)))
#define FM_AS(n) __attribute__((address_space(n)))
#else
#define FM_AS_CONST
#define FM_AS_GLOBAL
#define FM_AS(n)
#endif
// an opaque copy of a value the compiler must not hoist or fold (uniform "s" / per-lane "v" register classes on the GPU)
#ifdef FM_HOST_SIMT
#define FM_OPAQUE_S(x) asm volatile("" : "+r"(x))
#define FM_OPAQUE_V(x) asm volatile("" : "+r"(x))
#else
#define FM_OPAQUE_S(x) asm volatile("" : "+s"(x))
#define FM_OPAQUE_V(x) asm volatile("" : "+v"(x))
#endif
// address spaces by number (FM_AS(n)): 1 global, 3 LDS, 4 constant.  Non-inlined device functions take their
// pointer parameters in a named address space: a plain pointer parameter is generic inside the callee, and every
// access through it a FLAT instruction (tests/test_build_flags.py asserts that no step kernel has one)
enum { AS_GLOBAL = 1, AS_LDS = 3, AS_CONST = 4 };
template <typename X>
struct cptr {
  const X* p;
  cptr() = default;
  __host__ __device__ constexpr cptr(const X* q) : p(q) {}
  __host__ __device__ __forceinline__ operator const X*() const {
#if defined(__HIP_DEVICE_COMPILE__)
    return (const X*)(const X FM_AS_CONST*)p;
#else
    return p;
#endif
  }
};
template <typename X>
struct gptr {
  X* p;
  gptr() = default;
  __host__ __device__ constexpr gptr(X* q) : p(q) {}
  __host__ __device__ __forceinline__ operator X*() const {
#if defined(__HIP_DEVICE_COMPILE__)
    return (X*)(X FM_AS_GLOBAL*)p;
#else
    return p;
#endif
  }
};

constexpr int WAVE = 64;
// per-arena contact capacity: 64 for the benchmark scene (2, 4) (one contact per lane, one 64-bit tree mask
// word), 128 elsewhere (two contacts per lane, two mask words): with K cubes parked / hidden on the floor
// (4 contacts each) the larger scenes exceed 64 contacts (census: (4, 16) reaches 80, (2, 8) pile-ups > 64)
constexpr int MAXCON = 64;
constexpr int MAXCON_WIDE = 128;
constexpr int CJ = 18;        // Jacobian columns per contact (two trees of <= 9 dofs)
constexpr int MAXSURV = 512;  // broadphase survivors per chunk
constexpr int MAXPC = 8;      // contacts per geom pair (box-box)

// Flat per-arena record layouts (strides in elements)
struct Dims {
  static constexpr bool fixed = false;  // runtime dims (see FixedDims for compile-time scenes)
  static constexpr bool spill = false;  // Hessian + contact records in LDS (see DimsSpill)
  static constexpr bool midcache = false;  // cached midphase (FixedDims of the large scenes)
  static constexpr int MAXC = MAXCON_WIDE;  // upper bound of maxcon the code is built for
  static constexpr bool rerun = false;      // see FixedDims<A, K, true>
  static constexpr bool f64arms = false;    // see FixedDims
  static constexpr bool f64gl = false;      // see FixedDims
  static constexpr bool gl_lists = false;   // see FixedDims
  template <int TS>
  __host__ __device__ static constexpr bool gl_coll() {
    return false;
  }
  template <int TS>
  __host__ __device__ static constexpr bool gl_gx() {
    return false;
  }
  template <int TS>
  __host__ __device__ static constexpr bool gl_sp() {
    return false;
  }
  template <int TS>
  __host__ __device__ static constexpr bool gl_tbr() {
    return false;
  }
  static constexpr bool treeblk = false;    // see FixedDims
  template <int TS>
  __host__ __device__ static constexpr bool treeblk_for() {
    return false;
  }
  int N, A, K, nq, nv, nu, ngc, nbox, npair, nparam, ntree, obs_dim, act_dim, frame_skip;
  int ncb, ncbp;  // collision bodies, allowed collision-body pairs
  int maxcon, maxrow;
  int phys_stride;  // double: qpos nq | qvel nv | qpos_s nq | qvel_s nv | qacc_ws nv
  int dbl_stride;   // double: ctrl_target nu | spawn_freq | speed | play_time | last_grip A | last_bucket A | ep_return
                    //         | IK block A x 27 (fm_ik.hpp)
  int int_stride;   // int32:  in_scene K | out_scene K | n_in n_out step since fail hidden score0 score1 last0 last1 ep_len
                    //         | IK block A x (3 + A)
};

// indices into the int block after the two lists
enum { I_NIN = 0, I_NOUT, I_STEP, I_SINCE, I_FAIL, I_HIDDEN, I_S0, I_S1, I_LS0, I_LS1, I_EPLEN, I_NINT };

// IKPolicy's step counts and velocity compensation (ik_policy.py:56-67), from env.dt = timestep * frame_skip and
// env.pt_time on the host: int(0.5 / dt), int(1 / dt), int(1 / dt), int(3 / dt), pt_time * dt * 15
struct IkTiming {
  double pt_comp;
  int release_wait, grasp_wait, move_steps, timeout_steps;
};

// The experiment build (libfactorysim_exp.so, -DFM_EXPERIMENTS=1) carries a few runtime switches: the reference forms
// of the kernel's exact reformulations (the equivalence tests) and the rerun path's test hooks.  The product library
// is compiled without them: FM_XF(M) is the constant 0 there, so every switch branch folds away and Model has no
// dbg_flags field (tests/test_build_flags.py)
#ifndef FM_EXPERIMENTS
#define FM_EXPERIMENTS 0
#endif
#if FM_EXPERIMENTS
#define FM_XF(M) ((M).dbg_flags)
#else
#define FM_XF(M) 0
#endif

template <typename T>
struct Model {
  Dims dm;
  // scene scalars
  T dt, grav;
  double grav_d;  // 9.81 exactly (a free cube's acceleration is -g: formed in float64, scene.xml default gravity)
  T belt_mass, belt_kv, belt_damp, belt_invw_t;
  double timestep;  // model.opt.timestep, exact (solver gains)
  double init_speed, accel, pt_time, force_thr, spawn_freq0, spawn_inc;
  double w_grip, w_bucket, w_action, base_reward;
  double bucket_x0, bucket_x1, bucket_y, bucket_z;
  int env_class, solver_iter;
  double solver_tol;
  IkTiming ik_time;
  // arm template
  cptr<T> arm_base;  // [A][12]  world pos(3), R(9) of the iiwa frame (kernel frame: zshift)
  cptr<double> arm_base_w;  // [A][12] the same in float64, world frame (IK base policy, fm_ik.hpp)
  cptr<T> body;      // [10][32] local pos(3) local R(9) mass ipos(3) iR(9) I(3) invw_t invw_r pad(2)
  cptr<T> dof;       // [9][4]   range lo, hi, dof_invweight0, pad
  const double* dofd;  // [9][4]  the same in float64 (joint-limit rows)
  cptr<T> ctrlrange; // [nu][2]
  cptr<double> ctrlrange_d;  // [nu][2] float64 (actuator_ctrlrange as the reference clips with it)
  // geoms (compact, collidable)
  cptr<T> geom;      // [ngc][16]  pos(3) R(9) size(3) rbound
  cptr<double> geomd;  // the same table in float64 (the fp32 build's float64 narrowphase)
  cptr<int> geom_i;  // [ngc][4]   mjid, type, kbody, box slot
  cptr<uint32_t> pair;  // [npair]  c1 | c2 << 12 | param << 24 (reference list; the kernel uses cb*)
  cptr<int> ginfo;      // [ngc] packed: type code | arm << 2 | pclass << 3 | kbody << 8
  cptr<int> cbi;        // [ncb][4] kbody, flags, first index in cbg, geom count
  cptr<T> cbs;          // [ncb][8] static AABB centre(3), radius, half extents(3), pad
  cptr<uint16_t> cbg;   // geoms grouped by collision body
  cptr<uint32_t> cbp;   // [ncbp] allowed collision-body pairs b1 | b2 << 8
  int ptab[25];          // param index by (pclass g1, pclass g2)
  cptr<double> param;  // [nparam][8] mu, solref(2), solimp(5): float64 in both builds (impedance / R below)
  // per arena
  cptr<T> cube;      // [N][K][4] h, m, I, h - (T)h (the half size's rounding residue: h = [0] + [3] in float64)
  cptr<T> meaninertia;  // [N]
  cptr<uint32_t> tri;   // [nv (nv+1) / 2]  column-major lower triangle: i | j << 16
  unsigned long long* prof;  // [16] phase clocks (fm_profile), NULL when profiling is off
#if FM_EXPERIMENTS
  int dbg_flags;  // the experiment build's switches (fm_api.hip read_experiment_flags; FM_XF)
#endif
  int ovf_abort;             // 1: a stage above the contact capacity abandons the env-step (State::rerun), not cut it
  int obs64;                 // 1: observation rows (obs, terminal_obs) are float64 (fm_config.obs_float64)
};

template <typename T>
struct State {
  gptr<double> phys;  // float64 in both builds (the fp32 physics keeps a float64 master state)
  gptr<double> dbl;
  gptr<int32_t> ints;
  gptr<uint64_t> rng;      // [N][4]
  gptr<int64_t> counters;  // [N][4]
  // dispatch order of the env-step (longest first, fm_api.hip lpt_order_kernel): workgroup b steps arena
  // order[b]; cost[a] = arena a's last env-step in s_memrealtime ticks.  Null: workgroup b steps arena b.
  gptr<uint32_t> cost{nullptr};
  cptr<int32_t> order{nullptr};
  // DimsSpill: per-arena global scratch blocks (Lay::gtotal bytes each) for the Hessian and the contact records
  gptr<char> spill{nullptr};
  long long spill_stride{0};
  // (2,4) contact overflow: [0] = count, [1 + i] = 1 + the arena ids whose env-step the 64-contact kernel abandoned
  // (0: slot not yet written) for the wide rerun kernel.  Null: the capacity cut (counted in counters[0]) instead
  gptr<int32_t> rerun{nullptr};
  // IK classes with `rerun`: the arena's task records (dbl, ints) as the env-step found them, restored by the rerun
  // (the IK compose writes the FSM and the toggles' last actions before the substeps)
  gptr<char> bak{nullptr};
  // with `rerun`: per arena the substep state at which the 64-contact kernel abandoned its env-step (resume_stride
  // doubles: [0] substep t, [1] [2] the contact counters of the stages so far, qpos nq, qvel nv, qacc warmstart nv,
  // ctrl nu, clipped control target nu), so the wide kernel resumes at substep t instead of redoing the env-step;
  // t = 0: nothing done yet, the wide kernel runs the whole env-step
  gptr<double> resume{nullptr};
};
// doubles per arena of State::resume
__host__ __device__ constexpr int resume_stride(int nq, int nv, int nu) { return 3 + nq + 2 * nv + 2 * nu; }

// the arena's global scratch block (nullptr unless the kernel runs a spill layout; the (2,4) wide rerun kernel keeps its
// workspace in LDS)
template <typename DIM, typename T>
__device__ __forceinline__ char* spill_base(const State<T>& S, int arena) {
  static_assert(!(DIM::spill && DIM::rerun), "a spilled wide rerun kernel would need scratch blocks of its own");
  if constexpr (DIM::spill)
    return (char*)S.spill + (long long)arena * S.spill_stride;
  else
    return nullptr;
}

struct StepIO {
  cptr<float> actions;
  gptr<float> obs;
  gptr<float> reward;
  gptr<uint8_t> terminated;
  gptr<uint8_t> truncated;
  gptr<int32_t> scores;
  gptr<int32_t> num_obj;
  gptr<double> play_time;
  gptr<double> conveyor_speed;
  gptr<uint8_t> out_of_reach;
  gptr<uint8_t> force_terminate;
  gptr<float> terminal_obs;
  gptr<double> ep_return;
  gptr<int32_t> ep_len;
  gptr<int32_t> terminal_scores;
  cptr<uint8_t> reset_mask;
};

// opaque copy of a pointer: loads through the result cannot be CSE'd with, or hoisted above, earlier
// loads through the same pointer (keeps long-lived launch parameters out of the SGPR file)
template <typename P>
__device__ __forceinline__ const P* opaque(const P* p) {
  FM_OPAQUE_S(p);
  return p;
}

// the kernel's own parameter block, through a fresh opaque constant-address-space pointer at each use
template <typename P>
__device__ __forceinline__ const P& kparams() {
  const P FM_AS_CONST* p = (const P FM_AS_CONST*)__builtin_amdgcn_kernarg_segment_ptr();
  FM_OPAQUE_S(p);
  return *(const P*)p;
}

// the kernel's dynamic LDS (the CPU backend: the emulated wave's per-thread buffer)
#ifdef FM_HOST_SIMT
#define FM_SMEM_DECL(name) char* name = ::fm_simt::wave().lds
#else
#define FM_SMEM_DECL(name) extern __shared__ __attribute__((aligned(16))) char name[]
#endif

// LDS base with an opaque zero VGPR added: every workspace access becomes [vbase + immediate offset]
// instead of one hoisted SGPR per distinct LDS address (which the compiler otherwise keeps live across
// the whole substep loop and spills)
__device__ __forceinline__ char* lds_base(char* smem) {
#if FM_EXP_PLAINBASE
  return smem;
#endif
  unsigned int z;
#ifdef FM_HOST_SIMT
  z = 0;
  FM_OPAQUE_V(z);
#else
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
#endif
  return smem + z;
}

// byte offsets of the per-arena LDS workspace (computed on the host, see lds_layout())
struct Lay {
  int q, v, a, as, fs, fc, pb, g, dir, Ma, tmp, fa;
  int qd, vd;  // double master copies of q / v (fp32 build; the same arrays as q / v in fp64)
  int ctrl;   // double
  int aforce;
  int bpos, bR, bcom, bIw, bF, bN, dax, danc, site;
  int cR;
  int Marm;
  int gx;     // T [ngc][4]  geom world centre, rbound
  int ginfo, cbi, cbw, cbg;  // LDS copies of the geom / collision-body tables, body bounds T [ncb][8]
  int sp, gsurv;             // broadphase work lists
  int stage, skey, spw;      // staged contacts T [maxcon][8], keys, pair words
  int cube;                  // T [K][4] this arena's cube h, m, I
  int H;
  int c_i;    // int [maxcon][4]: g1 | g2 << 12, tree1, tree2, flags
  int c_r;    // T [maxcon][CR]
  int r_i;    // int [maxrow][4]
  int r_r;    // T [maxrow][8]
  int tmask;  // uint64 [ntree]
  int misc;   // int [16 + 64]
  int sort;   // int [K]
  int uctl;   // double [nu]  clipped control of this env-step
  int scal;   // double [4]   per-step scalars broadcast from lane 0
  int prof;   // uint64 [FM_NPROF]  phase clocks of this arena (profiling only)
  int bc;     // T [64]       broadcast row of the register-resident Cholesky
  int mcache, mpos;  // cached midphase: uint32 [mc_cap(nv)] hit list, T [ncb][3] body positions at the build
  int bposd, bRd;    // fp32 scenes with DIM::f64arms: double [A][10][3], [A][10][9] arm body poses (narrowphase)
  int tblk;          // (2,8), (2,10), (4,16), (2,4) wide: the tree-block Newton solve's workspace (T, TB_*; Newton phase)
  int tbr;           // with FixedDims::gl_tbr: its coupled system's matrix, a byte offset into the global block
  int total;
  // spill layouts (DimsSpill): H and c_r are byte offsets into the arena's global scratch block of gtotal bytes
  int spill, gtotal;
};

// fp32 builds place the world origin of the float copies at z = 1 m (the table / belt height): contact
// geometry then works with coordinates of 0..0.2 m instead of ~1.1 m, i.e. 8x finer float spacing in the
// contact distances the soft constraints amplify.  The float64 master state, the task layer, observations
// and the buckets stay in the reference's world frame.  fp64 builds use the world frame throughout.
template <typename T>
__host__ __device__ constexpr double zshift() {
  return sizeof(T) == 4 ? 1.0 : 0.0;
}

// per-contact real record; the Jacobian block first, so its three rows of CJ (even) start 8-byte aligned
// (records are CR_N = 84 reals, a multiple of 16 bytes) and read as 64-bit LDS loads.
// The Newton solver's per-contact iterate products are float64 in both builds (dslot(): CR_JA = B a and CR_JD =
// B dir, 3 doubles each; CR_F3 = the frame force D jar summed over the active edges, 3 doubles).  In the fp32
// record a double takes two slots: JA / JD overlay the contact geometry (dist, pos, frame: 13 slots, consumed
// when the rows are built), F3 shares its 6 slots with K_c (Hessian build only); every double starts on an
// even slot (8-byte aligned).
enum { CR_J = 0, CR_DIST = CR_J + 3 * CJ, CR_POS, CR_FR = CR_POS + 3, CR_MU = CR_FR + 9, CR_D, CR_KD, CR_BD, CR_VEL,
       CR_F3 = CR_VEL + 3, CR_F = CR_F3 + 6, CR_N = CR_F + 4,
       CR_JA = CR_DIST, CR_JD = CR_DIST + 6, CR_K = CR_F3 };
static_assert(CR_JA % 2 == 0 && CR_JD % 2 == 0 && CR_F3 % 2 == 0 && CR_JD + 6 <= CR_MU && CR_N % 4 == 0,
              "contact record: float64 slots aligned, JA / JD inside the geometry slots");
// generic row record (equality / joint limit); JAR = J a - aref and JD = J dir are float64 slots (2 reals in fp32)
enum { RR_C0 = 0, RR_C1, RR_POS, RR_D, RR_AREF, RR_F, RR_JAR, RR_JD = RR_JAR + 2, RR_N = RR_JD + 2 };
static_assert(RR_JAR % 2 == 0 && RR_N % 2 == 0, "row record: float64 slots aligned");
// float64 view of a record slot (both builds)
template <typename T>
__host__ __device__ __forceinline__ double* dslot(T* rec, int k) {
  return (double*)(rec + k);
}
template <typename T>
__host__ __device__ __forceinline__ const double* dslot(const T* rec, int k) {
  return (const double*)(rec + k);
}
// phase slots of the optional wall-clock profile (fm_profile)
// (slot PH_KHZ is the host's clock rate; PH_CBOUND .. PH_CNARROW split the collision phase: geom centres and body
// bounds, the body-pair midphase, the geom-pair expansion + narrowphase; PH_COLL keeps the contact ranking;
// PH_CHDIAG .. PH_CHSOLVE split the dense blocked Cholesky: diagonal blocks, panels, trailing updates, substitutions)
enum { PH_FK = 0, PH_GEOM, PH_COLL, PH_ROWS, PH_SMOOTH, PH_NSETUP, PH_NGRAD, PH_NHESS, PH_NCHOL, PH_NSOLVE, PH_NLS,
       PH_NFINAL, PH_INT, PH_TAIL, PH_NCON, PH_KHZ, PH_CBOUND, PH_CMID, PH_CNARROW, PH_CHDIAG, PH_CHPANEL, PH_CHTRAIL,
       PH_CHSOLVE, PH_LAST = 23, FM_NPROF = 24 };
enum { MISC_NCON = 0, MISC_NROW, MISC_NSURV, MISC_DROP, MISC_ITER, MISC_MAXIT, MISC_FLAG, MISC_NSTAGE, MISC_CSUM,
       MISC_CMAX, MISC_MC_OK, MISC_MC_N, MISC_MC_TOT, MISC_OVF };
// cached midphase (scenes with DIM::midcache): the body-pair hit list of an inflated bounding test is reused across
// substeps until a moving collision body has travelled MC_HALF from where it was when the list was built
// hit pairs a cached list holds (more: no caching that substep); the (2,4) scene has LDS room for 40 within its
// 4-arenas-per-CU budget
__host__ __device__ constexpr int mc_cap(int nv) { return nv > 48 ? 256 : 40; }
#ifndef FM_MC_MARGIN
#define FM_MC_MARGIN 0.01  // measured 4 / 2 / 1 cm: (4,16) equal, (2,8) best at 1 cm (gpurun_out/r03n)
#endif
constexpr double MC_MARGIN = FM_MC_MARGIN;    // m added to every bound (sphere radius, plane distance)
constexpr double MC_HALF = 0.5 * MC_MARGIN;  // rebuild once any moving body has moved this far (both ends: MC_MARGIN)
// per-arena int64 counters (fm_get_counters): contacts dropped for capacity, Newton iterations, Newton
// max-iteration hits, bucket-index anomalies, contacts summed over stages, max contacts in one stage,
// objects in scene summed over env-steps, episodes ended, env-steps rerun at the wide contact capacity
constexpr int FM_NCTR = 9;
// packed geom info
enum { GC_PLANE = 0, GC_SPHERE = 1, GC_BOX = 2, GI_ARM = 2, GI_PC = 3 };

// ------------------------------------------------------------------------------------------------
// math helpers
// ------------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T dsqrt(T x) {
  return sqrt(x);
}

template <typename T>
__device__ __forceinline__ void cross3(const T* a, const T* b, T* r) {
  T t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0;
  r[1] = t1;
  r[2] = t2;
}
template <typename T>
__device__ __forceinline__ T dot3(const T* a, const T* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
template <typename T>
__device__ __forceinline__ void matvec3(const T* R, const T* v, T* r) {
  T t0 = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  T t1 = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  T t2 = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
  r[0] = t0;
  r[1] = t1;
  r[2] = t2;
}
template <typename T>
__device__ __forceinline__ void mattvec3(const T* R, const T* v, T* r) {
  T t0 = R[0] * v[0] + R[3] * v[1] + R[6] * v[2];
  T t1 = R[1] * v[0] + R[4] * v[1] + R[7] * v[2];
  T t2 = R[2] * v[0] + R[5] * v[1] + R[8] * v[2];
  r[0] = t0;
  r[1] = t1;
  r[2] = t2;
}
template <typename T>
__device__ __forceinline__ void matmul3(const T* A, const T* B, T* C) {
  T t[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
#pragma unroll
  for (int k = 0; k < 9; k++) C[k] = t[k];
}

template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}
template <typename T>
__device__ __forceinline__ T wave_min(T x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T y = __shfl_xor(x, o);
    x = y < x ? y : x;
  }
  return x;
}
template <typename T>
__device__ __forceinline__ T wave_max(T x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T y = __shfl_xor(x, o);
    x = y > x ? y : x;
  }
  return x;
}

// fp32 wave reductions on DPP (row quad-perms / rotates, then the row broadcasts) instead of ds_swizzle /
// ds_bpermute: a VALU-latency chain, no LDS round trips.  The result is read from lane 63 (uniform).
// Every call site runs with the full wave active (EXEC = all 64 lanes).
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float x, float old) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(x), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_sum(float x) {
  x += dpp_f32<0xb1>(x, 0.0f);   // quad_perm [1,0,3,2]
  x += dpp_f32<0x4e>(x, 0.0f);   // quad_perm [2,3,0,1]
  x += dpp_f32<0x124>(x, 0.0f);  // row_ror:4
  x += dpp_f32<0x128>(x, 0.0f);  // row_ror:8
  x += dpp_f32<0x142>(x, 0.0f);  // row_bcast:15
  x += dpp_f32<0x143>(x, 0.0f);  // row_bcast:31
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}
__device__ __forceinline__ float wave_min(float x) {
  x = fminf(x, dpp_f32<0xb1>(x, x));
  x = fminf(x, dpp_f32<0x4e>(x, x));
  x = fminf(x, dpp_f32<0x124>(x, x));
  x = fminf(x, dpp_f32<0x128>(x, x));
  x = fminf(x, dpp_f32<0x142>(x, x));
  x = fminf(x, dpp_f32<0x143>(x, x));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}
// fp64 reductions (the Newton solver's cost, gradient and line search in both builds): the same DPP sequence
// moving both 32-bit halves, then the 64-bit read of lane 63
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x, double old) {
  const unsigned long long xi = (unsigned long long)__double_as_longlong(x);
  const unsigned long long oi = (unsigned long long)__double_as_longlong(old);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)oi, (int)(unsigned)xi, CTRL, 0xf, 0xf, false);
  const unsigned hi =
      (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)(oi >> 32), (int)(unsigned)(xi >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double lane63_f64(double x) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, 63);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), 63);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double wave_sum(double x) {
  x += dpp_f64<0xb1>(x, 0.0);
  x += dpp_f64<0x4e>(x, 0.0);
  x += dpp_f64<0x124>(x, 0.0);
  x += dpp_f64<0x128>(x, 0.0);
  x += dpp_f64<0x142>(x, 0.0);
  x += dpp_f64<0x143>(x, 0.0);
  return lane63_f64(x);
}
__device__ __forceinline__ double wave_min(double x) {
  x = fmin(x, dpp_f64<0xb1>(x, x));
  x = fmin(x, dpp_f64<0x4e>(x, x));
  x = fmin(x, dpp_f64<0x124>(x, x));
  x = fmin(x, dpp_f64<0x128>(x, x));
  x = fmin(x, dpp_f64<0x142>(x, x));
  x = fmin(x, dpp_f64<0x143>(x, x));
  return lane63_f64(x);
}

// inclusive prefix sum of an int over the wave on DPP (row shifts, then the row broadcasts; rocPRIM's
// warp_scan_dpp sequence); full wave active at every call site
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ int wave_incl_scan(int x) {
  const int lane = (int)threadIdx.x, rl = lane & 15;
  int t;
  t = dpp_i32<0x111>(x);  // row_shr:1
  if (rl >= 1) x += t;
  t = dpp_i32<0x112>(x);  // row_shr:2
  if (rl >= 2) x += t;
  t = dpp_i32<0x114>(x);  // row_shr:4
  if (rl >= 4) x += t;
  t = dpp_i32<0x118>(x);  // row_shr:8
  if (rl >= 8) x += t;
  t = dpp_i32<0x142>(x);  // row_bcast:15
  if ((lane & 31) >= 16) x += t;
  t = dpp_i32<0x143>(x);  // row_bcast:31
  if (lane >= 32) x += t;
  return x;
}

// inclusive prefix maximum of an int over the wave (the wave_incl_scan sequence with max)
__device__ __forceinline__ int wave_incl_max(int x) {
  const int lane = (int)threadIdx.x, rl = lane & 15;
  int t;
  t = dpp_i32<0x111>(x);
  if (rl >= 1) x = x > t ? x : t;
  t = dpp_i32<0x112>(x);
  if (rl >= 2) x = x > t ? x : t;
  t = dpp_i32<0x114>(x);
  if (rl >= 4) x = x > t ? x : t;
  t = dpp_i32<0x118>(x);
  if (rl >= 8) x = x > t ? x : t;
  t = dpp_i32<0x142>(x);
  if ((lane & 31) >= 16) x = x > t ? x : t;
  t = dpp_i32<0x143>(x);
  if (lane >= 32) x = x > t ? x : t;
  return x;
}

template <typename T>
struct StepParams {
  Model<T> M;
  State<T> S;
  Lay L;
  StepIO io;
};

// ------------------------------------------------------------------------------------------------
// LDS workspace layout of one arena (byte offsets), shared by host and device.  For a compile-time
// scene (FixedDims) every offset is a constant, so LDS accesses use immediate offsets off one
// lane-address register instead of one address register per array.
// ------------------------------------------------------------------------------------------------
// row stride of the Newton Hessian in LDS: fp32 scenes above 80 dofs factor it with the dense blocked matrix-core
// Cholesky, which wants whole 16 x 16 blocks (rows / columns padded to a multiple of 16: zero, diagonal 1)
__host__ __device__ constexpr int hstride(int tsize, int nv) { return (tsize == 4 && nv > 80) ? ((nv + 15) & ~15) : nv; }
// scratch floats after the padded Hessian (the dense Cholesky's inverse diagonal block)
__host__ __device__ constexpr int hextra(int tsize, int nv) { return (tsize == 4 && nv > 80) ? 256 : 0; }

// workspace of the tree-block Newton solve (fp32 (2,8), (2,10), (4,16)): per tree a 9 x 9 lower-triangle block (packed, P9) and its
// belt row, then the coupled trees' dense system (<= TB_MAXR positions incl. the belt, row stride = its size), its
// position -> (tree, local dof) map, and the coupled system's right-hand side (TB_MAXR doubles) and solution
// (TB_MAXR floats) -- their own slots: the solver's nv-double scratch w.tmp() is too small for them at (2,4)
// (nv = 43 < 1.5 TB_MAXR)
constexpr int TB_BLK = 54, TB_MAXR = 32;
// (glr: the coupled system's matrix lives in the arena's global block instead, Lay::tbr)
__host__ __device__ constexpr int tb_rest(int ntree) { return (TB_BLK * ntree + 3) & ~3; }
__host__ __device__ constexpr int tb_map(int ntree, bool glr = false) {
  return tb_rest(ntree) + (glr ? 0 : TB_MAXR * TB_MAXR);
}
__host__ __device__ constexpr int tb_rhs(int ntree, bool glr = false) {  // 16-byte aligned
  return (tb_map(ntree, glr) + TB_MAXR + 3) & ~3;
}
__host__ __device__ constexpr int tb_sol(int ntree, bool glr = false) { return tb_rhs(ntree, glr) + 2 * TB_MAXR; }
__host__ __device__ constexpr int tb_floats(int ntree, bool glr = false) { return tb_sol(ntree, glr) + TB_MAXR; }

__host__ __device__ constexpr Lay make_layout(int A, int K, int nq, int nv, int nu, int ngc, int ncb, int maxcon,
                                              int maxrow, int ntree, int tsize, bool spill = false,
                                              bool midcache = false, bool nobc = false, bool f64arms = false,
                                              bool gl_lists = false, bool treeblk = false, int tmask_words = 0,
                                              bool gl_stage = false, bool gl_tbr = false, bool f64gl = false,
                                              bool gl_gx = false) {
  Lay L{};
  int off = 0;
  auto take = [&off](int bytes) {
    int o = off;
    off += (bytes + 15) & ~15;
    return o;
  };
  // lane-broadcast row first: within ds_read2's 1 KiB offset reach of the workspace base
  L.bc = take(nobc ? 0 : tsize * WAVE);  // unused by the (2,4) kernel's register Cholesky
  L.q = take(tsize * nq);
  L.v = take(tsize * nv);
  L.a = take(8 * nv);  // Newton iterate (float64 in both builds; the next substep's warmstart)
  L.as = take(tsize * nv);
  L.fs = take(tsize * nv);
  L.fc = take(tsize * nv);
  L.pb = take(tsize * nv);
  L.dir = take(tsize * nv);
  L.fa = take(tsize * nv);
  // float64 master state: the fp32 physics reads the float copies q / v, the integrator accumulates in
  // double (an fp32 qpos cannot absorb increments below half an ulp: dt * qvel of a joint at rest)
  L.qd = tsize == 8 ? L.q : take(8 * nq);
  L.vd = tsize == 8 ? L.v : take(8 * nv);
  L.ctrl = take(8 * nu);
  L.aforce = take(tsize * nu);
  L.bpos = take(tsize * 30 * A);
  L.bR = take(tsize * 90 * A);
  L.bcom = take(tsize * 30 * A);
  L.bIw = take(tsize * 60 * A);
  L.bF = take(tsize * 30 * A);
  L.bN = take(tsize * 30 * A);
  L.dax = take(tsize * 27 * A);
  L.danc = take(tsize * 27 * A);
  L.site = take(tsize * 3 * A);
  L.cR = take(tsize * 9 * K);
  L.Marm = take(tsize * 81 * A);
  L.ginfo = take(4 * ngc);
  L.cbi = take(4 * 4 * ncb);
  L.cbg = take(2 * ngc);
  L.cube = take(tsize * 4 * K);
  // phase-local buffers share one region: collision work lists (stage) and the Newton Hessian + the solver's
  // float64 vectors (gradient, M (a - as), scratch; live from the solve to the integration) are never live
  // together
  const int u0 = off;
  if (!spill) L.H = take(tsize * (hstride(tsize, nv) * hstride(tsize, nv) + hextra(tsize, nv)));
  L.g = take(8 * nv);
  L.Ma = take(8 * nv);
  L.tmp = take(8 * nv);
  if (treeblk) L.tblk = take(tsize * tb_floats(ntree, gl_tbr));
  int uend = off;
  off = u0;
  if (!gl_gx) L.gx = take(tsize * 4 * ngc);
  L.cbw = take(tsize * 8 * ncb);
  if (!gl_lists) L.sp = take(4 * (ncb * (ncb - 1) / 2));  // every possible body pair can pass the midphase
  L.gsurv = take(4 * 4 * WAVE);
  if (!gl_stage) {
    L.stage = take(tsize * 8 * maxcon);
    L.skey = take(4 * maxcon);
    L.spw = take(4 * maxcon);
  }
  uend = off > uend ? off : uend;
  off = uend;
  L.c_i = take(4 * 4 * maxcon);
  if (!spill) L.c_r = take(tsize * CR_N * maxcon);
  L.r_i = take(4 * 4 * maxrow);
  L.r_r = take(tsize * RR_N * maxrow);
  // word h of tree t at [h * ntree + t]; the readers (and the zero fill past maxcon) cover DIM::MAXC / 64 words
  const int tmw = (maxcon + 63) / 64 > tmask_words ? (maxcon + 63) / 64 : tmask_words;
  L.tmask = take(8 * ntree * tmw);
  L.misc = take(4 * (16 + WAVE));  // 16 scalars + the Hessian assembly's block offsets
  L.sort = take(4 * K);
  L.uctl = take(8 * nu);
  L.scal = take(8 * 4);
  // phase clocks (profiling only): in the global block at (4,16) with its lists there (FM_GL416), the 144 B it misses
  // for 5 arenas per CU; elsewhere the global pointer costs the kernels ~10 VGPR spills
  const bool gl_prof = spill && gl_stage && A == 4;
  if (!gl_prof) L.prof = take(8 * FM_NPROF);
  if (midcache) {
    if (!gl_lists) L.mcache = take(4 * mc_cap(nv));  // a midphase list in the global block is its own cache
    L.mpos = take(tsize * 3 * ncb);
  }
  const bool f64a = f64arms && tsize == 4;
  f64gl = f64a && spill && (gl_lists || f64gl);
  if (f64a && !f64gl) {
    L.bposd = take(8 * 30 * A);
    L.bRd = take(8 * 90 * A);
  }
  L.total = off;
  if (spill) {  // the two largest arrays in the arena's global scratch block (L2 / HBM) instead of LDS
    L.spill = 1;
    L.H = 0;
    L.c_r = (tsize * (hstride(tsize, nv) * hstride(tsize, nv) + hextra(tsize, nv)) + 15) & ~15;
    int g = L.c_r + ((tsize * CR_N * maxcon + 255) & ~255);
    if (gl_lists) {  // also the midphase hit list (the (4,16) scene: 4 arenas per CU)
      L.sp = g;
      g += (4 * (ncb * (ncb - 1) / 2) + 255) & ~255;
    }
    if (f64gl) {  // the float64 arm poses ((4,16); the fp32 IK-class kernels of the other scenes)
      L.bposd = g;
      g += 8 * 30 * A;
      L.bRd = g;
      g += (8 * 90 * A + 255) & ~255;
    }
    if (gl_tbr) {  // the tree-block solve's coupled system (assembled and factored only on coupled substeps)
      L.tbr = g;
      g += (tsize * TB_MAXR * TB_MAXR + 255) & ~255;
    }
    if (gl_gx && spill) {  // the geom centres (the largest array left on the collision side of the union)
      L.gx = g;
      g += (tsize * 4 * ngc + 255) & ~255;
    }
    if (gl_stage) {  // the staged contacts, their keys and pair words (the collision side of the phase-local union)
      L.stage = g;
      g += (tsize * 8 * maxcon + 255) & ~255;
      L.skey = g;
      g += (4 * maxcon + 255) & ~255;
      L.spw = g;
      g += (4 * maxcon + 255) & ~255;
      if (gl_prof) {
        L.prof = g;
        g += (8 * FM_NPROF + 255) & ~255;
      }
    }
    L.gtotal = g;
  }
  return L;
}

// compile-time scene dimensions for the configurations the library specialises (A arms, K objects);
// runtime-only quantities stay members
// runtime dims whose arena workspace exceeds the CU's LDS (fp64 at 4 arms: the dense Newton Hessian alone is
// 141.5 KB at (4, 16)): the Hessian and the contact records live in a per-arena global scratch block (L2-resident,
// flat/global accesses; the wave's program order covers their hand-offs at SYNC() as it does for LDS), everything
// else in LDS.  The parity-grade fp64 build of those scenes.
struct DimsSpill : Dims {
  static constexpr bool spill = true;
  DimsSpill() = default;
  __host__ __device__ DimsSpill(const Dims& d) : Dims(d) {}
};

// WIDE_: the benchmark scene's rerun kernel -- the (2,4) scene at the wide contact capacity, stepping the arenas whose
// env-step the 64-contact kernel abandoned at a stage with more contacts (State::rerun), so no contact is dropped
// Compile-time scenes keep the Newton Hessian and the contact records -- the two largest arrays -- in a per-arena
// global scratch block (L2-resident; a wave's global accesses are ordered like its LDS accesses, so SYNC() covers
// their hand-offs), everything else in LDS: the arena workspace shrinks enough for more arenas per CU (round 4, one
// box: (2,4) fp32 167.9k -> 197.1k env-steps/s with two waves per SIMD, fp64 81.9k -> 105.6k; (4,16) config 5
// 9.5k -> 17.4k with four arenas per CU instead of one).  FM_SPILL_FIXED=0 (experiment builds): all in LDS.
#ifndef FM_SPILL_FIXED
#define FM_SPILL_FIXED 1
#endif
#ifndef FM_GL_LISTS
#define FM_GL_LISTS 1
#endif
#ifndef FM_TREEBLK
#define FM_TREEBLK 1
#endif
#ifndef FM_GL_COLL
#define FM_GL_COLL 1  // round 6: the (2,4) fp64 collision lists in the global block, 145.5k -> 164.3k env-steps/s fp64
#endif
#ifndef FM_GL28
#define FM_GL28 1  // round 6: the fp32 (2,8) collision lists + coupled system in the global block, 193.3k -> 231.4k (config 3)
#endif
#ifndef FM_GL210
#define FM_GL210 1  // round 6: the same for fp32 (2,10), 5 -> 8 arenas per CU, 155.0k -> 202.7k env-steps/s (16384 arenas)
#endif
#ifndef FM_GL416
#define FM_GL416 0
#endif
#ifndef FM_GL_GX
#define FM_GL_GX 1  // round 6: fp64 (2,4) 7 -> 8 arenas per CU, 167.5k -> 191.5k env-steps/s (profiles/r06t_glgx_ab/)
#endif
#ifndef FM_TREEBLK24
#define FM_TREEBLK24 0  // experiment: the (2,4) 64-contact kernel's non-arrowhead substeps through the tree-block solve
#endif
#ifndef FM_F64ARMS_IK
#define FM_F64ARMS_IK 1
#endif
// IKK_: the instantiation the IK classes' launches use (the same layout; only DIM::f64arms differs)
template <int A_, int K_, bool WIDE_ = false, bool IKK_ = false>
struct FixedDims {
  static constexpr bool fixed = true;
  static constexpr bool spill = FM_SPILL_FIXED && !WIDE_;
  static constexpr int A = A_, K = K_, nq = 1 + 7 * K_ + 9 * A_, nv = 1 + 6 * K_ + 9 * A_, nu = 1 + 8 * A_;
  static constexpr bool midcache = true;
  static constexpr int ngc = 13 + K_ + 55 * A_, ncb = 5 + A_ + K_ + 10 * A_, ntree = 1 + K_ + A_;
  static constexpr int maxrow = 10 * A_;
  static constexpr int MAXC = (A_ == 2 && K_ == 4 && !WIDE_) ? MAXCON : MAXCON_WIDE;
  static constexpr bool rerun = WIDE_;
  // the fp32 (4,16) scene (config 5: IK grasps) keeps float64 arm body poses for the narrowphase: a float forward
  // kinematics puts ~1e-7 m on the gripper / arm geoms' positions, which a contact on a cube turns into force errors
  // (tools/fp32_floor.py --probe 64: 1e-7 m of geom noise alone drops the (4,16) Pause toggle to 90 % within)
  // The IK classes' fp32 kernels of the other scenes too: a grasped cube sits between the gripper plates' contacts,
  // and the float arm chain's noise drops the (2,4) Pause toggle to 87 % of its env-steps within the SURVEY gate
  // (worst 0.54) against 100 % for the Backup toggle.  Those poses live in the global block -- both instantiations
  // share one layout, so the non-IK (benchmark) kernels' LDS is unchanged and they never touch the slots.
  static constexpr bool f64ik = spill && !WIDE_ && !(A_ == 4 && K_ == 16) && FM_F64ARMS_IK;
  static constexpr bool f64arms = (A_ == 4 && K_ == 16) || (IKK_ && f64ik);
  // the (4,16) scene also keeps its midphase hit list and float64 arm poses in the global block: 50.0 -> 37.9 KB of
  // LDS, four arenas per CU instead of three
  static constexpr bool gl_lists = spill && A_ == 4 && K_ == 16 && FM_GL_LISTS;
  static constexpr bool f64gl = gl_lists || f64ik;
  // the collision work lists -- staged contacts, keys, pair words and the midphase list -- in the global block too (the
  // larger side of the phase-local union at (2,4)): FM_GL_COLL=1 the fp64 kernel (29.9 KB of LDS hold 5 arenas per CU),
  // 2 both precisions
  template <int TS>
  __host__ __device__ static constexpr bool gl_coll() {
    return spill && !WIDE_ &&
           ((A_ == 2 && K_ == 4 && (FM_GL_COLL == 2 || (FM_GL_COLL == 1 && TS == 8))) ||
            gl2x<TS>());
  }
  // the fp32 (2,8) / (2,10) kernels: collision lists and the tree-block coupled system in the global
  // block (26.1 -> 17.9 KB of LDS at (2,8), 27.4 -> 19.6 KB at (2,10): 8 arenas per CU instead of 6 / 5); FM_GL416=1
  // (experiment) the (4,16) one too
  template <int TS>
  __host__ __device__ static constexpr bool gl2x() {
    return spill && !WIDE_ && TS == 4 &&
           ((A_ == 2 && ((K_ == 8 && FM_GL28) || (K_ == 10 && FM_GL210))) || (A_ == 4 && K_ == 16 && FM_GL416));
  }
  // the tree-block solve's coupled system in the global block (assembled and factored only on coupled substeps)
  template <int TS>
  __host__ __device__ static constexpr bool gl_tbr() {
    return spill && !WIDE_ && treeblk_for<TS>() && (gl2x<TS>() || (A_ == 2 && K_ == 4));
  }
  // the fp64 (2,4) kernel's geom centres in the global block too (22.7 -> 18.7 KB: 8 arenas per CU)
  template <int TS>
  __host__ __device__ static constexpr bool gl_gx() {
    return spill && !WIDE_ && A_ == 2 && K_ == 4 && TS == 8 && FM_GL_GX;
  }
  template <int TS>
  __host__ __device__ static constexpr bool gl_sp() {
    return gl_lists || gl_coll<TS>();
  }
  // the fp32 scenes with spilled records other than (2,4) solve the Newton system tree block by tree block
  // (newton_treeblk): their dense Hessian in the global block is only the fallback for more than TB_MAXR coupled
  // positions
  // (and so does the (2,4) scene's wide rerun kernel: its stages hold 65-128 contacts, where the dense register
  // factor's per-pivot LDS broadcasts cost ~25 ms for one arena's env-step)
  // (the (2,4) 64-contact kernel keeps its arrowhead register factor: with the tree-block code compiled in, round 4
  // measured 175.8k vs 189.5k env-steps/s -- the extra code alone costs its register allocation -- and neither the
  // tree-block solve on every substep nor only on heavy substeps (> 8 contacts on a tree) won that back)
  static constexpr bool treeblk = (WIDE_ || (spill && !(A_ == 2 && K_ == 4))) && FM_TREEBLK;
  // ... and, per precision, the (2,4) 64-contact kernel's non-arrowhead substeps (FM_TREEBLK24: 1 fp32, 2 both)
  template <int TS>
  __host__ __device__ static constexpr bool treeblk_for() {
    return treeblk || (spill && !WIDE_ && A_ == 2 && K_ == 4 && FM_TREEBLK &&
                       (FM_TREEBLK24 == 2 || (FM_TREEBLK24 == 1 && TS == 4)));
  }
  static constexpr int phys_stride = 2 * nq + 3 * nv, dbl_stride = nu + 3 + 2 * A_ + 1 + 27 * A_,
                       int_stride = 2 * K_ + I_NINT + (3 + A_) * A_;
  int N, nbox, npair, nparam, frame_skip, maxcon, ncbp, obs_dim, act_dim;  // obs / act dims depend on the env class
  __host__ __device__ FixedDims(const Dims& d)
      : N(d.N), nbox(d.nbox), npair(d.npair), nparam(d.nparam), frame_skip(d.frame_skip), maxcon(d.maxcon),
        ncbp(d.ncbp), obs_dim(d.obs_dim), act_dim(d.act_dim) {}
  template <int TS>
  __host__ __device__ static constexpr Lay layout() {
    return make_layout(A, K, nq, nv, nu, ngc, ncb, MAXC, maxrow, ntree, TS, spill, midcache, MAXC == WAVE,
                       (A_ == 4 && K_ == 16) || f64ik, gl_sp<TS>(), treeblk_for<TS>(), 0, gl_coll<TS>(), gl_tbr<TS>(),
                       f64gl, gl_gx<TS>());
  }
  static bool matches(const Dims& d) {
    return d.A == A && d.K == K && d.nq == nq && d.nv == nv && d.nu == nu && d.ngc == ngc && d.ncb == ncb &&
           d.ntree == ntree && d.maxrow == maxrow &&
           d.phys_stride == phys_stride && d.dbl_stride == dbl_stride && d.int_stride == int_stride;
  }
};

// the IK classes' instantiation: float64 arm poses in the fp32 kernels (FixedDims::f64ik)
template <typename T, int A, int K>
using FixedDimsIK = FixedDims<A, K, false, sizeof(T) == 4>;

}  // namespace fm
