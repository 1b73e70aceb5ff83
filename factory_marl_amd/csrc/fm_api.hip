// fm_api.hip -- host side of libfactorysim.so: scene upload, workspace layout, kernel dispatch and the
// C ABI declared in include/factorysim.h.  The runtime-dims kernels are instantiated here; the
// compile-time scene kernels live in fm_fixed.hip objects (one per scene in FM_FIXED_SCENES).
#include <cstdio>

#include "fm_device.hpp"
#include "fm_render.hpp"

// scenes with a compile-time specialised env-step kernel: X(num_arms, max_num_objects); must match the
// fm_fixed_<A>_<K>.o objects the Makefile links
#ifndef FM_FIXED_SCENES
#define FM_FIXED_SCENES X(2, 4) X(2, 8) X(2, 10)
#endif
// fp32-only compile-time scenes (fp64 runs them on the runtime-dims spill kernel)
#ifndef FM_FIXED_SCENES32
#define FM_FIXED_SCENES32 X(4, 16)
#endif

namespace fm {
template <typename T, int A, int K>
hipError_t rerun_set_attr();
template <typename T, int A, int K>
Lay rerun_layout();
template <typename T, int A, int K>
void rerun_launch(const StepParams<T>& p, int num_arenas, hipStream_t stream, bool ik);
template <typename T, int A, int K>
hipError_t fixed_set_attr(int lds_bytes);
template <typename T, int A, int K>
void fixed_launch(const StepParams<T>& p, int num_arenas, int lds_bytes, hipStream_t stream, bool ik);
}  // namespace fm

// =================================================================================================
// host side: handle, uploads, C ABI
// =================================================================================================
using namespace fm;

// the CPU backend's kernels (fm_cpu.cpp: fm_device.hpp compiled for the host, the wave emulated; fm_cpu_fixed.cpp: the
// compile-time scenes, one entry per scene -- wide = 1 the (2,4) float64 wide rerun kernel)
extern "C" void fm_cpu_step(int fp64, const void* params, int num_arenas, int lds_bytes, int ik);
#define X(a, k) extern "C" int fm_cpu_step_fixed_##a##_##k(int fp64, int wide, const void* params, int grid, int lds_bytes, int ik);
FM_FIXED_SCENES
FM_FIXED_SCENES32
X(2, 4)  // always linked (the wide rerun kernel)
#undef X
extern "C" void fm_cpu_reset(int fp64, const void* model, const void* state, const void* lay, float* obs,
                             const uint8_t* mask, int num_arenas, int lds_bytes);
extern "C" void fm_cpu_debug(int fp64, const void* model, const void* state, const void* lay, int arena, int actuated,
                             double* out, int lds_bytes);
namespace fm {
template <typename T>
static void cpu_step(const StepParams<T>& p, int num_arenas, int lds_bytes, bool ik) {
  fm_cpu_step(sizeof(T) == 8, &p, num_arenas, lds_bytes, ik ? 1 : 0);
}
template <typename T>
static void cpu_reset(const Model<T>& M, const State<T>& S, const Lay& L, float* obs, const uint8_t* mask,
                      int num_arenas, int lds_bytes) {
  fm_cpu_reset(sizeof(T) == 8, &M, &S, &L, obs, mask, num_arenas, lds_bytes);
}
template <typename T>
static void cpu_debug(const Model<T>& M, const State<T>& S, const Lay& L, int arena, int actuated, double* out,
                      int lds_bytes) {
  fm_cpu_debug(sizeof(T) == 8, &M, &S, &L, arena, actuated, out, lds_bytes);
}
}  // namespace fm

static thread_local std::string g_err;

static int set_err(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                                  \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) return set_err(FM_EDEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct fm_handle {
  fm_config cfg;
  SceneHost sc;
  Dims dm;
  int device = 0;
  hipStream_t stream = nullptr;      // stream every call runs on (the private one or the caller's)
  hipStream_t own_stream = nullptr;  // the private stream fm_create made; the only one fm_destroy destroys
  hipEvent_t handoff = nullptr;      // orders a new stream after the work queued on the previous one
  bool fp64 = false;
  bool cpu = false;  // device = -1: the CPU backend (fm_cpu.cpp), every array in host memory
  bool was_reset = false;
  Lay lay;
  std::vector<void*> allocs;
  // device model arrays: the precision-typed ones (and the frame-dependent float64 geom table) per kernel precision
  // -- `tab` for the handle's own kernels, `tab64` (fp32 handles of the benchmark scene) for the float64 wide rerun
  // kernel, which steps the abandoned env-steps of both builds
  struct Tables {
    void* arm_base = nullptr;
    void* body = nullptr;
    void* dof = nullptr;
    void* ctrlrange = nullptr;
    void* geom = nullptr;
    void* geomd = nullptr;  // float64, but in the kernel frame of its precision (zshift)
    void* cbs = nullptr;
    void* cube = nullptr;
    void* meaninertia = nullptr;
  } tab, tab64;
  double* ctrlrange_d = nullptr;
  double* arm_base_w = nullptr;
  double* dofd = nullptr;
  int* geom_i = nullptr;
  int* ginfo = nullptr;
  int* cbi = nullptr;
  uint16_t* cbg = nullptr;
  uint32_t* cbp = nullptr;
  uint32_t* pair = nullptr;
  void* param = nullptr;
  uint32_t* tri = nullptr;
  // state
  void* phys = nullptr;
  double* dbl = nullptr;
  int32_t* ints = nullptr;
  uint64_t* rng = nullptr;
  int64_t* counters = nullptr;
  uint32_t* cost = nullptr;   // [N] last env-step duration per arena (s_memrealtime ticks)
  int32_t* order = nullptr;   // [N] dispatch order of the next env-step, longest first
  unsigned long long* prof = nullptr;
  // rendering (fm_render): colour tables uploaded on first use, scratch grown on demand
  float* render_rgb = nullptr;   // [ngc][4]
  float* cube_rgba = nullptr;    // [N][K][4]
  float* render_frames = nullptr;
  int* render_arenas = nullptr;
  int* render_arenas_host = nullptr;   // pinned staging of the arena list (async H2D on the stream)
  hipEvent_t render_copied = nullptr;  // the last staging copy has been consumed
  size_t render_cap = 0;          // arenas the scratch holds
  bool prof_on = false;
  int fixed = -1;  // index into FM_FIXED_SCENES, -1 = runtime-dims kernel
  Lay lay_step{};  // workspace layout of the env-step kernel in use
  bool spill = false;          // DimsSpill: Hessian + contact records in per-arena global scratch (fp64, > 160 KiB)
  uint32_t xflags = 0;         // the experiment build's switches (Model::dbg_flags): read at fm_create, fm_set_param
  // the benchmark scene's lossless contacts: [1 + N] rerun list of the 64-contact launch (fm_dev.hpp State::rerun),
  // the IK classes' record backup, the (float64) wide kernel's layout
  int32_t* rerun = nullptr;
  char* bak = nullptr;
  double* resume = nullptr;    // [N][resume_stride] substep state of an abandoned env-step
  Lay lay_rerun{};
  char* spill_buf = nullptr;   // [N][spill_stride]
  bool ktime_on = false;                                   // fm_kernel_timing
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ktime;  // one event pair per step-kernel launch since the last read
  long long spill_stride = 0;  // Lay::gtotal of the spill layout in use (compile-time scenes; runtime fp64 (4,16))
};

// memory of the handle's arrays: device memory, or host memory for the CPU backend (device = -1)
template <typename P>
static hipError_t d_malloc(fm_handle* h, P** p, size_t n) {
  if (h->cpu) {
    *p = (P*)std::calloc(n ? n : 1, 1);
    return *p ? hipSuccess : hipErrorOutOfMemory;
  }
  return hipMalloc((void**)p, n);
}
static hipError_t d_free(fm_handle* h, void* p) {
  if (h->cpu) {
    std::free(p);
    return hipSuccess;
  }
  return hipFree(p);
}
static hipError_t d_memcpy(fm_handle* h, void* dst, const void* src, size_t n, hipMemcpyKind k) {
  if (h->cpu) {
    if (n) std::memcpy(dst, src, n);
    return hipSuccess;
  }
  return hipMemcpy(dst, src, n, k);
}
static hipError_t d_memset(fm_handle* h, void* p, int v, size_t n) {
  if (h->cpu) {
    std::memset(p, v, n);
    return hipSuccess;
  }
  return hipMemset(p, v, n);
}
static hipError_t d_setdev(fm_handle* h) { return h->cpu ? hipSuccess : hipSetDevice(h->device); }
static hipError_t d_sync(fm_handle* h) { return h->cpu ? hipSuccess : hipStreamSynchronize(h->stream); }

template <typename T>
static int upload(fm_handle* h, void** dst, const std::vector<double>& src) {
  std::vector<T> tmp(src.size());
  for (size_t i = 0; i < src.size(); i++) tmp[i] = (T)src[i];
  size_t bytes = std::max<size_t>(tmp.size(), 1) * sizeof(T);
  HIPCHK(d_malloc(h, dst, bytes));
  h->allocs.push_back(*dst);
  if (!tmp.empty()) HIPCHK(d_memcpy(h, *dst, tmp.data(), tmp.size() * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

template <typename U>
static int upload_raw(fm_handle* h, U** dst, const std::vector<U>& src) {
  size_t bytes = std::max<size_t>(src.size(), 1) * sizeof(U);
  HIPCHK(d_malloc(h, (void**)dst, bytes));
  h->allocs.push_back(*dst);
  if (!src.empty()) HIPCHK(d_memcpy(h, *dst, src.data(), src.size() * sizeof(U), hipMemcpyHostToDevice));
  return 0;
}

static Lay lds_layout(const Dims& d, int tsize, bool spill = false) {
  return make_layout(d.A, d.K, d.nq, d.nv, d.nu, d.ngc, d.ncb, d.maxcon, d.maxrow, d.ntree, tsize, spill, false, false,
                     false, false, false, Dims::MAXC / WAVE);
}

template <typename T>
static Model<T> make_model(const fm_handle* h) {
  Model<T> M;
  M.dm = h->dm;
  M.dt = T(0.001);
  M.timestep = 0.001;
  M.grav = T(9.81);
  M.grav_d = 9.81;
  M.belt_mass = T(1000);
  M.belt_kv = T(1e4);
  M.belt_damp = T(5e-4);
  M.belt_invw_t = T((1.0 / 1000.0) / 3.0);
  const fm_config& c = h->cfg;
  M.init_speed = c.initial_conveyor_speed;
  M.accel = c.conveyor_acceleration;
  M.pt_time = c.pt_time;
  M.force_thr = c.force_contact_threshold;
  M.spawn_freq0 = c.spawn_freq * h->dm.A;
  M.spawn_inc = c.spawn_freq_increase;
  M.w_grip = c.gripper_to_closest_cube_reward_factor;
  M.w_bucket = c.closest_cube_to_bucket_reward_factor;
  M.w_action = c.small_action_norm_reward_factor;
  M.base_reward = c.base_reward;
  M.bucket_x0 = h->sc.bucket_x[0];
  M.bucket_x1 = h->sc.bucket_x[1];
  M.bucket_y = h->sc.bucket_y;
  M.bucket_z = h->sc.bucket_z;
  M.env_class = c.env_class;
  M.solver_iter = c.solver_iterations;
  M.solver_tol = c.solver_tolerance;
  {
    const double dt = 0.001 * h->dm.frame_skip;  // env.dt = model.opt.timestep * frame_skip (base_env.py:201-202)
    M.ik_time.pt_comp = c.pt_time * dt * 15.0;
    M.ik_time.release_wait = (int)(0.5 / dt);
    M.ik_time.grasp_wait = (int)(1.0 / dt);
    M.ik_time.move_steps = (int)(1.0 / dt);
    M.ik_time.timeout_steps = (int)(3.0 / dt);
  }
  // a float64 model of an fp32 handle: the float64 wide rerun kernel's tables
  const fm_handle::Tables& t = (sizeof(T) == 8 && !h->fp64) ? h->tab64 : h->tab;
  M.arm_base = (const T*)t.arm_base;
  M.arm_base_w = h->arm_base_w;
  M.body = (const T*)t.body;
  M.dof = (const T*)t.dof;
  M.dofd = h->dofd;
  M.ctrlrange = (const T*)t.ctrlrange;
  M.ctrlrange_d = h->ctrlrange_d;
  M.geom = (const T*)t.geom;
  M.geomd = (const double*)t.geomd;
  M.geom_i = h->geom_i;
  M.pair = h->pair;
  M.ginfo = h->ginfo;
  M.cbi = h->cbi;
  M.cbs = (const T*)t.cbs;
  M.cbg = h->cbg;
  M.cbp = h->cbp;
  for (int a = 0; a < 5; a++)
    for (int b = 0; b < 5; b++) M.ptab[5 * a + b] = h->sc.ptab[a][b];
  M.param = (const double*)h->param;
  M.cube = (const T*)t.cube;
  M.meaninertia = (const T*)t.meaninertia;
  M.tri = h->tri;
  M.prof = h->prof_on ? h->prof : nullptr;
#if FM_EXPERIMENTS
  M.dbg_flags = h->xflags;
#endif
  M.ovf_abort = 0;
  M.obs64 = c.obs_float64 != 0;
  return M;
}

// the experiment build's switches (libfactorysim_exp.so, FM_EXPERIMENTS=1: the equivalence tests' reference forms and
// the rerun path's test hooks; every default is 0): read from the environment once, at fm_create, and reported on
// stderr when any is set; "experiment_flags" (fm_set_param) changes them on a live handle for later launches.  The
// product library has none (FM_XF is 0 in its kernels; fm_set_param rejects "experiment_flags")
constexpr uint32_t FM_XFLAGS_MASK = 2u | 4u | 8u | 16u | 512u | 1024u | 2048u | 16384u;
static uint32_t read_experiment_flags() {
#if FM_EXPERIMENTS
  struct Sw {
    const char* var;
    char val;
    uint32_t bit;
  };
  static const Sw sw[] = {
      {"FM_CHOL_LDS", '2', 2},         // (4,16): the sparse LDS Cholesky of the dense Hessian (no tree-block solve)
      {"FM_SERIAL_BOXBOX", '1', 4},    // one lane per box-box pair throughout
      {"FM_NO_MIDCACHE", '1', 8},      // the midphase list rebuilt at every substep
      {"FM_NO_ARROW", '1', 16},        // no block-parallel arrowhead Cholesky
      {"FM_FORCE_RERUN", '1', 512},    // (2,4): every env-step abandoned at its first stage and run by the wide kernel
      {"FM_NO_RERUN", '1', 1024},      // (2,4): contacts above 64 cut (counted), no wide rerun
      {"FM_NO_TREEBLK", '1', 2048},    // (2,8), (2,10), (4,16) fp32, wide rerun: the dense Hessian + factors on every substep
      {"FM_RERUN_AT_50", '1', 16384},  // (2,4): every env-step abandoned at substep 50, resumed there by the wide kernel
  };
  uint32_t f = 0;
  for (const Sw& x : sw) {
    const char* v = getenv(x.var);
    if (v && v[0] == x.val) f |= x.bit;
  }
  if (f) fprintf(stderr, "factorysim: experiment switches active (flags 0x%x)\n", f);
  return f;
#else
  return 0u;
#endif
}

template <typename T>
static State<T> make_state(const fm_handle* h) {
  State<T> S;
  S.phys = (double*)h->phys;
  S.dbl = h->dbl;
  S.ints = h->ints;
  S.rng = h->rng;
  S.counters = h->counters;
  S.cost = h->cost;
  S.order = h->order;
  S.spill = h->spill_buf;
  S.spill_stride = h->spill_stride;
  return S;
}

// the scene tables a kernel of precision U reads in its own kernel frame (zshift<U>()): arm bases, the arm template,
// dof ranges, control ranges, geoms (U and float64), collision-body bounds, cube sizes, mean inertia
template <typename U>
static int upload_tables(fm_handle* h, fm_handle::Tables& t) {
  const SceneHost& s = h->sc;
  std::vector<double> arm_base(12 * s.A), body(32 * ARM_NB, 0.0), dof(4 * ARM_ND, 0.0), ctrl(2 * s.nu);
  for (int i = 0; i < s.A; i++)
    for (int k = 0; k < 12; k++) arm_base[12 * i + k] = s.arm_base[i][k];
  // world -> kernel frame (zshift, fm_dev.hpp): every absolute position the kernel reads
  const double zs = zshift<U>();
  for (int i = 0; i < s.A; i++) arm_base[12 * i + 2] -= zs;
  for (int b = 0; b < ARM_NB; b++) {
    double* o = &body[32 * b];
    for (int k = 0; k < 12; k++) o[k] = s.body_local[b][k];
    o[12] = s.body_mass[b];
    for (int k = 0; k < 3; k++) o[13 + k] = s.body_ipos[b][k];
    for (int k = 0; k < 9; k++) o[16 + k] = s.body_iR[b][k];
    for (int k = 0; k < 3; k++) o[25 + k] = s.body_I[b][k];
    o[28] = s.body_invw[b][0];
    o[29] = s.body_invw[b][1];
    // the kernel folds ARM_BODY (fm_arm_table.hpp, generated at build time) into immediates: the scene
    // compiled now must be the one the library was built with
    for (int k = 0; k < 30; k++)
      if (o[k] != ARM_BODY[b][k]) {
        return set_err(FM_EINVAL, "arm template differs from the constants compiled into the kernel (rebuild)");
      }
  }
  for (int j = 0; j < ARM_ND; j++) {
    dof[4 * j] = s.dof_range[j][0];
    dof[4 * j + 1] = s.dof_range[j][1];
    dof[4 * j + 2] = s.dof_invw[j];
  }
  for (int u = 0; u < s.nu; u++) {
    ctrl[2 * u] = s.ctrlrange[u][0];
    ctrl[2 * u + 1] = s.ctrlrange[u][1];
  }
  const int ngc = (int)s.geoms.size();
  std::vector<double> geom(16 * ngc, 0.0);
  for (int g = 0; g < ngc; g++) {
    const GeomRec& r = s.geoms[g];
    for (int k = 0; k < 3; k++) geom[16 * g + k] = r.pos[k];
    if (r.kbody == 0) geom[16 * g + 2] -= zs;  // static geoms: world positions
    for (int k = 0; k < 9; k++) geom[16 * g + 3 + k] = r.R[k];
    for (int k = 0; k < 3; k++) geom[16 * g + 12 + k] = r.size[k];
    geom[16 * g + 15] = r.rbound;
  }
  // cube bounding radius depends on the per-arena size: use the largest possible (h <= 0.05)
  for (int g = 0; g < ngc; g++)
    if (s.geoms[g].kbody >= 2 && s.geoms[g].kbody < 2 + s.K) geom[16 * g + 15] = std::sqrt(3.0) * 0.05;
  std::vector<double> cbs(8 * s.cbodies.size(), 0.0);
  for (size_t b = 0; b < s.cbodies.size(); b++) {
    const CBody& c = s.cbodies[b];
    for (int k = 0; k < 3; k++) {
      cbs[8 * b + k] = c.c[k];
      cbs[8 * b + 4 + k] = c.e[k];
    }
    cbs[8 * b + 3] = c.r;
    if (c.flags & CB_STATIC) cbs[8 * b + 2] -= zs;
  }
  // slot 3: the rounding residue of the half size in this precision (0 in fp64), so the float64 narrowphase of the
  // fp32 build reads h exactly as (double)[0] + (double)[3]
  std::vector<double> cb = s.cube;
  for (size_t i = 0; i < cb.size(); i += 4) cb[i + 3] = cb[i] - (double)(U)cb[i];
  int r;
  if ((r = upload<U>(h, &t.arm_base, arm_base))) return r;
  if ((r = upload<U>(h, &t.body, body))) return r;
  if ((r = upload<U>(h, &t.dof, dof))) return r;
  if ((r = upload<U>(h, &t.ctrlrange, ctrl))) return r;
  if ((r = upload<U>(h, &t.geom, geom))) return r;
  if ((r = upload<double>(h, &t.geomd, geom))) return r;
  if ((r = upload<U>(h, &t.cbs, cbs))) return r;
  if ((r = upload<U>(h, &t.cube, cb))) return r;
  if ((r = upload<U>(h, &t.meaninertia, s.meaninertia))) return r;
  return 0;
}

template <typename T>
static int create_typed(fm_handle* h) {
  const SceneHost& s = h->sc;
  const Dims& d = h->dm;
  int r;
  if ((r = upload_tables<T>(h, h->tab))) return r;
  {
    std::vector<double> bw(12 * s.A), dof(4 * ARM_ND, 0.0), ctrl(2 * s.nu);
    for (int i = 0; i < s.A; i++)
      for (int k = 0; k < 12; k++) bw[12 * i + k] = s.arm_base[i][k];
    for (int j = 0; j < ARM_ND; j++) {
      dof[4 * j] = s.dof_range[j][0];
      dof[4 * j + 1] = s.dof_range[j][1];
      dof[4 * j + 2] = s.dof_invw[j];
    }
    for (int u = 0; u < s.nu; u++) {
      ctrl[2 * u] = s.ctrlrange[u][0];
      ctrl[2 * u + 1] = s.ctrlrange[u][1];
    }
    if ((r = upload_raw<double>(h, &h->arm_base_w, bw))) return r;
    if ((r = upload_raw<double>(h, &h->dofd, dof))) return r;
    if ((r = upload_raw<double>(h, &h->ctrlrange_d, ctrl))) return r;
  }
  const int ngc = (int)s.geoms.size();
  std::vector<double> param(8 * s.params.size(), 0.0);
  std::vector<int> geom_i(4 * ngc);
  for (int g = 0; g < ngc; g++) {
    const GeomRec& gr = s.geoms[g];
    geom_i[4 * g] = gr.mjid;
    geom_i[4 * g + 1] = gr.type;
    geom_i[4 * g + 2] = gr.kbody;
    geom_i[4 * g + 3] = s.box_slot[g];
  }
  for (size_t p = 0; p < s.params.size(); p++) {
    param[8 * p] = s.params[p].mu;
    param[8 * p + 1] = s.params[p].solref[0];
    param[8 * p + 2] = s.params[p].solref[1];
    for (int k = 0; k < 5; k++) param[8 * p + 3 + k] = s.params[p].solimp[k];
  }
  if ((r = upload_raw<int>(h, &h->geom_i, geom_i))) return r;
  if ((r = upload_raw<uint32_t>(h, &h->pair, s.pairs))) return r;
  {
    std::vector<int> gin(ngc), cbi(4 * s.cbodies.size());
    for (int g = 0; g < ngc; g++) {
      const GeomRec& G = s.geoms[g];
      int tc = G.type == GT_PLANE ? GC_PLANE : (G.type == GT_SPHERE ? GC_SPHERE : GC_BOX);
      int arm = G.mjid >= 13 + s.K ? 1 : 0;
      gin[g] = tc | (arm << GI_ARM) | (G.pclass << GI_PC) | (G.kbody << 8);
    }
    for (size_t b = 0; b < s.cbodies.size(); b++) {
      const CBody& c = s.cbodies[b];
      cbi[4 * b] = c.kbody;
      cbi[4 * b + 1] = c.flags;
      cbi[4 * b + 2] = c.g0;
      cbi[4 * b + 3] = c.ng;
    }
    if ((r = upload_raw<int>(h, &h->ginfo, gin))) return r;
    if ((r = upload_raw<int>(h, &h->cbi, cbi))) return r;
    if ((r = upload_raw<uint16_t>(h, &h->cbg, s.cb_geoms))) return r;
    if ((r = upload_raw<uint32_t>(h, &h->cbp, s.cb_pairs))) return r;
  }
  if ((r = upload<double>(h, &h->param, param))) return r;
  if ((r = upload_raw<uint32_t>(h, &h->tri, s.tri))) return r;
  // state
  size_t N = d.N;
  // the physics state is float64 in both precisions (fp32 computes from float copies of it)
  HIPCHK(d_malloc(h, &h->phys, N * d.phys_stride * sizeof(double)));
  h->allocs.push_back(h->phys);
  HIPCHK(d_memset(h, h->phys, 0, N * d.phys_stride * sizeof(double)));
  HIPCHK(d_malloc(h, (void**)&h->dbl, N * d.dbl_stride * sizeof(double)));
  h->allocs.push_back(h->dbl);
  HIPCHK(d_malloc(h, (void**)&h->ints, N * d.int_stride * sizeof(int32_t)));
  h->allocs.push_back(h->ints);
  {
    // IKPolicy.__init__ (ik_policy.py:76-81) + PauseIKToggleEnv.last_arm_actions (environments.py:592): idle,
    // no target, nothing ignored, last_ctrl = default pose; the rest is written by fm_reset
    std::vector<double> db(N * d.dbl_stride, 0.0);
    std::vector<int32_t> in(N * d.int_stride, 0);
    for (size_t n = 0; n < N; n++)
      for (int i = 0; i < d.A; i++) {
        double* dd = db.data() + n * d.dbl_stride + d.nu + 4 + 2 * d.A + 27 * i;
        for (int j = 0; j < 8; j++) dd[j] = IK_DEFAULT_POSE[j];
        int32_t* ii = in.data() + n * d.int_stride + 2 * d.K + I_NINT + (3 + d.A) * i;
        ii[2] = -1;
        for (int o = 0; o < d.A; o++) ii[3 + o] = -1;
      }
    HIPCHK(d_memcpy(h, h->dbl, db.data(), db.size() * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(d_memcpy(h, h->ints, in.data(), in.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  }
  if ((r = upload_raw<uint64_t>(h, &h->rng, s.rng_init))) return r;
  HIPCHK(d_malloc(h, (void**)&h->counters, N * FM_NCTR * sizeof(int64_t)));
  h->allocs.push_back(h->counters);
  HIPCHK(d_memset(h, h->counters, 0, N * FM_NCTR * sizeof(int64_t)));
  if (!getenv("FACTORYSIM_NO_LPT") && !h->cpu) {  // experiment switch: plain blockIdx -> arena dispatch
    HIPCHK(d_malloc(h, (void**)&h->cost, N * sizeof(uint32_t)));
    h->allocs.push_back(h->cost);
    HIPCHK(d_memset(h, h->cost, 0, N * sizeof(uint32_t)));
    HIPCHK(d_malloc(h, (void**)&h->order, N * sizeof(int32_t)));
    h->allocs.push_back(h->order);
  }
  h->lay = lds_layout(d, sizeof(T));
  // CPU backend: the compile-time scenes run their own kernels as on the GPU (fm_cpu_fixed.cpp: spill layouts, the
  // (2,4) wide rerun); other scenes the runtime-dims kernel with its whole workspace in the emulated wave's host "LDS"
  // (no 160 KiB limit, no DimsSpill layout); no dispatch order
  if (h->lay.total > 160 * 1024 && !h->cpu) {
    if constexpr (sizeof(T) == 8) {
      // fp64 scenes beyond the CU's LDS (4 arms): the parity-grade spill layout (DimsSpill, fm_dev.hpp)
      h->lay = lds_layout(d, sizeof(T), true);
      if (h->lay.total > 160 * 1024) return set_err(FM_EINVAL, "arena workspace exceeds 160 KiB of LDS");
      h->spill = true;
      h->spill_stride = h->lay.gtotal;
      HIPCHK(d_malloc(h, (void**)&h->spill_buf, (size_t)d.N * (size_t)h->lay.gtotal));
      h->allocs.push_back(h->spill_buf);
      HIPCHK(hipFuncSetAttribute((const void*)reset_kernel<T, DimsSpill>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 h->lay.total));
      HIPCHK(hipFuncSetAttribute((const void*)step_kernel<T, DimsSpill, true>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, h->lay.total));
      HIPCHK(hipFuncSetAttribute((const void*)step_kernel<T, DimsSpill, false>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, h->lay.total));
      h->lay_step = h->lay;
      return 0;
    } else {
      return set_err(FM_EINVAL, "arena workspace exceeds 160 KiB of LDS");
    }
  }
  if (!h->cpu)
    HIPCHK(hipFuncSetAttribute((const void*)reset_kernel<T, Dims>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               h->lay.total));
  // env-step kernel: a compile-time specialisation when the scene is one of FM_FIXED_SCENES
  h->fixed = -1;
  const char* force_dyn = getenv("FM_FORCE_DYNAMIC");
  int idx = 0;
#define X(a, k)                                                                                          \
  if (h->fixed < 0 && !(force_dyn && force_dyn[0] == '1') && FixedDims<a, k>::matches(d)) {             \
    h->fixed = idx;                                                                                      \
    h->lay_step = FixedDims<a, k>::template layout<sizeof(T)>();                                         \
    if (!h->cpu) HIPCHK((fixed_set_attr<T, a, k>(h->lay_step.total)));                                    \
  }                                                                                                      \
  idx++;
  FM_FIXED_SCENES
#undef X
  if constexpr (sizeof(T) == 4) {
#define X(a, k)                                                                                          \
  if (h->fixed < 0 && !(force_dyn && force_dyn[0] == '1') && FixedDims<a, k>::matches(d)) {             \
    h->fixed = idx;                                                                                      \
    h->lay_step = FixedDims<a, k>::template layout<sizeof(T)>();                                         \
    if (!h->cpu) HIPCHK((fixed_set_attr<T, a, k>(h->lay_step.total)));                                    \
  }                                                                                                      \
  idx++;
    FM_FIXED_SCENES32
#undef X
  }
  (void)idx;
  if (h->fixed >= 0 && h->lay_step.spill) {  // compile-time scenes: the Hessian + contact records in global scratch
    h->spill_stride = h->lay_step.gtotal;
    HIPCHK(d_malloc(h, (void**)&h->spill_buf, (size_t)d.N * (size_t)h->lay_step.gtotal));
    h->allocs.push_back(h->spill_buf);
    // the CPU backend's uninitialised-read probe (FACTORYSIM_CPU_POISON, fm_cpu.cpp): scratch blocks filled with the
    // poison byte, as the GPU's hold whatever the allocation held
    const char* pz = h->cpu ? getenv("FACTORYSIM_CPU_POISON") : nullptr;
    if (pz) std::memset(h->spill_buf, atoi(pz), (size_t)d.N * (size_t)h->lay_step.gtotal);
  }
  // the benchmark scene at its 64-contact capacity: an env-step with a stage above it is rerun by the wide kernel
  // The wide kernel runs in float64 for both builds (an abandoned env-step is rare -- about one arena in 60,000 --
  // and its 65-128 stiff contacts, arms pressed into the table, belt and each other with the gripper plates' small
  // masses among them, are where a float32 Hessian misses the SURVEY gate: round 5 measured 2.7e-2 on such states);
  // fp32 handles upload the float64 tables it reads
  if (h->fixed >= 0 && FixedDims<2, 4>::matches(d) && d.maxcon == MAXCON) {
    if constexpr (sizeof(T) == 4) {
      if ((r = upload_tables<double>(h, h->tab64))) return r;
    }
    if (!h->cpu) HIPCHK((rerun_set_attr<double, 2, 4>()));
    h->lay_rerun = rerun_layout<double, 2, 4>();
    HIPCHK(d_malloc(h, (void**)&h->rerun, (N + 1) * sizeof(int32_t)));
    h->allocs.push_back(h->rerun);
    HIPCHK(d_memset(h, h->rerun, 0, (N + 1) * sizeof(int32_t)));
    // the substep state of an abandoned env-step (the wide kernel resumes from it, fm_dev.hpp State::resume)
    HIPCHK(d_malloc(h, (void**)&h->resume, N * (size_t)resume_stride(d.nq, d.nv, d.nu) * sizeof(double)));
    h->allocs.push_back(h->resume);
    HIPCHK(d_memset(h, h->resume, 0, N * (size_t)resume_stride(d.nq, d.nv, d.nu) * sizeof(double)));
    if (h->cfg.env_class != FM_ENV_ALLFULLRL_PROGRESS) {
      HIPCHK(d_malloc(h, (void**)&h->bak, N * (8 * (size_t)d.dbl_stride + 4 * (size_t)d.int_stride)));
      h->allocs.push_back(h->bak);
    }
  }
  if (h->fixed < 0) {
    h->lay_step = h->lay;
    if (!h->cpu) {
      HIPCHK(hipFuncSetAttribute((const void*)step_kernel<T, Dims, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 h->lay.total));
      HIPCHK(hipFuncSetAttribute((const void*)step_kernel<T, Dims, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 h->lay.total));
    }
  }
  return 0;
}

static int state_record_size(const fm_handle* h) {
  return (int)((h->dm.phys_stride + h->dm.dbl_stride) * sizeof(double) + h->dm.int_stride * sizeof(int32_t) +
               4 * sizeof(uint64_t));
}

template <typename T>
static int get_state_typed(fm_handle* h, char* out) {
  const Dims& d = h->dm;
  size_t N = d.N;
  std::vector<double> ph(N * d.phys_stride);
  std::vector<double> db(N * d.dbl_stride);
  std::vector<int32_t> in(N * d.int_stride);
  std::vector<uint64_t> rg(N * 4);
  HIPCHK(d_sync(h));
  HIPCHK(d_memcpy(h, ph.data(), h->phys, ph.size() * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(d_memcpy(h, db.data(), h->dbl, db.size() * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(d_memcpy(h, in.data(), h->ints, in.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
  HIPCHK(d_memcpy(h, rg.data(), h->rng, rg.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  size_t rec = state_record_size(h);
  for (size_t n = 0; n < N; n++) {
    char* o = out + n * rec;
    double* dp = (double*)o;
    for (int i = 0; i < d.phys_stride; i++) dp[i] = ph[n * d.phys_stride + i];
    for (int i = 0; i < d.dbl_stride; i++) dp[d.phys_stride + i] = db[n * d.dbl_stride + i];
    int32_t* ip = (int32_t*)(o + (d.phys_stride + d.dbl_stride) * sizeof(double));
    for (int i = 0; i < d.int_stride; i++) ip[i] = in[n * d.int_stride + i];
    uint64_t* up = (uint64_t*)(o + (d.phys_stride + d.dbl_stride) * sizeof(double) + d.int_stride * sizeof(int32_t));
    for (int i = 0; i < 4; i++) up[i] = rg[n * 4 + i];
  }
  return FM_OK;
}

template <typename T>
static int set_state_typed(fm_handle* h, const char* src) {
  const Dims& d = h->dm;
  size_t N = d.N;
  std::vector<double> ph(N * d.phys_stride);
  std::vector<double> db(N * d.dbl_stride);
  std::vector<int32_t> in(N * d.int_stride);
  std::vector<uint64_t> rg(N * 4);
  size_t rec = state_record_size(h);
  for (size_t n = 0; n < N; n++) {
    const char* o = src + n * rec;
    const double* dp = (const double*)o;
    for (int i = 0; i < d.phys_stride; i++) ph[n * d.phys_stride + i] = dp[i];
    for (int i = 0; i < d.dbl_stride; i++) db[n * d.dbl_stride + i] = dp[d.phys_stride + i];
    const int32_t* ip = (const int32_t*)(o + (d.phys_stride + d.dbl_stride) * sizeof(double));
    for (int i = 0; i < d.int_stride; i++) in[n * d.int_stride + i] = ip[i];
    const uint64_t* up =
        (const uint64_t*)(o + (d.phys_stride + d.dbl_stride) * sizeof(double) + d.int_stride * sizeof(int32_t));
    for (int i = 0; i < 4; i++) rg[n * 4 + i] = up[i];
  }
  HIPCHK(d_sync(h));
  HIPCHK(d_memcpy(h, h->phys, ph.data(), ph.size() * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(d_memcpy(h, h->dbl, db.data(), db.size() * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(d_memcpy(h, h->ints, in.data(), in.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  HIPCHK(d_memcpy(h, h->rng, rg.data(), rg.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
  h->was_reset = true;
  return FM_OK;
}

// Longest-processing-time-first order of the next env-step's workgroups: a counting sort of the arenas by
// their last env-step duration (256 buckets of the range [0, max], longest first) in one workgroup.  The step
// kernel runs N workgroups over a few hundred CUs several rounds deep; with the plain order the kernel ends when
// the last expensive arena dispatched late finishes.  Order within a bucket is arbitrary (LDS atomics).
__global__ void __launch_bounds__(1024) lpt_order_kernel(const uint32_t* __restrict__ cost, int32_t* __restrict__ order,
                                                          int n) {
  __shared__ unsigned hist[256];
  __shared__ unsigned cmax;
  const int t = (int)threadIdx.x;
  if (t < 256) hist[t] = 0u;
  if (t == 0) cmax = 0u;
  __syncthreads();
  unsigned m = 0u;
  for (int i = t; i < n; i += (int)blockDim.x) m = cost[i] > m ? cost[i] : m;
  atomicMax(&cmax, m);
  __syncthreads();
  const unsigned long long range = (unsigned long long)cmax + 1ull;
  auto bucket = [&](int i) { return 255u - (unsigned)(((unsigned long long)cost[i] * 256ull) / range); };
  for (int i = t; i < n; i += (int)blockDim.x) atomicAdd(&hist[bucket(i)], 1u);
  __syncthreads();
  if (t == 0) {
    unsigned sum = 0u;
    for (int b = 0; b < 256; b++) {
      const unsigned c = hist[b];
      hist[b] = sum;
      sum += c;
    }
  }
  __syncthreads();
  for (int i = t; i < n; i += (int)blockDim.x) order[atomicAdd(&hist[bucket(i)], 1u)] = i;
}

// the wide-capacity rerun of the arenas the 64-contact launch abandoned, after it on the same stream: the float64
// kernel for both builds (a small grid; the workgroups past the list's count exit at once)
static void launch_rerun(fm_handle* h, const StepIO& io, bool ik) {
  StepParams<double> pr{make_model<double>(h), make_state<double>(h), h->lay_rerun, io};
  pr.S.order = nullptr;
  pr.S.rerun = h->rerun;
  pr.S.bak = h->bak;
  pr.S.resume = h->resume;
  pr.M.dm.maxcon = MAXCON_WIDE;  // the wide kernel keeps up to 128 contacts per stage
  rerun_launch<double, 2, 4>(pr, h->dm.N, h->stream, ik);
}

// kernel-only timing (fm_kernel_timing): a HIP event pair on the handle's stream around each env-step kernel launch
// -- the step kernel alone, without the dispatch-order kernel, the rerun-list reset or the wide rerun launch
static void ktime_begin(fm_handle* h) {
  if (!h->ktime_on) return;
  hipEvent_t a = nullptr, b = nullptr;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
  (void)hipEventRecord(a, h->stream);
  h->ktime.push_back({a, b});
}
static void ktime_end(fm_handle* h) {
  if (h->ktime_on && !h->ktime.empty()) (void)hipEventRecord(h->ktime.back().second, h->stream);
}
static void ktime_clear(fm_handle* h) {
  for (auto& e : h->ktime) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  h->ktime.clear();
}

// the CPU backend's env-step: the scene's compile-time kernel (and the (2,4) wide rerun after it) as on the GPU, or
// the runtime-dims kernel
template <typename T>
static void launch_step_cpu(fm_handle* h, const StepIO& io) {
  const bool ik = h->cfg.env_class != FM_ENV_ALLFULLRL_PROGRESS;
  const int fp64 = sizeof(T) == 8;
  StepParams<T> pf{make_model<T>(h), make_state<T>(h), h->lay_step, io};
  if (h->fixed < 0) {
    cpu_step<T>(pf, h->dm.N, h->lay.total, ik);
    return;
  }
  const bool rerun = h->rerun && !(h->xflags & 1024);
  if (rerun) {
    std::memset(h->rerun, 0, (h->dm.N + 1) * sizeof(int32_t));
    pf.M.ovf_abort = 1;
    pf.S.rerun = h->rerun;
    pf.S.bak = h->bak;
    pf.S.resume = h->resume;
  }
  int idx = 0;
#define X(a, k)                                                                                      \
  if (h->fixed == idx) (void)fm_cpu_step_fixed_##a##_##k(fp64, 0, &pf, h->dm.N, h->lay_step.total, ik); \
  idx++;
  FM_FIXED_SCENES
  if constexpr (sizeof(T) == 4) {
    FM_FIXED_SCENES32
  }
#undef X
  (void)idx;
  if (rerun) {
    StepParams<double> pr{make_model<double>(h), make_state<double>(h), h->lay_rerun, io};
    pr.S.order = nullptr;
    pr.S.rerun = h->rerun;
    pr.S.bak = h->bak;
    pr.S.resume = h->resume;
    pr.M.dm.maxcon = MAXCON_WIDE;
    (void)fm_cpu_step_fixed_2_4(1, 1, &pr, h->dm.N < 256 ? h->dm.N : 256, h->lay_rerun.total, ik);
  }
}

template <typename T>
static void launch_step(fm_handle* h, const StepIO& io) {
  if (h->cpu) {
    launch_step_cpu<T>(h, io);
    return;
  }
  if (h->order) hipLaunchKernelGGL(lpt_order_kernel, dim3(1), dim3(1024), 0, h->stream, h->cost, h->order, h->dm.N);
  bool rerun = h->rerun && !(h->xflags & 1024);
  if (rerun && hipMemsetAsync(h->rerun, 0, (h->dm.N + 1) * sizeof(int32_t), h->stream) != hipSuccess) {
    // a stale list would make the rerun kernel re-step the previous launch's abandoned arenas: run without the
    // rerun list instead (stages above 64 contacts are then cut and counted in counters[0])
    fprintf(stderr, "factorysim: clearing the rerun list failed; this launch cuts contacts above 64\n");
    rerun = false;
  }
  const StepParams<T> pd{make_model<T>(h), make_state<T>(h), h->lay, io};
  dim3 grid(h->dm.N), block(WAVE);
  const bool ik = h->cfg.env_class != FM_ENV_ALLFULLRL_PROGRESS;
  int idx = 0;
#define X(a, k)                                                                                        \
  if (h->fixed == idx) {                                                                               \
    StepParams<T> pf = pd;                                                                             \
    pf.L = h->lay_step;                                                                                \
    if (rerun) {                                                                                       \
      pf.M.ovf_abort = 1;                                                                              \
      pf.S.rerun = h->rerun;                                                                           \
      pf.S.bak = h->bak;                                                                               \
      pf.S.resume = h->resume;                                                                         \
    }                                                                                                  \
    ktime_begin(h);                                                                                    \
    fixed_launch<T, a, k>(pf, h->dm.N, h->lay_step.total, h->stream, ik);                              \
    ktime_end(h);                                                                                      \
    if (rerun) launch_rerun(h, io, ik);                                                                \
    return;                                                                                            \
  }                                                                                                    \
  idx++;
  FM_FIXED_SCENES
  if constexpr (sizeof(T) == 4) {
    FM_FIXED_SCENES32
  }
#undef X
  (void)idx;
  ktime_begin(h);
  if constexpr (sizeof(T) == 8) {
    if (h->spill) {
      if (ik)
        hipLaunchKernelGGL((step_kernel<T, DimsSpill, true>), grid, block, h->lay.total, h->stream, pd);
      else
        hipLaunchKernelGGL((step_kernel<T, DimsSpill, false>), grid, block, h->lay.total, h->stream, pd);
      ktime_end(h);
      return;
    }
  }
  if (ik)
    hipLaunchKernelGGL((step_kernel<T, Dims, true>), grid, block, h->lay.total, h->stream, pd);
  else
    hipLaunchKernelGGL((step_kernel<T, Dims, false>), grid, block, h->lay.total, h->stream, pd);
  ktime_end(h);
}

// base colour of each collidable geom (assets/scene.xml, scene.py, conveyor_belt.xml, iiwa14.xml materials;
// MuJoCo's default geom rgba 0.5 where none is given); cubes take the seed's draws (cube_rgba)
static std::vector<float> render_colours(const SceneHost& s) {
  const int ngc = (int)s.geoms.size(), K = s.K;
  std::vector<float> c(4 * (size_t)ngc, 0.5f);
  for (int g = 0; g < ngc; g++) {
    const GeomRec& G = s.geoms[g];
    float r = 0.5f, gr = 0.5f, b = 0.5f;
    if (G.mjid == 2) {
      r = gr = b = 0.3f;  // belt
    } else if (G.mjid >= 3 + K && G.mjid < 13 + K) {
      const bool target = (G.mjid - 3 - K) % 5 == 0;
      r = gr = b = target ? 1.0f : 0.2f;  // bucket target area / fences
    } else if (G.mjid >= 13 + K && G.pclass == 0) {
      int link = G.kbody == 0 ? 0 : (G.kbody - 2 - K) % 10 + 1;  // collision sphere of this iiwa link
      if (link == 2 || link == 4 || link == 6) {
        r = 1.0f;
        gr = 0.423529f;
        b = 0.0392157f;
      } else {
        r = gr = b = 0.4f;
      }
    }
    c[4 * g] = r;
    c[4 * g + 1] = gr;
    c[4 * g + 2] = b;
    c[4 * g + 3] = 1.0f;
  }
  return c;
}

template <typename T>
static int render_typed(fm_handle* h, int count, int width, int height, const RenderParams& rp0, float* frames,
                        uint8_t* rgb) {
  const int ngc = h->dm.ngc;
  RenderParams rp = rp0;
  rp.frames = frames;
  rp.rgb = rgb;
  HIPCHK(hipFuncSetAttribute((const void*)render_frames_kernel<T, Dims>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             h->lay.total));
  hipLaunchKernelGGL((render_frames_kernel<T, Dims>), dim3(count), dim3(WAVE), h->lay.total, h->stream,
                     make_model<T>(h), make_state<T>(h), h->lay, rp);
  HIPCHK(hipGetLastError());
  if (rgb) {
    const int lds = ngc * RF_N * (int)sizeof(float);
    HIPCHK(hipFuncSetAttribute((const void*)render_pixels_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    dim3 grid(rp.tiles_x * ((height + RTILE - 1) / RTILE), count);
    hipLaunchKernelGGL(render_pixels_kernel, grid, dim3(WAVE), lds, h->stream, rp, ngc);
    HIPCHK(hipGetLastError());
  }
  return FM_OK;
}

extern "C" {

int fm_abi_version(void) { return FM_ABI_VERSION; }
int fm_config_size(void) { return (int)sizeof(fm_config); }

void fm_config_default(fm_config* c) {
  std::memset(c, 0, sizeof *c);
  c->num_arenas = 1;
  c->num_arms = 2;
  c->max_num_objects = 10;
  c->env_class = FM_ENV_ALLFULLRL_PROGRESS;
  c->precision = FM_FP32;
  c->max_contacts = 0;
  c->initial_conveyor_speed = 0.1;
  c->conveyor_acceleration = 0.001;
  c->pt_time = 0.2;
  c->force_contact_threshold = 200.0;
  c->control_frequency = 10;
  c->spawn_freq = 1.0 / 10;
  c->spawn_freq_increase = 1.001;
  // ProgressRewardEnv (environments.py:252-258): the three factors are required keyword arguments there (no
  // reference default; the caller sets them), base_reward defaults to 0
  c->gripper_to_closest_cube_reward_factor = 0.0;
  c->closest_cube_to_bucket_reward_factor = 0.0;
  c->small_action_norm_reward_factor = 0.0;
  c->base_reward = 0.0;
  c->solver_iterations = 100;
  c->solver_tolerance = 0.0;  // 0 = precision default (see fm_create)
}

const char* fm_last_error(void) { return g_err.c_str(); }

int fm_create(const fm_config* cfg, int device, const uint64_t* seeds, fm_handle** out) {
  if (!cfg || !out) return set_err(FM_EINVAL, "null argument");
  *out = nullptr;
  fm_handle* h = new fm_handle();
  h->cfg = *cfg;
  h->device = device;
  h->fp64 = cfg->precision == FM_FP64;
  h->xflags = read_experiment_flags();
  if (cfg->env_class < FM_ENV_FACTORY || cfg->env_class > FM_ENV_BACKUP_IK_TOGGLE) {
    delete h;
    return set_err(FM_EINVAL, "unknown env_class");
  }
  if (cfg->num_arms > 16) {
    delete h;
    return set_err(FM_EINVAL, "num_arms > 16");
  }
  // fp32: MuJoCo's own default (opt.tolerance 1e-8, the reference's setting); fp64: the oracle's 1e-12
  if (h->cfg.solver_tolerance <= 0) h->cfg.solver_tolerance = h->fp64 ? 1e-12 : 1e-8;
  if (h->cfg.solver_iterations <= 0) h->cfg.solver_iterations = 100;
  std::string err;
  if (!build_scene(cfg->num_arms, cfg->max_num_objects, cfg->num_arenas, seeds, h->sc, err)) {
    delete h;
    return set_err(FM_EINVAL, err);
  }
  const SceneHost& s = h->sc;
  Dims& d = h->dm;
  d.N = s.N;
  d.A = s.A;
  d.K = s.K;
  d.nq = s.nq;
  d.nv = s.nv;
  d.nu = s.nu;
  d.ngc = (int)s.geoms.size();
  d.nbox = s.nbox;
  d.npair = (int)s.pairs.size();
  d.nparam = (int)s.params.size();
  d.ntree = 1 + s.K + s.A;
  d.ncb = (int)s.cbodies.size();
  d.ncbp = (int)s.cb_pairs.size();
  {
    const int ec = cfg->env_class;
    const bool toggle = ec == FM_ENV_PAUSE_IK_TOGGLE || ec == FM_ENV_BACKUP_IK_TOGGLE;
    d.obs_dim = 24 * s.A + 13 * s.K + (toggle ? 8 * s.A : 0);  // IKTogglingEnv (environments.py:553)
    d.act_dim = ec == FM_ENV_FACTORY ? 0
                : (ec == FM_ENV_SINGLEFULLRL_PROGRESS || ec == FM_ENV_SINGLEDELTA_PROGRESS) ? 8
                : toggle ? s.A : 8 * s.A;
  }
  d.frame_skip = (int)((1.0 / cfg->control_frequency) / 0.001);
  {
    // contact capacity: the (2, 4) benchmark scene keeps 64 (one contact per lane), every other scene 128
    const int cap = (s.A == 2 && s.K == 4) ? MAXCON : MAXCON_WIDE;
    d.maxcon = cfg->max_contacts > 0 ? std::min(cfg->max_contacts, cap) : cap;
  }
  d.maxrow = 10 * s.A;
  d.phys_stride = 2 * s.nq + 3 * s.nv;
  d.dbl_stride = s.nu + 3 + 2 * s.A + 1 + 27 * s.A;
  d.int_stride = 2 * s.K + I_NINT + (3 + s.A) * s.A;
  if (device < 0) {
    // device = -1: the CPU backend (BASELINE config 1, one env on the host): host arrays, the kernels
    // of fm_device.hpp run on host threads with the wave emulated (fm_cpu.cpp); every pointer argument is host memory
    h->cpu = true;
  } else {
    if (hipSetDevice(device) != hipSuccess) {
      delete h;
      return set_err(FM_EDEVICE, "hipSetDevice failed (no GPU?  device = -1 selects the CPU backend)");
    }
    if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess) {
      delete h;
      return set_err(FM_EDEVICE, "hipStreamCreate failed");
    }
    h->stream = h->own_stream;
    if (hipEventCreateWithFlags(&h->handoff, hipEventDisableTiming) != hipSuccess) {
      fm_destroy(h);
      return set_err(FM_EDEVICE, "hipEventCreate failed");
    }
  }
  int r = h->fp64 ? create_typed<double>(h) : create_typed<float>(h);
  if (r) {
    std::string e = g_err;
    fm_destroy(h);
    return set_err(r, e);
  }
  *out = h;
  return FM_OK;
}

void fm_destroy(fm_handle* h) {
  if (!h) return;
  if (h->cpu) {
    for (void* p : h->allocs) std::free(p);
    delete h;
    return;
  }
  (void)d_setdev(h);
  // the arena state may still be in use by work queued on the current stream (the caller's or ours)
  (void)d_sync(h);
  if (h->own_stream && h->own_stream != h->stream) (void)hipStreamSynchronize(h->own_stream);
  ktime_clear(h);
  for (void* p : h->allocs) (void)d_free(h, p);
  for (void* p : {(void*)h->render_rgb, (void*)h->cube_rgba, (void*)h->render_frames, (void*)h->render_arenas})
    if (p) (void)hipFree(p);
  if (h->render_arenas_host) (void)hipHostFree(h->render_arenas_host);
  if (h->render_copied) (void)hipEventDestroy(h->render_copied);
  if (h->handoff) (void)hipEventDestroy(h->handoff);
  if (h->own_stream) (void)hipStreamDestroy(h->own_stream);  // never a stream the caller handed in
  delete h;
}

int fm_set_stream(fm_handle* h, void* stream) {
  if (!h) return set_err(FM_EINVAL, "null handle");
  if (h->cpu) return FM_OK;  // the CPU backend runs synchronously in the calling thread's launches
  hipStream_t next = (hipStream_t)stream;  // NULL = the legacy default stream (torch's default stream)
  if (next == h->stream) return FM_OK;
  // arena state is shared by every call of the handle: work queued on the new stream must not start
  // before what is already queued on the old one (a step on stream B racing a step on stream A)
  HIPCHK(d_setdev(h));
  HIPCHK(hipEventRecord(h->handoff, h->stream));
  HIPCHK(hipStreamWaitEvent(next, h->handoff, 0));
  h->stream = next;
  return FM_OK;
}

// runtime-mutable scalars of the reference env (set_attr / get_attr): fields of the handle's config, read by every
// later launch's Model (make_model runs per launch, so a change is ordered with the queued work)
static double* param_slot(fm_handle* h, const char* name, double* scale) {
  *scale = 1.0;
  if (!name) return nullptr;
  fm_config& c = h->cfg;
  const std::string n(name);
  if (n == "pt_time") return &c.pt_time;
  if (n == "initial_conveyor_speed") return &c.initial_conveyor_speed;
  if (n == "conveyor_acceleration") return &c.conveyor_acceleration;
  if (n == "force_contact_threshold") return &c.force_contact_threshold;
  if (n == "spawn_freq_increase") return &c.spawn_freq_increase;
  if (n == "init_spawn_freq") {  // BaseEnv.init_spawn_freq = spawn_freq * num_arms (base_env.py:36, 139)
    *scale = (double)h->dm.A;
    return &c.spawn_freq;
  }
  if (n == "gripper_to_closest_cube_reward_factor") return &c.gripper_to_closest_cube_reward_factor;
  if (n == "closest_cube_to_bucket_reward_factor") return &c.closest_cube_to_bucket_reward_factor;
  if (n == "small_action_norm_reward_factor") return &c.small_action_norm_reward_factor;
  if (n == "base_reward") return &c.base_reward;
  return nullptr;
}

int fm_set_param(fm_handle* h, const char* name, double value) {
  if (!h) return set_err(FM_EINVAL, "null handle");
  if (name && std::string(name) == "experiment_flags") {
#if FM_EXPERIMENTS
    if (!(value >= 0 && value < 65536 && value == (double)(uint32_t)value) || ((uint32_t)value & ~FM_XFLAGS_MASK))
      return set_err(FM_EINVAL, "bad flags: the experiment switches are the bits of 0x4E1E (fm_api.hip read_experiment_flags)");
    h->xflags = (uint32_t)value;
    return FM_OK;
#else
    if (value == 0.0) return FM_OK;
    return set_err(FM_EINVAL, "experiment switches are compiled out of the product library (libfactorysim_exp.so has them)");
#endif
  }
  double scale;
  double* p = param_slot(h, name, &scale);
  if (!p) return set_err(FM_EINVAL, std::string("not a runtime-mutable parameter: ") + (name ? name : "(null)"));
  if (!std::isfinite(value)) return set_err(FM_EINVAL, "non-finite value");
  *p = value / scale;
  return FM_OK;
}

int fm_get_param(const fm_handle* h, const char* name, double* value) {
  if (!h || !value) return set_err(FM_EINVAL, "null argument");
  if (name && std::string(name) == "experiment_flags") {
    *value = (double)h->xflags;
    return FM_OK;
  }
  double scale;
  double* p = param_slot(const_cast<fm_handle*>(h), name, &scale);
  if (!p) return set_err(FM_EINVAL, std::string("not a runtime-mutable parameter: ") + (name ? name : "(null)"));
  *value = *p * scale;
  return FM_OK;
}

int fm_num_counters(void) { return FM_NCTR; }

int fm_sync(fm_handle* h) {
  if (!h) return set_err(FM_EINVAL, "null handle");
  HIPCHK(d_setdev(h));
  HIPCHK(d_sync(h));
  if (!h->cpu) HIPCHK(hipGetLastError());
  return FM_OK;
}

int fm_obs_dim(const fm_handle* h) { return h ? h->dm.obs_dim : -1; }
int fm_act_dim(const fm_handle* h) { return h ? h->dm.act_dim : -1; }
int fm_num_arenas(const fm_handle* h) { return h ? h->dm.N : -1; }
int fm_nq(const fm_handle* h) { return h ? h->dm.nq : -1; }
int fm_nv(const fm_handle* h) { return h ? h->dm.nv : -1; }
int fm_nu(const fm_handle* h) { return h ? h->dm.nu : -1; }
int fm_workspace_bytes(const fm_handle* h) { return h ? h->lay_step.total : -1; }

int fm_reset(fm_handle* h, const uint8_t* mask, void* obs_) {
  if (!h) return set_err(FM_EINVAL, "null handle");
  float* obs = (float*)obs_;  // float64 rows when cfg.obs_float64 (Model::obs64): the kernel writes the row type
  HIPCHK(d_setdev(h));
  if (h->cpu) {
    if (h->fp64)
      cpu_reset<double>(make_model<double>(h), make_state<double>(h), h->lay, obs, mask, h->dm.N, h->lay.total);
    else
      cpu_reset<float>(make_model<float>(h), make_state<float>(h), h->lay, obs, mask, h->dm.N, h->lay.total);
    h->was_reset = true;
    return FM_OK;
  }
  dim3 grid(h->dm.N), block(WAVE);
  if (h->fp64 && h->spill) {
    hipLaunchKernelGGL((reset_kernel<double, DimsSpill>), grid, block, h->lay.total, h->stream, make_model<double>(h),
                       make_state<double>(h), h->lay, obs, mask);
  } else if (h->fp64) {
    hipLaunchKernelGGL((reset_kernel<double, Dims>), grid, block, h->lay.total, h->stream, make_model<double>(h),
                       make_state<double>(h), h->lay, obs, mask);
  } else {
    hipLaunchKernelGGL((reset_kernel<float, Dims>), grid, block, h->lay.total, h->stream, make_model<float>(h),
                       make_state<float>(h), h->lay, obs, mask);
  }
  HIPCHK(hipGetLastError());
  h->was_reset = true;
  return FM_OK;
}

int fm_step(fm_handle* h, const float* actions, void* obs, float* reward, uint8_t* terminated, uint8_t* truncated,
            const fm_info* info) {
  if (!h) return set_err(FM_EINVAL, "null handle");
  if (!actions && h->dm.act_dim > 0) return set_err(FM_EINVAL, "actions is NULL");
  if (!h->was_reset) return set_err(FM_ESTATE, "fm_step before fm_reset");
  HIPCHK(d_setdev(h));
  StepIO io;
  std::memset(&io, 0, sizeof io);
  io.actions = actions;
  io.obs = (float*)obs;  // float64 rows when cfg.obs_float64 (Model::obs64)
  io.reward = reward;
  io.terminated = terminated;
  io.truncated = truncated;
  if (info) {
    io.scores = info->scores;
    io.num_obj = info->num_obj;
    io.play_time = info->play_time;
    io.conveyor_speed = info->conveyor_speed;
    io.out_of_reach = info->out_of_reach;
    io.force_terminate = info->force_terminate;
    io.terminal_obs = (float*)info->terminal_obs;
    io.ep_return = info->episode_return;
    io.ep_len = info->episode_length;
    io.terminal_scores = info->terminal_scores;
  }
  if (h->fp64)
    launch_step<double>(h, io);
  else
    launch_step<float>(h, io);
  if (!h->cpu) HIPCHK(hipGetLastError());
  return FM_OK;
}

// exported record: doubles [phys (2nq+3nv) | dbl_stride] , int32 [int_stride], uint64 [4]
int fm_state_size(const fm_handle* h) { return h ? state_record_size(h) : -1; }

int fm_get_state(fm_handle* h, void* host_out) {
  if (!h || !host_out) return set_err(FM_EINVAL, "null argument");
  HIPCHK(d_setdev(h));
  return h->fp64 ? get_state_typed<double>(h, (char*)host_out) : get_state_typed<float>(h, (char*)host_out);
}

int fm_set_state(fm_handle* h, const void* host_in) {
  if (!h || !host_in) return set_err(FM_EINVAL, "null argument");
  HIPCHK(d_setdev(h));
  return h->fp64 ? set_state_typed<double>(h, (const char*)host_in) : set_state_typed<float>(h, (const char*)host_in);
}

int fm_debug_dump(fm_handle* h, int arena, int actuated, double* host_out, int cap) {
  if (!h || !host_out || arena < 0 || arena >= h->dm.N) return set_err(FM_EINVAL, "bad argument");
  const Dims& d = h->dm;
  int need = 2 + 81 * d.A + 4 * d.nv + 3 * d.A + 60 * d.A + 27 * d.A + 17 * 64 + 6 * 20 * d.A;
  if (cap < need) return set_err(FM_EINVAL, "buffer too small: need " + std::to_string(need));
  HIPCHK(d_setdev(h));
  double* dbuf = nullptr;
  HIPCHK(d_malloc(h, &dbuf, need * sizeof(double)));
  HIPCHK(d_memset(h, dbuf, 0, need * sizeof(double)));
  if (h->cpu) {
    if (h->fp64)
      cpu_debug<double>(make_model<double>(h), make_state<double>(h), h->lay, arena, actuated, dbuf, h->lay.total);
    else
      cpu_debug<float>(make_model<float>(h), make_state<float>(h), h->lay, arena, actuated, dbuf, h->lay.total);
    std::memcpy(host_out, dbuf, need * sizeof(double));
    std::free(dbuf);
    return need;
  }
  if (h->fp64 && h->spill) {
    HIPCHK(hipFuncSetAttribute((const void*)debug_kernel<double, DimsSpill>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, h->lay.total));
    hipLaunchKernelGGL((debug_kernel<double, DimsSpill>), dim3(1), dim3(WAVE), h->lay.total, h->stream,
                       make_model<double>(h), make_state<double>(h), h->lay, arena, actuated, dbuf);
  } else if (h->fp64) {
    HIPCHK(hipFuncSetAttribute((const void*)debug_kernel<double, Dims>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               h->lay.total));
    hipLaunchKernelGGL((debug_kernel<double, Dims>), dim3(1), dim3(WAVE), h->lay.total, h->stream, make_model<double>(h),
                       make_state<double>(h), h->lay, arena, actuated, dbuf);
  } else {
    HIPCHK(hipFuncSetAttribute((const void*)debug_kernel<float, Dims>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               h->lay.total));
    hipLaunchKernelGGL((debug_kernel<float, Dims>), dim3(1), dim3(WAVE), h->lay.total, h->stream, make_model<float>(h),
                       make_state<float>(h), h->lay, arena, actuated, dbuf);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(d_sync(h));
  HIPCHK(d_memcpy(h, host_out, dbuf, need * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(hipFree(dbuf));
  return need;
}

int fm_profile(fm_handle* h, int mode, uint64_t* host_out) {
  if (!h) return set_err(FM_EINVAL, "null handle");
  if (h->cpu) return set_err(FM_EINVAL, "the phase profile is GPU-only (wall-clock ticks of the device)");
  HIPCHK(d_setdev(h));
  if (!h->prof) {
    HIPCHK(d_malloc(h, (void**)&h->prof, FM_NPROF * sizeof(unsigned long long)));
    h->allocs.push_back(h->prof);
    HIPCHK(d_memset(h, h->prof, 0, FM_NPROF * sizeof(unsigned long long)));
  }
  if (host_out) {
    HIPCHK(d_sync(h));
    HIPCHK(d_memcpy(h, host_out, h->prof, FM_NPROF * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    int khz = 0;
    HIPCHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->device));
    host_out[PH_KHZ] = (uint64_t)khz;
  }
  if (mode == 1) {
    HIPCHK(d_sync(h));
    HIPCHK(d_memset(h, h->prof, 0, FM_NPROF * sizeof(unsigned long long)));
    h->prof_on = true;
  } else if (mode == 0) {
    h->prof_on = false;
  }
  return FM_OK;
}

int fm_get_counters(fm_handle* h, int64_t* host_out) {
  if (!h || !host_out) return set_err(FM_EINVAL, "null argument");
  HIPCHK(d_setdev(h));
  HIPCHK(d_sync(h));
  HIPCHK(d_memcpy(h, host_out, h->counters, (size_t)h->dm.N * FM_NCTR * sizeof(int64_t), hipMemcpyDeviceToHost));
  return FM_OK;
}

int fm_get_costs(fm_handle* h, uint32_t* host_out) {
  if (!h || !host_out) return set_err(FM_EINVAL, "null argument");
  if (!h->cost) return set_err(FM_EINVAL, "no per-arena costs (FACTORYSIM_NO_LPT)");
  HIPCHK(d_setdev(h));
  HIPCHK(d_sync(h));
  HIPCHK(d_memcpy(h, host_out, h->cost, (size_t)h->dm.N * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return FM_OK;
}

int fm_kernel_timing(fm_handle* h, int enable) {
  if (!h) return set_err(FM_EINVAL, "null handle");
  HIPCHK(d_setdev(h));
  HIPCHK(d_sync(h));
  ktime_clear(h);
  h->ktime_on = enable != 0;
  return FM_OK;
}

int fm_get_kernel_time(fm_handle* h, double* total_ms, int* launches) {
  if (!h || !total_ms || !launches) return set_err(FM_EINVAL, "null argument");
  HIPCHK(d_setdev(h));
  HIPCHK(d_sync(h));
  double t = 0.0;
  for (auto& e : h->ktime) {
    float ms = 0.0f;
    HIPCHK(hipEventElapsedTime(&ms, e.first, e.second));
    t += ms;
  }
  *total_ms = t;
  *launches = (int)h->ktime.size();
  ktime_clear(h);
  return FM_OK;
}

int fm_render_ngeom(const fm_handle* h) { return h ? h->dm.ngc : -1; }

int fm_render(fm_handle* h, const int32_t* arenas, int count, int width, int height, const float* camera,
              uint8_t* rgb, float* geom_frames) {
  if (!h || !arenas) return set_err(FM_EINVAL, "null argument");
  if (h->cpu) return set_err(FM_EINVAL, "rendering is GPU-only");
  if (count < 0 || (count > 0 && (width < 1 || height < 1 || width > 8192 || height > 8192)))
    return set_err(FM_EINVAL, "bad image size");
  if (!rgb && !geom_frames) return set_err(FM_EINVAL, "nothing to write (rgb and geom_frames are both NULL)");
  if ((size_t)h->dm.ngc * RF_N * sizeof(float) > 160 * 1024) return set_err(FM_EINVAL, "scene too large to render");
  for (int i = 0; i < count; i++)
    if (arenas[i] < 0 || arenas[i] >= h->dm.N) return set_err(FM_EINVAL, "arena index out of range");
  if (count == 0) return FM_OK;
  HIPCHK(d_setdev(h));
  if (!h->render_rgb) {
    std::vector<float> c = render_colours(h->sc);
    HIPCHK(d_malloc(h, (void**)&h->render_rgb, c.size() * sizeof(float)));
    HIPCHK(d_memcpy(h, h->render_rgb, c.data(), c.size() * sizeof(float), hipMemcpyHostToDevice));
    HIPCHK(d_malloc(h, (void**)&h->cube_rgba, h->sc.cube_rgba.size() * sizeof(float)));
    HIPCHK(d_memcpy(h, h->cube_rgba, h->sc.cube_rgba.data(), h->sc.cube_rgba.size() * sizeof(float),
                     hipMemcpyHostToDevice));
  }
  if (!h->render_copied) HIPCHK(hipEventCreateWithFlags(&h->render_copied, hipEventDisableTiming));
  if ((size_t)count > h->render_cap) {
    // growing the scratch frees buffers queued work may still read: the one synchronising path (rare)
    HIPCHK(d_sync(h));
    if (h->render_frames) HIPCHK(hipFree(h->render_frames));
    if (h->render_arenas) HIPCHK(hipFree(h->render_arenas));
    if (h->render_arenas_host) HIPCHK(hipHostFree(h->render_arenas_host));
    h->render_frames = nullptr;
    h->render_arenas = nullptr;
    h->render_arenas_host = nullptr;
    HIPCHK(d_malloc(h, (void**)&h->render_frames, (size_t)count * h->dm.ngc * RF_N * sizeof(float)));
    HIPCHK(d_malloc(h, (void**)&h->render_arenas, (size_t)count * sizeof(int)));
    HIPCHK(hipHostMalloc((void**)&h->render_arenas_host, (size_t)count * sizeof(int), hipHostMallocDefault));
    h->render_cap = count;
  } else {
    // the staging buffer is reused: wait only for the previous render's arena copy (not for the stream)
    HIPCHK(hipEventSynchronize(h->render_copied));
  }
  // the arena list travels through pinned staging on the stream, ordered after queued env-steps; the caller's
  // array is free again when this call returns
  std::memcpy(h->render_arenas_host, arenas, (size_t)count * sizeof(int));
  HIPCHK(hipMemcpyAsync(h->render_arenas, h->render_arenas_host, (size_t)count * sizeof(int), hipMemcpyHostToDevice,
                        h->stream));
  HIPCHK(hipEventRecord(h->render_copied, h->stream));
  // MuJoCo free camera (mjv_cameraInModel): forward from azimuth / elevation, eye = lookat - distance * forward;
  // default = the reference viewer's initial camera (scene.py:164-169), fovy 45 deg
  const float def[6] = {-0.30914206f, -0.14805237f, 1.53675732f, 3.6720494f, 66.957422f, -28.843359f};
  const float* c = camera ? camera : def;
  const double az = c[4] * M_PI / 180.0, el = c[5] * M_PI / 180.0;
  const double fw[3] = {std::cos(el) * std::cos(az), std::cos(el) * std::sin(az), std::sin(el)};
  double rt[3] = {fw[1], -fw[0], 0.0};  // forward x z
  const double rn = std::sqrt(rt[0] * rt[0] + rt[1] * rt[1]);
  if (rn < 1e-9) return set_err(FM_EINVAL, "camera looks straight up or down");
  rt[0] /= rn;
  rt[1] /= rn;
  const double up[3] = {rt[1] * fw[2] - rt[2] * fw[1], rt[2] * fw[0] - rt[0] * fw[2], rt[0] * fw[1] - rt[1] * fw[0]};
  RenderParams rp{};
  for (int k = 0; k < 3; k++) {
    rp.eye[k] = (float)(c[k] - c[3] * fw[k]);
    rp.fwd[k] = (float)fw[k];
    rp.right[k] = (float)rt[k];
    rp.up[k] = (float)up[k];
  }
  rp.tan_y = (float)std::tan(0.5 * 45.0 * M_PI / 180.0);
  rp.aspect = (float)width / (float)height;
  rp.width = width;
  rp.height = height;
  rp.tiles_x = (width + RTILE - 1) / RTILE;
  rp.arenas = h->render_arenas;
  rp.geom_rgb = h->render_rgb;
  rp.cube_rgba = h->cube_rgba;
  float* frames = geom_frames ? geom_frames : h->render_frames;
  return h->fp64 ? render_typed<double>(h, count, width, height, rp, frames, rgb)
                 : render_typed<float>(h, count, width, height, rp, frames, rgb);
}

// host only (no device): the compiled scene as MJCF (scene.py:109-161), for the MuJoCo cross-check
int fm_scene_mjcf(int num_arms, int max_num_objects, uint64_t seed, const char* meshdir, char* buf, size_t cap,
                  size_t* len) {
  SceneHost s;
  std::string err;
  if (!build_scene(num_arms, max_num_objects, 1, &seed, s, err)) return set_err(FM_EINVAL, err);
  const std::string x = export_mjcf(s, seed, meshdir);
  if (len) *len = x.size();
  if (!buf) return FM_OK;
  if (cap < x.size() + 1) return set_err(FM_EINVAL, "buffer too small for the MJCF document (see *len)");
  std::memcpy(buf, x.c_str(), x.size() + 1);
  return FM_OK;
}

}  // extern "C"
