// fm_cpu.cpp -- the CPU backend's kernels (fm_create(..., device = -1)): the env-step, reset and
// debug kernels of fm_device.hpp -- the product's own sources, unchanged -- compiled for the host with the
// 64-lane wave emulated (fm_simt_host.hpp).  Config 1 of BASELINE.json (one env, CPU, src/visualisation.py:32-77)
// runs through the same C ABI as the GPU path; fm_api.hip dispatches here when the handle lives on the host.
//
// Emulation: a workgroup (= one arena, one wave) runs as 64 fibers on one host thread.  Each fiber has its own
// stack; fm_simt_switch swaps the callee-saved registers and the stack pointer (x86-64 System V), so the lanes run
// one after another up to their next cross-lane operation, where the scheduler resolves it for the whole wave and
// resumes them.  Arenas are spread over host threads (each thread owns one emulated wave: fibers, stacks, LDS).
#include <dlfcn.h>

#include <atomic>
#include <memory>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

// The host build of the kernels lives in its own namespace: fm_api.hip's HIP compile gives every __global__ kernel
// a host-side launch handle under the kernel's mangled name in namespace fm, which the host definitions here would
// otherwise collide with.  fm_api.hip reaches this TU through the extern "C" entry points at the end.
#define fm fm_cpu_ns
#include "fm_device.hpp"

// ---------------------------------------------------------------------------------------------------------------
// fibers (x86-64 System V: rbx, rbp, r12-r15 and rsp are callee-saved; mxcsr and the x87 control word too, but every
// lane runs the same kernel code under the launching thread's floating-point environment, which nothing changes --
// so the switch leaves them alone (the serialising ldmxcsr / fldcw pair cost ~40 % of a switch))
// ---------------------------------------------------------------------------------------------------------------
extern "C" void fm_simt_switch(void** save_sp, void* load_sp);
extern "C" void fm_simt_trampoline();
extern "C" __attribute__((visibility("hidden"))) void fm_simt_fiber_main();
asm(R"(
.text
.p2align 4
.globl fm_simt_switch
.hidden fm_simt_switch
.type fm_simt_switch,@function
fm_simt_switch:
  pushq %rbp
  pushq %rbx
  pushq %r12
  pushq %r13
  pushq %r14
  pushq %r15
  movq %rsp, (%rdi)
  movq %rsi, %rsp
  popq %r15
  popq %r14
  popq %r13
  popq %r12
  popq %rbx
  popq %rbp
  ret
.size fm_simt_switch,.-fm_simt_switch

.p2align 4
.globl fm_simt_trampoline
.hidden fm_simt_trampoline
.type fm_simt_trampoline,@function
fm_simt_trampoline:
  andq $-16, %rsp
  call fm_simt_fiber_main
  ud2
.size fm_simt_trampoline,.-fm_simt_trampoline
)");

namespace fm_simt {

static thread_local Wave* t_wave = nullptr;

Wave& wave() { return *t_wave; }

// a fresh fiber stack whose first switch "returns" into the trampoline with zeroed callee-saved registers
static void* fiber_init(char* stack, size_t bytes) {
  uintptr_t top = ((uintptr_t)(stack + bytes)) & ~(uintptr_t)15;
  uint64_t* p = (uint64_t*)top;
  *--p = 0;                              // alignment pad
  *--p = (uint64_t)&fm_simt_trampoline;  // return address of fm_simt_switch
  for (int i = 0; i < 6; i++) *--p = 0;  // rbp rbx r12 r13 r14 r15
  return (void*)p;
}

}  // namespace fm_simt

extern "C" void fm_simt_fiber_main() {
  fm_simt::Wave& w = *fm_simt::t_wave;
  w.entry(w.entry_arg);
  w.done[w.lane] = true;
  fm_simt_switch(&w.sp[w.lane], w.sched_sp);  // never resumed
  __builtin_trap();
}

namespace fm_simt {

int64_t cross(int op, int64_t a0, int64_t a1, int ctrl, int line) {
  Wave& w = *t_wave;
  const int l = w.lane;
  w.line[l] = line;
  w.op[l] = op;
  w.a0[l] = a0;
  w.a1[l] = a1;
  w.ctrl[l] = ctrl;
  fm_simt_switch(&w.sp[l], w.sched_sp);
  return w.out[l];
}

void mfma_16x16x4(float a, float b, const float* c, float* d) {
  Wave& w = *t_wave;
  const int l = w.lane;
  w.mf_a[l] = a;
  w.mf_b[l] = b;
  for (int r = 0; r < 4; r++) w.mf_c[l][r] = c[r];
  (void)cross(OP_MFMA, 0, 0, 0);
  for (int r = 0; r < 4; r++) d[r] = w.mf_d[l][r];
}

static const char* op_name(int op) {
  switch (op) {
    case OP_BARRIER: return "barrier";
    case OP_READLANE: return "readlane";
    case OP_READFIRST: return "readfirstlane";
    case OP_DPP: return "dpp";
    case OP_BPERMUTE: return "bpermute";
    case OP_BALLOT: return "ballot";
    case OP_MFMA: return "mfma";
  }
  return "?";
}

// the source lane of a DPP move for lane l, or -1 (out of the row / no source: the old value stays)
static int dpp_src(int ctrl, int l) {
  const int row = l & ~15, rl = l & 15;
  if (ctrl <= 0xff) return (l & ~3) | ((ctrl >> (2 * (l & 3))) & 3);  // quad_perm
  if (ctrl >= 0x101 && ctrl <= 0x10f) {                                // row_shl
    const int n = ctrl - 0x100;
    return rl + n <= 15 ? l + n : -1;
  }
  if (ctrl >= 0x111 && ctrl <= 0x11f) {  // row_shr
    const int n = ctrl - 0x110;
    return rl >= n ? l - n : -1;
  }
  if (ctrl >= 0x121 && ctrl <= 0x12f) {  // row_ror
    const int n = ctrl - 0x120;
    return row | ((rl - n) & 15);
  }
  if (ctrl == 0x142) return l >= 16 ? row - 1 : -1;  // row_bcast:15
  if (ctrl == 0x143) return l >= 32 ? 31 : -1;       // row_bcast:31
  std::fprintf(stderr, "factorysim cpu: DPP control 0x%x not emulated\n", ctrl);
  std::abort();
}

// resolve the cross-lane operation every live lane of the wave is waiting at
static void resolve(Wave& w) {
  w.epoch++;
  int first = -1;
  for (int l = 0; l < W; l++)
    if (!w.done[l]) {
      first = l;
      break;
    }
  const int op = w.op[first];
  static const bool trace = std::getenv("FACTORYSIM_CPU_TRACE") && !std::strcmp(std::getenv("FACTORYSIM_CPU_TRACE"), "ops");
  if (trace)
    std::fprintf(stderr, "[simt] block %u: %s 0x%x line %d (first live lane %d)\n", w.block.x, op_name(op),
                 w.ctrl[first], w.line[first], first);
  for (int l = 0; l < W; l++)
    if (!w.done[l] && (w.op[l] != op || ((op == OP_READLANE || op == OP_DPP) && w.ctrl[l] != w.ctrl[first]))) {
      std::fprintf(stderr,
                   "factorysim cpu: lanes of arena %u diverged at a cross-lane operation (lane %d: %s 0x%x at line %d, "
                   "lane %d: %s 0x%x at line %d)\n",
                   w.block.x, first, op_name(op), w.ctrl[first], w.line[first], l, op_name(w.op[l]), w.ctrl[l],
                   w.line[l]);
      // the suspended lanes' call chains (frame pointers: an -O0 build), for llvm-symbolizer
      for (int ln : {first, l}) {
        const uint64_t* fr = (const uint64_t*)w.sp[ln];  // saved r15 r14 r13 r12 rbx rbp, return address
        const uint64_t* bp = (const uint64_t*)fr[5];
        Dl_info di{};
        dladdr((const void*)fr[6], &di);
        std::fprintf(stderr, "  lane %d: %s+0x%lx", ln, di.dli_fname ? di.dli_fname : "?",
                     (long)((const char*)fr[6] - (const char*)di.dli_fbase));
        for (int d = 0; d < 24 && bp; d++) {
          const uint64_t ra = bp[1];
          if (!ra) break;
          std::fprintf(stderr, " 0x%lx", (long)((const char*)ra - (const char*)di.dli_fbase));
          bp = (const uint64_t*)bp[0];
        }
        std::fprintf(stderr, "\n");
      }
      std::abort();
    }
  switch (op) {
    case OP_BARRIER:
      break;
    case OP_READLANE: {
      const int s = w.ctrl[first] & 63;
      const int64_t v = w.done[s] ? 0 : (w.a0[s] & 0xffffffffll);
      for (int l = 0; l < W; l++) w.out[l] = v;
      break;
    }
    case OP_READFIRST:
      for (int l = 0; l < W; l++) w.out[l] = w.a0[first] & 0xffffffffll;
      break;
    case OP_DPP: {
      const int ctrl = w.ctrl[first];
      for (int l = 0; l < W; l++) {
        const int s = dpp_src(ctrl, l);
        w.out[l] = (s < 0 || w.done[s]) ? (w.a1[l] & 0xffffffffll) : (w.a0[s] & 0xffffffffll);
      }
      break;
    }
    case OP_BPERMUTE:
      for (int l = 0; l < W; l++) {
        const int s = (int)((w.a1[l] >> 2) & 63);
        w.out[l] = w.done[s] ? 0 : (w.a0[s] & 0xffffffffll);
      }
      break;
    case OP_BALLOT: {
      uint64_t m = 0;
      for (int l = 0; l < W; l++)
        if (!w.done[l] && (w.a0[l] & 1)) m |= 1ull << l;
      for (int l = 0; l < W; l++) w.out[l] = (int64_t)m;
      break;
    }
    case OP_MFMA:
      for (int l = 0; l < W; l++) {
        const int j = l & 15, r0 = 4 * (l >> 4);
        for (int r = 0; r < 4; r++) {
          const int i = r0 + r;
          float acc = w.mf_c[l][r];
          for (int k = 0; k < 4; k++) acc += w.mf_a[16 * k + i] * w.mf_b[16 * k + j];
          w.mf_d[l][r] = acc;
        }
      }
      break;
    default:
      std::fprintf(stderr, "factorysim cpu: unknown cross-lane operation %d\n", op);
      std::abort();
  }
}

// run one workgroup (blockIdx.x = b) of a kernel: 64 fibers from `entry`, until every lane has returned
static void run_block(Wave& w, unsigned b, unsigned grid, void (*entry)(void*), void* arg) {
  w.block = Dim3{b, 0u, 0u};
  w.epoch++;  // a new block starts a new phase
  w.grid = Dim3{grid, 1u, 1u};
  w.entry = entry;
  w.entry_arg = arg;
  // FACTORYSIM_CPU_POISON=<byte>: the top of every lane's stack (its locals at -O0) filled with that byte before the
  // block runs -- the uninitialised-read probe (tools/poison_probe.py) compares the results of two poison values
  static const int poison = std::getenv("FACTORYSIM_CPU_POISON") ? std::atoi(std::getenv("FACTORYSIM_CPU_POISON")) : -1;
  for (int l = 0; l < W; l++) {
    w.done[l] = false;
    if (poison >= 0) {
      const size_t top = std::min<size_t>(w.stack_bytes, 256 * 1024);
      std::memset(w.stacks + (size_t)(l + 1) * w.stack_bytes - top, poison, top);
    }
    w.sp[l] = fiber_init(w.stacks + (size_t)l * w.stack_bytes, w.stack_bytes);
  }
  static const bool reverse = std::getenv("FACTORYSIM_CPU_REVERSE") != nullptr;  // race probe: lanes in reverse order
  for (;;) {
    bool live = false;
    for (int ll = 0; ll < W; ll++) {
      const int l = reverse ? W - 1 - ll : ll;
      if (w.done[l]) continue;
      w.lane = l;
      fm_simt_switch(&w.sched_sp, w.sp[l]);  // run lane l to its next cross-lane point (or its end)
      live = live || !w.done[l];
    }
    if (!live) break;
    resolve(w);
  }
  w.lane = -1;  // between blocks: no lane runs
}

// the race / bounds detector build keeps guard zones around the emulated LDS: an access there is an out-of-bounds
// workspace access (fm_race::access reports it; on the GPU it would read 0 or be dropped, silently)
#ifdef FM_RACE_DETECT
constexpr size_t LDS_GUARD = 64 * 1024;
#else
constexpr size_t LDS_GUARD = 0;
#endif
struct WaveBox {
  Wave w;
  std::unique_ptr<char[]> stacks;
  std::vector<char> lds;
  WaveBox(size_t stack_bytes, size_t lds_bytes)
      : stacks(new char[stack_bytes * W]), lds(lds_bytes + 64 + 2 * LDS_GUARD) {
    std::memset(&w, 0, sizeof w);
    w.stacks = stacks.get();
    w.stack_bytes = stack_bytes;
    w.lds = (char*)(((uintptr_t)lds.data() + LDS_GUARD + 63) & ~(uintptr_t)63);
    w.lds_bytes = lds_bytes;
  }
};

// FACTORYSIM_CPU_TRACE: report the faulting instruction of a crash inside an emulated lane (no debugger needed)
#include <signal.h>
#include <ucontext.h>
static void segv_report(int sig, siginfo_t* si, void* uc_) {
  ucontext_t* uc = (ucontext_t*)uc_;
  Dl_info di{};
  const void* ip = (const void*)uc->uc_mcontext.gregs[REG_RIP];
  dladdr(ip, &di);
  std::fprintf(stderr, "[simt] signal %d at %p (ip %p = %s+0x%lx, lib %s base %p) lane %d block %u\n", sig, si->si_addr,
               ip, di.dli_sname ? di.dli_sname : "?", (long)((const char*)ip - (const char*)di.dli_saddr),
               di.dli_fname ? di.dli_fname : "?", di.dli_fbase, t_wave ? t_wave->lane : -1,
               t_wave ? t_wave->block.x : 0u);
  std::_Exit(139);
}
static void install_trace() {
  static bool done = false;
  if (done || !std::getenv("FACTORYSIM_CPU_TRACE")) return;
  done = true;
  struct sigaction sa {};
  sa.sa_sigaction = segv_report;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigaction(SIGSEGV, &sa, nullptr);
  sigaction(SIGILL, &sa, nullptr);  // -fsanitize-trap=bounds (the race / bounds detector build): an array index check
  static char altstack[1 << 16];
  stack_t ss{};
  ss.ss_sp = altstack;
  ss.ss_size = sizeof altstack;
  sigaltstack(&ss, nullptr);
}

// the rendezvous count of this host thread, carried over its launches of every kernel (the race detector's shadow
// outlives a launch: an epoch must never repeat on a thread)
static thread_local unsigned t_epoch = 0;

// a grid of `grid` workgroups, spread over host threads; `entry(arg)` is the kernel body of one lane
template <typename F>
static void launch(unsigned grid, size_t lds_bytes, const void* kernarg, F&& body) {
  static const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const char* env = std::getenv("FACTORYSIM_CPU_THREADS");
  unsigned nt = env ? (unsigned)std::max(1, std::atoi(env)) : std::min(hw, 16u);
  nt = std::min(nt, std::max(grid, 1u));
  std::atomic<unsigned> next{0};
  install_trace();
  auto worker = [&]() {
    static const size_t stack_mb = std::getenv("FACTORYSIM_CPU_STACK_MB") ? std::atoi(std::getenv("FACTORYSIM_CPU_STACK_MB")) : 1;
    WaveBox box(stack_mb << 20, lds_bytes);
    box.w.lane = -1;
    box.w.epoch = t_epoch;
    t_wave = &box.w;
    box.w.kernarg = kernarg;
    struct Ctx {
      F* f;
    } ctx{&body};
    auto entry = [](void* p) { (*((Ctx*)p)->f)(); };
    for (;;) {
      const unsigned b = next.fetch_add(1);
      if (b >= grid) break;
      // LDS starts zeroed (FACTORYSIM_CPU_POISON: filled with the poison byte -- the GPU's LDS holds whatever the
      // previous workgroup left)
      static const int lpoison =
          std::getenv("FACTORYSIM_CPU_POISON") ? std::atoi(std::getenv("FACTORYSIM_CPU_POISON")) : 0;
      std::memset(box.w.lds, lpoison, lds_bytes);
      run_block(box.w, b, grid, entry, &ctx);
    }
    t_epoch = box.w.epoch + 1;
    t_wave = nullptr;
  };
  if (nt <= 1) {
    worker();
  } else {
    std::vector<std::thread> th;
    for (unsigned i = 0; i < nt; i++) th.emplace_back(worker);
    for (auto& t : th) t.join();
  }
}

void launch_kernel(unsigned grid, size_t lds_bytes, const void* kernarg, void (*body)(const void*)) {
  launch(grid, lds_bytes, kernarg, [=]() { body(kernarg); });
}

}  // namespace fm_simt

#ifdef FM_RACE_DETECT
// ---------------------------------------------------------------------------------------------------------------
// LDS race detector (tools/lds_race_check.sh): this TU compiled with -fsanitize=thread for its instrumentation only
// (no TSan runtime) -- the hooks below keep a shadow word per 4 bytes of the emulated wave's LDS with the last writer
// lane and the lanes that read it since the last cross-lane rendezvous, and record every pair of accesses by two
// different lanes to the same word between two rendezvous with at least one write: a hand-off without a SYNC().
// On the GPU such code relies on the wave's lockstep; the CPU backend (one lane after another) needs the barrier.
// ---------------------------------------------------------------------------------------------------------------
#define FM_NO_INSTR __attribute__((disable_sanitizer_instrumentation))
#include <mutex>
#include <map>
#include <set>
#include <unordered_map>
namespace fm_race {
struct Shadow {
  unsigned wr_epoch = ~0u, rd_epoch = ~0u;
  int wr_lane = -1;
  uint64_t rd_mask = 0;
  const void* wr_pc = nullptr;
  const void* rd_pc = nullptr;
};
static thread_local Shadow* t_shadow = nullptr;  // one per LDS byte; malloc'ed: libc is not instrumented
static thread_local size_t t_nshadow = 0;
static thread_local const char* t_base = nullptr;
static thread_local bool t_in_hook = false;  // the map below is instrumented code: no hook re-entry from it
// global memory the block touches (the arena's scratch block and records): one entry per byte, cleared per block
static thread_local std::unordered_map<uintptr_t, Shadow>* t_gshadow = nullptr;
static thread_local unsigned t_gblock = ~0u;
static thread_local const void* t_gwave = nullptr;
static std::mutex g_mu;
// (pc, other pc, kind 0 RAW 1 WAR 2 WAW 3 LDS out of bounds 4 global scratch out of the arena's block) -> the first byte
// offset into LDS it was seen at (-1: global memory; kind 4: the offset into the scratch buffer)
static std::map<std::tuple<const void*, const void*, int>, long> g_races;
static thread_local long t_off = -1;
static int g_lay[sizeof(fm::Lay) / sizeof(int)];  // the LDS layout of the last step launch
// the launch's per-arena global scratch blocks ([n][stride] bytes at base; fm_cpu_note_launch): every access there must
// stay in the one block its workgroup's arena owns -- the first block a workgroup touches is its own
static const char* g_spill = nullptr;
static long long g_spill_stride = 0, g_spill_n = 0;
static thread_local long long t_slot = -1;
static thread_local unsigned t_slot_block = ~0u;
static thread_local const void* t_slot_wave = nullptr;

FM_NO_INSTR static void note(const void* pc, const void* other, int kind) {
  const bool was = t_in_hook;
  t_in_hook = true;
  {
    std::lock_guard<std::mutex> g(g_mu);
    g_races.emplace(std::make_tuple(pc, other, kind), t_off);
  }
  t_in_hook = was;
}
FM_NO_INSTR static void access(const void* addr, size_t n, bool write, const void* pc) {
  fm_simt::Wave* w = fm_simt::t_wave;
  if (!w || !w->lds || t_in_hook || w->lane < 0) return;
  const char* a = (const char*)addr;
  // bounds: the LDS guard zones (fm_simt::LDS_GUARD) and the arena's scratch block
  if ((a + n > w->lds + w->lds_bytes && a < w->lds + w->lds_bytes + fm_simt::LDS_GUARD) ||
      (a < w->lds && a + fm_simt::LDS_GUARD >= w->lds)) {
    t_off = (long)(a - w->lds);
    note(pc, nullptr, 3);
    return;
  }
  if (g_spill && g_spill_stride > 0 && a >= g_spill && a < g_spill + g_spill_n * g_spill_stride) {
    if (t_slot_block != w->block.x || t_slot_wave != (const void*)w) {
      t_slot = -1;
      t_slot_block = w->block.x;
      t_slot_wave = w;
    }
    const long long off = (long long)(a - g_spill), slot = off / g_spill_stride;
    const long long end_slot = (off + (long long)n - 1) / g_spill_stride;
    if (t_slot < 0 && slot < g_spill_n) t_slot = slot;
    if (slot != t_slot || end_slot != t_slot) {
      t_off = (long)off;
      note(pc, nullptr, 4);
    }
  }
  if (a < w->lds || a >= w->lds + w->lds_bytes) {
    // global memory: only addresses off this thread's stacks (the lanes' private variables live on the fibers)
    if (a >= w->stacks && a < w->stacks + (size_t)fm_simt::W * w->stack_bytes) return;
    if (a >= (const char*)w && a < (const char*)(w + 1)) return;  // the emulator's own wave record
    t_in_hook = true;
    if (!t_gshadow) t_gshadow = new std::unordered_map<uintptr_t, Shadow>();
    if (t_gblock != w->block.x || t_gwave != (const void*)w) {
      t_gshadow->clear();
      t_gblock = w->block.x;
      t_gwave = w;
    }
    const unsigned ep = w->epoch;
    const int l = w->lane;
    t_off = -1;
    for (size_t b = 0; b < n; b++) {
      // reads look only at bytes the block has written (the model tables, read by every lane, stay out of the map)
      auto it = write ? t_gshadow->try_emplace((uintptr_t)(a + b)).first : t_gshadow->find((uintptr_t)(a + b));
      if (it == t_gshadow->end()) continue;
      Shadow& s = it->second;
      if (!write) {
        if (s.wr_epoch == ep && s.wr_lane != l) note(pc, s.wr_pc, 0);
        if (s.rd_epoch != ep) {
          s.rd_epoch = ep;
          s.rd_mask = 0;
        }
        s.rd_mask |= 1ull << l;
        s.rd_pc = pc;
      } else {
        if (s.rd_epoch == ep && (s.rd_mask & ~(1ull << l))) note(pc, s.rd_pc, 1);
        if (s.wr_epoch == ep && s.wr_lane != l) note(pc, s.wr_pc, 2);
        s.wr_epoch = ep;
        s.wr_lane = l;
        s.wr_pc = pc;
      }
    }
    t_in_hook = false;
    return;
  }
  if (t_base != w->lds || t_nshadow < w->lds_bytes + 1) {
    std::free(t_shadow);
    t_nshadow = w->lds_bytes + 1;
    t_shadow = (Shadow*)std::malloc(t_nshadow * sizeof(Shadow));
    for (size_t i = 0; i < t_nshadow; i++) {
      t_shadow[i].wr_epoch = t_shadow[i].rd_epoch = ~0u;
      t_shadow[i].wr_lane = -1;
      t_shadow[i].rd_mask = 0;
      t_shadow[i].wr_pc = t_shadow[i].rd_pc = nullptr;
    }
    t_base = w->lds;
  }
  const unsigned ep = w->epoch;
  const int l = w->lane;
  for (size_t o = (size_t)(a - w->lds); o < (size_t)(a + n - w->lds) && o < t_nshadow; o++) {
    Shadow& s = t_shadow[o];
    t_off = (long)o;
    if (!write) {
      if (s.wr_epoch == ep && s.wr_lane != l) note(pc, s.wr_pc, 0);
      if (s.rd_epoch != ep) {
        s.rd_epoch = ep;
        s.rd_mask = 0;
      }
      s.rd_mask |= 1ull << l;
      s.rd_pc = pc;
    } else {
      if (s.rd_epoch == ep && (s.rd_mask & ~(1ull << l))) note(pc, s.rd_pc, 1);
      if (s.wr_epoch == ep && s.wr_lane != l) note(pc, s.wr_pc, 2);
      s.wr_epoch = ep;
      s.wr_lane = l;
      s.wr_pc = pc;
    }
  }
}
}  // namespace fm_race

#define FM_RD(n)                                                                                              \
  extern "C" FM_NO_INSTR void __tsan_read##n(void* a) {                          \
    fm_race::access(a, n, false, __builtin_return_address(0));                                              \
  }                                                                                                          \
  extern "C" FM_NO_INSTR void __tsan_write##n(void* a) {                         \
    fm_race::access(a, n, true, __builtin_return_address(0));                                               \
  }
FM_RD(1)
FM_RD(2)
FM_RD(4)
FM_RD(8)
FM_RD(16)
#define FM_URD(n)                                                                                             \
  extern "C" FM_NO_INSTR void __tsan_unaligned_read##n(void* a) {                \
    fm_race::access(a, n, false, __builtin_return_address(0));                                              \
  }                                                                                                          \
  extern "C" FM_NO_INSTR void __tsan_unaligned_write##n(void* a) {               \
    fm_race::access(a, n, true, __builtin_return_address(0));                                               \
  }
FM_URD(2)
FM_URD(4)
FM_URD(8)
FM_URD(16)
extern "C" FM_NO_INSTR void __tsan_init() {}
extern "C" FM_NO_INSTR void __tsan_func_entry(void*) {}
extern "C" FM_NO_INSTR void __tsan_func_exit() {}
extern "C" FM_NO_INSTR void __tsan_vptr_read(void**) {}
extern "C" FM_NO_INSTR void __tsan_vptr_update(void**, void*) {}
extern "C" FM_NO_INSTR void* __tsan_memcpy(void* d, const void* s, size_t n) {
  fm_race::access(s, n, false, __builtin_return_address(0));
  fm_race::access(d, n, true, __builtin_return_address(0));
  return std::memcpy(d, s, n);
}
extern "C" FM_NO_INSTR void* __tsan_memset(void* d, int c, size_t n) {
  fm_race::access(d, n, true, __builtin_return_address(0));
  return std::memset(d, c, n);
}
extern "C" FM_NO_INSTR uint32_t __tsan_atomic32_fetch_add(volatile uint32_t* a, uint32_t v,
                                                                                     int) {
  return __atomic_fetch_add(a, v, __ATOMIC_SEQ_CST);
}
extern "C" FM_NO_INSTR uint8_t __tsan_atomic8_load(const volatile uint8_t* a, int) {
  return __atomic_load_n(a, __ATOMIC_SEQ_CST);
}
// the recorded races as "kind pc_offset other_pc_offset" lines (offsets into this library, for llvm-symbolizer)
extern "C" FM_NO_INSTR int fm_race_report(char* out, int cap) {
  std::lock_guard<std::mutex> g(fm_race::g_mu);
  Dl_info di{};
  dladdr((void*)&fm_race_report, &di);
  std::string s = "lay";
  for (int v : fm_race::g_lay) s += " " + std::to_string(v);
  s += "\n";
  for (auto& r : fm_race::g_races) {
    char line[128];
    const void* other = std::get<1>(r.first);  // null for the bounds kinds (3, 4): printed as 0
    std::snprintf(line, sizeof line, "%d 0x%lx 0x%lx %ld\n", std::get<2>(r.first),
                  (long)((const char*)std::get<0>(r.first) - (const char*)di.dli_fbase),
                  other ? (long)((const char*)other - (const char*)di.dli_fbase) : 0L, r.second);
    s += line;
  }
  if (out && cap > 0) std::snprintf(out, (size_t)cap, "%s", s.c_str());
  return (int)fm_race::g_races.size();
}
#endif

// self-test of the emulated wave (tests/test_cpu_backend.py): every cross-lane operation the kernel uses against its
// ISA definition, on one workgroup.  Returns 0 or the number of the first failed check.
extern "C" int fm_cpu_selftest() {
  int fail = 0;
  fm_simt::launch(1u, 1024, nullptr, [&fail]() {
    const int l = (int)threadIdx.x;
    auto check = [&fail](bool ok, int id) {
      if (!ok && !fail) fail = id;
    };
    // ballot, readlane, readfirstlane
    const unsigned long long b = __ballot(l % 3 == 0);
    unsigned long long ref = 0;
    for (int i = 0; i < 64; i += 3) ref |= 1ull << i;
    check(b == ref, 1);
    check(__builtin_amdgcn_readlane(100 + l, 37) == 137, 2);
    check(__builtin_amdgcn_readfirstlane(7 * (l / 64) + 1) == 1, 3);  // applied to wave-uniform values only
    // bpermute / shfl
    check(__shfl(1000 + l, (l * 5) & 63) == 1000 + ((l * 5) & 63), 4);
    check(__shfl_xor(l, 13) == (l ^ 13), 5);
    check(__shfl(0.5 * l, 63 - l) == 0.5 * (63 - l), 6);
    // DPP: quad_perm [1,0,3,2], row_shr:1 (lane 0 of a row keeps old), row_ror:4, row_bcast:15 / 31
    check(__builtin_amdgcn_update_dpp(-1, l, 0xb1, 0xf, 0xf, false) == (l ^ 1), 7);
    check(__builtin_amdgcn_update_dpp(-1, l, 0x111, 0xf, 0xf, false) == ((l & 15) ? l - 1 : -1), 8);
    check(__builtin_amdgcn_update_dpp(-1, l, 0x124, 0xf, 0xf, false) == ((l & ~15) | ((l - 4) & 15)), 9);
    check(__builtin_amdgcn_update_dpp(-1, l, 0x142, 0xf, 0xf, false) == (l >= 16 ? (l & ~15) - 1 : -1), 10);
    check(__builtin_amdgcn_update_dpp(-1, l, 0x143, 0xf, 0xf, false) == (l >= 32 ? 31 : -1), 11);
    // mbcnt: lanes below this one in a mask
    const unsigned long long m = 0xF0F0F0F0F0F0F0F0ull;
    const unsigned c = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
    check((int)c == __builtin_popcountll(m & ((l == 0) ? 0ull : (~0ull >> (64 - l)))), 12);
    // MFMA 16x16x4: D = A B + C with A[i][k] = i + k, B[k][j] = k - j, C = 1
    const float a = (float)((l & 15) + (l >> 4)), bb = (float)((l >> 4) - (l & 15));
    fm_host_f32x4 cc = {1.f, 1.f, 1.f, 1.f};
    const fm_host_f32x4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bb, cc, 0, 0, 0);
    for (int r = 0; r < 4; r++) {
      const int i = 4 * (l >> 4) + r, j = l & 15;
      float e = 1.f;
      for (int k = 0; k < 4; k++) e += (float)(i + k) * (float)(k - j);
      check(d[r] == e, 13);
    }
    // the barrier orders LDS hand-offs between lanes
    int* lds = (int*)::fm_simt::wave().lds;
    lds[l] = 3 * l;
    __syncthreads();
    check(lds[63 - l] == 3 * (63 - l), 14);
  });
  return fail;
}

namespace fm {

template <typename T>
static void cpu_step(const StepParams<T>& p, int num_arenas, int lds_bytes, bool ik) {
  if (ik)
    fm_simt::launch((unsigned)num_arenas, (size_t)lds_bytes, &p, [&p]() { step_kernel<T, Dims, true>(p); });
  else
    fm_simt::launch((unsigned)num_arenas, (size_t)lds_bytes, &p, [&p]() { step_kernel<T, Dims, false>(p); });
}

template <typename T>
static void cpu_reset(const Model<T>& M, const State<T>& S, const Lay& L, float* obs, const uint8_t* mask,
                      int num_arenas, int lds_bytes) {
  fm_simt::launch((unsigned)num_arenas, (size_t)lds_bytes, nullptr,
                  [&]() { reset_kernel<T, Dims>(M, S, L, obs, mask); });
}

template <typename T>
static void cpu_debug(const Model<T>& M, const State<T>& S, const Lay& L, int arena, int actuated, double* out,
                      int lds_bytes) {
  fm_simt::launch(1u, (size_t)lds_bytes, nullptr, [&]() { debug_kernel<T, Dims>(M, S, L, arena, actuated, out); });
}

}  // namespace fm

// entry points for fm_api.hip (the parameter blocks are the same structs, laid out from the same fm_dev.hpp)
// the LDS layout and the scratch blocks of a step launch (tools/lds_race_check.py maps the racing offsets to the
// layout's arrays; the bounds checks use both; also called by the compile-time scene objects, fm_cpu_fixed.cpp)
extern "C" void fm_cpu_note_launch(const void* lay, const void* spill, long long stride, long long n) {
#ifdef FM_RACE_DETECT
  std::memcpy(fm_race::g_lay, lay, sizeof(fm::Lay));
  fm_race::g_spill = (const char*)spill;
  fm_race::g_spill_stride = stride;
  fm_race::g_spill_n = n;
#else
  (void)lay;
  (void)spill;
  (void)stride;
  (void)n;
#endif
}
template <typename T>
static void note_launch(const void* params, int num_arenas) {
  const fm::StepParams<T>& p = *(const fm::StepParams<T>*)params;
  fm_cpu_note_launch(&p.L, (const char*)p.S.spill, p.S.spill_stride, p.M.dm.N);
  (void)num_arenas;
}
extern "C" void fm_cpu_step(int fp64, const void* params, int num_arenas, int lds_bytes, int ik) {
  if (fp64)
    note_launch<double>(params, num_arenas);
  else
    note_launch<float>(params, num_arenas);
  if (fp64)
    fm::cpu_step<double>(*(const fm::StepParams<double>*)params, num_arenas, lds_bytes, ik != 0);
  else
    fm::cpu_step<float>(*(const fm::StepParams<float>*)params, num_arenas, lds_bytes, ik != 0);
}
extern "C" void fm_cpu_reset(int fp64, const void* model, const void* state, const void* lay, float* obs,
                             const uint8_t* mask, int num_arenas, int lds_bytes) {
  if (fp64)
    fm::cpu_reset<double>(*(const fm::Model<double>*)model, *(const fm::State<double>*)state, *(const fm::Lay*)lay, obs,
                          mask, num_arenas, lds_bytes);
  else
    fm::cpu_reset<float>(*(const fm::Model<float>*)model, *(const fm::State<float>*)state, *(const fm::Lay*)lay, obs,
                         mask, num_arenas, lds_bytes);
}
extern "C" void fm_cpu_debug(int fp64, const void* model, const void* state, const void* lay, int arena, int actuated,
                             double* out, int lds_bytes) {
  if (fp64)
    fm::cpu_debug<double>(*(const fm::Model<double>*)model, *(const fm::State<double>*)state, *(const fm::Lay*)lay,
                          arena, actuated, out, lds_bytes);
  else
    fm::cpu_debug<float>(*(const fm::Model<float>*)model, *(const fm::State<float>*)state, *(const fm::Lay*)lay, arena,
                         actuated, out, lds_bytes);
}
