// fm_cpu_fixed.cpp -- the CPU backend's compile-time scene kernels: step_kernel<T, FixedDims<FM_A, FM_K>> (and, for
// the benchmark scene, the float64 wide rerun kernel FixedDims<2, 4, true>) compiled for the host with the wave
// emulated (fm_simt_host.hpp; the emulator and the runtime-dims kernels live in fm_cpu.cpp).  One object per scene,
// like the GPU's fm_fixed.hip: the host runs exactly the code paths the GPU benchmarks run -- the spilled global
// scratch blocks, the cached midphase, the arrowhead / tree-block / matrix-core factors, the 64-contact capacity with
// its abandon-and-resume hand-off to the wide kernel -- so the race detector (FM_RACE_DETECT) and the host sanitizers
// see them too.
#define fm fm_cpu_ns
#include "fm_device.hpp"

#ifndef FM_A
#error "compile with -DFM_A=<arms> -DFM_K=<objects>"
#endif

#define FM_CAT2(a, b, c) a##_##b##_##c
#define FM_CAT(a, b, c) FM_CAT2(a, b, c)

extern "C" void fm_cpu_note_launch(const void* lay, const void* spill, long long stride, long long n);

namespace fm {

template <typename T, typename DIM, bool IK>
static void body(const void* p) {
  step_kernel<T, DIM, IK>(*(const StepParams<T>*)p);
}

template <typename T, typename DIM, typename DIK = DIM>
static void run(const void* params, int grid, int lds_bytes, bool ik) {
  const StepParams<T>& p = *(const StepParams<T>*)params;
  // the scratch blocks the kernel uses (none for the wide rerun kernel: its workspace is all LDS)
  fm_cpu_note_launch(&p.L, DIM::spill ? (const char*)p.S.spill : nullptr, p.S.spill_stride, p.M.dm.N);
  ::fm_simt::launch_kernel((unsigned)grid, (size_t)lds_bytes, params, ik ? &body<T, DIK, true> : &body<T, DIM, false>);
}

}  // namespace fm

// wide = 1: the scene's float64 wide-capacity rerun kernel (the benchmark scene (2,4) only)
extern "C" int FM_CAT(fm_cpu_step_fixed, FM_A, FM_K)(int fp64, int wide, const void* params, int grid, int lds_bytes,
                                                      int ik) {
  if (wide) {
#if FM_A == 2 && FM_K == 4
    if (!fp64) return 1;
    fm::run<double, fm::FixedDims<FM_A, FM_K, true>>(params, grid, lds_bytes, ik != 0);
    return 0;
#else
    return 1;
#endif
  }
  if (fp64)
    fm::run<double, fm::FixedDims<FM_A, FM_K>, fm::FixedDimsIK<double, FM_A, FM_K>>(params, grid, lds_bytes, ik != 0);
  else
    fm::run<float, fm::FixedDims<FM_A, FM_K>, fm::FixedDimsIK<float, FM_A, FM_K>>(params, grid, lds_bytes, ik != 0);
  return 0;
}
