// fm_fixed.hip -- one compile-time scene (FM_A arms, FM_K objects): instantiates the env-step kernel
// with FixedDims<FM_A, FM_K> (constexpr dims and LDS layout) for one precision (FM_PREC 32 or 64).  Built
// once per scene and precision by the Makefile (fm_fixed_<A>_<K>_f<P>.o) so they compile in parallel.
// FM_WIDE=1: the same scene's wide-capacity rerun kernel instead (fm_rerun_f64.o, the benchmark scene; float64 for the
// abandoned env-steps of both builds).
#include "fm_device.hpp"

#ifndef FM_WIDE
#define FM_WIDE 0
#endif
#ifndef FM_A
#error "compile with -DFM_A=<arms> -DFM_K=<objects> -DFM_PREC=<32|64>"
#endif
#if FM_PREC == 32
#define FM_REAL float
#elif FM_PREC == 64
#define FM_REAL double
#else
#error "FM_PREC must be 32 or 64"
#endif

namespace fm {

// the benchmark scene runs two waves (arenas) per SIMD, 8 per CU (FM_WAVES_PER_EU=2 for its objects, Makefile): its
// workspace must stay within an eighth of the CU's 160 KiB of LDS with the Hessian and contact records spilled
static_assert(!(FM_A == 2 && FM_K == 4 && FM_PREC == 32 && FM_SPILL_FIXED) ||
                  FixedDims<2, 4>::template layout<4>().total <= 160 * 1024 / 8,
              "(2,4) fp32 workspace above 20 KiB: fewer than 8 arenas per CU");

// the IK classes' kernels run in the handle's layout (FixedDimsIK differs only in DIM::f64arms)
static_assert(FixedDimsIK<FM_REAL, FM_A, FM_K>::template layout<sizeof(FM_REAL)>().total ==
                      FixedDims<FM_A, FM_K>::template layout<sizeof(FM_REAL)>().total &&
                  FixedDimsIK<FM_REAL, FM_A, FM_K>::template layout<sizeof(FM_REAL)>().gtotal ==
                      FixedDims<FM_A, FM_K>::template layout<sizeof(FM_REAL)>().gtotal,
              "the IK instantiation's layout differs");

template <typename T, int A, int K>
hipError_t fixed_set_attr(int lds_bytes) {
  hipError_t e = hipFuncSetAttribute((const void*)step_kernel<T, FixedDims<A, K>, false>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)step_kernel<T, FixedDimsIK<T, A, K>, true>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
}

// ik: the env class composes IK proposals (every class but AllFullRLProgressRewardEnv)
template <typename T, int A, int K>
void fixed_launch(const StepParams<T>& p, int num_arenas, int lds_bytes, hipStream_t stream, bool ik) {
  if (ik)
    hipLaunchKernelGGL((step_kernel<T, FixedDimsIK<T, A, K>, true>), dim3(num_arenas), dim3(WAVE), lds_bytes, stream,
                       p);
  else
    hipLaunchKernelGGL((step_kernel<T, FixedDims<A, K>, false>), dim3(num_arenas), dim3(WAVE), lds_bytes, stream, p);
}

#if FM_WIDE
// the benchmark scene's wide-capacity rerun (FixedDims<A, K, true>): the workgroups step the arenas S.rerun[1 + i],
// i < S.rerun[0], in a grid-stride loop; a small grid (the list is short and usually empty: one workgroup per arena
// of the handle cost 2.5 % of the config-2 env-step in dispatch alone, gpurun_out/r04c quick_c vs quick_c_norerun)
template <typename T, int A, int K>
hipError_t rerun_set_attr() {
  const int lds = FixedDims<A, K, true>::template layout<sizeof(T)>().total;
  hipError_t e = hipFuncSetAttribute((const void*)step_kernel<T, FixedDims<A, K, true>, false>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)step_kernel<T, FixedDims<A, K, true>, true>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, lds);
}

template <typename T, int A, int K>
Lay rerun_layout() {
  return FixedDims<A, K, true>::template layout<sizeof(T)>();
}

template <typename T, int A, int K>
void rerun_launch(const StepParams<T>& p, int num_arenas, hipStream_t stream, bool ik) {
  const int lds = FixedDims<A, K, true>::template layout<sizeof(T)>().total;
  const dim3 grid(num_arenas < 256 ? num_arenas : 256);
  if (ik)
    hipLaunchKernelGGL((step_kernel<T, FixedDims<A, K, true>, true>), grid, dim3(WAVE), lds, stream, p);
  else
    hipLaunchKernelGGL((step_kernel<T, FixedDims<A, K, true>, false>), grid, dim3(WAVE), lds, stream, p);
}

static_assert(FixedDims<FM_A, FM_K, true>::template layout<sizeof(FM_REAL)>().total <= 160 * 1024,
              "wide rerun workspace exceeds the CU's LDS");
template hipError_t rerun_set_attr<FM_REAL, FM_A, FM_K>();
template Lay rerun_layout<FM_REAL, FM_A, FM_K>();
template void rerun_launch<FM_REAL, FM_A, FM_K>(const StepParams<FM_REAL>&, int, hipStream_t, bool);
#else
template hipError_t fixed_set_attr<FM_REAL, FM_A, FM_K>(int);
template void fixed_launch<FM_REAL, FM_A, FM_K>(const StepParams<FM_REAL>&, int, int, hipStream_t, bool);
#endif

}  // namespace fm
