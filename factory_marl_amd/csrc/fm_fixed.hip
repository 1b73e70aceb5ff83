// fm_fixed.hip -- one compile-time scene (FM_A arms, FM_K objects): instantiates the env-step kernel
// with FixedDims<FM_A, FM_K> (constexpr dims and LDS layout) for one precision (FM_PREC 32 or 64).  Built
// once per scene and precision by the Makefile (fm_fixed_<A>_<K>_f<P>.o) so they compile in parallel.
#include "fm_device.hpp"

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

// the benchmark scene keeps 4 arenas (one wave per SIMD) per CU: its fp32 workspace must stay within a quarter of
// the CU's 160 KiB of LDS (the midphase cache was sized to fit, fm_dev.hpp mc_cap)
static_assert(!(FM_A == 2 && FM_K == 4 && FM_PREC == 32) || FixedDims<2, 4>::template layout<4>().total <= 160 * 1024 / 4,
              "(2,4) fp32 workspace above 40 KiB: 3 arenas per CU");

template <typename T, int A, int K>
hipError_t fixed_set_attr(int lds_bytes) {
  hipError_t e = hipFuncSetAttribute((const void*)step_kernel<T, FixedDims<A, K>, false>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)step_kernel<T, FixedDims<A, K>, true>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
}

// ik: the env class composes IK proposals (every class but AllFullRLProgressRewardEnv)
template <typename T, int A, int K>
void fixed_launch(const StepParams<T>& p, int num_arenas, int lds_bytes, hipStream_t stream, bool ik) {
  if (ik)
    hipLaunchKernelGGL((step_kernel<T, FixedDims<A, K>, true>), dim3(num_arenas), dim3(WAVE), lds_bytes, stream, p);
  else
    hipLaunchKernelGGL((step_kernel<T, FixedDims<A, K>, false>), dim3(num_arenas), dim3(WAVE), lds_bytes, stream, p);
}

template hipError_t fixed_set_attr<FM_REAL, FM_A, FM_K>(int);
template void fixed_launch<FM_REAL, FM_A, FM_K>(const StepParams<FM_REAL>&, int, int, hipStream_t, bool);

}  // namespace fm
