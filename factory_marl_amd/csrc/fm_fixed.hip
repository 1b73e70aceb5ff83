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

template <typename T, int A, int K>
hipError_t fixed_set_attr(int lds_bytes) {
  return hipFuncSetAttribute((const void*)step_kernel<T, FixedDims<A, K>>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             lds_bytes);
}

template <typename T, int A, int K>
void fixed_launch(const StepParams<T>& p, int num_arenas, int lds_bytes, hipStream_t stream) {
  hipLaunchKernelGGL((step_kernel<T, FixedDims<A, K>>), dim3(num_arenas), dim3(WAVE), lds_bytes, stream, p);
}

template hipError_t fixed_set_attr<FM_REAL, FM_A, FM_K>(int);
template void fixed_launch<FM_REAL, FM_A, FM_K>(const StepParams<FM_REAL>&, int, int, hipStream_t);

}  // namespace fm
