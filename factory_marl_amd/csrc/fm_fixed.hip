// fm_fixed.hip -- one compile-time scene (FM_A arms, FM_K objects): instantiates the env-step kernel
// with FixedDims<FM_A, FM_K> (constexpr dims and LDS layout) for fp32 and fp64.  Built once per scene by
// the Makefile (fm_fixed_<A>_<K>.o) so the scenes compile in parallel.
#include "fm_device.hpp"

#ifndef FM_A
#error "compile with -DFM_A=<arms> -DFM_K=<objects>"
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

template hipError_t fixed_set_attr<float, FM_A, FM_K>(int);
template hipError_t fixed_set_attr<double, FM_A, FM_K>(int);
template void fixed_launch<float, FM_A, FM_K>(const StepParams<float>&, int, int, hipStream_t);
template void fixed_launch<double, FM_A, FM_K>(const StepParams<double>&, int, int, hipStream_t);

}  // namespace fm
