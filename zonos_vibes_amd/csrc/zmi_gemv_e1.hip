// GEMV instantiations for epilogue ZMI_EPI_RESIDUAL (see zmi_gemv_impl.h)
#include "zmi_gemv_impl.h"

namespace zmi_gemv {
hipError_t launch_epi1(const ZmiGemvArgs& a, int mt, int nf, hipStream_t s) {
  return launch_mt<ZMI_EPI_RESIDUAL>(a, mt, nf, s);
}
}  // namespace zmi_gemv
