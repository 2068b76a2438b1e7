// GEMV instantiations for epilogue ZMI_EPI_SWIGLU (see zmi_gemv_impl.h)
#include "zmi_gemv_impl.h"

namespace zmi_gemv {
hipError_t launch_epi3(const ZmiGemvArgs& a, int mt, int nf, hipStream_t s) {
  return launch_mt<ZMI_EPI_SWIGLU>(a, mt, nf, s);
}
}  // namespace zmi_gemv
