// GEMV instantiations for epilogue ZMI_EPI_STORE (see zmi_gemv_impl.h)
#include "zmi_gemv_impl.h"

namespace zmi_gemv {
hipError_t launch_epi0(const ZmiGemvArgs& a, int mt, int nf, hipStream_t s) {
  return launch_mt<ZMI_EPI_STORE>(a, mt, nf, s);
}
}  // namespace zmi_gemv
