// GEMV instantiations for epilogue ZMI_EPI_LOGITS (see zmi_gemv_impl.h)
#include "zmi_gemv_impl.h"

namespace zmi_gemv {
hipError_t launch_epi4(const ZmiGemvArgs& a, int mt, int nf, hipStream_t s) {
  return launch_mt<ZMI_EPI_LOGITS>(a, mt, nf, s);
}
}  // namespace zmi_gemv
