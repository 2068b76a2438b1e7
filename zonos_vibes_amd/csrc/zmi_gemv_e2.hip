// GEMV instantiations for epilogue ZMI_EPI_QKV: the MFMA strip kernel (zmi_gemv_impl.h, prefill and
// batched decode) and the 8-column decode kernel (zmi_gemv8_impl.h, M <= 8)
#include "zmi_gemv_impl.h"
#include "zmi_gemv8_impl.h"

namespace zmi_gemv {
hipError_t launch_epi2(const ZmiGemvArgs& a, int mt, int nf, hipStream_t s) {
  return launch_mt<ZMI_EPI_QKV>(a, mt, nf, s);
}
hipError_t launch8_epi2(const ZmiGemvArgs& a, hipStream_t s) { return zmi_gemv8::launch8<ZMI_EPI_QKV>(a, s); }
}  // namespace zmi_gemv
