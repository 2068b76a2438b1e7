// GEMV instantiations for epilogue ZMI_EPI_SWIGLU: the MFMA strip kernel (zmi_gemv_impl.h, prefill and
// batched decode) and the 8-column decode kernel (zmi_gemv8_impl.h, M <= 8)
#include "zmi_gemv_impl.h"
#include "zmi_gemv8_impl.h"

namespace zmi_gemv {
hipError_t launch_epi3(const ZmiGemvArgs& a, int mt, int nf, hipStream_t s) {
  return launch_mt<ZMI_EPI_SWIGLU>(a, mt, nf, s);
}
hipError_t launch8_epi3(const ZmiGemvArgs& a, hipStream_t s) { return zmi_gemv8::launch8<ZMI_EPI_SWIGLU>(a, s); }
}  // namespace zmi_gemv
