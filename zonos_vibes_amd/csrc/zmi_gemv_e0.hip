// GEMV instantiations for the epilogue ZMI_EPI_STORE (one translation unit per epilogue: build parallelism)
#include "zmi_gemv_impl.h"

namespace zmi_gemv {
hipError_t launch_epi0(const ZmiGemvArgs& a, hipStream_t s) { return launch<ZMI_EPI_STORE>(a, s); }
}  // namespace zmi_gemv
