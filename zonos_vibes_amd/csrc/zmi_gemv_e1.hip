// GEMV instantiations for the epilogue ZMI_EPI_RESIDUAL (one translation unit per epilogue: build parallelism)
#include "zmi_gemv_impl.h"

namespace zmi_gemv {
hipError_t launch_epi1(const ZmiGemvArgs& a, hipStream_t s) { return launch<ZMI_EPI_RESIDUAL>(a, s); }
}  // namespace zmi_gemv
