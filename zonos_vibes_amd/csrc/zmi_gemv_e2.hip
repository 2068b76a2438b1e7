// GEMV instantiations for the epilogue ZMI_EPI_QKV (one translation unit per epilogue: build parallelism)
#include "zmi_gemv_impl.h"

namespace zmi_gemv {
hipError_t launch_epi2(const ZmiGemvArgs& a, hipStream_t s) { return launch<ZMI_EPI_QKV>(a, s); }
}  // namespace zmi_gemv
