// Library plumbing: error reporting, synthetic-weight fill, hipGraph capture helpers.
#include <stdio.h>
#include <string.h>

#include "zmi_common.h"
#include "zmi_kernels.h"

static thread_local char g_err[512] = "";

int zmi_fail(hipError_t e, const char* what, const char* file, int line) {
  snprintf(g_err, sizeof(g_err), "%s failed: %s (%s:%d)", what, hipGetErrorString(e), file, line);
  return (int)e == 0 ? -1 : (int)e;
}

int zmi_fail_msg(const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return -1;
}

extern "C" const char* zmi_last_error(void) { return g_err; }
extern "C" int zmi_version(void) { return 2; }

namespace {
// Same stream as zonos_vibes_amd/synthetic.py: key + (i+1)*GOLDEN -> splitmix64 -> 24-bit uniform.
__global__ void fill_kernel(void* dst, int64_t n, uint64_t key, float scale, float offset, int dtype) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t z = mix64(key + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull);
  const float u = ((float)(z >> 40) - 8388608.0f) * (1.0f / 8388608.0f);
  float v = u * scale;
  if (offset != 0.0f) v = v + offset;
  if (dtype == 0)
    reinterpret_cast<bf16_t*>(dst)[i] = (bf16_t)f2bf(v);
  else
    reinterpret_cast<float*>(dst)[i] = v;
}
}  // namespace

extern "C" int zmi_fill_uniform(void* dst, int64_t n, uint64_t key, float scale, float offset, int dtype,
                                void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fill_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, dst, n, key,
                     scale, offset, dtype);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_graph_begin(void* stream) {
  ZMI_CHECK(hipStreamBeginCapture((hipStream_t)stream, hipStreamCaptureModeRelaxed));
  return 0;
}

extern "C" int zmi_graph_end(void* stream, void** graph_exec) {
  hipGraph_t g;
  ZMI_CHECK(hipStreamEndCapture((hipStream_t)stream, &g));
  hipGraphExec_t ge;
  hipError_t e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  ZMI_CHECK(e);
  *graph_exec = (void*)ge;
  return 0;
}

extern "C" int zmi_graph_launch(void* graph_exec, int times, void* stream) {
  for (int i = 0; i < times; ++i) ZMI_CHECK(hipGraphLaunch((hipGraphExec_t)graph_exec, (hipStream_t)stream));
  return 0;
}

extern "C" int zmi_graph_destroy(void* graph_exec) {
  if (graph_exec) ZMI_CHECK(hipGraphExecDestroy((hipGraphExec_t)graph_exec));
  return 0;
}
