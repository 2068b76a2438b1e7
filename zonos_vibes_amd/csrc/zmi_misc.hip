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
extern "C" int zmi_version(void) { return 1; }

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

// ---- Infinity-Cache (MALL) prefetch: stream a byte range through the memory side so a later
// kernel's reads of it hit on-die (MI355X_MICROARCH.md "Infinity Cache"). Every lane keeps 8
// 16-B loads in flight; the loaded values are folded and stored only under a runtime-false flag
// so the loads cannot be elided.
namespace {
__global__ __launch_bounds__(256) void prefetch_kernel(const uint4* __restrict__ p, int64_t n16, unsigned* sink,
                                                       int never) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  unsigned acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += 8 * stride) {
    uint4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t e = i + j * stride;
      v[j] = p[e < n16 ? e : n16 - 1];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc ^= v[j].x ^ v[j].w;
  }
  if (never) sink[threadIdx.x] = acc;
}
}  // namespace

extern "C" int zmi_prefetch(const void* p, int64_t bytes, int blocks, void* stream) {
  if (bytes < 16) return 0;
  if (blocks <= 0) blocks = 256;
  hipLaunchKernelGGL(prefetch_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const uint4*)p, bytes / 16,
                     (unsigned*)nullptr, 0);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

// ---- LayerNorm rows (prefill pre-pass) ----------------------------------------------------------
// out[r] = bf16((x[r] rstd - mean rstd) * w + b), mean / centred variance in fp32 (nn.LayerNorm on
// bf16, reference zonos/backbone/_torch.py:88,90): the same formula as the GEMV LayerNorm prologue.
// Run once per prefill layer input so the (many-strip) prefill GEMMs take plain rows instead of
// re-normalising the whole row block in every workgroup.
namespace {
__global__ __launch_bounds__(256) void layernorm_rows_kernel(const bf16_t* x, int ldx, int k, const bf16_t* w,
                                                             const bf16_t* b, float eps, bf16_t* out, int ldo) {
  __shared__ float red[4];
  const int r = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const bf16_t* xr = x + (size_t)r * ldx;
  constexpr int MAXV = 4;  // uint4 (8 bf16) per thread: K <= 8192
  uint4 v[MAXV];
  const int nv = k / 8;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = t + i * 256;
    v[i] = c < nv ? reinterpret_cast<const uint4*>(xr)[c] : uint4{0u, 0u, 0u, 0u};
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const uint32_t u[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) s += bf2f(u[j]) + bf2f(u[j] >> 16);
  }
  s = wave_sum(s);
  if (lane == 0) red[wave] = s;
  __syncthreads();
  const float mean = ((red[0] + red[1]) + (red[2] + red[3])) / (float)k;
  __syncthreads();
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    if (t + i * 256 >= nv) continue;
    const uint32_t u[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d0 = bf2f(u[j]) - mean, d1 = bf2f(u[j] >> 16) - mean;
      ss += d0 * d0;
      ss += d1 * d1;
    }
  }
  ss = wave_sum(ss);
  if (lane == 0) red[wave] = ss;
  __syncthreads();
  const float rstd = 1.0f / sqrtf(((red[0] + red[1]) + (red[2] + red[3])) / (float)k + eps), nb = -mean * rstd;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = t + i * 256;
    if (c >= nv) continue;
    const uint32_t u[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
    const uint4 wv = reinterpret_cast<const uint4*>(w)[c], bv = reinterpret_cast<const uint4*>(b)[c];
    const uint32_t uw[4] = {wv.x, wv.y, wv.z, wv.w}, ub[4] = {bv.x, bv.y, bv.z, bv.w};
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float y0 = (bf2f(u[j]) * rstd + nb) * bf2f(uw[j]) + bf2f(ub[j]);
      const float y1 = (bf2f(u[j] >> 16) * rstd + nb) * bf2f(uw[j] >> 16) + bf2f(ub[j] >> 16);
      o[j] = f2bf(y0) | (f2bf(y1) << 16);
    }
    reinterpret_cast<uint4*>(out + (size_t)r * ldo)[c] = uint4{o[0], o[1], o[2], o[3]};
  }
}
}  // namespace

extern "C" int zmi_layernorm_rows(const void* x, int ldx, int m, int k, const void* w, const void* b, float eps,
                                  void* out, int ldo, void* stream) {
  if (k % 8 || k > 8192 || ldx % 8 || ldo % 8) return zmi_fail_msg("layernorm_rows: k, ldx, ldo must be multiples of 8, k <= 8192");
  if (m <= 0) return 0;
  hipLaunchKernelGGL(layernorm_rows_kernel, dim3(m), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, ldx, k,
                     (const bf16_t*)w, (const bf16_t*)b, eps, (bf16_t*)out, ldo);
  ZMI_CHECK(hipGetLastError());
  return 0;
}
