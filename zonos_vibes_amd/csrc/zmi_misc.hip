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
// 4: zmi_dac_conv / conv_t / conv_out take channel-blocked multi-tap weights [tap][ci / 32][co][32] (round 5), the
//    ZMI_OPT_GEMM_ROWS bit meanings of round 5; 5: ZMI_OPT_XC_HANDOFF (option 2) and zmi_xcd_dealing (round 6);
//    6: ZMI_PRO_GRMS_G and ZmiMamba2Args.gz_g (round 6)
extern "C" int zmi_version(void) { return 6; }

// launch-geometry knobs (speed only: no option changes a result bit); defaults in the table
static int g_opts[ZMI_OPT_COUNT] = {1, 3, 0, 0, 1, 8, 2, 1, 1, 0, 1, 256, 5, 29, 128, 0, 256, 1};
int zmi_option(int which) { return (which >= 0 && which < ZMI_OPT_COUNT) ? g_opts[which] : 0; }
extern "C" int zmi_set_option(int which, int value) {
  if (which < 0 || which >= ZMI_OPT_COUNT) return zmi_fail_msg("zmi_set_option: unknown option");
  g_opts[which] = value;
  return 0;
}
extern "C" int zmi_get_option(int which) { return zmi_option(which); }
static int g_cus = 0;
int zmi_cu_count() {
  if (!g_cus) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      g_cus = n;
    else
      g_cus = 256;
  }
  return g_cus;
}

namespace {
// zmi_xcd_dealing's probe: each workgroup records the XCD it runs on (a vector store of an SGPR read)
__global__ void xcc_kernel(unsigned* xcc) {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  if (threadIdx.x == 0) xcc[blockIdx.x] = v;
}
}  // namespace

extern "C" int zmi_xcd_dealing(void* stream) {
  constexpr int NB = 1024;
  unsigned* d = nullptr;
  unsigned h[NB];
  hipStream_t s = (hipStream_t)stream;
  ZMI_CHECK(hipMalloc(&d, NB * sizeof(unsigned)));
  hipLaunchKernelGGL(xcc_kernel, dim3(NB), dim3(64), 0, s, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(d);
  ZMI_CHECK(e);
  bool seen[8] = {};
  for (int b = 0; b < 8; ++b) {
    if (h[b] >= 8 || seen[h[b]]) return 0;
    seen[h[b]] = true;
  }
  for (int b = 8; b < NB; ++b)
    if (h[b] != h[b & 7]) return 0;
  return 1;
}

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

// ---- LayerNorm of whole rows (nn.LayerNorm, reference zonos/backbone/_torch.py:62,88,90) -------------
// One wave per row, the parts of zmi_common.h's LayerNorm arithmetic in order (the GEMV prologue spreads
// the same parts over waves: identical bits), bf16 output. Used for norm_f by the backbone plugin
// (zonos_vibes_amd/backbone.py); the decode step fuses its LayerNorms.
namespace {
template <int CPL>
__global__ __launch_bounds__(256) void layernorm_rows_kernel(const bf16_t* x, int ldx, int m, const bf16_t* w,
                                                             const bf16_t* b, float eps, bf16_t* out, int ldo) {
  constexpr int K = CPL * 512, NQ = ln_parts(K), CPQ = CPL / NQ;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= m) return;
  const bf16_t* xr = x + (size_t)r * ldx;
  uint4 xv[NQ][CPQ], gw[NQ][CPQ], gb[NQ][CPQ];
  float p[NQ];
  // the row, gamma and beta loads all in flight together (one memory round trip, not two)
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int i = 0; i < CPQ; ++i) {
      const int c = q * (K / NQ) / 8 + lane + 64 * i;
      xv[q][i] = *reinterpret_cast<const uint4*>(xr + q * (K / NQ) + (lane + 64 * i) * 8);
      gw[q][i] = reinterpret_cast<const uint4*>(w)[c];
      gb[q][i] = reinterpret_cast<const uint4*>(b)[c];
    }
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < CPQ; ++i) t += ln_chunk_sum(xv[q][i], 0.f, false);
    p[q] = wave_sum(t);
  }
  const float mean = ln_combine<NQ>(p) / (float)K;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < CPQ; ++i) t += ln_chunk_sum(xv[q][i], mean, true);
    p[q] = wave_sum(t);
  }
  const float rstd = 1.0f / sqrtf(ln_combine<NQ>(p) / (float)K + eps), nbias = -mean * rstd;
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int i = 0; i < CPQ; ++i) {
      const int c = q * (K / NQ) / 8 + lane + 64 * i;
      reinterpret_cast<uint4*>(out + (size_t)r * ldo)[c] = ln_apply(xv[q][i], gw[q][i], gb[q][i], rstd, nbias);
    }
}
}  // namespace

extern "C" int zmi_layernorm_rows(const void* x, int ldx, int m, int k, const void* w, const void* b, float eps,
                                  void* out, int ldo, void* stream) {
  if (ldx % 8 || ldo % 8) return zmi_fail_msg("layernorm_rows: ldx and ldo must be multiples of 8");
  if (m <= 0) return 0;
  const dim3 grid((m + 3) / 4);
  hipStream_t s = (hipStream_t)stream;
  switch (k) {
    case 512: hipLaunchKernelGGL(layernorm_rows_kernel<1>, grid, dim3(256), 0, s, (const bf16_t*)x, ldx, m,
                                 (const bf16_t*)w, (const bf16_t*)b, eps, (bf16_t*)out, ldo); break;
    case 1024: hipLaunchKernelGGL(layernorm_rows_kernel<2>, grid, dim3(256), 0, s, (const bf16_t*)x, ldx, m,
                                  (const bf16_t*)w, (const bf16_t*)b, eps, (bf16_t*)out, ldo); break;
    case 2048: hipLaunchKernelGGL(layernorm_rows_kernel<4>, grid, dim3(256), 0, s, (const bf16_t*)x, ldx, m,
                                  (const bf16_t*)w, (const bf16_t*)b, eps, (bf16_t*)out, ldo); break;
    case 4096: hipLaunchKernelGGL(layernorm_rows_kernel<8>, grid, dim3(256), 0, s, (const bf16_t*)x, ldx, m,
                                  (const bf16_t*)w, (const bf16_t*)b, eps, (bf16_t*)out, ldo); break;
    default: return zmi_fail_msg("layernorm_rows: k must be 512, 1024, 2048 or 4096");
  }
  ZMI_CHECK(hipGetLastError());
  return 0;
}
