// Weight-streaming GEMV / skinny GEMM entry points (kernel: zmi_gemv_impl.h) and the weight packer.
//
// out[m, n] = sum_k A[m, k] * W[n, k]   (nn.Linear, reference zonos/backbone/_torch.py:114-115,147-152,
//                                        heads: zonos/model.py:100-101)
#include "zmi_common.h"
#include "zmi_kernels.h"
#include "zmi_gemv_impl.h"

namespace zmi_gemv {
hipError_t launch_epi0(const ZmiGemvArgs& a, hipStream_t s);
hipError_t launch_epi1(const ZmiGemvArgs& a, hipStream_t s);
hipError_t launch_epi2(const ZmiGemvArgs& a, hipStream_t s);
hipError_t launch_epi3(const ZmiGemvArgs& a, hipStream_t s);
hipError_t launch_epi4(const ZmiGemvArgs& a, hipStream_t s);
hipError_t launch_epi5(const ZmiGemvArgs& a, hipStream_t s);
}  // namespace zmi_gemv

namespace {

// Pack a row-major [N_src][K] bf16 weight into the M8 layout (zmi_gemv_impl.h): 1 KiB chunk (g, kc),
// lane l = column 8g + (l & 7), k = 64 kc + 32 ((l >> 3) & 1) + 8 (l >> 4) .. +7; zero rows beyond
// N_src. SwiGLU mode interleaves fc1's value and gate halves per group: rows 0..3 of group g are
// value rows 4g.., rows 4..7 their gates F + 4g.. (F = N_src / 2).
__global__ void pack_kernel(const bf16_t* __restrict__ src, uint4* __restrict__ dst, int n_src, int k, int n_pad,
                            int mode) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int kc_n = k >> 6;
  const size_t total = (size_t)(n_pad >> 3) * kc_n * 64;
  if (idx >= total) return;
  const int l = idx & 63;
  const size_t t = idx >> 6;
  const int kc = (int)(t % kc_n), g = (int)(t / kc_n);
  const int r = l & 7, n = g * 8 + r, kk = kc * 64 + 32 * ((l >> 3) & 1) + 8 * (l >> 4);
  int srow = n;
  if (mode == ZMI_PACK_SWIGLU) {
    const int f = n_src >> 1;
    srow = r < 4 ? g * 4 + r : f + g * 4 + (r - 4);
  }
  uint4 v = {0u, 0u, 0u, 0u};
  if (srow < n_src) v = *reinterpret_cast<const uint4*>(src + (size_t)srow * k + kk);
  dst[idx] = v;
}

}  // namespace

extern "C" int zmi_gemv_launch(const ZmiGemvArgs* args, int epi, void* stream) {
  const ZmiGemvArgs& a = *args;
  zmi_gemv::Shape sh;
  if (a.N % 8) return zmi_fail_msg("gemv: N must be a multiple of 8");
  if (!zmi_gemv::shape_for(a.K, a.ln_w != nullptr, &sh))
    return zmi_fail_msg("gemv: K must be 512, 1024, 2048, 4096 or 8192");
  if (a.M < 1) return zmi_fail_msg("gemv: M must be >= 1");
  if (a.ldx % 8) return zmi_fail_msg("gemv: ldx must be a multiple of 8 (16-byte rows)");
  if (a.groups < 0 || a.groups > 2 || (a.groups == 2 && a.K != 2048 && a.K != 8192))
    return zmi_fail_msg("gemv: groups must be 0 (library choice), 1, or 2 for K = 2048 / 8192");
  if (a.pro != ZMI_PRO_AUTO && a.pro != ZMI_PRO_ADDLN && a.pro != ZMI_PRO_GRMS && a.pro != ZMI_PRO_GRMS_G)
    return zmi_fail_msg("gemv: unknown prologue");
  if (a.pro == ZMI_PRO_ADDLN && (!a.ln_w || !a.ln_b || !a.aux || a.ld_aux % 8 || a.res_out == a.aux))
    return zmi_fail_msg("gemv: ADDLN needs ln_w, ln_b, aux (ld_aux % 8 == 0) and res_out != aux");
  if ((a.pro == ZMI_PRO_GRMS || a.pro == ZMI_PRO_GRMS_G) && (!a.ln_w || !a.aux || a.ld_aux % 8 || a.M > 4))
    return zmi_fail_msg("gemv: GRMS needs ln_w (the norm weight), aux = the f32 gate or g rows (ld_aux % 8 == 0), M <= 4");
  if (epi == ZMI_EPI_QKV && (a.hd % 8 || a.smax <= 0 || !a.row_pos || !a.row_kv || !a.rope))
    return zmi_fail_msg("gemv: the QKV epilogue needs row_pos, row_kv, rope, smax and hd % 8 == 0");
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  switch (epi) {
    case ZMI_EPI_STORE: e = zmi_gemv::launch_epi0(a, s); break;
    case ZMI_EPI_RESIDUAL: e = zmi_gemv::launch_epi1(a, s); break;
    case ZMI_EPI_QKV: e = zmi_gemv::launch_epi2(a, s); break;
    case ZMI_EPI_SWIGLU: e = zmi_gemv::launch_epi3(a, s); break;
    case ZMI_EPI_LOGITS: e = zmi_gemv::launch_epi4(a, s); break;
    case ZMI_EPI_F32: e = zmi_gemv::launch_epi5(a, s); break;
    default: return zmi_fail_msg("gemv: unknown epilogue");
  }
  if (e == hipErrorInvalidValue && a.pro != ZMI_PRO_AUTO)
    return zmi_fail_msg("gemv: prologue not built for this K / epilogue / row count (ADDLN: K 512 or 2048; GRMS: K "
                        "1024 or 4096, ZMI_EPI_STORE, rows within the LDS image)");
  ZMI_CHECK(e);
  return 0;
}

extern "C" int zmi_pack_weight(const void* src, void* dst, int n_src, int k, int n_pad, int mode, void* stream) {
  if (n_pad % 8 || k % 64 || n_pad < n_src || (mode == ZMI_PACK_SWIGLU && (n_src % 8 || n_pad != n_src)))
    return zmi_fail_msg("pack: bad shape");
  const size_t total = (size_t)(n_pad / 8) * (k / 64) * 64;
  hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)src, (uint4*)dst, n_src, k, n_pad, mode);
  ZMI_CHECK(hipGetLastError());
  return 0;
}
