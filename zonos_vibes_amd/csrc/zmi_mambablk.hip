// Fused hybrid decode block: the Mamba2 in_proj GEMV (ADDLN prologue) and the Mamba2 step in ONE launch,
// mamba-ssm 2.2.4 Block.forward -> Mamba2.step up to the gated norm (reference zonos/backbone/_mamba_ssm.py:9-57;
// mamba-ssm is absent here: parity unpinned, oracle/hybrid_cpu.py).
//
// Why: as two launches the step (6.5 us per layer at C4) paid a kernel boundary plus a chain of loads (its
// state slice, conv-ring values, the in_proj output) after the in_proj's weight stream. Here the step
// workgroups are extra workgroups of the in_proj grid, as in the transformer's zmi_attn_block:
//   [0, n_in)          gemv_body in_proj role (G = 2, the K = 2048 shape): the bf16 zxbcdt row as before,
//                      and every column pair of an active row as an 8-byte {pair, tag = position + 1}
//                      granule (one sc1 store, data and flag at once);
//   [n_in, + M nheads) step role, one workgroup per (row, head): the SSM state slice, conv-ring values,
//                      conv weights and bias are loaded at launch start, under the in_proj's weight stream;
//                      wave 0 polls the head's 193 granules (its 64 x, the 256 B / C, its 64 z, its dt) with
//                      one lane per granule group and a bounded spin; then zmi_mamba2_step's arithmetic.
// Dispatch runs in block order, so a waiting step workgroup never holds a slot an in_proj workgroup still
// needs; the tag changes every step and a row's granules are zeroed when it starts an utterance, so
// nothing is re-armed. Outputs are bit-identical to zmi_gemv_launch(ADDLN) + zmi_mamba2_step (tested).
#include <algorithm>

#include "zmi_common.h"
#include "zmi_kernels.h"
#include "zmi_gemv_impl.h"
#include "zmi_mamba_step.h"
#include "zmi_prefetch.h"

namespace {

using namespace zmi_mamba;
#ifndef ZMI_MB_IG
#define ZMI_MB_IG 2
#endif
constexpr int IG = ZMI_MB_IG, IW = 4, INL = 8, IRT = 16;  // in_proj role: the K = 2048 shape, IG groups
constexpr int NT = IG * IW * 64;
static_assert(NT == MB_ST, "the fused step role runs zmi_mamba2_step's thread layout (the same readout order)");
constexpr int NGRAN = MB_HD / 2 + MB_DS + MB_HD / 2 + 1;  // x pairs, B / C pairs, z pairs, the dt pair
constexpr unsigned SPIN = 1u << 20;

// Diagnostic build only (-DZMI_GEMV_STAMPS, tools/hybrid_stamps.py): the step role stamps into the in_proj
// args' diag area like the GEMV role (slot 0 start, 2 granules received, 3 raw values in LDS, 6 end).
#ifdef ZMI_GEMV_STAMPS
#define ZMI_MSTAMP(i)                                                                                     \
  do {                                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                                    \
    if (threadIdx.x == 0 && ia.diag)                                                                      \
      reinterpret_cast<unsigned long long*>(ia.diag)[((size_t)ia.reserved * 4096 + blockIdx.x) * 8 + (i)] = \
          __builtin_amdgcn_s_memrealtime();                                                               \
    __builtin_amdgcn_sched_barrier(0);                                                                    \
  } while (0)
#else
#define ZMI_MSTAMP(i) \
  do {                \
  } while (0)
#endif

__global__ __launch_bounds__(NT) void mamba_block_kernel(const ZmiGemvArgs ia, int n_cb, int n_in,
                                                         const ZmiMamba2Args ma, uint64_t* gran, int gstride,
                                                         unsigned* err, const ZmiPrefetch pf, int n_pf, int xc_l2) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  if (b < n_in) {
    zmi_gemv::QkvFuse fz{gran, gstride};
    int cb = b;
    if (xc_l2) {
      // XCD-local column blocks (blocks 8 apart share an XCD, as the step workgroup of head h does: XCD h mod 8): the
      // first 3 x 8 blocks take the B / C / dt column blocks (every head needs them: written through, and dispatched
      // first so they land early); then block 8 (3 + 8 i + k) + x takes z (k < 4) or x (k >= 4) column block k mod 4
      // of head x + 8 i, whose granules stay in that XCD's L2 for the head's step workgroup
      const int x = b & 7, j = b >> 3;
      if (j < 3) {
        cb = 2 * ma.d_ssm / (8 * IG) + 8 * j + x;
      } else {
        const int i = (j - 3) >> 3, k = (j - 3) & 7, h = x + 8 * i;
        cb = (k < 4 ? 0 : ma.d_ssm / (8 * IG)) + (MB_HD / (8 * IG)) * h + (k & 3);
      }
      fz.l2_cols = 2 * ma.d_ssm;
    }
    zmi_gemv::gemv_body<IG, IW, INL, IRT, zmi_gemv::PRO_ADDLN, ZMI_EPI_STORE, 1, 2>(ia, n_cb, 1, cb, smem, fz);
    return;
  }
  const int n_step = ma.M * ma.nheads;
  if (b >= n_in + n_step) {  // prefetch role: the out_proj weights, under the step's latency chain
    prefetch_body<NT>(pf, b - n_in - n_step, n_pf);
    return;
  }
  const int b2 = b - n_in;
  const int m = b2 / ma.nheads, h = b2 - m * ma.nheads;
  ZMI_MSTAMP(0);
  const int pos = ma.row_pos[m];
  if (pos < 0) return;  // inactive row: block-uniform, before any barrier
  const int kv = ma.row_kv ? ma.row_kv[m] : m;
  bf16_t* raw = reinterpret_cast<bf16_t*>(smem);
  float* xs = reinterpret_cast<float*>(smem + 1024);
  float* bc = xs + MB_HD;
  StepPre<NT> pre;
  step_prefetch<NT>(ma, h, pos, kv, pre);

  if (threadIdx.x < 64) {  // wave 0: the head's granules, lane l holds groups l, l + 64, l + 128, l + 192
    const int lane = threadIdx.x, d = ma.d_ssm;
    const uint32_t tag = (uint32_t)pos + 1u;
    const uint64_t* g = gran + (size_t)m * gstride;
    auto pair_of = [&](int k) {  // granule group k -> pair index in the zxbcdt row
      if (k < MB_HD / 2) return (d + MB_HD * h) / 2 + k;                     // x of head h
      if (k < MB_HD / 2 + MB_DS) return d + (k - MB_HD / 2);                  // B, C (columns 2 d ..)
      if (k < NGRAN - 1) return MB_HD / 2 * h + (k - MB_HD / 2 - MB_DS);      // z of head h
      return (2 * d + 2 * MB_DS + h) >> 1;                                     // the pair holding dt
    };
    uint64_t v[4];
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = lane + 64 * i;
        v[i] = k < NGRAN ? ld_wt64(g + pair_of(k)) : ((uint64_t)tag << 32);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) ok = ok && (uint32_t)(v[i] >> 32) == tag;
      if (__all(ok)) break;
      if (spins > SPIN) {
        if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    ZMI_MSTAMP(2);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = lane + 64 * i;
      const bf16_t lo = (bf16_t)(v[i] & 0xffffu), hi = (bf16_t)((v[i] >> 16) & 0xffffu);
      if (k < MB_HD / 2) {
        raw[RAW_X + 2 * k] = lo;
        raw[RAW_X + 2 * k + 1] = hi;
      } else if (k < MB_HD / 2 + MB_DS) {
        raw[RAW_BC + 2 * (k - MB_HD / 2)] = lo;
        raw[RAW_BC + 2 * (k - MB_HD / 2) + 1] = hi;
      } else if (k < NGRAN - 1) {
        raw[RAW_Z + 2 * (k - MB_HD / 2 - MB_DS)] = lo;
        raw[RAW_Z + 2 * (k - MB_HD / 2 - MB_DS) + 1] = hi;
      } else if (k == NGRAN - 1) {
        raw[RAW_DT] = ((2 * d + 2 * MB_DS + h) & 1) ? hi : lo;
      }
    }
  }
  __syncthreads();
  ZMI_MSTAMP(3);
  step_core<NT>(ma, m, h, pos, kv, raw, pre, xs, bc);
  ZMI_MSTAMP(6);
}

}  // namespace

extern "C" int64_t zmi_mamba_block_gran_words(int rows, int d_in_proj) {
  return (rows <= 0 || d_in_proj <= 0 || d_in_proj % 2) ? -1 : (int64_t)rows * (d_in_proj / 2);
}

extern "C" int zmi_mamba_block_pf(const ZmiGemvArgs* in_proj, const ZmiMamba2Args* step, void* gran, unsigned* err,
                                  const ZmiPrefetch* prefetch, void* stream) {
  const ZmiGemvArgs& a = *in_proj;
  const ZmiMamba2Args& s = *step;
  if (a.K != 2048 || a.pro != ZMI_PRO_ADDLN || !a.ln_w || !a.ln_b || !a.aux || a.ld_aux % 8 || a.res_out == a.aux)
    return zmi_fail_msg("mamba_block: in_proj must be the ADDLN GEMV with K = 2048");
  if (a.M < 1 || a.M > IRT || s.M != a.M) return zmi_fail_msg("mamba_block: 1 <= M <= 16 rows, the same in both");
  if (s.headdim != MB_HD || s.d_state != MB_DS || s.d_conv != MB_DC || s.ngroups != 1 || s.nheads <= 0 ||
      s.d_ssm != s.nheads * MB_HD)
    return zmi_fail_msg("mamba_block: Mamba2 geometry headdim 64, d_state 128, d_conv 4, ngroups 1");
  const int d_in = 2 * s.d_ssm + 2 * MB_DS + s.nheads;
  if (a.N != d_in || a.n_valid != a.N || a.N % (8 * IG) || a.out != s.zxbcdt || a.ldo != s.ld_zx || !a.row_pos ||
      a.row_pos != s.row_pos || s.row_kv)
    return zmi_fail_msg("mamba_block: the step reads in_proj's output rows (N = d_in_proj, same rows and row_pos, "
                        "row_kv NULL)");
  if (!gran || !err || !s.conv_w || !s.conv_b || !s.dt_bias || !s.A || !s.D || !s.conv_ring || !s.ssm || !s.y)
    return zmi_fail_msg("mamba_block: missing buffers");
  const int n_cb = a.N / 8 / IG;
  const int n_in = (n_cb + 7) / 8 * 8;
  // XCD-local x / z hand-offs (ZMI_OPT_XC_HANDOFF 0): the in_proj blocks' column-block map covers exactly the
  // Mamba2 geometry of every hybrid config this library takes (64 heads x 64 dims: 3 x 8 blocks of B / C / dt, then
  // 8 x 8 x 8 of z / x)
  const int xc_l2 = zmi_option(ZMI_OPT_XC_HANDOFF) == 0 && IG == 2 && s.nheads == 64 && n_in == 8 * (3 + 64) &&
                    (2 * s.d_ssm + 2 * MB_DS + s.nheads) / 16 - 2 * s.d_ssm / 16 <= 24 ? 1 : 0;
  const size_t lds = std::max(zmi_gemv::Img<2048>::bytes(a.M, IG * IW, IRT, zmi_gemv::PRO_ADDLN), (size_t)2560);
  if (lds > zmi_gemv::LDS_MAX) return zmi_fail_msg("mamba_block: LDS image too large");
  if (lds > 64 * 1024) {
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&mamba_block_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)zmi_gemv::LDS_MAX);
    if (attr != hipSuccess) return zmi_fail(attr, "hipFuncSetAttribute", __FILE__, __LINE__);
  }
  ZmiPrefetch pf{};
  if (prefetch) {
    pf = *prefetch;
    if (zmi_prefetch_invalid(pf)) return zmi_fail_msg("mamba_block: bad prefetch ranges");
  }
  const int n_pf = (pf.bytes[0] > 0 || pf.bytes[1] > 0) ? pf.blocks : 0;
  hipLaunchKernelGGL(mamba_block_kernel, dim3((unsigned)(n_in + a.M * s.nheads + n_pf)), dim3(NT), lds,
                     (hipStream_t)stream, a, n_cb, n_in, s, (uint64_t*)gran, a.N / 2, err, pf, n_pf, xc_l2);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_mamba_block(const ZmiGemvArgs* in_proj, const ZmiMamba2Args* step, void* gran, unsigned* err,
                               void* stream) {
  return zmi_mamba_block_pf(in_proj, step, gran, err, nullptr, stream);
}
