// Weight-streaming skinny GEMM ("GEMV") for the decode step and the prefill, gfx950.
//
// out[m, n] = sum_k A[m, k] * W[n, k]   (nn.Linear, reference zonos/backbone/_torch.py:114-115,147-152,
//                                        heads: zonos/model.py:100-101)
//
// Design:
//  * W is re-laid out once at load time into MFMA-native 1 KiB tiles: tile (nt, kt) holds the
//    16 (n) x 32 (k) block in exactly the lane order of the B operand of
//    v_mfma_f32_16x16x32_bf16 (lane l: n = l&15, k = 8*(l>>4)..+7). A wave streams its tiles
//    with one fully coalesced, non-temporal 16 B/lane load per tile, straight into VGPRs.
//  * Activations (M <= 16*MT rows, zero-padded) form the A operand, loaded from L2.
//  * Every output element uses the same K-reduction tree regardless of M: per-wave MFMA chain
//    -> fixed 4-wave LDS sum -> fixed split-K slab sum. Results are therefore batch-invariant
//    (an utterance decodes identically alone or batched).
//  * Split-K partial slabs are combined in-launch by the last-arriving block (agent-scope
//    release/acquire, cdna_hip_programming.md §6 Guideline 16), which also runs the fused
//    epilogue: bf16 store, residual add, RoPE + KV-cache write, SwiGLU, or logits.
//  * Optional LayerNorm prologue (weight+bias, fp32 stats) fuses nn.LayerNorm into the GEMV;
//    weight loads are issued before the stats so HBM latency hides the reduction.
#include <cstdlib>
#include "zmi_common.h"
#include "zmi_kernels.h"
#include "zmi_gemv8_impl.h"

namespace zmi_gemv {
hipError_t launch_epi0(const ZmiGemvArgs& a, int mt, int nf, hipStream_t s);
hipError_t launch_epi1(const ZmiGemvArgs& a, int mt, int nf, hipStream_t s);
hipError_t launch_epi2(const ZmiGemvArgs& a, int mt, int nf, hipStream_t s);
hipError_t launch_epi3(const ZmiGemvArgs& a, int mt, int nf, hipStream_t s);
hipError_t launch_epi4(const ZmiGemvArgs& a, int mt, int nf, hipStream_t s);
hipError_t launch_epi5(const ZmiGemvArgs& a, int mt, int nf, hipStream_t s);
hipError_t launch8_epi0(const ZmiGemvArgs& a, hipStream_t s);
hipError_t launch8_epi1(const ZmiGemvArgs& a, hipStream_t s);
hipError_t launch8_epi2(const ZmiGemvArgs& a, hipStream_t s);
hipError_t launch8_epi3(const ZmiGemvArgs& a, hipStream_t s);
hipError_t launch8_epi4(const ZmiGemvArgs& a, hipStream_t s);
hipError_t launch8_epi5(const ZmiGemvArgs& a, hipStream_t s);
static hipError_t launch8_epi(const ZmiGemvArgs& a, int epi, hipStream_t s) {
  switch (epi) {
    case ZMI_EPI_STORE: return launch8_epi0(a, s);
    case ZMI_EPI_RESIDUAL: return launch8_epi1(a, s);
    case ZMI_EPI_QKV: return launch8_epi2(a, s);
    case ZMI_EPI_SWIGLU: return launch8_epi3(a, s);
    case ZMI_EPI_LOGITS: return launch8_epi4(a, s);
    case ZMI_EPI_F32: return launch8_epi5(a, s);
  }
  return hipErrorInvalidValue;
}
}

namespace {

// Pack a row-major [N_src][K] bf16 weight into the V8 layout (zmi_gemv8_impl.h): 1 KiB chunk
// (g, kc), lane l = column 8g + (l >> 3), k = 64 kc + 8 (l & 7) .. +7; zero rows beyond N_src.
// SwiGLU mode interleaves fc1's value and gate halves per group: rows 0..3 of group g are value
// rows 4g.., rows 4..7 their gates F + 4g.. (F = N_src / 2).
__global__ void pack_kernel(const bf16_t* __restrict__ src, uint4* __restrict__ dst, int n_src, int k, int n_pad,
                            int mode) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int kc_n = k >> 6;
  const size_t total = (size_t)(n_pad >> 3) * kc_n * 64;
  if (idx >= total) return;
  const int l = idx & 63;
  const size_t t = idx >> 6;
  const int kc = (int)(t % kc_n), g = (int)(t / kc_n);
  const int r = l >> 3, n = g * 8 + r, kk = kc * 64 + (l & 7) * 8;
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


// Choose (row tiles, fragments per wave, split-K) for an (M, N, K) problem. The K split
// depends only on (N, K), never on M, so results are identical for every batch size.
void zmi_gemv_plan(int M, int N, int K, int* mt, int* nf, int* ksplit, int* nchunk) {
  const int KT = K / 32;
  int m = M <= 16 ? 1 : (M <= 32 ? 2 : (M <= 64 ? 4 : 8));
  // Measured on MI355X (tools/bench_gemv.py, M = 2): split-K never pays at the decode shapes
  // (the extra hand-off and per-block activation staging cost more than the added parallelism),
  // so every block owns a full K column strip. Grids with >= 512 strips run 8 fragments per
  // chunk (lower VGPR use), smaller grids 16.
  const int nt = N / 16;
  const int ks = 1;
  const int per_wave = KT / 4;
  int f = (nt >= 512 ? 8 : 16);
  while (f > per_wave) f >>= 1;
  while (f > 2 && per_wave % f) f >>= 1;
  *mt = m;
  *nf = f;
  *ksplit = ks;
  *nchunk = per_wave / f;
}

extern "C" int zmi_gemv_launch(const ZmiGemvArgs* args, int epi, void* stream) {
  ZmiGemvArgs a = *args;
  int mt, nf, ks, nch;
  if (a.N % 16 || a.K % 128) return zmi_fail_msg("gemv: N must be a multiple of 16 and K of 128");
  if (a.M < 1) return zmi_fail_msg("gemv: M must be >= 1");
  static const bool mfma_only = getenv("ZMI_GEMV_MFMA") != nullptr;  // A/B switch for measurements
  if (!mfma_only && a.ksplit <= 1 && zmi_gemv8::use8(a.M, a.N, a.K, a.ln_w != nullptr)) {  // decode regime: 8-column VALU kernel
    a.nchunk = 1;
    if (epi < ZMI_EPI_STORE || epi > ZMI_EPI_F32) return zmi_fail_msg("gemv: unknown epilogue");
    ZMI_CHECK(zmi_gemv::launch8_epi(a, epi, (hipStream_t)stream));
    return 0;
  }
  zmi_gemv_plan(a.M, a.N, a.K, &mt, &nf, &ks, &nch);
  if (a.ksplit <= 0) {
    a.ksplit = ks;
    a.nchunk = nch;
  } else {
    const int per_wave = (a.K / 32) / (a.ksplit * 4);
    if (per_wave * a.ksplit * 4 != a.K / 32) return zmi_fail_msg("gemv: K/32 not divisible by 4*ksplit");
    if (a.nchunk > 0) {  // caller-chosen chunking (tuning): NF = per_wave / nchunk
      if (per_wave % a.nchunk) return zmi_fail_msg("gemv: nchunk must divide the fragments per wave");
      nf = per_wave / a.nchunk;
      if (nf != 2 && nf != 4 && nf != 8 && nf != 16) return zmi_fail_msg("gemv: fragments per chunk not in {2,4,8,16}");
    } else {
      nf = per_wave >= 16 ? 16 : (per_wave >= 8 ? 8 : (per_wave >= 4 ? 4 : 2));
      while (per_wave % nf) nf >>= 1;
      a.nchunk = per_wave / nf;
    }
  }
  if (nf < 2) return zmi_fail_msg("gemv: fewer than 2 fragments per wave");
  if (a.ksplit > 1) {
    const int groups = (a.M + mt * 16 - 1) / (mt * 16);
    const int64_t tiles = (int64_t)groups * (a.N / 16);
    if (!a.slab || !a.counters) return zmi_fail_msg("gemv: split-K needs slab + counters");
    if (tiles * a.ksplit * mt * 256 > a.slab_cap) return zmi_fail_msg("gemv: split-K slab too small");
    if (tiles > a.counters_cap) return zmi_fail_msg("gemv: split-K counters too small");
  }
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  switch (epi) {
    case ZMI_EPI_STORE: e = zmi_gemv::launch_epi0(a, mt, nf, s); break;
    case ZMI_EPI_RESIDUAL: e = zmi_gemv::launch_epi1(a, mt, nf, s); break;
    case ZMI_EPI_QKV: e = zmi_gemv::launch_epi2(a, mt, nf, s); break;
    case ZMI_EPI_SWIGLU: e = zmi_gemv::launch_epi3(a, mt, nf, s); break;
    case ZMI_EPI_LOGITS: e = zmi_gemv::launch_epi4(a, mt, nf, s); break;
    case ZMI_EPI_F32: e = zmi_gemv::launch_epi5(a, mt, nf, s); break;
    default: return zmi_fail_msg("gemv: unknown epilogue");
  }
  ZMI_CHECK(e);
  return 0;
}

extern "C" int zmi_pack_weight(const void* src, void* dst, int n_src, int k, int n_pad, int mode, void* stream) {
  if (n_pad % 16 || k % 64 || n_pad < (mode == ZMI_PACK_SWIGLU ? n_src : 0) ||
      (mode == ZMI_PACK_SWIGLU && (n_src % 8 || n_pad != n_src)))
    return zmi_fail_msg("pack: bad shape");
  const size_t total = (size_t)(n_pad / 8) * (k / 64) * 64;
  hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)src, (uint4*)dst, n_src, k, n_pad, mode);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int64_t zmi_gemv_slab_floats(int M, int N, int K, int ksplit) {
  int mt, nf, ks, nch;
  zmi_gemv_plan(M, N, K, &mt, &nf, &ks, &nch);
  if (ksplit > 0) ks = ksplit;
  const int groups = (M + mt * 16 - 1) / (mt * 16);
  return ks > 1 ? (int64_t)groups * (N / 16) * ks * mt * 256 : 0;
}
