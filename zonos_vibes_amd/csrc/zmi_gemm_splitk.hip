// Many-row fc2 and out_proj (reference zonos/backbone/_torch.py:152 and :140, x = x + ... at :100-101) as
// split-K GEMMs: one workgroup per (64-column block, K segment of the GEMV's wave split: fc2 8 x 1024, out_proj
// 4 x 512), then a reduce launch that sums the segments in order and applies the residual epilogue (optionally
// also the next op's LayerNorm).
//
// Why: the GEMV form (zmi_gemv_impl.h, W = 8 waves each owning one K segment of a column group) re-reads the
// whole activation block [M][8192] once per column group; at 128 rows (C3's 64 slots) that is 2 MB per
// workgroup, 256 MB of L2 -> LDS traffic per launch, and the launch took 37 us for 33.6 MB of weights. Here
// a workgroup reads only its K segment of the rows (256 KB at 128 rows; 64 MB per launch), its 64 columns'
// weights for that segment once (128 KB, in registers), and keeps the GEMV's arithmetic: per wave (one 8-column
// group) and row tile of 16 rows, the MFMA chain over the segment's 16 chunks of 64 (k-half 0 and k-half 1 in
// two accumulators, summed with the same DPP move), stored as that segment's fp32 sum; the reduce adds the
// segments in K order (the GEMV's wave order) and applies x = bf16(x + bf16(sum)). A row's result is
// bit-identical to zmi_gemv_launch's for any M (tested).
#include <algorithm>

#include "zmi_common.h"
#include "zmi_kernels.h"
#include "zmi_gemv_impl.h"

namespace {

using zmi_gemv::dma_piece;
using zmi_gemv::ror8;

// K segments are the GEMV's wave segments: K = 8192 (fc2) W = 8 x 16 chunks, K = 4096 (the hybrid's Mamba2
// out_proj over d_ssm) W = 4 x 16, K = 2048 (out_proj) W = 4 x 8 (zmi_gemv_impl.h shape_for)
template <int K>
struct Shape {
  static constexpr int NSEG = K == 8192 ? 8 : 4, KS = K / NSEG, NL = KS / 64, KC = K / 64;
  static constexpr int SROW = KS + 8;  // LDS row stride (bf16): bank-spread A reads
  static constexpr int TILE_BYTES = 16 * SROW * 2;
  static constexpr int RTS = KS >= 1024 ? 2 : 4;  // 16-row tiles per stage: two stages fill ~132 KB of LDS
};
constexpr int NWV = 8, NT = NWV * 64;  // wave g = column group cb * 8 + g
constexpr int RT = 16;                 // rows per tile (one MFMA tile)
// DN (dense pairs, zmi_gemv_impl.h gemm_rows_kernel): 4 waves, wave p = the column-group pair cb * 8 + 2p, +1 with a
// 16-column B operand per k-half gathered from the two groups' M8 chunks: half the MFMAs and A-fragment reads of
// the 8-wave form, the same bits
constexpr int DNWV = 4, DNT = DNWV * 64;

// Grid: (row group, K segment, column block), column blocks fastest. A row group is `rpg` consecutive 16-row tiles
// (several row groups re-read the segment's weights, from L2 when they run together; speed only: a row's sums
// do not depend on the grouping).
template <int K, bool DN, int RTS>
__global__ __launch_bounds__(DN ? DNT : NT) void splitk_kernel(const ZmiGemvArgs a, float* part, int n_cb, int rpg) {
  using S = Shape<K>;
  constexpr int NSEG = S::NSEG, KS = S::KS, NL = S::NL, KC = S::KC, SROW = S::SROW, TILE_BYTES = S::TILE_BYTES;
  constexpr int NW = DN ? DNWV : NWV;  // waves
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x % (n_cb * NSEG), rg = blockIdx.x / (n_cb * NSEG);
  const int seg = b / n_cb, cb = b - seg * n_cb;  // consecutive blocks: one segment, neighbouring columns
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  // the wave's group (DN: the group of lane l's column, 2 wave + ((l >> 3) & 1), of the wave's pair)
  const int g = DN ? cb * NWV + 2 * wave + ((lane >> 3) & 1) : cb * NWV + wave;
  const int M = a.M, N = a.N;
  const int rt0 = rg * rpg, n_rt = min((M + RT - 1) / RT, rt0 + rpg);
  if (rt0 >= n_rt) return;
  // a stage = RTS 16-row tiles (two stage buffers): the next stage's rows are in flight while this one's tiles run
  const int n_st = (n_rt - rt0 + RTS - 1) / RTS;
  bf16_t* tiles = reinterpret_cast<bf16_t*>(smem);
  const bf16_t* X = reinterpret_cast<const bf16_t*>(a.X) + (size_t)seg * KS;

  auto stage = [&](int st, int buf) {  // the stage's rows of this segment, 1 KiB pieces spread over the waves
    const int row0 = (rt0 + st * RTS) * RT, rows = min(min(RTS * RT, M - row0), (n_rt - rt0 - st * RTS) * RT);
    bf16_t* dst = tiles + (size_t)buf * RTS * (TILE_BYTES / 2);
    for (int pc = wave; pc < rows * (KS / 512); pc += NW) {
      const int r = pc / (KS / 512), p = pc - r * (KS / 512);
      dma_piece(X + (size_t)(row0 + r) * a.ldx + p * 512 + lane * 8, dst + r * SROW + p * 512);
    }
  };
  stage(0, 0);
  // the wave's weights for this segment: group g, chunks seg * NL .. + NL - 1 (layout M8), all in flight
  // (DN: k-half h of lane l's column = M8 lane (l & 7) + 8 h + 16 (l >> 4) of group g's chunk)
  constexpr int NH = DN ? 2 : 1;
  u32x4_t wf[NH][NL];
  if constexpr (DN) {
    const char* wbase = reinterpret_cast<const char*>(a.W) + ((size_t)cb * NWV * KC + seg * NL) * 1024;
    const __amdgpu_buffer_rsrc_t wrsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wbase), (short)0, NWV * KC * 1024, 0x00020000);
    const int vo = (g - cb * NWV) * KC * 1024 + ((lane & 7) + 16 * (lane >> 4)) * 16;
#pragma unroll
    for (int j = 0; j < NL; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) wf[h][j] = __builtin_amdgcn_raw_buffer_load_b128(wrsrc, vo + 128 * h, j * 1024, 2);
  } else {
    const char* wbase = reinterpret_cast<const char*>(a.W) + ((size_t)g * KC + seg * NL) * 1024;
    const __amdgpu_buffer_rsrc_t wrsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wbase), (short)0, NL * 1024, 0x00020000);
#pragma unroll
    for (int j = 0; j < NL; ++j) wf[0][j] = __builtin_amdgcn_raw_buffer_load_b128(wrsrc, lane * 16, j * 1024, 2);
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NH * NL) : "memory");  // the first stage's pieces (issued before)
  for (int st = 0; st < n_st; ++st) {
    __syncthreads();  // stage st landed for every wave's pieces; the other buffer is free
    if (st + 1 < n_st) stage(st + 1, (st + 1) & 1);
#pragma unroll
    for (int u = 0; u < RTS; ++u) {
      const int rt = rt0 + st * RTS + u;
      if (rt >= n_rt) break;
      const int row0 = rt * RT, rows = min(RT, M - row0);
      const bf16_t* xs = tiles + ((size_t)(st & 1) * RTS + u) * (TILE_BYTES / 2);
      f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      const int ar = min(lane & 15, rows - 1);
      const bf16_t* xa = xs + ar * SROW + (lane >> 4) * 8;
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        const uint4 x0 = *reinterpret_cast<const uint4*>(xa + j * 64);
        const uint4 x1 = *reinterpret_cast<const uint4*>(xa + j * 64 + 32);
        const bf16x8_t w0 = __builtin_bit_cast(bf16x8_t, wf[0][j]), w1 = __builtin_bit_cast(bf16x8_t, wf[NH - 1][j]);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x0), w0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x1), w1, acc1, 0, 0, 0);
      }
      // segment sum = k-half 0 (tile columns 0..7) + k-half 1 (columns 8..15 moved down): element q of lane l
      // is row 4 (l >> 4) + q, column l & 15 (DN: both halves in place, column l & 15 of the pair)
      const int c = lane & 15, rb = (lane >> 4) * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float v = DN ? acc0[q] + acc1[q] : acc0[q] + ror8(acc1[q]);
        if ((DN || c < 8) && rb + q < rows) part[((size_t)seg * M + row0 + rb + q) * N + g * 8 + (c & 7)] = v;
      }
    }
    if (st + 1 < n_st) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next stage's pieces
  }
}

// x[m][n] = bf16(x + bf16(sum over the segments in order)), the GEMV's EPI_RESIDUAL epilogue; RES false: out = bf16(sum),
// its EPI_STORE epilogue
template <int NSEG, bool RES>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* part, int M, int N, bf16_t* out, int ldo) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)M * N) return;
  const size_t m = i / N, n = i - m * N;
  float v = part[i];
#pragma unroll
  for (int s = 1; s < NSEG; ++s) v += part[(size_t)s * M * N + i];
  bf16_t* o = out + m * ldo + n;
  if (RES)
    *o = (bf16_t)f2bf(bf2f(*o) + bfround(v));
  else
    *o = (bf16_t)f2bf(v);
}

// The same reduce + residual for rows of 2048 columns, then the LayerNorm of each new row into `xn` (the next
// op's prologue, zmi_layernorm_rows' arithmetic: part q = wave q, lane L's chunk at q 512 + 8 L, parts combined
// (p0 + p1) + (p2 + p3), two passes): one 4-wave workgroup per row, so the next layer's LayerNorm pre-pass launch
// is not needed.
template <int NSEG>
__global__ __launch_bounds__(256) void splitk_reduce_ln_kernel(const float* part, int M, bf16_t* out, int ldo,
                                                               const bf16_t* lw, const bf16_t* lb, float eps,
                                                               bf16_t* xn, int ldn) {
  constexpr int N = 2048, NQ = ln_parts(N);
  static_assert(NQ == 4, "one wave per LayerNorm part");
  __shared__ float ps[2][NQ];
  const int m = blockIdx.x, t = threadIdx.x, lane = t & 63, q = t >> 6;
  const int e0 = q * 512 + lane * 8;
  bf16_t* orow = out + (size_t)m * ldo;
  const uint4 xv = *reinterpret_cast<const uint4*>(orow + e0);
  const uint4 gw = *reinterpret_cast<const uint4*>(lw + e0), gb = *reinterpret_cast<const uint4*>(lb + e0);
  float4 pv[NSEG][2];
#pragma unroll
  for (int s = 0; s < NSEG; ++s) {
    const float* pr = part + ((size_t)s * M + m) * N + e0;
    pv[s][0] = *reinterpret_cast<const float4*>(pr);
    pv[s][1] = *reinterpret_cast<const float4*>(pr + 4);
  }
  const uint32_t xu[4] = {xv.x, xv.y, xv.z, xv.w};
  uint32_t nu[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float v0 = j < 2 ? (j == 0 ? pv[0][0].x : pv[0][0].z) : (j == 2 ? pv[0][1].x : pv[0][1].z);
    float v1 = j < 2 ? (j == 0 ? pv[0][0].y : pv[0][0].w) : (j == 2 ? pv[0][1].y : pv[0][1].w);
#pragma unroll
    for (int s = 1; s < NSEG; ++s) {
      v0 += j < 2 ? (j == 0 ? pv[s][0].x : pv[s][0].z) : (j == 2 ? pv[s][1].x : pv[s][1].z);
      v1 += j < 2 ? (j == 0 ? pv[s][0].y : pv[s][0].w) : (j == 2 ? pv[s][1].y : pv[s][1].w);
    }
    nu[j] = f2bf(bf2f(xu[j]) + bfround(v0)) | (f2bf(bf2f(xu[j] >> 16) + bfround(v1)) << 16);
  }
  const uint4 nx = uint4{nu[0], nu[1], nu[2], nu[3]};
  *reinterpret_cast<uint4*>(orow + e0) = nx;
  const float s1 = wave_sum(ln_chunk_sum(nx, 0.f, false));
  if (lane == 0) ps[0][q] = s1;
  __syncthreads();
  const float mean = ln_combine<NQ>(ps[0]) / (float)N;
  const float s2 = wave_sum(ln_chunk_sum(nx, mean, true));
  if (lane == 0) ps[1][q] = s2;
  __syncthreads();
  const float rstd = 1.0f / sqrtf(ln_combine<NQ>(ps[1]) / (float)N + eps), nbias = -mean * rstd;
  *reinterpret_cast<uint4*>(xn + (size_t)m * ldn + e0) = ln_apply(nx, gw, gb, rstd, nbias);
}

}  // namespace

extern "C" int64_t zmi_gemv_splitk_floats(int M, int N) { return M <= 0 || N <= 0 ? -1 : (int64_t)8 * M * N; }

namespace {
template <int K>
int launch_splitk(const ZmiGemvArgs& a, int epi, float* part, const void* ln_w, const void* ln_b, float eps, void* xn,
                  int ldxn, hipStream_t s) {
  using S = Shape<K>;
  const int n_cb = a.N / (8 * NWV);
  // row groups: about ZMI_OPT_SPLITK_WGS workgroups in all (0: one row group)
  const int n_rt = (a.M + RT - 1) / RT, target = zmi_option(ZMI_OPT_SPLITK_WGS);
  const int n_rg = std::max(1, std::min(n_rt, target / (n_cb * S::NSEG)));
  const int rpg = (n_rt + n_rg - 1) / n_rg;
  const bool multi = zmi_option(ZMI_OPT_SPLITK_STAGE) != 0;
  const size_t lds = 2 * (size_t)(multi ? S::RTS : 1) * S::TILE_BYTES;
  // once per instantiation: allow the stage buffers' dynamic LDS
  static const hipError_t attr[4] = {
      hipFuncSetAttribute(reinterpret_cast<const void*>(&splitk_kernel<K, false, 1>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, 2 * S::TILE_BYTES),
      hipFuncSetAttribute(reinterpret_cast<const void*>(&splitk_kernel<K, true, 1>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, 2 * S::TILE_BYTES),
      hipFuncSetAttribute(reinterpret_cast<const void*>(&splitk_kernel<K, false, S::RTS>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, 2 * S::RTS * S::TILE_BYTES),
      hipFuncSetAttribute(reinterpret_cast<const void*>(&splitk_kernel<K, true, S::RTS>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, 2 * S::RTS * S::TILE_BYTES)};
  for (hipError_t e : attr) ZMI_CHECK(e);
  const dim3 grid(n_cb * S::NSEG * ((n_rt + rpg - 1) / rpg));
  const bool dn = zmi_option(ZMI_OPT_GEMM_ROWS) & 2;
  if (dn && multi)
    hipLaunchKernelGGL((splitk_kernel<K, true, S::RTS>), grid, dim3(DNT), lds, s, a, part, n_cb, rpg);
  else if (dn)
    hipLaunchKernelGGL((splitk_kernel<K, true, 1>), grid, dim3(DNT), lds, s, a, part, n_cb, rpg);
  else if (multi)
    hipLaunchKernelGGL((splitk_kernel<K, false, S::RTS>), grid, dim3(NT), lds, s, a, part, n_cb, rpg);
  else
    hipLaunchKernelGGL((splitk_kernel<K, false, 1>), grid, dim3(NT), lds, s, a, part, n_cb, rpg);
  ZMI_CHECK(hipGetLastError());
  if (ln_w) {
    hipLaunchKernelGGL(splitk_reduce_ln_kernel<S::NSEG>, dim3(a.M), dim3(256), 0, s, part, a.M, (bf16_t*)a.out, a.ldo,
                       (const bf16_t*)ln_w, (const bf16_t*)ln_b, eps, (bf16_t*)xn, ldxn);
  } else {
    const size_t total = (size_t)a.M * a.N;
    if (epi == ZMI_EPI_RESIDUAL)
      hipLaunchKernelGGL((splitk_reduce_kernel<S::NSEG, true>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                         part, a.M, a.N, (bf16_t*)a.out, a.ldo);
    else
      hipLaunchKernelGGL((splitk_reduce_kernel<S::NSEG, false>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                         part, a.M, a.N, (bf16_t*)a.out, a.ldo);
  }
  ZMI_CHECK(hipGetLastError());
  return 0;
}
}  // namespace

extern "C" int zmi_gemv_splitk_ln(const ZmiGemvArgs* args, int epi, float* part, int64_t part_floats, const void* ln_w,
                                  const void* ln_b, float eps, void* xn, int ldxn, void* stream) {
  const ZmiGemvArgs& a = *args;
  if (ln_w && (!ln_b || !xn || a.N != 2048 || ldxn < 2048 || ldxn % 8 || a.ldo % 8))
    return zmi_fail_msg("gemv_splitk_ln: the fused LayerNorm needs N = 2048, ln_b, xn (ldxn % 8) and ldo % 8");
  if (epi != ZMI_EPI_RESIDUAL && epi != ZMI_EPI_STORE) return zmi_fail_msg("gemv_splitk: EPI_RESIDUAL or EPI_STORE only");
  if (ln_w && epi != ZMI_EPI_RESIDUAL) return zmi_fail_msg("gemv_splitk_ln: the fused LayerNorm follows EPI_RESIDUAL");
  if ((a.K != 8192 && a.K != 4096 && a.K != 2048) || a.ln_w || a.pro != ZMI_PRO_AUTO)
    return zmi_fail_msg("gemv_splitk: plain K = 8192 (fc2), 4096 (Mamba2 out_proj) or 2048 (out_proj) only");
  if (a.N % (8 * NWV) || a.n_valid != a.N) return zmi_fail_msg("gemv_splitk: N a multiple of 64, unpadded");
  if (a.M < 1 || a.ldx % 8 || a.ldo < a.N) return zmi_fail_msg("gemv_splitk: rows / strides");
  const int nseg = a.K == 8192 ? Shape<8192>::NSEG : (a.K == 4096 ? Shape<4096>::NSEG : Shape<2048>::NSEG);
  if (!part || part_floats < (int64_t)nseg * a.M * a.N) return zmi_fail_msg("gemv_splitk: partial buffer too small");
  hipStream_t s = (hipStream_t)stream;
  if (a.K == 8192) return launch_splitk<8192>(a, epi, part, ln_w, ln_b, eps, xn, ldxn, s);
  if (a.K == 4096) return launch_splitk<4096>(a, epi, part, ln_w, ln_b, eps, xn, ldxn, s);
  return launch_splitk<2048>(a, epi, part, ln_w, ln_b, eps, xn, ldxn, s);
}

extern "C" int zmi_gemv_splitk(const ZmiGemvArgs* args, int epi, float* part, int64_t part_floats, void* stream) {
  return zmi_gemv_splitk_ln(args, epi, part, part_floats, nullptr, nullptr, 0.f, nullptr, 0, stream);
}
