// Fused decode launch: the attention output projection (+ residual) and the first FFN projection
// (LayerNorm + fc1 + SwiGLU) of one transformer block — reference zonos/backbone/_torch.py:100-101
// (x = x + mixer(...)), :101 norm2, :147-152 (fc1 -> chunk -> y * silu(gate)).
//
// Why: as two launches, out_proj is a latency chain (8.4 MB of weights but ~3 us of ramp, activation
// fetch, reduction and epilogue, plus a kernel boundary) during which HBM idles, and fc1 only starts
// streaming its 67 MB after it. Here every CU runs one workgroup that does both: it fetches its slice of
// out_proj's weights first, then streams its fc1 slice (256 KB) while the out_proj chain runs; the new
// residual rows reach every workgroup as 8-byte {bf16 pair, tag = position + 1} granules (the data is
// its own flag: cdna_hip_programming.md §6 Guideline 16 R2; nothing is counted or re-armed; a row that
// starts a new utterance has its granules zeroed by the engine). fc1's weights stream under the whole
// hand-off, so the launch costs about fc1's own streaming time.
//
// Workgroup b (1024 threads = 16 waves, one per CU, 256 of them):
//   out_proj  column group b (8 of the 2048 outputs): waves 0..3, one K segment each (the K = 2048
//             GEMV shape: W = 4 waves x NL = 8 chunks); wave 0's epilogue writes x and the granules;
//   fc1       column groups 8b .. 8b + 7 (64 packed columns = 32 values + 32 gates): wave w holds the
//             K segment w & 3 of groups (w >> 2) and (w >> 2) + 4.
// The arithmetic is zmi_gemv_impl.h's gemv_body operation for operation (per-wave MFMA chains, the
// segment sums in wave order, the residual / LayerNorm / SwiGLU steps), so the outputs are bit-identical
// to zmi_gemv_launch(out_proj, EPI_RESIDUAL) followed by zmi_gemv_launch(fc1 with LayerNorm, EPI_SWIGLU).
#include <algorithm>

#include "zmi_common.h"
#include "zmi_kernels.h"
#include "zonos_diag.h"
#include "zmi_gemv_impl.h"

namespace {

using zmi_gemv::dma_piece;
using zmi_gemv::ror8;

constexpr int K = 2048, W = 4, NL = 8, KC = K / 64, RT = 16;
constexpr int NW = 16, NT = NW * 64;
constexpr int XROW = K + 8;
constexpr int FG = 8;                 // fc1 column groups per workgroup
constexpr int NBLK = 256;             // workgroups: 2048 out_proj groups / 8 ... = 256, 16384 fc1 columns / 64
constexpr int GPAIRS = K / 2;         // granules per row (bf16 pairs of the new residual row)
constexpr unsigned SPIN = 1u << 18;

struct Img {
  // xa: attention rows (out_proj activations), xs: new residual rows (fc1 activations, LayerNorm'd in
  // place), gamma / beta, segment sums of fc1 (32 wave-group slots) and of out_proj (4 waves)
  static size_t bytes(int rows) {
    return (size_t)2 * rows * XROW * 2 + (size_t)2 * K * 2 + (size_t)NW * 2 * 8 * RT * 4 + (size_t)W * 8 * RT * 4 + 16;
  }
};

__device__ __forceinline__ uint32_t tag_of(uint64_t g) { return (uint32_t)(g >> 32); }

// Diagnostic build only (-DZMI_FFN_STAMPS, tools/ffnblk_stamps.py): thread 0 of every workgroup writes
// s_memrealtime (100 MHz) at phase boundaries into f.diag[block][8]; the real kernel has none.
#ifdef ZMI_FFN_STAMPS
#define ZMI_FSTAMP(i)                                                                                      \
  do {                                                                                                     \
    __builtin_amdgcn_sched_barrier(0);                                                                     \
    if (threadIdx.x == 0 && f.diag)                                                                        \
      reinterpret_cast<unsigned long long*>(f.diag)[(size_t)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                                     \
  } while (0)
#else
#define ZMI_FSTAMP(i) \
  do {                \
  } while (0)
#endif

__global__ __launch_bounds__(NT) void ffn_block_kernel(const ZmiGemvArgs o, const ZmiGemvArgs f, uint64_t* gran,
                                                       unsigned* err) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  const int rows = o.M;
  bf16_t* xa = reinterpret_cast<bf16_t*>(smem);
  bf16_t* xs = xa + (size_t)rows * XROW;
  bf16_t* gam = xs + (size_t)rows * XROW;
  bf16_t* bet = gam + K;
  float* red = reinterpret_cast<float*>(bet + K);   // [NW * 2][8][RT]
  float* redo = red + NW * 2 * 8 * RT;              // [W][8][RT]
  unsigned* arrive = reinterpret_cast<unsigned*>(redo + W * 8 * RT);  // out_proj waves' LDS barrier

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int NE = (8 * RT + 63) / 64;
  ZMI_FSTAMP(0);

  // (1) waves 0..3: the attention rows (DMA), the old residual values of the out_proj epilogue, the
  // out_proj weight slice; waves 4..7: LayerNorm gamma / beta (DMA). All issued before any fc1 weight,
  // so they are at the head of the CU's memory queue.
  const int col0 = b * 8;
  if (tid == 0) *arrive = 0u;
  uint32_t res_pre[NE];
  u32x4_t wo[NL];
  if (wave < W) {
    const bf16_t* X = reinterpret_cast<const bf16_t*>(o.X);
    for (int pc = wave; pc < rows * (K / 512); pc += W) {
      const int r = pc / (K / 512), p = pc - r * (K / 512);
      dma_piece(X + (size_t)r * o.ldx + p * 512 + lane * 8, xa + r * XROW + p * 512);
    }
    if (wave == 0) {
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const int e = lane + 64 * i, r = e >> 3, n = col0 + (e & 7);
        res_pre[i] = r < rows ? reinterpret_cast<const bf16_t*>(o.out)[(size_t)r * o.ldo + n] : 0u;
      }
    }
    const char* wb = reinterpret_cast<const char*>(o.W) + ((size_t)b * KC + wave * NL) * 1024;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wb), (short)0, NL * 1024, 0x00020000);
#pragma unroll
    for (int j = 0; j < NL; ++j) wo[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, j * 1024, 2);
  } else if (wave < 2 * W) {
    const int q = wave - W;  // 8 pieces: gamma 0..3, beta 4..7
    for (int pc = q; pc < 8; pc += W) {
      const bf16_t* src = reinterpret_cast<const bf16_t*>(pc < 4 ? f.ln_w : f.ln_b);
      dma_piece(src + (pc & 3) * 512 + lane * 8, (pc < 4 ? gam : bet) + (pc & 3) * 512);
    }
  }
  __syncthreads();  // (every wave passes here once the out_proj loads are issued)

  // (2) fc1 weight slices: waves 4..15 now; waves 0..3 after their out_proj chain and the hand-off
  u32x4_t wf[2][NL];
  const int wk = wave & 3;
  auto issue_fc1 = [&](int k_lo, int k_hi) {
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      if (k2 < k_lo || k2 >= k_hi) continue;
      const int g = b * FG + (wave >> 2) + 4 * k2;
      const char* wb = reinterpret_cast<const char*>(f.W) + ((size_t)g * KC + wk * NL) * 1024;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wb), (short)0, NL * 1024, 0x00020000);
#pragma unroll
      for (int j = 0; j < NL; ++j) wf[k2][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, j * 1024, 2);
    }
  };
  // (3) out_proj: waves 0..3 run their K segment's MFMA chain over the attention rows. The other waves
  // hold their fc1 loads until these operands have landed: under a saturated memory system a request is
  // not served in issue order, so the out_proj operands would otherwise arrive with the fc1 stream
  if (wave < 2 * W) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // DMA pieces, residual values, weights
  __syncthreads();
  ZMI_FSTAMP(1);
  // the first of each wave's two fc1 slices now, the second after the hand-off: a shallower memory queue
  // while the out_proj chain and the granule sweeps run (their loads wait behind whatever is queued)
  if (wave >= W) issue_fc1(0, 1);
  if (wave < W) {
    f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    const int ar = min(lane & 15, rows - 1);
    const bf16_t* xr = xa + ar * XROW + wave * NL * 64 + (lane >> 4) * 8;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const uint4 x0 = *reinterpret_cast<const uint4*>(xr + j * 64);
      const uint4 x1 = *reinterpret_cast<const uint4*>(xr + j * 64 + 32);
      const bf16x8_t wv = __builtin_bit_cast(bf16x8_t, wo[j]);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x0), wv, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x1), wv, acc1, 0, 0, 0);
    }
    const int c = lane & 15, rb = (lane >> 4) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float v = acc0[q] + ror8(acc1[q]);
      if (c < 8 && rb + q < RT) redo[(wave * 8 + c) * RT + rb + q] = v;
    }
    // a barrier of the four out_proj waves only (LDS arrival count): a workgroup barrier here would wait
    // for the other twelve waves, which are still issuing their fc1 loads into a full memory queue
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (wave == 0) {
      for (unsigned spins = 0; __hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (unsigned)W;
           ++spins)
        __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
  }
  // (4) wave 0: x = x + bf16(out_proj) (the EPI_RESIDUAL epilogue), stored to x and, for every active
  // row, as {pair, tag} granules to all workgroups
  if (wave == 0) {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = lane + 64 * i, r = e >> 3, c = e & 7, n = col0 + c;
      float v = redo[(0 * 8 + c) * RT + (r < RT ? r : 0)];
#pragma unroll
      for (int w = 1; w < W; ++w) v += redo[(w * 8 + c) * RT + (r < RT ? r : 0)];
      const uint32_t hv = f2bf(bf2f(res_pre[i]) + bfround(v));
      const uint32_t nb = (uint32_t)__shfl_down((int)hv, 1);
      if (r < rows) {
        reinterpret_cast<bf16_t*>(o.out)[(size_t)r * o.ldo + n] = (bf16_t)hv;
        const int pos = o.row_pos[r];
        if ((c & 1) == 0 && pos >= 0)
          st_wt64(gran + (size_t)r * GPAIRS + (n >> 1), (uint64_t)(hv | (nb << 16)) | ((uint64_t)(unsigned)(pos + 1) << 32));
      }
    }
  }
  ZMI_FSTAMP(2);
  // (5) waves 0..3: every row's new residual from the granules of all 256 workgroups into LDS (8 per lane
  // per sweep), then their own fc1 weight slices
  if (wave < W) {
    const int q = wave * 64 + lane;  // 0 .. 255
    for (int r = 0; r < rows; ++r) {
      const int pos = o.row_pos[r];
      uint32_t* dst = reinterpret_cast<uint32_t*>(xs + r * XROW);
      if (pos < 0) {  // inactive row: no granules; its fc1 output is never used
#pragma unroll
        for (int i = 0; i < GPAIRS / 256; ++i) dst[q + 256 * i] = 0u;
        continue;
      }
      const uint32_t tag = (uint32_t)pos + 1u;
      const uint64_t* src = gran + (size_t)r * GPAIRS;
      uint64_t g[GPAIRS / 256];
      unsigned pend = (1u << (GPAIRS / 256)) - 1u;
      for (unsigned spins = 0; pend; ++spins) {
#pragma unroll
        for (int i = 0; i < GPAIRS / 256; ++i)
          if ((pend >> i) & 1) g[i] = ld_wt64(src + q + 256 * i);
#pragma unroll
        for (int i = 0; i < GPAIRS / 256; ++i)
          if (((pend >> i) & 1) && tag_of(g[i]) == tag) {
            dst[q + 256 * i] = (uint32_t)g[i];
            pend &= ~(1u << i);
          }
        if (!pend) break;
        if (spins > SPIN) {
          if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    ZMI_FSTAMP(3);
    issue_fc1(0, 2);
  }
  __syncthreads();
  ZMI_FSTAMP(4);
  if (wave >= W) issue_fc1(1, 2);

  // (6) LayerNorm of the new residual rows (zmi_gemv_impl.h PRO_LN: one wave per row, the same sums)
  {
    constexpr int NQ = ln_parts(K), CPQ = K / (512 * NQ);
    for (int r = wave; r < rows; r += NW) {
      bf16_t* xr = xs + r * XROW;
      auto pass = [&](float mean, bool sq, float(&ps)[NQ]) {
        float tq[NQ];
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) {
          tq[qq] = 0.f;
#pragma unroll
          for (int i = 0; i < CPQ; ++i)
            tq[qq] += ln_chunk_sum(*reinterpret_cast<const uint4*>(xr + qq * (K / NQ) + (lane + 64 * i) * 8), mean, sq);
        }
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) ps[qq] = wave_sum(tq[qq]);
      };
      float ps[NQ];
      pass(0.f, false, ps);
      const float mean = ln_combine<NQ>(ps) / (float)K;
      pass(mean, true, ps);
      const float rstd = 1.0f / sqrtf(ln_combine<NQ>(ps) / (float)K + f.eps), nbias = -mean * rstd;
#pragma unroll
      for (int qq = 0; qq < NQ; ++qq)
#pragma unroll
        for (int i = 0; i < CPQ; ++i) {
          const int c = qq * (K / NQ) / 8 + lane + 64 * i;
          bf16_t* xc = xr + qq * (K / NQ) + (lane + 64 * i) * 8;
          const uint4 xv = *reinterpret_cast<const uint4*>(xc);
          *reinterpret_cast<uint4*>(xc) = ln_apply(xv, *reinterpret_cast<const uint4*>(gam + c * 8),
                                                   *reinterpret_cast<const uint4*>(bet + c * 8), rstd, nbias);
        }
    }
  }
  __syncthreads();
  ZMI_FSTAMP(5);

  // (7) fc1: each wave's two K-segment chains (weights landed: the compiler's vmcnt before each use)
  {
    const int ar = min(lane & 15, rows - 1);
    const bf16_t* xr = xs + ar * XROW + wk * NL * 64 + (lane >> 4) * 8;
    const int c = lane & 15, rb = (lane >> 4) * 4;
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        const uint4 x0 = *reinterpret_cast<const uint4*>(xr + j * 64);
        const uint4 x1 = *reinterpret_cast<const uint4*>(xr + j * 64 + 32);
        const bf16x8_t wv = __builtin_bit_cast(bf16x8_t, wf[k2][j]);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x0), wv, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x1), wv, acc1, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float v = acc0[q] + ror8(acc1[q]);
        if (c < 8 && rb + q < RT) red[((wave * 2 + k2) * 8 + c) * RT + rb + q] = v;
      }
    }
  }
  __syncthreads();
  ZMI_FSTAMP(6);
  // (8) SwiGLU epilogue (EPI_SWIGLU): group gl's segments are waves 4 (gl % 4) .. + 3, slot gl / 4; the
  // wave holding segment 0 writes it. Columns 0..3 of a group are values, 4..7 their gates.
  if (wk == 0) {
    const int r = lane >> 2, c = lane & 3;
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const int gl = (wave >> 2) + 4 * k2, g = b * FG + gl;
      auto colsum = [&](int cc) {
        float v = red[(((wave + 0) * 2 + k2) * 8 + cc) * RT + r];
#pragma unroll
        for (int w = 1; w < W; ++w) v += red[(((wave + w) * 2 + k2) * 8 + cc) * RT + r];
        return v;
      };
      if (r < rows) {
        const float y = bfround(colsum(c));
        const float gt = bfround(colsum(c + 4));
        const float sg = bfround(gt / (1.0f + expf(-gt)));
        reinterpret_cast<bf16_t*>(f.out)[(size_t)r * f.ldo + g * 4 + c] = (bf16_t)f2bf(y * sg);
      }
    }
  }
  ZMI_FSTAMP(7);
}

}  // namespace

extern "C" int64_t zmi_ffn_block_gran_words(int rows) { return rows <= 0 ? -1 : (int64_t)rows * GPAIRS; }

extern "C" int zmi_ffn_block(const ZmiGemvArgs* out_proj, const ZmiGemvArgs* fc1, void* gran, unsigned* err,
                             void* stream) {
  const ZmiGemvArgs& o = *out_proj;
  const ZmiGemvArgs& f = *fc1;
  if (o.K != K || o.N != K || o.n_valid != K || f.K != K || f.N != NBLK * FG * 8 || f.n_valid != f.N)
    return zmi_fail_msg("ffn_block: out_proj [2048 x 2048] and fc1 [16384 x 2048] (packed SwiGLU) only");
  if (o.M < 1 || o.M > RT || f.M != o.M) return zmi_fail_msg("ffn_block: 1 <= M <= 16 rows, equal for both");
  if (o.ln_w || o.pro != ZMI_PRO_AUTO || !f.ln_w || !f.ln_b || f.pro != ZMI_PRO_AUTO)
    return zmi_fail_msg("ffn_block: out_proj plain, fc1 LayerNorm'd");
  if (f.X != o.out || f.ldx != o.ldo) return zmi_fail_msg("ffn_block: fc1 must read the rows out_proj writes");
  if (!o.row_pos || !gran || !err || !o.X || !o.out || !f.out) return zmi_fail_msg("ffn_block: missing buffers");
  if (o.ldx % 8 || o.ldo % 8 || f.ldo % 4) return zmi_fail_msg("ffn_block: row strides");
  if (zmi_cu_count() < NBLK) return zmi_fail_msg("ffn_block: needs 256 CUs (all workgroups resident at once)");
  const size_t lds = std::max(Img::bytes(o.M), zmi_gemv::LDS_MAX / 2 + 1024);  // one workgroup per CU
  if (lds > zmi_gemv::LDS_MAX) return zmi_fail_msg("ffn_block: LDS");
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&ffn_block_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)zmi_gemv::LDS_MAX);
  ZMI_CHECK(attr);
  hipLaunchKernelGGL(ffn_block_kernel, dim3(NBLK), dim3(NT), lds, (hipStream_t)stream, o, f, (uint64_t*)gran, err);
  ZMI_CHECK(hipGetLastError());
  return 0;
}
