// Fused decode launch of a transformer block after its QKV projection: decode attention, the attention
// output projection (+ residual), LayerNorm and fc1 + SwiGLU — reference zonos/backbone/_torch.py:136
// (scaled_dot_product_attention over the KV cache), :140 (out_proj), :100-101 (x = x + mixer(...);
// norm2), :147-152 (fc1 -> chunk -> y * silu(gate)). The QKV projection (LayerNorm + QKV + RoPE + KV
// write, :114-133) is the launch before this one (zmi_gemv_launch with EPI_QKV).
//
// Why: the attention is a latency chain (two small hand-offs between the chunks of a query) during which
// HBM idles for ~5 us per layer, and fc1's 67 MB only started streaming after it (zmi_attn_block then
// zmi_ffn_block). Here the CUs that do not run the attention stream their whole share of the out_proj and
// fc1 weights into registers from the first cycle, so the chain runs under the weight stream:
//
//   workgroups [0, 64)    "attention" workgroups: the chunk-split attention of zmi_attn_block
//                         (zmi_attnblk.hip xc_body: one workgroup per (row, kv head, 128-key chunk); q and
//                         this position's K / V row are read from memory, the QKV launch wrote them), then
//                         out_proj column group b and 5 fc1 column groups, whose weights they load only after
//                         the chain (a CU's loads are served in order: polls queued behind a weight stream
//                         wait for it);
//   workgroups [64, 256)  out_proj column group b and 9 fc1 column groups, every weight issued at launch start.
// 64 x 5 + 192 x 9 = 2048 fc1 groups of 8 packed columns (16384 = 8192 values + 8192 gates).
//
// Hand-offs are 8-byte {bf16 pair or f32, tag = position + 1} granules (cdna_hip_programming.md §6
// Guideline 16 R2; nothing counted or re-armed; a row starting a new utterance has its words zeroed):
//   attention chunks -> attention chunks: maxima, P.V partials (xc_body's layout in the zmi_attn_block area);
//   attention -> every workgroup: the attention output rows (`ogran`, [row][1024]);
//   out_proj -> every workgroup: the new residual rows (`rgran`, zmi_ffn_block's layout).
// The arithmetic is the separate launches' operation for operation (the chunked attention kernel's chunk
// sums and merge recursion, the GEMV's per-wave MFMA chains with the segment sums in K order, the
// residual / LayerNorm / SwiGLU steps), so x, h and the attention rows are bit-identical to
// zmi_attn_block (SPLIT) + zmi_ffn_block, and to zmi_attention + two zmi_gemv_launch calls (tested).
#include <algorithm>

#include "zmi_common.h"
#include "zmi_kernels.h"
#include "zonos_diag.h"
#include "zmi_gemv_impl.h"
#include "zmi_attn_ds.h"

namespace {

using namespace zmi_attn;
using zmi_gemv::dma_piece;
using zmi_gemv::ror8;

constexpr int K = 2048, W = 4, NL = 8, KC = K / 64, RT = 16;
constexpr int NW = 16, NT = NW * 64;
constexpr int XROW = K + 8;
constexpr int NBLK = 256;
constexpr int GPAIRS = K / 2;           // granules per row (bf16 pairs)
constexpr int N_ATT = 64;               // attention-class workgroups (8 chunks x 8 units)
constexpr int G_ATT = 5, G_OTH = 9;     // fc1 column groups per attention / other workgroup
static_assert(N_ATT * G_ATT + (NBLK - N_ATT) * G_OTH == 2048, "every fc1 group once");
constexpr int MAX_SEG = 4 * G_OTH;      // fc1 K segments of a workgroup (4 per group)
static_assert(MAX_SEG == 4 + 12 + 12 + 8, "slots: 1 per out_proj wave, 2 per other wave, 8 in LDS");
constexpr unsigned SPIN = 1u << 18;

constexpr int XG = 4;                   // query heads per kv head
constexpr int XC_CH = 8;                // chunk workgroups per (row, kv head)
constexpr int XC_KEYS = XC_CH * CH;     // positions 0 .. 1023
constexpr int CPG = CH / 32;            // 32-key groups per chunk
// zmi_attn_block's granule area per unit: q / K / V pairs, then the chunk-split exchange words
constexpr int QKV_GRAN = (XG + 2) * HD / 2;
constexpr int GRAN_STRIDE = QKV_GRAN + XG * DS_KEYS;
constexpr int XC_GM = 0, XC_GL = XC_GM + XC_CH * XG, XC_GB = XC_GL + XC_CH * XG, XC_GO = XC_GB + XC_CH * XG;
static_assert(XC_GO + XC_CH * XG * HD <= XG * DS_KEYS, "exchange words fit the unit's area");
static_assert(CH == 128, "eight score waves: one 16-key tile each over a 128-key chunk");

struct Img {
  static constexpr size_t SC = 0;                               // f32 [XG][CH] chunk scores
  static constexpr size_t PB = SC + (size_t)XG * CH * 4;        // bf16 [XG][CH] P
  static constexpr size_t OP = PB + (size_t)XG * CH * 2;        // f32 [CPG][XG][HD] per-group P.V
  static constexpr size_t MJ = OP + (size_t)CPG * XG * HD * 4;  // f32 [XG] M_j of the chunk's block
  static constexpr size_t ARR = MJ + (size_t)XG * 4;            // u32 [4] arrival counters of waves 0..3
  static constexpr size_t FFN = (ARR + 16 + 15) / 16 * 16;
  // xa [rows][XROW] attention rows, xs [rows][XROW] new residual rows (LayerNorm'd in place), gamma, beta,
  // red [MAX_SEG][8][RT] fc1 segment sums, redo [W][8][RT] out_proj segment sums; then the fc1 slots kept in
  // LDS ([12][NL][1 KiB], by LDS-DMA): the third slot of waves 4..11, the one slot of waves 0..3
  __host__ __device__ static size_t wslot(int rows) {
    return FFN + (size_t)2 * rows * XROW * 2 + (size_t)2 * K * 2 + (size_t)MAX_SEG * 8 * RT * 4 + (size_t)W * 8 * RT * 4;
  }
  __host__ __device__ static size_t bytes(int rows) { return wslot(rows) + (size_t)12 * NL * 1024; }
};

__device__ __forceinline__ uint32_t tag_of(uint64_t g) { return (uint32_t)(g >> 32); }
__device__ __forceinline__ void give_up(unsigned* err) {
  __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// barrier of waves 0..3 only (LDS arrival count): the other waves may still be issuing weight loads
__device__ __forceinline__ void quad_barrier(unsigned* ctr, int lane) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  for (unsigned spins = 0; __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (unsigned)W; ++spins)
    __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Diagnostic build only (-DZMI_ATTNFFN_STAMPS, tools/attnffn_stamps.py): thread 0 of every workgroup writes
// s_memrealtime (100 MHz) at phase boundaries into f.diag[block][16]; the real kernel has none.
#ifdef ZMI_ATTNFFN_STAMPS
#define ZMI_YSTAMP(i)                                                                                      \
  do {                                                                                                     \
    __builtin_amdgcn_sched_barrier(0);                                                                     \
    if (threadIdx.x == 0 && f.diag)                                                                        \
      reinterpret_cast<unsigned long long*>(f.diag)[(size_t)blockIdx.x * 16 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                                     \
  } while (0)
#else
#define ZMI_YSTAMP(i) \
  do {                \
  } while (0)
#endif

// T: weight loads a streaming wave keeps in flight (0: all at once). Every request waits behind what the chip
// already has queued, so an unthrottled 75 MB stream (~300 KB per CU issued at launch start) delays the
// attention's K / V loads and every hand-off poll by the whole stream (~10 us, measured); T KiB per wave keeps
// the queue near bandwidth x latency.
template <int T>
__global__ __launch_bounds__(NT) void attn_ffn_kernel(const AttnArgs at, int n_units, const ZmiGemvArgs o,
                                                      const ZmiGemvArgs f, uint64_t* xgran, uint64_t* ogran,
                                                      uint64_t* rgran, int delay) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float(&sc)[XG][CH] = *reinterpret_cast<float(*)[XG][CH]>(smem + Img::SC);
  bf16_t(&pb)[XG][CH] = *reinterpret_cast<bf16_t(*)[XG][CH]>(smem + Img::PB);
  float(&opart)[CPG][XG][HD] = *reinterpret_cast<float(*)[CPG][XG][HD]>(smem + Img::OP);
  float* mj = reinterpret_cast<float*>(smem + Img::MJ);
  unsigned* arr = reinterpret_cast<unsigned*>(smem + Img::ARR);
  const int rows = o.M;
  bf16_t* xa = reinterpret_cast<bf16_t*>(smem + Img::FFN);
  bf16_t* xs = xa + (size_t)rows * XROW;
  bf16_t* gam = xs + (size_t)rows * XROW;
  bf16_t* bet = gam + K;
  float* red = reinterpret_cast<float*>(bet + K);  // [MAX_SEG][8][RT]
  float* redo = red + MAX_SEG * 8 * RT;             // [W][8][RT]
  char* wsl = smem + Img::wslot(rows);              // [12][NL][1 KiB] fc1 slots in LDS

  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int c16 = lane & 15, h4 = lane >> 4;
  constexpr int NE = (8 * RT + 63) / 64;
  ZMI_YSTAMP(0);
  if (t < 4) arr[t] = 0u;
  __syncthreads();

  // ---- roles of this workgroup ------------------------------------------------------------------------
  const bool att_class = b < N_ATT;
  const int n_grp = att_class ? G_ATT : G_OTH;
  const int g_base = att_class ? (NBLK - N_ATT) * G_OTH + G_ATT * b : G_OTH * (b - N_ATT);
  // xc_body's block -> (unit, chunk) map: the 8 chunks of a unit have equal b & 7 (one XCD)
  const int c = (b >> 3) % XC_CH, unit = 8 * ((b >> 3) / XC_CH) + (b & 7);
  const bool unit_ok = att_class && unit < n_units;
  const int qi = unit_ok ? unit / at.hkv : 0, kh = unit_ok ? unit - qi * at.hkv : 0;
  const int gs = wave >> 1, tt = wave & 1, gv = wave & 3, hv = wave >> 2;  // score tile / V fragment of wave < 8
  // the rows' positions, loaded once (the hand-off tags of the tail)
  const int rpos0 = o.row_pos[0], rpos1 = rows > 1 ? o.row_pos[1] : -1;
  auto row_pos_of = [&](int r) { return r == 0 ? rpos0 : rpos1; };

  const int col0 = b * 8;
  // fc1 slots. Waves 4..15 keep two slots in registers, and waves 4..11 a third in LDS; waves 0..3 (the
  // out_proj waves, which hold wx) keep their one slot in LDS. Slot 0 is K segment `wave`, slot 1 segment
  // 12 + wave (waves 4..15), slot 2 segment 24 + wave (waves 4..11); segment s = 4 x group + k-segment. LDS
  // slot index: wave - 4 for the third slots, 8 + wave for the out_proj waves' slot. Registers are allocated
  // for the union of what any wave keeps live, so the out_proj waves and the others run separate code paths
  // after the prologue (each path keeps only its own weights live).
  auto seg_of = [&](int k) { return k == 0 ? wave : (k == 1 ? 12 + wave : 24 + wave); };
  auto throttle = [&]() {
    if constexpr (T > 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(T) : "memory");
  };
  auto issue_slot = [&](int k, u32x4_t(&dst)[NL]) {
    const int s = seg_of(k);
    const int g = g_base + (s >> 2);
    const char* wb = reinterpret_cast<const char*>(f.W) + ((size_t)g * KC + (s & 3) * NL) * 1024;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wb), (short)0, NL * 1024, 0x00020000);
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      dst[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, j * 1024, 2);
      throttle();
    }
  };
  const int nseg = 4 * n_grp;
  const bool has1 = wave >= W && seg_of(1) < nseg, has2 = wave >= W && wave < 12 && seg_of(2) < nseg;
  auto issue_lds = [&](int k, int idx) {  // LDS-DMA, 1 KiB per piece
    const int s = seg_of(k);
    const bf16_t* src = reinterpret_cast<const bf16_t*>(f.W) + (((size_t)(g_base + (s >> 2)) * KC + (s & 3) * NL) * 1024) / 2;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      dma_piece(src + j * 512 + lane * 8, reinterpret_cast<bf16_t*>(wsl + (idx * NL + j) * 1024));
      throttle();
    }
  };
  auto issue_fc1_f = [&](u32x4_t(&wf)[2][NL]) {  // waves 4..15
    if (has2) issue_lds(2, wave - W);
    if (seg_of(0) < nseg) issue_slot(0, wf[0]);
    if (has1) issue_slot(1, wf[1]);
  };

  // ---- shared steps of the tail ----------------------------------------------------------------------
  const int q = (wave & 3) * 64 + lane;  // 0 .. 255 within waves 0..3
  // the rows of a {pair, tag} granule area into LDS (waves 0..3, 4 words per lane and row); inactive rows:
  // `fallback` rows as they stand in memory, or zeros
  auto gather = [&](const uint64_t* area, bf16_t* dst_rows, const bf16_t* fallback, int ld_fb) {
    for (int r = 0; r < rows; ++r) {
      const int rp = row_pos_of(r);
      uint32_t* dst = reinterpret_cast<uint32_t*>(dst_rows + r * XROW);
      if (rp < 0) {
        const uint4 v = fallback ? reinterpret_cast<const uint4*>(fallback + (size_t)r * ld_fb)[q] : uint4{0u, 0u, 0u, 0u};
        reinterpret_cast<uint4*>(dst)[q] = v;
        continue;
      }
      const uint32_t rtag = (uint32_t)rp + 1u;
      const uint64_t* src = area + (size_t)r * GPAIRS;
      uint64_t g[GPAIRS / 256];
      unsigned pend = (1u << (GPAIRS / 256)) - 1u;
      for (unsigned spins = 0; pend; ++spins) {
#pragma unroll
        for (int i = 0; i < GPAIRS / 256; ++i)
          if ((pend >> i) & 1) g[i] = ld_wt64(src + q + 256 * i);
#pragma unroll
        for (int i = 0; i < GPAIRS / 256; ++i)
          if (((pend >> i) & 1) && tag_of(g[i]) == rtag) {
            dst[q + 256 * i] = (uint32_t)g[i];
            pend &= ~(1u << i);
          }
        if (!pend) break;
        if (spins > SPIN) {
          if (lane == 0) give_up(at.err);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
  };
  // LayerNorm of new residual row r (zmi_gemv_impl.h PRO_LN arithmetic: one wave per row)
  auto layernorm = [&](int r) {
    constexpr int NQ = ln_parts(K), CPQ = K / (512 * NQ);
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
        const int cg = qq * (K / NQ) / 8 + lane + 64 * i;
        bf16_t* xc = xr + qq * (K / NQ) + (lane + 64 * i) * 8;
        const uint4 xv = *reinterpret_cast<const uint4*>(xc);
        *reinterpret_cast<uint4*>(xc) = ln_apply(xv, *reinterpret_cast<const uint4*>(gam + cg * 8),
                                                 *reinterpret_cast<const uint4*>(bet + cg * 8), rstd, nbias);
      }
  };
  // one K segment's MFMA chain (the GEMV's per-wave arithmetic) into red[segment]
  auto chain = [&](int s, auto wget) {
    const int ar = min(lane & 15, rows - 1);
    const int cc = lane & 15, rb = (lane >> 4) * 4;
    const bf16_t* xr = xs + ar * XROW + (s & 3) * NL * 64 + (lane >> 4) * 8;
    f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const uint4 x0 = *reinterpret_cast<const uint4*>(xr + j * 64);
      const uint4 x1 = *reinterpret_cast<const uint4*>(xr + j * 64 + 32);
      const bf16x8_t w8 = __builtin_bit_cast(bf16x8_t, wget(j));
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x0), w8, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x1), w8, acc1, 0, 0, 0);
    }
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const float v = acc0[qq] + ror8(acc1[qq]);
      if (cc < 8 && rb + qq < RT) red[(s * 8 + cc) * RT + rb + qq] = v;
    }
  };
  // SwiGLU epilogue (EPI_SWIGLU) of group gl: its K segments 4 gl .. 4 gl + 3 summed in K order; columns
  // 0..3 of a group are values, 4..7 their gates
  auto swiglu = [&](int gl) {
    const int r = lane >> 2, cl = lane & 3, g = g_base + gl;
    auto colsum = [&](int cc) {
      float v = red[((4 * gl) * 8 + cc) * RT + r];
#pragma unroll
      for (int w = 1; w < W; ++w) v += red[((4 * gl + w) * 8 + cc) * RT + r];
      return v;
    };
    if (r < rows) {
      const float y = bfround(colsum(cl));
      const float gt = bfround(colsum(cl + 4));
      const float sg = bfround(gt / (1.0f + expf(-gt)));
      reinterpret_cast<bf16_t*>(f.out)[(size_t)r * f.ldo + g * 4 + cl] = (bf16_t)f2bf(y * sg);
    }
  };

  // the out_proj waves' path to the end (wget_o: their out_proj weight fragments; slot_after: load the fc1 slot
  // into LDS only after the residual epilogue, the attention workgroups' order)
  auto o_tail = [&](auto wget_o, const uint32_t(&res_pre)[NE], bool slot_after) {
      // (B1) the attention rows (inactive rows: attn_out as it stands, as the separate launch reads it)
      gather(ogran, xa, reinterpret_cast<const bf16_t*>(o.X), o.ldx);
      ZMI_YSTAMP(5);
      quad_barrier(arr + 0, lane);
      // (B2) out_proj: wave w's K segment chain over the attention rows (weights in wx, or in LDS slot 8 + w
      // for the attention workgroups)
      auto oproj = [&](auto wget) {
        f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        const int ar = min(lane & 15, rows - 1);
        const bf16_t* xr = xa + ar * XROW + wave * NL * 64 + (lane >> 4) * 8;
  #pragma unroll
        for (int j = 0; j < NL; ++j) {
          const uint4 x0 = *reinterpret_cast<const uint4*>(xr + j * 64);
          const uint4 x1 = *reinterpret_cast<const uint4*>(xr + j * 64 + 32);
          const bf16x8_t wv = __builtin_bit_cast(bf16x8_t, wget(j));
          acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x0), wv, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x1), wv, acc1, 0, 0, 0);
        }
        const int cc = lane & 15, rb = (lane >> 4) * 4;
  #pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const float v = acc0[qq] + ror8(acc1[qq]);
          if (cc < 8 && rb + qq < RT) redo[(wave * 8 + cc) * RT + rb + qq] = v;
        }
      };
      oproj(wget_o);
      quad_barrier(arr + 1, lane);
      // (B3) wave 0: x = x + bf16(out_proj) (EPI_RESIDUAL), stored to x and, for every active row, as granules
      if (wave == 0) {
  #pragma unroll
        for (int i = 0; i < NE; ++i) {
          const int e = lane + 64 * i, r = e >> 3, cl = e & 7, n = col0 + cl;
          float v = redo[(0 * 8 + cl) * RT + (r < RT ? r : 0)];
  #pragma unroll
          for (int w = 1; w < W; ++w) v += redo[(w * 8 + cl) * RT + (r < RT ? r : 0)];
          const uint32_t hv16 = f2bf(bf2f(res_pre[i]) + bfround(v));
          const uint32_t nb = (uint32_t)__shfl_down((int)hv16, 1);
          if (r < rows) {
            reinterpret_cast<bf16_t*>(o.out)[(size_t)r * o.ldo + n] = (bf16_t)hv16;
            const int rp = row_pos_of(r);
            if ((cl & 1) == 0 && rp >= 0)
              st_wt64(rgran + (size_t)r * GPAIRS + (n >> 1), (uint64_t)(hv16 | (nb << 16)) | ((uint64_t)(unsigned)(rp + 1) << 32));
          }
        }
      }
      ZMI_YSTAMP(6);
      if (slot_after) issue_lds(0, 8 + wave);
      // (B4) every row's new residual from the granules of all 256 workgroups (inactive rows: zeros)
      gather(rgran, xs, nullptr, 0);
      ZMI_YSTAMP(7);
      __syncthreads();  // (S1) (waves 0..3 waited for their out_proj weights, so the gamma / beta DMA has landed)
      ZMI_YSTAMP(8);
      if (wave < rows) layernorm(wave);  // rows <= 2
      __syncthreads();  // (S2)
      ZMI_YSTAMP(9);
      {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA pieces (uncounted by the compiler)
        const char* ws = wsl + (size_t)(8 + wave) * NL * 1024 + lane * 16;
        chain(seg_of(0), [&](int j) { return *reinterpret_cast<const u32x4_t*>(ws + j * 1024); });
      }
      __syncthreads();  // (S3)
      ZMI_YSTAMP(10);
      if (wave < n_grp) swiglu(wave);
      ZMI_YSTAMP(11);
  };
  // the fc1 waves' path to the end
  auto f_tail = [&](u32x4_t(&wf)[2][NL]) {
      __syncthreads();  // (S1)
      __syncthreads();  // (S2)
      if (seg_of(0) < nseg) chain(seg_of(0), [&](int j) { return wf[0][j]; });
      if (has1) chain(seg_of(1), [&](int j) { return wf[1][j]; });
      if (has2) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA pieces (uncounted by the compiler)
        const char* ws = wsl + (size_t)(wave - W) * NL * 1024 + lane * 16;
        chain(seg_of(2), [&](int j) { return *reinterpret_cast<const u32x4_t*>(ws + j * 1024); });
      }
      __syncthreads();  // (S3)
      if (wave < n_grp) swiglu(wave);
  };
  // out_proj waves' operands: gamma / beta (waves 0, 1, by DMA, older than the weights: a wait for those
  // covers them), the old residual values (wave 0)
  auto o_operands = [&](uint32_t(&res_pre)[NE]) {
    if (wave < 2) {
      for (int pc = wave; pc < 8; pc += 2) {
        const bf16_t* src = reinterpret_cast<const bf16_t*>(pc < 4 ? f.ln_w : f.ln_b);
        dma_piece(src + (pc & 3) * 512 + lane * 8, (pc < 4 ? gam : bet) + (pc & 3) * 512);
      }
    }
#pragma unroll
    for (int i = 0; i < NE; ++i) res_pre[i] = 0u;
    if (wave == 0) {
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const int e = lane + 64 * i, r = e >> 3, n = col0 + (e & 7);
        res_pre[i] = r < rows ? reinterpret_cast<const bf16_t*>(o.out)[(size_t)r * o.ldo + n] : 0u;
      }
    }
  };
  const char* wo_src = reinterpret_cast<const char*>(o.W) + ((size_t)b * KC + wave * NL) * 1024;  // out_proj slice

  // Every path below runs to the end of the kernel: registers are allocated for the union of what is live at
  // any point, and a path joining another would keep both paths' weights live.
  if (att_class) {
    // ---- attention workgroup: the chunk's K / V^T / q, out_proj's slice into LDS (no registers held across
    // the chain), the attention chain, then the fc1 / out_proj paths
    // the chunk's K rows, V^T fragments and q, at addresses that do not depend on the position (keys past it
    // are masked as the chunked kernel masks them; clamped to the cache), so they go out with the position's
    // own load instead of after it
    uint4 kf[4], vf[4], qf[4];
    const int kvr = at.kv_row ? at.kv_row[qi] : qi;  // decode: NULL (query row r caches into KV row r)
    const size_t kvbase = ((size_t)kvr * at.hkv + kh) * at.smax * HD;
    if (unit_ok && wave < 8) {
      const bf16_t* kr = at.k + kvbase + (size_t)min(CH * c + 32 * gs + 16 * tt + c16, at.smax - 1) * HD + 8 * h4;
#pragma unroll
      for (int db = 0; db < 4; ++db) kf[db] = *reinterpret_cast<const uint4*>(kr + 32 * db);
      const bf16_t* qr = at.q + (size_t)qi * at.ldq + (size_t)(kh * XG + min(c16, XG - 1)) * HD + 8 * h4;
#pragma unroll
      for (int db = 0; db < 4; ++db) qf[db] = c16 < XG ? *reinterpret_cast<const uint4*>(qr + 32 * db) : uint4{0u, 0u, 0u, 0u};
      const int p0 = min(CH * c + 32 * gv + 8 * h4, at.smax - 8);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        vf[dt] = *reinterpret_cast<const uint4*>(at.v + kvbase + (size_t)(64 * hv + 16 * dt + c16) * at.smax + p0);
    }
    int pos = unit_ok ? at.pos[qi] : -1;
    if (pos >= XC_KEYS) {  // the engine never launches this form past its reach; refuse, don't read past it
      if (t == 0) give_up(at.err);
      pos = -1;
    }
    const bool att = pos >= 0;
    const int nk = pos + 1, n32 = (pos + 32) >> 5, nc = pos / CH + 1;
    const uint32_t tag = (uint32_t)pos + 1u;
    const uint64_t tag64 = (uint64_t)tag << 32;
    const bool chunk_live = att && c < nc;
    const bool sk = chunk_live && wave < 8 && CPG * c + gs < n32;
    const bool vk = chunk_live && wave < 8 && CPG * c + gv < n32;
    __builtin_amdgcn_sched_barrier(0);
    uint32_t res_pre[NE];
    if (wave < W) {
      o_operands(res_pre);
#pragma unroll
      for (int j = 0; j < NL; ++j)
        dma_piece(reinterpret_cast<const bf16_t*>(wo_src + j * 1024) + lane * 8,
                  reinterpret_cast<bf16_t*>(wsl + ((8 + wave) * NL + j) * 1024));
    }
    // ---- attention chain (xc_body steps 3-8) ------------------------------------------------------------
    uint64_t* gx = xgran + (size_t)unit * GRAN_STRIDE + QKV_GRAN;
    if (chunk_live) {
      // (3) the tile's scores (the chunked kernel's 4-MFMA chain)
      if (sk) {
        const int key = CH * c + 32 * gs + 16 * tt + c16;
        f32x4_t sv = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int db = 0; db < 4; ++db) sv = mfma16(qf[db], kf[db], sv);
        if (h4 == 0 && key <= pos) {
#pragma unroll
          for (int i = 0; i < XG; ++i) sc[i][key - CH * c] = sv[i] * at.scale;
        }
      }
      __syncthreads();
      ZMI_YSTAMP(1);
      // (4) wave 0: the chunk maxima out as granules, then M_j of the chunk's block from chunks 0 .. dep - 1
      if (wave == 0) {
        float m[XG];
#pragma unroll
        for (int g = 0; g < XG; ++g)
          m[g] = fmaxf(CH * c + lane < nk ? sc[g][lane] : -INFINITY, CH * c + lane + 64 < nk ? sc[g][lane + 64] : -INFINITY);
#pragma unroll
        for (int g = 0; g < XG; ++g) m[g] = wave_max(m[g]);
        if (lane < XG) {
          const float mine = lane == 0 ? m[0] : (lane == 1 ? m[1] : (lane == 2 ? m[2] : m[3]));
          st_wt64(gx + XC_GM + c * XG + lane, (uint64_t)__float_as_uint(mine) | tag64);
        }
        const int j = c / CPB, dep = min((j + 1) * CPB, nc);
        const int cc = lane / XG, g = lane - cc * XG;
        float v = -INFINITY;
        if (lane < dep * XG) {
          if (cc == c) {
            v = g == 0 ? m[0] : (g == 1 ? m[1] : (g == 2 ? m[2] : m[3]));
          } else {
            uint64_t w = ld_wt64(gx + XC_GM + lane);
            for (unsigned spins = 0; tag_of(w) != tag; ++spins) {
              if (spins > SPIN) {
                give_up(at.err);
                break;
              }
              __builtin_amdgcn_s_sleep(2);
              w = ld_wt64(gx + XC_GM + lane);
            }
            v = __uint_as_float((uint32_t)w);
          }
        }
        v = fmaxf(v, __shfl_xor(v, 4));
        v = fmaxf(v, __shfl_xor(v, 8));
        v = fmaxf(v, __shfl_xor(v, 16));
        if (lane < XG) mj[lane] = v;
      }
      __syncthreads();
      ZMI_YSTAMP(2);
      // (5) waves 0..3 (head w): e = exp(s - M_j), l, P = bf16(e)
      if (wave < XG) {
        const float M = mj[wave];
        float l = 0.f;
#pragma unroll
        for (int ii = 0; ii < CH / 64; ++ii) {
          const int kk = lane + 64 * ii;
          const float e = CH * c + kk < nk ? expf(sc[wave][kk] - M) : 0.f;
          l += e;
          pb[wave][kk] = (bf16_t)f2bf(e);
        }
        l = wave_sum(l);
        if (lane == 0) {
          st_wt64(gx + XC_GL + c * XG + wave, (uint64_t)__float_as_uint(l) | tag64);
          st_wt64(gx + XC_GB + c * XG + wave, (uint64_t)__float_as_uint(M) | tag64);
        }
      }
      __syncthreads();
      // (6) P.V of group w & 3 for dims 64 (w >> 2) .. + 63 (V of keys past the position zeroed)
      if (vk) {
        uint4 pf = uint4{0u, 0u, 0u, 0u};
        if (c16 < XG) pf = *reinterpret_cast<const uint4*>(&pb[c16][32 * gv + 8 * h4]);
        const int kbase = CH * c + 32 * gv + 8 * h4;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          uint4 v = vf[dt];
          if (kbase + 8 > nk) {
            uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const uint32_t lo = kbase + 2 * e < nk ? 0x0000ffffu : 0u;
              const uint32_t hi = kbase + 2 * e + 1 < nk ? 0xffff0000u : 0u;
              w[e] &= lo | hi;
            }
            v = uint4{w[0], w[1], w[2], w[3]};
          }
          const f32x4_t ov = mfma16(pf, v, f32x4_t{0.f, 0.f, 0.f, 0.f});
          if (h4 == 0) {
#pragma unroll
            for (int i = 0; i < XG; ++i) opart[gv][i][64 * hv + 16 * dt + c16] = ov[i];
          }
        }
      }
      __syncthreads();
      // (7) the chunk's P.V (groups summed in group order) out as granules, one (head, dim) per thread
      if (t < XG * HD) {
        const int g = t / HD, d = t - g * HD;
        float ov = opart[0][g][d];
#pragma unroll
        for (int w = 1; w < CPG; ++w)
          if (CPG * c + w < n32) ov += opart[w][g][d];
        st_wt64(gx + XC_GO + (c * XG + g) * HD + d, (uint64_t)__float_as_uint(ov) | tag64);
      }
      ZMI_YSTAMP(3);
    }
    // (8) dims 16 c .. + 15 of the unit's output: every chunk's partial, l and M_j, the block recursion of
    // zmi_attn_merge.h; out as attn_out (memory) and {pair, tag} granules to every workgroup
    if (att && t < XG * 16) {
      const int g = t >> 4, d = 16 * c + (t & 15);
      uint64_t ov[XC_CH], lv[XC_CH], mv[XC_CH / CPB];
      unsigned pend = 0;
#pragma unroll
      for (int k = 0; k < XC_CH; ++k)
        if (k < nc) pend |= 3u << (2 * k);
#pragma unroll
      for (int j = 0; j < XC_CH / CPB; ++j)
        if (j * CPB < nc) pend |= 1u << (2 * XC_CH + j);
      for (unsigned spins = 0; pend; ++spins) {
#pragma unroll
        for (int k = 0; k < XC_CH; ++k) {
          if ((pend >> (2 * k)) & 1) ov[k] = ld_wt64(gx + XC_GO + (k * XG + g) * HD + d);
          if ((pend >> (2 * k + 1)) & 1) lv[k] = ld_wt64(gx + XC_GL + k * XG + g);
        }
#pragma unroll
        for (int j = 0; j < XC_CH / CPB; ++j)
          if ((pend >> (2 * XC_CH + j)) & 1) mv[j] = ld_wt64(gx + XC_GB + j * CPB * XG + g);
#pragma unroll
        for (int k = 0; k < XC_CH; ++k) {
          if (((pend >> (2 * k)) & 1) && tag_of(ov[k]) == tag) pend &= ~(1u << (2 * k));
          if (((pend >> (2 * k + 1)) & 1) && tag_of(lv[k]) == tag) pend &= ~(1u << (2 * k + 1));
        }
#pragma unroll
        for (int j = 0; j < XC_CH / CPB; ++j)
          if (((pend >> (2 * XC_CH + j)) & 1) && tag_of(mv[j]) == tag) pend &= ~(1u << (2 * XC_CH + j));
        if (!pend) break;
        if (spins > SPIN) {
          give_up(at.err);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      float acc = 0.f, l = 0.f, ob = 0.f, lb = 0.f, mprev = 0.f, mb = 0.f;
#pragma unroll
      for (int k = 0; k < XC_CH; ++k) {
        if (k >= nc) break;
        const float ok = __uint_as_float((uint32_t)ov[k]), lk = __uint_as_float((uint32_t)lv[k]);
        if (k % CPB == 0) {
          ob = ok;
          lb = lk;
          mb = __uint_as_float((uint32_t)mv[k / CPB]);
        } else {
          ob += ok;
          lb += lk;
        }
        if (k % CPB == CPB - 1 || k == nc - 1) {
          if (k < CPB) {
            acc = ob;
            l = lb;
          } else {
            const float et = expf(mprev - mb);
            l = lb + et * l;
            acc = acc * et + ob;
          }
          mprev = mb;
        }
      }
      const float rl = 1.0f / l;
      const uint32_t hv16 = f2bf(acc * rl);
      const int col = (kh * XG + g) * HD + d;
      if (at.out) at.out[(size_t)qi * at.ldo + col] = (bf16_t)hv16;
      const uint32_t nb = (uint32_t)__shfl_down((int)hv16, 1);
      if ((t & 1) == 0) st_wt64(ogran + (size_t)qi * GPAIRS + (col >> 1), (uint64_t)(hv16 | (nb << 16)) | tag64);
    }
    ZMI_YSTAMP(4);
    if (wave < W) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA pieces of the out_proj slice
      const char* ws = wsl + (size_t)(8 + wave) * NL * 1024 + lane * 16;
      o_tail([&](int j) { return *reinterpret_cast<const u32x4_t*>(ws + j * 1024); }, res_pre, true);
    } else {
      u32x4_t wf[2][NL];
      issue_fc1_f(wf);
      f_tail(wf);
    }
  } else {
    // ---- streaming workgroup: every wave streams its weights from the start (after `delay` x ~0.85 us: the
    // attention workgroups' loads go out first)
    for (int i = 0; i < delay; ++i) __builtin_amdgcn_s_sleep(32);
    if (wave < W) {
      uint32_t res_pre[NE];
      o_operands(res_pre);
      u32x4_t wx[NL];
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wo_src), (short)0, NL * 1024, 0x00020000);
#pragma unroll
      for (int j = 0; j < NL; ++j) wx[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, j * 1024, 2);
      issue_lds(0, 8 + wave);
      ZMI_YSTAMP(1);
      o_tail([&](int j) { return wx[j]; }, res_pre, false);
    } else {
      u32x4_t wf[2][NL];
      issue_fc1_f(wf);
      f_tail(wf);
    }
  }
}

template <int T>
hipError_t launch(const AttnArgs& at, int n_units, const ZmiGemvArgs& o, const ZmiGemvArgs& f, void* xgran, void* ogran,
                  void* rgran, size_t lds, void* stream) {
  const int delay = zmi_option(ZMI_OPT_AF_DELAY);
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_ffn_kernel<T>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)zmi_gemv::LDS_MAX);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(attn_ffn_kernel<T>, dim3(NBLK), dim3(NT), lds, (hipStream_t)stream, at, n_units, o, f,
                     (uint64_t*)xgran, (uint64_t*)ogran, (uint64_t*)rgran, delay);
  return hipGetLastError();
}

}  // namespace

extern "C" int64_t zmi_attn_ffn_gran_words(int rows) { return rows <= 0 ? -1 : (int64_t)rows * GPAIRS; }

extern "C" int zmi_attn_ffn_max_pos(void) { return XC_KEYS - 1; }

extern "C" int zmi_attn_ffn_block(const ZmiGemvArgs* qkv, const ZmiGemvArgs* out_proj, const ZmiGemvArgs* fc1,
                                  void* xgran, void* ogran, void* rgran, unsigned* err, void* attn_out, int ldo,
                                  void* stream) {
  const ZmiGemvArgs& a = *qkv;
  const ZmiGemvArgs& o = *out_proj;
  const ZmiGemvArgs& f = *fc1;
  if (a.hd != HD || a.hkv <= 0 || a.hq != XG * a.hkv || a.hq * a.hd != K)
    return zmi_fail_msg("attn_ffn_block: head_dim 128, 4 query heads per kv head, hq x hd = 2048");
  if (a.M < 1 || a.M * a.hkv > 8 || a.M > 2)
    return zmi_fail_msg("attn_ffn_block: rows x kv heads <= 8 (64 chunk workgroups), rows <= 2");
  if (a.smax % 8 || !a.row_pos || !a.k_cache || !a.v_cache || !a.out || a.ldo % 8)
    return zmi_fail_msg("attn_ffn_block: qkv needs q (out, ldo % 8), the KV caches, row_pos and smax % 8");
  if (o.K != K || o.N != K || o.n_valid != K || f.K != K || f.N != 2048 * 8 || f.n_valid != f.N)
    return zmi_fail_msg("attn_ffn_block: out_proj [2048 x 2048] and fc1 [16384 x 2048] (packed SwiGLU) only");
  if (o.M != a.M || f.M != a.M) return zmi_fail_msg("attn_ffn_block: equal row counts");
  if (o.ln_w || o.pro != ZMI_PRO_AUTO || !f.ln_w || !f.ln_b || f.pro != ZMI_PRO_AUTO)
    return zmi_fail_msg("attn_ffn_block: out_proj plain, fc1 LayerNorm'd");
  if (f.X != o.out || f.ldx != o.ldo) return zmi_fail_msg("attn_ffn_block: fc1 must read the rows out_proj writes");
  if (o.X != attn_out || o.ldx != ldo) return zmi_fail_msg("attn_ffn_block: out_proj must read attn_out");
  if (o.row_pos != a.row_pos) return zmi_fail_msg("attn_ffn_block: out_proj->row_pos must be the rows' positions");
  if (!xgran || !ogran || !rgran || !err || !attn_out || !o.out || !f.out)
    return zmi_fail_msg("attn_ffn_block: missing buffers");
  if (o.ldo % 8 || f.ldo % 4 || ldo % 8) return zmi_fail_msg("attn_ffn_block: row strides");
  if (zmi_cu_count() < NBLK) return zmi_fail_msg("attn_ffn_block: needs 256 CUs (all workgroups resident at once)");
  const size_t lds = std::max(Img::bytes(a.M), zmi_gemv::LDS_MAX / 2 + 1024);  // one workgroup per CU
  if (lds > zmi_gemv::LDS_MAX) return zmi_fail_msg("attn_ffn_block: LDS");
  AttnArgs at{};
  at.q = (const bf16_t*)a.out;
  at.ldq = a.ldo;
  at.k = (const bf16_t*)a.k_cache;
  at.v = (const bf16_t*)a.v_cache;
  at.kv_row = a.row_kv;
  at.pos = a.row_pos;
  at.hkv = a.hkv;
  at.smax = a.smax;
  at.scale = 1.0f / sqrtf((float)HD);
  at.out = (bf16_t*)attn_out;
  at.ldo = ldo;
  at.err = err;
  const int depth = zmi_option(ZMI_OPT_AF_DEPTH);
  hipError_t e;
  switch (depth) {
    case 0: e = launch<0>(at, a.M * a.hkv, o, f, xgran, ogran, rgran, lds, stream); break;
    case 2: e = launch<2>(at, a.M * a.hkv, o, f, xgran, ogran, rgran, lds, stream); break;
    case 3: e = launch<3>(at, a.M * a.hkv, o, f, xgran, ogran, rgran, lds, stream); break;
    case 4: e = launch<4>(at, a.M * a.hkv, o, f, xgran, ogran, rgran, lds, stream); break;
    case 6: e = launch<6>(at, a.M * a.hkv, o, f, xgran, ogran, rgran, lds, stream); break;
    default: return zmi_fail_msg("attn_ffn_block: ZMI_OPT_AF_DEPTH must be 0, 2, 3, 4 or 6");
  }
  ZMI_CHECK(e);
  return 0;
}
