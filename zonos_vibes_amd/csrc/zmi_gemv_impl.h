// Weight-streaming GEMV / skinny GEMM for the decode step and the prefill, gfx950.
//
// out[m, n] = sum_k A[m, k] * W[n, k]   (nn.Linear, reference zonos/backbone/_torch.py:114-115,147-152,
//                                        heads: zonos/model.py:100-101)
//
// One kernel for every row count M (decode: M = 2 x slots; prefill: M = 2 x prefill length), so a
// row's result never depends on how many rows share the launch (batched output
// must equal the reference's batch_size=1 output, model.py:194):
//
//  * a workgroup owns G groups of 8 output columns over the WHOLE K, and a tile of RT rows;
//    W waves per group split K into fixed segments; every lane issues all of its weight loads
//    (NL x 16 B, straight into VGPRs) before it needs the first one. Row tiles of one column
//    block re-read the weights (from L2 when they run together: the block -> tile map below puts
//    them on one XCD, consecutive in dispatch order; speed only, never correctness).
//  * the products run on MFMA v_mfma_f32_16x16x32_bf16 with 8 real columns per 16-column tile:
//    lane l of a 1 KiB weight chunk holds column 8g + (l & 7) at k = 64 kc + 32 ((l >> 3) & 1) +
//    8 (l >> 4) .. +7 (layout "M8", zmi_pack_weight). Against the activation k-half 0 the
//    tile's columns 0..7 are exact partial sums, against k-half 1 its columns 8..15 are; the
//    other half of each tile is discarded. Each chunk therefore costs two MFMAs and no lane
//    movement, and a tile carries up to 16 rows for the same cost as one.
//  * fixed reduction order, independent of M and of the tile a row lands in: per wave a
//    chain of MFMAs over its k-segment (k-half 0 and k-half 1 in two accumulators), their sum,
//    then the W segment sums in wave order.
//  * optional LayerNorm prologue (nn.LayerNorm, _torch.py:62,88,90): (row, part) tasks over the waves, fp32
//    two-pass statistics, bf16-rounded output, the same arithmetic for every row.
//  * fused epilogues: bf16 store, residual add, RoPE + KV-cache write, SwiGLU, logits, raw f32.
#pragma once
#include <algorithm>
#include "zmi_common.h"
#include "zmi_kernels.h"

namespace zmi_gemv {

constexpr int PRO_PLAIN = 0, PRO_LN = 1, PRO_ADDLN = 2, PRO_GRMS = 3;
// GRMSG: RMSNormGated from aux rows that already hold g = y * gate (f32): no y rows staged (zmi_mamba_block's step
// writes g; the same bits as GRMS, one third fewer activation bytes per workgroup)
constexpr int PRO_GRMSG = 4;
constexpr size_t LDS_MAX = 160 * 1024;  // gfx950 LDS per workgroup

// DPP row_ror:8 — lane i of each 16-lane row reads lane (i + 8) & 15 of the same row
__device__ __forceinline__ float ror8(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
}

__device__ __forceinline__ void dma_piece(const bf16_t* gsrc, bf16_t* ldp) {
  // one 1 KiB LDS-DMA piece (64 lanes x 16 B, lane-linear). Inline asm: the compiler does not
  // count it, so the covering wait is the explicit vmcnt after the weight loads
  // (cdna_hip_programming.md §5.7).
  const unsigned ldst =
      __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) void*)ldp);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(ldst)
               : "memory");
}

// LDS image: rows of x at a stride of K + 8 bf16 (2K + 16 bytes: the 16 rows of an MFMA
// A-fragment read fall on distinct 16-byte bank slots), the aux rows (ADDLN residual / GRMS z) at the
// same stride, gamma (/ beta), then the segment sums.
template <int K>
struct Img {
  static constexpr int XROW = K + 8;
  static constexpr int GROW = K + 8;  // f32 gate rows (GRMS)
  static size_t bytes(int rows, int nwv, int rt, int pro) {
    const bool grms = pro == PRO_GRMS || pro == PRO_GRMSG;
    const size_t gb = (pro == PRO_LN || pro == PRO_ADDLN) ? (size_t)4 * K : (grms ? (size_t)2 * K : 0);
    const size_t aux = pro == PRO_ADDLN ? (size_t)rows * XROW * 2 : (grms ? (size_t)rows * GROW * 4 : 0);
    return (size_t)rows * XROW * 2 + aux + gb + (size_t)nwv * 8 * rt * 4;
  }
};

// fp32 sum of one 8-element chunk of x + aux (ADDLN: layer_norm_fn's fp32 residual sum), or of its
// squared deviations; pairs added as (a + b), the order of ln_chunk_sum and zmi_add_layernorm
__device__ __forceinline__ float addln_chunk_sum(const uint4& hv, const uint4& rv, float mean, bool sq) {
  const uint32_t h[4] = {hv.x, hv.y, hv.z, hv.w}, r[4] = {rv.x, rv.y, rv.z, rv.w};
  float t = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float s0 = bf2f(h[j]) + bf2f(r[j]), s1 = bf2f(h[j] >> 16) + bf2f(r[j] >> 16);
    if (sq) {
      const float d0 = s0 - mean, d1 = s1 - mean;
      t += d0 * d0 + d1 * d1;
    } else {
      t += s0 + s1;
    }
  }
  return t;
}
// RMSNormGated's g = y * gate of element e of a chunk (fp32; gate = z * sigmoid(z), zmi_mamba2_step), the
// value zmi_gated_rmsnorm forms as y * (z * sigmoid(z))
__device__ __forceinline__ float gate_elem(const uint32_t (&y)[4], const float (&gz)[8], int e) {
  return bf2f(y[e >> 1] >> (16 * (e & 1))) * gz[e];
}
__device__ __forceinline__ void load_gate(const float* p, float (&gz)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  gz[0] = a.x; gz[1] = a.y; gz[2] = a.z; gz[3] = a.w; gz[4] = b.x; gz[5] = b.y; gz[6] = b.z; gz[7] = b.w;
}

// Diagnostic build only (-DZMI_GEMV_STAMPS, tools/gemv_stamps.py): thread 0 of every workgroup
// writes s_memrealtime (100 MHz) at phase boundaries into diag[reserved][block][8].
#ifdef ZMI_GEMV_STAMPS
#define ZMI_GSTAMP(i)                                                                              \
  do {                                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                                             \
    if (threadIdx.x == 0 && a.diag)                                                                \
      reinterpret_cast<unsigned long long*>(a.diag)[((size_t)a.reserved * 4096 + blockIdx.x) * 8 + (i)] = \
          __builtin_amdgcn_s_memrealtime();                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                             \
  } while (0)
#else
#define ZMI_GSTAMP(i) \
  do {                \
  } while (0)
#endif

// In-launch hand-off of the QKV projection to the attention workgroups of zmi_attn_block
// (zmi_attnblk.hip): every bf16 pair of q and of this step's K / V rows is ALSO stored as an 8-byte
// {pair, tag = position + 1} granule (one sc1 store: the data is its own flag, cdna_hip_programming.md
// §6 Guideline 16 R2), so the consumer needs no counter and nothing is re-armed.
// Per query row and kv head the granule area holds QKV_GRAN words: q of the G heads (G HD / 2 pairs),
// then k (HD / 2) and v (HD / 2); the score granules follow (zmi_attnblk.hip).
struct QkvFuse {
  uint64_t* gran;   // [M][hkv][gran_stride] u64
  int gran_stride;
  // FUSE == 3 (zmi_attn_block's out_proj role): the GEMV's activation rows are the attention output, gathered
  // from the units' output granules (word og_off of a unit's area: 256 {bf16 pair, tag} words, dims in order)
  // once the unit's 8 merge-workgroup flags (word of_off + c: {0, tag}) carry the row's tag (position + 1)
  int og_off = 0, of_off = 0, hkv = 0;
  const int* pos = nullptr;
  unsigned* err = nullptr;
  // FUSE == 2 (zmi_mamba_block's in_proj role): granules of columns < l2_cols are stored workgroup-scope, kept in
  // the XCD's L2 for a step workgroup on the same XCD (st_xc64); the others write through
  int l2_cols = 0;
};

// (6) fused epilogues of one group's 8 columns over a row tile, run by one wave; colsum(c, r) = the
// group's finished column sum. Shared by every launch form (gemv_body, gemm_rows_kernel): the same bits.
template <int EPI, int RT, int FUSE, class ColSum>
__device__ __forceinline__ void epilogue(const ZmiGemvArgs& a, const ColSum& colsum, int lane, int rows, int row0,
                                         int g, const uint32_t (&res_pre)[(8 * RT + 63) / 64], int q_pos, int q_kvr,
                                         const QkvFuse& fz, unsigned act_rows = ~0u, const float2* rope_pre = nullptr) {
  constexpr int NE = (8 * RT + 63) / 64;
  const int col0 = g * 8;
  if (EPI == ZMI_EPI_STORE && FUSE == 2) {
    // plain bf16 store, and every column pair of an active row also goes out as an 8-byte {pair,
    // tag = position + 1} granule (zmi_mamba_block's step role reads the in_proj output from these)
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = lane + 64 * i, r = e >> 3, c = e & 7, n = col0 + c;
      const bool ok = r < rows && n < a.n_valid;
      const uint32_t hv = ok ? f2bf(colsum(c, r)) : 0u;
      const uint32_t nb = (uint32_t)__shfl_down((int)hv, 1);
      if (ok) {
        const size_t m = (size_t)(row0 + r);
        reinterpret_cast<bf16_t*>(a.out)[m * a.ldo + n] = (bf16_t)hv;
        const int pos = a.row_pos[m];
        if ((c & 1) == 0 && pos >= 0)
          st_xc64(fz.gran + m * fz.gran_stride + (n >> 1), (uint64_t)(hv | (nb << 16)) | ((uint64_t)(unsigned)(pos + 1) << 32),
                  n < fz.l2_cols);
      }
    }
  } else if (EPI == ZMI_EPI_STORE || EPI == ZMI_EPI_RESIDUAL || EPI == ZMI_EPI_F32 || EPI == ZMI_EPI_LOGITS) {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = lane + 64 * i, r = e >> 3, c = e & 7, n = col0 + c;
      if (r >= rows || n >= a.n_valid || !((act_rows >> r) & 1u)) continue;  // act_rows: FUSE 3's rows with pos >= 0
      const float v = colsum(c, r);
      const size_t m = (size_t)(row0 + r);
      if (EPI == ZMI_EPI_F32) {
        reinterpret_cast<float*>(a.out)[m * a.ldo + n] = v;
      } else if (EPI == ZMI_EPI_STORE) {
        reinterpret_cast<bf16_t*>(a.out)[m * a.ldo + n] = (bf16_t)f2bf(v);
      } else if (EPI == ZMI_EPI_RESIDUAL) {
        // x + bf16(linear(x))  (_torch.py:100-101)
        reinterpret_cast<bf16_t*>(a.out)[m * a.ldo + n] = (bf16_t)f2bf(bf2f(res_pre[i]) + bfround(v));
      } else {
        // 9 heads back to back, 1026 columns each (1025 real + the zero pad row)
        const int cbk = n / 1026, vv = n - cbk * 1026;
        reinterpret_cast<float*>(a.out)[(m * 9 + cbk) * 1026 + vv] = bfround(v);
      }
    }
  } else if (EPI == ZMI_EPI_SWIGLU) {
    // M8 SwiGLU packing: columns 0..3 = value rows 4g.., 4..7 = gate rows F + 4g..  (_torch.py:150-152)
    const int r = lane >> 2, c = lane & 3;
    if (r < rows) {
      const float y = bfround(colsum(c, r));
      const float gt = bfround(colsum(c + 4, r));
      const float sg = bfround(gt / (1.0f + expf(-gt)));
      reinterpret_cast<bf16_t*>(a.out)[(size_t)(row0 + r) * a.ldo + g * 4 + c] = (bf16_t)f2bf(y * sg);
    }
  } else if (EPI == ZMI_EPI_QKV) {
    // q | k | v split, interleaved-pair RoPE in fp32 on q and k, KV-cache write (_torch.py:18-49,117-126)
    const int r = lane >> 2, c = (lane & 3) * 2;
    if (r < rows && q_pos >= 0 && q_pos < a.smax) {  // the launchers check positions against smax; never write past it
      const int n = col0 + c;
      const int qcols = a.hq * a.hd, kcols = a.hkv * a.hd;
      float x0 = bfround(colsum(c, r)), x1 = bfround(colsum(c + 1, r));
      if (n < qcols + kcols) {
        const int d = (n < qcols ? n : n - qcols) % a.hd;
        // rope_pre: the cos / sin pair loaded by the caller before its LayerNorm (a load here is a memory round trip on
        // the decode step's critical path)
        const float2 cs = rope_pre ? *rope_pre
                                   : *reinterpret_cast<const float2*>(a.rope + ((size_t)q_pos * (a.hd >> 1) + (d >> 1)) * 2);
        const float co = cs.x, si = cs.y;
        const float r0 = x0 * co - x1 * si;
        const float r1 = x1 * co + x0 * si;
        x0 = r0;
        x1 = r1;
      }
      const uint32_t packed = f2bf(x0) | (f2bf(x1) << 16);
      int gkh = 0, gslot = 0;  // granule of this pair (FUSE)
      if (n < qcols) {
        *reinterpret_cast<uint32_t*>(reinterpret_cast<bf16_t*>(a.out) + (size_t)(row0 + r) * a.ldo + n) = packed;
        const int gq = a.hq / a.hkv;
        gkh = n / (gq * a.hd);
        gslot = (n - gkh * gq * a.hd) >> 1;
      } else if (n < qcols + kcols) {  // K cache [row][kv head][position][hd]
        const int nn = n - qcols, kh = nn / a.hd, d = nn - kh * a.hd;
        const size_t o = (((size_t)q_kvr * a.hkv + kh) * a.smax + q_pos) * a.hd + d;
        *reinterpret_cast<uint32_t*>(reinterpret_cast<bf16_t*>(a.k_cache) + o) = packed;
        gkh = kh;
        gslot = (a.hq / a.hkv) * (a.hd >> 1) + (d >> 1);
      } else {  // V cache, transposed: [row][kv head][hd][position] (zmi_attn.hip's P.V operand)
        const int nn = n - qcols - kcols, kh = nn / a.hd, d = nn - kh * a.hd;
        bf16_t* vt = reinterpret_cast<bf16_t*>(a.v_cache) + (((size_t)q_kvr * a.hkv + kh) * a.hd + d) * a.smax + q_pos;
        vt[0] = (bf16_t)(packed & 0xffffu);
        vt[a.smax] = (bf16_t)(packed >> 16);
        gkh = kh;
        gslot = (a.hq / a.hkv + 1) * (a.hd >> 1) + (d >> 1);
      }
      if (FUSE)
        st_wt64(fz.gran + ((size_t)(row0 + r) * a.hkv + gkh) * fz.gran_stride + gslot,
                (uint64_t)packed | ((uint64_t)(unsigned)(q_pos + 1) << 32));
    }
  }
}

template <int G, int W, int NL, int RT, int PRO, int EPI, int NTW, int FUSE = 0>
__device__ __forceinline__ void gemv_body(const ZmiGemvArgs& a, int n_cb, int n_rt, int b, char* smem,
                                          const QkvFuse& fz, int rpw = 1) {
  constexpr int K = W * NL * 64;
  constexpr int KC = K / 64;
  constexpr int NWV = G * W;
  constexpr int XROW = Img<K>::XROW;
  static_assert(RT == 8 || RT == 16, "row tile");
  static_assert(!FUSE || EPI == ZMI_EPI_QKV || EPI == ZMI_EPI_STORE || FUSE == 3, "in-launch hand-off: QKV or plain store");
  static_assert(FUSE != 2 || NTW, "the store hand-off runs on single-tile (decode) launches");
  static_assert(FUSE != 3 || (NTW && (EPI == ZMI_EPI_RESIDUAL || EPI == ZMI_EPI_STORE) && PRO == PRO_PLAIN && K == 2048 &&
                              RT == 16),
                "the gathered-input form is zmi_attn_block's out_proj role (one tile, plain, residual or store epilogue)");

  // block -> (column block, group of rpw row tiles): the groups of one column block take ids 8 apart.
  // A workgroup keeps its weight slice in registers and runs its row tiles one after the other, each
  // with the arithmetic of a lone tile (a row's result does not depend on rpw or M).
  const int idx = b >> 3;
  const int n_rg = (n_rt + rpw - 1) / rpw;
  const int cb = (idx / n_rg) * 8 + (b & 7), rg = idx - (idx / n_rg) * n_rg;
  if (cb >= n_cb) return;  // padding block: exits before any barrier
  ZMI_GSTAMP(0);
  const int alloc_rows = a.M < RT ? a.M : RT;
  int rt = rg * rpw;
  const int rt_end = min(n_rt, rt + rpw);
  int row0 = rt * RT;
  int rows = min(RT, a.M - row0);
  constexpr bool GRMS = PRO == PRO_GRMS || PRO == PRO_GRMSG;
  constexpr bool AUX = PRO == PRO_ADDLN || GRMS;
  constexpr int GB = (PRO == PRO_LN || PRO == PRO_ADDLN) ? 2 : (GRMS ? 1 : 0);  // gamma / beta rows
  constexpr int GROW = Img<K>::GROW;
  bf16_t* xs = reinterpret_cast<bf16_t*>(smem);
  bf16_t* xa = xs + (size_t)alloc_rows * XROW;  // aux rows: ADDLN bf16 residual, GRMS f32 gate
  float* xg = reinterpret_cast<float*>(xa);
  bf16_t* gam = xa + (PRO == PRO_ADDLN ? (size_t)alloc_rows * XROW : (GRMS ? (size_t)alloc_rows * GROW * 2 : 0));
  bf16_t* bet = gam + K;
  float* red = reinterpret_cast<float*>(gam + (size_t)GB * K);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR descriptors, no waterfalls
  const int gi = wave / W, wk = wave - gi * W;
  const int ngroups = a.N >> 3;
  const int g_raw = cb * G + gi;
  const bool g_ok = g_raw < ngroups;
  const int g = g_ok ? g_raw : ngroups - 1;  // clamped: every wave joins the barriers
  const int col0 = g * 8;
  const bf16_t* X = reinterpret_cast<const bf16_t*>(a.X) + (size_t)row0 * a.ldx;
  // epilogue operands that need no other load (older than the weights: covered by the vmcnt below).
  // The group's first wave runs the epilogue; its lane handles outputs e = lane + 64 i.
  const bool ew = (wk == 0) && g_ok;
  constexpr int NE = (8 * RT + 63) / 64;
  uint32_t res_pre[NE];
  int q_pos = -1, q_kvr = 0;
  unsigned act_rows = ~0u;  // FUSE 3: rows whose position is >= 0 (the others ran no attention: no residual store)

  // (1) activation rows (+ LayerNorm gamma / beta, first tile only) into LDS by DMA, 1 KiB pieces
  // spread over waves; then the tile's epilogue operands
  // the DMA of a tile's rows (s_row0, s_rows, s_X) is split from its epilogue operands: in the multi-tile
  // loop the next tile's rows are issued as soon as every wave's MFMA chain has left the LDS image, under
  // the current tile's reduction and epilogue
  auto stage_rows = [&](bool first, int s_row0, int s_rows, const bf16_t* s_X) {
    constexpr int PPR = K / 512;
    const int n_x = PRO == PRO_GRMSG ? 0 : s_rows * PPR;  // GRMSG: no y rows
    constexpr int APR = GRMS ? 2 * PPR : PPR;  // aux pieces per row (f32 gate rows: twice the bytes)
    const int n_a = AUX ? s_rows * APR : 0;
    const int n_pc = n_x + n_a + (first ? GB * PPR : 0);
    const bf16_t* XA = AUX ? reinterpret_cast<const bf16_t*>(a.aux) + (size_t)s_row0 * a.ld_aux * (GRMS ? 2 : 1)
                           : nullptr;
    for (int pc = wave; pc < n_pc; pc += NWV) {
      if (pc < n_x) {
        const int r = pc / PPR, p = pc - r * PPR;
        dma_piece(s_X + (size_t)r * a.ldx + p * 512 + lane * 8, xs + r * XROW + p * 512);
      } else if (pc < n_x + n_a) {
        const int r = (pc - n_x) / APR, p = (pc - n_x) - r * APR;
        if (GRMS)  // 1 KiB = 256 f32 of the gate (GRMSG: g) row
          dma_piece(XA + ((size_t)r * a.ld_aux + p * 256) * 2 + lane * 8,
                    reinterpret_cast<bf16_t*>(xg + r * GROW + p * 256));
        else
          dma_piece(XA + (size_t)r * a.ld_aux + p * 512 + lane * 8, xa + r * XROW + p * 512);
      } else {
        const int q = pc - n_x - n_a, which = q / PPR, p = q - which * PPR;
        const bf16_t* src = reinterpret_cast<const bf16_t*>(which ? a.ln_b : a.ln_w);
        dma_piece(src + p * 512 + lane * 8, (which ? bet : gam) + p * 512);
      }
    }
  };
  auto stage_epi = [&]() {
#pragma unroll
    for (int i = 0; i < NE; ++i) res_pre[i] = 0;
    q_pos = -1;
    q_kvr = 0;
    if (EPI == ZMI_EPI_RESIDUAL && ew) {
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const int e = lane + 64 * i, r = e >> 3, n = col0 + (e & 7);
        if (r < rows && n < a.n_valid)
          res_pre[i] = reinterpret_cast<const bf16_t*>(a.out)[(size_t)(row0 + r) * a.ldo + n];
      }
    }
    if (EPI == ZMI_EPI_QKV && ew && (lane >> 2) < rows) {
      q_pos = a.row_pos[row0 + (lane >> 2)];
      q_kvr = a.row_kv[row0 + (lane >> 2)];
    }
  };
  if (FUSE != 3) stage_rows(true, row0, rows, X);  // FUSE 3: the rows come from the attention's granules (below)
  stage_epi();
  __builtin_amdgcn_sched_barrier(0);
  // (2) the whole weight slice of this lane, in flight at once: one buffer descriptor per wave
  // (wave-uniform base), lane offset in the VGPR, chunk offset j KiB folded into the instruction
  // (cdna_hip_programming.md T8). Non-temporal when each weight is read once (one row tile).
  const char* wbase = reinterpret_cast<const char*>(a.W) + ((size_t)g * KC + wk * NL) * 1024;
  const __amdgpu_buffer_rsrc_t wrsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wbase), (short)0, NL * 1024, 0x00020000);
  u32x4_t wf[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) wf[j] = __builtin_amdgcn_raw_buffer_load_b128(wrsrc, lane * 16, j * 1024, NTW ? 2 : 0);
  __builtin_amdgcn_sched_barrier(0);
  ZMI_GSTAMP(1);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NL) : "memory");  // DMA pieces + epilogue operands landed
  // single-tile QKV launches (every decode step): the epilogue's RoPE cos / sin pair, issued now that the row's
  // position has landed, so it arrives under the LayerNorm and the MFMA chain instead of after them
  float2 rope_cs = {1.f, 0.f};
  if (EPI == ZMI_EPI_QKV && NTW && ew && (lane >> 2) < rows && q_pos >= 0 && q_pos < a.smax) {
    const int n = col0 + (lane & 3) * 2, qcols = a.hq * a.hd;
    if (n < qcols + a.hkv * a.hd) {
      const int d = (n < qcols ? n : n - qcols) % a.hd;
      rope_cs = *reinterpret_cast<const float2*>(a.rope + ((size_t)q_pos * (a.hd >> 1) + (d >> 1)) * 2);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (FUSE == 3) {
    // the rows' positions (tags) in LDS first: every later check reads them without a dependent global load
    int* qpos = reinterpret_cast<int*>(red);  // the segment-sum area, free until the MFMA chain
    if (tid < rows) qpos[tid] = fz.pos[row0 + tid];
    __syncthreads();
    act_rows = 0u;
    for (int r = 0; r < rows; ++r) act_rows |= (qpos[r] >= 0 ? 1u : 0u) << r;
    // (1') wave 0 polls the merge workgroups' flags of the launch's units (8 per (row, kv head); rows whose position
    // is < 0 run no attention and contribute zero rows), sleeping between sweeps, until a unit has a flag up (below):
    // the merges are then nearly done (64 cheap flags instead of 2048 granules while the attention runs)
    const int n_units = rows * fz.hkv;
#ifndef ZMI_OPROJ_FLAGS
// how long wave 0 waits on the flags before every thread polls its granules: 1 = until ANY unit has a flag up (the
// merges finish within ~0.4 us of each other; a granule published after the sweep is picked up by the next one), 0 =
// until every unit has one (a flag round trip, then a granule round trip: C2 step 922 us against 902-904 with 1),
// 2 = no wait (every thread polls from dispatch: 908) (profiles/r06_oproj_flag_wait_ab.jsonl)
#define ZMI_OPROJ_FLAGS 1
#endif
#ifndef ZMI_OPROJ_SLEEP
#define ZMI_OPROJ_SLEEP 1
#endif
    if (wave == 0 && ZMI_OPROJ_FLAGS != 2) {
      for (unsigned spins = 0;; ++spins) {
        bool ok = ZMI_OPROJ_FLAGS == 0;
        for (int u0 = 0; u0 < n_units; u0 += 8) {  // lane = (unit u0 + lane / 8, merge workgroup lane % 8)
          const int u = u0 + (lane >> 3), qp = u < n_units ? qpos[u / fz.hkv] : -1;
          const bool up = qp < 0 || (uint32_t)(ld_wt64(fz.gran + (size_t)(row0 * fz.hkv + u) * fz.gran_stride + fz.of_off +
                                                          (lane & 7)) >> 32) == (uint32_t)qp + 1u;
          // any flag of the unit: OR over the 8 lanes of the unit (DPP within each 8-lane group)
          float f = up ? 1.f : 0.f;
          f = fmaxf(f, dpp_mov<DPP_XOR1>(f));
          f = fmaxf(f, dpp_mov<DPP_XOR2>(f));
          f = fmaxf(f, dpp_mov<DPP_HALF_MIRROR>(f));
          if (ZMI_OPROJ_FLAGS == 0)
            ok = ok && f > 0.f;
          else
            ok = ok || (u < n_units && f > 0.f);
        }
        if (ZMI_OPROJ_FLAGS == 0 ? __all(ok) : __any(ok)) break;
        if (spins > (1u << 18)) {
          if (lane == 0) __hip_atomic_store(fz.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    ZMI_GSTAMP(7);
    __syncthreads();
    // (2') every thread polls its own {pair, tag} granules of the units' outputs (unit (r, kh), pair j: dims
    // kh hq/hkv hd + 2 j, + 1 of row r; a unit's output is 4 heads x 128 dims = 512 columns of K: the attention block
    // checks hq = 4 hkv, hd = 128) until each carries its row's tag, then writes them into the LDS rows. GB granules
    // per thread per batch (2 rows x 4 kv heads: one batch), every load of a sweep issued before the first check.
    constexpr int GB = 4;
    for (int e0 = tid; e0 < n_units * 256; e0 += GB * NWV * 64) {
      uint64_t gv[GB];
      int gq[GB];
      unsigned need = 0;
#pragma unroll
      for (int i = 0; i < GB; ++i) {
        const int e = e0 + NWV * 64 * i;
        gq[i] = e < n_units * 256 ? qpos[(e >> 8) / fz.hkv] : -1;
        gv[i] = 0ull;
        if (gq[i] >= 0) need |= 1u << i;
      }
      for (unsigned spins = 0; need; ++spins) {
#pragma unroll
        for (int i = 0; i < GB; ++i)
          if ((need >> i) & 1)
            gv[i] = ld_wt64(fz.gran + (size_t)(row0 * fz.hkv + ((e0 + NWV * 64 * i) >> 8)) * fz.gran_stride + fz.og_off +
                            ((e0 + NWV * 64 * i) & 255));
#pragma unroll
        for (int i = 0; i < GB; ++i)
          if (((need >> i) & 1) && (uint32_t)(gv[i] >> 32) == (uint32_t)gq[i] + 1u) need &= ~(1u << i);
        if (!need) break;
        if (spins > (1u << 18)) {
          __hip_atomic_store(fz.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(ZMI_OPROJ_SLEEP);
      }
#pragma unroll
      for (int i = 0; i < GB; ++i) {
        const int e = e0 + NWV * 64 * i;
        if (e < n_units * 256) {
          const int u = e >> 8, j = e & 255, r = u / fz.hkv, kh = u - r * fz.hkv;
          *reinterpret_cast<uint32_t*>(xs + r * XROW + kh * 512 + 2 * j) = gq[i] >= 0 ? (uint32_t)gv[i] : 0u;
        }
      }
    }
  }
  for (;;) {  // the workgroup's row tiles
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  ZMI_GSTAMP(2);

  // (3) LayerNorm (zmi_common.h arithmetic): task (row, part) per wave, so the few rows of a decode
  // step use every wave; partial sums meet in the segment-sum area (free until the MFMA chain).
  // Each pass re-reads its chunks from LDS (no row copy in VGPRs: the weight slice in flight
  // already holds 4 NL of them, and occupancy decides whether every workgroup of a wide GEMV is
  // resident at once).
#ifndef ZMI_LN_ROWWAVE  // (row, part) tasks spread over the waves, barriers between the passes; the A/B build
                        // -DZMI_LN_ROWWAVE (one wave per row, no barriers) measured slower: C2 step 1001 vs 973 us
  if (PRO == PRO_LN) {
    constexpr int NQ = ln_parts(K), CPQ = K / (512 * NQ);
    float* part = red;
    const int ntask = rows * NQ;
    auto pass = [&](int task, float mean, bool sq) {
      const int r = task / NQ, q = task - r * NQ;
      const bf16_t* xr = xs + r * XROW + q * (K / NQ);
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < CPQ; ++i) t += ln_chunk_sum(*reinterpret_cast<const uint4*>(xr + (lane + 64 * i) * 8), mean, sq);
      return wave_sum(t);
    };
    for (int task = wave; task < ntask; task += NWV) {
      const float v = pass(task, 0.f, false);
      if (lane == 0) part[task] = v;
    }
    __syncthreads();
#if defined(ZMI_LN_STAMP) && ZMI_LN_STAMP == 1  // diagnostic builds only (tools/build_attnblk_stamps.sh)
    ZMI_GSTAMP(7);
#endif
    for (int task = wave; task < ntask; task += NWV) {
      const float mean = ln_combine<NQ>(part + (task / NQ) * NQ) / (float)K;
      const float v = pass(task, mean, true);
      if (lane == 0) part[RT * NQ + task] = v;
    }
    __syncthreads();
#if defined(ZMI_LN_STAMP) && ZMI_LN_STAMP == 2
    ZMI_GSTAMP(7);
#endif
    for (int task = wave; task < ntask; task += NWV) {
      const int r = task / NQ, q = task - r * NQ;
      const float mean = ln_combine<NQ>(part + r * NQ) / (float)K;
      const float rstd = 1.0f / sqrtf(ln_combine<NQ>(part + RT * NQ + r * NQ) / (float)K + a.eps), nbias = -mean * rstd;
      bf16_t* xr = xs + r * XROW + q * (K / NQ);
#pragma unroll
      for (int i = 0; i < CPQ; ++i) {
        const int c = q * (K / NQ) / 8 + lane + 64 * i;
        const uint4 xv = *reinterpret_cast<const uint4*>(xr + (lane + 64 * i) * 8);
        *reinterpret_cast<uint4*>(xr + (lane + 64 * i) * 8) = ln_apply(
            xv, *reinterpret_cast<const uint4*>(gam + c * 8), *reinterpret_cast<const uint4*>(bet + c * 8), rstd, nbias);
      }
    }
    __syncthreads();
  }
#else
  if (PRO == PRO_LN) {
    // one wave per row: the row's NQ part sums (each the wave_sum of its lanes' chunk sums, as
    // zmi_layernorm_rows forms them) are all held by that wave, so the three passes need no workgroup
    // barrier; the row's own LDS writes and reads are ordered within the wave
    constexpr int NQ = ln_parts(K), CPQ = K / (512 * NQ);
    for (int r = wave; r < rows; r += NWV) {
      bf16_t* xr = xs + r * XROW;
      auto pass = [&](float mean, bool sq, float(&ps)[NQ]) {
        float tq[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          tq[q] = 0.f;
#pragma unroll
          for (int i = 0; i < CPQ; ++i)
            tq[q] += ln_chunk_sum(*reinterpret_cast<const uint4*>(xr + q * (K / NQ) + (lane + 64 * i) * 8), mean, sq);
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) ps[q] = wave_sum(tq[q]);
      };
      float ps[NQ];
      pass(0.f, false, ps);
      const float mean = ln_combine<NQ>(ps) / (float)K;
      pass(mean, true, ps);
      const float rstd = 1.0f / sqrtf(ln_combine<NQ>(ps) / (float)K + a.eps), nbias = -mean * rstd;
#pragma unroll
      for (int q = 0; q < NQ; ++q)
#pragma unroll
        for (int i = 0; i < CPQ; ++i) {
          const int c = q * (K / NQ) / 8 + lane + 64 * i;
          bf16_t* xc = xr + q * (K / NQ) + (lane + 64 * i) * 8;
          const uint4 xv = *reinterpret_cast<const uint4*>(xc);
          *reinterpret_cast<uint4*>(xc) = ln_apply(xv, *reinterpret_cast<const uint4*>(gam + c * 8),
                                                   *reinterpret_cast<const uint4*>(bet + c * 8), rstd, nbias);
        }
    }
    __syncthreads();
  }
#endif
  if (PRO == PRO_ADDLN) {
    // layer_norm_fn prenorm: s = x + residual (fp32), LayerNorm(s) with (s - mean) rstd w + b; the column
    // block 0 workgroup of each row tile writes bf16(s), the next block's residual
    constexpr int NQ = ln_parts(K), CPQ = K / (512 * NQ);
    float* part = red;
    const int ntask = rows * NQ;
    auto pass = [&](int task, float mean, bool sq) {
      const int r = task / NQ, q = task - r * NQ;
      const bf16_t* hr = xs + r * XROW + q * (K / NQ);
      const bf16_t* rr = xa + r * XROW + q * (K / NQ);
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < CPQ; ++i)
        t += addln_chunk_sum(*reinterpret_cast<const uint4*>(hr + (lane + 64 * i) * 8),
                             *reinterpret_cast<const uint4*>(rr + (lane + 64 * i) * 8), mean, sq);
      return wave_sum(t);
    };
    for (int task = wave; task < ntask; task += NWV) {
      const float v = pass(task, 0.f, false);
      if (lane == 0) part[task] = v;
    }
    __syncthreads();
    for (int task = wave; task < ntask; task += NWV) {
      const int r = task / NQ;
      const float mean = ln_combine<NQ>(part + r * NQ) / (float)K;
      const float v = pass(task, mean, true);
      if (lane == 0) part[RT * NQ + task] = v;
    }
    __syncthreads();
    const bool wres = a.res_out != nullptr && cb == 0;
    for (int task = wave; task < ntask; task += NWV) {
      const int r = task / NQ, q = task - r * NQ;
      const float mean = ln_combine<NQ>(part + r * NQ) / (float)K;
      const float rstd = 1.0f / sqrtf(ln_combine<NQ>(part + RT * NQ + r * NQ) / (float)K + a.eps);
      bf16_t* hr = xs + r * XROW + q * (K / NQ);
      const bf16_t* rr = xa + r * XROW + q * (K / NQ);
#pragma unroll
      for (int i = 0; i < CPQ; ++i) {
        const int c = q * (K / NQ) / 8 + lane + 64 * i;
        const uint4 hv = *reinterpret_cast<const uint4*>(hr + (lane + 64 * i) * 8);
        const uint4 rv = *reinterpret_cast<const uint4*>(rr + (lane + 64 * i) * 8);
        const uint4 gw = *reinterpret_cast<const uint4*>(gam + c * 8), gbv = *reinterpret_cast<const uint4*>(bet + c * 8);
        const uint32_t h[4] = {hv.x, hv.y, hv.z, hv.w}, rs[4] = {rv.x, rv.y, rv.z, rv.w};
        const uint32_t uw[4] = {gw.x, gw.y, gw.z, gw.w}, ub[4] = {gbv.x, gbv.y, gbv.z, gbv.w};
        uint32_t o[4], so[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float s0 = bf2f(h[j]) + bf2f(rs[j]), s1 = bf2f(h[j] >> 16) + bf2f(rs[j] >> 16);
          const float y0 = ((s0 - mean) * rstd) * bf2f(uw[j]) + bf2f(ub[j]);
          const float y1 = ((s1 - mean) * rstd) * bf2f(uw[j] >> 16) + bf2f(ub[j] >> 16);
          o[j] = f2bf(y0) | (f2bf(y1) << 16);
          so[j] = f2bf(s0) | (f2bf(s1) << 16);
        }
        *reinterpret_cast<uint4*>(hr + (lane + 64 * i) * 8) = uint4{o[0], o[1], o[2], o[3]};
        if (wres)
          reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.res_out) + (size_t)(row0 + r) * a.ld_aux)[c] =
              uint4{so[0], so[1], so[2], so[3]};
      }
    }
    __syncthreads();
  }
  if (GRMS) {
    // RMSNormGated (norm_before_gate=False): g = y (z sigmoid(z)), out = g rstd w; g recomputed in the
    // apply pass (the same bits), sums of g^2 element by element as zmi_gated_rmsnorm. A wave takes its
    // (row, part) tasks two at a time (the second clamped, its results dropped): two independent dependent-add
    // chains in one straight-line body instead of one after the other (the K = 4096 out_proj has 4 waves for
    // 2 rows x 4 parts)
    constexpr int NQ = ln_parts(K), CPQ = K / (512 * NQ);
    float* part = red;
    const int ntask = rows * NQ;
    for (int task0 = wave; task0 < ntask; task0 += 2 * NWV) {
      float t[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int task = min(task0 + u * NWV, ntask - 1);
        const int r = task / NQ, q = task - r * NQ;
        const bf16_t* yr = xs + r * XROW + q * (K / NQ);
        const float* zr = xg + r * GROW + q * (K / NQ);
        t[u] = 0.f;
#pragma unroll
        for (int i = 0; i < CPQ; ++i) {
          uint32_t y[4] = {0u, 0u, 0u, 0u};
          if constexpr (PRO == PRO_GRMS) {
            const uint4 yv = *reinterpret_cast<const uint4*>(yr + (lane + 64 * i) * 8);
            y[0] = yv.x; y[1] = yv.y; y[2] = yv.z; y[3] = yv.w;
          }
          float gz[8];
          load_gate(zr + (lane + 64 * i) * 8, gz);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float g = PRO == PRO_GRMSG ? gz[e] : gate_elem(y, gz, e);
            t[u] += g * g;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) t[u] = wave_sum(t[u]);
      if (lane == 0) {
        part[task0] = t[0];
        if (task0 + NWV < ntask) part[task0 + NWV] = t[1];
      }
    }
    __syncthreads();
    for (int task0 = wave; task0 < ntask; task0 += 2 * NWV) {
      uint4 res[2][CPQ];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int task = min(task0 + u * NWV, ntask - 1);
        const int r = task / NQ, q = task - r * NQ;
        const float rstd = 1.0f / sqrtf(ln_combine<NQ>(part + r * NQ) / (float)K + a.eps);
        const bf16_t* yr = xs + r * XROW + q * (K / NQ);
        const float* zr = xg + r * GROW + q * (K / NQ);
#pragma unroll
        for (int i = 0; i < CPQ; ++i) {
          const int c = q * (K / NQ) / 8 + lane + 64 * i;
          uint32_t y[4] = {0u, 0u, 0u, 0u};
          if constexpr (PRO == PRO_GRMS) {
            const uint4 yv = *reinterpret_cast<const uint4*>(yr + (lane + 64 * i) * 8);
            y[0] = yv.x; y[1] = yv.y; y[2] = yv.z; y[3] = yv.w;
          }
          const uint4 gw = *reinterpret_cast<const uint4*>(gam + c * 8);
          const uint32_t uw[4] = {gw.x, gw.y, gw.z, gw.w};
          float gz[8];
          load_gate(zr + (lane + 64 * i) * 8, gz);
          auto gv = [&](int e) { return PRO == PRO_GRMSG ? gz[e] : gate_elem(y, gz, e); };
          uint32_t o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            o[j] = f2bf((gv(2 * j) * rstd) * bf2f(uw[j])) | (f2bf((gv(2 * j + 1) * rstd) * bf2f(uw[j] >> 16)) << 16);
          res[u][i] = uint4{o[0], o[1], o[2], o[3]};
        }
      }
      // stores after both tasks' reads: the clamped duplicate task reads what the real one overwrites
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int task = task0 + u * NWV;
        if (task < ntask) {
          const int r = task / NQ, q = task - r * NQ;
          bf16_t* yr = xs + r * XROW + q * (K / NQ);
#pragma unroll
          for (int i = 0; i < CPQ; ++i) *reinterpret_cast<uint4*>(yr + (lane + 64 * i) * 8) = res[u][i];
        }
      }
    }
    __syncthreads();
  }
  ZMI_GSTAMP(3);

  // (4) MFMA chain over this wave's k-segment. A operand: lane l reads row l & 15 (rows past the
  // tile re-read its last row; those outputs are discarded), k = 8 (l >> 4) .. +7 of the k-half.
  f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  {
    const int ar = min(lane & 15, rows - 1);
    const bf16_t* xa = xs + ar * XROW + wk * NL * 64 + (lane >> 4) * 8;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const uint4 x0 = *reinterpret_cast<const uint4*>(xa + j * 64);
      const uint4 x1 = *reinterpret_cast<const uint4*>(xa + j * 64 + 32);
      const bf16x8_t wv = __builtin_bit_cast(bf16x8_t, wf[j]);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x0), wv, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x1), wv, acc1, 0, 0, 0);
    }
  }
  ZMI_GSTAMP(4);
  // (5) segment sum = k-half 0 (tile columns 0..7) + k-half 1 (tile columns 8..15, moved down by
  // DPP); accumulator element q of lane l is row 4 (l >> 4) + q, column l & 15
  {
    const int c = lane & 15, rb = (lane >> 4) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float v = acc0[q] + ror8(acc1[q]);
      if (c < 8 && rb + q < RT) red[(wave * 8 + c) * RT + rb + q] = v;
    }
  }
  __syncthreads();
  ZMI_GSTAMP(5);
  if (!NTW && rt + 1 < rt_end) {  // every chain is done with the LDS image: the next tile's rows go in now
    const int n_row0 = (rt + 1) * RT;
    stage_rows(false, n_row0, min(RT, a.M - n_row0), reinterpret_cast<const bf16_t*>(a.X) + (size_t)n_row0 * a.ldx);
  }
  if (ew) {
    auto colsum = [&](int c, int r) {  // the group's W segment sums, in wave order
      float v = red[((gi * W) * 8 + c) * RT + r];
#pragma unroll
      for (int w = 1; w < W; ++w) v += red[((gi * W + w) * 8 + c) * RT + r];
      return v;
    };
    epilogue<EPI, RT, FUSE>(a, colsum, lane, rows, row0, g, res_pre, q_pos, q_kvr, fz, act_rows,
                            (EPI == ZMI_EPI_QKV && NTW) ? &rope_cs : nullptr);  // (6)
  }
  ZMI_GSTAMP(6);
  // one tile when each weight is read once (NTW: M <= RT, every decode launch): no loop state there
  if (NTW || ++rt >= rt_end) break;
  __syncthreads();  // every wave is done with this tile's LDS image and segment sums
  row0 = rt * RT;
  rows = min(RT, a.M - row0);
  X = reinterpret_cast<const bf16_t*>(a.X) + (size_t)row0 * a.ldx;
  stage_epi();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this tile's rows (the weights landed long ago)
  }  // row tiles
}

template <int G, int W, int NL, int RT, int PRO, int EPI, int NTW>
__global__ __launch_bounds__(G * W * 64) void gemv_kernel(const ZmiGemvArgs a, int n_cb, int n_rt, int rpw) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  gemv_body<G, W, NL, RT, PRO, EPI, NTW>(a, n_cb, n_rt, blockIdx.x, smem, QkvFuse{nullptr, 0}, rpw);
}

// s_waitcnt vmcnt(n) as the builtin (gfx9 encoding, expcnt / lgkmcnt left at their maxima): unlike an asm
// wait, the compiler's own wait insertion sees it, so loads it covers are not waited for again after
// later (uncounted) LDS-DMA issues
#define ZMI_WAIT_VM(n) __builtin_amdgcn_s_waitcnt(((n) & 15) | (((n) >> 4) << 14) | 0x0F70)

// Many-row form of the K = 2048 GEMV (multi-slot decode and prefill, M > 16), the same per-row arithmetic as
// gemv_body's (W, NL, RT) = (4, 8, 16) shape: a wave's chain of MFMAs over one k-segment (k-half 0 / 1 in
// two accumulators, acc0 + ror8(acc1)), then the 4 segment sums in segment order, then epilogue().
// What changes is the reuse and the pipelining:
//  * a workgroup owns 8 groups (64 columns) and each wave GPW of them over one segment (GPW x 32 weight
//    VGPRs), so every activation tile it stages serves 64 columns (gemv_body's 4-group form: 32, twice the
//    activation traffic per column) and each A fragment read from LDS feeds GPW groups;
//  * the activation tiles (and the epilogue operands) come by LDS-DMA two tiles ahead into two buffers;
//  * one barrier per tile: group gi's epilogue runs on wave gi after it, while the other waves start the
//    next tile's chains; an LDS arrival counter keeps those from overwriting the segment sums before every
//    epilogue of the tile has read them.
// One workgroup per CU.
constexpr int GR_G = 8, GR_RT = 16, GR_XROW = 2048 + 8;
constexpr size_t GR_RED = (size_t)2 * GR_RT * GR_XROW * 2;             // after the two activation tiles
constexpr size_t GR_OPS = GR_RED + (size_t)GR_G * 4 * 8 * GR_RT * 4;   // epilogue operands, 2 x 2 KiB
constexpr size_t GR_CNT = GR_OPS + 2 * 2048;
constexpr size_t GR_LDS = GR_CNT + 16;

// one 256-byte LDS-DMA piece (64 lanes x 4 B, lane-linear)
__device__ __forceinline__ void dma_dword(const void* gsrc, void* ldp) {
  const unsigned ldst =
      __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) void*)ldp);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(ldst)
               : "memory");
}

//  * DN (dense pairs): each wave owns one PAIR of groups (16 columns) and feeds the MFMA a 16-column B operand per
//    k-half: lane l = column l & 15 of the pair, k = 64 kc + 32 h + 8 (l >> 4) .. + 7, gathered from the two groups'
//    M8 chunks at load time (lane (l & 7) + 8 h + 16 (l >> 4) of group 2p + ((l >> 3) & 1)). acc0 then holds every
//    column's k-half-0 chain and acc1 its k-half-1 chain, the same products in the same MFMA accumulations as the M8
//    form's columns 0..7 / 8..15 (a column's MFMA result does not depend on the column's place in the tile), and
//    acc0 + acc1 is the M8 form's acc0 + ror8(acc1) for all 16 lanes: half the MFMAs of the M8 form, same bits.
template <int EPI, int GPW, bool DN = false>
__global__ __launch_bounds__(GR_G * 4 / GPW * 64 / (DN ? 2 : 1)) void gemm_rows_kernel(const ZmiGemvArgs a, int n_cb,
                                                                                       int n_rt, int rpw) {
  constexpr int W = 4, NL = 8, RT = GR_RT, K = 2048, KC = K / 64, XROW = GR_XROW, NE = 2;
  // group sets (DN: pair sets, GPW pairs per wave), waves
  constexpr int NGS = DN ? GR_G / 2 / GPW : GR_G / GPW, NWV = NGS * W;
  static_assert(!DN || GPW == 1, "dense pairs: one pair per wave");
  // the activation tiles are DMA'd by the upper half of the waves only (PPW pieces each): the epilogue waves
  // (wave < 8) then never wait on memory inside the tile loop, so their output stores stay in flight
  constexpr int NDW = NWV / 2, PPW = RT * (K / 512) / NDW;
  static_assert(NDW >= GR_G, "the epilogue waves and the DMA waves are disjoint");
  // operand pieces per tile, issued by the last wave: residual inputs (16 rows x 8 groups x 16 B), or the rows'
  // positions and cache rows (dwords)
  constexpr int EP = EPI == ZMI_EPI_RESIDUAL ? 2 : (EPI == ZMI_EPI_QKV ? 1 : 0);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* xs = reinterpret_cast<bf16_t*>(smem);                 // [2][RT][XROW] activation tiles
  float* red = reinterpret_cast<float*>(smem + GR_RED);          // [group][segment][8][RT] segment sums
  char* ops = smem + GR_OPS;                                     // [2][2 KiB]
  unsigned* cnt = reinterpret_cast<unsigned*>(smem + GR_CNT);    // epilogues finished
  const int b = blockIdx.x, idx = b >> 3;
  const int n_rg = (n_rt + rpw - 1) / rpw;
  const int cb = (idx / n_rg) * 8 + (b & 7), rg = idx - (idx / n_rg) * n_rg;  // gemv_body's XCD-aware map
  if (cb >= n_cb) return;
  ZMI_GSTAMP(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int gs = wave % NGS, wk = wave / NGS;  // groups gs + NGS h (h < GPW) over segment wk
  const int ngroups = a.N >> 3;
  int gg[GPW];
#pragma unroll
  for (int h = 0; h < GPW; ++h) gg[h] = min(cb * GR_G + gs + NGS * h, ngroups - 1);  // clamped: discarded
  const int n_ew = min(GR_G, ngroups - cb * GR_G);  // epilogue waves: group cb * 8 + wave on wave < n_ew
  const bool ew = wave < n_ew;
  const int eg = cb * GR_G + wave;
  const int t0 = rg * rpw;
  const int rt_end = min(n_rt, t0 + rpw);
  const bf16_t* X = reinterpret_cast<const bf16_t*>(a.X);
  const bool opw = EP && wave == NWV - 1;  // the operand-piece wave
  const bool dw = wave >= NDW;              // a DMA wave
  if (tid == 0) *cnt = 0;
  volatile __attribute__((address_space(3))) unsigned* lcnt = (volatile __attribute__((address_space(3))) unsigned*)cnt;

  // tile t = 16 rows x 4 KiB = 64 DMA pieces, PPW per wave (rows past M re-read row M - 1: their outputs are
  // discarded, and the waves' counts are fixed, which the vmcnt waits rely on), then its epilogue operands
  auto dma_tile = [&](int t) {
    if (!dw) return;
    bf16_t* dst = xs + (t & 1) * RT * XROW;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave - NDW + NDW * i, r = pc >> 2, p = pc & 3;
      const int sr = min(t * RT + r, a.M - 1);
      dma_piece(X + (size_t)sr * a.ldx + p * 512 + lane * 8, dst + r * XROW + p * 512);
    }
    if (opw) {
      char* od = ops + (t & 1) * 2048;
      if (EPI == ZMI_EPI_RESIDUAL) {  // [row][group] 16 B: out[row][8 g .. 8 g + 7]
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int e = lane + 64 * i, r = e >> 3, gi = min(cb * GR_G + (e & 7), ngroups - 1);
          dma_piece(reinterpret_cast<const bf16_t*>(a.out) + (size_t)min(t * RT + r, a.M - 1) * a.ldo + gi * 8,
                    reinterpret_cast<bf16_t*>(od + i * 1024));
        }
      } else if (EPI == ZMI_EPI_QKV) {  // dwords 0..15 the rows' positions, 16..31 their cache rows
        const int r = min(t * RT + (lane & 15), a.M - 1);
        dma_dword((lane & 16) ? a.row_kv + r : a.row_pos + r, od);
      }
    }
  };

  dma_tile(t0);
  if (t0 + 1 < rt_end) dma_tile(t0 + 1);
  __builtin_amdgcn_sched_barrier(0);
  // the weight slices of the wave's groups (GPW NL x 16 B per lane), in flight at once, in chain order (chunk
  // j of every group before chunk j + 1): the first tile's chains follow them as they land. Re-read by the
  // other row groups of this column block from L2 (temporal).
  u32x4_t wf[DN ? 2 : GPW][NL];  // DN: wf[h][j] = k-half h of chunk j for the wave's pair
  if constexpr (DN) {
    // lane l: column l & 15 of pair gs (group cb * 8 + 2 gs + ((l >> 3) & 1), clamped: discarded), M8 lane
    // (l & 7) + 8 h + 16 (l >> 4) of that group's chunk
    const int grp = min(cb * GR_G + 2 * gs + ((lane >> 3) & 1), ngroups - 1) - cb * GR_G;
    const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(reinterpret_cast<const char*>(a.W) + (size_t)cb * GR_G * KC * 1024), (short)0,
        GR_G * KC * 1024, 0x00020000);
    const int vo = (grp * KC + wk * NL) * 1024 + ((lane & 7) + 16 * (lane >> 4)) * 16;
#pragma unroll
    for (int j = 0; j < NL; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) wf[h][j] = __builtin_amdgcn_raw_buffer_load_b128(wrsrc, vo + 128 * h, j * 1024, 0);
  } else {
    __amdgpu_buffer_rsrc_t wrsrc[GPW];
#pragma unroll
    for (int h = 0; h < GPW; ++h)
      wrsrc[h] = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<char*>(reinterpret_cast<const char*>(a.W) + ((size_t)gg[h] * KC + wk * NL) * 1024), (short)0,
          NL * 1024, 0x00020000);
#pragma unroll
    for (int j = 0; j < NL; ++j)
#pragma unroll
      for (int h = 0; h < GPW; ++h) wf[h][j] = __builtin_amdgcn_raw_buffer_load_b128(wrsrc[h], lane * 16, j * 1024, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  // every weight slice and the first two tiles' pieces: waiting here for all of them keeps the compiler's own
  // waits for the weights out of the tile loop (a vmcnt(0) there would also wait for the DMA of later tiles
  // and for the epilogue stores)
  ZMI_WAIT_VM(0);
  __syncthreads();

  for (int t = t0;; ++t) {  // invariant: tile t's rows and operands are in LDS, visible to every wave
    const int ti = t - t0;
    if (ti == 1) ZMI_GSTAMP(2);
    const int row0 = t * RT, rows = min(RT, a.M - row0);
    const bool more = t + 1 < rt_end;
    f32x4_t acc0[GPW], acc1[GPW];
#pragma unroll
    for (int h = 0; h < GPW; ++h) acc0[h] = acc1[h] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    {
      const bf16_t* xa = xs + (t & 1) * RT * XROW + (lane & 15) * XROW + wk * NL * 64 + (lane >> 4) * 8;
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        const bf16x8_t x0 = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(xa + j * 64));
        const bf16x8_t x1 = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(xa + j * 64 + 32));
        if constexpr (DN) {
          acc0[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, __builtin_bit_cast(bf16x8_t, wf[0][j]), acc0[0], 0, 0, 0);
          acc1[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, __builtin_bit_cast(bf16x8_t, wf[1][j]), acc1[0], 0, 0, 0);
        } else {
#pragma unroll
          for (int h = 0; h < GPW; ++h) {
            const bf16x8_t wv = __builtin_bit_cast(bf16x8_t, wf[h][j]);
            acc0[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, wv, acc0[h], 0, 0, 0);
            acc1[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, wv, acc1[h], 0, 0, 0);
          }
        }
      }
    }
    if (ti == 0) ZMI_GSTAMP(1);
    if (ti == 1) ZMI_GSTAMP(3);
    // the previous tile's epilogues have read the segment sums (bounded: they are a few hundred cycles of work)
    if (ti > 0) {
      const unsigned want = (unsigned)(n_ew * ti);
      for (int spin = 0; *lcnt < want && spin < (1 << 20); ++spin)
        __builtin_amdgcn_s_sleep(1);
    }
    {
      const int c = lane & 15, rb = (lane >> 4) * 4;
      if constexpr (DN) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          red[(((2 * gs + (c >> 3)) * W + wk) * 8 + (c & 7)) * RT + rb + q] = acc0[0][q] + acc1[0][q];
      } else {
#pragma unroll
        for (int h = 0; h < GPW; ++h)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float v = acc0[h][q] + ror8(acc1[h][q]);
            if (c < 8) red[(((gs + NGS * h) * W + wk) * 8 + c) * RT + rb + q] = v;
          }
      }
    }
    // this tile's epilogue operands into registers before the buffer is re-filled
    uint32_t res_pre[NE] = {0u, 0u};
    int q_pos = -1, q_kvr = 0;
    if (ew) {
      const char* od = ops + (t & 1) * 2048;
      if (EPI == ZMI_EPI_RESIDUAL) {
#pragma unroll
        for (int i = 0; i < NE; ++i) {
          const int e = lane + 64 * i, r = e >> 3, c = e & 7;
          res_pre[i] = *reinterpret_cast<const uint16_t*>(od + (r * GR_G + wave) * 16 + c * 2);
        }
      }
      if (EPI == ZMI_EPI_QKV && (lane >> 2) < rows) {
        q_pos = reinterpret_cast<const int*>(od)[lane >> 2];
        q_kvr = reinterpret_cast<const int*>(od)[16 + (lane >> 2)];
      }
    }
    if (dw) ZMI_WAIT_VM(0);  // the next tile's pieces (DMA waves; the epilogue waves' stores stay in flight)
    // segment sums complete; the next tile's rows visible; this tile's buffers free (LDS-only fence: no wait
    // for global stores)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    if (ti == 1) ZMI_GSTAMP(4);
    if (t + 2 < rt_end) dma_tile(t + 2);
    if (ew) {
      auto colsum = [&](int c, int r) {  // segment sums in segment order (gemv_body's wave order)
        float v = red[((wave * W) * 8 + c) * RT + r];
#pragma unroll
        for (int w = 1; w < W; ++w) v += red[((wave * W + w) * 8 + c) * RT + r];
        return v;
      };
      epilogue<EPI, RT, 0>(a, colsum, lane, rows, row0, eg, res_pre, q_pos, q_kvr, QkvFuse{nullptr, 0});
      if (more && lane == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (ti == 1) ZMI_GSTAMP(5);
    if (!more) break;
  }
  ZMI_GSTAMP(7);
}


// row tiles per workgroup: enough workgroups to fill the chip (~4 per CU), each re-reading its weight
// slice as few times as that allows (speed only: a row's arithmetic does not depend on it)
inline int rows_per_wg(int n_cb, int n_rt, int target) {
  if (n_rt <= 1) return 1;
  // about `target` workgroups: fewer row groups re-read each weight slice. Measured on the C3 sample:
  // 512 (K = 2048) against ~1024: 102 -> 104x, 256 and 2048 slower, the prefill unmoved; 256 for the
  // K = 8192 fc2 (1024-thread workgroups, 256 KB weight slices): 9,740 -> 9,960 frames/s, 128 slower
  const int n_rg = std::max(1, std::min(n_rt, target / std::max(1, n_cb)));
  return (n_rt + n_rg - 1) / n_rg;
}

// (W, NL, RT) from K: K = 64 W NL. The shape fixes a row's reduction order, so it depends on K
// only (every M, every launch form: decode, prefill and zmi_attn_block's QKV role agree bit for
// bit). K = 2048 streams 8 chunks per lane from 4 waves per group (with G = 2: 512 threads, the
// fused QKV + attention launch's block size); K = 8192 holds 8 rows per tile (8 x 16 KiB of LDS).
struct Shape {
  int W, NL, RT;
};
inline bool shape_for(int K, bool ln, Shape* s) {
  switch (K) {
    case 512: *s = {2, 4, 16}; return true;
    case 1024: *s = {4, 4, 16}; return true;
    case 2048: *s = {4, 8, 16}; return true;
    case 4096: *s = {4, 16, 16}; return true;
    case 8192: *s = {8, 16, 8}; return true;
  }
  return false;
}

// column groups per block: 2 for the many-group K = 2048 projections with a prologue or many rows (qkv, fc1, heads: the
// block's LayerNorm and activation staging are then shared by 16 columns), 4 for the plain ones over many rows;
// `groups` > 0 overrides.
// Speed only: a group's arithmetic does not depend on G.
inline int groups_for(const ZmiGemvArgs& a, const Shape& s) {
  if (a.groups > 0) return a.groups;
  // two groups also for plain rows when there are many of them: each workgroup's activation tiles
  // then serve 16 columns (a 128-row fc1 re-read its rows from L2 per 8-column group: ~1 GB a launch)
  // (from 5 rows: the pre-normalised plans; C5's 16-row step 2.03 -> 1.87 ms with both K = 2048 and 8192 at 2)
  if (a.K == 8192 && a.M > 4 && a.N / 8 >= 256) return 2;  // fc2 over many rows: 16 KB activation rows
  // 4 groups (1024 threads) for the plain K = 2048 GEMVs over many rows (qkv, out_proj, fc1, heads of the
  // multi-slot decode and the prefill): each staged activation tile serves 32 columns, halving the tile
  // re-reads of 2 groups (C3 sample 9,050 -> 9,710 frames/s)
  if (a.K == 2048 && a.M > 16 && a.N / 8 >= 256 && a.ln_w == nullptr && a.pro == ZMI_PRO_AUTO) return 4;
  return (a.K == 2048 && a.N / 8 >= 384 && (a.ln_w != nullptr || a.pro != ZMI_PRO_AUTO || a.M > 4)) ? 2 : 1;
}

template <int G, int W, int NL, int RT, int PRO, int EPI, int NTW>
hipError_t launch_p(const ZmiGemvArgs& a, hipStream_t s) {
  constexpr int K = W * NL * 64;
  auto fn = gemv_kernel<G, W, NL, RT, PRO, EPI, NTW>;
  const int n_cb = (a.N / 8 + G - 1) / G;
  const int n_rt = (a.M + RT - 1) / RT;
  size_t lds = Img<K>::bytes(a.M < RT ? a.M : RT, G * W, RT, PRO);
  if (lds > LDS_MAX) return hipErrorInvalidValue;
  const int rpw = rows_per_wg(n_cb, n_rt, K == 8192 ? 256 : 512);
  const int64_t blocks = (int64_t)((n_cb + 7) / 8) * 8 * ((n_rt + rpw - 1) / rpw);
  if (NTW && zmi_option(ZMI_OPT_GEMV_SPREAD)) {
    // a decode launch streams each weight once: its rate is the number of CUs it keeps busy (one CU
    // pulls ~25 GB/s), so reserve LDS such that at most ceil(blocks / CUs) workgroups share a CU
    // (ZMI_OPT_GEMV_SPREAD > 1 caps the workgroups per CU at that value: an occupancy probe; 2 cost fc1 ~0.85 us per
    // launch, 3 measured the same as 4, profiles/r06_gemv_spread_ab.jsonl)
    int64_t per_cu = (blocks + zmi_cu_count() - 1) / zmi_cu_count();
    if (zmi_option(ZMI_OPT_GEMV_SPREAD) > 1) per_cu = std::min<int64_t>(per_cu, zmi_option(ZMI_OPT_GEMV_SPREAD));
    if (per_cu < 8) lds = std::max(lds, LDS_MAX / (size_t)(per_cu + 1) + 1024);
  }
  if (lds > 64 * 1024) {
    static const hipError_t attr =  // once per instantiation: allow > 64 KiB of dynamic LDS
        hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)LDS_MAX);
    if (attr != hipSuccess) return attr;
  }
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(G * W * 64), lds, s, a, n_cb, n_rt, rpw);
  return hipGetLastError();
}

template <int G, int W, int NL, int RT, int EPI>
hipError_t launch_g(const ZmiGemvArgs& a, hipStream_t s) {
  constexpr int K = W * NL * 64;
  const bool ln = a.ln_w != nullptr;
  const bool once = a.M <= RT;  // each weight read once: non-temporal loads
  if (a.pro == ZMI_PRO_ADDLN) {  // the hybrid blocks' d_model GEMVs
    if constexpr ((K == 512 || K == 2048) && EPI != ZMI_EPI_RESIDUAL && EPI != ZMI_EPI_F32)
      return once ? launch_p<G, W, NL, RT, PRO_ADDLN, EPI, 1>(a, s) : launch_p<G, W, NL, RT, PRO_ADDLN, EPI, 0>(a, s);
    return hipErrorInvalidValue;
  }
  if (a.pro == ZMI_PRO_GRMS) {  // the Mamba2 out_proj (K = d_ssm)
    if constexpr ((K == 1024 || K == 4096) && EPI == ZMI_EPI_STORE)
      return once ? launch_p<G, W, NL, RT, PRO_GRMS, EPI, 1>(a, s) : launch_p<G, W, NL, RT, PRO_GRMS, EPI, 0>(a, s);
    return hipErrorInvalidValue;
  }
  if (a.pro == ZMI_PRO_GRMS_G) {  // the same from g = y * gate rows (decode: one tile)
    if constexpr ((K == 1024 || K == 4096) && EPI == ZMI_EPI_STORE)
      return once ? launch_p<G, W, NL, RT, PRO_GRMSG, EPI, 1>(a, s) : hipErrorInvalidValue;
    return hipErrorInvalidValue;
  }
  if (ln) return once ? launch_p<G, W, NL, RT, PRO_LN, EPI, 1>(a, s) : launch_p<G, W, NL, RT, PRO_LN, EPI, 0>(a, s);
  return once ? launch_p<G, W, NL, RT, PRO_PLAIN, EPI, 1>(a, s) : launch_p<G, W, NL, RT, PRO_PLAIN, EPI, 0>(a, s);
}

// where the many-row form beats gemv_body's 4-group tile loop (C3 decode shapes, tools/kernel_bench.py
// --gemm-rows 1,0): 128 rows qkv 18.1 -> 13.0 us, fc1 41.9 -> 31.1, heads 36.9 -> 24.0, out_proj 9.8 -> 7.0;
// 64 rows qkv 12.1 -> 9.6, fc1 26.2 -> 22.8, heads 21.3 -> 15.3 but out_proj 5.8 -> 6.8; 32 rows only the
// wide ones (heads 13.3 -> 11.6; qkv 7.6 -> 9.7, out_proj 5.8 -> 8.3)
inline bool rows_form(int M, int N) { return M > 64 || (M > 32 && N >= 3072) || N >= 8192; }

template <int EPI, int GPW, bool DN>
hipError_t launch_rows(const ZmiGemvArgs& a, hipStream_t s) {
  auto fn = gemm_rows_kernel<EPI, GPW, DN>;
  const int n_cb = (a.N / 8 + GR_G - 1) / GR_G;
  const int n_rt = (a.M + GR_RT - 1) / GR_RT;
  const int rpw = rows_per_wg(n_cb, n_rt, zmi_cu_count());  // one workgroup per CU
  const int64_t blocks = (int64_t)((n_cb + 7) / 8) * 8 * ((n_rt + rpw - 1) / rpw);
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX);
  if (attr != hipSuccess) return attr;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(GR_G * 4 / GPW * 64 / (DN ? 2 : 1)), GR_LDS, s, a, n_cb, n_rt, rpw);
  return hipGetLastError();
}

template <int EPI>
hipError_t launch(const ZmiGemvArgs& a, hipStream_t s) {
  Shape sh;
  if (!shape_for(a.K, a.ln_w != nullptr, &sh)) return hipErrorInvalidValue;
  const int g = groups_for(a, sh);
  if (a.K == 2048 && a.M > GR_RT && a.ln_w == nullptr && a.pro == ZMI_PRO_AUTO && a.groups == 0 &&
      zmi_option(ZMI_OPT_GEMM_ROWS) && rows_form(a.M, a.N))
    return (zmi_option(ZMI_OPT_GEMM_ROWS) & 2) ? launch_rows<EPI, 1, true>(a, s) : launch_rows<EPI, 2, false>(a, s);
  if (g == 4 && sh.W == 4 && sh.NL == 8 && sh.RT == 16 && a.M > sh.RT && a.ln_w == nullptr && a.pro == ZMI_PRO_AUTO)
    return launch_p<4, 4, 8, 16, PRO_PLAIN, EPI, 0>(a, s);  // groups_for's many-row plain case only
#define ZMI_SHAPE(G_, W_, NL_, RT_) \
  if (g == G_ && sh.W == W_ && sh.NL == NL_ && sh.RT == RT_) return launch_g<G_, W_, NL_, RT_, EPI>(a, s);
  ZMI_SHAPE(1, 2, 4, 16)
  ZMI_SHAPE(1, 4, 4, 16)
  ZMI_SHAPE(1, 4, 8, 16)
  ZMI_SHAPE(2, 4, 8, 16)
  ZMI_SHAPE(1, 4, 16, 16)
  ZMI_SHAPE(1, 8, 16, 8)
  ZMI_SHAPE(2, 8, 16, 8)
#undef ZMI_SHAPE
  return hipErrorInvalidValue;  // e.g. groups = 2 outside the LayerNorm'd K = 2048 shape
}

}  // namespace zmi_gemv
