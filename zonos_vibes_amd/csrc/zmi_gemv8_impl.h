// Decode GEMV for few rows (M <= 16), gfx950: one workgroup per 8-column group, full K.
//
// out[m, n] = sum_k A[m, k] * W[n, k]   (nn.Linear, reference zonos/backbone/_torch.py:114-115,147-152,
//                                        heads: zonos/model.py:100-101)
//
// Why not the MFMA strip kernel (zmi_gemv_impl.h) at decode sizes: with 16-column MFMA strips an
// N = 2048 projection (out_proj, fc2) has only 128 strips, so half the CUs stay idle and the other
// half are bound by what one CU can keep in flight (MI355X_MICROARCH.md: ~24 GB/s per CU at
// ~72 KB in flight). Here a workgroup owns 8 output columns over the whole K, so N = 2048 gives
// 256 workgroups (one per CU) and N = 16384 gives 2048, and every lane issues ALL of its weight
// loads before it needs the first one (NL x 16 B per lane, non-temporal, straight into VGPRs).
// With M <= 16 rows the arithmetic (2 M FLOP per weight) is far below the VALU rate, so the dot
// products run on VALU fp32 FMAs — no MFMA padding of 2 rows up to 16.
//
// Weight layout "V8" (zmi_pack_weight): 1 KiB chunk (g, kc) holds columns 8g..8g+7 x k 64kc..64kc+63,
// lane l of the wave instruction reading it gets column 8g + (l >> 3), k = 64 kc + 8 (l & 7) .. +7.
// A wave's chunks are consecutive in memory.
//
// Reduction order is fixed and independent of M: per lane a sequential fp32 FMA chain over its
// k-range, then a fixed 8-lane DPP tree, then the W waves summed in wave order. Every row of a
// launch is therefore computed identically whatever the batch (SURVEY.md §0.3 batch invariance).
#pragma once
#include "zmi_common.h"
#include "zmi_kernels.h"

namespace zmi_gemv8 {

// Diagnostic build only (-DZMI_STAMPS, tools/stamps.py): wave 0 lane 0 of every block writes
// s_memrealtime (100 MHz) at fixed points into a.slab[block * 8 + i]; the real kernel has none.
#ifdef ZMI_STAMPS
#define ZMI_STAMP(i)                                                                       \
  do {                                                                                     \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    unsigned long long _t;                                                                 \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");         \
    if (threadIdx.x == 0) reinterpret_cast<unsigned long long*>(a.slab)[blockIdx.x * 8 + (i)] = _t; \
    __builtin_amdgcn_sched_barrier(0);                                                     \
  } while (0)
#else
#define ZMI_STAMP(i) \
  do {               \
  } while (0)
#endif

constexpr int PRO_PLAIN = 0, PRO_LN = 1;

template <int G, int W, int MR>
struct Lds8 {
  // [x rows: M*K bf16][gamma K][beta K]  then  red[G][W][8][MR] f32, ln_red[G*W][MR][2] f32
  static size_t bytes(int M, int K, bool ln) {
    return (size_t)M * K * 2 + (ln ? (size_t)4 * K : 0) + (size_t)G * W * 8 * MR * 4 + (size_t)G * W * MR * 2 * 4;
  }
};

__device__ __forceinline__ float sum8_lanes(float v) {
  // all 8 lanes of an aligned octet end with the bit-identical sum (commutative pairings)
  v += dpp_mov<DPP_XOR1>(v);
  v += dpp_mov<DPP_XOR2>(v);
  return v + dpp_mov<DPP_HALF_MIRROR>(v);
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

// Block = G column groups x W waves per group (wave = gi * W + w). Wave (gi, w) streams group
// blockIdx.x * G + gi over k in [w * NL * 64, (w + 1) * NL * 64). The LayerNorm of the block's
// rows is computed once per block and shared by its G groups.
// waves per SIMD the register allocation must allow: all of a launch resident at once at decode
// shapes (e.g. fc1: 2048 blocks x 4 waves = 8 per SIMD -> <= 64 VGPRs)
template <int NL, int MR>
constexpr int occ8() { return MR > 2 ? 2 : (NL <= 8 ? 8 : 4); }

template <int G, int W, int NL, int MR, int PRO, int EPI>
__global__ __launch_bounds__(G * W * 64, (occ8<NL, MR>())) void gemv8_kernel(const ZmiGemvArgs a) {
  constexpr int K = W * NL * 64;
  constexpr int KC = K / 64;
  constexpr int NT = G * W * 64;
  constexpr int NWV = G * W;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M = a.M;
  bf16_t* xs = reinterpret_cast<bf16_t*>(smem);
  bf16_t* gam = xs + (size_t)M * K;
  bf16_t* bet = gam + K;
  float* red = reinterpret_cast<float*>(smem + (size_t)M * K * 2 + (PRO == PRO_LN ? 4 * K : 0));
  float* ln_red = red + NWV * 8 * MR;  // [NWV][MR][2]

  ZMI_STAMP(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR descriptors, no waterfalls
  const int gi = wave / W, wk = wave - gi * W;
  const int ngroups = a.N >> 3;
  const int g_raw = blockIdx.x * G + gi;
  const bool g_ok = g_raw < ngroups;
  const int g = g_ok ? g_raw : ngroups - 1;  // clamped: every wave joins the barriers
  const int col0 = g * 8;
  const bf16_t* X = reinterpret_cast<const bf16_t*>(a.X);

  // (1) activation rows (+ LayerNorm gamma/beta) into LDS by DMA, 1 KiB pieces spread over waves
  {
    constexpr int PPR = K / 512;
    const int n_x = M * PPR;
    const int n_pc = n_x + (PRO == PRO_LN ? 2 * PPR : 0);
    for (int pc = wave; pc < n_pc; pc += NWV) {
      if (pc < n_x) {
        const int r = pc / PPR, p = pc - r * PPR;
        dma_piece(X + (size_t)r * a.ldx + p * 512 + lane * 8, xs + r * K + p * 512);
      } else {
        const int q = pc - n_x, which = q / PPR, p = q - which * PPR;
        const bf16_t* src = reinterpret_cast<const bf16_t*>(which ? a.ln_b : a.ln_w);
        dma_piece(src + p * 512 + lane * 8, (which ? bet : gam) + p * 512);
      }
    }
  }
  // epilogue operands that need no other load (older than the weights: covered by the vmcnt below)
  // epilogue thread t of group gi: t = tid - gi * 64 in [0, 64) within the group's first wave
  const int et = lane;
  const bool ew = (wk == 0) && g_ok;  // the group's first wave runs its epilogue
  uint32_t res_pre = 0;
  int q_pos = -1, q_kvr = 0;
  if (EPI == ZMI_EPI_RESIDUAL && ew && et < 8 * M) {
    const int n = col0 + (et & 7);
    if (n < a.n_valid) res_pre = reinterpret_cast<const bf16_t*>(a.out)[(size_t)(et >> 3) * a.ldo + n];
  }
  if (EPI == ZMI_EPI_QKV && ew && et < 4 * M) {
    q_pos = a.row_pos[et >> 2];
    q_kvr = a.row_kv[et >> 2];
  }
  __builtin_amdgcn_sched_barrier(0);
  // (2) the whole weight slice of this lane, in flight at once: one buffer descriptor per wave
  // (wave-uniform base), lane offset in the VGPR, chunk offset j KiB folded into the instruction, so
  // no address VGPRs are recycled while loads are pending (cdna_hip_programming.md T8)
  const char* wbase = reinterpret_cast<const char*>(a.W) + ((size_t)g * KC + wk * NL) * 1024;
  const __amdgpu_buffer_rsrc_t wrsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wbase), (short)0, NL * 1024, 0x00020000);
  u32x4_t wf[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) wf[j] = __builtin_amdgcn_raw_buffer_load_b128(wrsrc, lane * 16, j * 1024, 2 /* nt */);
  __builtin_amdgcn_sched_barrier(0);
  ZMI_STAMP(1);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NL) : "memory");  // DMA pieces + prefetches landed
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  ZMI_STAMP(2);

  // (3) LayerNorm (nn.LayerNorm, _torch.py:62,88,90): fp32 two-pass statistics, bf16-rounded output.
  // Thread-owned 8-element chunks e = tid + i*NT of the [M][K/8] chunk array stay in registers
  // through both passes; per-row partials reduce over lanes (DPP) then waves (LDS, wave order).
  if (PRO == PRO_LN) {
    constexpr int CPR = K / 8;                   // 8-element chunks per row
    constexpr int CI = (CPR + NT - 1) / NT;      // chunks per row per thread
    uint4 xv[MR][CI];
    float s[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      const int mr = m < M ? m : M - 1;          // rows past M: harmless duplicates, never stored
      s[m] = 0.f;
#pragma unroll
      for (int i = 0; i < CI; ++i) {
        const int c = tid + i * NT;
        xv[m][i] = *reinterpret_cast<const uint4*>(xs + mr * K + (c < CPR ? c : 0) * 8);
        if (c < CPR) {
          const uint32_t u[4] = {xv[m][i].x, xv[m][i].y, xv[m][i].z, xv[m][i].w};
          float t = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) t += bf2f(u[j]) + bf2f(u[j] >> 16);
          s[m] += t;
        }
      }
    }
    auto block_rows = [&](float* v, int slot) {  // v[m] -> block total per row, same order everywhere
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const float w = wave_sum(v[m]);
        if (lane == 0) ln_red[(wave * MR + m) * 2 + slot] = w;
      }
      __syncthreads();
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        float t = ln_red[m * 2 + slot];
        for (int w = 1; w < NWV; ++w) t += ln_red[(w * MR + m) * 2 + slot];
        v[m] = t;
      }
    };
    block_rows(s, 0);
    float mean[MR], ss[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      mean[m] = s[m] / (float)K;
      ss[m] = 0.f;
#pragma unroll
      for (int i = 0; i < CI; ++i) {
        if (tid + i * NT < CPR) {
          const uint32_t u[4] = {xv[m][i].x, xv[m][i].y, xv[m][i].z, xv[m][i].w};
          float t = 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d0 = bf2f(u[j]) - mean[m], d1 = bf2f(u[j] >> 16) - mean[m];
            t += d0 * d0 + d1 * d1;
          }
          ss[m] += t;
        }
      }
    }
    block_rows(ss, 1);
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      const float rstd = 1.0f / sqrtf(ss[m] / (float)K + a.eps), nbias = -mean[m] * rstd;
#pragma unroll
      for (int i = 0; i < CI; ++i) {
        const int c = tid + i * NT;
        if (m < M && c < CPR) {
          const uint4 gw = *reinterpret_cast<const uint4*>(gam + c * 8);
          const uint4 gb = *reinterpret_cast<const uint4*>(bet + c * 8);
          uint32_t u[4] = {xv[m][i].x, xv[m][i].y, xv[m][i].z, xv[m][i].w};
          const uint32_t uw[4] = {gw.x, gw.y, gw.z, gw.w}, ub[4] = {gb.x, gb.y, gb.z, gb.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float y0 = (bf2f(u[j]) * rstd + nbias) * bf2f(uw[j]) + bf2f(ub[j]);
            const float y1 = (bf2f(u[j] >> 16) * rstd + nbias) * bf2f(uw[j] >> 16) + bf2f(ub[j] >> 16);
            u[j] = f2bf(y0) | (f2bf(y1) << 16);
          }
          *reinterpret_cast<uint4*>(xs + m * K + c * 8) = uint4{u[0], u[1], u[2], u[3]};
        }
      }
    }
    __syncthreads();
  }

  ZMI_STAMP(3);
  // (4) dot products: lane owns column col0 + (lane >> 3), k = 64 (wk*NL + j) + 8 (lane & 7) .. +7.
  // fp32 FMAs on exactly widened bf16 (products exact, one rounding per add), branch-free over MR
  // rows (rows past M re-read row M-1; their sums are never stored)
  float acc[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) acc[m] = 0.f;
  const int kl = (lane & 7) * 8;
  const bf16_t* xrow[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) xrow[m] = xs + (m < M ? m : M - 1) * K + wk * NL * 64 + kl;
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    uint4 xq[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) xq[m] = *reinterpret_cast<const uint4*>(xrow[m] + j * 64);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float wlo = __uint_as_float(wf[j][i] << 16), whi = __uint_as_float(wf[j][i] & 0xffff0000u);
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const uint32_t u = i == 0 ? xq[m].x : (i == 1 ? xq[m].y : (i == 2 ? xq[m].z : xq[m].w));
        acc[m] = __builtin_fmaf(wlo, __uint_as_float(u << 16), acc[m]);
        acc[m] = __builtin_fmaf(whi, __uint_as_float(u & 0xffff0000u), acc[m]);
      }
    }
    // every row's chain passes through this point each chunk: without it the compiler runs row 0's
    // whole chain first and parks the widened weights in scratch for the other rows
#pragma unroll
    for (int m = 0; m < MR; ++m) asm volatile("" : "+v"(acc[m]));
  }
  ZMI_STAMP(4);
  // (5) 8-lane tree, then one partial per (wave, column, row) in LDS
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    const float v = sum8_lanes(acc[m]);
    if ((lane & 7) == 0) red[(wave * 8 + (lane >> 3)) * MR + m] = v;
  }
  __syncthreads();
  ZMI_STAMP(5);
  if (!ew) return;
  auto colsum = [&](int c, int m) {  // the group's W wave partials, in wave order
    float v = red[((gi * W) * 8 + c) * MR + m];
#pragma unroll
    for (int w = 1; w < W; ++w) v += red[((gi * W + w) * 8 + c) * MR + m];
    return v;
  };

  // (6) fused epilogues (the group's first wave; lane = (row, column) of the 8-column group)
  if (EPI == ZMI_EPI_STORE || EPI == ZMI_EPI_RESIDUAL || EPI == ZMI_EPI_F32 || EPI == ZMI_EPI_LOGITS) {
    if (et < 8 * M) {
      const int m = et >> 3, c = et & 7, n = col0 + c;
      if (n < a.n_valid) {
        const float v = colsum(c, m);
        if (EPI == ZMI_EPI_F32) {
          reinterpret_cast<float*>(a.out)[(size_t)m * a.ldo + n] = v;
        } else if (EPI == ZMI_EPI_STORE) {
          reinterpret_cast<bf16_t*>(a.out)[(size_t)m * a.ldo + n] = (bf16_t)f2bf(v);
        } else if (EPI == ZMI_EPI_RESIDUAL) {
          // x + bf16(linear(x))  (_torch.py:100-101)
          reinterpret_cast<bf16_t*>(a.out)[(size_t)m * a.ldo + n] = (bf16_t)f2bf(bf2f(res_pre) + bfround(v));
        } else {
          // 9 heads back to back, 1026 columns each (1025 real + the zero pad row)
          const int cb = n / 1026, vv = n - cb * 1026;
          reinterpret_cast<float*>(a.out)[((size_t)m * 9 + cb) * 1026 + vv] = bfround(v);
        }
      }
    }
  } else if (EPI == ZMI_EPI_SWIGLU) {
    // V8 SwiGLU packing: columns 0..3 = value rows 4g.., 4..7 = gate rows F + 4g..  (_torch.py:150-152)
    if (et < 4 * M) {
      const int m = et >> 2, c = et & 3;
      const float y = bfround(colsum(c, m));
      const float gt = bfround(colsum(c + 4, m));
      const float sg = bfround(gt / (1.0f + expf(-gt)));
      reinterpret_cast<bf16_t*>(a.out)[(size_t)m * a.ldo + g * 4 + c] = (bf16_t)f2bf(y * sg);
    }
  } else if (EPI == ZMI_EPI_QKV) {
    // q | k | v split, interleaved-pair RoPE in fp32 on q and k, KV-cache write (_torch.py:18-49,117-126)
    if (et < 4 * M && q_pos >= 0) {
      const int m = et >> 2, c = (et & 3) * 2;
      const int n = col0 + c;
      const int qcols = a.hq * a.hd, kcols = a.hkv * a.hd;
      float x0 = bfround(colsum(c, m)), x1 = bfround(colsum(c + 1, m));
      if (n < qcols + kcols) {
        // (cos, sin) of this position and dim pair: an L2-hot 512 B table row, loaded after the
        // stream so no wait on it can hold the weight loads
        const int d = (n < qcols ? n : n - qcols) % a.hd;
        const float2 cs = *reinterpret_cast<const float2*>(a.rope + ((size_t)q_pos * (a.hd >> 1) + (d >> 1)) * 2);
        const float co = cs.x, si = cs.y;
        const float r0 = x0 * co - x1 * si;
        const float r1 = x1 * co + x0 * si;
        x0 = r0;
        x1 = r1;
      }
      const uint32_t packed = f2bf(x0) | (f2bf(x1) << 16);
      if (n < qcols) {
        *reinterpret_cast<uint32_t*>(reinterpret_cast<bf16_t*>(a.out) + (size_t)m * a.ldo + n) = packed;
      } else {
        const bool is_k = n < qcols + kcols;
        const int nn = is_k ? n - qcols : n - qcols - kcols;
        const int kh = nn / a.hd, d = nn - kh * a.hd;
        bf16_t* cache = reinterpret_cast<bf16_t*>(is_k ? a.k_cache : a.v_cache);
        const size_t o = (((size_t)q_kvr * a.hkv + kh) * a.smax + q_pos) * a.hd + d;
        *reinterpret_cast<uint32_t*>(cache + o) = packed;
      }
    }
  }
  ZMI_STAMP(6);
}

// (W, NL) from K: K = 64 * W * NL. K = 2048 (every LayerNorm'd projection) streams 16 chunks per
// lane from 2 waves per group: the in-flight weights then fit the 128-VGPR budget of 4 waves per
// SIMD next to the LayerNorm's registers (at 8 chunks per lane the 64-VGPR budget that an
// all-resident fc1 needs spills, and scratch traffic queues behind the weight loads).
inline bool shape8(int K, bool ln, int* w, int* nl) {
  int W, n;
  switch (K) {
    case 512: W = 2; n = 4; break;
    case 1024: W = 4; n = 4; break;
    case 2048: W = ln ? 2 : 4; n = ln ? 16 : 8; break;  // no LayerNorm (out_proj): 4 x 8 measured faster
    case 4096: W = 4; n = 16; break;
    case 8192: W = 8; n = 16; break;
    default: return false;
  }
  *w = W;
  *nl = n;
  return true;
}

constexpr size_t LDS_MAX = 160 * 1024;  // gfx950 LDS per workgroup
constexpr int M_MAX = 8;                 // decode regime of this kernel (<= 4 CFG slot pairs)

template <int PRO, int G, int W, int NL, int MR, int EPI>
hipError_t launch8_p(const ZmiGemvArgs& a, size_t lds, hipStream_t s) {
  auto fn = gemv8_kernel<G, W, NL, MR, PRO, EPI>;
  if (lds > 64 * 1024) {
    static const hipError_t attr =  // once per instantiation: allow > 64 KiB of dynamic LDS
        hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)LDS_MAX);
    if (attr != hipSuccess) return attr;
  }
  hipLaunchKernelGGL(fn, dim3((a.N / 8 + G - 1) / G), dim3(G * W * 64), lds, s, a);
  return hipGetLastError();
}

template <int G, int W, int NL, int MR, int EPI>
hipError_t launch8_t(const ZmiGemvArgs& a, hipStream_t s) {
  const bool ln = a.ln_w != nullptr;
  const size_t lds = Lds8<G, W, MR>::bytes(a.M, a.K, ln);
  if (lds > LDS_MAX) return hipErrorInvalidValue;
  return ln ? launch8_p<PRO_LN, G, W, NL, MR, EPI>(a, lds, s) : launch8_p<PRO_PLAIN, G, W, NL, MR, EPI>(a, lds, s);
}

template <int G, int W, int NL, int EPI>
hipError_t launch8_mr(const ZmiGemvArgs& a, hipStream_t s) {
  if (a.M <= 2) return launch8_t<G, W, NL, 2, EPI>(a, s);
  if (a.M <= 4) return launch8_t<G, W, NL, 4, EPI>(a, s);
  if (a.M <= 8) return launch8_t<G, W, NL, 8, EPI>(a, s);
  return hipErrorInvalidValue;
}

// column groups per block: amortise the per-block LayerNorm / activation staging over more
// columns when there are many groups; `ksplit` < 0 in the args overrides (tuning: G = -ksplit)
inline int groups8(const ZmiGemvArgs& a, int w, int nl) {
  if (a.ksplit < 0) return -a.ksplit;
  const int ng = a.N / 8;
  // qkv (384 groups) and fc1 / heads: 2 groups per block measured fastest (tools/bench_graph.py)
  return (w == 2 && nl == 16 && ng >= 384) ? 2 : 1;
}

// true when the decode kernel takes this problem; the choice depends on M only through M <= M_MAX,
// so every batch of up to M_MAX rows runs the same kernel (bit-identical rows)
inline bool use8(int M, int N, int K, bool ln) {
  int w, nl;
  return M >= 1 && M <= M_MAX && N % 8 == 0 && shape8(K, ln, &w, &nl) &&
         (size_t)M_MAX * K * 2 + (ln ? 4 * (size_t)K : 0) + (size_t)4 * w * 8 * M_MAX * 4 * 2 <= LDS_MAX;
}

template <int EPI>
hipError_t launch8(const ZmiGemvArgs& a, hipStream_t s) {
  int w, nl;
  if (!shape8(a.K, a.ln_w != nullptr, &w, &nl)) return hipErrorInvalidValue;
  const int g = groups8(a, w, nl);
  if (w == 2 && nl == 4 && g == 1) return launch8_mr<1, 2, 4, EPI>(a, s);
  if (w == 4 && nl == 4 && g == 1) return launch8_mr<1, 4, 4, EPI>(a, s);
  if (w == 4 && nl == 8 && g == 1) return launch8_mr<1, 4, 8, EPI>(a, s);
  if (w == 2 && nl == 16 && g == 1) return launch8_mr<1, 2, 16, EPI>(a, s);
  if (w == 2 && nl == 16 && g == 2) return launch8_mr<2, 2, 16, EPI>(a, s);
  if (w == 2 && nl == 16 && g == 4) return launch8_mr<4, 2, 16, EPI>(a, s);
  if (w == 4 && nl == 16 && g == 1) return launch8_mr<1, 4, 16, EPI>(a, s);
  if (w == 8 && nl == 16 && g == 1) return launch8_mr<1, 8, 16, EPI>(a, s);
  return hipErrorInvalidValue;
}

}  // namespace zmi_gemv8
