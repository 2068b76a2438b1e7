// GEMV kernel template + launch helpers, included by the per-epilogue translation units
// (zmi_gemv_e*.hip) so the ~100 instantiations compile in parallel.
#pragma once
#include "zmi_common.h"
#include "zmi_kernels.h"

namespace zmi_gemv {


constexpr int PRO_PLAIN = 0, PRO_LN = 1;
constexpr int XS_GLOBAL = 0, XS_REG = 1, XS_DMA = 2;  // where the A-operand rows come from

template <int MT>
struct GemvLds {
  static constexpr int RED = 0;
  static constexpr int TILE = RED + 4 * MT * 64 * 4 * 4;
  static constexpr int LN = TILE + MT * 16 * 17 * 4;
  static constexpr int FLAG = LN + 2 * MT * 16 * 4;
  static constexpr int XS = FLAG + 16;
};

template <int MT, int NF, int PRO, int EPI, int XLDS>
__global__ __launch_bounds__(256) void gemv_kernel(const ZmiGemvArgs a) {
  // all LDS in one dynamic block, carved at 16 B multiples (no static __shared__ shifting the base:
  // cdna_hip_programming.md §6 Guideline 17)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float(&red)[4][MT][64][4] = *reinterpret_cast<float(*)[4][MT][64][4]>(smem);
  float(&tile)[MT * 16][17] = *reinterpret_cast<float(*)[MT * 16][17]>(smem + GemvLds<MT>::TILE);
  float* ln_mean = reinterpret_cast<float*>(smem + GemvLds<MT>::LN);
  float* ln_rstd = ln_mean + MT * 16;
  unsigned& last_flag = *reinterpret_cast<unsigned*>(smem + GemvLds<MT>::FLAG);
  bf16_t* xs = reinterpret_cast<bf16_t*>(smem + GemvLds<MT>::XS);  // XLDS: activation rows [rows][ldx_s]

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int NT = a.N >> 4, KT = a.K >> 5;
  int b = blockIdx.x;
  const int nb = gridDim.x;
  if ((nb & 7) == 0) b = (b & 7) * (nb >> 3) + (b >> 3);  // XCD-contiguous tiles (speed only)
  const int nt = b / a.ksplit, ks = b - nt * a.ksplit;
  const int row0 = blockIdx.y * (MT * 16);
  const int rows = min(MT * 16, a.M - row0);
  const int kt_blk = KT / a.ksplit;
  const int kt_base = ks * kt_blk;
  const int kb0 = kt_base * 32, KB = kt_blk * 32;

  const bf16_t* X = reinterpret_cast<const bf16_t*>(a.X);
  const bf16_t* lnw = reinterpret_cast<const bf16_t*>(a.ln_w);
  const bf16_t* lnb = reinterpret_cast<const bf16_t*>(a.ln_b);
  // V8 weight layout (zmi_gemv8_impl.h): the MFMA B fragment (n = lane & 15, k = 8 (lane >> 4) of a
  // 16 x 32 tile) of K-tile kt sits at  wlane + (kt >> 1) * 64 + (kt & 1) * 4  (uint4 units)
  const int wn = nt * 16 + (lane & 15);
  const u32x4_t* wlane = reinterpret_cast<const u32x4_t*>(a.W) + ((size_t)(wn >> 3) * (a.K >> 6)) * 64 +
                         (wn & 7) * 8 + (lane >> 4);
  auto wfrag = [&](int kt) { return __builtin_nontemporal_load(wlane + (size_t)(kt >> 1) * 64 + (kt & 1) * 4); };
  const int arow = lane & 15, kq = (lane >> 4) * 8;

  // (1) activation rows first (they gate the LayerNorm): up to 4 x 16 B per thread into registers,
  //     unconditional loads from clamped addresses (no branch -> no vmcnt(0) per load)
  const int xw = (PRO == PRO_LN) ? a.K : KB;          // columns staged per row
  const int xk0 = (PRO == PRO_LN) ? 0 : kb0;          // first staged column
  const int ldx_s = xw + 8;
  const int per_row = xw >> 3, n_x = rows * per_row;
  uint4 xr[4];
  if (XLDS == XS_DMA) {
    // 1 KiB LDS-DMA pieces (64 lanes x 16 B, lane-linear, never crossing a row): no VGPRs, so the
    // weight stream below is not held back by register reuse
    // Issued as inline asm: the compiler then does not treat the in-flight DMA as a pending LDS
    // write and does not drain the whole vm queue (the weights) before the first ds_read; the
    // covering wait is the explicit vmcnt(NF) below (cdna_hip_programming.md §5.7).
    // pieces: activation rows, then (LayerNorm) gamma and beta of this block's k-range
    const int ppr = xw >> 9, n_x_pc = rows * ppr, ppk = KB >> 9;
    const int n_pc = n_x_pc + (PRO == PRO_LN ? 2 * ppk : 0);
    for (int pc = wave; pc < n_pc; pc += 4) {
      const bf16_t* gsrc;
      bf16_t* ldp;
      if (pc < n_x_pc) {
        const int r = pc / ppr, p = pc - r * ppr;
        gsrc = X + (size_t)(row0 + r) * a.ldx + xk0 + p * 512 + lane * 8;
        ldp = xs + r * ldx_s + p * 512;
      } else {
        const int q = pc - n_x_pc, which = q / ppk, p = q - which * ppk;
        gsrc = (which ? lnb : lnw) + kb0 + p * 512 + lane * 8;
        ldp = xs + rows * ldx_s + which * KB + p * 512;
      }
      const unsigned ldst = __builtin_amdgcn_readfirstlane(
          (unsigned)(size_t)(__attribute__((address_space(3))) void*)ldp);
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                   "s_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(gsrc), "s"(ldst)
                   : "memory");
    }
  } else if (XLDS == XS_REG) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int e = threadIdx.x + i * 256;
      e = e < n_x ? e : n_x - 1;
      const int r = e / per_row, c = (e - r * per_row) * 8;
      xr[i] = *reinterpret_cast<const uint4*>(X + (size_t)(row0 + r) * a.ldx + xk0 + c);
    }
  }
  // epilogue operands needed only at the end, fetched now so their latency hides under the stream
  // (decode-sized blocks: one (row, column pair) per thread)
  const int col0 = nt * 16;
  const bool pre = rows * 16 <= 256;
  int q_pos = -1, q_kvr = 0;
  if (EPI == ZMI_EPI_QKV && pre && (int)threadIdx.x < rows * 8) {
    q_pos = a.row_pos[row0 + (threadIdx.x >> 3)];
    q_kvr = a.row_kv[row0 + (threadIdx.x >> 3)];
  }
  __builtin_amdgcn_sched_barrier(0);  // keep the activation loads ahead of the weight stream
  // (2) the weight stream does not depend on the activations: issue chunk 0 right away
  u32x4_t wf[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) wf[f] = wfrag(kt_base + wave * NF + f);
  __builtin_amdgcn_sched_barrier(0);
  uint32_t res_pre = 0;
  float2 rope_pre = {1.f, 0.f};
  if (EPI == ZMI_EPI_RESIDUAL && pre && (int)threadIdx.x < rows * 16) {
    const int n = col0 + (threadIdx.x & 15);
    if (n < a.n_valid)
      res_pre = reinterpret_cast<const bf16_t*>(a.out)[(size_t)(row0 + (threadIdx.x >> 4)) * a.ldo + n];
  }
  if (EPI == ZMI_EPI_QKV && pre && q_pos >= 0) {
    const int n = col0 + (threadIdx.x & 7) * 2;
    if (n < (a.hq + a.hkv) * a.hd) {
      const int d = (n < a.hq * a.hd ? n : n - a.hq * a.hd) % a.hd;
      rope_pre = *reinterpret_cast<const float2*>(a.rope + ((size_t)q_pos * (a.hd >> 1) + (d >> 1)) * 2);
    }
  }

  // (3) activations visible in LDS while the weights are still in flight; LayerNorm statistics
  if (XLDS == XS_DMA) {
    // this wave's DMA pieces are older than its NF weight loads; a raw barrier (no vmcnt(0) drain)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NF) : "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  } else if (XLDS == XS_REG) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = threadIdx.x + i * 256;
      if (e < n_x) {
        const int r = e / per_row, c = (e - r * per_row) * 8;
        *reinterpret_cast<uint4*>(xs + r * ldx_s + c) = xr[i];
      }
    }
    for (int e = threadIdx.x + 1024; e < n_x; e += 256) {
      const int r = e / per_row, c = (e - r * per_row) * 8;
      *reinterpret_cast<uint4*>(xs + r * ldx_s + c) =
          *reinterpret_cast<const uint4*>(X + (size_t)(row0 + r) * a.ldx + xk0 + c);
    }
    __syncthreads();
  }
  if (PRO == PRO_LN) {
    for (int r = wave; r < rows; r += 4) {
      float s = 0.f;
      for (int k = lane * 8; k < a.K; k += 512) {
        const uint4 v = XLDS ? *reinterpret_cast<const uint4*>(xs + r * ldx_s + k)
                             : *reinterpret_cast<const uint4*>(X + (size_t)(row0 + r) * a.ldx + k);
        const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) s += bf2f(u[j]) + bf2f(u[j] >> 16);
      }
      const float mean = wave_sum(s) / (float)a.K;
      float ss = 0.f;
      for (int k = lane * 8; k < a.K; k += 512) {
        const uint4 v = XLDS ? *reinterpret_cast<const uint4*>(xs + r * ldx_s + k)
                             : *reinterpret_cast<const uint4*>(X + (size_t)(row0 + r) * a.ldx + k);
        const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d0 = bf2f(u[j]) - mean, d1 = bf2f(u[j] >> 16) - mean;
          ss += d0 * d0 + d1 * d1;
        }
      }
      const float rstd = 1.0f / sqrtf(wave_sum(ss) / (float)a.K + a.eps);  // all lanes: wave reduction
      if (lane == 0) {
        ln_mean[r] = mean;
        ln_rstd[r] = rstd;
      }
    }
    __syncthreads();
    if (XLDS) {  // normalise this block's k-range in place: (x * rstd + (-mean * rstd)) * gamma + beta
      const int per_row = KB >> 3;
      for (int e = threadIdx.x; e < rows * per_row; e += 256) {
        const int r = e / per_row, c = kb0 + (e - r * per_row) * 8;
        uint4* p = reinterpret_cast<uint4*>(xs + r * ldx_s + c);
        uint4 gw, gb;
        if (XLDS == XS_DMA) {  // gamma / beta were DMA'd next to the rows
          gw = *reinterpret_cast<const uint4*>(xs + rows * ldx_s + (c - kb0));
          gb = *reinterpret_cast<const uint4*>(xs + rows * ldx_s + KB + (c - kb0));
        } else {
          gw = *reinterpret_cast<const uint4*>(lnw + c);
          gb = *reinterpret_cast<const uint4*>(lnb + c);
        }
        const uint4 v = *p;
        const float rstd = ln_rstd[r], nbias = -ln_mean[r] * rstd;
        uint32_t u[4] = {v.x, v.y, v.z, v.w};
        const uint32_t uw[4] = {gw.x, gw.y, gw.z, gw.w}, ub[4] = {gb.x, gb.y, gb.z, gb.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float y0 = (bf2f(u[j]) * rstd + nbias) * bf2f(uw[j]) + bf2f(ub[j]);
          const float y1 = (bf2f(u[j] >> 16) * rstd + nbias) * bf2f(uw[j] >> 16) + bf2f(ub[j] >> 16);
          u[j] = f2bf(y0) | (f2bf(y1) << 16);
        }
        *p = uint4{u[0], u[1], u[2], u[3]};
      }
      __syncthreads();
    }
  }

  f32x4_t acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int c = 0; c < a.nchunk; ++c) {
    const int ktc = (c * 4 + wave) * NF;
    if (c > 0) {
#pragma unroll
      for (int f = 0; f < NF; ++f) wf[f] = wfrag(kt_base + ktc + f);
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int k0 = (kt_base + ktc + f) * 32 + kq;  // absolute k of this lane's 8 elements
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int r = mt * 16 + arow;
        const int rc = r < rows ? r : rows - 1;       // clamped: no branch around the load
        const uint32_t keep = r < rows ? 0xffffffffu : 0u;
        uint4 xv;
        if (XLDS) {
          xv = *reinterpret_cast<const uint4*>(xs + rc * ldx_s + (k0 - xk0));
        } else {
          xv = *reinterpret_cast<const uint4*>(X + (size_t)(row0 + rc) * a.ldx + k0);
          if (PRO == PRO_LN) {
            const uint4 lw = *reinterpret_cast<const uint4*>(lnw + k0);
            const uint4 lb = *reinterpret_cast<const uint4*>(lnb + k0);
            const float rstd = ln_rstd[rc], nbias = -ln_mean[rc] * rstd;
            uint32_t u[4] = {xv.x, xv.y, xv.z, xv.w};
            const uint32_t uw[4] = {lw.x, lw.y, lw.z, lw.w}, ub[4] = {lb.x, lb.y, lb.z, lb.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float y0 = (bf2f(u[j]) * rstd + nbias) * bf2f(uw[j]) + bf2f(ub[j]);
              const float y1 = (bf2f(u[j] >> 16) * rstd + nbias) * bf2f(uw[j] >> 16) + bf2f(ub[j] >> 16);
              u[j] = f2bf(y0) | (f2bf(y1) << 16);
            }
            xv = uint4{u[0], u[1], u[2], u[3]};
          }
        }
        xv.x &= keep;
        xv.y &= keep;
        xv.z &= keep;
        xv.w &= keep;
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, xv),
                                                          __builtin_bit_cast(bf16x8_t, wf[f]), acc[mt], 0, 0, 0);
      }
    }
  }

  // ---- fixed-order cross-wave reduction -> tile[m][n] ----
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][mt][lane][r] = acc[mt][r];
  __syncthreads();
  for (int e = threadIdx.x; e < MT * 256; e += 256) {
    const int mt = e >> 8, l = (e >> 2) & 63, r = e & 3;
    const float v = ((red[0][mt][l][r] + red[1][mt][l][r]) + red[2][mt][l][r]) + red[3][mt][l][r];
    tile[mt * 16 + (l >> 4) * 4 + r][l & 15] = v;
  }
  __syncthreads();

  // ---- split-K: publish slab, last arriver sums slabs in ks order ----
  if (a.ksplit > 1) {
    const size_t tid = (size_t)blockIdx.y * NT + nt;
    float* slab = a.slab + tid * (size_t)a.ksplit * (MT * 256);
    for (int e = threadIdx.x; e < rows * 16; e += 256) st_wt(slab + (size_t)ks * (MT * 256) + e, tile[e >> 4][e & 15]);
    if (!zmi_last_arriver_wt(a.counters + tid, (unsigned)a.ksplit, &last_flag)) return;
    for (int e = threadIdx.x; e < rows * 16; e += 256) {
      float v = ld_wt(slab + e);
      for (int s = 1; s < a.ksplit; ++s) v += ld_wt(slab + (size_t)s * (MT * 256) + e);
      tile[e >> 4][e & 15] = v;
    }
    __syncthreads();
  }

  // ---- fused epilogues ----
  if (EPI == ZMI_EPI_STORE || EPI == ZMI_EPI_RESIDUAL || EPI == ZMI_EPI_F32) {
    for (int e = threadIdx.x; e < rows * 16; e += 256) {
      const int m = e >> 4, n = col0 + (e & 15);
      if (n >= a.n_valid) continue;
      const float v = tile[m][e & 15];
      const size_t o = (size_t)(row0 + m) * a.ldo + n;
      if (EPI == ZMI_EPI_F32) {
        reinterpret_cast<float*>(a.out)[o] = v;
      } else if (EPI == ZMI_EPI_STORE) {
        reinterpret_cast<bf16_t*>(a.out)[o] = (bf16_t)f2bf(v);
      } else {
        bf16_t* p = reinterpret_cast<bf16_t*>(a.out) + o;
        const uint32_t xin = pre ? res_pre : (uint32_t)*p;  // prefetched when one element per thread
        *p = (bf16_t)f2bf(bf2f(xin) + bfround(v));  // x + bf16(linear(x))  (_torch.py:100-101)
      }
    }
  } else if (EPI == ZMI_EPI_LOGITS) {
    // 9 heads packed back to back, 1026 columns each (1025 real + the zero pad row)
    for (int e = threadIdx.x; e < rows * 16; e += 256) {
      const int m = e >> 4, n = col0 + (e & 15);
      if (n >= a.n_valid) continue;
      const int cb = n / 1026, v = n - cb * 1026;
      reinterpret_cast<float*>(a.out)[((size_t)(row0 + m) * 9 + cb) * 1026 + v] = bfround(tile[m][e & 15]);
    }
  } else if (EPI == ZMI_EPI_SWIGLU) {
    // V8 SwiGLU packing: each 8-column group = 4 value rows then their 4 gate rows, so tile
    // column 8h + c (c < 4) is value row 8nt + 4h + c and 8h + 4 + c its gate  (_torch.py:150-152)
    for (int e = threadIdx.x; e < rows * 8; e += 256) {
      const int m = e >> 3, c = e & 7, h = c >> 2, c4 = c & 3;
      const float y = bfround(tile[m][h * 8 + c4]);
      const float g = bfround(tile[m][h * 8 + 4 + c4]);
      const float sg = bfround(g / (1.0f + expf(-g)));
      reinterpret_cast<bf16_t*>(a.out)[(size_t)(row0 + m) * a.ldo + nt * 8 + c] = (bf16_t)f2bf(y * sg);
    }
  } else if (EPI == ZMI_EPI_QKV) {
    // q | k | v split, interleaved-pair RoPE in fp32 on q and k, then KV-cache write (_torch.py:18-49,117-126)
    const int qcols = a.hq * a.hd, kcols = a.hkv * a.hd;
    for (int e = threadIdx.x; e < rows * 8; e += 256) {
      const int m = e >> 3, c = (e & 7) * 2;
      const int row = row0 + m;
      const int pos = pre ? q_pos : a.row_pos[row];
      if (pos < 0) continue;
      const int n = col0 + c;
      float x0 = bfround(tile[m][c]), x1 = bfround(tile[m][c + 1]);
      if (n < qcols + kcols) {
        const int d = (n < qcols ? n : n - qcols) % a.hd;
        const float2 cs =
            pre ? rope_pre : *reinterpret_cast<const float2*>(a.rope + ((size_t)pos * (a.hd >> 1) + (d >> 1)) * 2);
        const float co = cs.x, si = cs.y;
        const float r0 = x0 * co - x1 * si;
        const float r1 = x1 * co + x0 * si;
        x0 = r0;
        x1 = r1;
      }
      const uint32_t packed = f2bf(x0) | (f2bf(x1) << 16);
      if (n < qcols) {
        *reinterpret_cast<uint32_t*>(reinterpret_cast<bf16_t*>(a.out) + (size_t)row * a.ldo + n) = packed;
      } else {
        const bool is_k = n < qcols + kcols;
        const int nn = is_k ? n - qcols : n - qcols - kcols;
        const int kh = nn / a.hd, d = nn - kh * a.hd;
        bf16_t* cache = reinterpret_cast<bf16_t*>(is_k ? a.k_cache : a.v_cache);
        const size_t o = (((size_t)(pre ? q_kvr : a.row_kv[row]) * a.hkv + kh) * a.smax + pos) * a.hd + d;
        *reinterpret_cast<uint32_t*>(cache + o) = packed;
      }
    }
  }
}

template <int MT, int NF, int PRO, int EPI>
hipError_t launch_t(const ZmiGemvArgs& a, hipStream_t s) {
  dim3 grid((a.N >> 4) * a.ksplit, (a.M + MT * 16 - 1) / (MT * 16));
  // stage the activation rows in LDS when they fit (always for decode-sized M)
  const int rows = a.M < MT * 16 ? a.M : MT * 16;
  const int xw = PRO == PRO_LN ? a.K : a.K / a.ksplit;
  const int kb = a.K / a.ksplit;
  const size_t lds = (size_t)rows * (xw + 8) * sizeof(bf16_t);
  const size_t lds_dma = lds + (PRO == PRO_LN ? 2 * (size_t)kb * sizeof(bf16_t) : 0);
  if (lds_dma <= 64 * 1024 && xw % 512 == 0 && kb % 512 == 0)
    hipLaunchKernelGGL((gemv_kernel<MT, NF, PRO, EPI, XS_DMA>), grid, dim3(256), GemvLds<MT>::XS + lds_dma, s, a);
  else if (lds <= 64 * 1024)
    hipLaunchKernelGGL((gemv_kernel<MT, NF, PRO, EPI, XS_REG>), grid, dim3(256), GemvLds<MT>::XS + lds, s, a);
  else
    hipLaunchKernelGGL((gemv_kernel<MT, NF, PRO, EPI, XS_GLOBAL>), grid, dim3(256), GemvLds<MT>::XS, s, a);
  return hipGetLastError();
}

template <int MT, int NF, int EPI>
hipError_t launch_pro(const ZmiGemvArgs& a, hipStream_t s) {
  return a.ln_w ? launch_t<MT, NF, PRO_LN, EPI>(a, s) : launch_t<MT, NF, PRO_PLAIN, EPI>(a, s);
}

template <int MT, int EPI>
hipError_t launch_nf(const ZmiGemvArgs& a, int nf, hipStream_t s) {
  switch (nf) {
    case 2: return launch_pro<MT, 2, EPI>(a, s);
    case 4: return launch_pro<MT, 4, EPI>(a, s);
    case 8: return launch_pro<MT, 8, EPI>(a, s);
    case 16: return launch_pro<MT, 16, EPI>(a, s);
  }
  return hipErrorInvalidValue;
}

template <int EPI>
hipError_t launch_mt(const ZmiGemvArgs& a, int mt, int nf, hipStream_t s) {
  switch (mt) {
    case 1: return launch_nf<1, EPI>(a, nf, s);
    case 2: return launch_nf<2, EPI>(a, nf, s);
    case 4: return launch_nf<4, EPI>(a, nf, s);
    case 8: return launch_nf<8, EPI>(a, nf, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace zmi_gemv
