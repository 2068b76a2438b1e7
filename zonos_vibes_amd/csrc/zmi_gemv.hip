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
#include "zmi_common.h"
#include "zmi_kernels.h"

namespace {

constexpr int PRO_PLAIN = 0, PRO_LN = 1;

template <int MT, int NF, int PRO, int EPI>
__global__ __launch_bounds__(256) void gemv_kernel(const ZmiGemvArgs a) {
  __shared__ float red[4][MT][64][4];
  __shared__ float tile[MT * 16][17];
  __shared__ float ln_mean[MT * 16], ln_rstd[MT * 16];
  __shared__ unsigned last_flag;

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

  f32x4_t acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const bf16_t* X = reinterpret_cast<const bf16_t*>(a.X);
  const bf16_t* lnw = reinterpret_cast<const bf16_t*>(a.ln_w);
  const bf16_t* lnb = reinterpret_cast<const bf16_t*>(a.ln_b);
  const u32x4_t* wbase = reinterpret_cast<const u32x4_t*>(a.W) + ((size_t)nt * KT + kt_base) * 64 + lane;
  const int arow = lane & 15, kq = (lane >> 4) * 8;

  for (int c = 0; c < a.nchunk; ++c) {
    const int ktc = (c * 4 + wave) * NF;
    u32x4_t wf[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) wf[f] = __builtin_nontemporal_load(wbase + (size_t)(ktc + f) * 64);

    if (PRO == PRO_LN && c == 0) {
      for (int r = wave; r < MT * 16; r += 4) {
        float mean = 0.f, rstd = 0.f;
        if (r < rows) {
          const bf16_t* xr = X + (size_t)(row0 + r) * a.ldx;
          float s = 0.f;
          for (int k = lane * 8; k < a.K; k += 512) {
            uint4 v = *reinterpret_cast<const uint4*>(xr + k);
            const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) s += bf2f(u[j]) + bf2f(u[j] >> 16);
          }
          mean = wave_sum(s) / (float)a.K;
          float ss = 0.f;
          for (int k = lane * 8; k < a.K; k += 512) {
            uint4 v = *reinterpret_cast<const uint4*>(xr + k);
            const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float d0 = bf2f(u[j]) - mean, d1 = bf2f(u[j] >> 16) - mean;
              ss += d0 * d0 + d1 * d1;
            }
          }
          rstd = 1.0f / sqrtf(wave_sum(ss) / (float)a.K + a.eps);
        }
        if (lane == 0) {
          ln_mean[r] = mean;
          ln_rstd[r] = rstd;
        }
      }
      __syncthreads();
    }

#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int k0 = (kt_base + ktc + f) * 32 + kq;
      uint4 lw, lb;
      if (PRO == PRO_LN) {
        lw = *reinterpret_cast<const uint4*>(lnw + k0);
        lb = *reinterpret_cast<const uint4*>(lnb + k0);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int r = mt * 16 + arow;
        uint4 xv = {0u, 0u, 0u, 0u};
        if (r < rows) {
          xv = *reinterpret_cast<const uint4*>(X + (size_t)(row0 + r) * a.ldx + k0);
          if (PRO == PRO_LN) {
            // torch CPU LayerNorm form: (x * rstd + (-mean * rstd)) * gamma + beta, separate ops
            const float rstd = ln_rstd[r], nb = -ln_mean[r] * rstd;
            uint32_t u[4] = {xv.x, xv.y, xv.z, xv.w};
            const uint32_t uw[4] = {lw.x, lw.y, lw.z, lw.w};
            const uint32_t ub[4] = {lb.x, lb.y, lb.z, lb.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float y0 = (bf2f(u[j]) * rstd + nb) * bf2f(uw[j]) + bf2f(ub[j]);
              float y1 = (bf2f(u[j] >> 16) * rstd + nb) * bf2f(uw[j] >> 16) + bf2f(ub[j] >> 16);
              u[j] = f2bf(y0) | (f2bf(y1) << 16);
            }
            xv = uint4{u[0], u[1], u[2], u[3]};
          }
        }
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
    for (int e = threadIdx.x; e < rows * 16; e += 256) slab[(size_t)ks * (MT * 256) + e] = tile[e >> 4][e & 15];
    if (!zmi_last_arriver(a.counters + tid, (unsigned)a.ksplit, &last_flag)) return;
    for (int e = threadIdx.x; e < rows * 16; e += 256) {
      float v = slab[e];
      for (int s = 1; s < a.ksplit; ++s) v += slab[(size_t)s * (MT * 256) + e];
      tile[e >> 4][e & 15] = v;
    }
    __syncthreads();
  }

  // ---- fused epilogues ----
  const int col0 = nt * 16;
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
        *p = (bf16_t)f2bf(bf2f(*p) + bfround(v));  // x + bf16(linear(x))  (_torch.py:100-101)
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
    // packed tile: columns 0..7 = value rows 8*nt.., 8..15 = gate rows F + 8*nt..  (_torch.py:150-152)
    for (int e = threadIdx.x; e < rows * 8; e += 256) {
      const int m = e >> 3, c = e & 7;
      const float y = bfround(tile[m][c]);
      const float g = bfround(tile[m][c + 8]);
      const float sg = bfround(g / (1.0f + expf(-g)));
      reinterpret_cast<bf16_t*>(a.out)[(size_t)(row0 + m) * a.ldo + nt * 8 + c] = (bf16_t)f2bf(y * sg);
    }
  } else if (EPI == ZMI_EPI_QKV) {
    // q | k | v split, interleaved-pair RoPE in fp32 on q and k, then KV-cache write (_torch.py:18-49,117-126)
    const int qcols = a.hq * a.hd, kcols = a.hkv * a.hd;
    for (int e = threadIdx.x; e < rows * 8; e += 256) {
      const int m = e >> 3, c = (e & 7) * 2;
      const int row = row0 + m;
      const int pos = a.row_pos[row];
      if (pos < 0) continue;
      const int n = col0 + c;
      float x0 = bfround(tile[m][c]), x1 = bfround(tile[m][c + 1]);
      if (n < qcols + kcols) {
        const int d = (n < qcols ? n : n - qcols) % a.hd;
        const float co = a.rope[((size_t)pos * (a.hd >> 1) + (d >> 1)) * 2];
        const float si = a.rope[((size_t)pos * (a.hd >> 1) + (d >> 1)) * 2 + 1];
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
        const size_t o = (((size_t)a.row_kv[row] * a.hkv + kh) * a.smax + pos) * a.hd + d;
        *reinterpret_cast<uint32_t*>(cache + o) = packed;
      }
    }
  }
}

// Pack a row-major [N_src][K] bf16 weight into MFMA-native tiles (zero rows beyond N_src).
__global__ void pack_kernel(const bf16_t* __restrict__ src, uint4* __restrict__ dst, int n_src, int k, int n_pad,
                            int mode) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int kt_n = k >> 5;
  const size_t total = (size_t)(n_pad >> 4) * kt_n * 64;
  if (idx >= total) return;
  const int l = idx & 63;
  const size_t t = idx >> 6;
  const int kt = (int)(t % kt_n), nt = (int)(t / kt_n);
  const int n = nt * 16 + (l & 15), kk = kt * 32 + (l >> 4) * 8;
  int srow = n;
  if (mode == ZMI_PACK_SWIGLU) {
    const int f = n_src >> 1, c = n & 15;
    srow = c < 8 ? nt * 8 + c : f + nt * 8 + (c - 8);
  }
  uint4 v = {0u, 0u, 0u, 0u};
  if (srow < n_src) v = *reinterpret_cast<const uint4*>(src + (size_t)srow * k + kk);
  dst[idx] = v;
}

template <int MT, int NF, int PRO, int EPI>
hipError_t launch_t(const ZmiGemvArgs& a, hipStream_t s) {
  dim3 grid((a.N >> 4) * a.ksplit, (a.M + MT * 16 - 1) / (MT * 16));
  hipLaunchKernelGGL((gemv_kernel<MT, NF, PRO, EPI>), grid, dim3(256), 0, s, a);
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

}  // namespace

// Choose (row tiles, fragments per wave, split-K) for an (M, N, K) problem. The K split
// depends only on (N, K), never on M, so results are identical for every batch size.
void zmi_gemv_plan(int M, int N, int K, int* mt, int* nf, int* ksplit, int* nchunk) {
  const int KT = K / 32;
  int m = M <= 16 ? 1 : (M <= 32 ? 2 : (M <= 64 ? 4 : 8));
  // target >= ~512 blocks for the HBM stream; fragments per wave <= 16
  const int nt = N / 16;
  int ks = 1;
  while (nt * ks < 512 && (KT % (ks * 2 * 4)) == 0 && KT / (ks * 2 * 4) >= 4) ks *= 2;
  int per_wave = KT / (ks * 4);
  int f = per_wave >= 16 ? 16 : (per_wave >= 8 ? 8 : (per_wave >= 4 ? 4 : 2));
  while (per_wave % f) f >>= 1;
  *mt = m;
  *nf = f;
  *ksplit = ks;
  *nchunk = per_wave / f;
}

extern "C" int zmi_gemv_launch(const ZmiGemvArgs* args, int epi, void* stream) {
  ZmiGemvArgs a = *args;
  int mt, nf, ks, nch;
  if (a.N % 16 || a.K % 128) return zmi_fail_msg("gemv: N must be a multiple of 16 and K of 128");
  zmi_gemv_plan(a.M, a.N, a.K, &mt, &nf, &ks, &nch);
  if (a.ksplit <= 0) {
    a.ksplit = ks;
    a.nchunk = nch;
  } else {
    const int per_wave = (a.K / 32) / (a.ksplit * 4);
    if (per_wave * a.ksplit * 4 != a.K / 32) return zmi_fail_msg("gemv: K/32 not divisible by 4*ksplit");
    nf = per_wave >= 16 ? 16 : (per_wave >= 8 ? 8 : (per_wave >= 4 ? 4 : 2));
    while (per_wave % nf) nf >>= 1;
    a.nchunk = per_wave / nf;
  }
  if (nf < 2) return zmi_fail_msg("gemv: fewer than 2 fragments per wave");
  if (a.ksplit > 1 && (!a.slab || !a.counters)) return zmi_fail_msg("gemv: split-K needs slab + counters");
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  switch (epi) {
    case ZMI_EPI_STORE: e = launch_mt<ZMI_EPI_STORE>(a, mt, nf, s); break;
    case ZMI_EPI_RESIDUAL: e = launch_mt<ZMI_EPI_RESIDUAL>(a, mt, nf, s); break;
    case ZMI_EPI_QKV: e = launch_mt<ZMI_EPI_QKV>(a, mt, nf, s); break;
    case ZMI_EPI_SWIGLU: e = launch_mt<ZMI_EPI_SWIGLU>(a, mt, nf, s); break;
    case ZMI_EPI_LOGITS: e = launch_mt<ZMI_EPI_LOGITS>(a, mt, nf, s); break;
    case ZMI_EPI_F32: e = launch_mt<ZMI_EPI_F32>(a, mt, nf, s); break;
    default: return zmi_fail_msg("gemv: unknown epilogue");
  }
  ZMI_CHECK(e);
  return 0;
}

extern "C" int zmi_pack_weight(const void* src, void* dst, int n_src, int k, int n_pad, int mode, void* stream) {
  if (n_pad % 16 || k % 32 || n_pad < (mode == ZMI_PACK_SWIGLU ? n_src : 0))
    return zmi_fail_msg("pack: bad shape");
  const size_t total = (size_t)(n_pad / 16) * (k / 32) * 64;
  hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)src, (uint4*)dst, n_src, k, n_pad, mode);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int64_t zmi_gemv_slab_floats(int M, int N, int K) {
  int mt, nf, ks, nch;
  zmi_gemv_plan(M, N, K, &mt, &nf, &ks, &nch);
  const int groups = (M + mt * 16 - 1) / (mt * 16);
  return ks > 1 ? (int64_t)groups * (N / 16) * ks * mt * 256 : 0;
}
