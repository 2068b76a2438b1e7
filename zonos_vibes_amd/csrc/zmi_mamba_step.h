// Mamba2 decode-step device code shared by zmi_mamba.hip (zmi_mamba2_step) and zmi_mambablk.hip (the step
// role of zmi_mamba_block). See zmi_mamba.hip for the reference mapping (mamba-ssm 2.2.4 Mamba2.step).
#pragma once
#include "zmi_common.h"
#include "zmi_kernels.h"

namespace zmi_mamba {

constexpr int MB_HD = 64;    // headdim
constexpr int MB_DS = 128;   // d_state (ngroups = 1)
constexpr int MB_DC = 4;     // d_conv
constexpr int MB_NT = 256;   // threads of the prefill scan kernels: (p = t / 4, n-quarter = t % 4)
constexpr int MB_ST = 512;   // threads of a decode step workgroup: (p = t / 8, n-eighth = t % 8)
constexpr int MB_NCH = MB_HD + 2 * MB_DS;  // conv channels one head needs: its x, then B, C

__device__ __forceinline__ float silu_f(float v) { return v / (1.0f + expf(-v)); }
// mamba_ssm/ops/triton/softplus.py; selective_state_update applies it below 20 only
__device__ __forceinline__ float softplus_f(float v) { return v <= 20.f ? log1pf(expf(v)) : v; }

// xBC channel index of local conv channel i of head h
__device__ __forceinline__ int conv_channel(int i, int h, int d_ssm) {
  return i < MB_HD ? h * MB_HD + i : d_ssm + (i - MB_HD);
}

// causal depthwise conv1d of one channel: bias first, taps oldest first, fp32 (causal_conv1d
// update / fwd kernels), then SiLU; the caller rounds to bf16 (the conv output tensor is bf16)
__device__ __forceinline__ float conv4(const bf16_t* w4, float bias, float x0, float x1, float x2, float x3) {
  float acc = bias;
  acc = fmaf(bf2f(w4[0]), x0, acc);
  acc = fmaf(bf2f(w4[1]), x1, acc);
  acc = fmaf(bf2f(w4[2]), x2, acc);
  acc = fmaf(bf2f(w4[3]), x3, acc);
  return silu_f(acc);
}

// ---------------------------------------------------------------------------- decode step
// The step of one (row, head), shared by zmi_mamba2_step and zmi_mamba_block's step role: the raw
// in_proj values the head needs sit in LDS (raw[0, 64) its x channels, [64, 320) B and C, [320, 384) its z
// channels, [384] its dt); the state slice, conv-ring values, conv weights and bias were loaded first.
constexpr int RAW_X = 0, RAW_BC = MB_HD, RAW_Z = MB_NCH, RAW_DT = MB_NCH + MB_HD, RAW_N = RAW_DT + 2;

template <int NT>
struct StepPre {
  static constexpr int NI = (MB_NCH + NT - 1) / NT;  // conv channels per thread
  static constexpr int PARTS = NT / MB_HD;           // threads per state row p (8 at 512 threads)
  static constexpr int SVN = MB_DS / 8 / PARTS;      // uint4 of the state row per thread
  static_assert(PARTS == 4 || PARTS == 8, "a state row split over 4 or 8 lanes");
  uint4 sv[SVN];            // state slice
  float ring[NI][MB_DC - 1];
  float w[NI][MB_DC];
  float bias[NI];
  float dt_bias, A, D;      // the head's scalars: loaded with the rest, not after the in_proj values arrive
};

template <int NT>
__device__ __forceinline__ void step_prefetch(const ZmiMamba2Args& a, int h, int pos, int kv, StepPre<NT>& pre) {
  const int t = threadIdx.x, conv_dim = a.d_ssm + 2 * MB_DS;
  {
    constexpr int P = StepPre<NT>::PARTS;
    const bf16_t* st = reinterpret_cast<const bf16_t*>(a.ssm) +
                       (((size_t)kv * a.nheads + h) * MB_HD + t / P) * MB_DS + (t % P) * (MB_DS / P);
#pragma unroll
    for (int j = 0; j < StepPre<NT>::SVN; ++j) pre.sv[j] = reinterpret_cast<const uint4*>(st)[j];
  }
  pre.dt_bias = a.dt_bias[h];
  pre.A = a.A[h];
  pre.D = a.D[h];
  const bf16_t* ring = reinterpret_cast<const bf16_t*>(a.conv_ring) + (size_t)kv * MB_DC * conv_dim;
  const bf16_t* cw = reinterpret_cast<const bf16_t*>(a.conv_w);
  const bf16_t* cb = reinterpret_cast<const bf16_t*>(a.conv_b);
#pragma unroll
  for (int k = 0; k < StepPre<NT>::NI; ++k) {
    const int i = t + NT * k;
    if (i < MB_NCH) {
      const int c = conv_channel(i, h, a.d_ssm);
#pragma unroll
      for (int j = 0; j < MB_DC - 1; ++j) {
        const int q = pos - (MB_DC - 1) + j;
        pre.ring[k][j] = q >= 0 ? bf2f(ring[(size_t)(q & 3) * conv_dim + c]) : 0.f;
      }
#pragma unroll
      for (int j = 0; j < MB_DC; ++j) pre.w[k][j] = bf2f(cw[(size_t)c * MB_DC + j]);
      pre.bias[k] = bf2f(cb[c]);
    }
  }
}

template <int NT>
__device__ __forceinline__ void step_core(const ZmiMamba2Args& a, int m, int h, int pos, int kv, const bf16_t* raw,
                                          StepPre<NT>& pre, float* xs, float* bc) {
  const int t = threadIdx.x, conv_dim = a.d_ssm + 2 * MB_DS;
  bf16_t* ring = reinterpret_cast<bf16_t*>(a.conv_ring) + (size_t)kv * MB_DC * conv_dim;
  // (1) conv + SiLU of this head's 64 x channels and the 256 B / C channels (bias first, taps oldest
  // first, fp32: causal_conv1d_update; every head recomputes B / C, head 0 alone writes their ring slot)
#pragma unroll
  for (int k = 0; k < StepPre<NT>::NI; ++k) {
    const int i = t + NT * k;
    if (i < MB_NCH) {
      const bf16_t rv = raw[i];
      float acc = pre.bias[k];
      acc = fmaf(pre.w[k][0], pre.ring[k][0], acc);
      acc = fmaf(pre.w[k][1], pre.ring[k][1], acc);
      acc = fmaf(pre.w[k][2], pre.ring[k][2], acc);
      acc = fmaf(pre.w[k][3], bf2f(rv), acc);
      const float o = bfround(silu_f(acc));
      if (i < MB_HD) xs[i] = o; else bc[i - MB_HD] = o;
      if (i < MB_HD || h == 0) ring[(size_t)(pos & 3) * conv_dim + conv_channel(i, h, a.d_ssm)] = rv;
    }
  }
  // (2) dt = softplus(dt + dt_bias), dA = exp(A dt)  (selective_state_update, tie_hdim)
  const float dtv = softplus_f(bf2f(raw[RAW_DT]) + pre.dt_bias);
  const float dA = expf(pre.A * dtv);
  __syncthreads();
  // (3) state update and readout: lane (p, part) owns state[p][MB_DS / P part .. +MB_DS / P - 1] (P = NT / 64 lanes per
  // row p: 8 at the decode step's 512 threads, so each lane's readout chain is 16 terms long)
  constexpr int P = StepPre<NT>::PARTS, SVN = StepPre<NT>::SVN;
  const int p = t / P, nq = t % P;
  bf16_t* st = reinterpret_cast<bf16_t*>(a.ssm) + (((size_t)kv * a.nheads + h) * MB_HD + p) * MB_DS + nq * (MB_DS / P);
  const float x = xs[p];
  const float* B = bc + nq * (MB_DS / P);
  const float* C = bc + MB_DS + nq * (MB_DS / P);
  float out = 0.f;
#pragma unroll
  for (int j = 0; j < SVN; ++j) {
    uint32_t w[4] = {pre.sv[j].x, pre.sv[j].y, pre.sv[j].z, pre.sv[j].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = 8 * j + 2 * e;
      float s0 = bf2f(w[e]), s1 = bf2f(w[e] >> 16);
      s0 = s0 * dA + (B[n] * dtv) * x;
      s1 = s1 * dA + (B[n + 1] * dtv) * x;
      out += s0 * C[n];
      out += s1 * C[n + 1];
      w[e] = f2bf(s0) | (f2bf(s1) << 16);
    }
    pre.sv[j] = uint4{w[0], w[1], w[2], w[3]};
  }
#pragma unroll
  for (int j = 0; j < SVN; ++j) reinterpret_cast<uint4*>(st)[j] = pre.sv[j];
  out = quad_sum(out);  // the P parts of row p are lanes P p .. P p + P - 1
  if constexpr (P == 8) out += dpp_mov<DPP_HALF_MIRROR>(out);
  if (nq == 0) {
    const uint32_t yb = f2bf(out + x * pre.D);
    reinterpret_cast<bf16_t*>(a.y)[(size_t)m * a.ldy + h * MB_HD + p] = (bf16_t)yb;
    if (a.gz) {  // RMSNormGated's gate of this channel, once (the out_proj GEMV's GRMS prologue multiplies), or (gz_g)
                 // g = y * gate itself, the product gate_elem forms (GRMS_G: the out_proj then stages no y rows)
      const float zz = bf2f(raw[RAW_Z + p]);
      const float gate = zz * (1.0f / (1.0f + expf(-zz)));
      a.gz[(size_t)m * a.ldy + h * MB_HD + p] = a.gz_g ? bf2f(yb) * gate : gate;
    }
  }
}

}  // namespace zmi_mamba
