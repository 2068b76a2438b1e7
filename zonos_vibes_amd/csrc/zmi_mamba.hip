// Hybrid backbone kernels (Zonos-v0.1-hybrid, BASELINE config C4), gfx950.
//
// Reference: zonos/backbone/_mamba_ssm.py:9-57 builds its layers with mamba-ssm 2.2.4's
// `create_block` (absent from this image, so parity is unpinned; oracle/hybrid_cpu.py restates the
// published algorithm). A decode step of one Mamba2 block is
//
//   hidden, residual = layer_norm_fn(hidden, norm.w, norm.b, residual, prenorm=True)  (Block.forward)
//   zxbcdt = in_proj(hidden)                                                            (GEMV kernel)
//   xBC    = silu(causal_conv1d_update(xBC, conv_state, conv1d.w, conv1d.b))            (mamba2_step)
//   y      = selective_state_update(ssm_state, x, dt, A, B, C, D, dt_bias, softplus)    (mamba2_step)
//   y      = RMSNormGated(y, z)                                                         (gated_rmsnorm)
//   out    = out_proj(y)                                                                (GEMV kernel)
//
// and the prefill is the same block over a whole sequence (causal_conv1d_fn + mamba_chunk_scan_combined;
// mamba2_scan here: the recurrence in fp32 registers, one workgroup per (sequence, head)).
//
// State layouts (this library's, not the reference's roll buffer):
//   conv ring  bf16 [row][4][conv_dim]: the raw xBC input of position q sits in slot q & 3. A step at
//              position p reads slots of p-3 .. p-1 and writes slot p & 3 (that of p-4, which nobody
//              reads), so the workgroups of one row never race; negative positions read as zero.
//   ssm state  bf16 [row][nheads][headdim 64][d_state 128] (the reference keeps it in the cache dtype).
#include <algorithm>

#include "zmi_common.h"
#include "zmi_kernels.h"
#include "zmi_mamba_step.h"

namespace {

using namespace zmi_mamba;

__global__ __launch_bounds__(MB_ST) void mamba2_step_kernel(const ZmiMamba2Args a) {
  const int m = blockIdx.x / a.nheads, h = blockIdx.x - m * a.nheads;
  const int pos = a.row_pos[m];
  if (pos < 0) return;
  const int kv = a.row_kv ? a.row_kv[m] : m;
  __shared__ float xs[MB_HD], bc[2 * MB_DS];
  __shared__ bf16_t raw[RAW_N];
  StepPre<MB_ST> pre;
  step_prefetch<MB_ST>(a, h, pos, kv, pre);  // the state slice first: the longest loads, under the rest
  const bf16_t* zx = reinterpret_cast<const bf16_t*>(a.zxbcdt) + (size_t)m * a.ld_zx;
  for (int i = threadIdx.x; i < RAW_DT + 1; i += MB_ST) {
    const int col = i < RAW_Z ? a.d_ssm + conv_channel(i, h, a.d_ssm)
                              : (i < RAW_DT ? h * MB_HD + (i - RAW_Z) : 2 * a.d_ssm + 2 * MB_DS + h);
    raw[i] = zx[col];
  }
  __syncthreads();
  step_core<MB_ST>(a, m, h, pos, kv, raw, pre, xs, bc);
}

// ---------------------------------------------------------------------------- prefill scan
constexpr int SC_TT = 32;  // positions staged per tile

__global__ __launch_bounds__(MB_NT) void mamba2_scan_kernel(const ZmiMamba2Args a, int seq_len) {
  const int sq = blockIdx.x / a.nheads, h = blockIdx.x - sq * a.nheads;
  const int row0 = sq * seq_len;
  const int kv = a.row_kv ? a.row_kv[row0] : sq;
  const int conv_dim = a.d_ssm + 2 * MB_DS;
  const bf16_t* zx0 = reinterpret_cast<const bf16_t*>(a.zxbcdt) + (size_t)row0 * a.ld_zx;
  const bf16_t* cw = reinterpret_cast<const bf16_t*>(a.conv_w);
  const bf16_t* cb = reinterpret_cast<const bf16_t*>(a.conv_b);
  __shared__ float xs[SC_TT][MB_HD], bs[SC_TT][MB_DS], cs[SC_TT][MB_DS], dts[SC_TT], das[SC_TT];
  const int t = threadIdx.x, p = t >> 2, nq = t & 3;
  const float Ah = a.A[h], Dh = a.D[h], dtb = a.dt_bias[h];
  auto raw = [&](int q, int c) { return q >= 0 ? bf2f(zx0[(size_t)q * a.ld_zx + a.d_ssm + c]) : 0.f; };

  float s[32];
#pragma unroll
  for (int j = 0; j < 32; ++j) s[j] = 0.f;
  for (int t0 = 0; t0 < seq_len; t0 += SC_TT) {
    const int nt = min(SC_TT, seq_len - t0);
    __syncthreads();  // the previous tile's readers are done
    for (int idx = t; idx < nt * MB_NCH; idx += MB_NT) {
      const int tt = idx / MB_NCH, i = idx - tt * MB_NCH, q = t0 + tt;
      const int c = conv_channel(i, h, a.d_ssm);
      const float o = bfround(conv4(cw + (size_t)c * MB_DC, bf2f(cb[c]), raw(q - 3, c), raw(q - 2, c), raw(q - 1, c),
                                    raw(q, c)));
      if (i < MB_HD) xs[tt][i] = o;
      else if (i < MB_HD + MB_DS) bs[tt][i - MB_HD] = o;
      else cs[tt][i - MB_HD - MB_DS] = o;
    }
    if (t < nt) {
      const float dtv = softplus_f(bf2f(zx0[(size_t)(t0 + t) * a.ld_zx + 2 * a.d_ssm + 2 * MB_DS + h]) + dtb);
      dts[t] = dtv;
      das[t] = expf(Ah * dtv);
    }
    __syncthreads();
    for (int tt = 0; tt < nt; ++tt) {
      const float x = xs[tt][p], dtv = dts[tt], dA = das[tt];
      const float4* B4 = reinterpret_cast<const float4*>(&bs[tt][nq * 32]);
      const float4* C4 = reinterpret_cast<const float4*>(&cs[tt][nq * 32]);
      float out = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float4 b = B4[j], c = C4[j];
        s[4 * j + 0] = s[4 * j + 0] * dA + (b.x * dtv) * x;
        s[4 * j + 1] = s[4 * j + 1] * dA + (b.y * dtv) * x;
        s[4 * j + 2] = s[4 * j + 2] * dA + (b.z * dtv) * x;
        s[4 * j + 3] = s[4 * j + 3] * dA + (b.w * dtv) * x;
        out += s[4 * j + 0] * c.x;
        out += s[4 * j + 1] * c.y;
        out += s[4 * j + 2] * c.z;
        out += s[4 * j + 3] * c.w;
      }
      out = quad_sum(out);
      if (nq == 0)
        reinterpret_cast<bf16_t*>(a.y)[(size_t)(row0 + t0 + tt) * a.ldy + h * MB_HD + p] = (bf16_t)f2bf(out + x * Dh);
    }
  }
  // final state (bf16, the cache dtype) and the ring slots of the last four positions (zero below 0)
  bf16_t* st = reinterpret_cast<bf16_t*>(a.ssm) + (((size_t)kv * a.nheads + h) * MB_HD + p) * MB_DS + nq * 32;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) w[e] = f2bf(s[8 * j + 2 * e]) | (f2bf(s[8 * j + 2 * e + 1]) << 16);
    reinterpret_cast<uint4*>(st)[j] = uint4{w[0], w[1], w[2], w[3]};
  }
  bf16_t* ring = reinterpret_cast<bf16_t*>(a.conv_ring) + (size_t)kv * MB_DC * conv_dim;
  for (int idx = t; idx < MB_DC * MB_NCH; idx += MB_NT) {
    const int k = idx / MB_NCH, i = idx - k * MB_NCH;
    if (i >= MB_HD && h != 0) continue;
    const int q = seq_len - MB_DC + k, c = conv_channel(i, h, a.d_ssm);
    ring[(size_t)(q & 3) * conv_dim + c] = q >= 0 ? zx0[(size_t)q * a.ld_zx + a.d_ssm + c] : (bf16_t)0;
  }
}

// ---------------------------------------------------------------------------- parallel prefill scan
// zmi_mamba2_scan_ws: the same Mamba2.forward from an empty state in two launches.
//  (1) mamba2_conv_kernel, one workgroup per row: causal conv + SiLU of every xBC channel (conv4, bf16-rounded as
//      the reference's conv output tensor) into the workspace, dt = softplus(dt + dt_bias) and dA = exp(A dt) per
//      head, and, on each sequence's last row, the conv ring's four slots (the last raw inputs, zero below 0).
//  (2) mamba2_scan2_kernel, one workgroup per (sequence, head, quarter of the 64 head dims): thread (p, n-block)
//      owns state[p][8 n-block .. + 7] in fp32 registers and walks the positions in order,
//          s = fma(s, dA, (B dt) x),   y_p = sum_n fma(s, C) (+ x D),
//      the 16 n-blocks of a row summed by DPP (each block's 8 terms as two interleaved chains). The (sequence, head) recurrence the single-workgroup kernel runs on
//      256 threads is spread over 1,024 (4x the workgroups, a quarter of each thread's state and FMA chain), and
//      the conv no longer sits inside it. Its arithmetic differs from mamba2_scan_kernel's in fp32 rounding (fused
//      multiply-adds, the readout summed over 8-wide blocks): both are checked against the oracle's recurrence.
constexpr int S2_NB = MB_DS / 8;        // 16 n-blocks of 8 state columns
constexpr int S2_TT = 32;               // positions staged per tile

__global__ __launch_bounds__(256) void mamba2_conv_kernel(const ZmiMamba2Args a, int seq_len, bf16_t* xc, float* dts,
                                                          float* das) {
  // one thread per (row, channel): grid (rows, channel blocks of 256), every load of the launch in flight at once
  const int row = blockIdx.x, sq = row / seq_len, q = row - sq * seq_len, row0 = sq * seq_len;
  const int conv_dim = a.d_ssm + 2 * MB_DS, c = blockIdx.y * 256 + threadIdx.x;
  const bf16_t* zx0 = reinterpret_cast<const bf16_t*>(a.zxbcdt) + (size_t)row0 * a.ld_zx + a.d_ssm;
  if (c < conv_dim) {
    const bf16_t* cw = reinterpret_cast<const bf16_t*>(a.conv_w);
    const bf16_t* cb = reinterpret_cast<const bf16_t*>(a.conv_b);
    float r[MB_DC];
#pragma unroll
    for (int k = 0; k < MB_DC; ++k) {
      const int qq = q - (MB_DC - 1) + k;
      r[k] = qq >= 0 ? bf2f(zx0[(size_t)qq * a.ld_zx + c]) : 0.f;
    }
    xc[(size_t)row * conv_dim + c] = (bf16_t)f2bf(conv4(cw + (size_t)c * MB_DC, bf2f(cb[c]), r[0], r[1], r[2], r[3]));
    if (q == seq_len - 1) {  // the conv ring: slot qq % 4 holds the raw input of qq, for the last d_conv positions
      const int kv = a.row_kv ? a.row_kv[row0] : sq;
      bf16_t* ring = reinterpret_cast<bf16_t*>(a.conv_ring) + (size_t)kv * MB_DC * conv_dim;
#pragma unroll
      for (int k = 0; k < MB_DC; ++k) {
        const int qq = seq_len - MB_DC + k;
        ring[(size_t)(qq & 3) * conv_dim + c] = qq >= 0 ? zx0[(size_t)qq * a.ld_zx + c] : (bf16_t)0;
      }
    }
  }
  if (blockIdx.y == 0)
    for (int h = threadIdx.x; h < a.nheads; h += 256) {
      const float dtv = softplus_f(bf2f(zx0[(size_t)q * a.ld_zx + a.d_ssm + 2 * MB_DS + h]) + a.dt_bias[h]);
      dts[(size_t)row * a.nheads + h] = dtv;
      das[(size_t)row * a.nheads + h] = expf(a.A[h] * dtv);
    }
}

// PQ workgroups per (sequence, head), each 64 / PQ head dims; thread (p-group, n-block) owns PR = 4 / PQ rows p
// x 8 state columns, so each B / C value it reads from LDS serves PR rows
#ifdef ZMI_SCAN_STAMPS
// diagnostic builds only (tools/scan_probe.py --stamps): thread 0 of each workgroup stores s_memtime at the start,
// and per tile k < 12 after its operands are in LDS [1 + 2k] and after its positions [2 + 2k]
__device__ unsigned long long g_scan_stamps[1024][32];
extern "C" int zmi_scan_stamps_read(void* dst, size_t bytes) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_scan_stamps), bytes) == hipSuccess ? 0 : -1;
}
#define ZMI_SSTAMP(i_)                                                                      \
  do {                                                                                      \
    if (threadIdx.x == 0 && blockIdx.x < 1024) g_scan_stamps[blockIdx.x][i_] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define ZMI_SSTAMP(i_) \
  do {                 \
  } while (0)
#endif

template <int PQ>
__global__ __launch_bounds__(256) void mamba2_scan2_kernel(const ZmiMamba2Args a, int seq_len, const bf16_t* xc,
                                                           const float* dts, const float* das) {
  constexpr int PW = MB_HD / PQ, PR = PW / 16;  // head dims per workgroup, rows per thread
  const int pq = blockIdx.x % PQ, sh = blockIdx.x / PQ, h = sh % a.nheads, sq = sh / a.nheads;
  const int row0 = sq * seq_len, conv_dim = a.d_ssm + 2 * MB_DS;
  const int kv = a.row_kv ? a.row_kv[row0] : sq;
  const int t = threadIdx.x, pg = t / S2_NB, nb = t % S2_NB, p0 = pq * PW + pg * PR;
  __shared__ float xs[S2_TT][PW], bdt[S2_TT][MB_DS], cs[S2_TT][MB_DS], dA[S2_TT];
  const float Dh = a.D[h];
  // a tile's operands, one thread's share: (B dt, C) of (position tt = (t + 256 i) / 128, state column
  // (t + 256 i) % 128) for i < 16, x of (t + 256 i) / PW, % PW, dA of position t; loaded into registers one
  // tile ahead so their latency hides under the previous tile's recurrence
  constexpr int NBC = S2_TT * MB_DS / 256, NX = S2_TT * PW / 256;
  float rb[NBC], rc[NBC], rx[NX], rd = 0.f;
  auto load = [&](int t0) {
    const int nt = min(S2_TT, seq_len - t0);
#pragma unroll
    for (int i = 0; i < NBC; ++i) {
      const int idx = t + 256 * i, tt = idx / MB_DS, n = idx - tt * MB_DS;
      if (tt < nt) {
        const size_t r = (size_t)(row0 + t0 + tt);
        rb[i] = bf2f(xc[r * conv_dim + a.d_ssm + n]) * dts[r * a.nheads + h];
        rc[i] = bf2f(xc[r * conv_dim + a.d_ssm + MB_DS + n]);
      }
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int idx = t + 256 * i, tt = idx / PW, j = idx - tt * PW;
      if (tt < nt) rx[i] = bf2f(xc[(size_t)(row0 + t0 + tt) * conv_dim + h * MB_HD + pq * PW + j]);
    }
    if (t < nt) rd = das[(size_t)(row0 + t0 + t) * a.nheads + h];
  };
  float st[PR][8];
#pragma unroll
  for (int r = 0; r < PR; ++r)
#pragma unroll
    for (int k = 0; k < 8; ++k) st[r][k] = 0.f;
  bf16_t* y = reinterpret_cast<bf16_t*>(a.y);
  ZMI_SSTAMP(0);
  load(0);
  for (int t0 = 0; t0 < seq_len; t0 += S2_TT) {
    const int nt = min(S2_TT, seq_len - t0);
    __syncthreads();  // the previous tile's readers are done
#pragma unroll
    for (int i = 0; i < NBC; ++i) {
      const int idx = t + 256 * i, tt = idx / MB_DS, n = idx - tt * MB_DS;
      bdt[tt][n] = rb[i];
      cs[tt][n] = rc[i];
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int idx = t + 256 * i;
      xs[idx / PW][idx % PW] = rx[i];
    }
    if (t < S2_TT) dA[t] = rd;
    __syncthreads();
    if (t0 / S2_TT < 12) ZMI_SSTAMP(1 + 2 * (t0 / S2_TT));
    if (t0 + S2_TT < seq_len) load(t0 + S2_TT);
    // positions in groups of 4 with their stores behind one branch at the end: a position's readout (FMA
    // chains, DPP sums) is off the state's critical path, so the next positions' LDS reads and state updates
    // issue under it
    auto step = [&](int tt, float (&v)[PR]) {
      const float d = dA[tt];
      const float4 b0 = *reinterpret_cast<const float4*>(&bdt[tt][nb * 8]);
      const float4 b1 = *reinterpret_cast<const float4*>(&bdt[tt][nb * 8 + 4]);
      const float4 c0 = *reinterpret_cast<const float4*>(&cs[tt][nb * 8]);
      const float4 c1 = *reinterpret_cast<const float4*>(&cs[tt][nb * 8 + 4]);
      const float b[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      const float c[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
      for (int r = 0; r < PR; ++r) {
        const float x = xs[tt][pg * PR + r];
        float o0 = 0.f, o1 = 0.f;
#pragma unroll
        for (int k = 0; k < 8; k += 2) {
          st[r][k] = fmaf(st[r][k], d, b[k] * x);
          st[r][k + 1] = fmaf(st[r][k + 1], d, b[k + 1] * x);
          o0 = fmaf(st[r][k], c[k], o0);
          o1 = fmaf(st[r][k + 1], c[k + 1], o1);
        }
        v[r] = row16_sum(o0 + o1) + x * Dh;  // the 16 n-blocks of row p: 16 consecutive lanes
      }
    };
    bf16_t* yp = y + (size_t)(row0 + t0) * a.ldy + h * MB_HD + p0;
    int tt = 0;
    for (; tt + 4 <= nt; tt += 4) {
      float v[4][PR];
      step(tt, v[0]);
      step(tt + 1, v[1]);
      step(tt + 2, v[2]);
      step(tt + 3, v[3]);
      if (nb == 0)
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int r = 0; r < PR; ++r) yp[(size_t)(tt + u) * a.ldy + r] = (bf16_t)f2bf(v[u][r]);
    }
    for (; tt < nt; ++tt) {
      float v[PR];
      step(tt, v);
      if (nb == 0)
#pragma unroll
        for (int r = 0; r < PR; ++r) yp[(size_t)tt * a.ldy + r] = (bf16_t)f2bf(v[r]);
    }
    if (t0 / S2_TT < 12) ZMI_SSTAMP(2 + 2 * (t0 / S2_TT));
  }
  // final state, bf16 (the cache dtype): 8 consecutive n per row
#pragma unroll
  for (int r = 0; r < PR; ++r) {
    bf16_t* sp = reinterpret_cast<bf16_t*>(a.ssm) + (((size_t)kv * a.nheads + h) * MB_HD + p0 + r) * MB_DS + nb * 8;
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) w[e] = f2bf(st[r][2 * e]) | (f2bf(st[r][2 * e + 1]) << 16);
    *reinterpret_cast<uint4*>(sp) = uint4{w[0], w[1], w[2], w[3]};
  }
}

// ---------------------------------------------------------------------------- quadratic (SSD) prefill
// zmi_mamba2_scan_ws with ZMI_OPT_SCAN_PQ = 0, sequences of at most SSD_TMAX positions: the state-space dual of the
// recurrence (the matrix form mamba_chunk_scan_combined evaluates within a chunk; here the whole sequence is one chunk).
// With cum[t] = sum_{tau <= t} A dt_tau (the log of the decays' product),
//     y_t = sum_{s <= t} (C_t . B_s) exp(cum[t] - cum[s]) dt_s x_s + D x_t,
//     state = sum_s exp(cum[T-1] - cum[s]) dt_s x_s B_s^T   (the recurrence's final state),
// as MFMA tiles instead of T dependent steps. Two 1024-thread workgroups per (sequence, head): one writes y, 32 rows at
// a time (the next block's C rows loaded under the current block's tiles), the other the final state.
//   G = C_blk B^T          bf16 MFMA (B, C are the conv output, exactly bf16), fp32 sums;
//   M = G exp(cum_t - cum_s) dt_s (s <= t, else 0), fp32, then split M = hi + lo into two bf16 terms;
//   y = M_hi X + M_lo X    bf16 MFMA (x exactly bf16), fp32 sums, + D x, rounded to bf16;
//   state = W^T B with W[s][p] = exp(cum[T-1] - cum[s]) dt_s x_s[p] split the same way, rounded to bf16 (the cache dtype).
// cum is a fixed-shape scan (lane L owns positions 4L .. 4L + 3, lane totals by a shuffle scan) computed identically by
// every role. Arithmetic differs from the recurrence in fp32 rounding (and the hi / lo split keeps ~16 mantissa bits
// of M and W): checked against the oracle's recurrence like the scan forms.
constexpr int SSD_TB = 32;      // y rows per block of the y workgroup
constexpr int SSD_NT = 1024;    // threads: 16 waves
constexpr int SSD_TMAX = 256;   // longest sequence of this form
constexpr int SSD_BROW = MB_DS + 8;  // B / C row stride (bf16): 272 B, MFMA fragment reads spread over the banks
constexpr int SSD_XROW = MB_HD + 8;  // x / W row stride (bf16)

// Every operand stays row-major in LDS (position-major, as the workspace holds it: coalesced 16-byte copies, no
// transposing stores); an MFMA operand whose k runs over positions is gathered as 8 bf16 of one column (8 ds_read_u16).
struct SsdLds {
  int S32;  // positions rounded up to 32
  __device__ __host__ SsdLds(int T) : S32((T + 31) / 32 * 32) {}
  // y role: cum, dt | B rows [S32][SSD_BROW] | C rows [32][SSD_BROW] | M hi / lo [32][S32 + 8] | x rows [S32][SSD_XROW]
  __device__ __host__ int MP() const { return S32 + 8; }
  __device__ __host__ size_t b_off() const { return 2 * SSD_TMAX * 4; }
  __device__ __host__ size_t c_off() const { return b_off() + (size_t)S32 * SSD_BROW * 2; }
  __device__ __host__ size_t mh_off() const { return c_off() + (size_t)SSD_TB * SSD_BROW * 2; }
  __device__ __host__ size_t ml_off() const { return mh_off() + (size_t)SSD_TB * MP() * 2; }
  __device__ __host__ size_t x_off() const { return ml_off() + (size_t)SSD_TB * MP() * 2; }
  __device__ __host__ size_t y_bytes() const { return x_off() + (size_t)S32 * SSD_XROW * 2; }
  // state role: cum, dt | B rows [S32][SSD_BROW] | W hi / lo rows [S32][SSD_XROW]
  __device__ __host__ size_t wh_off() const { return b_off() + (size_t)S32 * SSD_BROW * 2; }
  __device__ __host__ size_t wl_off() const { return wh_off() + (size_t)S32 * SSD_XROW * 2; }
  __device__ __host__ size_t s_bytes() const { return wl_off() + (size_t)S32 * SSD_XROW * 2; }
};

__device__ __forceinline__ f32x4_t mfma_bf16(const uint4& a, const uint4& b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c, 0,
                                                 0, 0);
}

// 8 bf16 of one column, rows r .. r + 7 of a row-major LDS array (stride in elements), packed as an MFMA k-fragment
__device__ __forceinline__ uint4 gather8(const bf16_t* p, int stride) {
  const uint16_t* q = reinterpret_cast<const uint16_t*>(p);
  uint32_t w[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) w[e] = (uint32_t)q[(2 * e) * stride] | ((uint32_t)q[(2 * e + 1) * stride] << 16);
  return uint4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ uint32_t split_bf16(float v, uint32_t* lo) {
  const uint32_t h = f2bf(v);
  *lo = f2bf(v - bf2f(h));
  return h;
}

__global__ __launch_bounds__(SSD_NT) void mamba2_ssd_kernel(const ZmiMamba2Args a, int seq_len, const bf16_t* xc,
                                                         const float* dts) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int T = seq_len;
  const int role = blockIdx.x & 1, sh = blockIdx.x >> 1, h = sh % a.nheads, sq = sh / a.nheads;
  const int row0 = sq * T, conv_dim = a.d_ssm + 2 * MB_DS;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const SsdLds L(T);
  float* cum = reinterpret_cast<float*>(smem);
  float* dtl = cum + SSD_TMAX;
  const float Ah = a.A[h];
  const bool state_role = role == 1;
  const int s32 = L.S32;
  bf16_t* Bs = reinterpret_cast<bf16_t*>(smem + L.b_off());
  // (1) B rows s < s_end (zero to s32) for both roles; dt and cum for every position (the same fixed-shape scan in
  // every role: lane L owns positions 4L .. 4L + 3)
  for (int i = t; i < s32 * (MB_DS / 8); i += SSD_NT) {
    const int r = i / (MB_DS / 8), c = i % (MB_DS / 8);
    uint4 v = uint4{0u, 0u, 0u, 0u};
    if (r < T) v = *reinterpret_cast<const uint4*>(xc + (size_t)(row0 + r) * conv_dim + a.d_ssm + 8 * c);
    *reinterpret_cast<uint4*>(Bs + r * SSD_BROW + 8 * c) = v;
  }
  if (wave == 0) {
    float v[4], run = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = 4 * lane + i;
      const float d = q < T ? dts[(size_t)(row0 + q) * a.nheads + h] : 0.f;
      dtl[q] = d;
      run += Ah * d;
      v[i] = run;
    }
    float pre = run;  // inclusive scan of the lane totals
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const float o = __shfl_up(pre, d, 64);
      if (lane >= d) pre += o;
    }
    const float excl = pre - run;
#pragma unroll
    for (int i = 0; i < 4; ++i) cum[4 * lane + i] = excl + v[i];
  }
  if (!state_role) {
    bf16_t* Cs = reinterpret_cast<bf16_t*>(smem + L.c_off());
    bf16_t* Mh = reinterpret_cast<bf16_t*>(smem + L.mh_off());
    bf16_t* Ml = reinterpret_cast<bf16_t*>(smem + L.ml_off());
    bf16_t* Xs = reinterpret_cast<bf16_t*>(smem + L.x_off());
    const int MP = L.MP();
    // (2) x rows (zero to s32); the first row block's C rows into registers (2 x 16 B per thread), each later block's
    // loaded while the previous one computes
    for (int i = t; i < s32 * (MB_HD / 8); i += SSD_NT) {
      const int r = i / (MB_HD / 8), c = i % (MB_HD / 8);
      uint4 v = uint4{0u, 0u, 0u, 0u};
      if (r < T) v = *reinterpret_cast<const uint4*>(xc + (size_t)(row0 + r) * conv_dim + h * MB_HD + 8 * c);
      *reinterpret_cast<uint4*>(Xs + r * SSD_XROW + 8 * c) = v;
    }
    constexpr int CP = SSD_TB * (MB_DS / 8), CPT = (CP + SSD_NT - 1) / SSD_NT;  // C pieces (16 B), per thread
    uint4 cr[CPT];
    auto load_c = [&](int tb0) {
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        const int i = t + SSD_NT * j, r = i / (MB_DS / 8), c = i % (MB_DS / 8);
        cr[j] = i < CP && tb0 + r < T
                    ? *reinterpret_cast<const uint4*>(xc + (size_t)(row0 + tb0 + r) * conv_dim + a.d_ssm + MB_DS + 8 * c)
                    : uint4{0u, 0u, 0u, 0u};
      }
    };
    load_c(0);
    const float Dh = a.D[h];
    for (int t0 = 0; t0 < T; t0 += SSD_TB) {
      const int tn = min(SSD_TB, T - t0), s_end = t0 + tn, sk = (s_end + 31) / 32;  // k-blocks of 32 positions
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        const int i = t + SSD_NT * j, r = i / (MB_DS / 8), c = i % (MB_DS / 8);
        if (i < CP) *reinterpret_cast<uint4*>(Cs + r * SSD_BROW + 8 * c) = cr[j];
      }
      __syncthreads();  // C block (and, the first time, B / x / cum) visible; the previous block's y reads are done
      if (t0 + SSD_TB < T) load_c(t0 + SSD_TB);
      // (3) M tiles (16 t x 16 s) over s < 32 sk: G = C B^T on the tiles that reach s <= t, zeros elsewhere
      for (int tile = wave; tile < 4 * sk; tile += SSD_NT / 64) {
        const int ti = tile & 1, si = tile >> 1;
        const bool live = 16 * ti < tn && 16 * si <= t0 + 16 * ti + 15;
        f32x4_t g = {0.f, 0.f, 0.f, 0.f};
        if (live) {
#pragma unroll
          for (int kk = 0; kk < MB_DS / 32; ++kk) {
            const uint4 av = *reinterpret_cast<const uint4*>(Cs + (16 * ti + (lane & 15)) * SSD_BROW + 32 * kk + 8 * (lane >> 4));
            const uint4 bv = *reinterpret_cast<const uint4*>(Bs + (16 * si + (lane & 15)) * SSD_BROW + 32 * kk + 8 * (lane >> 4));
            g = mfma_bf16(av, bv, g);
          }
        }
        const int s = 16 * si + (lane & 15);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int tl = 16 * ti + 4 * (lane >> 4) + i, tt = t0 + tl;
          float m = 0.f;
          if (live && tl < tn && s <= tt) m = g[i] * expf(cum[tt] - cum[s]) * dtl[s];
          uint32_t lo;
          const uint32_t hi = split_bf16(m, &lo);
          Mh[tl * MP + s] = (bf16_t)hi;
          Ml[tl * MP + s] = (bf16_t)lo;
        }
      }
      __syncthreads();
      // (4) y tiles (16 t x 16 p): wave w < 8 -> t tile w & 1, p tile w >> 1; the x fragment of a k-block (8 consecutive
      // positions of column p) gathered from the row-major x rows
      const int ti = wave & 1;
      if (wave < 8 && 16 * ti < tn) {
        {
          const int pj = wave >> 1, p = 16 * pj + (lane & 15);
          f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
          for (int kk = 0; kk < sk; ++kk) {
            const int mo = (16 * ti + (lane & 15)) * MP + 32 * kk + 8 * (lane >> 4);
            const uint4 bv = gather8(Xs + (32 * kk + 8 * (lane >> 4)) * SSD_XROW + p, SSD_XROW);
            acc = mfma_bf16(*reinterpret_cast<const uint4*>(Mh + mo), bv, acc);
            acc = mfma_bf16(*reinterpret_cast<const uint4*>(Ml + mo), bv, acc);
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int tl = 16 * ti + 4 * (lane >> 4) + i;
            if (tl < tn) {
              const float x = bf2f((uint32_t)reinterpret_cast<const uint16_t*>(Xs)[(t0 + tl) * SSD_XROW + p]);
              reinterpret_cast<bf16_t*>(a.y)[(size_t)(row0 + t0 + tl) * a.ldy + h * MB_HD + p] =
                  (bf16_t)f2bf(acc[i] + x * Dh);
            }
          }
        }
      }
    }
  } else {
    bf16_t* Wh = reinterpret_cast<bf16_t*>(smem + L.wh_off());
    bf16_t* Wl = reinterpret_cast<bf16_t*>(smem + L.wl_off());
    __syncthreads();  // cum / dt
    const float cT = cum[T - 1];
    // (2) W rows [s][p] = exp(cum[T-1] - cum[s]) dt_s x_s[p] as hi / lo bf16, zero past T
    for (int i = t; i < s32 * (MB_HD / 8); i += SSD_NT) {
      const int r = i / (MB_HD / 8), c = i % (MB_HD / 8);
      uint32_t hv[4] = {0u, 0u, 0u, 0u}, lv[4] = {0u, 0u, 0u, 0u};
      if (r < T) {
        const uint4 v = *reinterpret_cast<const uint4*>(xc + (size_t)(row0 + r) * conv_dim + h * MB_HD + 8 * c);
        const float w = expf(cT - cum[r]) * dtl[r];
        const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          uint32_t l0, l1;
          const uint32_t h0 = split_bf16(w * bf2f(u[e]), &l0), h1 = split_bf16(w * bf2f(u[e] >> 16), &l1);
          hv[e] = h0 | (h1 << 16);
          lv[e] = l0 | (l1 << 16);
        }
      }
      *reinterpret_cast<uint4*>(Wh + r * SSD_XROW + 8 * c) = uint4{hv[0], hv[1], hv[2], hv[3]};
      *reinterpret_cast<uint4*>(Wl + r * SSD_XROW + 8 * c) = uint4{lv[0], lv[1], lv[2], lv[3]};
    }
    __syncthreads();
    // (3) state tiles (16 p x 16 n): wave w -> p tile w & 3, n tiles 4 (w >> 2) .. + 3; A = W^T and B fragments
    // gathered per k-block
    constexpr int NPW = MB_DS / 16 / (SSD_NT / 64 / 4);  // n tiles per wave
    const int kv = a.row_kv ? a.row_kv[row0] : sq;
    bf16_t* st = reinterpret_cast<bf16_t*>(a.ssm) + ((size_t)kv * a.nheads + h) * MB_HD * MB_DS;
    const int pi = wave & 3, nb = (wave >> 2) * NPW;
    f32x4_t acc[NPW];
#pragma unroll
    for (int ni = 0; ni < NPW; ++ni) acc[ni] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int kk = 0; kk < s32 / 32; ++kk) {
      const int r = 32 * kk + 8 * (lane >> 4);
      const uint4 ah = gather8(Wh + r * SSD_XROW + 16 * pi + (lane & 15), SSD_XROW);
      const uint4 al = gather8(Wl + r * SSD_XROW + 16 * pi + (lane & 15), SSD_XROW);
#pragma unroll
      for (int ni = 0; ni < NPW; ++ni) {
        const uint4 bv = gather8(Bs + r * SSD_BROW + 16 * (nb + ni) + (lane & 15), SSD_BROW);
        acc[ni] = mfma_bf16(ah, bv, acc[ni]);
        acc[ni] = mfma_bf16(al, bv, acc[ni]);
      }
    }
#pragma unroll
    for (int ni = 0; ni < NPW; ++ni) {
      const int n = 16 * (nb + ni) + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i) st[(size_t)(16 * pi + 4 * (lane >> 4) + i) * MB_DS + n] = (bf16_t)f2bf(acc[ni][i]);
    }
  }
}

// Row reductions of the two norms below: one 256-thread workgroup per row; the row is cut into NW
// contiguous parts (4, or K / 512 below K = 2048), wave w < NW owns part w, lane L its 8-element chunks
// L + 64 i; fp32 sums in chunk order, DPP wave sums, parts combined as (p0 + p1) + (p2 + p3) (absent parts
// add +0, exactly). A row's bits do not depend on M.
template <int K>
struct RowSplit {
  static constexpr int NW = K >= 2048 ? 4 : K / 512;
  static constexpr int CPL = K / (512 * NW);
  static_assert(NW >= 1 && CPL >= 1 && NW * CPL * 512 == K, "row split");
};
__device__ __forceinline__ float block_sum4(float v, float* part) {
  v = wave_sum(v);
  const int wave = threadIdx.x >> 6;
  __syncthreads();  // part[] may still be read by the previous reduction
  if ((threadIdx.x & 63) == 0) part[wave] = v;
  __syncthreads();
  return (part[0] + part[1]) + (part[2] + part[3]);
}

// ---------------------------------------------------------------------------- add + LayerNorm
// layer_norm_fn(x, w, b, residual, prenorm=True, residual_in_fp32=False) (mamba_ssm/ops/triton/
// layer_norm.py): s = x + residual in fp32; residual_out = bf16(s); y = (s - mean) * rstd * w + b on the
// fp32 sum (two-pass statistics).
template <int K>
__global__ __launch_bounds__(256) void add_ln_kernel(const bf16_t* hid, int ldh, bf16_t* res, int ldr,
                                                     const bf16_t* w, const bf16_t* b, float eps, bf16_t* out, int ldo,
                                                     int store_res) {
  constexpr int NW = RowSplit<K>::NW, CPL = RowSplit<K>::CPL;
  __shared__ float part[4];
  const int r = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const bool on = wave < NW;
  float v[CPL][8];
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
    if (!on) continue;
    const int c = wave * (K / (8 * NW)) + lane + 64 * i;  // 8-element chunk index in the row
    const uint4 rv = reinterpret_cast<const uint4*>(res + (size_t)r * ldr)[c];
    uint32_t u[4] = {rv.x, rv.y, rv.z, rv.w};
    uint32_t hu[4] = {0u, 0u, 0u, 0u};
    if (hid) {
      const uint4 hv = reinterpret_cast<const uint4*>(hid + (size_t)r * ldh)[c];
      hu[0] = hv.x; hu[1] = hv.y; hu[2] = hv.z; hu[3] = hv.w;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[i][2 * e] = hid ? bf2f(hu[e]) + bf2f(u[e]) : bf2f(u[e]);
      v[i][2 * e + 1] = hid ? bf2f(hu[e] >> 16) + bf2f(u[e] >> 16) : bf2f(u[e] >> 16);
      sum += v[i][2 * e] + v[i][2 * e + 1];
    }
    if (store_res && hid) {
#pragma unroll
      for (int e = 0; e < 4; ++e) u[e] = f2bf(v[i][2 * e]) | (f2bf(v[i][2 * e + 1]) << 16);
      reinterpret_cast<uint4*>(res + (size_t)r * ldr)[c] = uint4{u[0], u[1], u[2], u[3]};
    }
  }
  const float mean = block_sum4(sum, part) / (float)K;
  float sq = 0.f;  // pairs as (a + b): the GEMV ADDLN prologue's order (zmi_gemv_impl.h addln_chunk_sum)
#pragma unroll
  for (int i = 0; i < CPL; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d0 = v[i][2 * e] - mean, d1 = v[i][2 * e + 1] - mean;
      sq += on ? d0 * d0 + d1 * d1 : 0.f;
    }
  const float rstd = 1.0f / sqrtf(block_sum4(sq, part) / (float)K + eps);
  if (!on) return;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = wave * (K / (8 * NW)) + lane + 64 * i;
    const uint4 gw = reinterpret_cast<const uint4*>(w)[c], gb = reinterpret_cast<const uint4*>(b)[c];
    const uint32_t uw[4] = {gw.x, gw.y, gw.z, gw.w}, ub[4] = {gb.x, gb.y, gb.z, gb.w};
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float y0 = ((v[i][2 * e] - mean) * rstd) * bf2f(uw[e]) + bf2f(ub[e]);
      const float y1 = ((v[i][2 * e + 1] - mean) * rstd) * bf2f(uw[e] >> 16) + bf2f(ub[e] >> 16);
      o[e] = f2bf(y0) | (f2bf(y1) << 16);
    }
    reinterpret_cast<uint4*>(out + (size_t)r * ldo)[c] = uint4{o[0], o[1], o[2], o[3]};
  }
}

// ---------------------------------------------------------------------------- gated RMSNorm
// RMSNormGated(norm_before_gate=False, one group) (mamba_ssm/ops/triton/layernorm_gated.py):
// g = y * (z * sigmoid(z)) in fp32, out = g * rstd * w with rstd = 1 / sqrt(mean(g^2) + eps), bf16.
template <int K>
__global__ __launch_bounds__(256) void gated_rms_kernel(const bf16_t* y, int ldy, const bf16_t* z, int ldz,
                                                        const bf16_t* w, float eps, bf16_t* out, int ldo) {
  constexpr int NW = RowSplit<K>::NW, CPL = RowSplit<K>::CPL;
  __shared__ float part[4];
  const int r = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const bool on = wave < NW;
  float g[CPL][8];
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
#pragma unroll
    for (int e = 0; e < 8; ++e) g[i][e] = 0.f;
    if (!on) continue;
    const int c = wave * (K / (8 * NW)) + lane + 64 * i;
    const uint4 yv = reinterpret_cast<const uint4*>(y + (size_t)r * ldy)[c];
    const uint4 zv = reinterpret_cast<const uint4*>(z + (size_t)r * ldz)[c];
    const uint32_t uy[4] = {yv.x, yv.y, yv.z, yv.w}, uz[4] = {zv.x, zv.y, zv.z, zv.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float zz = bf2f(uz[e >> 1] >> (16 * (e & 1)));
      const float sg = 1.0f / (1.0f + expf(-zz));
      g[i][e] = bf2f(uy[e >> 1] >> (16 * (e & 1))) * (zz * sg);
      sq += g[i][e] * g[i][e];
    }
  }
  const float rstd = 1.0f / sqrtf(block_sum4(sq, part) / (float)K + eps);
  if (!on) return;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = wave * (K / (8 * NW)) + lane + 64 * i;
    const uint4 gw = reinterpret_cast<const uint4*>(w)[c];
    const uint32_t uw[4] = {gw.x, gw.y, gw.z, gw.w};
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      o[e] = f2bf((g[i][2 * e] * rstd) * bf2f(uw[e])) | (f2bf((g[i][2 * e + 1] * rstd) * bf2f(uw[e] >> 16)) << 16);
    reinterpret_cast<uint4*>(out + (size_t)r * ldo)[c] = uint4{o[0], o[1], o[2], o[3]};
  }
}

int check_mamba(const ZmiMamba2Args* a) {
  if (!a || !a->zxbcdt || !a->conv_w || !a->conv_b || !a->dt_bias || !a->A || !a->D || !a->conv_ring || !a->ssm ||
      !a->y || !a->row_pos)
    return zmi_fail_msg("mamba2: missing buffers");
  if (a->headdim != MB_HD || a->d_state != MB_DS || a->d_conv != MB_DC || a->ngroups != 1)
    return zmi_fail_msg("mamba2: built for headdim 64, d_state 128, d_conv 4, ngroups 1");
  if (a->nheads <= 0 || a->d_ssm != a->nheads * MB_HD) return zmi_fail_msg("mamba2: d_ssm = nheads x 64");
  if (a->ld_zx < 2 * a->d_ssm + 2 * MB_DS + a->nheads || a->ldy < a->d_ssm)
    return zmi_fail_msg("mamba2: ld_zx >= 2 d_ssm + 2 d_state + nheads, ldy >= d_ssm");
  return 0;
}

}  // namespace

extern "C" int zmi_mamba2_step(const ZmiMamba2Args* a, void* stream) {
  if (int e = check_mamba(a)) return e;
  if (a->M <= 0) return 0;
  hipLaunchKernelGGL(mamba2_step_kernel, dim3((unsigned)(a->M * a->nheads)), dim3(MB_ST), 0, (hipStream_t)stream, *a);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_mamba2_scan(const ZmiMamba2Args* a, int seq_len, void* stream) {
  if (int e = check_mamba(a)) return e;
  if (seq_len <= 0 || a->M % seq_len) return zmi_fail_msg("mamba2_scan: M must be a multiple of seq_len > 0");
  hipLaunchKernelGGL(mamba2_scan_kernel, dim3((unsigned)(a->M / seq_len * a->nheads)), dim3(MB_NT), 0,
                     (hipStream_t)stream, *a, seq_len);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int64_t zmi_mamba2_scan_ws_bytes(int m, int d_ssm, int nheads) {
  if (m <= 0 || d_ssm <= 0 || nheads <= 0) return 0;
  const int64_t xc = ((int64_t)m * (d_ssm + 2 * MB_DS) * 2 + 255) / 256 * 256;
  return xc + 2 * (((int64_t)m * nheads * 4 + 255) / 256 * 256);
}

extern "C" int zmi_mamba2_scan_ws(const ZmiMamba2Args* a, int seq_len, void* ws, int64_t ws_bytes, void* stream) {
  if (int e = check_mamba(a)) return e;
  if (seq_len <= 0 || a->M % seq_len) return zmi_fail_msg("mamba2_scan_ws: M must be a multiple of seq_len > 0");
  if (!ws || ws_bytes < zmi_mamba2_scan_ws_bytes(a->M, a->d_ssm, a->nheads))
    return zmi_fail_msg("mamba2_scan_ws: workspace smaller than zmi_mamba2_scan_ws_bytes");
  const int64_t xcb = ((int64_t)a->M * (a->d_ssm + 2 * MB_DS) * 2 + 255) / 256 * 256;
  const int64_t hb = ((int64_t)a->M * a->nheads * 4 + 255) / 256 * 256;
  bf16_t* xc = (bf16_t*)ws;
  float* dts = (float*)((char*)ws + xcb);
  float* das = (float*)((char*)ws + xcb + hb);
  hipStream_t s = (hipStream_t)stream;
  const int conv_dim = a->d_ssm + 2 * MB_DS;
  hipLaunchKernelGGL(mamba2_conv_kernel, dim3((unsigned)a->M, (unsigned)((conv_dim + 255) / 256)), dim3(256), 0, s, *a,
                     seq_len, xc, dts, das);
  ZMI_CHECK(hipGetLastError());
  const int pq = zmi_option(ZMI_OPT_SCAN_PQ);
  if (pq == 0 && seq_len <= SSD_TMAX) {  // the quadratic (SSD) form
    const SsdLds L(seq_len);
    const size_t lds = std::max(L.y_bytes(), L.s_bytes());
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&mamba2_ssd_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    ZMI_CHECK(attr);
    hipLaunchKernelGGL(mamba2_ssd_kernel, dim3((unsigned)(a->M / seq_len * a->nheads * 2)), dim3(SSD_NT), lds, s, *a,
                       seq_len, (const bf16_t*)xc, (const float*)dts);
    ZMI_CHECK(hipGetLastError());
    return 0;
  }
  const dim3 grid((unsigned)(a->M / seq_len * a->nheads * (pq == 0 ? 4 : pq)));
  if (pq == 1)
    hipLaunchKernelGGL(mamba2_scan2_kernel<1>, grid, dim3(256), 0, s, *a, seq_len, (const bf16_t*)xc,
                       (const float*)dts, (const float*)das);
  else if (pq == 2)
    hipLaunchKernelGGL(mamba2_scan2_kernel<2>, grid, dim3(256), 0, s, *a, seq_len, (const bf16_t*)xc,
                       (const float*)dts, (const float*)das);
  else if (pq == 4 || pq == 0)  // 0: sequences past the quadratic form's reach
    hipLaunchKernelGGL(mamba2_scan2_kernel<4>, grid, dim3(256), 0, s, *a, seq_len, (const bf16_t*)xc,
                       (const float*)dts, (const float*)das);
  else
    return zmi_fail_msg("mamba2_scan_ws: ZMI_OPT_SCAN_PQ must be 1, 2 or 4");
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_add_layernorm(const void* hidden, int ldh, void* residual, int ldr, int m, int k, const void* w,
                                 const void* b, float eps, void* out, int ldo, int store_residual, void* stream) {
  if (ldh % 8 || ldr % 8 || ldo % 8) return zmi_fail_msg("add_layernorm: leading dimensions must be multiples of 8");
  if (!residual || !w || !b || !out) return zmi_fail_msg("add_layernorm: missing buffers");
  if (m <= 0) return 0;
  const dim3 grid((unsigned)m);
  hipStream_t s = (hipStream_t)stream;
#define ZMI_ADDLN(KK)                                                                                         \
  hipLaunchKernelGGL(add_ln_kernel<KK>, grid, dim3(256), 0, s, (const bf16_t*)hidden, ldh, (bf16_t*)residual, \
                     ldr, (const bf16_t*)w, (const bf16_t*)b, eps, (bf16_t*)out, ldo, store_residual)
  switch (k) {
    case 512: ZMI_ADDLN(512); break;
    case 1024: ZMI_ADDLN(1024); break;
    case 2048: ZMI_ADDLN(2048); break;
    case 4096: ZMI_ADDLN(4096); break;
    default: return zmi_fail_msg("add_layernorm: k must be 512, 1024, 2048 or 4096");
  }
#undef ZMI_ADDLN
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_gated_rmsnorm(const void* y, int ldy, const void* z, int ldz, int m, int k, const void* w,
                                 float eps, void* out, int ldo, void* stream) {
  if (ldy % 8 || ldz % 8 || ldo % 8) return zmi_fail_msg("gated_rmsnorm: leading dimensions must be multiples of 8");
  if (!y || !z || !w || !out) return zmi_fail_msg("gated_rmsnorm: missing buffers");
  if (m <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
#define ZMI_GRMS(KK)                                                                                          \
  hipLaunchKernelGGL(gated_rms_kernel<KK>, dim3((unsigned)m), dim3(256), 0, s, (const bf16_t*)y, ldy,         \
                     (const bf16_t*)z, ldz, (const bf16_t*)w, eps, (bf16_t*)out, ldo)
  switch (k) {
    case 512: ZMI_GRMS(512); break;
    case 1024: ZMI_GRMS(1024); break;
    case 2048: ZMI_GRMS(2048); break;
    case 4096: ZMI_GRMS(4096); break;
    default: return zmi_fail_msg("gated_rmsnorm: k must be 512, 1024, 2048 or 4096");
  }
#undef ZMI_GRMS
  ZMI_CHECK(hipGetLastError());
  return 0;
}
