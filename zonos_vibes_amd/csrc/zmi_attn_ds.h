// Decode attention, whole-query form: shared by the standalone kernel (zmi_attn.hip, variant 4 / 8)
// and the attention workgroups of the fused QKV + attention launch (zmi_attnblk.hip).
//
// One workgroup of DNW waves per (query, kv head, slice of HD / DS output dims) covers EVERY key of
// its query: all scores and softmax statistics (K is read by each of the DS slices of a unit; they
// share one XCD under round-robin placement, so most of them read it from L2), and P.V for its own
// dims only. No workgroup waits on another. The arithmetic is zmi_attn.hip's chunked kernel's,
// operation for operation, so every variant returns identical bits and the launcher may pick any:
//   * scores per 32-key group: the same 4-MFMA chain over the same operand layout;
//   * chunk maxima over CH keys; M_j over the chunks of blocks 0..j (max is exact);
//   * per chunk and head: lane L takes keys L, L + 64 (e = 0 past the position), wave_sum -> l_c;
//   * P.V per 32-key group from a zero accumulator, chunk o = group sums in group order (groups
//     wholly past the position contribute +0 there, which is the identity: an MFMA from a +0
//     accumulator never returns -0, so they are skipped here);
//   * zmi_attn_merge.h's block recursion per (head, dim).
// Keys up to DS_KEYS: a wave holds the K and V^T fragments of all its groups (DKM per wave) in
// registers, all issued before the first MFMA.

#pragma once
#include "zmi_common.h"
#include "zmi_kernels.h"
#include "zmi_attn_merge.h"

// Diagnostic build only (-DZMI_ATTN_STAMPS, tools/attn_stamps.py): thread 0 of every workgroup
// writes s_memrealtime (100 MHz) at phase boundaries into a.stamps[block][8]; the real kernel has none.
#ifdef ZMI_ATTN_STAMPS
#define ZMI_ASTAMP(i)                                                                                    \
  do {                                                                                                   \
    if (threadIdx.x == 0 && a.stamps) a.stamps[(size_t)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define ZMI_ASTAMP(i) \
  do {                \
  } while (0)
#endif

namespace zmi_attn {

struct AttnArgs {
  const bf16_t* q;
  int ldq;
  const bf16_t* k;
  const bf16_t* v;
  const int* kv_row;
  const int* pos;
  int hkv, smax, nch;
  float scale;
  bf16_t* out;
  int ldo;
  unsigned* err;       // nonzero after a hand-off poll gave up
  unsigned* tickets;   // [unit]
  uint64_t* gran;      // [unit][nch][G]   {chunk max, tag}
  float* part_o;       // [unit][nch][G][HD]
  float* part_lm;      // [unit][nch][G][2]   l, M_j
  unsigned long long* stamps;  // diagnostic build only
  ZmiPrefetch pf;      // chunked kernel, one-launch form: prefetch-only workgroups after the n_att chunk ones
  int n_att, n_pf;
  int xc_l2;           // zmi_attn_block chunk-split form: hand-offs inside a unit through the XCD's L2 (ZMI_OPT_XC_HANDOFF)
};

__device__ __forceinline__ f32x4_t mfma16(const uint4& a, const uint4& b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

constexpr int DNW = 8;                    // waves per workgroup
constexpr int DKM = 5;                    // 32-key groups per wave
constexpr int DS_KEYS = 32 * DNW * DKM;   // 1280 keys (positions 0..1279)
constexpr int DS_CH = DS_KEYS / CH;       // chunks
constexpr int DS_BLK = (DS_KEYS + BLK - 1) / BLK;
constexpr unsigned DS_SPIN_LIMIT = 1u << 18;

template <int G, int DS>
struct DsImg {
  static constexpr int DSD = HD / DS;
  static constexpr int NG = DNW * DKM;
  static constexpr size_t SC = 0;                                      // float [G][DS_KEYS]
  static constexpr size_t PB = SC + (size_t)G * DS_KEYS * 4;           // bf16  [G][DS_KEYS]
  static constexpr size_t OP = PB + (size_t)G * DS_KEYS * 2;           // float [NG][G][DSD]
  static constexpr size_t MJ = OP + (size_t)NG * G * DSD * 4;          // float [DS_CH][G]
  static constexpr size_t LJ = MJ + (size_t)DS_CH * G * 4;             // float [DS_CH][G]
  static constexpr size_t MB = LJ + (size_t)DS_CH * G * 4;             // float [DS_BLK][G]
  static constexpr size_t BYTES = (MB + (size_t)DS_BLK * G * 4 + 15) / 16 * 16;
};

// Everything after the scores: sc[G][key] (scaled fp32 scores of keys 0..pos) is in LDS and the
// workgroup's V^T fragments of its dim slice are in vf (group k = wave + DNW r). Chunk maxima, M_j,
// e / l / P, P.V of the slice, chunk sums and the block recursion, output of the slice's dims.
// V^T fragments: group k is held by wave W0 + (k % NWK) as vf[k / NWK] (VR rounds); waves below W0
// hold none. Which wave multiplies a group does not change any sum (the merge orders by group).
template <int G, int DS, int W0 = 0, int NWK = DNW, int VR = DKM>
__device__ __forceinline__ void ds_tail(const AttnArgs& a, char* smem, uint4 (&vf)[VR][8 / DS], int qi, int kh,
                                        int s, int pos) {
  constexpr int CPG = CH / 32;     // 32-key groups per chunk (the chunked kernel's waves)
  constexpr int DT = 8 / DS;       // 16-dim MFMA column tiles per slice
  using I = DsImg<G, DS>;
  constexpr int DSD = I::DSD;
  float(&sc)[G][DS_KEYS] = *reinterpret_cast<float(*)[G][DS_KEYS]>(smem + I::SC);
  bf16_t(&pb)[G][DS_KEYS] = *reinterpret_cast<bf16_t(*)[G][DS_KEYS]>(smem + I::PB);
  float(&opart)[I::NG][G][DSD] = *reinterpret_cast<float(*)[I::NG][G][DSD]>(smem + I::OP);
  float(&mjc)[DS_CH][G] = *reinterpret_cast<float(*)[DS_CH][G]>(smem + I::MJ);
  float(&ljc)[DS_CH][G] = *reinterpret_cast<float(*)[DS_CH][G]>(smem + I::LJ);
  float(&mblk)[DS_BLK][G] = *reinterpret_cast<float(*)[DS_BLK][G]>(smem + I::MB);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c16 = lane & 15, h4 = lane >> 4;
  const int nk = pos + 1, n32 = (nk + 31) >> 5, nc = pos / CH + 1;
  ZMI_ASTAMP(3);
  // Softmax statistics. A wave takes the (chunk, head) tasks wave + DNW i; its tasks run interleaved
  // (independent LDS reads and DPP reductions), each with the chunked kernel's per-task arithmetic.
  constexpr int NTASK = (DS_CH * G + DNW - 1) / DNW;
  const int ntask = nc * G;
  {  // chunk maxima
    float m[NTASK];
#pragma unroll
    for (int i = 0; i < NTASK; ++i) {
      const int task = wave + DNW * i, c = task / G, g = task - c * G;
      m[i] = -INFINITY;
      if (task < ntask) {
#pragma unroll
        for (int ii = 0; ii < CH / 64; ++ii) {
          const int key = c * CH + lane + 64 * ii;
          m[i] = fmaxf(m[i], key < nk ? sc[g][key] : -INFINITY);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NTASK; ++i) m[i] = wave_max(m[i]);
#pragma unroll
    for (int i = 0; i < NTASK; ++i) {
      const int task = wave + DNW * i, c = task / G, g = task - c * G;
      if (task < ntask && lane == 0) mjc[c][g] = m[i];
    }
  }
  __syncthreads();
  ZMI_ASTAMP(4);
  {  // M_j = max over the chunks of blocks 0..j; e = exp(s - M_j), l per chunk, P = bf16(e)
    float l[NTASK];
#pragma unroll
    for (int i = 0; i < NTASK; ++i) {
      const int task = wave + DNW * i, c = task / G, g = task - c * G;
      l[i] = 0.f;
      if (task < ntask) {
        const int j = c / CPB, dep = min((j + 1) * CPB, nc);
        const float M = wave_max(lane < dep ? mjc[lane][g] : -INFINITY);  // exact: max is order-free
        if (c % CPB == 0 && lane == 0) mblk[j][g] = M;
#pragma unroll
        for (int ii = 0; ii < CH / 64; ++ii) {
          const int key = c * CH + lane + 64 * ii;
          const float e = key < nk ? expf(sc[g][key] - M) : 0.f;
          l[i] += e;
          pb[g][key] = (bf16_t)f2bf(e);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NTASK; ++i) l[i] = wave_sum(l[i]);
#pragma unroll
    for (int i = 0; i < NTASK; ++i) {
      const int task = wave + DNW * i, c = task / G, g = task - c * G;
      if (task < ntask && lane == 0) ljc[c][g] = l[i];
    }
  }
  __syncthreads();
  ZMI_ASTAMP(5);
  // P.V of this slice's dims, per live group
#pragma unroll
  for (int r = 0; r < VR; ++r) {
    const int k = (wave - W0) + NWK * r;
    if (wave >= W0 && k < n32) {
      uint4 pf = uint4{0u, 0u, 0u, 0u};
      if (c16 < G) pf = *reinterpret_cast<const uint4*>(&pb[c16][32 * k + 8 * h4]);
      const int kbase = 32 * k + 8 * h4;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        uint4 v = vf[r][dt];
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
        const f32x4_t o = mfma16(pf, v, f32x4_t{0.f, 0.f, 0.f, 0.f});
        if (h4 == 0) {
#pragma unroll
          for (int i = 0; i < G; ++i) opart[k][i][16 * dt + c16] = o[i];
        }
      }
    }
  }
  __syncthreads();
  ZMI_ASTAMP(6);
  // chunk sums and the block recursion (zmi_attn_merge.h), one thread per (head, dim of the slice);
  // the chunk loop is unrolled to its bound so every LDS read issues ahead of the dependent adds
  if (t < G * DSD) {
    const int g = t / DSD, dl = t - g * DSD;
    float acc = 0.f, l = 0.f, ob = 0.f, lb = 0.f, mprev = 0.f, mb = 0.f;
#pragma unroll
    for (int c = 0; c < DS_CH; ++c) {
      if (c < nc) {
        float oc = opart[CPG * c][g][dl];
#pragma unroll
        for (int w = 1; w < CPG; ++w)
          if (CPG * c + w < n32) oc += opart[CPG * c + w][g][dl];
        if (c % CPB == 0) {
          ob = oc;
          lb = ljc[c][g];
          mb = mblk[c / CPB][g];
        } else {
          ob += oc;
          lb += ljc[c][g];
        }
        if (c % CPB == CPB - 1 || c == nc - 1) {
          if (c < CPB) {
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
    }
    const float rl = 1.0f / l;
    a.out[(size_t)qi * a.ldo + (kh * G + g) * HD + DSD * s + dl] = (bf16_t)f2bf(acc * rl);
  }
  ZMI_ASTAMP(7);
}

// b = the workgroup's index in the (query, kv head, slice) grid; the DS slices of a unit take ids
// 8 apart (one XCD, speed only)
template <int G, int DS>
__device__ __forceinline__ void ds_body(const AttnArgs& a, int n_units, int b, char* smem) {
  constexpr int CPG = CH / 32;     // 32-key groups per chunk (the chunked kernel's waves)
  constexpr int DT = 8 / DS;       // 16-dim MFMA column tiles per slice
  using I = DsImg<G, DS>;
  float(&sc)[G][DS_KEYS] = *reinterpret_cast<float(*)[G][DS_KEYS]>(smem + I::SC);

  const int y = b >> 3;
  const int s = y % DS, unit = 8 * (y / DS) + (b & 7);
  if (unit >= n_units) return;
  const int qi = unit / a.hkv, kh = unit - qi * a.hkv;
  const int pos = a.pos[qi];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (pos < 0) return;
  ZMI_ASTAMP(0);
  const int c16 = lane & 15, h4 = lane >> 4;
  const int kvr = a.kv_row ? a.kv_row[qi] : qi;
  const size_t kvbase = ((size_t)kvr * a.hkv + kh) * a.smax * HD;
  const int nk = pos + 1, n32 = (nk + 31) >> 5, nc = pos / CH + 1;

  // every K and V^T fragment of this wave's groups k = wave + DNW r, in flight at once
  uint4 kf[DKM][2][4], vf[DKM][DT];
#pragma unroll
  for (int r = 0; r < DKM; ++r) {
    const int k = wave + DNW * r;
    if (k < n32) {
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int key = min(32 * k + 16 * tt + c16, pos);
        const bf16_t* kr = a.k + kvbase + (size_t)key * HD + 8 * h4;
#pragma unroll
        for (int db = 0; db < 4; ++db) kf[r][tt][db] = *reinterpret_cast<const uint4*>(kr + 32 * db);
      }
      const int p0 = min(32 * k + 8 * h4, pos & ~7);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
        vf[r][dt] = *reinterpret_cast<const uint4*>(a.v + kvbase + (size_t)(16 * (DT * s + dt) + c16) * a.smax + p0);
    }
  }
  uint4 qf[4];
  {
    const bool real = c16 < G;
    const bf16_t* qr = a.q + (size_t)qi * a.ldq + (kh * G + (real ? c16 : 0)) * HD + 8 * h4;
#pragma unroll
    for (int db = 0; db < 4; ++db)
      qf[db] = real ? *reinterpret_cast<const uint4*>(qr + 32 * db) : uint4{0u, 0u, 0u, 0u};
  }
  // scores of every live key (keys past the position stay out of every max / sum below)
#pragma unroll
  for (int r = 0; r < DKM; ++r) {
    const int k = wave + DNW * r;
    if (k < n32) {
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        f32x4_t sv = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int db = 0; db < 4; ++db) sv = mfma16(qf[db], kf[r][tt][db], sv);
        const int key = 32 * k + 16 * tt + c16;
        if (h4 == 0) {
#pragma unroll
          for (int i = 0; i < G; ++i) sc[i][key] = sv[i] * a.scale;
        }
      }
    }
  }
  __syncthreads();
  ds_tail<G, DS>(a, smem, vf, qi, kh, s, pos);
}

}  // namespace zmi_attn
