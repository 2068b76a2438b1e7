// Fused QKV projection + decode attention: ONE launch for reference zonos/backbone/_torch.py:114-136
// (norm -> in_proj -> rotary -> KV-cache update -> scaled_dot_product_attention) of a decode step.
//
// Why: as separate launches the attention paid a kernel boundary plus its own K / V load latency,
// ~12 us per layer at C2 against ~6 us for the projection before it. One CU moves only ~64 KB at a
// time (~20-40 GB/s), so a query's 300 KB of K / V (position 591) must be spread over several CUs,
// and those CUs must then combine results. Here the attention workgroups are extra workgroups of the
// projection's launch: they load their share of the cached K / V (positions < pos, written by
// earlier launches) at launch start, under the projection's weight stream, and the hand-offs are
// 8-byte {value, tag} granules (cdna_hip_programming.md §6 Guideline 16 R2: the data is its own
// flag; tag = position + 1, so consecutive steps never mistake each other's granules and nothing is
// re-armed; a row that starts a new utterance has its granules zeroed by the engine):
//   1. projection -> attention: every bf16 pair of q and of the new K / V row (zmi_gemv_impl.h);
//   2. attention -> attention: each of the S workgroups of a (query, kv head) computes the scores of
//      every S-th 32-key group and publishes them; every workgroup gathers all scores, then runs the
//      softmax and P.V for its own HD / S output dims (zmi_attn_ds.h ds_tail).
// Roles by block index (dispatch runs in index order, so a waiting attention workgroup never holds
// a slot a projection workgroup still needs; every spin is bounded and reports to `err`):
//   [0, n_qkv)           gemv_body (zmi_gemv_impl.h): LayerNorm prologue, the QKV projection for 16
//                        columns, epilogue RoPE + KV-cache write + granules;
//   [n_qkv, +units x S)  xs_body below.
// The arithmetic is the separate kernels' operation for operation (bit-identical outputs, tested);
// both roles run 512-thread workgroups: the projection with G = 2 groups x W = 4 waves, the K = 2048
// shape every launch form uses.
#include <algorithm>

#include "zmi_common.h"
#include "zmi_kernels.h"
#include "zmi_gemv_impl.h"
#include "zmi_prefetch.h"
#include "zmi_attn_ds.h"

namespace {

using namespace zmi_attn;
constexpr int QG = 2, QW = 4, QNL = 8, QRT = 16;  // the projection role's gemv_body shape
static_assert(QG * QW == DNW, "both roles run the same block size");
constexpr int XG = 4;                         // query heads per kv head
// the chunk-split form's hand-offs inside a (row, kv head) unit go through the XCD's L2 (st_xc64, zmi_common.h)
constexpr int QKV_GRAN = (XG + 2) * HD / 2;   // q pairs | k pairs | v pairs per (row, kv head)
constexpr int XC_CH_MAX = 24;                 // widest chunk-split form (chunk workgroups per unit)
// its granules (layout below: maxima, l, M_j, P.V partials), then the fused out_proj role's output granules and
// merge flags
constexpr int XC_WORDS_MAX = 3 * XC_CH_MAX * XG + XC_CH_MAX * XG * HD + XG * HD / 2 + HD / 16;
// + the score granules [XG][DS_KEYS] of the score-exchange forms, or the chunk-split form's granules
constexpr int GRAN_STRIDE = QKV_GRAN + (XG * DS_KEYS > XC_WORDS_MAX ? XG * DS_KEYS : XC_WORDS_MAX);
constexpr int NT = DNW * 64;
constexpr unsigned XS_SPIN = 1u << 16;

__device__ __forceinline__ uint32_t tag_of(uint64_t g) { return (uint32_t)(g >> 32); }

__device__ __forceinline__ void give_up(const AttnArgs& a) {
  __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave 0 of an attention workgroup only receives the projection's granules (it issues no K / V
// loads, so its polls are not queued behind them); waves 1..7 ("workers") hold the K / V fragments.
// Worker ww owns the 128-key chunks c = ww + XNWK rc: the V^T fragments of their four 32-key groups
// (its P.V sums a chunk's groups in group order in registers: the chunked kernel's chunk sum).
constexpr int XNWK = DNW - 1;                         // worker waves
constexpr int XCH = DS_KEYS / CH;                     // chunks
constexpr int XRC = (XCH + XNWK - 1) / XNWK;          // chunks per worker
constexpr int CPG = CH / 32;                          // 32-key groups per chunk
constexpr int XKPT = (DS_KEYS + NT - 1) / NT;         // keys per thread in the score gather

template <int S>
struct XsImg {
  static constexpr int DSD = HD / S;
  static constexpr size_t SC = 0;                                   // float [XG][DS_KEYS] scores
  static constexpr size_t PB = SC + (size_t)XG * DS_KEYS * 4;       // bf16  [XG][DS_KEYS] P
  static constexpr size_t OC = PB + (size_t)XG * DS_KEYS * 2;       // float [XCH][XG][DSD] chunk P.V
  static constexpr size_t MJ = OC + (size_t)XCH * XG * DSD * 4;     // float [XCH][XG] chunk maxima
  static constexpr size_t LJ = MJ + (size_t)XCH * XG * 4;           // float [XCH][XG] chunk exp sums
  static constexpr size_t MB = LJ + (size_t)XCH * XG * 4;           // float [DS_BLK][XG] M_j
  static constexpr size_t QKV = MB + (size_t)DS_BLK * XG * 4;       // u32 [QKV_GRAN] q | k | v pairs of pos
  static constexpr size_t BYTES = (QKV + (size_t)QKV_GRAN * 4 + 15) / 16 * 16;
};

template <int S>
__device__ __forceinline__ void xs_body(const AttnArgs& a, int n_units, int b, char* smem, uint64_t* gran) {
  constexpr int OWN = (DS_KEYS / 32 + S - 1) / S;       // score groups of one workgroup
  constexpr int KPW = (OWN + XNWK - 1) / XNWK;          // score groups per worker wave
  constexpr int DT = 8 / S;
  using I = XsImg<S>;
  constexpr int DSD = I::DSD;
  float(&sc)[XG][DS_KEYS] = *reinterpret_cast<float(*)[XG][DS_KEYS]>(smem + I::SC);
  bf16_t(&pb)[XG][DS_KEYS] = *reinterpret_cast<bf16_t(*)[XG][DS_KEYS]>(smem + I::PB);
  float(&ocs)[XCH][XG][DSD] = *reinterpret_cast<float(*)[XCH][XG][DSD]>(smem + I::OC);
  float(&mjc)[XCH][XG] = *reinterpret_cast<float(*)[XCH][XG]>(smem + I::MJ);
  float(&ljc)[XCH][XG] = *reinterpret_cast<float(*)[XCH][XG]>(smem + I::LJ);
  float(&mblk)[DS_BLK][XG] = *reinterpret_cast<float(*)[DS_BLK][XG]>(smem + I::MB);
  uint32_t* qkv_lds = reinterpret_cast<uint32_t*>(smem + I::QKV);

  const int y = b >> 3;
  const int s = y % S, unit = 8 * (y / S) + (b & 7);
  if (unit >= n_units) return;
  const int qi = unit / a.hkv, kh = unit - qi * a.hkv;
  const int pos = a.pos[qi];
  if (pos < 0) return;
  if (pos >= DS_KEYS) {  // the engine never launches this form past its capacity; refuse, don't read past it
    if (threadIdx.x == 0) give_up(a);
    return;
  }
  ZMI_ASTAMP(0);
  const uint32_t tag = (uint32_t)pos + 1u;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, ww = wave - 1;
  const int c16 = lane & 15, h4 = lane >> 4;
  const int kvr = a.kv_row ? a.kv_row[qi] : qi;
  const size_t kvbase = ((size_t)kvr * a.hkv + kh) * a.smax * HD;
  const int nk = pos + 1, n32 = (pos + 32) >> 5, nc = pos / CH + 1;
  uint64_t* gu = gran + (size_t)unit * GRAN_STRIDE;  // unit = query row x hkv + kv head, as the producers index
  uint64_t* gs = gu + QKV_GRAN;

  // (1) workers: the cached K rows of the workgroup's score groups k = s + S (ww + XNWK j) and the
  // V^T fragments of their chunks' groups (dim slice s): positions < pos only
  const int pc = max(pos - 1, 0);
  uint4 kf[KPW][2][4], vf[XRC][CPG][DT];
  if (wave > 0) {
#pragma unroll
    for (int j = 0; j < KPW; ++j) {
      const int k = s + S * (ww + XNWK * j);
      if (ww + XNWK * j < OWN && k < n32) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const bf16_t* kr = a.k + kvbase + (size_t)min(32 * k + 16 * tt + c16, pc) * HD + 8 * h4;
#pragma unroll
          for (int db = 0; db < 4; ++db) kf[j][tt][db] = *reinterpret_cast<const uint4*>(kr + 32 * db);
        }
      }
    }
#pragma unroll
    for (int rc = 0; rc < XRC; ++rc)
#pragma unroll
      for (int q4 = 0; q4 < CPG; ++q4) {
        const int k = CPG * (ww + XNWK * rc) + q4;
        if (k < n32) {
          const int p0 = min(32 * k + 8 * h4, pos & ~7);
#pragma unroll
          for (int dt = 0; dt < DT; ++dt)
            vf[rc][q4][dt] =
                *reinterpret_cast<const uint4*>(a.v + kvbase + (size_t)(16 * (DT * s + dt) + c16) * a.smax + p0);
        }
      }
  } else {
    // (2) wave 0: this position's q, K row and V row (QKV_GRAN pairs; 6 per lane), polled with two
    // sweeps in flight a fraction of a round trip apart, then staged in LDS for the workers
    uint64_t A[6], B[6];
    auto sweep = [&](uint64_t(&g)[6]) {
#pragma unroll
      for (int i = 0; i < 6; ++i) g[i] = ld_wt64(gu + lane + 64 * i);
    };
    auto ready = [&](const uint64_t(&g)[6]) {
      bool ok = true;
#pragma unroll
      for (int i = 0; i < 6; ++i) ok = ok && tag_of(g[i]) == tag;
      return __all(ok);
    };
    auto stage = [&](const uint64_t(&g)[6]) {
#pragma unroll
      for (int i = 0; i < 6; ++i) qkv_lds[lane + 64 * i] = (uint32_t)g[i];
    };
    sweep(A);
    __builtin_amdgcn_s_sleep(8);
    sweep(B);
    for (unsigned spins = 0;; spins += 2) {
      if (ready(A)) {
        stage(A);
        break;
      }
      sweep(A);
      __builtin_amdgcn_s_sleep(8);
      if (ready(B)) {
        stage(B);
        break;
      }
      sweep(B);
      __builtin_amdgcn_s_sleep(8);
      if (spins > XS_SPIN) {
        give_up(a);
        stage(A);
        break;
      }
    }
    ZMI_ASTAMP(1);
  }
  __syncthreads();
  uint4 qf[4];
  if (wave > 0) {
    const uint4* q4p = reinterpret_cast<const uint4*>(qkv_lds);
#pragma unroll
    for (int db = 0; db < 4; ++db)
      qf[db] = c16 < XG ? q4p[(c16 * HD + 8 * h4 + 32 * db) >> 3] : uint4{0u, 0u, 0u, 0u};
    // the K row of pos replaces the fragment of the lane whose key it is; the V^T slot of pos is
    // patched in the fragment whose 8 positions hold it
#pragma unroll
    for (int j = 0; j < KPW; ++j)
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
        if (ww + XNWK * j < OWN && 32 * (s + S * (ww + XNWK * j)) + 16 * tt + c16 == pos) {
#pragma unroll
          for (int db = 0; db < 4; ++db) kf[j][tt][db] = q4p[(XG * HD + 8 * h4 + 32 * db) >> 3];
        }
#pragma unroll
    for (int rc = 0; rc < XRC; ++rc)
#pragma unroll
      for (int q4 = 0; q4 < CPG; ++q4) {
        const int kb = 32 * (CPG * (ww + XNWK * rc) + q4) + 8 * h4;
        if (kb <= pos && pos < kb + 8) {
          const int sl = pos - kb, wi = sl >> 1, sh = (sl & 1) * 16;
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            const int d = 16 * (DT * s + dt) + c16;
            const uint32_t pr = qkv_lds[(XG + 1) * HD / 2 + (d >> 1)];
            const uint32_t val = (d & 1) ? (pr >> 16) : (pr & 0xffffu);
            uint32_t w[4] = {vf[rc][q4][dt].x, vf[rc][q4][dt].y, vf[rc][q4][dt].z, vf[rc][q4][dt].w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (e == wi) w[e] = (w[e] & ~(0xffffu << sh)) | (val << sh);
            vf[rc][q4][dt] = uint4{w[0], w[1], w[2], w[3]};
          }
        }
      }
  }

  // (3) scores of this workgroup's groups (the chunked kernel's MFMA chain): into LDS and out as
  // granules for the other S - 1 workgroups of the query
#pragma unroll
  for (int j = 0; j < KPW; ++j) {
    const int k = s + S * (ww + XNWK * j);
    if (wave > 0 && ww + XNWK * j < OWN && k < n32) {
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        f32x4_t sv = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int db = 0; db < 4; ++db) sv = mfma16(qf[db], kf[j][tt][db], sv);
        const int key = 32 * k + 16 * tt + c16;
        if (h4 == 0 && key <= pos) {
#pragma unroll
          for (int i = 0; i < XG; ++i) {
            const float v = sv[i] * a.scale;
            sc[i][key] = v;
            st_wt64(gs + (size_t)i * DS_KEYS + key, (uint64_t)__float_as_uint(v) | ((uint64_t)tag << 32));
          }
        }
      }
    }
  }

  // (4) gather the other workgroups' scores: thread t takes keys t + NT i (all heads), two sweeps
  // in flight; a key's four granules are kept once all carry the tag
  {
    unsigned pend = 0;
#pragma unroll
    for (int i = 0; i < XKPT; ++i) {
      const int key = t + NT * i;
      if (key < nk && (key >> 5) % S != s) pend |= 1u << i;
    }
    uint64_t A[XKPT][XG], B[XKPT][XG];
    auto sweep = [&](uint64_t(&g)[XKPT][XG]) {
#pragma unroll
      for (int i = 0; i < XKPT; ++i)
#pragma unroll
        for (int h = 0; h < XG; ++h) g[i][h] = ((pend >> i) & 1) ? ld_wt64(gs + h * DS_KEYS + t + NT * i) : 0ull;
    };
    auto take = [&](const uint64_t(&g)[XKPT][XG]) {
#pragma unroll
      for (int i = 0; i < XKPT; ++i) {
        bool ok = (pend >> i) & 1;
#pragma unroll
        for (int h = 0; h < XG; ++h) ok = ok && tag_of(g[i][h]) == tag;
        if (ok) {
#pragma unroll
          for (int h = 0; h < XG; ++h) sc[h][t + NT * i] = __uint_as_float((uint32_t)g[i][h]);
          pend &= ~(1u << i);
        }
      }
    };
    if (pend) {
      sweep(A);
      __builtin_amdgcn_s_sleep(6);
      sweep(B);
    }
    for (unsigned spins = 0; pend; spins += 2) {
      take(A);
      if (!pend) break;
      sweep(A);
      __builtin_amdgcn_s_sleep(6);
      take(B);
      if (!pend) break;
      sweep(B);
      __builtin_amdgcn_s_sleep(6);
      if (spins > XS_SPIN) {
        give_up(a);
        break;
      }
    }
  }
  __syncthreads();
  ZMI_ASTAMP(2);

  // (5) softmax statistics: (chunk, head) tasks, wave + DNW i of them per wave. The chunk maxima
  // are per-thread partials over 16-key segments (8 per chunk) folded by three DPP steps: max is
  // exact in any order. e / l keep the chunked kernel's lane order and wave_sum.
  constexpr int NTASK = (XCH * XG + DNW - 1) / DNW;
  const int ntask = nc * XG;
  if (t < nc * XG * 8) {  // thread = (chunk, head, segment): t = ((c * XG + g) << 3) | seg
    const int seg = t & 7, cg = t >> 3, c = cg / XG, g = cg - c * XG;
    const int k0 = c * CH + 16 * seg;
    const float4* p4 = reinterpret_cast<const float4*>(&sc[g][k0]);
    float m = -INFINITY;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float4 f = p4[v];
      const int kb = k0 + 4 * v;
      m = fmaxf(m, kb < nk ? f.x : -INFINITY);
      m = fmaxf(m, kb + 1 < nk ? f.y : -INFINITY);
      m = fmaxf(m, kb + 2 < nk ? f.z : -INFINITY);
      m = fmaxf(m, kb + 3 < nk ? f.w : -INFINITY);
    }
    m = fmaxf(m, dpp_mov<DPP_XOR1>(m));
    m = fmaxf(m, dpp_mov<DPP_XOR2>(m));
    m = fmaxf(m, dpp_mov<DPP_HALF_MIRROR>(m));  // lanes 8j .. 8j+7 now all hold the chunk maximum
    if (seg == 0) mjc[c][g] = m;
  }
  __syncthreads();
  ZMI_ASTAMP(3);
#ifdef ZMI_ATTN_STAMPS
  const unsigned long long cyc0 = __builtin_amdgcn_s_memtime();
#endif
  {  // M_j = max over the chunks of blocks 0..j; e = exp(s - M_j), l per chunk, P = bf16(e)
#pragma unroll
    for (int i = 0; i < NTASK; ++i) {
      const int task = wave + DNW * i, c = task / XG, g = task - c * XG;
      if (task < ntask) {  // wave-uniform
        const int j = c / CPB, dep = min((j + 1) * CPB, nc);
        float M = mjc[0][g];
#pragma unroll
        for (int cc = 1; cc < XCH; ++cc)  // unrolled: the LDS reads issue together
          if (cc < dep) M = fmaxf(M, mjc[cc][g]);
        if (c % CPB == 0 && lane == 0) mblk[j][g] = M;
        float l = 0.f;
#pragma unroll
        for (int ii = 0; ii < CH / 64; ++ii) {
          const int key = c * CH + lane + 64 * ii;
          const float e = key < nk ? expf(sc[g][key] - M) : 0.f;
          l += e;
          pb[g][key] = (bf16_t)f2bf(e);
        }
        l = wave_sum(l);
        if (lane == 0) ljc[c][g] = l;
      }
    }
  }
  __syncthreads();
  ZMI_ASTAMP(4);
#ifdef ZMI_ATTN_STAMPS
  if (threadIdx.x == 0 && a.stamps) a.stamps[(size_t)blockIdx.x * 8 + 7] = __builtin_amdgcn_s_memtime() - cyc0;
#endif
  // (6) workers: P.V of the slice's dims, each chunk's groups summed in group order in registers
  if (wave > 0) {
#pragma unroll
    for (int rc = 0; rc < XRC; ++rc) {
      const int c = ww + XNWK * rc;
      if (c < nc) {
        f32x4_t oc[DT];
#pragma unroll
        for (int q4 = 0; q4 < CPG; ++q4) {
          const int k = CPG * c + q4;
          if (k < n32) {
            uint4 pf = uint4{0u, 0u, 0u, 0u};
            if (c16 < XG) pf = *reinterpret_cast<const uint4*>(&pb[c16][32 * k + 8 * h4]);
            const int kbase = 32 * k + 8 * h4;
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
              uint4 v = vf[rc][q4][dt];
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
              if (q4 == 0) {
                oc[dt] = o;
              } else {
                oc[dt][0] += o[0];
                oc[dt][1] += o[1];
                oc[dt][2] += o[2];
                oc[dt][3] += o[3];
              }
            }
          }
        }
        if (h4 == 0) {
#pragma unroll
          for (int dt = 0; dt < DT; ++dt)
#pragma unroll
            for (int i = 0; i < XG; ++i) ocs[c][i][16 * dt + c16] = oc[dt][i];
        }
      }
    }
  }
  __syncthreads();
  ZMI_ASTAMP(5);
  // (7) the block recursion (zmi_attn_merge.h), one thread per (head, dim of the slice)
  if (t < XG * DSD) {
    const int g = t / DSD, dl = t - g * DSD;
    float acc = 0.f, l = 0.f, ob = 0.f, lb = 0.f, mprev = 0.f, mb = 0.f;
    float ocv[XCH], lcv[XCH];
#pragma unroll
    for (int c = 0; c < XCH; ++c) {  // every read first (clamped rows past nc are never used)
      const int cr = min(c, nc - 1);
      ocv[c] = ocs[cr][g][dl];
      lcv[c] = ljc[cr][g];
    }
#pragma unroll
    for (int c = 0; c < XCH; ++c) {
      if (c >= nc) break;
      const float oc = ocv[c];
      if (c % CPB == 0) {
        ob = oc;
        lb = lcv[c];
        mb = mblk[c / CPB][g];
      } else {
        ob += oc;
        lb += lcv[c];
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
    const float rl = 1.0f / l;
    a.out[(size_t)qi * a.ldo + (kh * XG + g) * HD + DSD * s + dl] = (bf16_t)f2bf(acc * rl);
  }
  ZMI_ASTAMP(6);
}

// ---- self-scoring form (ZMI_ATTNBLK_SELF): no score exchange -------------------------------------
// Each of the S workgroups of a (query, kv head) loads EVERY cached K row of its query (the S slices
// sit on one XCD, so S - 1 of them read K from L2) and the V^T rows of its own HD / S output dims, and
// computes all scores, the softmax statistics and P itself; only P.V and the output are split by
// dims. The one hand-off left is projection -> attention (q and this position's K / V row). Wave w
// owns 128-key chunk w for the whole chain (scores, chunk maximum, e / l / P, P.V); the waves meet
// at three workgroup barriers (q staged, chunk maxima, chunk P.V). The arithmetic is xs_body's /
// the chunked kernel's operation for operation (bit-identical).
// Positions < XR_KEYS: wave w holds chunk w's K fragments (128 VGPRs) in registers.
constexpr int FORM_XS = 0, FORM_SELF = 1, FORM_SPLIT = 2;  // attention roles of attn_block_kernel
constexpr int XR_CH = DNW;              // chunks, one per wave
constexpr int XR_KEYS = XR_CH * CH;     // 1024 keys (positions 0 .. 1023)
constexpr int XR_POLL = DNW - 1;        // the wave that also receives the projection's granules

template <int S>
struct XrImg {
  static constexpr int DSD = HD / S;
  static constexpr size_t SC = 0;                                   // float [XG][XR_KEYS] scores
  static constexpr size_t PB = SC + (size_t)XG * XR_KEYS * 4;       // bf16  [XG][XR_KEYS] P
  static constexpr size_t OC = PB + (size_t)XG * XR_KEYS * 2;       // float [XR_CH][XG][DSD] chunk P.V
  static constexpr size_t MJ = OC + (size_t)XR_CH * XG * DSD * 4;   // float [XR_CH][XG] chunk maxima
  static constexpr size_t LJ = MJ + (size_t)XR_CH * XG * 4;         // float [XR_CH][XG] chunk exp sums
  static constexpr size_t MB = LJ + (size_t)XR_CH * XG * 4;         // float [XR_CH / CPB][XG] M_j
  static constexpr size_t QKV = MB + (size_t)(XR_CH / CPB) * XG * 4; // u32 [QKV_GRAN] q | k | v pairs of pos
  static constexpr size_t BYTES = (QKV + (size_t)QKV_GRAN * 4 + 15) / 16 * 16;
};

template <int S>
__device__ __forceinline__ void xr_body(const AttnArgs& a, int n_units, int b, char* smem, uint64_t* gran) {
  constexpr int DT = 8 / S;
  using I = XrImg<S>;
  constexpr int DSD = I::DSD;
  float(&sc)[XG][XR_KEYS] = *reinterpret_cast<float(*)[XG][XR_KEYS]>(smem + I::SC);
  bf16_t(&pb)[XG][XR_KEYS] = *reinterpret_cast<bf16_t(*)[XG][XR_KEYS]>(smem + I::PB);
  float(&ocs)[XR_CH][XG][DSD] = *reinterpret_cast<float(*)[XR_CH][XG][DSD]>(smem + I::OC);
  float(&mjc)[XR_CH][XG] = *reinterpret_cast<float(*)[XR_CH][XG]>(smem + I::MJ);
  float(&ljc)[XR_CH][XG] = *reinterpret_cast<float(*)[XR_CH][XG]>(smem + I::LJ);
  float(&mblk)[XR_CH / CPB][XG] = *reinterpret_cast<float(*)[XR_CH / CPB][XG]>(smem + I::MB);
  uint32_t* qkv_lds = reinterpret_cast<uint32_t*>(smem + I::QKV);

  const int y = b >> 3;
  const int s = y % S, unit = 8 * (y / S) + (b & 7);
  if (unit >= n_units) return;
  const int qi = unit / a.hkv, kh = unit - qi * a.hkv;
  const int pos = a.pos[qi];
  if (pos < 0) return;
  if (pos >= XR_KEYS) {  // the engine never launches this form past its capacity; refuse, don't read past it
    if (threadIdx.x == 0) give_up(a);
    return;
  }
  ZMI_ASTAMP(0);
  const uint32_t tag = (uint32_t)pos + 1u;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c16 = lane & 15, h4 = lane >> 4;
  const int kvr = a.kv_row ? a.kv_row[qi] : qi;
  const size_t kvbase = ((size_t)kvr * a.hkv + kh) * a.smax * HD;
  const int nk = pos + 1, n32 = (pos + 32) >> 5, nc = pos / CH + 1;
  const int c = wave;                      // this wave's chunk
  const bool live = c < nc;
  uint64_t* gu = gran + (size_t)unit * GRAN_STRIDE;

  // (1) the chunk's cached K rows (positions < pos; the row of pos comes from the granules) and the
  // V^T fragments of its four 32-key groups for dim slice s, all in flight at once
  const int pc = max(pos - 1, 0);
  uint4 kf[CPG][2][4], vf[CPG][DT];
  if (live) {
#pragma unroll
    for (int q4 = 0; q4 < CPG; ++q4) {
      const int k = CPG * c + q4;
      if (k < n32) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const bf16_t* kr = a.k + kvbase + (size_t)min(32 * k + 16 * tt + c16, pc) * HD + 8 * h4;
#pragma unroll
          for (int db = 0; db < 4; ++db) kf[q4][tt][db] = *reinterpret_cast<const uint4*>(kr + 32 * db);
        }
      }
    }
#pragma unroll
    for (int q4 = 0; q4 < CPG; ++q4) {
      const int k = CPG * c + q4;
      if (k < n32) {
        const int p0 = min(32 * k + 8 * h4, pos & ~7);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
          vf[q4][dt] = *reinterpret_cast<const uint4*>(a.v + kvbase + (size_t)(16 * (DT * s + dt) + c16) * a.smax + p0);
      }
    }
  }
  if (wave == XR_POLL) {
    // (2) this position's q, K row and V row (QKV_GRAN pairs; 6 per lane), two sweeps in flight
    uint64_t A[6], B[6];
    auto sweep = [&](uint64_t(&g)[6]) {
#pragma unroll
      for (int i = 0; i < 6; ++i) g[i] = ld_wt64(gu + lane + 64 * i);
    };
    auto ready = [&](const uint64_t(&g)[6]) {
      bool ok = true;
#pragma unroll
      for (int i = 0; i < 6; ++i) ok = ok && tag_of(g[i]) == tag;
      return __all(ok);
    };
    auto stage = [&](const uint64_t(&g)[6]) {
#pragma unroll
      for (int i = 0; i < 6; ++i) qkv_lds[lane + 64 * i] = (uint32_t)g[i];
    };
    sweep(A);
    __builtin_amdgcn_s_sleep(8);
    sweep(B);
    for (unsigned spins = 0;; spins += 2) {
      if (ready(A)) {
        stage(A);
        break;
      }
      sweep(A);
      __builtin_amdgcn_s_sleep(8);
      if (ready(B)) {
        stage(B);
        break;
      }
      sweep(B);
      __builtin_amdgcn_s_sleep(8);
      if (spins > XS_SPIN) {
        give_up(a);
        stage(A);
        break;
      }
    }
    ZMI_ASTAMP(1);
  }
  __syncthreads();

  // (3) scores of the chunk: q from LDS, the K row / V^T slot of pos patched in, the chunked kernel's
  // 4-MFMA chain per 16 keys; then the chunk maximum per head (exact in any order)
  if (live) {
    const uint4* q4p = reinterpret_cast<const uint4*>(qkv_lds);
    uint4 qf[4];
#pragma unroll
    for (int db = 0; db < 4; ++db)
      qf[db] = c16 < XG ? q4p[(c16 * HD + 8 * h4 + 32 * db) >> 3] : uint4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int q4 = 0; q4 < CPG; ++q4)
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
        if (32 * (CPG * c + q4) + 16 * tt + c16 == pos) {
#pragma unroll
          for (int db = 0; db < 4; ++db) kf[q4][tt][db] = q4p[(XG * HD + 8 * h4 + 32 * db) >> 3];
        }
#pragma unroll
    for (int q4 = 0; q4 < CPG; ++q4) {
      const int kb = 32 * (CPG * c + q4) + 8 * h4;
      if (kb <= pos && pos < kb + 8) {
        const int sl = pos - kb, wi = sl >> 1, sh = (sl & 1) * 16;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int d = 16 * (DT * s + dt) + c16;
          const uint32_t pr = qkv_lds[(XG + 1) * HD / 2 + (d >> 1)];
          const uint32_t val = (d & 1) ? (pr >> 16) : (pr & 0xffffu);
          uint32_t w[4] = {vf[q4][dt].x, vf[q4][dt].y, vf[q4][dt].z, vf[q4][dt].w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (e == wi) w[e] = (w[e] & ~(0xffffu << sh)) | (val << sh);
          vf[q4][dt] = uint4{w[0], w[1], w[2], w[3]};
        }
      }
    }
#pragma unroll
    for (int q4 = 0; q4 < CPG; ++q4) {
      const int k = CPG * c + q4;
      if (k < n32) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          f32x4_t sv = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int db = 0; db < 4; ++db) sv = mfma16(qf[db], kf[q4][tt][db], sv);
          const int key = 32 * k + 16 * tt + c16;
          if (h4 == 0 && key <= pos) {
#pragma unroll
            for (int i = 0; i < XG; ++i) sc[i][key] = sv[i] * a.scale;
          }
        }
      }
    }
    ZMI_ASTAMP(2);
    asm volatile("" ::: "memory");  // this wave's LDS writes stay ahead of its reads below (LDS is in order per wave)
    float m[XG];
#pragma unroll
    for (int g = 0; g < XG; ++g) {
      const int k0 = c * CH + lane;
      m[g] = fmaxf(k0 < nk ? sc[g][k0] : -INFINITY, k0 + 64 < nk ? sc[g][k0 + 64] : -INFINITY);
    }
#pragma unroll
    for (int g = 0; g < XG; ++g) m[g] = wave_max(m[g]);
    if (lane == 0) {
#pragma unroll
      for (int g = 0; g < XG; ++g) mjc[c][g] = m[g];
    }
  }
  __syncthreads();
  ZMI_ASTAMP(3);

  // (4) M_j = max over the chunks of blocks 0..j; e = exp(s - M_j), l, P = bf16(e); then P.V of the
  // slice's dims, the chunk's four groups summed in group order in registers
  if (live) {
    const int j = c / CPB, dep = min((j + 1) * CPB, nc);
    float l[XG];
#pragma unroll
    for (int g = 0; g < XG; ++g) {
      float M = mjc[0][g];
#pragma unroll
      for (int cc = 1; cc < XR_CH; ++cc)
        if (cc < dep) M = fmaxf(M, mjc[cc][g]);
      if (c % CPB == 0 && lane == 0) mblk[j][g] = M;
      l[g] = 0.f;
#pragma unroll
      for (int ii = 0; ii < CH / 64; ++ii) {
        const int key = c * CH + lane + 64 * ii;
        const float e = key < nk ? expf(sc[g][key] - M) : 0.f;
        l[g] += e;
        pb[g][key] = (bf16_t)f2bf(e);
      }
    }
#pragma unroll
    for (int g = 0; g < XG; ++g) l[g] = wave_sum(l[g]);
    if (lane == 0) {
#pragma unroll
      for (int g = 0; g < XG; ++g) ljc[c][g] = l[g];
    }
    ZMI_ASTAMP(4);
    asm volatile("" ::: "memory");
    f32x4_t oc[DT];
#pragma unroll
    for (int q4 = 0; q4 < CPG; ++q4) {
      const int k = CPG * c + q4;
      if (k < n32) {
        uint4 pf = uint4{0u, 0u, 0u, 0u};
        if (c16 < XG) pf = *reinterpret_cast<const uint4*>(&pb[c16][32 * k + 8 * h4]);
        const int kbase = 32 * k + 8 * h4;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          uint4 v = vf[q4][dt];
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
          if (q4 == 0) {
            oc[dt] = o;
          } else {
            oc[dt][0] += o[0];
            oc[dt][1] += o[1];
            oc[dt][2] += o[2];
            oc[dt][3] += o[3];
          }
        }
      }
    }
    if (h4 == 0) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int i = 0; i < XG; ++i) ocs[c][i][16 * dt + c16] = oc[dt][i];
    }
  }
  __syncthreads();
  ZMI_ASTAMP(5);
  // (5) the block recursion (zmi_attn_merge.h), one thread per (head, dim of the slice)
  if (t < XG * DSD) {
    const int g = t / DSD, dl = t - g * DSD;
    float acc = 0.f, l = 0.f, ob = 0.f, lb = 0.f, mprev = 0.f, mb = 0.f;
    float ocv[XR_CH], lcv[XR_CH];
#pragma unroll
    for (int cc = 0; cc < XR_CH; ++cc) {
      const int cr = min(cc, nc - 1);
      ocv[cc] = ocs[cr][g][dl];
      lcv[cc] = ljc[cr][g];
    }
#pragma unroll
    for (int cc = 0; cc < XR_CH; ++cc) {
      if (cc >= nc) break;
      const float o = ocv[cc];
      if (cc % CPB == 0) {
        ob = o;
        lb = lcv[cc];
        mb = mblk[cc / CPB][g];
      } else {
        ob += o;
        lb += lcv[cc];
      }
      if (cc % CPB == CPB - 1 || cc == nc - 1) {
        if (cc < CPB) {
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
    a.out[(size_t)qi * a.ldo + (kh * XG + g) * HD + DSD * s + dl] = (bf16_t)f2bf(acc * rl);
  }
  ZMI_ASTAMP(6);
}

// ---- chunk-split form (ZMI_ATTNBLK_SPLIT): one workgroup per 128-key chunk -----------------------
// Workgroup c of a (query, kv head) loads only chunk c's K rows and V^T columns (64 KB: the cached K / V
// of a query are read once, spread over its chunks' CUs), computes the chunk's scores, maximum,
// e / l / P and P.V for all 128 dims: the chunked kernel's (zmi_attn.hip) per-chunk arithmetic. Two
// granule hand-offs between the chunks of a query, both small: the chunk maxima (4 per chunk: M_j of
// the chunk's block), then each chunk's P.V partial, l and M_j, of which workgroup c merges dims
// 16 c .. 16 c + 15 (zmi_attn_merge.h's recursion). Workgroups of chunks past the position only merge.
// Positions < XCH x 128 for XCH chunk workgroups per (query, kv head): 8 (positions < 1024, the C2 form) or 24
// (< 3072, batch-1 utterances past the 8-chunk reach). Granules (after the unit's q / K / V pairs, tag =
// position + 1): GM [chunk][head] maxima, GL [chunk][head] l, GB [chunk][head] M_j, GO [chunk][head][dim] P.V
// partials. Workgroups 0..7 merge (16 dims each) whatever XCH is.
template <int XCH>
struct XcG {
  static constexpr int KEYS = XCH * CH;
  static constexpr int GM = 0, GL = GM + XCH * XG, GB = GL + XCH * XG, GO = GB + XCH * XG;
  static constexpr int WORDS = GO + XCH * XG * HD;
  // the fused out_proj role (OPROJ): the unit's output as XG HD / 2 {bf16 pair, tag} granules, then one flag per
  // merging workgroup, after the chunk granules
  static constexpr int OG = WORDS, OF = OG + XG * HD / 2, OWORDS = OF + HD / 16;
  static constexpr bool OPROJ_FITS = QKV_GRAN + OWORDS <= GRAN_STRIDE;
  static_assert(WORDS <= GRAN_STRIDE - QKV_GRAN, "the chunk-split granules fit the unit's area");
  static_assert(XCH >= HD / 16 && XCH % CPB == 0 && XCH <= XC_CH_MAX, "8 merging workgroups; whole 512-key blocks");
};
constexpr int XC_KEYS = XcG<8>::KEYS;  // the 8-chunk form's reach (1024 keys)
static_assert(CH == 128 && DNW == 8, "eight waves: one 16-key score tile each over a 128-key chunk");

struct XcImg {
  static constexpr size_t SC = 0;                              // float [XG][CH] scores of the chunk
  static constexpr size_t PB = SC + (size_t)XG * CH * 4;       // bf16  [XG][CH] P
  static constexpr size_t OP = PB + (size_t)XG * CH * 2;       // float [CPG][XG][HD] per-group P.V
  static constexpr size_t MJ = OP + (size_t)CPG * XG * HD * 4; // float [XG] M_j of the chunk's block
  static constexpr size_t QKV = MJ + (size_t)XG * 4;           // u32 [QKV_GRAN] q | k | v pairs of pos
  static constexpr size_t BYTES = (QKV + (size_t)QKV_GRAN * 4 + 15) / 16 * 16;
};

#ifndef ZMI_XC_QKV_SLEEP
#define ZMI_XC_QKV_SLEEP 2  // the chunk-split form's q / K / V poll: s_sleep between its two sweeps in flight (8 before
                            // round 6's end: C2 step 890-902 vs 881-884 us with 2, 889-898 with 4, 905-919 with 16)
#endif
template <int XCH, bool OPROJ>
__device__ __forceinline__ void xc_body(const AttnArgs& a, int n_units, int b, char* smem, uint64_t* gran) {
  using X = XcG<XCH>;
  constexpr int XC_CH = XCH, XC_GM = X::GM, XC_GL = X::GL, XC_GB = X::GB, XC_GO = X::GO;
  float(&sc)[XG][CH] = *reinterpret_cast<float(*)[XG][CH]>(smem + XcImg::SC);
  bf16_t(&pb)[XG][CH] = *reinterpret_cast<bf16_t(*)[XG][CH]>(smem + XcImg::PB);
  float(&opart)[CPG][XG][HD] = *reinterpret_cast<float(*)[CPG][XG][HD]>(smem + XcImg::OP);
  float* mj = reinterpret_cast<float*>(smem + XcImg::MJ);
  uint32_t* qkv_lds = reinterpret_cast<uint32_t*>(smem + XcImg::QKV);

  const int y = b >> 3;
  const int c = y % XC_CH, unit = 8 * (y / XC_CH) + (b & 7);
  if (unit >= n_units) return;
  const int qi = unit / a.hkv, kh = unit - qi * a.hkv;
  const int pos = a.pos[qi];
  if (pos < 0) return;
  if (pos >= X::KEYS) {  // the engine never launches this form past its capacity; refuse, don't read past it
    if (threadIdx.x == 0) give_up(a);
    return;
  }
  ZMI_ASTAMP(0);
  const uint32_t tag = (uint32_t)pos + 1u;
  const uint64_t tag64 = (uint64_t)tag << 32;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c16 = lane & 15, h4 = lane >> 4;
  const int nk = pos + 1, n32 = (pos + 32) >> 5, nc = pos / CH + 1;
  uint64_t* gu = gran + (size_t)unit * GRAN_STRIDE;
  uint64_t* gx = gu + QKV_GRAN;

  if (c < nc) {
    const int kvr = a.kv_row ? a.kv_row[qi] : qi;
    const size_t kvbase = ((size_t)kvr * a.hkv + kh) * a.smax * HD;
    // (1) wave w: score tile (group w >> 1, 16 keys w & 1) K rows and the V^T fragments of group w & 3,
    // dims 64 (w >> 2) .. + 63, positions < pos (the row of pos comes from the granules)
    const int gs = wave >> 1, tt = wave & 1, gv = wave & 3, hv = wave >> 2;
    const int pc = max(pos - 1, 0);
    const bool sk = CPG * c + gs < n32, vk = CPG * c + gv < n32;
    uint4 kf[4], vf[4];
    if (sk) {
      const bf16_t* kr = a.k + kvbase + (size_t)min(CH * c + 32 * gs + 16 * tt + c16, pc) * HD + 8 * h4;
#pragma unroll
      for (int db = 0; db < 4; ++db) kf[db] = *reinterpret_cast<const uint4*>(kr + 32 * db);
    }
    if (vk) {
      const int p0 = min(CH * c + 32 * gv + 8 * h4, pos & ~7);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        vf[dt] = *reinterpret_cast<const uint4*>(a.v + kvbase + (size_t)(64 * hv + 16 * dt + c16) * a.smax + p0);
    }
    if (wave == 0) {
      // (2) this position's q, K row and V row (QKV_GRAN pairs; 6 per lane), two sweeps in flight
      uint64_t A[6], B[6];
      auto sweep = [&](uint64_t(&g)[6]) {
#pragma unroll
        for (int i = 0; i < 6; ++i) g[i] = ld_wt64(gu + lane + 64 * i);
      };
      auto ready = [&](const uint64_t(&g)[6]) {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < 6; ++i) ok = ok && tag_of(g[i]) == tag;
        return __all(ok);
      };
      auto stage = [&](const uint64_t(&g)[6]) {
#pragma unroll
        for (int i = 0; i < 6; ++i) qkv_lds[lane + 64 * i] = (uint32_t)g[i];
      };
      sweep(A);
      __builtin_amdgcn_s_sleep(ZMI_XC_QKV_SLEEP);
      sweep(B);
      for (unsigned spins = 0;; spins += 2) {
        if (ready(A)) {
          stage(A);
          break;
        }
        sweep(A);
        __builtin_amdgcn_s_sleep(ZMI_XC_QKV_SLEEP);
        if (ready(B)) {
          stage(B);
          break;
        }
        sweep(B);
        __builtin_amdgcn_s_sleep(ZMI_XC_QKV_SLEEP);
        if (spins > XS_SPIN) {
          give_up(a);
          stage(A);
          break;
        }
      }
      ZMI_ASTAMP(1);
    }
    __syncthreads();
    // (3) the tile's scores (the chunked kernel's 4-MFMA chain; the K row of pos patched in)
    const uint4* q4p = reinterpret_cast<const uint4*>(qkv_lds);
    if (sk) {
      uint4 qf[4];
#pragma unroll
      for (int db = 0; db < 4; ++db)
        qf[db] = c16 < XG ? q4p[(c16 * HD + 8 * h4 + 32 * db) >> 3] : uint4{0u, 0u, 0u, 0u};
      const int key = CH * c + 32 * gs + 16 * tt + c16;
      if (key == pos) {
#pragma unroll
        for (int db = 0; db < 4; ++db) kf[db] = q4p[(XG * HD + 8 * h4 + 32 * db) >> 3];
      }
      f32x4_t sv = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int db = 0; db < 4; ++db) sv = mfma16(qf[db], kf[db], sv);
      if (h4 == 0 && key <= pos) {
#pragma unroll
        for (int i = 0; i < XG; ++i) sc[i][key - CH * c] = sv[i] * a.scale;
      }
    }
    if (vk) {  // the V^T slot of pos, in the fragment whose 8 positions hold it
      const int kb = CH * c + 32 * gv + 8 * h4;
      if (kb <= pos && pos < kb + 8) {
        const int sl = pos - kb, wi = sl >> 1, sh = (sl & 1) * 16;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const int d = 64 * hv + 16 * dt + c16;
          const uint32_t pr = qkv_lds[(XG + 1) * HD / 2 + (d >> 1)];
          const uint32_t val = (d & 1) ? (pr >> 16) : (pr & 0xffffu);
          uint32_t w[4] = {vf[dt].x, vf[dt].y, vf[dt].z, vf[dt].w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (e == wi) w[e] = (w[e] & ~(0xffffu << sh)) | (val << sh);
          vf[dt] = uint4{w[0], w[1], w[2], w[3]};
        }
      }
    }
    __syncthreads();
    ZMI_ASTAMP(2);
    // (4) wave 0: the chunk maxima (exact in any order) out as granules, then M_j of the chunk's block
    // from the maxima of chunks 0 .. dep - 1 (lane = chunk x XG + head)
    if (wave == 0) {
      float m[XG];
#pragma unroll
      for (int g = 0; g < XG; ++g)
        m[g] = fmaxf(CH * c + lane < nk ? sc[g][lane] : -INFINITY, CH * c + lane + 64 < nk ? sc[g][lane + 64] : -INFINITY);
#pragma unroll
      for (int g = 0; g < XG; ++g) m[g] = wave_max(m[g]);
      if (lane < XG) {
        const float mine = lane == 0 ? m[0] : (lane == 1 ? m[1] : (lane == 2 ? m[2] : m[3]));
        st_xc64(gx + XC_GM + c * XG + lane, (uint64_t)__float_as_uint(mine) | tag64, a.xc_l2);
      }
      const int j = c / CPB, dep = min((j + 1) * CPB, nc);
      float v = -INFINITY;
#pragma unroll
      for (int h = 0; h < (XCH * XG + 63) / 64; ++h) {  // entry e = chunk x XG + head; e and e + 64: one head
        const int e = lane + 64 * h, cc = e / XG, g = e - cc * XG;
        if (e < dep * XG) {
          if (cc == c) {
            v = fmaxf(v, g == 0 ? m[0] : (g == 1 ? m[1] : (g == 2 ? m[2] : m[3])));
          } else {
            uint64_t w = ld_wt64(gx + XC_GM + e);
            for (unsigned spins = 0; tag_of(w) != tag; ++spins) {
              if (spins > XS_SPIN) {
                give_up(a);
                break;
              }
              __builtin_amdgcn_s_sleep(2);
              w = ld_wt64(gx + XC_GM + e);
            }
            v = fmaxf(v, __uint_as_float((uint32_t)w));
          }
        }
      }
      // max over the chunks of each head: lanes g, g + 4, ..., g + 60 (exact in any order)
      v = fmaxf(v, __shfl_xor(v, 4));
      v = fmaxf(v, __shfl_xor(v, 8));
      v = fmaxf(v, __shfl_xor(v, 16));
      if constexpr (XCH * XG > 32) v = fmaxf(v, __shfl_xor(v, 32));
      if (lane < XG) mj[lane] = v;
    }
    __syncthreads();
    ZMI_ASTAMP(3);
    // (5) waves 0..3 (head w): e = exp(s - M_j), l (lane L: keys L, L + 64, then wave_sum), P = bf16(e)
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
        st_xc64(gx + XC_GL + c * XG + wave, (uint64_t)__float_as_uint(l) | tag64, a.xc_l2);
        st_xc64(gx + XC_GB + c * XG + wave, (uint64_t)__float_as_uint(M) | tag64, a.xc_l2);
      }
    }
    __syncthreads();
    ZMI_ASTAMP(4);
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
        const f32x4_t o = mfma16(pf, v, f32x4_t{0.f, 0.f, 0.f, 0.f});
        if (h4 == 0) {
#pragma unroll
          for (int i = 0; i < XG; ++i) opart[gv][i][64 * hv + 16 * dt + c16] = o[i];
        }
      }
    }
    __syncthreads();
    // (7) the chunk's P.V (groups summed in group order) out as granules, one (head, dim) per thread
    {
      const int g = t / HD, d = t - g * HD;
      float o = opart[0][g][d];
#pragma unroll
      for (int w = 1; w < CPG; ++w)
        if (CPG * c + w < n32) o += opart[w][g][d];
      st_xc64(gx + XC_GO + (c * XG + g) * HD + d, (uint64_t)__float_as_uint(o) | tag64, a.xc_l2);
    }
    ZMI_ASTAMP(5);
  }
  // (8) dims 16 c .. + 15 of the unit's output: every chunk's partial, l and M_j, gathered by all eight waves (wave w
  // polls chunks w, w + 8, w + 16 and block maximum w, lane = (head, dim) as below) into LDS (the score / partial areas,
  // free after (7)), then the block recursion of zmi_attn_merge.h by wave 0, one lane per (head, dim). Spreading the
  // polls over the waves keeps each wave's granules in flight to a few (the 24-chunk form held all 54 per lane).
  if (c < HD / 16) {
    constexpr int KPW = (XC_CH + DNW - 1) / DNW, NBLK = XC_CH / CPB;
    static_assert(NBLK <= DNW && 2 * KPW + 1 <= 32, "one block maximum per wave; one pending bit per granule");
    float* mO = reinterpret_cast<float*>(smem + XcImg::OP);   // [XC_CH][XG x 16] partials of the (head, dim)s
    float* mL = reinterpret_cast<float*>(smem + XcImg::SC);   // [XC_CH][XG] chunk l
    float* mM = mL + XC_CH * XG;                              // [NBLK][XG] block M_j
    static_assert((size_t)XC_CH * XG * 16 * 4 <= XcImg::MJ - XcImg::OP &&
                  (size_t)(XC_CH + NBLK) * XG * 4 <= XcImg::PB - XcImg::SC, "the merge staging fits the freed areas");
    __syncthreads();  // (7)'s partial reads are done before its LDS is reused
    const int l64 = t & 63, g = l64 >> 4, d = 16 * c + (l64 & 15);
    uint64_t ov[KPW], lv[KPW], mv = 0ull;
    unsigned pend = 0;
#pragma unroll
    for (int i = 0; i < KPW; ++i)
      if (wave + DNW * i < nc) pend |= 3u << (2 * i);
    if (wave < NBLK && wave * CPB < nc) pend |= 1u << (2 * KPW);
    for (unsigned spins = 0; pend; ++spins) {
#pragma unroll
      for (int i = 0; i < KPW; ++i) {
        const int k = wave + DNW * i;
        if ((pend >> (2 * i)) & 1) ov[i] = ld_wt64(gx + XC_GO + (k * XG + g) * HD + d);
        if ((pend >> (2 * i + 1)) & 1) lv[i] = ld_wt64(gx + XC_GL + k * XG + g);
      }
      if ((pend >> (2 * KPW)) & 1) mv = ld_wt64(gx + XC_GB + wave * CPB * XG + g);
#pragma unroll
      for (int i = 0; i < KPW; ++i) {
        if (((pend >> (2 * i)) & 1) && tag_of(ov[i]) == tag) pend &= ~(1u << (2 * i));
        if (((pend >> (2 * i + 1)) & 1) && tag_of(lv[i]) == tag) pend &= ~(1u << (2 * i + 1));
      }
      if (((pend >> (2 * KPW)) & 1) && tag_of(mv) == tag) pend &= ~(1u << (2 * KPW));
      if (__all(pend == 0)) break;
      if (spins > XS_SPIN) {
        give_up(a);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
#pragma unroll
    for (int i = 0; i < KPW; ++i) {
      const int k = wave + DNW * i;
      if (k < nc) {
        mO[k * (XG * 16) + l64] = __uint_as_float((uint32_t)ov[i]);
        if ((l64 & 15) == 0) mL[k * XG + g] = __uint_as_float((uint32_t)lv[i]);
      }
    }
    if (wave < NBLK && wave * CPB < nc && (l64 & 15) == 0) mM[wave * XG + g] = __uint_as_float((uint32_t)mv);
    __syncthreads();
  }
  if (c < HD / 16 && t < XG * 16) {
    const int g = t >> 4, d = 16 * c + (t & 15);
    const float* mO = reinterpret_cast<const float*>(smem + XcImg::OP);
    const float* mL = reinterpret_cast<const float*>(smem + XcImg::SC);
    const float* mM = mL + XC_CH * XG;
    float acc = 0.f, l = 0.f, ob = 0.f, lb = 0.f, mprev = 0.f, mb = 0.f;
    for (int k = 0; k < nc; ++k) {
      const float o = mO[k * (XG * 16) + t], lk = mL[k * XG + g];
      if (k % CPB == 0) {
        ob = o;
        lb = lk;
        mb = mM[(k / CPB) * XG + g];
      } else {
        ob += o;
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
    const uint32_t ov16 = f2bf(acc * rl);
    a.out[(size_t)qi * a.ldo + (kh * XG + g) * HD + d] = (bf16_t)ov16;
    if constexpr (OPROJ) {
      // the same 64 values as 32 {bf16 pair, tag} granules for the out_proj role (this is wave 0: its lanes t hold
      // (head t >> 4, dim 16 c + (t & 15))), then this workgroup's flag. The flag is only a cheap "look now" for
      // the out_proj role's poller (64 flags instead of 2048 granules): it is not ordered after the granules,
      // whose own tags the gather checks
      static_assert(X::OPROJ_FITS, "the output granules fit the unit's area");
      const uint32_t nb = (uint32_t)__shfl_xor((int)ov16, 1);
      if ((t & 1) == 0) st_wt64(gu + QKV_GRAN + X::OG + ((g * HD + d) >> 1), (uint64_t)(ov16 | (nb << 16)) | tag64);
      if (t == 0) st_wt64(gu + QKV_GRAN + X::OF + c, tag64);
    }
  }
  ZMI_ASTAMP(6);
}

// PRO: the projection's prologue, LayerNorm (transformer blocks) or ADDLN (the hybrid's MHA blocks:
// layer_norm_fn(hidden, residual) with the new residual written by column block 0). SELF: the
// attention role is xr_body (self-scoring) instead of xs_body (score exchange).
// OPROJ (chunk-split forms, 8 or 24 chunks): a fourth role after the attention workgroups runs the layer's out_proj GEMV
// (_torch.py:115,140 + the residual :100), its weights loaded at its start and its activation rows gathered from the
// merging workgroups' output granules (zmi_gemv_impl.h FUSE 3), so out_proj needs no launch of its own.
// Ordering rule: this role writes the residual rows x in place while the same launch's QKV role reads x for its
// LayerNorm. That is safe because it stores a row only after gathering that row's attention output, which exists
// only after every QKV column block feeding the row's units has published its granules (each QKV block feeds
// some (row, kv head) unit that the gather waits on), i.e. after every QKV workgroup has read x. Rows with
// position < 0 run no attention, so the role neither waits on them nor stores them (act_rows).
template <int S, int PRO, int FORM, bool OPROJ>
__global__ __launch_bounds__(NT) void attn_block_kernel(const ZmiGemvArgs qa, int n_cb, int n_qkv, const AttnArgs at,
                                                        int n_units, uint64_t* gran, const ZmiPrefetch pf, int n_pf,
                                                        const ZmiGemvArgs oa, int n_op) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  const int n_xs = (n_units + 7) / 8 * 8 * S;
  if (b < n_qkv)
    zmi_gemv::gemv_body<QG, QW, QNL, QRT, PRO, ZMI_EPI_QKV, 1, 1>(
        qa, n_cb, 1, b, smem, zmi_gemv::QkvFuse{gran, GRAN_STRIDE});
  else if (b < n_qkv + n_xs) {
    if constexpr (FORM == FORM_SELF)
      xr_body<S>(at, n_units, b - n_qkv, smem, gran);
    else if constexpr (FORM == FORM_SPLIT)
      xc_body<S, OPROJ>(at, n_units, b - n_qkv, smem, gran);
    else
      xs_body<S>(at, n_units, b - n_qkv, smem, gran);
  } else if (OPROJ && b < n_qkv + n_xs + n_op) {
    if constexpr (OPROJ) {
      using X = XcG<S>;
      zmi_gemv::QkvFuse fz{gran, GRAN_STRIDE};
      fz.og_off = QKV_GRAN + X::OG;
      fz.of_off = QKV_GRAN + X::OF;
      fz.hkv = at.hkv;
      fz.pos = at.pos;
      fz.err = at.err;
      // transformer blocks: x + bf16(out_proj) in place (_torch.py:100); the hybrid's MHA blocks (ADDLN projection):
      // bf16(out_proj) into the hidden rows, which the next block's add + LayerNorm adds to the residual
      constexpr int OEPI = PRO == zmi_gemv::PRO_ADDLN ? ZMI_EPI_STORE : ZMI_EPI_RESIDUAL;
      zmi_gemv::gemv_body<QG, QW, QNL, QRT, zmi_gemv::PRO_PLAIN, OEPI, 1, 3>(oa, oa.N / 8 / QG, 1, b - n_qkv - n_xs,
                                                                             smem, fz);
    }
  } else
    prefetch_body<NT>(pf, b - n_qkv - n_xs - n_op, n_pf);
}

template <int S, int PRO, int FORM, bool OPROJ = false>
hipError_t launch_block(const ZmiGemvArgs& a, int n_cb, int n_qkv, const AttnArgs& at, int n_units, uint64_t* gran,
                        const ZmiPrefetch& pf, hipStream_t s, const ZmiGemvArgs* oa = nullptr) {
  // at least half the CU's LDS: one workgroup per CU, so the ~256 workgroups spread over the chip
  // instead of sharing a CU's ~64 KB of loads in flight
  // (the wide chunk-split form with co-resident workgroups instead measured the same: profiles/r04_split24_ab.jsonl)
  // (ZMI_OPT_ATTNBLK_SPREAD bits 0-1: the floor of the 8-chunk / score-exchange / self forms, bits 2-3: of the
  // 24-chunk form, whose 384 workgroups otherwise leave 128 of its attention workgroups waiting for projection CUs;
  // 0 = none, 1 = one workgroup per CU, 2 = at most two)
  const int fl = (zmi_option(ZMI_OPT_ATTNBLK_SPREAD) >> (S == 24 ? 2 : 0)) & 3;
  const size_t spread = fl == 1 ? zmi_gemv::LDS_MAX / 2 + 1024 : (fl == 2 ? zmi_gemv::LDS_MAX / 3 + 1024 : 0);
  const size_t lds = std::max({zmi_gemv::Img<2048>::bytes(a.M, DNW, QRT, PRO),
                               FORM == FORM_SELF ? XrImg<S>::BYTES : (FORM == FORM_SPLIT ? XcImg::BYTES : XsImg<S>::BYTES),
                               spread});
  if (lds > zmi_gemv::LDS_MAX) return hipErrorInvalidValue;
  if (lds > 64 * 1024) {
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&attn_block_kernel<S, PRO, FORM, OPROJ>), hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)zmi_gemv::LDS_MAX);
    if (attr != hipSuccess) return attr;
  }
  const int n_xs = (n_units + 7) / 8 * 8 * S;
  const int n_pf = (pf.bytes[0] > 0 || pf.bytes[1] > 0) ? pf.blocks : 0;
  const int n_op = OPROJ ? (oa->N / 8 / QG + 7) / 8 * 8 : 0;
  hipLaunchKernelGGL((attn_block_kernel<S, PRO, FORM, OPROJ>), dim3((unsigned)(n_qkv + n_xs + n_op + n_pf)), dim3(NT),
                     lds, s, a, n_cb, n_qkv, at, n_units, gran, pf, n_pf, OPROJ ? *oa : a, n_op);
  return hipGetLastError();
}

}  // namespace

extern "C" int64_t zmi_attn_block_gran_words(int rows, int hkv) {
  return (rows <= 0 || hkv <= 0) ? -1 : (int64_t)rows * hkv * GRAN_STRIDE;
}

namespace {
int attn_block(const ZmiGemvArgs* qkv, const ZmiGemvArgs* oproj, void* gran, unsigned* err, void* attn_out, int ldo,
               int slices, const ZmiPrefetch* prefetch, void* stream) {
  const ZmiGemvArgs& a = *qkv;
  if (a.K != 2048 || !a.ln_w) return zmi_fail_msg("attn_block: the QKV projection must be LayerNorm'd with K = 2048");
  const bool addln = a.pro == ZMI_PRO_ADDLN;
  if (a.pro != ZMI_PRO_AUTO && !addln) return zmi_fail_msg("attn_block: prologue must be LayerNorm or ADDLN");
  if (addln && (!a.ln_b || !a.aux || a.ld_aux % 8 || a.res_out == a.aux))
    return zmi_fail_msg("attn_block: ADDLN needs ln_b, the residual rows (ld_aux % 8) and a separate res_out");
  if (a.M < 1 || a.M > QRT) return zmi_fail_msg("attn_block: 1 <= M <= 16 rows (one row tile)");
  if (a.hd != HD || a.hkv <= 0 || a.hq != XG * a.hkv)
    return zmi_fail_msg("attn_block: head_dim 128, 4 query heads per kv head");
  if (a.N != (a.hq + 2 * a.hkv) * a.hd || a.n_valid != a.N) return zmi_fail_msg("attn_block: N = (hq + 2 hkv) hd");
  if (a.smax % 8 || !a.row_pos || !a.row_kv || !a.rope || !a.k_cache || !a.v_cache || !gran || !err || !attn_out)
    return zmi_fail_msg("attn_block: missing buffers (or smax % 8)");
  if (ldo % 8 || a.ldx % 8) return zmi_fail_msg("attn_block: ldo / ldx must be multiples of 8");
  const int n_cb = a.N / 8 / QG;
  const int n_qkv = (n_cb + 7) / 8 * 8;
  const int n_units = a.M * a.hkv;

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
  at.xc_l2 = zmi_option(ZMI_OPT_XC_HANDOFF) == 0 ? 1 : 0;
  // diagnostic builds (-DZMI_ATTN_STAMPS -DZMI_GEMV_STAMPS): both roles stamp into qkv->diag, indexed
  // by block (tools/attnblk_stamps.py)
  at.stamps = a.diag ? reinterpret_cast<unsigned long long*>(a.diag) + (size_t)a.reserved * 4096 * 8 : nullptr;
  ZmiPrefetch pf{};
  if (prefetch) {
    pf = *prefetch;
    if (zmi_prefetch_invalid(pf)) return zmi_fail_msg("attn_block: bad prefetch ranges");
  }
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  using zmi_gemv::PRO_ADDLN;
  using zmi_gemv::PRO_LN;
  const int form = (slices & ZMI_ATTNBLK_SPLIT) ? FORM_SPLIT : ((slices & ZMI_ATTNBLK_SELF) ? FORM_SELF : FORM_XS);
  const int sl = slices & ~(ZMI_ATTNBLK_SELF | ZMI_ATTNBLK_SPLIT);
  if (form == FORM_SPLIT ? (sl != 8 && sl != 24) : (sl != 4 && sl != 8))
    return zmi_fail_msg("attn_block: slices must be 4 or 8 (| ZMI_ATTNBLK_SELF), or 8 or 24 | ZMI_ATTNBLK_SPLIT");
  if (oproj) {  // the out_proj role (split forms; LayerNorm'd transformer blocks: residual epilogue; ADDLN hybrid MHA
               // blocks: plain store into the hidden rows)
    const ZmiGemvArgs& o = *oproj;
    if (form != FORM_SPLIT)
      return zmi_fail_msg("attn_block: the fused out_proj runs with the chunk-split forms");
    if (o.K != a.hq * a.hd || o.N % (8 * QG) || o.n_valid != o.N || o.M != a.M || o.ln_w || o.pro != ZMI_PRO_AUTO ||
        !o.out || o.ldo % 8 || o.ldo < o.N || o.X != attn_out)
      return zmi_fail_msg("attn_block: out_proj must be the plain residual GEMV over the attention output "
                          "(K = hq hd, N % 16 == 0, same rows, X = attn_out)");
    if (addln && (o.out == a.aux || o.out == a.res_out))
      return zmi_fail_msg("attn_block: the ADDLN block's out_proj writes the hidden rows, not the residual buffers");
    if (sl == 8)
      ZMI_CHECK(addln ? (launch_block<8, zmi_gemv::PRO_ADDLN, FORM_SPLIT, true>(a, n_cb, n_qkv, at, n_units,
                                                                                 (uint64_t*)gran, pf, s, oproj))
                      : (launch_block<8, zmi_gemv::PRO_LN, FORM_SPLIT, true>(a, n_cb, n_qkv, at, n_units, (uint64_t*)gran,
                                                                              pf, s, oproj)));
    else
      ZMI_CHECK(addln ? (launch_block<24, zmi_gemv::PRO_ADDLN, FORM_SPLIT, true>(a, n_cb, n_qkv, at, n_units,
                                                                                  (uint64_t*)gran, pf, s, oproj))
                      : (launch_block<24, zmi_gemv::PRO_LN, FORM_SPLIT, true>(a, n_cb, n_qkv, at, n_units, (uint64_t*)gran,
                                                                               pf, s, oproj)));
    return 0;
  }
#define ZMI_BLK(S_, P_, F_) launch_block<S_, P_, F_>(a, n_cb, n_qkv, at, n_units, (uint64_t*)gran, pf, s)
#define ZMI_BLK_P(P_)                                                                                \
  (form == FORM_SPLIT ? (sl == 8 ? ZMI_BLK(8, P_, FORM_SPLIT) : ZMI_BLK(24, P_, FORM_SPLIT))           \
                      : form == FORM_SELF ? (sl == 4 ? ZMI_BLK(4, P_, FORM_SELF) : ZMI_BLK(8, P_, FORM_SELF)) \
                                          : (sl == 4 ? ZMI_BLK(4, P_, FORM_XS) : ZMI_BLK(8, P_, FORM_XS)))
  e = addln ? ZMI_BLK_P(PRO_ADDLN) : ZMI_BLK_P(PRO_LN);
#undef ZMI_BLK_P
#undef ZMI_BLK
  ZMI_CHECK(e);
  return 0;
}
}  // namespace

extern "C" int zmi_attn_block_pf(const ZmiGemvArgs* qkv, void* gran, unsigned* err, void* attn_out, int ldo, int slices,
                                 const ZmiPrefetch* prefetch, void* stream) {
  return attn_block(qkv, nullptr, gran, err, attn_out, ldo, slices, prefetch, stream);
}

extern "C" int zmi_attn_block_oproj(const ZmiGemvArgs* qkv, const ZmiGemvArgs* oproj, void* gran, unsigned* err,
                                    void* attn_out, int ldo, int slices, const ZmiPrefetch* prefetch, void* stream) {
  if (!oproj) return zmi_fail_msg("attn_block_oproj: out_proj arguments required");
  return attn_block(qkv, oproj, gran, err, attn_out, ldo, slices, prefetch, stream);
}

extern "C" int zmi_attn_block_max_pos(int slices) {
  const int sl = slices & ~(ZMI_ATTNBLK_SELF | ZMI_ATTNBLK_SPLIT);
  return (slices & ZMI_ATTNBLK_SPLIT) ? (sl == 24 ? XcG<24>::KEYS : XC_KEYS) - 1
                                      : ((slices & ZMI_ATTNBLK_SELF) ? XR_KEYS - 1 : DS_KEYS - 1);
}

extern "C" int zmi_attn_block(const ZmiGemvArgs* qkv, void* gran, unsigned* err, void* attn_out, int ldo, int slices,
                              void* stream) {
  return zmi_attn_block_pf(qkv, gran, err, attn_out, ldo, slices, nullptr, stream);
}
