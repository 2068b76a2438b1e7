// GQA attention over the KV cache for decode (one query per row) and prefill (causal),
// gfx950. Replaces F.scaled_dot_product_attention(..., enable_gqa=True) at
// reference zonos/backbone/_torch.py:136 (scale 1/sqrt(hd); causal for the prefill).
//
// One workgroup = (query, kv head, chunk of CH=64 key positions). The G = Hq/Hkv query heads
// of the group share every K/V row the block reads (K/V bytes are read once per group):
//   scores : 4 lanes per key row, each 64 contiguous bytes of K (16 B/lane loads), G dots,
//            2-step lane reduction;
//   softmax: one wave per head, lane = key position (wave-reduced max / sum);
//   P.V    : lane pair-of-dims over a V row (one 256 B row per wave instruction).
// Chunk partials (m, l, o[hd]) are merged by the last-arriving chunk in chunk order, so the
// result depends only on the position, never on batch size or scheduling (batch-invariant).
// KV layout: [row][kv head][position][hd] bf16, contiguous per (row, head) stream.
#include "zmi_common.h"
#include "zmi_kernels.h"

namespace {

constexpr int CH = 64;
constexpr int HD = 128;
constexpr int MAXCH = 16384 / CH;  // RoPE table limit (_torch.py:67) bounds the positions

struct AttnArgs {
  const bf16_t* q;
  int ldq;
  const bf16_t* k;
  const bf16_t* v;
  const int* kv_row;
  const int* pos;
  int hkv, smax, maxch;
  float scale;
  bf16_t* out;
  int ldo;
  float* part;
  unsigned* counters;
};

template <int G>
__global__ __launch_bounds__(256) void attn_kernel(const AttnArgs a) {
  __shared__ float qs[G][HD];
  __shared__ float sc[G][CH];
  __shared__ float opart[4][G][HD];
  __shared__ float mlv[G][2];
  __shared__ unsigned last_flag;

  const int qi = blockIdx.x / a.hkv, kh = blockIdx.x - qi * a.hkv, c = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  // Decode passes kv_row = NULL (row qi caches into KV row qi): the K/V addresses then do not
  // depend on any load, and the chunk's K/V are requested together with the query position
  // (rows past the position are loaded but masked; all addresses stay below smax).
  const int pos = a.pos[qi];
  const int kvr = a.kv_row ? a.kv_row[qi] : qi;
  const size_t kvbase = ((size_t)kvr * a.hkv + kh) * a.smax * HD;
  const int pl = t >> 2, qq = t & 3;                          // scores: key row, quarter of hd
  const int prow = min(c * CH + pl, a.smax - 1);
  const uint4* kr = reinterpret_cast<const uint4*>(a.k + kvbase + (size_t)prow * HD + qq * 32);
  uint4 kv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) kv[i] = kr[i];
  const int dp = lane * 2, ph = wave;                          // P.V: dim pair, position phase
  uint32_t vv[CH / 4];
#pragma unroll
  for (int j = 0; j < CH / 4; ++j) {
    const int pc = min(c * CH + ph + 4 * j, a.smax - 1);
    vv[j] = *reinterpret_cast<const uint32_t*>(a.v + kvbase + (size_t)pc * HD + dp);
  }
  uint32_t qv[(G * HD / 2 + 255) / 256];
#pragma unroll
  for (int i = 0; i < (G * HD / 2 + 255) / 256; ++i) {
    const int e = min(t + i * 256, G * HD / 2 - 1);
    const int g = e / (HD / 2), d = (e % (HD / 2)) * 2;
    qv[i] = *reinterpret_cast<const uint32_t*>(a.q + (size_t)qi * a.ldq + (kh * G + g) * HD + d);
  }
  if (pos < 0) return;
  const int nch = pos / CH + 1;
  if (c >= nch) return;
  const int plim = min(CH, pos - c * CH + 1);   // valid keys in this chunk
#pragma unroll
  for (int i = 0; i < (G * HD / 2 + 255) / 256; ++i) {
    const int e = t + i * 256;
    if (e < G * HD / 2) {
      const int g = e / (HD / 2), d = (e % (HD / 2)) * 2;
      qs[g][d] = bf2f(qv[i]);
      qs[g][d + 1] = bf2f(qv[i] >> 16);
    }
  }
  __syncthreads();

  // ---- scores ----
  {
    float dot[G];
#pragma unroll
    for (int g = 0; g < G; ++g) dot[g] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t u[4] = {kv[i].x, kv[i].y, kv[i].z, kv[i].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float k0 = bf2f(u[j]), k1 = bf2f(u[j] >> 16);
        const int d = qq * 32 + i * 8 + j * 2;
#pragma unroll
        for (int g = 0; g < G; ++g) dot[g] += qs[g][d] * k0 + qs[g][d + 1] * k1;
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      dot[g] = quad_sum(dot[g]);
    }
    if (qq == 0) {
#pragma unroll
      for (int g = 0; g < G; ++g) sc[g][pl] = (pl < plim) ? dot[g] * a.scale : -INFINITY;
    }
  }
  __syncthreads();

  // ---- chunk softmax: one wave per head ----
  for (int g = wave; g < G; g += 4) {
    const float s = sc[g][lane];
    const float m = wave_max(s);
    const float e = (s == -INFINITY) ? 0.f : expf(s - m);
    const float l = wave_sum(e);
    sc[g][lane] = e;
    if (lane == 0) {
      mlv[g][0] = m;
      mlv[g][1] = l;
    }
  }
  __syncthreads();

  // ---- P.V (probabilities of clamped padding rows are 0) ----
  {
    float o0[G], o1[G];
#pragma unroll
    for (int g = 0; g < G; ++g) o0[g] = o1[g] = 0.f;
#pragma unroll
    for (int j = 0; j < CH / 4; ++j) {
      const int p = ph + 4 * j;
      const bool ok = p < plim;  // rows past the position were loaded speculatively: never let them in
      const float v0 = ok ? bf2f(vv[j]) : 0.f, v1 = ok ? bf2f(vv[j] >> 16) : 0.f;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        o0[g] += sc[g][p] * v0;
        o1[g] += sc[g][p] * v1;
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      opart[ph][g][dp] = o0[g];
      opart[ph][g][dp + 1] = o1[g];
    }
  }
  __syncthreads();

  // finalising thread -> (head, dim pair): 64 threads per head, 2 dims each
  constexpr int TPH = HD / 2;
  if (nch == 1) {
    if (t >= G * TPH) return;
    const int g_t = t / TPH, d_t = (t % TPH) * 2;
    const float inv_l = 1.0f / mlv[g_t][1];
    for (int i = 0; i < 2; ++i) {
      const int d = d_t + i;
      const float o = ((opart[0][g_t][d] + opart[1][g_t][d]) + opart[2][g_t][d]) + opart[3][g_t][d];
      a.out[(size_t)qi * a.ldo + (kh * G + g_t) * HD + d] = (bf16_t)f2bf(o * inv_l);
    }
    return;
  }

  // ---- publish chunk partial; last chunk merges in chunk order ----
  const size_t pstride = (size_t)G * (HD + 2);
  float* base = a.part + (size_t)blockIdx.x * a.maxch * pstride;
  // write-through (sc1) stores + ticket; the last chunk reads every partial with sc1 loads
  for (int e = t; e < G * HD / 2; e += 256) {
    const int g = e / (HD / 2), d = (e % (HD / 2)) * 2;
    const float v0 = ((opart[0][g][d] + opart[1][g][d]) + opart[2][g][d]) + opart[3][g][d];
    const float v1 = ((opart[0][g][d + 1] + opart[1][g][d + 1]) + opart[2][g][d + 1]) + opart[3][g][d + 1];
    st_wt64(reinterpret_cast<uint64_t*>(base + c * pstride + g * (HD + 2) + 2 + d), pack_f2(v0, v1));
  }
  if (t < G) st_wt64(reinterpret_cast<uint64_t*>(base + c * pstride + t * (HD + 2)), pack_f2(mlv[t][0], mlv[t][1]));
  if (!zmi_last_arriver_wt(a.counters + blockIdx.x, (unsigned)nch, &last_flag)) return;

  // merge, one memory round trip: each thread issues the (m, l) pair and its own two output dims of
  // every chunk as 8-byte sc1 loads before using any of them (pstride and the slab offsets are even,
  // so both pairs are 8-byte aligned). Accumulation runs in fixed chunk order (deterministic).
  if (t >= G * TPH) return;
  const int g_t = t / TPH, d_t = (t % TPH) * 2;
  const uint64_t* mlp = reinterpret_cast<const uint64_t*>(base + g_t * (HD + 2));
  const uint64_t* op = reinterpret_cast<const uint64_t*>(base + g_t * (HD + 2) + 2 + d_t);
  const size_t cs = pstride / 2;  // chunk stride in 8-byte units
  constexpr int NB = 32;
  float L = 0.f, o0 = 0.f, o1 = 0.f;
  if (nch <= NB) {
    uint64_t mlr[NB], orr[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int cc = min(u, nch - 1);  // clamped loads, never used past the end
      mlr[u] = ld_wt64(mlp + cc * cs);
      orr[u] = ld_wt64(op + cc * cs);
    }
    float mmax = -INFINITY;
#pragma unroll
    for (int u = 0; u < NB; ++u)
      if (u < nch) mmax = fmaxf(mmax, lo_f(mlr[u]));
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      if (u < nch) {
        const float w = expf(lo_f(mlr[u]) - mmax);
        L += w * hi_f(mlr[u]);
        o0 += w * lo_f(orr[u]);
        o1 += w * hi_f(orr[u]);
      }
    }
  } else {
    float mmax = -INFINITY;
    for (int c0 = 0; c0 < nch; c0 += NB) {
      uint64_t mlr[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) mlr[u] = ld_wt64(mlp + min(c0 + u, nch - 1) * cs);
#pragma unroll
      for (int u = 0; u < NB; ++u)
        if (c0 + u < nch) mmax = fmaxf(mmax, lo_f(mlr[u]));
    }
    for (int c0 = 0; c0 < nch; c0 += NB) {
      uint64_t mlr[NB], orr[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int cc = min(c0 + u, nch - 1);
        mlr[u] = ld_wt64(mlp + cc * cs);
        orr[u] = ld_wt64(op + cc * cs);
      }
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        if (c0 + u < nch) {
          const float w = expf(lo_f(mlr[u]) - mmax);
          L += w * hi_f(mlr[u]);
          o0 += w * lo_f(orr[u]);
          o1 += w * hi_f(orr[u]);
        }
      }
    }
  }
  const float inv_l = 1.0f / L;
  bf16_t* dst = a.out + (size_t)qi * a.ldo + (kh * G + g_t) * HD + d_t;
  dst[0] = (bf16_t)f2bf(o0 * inv_l);
  dst[1] = (bf16_t)f2bf(o1 * inv_l);
}

}  // namespace

extern "C" int64_t zmi_attention_partial_floats(int n_query, int hq, int hkv, int hd, int max_pos) {
  const int maxch = max_pos / CH + 1;
  return (int64_t)n_query * hkv * maxch * (hq / hkv) * (hd + 2);
}

extern "C" int zmi_attention(const void* q, int ldq, const void* k_cache, const void* v_cache, const int* q_kv_row,
                             const int* q_pos, int n_query, int hq, int hkv, int hd, int smax, int max_pos, void* out,
                             int ldo, float* partials, unsigned* counters, void* stream) {
  if (hd != HD) return zmi_fail_msg("attention: head_dim must be 128");
  if (max_pos >= smax) return zmi_fail_msg("attention: max_pos must be < smax");
  AttnArgs a;
  a.q = (const bf16_t*)q;
  a.ldq = ldq;
  a.k = (const bf16_t*)k_cache;
  a.v = (const bf16_t*)v_cache;
  a.kv_row = q_kv_row;
  a.pos = q_pos;
  a.hkv = hkv;
  a.smax = smax;
  a.maxch = max_pos / CH + 1;
  a.scale = 1.0f / sqrtf((float)hd);
  a.out = (bf16_t*)out;
  a.ldo = ldo;
  a.part = partials;
  a.counters = counters;
  dim3 grid(n_query * hkv, a.maxch);
  hipStream_t s = (hipStream_t)stream;
  switch (hq / hkv) {
    case 1: hipLaunchKernelGGL(attn_kernel<1>, grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL(attn_kernel<2>, grid, dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL(attn_kernel<4>, grid, dim3(256), 0, s, a); break;
    default: return zmi_fail_msg("attention: unsupported GQA group (1, 2, 4)");
  }
  ZMI_CHECK(hipGetLastError());
  return 0;
}
