// GQA attention over the KV cache for decode (one query per row) and prefill (causal), gfx950.
// Replaces F.scaled_dot_product_attention(..., enable_gqa=True) at reference
// zonos/backbone/_torch.py:136 (scale 1/sqrt(hd); causal for the prefill).
//
// Arithmetic: the block structure of the reference's CPU kernel (ATen's flash-attention CPU
// path, which the reference runs on its bf16 q/k/v), so that the softmax probabilities are
// rounded to bf16 at the same points:
//   s_k   = fp32(q . K_k) * scale
//   for each 512-key block j:  M_j = max(M_{j-1}, max_{k in j} s_k)
//                              e_k = exp(s_k - M_j),  P_k = bf16(e_k)
//                              l   = sum_j(e) + exp(M_{j-1} - M_j) * l
//                              acc = acc * exp(M_{j-1} - M_j) + sum_j(P_k V_k)   (fp32)
//   out   = bf16(acc * (1 / l))
// (tests/test_oracle_golden.py::test_attention_block_structure pins this against torch's CPU SDPA.)
//
// Parallel form: one 1024-thread workgroup (16 waves) per (query, kv head, 512-key block); the G
// query heads of the group share every K/V byte the block reads. Wave w owns keys 32w .. 32w+31:
//   scores : v_mfma_f32_16x16x32_bf16, A = q (rows = the G heads, padded to 16), B = K rows
//            (16 keys x 32 dims per fragment, straight from the cache);
//   softmax: block max / exp / exp sum / bf16 P, one wave per head, through LDS;
//   P.V    : v_mfma_f32_16x16x32_bf16, A = P (16 heads x the wave's 32 keys), B = V^T fragments
//            read straight from the transposed V cache ([dim][position]: 8 positions per lane).
// The 16 wave partials are summed in wave order. A block needs the maxima of the blocks before
// it (M_{j-1}): each block publishes its block maxima as 8-byte {value, tag} granules and block j
// polls those of blocks 0..j-1 (lower workgroup ids only: the blocks of a query are consecutive
// in the grid). The partials (o, l, M_j) are merged in block order by the last-arriving block of
// the query, which also re-arms the tags. The result depends only on the query's position,
// never on batch size or scheduling.
// Cache layouts: K [row][kv head][position][128], V^T [row][kv head][128][position], bf16.
#include "zmi_common.h"
#include "zmi_kernels.h"

namespace {

constexpr int HD = 128;
constexpr int BLK = 512;  // kvSplitSize of the reference's CPU attention
constexpr int NW = 16;    // waves per workgroup
constexpr int KPW = BLK / NW;
constexpr int NT = NW * 64;
constexpr unsigned SPIN_LIMIT = 1u << 20;

struct AttnArgs {
  const bf16_t* q;
  int ldq;
  const bf16_t* k;
  const bf16_t* v;
  const int* kv_row;
  const int* pos;
  int hkv, smax, nblk;
  float scale;
  bf16_t* out;
  int ldo;
  unsigned* err;       // nonzero after a hand-off poll gave up
  unsigned* tickets;   // [unit]
  uint64_t* gran;      // [unit][nblk][G]   {block max, tag}
  float* part;         // [unit][nblk][G][HD + 2]   o[HD], l, M_j
};

__device__ __forceinline__ f32x4_t mfma16(const uint4& a, const uint4& b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

template <int G>
__global__ __launch_bounds__(NT) void attn_kernel(const AttnArgs a) {
  __shared__ float sc[G][BLK];
  __shared__ __attribute__((aligned(16))) bf16_t pb[G][BLK];
  __shared__ float opart[NW][G][HD];
  __shared__ float mj[G], lj[G];
  __shared__ unsigned last_flag;

  const int unit = blockIdx.x / a.nblk, j = blockIdx.x - unit * a.nblk;
  const int qi = unit / a.hkv, kh = unit - qi * a.hkv;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int pos = a.pos[qi];
  if (pos < 0) return;
  const int nb = pos / BLK + 1;
  if (j >= nb) return;
  const int key0 = j * BLK;
  const int nkeys = min(BLK, pos + 1 - key0);
  const int kvr = a.kv_row ? a.kv_row[qi] : qi;
  const size_t kvbase = ((size_t)kvr * a.hkv + kh) * a.smax * HD;
  const int last_key = key0 + nkeys - 1;
  const int c16 = lane & 15, h4 = lane >> 4;

  // ---- q (A operand: row = head, zero rows past G) and this wave's K rows (B operand) ----
  uint4 qf[4];
  {
    const bool real = c16 < G;
    const bf16_t* qr = a.q + (size_t)qi * a.ldq + (kh * G + (real ? c16 : 0)) * HD + 8 * h4;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      qf[db] = *reinterpret_cast<const uint4*>(qr + 32 * db);
      if (!real) qf[db] = uint4{0u, 0u, 0u, 0u};
    }
  }
  uint4 kf[2][4];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int key = min(key0 + wave * KPW + 16 * tt + c16, last_key);
    const bf16_t* kr = a.k + kvbase + (size_t)key * HD + 8 * h4;
#pragma unroll
    for (int db = 0; db < 4; ++db) kf[tt][db] = *reinterpret_cast<const uint4*>(kr + 32 * db);
  }

  // ---- scores s = fp32(q . k) * scale; keys past the position are -inf ----
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    f32x4_t s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int db = 0; db < 4; ++db) s = mfma16(qf[db], kf[tt][db], s);
    const int key = wave * KPW + 16 * tt + c16;  // accumulator: column = key, row = head 4 h4 + i
    if (h4 == 0) {
#pragma unroll
      for (int i = 0; i < G; ++i) sc[i][key] = key < nkeys ? s[i] * a.scale : -INFINITY;
    }
  }
  // ---- V^T fragments for P.V (B operand: dim = 16 dt + c16, positions 32 w + 8 h4 .. +7) ----
  __builtin_amdgcn_sched_barrier(0);
  uint4 vf[8];
  {
    const int p0 = min(key0 + wave * KPW + 8 * h4, a.smax - 8);  // 8 positions stay inside the row
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
      vf[dt] = *reinterpret_cast<const uint4*>(a.v + kvbase + (size_t)(16 * dt + c16) * a.smax + p0);
  }
  __builtin_amdgcn_sched_barrier(0);
  __syncthreads();

  // ---- block maxima (one wave per head) ----
  if (wave < G) {
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < BLK / 64; ++i) m = fmaxf(m, sc[wave][lane + 64 * i]);
    m = wave_max(m);
    if (lane == 0) mj[wave] = m;
  }
  __syncthreads();

  // ---- running maximum M_j = max(block max, maxima of blocks 0..j-1) ----
  uint64_t* gu = a.gran + (size_t)unit * a.nblk * G;
  if (nb > 1 && t < G) {
    const float m = mj[t];
    st_wt64(gu + j * G + t, pack_f2(m, 1.0f));  // {value, tag = 1.0f}: one untorn 8-byte granule
    float mm = m;
    for (int jj = 0; jj < j; ++jj) {
      uint64_t v = ld_wt64(gu + jj * G + t);
      unsigned spins = 0;
      while (hi_f(v) != 1.0f) {
        if (++spins > SPIN_LIMIT) {
          __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        v = ld_wt64(gu + jj * G + t);
      }
      mm = fmaxf(mm, lo_f(v));
    }
    mj[t] = mm;
  }
  __syncthreads();

  // ---- e = exp(s - M_j), l = sum e (fp32), P = bf16(e) ----
  if (wave < G) {
    const float M = mj[wave];
    float l = 0.f;
#pragma unroll
    for (int i = 0; i < BLK / 64; ++i) {
      const int kk = lane + 64 * i;
      const float e = kk < nkeys ? expf(sc[wave][kk] - M) : 0.f;
      l += e;
      pb[wave][kk] = (bf16_t)f2bf(e);
    }
    l = wave_sum(l);
    if (lane == 0) lj[wave] = l;
  }
  __syncthreads();

  // ---- P.V: this wave's 32 keys x 128 dims (V of keys past the position is zeroed: never let
  // stale cache bytes into the sum) ----
  {
    uint4 pf = uint4{0u, 0u, 0u, 0u};
    if (c16 < G) pf = *reinterpret_cast<const uint4*>(&pb[c16][wave * KPW + 8 * h4]);
    const int kbase = wave * KPW + 8 * h4;  // first key of this lane's 8 positions
    if (kbase + 8 > nkeys) {
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        uint32_t w[4] = {vf[dt].x, vf[dt].y, vf[dt].z, vf[dt].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t lo = kbase + 2 * e < nkeys ? 0x0000ffffu : 0u;
          const uint32_t hi = kbase + 2 * e + 1 < nkeys ? 0xffff0000u : 0u;
          w[e] &= lo | hi;
        }
        vf[dt] = uint4{w[0], w[1], w[2], w[3]};
      }
    }
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      const f32x4_t o = mfma16(pf, vf[dt], f32x4_t{0.f, 0.f, 0.f, 0.f});
      if (h4 == 0) {  // column = dim 16 dt + c16, row = head i
#pragma unroll
        for (int i = 0; i < G; ++i) opart[wave][i][16 * dt + c16] = o[i];
      }
    }
  }
  __syncthreads();

  constexpr int NOUT = G * HD;  // (head, dim) outputs; thread t < NOUT owns one
  float o = 0.f;
  const int g_t = t / HD, d_t = t - g_t * HD;
  if (t < NOUT) {
    o = opart[0][g_t][d_t];
#pragma unroll
    for (int w = 1; w < NW; ++w) o += opart[w][g_t][d_t];
  }
  bf16_t* dst = a.out + (size_t)qi * a.ldo + kh * G * HD;
  if (nb == 1) {
    if (t < NOUT) dst[t] = (bf16_t)f2bf(o * (1.0f / lj[g_t]));
    return;
  }

  // ---- publish this block's partial; the last-arriving block merges in block order ----
  float* pu = a.part + (size_t)unit * a.nblk * G * (HD + 2);
  if (t < NOUT) st_wt(pu + ((size_t)j * G + g_t) * (HD + 2) + d_t, o);
  if (t < G) {
    st_wt(pu + ((size_t)j * G + t) * (HD + 2) + HD, lj[t]);
    st_wt(pu + ((size_t)j * G + t) * (HD + 2) + HD + 1, mj[t]);
  }
  if (!zmi_last_arriver_wt(a.tickets + unit, (unsigned)nb, &last_flag)) return;
  if (t < nb * G) st_wt64(gu + t, 0ull);  // re-arm the granules (every block of the query has polled)
  if (t >= NOUT) return;
  const float* pg = pu + (size_t)g_t * (HD + 2);
  const size_t bs = (size_t)G * (HD + 2);
  float acc = ld_wt(pg + d_t), l = ld_wt(pg + HD), mprev = ld_wt(pg + HD + 1);
  for (int jj = 1; jj < nb; ++jj) {
    const float* pj = pg + jj * bs;
    const float oj = ld_wt(pj + d_t), lb = ld_wt(pj + HD), mb = ld_wt(pj + HD + 1);
    const float et = expf(mprev - mb);
    l = lb + et * l;
    acc = acc * et + oj;
    mprev = mb;
  }
  dst[t] = (bf16_t)f2bf(acc * (1.0f / l));
}

struct WorkLayout {
  size_t tickets, gran, part, total;
};
WorkLayout work_layout(int n_query, int g, int hkv, int max_pos) {
  const size_t units = (size_t)n_query * hkv, nblk = (size_t)max_pos / BLK + 1;
  WorkLayout w;
  w.tickets = 256;
  w.gran = w.tickets + ((units * 4 + 255) / 256) * 256;
  w.part = w.gran + ((units * nblk * g * 8 + 255) / 256) * 256;
  w.total = w.part + units * nblk * g * (HD + 2) * 4;
  return w;
}

}  // namespace

extern "C" int64_t zmi_attention_work_bytes(int n_query, int hq, int hkv, int hd, int max_pos) {
  if (hd != HD || hkv <= 0 || hq % hkv || n_query <= 0 || max_pos < 0) return -1;
  return (int64_t)work_layout(n_query, hq / hkv, hkv, max_pos).total;
}

extern "C" int zmi_attention(const void* q, int ldq, const void* k_cache, const void* v_cache, const int* q_kv_row,
                             const int* q_pos, int n_query, int hq, int hkv, int hd, int smax, int max_pos, void* out,
                             int ldo, void* work, void* stream) {
  if (hd != HD) return zmi_fail_msg("attention: head_dim must be 128");
  if (max_pos >= smax) return zmi_fail_msg("attention: max_pos must be < smax");
  if (smax % 8) return zmi_fail_msg("attention: smax must be a multiple of 8");
  if (ldq % 8) return zmi_fail_msg("attention: ldq must be a multiple of 8");
  if (n_query <= 0) return 0;
  if (!work) return zmi_fail_msg("attention: work buffer required (zmi_attention_work_bytes)");
  const int g = hkv > 0 ? hq / hkv : 0;
  if (g * hkv != hq) return zmi_fail_msg("attention: hq must be a multiple of hkv");
  const WorkLayout w = work_layout(n_query, g, hkv, max_pos);
  char* wb = (char*)work;
  AttnArgs a;
  a.q = (const bf16_t*)q;
  a.ldq = ldq;
  a.k = (const bf16_t*)k_cache;
  a.v = (const bf16_t*)v_cache;
  a.kv_row = q_kv_row;
  a.pos = q_pos;
  a.hkv = hkv;
  a.smax = smax;
  a.nblk = max_pos / BLK + 1;
  a.scale = 1.0f / sqrtf((float)hd);
  a.out = (bf16_t*)out;
  a.ldo = ldo;
  a.err = (unsigned*)wb;
  a.tickets = (unsigned*)(wb + w.tickets);
  a.gran = (uint64_t*)(wb + w.gran);
  a.part = (float*)(wb + w.part);
  const int64_t blocks = (int64_t)n_query * hkv * a.nblk;
  if (blocks > 0x7fffffff) return zmi_fail_msg("attention: grid too large");
  hipStream_t s = (hipStream_t)stream;
  switch (g) {
    case 1: hipLaunchKernelGGL(attn_kernel<1>, dim3((unsigned)blocks), dim3(NT), 0, s, a); break;
    case 2: hipLaunchKernelGGL(attn_kernel<2>, dim3((unsigned)blocks), dim3(NT), 0, s, a); break;
    case 4: hipLaunchKernelGGL(attn_kernel<4>, dim3((unsigned)blocks), dim3(NT), 0, s, a); break;
    default: return zmi_fail_msg("attention: unsupported GQA group (1, 2, 4)");
  }
  ZMI_CHECK(hipGetLastError());
  return 0;
}
