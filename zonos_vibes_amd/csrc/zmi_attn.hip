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
// Parallel form: one workgroup of NWC waves per (query, kv head, chunk of CH = 32 NWC keys); a
// 512-key block is CPB = 512 / CH chunks. The G query heads of the group share every K/V byte the
// chunk reads. Wave w owns 32 keys of the chunk:
//   scores : v_mfma_f32_16x16x32_bf16, A = q (rows = the G heads, padded to 16), B = K rows
//            (16 keys x 32 dims per fragment, straight from the cache);
//   softmax: chunk max / exp / exp sum / bf16 P through LDS;
//   P.V    : v_mfma_f32_16x16x32_bf16, A = P (16 heads x the wave's 32 keys), B = V^T fragments
//            read straight from the transposed V cache ([dim][position]: 8 positions per lane).
// M_j needs the maxima of every chunk of blocks 0..j: each chunk publishes its maxima as 8-byte
// {value, tag} granules and polls the others' (bounded spin; a give-up sets the error word).
// The chunk partials (o, l, M_j; layout and merge order in zmi_attn_merge.h) are merged by the
// last-arriving chunk of the query. (Deferring the merge into out_proj's prologue was measured:
// attention 12.2 -> 9.2 us but out_proj 4.0 -> 7.8 us per layer at C2, so it is not done.) Every query runs the same
// arithmetic whatever the batch: the result depends only on its position (CH is a constant).
// Cache layouts: K [row][kv head][position][128], V^T [row][kv head][128][position], bf16.
#include "zmi_common.h"
#include "zmi_kernels.h"
#include "zmi_attn_merge.h"
#include "zmi_attn_ds.h"
#include "zmi_gemv_impl.h"
#include "zmi_prefetch.h"

namespace {

using namespace zmi_attn;
constexpr int NT = NWC * 64;
constexpr unsigned SPIN_LIMIT = 1u << 20;




// MODE 0: one launch, the cross-chunk maxima exchanged by granules while the chunks wait. MODE 1 + MODE 2: two
// launches with no waiting: 1 computes the chunk's scores and maxima and leaves them in its own partial slots
// (scores in part_o, maxima in part_lm's M word); 2 forms M_j from those maxima, reads its scores back and
// finishes as MODE 0 does. MODE 3 is MODE 2 without the ticket: it leaves its chunk partial (plain stores) for
// attn_merge_kernel, a third launch. All give the same bits: max is exact in any order, every other step is shared
// code (merge2 performs merge4's operations per element).
template <int G, int MODE>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(G == 4 ? 6 : 1, 8))) void attn_kernel(const AttnArgs a) {
  __shared__ float sc[G][CH];
  __shared__ __attribute__((aligned(16))) bf16_t pb[G][CH];
  __shared__ float opart[NWC][G][HD];
  __shared__ float mj[G], lj[G];
  __shared__ float pmax[NT];
  __shared__ unsigned last_flag;

  if constexpr (MODE == 0) {
    if ((int)blockIdx.x >= a.n_att) {  // prefetch-only workgroup (zmi_attention_pf), dispatched after the chunks
      prefetch_body<NT>(a.pf, (int)blockIdx.x - a.n_att, a.n_pf);
      return;
    }
  }
  const int unit = blockIdx.x / a.nch, c = blockIdx.x - unit * a.nch;
  const int qi = unit / a.hkv, kh = unit - qi * a.hkv;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int pos = a.pos[qi];
  const int nc = chunks_of(pos);  // chunks of this query
  if (c >= nc) return;
  const int j = c / CPB;                               // its 512-key block
  const int dep = min((j + 1) * CPB, nc);              // chunks 0 .. dep-1 make up M_j
  const int key0 = c * CH;
  const int nkeys = min(CH, pos + 1 - key0);
  const int kvr = a.kv_row ? a.kv_row[qi] : qi;
  const size_t kvbase = ((size_t)kvr * a.hkv + kh) * a.smax * HD;
  const int last_key = key0 + nkeys - 1;
  const int c16 = lane & 15, h4 = lane >> 4;
  ZMI_ASTAMP(0);

  // ---- q (A operand: row = head, zero rows past G) and this wave's K rows (B operand). With G = 4 the
  // group's q (4 heads x 128 dims = 1 KiB) comes into LDS by one LDS-DMA piece, so no q registers are live
  // under the K / V loads (98 -> 78 VGPRs: 6 workgroups per CU instead of 4) ----
  __shared__ __attribute__((aligned(16))) bf16_t qs[G == 4 ? G * HD : 8];
  uint4 qf[4];
  uint4 kf[2][4];
  uint4 vf[8];
  float* po = a.part_o + ((size_t)unit * a.nch + c) * G * HD;
  float* plm = a.part_lm + ((size_t)unit * a.nch + c) * G * 2;
  if constexpr (MODE >= 2) {
    // launch 1's maxima of chunks 0..dep-1 and this chunk's scores first, then V^T: loads complete in order, so
    // M_j is formed while V^T is in flight (one memory round trip, not two)
    const float* lu = a.part_lm + (size_t)unit * a.nch * G * 2;
    const int p0 = min(key0 + wave * 32 + 8 * h4, (last_key & ~7));
    const float mine = t < dep * G ? lu[2 * t + 1] : -INFINITY;  // e = t = chunk * G + head
    const float4 sv = t * 4 < G * CH ? ld4(po + t * 4) : float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
      vf[dt] = *reinterpret_cast<const uint4*>(a.v + kvbase + (size_t)(16 * dt + c16) * a.smax + p0);
    float m = mine;
    for (int e = t + NT; e < dep * G; e += NT) m = fmaxf(m, lu[2 * e + 1]);  // positions >= 64 NT / G only
    if (t * 4 < G * CH) *reinterpret_cast<float4*>(&sc[(t * 4) / CH][(t * 4) % CH]) = sv;
    pmax[t] = m;
    __syncthreads();
    if (t < G) {  // thread t gathers head t: entries e = t, t + G, ... hold head t (NT % G == 0)
      float mm = -INFINITY;
      for (int e = t; e < NT; e += G) mm = fmaxf(mm, pmax[e]);
      mj[t] = mm;
    }
    __syncthreads();
    ZMI_ASTAMP(1);
  } else {
  if constexpr (G == 4) {
    if (wave == 0) zmi_gemv::dma_piece(a.q + (size_t)qi * a.ldq + kh * G * HD + lane * 8, qs);
  } else {
    const bool real = c16 < G;
    const bf16_t* qr = a.q + (size_t)qi * a.ldq + (kh * G + (real ? c16 : 0)) * HD + 8 * h4;
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      qf[db] = *reinterpret_cast<const uint4*>(qr + 32 * db);
      if (!real) qf[db] = uint4{0u, 0u, 0u, 0u};
    }
  }
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int key = min(key0 + wave * 32 + 16 * tt + c16, last_key);
    const bf16_t* kr = a.k + kvbase + (size_t)key * HD + 8 * h4;
#pragma unroll
    for (int db = 0; db < 4; ++db) kf[tt][db] = *reinterpret_cast<const uint4*>(kr + 32 * db);
  }
  // V^T fragments for P.V, issued with K so both streams share one memory latency (B operand:
  // dim = 16 dt + c16, positions 32 w + 8 h4 .. +7; groups wholly past the position re-read the
  // last valid group, their keys are masked below)
  if constexpr (MODE == 0) {
    const int p0 = min(key0 + wave * 32 + 8 * h4, (last_key & ~7));
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
      vf[dt] = *reinterpret_cast<const uint4*>(a.v + kvbase + (size_t)(16 * dt + c16) * a.smax + p0);
  }

  if constexpr (G == 4) {  // the q piece (issued before the 16 K / V loads, or the 8 K loads, which complete after it)
    if constexpr (MODE == 0) {
      if (wave == 0) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else {
      if (wave == 0) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    }
    __syncthreads();
  }
  // ---- scores s = fp32(q . k) * scale (dim blocks in order per key tile); keys past the position are -inf ----
  f32x4_t st[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int db = 0; db < 4; ++db) {
    uint4 qv = qf[db];
    if constexpr (G == 4)
      qv = c16 < G ? *reinterpret_cast<const uint4*>(&qs[c16 * HD + 8 * h4 + 32 * db]) : uint4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) st[tt] = mfma16(qv, kf[tt][db], st[tt]);
  }
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const f32x4_t s = st[tt];
    const int key = wave * 32 + 16 * tt + c16;  // accumulator: column = key, row = head 4 h4 + i
    if (h4 == 0) {
#pragma unroll
      for (int i = 0; i < G; ++i) sc[i][key] = key < nkeys ? s[i] * a.scale : -INFINITY;
    }
  }
  __syncthreads();
  ZMI_ASTAMP(1);

  // ---- chunk maxima: a wave per head, lane scans keys lane, lane + 64 .. ----
  for (int g = wave; g < G; g += NWC) {
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < CH / 64; ++i) m = fmaxf(m, sc[g][lane + 64 * i]);
    m = wave_max(m);
    if (lane == 0) mj[g] = m;
  }
  __syncthreads();
  ZMI_ASTAMP(2);
  if constexpr (MODE == 1) {  // leave the scores and maxima in the chunk's own partial slots for launch 2
#pragma unroll
    for (int e = t * 4; e < G * CH; e += NT * 4) *reinterpret_cast<float4*>(po + e) = *reinterpret_cast<const float4*>(&sc[e / CH][e % CH]);
    if (t < G) plm[2 * t + 1] = mj[t];
    return;
  }
  }  // MODE != 2

  // ---- running maximum M_j = max over the chunks of blocks 0..j: {value, tag} granule exchange ----
  uint64_t* gu = a.gran + (size_t)unit * a.nch * G;
  if (MODE == 0 && nc > 1 && t < G) st_wt64(gu + c * G + t, pack_f2(mj[t], 1.0f));  // {value, tag 1.0f}: untorn granule
  if (MODE == 0 && dep > 1) {
    float m = -INFINITY;
    for (int e = t; e < dep * G; e += NT) {  // e = chunk * G + head
      if (e / G == c) {
        m = fmaxf(m, mj[e % G]);
        continue;
      }
      uint64_t v = ld_wt64(gu + e);
      unsigned spins = 0;
      while (hi_f(v) != 1.0f) {
        if (++spins > SPIN_LIMIT) {
          __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        v = ld_wt64(gu + e);
      }
      m = fmaxf(m, lo_f(v));
    }
    pmax[t] = m;
    __syncthreads();
    if (t < G) {  // thread t gathers head t: entries e = t, t + G, ... hold head t (NT % G == 0)
      float mm = -INFINITY;
      for (int e = t; e < NT; e += G) mm = fmaxf(mm, pmax[e]);
      mj[t] = mm;
    }
    __syncthreads();
  }
  ZMI_ASTAMP(3);

  // ---- e = exp(s - M_j), l = sum e (fp32), P = bf16(e) ----
  for (int g = wave; g < G; g += NWC) {
    const float M = mj[g];
    float l = 0.f;
#pragma unroll
    for (int i = 0; i < CH / 64; ++i) {
      const int kk = lane + 64 * i;
      const float e = kk < nkeys ? expf(sc[g][kk] - M) : 0.f;
      l += e;
      pb[g][kk] = (bf16_t)f2bf(e);
    }
    l = wave_sum(l);
    if (lane == 0) lj[g] = l;
  }
  __syncthreads();
  ZMI_ASTAMP(4);

  // ---- P.V: this wave's 32 keys x 128 dims (V of keys past the position is zeroed: never let
  // stale cache bytes into the sum) ----
  {
    uint4 pf = uint4{0u, 0u, 0u, 0u};
    if (c16 < G) pf = *reinterpret_cast<const uint4*>(&pb[c16][wave * 32 + 8 * h4]);
    const int kbase = wave * 32 + 8 * h4;  // first key of this lane's 8 positions
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

  // ---- chunk partial (waves in order) ----
  bf16_t* dst = a.out + (size_t)qi * a.ldo + kh * G * HD;
  if constexpr (MODE == 3) {  // plain stores, 4 dims per thread; attn_merge_kernel merges after the launch
    for (int e = t * 4; e < G * HD; e += NT * 4) {
      const int g = e / HD, d = e - g * HD;
      float4 o = *reinterpret_cast<const float4*>(&opart[0][g][d]);
#pragma unroll
      for (int w = 1; w < NWC; ++w) {
        const float4 p = *reinterpret_cast<const float4*>(&opart[w][g][d]);
        o.x += p.x;
        o.y += p.y;
        o.z += p.z;
        o.w += p.w;
      }
      if (nc == 1) {
        const float r = 1.0f / lj[g];
        *reinterpret_cast<uint2*>(dst + e) =
            uint2{f2bf(o.x * r) | (f2bf(o.y * r) << 16), f2bf(o.z * r) | (f2bf(o.w * r) << 16)};
      } else {
        *reinterpret_cast<float4*>(po + e) = o;
      }
    }
    if (nc > 1 && t < G) *reinterpret_cast<float2*>(plm + 2 * t) = float2{lj[t], mj[t]};
    return;
  }
  for (int e = t; e < G * HD; e += NT) {
    const int g = e / HD, d = e - g * HD;
    float o = opart[0][g][d];
#pragma unroll
    for (int w = 1; w < NWC; ++w) o += opart[w][g][d];
    if (nc == 1)  // a one-chunk query is finished here
      dst[e] = (bf16_t)f2bf(o * (1.0f / lj[g]));
    else
      st_wt(po + e, o);
  }
  if (nc == 1) return;
  if (t < G) {
    st_wt(plm + 2 * t, lj[t]);
    st_wt(plm + 2 * t + 1, mj[t]);
  }
  ZMI_ASTAMP(5);
  if (!zmi_last_arriver_wt(a.tickets + unit, (unsigned)nc, &last_flag)) return;
  ZMI_ASTAMP(6);
  if constexpr (MODE == 0)
    for (int e = t; e < nc * G; e += NT) st_wt64(gu + e, 0ull);  // re-arm (every chunk has polled)

  // ---- merge (zmi_attn_merge.h), 4 dims per thread. The partials were stored write-through by
  // their chunks; one agent-scope acquire here, then plain loads (MI355X_MICROARCH.md, Valid forms) ----
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const float* ou = a.part_o + (size_t)unit * a.nch * G * HD;
  const float* lu = a.part_lm + (size_t)unit * a.nch * G * 2;
  if constexpr (MODE == 2) {  // 2 dims per thread, 16 chunks' loads in flight
    for (int e = t * 2; e < G * HD; e += NT * 2) {
      const int g = e / HD, d = e - g * HD;
      const float2 r = merge2<16>(ou, lu, nc, g, d, G);
      *reinterpret_cast<uint32_t*>(dst + e) = f2bf(r.x) | (f2bf(r.y) << 16);
    }
  } else {
    for (int e = t * 4; e < G * HD; e += NT * 4) {
      const int g = e / HD, d = e - g * HD;
      const float4 r = merge4(ou, lu, nc, g, d, G);
      *reinterpret_cast<uint2*>(dst + e) = uint2{f2bf(r.x) | (f2bf(r.y) << 16), f2bf(r.z) | (f2bf(r.w) << 16)};
    }
  }
  ZMI_ASTAMP(7);
}

// ---- block form (variant 5): one 8-wave workgroup per (query, kv head, 512-key softmax block) ----
// Wave w owns keys 64 w .. 64 w + 63 of the block as two 32-key tiles (the chunked kernel's wave unit), so a
// 128-key chunk is tiles 4 cc .. 4 cc + 3. Every per-chunk operation is the chunked kernel's: the same score
// MFMA chain, l of chunk cc and head g summed by one wave over lanes L and L + 64, P = bf16(e), P.V per tile
// from zero, the chunk's tiles summed in tile order, then (zmi_attn_merge.h) the block's chunks in chunk order
// and the blocks folded by the reference recursion. What changes is who waits: the chunks of a block need no
// exchange (the block maximum is local), and block j only needs the maxima of blocks 0 .. j - 1, whose
// workgroups come earlier in the grid; one partial and one ticket per block instead of per chunk. The V^T
// loads are issued after the scores (the K registers are dead by then), so they run during that wait.
constexpr int BNW = 8, BNT = BNW * 64;
constexpr int BTL = BLK / 32;  // 32-key tiles per block

template <int G>
__global__ __launch_bounds__(BNT) __attribute__((amdgpu_waves_per_eu(4, 8))) void attn_blk_kernel(const AttnArgs a) {
  __shared__ float sc[G][BLK];
  __shared__ __attribute__((aligned(16))) bf16_t pb[G][BLK];
  __shared__ float opart[BTL][G][HD];
  __shared__ __attribute__((aligned(16))) bf16_t qs[G * HD];
  __shared__ float mj[G], bmx[G], lch[CPB][G];
  __shared__ unsigned last_flag;

  if ((int)blockIdx.x >= a.n_att) {  // prefetch-only workgroup (zmi_attention_pf)
    prefetch_body<BNT>(a.pf, (int)blockIdx.x - a.n_att, a.n_pf);
    return;
  }
  // block-major order: the live blocks (j < the row's block count) come first and every unit's blocks spread
  // over the XCDs (workgroups are dealt round-robin; unit-major order with the KV capacity's 12 blocks put all
  // live blocks of a C5 step on 4 of the 8 XCDs: 26.8 against 17.1 us at 16 rows x 1000 keys); block j waits
  // only for blocks 0 .. j - 1 of its unit, which this order dispatches earlier
  const int n_units = a.n_att / ((a.nch + CPB - 1) / CPB);
  const int j = blockIdx.x / n_units, unit = blockIdx.x - j * n_units;
  const int qi = unit / a.hkv, kh = unit - qi * a.hkv;
  const int pos = a.pos[qi];
  const int nc = chunks_of(pos), nb = (nc + CPB - 1) / CPB;
  if (j >= nb) return;
  ZMI_ASTAMP(0);  // diagnostic builds (tools/attn_blk_stamps.py): 0 start, 1 q in LDS, 2 scores, 3 block maxima
                  // exchanged, 4 P, 5 P.V (V landed), 6 partial out, 7 end (the last arriver: merge done)
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c16 = lane & 15, h4 = lane >> 4;
  const int key0 = j * BLK;
  const int nkeys = min(BLK, pos + 1 - key0), last_key = key0 + nkeys - 1;
  const int ncb = (nkeys + CH - 1) / CH;  // chunks of this block
  const int kvr = a.kv_row ? a.kv_row[qi] : qi;
  const size_t kvbase = ((size_t)kvr * a.hkv + kh) * a.smax * HD;

  // q: with G = 4 one 1 KiB LDS-DMA piece that lands under the K loads (a load + LDS store would make the wave
  // wait for q before issuing any K load); smaller groups by plain loads
  if constexpr (G == 4) {
    if (wave == 0) zmi_gemv::dma_piece(a.q + (size_t)qi * a.ldq + kh * G * HD + lane * 8, qs);
  } else {
    if (t < G * HD / 8)
      *reinterpret_cast<uint4*>(&qs[t * 8]) = *reinterpret_cast<const uint4*>(a.q + (size_t)qi * a.ldq + kh * G * HD + t * 8);
  }
  uint4 kf[2][2][4];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int key = min(key0 + 32 * (2 * wave + k) + 16 * tt + c16, last_key);
      const bf16_t* kr = a.k + kvbase + (size_t)key * HD + 8 * h4;
#pragma unroll
      for (int db = 0; db < 4; ++db) kf[k][tt][db] = *reinterpret_cast<const uint4*>(kr + 32 * db);
    }
  if constexpr (G == 4) {  // the q piece was issued before the 16 K loads, which complete after it
    if (wave == 0) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  }
  __syncthreads();  // q in LDS
  ZMI_ASTAMP(1);
  // ---- scores (the chunked kernel's chain per 16-key sub-tile); keys past the position are -inf ----
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    f32x4_t st[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int db = 0; db < 4; ++db) {
      const uint4 qv = c16 < G ? *reinterpret_cast<const uint4*>(&qs[c16 * HD + 8 * h4 + 32 * db]) : uint4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) st[tt] = mfma16(qv, kf[k][tt][db], st[tt]);
    }
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int key = 32 * (2 * wave + k) + 16 * tt + c16;  // block-local
      if (h4 == 0) {
#pragma unroll
        for (int i = 0; i < G; ++i) sc[i][key] = key < nkeys ? st[tt][i] * a.scale : -INFINITY;
      }
    }
  }
  __syncthreads();
  ZMI_ASTAMP(2);
  // ---- V^T fragments of the wave's two tiles (issued now, landing while the block maxima are exchanged) ----
  uint4 vf[2][8];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int p0 = min(key0 + 32 * (2 * wave + k) + 8 * h4, last_key & ~7);
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
      vf[k][dt] = *reinterpret_cast<const uint4*>(a.v + kvbase + (size_t)(16 * dt + c16) * a.smax + p0);
  }
  // ---- block maxima (exact in any order), out as {value, tag} granules; M_j = max over blocks 0..j ----
  if (wave < G) {
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < BLK / 64; ++i) m = fmaxf(m, sc[wave][lane + 64 * i]);
    m = wave_max(m);
    if (lane == 0) bmx[wave] = m;
  }
  __syncthreads();
  uint64_t* gu = a.gran + (size_t)unit * a.nch * G;  // [block][head] in the unit's granule area
  if (wave == 0) {
    if (nb > 1 && lane < G) st_xc64(gu + j * G + lane, pack_f2(bmx[lane], 1.0f), a.xc_l2);
    float m = lane < G ? bmx[lane] : -INFINITY;
    for (int e = lane; e < j * G; e += 64) {  // e = block x G + head (64 % G == 0: lane's head is lane % G)
      uint64_t v = ld_wt64(gu + e);
      for (unsigned spins = 0; hi_f(v) != 1.0f; ++spins) {
        if (spins > SPIN_LIMIT) {
          __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        v = ld_wt64(gu + e);
      }
      m = fmaxf(m, lo_f(v));
    }
#pragma unroll
    for (int off = G; off < 64; off <<= 1) m = fmaxf(m, __shfl_xor(m, off));
    if (lane < G) mj[lane] = m;
  }
  __syncthreads();
  ZMI_ASTAMP(3);
  // ---- e = exp(s - M_j), l per (chunk, head) as the chunked kernel's wave does it, P = bf16(e) ----
  for (int task = wave; task < CPB * G; task += BNW) {
    const int cc = task / G, g = task - cc * G;
    const float M = mj[g];
    float l = 0.f;
#pragma unroll
    for (int i = 0; i < CH / 64; ++i) {
      const int kk = cc * CH + lane + 64 * i;
      const float e = kk < nkeys ? expf(sc[g][kk] - M) : 0.f;
      l += e;
      pb[g][kk] = (bf16_t)f2bf(e);
    }
    l = wave_sum(l);
    if (lane == 0) lch[cc][g] = l;
  }
  __syncthreads();
  ZMI_ASTAMP(4);
  // ---- P.V per 32-key tile (V of keys past the position zeroed) ----
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int tl = 2 * wave + k;
    uint4 pf = uint4{0u, 0u, 0u, 0u};
    if (c16 < G) pf = *reinterpret_cast<const uint4*>(&pb[c16][32 * tl + 8 * h4]);
    const int kbase = 32 * tl + 8 * h4;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      uint4 v = vf[k][dt];
      if (kbase + 8 > nkeys) {
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t lo = kbase + 2 * e < nkeys ? 0x0000ffffu : 0u;
          const uint32_t hi = kbase + 2 * e + 1 < nkeys ? 0xffff0000u : 0u;
          w[e] &= lo | hi;
        }
        v = uint4{w[0], w[1], w[2], w[3]};
      }
      const f32x4_t o = mfma16(pf, v, f32x4_t{0.f, 0.f, 0.f, 0.f});
      if (h4 == 0) {
#pragma unroll
        for (int i = 0; i < G; ++i) opart[tl][i][16 * dt + c16] = o[i];
      }
    }
  }
  __syncthreads();
  ZMI_ASTAMP(5);
  // ---- the block's partial: chunks' tiles in tile order, then the chunks in chunk order ----
  float* po = a.part_o + ((size_t)unit * a.nch + j) * G * HD;
  float* plm = a.part_lm + ((size_t)unit * a.nch + j) * G * 2;
  bf16_t* dst = a.out + (size_t)qi * a.ldo + kh * G * HD;
  for (int e = t; e < G * HD; e += BNT) {
    const int g = e / HD, d = e - g * HD;
    float ob = 0.f, lb = 0.f;
    for (int cc = 0; cc < ncb; ++cc) {
      float o = opart[4 * cc][g][d];
#pragma unroll
      for (int w = 1; w < 4; ++w) o += opart[4 * cc + w][g][d];
      ob = cc == 0 ? o : ob + o;
      lb = cc == 0 ? lch[0][g] : lb + lch[cc][g];
    }
    if (nb == 1)  // one block: finished here (acc = ob, l = lb, as merge4 leaves them)
      dst[e] = (bf16_t)f2bf(ob * (1.0f / lb));
    else
      st_xc(po + e, ob, a.xc_l2);
    if (nb > 1 && d == 0) {
      st_xc(plm + 2 * g, lb, a.xc_l2);
      st_xc(plm + 2 * g + 1, mj[g], a.xc_l2);
    }
  }
  ZMI_ASTAMP(6);
  if (nb == 1) {
    ZMI_ASTAMP(7);
    return;
  }
  if (!zmi_last_arriver_wt(a.tickets + unit, (unsigned)nb, &last_flag)) {
    ZMI_ASTAMP(7);
    return;
  }
  for (int e = t; e < nb * G; e += BNT) st_xc64(gu + e, 0ull, a.xc_l2);  // re-arm (every block has read its maxima)
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // ---- fold the blocks (the reference recursion, as merge4 does after its per-block sums) ----
  const float* ou = a.part_o + (size_t)unit * a.nch * G * HD;
  const float* lu = a.part_lm + (size_t)unit * a.nch * G * 2;
  for (int e = t; e < G * HD; e += BNT) {
    const int g = e / HD, d = e - g * HD;
    float acc = 0.f, l = 0.f, mprev = 0.f;
    for (int b = 0; b < nb; ++b) {
      const float ob = ou[(size_t)b * G * HD + e];
      const float2 lm = ld2(lu + (size_t)b * G * 2 + 2 * g);
      if (b == 0) {
        acc = ob;
        l = lm.x;
      } else {
        const float et = expf(mprev - lm.y);
        l = lm.x + et * l;
        acc = acc * et + ob;
      }
      mprev = lm.y;
    }
    dst[e] = (bf16_t)f2bf(acc * (1.0f / l));
  }
  ZMI_ASTAMP(7);
}

// third launch of variant 3: one 64-thread workgroup per (unit, query head), 2 dims per thread, the unit's chunk
// partials (left by attn_kernel<G, 3>) merged as the last-arriving chunk merges in MODE 0 / 2
template <int G>
__global__ __launch_bounds__(64) void attn_merge_kernel(const AttnArgs a) {
  const int unit = blockIdx.x / G, g = blockIdx.x - unit * G;
  const int qi = unit / a.hkv, kh = unit - qi * a.hkv;
  const int nc = chunks_of(a.pos[qi]);
  if (nc <= 1) return;  // finished by its only chunk
  const float* ou = a.part_o + (size_t)unit * a.nch * G * HD;
  const float* lu = a.part_lm + (size_t)unit * a.nch * G * 2;
  const int d = threadIdx.x * 2;
  const float2 r = merge2<16>(ou, lu, nc, g, d, G);
  *reinterpret_cast<uint32_t*>(a.out + (size_t)qi * a.ldo + (kh * G + g) * HD + d) = f2bf(r.x) | (f2bf(r.y) << 16);
}

template <int G, int DS>
__global__ __launch_bounds__(DNW * 64) void attn_ds_kernel(const AttnArgs a, int n_units) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  ds_body<G, DS>(a, n_units, blockIdx.x, smem);
}

struct WorkLayout {
  size_t tickets, gran, stamps, total;
};
WorkLayout work_layout(int n_query, int g, int hkv, int max_pos) {
  const size_t units = (size_t)n_query * hkv, nch = (size_t)max_pos / CH + 1;
  WorkLayout w;
  w.tickets = 256;
  w.gran = w.tickets + ((units * 4 + 255) / 256) * 256;
  w.stamps = w.gran + ((units * nch * g * 8 + 255) / 256) * 256;
  w.total = w.stamps;
#ifdef ZMI_ATTN_STAMPS
  w.total += units * nch * 8 * 8;
#endif
  return w;
}

}  // namespace

extern "C" int64_t zmi_attention_work_bytes(int n_query, int hq, int hkv, int hd, int max_pos) {
  if (hd != HD || hkv <= 0 || hq % hkv || n_query <= 0 || max_pos < 0) return -1;
  return (int64_t)work_layout(n_query, hq / hkv, hkv, max_pos).total;
}

extern "C" int64_t zmi_attention_partial_floats(int n_query, int hq, int hkv, int hd, int max_pos) {
  if (hd != HD || hkv <= 0 || hq % hkv || n_query <= 0 || max_pos < 0) return -1;
  return (int64_t)n_query * hkv * (max_pos / CH + 1) * (hq / hkv) * HD;
}

extern "C" int zmi_attention_chunk(void) { return CH; }

namespace {
template <int G>
hipError_t launch_ds(const AttnArgs& a, int n_units, int ds, hipStream_t s) {
  const unsigned blocks = (unsigned)((n_units + 7) / 8) * 8 * ds;
  switch (ds) {
    case 4:
      hipLaunchKernelGGL((attn_ds_kernel<G, 4>), dim3(blocks), dim3(DNW * 64), (DsImg<G, 4>::BYTES), s, a, n_units);
      break;
    case 8:
      hipLaunchKernelGGL((attn_ds_kernel<G, 8>), dim3(blocks), dim3(DNW * 64), (DsImg<G, 8>::BYTES), s, a, n_units);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// chunked attention: one launch (MODE 0) or the scores / finish pair (MODE 1, 2)
template <int G>
hipError_t launch_chunked(const AttnArgs& a, unsigned blocks, int variant, hipStream_t s) {
  if (variant == 1) {
    hipLaunchKernelGGL((attn_kernel<G, 0>), dim3(blocks + a.n_pf), dim3(NT), 0, s, a);
  } else if (variant == 2) {
    hipLaunchKernelGGL((attn_kernel<G, 1>), dim3(blocks), dim3(NT), 0, s, a);
    hipLaunchKernelGGL((attn_kernel<G, 2>), dim3(blocks), dim3(NT), 0, s, a);
  } else if (variant == 3) {
    hipLaunchKernelGGL((attn_kernel<G, 1>), dim3(blocks), dim3(NT), 0, s, a);
    hipLaunchKernelGGL((attn_kernel<G, 3>), dim3(blocks), dim3(NT), 0, s, a);
    hipLaunchKernelGGL((attn_merge_kernel<G>), dim3(blocks / a.nch * G), dim3(64), 0, s, a);
  } else {  // 5: block form, one workgroup per (query, kv head, 512-key block) + the prefetch workgroups
    hipLaunchKernelGGL((attn_blk_kernel<G>), dim3((unsigned)a.n_att + a.n_pf), dim3(BNT), 0, s, a);
  }
  return hipGetLastError();
}
}  // namespace

extern "C" int zmi_attention_max_keys_whole(void) { return DS_KEYS; }

// The kernel zmi_attention_pf launches for `variant` (0 = the library's choice, resolved here): the launcher
// calls this too, so a caller (tests/test_gpu_scale.py) can assert which form a decode step's plan takes.
extern "C" int zmi_attention_pick(int n_query, int hkv, int variant) {
  if (variant != 0) return variant;
  return (int64_t)n_query * hkv >= 32 ? 5 : 1;
}

extern "C" int zmi_attention(const void* q, int ldq, const void* k_cache, const void* v_cache, const int* q_kv_row,
                             const int* q_pos, int n_query, int hq, int hkv, int hd, int smax, int max_pos, void* out,
                             int ldo, float* part_o, float* part_lm, void* work, void* stream) {
  return zmi_attention_variant(q, ldq, k_cache, v_cache, q_kv_row, q_pos, n_query, hq, hkv, hd, smax, max_pos, out,
                               ldo, part_o, part_lm, work, 0, stream);
}

extern "C" int zmi_attention_variant(const void* q, int ldq, const void* k_cache, const void* v_cache,
                                     const int* q_kv_row, const int* q_pos, int n_query, int hq, int hkv, int hd,
                                     int smax, int max_pos, void* out, int ldo, float* part_o, float* part_lm,
                                     void* work, int variant, void* stream) {
  return zmi_attention_pf(q, ldq, k_cache, v_cache, q_kv_row, q_pos, n_query, hq, hkv, hd, smax, max_pos, out, ldo,
                          part_o, part_lm, work, variant, nullptr, stream);
}

extern "C" int zmi_attention_pf(const void* q, int ldq, const void* k_cache, const void* v_cache, const int* q_kv_row,
                                const int* q_pos, int n_query, int hq, int hkv, int hd, int smax, int max_pos, void* out,
                                int ldo, float* part_o, float* part_lm, void* work, int variant,
                                const ZmiPrefetch* prefetch, void* stream) {
  if (hd != HD) return zmi_fail_msg("attention: head_dim must be 128");
  if (max_pos >= smax) return zmi_fail_msg("attention: max_pos must be < smax");
  if (smax % 8) return zmi_fail_msg("attention: smax must be a multiple of 8");
  if (ldq % 8 || ldo % 4) return zmi_fail_msg("attention: ldq must be a multiple of 8, ldo of 4");
  if (n_query <= 0) return 0;
  if (!work || !part_o || !part_lm) return zmi_fail_msg("attention: work and partial buffers required");
  const int g = hkv > 0 ? hq / hkv : 0;
  if (g * hkv != hq) return zmi_fail_msg("attention: hq must be a multiple of hkv");
  const WorkLayout w = work_layout(n_query, g, hkv, max_pos);
  char* wb = (char*)work;
  AttnArgs a{};
  a.q = (const bf16_t*)q;
  a.ldq = ldq;
  a.k = (const bf16_t*)k_cache;
  a.v = (const bf16_t*)v_cache;
  a.kv_row = q_kv_row;
  a.pos = q_pos;
  a.hkv = hkv;
  a.smax = smax;
  a.nch = max_pos / CH + 1;
  a.scale = 1.0f / sqrtf((float)hd);
  a.out = (bf16_t*)out;
  a.ldo = ldo;
  a.err = (unsigned*)wb;
  a.tickets = (unsigned*)(wb + w.tickets);
  a.gran = (uint64_t*)(wb + w.gran);
  a.part_o = part_o;
  a.part_lm = part_lm;
  a.stamps = (unsigned long long*)(wb + w.stamps);
  a.pf = ZmiPrefetch{};
  a.n_pf = 0;
  if (prefetch) {
    if (zmi_prefetch_invalid(*prefetch)) return zmi_fail_msg("attention: bad prefetch ranges");
    a.pf = *prefetch;
    a.n_pf = (a.pf.bytes[0] > 0 || a.pf.bytes[1] > 0) ? a.pf.blocks : 0;
  }
  hipStream_t s = (hipStream_t)stream;
  // variant: 0 = library choice, 1 = chunked (any length, one launch), 2 = chunked as the scores / finish
  // launch pair, 3 = scores / partials / merge launches, 5 = one workgroup per 512-key block, 4 / 8 = whole-query kernel with that many dim slices (max_pos < DS_KEYS). All give identical
  // bits; the choice is speed only. As its
  // own launch the whole-query kernel is bound by one CU's ~40 GB/s of K reads (C2 decode: 8.3 /
  // 10.1 / 15.1 us at positions 300 / 591 / 1000 against 10.4 / 10.6 / 10.8 chunked), so the
  // library picks the chunked kernel; the whole-query form pays off where its K/V loads overlap
  // the QKV projection (zmi_attn_block).
  // The block form (5) needs enough (query, kv head) units to fill the chip with one workgroup per 512 keys.
  // 16 rows at the engine's launch shape (max_pos = the C5 KV capacity 5783) x 1000 / 1600 / 2600 / 5000 keys:
  // 17.5 / 19.9 / 30.3 / 44.8 us against 21.4 / 26.6 / 32.8 / 52.6 chunked; 8 rows x 3200 20.4 against 25.3;
  // 128 rows x 1000 equal; 2 rows x 3200 18.1 against 15.6 (profiles/r04_attn_block_form.jsonl).
  variant = zmi_attention_pick(n_query, hkv, variant);
  if (variant < 1 || (variant > 3 && variant != 5)) {
    a.stamps = nullptr;  // the diagnostic stamp area is laid out for the chunked grid
    if (max_pos >= DS_KEYS) return zmi_fail_msg("attention: the whole-query variant covers positions < 1280");
    if ((int64_t)n_query * hkv * variant > 0x7fffffff) return zmi_fail_msg("attention: grid too large");
    const int n_units = n_query * hkv;
    hipError_t e;
    switch (g) {
      case 1: e = launch_ds<1>(a, n_units, variant, s); break;
      case 2: e = launch_ds<2>(a, n_units, variant, s); break;
      case 4: e = launch_ds<4>(a, n_units, variant, s); break;
      default: return zmi_fail_msg("attention: unsupported GQA group (1, 2, 4)");
    }
    if (e == hipErrorInvalidValue) return zmi_fail_msg("attention: variant must be 0, 1, 2, 3, 4, 5 or 8");
    ZMI_CHECK(e);
    return 0;
  }
  const int64_t blocks = (int64_t)n_query * hkv * a.nch;
  if (blocks + a.n_pf > 0x7fffffff) return zmi_fail_msg("attention: grid too large");
  a.n_att = variant == 5 ? (int)((int64_t)n_query * hkv * ((a.nch + CPB - 1) / CPB)) : (int)blocks;
  // the block form's blocks of one unit are n_units apart in the grid: on one XCD when n_units is a multiple of 8, so
  // their maxima and partials can stay in that XCD's L2 (ZMI_OPT_XC_HANDOFF 0)
  a.xc_l2 = variant == 5 && (n_query * hkv) % 8 == 0 && zmi_option(ZMI_OPT_XC_HANDOFF) == 0 ? 1 : 0;
  if (variant != 1 && variant != 5) a.n_pf = 0;  // the split-launch forms take no prefetch role
  hipError_t e;
  switch (g) {
    case 1: e = launch_chunked<1>(a, (unsigned)blocks, variant, s); break;
    case 2: e = launch_chunked<2>(a, (unsigned)blocks, variant, s); break;
    case 4: e = launch_chunked<4>(a, (unsigned)blocks, variant, s); break;
    default: return zmi_fail_msg("attention: unsupported GQA group (1, 2, 4)");
  }
  ZMI_CHECK(e);
  return 0;
}
