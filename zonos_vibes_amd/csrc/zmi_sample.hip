// Per-step token selection and frame bookkeeping for every active utterance slot, gfx950.
//
// One workgroup per (codebook, slot) computes, over the 1026-entry vocabulary:
//   CFG            u + (c - u) * cfg, column 1025 = -inf          reference model.py:112-115
//   EOS bias       -inf on EOS for codebooks 1..8 (decode only)    model.py:266-267,280
//   rep. penalty   penalty^count over generated[..., -window:]   sampling.py:99-114,164-165 (any window)
//   greedy         argmax, first index on ties                      sampling.py:180
//   stochastic     softmax(l/T) -> [unified] -> [top-p] -> [top-k] -> [min-p] -> argmax(p/q),
//                  q ~ Exp(1) from a counter-based hash (or a caller noise buffer)  sampling.py:4-96,167-178
// The last of the 9 codebook workgroups of a slot (in-launch ticket) then runs the EOS state
// machine and the delay-pattern frame write with the reference's masked_scatter_ compaction
// (model.py:283-299): the k-th still-unknown (-1) slot of the frame gets the k-th token.
#include "zmi_common.h"
#include "zmi_kernels.h"

namespace {

constexpr int NV = ZMI_VOCAB;   // 1026
constexpr int PER = 5;          // ceil(1026 / 256)
constexpr int SORTN = 2048;

struct SampleArgs {
  ZmiSlots sl;
  const float* logits;
  const float* noise;
  int* next;
  unsigned* counters;
  int mode;
  int slot_begin;
  const bf16_t* emb;  // optional fused embedding of the next input frame
  int d;
  bf16_t* x;
  int* row_kv;
  int* row_pos;
  // standalone sample_from_logits (mode 2): logits [B][9][NV] as given (no CFG), generated tokens
  // [B][9][gen_len] int32 (or NULL), one shared parameter block; tokens to next [B][9] only
  const int* gen;
  int gen_len;
  const ZmiSampling* params1;
};

__device__ void embed_row(const int* toks, const bf16_t* emb, int d, bf16_t* out0, bf16_t* out1);

__device__ float block_reduce_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  return ((red[0] + red[1]) + red[2]) + red[3];
}
__device__ float block_reduce_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}
// argmax with first-index tie break
__device__ int block_argmax(float v, int idx, float* redv, int* redi) {
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    if (ov > v || (ov == v && oi < idx)) {
      v = ov;
      idx = oi;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) {
    redv[w] = v;
    redi[w] = idx;
  }
  __syncthreads();
  float bv = redv[0];
  int bi = redi[0];
  for (int i = 1; i < 4; ++i)
    if (redv[i] > bv || (redv[i] == bv && redi[i] < bi)) {
      bv = redv[i];
      bi = redi[i];
    }
  return bi;
}

// the keys are distinct (the index is in the low word), so any correct sort gives the same array; each thread
// owns SORTN / 512 compare-exchange pairs per stage (pair p: i = p with a zero bit inserted at j, partner i + j).
// Requires exactly 256 threads (pair p = threadIdx.x + 256 q) and 64-lane waves (one wave's 64 consecutive pairs
// cover one 128-key block: the barrier-free stages below rely on it); the launchers use 256-thread workgroups.
constexpr int SORT_THREADS = 256;
static_assert(SORTN % (2 * SORT_THREADS) == 0, "whole compare-exchange pairs per thread");
__device__ void bitonic_desc(uint64_t* keys) {
#if defined(__AMDGCN_WAVEFRONT_SIZE) && __AMDGCN_WAVEFRONT_SIZE != 64
#error "bitonic_desc's barrier-free stages assume 64-lane waves"
#endif
  for (int k = 2; k <= SORTN; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      constexpr int NQ = SORTN / (2 * SORT_THREADS);
      int ii[NQ];
      uint64_t xv[NQ], yv[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {  // every pair's two keys in flight before the first compare
        const int p = threadIdx.x + SORT_THREADS * q;
        ii[q] = ((p & ~(j - 1)) << 1) | (p & (j - 1));
        xv[q] = keys[ii[q]];
        yv[q] = keys[ii[q] + j];
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const bool first_desc = (ii[q] & k) == 0;
        if (first_desc ? (xv[q] < yv[q]) : (xv[q] > yv[q])) {
          keys[ii[q]] = yv[q];
          keys[ii[q] + j] = xv[q];
        }
      }
      // stages with j <= 64 touch only the wave's own 128-key blocks (pairs p of one wave span 64 consecutive
      // p per q): between two such stages the wave's own LDS order suffices (a wave's LDS operations complete
      // in order), every other edge is a workgroup barrier
      const int jn = j > 1 ? j >> 1 : k;  // the next stage's distance (k doubles after j = 1)
      if (j <= 64 && jn <= 64 && !(j == 1 && k == SORTN))
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else
        __syncthreads();
    }
}

// Sort probs descending (ties: lower index first) into keys; returns nothing.
__device__ void sort_probs(const float* probs, uint64_t* keys) {
  for (int i = threadIdx.x; i < SORTN; i += 256) {
    const float p = i < NV ? probs[i] : 0.f;
    keys[i] = ((uint64_t)__float_as_uint(p) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)i);
  }
  __syncthreads();
  bitonic_desc(keys);
}

__device__ __forceinline__ float key_prob(uint64_t k) { return __uint_as_float((uint32_t)(k >> 32)); }
__device__ __forceinline__ int key_index(uint64_t k) { return (int)(0xFFFFFFFFu - (uint32_t)k); }

__device__ void renormalize(float* probs, float* red) {
  float s = 0.f;
  for (int v = threadIdx.x; v < NV; v += 256) s += probs[v];
  s = block_reduce_sum(s, red);
  __syncthreads();
  for (int v = threadIdx.x; v < NV; v += 256) probs[v] = probs[v] / s;
  __syncthreads();
}

__device__ void softmax_inplace(float* x, float* red) {
  float m = -INFINITY;
  for (int v = threadIdx.x; v < NV; v += 256) m = fmaxf(m, x[v]);
  m = block_reduce_max(m, red);
  float s = 0.f;
  for (int v = threadIdx.x; v < NV; v += 256) {
    const float e = expf(x[v] - m);
    x[v] = e;
    s += e;
  }
  s = block_reduce_sum(s, red);
  __syncthreads();
  for (int v = threadIdx.x; v < NV; v += 256) x[v] = x[v] / s;
  __syncthreads();
}

__global__ __launch_bounds__(SORT_THREADS) void sample_kernel(const SampleArgs a) {
  __shared__ float probs[NV + 2];
  __shared__ int cnt[NV];
  __shared__ uint64_t keys[SORTN];
  __shared__ double dscan[256];
  __shared__ float red[4];
  __shared__ float redv[4];
  __shared__ int redi[4];
  __shared__ unsigned last_flag;

  const int cb = blockIdx.x, t = threadIdx.x;
  const bool alone = a.mode == 2;
  const int s = alone ? blockIdx.y : a.slot_begin + blockIdx.y;
  if (!alone && !a.sl.active[s]) return;
  const ZmiSampling P = alone ? *a.params1 : a.sl.params[s];
  const int lrow = alone ? blockIdx.y : 2 * blockIdx.y;
  const float* lc = a.logits + ((size_t)lrow * ZMI_NCB + cb) * NV;
  const float* lu = alone ? lc : a.logits + ((size_t)(lrow + 1) * ZMI_NCB + cb) * NV;
  const bool decode = a.mode == 0;
  const int* dl = alone ? a.gen + ((size_t)s * ZMI_NCB + cb) * a.gen_len
                        : a.sl.delayed + ((size_t)s * ZMI_NCB + cb) * a.sl.tcap;
  const int o = alone ? a.gen_len : a.sl.offset[s] + 1;  // frames before the one sampled now

  // ---- CFG, padding, EOS bias, repetition penalty ----
  // window = generated_tokens[..., -window:] over the delayed frames 0 .. o-1 (Python slice
  // semantics: window <= 0 gives [-window:], i.e. the whole history for 0); counts per token in LDS
  const bool pen = (decode || (alone && a.gen)) && P.rep_penalty != 1.0f;
  if (pen) {
    const int win_lo = P.rep_window > 0 ? max(0, o - P.rep_window) : min(o, -P.rep_window);
    for (int v = t; v < NV; v += 256) cnt[v] = 0;
    __syncthreads();
    for (int i = win_lo + t; i < o; i += 256) atomicAdd(&cnt[min(dl[i], NV - 1)], 1);
    __syncthreads();
  }
  float cv[PER], uv[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {  // all logit loads in flight together (clamped index)
    const int v = min(t + i * 256, NV - 1);
    cv[i] = lc[v];
    uv[i] = lu[v];
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int v = t + i * 256;
    if (v >= NV) break;
    const float c = cv[i], u = uv[i];
    float l = alone ? c : u + (c - u) * P.cfg_scale;
    if (v >= 1025) l = -INFINITY;
    if (decode) l = l + ((cb >= 1 && v == ZMI_EOS) ? -INFINITY : 0.0f);
    if (pen) {  // factor = penalty^count as the reference's scatter_reduce(prod) builds it
      float f = 1.0f;
      for (int k = cnt[v]; k > 0; --k) f = f * P.rep_penalty;
      l = (l <= 0.f) ? l * f : l / f;
    }
    probs[v] = l;
  }
  __syncthreads();

  int tok;
  if (P.temperature <= 0.f) {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int v = t; v < NV; v += 256)
      if (probs[v] > bv || bi == 0x7fffffff) {
        bv = probs[v];
        bi = v;
      }
    tok = block_argmax(bv, bi, redv, redi);
  } else {
    for (int v = t; v < NV; v += 256) probs[v] = probs[v] / P.temperature;
    __syncthreads();
    softmax_inplace(probs, red);
    if (P.linear > 0.f) {  // unified sampler (sampling.py:29-43)
      float ent = 0.f;
      for (int v = t; v < NV; v += 256) {
        const float lp = logf(fmaxf(probs[v], 1e-20f));
        ent += probs[v] * lp;
      }
      ent = -block_reduce_sum(ent, red);
      __syncthreads();
      for (int v = t; v < NV; v += 256) {
        const float lp = logf(fmaxf(probs[v], 1e-20f));
        probs[v] = lp * (P.linear + ent * P.conf) - (lp * lp) * P.quad;
      }
      __syncthreads();
      softmax_inplace(probs, red);
    }
    if (P.top_p > 0.f) {  // sampling.py:64-79: keep sorted i unless cumsum_i - p_i > top_p
      sort_probs(probs, keys);
      double run = 0.0;
      double loc[SORTN / 256];
      for (int j = 0; j < SORTN / 256; ++j) {
        run += (double)key_prob(keys[t * (SORTN / 256) + j]);
        loc[j] = run;
      }
      dscan[t] = run;
      __syncthreads();
      if (t == 0) {  // exclusive scan of the 256 thread totals, in order (loads batched ahead of the add chain)
        double acc = 0.0;
        for (int i0 = 0; i0 < 256; i0 += 16) {
          double x[16];
#pragma unroll
          for (int i = 0; i < 16; ++i) x[i] = dscan[i0 + i];
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            dscan[i0 + i] = acc;
            acc += x[i];
          }
        }
      }
      __syncthreads();
      for (int j = 0; j < SORTN / 256; ++j) {
        const int i = t * (SORTN / 256) + j;
        if (i >= NV) break;
        const uint64_t k = keys[i];
        const float p = key_prob(k);
        const float csum = (float)(dscan[t] + loc[j]);
        if (csum - p > P.top_p) probs[key_index(k)] = 0.f;
      }
      __syncthreads();
      renormalize(probs, red);
    }
    if (P.top_k > 0) {  // sampling.py:45-61
      sort_probs(probs, keys);
      const int kk = min(P.top_k, NV);
      const float pivot = key_prob(keys[kk - 1]);
      for (int v = t; v < NV; v += 256)
        if (probs[v] < pivot) probs[v] = 0.f;
      __syncthreads();
      renormalize(probs, red);
    }
    if (P.min_p > 0.f) {  // sampling.py:82-96
      float m = 0.f;
      for (int v = t; v < NV; v += 256) m = fmaxf(m, probs[v]);
      m = block_reduce_max(m, red);
      const float thr = P.min_p * m;
      __syncthreads();
      for (int v = t; v < NV; v += 256)
        if (probs[v] < thr) probs[v] = 0.f;
      __syncthreads();
      renormalize(probs, red);
    }
    // exponential race: argmax(p / q), q ~ Exp(1)  (sampling.py:19-21)
    const uint64_t ctr_base = ((uint64_t)(decode ? a.sl.step[s] + 1 : 0) * ZMI_NCB + cb) * NV +
                              (alone ? (uint64_t)s * ZMI_NCB * NV : 0);
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int v = t; v < NV; v += 256) {
      float q;
      if (a.noise) {
        q = a.noise[((size_t)blockIdx.y * ZMI_NCB + cb) * NV + v];
      } else {
        const uint64_t z = mix64(P.seed + 0x9E3779B97F4A7C15ull * (ctr_base + v + 1));
        const float u = ((float)(z >> 40) + 0.5f) * (1.0f / 16777216.0f);
        q = -logf(u);
      }
      const float r = probs[v] / q;
      if (r > bv || bi == 0x7fffffff) {
        bv = r;
        bi = v;
      }
    }
    tok = block_argmax(bv, bi, redv, redi);
  }

  if (alone) {
    if (t == 0) a.next[(size_t)s * ZMI_NCB + cb] = tok;
    return;
  }
  if (t == 0) st_wt(a.next + (size_t)s * ZMI_NCB + cb, tok);
  if (!zmi_last_arriver_wt(a.counters + s, ZMI_NCB, &last_flag)) return;

  // ---- EOS state machine + frame compaction write (thread 0 of the slot's last block) ----
  __shared__ int frame[ZMI_NCB + 2];
  if (t == 0) {
    int nt[ZMI_NCB];
    for (int k = 0; k < ZMI_NCB; ++k) nt[k] = ld_wt(a.next + (size_t)s * ZMI_NCB + k);
    int rem = a.sl.remaining[s];
    int stop = a.sl.stopping[s];
    if (decode) {
      if (nt[0] == ZMI_EOS) {
        rem = min(rem, 9);
        stop = 1;
      }
      if (stop) {
        const int idx = min(9 - rem, 8);
        for (int k = 0; k < idx; ++k) nt[k] = ZMI_MASK;
        nt[idx] = ZMI_EOS;
      }
    }
    const bool in_range = o < a.sl.total_len[s];
    const int oc = min(o, a.sl.tcap - 1);
    int cells[ZMI_NCB];
#pragma unroll
    for (int k = 0; k < ZMI_NCB; ++k) cells[k] = a.sl.delayed[((size_t)s * ZMI_NCB + k) * a.sl.tcap + oc];
    int kk = 0;
#pragma unroll
    for (int k = 0; k < ZMI_NCB; ++k) {
      int v = in_range ? cells[k] : ZMI_MASK;
      if (in_range && v == -1) {
        v = nt[kk++];
        a.sl.delayed[((size_t)s * ZMI_NCB + k) * a.sl.tcap + o] = v;
      }
      frame[k] = v < 0 ? 0 : (v > ZMI_MASK ? ZMI_MASK : v);  // next step's input frame
    }
    a.sl.offset[s] = o;
    int pos = a.sl.pos[s], act = 1;
    if (decode) {
      pos += 1;
      a.sl.pos[s] = pos;
      rem -= 1;
      a.sl.remaining[s] = rem;
      a.sl.stopping[s] = stop;
      a.sl.step[s] += 1;
      if (rem <= 0) {
        a.sl.active[s] = 0;
        act = 0;
      }
    }
    frame[ZMI_NCB] = act;
    if (a.row_pos) {  // (kv row, position) of the next step's CFG pair
      a.row_kv[2 * s] = 2 * s;
      a.row_kv[2 * s + 1] = 2 * s + 1;
      a.row_pos[2 * s] = act ? pos : -1;
      a.row_pos[2 * s + 1] = act ? pos : -1;
    }
  }
  // ---- next step's input embedding: x[2s] = x[2s+1] = sum_k emb_k[frame_k]  (model.py:97-98,142)
  if (a.emb) {
    __syncthreads();
    if (frame[ZMI_NCB])
      embed_row(frame, a.emb, a.d, a.x + (size_t)(2 * s) * a.d, a.x + (size_t)(2 * s + 1) * a.d);
  }
}

// Greedy decode step (the caller guarantees every slot of the launch samples with temperature <= 0): one
// workgroup of 9 waves per slot, wave k = codebook k. sample_kernel's greedy path value for value (CFG,
// padding, EOS bias, penalty^count, argmax with the first index on ties), then the same EOS state machine,
// frame write and next-step embedding. Every load that does not depend on another (logits, slot state, the
// penalty window, the frame cells) is issued at launch start, and there is no in-launch ticket between
// codebook workgroups: the step's sampler is ~3 dependent memory round trips instead of ~7.
__global__ __launch_bounds__(64 * ZMI_NCB) void sample_greedy_kernel(const SampleArgs a) {
  __shared__ int cnt[ZMI_NCB][NV];
  __shared__ int tokv[ZMI_NCB];
  __shared__ int cellv[ZMI_NCB];
  __shared__ int frame[ZMI_NCB + 2];
  constexpr int NP = NV / 2;              // 513 value pairs per codebook row
  constexpr int PP = (NP + 63) / 64;      // pairs per lane
  const int s = a.slot_begin + blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, k = t >> 6;
  // no exit before the argmax: a branch on `active` up here would let the compiler sink every load below
  // behind that round trip (sampler 8.25 -> 8.09 us, profiles/r04_sampler_hoist_ab.jsonl). An inactive slot's
  // state is valid (its last utterance's), the penalty indices are clamped, and it leaves before any write.
  const int act0 = a.sl.active[s];
  const int lrow = 2 * blockIdx.x;
  const float2* lc = reinterpret_cast<const float2*>(a.logits + ((size_t)lrow * ZMI_NCB + k) * NV);
  const float2* lu = reinterpret_cast<const float2*>(a.logits + ((size_t)(lrow + 1) * ZMI_NCB + k) * NV);
  float2 cv[PP], uv[PP];
#pragma unroll
  for (int i = 0; i < PP; ++i) {  // all logit loads in flight together (clamped index)
    const int p = min(lane + 64 * i, NP - 1);
    cv[i] = lc[p];
    uv[i] = lu[p];
  }
  const ZmiSampling P = a.sl.params[s];
  const int o = a.sl.offset[s] + 1;  // frames before the one sampled now
  const int rem0 = a.sl.remaining[s], stop0 = a.sl.stopping[s], pos0 = a.sl.pos[s], tl = a.sl.total_len[s];
  const int step0 = a.sl.step[s];
  const int* dl = a.sl.delayed + ((size_t)s * ZMI_NCB + k) * a.sl.tcap;
  if (lane == 0) cellv[k] = dl[min(o, a.sl.tcap - 1)];
  const bool pen = P.rep_penalty != 1.0f;
  if (pen) {  // penalty counts over generated[..., -window:] (sampling.py:99-114), one LDS row per codebook
    const int win_lo = P.rep_window > 0 ? max(0, o - P.rep_window) : min(o, -P.rep_window);
    for (int v = lane; v < NV; v += 64) cnt[k][v] = 0;
    __syncthreads();
    for (int i = win_lo + lane; i < min(o, a.sl.tcap); i += 64) atomicAdd(&cnt[k][min(max(dl[i], 0), NV - 1)], 1);
    __syncthreads();
  }
  float bv = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int i = 0; i < PP; ++i) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int v = 2 * (lane + 64 * i) + h;
      if (v >= NV) break;
      const float c = h ? cv[i].y : cv[i].x, u = h ? uv[i].y : uv[i].x;
      float l = u + (c - u) * P.cfg_scale;
      if (v >= 1025) l = -INFINITY;
      l = l + ((k >= 1 && v == ZMI_EOS) ? -INFINITY : 0.0f);
      if (pen) {
        float f = 1.0f;
        for (int kk = cnt[k][v]; kk > 0; --kk) f = f * P.rep_penalty;
        l = (l <= 0.f) ? l * f : l / f;
      }
      if (l > bv || bi == 0x7fffffff) {
        bv = l;
        bi = v;
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {  // first index on ties
    const float ov = __shfl_xor(bv, off, 64);
    const int oi = __shfl_xor(bi, off, 64);
    if (ov > bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  }
  if (!act0) return;  // slot-uniform; nothing written before it
  if (lane == 0) {
    tokv[k] = bi;
    a.next[(size_t)s * ZMI_NCB + k] = bi;
  }
  __syncthreads();
  // ---- EOS state machine + frame compaction write (model.py:266-307), as sample_kernel's last block ----
  if (t == 0) {
    int nt[ZMI_NCB];
#pragma unroll
    for (int kk = 0; kk < ZMI_NCB; ++kk) nt[kk] = tokv[kk];
    int rem = rem0, stop = stop0;
    if (nt[0] == ZMI_EOS) {
      rem = min(rem, 9);
      stop = 1;
    }
    if (stop) {
      const int idx = min(9 - rem, 8);
      for (int kk = 0; kk < idx; ++kk) nt[kk] = ZMI_MASK;
      nt[idx] = ZMI_EOS;
    }
    const bool in_range = o < tl;
    int kn = 0;
#pragma unroll
    for (int kk = 0; kk < ZMI_NCB; ++kk) {
      int v = in_range ? cellv[kk] : ZMI_MASK;
      if (in_range && v == -1) {
        v = nt[kn++];
        a.sl.delayed[((size_t)s * ZMI_NCB + kk) * a.sl.tcap + o] = v;
      }
      frame[kk] = v < 0 ? 0 : (v > ZMI_MASK ? ZMI_MASK : v);  // next step's input frame
    }
    a.sl.offset[s] = o;
    const int pos = pos0 + 1;
    a.sl.pos[s] = pos;
    rem -= 1;
    a.sl.remaining[s] = rem;
    a.sl.stopping[s] = stop;
    a.sl.step[s] = step0 + 1;
    const int act = rem > 0;
    if (!act) a.sl.active[s] = 0;
    frame[ZMI_NCB] = act;
    if (a.row_pos) {  // (kv row, position) of the next step's CFG pair
      a.row_kv[2 * s] = 2 * s;
      a.row_kv[2 * s + 1] = 2 * s + 1;
      a.row_pos[2 * s] = act ? pos : -1;
      a.row_pos[2 * s + 1] = act ? pos : -1;
    }
  }
  // ---- next step's input embedding: x[2s] = x[2s+1] = sum_k emb_k[frame_k]  (model.py:97-98,142)
  if (a.emb) {
    __syncthreads();
    if (frame[ZMI_NCB] && t < 256)
      embed_row(frame, a.emb, a.d, a.x + (size_t)(2 * s) * a.d, a.x + (size_t)(2 * s + 1) * a.d);
  }
}

// ---- embeddings (model.py:97-98): sum over codebooks 0..8, bf16 rounding after each add ----
__device__ void embed_row(const int* toks, const bf16_t* emb, int d, bf16_t* out0, bf16_t* out1) {
  for (int c = threadIdx.x * 8; c < d; c += 256 * 8) {
    float acc[8];
#pragma unroll
    for (int k = 0; k < ZMI_NCB; ++k) {
      const uint4 e = *reinterpret_cast<const uint4*>(emb + ((size_t)k * ZMI_VOCAB + toks[k]) * d + c);
      const uint32_t u[4] = {e.x, e.y, e.z, e.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float lo = bf2f(u[j]), hi = bf2f(u[j] >> 16);
        if (k == 0) {
          acc[2 * j] = lo;
          acc[2 * j + 1] = hi;
        } else {
          acc[2 * j] = bfround(acc[2 * j] + lo);
          acc[2 * j + 1] = bfround(acc[2 * j + 1] + hi);
        }
      }
    }
    uint4 r;
    r.x = f2bf(acc[0]) | (f2bf(acc[1]) << 16);
    r.y = f2bf(acc[2]) | (f2bf(acc[3]) << 16);
    r.z = f2bf(acc[4]) | (f2bf(acc[5]) << 16);
    r.w = f2bf(acc[6]) | (f2bf(acc[7]) << 16);
    *reinterpret_cast<uint4*>(out0 + c) = r;
    if (out1) *reinterpret_cast<uint4*>(out1 + c) = r;
  }
}

__global__ __launch_bounds__(256) void embed_step_kernel(const ZmiSlots sl, const bf16_t* emb, int d, bf16_t* x,
                                                          int* row_kv, int* row_pos) {
  const int s = blockIdx.x;
  const int act = sl.active[s];
  if (threadIdx.x < 2) {
    row_kv[2 * s + threadIdx.x] = 2 * s + threadIdx.x;
    row_pos[2 * s + threadIdx.x] = act ? sl.pos[s] : -1;
  }
  if (!act) return;
  int toks[ZMI_NCB];
  const int off = sl.offset[s];
  for (int k = 0; k < ZMI_NCB; ++k) {
    int tk = sl.delayed[((size_t)s * ZMI_NCB + k) * sl.tcap + off];
    toks[k] = tk < 0 ? 0 : (tk > ZMI_MASK ? ZMI_MASK : tk);
  }
  embed_row(toks, emb, d, x + (size_t)(2 * s) * d, x + (size_t)(2 * s + 1) * d);
}

__global__ __launch_bounds__(256) void embed_codes_kernel(const int* codes, int ld, const bf16_t* emb, int d,
                                                           bf16_t* x, int ldx) {
  const int r = blockIdx.x;
  int toks[ZMI_NCB];
  for (int k = 0; k < ZMI_NCB; ++k) {
    int tk = codes[(size_t)k * ld + r];
    toks[k] = tk < 0 ? 0 : (tk > ZMI_MASK ? ZMI_MASK : tk);
  }
  embed_row(toks, emb, d, x + (size_t)r * ldx, nullptr);
}

// ---- delay pattern (codebook_pattern.py:5-12) ----
__global__ void delay_init_kernel(const ZmiSlots sl, int slot, const int* prefix, int plen, int total) {
  const int t = blockIdx.x * 256 + threadIdx.x, k = blockIdx.y;
  if (t >= sl.tcap) return;
  const int n_audio = total - ZMI_NCB;  // P + N
  int v = ZMI_MASK;
  const int src = t - k - 1;
  if (t < total && src >= 0 && src < n_audio) v = src < plen ? prefix[(size_t)k * plen + src] : -1;
  sl.delayed[((size_t)slot * ZMI_NCB + k) * sl.tcap + t] = v;
}

__global__ void delay_revert_kernel(const ZmiSlots sl, int slot, int64_t* out, int t_out) {
  const int t = blockIdx.x * 256 + threadIdx.x, k = blockIdx.y;
  if (t >= t_out) return;
  const int v = sl.delayed[((size_t)slot * ZMI_NCB + k) * sl.tcap + t + k + 1];
  out[(size_t)k * t_out + t] = v >= 1024 ? 0 : v;
}

// standalone apply / revert over [B][9][T] int64 tensors (codebook_pattern.py:5-12)
__global__ void apply_delay_kernel(const int64_t* codes, int64_t* out, int T, int64_t mask) {
  const int t = blockIdx.x * 256 + threadIdx.x, k = blockIdx.y, b = blockIdx.z;
  if (t >= T + ZMI_NCB) return;
  const int src = t - k - 1;  // roll by k + 1 of the mask-padded row
  out[((size_t)b * ZMI_NCB + k) * (T + ZMI_NCB) + t] =
      (src >= 0 && src < T) ? codes[((size_t)b * ZMI_NCB + k) * T + src] : mask;
}

__global__ void revert_delay_kernel(const int64_t* codes, int64_t* out, int T) {
  const int t = blockIdx.x * 256 + threadIdx.x, k = blockIdx.y, b = blockIdx.z;
  if (t >= T - ZMI_NCB) return;
  out[((size_t)b * ZMI_NCB + k) * (T - ZMI_NCB) + t] = codes[((size_t)b * ZMI_NCB + k) * T + t + k + 1];
}

}  // namespace

extern "C" int zmi_apply_delay_pattern(const int64_t* codes, int64_t* out, int batch, int T, int64_t mask_token,
                                       void* stream) {
  if (batch <= 0 || T < 0) return zmi_fail_msg("apply_delay_pattern: bad shape");
  hipLaunchKernelGGL(apply_delay_kernel, dim3((T + ZMI_NCB + 255) / 256, ZMI_NCB, batch), dim3(256), 0,
                     (hipStream_t)stream, codes, out, T, mask_token);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_revert_delay_pattern(const int64_t* codes, int64_t* out, int batch, int T, void* stream) {
  if (batch <= 0 || T < ZMI_NCB) return zmi_fail_msg("revert_delay_pattern: bad shape");
  if (T == ZMI_NCB) return 0;
  hipLaunchKernelGGL(revert_delay_kernel, dim3((T - ZMI_NCB + 255) / 256, ZMI_NCB, batch), dim3(256), 0,
                     (hipStream_t)stream, codes, out, T);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_sample_logits(const float* logits, const int* generated, int gen_len, int batch,
                                 const ZmiSampling* params, const float* noise, int* tokens, void* stream) {
  if (batch <= 0) return 0;
  if (!params || !tokens || !logits || (generated && gen_len <= 0)) return zmi_fail_msg("sample_logits: arguments");
  SampleArgs a = {};
  a.logits = logits;
  a.noise = noise;
  a.next = tokens;
  a.mode = 2;
  a.gen = generated;
  a.gen_len = generated ? gen_len : 0;
  a.params1 = params;
  hipLaunchKernelGGL(sample_kernel, dim3(ZMI_NCB, batch), dim3(SORT_THREADS), 0, (hipStream_t)stream, a);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_sample_step(const ZmiSlots* slots, const float* logits_rows, const float* noise, int* next_tokens,
                               unsigned* counters, int mode, int slot_begin, int slot_count, const void* emb, int d,
                               void* x, int* row_kv, int* row_pos, void* stream) {
  if (mode != 0 && mode != 1) return zmi_fail_msg("sample: mode must be 0 (decode) or 1 (prefill)");
  if (slot_begin < 0 || slot_begin + slot_count > slots->n_slots) return zmi_fail_msg("sample: slot range");
  if (emb && (d % 8 || !x)) return zmi_fail_msg("sample: fused embedding needs x and d % 8 == 0");
  if (!row_kv != !row_pos) return zmi_fail_msg("sample: row_kv and row_pos go together");
  SampleArgs a;
  a.sl = *slots;
  a.logits = logits_rows;
  a.noise = noise;
  a.next = next_tokens;
  a.counters = counters;
  a.mode = mode;
  a.slot_begin = slot_begin;
  a.emb = (const bf16_t*)emb;
  a.d = d;
  a.x = (bf16_t*)x;
  a.row_kv = row_kv;
  a.row_pos = row_pos;
  hipLaunchKernelGGL(sample_kernel, dim3(ZMI_NCB, slot_count), dim3(SORT_THREADS), 0, (hipStream_t)stream, a);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_sample_step_greedy(const ZmiSlots* slots, const float* logits_rows, int* next_tokens,
                                      int slot_begin, int slot_count, const void* emb, int d, void* x, int* row_kv,
                                      int* row_pos, void* stream) {
  if (slot_begin < 0 || slot_count < 0 || slot_begin + slot_count > slots->n_slots)
    return zmi_fail_msg("sample_greedy: slot range");
  if (emb && (d % 8 || !x)) return zmi_fail_msg("sample_greedy: fused embedding needs x and d % 8 == 0");
  if (!row_kv != !row_pos) return zmi_fail_msg("sample_greedy: row_kv and row_pos go together");
  if (slot_count == 0) return 0;
  SampleArgs a{};
  a.sl = *slots;
  a.logits = logits_rows;
  a.next = next_tokens;
  a.mode = 0;
  a.slot_begin = slot_begin;
  a.emb = (const bf16_t*)emb;
  a.d = d;
  a.x = (bf16_t*)x;
  a.row_kv = row_kv;
  a.row_pos = row_pos;
  hipLaunchKernelGGL(sample_greedy_kernel, dim3(slot_count), dim3(64 * ZMI_NCB), 0, (hipStream_t)stream, a);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_embed_step(const ZmiSlots* slots, const void* emb, int d, void* x, int* row_kv, int* row_pos,
                              void* stream) {
  if (d % 8) return zmi_fail_msg("embed: d % 8");
  hipLaunchKernelGGL(embed_step_kernel, dim3(slots->n_slots), dim3(256), 0, (hipStream_t)stream, *slots,
                     (const bf16_t*)emb, d, (bf16_t*)x, row_kv, row_pos);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_embed_codes(const int* codes, int ld_codes, int n, const void* emb, int d, void* x, int ldx,
                               void* stream) {
  if (d % 8 || n <= 0) return zmi_fail_msg("embed_codes: bad shape");
  hipLaunchKernelGGL(embed_codes_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, codes, ld_codes,
                     (const bf16_t*)emb, d, (bf16_t*)x, ldx);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_delay_init(const ZmiSlots* slots, int slot, const int* prefix, int prefix_len, int total_len,
                              void* stream) {
  if (total_len > slots->tcap || slot < 0 || slot >= slots->n_slots) return zmi_fail_msg("delay_init: bounds");
  hipLaunchKernelGGL(delay_init_kernel, dim3((slots->tcap + 255) / 256, ZMI_NCB), dim3(256), 0,
                     (hipStream_t)stream, *slots, slot, prefix, prefix_len, total_len);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_delay_revert(const ZmiSlots* slots, int slot, int64_t* out, int t_out, void* stream) {
  if (t_out <= 0) return 0;
  if (t_out + ZMI_NCB > slots->tcap) return zmi_fail_msg("delay_revert: bounds");
  hipLaunchKernelGGL(delay_revert_kernel, dim3((t_out + 255) / 256, ZMI_NCB), dim3(256), 0, (hipStream_t)stream,
                     *slots, slot, out, t_out);
  ZMI_CHECK(hipGetLastError());
  return 0;
}
