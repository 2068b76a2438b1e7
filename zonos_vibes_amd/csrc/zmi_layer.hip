// Persistent decode engine for one whole transformer block at batch 1 (the CFG cond / uncond row pair), ONE
// launch of 256 workgroups (one per CU) per layer instead of four (attention block, out_proj, fc1, fc2):
//   attention(L)   reference zonos/backbone/_torch.py:136 (q and the KV cache as the previous launch left them)
//   out_proj(L)    :140, + residual :100-101
//   norm2, fc1, SwiGLU, fc2(L)  :101, :147-152, + residual
//   then the NEXT op on the new residual rows: LayerNorm + QKV projection of layer L + 1 (:114-126: RoPE,
//   KV-cache write of position p, q for the next launch), or on the last layer norm_f + the 9 heads
//   (zonos/model.py:100-101: logits).
// Why (MI355X_MICROARCH.md rows launches-baseline, engine-vs-launches, prefetch-credit): every CU streams its
// slice of all the layer's weights (464 KB) through per-wave LDS rings of non-temporal LDS-DMA slots that
// run ahead of the data dependencies, so HBM keeps streaming while the attention chain and the hand-offs
// between the projections run; no kernel boundary sits inside the layer.
//
// Workgroup b (8 waves):
//   waves 0..3  consumers: wave c owns K segment c of every K = 2048 GEMV (the GEMV's W = 4 x NL = 8 split)
//               and streams its items through a private ring of DEPTH 8 KiB slots, counting its own DMAs
//               with vmcnt; fc2 items are (group, K segment of 1024) pairs, the GEMV's W = 8 split;
//   waves 4..7  service: the attention chunk, epilogues, {value, tag = position + 1} granule hand-offs
//               (cdna_hip_programming.md §6 Guideline 16 R2), gathers, LayerNorms.
// Work of block b (s = b & 7: its XCD under round-robin placement, m = b >> 3):
//   attention   unit u = b & 7 (row u >> 2, kv head u & 3), 128-key chunk m (positions < 32 x 128): the
//               chunked kernel's per-chunk arithmetic (zmi_attn.hip / zmi_attnblk.hip xc_body), chunk
//               maxima and partials exchanged as granules, and the merge of output dims 4 m .. 4 m + 3
//   out_proj    column group b                                      -> x' (every block gathers)
//   fc1         groups 256 s + 8 m + j, j < 8: h[1024 s + 32 m ..]  -> h (team s = blocks b' & 7 == s gathers)
//   fc2         groups 8 m + j, j < 8, K segment s                  -> fp32 segment sums
//   combine     group b: the 8 segment sums in order + residual     -> x'' (every block gathers)
//   next        QKV groups b and 256 + b (b < 128), or heads groups b + 256 i (< 1156)
// Every result is bit-identical to the launch plan it replaces (same per-(group, segment) MFMA chains,
// segment sums in order, LayerNorm / residual / SwiGLU / RoPE / logits arithmetic, attention operations).
#include <algorithm>

#include "zmi_common.h"
#include "zmi_kernels.h"
#include "zonos_diag.h"
#include "zmi_gemv_impl.h"
#include "zmi_attn_ds.h"
#include "zmi_engine.h"

namespace {

using namespace zmi_eng;
using zmi_attn::CH;
using zmi_attn::CPB;
using zmi_attn::HD;
using zmi_attn::mfma16;

constexpr int DM = 2048, FF = 8192, XG = 4, HKV = 4, QCOLS = 2048, KCOLS = 512;
constexpr int NBLK = 256, NLW = 2, NCW = 4, NSW = 4, NPW = 1, NWV = NLW + NCW + NSW + NPW, NT = NWV * 64;
constexpr int CPL = NCW / NLW;  // consumers per loader wave
constexpr int MAXFLY = 8;  // ring slots the loader may keep in flight (its vmcnt waits encode up to 8 x 7 pieces)
constexpr int MAXR = 2, DEPTH = 4;
constexpr int NCH = 32;                 // chunk blocks per attention unit: positions < NCH x CH = 4096
constexpr int NUNIT = 8;                // (row, kv head) units
constexpr int NMRG = 8;                 // chunk blocks 0..7 of a unit merge its output, 16 dims each
constexpr int MDIM = HD / NMRG;
constexpr int CPG = CH / 32;            // 32-key groups per chunk
constexpr int NEXT_QKV = 0, NEXT_HEADS = 1;
constexpr int HEADS_GROUPS = 9248 / 8, HEADS_VALID = 9 * 1026 - 0;  // 9 x 1026 columns (1025 real + pad row each)
constexpr int MAXNEXT = 5;
constexpr int NSLOT_MAX = 13 + MAXNEXT;
constexpr int XROW = DM + 8;
static_assert(NCH * NUNIT == NBLK && CPG == 4 && MDIM == 16, "geometry");

// granule areas (u64 words) of one layer for M rows
struct Gran {
  size_t gm, gl, gb, go, ga, gx, gh, gp, gy, total;
  __host__ __device__ explicit Gran(int M) {
    gm = 0;
    gl = gm + (size_t)NUNIT * NCH * XG;
    gb = gl + (size_t)NUNIT * NCH * XG;
    go = gb + (size_t)NUNIT * NCH * XG;
    ga = go + (size_t)NUNIT * NCH * XG * HD;
    gx = ga + (size_t)M * (DM / 2);
    gh = gx + (size_t)M * (DM / 2);
    gp = gh + (size_t)M * (FF / 2);
    gy = gp + (size_t)256 * 8 * M * 8;
    total = gy + (size_t)M * (DM / 2);
  }
};

// LDS
constexpr size_t L_RING = 0;                                             // [NCW][DEPTH][8 KiB]
constexpr size_t L_BUFA = L_RING + (size_t)NCW * DEPTH * SLOT;           // bf16 [MAXR][XROW]
constexpr size_t L_BUFB = L_BUFA + (size_t)MAXR * XROW * 2;              // bf16 [MAXR][XROW]
constexpr size_t L_REDO = L_BUFB + (size_t)MAXR * XROW * 2;              // f32 [NCW][8][MAXR]
constexpr size_t L_REDF = L_REDO + (size_t)NCW * 8 * MAXR * 4;           // f32 [8][NCW][8][MAXR]
constexpr size_t L_REDN = L_REDF + (size_t)8 * NCW * 8 * MAXR * 4;       // f32 [MAXNEXT][NCW][8][MAXR]
constexpr size_t L_CNT = L_REDN + (size_t)MAXNEXT * NCW * 8 * MAXR * 4;  // u32 [64]
constexpr size_t L_SINK = L_CNT + 64 * 4;                                  // 1 KiB landing area of the prefetch wave
constexpr size_t L_BYTES = L_SINK + 1024;
// the attention scratch lives in BUFA + BUFB (free until the attention output is gathered)
constexpr size_t A_SC = L_BUFA;                                          // f32 [XG][CH] scores
constexpr size_t A_PB = A_SC + (size_t)XG * CH * 4;                      // bf16 [XG][CH] P
constexpr size_t A_OP = A_PB + (size_t)XG * CH * 2;                      // f32 [CPG][XG][HD] per-group P.V
constexpr size_t A_MJ = A_OP + (size_t)CPG * XG * HD * 4;                // f32 [XG] M_j
static_assert(A_MJ + 16 <= L_REDO, "attention scratch");
static_assert(L_BYTES <= 160 * 1024, "LDS");
static_assert(L_BUFA % 16 == 0 && L_BUFB % 16 == 0 && L_CNT % 16 == 0, "alignment");
// C_F1 + j (j < 8), C_N + i (i < MAXNEXT); C_FULL / C_FREE + c DEPTH + ring slot: k + 1 once slot k of consumer c
// has landed / been read; C_THIN > 0 while a service wave polls (the loader then keeps few slots in flight)
// C_HOLD: nonzero while this block's attention chunk still loads its K / V (the loaders issue nothing then)
// C_PFGO / C_PFSTOP: the prefetch wave may start / must stop
enum { C_READY = 0, C_SVC = 1, C_O = 2, C_F1 = 3, C_N = 11, C_THIN = 16, C_FULL = 17, C_FREE = 33, C_HOLD = 49,
       C_PFGO = 50, C_PFSTOP = 51, C_WORDS = 52 };
static_assert(C_WORDS <= 64, "LDS words");

struct LArgs {
  const char* w_out;
  const char* w_fc1;
  const char* w_fc2;
  const char* w_next;
  const bf16_t* ln2_w;
  const bf16_t* ln2_b;
  const bf16_t* lnn_w;
  const bf16_t* lnn_b;
  float eps, scale;
  int M, smax;
  const int* row_pos;
  bf16_t* x;
  bf16_t* q;
  const bf16_t* kc;
  const bf16_t* vc;
  bf16_t* kn;
  bf16_t* vn;
  const float* rope;
  bf16_t* attn_out;
  float* logits;
  uint64_t* gran;
  unsigned* err;
  unsigned long long* diag;
  int fly, thin;  // ZMI_OPT_ENG_FLY / ZMI_OPT_ENG_THIN: slots per loader in flight, and while a service wave polls
  int hold;       // ZMI_OPT_ENG_HOLD: attention-chunk blocks issue no weights until their K / V landed
  int pf;         // ZMI_OPT_ENG_PF: the prefetch wave warms the Infinity Cache with the block's later slots
  int delay;      // ZMI_OPT_ENG_DELAY: ns the other blocks' loaders wait at launch start
};

__device__ __forceinline__ void stamp(const LArgs& a, int i) {
  if (a.diag && (threadIdx.x & 63) == 0) a.diag[(size_t)blockIdx.x * 64 + i] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ lds_u32* cnt(char* smem, int i) { return lds_word(smem, L_CNT + 4 * i); }

template <int NEXT>
__device__ __forceinline__ int n_next(int b) {
  if (NEXT == NEXT_QKV) return b < 128 ? 2 : 1;
  return (HEADS_GROUPS - b + 255) / 256;
}

// slot k of consumer wave c in block b: 8 KiB of one packed weight (M8 layout: group g's chunks contiguous)
template <int NEXT>
__device__ __forceinline__ const char* slot_src(const LArgs& a, int k, int b, int c) {
  const int s = b & 7, m = b >> 3;
  if (k == 0) return a.w_out + ((size_t)b * 32 + c * 8) * 1024;
  if (k <= 8) return a.w_fc1 + ((size_t)(256 * s + 8 * m + (k - 1)) * 32 + c * 8) * 1024;
  if (k <= 12) {
    const int kk = k - 9, g = 8 * m + 2 * c + (kk >> 1);
    return a.w_fc2 + ((size_t)g * 128 + s * 16 + (kk & 1) * 8) * 1024;
  }
  return a.w_next + ((size_t)(b + 256 * (k - 13)) * 32 + c * 8) * 1024;
}

__device__ __forceinline__ unsigned lds_ld(char* smem, int i) {
  return __hip_atomic_load(cnt(smem, i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(char* smem, int i, unsigned v) {
  __hip_atomic_store(cnt(smem, i), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// the oldest of `n + 1` outstanding slots has landed (loads complete in order)
__device__ __forceinline__ void wait_oldest(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(56)" ::: "memory"); break;
  }
}
static_assert(MAXFLY <= 8, "wait_oldest encodes up to 7 slots issued after the awaited one");

// The loader wave: every consumer's slots in (slot, consumer) order through the consumers' rings, by
// non-temporal LDS-DMA; slot k of consumer c is published FULL once landed and re-filled once the consumer
// marked it FREE. It keeps `a.fly` slots in flight, `a.thin` while a service wave of the block polls
// (MI355X_MICROARCH.md gather-pass: a poll queues behind the CU's own refill burst). It issues nothing
// else, so its vmcnt counts exactly its DMA pieces.
template <int NEXT>
__device__ __forceinline__ void loader(const LArgs& a, char* smem, int b, int lw, int lane) {
  const unsigned ring0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(__attribute__((address_space(3))) char*)(smem + L_RING));
  const int ns = CPL * (13 + n_next<NEXT>(b));
  if (a.delay > 0) {  // let the attention chunks' K / V loads reach HBM ahead of the weight streams
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime() + (unsigned long long)(a.delay / 10);
    while (__builtin_amdgcn_s_memrealtime() < t_end) __builtin_amdgcn_s_sleep(2);
  }
  int issued = 0, landed = 0;
  for (unsigned spin = 0; landed < ns;) {
    while (issued < ns) {
      const int k = issued / CPL, c = lw * CPL + (issued - k * CPL);
      const int lim = lds_ld(smem, C_HOLD) ? 0 : (lds_ld(smem, C_THIN) ? a.thin : a.fly);
      if (issued - landed >= lim) break;
      if (k >= DEPTH && lds_ld(smem, C_FREE + c * DEPTH + k % DEPTH) < (unsigned)(k - DEPTH + 1)) break;
      issue_slot(slot_src<NEXT>(a, k, b, c), ring0 + (c * DEPTH + k % DEPTH) * SLOT, lane);
      if (c == NCW - 1 && (k == 0 || k == 1 || k == 4 || k == 8 || k == 9 || k == 12 || k == 13)) stamp(a, 40 + (k < 2 ? k : (k == 4 ? 2 : (k == 8 ? 3 : (k == 9 ? 4 : (k == 12 ? 5 : 6))))));
      ++issued;
    }
    if (issued > landed) {
      wait_oldest(issued - landed - 1);
      const int k = landed / CPL, c = lw * CPL + (landed - k * CPL);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      if (lane == 0) lds_st(smem, C_FULL + c * DEPTH + k % DEPTH, (unsigned)(k + 1));
      if (c == NCW - 1 && (k == 0 || k == 8 || k == 12)) stamp(a, 48 + (k == 0 ? 0 : (k == 8 ? 1 : 2)));
      ++landed;
      spin = 0;
    } else {  // nothing in flight and nothing issuable: a consumer has not freed its slot yet
      if (++spin > SPIN) {
        give_up(a.err);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The prefetch wave: default-policy LDS-DMA reads (into a 1 KiB sink) of the block's weight slots past the
// loaders' first ring fill, in stream order, while the block waits on the attention chain (HBM is otherwise
// idle then); the loaders' later reads of those slots hit the Infinity Cache. It starts once C_PFGO is set
// and stops at C_PFSTOP (before the block's first latency-critical gather of its own), at most 40 KiB in flight.
template <int NEXT>
__device__ __forceinline__ void prefetcher(const LArgs& a, char* smem, int b, int lane) {
  if (!a.pf) return;
  const unsigned sink = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(__attribute__((address_space(3))) char*)(smem + L_SINK));
  for (unsigned spin = 0; !lds_ld(smem, C_PFGO); ++spin) {
    if (lds_ld(smem, C_PFSTOP) || spin > SPIN) return;
    __builtin_amdgcn_s_sleep(2);
  }
  const int ns = NCW * (13 + n_next<NEXT>(b));
  for (int t = NCW * DEPTH; t < ns; ++t) {
    if (lds_ld(smem, C_PFSTOP)) break;
    const int k = t / NCW, c = t - k * NCW;
    const char* g = slot_src<NEXT>(a, k, b, c) + lane * 16;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(g + j * 1024), "s"(sink)
                   : "memory");
    }
    asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int NEXT>
__device__ __forceinline__ void consumer(const LArgs& a, char* smem, int b, int c, int lane, const unsigned (&tag)[MAXR]) {
  const int nslot = 13 + n_next<NEXT>(b);
  const bf16_t* bufA = reinterpret_cast<const bf16_t*>(smem + L_BUFA);
  const bf16_t* bufB = reinterpret_cast<const bf16_t*>(smem + L_BUFB);
  float* redo = reinterpret_cast<float*>(smem + L_REDO);
  float* redf = reinterpret_cast<float*>(smem + L_REDF);
  float* redn = reinterpret_cast<float*>(smem + L_REDN);
  const int s = b & 7, m = b >> 3;
  const int col = lane & 15, quad = lane >> 4;
  const int ar = min(col, a.M - 1);
  f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < NSLOT_MAX; ++k) {
    if (k >= 13 && k >= nslot) continue;  // blocks with fewer next-op slots (compile-time trip count: unrolled)
    if (k == 0)
      lds_wait_ge(cnt(smem, C_READY), NSW * 1, a.err);
    else if (k == 1)
      lds_wait_ge(cnt(smem, C_READY), NSW * 2, a.err);
    else if (k == 9)
      lds_wait_ge(cnt(smem, C_READY), NSW * 3, a.err);
    else if (k == 13)
      lds_wait_ge(cnt(smem, C_READY), NSW * 4, a.err);
    // this item's activation rows (gemv_body step 4's A operand: lane l reads row min(l & 15, M - 1), k =
    // 8 (l >> 4) .. + 7 of each 32-wide k-half), read per chunk from LDS
    const bool f2 = k >= 9 && k <= 12;
    const bool second = f2 && ((k - 9) & 1);  // second half of an fc2 segment: the chain continues
    const bf16_t* xb = (k == 0 || f2 ? bufA : bufB) + ar * XROW + (f2 ? 8 * 64 * (second ? 1 : 0) : c * 512) + quad * 8;
    // the slot: landed (FULL), read, then FREE for the loader
    {
      lds_u32* full = cnt(smem, C_FULL + c * DEPTH + k % DEPTH);
      for (unsigned spin = 0; __hip_atomic_load(full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != (unsigned)(k + 1);
           ++spin) {
        if (spin > SPIN) {
          give_up(a.err);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    }
    if (c == 0 && (k == 0 || k == 1 || k == 9 || k == 13)) stamp(a, 16 + (k == 0 ? 0 : (k == 1 ? 1 : (k == 9 ? 2 : 3))));
    u32x4_t wv[8];
    const u32x4_t* rp = reinterpret_cast<const u32x4_t*>(smem + L_RING + ((size_t)c * DEPTH + k % DEPTH) * SLOT) + lane;
#pragma unroll
    for (int j = 0; j < 8; ++j) wv[j] = rp[j * 64];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) lds_st(smem, C_FREE + c * DEPTH + k % DEPTH, (unsigned)(k + 1));
    if (!second) acc0 = acc1 = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bf16x8_t w = __builtin_bit_cast(bf16x8_t, wv[j]);
      const uint4 x0 = *reinterpret_cast<const uint4*>(xb + j * 64);
      const uint4 x1 = *reinterpret_cast<const uint4*>(xb + j * 64 + 32);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x0), w, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x1), w, acc1, 0, 0, 0);
    }
    if (f2 && !second) continue;
    float v[MAXR];
#pragma unroll
    for (int q = 0; q < MAXR; ++q) v[q] = acc0[q] + ror8(acc1[q]);  // gemv_body step 5
    const bool mine = col < 8 && quad == 0;
    if (k == 0) {
      if (mine)
#pragma unroll
        for (int q = 0; q < MAXR; ++q) redo[(c * 8 + col) * MAXR + q] = v[q];
      lds_arrive(cnt(smem, C_O), lane);
    } else if (k <= 8) {
      if (mine)
#pragma unroll
        for (int q = 0; q < MAXR; ++q) redf[(((k - 1) * NCW + c) * 8 + col) * MAXR + q] = v[q];
      lds_arrive(cnt(smem, C_F1 + k - 1), lane);
      if (k == 8) stamp(a, 20 + c);
    } else if (f2) {
      const int g = 8 * m + 2 * c + ((k - 9) >> 1);
      uint64_t* gp = a.gran + Gran(a.M).gp;
      if (mine)
#pragma unroll
        for (int q = 0; q < MAXR; ++q)
          if (q < a.M)
            st_wt64(gp + (((size_t)g * 8 + s) * a.M + q) * 8 + col,
                    (uint64_t)__float_as_uint(v[q]) | ((uint64_t)tag[q] << 32));
      if (k == 12) stamp(a, 24 + c);
    } else {
      if (mine)
#pragma unroll
        for (int q = 0; q < MAXR; ++q) redn[(((k - 13) * NCW + c) * 8 + col) * MAXR + q] = v[q];
      lds_arrive(cnt(smem, C_N + k - 13), lane);
    }
  }
}

// a service wave polls: the block's loader keeps `a.thin` slots in flight meanwhile
__device__ __forceinline__ void thin_on(char* smem, int lane) {
  if (lane == 0) __hip_atomic_fetch_add(cnt(smem, C_THIN), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void thin_off(char* smem, int lane) {
  if (lane == 0) __hip_atomic_fetch_sub(cnt(smem, C_THIN), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// service-wave barrier (the consumers do not take part); n counts this wave's barriers, the same count in
// every service wave of a block (all take the same path)
__device__ __forceinline__ void svc_sync(char* smem, unsigned& n, int lane, unsigned* err) {
  ++n;
  lds_arrive(cnt(smem, C_SVC), lane);
  lds_wait_ge(cnt(smem, C_SVC), NSW * n, err);
}

__device__ __forceinline__ uint32_t tag_of(uint64_t g) { return (uint32_t)(g >> 32); }

// poll granule *p until its tag matches (one lane's view; the caller keeps the wave together)
__device__ __forceinline__ uint64_t poll1(const uint64_t* p, uint32_t tag, unsigned* err) {
  uint64_t w = ld_wt64(p);
  for (unsigned spin = 0; tag_of(w) != tag; ++spin) {
    if (spin > SPIN) {
      give_up(err);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
    w = ld_wt64(p);
  }
  return w;
}

// The attention of unit u (row r, kv head kh), chunk c = 128 keys, by the 4 service waves: xc_body's
// (zmi_attnblk.hip) roles 0..7 on waves sw and sw + 4, the operations of the chunked kernel.
__device__ __forceinline__ void attention(const LArgs& a, char* smem, int b, int sw, int lane, unsigned& nsync,
                                          unsigned* err) {
  const int u = b & 7, r = u >> 2, kh = u & 3, c = b >> 3;
  if (r >= a.M) return;
  const int pos = a.row_pos[r];
  if (pos < 0) return;
  if (pos >= NCH * CH) {
    if (sw == 0 && lane == 0) give_up(err);
    return;
  }
  const uint32_t tag = (uint32_t)pos + 1u;
  const uint64_t tag64 = (uint64_t)tag << 32;
  float(&sc)[XG][CH] = *reinterpret_cast<float(*)[XG][CH]>(smem + A_SC);
  bf16_t(&pb)[XG][CH] = *reinterpret_cast<bf16_t(*)[XG][CH]>(smem + A_PB);
  float(&opart)[CPG][XG][HD] = *reinterpret_cast<float(*)[CPG][XG][HD]>(smem + A_OP);
  float* mj = reinterpret_cast<float*>(smem + A_MJ);
  const Gran G(a.M);
  uint64_t* gm = a.gran + G.gm + (size_t)u * NCH * XG;
  uint64_t* gl = a.gran + G.gl + (size_t)u * NCH * XG;
  uint64_t* gbm = a.gran + G.gb + (size_t)u * NCH * XG;
  uint64_t* go = a.gran + G.go + (size_t)u * NCH * XG * HD;
  const int c16 = lane & 15, h4 = lane >> 4;
  const int nk = pos + 1, n32 = (pos + 32) >> 5, nc = pos / CH + 1;
  const int t = sw * 64 + lane;
  if (c < nc) {
    const size_t kvbase = ((size_t)r * HKV + kh) * a.smax * HD;
    // (1) K rows of score tiles (gs, tt) = ((sw >> 1) + 2 i, sw & 1) and V^T of group gv = sw, dims 64 hv ..
    const int tt = sw & 1, gv = sw;
    bool sk[2];
    uint4 kf[2][4], vf[2][4], qf[4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int gs = (sw >> 1) + 2 * i;
      sk[i] = CPG * c + gs < n32;
      if (sk[i]) {
        const bf16_t* kr = a.kc + kvbase + (size_t)min(CH * c + 32 * gs + 16 * tt + c16, pos) * HD + 8 * h4;
#pragma unroll
        for (int db = 0; db < 4; ++db) kf[i][db] = *reinterpret_cast<const uint4*>(kr + 32 * db);
      }
    }
    const bool vk = CPG * c + gv < n32;
    if (vk) {
      const int p0 = min(CH * c + 32 * gv + 8 * h4, pos & ~7);
#pragma unroll
      for (int hv = 0; hv < 2; ++hv)
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          vf[hv][dt] = *reinterpret_cast<const uint4*>(a.vc + kvbase + (size_t)(64 * hv + 16 * dt + c16) * a.smax + p0);
    }
    {
      const bf16_t* qr = a.q + (size_t)r * QCOLS + (kh * XG + (c16 < XG ? c16 : 0)) * HD + 8 * h4;
#pragma unroll
      for (int db = 0; db < 4; ++db) qf[db] = c16 < XG ? *reinterpret_cast<const uint4*>(qr + 32 * db) : uint4{0u, 0u, 0u, 0u};
    }
    // (2) scores
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (!sk[i]) continue;
      const int gs = (sw >> 1) + 2 * i;
      f32x4_t sv = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int db = 0; db < 4; ++db) sv = mfma16(qf[db], kf[i][db], sv);
      const int key = CH * c + 32 * gs + 16 * tt + c16;
      if (h4 == 0 && key <= pos) {
#pragma unroll
        for (int g = 0; g < XG; ++g) sc[g][key - CH * c] = sv[g] * a.scale;
      }
    }
    if (sw == 0) stamp(a, 10);
    svc_sync(smem, nsync, lane, err);
    if (sw == 0 && lane == 0) lds_st(smem, C_HOLD, 0u);  // the chunk's K / V have landed: weights may stream
    if (sw == 0) stamp(a, 11);
    // (3) wave 0: the chunk maxima out as granules, then M_j of the chunk's block from the maxima of
    // chunks 0 .. dep - 1 (max is exact in any order)
    if (sw == 0) {
      float mx[XG];
#pragma unroll
      for (int g = 0; g < XG; ++g)
        mx[g] = fmaxf(CH * c + lane < nk ? sc[g][lane] : -INFINITY, CH * c + lane + 64 < nk ? sc[g][lane + 64] : -INFINITY);
#pragma unroll
      for (int g = 0; g < XG; ++g) mx[g] = wave_max(mx[g]);
      if (lane < XG) {
        const float mine = lane == 0 ? mx[0] : (lane == 1 ? mx[1] : (lane == 2 ? mx[2] : mx[3]));
        st_wt64(gm + c * XG + lane, (uint64_t)__float_as_uint(mine) | tag64);
      }
      const int j = c / CPB, dep = min((j + 1) * CPB, nc);
      float v = -INFINITY;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = lane + 64 * h, cc = e / XG, g = e - cc * XG;
        if (e < dep * XG) {
          float w;
          if (cc == c)
            w = g == 0 ? mx[0] : (g == 1 ? mx[1] : (g == 2 ? mx[2] : mx[3]));
          else
            w = __uint_as_float((uint32_t)poll1(gm + e, tag, err));
          v = fmaxf(v, w);
        }
      }
      v = fmaxf(v, __shfl_xor(v, 4));
      v = fmaxf(v, __shfl_xor(v, 8));
      v = fmaxf(v, __shfl_xor(v, 16));
      v = fmaxf(v, __shfl_xor(v, 32));
      if (lane < XG) mj[lane] = v;
    }
    if (sw == 0) stamp(a, 12);
    svc_sync(smem, nsync, lane, err);
    // (4) wave g: e = exp(s - M_j), l (lane L: keys L, L + 64, then wave_sum), P = bf16(e)
    {
      const int g = sw;
      const float M = mj[g];
      float l = 0.f;
#pragma unroll
      for (int ii = 0; ii < CH / 64; ++ii) {
        const int kk = lane + 64 * ii;
        const float e = CH * c + kk < nk ? expf(sc[g][kk] - M) : 0.f;
        l += e;
        pb[g][kk] = (bf16_t)f2bf(e);
      }
      l = wave_sum(l);
      if (lane == 0) {
        st_wt64(gl + c * XG + g, (uint64_t)__float_as_uint(l) | tag64);
        st_wt64(gbm + c * XG + g, (uint64_t)__float_as_uint(M) | tag64);
      }
    }
    svc_sync(smem, nsync, lane, err);
    // (5) P.V of group gv for dims 64 hv .. + 63 (V of keys past the position zeroed)
    if (vk) {
      uint4 pf = uint4{0u, 0u, 0u, 0u};
      if (c16 < XG) pf = *reinterpret_cast<const uint4*>(&pb[c16][32 * gv + 8 * h4]);
      const int kbase = CH * c + 32 * gv + 8 * h4;
#pragma unroll
      for (int hv = 0; hv < 2; ++hv)
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          uint4 v = vf[hv][dt];
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
    svc_sync(smem, nsync, lane, err);
    if (sw == 0) stamp(a, 13);
    // (6) the chunk's P.V (groups summed in group order) out as granules, two (head, dim) per thread
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int idx = t + 256 * h, g = idx / HD, d = idx - g * HD;
      float o = opart[0][g][d];
#pragma unroll
      for (int w = 1; w < CPG; ++w)
        if (CPG * c + w < n32) o += opart[w][g][d];
      st_wt64(go + ((size_t)c * XG + g) * HD + d, (uint64_t)__float_as_uint(o) | tag64);
    }
  } else {
    svc_sync(smem, nsync, lane, err);  // the chunk-live blocks' last barrier count is theirs alone: harmless
  }
  // (7) chunk blocks 0..7: dims 16 c .. 16 c + 15 of the unit's output, the block recursion of zmi_attn_merge.h
  // over every chunk's partial, l and M_j, one (head, dim) per lane of wave 0; out as {pair, tag} granules of
  // the attention rows
  if (sw == 0 && c < NMRG) {
    thin_on(smem, lane);
    const int g = lane >> 4, d = MDIM * c + (lane & 15);
    float acc = 0.f, l = 0.f, ob = 0.f, lb = 0.f, mprev = 0.f, mb = 0.f;
    for (int k0 = 0; k0 < nc; k0 += 8) {
      uint64_t ov[8], lv[8], mv[2];
      unsigned pend = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k0 + k < nc) pend |= 3u << (2 * k);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (k0 + j * CPB < nc) pend |= 1u << (16 + j);
      for (unsigned spin = 0;; ++spin) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if ((pend >> (2 * k)) & 1) ov[k] = ld_wt64(go + ((size_t)(k0 + k) * XG + g) * HD + d);
          if ((pend >> (2 * k + 1)) & 1) lv[k] = ld_wt64(gl + (k0 + k) * XG + g);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if ((pend >> (16 + j)) & 1) mv[j] = ld_wt64(gbm + (k0 + j * CPB) * XG + g);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (((pend >> (2 * k)) & 1) && tag_of(ov[k]) == tag) pend &= ~(1u << (2 * k));
          if (((pend >> (2 * k + 1)) & 1) && tag_of(lv[k]) == tag) pend &= ~(1u << (2 * k + 1));
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (((pend >> (16 + j)) & 1) && tag_of(mv[j]) == tag) pend &= ~(1u << (16 + j));
        if (__all(pend == 0)) break;
        if (spin > SPIN) {
          give_up(err);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        const int k = k0 + kk;
        if (k >= nc) continue;
        const float o = __uint_as_float((uint32_t)ov[kk]), lk = __uint_as_float((uint32_t)lv[kk]);
        if (k % CPB == 0) {
          ob = o;
          lb = lk;
          mb = __uint_as_float((uint32_t)mv[kk / CPB]);
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
    }
    stamp(a, 14);
    const float rl = 1.0f / l;
    const uint32_t ov = f2bf(acc * rl);
    const uint32_t nb = (uint32_t)__shfl_down((int)ov, 1);
    const int col = (kh * XG + g) * HD + d;
    {
      if ((lane & 1) == 0)
        st_wt64(a.gran + G.ga + (size_t)r * (DM / 2) + (col >> 1), (uint64_t)(ov | (nb << 16)) | tag64);
      if (a.attn_out) a.attn_out[(size_t)r * DM + col] = (bf16_t)ov;
    }
    thin_off(smem, lane);
  }
}

template <int NEXT>
__device__ __forceinline__ void service(const LArgs& a, char* smem, int b, int sw, int lane, const unsigned (&tag)[MAXR]) {
  const int s = b & 7, m = b >> 3;
  bf16_t* bufA = reinterpret_cast<bf16_t*>(smem + L_BUFA);
  bf16_t* bufB = reinterpret_cast<bf16_t*>(smem + L_BUFB);
  const float* redo = reinterpret_cast<const float*>(smem + L_REDO);
  const float* redf = reinterpret_cast<const float*>(smem + L_REDF);
  const float* redn = reinterpret_cast<const float*>(smem + L_REDN);
  const Gran G(a.M);
  uint64_t* gr = a.gran;
  // this wave's row in the row-split phases, and the half of that row it gathers
  const int rr = sw >> 1, half = sw & 1;
  const bool rlive = rr < a.M && a.row_pos[rr] >= 0;
  const unsigned rtag = rr < a.M ? tag[rr] : 0u;
  // the row of the wave's row-owned phases (epilogues, LayerNorm): waves 0 and 1
  const bool own = sw < a.M && a.row_pos[sw] >= 0;
  const unsigned otag = sw < a.M ? tag[sw] : 0u;
  if (sw == 0) stamp(a, 0);
  // residual values of out_proj's columns (row sw), loaded early
  uint32_t xres = 0;
  if (own && lane < 8) xres = a.x[(size_t)sw * DM + 8 * b + lane];
  unsigned nsync = 0;
  attention(a, smem, b, sw, lane, nsync, a.err);
  if (sw == 0 && lane == 0) lds_st(smem, C_PFGO, 1u);
  // the norm2 / next-norm parameters into registers now (their loads are far from the critical path here)
  uint4 ln2g[4], ln2b[4], lnng[4], lnnb[4];
  if (own) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      ln2g[q] = *reinterpret_cast<const uint4*>(a.ln2_w + q * 512 + lane * 8);
      ln2b[q] = *reinterpret_cast<const uint4*>(a.ln2_b + q * 512 + lane * 8);
      lnng[q] = *reinterpret_cast<const uint4*>(a.lnn_w + q * 512 + lane * 8);
      lnnb[q] = *reinterpret_cast<const uint4*>(a.lnn_b + q * 512 + lane * 8);
    }
  }
  thin_on(smem, lane);
  if (sw == 0) stamp(a, 1);
  stamp(a, 28 + sw);
  svc_sync(smem, nsync, lane, a.err);  // the attention scratch (BUFA / BUFB) is free
  // (1) the attention rows -> BUFA (out_proj's activations)
  if (rlive)
    gather<512 / 64>(gr + G.ga + (size_t)rr * (DM / 2) + 512 * half, reinterpret_cast<uint32_t*>(bufA + rr * XROW) + 512 * half,
                     rtag, lane, a.err);
  thin_off(smem, lane);
  if (sw == 0) stamp(a, 2);
  lds_arrive(cnt(smem, C_READY), lane);
  // (2) out_proj epilogue (EPI_RESIDUAL) of row sw: x' = bf16(x + bf16(segment sums in order)), out as granules
  lds_wait_ge(cnt(smem, C_O), NCW, a.err);
  uint32_t xnew = 0;
  if (own) {
    float v = 0.f;
    if (lane < 8) {
      v = redo[(0 * 8 + lane) * MAXR + sw];
#pragma unroll
      for (int w = 1; w < NCW; ++w) v += redo[(w * 8 + lane) * MAXR + sw];
    }
    xnew = f2bf(bf2f(xres) + bfround(v));
    const uint32_t nb = (uint32_t)__shfl_down((int)xnew, 1);
    if (lane < 8 && (lane & 1) == 0)
      st_wt64(gr + G.gx + (size_t)sw * (DM / 2) + 4 * b + (lane >> 1), (uint64_t)(xnew | (nb << 16)) | ((uint64_t)otag << 32));
  }
  if (sw == 0) stamp(a, 3);
  // (3) x' of every block -> BUFB, then norm2 in place (fc1's activations)
  if (sw == 0 && lane == 0) lds_st(smem, C_PFSTOP, 1u);
  thin_on(smem, lane);
  if (rlive)
    gather<512 / 64>(gr + G.gx + (size_t)rr * (DM / 2) + 512 * half, reinterpret_cast<uint32_t*>(bufB + rr * XROW) + 512 * half,
                     rtag, lane, a.err);
  thin_off(smem, lane);
  if (sw == 0) stamp(a, 4);
  svc_sync(smem, nsync, lane, a.err);
  if (own) ln_row_r(bufB + sw * XROW, ln2g, ln2b, a.eps, lane);
  lds_arrive(cnt(smem, C_READY), lane);
  // (4) fc1 epilogues (EPI_SWIGLU, M8 packing: columns 0..3 values, 4..7 gates): groups sw and sw + 4, lane =
  // (row, column), out as h granules
  {
    const int r = lane >> 2, cc = lane & 3;
    const bool ok = r < a.M && a.row_pos[r < a.M ? r : 0] >= 0;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = sw + 4 * jj;
      lds_wait_ge(cnt(smem, C_F1 + j), NCW, a.err);
      auto colsum = [&](int col) {
        float v = redf[((j * NCW + 0) * 8 + col) * MAXR + r];
#pragma unroll
        for (int w = 1; w < NCW; ++w) v += redf[((j * NCW + w) * 8 + col) * MAXR + r];
        return v;
      };
      uint32_t hv = 0;
      if (lane < 4 * MAXR && r < a.M) {
        const float y = bfround(colsum(cc));
        const float gt = bfround(colsum(cc + 4));
        const float sg = bfround(gt / (1.0f + expf(-gt)));
        hv = f2bf(y * sg);
      }
      const uint32_t nb = (uint32_t)__shfl_down((int)hv, 1);
      const int hi = 1024 * s + 32 * m + 4 * j + cc;
      if (lane < 4 * MAXR && ok && (cc & 1) == 0)
        st_wt64(gr + G.gh + (size_t)r * (FF / 2) + (hi >> 1), (uint64_t)(hv | (nb << 16)) | ((uint64_t)tag[r < MAXR ? r : 0] << 32));
    }
  }
  if (sw == 0) stamp(a, 5);
  stamp(a, 32 + sw);
  // (5) h segment s (fc2's activations for this block's K segment), produced by team s -> BUFA
  thin_on(smem, lane);
  if (rlive)
    gather<256 / 64>(gr + G.gh + (size_t)rr * (FF / 2) + 512 * s + 256 * half,
                     reinterpret_cast<uint32_t*>(bufA + rr * XROW) + 256 * half, rtag, lane, a.err);
  thin_off(smem, lane);
  if (sw == 0) stamp(a, 6);
  lds_arrive(cnt(smem, C_READY), lane);
  thin_on(smem, lane);
  // (6) fc2 group b of row sw: the 8 segment sums (blocks 8 (b >> 3) + s') in segment order + the residual x'
  if (own) {
    const int sp = lane >> 3, cc = lane & 7;
    const uint64_t w = poll1(gr + G.gp + (((size_t)b * 8 + sp) * a.M + sw) * 8 + cc, otag, a.err);
    const float val = __uint_as_float((uint32_t)w);
    float v = __shfl(val, cc);
#pragma unroll
    for (int q = 1; q < 8; ++q) v += __shfl(val, 8 * q + cc);
    const uint32_t xo = f2bf(bf2f(xnew) + bfround(v));
    const uint32_t nb = (uint32_t)__shfl_down((int)xo, 1);
    if (lane < 8) a.x[(size_t)sw * DM + 8 * b + lane] = (bf16_t)xo;
    if (lane < 8 && (lane & 1) == 0)
      st_wt64(gr + G.gy + (size_t)sw * (DM / 2) + 4 * b + (lane >> 1), (uint64_t)(xo | (nb << 16)) | ((uint64_t)otag << 32));
  }
  if (sw == 0) stamp(a, 7);
  // (7) x'' of every block -> BUFB, then the next op's LayerNorm in place
  if (rlive)
    gather<512 / 64>(gr + G.gy + (size_t)rr * (DM / 2) + 512 * half, reinterpret_cast<uint32_t*>(bufB + rr * XROW) + 512 * half,
                     rtag, lane, a.err);
  thin_off(smem, lane);
  if (sw == 0) stamp(a, 8);
  svc_sync(smem, nsync, lane, a.err);
  if (own) ln_row_r(bufB + sw * XROW, lnng, lnnb, a.eps, lane);
  lds_arrive(cnt(smem, C_READY), lane);
  // (8) the next op's epilogues: item i (column group b + 256 i) on wave i % 4
  const int nn = n_next<NEXT>(b);
  for (int i = sw; i < nn; i += NSW) {
    lds_wait_ge(cnt(smem, C_N + i), NCW, a.err);
    const int g = b + 256 * i;
    auto colsum = [&](int col, int r) {
      float v = redn[((i * NCW + 0) * 8 + col) * MAXR + r];
#pragma unroll
      for (int w = 1; w < NCW; ++w) v += redn[((i * NCW + w) * 8 + col) * MAXR + r];
      return v;
    };
    if (NEXT == NEXT_QKV) {
      // zmi_gemv_impl.h epilogue EPI_QKV: q | k | v split, interleaved-pair RoPE in fp32, KV-cache write
      const int r = lane >> 2, c = (lane & 3) * 2;
      const int q_pos = r < a.M ? a.row_pos[r] : -1;
      if (r < a.M && q_pos >= 0 && q_pos < a.smax) {
        const int n = g * 8 + c;
        float x0 = bfround(colsum(c, r)), x1 = bfround(colsum(c + 1, r));
        if (n < QCOLS + KCOLS) {
          const int d = (n < QCOLS ? n : n - QCOLS) % HD;
          const float2 cs = *reinterpret_cast<const float2*>(a.rope + ((size_t)q_pos * (HD >> 1) + (d >> 1)) * 2);
          const float co = cs.x, si = cs.y;
          const float r0 = x0 * co - x1 * si;
          const float r1 = x1 * co + x0 * si;
          x0 = r0;
          x1 = r1;
        }
        const uint32_t packed = f2bf(x0) | (f2bf(x1) << 16);
        if (n < QCOLS) {
          *reinterpret_cast<uint32_t*>(a.q + (size_t)r * QCOLS + n) = packed;
        } else if (n < QCOLS + KCOLS) {
          const int nn2 = n - QCOLS, kh = nn2 / HD, d = nn2 - kh * HD;
          *reinterpret_cast<uint32_t*>(a.kn + (((size_t)r * HKV + kh) * a.smax + q_pos) * HD + d) = packed;
        } else {
          const int nn2 = n - QCOLS - KCOLS, kh = nn2 / HD, d = nn2 - kh * HD;
          bf16_t* vt = a.vn + (((size_t)r * HKV + kh) * HD + d) * a.smax + q_pos;
          vt[0] = (bf16_t)(packed & 0xffffu);
          vt[a.smax] = (bf16_t)(packed >> 16);
        }
      }
    } else {
      // EPI_LOGITS: 9 heads back to back, 1026 columns each
      const int r = lane >> 3, c = lane & 7, n = g * 8 + c;
      if (r < a.M && n < HEADS_VALID) {
        const float v = colsum(c, r);
        const int cbk = n / 1026, vv = n - cbk * 1026;
        a.logits[((size_t)r * 9 + cbk) * 1026 + vv] = bfround(v);
      }
    }
  }
  if (sw == 0) stamp(a, 9);
  stamp(a, 36 + sw);
}

template <int NEXT>
__global__ __launch_bounds__(NT) void layer_engine_kernel(const LArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  unsigned tag[MAXR];
#pragma unroll
  for (int r = 0; r < MAXR; ++r) tag[r] = r < a.M ? (unsigned)(a.row_pos[r] + 1) : 0u;
  if (tid < C_WORDS) {
    unsigned v = 0u;
    const int r = (b & 7) >> 2, pos = r < a.M ? a.row_pos[r] : -1;
    const bool live = pos >= 0 && (b >> 3) <= pos / CH, merge = pos >= 0 && (b >> 3) < NMRG;
    if (tid == C_HOLD && a.hold) v = live ? 1u : 0u;  // this block loads a live attention chunk's K / V first
    if (tid == C_PFGO) v = (live || merge) ? 0u : 1u;  // attention blocks prefetch once their chunk is done
    *cnt(smem, tid) = v;
  }
  __syncthreads();
  if (wave < NLW)
    loader<NEXT>(a, smem, b, wave, lane);
  else if (wave < NLW + NCW)
    consumer<NEXT>(a, smem, b, wave - NLW, lane, tag);
  else if (wave < NLW + NCW + NSW)
    service<NEXT>(a, smem, b, wave - NLW - NCW, lane, tag);
  else
    prefetcher<NEXT>(a, smem, b, lane);
}

}  // namespace

extern "C" int64_t zmi_layer_engine_gran_words(int rows) {
  return (rows < 1 || rows > MAXR) ? -1 : (int64_t)Gran(rows).total;
}

extern "C" int zmi_layer_engine_max_pos(void) { return NCH * CH - 1; }

extern "C" int zmi_layer_engine(const ZmiLayerEngineArgs* args, void* stream) {
  const ZmiLayerEngineArgs& e = *args;
  if (e.M < 1 || e.M > MAXR) return zmi_fail_msg("layer_engine: 1 <= M <= 2 rows");
  if (e.next != 0 && e.next != 1) return zmi_fail_msg("layer_engine: next must be 0 (QKV) or 1 (heads)");
  if (!e.w_out || !e.w_fc1 || !e.w_fc2 || !e.w_next || !e.ln2_w || !e.ln2_b || !e.lnn_w || !e.lnn_b || !e.x || !e.q ||
      !e.k_cache || !e.v_cache || !e.row_pos || !e.gran || !e.err)
    return zmi_fail_msg("layer_engine: missing buffers");
  if (e.next == 0 && (!e.k_next || !e.v_next || !e.rope)) return zmi_fail_msg("layer_engine: QKV needs k_next, v_next, rope");
  if (e.next == 1 && !e.logits) return zmi_fail_msg("layer_engine: heads need logits");
  if (e.smax <= 0 || e.smax % 8) return zmi_fail_msg("layer_engine: smax must be a positive multiple of 8");
  if (zmi_cu_count() < NBLK) return zmi_fail_msg("layer_engine: needs 256 CUs (one resident workgroup per CU)");
  LArgs a{};
  a.w_out = (const char*)e.w_out;
  a.w_fc1 = (const char*)e.w_fc1;
  a.w_fc2 = (const char*)e.w_fc2;
  a.w_next = (const char*)e.w_next;
  a.ln2_w = (const bf16_t*)e.ln2_w;
  a.ln2_b = (const bf16_t*)e.ln2_b;
  a.lnn_w = (const bf16_t*)e.lnn_w;
  a.lnn_b = (const bf16_t*)e.lnn_b;
  a.eps = e.eps;
  a.scale = 1.0f / sqrtf((float)HD);
  a.M = e.M;
  a.smax = e.smax;
  a.row_pos = e.row_pos;
  a.x = (bf16_t*)e.x;
  a.q = (bf16_t*)e.q;
  a.kc = (const bf16_t*)e.k_cache;
  a.vc = (const bf16_t*)e.v_cache;
  a.kn = (bf16_t*)e.k_next;
  a.vn = (bf16_t*)e.v_next;
  a.rope = e.rope;
  a.attn_out = (bf16_t*)e.attn_out;
  a.logits = e.logits;
  a.gran = (uint64_t*)e.gran;
  a.err = e.err;
  a.diag = (unsigned long long*)e.diag;
  a.fly = std::max(1, std::min(MAXFLY, zmi_option(ZMI_OPT_ENG_FLY)));
  a.thin = std::max(1, std::min(a.fly, zmi_option(ZMI_OPT_ENG_THIN)));
  a.hold = zmi_option(ZMI_OPT_ENG_HOLD);
  a.pf = zmi_option(ZMI_OPT_ENG_PF);
  a.delay = zmi_option(ZMI_OPT_ENG_DELAY);
  hipStream_t s = (hipStream_t)stream;
  if (e.next == 0) {
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&layer_engine_kernel<NEXT_QKV>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)L_BYTES);
    ZMI_CHECK(attr);
    hipLaunchKernelGGL(layer_engine_kernel<NEXT_QKV>, dim3(NBLK), dim3(NT), L_BYTES, s, a);
  } else {
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&layer_engine_kernel<NEXT_HEADS>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)L_BYTES);
    ZMI_CHECK(attr);
    hipLaunchKernelGGL(layer_engine_kernel<NEXT_HEADS>, dim3(NBLK), dim3(NT), L_BYTES, s, a);
  }
  ZMI_CHECK(hipGetLastError());
  return 0;
}
