// Persistent decode step for gfx950: the whole Zonos transformer backbone + norm_f + heads for one
// decode position in ONE launch (reference zonos/backbone/_torch.py:73-152, zonos/model.py:100-116).
//
// Why one launch: a batch-1 decode layer is five dependent weight streams (qkv 12.6 MB, attention,
// out 8.4 MB, fc1 67.1 MB, fc2 33.6 MB). As separate kernels every boundary drains the HBM pipe:
// the next kernel's weights are requested only after its launch, so each phase pays a launch gap, a
// fill and a tail (MI355X_MICROARCH.md price list, rows boundary / launches-baseline). Here the
// weights never wait for the chain: every wave owns a static list of weight-slice tasks and issues
// a task's whole slice (16 x 16 B per lane, non-temporal) BEFORE it waits for that task's input,
// so up to 15 x 16 KiB per CU are in flight through every dependency edge of the layer.
//
// Geometry: one 1024-thread workgroup per CU (grid = CU count, all resident). Waves 0..14 run
// tasks; wave 15 is the stager: it gathers the residual rows, computes the LayerNorm once per CU
// and publishes the normalised rows in LDS for the GEMV tasks that need them.
//
// Tasks (host plan: zonos_vibes_amd/step_plan.py), per layer in chain order:
//   QKV   (group g of 8 columns, part wk of K)  LN1 rows -> q granules, new k/v granules + KV cache
//   ATT   (unit = (row, kv head), CU j of the unit's att_cus) positions j, j+att_cus, ... <= pos:
//         history K/V prefetched into LDS by DMA at task start, then scores/softmax/PV partial,
//         published; then the CU merges a 512/att_cus-dim slice of the unit's 4 heads
//   OUT   attention rows (granules) -> out_proj + residual -> x granules
//   FC1   LN2 rows -> fc1 + SwiGLU -> h granules
//   FC2   h rows (granules) -> fc2 + residual -> x granules
// then HEADS (norm_f rows -> 9 heads -> f32 logits, plain stores read by the next launch).
//
// Hand-offs: every activation crossing CUs is an 8-byte granule {tag, 32-bit value} written by
// ONE agent-scope (sc1) store; consumers re-read with sc1 loads until every tag matches
// (MI355X_MICROARCH.md "Valid forms", R2 / cdna_hip_programming.md Guideline 16). tag =
// epoch << 6 | layer << 1 | sub, where the epoch is a device word bumped by the last workgroup
// to finish, so tags never repeat across launches (graph replays included).
//
// GEMV numerics are bit-identical to zmi_gemv8::gemv8_kernel (same per-lane k ranges, FMA order,
// 8-lane DPP tree, part order of the final sum, LayerNorm reduction order and epilogues).
#include "zmi_common.h"
#include "zmi_kernels.h"

namespace zmi_step {

typedef unsigned long long u64;
typedef __attribute__((address_space(1))) u64 gu64;
typedef __attribute__((address_space(1))) unsigned gu32;
#define ZLDS __attribute__((address_space(3)))
#define ZG __attribute__((address_space(1)))  // explicit global space: generic (flat) accesses count
                                              // in both vmcnt and lgkmcnt and force full drains
typedef ZLDS bf16_t lbf;  // LDS pointers are declared as such: generic (flat) LDS access is slower
typedef ZLDS float lfl;

constexpr int NWAVES = 16, NCW = 15, NT = NWAVES * 64;
constexpr int D = 2048, F = 8192, HD = 128, HQ = 16, HKV = 4, GQ = HQ / HKV;
constexpr int QN = HQ * HD, KVN = HKV * HD;  // 2048, 512
constexpr int NSLOT = 32;
constexpr int REC = HD + 2;                  // attention partial record per head: m, l, o[128]
constexpr float ATT_SCALE = 0.08838834764831845f;  // 1 / sqrt(128), SDPA default scale
constexpr int T_QKV = 0, T_ATT = 1, T_OUT = 2, T_FC1 = 3, T_FC2 = 4, T_HEADS = 5;
constexpr int FLAGS = 0x00020000;            // buffer descriptor dword3 (as zmi_gemv8)
constexpr unsigned long long SPIN_LIMIT = 20000000ull;  // 200 ms of s_memrealtime (100 MHz)

struct Gran {  // granule arrays inside the caller's buffer
  gu64 *xg, *qg, *kvg, *ag, *hg, *pg;
  gu32* hint;  // [layer][nhint] completion counters (hints only: every read is tag-checked)
};

// Completion hints. A consumer polls a few 4-byte counters (one lane each) until the producers
// of an edge have all reported, and only then sweeps the edge's granules (once, usually): the
// granule tags stay the correctness check, the hints keep waiting waves from re-reading whole
// edges through the fabric. Shard counters: one per b % 8 (the CUs of one XCD under the observed
// placement), bumped once per launch by every workgroup of the shard (each owns work of every
// phase); attention-unit counters: once per launch by each member. Counts accumulate over
// launches, so the target is epoch x contributors.
constexpr int H_QKV = 0, H_MERGED = 8, H_OUT = 16, H_FC1 = 24, H_FC2 = 32, H_ATT = 40;
constexpr int HS = 32;  // u32 stride between counters: each on a 128-B line of its own
// hint kinds polled per CU (one elected poller each, the other waves wait on the LDS copy)
constexpr int K_QKV = 0, K_MERGED = 1, K_OUT = 2, K_FC1 = 3, K_FC2 = 4, K_ATT = 5, NKIND = 6;
__host__ __device__ inline int nhint(int units) { return H_ATT + units; }

__device__ __forceinline__ Gran carve(uint64_t* base, int R, int nb) {
  Gran g;
  gu64* p = ((gu64*)(base));
  g.xg = p;
  g.qg = g.xg + R * (D / 2);
  g.kvg = g.qg + R * (QN / 2);
  g.ag = g.kvg + R * KVN;
  g.hg = g.ag + R * (QN / 2);
  g.pg = g.hg + R * (F / 2);
  g.hint = (gu32*)(g.pg + (size_t)nb * GQ * REC);
  return g;
}

struct Ctl {  // LDS control words
  unsigned cnt[NSLOT];
  unsigned pdone[8];  // groups of each task type completed on this CU (reset by the last one)
  int tokens;         // free weight-stream tokens (16 KiB in transit each) of this CU
  int hseen[8];       // per hint kind: highest layer + 1 this CU has seen complete
  int hpoll[8];       // per hint kind: 1 while one wave of this CU polls the global counters
  int flag_a, flag_b, att_done, abort_;
};
typedef ZLDS Ctl lctl;

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 lds16(const lbf* p) {
  const u32x4_t v = *(const ZLDS u32x4_t*)p;
  return uint4{v[0], v[1], v[2], v[3]};
}
__device__ __forceinline__ void lds16(lbf* p, uint4 v) { *(ZLDS u32x4_t*)p = u32x4_t{v.x, v.y, v.z, v.w}; }
__device__ __forceinline__ void lds8(lbf* p, uint32_t lo, uint32_t hi) { *(ZLDS u32x2_t*)p = u32x2_t{lo, hi}; }

template <int MR>
struct Lds {
  lbf* xln_a;   // [MR][D] LN1 rows (QKV input)
  lbf* xln_b;   // [MR][D] LN2 rows (FC1) / norm_f rows (HEADS)
  lbf* xraw_a;  // [MR][D] x_in of the layer (out_proj residual)
  lbf* xraw_b;  // [MR][D] x_mid of the layer (fc2 residual)
  lbf* win;     // [NCW][MR][1024] per-wave input slices (OUT, FC2)
  lfl* red;     // [NSLOT][8 parts][8 cols][MR]
  lfl* qs;      // [GQ][HD]
  lfl* sc;      // [GQ][pmax4]
  lbf* ks;      // [pmax4][HD]
  lbf* vs;      // [pmax4][HD]
  lctl* ctl;
  const ZLDS struct Args* args;          // the kernel arguments, copied at kernel start
  const ZLDS ZmiStepLayer* layers;       // the layer table, copied at kernel start
  const ZLDS int* row_pos;               // [MR]
  int pmax4;
};
constexpr int MAXL = 32;  // layer table capacity in LDS

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

struct Args;
constexpr size_t ARGS_LDS = 256;  // >= sizeof(Args), checked below
template <int MR>
__host__ __device__ inline size_t lds_bytes(int pmax4) {
  size_t b = align16(sizeof(Ctl)) + ARGS_LDS + align16(MAXL * sizeof(ZmiStepLayer)) + align16(MR * 4);
  b += 4 * align16((size_t)MR * D * 2);
  b += align16((size_t)NCW * MR * 1024 * 2);
  b += align16((size_t)NSLOT * 64 * MR * 4);
  b += align16((size_t)GQ * HD * 4);
  b += align16((size_t)GQ * pmax4 * 4);
  b += 2 * align16((size_t)pmax4 * HD * 2);
  return b;
}

template <int MR>
__device__ __forceinline__ Lds<MR> carve_lds(ZLDS char* smem, int pmax4) {
  Lds<MR> s;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    ZLDS char* p = smem + o;
    o += align16(bytes);
    return p;
  };
  // fixed offsets first (readable before pmax4 is known)
  s.ctl = (lctl*)take(sizeof(Ctl));
  s.args = (const ZLDS Args*)take(ARGS_LDS);
  s.layers = (const ZLDS ZmiStepLayer*)take(MAXL * sizeof(ZmiStepLayer));
  s.row_pos = (const ZLDS int*)take(MR * 4);
  s.xln_a = (lbf*)take((size_t)MR * D * 2);
  s.xln_b = (lbf*)take((size_t)MR * D * 2);
  s.xraw_a = (lbf*)take((size_t)MR * D * 2);
  s.xraw_b = (lbf*)take((size_t)MR * D * 2);
  s.win = (lbf*)take((size_t)NCW * MR * 1024 * 2);
  s.red = (lfl*)take((size_t)NSLOT * 64 * MR * 4);
  s.qs = (lfl*)take((size_t)GQ * HD * 4);
  s.sc = (lfl*)take((size_t)GQ * pmax4 * 4);
  s.ks = (lbf*)take((size_t)pmax4 * HD * 2);
  s.vs = (lbf*)take((size_t)pmax4 * HD * 2);
  s.pmax4 = pmax4;
  return s;
}

struct Args {
  const ZmiStepLayer* layers;
  const uint32_t* tasks;
  const int4* hdr;
  const bf16_t* x;
  const int* row_pos;
  const float* rope;
  const char* heads;
  const bf16_t *nf_w, *nf_b;
  float* logits;
  uint64_t* gran;
  uint32_t* ctl;
  unsigned long long* stamps;
  int L, smax, att_cus, pmax4, tokens;
  float eps, scale;
};
static_assert(sizeof(Args) <= ARGS_LDS, "Args must fit its LDS copy");

extern __shared__ __attribute__((aligned(16))) char zsmem[];
// the view every task function rebuilds from LDS (no pointer to the caller's stack: those are
// generic and every generic load would drain this wave's outstanding stores)
template <int MR>
__device__ __forceinline__ Lds<MR> lds_view() {
  ZLDS char* base = (ZLDS char*)zsmem;
  const ZLDS Args* a = (const ZLDS Args*)(base + align16(sizeof(Ctl)));
  return carve_lds<MR>(base, __builtin_amdgcn_readfirstlane(a->pmax4));
}

// ---------------------------------------------------------------------------- small helpers
__device__ __forceinline__ void gran_store(gu64* p, uint32_t tag, uint32_t v) {
  __hip_atomic_store(p, ((u64)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Buffer descriptors from wave-uniform bases: the readfirstlane makes the uniformity provable
// (pointers read through a reference are VGPRs to the compiler, which would otherwise wrap every
// buffer instruction in a waterfall loop).
__device__ __forceinline__ void* uni(const void* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (void*)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(uni(p), (short)0, __builtin_amdgcn_readfirstlane(bytes), FLAGS);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const gu64* p, int bytes) {
  return rsrc_of((const void*)(p), bytes);
}
__device__ __forceinline__ u32x4_t ld_sc1(__amdgpu_buffer_rsrc_t r, int voff) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 16 /* sc1 */);
}
__device__ __forceinline__ float sum8_lanes(float v) {  // as zmi_gemv8::sum8_lanes
  v += dpp_mov<DPP_XOR1>(v);
  v += dpp_mov<DPP_XOR2>(v);
  return v + dpp_mov<DPP_HALF_MIRROR>(v);
}
__device__ __forceinline__ int bcast(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Bounded spin: false (and the CU's abort flag set, the error word tagged) after SPIN_LIMIT.
// A CU runs 4 waves per SIMD and most of them wait most of the time: a short-sleep spin would
// take the issue slots the computing wave on the same SIMD needs. Waits on LDS state therefore
// sleep long (SLEEP_LDS x 64 clocks) and whoever changes that state issues s_wakeup, which ends
// the sleep of every wave of the workgroup; waits on global state (hint counters, granules:
// nothing on this CU can signal them) poll with a short sleep from one wave per CU.
constexpr int SLEEP_LDS = 16, SLEEP_GLOBAL = 2;
__device__ __forceinline__ void wake_all() { asm volatile("s_wakeup" ::: "memory"); }
struct Spin {
  unsigned long long t0;
  unsigned n;
};
template <int SLEEP = SLEEP_GLOBAL>
__device__ __forceinline__ bool spin_on(Spin& sp, lctl* c, uint32_t* ctl, uint32_t code) {
  __builtin_amdgcn_s_sleep(SLEEP);
  if ((++sp.n & 31) == 0) {
    if (__hip_atomic_load(&c->abort_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    if (sp.t0 == 0) {
      sp.t0 = now;
    } else if (now - sp.t0 > SPIN_LIMIT) {
      if ((threadIdx.x & 63) == 0) {
        __hip_atomic_fetch_or(((gu32*)(ctl + 2)), code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&c->abort_, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      return false;
    }
  }
  return true;
}

__device__ __forceinline__ bool wait_flag(lctl* c, const ZLDS int* flag, int want, uint32_t* ctl, uint32_t code) {
  Spin sp{0, 0};
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < want)
    if (!spin_on<SLEEP_LDS>(sp, c, ctl, code)) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return true;
}

__device__ __forceinline__ uint32_t tag_of(uint32_t epoch, int l, int sub) {
  return (epoch << 6) | ((uint32_t)l << 1) | (uint32_t)sub;
}

// Wait until counters h[0], h[HS], ... h[(n-1) HS] have all reached `target` (wrap-safe), i.e.
// layer `want - 1` of hint kind `kind` is complete. One wave per CU polls the global counters
// (lane i reads counter i); the CU's other waves wait on the LDS copy `hseen[kind]`.
__device__ __forceinline__ bool wait_hint(lctl* c, int kind, int want, const gu32* h, int n, uint32_t target,
                                       uint32_t* ctl, uint32_t code, int lane) {
  Spin sp{0, 0};
  for (;;) {
    if (__hip_atomic_load(&c->hseen[kind], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= want) return true;
    int won = 0;
    if (lane == 0) {
      int expect = 0;
      won = __hip_atomic_compare_exchange_strong(&c->hpoll[kind], &expect, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (bcast(won)) {
      bool ok = true;
      for (;;) {
        if (__hip_atomic_load(&c->hseen[kind], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= want) break;
        uint32_t v = target;
        if (lane < n) v = __hip_atomic_load(h + lane * HS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__all((int)(v - target) >= 0)) {
          if (lane == 0) __hip_atomic_fetch_max(&c->hseen[kind], want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          wake_all();
          break;
        }
        if (!spin_on(sp, c, ctl, code)) {
          ok = false;
          break;
        }
      }
      if (lane == 0) __hip_atomic_store(&c->hpoll[kind], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      wake_all();
      return ok;
    }
    if (!spin_on<SLEEP_LDS>(sp, c, ctl, code)) return false;
  }
}
__device__ __forceinline__ gu32* hint_at(const Gran& g, int units, int l, int k) {
  return g.hint + ((size_t)l * nhint(units) + k) * HS;
}
// one lane bumps a hint counter after this wave's granule stores have been issued (not drained:
// a hint that overtakes its granules costs the consumer one more sweep, never a wrong value)
__device__ __forceinline__ void bump(gu32* h, int lane) {
  if (lane == 0) __hip_atomic_fetch_add(h, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Weight-stream tokens. A CU's vector memory path serves its requests in order, so every byte a
// CU has issued and not yet received sits in front of its next hand-off load. Past ~64 KiB in
// transit a CU gains no bandwidth (MI355X_MICROARCH.md: ~24 GB/s per CU), only queueing: a
// wave takes a token before issuing its 16 KiB slice, waits for the slice to land (it has
// nothing else to do before its input arrives) and returns the token, so at most `tokens`
// slices are in transit per CU while every wave may hold a landed slice.
__device__ __forceinline__ bool take_token(lctl* c, uint32_t* ctl, int lane) {
  Spin sp{0, 0};
  for (;;) {
    int old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(&c->tokens, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    old = bcast(old);
    if (old > 0) return true;
    if (lane == 0) __hip_atomic_fetch_add(&c->tokens, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (!spin_on<SLEEP_LDS>(sp, c, ctl, 11u)) return false;
  }
}
__device__ __forceinline__ void give_token(lctl* c, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slice has landed
  if (lane == 0) __hip_atomic_fetch_add(&c->tokens, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  wake_all();
}

// a group of task type `type` finished on this CU; the CU's last one of the phase bumps the shard
__device__ __forceinline__ void group_done(lctl* c, int type, int n_on_cu, gu32* shard, int lane) {
  int old = 0;
  if (lane == 0)
    old = (int)__hip_atomic_fetch_add(&c->pdone[type], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  old = bcast(old);
  if (old == n_on_cu - 1 && lane == 0) {
    __hip_atomic_store(&c->pdone[type], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_add(shard, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ int groups_on(int total, int b, int nb) { return b < total ? (total - 1 - b) / nb + 1 : 0; }
__device__ __forceinline__ uint32_t shard_target(uint32_t epoch) { return epoch * (gridDim.x / 8); }

// Diagnostic build only (-DZMI_STEP_STAMPS, tools/step_stamps.py): lane 0 writes s_memrealtime (100 MHz)
// to stamps[(block, layer, k)]; the product kernel has none.
#ifdef ZMI_STEP_STAMPS
#define STEP_STAMP(a, l, k)                                                                         \
  do {                                                                                              \
    if ((a).stamps && (threadIdx.x & 63) == 0)                                                      \
      ((ZG unsigned long long*)(a).stamps)[((size_t)blockIdx.x * ((a).L + 1) + (l)) * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// per-task trace of workgroups 0..7: [block][wave][seq][8] after the per-layer stamps
#define STEP_TRACE(a, seq, k, v)                                                                       \
  do {                                                                                                \
    if ((a).stamps && blockIdx.x < 8 && (threadIdx.x & 63) == 0 && (seq) < 128)                        \
      ((ZG unsigned long long*)(a).stamps)[(size_t)gridDim.x * ((a).L + 1) * 16 +                     \
                 (((size_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * 128 + (seq)) * 8 + (k)] = (v);      \
  } while (0)
#define STEP_TICK(a, seq, k) STEP_TRACE(a, seq, k, __builtin_amdgcn_s_memrealtime())
#else
#define STEP_STAMP(a, l, k) \
  do {                      \
  } while (0)
#define STEP_TRACE(a, seq, k, v) \
  do {                           \
  } while (0)
#define STEP_TICK(a, seq, k) \
  do {                       \
  } while (0)
#endif

// ---------------------------------------------------------------------------- stager (wave 15)
// LayerNorm of MR rows exactly as zmi_gemv8's 256-thread prologue: "thread" c (0..255) owns the
// 8-element chunk c of each row; lane owns chunks lane + 64 w, w = that prologue's wave.
template <int MR>
__device__ __forceinline__ void ln_rows(const lbf* src, const bf16_t* gw, const bf16_t* gb, float eps, lbf* ln_out,
                                        int lane) {
  uint4 gv[4], bv[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const u32x4_t g4 = *(const ZG u32x4_t*)(gw + (lane + 64 * w) * 8);
    const u32x4_t b4 = *(const ZG u32x4_t*)(gb + (lane + 64 * w) * 8);
    gv[w] = uint4{g4[0], g4[1], g4[2], g4[3]};
    bv[w] = uint4{b4[0], b4[1], b4[2], b4[3]};
  }
#pragma unroll 1
  for (int m = 0; m < MR; ++m) {
    uint4 xv[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) xv[w] = lds16(src + m * D + (lane + 64 * w) * 8);
    float part[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t u[4] = {xv[w].x, xv[w].y, xv[w].z, xv[w].w};
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) t += bf2f(u[j]) + bf2f(u[j] >> 16);
      part[w] = wave_sum(0.f + t);
    }
    const float mean = (((part[0] + part[1]) + part[2]) + part[3]) / (float)D;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t u[4] = {xv[w].x, xv[w].y, xv[w].z, xv[w].w};
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d0 = bf2f(u[j]) - mean, d1 = bf2f(u[j] >> 16) - mean;
        t += d0 * d0 + d1 * d1;
      }
      part[w] = wave_sum(0.f + t);
    }
    const float ss = ((part[0] + part[1]) + part[2]) + part[3];
    const float rstd = 1.0f / sqrtf(ss / (float)D + eps), nbias = -mean * rstd;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int c = lane + 64 * w;
      uint32_t u[4] = {xv[w].x, xv[w].y, xv[w].z, xv[w].w};
      const uint32_t uw[4] = {gv[w].x, gv[w].y, gv[w].z, gv[w].w}, ub[4] = {bv[w].x, bv[w].y, bv[w].z, bv[w].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float y0 = (bf2f(u[j]) * rstd + nbias) * bf2f(uw[j]) + bf2f(ub[j]);
        const float y1 = (bf2f(u[j] >> 16) * rstd + nbias) * bf2f(uw[j] >> 16) + bf2f(ub[j] >> 16);
        u[j] = f2bf(y0) | (f2bf(y1) << 16);
      }
      lds16(ln_out + m * D + c * 8, uint4{u[0], u[1], u[2], u[3]});
    }
  }
}

// gather MR residual rows from the x granules (tag) into LDS rows dst[MR][D]
template <int MR>
__device__ __forceinline__ bool gather_x(lctl* c, const Gran& g, uint32_t tag, lbf* dst, uint32_t* ctl, int lane) {
  const __amdgpu_buffer_rsrc_t r = rsrc_of(g.xg, MR * (D / 2) * 8);
  Spin sp{0, 0};
  for (;;) {
    u32x4_t v[MR][4][2];
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
      for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int h = 0; h < 2; ++h) v[m][w][h] = ld_sc1(r, ((m * (D / 2) + (lane + 64 * w) * 4 + 2 * h) * 8));
    bool ok = true;
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
      for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int h = 0; h < 2; ++h) ok &= (v[m][w][h][1] == tag) & (v[m][w][h][3] == tag);
    if (__all(ok)) {
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int w = 0; w < 4; ++w)
          lds16(dst + m * D + (lane + 64 * w) * 8, uint4{v[m][w][0][0], v[m][w][0][2], v[m][w][1][0], v[m][w][1][2]});
      return true;
    }
    asm volatile("" ::: "memory");
    if (!spin_on(sp, c, ctl, 1u)) return false;
  }
}

// Stage k = 2 l + 0: QKV(l) input (layer 0: the step input written by the previous launch; later
// layers: the x_out(l-1) granules) -> x_in raw + LN1 rows, flag_a = l + 1.
// Stage k = 2 l + 1: FC1(l) input (x_mid(l) granules) -> x_mid raw + LN2 rows, flag_b = l + 1.
// Stage k = 2 L: x_out(L-1) -> norm_f rows, flag_b = L + 1. One call site per helper (code size).
template <int MR>
__device__ __forceinline__ void stager(uint32_t epoch, int lane) {
  const Lds<MR> s = lds_view<MR>();
  const ZLDS Args& a = *s.args;
  const Gran g = carve((uint64_t*)uni(a.gran), MR, gridDim.x);
  epoch = __builtin_amdgcn_readfirstlane(epoch);
#pragma unroll 1
  for (int k = 0; k <= 2 * a.L; ++k) {
    const int l = k >> 1;
    const bool second = (k & 1) != 0, last = k == 2 * a.L;
    // raw rows: x_in (out_proj residual), x_mid (fc2 residual); norm_f normalises in place
    lbf* raw = last ? s.xln_b : (second ? s.xraw_b : s.xraw_a);
    STEP_TICK(a, k, 0);
    STEP_TRACE(a, k, 6, (unsigned long long)l);
    STEP_TRACE(a, k, 7, (unsigned long long)(7 | (k << 8)));
    if (k == 0) {
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int w = 0; w < 4; ++w)
        {
          const u32x4_t v = *(const ZG u32x4_t*)(a.x + m * D + (lane + 64 * w) * 8);
          lds16(raw + m * D + (lane + 64 * w) * 8, uint4{v[0], v[1], v[2], v[3]});
        }
    } else {
      const uint32_t tag = second ? tag_of(epoch, l, 0) : tag_of(epoch, l - 1, 1);
      const gu32* h = hint_at(g, MR * HKV, second ? l : l - 1, second ? H_OUT : H_FC2);
      if (!wait_hint(s.ctl, second ? K_OUT : K_FC2, second ? l + 1 : l, h, 8, shard_target(epoch), a.ctl, 7u, lane))
        return;
      STEP_TICK(a, k, 1);
      if (!gather_x<MR>(s.ctl, g, tag, raw, a.ctl, lane)) return;
    }
    STEP_TICK(a, k, 2);
    STEP_STAMP(a, l, second ? 2 : 0);
    const bf16_t *gw, *gb;
    if (last) {
      gw = a.nf_w;
      gb = a.nf_b;
    } else {
      const ZLDS ZmiStepLayer& ly = s.layers[l];
      gw = (const bf16_t*)(second ? ly.ln2_w : ly.ln1_w);
      gb = (const bf16_t*)(second ? ly.ln2_b : ly.ln1_b);
    }
    ln_rows<MR>(raw, gw, gb, a.eps, second || last ? s.xln_b : s.xln_a, lane);
    __hip_atomic_store(second || last ? &s.ctl->flag_b : &s.ctl->flag_a, l + 1, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
    wake_all();
    STEP_STAMP(a, l, second ? 3 : 1);
    STEP_TICK(a, k, 4);
  }
}

// ---------------------------------------------------------------------------- GEMV tasks
// (W, NL) per phase = zmi_gemv8::shape8: K 2048 with LN -> (2, 16); out_proj (2048, no LN) -> (4, 8);
// fc2 (8192) -> (8, 16)
template <int KIND>
struct Phase {
  static constexpr int W = KIND == T_OUT ? 4 : (KIND == T_FC2 ? 8 : 2);
  static constexpr int NL = KIND == T_OUT ? 8 : 16;
  static constexpr int K = KIND == T_FC2 ? 8192 : 2048;
};

// this wave's input k-range of MR rows from granules (row stride row_words) into its LDS slice
template <int MR, int NL>
__device__ __forceinline__ bool sweep_slice(lctl* c, const gu64* src, int row_words, int g0, uint32_t tag,
                                            lbf* dst, uint32_t* ctl, int lane) {
  constexpr int PER = MR * NL / 4;  // 16-B loads per lane (2 granules each)
  const __amdgpu_buffer_rsrc_t r = rsrc_of(src, MR * row_words * 8);
  Spin sp{0, 0};
  for (;;) {
    u32x4_t v[PER];
#pragma unroll
    for (int t = 0; t < PER; ++t) {
      const int q = lane + 64 * t, m = q / (NL * 16), off = q - m * (NL * 16);
      v[t] = ld_sc1(r, (m * row_words + g0 + 2 * off) * 8);
    }
    bool ok = true;
#pragma unroll
    for (int t = 0; t < PER; ++t) ok &= (v[t][1] == tag) & (v[t][3] == tag);
    if (__all(ok)) {
#pragma unroll
      for (int t = 0; t < PER; ++t) {
        const int q = lane + 64 * t, m = q / (NL * 16), off = q - m * (NL * 16);
        lds8(dst + m * (NL * 64) + off * 4, v[t][0], v[t][2]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      return true;
    }
    asm volatile("" ::: "memory");
    if (!spin_on(sp, c, ctl, 2u)) return false;
  }
}

template <int MR, int KIND>
__device__ __forceinline__ bool gemv_task(uint32_t epoch, int l, int g, int wk, int slot, int wave, int lane, int seq) {
  const Lds<MR> s = lds_view<MR>();
  const ZLDS Args& a = *s.args;
  const Gran gr = carve((uint64_t*)uni(a.gran), MR, gridDim.x);
  epoch = __builtin_amdgcn_readfirstlane(epoch);
  l = __builtin_amdgcn_readfirstlane(l);
  g = __builtin_amdgcn_readfirstlane(g);
  wk = __builtin_amdgcn_readfirstlane(wk);
  slot = __builtin_amdgcn_readfirstlane(slot);
  wave = __builtin_amdgcn_readfirstlane(wave);
  seq = __builtin_amdgcn_readfirstlane(seq);
  STEP_TICK(a, seq, 0);
  using P = Phase<KIND>;
  constexpr int W = P::W, NL = P::NL, K = P::K, KC = K / 64;
  const ZLDS ZmiStepLayer* ly = s.layers + (KIND == T_HEADS ? 0 : l);
  const char* wp = KIND == T_QKV   ? (const char*)ly->qkv
                   : KIND == T_OUT ? (const char*)ly->out
                   : KIND == T_FC1 ? (const char*)ly->fc1
                   : KIND == T_FC2 ? (const char*)ly->fc2
                                   : a.heads;
  const int col0 = g * 8;
  const int et = lane;
  // epilogue operands that depend on nothing of this step (issued ahead of the weights)
  int q_pos = -1;
  float2 cs = {1.f, 0.f};
  if (KIND == T_QKV && et < 4 * MR) {
    q_pos = s.row_pos[et >> 2];
    const int n = col0 + (et & 3) * 2;
    if (n < QN + KVN && q_pos >= 0) {
      const int d = (n < QN ? n : n - QN) % HD;
      const ZG float* rp = (const ZG float*)a.rope + ((size_t)q_pos * (HD / 2) + (d >> 1)) * 2;
      cs = float2{rp[0], rp[1]};
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  if (!take_token(s.ctl, a.ctl, lane)) return false;
  const __amdgpu_buffer_rsrc_t wr = rsrc_of(wp + ((size_t)g * KC + wk * NL) * 1024, NL * 1024);
  u32x4_t wf[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) wf[j] = __builtin_amdgcn_raw_buffer_load_b128(wr, lane * 16, j * 1024, 2 /* nt */);
  __builtin_amdgcn_sched_barrier(0);
  give_token(s.ctl, lane);
  __builtin_amdgcn_sched_barrier(0);
  STEP_TICK(a, seq, 1);

  // input rows of this task's k-range
  const lbf* xrow[MR];
  if (KIND == T_QKV || KIND == T_FC1 || KIND == T_HEADS) {
    const ZLDS int* flag = KIND == T_QKV ? &s.ctl->flag_a : &s.ctl->flag_b;
    if (!wait_flag(s.ctl, flag, l + 1, a.ctl, 3u)) return false;
    const lbf* xs = KIND == T_QKV ? s.xln_a : s.xln_b;
#pragma unroll
    for (int m = 0; m < MR; ++m) xrow[m] = xs + m * K + wk * NL * 64 + (lane & 7) * 8;
  } else {
    lbf* dst = s.win + wave * MR * 1024;
    const gu64* src = KIND == T_OUT ? gr.ag : gr.hg;
    const int row_words = KIND == T_OUT ? QN / 2 : F / 2;
    const gu32* h = hint_at(gr, MR * HKV, l, KIND == T_OUT ? H_MERGED : H_FC1);
    if (!wait_hint(s.ctl, KIND == T_OUT ? K_MERGED : K_FC1, l + 1, h, 8, shard_target(epoch), a.ctl, 8u, lane))
      return false;
    if (!sweep_slice<MR, NL>(s.ctl, src, row_words, wk * NL * 32, tag_of(epoch, l, 0), dst, a.ctl, lane))
      return false;
#pragma unroll
    for (int m = 0; m < MR; ++m) xrow[m] = dst + m * (NL * 64) + (lane & 7) * 8;
  }
  STEP_TICK(a, seq, 2);
  if (KIND == T_OUT) STEP_STAMP(a, l, 7);
  if (KIND == T_FC1) STEP_STAMP(a, l, 8);
  if (KIND == T_FC2) STEP_STAMP(a, l, 9);
  if (KIND == T_QKV) STEP_STAMP(a, l, 11);

  // dot products (zmi_gemv8 step 4, verbatim order)
  float acc[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) acc[m] = 0.f;
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    uint4 xq[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) xq[m] = lds16(xrow[m] + j * 64);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float wlo = __uint_as_float(wf[j][i] << 16), whi = __uint_as_float(wf[j][i] & 0xffff0000u);
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const uint32_t u = i == 0 ? xq[m].x : (i == 1 ? xq[m].y : (i == 2 ? xq[m].z : xq[m].w));
        acc[m] = __builtin_fmaf(wlo, __uint_as_float(u << 16), acc[m]);
        acc[m] = __builtin_fmaf(whi, __uint_as_float(u & 0xffff0000u), acc[m]);
      }
    }
#pragma unroll
    for (int m = 0; m < MR; ++m) asm volatile("" : "+v"(acc[m]));
  }
  // partial of this part: [wk][8 cols][MR]
  lfl* red = s.red + slot * (64 * MR);
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    const float v = sum8_lanes(acc[m]);
    if ((lane & 7) == 0) red[(wk * 8 + (lane >> 3)) * MR + m] = v;
  }
  int old = 0;
  if (lane == 0)
    old = (int)__hip_atomic_fetch_add(&s.ctl->cnt[slot], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
  old = bcast(old);
  STEP_TICK(a, seq, 3);
  STEP_TRACE(a, seq, 6, (unsigned long long)l);
  STEP_TRACE(a, seq, 7, (unsigned long long)(KIND | (g << 8) | (old << 24)));
  if (old != W - 1) return true;
  if (lane == 0) __hip_atomic_store(&s.ctl->cnt[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  auto colsum = [&](int c, int m) {
    float v = red[c * MR + m];
#pragma unroll
    for (int w = 1; w < W; ++w) v += red[(w * 8 + c) * MR + m];
    return v;
  };

  // fused epilogues, one granule (2 bf16) per lane
  if (KIND == T_QKV) {
    if (et < 4 * MR) {
      const int m = et >> 2, c = (et & 3) * 2, n = col0 + c;
      float x0 = bfround(colsum(c, m)), x1 = bfround(colsum(c + 1, m));
      if (n < QN + KVN) {  // interleaved-pair RoPE on q and k (_torch.py:18-30)
        const float r0 = x0 * cs.x - x1 * cs.y;
        const float r1 = x1 * cs.x + x0 * cs.y;
        x0 = r0;
        x1 = r1;
      }
      const uint32_t packed = f2bf(x0) | (f2bf(x1) << 16);
      const uint32_t tag = tag_of(epoch, l, 0);
      if (n < QN) {
        gran_store(gr.qg + m * (QN / 2) + n / 2, tag, packed);
      } else {
        const int nn = n - QN;  // k: [0, 512), v: [512, 1024)
        gran_store(gr.kvg + m * KVN + nn / 2, tag, packed);
        if (q_pos >= 0) {  // KV cache write at this position (_torch.py:33-49)
          const bool is_k = nn < KVN;
          const int kk = is_k ? nn : nn - KVN, kh = kk / HD, d = kk - kh * HD;
          ZG bf16_t* cache = (ZG bf16_t*)(is_k ? ly->k_cache : ly->v_cache);
          *(ZG uint32_t*)(cache + (((size_t)m * HKV + kh) * a.smax + q_pos) * HD + d) = packed;
        }
      }
    }
  } else if (KIND == T_OUT || KIND == T_FC2) {
    if (et < 4 * MR) {  // x + bf16(linear(x))  (_torch.py:100-101)
      const int m = et >> 2, c = (et & 3) * 2, n = col0 + c;
      const lbf* xr = (KIND == T_OUT ? s.xraw_a : s.xraw_b) + m * D + n;
      const uint32_t res = *(const ZLDS uint32_t*)xr;
      const uint32_t y0 = f2bf(bf2f(res) + bfround(colsum(c, m)));
      const uint32_t y1 = f2bf(bf2f(res >> 16) + bfround(colsum(c + 1, m)));
      gran_store(gr.xg + m * (D / 2) + n / 2, tag_of(epoch, l, KIND == T_OUT ? 0 : 1), y0 | (y1 << 16));
    }
  } else if (KIND == T_FC1) {
    if (et < 2 * MR) {  // SwiGLU (_torch.py:150-152), V8 packing: cols 0..3 value, 4..7 gate
      const int m = et >> 1, cp = (et & 1) * 2;
      uint32_t hv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float y = bfround(colsum(cp + i, m));
        const float gt = bfround(colsum(cp + i + 4, m));
        const float sg = bfround(gt / (1.0f + expf(-gt)));
        hv[i] = f2bf(y * sg);
      }
      gran_store(gr.hg + m * (F / 2) + g * 2 + (et & 1), tag_of(epoch, l, 0), hv[0] | (hv[1] << 16));
    }
  } else {  // HEADS: 9 heads back to back, 1026 columns each
    if (et < 8 * MR) {
      const int m = et >> 3, c = et & 7, n = col0 + c;
      if (n < ZMI_NCB * ZMI_VOCAB) {
        const int cb = n / ZMI_VOCAB, vv = n - cb * ZMI_VOCAB;
        ((ZG float*)a.logits)[((size_t)m * ZMI_NCB + cb) * ZMI_VOCAB + vv] = bfround(colsum(c, m));
      }
    }
  }
  if (KIND != T_HEADS) {
    constexpr int H = KIND == T_QKV ? H_QKV : (KIND == T_OUT ? H_OUT : (KIND == T_FC1 ? H_FC1 : H_FC2));
    constexpr int G = KIND == T_QKV ? (QN + 2 * KVN) / 8 : (KIND == T_FC1 ? 2 * F / 8 : D / 8);
    group_done(s.ctl, KIND, groups_on(G, blockIdx.x, gridDim.x), hint_at(gr, MR * HKV, l, H + (blockIdx.x & 7)),
               lane);
  }
  STEP_TICK(a, seq, 4);
  if (KIND == T_FC2) STEP_STAMP(a, l, 10);
  if (KIND == T_QKV) STEP_STAMP(a, l, 12);
  if (KIND == T_FC1) STEP_STAMP(a, l, 13);
  if (KIND == T_OUT) STEP_STAMP(a, l, 14);
  return true;
}

// ---------------------------------------------------------------------------- attention task
// Unit u = (row r, kv head kvh); this CU is member j of the unit's att_cus CUs and owns positions
// j, j + att_cus, ... <= pos. GQA: the 4 query heads of kvh share every K/V row (_torch.py:136,
// SDPA scale 1/sqrt(128)). Partials (m, l, o) are published as granules; then every member merges
// its 512 / att_cus dims of the 4 heads over all members (fixed lane-tree order: deterministic).
template <int MR>
__device__ __forceinline__ bool att_task(uint32_t epoch, int l, int u, int j, int lane, int seq) {
  const Lds<MR> s = lds_view<MR>();
  const ZLDS Args& a = *s.args;
  const Gran gr = carve((uint64_t*)uni(a.gran), MR, gridDim.x);
  epoch = __builtin_amdgcn_readfirstlane(epoch);
  l = __builtin_amdgcn_readfirstlane(l);
  u = __builtin_amdgcn_readfirstlane(u);
  j = __builtin_amdgcn_readfirstlane(j);
  seq = __builtin_amdgcn_readfirstlane(seq);
  STEP_TICK(a, seq, 0);
  STEP_TRACE(a, seq, 6, (unsigned long long)l);
  STEP_TRACE(a, seq, 7, (unsigned long long)(T_ATT | (u << 8)));
  const int r = u / HKV, kvh = u - r * HKV, ncu = a.att_cus;
  // the previous layer's attention on this CU must be done with the LDS scratch
  if (!wait_flag(s.ctl, &s.ctl->att_done, l, a.ctl, 4u)) return false;
  const int pos = __builtin_amdgcn_readfirstlane(s.row_pos[r]);
  const ZLDS ZmiStepLayer& ly = s.layers[l];
  const uint32_t tag = tag_of(epoch, l, 0);
  const int np = (pos >= j) ? (pos - j) / ncu + 1 : 0;  // my positions, the last may be `pos`
  const bool own_new = np > 0 && (j + (np - 1) * ncu == pos);
  const int nhist = own_new ? np - 1 : np;
  const size_t kvbase = ((size_t)r * HKV + kvh) * a.smax * HD;
  // (1) history K/V rows -> LDS by DMA, 4 rows (1 KiB) per instruction
  if (!take_token(s.ctl, a.ctl, lane)) return false;
  {
    const int pl = lane >> 4;  // row within the 4-row piece
    for (int t = 0; t < (nhist + 3) / 4; ++t) {
      const int i = 4 * t + pl;
      const int p = i < nhist ? j + i * ncu : 0;
      const size_t off = kvbase + (size_t)p * HD + (lane & 15) * 8;
#pragma unroll
      for (int kv = 0; kv < 2; ++kv) {
        const bf16_t* src = reinterpret_cast<const bf16_t*>(kv ? ly.v_cache : ly.k_cache) + off;
        lbf* dstp = (kv ? s.vs : s.ks) + t * 4 * HD;
        const unsigned ldst = __builtin_amdgcn_readfirstlane((unsigned)(size_t)dstp);
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(src), "s"(ldst)
                     : "memory");
      }
    }
  }
  give_token(s.ctl, lane);
  STEP_TICK(a, seq, 1);
  if (pos < 0) {  // inactive row: zero output slice, nothing else to hand off
    const int dpc = (GQ * HD) / ncu;
    const int h = (j * dpc) / HD, d0 = (j * dpc) % HD;
    if (lane < dpc / 2) gran_store(gr.ag + r * (QN / 2) + ((kvh * GQ + h) * HD + d0) / 2 + lane, tag, 0u);
    if (lane == 0) __hip_atomic_store(&s.ctl->att_done, l + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    wake_all();
    bump(hint_at(gr, MR * HKV, l, H_ATT + u), lane);  // counts accumulate over launches: every path adds
    bump(hint_at(gr, MR * HKV, l, H_MERGED + (blockIdx.x & 7)), lane);
    return true;
  }
  // (2) q of the 4 heads (+ the new k/v row when this CU owns `pos`), granules
  if (!wait_hint(s.ctl, K_QKV, l + 1, hint_at(gr, MR * HKV, l, H_QKV), 8, shard_target(epoch), a.ctl, 9u, lane))
    return false;
  {
    const __amdgpu_buffer_rsrc_t rq = rsrc_of(gr.qg + r * (QN / 2) + kvh * GQ * (HD / 2), GQ * (HD / 2) * 8);
    const __amdgpu_buffer_rsrc_t rk = rsrc_of(gr.kvg + r * KVN + kvh * (HD / 2), (HD / 2) * 8);
    const __amdgpu_buffer_rsrc_t rv = rsrc_of(gr.kvg + r * KVN + (KVN / 2) + kvh * (HD / 2), (HD / 2) * 8);
    Spin sp{0, 0};
    for (;;) {
      const u32x4_t q0 = ld_sc1(rq, lane * 32), q1 = ld_sc1(rq, lane * 32 + 16);
      u32x4_t kn = {0u, tag, 0u, tag}, vn = {0u, tag, 0u, tag};
      if (own_new && lane < 32) {
        kn = ld_sc1(rk, lane * 16);
        vn = ld_sc1(rv, lane * 16);
      }
      const bool ok = (q0[1] == tag) & (q0[3] == tag) & (q1[1] == tag) & (q1[3] == tag) & (kn[1] == tag) &
                      (kn[3] == tag) & (vn[1] == tag) & (vn[3] == tag);
      if (__all(ok)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA rows have landed too
        const int h = lane >> 4, d = (lane & 15) * 8;     // 8 q values per lane
        const uint32_t qu[4] = {q0[0], q0[2], q1[0], q1[2]};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          s.qs[h * HD + d + 2 * i] = bf2f(qu[i]);
          s.qs[h * HD + d + 2 * i + 1] = bf2f(qu[i] >> 16);
        }
        if (own_new && lane < 32) {
          lds8(s.ks + (np - 1) * HD + lane * 4, kn[0], kn[2]);
          lds8(s.vs + (np - 1) * HD + lane * 4, vn[0], vn[2]);
        }
        break;
      }
      asm volatile("" ::: "memory");
      if (!spin_on(sp, s.ctl, a.ctl, 5u)) return false;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  STEP_STAMP(a, l, 4);
  STEP_TICK(a, seq, 2);
  // (3) scores: 4 lanes per key row (32 dims each), 16 rows per pass
  const int pm = s.pmax4;
  {
    const int qq = lane & 3;
    for (int i0 = 0; i0 < np; i0 += 16) {
      const int i = i0 + (lane >> 2);
      const int ic = i < np ? i : np - 1;
      const lbf* kr = s.ks + ic * HD + qq * 32;
      float dot[GQ] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
      for (int c = 0; c < 4; ++c) {
        const uint4 kv = lds16(kr + c * 8);
        const uint32_t uu[4] = {kv.x, kv.y, kv.z, kv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float k0 = bf2f(uu[e]), k1 = bf2f(uu[e] >> 16);
          const int d = qq * 32 + c * 8 + e * 2;
#pragma unroll
          for (int h = 0; h < GQ; ++h) dot[h] += s.qs[h * HD + d] * k0 + s.qs[h * HD + d + 1] * k1;
        }
      }
#pragma unroll
      for (int h = 0; h < GQ; ++h) {
        const float v = quad_sum(dot[h]);
        if (qq == 0 && i < np) s.sc[h * pm + i] = v * ATT_SCALE;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  // (4) local softmax statistics per head
  float mh[GQ], lh[GQ];
#pragma unroll
  for (int h = 0; h < GQ; ++h) {
    float m = -INFINITY;
    for (int i = lane; i < np; i += 64) m = fmaxf(m, s.sc[h * pm + i]);
    m = wave_max(m);
    float sum = 0.f;
    for (int i = lane; i < np; i += 64) {
      const float e = expf(s.sc[h * pm + i] - m);
      s.sc[h * pm + i] = e;
      sum += e;
    }
    mh[h] = m;
    lh[h] = wave_sum(sum);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  // (5) P.V: lane = dim pair
  float o[GQ][2];
#pragma unroll
  for (int h = 0; h < GQ; ++h) o[h][0] = o[h][1] = 0.f;
  for (int i = 0; i < np; ++i) {
    const uint32_t vv = *(const ZLDS uint32_t*)(s.vs + i * HD + 2 * lane);
    const float v0 = bf2f(vv), v1 = bf2f(vv >> 16);
#pragma unroll
    for (int h = 0; h < GQ; ++h) {
      const float p = s.sc[h * pm + i];
      o[h][0] += p * v0;
      o[h][1] += p * v1;
    }
  }
  // (6) publish this member's partial: pg[u][j][h] = {m, l, o[128]}
  gu64* rec = gr.pg + ((size_t)u * ncu + j) * GQ * REC;
#pragma unroll
  for (int h = 0; h < GQ; ++h) {
    gran_store(rec + h * REC + 2 + 2 * lane, tag, __float_as_uint(o[h][0]));
    gran_store(rec + h * REC + 3 + 2 * lane, tag, __float_as_uint(o[h][1]));
  }
  if (lane < GQ) {
    float m = mh[0], lsum = lh[0];
#pragma unroll
    for (int h = 1; h < GQ; ++h)
      if (lane == h) m = mh[h], lsum = lh[h];
    gran_store(rec + lane * REC, tag, __float_as_uint(m));
    gran_store(rec + lane * REC + 1, tag, __float_as_uint(lsum));
  }
  STEP_TICK(a, seq, 3);
  bump(hint_at(gr, MR * HKV, l, H_ATT + u), lane);
  // the LDS scratch is free again
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  STEP_STAMP(a, l, 5);
  if (lane == 0) __hip_atomic_store(&s.ctl->att_done, l + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  wake_all();

  // (7) merge my slice: dims [d0, d0 + dpc) of head hm, over all members jj (lpp lanes each,
  // 8 dims per lane)
  const int dpc = (GQ * HD) / ncu, lpp = 64 / ncu;
  const int hm = (j * dpc) / HD, d0 = (j * dpc) % HD;
  const int jj = lane / lpp, sub = lane - jj * lpp;
  // descriptor on the unit's (uniform) record base; the member index goes into the lane offset
  const __amdgpu_buffer_rsrc_t rm = rsrc_of(gr.pg + (size_t)u * ncu * GQ * REC, ncu * GQ * REC * 8);
  const int mo = (jj * GQ * REC + hm * REC) * 8;
  float mv = 0.f, lv = 0.f, ov[8];
  if (!wait_hint(s.ctl, K_ATT, l + 1, hint_at(gr, MR * HKV, l, H_ATT + u), 1, epoch * (uint32_t)ncu, a.ctl, 10u,
                 lane))
    return false;
  {
    Spin sp{0, 0};
    for (;;) {
      const u32x4_t ml = ld_sc1(rm, mo);
      u32x4_t ob[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) ob[t] = ld_sc1(rm, mo + (2 + d0 + sub * 8 + 2 * t) * 8);
      bool ok = (ml[1] == tag) & (ml[3] == tag);
#pragma unroll
      for (int t = 0; t < 4; ++t) ok &= (ob[t][1] == tag) & (ob[t][3] == tag);
      if (__all(ok)) {
        mv = __uint_as_float(ml[0]);
        lv = __uint_as_float(ml[2]);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          ov[2 * t] = __uint_as_float(ob[t][0]);
          ov[2 * t + 1] = __uint_as_float(ob[t][2]);
        }
        break;
      }
      asm volatile("" ::: "memory");
      if (!spin_on(sp, s.ctl, a.ctl, 6u)) return false;
    }
  }
  const float mmax = wave_max(mv);  // member 0 always holds position 0, so mmax is finite
  const float w = (mv == -INFINITY) ? 0.f : expf(mv - mmax);
  const float lw = wave_sum((sub == 0) ? w * lv : 0.f);
#pragma unroll
  for (int e = 0; e < 8; ++e) ov[e] *= w;
  // sum over members: lanes with equal `sub` (xor over the member bits)
  for (int msk = lpp; msk < 64; msk <<= 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) ov[e] += __shfl_xor(ov[e], msk);
  }
  if (jj == 0) {
    const float inv = 1.0f / lw;
    gu64* dst = gr.ag + r * (QN / 2) + ((kvh * GQ + hm) * HD + d0 + sub * 8) / 2;
#pragma unroll
    for (int e = 0; e < 4; ++e) gran_store(dst + e, tag, f2bf(ov[2 * e] * inv) | (f2bf(ov[2 * e + 1] * inv) << 16));
  }
  STEP_TICK(a, seq, 5);
  bump(hint_at(gr, MR * HKV, l, H_MERGED + (blockIdx.x & 7)), lane);
  STEP_STAMP(a, l, 6);
  STEP_TICK(a, seq, 4);
  return true;
}

// ---------------------------------------------------------------------------- the kernel
template <int MR>
__global__ __launch_bounds__(NT, 4) void step_kernel(const Args a) {
  const Lds<MR> s = carve_lds<MR>((ZLDS char*)zsmem, a.pmax4);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid < NSLOT) s.ctl->cnt[tid] = 0;
  if (tid < 8) {
    s.ctl->pdone[tid] = 0;
    s.ctl->hseen[tid] = 0;
    s.ctl->hpoll[tid] = 0;
  }
  if (tid == 0) {
    s.ctl->flag_a = 0;
    s.ctl->flag_b = 0;
    s.ctl->att_done = 0;
    s.ctl->abort_ = 0;
    s.ctl->tokens = a.tokens;
  }
  // kernel arguments, layer table and row positions into LDS (task functions read them there)
  if (tid < (int)(sizeof(Args) / 4)) ((ZLDS uint32_t*)s.args)[tid] = reinterpret_cast<const uint32_t*>(&a)[tid];
  for (int i = tid; i < a.L * (int)(sizeof(ZmiStepLayer) / 8); i += NT)
    ((ZLDS uint64_t*)s.layers)[i] = ((const ZG uint64_t*)a.layers)[i];
  if (tid < MR) ((ZLDS int*)s.row_pos)[tid] = ((const ZG int*)a.row_pos)[tid];
  __syncthreads();
  const uint32_t epoch = __builtin_amdgcn_readfirstlane(
      __hip_atomic_load(((gu32*)(a.ctl)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const Gran g = carve((uint64_t*)uni(a.gran), MR, gridDim.x);

  if (wave == NWAVES - 1) {
    stager<MR>(epoch, lane);
  } else {
    const int4 h = a.hdr[blockIdx.x];
    const int nlayer = a.L * h.y, total = nlayer + h.w;
    for (int i = wave; i < total; i += NCW) {
      int l;
      uint32_t t;
      if (i < nlayer) {
        l = i / h.y;
        t = a.tasks[h.x + i - l * h.y];
      } else {
        l = a.L;
        t = a.tasks[h.z + i - nlayer];
      }
      t = __builtin_amdgcn_readfirstlane(t);
      const int type = t & 7, wk = (t >> 3) & 15, grp = (t >> 7) & 8191, slot = (t >> 20) & 255;
      bool ok = true;
      const int seq = i / NCW;
      switch (type) {
        case T_QKV: ok = gemv_task<MR, T_QKV>(epoch, l, grp, wk, slot, wave, lane, seq); break;
        case T_ATT: ok = att_task<MR>(epoch, l, grp, slot, lane, seq); break;
        case T_OUT: ok = gemv_task<MR, T_OUT>(epoch, l, grp, wk, slot, wave, lane, seq); break;
        case T_FC1: ok = gemv_task<MR, T_FC1>(epoch, l, grp, wk, slot, wave, lane, seq); break;
        case T_FC2: ok = gemv_task<MR, T_FC2>(epoch, l, grp, wk, slot, wave, lane, seq); break;
        default: ok = gemv_task<MR, T_HEADS>(epoch, a.L, grp, wk, slot, wave, lane, seq); break;
      }
      if (!ok) break;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {  // the last workgroup out bumps the epoch (every workgroup has read it by then)
    const unsigned t = __hip_atomic_fetch_add(((gu32*)(a.ctl + 1)), 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      __hip_atomic_store(((gu32*)(a.ctl + 1)), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(((gu32*)(a.ctl)), epoch + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int MR>
int launch(const ZmiStepArgs* z, hipStream_t stream) {
  Args a;
  a.layers = z->layers;
  a.tasks = z->tasks;
  a.hdr = reinterpret_cast<const int4*>(z->task_hdr);
  a.x = (const bf16_t*)z->x;
  a.row_pos = z->row_pos;
  a.rope = z->rope;
  a.heads = (const char*)z->heads;
  a.nf_w = (const bf16_t*)z->nf_w;
  a.nf_b = (const bf16_t*)z->nf_b;
  a.logits = z->logits;
  a.gran = z->granules;
  a.ctl = z->ctl;
  a.stamps = (unsigned long long*)z->stamps;
  a.L = z->n_layer;
  a.smax = z->smax;
  a.att_cus = z->att_cus;
  a.pmax4 = (z->att_pmax + 3) & ~3;
  a.tokens = z->tokens > 0 ? z->tokens : 16;
  a.eps = z->eps;
  a.scale = 1.0f / sqrtf((float)HD);
  const size_t lds = lds_bytes<MR>(a.pmax4);
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(step_kernel<MR>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  ZMI_CHECK(attr);
  hipLaunchKernelGGL(step_kernel<MR>, dim3(z->n_blocks), dim3(NT), lds, stream, a);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

}  // namespace zmi_step

using namespace zmi_step;

extern "C" int64_t zmi_step_granule_words(int rows, int n_blocks, int n_layer) {
  return (int64_t)rows * (D / 2 + QN / 2 + KVN + QN / 2 + F / 2) + (int64_t)n_blocks * GQ * REC +
         (int64_t)n_layer * nhint(rows * HKV) * HS / 2;
}

extern "C" int64_t zmi_step_lds_bytes(int rows, int att_pmax) {
  const int p4 = (att_pmax + 3) & ~3;
  if (rows != 2) return -1;
  const size_t b = lds_bytes<2>(p4);
  return b <= 160 * 1024 ? (int64_t)b : -1;
}

extern "C" int zmi_step_blocks(int rows, int att_pmax) {
  const int64_t lds = zmi_step_lds_bytes(rows, att_pmax);
  if (lds < 0) return 0;
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(step_kernel<2>), hipFuncAttributeMaxDynamicSharedMemorySize,
                          160 * 1024) != hipSuccess)
    return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(step_kernel<2>), NT,
                                                   (size_t)lds) != hipSuccess)
    return 0;
  return per >= 1 ? cus : 0;
}

extern "C" int zmi_step_launch(const ZmiStepArgs* z, void* stream) {
  if (!z || !z->layers || !z->tasks || !z->task_hdr || !z->granules || !z->ctl)
    return zmi_fail_msg("step: null argument");
  if (z->n_blocks % 8) return zmi_fail_msg("step: n_blocks must be a multiple of 8 (hint shards)");
  if (z->n_blocks <= 0 || z->att_cus < 8 || 64 % z->att_cus != 0 || z->rows * HKV * z->att_cus != z->n_blocks)
    return zmi_fail_msg("step: n_blocks must equal rows * 4 * att_cus with att_cus in {8, 16, 32, 64}");
  if ((int64_t)z->att_pmax * z->att_cus < z->smax) return zmi_fail_msg("step: att_pmax * att_cus < smax");
  if (z->n_layer < 1 || z->n_layer > MAXL) return zmi_fail_msg("step: n_layer must be in [1, 32]");
  if (zmi_step_lds_bytes(z->rows, z->att_pmax) < 0) return zmi_fail_msg("step: configuration exceeds LDS");
  switch (z->rows) {
    case 2: return launch<2>(z, (hipStream_t)stream);
    default: return zmi_fail_msg("step: rows must be 2 (one CFG slot pair)");
  }
}
