// Common device helpers for the Zonos MI355X (gfx950 / CDNA4) hot path.
//
// Numerics conventions (mirroring the reference's bf16 rounding points):
//   * every GEMM output is rounded to bf16 before any consumer sees it (nn.Linear in bf16),
//   * elementwise fp32 math is written without fused multiply-adds where the reference
//     evaluates separate tensor ops (the library is compiled with -ffp-contract=off),
//   * bf16 rounding is round-to-nearest-even.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;
typedef uint16_t f16_t;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

#define ZMI_WAVE 64

__device__ __forceinline__ float bf2f(uint32_t h) { return __uint_as_float((h & 0xffffu) << 16); }

// fp32 -> bf16 round-to-nearest-even: one v_cvt_pk_bf16_f32 on gfx950 (branch-free; the software
// form with its NaN test compiles to an exec-mask branch per element)
__device__ __forceinline__ uint32_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

// round-trip through bf16
__device__ __forceinline__ float bfround(float f) { return bf2f(f2bf(f)); }

__device__ __forceinline__ float h2f(uint32_t h) {
  _Float16 v = __builtin_bit_cast(_Float16, (uint16_t)(h & 0xffffu));
  return (float)v;
}
__device__ __forceinline__ uint32_t f2h(float f) {
  _Float16 v = (_Float16)f;
  return (uint32_t)__builtin_bit_cast(uint16_t, v);
}

// ---- cross-lane reductions on DPP (VALU-speed lane moves, no LDS round trip as ds_bpermute has).
// All lanes must be active. Each step pairs lanes symmetrically (a+b and b+a), so every lane of a
// 16-lane row ends with the bit-identical value; the wave total combines the four row values in a
// fixed order through readlane, so it is uniform too.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
constexpr int DPP_XOR1 = 0xB1;         // quad_perm [1,0,3,2]
constexpr int DPP_XOR2 = 0x4E;         // quad_perm [2,3,0,1]
constexpr int DPP_HALF_MIRROR = 0x141; // lane i <- 7-i within 8
constexpr int DPP_MIRROR = 0x140;      // lane i <- 15-i within 16

__device__ __forceinline__ float quad_sum(float v) {
  v += dpp_mov<DPP_XOR1>(v);
  return v + dpp_mov<DPP_XOR2>(v);
}
__device__ __forceinline__ float row16_sum(float v) {
  v = quad_sum(v);
  v += dpp_mov<DPP_HALF_MIRROR>(v);
  return v + dpp_mov<DPP_MIRROR>(v);
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_mov<DPP_XOR1>(v));
  v = fmaxf(v, dpp_mov<DPP_XOR2>(v));
  v = fmaxf(v, dpp_mov<DPP_HALF_MIRROR>(v));
  return fmaxf(v, dpp_mov<DPP_MIRROR>(v));
}
__device__ __forceinline__ float lane_read(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float wave_sum(float v) {
  v = row16_sum(v);
  return (lane_read(v, 0) + lane_read(v, 16)) + (lane_read(v, 32) + lane_read(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
  v = row16_max(v);
  return fmaxf(fmaxf(lane_read(v, 0), lane_read(v, 16)), fmaxf(lane_read(v, 32), lane_read(v, 48)));
}

// ---- LayerNorm row arithmetic (nn.LayerNorm, reference _torch.py:62,88,90), shared by the GEMV
// prologue (zmi_gemv_impl.h) and zmi_layernorm_rows so both give the same bits. A row of K elements
// is cut into ln_parts(K) contiguous parts, each reduced by one wave: lane L owns the 8-element
// chunks at q K / NQ + 8 (L + 64 i), i < K / (512 NQ); fp32 sums in chunk order, DPP wave sum per
// part, parts combined as (p0 + p1) + (p2 + p3). Two passes (mean, then squared deviations).
__host__ __device__ constexpr int ln_parts(int K) { return K >= 2048 ? 4 : (K >= 1024 ? 2 : 1); }
__device__ __forceinline__ float ln_chunk_sum(const uint4& xv, float mean, bool sq) {
  const uint32_t u[4] = {xv.x, xv.y, xv.z, xv.w};
  float t = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (sq) {
      const float d0 = bf2f(u[j]) - mean, d1 = bf2f(u[j] >> 16) - mean;
      t += d0 * d0 + d1 * d1;
    } else {
      t += bf2f(u[j]) + bf2f(u[j] >> 16);
    }
  }
  return t;
}
template <int NQ>
__device__ __forceinline__ float ln_combine(const float* p) {
  if (NQ == 4) return (p[0] + p[1]) + (p[2] + p[3]);
  if (NQ == 2) return p[0] + p[1];
  return p[0];
}
// y = bf16((x * rstd - mean * rstd) * w + b) on one 8-element chunk
__device__ __forceinline__ uint4 ln_apply(const uint4& xv, const uint4& gw, const uint4& gb, float rstd, float nbias) {
  uint32_t u[4] = {xv.x, xv.y, xv.z, xv.w};
  const uint32_t uw[4] = {gw.x, gw.y, gw.z, gw.w}, ub[4] = {gb.x, gb.y, gb.z, gb.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float y0 = (bf2f(u[j]) * rstd + nbias) * bf2f(uw[j]) + bf2f(ub[j]);
    const float y1 = (bf2f(u[j] >> 16) * rstd + nbias) * bf2f(uw[j] >> 16) + bf2f(ub[j] >> 16);
    u[j] = f2bf(y0) | (f2bf(y1) << 16);
  }
  return uint4{u[0], u[1], u[2], u[3]};
}

// splitmix64 finaliser (shared with zonos_vibes_amd/synthetic.py)
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// ---- inter-workgroup hand-off (cdna_hip_programming.md §6 Guideline 16 recipe) ----------
// Producer: all waves drained, barrier, one lane releases (agent) and bumps the ticket.
// Returns true in every thread of the block that drew the last ticket; that block then
// acquires (agent) before plain-loading the other blocks' slabs.
__device__ __forceinline__ bool zmi_last_arriver(unsigned* counter, unsigned total, unsigned* lds_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned last = (t == total - 1) ? 1u : 0u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm for next launch
    }
    *lds_flag = last;
  }
  __syncthreads();
  return *lds_flag != 0;
}

// Write-through variant (MI355X_MICROARCH.md "Valid forms", table row 1): every byte handed off is
// stored with an agent-scope relaxed atomic store (global_store ... sc1, drained by vmcnt(0) in every
// storing wave before the barrier), one lane bumps the ticket; the last arriver reads the slabs
// with agent-scope relaxed loads (sc1). No release/acquire fences, no L2 write-back.
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_wt64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt64(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Hand-offs between workgroups on ONE XCD (blocks 8 apart under the round-robin dealing zmi_xcd_dealing checks):
// with l2 (ZMI_OPT_XC_HANDOFF 0) a workgroup-scope store keeps the line in that XCD's L2, where the consumers'
// agent-scope (L2-served) polls or post-acquire loads find it, instead of writing it through to memory and dropping
// it from L2 (tools/hop_probe.hip: 228 against 449 ns per hop idle). Never across XCDs: such a store is not visible
// there until the kernel ends.
__device__ __forceinline__ void st_xc64(uint64_t* p, uint64_t v, int l2) {
  if (l2)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_xc(float* p, float v, int l2) {
  if (l2)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t pack_f2(float lo, float hi) {
  return (uint64_t)__float_as_uint(lo) | ((uint64_t)__float_as_uint(hi) << 32);
}
__device__ __forceinline__ float lo_f(uint64_t v) { return __uint_as_float((uint32_t)v); }
__device__ __forceinline__ float hi_f(uint64_t v) { return __uint_as_float((uint32_t)(v >> 32)); }
__device__ __forceinline__ void st_wt(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ int ld_wt(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ bool zmi_last_arriver_wt(unsigned* counter, unsigned total, unsigned* lds_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned last = (t == total - 1) ? 1u : 0u;
    if (last) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *lds_flag = last;
  }
  __syncthreads();
  return *lds_flag != 0;
}

#define ZMI_CHECK(expr)                                                   \
  do {                                                                      \
    hipError_t _e = (expr);                                                 \
    if (_e != hipSuccess) return zmi_fail(_e, #expr, __FILE__, __LINE__);   \
  } while (0)

int zmi_fail(hipError_t e, const char* what, const char* file, int line);
int zmi_fail_msg(const char* msg);
int zmi_option(int which);  // zmi_set_option knobs (zonos_hip.h ZMI_OPT_*)
int zmi_cu_count();         // CUs of the current device (cached)
