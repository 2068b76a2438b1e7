// Shared pieces of the persistent decode engines (zmi_engine.hip: zmi_ffn_engine, zmi_layer_engine):
// per-wave LDS-DMA weight rings, LDS arrival counters, granule gathers, the LayerNorm row of one wave.
#pragma once
#include "zmi_common.h"
#include "zmi_kernels.h"
#include "zmi_gemv_impl.h"

namespace zmi_eng {

using zmi_gemv::ror8;
typedef __attribute__((address_space(3))) unsigned lds_u32;

constexpr int SLOT = 8192;           // ring slot: 8 KiB = one K segment (8 chunks) of a K = 2048 column group
constexpr unsigned SPIN = 1u << 20;  // bounded spins (~30 ms with s_sleep 1), then the error word is set

__device__ __forceinline__ void give_up(unsigned* err) {
  __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ lds_u32* lds_word(char* smem, size_t off) {
  return reinterpret_cast<lds_u32*>((__attribute__((address_space(3))) char*)smem + off);
}

// LDS arrival: this wave's LDS writes, then one lane's add
__device__ __forceinline__ void lds_arrive(lds_u32* c, int lane) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if (lane == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_wait_ge(lds_u32* c, unsigned want, unsigned* err) {
  for (unsigned spin = 0; __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < want; ++spin) {
    if (spin > SPIN) {
      give_up(err);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// one 1 KiB LDS-DMA piece, non-temporal (lane-linear: lane l's 16 B land at lds + 16 l). Inline asm: the
// compiler does not count it; the consumer's own vmcnt waits do (cdna_hip_programming.md §5.7)
__device__ __forceinline__ void dma_nt(const char* g, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(lds)
               : "memory");
}

// one ring slot (8 contiguous KiB of a packed weight) into LDS at `lds` (wave-uniform)
__device__ __forceinline__ void issue_slot(const char* src, unsigned lds, int lane) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the slot have returned
  const char* g = src + lane * 16;
#pragma unroll
  for (int j = 0; j < 8; ++j) dma_nt(g + j * 1024, lds + j * 1024);
}

// a slot has landed when at most `after` x 8 DMA pieces (the slots issued after it) are outstanding: loads
// complete in order, so stores the wave issues in between only make the wait longer
__device__ __forceinline__ void wait_slot(int after) {
  if (after <= 0)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (after == 1)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (after == 2)
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
}

// one wave gathers 64 PER granules g[0 .. 64 PER) carrying `tag` into dst[0 .. 64 PER) (their low words)
template <int PER>
__device__ __forceinline__ void gather(const uint64_t* g, uint32_t* dst, uint32_t tag, int lane, unsigned* err) {
  uint32_t pend = PER >= 32 ? 0xffffffffu : ((1u << PER) - 1u);
  for (unsigned spin = 0;; ++spin) {
    uint64_t v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = ((pend >> i) & 1) ? ld_wt64(g + lane + 64 * i) : 0ull;
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (((pend >> i) & 1) && (uint32_t)(v[i] >> 32) == tag) {
        dst[lane + 64 * i] = (uint32_t)v[i];
        pend &= ~(1u << i);
      }
    if (__all(pend == 0)) break;
    if (spin > SPIN) {
      give_up(err);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// nn.LayerNorm of one 2048-element bf16 row in LDS, in place, by one wave: the GEMV LayerNorm prologue's
// arithmetic (zmi_common.h: 4 parts of 512, lane L's chunk 8 L of each part, part sums by wave_sum,
// (p0 + p1) + (p2 + p3), two passes)
__device__ __forceinline__ void ln_row(bf16_t* xr, const bf16_t* gw, const bf16_t* gb, float eps, int lane) {
  constexpr int NQ = 4, K = 2048;
  uint4 xv[NQ], gv[NQ], bv[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    gv[q] = *reinterpret_cast<const uint4*>(gw + q * 512 + lane * 8);
    bv[q] = *reinterpret_cast<const uint4*>(gb + q * 512 + lane * 8);
    xv[q] = *reinterpret_cast<const uint4*>(xr + q * 512 + lane * 8);
  }
  float part[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    float t = 0.f;
    t += ln_chunk_sum(xv[q], 0.f, false);
    part[q] = wave_sum(t);
  }
  const float mean = ln_combine<NQ>(part) / (float)K;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    float t = 0.f;
    t += ln_chunk_sum(xv[q], mean, true);
    part[q] = wave_sum(t);
  }
  const float rstd = 1.0f / sqrtf(ln_combine<NQ>(part) / (float)K + eps), nbias = -mean * rstd;
#pragma unroll
  for (int q = 0; q < NQ; ++q)
    *reinterpret_cast<uint4*>(xr + q * 512 + lane * 8) = ln_apply(xv[q], gv[q], bv[q], rstd, nbias);
}

// ln_row with the LayerNorm weight / bias chunks of the lane already in registers (gw[q] = w[q 512 + 8 lane ..])
__device__ __forceinline__ void ln_row_r(bf16_t* xr, const uint4 (&gv)[4], const uint4 (&bv)[4], float eps, int lane) {
  constexpr int NQ = 4, K = 2048;
  uint4 xv[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) xv[q] = *reinterpret_cast<const uint4*>(xr + q * 512 + lane * 8);
  float part[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    float t = 0.f;
    t += ln_chunk_sum(xv[q], 0.f, false);
    part[q] = wave_sum(t);
  }
  const float mean = ln_combine<NQ>(part) / (float)K;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    float t = 0.f;
    t += ln_chunk_sum(xv[q], mean, true);
    part[q] = wave_sum(t);
  }
  const float rstd = 1.0f / sqrtf(ln_combine<NQ>(part) / (float)K + eps), nbias = -mean * rstd;
#pragma unroll
  for (int q = 0; q < NQ; ++q)
    *reinterpret_cast<uint4*>(xr + q * 512 + lane * 8) = ln_apply(xv[q], gv[q], bv[q], rstd, nbias);
}

}  // namespace zmi_eng
