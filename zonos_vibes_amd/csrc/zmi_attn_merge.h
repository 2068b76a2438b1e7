// Attention chunk partials and their merge (zmi_attn.hip: the last-arriving chunk of a query merges).
//
// A query's keys are cut into chunks of CH keys; a 512-key softmax block (the reference CPU
// kernel's kvSplitSize) is CPB chunks. Chunk c of unit u (= query row x kv head) leaves, per
// query head g of the group:
//   o[u][c][g][0..128)  = sum over the chunk's keys of P_k V_k     (fp32)
//   lm[u][c][g]         = {sum over the chunk's keys of e_k, M_j}   (fp32; M_j of the chunk's block)
// The merge is a fixed sequence of fp32 operations (independent of batch and scheduling):
//   per block: ob = o_c0 + o_c0+1 + ...,  lb = l_c0 + l_c0+1 + ...          (chunk order)
//   blocks:    acc = ob_0, l = lb_0;  then l = lb_j + exp(M_{j-1} - M_j) * l,
//              acc = acc * exp(M_{j-1} - M_j) + ob_j                        (reference recursion)
//   out = bf16(acc * (1 / l))
#pragma once
#include "zmi_common.h"

namespace zmi_attn {

constexpr int HD = 128;
constexpr int BLK = 512;  // kvSplitSize of the reference's CPU attention
#ifndef ZMI_ATTN_NWC
#define ZMI_ATTN_NWC 4
#endif
constexpr int NWC = ZMI_ATTN_NWC;  // waves per chunk workgroup (32 keys each); CH fixes the arithmetic
constexpr int CH = 32 * NWC;
constexpr int CPB = BLK / CH;

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float2 ld2(const float* p) { return *reinterpret_cast<const float2*>(p); }

// Merged output of dims d .. d+3 of query head g of one unit. o / lm point at the unit's chunk 0;
// g_heads = heads per kv head. Loads are issued for up to MG chunks at a time before any is used.
__device__ __forceinline__ float4 merge4(const float* o, const float* lm, int nc, int g, int d, int g_heads) {
  constexpr int MG = 8;
  const size_t os = (size_t)g_heads * HD, ls = (size_t)g_heads * 2;
  float4 acc = {0.f, 0.f, 0.f, 0.f}, ob = acc;
  float l = 0.f, lb = 0.f, mprev = 0.f, mb = 0.f;
  for (int c0 = 0; c0 < nc; c0 += MG) {
    float4 ov[MG];
    float2 lv[MG];
#pragma unroll
    for (int u = 0; u < MG; ++u) {
      const int cc = min(c0 + u, nc - 1);  // clamped loads past the end are never used
      ov[u] = ld4(o + cc * os + (size_t)g * HD + d);
      lv[u] = ld2(lm + cc * ls + (size_t)g * 2);
    }
#pragma unroll
    for (int u = 0; u < MG; ++u) {
      const int cc = c0 + u;
      if (cc >= nc) break;
      if (cc % CPB == 0) {  // first chunk of its block
        ob = ov[u];
        lb = lv[u].x;
        mb = lv[u].y;
      } else {
        ob.x += ov[u].x;
        ob.y += ov[u].y;
        ob.z += ov[u].z;
        ob.w += ov[u].w;
        lb += lv[u].x;
      }
      if (cc % CPB == CPB - 1 || cc == nc - 1) {  // block complete: fold it into the running sums
        if (cc < CPB) {
          acc = ob;
          l = lb;
        } else {
          const float et = expf(mprev - mb);
          l = lb + et * l;
          acc.x = acc.x * et + ob.x;
          acc.y = acc.y * et + ob.y;
          acc.z = acc.z * et + ob.z;
          acc.w = acc.w * et + ob.w;
        }
        mprev = mb;
      }
    }
  }
  const float r = 1.0f / l;
  return float4{acc.x * r, acc.y * r, acc.z * r, acc.w * r};
}

// merge4's arithmetic for dims d, d+1 (the same operations per element, so the same bits), MG chunks' loads in
// flight at a time
template <int MG>
__device__ __forceinline__ float2 merge2(const float* o, const float* lm, int nc, int g, int d, int g_heads) {
  const size_t os = (size_t)g_heads * HD, ls = (size_t)g_heads * 2;
  float2 acc = {0.f, 0.f}, ob = acc;
  float l = 0.f, lb = 0.f, mprev = 0.f, mb = 0.f;
  for (int c0 = 0; c0 < nc; c0 += MG) {
    float2 ov[MG], lv[MG];
#pragma unroll
    for (int u = 0; u < MG; ++u) {
      const int cc = min(c0 + u, nc - 1);  // clamped loads past the end are never used
      ov[u] = ld2(o + cc * os + (size_t)g * HD + d);
      lv[u] = ld2(lm + cc * ls + (size_t)g * 2);
    }
#pragma unroll
    for (int u = 0; u < MG; ++u) {
      const int cc = c0 + u;
      if (cc >= nc) continue;  // (a break here would index ov / lv dynamically: scratch)
      if (cc % CPB == 0) {
        ob = ov[u];
        lb = lv[u].x;
        mb = lv[u].y;
      } else {
        ob.x += ov[u].x;
        ob.y += ov[u].y;
        lb += lv[u].x;
      }
      if (cc % CPB == CPB - 1 || cc == nc - 1) {
        if (cc < CPB) {
          acc = ob;
          l = lb;
        } else {
          const float et = expf(mprev - mb);
          l = lb + et * l;
          acc.x = acc.x * et + ob.x;
          acc.y = acc.y * et + ob.y;
        }
        mprev = mb;
      }
    }
  }
  const float r = 1.0f / l;
  return float2{acc.x * r, acc.y * r};
}

// Chunks of the query at position pos (pos < 0: inactive row, 0 chunks).
__device__ __forceinline__ int chunks_of(int pos) { return pos < 0 ? 0 : pos / CH + 1; }

}  // namespace zmi_attn
