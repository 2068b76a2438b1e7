// Many-row fc2 and out_proj (reference zonos/backbone/_torch.py:152 and :140, x = x + ... at :100-101) as
// split-K GEMMs: one workgroup per (64-column block, K segment of the GEMV's wave split: fc2 8 x 1024, out_proj
// 4 x 512), then a reduce that sums the segments in order and applies the residual epilogue (optionally also the
// next op's LayerNorm). Up to FUSED_MAX_ROWS rows (C5's 16-row steps) the reduce runs in the SAME launch: reduce
// workgroups appended to the grid (one per row) wait for every GEMM workgroup's arrival, then reduce their rows;
// beyond that (prefill) it is a second launch. Both give the same bits.
//
// Why: the GEMV form (zmi_gemv_impl.h, W = 8 waves each owning one K segment of a column group) re-reads the
// whole activation block [M][8192] once per column group; at 128 rows (C3's 64 slots) that is 2 MB per
// workgroup, 256 MB of L2 -> LDS traffic per launch, and the launch took 37 us for 33.6 MB of weights. Here
// a workgroup reads only its K segment of the rows (256 KB at 128 rows; 64 MB per launch), its 64 columns'
// weights for that segment once (128 KB, in registers), and keeps the GEMV's arithmetic: per wave (one 8-column
// group) and row tile of 16 rows, the MFMA chain over the segment's 16 chunks of 64 (k-half 0 and k-half 1 in
// two accumulators, summed with the same DPP move), stored as that segment's fp32 sum; the reduce adds the
// segments in K order (the GEMV's wave order) and applies x = bf16(x + bf16(sum)). A row's result is
// bit-identical to zmi_gemv_launch's for any M (tested).
#include <algorithm>

#include "zmi_common.h"
#include "zmi_kernels.h"
#include "zmi_gemv_impl.h"

namespace {

using zmi_gemv::dma_piece;
using zmi_gemv::ror8;

// K segments are the GEMV's wave segments: K = 8192 (fc2) W = 8 x 16 chunks, K = 2048 (out_proj) W = 4 x 8
template <int K>
struct Shape {
  static constexpr int NSEG = K == 8192 ? 8 : 4, KS = K / NSEG, NL = KS / 64, KC = K / 64;
  static constexpr int SROW = KS + 8;  // LDS row stride (bf16): bank-spread A reads
  static constexpr int TILE_BYTES = 16 * SROW * 2;
};
constexpr int NWV = 8, NT = NWV * 64;  // wave g = column group cb * 8 + g
constexpr int RT = 16;                 // rows per tile (one MFMA tile)
// `part` starts with PART_HDR floats of in-launch reduce state (zeroed once by the caller, re-armed by every fused
// launch): HDR_SHARDS words counting the GEMM workgroups' arrivals, sharded by block index % 8 (one shard per XCD under
// round-robin dispatch), each on its own 512-byte line (the adds to one line serialize at the memory side:
// with all eight words in one line the last arrival was seen 3.4 us after the last GEMM workgroup drained, at 16
// rows, tools/splitk_bench.py --stamps), then the reduce workgroups' ticket and the error word (a reduce workgroup
// gave up waiting), each on a line of its own. The fp32 segment sums follow.
constexpr int HDR_SHARDS = 8, HDR_LINE = 128;  // words per shard line
constexpr int HDR_TICKET = HDR_SHARDS * HDR_LINE, HDR_ERR = HDR_TICKET + HDR_LINE;
constexpr int PART_HDR = HDR_ERR + HDR_LINE;   // 1280 floats (5 KB; keeps the sums 16-byte aligned)
// in-launch reduce (ZMI_OPT_SPLITK_REDUCE = 1) up to 32 rows: beyond, the write-through partial stores (32 KB per GEMM workgroup at 128 rows) take
// longer to drain than a second launch costs (C3's 128-row fc2: 37.8 us fused against 25.4 for two launches)
constexpr int FUSED_MAX_ROWS = 32;
constexpr unsigned RED_SPIN = 1u << 22;

// Diagnostic build only (-DZMI_SPLITK_STAMPS, tools/splitk_bench.py): thread 0 of every workgroup writes
// s_memrealtime (100 MHz) at phase boundaries into a.diag[block][8].
#ifdef ZMI_SPLITK_STAMPS
#define ZMI_KSTAMP(i)                                                                                           \
  do {                                                                                                          \
    if (threadIdx.x == 0 && a.diag)                                                                             \
      reinterpret_cast<unsigned long long*>(a.diag)[(size_t)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define ZMI_KSTAMP(i) \
  do {                \
  } while (0)
#endif

struct RedArgs {  // the reduce's next-op LayerNorm (ln_w == nullptr: residual only)
  const bf16_t* ln_w;
  const bf16_t* ln_b;
  float eps;
  bf16_t* xn;
  int ldxn;
};

// a 16-byte sc1 load (buffer form, L1 bypassed: MI355X_MICROARCH.md "Valid forms", row 1) of another
// workgroup's write-through partial sums
__device__ __forceinline__ float4 ld_wt128(const __amdgpu_buffer_rsrc_t& r, unsigned off) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);  // cache policy 16 = sc1
  return float4{__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3])};
}

template <int NSEG, bool LN, bool INL>
__device__ void reduce_row(const ZmiGemvArgs& a, float* part, unsigned* hdr, int n_gemm, int m, const RedArgs& r,
                           char* smem);

template <int K, bool FUSED, bool LN>
__global__ __launch_bounds__(NT) void splitk_kernel(const ZmiGemvArgs a, float* part_base, int n_cb, const RedArgs r) {
  using S = Shape<K>;
  constexpr int NSEG = S::NSEG, KS = S::KS, NL = S::NL, KC = S::KC, SROW = S::SROW, TILE_BYTES = S::TILE_BYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  float* part = part_base + PART_HDR;
  unsigned* hdr = reinterpret_cast<unsigned*>(part_base);
  const int n_gemm = n_cb * NSEG;
  if (FUSED && b >= n_gemm) {
    reduce_row<NSEG, LN, true>(a, part, hdr, n_gemm, b - n_gemm, r, smem);
    return;
  }
  const int seg = b / n_cb, cb = b - seg * n_cb;  // consecutive blocks: one segment, neighbouring columns
  ZMI_KSTAMP(0);
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int g = cb * NWV + wave;
  const int M = a.M, N = a.N;
  const int n_rt = (M + RT - 1) / RT;
  bf16_t* tiles = reinterpret_cast<bf16_t*>(smem);  // two tile buffers
  const bf16_t* X = reinterpret_cast<const bf16_t*>(a.X) + (size_t)seg * KS;

  auto stage = [&](int rt, int buf) {  // the tile's rows of this segment, 1 KiB pieces spread over the waves
    const int row0 = rt * RT, rows = min(RT, M - row0);
    bf16_t* dst = tiles + (size_t)buf * (TILE_BYTES / 2);
    for (int pc = wave; pc < rows * (KS / 512); pc += NWV) {
      const int r = pc / (KS / 512), p = pc - r * (KS / 512);
      dma_piece(X + (size_t)(row0 + r) * a.ldx + p * 512 + lane * 8, dst + r * SROW + p * 512);
    }
  };
  stage(0, 0);
  // the wave's weights for this segment: group g, chunks seg * 16 .. + 15 (layout M8), all in flight
  const char* wbase = reinterpret_cast<const char*>(a.W) + ((size_t)g * KC + seg * NL) * 1024;
  const __amdgpu_buffer_rsrc_t wrsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wbase), (short)0, NL * 1024, 0x00020000);
  u32x4_t wf[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) wf[j] = __builtin_amdgcn_raw_buffer_load_b128(wrsrc, lane * 16, j * 1024, 2);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NL) : "memory");  // the first tile's pieces (issued before)
  for (int rt = 0; rt < n_rt; ++rt) {
    __syncthreads();  // tile rt landed for every wave's pieces; buffer rt + 1 is free
    if (rt + 1 < n_rt) stage(rt + 1, (rt + 1) & 1);
    const int row0 = rt * RT, rows = min(RT, M - row0);
    const bf16_t* xs = tiles + (size_t)(rt & 1) * (TILE_BYTES / 2);
    f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    const int ar = min(lane & 15, rows - 1);
    const bf16_t* xa = xs + ar * SROW + (lane >> 4) * 8;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const uint4 x0 = *reinterpret_cast<const uint4*>(xa + j * 64);
      const uint4 x1 = *reinterpret_cast<const uint4*>(xa + j * 64 + 32);
      const bf16x8_t wv = __builtin_bit_cast(bf16x8_t, wf[j]);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x0), wv, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, x1), wv, acc1, 0, 0, 0);
    }
    // segment sum = k-half 0 (tile columns 0..7) + k-half 1 (columns 8..15 moved down): element q of lane l
    // is row 4 (l >> 4) + q, column l & 15
    const int c = lane & 15, rb = (lane >> 4) * 4;
    if (FUSED) {
      // the tile's [16 rows][64 columns] sums staged in LDS, then stored write-through (sc1) as 16-byte pieces, one
      // per lane of waves 0..3: 4-byte write-through stores would each be a fabric write of their own
      float* st = reinterpret_cast<float*>(smem + 2 * (size_t)TILE_BYTES);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float v = acc0[q] + ror8(acc1[q]);
        if (c < 8) st[(rb + q) * 64 + wave * 8 + c] = v;
      }
      __syncthreads();
      if (wave < 4) {
        const int rr = wave * 4 + (lane >> 4), c4 = (lane & 15) * 4;
        if (rr < rows) {
          const float4 v = *reinterpret_cast<const float4*>(st + rr * 64 + c4);
          const u32x4_t u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
          const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
              part + ((size_t)seg * M + row0 + rr) * N + cb * 64, (short)0, 256, 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b128(u, prs, c4 * 4, 0, 16);  // cache policy 16 = sc1
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float v = acc0[q] + ror8(acc1[q]);
        if (c < 8 && rb + q < rows) part[((size_t)seg * M + row0 + rb + q) * N + g * 8 + c] = v;
      }
    }
    if (rt + 1 < n_rt) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next tile's pieces
  }
  ZMI_KSTAMP(1);
  if (FUSED) {  // every wave's partial stores drained, then one lane signals this workgroup's arrival
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ZMI_KSTAMP(2);
    if (t == 0)
      __hip_atomic_fetch_add(hdr + (b & (HDR_SHARDS - 1)) * HDR_LINE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Reduce workgroup m: row m. Lanes 0..7 of wave 0 poll the eight arrival shards together (sc1 loads, with sleeps:
// pollers beside the GEMM's weight stream) until every GEMM workgroup has published; the segment sums are then read
// with sc1 loads, 4 columns per thread (all 512 threads: the row's 8 x 8 KB of fc2 sums in one round of loads).
// Arithmetic per element: splitk_reduce_kernel's (segments added in K order, x + bf16(sum)); the LayerNorm runs on
// the new row staged in LDS with splitk_reduce_ln_kernel's structure (wave q = part q, lane L's 8 columns at
// q 512 + 8 L), so the bits equal the two-launch form's. The last reduce workgroup re-arms the counters for the
// next launch (stream order: no launch of this buffer overlaps).
template <int NSEG, bool LN, bool INL>
__device__ void reduce_row(const ZmiGemvArgs& a, float* part, unsigned* hdr, int n_gemm, int m, const RedArgs& r,
                           char* smem) {
  constexpr int NQ = 4;
  float(&ps)[2][NQ] = *reinterpret_cast<float(*)[2][NQ]>(smem);
  unsigned* flag = reinterpret_cast<unsigned*>(smem + 64);
  bf16_t* xrow = reinterpret_cast<bf16_t*>(smem + 128);  // the new row (LN): 2048 bf16
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int M = a.M, N = a.N;
  ZMI_KSTAMP(4);
  if (INL && wave == 0) {
    const unsigned want = lane < HDR_SHARDS ? (unsigned)((n_gemm - lane + HDR_SHARDS - 1) / HDR_SHARDS) : 0u;
    unsigned* mine = hdr + (lane < HDR_SHARDS ? lane : 0) * HDR_LINE;
    for (unsigned spins = 0;; ++spins) {
      const unsigned v = lane < HDR_SHARDS ? __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      if (__all(v >= want)) break;
      if (spins > RED_SPIN) {
        if (lane == 0) __hip_atomic_store(hdr + HDR_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  ZMI_KSTAMP(5);
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
      part, (short)0, (int)min((size_t)NSEG * M * N * 4, (size_t)0x7fffffff), 0x00020000);
  bf16_t* orow = reinterpret_cast<bf16_t*>(a.out) + (size_t)m * a.ldo;
  for (int e0 = 4 * t; e0 < N; e0 += 4 * NT) {  // columns e0 .. e0 + 3: bf16(x + bf16(sum of segments))
    float4 pv[NSEG];
#pragma unroll
    for (int sg = 0; sg < NSEG; ++sg) pv[sg] = ld_wt128(prs, (unsigned)((((size_t)sg * M + m) * N + e0) * 4));
    const uint2 xv = *reinterpret_cast<const uint2*>(orow + e0);
    float v0 = pv[0].x, v1 = pv[0].y, v2 = pv[0].z, v3 = pv[0].w;
#pragma unroll
    for (int sg = 1; sg < NSEG; ++sg) {
      v0 += pv[sg].x;
      v1 += pv[sg].y;
      v2 += pv[sg].z;
      v3 += pv[sg].w;
    }
    const uint2 nx = uint2{f2bf(bf2f(xv.x) + bfround(v0)) | (f2bf(bf2f(xv.x >> 16) + bfround(v1)) << 16),
                           f2bf(bf2f(xv.y) + bfround(v2)) | (f2bf(bf2f(xv.y >> 16) + bfround(v3)) << 16)};
    *reinterpret_cast<uint2*>(orow + e0) = nx;
    if (LN) *reinterpret_cast<uint2*>(xrow + e0) = nx;
  }
  ZMI_KSTAMP(6);
  if (LN) {  // N = 2048: wave q < 4, lane L owns columns q 512 + 8 L .. + 7 (zmi_layernorm_rows' part q)
    __syncthreads();
    const int q = wave & 3, e0 = q * 512 + lane * 8;
    const uint4 nx = *reinterpret_cast<const uint4*>(xrow + e0);
    const float s1 = wave_sum(ln_chunk_sum(nx, 0.f, false));
    if (lane == 0 && wave < 4) ps[0][q] = s1;
    __syncthreads();
    const float mean = ln_combine<NQ>(ps[0]) / (float)N;
    const float s2 = wave_sum(ln_chunk_sum(nx, mean, true));
    if (lane == 0 && wave < 4) ps[1][q] = s2;
    __syncthreads();
    const float rstd = 1.0f / sqrtf(ln_combine<NQ>(ps[1]) / (float)N + r.eps), nbias = -mean * rstd;
    if (wave < 4) {
      const uint4 gw = *reinterpret_cast<const uint4*>(r.ln_w + e0), gb = *reinterpret_cast<const uint4*>(r.ln_b + e0);
      *reinterpret_cast<uint4*>(r.xn + (size_t)m * r.ldxn + e0) = ln_apply(nx, gw, gb, rstd, nbias);
    }
  }
  ZMI_KSTAMP(7);
  // the last reduce workgroup re-arms the arrival shards (every reduce workgroup has passed its wait by then)
  if (INL && zmi_last_arriver_wt(hdr + HDR_TICKET, (unsigned)M, flag) && t < HDR_SHARDS)
    __hip_atomic_store(hdr + t * HDR_LINE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The same reduce as its own launch (after the GEMM launch; plain loads would do, the sc1 ones cost the same):
// one 512-thread workgroup per row, 4 columns per thread, the LayerNorm on the row staged in LDS.
template <int NSEG, bool LN>
__global__ __launch_bounds__(NT) void splitk_reduce_row_kernel(const ZmiGemvArgs a, float* part, const RedArgs r) {
  __shared__ __attribute__((aligned(16))) char smem[128 + 2048 * 2];
  reduce_row<NSEG, LN, false>(a, part, nullptr, 0, blockIdx.x, r, smem);
}

// x[m][n] = bf16(x + bf16(sum over the segments in order)), the GEMV's EPI_RESIDUAL epilogue
template <int NSEG>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* part, int M, int N, bf16_t* out, int ldo) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)M * N) return;
  const size_t m = i / N, n = i - m * N;
  float v = part[i];
#pragma unroll
  for (int s = 1; s < NSEG; ++s) v += part[(size_t)s * M * N + i];
  bf16_t* o = out + m * ldo + n;
  *o = (bf16_t)f2bf(bf2f(*o) + bfround(v));
}

// The same reduce + residual for rows of 2048 columns, then the LayerNorm of each new row into `xn` (the next
// op's prologue, zmi_layernorm_rows' arithmetic: part q = wave q, lane L's chunk at q 512 + 8 L, parts combined
// (p0 + p1) + (p2 + p3), two passes): one 4-wave workgroup per row, so the next layer's LayerNorm pre-pass launch
// is not needed.
template <int NSEG>
__global__ __launch_bounds__(256) void splitk_reduce_ln_kernel(const float* part, int M, bf16_t* out, int ldo,
                                                               const bf16_t* lw, const bf16_t* lb, float eps,
                                                               bf16_t* xn, int ldn) {
  constexpr int N = 2048, NQ = ln_parts(N);
  static_assert(NQ == 4, "one wave per LayerNorm part");
  __shared__ float ps[2][NQ];
  const int m = blockIdx.x, t = threadIdx.x, lane = t & 63, q = t >> 6;
  const int e0 = q * 512 + lane * 8;
  bf16_t* orow = out + (size_t)m * ldo;
  const uint4 xv = *reinterpret_cast<const uint4*>(orow + e0);
  const uint4 gw = *reinterpret_cast<const uint4*>(lw + e0), gb = *reinterpret_cast<const uint4*>(lb + e0);
  float4 pv[NSEG][2];
#pragma unroll
  for (int s = 0; s < NSEG; ++s) {
    const float* pr = part + ((size_t)s * M + m) * N + e0;
    pv[s][0] = *reinterpret_cast<const float4*>(pr);
    pv[s][1] = *reinterpret_cast<const float4*>(pr + 4);
  }
  const uint32_t xu[4] = {xv.x, xv.y, xv.z, xv.w};
  uint32_t nu[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float v0 = j < 2 ? (j == 0 ? pv[0][0].x : pv[0][0].z) : (j == 2 ? pv[0][1].x : pv[0][1].z);
    float v1 = j < 2 ? (j == 0 ? pv[0][0].y : pv[0][0].w) : (j == 2 ? pv[0][1].y : pv[0][1].w);
#pragma unroll
    for (int s = 1; s < NSEG; ++s) {
      v0 += j < 2 ? (j == 0 ? pv[s][0].x : pv[s][0].z) : (j == 2 ? pv[s][1].x : pv[s][1].z);
      v1 += j < 2 ? (j == 0 ? pv[s][0].y : pv[s][0].w) : (j == 2 ? pv[s][1].y : pv[s][1].w);
    }
    nu[j] = f2bf(bf2f(xu[j]) + bfround(v0)) | (f2bf(bf2f(xu[j] >> 16) + bfround(v1)) << 16);
  }
  const uint4 nx = uint4{nu[0], nu[1], nu[2], nu[3]};
  *reinterpret_cast<uint4*>(orow + e0) = nx;
  const float s1 = wave_sum(ln_chunk_sum(nx, 0.f, false));
  if (lane == 0) ps[0][q] = s1;
  __syncthreads();
  const float mean = ln_combine<NQ>(ps[0]) / (float)N;
  const float s2 = wave_sum(ln_chunk_sum(nx, mean, true));
  if (lane == 0) ps[1][q] = s2;
  __syncthreads();
  const float rstd = 1.0f / sqrtf(ln_combine<NQ>(ps[1]) / (float)N + eps), nbias = -mean * rstd;
  *reinterpret_cast<uint4*>(xn + (size_t)m * ldn + e0) = ln_apply(nx, gw, gb, rstd, nbias);
}

}  // namespace

extern "C" int zmi_gemv_splitk_layout(int which) { return which == 0 ? PART_HDR : (which == 1 ? HDR_ERR : -1); }

extern "C" int64_t zmi_gemv_splitk_floats(int M, int N) {
  return M <= 0 || N <= 0 ? -1 : PART_HDR + (int64_t)8 * M * N;
}

namespace {
template <int K, bool FUSED, bool LN>
hipError_t launch_gemm(const ZmiGemvArgs& a, float* part_base, int n_cb, int n_red, const RedArgs& r, hipStream_t s) {
  // two activation tiles, then (fused) the [16][64] f32 staging tile of the write-through partial stores; the
  // reduce workgroups reuse the front for their row (4 KB) and LayerNorm sums
  const size_t lds = 2 * (size_t)Shape<K>::TILE_BYTES + (FUSED ? 16 * 64 * 4 : 0);
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&splitk_kernel<K, FUSED, LN>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((splitk_kernel<K, FUSED, LN>), dim3(n_cb * Shape<K>::NSEG + n_red), dim3(NT), lds, s, a, part_base,
                     n_cb, r);
  return hipGetLastError();
}

template <int K>
int launch_splitk(const ZmiGemvArgs& a, float* part_base, const void* ln_w, const void* ln_b, float eps, void* xn,
                  int ldxn, hipStream_t s) {
  using S = Shape<K>;
  const int n_cb = a.N / (8 * NWV);
  const RedArgs r{(const bf16_t*)ln_w, (const bf16_t*)ln_b, eps, (bf16_t*)xn, ldxn};
  const int form = zmi_option(ZMI_OPT_SPLITK_REDUCE);
  if (a.M <= FUSED_MAX_ROWS && form == 1) {  // reduce in the same launch
    const int n_red = a.M;  // one reduce workgroup per row
    const hipError_t e = ln_w ? launch_gemm<K, true, true>(a, part_base, n_cb, n_red, r, s)
                              : launch_gemm<K, true, false>(a, part_base, n_cb, n_red, r, s);
    ZMI_CHECK(e);
    return 0;
  }
  ZMI_CHECK((launch_gemm<K, false, false>(a, part_base, n_cb, 0, r, s)));
  float* part = part_base + PART_HDR;
  if (form == 2 && a.N == 2048) {  // one 512-thread workgroup per row
    if (ln_w)
      hipLaunchKernelGGL((splitk_reduce_row_kernel<S::NSEG, true>), dim3(a.M), dim3(NT), 0, s, a, part, r);
    else
      hipLaunchKernelGGL((splitk_reduce_row_kernel<S::NSEG, false>), dim3(a.M), dim3(NT), 0, s, a, part, r);
  } else if (ln_w) {
    hipLaunchKernelGGL(splitk_reduce_ln_kernel<S::NSEG>, dim3(a.M), dim3(256), 0, s, part, a.M, (bf16_t*)a.out, a.ldo,
                       (const bf16_t*)ln_w, (const bf16_t*)ln_b, eps, (bf16_t*)xn, ldxn);
  } else {
    const size_t total = (size_t)a.M * a.N;
    hipLaunchKernelGGL(splitk_reduce_kernel<S::NSEG>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, part, a.M,
                       a.N, (bf16_t*)a.out, a.ldo);
  }
  ZMI_CHECK(hipGetLastError());
  return 0;
}
}  // namespace

extern "C" int zmi_gemv_splitk_ln(const ZmiGemvArgs* args, int epi, float* part, int64_t part_floats, const void* ln_w,
                                  const void* ln_b, float eps, void* xn, int ldxn, void* stream) {
  const ZmiGemvArgs& a = *args;
  if (ln_w && (!ln_b || !xn || a.N != 2048 || ldxn < 2048 || ldxn % 8 || a.ldo % 8))
    return zmi_fail_msg("gemv_splitk_ln: the fused LayerNorm needs N = 2048, ln_b, xn (ldxn % 8) and ldo % 8");
  if (epi != ZMI_EPI_RESIDUAL) return zmi_fail_msg("gemv_splitk: EPI_RESIDUAL only");
  if ((a.K != 8192 && a.K != 2048) || a.ln_w || a.pro != ZMI_PRO_AUTO)
    return zmi_fail_msg("gemv_splitk: plain K = 8192 (fc2) or 2048 (out_proj) only");
  if (a.N % (8 * NWV) || a.n_valid != a.N) return zmi_fail_msg("gemv_splitk: N a multiple of 64, unpadded");
  if (a.M < 1 || a.ldx % 8 || a.ldo < a.N || a.ldo % 8) return zmi_fail_msg("gemv_splitk: rows / strides");
  const int nseg = a.K == 8192 ? Shape<8192>::NSEG : Shape<2048>::NSEG;
  if (!part || part_floats < PART_HDR + (int64_t)nseg * a.M * a.N)
    return zmi_fail_msg("gemv_splitk: partial buffer too small (zmi_gemv_splitk_floats)");
  hipStream_t s = (hipStream_t)stream;
  return a.K == 8192 ? launch_splitk<8192>(a, part, ln_w, ln_b, eps, xn, ldxn, s)
                     : launch_splitk<2048>(a, part, ln_w, ln_b, eps, xn, ldxn, s);
}

extern "C" int zmi_gemv_splitk(const ZmiGemvArgs* args, int epi, float* part, int64_t part_floats, void* stream) {
  return zmi_gemv_splitk_ln(args, epi, part, part_floats, nullptr, nullptr, 0.f, nullptr, 0, stream);
}
