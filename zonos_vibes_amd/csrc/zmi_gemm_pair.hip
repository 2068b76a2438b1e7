// K-split pair form of the many-row K = 2048 GEMM (zmi_gemv_rows_pair; the engine's `rows_pair` route).
//
// out[m, n] = sum_k A[m, k] * W[n, k]  (nn.Linear, reference zonos/backbone/_torch.py:114-115,147-152; heads
// zonos/model.py:100-101), bit-identical to zmi_gemv_launch for every row: the same per-segment MFMA chains
// (4 segments of 512 k, two k-half accumulators each, 16 real columns per MFMA as the dense-pair rows form),
// the column sum ((s0 + s1) + s2) + s3 in segment order, then the same epilogue() (zmi_gemv_impl.h).
//
// Why: gemm_rows_kernel keeps a 64-column weight slice in registers (256 KB: half the CU's register file) and
// streams every row's 4 KB activation from L2 per 16-row tile; that read is at the guide's ceiling for rows every
// workgroup shares (66-73 GB/s per CU) and its two 64 KB tile buffers leave no room for a third. Here a unit of
// 128 columns is split over two workgroups by K: the upper one (segments 2, 3) reads only the upper 2 KB of each row,
// the lower one (segments 0, 1) the lower 2 KB, so each CU reads half of every row into 32 KB tiles, three of which
// fit. The upper workgroup hands its two fp32 segment sums per (row, column) to the lower one as one 8-byte
// write-through store and bumps a per-tile counter; the lower one folds them after its own and runs the epilogue.
// The upper workgroups take the lower block indices, so they are dispatched first and never wait: no grid size can
// deadlock the pair. Both of a pair sit on one XCD (indices `half` apart, `half` a multiple of 8).
#include "zmi_common.h"
#include "zmi_kernels.h"
#include "zmi_gemv_impl.h"

namespace {
using namespace zmi_gemv;

constexpr int GP_G = 16;                 // 8-column groups per unit (8 dense pairs)
constexpr int GP_XROW = 1024 + 8;        // a tile row: the workgroup's K half + 16 B of padding
constexpr int GP_NBUF = 3;               // tile buffers: the DMA of tile t + 3 goes out after tile t's barrier
constexpr size_t GP_TILE = (size_t)GR_RT * GP_XROW * 2;
constexpr size_t GP_RED = GP_NBUF * GP_TILE;                            // after the tile buffers
constexpr size_t GP_OPS = GP_RED + (size_t)GP_G * 2 * 8 * GR_RT * 4;    // segment sums [group][2][8][RT]
constexpr size_t GP_CNT = GP_OPS + (size_t)GP_NBUF * 4096;              // epilogue operands per buffer
constexpr size_t GP_LDS = GP_CNT + 16;
static_assert(GP_LDS <= 160 * 1024, "LDS");
constexpr unsigned GP_SPIN = 1u << 22;   // bounded wait for the partner's tile (never reached in a sound launch)

template <int EPI>
__global__ __launch_bounds__(1024) void gemm_pair_kernel(const ZmiGemvArgs a, int n_pb, int n_rt, int rpw, int half,
                                                         uint64_t* __restrict__ hp, unsigned* __restrict__ flags) {
  constexpr int NL = 8, RT = GR_RT, KC = 2048 / 64, XROW = GP_XROW, NE = 2;
  constexpr int NWV = 16, NDW = 8, PPW = RT * 2 / NDW;  // 32 pieces of 1 KiB per tile, 4 per DMA wave
  constexpr int EP = EPI == ZMI_EPI_RESIDUAL ? 4 : (EPI == ZMI_EPI_QKV ? 1 : 0);  // operand pieces per tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* xs = reinterpret_cast<bf16_t*>(smem);                // [NBUF][RT][XROW]
  float* red = reinterpret_cast<float*>(smem + GP_RED);         // [group][segment of the half][8][RT]
  char* ops = smem + GP_OPS;                                    // [NBUF][4 KiB]
  unsigned* cnt = reinterpret_cast<unsigned*>(smem + GP_CNT);   // epilogues (stores) finished
  const int b = blockIdx.x;
  const bool up = b < half;
  const int u = up ? b : b - half, idx = u >> 3;
  const int n_rg = (n_rt + rpw - 1) / rpw;
  const int pb = (idx / n_rg) * 8 + (u & 7), rg = idx - (idx / n_rg) * n_rg;
  if (pb >= n_pb) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ps = wave & 7, sk = wave >> 3;  // dense pair ps of the unit over segment sk of the half
  const int wk = (up ? 2 : 0) + sk;         // the segment in K
  const int ngroups = a.N >> 3;
  const int n_gl = min(GP_G, ngroups - pb * GP_G);  // live groups of the unit
  const int n_ew = (n_gl + 1) >> 1;                 // epilogue / store waves: wave w < n_ew owns groups 2w, 2w + 1
  const bool ew = wave < n_ew;
  const int t0 = rg * rpw, rt_end = min(n_rt, t0 + rpw);
  const int kh0 = up ? 1024 : 0;
  const bf16_t* X = reinterpret_cast<const bf16_t*>(a.X);
  const bool dw = wave >= NDW;
  const bool opw = !up && EP && wave == NWV - 1;
  if (tid == 0) *cnt = 0;
  volatile __attribute__((address_space(3))) unsigned* lcnt = (volatile __attribute__((address_space(3))) unsigned*)cnt;

  auto dma_tile = [&](int t) {
    if (!dw) return;
    bf16_t* dst = xs + (t % GP_NBUF) * RT * XROW;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave - NDW + NDW * i, r = pc >> 1, p = pc & 1;
      const int sr = min(t * RT + r, a.M - 1);
      dma_piece(X + (size_t)sr * a.ldx + kh0 + p * 512 + lane * 8, dst + r * XROW + p * 512);
    }
    if (opw) {
      char* od = ops + (t % GP_NBUF) * 4096;
      if (EPI == ZMI_EPI_RESIDUAL) {  // [row][group] 16 B: out[row][8 g .. 8 g + 7]
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int e = lane + 64 * i, r = e >> 4, gi = min(pb * GP_G + (e & 15), ngroups - 1);
          dma_piece(reinterpret_cast<const bf16_t*>(a.out) + (size_t)min(t * RT + r, a.M - 1) * a.ldo + gi * 8,
                    reinterpret_cast<bf16_t*>(od + i * 1024));
        }
      } else if (EPI == ZMI_EPI_QKV) {  // dwords 0..15 the rows' positions, 16..31 their cache rows
        const int r = min(t * RT + (lane & 15), a.M - 1);
        dma_dword((lane & 16) ? a.row_kv + r : a.row_pos + r, od);
      }
    }
  };

  dma_tile(t0);
  if (t0 + 1 < rt_end) dma_tile(t0 + 1);
  if (t0 + 2 < rt_end) dma_tile(t0 + 2);
  __builtin_amdgcn_sched_barrier(0);
  // the wave's pair over its segment: lane l = column l & 15 of the pair, M8 lane (l & 7) + 8 h + 16 (l >> 4) of
  // group 2 ps + ((l >> 3) & 1) (clamped: discarded), as gemm_rows_kernel's DN form
  u32x4_t wf[2][NL];
  {
    const int grp = min(pb * GP_G + 2 * ps + ((lane >> 3) & 1), ngroups - 1) - pb * GP_G;
    const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(reinterpret_cast<const char*>(a.W) + (size_t)pb * GP_G * KC * 1024), (short)0,
        GP_G * KC * 1024, 0x00020000);
    const int vo = (grp * KC + wk * NL) * 1024 + ((lane & 7) + 16 * (lane >> 4)) * 16;
#pragma unroll
    for (int j = 0; j < NL; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) wf[h][j] = __builtin_amdgcn_raw_buffer_load_b128(wrsrc, vo + 128 * h, j * 1024, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  ZMI_WAIT_VM(0);
  __syncthreads();

  // the two elements (c, r) of a group that lane `lane` finishes in epilogue<EPI> (zmi_gemv_impl.h), i = 0, 1
  auto coord = [&](int i, int& c, int& r) {
    if (EPI == ZMI_EPI_SWIGLU) {
      c = (lane & 3) + 4 * i;
      r = lane >> 2;
    } else if (EPI == ZMI_EPI_QKV) {
      c = (lane & 3) * 2 + i;
      r = lane >> 2;
    } else {
      c = (lane + 64 * i) & 7;
      r = (lane + 64 * i) >> 3;
    }
  };
  auto which = [&](int c, int r) {  // coord's i for (c, r)
    if (EPI == ZMI_EPI_SWIGLU) return c >= 4 ? 1 : 0;
    if (EPI == ZMI_EPI_QKV) return c & 1;
    return r * 8 + c >= 64 ? 1 : 0;
  };
  // a store wave whose second group is past the unit's end issues fewer stores: it drains fully instead
  const bool full_sw = 2 * wave + 1 < n_gl;

  for (int t = t0;; ++t) {  // invariant: tile t's rows and operands are in LDS, visible to every wave
    const int ti = t - t0;
    const int row0 = t * RT, rows = min(RT, a.M - row0);
    const bool more = t + 1 < rt_end;
    unsigned* flag = flags + (size_t)pb * n_rt + t;
    // lower epilogue waves: the partner's {s2, s3} of tile t (published once its stores of tile t + 1 are out),
    // loaded now, used after this tile's chains
    uint64_t hv[2][2] = {{0ull, 0ull}, {0ull, 0ull}};
    if (!up && ew) {
      if (lane == 0) {
        for (unsigned spin = 0; __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)n_ew &&
                                spin < GP_SPIN; ++spin)
          __builtin_amdgcn_s_sleep(1);
      }
      // the loads below issue only once lane 0 left the loop (the wave's branch waits for the counter's value); they
      // read the coherence point (sc1) that the partner's write-through stores reached before it bumped the counter
      asm volatile("" ::: "memory");
      const uint64_t* src = hp + (size_t)row0 * a.N + pb * GP_G * 8;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int gl = min(2 * wave + h, n_gl - 1);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          int c, r;
          coord(i, c, r);
          hv[h][i] = ld_wt64(src + (size_t)r * a.N + gl * 8 + c);
        }
      }
    }
    f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    {
      const bf16_t* xa = xs + (t % GP_NBUF) * RT * XROW + (lane & 15) * XROW + sk * NL * 64 + (lane >> 4) * 8;
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        const bf16x8_t x0 = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(xa + j * 64));
        const bf16x8_t x1 = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(xa + j * 64 + 32));
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, __builtin_bit_cast(bf16x8_t, wf[0][j]), acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, __builtin_bit_cast(bf16x8_t, wf[1][j]), acc1, 0, 0, 0);
      }
    }
    // the previous tile's epilogues (stores) have read the segment sums
    if (ti > 0) {
      const unsigned want = (unsigned)(n_ew * ti);
      for (int spin = 0; *lcnt < want && spin < (1 << 20); ++spin) __builtin_amdgcn_s_sleep(1);
    }
    {
      const int c = lane & 15, rb = (lane >> 4) * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) red[(((2 * ps + (c >> 3)) * 2 + sk) * 8 + (c & 7)) * RT + rb + q] = acc0[q] + acc1[q];
    }
    uint32_t res_pre[2][NE] = {{0u, 0u}, {0u, 0u}};
    int q_pos = -1, q_kvr = 0;
    if (!up && ew) {
      const char* od = ops + (t % GP_NBUF) * 4096;
      if (EPI == ZMI_EPI_RESIDUAL) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < NE; ++i) {
            const int e = lane + 64 * i, r = e >> 3, c = e & 7;
            res_pre[h][i] = *reinterpret_cast<const uint16_t*>(od + (r * GP_G + 2 * wave + h) * 16 + c * 2);
          }
      }
      if (EPI == ZMI_EPI_QKV && (lane >> 2) < rows) {
        q_pos = reinterpret_cast<const int*>(od)[lane >> 2];
        q_kvr = reinterpret_cast<const int*>(od)[16 + (lane >> 2)];
      }
    }
    // DMA waves: tile t + 1 landed (tile t + 2's pieces, issued one iteration later, may stay in flight)
    if (dw) {
      if (t + 2 < rt_end) {
        if (opw) ZMI_WAIT_VM(PPW + EP);
        else ZMI_WAIT_VM(PPW);
      } else {
        ZMI_WAIT_VM(0);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    if (!up && tid == 0)  // every epilogue wave has read tile t's counter (before this barrier)
      __hip_atomic_store(flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t + 3 < rt_end) dma_tile(t + 3);
    if (ew && up) {
      // hand-off: {s2, s3} of (row, column) for groups 2w, 2w + 1; lane = (row, 4 columns)
      const int r = lane >> 2, cq = lane & 3, gl = 2 * wave + (cq >> 1);
      if (gl < n_gl) {
        uint64_t* dst = hp + (size_t)(row0 + r) * a.N + (pb * GP_G + gl) * 8 + (cq & 1) * 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = (cq & 1) * 4 + i;
          st_wt64(dst + i, pack_f2(red[((gl * 2 + 0) * 8 + c) * RT + r], red[((gl * 2 + 1) * 8 + c) * RT + r]));
        }
      }
      if (more && lane == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      // tile t - 1's stores (issued a tile ago) are at the coherence point: publish it (this tile's 4 stay in flight)
      if (ti > 0) {
        if (full_sw) ZMI_WAIT_VM(4);
        else ZMI_WAIT_VM(0);
        if (lane == 0) __hip_atomic_fetch_add(flag - 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else if (ew) {
#pragma unroll 1
      for (int h = 0; h < 2; ++h) {
        const int gl = 2 * wave + h;
        if (gl >= n_gl) break;
        auto colsum = [&](int c, int r) {  // ((s0 + s1) + s2) + s3: gemm_rows_kernel's segment order
          const uint64_t g = which(c, r) ? hv[h][1] : hv[h][0];
          float v = red[((gl * 2 + 0) * 8 + c) * RT + r];
          v += red[((gl * 2 + 1) * 8 + c) * RT + r];
          v += lo_f(g);
          v += hi_f(g);
          return v;
        };
        epilogue<EPI, RT, 0>(a, colsum, lane, rows, row0, pb * GP_G + gl, res_pre[h], q_pos, q_kvr,
                             QkvFuse{nullptr, 0});
      }
      if (more && lane == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (!more) break;
  }
  if (up && ew) {  // the last tile
    ZMI_WAIT_VM(0);
    if (lane == 0)
      __hip_atomic_fetch_add(flags + (size_t)pb * n_rt + rt_end - 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

struct PairLayout {
  int n_pb, n_rt;
  size_t flags_bytes, total;
};
PairLayout pair_layout(int M, int N) {
  PairLayout l;
  l.n_pb = (N / 8 + GP_G - 1) / GP_G;
  l.n_rt = (M + GR_RT - 1) / GR_RT;
  l.flags_bytes = (((size_t)l.n_pb * l.n_rt * 4) + 255) / 256 * 256;
  l.total = l.flags_bytes + (size_t)l.n_rt * GR_RT * N * 8;
  return l;
}

template <int EPI>
hipError_t launch_pair(const ZmiGemvArgs& a, char* work, hipStream_t s) {
  auto fn = gemm_pair_kernel<EPI>;
  const PairLayout l = pair_layout(a.M, a.N);
  const int rpw = rows_per_wg(l.n_pb, l.n_rt, std::max(1, zmi_cu_count() / 2));  // a pair of CUs per unit
  const int64_t half = (int64_t)((l.n_pb + 7) / 8) * 8 * ((l.n_rt + rpw - 1) / rpw);
  static const hipError_t attr =
      hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, (int)GP_LDS);
  if (attr != hipSuccess) return attr;
  if (2 * half > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fn, dim3((unsigned)(2 * half)), dim3(1024), GP_LDS, s, a, l.n_pb, l.n_rt, rpw, (int)half,
                     reinterpret_cast<uint64_t*>(work + l.flags_bytes), reinterpret_cast<unsigned*>(work));
  return hipGetLastError();
}

}  // namespace

extern "C" int64_t zmi_gemv_rows_pair_bytes(int M, int N) {
  if (M < 1 || N < 8 || N % 8) return -1;
  return (int64_t)pair_layout(M, N).total;
}

extern "C" int zmi_gemv_rows_pair(const ZmiGemvArgs* args, int epi, void* work, int64_t work_bytes, void* stream) {
  const ZmiGemvArgs& a = *args;
  if (a.K != 2048 || a.N % 8 || a.M < 1 || a.ldx % 8) return zmi_fail_msg("gemv_rows_pair: K = 2048, N % 8 == 0, M >= 1");
  if (a.ln_w || a.pro != ZMI_PRO_AUTO || a.groups != 0)
    return zmi_fail_msg("gemv_rows_pair: plain GEMM only (no LayerNorm, prologue or group override)");
  if (!work || work_bytes < zmi_gemv_rows_pair_bytes(a.M, a.N))
    return zmi_fail_msg("gemv_rows_pair: work must hold zmi_gemv_rows_pair_bytes(M, N) bytes (zeroed once)");
  if (epi == ZMI_EPI_QKV && (a.hd % 8 || a.smax <= 0 || !a.row_pos || !a.row_kv || !a.rope))
    return zmi_fail_msg("gemv_rows_pair: the QKV epilogue needs row_pos, row_kv, rope, smax and hd % 8 == 0");
  hipStream_t s = (hipStream_t)stream;
  char* w = reinterpret_cast<char*>(work);
  hipError_t e;
  switch (epi) {
    case ZMI_EPI_STORE: e = launch_pair<ZMI_EPI_STORE>(a, w, s); break;
    case ZMI_EPI_RESIDUAL: e = launch_pair<ZMI_EPI_RESIDUAL>(a, w, s); break;
    case ZMI_EPI_QKV: e = launch_pair<ZMI_EPI_QKV>(a, w, s); break;
    case ZMI_EPI_SWIGLU: e = launch_pair<ZMI_EPI_SWIGLU>(a, w, s); break;
    case ZMI_EPI_LOGITS: e = launch_pair<ZMI_EPI_LOGITS>(a, w, s); break;
    case ZMI_EPI_F32: e = launch_pair<ZMI_EPI_F32>(a, w, s); break;
    default: return zmi_fail_msg("gemv_rows_pair: unknown epilogue");
  }
  ZMI_CHECK(e);
  return 0;
}
