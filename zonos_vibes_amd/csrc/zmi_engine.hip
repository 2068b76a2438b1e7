// Persistent decode engine for the second half of a transformer block at batch 1 (2 rows: the CFG
// cond / uncond pair): reference zonos/backbone/_torch.py:100-101 (x = x + out_proj(attn)), :101 norm2,
// :147-152 (fc1 -> y * silu(gate) -> fc2) and the second residual add, in ONE launch of 256 workgroups
// (one per CU) instead of three GEMV launches.
//
// Why (MI355X_MICROARCH.md rows launches-baseline / engine-vs-launches / prefetch-credit): as launches,
// every op pays a boundary plus a ramp, and HBM idles while the small out_proj and each op's epilogue
// run. Here each CU streams its slice of all three weight matrices through an LDS ring that runs ahead
// of the data dependencies, so the weights of fc1 / fc2 are already in LDS when the activation they
// need arrives from the other CUs.
//
// Workgroup b (6 waves):
//   waves 0..3  consumers: wave c owns K segment c of the K = 2048 GEMVs (the GEMV's wave split, W = 4 x
//               NL = 8 chunks) and streams its own items through a private ring of DEPTH 8 KiB slots by
//               LDS-DMA with the non-temporal policy (nt-weights); it counts its own DMAs with vmcnt, so
//               the ring needs no handshake with another wave;
//   waves 4..5  service: wave 4 + r owns row r: activation loads, the epilogues, the granule hand-offs
//               (8-byte {value, tag = position + 1} words, cdna_hip_programming.md §6 Guideline 16 R2),
//               the gathers, norm2.
// Work of block b (team s = b & 7, one XCD under round-robin placement; member m = b >> 3):
//   out_proj  column group b (8 of 2048 outputs)                             -> x' granules (all blocks gather)
//   fc1       groups 256 s + 8 m + j, j < 8 (h[1024 s + 32 m .. + 31])       -> h granules (team s gathers)
//   fc2       groups 8 m + j, j < 8, K segment s (16 chunks, the GEMV's W = 8 split) -> fp32 segment sums
//   combine   group b: the 8 segment sums in segment order + residual         -> x
// Every sum is the GEMV's (zmi_gemv_impl.h): per (group, segment) one chain of MFMAs over the segment's
// chunks (k-half 0 / 1 in two accumulators, acc0 + ror8(acc1)), the segment sums added in segment order,
// the same residual / LayerNorm / SwiGLU arithmetic. x and h are bit-identical to zmi_gemv_launch of
// out_proj (EPI_RESIDUAL), fc1 (LayerNorm prologue, EPI_SWIGLU) and fc2 (EPI_RESIDUAL).
#include <algorithm>

#include "zmi_common.h"
#include "zmi_kernels.h"
#include "zonos_diag.h"
#include "zmi_gemv_impl.h"
#include "zmi_engine.h"

namespace {

using namespace zmi_eng;

constexpr int DM = 2048, FF = 8192;
constexpr int NBLK = 256;
constexpr int NCW = 4, NSW = 2, NWV = NCW + NSW, NT = NWV * 64;
constexpr int MAXR = 2;
constexpr int DEPTH = 4;
constexpr int NSLOT = 13;                 // out_proj 1 + fc1 8 + fc2 2 x 2 slots per consumer wave
constexpr int XROW = DM + 8;
constexpr int GX_W = DM / 2, GH_W = FF / 2, GP_W = 256 * 8 * 8;  // granule words per row

// LDS
constexpr size_t L_RING = 0;                                            // [NCW][DEPTH][8 KiB]
constexpr size_t L_BUFA = L_RING + (size_t)NCW * DEPTH * SLOT;          // bf16 [MAXR][XROW] attn rows, then h segment
constexpr size_t L_BUFB = L_BUFA + (size_t)MAXR * XROW * 2;             // bf16 [MAXR][XROW] norm2(x')
constexpr size_t L_REDO = L_BUFB + (size_t)MAXR * XROW * 2;             // f32 [NCW][8][MAXR] out_proj segment sums
constexpr size_t L_REDF = L_REDO + (size_t)NCW * 8 * MAXR * 4;          // f32 [8][NCW][8][MAXR] fc1 segment sums
constexpr size_t L_CNT = L_REDF + (size_t)8 * NCW * 8 * MAXR * 4;       // u32 [16] arrival counters
constexpr size_t L_BYTES = L_CNT + 16 * 4;
static_assert(L_BYTES <= 160 * 1024, "LDS");
static_assert(L_BUFA % 16 == 0 && L_BUFB % 16 == 0 && L_CNT % 16 == 0, "alignment");
enum { C_READY = 0, C_O = 1, C_F1 = 2 };  // C_F1 + j: fc1 group j

struct Args {
  const char* w_out;
  const char* w_fc1;
  const char* w_fc2;
  const bf16_t* ln_w;
  const bf16_t* ln_b;
  float eps;
  int M;
  const bf16_t* attn;
  bf16_t* x;
  bf16_t* h;
  int ld_attn, ldx, ldh;
  const int* row_pos;
  uint64_t* gran;
  unsigned* err;
  unsigned long long* diag;
  int start, spare;  // ZMI_OPT_ENG_START / _SPARE
};

__device__ __forceinline__ void stamp(const Args& a, int i) {
  if (a.diag && (threadIdx.x & 63) == 0)
    a.diag[(size_t)blockIdx.x * 16 + i] = __builtin_amdgcn_s_memrealtime();
}

// slot k of consumer wave c in block b: 8 KiB of one weight matrix (M8 layout: group g's chunks
// contiguous, 1 KiB each)
__device__ __forceinline__ const char* slot_src(const Args& a, int k, int b, int c) {
  const int s = b & 7, m = b >> 3;
  if (k == 0) return a.w_out + ((size_t)b * 32 + c * 8) * 1024;  // out_proj group b, segment c
  if (k <= 8) {                                                  // fc1 group 256 s + 8 m + j, segment c
    const int G = 256 * s + 8 * m + (k - 1);
    return a.w_fc1 + ((size_t)G * 32 + c * 8) * 1024;
  }
  const int kk = k - 9, g = 8 * m + 2 * c + (kk >> 1);           // fc2 group, segment s, half kk & 1
  return a.w_fc2 + ((size_t)g * 128 + s * 16 + (kk & 1) * 8) * 1024;
}

__device__ __forceinline__ lds_u32* lds_cnt(char* smem, int i) { return lds_word(smem, L_CNT + 4 * i); }

__device__ __forceinline__ void consumer(const Args& a, char* smem, int b, int c, int lane, const unsigned (&tag)[MAXR]) {
  const unsigned ring = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(__attribute__((address_space(3))) char*)(smem + L_RING + (size_t)c * DEPTH * SLOT));
  // the first DEPTH slots before anything else; out_proj's slot is on the critical path (its result goes to
  // every block), so by default it is requested first and has landed before the fc1 slots are requested
  issue_slot(slot_src(a, 0, b, c), ring, lane);
  if (a.start == 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (a.start == 2) {
    issue_slot(slot_src(a, 1, b, c), ring + SLOT, lane);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  }
  if (c == 0) stamp(a, 7);
#pragma unroll
  for (int k = 1; k < DEPTH; ++k)
    if (k > 1 || a.start != 2) issue_slot(slot_src(a, k, b, c), ring + k * SLOT, lane);
  const bf16_t* bufA = reinterpret_cast<const bf16_t*>(smem + L_BUFA);
  const bf16_t* bufB = reinterpret_cast<const bf16_t*>(smem + L_BUFB);
  float* redo = reinterpret_cast<float*>(smem + L_REDO);
  float* redf = reinterpret_cast<float*>(smem + L_REDF);
  const int s = b & 7, m = b >> 3;
  const int col = lane & 15, quad = lane >> 4;
  uint4 xa0[16], xa1[16];
  // A fragments of this wave's K segment (gemv_body step 4): lane l reads row min(l & 15, M - 1),
  // k = 8 (l >> 4) .. + 7 of each 32-wide k-half
  auto load_frag = [&](const bf16_t* buf, int koff, int nch) {
    const int ar = min(col, a.M - 1);
    const bf16_t* p = buf + ar * XROW + koff + quad * 8;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (j < nch) {
        xa0[j] = *reinterpret_cast<const uint4*>(p + j * 64);
        xa1[j] = *reinterpret_cast<const uint4*>(p + j * 64 + 32);
      }
  };
  f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < NSLOT; ++k) {
    if (k == 0) {
      lds_wait_ge(lds_cnt(smem, C_READY), NSW * 1, a.err);
      load_frag(bufA, c * 512, 8);
    } else if (k == 1) {
      lds_wait_ge(lds_cnt(smem, C_READY), NSW * 2, a.err);
      load_frag(bufB, c * 512, 8);
    } else if (k == 9) {
      lds_wait_ge(lds_cnt(smem, C_READY), NSW * 3, a.err);
      load_frag(bufA, 0, 16);
    }
    wait_slot(std::min(DEPTH - 1, NSLOT - 1 - k));
    u32x4_t wv[8];
    const u32x4_t* rp = reinterpret_cast<const u32x4_t*>(smem + L_RING + ((size_t)c * DEPTH + k % DEPTH) * SLOT) + lane;
#pragma unroll
    for (int j = 0; j < 8; ++j) wv[j] = rp[j * 64];
    if (k + DEPTH < NSLOT) issue_slot(slot_src(a, k + DEPTH, b, c), ring + ((k + DEPTH) % DEPTH) * SLOT, lane);
    const bool second = k >= 9 && ((k - 9) & 1);  // second 8 chunks of an fc2 segment: the chain continues
    const int base = second ? 8 : 0;
    if (!second) acc0 = acc1 = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bf16x8_t w = __builtin_bit_cast(bf16x8_t, wv[j]);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, xa0[base + j]), w, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, xa1[base + j]), w, acc1, 0, 0, 0);
    }
    if (k >= 9 && !second) continue;
    // segment sum (gemv_body step 5): column l & 15 < 8, row 4 (l >> 4) + q
    float v[MAXR];
#pragma unroll
    for (int q = 0; q < MAXR; ++q) v[q] = acc0[q] + ror8(acc1[q]);
    const bool mine = col < 8 && quad == 0;
    if (k == 0) {
      if (mine)
#pragma unroll
        for (int q = 0; q < MAXR; ++q) redo[(c * 8 + col) * MAXR + q] = v[q];
      lds_arrive(lds_cnt(smem, C_O), lane);
      if (c == 0) stamp(a, 8);
    } else if (k <= 8) {
      if (mine)
#pragma unroll
        for (int q = 0; q < MAXR; ++q) redf[(((k - 1) * NCW + c) * 8 + col) * MAXR + q] = v[q];
      lds_arrive(lds_cnt(smem, C_F1 + k - 1), lane);
      if (k == 8 && c == 0) stamp(a, 9);
    } else {
      // fc2 group g, segment s: the fp32 segment sums out as {f32, tag} granules for group g's combiner
      const int g = 8 * m + 2 * c + ((k - 9) >> 1);
      uint64_t* gp = a.gran + (size_t)a.M * (GX_W + GH_W);
      if (mine)
#pragma unroll
        for (int q = 0; q < MAXR; ++q)
          if (q < a.M)
            st_wt64(gp + (((size_t)g * 8 + s) * a.M + q) * 8 + col,
                    (uint64_t)__float_as_uint(v[q]) | ((uint64_t)tag[q] << 32));
      if (k == NSLOT - 1 && c == 0) stamp(a, 10);
    }
  }
}

__device__ __forceinline__ void service(const Args& a, char* smem, int b, int r, int lane, const unsigned (&tag)[MAXR]) {
  const bool live = r < a.M;
  const int s = b & 7, m = b >> 3;
  bf16_t* bufA = reinterpret_cast<bf16_t*>(smem + L_BUFA);
  bf16_t* bufB = reinterpret_cast<bf16_t*>(smem + L_BUFB);
  const float* redo = reinterpret_cast<const float*>(smem + L_REDO);
  const float* redf = reinterpret_cast<const float*>(smem + L_REDF);
  uint64_t* gx = a.gran;
  uint64_t* gh = a.gran + (size_t)a.M * GX_W;
  const uint64_t* gp = a.gran + (size_t)a.M * (GX_W + GH_W);
  const unsigned tg = live ? tag[r] : 0u;
  if (r == 0) stamp(a, 0);
  // (1) the attention row (out_proj activations) and the residual values of out_proj's columns
  uint32_t xres = 0;
  if (live) {
    const uint4* src = reinterpret_cast<const uint4*>(a.attn + (size_t)r * a.ld_attn);
    uint4* dst = reinterpret_cast<uint4*>(bufA + r * XROW);
#pragma unroll
    for (int i = 0; i < DM / 512; ++i) dst[lane + 64 * i] = src[lane + 64 * i];
    if (lane < 8) xres = a.x[(size_t)r * a.ldx + 8 * b + lane];
  }
  lds_arrive(lds_cnt(smem, C_READY), lane);
  // (2) out_proj epilogue (EPI_RESIDUAL): x' = bf16(x + bf16(segment sums in order)), out as granules
  lds_wait_ge(lds_cnt(smem, C_O), NCW, a.err);
  uint32_t xnew = 0;
  if (live) {
    float v = 0.f;
    if (lane < 8) {
      v = redo[(0 * 8 + lane) * MAXR + r];
#pragma unroll
      for (int w = 1; w < NCW; ++w) v += redo[(w * 8 + lane) * MAXR + r];
    }
    xnew = f2bf(bf2f(xres) + bfround(v));
    const uint32_t nb = (uint32_t)__shfl_down((int)xnew, 1);
    if (lane < 8 && (lane & 1) == 0)
      st_wt64(gx + (size_t)r * GX_W + 4 * b + (lane >> 1), (uint64_t)(xnew | (nb << 16)) | ((uint64_t)tg << 32));
  }
  if (r == 0) stamp(a, 1);
  // (3) x' of every block, then norm2 in place: fc1's activations
  if (live) {
    gather<GX_W / 64>(gx + (size_t)r * GX_W, reinterpret_cast<uint32_t*>(bufB + r * XROW), tg, lane, a.err);
    if (r == 0) stamp(a, 2);
    ln_row(bufB + r * XROW, a.ln_w, a.ln_b, a.eps, lane);
  }
  if (r == 0) stamp(a, 3);
  lds_arrive(lds_cnt(smem, C_READY), lane);
  // (4) fc1 epilogues (EPI_SWIGLU, M8 packing: columns 0..3 values, 4..7 gates), out as h granules
  for (int j = 0; j < 8; ++j) {
    lds_wait_ge(lds_cnt(smem, C_F1 + j), NCW, a.err);
    if (!live) continue;
    auto colsum = [&](int cc) {
      float v = redf[((j * NCW + 0) * 8 + cc) * MAXR + r];
#pragma unroll
      for (int w = 1; w < NCW; ++w) v += redf[((j * NCW + w) * 8 + cc) * MAXR + r];
      return v;
    };
    uint32_t hv = 0;
    if (lane < 4) {
      const float y = bfround(colsum(lane));
      const float gt = bfround(colsum(lane + 4));
      const float sg = bfround(gt / (1.0f + expf(-gt)));
      hv = f2bf(y * sg);
    }
    const uint32_t nb = (uint32_t)__shfl_down((int)hv, 1);
    const int hi = 1024 * s + 32 * m + 4 * j + lane;  // h column of lane < 4
    if (lane < 4 && (lane & 1) == 0)
      st_wt64(gh + (size_t)r * GH_W + (hi >> 1), (uint64_t)(hv | (nb << 16)) | ((uint64_t)tg << 32));
    if (a.h && lane < 4) a.h[(size_t)r * a.ldh + hi] = (bf16_t)hv;
  }
  if (r == 0) stamp(a, 4);
  // (5) h segment s (fc2's activations for this block's K segment), produced by team s
  if (live)
    gather<512 / 64>(gh + (size_t)r * GH_W + 512 * s, reinterpret_cast<uint32_t*>(bufA + r * XROW), tg, lane, a.err);
  if (r == 0) stamp(a, 5);
  lds_arrive(lds_cnt(smem, C_READY), lane);
  // (6) fc2 group b: the 8 segment sums (blocks 8 (b >> 3) + s') added in segment order, + the residual x'
  if (live) {
    const int sp = lane >> 3, cc = lane & 7;
    const uint64_t* src = gp + (((size_t)b * 8 + sp) * a.M + r) * 8 + cc;
    uint64_t w = ld_wt64(src);
    for (unsigned spin = 0; !__all((uint32_t)(w >> 32) == tg); ++spin) {
      if (spin > SPIN) {
        give_up(a.err);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      if ((uint32_t)(w >> 32) != tg) w = ld_wt64(src);
    }
    const float val = __uint_as_float((uint32_t)w);
    float v = __shfl(val, cc);
#pragma unroll
    for (int q = 1; q < 8; ++q) v += __shfl(val, 8 * q + cc);
    if (lane < 8) a.x[(size_t)r * a.ldx + 8 * b + lane] = (bf16_t)f2bf(bf2f(xnew) + bfround(v));
  }
  if (r == 0) stamp(a, 6);
}

__global__ __launch_bounds__(NT) void ffn_engine_kernel(const Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (tid < 16) *lds_cnt(smem, tid) = 0u;
  unsigned tag[MAXR];
#pragma unroll
  for (int r = 0; r < MAXR; ++r) tag[r] = r < a.M ? (unsigned)(a.row_pos[r] + 1) : 0u;
  __syncthreads();
  if (wave < NCW)
    consumer(a, smem, b, wave, lane, tag);
  else
    service(a, smem, b, wave - NCW, lane, tag);
}

}  // namespace

extern "C" int64_t zmi_ffn_engine_gran_words(int rows) {
  return (rows < 1 || rows > MAXR) ? -1 : (int64_t)rows * (GX_W + GH_W + GP_W);
}

extern "C" int zmi_ffn_engine(const ZmiFfnEngineArgs* args, void* stream) {
  const ZmiFfnEngineArgs& e = *args;
  if (e.M < 1 || e.M > MAXR) return zmi_fail_msg("ffn_engine: 1 <= M <= 2 rows");
  if (!e.w_out || !e.w_fc1 || !e.w_fc2 || !e.ln_w || !e.ln_b || !e.attn || !e.x || !e.row_pos || !e.gran || !e.err)
    return zmi_fail_msg("ffn_engine: missing buffers");
  if (e.ld_attn % 8 || e.ldx % 8 || (e.h && e.ldh % 8)) return zmi_fail_msg("ffn_engine: row strides must be multiples of 8");
  if (zmi_cu_count() < NBLK) return zmi_fail_msg("ffn_engine: needs 256 CUs (one resident workgroup per CU)");
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&ffn_engine_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)L_BYTES);
  ZMI_CHECK(attr);
  Args a{};
  a.w_out = (const char*)e.w_out;
  a.w_fc1 = (const char*)e.w_fc1;
  a.w_fc2 = (const char*)e.w_fc2;
  a.ln_w = (const bf16_t*)e.ln_w;
  a.ln_b = (const bf16_t*)e.ln_b;
  a.eps = e.eps;
  a.M = e.M;
  a.attn = (const bf16_t*)e.attn;
  a.x = (bf16_t*)e.x;
  a.h = (bf16_t*)e.h;
  a.ld_attn = e.ld_attn;
  a.ldx = e.ldx;
  a.ldh = e.ldh;
  a.row_pos = e.row_pos;
  a.gran = (uint64_t*)e.gran;
  a.err = e.err;
  a.diag = (unsigned long long*)e.diag;
  a.start = zmi_option(ZMI_OPT_ENG_START);
  a.spare = 0;
  hipLaunchKernelGGL(ffn_engine_kernel, dim3(NBLK), dim3(NT), L_BYTES, (hipStream_t)stream, a);
  ZMI_CHECK(hipGetLastError());
  return 0;
}
