// DAC 44.1 kHz decoder conv stack on MFMA, gfx950 (DACAutoencoder.decode, reference
// zonos/autoencoder.py:25-27 -> transformers DacModel.decode, modeling_dac.py:610-640).
//
// Every convolution of the decoder (k7 dilated convs, 1x1 convs, the k=2s transposed convs
// in polyphase form) is one implicit GEMM:
//     out[t_out][co] = epi( bias[co] + sum_tap sum_ci W[tap][co][ci] * x[t_in][ci] )
//     t_in = q + in_off + tap * tap_step,  t_out = q * out_stride + out_phase
// Activations are channels-last fp16 so both MFMA operands are 16 B contiguous per lane:
//   A (weights) lane l: co = l&15, ci = 8*(l>>4)..+7      B (activations) lane l: t = l&15, same ci
// fp32 accumulation (v_mfma_f32_16x16x32_f16), fp16 storage as the reference's GPU autocast.
// Snake (x + sin^2(a x)/(a + 1e-9), modeling_dac.py:86-100) is evaluated ONCE per element in
// the producing epilogue, which stores the raw tensor (for the residual skip) and/or its
// Snake'd copy (the next conv's input); the residual add of DacResidualUnit
// (modeling_dac.py:189-209) is fused in the 1x1 conv's epilogue.
#include "zmi_common.h"
#include "zmi_kernels.h"

namespace {

struct ConvArgs {
  const f16_t* x;
  int t_in, c_in;
  const f16_t* w;
  const float* bias;
  int c_out, taps, tap_step, in_off, n_out, out_stride, out_phase, t_out;
  const f16_t* skip;
  f16_t* out_raw;
  f16_t* out_snake;
  const float* alpha;
  float* out_f32;
  int tanh_c0;  // decoder.conv2: out_f32[t] = tanh(y[t][0]) only (c_out zero-padded to 32 for the MFMA tile)
  // polyphase ConvTranspose as ONE launch (blockIdx.z = phase rho, nphase = stride): phase rho reads its
  // own [taps][c_in / 32][c_out][32] weights at w + rho * w_phase, in_off = (rho + phase_pad) / out_stride,
  // out_phase = rho. nphase == 1: in_off / out_phase / w as given.
  int nphase, phase_pad;
  size_t w_phase;
};

__device__ __forceinline__ float snake(float y, float a, float inv_a) {
  // hardware v_sin_f32 (input in revolutions) instead of the libm range-reduced sinf: the epilogue,
  // not the MFMA K loop, bounds the many-sample / few-channel stages, and its error (~1e-6 abs for
  // the |a y| seen here) is far below the fp16 storage rounding that follows
  const float s = __sinf(a * y);
  return y + inv_a * (s * s);  // inv_a = 1 / (a + 1e-9), the reference's reciprocal (modeling_dac.py:97)
}

#ifdef ZMI_DAC_STAMPS
// diagnostic builds only (tools/dac_stamps.py): per workgroup of the conv_stage_kernel launches with c_out ==
// ZMI_DAC_STAMPS and tap_step == 1, thread 0 stores s_memrealtime stamps: [0] start, for stage s < 8: [1 + 3 s]
// its loads landed (after its barrier), [2 + 3 s] = [1 + 3 s] (the next stage's loads are issued inside the MFMA
// groups), [3 + 3 s] its MFMAs issued; [30] all MFMAs done, [31] epilogue done
__device__ unsigned long long g_dac_stamps[8192][32];
extern "C" int zmi_dac_stamps_read(void* dst, size_t bytes) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_dac_stamps), bytes) == hipSuccess ? 0 : -1;
}
#define ZMI_DSTAMP(i_)                                                                          \
  do {                                                                                          \
    if (stamp && threadIdx.x == 0) g_dac_stamps[blockIdx.x + gridDim.x * blockIdx.y][i_] =       \
        __builtin_amdgcn_s_memrealtime();                                                       \
  } while (0)
#else
#define ZMI_DSTAMP(i_) \
  do {                 \
  } while (0)
#endif

// Weight layout (halfs): channel-blocked [tap][c_in / 32][c_out][32] (one 32-channel step of 16 output channels, a
// 1 KiB LDS-DMA piece, contiguous) for convs with taps > 1; [c_out][c_in] for the 1x1 convs, whose pieces every
// workgroup requests at the same moment (the staged form does not run them by default): rows 2 c_in bytes apart
// spread a piece over the L2's channels where a contiguous 1 KiB is one channel's queue (measured 57 -> 70 us on
// the 384-channel 1x1 conv at 861 frames, profiles/r05_dac_stage_ab.jsonl)
__device__ __forceinline__ size_t conv_w_off(const ConvArgs& a, int nci, int tap, int cs, int row) {
  return a.taps == 1 ? (size_t)row * a.c_in + cs * 32 : (((size_t)tap * nci + cs) * a.c_out + row) * 32;
}

// all-zero source for the LDS-DMA lanes whose time row lies outside the input (the conv's zero padding)
__device__ __attribute__((aligned(64))) uint4 g_conv_zero[4];

__device__ __forceinline__ void glds16(const void* gsrc, const void* lds) {
  // one 1 KiB LDS-DMA piece: lane l's 16 B land at lds + 16 l (wave-uniform base). Not counted by the
  // compiler: the K loop's explicit vmcnt waits cover it (cdna_hip_programming.md §5 'Async global->LDS')
  const unsigned ldst =
      __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) const void*)lds);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(ldst)
               : "memory");
}

// glds16 with the destination as a wave-uniform LDS byte address (base + offset computed once per kernel: a
// generic -> LDS pointer cast per piece made the compiler emit a null check on src_shared_base that gfx950 rejects)
__device__ __forceinline__ void glds16_at(const void* gsrc, unsigned ldst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(ldst)
               : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 12]
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
#define ZMI_WAIT_VM(k_) \
  case k_: asm volatile("s_waitcnt vmcnt(" #k_ ")" ::: "memory"); break;
    ZMI_WAIT_VM(1) ZMI_WAIT_VM(2) ZMI_WAIT_VM(3) ZMI_WAIT_VM(4) ZMI_WAIT_VM(5) ZMI_WAIT_VM(6)
    ZMI_WAIT_VM(7) ZMI_WAIT_VM(8) ZMI_WAIT_VM(9) ZMI_WAIT_VM(10) ZMI_WAIT_VM(11) ZMI_WAIT_VM(12)
#undef ZMI_WAIT_VM
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

constexpr int HALO_TAPS_ROWS = 64;  // the halo K order's activation tile: BN + up to 64 rows of taps

// One 32-channel K step of a wave's WM x WN block of 16 x 16 output tiles: A fragments from the weight tile `as`
// ([BM co][32 ci], 64 B rows), B fragments from the activation rows `bs` starting at row boff (64 B rows).
// Operand tiles are copied global -> LDS by LDS-DMA (no register staging). The DMA writes lane-linearly (16 rows
// x 64 B per piece), so the bank-conflict swizzle sits on the SOURCE: LDS chunk c' of row r holds channel chunk
// c' ^ swz(r), swz(r) = 2 ((r >> 2) & 1), and the fragment reads apply the same XOR. A ds_read_b128 is served in
// four 16-lane groups ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and the same +32, MI355X_MICROARCH.md §LDS):
// each group reads 16 consecutive rows, rows 0-3 and 12-15 of the window at one chunk and rows 4-11 at the next,
// and swz makes the 16 (row mod 4, chunk) slots distinct at every starting row (4 LDS cycles per read). The
// earlier ((r >> 2) & 3) swizzle, conflict-free for 16 CONSECUTIVE lanes, is 2-way conflicted under these
// groups at every row offset but two (8 cycles per read).
template <int WM, int WN>
struct ConvFrag {
  uint4 a[WM], b[WN];
};

template <int WM, int WN>
__device__ __forceinline__ void conv_load(ConvFrag<WM, WN>& f, const char* as, const char* bs, int boff, int am,
                                          int bn, int lane) {
  const int lr = lane & 15;
  const int rslot = ((lane >> 4) ^ (((lr >> 2) & 1) << 1)) * 16;  // swizzled byte offset of this lane's A fragment
#pragma unroll
  for (int i = 0; i < WM; ++i) f.a[i] = *reinterpret_cast<const uint4*>(as + (am + i * 16 + lr) * 64 + rslot);
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    const int r = bn + j * 16 + lr + boff;
    f.b[j] = *reinterpret_cast<const uint4*>(bs + r * 64 + (((lane >> 4) ^ (((r >> 2) & 1) << 1)) * 16));
  }
}

template <int WM, int WN>
__device__ __forceinline__ void conv_compute(f32x4_t (&acc)[WM][WN], const ConvFrag<WM, WN>& f) {
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, f.a[i]),
                                                         __builtin_bit_cast(f16x8_t, f.b[j]), acc[i][j], 0, 0, 0);
}

template <int WM, int WN>
__device__ __forceinline__ void conv_mfma(f32x4_t (&acc)[WM][WN], const char* as, const char* bs, int boff, int am,
                                          int bn, int lane) {
  ConvFrag<WM, WN> f;
  conv_load(f, as, bs, boff, am, bn, lane);
  conv_compute(acc, f);
}

// Per-thread epilogue channels: thread tid finishes the 8 consecutive channels c8 = tid % (BM / 8) of time rows
// tid / (BM / 8), + RPT, ... of the tile (threads past CPR8 * RPT idle), so its bias, Snake alpha and the
// alpha reciprocal are loaded (and divided) once, at kernel start, where the K loop hides their latency.
template <int WM, int NT>
struct ConvEpiChan {
  static constexpr int CPR8 = 4 * WM, RPT = NT / CPR8;
  float bias[8], al[8], inv[8];
  int c8, row0;
  bool on;
  __device__ __forceinline__ void load(const ConvArgs& a, int co_blk) {
    const int tid = threadIdx.x;
    c8 = tid % CPR8;
    row0 = tid / CPR8;
    on = row0 < RPT;
    const int co = co_blk + c8 * 8;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      bias[r] = on ? a.bias[co + r] : 0.f;
      al[r] = on && a.out_snake ? a.alpha[co + r] : 1.f;
      inv[r] = 1.0f / (al[r] + 1e-9f);  // the reference's reciprocal (modeling_dac.py:97), once per channel
    }
  }
};

// Epilogue of a [BM = 32 WM co] x [BN = 64 NWN t] tile, in PARTS parts of the time tile (PARTS = NWN: the waves
// with wn == part own one, a [64 t][BM co] fp32 LDS tile; PARTS = 1: all of it at once, a [BN t][BM co] tile): the
// accumulators go through LDS, then every thread finishes 8 consecutive channels of its time rows, so the skip
// loads and the raw / snake / f32 stores are whole 16-32 B per lane and each row's BM channels are written
// contiguously. The caller has synchronised the workgroup (lds_raw free).
template <int WM, int WN, int NWN, int PARTS>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, const f32x4_t (&acc)[WM][WN], char* lds_raw, int wn,
                                              int am, int lane, int q_blk, int co_blk, int out_phase,
                                              const ConvEpiChan<WM, 128 * NWN>& ch, bool writer = true) {
  static_assert(NWN % PARTS == 0, "a part is whole wave columns");
  constexpr int BM = 32 * WM, BN = 16 * WN * NWN, TP = BM + 4, WPP = NWN / PARTS;
  constexpr int ROWS = BN / PARTS, RPT = ConvEpiChan<WM, 128 * NWN>::RPT;
  float(&tile)[ROWS][TP] = *reinterpret_cast<float(*)[ROWS][TP]>(lds_raw);
  const int lr = lane & 15, kq = (lane >> 4) * 8;
  const int co = co_blk + ch.c8 * 8;
#pragma unroll
  for (int part = 0; part < PARTS; ++part) {
    if (writer && wn / WPP == part) {
      const int rb = (wn % WPP) * 16 * WN;
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
          *reinterpret_cast<f32x4_t*>(&tile[rb + j * 16 + lr][am + i * 16 + kq / 2]) = acc[i][j];
    }
    __syncthreads();
    if (ch.on) {
      for (int row = ch.row0; row < ROWS; row += RPT) {
        const int q = q_blk + part * ROWS + row;
        if (q >= a.n_out) break;
        const size_t to = (size_t)q * a.out_stride + out_phase;
        const f32x4_t v0 = *reinterpret_cast<const f32x4_t*>(&tile[row][ch.c8 * 8]);
        const f32x4_t v1 = *reinterpret_cast<const f32x4_t*>(&tile[row][ch.c8 * 8 + 4]);
        float y[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        uint4 sk = {0u, 0u, 0u, 0u};
        if (a.skip) sk = *reinterpret_cast<const uint4*>(a.skip + to * a.c_out + co);
        const uint32_t su[4] = {sk.x, sk.y, sk.z, sk.w};
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          y[r] = y[r] + ch.bias[r];
          if (a.skip) y[r] = y[r] + h2f(su[r >> 1] >> ((r & 1) * 16));
        }
        if (a.out_raw) {
          uint4 o;
          o.x = f2h(y[0]) | (f2h(y[1]) << 16);
          o.y = f2h(y[2]) | (f2h(y[3]) << 16);
          o.z = f2h(y[4]) | (f2h(y[5]) << 16);
          o.w = f2h(y[6]) | (f2h(y[7]) << 16);
          *reinterpret_cast<uint4*>(a.out_raw + to * a.c_out + co) = o;
        }
        if (a.tanh_c0) {
          if (co == 0) a.out_f32[to] = tanhf(y[0]);
        } else if (a.out_f32) {
          float4* dst = reinterpret_cast<float4*>(a.out_f32 + to * a.c_out + co);
          dst[0] = float4{y[0], y[1], y[2], y[3]};
          dst[1] = float4{y[4], y[5], y[6], y[7]};
        }
        if (a.out_snake) {
          float z[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) z[r] = snake(y[r], ch.al[r], ch.inv[r]);
          uint4 o;
          o.x = f2h(z[0]) | (f2h(z[1]) << 16);
          o.y = f2h(z[2]) | (f2h(z[3]) << 16);
          o.z = f2h(z[4]) | (f2h(z[5]) << 16);
          o.w = f2h(z[6]) | (f2h(z[7]) << 16);
          *reinterpret_cast<uint4*>(a.out_snake + to * a.c_out + co) = o;
        }
      }
    }
    if (PARTS > 1) __syncthreads();
  }
}

// NWN waves along the time tile (2: 256 threads, BN = 128 rows; 4: 512 threads, BN = 256 rows), 2 along the
// channels: the wide tile issues each weight tile once per 256 output rows (twice the MFMAs per A piece and
// per barrier). Every output's K order and MFMA chain are the tile's own, so both give the same bits.
template <int WM, int WN, int NS, bool HALO, int NWN>
__global__ __launch_bounds__(128 * NWN) void conv_kernel(const ConvArgs a) {
  constexpr int NW = 2 * NWN;
  constexpr int HALO_PIECES = (16 * WN * NWN + HALO_TAPS_ROWS) / 16;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / NWN, wn = wave - wm * NWN;

  f32x4_t acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  //  HALO = false: K steps in (tap, 32-channel) order; each step's A tile [BM co][32 ci] and B tile
  //   [BN t][32 ci] go into an NS-deep ring, step st + NS - 1 issued while step st's MFMAs run, a counted
  //   vmcnt waits for the wave's own pieces of step st.
  //  HALO = true: K steps in (32-channel, tap) order; per channel step the activation rows of ALL taps
  //   (BN + (taps - 1) |tap_step| rows, the halo) are copied once into one of two halo buffers and each
  //   tap reads its fragments at its row offset, so a step streams only its A tile (8 KB at BM = 128,
  //   against 16 KB with the B tile): the next channel step's halo is issued at this one's first tap.
  constexpr int BM = 32 * WM, BN = 16 * WN * NWN;
  constexpr int NPA = BM / 16, NP = (BM + BN) / 16;  // 1 KiB pieces per step
  constexpr int STAGE = HALO ? BM * 64 : (BM + BN) * 64, NSA = HALO ? 2 : NS;
  constexpr int HBUF = HALO ? HALO_PIECES * 1024 : 0;
  constexpr int TP = BM + 4, TILE_BYTES = (BN / NWN) * TP * 4;
  constexpr int RING = NSA * STAGE + 2 * HBUF;
  constexpr int LDS_BYTES = RING > TILE_BYTES ? RING : TILE_BYTES;
  __shared__ __attribute__((aligned(1024))) char lds_raw[LDS_BYTES];
  const int co_blk = blockIdx.y * BM, q_blk = blockIdx.x * BN;
  const int rho = blockIdx.z;
  const f16_t* const wts = a.w + (size_t)rho * a.w_phase;
  const int in_off = a.nphase > 1 ? (rho + a.phase_pad) / a.out_stride : a.in_off;
  const int out_phase = a.nphase > 1 ? rho : a.out_phase;
  const int nci = a.c_in / 32, nsteps = a.taps * nci;
  ConvEpiChan<WM, 128 * NWN> ch;
  ch.load(a, co_blk);
  // per-lane piece geometry: row 16 p + (lane >> 2), LDS chunk lane & 3, source chunk swizzled
  const int prow = lane >> 2, pchunk = (lane & 3) ^ (((lane >> 4) & 1) << 1);
  const int am = wm * (16 * WM), bn = wn * (16 * WN);
  if constexpr (HALO) {
    const int span = (a.taps - 1) * abs(a.tap_step);
    const int omin = in_off + min(0, (a.taps - 1) * a.tap_step);  // first input row of the halo, from q_blk
    const int nbp = (BN + span + 15) / 16;                        // halo pieces (host-checked <= HALO_PIECES)
    char* const abuf = lds_raw;
    char* const hbuf = lds_raw + 2 * STAGE;
    auto issue_a = [&](int st_) {
      const int cs = st_ / a.taps, tap_ = st_ - cs * a.taps;
#pragma unroll
      for (int k = 0; k < (NPA + NW - 1) / NW; ++k) {
        const int p = wave + NW * k;
        if (p < NPA)
          glds16(wts + conv_w_off(a, nci, tap_, cs, co_blk + 16 * p + prow) + pchunk * 8, abuf + (st_ & 1) * STAGE + p * 1024);
      }
    };
    auto issue_halo = [&](int cs) {
      const int ci_ = cs * 32 + pchunk * 8;
      for (int p = wave; p < nbp; p += NW) {
        const int tin = q_blk + omin + 16 * p + prow;
        const bool ok = tin >= 0 && tin < a.t_in;
        glds16(ok ? (const void*)(a.x + (size_t)tin * a.c_in + ci_) : (const void*)&g_conv_zero[lane & 3],
               hbuf + (cs & 1) * HBUF + p * 1024);
      }
    };
    issue_halo(0);
    issue_a(0);
    int cs = 0, tap = 0;
    for (int st = 0; st < nsteps; ++st) {
      wait_vm(0);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // after the barrier every wave is done with step st - 1: its A buffer and (at tap 0) the halo
      // buffer of channel step cs - 1 are free
      if (st + 1 < nsteps) issue_a(st + 1);
      if (tap == 0 && cs + 1 < nci) issue_halo(cs + 1);
      conv_mfma<WM, WN>(acc, abuf + (st & 1) * STAGE, hbuf + (cs & 1) * HBUF, in_off + tap * a.tap_step - omin, am,
                        bn, lane);
      asm volatile("" ::: "memory");
      if (++tap == a.taps) {
        tap = 0;
        ++cs;
      }
    }
  } else {
    const int npw = (NP - wave + NW - 1) / NW;  // this wave's pieces per step: p = wave, wave + NW, ...
    auto issue = [&](int st_) {
      const int tap_ = st_ / nci, ci_ = (st_ - tap_ * nci) * 32 + pchunk * 8;
      char* stg = lds_raw + (st_ % NS) * STAGE;
#pragma unroll
      for (int k = 0; k < (NP + NW - 1) / NW; ++k) {
        const int p = wave + NW * k;
        if (p < NP) {
          const void* src;
          if (p < NPA) {
            src = wts + conv_w_off(a, nci, tap_, st_ - tap_ * nci, co_blk + 16 * p + prow) + pchunk * 8;
          } else {
            const int q = q_blk + 16 * (p - NPA) + prow;
            const int tin = q + in_off + tap_ * a.tap_step;
            const bool ok = q < a.n_out && tin >= 0 && tin < a.t_in;
            src = ok ? (const void*)(a.x + (size_t)tin * a.c_in + ci_) : (const void*)&g_conv_zero[lane & 3];
          }
          glds16(src, stg + p * 1024);
        }
      }
    };
#pragma unroll
    for (int k = 0; k < NS - 1; ++k)
      if (k < nsteps) issue(k);
    for (int st = 0; st < nsteps; ++st) {
      // outstanding after step st's pieces: those of steps st + 1 .. st + NS - 2 that were issued
      wait_vm(npw * (min(nsteps - 1, st + NS - 2) - st));
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (st + NS - 1 < nsteps) issue(st + NS - 1);
      const char* stg = lds_raw + (st % NS) * STAGE;
      conv_mfma<WM, WN>(acc, stg, stg + BM * 64, 0, am, bn, lane);
      asm volatile("" ::: "memory");
    }
  }
  __syncthreads();  // every wave's last fragment reads are done before the ring is reused as the output tile
  conv_epilogue<WM, WN, NWN, NWN>(a, acc, lds_raw, wn, am, lane, q_blk, co_blk, out_phase, ch);
}

// Staged form of the halo K order: one barrier per STAGE of CG 32-channel steps x all TAPS taps instead of one per
// (channel step, tap). A stage's weight tiles (TAPS x CG x [BM co][32 ci]) and activation halos (CG x [256 + span
// rows][32 ci]) go into one of two stage buffers; stage s + 1 is issued right after the barrier that opens stage
// s, so its loads have the whole stage's MFMAs (TAPS x CG x 16 per wave at BM = 128) to land in, against one
// step's 16 in conv_kernel. The price is LDS: 2 stages of a k7 conv at BM = 128 are 152 KiB, one 512-thread
// workgroup per CU. K order: (channel step, tap), conv_kernel's halo order, so every output's MFMA chain and
// bits are the same as conv_kernel's.
template <int WM, int WN, int TAPS, int CG, int HROWS>
__global__ __launch_bounds__(512) void conv_stage_kernel(const ConvArgs a) {
  constexpr int NWN = 4, NW = 8;
  constexpr int BM = 32 * WM, BN = 64 * WN, NPA = BM / 16;
  constexpr int HP = (BN + HROWS + 15) / 16;  // halo pieces per channel step (host-checked)
  constexpr int NA = TAPS * CG * NPA;         // weight pieces per stage
  constexpr int A_BYTES = NA * 1024, STAGE = A_BYTES + CG * HP * 1024;
  // epilogue: the whole [BN t][BM co] fp32 tile at once where the stage buffers hold it, else in halves
  constexpr int PARTS = BN * (BM + 4) * 4 <= 2 * STAGE ? 1 : 2, TILE_BYTES = BN / PARTS * (BM + 4) * 4;
  constexpr int LDS_BYTES = 2 * STAGE > TILE_BYTES ? 2 * STAGE : TILE_BYTES;
  static_assert(LDS_BYTES <= 160 * 1024, "stage buffers exceed the CU's LDS");
  __shared__ __attribute__((aligned(1024))) char lds_raw[LDS_BYTES];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / NWN, wn = wave - wm * NWN;
  f32x4_t acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int co_blk = blockIdx.y * BM, q_blk = blockIdx.x * BN;
  const int rho = blockIdx.z;
  const f16_t* const wts = a.w + (size_t)rho * a.w_phase;
  const int in_off = a.nphase > 1 ? (rho + a.phase_pad) / a.out_stride : a.in_off;
  const int out_phase = a.nphase > 1 ? rho : a.out_phase;
  const int prow = lane >> 2, pchunk = (lane & 3) ^ (((lane >> 4) & 1) << 1);
  const int am = wm * (16 * WM), bn = wn * (16 * WN);
  const int span = (TAPS - 1) * abs(a.tap_step);
  const int omin = in_off + min(0, (TAPS - 1) * a.tap_step);
  const int nbp = (BN + span + 15) / 16;
  const int nstages = a.c_in / (32 * CG);
  // per-lane LDS-DMA sources: the weight piece (g, tap, p) of stage s is 1 KiB at a_src + ((tap nci + s CG + g) c_out
  // + 16 p) 32 halfs (channel-blocked weights); halo piece (g, p) rows q_blk + omin + 16 p + prow
  const int nci = a.c_in / 32;
  const f16_t* const a_src = wts + (TAPS == 1 ? (size_t)(co_blk + prow) * a.c_in : (size_t)(co_blk + prow) * 32) +
                             pchunk * 8;
  auto issue_a = [&](int s, int P) {  // weight piece P = (g TAPS + tap) NPA + p of stage s
    const int g = P / (TAPS * NPA), r = P - g * (TAPS * NPA), tap = r / NPA, p = r - tap * NPA;
    glds16(a_src + (TAPS == 1 ? (size_t)16 * p * a.c_in + (s * CG + g) * 32
                              : ((size_t)(tap * nci + s * CG + g) * a.c_out + 16 * p) * 32),
           lds_raw + (s & 1) * STAGE + P * 1024);
  };
  auto issue_halo = [&](int s) {  // all of this wave's halo pieces of stage s
    char* const hb = lds_raw + (s & 1) * STAGE + A_BYTES;
    for (int P = wave; P < CG * nbp; P += NW) {
      const int g = CG == 1 ? 0 : P / nbp, p = P - g * nbp;
      const int tin = q_blk + omin + 16 * p + prow;
      const bool ok = tin >= 0 && tin < a.t_in;
      glds16(ok ? (const void*)(a.x + (size_t)tin * a.c_in + (s * CG + g) * 32 + pchunk * 8)
                : (const void*)&g_conv_zero[lane & 3],
             hb + (g * HP + p) * 1024);
    }
  };
#ifdef ZMI_DAC_STAMPS
  const bool stamp = a.c_out == ZMI_DAC_STAMPS && a.tap_step == 1 && blockIdx.x + gridDim.x * blockIdx.y < 8192;
#endif
  ZMI_DSTAMP(0);
  issue_halo(0);
#pragma unroll
  for (int k = 0; k < (NA + NW - 1) / NW; ++k)
    if (wave + NW * k < NA) issue_a(0, wave + NW * k);
  ConvEpiChan<WM, 512> ch;  // after the first stage's loads: its latency hides behind theirs (the 512-row tile
  if (WN == 4) ch.load(a, co_blk);  // has no registers to spare in its K loop: loaded after it)
  // Stage s + 1's loads are issued INSIDE stage s, spread over its first GI MFMA groups (the halo and the first
  // taps' weights first), so no wave stalls on a burst of LDS-DMA issues after the barrier and the pieces flow at
  // a rate the CU's load path takes without back-pressure; the last groups issue nothing, so the pieces have the
  // rest of the stage to land before the next barrier's wait.
  constexpr int G = CG * TAPS, GI = G > 3 ? G - 2 : 1, KA = (NA + NW - 1) / NW;
  for (int s = 0; s < nstages; ++s) {
    wait_vm(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s < 8) ZMI_DSTAMP(1 + 3 * s);
    // every wave is done with stage s - 1, whose buffer stage s + 1 fills during this stage
    const bool more = s + 1 < nstages;
    const char* const buf = lds_raw + (s & 1) * STAGE;
    if (s < 8) ZMI_DSTAMP(2 + 3 * s);
    // the stage's (channel step, tap) MFMA groups with their fragments one group ahead in registers: the reads of
    // group u + 1 are issued before group u's MFMAs (a scheduling barrier keeps them there), so each group's 4-7
    // LDS reads have the previous group's 12-16 MFMAs to land in instead of stalling the wave
    ConvFrag<WM, WN> fr[2];
    conv_load(fr[0], buf, buf + A_BYTES, in_off - omin, am, bn, lane);
#pragma unroll
    for (int u = 0; u < G; ++u) {
      if (u + 1 < G) {
        const int g = (u + 1) / TAPS, tap = (u + 1) - g * TAPS;
        conv_load(fr[(u + 1) & 1], buf + (u + 1) * NPA * 1024, buf + A_BYTES + g * HP * 1024,
                  in_off + tap * a.tap_step - omin, am, bn, lane);
      }
      if (more && u < GI) {
        if (u == 0) issue_halo(s + 1);
#pragma unroll
        for (int k = KA * u / GI; k < KA * (u + 1) / GI; ++k)
          if (wave + NW * k < NA) issue_a(s + 1, wave + NW * k);
      }
      __builtin_amdgcn_sched_barrier(0);
      conv_compute(acc, fr[u & 1]);
    }
    asm volatile("" ::: "memory");
    if (s < 8) ZMI_DSTAMP(3 + 3 * s);
  }
  if (WN != 4) ch.load(a, co_blk);
  __syncthreads();
  ZMI_DSTAMP(30);
  conv_epilogue<WM, WN, NWN, PARTS>(a, acc, lds_raw, wn, am, lane, q_blk, co_blk, out_phase, ch);
  ZMI_DSTAMP(31);
}

// The staged K loop with dedicated loader waves (ZMI_OPT_DAC_STAGE bit 4): 8 MFMA waves (2 along the channels x 4
// along 256 time rows, WN = 4) and 4 loader waves, one per SIMD. Only the loaders issue LDS-DMA, so an MFMA wave's
// instruction stream holds nothing but fragment reads and MFMAs, and a loader stalled on the load path's
// back-pressure stalls no MFMA: stage s + 1's pieces are issued right after the barrier that opens stage s and
// land while its MFMAs run. Same stage buffers, K order and epilogue as conv_stage_kernel (bit-identical).
template <int WM, int TAPS, int CG, int HROWS>
__global__ __launch_bounds__(768) void conv_ldr_kernel(const ConvArgs a) {
  constexpr int NWN = 4, WN = 4, NW = 8, NLD = 4;
  constexpr int BM = 32 * WM, BN = 64 * WN, NPA = BM / 16;
  constexpr int HP = (BN + HROWS + 15) / 16;
  constexpr int NA = TAPS * CG * NPA;
  constexpr int A_BYTES = NA * 1024, STAGE = A_BYTES + CG * HP * 1024;
  constexpr int PARTS = BN * (BM + 4) * 4 <= 2 * STAGE ? 1 : 2, TILE_BYTES = BN / PARTS * (BM + 4) * 4;
  constexpr int LDS_BYTES = 2 * STAGE > TILE_BYTES ? 2 * STAGE : TILE_BYTES;
  static_assert(LDS_BYTES <= 160 * 1024, "stage buffers exceed the CU's LDS");
  __shared__ __attribute__((aligned(1024))) char lds_raw[LDS_BYTES];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool loader = wave >= NW;
  const int lw = wave - NW;
  const int wm = (loader ? 0 : wave) / NWN, wn = (loader ? 0 : wave) % NWN;
  f32x4_t acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int co_blk = blockIdx.y * BM, q_blk = blockIdx.x * BN;
  const int rho = blockIdx.z;
  const f16_t* const wts = a.w + (size_t)rho * a.w_phase;
  const int in_off = a.nphase > 1 ? (rho + a.phase_pad) / a.out_stride : a.in_off;
  const int out_phase = a.nphase > 1 ? rho : a.out_phase;
  const int prow = lane >> 2, pchunk = (lane & 3) ^ (((lane >> 4) & 1) << 1);
  const int am = wm * (16 * WM), bn = wn * (16 * WN);
  const int span = (TAPS - 1) * abs(a.tap_step);
  const int omin = in_off + min(0, (TAPS - 1) * a.tap_step);
  const int nbp = (BN + span + 15) / 16;
  const int nstages = a.c_in / (32 * CG);
  const int nci = a.c_in / 32;
  const f16_t* const a_src = wts + (TAPS == 1 ? (size_t)(co_blk + prow) * a.c_in : (size_t)(co_blk + prow) * 32) +
                             pchunk * 8;
  const unsigned lbase =
      __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) char*)lds_raw);
  auto issue = [&](int s) {  // this loader's pieces of stage s: weight pieces lw, lw + 4, ..., then halo pieces
    const unsigned buf = lbase + (unsigned)((s & 1) * STAGE);
#pragma unroll
    for (int k = 0; k < (NA + NLD - 1) / NLD; ++k) {
      const int P = lw + NLD * k;
      if (P < NA) {
        const int g = P / (TAPS * NPA), r = P - g * (TAPS * NPA), tap = r / NPA, p = r - tap * NPA;
        glds16_at(a_src + (TAPS == 1 ? (size_t)16 * p * a.c_in + (s * CG + g) * 32
                                     : ((size_t)(tap * nci + s * CG + g) * a.c_out + 16 * p) * 32),
                  buf + (unsigned)(P * 1024));
      }
    }
    for (int P = lw; P < CG * nbp; P += NLD) {
      const int g = CG == 1 ? 0 : P / nbp, p = P - g * nbp;
      const int tin = q_blk + omin + 16 * p + prow;
      const bool ok = tin >= 0 && tin < a.t_in;
      glds16_at(ok ? (const void*)(a.x + (size_t)tin * a.c_in + (s * CG + g) * 32 + pchunk * 8)
                   : (const void*)&g_conv_zero[lane & 3],
                buf + (unsigned)(A_BYTES + (g * HP + p) * 1024));
    }
  };
  if (loader) issue(0);
  ConvEpiChan<WM, 512> ch;
  ch.load(a, co_blk);
  constexpr int G = CG * TAPS;
  for (int s = 0; s < nstages; ++s) {
    if (loader) wait_vm(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // every wave is done with stage s - 1, whose buffer the loaders now fill with stage s + 1
    if (loader) {
      if (s + 1 < nstages) issue(s + 1);
    } else {
      const char* const buf = lds_raw + (s & 1) * STAGE;
      if constexpr (WM >= 4) {  // 168 VGPRs (3 waves per SIMD): no room for a second fragment set
#pragma unroll
        for (int u = 0; u < G; ++u) {
          const int g = u / TAPS, tap = u - g * TAPS;
          conv_mfma<WM, WN>(acc, buf + u * NPA * 1024, buf + A_BYTES + g * HP * 1024, in_off + tap * a.tap_step - omin,
                            am, bn, lane);
        }
      } else {
        ConvFrag<WM, WN> fr[2];
        conv_load(fr[0], buf, buf + A_BYTES, in_off - omin, am, bn, lane);
#pragma unroll
        for (int u = 0; u < G; ++u) {
          if (u + 1 < G) {
            const int g = (u + 1) / TAPS, tap = (u + 1) - g * TAPS;
            conv_load(fr[(u + 1) & 1], buf + (u + 1) * NPA * 1024, buf + A_BYTES + g * HP * 1024,
                      in_off + tap * a.tap_step - omin, am, bn, lane);
          }
          __builtin_amdgcn_sched_barrier(0);
          conv_compute(acc, fr[u & 1]);
        }
      }
    }
    asm volatile("" ::: "memory");
  }
  __syncthreads();
  conv_epilogue<WM, WN, NWN, PARTS>(a, acc, lds_raw, wn, am, lane, q_blk, co_blk, out_phase, ch, !loader);
}

// quantizer.from_codes (modeling_dac.py:347-371): 9 x [codebook gather (8-d) -> 1x1 conv to 1024 + bias], summed
__global__ __launch_bounds__(256) void from_codes_kernel(const int64_t* codes, int T, const float* cbooks,
                                                          const float* pw, const float* pb, f16_t* z) {
  const int t = blockIdx.x;
  __shared__ float lat[ZMI_NCB][8];
  if (threadIdx.x < ZMI_NCB * 8) {
    const int i = threadIdx.x >> 3, j = threadIdx.x & 7;
    int64_t tok = codes[(size_t)i * T + t];
    tok = tok < 0 ? 0 : (tok > 1023 ? 1023 : tok);
    lat[i][j] = cbooks[((size_t)i * 1024 + tok) * 8 + j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 1024; c += 256) {
    float acc = 0.f;
    for (int i = 0; i < ZMI_NCB; ++i) {
      float s = 0.f;
      const float* wr = pw + ((size_t)i * 1024 + c) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) s += wr[j] * lat[i][j];
      acc = acc + (s + pb[i * 1024 + c]);
    }
    z[(size_t)t * 1024 + c] = (f16_t)f2h(acc);
  }
}

// encoder.conv1 input (modeling_dac.py:451, Conv1d(1, 64, k7, pad 3)) as a 32-channel im2col row per
// sample: col[t][k] = wav[t + k - 3] for k < 7 (0 outside the signal), 0 for k >= 7, so the conv runs on
// the MFMA conv kernel with one tap and c_in = 32
__global__ __launch_bounds__(256) void im2col7_kernel(const float* wav, int T, f16_t* col) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= T) return;
  uint32_t w[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    float v0 = 0.f, v1 = 0.f;
    const int k0 = 2 * k, k1 = 2 * k + 1;
    if (k0 < 7 && t + k0 - 3 >= 0 && t + k0 - 3 < T) v0 = wav[t + k0 - 3];
    if (k1 < 7 && t + k1 - 3 >= 0 && t + k1 - 3 < T) v1 = wav[t + k1 - 3];
    w[k] = f2h(v0) | (f2h(v1) << 16);
  }
  uint4* dst = reinterpret_cast<uint4*>(col + (size_t)t * 32);
#pragma unroll
  for (int i = 0; i < 4; ++i) dst[i] = uint4{w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]};
}

// Residual vector quantizer, one workgroup per frame (modeling_dac.py:283-345 with DacVectorQuantize
// :123-173): for each of the 9 codebooks, proj = in_proj(r) (8 outputs), e = proj / max(|proj|, 1e-12),
// score_j = -(|e|^2 - 2 e.cbn_j) + |cbn_j|^2 over the l2-normalised codebook, idx = first argmax,
// z = proj + (codebook[idx] - proj), r -= out_proj(z). fp32 throughout; latents [T][1024].
__global__ __launch_bounds__(256) void vq_kernel(const float* lat, int T, const float* in_w, const float* in_b,
                                                 const float* cb, const float* cbn, const float* cbn2,
                                                 const float* out_w, const float* out_b, int64_t* codes) {
  __shared__ float r[1024];
  __shared__ float proj[8], zq[8];
  __shared__ float bv[4];
  __shared__ int bi[4];
  const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  for (int c = t; c < 1024; c += 256) r[c] = lat[(size_t)f * 1024 + c];
  __syncthreads();
  for (int i = 0; i < ZMI_NCB; ++i) {
    // in_proj: wave w -> outputs 2w, 2w+1
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 2 * wave + h;
      const float* wr = in_w + ((size_t)i * 8 + k) * 1024;
      float s = 0.f;
#pragma unroll
      for (int m = 0; m < 16; ++m) s += wr[lane + 64 * m] * r[lane + 64 * m];
      s = wave_sum(s);
      if (lane == 0) proj[k] = s + in_b[i * 8 + k];
    }
    __syncthreads();
    float p[8], e[8], nrm = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      p[k] = proj[k];
      nrm += p[k] * p[k];
    }
    const float den = fmaxf(sqrtf(nrm), 1e-12f);
    float l2 = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      e[k] = p[k] / den;
      l2 += e[k] * e[k];
    }
    float best = -INFINITY;
    int bidx = 0;
    for (int m = 0; m < 4; ++m) {
      const int j = t + 256 * m;
      const float* cr = cbn + ((size_t)i * 1024 + j) * 8;
      float dot = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) dot += e[k] * cr[k];
      const float sc = -(l2 - 2.f * dot) + cbn2[i * 1024 + j];
      if (sc > best) {
        best = sc;
        bidx = j;
      }
    }
    // block argmax, ties -> lowest index
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const float ov = __shfl_xor(best, off);
      const int oi = __shfl_xor(bidx, off);
      if (ov > best || (ov == best && oi < bidx)) {
        best = ov;
        bidx = oi;
      }
    }
    if (lane == 0) {
      bv[wave] = best;
      bi[wave] = bidx;
    }
    __syncthreads();
    if (t == 0) {
      float bb = bv[0];
      int ii = bi[0];
      for (int w = 1; w < 4; ++w)
        if (bv[w] > bb || (bv[w] == bb && bi[w] < ii)) {
          bb = bv[w];
          ii = bi[w];
        }
      codes[(size_t)i * T + f] = ii;
#pragma unroll
      for (int k = 0; k < 8; ++k) zq[k] = p[k] + (cb[((size_t)i * 1024 + ii) * 8 + k] - p[k]);
    }
    __syncthreads();
    float z[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = zq[k];
    for (int c = t; c < 1024; c += 256) {
      const float* wr = out_w + ((size_t)i * 1024 + c) * 8;
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) s += wr[k] * z[k];
      r[c] = r[c] - (s + out_b[i * 1024 + c]);
    }
    __syncthreads();
  }
}

}  // namespace

extern "C" int zmi_dac_im2col7(const float* wav, int t, void* col, void* stream) {
  if (t <= 0) return 0;
  hipLaunchKernelGGL(im2col7_kernel, dim3((t + 255) / 256), dim3(256), 0, (hipStream_t)stream, wav, t, (f16_t*)col);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_dac_vq(const float* latents, int t, const float* in_w, const float* in_b, const float* codebooks,
                          const float* codebooks_n, const float* codebooks_n2, const float* out_w, const float* out_b,
                          int64_t* codes, void* stream) {
  if (t <= 0) return 0;
  hipLaunchKernelGGL(vq_kernel, dim3(t), dim3(256), 0, (hipStream_t)stream, latents, t, in_w, in_b, codebooks,
                     codebooks_n, codebooks_n2, out_w, out_b, codes);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_dac_from_codes(const int64_t* codes, int T, const float* codebooks, const float* proj_w,
                                  const float* proj_b, void* z, void* stream) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(from_codes_kernel, dim3(T), dim3(256), 0, (hipStream_t)stream, codes, T, codebooks, proj_w,
                     proj_b, (f16_t*)z);
  ZMI_CHECK(hipGetLastError());
  return 0;
}

// Tile height: the largest BM = 32 WM (WM in 4, 3, 2, 1, dividing c_out) whose grid still gives every CU
// about two workgroups; the early, few-frame stages (conv1 and block 0 at 861 frames: 84-336 workgroups at
// BM = 128) are latency-bound per workgroup, so more, shorter tiles finish sooner there.
template <int NWN>
static int launch_conv_t(const ConvArgs& a, hipStream_t s) {
  constexpr int WN = 4, BN = 16 * WN * NWN, NT = 128 * NWN;
  const unsigned nq = (unsigned)((a.n_out + BN - 1) / BN), nz = (unsigned)a.nphase;
  const int want = 256 / (NWN / 2);
  int wm = 0;
  for (int c : {4, 3, 2, 1})
    if (a.c_out % (32 * c) == 0) {
      wm = c;
      if ((long)nq * nz * (a.c_out / (32 * c)) >= want) break;
    }
  if (!wm) return zmi_fail_msg("dac_conv: c_out must be a multiple of 32");
  const dim3 grid(nq, (unsigned)(a.c_out / (32 * wm)), nz);
  // ring depth 2: measured against 3 and 4 (3.60 / 3.74 / 4.14 ms DAC decode at 861 frames): the deeper
  // rings' LDS costs more than their extra step of load lookahead gains
  const int span = (a.taps - 1) * abs(a.tap_step);
  // the halo K order wherever the taps' rows fit its buffer (every DAC conv: dilation <= 9, span <= 54);
  // measured 3.7 -> 3.15 ms DAC decode, 2.11 -> 1.83 ms encode at 861 frames against the tap-major order
  const bool halo = span <= HALO_TAPS_ROWS;
#define ZMI_CONV_L(wm_)                                                                               \
  do {                                                                                                \
    if (halo) hipLaunchKernelGGL((conv_kernel<wm_, WN, 2, true, NWN>), grid, dim3(NT), 0, s, a);      \
    else hipLaunchKernelGGL((conv_kernel<wm_, WN, 2, false, NWN>), grid, dim3(NT), 0, s, a);          \
  } while (0)
  switch (wm) {
    case 4: ZMI_CONV_L(4); break;
    case 3: ZMI_CONV_L(3); break;
    case 2: ZMI_CONV_L(2); break;
    default: ZMI_CONV_L(1); break;
  }
#undef ZMI_CONV_L
  return 0;
}

// Tile height: the largest BM = 32 WM (WM in 4, 3, 2, 1, dividing c_out) whose grid still gives every CU
// about two workgroups; the early, few-frame stages (conv1 and block 0 at 861 frames: 84-336 workgroups at
// BM = 128) are latency-bound per workgroup, so more, shorter tiles finish sooner there. Time tile: 256 rows
// (512 threads) where ZMI_OPT_DAC_WIDE allows it and the output has at least that many rows per CU-pair of
// workgroups, else 128 (256 threads).
// The staged form (conv_stage_kernel) for the conv classes ZMI_OPT_DAC_STAGE enables (bit 0: the k7 convs, bit 1:
// the 1x1 convs, bit 2: the transposed convs' 2-tap phases), at the largest tile height whose grid has at least
// ZMI_OPT_DAC_STAGE_MIN workgroups (one per CU: the stage buffers take most of the LDS). Returns 1 where the
// conv is not one of those (the caller launches conv_kernel), else 0 or the launch error.
static int launch_stage(const ConvArgs& a, hipStream_t s) {
  const int mask = zmi_option(ZMI_OPT_DAC_STAGE);
  const int span = (a.taps - 1) * abs(a.tap_step);
  int cls, cg;
  if (a.taps == 7 && span <= 64) cls = 0, cg = 1;
  else if (a.taps == 1) cls = 1, cg = a.c_in % 64 == 0 ? 2 : (a.c_in % 96 == 0 ? 3 : 0);
  else if (a.taps == 2 && span <= 16) cls = 2, cg = a.c_in % 64 == 0 ? 2 : 0;
  else return 1;
  // decoder.conv2's 32-channel (zero-padded) tile: 16 channels per wave and 8 waves along time, slower than
  // conv_kernel there (40.7 against 31-33 us at 861 frames)
  if (!(mask >> cls & 1) || !cg || a.c_out < 64) return 1;
  // 512-row time tiles (WN = 8, bit 3) for the k7 convs: half the weight bytes per MFMA of the 256-row tile, at
  // most 96 channels per tile (LDS)
  // A grid with too few 512-row tiles (conv1 at 861 frames: 96) takes the 256-row tiles before conv_kernel (its 192
  // workgroups: 40 us against 136 on conv_kernel).
  const long min_wg = zmi_option(ZMI_OPT_DAC_STAGE_MIN);
  const unsigned nz = (unsigned)a.nphase;
  auto pick = [&](int bn, int wm_max, unsigned* nq_out) {  // the largest tile height whose grid reaches min_wg
    const unsigned nq = (unsigned)((a.n_out + bn - 1) / bn);
    int w = 0;
    for (int c : {4, 3, 2, 1})
      if (c <= wm_max && a.c_out % (32 * c) == 0) {
        w = c;
        if ((long)nq * nz * (a.c_out / (32 * c)) >= min_wg) break;
      }
    *nq_out = nq;
    return w && (long)nq * nz * (a.c_out / (32 * w)) >= min_wg ? w : 0;
  };
  unsigned nq = 0;
  bool wide = cls == 0 && (mask & 8);
  int wm = wide ? pick(512, 3, &nq) : 0;
  if (!wm) {
    wide = false;
    wm = pick(256, 4, &nq);
  }
  if (!wm) return 1;
  if (cls == 1 && cg == 3 && wm < 3) return 1;  // instantiated for the 96-channel stages only
  const dim3 grid(nq, (unsigned)(a.c_out / (32 * wm)), nz);
#define ZMI_STAGE_L(wm_, wn_, taps_, cg_, hrows_) \
  hipLaunchKernelGGL((conv_stage_kernel<wm_, wn_, taps_, cg_, hrows_>), grid, dim3(512), 0, s, a)
#define ZMI_STAGE_WM(wn_, taps_, cg_, hrows_)                \
  switch (wm) {                                              \
    case 4: ZMI_STAGE_L(4, wn_, taps_, cg_, hrows_); break;  \
    case 3: ZMI_STAGE_L(3, wn_, taps_, cg_, hrows_); break;  \
    case 2: ZMI_STAGE_L(2, wn_, taps_, cg_, hrows_); break;  \
    default: ZMI_STAGE_L(1, wn_, taps_, cg_, hrows_); break; \
  }
  if ((mask & 16) && !wide && (cls == 0 || cls == 2)) {
#define ZMI_LDR_L(wm_, taps_, cg_, hrows_) \
  hipLaunchKernelGGL((conv_ldr_kernel<wm_, taps_, cg_, hrows_>), grid, dim3(768), 0, s, a)
    if (cls == 0) {
      switch (wm) {
        case 4: ZMI_LDR_L(4, 7, 1, 64); break;
        case 3: ZMI_LDR_L(3, 7, 1, 64); break;
        case 2: ZMI_LDR_L(2, 7, 1, 64); break;
        default: ZMI_LDR_L(1, 7, 1, 64); break;
      }
    } else {
      switch (wm) {
        case 4: ZMI_LDR_L(4, 2, 2, 16); break;
        case 3: ZMI_LDR_L(3, 2, 2, 16); break;
        case 2: ZMI_LDR_L(2, 2, 2, 16); break;
        default: ZMI_LDR_L(1, 2, 2, 16); break;
      }
    }
#undef ZMI_LDR_L
  } else if (wide) {
    switch (wm) {
      case 3: ZMI_STAGE_L(3, 8, 7, 1, 64); break;
      case 2: ZMI_STAGE_L(2, 8, 7, 1, 64); break;
      default: ZMI_STAGE_L(1, 8, 7, 1, 64); break;
    }
  } else if (cls == 0) {
    ZMI_STAGE_WM(4, 7, 1, 64)
  } else if (cls == 2) {
    ZMI_STAGE_WM(4, 2, 2, 16)
  } else if (cg == 2) {
    ZMI_STAGE_WM(4, 1, 2, 0)
  } else if (wm == 4) {
    ZMI_STAGE_L(4, 4, 1, 3, 0);
  } else {
    ZMI_STAGE_L(3, 4, 1, 3, 0);
  }
#undef ZMI_STAGE_WM
#undef ZMI_STAGE_L
  return 0;
}

static int launch_conv(const ConvArgs& a, hipStream_t s) {
  const int st = launch_stage(a, s);
  if (st != 1) return st;
  const int wide = zmi_option(ZMI_OPT_DAC_WIDE);
  if (wide == 2 || (wide == 1 && (long)a.n_out * a.nphase * (a.c_out / 32) >= (long)zmi_option(ZMI_OPT_DAC_WIDE_MIN) * 256))
    return launch_conv_t<4>(a, s);
  return launch_conv_t<2>(a, s);
}

extern "C" int zmi_dac_conv(const void* x, int t_in, int c_in, const void* w, const float* bias, int c_out, int taps,
                            int tap_step, int in_off, int n_out, int out_stride, int out_phase, int t_out,
                            const void* skip, void* out_raw, void* out_snake, const float* alpha, float* out_f32,
                            void* stream) {
  if (c_in % 32) return zmi_fail_msg("dac_conv: c_in % 32");
  if (n_out <= 0) return 0;
  if ((size_t)(n_out - 1) * out_stride + out_phase >= (size_t)t_out) return zmi_fail_msg("dac_conv: output bounds");
  ConvArgs a{(const f16_t*)x, t_in, c_in, (const f16_t*)w, bias, c_out, taps, tap_step, in_off, n_out,
             out_stride, out_phase, t_out, (const f16_t*)skip, (f16_t*)out_raw, (f16_t*)out_snake, alpha, out_f32, 0, 1, 0, 0};
  hipStream_t s = (hipStream_t)stream;
  // 128-step time tiles: 64- and 32-step tiles measured 15 % and 65 % slower (more workgroups do
  // not hide the per-K-step load latency)
  const int rc = launch_conv(a, s);
  if (rc) return rc;
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_dac_conv_out(const void* x, int t, int c_in, const void* w_pad, const float* bias_pad, float* out,
                                void* stream) {
  // decoder.conv2 (c_in -> 1, k7, pad 3) + tanh (modeling_dac.py:438-441) on the MFMA conv kernel: w_pad is
  // [7][32][c_in] fp16 with output channel 0 the real filter and 1..31 zero, bias_pad [32]; x already Snake'd
  if (c_in % 32) return zmi_fail_msg("dac_conv_out: c_in % 32");
  if (t <= 0) return 0;
  ConvArgs a{(const f16_t*)x, t, c_in, (const f16_t*)w_pad, bias_pad, 32, 7, 1, -3, t, 1, 0, t,
             nullptr, nullptr, nullptr, nullptr, out, 1, 1, 0, 0};
  const int rc = launch_conv(a, (hipStream_t)stream);
  if (rc) return rc;
  ZMI_CHECK(hipGetLastError());
  return 0;
}

extern "C" int zmi_dac_conv_t(const void* x, int t_in, int c_in, const void* w_phases, const float* bias, int c_out,
                              int stride, int pad, void* out_raw, void* out_snake, const float* alpha, void* stream) {
  // ConvTranspose1d(c_in, c_out, k = 2 stride, stride, padding = pad) (modeling_dac.py:222-240) in polyphase
  // form, all phases in one launch: out[stride q + rho] = bias + W_rho[0] x[q + c] + W_rho[1] x[q + c - 1],
  // c = (rho + pad) / stride; w_phases fp16 [stride][2][c_in / 32][c_out][32] (W_rho[j] = w[:, :, (rho + pad) % stride
  // + j stride]^T); output length stride * t_in
  if (c_in % 32) return zmi_fail_msg("dac_conv_t: c_in % 32");
  if (t_in <= 0) return 0;
  if (stride < 1 || pad < 0) return zmi_fail_msg("dac_conv_t: stride >= 1, pad >= 0");
  ConvArgs a{(const f16_t*)x, t_in, c_in, (const f16_t*)w_phases, bias, c_out, 2, -1, 0, t_in, stride, 0,
             stride * t_in, nullptr, (f16_t*)out_raw, (f16_t*)out_snake, alpha, nullptr, 0, stride, pad,
             (size_t)2 * c_out * c_in};
  const int rc = launch_conv(a, (hipStream_t)stream);
  if (rc) return rc;
  ZMI_CHECK(hipGetLastError());
  return 0;
}
