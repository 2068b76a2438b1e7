// Timing-only probe (not product code): how fast can the decode attention's K / V cache reads run, alone?
// Reads the caches of zmi_attn.hip's layout (K [row][kv head][pos][128], V^T [row][kv head][128][smax], bf16)
// for `rows` x `hkv` units of `pos + 1` keys, in 128-key chunks, and folds every loaded word into one
// XOR per wave (so no load is dead). Modes:
//   0 attn     one 4-wave workgroup per (unit, chunk), the attention kernel's loads (K: 16 keys x 64 B per
//              instruction, V^T: 16 dim rows x 64 B), all issued at once
//   1 linear   same workgroups and bytes, 1 KiB-contiguous instructions (K: 4 keys, V^T: 4 dim rows)
//   3 konly    the attention's K loads only;  4 vonly  its V^T loads only;  5 vlin  V^T only, 1 KiB-contiguous
//              instructions (4 dim rows x 256 B)
//   6 vtile    V^T only, stored in 128-position tiles ([unit][tile][128 dims][128 positions]: a chunk's V is one
//              contiguous 32 KiB), the attention's per-instruction shape (16 dim rows x 64 B)
//   7 vfinish  mode 4 plus the finish launch's other reads: 2 KiB of scores and the maxima of the chunks before
//   2 stream   persistent: gridDim workgroups walk the chunks (c = blockIdx, + gridDim), the attention
//              loads of the next chunk issued before the current one is folded (2 chunks in flight)
// Occupancy is capped by the dynamic LDS size the driver passes. Built by tools/kv_probe.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int HD = 128, CH = 128;

struct Args {
  const uint16_t* k;
  const uint16_t* v;
  uint32_t* out;
  int units, nch, smax, pos;
};

__device__ __forceinline__ uint32_t fold(uint4 a) { return a.x ^ a.y ^ a.z ^ a.w; }

__device__ __forceinline__ void chunk_loads(const Args& a, int unit, int c, int wave, int lane, uint4 (&kf)[8],
                                            uint4 (&vf)[8]) {
  const int c16 = lane & 15, h4 = lane >> 4;
  const size_t base = (size_t)unit * a.smax * HD;
  const int key0 = c * CH, last = min(key0 + CH - 1, a.pos);
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int key = min(key0 + wave * 32 + 16 * tt + c16, last);
#pragma unroll
    for (int db = 0; db < 4; ++db)
      kf[tt * 4 + db] = *reinterpret_cast<const uint4*>(a.k + base + (size_t)key * HD + 8 * h4 + 32 * db);
  }
  const int p0 = min(key0 + wave * 32 + 8 * h4, last & ~7);
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
    vf[dt] = *reinterpret_cast<const uint4*>(a.v + base + (size_t)(16 * dt + c16) * a.smax + p0);
}

__global__ __launch_bounds__(256) void probe_attn(Args a) {
  extern __shared__ char pad[];
  const int unit = blockIdx.x / a.nch, c = blockIdx.x % a.nch;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint4 kf[8], vf[8];
  chunk_loads(a, unit, c, wave, lane, kf, vf);
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x ^= fold(kf[i]) ^ fold(vf[i]);
  if (x == 0x9e3779b9u) pad[threadIdx.x] = 1;  // never (keeps the LDS allocation)
  a.out[blockIdx.x * 256 + threadIdx.x] = x;
}

template <int WHICH>  // 3 K only, 4 V^T only, 5 V^T linear, 6 V^T tiled, 7 V^T + finish reads
__global__ __launch_bounds__(256) void probe_half(Args a) {
  extern __shared__ char pad[];
  const int unit = blockIdx.x / a.nch, c = blockIdx.x % a.nch;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c16 = lane & 15, h4 = lane >> 4;
  const size_t base = (size_t)unit * a.smax * HD;
  const int key0 = c * CH, last = min(key0 + CH - 1, a.pos);
  uint4 f[8];
  if constexpr (WHICH == 3) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int key = min(key0 + wave * 32 + 16 * tt + c16, last);
#pragma unroll
      for (int db = 0; db < 4; ++db)
        f[tt * 4 + db] = *reinterpret_cast<const uint4*>(a.k + base + (size_t)key * HD + 8 * h4 + 32 * db);
    }
  } else if constexpr (WHICH == 4 || WHICH == 7) {
    const int p0 = min(key0 + wave * 32 + 8 * h4, last & ~7);
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
      f[dt] = *reinterpret_cast<const uint4*>(a.v + base + (size_t)(16 * dt + c16) * a.smax + p0);
  } else if constexpr (WHICH == 6) {
    const int p0 = min(key0 + wave * 32 + 8 * h4, last & ~7);
    const size_t tb = base + (size_t)(p0 / 128) * 128 * 128 + (p0 % 128);
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) f[dt] = *reinterpret_cast<const uint4*>(a.v + tb + (size_t)(16 * dt + c16) * 128);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wave * 32 + i * 4 + (lane >> 4);
      f[i] = *reinterpret_cast<const uint4*>(a.v + base + (size_t)row * a.smax + min(key0 + 8 * (lane & 15), a.pos & ~7));
    }
  }
  uint32_t x = 0;
  if constexpr (WHICH == 7) {  // the scores slot (2 KiB) and the maxima of chunks 0 .. c (4 B each, stride 8 B)
    const float* sc = reinterpret_cast<const float*>(a.out) + (size_t)(gridDim.x + blockIdx.x) * 512;
    if (threadIdx.x < 128) x ^= fold(*reinterpret_cast<const uint4*>(sc + threadIdx.x * 4));
    const int dep = min((c / 4 + 1) * 4, a.nch);
    const float* lm = reinterpret_cast<const float*>(a.out) + (size_t)3 * gridDim.x * 512 + (size_t)unit * a.nch * 8;
    if (threadIdx.x < dep * 4) x ^= __float_as_uint(lm[2 * threadIdx.x + 1]);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) x ^= fold(f[i]);
  if (x == 0x9e3779b9u) pad[threadIdx.x] = 1;
  a.out[blockIdx.x * 256 + threadIdx.x] = x;
}

__global__ __launch_bounds__(256) void probe_linear(Args a) {
  extern __shared__ char pad[];
  const int unit = blockIdx.x / a.nch, c = blockIdx.x % a.nch;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t base = (size_t)unit * a.smax * HD;
  const int key0 = c * CH;
  uint4 f[16];
  // K: the chunk's 128 keys x 256 B = 32 KiB, wave w its 8 KiB, 1 KiB per instruction
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int key = min(key0 + wave * 32 + i * 4 + (lane >> 4), a.pos);
    f[i] = *reinterpret_cast<const uint4*>(a.k + base + (size_t)key * HD + 8 * (lane & 15));
  }
  // V^T: 128 dim rows x 256 B at the chunk's positions, wave w rows 32 w .., 4 rows per instruction
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = wave * 32 + i * 4 + (lane >> 4);
    f[8 + i] = *reinterpret_cast<const uint4*>(a.v + base + (size_t)row * a.smax + min(key0 + 8 * (lane & 15), a.pos & ~7));
  }
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) x ^= fold(f[i]);
  if (x == 0x9e3779b9u) pad[threadIdx.x] = 1;
  a.out[blockIdx.x * 256 + threadIdx.x] = x;
}

__global__ __launch_bounds__(256) void probe_stream(Args a) {
  extern __shared__ char pad[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int total = a.units * a.nch;
  uint32_t x = 0;
  uint4 kf[2][8], vf[2][8];
  int b = blockIdx.x;
  if (b < total) chunk_loads(a, b / a.nch, b % a.nch, wave, lane, kf[0], vf[0]);
  for (int it = 0; b < total; ++it, b += gridDim.x) {
    const int nb = b + gridDim.x;
    if (nb < total) chunk_loads(a, nb / a.nch, nb % a.nch, wave, lane, kf[(it + 1) & 1], vf[(it + 1) & 1]);
    const int cur = it & 1;
#pragma unroll
    for (int i = 0; i < 8; ++i) x ^= fold(kf[cur][i]) ^ fold(vf[cur][i]);
  }
  if (x == 0x9e3779b9u) pad[threadIdx.x] = 1;
  a.out[blockIdx.x * 256 + threadIdx.x] = x;
}
}  // namespace

extern "C" int kv_probe(int mode, const void* k, const void* v, void* out, int units, int smax, int pos, int grid,
                        int lds_bytes, void* stream) {
  Args a{(const uint16_t*)k, (const uint16_t*)v, (uint32_t*)out, units, pos / CH + 1, smax, pos};
  hipStream_t s = (hipStream_t)stream;
  const unsigned blocks = (unsigned)(units * a.nch);
  if (mode == 0)
    hipLaunchKernelGGL(probe_attn, dim3(blocks), dim3(256), lds_bytes, s, a);
  else if (mode == 1)
    hipLaunchKernelGGL(probe_linear, dim3(blocks), dim3(256), lds_bytes, s, a);
  else if (mode == 2)
    hipLaunchKernelGGL(probe_stream, dim3(grid), dim3(256), lds_bytes, s, a);
  else if (mode == 3)
    hipLaunchKernelGGL(probe_half<3>, dim3(blocks), dim3(256), lds_bytes, s, a);
  else if (mode == 4)
    hipLaunchKernelGGL(probe_half<4>, dim3(blocks), dim3(256), lds_bytes, s, a);
  else if (mode == 5)
    hipLaunchKernelGGL(probe_half<5>, dim3(blocks), dim3(256), lds_bytes, s, a);
  else if (mode == 6)
    hipLaunchKernelGGL(probe_half<6>, dim3(blocks), dim3(256), lds_bytes, s, a);
  else
    hipLaunchKernelGGL(probe_half<7>, dim3(blocks), dim3(256), lds_bytes, s, a);
  return (int)hipGetLastError();
}
