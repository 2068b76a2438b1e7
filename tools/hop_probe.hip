// Hand-off latency probe (gfx950): ping-pong between two workgroups through 8-byte {round, tag} words.
//   hipcc -O3 --offload-arch=gfx950 tools/hop_probe.hip -o tools/hop_probe && tools/hop_probe
// store: 0 = agent-scope relaxed store (global_store sc1: write-through, the line leaves the XCD's L2),
//        1 = workgroup-scope relaxed store (plain global_store: the line stays in the writer's L2)
// loads: always agent-scope relaxed (sc1: bypass L1, L2-served). pair: 8 = partner block b ^ 8 (same XCD under
// round-robin dealing), 1 = b ^ 1 (another XCD). Spins are bounded: a hand-off that never becomes visible
// (expected for store 1 across XCDs) ends with the error word set instead of hanging.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void pingpong(uint64_t* slots, int rounds, int store, int pair, unsigned long long* out, unsigned* err) {
  const int b = blockIdx.x, p = b ^ pair;
  if (threadIdx.x != 0) return;
  const bool init = b < p;
  uint64_t* mine = slots + (size_t)b * 16;   // 128 B apart
  const uint64_t* theirs = slots + (size_t)p * 16;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int r = 1; r <= rounds; ++r) {
    if (init) {
      if (store) __hip_atomic_store(mine, (uint64_t)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else __hip_atomic_store(mine, (uint64_t)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    unsigned spins = 0;
    while (__hip_atomic_load(theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (uint64_t)r) {
      if (++spins > (1u << 20)) {
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        out[b * 2] = 0;
        return;
      }
    }
    if (!init) {
      if (store) __hip_atomic_store(mine, (uint64_t)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else __hip_atomic_store(mine, (uint64_t)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  out[b * 2] = __builtin_amdgcn_s_memrealtime() - t0;
  out[b * 2 + 1] = xcc;
}

int main() {
  uint64_t* slots;
  unsigned long long* out;
  unsigned* err;
  hipMalloc(&slots, 16 * 16 * 8);
  hipMalloc(&out, 16 * 2 * 8);
  hipMalloc(&err, 4);
  const int rounds = 2000;
  for (int store = 0; store < 2; ++store)
    for (int pair : {8, 1}) {
      hipMemset(slots, 0, 16 * 16 * 8);
      hipMemset(err, 0, 4);
      hipMemset(out, 0, 16 * 2 * 8);
      hipLaunchKernelGGL(pingpong, dim3(16), dim3(64), 0, 0, slots, rounds, store, pair, out, err);
      hipDeviceSynchronize();
      unsigned long long h[32];
      unsigned e;
      hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
      hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
      double us = 0;
      int n = 0;
      for (int b = 0; b < 16; ++b)
        if (h[2 * b]) { us += h[2 * b] / 100.0; ++n; }
      printf("{\"store\": \"%s\", \"pair\": \"b^%d\", \"err\": %u, \"ns_per_hop\": %.1f, \"xcc\": [", store ? "plain" : "sc1",
             pair, e, n ? us / n / (2.0 * rounds) * 1000.0 : -1.0);
      for (int b = 0; b < 16; ++b) printf("%llu%s", h[2 * b + 1], b < 15 ? ", " : "");
      printf("]}\n");
    }
  return 0;
}
