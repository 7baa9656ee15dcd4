// Exchange-latency probe: how long does one all-to-all granule exchange between G workgroups
// take when the workgroups sit on ONE XCD (its L2 is their coherence point) versus spread over
// all eight (every granule crosses the fabric)?  k_simple's per-pod exchange (C2: 40 shards)
// is the single largest phase of the headline loop, so this decides whether an
// XCD-local shard group is worth building.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/xcd_exchange_probe tools/xcd_exchange_probe.hip
//   tools/xcd_exchange_probe [G] [rounds]
//
// One wave per workgroup exchanges.  Round r: lane 0 publishes {r, shard} into slot
// [r & 1][shard] of the granule buffer; lanes 0..G-1 poll slot [r & 1][lane] until it carries
// epoch r (data-is-flag, MI355X_MICROARCH.md R2).  Variants:
//   spread/sc1     workgroups 0..G-1 (round-robin over the XCDs), sc1 stores and loads
//   xcd0/sc1       the first G workgroups that find themselves on XCD 0, sc1 stores and loads
//   xcd0/volatile  the same group, volatile stores (gfx950: sc0 sc1) and sc1 loads
//   spread/volat   workgroups 0..G-1, volatile stores, sc1 loads
//   xcd0/plain     the XCD-0 group, plain stores (no cache bits: the line stays in XCD 0's L2)
//                  and sc1 loads (L1 bypassed, served by that L2)
// Every spin is bounded (the run reports a timeout instead of hanging).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                              \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      exit(2);                                                                                \
    }                                                                                         \
  } while (0)

__device__ __forceinline__ int xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xF;
}

constexpr long long WAIT = 200000000ll;  // 2 s of s_memrealtime (100 MHz)

template <int MODE>  // 0 spread/sc1, 1 xcd0/sc1, 2 xcd0/volatile, 3 spread/volatile, 4 xcd0/plain
__global__ __launch_bounds__(64) void k_probe(unsigned long long* gran, int G, int rounds, int* cnt, long long* out,
                                              int* fail) {
  __shared__ int sh_slot;
  const int lane = threadIdx.x;
  if (lane == 0) {
    int slot = -1;
    if (MODE == 0 || MODE == 3) {
      slot = blockIdx.x < (unsigned)G ? (int)blockIdx.x : -1;
    } else if (xcc_id() == 0) {
      const int s = atomicAdd(cnt, 1);
      slot = s < G ? s : -1;
    }
    sh_slot = slot;
  }
  __syncthreads();
  const int me = sh_slot;
  if (me < 0) return;
  long long t0 = 0;
  for (int r = 1; r <= rounds; r++) {
    if (r == 2 && me == 0 && lane == 0) t0 = (long long)__builtin_amdgcn_s_memrealtime();  // round 1 = the handshake
    unsigned long long* base = gran + (size_t)(r & 1) * 256;
    const unsigned long long v = ((unsigned long long)r << 32) | (unsigned)me;
    if (lane == 0) {
      if (MODE == 2 || MODE == 3) {
        *(volatile __attribute__((address_space(1))) unsigned long long*)(base + me) = v;
      } else if (MODE == 4) {
        asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(base + me), "v"(v) : "memory");
      } else {
        __hip_atomic_store(base + me, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    const long long ts = (long long)__builtin_amdgcn_s_memrealtime();
    for (unsigned spins = 0;; spins++) {
      bool ok = true;
      if (lane < G) {
        const unsigned long long g = __hip_atomic_load(base + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = (g >> 32) == (unsigned long long)r;
      }
      if (__all(ok)) break;
      if ((spins & 63) == 63 && (long long)__builtin_amdgcn_s_memrealtime() - ts > WAIT) {
        if (lane == 0) atomicAdd(fail, 1);
        return;
      }
    }
  }
  if (me == 0 && lane == 0) out[0] = (long long)__builtin_amdgcn_s_memrealtime() - t0;
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? atoi(argv[1]) : 32;
  const int rounds = argc > 2 ? atoi(argv[2]) : 20000;
  if (G < 1 || G > 64) return fprintf(stderr, "G in [1, 64]\n"), 2;
  unsigned long long* gran;
  int *cnt, *fail;
  long long* out;
  CHECK(hipMalloc(&gran, 2 * 256 * 8));
  CHECK(hipMalloc(&cnt, 4));
  CHECK(hipMalloc(&fail, 4));
  CHECK(hipMalloc(&out, 8));
  const char* names[5] = {"spread/sc1", "xcd0/sc1", "xcd0/volatile", "spread/volat", "xcd0/plain"};
  for (int rep = 0; rep < 2; rep++) {
    for (int mode = 0; mode < 5; mode++) {
      CHECK(hipMemset(gran, 0, 2 * 256 * 8));
      CHECK(hipMemset(cnt, 0, 4));
      CHECK(hipMemset(fail, 0, 4));
      CHECK(hipMemset(out, 0, 8));
      const bool spread = mode == 0 || mode == 3;
      const int blocks = spread ? G : 8 * 64;  // enough workgroups for G of them to land on XCD 0
      if (mode == 0) hipLaunchKernelGGL(k_probe<0>, dim3(blocks), dim3(64), 0, 0, gran, G, rounds, cnt, out, fail);
      if (mode == 1) hipLaunchKernelGGL(k_probe<1>, dim3(blocks), dim3(64), 0, 0, gran, G, rounds, cnt, out, fail);
      if (mode == 2) hipLaunchKernelGGL(k_probe<2>, dim3(blocks), dim3(64), 0, 0, gran, G, rounds, cnt, out, fail);
      if (mode == 3) hipLaunchKernelGGL(k_probe<3>, dim3(blocks), dim3(64), 0, 0, gran, G, rounds, cnt, out, fail);
      if (mode == 4) hipLaunchKernelGGL(k_probe<4>, dim3(blocks), dim3(64), 0, 0, gran, G, rounds, cnt, out, fail);
      CHECK(hipGetLastError());
      CHECK(hipDeviceSynchronize());
      int f = 0, c = 0;
      long long t = 0;
      CHECK(hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(&c, cnt, 4, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(&t, out, 8, hipMemcpyDeviceToHost));
      printf("rep %d %-11s G=%d on-XCD0=%d failures=%d  %.3f us per exchange round\n", rep, names[mode], G,
             spread ? -1 : c, f, f ? -1.0 : t * 0.01 / (rounds - 1));
    }
  }
  return 0;
}
