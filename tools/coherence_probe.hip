// Coherence probe: can a kernel read a value that a host-side copy (hipMemcpyAsync /
// hipMemsetAsync) overwrote after an earlier kernel stored it?  The many-chunk split-grid
// failure looked exactly like that: at the start of a run, a count row held the
// value the previous run had left, although kss_reset_node_state had copied the snapshot
// back in between.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/coherence_probe tools/coherence_probe.hip
//   tools/coherence_probe            (one line per variant: stale words out of checked words)
//
// Each iteration: K1 (one workgroup per CU) loads its slice (agent-scope loads, as k_spread's
// prologue), stores iteration-tagged values (as its epilogue); the host-side reset writes
// zeros; K2 loads every slice and counts nonzero words.  Variants change the reset, the load
// and store forms and the allocation.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#define CHECK(x)                                                                              \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      exit(2);                                                                                \
    }                                                                                         \
  } while (0)

constexpr int SLICE = 2048;

__device__ __forceinline__ int xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xF;
}

template <int LD, int ST>
__global__ void k_write(int* buf, int tag, int* xcc) {
  int* s = buf + (size_t)blockIdx.x * SLICE;
  int acc = 0;
  for (int i = threadIdx.x; i < SLICE; i += blockDim.x) {
    int v = LD ? __hip_atomic_load(s + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : s[i];
    acc += v;
  }
  for (int i = threadIdx.x; i < SLICE; i += blockDim.x) {
    const int v = tag + (acc & 0);
    if (ST) __hip_atomic_store(s + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else s[i] = v;
  }
  if (threadIdx.x == 0) xcc[blockIdx.x] = xcc_id();
}

// reset by a kernel: agent-scope stores of zero
__global__ void k_zero(int* buf, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    __hip_atomic_store(buf + i, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int LD, int ACQ>
__global__ void k_check(const int* buf, int* stale, int* xcc) {
  if (ACQ) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system-scope acquire
  const int* s = buf + (size_t)blockIdx.x * SLICE;
  int bad = 0;
  for (int i = threadIdx.x; i < SLICE; i += blockDim.x) {
    const int v = LD ? __hip_atomic_load(s + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : s[i];
    bad += v != 0;
  }
  if (bad) atomicAdd(&stale[blockIdx.x], bad);
  if (threadIdx.x == 0) xcc[blockIdx.x] = xcc_id();
}

// Cross-XCD hand-off between launches: every workgroup reads EVERY slice (so each XCD's L2
// may hold every line), then workgroup g rewrites slice g with a new tag, then every
// workgroup reads every slice again and counts words that are not the new tag.
template <int LD, int ACQ>
__global__ void k_read_all(const int* buf, size_t n, int tag, int* stale) {
  if (ACQ == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (ACQ == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  int bad = 0;
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) {
    const int v = LD ? __hip_atomic_load(buf + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : buf[i];
    bad += v != tag;
  }
  if (bad) atomicAdd(&stale[blockIdx.x], bad);
}

// writer that ends with an agent release (buffer_wbl2) after its stores
__global__ void k_write_rel(int* buf, int tag) {
  int* s = buf + (size_t)blockIdx.x * SLICE;
  for (int i = threadIdx.x; i < SLICE; i += blockDim.x) __hip_atomic_store(s + i, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
}

// background traffic on a second stream: short kernels whose starts and ends bring the
// runtime's cache maintenance while the hand-off runs
__global__ void k_noise(int* junk, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) junk[i] += 1;
}

// a part-1-like poller on another stream: 16 workgroups polling uncached memory with
// system-scope loads (s_sleep(1) between polls) until `ticks` of the 100 MHz clock pass
__global__ void k_poll(const unsigned long long* inbox, long long ticks, int* sink) {
  const long long t0 = wall_clock64();
  unsigned long long acc = 0;
  while (wall_clock64() - t0 < ticks) {
    acc += __hip_atomic_load(inbox + (threadIdx.x & 511), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_s_sleep(1);
  }
  if (acc == 12345) sink[0] = 1;
}

// writer whose every wave drains its stores (vmcnt(0)), then one agent release per workgroup
__global__ void k_write_drain(int* buf, int tag) {
  int* s = buf + (size_t)blockIdx.x * SLICE;
  int acc = 0;
  for (int i = threadIdx.x; i < SLICE; i += blockDim.x) acc += __hip_atomic_load(s + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int i = threadIdx.x; i < SLICE; i += blockDim.x) __hip_atomic_store(s + i, tag + (acc & 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// the split grid's exchange traffic: granules on the first line of 4 KiB blocks (G_XW = 512
// u64 per shard), polled with agent-scope loads and stored with system-scope stores, in
// uncached memory, by `npoll` workgroups, until `ticks` pass
__global__ void k_gran_poll(unsigned long long* inbox, int blocks, long long ticks, int* sink) {
  const long long t0 = wall_clock64();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned long long acc = 0;
  unsigned it = 0;
  while (wall_clock64() - t0 < ticks) {
    const int b = (lane + wave * 64 + (int)it) % blocks;
    unsigned long long* g = inbox + (size_t)b * 512 + (lane & 15);
    acc += __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wave == 0 && lane < 16 && (it & 7) == 0)
      __hip_atomic_store(inbox + (size_t)((blockIdx.x + it) % blocks) * 512 + lane, acc + it, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    ++it;
    __builtin_amdgcn_s_sleep(1);
  }
  if (acc == 12345) sink[0] = 1;
}

// every stale word's page-offset line (0 = the first 128 B of a 4 KiB page)
template <int LD>
__global__ void k_read_all_lines(const int* buf, size_t n, int tag, int* stale, int* by_line) {
  int bad = 0;
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) {
    const int v = LD ? __hip_atomic_load(buf + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : buf[i];
    if (v != tag) {
      bad++;
      atomicAdd(&by_line[(i * 4 % 4096) / 128], 1);
    }
  }
  if (bad) atomicAdd(&stale[blockIdx.x], bad);
}

enum Reset { R_MEMCPY_D2D, R_MEMCPY_H2D, R_MEMSET, R_KERNEL };
enum Alloc { A_DEFAULT, A_UNCACHED, A_FINE };

struct Variant {
  const char* name;
  Reset reset;
  Alloc alloc;
  int ld, st, acq;
};

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  int dev = 0, ncu = 0;
  CHECK(hipSetDevice(dev));
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int G = ncu;
  const size_t n = (size_t)G * SLICE, bytes = n * 4;
  const Variant vs[] = {
      {"d2d-copy   agent ld/st", R_MEMCPY_D2D, A_DEFAULT, 1, 1, 0},
      {"h2d-copy   agent ld/st", R_MEMCPY_H2D, A_DEFAULT, 1, 1, 0},
      {"memset     agent ld/st", R_MEMSET, A_DEFAULT, 1, 1, 0},
      {"kernel     agent ld/st", R_KERNEL, A_DEFAULT, 1, 1, 0},
      {"d2d-copy   plain ld/st", R_MEMCPY_D2D, A_DEFAULT, 0, 0, 0},
      {"d2d-copy   agent + sys acquire", R_MEMCPY_D2D, A_DEFAULT, 1, 1, 1},
      {"d2d-copy   uncached", R_MEMCPY_D2D, A_UNCACHED, 1, 1, 0},
      {"d2d-copy   fine-grained", R_MEMCPY_D2D, A_FINE, 1, 1, 0},
      {"memset     uncached", R_MEMSET, A_UNCACHED, 1, 1, 0},
  };
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int *zero_d, *stale_d, *xw_d, *xr_d;
  CHECK(hipMalloc(&zero_d, bytes));
  CHECK(hipMemset(zero_d, 0, bytes));
  CHECK(hipMalloc(&stale_d, 4 * G));
  CHECK(hipMalloc(&xw_d, 4 * G));
  CHECK(hipMalloc(&xr_d, 4 * G));
  std::vector<int> zero_h(n, 0), stale(G), xw(G), xr(G);
  int* zero_pinned;
  CHECK(hipHostMalloc(&zero_pinned, bytes, hipHostMallocDefault));
  memset(zero_pinned, 0, bytes);
  CHECK(hipDeviceSynchronize());
  // the hand-off under granule traffic on the first lines of 4 KiB blocks (mode 3)
  if (argc > 2 && atoi(argv[2]) == 3) {
    hipStream_t nb;
    CHECK(hipStreamCreateWithFlags(&nb, hipStreamNonBlocking));
    const int blocks = 64;
    unsigned long long* inbox;
    CHECK(hipExtMallocWithFlags((void**)&inbox, (size_t)blocks * 4096, hipDeviceMallocUncached));
    CHECK(hipMemset(inbox, 0, (size_t)blocks * 4096));
    int *sink, *by_line;
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMalloc(&by_line, 4 * 32));
    CHECK(hipMemset(by_line, 0, 4 * 32));
    int* buf = nullptr;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMemset(buf, 0, bytes));
    CHECK(hipDeviceSynchronize());
    long long bad_words = 0, bad_iters = 0, total = 0;
    for (int it = 0; it < iters; it++) {
      hipLaunchKernelGGL(k_gran_poll, dim3(32), dim3(512), 0, nb, inbox, blocks, 200000LL, sink);  // ~2 ms
      for (int rep = 0; rep < 8; rep++) {
        const int t = 8 * it + rep;
        hipLaunchKernelGGL((k_read_all_lines<1>), dim3(G), dim3(256), 0, st, buf, n, t, stale_d, by_line);
        hipLaunchKernelGGL((k_write<1, 1>), dim3(G), dim3(256), 0, st, buf, t + 1, xw_d);
        CHECK(hipMemsetAsync(stale_d, 0, 4 * G, st));
        hipLaunchKernelGGL((k_read_all_lines<1>), dim3(G), dim3(256), 0, st, buf, n, t + 1, stale_d, by_line);
        CHECK(hipGetLastError());
        CHECK(hipMemcpyAsync(stale.data(), stale_d, 4 * G, hipMemcpyDeviceToHost, st));
        CHECK(hipStreamSynchronize(st));
        long long b = 0;
        for (int g = 0; g < G; g++) b += stale[g];
        bad_words += b;
        bad_iters += b != 0;
        total++;
      }
      CHECK(hipStreamSynchronize(nb));
    }
    std::vector<int> bl(32);
    CHECK(hipMemcpy(bl.data(), by_line, 4 * 32, hipMemcpyDeviceToHost));
    printf("granule traffic: hand-off stale words %lld, hand-offs with stale %lld of %lld; stale by page line:", bad_words,
           bad_iters, total);
    for (int i = 0; i < 32; i++) printf(" %d", bl[i]);
    printf("\n");
    return 0;
  }
  // the hand-off while a second stream's persistent grid polls uncached memory (the split
  // grid's other part): mode 0 plain end, 1 drained + released end; each with / without reset
  if (argc > 2 && atoi(argv[2]) == 2) {
    hipStream_t nb;
    CHECK(hipStreamCreateWithFlags(&nb, hipStreamNonBlocking));
    unsigned long long* inbox;
    CHECK(hipExtMallocWithFlags((void**)&inbox, 1 << 16, hipDeviceMallocUncached));
    CHECK(hipMemset(inbox, 0, 1 << 16));
    int* sink;
    CHECK(hipMalloc(&sink, 64));
    const char* nm[] = {"poll: hand-off plain end", "poll: hand-off drained end", "poll: reset, plain end",
                        "poll: reset, drained end"};
    for (int mode = 0; mode < 4; mode++) {
      int* buf = nullptr;
      CHECK(hipMalloc(&buf, bytes));
      CHECK(hipMemset(buf, 0, bytes));
      CHECK(hipDeviceSynchronize());
      long long bad_words = 0, bad_iters = 0;
      const bool drain = mode & 1, reset = mode >= 2;
      for (int it = 0; it < iters; it++) {
        hipLaunchKernelGGL(k_poll, dim3(16), dim3(512), 0, nb, inbox, 100000LL, sink);  // ~1 ms
        for (int rep = 0; rep < 4; rep++) {
          const int t0 = reset ? 0 : 4 * it + rep, t1 = reset ? 0 : 4 * it + rep + 1;
          hipLaunchKernelGGL((k_read_all<1, 0>), dim3(G), dim3(256), 0, st, buf, n, t0, stale_d);
          if (drain) hipLaunchKernelGGL(k_write_drain, dim3(G), dim3(256), 0, st, buf, 4 * it + rep + 1);
          else hipLaunchKernelGGL((k_write<1, 1>), dim3(G), dim3(256), 0, st, buf, 4 * it + rep + 1, xw_d);
          if (reset) CHECK(hipMemcpyAsync(buf, zero_d, bytes, hipMemcpyDeviceToDevice, st));
          CHECK(hipMemsetAsync(stale_d, 0, 4 * G, st));
          hipLaunchKernelGGL((k_read_all<1, 0>), dim3(G), dim3(256), 0, st, buf, n, t1, stale_d);
          CHECK(hipGetLastError());
          CHECK(hipMemcpyAsync(stale.data(), stale_d, 4 * G, hipMemcpyDeviceToHost, st));
          CHECK(hipStreamSynchronize(st));
          long long b = 0;
          for (int g = 0; g < G; g++) b += stale[g];
          bad_words += b;
          bad_iters += b != 0;
        }
        CHECK(hipStreamSynchronize(nb));
      }
      printf("%-34s stale words %lld, hand-offs with stale %lld of %d\n", nm[mode], bad_words, bad_iters, 4 * iters);
      fflush(stdout);
      CHECK(hipFree(buf));
    }
    return 0;
  }
  // the hand-off (agent ld/st, d2d reset) while a second stream launches short kernels
  if (argc > 2 && atoi(argv[2]) == 1) {
    hipStream_t nb;
    CHECK(hipStreamCreateWithFlags(&nb, hipStreamNonBlocking));
    int* junk;
    CHECK(hipMalloc(&junk, 1 << 20));
    CHECK(hipMemset(junk, 0, 1 << 20));
    for (int mode = 0; mode < 2; mode++) {
      int* buf = nullptr;
      CHECK(hipMalloc(&buf, bytes));
      CHECK(hipMemset(buf, 0, bytes));
      CHECK(hipDeviceSynchronize());
      long long bad_words = 0, bad_iters = 0;
      for (int it = 0; it < iters; it++) {
        for (int j = 0; j < 16; j++) hipLaunchKernelGGL(k_noise, dim3(64), dim3(256), 0, nb, junk, 1 << 18);
        hipLaunchKernelGGL((k_read_all<1, 0>), dim3(G), dim3(256), 0, st, buf, n, mode == 1 ? 0 : it, stale_d);
        hipLaunchKernelGGL((k_write<1, 1>), dim3(G), dim3(256), 0, st, buf, it + 1, xw_d);
        if (mode == 1) CHECK(hipMemcpyAsync(buf, zero_d, bytes, hipMemcpyDeviceToDevice, st));
        for (int j = 0; j < 16; j++) hipLaunchKernelGGL(k_noise, dim3(64), dim3(256), 0, nb, junk, 1 << 18);
        CHECK(hipMemsetAsync(stale_d, 0, 4 * G, st));
        hipLaunchKernelGGL((k_read_all<1, 0>), dim3(G), dim3(256), 0, st, buf, n, mode == 1 ? 0 : it + 1, stale_d);
        CHECK(hipGetLastError());
        CHECK(hipMemcpyAsync(stale.data(), stale_d, 4 * G, hipMemcpyDeviceToHost, st));
        CHECK(hipStreamSynchronize(st));
        long long b = 0;
        for (int g = 0; g < G; g++) b += stale[g];
        bad_words += b;
        bad_iters += b != 0;
      }
      CHECK(hipDeviceSynchronize());
      printf("%-34s stale words %lld, iterations with stale %lld of %d\n",
             mode ? "noise: d2d reset hand-off" : "noise: xcd hand-off", bad_words, bad_iters, iters);
      fflush(stdout);
      CHECK(hipFree(buf));
    }
    return 0;
  }
  // cross-XCD hand-off between launches: mode 0 agent ld/st, 1 plain, 2 agent + consumer agent
  // acquire, 3 agent + consumer system acquire, 4 agent + producer release, 5 uncached memory
  const char* xname[] = {"xcd hand-off agent ld/st", "xcd hand-off plain ld/st", "xcd hand-off + agent acquire",
                         "xcd hand-off + system acquire", "xcd hand-off + producer release", "xcd hand-off uncached"};
  for (int mode = 0; mode < 6; mode++) {
    int* buf = nullptr;
    if (mode == 5) CHECK(hipExtMallocWithFlags((void**)&buf, bytes, hipDeviceMallocUncached));
    else CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMemset(buf, 0, bytes));
    CHECK(hipDeviceSynchronize());
    long long bad_words = 0, bad_iters = 0;
    const int xi = std::min(iters, 100);
    auto rd = [&](int tag) {
      if (mode == 1) hipLaunchKernelGGL((k_read_all<0, 0>), dim3(G), dim3(256), 0, st, buf, n, tag, stale_d);
      else if (mode == 2) hipLaunchKernelGGL((k_read_all<1, 1>), dim3(G), dim3(256), 0, st, buf, n, tag, stale_d);
      else if (mode == 3) hipLaunchKernelGGL((k_read_all<1, 2>), dim3(G), dim3(256), 0, st, buf, n, tag, stale_d);
      else hipLaunchKernelGGL((k_read_all<1, 0>), dim3(G), dim3(256), 0, st, buf, n, tag, stale_d);
    };
    for (int it = 0; it < xi; it++) {
      rd(it);  // lines into every XCD's L2
      if (mode == 1) hipLaunchKernelGGL((k_write<0, 0>), dim3(G), dim3(256), 0, st, buf, it + 1, xw_d);
      else if (mode == 4) hipLaunchKernelGGL(k_write_rel, dim3(G), dim3(256), 0, st, buf, it + 1);
      else hipLaunchKernelGGL((k_write<1, 1>), dim3(G), dim3(256), 0, st, buf, it + 1, xw_d);
      CHECK(hipMemsetAsync(stale_d, 0, 4 * G, st));
      rd(it + 1);
      CHECK(hipGetLastError());
      CHECK(hipMemcpyAsync(stale.data(), stale_d, 4 * G, hipMemcpyDeviceToHost, st));
      CHECK(hipStreamSynchronize(st));
      long long b = 0;
      for (int g = 0; g < G; g++) b += stale[g];
      bad_words += b;
      bad_iters += b != 0;
    }
    printf("%-34s stale words %lld of %lld, iterations with stale %lld of %d\n", xname[mode], bad_words,
           (long long)n * G * xi, bad_iters, xi);
    fflush(stdout);
    CHECK(hipFree(buf));
  }
  for (const Variant& v : vs) {
    int* buf = nullptr;
    if (v.alloc == A_UNCACHED) CHECK(hipExtMallocWithFlags((void**)&buf, bytes, hipDeviceMallocUncached));
    else if (v.alloc == A_FINE) CHECK(hipExtMallocWithFlags((void**)&buf, bytes, hipDeviceMallocFinegrained));
    else CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMemset(buf, 0, bytes));
    CHECK(hipDeviceSynchronize());
    long long bad_words = 0, bad_iters = 0, same_xcd = 0, bad_blocks = 0;
    for (int it = 0; it < iters; it++) {
      if (v.ld && v.st) hipLaunchKernelGGL((k_write<1, 1>), dim3(G), dim3(256), 0, st, buf, it + 1, xw_d);
      else hipLaunchKernelGGL((k_write<0, 0>), dim3(G), dim3(256), 0, st, buf, it + 1, xw_d);
      CHECK(hipGetLastError());
      CHECK(hipStreamSynchronize(st));  // as kss: the run is synchronised before the reset
      switch (v.reset) {
        case R_MEMCPY_D2D: CHECK(hipMemcpyAsync(buf, zero_d, bytes, hipMemcpyDeviceToDevice, st)); break;
        case R_MEMCPY_H2D: CHECK(hipMemcpyAsync(buf, zero_pinned, bytes, hipMemcpyHostToDevice, st)); break;
        case R_MEMSET: CHECK(hipMemsetAsync(buf, 0, bytes, st)); break;
        case R_KERNEL: hipLaunchKernelGGL(k_zero, dim3(G), dim3(256), 0, st, buf, n); break;
      }
      CHECK(hipStreamSynchronize(st));
      CHECK(hipMemsetAsync(stale_d, 0, 4 * G, st));
      if (v.acq) hipLaunchKernelGGL((k_check<1, 1>), dim3(G), dim3(256), 0, st, buf, stale_d, xr_d);
      else if (v.ld) hipLaunchKernelGGL((k_check<1, 0>), dim3(G), dim3(256), 0, st, buf, stale_d, xr_d);
      else hipLaunchKernelGGL((k_check<0, 0>), dim3(G), dim3(256), 0, st, buf, stale_d, xr_d);
      CHECK(hipGetLastError());
      CHECK(hipMemcpyAsync(stale.data(), stale_d, 4 * G, hipMemcpyDeviceToHost, st));
      CHECK(hipMemcpyAsync(xw.data(), xw_d, 4 * G, hipMemcpyDeviceToHost, st));
      CHECK(hipMemcpyAsync(xr.data(), xr_d, 4 * G, hipMemcpyDeviceToHost, st));
      CHECK(hipStreamSynchronize(st));
      long long b = 0;
      for (int g = 0; g < G; g++) {
        b += stale[g];
        if (stale[g]) {
          bad_blocks++;
          same_xcd += xw[g] == xr[g];
        }
      }
      bad_words += b;
      bad_iters += b != 0;
    }
    printf("%-34s stale words %lld of %lld, iterations with stale %lld of %d, stale blocks %lld (same XCD as writer %lld)\n",
           v.name, bad_words, (long long)n * iters, bad_iters, iters, bad_blocks, same_xcd);
    fflush(stdout);
    CHECK(hipFree(buf));
  }
  return 0;
}
