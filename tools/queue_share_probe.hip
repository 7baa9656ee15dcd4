// Queue-sharing probe: what happens to kernels of several streams of one process when the HIP
// runtime maps more streams than GPU_MAX_HW_QUEUES onto its hardware queues (the r5d split
// failure).
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/queue_share_probe tools/queue_share_probe.hip -lpthread
//   tools/queue_share_probe QUEUES STREAMS [MODE]   (sets GPU_MAX_HW_QUEUES before HIP starts)
//   MODE: plain (hipStreamCreateWithFlags), cumask (hipExtStreamCreateWithCUMask, every CU set),
//         prio (hipStreamCreateWithPriority, the highest priority)
//
// order:  on every stream, K_long (one workgroup: waits ~20 ms of wall time, then stores 1 into
//         the stream's done word) followed by K_check on the SAME stream (loads the done word).
//         In-order streams: every K_check must see 1.
// peers:  the split grid's shape: stream s's K_wait spins (bounded, 1 s) until every other
//         stream's K_wait has raised its arrival word, then stores its done word; K_check
//         follows on the same stream.  Launched from one host thread per stream, as
//         kss/split.py's InProcessSplit does.  Outcomes per stream: timed out (a peer never ran
//         beside it: serialised on a shared queue), check saw 0 (K_check ran before K_wait's
//         store), ok.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CHECK(x)                                                                              \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      exit(2);                                                                                \
    }                                                                                         \
  } while (0)

__device__ __forceinline__ long long now() { return (long long)__builtin_amdgcn_s_memrealtime(); }  // 100 MHz

__global__ void k_long(int* done, long long ticks) {
  if (threadIdx.x == 0) {
    const long long t0 = now();
    while (now() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
    __hip_atomic_store(done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void k_check(const int* done, int* seen) {
  if (threadIdx.x == 0) seen[0] = __hip_atomic_load(done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}

// arrive[s] = 1, then wait for every arrive[] (bounded), then done = 1 (or 2 on a timeout)
__global__ void k_wait(int* arrive, int n, int s, int* done, long long ticks) {
  if (threadIdx.x == 0) {
    __hip_atomic_store(&arrive[s], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    const long long t0 = now();
    int ok = 0;
    while (!ok) {
      ok = 1;
      for (int i = 0; i < n; i++) ok &= __hip_atomic_load(&arrive[i], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      if (!ok && now() - t0 > ticks) break;
      __builtin_amdgcn_s_sleep(4);
    }
    __hip_atomic_store(done, ok ? 1 : 2, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

int main(int argc, char** argv) {
  const int queues = argc > 1 ? atoi(argv[1]) : 4, n = argc > 2 ? atoi(argv[2]) : 5;
  const char* mode = argc > 3 ? argv[3] : "plain";
  char qs[16];
  snprintf(qs, sizeof qs, "%d", queues);
  setenv("GPU_MAX_HW_QUEUES", qs, 1);
  CHECK(hipSetDevice(0));
  std::vector<hipStream_t> st(n);
  int n_cu = 0;
  CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<uint32_t> mask((n_cu + 31) / 32, 0xffffffffu);
  if (n_cu % 32) mask.back() = (1u << (n_cu % 32)) - 1;
  int lo = 0, hi = 0;
  CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  for (auto& s : st) {
    if (!strcmp(mode, "cumask")) CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    else if (!strcmp(mode, "prio")) CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
    else CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  }
  printf("mode %s (%d CUs, priorities %d..%d)\n", mode, n_cu, lo, hi);
  int *done, *seen, *arrive;
  CHECK(hipMalloc(&done, 4 * n));
  CHECK(hipMalloc(&seen, 4 * n));
  CHECK(hipMalloc(&arrive, 4 * n));
  std::vector<int> hd(n), hs(n);

  for (int rep = 0; rep < 3; rep++) {  // order
    CHECK(hipMemset(done, 0, 4 * n));
    CHECK(hipMemset(seen, 0xff, 4 * n));
    CHECK(hipDeviceSynchronize());
    for (int s = 0; s < n; s++) {
      hipLaunchKernelGGL(k_long, dim3(1), dim3(64), 0, st[s], done + s, 2000000ll);
      hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, st[s], done + s, seen + s);
    }
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(hs.data(), seen, 4 * n, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int s = 0; s < n; s++) bad += hs[s] != 1;
    printf("queues %d streams %d order rep %d: K_check saw the same stream's K_long unfinished on %d of %d streams\n",
           queues, n, rep, bad, n);
  }

  for (int rep = 0; rep < 3; rep++) {  // peers
    CHECK(hipMemset(done, 0, 4 * n));
    CHECK(hipMemset(seen, 0xff, 4 * n));
    CHECK(hipMemset(arrive, 0, 4 * n));
    CHECK(hipDeviceSynchronize());
    std::vector<std::thread> th;
    for (int s = 0; s < n; s++)
      th.emplace_back([&, s] {
        hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, st[s], arrive, n, s, done + s, 100000000ll);
        hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, st[s], done + s, seen + s);
      });
    for (auto& t : th) t.join();
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(hs.data(), seen, 4 * n, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(hd.data(), done, 4 * n, hipMemcpyDeviceToHost));
    printf("queues %d streams %d peers rep %d: check/done per stream:", queues, n, rep);
    int tmo = 0, early = 0;
    for (int s = 0; s < n; s++) {
      printf(" %d/%d", hs[s], hd[s]);
      tmo += hd[s] == 2;
      early += hs[s] == 0;
    }
    printf("  -> %d timed out, %d checks before their stream's wait ended\n", tmo, early);
  }
  for (auto& s : st) CHECK(hipStreamDestroy(s));
  return 0;
}
