// kss_lib.hip — C ABI of libkss.so (include/kss.h): device context, snapshot upload,
// and the launches of the gfx950 scheduling kernels.
//
// Kernel map:
//   k_schedule   one workgroup per cluster; sequential pods; every phase of the
//                scheduling cycle in the workgroup (kss_sched.cuh).  Used for the
//                sequential batch (kss_schedule_batch), the drop-in per-pod call
//                (kss_eval_pod, no commit) and the what-if scenario sweep
//                (kss_schedule_scenarios, grid = #scenarios).
//   k_static     batches without PodTopologySpread / InterPodAffinity programs: the
//                commit-invariant part of every (pod, node) evaluation, one lane each,
//                packed into 32-bit static words in HBM (kss_simple.cuh).
//   k_simple     the sequential loop of those batches (no result record): node rows
//                in LDS, compact pod records and static words in LDS rings, only the
//                state-dependent filter / scores per pod, one exchange per pod.
//   k_spread     the sequential loop of batches WITH spread / inter-pod-affinity programs
//                (no result record): node rows, label ids, the pod's count rows and
//                the launch's commits in LDS, host-resolved pod programs (GPod),
//                32-bit exchanges (kss_spread.cuh).
//   k_commit     one lane: AssumePod / ForgetPod delta on one node row.
//   k_preempt    one workgroup: the DefaultPreemption PostFilter dry run of one pod
//                (kss_preempt.cuh).
#include <hip/hip_runtime.h>

#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <memory>
#include <thread>
#include <cstdio>
#include <cstring>
#include <unordered_map>
#include <mutex>
#include <atomic>
#include <string>
#include <vector>

#include "kss_host.h"
#include "kss_sched.cuh"
#include "kss_simple.cuh"
#include "kss_spread.cuh"
#include "kss_axis.cuh"
#include "kss_preempt.cuh"

using namespace kss;

namespace {

thread_local std::string g_err;
thread_local int g_rc = 0;  // code of the last failure (calls that return a handle report it this way)

int fail(int code, const std::string& msg) {
  g_err = msg;
  g_rc = code;
  return code;
}

// Tuning and diagnosis options (kss_set_option, include/kss.h): process-wide, changed only by an
// explicit call.  The product library reads no environment variable, so a plugin host's
// environment changes nothing; experiment builds (make exp, -DKSS_EXPERIMENTS) start each
// option from KSS_<ENV> for the A/B recipes in tools/.
enum KssOpt {
  O_SHARDS, O_XCD, O_XCD_SHARDS, O_NO_SIMPLE, O_NO_SPREAD, O_AXIS_BLOCKS, O_AXIS_NO_FOLD, O_NODES_PER_SHARD,
  O_THREADS, O_FORCE_THREADS, O_COOP_LAUNCH, O_NO_CACHE, O_STATIC_BYTES, O_STATIC_PPB, O_FOLD, O_TRACE_PATH,
  O_SVC_INLINE_SWEEP, O_SERVICE_STAMPS, O_SVC_FULL_FENCE, O_SERVICE_GENERAL, O_SVC_XCD, O_SVC_NO_STATIC,
  O_SWEEP_PIPE, O_SERVICE_NO_DIFF, O_SVC_HUGE, O_XCD_FORCE_FALLBACK, O_SPREAD_TWO_LEVEL, O_SPREAD_LB256, O_N
};
struct OptDef {
  const char* name;
  const char* env;
  long long dflt;
};
const OptDef kOptDefs[O_N] = {
    {"shards", "KSS_SHARDS", 0},                    // shards per cluster (0: automatic)
    {"xcd", "KSS_XCD", 1},                          // XCD-local grids where the shards fit one XCD
    {"xcd_shards", "KSS_XCD_SHARDS", 0},            // shards of an XCD-local grid (0: CUs per XCD)
    {"no_simple", "KSS_NO_SIMPLE", 0},              // never k_simple
    {"no_spread", "KSS_NO_SPREAD", 0},              // never k_spread
    {"axis_blocks", "KSS_AXIS_BLOCKS", 0},          // cap on the node-axis grid
    {"axis_no_fold", "KSS_AXIS_NO_FOLD", 0},        // timing experiment only (wrong results)
    {"nodes_per_shard", "KSS_NODES_PER_SHARD", 128},
    {"threads", "KSS_THREADS", 0},                  // preferred workgroup size (0: automatic)
    {"force_threads", "KSS_FORCE_THREADS", 0},      // exact workgroup size (0: automatic)
    {"coop_launch", "KSS_COOP_LAUNCH", 0},          // hipLaunchCooperativeKernel for sharded grids
    {"no_cache", "KSS_NO_CACHE", 0},                // k_schedule without its LDS node cache
    {"static_bytes", "KSS_STATIC_BYTES", 0},        // k_static budget (0: an eighth of free memory)
    {"static_ppb", "KSS_STATIC_PPB", 0},            // k_static pods per block (0: automatic)
    {"fold", "KSS_FOLD", 0},                        // k_spread statistics fold
    {"trace_path", "KSS_TRACE_PATH", 0},            // print the batch routing decision
    {"svc_inline_sweep", "KSS_SVC_INLINE_SWEEP", 0},
    {"service_stamps", "KSS_SERVICE_STAMPS", 0},
    {"svc_full_fence", "KSS_SVC_FULL_FENCE", 0},
    {"service_general", "KSS_SERVICE_GENERAL", 0},  // the service's general chain for every pod
    {"svc_xcd", "KSS_SVC_XCD", 0},
    {"svc_no_static", "KSS_SVC_NO_STATIC", 0},
    {"sweep_pipe", "KSS_SWEEP_PIPE", 0},
    {"service_no_diff", "KSS_SERVICE_NO_DIFF", 0},
    {"svc_huge", "KSS_SVC_HUGE", 0},
    {"xcd_force_fallback", "KSS_XCD_FORCE_FALLBACK", 0},  // XCD-local launches report failed placement
    {"spread_two_level", "KSS_SPREAD_TWO_LEVEL", 1},      // k_spread at W > 64: 1 two-level selectHost exchange, 2 + reductions
    {"spread_lb256", "KSS_SPREAD_LB256", 1},              // k_spread compiled for <= 256 lanes when the shard fits
};
std::atomic<long long> g_opt[O_N];
std::once_flag g_opt_once;
std::mutex g_stamps_mu;
std::string g_stamps_path;  // kss_set_stamps_file

void opt_defaults() {
  for (int i = 0; i < O_N; i++) {
    long long v = kOptDefs[i].dflt;
#ifdef KSS_EXPERIMENTS
    if (const char* e = getenv(kOptDefs[i].env)) v = (*e >= '0' && *e <= '9') || *e == '-' ? atoll(e) : 1;
#endif
    g_opt[i].store(v, std::memory_order_relaxed);
  }
#ifdef KSS_EXPERIMENTS
  if (const char* e = getenv("KSS_STAMPS_FILE")) g_stamps_path = e;
#endif
}
long long opt(KssOpt o) {
  std::call_once(g_opt_once, opt_defaults);
  return g_opt[o].load(std::memory_order_relaxed);
}

// A stream on a hardware queue of its own.  The HIP runtime maps a process's plain streams onto
// at most GPU_MAX_HW_QUEUES queues (4 on the box), and a kernel queued behind another stream's
// kernel on a shared queue does not start before that one ends: the parts of a split grid, which
// poll each other's granules, then wait out the exchange bound (tools/queue_share_probe.hip,
// profiles/r8a_queue_share_probe.txt: 4 queues, 6 streams -> 4 of 6 waits timed out; the r5d
// split failure).  A CU-masked stream gets a queue of its own whatever the queue
// count: every CU in the mask, 0 of 6 waits timed out at 4 queues and 0 of 4 at 1 queue.
hipError_t dedicated_stream(int n_cu, hipStream_t* st) {
  std::vector<uint32_t> mask((size_t)(std::max(n_cu, 1) + 31) / 32, 0xffffffffu);
  if (n_cu % 32) mask.back() = (1u << (n_cu % 32)) - 1u;
  return hipExtStreamCreateWithCUMask(st, (uint32_t)mask.size(), mask.data());
}


#define HIP_TRY(expr)                                                                        \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) return fail(KSS_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// per-pod output slot layout (record format), N nodes
struct SlotLayout {
  size_t fail, detail, raw, norm, total, bytes;
  __host__ __device__ explicit SlotLayout(size_t N) {
    // verdicts and totals first: a caller that wants only those (one plugin answering Filter
    // and Score) copies back the first ~11 B per node, not the ~140 B of per-plugin scores
    fail = 0;
    detail = align_up(N, 256);
    total = align_up(detail + 2 * N, 256);
    raw = align_up(total + 8 * N, 256);
    norm = raw + 8 * KSS_NSCORE * N;
    bytes = align_up(norm + 8 * KSS_NSCORE * N, 256);
  }
};

// The service grid's compact host record (kss_service_eval_compact): a slot's rows with the
// scores narrowed, raw and total to int32 and normalised scores (0..MaxNodeScore) to uint8:
// 47 instead of 139 bytes per node over the host link.  Fields start 256-byte aligned.
struct CompactLayout {
  size_t fail, detail, total, raw, norm, bytes;
  __host__ __device__ explicit CompactLayout(size_t N) {
    fail = 0;
    detail = align_up(N, 256);
    total = align_up(detail + 2 * N, 256);
    raw = align_up(total + 4 * N, 256);
    norm = align_up(raw + 4 * KSS_NSCORE * N, 256);
    bytes = align_up(norm + KSS_NSCORE * N, 256);
  }
};

// one workgroup's job
struct DevJob {
  DevCluster c;
  DevPods P;
  int32_t n_pods;
  int32_t commit;     // apply AssumePod after each pod
  int32_t keep_norm;  // write norm/total into the slot(s)
  int32_t record;     // one slot per pod (else slot 0 reused)
  uint8_t* slots;
  size_t slot_bytes;
  int32_t* chosen;
  PodMeta* meta;
  const SPod* spods;  // k_simple: compact pod records [n_pods]
  uint32_t* stat;     // k_static -> k_simple / k_spread: static words of the current pod chunk [chunk][N]
  const GPod* gpods;  // k_spread: host-resolved pod programs [n_pods]
  const int32_t* res_rows;  // k_spread: the count rows resident in LDS (GpodNeeds::res_rows)
  kss_profile prof;   // k_simple<false>: staged word by word into LDS (a by-value kernel argument would land in scratch)
  GTrace trace;       // k_spread diagnostic trace (KSS_SPREAD_TRACE builds only; null otherwise)
  int32_t* cursor;    // k_schedule / the service: the cluster's nextStartNodeIndex word (null: 0, not kept)
  const DevNom* nom;  // k_schedule: the nominator's entries (kss_nominate), all nominated at launch
  int32_t n_nom;      // entries (<= KSS_NOM_MAX; 0: none)
  int32_t pod_base;   // pod pi is pod pod_base + pi of the caller's podset (its identity when its uid is 0)
};

// The nominator's pod identity: the caller's uid, else -1 - the pod's podset index
__host__ __device__ inline int32_t pod_identity(const kss_pod& p, int index) { return p.uid > 0 ? p.uid : -1 - index; }

}  // namespace

#include "kss_service.cuh"

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
// grid = n_jobs * W; workgroup b serves shard (b % W) of cluster (b / W); each lane
// owns npt node slots.
template <bool GEN>
__global__ __launch_bounds__(KSS_MAX_THREADS) void k_schedule(const DevJob* __restrict__ jobs, kss_profile prof,
                                                              int W, int npt, int bins_cap, int cache_keys,
                                                              unsigned long long* gran, int* err,
                                                              unsigned long long* stamps, unsigned epoch0) {
  extern __shared__ __attribute__((aligned(16))) long long smem[];
  const int ji = blockIdx.x / W, w = blockIdx.x % W;
  const DevJob job = jobs[ji];  // by value: the descriptors stay in registers for the whole launch
  DevCluster c = job.c;
  const size_t N = (size_t)c.N;
  const SlotLayout L(N);
  if (threadIdx.x == 0) shdr(smem).abort = 0;
  __syncthreads();
  Shard S;
  const int per = (c.N + W - 1) / W;
  S.lo = min(c.N, w * per);
  S.hi = min(c.N, S.lo + per);
  S.W = W;
  S.w = w;
  S.epoch = epoch0;  // granule tags of earlier launches are all below epoch0 (host-tracked)
  S.gran = gran ? gran + (size_t)ji * 2 * W * 2 * XW_MAX : nullptr;
  S.err = err;
  S.stamps = nullptr;
  S.cursor = job.cursor ? *job.cursor : 0;  // written by the previous launch / the host (stream order)
  const bool want_out = job.record || job.keep_norm;
  // shard node cache: the hot node columns stay in LDS for the whole launch
  const int cap = npt * (int)blockDim.x;
  if (cache_keys >= 0) {
    long long* b = xvec(smem) + NSCAL + bins_cap + slot_arrays_bytes(cap) / 8;
    c.nc64 = reinterpret_cast<int64_t*>(b);
    c.nct = reinterpret_cast<uint64_t*>(b + 8 * (size_t)cap);
    c.nc32 = reinterpret_cast<int32_t*>(b + 10 * (size_t)cap);
    c.ncl = cache_keys > 0 && cache_keys >= c.n_keys ? c.nc32 + 3 * (size_t)cap : nullptr;
    c.nc_lo = S.lo;
    c.nc_cap = cap;
    cache_fill(c, S.hi, c.ncl ? c.n_keys : 0);
    __syncthreads();
  }
  NomView nv{job.nom, job.n_nom, -1, job.n_nom >= 64 ? ~0ull : ((1ull << job.n_nom) - 1ull)};
  for (int pi = 0; pi < job.n_pods; pi++) {
    uint8_t* base = job.slots + (job.record ? (size_t)pi * job.slot_bytes : 0);
    Slot s;
    nv.pod = pod_identity(job.P.pods[pi], job.pod_base + pi);
    s.fail = base + L.fail;
    s.detail = (uint16_t*)(base + L.detail);
    s.raw = (int64_t*)(base + L.raw);
    s.norm = (int64_t*)(base + L.norm);
    s.total = (int64_t*)(base + L.total);
    PodMeta m;
    S.stamps = (stamps && ji == 0 && w == 0 && pi < KSS_NSTAMP_PODS) ? stamps + (size_t)pi * 8 : nullptr;
    KSS_STAMP(S, 0);
    if (!schedule_pod<GEN>(c, job.P, prof, pi, smem, S, bins_cap, npt, want_out ? &s : nullptr, job.keep_norm != 0, m,
                           nv))
      return;  // exchange timeout: the error word is set, leave the launch
    if (job.commit && m.chosen >= 0)  // assume -> DeleteNominatedPodIfExists (every shard knows the choice)
      for (int j = 0; j < nv.n; j++)
        if (job.nom[j].pod == nv.pod) nv.active &= ~(1ull << j);
    if (threadIdx.x == 0) {
      if (w == 0) {
        if (job.chosen) job.chosen[pi] = m.chosen;
        if (job.meta) job.meta[pi] = m;
      }
      const int local = m.chosen - c.node_base;
      if (job.commit && m.chosen >= 0 && local >= S.lo && local < S.hi) commit_pod(c, job.P, job.P.pods[pi], local, 1);
      // the binder's assume cache is global: every shard applies AssumePodVolumes (identical
      // values; every shard finished this pod's filters before the argmax exchange ended)
      if (job.commit && m.chosen >= 0 && job.P.pods[pi].vol_len > 0)
        wffc_commit(c, job.P.reqs, job.P.terms, job.P.ints, job.P.vols, job.P.pods[pi], local, 1,
                    [&](int key) { return c.label_value[(size_t)key * N + local]; });
    }
    __syncthreads();
    KSS_STAMP(S, 6);
  }
  if (job.cursor && w == 0 && threadIdx.x == 0) *job.cursor = S.cursor;  // every shard holds the same value
  if (c.nc64 && job.commit) cache_writeback(c, S.hi);
}

// The per-pod service grid (kss_service.cuh): W shards of one cluster, commands from the
// pinned ring starting at command `seq`.
template <bool GEN, bool SIMPLE, bool INL = false>
__global__ __launch_bounds__(KSS_MAX_THREADS) void k_service(const DevJob* __restrict__ jobs, kss_profile prof, int W,
                                                             int npt, int bins_cap, int cache_keys,
                                                             unsigned long long* gran, int* err, SvcBox* box,
                                                             unsigned long long* relay, unsigned long long* seen,
                                                             uint8_t* rec_host, unsigned long long seq, int stamps,
                                                             int xcd) {
  extern __shared__ __attribute__((aligned(16))) long long smem[];
  const DevJob job = jobs[0];
  service_loop<GEN, SIMPLE, INL>(job.c, job, prof, W, npt, bins_cap, cache_keys, gran, err, box, relay, seen, rec_host,
                                 seq, 0u, stamps, smem, xcd);
}

#ifndef KSS_SIMPLE_PW
#define KSS_SIMPLE_PW 1  // experiment builds: -DKSS_SIMPLE_PW=0 keeps the two-reduction loop everywhere
#endif
// grid = n_jobs * W, as k_schedule; each shard's nodes live in LDS (cap slots).
// DEF: the profile is the v1.26 default, folded into the code.
// Pods [k0, min(k1, n_pods)) of every job; the job's stat buffer holds their static words.
// WIN: percentageOfNodesToScore < 100 (one job): k_find = numFeasibleNodesToFind, the window of
// simple_sync_win, nextStartNodeIndex in job.cursor.
template <bool DEF, bool WIN>
__global__ __launch_bounds__(KSS_MAX_THREADS) void k_simple(const DevJob* __restrict__ jobs, kss_profile prof, int W,
                                                            int cap, int k0, int k1, unsigned long long* gran, int* err,
                                                            unsigned long long* stamps, XPeers X, unsigned epoch0,
                                                            int stat_row0, int k_find) {
  extern __shared__ __attribute__((aligned(16))) long long smem[];
  const int Wl = X.n > 1 ? X.wl : W;  // shards of this launch (a split grid runs [w_off, w_off + wl))
  SimpleHdr& H = *reinterpret_cast<SimpleHdr*>(smem);
  int xs = 0;
  if (X.xcd_local) {  // one cluster, every shard on XCD 0 (xcd_slot); the other workgroups leave
    if (threadIdx.x == 0)  // the counters behind the granules (and the window's cut granules)
      H.pad[0] = xcd_slot(reinterpret_cast<int*>(gran + (WIN ? 2 * (size_t)W * SXW_VALS + 2 * SXW_E2 : 2 * (size_t)W * SX_VALS)),
                          W, (int)gridDim.x, err, X.xcd_local == 2);
    __syncthreads();
    xs = H.pad[0];
    if (xs < 0) return;
  }
  const int ji = X.xcd_local ? 0 : blockIdx.x / Wl, w = X.xcd_local ? xs : X.w_off + (int)(blockIdx.x % Wl);
  const DevJob job = jobs[ji];
  constexpr kss_profile def_prof = default_profile_c();
  if (!DEF) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&jobs[ji].prof);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&H.prof);
    for (int i = threadIdx.x; i < (int)(sizeof(kss_profile) / 4); i += blockDim.x) dst[i] = src[i];
    __syncthreads();
  }
  const kss_profile& P = DEF ? def_prof : H.prof;
  // per-wave mode when every shard's nodes fit PW_LANES slots per wave (one node per lane)
  const int per = (job.c.N + W - 1) / W, nwave = (int)(blockDim.x >> 6);
  unsigned long long* g = gran ? gran + (size_t)ji * 2 * W * SX_VALS : nullptr;  // (WIN: one job)
  unsigned long long* sp = ji == 0 ? stamps : nullptr;
  const uint32_t* stat = job.stat + (size_t)stat_row0 * (size_t)job.c.N;  // the chunk's half of a double-buffered table
  if (per <= PW_LANES * nwave && KSS_SIMPLE_PW)
    simple_schedule<DEF, true, WIN>(job.c, job.spods, stat, job.P.ints, k0, min(k1, job.n_pods), job.chosen, job.meta, P,
                                    W, w, cap, g, X, epoch0, err, sp, smem, k_find, job.cursor);
  else
    simple_schedule<DEF, false, WIN>(job.c, job.spods, stat, job.P.ints, k0, min(k1, job.n_pods), job.chosen, job.meta,
                                     P, W, w, cap, g, X, epoch0, err, sp, smem, k_find, job.cursor);
}

// grid = W (one cluster); each shard's nodes live in LDS (cap slots); bins_cap: histogram +
// presence values of the exchange vector.  DEF: the v1.26 default profile, folded.  FOLD: the
// statistics fold compiled in (KSS_FOLD=1; a separate kernel, so the default one keeps the
// register allocation the fold's code would spill: 36 against 164 B of scratch per lane).
// LB: the workgroup-size bound the register allocation is made for.  At <= 256 lanes (C3's
// 192-lane shards) one wave per SIMD: 512 registers per lane (256 VGPRs + 256 AGPRs), so the
// allocator keeps in registers what the 512-lane bound spills to scratch.
// WIN: percentageOfNodesToScore < 100 (one job): k_find = numFeasibleNodesToFind, the window's
// nextStartNodeIndex in job.cursor (kss_spread.cuh spread_schedule)
template <bool DEF, bool FOLD, int LB, bool WIN>
__global__ __launch_bounds__(LB) void k_spread(const DevJob* __restrict__ jobs, int W, int cap, int bins_cap,
                                                            int n_res, int gq, int gs, int k0, int k1, unsigned long long* gran,
                                                            int* err, unsigned long long* stamps, int nst, XPeers X,
                                                            unsigned epoch0, HandoffCheck hc, int k_find) {
  extern __shared__ __attribute__((aligned(16))) long long smem[];
  const int Wl = X.n > 1 ? X.wl : W;
  SpreadHdr& H = *reinterpret_cast<SpreadHdr*>(smem);
  int xs = 0;
  if (X.xcd_local) {  // one cluster, every shard on XCD 0 (xcd_slot); the other workgroups leave
    if (threadIdx.x == 0)
      H.pad[0] = xcd_slot(reinterpret_cast<int*>(gran + 2 * (size_t)W * gs), W, (int)gridDim.x, err, X.xcd_local == 2);
    __syncthreads();
    xs = H.pad[0];
    if (xs < 0) return;
  }
  const int ji = X.xcd_local ? 0 : blockIdx.x / Wl, w = X.xcd_local ? xs : X.w_off + (int)(blockIdx.x % Wl);
  if (X.tl) {  // the two-level selectHost exchange: the shard's XCD and rank there (tl_register)
    if (threadIdx.x == 0) tl_register(H, X.tl, W, err);
    __syncthreads();
  }
  const DevJob job = jobs[ji];
  constexpr kss_profile def_prof = default_profile_c();
#ifdef KSS_LDS_POISON  // experiment builds: the shard's LDS image filled with a pattern first
  {
    const size_t words = spread_lds_bytes(cap, bins_cap, job.c.n_keys, n_res, gq, job.c.n_scalar, FOLD) / 4;
    uint32_t* p = reinterpret_cast<uint32_t*>(smem);
    for (size_t i = threadIdx.x; i < words; i += blockDim.x) p[i] = 0x5A5A5A5Au;
    __syncthreads();
  }
#endif
  if (!DEF) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&jobs[ji].prof);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&H.prof);
    for (int i = threadIdx.x; i < (int)(sizeof(kss_profile) / 4); i += blockDim.x) dst[i] = src[i];
    __syncthreads();
  }
  const kss_profile& P = DEF ? def_prof : H.prof;
  spread_schedule<DEF, FOLD, WIN>(job.trace, job.c, job.gpods, job.stat, job.res_rows, n_res, k0, min(k1, job.n_pods), job.chosen, job.meta, P, W, w,
                  cap, bins_cap, gq, gs, gran ? gran + (size_t)ji * 2 * W * gs : nullptr, X, epoch0, err, stamps, nst, hc,
                  smem, k_find, job.cursor);
}

// Class / term counts of the chosen nodes of pods [k0, min(k1, n_pods)) of every job
// (grid: x = 256-pod tiles, y = job).
__global__ __launch_bounds__(256) void k_counts(const DevJob* __restrict__ jobs, int k0, int k1) {
  const DevJob& job = jobs[blockIdx.y];
  const int k = k0 + (int)(blockIdx.x * 256 + threadIdx.x);
  if (k >= min(k1, job.n_pods) || !job.chosen) return;
  simple_counts(job.c, job.spods, job.P.ints, job.chosen, k);
  handoff_drain();
}

// The final check of a k_spread run's last write-back (handoff_final_check): grid = the
// part's shards, w_off the first of them.
__global__ __launch_bounds__(256) void k_handoff_final(const DevJob* __restrict__ jobs, int W, int w_off, int n_res,
                                                       HandoffCheck hc, int* err) {
  __shared__ long long scratch[4];
  const DevJob& job = jobs[0];
  handoff_final_check(job.c, job.res_rows, n_res, W, w_off + (int)blockIdx.x, hc, err, scratch);
}

// Static words of pods [k0, min(k1, n_pods)) x every node of every job.  grid: x = 1024-node
// tiles, y = groups of STATIC_PODS pods, z = job.  One lane per QUAD of adjacent nodes walks its
// group: the quad's four words leave as one 16-byte agent-scope (sc1, write-through) store where
// the row layout keeps it aligned (N and n_lo multiples of 4, the job's stat buffer 16-byte
// aligned), as 8- or 4-byte agent-scope stores otherwise.  Per byte a 16-byte sc1 store costs
// about a third of an 8-byte one (MI355X_MICROARCH.md: dwordx2 2.7x, dword ~6x the dwordx4 time).
typedef unsigned int kss_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_ag16(uint32_t* p, kss_u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
// lkeys > 0: the block's 1024 nodes' label values of the first lkeys keys are copied into LDS
// once ([key][node], 4 bytes each) and every requirement reads them there: the label columns were
// read from L2 / HBM once per (pod, node, requirement) -- ~14 vector loads per static word, the
// wait that dominated k_static (profiles/r5v: SQ_WAIT_ANY 70% of wave cycles).
constexpr int STATIC_LKEYS = 16;  // label keys cached (more: the loads stay global)
template <bool DEF>
__global__ __launch_bounds__(256) void k_static(const DevJob* __restrict__ jobs, kss_profile prof_arg, int k0, int k1,
                                                int n_lo, int n_hi, int lkeys, int row0, int ppb) {
  extern __shared__ int32_t slab[];  // [lkeys][1024]
  const DevJob& job = jobs[blockIdx.z];
  const int N = job.c.N;
  const int nb = n_lo + 4 * (int)(blockIdx.x * 256);  // the block's first node
  const int n = nb + 4 * (int)threadIdx.x;  // rows [n_lo, min(n_hi, N)): a split grid's own rows
  const int kend = min(k1, job.n_pods);
  const int kb = k0 + (int)blockIdx.y * ppb;  // the block's pods: [kb, kb + ppb)
  const int lim = min(N, n_hi);
  const bool lds = lkeys > 0 && job.c.n_keys <= lkeys;
  if (lds) {  // every lane reaches the barrier (no early exit above it)
    const int nk = job.c.n_keys;
    for (int i = (int)threadIdx.x; i < nk * 1024; i += 256) {
      const int key = i >> 10, j = i & 1023;
      slab[i] = nb + j < lim ? gp(job.c.label_value)[(size_t)key * N + nb + j] : -1;
    }
    __syncthreads();
  }
  if (kb >= kend || n >= lim) return;
  const int cnt = min(4, lim - n);
  uint32_t* stat = job.stat;
  const uintptr_t sa = reinterpret_cast<uintptr_t>(stat);
  const bool quad = cnt == 4 && ((N | n_lo) & 3) == 0 && (sa & 15) == 0;
  const bool pair = ((N | n_lo) & 1) == 0 && (sa & 7) == 0;  // 8-byte pairs at even offsets
  const DevCluster c = job.c;
  const DevPodsK P = pods_k(job.P);
  const kss_profile prof = DEF ? default_profile_c() : prof_arg;
  uint32_t f[4];
  uint64_t th[4], ts[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int ni = n + min(i, cnt - 1);
    f[i] = gp(c.node_flags)[ni];
    th[i] = gp(c.taint_hard)[ni];
    ts[i] = gp(c.taint_soft)[ni];
  }
  for (int t = 0; t < ppb; t++) {
    const int k = kb + t;
    if (k >= kend) break;
    const auto& pod = P.pods[k];
    uint32_t w[4];
    if (lds)
      static_words4(c, P, pod, prof, n, cnt, f, th, ts,
                    [&](int key, int i) { return slab[(key << 10) + (n + min(i, cnt - 1) - nb)]; }, w);
    else
      static_words4(c, P, pod, prof, n, cnt, f, th, ts,
                    [&](int key, int i) {
                      const int ni = n + min(i, cnt - 1);
                      return c.ncl ? label_of(c, key, ni) : gp(c.label_value)[(size_t)key * N + ni];
                    }, w);
    uint32_t* dst = &stat[(size_t)(row0 + k - k0) * N + n];  // row0: the half of a double-buffered table
    if (quad) {
      st_ag16(dst, kss_u32x4{w[0], w[1], w[2], w[3]});
    } else if (pair) {
      if (cnt >= 2) st_ag(reinterpret_cast<unsigned long long*>(dst), (unsigned long long)w[0] | ((unsigned long long)w[1] << 32));
      else st_ag(dst, w[0]);
      if (cnt == 4) st_ag(reinterpret_cast<unsigned long long*>(dst + 2), (unsigned long long)w[2] | ((unsigned long long)w[3] << 32));
      else if (cnt == 3) st_ag(dst + 2, w[2]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; i++)
        if (i < cnt) st_ag(dst + i, w[i]);
    }
  }
  // every store above is agent-scope (sc1, written through): the kernel boundary orders them
  // for the loop kernel's agent-scope loads, no L2 write-back per wave (C5: 256k workgroups,
  // an agent release in each cost 9 ms per sweep step)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__global__ void k_go_log(const double* x, double* y, int n) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i < n) y[i] = go_log_dev(x[i]);
}

// AssumePod / ForgetPod deltas of one pod, carried in the kernel arguments (no upload).
struct CommitArgs {
  int64_t req[KSS_NRES];
  int64_t nz[2];
  uint64_t port_add;
  int32_t cls, n_own, local, sign;
  int32_t own[8];
  int32_t n_vrow, n_vpriv;   // the pod's KSS_VOL_OWN / KSS_VOL_OWN_PRIVATE entries
  int32_t vrow[8];
  int32_t vpriv_key[4], vpriv_cnt[4];
};

__global__ void k_commit(DevCluster c, CommitArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const size_t N = (size_t)c.N;
  for (int r = 0; r < KSS_NRES; r++) c.requested[(size_t)r * N + a.local] += a.sign * a.req[r];
  c.nonzero[a.local] += a.sign * a.nz[0];
  c.nonzero[N + a.local] += a.sign * a.nz[1];
  c.pod_count[a.local] += a.sign;
  if (a.cls >= 0) c.class_count[(size_t)a.cls * N + a.local] += a.sign;
  for (int i = 0; i < a.n_own; i++) c.term_count[(size_t)a.own[i] * N + a.local] += a.sign;
  if (a.port_add) c.port_used[a.local] = a.sign > 0 ? (c.port_used[a.local] | a.port_add) : (c.port_used[a.local] & ~a.port_add);
  for (int i = 0; i < a.n_vrow; i++) vol_commit_row(c, a.vrow[i], a.local, a.sign);
  for (int i = 0; i < a.n_vpriv; i++) c.vol_attached[(size_t)a.vpriv_key[i] * N + a.local] += a.sign * a.vpriv_cnt[i];
  handoff_drain();
}

// The binder's AssumePodVolumes / RevertAssumedPodVolumes of pod 0 of P on node `local`
// (kss_commit / kss_rollback of a pod with WaitForFirstConsumer claims; wffc_commit).
__global__ void k_wffc_commit(DevCluster c, DevPods P, int local, int sign) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const size_t N = (size_t)c.N;
  wffc_commit(c, P.reqs, P.terms, P.ints, P.vols, P.pods[0], local, sign,
              [&](int key) { return c.label_value[(size_t)key * N + local]; });
  handoff_drain();
}

// DefaultPreemption PostFilter dry run of one pod (kss_postfilter_pod): three launches.
__global__ __launch_bounds__(PRE_THREADS) void k_preempt_stats(const PreemptJob* __restrict__ job) {
  extern __shared__ __attribute__((aligned(16))) long long smem[];
  preempt_stats(*job, smem);  // descriptors read through the scalar cache
}
__global__ __launch_bounds__(PRE_NODE_THREADS) void k_preempt_nodes(const PreemptJob* __restrict__ job) {
  extern __shared__ __attribute__((aligned(16))) long long smem[];
  preempt_nodes(*job, smem);
}

// Volume state sync (kss_apply_volume_delta): rows < n_vol_rows are vol_count, the rest
// vol_attached keys.  Entries are applied in order by one lane (repeated cells accumulate).
__global__ void k_volume_delta(DevCluster c, const int32_t* node, const int32_t* row, const int32_t* val, int n, int mode) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  const size_t N = (size_t)c.N;
  for (int i = 0; i < n; i++) {
    int32_t* cell = row[i] < c.n_vol_rows ? c.vol_count + (size_t)row[i] * N + node[i]
                                         : c.vol_attached + (size_t)(row[i] - c.n_vol_rows) * N + node[i];
    *cell = mode ? val[i] : *cell + val[i];
  }
  handoff_drain();
}

// Delta sync of node rows (kss_apply_node_delta): one packed upload, one scatter.
__global__ void k_node_delta(DevCluster c, const int32_t* idx, const int64_t* req, const int64_t* nz, const int32_t* pc,
                             int n) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  const size_t N = (size_t)c.N;
  const int r0 = idx[i];
  for (int r = 0; r < KSS_NRES; r++) c.requested[(size_t)r * N + r0] = req[(size_t)i * KSS_NRES + r];
  c.nonzero[r0] = nz[2 * (size_t)i];
  c.nonzero[N + r0] = nz[2 * (size_t)i + 1];
  c.pod_count[r0] = pc[i];
  handoff_drain();
}

// Class / term count sync (kss_apply_count_delta): add (mode 0) or overwrite (mode 1).
__global__ void k_count_delta(DevCluster c, const int32_t* node, const int32_t* row, const int32_t* val, int n, int mode) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  const size_t N = (size_t)c.N;
  int32_t* cell = row[i] < c.n_classes ? c.class_count + (size_t)row[i] * N + node[i]
                                       : c.term_count + (size_t)(row[i] - c.n_classes) * N + node[i];
  if (mode) *cell = val[i];
  else atomicAdd(cell, val[i]);
  handoff_drain();
}

// kss_reset_node_state: the mutable columns back to their load-time copy, as a kernel (the
// same hand-off path as every other writer of node state, not a copy engine): up to 8
// (destination, source, 32-bit words) ranges, grid-stride, agent-scope stores.
constexpr int KSS_NMUT = 10;  // mutable cluster columns (reset / pristine copies)
struct ResetArgs {
  uint32_t* dst[KSS_NMUT];
  const uint32_t* src[KSS_NMUT];
  size_t n4[KSS_NMUT];
};
__global__ __launch_bounds__(256) void k_reset_state(ResetArgs a) {
  for (int r = 0; r < KSS_NMUT; r++)
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < a.n4[r]; i += (size_t)gridDim.x * blockDim.x)
      st_ag(a.dst[r] + i, ld_ag(a.src[r] + i));
  handoff_release();
}

// Zero fill of device memory with agent-scope (sc1) stores, in place of the runtime's fill
// kernel (hipMemsetAsync).  The many-chunk split-grid corruption was a class
// count word of node state reading 0 after a chunk had stored 1 into it, in the first run
// after the cluster upload, whose count rows a hipMemsetAsync zeroed before the host rows
// were copied over them; no library buffer is zeroed by the runtime's fill kernel any more.
__global__ __launch_bounds__(256) void k_zero(uint32_t* p, size_t n4) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
  const size_t n8 = ((uintptr_t)p & 7) ? 0 : n4 / 2, stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n8; i += stride) st_ag(q + i, 0ull);
  for (size_t i = 2 * n8 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += stride) st_ag(p + i, 0u);
  handoff_release();
}
// bytes: a multiple of 4 (every library buffer's element size is)
static hipError_t dev_zero(void* p, size_t bytes, hipStream_t st) {
  if (bytes & 3) return hipErrorInvalidValue;  // every library buffer is a whole number of 32-bit words
  const size_t n4 = bytes / 4;
  if (!p || n4 == 0) return hipSuccess;
  const unsigned grid = (unsigned)std::min<size_t>(1024, (n4 / 2 + 255) / 256 + 1);
  hipLaunchKernelGGL(k_zero, dim3(grid), dim3(256), 0, st, (uint32_t*)p, n4);
  return hipGetLastError();
}

// Sets *flag when any of n outcomes has status 4 (a pod program past the device limits): the
// sweep reads one word back instead of every scenario's outcome table (24 B per pod; 98 MB at
// C5's 4,096 x 1,000 pods, a 6-7 ms pageable copy per run).  Lanes store the same value.
__global__ __launch_bounds__(256) void k_status4(const PodMeta* __restrict__ m, int n, int* flag) {
  bool any = false;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) any |= m[i].status == 4;
  if (any) st_ag(flag, 1);
}

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    size_t nb = std::max(bytes, (size_t)4096);
    if (hipMalloc(&p, nb) != hipSuccess) return fail(KSS_E_NOMEM, "hipMalloc failed");
    cap = nb;
    return 0;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// k_simple exactness bounds (f64_bounds_cluster / f64_bounds_pods / f64_exact below).
struct F64Bounds {
  double max_req0 = 0, max_nz0 = 0, max_creq = 0, max_cnz = 0, max_pod = 0;
  bool neg = false;
};

// What the staged batch asks of k_spread (the host side of the GPod plans).
struct GpodNeeds {
  int bins_cap = 0;       // max histogram + presence bins of a pod
  int max_mult = 1;       // max commits one pod adds to one count row
  int64_t ref_weight = 1; // max Σ|coefficient| over the references of one constraint / entry
  int max_soft = 0;       // max ScheduleAnyway constraints of a pod with more than one
  int64_t max_skew = 0;   // their largest maxSkew
  std::vector<int32_t> res_rows;  // the resident count rows: class r as r, term r as n_classes + r
  int gq = 0;             // record stride (uint4) of the batch
  int xw = 2;             // longest exchange of the batch (values per shard; the argmax's 2 at least)
  int fold_xw = 0;        // fold: max bins + hard presence of a folding pod (carried by the previous pod's E2)
  int soft_xw = 0;        // max soft presence bins of a pod (its own E2)
  int gs() const { return (xw + 15) / 16 * 16; }  // granule stride per shard: whole 128-byte lines
  int fail_code = 0, fail_pod = -1;  // why / where build_gpods refused (GP_*)
};

// Per-batch LDS / exchange sizing: the host restatement of make_plan's bin counts.
struct PlanNeeds {
  bool ports_images = false;  // some pod has host ports, ImageLocality rows or a volume program
  int bins_cap = 0;  // max over pods of histogram + presence bins
  int xw = 0;        // max exchange payload length (values) over pods and exchanges
  bool general = false;  // some pod carries spread / inter-pod-affinity programs
};

// One pod of the PostFilter bound table (kss_boundset row, or a pod committed since).
struct BoundPod {
  int64_t id;
  int64_t start;
  int64_t req[KSS_NRES];
  int64_t nz[2];     // NonZeroRequested cpu / memory (valid when has_nz)
  uint64_t ports;    // UsedPorts bits it holds
  int32_t prio, cls, tlen;
  int32_t terms[8];
  int32_t has_nz;    // the loaded boundset carried nonzero (kss_remove_bound needs it)
  int32_t has_vols;  // a committed pod with volumes (kss_remove_bound refuses it)
};
// A commit (add) or rollback (remove) applied to the loaded table, in call order.
struct BoundOp {
  int32_t node;  // local row
  int32_t add;
  BoundPod b;
};

struct kss_ctx {
  kss_config cfg{};
  kss_profile prof{};
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::mutex mu;  // rollback may arrive from the binding goroutine
  // cluster
  bool loaded = false;
  kss_cluster host{};  // sizes only (pointers not retained)
  DevCluster dc{};
  DevBuf cluster_buf;
  DevBuf pristine_buf;  // load-time copy of the mutable columns (kss_reset_node_state)
  size_t mut_bytes[KSS_NMUT] = {};
  size_t pristine_off[KSS_NMUT] = {};
  // pods
  DevBuf pod_buf;      // staged pod programs (kss_stage_pods / kss_schedule_batch)
  DevPods dp{};
  int staged_n = -1;   // pods staged in pod_buf (-1: none)
  DevBuf tmp_pod_buf;  // eval / commit / rollback uploads (never clobber the staged batch)
  DevPods tdp{};
  // outputs
  DevBuf slot_buf, meta_buf, chosen_buf, job_buf;
  size_t slot_bytes = 0;
  int recorded = 0;
  std::vector<PodMeta> meta_host;
  double last_ms = 0;
  int last_launches = 0;
  kss_host_names names;
  // host copies of the per-key tables (plan sizing), and the exchange buffers
  std::vector<int32_t> key_card_h;
  std::vector<uint32_t> key_flags_h;
  DevBuf gran_buf, err_buf;
  DevBuf cursor_buf;  // nextStartNodeIndex (one int32), kept on the device across launches
  DevBuf wffc_pod_buf;  // kss_commit / kss_rollback: the pod's program for k_wffc_commit
  // the scheduling queue's nominator (kss_nominate): host mirror in AddNominatedPod order, uploaded
  // before a launch that reads it; run_pod_base = the podset index of the launch's pod 0
  std::vector<DevNom> nom;
  std::unordered_map<int32_t, const kss_podset*> nom_src;  // index-keyed entries: the podset they index
  std::vector<int32_t> staged_uid;  // the staged pods' nominator identities (batch commits leave it)
  DevBuf nom_buf;
  bool nom_dirty = true;
  int32_t run_pod_base = 0;
  DevBuf ck_buf;                    // k_spread's checked hand-off between chunks: {sum, tag} per shard
  unsigned long long ck_seq = 0;    // the last tag a chunk wrote
  int last_handoff_retries = 0;     // prologue loads repeated in the last run (HandoffCheck)
  int last_handoff_recovered = 0;   // ... of which the shadow copy answered
  int last_handoff_final = 0;       // shards whose last write-back failed the final check (the run failed)
  size_t ck_diag_off = 0;           // ck_buf word of the diagnosis list
  bool last_kernel_spread = false;
#if KSS_SPREAD_TRACE
  DevBuf trace_buf, trace_list_buf;  // k_spread trace of the last run (kss_trace_spread)
  size_t trace_words = 0;
#endif
  int n_cu = 0;
  int force_w = 0;            // KSS_SHARDS env override (tuning / tests)
  bool xcd_mode = true;       // KSS_XCD=0: no XCD-local k_simple grids
  int xcd_w = 0;              // KSS_XCD_SHARDS: shards of an XCD-local grid (tuning; default: CUs per XCD)
  int last_xcd[2] = {0, 0};   // the last run: XCD-local grid used, chunks that fell back to an unrestricted grid
  int nodes_per_shard = 128;  // KSS_NODES_PER_SHARD (C2 sweep: 128 > 256 > 512 nodes per shard)
  int pref_threads = 256;     // KSS_THREADS
  PlanNeeds staged_need;
  int last_geom[3] = {0, 0, 0};
  bool stream_dedicated = false;      // `stream` has a hardware queue of its own (split parts: dedicated_stream)
  const char* stamps_file = nullptr;  // kss_set_stamps_file: dump per-phase timestamps of each launch
  std::string stamps_path;
  DevBuf stamp_buf;
  // compact records of the staged pods for k_simple (spod_ok false: some pod needs
  // k_schedule) and the static-word scratch of the current chunk
  DevBuf spod_buf, stat_buf;
  std::vector<SPod> spod_host;
  bool spod_ok = false;
  bool staged_names = false;  // some staged pod has a NodeAffinity PreFilterResult node list
  // host-resolved programs of the staged pods for k_spread (gpod_ok false: k_schedule)
  DevBuf gpod_buf;
  std::vector<uint4> gpod_host;  // records, gneed.gq uint4 each
  bool gpod_ok = false;
  GpodNeeds gneed;
  bool no_spread = false;     // KSS_NO_SPREAD: batches with programs always take k_schedule
  double count_bound0 = 0;    // max(Σ class_count, Σ term_count) of the loaded snapshot
  double count_bound = 0;     // the same, plus every commit since (spread_bounds_ok)
  double cell_bound0 = 0;     // max single class_count / term_count entry of the loaded snapshot
  double cell_bound = 0;      // the same, plus every commit since
  DevBuf res_buf;             // GpodNeeds::res_rows on the device
  DevBuf delta_buf;           // kss_apply_node_delta / kss_apply_count_delta staging on the device
  std::vector<char> stage_host;  // packed host image of a delta upload
  void* pinned = nullptr;     // kss_eval_pod's one-copy result staging (pinned)
  size_t pinned_cap = 0;
  void* rb = nullptr;         // run_single's read-back staging (pinned): err word, meta, chosen, slot
  size_t rb_cap = 0;
  void* up = nullptr;         // per-pod calls: pinned image of the pod's pools + the job, one upload
  size_t up_cap = 0;
  // k_schedule granules are not cleared between its launches: each launch starts its epochs
  // above every tag an earlier launch can have left (gran_epoch); 0 = clear before the next
  unsigned gran_epoch = 0;
  int staged_max_own = 0;     // max own term rows of a staged pod
  std::vector<int32_t> key_empty_h;
  bool no_simple = false;  // KSS_NO_SIMPLE: always launch k_schedule
  int last_kernel = 0;     // 0 k_schedule, 1 k_simple, 2 k_spread
  int meta_n = 0;          // pods with an outcome in meta_host
  bool small_values = false;  // every allocatable cpu/mem/eph < 2^46: k_simple's divisions stay below 2^53
  F64Bounds f64_cluster, f64_pods;  // k_simple exactness bounds of the loaded snapshot / staged pods
  bool axis_meta_dirty = false;  // meta_buf holds node-axis outcomes not yet copied to meta_host
  DevBuf axis_cv;
  int axis_max_blocks = 0;  // KSS_AXIS_BLOCKS: cap on the node-axis grid (tuning)
  int axis_no_fold = 0;      // KSS_AXIS_NO_FOLD: timing experiment only, statistics not folded (wrong results)
  std::vector<hipEvent_t> loop_ev;  // around each k_simple launch of the last batch
  double last_loop_ms = 0;          // device time of the sequential-loop kernel(s) of the last batch
  // PostFilter bound table: the loaded rows (table order), the commits / rollbacks since
  // (the load or the last kss_reset_node_state), the staged pods as bound pods, and the
  // device CSR built from them on the next dry run
  std::vector<BoundPod> bound0;
  std::vector<int32_t> bound0_node;  // local rows
  std::vector<BoundOp> bound_log;
  std::vector<BoundPod> staged_bp;
  bool bound_dirty = true;
  // a committing run failed on the device (exchange timeout): the pods it committed before the
  // abort stay on the device rows but are not in the bound-pod log; PostFilter refuses until
  // kss_reset_node_state / kss_load_cluster
  bool state_unknown = false;
  DevBuf bound_buf, pre_buf;
  DevBound bound_dev{};
  size_t bound_total = 0;  // bound pods in the table
  // the per-pod service grid (kss_service_*, kss_service.cuh)
  struct Service {
    bool running = false;          // launched and not known to have left
    hipStream_t stream = nullptr;  // its own stream (the ctx stream stays free for the copies)
    SvcBox* box = nullptr;         // pinned, coherent: ring, head, consumed, done flags, outcome
    uint8_t* rec = nullptr;        // pinned, coherent: the record (SlotLayout(N)), written by the grid
    uint8_t* rec_dev = nullptr;    // its device address
    SvcBox* box_dev = nullptr;
    size_t rec_bytes = 0;
    void* rec_map = nullptr;       // KSS_SVC_HUGE: the record in a registered 2 MiB-aligned mapping
    size_t rec_map_bytes = 0;
    DevBuf relay, gran, err, job;  // device relay ring + seen counters, granules, error word, DevJob
    unsigned long long posted = 0; // commands written to the ring
    int W = 0, threads = 0, npt = 0, bins_cap = 0, cache_keys = -1;
    size_t shmem = 0;
    bool gen = false;
    bool simple = false;  // the k_simple-shaped evaluation (svc_simple_eval)
    DevBuf stat;          // its static words of every staged pod (k_static at the start)
    bool xcd = false;     // ... on an XCD-local grid (xcd_slot)
  } svc;
  // split grid (kss_split_*): this context runs part split_part of split_n, split_wl shards
  // each; split_inbox is its exchange inbox (uncached device memory, zeroed once), split_peer
  // every part's inbox as addressable here (IPC-mapped for other processes / GPUs)
  int split_n = 0, split_part = 0, split_wl = 0;
  void* split_inbox = nullptr;
  size_t split_inbox_bytes = 0;
  unsigned long long* split_peer[KSS_MAX_PARTS] = {};
  std::vector<void*> split_opened;  // hipIpcOpenMemHandle mappings to close
  bool split_ready = false;
  bool split_broken = false;  // a failed split run: refuse until re-armed (run_single)
  unsigned split_epoch = 0;
  // loop-kernel launches (chunks) run so far on this part since the last re-arm: chunk q
  // exchanges through inbox half q & 1, so a fast part starting chunk q + 1 never overwrites
  // a granule of chunk q that a slower peer has yet to read (every part runs the same chunks)
  unsigned long long split_chunks = 0;
};

namespace {

// Copy a host podset into a device buffer; fills dp with device pointers.
int upload_podset(hipStream_t st, DevBuf& buf, const kss_podset* ps, DevPods& dp) {
  const size_t sz_pods = sizeof(kss_pod) * (size_t)std::max(ps->n_pods, 1);
  const size_t sz_reqs = sizeof(kss_req) * (size_t)std::max(ps->n_reqs, 1);
  const size_t sz_terms = sizeof(kss_term) * (size_t)std::max(ps->n_terms, 1);
  const size_t sz_spr = sizeof(kss_spread) * (size_t)std::max(ps->n_spreads, 1);
  const size_t sz_ipa = sizeof(kss_ipa) * (size_t)std::max(ps->n_ipa, 1);
  const size_t sz_ints = sizeof(int32_t) * (size_t)std::max(ps->n_ints, 1);
  const size_t sz_vols = sizeof(kss_vol) * (size_t)std::max(ps->n_vols, 1);
  size_t o_pods = 0, o_reqs = align_up(o_pods + sz_pods, 256), o_terms = align_up(o_reqs + sz_reqs, 256),
         o_spr = align_up(o_terms + sz_terms, 256), o_ipa = align_up(o_spr + sz_spr, 256),
         o_ints = align_up(o_ipa + sz_ipa, 256), o_vols = align_up(o_ints + sz_ints, 256),
         total = align_up(o_vols + sz_vols, 256);
  int rc = buf.ensure(total);
  if (rc) return rc;
  char* b = (char*)buf.p;
  if (ps->n_pods) HIP_TRY(hipMemcpyAsync(b + o_pods, ps->pods, sizeof(kss_pod) * ps->n_pods, hipMemcpyHostToDevice, st));
  if (ps->n_reqs) HIP_TRY(hipMemcpyAsync(b + o_reqs, ps->reqs, sizeof(kss_req) * ps->n_reqs, hipMemcpyHostToDevice, st));
  if (ps->n_terms) HIP_TRY(hipMemcpyAsync(b + o_terms, ps->terms, sizeof(kss_term) * ps->n_terms, hipMemcpyHostToDevice, st));
  if (ps->n_spreads) HIP_TRY(hipMemcpyAsync(b + o_spr, ps->spreads, sizeof(kss_spread) * ps->n_spreads, hipMemcpyHostToDevice, st));
  if (ps->n_ipa) HIP_TRY(hipMemcpyAsync(b + o_ipa, ps->ipa, sizeof(kss_ipa) * ps->n_ipa, hipMemcpyHostToDevice, st));
  if (ps->n_ints) HIP_TRY(hipMemcpyAsync(b + o_ints, ps->ints, sizeof(int32_t) * ps->n_ints, hipMemcpyHostToDevice, st));
  if (ps->n_vols) HIP_TRY(hipMemcpyAsync(b + o_vols, ps->vols, sizeof(kss_vol) * ps->n_vols, hipMemcpyHostToDevice, st));
  dp.pods = (const kss_pod*)(b + o_pods);
  dp.reqs = (const kss_req*)(b + o_reqs);
  dp.terms = (const kss_term*)(b + o_terms);
  dp.spreads = (const kss_spread*)(b + o_spr);
  dp.ipa = (const kss_ipa*)(b + o_ipa);
  dp.ints = (const int32_t*)(b + o_ints);
  dp.vols = (const kss_vol*)(b + o_vols);
  return 0;
}

// One upload for a per-pod call: the pod's pools and `extra` trailing bytes (the launch's
// job) as one pinned image; run_single fills the job and issues the single copy.
struct PackedUpload {
  char* host = nullptr;  // pinned image
  char* dev = nullptr;
  size_t bytes = 0;
  size_t extra_off = 0;
  size_t tail = 0;        // device bytes reserved after the image (not uploaded): the per-pod record slot
  char* slot = nullptr;   // dev + align_up(bytes, 256) when tail > 0
};

int pack_podset(DevBuf& buf, void*& pin, size_t& pin_cap, const kss_podset* ps, size_t extra, DevPods& dp,
                PackedUpload& pu) {
  const size_t sz[7] = {sizeof(kss_pod) * (size_t)ps->n_pods, sizeof(kss_req) * (size_t)ps->n_reqs,
                        sizeof(kss_term) * (size_t)ps->n_terms, sizeof(kss_spread) * (size_t)ps->n_spreads,
                        sizeof(kss_ipa) * (size_t)ps->n_ipa, sizeof(int32_t) * (size_t)ps->n_ints,
                        sizeof(kss_vol) * (size_t)ps->n_vols};
  const void* src[7] = {ps->pods, ps->reqs, ps->terms, ps->spreads, ps->ipa, ps->ints, ps->vols};
  size_t off[7], o = 0;
  for (int i = 0; i < 7; i++) {
    off[i] = o;
    o = align_up(o + std::max(sz[i], (size_t)16), 64);
  }
  pu.extra_off = o;
  pu.bytes = align_up(o + extra, 64);
  int rc = buf.ensure(align_up(pu.bytes, 256) + pu.tail);
  if (rc) return rc;
  if (pin_cap < pu.bytes) {
    if (pin) HIP_TRY(hipHostFree(pin));
    pin = nullptr;
    pin_cap = 0;
    HIP_TRY(hipHostMalloc(&pin, std::max(pu.bytes, (size_t)65536), hipHostMallocDefault));
    pin_cap = std::max(pu.bytes, (size_t)65536);
  }
  pu.host = (char*)pin;
  pu.dev = (char*)buf.p;
  pu.slot = pu.tail ? pu.dev + align_up(pu.bytes, 256) : nullptr;
  for (int i = 0; i < 7; i++)
    if (sz[i]) std::memcpy(pu.host + off[i], src[i], sz[i]);
  dp.pods = (const kss_pod*)(pu.dev + off[0]);
  dp.reqs = (const kss_req*)(pu.dev + off[1]);
  dp.terms = (const kss_term*)(pu.dev + off[2]);
  dp.spreads = (const kss_spread*)(pu.dev + off[3]);
  dp.ipa = (const kss_ipa*)(pu.dev + off[4]);
  dp.ints = (const int32_t*)(pu.dev + off[5]);
  dp.vols = (const kss_vol*)(pu.dev + off[6]);
  return 0;
}

// Validate podset references against the cluster shape (a malformed program must
// never reach the kernel: out-of-range ids would fault the device).
int validate(const kss_cluster* cl, const kss_podset* ps, int n) {
  if (n < 0 || n > ps->n_pods) return fail(KSS_E_INVAL, "pod count out of range");
  auto in = [](int64_t off, int64_t len, int64_t cap) { return off >= 0 && len >= 0 && off + len <= cap; };
  for (int i = 0; i < ps->n_reqs; i++) {
    const kss_req& r = ps->reqs[i];
    const bool keyed = r.op >= KSS_OP_MASK && r.op <= KSS_OP_LT;
    if (r.op < KSS_OP_FALSE || r.op > KSS_OP_NAME_NOTIN) return fail(KSS_E_INVAL, "bad requirement op");
    if (keyed && (r.key < 0 || r.key >= cl->n_label_keys)) return fail(KSS_E_INVAL, "requirement key out of range");
    if ((r.op == KSS_OP_IN || r.op == KSS_OP_NOTIN) && !in(r.list_off, r.list_len, ps->n_ints))
      return fail(KSS_E_INVAL, "requirement list out of range");
  }
  for (int i = 0; i < ps->n_terms; i++)
    if (!in(ps->terms[i].req_off, ps->terms[i].req_len, ps->n_reqs)) return fail(KSS_E_INVAL, "term out of range");
  for (int i = 0; i < ps->n_spreads; i++) {
    const kss_spread& s = ps->spreads[i];
    if (s.key < 0 || s.key >= cl->n_label_keys) return fail(KSS_E_INVAL, "spread key out of range");
    if (!in(s.cls_off, s.cls_len, ps->n_ints)) return fail(KSS_E_INVAL, "spread class list out of range");
    for (int j = 0; j < s.cls_len; j++)
      if (ps->ints[s.cls_off + j] < 0 || ps->ints[s.cls_off + j] >= cl->n_classes) return fail(KSS_E_INVAL, "class id out of range");
    if (!(cl->key_flags[s.key] & (KSS_KEY_UNIQUE | KSS_KEY_HOSTNAME)) && cl->key_card[s.key] + 1 > KSS_MAX_BINS)
      return fail(KSS_E_UNSUPPORTED, "non-unique topology key with more than KSS_MAX_BINS domains");
  }
  for (int i = 0; i < ps->n_ipa; i++) {
    const kss_ipa& e = ps->ipa[i];
    if (e.key < 0 || e.key >= cl->n_label_keys) return fail(KSS_E_INVAL, "ipa key out of range");
    if (!in(e.row_off, e.row_len, ps->n_ints)) return fail(KSS_E_INVAL, "ipa rows out of range");
    const bool terms = e.kind == KSS_IPA_EXISTING_ANTI || e.kind == KSS_IPA_SCORE_TERM;
    const int cap = terms ? cl->n_terms : cl->n_classes;
    for (int j = 0; j < e.row_len; j++)
      if (ps->ints[e.row_off + j] < 0 || ps->ints[e.row_off + j] >= cap) return fail(KSS_E_INVAL, "ipa row id out of range");
    if (!(cl->key_flags[e.key] & KSS_KEY_UNIQUE) && cl->key_card[e.key] + 1 > KSS_MAX_BINS)
      return fail(KSS_E_UNSUPPORTED, "non-unique topology key with more than KSS_MAX_BINS domains");
  }
  if (ps->n_vols < 0 || (ps->n_vols > 0 && !ps->vols)) return fail(KSS_E_INVAL, "bad volume pool");
  for (int i = 0; i < ps->n_vols; i++) {
    const kss_vol& v = ps->vols[i];
    switch (v.kind) {
      case KSS_VOL_CONFLICT:
      case KSS_VOL_OWN:
        if (v.row < 0 || v.row >= cl->n_vol_rows) return fail(KSS_E_INVAL, "volume row out of range");
        break;
      case KSS_VOL_LIMIT:
        if (v.key < 0 || v.key >= cl->n_vol_keys || v.row >= cl->n_vol_rows || (v.row < 0 && v.count < 0))
          return fail(KSS_E_INVAL, "volume limit entry out of range");
        break;
      case KSS_VOL_OWN_PRIVATE:
        if (v.key < 0 || v.key >= cl->n_vol_keys || v.count < 0) return fail(KSS_E_INVAL, "volume key out of range");
        break;
      case KSS_VOL_BIND_AFFINITY:
        if (!in(v.a, v.b, ps->n_terms)) return fail(KSS_E_INVAL, "volume node affinity terms out of range");
        break;
      case KSS_VOL_ZONE:
        if (!in(v.a, v.b, ps->n_reqs)) return fail(KSS_E_INVAL, "volume zone requirements out of range");
        break;
      case KSS_VOL_ZONE_ERROR:
        if (v.a < 0 || v.a > 65534) return fail(KSS_E_INVAL, "volume zone message out of range");
        break;
      case KSS_VOL_BIND_PV_MISSING:
        break;
      case KSS_VOL_BIND_WFFC:
        if (v.key < 0 || v.key >= cl->n_wclaims || v.b < 0 || !in(v.a, 3 * (int64_t)v.b, ps->n_ints) ||
            !in(v.row, v.count >> 1, ps->n_terms) || v.count < 0)
          return fail(KSS_E_INVAL, "WaitForFirstConsumer claim entry out of range");
        for (int j = 0; j < v.b; j++) {
          const int32_t pv = ps->ints[v.a + 3 * j], ta = ps->ints[v.a + 3 * j + 1], tb = ps->ints[v.a + 3 * j + 2];
          if (pv < 0 || pv >= cl->n_pvs || (tb >= 0 && !in(ta, tb, ps->n_terms)) || tb < -1)
            return fail(KSS_E_INVAL, "WaitForFirstConsumer candidate out of range");
        }
        break;
      default:
        return fail(KSS_E_INVAL, "bad volume entry kind");
    }
  }
  for (int i = 0; i < n; i++) {
    const kss_pod& p = ps->pods[i];
    if (p.prefilter_status < KSS_PF_OK || p.prefilter_status > KSS_PF_VOLUME_BINDING)
      return fail(KSS_E_INVAL, "bad prefilter status");
    if (!in(p.vol_off, p.vol_len, ps->n_vols)) return fail(KSS_E_INVAL, "pod volume program out of range");
    {
      int nw = 0;
      for (int e = 0; e < p.vol_len; e++) nw += ps->vols[p.vol_off + e].kind == KSS_VOL_BIND_WFFC;
      if (nw > KSS_MAX_WFFC) return fail(KSS_E_UNSUPPORTED, "more than KSS_MAX_WFFC delayed claims in one pod");
    }
    if (!in(p.sel_off, p.sel_len, ps->n_reqs) || !in(p.aff_off, p.aff_len, ps->n_terms) ||
        !in(p.pref_off, p.pref_len, ps->n_terms) || !in(p.spread_off, (int64_t)p.n_hard + p.n_soft, ps->n_spreads) ||
        !in(p.ipa_off, p.ipa_len, ps->n_ipa) || !in(p.own_terms_off, p.own_terms_len, ps->n_ints))
      return fail(KSS_E_INVAL, "pod program out of range");
    if (p.names_len >= 0 && !in(p.names_off, p.names_len, ps->n_ints)) return fail(KSS_E_INVAL, "pod names out of range");
    for (int j = 0; j < p.names_len; j++)  // the PreFilterResult list in canonical order (findNodesThatPassFilters' node list)
      if (ps->ints[p.names_off + j] < 0 || (j > 0 && ps->ints[p.names_off + j] <= ps->ints[p.names_off + j - 1]))
        return fail(KSS_E_INVAL, "PreFilterResult node indices must be ascending and distinct");
    if (p.cls >= cl->n_classes) return fail(KSS_E_INVAL, "pod class out of range");
    for (int j = 0; j < p.own_terms_len; j++)
      if (ps->ints[p.own_terms_off + j] < 0 || ps->ints[p.own_terms_off + j] >= cl->n_terms)
        return fail(KSS_E_INVAL, "own term id out of range");
    if (p.n_hard > MAXH || p.n_soft > MAXS) return fail(KSS_E_UNSUPPORTED, "too many spread constraints for the device path");
    if (cl->n_ports < KSS_MAX_PORTS && ((p.port_conflict | p.port_add) >> cl->n_ports))
      return fail(KSS_E_INVAL, "pod port bit outside the port dictionary");
    if (p.img_len > 0) {
      if (!in(p.img_off, p.img_len, ps->n_ints) || p.n_containers < 1) return fail(KSS_E_INVAL, "pod image rows out of range");
      for (int j = 0; j < p.img_len; j++)
        if (ps->ints[p.img_off + j] < 0 || ps->ints[p.img_off + j] >= cl->n_images)
          return fail(KSS_E_INVAL, "image row id out of range");
    }
  }
  return 0;
}

// k_simple holds node state and pod requests as integers in doubles (kss_simple.cuh
// SPod): exact while every value and every sum the loop can form stays below 2^53.
// Cluster side: the largest snapshot Requested / NonZeroRequested (cpu, memory,
// ephemeral); pod side: the largest request of any kind.  A node's Requested grows by
// at most n_pods commits of the largest commit delta (a bound that holds even without
// the NodeResourcesFit filter).
void f64_bounds_cluster(const kss_cluster* cl, F64Bounds& b) {
  const size_t N = (size_t)cl->n_nodes;
  for (size_t i = 0; i < 3 * N; i++) {
    b.neg |= cl->requested[i] < 0;
    b.max_req0 = std::max(b.max_req0, (double)cl->requested[i]);
  }
  for (size_t i = 0; i < 2 * N; i++) {
    b.neg |= cl->nonzero[i] < 0;
    b.max_nz0 = std::max(b.max_nz0, (double)cl->nonzero[i]);
  }
}
void f64_bounds_pods(const kss_podset* ps, F64Bounds& b) {
  for (int i = 0; i < ps->n_pods; i++) {
    const kss_pod& p = ps->pods[i];
    for (int r = 0; r < 3; r++) {
      const int64_t v[4] = {p.fit_request[r], p.score_req_nz[r], p.score_req[r], p.commit_req[r]};
      for (int64_t x : v) {
        b.neg |= x < 0;
        b.max_pod = std::max(b.max_pod, (double)x);
      }
      b.max_creq = std::max(b.max_creq, (double)p.commit_req[r]);
    }
    for (int r = 0; r < 2; r++) {
      b.neg |= p.commit_nz[r] < 0;
      b.max_cnz = std::max(b.max_cnz, (double)p.commit_nz[r]);
      b.max_pod = std::max(b.max_pod, (double)p.commit_nz[r]);
    }
  }
}
bool f64_exact(const F64Bounds& c, const F64Bounds& p, int n_pods) {
  const double lim = 4503599627370496.0;  // 2^52: sums of two such values stay below 2^53
  return !c.neg && !p.neg && p.max_pod < lim && c.max_req0 + (double)n_pods * p.max_creq < lim &&
         c.max_nz0 + (double)n_pods * p.max_cnz < lim;
}

// Compact record of one pod (kss_simple.cuh SPod); false when the preferred NodeAffinity
// weights do not fit the static word's 20 bits.
bool fill_spod(const kss_podset* ps, const kss_pod& p, int n_scalar, SPod& q) {
  if (p.port_conflict | p.port_add || p.img_len > 0 || p.vol_len > 0) return false;  // NodePorts / ImageLocality / volumes: k_schedule
  int64_t wsum = 0;
  for (int t = 0; t < p.pref_len; t++) wsum += std::max(0, ps->terms[p.pref_off + t].weight);
  if (wsum > 0xFFFFF) return false;  // static word: 20 bits of raw NodeAffinity
  q = SPod{};
  bool all_zero = true;
  for (int r = 0; r < 3 + n_scalar; r++) all_zero &= p.fit_request[r] == 0;
  for (int r = 0; r < 3; r++) {
    q.fit_req[r] = (double)p.fit_request[r];
    q.snz[r] = (double)p.score_req_nz[r];
    q.sreq[r] = (double)p.score_req[r];
    q.creq[r] = (double)p.commit_req[r];
  }
  q.cnz[0] = (double)p.commit_nz[0];
  q.cnz[1] = (double)p.commit_nz[1];
  for (int s = 0; s < n_scalar; s++) {
    q.sc_fit[s] = p.fit_request[3 + s];
    q.sc_req[s] = p.commit_req[3 + s];
  }
  q.flags = all_zero ? SP_ALLZERO : 0;
  q.status = p.prefilter_status;
  q.cls = p.cls;
  q.own_off = p.own_terms_off;
  q.own_len = p.own_terms_len;
  return true;
}

// Compact records of every pod of a (validated) podset for k_simple; false when some pod
// needs another kernel (spread / inter-pod-affinity programs, or fill_spod refuses it).
bool build_spods(const kss_podset* ps, int n_scalar, std::vector<SPod>& out) {
  out.assign((size_t)std::max(ps->n_pods, 1), SPod{});
  for (int i = 0; i < ps->n_pods; i++) {
    const kss_pod& p = ps->pods[i];
    if (p.n_hard | p.n_soft | p.ipa_len) return false;
    if (!fill_spod(ps, p, n_scalar, out[(size_t)i])) return false;
  }
  return true;
}

// Host-resolved programs (kss_spread.cuh GPod) of every pod of a validated podset: the
// restatement of make_plan (kss_sched.cuh), every constraint / entry as (resident count row,
// coefficient) references, InterPodAffinity score entries merged per topology key, and the
// batch's resident row set (every row some pod reads).  False when some pod exceeds the
// record's fixed tables or an exchange's payload (the batch then runs on k_schedule).
// Why build_gpods refused a batch (kss_plan_podset): code, pod.
enum {
  GP_OK = 0,
  GP_NA_WEIGHTS,
  GP_CONSTRAINTS,
  GP_ROWS,
  GP_COEF,
  GP_REFS,
  GP_KEYS,
  GP_BINS,
  GP_XW,
  GP_COMMIT,
  GP_RECORD,
  GP_IPA,
  GP_SCALAR,
  GP_PORTS_IMAGES,
  GP_PCT,
  GP_SCALAR_SCORED,
  GP_NCODES
};
const char* const kGpReason[GP_NCODES] = {
    "eligible",
    "preferred NodeAffinity weights exceed the static word",
    "more than 4 spread constraints of one kind",
    "more than 65536 resident count rows",
    "a merged score coefficient exceeds 16 bits",
    "too many count-row references",
    "more than 4 inter-pod-affinity topology keys",
    "too many histogram bins",
    "exchange payload too large",
    "the commit adds to more than 8 count rows",
    "a pod's record exceeds 2 KiB (too many references)",
    "more than 16 inter-pod-affinity entries after merging",
    "the profile scores an extended (scalar) resource: k_simple / k_spread score cpu, memory and ephemeral-storage only",
    "host ports (NodePorts), node-cached images (ImageLocality) or volumes: k_schedule only",
    "percentageOfNodesToScore below 100 (numFeasibleNodesToFind / nextStartNodeIndex window): k_simple, and k_spread "
    "under the default profile, for pods without a NodeAffinity PreFilterResult list, else k_schedule",
    "the profile scores an extended (scalar) resource and the cluster has extended resources: k_schedule only",
};

bool gfail(GpodNeeds& need, int code, int pod) {
  need.fail_code = code;
  need.fail_pod = pod;
  return false;
}

bool build_gpods(const kss_podset* ps, int n_scalar, int n_classes, const int32_t* key_card, const uint32_t* key_flags,
                 const int32_t* key_empty, std::vector<uint4>& words, GpodNeeds& need) {
  std::vector<GPod> out((size_t)std::max(ps->n_pods, 1), GPod{});
  std::vector<std::vector<uint32_t>> refs_of((size_t)std::max(ps->n_pods, 1));
  need = GpodNeeds{};
  std::vector<int32_t> local;  // count row -> resident index (-1 none)
  auto res_of = [&](int rowid) -> int {
    if ((size_t)rowid >= local.size()) local.resize((size_t)rowid + 1, -1);
    if (local[(size_t)rowid] < 0) {
      local[(size_t)rowid] = (int32_t)need.res_rows.size();
      need.res_rows.push_back(rowid);
    }
    return local[(size_t)rowid];
  };
  for (int i = 0; i < ps->n_pods; i++) {
    const kss_pod& p = ps->pods[i];
    GPod& g = out[(size_t)i];
    std::vector<uint32_t>& R = refs_of[(size_t)i];
    if (p.port_conflict | p.port_add || p.img_len > 0 || p.vol_len > 0) return gfail(need, GP_PORTS_IMAGES, i);
    if (!fill_spod(ps, p, n_scalar, g.dyn)) return gfail(need, GP_NA_WEIGHTS, i);
    if (p.n_hard > MAXH || p.n_soft > MAXS) return gfail(need, GP_CONSTRAINTS, i);
    g.pflags = (int32_t)p.flags;
    g.n_hard = p.n_hard;
    g.n_soft = p.n_soft;
    // references [ri_off, +ri_len) for (rowid, coef) pairs, equal rows merged:
    // resident row index | coefficient << 16
    std::vector<int64_t> coef;
    auto refs = [&](const std::vector<std::pair<int, int64_t>>& rows, int16_t& ri_off, int16_t& ri_len) -> bool {
      const int o = (int)R.size();
      for (const auto& rc : rows) {
        const int l = res_of(rc.first);
        if (l > 0xFFFF) return gfail(need, GP_ROWS, i);
        int j = o;
        while (j < (int)R.size() && (int)(R[(size_t)j] & 0xFFFFu) != l) j++;
        if (j == (int)R.size()) {
          R.push_back((uint32_t)l);
          coef.push_back(0);
        }
        coef[(size_t)j] += rc.second;
        if (coef[(size_t)j] < -32768 || coef[(size_t)j] > 32767) return gfail(need, GP_COEF, i);
      }
      int64_t wsum = 0;
      for (size_t j = (size_t)o; j < R.size(); j++) {
        R[j] = (R[j] & 0xFFFFu) | ((uint32_t)(uint16_t)(int16_t)coef[j] << 16);
        wsum += std::abs(coef[j]);
      }
      if (R.size() > 32767) return gfail(need, GP_REFS, i);
      ri_off = (int16_t)o;
      ri_len = (int16_t)(R.size() - (size_t)o);
      need.ref_weight = std::max(need.ref_weight, wsum);
      return true;
    };
    auto list = [&](int off, int len, bool term) {
      std::vector<std::pair<int, int64_t>> v;
      for (int j = 0; j < len; j++) v.push_back({(term ? n_classes : 0) + ps->ints[off + j], 1});
      return v;
    };
    int off = 0, poff = 0;
    bool stats = false;
    const kss_spread* sp = ps->spreads + p.spread_off;
    for (int c = 0; c < p.n_hard + p.n_soft; c++) {
      const kss_spread& s = sp[c];
      GSpread& d = g.sp[c];
      d.key = (int16_t)s.key;
      d.max_skew = s.max_skew;
      d.self_match = (int16_t)s.self_match;
      d.flags = (int16_t)s.flags;
      if (!refs(list(s.cls_off, s.cls_len, false), d.ri_off, d.ri_len)) return gfail(need, GP_REFS, i);
      d.empty = (int16_t)key_empty[s.key];
      d.nb = (int16_t)(key_card[s.key] + 1);
      d.off = d.poff = -1;
      d.mode = SOFT_HOST;
    }
    // groups: constraints of one kind on one topology key share the leader's bins (v1.26
    // keys the counts by topology pair; kss_spread.cuh GSpread)
    auto leader = [&](int c, int lo_c) {
      for (int j = lo_c; j < c; j++)
        if (g.sp[j].key == g.sp[c].key) return j;
      return c;
    };
    for (int c = 0; c < p.n_hard; c++) {  // make_plan: hard bins first
      GSpread& d = g.sp[c];
      stats = true;
      d.own = (int16_t)leader(c, 0);
      if (d.own != c) {
        d.off = g.sp[d.own].off;
        d.poff = g.sp[d.own].poff;
      } else if (!(key_flags[d.key] & KSS_KEY_UNIQUE)) {
        d.off = (int16_t)off;
        d.poff = (int16_t)poff;
        off += d.nb;
        poff += d.nb;
      }
    }
    g.hard_pbins = poff;
    for (int c = p.n_hard; c < p.n_hard + p.n_soft; c++) {
      GSpread& d = g.sp[c];
      const bool host = (key_flags[d.key] & KSS_KEY_HOSTNAME) != 0;
      d.own = (int16_t)(host ? c : leader(c, p.n_hard));  // hostname constraints are never grouped
      if (host) {
        d.mode = SOFT_HOST;
      } else if (key_flags[d.key] & KSS_KEY_UNIQUE) {
        d.mode = SOFT_DIRECT;
      } else {
        d.mode = SOFT_HIST;
        stats = true;
        if (d.own != c) {
          d.off = g.sp[d.own].off;
          d.poff = g.sp[d.own].poff;
        } else {
          d.off = (int16_t)off;
          d.poff = (int16_t)poff;
          off += d.nb;
          poff += d.nb;
        }
      }
      if (p.n_soft > 1) {
        need.max_soft = std::max(need.max_soft, (int)p.n_soft);
        need.max_skew = std::max<int64_t>(need.max_skew, std::abs((int64_t)d.max_skew));
      }
    }
    // inter-pod affinity: key slots in entry order (make_plan), score entries merged per slot
    const kss_ipa* ip = ps->ipa + p.ipa_off;
    std::vector<int> slot_of((size_t)std::max(p.ipa_len, 1));
    for (int e = 0; e < p.ipa_len; e++) {
      int k = -1;
      for (int j = 0; j < g.n_keys; j++)
        if (g.key[j] == ip[e].key) k = j;
      if (k < 0) {
        if (g.n_keys >= MAXK) return gfail(need, GP_KEYS, i);
        k = g.n_keys++;
        g.key[k] = ip[e].key;
        for (int h = 0; h < 4; h++) g.hoff[k][h] = -1;
      }
      slot_of[e] = k;
    }
    bool used[MAXK][4] = {};
    for (int e = 0; e < p.ipa_len; e++) {
      const kss_ipa& en = ip[e];
      stats = true;
      if (en.kind == KSS_IPA_SCORE_CLASS || en.kind == KSS_IPA_SCORE_TERM) continue;
      if (g.n_ipa >= G_IPA) return gfail(need, GP_IPA, i);
      GIpa& d = g.ipa[g.n_ipa++];
      d.kind = (int16_t)en.kind;
      d.key = (int16_t)en.key;
      d.slot = (int16_t)slot_of[e];
      if (!refs(list(en.row_off, en.row_len, en.kind == KSS_IPA_EXISTING_ANTI), d.ri_off, d.ri_len)) return gfail(need, GP_REFS, i);
      used[slot_of[e]][en.kind == KSS_IPA_EXISTING_ANTI ? 0 : (en.kind == KSS_IPA_REQ_AFFINITY ? 1 : 2)] = true;
    }
    for (int k = 0; k < g.n_keys; k++) {
      std::vector<std::pair<int, int64_t>> rows;
      for (int e = 0; e < p.ipa_len; e++) {
        const kss_ipa& en = ip[e];
        if (slot_of[e] != k || (en.kind != KSS_IPA_SCORE_CLASS && en.kind != KSS_IPA_SCORE_TERM)) continue;
        for (int j = 0; j < en.row_len; j++)
          rows.push_back({(en.kind == KSS_IPA_SCORE_TERM ? n_classes : 0) + ps->ints[en.row_off + j], (int64_t)en.coef});
      }
      if (rows.empty()) continue;
      if (g.n_ipa >= G_IPA) return gfail(need, GP_IPA, i);
      GIpa& d = g.ipa[g.n_ipa++];
      d.kind = G_SCORE;
      d.key = (int16_t)g.key[k];
      d.slot = (int16_t)k;
      if (!refs(rows, d.ri_off, d.ri_len)) return gfail(need, GP_REFS, i);
      used[k][3] = true;
    }
    for (int k = 0; k < g.n_keys; k++) {  // one histogram per (shared key, kind) some entry feeds
      if (key_flags[g.key[k]] & KSS_KEY_UNIQUE) continue;
      for (int h = 0; h < 4; h++)
        if (used[k][h]) {
          g.hoff[k][h] = off;
          off += key_card[g.key[k]] + 1;
        }
    }
    g.total_bins = off;
    g.total_pbins = poff;
    g.need_stats = stats ? 1 : 0;
    if (off + poff > LDS_BINS || off > 32767 || poff > 32767) return gfail(need, GP_BINS, i);
    // exchanges: E1 (scalars + bins), E2 (scalars + soft presence)
    if (MAXH + 1 + off + g.hard_pbins > G_XW || 13 + (poff - g.hard_pbins) > G_XW) return gfail(need, GP_XW, i);
    need.xw = std::max(need.xw, std::max(MAXH + 1 + off + g.hard_pbins, 13 + (poff - g.hard_pbins)));
    // the statistics exchange folded into the previous pod's filter exchange and argmax
    // (kss_spread.cuh spread_argmax_pay): histogram-valued DoNotSchedule groups only (a
    // node-valued group's critical path is a minimum over nodes, which a single node's delta
    // cannot update); the previous pod's filter exchange (at most 14 scalars and its soft
    // presence) carries this pod's bins and hard presence, its argmax one payload per
    // constraint / entry.  need.fold_xw / soft_xw bound the widest such pair (checked below).
    g.fold = 0;
    if (stats) {
      bool node_valued = false;
      for (int c = 0; c < p.n_hard; c++) node_valued |= g.sp[c].off < 0;
      const int np = p.n_hard + p.n_soft + g.n_ipa + (g.n_ipa > 0 ? 1 : 0);
      if (!node_valued && np <= G_PAY && 1 + np <= G_XW && off + g.hard_pbins <= G_XW) {
        g.fold = 1;
        need.fold_xw = std::max(need.fold_xw, off + g.hard_pbins);
        need.xw = std::max(need.xw, 1 + np);
      }
    }
    need.soft_xw = std::max(need.soft_xw, poff - g.hard_pbins);
    need.bins_cap = std::max(need.bins_cap, off + poff);
    // AssumePod's count rows: the pod's class, its own term rows
    if (1 + p.own_terms_len > G_CMT) return gfail(need, GP_COMMIT, i);
    auto cmt_of = [&](int rowid) -> int32_t {
      const int l = (size_t)rowid < local.size() ? local[(size_t)rowid] : -1;
      return l >= 0 ? l : -1 - rowid;
    };
    g.n_cmt = 0;
    if (p.cls >= 0) g.cmt[g.n_cmt++] = cmt_of(p.cls);
    for (int j = 0; j < p.own_terms_len; j++) {
      g.cmt[g.n_cmt++] = cmt_of(n_classes + ps->ints[p.own_terms_off + j]);
      int m = 0;
      for (int x = 0; x < p.own_terms_len; x++) m += ps->ints[p.own_terms_off + x] == ps->ints[p.own_terms_off + j];
      need.max_mult = std::max(need.max_mult, m);
    }
  }
  // a folded delta travels as int16 (payload low half): Σ|coefficient| x commits per row bounds it.
  // Opt-in (KSS_FOLD=1): measured no faster on C4 and slower on C3
  if (need.ref_weight * need.max_mult > 32767 || !opt(O_FOLD) || 14 + need.soft_xw + need.fold_xw > G_XW)
    for (int i = 0; i < ps->n_pods; i++) out[(size_t)i].fold = 0;
  else
    need.xw = std::max(need.xw, 14 + need.soft_xw + need.fold_xw);
  // rows first read by a later pod than one committing to them: re-resolve the commits
  size_t rmax = 0;
  int rmax_pod = 0;
  for (int i = 0; i < ps->n_pods; i++) {
    GPod& g = out[(size_t)i];
    for (int j = 0; j < g.n_cmt; j++)
      if (g.cmt[j] < 0) {
        const int rowid = -1 - g.cmt[j];
        if ((size_t)rowid < local.size() && local[(size_t)rowid] >= 0) g.cmt[j] = local[(size_t)rowid];
      }
    if (refs_of[(size_t)i].size() > rmax) {
      rmax = refs_of[(size_t)i].size();
      rmax_pod = i;
    }
  }
  // records: header + references, one stride of gq uint4 each
  const size_t gq = (sizeof(GPod) + 4 * rmax + 15) / 16;
  if (gq > (size_t)G_QMAX) return gfail(need, GP_RECORD, rmax_pod);
  need.gq = (int)gq;
  words.assign(gq * out.size(), uint4{0, 0, 0, 0});
  for (size_t i = 0; i < out.size(); i++) {
    char* rec = reinterpret_cast<char*>(words.data() + i * gq);
    std::memcpy(rec, &out[i], sizeof(GPod));
    if (!refs_of[i].empty()) std::memcpy(rec + sizeof(GPod), refs_of[i].data(), 4 * refs_of[i].size());
  }
  return true;
}

// k_spread keeps counts, histograms and scores in 32 bits and resident counts in 16: with
// `total` a bound on every count row's sum over the cluster after the batch and `cell` a
// bound on every single count, a reference sum (one constraint / entry) is below
// ref_weight * total over any node set, an InterPodAffinity score below MAXK times that,
// and a multi-constraint PodTopologySpread raw score below
// max_soft * (count * log(N + 2) + maxSkew).
bool spread_bounds_ok(const GpodNeeds& q, double total, double cell, int N) {
  const double lim = 2147483647.0;
  const double ref = (double)q.ref_weight * total;
  if (cell > 65535.0 || (double)MAXK * ref >= lim) return false;
  if (q.max_soft > 1 && (double)q.max_soft * (ref * std::log((double)N + 2.0) + (double)q.max_skew + 1.0) >= lim)
    return false;
  return true;
}

struct ClusterLayout {
  size_t o_alloc, o_req, o_nz, o_allowed, o_podc, o_flags, o_th, o_ts, o_to, o_lv, o_kb, o_kc, o_kf, o_ke, o_vi, o_vii,
      o_cc, o_tc, o_log, o_pu, o_img, o_vc, o_va, o_vl, o_vrk, o_vkp, o_pvo, o_cln, total;
  ClusterLayout(const kss_cluster* cl, int class_cap, int term_cap) {
    const size_t N = (size_t)cl->n_nodes;
    size_t o = 0;
    auto take = [&](size_t bytes) {
      size_t r = o;
      o = align_up(o + std::max(bytes, (size_t)8), 256);
      return r;
    };
    o_alloc = take(8 * KSS_NRES * N);
    o_req = take(8 * KSS_NRES * N);
    o_nz = take(8 * 2 * N);
    o_allowed = take(4 * N);
    o_podc = take(4 * N);
    o_flags = take(4 * N);
    o_th = take(8 * N);
    o_ts = take(8 * N);
    o_to = take((size_t)KSS_TAINT_ORDER * N);
    o_lv = take(4 * (size_t)cl->n_label_keys * N);
    o_kb = take(4 * (size_t)cl->n_label_keys);
    o_kc = take(4 * (size_t)cl->n_label_keys);
    o_kf = take(4 * (size_t)cl->n_label_keys);
    o_ke = take(4 * (size_t)cl->n_label_keys);
    o_vi = take(8 * (size_t)cl->n_label_values);
    o_vii = take((size_t)cl->n_label_values);
    o_cc = take(4 * (size_t)class_cap * N);
    o_tc = take(4 * (size_t)term_cap * N);
    o_log = take(8 * (N + 3));
    o_pu = take(8 * N);
    o_img = take(8 * (size_t)cl->n_images * N);
    o_vc = take(4 * (size_t)cl->n_vol_rows * N);
    o_va = take(4 * (size_t)cl->n_vol_keys * N);
    o_vl = take(4 * (size_t)cl->n_vol_keys * N);
    o_vrk = take(4 * (size_t)cl->n_vol_rows);
    o_vkp = take(4 * (size_t)cl->n_vol_keys);
    o_pvo = take(4 * (size_t)cl->n_pvs);
    o_cln = take(4 * (size_t)cl->n_wclaims);
    total = o;
  }
};

int fill_cluster(hipStream_t st, const kss_cluster* cl, int class_cap, int term_cap, char* b, const ClusterLayout& L,
                 DevCluster& dc, std::vector<double>& logtab) {
  const size_t N = (size_t)cl->n_nodes;
  auto cp = [&](size_t off, const void* src, size_t bytes) -> int {
    if (bytes && src) HIP_TRY(hipMemcpyAsync(b + off, src, bytes, hipMemcpyHostToDevice, st));
    return 0;
  };
  int rc = 0;
  rc |= cp(L.o_alloc, cl->alloc, 8 * KSS_NRES * N);
  rc |= cp(L.o_req, cl->requested, 8 * KSS_NRES * N);
  rc |= cp(L.o_nz, cl->nonzero, 8 * 2 * N);
  rc |= cp(L.o_allowed, cl->allowed_pods, 4 * N);
  rc |= cp(L.o_podc, cl->pod_count, 4 * N);
  rc |= cp(L.o_flags, cl->node_flags, 4 * N);
  rc |= cp(L.o_th, cl->taint_hard, 8 * N);
  rc |= cp(L.o_ts, cl->taint_soft, 8 * N);
  rc |= cp(L.o_to, cl->taint_order, (size_t)KSS_TAINT_ORDER * N);
  rc |= cp(L.o_lv, cl->label_value, 4 * (size_t)cl->n_label_keys * N);
  rc |= cp(L.o_kb, cl->key_base, 4 * (size_t)cl->n_label_keys);
  rc |= cp(L.o_kc, cl->key_card, 4 * (size_t)cl->n_label_keys);
  rc |= cp(L.o_kf, cl->key_flags, 4 * (size_t)cl->n_label_keys);
  rc |= cp(L.o_ke, cl->key_empty, 4 * (size_t)cl->n_label_keys);
  rc |= cp(L.o_vi, cl->value_int, 8 * (size_t)cl->n_label_values);
  rc |= cp(L.o_vii, cl->value_is_int, (size_t)cl->n_label_values);
  if (class_cap) HIP_TRY(dev_zero(b + L.o_cc, 4 * (size_t)class_cap * N, st));
  if (term_cap) HIP_TRY(dev_zero(b + L.o_tc, 4 * (size_t)term_cap * N, st));
  rc |= cp(L.o_cc, cl->class_count, 4 * (size_t)cl->n_classes * N);
  rc |= cp(L.o_tc, cl->term_count, 4 * (size_t)cl->n_terms * N);
  if (cl->port_used) rc |= cp(L.o_pu, cl->port_used, 8 * N);
  else HIP_TRY(dev_zero(b + L.o_pu, 8 * std::max<size_t>(N, 1), st));
  rc |= cp(L.o_img, cl->image_score, 8 * (size_t)cl->n_images * N);
  rc |= cp(L.o_vc, cl->vol_count, 4 * (size_t)cl->n_vol_rows * N);
  rc |= cp(L.o_va, cl->vol_attached, 4 * (size_t)cl->n_vol_keys * N);
  rc |= cp(L.o_vl, cl->vol_limit, 4 * (size_t)cl->n_vol_keys * N);
  rc |= cp(L.o_vrk, cl->vol_row_key, 4 * (size_t)cl->n_vol_rows);
  rc |= cp(L.o_vkp, cl->vol_key_plugin, 4 * (size_t)cl->n_vol_keys);
  rc |= cp(L.o_pvo, cl->pv_owner, 4 * (size_t)cl->n_pvs);
  rc |= cp(L.o_cln, cl->claim_node, 4 * (size_t)cl->n_wclaims);
  logtab.resize(N + 3);
  for (size_t k = 0; k < N + 3; k++) logtab[k] = kss_go_log((double)(k + 2));
  rc |= cp(L.o_log, logtab.data(), 8 * (N + 3));
  if (rc) return rc;
  dc.N = cl->n_nodes;
  dc.n_scalar = cl->n_scalar;
  dc.n_keys = cl->n_label_keys;
  dc.n_classes = cl->n_classes;
  dc.n_terms = cl->n_terms;
  dc.node_base = cl->node_base;
  dc.class_cap = class_cap;
  dc.term_cap = term_cap;
  dc.alloc = (const int64_t*)(b + L.o_alloc);
  dc.requested = (int64_t*)(b + L.o_req);
  dc.nonzero = (int64_t*)(b + L.o_nz);
  dc.allowed_pods = (const int32_t*)(b + L.o_allowed);
  dc.pod_count = (int32_t*)(b + L.o_podc);
  dc.node_flags = (const uint32_t*)(b + L.o_flags);
  dc.taint_hard = (const uint64_t*)(b + L.o_th);
  dc.taint_soft = (const uint64_t*)(b + L.o_ts);
  dc.taint_order = (const uint8_t*)(b + L.o_to);
  dc.label_value = (const int32_t*)(b + L.o_lv);
  dc.key_base = (const int32_t*)(b + L.o_kb);
  dc.key_card = (const int32_t*)(b + L.o_kc);
  dc.key_flags = (const uint32_t*)(b + L.o_kf);
  dc.key_empty = (const int32_t*)(b + L.o_ke);
  dc.value_int = (const int64_t*)(b + L.o_vi);
  dc.value_is_int = (const uint8_t*)(b + L.o_vii);
  dc.class_count = (int32_t*)(b + L.o_cc);
  dc.term_count = (int32_t*)(b + L.o_tc);
  dc.log_table = (const double*)(b + L.o_log);
  dc.port_used = (uint64_t*)(b + L.o_pu);
  dc.image_score = (const int64_t*)(b + L.o_img);
  dc.n_images = cl->n_images;
  dc.n_vol_rows = cl->n_vol_rows;
  dc.n_vol_keys = cl->n_vol_keys;
  dc.vol_count = (int32_t*)(b + L.o_vc);
  dc.vol_attached = (int32_t*)(b + L.o_va);
  dc.vol_limit = (const int32_t*)(b + L.o_vl);
  dc.vol_row_key = (const int32_t*)(b + L.o_vrk);
  dc.vol_key_plugin = (const int32_t*)(b + L.o_vkp);
  dc.n_pvs = cl->n_pvs;
  dc.n_wclaims = cl->n_wclaims;
  dc.pv_owner = (int32_t*)(b + L.o_pvo);
  dc.claim_node = (int32_t*)(b + L.o_cln);
  dc.pv_owner0 = dc.pv_owner;  // the pristine copies once kss_load_cluster has made them
  dc.claim_node0 = dc.claim_node;
  return 0;
}

int check_cluster(const kss_cluster* cl) {
  if (!cl || cl->n_nodes < 0) return fail(KSS_E_INVAL, "null cluster");
  if (cl->n_scalar < 0 || cl->n_scalar > KSS_MAX_SCALAR) return fail(KSS_E_INVAL, "n_scalar out of range");
  if (cl->n_taints < 0 || cl->n_taints > KSS_MAX_TAINTS) return fail(KSS_E_INVAL, "n_taints out of range");
  if (cl->n_nodes > 0 && (!cl->alloc || !cl->requested || !cl->nonzero || !cl->allowed_pods || !cl->pod_count ||
                          !cl->node_flags || !cl->taint_hard || !cl->taint_soft || !cl->taint_order))
    return fail(KSS_E_INVAL, "missing node column");
  for (int k = 0; k < cl->n_label_keys; k++) {
    if (cl->key_base[k] < 0 || cl->key_base[k] + cl->key_card[k] > cl->n_label_values)
      return fail(KSS_E_INVAL, "key value table out of range");
    if (cl->key_empty[k] < 0 || cl->key_empty[k] > cl->key_card[k]) return fail(KSS_E_INVAL, "key_empty out of range");
  }
  const size_t N = (size_t)cl->n_nodes;
  for (size_t i = 0; i < (size_t)cl->n_label_keys * N; i++) {
    const int k = (int)(i / (N ? N : 1));
    if (cl->label_value[i] < -1 || cl->label_value[i] >= cl->key_card[k]) return fail(KSS_E_INVAL, "label value id out of range");
  }
  for (size_t i = 0; i < N * KSS_TAINT_ORDER; i++)
    if (cl->taint_order[i] != 0xFF && cl->taint_order[i] >= cl->n_taints) return fail(KSS_E_INVAL, "taint id out of range");
  if (cl->n_ports < 0 || cl->n_ports > KSS_MAX_PORTS) return fail(KSS_E_INVAL, "n_ports out of range");
  if (cl->n_images < 0 || (cl->n_images > 0 && N > 0 && !cl->image_score)) return fail(KSS_E_INVAL, "missing image scores");
  if (cl->port_used && cl->n_ports < KSS_MAX_PORTS)
    for (size_t i = 0; i < N; i++)
      if (cl->port_used[i] >> cl->n_ports) return fail(KSS_E_INVAL, "port bit outside the port dictionary");
  for (size_t i = 0; i < (size_t)cl->n_images * N; i++)
    if (cl->image_score[i] < 0) return fail(KSS_E_INVAL, "negative image score");
  if (cl->n_vol_rows < 0 || cl->n_vol_keys < 0 || cl->n_vol_keys > KSS_MAX_VOL_KEYS)
    return fail(KSS_E_INVAL, "volume row / key count out of range");
  if (N > 0 && ((cl->n_vol_rows > 0 && (!cl->vol_count || !cl->vol_row_key)) ||
                (cl->n_vol_keys > 0 && (!cl->vol_attached || !cl->vol_limit || !cl->vol_key_plugin))))
    return fail(KSS_E_INVAL, "missing volume columns");
  for (int r = 0; r < cl->n_vol_rows; r++)
    if (cl->vol_row_key[r] < -1 || cl->vol_row_key[r] >= cl->n_vol_keys) return fail(KSS_E_INVAL, "volume row key out of range");
  for (int k = 0; k < cl->n_vol_keys; k++)
    if (cl->vol_key_plugin[k] < KSS_F_EBS_LIMITS || cl->vol_key_plugin[k] > KSS_F_AZURE_DISK_LIMITS)
      return fail(KSS_E_INVAL, "volume key plugin out of range");
  if (cl->n_pvs < 0 || cl->n_wclaims < 0 || (cl->n_pvs > 0 && !cl->pv_owner) || (cl->n_wclaims > 0 && !cl->claim_node))
    return fail(KSS_E_INVAL, "bad WaitForFirstConsumer columns");
  for (int v = 0; v < cl->n_pvs; v++)
    if (cl->pv_owner[v] < 0 || cl->pv_owner[v] > cl->n_wclaims) return fail(KSS_E_INVAL, "pv_owner out of range");
  for (int c = 0; c < cl->n_wclaims; c++)
    if (cl->claim_node[c] < -2 || cl->claim_node[c] >= cl->n_nodes) return fail(KSS_E_INVAL, "claim_node out of range");
  return 0;
}

// Profile limits of the device path.  percentageOfNodesToScore in [0, 100] (0: the adaptive
// default; below 100 the batch runs on k_schedule).  The selectHost key packs TotalScore into the upper 32 bits of a signed 64-bit
// key, so Σ weight·MaxNodeScore over the enabled score plugins must stay below 2^31; the
// reference accepts any positive int32 weight whose sum fits int64 (framework.go
// MaxTotalScore), so larger profiles are refused here rather than mis-ranked.
int check_profile(const kss_profile* prof) {
  if (prof->pct_nodes_to_score < 0 || prof->pct_nodes_to_score > 100)  // ValidateKubeSchedulerConfiguration
    return fail(KSS_E_INVAL, "percentageOfNodesToScore must be between 0 and 100");
  int64_t sum = 0;
  for (int s = 0; s < KSS_NSCORE; s++) {
    if (!((prof->score_enabled >> s) & 1u)) continue;
    if (prof->weight[s] < 0) return fail(KSS_E_INVAL, "negative score plugin weight");
    sum += (int64_t)prof->weight[s] * 100;
  }
  if (sum >= (1ll << 31)) return fail(KSS_E_UNSUPPORTED, "sum of score weights x 100 must be below 2^31 on the device path");
  if (prof->fit_n < 0 || prof->fit_n > 4 || prof->ba_n < 0 || prof->ba_n > 4)
    return fail(KSS_E_INVAL, "scoring resource count out of range");
  for (int i = 0; i < prof->fit_n; i++)
    if (prof->fit_res[i] < 0 || prof->fit_res[i] >= KSS_NRES || prof->fit_weight[i] < 0)
      return fail(KSS_E_INVAL, "NodeResourcesFit scoring resource out of range");
  for (int i = 0; i < prof->ba_n; i++)
    if (prof->ba_res[i] < 0 || prof->ba_res[i] >= KSS_NRES)
      return fail(KSS_E_INVAL, "BalancedAllocation resource out of range");
  return 0;
}

}  // namespace

static int svc_stop(kss_ctx* ctx);
static void svc_free(kss_ctx* ctx);

// Entry points that use the device state themselves stop the service first.
#define KSS_SVC_QUIESCE(ctx)                    \
  do {                                          \
    if ((ctx) && (ctx)->svc.running) {          \
      if (int rc_ = svc_stop(ctx)) return rc_;  \
    }                                           \
  } while (0)

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

int kss_abi_version(void) { return KSS_ABI_VERSION; }
const char* kss_last_error(void) { return g_err.c_str(); }

int kss_set_option(const char* name, int64_t value) {
  if (!name) return fail(KSS_E_INVAL, "null option name");
  std::call_once(g_opt_once, opt_defaults);
  for (int i = 0; i < O_N; i++)
    if (!strcmp(name, kOptDefs[i].name)) {
      g_opt[i].store((long long)value, std::memory_order_relaxed);
      return 0;
    }
  return fail(KSS_E_NOTFOUND, std::string("unknown option ") + name);
}

int kss_get_option(const char* name, int64_t* value) {
  if (!name || !value) return fail(KSS_E_INVAL, "bad arguments");
  for (int i = 0; i < O_N; i++)
    if (!strcmp(name, kOptDefs[i].name)) {
      *value = opt((KssOpt)i);
      return 0;
    }
  return fail(KSS_E_NOTFOUND, std::string("unknown option ") + name);
}

int kss_reset_options(void) {
  std::call_once(g_opt_once, opt_defaults);
  for (int i = 0; i < O_N; i++) g_opt[i].store(kOptDefs[i].dflt, std::memory_order_relaxed);
  std::lock_guard<std::mutex> lk(g_stamps_mu);
  g_stamps_path.clear();
  return 0;
}

int kss_set_stamps_file(const char* path) {
  std::call_once(g_opt_once, opt_defaults);
  std::lock_guard<std::mutex> lk(g_stamps_mu);
  g_stamps_path = path ? path : "";
  return 0;
}

#if KSS_SPREAD_TRACE
// Trace builds only (not in kss.h): the last k_spread run's trace words [n][W][G_TW], its
// count list (1 + 4 G_TLIST words) and resident rows.  Returns the words copied.
int kss_trace_spread(kss_ctx* ctx, int32_t* words, int64_t n_words, int32_t* list, int64_t n_list, int32_t* rows,
                     int32_t n_rows) {
  if (!ctx || n_words < 0 || n_list < 0) return fail(KSS_E_INVAL, "bad arguments");
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  const size_t n = std::min((size_t)n_words, ctx->trace_words), nl = std::min((size_t)n_list, (size_t)(4 + 4 * G_TLIST));
  if (words && n) HIP_TRY(hipMemcpy(words, ctx->trace_buf.p, 4 * n, hipMemcpyDeviceToHost));
  if (list && nl && ctx->trace_list_buf.p) HIP_TRY(hipMemcpy(list, ctx->trace_list_buf.p, 4 * nl, hipMemcpyDeviceToHost));
  for (int i = 0; rows && i < n_rows && i < (int)ctx->gneed.res_rows.size(); i++) rows[i] = ctx->gneed.res_rows[i];
  return (int)std::min(n, (size_t)INT32_MAX);
}
#endif

int kss_abi_sizes(int32_t* out, int32_t n) {
  const int32_t s[] = {(int32_t)sizeof(kss_cluster), (int32_t)sizeof(kss_req),     (int32_t)sizeof(kss_term),
                       (int32_t)sizeof(kss_spread),  (int32_t)sizeof(kss_ipa),     (int32_t)sizeof(kss_pod),
                       (int32_t)sizeof(kss_podset),  (int32_t)sizeof(kss_profile), (int32_t)sizeof(kss_pod_result),
                       (int32_t)sizeof(kss_config),  (int32_t)sizeof(kss_names),   (int32_t)sizeof(kss_synth),
                       (int32_t)sizeof(kss_boundset), (int32_t)sizeof(kss_preempt_result), (int32_t)sizeof(kss_vol),
                       (int32_t)sizeof(kss_pod_view), (int32_t)sizeof(kss_pod_cview)};
  const int32_t k = (int32_t)(sizeof(s) / sizeof(s[0]));
  for (int i = 0; i < n && i < k; i++) out[i] = s[i];
  return k;
}

kss_ctx* kss_create(const kss_config* cfg, const kss_profile* prof) {
  if (!cfg || !prof) {
    fail(KSS_E_INVAL, "null config/profile");
    return nullptr;
  }
  if (check_profile(prof)) return nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    fail(KSS_E_DEVICE, "no HIP device visible");
    return nullptr;
  }
  if (cfg->device < 0 || cfg->device >= ndev) {
    fail(KSS_E_INVAL, "device ordinal out of range");
    return nullptr;
  }
  kss_ctx* ctx = new kss_ctx();
  ctx->cfg = *cfg;
  ctx->prof = *prof;
  hipDeviceProp_t dp{};
  if (hipGetDeviceProperties(&dp, cfg->device) == hipSuccess) ctx->n_cu = dp.multiProcessorCount;
  if (ctx->n_cu <= 0) ctx->n_cu = 1;
  ctx->force_w = (int)std::max(0ll, opt(O_SHARDS));
  ctx->xcd_mode = opt(O_XCD) != 0;
  ctx->xcd_w = (int)std::max(0ll, std::min((long long)(64 * SX_CHUNKS), opt(O_XCD_SHARDS)));
  {
    std::lock_guard<std::mutex> lk(g_stamps_mu);
    ctx->stamps_path = g_stamps_path;
  }
  ctx->stamps_file = ctx->stamps_path.empty() ? nullptr : ctx->stamps_path.c_str();
  ctx->no_simple = opt(O_NO_SIMPLE) != 0;
  ctx->no_spread = opt(O_NO_SPREAD) != 0;
  ctx->axis_max_blocks = (int)std::max(0ll, opt(O_AXIS_BLOCKS));
  ctx->axis_no_fold = opt(O_AXIS_NO_FOLD) != 0;
  ctx->nodes_per_shard = (int)std::max(1ll, opt(O_NODES_PER_SHARD));
  if (opt(O_THREADS) > 0) ctx->pref_threads = (int)std::min<long long>(KSS_MAX_THREADS, std::max(64ll, opt(O_THREADS)));
  if (hipSetDevice(cfg->device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess) {
    fail(KSS_E_DEVICE, "stream/event creation failed");
    delete ctx;
    return nullptr;
  }
  return ctx;
}

static void split_release(kss_ctx* ctx);

void kss_destroy(kss_ctx* ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->cfg.device);
  svc_stop(ctx);
  svc_free(ctx);
  if (ctx->stream) hipStreamSynchronize(ctx->stream);
  ctx->cluster_buf.release();
  ctx->pristine_buf.release();
  ctx->pod_buf.release();
  ctx->tmp_pod_buf.release();
  ctx->wffc_pod_buf.release();
  ctx->slot_buf.release();
  ctx->meta_buf.release();
  ctx->chosen_buf.release();
  ctx->job_buf.release();
  ctx->spod_buf.release();
  ctx->stat_buf.release();
  ctx->bound_buf.release();
  ctx->pre_buf.release();
  ctx->stamp_buf.release();
  ctx->gran_buf.release();
  ctx->err_buf.release();
  ctx->axis_cv.release();
  ctx->gpod_buf.release();
  ctx->res_buf.release();
  ctx->delta_buf.release();
  ctx->ck_buf.release();
  split_release(ctx);
  if (ctx->pinned) hipHostFree(ctx->pinned);
  if (ctx->rb) hipHostFree(ctx->rb);
  if (ctx->up) hipHostFree(ctx->up);
  for (hipEvent_t e : ctx->loop_ev) hipEventDestroy(e);
  if (ctx->ev0) hipEventDestroy(ctx->ev0);
  if (ctx->ev1) hipEventDestroy(ctx->ev1);
  if (ctx->stream) hipStreamDestroy(ctx->stream);
  delete ctx;
}

int kss_load_cluster(kss_ctx* ctx, const kss_cluster* cl) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx) return fail(KSS_E_INVAL, "null ctx");
  int rc = check_cluster(cl);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  const int class_cap = std::max(cl->n_classes, ctx->cfg.class_capacity);
  const int term_cap = std::max(cl->n_terms, ctx->cfg.term_capacity);
  ClusterLayout L(cl, class_cap, term_cap);
  rc = ctx->cluster_buf.ensure(L.total);
  if (rc) return rc;
  std::vector<double> logtab;
  rc = fill_cluster(ctx->stream, cl, class_cap, term_cap, (char*)ctx->cluster_buf.p, L, ctx->dc, logtab);
  if (rc) return rc;
  // pristine copy of the mutable columns
  const size_t N = (size_t)cl->n_nodes;
  const size_t mb[KSS_NMUT] = {8 * KSS_NRES * N,
                               8 * 2 * N,
                               4 * N,
                               4 * (size_t)class_cap * N,
                               4 * (size_t)term_cap * N,
                               8 * N,
                               4 * (size_t)cl->n_vol_rows * N,
                               4 * (size_t)cl->n_vol_keys * N,
                               4 * (size_t)cl->n_pvs,
                               4 * (size_t)cl->n_wclaims};
  size_t tot = 0;
  for (int i = 0; i < KSS_NMUT; i++) {
    ctx->mut_bytes[i] = mb[i];
    ctx->pristine_off[i] = tot;
    tot = align_up(tot + mb[i], 256);
  }
  rc = ctx->pristine_buf.ensure(tot);
  if (rc) return rc;
  void* src[KSS_NMUT] = {ctx->dc.requested,  ctx->dc.nonzero,   ctx->dc.pod_count,    ctx->dc.class_count,
                         ctx->dc.term_count, ctx->dc.port_used, ctx->dc.vol_count,    ctx->dc.vol_attached,
                         ctx->dc.pv_owner,   ctx->dc.claim_node};
  ctx->dc.pv_owner0 = (const int32_t*)((char*)ctx->pristine_buf.p + ctx->pristine_off[8]);
  ctx->dc.claim_node0 = (const int32_t*)((char*)ctx->pristine_buf.p + ctx->pristine_off[9]);
  {  // the copy by the reset kernel (agent-scope loads and stores), not the runtime's copy path
    ResetArgs a{};
    size_t most = 0;
    for (int i = 0; i < KSS_NMUT; i++) {
      a.dst[i] = (uint32_t*)((char*)ctx->pristine_buf.p + ctx->pristine_off[i]);
      a.src[i] = (const uint32_t*)src[i];
      a.n4[i] = src[i] ? mb[i] / 4 : 0;
      most = std::max(most, a.n4[i]);
    }
    if (most) {
      hipLaunchKernelGGL(k_reset_state, dim3((unsigned)std::min<size_t>(1024, (most + 255) / 256)), dim3(256), 0,
                         ctx->stream, a);
      HIP_TRY(hipGetLastError());
    }
  }
  // nextStartNodeIndex starts at 0 with a new snapshot (a new scheduler)
  if ((rc = ctx->cursor_buf.ensure(16))) return rc;
  HIP_TRY(dev_zero(ctx->cursor_buf.p, 16, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  ctx->host = *cl;
  {
    bool small = true;
    for (size_t i = 0; i < 3 * N && small; i++) small = cl->alloc[i] >= 0 && cl->alloc[i] < (1ll << 46);
    for (int i = 0; i < ctx->prof.fit_n && small; i++) small = ctx->prof.fit_weight[i] >= 0 && ctx->prof.fit_weight[i] < (1ll << 20);
    ctx->small_values = small;
    ctx->f64_cluster = F64Bounds{};
    f64_bounds_cluster(cl, ctx->f64_cluster);
  }
  ctx->key_card_h.assign(cl->key_card, cl->key_card + cl->n_label_keys);
  ctx->key_flags_h.assign(cl->key_flags, cl->key_flags + cl->n_label_keys);
  ctx->key_empty_h.assign(cl->key_empty, cl->key_empty + cl->n_label_keys);
  {
    double sc = 0, st = 0;
    if (cl->class_count)
      for (size_t i = 0; i < (size_t)cl->n_classes * N; i++) sc += std::abs((double)cl->class_count[i]);
    if (cl->term_count)
      for (size_t i = 0; i < (size_t)cl->n_terms * N; i++) st += std::abs((double)cl->term_count[i]);
    ctx->count_bound0 = ctx->count_bound = std::max(sc, st);
    double cm = 0;
    if (cl->class_count)
      for (size_t i = 0; i < (size_t)cl->n_classes * N; i++) cm = std::max(cm, std::abs((double)cl->class_count[i]));
    if (cl->term_count)
      for (size_t i = 0; i < (size_t)cl->n_terms * N; i++) cm = std::max(cm, std::abs((double)cl->term_count[i]));
    ctx->cell_bound0 = ctx->cell_bound = cm;
  }
  ctx->loaded = true;
  ctx->bound0.clear();
  ctx->bound0_node.clear();
  ctx->bound_log.clear();
  ctx->bound_dirty = true;
  ctx->nom.clear();
  ctx->nom_dirty = true;
  ctx->state_unknown = false;
  ctx->recorded = 0;
  ctx->meta_n = 0;
  ctx->axis_meta_dirty = false;
  ctx->staged_n = -1;
  return 0;
}

static bool same_profile(const kss_profile& a, const kss_profile& b);

int kss_load_cluster_rows(kss_ctx* ctx, const kss_cluster* cl, int32_t lo, int32_t hi) {
  if (!ctx) return fail(KSS_E_INVAL, "null ctx");
  int rc = check_cluster(cl);
  if (rc) return rc;
  if (lo < 0 || hi < lo || hi > cl->n_nodes) return fail(KSS_E_INVAL, "row range out of range");
  const size_t N = (size_t)cl->n_nodes, M = (size_t)(hi - lo);
  // column-blocked [attr][N] matrices: take columns [lo, hi) of every attribute row
  auto rows64 = [&](const int64_t* src, int nrow, std::vector<int64_t>& dst) {
    dst.resize(std::max<size_t>(nrow * M, 1));
    for (int r = 0; r < nrow; r++) std::copy(src + r * N + lo, src + r * N + hi, dst.begin() + r * M);
  };
  auto rows32 = [&](const int32_t* src, int nrow, std::vector<int32_t>& dst) {
    dst.resize(std::max<size_t>(nrow * M, 1));
    if (src)
      for (int r = 0; r < nrow; r++) std::copy(src + r * N + lo, src + r * N + hi, dst.begin() + r * M);
  };
  std::vector<int64_t> alloc, req, nz;
  std::vector<int32_t> allowed, podc, lv, cc, tc;
  rows64(cl->alloc, KSS_NRES, alloc);
  rows64(cl->requested, KSS_NRES, req);
  rows64(cl->nonzero, 2, nz);
  rows32(cl->allowed_pods, 1, allowed);
  rows32(cl->pod_count, 1, podc);
  rows32(cl->label_value, cl->n_label_keys, lv);
  rows32(cl->class_count, cl->n_classes, cc);
  rows32(cl->term_count, cl->n_terms, tc);
  std::vector<uint32_t> flags(cl->node_flags + lo, cl->node_flags + hi);
  std::vector<uint64_t> th(cl->taint_hard + lo, cl->taint_hard + hi), ts(cl->taint_soft + lo, cl->taint_soft + hi);
  std::vector<uint8_t> to(cl->taint_order + (size_t)lo * KSS_TAINT_ORDER, cl->taint_order + (size_t)hi * KSS_TAINT_ORDER);
  std::vector<uint64_t> pu(std::max<size_t>(M, 1), 0);
  if (cl->port_used) std::copy(cl->port_used + lo, cl->port_used + hi, pu.begin());
  std::vector<int64_t> img;
  if (cl->n_images) rows64(cl->image_score, cl->n_images, img);
  std::vector<int32_t> vc, va, vl;
  rows32(cl->vol_count, cl->n_vol_rows, vc);
  rows32(cl->vol_attached, cl->n_vol_keys, va);
  rows32(cl->vol_limit, cl->n_vol_keys, vl);
  kss_cluster s = *cl;
  s.n_nodes = (int32_t)M;
  s.node_base = cl->node_base + lo;
  s.alloc = alloc.data();
  s.requested = req.data();
  s.nonzero = nz.data();
  s.allowed_pods = allowed.data();
  s.pod_count = podc.data();
  s.node_flags = flags.data();
  s.taint_hard = th.data();
  s.taint_soft = ts.data();
  s.taint_order = to.data();
  s.label_value = lv.data();
  s.class_count = cl->class_count ? cc.data() : nullptr;
  s.term_count = cl->term_count ? tc.data() : nullptr;
  s.port_used = pu.data();
  s.image_score = cl->n_images ? img.data() : nullptr;
  s.vol_count = cl->n_vol_rows ? vc.data() : nullptr;
  s.vol_attached = cl->n_vol_keys ? va.data() : nullptr;
  s.vol_limit = cl->n_vol_keys ? vl.data() : nullptr;
  return kss_load_cluster(ctx, &s);  // synchronous: the temporaries outlive the upload
}

static hipStream_t axis_stream(kss_ctx* ctx, void* stream) { return stream ? (hipStream_t)stream : ctx->stream; }

static int axis_check(kss_ctx* ctx, int32_t pod_index) {
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  if (ctx->prof.pct_nodes_to_score < 100)
    return fail(KSS_E_UNSUPPORTED, "node-axis path: percentageOfNodesToScore below 100 runs on k_schedule");
  if (pod_index < 0 || pod_index >= ctx->staged_n) return fail(KSS_E_INVAL, "pod index outside the staged pods");
  if (ctx->staged_need.general)
    return fail(KSS_E_UNSUPPORTED, "node-axis path: spread / inter-pod programs need the replicated domain histograms");
  if (ctx->staged_need.ports_images)
    return fail(KSS_E_UNSUPPORTED, "node-axis path: host ports / image locality / volumes are not folded into the axis key");
  return ctx->axis_cv.ensure(sizeof(int32_t) * 5 * (size_t)std::max(ctx->dc.N, 1));
}

static dim3 axis_grid(kss_ctx* ctx) {
  const int blocks = (ctx->dc.N + AXIS_THREADS - 1) / AXIS_THREADS;
  return dim3((unsigned)std::max(1, std::min(blocks, ctx->axis_max_blocks > 0 ? ctx->axis_max_blocks : 4 * ctx->n_cu)));
}

int kss_axis_eval(kss_ctx* ctx, int32_t pod_index, int64_t* stats_dev, const int64_t* prev_key_dev,
                  const int64_t* prev_gathered_dev, int32_t world, int64_t* key_zero_dev, int32_t* chosen_dev,
                  void* stream) {
  KSS_SVC_QUIESCE(ctx);
  int rc = axis_check(ctx, pod_index);
  if (rc) return rc;
  if (!ctx->nom.empty()) return fail(KSS_E_UNSUPPORTED, "the node axis does not read the nominator");
  if (!stats_dev || !key_zero_dev || world < 1) return fail(KSS_E_INVAL, "bad eval arguments");
  if (prev_key_dev && (pod_index < 1 || !prev_gathered_dev)) return fail(KSS_E_INVAL, "pending commit without a previous pod");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  rc = ctx->meta_buf.ensure(sizeof(PodMeta) * (size_t)std::max(ctx->staged_n, 1));
  if (rc) return rc;
  auto fn = same_profile(ctx->prof, default_profile_c()) ? k_axis_eval<true> : k_axis_eval<false>;
  hipLaunchKernelGGL(fn, axis_grid(ctx), dim3(AXIS_THREADS), 0, axis_stream(ctx, stream), ctx->dc, ctx->dp, ctx->prof,
                     pod_index, (int32_t*)ctx->axis_cv.p, (long long*)stats_dev, (const long long*)prev_key_dev,
                     (const long long*)prev_gathered_dev, world, (long long*)key_zero_dev, chosen_dev,
                     (PodMeta*)ctx->meta_buf.p, ctx->axis_no_fold);
  HIP_TRY(hipGetLastError());
  if (prev_key_dev) {
    ctx->meta_n = std::max(ctx->meta_n, (int)pod_index);
    ctx->axis_meta_dirty = true;
  }
  return 0;
}

int kss_axis_select(kss_ctx* ctx, const int64_t* gathered_dev, int32_t world, int64_t* key_dev, int64_t* stats_zero_dev,
                    void* stream) {
  KSS_SVC_QUIESCE(ctx);
  int rc = axis_check(ctx, 0);
  if (rc) return rc;
  if (!gathered_dev || !key_dev || !stats_zero_dev || world < 1) return fail(KSS_E_INVAL, "bad select arguments");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  hipLaunchKernelGGL(k_axis_select, axis_grid(ctx), dim3(AXIS_THREADS), 0, axis_stream(ctx, stream), ctx->dc, ctx->prof,
                     (const int32_t*)ctx->axis_cv.p, (const long long*)gathered_dev, world, (long long*)key_dev,
                     (long long*)stats_zero_dev);
  HIP_TRY(hipGetLastError());
  return 0;
}

int kss_axis_commit(kss_ctx* ctx, int32_t pod_index, const int64_t* key_dev, const int64_t* gathered_dev, int32_t world,
                    int32_t* chosen_dev, void* stream) {
  KSS_SVC_QUIESCE(ctx);
  int rc = axis_check(ctx, pod_index);
  if (rc) return rc;
  if (!key_dev || !gathered_dev || world < 1) return fail(KSS_E_INVAL, "bad commit arguments");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  rc = ctx->meta_buf.ensure(sizeof(PodMeta) * (size_t)std::max(ctx->staged_n, 1));
  if (rc) return rc;
  hipLaunchKernelGGL(k_axis_commit, dim3(1), dim3(64), 0, axis_stream(ctx, stream), ctx->dc, ctx->dp, pod_index,
                     (const long long*)key_dev, (const long long*)gathered_dev, world, chosen_dev,
                     (PodMeta*)ctx->meta_buf.p);
  HIP_TRY(hipGetLastError());
  ctx->meta_n = std::max(ctx->meta_n, pod_index + 1);
  ctx->axis_meta_dirty = true;
  return 0;
}

int kss_reset_node_state(kss_ctx* ctx) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  void* dst[KSS_NMUT] = {ctx->dc.requested,  ctx->dc.nonzero,   ctx->dc.pod_count,    ctx->dc.class_count,
                         ctx->dc.term_count, ctx->dc.port_used, ctx->dc.vol_count,    ctx->dc.vol_attached,
                         ctx->dc.pv_owner,   ctx->dc.claim_node};
  ctx->count_bound = ctx->count_bound0;
  ctx->cell_bound = ctx->cell_bound0;
  ctx->bound_log.clear();
  ctx->bound_dirty = true;
  ctx->state_unknown = false;
  ResetArgs a{};
  size_t most = 0;
  for (int i = 0; i < KSS_NMUT; i++) {
    a.dst[i] = (uint32_t*)dst[i];
    a.src[i] = (const uint32_t*)((char*)ctx->pristine_buf.p + ctx->pristine_off[i]);
    a.n4[i] = ctx->mut_bytes[i] / 4;
    most = std::max(most, a.n4[i]);
  }
  if (most) {
    hipLaunchKernelGGL(k_reset_state, dim3((unsigned)std::min<size_t>(1024, (most + 255) / 256)), dim3(256), 0,
                       ctx->stream, a);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(dev_zero(ctx->cursor_buf.p, 16, ctx->stream));  // the simulator's reset starts a new scheduler
  ctx->nom.clear();  // ... with an empty scheduling queue (no nominator entries)
  ctx->nom_dirty = true;
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int kss_next_start_node_index(kss_ctx* ctx, int32_t* out) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded || !out) return fail(KSS_E_INVAL, "bad arguments");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  HIP_TRY(hipMemcpyAsync(out, ctx->cursor_buf.p, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

// The nominator entry of ps.pods[pod_index] on local row `local` (AddNominatedPod's NominatedPod)
static int nom_entry(const kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, int32_t local, DevNom& e) {
  const kss_pod& p = ps->pods[pod_index];
  if (p.vol_len > 0) return fail(KSS_E_UNSUPPORTED, "a nominated pod with volumes (the volume filters do not add nominees)");
  if (p.cls < 0 || p.cls >= ctx->host.n_classes) return fail(KSS_E_INVAL, "pod class out of range");
  if (p.own_terms_len < 0 || p.own_terms_off < 0 || p.own_terms_off + p.own_terms_len > ps->n_ints)
    return fail(KSS_E_INVAL, "own terms out of range");
  if (p.own_terms_len > 8) return fail(KSS_E_UNSUPPORTED, "a nominated pod with more than 8 own term rows");
  if (ctx->host.n_ports < KSS_MAX_PORTS && (p.port_add >> ctx->host.n_ports))
    return fail(KSS_E_INVAL, "pod port bit outside the port dictionary");
  e = DevNom{};
  e.node = local;
  e.prio = p.priority;
  e.pod = pod_identity(p, pod_index);
  e.cls = p.cls;
  e.n_terms = p.own_terms_len;
  for (int t = 0; t < p.own_terms_len; t++) {
    e.terms[t] = ps->ints[p.own_terms_off + t];
    if (e.terms[t] < 0 || e.terms[t] >= ctx->host.n_terms) return fail(KSS_E_INVAL, "own term id out of range");
  }
  e.ports = p.port_add;
  for (int r = 0; r < KSS_NRES; r++) e.req[r] = p.commit_req[r];
  return 0;
}

// An index-keyed identity (-1 - index: a pod without uid) names a pod of one pod list.  Every
// entry point that takes a podset first drops the index-keyed entries that belong to another
// podset, or whose index now holds a different pod (restaged or edited list), so no pod
// inherits another's nomination: PreferNominatedNode and RunFilterPluginsWithNominatedPods'
// self-exclusion follow the pod, not the slot.  uid-keyed entries are left alone.  Call with
// ctx->mu held.
static void nom_check_podset(kss_ctx* ctx, const kss_podset* ps) {
  if (ctx->nom.empty()) return;
  const size_t before = ctx->nom.size();
  ctx->nom.erase(std::remove_if(ctx->nom.begin(), ctx->nom.end(),
                                [&](const DevNom& e) {
                                  if (e.pod >= 0) return false;
                                  auto it = ctx->nom_src.find(e.pod);
                                  if (it == ctx->nom_src.end() || it->second != ps) return true;
                                  const int idx = -1 - e.pod;
                                  if (idx >= ps->n_pods || ps->pods[idx].uid > 0) return true;
                                  DevNom now;
                                  if (nom_entry(ctx, ps, idx, e.node, now)) return true;
                                  return std::memcmp(&now, &e, sizeof(DevNom)) != 0;
                                }),
                 ctx->nom.end());
  if (ctx->nom.size() != before) ctx->nom_dirty = true;
}

int kss_nominate(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, int32_t node) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded || !ps) return fail(KSS_E_INVAL, "bad arguments");
  if (pod_index < 0 || pod_index >= ps->n_pods) return fail(KSS_E_INVAL, "pod index out of range");
  const int local = node - ctx->dc.node_base;
  if (local < 0 || local >= ctx->dc.N) return fail(KSS_E_INVAL, "node out of range");
  if (ctx->split_n > 1) return fail(KSS_E_UNSUPPORTED, "split grids do not read the nominator");
  DevNom e;
  if (int rc = nom_entry(ctx, ps, pod_index, local, e)) return rc;
  std::lock_guard<std::mutex> lk(ctx->mu);
  nom_check_podset(ctx, ps);
  // AddNominatedPod: an earlier nomination of the pod is replaced (it moves to the end)
  ctx->nom.erase(std::remove_if(ctx->nom.begin(), ctx->nom.end(), [&](const DevNom& x) { return x.pod == e.pod; }),
                 ctx->nom.end());
  if ((int)ctx->nom.size() >= KSS_NOM_MAX) return fail(KSS_E_UNSUPPORTED, "more than 64 nominated pods");
  ctx->nom.push_back(e);
  if (e.pod < 0) ctx->nom_src[e.pod] = ps;
  ctx->nom_dirty = true;
  return 0;
}

int kss_clear_nomination(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ps) return fail(KSS_E_INVAL, "bad arguments");
  if (pod_index < 0 || pod_index >= ps->n_pods) return fail(KSS_E_INVAL, "pod index out of range");
  const int32_t id = pod_identity(ps->pods[pod_index], pod_index);
  std::lock_guard<std::mutex> lk(ctx->mu);
  nom_check_podset(ctx, ps);
  const size_t before = ctx->nom.size();
  ctx->nom.erase(std::remove_if(ctx->nom.begin(), ctx->nom.end(), [&](const DevNom& x) { return x.pod == id; }),
                 ctx->nom.end());
  if (ctx->nom.size() != before) ctx->nom_dirty = true;
  return 0;
}

int kss_nominations(kss_ctx* ctx, int32_t* pods, int32_t* nodes, int32_t cap, int32_t* n) {
  if (!ctx || !n || cap < 0 || (cap > 0 && (!pods || !nodes))) return fail(KSS_E_INVAL, "bad arguments");  // pods: identities
  std::lock_guard<std::mutex> lk(ctx->mu);
  *n = (int32_t)ctx->nom.size();
  for (int i = 0; i < *n && i < cap; i++) {
    pods[i] = ctx->nom[i].pod;
    nodes[i] = ctx->dc.node_base + ctx->nom[i].node;
  }
  return 0;
}

int kss_set_next_start_node_index(kss_ctx* ctx, int32_t v) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded || v < 0) return fail(KSS_E_INVAL, "bad arguments");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  HIP_TRY(hipMemcpyAsync(ctx->cursor_buf.p, &v, sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int kss_apply_node_delta(kss_ctx* ctx, const int32_t* idx, int32_t n, const int64_t* requested, const int64_t* nonzero,
                         const int32_t* pod_count) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  if (n < 0 || (n > 0 && (!idx || !requested || !nonzero || !pod_count))) return fail(KSS_E_INVAL, "bad arguments");
  if (n == 0) return 0;
  for (int i = 0; i < n; i++)
    if (idx[i] < 0 || idx[i] >= ctx->dc.N) return fail(KSS_E_INVAL, "delta row out of range");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  // one packed image: rows | requested | nonzero | pod counts
  const size_t o_req = align_up(4 * (size_t)n, 16), o_nz = o_req + 8 * KSS_NRES * (size_t)n,
               o_pc = o_nz + 16 * (size_t)n, total = o_pc + 4 * (size_t)n;
  ctx->stage_host.resize(total);
  char* h = ctx->stage_host.data();
  std::memcpy(h, idx, 4 * (size_t)n);
  std::memcpy(h + o_req, requested, 8 * KSS_NRES * (size_t)n);
  std::memcpy(h + o_nz, nonzero, 16 * (size_t)n);
  std::memcpy(h + o_pc, pod_count, 4 * (size_t)n);
  int rc = ctx->delta_buf.ensure(total);
  if (rc) return rc;
  char* d = (char*)ctx->delta_buf.p;
  HIP_TRY(hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_node_delta, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, ctx->dc,
                     (const int32_t*)d, (const int64_t*)(d + o_req), (const int64_t*)(d + o_nz),
                     (const int32_t*)(d + o_pc), n);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  // k_simple's exactness bounds track the largest requested / non-zero values
  for (int i = 0; i < n; i++) {
    for (int r = 0; r < 3; r++) {
      const int64_t v = requested[(size_t)i * KSS_NRES + r];
      ctx->f64_cluster.neg |= v < 0;
      ctx->f64_cluster.max_req0 = std::max(ctx->f64_cluster.max_req0, (double)v);
    }
    for (int r = 0; r < 2; r++) {
      const int64_t v = nonzero[(size_t)i * 2 + r];
      ctx->f64_cluster.neg |= v < 0;
      ctx->f64_cluster.max_nz0 = std::max(ctx->f64_cluster.max_nz0, (double)v);
    }
  }
  return 0;
}

int kss_apply_count_delta(kss_ctx* ctx, const int32_t* node, const int32_t* row, const int32_t* value, int32_t n,
                          int32_t mode) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  if (n < 0 || (n > 0 && (!node || !row || !value)) || (mode != 0 && mode != 1)) return fail(KSS_E_INVAL, "bad arguments");
  if (n == 0) return 0;
  const int nc = ctx->host.n_classes, nt = ctx->host.n_terms;
  double add = 0, top = 0;
  for (int i = 0; i < n; i++) {
    if (node[i] < 0 || node[i] >= ctx->dc.N) return fail(KSS_E_INVAL, "count delta node out of range");
    if (row[i] < 0 || row[i] >= nc + nt) return fail(KSS_E_INVAL, "count delta row out of range");
    if (mode == 1 && value[i] < 0) return fail(KSS_E_INVAL, "negative count");
    add += std::max(0, value[i]);
    top = std::max(top, (double)value[i]);
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  const size_t b = 4 * (size_t)n, total = 3 * align_up(b, 16);
  ctx->stage_host.resize(total);
  char* h = ctx->stage_host.data();
  std::memcpy(h, node, b);
  std::memcpy(h + align_up(b, 16), row, b);
  std::memcpy(h + 2 * align_up(b, 16), value, b);
  int rc = ctx->delta_buf.ensure(total);
  if (rc) return rc;
  char* d = (char*)ctx->delta_buf.p;
  HIP_TRY(hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_count_delta, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, ctx->dc,
                     (const int32_t*)d, (const int32_t*)(d + align_up(b, 16)),
                     (const int32_t*)(d + 2 * align_up(b, 16)), n, mode);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  // the 32-bit / 16-bit bounds of k_spread (spread_bounds_ok)
  ctx->count_bound += add;
  ctx->cell_bound = mode ? std::max(ctx->cell_bound, top) : ctx->cell_bound + add;
  return 0;
}

int kss_read_node_state(kss_ctx* ctx, int64_t* requested, int64_t* nonzero, int32_t* pod_count, int32_t* class_count,
                        int32_t* term_count) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  const size_t N = (size_t)ctx->dc.N;
  if (requested) HIP_TRY(hipMemcpyAsync(requested, ctx->dc.requested, 8 * KSS_NRES * N, hipMemcpyDeviceToHost, ctx->stream));
  if (nonzero) HIP_TRY(hipMemcpyAsync(nonzero, ctx->dc.nonzero, 8 * 2 * N, hipMemcpyDeviceToHost, ctx->stream));
  if (pod_count) HIP_TRY(hipMemcpyAsync(pod_count, ctx->dc.pod_count, 4 * N, hipMemcpyDeviceToHost, ctx->stream));
  if (class_count && ctx->host.n_classes)
    HIP_TRY(hipMemcpyAsync(class_count, ctx->dc.class_count, 4 * (size_t)ctx->host.n_classes * N, hipMemcpyDeviceToHost, ctx->stream));
  if (term_count && ctx->host.n_terms)
    HIP_TRY(hipMemcpyAsync(term_count, ctx->dc.term_count, 4 * (size_t)ctx->host.n_terms * N, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

static_assert(sizeof(hipIpcMemHandle_t) == KSS_IPC_HANDLE_BYTES, "IPC handle size");
static_assert(KSS_MAX_PARTS == KSS_SPLIT_MAX_PARTS, "kss.h split limit");

static void split_release(kss_ctx* ctx) {
  for (void* p : ctx->split_opened) hipIpcCloseMemHandle(p);
  ctx->split_opened.clear();
  if (ctx->split_inbox) hipFree(ctx->split_inbox);
  ctx->split_inbox = nullptr;
  ctx->split_inbox_bytes = 0;
  for (auto& q : ctx->split_peer) q = nullptr;
  ctx->split_n = ctx->split_part = ctx->split_wl = 0;
  ctx->split_ready = false;
  ctx->split_broken = false;
  ctx->split_epoch = 0;
  ctx->split_chunks = 0;
}

int kss_split_config(kss_ctx* ctx, int32_t n_parts, int32_t part, int32_t shards_per_part) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx) return fail(KSS_E_INVAL, "null ctx");
  if (n_parts < 1 || n_parts > KSS_SPLIT_MAX_PARTS || part < 0 || part >= n_parts || shards_per_part < 1)
    return fail(KSS_E_INVAL, "bad split configuration");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  split_release(ctx);
  if (n_parts == 1) return 0;  // one part: the whole grid on this device, no inbox
  if (!ctx->stream_dedicated) {  // every part's grid must run beside the others': a queue of its own
    hipStream_t st = nullptr;
    HIP_TRY(dedicated_stream(ctx->n_cu, &st));
    HIP_TRY(hipStreamDestroy(ctx->stream));
    ctx->stream = st;
    ctx->stream_dedicated = true;
  }
  const size_t W = (size_t)n_parts * (size_t)shards_per_part;
  // two halves (chunk parity, split_chunks), each double-buffered by epoch parity
  const size_t bytes = 2 * sizeof(unsigned long long) * 2 * W * (size_t)std::max(2 * XW_MAX, G_XW);
  // uncached: the inbox is polled while other GPUs' stores land in it
  if (hipExtMallocWithFlags(&ctx->split_inbox, bytes, hipDeviceMallocUncached) != hipSuccess) {
    ctx->split_inbox = nullptr;
    if (hipMalloc(&ctx->split_inbox, bytes) != hipSuccess) return fail(KSS_E_NOMEM, "split inbox allocation failed");
  }
  HIP_TRY(dev_zero(ctx->split_inbox, bytes, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  HIP_TRY(hipDeviceSynchronize());
  ctx->split_inbox_bytes = bytes;
  ctx->split_n = n_parts;
  ctx->split_part = part;
  ctx->split_wl = shards_per_part;
  return 0;
}

int kss_split_inbox(kss_ctx* ctx, void** dev_ptr, size_t* bytes, void* ipc_handle) {
  if (!ctx || ctx->split_n < 2) return fail(KSS_E_INVAL, "no split grid configured");
  if (dev_ptr) *dev_ptr = ctx->split_inbox;
  if (bytes) *bytes = ctx->split_inbox_bytes;
  if (ipc_handle) {
    HIP_TRY(hipSetDevice(ctx->cfg.device));
    hipIpcMemHandle_t h;
    HIP_TRY(hipIpcGetMemHandle(&h, ctx->split_inbox));
    std::memcpy(ipc_handle, &h, sizeof(h));
  }
  return 0;
}

int kss_split_peers(kss_ctx* ctx, void* const* inboxes) {
  if (!ctx || ctx->split_n < 2 || !inboxes) return fail(KSS_E_INVAL, "no split grid configured");
  for (int i = 0; i < ctx->split_n; i++)
    if (!inboxes[i]) return fail(KSS_E_INVAL, "null peer inbox");
  if (inboxes[ctx->split_part] != ctx->split_inbox) return fail(KSS_E_INVAL, "this part's entry must be its own inbox");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  // inboxes of parts on other devices of this process: this device stores into them over
  // xGMI, which needs peer access from this device to theirs
  for (int i = 0; i < ctx->split_n; i++) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, inboxes[i]) != hipSuccess) return fail(KSS_E_INVAL, "peer inbox is not device memory");
    if (a.device == ctx->cfg.device) continue;
    int can = 0;
    HIP_TRY(hipDeviceCanAccessPeer(&can, ctx->cfg.device, a.device));
    if (!can) return fail(KSS_E_UNSUPPORTED, "split grid: no peer access between the parts' devices");
    const hipError_t e = hipDeviceEnablePeerAccess(a.device, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return fail(KSS_E_DEVICE, "hipDeviceEnablePeerAccess failed");
    (void)hipGetLastError();  // clear hipErrorPeerAccessAlreadyEnabled
  }
  for (int i = 0; i < ctx->split_n; i++) ctx->split_peer[i] = (unsigned long long*)inboxes[i];
  ctx->split_ready = true;
  return 0;
}

int kss_split_open(kss_ctx* ctx, const void* handles) {
  if (!ctx || ctx->split_n < 2 || !handles) return fail(KSS_E_INVAL, "no split grid configured");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  for (void* p : ctx->split_opened) hipIpcCloseMemHandle(p);
  ctx->split_opened.clear();
  for (int i = 0; i < ctx->split_n; i++) {
    if (i == ctx->split_part) {
      ctx->split_peer[i] = (unsigned long long*)ctx->split_inbox;
      continue;
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, (const char*)handles + (size_t)i * KSS_IPC_HANDLE_BYTES, sizeof(h));
    void* p = nullptr;
    HIP_TRY(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    ctx->split_opened.push_back(p);
    ctx->split_peer[i] = (unsigned long long*)p;
  }
  ctx->split_ready = true;
  return 0;
}

int kss_read_port_state(kss_ctx* ctx, uint64_t* port_used) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded || !port_used) return fail(KSS_E_INVAL, "bad arguments");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  HIP_TRY(hipMemcpyAsync(port_used, ctx->dc.port_used, 8 * (size_t)ctx->dc.N, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int kss_apply_port_delta(kss_ctx* ctx, const int32_t* idx, int32_t n, const uint64_t* port_used) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  if (n < 0 || (n > 0 && (!idx || !port_used))) return fail(KSS_E_INVAL, "bad arguments");
  for (int i = 0; i < n; i++) {
    if (idx[i] < 0 || idx[i] >= ctx->dc.N) return fail(KSS_E_INVAL, "port delta row out of range");
    if (ctx->host.n_ports < KSS_MAX_PORTS && (port_used[i] >> ctx->host.n_ports))
      return fail(KSS_E_INVAL, "port bit outside the port dictionary");
  }
  if (n == 0) return 0;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  // rows are few (pods bound elsewhere): one 8-byte copy per row, ordered on the stream
  for (int i = 0; i < n; i++)
    HIP_TRY(hipMemcpyAsync(ctx->dc.port_used + idx[i], port_used + i, 8, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int kss_read_binding_state(kss_ctx* ctx, int32_t* pv_owner, int32_t* claim_node) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  if (pv_owner && ctx->dc.n_pvs)
    HIP_TRY(hipMemcpyAsync(pv_owner, ctx->dc.pv_owner, 4 * (size_t)ctx->dc.n_pvs, hipMemcpyDeviceToHost, ctx->stream));
  if (claim_node && ctx->dc.n_wclaims)
    HIP_TRY(hipMemcpyAsync(claim_node, ctx->dc.claim_node, 4 * (size_t)ctx->dc.n_wclaims, hipMemcpyDeviceToHost,
                           ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int kss_read_volume_state(kss_ctx* ctx, int32_t* vol_count, int32_t* vol_attached) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  const size_t N = (size_t)ctx->dc.N;
  if (vol_count && ctx->dc.n_vol_rows)
    HIP_TRY(hipMemcpyAsync(vol_count, ctx->dc.vol_count, 4 * (size_t)ctx->dc.n_vol_rows * N, hipMemcpyDeviceToHost, ctx->stream));
  if (vol_attached && ctx->dc.n_vol_keys)
    HIP_TRY(hipMemcpyAsync(vol_attached, ctx->dc.vol_attached, 4 * (size_t)ctx->dc.n_vol_keys * N, hipMemcpyDeviceToHost,
                           ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int kss_apply_volume_delta(kss_ctx* ctx, const int32_t* node, const int32_t* row, const int32_t* value, int32_t n,
                           int32_t mode) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  if (n < 0 || (n > 0 && (!node || !row || !value)) || (mode != 0 && mode != 1)) return fail(KSS_E_INVAL, "bad arguments");
  const int R = ctx->dc.n_vol_rows, K = ctx->dc.n_vol_keys;
  for (int i = 0; i < n; i++) {
    if (node[i] < 0 || node[i] >= ctx->dc.N) return fail(KSS_E_INVAL, "delta node out of range");
    if (row[i] < 0 || row[i] >= R + K) return fail(KSS_E_INVAL, "delta volume row out of range");
  }
  if (n == 0) return 0;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  // one packed upload (node, row, value) and one scatter on the ctx stream
  const size_t bytes = 12 * (size_t)n;
  int rc = ctx->delta_buf.ensure(bytes);
  if (rc) return rc;
  std::vector<int32_t> h(3 * (size_t)n);
  std::memcpy(h.data(), node, 4 * (size_t)n);
  std::memcpy(h.data() + n, row, 4 * (size_t)n);
  std::memcpy(h.data() + 2 * (size_t)n, value, 4 * (size_t)n);
  HIP_TRY(hipMemcpyAsync(ctx->delta_buf.p, h.data(), bytes, hipMemcpyHostToDevice, ctx->stream));
  const int32_t* d = (const int32_t*)ctx->delta_buf.p;
  hipLaunchKernelGGL(k_volume_delta, dim3(1), dim3(64), 0, ctx->stream, ctx->dc, d, d + n,
                     d + 2 * (size_t)n, n, mode);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));  // the host copy h dies here
  return 0;
}

static PlanNeeds plan_needs(const int32_t* key_card, const uint32_t* key_flags, const kss_podset* ps, int n) {
  PlanNeeds r;
  r.xw = 12;  // the filter exchange's scalars
  for (int i = 0; i < n; i++) {
    const kss_pod& p = ps->pods[i];
    int bins = 0, hp = 0, sp = 0;
    if (p.n_hard | p.n_soft | p.ipa_len) r.general = true;
    if (p.port_conflict | p.port_add || p.img_len > 0 || p.vol_len > 0) r.ports_images = true;
    for (int h = 0; h < p.n_hard && h < MAXH; h++) {
      const int key = ps->spreads[p.spread_off + h].key;
      if (!(key_flags[key] & KSS_KEY_UNIQUE)) {
        bins += key_card[key] + 1;
        hp += key_card[key] + 1;
      }
    }
    for (int q = 0; q < p.n_soft && q < MAXS; q++) {
      const int key = ps->spreads[p.spread_off + p.n_hard + q].key;
      if (!(key_flags[key] & (KSS_KEY_HOSTNAME | KSS_KEY_UNIQUE))) {
        bins += key_card[key] + 1;
        sp += key_card[key] + 1;
      }
    }
    int keys[MAXK + 1], nk = 0;
    for (int e = 0; e < p.ipa_len; e++) {
      const int key = ps->ipa[p.ipa_off + e].key;
      bool seen = false;
      for (int j = 0; j < nk; j++) seen |= keys[j] == key;
      if (seen) continue;
      if (nk <= MAXK) keys[nk++] = key;
      if (!(key_flags[key] & KSS_KEY_UNIQUE)) bins += 4 * (key_card[key] + 1);
    }
    r.bins_cap = std::max(r.bins_cap, bins + hp + sp);
    r.xw = std::max(r.xw, std::max(MAXH + 1 + bins + hp, 12 + sp));
  }
  r.bins_cap = std::min(r.bins_cap, LDS_BINS);
  return r;
}

static size_t lds_bytes(int bins_cap, int slots) {
  return sizeof(SharedHdr) + 8 * (size_t)(NSCAL + bins_cap) + slot_arrays_bytes(slots);
}

// Geometry for clusters of at most maxN nodes split in W shards.
struct Geometry {
  int W = 1, threads = 64, npt = 1;
};

static bool pick_geometry(int maxN, int W, int pref_threads, Geometry& g) {
  g.W = W;
  const int per = (std::max(maxN, 1) + W - 1) / W;
  int t = std::min(KSS_MAX_THREADS, std::max(pref_threads, 64));
  if (per < t) t = std::max(64, (per + 63) / 64 * 64);
  int npt = (per + t - 1) / t;
  const long long ft = opt(O_FORCE_THREADS);  // tuning / diagnosis: exact workgroup size
  if (ft > 0) {
    t = (int)std::min<long long>(KSS_MAX_THREADS, std::max(64ll, ft / 64 * 64));
    npt = (per + t - 1) / t;
  }
  while (ft <= 0 && npt > 4 && t < KSS_MAX_THREADS) {
    t = std::min(KSS_MAX_THREADS, t * 2);
    npt = (per + t - 1) / t;
  }
  g.threads = t;
  g.npt = npt;
  return npt <= KSS_MAX_NPT;
}

// Launch of a sharded (W > 1) grid whose workgroups must all be resident at once: the
// host checks the occupancy (one workgroup per CU at this LDS / register footprint, and
// no more workgroups than CUs) and launches plainly.  KSS_COOP_LAUNCH=1 uses the
// cooperative launch instead (same residency, runtime-checked).
static int launch_resident(const void* fn, dim3 grid, dim3 block, void** args, size_t shmem, hipStream_t st) {
  if (opt(O_COOP_LAUNCH)) {
    HIP_TRY(hipLaunchCooperativeKernel(fn, grid, block, args, (unsigned)shmem, st));
    return 0;
  }
  int dev = 0, n_cu = 0, per_cu = 0;
  HIP_TRY(hipGetDevice(&dev));
  HIP_TRY(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, (int)(block.x * block.y * block.z), shmem));
  if (per_cu < 1 || (long long)grid.x > (long long)per_cu * n_cu)
    return fail(KSS_E_UNSUPPORTED, "sharded grid cannot be co-resident on this device");
  HIP_TRY(hipLaunchKernel(fn, grid, block, args, shmem, st));
  return 0;
}

// Launch k_schedule over n_jobs clusters (jobs already in device memory).  W > 1 needs
// every workgroup resident: cooperative launch (the runtime checks the grid fits).
static int launch_schedule(hipStream_t st, const Geometry& g, int n_jobs, int bins_cap, bool need_general, int n_keys,
                           const DevJob* jobs, const kss_profile& prof, unsigned long long* gran, int* err,
                           unsigned long long* stamps = nullptr, unsigned epoch0 = 0) {
  const int cap = g.threads * g.npt;
  const size_t base = lds_bytes(bins_cap, cap);
  if (base > KSS_LDS_BUDGET) return fail(KSS_E_UNSUPPORTED, "per-workgroup LDS budget exceeded (too many nodes per shard)");
  // node cache with every label key, without labels, or none, whatever fits
  int cache_keys = -1;
  if (!opt(O_NO_CACHE)) {
    if (base + node_cache_bytes(cap, n_keys) <= KSS_LDS_BUDGET) cache_keys = n_keys;
    else if (base + node_cache_bytes(cap, 0) <= KSS_LDS_BUDGET) cache_keys = 0;
  }
  const size_t shmem = base + (cache_keys >= 0 ? node_cache_bytes(cap, cache_keys) : 0);
  const bool gen = bins_cap > 0 || need_general;
  const void* fn = gen ? (const void*)k_schedule<true> : (const void*)k_schedule<false>;
  HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
  const dim3 grid((unsigned)(n_jobs * g.W)), block((unsigned)g.threads);
  kss_profile pr = prof;
  int W = g.W, npt = g.npt;
  if (g.W > 1) {
    void* args[] = {(void*)&jobs, (void*)&pr,   (void*)&W,   (void*)&npt,   (void*)&bins_cap,
                    (void*)&cache_keys, (void*)&gran, (void*)&err, (void*)&stamps, (void*)&epoch0};
    if (int rc = launch_resident(fn, grid, block, args, shmem, st)) return rc;
  } else {
    if (gen)
      hipLaunchKernelGGL(k_schedule<true>, grid, block, shmem, st, jobs, pr, W, npt, bins_cap, cache_keys, gran, err, stamps,
                         epoch0);
    else
      hipLaunchKernelGGL(k_schedule<false>, grid, block, shmem, st, jobs, pr, W, npt, bins_cap, cache_keys, gran, err, stamps,
                         epoch0);
    HIP_TRY(hipGetLastError());
  }
  return 0;
}

// Field-wise profile equality (padding excluded).
static bool same_profile(const kss_profile& a, const kss_profile& b) {
  bool eq = a.filter_enabled == b.filter_enabled && a.score_enabled == b.score_enabled &&
            a.fit_strategy == b.fit_strategy && a.fit_n == b.fit_n && a.ba_n == b.ba_n &&
            a.hard_pod_affinity_weight == b.hard_pod_affinity_weight && a.system_defaulted == b.system_defaulted;
  for (int i = 0; i < KSS_NSCORE; i++) eq &= a.weight[i] == b.weight[i];
  for (int i = 0; i < 4; i++) eq &= a.fit_res[i] == b.fit_res[i] && a.fit_weight[i] == b.fit_weight[i] && a.ba_res[i] == b.ba_res[i];
  return eq;
}

// Node slots per shard for k_simple: every lane's share (the first slot without a node
// re-evaluates the candidate after the previous commit).
static int simple_cap(const Geometry& g) { return g.npt * g.threads; }

static bool simple_fits(const Geometry& g, int nsc) {
  const int pf_n = g.threads > 64 ? g.threads - 64 : g.threads;  // prefetch lanes (kss_simple.cuh)
  return g.W <= 64 * SX_CHUNKS && g.npt <= KSS_MAX_NPT && (simple_cap(g) + pf_n - 1) / pf_n <= PF_MAX &&
         simple_lds_bytes(simple_cap(g), nsc) <= KSS_LDS_BUDGET;
}

// Extended (scalar) resources on k_simple / k_spread: their NodeResourcesFit filter and
// AssumePod run in LDS; a profile that scores one (fit / BalancedAllocation resources past
// ephemeral-storage) keeps the batch on k_schedule.
static bool scalar_fast_ok(const kss_profile& p, int n_scalar) {
  if (n_scalar == 0) return true;
  for (int i = 0; i < p.fit_n && i < 4; i++)
    if (p.fit_res[i] >= KSS_RES_SCALAR0) return false;
  for (int i = 0; i < p.ba_n && i < 4; i++)
    if (p.ba_res[i] >= KSS_RES_SCALAR0) return false;
  return true;
}

// Static-word scratch bound (KSS_STATIC_BYTES): pods are processed in chunks whose words
// fit; each chunk is one k_static launch and one k_simple launch (node state stays in HBM
// between them).  Default: an eighth of the current device's free memory, between 1 and 16 GiB
// (MI355X: 16 GiB) -- C2 (5,000 x 10,000 x 4 B = 200 MB), C4 (100,000 x 20,000: 8 GB) and the
// c5_sweep leg (4,096 scenarios x 1,000 x 1,000: 16.4 GB) in one chunk, without per-chunk
// relaunches of the loop kernel.
static size_t static_budget() {
  const long long v = opt(O_STATIC_BYTES);
  if (v > 0) return (size_t)v;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = 0;
  return std::min((size_t)16 << 30, std::max((size_t)1 << 30, fr / 8));
}

// Pods per chunk for jobs whose node counts sum to sum_nodes.
static int static_chunk(size_t sum_nodes, int n_pods) {
  const size_t per_pod = 4 * std::max<size_t>(sum_nodes, 1);
  const size_t c = std::max<size_t>(1, static_budget() / per_pod);
  return (int)std::min<size_t>(c, (size_t)std::max(n_pods, 1));
}

// k_static + k_simple over pods [0, n_pods_max) of n_jobs jobs, `chunk` pods at a time.
// The jobs' stat pointers must hold chunk x N words each.  Every polled granule is zeroed
// before each k_simple launch (epochs restart at 1).
// ev (optional): 2 events per chunk recorded around each k_simple launch.
// Split grids (X->n > 1): this launch runs shards [w_off, w_off + wl) of g.W and k_static
// only their rows; granules are never cleared (a peer may already publish into the inbox):
// chunk c starts its epochs at epoch0 + c * span, above every tag an earlier chunk left.
struct SplitRun {
  XPeers X{};
  unsigned epoch0 = 0;
  unsigned long long chunk0 = 0;  // global chunk sequence number of this run's first chunk
  size_t half_words = 0;          // inbox half (one chunk's exchange buffer), in 8-byte words
};

// The exchange buffer and peer inboxes of chunk ci of a split run: half (chunk0 + ci) & 1.
static void split_chunk_view(const SplitRun& sr, int ci, unsigned long long* gran, unsigned long long*& g_out,
                             XPeers& x_out) {
  const size_t off = (size_t)((sr.chunk0 + (unsigned long long)ci) & 1ull) * sr.half_words;
  x_out = sr.X;
  for (int i = 0; i < x_out.n; i++) x_out.inbox[i] = sr.X.inbox[i] + off;
  g_out = gran + off;
}

static unsigned chunk_span(int pods) { return 8u * (unsigned)std::max(pods, 1) + 16u; }

static void static_rows(const Geometry& g, const XPeers& X, int max_nodes, int& n_lo, int& n_hi) {
  n_lo = 0;
  n_hi = max_nodes;
  if (X.n <= 1) return;
  const int per = (max_nodes + g.W - 1) / g.W;
  n_lo = std::min(max_nodes, X.w_off * per);
  n_hi = std::min(max_nodes, (X.w_off + X.wl) * per);
}

// k_static over pods [k0, k1) x rows [n_lo, n_hi) of n_jobs jobs; max_keys: the jobs' largest label-key count
// (the LDS label copy when it is at most STATIC_LKEYS)
static void launch_static(hipStream_t st, bool def, const DevJob* jobs, const kss_profile& pr, int n_jobs, int k0, int k1,
                          int n_lo, int n_hi, int max_keys, int row0 = 0) {
  const int lk = max_keys > 0 && max_keys <= STATIC_LKEYS ? max_keys : 0;
  // pods per block: with the LDS label copy, enough pods to amortise loading it (C5: 64 pods of
  // 1,000 nodes per block; r6c: 8 / 16 / 32 / 64 within 1 % of each other)
  int ppb = lk ? 8 * STATIC_PODS : STATIC_PODS;
  if (opt(O_STATIC_PPB) > 0) ppb = (int)std::min(256ll, opt(O_STATIC_PPB));
  const dim3 sgrid((unsigned)(std::max(n_hi - n_lo, 1) + 1023) / 1024, (unsigned)((k1 - k0 + ppb - 1) / ppb),
                   (unsigned)n_jobs);
  const size_t sh = sizeof(int32_t) * 1024 * (size_t)lk;
  if (def)
    hipLaunchKernelGGL(k_static<true>, sgrid, dim3(256), sh, st, jobs, pr, k0, k1, n_lo, n_hi, lk, row0, ppb);
  else
    hipLaunchKernelGGL(k_static<false>, sgrid, dim3(256), sh, st, jobs, pr, k0, k1, n_lo, n_hi, lk, row0, ppb);
}

// xcd: one job on an XCD-local grid (xcd_slot); a chunk whose launch reports the placement
// failure (err = 3, no state touched) is synchronised on and run again unrestricted.
static int launch_simple(hipStream_t st, const Geometry& g, int n_jobs, const DevJob* jobs, const kss_profile& prof,
                         int n_pods_max, int max_nodes, int chunk, unsigned long long* gran, size_t gran_bytes, int* err,
                         unsigned long long* stamps = nullptr, hipEvent_t* ev = nullptr, const SplitRun* split = nullptr,
                         int nsc = 0, bool xcd = false, int* xcd_fallbacks = nullptr, int max_keys = 0,
                         hipStream_t st2 = nullptr, std::vector<hipEvent_t>* pev = nullptr, int k_find = 0) {
  // st2 (with pev, two events per chunk): the static words of chunk i+1 are computed on st2 into the
  // other half of a double-buffered table while k_simple runs chunk i on st (each job's table holds
  // 2 x chunk rows); k_simple of chunk i waits for its k_static, k_static of chunk i+1 for
  // k_simple of chunk i-1 (the last reader of that half)
  int cap = simple_cap(g);
  const size_t shmem = simple_lds_bytes(cap, nsc);
  const bool def = same_profile(prof, default_profile_c());
  // k_find > 0: the percentageOfNodesToScore window (one job, not split)
  const bool win = k_find > 0;
  const void* fn = win ? (def ? (const void*)k_simple<true, true> : (const void*)k_simple<false, true>)
                       : (def ? (const void*)k_simple<true, false> : (const void*)k_simple<false, false>);
  HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
  XPeers X = split ? split->X : XPeers{};
  const bool sp_grid = X.n > 1;
  xcd = xcd && !sp_grid && n_jobs == 1 && gran;
  const dim3 grid((unsigned)(n_jobs * (sp_grid ? X.wl : g.W))), block((unsigned)g.threads);
  const dim3 xgrid((unsigned)(XCD_GRID_MULT * g.W));
  kss_profile pr = prof;
  int W = g.W, n_lo = 0, n_hi = 0;
  static_rows(g, X, max_nodes, n_lo, n_hi);
  const bool pipe = st2 && pev && !sp_grid && !xcd;
  const int n_chunks = (n_pods_max + chunk - 1) / std::max(chunk, 1);
  if (pipe) {
    while ((int)pev->size() < 2 * n_chunks) {
      hipEvent_t e;
      HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      pev->push_back(e);
    }
    // (*pev)[2i]: k_static of chunk i done (st2), (*pev)[2i+1]: k_simple of chunk i done (st)
    HIP_TRY(hipEventRecord((*pev)[1], st));  // st's work so far (the reset) before st2 writes the table
    HIP_TRY(hipStreamWaitEvent(st2, (*pev)[1], 0));
    launch_static(st2, def, jobs, pr, n_jobs, 0, std::min(n_pods_max, chunk), n_lo, n_hi, max_keys, 0);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord((*pev)[0], st2));
  }
  for (int k0 = 0; k0 < n_pods_max; k0 += chunk) {
    int k1 = std::min(n_pods_max, k0 + chunk);
    const int ci_ = k0 / std::max(chunk, 1);
    int row0 = pipe ? (ci_ & 1) * chunk : 0;
    if (pipe) {
      HIP_TRY(hipStreamWaitEvent(st, (*pev)[2 * ci_], 0));  // this chunk's static words
      if (k1 < n_pods_max) {  // the next chunk's, into the other half, once chunk ci-1 no longer reads it
        if (ci_ > 0) HIP_TRY(hipStreamWaitEvent(st2, (*pev)[2 * (ci_ - 1) + 1], 0));
        launch_static(st2, def, jobs, pr, n_jobs, k1, std::min(n_pods_max, k1 + chunk), n_lo, n_hi, max_keys,
                      ((ci_ + 1) & 1) * chunk);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord((*pev)[2 * (ci_ + 1)], st2));
      }
    } else {
      launch_static(st, def, jobs, pr, n_jobs, k0, k1, n_lo, n_hi, max_keys);
      HIP_TRY(hipGetLastError());
    }
    unsigned epoch0 = 0;
    unsigned long long* gc = gran;
    if (sp_grid) {
      epoch0 = split->epoch0 + (unsigned)(k0 / std::max(chunk, 1)) * chunk_span(chunk);
      split_chunk_view(*split, k0 / std::max(chunk, 1), gran, gc, X);
    } else if (gran && k0 > 0) {
      HIP_TRY(dev_zero(gran, gran_bytes, st));
    }
    unsigned long long* sp = k0 == 0 ? stamps : nullptr;
    void* args[] = {(void*)&jobs, (void*)&pr, (void*)&W,  (void*)&cap, (void*)&k0,     (void*)&k1,
                    (void*)&gc,   (void*)&err, (void*)&sp, (void*)&X,   (void*)&epoch0, (void*)&row0, (void*)&k_find};
    const int ci = k0 / chunk;
    if (ev) HIP_TRY(hipEventRecord(ev[2 * ci], st));
    if (xcd) {
      X.xcd_local = opt(O_XCD_FORCE_FALLBACK) ? 2 : 1;  // 2: placement reported failed (tests)
      if (int rc = launch_resident(fn, xgrid, block, args, shmem, st)) return rc;
      int e = 0;
      HIP_TRY(hipMemcpyAsync(&e, err, sizeof(int), hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      X.xcd_local = 0;
      if (e == 3) {  // XCD 0 did not get W workgroups: nothing ran; again, unrestricted
        if (xcd_fallbacks) ++*xcd_fallbacks;
        xcd = false;
        HIP_TRY(dev_zero(err, 4, st));
        HIP_TRY(dev_zero(gran, gran_bytes, st));
        if (int rc = launch_resident(fn, grid, block, args, shmem, st)) return rc;
      }
    } else if (g.W > 1) {
      if (int rc = launch_resident(fn, grid, block, args, shmem, st)) return rc;
    } else {
      HIP_TRY(hipLaunchKernel(fn, grid, block, args, shmem, st));
    }
    if (ev) HIP_TRY(hipEventRecord(ev[2 * ci + 1], st));
    if (pipe) HIP_TRY(hipEventRecord((*pev)[2 * ci + 1], st));
  }
  hipLaunchKernelGGL(k_counts, dim3((unsigned)((n_pods_max + 255) / 256), (unsigned)n_jobs), dim3(256), 0, st, jobs, 0,
                     n_pods_max);
  HIP_TRY(hipGetLastError());
  return 0;
}

#ifndef KSS_SPREAD_PREF_THREADS
#define KSS_SPREAD_PREF_THREADS 512
#endif

// k_spread's per-slot LDS arrays are strided by the largest shard's node count (rounded up
// to 16 slots), not by threads x slots per lane: a 391-node shard of a 100k-node cluster
// keeps 400 slots, not 512.
static int spread_cap(const Geometry& g, size_t N) {
  const size_t per = (N + (size_t)g.W - 1) / (size_t)g.W;
  return (int)align_up(std::max(per, (size_t)1), 16);
}

static size_t spread_lds(const Geometry& g, const GpodNeeds& q, int n_keys, int n_res, size_t N, int nsc) {
  return spread_lds_bytes(spread_cap(g, N), q.bins_cap, n_keys, n_res, q.gq, nsc, opt(O_FOLD) != 0);
}

static bool spread_fits(const Geometry& g, const GpodNeeds& q, int n_keys, int n_res, size_t N, int nsc) {
  const int pf_n = g.threads > 64 ? g.threads - 64 : g.threads;  // prefetch lanes (kss_spread.cuh)
  const int per = (int)((N + (size_t)g.W - 1) / (size_t)g.W);
  return (per + pf_n - 1) / pf_n <= G_PF && per <= g.npt * g.threads &&
         spread_lds(g, q, n_keys, n_res, N, nsc) <= KSS_LDS_BUDGET;
}

// The checked hand-off's buffer (ck_buf), in 8-byte words: {sum, tag} per shard, the XCC of
// each shard's last epilogue (int), the diagnosis list, the shadow copy of the node state.
struct HandoffLayout {
  size_t o_xcc, o_diag, o_shadow, words;
  HandoffLayout(int W, int n_res, int N, int nsc) {
    o_xcc = 2 * (size_t)W;
    o_diag = o_xcc + ((size_t)W + 1) / 2;
    o_shadow = (o_diag + 1 + (size_t)HANDOFF_DIAG * HANDOFF_DIAG_W + 15) / 16 * 16;
    words = o_shadow + (6 + (size_t)std::max(n_res, 0) + (size_t)std::max(nsc, 0)) * (size_t)std::max(N, 1);
  }
};

// k_static + k_spread over pods [0, n_pods) of one job, `chunk` pods at a time (node state
// and counts back in HBM between launches).  ev (optional): 2 events per chunk.
static int launch_spread(hipStream_t st, const Geometry& g, const GpodNeeds& q, int n_keys, int n_res,
                         const DevJob* jobs, const kss_profile& prof, int n_pods, int max_nodes, int chunk,
                         unsigned long long* gran, size_t gran_bytes, int* err, unsigned long long* stamps = nullptr,
                         hipEvent_t* ev = nullptr, const SplitRun* split = nullptr, unsigned long long* ck = nullptr,
                         unsigned long long* ck_seq = nullptr, int nsc = 0, bool xcd = false, int* xcd_fallbacks = nullptr,
                         int k_find = 0) {
  int cap = spread_cap(g, (size_t)max_nodes), bins_cap = q.bins_cap, nr = n_res, gq = q.gq, gs = q.gs();
  size_t shmem = spread_lds(g, q, n_keys, n_res, (size_t)max_nodes, nsc);
  // diagnostic stamps in LDS: as many pods (<= G_NSTAMP, >= 8) as fit beside the shard state
  int nst = 0;
  if (stamps && shmem < KSS_LDS_BUDGET) nst = (int)std::min<size_t>(G_NSTAMP, (KSS_LDS_BUDGET - shmem) / (16 * 8));
  if (nst < 8) stamps = nullptr, nst = 0;
  shmem += (size_t)nst * 16 * 8;
#ifdef KSS_EXPERIMENTS
  if (const char* e = getenv("KSS_SPREAD_MIN_LDS"))  // diagnosis: at most one shard per CU
    shmem = std::max(shmem, std::min((size_t)KSS_LDS_BUDGET, (size_t)std::max(0, atoi(e))));
#endif
  const bool def = same_profile(prof, default_profile_c());
  const bool fold = opt(O_FOLD) != 0;
  const bool lb = g.threads <= 256 && opt(O_SPREAD_LB256);
  const void* fn = lb ? (def ? (fold ? (const void*)k_spread<true, true, 256, false> : (const void*)k_spread<true, false, 256, false>)
                             : (fold ? (const void*)k_spread<false, true, 256, false> : (const void*)k_spread<false, false, 256, false>))
                      : (def ? (fold ? (const void*)k_spread<true, true, KSS_MAX_THREADS, false>
                                     : (const void*)k_spread<true, false, KSS_MAX_THREADS, false>)
                             : (fold ? (const void*)k_spread<false, true, KSS_MAX_THREADS, false>
                                     : (const void*)k_spread<false, false, KSS_MAX_THREADS, false>));
  // the window (default profile, no fold): its own instantiations
  if (k_find > 0) {
    if (!def || fold) return fail(KSS_E_INVAL, "k_spread window: default profile, no statistics fold");
    fn = lb ? (const void*)k_spread<true, false, 256, true> : (const void*)k_spread<true, false, KSS_MAX_THREADS, true>;
  }
  HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
  XPeers X = split ? split->X : XPeers{};
  const bool sp_grid = X.n > 1;
  xcd = xcd && !sp_grid && gran && g.W > 1;
  const dim3 grid((unsigned)(sp_grid ? X.wl : g.W)), block((unsigned)g.threads);
  const dim3 xgrid((unsigned)(XCD_GRID_MULT * g.W));
  // many shards on one part: the two-level selectHost exchange, its area at the end of the
  // granule buffer (run_single reserves tl_words)
  const size_t tlw = tl_words(g.W);
  if (!sp_grid && !xcd && gran && g.W > 64 && opt(O_SPREAD_TWO_LEVEL) &&
      gran_bytes / 8 >= tlw + 2 * (size_t)g.W * (size_t)gs + 16)
    X.tl = gran + gran_bytes / 8 - tlw, X.tl_red = opt(O_SPREAD_TWO_LEVEL) >= 2;
  kss_profile pr = prof;
  int W = g.W, n_lo = 0, n_hi = 0;
  static_rows(g, X, max_nodes, n_lo, n_hi);
  for (int k0 = 0; k0 < n_pods; k0 += chunk) {
    int k1 = std::min(n_pods, k0 + chunk);
    launch_static(st, def, jobs, pr, 1, k0, k1, n_lo, n_hi, n_keys);
    HIP_TRY(hipGetLastError());
    // every chunk's tags above the previous chunk's (a line an earlier chunk left in an XCD's
    // L2 never carries a current tag), the buffer zeroed as well
    unsigned epoch0 = (unsigned)(k0 / std::max(chunk, 1)) * chunk_span(chunk);
    unsigned long long* gc = gran;
    if (sp_grid) {
      epoch0 += split->epoch0;
      split_chunk_view(*split, k0 / std::max(chunk, 1), gran, gc, X);
    } else if (gran && k0 > 0) {
      HIP_TRY(dev_zero(gran, gran_bytes, st));
    }
    unsigned long long* sp = k0 == 0 ? stamps : nullptr;
    // the checked node-state hand-off between this call's chunks (HandoffCheck): tags increase
    // over the context's life, the first chunk of a call checks nothing
    HandoffCheck hc{};
    if (ck && ck_seq) {
      const HandoffLayout hl(g.W, n_res, max_nodes, nsc);
      hc.sum = ck;
      hc.expect = k0 > 0 ? *ck_seq : 0ull;
      hc.write = ++*ck_seq;
      hc.retries = err + 1;
      hc.xcc = (int*)(ck + hl.o_xcc);
      hc.diag = (long long*)(ck + hl.o_diag);
      hc.shadow = (long long*)(ck + hl.o_shadow);
    }
    void* args[] = {(void*)&jobs, (void*)&W,  (void*)&cap, (void*)&bins_cap, (void*)&nr,  (void*)&gq, (void*)&gs, (void*)&k0,
                    (void*)&k1,   (void*)&gc, (void*)&err, (void*)&sp,       (void*)&nst, (void*)&X,  (void*)&epoch0,
                    (void*)&hc,   (void*)&k_find};
    const int ci = k0 / chunk;
    if (ev) HIP_TRY(hipEventRecord(ev[2 * ci], st));
    if (xcd) {  // as launch_simple: an XCD-local grid, run again unrestricted when placement failed
      X.xcd_local = opt(O_XCD_FORCE_FALLBACK) ? 2 : 1;  // 2: placement reported failed (tests)
      if (int rc = launch_resident(fn, xgrid, block, args, shmem, st)) return rc;
      int e = 0;
      HIP_TRY(hipMemcpyAsync(&e, err, sizeof(int), hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      X.xcd_local = 0;
      if (e == 3) {
        if (xcd_fallbacks) ++*xcd_fallbacks;
        xcd = false;
        HIP_TRY(dev_zero(err, 4, st));
        HIP_TRY(dev_zero(gran, gran_bytes, st));
        if (int rc = launch_resident(fn, grid, block, args, shmem, st)) return rc;
      }
    } else if (g.W > 1) {
      if (int rc = launch_resident(fn, grid, block, args, shmem, st)) return rc;
    } else {
      HIP_TRY(hipLaunchKernel(fn, grid, block, args, shmem, st));
    }
    if (ev) HIP_TRY(hipEventRecord(ev[2 * ci + 1], st));
  }
  if (ck && ck_seq && n_pods > 0) {  // the last chunk's write-back, checked (nothing repairs it)
    const HandoffLayout hl(g.W, n_res, max_nodes, nsc);
    HandoffCheck hc{};
    hc.sum = ck;
    hc.expect = *ck_seq;
    hc.retries = err + 1;
    hc.xcc = (int*)(ck + hl.o_xcc);
    hc.diag = (long long*)(ck + hl.o_diag);
    hc.shadow = (long long*)(ck + hl.o_shadow);
    hipLaunchKernelGGL(k_handoff_final, grid, dim3(256), 0, st, jobs, W, sp_grid ? X.w_off : 0, n_res, hc, err);
    HIP_TRY(hipGetLastError());
  }
  return 0;
}

// run k_schedule / k_simple / k_spread on the loaded cluster for pods [0, n); results stay on the device
// A device range copied back with the launch's outcome (one pinned staging, one sync).
struct ReadBack {
  const void* src = nullptr;
  size_t bytes = 0;
  const char* host = nullptr;  // set by run_single: the bytes in pinned memory until the next call
};

static int ensure_pinned(void*& p, size_t& cap, size_t need) {
  if (cap >= need) return 0;
  if (p) HIP_TRY(hipHostFree(p));
  p = nullptr;
  cap = 0;
  HIP_TRY(hipHostMalloc(&p, std::max(need, (size_t)4096), hipHostMallocDefault));
  cap = std::max(need, (size_t)4096);
  return 0;
}

static int run_single_impl(kss_ctx* ctx, const PlanNeeds& need, const DevPods& dp, int n, bool commit, bool record,
                           bool keep_norm, uint32_t flags, int32_t* chosen_out, bool staged, ReadBack* rbk,
                           const PackedUpload* pu);

// A split run that fails once its granule epochs are assigned (an exchange timed out, or the
// launch failed) leaves this part's epochs apart from its peers': the context then refuses
// split runs until kss_split_config re-arms it (fresh zeroed inbox, epochs from 0) — on
// every part, with the peers exchanged again.
static int run_single(kss_ctx* ctx, const PlanNeeds& need, const DevPods& dp, int n, bool commit, bool record,
                      bool keep_norm, uint32_t flags, int32_t* chosen_out, bool staged = false, ReadBack* rbk = nullptr,
                      const PackedUpload* pu = nullptr) {
  const bool split = ctx->split_n > 1;
  if (split && ctx->split_broken)
    return fail(KSS_E_INVAL, "split grid: an earlier run failed; re-arm every part (kss_split_config, then the peers)");
  const unsigned e0 = ctx->split_epoch;
  const int rc = run_single_impl(ctx, need, dp, n, commit, record, keep_norm, flags, chosen_out, staged, rbk, pu);
  if (rc && split && ctx->split_epoch != e0) ctx->split_broken = true;
  return rc;
}

static int run_single_impl(kss_ctx* ctx, const PlanNeeds& need, const DevPods& dp, int n, bool commit, bool record,
                           bool keep_norm, uint32_t flags, int32_t* chosen_out, bool staged, ReadBack* rbk,
                           const PackedUpload* pu) {
  const size_t N = (size_t)ctx->dc.N;
  const SlotLayout SL(N);
  const int nslots = record ? std::max(n, 1) : 1;
  int rc = ctx->slot_buf.ensure(SL.bytes * (size_t)nslots);
  if (rc) return rc;
  rc = ctx->meta_buf.ensure(sizeof(PodMeta) * (size_t)std::max(n, 1));
  if (rc) return rc;
  rc = ctx->chosen_buf.ensure(sizeof(int32_t) * (size_t)std::max(n, 1));
  if (rc) return rc;
  // shard count: ~nodes_per_shard nodes per workgroup, at most one workgroup per CU
  int W = std::max(1, std::min(ctx->n_cu, (int)((N + ctx->nodes_per_shard - 1) / ctx->nodes_per_shard)));
  if (ctx->force_w > 0) W = std::min(ctx->force_w, ctx->n_cu);
  // split grid (kss_split_config): the shard count is fixed by the parts, every part the same
  const bool split = ctx->split_n > 1;
  if (split) {
    if (!staged || !commit || record || keep_norm || (flags & (KSS_SCHED_FORCE_SINGLE_WG | KSS_SCHED_FORCE_MULTI_WG)))
      return fail(KSS_E_UNSUPPORTED, "split grids run staged, unrecorded batches (kss_run_staged)");
    if (!ctx->split_ready) return fail(KSS_E_INVAL, "split grid: peers not set (kss_split_peers / kss_split_open)");
    W = ctx->split_n * ctx->split_wl;
  }
  if (flags & KSS_SCHED_FORCE_SINGLE_WG) W = 1;
  if (flags & KSS_SCHED_FORCE_MULTI_WG) W = std::max(W, std::min(4, ctx->n_cu));
  W = std::max(1, std::min(W, std::max(1, (int)N)));
  // a split grid's shard count is fixed by its parts: never clamp it (a shard past W would
  // publish into the other epoch parity's granules)
  if (split && W != ctx->split_n * ctx->split_wl)
    return fail(KSS_E_UNSUPPORTED, "split grid: more shards than nodes (fewer shards per part)");
  // a k_simple-eligible batch keeps W within k_simple's exchange sweep (64 * SX_CHUNKS
  // shards): at 100k nodes, 98-128 k_simple shards beat 256 k_schedule shards (69.8k
  // against 44.2k pods/s)
  // percentageOfNodesToScore below 100: findNodesThatPassFilters' window (numFeasibleNodesToFind,
  // nextStartNodeIndex) runs on k_schedule only; its per-shard count exchange needs W + 1 values
  const bool window = ctx->prof.pct_nodes_to_score < 100;
  // k_simple runs the window itself (simple_sync_win) for pods without a PreFilterResult list on an
  // unsplit grid; k_find = N: the list is too short for a window (every node processed)
  const int k_find = window ? num_feasible_to_find((int)N, ctx->prof.pct_nodes_to_score) : (int)N;
  const bool simple_win_ok = !window || k_find >= (int)N || (!split && !ctx->staged_names);
  if (window) W = std::min(W, XW_MAX - NSCAL);  // k_schedule's window exchange: W + 1 values
  // nominated pods (kss_nominate): RunFilterPluginsWithNominatedPods and PreferNominatedNode run on
  // k_schedule only
  const bool nomq = !ctx->nom.empty();
  if (nomq && split) return fail(KSS_E_UNSUPPORTED, "split grids do not read the nominator");
  const bool simple_ok = simple_win_ok && !nomq && staged && ctx->spod_ok && commit && !record && !keep_norm && !need.general &&
                         scalar_fast_ok(ctx->prof, ctx->dc.n_scalar) && ctx->small_values && f64_exact(ctx->f64_cluster, ctx->f64_pods, n) &&
                         !ctx->no_simple && !(flags & KSS_SCHED_GENERAL_KERNEL);
  if (simple_ok && ctx->force_w <= 0 && !split) W = std::min(W, 64 * SX_CHUNKS);
  // XCD-local k_simple (launch_simple xcd, xcd_slot): a cluster whose shards fit one XCD's CUs
  // at one node per lane runs every shard on XCD 0, so the per-pod exchange stays in that
  // XCD's L2 (KSS_XCD=0: off)
  const int xcd_cus = ctx->n_cu / XCD_GRID_MULT;
  const bool xcd_try = simple_ok && !split && ctx->force_w <= 0 && ctx->xcd_mode && ctx->n_cu % XCD_GRID_MULT == 0 &&
                       !(flags & (KSS_SCHED_FORCE_SINGLE_WG | KSS_SCHED_FORCE_MULTI_WG)) &&
                       N <= (size_t)(ctx->xcd_w > 0 ? ctx->xcd_w : xcd_cus) * PW_LANES * (KSS_MAX_THREADS / 64);
  if (xcd_try) W = std::min(W, ctx->xcd_w > 0 ? ctx->xcd_w : xcd_cus);
  // a batch with programs on k_spread: 32-bit counts and scores (spread_bounds_ok)
  const double count_total = ctx->count_bound + (commit ? (double)n * (1.0 + ctx->staged_max_own) : 0.0);
  const double cell_total = ctx->cell_bound + (commit ? (double)n * ctx->gneed.max_mult : 0.0);
  // k_spread runs the window itself (spread_schedule WIN) for default-profile pods without a
  // PreFilterResult list on an unsplit grid, the statistics fold off
  const bool spread_win = window && k_find < (int)N;
  const bool spread_win_ok = !spread_win || (!split && !ctx->staged_names && !opt(O_FOLD) &&
                                             same_profile(ctx->prof, default_profile_c()));
  const bool spread_ok = spread_win_ok && !nomq && staged && ctx->gpod_ok && commit && !record && !keep_norm && need.general &&
                         scalar_fast_ok(ctx->prof, ctx->dc.n_scalar) && ctx->small_values && f64_exact(ctx->f64_cluster, ctx->f64_pods, n) &&
                         !ctx->no_simple && !ctx->no_spread && !(flags & KSS_SCHED_GENERAL_KERNEL) &&
                         spread_bounds_ok(ctx->gneed, count_total, cell_total, (int)N);
  if (opt(O_TRACE_PATH))  // diagnosis: why a batch with programs is (not) on k_spread
    fprintf(stderr,
            "kss path: staged=%d gpod_ok=%d commit=%d record=%d general=%d scalar=%d small=%d f64=%d bounds=%d "
            "(ref_weight=%lld total=%.0f cell=%.0f) n_res=%zu bins=%d\n",
            (int)staged, (int)ctx->gpod_ok, (int)commit, (int)record, (int)need.general, ctx->dc.n_scalar,
            (int)ctx->small_values, (int)f64_exact(ctx->f64_cluster, ctx->f64_pods, n),
            (int)spread_bounds_ok(ctx->gneed, count_total, cell_total, (int)N), (long long)ctx->gneed.ref_weight,
            count_total, cell_total, ctx->gneed.res_rows.size(), ctx->gneed.bins_cap);
  const int w_min = (int)((N + KSS_MAX_NPT * KSS_MAX_THREADS - 1) / (KSS_MAX_NPT * KSS_MAX_THREADS));
  if (split && W < w_min) return fail(KSS_E_UNSUPPORTED, "split grid: too few shards for this cluster");
  W = std::max(W, w_min);
  if (W > 1 && need.xw > XW_MAX && !spread_ok) {
    if (w_min > 1) return fail(KSS_E_UNSUPPORTED, "topology histograms too large for a sharded cluster");
    W = 1;  // exchange payload too large for granules: one workgroup
  }
  if (!split && W > ctx->n_cu) return fail(KSS_E_UNSUPPORTED, "cluster too large for one device");
  if (split && ctx->split_wl > ctx->n_cu) return fail(KSS_E_UNSUPPORTED, "split grid: more shards per part than CUs");
  Geometry g;
  if (!pick_geometry((int)N, W, ctx->pref_threads, g)) return fail(KSS_E_UNSUPPORTED, "no geometry for this cluster");
  const bool simple = simple_ok && simple_fits(g, ctx->dc.n_scalar);
  const int n_res = (int)ctx->gneed.res_rows.size();
  bool spread = spread_ok && spread_fits(g, ctx->gneed, ctx->dc.n_keys, n_res, N, ctx->dc.n_scalar);
  if (spread && !simple && opt(O_THREADS) <= 0 && opt(O_FORCE_THREADS) <= 0) {
    // k_spread: one node per lane where the workgroup allows it (up to KSS_SPREAD_PREF_THREADS):
    // its per-node passes are the chain between exchanges (C4: 256 -> 512 lanes, stats +
    // filter + normalise 4.4 -> 2.6 us per pod)
    Geometry g2;
    if (pick_geometry((int)N, W, KSS_SPREAD_PREF_THREADS, g2) && g2.threads > g.threads &&
        spread_fits(g2, ctx->gneed, ctx->dc.n_keys, n_res, N, ctx->dc.n_scalar))
      g = g2;
  }
  if (split && simple && g.W > 64 * SX_CHUNKS) return fail(KSS_E_UNSUPPORTED, "split grid: k_simple sweeps at most 128 shards");
  if (spread_ok && !spread && g.threads < KSS_MAX_THREADS) {  // more prefetch lanes per shard
    Geometry g2 = g;
    const int per = (int)((N + g.W - 1) / g.W);
    g2.threads = KSS_MAX_THREADS;
    g2.npt = (per + KSS_MAX_THREADS - 1) / KSS_MAX_THREADS;
    if (spread_fits(g2, ctx->gneed, ctx->dc.n_keys, n_res, N, ctx->dc.n_scalar)) {
      g = g2;
      spread = true;
    }
  }
  // more shards when the resident count rows of a shard exceed its LDS (not when the caller
  // fixed the shard count)
  for (int W2 = g.W * 2; spread_ok && !spread && ctx->force_w <= 0 && !split && !(flags & KSS_SCHED_FORCE_SINGLE_WG) &&
                         W2 <= ctx->n_cu && W2 <= (int)N;
       W2 *= 2) {
    Geometry g2;
    if (pick_geometry((int)N, W2, ctx->pref_threads, g2) && spread_fits(g2, ctx->gneed, ctx->dc.n_keys, n_res, N, ctx->dc.n_scalar)) {
      g = g2;
      spread = true;
    }
  }
  if (!spread && g.W > 1 && need.xw > XW_MAX) {  // k_schedule after all: its exchange payload needs one workgroup
    if (w_min > 1) return fail(KSS_E_UNSUPPORTED, "topology histograms too large for a sharded cluster");
    if (!pick_geometry((int)N, 1, ctx->pref_threads, g)) return fail(KSS_E_UNSUPPORTED, "no geometry for this cluster");
  }
  // XCD-local k_spread (launch_spread xcd): the shards on one XCD when they fit its CUs
  bool xcd_spread = false;
  if (spread && !simple && !split && ctx->force_w <= 0 && ctx->xcd_mode && ctx->n_cu % XCD_GRID_MULT == 0 &&
      !(flags & (KSS_SCHED_FORCE_SINGLE_WG | KSS_SCHED_FORCE_MULTI_WG))) {
    const int xw = ctx->xcd_w > 0 ? ctx->xcd_w : xcd_cus;
    Geometry g2;
    if (g.W > 1 && g.W <= xw) {
      xcd_spread = true;
    } else if (g.W > xw && pick_geometry((int)N, xw, KSS_SPREAD_PREF_THREADS, g2) &&
               spread_fits(g2, ctx->gneed, ctx->dc.n_keys, n_res, N, ctx->dc.n_scalar)) {
      g = g2;
      xcd_spread = true;
    }
  }
  const bool loop = simple || spread;  // k_static + a persistent loop kernel
  if (split && !loop)
    return fail(KSS_E_UNSUPPORTED, spread_ok ? "split grid: a k_spread shard exceeds LDS (more shards per part)"
                                             : "split grid: the batch needs k_schedule (kss_plan_podset)");
  const int chunk = loop ? static_chunk(N, n) : 0;
  if (loop && (rc = ctx->stat_buf.ensure(sizeof(uint32_t) * (size_t)chunk * std::max<size_t>(N, 1)))) return rc;
  DevJob job{};
  job.c = ctx->dc;
  job.P = dp;
  job.n_pods = n;
  job.commit = commit ? 1 : 0;
  job.keep_norm = keep_norm ? 1 : 0;
  job.record = record ? 1 : 0;
  job.slots = (uint8_t*)ctx->slot_buf.p;
  job.slot_bytes = SL.bytes;
  job.chosen = (int32_t*)ctx->chosen_buf.p;
  job.meta = (PodMeta*)ctx->meta_buf.p;
  // per-pod calls: error word, outcome and record slot contiguous behind the uploaded image,
  // so the whole read-back is one copy
  const bool one_copy = pu && pu->slot && n == 1 && !chosen_out;
  const size_t pp_err = pu ? pu->extra_off + align_up(sizeof(DevJob), 16) : 0, pp_meta = pp_err + 64;
  if (one_copy) {
    job.meta = (PodMeta*)(pu->dev + pp_meta);
    job.slots = (uint8_t*)pu->slot;
  }
  job.spods = simple ? (const SPod*)ctx->spod_buf.p : nullptr;
  job.stat = loop ? (uint32_t*)ctx->stat_buf.p : nullptr;
  job.gpods = spread ? (const GPod*)ctx->gpod_buf.p : nullptr;
  job.res_rows = spread ? (const int32_t*)ctx->res_buf.p : nullptr;
  job.trace = GTrace{nullptr, nullptr};
  job.cursor = (int32_t*)ctx->cursor_buf.p;
  if (nomq) {
    if (ctx->nom_dirty) {
      if ((rc = ctx->nom_buf.ensure(sizeof(DevNom) * ctx->nom.size()))) return rc;
      HIP_TRY(hipMemcpyAsync(ctx->nom_buf.p, ctx->nom.data(), sizeof(DevNom) * ctx->nom.size(), hipMemcpyHostToDevice,
                             ctx->stream));
      ctx->nom_dirty = false;
    }
    job.nom = (const DevNom*)ctx->nom_buf.p;
    job.n_nom = (int32_t)ctx->nom.size();
  }
  job.pod_base = ctx->run_pod_base;
#if KSS_SPREAD_TRACE
  if (spread) {  // every pod and shard, and the list of nonzero counts loaded / written back
    ctx->trace_words = (size_t)n * (size_t)g.W * G_TW;
    if ((rc = ctx->trace_buf.ensure(4 * ctx->trace_words))) return rc;
    HIP_TRY(dev_zero(ctx->trace_buf.p, 4 * ctx->trace_words, ctx->stream));
    job.trace.words = (int32_t*)ctx->trace_buf.p;
    if ((rc = ctx->trace_list_buf.ensure(4 * (4 + 4 * (size_t)G_TLIST)))) return rc;
    HIP_TRY(dev_zero(ctx->trace_list_buf.p, 16, ctx->stream));
    job.trace.list = (int32_t*)ctx->trace_list_buf.p;
  }
#endif
  job.prof = ctx->prof;
  rc = ctx->job_buf.ensure(sizeof(DevJob));
  if (rc) return rc;
  rc = ctx->err_buf.ensure(16);
  if (rc) return rc;
  unsigned long long* gran = nullptr;
  // k_spread on one part: the two-level exchanges' area behind the granules (launch_spread); a
  // split grid's inbox holds the granules alone
  const size_t gb = sizeof(unsigned long long) *
                    (2 * (size_t)g.W * std::max(2 * XW_MAX, G_XW) + (spread && !split ? tl_words(g.W) : 0));
  unsigned epoch0 = 0;
  SplitRun srun;
  if (split) {  // the local inbox, never cleared: this run's epochs start above every earlier tag
    if (2 * gb > ctx->split_inbox_bytes) return fail(KSS_E_INVAL, "split grid: inbox smaller than the exchange buffer");
    gran = (unsigned long long*)ctx->split_inbox;
    srun.half_words = ctx->split_inbox_bytes / 2 / sizeof(unsigned long long);
    srun.chunk0 = ctx->split_chunks;
    ctx->split_chunks += (unsigned long long)((n + chunk - 1) / std::max(chunk, 1));
    srun.X.n = ctx->split_n;
    srun.X.w_off = ctx->split_part * ctx->split_wl;
    srun.X.wl = ctx->split_wl;
    for (int i = 0; i < ctx->split_n; i++) srun.X.inbox[i] = ctx->split_peer[i];
    srun.epoch0 = ctx->split_epoch;
    const unsigned span = (unsigned)((n + chunk - 1) / std::max(chunk, 1) + 1) * chunk_span(chunk) + 16u;
    if ((uint64_t)ctx->split_epoch + span >= (1ull << 31)) return fail(KSS_E_RANGE, "split grid: granule epochs exhausted");
    ctx->split_epoch += span;
  } else if (g.W > 1) {
    const void* before = ctx->gran_buf.p;
    rc = ctx->gran_buf.ensure(gb);
    if (rc) return rc;
    gran = (unsigned long long*)ctx->gran_buf.p;
    // k_schedule after k_schedule continues the epochs (a stale tag never equals a new epoch);
    // the loop kernels restart theirs, so they, a fresh buffer, or a near-wrap clear it
    const unsigned span = 8u * (unsigned)std::max(n, 1) + 16u;
    const bool reuse = !loop && before == ctx->gran_buf.p && ctx->gran_epoch != 0 &&
                       (uint64_t)ctx->gran_epoch + span < (1ull << 31);
    if (reuse) {
      epoch0 = ctx->gran_epoch;
    } else {
      HIP_TRY(dev_zero(gran, gb, ctx->stream));  // every polled word zeroed
    }
    ctx->gran_epoch = loop ? 0 : epoch0 + span;
  }
  int* errp = (int*)ctx->err_buf.p;
  if (pu) {
    errp = (int*)(pu->dev + pu->extra_off + align_up(sizeof(DevJob), 16));  // zero in the upload image
    std::memset(pu->host + pu->extra_off + align_up(sizeof(DevJob), 16), 0, 16);
  } else {
    HIP_TRY(dev_zero(ctx->err_buf.p, 16, ctx->stream));
  }
  const DevJob* jd = (const DevJob*)ctx->job_buf.p;
  if (pu) {  // the job rides in the per-pod call's single upload
    std::memcpy(pu->host + pu->extra_off, &job, sizeof(DevJob));
    HIP_TRY(hipMemcpyAsync(pu->dev, pu->host, pu->bytes, hipMemcpyHostToDevice, ctx->stream));
    jd = (const DevJob*)(pu->dev + pu->extra_off);
  } else {
    HIP_TRY(hipMemcpyAsync(ctx->job_buf.p, &job, sizeof(DevJob), hipMemcpyHostToDevice, ctx->stream));
  }
  HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
  unsigned long long* stamps = nullptr;
  // k_schedule: shard 0 only; k_simple: every shard (arrival skew of the exchanges)
  const size_t stamp_bytes = sizeof(unsigned long long) * 8 * KSS_NSTAMP_PODS * (loop ? g.W : 1);
  if (ctx->stamps_file) {
    if ((rc = ctx->stamp_buf.ensure(stamp_bytes))) return rc;
    stamps = (unsigned long long*)ctx->stamp_buf.p;
    HIP_TRY(dev_zero(stamps, stamp_bytes, ctx->stream));
  }
  const int n_chunks = loop ? (n + chunk - 1) / std::max(chunk, 1) : 0;
  while ((int)ctx->loop_ev.size() < 2 * n_chunks) {
    hipEvent_t e;
    HIP_TRY(hipEventCreate(&e));
    ctx->loop_ev.push_back(e);
  }
  ctx->last_xcd[0] = (simple && xcd_try && g.W > 1) || xcd_spread ? 1 : 0;
  ctx->last_xcd[1] = 0;
  if (simple)
    rc = launch_simple(ctx->stream, g, 1, jd, ctx->prof, n, (int)N, chunk, gran, gb,
                       errp, stamps, ctx->loop_ev.data(), split ? &srun : nullptr, ctx->dc.n_scalar, ctx->last_xcd[0] != 0,
                       &ctx->last_xcd[1], ctx->dc.n_keys, nullptr, nullptr, k_find < (int)N ? k_find : 0);
  else if (spread)
  {
    const HandoffLayout hl(g.W, n_res, (int)N, ctx->dc.n_scalar);
    if ((rc = ctx->ck_buf.ensure(sizeof(unsigned long long) * hl.words))) return rc;
    HIP_TRY(dev_zero((unsigned long long*)ctx->ck_buf.p + hl.o_diag, sizeof(unsigned long long), ctx->stream));
    ctx->ck_diag_off = hl.o_diag;
    // the window's count exchange: W SUM values behind the pod's bins, one scalar
    GpodNeeds qw = ctx->gneed;
    if (spread_win) {
      qw.bins_cap += g.W;
      qw.xw = std::max(qw.xw, g.W + 1);
    }
    rc = launch_spread(ctx->stream, g, qw, ctx->dc.n_keys, n_res, jd, ctx->prof, n,
                       (int)N, chunk, gran, gb, errp, stamps, ctx->loop_ev.data(), split ? &srun : nullptr,
                       (unsigned long long*)ctx->ck_buf.p, &ctx->ck_seq, ctx->dc.n_scalar, xcd_spread, &ctx->last_xcd[1],
                       spread_win ? k_find : 0);
  }
  else  // window: the per-shard feasible counts sit behind the plan's bins
    rc = launch_schedule(ctx->stream, g, 1, std::max(need.bins_cap, 0) + (window ? g.W : 0), need.general, ctx->dc.n_keys,
                         jd, ctx->prof, gran, errp, stamps, epoch0);
  if (rc) return rc;
  ctx->last_kernel = simple ? 1 : (spread ? 2 : 0);
  HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
  // diagnostic stamps -> KSS_STAMPS_FILE, one record per launch: {kernel (0 k_schedule,
  // 1 k_simple, 2 k_spread), shards} then the stamps
  auto dump_stamps = [&]() -> int {
    if (!stamps) return 0;
    std::vector<unsigned long long> h(2 + stamp_bytes / 8);
    h[0] = simple ? 1 : (spread ? 2 : 0);
    h[1] = loop ? (unsigned long long)g.W : 1;
    HIP_TRY(hipMemcpy(h.data() + 2, stamps, stamp_bytes, hipMemcpyDeviceToHost));
    if (FILE* f = fopen(ctx->stamps_file, "ab")) {
      fwrite(h.data(), 8, h.size(), f);
      fclose(f);
    }
    return 0;
  };
  if (one_copy) {  // [error word .. outcome .. record slot up to the requested span]: one copy, one sync
    const size_t span = (size_t)(pu->slot - (pu->dev + pp_err)) + (rbk ? rbk->bytes : 0);
    if ((rc = ensure_pinned(ctx->rb, ctx->rb_cap, span))) return rc;
    char* hb = (char*)ctx->rb;
    HIP_TRY(hipMemcpyAsync(hb, pu->dev + pp_err, span, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->last_ms = ctx->last_loop_ms = ms;
    ctx->last_launches = 1;
    ctx->last_geom[0] = g.W;
    ctx->last_geom[1] = g.threads;
    ctx->last_geom[2] = g.npt;
    int errw = 0;
    std::memcpy(&errw, hb, sizeof(int));
    if (errw) return fail(KSS_E_DEVICE, "shard exchange timed out (workgroups not co-resident?)");
    ctx->meta_host.resize(1);
    std::memcpy(ctx->meta_host.data(), hb + (pp_meta - pp_err), sizeof(PodMeta));
    if (rbk) rbk->host = hb + (pu->slot - (pu->dev + pp_err));
    ctx->recorded = 0;  // the record went to the caller; kss_fetch_record has nothing to serve
    ctx->meta_n = 1;
    ctx->axis_meta_dirty = false;
    return dump_stamps();
  }
  // every read-back of the launch into one pinned staging, then one synchronisation
  const size_t mb = sizeof(PodMeta) * (size_t)std::max(n, 1), cb = chosen_out && n ? sizeof(int32_t) * (size_t)n : 0;
  const size_t o_meta = 16, o_chosen = align_up(o_meta + mb, 16), o_rb = align_up(o_chosen + cb, 16);
  if ((rc = ensure_pinned(ctx->rb, ctx->rb_cap, o_rb + (rbk ? rbk->bytes : 0)))) return rc;
  char* hb = (char*)ctx->rb;
  HIP_TRY(hipMemcpyAsync(hb, errp, 4 * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipMemcpyAsync(hb + o_meta, ctx->meta_buf.p, mb, hipMemcpyDeviceToHost, ctx->stream));
  if (cb) HIP_TRY(hipMemcpyAsync(hb + o_chosen, ctx->chosen_buf.p, cb, hipMemcpyDeviceToHost, ctx->stream));
  if (rbk && rbk->bytes) HIP_TRY(hipMemcpyAsync(hb + o_rb, rbk->src, rbk->bytes, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  if (rbk) rbk->host = hb + o_rb;
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  ctx->last_ms = ms;
  ctx->last_launches = loop ? 2 * n_chunks : 1;
  ctx->last_loop_ms = loop ? 0.0 : ms;
  for (int i = 0; i < n_chunks; i++) {
    float t = 0;
    HIP_TRY(hipEventElapsedTime(&t, ctx->loop_ev[2 * i], ctx->loop_ev[2 * i + 1]));
    ctx->last_loop_ms += t;
  }
  ctx->last_geom[0] = g.W;
  ctx->last_geom[1] = g.threads;
  ctx->last_geom[2] = g.npt;
  int errw = 0;
  std::memcpy(&errw, hb, sizeof(int));
  std::memcpy(&ctx->last_handoff_retries, hb + sizeof(int), sizeof(int));
  std::memcpy(&ctx->last_handoff_recovered, hb + 2 * sizeof(int), sizeof(int));
  std::memcpy(&ctx->last_handoff_final, hb + 3 * sizeof(int), sizeof(int));
  ctx->last_kernel_spread = spread;
  if (errw && commit) {  // bounds as if every pod committed (upper bounds stay safe); log unknown
    ctx->count_bound = count_total;
    ctx->cell_bound = std::max(ctx->cell_bound, cell_total);
    ctx->state_unknown = true;
  }
  if (errw == 2)
    return fail(KSS_E_DEVICE, ctx->last_handoff_final ? "the last chunk's node-state write-back failed its final check"
                                                       : "node state handed between chunk launches failed its check");
  if (errw) return fail(KSS_E_DEVICE, "shard exchange timed out (workgroups not co-resident?)");
  if (commit) {
    ctx->count_bound = count_total;
    ctx->cell_bound = std::max(ctx->cell_bound, cell_total);
  }
  ctx->meta_host.resize((size_t)std::max(n, 1));
  std::memcpy(ctx->meta_host.data(), hb + o_meta, mb);
  if (cb) std::memcpy(chosen_out, hb + o_chosen, cb);
  ctx->recorded = record ? n : (n > 0 && !loop ? 1 : 0);
  ctx->meta_n = n;
  ctx->axis_meta_dirty = false;
  return dump_stamps();
}

// compact records (k_simple) or resolved programs (k_spread) of the staged podset (host copy
// kept alive for the async upload)
static int stage_spods(kss_ctx* ctx, const kss_podset* ps) {
  ctx->f64_pods = F64Bounds{};
  f64_bounds_pods(ps, ctx->f64_pods);
  ctx->staged_max_own = 0;
  ctx->staged_names = false;
  for (int i = 0; i < ps->n_pods; i++) {
    ctx->staged_max_own = std::max(ctx->staged_max_own, (int)ps->pods[i].own_terms_len);
    ctx->staged_names |= ps->pods[i].names_len >= 0;
  }
  ctx->spod_ok = build_spods(ps, ctx->dc.n_scalar, ctx->spod_host);
  ctx->gpod_ok = false;
  if (!ctx->spod_ok) {  // programs: the resolved records of k_spread
    ctx->gpod_ok = build_gpods(ps, ctx->dc.n_scalar, ctx->dc.n_classes, ctx->key_card_h.data(), ctx->key_flags_h.data(),
                               ctx->key_empty_h.data(), ctx->gpod_host, ctx->gneed);
    if (!ctx->gpod_ok) return 0;
    int rc = ctx->gpod_buf.ensure(sizeof(uint4) * ctx->gpod_host.size());
    if (rc) return rc;
    if ((rc = ctx->res_buf.ensure(sizeof(int32_t) * std::max<size_t>(ctx->gneed.res_rows.size(), 1)))) return rc;
    if (!ctx->gneed.res_rows.empty())
      HIP_TRY(hipMemcpyAsync(ctx->res_buf.p, ctx->gneed.res_rows.data(), sizeof(int32_t) * ctx->gneed.res_rows.size(),
                             hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(ctx->gpod_buf.p, ctx->gpod_host.data(), sizeof(uint4) * ctx->gpod_host.size(),
                           hipMemcpyHostToDevice, ctx->stream));
    return 0;
  }
  int rc = ctx->spod_buf.ensure(sizeof(SPod) * ctx->spod_host.size());
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(ctx->spod_buf.p, ctx->spod_host.data(), sizeof(SPod) * ctx->spod_host.size(),
                         hipMemcpyHostToDevice, ctx->stream));
  return 0;
}

// One record slot to the caller's arrays: the span of the requested fields in one D2H copy
// through pinned staging (the slot is contiguous: SlotLayout), then host copies.
// The byte range [lo, hi) of a slot that a result's requested arrays cover.
struct SlotRange {
  size_t lo, hi;
};

static SlotRange slot_range_fields(size_t N, uint32_t fields) {
  const SlotLayout SL(N);
  const uint32_t bit[5] = {KSS_FIELD_FAIL, KSS_FIELD_DETAIL, KSS_FIELD_RAW, KSS_FIELD_NORM, KSS_FIELD_TOTAL};
  const size_t off[5] = {SL.fail, SL.detail, SL.raw, SL.norm, SL.total};
  const size_t bytes[5] = {N, 2 * N, 8 * KSS_NSCORE * N, 8 * KSS_NSCORE * N, 8 * N};
  SlotRange r{SL.bytes, 0};
  for (int i = 0; i < 5; i++)
    if ((fields & bit[i]) && bytes[i]) {
      r.lo = std::min(r.lo, off[i]);
      r.hi = std::max(r.hi, off[i] + bytes[i]);
    }
  return r;
}

static SlotRange slot_range(size_t N, const kss_pod_result* out) {
  return slot_range_fields(N, (out->fail_plugin ? KSS_FIELD_FAIL : 0u) | (out->fail_detail ? KSS_FIELD_DETAIL : 0u) |
                                  (out->raw ? KSS_FIELD_RAW : 0u) | (out->norm ? KSS_FIELD_NORM : 0u) |
                                  (out->total ? KSS_FIELD_TOTAL : 0u));
}

// slot bytes [r.lo, r.hi) at `src` (host) -> the result's arrays, plus the pod's outcome
static int scatter_slot(size_t N, const SlotRange& r, const char* src, const PodMeta& m, kss_pod_result* out) {
  const SlotLayout SL(N);
  void* dst[5] = {out->fail_plugin, out->fail_detail, out->raw, out->norm, out->total};
  const size_t off[5] = {SL.fail, SL.detail, SL.raw, SL.norm, SL.total};
  const size_t bytes[5] = {N, 2 * N, 8 * KSS_NSCORE * N, 8 * KSS_NSCORE * N, 8 * N};
  if (r.hi > r.lo)
    for (int i = 0; i < 5; i++)
      if (dst[i] && bytes[i]) std::memcpy(dst[i], src + (off[i] - r.lo), bytes[i]);
  out->n_feasible = m.n_feasible;
  out->chosen = m.chosen;
  out->best_total = m.best_total;
  out->scored = m.scored;
  out->status = m.status;
  if (m.status == 4) return fail(KSS_E_UNSUPPORTED, "pod program exceeds the device path's per-pod limits");
  return 0;
}

// One recorded slot -> the caller's arrays: only the requested span, in one copy through
// pinned staging (the slot is contiguous: SlotLayout), then host copies.
static int copy_slot(kss_ctx* ctx, int slot, const PodMeta& m, kss_pod_result* out) {
  const size_t N = (size_t)ctx->dc.N;
  const SlotLayout SL(N);
  const char* base = (const char*)ctx->slot_buf.p + (size_t)slot * SL.bytes;
  const SlotRange r = slot_range(N, out);
  if (r.hi > r.lo) {
    if (int rc = ensure_pinned(ctx->pinned, ctx->pinned_cap, r.hi - r.lo)) return rc;
    HIP_TRY(hipMemcpyAsync(ctx->pinned, base + r.lo, r.hi - r.lo, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
  }
  return scatter_slot(N, r, (const char*)ctx->pinned, m, out);
}

// One pod of a podset with its own compact pools (every pool reference remapped): the
// per-pod calls upload and validate only what that pod references.
struct OnePod {
  kss_pod pod{};
  std::vector<kss_req> reqs;
  std::vector<kss_term> terms;
  std::vector<kss_spread> spreads;
  std::vector<kss_ipa> ipa;
  std::vector<int32_t> ints;
  std::vector<kss_vol> vols;
  kss_podset ps{};
};

static int compact_pod(const kss_podset* ps, int i, OnePod& o) {
  const kss_pod& p = ps->pods[i];
  auto in = [](int64_t off, int64_t len, int64_t cap) { return off >= 0 && len >= 0 && off + len <= cap; };
  if (!in(p.sel_off, p.sel_len, ps->n_reqs) || !in(p.aff_off, p.aff_len, ps->n_terms) ||
      !in(p.pref_off, p.pref_len, ps->n_terms) || !in(p.spread_off, (int64_t)p.n_hard + p.n_soft, ps->n_spreads) ||
      !in(p.ipa_off, p.ipa_len, ps->n_ipa) || !in(p.own_terms_off, p.own_terms_len, ps->n_ints) ||
      (p.names_len >= 0 && !in(p.names_off, p.names_len, ps->n_ints)) ||
      (p.img_len > 0 && !in(p.img_off, p.img_len, ps->n_ints)) || !in(p.vol_off, p.vol_len, ps->n_vols))
    return fail(KSS_E_INVAL, "pod program out of range");
  o = OnePod{};
  o.pod = p;
  auto list = [&](int off, int len) -> int32_t {
    const int32_t at = (int32_t)o.ints.size();
    if (in(off, len, ps->n_ints)) o.ints.insert(o.ints.end(), ps->ints + off, ps->ints + off + len);
    return at;
  };
  auto req = [&](const kss_req& r) {
    kss_req q = r;
    if (r.op == KSS_OP_IN || r.op == KSS_OP_NOTIN) q.list_off = list(r.list_off, r.list_len);
    o.reqs.push_back(q);
  };
  auto term = [&](const kss_term& t) -> bool {
    if (!in(t.req_off, t.req_len, ps->n_reqs)) return false;
    kss_term u = t;
    u.req_off = (int32_t)o.reqs.size();
    for (int k = 0; k < t.req_len; k++) req(ps->reqs[t.req_off + k]);
    o.terms.push_back(u);
    return true;
  };
  o.pod.sel_off = 0;
  for (int k = 0; k < p.sel_len; k++) req(ps->reqs[p.sel_off + k]);
  // the terms of the pod are contiguous: aff then pref; each term's requirements contiguous
  o.pod.aff_off = 0;
  for (int t = 0; t < p.aff_len; t++)
    if (!term(ps->terms[p.aff_off + t])) return fail(KSS_E_INVAL, "term out of range");
  o.pod.pref_off = (int32_t)o.terms.size();
  for (int t = 0; t < p.pref_len; t++)
    if (!term(ps->terms[p.pref_off + t])) return fail(KSS_E_INVAL, "term out of range");
  o.pod.spread_off = 0;
  for (int c = 0; c < p.n_hard + p.n_soft; c++) {
    kss_spread sp = ps->spreads[p.spread_off + c];
    sp.cls_off = list(sp.cls_off, sp.cls_len);
    o.spreads.push_back(sp);
  }
  o.pod.ipa_off = 0;
  for (int e = 0; e < p.ipa_len; e++) {
    kss_ipa en = ps->ipa[p.ipa_off + e];
    en.row_off = list(en.row_off, en.row_len);
    o.ipa.push_back(en);
  }
  o.pod.own_terms_off = list(p.own_terms_off, p.own_terms_len);
  if (p.names_len >= 0) o.pod.names_off = list(p.names_off, p.names_len);
  if (p.img_len > 0) o.pod.img_off = list(p.img_off, p.img_len);
  // the volume program: VolumeBinding terms and VolumeZone requirements follow into the
  // pod's own pools; rows and keys are the cluster's
  o.pod.vol_off = 0;
  for (int e = 0; e < p.vol_len; e++) {
    kss_vol v = ps->vols[p.vol_off + e];
    if (v.kind == KSS_VOL_BIND_AFFINITY) {
      if (!in(v.a, v.b, ps->n_terms)) return fail(KSS_E_INVAL, "volume node affinity terms out of range");
      const int32_t at = (int32_t)o.terms.size();
      for (int t = 0; t < v.b; t++)
        if (!term(ps->terms[v.a + t])) return fail(KSS_E_INVAL, "term out of range");
      v.a = at;
    } else if (v.kind == KSS_VOL_ZONE) {
      if (!in(v.a, v.b, ps->n_reqs)) return fail(KSS_E_INVAL, "volume zone requirements out of range");
      const int32_t at = (int32_t)o.reqs.size();
      for (int k = 0; k < v.b; k++) req(ps->reqs[v.a + k]);
      v.a = at;
    } else if (v.kind == KSS_VOL_BIND_WFFC) {  // candidate triplets and their terms, the class's topology terms
      if (v.b < 0 || v.count < 0 || !in(v.a, 3 * (int64_t)v.b, ps->n_ints) || !in(v.row, v.count >> 1, ps->n_terms))
        return fail(KSS_E_INVAL, "WaitForFirstConsumer claim entry out of range");
      std::vector<int32_t> trip(ps->ints + v.a, ps->ints + v.a + 3 * (size_t)v.b);
      for (int j = 0; j < v.b; j++) {
        const int32_t ta = trip[3 * j + 1], tb = trip[3 * j + 2];
        if (tb < 0) continue;
        if (!in(ta, tb, ps->n_terms)) return fail(KSS_E_INVAL, "WaitForFirstConsumer candidate out of range");
        trip[3 * j + 1] = (int32_t)o.terms.size();
        for (int t = 0; t < tb; t++)
          if (!term(ps->terms[ta + t])) return fail(KSS_E_INVAL, "term out of range");
      }
      const int32_t at = (int32_t)o.terms.size();
      for (int t = 0; t < (v.count >> 1); t++)
        if (!term(ps->terms[v.row + t])) return fail(KSS_E_INVAL, "term out of range");
      v.row = at;
      v.a = (int32_t)o.ints.size();
      o.ints.insert(o.ints.end(), trip.begin(), trip.end());
    }
    o.vols.push_back(v);
  }
  o.ps.n_pods = 1;  // empty pools stay empty (upload_podset sizes them; validate skips them)
  o.ps.n_reqs = (int32_t)o.reqs.size();
  o.ps.n_terms = (int32_t)o.terms.size();
  o.ps.n_spreads = (int32_t)o.spreads.size();
  o.ps.n_ipa = (int32_t)o.ipa.size();
  o.ps.n_ints = (int32_t)o.ints.size();
  o.ps.n_vols = (int32_t)o.vols.size();
  o.ps.vols = o.vols.data();
  o.ps.pods = &o.pod;
  o.ps.reqs = o.reqs.data();
  o.ps.terms = o.terms.data();
  o.ps.spreads = o.spreads.data();
  o.ps.ipa = o.ipa.data();
  o.ps.ints = o.ints.data();
  return 0;
}

// kss_eval_pod's device work: the pod's own program uploaded with the job, one launch, and
// slot bytes [0, r.hi) read back in the same copy as the error word and the outcome
// (rbk.host: the slot in the pinned staging).
static int eval_pod_slot(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, const SlotRange& r, ReadBack& rbk) {
  if (!ctx || !ctx->loaded || !ps) return fail(KSS_E_INVAL, "bad arguments");
  if (pod_index < 0 || pod_index >= ps->n_pods) return fail(KSS_E_INVAL, "pod index out of range");
  nom_check_podset(ctx, ps);
  OnePod one;
  int rc = compact_pod(ps, pod_index, one);
  if (rc) return rc;
  if ((rc = validate(&ctx->host, &one.ps, 1))) return rc;
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  const size_t N = (size_t)ctx->dc.N;
  PackedUpload pu;
  pu.tail = SlotLayout(N).bytes;  // the record slot lives right behind the image (one read-back)
  // extra: the job, then the error word (zeroed by the upload) and the outcome (64 B further)
  rc = pack_podset(ctx->tmp_pod_buf, ctx->up, ctx->up_cap, &one.ps, align_up(sizeof(DevJob), 16) + 64 + sizeof(PodMeta),
                   ctx->tdp, pu);
  if (rc) return rc;
  const PlanNeeds need = plan_needs(ctx->key_card_h.data(), ctx->key_flags_h.data(), &one.ps, 1);
  rbk.bytes = r.hi > r.lo ? r.hi : 0;  // slot bytes [0, r.hi) ride in the one copy
  ctx->run_pod_base = pod_index;  // the uploaded pod is pod_index of the caller's podset (nominator identity)
  rc = run_single(ctx, need, ctx->tdp, 1, /*commit=*/false, /*record=*/false, /*keep_norm=*/true, 0, nullptr,
                  /*staged=*/false, &rbk, &pu);
  ctx->run_pod_base = 0;
  return rc;
}

int kss_eval_pod(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, kss_pod_result* out) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !out) return fail(KSS_E_INVAL, "bad arguments");
  std::lock_guard<std::mutex> lk(ctx->mu);
  const size_t N = (size_t)ctx->dc.N;
  const SlotRange r = slot_range(N, out);
  ReadBack rbk;
  if (int rc = eval_pod_slot(ctx, ps, pod_index, r, rbk)) return rc;
  return scatter_slot(N, r, r.hi > r.lo ? rbk.host + r.lo : nullptr, ctx->meta_host[0], out);
}

int kss_eval_pod_view(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, uint32_t fields, kss_pod_view* out) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !out) return fail(KSS_E_INVAL, "bad arguments");
  std::lock_guard<std::mutex> lk(ctx->mu);
  const size_t N = (size_t)ctx->dc.N;
  const SlotLayout SL(N);
  const SlotRange r = slot_range_fields(N, fields);
  ReadBack rbk;
  if (int rc = eval_pod_slot(ctx, ps, pod_index, r, rbk)) return rc;
  const char* b = r.hi > r.lo ? rbk.host : nullptr;  // the slot in the pinned staging
  out->fail_plugin = b && (fields & KSS_FIELD_FAIL) ? (const uint8_t*)(b + SL.fail) : nullptr;
  out->fail_detail = b && (fields & KSS_FIELD_DETAIL) ? (const uint16_t*)(b + SL.detail) : nullptr;
  out->raw = b && (fields & KSS_FIELD_RAW) ? (const int64_t*)(b + SL.raw) : nullptr;
  out->norm = b && (fields & KSS_FIELD_NORM) ? (const int64_t*)(b + SL.norm) : nullptr;
  out->total = b && (fields & KSS_FIELD_TOTAL) ? (const int64_t*)(b + SL.total) : nullptr;
  const PodMeta& m = ctx->meta_host[0];
  out->n_feasible = m.n_feasible;
  out->chosen = m.chosen;
  out->best_total = m.best_total;
  out->scored = m.scored;
  out->status = m.status;
  if (m.status == 4) return fail(KSS_E_UNSUPPORTED, "pod program exceeds the device path's per-pod limits");
  return 0;
}

// A pending pod as a bound pod of the PostFilter table once committed (id -1 - index,
// status.startTime unset: it has not started).
static BoundPod bound_from_pod(const kss_podset* ps, int i) {
  const kss_pod& p = ps->pods[i];
  BoundPod b{};
  b.id = -1 - (int64_t)i;
  b.start = KSS_START_UNSET;
  for (int r = 0; r < KSS_NRES; r++) b.req[r] = p.commit_req[r];
  b.nz[0] = p.commit_nz[0];
  b.nz[1] = p.commit_nz[1];
  b.ports = p.port_add;
  b.has_nz = 1;
  b.has_vols = p.vol_len > 0 ? 1 : 0;
  b.prio = p.priority;
  b.cls = p.cls;
  b.tlen = std::min(p.own_terms_len, 8);
  for (int t = 0; t < b.tlen; t++) b.terms[t] = ps->ints[p.own_terms_off + t];
  return b;
}

static void stage_bound(kss_ctx* ctx, const kss_podset* ps) {
  ctx->staged_bp.resize(ps->n_pods);
  ctx->staged_uid.resize(ps->n_pods);
  for (int i = 0; i < ps->n_pods; i++) {
    ctx->staged_bp[i] = bound_from_pod(ps, i);
    ctx->staged_uid[i] = pod_identity(ps->pods[i], i);
  }
}

// SchedulingQueue.DeleteNominatedPodIfExists for every assumed pod of a batch (the device did the
// same for its own copy as it went)
static void drop_committed_nominations(kss_ctx* ctx, int n) {
  if (ctx->nom.empty()) return;
  const size_t before = ctx->nom.size();
  ctx->nom.erase(std::remove_if(ctx->nom.begin(), ctx->nom.end(),
                                [&](const DevNom& e) {
                                  for (int i = 0; i < n && i < (int)ctx->staged_uid.size(); i++)
                                    if (ctx->staged_uid[i] == e.pod && ctx->meta_host[i].chosen >= 0) return true;
                                  return false;
                                }),
                 ctx->nom.end());
  if (ctx->nom.size() != before) ctx->nom_dirty = true;
}

// the batch's AssumePods, as NodeInfo.AddPod appends them
static void log_batch_commits(kss_ctx* ctx, int n) {
  drop_committed_nominations(ctx, n);
  for (int i = 0; i < n && i < (int)ctx->staged_bp.size(); i++) {
    const int local = ctx->meta_host[i].chosen - ctx->dc.node_base;
    if (local >= 0 && local < ctx->dc.N) ctx->bound_log.push_back(BoundOp{local, 1, ctx->staged_bp[i]});
  }
  ctx->bound_dirty = true;
}

// AssumePod (sign 1) / ForgetPod (-1) of ps.pods[pod_index] on a node: the deltas travel in
// the kernel's arguments.
static int commit_one(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, int32_t node, int sign) {
  if (!ctx || !ctx->loaded || !ps) return fail(KSS_E_INVAL, "bad arguments");
  if (pod_index < 0 || pod_index >= ps->n_pods) return fail(KSS_E_INVAL, "pod index out of range");
  const int local = node - ctx->dc.node_base;
  if (local < 0 || local >= ctx->dc.N) return fail(KSS_E_INVAL, "node out of range");
  const kss_pod& p = ps->pods[pod_index];
  if (p.cls >= ctx->host.n_classes) return fail(KSS_E_INVAL, "pod class out of range");
  if (p.own_terms_len < 0 || p.own_terms_off < 0 || p.own_terms_off + p.own_terms_len > ps->n_ints)
    return fail(KSS_E_INVAL, "own terms out of range");
  if (p.own_terms_len > 8) return fail(KSS_E_UNSUPPORTED, "more than 8 own term rows");
  CommitArgs a{};
  for (int r = 0; r < KSS_NRES; r++) a.req[r] = p.commit_req[r];
  a.nz[0] = p.commit_nz[0];
  a.nz[1] = p.commit_nz[1];
  a.port_add = p.port_add;
  if (ctx->host.n_ports < KSS_MAX_PORTS && (p.port_add >> ctx->host.n_ports))
    return fail(KSS_E_INVAL, "pod port bit outside the port dictionary");
  a.cls = p.cls;
  a.n_own = p.own_terms_len;
  for (int i = 0; i < p.own_terms_len; i++) {
    a.own[i] = ps->ints[p.own_terms_off + i];
    if (a.own[i] < 0 || a.own[i] >= ctx->host.n_terms) return fail(KSS_E_INVAL, "own term id out of range");
  }
  if (p.vol_off < 0 || p.vol_len < 0 || p.vol_off + p.vol_len > ps->n_vols) return fail(KSS_E_INVAL, "pod volume program out of range");
  for (int e = 0; e < p.vol_len; e++) {
    const kss_vol& v = ps->vols[p.vol_off + e];
    if (v.kind == KSS_VOL_OWN) {
      if (a.n_vrow == 8) return fail(KSS_E_UNSUPPORTED, "more than 8 own volume rows");
      if (v.row < 0 || v.row >= ctx->host.n_vol_rows) return fail(KSS_E_INVAL, "volume row out of range");
      a.vrow[a.n_vrow++] = v.row;
    } else if (v.kind == KSS_VOL_OWN_PRIVATE) {
      if (a.n_vpriv == 4) return fail(KSS_E_UNSUPPORTED, "more than 4 attach-limit keys");
      if (v.key < 0 || v.key >= ctx->host.n_vol_keys || v.count < 0) return fail(KSS_E_INVAL, "volume key out of range");
      a.vpriv_key[a.n_vpriv] = v.key;
      a.vpriv_cnt[a.n_vpriv++] = v.count;
    }
  }
  a.local = local;
  a.sign = sign;
  std::lock_guard<std::mutex> lk(ctx->mu);
  nom_check_podset(ctx, ps);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  if (sign > 0) {
    ctx->count_bound += 1.0 + (double)p.own_terms_len;
    ctx->cell_bound += 1.0 + (double)p.own_terms_len;
  }
  hipLaunchKernelGGL(k_commit, dim3(1), dim3(64), 0, ctx->stream, ctx->dc, a);
  HIP_TRY(hipGetLastError());  // no synchronisation: every later call on the ctx stream is ordered after it
  bool wffc = false;
  for (int e = 0; e < p.vol_len; e++) wffc |= ps->vols[p.vol_off + e].kind == KSS_VOL_BIND_WFFC;
  if (wffc) {  // AssumePodVolumes / RevertAssumedPodVolumes on the device (the assume cache lives there)
    OnePod one;
    if (int rc = compact_pod(ps, pod_index, one)) return rc;
    DevPods dpw{};
    if (int rc = upload_podset(ctx->stream, ctx->wffc_pod_buf, &one.ps, dpw)) return rc;
    hipLaunchKernelGGL(k_wffc_commit, dim3(1), dim3(64), 0, ctx->stream, ctx->dc, dpw, local, sign);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(ctx->stream));  // `one` (the upload's host source) goes out of scope
  }
  if (sign > 0) {  // assume -> SchedulingQueue.DeleteNominatedPodIfExists
    const size_t before = ctx->nom.size();
    const int32_t id = pod_identity(p, pod_index);
    ctx->nom.erase(std::remove_if(ctx->nom.begin(), ctx->nom.end(), [&](const DevNom& e) { return e.pod == id; }),
                   ctx->nom.end());
    if (ctx->nom.size() != before) ctx->nom_dirty = true;
  }
  ctx->bound_log.push_back(BoundOp{local, sign > 0 ? 1 : 0, bound_from_pod(ps, pod_index)});
  ctx->bound_dirty = true;
  return 0;
}

int kss_commit(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, int32_t node) {
  KSS_SVC_QUIESCE(ctx);
  return commit_one(ctx, ps, pod_index, node, 1);
}

int kss_rollback(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, int32_t node) {
  KSS_SVC_QUIESCE(ctx);
  return commit_one(ctx, ps, pod_index, node, -1);
}

int kss_schedule_batch(kss_ctx* ctx, const kss_podset* ps, int32_t n, uint32_t flags, int32_t* chosen_out) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded || !ps) return fail(KSS_E_INVAL, "bad arguments");
  if (n < 0 || n > ps->n_pods) return fail(KSS_E_INVAL, "pod count out of range");
  // every pod is staged (and may be run later by kss_run_staged / the node axis): all of
  // them are validated, not only the first n
  int rc = validate(&ctx->host, ps, ps->n_pods);
  if (rc) return rc;
  const bool record = (flags & KSS_SCHED_RECORD) != 0;
  if (record && n > ctx->cfg.max_pods_record) return fail(KSS_E_INVAL, "record capacity (max_pods_record) exceeded");
  std::lock_guard<std::mutex> lk(ctx->mu);
  nom_check_podset(ctx, ps);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  rc = upload_podset(ctx->stream, ctx->pod_buf, ps, ctx->dp);
  if (rc) return rc;
  if ((rc = stage_spods(ctx, ps))) return rc;
  stage_bound(ctx, ps);
  ctx->staged_n = ps->n_pods;
  ctx->staged_need = plan_needs(ctx->key_card_h.data(), ctx->key_flags_h.data(), ps, ps->n_pods);
  rc = run_single(ctx, ctx->staged_need, ctx->dp, n, /*commit=*/true, record, /*keep_norm=*/record, flags, chosen_out,
                  /*staged=*/true);
  if (rc) return rc;
  log_batch_commits(ctx, n);
  for (int i = 0; i < n; i++)
    if (ctx->meta_host[i].status == 4) return fail(KSS_E_UNSUPPORTED, "pod program exceeds the device path's per-pod limits");
  return 0;
}

int kss_stage_pods(kss_ctx* ctx, const kss_podset* ps) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded || !ps) return fail(KSS_E_INVAL, "bad arguments");
  int rc = validate(&ctx->host, ps, ps->n_pods);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(ctx->mu);
  nom_check_podset(ctx, ps);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  rc = upload_podset(ctx->stream, ctx->pod_buf, ps, ctx->dp);
  if (rc) return rc;
  if ((rc = stage_spods(ctx, ps))) return rc;
  stage_bound(ctx, ps);
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  ctx->staged_n = ps->n_pods;
  ctx->staged_need = plan_needs(ctx->key_card_h.data(), ctx->key_flags_h.data(), ps, ps->n_pods);
  return 0;
}

int kss_run_staged(kss_ctx* ctx, int32_t n, uint32_t flags, int32_t* chosen_out) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  if (n < 0 || n > ctx->staged_n) return fail(KSS_E_INVAL, "n exceeds the staged pods");
  const bool record = (flags & KSS_SCHED_RECORD) != 0;
  if (record && n > ctx->cfg.max_pods_record) return fail(KSS_E_INVAL, "record capacity (max_pods_record) exceeded");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  int rc = run_single(ctx, ctx->staged_need, ctx->dp, n, /*commit=*/true, record, /*keep_norm=*/record, flags, chosen_out,
                      /*staged=*/true);
  if (rc) return rc;
  log_batch_commits(ctx, n);
  for (int i = 0; i < n; i++)
    if (ctx->meta_host[i].status == 4) return fail(KSS_E_UNSUPPORTED, "pod program exceeds the device path's per-pod limits");
  return 0;
}

// ---------------------------------------------------------------------------
// the per-pod service grid (kss_service_*): host side (kernel: kss_service.cuh)
// ---------------------------------------------------------------------------
static void svc_free_rec(kss_ctx::Service& v) {
  if (v.rec && v.rec_map) {
    hipHostUnregister(v.rec);
    munmap(v.rec_map, v.rec_map_bytes);
  } else if (v.rec) {
    hipHostFree(v.rec);
  }
  v.rec = nullptr;
  v.rec_map = nullptr;
  v.rec_map_bytes = 0;
  v.rec_bytes = 0;
}

static void svc_free(kss_ctx* ctx) {
  auto& v = ctx->svc;
  if (v.box) hipHostFree(v.box);
  svc_free_rec(v);
  if (v.stream) hipStreamDestroy(v.stream);
  v.relay.release();
  v.stat.release();
  v.gran.release();
  v.err.release();
  v.job.release();
  v = kss_ctx::Service{};
}

static bool svc_alive(kss_ctx* ctx) {
  return ctx->svc.running && hipStreamQuery(ctx->svc.stream) == hipErrorNotReady;
}

// (Re)launch the grid at the first command shard 0 has not relayed yet.
static int svc_launch(kss_ctx* ctx) {
  auto& v = ctx->svc;
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  const unsigned long long seq0 = __atomic_load_n(&v.box->consumed, __ATOMIC_ACQUIRE);
  const size_t relay_bytes = sizeof(unsigned long long) * 2 * SVC_DRING;
  HIP_TRY(dev_zero(v.relay.p, relay_bytes, v.stream));
  std::vector<unsigned long long> seen((size_t)v.W, seq0);  // the relay throttle starts from here
  HIP_TRY(hipMemcpyAsync((char*)v.relay.p + relay_bytes, seen.data(), 8 * seen.size(), hipMemcpyHostToDevice, v.stream));
  if (v.W > 1) HIP_TRY(dev_zero(v.gran.p, v.gran.cap, v.stream));  // epochs restart at 0
  HIP_TRY(dev_zero(v.err.p, 16, v.stream));  // the error word and xcd_slot's two counters
  v.box->err = 0;
  v.box->xcd_fail = 0;
  const bool inl = opt(O_SVC_INLINE_SWEEP) != 0;
  const void* fn = v.gen ? (const void*)k_service<true, false>
                         : (v.simple ? (inl ? (const void*)k_service<false, true, true> : (const void*)k_service<false, true>)
                                     : (const void*)k_service<false, false>);
  HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)v.shmem));
  const DevJob* jd = (const DevJob*)v.job.p;
  kss_profile pr = ctx->prof;
  int W = v.W, npt = v.npt, bins = v.bins_cap, ck = v.cache_keys;
  unsigned long long* gran = (unsigned long long*)v.gran.p;
  int* err = (int*)v.err.p;
  SvcBox* box = v.box_dev;
  unsigned long long* relay = (unsigned long long*)v.relay.p;
  unsigned long long* seenp = relay + 2 * SVC_DRING;
  uint8_t* rec = v.rec_dev;
  unsigned long long s0 = seq0;
  int stamps = opt(O_SERVICE_STAMPS) ? 1 : 0;
  if (opt(O_SVC_FULL_FENCE)) stamps |= 4;  // the simple evaluation's record fence as the general chain's
  if (opt(O_SERVICE_NO_DIFF)) stamps |= 2;  // every requested row resent (no row diff)
  int xcd = v.xcd ? 1 : 0;
  void* args[] = {(void*)&jd,  (void*)&pr,  (void*)&W,     (void*)&npt,   (void*)&bins, (void*)&ck, (void*)&gran,
                  (void*)&err, (void*)&box, (void*)&relay, (void*)&seenp, (void*)&rec, (void*)&s0, (void*)&stamps,
                  (void*)&xcd};
  const unsigned grid = (unsigned)(v.xcd ? XCD_GRID_MULT * W : W);
  if (int rc = launch_resident(fn, dim3(grid), dim3((unsigned)v.threads), args, v.shmem, v.stream)) return rc;
  v.running = true;
  return 0;
}

// The grid with the staged pods' programs; geometry as a per-pod k_schedule launch.
static int svc_start_locked(kss_ctx* ctx) {
  if (!ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  if (ctx->staged_n <= 0) return fail(KSS_E_INVAL, "the service evaluates staged pods: kss_stage_pods first");
  if (ctx->split_n > 1) return fail(KSS_E_UNSUPPORTED, "the service runs the whole cluster on one device");
  if (!ctx->nom.empty())
    return fail(KSS_E_UNSUPPORTED, "the service grid does not read the nominator: kss_eval_pod / batches while pods are nominated");
  auto& v = ctx->svc;
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  HIP_TRY(hipStreamSynchronize(ctx->stream));  // every earlier launch / copy on the ctx stream is done
  const size_t N = (size_t)ctx->dc.N;
  int W = std::max(1, std::min(ctx->n_cu, (int)((N + ctx->nodes_per_shard - 1) / ctx->nodes_per_shard)));
  if (ctx->force_w > 0) W = std::min(ctx->force_w, ctx->n_cu);
  W = std::max(W, (int)((N + KSS_MAX_NPT * KSS_MAX_THREADS - 1) / (KSS_MAX_NPT * KSS_MAX_THREADS)));
  W = std::min(W, std::max(1, (int)N));
  const bool window = ctx->prof.pct_nodes_to_score < 100;  // k_schedule's window exchange: W + 1 values
  if (window) W = std::min(W, XW_MAX - NSCAL);
  const PlanNeeds& need = ctx->staged_need;
  // the k_simple-shaped evaluation (svc_simple_eval): staged default-profile pods (compact records,
  // no programs; under percentageOfNodesToScore < 100 no PreFilterResult node lists: svc_window),
  // no extended resources, exact f64 arithmetic, W <= 64 (its exchange:
  // one lane per shard), the node rows cached in LDS (checked below); KSS_SERVICE_GENERAL=1 keeps
  // the general chain, for comparison.  On an XCD-local grid when its shards fit one XCD's CUs.
  const bool simple_pre = ctx->spod_ok && (!window || !ctx->staged_names) && !need.general && ctx->dc.n_scalar == 0 && ctx->small_values &&
                          f64_exact(ctx->f64_cluster, ctx->f64_pods, ctx->staged_n) && !opt(O_SERVICE_GENERAL);
  const int xcd_cus = ctx->n_cu / XCD_GRID_MULT;
  // (off by default: the record's stores to host memory from one XCD were slower than the L2
  // exchange saved -- C2 slim 20.9 -> 29.0 us, r5o_perpod.json; KSS_SVC_XCD=1 turns it on)
  const bool svc_xcd = opt(O_SVC_XCD) != 0;
  const bool xcd_ok = svc_xcd && simple_pre && ctx->xcd_mode && ctx->n_cu % XCD_GRID_MULT == 0 && ctx->force_w <= 0 &&
                      N <= (size_t)xcd_cus * KSS_MAX_THREADS * KSS_MAX_NPT;
  if (xcd_ok) W = std::min(W, xcd_cus);
  if (W > 1 && need.xw > XW_MAX) return fail(KSS_E_UNSUPPORTED, "topology histograms too large for the service grid");
  if (W > SVC_MAX_SHARDS || W > ctx->n_cu) return fail(KSS_E_UNSUPPORTED, "cluster too large for the service grid");
  Geometry g;
  if (!pick_geometry((int)N, W, ctx->pref_threads, g)) return fail(KSS_E_UNSUPPORTED, "no geometry for this cluster");
  const int bins_cap = std::max(need.bins_cap, 0) + (window ? g.W : 0);
  const int cap = g.threads * g.npt;
  const size_t base = lds_bytes(bins_cap, cap);
  if (base > KSS_LDS_BUDGET) return fail(KSS_E_UNSUPPORTED, "per-workgroup LDS budget exceeded");
  int cache_keys = -1;
  if (base + node_cache_bytes(cap, ctx->dc.n_keys) <= KSS_LDS_BUDGET) cache_keys = ctx->dc.n_keys;
  else if (base + node_cache_bytes(cap, 0) <= KSS_LDS_BUDGET) cache_keys = 0;
  // the resident grid on a queue of its own: no other stream's kernel waits behind it
  if (!v.stream) HIP_TRY(dedicated_stream(ctx->n_cu, &v.stream));
  const SlotLayout SL(N);
  if (!v.box) {
    HIP_TRY(hipHostMalloc((void**)&v.box, sizeof(SvcBox), hipHostMallocCoherent | hipHostMallocMapped));
    std::memset((void*)v.box, 0, sizeof(SvcBox));
    HIP_TRY(hipHostGetDevicePointer((void**)&v.box_dev, v.box, 0));
    v.posted = 0;
  }
  const size_t rec_bytes = SL.bytes + CompactLayout(N).bytes;  // the full record, then the compact one
  if (v.rec_bytes < rec_bytes) {
    svc_free_rec(v);
    const bool huge = opt(O_SVC_HUGE) != 0;
    if (huge) {
      // experiment: the record in transparent huge pages (madvise), registered with the device,
      // so that its rows do not each take their own 4 KiB translation
      const size_t H = (size_t)2 << 20, sz = align_up(rec_bytes, H);
      void* m = mmap(nullptr, sz + H, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (m == MAP_FAILED) return fail(KSS_E_NOMEM, "record mapping failed");
      uint8_t* a = (uint8_t*)align_up((size_t)m, H);
      madvise(a, sz, MADV_HUGEPAGE);
      std::memset(a, 0, sz);
      if (hipHostRegister(a, sz, hipHostRegisterMapped) != hipSuccess) {
        munmap(m, sz + H);
        return fail(KSS_E_DEVICE, "record registration failed");
      }
      v.rec_map = m;
      v.rec_map_bytes = sz + H;
      v.rec = a;
    } else {
      HIP_TRY(hipHostMalloc((void**)&v.rec, rec_bytes, hipHostMallocCoherent | hipHostMallocMapped));
    }
    HIP_TRY(hipHostGetDevicePointer((void**)&v.rec_dev, v.rec, 0));
    v.rec_bytes = rec_bytes;
  }
  int rc = ctx->slot_buf.ensure(2 * SL.bytes);  // two record slots used in turn (kss_service.cuh)
  if (!rc) rc = v.relay.ensure(sizeof(unsigned long long) * (2 * SVC_DRING + (size_t)W));
  if (!rc) rc = v.gran.ensure(sizeof(unsigned long long) * 2 * (size_t)W * 2 * XW_MAX);
  if (!rc) rc = v.err.ensure(16);
  if (!rc) rc = v.job.ensure(sizeof(DevJob));
  if (rc) return rc;
  DevJob job{};
  job.c = ctx->dc;
  job.P = ctx->dp;
  job.n_pods = ctx->staged_n;
  job.commit = 1;
  job.keep_norm = 1;
  job.record = 0;
  job.slots = (uint8_t*)ctx->slot_buf.p;
  job.slot_bytes = SL.bytes;
  job.prof = ctx->prof;
  job.cursor = (int32_t*)ctx->cursor_buf.p;
  v.simple = simple_pre && cache_keys >= 0 && g.W <= 64;
  v.xcd = v.simple && xcd_ok && g.W <= xcd_cus && g.W > 1;
  job.spods = v.simple ? (const SPod*)ctx->spod_buf.p : nullptr;
  // the static words of every staged pod (4 bytes per pod and node, at most 4 GiB): one load per
  // evaluation instead of the pod's requirement chains from HBM (KSS_SVC_NO_STATIC=1: inline)
  const size_t stat_bytes = sizeof(uint32_t) * (size_t)std::max(ctx->staged_n, 1) * std::max<size_t>(N, 1);
  const bool pre_static = v.simple && stat_bytes <= ((size_t)4 << 30) && !opt(O_SVC_NO_STATIC);
  if (pre_static && (rc = v.stat.ensure(stat_bytes))) return rc;
  job.stat = pre_static ? (uint32_t*)v.stat.p : nullptr;
  HIP_TRY(hipMemcpyAsync(v.job.p, &job, sizeof(DevJob), hipMemcpyHostToDevice, v.stream));
  if (pre_static) {
    launch_static(v.stream, same_profile(ctx->prof, default_profile_c()), (const DevJob*)v.job.p, ctx->prof, 1, 0,
                  ctx->staged_n, 0, (int)N, ctx->dc.n_keys);
    HIP_TRY(hipGetLastError());
  }
  v.W = g.W;
  v.threads = g.threads;
  v.npt = g.npt;
  v.bins_cap = bins_cap;
  v.cache_keys = cache_keys;
  v.shmem = base + (cache_keys >= 0 ? node_cache_bytes(cap, cache_keys) : 0);
  v.gen = std::max(need.bins_cap, 0) > 0 || need.general;
  ctx->last_geom[0] = g.W;
  ctx->last_geom[1] = g.threads;
  ctx->last_geom[2] = g.npt;
  return svc_launch(ctx);
}

// Post one command (the ring never overruns what shard 0 has relayed).
static int svc_post(kss_ctx* ctx, int op, int pod, int node, int fields, unsigned long long* seq_out) {
  auto& v = ctx->svc;
  const auto t0 = std::chrono::steady_clock::now();
  while (v.posted - __atomic_load_n(&v.box->consumed, __ATOMIC_ACQUIRE) >= (unsigned long long)SVC_RING) {
    if (!svc_alive(ctx)) {
      if (int rc = svc_launch(ctx)) return rc;
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) return fail(KSS_E_DEVICE, "service ring full");
  }
  SvcCmd& c = v.box->cmd[v.posted % SVC_RING];
  // the two tagged words: either may land first, the grid takes the entry once both carry the tag
  __atomic_store_n(&c.w1, svc_w1(v.posted, node), __ATOMIC_RELEASE);
  __atomic_store_n(&c.w0, svc_w0(v.posted, op, fields, pod), __ATOMIC_RELEASE);
  *seq_out = v.posted;
  ++v.posted;
  return 0;
}

// Stop the grid (STOP command, then the stream drains: every wait in the grid is bounded).
// Relaunch a grid that left after its idle timeout while commands it has not taken are in
// the ring (a commit / rollback posted as it left): they run before anything else.
static int svc_revive(kss_ctx* ctx) {
  auto& v = ctx->svc;
  if (!v.running || svc_alive(ctx)) return 0;
  HIP_TRY(hipStreamSynchronize(v.stream));
  if (v.box->err) return 0;  // a failed grid: svc_stop reports it
  if (__atomic_load_n(&v.box->consumed, __ATOMIC_ACQUIRE) >= v.posted) return 0;
  return svc_launch(ctx);
}

static int svc_stop(kss_ctx* ctx) {
  auto& v = ctx->svc;
  if (!v.running) return 0;
  unsigned long long seq = 0;
  bool stop_queued = false;
  if (int rc = svc_revive(ctx)) return rc;  // never drop a queued commit / rollback
  if (svc_alive(ctx)) {
    if (int rc = svc_post(ctx, SVC_STOP, 0, 0, 0, &seq)) return rc;
    stop_queued = true;
  }
  HIP_TRY(hipStreamSynchronize(v.stream));
  // the grid may have left on its idle timeout between the check above and the STOP: it is
  // relaunched for the commands it did not take, a STOP behind them
  for (int again = 0; again < 4 && !v.box->err && __atomic_load_n(&v.box->consumed, __ATOMIC_ACQUIRE) < v.posted;
       again++) {
    if (int rc = svc_launch(ctx)) return rc;
    if (!stop_queued) {
      if (int rc = svc_post(ctx, SVC_STOP, 0, 0, 0, &seq)) return rc;
      stop_queued = true;
    }
    HIP_TRY(hipStreamSynchronize(v.stream));
  }
  v.running = false;
  const bool err = v.box->err != 0;
  if (!err && __atomic_load_n(&v.box->consumed, __ATOMIC_ACQUIRE) < v.posted)
    return fail(KSS_E_DEVICE, "service grid: queued commands were not taken");
  // after a failure the queued commands are dropped (a later start resumes after them)
  __atomic_store_n(&v.box->consumed, v.posted, __ATOMIC_RELEASE);
  if (err) {
    ctx->state_unknown = true;
    return fail(KSS_E_DEVICE, "service grid: a shard exchange timed out");
  }
  return 0;
}

int kss_service_mode(kss_ctx* ctx, int32_t* mode) {
  if (!ctx || !mode) return fail(KSS_E_INVAL, "bad arguments");
  std::lock_guard<std::mutex> lk(ctx->mu);
  *mode = ctx->svc.W > 0 ? (ctx->svc.simple ? (ctx->svc.xcd ? 2 : 1) : 0) : -1;
  return 0;
}

int kss_service_start(kss_ctx* ctx) {
  if (!ctx) return fail(KSS_E_INVAL, "null ctx");
  KSS_SVC_QUIESCE(ctx);
  std::lock_guard<std::mutex> lk(ctx->mu);
  return svc_start_locked(ctx);
}

int kss_service_stop(kss_ctx* ctx) {
  if (!ctx) return fail(KSS_E_INVAL, "null ctx");
  std::lock_guard<std::mutex> lk(ctx->mu);
  return svc_stop(ctx);
}

// One EVAL command on the service grid and the wait for every shard's done flag (restarting
// a grid that left idle before taking the command).  ovf: some shard's compact record value
// did not fit its narrow type.
static int svc_eval_wait(kss_ctx* ctx, int32_t pod_index, uint32_t fields, bool compact, bool& ovf,
                         bool repeat = false) {
  auto& v = ctx->svc;
  if (!v.running) {
    if (int rc = svc_start_locked(ctx)) return rc;
  }
  unsigned long long seq = 0;
  // node bit 0: the compact record; bit 1: the same cycle again (nextStartNodeIndex as before the last one)
  if (int rc = svc_post(ctx, SVC_EVAL, pod_index, (compact ? 1 : 0) | (repeat ? 2 : 0), (int)(fields & KSS_FIELD_ALL), &seq))
    return rc;
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spins = 0;; ++spins) {
    bool all = true;
    for (int w = 0; w < v.W && all; w++) all = (__atomic_load_n(&v.box->done[w], __ATOMIC_ACQUIRE) & ~SVC_DONE_OVF) > seq;
    if (all) break;
    if ((spins & 1023) == 1023) {
      if (v.box->err) {
        svc_stop(ctx);
        ctx->state_unknown = true;
        return fail(KSS_E_DEVICE, "service grid: a shard exchange timed out");
      }
      if (!svc_alive(ctx)) {
        if (__atomic_load_n(&v.box->consumed, __ATOMIC_ACQUIRE) <= seq) {  // left idle before taking it
          v.running = false;
          if (v.box->xcd_fail) v.xcd = false;  // XCD 0 had too few free CUs: relaunch unrestricted
          if (int rc = svc_launch(ctx)) return rc;
        } else {
          v.running = false;
          return fail(KSS_E_DEVICE, "service grid left during an evaluation");
        }
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
        svc_stop(ctx);
        return fail(KSS_E_DEVICE, "service evaluation timed out");
      }
    }
  }
  ovf = false;
  for (int w = 0; w < v.W; w++) ovf |= (__atomic_load_n(&v.box->done[w], __ATOMIC_ACQUIRE) & SVC_DONE_OVF) != 0;
  if (v.box->meta.status == 4) return fail(KSS_E_UNSUPPORTED, "pod program exceeds the device path's per-pod limits");
  return 0;
}

static void svc_full_view(kss_ctx* ctx, uint32_t fields, kss_pod_view* out) {
  const PodMeta m = ctx->svc.box->meta;
  const SlotLayout SL((size_t)ctx->dc.N);
  const uint8_t* r = ctx->svc.rec;
  out->fail_plugin = (fields & KSS_FIELD_FAIL) ? r + SL.fail : nullptr;
  out->fail_detail = (fields & KSS_FIELD_DETAIL) ? (const uint16_t*)(r + SL.detail) : nullptr;
  out->raw = (fields & KSS_FIELD_RAW) ? (const int64_t*)(r + SL.raw) : nullptr;
  out->norm = (fields & KSS_FIELD_NORM) ? (const int64_t*)(r + SL.norm) : nullptr;
  out->total = (fields & KSS_FIELD_TOTAL) ? (const int64_t*)(r + SL.total) : nullptr;
  out->chosen = m.chosen;
  out->n_feasible = m.n_feasible;
  out->best_total = m.best_total;
  out->scored = m.scored;
  out->status = m.status;
}

int kss_service_eval(kss_ctx* ctx, int32_t pod_index, uint32_t fields, kss_pod_view* out) {
  if (!ctx || !ctx->loaded || !out) return fail(KSS_E_INVAL, "bad arguments");
  if (pod_index < 0 || pod_index >= ctx->staged_n || pod_index >= (1 << 24)) return fail(KSS_E_INVAL, "pod index outside the staged pods");
  std::lock_guard<std::mutex> lk(ctx->mu);
  bool ovf = false;
  if (int rc = svc_eval_wait(ctx, pod_index, fields, false, ovf)) return rc;
  svc_full_view(ctx, fields, out);
  return 0;
}

int kss_service_eval_compact(kss_ctx* ctx, int32_t pod_index, uint32_t fields, kss_pod_cview* out) {
  if (!ctx || !ctx->loaded || !out) return fail(KSS_E_INVAL, "bad arguments");
  if (pod_index < 0 || pod_index >= ctx->staged_n || pod_index >= (1 << 24)) return fail(KSS_E_INVAL, "pod index outside the staged pods");
  std::lock_guard<std::mutex> lk(ctx->mu);
  bool ovf = false;
  if (int rc = svc_eval_wait(ctx, pod_index, fields, true, ovf)) return rc;
  *out = kss_pod_cview{};
  if (ovf) {  // a score outside int32 / a normalised score above 255: the same pod, full record
    if (int rc = svc_eval_wait(ctx, pod_index, fields, false, ovf, /*repeat=*/true)) return rc;
    out->is_wide = 1;
    svc_full_view(ctx, fields, &out->wide);
  } else {
    const CompactLayout CL((size_t)ctx->dc.N);
    const uint8_t* r = ctx->svc.rec + SlotLayout((size_t)ctx->dc.N).bytes;
    out->fail_plugin = (fields & KSS_FIELD_FAIL) ? r + CL.fail : nullptr;
    out->fail_detail = (fields & KSS_FIELD_DETAIL) ? (const uint16_t*)(r + CL.detail) : nullptr;
    out->raw = (fields & KSS_FIELD_RAW) ? (const int32_t*)(r + CL.raw) : nullptr;
    out->norm = (fields & KSS_FIELD_NORM) ? r + CL.norm : nullptr;
    out->total = (fields & KSS_FIELD_TOTAL) ? (const int32_t*)(r + CL.total) : nullptr;
  }
  const PodMeta m = ctx->svc.box->meta;
  out->chosen = m.chosen;
  out->n_feasible = m.n_feasible;
  out->best_total = m.best_total;
  out->scored = m.scored;
  out->status = m.status;
  return 0;
}

static int svc_commit(kss_ctx* ctx, int32_t pod_index, int32_t node, int sign) {
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "bad arguments");
  if (pod_index < 0 || pod_index >= ctx->staged_n || pod_index >= (1 << 24)) return fail(KSS_E_INVAL, "pod index outside the staged pods");
  const int local = node - ctx->dc.node_base;
  if (local < 0 || local >= ctx->dc.N) return fail(KSS_E_INVAL, "node out of range");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (!ctx->svc.running) {
    if (int rc = svc_start_locked(ctx)) return rc;
  } else if (!svc_alive(ctx)) {  // left idle: relaunch it to take the command (svc_stop also would)
    HIP_TRY(hipStreamSynchronize(ctx->svc.stream));
    if (ctx->svc.box->err) {
      svc_stop(ctx);
      ctx->state_unknown = true;
      return fail(KSS_E_DEVICE, "service grid: a shard exchange timed out");
    }
    if (int rc = svc_launch(ctx)) return rc;
  }
  unsigned long long seq = 0;
  if (int rc = svc_post(ctx, sign > 0 ? SVC_COMMIT : SVC_ROLLBACK, pod_index, node, 0, &seq)) return rc;
  if (sign > 0) {  // the same host bookkeeping as kss_commit (bounds, PostFilter table)
    const double own = pod_index < (int)ctx->staged_bp.size() ? (double)ctx->staged_bp[pod_index].tlen : 0.0;
    ctx->count_bound += 1.0 + own;
    ctx->cell_bound += 1.0 + own;
  }
  if (pod_index < (int)ctx->staged_bp.size())
    ctx->bound_log.push_back(BoundOp{local, sign > 0 ? 1 : 0, ctx->staged_bp[pod_index]});
  ctx->bound_dirty = true;
  return 0;
}

int kss_service_commit(kss_ctx* ctx, int32_t pod_index, int32_t node) { return svc_commit(ctx, pod_index, node, 1); }
int kss_service_stamps(kss_ctx* ctx, uint64_t* out8) {
  if (!ctx || !out8) return fail(KSS_E_INVAL, "bad arguments");
  if (!ctx->svc.box) return fail(KSS_E_INVAL, "no service grid");
  for (int i = 0; i < 8; i++) out8[i] = __atomic_load_n(&ctx->svc.box->stamp[i], __ATOMIC_ACQUIRE);
  return 0;
}

int kss_service_rollback(kss_ctx* ctx, int32_t pod_index, int32_t node) { return svc_commit(ctx, pod_index, node, -1); }

int kss_fetch_record(kss_ctx* ctx, int32_t pod_index, kss_pod_result* out) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !out) return fail(KSS_E_INVAL, "bad arguments");
  if (pod_index < 0 || pod_index >= ctx->recorded) return fail(KSS_E_NOTFOUND, "pod not recorded");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  return copy_slot(ctx, pod_index, ctx->meta_host[pod_index], out);
}

int kss_last_timing(kss_ctx* ctx, double* device_ms, int32_t* launches) {
  if (!ctx) return fail(KSS_E_INVAL, "null ctx");
  if (device_ms) *device_ms = ctx->last_ms;
  if (launches) *launches = ctx->last_launches;
  return 0;
}

int kss_last_handoff_retries(kss_ctx* ctx, int32_t* retries) {
  if (!ctx || !retries) return fail(KSS_E_INVAL, "bad arguments");
  *retries = ctx->last_handoff_retries;
  return 0;
}

int kss_last_handoff_status(kss_ctx* ctx, int32_t* out3) {
  if (!ctx || !out3) return fail(KSS_E_INVAL, "bad arguments");
  out3[0] = ctx->last_kernel_spread ? ctx->last_handoff_retries : 0;
  out3[1] = ctx->last_kernel_spread ? ctx->last_handoff_recovered : 0;
  out3[2] = ctx->last_kernel_spread ? ctx->last_handoff_final : 0;
  return 0;
}
int kss_buffer_map(kss_ctx* ctx, uint64_t* base, uint64_t* bytes, int32_t cap, int32_t* n) {
  if (!ctx || !n || cap < 0 || (cap && (!base || !bytes))) return fail(KSS_E_INVAL, "bad arguments");
  const DevBuf* bufs[] = {&ctx->cluster_buf, &ctx->pristine_buf, &ctx->pod_buf, &ctx->tmp_pod_buf, &ctx->slot_buf,
                          &ctx->meta_buf,    &ctx->chosen_buf,   &ctx->job_buf, &ctx->gran_buf,    &ctx->err_buf,
                          &ctx->ck_buf,      &ctx->stamp_buf,    &ctx->spod_buf, &ctx->stat_buf,   &ctx->gpod_buf,
                          &ctx->res_buf,     &ctx->delta_buf,    &ctx->axis_cv, &ctx->bound_buf,   &ctx->pre_buf};
  const int nb = (int)(sizeof(bufs) / sizeof(bufs[0]));
  *n = nb + 1;
  for (int i = 0; i < nb && i < cap; i++) {
    base[i] = (uint64_t)(uintptr_t)bufs[i]->p;
    bytes[i] = bufs[i]->cap;
  }
  if (nb < cap) {
    base[nb] = (uint64_t)(uintptr_t)ctx->split_inbox;
    bytes[nb] = ctx->split_inbox_bytes;
  }
  return 0;
}

int kss_last_handoff_diag(kss_ctx* ctx, int32_t* recovered, int64_t* entries, int32_t cap, int32_t* n_entries) {
  if (!ctx || !recovered || !n_entries || cap < 0 || (cap && !entries)) return fail(KSS_E_INVAL, "bad arguments");
  std::lock_guard<std::mutex> lk(ctx->mu);
  *recovered = ctx->last_handoff_recovered;
  *n_entries = 0;
  if (!ctx->last_kernel_spread || !ctx->ck_buf.p || !(ctx->last_handoff_retries || ctx->last_handoff_final)) return 0;
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  std::vector<long long> h(1 + (size_t)HANDOFF_DIAG * HANDOFF_DIAG_W);
  HIP_TRY(hipMemcpy(h.data(), (unsigned long long*)ctx->ck_buf.p + ctx->ck_diag_off, h.size() * 8, hipMemcpyDeviceToHost));
  const int n = (int)std::min<long long>(h[0], HANDOFF_DIAG);
  const int m = std::min(n, cap);
  std::memcpy(entries, h.data() + 1, sizeof(int64_t) * HANDOFF_DIAG_W * (size_t)m);
  *n_entries = n;
  return 0;
}

int kss_last_loop_timing(kss_ctx* ctx, double* loop_ms) {
  if (!ctx || !loop_ms) return fail(KSS_E_INVAL, "bad arguments");
  *loop_ms = ctx->last_loop_ms;
  return 0;
}

int kss_last_geometry(kss_ctx* ctx, int32_t* out3) {
  if (!ctx || !out3) return fail(KSS_E_INVAL, "bad arguments");
  for (int i = 0; i < 3; i++) out3[i] = ctx->last_geom[i];
  return 0;
}

int kss_last_xcd_local(kss_ctx* ctx, int32_t* out2) {
  if (!ctx || !out2) return fail(KSS_E_INVAL, "bad arguments");
  out2[0] = ctx->last_xcd[0];
  out2[1] = ctx->last_xcd[1];
  return 0;
}

int kss_last_kernel(kss_ctx* ctx) {
  if (!ctx) return fail(KSS_E_INVAL, "null ctx");
  return ctx->last_kernel;
}

int kss_fetch_meta(kss_ctx* ctx, int32_t first, int32_t n, int64_t* out) {
  if (!ctx || (n > 0 && !out)) return fail(KSS_E_INVAL, "bad arguments");
  if (first < 0 || n < 0 || first + n > ctx->meta_n) return fail(KSS_E_NOTFOUND, "pod outcome not available");
  if (ctx->axis_meta_dirty) {  // node-axis outcomes were written on the caller's stream
    HIP_TRY(hipSetDevice(ctx->cfg.device));
    HIP_TRY(hipDeviceSynchronize());
    ctx->meta_host.resize((size_t)ctx->meta_n);
    HIP_TRY(hipMemcpy(ctx->meta_host.data(), ctx->meta_buf.p, sizeof(PodMeta) * (size_t)ctx->meta_n, hipMemcpyDeviceToHost));
    ctx->axis_meta_dirty = false;
  }
  for (int i = 0; i < n; i++) {
    const PodMeta& m = ctx->meta_host[first + i];
    int64_t* o = out + 5 * (size_t)i;
    o[0] = m.chosen;
    o[1] = m.n_feasible;
    o[2] = m.scored;
    o[3] = m.status;
    o[4] = m.best_total;
  }
  return 0;
}

// ---------------------------------------------------------------------------
// what-if scenario sweeps (KEP-184; BASELINE C5): many independent clusters, one
// workgroup each, no inter-scenario communication.  kss_sweep_create packs every input
// into one host image and uploads it with ONE copy; kss_sweep_run restores the node
// state from the uploaded pristine copy (one device copy) and schedules every scenario.
// ---------------------------------------------------------------------------
}  // extern "C"

namespace {

// Bump allocator over one host image / device arena pair (offsets 256-B aligned).  With
// h == nullptr it only sizes.
struct Packer {
  char* h = nullptr;
  char* d = nullptr;
  size_t o = 0, last = 0;
  template <class T>
  T* put(const T* src, size_t count, size_t reserve = 0) {
    const size_t n = std::max(std::max(count, reserve), (size_t)1);
    last = o;
    o = align_up(o + sizeof(T) * n, 256);
    if (h) {
      const size_t done = src ? sizeof(T) * count : 0;
      if (done) memcpy(h + last, src, done);
      if (sizeof(T) * n > done) memset(h + last + done, 0, sizeof(T) * n - done);
    }
    return reinterpret_cast<T*>(d + last);
  }
};

// The read-only part of one scenario: cluster columns except the mutable ones, the pod
// programs and (simple sweeps) the compact pod records.
void pack_inputs(Packer& P, const kss_cluster* cl, const kss_podset* ps, const std::vector<SPod>* spods, DevJob& j) {
  const size_t N = (size_t)cl->n_nodes, K = (size_t)cl->n_label_keys;
  DevCluster& c = j.c;
  c.N = cl->n_nodes;
  c.n_scalar = cl->n_scalar;
  c.n_keys = cl->n_label_keys;
  c.n_classes = cl->n_classes;
  c.n_terms = cl->n_terms;
  c.node_base = cl->node_base;
  c.class_cap = cl->n_classes;
  c.term_cap = cl->n_terms;
  c.alloc = P.put(cl->alloc, KSS_NRES * N);
  c.allowed_pods = P.put(cl->allowed_pods, N);
  c.node_flags = P.put(cl->node_flags, N);
  c.taint_hard = P.put(cl->taint_hard, N);
  c.taint_soft = P.put(cl->taint_soft, N);
  c.taint_order = P.put(cl->taint_order, (size_t)KSS_TAINT_ORDER * N);
  c.label_value = P.put(cl->label_value, K * N);
  c.key_base = P.put(cl->key_base, K);
  c.key_card = P.put(cl->key_card, K);
  c.key_flags = P.put(cl->key_flags, K);
  c.key_empty = P.put(cl->key_empty, K);
  c.value_int = P.put(cl->value_int, (size_t)cl->n_label_values);
  c.value_is_int = P.put(cl->value_is_int, (size_t)cl->n_label_values);
  c.log_table = P.put<double>(nullptr, N + 3);
  if (P.h) {
    double* lt = reinterpret_cast<double*>(P.h + P.last);
    for (size_t k = 0; k < N + 3; k++) lt[k] = kss_go_log((double)(k + 2));
  }
  c.nc64 = nullptr;
  c.nct = nullptr;
  c.nc32 = nullptr;
  c.ncl = nullptr;
  c.n_vol_rows = c.n_vol_keys = 0;  // sweeps refuse pods with volume programs (ports_images)
  c.vol_count = c.vol_attached = nullptr;
  c.vol_limit = c.vol_row_key = c.vol_key_plugin = nullptr;
  j.P.vols = nullptr;
  j.P.pods = P.put(ps->pods, (size_t)ps->n_pods);
  j.P.reqs = P.put(ps->reqs, (size_t)ps->n_reqs);
  j.P.terms = P.put(ps->terms, (size_t)ps->n_terms);
  j.P.spreads = P.put(ps->spreads, (size_t)ps->n_spreads);
  j.P.ipa = P.put(ps->ipa, (size_t)ps->n_ipa);
  j.P.ints = P.put(ps->ints, (size_t)ps->n_ints);
  j.spods = spods ? P.put(spods->data(), spods->size()) : nullptr;
}

// The mutable columns of one scenario (AssumePod targets): the host image holds the
// snapshot (the device's pristine copy); the device pointers address the live copy.
void pack_mutable(Packer& P, const kss_cluster* cl, DevJob& j) {
  const size_t N = (size_t)cl->n_nodes;
  j.c.requested = P.put(cl->requested, KSS_NRES * N);
  j.c.nonzero = P.put(cl->nonzero, 2 * N);
  j.c.pod_count = P.put(cl->pod_count, N);
  j.c.class_count = P.put(cl->class_count, (size_t)cl->n_classes * N);
  j.c.term_count = P.put(cl->term_count, (size_t)cl->n_terms * N);
}

}  // namespace

struct kss_sweep {
  int device = 0;
  kss_profile prof{};
  int n_scen = 0;
  hipStream_t st = nullptr, st2 = nullptr;  // st2: k_static of the next chunk (double-buffered table)
  hipEvent_t e0 = nullptr, e1 = nullptr;
  std::vector<hipEvent_t> pev;
  char* arena = nullptr;
  size_t up_bytes = 0;                   // [0, up_bytes): uploaded once (inputs, pristine state, jobs)
  size_t pristine_off = 0, live_off = 0, mut_bytes = 0;
  size_t chosen_off = 0, meta_off = 0, err_off = 0, gran_off = 0, gran_bytes = 0, stat_off = 0, jobs_off = 0;
  size_t cursor_off = 0;  // one nextStartNodeIndex per scenario (percentageOfNodesToScore < 100)
  std::vector<int32_t> n_pods;
  int total_pods = 0, max_pods = 0, max_nodes = 0, max_keys = 0;
  bool simple = false;
  int chunk = 0;
  Geometry g;
  PlanNeeds need;
  double stage_ms = 0;
  ~kss_sweep() {
    if (st) hipStreamSynchronize(st);
    if (arena) hipFree(arena);
    if (e0) hipEventDestroy(e0);
    if (e1) hipEventDestroy(e1);
    for (hipEvent_t e : pev) hipEventDestroy(e);
    if (st2) hipStreamSynchronize(st2), hipStreamDestroy(st2);
    if (st) hipStreamDestroy(st);
  }
};

extern "C" {

kss_sweep* kss_sweep_create(int32_t device, const kss_profile* prof, int32_t n_scen, const kss_cluster* clusters,
                            const kss_podset* podsets) {
  if (!prof || n_scen <= 0 || !clusters || !podsets) {
    fail(KSS_E_INVAL, "bad arguments");
    return nullptr;
  }
  if (check_profile(prof)) return nullptr;
  for (int s = 0; s < n_scen; s++)
    if (check_cluster(&clusters[s]) || validate(&clusters[s], &podsets[s], podsets[s].n_pods)) return nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  std::unique_ptr<kss_sweep> sw(new kss_sweep());
  sw->device = device;
  sw->prof = *prof;
  sw->n_scen = n_scen;
  sw->n_pods.resize(n_scen);
  for (int s = 0; s < n_scen; s++) {
    sw->n_pods[s] = podsets[s].n_pods;
    sw->total_pods += podsets[s].n_pods;
    sw->max_pods = std::max(sw->max_pods, podsets[s].n_pods);
    sw->max_nodes = std::max(sw->max_nodes, clusters[s].n_nodes);
    sw->max_keys = std::max(sw->max_keys, clusters[s].n_label_keys);
    const PlanNeeds q = plan_needs(clusters[s].key_card, clusters[s].key_flags, &podsets[s], podsets[s].n_pods);
    sw->need.bins_cap = std::max(sw->need.bins_cap, q.bins_cap);
    sw->need.general |= q.general;
    if (q.ports_images) {  // the sweep packs no UsedPorts / image-score columns
      fail(KSS_E_UNSUPPORTED, "scenario sweeps: pods with host ports, ImageLocality rows or volumes take kss_schedule_batch");
      return nullptr;
    }
  }
  // one workgroup per scenario: at most two node slots per lane (C5, 1,000 nodes: 512
  // threads ran the 512-scenario sweep in 16.5 ms against 23.7 ms at 256)
  int pref = sw->max_nodes > 512 ? 512 : 256;
  if (opt(O_THREADS) > 0) pref = (int)std::min<long long>(KSS_MAX_THREADS, std::max(64ll, opt(O_THREADS)));
  if (!pick_geometry(sw->max_nodes, 1, pref, sw->g)) {
    fail(KSS_E_UNSUPPORTED, "scenario cluster too large for one workgroup");
    return nullptr;
  }
  // k_static + k_simple for the whole sweep when every scenario qualifies (no spread /
  // inter-pod programs, no scalar resources, values inside the exact f64 envelope)
  std::vector<std::vector<SPod>> spods(n_scen);
  bool simple = !opt(O_NO_SIMPLE) && !sw->need.general && simple_fits(sw->g, 0) &&
                prof->pct_nodes_to_score >= 100;  // the window runs on k_schedule
  for (int i = 0; i < prof->fit_n && simple; i++) simple = prof->fit_weight[i] >= 0 && prof->fit_weight[i] < (1ll << 20);
  for (int s = 0; s < n_scen && simple; s++) {
    const kss_cluster& cl = clusters[s];
    simple = cl.n_scalar == 0;
    for (size_t i = 0; i < 3 * (size_t)cl.n_nodes && simple; i++) simple = cl.alloc[i] >= 0 && cl.alloc[i] < (1ll << 46);
    if (simple) {
      F64Bounds bc, bp;
      f64_bounds_cluster(&cl, bc);
      f64_bounds_pods(&podsets[s], bp);
      simple = f64_exact(bc, bp, podsets[s].n_pods);
    }
    if (simple) simple = build_spods(&podsets[s], 0, spods[s]);
  }
  sw->simple = simple;
  // layout: [inputs][pristine state][jobs] uploaded; [live state][chosen][meta][err][gran][stat]
  std::vector<DevJob> jobs(n_scen);
  std::vector<size_t> in_off(n_scen), mut_off(n_scen);
  Packer dry;
  for (int s = 0; s < n_scen; s++) {
    in_off[s] = dry.o;
    pack_inputs(dry, &clusters[s], &podsets[s], simple ? &spods[s] : nullptr, jobs[s]);
  }
  sw->pristine_off = dry.o;
  for (int s = 0; s < n_scen; s++) {
    mut_off[s] = dry.o;
    pack_mutable(dry, &clusters[s], jobs[s]);
  }
  sw->mut_bytes = dry.o - sw->pristine_off;
  sw->jobs_off = dry.o;
  dry.put<DevJob>(nullptr, (size_t)n_scen);
  sw->up_bytes = dry.o;
  sw->live_off = dry.o;
  dry.o = align_up(dry.o + sw->mut_bytes, 256);
  dry.put<int32_t>(nullptr, (size_t)sw->total_pods);
  sw->chosen_off = dry.last;
  dry.put<PodMeta>(nullptr, (size_t)sw->total_pods);
  sw->meta_off = dry.last;
  dry.put<int32_t>(nullptr, 4);
  sw->err_off = dry.last;
  dry.put<int32_t>(nullptr, (size_t)n_scen);
  sw->cursor_off = dry.last;
  size_t sum_nodes = 0;
  for (int s = 0; s < n_scen; s++) sum_nodes += (size_t)clusters[s].n_nodes;
  // KSS_SWEEP_PIPE (more than one chunk): two halves of chunk rows per scenario within the same
  // budget, the next chunk's static words computed on a second stream while k_simple runs this one.
  // Off by default: C5 ran 13.5 against 12.6 ms per step (r5y: k_simple slows by more than the
  // k_static time it hides when both share the CUs)
  if (simple) hipSetDevice(device);  // the budget follows this device's free memory
  sw->chunk = simple ? static_chunk(sum_nodes, sw->max_pods) : 0;
  const bool dbl = simple && sw->chunk < sw->max_pods && opt(O_SWEEP_PIPE) != 0;
  if (dbl) sw->chunk = static_chunk(2 * sum_nodes, sw->max_pods);
  const int halves = dbl ? 2 : 1;
  if (simple) {
    dry.put<uint32_t>(nullptr, (size_t)halves * sw->chunk * sum_nodes + 4 * (size_t)n_scen);  // + 16-byte alignment per scenario
    sw->stat_off = dry.last;
  }
  const size_t total = dry.o;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&sw->st, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&sw->e0) != hipSuccess || hipEventCreate(&sw->e1) != hipSuccess ||
      (dbl && hipStreamCreateWithFlags(&sw->st2, hipStreamNonBlocking) != hipSuccess)) {
    fail(KSS_E_DEVICE, "stream/event creation failed");
    return nullptr;
  }
  if (hipMalloc(&sw->arena, total) != hipSuccess) {
    sw->arena = nullptr;
    fail(KSS_E_NOMEM, "scenario arena allocation failed");
    return nullptr;
  }
  // host image of [0, up_bytes), packed by scenario in parallel, then one upload
  std::unique_ptr<char[]> img(new (std::nothrow) char[sw->up_bytes]);
  if (!img) {
    fail(KSS_E_NOMEM, "host staging allocation failed");
    return nullptr;
  }
  const int nth = std::max(1, std::min<int>(16, (int)std::thread::hardware_concurrency()));
  auto work = [&](int t) {
    for (int s = t; s < n_scen; s += nth) {
      Packer P{img.get(), sw->arena, in_off[s]};
      pack_inputs(P, &clusters[s], &podsets[s], simple ? &spods[s] : nullptr, jobs[s]);
      // host bytes at the pristine position, device pointers at the live position
      Packer M{img.get(), sw->arena + (sw->live_off - sw->pristine_off), mut_off[s]};
      pack_mutable(M, &clusters[s], jobs[s]);
      DevJob& j = jobs[s];
      j.n_pods = podsets[s].n_pods;
      j.commit = 1;
      j.keep_norm = 0;
      j.record = 0;
      j.prof = *prof;
      j.slots = nullptr;  // no per-node records in a sweep (record = keep_norm = 0)
      j.slot_bytes = 0;
      j.stat = nullptr;
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nth; t++) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  size_t o_chosen = 0, o_stat = 0;
  for (int s = 0; s < n_scen; s++) {
    jobs[s].chosen = reinterpret_cast<int32_t*>(sw->arena + sw->chosen_off) + o_chosen;
    jobs[s].meta = reinterpret_cast<PodMeta*>(sw->arena + sw->meta_off) + o_chosen;
    jobs[s].cursor = reinterpret_cast<int32_t*>(sw->arena + sw->cursor_off) + s;
    o_chosen += (size_t)podsets[s].n_pods;
    if (simple) {
      jobs[s].stat = reinterpret_cast<uint32_t*>(sw->arena + sw->stat_off) + o_stat;
      o_stat += ((size_t)halves * sw->chunk * (size_t)clusters[s].n_nodes + 3) / 4 * 4;  // 16-byte aligned per scenario
    }
  }
  memcpy(img.get() + sw->jobs_off, jobs.data(), sizeof(DevJob) * n_scen);
  if (hipMemcpy(sw->arena, img.get(), sw->up_bytes, hipMemcpyHostToDevice) != hipSuccess) {
    fail(KSS_E_DEVICE, "sweep upload failed");
    return nullptr;
  }
  sw->stage_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return sw.release();
}

int kss_sweep_run(kss_sweep* sw, int32_t* chosen_out, double* device_ms) {
  if (!sw || (sw->total_pods && !chosen_out)) return fail(KSS_E_INVAL, "bad arguments");
  HIP_TRY(hipSetDevice(sw->device));
  hipStream_t st = sw->st;
  HIP_TRY(hipEventRecord(sw->e0, st));
  // every run starts from the snapshot: all scenarios' mutable columns copied back by the reset
  // kernel (agent-scope loads and stores, then a release: the same hand-off as every other
  // writer of node state, not the runtime's copy engine)
  {
    ResetArgs a{};
    a.dst[0] = reinterpret_cast<uint32_t*>(sw->arena + sw->live_off);
    a.src[0] = reinterpret_cast<const uint32_t*>(sw->arena + sw->pristine_off);
    a.n4[0] = sw->mut_bytes / 4;
    if (a.n4[0]) {
      hipLaunchKernelGGL(k_reset_state, dim3((unsigned)std::min<size_t>(2048, (a.n4[0] + 255) / 256)), dim3(256), 0, st, a);
      HIP_TRY(hipGetLastError());
    }
  }
  int* err = reinterpret_cast<int*>(sw->arena + sw->err_off);
  HIP_TRY(dev_zero(err, 16, st));
  HIP_TRY(dev_zero(sw->arena + sw->cursor_off, 4 * (size_t)sw->n_scen, st));  // every scenario's scheduler starts at node 0
  const DevJob* jobs = reinterpret_cast<const DevJob*>(sw->arena + sw->jobs_off);
  int rc;
  if (sw->simple)
    rc = launch_simple(st, sw->g, sw->n_scen, jobs, sw->prof, sw->max_pods, sw->max_nodes, sw->chunk, nullptr, 0, err, nullptr,
                       nullptr, nullptr, 0, false, nullptr, sw->max_keys, sw->st2, &sw->pev);
  else
    rc = launch_schedule(st, sw->g, sw->n_scen, sw->need.bins_cap + (sw->prof.pct_nodes_to_score < 100 ? 1 : 0),
                         sw->need.general, sw->max_keys, jobs, sw->prof, nullptr, err);
  if (rc) return rc;
  // a pod whose program exceeds the device limits (status 4: k_schedule's plan) fails the call
  // instead of looking unschedulable; the scan writes err[1]
  if (!sw->simple && sw->total_pods) {
    hipLaunchKernelGGL(k_status4, dim3((unsigned)std::min(1024, (sw->total_pods + 255) / 256)), dim3(256), 0, st,
                       reinterpret_cast<const PodMeta*>(sw->arena + sw->meta_off), sw->total_pods, err + 1);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipEventRecord(sw->e1, st));
  if (sw->total_pods)
    HIP_TRY(hipMemcpyAsync(chosen_out, sw->arena + sw->chosen_off, sizeof(int32_t) * sw->total_pods,
                           hipMemcpyDeviceToHost, st));
  int errw[2] = {0, 0};
  HIP_TRY(hipMemcpyAsync(errw, err, sizeof(errw), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, sw->e0, sw->e1));
  if (device_ms) *device_ms = ms;
  if (errw[0]) return fail(KSS_E_DEVICE, "scenario launch aborted");
  if (errw[1]) return fail(KSS_E_UNSUPPORTED, "pod program exceeds the device path's per-pod limits");
  return 0;
}

int kss_sweep_info(kss_sweep* sw, double* stage_ms, int32_t* kernel, int64_t* upload_bytes) {
  if (!sw) return fail(KSS_E_INVAL, "null sweep");
  if (stage_ms) *stage_ms = sw->stage_ms;
  if (kernel) *kernel = sw->simple ? 1 : 0;
  if (upload_bytes) *upload_bytes = (int64_t)sw->up_bytes;
  return 0;
}

void kss_sweep_destroy(kss_sweep* sw) {
  if (!sw) return;
  hipSetDevice(sw->device);
  delete sw;
}

int kss_schedule_scenarios(int32_t device, const kss_profile* prof, int32_t n_scen, const kss_cluster* clusters,
                           const kss_podset* podsets, int32_t* chosen_out, double* device_ms) {
  if (!prof || n_scen < 0 || (n_scen && (!clusters || !podsets || !chosen_out))) return fail(KSS_E_INVAL, "bad arguments");
  int rc = check_profile(prof);
  if (rc) return rc;
  if (n_scen == 0) return 0;
  kss_sweep* sw = kss_sweep_create(device, prof, n_scen, clusters, podsets);
  if (!sw) return g_rc ? g_rc : KSS_E_INVAL;
  rc = kss_sweep_run(sw, chosen_out, device_ms);
  kss_sweep_destroy(sw);
  return rc;
}

int kss_load_bound(kss_ctx* ctx, const kss_boundset* bs) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded || !bs || bs->n < 0 || bs->n_ints < 0) return fail(KSS_E_INVAL, "bad arguments");
  if (bs->n && (!bs->id || !bs->node || !bs->priority || !bs->start || !bs->cls || !bs->req || !bs->terms_off ||
                !bs->terms_len))
    return fail(KSS_E_INVAL, "null boundset array");
  std::vector<BoundPod> rows;
  std::vector<int32_t> nodes;
  for (int i = 0; i < bs->n; i++) {
    const int local = bs->node[i] - ctx->dc.node_base;
    if (local < 0 || local >= ctx->dc.N) continue;  // another shard's node
    if (bs->cls[i] < -1 || bs->cls[i] >= ctx->host.n_classes) return fail(KSS_E_INVAL, "bound pod class out of range");
    if (bs->terms_len[i] < 0 || bs->terms_off[i] < 0 || bs->terms_off[i] + bs->terms_len[i] > bs->n_ints ||
        (bs->terms_len[i] && !bs->ints))
      return fail(KSS_E_INVAL, "bound pod terms out of range");
    if (bs->terms_len[i] > 8) return fail(KSS_E_UNSUPPORTED, "a bound pod with more than 8 affinity term rows");
    BoundPod b{};
    b.id = bs->id[i];
    b.start = bs->start[i];
    for (int r = 0; r < KSS_NRES; r++) b.req[r] = bs->req[(size_t)r * bs->n + i];
    b.prio = bs->priority[i];
    b.cls = bs->cls[i];
    b.tlen = bs->terms_len[i];
    if (bs->nonzero) {
      b.nz[0] = bs->nonzero[i];
      b.nz[1] = bs->nonzero[(size_t)bs->n + i];
      b.has_nz = 1;
    }
    b.ports = bs->ports ? bs->ports[i] : 0;
    if (ctx->host.n_ports < KSS_MAX_PORTS && (b.ports >> ctx->host.n_ports))
      return fail(KSS_E_INVAL, "bound pod port bit outside the port dictionary");
    for (int t = 0; t < b.tlen; t++) {
      b.terms[t] = bs->ints[bs->terms_off[i] + t];
      if (b.terms[t] < 0 || b.terms[t] >= ctx->host.n_terms) return fail(KSS_E_INVAL, "bound pod term row out of range");
    }
    rows.push_back(b);
    nodes.push_back(local);
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->bound0.swap(rows);
  ctx->bound0_node.swap(nodes);
  ctx->bound_log.clear();
  ctx->bound_dirty = true;
  return 0;
}

int kss_remove_bound(kss_ctx* ctx, const int64_t* ids, int32_t n) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded || n < 0 || (n > 0 && !ids)) return fail(KSS_E_INVAL, "bad arguments");
  std::lock_guard<std::mutex> lk(ctx->mu);
  // the table as it stands: the loaded rows, then the commits / rollbacks in call order
  std::vector<std::pair<int32_t, BoundPod>> found((size_t)n, {-1, BoundPod{}});
  auto see = [&](int32_t node, const BoundPod& b, bool add) {
    for (int i = 0; i < n; i++)
      if (ids[i] == b.id) found[i] = add ? std::make_pair(node, b) : std::make_pair(-1, BoundPod{});
  };
  for (size_t i = 0; i < ctx->bound0.size(); i++) see(ctx->bound0_node[i], ctx->bound0[i], true);
  for (const BoundOp& op : ctx->bound_log) see(op.node, op.b, op.add != 0);
  for (int i = 0; i < n; i++) {
    if (found[i].first < 0) return fail(KSS_E_INVAL, "id not in the bound-pod table");
    for (int j = 0; j < i; j++)
      if (ids[j] == ids[i]) return fail(KSS_E_INVAL, "id listed twice");
    if (!found[i].second.has_nz) return fail(KSS_E_UNSUPPORTED, "bound pod loaded without nonzero requests");
    if (found[i].second.has_vols) return fail(KSS_E_UNSUPPORTED, "bound pod with volumes (kss_apply_volume_delta)");
  }
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  for (int i = 0; i < n; i++) {
    const BoundPod& b = found[i].second;
    CommitArgs a{};
    for (int r = 0; r < KSS_NRES; r++) a.req[r] = b.req[r];
    a.nz[0] = b.nz[0];
    a.nz[1] = b.nz[1];
    a.port_add = b.ports;
    a.cls = b.cls;
    a.n_own = b.tlen;
    for (int t = 0; t < b.tlen; t++) a.own[t] = b.terms[t];
    a.local = found[i].first;
    a.sign = -1;
    hipLaunchKernelGGL(k_commit, dim3(1), dim3(64), 0, ctx->stream, ctx->dc, a);
    HIP_TRY(hipGetLastError());
    ctx->bound_log.push_back(BoundOp{found[i].first, 0, b});
  }
  ctx->bound_dirty = true;
  return 0;
}

namespace {

// NodeInfo.Pods of every node: the loaded rows, then the commits / rollbacks in call order
// (RemovePod moves the node's last pod into the freed slot), as one CSR upload.
int upload_bound(kss_ctx* ctx) {
  const int N = ctx->dc.N;
  std::vector<std::vector<BoundPod>> per((size_t)N);
  for (size_t i = 0; i < ctx->bound0.size(); i++) per[ctx->bound0_node[i]].push_back(ctx->bound0[i]);
  for (const BoundOp& op : ctx->bound_log) {
    auto& v = per[op.node];
    if (op.add) {
      v.push_back(op.b);
    } else {
      for (size_t k = 0; k < v.size(); k++)
        if (v[k].id == op.b.id) {
          v[k] = v.back();
          v.pop_back();
          break;
        }
    }
  }
  size_t nb = 0, ni = 0;
  for (auto& v : per) {
    nb += v.size();
    for (auto& b : v) ni += b.tlen;
  }
  const size_t NB = std::max(nb, (size_t)1);
  size_t o_ptr = 0, o_id = align_up(4 * (N + 1), 256), o_prio = align_up(o_id + 8 * NB, 256),
         o_start = align_up(o_prio + 4 * NB, 256), o_cls = align_up(o_start + 8 * NB, 256),
         o_req = align_up(o_cls + 4 * NB, 256), o_toff = align_up(o_req + 8 * KSS_NRES * NB, 256),
         o_tlen = align_up(o_toff + 4 * NB, 256), o_ints = align_up(o_tlen + 4 * NB, 256),
         total = align_up(o_ints + 4 * std::max(ni, (size_t)1), 256);
  std::vector<char>& h = ctx->stage_host;
  h.assign(total, 0);
  int32_t* ptr = (int32_t*)(h.data() + o_ptr);
  int64_t* id = (int64_t*)(h.data() + o_id);
  int32_t* prio = (int32_t*)(h.data() + o_prio);
  int64_t* start = (int64_t*)(h.data() + o_start);
  int32_t* cls = (int32_t*)(h.data() + o_cls);
  int64_t* req = (int64_t*)(h.data() + o_req);
  int32_t* toff = (int32_t*)(h.data() + o_toff);
  int32_t* tlen = (int32_t*)(h.data() + o_tlen);
  int32_t* ints = (int32_t*)(h.data() + o_ints);
  size_t e = 0, t = 0;
  std::vector<int32_t> perm;
  for (int n = 0; n < N; n++) {
    ptr[n] = (int32_t)e;
    // the node's pods in MoreImportantPod order (priority descending, start ascending, NodeInfo
    // order on ties — the preemptor does not enter it): SelectVictimsOnNode's reprieve order,
    // and the pods below a priority form a contiguous suffix of it.  Nothing on the device
    // needs NodeInfo order itself (the dry run's sums do not depend on it).
    const auto& v = per[n];
    perm.resize(v.size());
    for (size_t k = 0; k < v.size(); k++) perm[k] = (int32_t)k;
    std::stable_sort(perm.begin(), perm.end(), [&](int32_t a, int32_t b) {
      if (v[a].prio != v[b].prio) return v[a].prio > v[b].prio;
      return v[a].start < v[b].start;
    });
    for (const int32_t pi : perm) {
      const BoundPod& b = v[pi];
      id[e] = b.id;
      prio[e] = b.prio;
      start[e] = b.start;
      cls[e] = b.cls;
      for (int r = 0; r < KSS_NRES; r++) req[e * KSS_NRES + r] = b.req[r];
      toff[e] = (int32_t)t;
      tlen[e] = b.tlen;
      for (int k = 0; k < b.tlen; k++) ints[t++] = b.terms[k];
      e++;
    }
  }
  ptr[N] = (int32_t)e;
  ctx->bound_total = e;
  int rc = ctx->bound_buf.ensure(total);
  if (rc) return rc;
  char* d = (char*)ctx->bound_buf.p;
  HIP_TRY(hipMemcpyAsync(d, h.data(), total, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  DevBound& B = ctx->bound_dev;
  B.ptr = (const int32_t*)(d + o_ptr);
  B.id = (const int64_t*)(d + o_id);
  B.prio = (const int32_t*)(d + o_prio);
  B.start = (const int64_t*)(d + o_start);
  B.cls = (const int32_t*)(d + o_cls);
  B.req = (const int64_t*)(d + o_req);
  B.toff = (const int32_t*)(d + o_toff);
  B.tlen = (const int32_t*)(d + o_tlen);
  B.ints = (const int32_t*)(d + o_ints);
  ctx->bound_dirty = false;
  return 0;
}

}  // namespace

int kss_postfilter_pod(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, kss_preempt_result* out) {
  KSS_SVC_QUIESCE(ctx);
  if (!ctx || !ctx->loaded || !ps || !out) return fail(KSS_E_INVAL, "bad arguments");
  if (pod_index < 0 || pod_index >= ps->n_pods) return fail(KSS_E_INVAL, "pod index out of range");
  if (out->victims_cap < 0 || (out->victims_cap > 0 && !out->victims)) return fail(KSS_E_INVAL, "bad victims buffer");
  if (ctx->state_unknown)
    return fail(KSS_E_INVAL, "node state after a failed run is unknown: kss_reset_node_state or reload first");
  out->status = KSS_PREEMPT_NO_CANDIDATE;
  out->nominated = -1;
  out->n_potential = out->n_candidates = out->n_victims = 0;
  out->highest_priority = 0;
  out->sum_priority = out->earliest_start = 0;
  if (ps->pods[pod_index].flags & KSS_POD_PREEMPT_NEVER) {  // PodEligibleToPreemptOthers
    out->status = KSS_PREEMPT_NOT_ELIGIBLE;
    return 0;
  }
  // the victims' host ports are not in the bound-pod table: a preemptor that wants host ports
  // (NodePorts failures are resolvable by eviction) is refused rather than mis-evaluated
  if (ps->pods[pod_index].port_conflict)
    return fail(KSS_E_UNSUPPORTED, "PostFilter dry run of a pod with host ports (victims' UsedPorts are not tabled)");
  // likewise the victims' volumes (disk conflicts and attach limits are resolvable by eviction)
  if (ps->pods[pod_index].vol_len > 0)
    return fail(KSS_E_UNSUPPORTED, "PostFilter dry run of a pod with volumes (victims' volumes are not tabled)");
  OnePod one;
  int rc = compact_pod(ps, pod_index, one);
  if (rc) return rc;
  if ((rc = validate(&ctx->host, &one.ps, 1))) return rc;
  std::lock_guard<std::mutex> lk(ctx->mu);
  nom_check_podset(ctx, ps);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  rc = upload_podset(ctx->stream, ctx->tmp_pod_buf, &one.ps, ctx->tdp);
  if (rc) return rc;
  if (ctx->bound_dirty && (rc = upload_bound(ctx))) return rc;
  const PlanNeeds need = plan_needs(ctx->key_card_h.data(), ctx->key_flags_h.data(), &one.ps, 1);
  const int bins_cap = std::max(need.bins_cap, 1);
  const size_t lds = sizeof(PreHdr) + 8 * (size_t)bins_cap;
  if (lds > KSS_LDS_BUDGET) return fail(KSS_E_UNSUPPORTED, "the pod's topology histograms exceed LDS");
  const size_t N = (size_t)ctx->dc.N;
  const int cap = out->victims_cap;
  const size_t o_job = 0, o_out = align_up(sizeof(PreemptJob), 256), o_vic = o_out + sizeof(PreemptOut),
               o_key = align_up(o_vic + 8 * (size_t)std::max(cap, 1), 256),
               o_g = align_up(o_key + 5 * 8 * std::max(N, (size_t)1), 256), o_bins = align_up(o_g + sizeof(PreGlobal), 256),
               o_top = align_up(o_bins + 8 * (size_t)bins_cap, 256),
               o_vs = align_up(o_top + 8 * 2 * MAXH * (size_t)PRE_STATS_MAX_BLOCKS, 256),
               total = o_vs + 8 * std::max<size_t>(ctx->bound_total, 1);
  if ((rc = ctx->pre_buf.ensure(total))) return rc;
  char* d = (char*)ctx->pre_buf.p;
  PreemptJob J{};
  J.c = ctx->dc;
  J.c.nc64 = nullptr;
  J.c.nct = nullptr;
  J.c.nc32 = nullptr;
  J.c.ncl = nullptr;
  J.P = ctx->tdp;
  J.B = ctx->bound_dev;
  J.prof = ctx->prof;
  J.pi = 0;
  J.bins_cap = bins_cap;
  J.victims_cap = cap;
  {  // the pod's bin plan, on the host: every kernel copies it instead of rebuilding it on one lane
    DevCluster hc{};
    hc.key_card = ctx->key_card_h.data();
    hc.key_flags = ctx->key_flags_h.data();
    DevPods hp{};
    hp.spreads = one.ps.spreads;
    hp.ipa = one.ps.ipa;
    J.plan_ok = make_plan(hc, hp, one.ps.pods[0], J.plan, bins_cap) ? 1 : 0;
  }
  if (!ctx->nom.empty()) {  // RunFilterPluginsWithNominatedPods in every dry-run filter call
    if (ctx->nom_dirty) {
      if ((rc = ctx->nom_buf.ensure(sizeof(DevNom) * ctx->nom.size()))) return rc;
      HIP_TRY(hipMemcpyAsync(ctx->nom_buf.p, ctx->nom.data(), sizeof(DevNom) * ctx->nom.size(), hipMemcpyHostToDevice,
                             ctx->stream));
      ctx->nom_dirty = false;
    }
    J.nom = (const DevNom*)ctx->nom_buf.p;
    J.n_nom = (int32_t)ctx->nom.size();
  }
  J.pod_id = pod_identity(ps->pods[pod_index], pod_index);
  J.key = (int64_t*)(d + o_key);
  J.n_blocks = (int32_t)std::max<size_t>((N + PRE_NODE_THREADS - 1) / PRE_NODE_THREADS, 1);
  J.victims = (int64_t*)(d + o_vic);
  J.out = (PreemptOut*)(d + o_out);
  J.G = (PreGlobal*)(d + o_g);
  J.gbins = (long long*)(d + o_bins);
  J.stop2 = (long long*)(d + o_top);
  J.vscratch = (int64_t*)(d + o_vs);
  // stats workgroups: about 256 nodes each (the histograms are added into the zeroed HBM bins)
  const unsigned nsb = (unsigned)std::min<size_t>(std::max<size_t>((N + 255) / 256, 1), PRE_STATS_MAX_BLOCKS);
  HIP_TRY(hipMemcpyAsync(d + o_job, &J, sizeof(J), hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
  HIP_TRY(dev_zero(d + o_g, o_top - o_g, ctx->stream));  // PreGlobal (ticket, sums) and the bins
  const PreemptJob* jd = (const PreemptJob*)(d + o_job);
  hipLaunchKernelGGL(k_preempt_stats, dim3(nsb), dim3(256), lds, ctx->stream, jd);  // a lane per node of the range
  const unsigned nb = (unsigned)((N + PRE_NODE_THREADS - 1) / PRE_NODE_THREADS);
  hipLaunchKernelGGL(k_preempt_nodes, dim3(std::max(nb, 1u)), dim3(PRE_NODE_THREADS), sizeof(PreHdr), ctx->stream, jd);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
  const size_t back = sizeof(PreemptOut) + 8 * (size_t)cap;
  if (ctx->pinned_cap < back) {
    if (ctx->pinned) hipHostFree(ctx->pinned);
    ctx->pinned = nullptr;
    ctx->pinned_cap = 0;
    HIP_TRY(hipHostMalloc(&ctx->pinned, back));
    ctx->pinned_cap = back;
  }
  HIP_TRY(hipMemcpyAsync(ctx->pinned, d + o_out, back, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  ctx->last_ms = ms;
  ctx->last_launches = 2;
  ctx->last_kernel = 3;
  PreemptOut o;
  std::memcpy(&o, ctx->pinned, sizeof(o));
  if (o.status < 0) return fail(KSS_E_UNSUPPORTED, "pod program exceeds the device path's per-pod limits");
  out->status = o.status;
  out->nominated = o.nominated;
  out->n_potential = o.n_potential;
  out->n_candidates = o.n_candidates;
  out->n_victims = o.n_victims;
  out->highest_priority = o.highest_priority;
  out->sum_priority = o.sum_priority;
  out->earliest_start = o.earliest_start;
  if (o.status == KSS_PREEMPT_NOMINATED && cap > 0)
    std::memcpy(out->victims, (char*)ctx->pinned + sizeof(PreemptOut), 8 * (size_t)std::min(cap, o.n_victims));
  return 0;
}

int kss_set_names(kss_ctx* ctx, const kss_names* names) {
  if (!ctx || !names) return fail(KSS_E_INVAL, "bad arguments");
  return kss_host_set_names(&ctx->names, names, ctx->host.n_nodes, ctx->host.n_taints, ctx->host.n_scalar);
}

int kss_format_annotations(kss_ctx* ctx, const kss_pod_result* res, int32_t n_nodes, char* buf, size_t cap, size_t* need) {
  if (!ctx || !res || !need) return fail(KSS_E_INVAL, "bad arguments");
  return kss_host_format(&ctx->names, &ctx->prof, res, n_nodes, buf, cap, need);
}

int kss_format_pod_annotations(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, const kss_pod_result* res,
                               int32_t n_nodes, char* buf, size_t cap, size_t* need) {
  if (!ctx || !res || !need) return fail(KSS_E_INVAL, "bad arguments");
  std::vector<int> pf;
  int has = 0;
  if (kss_host_prefilter_nodes(ps, pod_index, n_nodes, &pf, &has)) return fail(KSS_E_INVAL, "bad pod index or node set");
  return kss_host_format(&ctx->names, &ctx->prof, res, n_nodes, buf, cap, need, has ? &pf : nullptr, &ps->pods[pod_index]);
}

}  // extern "C"

int kss_device_go_log(int32_t device, const double* x, double* y, int32_t n) {
  if (!x || !y || n < 0) return fail(KSS_E_INVAL, "bad arguments");
  if (n == 0) return 0;
  HIP_TRY(hipSetDevice(device));
  double* d = nullptr;
  HIP_TRY(hipMalloc(&d, 16 * (size_t)n));
  std::unique_ptr<double, void (*)(double*)> hold(d, [](double* p) { hipFree(p); });
  HIP_TRY(hipMemcpy(d, x, 8 * (size_t)n, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_go_log, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr, d, d + n, n);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpy(y, d + n, 8 * (size_t)n, hipMemcpyDeviceToHost));
  return 0;
}

int kss_plan_podset(const kss_cluster* cl, const kss_podset* ps, int32_t* out3) {
  if (!cl || !ps || !out3) return fail(KSS_E_INVAL, "bad arguments");
  int rc = check_cluster(cl);
  if (rc) return rc;
  if ((rc = validate(cl, ps, ps->n_pods))) return rc;
  std::vector<SPod> sp;
  out3[0] = 0;
  out3[1] = -1;
  out3[2] = GP_OK;
  if (build_spods(ps, cl->n_scalar, sp)) {
    out3[0] = 1;
    return 0;
  }
  std::vector<uint4> words;
  GpodNeeds need;
  if (build_gpods(ps, cl->n_scalar, cl->n_classes, cl->key_card, cl->key_flags, cl->key_empty, words, need)) {
    out3[0] = 2;
    return 0;
  }
  out3[1] = need.fail_pod;
  out3[2] = need.fail_code;
  return 0;
}

int kss_plan_podset_ex(const kss_cluster* cl, const kss_podset* ps, const kss_profile* prof, int32_t* out3) {
  if (!prof) return kss_plan_podset(cl, ps, out3);
  if (int rc = check_profile(prof)) return rc;
  if (int rc = kss_plan_podset(cl, ps, out3)) return rc;
  if (out3[0] == 0) return 0;  // the programs already rule out both loop kernels
  // the window (percentageOfNodesToScore < 100 on a list long enough to stop early) runs on k_simple
  // (simple_sync_win) and, under the default profile, on k_spread (spread_schedule WIN) for pods
  // without a PreFilterResult node list
  int names_pod = -1;
  for (int i = 0; i < ps->n_pods && names_pod < 0; i++)
    if (ps->pods[i].names_len >= 0) names_pod = i;
  const bool win = num_feasible_to_find(cl->n_nodes, prof->pct_nodes_to_score) < cl->n_nodes;
  const bool spread_def = out3[0] == 2 && same_profile(*prof, default_profile_c()) && !opt(O_FOLD);
  if (win && ((out3[0] == 2 && !spread_def) || names_pod >= 0)) {
    out3[1] = names_pod >= 0 ? names_pod : (ps->n_pods > 0 ? 0 : -1);
    out3[0] = 0;
    out3[2] = GP_PCT;
  } else if (!scalar_fast_ok(*prof, cl->n_scalar)) {
    out3[0] = 0;
    out3[1] = ps->n_pods > 0 ? 0 : -1;
    out3[2] = GP_SCALAR_SCORED;
  }
  return 0;
}

const char* kss_plan_reason(int32_t code) { return code >= 0 && code < GP_NCODES ? kGpReason[code] : "unknown"; }
