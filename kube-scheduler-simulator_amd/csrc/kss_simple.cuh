// kss_simple.cuh — the sequential scheduling loop for batches without PodTopologySpread /
// InterPodAffinity programs (the default-profile workload of BASELINE C1/C2/C5), built
// around ONE cross-shard exchange per pod.
//
// Same semantics as schedule_pod<false> (kss_sched.cuh), split in two kernels:
//
//   k_static  (massively parallel, one lane per (pod, node)): everything of a pod's
//             evaluation that no commit can change — the NodeUnschedulable, NodeName,
//             TaintToleration and NodeAffinity filters (node flags, taints and labels are
//             not touched by AssumePod) and the raw TaintToleration and NodeAffinity
//             scores — packed in one 32-bit "static word" per (pod, node) in HBM.
//   k_simple  (persistent, one workgroup per shard of W): the sequential loop.  Per pod it
//             only evaluates what the state changes: the NodeResourcesFit filter, the Fit
//             and BalancedAllocation scores (exact reciprocal arithmetic, kss_fastmath.cuh),
//             then NormalizeScore, the packed selectHost key and the commit.
//
// The persistent loop:
//   * the shard's node rows and their Allocatable reciprocals live in LDS for the launch;
//   * the compact pod records (SPod) and the static words of pod k+2 are loaded into
//     registers while pod k is scheduled and stored into 3-slot LDS rings at its end;
//   * pod k's argmax and pod k+1's normalisation statistics travel in the same exchange.
//     Pod k+1's statistics depend on pod k's commit, which touches one node only: the
//     winner, which is some shard's local best.  Each shard therefore evaluates pod k+1
//     on its local best node twice — before the commit (H0) and after it (H1) — and
//     publishes both statistic sets next to its pod-k key.  Once the global winner is
//     known, the winner's shard contributes H1 and every other shard H0, which is the
//     statistic of pod k+1 on the committed state.
#pragma once
#include "kss_fastmath.cuh"
#include "kss_sched.cuh"

namespace kss {

// Global-memory accesses of the persistent loop go through address-space-1 pointers:
// from a generic pointer the compiler emits flat instructions, which also count in
// lgkmcnt, so every LDS-only barrier (s_waitcnt lgkmcnt(0)) would wait for the HBM
// prefetches and the commit's atomics.
#define KSS_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ KSS_GLOBAL T* gp(T* p) {
  return (KSS_GLOBAL T*)p;
}

// Node state and static words handed from one launch to the next (k_static -> loop kernel,
// a chunk's write-back -> the next chunk's load, a reset copy -> the first load) go through
// agent-scope (sc1) stores and loads: the per-XCD L2s are not coherent with each other, and a
// line a workgroup of an earlier launch left in its XCD's L2 must not satisfy a later load on
// that XCD.  (Observed: a split-grid run reading one stale class count at a chunk boundary.)
// (through address-space-1 pointers: a flat access would also count in lgkmcnt, and every
// following LDS wait would then wait on it)
template <class T>
__device__ __forceinline__ T ld_ag(const T* p) {
  return __hip_atomic_load(gp(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ T ld_ag(KSS_GLOBAL const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void st_ag(T* p, T v) {
  __hip_atomic_store(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The ends of a launch-to-launch hand-off of node state (a chunk's write-back -> the next
// chunk's load, k_static -> the loop kernel, a reset / delta -> the next launch), in the
// producer / consumer forms of MI355X_MICROARCH.md ("Valid forms"): every storing wave
// waits for its own stores, then (after a workgroup barrier where the caller has one) an
// agent-scope release writes the XCD's L2 back; the consumer starts with an agent-scope
// acquire.  The kernel boundary alone did not order them under a concurrent split-grid part
// (DESIGN §5).
__device__ __forceinline__ void handoff_drain() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void handoff_release() {  // whole workgroup, no thread exited
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) handoff_drain();
}
__device__ __forceinline__ void handoff_acquire() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ int xcc_id() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xF;
}

// Publish one granule at offset `off` of the exchange buffer (the local inbox `gran`);
// address-space-1 stores (a flat store would also count in lgkmcnt).  An XCD-local grid
// (X.xcd_local: every shard runs on the same XCD, xcd_slot) publishes with a plain store (no
// cache-policy bits): the line stays in that XCD's L2, which every shard's agent-scope
// (L1-bypassing) poll reads -- a third of the latency of a write-through granule
// (tools/xcd_exchange_probe.hip, 32-way rounds: 0.41 against 1.23 us).
__device__ __forceinline__ void xpub(const XPeers& X, unsigned long long* gran, size_t off, unsigned long long v) {
  if (X.n <= 1) {
    if (X.xcd_local) asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(gran + off), "v"(v) : "memory");
    else __hip_atomic_store(gp(gran) + off, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  for (int p = 0; p < X.n; p++) __hip_atomic_store(gp(X.inbox[p]) + off, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr int SX_VALS = 8;    // granules per shard per exchange: key lo/hi, H0 (nf, tt, na), H1 (nf, tt, na)

// An XCD-local k_simple grid (one cluster, W <= CUs per XCD): the launch has XCD_GRID_MULT x W
// workgroups; the first W that run on XCD 0 become shards 0 .. W-1 in arrival order and every
// other workgroup leaves at once.  Correctness never rests on where the hardware places a
// workgroup: a shard is one that READ its XCC id as 0, so all shards share XCD 0's L2.  When
// XCD 0 gets fewer than W of them (counted once every workgroup of the grid has started), the
// launch fails with err = 3 before touching any state and the host runs it again unrestricted.
// ctr: two zeroed words behind the launch's granules, [0] shards taken, [1] workgroups started.
// Returns the shard, -1 (leave), -2 (placement failed).  force_fail (kss_set_option
// "xcd_force_fallback", tests): workgroup 0 reports failed placement and every workgroup leaves,
// so the host's unrestricted rerun is what schedules the batch.
constexpr int XCD_GRID_MULT = 8;
__device__ __forceinline__ int xcd_slot(int* ctr, int W, int grid, int* err, bool force_fail = false) {
  if (force_fail) {
    if (blockIdx.x == 0) err_raise(err, 3);
    return blockIdx.x == 0 ? -2 : -1;
  }
  int slot = -1;
  if (xcc_id() == 0) {
    slot = atomicAdd(&ctr[0], 1);
    if (slot >= W) slot = -1;
  }
  atomicAdd(&ctr[1], 1);  // after the slot: every workgroup started => every XCD-0 slot taken
  if (slot < 0) return -1;
  long long t0 = 0;
  for (unsigned spins = 0;; ++spins) {
    if (__hip_atomic_load(&ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= W) return slot;
    if (__hip_atomic_load(&ctr[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= grid &&
        __hip_atomic_load(&ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < W)
      break;
    if (spin_expired(spins, t0)) break;
    __builtin_amdgcn_s_sleep(1);
  }
  err_raise(err, 3);
  return -2;
}
constexpr int SX_CHUNKS = 2;  // shards swept 64 at a time: W <= 128
constexpr int STATIC_PODS = 8;  // pods per k_static lane
constexpr int PF_MAX = 8;       // static words per prefetch lane (host-checked: simple_fits)

// The v1.26 default profile (kss_default_profile, kss_host.cpp; plugins_test.go:184-204,
// 878-1096) as a compile-time constant: k_simple<true> folds every weight and resource
// choice of the scoring path into the code.
__host__ __device__ constexpr kss_profile default_profile_c() {
  kss_profile p{};
  p.weight[KSS_S_TAINT_TOLERATION] = 3;
  p.weight[KSS_S_NODE_AFFINITY] = 2;
  p.weight[KSS_S_NODE_RESOURCES_FIT] = 1;
  p.weight[KSS_S_VOLUME_BINDING] = 1;
  p.weight[KSS_S_POD_TOPOLOGY_SPREAD] = 2;
  p.weight[KSS_S_INTER_POD_AFFINITY] = 2;
  p.weight[KSS_S_BALANCED_ALLOCATION] = 1;
  p.weight[KSS_S_IMAGE_LOCALITY] = 1;
  for (int i = 1; i <= KSS_NFILTER; i++) p.filter_enabled |= 1u << i;
  p.score_enabled = (1u << KSS_NSCORE) - 1;
  p.fit_strategy = KSS_FIT_LEAST_ALLOCATED;
  p.fit_n = 2;
  p.fit_res[0] = KSS_RES_CPU;
  p.fit_res[1] = KSS_RES_MEMORY;
  p.fit_weight[0] = 1;
  p.fit_weight[1] = 1;
  p.ba_n = 2;
  p.ba_res[0] = KSS_RES_CPU;
  p.ba_res[1] = KSS_RES_MEMORY;
  p.hard_pod_affinity_weight = 1;
  p.pct_nodes_to_score = 100;
  p.system_defaulted = 1;
  return p;
}

// Compact per-pod record of the simple path (host: build_spods): only what the
// state-dependent part of the cycle reads.  Quantities are integers held in doubles: the
// host admits a batch to this path only if every operand and every sum the loop can form
// stays below 2^53 (exact_f64 in kss_lib.hip), so all arithmetic on them is exact.
constexpr int32_t SP_ALLZERO = 1;  // computePodResourceRequest is all zero: fitsRequest checks pods only
struct SPod {
  double fit_req[3];  // NodeResourcesFit PreFilter request cpu / memory / ephemeral
  double snz[3];      // LeastAllocated request (non-zero defaults)
  double sreq[3];     // BalancedAllocation request
  double creq[3];     // AssumePod Requested delta
  double cnz[2];      // AssumePod NonZeroRequested delta
  int32_t flags;       // SP_*
  int32_t status;      // kss_pod.prefilter_status
  int32_t cls;         // class_count row the pod joins (-1 none)
  int32_t own_off, own_len;  // term_count rows it adds: ints[own_off .. +own_len) of the staged pool
  int32_t pad[3];
  int64_t sc_fit[KSS_MAX_SCALAR];  // NodeResourcesFit PreFilter request of each extended (scalar) resource
  int64_t sc_req[KSS_MAX_SCALAR];  // AssumePod Requested delta of each scalar resource
};
static_assert(sizeof(SPod) % 16 == 0, "SPod is copied as uint4");

// Static word of one (pod, node):
//   bits 0-2   the first failing static filter: 0 pass, 1-4 KSS_F_NODE_UNSCHEDULABLE ..
//              KSS_F_NODE_AFFINITY, 7 not evaluated (PreFilter failure, or outside the
//              NodeAffinity PreFilterResult);
//   bit 3      the pod's required node affinity matches the node (PodTopologySpread
//              NodeAffinityPolicy=Honor), bit 4 its NoSchedule/NoExecute taints are all
//              tolerated (NodeTaintsPolicy=Honor) — for every node, whatever bits 0-2 say;
//   bits 5-11  raw TaintToleration (<= 64), bits 12-31 raw NodeAffinity (host-checked:
//              Σ preferred weights < 2^20); both 0 unless bits 0-2 are 0.
constexpr uint32_t SW_NOT_EVALUATED = 7, SW_AFF_OK = 1u << 3, SW_TAINT_OK = 1u << 4;
__device__ __forceinline__ int sw_code(uint32_t w) {
  const int c = (int)(w & 7u);
  return c == (int)SW_NOT_EVALUATED ? KSS_F_NOT_EVALUATED : c;
}
__device__ __forceinline__ int sw_tt(uint32_t w) { return (int)((w >> 5) & 0x7Fu); }
__device__ __forceinline__ int sw_na(uint32_t w) { return (int)(w >> 12); }

// lab(key): the node's interned label value (label_of by default; k_static reads an LDS copy)
template <class Lab>
__device__ __forceinline__ uint32_t static_word_l(const DevCluster& c, const DevPods& P, const kss_pod& p,
                                                  const kss_profile& prof, int n, uint32_t flags, uint64_t th,
                                                  uint64_t ts, Lab lab) {
  const int64_t g = (int64_t)c.node_base + n;
  if (p.prefilter_status != 0) return SW_NOT_EVALUATED;
  const bool aff = required_affinity_t(c, P.reqs, P.terms, P.ints, p, g, lab);
  const bool tol = (th & ~p.tol_hard) == 0;
  const uint32_t pol = (aff ? SW_AFF_OK : 0u) | (tol ? SW_TAINT_OK : 0u);
  if (p.names_len >= 0) {  // NodeAffinity PreFilterResult: nodes outside the set are not evaluated
    bool in = false;
    for (int i = 0; i < p.names_len; i++) in |= (int64_t)P.ints[p.names_off + i] == g;
    if (!in) return pol | SW_NOT_EVALUATED;
  }
  const uint32_t en = prof.filter_enabled;
  // RunFilterPlugins order (plugin_test.go:15-36): the first four filters are static
  if (((en >> KSS_F_NODE_UNSCHEDULABLE) & 1u) && (flags & KSS_NODE_UNSCHEDULABLE) && !(p.flags & KSS_POD_TOL_UNSCHEDULABLE))
    return pol | KSS_F_NODE_UNSCHEDULABLE;
  if (((en >> KSS_F_NODE_NAME) & 1u) && p.node_name != -1 && (int64_t)p.node_name != g) return pol | KSS_F_NODE_NAME;
  if (((en >> KSS_F_TAINT_TOLERATION) & 1u) && !tol) return pol | KSS_F_TAINT_TOLERATION;
  if (((en >> KSS_F_NODE_AFFINITY) & 1u) && !aff) return pol | KSS_F_NODE_AFFINITY;
  const uint32_t tt = (uint32_t)__popcll(ts & ~p.tol_soft);                         // TaintToleration.Score
  const uint32_t na = (uint32_t)na_score_t(c, P.reqs, P.terms, P.ints, p, g, lab);  // NodeAffinity.Score
  return pol | (tt << 5) | (na << 12);
}

__device__ __forceinline__ uint32_t static_word(const DevCluster& c, const DevPods& P, const kss_pod& p,
                                                const kss_profile& prof, int n, uint32_t flags, uint64_t th,
                                                uint64_t ts) {
  return static_word_l(c, P, p, prof, n, flags, th, ts, [&](int key) { return label_of(c, key, n); });
}

// k_static's form: the words of one pod on a lane's four nodes at once.  Every requirement of
// the pod is decoded once (scalar loads of the wave-uniform program) and matched against the
// four nodes' label values into a 4-bit mask, so the pod's program is walked once per lane
// instead of once per node and no loop diverges between the four nodes.  Word for word equal
// to static_word_l (req_match_t / required_affinity_t / na_score_t, kss_eval.cuh).
// lab(key, i): the label value id of node g[i] (-1 absent).
// The pod program is read through constant-address-space pointers (DevPodsK): a wave-uniform
// address there becomes a scalar load (the program never changes during a launch); through
// generic pointers every field was a per-lane flat load (k_static r6a: 557 vector loads per
// wave, waves waiting 77 % of their cycles).
#define KSS_CONST __attribute__((address_space(4)))
struct DevPodsK {
  const KSS_CONST kss_pod* pods;
  const KSS_CONST kss_req* reqs;
  const KSS_CONST kss_term* terms;
  const KSS_CONST int32_t* ints;
};
__device__ __forceinline__ DevPodsK pods_k(const DevPods& P) {
  return DevPodsK{(const KSS_CONST kss_pod*)P.pods, (const KSS_CONST kss_req*)P.reqs,
                  (const KSS_CONST kss_term*)P.terms, (const KSS_CONST int32_t*)P.ints};
}
template <class Ints, class Req, class Lab4>
__device__ __forceinline__ uint32_t req_mask4(const DevCluster& c, Ints ints, const Req& r,
                                              const int64_t (&g)[4], Lab4 lab) {
  const int op = r.op;
  if (op == KSS_OP_FALSE) return 0u;
  if (op == KSS_OP_TRUE) return 15u;
  uint32_t m = 0;
  if (op == KSS_OP_NAME_IN || op == KSS_OP_NAME_NOTIN) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const bool hit = r.ival >= 0 && g[i] == r.ival;
      m |= (uint32_t)(op == KSS_OP_NAME_IN ? hit : !hit) << i;
    }
    return m;
  }
  int32_t v[4];
#pragma unroll
  for (int i = 0; i < 4; i++) v[i] = lab(r.key, i);
  switch (op) {
    case KSS_OP_MASK:
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint64_t b = v[i] < 0 ? (r.mask >> 63) : (v[i] < 63 ? (r.mask >> v[i]) : 0ull);
        m |= (uint32_t)(b & 1ull) << i;
      }
      return m;
    case KSS_OP_IN:
    case KSS_OP_NOTIN: {
      uint32_t hit = 0;
      for (int j = 0; j < r.list_len; j++) {
        const int32_t x = ints[r.list_off + j];
#pragma unroll
        for (int i = 0; i < 4; i++) hit |= (uint32_t)(x == v[i]) << i;
      }
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const bool b = ((hit >> i) & 1u) != 0;
        m |= (uint32_t)(op == KSS_OP_IN ? (v[i] >= 0 && b) : (v[i] < 0 || !b)) << i;
      }
      return m;
    }
    case KSS_OP_EXISTS:
    case KSS_OP_DNE:
#pragma unroll
      for (int i = 0; i < 4; i++) m |= (uint32_t)((v[i] >= 0) == (op == KSS_OP_EXISTS)) << i;
      return m;
    case KSS_OP_GT:
    case KSS_OP_LT:
#pragma unroll
      for (int i = 0; i < 4; i++) {
        if (v[i] < 0) continue;
        const int32_t gi = gp(c.key_base)[r.key] + v[i];
        if (!gp(c.value_is_int)[gi]) continue;
        const int64_t x = gp(c.value_int)[gi];
        m |= (uint32_t)(op == KSS_OP_GT ? x > r.ival : x < r.ival) << i;
      }
      return m;
    default:
      return 0u;
  }
}

template <class PV, class Term, class Lab4>
__device__ __forceinline__ uint32_t term_mask4(const DevCluster& c, const PV& P, const Term& t,
                                               const int64_t (&g)[4], Lab4 lab) {
  uint32_t m = 15u;
  for (int i = 0; i < t.req_len; i++) m &= req_mask4(c, P.ints, P.reqs[t.req_off + i], g, lab);
  return m;
}

// words w[i] of pod p on nodes n + min(i, cnt - 1), i < 4 (flags / th / ts: those nodes' columns)
template <class PV, class Pod, class Lab4>
__device__ __forceinline__ void static_words4(const DevCluster& c, const PV& P, const Pod& p,
                                              const kss_profile& prof, int n, int cnt, const uint32_t (&flags)[4],
                                              const uint64_t (&th)[4], const uint64_t (&ts)[4], Lab4 lab,
                                              uint32_t (&w)[4]) {
  if (p.prefilter_status != 0) {
#pragma unroll
    for (int i = 0; i < 4; i++) w[i] = SW_NOT_EVALUATED;
    return;
  }
  int64_t g[4];
#pragma unroll
  for (int i = 0; i < 4; i++) g[i] = (int64_t)c.node_base + n + min(i, cnt - 1);
  // nodeaffinity.RequiredNodeAffinity.Match: nodeSelector AND (OR over terms)
  uint32_t aff = 15u;
  for (int i = 0; i < p.sel_len; i++) aff &= req_mask4(c, P.ints, P.reqs[p.sel_off + i], g, lab);
  if (p.flags & KSS_POD_HAS_REQ_AFFINITY) {
    uint32_t any = 0;
    for (int t = 0; t < p.aff_len; t++) any |= term_mask4(c, P, P.terms[p.aff_off + t], g, lab);
    aff &= any;
  }
  uint32_t in = 15u;  // NodeAffinity PreFilterResult
  if (p.names_len >= 0) {
    in = 0;
    for (int j = 0; j < p.names_len; j++) {
      const int64_t x = (int64_t)P.ints[p.names_off + j];
#pragma unroll
      for (int i = 0; i < 4; i++) in |= (uint32_t)(x == g[i]) << i;
    }
  }
  uint32_t na[4] = {0, 0, 0, 0};  // NodeAffinity.Score
  for (int t = 0; t < p.pref_len; t++) {
    const auto& term = P.terms[p.pref_off + t];
    const uint32_t tm = term_mask4(c, P, term, g, lab);
#pragma unroll
    for (int i = 0; i < 4; i++)
      if ((tm >> i) & 1u) na[i] += (uint32_t)term.weight;
  }
  const uint32_t en = prof.filter_enabled;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const bool a = (aff >> i) & 1u;
    const bool tol = (th[i] & ~p.tol_hard) == 0;
    const uint32_t pol = (a ? SW_AFF_OK : 0u) | (tol ? SW_TAINT_OK : 0u);
    uint32_t r;
    if (!((in >> i) & 1u)) r = pol | SW_NOT_EVALUATED;
    else if (((en >> KSS_F_NODE_UNSCHEDULABLE) & 1u) && (flags[i] & KSS_NODE_UNSCHEDULABLE) && !(p.flags & KSS_POD_TOL_UNSCHEDULABLE))
      r = pol | KSS_F_NODE_UNSCHEDULABLE;
    else if (((en >> KSS_F_NODE_NAME) & 1u) && p.node_name != -1 && (int64_t)p.node_name != g[i])
      r = pol | KSS_F_NODE_NAME;
    else if (((en >> KSS_F_TAINT_TOLERATION) & 1u) && !tol)
      r = pol | KSS_F_TAINT_TOLERATION;
    else if (((en >> KSS_F_NODE_AFFINITY) & 1u) && !a)
      r = pol | KSS_F_NODE_AFFINITY;
    else
      r = pol | ((uint32_t)__popcll(ts[i] & ~p.tol_soft) << 5) | (na[i] << 12);
    w[i] = r;
  }
}

// One (pod, node) result of the compact path: filter verdict and raw scores.
struct SVal {
  int f, tt, na, fit, ba;
};

// A node row as the state-dependent filter and scores read it.
struct DynRow {
  double alloc[3], req[3], nz[2];
  double inv[3];  // RN(1 / alloc), 0 for alloc 0
  int32_t pods, allowed;
};

// v[r] of a three-element row for a runtime resource id r in [0, 3), as masks: a select
// chain would be folded back into an indexed access, which puts the row in scratch.
__device__ __forceinline__ int64_t pick3m(int r, int64_t a, int64_t b, int64_t c) {
  return (a & -(int64_t)(r == 0)) | (b & -(int64_t)(r == 1)) | (c & -(int64_t)(r == 2));
}
__device__ __forceinline__ double pick3d(int r, double a, double b, double c) {
  return __longlong_as_double(pick3m(r, __double_as_longlong(a), __double_as_longlong(b), __double_as_longlong(c)));
}

// NodeResourcesFit.Score (resourceAllocationScorer.score, useRequested=false, no scalar
// resources on this path: calculateResourceAllocatableRequest skips them at request 0).
__device__ __forceinline__ int32_t fit_fast(const kss_profile& prof, const SPod& q, const DynRow& r) {
  int32_t node_score = 0, weight_sum = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (i >= prof.fit_n) break;
    const int res = prof.fit_res[i];
    if (res >= KSS_RES_SCALAR0) continue;
    const double A = pick3d(res, r.alloc[0], r.alloc[1], r.alloc[2]);
    if (A == 0.0) continue;
    const double base = pick3d(res, r.nz[0], r.nz[1], r.req[2]);
    const double inv = pick3d(res, r.inv[0], r.inv[1], r.inv[2]);
    const double preq = pick3d(res, q.snz[0], q.snz[1], q.snz[2]);
    const int32_t w = (int32_t)prof.fit_weight[i];
    node_score += alloc_score_d(prof.fit_strategy, base + preq, A, inv) * w;
    weight_sum += w;
  }
  if (weight_sum <= 1) return weight_sum == 0 ? 0 : node_score;
  if (weight_sum == 2) return node_score >> 1;
  return small_div(node_score, weight_sum, __builtin_amdgcn_rcpf((float)weight_sum));
}

// NodeResourcesBalancedAllocation.Score (balancedResourceScorer, useRequested=true); the
// float64 operations in the reference's order, divisions correctly rounded (div_rn).
__device__ __forceinline__ int32_t ba_fast(const kss_profile& prof, const SPod& q, const DynRow& r) {
  double fr[4] = {0.0, 0.0, 0.0, 0.0};
  bool use[4] = {false, false, false, false};
  int nf = 0;
  double total = 0.0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (i >= prof.ba_n) break;
    const int res = prof.ba_res[i];
    if (res >= KSS_RES_SCALAR0) continue;
    const double A = pick3d(res, r.alloc[0], r.alloc[1], r.alloc[2]);
    if (A == 0.0) continue;
    const double R = pick3d(res, r.req[0], r.req[1], r.req[2]) + pick3d(res, q.sreq[0], q.sreq[1], q.sreq[2]);
    const double inv = pick3d(res, r.inv[0], r.inv[1], r.inv[2]);
    double f = div_rn_d(R, A, inv);
    if (f > 1.0) f = 1.0;
    total += f;
    fr[i] = f;
    use[i] = true;
    nf++;
  }
  double sd = 0.0;
  if (nf == 2) {
    double a = 0.0, b = 0.0;
    bool got = false;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if (!use[i]) continue;
      if (!got) {
        a = fr[i];
        got = true;
      } else {
        b = fr[i];
      }
    }
    sd = fabs((a - b) / 2.0);
  } else if (nf > 2) {
    const double mean = total / (double)nf;
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if (!use[i]) continue;
      const double d = fr[i] - mean;
      const double sq = d * d;
      sum = sum + sq;
    }
    sd = sqrt(sum / (double)nf);
  }
  return (int32_t)((1.0 - sd) * 100.0);  // in [0, 100]: int32 truncation == int64(...)
}

// The state-dependent rest of one evaluation: NodeResourcesFit.Filter (fitsRequest) and
// the Fit / BalancedAllocation scores, after the static word's filters.
__device__ __forceinline__ SVal dyn_eval(const kss_profile& prof, const SPod& q, uint32_t w, const DynRow& r) {
  SVal e{sw_code(w), 0, 0, 0, 0};
  if (e.f) return e;
  if ((prof.filter_enabled >> KSS_F_NODE_RESOURCES_FIT) & 1u) {
    bool bad = (int64_t)r.pods + 1 > (int64_t)r.allowed;
    if (!(q.flags & SP_ALLZERO)) {
#pragma unroll
      for (int k = 0; k < 3; k++) bad |= q.fit_req[k] > r.alloc[k] - r.req[k];
    }
    if (bad) {
      e.f = KSS_F_NODE_RESOURCES_FIT;
      return e;
    }
  }
  e.tt = sw_tt(w);
  e.na = sw_na(w);
  e.fit = fit_fast(prof, q, r);
  e.ba = ba_fast(prof, q, r);
  return e;
}

// NormalizeScore + weights + packed selectHost key of one feasible node (the scored
// branch of schedule_pod<false>: PodTopologySpread normalises to 100 without
// constraints, InterPodAffinity keeps its raw 0).  rtt / rna: reciprocals of the maxima.
__device__ __forceinline__ long long simple_key(const kss_profile& prof, const SVal& e, bool scored, int max_tt,
                                                float rtt, int max_na, float rna, uint32_t g) {
  int64_t total = 0;
  if (scored) {
    // DefaultNormalizeScore(100, reverse=true) / (100, reverse=false); quotients <= 100
    const int32_t tt = max_tt == 0 ? 100 : 100 - small_div(100 * e.tt, max_tt, rtt);
    const int32_t na = max_na != 0 ? small_div(100 * e.na, max_na, rna) : e.na;
    const uint32_t se = prof.score_enabled;
    if ((se >> KSS_S_TAINT_TOLERATION) & 1u) total += (int64_t)tt * prof.weight[KSS_S_TAINT_TOLERATION];
    if ((se >> KSS_S_NODE_AFFINITY) & 1u) total += (int64_t)na * prof.weight[KSS_S_NODE_AFFINITY];
    if ((se >> KSS_S_NODE_RESOURCES_FIT) & 1u) total += (int64_t)e.fit * prof.weight[KSS_S_NODE_RESOURCES_FIT];
    if ((se >> KSS_S_POD_TOPOLOGY_SPREAD) & 1u) total += 100 * (int64_t)prof.weight[KSS_S_POD_TOPOLOGY_SPREAD];
    if ((se >> KSS_S_BALANCED_ALLOCATION) & 1u) total += (int64_t)e.ba * prof.weight[KSS_S_BALANCED_ALLOCATION];
  }
  return (long long)(((unsigned long long)(uint32_t)total << 32) | (0xFFFFFFFFull - g));
}

// ---------------------------------------------------------------------------
// wave reductions on the DPP network (no LDS): xor 1, xor 2, half-row mirror, row
// mirror, then row_bcast15 / row_bcast31 carry rows 0..2 into row 3; lane 63 holds the
// result.  64-bit values move as two 32-bit halves.
// ---------------------------------------------------------------------------
template <int OP>
__device__ __forceinline__ long long op_t(long long a, long long b) {
  if (OP == OP_SUM) return a + b;
  if (OP == OP_MAX) return b > a ? b : a;
  return b < a ? b : a;
}

template <int OP>
__device__ __forceinline__ constexpr long long ident_t() {
  return OP == OP_MAX ? INT64_MIN : (OP == OP_MIN ? INT64_MAX : 0);
}

template <int OP, int CTRL, int ROWS>
__device__ __forceinline__ long long dpp_step(long long v) {
  const unsigned long long id = (unsigned long long)ident_t<OP>();
  const unsigned long long u = (unsigned long long)v;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)id, (int)(uint32_t)u, CTRL, ROWS, 0xF, false);
  const uint32_t hi =
      (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(id >> 32), (int)(uint32_t)(u >> 32), CTRL, ROWS, 0xF, false);
  return op_t<OP>(v, (long long)(((unsigned long long)hi << 32) | lo));
}

template <int OP>
__device__ __forceinline__ long long wave_red(long long v) {
  v = dpp_step<OP, 0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
  v = dpp_step<OP, 0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
  v = dpp_step<OP, 0x141, 0xF>(v);  // row_half_mirror
  v = dpp_step<OP, 0x140, 0xF>(v);  // row_mirror
  v = dpp_step<OP, 0x142, 0xA>(v);  // row_bcast:15 -> rows 1, 3
  v = dpp_step<OP, 0x143, 0xC>(v);  // row_bcast:31 -> rows 2, 3
  const unsigned long long u = (unsigned long long)v;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), 63);
  return (long long)(((unsigned long long)hi << 32) | lo);
}

// Six non-negative 32-bit statistics {nf0, tt0, na0, nf1, tt1, na1} reduced together
// (SUM, MAX, MAX, SUM, MAX, MAX): each DPP step issues all six moves before combining,
// so the six chains overlap instead of paying the DPP latency six times.
template <int CTRL, int ROWS>
__device__ __forceinline__ void dpp_stats_step(uint32_t (&v)[6]) {
  uint32_t t[6];
#pragma unroll
  for (int i = 0; i < 6; i++) t[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[i], CTRL, ROWS, 0xF, false);
  v[0] += t[0];
  v[1] = max(v[1], t[1]);
  v[2] = max(v[2], t[2]);
  v[3] += t[3];
  v[4] = max(v[4], t[4]);
  v[5] = max(v[5], t[5]);
}

__device__ __forceinline__ void wave_red_stats(uint32_t (&v)[6]) {
  dpp_stats_step<0xB1, 0xF>(v);
  dpp_stats_step<0x4E, 0xF>(v);
  dpp_stats_step<0x141, 0xF>(v);
  dpp_stats_step<0x140, 0xF>(v);
  dpp_stats_step<0x142, 0xA>(v);
  dpp_stats_step<0x143, 0xC>(v);
#pragma unroll
  for (int i = 0; i < 6; i++) v[i] = (uint32_t)__builtin_amdgcn_readlane((int)v[i], 63);
}

// Per-wave mode's statistics of one wave, {nf0, tt0, na0, nf1, tt1, na1}: the counts by
// ballot, the TaintToleration maxima (7-bit raw values) as one packed 16-bit pair, so three
// DPP chains instead of six.  Lane-uniform results.
typedef unsigned short kss_u16x2 __attribute__((ext_vector_type(2)));
template <int CTRL, int ROWS>
__device__ __forceinline__ void dpp_pw_step(uint32_t& tp, uint32_t& n0, uint32_t& n1) {
  const uint32_t a = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)tp, CTRL, ROWS, 0xF, false);
  const uint32_t b = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)n0, CTRL, ROWS, 0xF, false);
  const uint32_t c = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)n1, CTRL, ROWS, 0xF, false);
  tp = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(kss_u16x2, tp),
                                                              __builtin_bit_cast(kss_u16x2, a)));
  n0 = max(n0, b);
  n1 = max(n1, c);
}
__device__ __forceinline__ void wave_red_stats_pw(uint32_t (&v)[6]) {
  const uint32_t nf0 = (uint32_t)__popcll(__ballot(v[0] != 0)), nf1 = (uint32_t)__popcll(__ballot(v[3] != 0));
  uint32_t tp = v[1] | (v[4] << 16), n0 = v[2], n1 = v[5];
  dpp_pw_step<0xB1, 0xF>(tp, n0, n1);
  dpp_pw_step<0x4E, 0xF>(tp, n0, n1);
  dpp_pw_step<0x141, 0xF>(tp, n0, n1);
  dpp_pw_step<0x140, 0xF>(tp, n0, n1);
  dpp_pw_step<0x142, 0xA>(tp, n0, n1);
  dpp_pw_step<0x143, 0xC>(tp, n0, n1);
  tp = (uint32_t)__builtin_amdgcn_readlane((int)tp, 63);
  v[0] = nf0;
  v[1] = tp & 0xFFFFu;
  v[2] = (uint32_t)__builtin_amdgcn_readlane((int)n0, 63);
  v[3] = nf1;
  v[4] = tp >> 16;
  v[5] = (uint32_t)__builtin_amdgcn_readlane((int)n1, 63);
}

// The selectHost key of a wave, reduced as 32 bits when it fits: total << kb | (2^kb - 1 -
// local node index) keeps the order of the 64-bit key (total << 32 | ~global index) whenever
// every total is below 2^(32 - kb) and 2^kb > N (key_bits: 0 when they do not), and
// 0 stays "no feasible node".  One DPP max per step instead of a 64-bit compare and select.
__device__ __forceinline__ int key_bits(const kss_profile& prof, int N) {
  const uint32_t se = prof.score_enabled;
  long long tmax = 0;  // every normalised score is at most MaxNodeScore (100)
  for (int p = 0; p < KSS_NSCORE; p++)
    if ((se >> p) & 1u) tmax += 100ll * (long long)max(prof.weight[p], 0);
  const int kb = 32 - __clz((unsigned)max(N, 1));  // 2^kb > N
  return tmax < (1ll << (32 - kb)) ? kb : 0;
}
__device__ __forceinline__ uint32_t key_compress(long long key, int kb, int node_base) {
  if (!key) return 0;
  const uint32_t m = (1u << kb) - 1u;
  const uint32_t li = (0xFFFFFFFFu - (uint32_t)(unsigned long long)key) - (uint32_t)node_base;
  return ((uint32_t)((unsigned long long)key >> 32) << kb) | (m - li);
}
__device__ __forceinline__ long long key_expand(uint32_t k, int kb, int node_base) {
  if (!k) return 0;
  const uint32_t m = (1u << kb) - 1u;
  const uint32_t li = m - (k & m);
  return (long long)(((unsigned long long)(k >> kb) << 32) | (0xFFFFFFFFull - ((uint32_t)node_base + li)));
}
__device__ __forceinline__ long long wave_max_key(long long key, int kb, int node_base) {
  if (!kb) return wave_red<OP_MAX>(key);
  uint32_t k = key_compress(key, kb, node_base);
#define KSS_KSTEP(CTRL, ROWS) k = max(k, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)k, CTRL, ROWS, 0xF, false))
  KSS_KSTEP(0xB1, 0xF);
  KSS_KSTEP(0x4E, 0xF);
  KSS_KSTEP(0x141, 0xF);
  KSS_KSTEP(0x140, 0xF);
  KSS_KSTEP(0x142, 0xA);
  KSS_KSTEP(0x143, 0xC);
#undef KSS_KSTEP
  k = (uint32_t)__builtin_amdgcn_readlane((int)k, 63);
  return key_expand(k, kb, node_base);
}

// LDS image of the loop head: reduction scratch (double-buffered), exchange results.
constexpr int SX_RED = 16;  // per-wave reduction row: the key and up to 15 statistics (the window's 12)
struct alignas(16) SimpleHdr {
  long long red[2][MAXWAVES][SX_RED];
  long long res[4];  // winner key of the previous pod; nf, max TT, max NA of the next pod
  long long win[12];  // window (simple_sync_win): F, TT / NA of the wholly kept segments, cut shard, part, j; d, TT, NA; E2 needed
  int cutc[2][MAXWAVES];  // window cut scan: feasible nodes of the part per wave
  int cutm[MAXWAVES][2];  // ... and the waves' maxima of the kept ones
  kss_profile prof;  // a runtime (non-default) profile: indexed by resource id, so in LDS, not scratch
  int abort;
  int pad[3];
};

// Workgroup barrier that orders LDS only.  HIP's __syncthreads() also drains every
// outstanding global load (vmcnt), which would put the prefetches on the critical path.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Workgroup reduction of K values; ONE barrier.  Parity alternates between calls, so a
// fast wave writing the next reduction never overwrites a slot a slow wave still reads.
template <int K>
__device__ __forceinline__ void block_red(SimpleHdr& H, int parity, long long (&v)[K], const int (&ops)[K]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < K; k++) {
    const long long r = ops[k] == OP_SUM ? wave_red<OP_SUM>(v[k])
                                         : (ops[k] == OP_MAX ? wave_red<OP_MAX>(v[k]) : wave_red<OP_MIN>(v[k]));
    if (lane == 0) H.red[parity][wave][k] = r;
  }
  lds_barrier();
#pragma unroll
  for (int k = 0; k < K; k++) {
    long long a = H.red[parity][0][k];
    for (int w = 1; w < nw; w++) a = op_apply(ops[k], a, H.red[parity][w][k]);
    v[k] = a;
  }
}

// Cross-shard exchange, wave 0 only.  v = {key, nf0, tt0, na0, nf1, tt1, na1} of this
// shard.  Publishes 8 granules {epoch, 32-bit value}, sweeps all W shards (64 per chunk,
// every load of a chunk in flight at once), then: winner = max key; the winner's shard
// (its node index / per) contributes H1, the others H0.  Results -> H.res.
__device__ __forceinline__ bool simple_exchange(SimpleHdr& H, unsigned long long* gran, const XPeers& X, int W, int wself,
                                                unsigned epoch,
                                                int* err, const long long (&v)[7], int per, int node_base, int kb) {
  const int lane = threadIdx.x & 63;
  const unsigned long long tag = (unsigned long long)epoch << 32;
  const unsigned long long key = (unsigned long long)v[0];
  if (lane < SX_VALS) {
    uint32_t x = (uint32_t)key;
    x = lane == 1 ? (uint32_t)(key >> 32) : x;
#pragma unroll
    for (int i = 1; i < 7; i++) x = lane == i + 1 ? (uint32_t)v[i] : x;
    xpub(X, gran, ((size_t)(epoch & 1) * W + wself) * SX_VALS + lane, tag | x);
  }
  const unsigned long long* base = gran + (size_t)(epoch & 1) * W * SX_VALS;
  uint32_t got[SX_CHUNKS][SX_VALS];
  long long best = 0;
#pragma unroll
  for (int ch = 0; ch < SX_CHUNKS; ch++) {
#pragma unroll
    for (int i = 0; i < SX_VALS; i++) got[ch][i] = 0;
    if (ch * 64 >= W) continue;
    const int s = ch * 64 + lane;
    const bool valid = s < W;
    long long t0_ = 0;
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
      unsigned long long g[SX_VALS];
      // every load issued (lanes past W read shard 0's granules), no exec-mask region per load
#pragma unroll
      for (int i = 0; i < SX_VALS; i++)
        g[i] = __hip_atomic_load(base + (size_t)(valid ? s : 0) * SX_VALS + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int i = 0; i < SX_VALS; i++) {
        ok &= !valid || (g[i] >> 32) == epoch;
        got[ch][i] = valid ? (uint32_t)g[i] : 0u;
      }
      if (__all(ok)) break;
      if (spin_expired(spins, t0_)) {
        if (lane == 0) {
          H.abort = 1;
          err_raise(err, 1);
        }
        return false;
      }
      spin_pause();
    }
    const long long k = (long long)(((unsigned long long)got[ch][1] << 32) | got[ch][0]);
    best = k > best ? k : best;
  }
  best = wave_max_key(best, kb, node_base);
  // the winner's shard: the one whose row range [s * per, (s + 1) * per) holds it
  const int gl = best != 0 ? (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)best) - node_base : -1;
  // {nf, tt, na} of every shard's hypothesis, reduced in one interleaved DPP pass
  uint32_t u[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int ch = 0; ch < SX_CHUNKS; ch++) {
    const int s = ch * 64 + lane;
    if (s >= W) continue;
    const bool h1 = gl >= s * per && gl < s * per + per;
    u[0] += h1 ? got[ch][5] : got[ch][2];
    u[1] = max(u[1], h1 ? got[ch][6] : got[ch][3]);
    u[2] = max(u[2], h1 ? got[ch][7] : got[ch][4]);
  }
  wave_red_stats(u);
  if (lane == 0) {
    H.res[0] = best;
    H.res[1] = u[0];
    H.res[2] = u[1];
    H.res[3] = u[2];
  }
  return true;
}

// The poll half of simple_exchange for any wave (KSS_PW_ALLPOLL): every shard's row of the
// exchange at `epoch` (this shard's own row included, published by its wave 0), the winner key
// and the statistics (the winner's shard contributing its H1), into R of every lane of the
// calling wave.  False after the wait bound (H.abort set).
__device__ __forceinline__ bool simple_exchange_poll(SimpleHdr& H, unsigned long long* gran, int W, unsigned epoch,
                                                     int* err, int per, int node_base, int kb, long long (&R)[4]) {
  const int lane = threadIdx.x & 63;
  const unsigned long long* base = gran + (size_t)(epoch & 1) * W * SX_VALS;
  uint32_t got[SX_CHUNKS][SX_VALS];
  long long best = 0;
#pragma unroll
  for (int ch = 0; ch < SX_CHUNKS; ch++) {
#pragma unroll
    for (int i = 0; i < SX_VALS; i++) got[ch][i] = 0;
    if (ch * 64 >= W) continue;
    const int s = ch * 64 + lane;
    const bool valid = s < W;
    long long t0_ = 0;
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
      unsigned long long g[SX_VALS];
#pragma unroll
      for (int i = 0; i < SX_VALS; i++)
        g[i] = __hip_atomic_load(base + (size_t)(valid ? s : 0) * SX_VALS + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int i = 0; i < SX_VALS; i++) {
        ok &= !valid || (g[i] >> 32) == epoch;
        got[ch][i] = valid ? (uint32_t)g[i] : 0u;
      }
      if (__all(ok)) break;
      if (spin_expired(spins, t0_)) {
        if (lane == 0) {
          H.abort = 1;
          err_raise(err, 1);
        }
        return false;
      }
      spin_pause();
    }
    const long long k = (long long)(((unsigned long long)got[ch][1] << 32) | got[ch][0]);
    best = k > best ? k : best;
  }
  best = wave_max_key(best, kb, node_base);
  const int gl = best != 0 ? (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)best) - node_base : -1;
  uint32_t u[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int ch = 0; ch < SX_CHUNKS; ch++) {
    const int s = ch * 64 + lane;
    if (s >= W) continue;
    const bool h1 = gl >= s * per && gl < s * per + per;
    u[0] += h1 ? got[ch][5] : got[ch][2];
    u[1] = max(u[1], h1 ? got[ch][6] : got[ch][3]);
    u[2] = max(u[2], h1 ? got[ch][7] : got[ch][4]);
  }
  wave_red_stats(u);
  R[0] = best;
  R[1] = u[0];
  R[2] = u[1];
  R[3] = u[2];
  return true;
}

// Block-reduce the six partial statistics of the next pod, exchange them with the
// current pod's shard-best key, and leave {winner key, nf, max TT, max NA} in R[] of
// every lane.  False if the launch aborted (exchange timeout).
__device__ __forceinline__ bool simple_sync(SimpleHdr& H, int& parity, long long key, long long (&st)[6], int W, int w,
                                            unsigned epoch, unsigned long long* gran, const XPeers& X, int* err, int per,
                                            int node_base, int kb,
                                            long long (&R)[4], KSS_GLOBAL unsigned long long* sp) {
  {
    uint32_t u[6];
#pragma unroll
    for (int i = 0; i < 6; i++) u[i] = (uint32_t)st[i];
    wave_red_stats(u);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 6; i++) H.red[parity][wave][i] = u[i];
    }
    lds_barrier();
#pragma unroll
    for (int i = 0; i < 6; i++) st[i] = H.red[parity][0][i];
    for (int wv = 1; wv < nw; wv++) {
      st[0] += H.red[parity][wv][0];
      st[3] += H.red[parity][wv][3];
#pragma unroll
      for (int i : {1, 2, 4, 5}) st[i] = max(st[i], H.red[parity][wv][i]);
    }
  }
  parity ^= 1;
  if (sp && threadIdx.x == 0) sp[4] = wall_clock64();
  if (W == 1) {  // the winner (if any) is this shard's candidate
    const bool h1 = key != 0;
    R[0] = key;
    R[1] = h1 ? st[3] : st[0];
    R[2] = h1 ? st[4] : st[1];
    R[3] = h1 ? st[5] : st[2];
    return true;
  }
  if (threadIdx.x < 64) {
    const long long v[7] = {key, st[0], st[1], st[2], st[3], st[4], st[5]};
    simple_exchange(H, gran, X, W, w, epoch, err, v, per, node_base, kb);
  }
  lds_barrier();
  if (H.abort) return false;
#pragma unroll
  for (int i = 0; i < 4; i++) R[i] = H.res[i];
  return true;
}

// The shard's node state in LDS for the whole launch (slot s = node lo + s), the per-slot
// results of the next pod (slot `cap` of the results holds the candidate node
// re-evaluated after the previous pod's commit, H1) and the static-word ring.
struct SimpleShard {
  double* r64;    // [8][cap]: allocatable cpu/mem/eph, requested cpu/mem/eph, non-zero cpu/mem (exact integers)
  double* inv;    // [3][cap]: RN(1 / allocatable)
  int32_t* r32;   // [2][cap]: pod count, allowed pods
  uint32_t* st;   // [RING][cap]: static words of the pods in flight (ring slot = pod % RING)
  int32_t* cv;    // [5][cap + CV_EXTRA]: filter verdict, TT, NA, Fit, BA (slots cap + i: H1 values)
  SPod* ring;     // [RING]: pod records (ring slot = pod % RING)
  int64_t* sc;    // [2 nsc][cap]: allocatable, then requested, of each extended (scalar) resource
  int cap, nsc;
};

constexpr int RING = 4;                // record / static-word ring slots
constexpr int CV_EXTRA = MAXWAVES;     // H1 slots past the shard's nodes: one per wave (per-wave mode)
constexpr int PW_LANES = 63;           // per-wave mode: node slots per wave (lane 63 is the wave's H1 lane)

__host__ __device__ inline size_t simple_lds_bytes(int cap, int nsc = 0) {
  return sizeof(SimpleHdr) + RING * sizeof(SPod) + (size_t)cap * (8 * 8 + 3 * 8 + 2 * 4 + RING * 4 + 16 * (size_t)nsc) +
         20 * ((size_t)cap + CV_EXTRA);
}

__device__ __forceinline__ SimpleShard shard_view(uint8_t* base, int cap, int nsc) {
  SimpleShard L;
  L.cap = cap;
  L.nsc = nsc;
  L.ring = reinterpret_cast<SPod*>(base);
  L.sc = reinterpret_cast<int64_t*>(base + RING * sizeof(SPod));
  uint8_t* b = base + RING * sizeof(SPod) + 16 * (size_t)nsc * (size_t)cap;
  L.r64 = reinterpret_cast<double*>(b);
  L.inv = reinterpret_cast<double*>(b + 64 * (size_t)cap);
  L.r32 = reinterpret_cast<int32_t*>(b + 88 * (size_t)cap);
  L.st = reinterpret_cast<uint32_t*>(L.r32 + 2 * (size_t)cap);
  L.cv = reinterpret_cast<int32_t*>(L.st + RING * (size_t)cap);
  return L;
}

__device__ __forceinline__ DynRow shard_row(const SimpleShard& L, int s) {
  DynRow r;
  const int C = L.cap;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    r.alloc[k] = L.r64[k * C + s];
    r.req[k] = L.r64[(3 + k) * C + s];
    r.inv[k] = L.inv[k * C + s];
  }
  r.nz[0] = L.r64[6 * C + s];
  r.nz[1] = L.r64[7 * C + s];
  r.pods = L.r32[s];
  r.allowed = L.r32[C + s];
  return r;
}

__device__ __forceinline__ SVal cv_get(const SimpleShard& L, int s) {
  const int C1 = L.cap + CV_EXTRA;
  return SVal{L.cv[s], L.cv[C1 + s], L.cv[2 * C1 + s], L.cv[3 * C1 + s], L.cv[4 * C1 + s]};
}

__device__ __forceinline__ void cv_put(const SimpleShard& L, int s, const SVal& e) {
  const int C1 = L.cap + CV_EXTRA;
  L.cv[s] = e.f;
  L.cv[C1 + s] = e.tt;
  L.cv[2 * C1 + s] = e.na;
  L.cv[3 * C1 + s] = e.fit;
  L.cv[4 * C1 + s] = e.ba;
}

// NodeResourcesFit.Filter over the extended (scalar) resources (fitsRequest; a zero request
// is skipped): true when some requested scalar exceeds the node's free amount.  sc: [2 nsc][cap]
// allocatable, then requested; add: pod q0's AssumePod delta is added to the row first (H1).
__device__ __forceinline__ bool scalar_short(const int64_t* sc, int nsc, int cap, int s, const SPod& q, bool add,
                                             const SPod& q0) {
  bool bad = false;
#pragma unroll
  for (int i = 0; i < KSS_MAX_SCALAR; i++) {
    if (i >= nsc) break;
    const int64_t req = q.sc_fit[i];
    const int64_t used = sc[(size_t)(nsc + i) * cap + s] + (add ? q0.sc_req[i] : 0);
    bad |= req != 0 && req > sc[(size_t)i * cap + s] - used;
  }
  return bad;
}

// NodeInfo.AddPod on a node row (requested, non-zero requested, pod count).
__device__ __forceinline__ void add_commit(DynRow& r, const SPod& p) {
#pragma unroll
  for (int k = 0; k < 3; k++) r.req[k] += p.creq[k];
  r.nz[0] += p.cnz[0];
  r.nz[1] += p.cnz[1];
  r.pods += 1;
}

// leastRequestedScore for the branch-free default-profile evaluation: 0 when requested >
// capacity; the caller masks capacity 0 (inv 0).
__device__ __forceinline__ int32_t least_bf(double requested, double capacity, double inv) {
  const bool over = requested > capacity;
  const double x = (capacity - (over ? capacity : requested)) * 100.0;  // integers below 2^53: exact, >= 0
  int32_t q = (int32_t)(x * inv);
  const double r = fma(-(double)q, capacity, x);
  q += (r >= capacity ? 1 : 0) - (r < 0.0 ? 1 : 0);
  return over ? 0 : q;
}

// dyn_eval of the v1.26 default profile (NodeResourcesFit LeastAllocated over cpu / memory
// with weights 1 / 1, BalancedAllocation over cpu / memory), branch-free: every lane
// computes every score and selects, so the node loop carries no exec-mask regions.  The
// scores of an infeasible node are not read (pass B skips it).
__device__ __forceinline__ SVal dyn_eval_def(const SPod& q, uint32_t w, const DynRow& r) {
  const int code = sw_code(w);
  bool bad = (int64_t)r.pods + 1 > (int64_t)r.allowed;
  const bool rq = !(q.flags & SP_ALLZERO);
  bad |= rq & ((q.fit_req[0] > r.alloc[0] - r.req[0]) | (q.fit_req[1] > r.alloc[1] - r.req[1]) |
               (q.fit_req[2] > r.alloc[2] - r.req[2]));
  SVal e;
  e.f = code ? code : (bad ? KSS_F_NODE_RESOURCES_FIT : 0);
  e.tt = sw_tt(w);
  e.na = sw_na(w);
  const bool u0 = r.alloc[0] != 0.0, u1 = r.alloc[1] != 0.0;
  // NodeResourcesFit.Score: capacity-0 resources drop out of the score and the weight sum
  const int32_t s0 = u0 ? least_bf(r.nz[0] + q.snz[0], r.alloc[0], r.inv[0]) : 0;
  const int32_t s1 = u1 ? least_bf(r.nz[1] + q.snz[1], r.alloc[1], r.inv[1]) : 0;
  e.fit = (u0 && u1) ? (s0 + s1) >> 1 : s0 + s1;
  // BalancedAllocation: two used resources give |f0 - f1| / 2, fewer a zero deviation
  double f0 = div_rn_d(r.req[0] + q.sreq[0], r.alloc[0], r.inv[0]);
  double f1 = div_rn_d(r.req[1] + q.sreq[1], r.alloc[1], r.inv[1]);
  f0 = f0 > 1.0 ? 1.0 : f0;
  f1 = f1 > 1.0 ? 1.0 : f1;
  const double sd = (u0 && u1) ? fabs((f0 - f1) / 2.0) : 0.0;
  e.ba = (int32_t)((1.0 - sd) * 100.0);
  return e;
}

// Pass A for pod q (static words in ring slot `sl`) over the shard's `own` nodes on the
// current state (H0), plus the candidate slot `cand_s` (-1 none) re-evaluated with the
// previous pod `q0` committed on it (H1), by the first slot without a node (slot `own`,
// which is slot `cap` of lane 0 when the shard is full).  st = {nf0, tt0, na0, nf1, tt1, na1}.
// Both records are copied to registers before the node loop (its LDS stores would otherwise
// make the compiler re-read every record field inside the loop, one LDS round trip each).
template <bool DEF>
__device__ __forceinline__ void simple_pass_a(const kss_profile& prof, const SPod& q_lds, const SPod& q0_lds,
                                              const SimpleShard& L, int sl, int own, int cand_s, long long (&st)[6]) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const uint32_t* sw = L.st + (size_t)sl * L.cap;
  const SPod q = q_lds;
  SPod q0;
#pragma unroll
  for (int k = 0; k < 3; k++) q0.creq[k] = q0_lds.creq[k];
  q0.cnz[0] = q0_lds.cnz[0];
  q0.cnz[1] = q0_lds.cnz[1];
  // extended resources: read from the LDS records inside the (rare) branch, not copied here
  const bool scal = L.nsc > 0 && (DEF || ((prof.filter_enabled >> KSS_F_NODE_RESOURCES_FIT) & 1u));
  int32_t nf = 0, tt = 0, na = 0, nf1 = 0, tt1 = 0, na1 = 0;  // raw TT <= 64, NA < 2^20
  for (int s = tid; s <= L.cap; s += nt) {
    const bool extra = s == own && cand_s >= 0;
    if (s >= own && !extra) continue;
    const int ns = extra ? cand_s : s;
    const uint32_t wd = sw[ns];
    DynRow r = shard_row(L, ns);
    if (extra) add_commit(r, q0);
    SVal e = DEF ? dyn_eval_def(q, wd, r) : dyn_eval(prof, q, wd, r);
    if (scal && e.f == 0 && scalar_short(L.sc, L.nsc, L.cap, ns, q_lds, extra, q0_lds)) e.f = KSS_F_NODE_RESOURCES_FIT;
    cv_put(L, extra ? L.cap : s, e);
    // H0 counts the shard's own slots, H1 every slot but the candidate's (whose H1 value is
    // the extra slot's); selects, no exec-mask region
    const bool c0 = e.f == 0 && !extra, c1 = e.f == 0 && s != cand_s;
    nf += c0 ? 1 : 0;
    tt = max(tt, c0 ? e.tt : 0);
    na = max(na, c0 ? e.na : 0);
    nf1 += c1 ? 1 : 0;
    tt1 = max(tt1, c1 ? e.tt : 0);
    na1 = max(na1, c1 ? e.na : 0);
  }
  st[0] = nf;
  st[1] = tt;
  st[2] = na;
  st[3] = nf1;
  st[4] = tt1;
  st[5] = na1;
}

// Per-wave mode (every shard's nodes fit in PW_LANES slots per wave, one per lane): wave v
// owns slots [v * pwv, v * pwv + pwv) of its shard and its lane pwv re-evaluates the WAVE's best
// candidate of the previous pod with that pod committed (the wave's H1).  The shard then never
// reduces its best key by itself: the waves' bests ride with the statistics, one workgroup
// reduction per pod instead of two (simple_sync_pw).  u = the wave lane's {nf0, tt0, na0, nf1,
// tt1, na1} (H1: the wave's slots but its candidate, plus the candidate re-evaluated).
template <bool DEF>
__device__ __forceinline__ void simple_pass_a_pw(const kss_profile& prof, const SPod& q_lds, const SPod& q0_lds,
                                                 const SimpleShard& L, int sl, int own, int pwv, int cand_w,
                                                 uint32_t (&u)[6]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t* sw = L.st + (size_t)sl * L.cap;
  const SPod q = q_lds;
  SPod q0;
#pragma unroll
  for (int k = 0; k < 3; k++) q0.creq[k] = q0_lds.creq[k];
  q0.cnz[0] = q0_lds.cnz[0];
  q0.cnz[1] = q0_lds.cnz[1];
  // extended resources: read from the LDS records inside the (rare) branch, not copied here
  const bool scal = L.nsc > 0 && (DEF || ((prof.filter_enabled >> KSS_F_NODE_RESOURCES_FIT) & 1u));
  const int s = wv * pwv + lane;
  const bool extra = lane == pwv && cand_w >= 0;
  const bool mine = lane < pwv && s < own;
#pragma unroll
  for (int i = 0; i < 6; i++) u[i] = 0;
  if (mine || extra) {
    const int ns = extra ? cand_w : s;
    const uint32_t wd = sw[ns];
    DynRow r = shard_row(L, ns);
    if (extra) add_commit(r, q0);
    SVal e = DEF ? dyn_eval_def(q, wd, r) : dyn_eval(prof, q, wd, r);
    if (scal && e.f == 0 && scalar_short(L.sc, L.nsc, L.cap, ns, q_lds, extra, q0_lds)) e.f = KSS_F_NODE_RESOURCES_FIT;
    cv_put(L, extra ? L.cap + wv : s, e);
    const bool c0 = e.f == 0 && !extra, c1 = e.f == 0 && (extra || s != cand_w);
    u[0] = c0 ? 1u : 0u;
    u[1] = c0 ? (uint32_t)e.tt : 0u;
    u[2] = c0 ? (uint32_t)e.na : 0u;
    u[3] = c1 ? 1u : 0u;
    u[4] = c1 ? (uint32_t)e.tt : 0u;
    u[5] = c1 ? (uint32_t)e.na : 0u;
  }
}

// AssumePod of pk on shard slot s (LDS node rows; the class / term counts follow after the
// launch, k_counts).
// KSS_LANE_COMMIT: the winner's AssumePod over the lanes of one wave (simple_commit_lanes)
#ifndef KSS_LANE_COMBINE
#define KSS_LANE_COMBINE 1  // simple_sync_pw: the waves' partials combined lane-parallel (r7d A/B: C2 291.8k -> 301.3k pods/s)
#endif
#ifndef KSS_PF_LAST_WAVE
// per-wave mode with 3+ waves: the last wave (fewest slots) alone prefetches the next records and
// static words, so the first prefetch wave reaches the statistics barrier with the others (r8u
// A/B, C2: 303.3 / 303.6 k against 301.6 / 301.5 k pods/s)
#define KSS_PF_LAST_WAVE 1
#endif
#ifndef KSS_PW_ALLPOLL
// simple_sync_pw: every wave polls the exchange itself, no closing barrier.  r8t A/B: C2 261k
// against 304k pods/s -- the prefetch waves' polls queue behind their own HBM prefetch loads
// (vmcnt is in order), so the pod waits for them: off
#define KSS_PW_ALLPOLL 0
#endif
#ifndef KSS_LANE_COMMIT
#define KSS_LANE_COMMIT 1  // r7c A/B: C2 284.7k -> 290.7k pods/s, C4 unchanged; 0 keeps one lane
#endif
static_assert(offsetof(SPod, cnz) == offsetof(SPod, creq) + 3 * sizeof(double), "creq, cnz adjacent");
// The same AssumePod spread over the lanes of one wave: lane r < 5 adds row 3 + r (Requested cpu /
// memory / ephemeral, then NonZeroRequested cpu / memory: creq and cnz are adjacent), lane 5 the
// pod count, lanes 8.. the extended resources -- the rows' LDS round trips overlap instead of
// following each other on one lane.
__device__ __forceinline__ void simple_commit_lanes(const SimpleShard& L, const SPod& pk, int s, int lane) {
  const int cap = L.cap;
  if (lane < 5) L.r64[(3 + lane) * cap + s] += (&pk.creq[0])[lane];
  if (lane == 5) L.r32[s] += 1;
  if (lane >= 8 && lane < 8 + L.nsc) L.sc[(size_t)(L.nsc + lane - 8) * cap + s] += pk.sc_req[lane - 8];
}
__device__ __forceinline__ void simple_commit_slot(const SimpleShard& L, const SPod& pk, int s) {
  const int cap = L.cap;
#pragma unroll
  for (int r = 0; r < 3; r++) L.r64[(3 + r) * cap + s] += pk.creq[r];
  L.r64[6 * cap + s] += pk.cnz[0];
  L.r64[7 * cap + s] += pk.cnz[1];
  L.r32[s] += 1;
  for (int i = 0; i < L.nsc; i++) L.sc[(size_t)(L.nsc + i) * cap + s] += pk.sc_req[i];
}

// Per-wave mode's one reduction per pod: the waves' best keys and H0 / H1 statistics in one
// LDS pass (the shard's H1 is the best wave's H1 with every other wave's H0), the cross-shard
// exchange, and pod k's AssumePod on the winner's slot by wave 0 BEFORE the closing barrier
// (the next pod's pass A reads that row with no barrier of its own in between).
// R = {winner key, nf, max TT, max NA of the next pod}.  False if the launch aborted.
// `idle` runs on every wave right after the statistics barrier: the waves other than wave 0
// wait out the exchange there (the prefetch loads are issued from it).
template <typename Idle>
__device__ __forceinline__ bool simple_sync_pw(SimpleHdr& H, int& parity, long long wbest, uint32_t (&u)[6], int W,
                                               int w, unsigned epoch, unsigned long long* gran, const XPeers& X,
                                               int* err, int per, int node_base, int lo, int own, const SPod& pk,
                                               bool commit, const SimpleShard& L, int kb, long long (&R)[4],
                                               KSS_GLOBAL unsigned long long* sp, Idle&& idle) {
  wave_red_stats_pw(u);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (sp && threadIdx.x == 0) sp[7] = wall_clock64();
  if (sp && (threadIdx.x == 64 || threadIdx.x == 128)) sp[9 + (threadIdx.x >> 6)] = wall_clock64();  // waves 1, 2 reach it
  if (lane == 0) {
    H.red[parity][wave][0] = wbest;
#pragma unroll
    for (int i = 0; i < 6; i++) H.red[parity][wave][1 + i] = u[i];
  }
  lds_barrier();
  if (sp && threadIdx.x == 0) sp[8] = wall_clock64();
  idle();
  if (wave == 0) {  // wave 0 alone combines (every lane the same few LDS words: broadcasts) and exchanges
#if KSS_LANE_COMBINE
    // lane v < nw reads wave v's partials (one LDS round trip for all waves), then three DPP
    // steps over the (at most 8) lanes: the largest key, and the six statistics with the best
    // wave contributing its H1
    const bool in = lane < nw;
    const long long* hv = H.red[parity][in ? lane : 0];
    const long long kv = in ? hv[0] : 0;
    uint32_t xv[6];
#pragma unroll
    for (int i = 0; i < 6; i++) xv[i] = in ? (uint32_t)hv[1 + i] : 0u;
    long long best = kv;
    best = dpp_step<OP_MAX, 0xB1, 0xF>(best);
    best = dpp_step<OP_MAX, 0x4E, 0xF>(best);
    best = dpp_step<OP_MAX, 0x141, 0xF>(best);
    {
      const unsigned long long ub = (unsigned long long)best;
      best = (long long)(((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(ub >> 32), 0) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ub, 0));
    }
    const bool me = in && best != 0 && kv == best;  // keys carry the node index: one wave at most
    uint32_t t[6] = {xv[0], xv[1], xv[2], me ? xv[3] : xv[0], me ? xv[4] : xv[1], me ? xv[5] : xv[2]};
    dpp_stats_step<0xB1, 0xF>(t);
    dpp_stats_step<0x4E, 0xF>(t);
    dpp_stats_step<0x141, 0xF>(t);
#pragma unroll
    for (int i = 0; i < 6; i++) t[i] = (uint32_t)__builtin_amdgcn_readlane((int)t[i], 0);
#else
    // waves 0 and 1 (the usual per-wave geometry) read at once, unconditionally; waves 2.. in a loop
    const long long* h0 = H.red[parity][0];
    const long long* h1 = H.red[parity][nw > 1 ? 1 : 0];
    long long a0[7], a1[7];
#pragma unroll
    for (int i = 0; i < 7; i++) {
      a0[i] = h0[i];
      a1[i] = h1[i];
    }
    if (nw < 2) a1[0] = 0;
    // the wave holding the shard's best (keys carry the node index: one wave at most)
    long long best = a0[0];
    int ws = best ? 0 : -1;
    if (a1[0] > best) {
      best = a1[0];
      ws = 1;
    }
    for (int v = 2; v < nw; v++) {
      const long long b = H.red[parity][v][0];
      ws = b > best ? v : ws;
      best = b > best ? b : best;
    }
    // the best wave contributes its H1, the others their H0
    const bool w0 = ws == 0, w1 = ws == 1;
    uint32_t t[6];
    t[0] = (uint32_t)a0[1] + (nw > 1 ? (uint32_t)a1[1] : 0u);
    t[1] = max((uint32_t)a0[2], nw > 1 ? (uint32_t)a1[2] : 0u);
    t[2] = max((uint32_t)a0[3], nw > 1 ? (uint32_t)a1[3] : 0u);
    t[3] = (uint32_t)(w0 ? a0[4] : a0[1]) + (nw > 1 ? (uint32_t)(w1 ? a1[4] : a1[1]) : 0u);
    t[4] = max((uint32_t)(w0 ? a0[5] : a0[2]), nw > 1 ? (uint32_t)(w1 ? a1[5] : a1[2]) : 0u);
    t[5] = max((uint32_t)(w0 ? a0[6] : a0[3]), nw > 1 ? (uint32_t)(w1 ? a1[6] : a1[3]) : 0u);
    for (int v = 2; v < nw; v++) {
      const long long* h = H.red[parity][v];
      const int o = v == ws ? 4 : 1;
      t[0] += (uint32_t)h[1];
      t[1] = max(t[1], (uint32_t)h[2]);
      t[2] = max(t[2], (uint32_t)h[3]);
      t[3] += (uint32_t)h[o];
      t[4] = max(t[4], (uint32_t)h[o + 1]);
      t[5] = max(t[5], (uint32_t)h[o + 2]);
    }
#endif
    if (sp && lane == 0) sp[4] = wall_clock64();
    if (W == 1) {  // the winner (if any) is this shard's best
      const bool h1 = best != 0;
      const int slot = (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)best) - node_base - lo;
      if (lane == 0) {
        H.res[0] = best;
        H.res[1] = h1 ? t[3] : t[0];
        H.res[2] = h1 ? t[4] : t[1];
        H.res[3] = h1 ? t[5] : t[2];
        if (!KSS_LANE_COMMIT && commit && h1) simple_commit_slot(L, pk, slot);
      }
      if (KSS_LANE_COMMIT && commit && h1) simple_commit_lanes(L, pk, slot, lane);
    } else if (KSS_PW_ALLPOLL) {  // publish only: every wave polls below
      if (lane < SX_VALS) {
        const unsigned long long key = (unsigned long long)best, tag = (unsigned long long)epoch << 32;
        uint32_t x = (uint32_t)key;
        x = lane == 1 ? (uint32_t)(key >> 32) : x;
#pragma unroll
        for (int i = 0; i < 6; i++) x = lane == i + 2 ? t[i] : x;
        xpub(X, gran, ((size_t)(epoch & 1) * W + w) * SX_VALS + lane, tag | x);
      }
    } else {
      const long long v[7] = {best, t[0], t[1], t[2], t[3], t[4], t[5]};
      if (simple_exchange(H, gran, X, W, w, epoch, err, v, per, node_base, kb) && commit && (KSS_LANE_COMMIT || lane == 0)) {
        const long long K = H.res[0];  // (written by lane 0 of this wave: in order)
        const int x = K ? (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)K) - node_base - lo : -1;
        if (x >= 0 && x < own) {
          if (KSS_LANE_COMMIT) simple_commit_lanes(L, pk, x, lane);
          else simple_commit_slot(L, pk, x);
        }
      }
    }
  }
  if (KSS_PW_ALLPOLL && W > 1) {
    // every wave polls the shards' rows itself and commits pod k on the winner's slot if that slot
    // is one of its own: no closing barrier.  Each wave's next reads (pass B / pass A) touch only
    // its own slots, and a wave reaching the next statistics barrier has finished this pod's poll,
    // so the reduction rows (parity-alternated) are never overwritten while read.
    parity ^= 1;
    if (!simple_exchange_poll(H, gran, W, epoch, err, per, node_base, kb, R)) return false;
    const long long K = R[0];
    const int x = K ? (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)K) - node_base - lo : -1;
    const int pwv = (own + nw - 1) / nw;  // the wave's slots (simple_schedule's per-wave split)
    if (commit && x >= 0 && x < own && x / max(pwv, 1) == wave) simple_commit_lanes(L, pk, x, lane);
    return true;
  }
  parity ^= 1;
  lds_barrier();
  if (H.abort) return false;
#pragma unroll
  for (int i = 0; i < 4; i++) R[i] = H.res[i];
  return true;
}

// ---------------------------------------------------------------------------
// percentageOfNodesToScore < 100: findNodesThatPassFilters' window on k_simple
// ---------------------------------------------------------------------------
// v1.26 findNodesThatPassFilters (Parallelism = 1, the deterministic form) checks
// the nodes from nextStartNodeIndex s in canonical order, wrapping, and stops once K + 1 feasible
// nodes were found (K = numFeasibleNodesToFind): the first K are kept (scored, selectHost's
// candidates); the (K+1)-th, d, was filtered but dropped, and nextStartNodeIndex becomes d (the
// processed count is the d - s nodes before it).  With F <= K feasible nodes every node is
// visited, every feasible one kept, and s stays.
// Here the window rides on the pod's statistics exchange.  Each shard splits its slots at the
// pod's start node into part a (node >= s) and part b (node < s), so the visiting order is the
// segments a_0 .. a_{W-1}, b_0 .. b_{W-1}, and publishes per part {feasible count, max raw TT,
// max raw NA} for H0 and H1 (SXW_VALS granules).  After the sweep every shard knows from the
// segments' counts the segment holding the (K+1)-th feasible node (the cut) and the maxima of
// the segments wholly before it.  Only the cut segment's shard needs d: every other shard's
// segments lie wholly before or after the cut, so pass B keeps node n iff feasible and (no cut,
// or seg(n) < cut segment, or seg(n) == cut segment and n < d), and the next pod's split needs
// only the start SHARD elsewhere (shards before it: every node in part b; after it: part a).
// The cut shard ranks its feasible nodes (ballots) for d and the maxima over its first j; a
// second exchange (SXW_E2 granules, polled from that one shard) carries those maxima only when
// the cut segment's maxima over ALL its feasible nodes exceed the wholly kept segments' (known
// to every shard from the first exchange): otherwise they cannot change the result.
// Statistics index: (h * 2 + part) * 3 + {0 F, 1 TT, 2 NA}, h = 0 H0, 1 H1.
constexpr int SXW_VALS = 10;  // granules per shard: key lo / hi, then {F << 16 | TT, NA} of a0, b0, a1, b1
constexpr int SXW_E2 = 4;     // the cut shard's granules per epoch parity: d, TT, NA (+ pad)

__device__ __forceinline__ void win_acc(uint32_t (&u)[12], bool c0, bool c1, int part, const SVal& e) {
#pragma unroll
  for (int v = 0; v < 4; v++) {
    const bool on = ((v >> 1) ? c1 : c0) && (v & 1) == part;
    u[v * 3] += on ? 1u : 0u;
    u[v * 3 + 1] = max(u[v * 3 + 1], on ? (uint32_t)e.tt : 0u);
    u[v * 3 + 2] = max(u[v * 3 + 2], on ? (uint32_t)e.na : 0u);
  }
}

// simple_pass_a with the window's split: part a / b of each slot by its node against `start`
template <bool DEF>
__device__ __forceinline__ void simple_pass_a_win(const kss_profile& prof, const SPod& q_lds, const SPod& q0_lds,
                                                  const SimpleShard& L, int sl, int own, int cand_s, int lo, int start,
                                                  uint32_t (&u)[12]) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const uint32_t* sw = L.st + (size_t)sl * L.cap;
  const SPod q = q_lds;
  SPod q0;
#pragma unroll
  for (int k = 0; k < 3; k++) q0.creq[k] = q0_lds.creq[k];
  q0.cnz[0] = q0_lds.cnz[0];
  q0.cnz[1] = q0_lds.cnz[1];
  const bool scal = L.nsc > 0 && (DEF || ((prof.filter_enabled >> KSS_F_NODE_RESOURCES_FIT) & 1u));
#pragma unroll
  for (int i = 0; i < 12; i++) u[i] = 0;
  for (int s = tid; s <= L.cap; s += nt) {
    const bool extra = s == own && cand_s >= 0;
    if (s >= own && !extra) continue;
    const int ns = extra ? cand_s : s;
    const uint32_t wd = sw[ns];
    DynRow r = shard_row(L, ns);
    if (extra) add_commit(r, q0);
    SVal e = DEF ? dyn_eval_def(q, wd, r) : dyn_eval(prof, q, wd, r);
    if (scal && e.f == 0 && scalar_short(L.sc, L.nsc, L.cap, ns, q_lds, extra, q0_lds)) e.f = KSS_F_NODE_RESOURCES_FIT;
    cv_put(L, extra ? L.cap : s, e);
    win_acc(u, e.f == 0 && !extra, e.f == 0 && s != cand_s, lo + ns >= start ? 0 : 1, e);
  }
}

// simple_pass_a_pw with the window's split
template <bool DEF>
__device__ __forceinline__ void simple_pass_a_pw_win(const kss_profile& prof, const SPod& q_lds, const SPod& q0_lds,
                                                     const SimpleShard& L, int sl, int own, int pwv, int cand_w, int lo,
                                                     int start, uint32_t (&u)[12]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t* sw = L.st + (size_t)sl * L.cap;
  const SPod q = q_lds;
  SPod q0;
#pragma unroll
  for (int k = 0; k < 3; k++) q0.creq[k] = q0_lds.creq[k];
  q0.cnz[0] = q0_lds.cnz[0];
  q0.cnz[1] = q0_lds.cnz[1];
  const bool scal = L.nsc > 0 && (DEF || ((prof.filter_enabled >> KSS_F_NODE_RESOURCES_FIT) & 1u));
  const int s = wv * pwv + lane;
  const bool extra = lane == pwv && cand_w >= 0;
  const bool mine = lane < pwv && s < own;
#pragma unroll
  for (int i = 0; i < 12; i++) u[i] = 0;
  if (mine || extra) {
    const int ns = extra ? cand_w : s;
    const uint32_t wd = sw[ns];
    DynRow r = shard_row(L, ns);
    if (extra) add_commit(r, q0);
    SVal e = DEF ? dyn_eval_def(q, wd, r) : dyn_eval(prof, q, wd, r);
    if (scal && e.f == 0 && scalar_short(L.sc, L.nsc, L.cap, ns, q_lds, extra, q0_lds)) e.f = KSS_F_NODE_RESOURCES_FIT;
    cv_put(L, extra ? L.cap + wv : s, e);
    win_acc(u, e.f == 0 && !extra, e.f == 0 && (extra || s != cand_w), lo + ns >= start ? 0 : 1, e);
  }
}

// the twelve window statistics over DPP lanes: counts summed, maxima kept
template <int CTRL, int ROWS>
__device__ __forceinline__ void dpp_win_step(uint32_t (&v)[12]) {
  uint32_t t[12];
#pragma unroll
  for (int i = 0; i < 12; i++) t[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[i], CTRL, ROWS, 0xF, false);
#pragma unroll
  for (int i = 0; i < 12; i++) v[i] = (i % 3 == 0) ? v[i] + t[i] : max(v[i], t[i]);
}

// inclusive prefix sum over the wave in DPP: row_shr 1, 2, 4, 8 scan each row of 16 lanes (lanes
// whose source falls outside the row add 0), row_bcast:15 adds row 0's total to row 1 and row 2's to
// row 3, row_bcast:31 adds rows 0-1's total to rows 2 and 3
template <int CTRL, int ROWS>
__device__ __forceinline__ void dpp_add2(uint32_t& a, uint32_t& b) {
  const uint32_t ta = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a, CTRL, ROWS, 0xF, false);
  const uint32_t tb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)b, CTRL, ROWS, 0xF, false);
  a += ta;
  b += tb;
}
__device__ __forceinline__ void wave_incl_scan2(uint32_t& a, uint32_t& b) {
  dpp_add2<0x111, 0xF>(a, b);
  dpp_add2<0x112, 0xF>(a, b);
  dpp_add2<0x114, 0xF>(a, b);
  dpp_add2<0x118, 0xF>(a, b);
  dpp_add2<0x142, 0xA>(a, b);
  dpp_add2<0x143, 0xC>(a, b);
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  uint32_t z = 0;
  wave_incl_scan2(v, z);
  return v;
}
// the maxima of two non-negative 32-bit values over the wave (uniform results)
__device__ __forceinline__ void wave_max2(uint32_t& a, uint32_t& b) {
  uint32_t t[2] = {a, b};
  auto step = [&](auto ctrl, auto rows) {
    constexpr int C = decltype(ctrl)::value, R = decltype(rows)::value;
    const uint32_t x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t[0], C, R, 0xF, false);
    const uint32_t y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t[1], C, R, 0xF, false);
    t[0] = max(t[0], x);
    t[1] = max(t[1], y);
  };
  step(std::integral_constant<int, 0xB1>{}, std::integral_constant<int, 0xF>{});
  step(std::integral_constant<int, 0x4E>{}, std::integral_constant<int, 0xF>{});
  step(std::integral_constant<int, 0x141>{}, std::integral_constant<int, 0xF>{});
  step(std::integral_constant<int, 0x140>{}, std::integral_constant<int, 0xF>{});
  step(std::integral_constant<int, 0x142>{}, std::integral_constant<int, 0xA>{});
  step(std::integral_constant<int, 0x143>{}, std::integral_constant<int, 0xC>{});
  a = (uint32_t)__builtin_amdgcn_readlane((int)t[0], 63);
  b = (uint32_t)__builtin_amdgcn_readlane((int)t[1], 63);
}

// The cut shard: rank the feasible nodes of `part` (pod k+1's verdicts; the winner's slot takes
// its H1 verdict) in canonical order; d = the node of rank j, TT / NA = the maxima over ranks < j.
// Whole workgroup; results uniform.
template <bool PW>
__device__ __forceinline__ void win_cut_scan(SimpleHdr& H, const SimpleShard& L, int own, int lo, int start, int part,
                                             int j, int sub_s, int sub_h, int pwv, int& d, int& ptt, int& pna,
                                             bool maxima = true) {
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wave = tid >> 6, nw = nt >> 6;
  const int iters = PW ? 1 : (own + nt - 1) / nt;
  int carry = 0, mt = 0, mn = 0;
  for (int it = 0; it < iters; it++) {
    const int s = PW ? wave * pwv + lane : it * nt + tid;
    const bool valid = PW ? (lane < pwv && s < own) : s < own;
    bool f = false;
    SVal e{0, 0, 0, 0, 0};
    if (valid && (part == 0 ? lo + s >= start : lo + s < start)) {
      e = cv_get(L, s == sub_s ? sub_h : s);
      f = e.f == 0;
    }
    const unsigned long long b = __ballot(f);
    if (lane == 0) H.cutc[it & 1][wave] = (int)__popcll(b);
    lds_barrier();
    int before = 0, tot = 0;
    for (int x = 0; x < nw; x++) {
      const int cx = H.cutc[it & 1][x];
      before += x < wave ? cx : 0;
      tot += cx;
    }
    const int rank = carry + before + (int)__popcll(b & ((1ull << lane) - 1ull));
    if (f && rank == j) H.win[6] = lo + s;
    mt = max(mt, (f && rank < j) ? e.tt : 0);
    mn = max(mn, (f && rank < j) ? e.na : 0);
    carry += tot;
  }
  ptt = 0;
  pna = 0;
  if (!maxima) {  // the cut segment's maxima cannot exceed the kept ones: only d is needed
    lds_barrier();  // H.win[6] written by its lane
    d = (int)H.win[6];
    return;
  }
  mt = (int)wave_red<OP_MAX>(mt);
  mn = (int)wave_red<OP_MAX>(mn);
  if (lane == 0) {
    H.cutm[wave][0] = mt;
    H.cutm[wave][1] = mn;
  }
  lds_barrier();
  for (int x = 0; x < nw; x++) {
    ptt = max(ptt, H.cutm[x][0]);
    pna = max(pna, H.cutm[x][1]);
  }
  d = (int)H.win[6];
}

// The window's statistics exchange (both per-wave and per-thread modes; PW: the best wave contributes
// its H1, else every wave's H1 set already accounts for the shard's candidate).  Pod k's AssumePod
// on the winner's slot is applied here (wave 0, lane-parallel) before the closing barrier.
// R = {winner key of pod k, kept count, max TT, max NA of pod k+1 over its kept nodes}; cs_out = pod
// k+1's cut segment (part * W + shard, -1: no cut), d_out = its dropped node (on the cut shard;
// -1 elsewhere).  start: this shard's split of pod k+1's node list (win_start).  False if the
// launch aborted.
template <bool PW, typename Idle>
__device__ __forceinline__ bool simple_sync_win(SimpleHdr& H, int& parity, long long wkey, uint32_t (&u)[12], int W,
                                                int w, unsigned epoch, unsigned long long* gran, const XPeers& X,
                                                int* err, int per, int node_base, int lo, int own, const SPod& pk,
                                                bool commit, const SimpleShard& L, int kb, int k_find, int start,
                                                int pwv, long long (&R)[4], int& d_out, int& cs_out,
                                                KSS_GLOBAL unsigned long long* sp, Idle&& idle) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (PW) {
    // one node (or the H1 re-evaluation) per lane: the four counts are ballot popcounts, the four
    // TaintToleration maxima (<= 64) ride as two packed 16-bit pairs, the NodeAffinity maxima alone:
    // six DPP chains instead of twelve
    uint32_t c4[4];
#pragma unroll
    for (int v = 0; v < 4; v++) c4[v] = (uint32_t)__popcll(__ballot(u[3 * v] != 0));
    uint32_t tp0 = u[1] | (u[4] << 16), tp1 = u[7] | (u[10] << 16), n0 = u[2], n1 = u[5], n2 = u[8], n3 = u[11];
    auto step = [&](auto ctrl, auto rows) {
      constexpr int C = decltype(ctrl)::value, R = decltype(rows)::value;
      dpp_pw_step<C, R>(tp0, n0, n1);
      dpp_pw_step<C, R>(tp1, n2, n3);
    };
    step(std::integral_constant<int, 0xB1>{}, std::integral_constant<int, 0xF>{});
    step(std::integral_constant<int, 0x4E>{}, std::integral_constant<int, 0xF>{});
    step(std::integral_constant<int, 0x141>{}, std::integral_constant<int, 0xF>{});
    step(std::integral_constant<int, 0x140>{}, std::integral_constant<int, 0xF>{});
    step(std::integral_constant<int, 0x142>{}, std::integral_constant<int, 0xA>{});
    step(std::integral_constant<int, 0x143>{}, std::integral_constant<int, 0xC>{});
#pragma unroll
    for (int v = 0; v < 4; v++) u[3 * v] = c4[v];
    u[1] = tp0 & 0xFFFFu;
    u[4] = tp0 >> 16;
    u[7] = tp1 & 0xFFFFu;
    u[10] = tp1 >> 16;
    u[2] = n0;
    u[5] = n1;
    u[8] = n2;
    u[11] = n3;
  } else {
    dpp_win_step<0xB1, 0xF>(u);
    dpp_win_step<0x4E, 0xF>(u);
    dpp_win_step<0x141, 0xF>(u);
    dpp_win_step<0x140, 0xF>(u);
    dpp_win_step<0x142, 0xA>(u);
    dpp_win_step<0x143, 0xC>(u);
  }
  if (sp && threadIdx.x == 0) sp[7] = wall_clock64();
  if (lane == 63) {  // the reduced values sit in lane 63
    H.red[parity][wave][0] = wkey;
#pragma unroll
    for (int i = 0; i < 12; i++) H.red[parity][wave][1 + i] = u[i];
  }
  lds_barrier();
  if (sp && threadIdx.x == 0) sp[8] = wall_clock64();
  idle();
  if (wave == 0) {
    // the shard: lane v < nw reads wave v's row, three DPP steps over the (at most 8) lanes
    const bool in = lane < nw;
    const long long* hv = H.red[parity][in ? lane : 0];
    const long long kv = in ? hv[0] : 0;
    long long best = kv;
    best = dpp_step<OP_MAX, 0xB1, 0xF>(best);
    best = dpp_step<OP_MAX, 0x4E, 0xF>(best);
    best = dpp_step<OP_MAX, 0x141, 0xF>(best);
    {
      const unsigned long long ub = (unsigned long long)best;
      best = (long long)(((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(ub >> 32), 0) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ub, 0));
    }
    const bool me = PW ? (in && best != 0 && kv == best) : in;
    // per set (0: every wave's H0 values, 1: the best wave's H1 in place of its H0) the part a / b
    // counts and TaintToleration maxima as packed 16-bit pairs (both below 2^16: the exchange packs
    // them the same way), the NodeAffinity maxima alone: 8 words over three DPP steps
    kss_u16x2 pc[2], pt[2];
    uint32_t pn[4];
#pragma unroll
    for (int st = 0; st < 2; st++) {
      const int b = st == 0 ? 1 : (me ? 7 : 1);
      pc[st] = __builtin_bit_cast(kss_u16x2, in ? (uint32_t)hv[b] | ((uint32_t)hv[b + 3] << 16) : 0u);
      pt[st] = __builtin_bit_cast(kss_u16x2, in ? (uint32_t)hv[b + 1] | ((uint32_t)hv[b + 4] << 16) : 0u);
      pn[2 * st] = in ? (uint32_t)hv[b + 2] : 0u;
      pn[2 * st + 1] = in ? (uint32_t)hv[b + 5] : 0u;
    }
    auto cstep = [&](auto ctrl) {
      constexpr int C = decltype(ctrl)::value;
      uint32_t m[8];
#pragma unroll
      for (int st = 0; st < 2; st++) {
        m[st] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)__builtin_bit_cast(uint32_t, pc[st]), C, 0xF, 0xF, false);
        m[2 + st] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)__builtin_bit_cast(uint32_t, pt[st]), C, 0xF, 0xF, false);
      }
#pragma unroll
      for (int i = 0; i < 4; i++) m[4 + i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pn[i], C, 0xF, 0xF, false);
#pragma unroll
      for (int st = 0; st < 2; st++) {
        pc[st] = pc[st] + __builtin_bit_cast(kss_u16x2, m[st]);
        pt[st] = __builtin_elementwise_max(pt[st], __builtin_bit_cast(kss_u16x2, m[2 + st]));
      }
#pragma unroll
      for (int i = 0; i < 4; i++) pn[i] = max(pn[i], m[4 + i]);
    };
    cstep(std::integral_constant<int, 0xB1>{});
    cstep(std::integral_constant<int, 0x4E>{});
    cstep(std::integral_constant<int, 0x141>{});
    uint32_t t[12];
#pragma unroll
    for (int st = 0; st < 2; st++) {
      const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)__builtin_bit_cast(uint32_t, pc[st]), 0);
      const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)__builtin_bit_cast(uint32_t, pt[st]), 0);
      t[6 * st + 0] = c & 0xFFFFu;
      t[6 * st + 1] = x & 0xFFFFu;
      t[6 * st + 2] = (uint32_t)__builtin_amdgcn_readlane((int)pn[2 * st], 0);
      t[6 * st + 3] = c >> 16;
      t[6 * st + 4] = x >> 16;
      t[6 * st + 5] = (uint32_t)__builtin_amdgcn_readlane((int)pn[2 * st + 1], 0);
    }
    if (sp && lane == 0) sp[4] = wall_clock64();
    // every shard's packed values in the lane of that shard (W == 1: this shard in lane 0)
    uint32_t got[SX_CHUNKS][8];
    long long gbest = best;
    bool ok = true;
    if (W == 1) {
#pragma unroll
      for (int v = 0; v < 4; v++) {
        got[0][2 * v] = lane == 0 ? (t[3 * v] << 16) | t[3 * v + 1] : 0u;
        got[0][2 * v + 1] = lane == 0 ? t[3 * v + 2] : 0u;
      }
#pragma unroll
      for (int ch = 1; ch < SX_CHUNKS; ch++)
#pragma unroll
        for (int i = 0; i < 8; i++) got[ch][i] = 0;
    } else {
      const unsigned long long tag = (unsigned long long)epoch << 32;
      if (lane < SXW_VALS) {
        uint32_t x = (uint32_t)(unsigned long long)best;
        x = lane == 1 ? (uint32_t)((unsigned long long)best >> 32) : x;
#pragma unroll
        for (int v = 0; v < 4; v++) {
          x = lane == 2 + 2 * v ? ((t[3 * v] << 16) | t[3 * v + 1]) : x;
          x = lane == 3 + 2 * v ? t[3 * v + 2] : x;
        }
        xpub(X, gran, ((size_t)(epoch & 1) * W + w) * SXW_VALS + lane, tag | x);
      }
      const unsigned long long* base = gran + (size_t)(epoch & 1) * W * SXW_VALS;
      long long kbest = 0;
#pragma unroll
      for (int ch = 0; ch < SX_CHUNKS; ch++) {
#pragma unroll
        for (int i = 0; i < 8; i++) got[ch][i] = 0;
        if (ch * 64 >= W || !ok) continue;
        const int s = ch * 64 + lane;
        const bool valid = s < W;
        long long t0_ = 0;
        uint32_t k2[2] = {0, 0};
        for (unsigned spins = 0;; ++spins) {
          bool okp = true;
          unsigned long long g[SXW_VALS];
#pragma unroll
          for (int i = 0; i < SXW_VALS; i++)
            g[i] = __hip_atomic_load(base + (size_t)(valid ? s : 0) * SXW_VALS + i, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
          for (int i = 0; i < SXW_VALS; i++) okp &= !valid || (g[i] >> 32) == epoch;
          if (__all(okp)) {
            k2[0] = valid ? (uint32_t)g[0] : 0u;
            k2[1] = valid ? (uint32_t)g[1] : 0u;
#pragma unroll
            for (int i = 0; i < 8; i++) got[ch][i] = valid ? (uint32_t)g[2 + i] : 0u;
            break;
          }
          if (spin_expired(spins, t0_)) {
            if (lane == 0) {
              H.abort = 1;
              err_raise(err, 1);
            }
            ok = false;
            break;
          }
          spin_pause();
        }
        const long long kk = (long long)(((unsigned long long)k2[1] << 32) | k2[0]);
        kbest = kk > kbest ? kk : kbest;
      }
      gbest = wave_max_key(kbest, kb, node_base);
    }
    if (sp && lane == 0) sp[10] = wall_clock64();
    if (ok) {
      const int gl = gbest != 0 ? (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)gbest) - node_base : -1;
      // each lane's shard: H1 when the winner is one of its nodes
      uint32_t Fa[SX_CHUNKS], Fb[SX_CHUNKS], ta[SX_CHUNKS], tb[SX_CHUNKS], na_[SX_CHUNKS], nb_[SX_CHUNKS];
      uint32_t A = 0, B = 0, sa[SX_CHUNKS], sb[SX_CHUNKS], TA[SX_CHUNKS], TB[SX_CHUNKS];
#pragma unroll
      for (int ch = 0; ch < SX_CHUNKS; ch++) {
        const int s = ch * 64 + lane;
        const bool h1 = W > 1 ? (gl >= s * per && gl < s * per + per) : gbest != 0;
        const int o = h1 ? 4 : 0;
        Fa[ch] = got[ch][o] >> 16;
        ta[ch] = got[ch][o] & 0xFFFFu;
        na_[ch] = got[ch][o + 1];
        Fb[ch] = got[ch][o + 2] >> 16;
        tb[ch] = got[ch][o + 2] & 0xFFFFu;
        nb_[ch] = got[ch][o + 3];
        // per chunk: the inclusive scans of the part a / b counts and their totals
        sa[ch] = Fa[ch];
        sb[ch] = Fb[ch];
        TA[ch] = TB[ch] = 0;
        if (ch * 64 < W) {  // (uniform)
          wave_incl_scan2(sa[ch], sb[ch]);
          TA[ch] = (uint32_t)__builtin_amdgcn_readlane((int)sa[ch], 63);
          TB[ch] = (uint32_t)__builtin_amdgcn_readlane((int)sb[ch], 63);
        }
        A += TA[ch];
        B += TB[ch];
      }
      const uint32_t F = A + B, K = (uint32_t)k_find;
      uint32_t ftt = 0, fna = 0, cut_tt = 0, cut_na = 0;  // cut_*: the cut segment's maxima over all its feasible nodes
      int cut = -1, part = 0, j = 0;
      if (F <= K) {
#pragma unroll
        for (int ch = 0; ch < SX_CHUNKS; ch++) {
          ftt = max(ftt, max(ta[ch], tb[ch]));
          fna = max(fna, max(na_[ch], nb_[ch]));
        }
      } else {
        uint32_t ca = 0, cb = A;  // segments before this chunk
        unsigned long long hit = 0;
        int hit_ch = -1;
        uint32_t pre_hit = 0;
#pragma unroll
        for (int ch = 0; ch < SX_CHUNKS; ch++) {
          if (ch * 64 >= W) break;  // (uniform) no shard in this chunk
          const uint32_t pa = ca + sa[ch] - Fa[ch], pb = cb + sb[ch] - Fb[ch];
          ftt = max(ftt, pa + Fa[ch] <= K ? ta[ch] : 0u);
          fna = max(fna, pa + Fa[ch] <= K ? na_[ch] : 0u);
          ftt = max(ftt, pb + Fb[ch] <= K ? tb[ch] : 0u);
          fna = max(fna, pb + Fb[ch] <= K ? nb_[ch] : 0u);
          const bool cA = pa <= K && K < pa + Fa[ch], cB = pb <= K && K < pb + Fb[ch];
          const unsigned long long ba = __ballot(cA), bb = __ballot(cB);
          if (hit_ch < 0 && (ba | bb)) {
            const int l = __ffsll((long long)(ba ? ba : bb)) - 1;
            hit_ch = ch;
            hit = ba ? 0ull : 1ull;
            cut = ch * 64 + l;
            pre_hit = (uint32_t)__builtin_amdgcn_readlane((int)(ba ? pa : pb), l);
            cut_tt = (uint32_t)__builtin_amdgcn_readlane((int)(ba ? ta[ch] : tb[ch]), l);
            cut_na = (uint32_t)__builtin_amdgcn_readlane((int)(ba ? na_[ch] : nb_[ch]), l);
          }
          ca += TA[ch];
          cb += TB[ch];
        }
        part = (int)hit;
        j = (int)(K - pre_hit);
      }
      wave_max2(ftt, fna);
      // pod k's AssumePod on the winner's slot (before the closing barrier: the next pod's pass A
      // reads that row without a barrier of its own)
      if (commit && gbest != 0) {
        const int x = gl - lo;
        if (x >= 0 && x < own) simple_commit_lanes(L, pk, x, lane);
      }
      if (lane == 0) {
        H.res[0] = gbest;
        H.win[0] = F;
        H.win[1] = ftt;
        H.win[2] = fna;
        H.win[3] = cut;
        H.win[4] = part;
        H.win[5] = j;
        H.win[10] = cut >= 0 && (cut_tt > ftt || cut_na > fna);  // the cut shard's partial maxima can matter
        if (sp) {
          sp[11] = wall_clock64();
          sp[14] = 1 + (cut == w ? 2 : 0) + (H.win[10] ? 4 : 0);
        }
      }
    }
  }
  parity ^= 1;
  lds_barrier();
  if (H.abort) return false;
  const long long F = H.win[0];
  const int cut = (int)H.win[3];
  long long mtt = H.win[1], mna = H.win[2], nf = F;
  int d = -1;
  cs_out = cut >= 0 ? (int)H.win[4] * W + cut : -1;
  if (cut >= 0) {
    nf = k_find;
    const bool need = H.win[10] != 0;
    const long long best = H.res[0];
    const int gl = best != 0 ? (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)best) - node_base : -1;
    const bool won = gl >= lo && gl < lo + own;
    const int sub_s = won ? gl - lo : -1;
    const int sub_h = PW ? L.cap + (won ? (gl - lo) / max(pwv, 1) : 0) : L.cap;
    const size_t e2 = 2 * (size_t)W * SXW_VALS + (size_t)(epoch & 1) * SXW_E2;
    if (cut == w) {  // uniform over the workgroup
      int cd = -1, ctt = 0, cna = 0;
      win_cut_scan<PW>(H, L, own, lo, start, (int)H.win[4], (int)H.win[5], sub_s, sub_h, pwv, cd, ctt, cna, need);
      d = cd;
      if (W == 1) {
        mtt = max(mtt, (long long)ctt);
        mna = max(mna, (long long)cna);
      } else if (need && threadIdx.x < 3) {
        const unsigned long long tag = (unsigned long long)epoch << 32;
        const uint32_t x = threadIdx.x == 0 ? (uint32_t)cd : (threadIdx.x == 1 ? (uint32_t)ctt : (uint32_t)cna);
        xpub(X, gran, e2 + threadIdx.x, tag | x);
      }
      if (sp && threadIdx.x == 0) sp[12] = wall_clock64();
    }
    if (W > 1 && need) {
      if (wave == 0) {
        const unsigned long long* b2 = gran + e2;
        long long t0_ = 0;
        for (unsigned spins = 0;; ++spins) {
          const unsigned long long g = __hip_atomic_load(b2 + min(lane, 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (__all((g >> 32) == epoch)) {
            if (lane < 3) H.win[7 + lane] = (long long)(uint32_t)g;
            break;
          }
          if (spin_expired(spins, t0_)) {
            if (lane == 0) {
              H.abort = 1;
              err_raise(err, 1);
            }
            break;
          }
          spin_pause();
        }
      }
      lds_barrier();
      if (H.abort) return false;
      mtt = max(mtt, H.win[8]);
      mna = max(mna, H.win[9]);
    }
  }
  R[0] = H.res[0];
  R[1] = nf;
  R[2] = mtt;
  R[3] = mna;
  d_out = d;
  return true;
}

// Pods [k0, k1) of the batch for shard w of one cluster (every pod commits).  `stat`
// holds the static words of those pods ([k - k0][N]).  On an exchange timeout the error
// word is set and the shard leaves without writing node state back.  PW: per-wave mode
// (simple_sync_pw; the caller checks that every shard's nodes fit it).  WIN: percentageOfNodesToScore
// < 100 (simple_sync_win): k_find = numFeasibleNodesToFind, cursor = the cluster's nextStartNodeIndex
// word (read at the start, written back by shard 0 at the end).
template <bool DEF, bool PW, bool WIN>
__device__ __forceinline__ void simple_schedule(DevCluster c, const SPod* __restrict__ spods,
                                                const uint32_t* __restrict__ stat, const int32_t* __restrict__ ints,
                                                int k0, int k1, int32_t* chosen, PodMeta* meta, const kss_profile& prof,
                                                int W, int w, int cap, unsigned long long* gran, const XPeers& X,
                                                unsigned epoch0, int* err, unsigned long long* stamps, long long* smem,
                                                int k_find = 0, int32_t* cursor = nullptr) {
  const int tid = threadIdx.x, nt = blockDim.x;
  SimpleHdr& H = *reinterpret_cast<SimpleHdr*>(smem);
  const SimpleShard L = shard_view(reinterpret_cast<uint8_t*>(smem) + sizeof(SimpleHdr), cap, c.n_scalar);
  const size_t N = (size_t)c.N;
  const int per = (c.N + W - 1) / W;
  const int lo = min(c.N, w * per), hi = min(c.N, lo + per), own = hi - lo;
  if (k1 <= k0) return;
  constexpr int NQ = (int)(sizeof(SPod) / 16);
  // prefetch distance: the record and static words of pod k + PD are loaded while pod k is
  // scheduled.  Per-wave mode has no barrier between a pod's end and the next pod's pass A, so
  // its prefetch stores land one pod earlier (behind two barriers) than the pass that reads them.
  constexpr int PD = PW ? 3 : 2;
  // shard rows, reciprocals, static words and records of pods k0 .. k0 + PD - 1 -> LDS
  handoff_acquire();
  for (int s = tid; s < own; s += nt) {
    const int n = lo + s;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const int64_t A = c.alloc[k * N + n];
      L.r64[k * cap + s] = (double)A;
      L.r64[(3 + k) * cap + s] = (double)ld_ag(&c.requested[k * N + n]);
      L.inv[k * cap + s] = A > 0 ? 1.0 / (double)A : 0.0;
    }
    L.r64[6 * cap + s] = (double)ld_ag(&c.nonzero[n]);
    L.r64[7 * cap + s] = (double)ld_ag(&c.nonzero[N + n]);
    L.r32[s] = ld_ag(&c.pod_count[n]);
    L.r32[cap + s] = c.allowed_pods[n];
    for (int i = 0; i < L.nsc; i++) {
      L.sc[(size_t)i * cap + s] = c.alloc[(size_t)(3 + i) * N + n];
      L.sc[(size_t)(L.nsc + i) * cap + s] = ld_ag(&c.requested[(size_t)(3 + i) * N + n]);
    }
    for (int d = 0; d < PD && k0 + d < k1; d++) L.st[((k0 + d) % RING) * cap + s] = ld_ag(&stat[(size_t)d * N + lo + s]);
  }
  for (int i = tid; i < min(k1 - k0, PD) * NQ; i += nt) {
    const int j = k0 + i / NQ;
    reinterpret_cast<uint4*>(L.ring + j % RING)[i % NQ] = reinterpret_cast<const uint4*>(spods + j)[i % NQ];
  }
  if (tid == 0) H.abort = 0;
  __syncthreads();
  // the window (WIN).  A shard splits its slots at a pod's start node s into part a (node >= s) and
  // part b by `wsl`: s itself on the shard holding s (the start shard, wss), past its last node on
  // shards before it (every node in part b), its first node on shards after it (every node in part
  // a).  wsx: s, on the start shard.  wcs: pod k's cut segment (-1 none), wd: its dropped node, on
  // the cut shard (pass B).  Pod k0 starts at the cursor word.
  const int cur0 = WIN && cursor && c.N > 0 ? (int)(((long long)ld_ag(cursor) % c.N + c.N) % c.N) : 0;
  auto win_start = [&](int sh, int x) { return w < sh ? lo + own : (w > sh ? lo : x); };
  int wss = WIN ? min(cur0 / max(per, 1), W - 1) : 0, wsx = cur0;
  int wsl = win_start(wss, cur0), wcs = -1, wd = -1;

  KSS_GLOBAL const uint32_t* gstat = gp(stat);
  KSS_GLOBAL const uint4* gspod = gp(reinterpret_cast<const uint4*>(spods));
  KSS_GLOBAL unsigned long long* gstamps = gp(stamps);
  long long st[6], R[4] = {0, 0, 0, 0};
  // the outcome of pod pend_k, not yet stored (thread out_tid of shard w_off)
  const int out_tid = (nt >> 6) > 1 ? 64 : 0;
  const bool defer_out = PW && (nt >> 6) > 1;
  PodMeta pend{};
  int pend_k = -1;
  auto store_pending = [&]() {
    if (pend_k < 0) return;
    if (chosen) gp(chosen)[pend_k] = pend.chosen;
    if (meta) {
      KSS_GLOBAL PodMeta* mm = gp(meta) + pend_k;
      mm->chosen = pend.chosen;
      mm->n_feasible = pend.n_feasible;
      mm->scored = pend.scored;
      mm->status = pend.status;
      mm->best_total = pend.best_total;
    }
    pend_k = -1;
  };
  int parity = 0, sub_s = -1;  // slot whose pass-B values are the H1 ones (the previous winner)
  int sub_h = cap;             // ... and the cv slot holding them
  unsigned epoch = epoch0;  // granule tags above every tag an earlier launch left (split grids)
  const int nwave = nt >> 6;
  const int lane = tid & 63, wv = tid >> 6;
  const int pwv = (own + nwave - 1) / nwave;  // per-wave mode: the wave's node slots (<= PW_LANES)
  const int kb = key_bits(prof, c.N);  // 32-bit key reductions when the keys fit (0: 64-bit)
  // prefetch lanes: every wave but wave 0 (readfirstlane: a wave-uniform, scalar branch)
  // (KSS_PF_LAST_WAVE, per-wave mode with 3+ waves: the last wave alone prefetches -- A/B)
  const int pf_w0 = (PW && KSS_PF_LAST_WAVE && nwave >= 3) ? nwave - 1 : 1;
  const bool pf_wave = nwave == 1 || __builtin_amdgcn_readfirstlane(tid >> 6) >= pf_w0;
  uint4 pfq = make_uint4(0, 0, 0, 0);  // prefetched record / static words of pod k+PD, live across the loop
  uint32_t pfw[PF_MAX];
#pragma unroll
  for (int j = 0; j < PF_MAX; j++) pfw[j] = 0;
  const int pf_lane = nwave == 1 ? tid : tid - 64 * pf_w0, pf_n = nwave == 1 ? nt : nt - 64 * pf_w0;
  const int pf_per = (own + pf_n - 1) / pf_n;  // static words per prefetch lane (<= PF_MAX)
  // k = k0 - 1 is the prologue: pass A of pod k0 and the exchange of its statistics
  for (int k = k0 - 1; k < k1; k++) {
    // diagnostic phase stamps (KSS_STAMPS_FILE): lane 0 of every shard, the first pods
    KSS_GLOBAL unsigned long long* sp = (stamps && k >= k0 && k - k0 < KSS_NSTAMP_PODS / 2)
                                            ? gstamps + (size_t)w * 8 * KSS_NSTAMP_PODS + (size_t)(k - k0) * 16
                                            : nullptr;
    if (sp && tid == 0) sp[0] = wall_clock64();
    if (sp && tid == 64) sp[9] = wall_clock64();  // wave 1's start of the pod
    const SPod& pk = L.ring[(k + RING) % RING];
    // pod k+PD: record and static words -> registers now, -> their ring slots at the end
    // Only the prefetch waves (all but wave 0, unless there is one wave) issue these loads:
    // vmcnt is per wave and counts stores too, so wave 0 — which publishes granules and
    // writes the outcomes — never waits on an HBM prefetch, and the prefetch waves never
    // wait on a store.
    // The branch is wave-uniform and every load inside it is unconditional (clamped
    // indices), so the compiler's wait for these registers stays on the prefetch path.
    const bool pf_on = pf_wave && k >= k0 && k + PD < k1 && own > 0;
    auto prefetch = [&]() {
      if (pf_on) {
        KSS_GLOBAL const uint4& src = gspod[(size_t)(k + PD) * NQ + min(pf_lane, NQ - 1)];
        pfq = make_uint4(src.x, src.y, src.z, src.w);
#pragma unroll
        for (int j = 0; j < PF_MAX; j++)
          if (j < pf_per) pfw[j] = ld_ag(&gstat[(size_t)(k + PD - k0) * N + lo + min(j * pf_n + pf_lane, own - 1)]);
      }
    };
    auto ring_store = [&]() {  // lanes past the end rewrite the last element with its own value
      if (pf_on) {
        reinterpret_cast<uint4*>(L.ring + (k + PD) % RING)[min(pf_lane, NQ - 1)] = pfq;
#pragma unroll
        for (int j = 0; j < PF_MAX; j++)
          if (j < pf_per) L.st[((k + PD) % RING) * cap + min(j * pf_n + pf_lane, own - 1)] = pfw[j];
      }
    };
    // issued here; per-wave mode with several waves stores them into the ring while wave 0
    // exchanges (simple_sync_pw's idle hook: slot (k + PD) % RING held pod k - 1, whose last
    // reader finished before the statistics barrier), then this pod's HBM stores follow, after
    // every wait on a load of this wave
    prefetch();
    auto prefetch_idle = [&]() {
      if (defer_out) {
        ring_store();
        if (tid == out_tid) store_pending();  // the previous pod's outcome
      }
    };
    // pass B: NormalizeScore, weights, shard-best selectHost key of pod k
    const long long nf = R[1];
    const int max_tt = (int)R[2], max_na = (int)R[3];
    const bool scored = nf > 1;
    long long best = 0;
    int cand = -1;  // the candidate slot whose H1 pass A evaluates (the shard's / the wave's best)
    const bool keys = k >= k0 && pk.status == 0 && nf > 0;
    const float rtt = __builtin_amdgcn_rcpf((float)max(max_tt, 1));
    const float rna = __builtin_amdgcn_rcpf((float)max(max_na, 1));
    if constexpr (PW) {
      // every slot's five values read at once and its key computed whatever the verdict, then
      // selected: one LDS round trip per slot, no exec-mask region; the wave's best by DPP
      const int s = wv * pwv + lane;
      if (keys && lane < pwv && s < own) {
        const SVal e = cv_get(L, s == sub_s ? sub_h : s);
        const long long key = simple_key(prof, e, scored, max_tt, rtt, max_na, rna, (uint32_t)(c.node_base + lo + s));
        bool kept = true;
        if (WIN && wcs >= 0) {  // the node's segment before the cut segment, or before d inside it
          const int n = lo + s, seg = (n >= wsl ? 0 : W) + w;
          kept = seg < wcs || (seg == wcs && n < wd);
        }
        best = (e.f == 0 && kept) ? key : 0;
      }
      if (sp && tid == 0) sp[1] = wall_clock64();
      best = wave_max_key(best, kb, c.node_base);
      if (sp && tid == 0) sp[2] = wall_clock64();
    } else {
      if (k >= k0) {
        if (keys) {
          for (int s = tid; s < own; s += nt) {
            const SVal e = cv_get(L, s == sub_s ? sub_h : s);
            const long long key = simple_key(prof, e, scored, max_tt, rtt, max_na, rna, (uint32_t)(c.node_base + lo + s));
            bool kept = true;
            if (WIN && wcs >= 0) {
              const int n = lo + s, seg = (n >= wsl ? 0 : W) + w;
              kept = seg < wcs || (seg == wcs && n < wd);
            }
            best = (e.f == 0 && kept && key > best) ? key : best;
          }
        }
        if (sp && tid == 0) sp[1] = wall_clock64();
        long long b[1] = {best};
        const int op[1] = {OP_MAX};
        block_red(H, parity, b, op);
        parity ^= 1;
        best = b[0];
        if (sp && tid == 0) sp[2] = wall_clock64();
      }
    }
    cand = best ? (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)best) - c.node_base - lo : -1;
    // pass A: pod k+1 before pod k's commit, and on the candidate after it
    const SPod& qn = L.ring[(k + 1) % RING];
    const int sln = (k + 1) % RING;
    if constexpr (WIN) {
      // pod k+1 starts where pod k's window stopped (its dropped node, on the cut shard), else
      // where pod k started
      if (k >= k0 && wcs >= 0) {
        wss = wcs % W;
        if (w == wss) wsx = wd;
        wsl = win_start(wss, wd);
      }
      uint32_t u[12];
      if (k + 1 < k1) {
        if constexpr (PW) simple_pass_a_pw_win<DEF>(prof, qn, pk, L, sln, own, pwv, cand, lo, wsl, u);
        else simple_pass_a_win<DEF>(prof, qn, pk, L, sln, own, cand, lo, wsl, u);
      } else {
#pragma unroll
        for (int i = 0; i < 12; i++) u[i] = 0;
      }
      if (sp && tid == 0) sp[3] = wall_clock64();
      if (!simple_sync_win<PW>(H, parity, best, u, W, w, ++epoch, gran, X, err, per, c.node_base, lo, own, pk, k >= k0, L,
                               kb, k_find, wsl, pwv, R, wd, wcs, sp, prefetch_idle))
        return;
    } else if constexpr (PW) {
      uint32_t u[6];
      if (k + 1 < k1) {
        simple_pass_a_pw<DEF>(prof, qn, pk, L, sln, own, pwv, cand, u);
      } else {
#pragma unroll
        for (int i = 0; i < 6; i++) u[i] = 0;
      }
      if (sp && tid == 0) sp[3] = wall_clock64();
      if (!simple_sync_pw(H, parity, best, u, W, w, ++epoch, gran, X, err, per, c.node_base, lo, own, pk, k >= k0, L, kb,
                          R, sp, prefetch_idle))
        return;
    } else {
      if (k + 1 < k1) {
        simple_pass_a<DEF>(prof, qn, pk, L, sln, own, cand, st);
      } else {
#pragma unroll
        for (int i = 0; i < 6; i++) st[i] = 0;
      }
      if (sp && tid == 0) sp[3] = wall_clock64();
      if (!simple_sync(H, parity, best, st, W, w, ++epoch, gran, X, err, per, c.node_base, kb, R, sp)) return;
    }
    if (sp && tid == 0) sp[5] = wall_clock64();
    if (k >= k0) {
      const long long K = R[0];
      const int x = K ? (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)K) - c.node_base : -1;
      // AssumePod on the winner's shard (per-wave mode: done inside the sync); pass B of pod
      // k+1 takes that slot's H1 values: cv slot cap (cap + the slot's wave in per-wave mode)
      const bool won = x >= lo && x < hi;
      sub_s = won ? x - lo : -1;
      sub_h = PW ? cap + (won ? (x - lo) / max(pwv, 1) : 0) : cap;
      if (!PW && !WIN && won && (KSS_LANE_COMMIT ? tid < 64 : tid == 0)) {
        if (KSS_LANE_COMMIT) simple_commit_lanes(L, pk, x - lo, tid);
        else simple_commit_slot(L, pk, x - lo);
      }
      // the HBM-only class / term counts are applied after the launch (k_counts): nothing in
      // this loop reads them
    }
    if (!defer_out) ring_store();
    // every part keeps the outcomes.  Their HBM stores are issued off wave 0 (whose vmcnt stays
    // free for the exchange polls); with several waves in per-wave mode they are held in
    // registers and issued while the NEXT pod's exchange runs (store_pending in the idle hook,
    // ahead of that wave's prefetch loads), so no wait on a store lands on the pod chain
    if (k >= k0 && w == X.w_off && tid == out_tid) {
      const long long K = R[0];
      const int x = K ? (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)K) - c.node_base : -1;
      pend.chosen = K ? x + c.node_base : -1;
      pend.n_feasible = (int)nf;
      pend.scored = (K && scored) ? 1 : 0;
      pend.status = pk.status != 0 ? (pk.status == KSS_PF_ERROR ? 3 : 2) : (nf == 0 ? 1 : 0);
      pend.best_total = pend.scored ? (int64_t)((unsigned long long)K >> 32) : 0;
      pend_k = k;
      if (!defer_out) store_pending();
    }
    if (sp && tid == 0) sp[6] = wall_clock64();
  }
  if (tid == out_tid) store_pending();  // the last pod's outcome
  // nextStartNodeIndex after the last pod: the start shard of the pod after it writes it (the last
  // iteration's pass A, for no pod, already moved the start past the last pod's cut)
  if (WIN && cursor && w == wss && tid == 0) st_ag(cursor, (int32_t)wsx);
  // node state back to HBM
  __syncthreads();
  for (int s = tid; s < own; s += nt) {
    const int n = lo + s;
#pragma unroll
    for (int r = 0; r < 3; r++) st_ag(&c.requested[(size_t)r * N + n], (int64_t)L.r64[(3 + r) * cap + s]);
    st_ag(&c.nonzero[n], (int64_t)L.r64[6 * cap + s]);
    st_ag(&c.nonzero[N + n], (int64_t)L.r64[7 * cap + s]);
    st_ag(&c.pod_count[n], L.r32[s]);
    for (int i = 0; i < L.nsc; i++) st_ag(&c.requested[(size_t)(3 + i) * N + n], L.sc[(size_t)(L.nsc + i) * cap + s]);
  }
  handoff_release();
}

// The class / term count part of AssumePod for pods [k0, k1) of a k_simple batch, from
// their chosen nodes (one lane per pod; counts commute, so the order is immaterial).
__device__ __forceinline__ void simple_counts(const DevCluster& c, const SPod* __restrict__ spods,
                                              const int32_t* __restrict__ ints, const int32_t* __restrict__ chosen,
                                              int k) {
  const int x = chosen[k] - c.node_base;
  if (x < 0 || x >= c.N) return;
  const SPod& q = spods[k];
  const size_t N = (size_t)c.N;
  if (q.cls >= 0) atomicAdd(&c.class_count[(size_t)q.cls * N + x], 1);
  for (int i = 0; i < q.own_len; i++) atomicAdd(&c.term_count[(size_t)ints[q.own_off + i] * N + x], 1);
}

}  // namespace kss
