// kss_simple.cuh — the sequential scheduling loop for batches without PodTopologySpread /
// InterPodAffinity programs (the default-profile workload of BASELINE C1/C2/C5), built
// around ONE cross-shard exchange per pod.
//
// Same semantics as schedule_pod<false> (kss_sched.cuh), different pipeline:
//   * every node row of the shard lives in registers for the whole launch (lane t owns
//     nodes lo + j*blockDim + t, j < NPT); label value ids live in LDS;
//   * pod programs arrive as position-independent blobs (host: build_blobs) staged in a
//     3-slot LDS ring; blob k+2 is loaded into registers while pod k is scheduled;
//   * pod k's argmax and pod k+1's normalisation statistics travel in the same exchange.
//     Pod k+1's statistics depend on pod k's commit, which touches one node only: the
//     winner, which is some shard's local best.  Each shard therefore evaluates pod k+1
//     on its local best node twice — before the commit (H0) and after it (H1) — and
//     publishes both statistic sets next to its pod-k key.  Once the global winner is
//     known, the winner's shard contributes H1 and every other shard H0, which is the
//     statistic of pod k+1 on the committed state.
// Per pod: one block reduction for the shard's best key, one for the six partial
// statistics, one exchange (8 granules per shard) — instead of two block reductions and
// two exchanges separated by a full filter pass.
#pragma once
#include "kss_sched.cuh"

namespace kss {

constexpr int BLOB_MAX = 4096;  // bytes per serialized pod program (host-checked)
constexpr int SX_VALS = 8;      // granules per shard per exchange: key lo/hi, H0 (nf, tt, na), H1 (nf, tt, na)
constexpr int SX_CHUNKS = 2;    // shards swept 64 at a time: W <= 128

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

// Blob layout: kss_pod (every offset rebased into the blob) | BlobHdr | reqs | terms | ints.
struct BlobHdr {
  int32_t req_off, term_off, ints_off;  // byte offsets from the blob start
  int32_t n_reqs, n_terms, n_ints;
  int32_t pad[2];
};
__host__ __device__ constexpr size_t blob_hdr_off() { return (sizeof(kss_pod) + 15) / 16 * 16; }
__host__ __device__ constexpr size_t blob_body_off() { return blob_hdr_off() + (sizeof(BlobHdr) + 15) / 16 * 16; }

struct BlobView {
  const kss_pod* pod;
  const kss_req* reqs;
  const kss_term* terms;
  const int32_t* ints;
};

__device__ __forceinline__ BlobView blob_view(const uint8_t* b) {
  const BlobHdr* h = reinterpret_cast<const BlobHdr*>(b + blob_hdr_off());
  BlobView v;
  v.pod = reinterpret_cast<const kss_pod*>(b);
  v.reqs = reinterpret_cast<const kss_req*>(b + h->req_off);
  v.terms = reinterpret_cast<const kss_term*>(b + h->term_off);
  v.ints = reinterpret_cast<const int32_t*>(b + h->ints_off);
  return v;
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

// LDS image of the loop head: reduction scratch (double-buffered), exchange results.
struct SimpleHdr {
  long long red[2][MAXWAVES][SX_VALS];
  long long res[4];  // winner key of the previous pod; nf, max TT, max NA of the next pod
  int abort;
  int pad[3];
};

// Workgroup barrier that orders LDS only.  HIP's __syncthreads() also drains every
// outstanding global load (vmcnt), which would put the blob prefetch on the critical path.
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
__device__ __forceinline__ bool simple_exchange(SimpleHdr& H, unsigned long long* gran, int W, int wself, unsigned epoch,
                                                int* err, const long long (&v)[7], int per, int node_base) {
  const int lane = threadIdx.x & 63;
  const unsigned long long tag = (unsigned long long)epoch << 32;
  const unsigned long long key = (unsigned long long)v[0];
  if (lane < SX_VALS) {
    uint32_t x = (uint32_t)key;
    x = lane == 1 ? (uint32_t)(key >> 32) : x;
#pragma unroll
    for (int i = 1; i < 7; i++) x = lane == i + 1 ? (uint32_t)v[i] : x;
    unsigned long long* mine = gran + ((size_t)(epoch & 1) * W + wself) * SX_VALS;
    __hip_atomic_store(mine + lane, tag | x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
      unsigned long long g[SX_VALS];
#pragma unroll
      for (int i = 0; i < SX_VALS; i++)
        g[i] = valid ? __hip_atomic_load(base + (size_t)s * SX_VALS + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : tag;
#pragma unroll
      for (int i = 0; i < SX_VALS; i++) {
        ok &= (g[i] >> 32) == epoch;
        got[ch][i] = valid ? (uint32_t)g[i] : 0u;
      }
      if (__all(ok)) break;
      if (spins >= SPIN_LIMIT) {
        if (lane == 0) {
          H.abort = 1;
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const long long k = (long long)(((unsigned long long)got[ch][1] << 32) | got[ch][0]);
    best = k > best ? k : best;
  }
  best = wave_red<OP_MAX>(best);
  int wstar = -1;
  if (best != 0) {
    const int g = (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)best);
    wstar = (g - node_base) / per;
  }
  long long nf = 0, tt = 0, na = 0;
#pragma unroll
  for (int ch = 0; ch < SX_CHUNKS; ch++) {
    const int s = ch * 64 + lane;
    if (s >= W) continue;
    const bool h1 = s == wstar;
    nf += (long long)(h1 ? got[ch][5] : got[ch][2]);
    const long long t = (long long)(h1 ? got[ch][6] : got[ch][3]);
    const long long a = (long long)(h1 ? got[ch][7] : got[ch][4]);
    tt = t > tt ? t : tt;
    na = a > na ? a : na;
  }
  nf = wave_red<OP_SUM>(nf);
  tt = wave_red<OP_MAX>(tt);
  na = wave_red<OP_MAX>(na);
  if (lane == 0) {
    H.res[0] = best;
    H.res[1] = nf;
    H.res[2] = tt;
    H.res[3] = na;
  }
  return true;
}

// Block-reduce the six partial statistics of the next pod, exchange them with the
// current pod's shard-best key, and leave {winner key, nf, max TT, max NA} in R[] of
// every lane.  False if the launch aborted (exchange timeout).
__device__ __forceinline__ bool simple_sync(SimpleHdr& H, int& parity, long long key, long long (&st)[6], int W, int w,
                                            unsigned epoch, unsigned long long* gran, int* err, int per, int node_base,
                                            long long (&R)[4], unsigned long long* sp) {
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
    simple_exchange(H, gran, W, w, epoch, err, v, per, node_base);
  }
  lds_barrier();
  if (H.abort) return false;
#pragma unroll
  for (int i = 0; i < 4; i++) R[i] = H.res[i];
  return true;
}

// One (pod, node) evaluation of the compact path: filter verdict and raw scores.
struct SVal {
  int f, tt, na, fit, ba;
};

// The filters of filter_local (kss_eval.cuh) and the four raw scores, with node labels
// from the shard's LDS table and the pod program from its LDS blob.  The TaintToleration
// / Fit failure details are not needed here (no record is kept on this path).
__device__ __forceinline__ SVal simple_eval(const DevCluster& c, const kss_profile& prof, const BlobView& B,
                                            const kss_pod& p, int n, const NodeRow& row, const int32_t* lbl, int cap,
                                            int si, unsigned long long* sp = nullptr) {
  SVal e{0, 0, 0, 0, 0};
  const int64_t g = (int64_t)c.node_base + n;
  auto lab = [&](int key) { return lbl[key * cap + si]; };
  if (p.names_len >= 0) {  // NodeAffinity PreFilterResult: nodes outside the set are not evaluated
    bool in = false;
    for (int i = 0; i < p.names_len; i++) in |= (int64_t)B.ints[p.names_off + i] == g;
    if (!in) {
      e.f = KSS_F_NOT_EVALUATED;
      return e;
    }
  }
  const uint32_t en = prof.filter_enabled;
  if (((en >> KSS_F_NODE_UNSCHEDULABLE) & 1u) && (row.flags & KSS_NODE_UNSCHEDULABLE) &&
      !(p.flags & KSS_POD_TOL_UNSCHEDULABLE)) {
    e.f = KSS_F_NODE_UNSCHEDULABLE;
  } else if (((en >> KSS_F_NODE_NAME) & 1u) && p.node_name != -1 && (int64_t)p.node_name != g) {
    e.f = KSS_F_NODE_NAME;
  } else if (((en >> KSS_F_TAINT_TOLERATION) & 1u) && (row.th & ~p.tol_hard)) {
    e.f = KSS_F_TAINT_TOLERATION;
  } else if (((en >> KSS_F_NODE_AFFINITY) & 1u) && !required_affinity_t(c, B.reqs, B.terms, B.ints, p, g, lab)) {
    e.f = KSS_F_NODE_AFFINITY;
  } else if ((en >> KSS_F_NODE_RESOURCES_FIT) & 1u) {
    bool bad = (int64_t)row.pods + 1 > (int64_t)row.allowed;
    const bool all_zero = p.fit_request[0] == 0 && p.fit_request[1] == 0 && p.fit_request[2] == 0;
    if (!all_zero) {
#pragma unroll
      for (int r = 0; r < 3; r++) bad |= p.fit_request[r] > row.alloc[r] - row.req[r];
    }
    if (bad) e.f = KSS_F_NODE_RESOURCES_FIT;
  }
  if (sp) sp[8] = wall_clock64();
  if (e.f) return e;
  e.tt = (int)tt_score(row, p);
  e.na = (int)na_score_t(c, B.reqs, B.terms, B.ints, p, g, lab);
  if (sp) sp[9] = wall_clock64();
  e.fit = (int)fit_score<true>(c, prof, p, n, row);
  if (sp) sp[10] = wall_clock64();
  e.ba = (int)ba_score(c, prof, p, n, row);
  if (sp) sp[11] = wall_clock64();
  return e;
}

// NormalizeScore + weights + packed selectHost key of one feasible node (the scored
// branch of schedule_pod<false>: PodTopologySpread normalises to 100 without
// constraints, InterPodAffinity keeps its raw 0).
__device__ __forceinline__ long long simple_key(const kss_profile& prof, const SVal& e, bool scored, long long max_tt,
                                                long long max_na, uint32_t g) {
  int64_t total = 0;
  if (scored) {
    const int64_t tt = max_tt == 0 ? 100 : 100 - div_i64<true>(100 * (int64_t)e.tt, max_tt);
    const int64_t na = max_na != 0 ? div_i64<true>(100 * (int64_t)e.na, max_na) : (int64_t)e.na;
    const uint32_t se = prof.score_enabled;
    if ((se >> KSS_S_TAINT_TOLERATION) & 1u) total += tt * prof.weight[KSS_S_TAINT_TOLERATION];
    if ((se >> KSS_S_NODE_AFFINITY) & 1u) total += na * prof.weight[KSS_S_NODE_AFFINITY];
    if ((se >> KSS_S_NODE_RESOURCES_FIT) & 1u) total += (int64_t)e.fit * prof.weight[KSS_S_NODE_RESOURCES_FIT];
    if ((se >> KSS_S_POD_TOPOLOGY_SPREAD) & 1u) total += 100 * (int64_t)prof.weight[KSS_S_POD_TOPOLOGY_SPREAD];
    if ((se >> KSS_S_BALANCED_ALLOCATION) & 1u) total += (int64_t)e.ba * prof.weight[KSS_S_BALANCED_ALLOCATION];
  }
  return (long long)(((unsigned long long)(uint32_t)total << 32) | (0xFFFFFFFFull - g));
}

// NodeInfo.AddPod on a node row (requested, non-zero requested, pod count).
__device__ __forceinline__ void add_commit(NodeRow& r, const kss_pod& p) {
#pragma unroll
  for (int k = 0; k < 3; k++) r.req[k] += p.commit_req[k];
  r.nz[0] += p.commit_nz[0];
  r.nz[1] += p.commit_nz[1];
  r.pods += 1;
}

// The shard's node state in LDS for the whole launch (slot s = node lo + s), and the
// per-slot results of the next pod; slot `cap` of the results holds the candidate node
// re-evaluated after the previous pod's commit (H1).
struct SimpleShard {
  int64_t* r64;  // [8][cap]: allocatable cpu/mem/eph, requested cpu/mem/eph, non-zero cpu/mem
  uint64_t* rt;  // [2][cap]: NoSchedule/NoExecute taints, PreferNoSchedule taints
  int32_t* r32;  // [3][cap]: pod count, allowed pods, node flags
  int32_t* lbl;  // [n_keys][cap]: label value ids
  int32_t* cv;   // [5][cap + 1]: filter verdict, TT, NA, Fit, BA
  int cap;
};

__host__ __device__ inline size_t simple_lds_bytes(int stride, int n_keys, int cap) {
  return sizeof(SimpleHdr) + 3 * (size_t)stride + (size_t)cap * (8 * 8 + 2 * 8 + 3 * 4 + 4 * (size_t)n_keys) +
         20 * ((size_t)cap + 1);
}

__device__ __forceinline__ SimpleShard shard_view(uint8_t* base, int n_keys, int cap) {
  SimpleShard L;
  L.cap = cap;
  L.r64 = reinterpret_cast<int64_t*>(base);
  L.rt = reinterpret_cast<uint64_t*>(base + 64 * (size_t)cap);
  L.r32 = reinterpret_cast<int32_t*>(base + 80 * (size_t)cap);
  L.lbl = L.r32 + 3 * (size_t)cap;
  L.cv = L.lbl + (size_t)n_keys * cap;
  return L;
}

__device__ __forceinline__ NodeRow shard_row(const SimpleShard& L, int s) {
  NodeRow r;
  const int C = L.cap;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    r.alloc[k] = L.r64[k * C + s];
    r.req[k] = L.r64[(3 + k) * C + s];
  }
  r.nz[0] = L.r64[6 * C + s];
  r.nz[1] = L.r64[7 * C + s];
  r.th = L.rt[s];
  r.ts = L.rt[C + s];
  r.pods = L.r32[s];
  r.allowed = L.r32[C + s];
  r.flags = (uint32_t)L.r32[2 * C + s];
  return r;
}

__device__ __forceinline__ SVal cv_get(const SimpleShard& L, int s) {
  const int C1 = L.cap + 1;
  return SVal{L.cv[s], L.cv[C1 + s], L.cv[2 * C1 + s], L.cv[3 * C1 + s], L.cv[4 * C1 + s]};
}

__device__ __forceinline__ void cv_put(const SimpleShard& L, int s, const SVal& e) {
  const int C1 = L.cap + 1;
  L.cv[s] = e.f;
  L.cv[C1 + s] = e.tt;
  L.cv[2 * C1 + s] = e.na;
  L.cv[3 * C1 + s] = e.fit;
  L.cv[4 * C1 + s] = e.ba;
}

// Pass A for the pod of blob B over the shard's `own` nodes on the current state (H0),
// plus the candidate slot `cand_s` (-1 none) re-evaluated with the previous pod `q`
// committed on it (H1), by the first slot without a node (slot `own`, which is slot
// `cap` of lane 0 when the shard is full).  st = {nf0, tt0, na0, nf1, tt1, na1}.
__device__ __forceinline__ void simple_pass_a(const DevCluster& c, const kss_profile& prof, const BlobView& B,
                                              const SimpleShard& L, int lo, int own, int cand_s, const kss_pod& q,
                                              long long (&st)[6], unsigned long long* sp) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const kss_pod& p = *B.pod;
  const bool pre_ok = p.prefilter_status == 0;
  long long nf = 0, tt = 0, na = 0, nf1 = 0, tt1 = 0, na1 = 0;
  for (int s = tid; s <= L.cap; s += nt) {
    const bool extra = s == own && cand_s >= 0;
    if (s >= own && !extra) continue;
    const int ns = extra ? cand_s : s;
    NodeRow r = shard_row(L, ns);
    if (extra) add_commit(r, q);
    if (sp && s == 0) sp[7] = wall_clock64();
    SVal e{KSS_F_NOT_EVALUATED, 0, 0, 0, 0};
    if (pre_ok) e = simple_eval(c, prof, B, p, lo + ns, r, L.lbl, L.cap, ns, (sp && s == 0) ? sp : nullptr);
    cv_put(L, extra ? L.cap : s, e);
    if (e.f == 0) {
      if (!extra) {
        nf++;
        tt = e.tt > tt ? e.tt : tt;
        na = e.na > na ? e.na : na;
      }
      if (s != cand_s) {
        nf1++;
        tt1 = e.tt > tt1 ? e.tt : tt1;
        na1 = e.na > na1 ? e.na : na1;
      }
    }
  }
  st[0] = nf;
  st[1] = tt;
  st[2] = na;
  st[3] = nf1;
  st[4] = tt1;
  st[5] = na1;
}

// The whole batch for shard w of one cluster (every pod commits).  On an exchange
// timeout the error word is set and the shard leaves without writing node state back.
__device__ __forceinline__ void simple_schedule(DevCluster c, const uint8_t* __restrict__ blobs, int stride, int n_pods,
                                                int32_t* chosen, PodMeta* meta, const kss_profile& prof, int W, int w,
                                                int cap, unsigned long long* gran, int* err,
                                                unsigned long long* stamps, long long* smem) {
  const int tid = threadIdx.x, nt = blockDim.x;
  SimpleHdr& H = *reinterpret_cast<SimpleHdr*>(smem);
  uint8_t* ring = reinterpret_cast<uint8_t*>(smem) + sizeof(SimpleHdr);
  const SimpleShard L = shard_view(ring + 3 * (size_t)stride, c.n_keys, cap);
  const size_t N = (size_t)c.N;
  const int per = (c.N + W - 1) / W;
  const int lo = min(c.N, w * per), hi = min(c.N, lo + per), own = hi - lo;
  if (n_pods <= 0) return;
  // shard rows and label ids -> LDS, blobs 0 and 1 -> ring
  for (int s = tid; s < own; s += nt) {
    const int n = lo + s;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      L.r64[k * cap + s] = c.alloc[k * N + n];
      L.r64[(3 + k) * cap + s] = c.requested[k * N + n];
    }
    L.r64[6 * cap + s] = c.nonzero[n];
    L.r64[7 * cap + s] = c.nonzero[N + n];
    L.rt[s] = c.taint_hard[n];
    L.rt[cap + s] = c.taint_soft[n];
    L.r32[s] = c.pod_count[n];
    L.r32[cap + s] = c.allowed_pods[n];
    L.r32[2 * cap + s] = (int32_t)c.node_flags[n];
  }
  for (int i = tid; i < c.n_keys * cap; i += nt) {
    const int k = i / cap, s = i - k * cap;
    L.lbl[i] = s < own ? c.label_value[(size_t)k * N + lo + s] : -1;
  }
  const int nq = stride / 16;
  for (int i = tid; i < min(n_pods, 2) * nq; i += nt)
    reinterpret_cast<uint4*>(ring)[i] = reinterpret_cast<const uint4*>(blobs)[i];
  if (tid == 0) H.abort = 0;
  __syncthreads();

  long long st[6], R[4] = {0, 0, 0, 0};
  int parity = 0, sub_s = -1;  // slot whose pass-B values are the H1 ones (the previous winner)
  unsigned epoch = 0;
  // k = -1 is the prologue: pass A of pod 0 and the exchange of its statistics
  for (int k = -1; k < n_pods; k++) {
    // diagnostic phase stamps (KSS_STAMPS_FILE), lane 0 of shard 0, first pods only
    unsigned long long* sp = (stamps && w == 0 && k >= 0 && k < KSS_NSTAMP_PODS / 2) ? stamps + (size_t)k * 16 : nullptr;
    if (sp && tid == 0) sp[0] = wall_clock64();
    const BlobView Bk = blob_view(ring + (size_t)((k + 3) % 3) * stride);
    const kss_pod& pk = *Bk.pod;
    // blob k+2 -> registers now, -> its ring slot at the end of this pod
    const bool pf_on = k >= 0 && k + 2 < n_pods;
    const uint4* pf_src = reinterpret_cast<const uint4*>(blobs + (size_t)(k + 2) * stride);
    uint4 pf[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const int i = q * nt + tid;
      pf[q] = make_uint4(0, 0, 0, 0);
      if (pf_on && i < nq) pf[q] = pf_src[i];
    }
    // pass B: NormalizeScore, weights, shard-best selectHost key of pod k
    const long long nf = R[1], max_tt = R[2], max_na = R[3];
    const bool scored = nf > 1;
    long long best = 0;
    if (k >= 0) {
      if (pk.prefilter_status == 0 && nf > 0) {
        for (int s = tid; s < own; s += nt) {
          const SVal e = cv_get(L, s == sub_s ? cap : s);
          if (e.f != 0) continue;
          const long long key = simple_key(prof, e, scored, max_tt, max_na, (uint32_t)(c.node_base + lo + s));
          best = key > best ? key : best;
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
    const int cand_s = best ? (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)best) - c.node_base - lo : -1;
    // pass A: pod k+1 before pod k's commit, and on the candidate after it
    if (k + 1 < n_pods) {
      const BlobView B1 = blob_view(ring + (size_t)((k + 1) % 3) * stride);
      simple_pass_a(c, prof, B1, L, lo, own, cand_s, pk, st, sp);
    } else {
#pragma unroll
      for (int i = 0; i < 6; i++) st[i] = 0;
    }
    if (sp && tid == 0) sp[3] = wall_clock64();
    if (!simple_sync(H, parity, best, st, W, w, ++epoch, gran, err, per, c.node_base, R, sp)) return;
    if (sp && tid == 0) sp[5] = wall_clock64();
    if (k < 0) continue;
    const long long K = R[0];
    const int x = K ? (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)K) - c.node_base : -1;
    if (w == 0 && tid == 0) {
      PodMeta m;
      m.chosen = K ? x + c.node_base : -1;
      m.n_feasible = (int)nf;
      m.scored = (K && scored) ? 1 : 0;
      m.status = pk.prefilter_status != 0 ? (pk.prefilter_status == 1 ? 2 : 3) : (nf == 0 ? 1 : 0);
      m.best_total = m.scored ? (int64_t)((unsigned long long)K >> 32) : 0;
      if (chosen) chosen[k] = m.chosen;
      if (meta) meta[k] = m;
    }
    // AssumePod on the winner's shard; pass B of pod k+1 takes that slot's H1 values
    const bool won = x >= lo && x < hi;
    sub_s = won ? x - lo : -1;
    if (won && tid == 0) {
      const int s = x - lo;
#pragma unroll
      for (int r = 0; r < 3; r++) L.r64[(3 + r) * cap + s] += pk.commit_req[r];
      L.r64[6 * cap + s] += pk.commit_nz[0];
      L.r64[7 * cap + s] += pk.commit_nz[1];
      L.r32[s] += 1;
      // HBM-only columns: no-return atomics, so the commit never waits on a load
      if (pk.cls >= 0) atomicAdd(&c.class_count[(size_t)pk.cls * N + x], 1);
      for (int i = 0; i < pk.own_terms_len; i++) atomicAdd(&c.term_count[(size_t)Bk.ints[pk.own_terms_off + i] * N + x], 1);
    }
    if (pf_on) {
      uint4* dst = reinterpret_cast<uint4*>(ring + (size_t)((k + 2) % 3) * stride);
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const int i = q * nt + tid;
        if (i < nq) dst[i] = pf[q];
      }
    }
    if (sp && tid == 0) sp[6] = wall_clock64();
  }
  // node state back to HBM
  __syncthreads();
  for (int s = tid; s < own; s += nt) {
    const int n = lo + s;
#pragma unroll
    for (int r = 0; r < 3; r++) c.requested[(size_t)r * N + n] = L.r64[(3 + r) * cap + s];
    c.nonzero[n] = L.r64[6 * cap + s];
    c.nonzero[N + n] = L.r64[7 * cap + s];
    c.pod_count[n] = L.r32[s];
  }
}

}  // namespace kss
