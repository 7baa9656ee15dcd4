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
constexpr int SX_CHUNKS = 1;    // shards swept 64 at a time: W <= 64

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

// LDS image of the loop head: reduction scratch (double-buffered), exchange results.
struct SimpleHdr {
  long long red[2][MAXWAVES][SX_VALS];
  long long res[4];  // winner key of the previous pod; nf, max TT, max NA of the next pod
  int abort;
  int pad[3];
};

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
  __syncthreads();
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
  const int ops[6] = {OP_SUM, OP_MAX, OP_MAX, OP_SUM, OP_MAX, OP_MAX};
  block_red(H, parity, st, ops);
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
  __syncthreads();
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

// NodeInfo.AddPod on a register row (requested, non-zero requested, pod count).
__device__ __forceinline__ void add_commit(NodeRow& r, const kss_pod& p) {
#pragma unroll
  for (int k = 0; k < 3; k++) r.req[k] += p.commit_req[k];
  r.nz[0] += p.commit_nz[0];
  r.nz[1] += p.commit_nz[1];
  r.pods += 1;
}

// Pass A for the pod of blob B: evaluate every owned node on the current state (H0),
// and the candidate node `cand` (cluster-local index, -1 none) once more with the
// previous pod `q` committed on it (H1, into alt).  st = {nf0, tt0, na0, nf1, tt1, na1}.
// The slot loop is kept rolled (slot NPT is the candidate's second evaluation), so the
// evaluation body exists once in the kernel; register arrays are only touched through
// constant-index select chains.
template <int NPT>
__device__ __forceinline__ void simple_pass_a(const DevCluster& c, const kss_profile& prof, const BlobView& B, int lo,
                                              int hi, const NodeRow (&row)[NPT], SVal (&cur)[NPT], SVal& alt,
                                              int cand, const kss_pod& q, const int32_t* lbl, int cap,
                                              long long (&st)[6], unsigned long long* sp = nullptr) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const kss_pod& p = *B.pod;
  const bool pre_ok = p.prefilter_status == 0;
  long long nf = 0, tt = 0, na = 0, nf1 = 0, tt1 = 0, na1 = 0;
  int cj = -1;
#pragma unroll
  for (int j = 0; j < NPT; j++)
    if (lo + j * nt + tid == cand) cj = j;
#pragma unroll 1
  for (int j = 0; j <= NPT; j++) {
    const bool extra = j == NPT;
    const int jj = extra ? (cj < 0 ? 0 : cj) : j;
    const int n = lo + jj * nt + tid;
    NodeRow r = row[0];
#pragma unroll
    for (int t = 1; t < NPT; t++)
      if (t == jj) r = row[t];
    if (extra) add_commit(r, q);
    SVal e{KSS_F_NOT_EVALUATED, 0, 0, 0, 0};
    if (sp && tid == 0 && !extra) sp[7] = wall_clock64();
    if (n < hi && pre_ok && (!extra || cj >= 0))
      e = simple_eval(c, prof, B, p, n, r, lbl, cap, jj * nt + tid, (sp && tid == 0 && !extra) ? sp : nullptr);
    const bool pass = e.f == 0;
    if (!extra) {
#pragma unroll
      for (int t = 0; t < NPT; t++)
        if (t == j) cur[t] = e;
      if (pass) {
        nf++;
        tt = e.tt > tt ? e.tt : tt;
        na = e.na > na ? e.na : na;
      }
    } else {
      alt = e;
    }
    if (pass && (extra || j != cj)) {
      nf1++;
      tt1 = e.tt > tt1 ? e.tt : tt1;
      na1 = e.na > na1 ? e.na : na1;
    }
  }
  st[0] = nf;
  st[1] = tt;
  st[2] = na;
  st[3] = nf1;
  st[4] = tt1;
  st[5] = na1;
}

__host__ __device__ inline size_t simple_lds_bytes(int stride, int n_keys, int cap) {
  return sizeof(SimpleHdr) + 3 * (size_t)stride + 4 * (size_t)n_keys * (size_t)cap;
}

// The whole batch for shard w of one cluster (every pod commits).  On an exchange
// timeout the error word is set and the shard leaves without writing node state back.
template <int NPT>
__device__ __forceinline__ void simple_schedule(DevCluster c, const uint8_t* __restrict__ blobs, int stride, int n_pods,
                                                int32_t* chosen, PodMeta* meta, const kss_profile& prof, int W, int w,
                                                unsigned long long* gran, int* err, unsigned long long* stamps,
                                                long long* smem) {
  const int tid = threadIdx.x, nt = blockDim.x, cap = NPT * nt;
  SimpleHdr& H = *reinterpret_cast<SimpleHdr*>(smem);
  uint8_t* ring = reinterpret_cast<uint8_t*>(smem) + sizeof(SimpleHdr);
  int32_t* lbl = reinterpret_cast<int32_t*>(ring + 3 * (size_t)stride);
  const size_t N = (size_t)c.N;
  const int per = (c.N + W - 1) / W;
  const int lo = min(c.N, w * per), hi = min(c.N, lo + per);
  if (n_pods <= 0) return;
  // shard rows -> registers, label ids -> LDS, blobs 0 and 1 -> ring
  NodeRow row[NPT];
#pragma unroll
  for (int j = 0; j < NPT; j++) {
    const int n = lo + j * nt + tid;
    row[j] = n < hi ? row_from_hbm(c, n) : NodeRow{};
  }
  for (int i = tid; i < c.n_keys * cap; i += nt) {
    const int k = i / cap, n = lo + (i - k * cap);
    lbl[i] = n < hi ? c.label_value[(size_t)k * N + n] : -1;
  }
  const int nq = stride / 16;
  for (int i = tid; i < min(n_pods, 2) * nq; i += nt)
    reinterpret_cast<uint4*>(ring)[i] = reinterpret_cast<const uint4*>(blobs)[i];
  if (tid == 0) H.abort = 0;
  __syncthreads();

  SVal cur[NPT];
  SVal alt{KSS_F_NOT_EVALUATED, 0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < NPT; j++) cur[j] = alt;
  long long st[6], R[4] = {0, 0, 0, 0};
  int parity = 0;
  unsigned epoch = 0;
  // k = -1 is the prologue: pass A of pod 0 and the exchange of its statistics
  for (int k = -1; k < n_pods; k++) {
    // diagnostic phase stamps (KSS_STAMPS_FILE), lane 0 of shard 0, first pods only
    unsigned long long* sp = (stamps && w == 0 && k >= 0 && k < KSS_NSTAMP_PODS / 2) ? stamps + (size_t)k * 16 : nullptr;
    if (sp && tid == 0) sp[0] = wall_clock64();
    const BlobView Bk = blob_view(ring + (size_t)((k + 3) % 3) * stride);
    const kss_pod& pk = *Bk.pod;
    // blob k+2 -> registers now, -> its ring slot once pod k-1's last reader is past
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
#pragma unroll
        for (int j = 0; j < NPT; j++) {
          if (cur[j].f != 0) continue;  // also every slot past hi (NOT_EVALUATED)
          const int n = lo + j * nt + tid;
          const long long key = simple_key(prof, cur[j], scored, max_tt, max_na, (uint32_t)(c.node_base + n));
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
    const int cand = best ? (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)best) - c.node_base : -1;
    // pass A: pod k+1 before pod k's commit, and on the candidate after it
    if (k + 1 < n_pods) {
      const BlobView B1 = blob_view(ring + (size_t)((k + 1) % 3) * stride);
      simple_pass_a<NPT>(c, prof, B1, lo, hi, row, cur, alt, cand, pk, lbl, cap, st, sp);
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
    // AssumePod by the owner lane: its row, and its pod k+1 values become the H1 ones
#pragma unroll
    for (int j = 0; j < NPT; j++) {
      const int n = lo + j * nt + tid;
      if (n == x && n < hi) {
        add_commit(row[j], pk);
        if (k + 1 < n_pods) cur[j] = alt;
        if (pk.cls >= 0) c.class_count[(size_t)pk.cls * N + n] += 1;
        for (int i = 0; i < pk.own_terms_len; i++) c.term_count[(size_t)Bk.ints[pk.own_terms_off + i] * N + n] += 1;
      }
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
#pragma unroll
  for (int j = 0; j < NPT; j++) {
    const int n = lo + j * nt + tid;
    if (n >= hi) continue;
#pragma unroll
    for (int r = 0; r < 3; r++) c.requested[(size_t)r * N + n] = row[j].req[r];
    c.nonzero[n] = row[j].nz[0];
    c.nonzero[N + n] = row[j].nz[1];
    c.pod_count[n] = row[j].pods;
  }
}

}  // namespace kss
