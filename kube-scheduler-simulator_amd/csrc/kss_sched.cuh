// kss_sched.cuh — the scheduling cycle for one pod over all nodes of one cluster.
//
// A cluster is served by W workgroups ("shards"); shard w owns the canonical node
// range [lo, hi) and is the only workgroup that reads or writes those nodes'
// mutable state, so node state never crosses workgroups.  Each lane owns NPT node
// slots (n = lo + k*blockDim + tid) and keeps every per-node intermediate of the
// cycle (verdict, raw scores) in registers: nothing per node goes to HBM unless the
// caller asked for a result record.
//
// Per pod (schedulePod) the phases are separated by cluster
// reductions ("exchanges"):
//   stats   PreFilter of PodTopologySpread (calPreFilterState) and InterPodAffinity
//           (existing / incoming (anti-)affinity counts) and InterPodAffinity PreScore
//           topologyScore: LDS-privatised histograms over topology domains for
//           non-unique keys; unique keys (hostname) are evaluated in place.
//           -> exchange: histogram SUM, presence OR, unique-key minima.
//   filter  findNodesThatPassFilters (first failing plugin wins) + raw Score of every
//           plugin on feasible nodes -> exchange: #feasible, max TT/NA, IPA min/max,
//           PTS ignored / domain presence.
//   pts     PodTopologySpread Score (needs the feasible-domain count) -> exchange min/max.
//   select  NormalizeScore, weights, TotalScore, selectHost (max total, lowest index)
//           -> exchange: packed (total, ~index) MAX.
//   commit  Cache.AssumePod -> NodeInfo.AddPod on the chosen row, by its owner shard.
//
// With W == 1 an exchange is a plain workgroup reduction (LDS + s_barrier).  With
// W > 1 wave 0 of every shard publishes the workgroup's partials as 8-byte
// {epoch, 32-bit half} granules with agent-scope (sc1) stores and sweeps every
// shard's granules with agent-scope loads until all tags carry the current epoch
// (MI355X_MICROARCH.md, "R2: the data is the flag"; no fences, no counters).  The
// granule slots are double-buffered by epoch parity: a shard can only publish
// epoch e+2 after every shard published e+1, i.e. after every shard finished
// reading epoch e.  Every spin is bounded; a timeout sets an error word and the
// workgroup leaves the kernel.
#pragma once
#include "kss_eval.cuh"

namespace kss {

constexpr int MAXH = 4;  // hard spread constraints per pod on the device path
constexpr int MAXS = 4;  // soft spread constraints
constexpr int MAXK = 4;  // distinct inter-pod-affinity topology keys
constexpr int MAXWAVES = 16;
constexpr int NSCAL = 16;      // scalar slots at the head of the exchange vector
constexpr int LDS_BINS = 4096; // histogram + presence values per pod (device limit)
constexpr int XW_MAX = 256;    // exchange length allowed when W > 1 (host-checked)
// Every exchange wait is bounded by wall time (s_memrealtime, 100 MHz), read every 64
// polls.  The bound is far above any exchange (microseconds) and above the start-up skew
// between the parts of a split grid, whose first launches are not aligned (code-object
// load, IPC open, a peer process starting late): the first exchange of a launch is the
// parts' handshake.
constexpr long long KSS_WAIT_TICKS = 1000000000ll;  // 10 s
__device__ __forceinline__ bool spin_expired(unsigned spins, long long& t0) {
  if (spins == 0) t0 = (long long)__builtin_amdgcn_s_memrealtime();
  if ((spins & 63u) != 63u) return false;
  return (long long)__builtin_amdgcn_s_memrealtime() - t0 > KSS_WAIT_TICKS;
}
// The launch error word only grows (atomic max): a state-check failure (2) is never
// overwritten by the exchange timeouts (1) it causes in the shards still waiting for it.
// The pause between two polls of an exchange granule (experiment builds: -DKSS_SPIN_SLEEP=0 polls
// back to back, larger values sleep longer; s_sleep n waits about 64 n clocks)
#ifndef KSS_SPIN_SLEEP
#define KSS_SPIN_SLEEP 1
#endif
__device__ __forceinline__ void spin_pause() {
  if (KSS_SPIN_SLEEP > 0) __builtin_amdgcn_s_sleep(KSS_SPIN_SLEEP);
}
__device__ __forceinline__ void err_raise(int* err, int code) {
  __hip_atomic_fetch_max(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// An exchange spin ends on the wall-time bound, or as soon as the launch has failed elsewhere
// (err != 0, read every 64 polls): the peers of a shard that left do not wait out the bound.
__device__ __forceinline__ bool spread_spin_over(unsigned spins, long long& t0, int* err) {
  if (spin_expired(spins, t0)) return true;
  return (spins & 63u) == 63u && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}
constexpr int KSS_MAX_THREADS = 512;  // workgroup size cap (2 waves per SIMD: 256 VGPRs per lane)
constexpr int KSS_NSTAMP_PODS = 256;  // pods with diagnostic phase stamps per launch
constexpr int KSS_MAX_NPT = 6;
constexpr size_t KSS_LDS_BUDGET = 160 * 1024;  // LDS per workgroup (one workgroup may own a whole CU's LDS)        // node slots per lane (LDS: 40 B per slot)

enum { OP_SUM = 0, OP_MAX = 1, OP_MIN = 2, OP_OR = 3 };
enum { SOFT_HOST = 0, SOFT_DIRECT = 1, SOFT_HIST = 2 };

// Per-pod plan, identical in every lane (computed from wave-uniform pod data).
// Constraints of one kind on one topology key form a group led by its first member (v1.26
// keys PodTopologySpread's counts by topology pair; kss_spread.cuh GSpread): hard_own /
// soft_own index the leader, whose bins the members share.
struct Plan {
  int n_hard, n_soft, n_keys;
  int hard_own[MAXH];
  int soft_own[MAXS];  // hostname constraints lead themselves (never grouped)
  int hard_off[MAXH];  // bin offset, -1 = unique key (direct)
  int hard_poff[MAXH]; // presence offset of the pair (key, domain)
  int soft_mode[MAXS];
  int soft_off[MAXS];  // count bins
  int soft_poff[MAXS]; // presence bins
  int key[MAXK];
  int key_off[MAXK];   // 4 consecutive histograms (x, a, b, s), -1 = unique (direct)
  int key_bins[MAXK];
  int total_bins;
  int hard_pbins;      // presence bins of hard constraints: [0, hard_pbins)
  int total_pbins;     // soft presence bins: [hard_pbins, total_pbins)
  bool need_stats;
};

// Nominated pods: per hard spread owner, the pairs at the critical-path minimum and the smallest
// count above it (uniform over the workgroup: kept in LDS, see NomView below)
struct NomPts {
  long long cnt[MAXH];  // pairs whose count equals the minimum (only 1 vs more matters)
  long long gt[MAXH];   // the smallest pair count above the minimum (INT32_MAX: none)
};

// Dynamic LDS image (Guideline 17: one 16-byte aligned dynamic region, no statics).
struct SharedHdr {
  NomPts npts;
  long long red[MAXWAVES][NSCAL];
  kss_pod pod;  // the current pod's record, copied once per pod
  Plan plan;    // computed by lane 0 of the workgroup each pod, read by all
  int plan_ok;
  int abort;
  unsigned svc_dirty;  // the service grid: record rows whose shard segment changed (kss_service.cuh)
  unsigned svc_ovf;    // the service grid: a compact record value did not fit its narrow type
  int cmd[4];   // the service grid's current command (kss_service.cuh)
  int svc_pf;   // the service grid's prefetched pod (its static words and record in LDS), -1 none
  int pad_[3];
};

__device__ __forceinline__ SharedHdr& shdr(long long* smem) { return *reinterpret_cast<SharedHdr*>(smem); }
// exchange vector: [0, NSCAL) scalars, then bins, then presence bins
__device__ __forceinline__ long long* xvec(long long* smem) { return smem + sizeof(SharedHdr) / 8; }

// Output slot for one pod: per-node verdicts and scores (the record format).
struct Slot {
  uint8_t* fail;
  uint16_t* detail;
  int64_t* raw;   // [KSS_NSCORE][N]
  int64_t* norm;  // [KSS_NSCORE][N]
  int64_t* total; // [N]
  bool canon = false;  // also write 0 to the entries the record leaves undefined (infeasible nodes'
                       // scores, an unscored pod's normalised scores and totals): the service grid
                       // sends only row segments that changed, so every entry must be a function
                       // of the pod and the state
};

struct PodMeta {
  int32_t chosen, n_feasible, scored, status;
  int64_t best_total;
};

// Shard geometry + exchange context of one workgroup.
struct Shard {
  int lo, hi;       // owned local node range
  int W, w;         // shards per cluster, this shard
  unsigned epoch;   // exchanges done so far in this launch (uniform over the cluster)
  unsigned long long* gran;  // this cluster's granules: [2][W][2*XW_MAX]
  int* err;         // launch error word (timeouts)
  unsigned long long* stamps;  // KSS_STAMPS diagnostics: phase timestamps of this pod, or null
  int cursor;       // nextStartNodeIndex of the cluster (identical in every shard; advanced per pod)
};

// numFeasibleNodesToFind (v1.26 schedule_one.go): every node when the list is short
// (< minFeasibleNodesToFind = 100) or pct >= 100; pct <= 0 is the adaptive default
// 50 - N/125 percent, at least minFeasibleNodesPercentageToFind = 5; at least 100 nodes.
__host__ __device__ __forceinline__ int num_feasible_to_find(int m, int pct) {
  if (m < 100 || pct >= 100) return m;
  int a = pct;
  if (a <= 0) {
    a = 50 - m / 125;
    if (a < 5) a = 5;
  }
  const int k = (int)((long long)m * a / 100);
  return k < 100 ? 100 : k;
}

// Diagnostic phase stamps (s_memrealtime, 100 MHz), lane 0 of shard 0 only.
#define KSS_STAMP(S, i)                                              \
  do {                                                               \
    if ((S).stamps && threadIdx.x == 0) (S).stamps[i] = wall_clock64(); \
  } while (0)

__device__ __forceinline__ long long op_apply(int op, long long a, long long b) {
  if (op == OP_SUM) return a + b;
  if (op == OP_MAX) return b > a ? b : a;
  if (op == OP_MIN) return b < a ? b : a;
  return a | b;
}

__device__ __forceinline__ long long op_identity(int op) {
  if (op == OP_MAX) return INT64_MIN;
  if (op == OP_MIN) return INT64_MAX;
  return 0;
}

__device__ __forceinline__ long long wave_reduce(long long v, int op) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = op_apply(op, v, __shfl_xor(v, m, 64));
  return v;
}

// Cross-shard part of an exchange, run by wave 0 only.  Payload j maps to
// xv[j] (j < K), then xv[NSCAL+sum_lo ...] (SUM), then xv[NSCAL+or_lo ...] (OR).
// Publish: two {epoch, half} granules per value.  Sweep: the W*M (shard, value)
// pairs are spread over the 64 lanes, XB pairs per lane per chunk with all loads in
// flight at once; a chunk is re-read until every tag carries the epoch (a matched
// granule is final: it can only change at epoch+2), then combined into the LDS
// value with a 64-bit LDS atomic of the value's operator.
__device__ __noinline__ void shard_exchange(long long* smem, unsigned long long* gran, int W, int wself, unsigned epoch,
                                            int* err, int K, unsigned opbits, int sum_lo, int ns, int or_lo, int no) {
  constexpr int XB = 8;
  long long* xv = xvec(smem);
  const int lane = threadIdx.x & 63;
  const int M = K + ns + no;
  const size_t per = 2 * (size_t)XW_MAX;
  unsigned long long* mine = gran + ((size_t)(epoch & 1) * W + wself) * per;
  auto slot = [&](int j) -> long long* {
    if (j < K) return xv + j;
    if (j < K + ns) return xv + NSCAL + sum_lo + (j - K);
    return xv + NSCAL + or_lo + (j - K - ns);
  };
  auto opof = [&](int j) { return j < K ? (int)((opbits >> (2 * j)) & 3u) : (j < K + ns ? OP_SUM : OP_OR); };
  const unsigned long long tag = (unsigned long long)epoch << 32;
  for (int j = lane; j < M; j += 64) {
    long long* sl = slot(j);
    const unsigned long long v = (unsigned long long)*sl;
    __hip_atomic_store(mine + 2 * j, tag | (v & 0xFFFFFFFFull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(mine + 2 * j + 1, tag | (v >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *sl = op_identity(opof(j));  // the own contribution comes back through the sweep
  }
  const unsigned long long* base = gran + (size_t)(epoch & 1) * W * per;
  const int Q = W * M;
  for (int q0 = 0; q0 < Q; q0 += 64 * XB) {
    unsigned long long lo[XB], hi[XB];
    long long t0_ = 0;
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int b = 0; b < XB; b++) {
        const int q = q0 + b * 64 + lane;
        lo[b] = hi[b] = tag;
        if (q < Q) {
          const int w = q / M, j = q - w * M;
          const unsigned long long* g = base + (size_t)w * per + 2 * j;
          lo[b] = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          hi[b] = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
#pragma unroll
      for (int b = 0; b < XB; b++) ok &= ((lo[b] >> 32) == epoch) & ((hi[b] >> 32) == epoch);
      if (__all(ok)) break;
      if (spin_expired(spins, t0_)) {
        if (lane == 0) {
          shdr(smem).abort = 1;
          err_raise(err, 1);
        }
        return;
      }
      __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int b = 0; b < XB; b++) {
      const int q = q0 + b * 64 + lane;
      if (q < Q) {
        const int w = q / M, j = q - w * M;
        const long long v = (long long)((hi[b] << 32) | (lo[b] & 0xFFFFFFFFull));
        long long* sl = slot(j);
        switch (opof(j)) {
          case OP_SUM: atomicAdd((unsigned long long*)sl, (unsigned long long)v); break;
          case OP_MAX: atomicMax(sl, v); break;
          case OP_MIN: atomicMin(sl, v); break;
          default: atomicOr((unsigned long long*)sl, (unsigned long long)v); break;
        }
      }
    }
  }
}

// Cluster reduction of K per-thread scalars v[] (ops[]), plus (W > 1 only) the
// cross-shard combination of the LDS bin ranges [sum_lo, sum_lo+ns) (SUM) and
// [or_lo, or_lo+no) (OR) of the exchange vector.  local = true reduces within the
// workgroup only (values already identical across shards).  On return v[] holds
// the cluster-wide results in every lane; returns false if the launch aborted.
template <int K>
__device__ __forceinline__ bool cluster_reduce(long long* smem, Shard& S, long long (&v)[K], const int (&ops)[K],
                                               int sum_lo = 0, int ns = 0, int or_lo = 0, int no = 0,
                                               bool local = false) {
  static_assert(K <= NSCAL, "too many values");
  SharedHdr& h = shdr(smem);
  long long* xv = xvec(smem);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < K; k++) {
    const long long r = wave_reduce(v[k], ops[k]);
    if (lane == 0) h.red[wave][k] = r;
  }
  __syncthreads();
  if (threadIdx.x < K) {
    const int k = threadIdx.x;
    int op = OP_SUM;
#pragma unroll
    for (int q = 0; q < K; q++)
      if (q == k) op = ops[q];
    long long r = h.red[0][k];
    for (int w = 1; w < nw; w++) r = op_apply(op, r, h.red[w][k]);
    xv[k] = r;
  }
  __syncthreads();
  if (S.W > 1 && !local) {
    unsigned opbits = 0;
#pragma unroll
    for (int k = 0; k < K; k++) opbits |= (unsigned)ops[k] << (2 * k);
    ++S.epoch;
    if (wave == 0) shard_exchange(smem, S.gran, S.W, S.w, S.epoch, S.err, K, opbits, sum_lo, ns, or_lo, no);
    __syncthreads();
    if (h.abort) return false;
  }
#pragma unroll
  for (int k = 0; k < K; k++) v[k] = xv[k];
  __syncthreads();  // xv[0..K) may be rewritten by the next reduction
  return true;
}

__host__ __device__ __forceinline__ bool key_unique(const DevCluster& c, int key) {
  return (c.key_flags[key] & KSS_KEY_UNIQUE) != 0;
}

// Returns false if the pod needs more LDS bins / slots than the device path has.  Host and
// device: the PostFilter dry run builds it on the host (key tables and the pod's programs in
// host memory) and ships it with the job.
__host__ __device__ __forceinline__ bool make_plan(const DevCluster& c, const DevPods& P, const kss_pod& p, Plan& pl,
                                          int bins_cap) {
  pl.n_hard = p.n_hard;
  pl.n_soft = p.n_soft;
  pl.n_keys = 0;
  pl.need_stats = false;
  int off = 0, poff = 0;
  if (p.n_hard > MAXH || p.n_soft > MAXS) return false;
  const kss_spread* sp = P.spreads + p.spread_off;
  for (int i = 0; i < p.n_hard; i++) {
    const int key = sp[i].key;
    pl.need_stats = true;
    int o = i;
    for (int j = 0; j < i; j++)
      if (sp[j].key == key) {
        o = j;
        break;
      }
    pl.hard_own[i] = o;
    if (o != i) {
      pl.hard_off[i] = pl.hard_off[o];
      pl.hard_poff[i] = pl.hard_poff[o];
    } else if (key_unique(c, key)) {
      pl.hard_off[i] = -1;
      pl.hard_poff[i] = -1;
    } else {
      pl.hard_off[i] = off;
      pl.hard_poff[i] = poff;
      off += c.key_card[key] + 1;
      poff += c.key_card[key] + 1;
    }
  }
  pl.hard_pbins = poff;
  for (int i = 0; i < p.n_soft; i++) {
    const int key = sp[p.n_hard + i].key;
    int o = i;
    if (!(c.key_flags[key] & KSS_KEY_HOSTNAME))
      for (int j = 0; j < i; j++)
        if (sp[p.n_hard + j].key == key) {
          o = j;
          break;
        }
    pl.soft_own[i] = o;
    if (c.key_flags[key] & KSS_KEY_HOSTNAME) {
      pl.soft_mode[i] = SOFT_HOST;
    } else if (key_unique(c, key)) {
      pl.soft_mode[i] = SOFT_DIRECT;
    } else {
      pl.soft_mode[i] = SOFT_HIST;
      pl.need_stats = true;
      if (o != i) {
        pl.soft_off[i] = pl.soft_off[o];
        pl.soft_poff[i] = pl.soft_poff[o];
      } else {
        pl.soft_off[i] = off;
        pl.soft_poff[i] = poff;
        off += c.key_card[key] + 1;
        poff += c.key_card[key] + 1;
      }
    }
  }
  const kss_ipa* ip = P.ipa + p.ipa_off;
  for (int e = 0; e < p.ipa_len; e++) {
    const int key = ip[e].key;
    int k = -1;
    for (int j = 0; j < pl.n_keys; j++)
      if (pl.key[j] == key) k = j;
    if (k < 0) {
      if (pl.n_keys >= MAXK) return false;
      k = pl.n_keys++;
      pl.key[k] = key;
      pl.key_bins[k] = c.key_card[key] + 1;
      if (key_unique(c, key)) {
        pl.key_off[k] = -1;
      } else {
        pl.key_off[k] = off;
        off += 4 * pl.key_bins[k];
      }
    }
    pl.need_stats = true;
  }
  pl.total_bins = off;
  pl.total_pbins = poff;
  return off + poff <= bins_cap;
}

__device__ __forceinline__ int slot_of(const Plan& pl, int key) {
  for (int j = 0; j < pl.n_keys; j++)
    if (pl.key[j] == key) return j;
  return -1;
}

// topologySpreadConstraint.matchNodeInclusionPolicies
__device__ __forceinline__ bool spread_policy_ok(const DevCluster& c, const DevPods& P, const kss_pod& p,
                                                 const kss_spread& s, int n) {
  if ((s.flags & KSS_SPREAD_POLICY_AFFINITY_HONOR) && !required_affinity(c, P, p, n)) return false;
  if ((s.flags & KSS_SPREAD_POLICY_TAINTS_HONOR) && first_untolerated(c, p, n, taint_hard_of(c, n)) >= 0) return false;
  return true;
}

__device__ __forceinline__ bool has_keys(const DevCluster& c, const kss_spread* s, int cnt, int n) {
  for (int i = 0; i < cnt; i++)
    if (label_of(c, s[i].key, n) < 0) return false;
  return true;
}

__device__ __forceinline__ int64_t spread_count(const DevCluster& c, const DevPods& P, const kss_spread& s, int n) {
  return sum_rows(c.class_count, (size_t)c.N, P.ints + s.cls_off, s.cls_len, n);
}

// ---------------------------------------------------------------------------
// stats pass for node n: accumulate LDS histograms (bins = xv+NSCAL, pres =
// bins+total_bins) and per-lane partials: hard_min[] for unique hard keys;
// flags bit0 ex, bit1 aff, bit2 anti, bit3 score nonempty
// ---------------------------------------------------------------------------
__device__ __forceinline__ void stats_node(const DevCluster& c, const DevPods& P, const kss_pod& p, const Plan& pl,
                                           long long* bins, long long* pres, int n, long long (&hard_min)[MAXH],
                                           long long& flags, bool scoring = true) {
  const kss_spread* sp = P.spreads + p.spread_off;
  if (p.n_hard > 0 && has_keys(c, sp, p.n_hard, n)) {  // nodeLabelsMatchSpreadConstraints
    for (int i = 0; i < p.n_hard; i++) {
      if (pl.hard_own[i] != i) continue;
      int64_t cnt = -1;  // tpCounts[pair]: the count of the group's last member admitting n
      for (int j = i; j < p.n_hard; j++)
        if (pl.hard_own[j] == i && spread_policy_ok(c, P, p, sp[j], n)) cnt = spread_count(c, P, sp[j], n);
      if (cnt < 0) continue;
      if (pl.hard_off[i] < 0) {
        hard_min[i] = cnt < hard_min[i] ? cnt : hard_min[i];
      } else {
        const int d = label_of(c, sp[i].key, n);
        atomicAdd((unsigned long long*)&bins[pl.hard_off[i] + d], (unsigned long long)cnt);
        pres[pl.hard_poff[i] + d] = 1;  // the pair (key, value) exists
      }
    }
  }
  if (scoring && p.n_soft > 0) {  // ScheduleAnyway: PreScore state (a filter-only caller skips it)
    const kss_spread* so = sp + p.n_hard;
    const bool req_all = (p.flags & KSS_POD_PTS_REQUIRE_ALL) != 0;
    if (!req_all || has_keys(c, so, p.n_soft, n)) {
      for (int i = 0; i < p.n_soft; i++) {
        if (pl.soft_mode[i] != SOFT_HIST) continue;
        if (!spread_policy_ok(c, P, p, so[i], n)) continue;
        int d = label_of(c, so[i].key, n);
        if (d < 0) d = c.key_empty[so[i].key];
        const int64_t cnt = spread_count(c, P, so[i], n);
        if (cnt) atomicAdd((unsigned long long*)&bins[pl.soft_off[i] + d], (unsigned long long)cnt);
      }
    }
  }
  if (p.ipa_len > 0) {
    const kss_ipa* ip = P.ipa + p.ipa_off;
    const bool has_labels = (node_flags_of(c, n) & KSS_NODE_HAS_LABELS) != 0;
    const size_t N = (size_t)c.N;
    for (int e = 0; e < p.ipa_len; e++) {
      const kss_ipa& en = ip[e];
      const int d = label_of(c, en.key, n);
      if (d < 0) continue;
      const int k = slot_of(pl, en.key);
      const int base = pl.key_off[k];
      const int nb = pl.key_bins[k];
      if (en.kind == KSS_IPA_SCORE_CLASS || en.kind == KSS_IPA_SCORE_TERM) {
        if (!scoring || !has_labels) continue;
        const int32_t* mat = en.kind == KSS_IPA_SCORE_CLASS ? c.class_count : c.term_count;
        const int64_t v = sum_rows(mat, N, P.ints + en.row_off, en.row_len, n);
        if (v > 0) flags |= 8;
        if (base >= 0 && v) atomicAdd((unsigned long long*)&bins[base + 3 * nb + d], (unsigned long long)(v * en.coef));
      } else {
        const int32_t* mat = en.kind == KSS_IPA_EXISTING_ANTI ? c.term_count : c.class_count;
        const int64_t v = sum_rows(mat, N, P.ints + en.row_off, en.row_len, n);
        const int h = en.kind == KSS_IPA_EXISTING_ANTI ? 0 : (en.kind == KSS_IPA_REQ_AFFINITY ? 1 : 2);
        if (v > 0) flags |= (1ll << h);
        if (base >= 0 && v) atomicAdd((unsigned long long*)&bins[base + h * nb + d], (unsigned long long)v);
      }
    }
  }
}

// value of an IPA histogram h (0 x, 1 a, 2 b) at node n's domain for key slot k
__device__ __forceinline__ int64_t ipa_value(const DevCluster& c, const DevPods& P, const kss_pod& p, const Plan& pl,
                                             const long long* bins, int k, int h, int d, int n) {
  if (pl.key_off[k] >= 0) return bins[pl.key_off[k] + h * pl.key_bins[k] + d];
  // unique key: the domain holds node n only -> recompute n's own contribution
  const int kind = h == 0 ? KSS_IPA_EXISTING_ANTI : (h == 1 ? KSS_IPA_REQ_AFFINITY : KSS_IPA_REQ_ANTI);
  const kss_ipa* ip = P.ipa + p.ipa_off;
  int64_t s = 0;
  for (int e = 0; e < p.ipa_len; e++) {
    if (ip[e].kind != kind || ip[e].key != pl.key[k]) continue;
    const int32_t* mat = kind == KSS_IPA_EXISTING_ANTI ? c.term_count : c.class_count;
    s += sum_rows(mat, (size_t)c.N, P.ints + ip[e].row_off, ip[e].row_len, n);
  }
  return s;
}

// ---------------------------------------------------------------------------
// Nominated pods (the scheduling queue's nominator, kss_nominate).  RunFilterPluginsWithNominatedPods
// (v1.26 runtime/framework.go) runs a node's filters first with the nominees of equal or higher
// priority (other than the pod itself) added -- addNominatedPods: NodeInfo.AddPodInfo plus the
// AddPod PreFilter extensions, which move only the node's own pairs -- and, when that passes, again
// on the plain node.  NomView is the table and the entries still nominated in this launch (an
// entry leaves when its pod is assumed: DeleteNominatedPodIfExists); NomPts, per hard spread
// owner, the pairs at the critical-path minimum and the smallest count above it, so that the
// minimum after the node's pair grows is min(the other pairs' minimum, the new count) -- what
// criticalPaths.update keeps when one pair changes.
// ---------------------------------------------------------------------------
struct NomView {
  const DevNom* e;
  int n;            // entries (0: no nominator, every nominee path compiles away at run time)
  int pod;          // the pod's identity (podset index)
  uint64_t active;  // entries still nominated
};

// the nominees RunFilterPluginsWithNominatedPods adds on node n for a pod of priority prio
__device__ __forceinline__ uint64_t nom_here(const NomView& nv, int n, int prio) {
  uint64_t m = 0;
  for (int j = 0; j < nv.n; j++) {
    const DevNom& e = nv.e[j];
    if (((nv.active >> j) & 1u) && e.node == n && e.pod != nv.pod && e.prio >= prio) m |= 1ull << j;
  }
  return m;
}

// podtopologyspread updateWithPod for hard owner o: one per matching constraint of the group, per nominee
__device__ __forceinline__ int64_t nom_pts_delta(const DevPods& P, const kss_pod& p, const Plan& pl, const NomView& nv,
                                                 uint64_t here, int o) {
  const kss_spread* sp = P.spreads + p.spread_off;
  int64_t dl = 0;
  for (uint64_t m = here; m; m &= m - 1) {
    const int cls = nv.e[__ffsll((unsigned long long)m) - 1].cls;
    for (int j = o; j < p.n_hard; j++)
      if (pl.hard_own[j] == o) {
        for (int i = 0; i < sp[j].cls_len; i++) dl += P.ints[sp[j].cls_off + i] == cls ? 1 : 0;
      }
  }
  return dl;
}

// interpodaffinity updateWithPod on histogram (key, kind): the nominees' required anti-affinity terms
// matching the pod (existing anti), or their class matching the pod's terms (affinity / anti)
__device__ __forceinline__ int64_t nom_ipa_delta(const DevPods& P, const kss_pod& p, const NomView& nv, uint64_t here,
                                                 int key, int kind) {
  const kss_ipa* ip = P.ipa + p.ipa_off;
  int64_t dl = 0;
  for (int e = 0; e < p.ipa_len; e++) {
    if (ip[e].kind != kind || ip[e].key != key) continue;
    for (uint64_t m = here; m; m &= m - 1) {
      const DevNom& q = nv.e[__ffsll((unsigned long long)m) - 1];
      if (kind == KSS_IPA_EXISTING_ANTI) {
        for (int t = 0; t < q.n_terms; t++)
          for (int i = 0; i < ip[e].row_len; i++) dl += P.ints[ip[e].row_off + i] == q.terms[t] ? 1 : 0;
      } else {
        for (int i = 0; i < ip[e].row_len; i++) dl += P.ints[ip[e].row_off + i] == q.cls ? 1 : 0;
      }
    }
  }
  return dl;
}

// PodTopologySpread.Filter (hard constraints) — returns detail+1 on failure, 0 on pass.  With nv /
// here / np: the first pass of RunFilterPluginsWithNominatedPods (bins: the histograms with the
// presence bins behind them, at total_bins).
__device__ __forceinline__ int filter_pts(const DevCluster& c, const DevPods& P, const kss_pod& p, const Plan& pl,
                                          const long long* bins, const long long (&hard_min)[MAXH], int n,
                                          const NomView* nv = nullptr, uint64_t here = 0, const NomPts* np = nullptr) {
  const kss_spread* sp = P.spreads + p.spread_off;
  // updateWithPod applies only on nodes with every constraint key whose labels match the pod's
  // required node affinity
  const bool upd = nv && has_keys(c, sp, p.n_hard, n) && required_affinity(c, P, p, n);
  for (int i = 0; i < p.n_hard; i++) {
    const int d = label_of(c, sp[i].key, n);
    if (d < 0) return 1 + KSS_PTS_MISSING_LABEL;
    const int o = pl.hard_own[i];
    int64_t match = 0;  // TpPairToMatchNum[(key, value)]
    bool present = false;
    if (pl.hard_off[i] >= 0) {
      match = bins[pl.hard_off[i] + d];
      if (nv) present = bins[pl.total_bins + pl.hard_poff[o] + d] != 0;
    } else if (has_keys(c, sp, p.n_hard, n)) {  // a node-valued key: the node's own group count
      for (int j = o; j < p.n_hard; j++)
        if (pl.hard_own[j] == o && spread_policy_ok(c, P, p, sp[j], n)) {
          match = spread_count(c, P, sp[j], n);
          present = true;
        }
    }
    int64_t mn = hard_min[o];
    if (upd) {
      const int64_t dl = nom_pts_delta(P, p, pl, *nv, here, o);
      if (dl) {
        int64_t others = mn;  // the minimum over the key's other pairs
        if (present && match == mn && np->cnt[o] == 1) others = np->gt[o];
        match += dl;
        mn = match < others ? match : others;
      }
    }
    const int64_t skew = match + (int64_t)sp[i].self_match - mn;
    if (skew > (int64_t)sp[i].max_skew) return 1 + KSS_PTS_CONSTRAINTS_NOT_MATCH;
  }
  return 0;
}

// InterPodAffinity.Filter — returns detail+1 on failure, 0 on pass.  flags: bit0 ex, bit1 aff, bit2 anti
// (len(counts) > 0).  With nv / here: the first pass of RunFilterPluginsWithNominatedPods (the
// nominees' contributions to the node's pairs, and the maps they make non-empty).
__device__ __forceinline__ int filter_ipa(const DevCluster& c, const DevPods& P, const kss_pod& p, const Plan& pl,
                                          const long long* bins, long long flags, int n, const NomView* nv = nullptr,
                                          uint64_t here = 0) {
  const kss_ipa* ip = P.ipa + p.ipa_off;
  auto value = [&](int key, int h, int d) -> int64_t {
    int64_t v = ipa_value(c, P, p, pl, bins, slot_of(pl, key), h, d, n);
    if (nv) v += nom_ipa_delta(P, p, *nv, here, key, h == 0 ? KSS_IPA_EXISTING_ANTI : (h == 1 ? KSS_IPA_REQ_AFFINITY : KSS_IPA_REQ_ANTI));
    return v;
  };
  if (nv) {
    for (int e = 0; e < p.ipa_len; e++) {
      const int kind = ip[e].kind;
      if (kind > KSS_IPA_REQ_ANTI || label_of(c, ip[e].key, n) < 0) continue;
      if (nom_ipa_delta(P, p, *nv, here, ip[e].key, kind) > 0)
        flags |= kind == KSS_IPA_EXISTING_ANTI ? 1 : (kind == KSS_IPA_REQ_AFFINITY ? 2 : 4);
    }
  }
  // satisfyPodAffinity
  bool have = false, exist = true;
  for (int e = 0; e < p.ipa_len; e++) {
    if (ip[e].kind != KSS_IPA_REQ_AFFINITY) continue;
    have = true;
    const int d = label_of(c, ip[e].key, n);
    if (d < 0) return 1 + KSS_IPA_AFFINITY;
    if (value(ip[e].key, 1, d) <= 0) exist = false;
  }
  if (have && !exist && !(!(flags & 2) && (p.flags & KSS_POD_IPA_SELF_MATCH))) return 1 + KSS_IPA_AFFINITY;
  // satisfyPodAntiAffinity
  if (flags & 4) {
    for (int e = 0; e < p.ipa_len; e++) {
      if (ip[e].kind != KSS_IPA_REQ_ANTI) continue;
      const int d = label_of(c, ip[e].key, n);
      if (d < 0) continue;
      if (value(ip[e].key, 2, d) > 0) return 1 + KSS_IPA_ANTI_AFFINITY;
    }
  }
  // satisfyExistingPodsAntiAffinity
  if (flags & 1) {
    for (int e = 0; e < p.ipa_len; e++) {
      if (ip[e].kind != KSS_IPA_EXISTING_ANTI) continue;
      const int d = label_of(c, ip[e].key, n);
      if (d < 0) continue;
      if (value(ip[e].key, 0, d) > 0) return 1 + KSS_IPA_EXISTING_ANTI_AFFINITY;
    }
  }
  return 0;
}

// InterPodAffinity.Score: Σ topologyScore[key][node value] over keys the node has
__device__ __forceinline__ int64_t ipa_score(const DevCluster& c, const DevPods& P, const kss_pod& p, const Plan& pl,
                                             const long long* bins, int n) {
  int64_t s = 0;
  const bool has_labels = (node_flags_of(c, n) & KSS_NODE_HAS_LABELS) != 0;
  for (int k = 0; k < pl.n_keys; k++) {
    const int d = label_of(c, pl.key[k], n);
    if (d < 0) continue;
    if (pl.key_off[k] >= 0) {
      s += bins[pl.key_off[k] + 3 * pl.key_bins[k] + d];
    } else if (has_labels) {
      const kss_ipa* ip = P.ipa + p.ipa_off;
      for (int e = 0; e < p.ipa_len; e++) {
        if (ip[e].key != pl.key[k]) continue;
        if (ip[e].kind != KSS_IPA_SCORE_CLASS && ip[e].kind != KSS_IPA_SCORE_TERM) continue;
        const int32_t* mat = ip[e].kind == KSS_IPA_SCORE_CLASS ? c.class_count : c.term_count;
        s += (int64_t)ip[e].coef * sum_rows(mat, (size_t)c.N, P.ints + ip[e].row_off, ip[e].row_len, n);
      }
    }
  }
  return s;
}

__device__ __forceinline__ bool in_names(const DevPods& P, const kss_pod& p, int64_t g) {
  for (int i = 0; i < p.names_len; i++)
    if ((int64_t)P.ints[p.names_off + i] == g) return true;
  return false;
}

// Per-node-slot intermediates of one pod, in LDS (slot s = k*blockDim + tid).
struct SlotArrays {
  long long* na;   // NodeAffinity raw
  long long* ipa;  // InterPodAffinity raw
  long long* pts;  // PodTopologySpread raw
  int* fail;       // verdict | ignored << 16
  int* tt;         // TaintToleration raw
  int* fit;        // NodeResourcesFit raw
  int* ba;         // BalancedAllocation raw
};

__host__ __device__ inline size_t slot_arrays_bytes(int cap) { return (size_t)cap * (3 * 8 + 4 * 4); }
// shard node cache: 10 x 8 B + 3 x 4 B per node, plus 4 B per cached label key
__host__ __device__ inline size_t node_cache_bytes(int cap, int n_keys) { return (size_t)cap * (10 * 8 + 3 * 4 + 4 * n_keys); }

__device__ __forceinline__ SlotArrays slot_arrays(long long* smem, int bins_cap, int cap) {
  long long* b = xvec(smem) + NSCAL + bins_cap;
  SlotArrays a;
  a.na = b;
  a.ipa = b + cap;
  a.pts = b + 2 * cap;
  int* i = reinterpret_cast<int*>(b + 3 * cap);
  a.fail = i;
  a.tt = i + cap;
  a.fit = i + 2 * cap;
  a.ba = i + 3 * cap;
  return a;
}

// RunFilterPlugins for node n: the verdict (first failing plugin, 0 = passed) and its detail;
// row holds the node's columns afterwards (the score pass reads them).
template <bool GEN>
__device__ __forceinline__ int filter_chain(const DevCluster& c, const DevPods& P, const kss_pod& p, const Plan& pl,
                                            const long long* bins, const long long (&hard_min)[MAXH], long long flags,
                                            uint32_t en, bool has_ipa, int n, NodeRow& row, uint16_t* detail,
                                            const NomView* nv = nullptr, uint64_t here = 0, const NomPts* np = nullptr) {
  row = load_row(c, n);
  int f = filter_local(c, P, p, en, n, row, detail, nv ? nv->e : nullptr, here);
  if (!f) f = filter_volumes(c, P, p, en, n, detail);
  if (GEN && !f && ((en >> KSS_F_POD_TOPOLOGY_SPREAD) & 1u) && p.n_hard > 0) {
    const int r = filter_pts(c, P, p, pl, bins, hard_min, n, nv, here, np);
    if (r) {
      f = KSS_F_POD_TOPOLOGY_SPREAD;
      *detail = (uint16_t)(r - 1);
    }
  }
  if (!f && ((en >> KSS_F_INTER_POD_AFFINITY) & 1u) && has_ipa) {
    const int r = filter_ipa(c, P, p, pl, bins, flags, n, nv, here);
    if (r) {
      f = KSS_F_INTER_POD_AFFINITY;
      *detail = (uint16_t)(r - 1);
    }
  }
  return f;
}

// RunFilterPluginsWithNominatedPods for node n: with nominees on n the first pass (nominees added)
// decides when it fails, the plain pass otherwise.  A failure of the plain pass after a passing
// first pass can only be InterPodAffinity's required affinity -- the last filter plugin -- so the
// plain record is the simulator's (store.go:423 overwrites per plugin) as it stands.
template <bool GEN>
__device__ __forceinline__ int filter_nominated(const DevCluster& c, const DevPods& P, const kss_pod& p, const Plan& pl,
                                                const long long* bins, const long long (&hard_min)[MAXH],
                                                long long flags, uint32_t en, bool has_ipa, int n, NodeRow& row,
                                                uint16_t* detail, const NomView& nv, const NomPts& np) {
  const int f = filter_chain<GEN>(c, P, p, pl, bins, hard_min, flags, en, has_ipa, n, row, detail);
  if (nv.n == 0) return f;
  const uint64_t here = nom_here(nv, n, p.priority);
  if (!here) return f;
  NodeRow r1;
  uint16_t d1 = 0;
  const int f1 = filter_chain<GEN>(c, P, p, pl, bins, hard_min, flags, en, has_ipa, n, r1, &d1, &nv, here, &np);
  if (f1 == KSS_F_PASS) return f;
  *detail = d1;
  return f1;
}

// Position of global node g in the pod's ascending PreFilterResult list (binary search).
__device__ __forceinline__ int names_rank(const DevPods& P, const kss_pod& p, int64_t g) {
  int lo = 0, hi = p.names_len;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int64_t)P.ints[p.names_off + mid] < g) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// ---------------------------------------------------------------------------
// one scheduling cycle for pod pi, executed by every shard of the cluster.
// Returns false if the launch aborted (exchange timeout).
// ---------------------------------------------------------------------------
// GEN = false compiles the cycle without PodTopologySpread / InterPodAffinity programs
// (the host picks it when no pod of the batch carries one): a compact kernel whose hot
// loop stays in the instruction cache.
template <bool GEN>
__device__ __forceinline__ bool schedule_pod(const DevCluster& c, const DevPods& P, const kss_profile& prof, int pi, long long* smem,
                             Shard& S, int bins_cap, int npt, const Slot* out, bool keep_norm, PodMeta& meta,
                             const NomView& nv) {
  const int tid = threadIdx.x, nt = blockDim.x;
  SharedHdr& H = shdr(smem);
  {
    // pod record -> LDS (one coalesced copy), plan by lane 0; one barrier
    constexpr int PD = (int)(sizeof(kss_pod) / 4);
    const uint32_t* src = reinterpret_cast<const uint32_t*>(P.pods + pi);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&H.pod);
    for (int i = tid; i < PD; i += nt) dst[i] = src[i];
    if (tid == 0) {
      if (GEN) {
        H.plan_ok = make_plan(c, P, P.pods[pi], H.plan, bins_cap) ? 1 : 0;
      } else {
        const kss_pod& q = P.pods[pi];
        H.plan_ok = (q.n_hard | q.n_soft | q.ipa_len) == 0 ? 1 : 0;  // the host guarantees it
        H.plan.total_bins = H.plan.hard_pbins = H.plan.total_pbins = 0;
        H.plan.need_stats = false;
      }
    }
    __syncthreads();
  }
  const kss_pod& p = H.pod;
  const size_t NN = (size_t)c.N;
  long long* xv = xvec(smem);
  long long* bins = xv + NSCAL;
  const SlotArrays sa = slot_arrays(smem, bins_cap, npt * nt);
  meta.chosen = -1;
  meta.n_feasible = 0;
  meta.scored = 0;
  meta.status = 0;
  meta.best_total = 0;

  const Plan& pl = H.plan;
  const bool plan_ok = H.plan_ok != 0;
  long long* pres = bins + pl.total_bins;
  KSS_STAMP(S, 1);
  if (p.prefilter_status != 0 || !plan_ok) {
    if (out) {
      for (int k = 0; k < npt; k++) {
        const int n = S.lo + k * nt + tid;
        if (n < S.hi) {
          out->fail[n] = KSS_F_NOT_EVALUATED;
          out->detail[n] = 0;
        }
      }
    }
    meta.status = !plan_ok ? 4 : (p.prefilter_status == KSS_PF_ERROR ? 3 : 2);
    return true;
  }

  // ---- stats -----------------------------------------------------------
  long long hard_min[MAXH];
  long long flags = 0;
  NomPts& npts = H.npts;
#pragma unroll
  for (int i = 0; i < MAXH; i++) hard_min[i] = INT32_MAX;
  if (GEN && pl.need_stats) {
    for (int b = tid; b < pl.total_bins + pl.total_pbins; b += nt) bins[b] = 0;
    __syncthreads();
    for (int k = 0; k < npt; k++) {
      const int n = S.lo + k * nt + tid;
      if (n < S.hi) stats_node(c, P, p, pl, bins, pres, n, hard_min, flags);
    }
    long long v[MAXH + 1];
    const int op[MAXH + 1] = {OP_MIN, OP_MIN, OP_MIN, OP_MIN, OP_OR};
#pragma unroll
    for (int i = 0; i < MAXH; i++) v[i] = hard_min[i];
    v[MAXH] = flags;
    // histogram SUM over every bin, hard-pair presence OR (soft presence is filled later)
    if (!cluster_reduce(smem, S, v, op, 0, pl.total_bins, pl.total_bins, pl.hard_pbins)) return false;
    flags = v[MAXH];
    // minima over present bins of non-unique hard keys (bins are cluster-wide now)
    const kss_spread* sp = P.spreads + p.spread_off;
    long long m[MAXH];
#pragma unroll
    for (int i = 0; i < MAXH; i++) m[i] = v[i];
    bool any_hist = false;
#pragma unroll
    for (int i = 0; i < MAXH; i++) {
      if (i >= p.n_hard) break;
      if (pl.hard_off[i] < 0 || pl.hard_own[i] != i) continue;
      any_hist = true;
      const int nb = c.key_card[sp[i].key] + 1;
      for (int b = tid; b < nb; b += nt) {
        const int g = pl.hard_off[i] + b;
        if (pres[pl.hard_poff[i] + b]) m[i] = bins[g] < m[i] ? bins[g] : m[i];
      }
    }
    if (any_hist) {
      const int opm[MAXH] = {OP_MIN, OP_MIN, OP_MIN, OP_MIN};
      cluster_reduce(smem, S, m, opm, 0, 0, 0, 0, /*local=*/true);
    }
#pragma unroll
    for (int i = 0; i < MAXH; i++) hard_min[i] = m[i];
    // soft presence bins start empty for the filter pass
    for (int b = pl.hard_pbins + tid; b < pl.total_pbins; b += nt) pres[b] = 0;
    __syncthreads();
    if (nv.n && p.n_hard > 0) {
      // nominees: per hard owner, the pairs at the minimum and the smallest count above it (one
      // more exchange; histogram keys are cluster-wide already, so shard 0 alone adds them)
      long long v2[2 * MAXH];
      const int op2[2 * MAXH] = {OP_SUM, OP_SUM, OP_SUM, OP_SUM, OP_MIN, OP_MIN, OP_MIN, OP_MIN};
#pragma unroll
      for (int i = 0; i < MAXH; i++) {
        v2[i] = 0;
        v2[MAXH + i] = INT32_MAX;
      }
#pragma unroll
      for (int i = 0; i < MAXH; i++) {
        if (i >= p.n_hard || pl.hard_own[i] != i) continue;
        const long long mn = hard_min[i];
        if (pl.hard_off[i] >= 0) {
          if (S.w != 0) continue;
          const int nb = c.key_card[sp[i].key] + 1;
          for (int b = tid; b < nb; b += nt) {
            if (!pres[pl.hard_poff[i] + b]) continue;
            const long long x = bins[pl.hard_off[i] + b];
            v2[i] += x == mn ? 1 : 0;
            if (x > mn && x < v2[MAXH + i]) v2[MAXH + i] = x;
          }
        } else {
          for (int k = 0; k < npt; k++) {
            const int n = S.lo + k * nt + tid;
            if (n >= S.hi || !has_keys(c, sp, p.n_hard, n)) continue;
            long long x = -1;
            for (int j = i; j < p.n_hard; j++)
              if (pl.hard_own[j] == i && spread_policy_ok(c, P, p, sp[j], n)) x = spread_count(c, P, sp[j], n);
            if (x < 0) continue;
            v2[i] += x == mn ? 1 : 0;
            if (x > mn && x < v2[MAXH + i]) v2[MAXH + i] = x;
          }
        }
      }
      if (!cluster_reduce(smem, S, v2, op2)) return false;
      if (tid == 0)
#pragma unroll
        for (int i = 0; i < MAXH; i++) {
          npts.cnt[i] = v2[i];
          npts.gt[i] = v2[MAXH + i];
        }
      __syncthreads();
    }
  }

  KSS_STAMP(S, 7);  // the PodTopologySpread / InterPodAffinity statistics and their exchange done
  // ---- PreferNominatedNode (findNodesThatFitPod -> evaluateNominatedNode) ---------------------
  // A pod an earlier preemption nominated first runs findNodesThatPassFilters on [its node] alone,
  // whatever its PreFilterResult; the one-node list resets nextStartNodeIndex to 0.  A feasible
  // node is chosen without scoring (only its record is written); otherwise its status stands in
  // the diagnosis and the full search follows (the same verdict if it reaches the node again).
  int nom_m = -1, nom_f = KSS_F_PASS;
  uint16_t nom_d = 0;
  bool nom_failed = false;  // uniform: evaluateNominatedNode's failure is in the diagnosis map
  if (nv.n) {
    for (int j = 0; j < nv.n; j++)
      if (((nv.active >> j) & 1u) && nv.e[j].pod == nv.pod) nom_m = nv.e[j].node;
  }
  if (nom_m >= 0 && nom_m < c.N) {
    long long v[1] = {0};
    const bool mine = nom_m >= S.lo && nom_m < S.hi && ((nom_m - S.lo) % nt) == tid;
    if (mine) {
      NodeRow row;
      nom_f = filter_nominated<GEN>(c, P, p, pl, bins, hard_min, flags, prof.filter_enabled, GEN && p.ipa_len > 0,
                                    nom_m, row, &nom_d, nv, npts);
      v[0] = nom_f == KSS_F_PASS ? 1 : 0;
    }
    const int op[1] = {OP_MAX};
    if (!cluster_reduce(smem, S, v, op)) return false;
    S.cursor = 0;
    if (v[0]) {
      if (out) {
        for (int k = 0; k < npt; k++) {
          const int n = S.lo + k * nt + tid;
          if (n >= S.hi) continue;
          out->fail[n] = n == nom_m ? (uint8_t)KSS_F_PASS : (uint8_t)KSS_F_NOT_EVALUATED;
          out->detail[n] = 0;
          if (out->canon) {
#pragma unroll
            for (int x = 0; x < KSS_NSCORE; x++) out->raw[(size_t)x * NN + n] = 0;
            if (keep_norm) {
#pragma unroll
              for (int x = 0; x < KSS_NSCORE; x++) out->norm[(size_t)x * NN + n] = 0;
              out->total[n] = 0;
            }
          }
        }
      }
      meta.n_feasible = 1;
      meta.chosen = (int)(c.node_base + nom_m);
      return true;
    }
    nom_failed = true;
    if (!mine) nom_m = -1;  // only the owning lane overrides the node's record below
  } else {
    nom_m = -1;
  }

  // ---- filter + raw scores -------------------------------------------------
  const uint32_t en = prof.filter_enabled;
  const bool restrict_names = p.names_len >= 0;
  const kss_spread* soft = P.spreads + p.spread_off + p.n_hard;
  const bool req_all = (p.flags & KSS_POD_PTS_REQUIRE_ALL) != 0;
  const bool has_soft = GEN && p.n_soft > 0;
  const bool has_ipa = GEN && p.ipa_len > 0;

  // ---- percentageOfNodesToScore: findNodesThatPassFilters' window ------------
  // The node list (every node, or the PreFilterResult set in canonical order) is visited from
  // nextStartNodeIndex, one node at a time (Parallelism = 1, the deterministic form), until
  // one feasible node more than K = numFeasibleNodesToFind has been found: that node was
  // filtered (its record says passed) but is neither counted nor scored, and the nodes after
  // it were never evaluated.  With Fb(n) = the feasible nodes strictly before n in visiting
  // order: n is visited iff Fb <= K, and scored iff feasible and Fb < K.  A pre-pass counts the
  // feasible nodes per shard (one exchange: the per-shard counts and the feasible nodes before
  // the start node); the stopping node's shard reports the nodes processed with the selectHost
  // exchange, and nextStartNodeIndex advances by them.
  const int m_list = restrict_names ? p.names_len : c.N;
  const int k_find = num_feasible_to_find(m_list, prof.pct_nodes_to_score);
  const bool win = k_find < m_list;
  long long w_total = 0, w_gstar = 0, w_pre = 0;
  int nstar = 0, spos = 0;
  if (m_list > 0 && !win) S.cursor = (int)(((long long)S.cursor + m_list) % m_list);  // every node processed
  if (win) {
    const int lane = tid & 63, wave = tid >> 6, nw = nt >> 6;
    spos = (int)((long long)S.cursor % m_list);
    nstar = restrict_names ? (int)((int64_t)P.ints[p.names_off + spos] - c.node_base) : spos;
    long long lt = 0;  // this lane's feasible nodes before the start node
    for (int k = 0; k < npt; k++) {
      const int n = S.lo + k * nt + tid;
      bool fe = false;
      if (n < S.hi && (!restrict_names || in_names(P, p, (int64_t)c.node_base + n))) {
        NodeRow row;
        uint16_t d = 0;
        fe = filter_nominated<GEN>(c, P, p, pl, bins, hard_min, flags, en, has_ipa, n, row, &d, nv, npts) == KSS_F_PASS;
      }
      const unsigned long long b = __ballot(fe);
      sa.fit[k * nt + tid] = (int)__popcll(b & ((1ull << lane) - 1ull));  // feasible lanes before this one, row k
      if (lane == 0) H.red[wave][k] = (long long)__popcll(b);
      lt += (fe && n < nstar) ? 1 : 0;
    }
    __syncthreads();
    long long run = 0;  // shard-local exclusive prefix in canonical order: rows before k, waves before this one
    for (int k = 0; k < npt; k++) {
      long long row_tot = 0, before = 0;
      for (int x = 0; x < nw; x++) {
        row_tot += H.red[x][k];
        before += x < wave ? H.red[x][k] : 0;
      }
      sa.fit[k * nt + tid] += (int)(run + before);
      run += row_tot;
    }
    __syncthreads();  // H.red is the reduction scratch of the exchange below
    const int wb = bins_cap - S.W;  // the per-shard counts, behind the plan's bins (the host reserves W)
    for (int j = tid; j < S.W; j += nt) bins[wb + j] = j == S.w ? run : 0;
    long long v[1] = {lt};
    const int op[1] = {OP_SUM};
    if (!cluster_reduce(smem, S, v, op, wb, S.W)) return false;
    w_gstar = v[0];
    for (int j = 0; j < S.W; j++) {
      const long long t = bins[wb + j];
      w_total += t;
      w_pre += j < S.w ? t : 0;
    }
    if (w_total <= k_find) S.cursor = (int)(((long long)S.cursor + m_list) % m_list);  // no stop: all processed
  }
  long long w_proc = 0;  // nodes processed before the stopping node (its lane only)
  // the nominated node's map entry counts once more unless the search reaches that node again
  // (it is outside the list, or after the stopping node): its lane only
  long long nom_x = 0;

  long long nf = 0, max_tt = 0, max_na = 0;
  long long nign = 0, ipa_min = INT64_MAX, ipa_max = INT64_MIN, smissing = 0;
  long long sdirect[MAXS];
#pragma unroll
  for (int i = 0; i < MAXS; i++) sdirect[i] = 0;
  for (int k = 0; k < npt; k++) {
    const int n = S.lo + k * nt + tid;
    const int si = k * nt + tid;
    if (n >= S.hi) {
      sa.fail[si] = KSS_F_NOT_EVALUATED;
      continue;
    }
    uint16_t detail = 0;
    int f;
    NodeRow row;
    if (restrict_names && !in_names(P, p, (int64_t)c.node_base + n)) {
      f = KSS_F_NOT_EVALUATED;
    } else {
      f = filter_nominated<GEN>(c, P, p, pl, bins, hard_min, flags, en, has_ipa, n, row, &detail, nv, npts);
    }
    bool kept = f == KSS_F_PASS;
    if (win && f != KSS_F_NOT_EVALUATED) {
      const long long g = w_pre + sa.fit[si];  // feasible nodes before n in canonical order
      const long long fb = n >= nstar ? g - w_gstar : w_total - w_gstar + g;
      if (fb > k_find) {  // the search stopped before reaching n
        f = KSS_F_NOT_EVALUATED;
        detail = 0;
        kept = false;
      } else if (kept && fb == k_find) {  // the stopping node: filtered, dropped, not scored
        kept = false;
        detail = KSS_PASS_NOT_KEPT;
        w_proc = restrict_names ? ((long long)names_rank(P, p, (int64_t)c.node_base + n) - spos + m_list) % m_list
                                : ((long long)n - nstar + m_list) % m_list;
      }
    }
    if (n == nom_m) {  // evaluateNominatedNode's status (infeasible, so never kept): it stands
      nom_x = f == KSS_F_NOT_EVALUATED ? 1 : 0;
      f = nom_f;
      detail = nom_d;
      kept = false;
    }
    if (out) {
      KSS_DCHECK(n >= 0 && n < c.N, "out n", n, c.N);
      out->fail[n] = (uint8_t)f;
      out->detail[n] = detail;
      if (out->canon && !kept)
#pragma unroll
        for (int x = 0; x < KSS_NSCORE; x++) out->raw[(size_t)x * NN + n] = 0;
    }
    if (!kept) f = f == KSS_F_PASS ? KSS_F_NOT_EVALUATED : f;  // the dropped node leaves the feasible list
    int ign = 0, il = 0;
    if (f == KSS_F_PASS) {
      nf++;
      il = (int)il_score(c, P, p, n);  // ImageLocality.Score in [0, 100], carried in the fail word
      const int64_t tt = tt_score(row, p);
      const int64_t na = na_score(c, P, p, n);
      const int64_t fit = fit_score(c, prof, p, n, row);
      const int64_t ba = ba_score(c, prof, p, n, row);
      sa.tt[si] = (int)tt;
      sa.na[si] = na;
      sa.fit[si] = (int)fit;
      sa.ba[si] = (int)ba;
      max_tt = tt > max_tt ? tt : max_tt;
      max_na = na > max_na ? na : max_na;
      int64_t ipa = 0;
      if (has_ipa) {
        ipa = ipa_score(c, P, p, pl, bins, n);
        ipa_min = ipa < ipa_min ? ipa : ipa_min;
        ipa_max = ipa > ipa_max ? ipa : ipa_max;
      }
      sa.ipa[si] = ipa;
      sa.pts[si] = 0;
      if (out) {
        out->raw[KSS_S_TAINT_TOLERATION * NN + n] = tt;
        out->raw[KSS_S_NODE_AFFINITY * NN + n] = na;
        out->raw[KSS_S_NODE_RESOURCES_FIT * NN + n] = fit;
        out->raw[KSS_S_VOLUME_BINDING * NN + n] = 0;
        out->raw[KSS_S_INTER_POD_AFFINITY * NN + n] = ipa;
        out->raw[KSS_S_BALANCED_ALLOCATION * NN + n] = ba;
        out->raw[KSS_S_IMAGE_LOCALITY * NN + n] = il;
      }
      if (has_soft) {
        if (req_all && !has_keys(c, soft, p.n_soft, n)) {
          nign++;
          ign = 1;
        } else {
#pragma unroll
          for (int i = 0; i < MAXS; i++) {
            if (i >= p.n_soft) break;
            int d = label_of(c, soft[i].key, n);
            if (pl.soft_mode[i] == SOFT_DIRECT) {
              if (d >= 0) sdirect[i]++;
              else smissing |= 1ll << i;
            } else if (pl.soft_mode[i] == SOFT_HIST) {
              if (d < 0) d = c.key_empty[soft[i].key];
              pres[pl.soft_poff[i] + d] = 1;
            }
          }
        }
      }
    }
    sa.fail[si] = f | (ign << 16) | (il << 24);  // verdict | PTS-ignored bit | ImageLocality raw
  }
  KSS_STAMP(S, 2);
  if (!has_soft && !has_ipa) {
    long long v[3] = {nf, max_tt, max_na};
    const int op[3] = {OP_SUM, OP_MAX, OP_MAX};
    if (!cluster_reduce(smem, S, v, op)) return false;
    nf = v[0];
    max_tt = v[1];
    max_na = v[2];
  } else {
    long long v[7 + MAXS] = {nf, nign, max_tt, max_na, ipa_min, ipa_max, smissing};
    const int op[7 + MAXS] = {OP_SUM, OP_SUM, OP_MAX, OP_MAX, OP_MIN, OP_MAX, OP_OR, OP_SUM, OP_SUM, OP_SUM, OP_SUM};
#pragma unroll
    for (int i = 0; i < MAXS; i++) v[7 + i] = sdirect[i];
    // soft presence bins (filled during the pass) are OR-ed across shards
    if (!cluster_reduce(smem, S, v, op, 0, 0, pl.total_bins + pl.hard_pbins, pl.total_pbins - pl.hard_pbins)) return false;
    nf = v[0];
    nign = v[1];
    max_tt = v[2];
    max_na = v[3];
    ipa_min = v[4];
    ipa_max = v[5];
    smissing = v[6];
#pragma unroll
    for (int i = 0; i < MAXS; i++) sdirect[i] = v[7 + i];
  }
  KSS_STAMP(S, 3);
  meta.n_feasible = (int)nf;
  if (nf == 0) {
    if (nom_failed && m_list > 0) {  // no window stop: only the nominated node's count is left
      long long v[1] = {nom_x};
      const int op[1] = {OP_SUM};
      if (!cluster_reduce(smem, S, v, op)) return false;
      S.cursor = (int)(((long long)S.cursor + v[0]) % m_list);
    }
    meta.status = 1;
    return true;
  }
  const bool scored = nf > 1;  // a single feasible node is selected without scoring

  // ---- PodTopologySpread PreScore sizes + Score ---------------------------
  long long pts_min = 0, pts_max = 0;
  if (scored && has_soft) {
    double w[MAXS];
    long long sz[MAXS];
    const int op[MAXS] = {OP_SUM, OP_SUM, OP_SUM, OP_SUM};
#pragma unroll
    for (int i = 0; i < MAXS; i++) sz[i] = 0;
#pragma unroll
    for (int i = 0; i < MAXS; i++) {
      if (i >= p.n_soft) break;
      if (pl.soft_mode[i] != SOFT_HIST || pl.soft_own[i] != i) continue;
      const int nb = c.key_card[soft[i].key] + 1;
      for (int b = tid; b < nb; b += nt) sz[i] += pres[pl.soft_poff[i] + b] ? 1 : 0;
    }
    cluster_reduce(smem, S, sz, op, 0, 0, 0, 0, /*local=*/true);
#pragma unroll
    for (int i = 0; i < MAXS; i++) {
      if (i >= p.n_soft) break;
      long long size;  // topoSize: a group's domains count for its leader only
      if (pl.soft_mode[i] == SOFT_HOST) size = nf - nign;
      else if (pl.soft_own[i] != i) size = 0;
      else if (pl.soft_mode[i] == SOFT_DIRECT) size = sdirect[i] + ((smissing >> i) & 1);
      else size = sz[i];
      KSS_DCHECK(size >= 0 && size <= c.N + 2, "log_table size", size, c.N);
      w[i] = c.log_table[size];  // topologyNormalizingWeight = math.Log(float64(size+2))
    }
    pts_min = INT64_MAX;
    for (int k = 0; k < npt; k++) {
      const int n = S.lo + k * nt + tid;
      const int si = k * nt + tid;
      const int fi = sa.fail[si];
      if ((fi & 0xFFFF) != KSS_F_PASS) continue;
      int64_t raw = 0;
      if (!((fi >> 16) & 1)) {
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < MAXS; i++) {
          if (i >= p.n_soft) break;
          const int d = label_of(c, soft[i].key, n);
          if (d < 0) continue;
          int64_t cnt = 0;
          if (pl.soft_mode[i] == SOFT_HOST) {
            cnt = spread_count(c, P, soft[i], n);
          } else if (pl.soft_mode[i] == SOFT_DIRECT) {  // the node's pair counter: every admitting member
            for (int j = 0; j < p.n_soft; j++)
              if (pl.soft_own[j] == pl.soft_own[i] && spread_policy_ok(c, P, p, soft[j], n))
                cnt += spread_count(c, P, soft[j], n);
          } else {
            cnt = bins[pl.soft_off[i] + d];
          }
          const double a = (double)cnt * w[i];
          s = s + (a + (double)(soft[i].max_skew - 1));  // scoreForCount
        }
        raw = (int64_t)round(s);
        pts_min = raw < pts_min ? raw : pts_min;
        pts_max = raw > pts_max ? raw : pts_max;
      }
      sa.pts[si] = raw;
      if (out) out->raw[KSS_S_POD_TOPOLOGY_SPREAD * NN + n] = raw;
    }
    long long v[2] = {pts_min, pts_max};
    const int op2[2] = {OP_MIN, OP_MAX};
    if (!cluster_reduce(smem, S, v, op2)) return false;
    pts_min = v[0];
    pts_max = v[1];
  } else if (out) {
    for (int k = 0; k < npt; k++) {
      const int n = S.lo + k * nt + tid;
      if ((sa.fail[k * nt + tid] & 0xFFFF) == KSS_F_PASS) out->raw[KSS_S_POD_TOPOLOGY_SPREAD * NN + n] = 0;
    }
  }

  // ---- NormalizeScore + weights + selectHost --------------------------------
  const bool ipa_norm = GEN && (flags & 8) != 0;
  const int64_t ipa_diff = ipa_max - ipa_min;
  const bool rec = out && keep_norm && scored;
  long long best = 0;
  for (int k = 0; k < npt; k++) {
    const int n = S.lo + k * nt + tid;
    const int si = k * nt + tid;
    const int fi = sa.fail[si];
    if (out && out->canon && keep_norm && n < S.hi && ((fi & 0xFFFF) != KSS_F_PASS || !scored)) {
#pragma unroll
      for (int x = 0; x < KSS_NSCORE; x++) out->norm[(size_t)x * NN + n] = 0;
      out->total[n] = 0;
    }
    if ((fi & 0xFFFF) != KSS_F_PASS) continue;
    int64_t total = 0;
    if (scored) {
      int64_t nm[KSS_NSCORE];
      nm[KSS_S_TAINT_TOLERATION] = sa.tt[si];
      nm[KSS_S_NODE_AFFINITY] = sa.na[si];
      nm[KSS_S_NODE_RESOURCES_FIT] = sa.fit[si];
      nm[KSS_S_VOLUME_BINDING] = 0;
      nm[KSS_S_POD_TOPOLOGY_SPREAD] = sa.pts[si];
      nm[KSS_S_INTER_POD_AFFINITY] = sa.ipa[si];
      nm[KSS_S_BALANCED_ALLOCATION] = sa.ba[si];
      nm[KSS_S_IMAGE_LOCALITY] = fi >> 24;  // no NormalizeScore
      // TaintToleration: DefaultNormalizeScore(100, reverse=true)
      if (max_tt == 0) nm[KSS_S_TAINT_TOLERATION] = 100;
      else nm[KSS_S_TAINT_TOLERATION] = 100 - div_i64(100 * nm[KSS_S_TAINT_TOLERATION], max_tt);
      // NodeAffinity: DefaultNormalizeScore(100, reverse=false)
      if (max_na != 0) nm[KSS_S_NODE_AFFINITY] = div_i64(100 * nm[KSS_S_NODE_AFFINITY], max_na);
      // PodTopologySpread.NormalizeScore
      {
        int64_t& v = nm[KSS_S_POD_TOPOLOGY_SPREAD];
        if (has_soft && ((fi >> 16) & 1)) v = 0;
        else if (pts_max == 0) v = 100;
        else v = div_i64(100 * (pts_max + pts_min - v), pts_max);
      }
      // InterPodAffinity.NormalizeScore (skipped when topologyScore is empty)
      if (ipa_norm) {
        double f = 0.0;
        if (ipa_diff > 0) f = 100.0 * ((double)(nm[KSS_S_INTER_POD_AFFINITY] - ipa_min) / (double)ipa_diff);
        nm[KSS_S_INTER_POD_AFFINITY] = (int64_t)f;
      }
#pragma unroll
      for (int s = 0; s < KSS_NSCORE; s++)
        if ((prof.score_enabled >> s) & 1u) total += nm[s] * (int64_t)prof.weight[s];
      if (rec) {
#pragma unroll
        for (int s = 0; s < KSS_NSCORE; s++) out->norm[(size_t)s * NN + n] = nm[s];
        out->total[n] = total;
      }
    }
    const uint32_t g = (uint32_t)(c.node_base + n);
    // totals are >= 0 and < 2^31, so the packed key's sign bit is clear and signed max == unsigned max
    const long long key = (long long)(((unsigned long long)(uint32_t)total << 32) | (0xFFFFFFFFull - g));
    best = key > best ? key : best;
  }
  KSS_STAMP(S, 4);
  if ((win && w_total > k_find) || (nom_failed && m_list > 0)) {  // with the processed count still to add
    long long v[2] = {best, w_proc + nom_x};
    const int op[2] = {OP_MAX, OP_SUM};
    if (!cluster_reduce(smem, S, v, op)) return false;
    best = v[0];
    S.cursor = (int)(((long long)S.cursor + v[1]) % m_list);
  } else {
    long long v[1] = {best};
    const int op[1] = {OP_MAX};
    if (!cluster_reduce(smem, S, v, op)) return false;
    best = v[0];
  }
  KSS_STAMP(S, 5);
  const unsigned long long ub = (unsigned long long)best;
  meta.chosen = (int)(0xFFFFFFFFull - (ub & 0xFFFFFFFFull));
  meta.scored = scored ? 1 : 0;
  meta.best_total = scored ? (int64_t)(ub >> 32) : 0;
  return true;
}

// Cache.AssumePod -> NodeInfo.AddPod; executed by one lane.  With a shard cache the
// hot columns are updated in LDS (written back to HBM when the launch ends).
__device__ __forceinline__ void commit_pod(const DevCluster& c, const DevPods& P, const kss_pod& p, int local, int sign) {
  const size_t N = (size_t)c.N;
  KSS_DCHECK(local >= 0 && local < c.N && p.cls < c.class_cap, "commit local/cls", local, p.cls);
  if (c.nc64) {
    const int i = local - c.nc_lo, C = c.nc_cap;
#pragma unroll
    for (int r = 0; r < 3; r++) c.nc64[(3 + r) * C + i] += sign * p.commit_req[r];
    c.nc64[6 * C + i] += sign * p.commit_nz[0];
    c.nc64[7 * C + i] += sign * p.commit_nz[1];
    c.nc32[i] += sign;
    for (int r = 3; r < KSS_NRES; r++) c.requested[(size_t)r * N + local] += sign * p.commit_req[r];
  } else {
    for (int r = 0; r < KSS_NRES; r++) c.requested[(size_t)r * N + local] += sign * p.commit_req[r];
    c.nonzero[local] += sign * p.commit_nz[0];
    c.nonzero[N + local] += sign * p.commit_nz[1];
    c.pod_count[local] += sign;
  }
  if (p.cls >= 0) c.class_count[(size_t)p.cls * N + local] += sign;
  for (int i = 0; i < p.own_terms_len; i++) c.term_count[(size_t)P.ints[p.own_terms_off + i] * N + local] += sign;
  // NodeInfo.AddPod / RemovePod updateUsedPorts (a set: removal clears the entries)
  if (p.port_add) c.port_used[local] = sign > 0 ? (c.port_used[local] | p.port_add) : (c.port_used[local] & ~p.port_add);
  // the pod's volumes (NodeInfo.Pods' volumes, re-read by the volume filters upstream)
  for (int e = 0; e < p.vol_len; e++) {
    const kss_vol& v = P.vols[p.vol_off + e];
    if (v.kind == KSS_VOL_OWN) vol_commit_row(c, v.row, local, sign);
    else if (v.kind == KSS_VOL_OWN_PRIVATE) c.vol_attached[(size_t)v.key * N + local] += sign * v.count;
  }
}

// Shard cache fill / write-back (all lanes of the workgroup).
__device__ __forceinline__ void cache_fill(const DevCluster& c, int hi, int n_keys_cached) {
  const size_t N = (size_t)c.N;
  const int C = c.nc_cap;
  for (int n = c.nc_lo + threadIdx.x; n < hi; n += blockDim.x) {
    const int i = n - c.nc_lo;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      c.nc64[k * C + i] = c.alloc[k * N + n];
      c.nc64[(3 + k) * C + i] = c.requested[k * N + n];
    }
    c.nc64[6 * C + i] = c.nonzero[n];
    c.nc64[7 * C + i] = c.nonzero[N + n];
    c.nct[i] = c.taint_hard[n];
    c.nct[C + i] = c.taint_soft[n];
    c.nc32[i] = c.pod_count[n];
    c.nc32[C + i] = c.allowed_pods[n];
    c.nc32[2 * C + i] = (int32_t)c.node_flags[n];
    for (int k = 0; k < n_keys_cached; k++) c.ncl[k * C + i] = c.label_value[(size_t)k * N + n];
  }
}

__device__ __forceinline__ void cache_writeback(const DevCluster& c, int hi) {
  const size_t N = (size_t)c.N;
  const int C = c.nc_cap;
  for (int n = c.nc_lo + threadIdx.x; n < hi; n += blockDim.x) {
    const int i = n - c.nc_lo;
#pragma unroll
    for (int k = 0; k < 3; k++) c.requested[k * N + n] = c.nc64[(3 + k) * C + i];
    c.nonzero[n] = c.nc64[6 * C + i];
    c.nonzero[N + n] = c.nc64[7 * C + i];
    c.pod_count[n] = c.nc32[i];
  }
}

}  // namespace kss
