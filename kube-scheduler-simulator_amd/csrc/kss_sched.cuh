// kss_sched.cuh — the scheduling cycle for one pod over all nodes of one cluster,
// executed by ONE workgroup (all reductions are workgroup-level: LDS + s_barrier,
// no inter-workgroup communication, so no spin can hang the device).
//
// Per pod (schedulePod):
//   stats   PreFilter of PodTopologySpread (calPreFilterState) and InterPodAffinity
//           (existing / incoming (anti-)affinity counts) and InterPodAffinity PreScore
//           topologyScore: LDS-privatised histograms over topology domains for
//           non-unique keys; unique keys (hostname) are evaluated in place.
//   filter  findNodesThatPassFilters (first failing plugin wins) + raw Score of every
//           plugin on feasible nodes; reductions: #feasible, max TT/NA, IPA min/max,
//           PTS ignored / domain presence.
//   pts     PodTopologySpread Score (needs the feasible-domain count) + min/max.
//   select  NormalizeScore, weights, TotalScore, selectHost (max total, lowest index).
//   commit  Cache.AssumePod -> NodeInfo.AddPod on the chosen row.
#pragma once
#include "kss_eval.cuh"

namespace kss {

constexpr int MAXH = 4;  // hard spread constraints per pod on the device path
constexpr int MAXS = 4;  // soft spread constraints
constexpr int MAXK = 4;  // distinct inter-pod-affinity topology keys
constexpr int LDS_BINS = 4096;  // int64 histogram bins per workgroup
constexpr int MAXWAVES = 16;
constexpr int NRED = 16;  // values per block reduction

enum { SOFT_HOST = 0, SOFT_DIRECT = 1, SOFT_HIST = 2 };

// Per-pod plan, identical in every lane (computed from wave-uniform pod data).
struct Plan {
  int n_hard, n_soft, n_keys;
  int hard_off[MAXH];  // bin offset, -1 = unique key (direct)
  int hard_poff[MAXH]; // presence offset of the pair (key, domain)
  int soft_mode[MAXS];
  int soft_off[MAXS];  // count bins
  int soft_poff[MAXS]; // presence bins
  int key[MAXK];
  int key_off[MAXK];   // 4 consecutive histograms (x, a, b, s), -1 = unique (direct)
  int key_bins[MAXK];
  int total_bins;
  int total_pbins;
  bool need_stats;
};

struct Shared {
  long long bins[LDS_BINS];
  unsigned int pres[LDS_BINS];
  long long red[MAXWAVES][NRED];
};

// Output slot for one pod: per-node verdicts and scores (also the record format).
struct Slot {
  uint8_t* fail;
  uint16_t* detail;
  int64_t* raw;   // [KSS_NSCORE][N]
  int64_t* norm;  // [KSS_NSCORE][N]  (nullptr: not kept)
  int64_t* total; // [N]              (nullptr: not kept)
};

struct PodMeta {
  int32_t chosen, n_feasible, scored, status;
  int64_t best_total;
};

__device__ __forceinline__ long long wave_reduce(long long v, int op) {
  // op: 0 sum, 1 max, 2 min, 3 or
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    long long o = __shfl_xor(v, m, 64);
    if (op == 0) v += o;
    else if (op == 1) v = o > v ? o : v;
    else if (op == 2) v = o < v ? o : v;
    else v |= o;
  }
  return v;
}

// Reduce up to NRED values across the workgroup; every lane gets the results.
template <int K>
__device__ __forceinline__ void block_reduce(Shared& sh, long long (&v)[K], const int (&op)[K]) {
  static_assert(K <= NRED, "too many values");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < K; k++) {
    long long r = wave_reduce(v[k], op[k]);
    if (lane == 0) sh.red[wave][k] = r;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; k++) {
    long long r = sh.red[0][k];
    for (int w = 1; w < nw; w++) {
      long long o = sh.red[w][k];
      if (op[k] == 0) r += o;
      else if (op[k] == 1) r = o > r ? o : r;
      else if (op[k] == 2) r = o < r ? o : r;
      else r |= o;
    }
    v[k] = r;
  }
  __syncthreads();
}

__device__ __forceinline__ bool key_unique(const DevCluster& c, int key) {
  return (c.key_flags[key] & KSS_KEY_UNIQUE) != 0;
}

// Returns false if the pod needs more LDS bins / slots than the device path has.
__device__ __forceinline__ bool make_plan(const DevCluster& c, const DevPods& P, const kss_pod& p, Plan& pl) {
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
    if (key_unique(c, key)) {
      pl.hard_off[i] = -1;
      pl.hard_poff[i] = -1;
    } else {
      pl.hard_off[i] = off;
      pl.hard_poff[i] = poff;
      off += c.key_card[key] + 1;
      poff += c.key_card[key] + 1;
    }
  }
  for (int i = 0; i < p.n_soft; i++) {
    const int key = sp[p.n_hard + i].key;
    if (c.key_flags[key] & KSS_KEY_HOSTNAME) {
      pl.soft_mode[i] = SOFT_HOST;
    } else if (key_unique(c, key)) {
      pl.soft_mode[i] = SOFT_DIRECT;
    } else {
      pl.soft_mode[i] = SOFT_HIST;
      pl.soft_off[i] = off;
      pl.soft_poff[i] = poff;
      off += c.key_card[key] + 1;
      poff += c.key_card[key] + 1;
      pl.need_stats = true;
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
  return off <= LDS_BINS && poff <= LDS_BINS;
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
  if ((s.flags & KSS_SPREAD_POLICY_TAINTS_HONOR) && first_untolerated(c, p, n) >= 0) return false;
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
// stats pass for node n: accumulate LDS histograms and per-lane partials
//   part[0..MAXH) : min count over eligible nodes for unique hard keys
//   flags bit0 ex, bit1 aff, bit2 anti, bit3 score nonempty
// ---------------------------------------------------------------------------
__device__ __forceinline__ void stats_node(const DevCluster& c, const DevPods& P, const kss_pod& p, const Plan& pl,
                                           Shared& sh, int n, long long* hard_min, long long& flags) {
  const kss_spread* sp = P.spreads + p.spread_off;
  if (p.n_hard > 0 && has_keys(c, sp, p.n_hard, n)) {  // nodeLabelsMatchSpreadConstraints
    for (int i = 0; i < p.n_hard; i++) {
      if (!spread_policy_ok(c, P, p, sp[i], n)) continue;
      const int64_t cnt = spread_count(c, P, sp[i], n);
      if (pl.hard_off[i] < 0) {
        hard_min[i] = cnt < hard_min[i] ? cnt : hard_min[i];
      } else {
        const int d = label_of(c, sp[i].key, n);
        atomicAdd((unsigned long long*)&sh.bins[pl.hard_off[i] + d], (unsigned long long)cnt);
        sh.pres[pl.hard_poff[i] + d] = 1u;  // the pair (key, value) exists
      }
    }
  }
  if (p.n_soft > 0) {
    const kss_spread* so = sp + p.n_hard;
    const bool req_all = (p.flags & KSS_POD_PTS_REQUIRE_ALL) != 0;
    if (!req_all || has_keys(c, so, p.n_soft, n)) {
      for (int i = 0; i < p.n_soft; i++) {
        if (pl.soft_mode[i] != SOFT_HIST) continue;
        if (!spread_policy_ok(c, P, p, so[i], n)) continue;
        int d = label_of(c, so[i].key, n);
        if (d < 0) d = c.key_empty[so[i].key];
        const int64_t cnt = spread_count(c, P, so[i], n);
        if (cnt) atomicAdd((unsigned long long*)&sh.bins[pl.soft_off[i] + d], (unsigned long long)cnt);
      }
    }
  }
  if (p.ipa_len > 0) {
    const kss_ipa* ip = P.ipa + p.ipa_off;
    const bool has_labels = (c.node_flags[n] & KSS_NODE_HAS_LABELS) != 0;
    const size_t N = (size_t)c.N;
    for (int e = 0; e < p.ipa_len; e++) {
      const kss_ipa& en = ip[e];
      const int d = label_of(c, en.key, n);
      if (d < 0) continue;
      const int k = slot_of(pl, en.key);
      const int base = pl.key_off[k];
      const int nb = pl.key_bins[k];
      if (en.kind == KSS_IPA_SCORE_CLASS || en.kind == KSS_IPA_SCORE_TERM) {
        if (!has_labels) continue;
        const int32_t* mat = en.kind == KSS_IPA_SCORE_CLASS ? c.class_count : c.term_count;
        const int64_t v = sum_rows(mat, N, P.ints + en.row_off, en.row_len, n);
        if (v > 0) flags |= 8;
        if (base >= 0 && v) atomicAdd((unsigned long long*)&sh.bins[base + 3 * nb + d], (unsigned long long)(v * en.coef));
      } else {
        const int32_t* mat = en.kind == KSS_IPA_EXISTING_ANTI ? c.term_count : c.class_count;
        const int64_t v = sum_rows(mat, N, P.ints + en.row_off, en.row_len, n);
        const int h = en.kind == KSS_IPA_EXISTING_ANTI ? 0 : (en.kind == KSS_IPA_REQ_AFFINITY ? 1 : 2);
        if (v > 0) flags |= (1ll << h);
        if (base >= 0 && v) atomicAdd((unsigned long long*)&sh.bins[base + h * nb + d], (unsigned long long)v);
      }
    }
  }
}

// value of an IPA histogram h (0 x, 1 a, 2 b) at node n's domain for key slot k
__device__ __forceinline__ int64_t ipa_value(const DevCluster& c, const DevPods& P, const kss_pod& p, const Plan& pl,
                                             const Shared& sh, int k, int h, int d, int n) {
  if (pl.key_off[k] >= 0) return sh.bins[pl.key_off[k] + h * pl.key_bins[k] + d];
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

// PodTopologySpread.Filter (hard constraints) — returns detail+1 on failure, 0 on pass
__device__ __forceinline__ int filter_pts(const DevCluster& c, const DevPods& P, const kss_pod& p, const Plan& pl,
                                          const Shared& sh, const long long* hard_min, int n) {
  const kss_spread* sp = P.spreads + p.spread_off;
  for (int i = 0; i < p.n_hard; i++) {
    const int d = label_of(c, sp[i].key, n);
    if (d < 0) return 1 + KSS_PTS_MISSING_LABEL;
    int64_t match;
    if (pl.hard_off[i] >= 0) {
      match = sh.bins[pl.hard_off[i] + d];
    } else {
      match = (has_keys(c, sp, p.n_hard, n) && spread_policy_ok(c, P, p, sp[i], n)) ? spread_count(c, P, sp[i], n) : 0;
    }
    const int64_t skew = match + (int64_t)sp[i].self_match - hard_min[i];
    if (skew > (int64_t)sp[i].max_skew) return 1 + KSS_PTS_CONSTRAINTS_NOT_MATCH;
  }
  return 0;
}

// InterPodAffinity.Filter — returns detail+1 on failure, 0 on pass.  flags: bit0 ex, bit1 aff, bit2 anti
__device__ __forceinline__ int filter_ipa(const DevCluster& c, const DevPods& P, const kss_pod& p, const Plan& pl,
                                          const Shared& sh, long long flags, int n) {
  const kss_ipa* ip = P.ipa + p.ipa_off;
  // satisfyPodAffinity
  bool have = false, exist = true;
  for (int e = 0; e < p.ipa_len; e++) {
    if (ip[e].kind != KSS_IPA_REQ_AFFINITY) continue;
    have = true;
    const int d = label_of(c, ip[e].key, n);
    if (d < 0) return 1 + KSS_IPA_AFFINITY;
    const int k = slot_of(pl, ip[e].key);
    if (ipa_value(c, P, p, pl, sh, k, 1, d, n) <= 0) exist = false;
  }
  if (have && !exist && !(!(flags & 2) && (p.flags & KSS_POD_IPA_SELF_MATCH))) return 1 + KSS_IPA_AFFINITY;
  // satisfyPodAntiAffinity
  if (flags & 4) {
    for (int e = 0; e < p.ipa_len; e++) {
      if (ip[e].kind != KSS_IPA_REQ_ANTI) continue;
      const int d = label_of(c, ip[e].key, n);
      if (d < 0) continue;
      const int k = slot_of(pl, ip[e].key);
      if (ipa_value(c, P, p, pl, sh, k, 2, d, n) > 0) return 1 + KSS_IPA_ANTI_AFFINITY;
    }
  }
  // satisfyExistingPodsAntiAffinity
  if (flags & 1) {
    for (int e = 0; e < p.ipa_len; e++) {
      if (ip[e].kind != KSS_IPA_EXISTING_ANTI) continue;
      const int d = label_of(c, ip[e].key, n);
      if (d < 0) continue;
      const int k = slot_of(pl, ip[e].key);
      if (ipa_value(c, P, p, pl, sh, k, 0, d, n) > 0) return 1 + KSS_IPA_EXISTING_ANTI_AFFINITY;
    }
  }
  return 0;
}

// InterPodAffinity.Score: Σ topologyScore[key][node value] over keys the node has
__device__ __forceinline__ int64_t ipa_score(const DevCluster& c, const DevPods& P, const kss_pod& p, const Plan& pl,
                                             const Shared& sh, int n) {
  int64_t s = 0;
  const bool has_labels = (c.node_flags[n] & KSS_NODE_HAS_LABELS) != 0;
  for (int k = 0; k < pl.n_keys; k++) {
    const int d = label_of(c, pl.key[k], n);
    if (d < 0) continue;
    if (pl.key_off[k] >= 0) {
      s += sh.bins[pl.key_off[k] + 3 * pl.key_bins[k] + d];
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

// ---------------------------------------------------------------------------
// one scheduling cycle for pod p, executed by the whole workgroup
// ---------------------------------------------------------------------------
__device__ void schedule_pod(const DevCluster& c, const DevPods& P, const kss_profile& prof, int pi, Shared& sh,
                             const Slot& out, PodMeta& meta, bool keep_norm) {
  const kss_pod& p = P.pods[pi];
  const int N = c.N;
  const int tid = threadIdx.x, nt = blockDim.x;
  const size_t NN = (size_t)N;
  meta.chosen = -1;
  meta.n_feasible = 0;
  meta.scored = 0;
  meta.status = 0;
  meta.best_total = 0;

  Plan pl;
  const bool plan_ok = make_plan(c, P, p, pl);
  if (p.prefilter_status != 0 || !plan_ok) {
    for (int n = tid; n < N; n += nt) {
      out.fail[n] = KSS_F_NOT_EVALUATED;
      out.detail[n] = 0;
    }
    meta.status = !plan_ok ? 4 : (p.prefilter_status == 1 ? 2 : 3);
    __syncthreads();
    return;
  }

  // ---- stats -----------------------------------------------------------
  long long hard_min[MAXH];
  long long flags = 0;
#pragma unroll
  for (int i = 0; i < MAXH; i++) hard_min[i] = INT32_MAX;
  if (pl.need_stats) {
    for (int b = tid; b < pl.total_bins; b += nt) sh.bins[b] = 0;
    for (int b = tid; b < pl.total_pbins; b += nt) sh.pres[b] = 0;
    __syncthreads();
    for (int n = tid; n < N; n += nt) stats_node(c, P, p, pl, sh, n, hard_min, flags);
    __syncthreads();
    // minima over present bins of non-unique hard keys
    const kss_spread* sp = P.spreads + p.spread_off;
    for (int i = 0; i < p.n_hard; i++) {
      if (pl.hard_off[i] < 0) continue;
      const int nb = c.key_card[sp[i].key] + 1;
      for (int b = tid; b < nb; b += nt) {
        const int g = pl.hard_off[i] + b;
        if (sh.pres[pl.hard_poff[i] + b]) hard_min[i] = sh.bins[g] < hard_min[i] ? sh.bins[g] : hard_min[i];
      }
    }
    long long v[MAXH + 1];
    int op[MAXH + 1];
#pragma unroll
    for (int i = 0; i < MAXH; i++) {
      v[i] = hard_min[i];
      op[i] = 2;
    }
    v[MAXH] = flags;
    op[MAXH] = 3;
    block_reduce(sh, v, op);
#pragma unroll
    for (int i = 0; i < MAXH; i++) hard_min[i] = v[i];
    flags = v[MAXH];
  }

  // ---- filter + raw scores ---------------------------------------------
  const uint32_t en = prof.filter_enabled;
  const bool restrict_names = p.names_len >= 0;
  const kss_spread* soft = P.spreads + p.spread_off + p.n_hard;
  const bool req_all = (p.flags & KSS_POD_PTS_REQUIRE_ALL) != 0;
  long long nf = 0, nign = 0, max_tt = 0, max_na = 0, ipa_min = INT64_MAX, ipa_max = INT64_MIN, first = INT64_MAX;
  long long sdirect[MAXS], smissing = 0;
#pragma unroll
  for (int i = 0; i < MAXS; i++) sdirect[i] = 0;
  for (int n = tid; n < N; n += nt) {
    uint16_t detail = 0;
    int fail;
    if (restrict_names && !in_names(P, p, (int64_t)c.node_base + n)) {
      fail = KSS_F_NOT_EVALUATED;
    } else {
      fail = filter_local(c, P, p, en, n, &detail);
      if (!fail && ((en >> KSS_F_POD_TOPOLOGY_SPREAD) & 1u) && p.n_hard > 0) {
        const int r = filter_pts(c, P, p, pl, sh, hard_min, n);
        if (r) {
          fail = KSS_F_POD_TOPOLOGY_SPREAD;
          detail = (uint16_t)(r - 1);
        }
      }
      if (!fail && ((en >> KSS_F_INTER_POD_AFFINITY) & 1u) && p.ipa_len > 0) {
        const int r = filter_ipa(c, P, p, pl, sh, flags, n);
        if (r) {
          fail = KSS_F_INTER_POD_AFFINITY;
          detail = (uint16_t)(r - 1);
        }
      }
    }
    out.fail[n] = (uint8_t)fail;
    out.detail[n] = detail;
    if (fail == KSS_F_PASS) {
      nf++;
      first = n < first ? n : first;
      const int64_t tt = tt_score(c, p, n);
      const int64_t na = na_score(c, P, p, n);
      const int64_t ipa = p.ipa_len > 0 ? ipa_score(c, P, p, pl, sh, n) : 0;
      out.raw[KSS_S_TAINT_TOLERATION * NN + n] = tt;
      out.raw[KSS_S_NODE_AFFINITY * NN + n] = na;
      out.raw[KSS_S_NODE_RESOURCES_FIT * NN + n] = fit_score(c, prof, p, n);
      out.raw[KSS_S_VOLUME_BINDING * NN + n] = 0;
      out.raw[KSS_S_INTER_POD_AFFINITY * NN + n] = ipa;
      out.raw[KSS_S_BALANCED_ALLOCATION * NN + n] = ba_score(c, prof, p, n);
      out.raw[KSS_S_IMAGE_LOCALITY * NN + n] = 0;
      max_tt = tt > max_tt ? tt : max_tt;
      max_na = na > max_na ? na : max_na;
      ipa_min = ipa < ipa_min ? ipa : ipa_min;
      ipa_max = ipa > ipa_max ? ipa : ipa_max;
      if (p.n_soft > 0) {
        const bool ignored = req_all && !has_keys(c, soft, p.n_soft, n);
        if (ignored) {
          nign++;
        } else {
          for (int i = 0; i < p.n_soft; i++) {
            int d = label_of(c, soft[i].key, n);
            if (pl.soft_mode[i] == SOFT_DIRECT) {
              if (d >= 0) sdirect[i]++;
              else smissing |= 1ll << i;
            } else if (pl.soft_mode[i] == SOFT_HIST) {
              if (d < 0) d = c.key_empty[soft[i].key];
              sh.pres[pl.soft_poff[i] + d] = 1;
            }
          }
        }
      }
    }
  }
  {
    long long v[8 + MAXS] = {nf, nign, max_tt, max_na, ipa_min, ipa_max, first, smissing};
    int op[8 + MAXS] = {0, 0, 1, 1, 2, 1, 2, 3};
#pragma unroll
    for (int i = 0; i < MAXS; i++) {
      v[8 + i] = sdirect[i];
      op[8 + i] = 0;
    }
    block_reduce(sh, v, op);
    nf = v[0];
    nign = v[1];
    max_tt = v[2];
    max_na = v[3];
    ipa_min = v[4];
    ipa_max = v[5];
    first = v[6];
    smissing = v[7];
#pragma unroll
    for (int i = 0; i < MAXS; i++) sdirect[i] = v[8 + i];
  }
  meta.n_feasible = (int)nf;
  if (nf == 0) {
    meta.status = 1;
    return;
  }
  if (nf == 1) {
    meta.chosen = (int)(c.node_base + first);
    return;
  }
  meta.scored = 1;

  // ---- PodTopologySpread PreScore sizes + Score ---------------------------
  double w[MAXS];
  long long pts_min = INT64_MAX, pts_max = 0;
  if (p.n_soft > 0) {
    long long sz[MAXS];
    int op[MAXS];
#pragma unroll
    for (int i = 0; i < MAXS; i++) {
      sz[i] = 0;
      op[i] = 0;
    }
    for (int i = 0; i < p.n_soft; i++) {
      if (pl.soft_mode[i] != SOFT_HIST) continue;
      const int nb = c.key_card[soft[i].key] + 1;
      for (int b = tid; b < nb; b += nt) sz[i] += sh.pres[pl.soft_poff[i] + b] ? 1 : 0;
    }
    block_reduce(sh, sz, op);
    for (int i = 0; i < p.n_soft; i++) {
      long long size;
      if (pl.soft_mode[i] == SOFT_HOST) size = nf - nign;
      else if (pl.soft_mode[i] == SOFT_DIRECT) size = sdirect[i] + ((smissing >> i) & 1);
      else size = sz[i];
      w[i] = c.log_table[size];  // topologyNormalizingWeight = math.Log(float64(size+2))
    }
    for (int n = tid; n < N; n += nt) {
      if (out.fail[n] != KSS_F_PASS) continue;
      int64_t raw = 0;
      const bool ignored = req_all && !has_keys(c, soft, p.n_soft, n);
      if (!ignored) {
        double s = 0.0;
        for (int i = 0; i < p.n_soft; i++) {
          const int d = label_of(c, soft[i].key, n);
          if (d < 0) continue;
          int64_t cnt;
          if (pl.soft_mode[i] == SOFT_HOST) cnt = spread_count(c, P, soft[i], n);
          else if (pl.soft_mode[i] == SOFT_DIRECT) cnt = spread_policy_ok(c, P, p, soft[i], n) ? spread_count(c, P, soft[i], n) : 0;
          else cnt = sh.bins[pl.soft_off[i] + d];
          const double a = (double)cnt * w[i];
          s = s + (a + (double)(soft[i].max_skew - 1));  // scoreForCount
        }
        raw = (int64_t)round(s);
        pts_min = raw < pts_min ? raw : pts_min;
        pts_max = raw > pts_max ? raw : pts_max;
      } else {
        raw = 0;
      }
      out.raw[KSS_S_POD_TOPOLOGY_SPREAD * NN + n] = raw;
    }
    long long v[2] = {pts_min, pts_max};
    int op2[2] = {2, 1};
    block_reduce(sh, v, op2);
    pts_min = v[0];
    pts_max = v[1];
  } else {
    for (int n = tid; n < N; n += nt)
      if (out.fail[n] == KSS_F_PASS) out.raw[KSS_S_POD_TOPOLOGY_SPREAD * NN + n] = 0;
    pts_min = 0;
    pts_max = 0;
  }

  // ---- NormalizeScore + weights + selectHost --------------------------------
  const bool ipa_norm = (flags & 8) != 0;
  const int64_t ipa_diff = ipa_max - ipa_min;
  unsigned long long best = 0;
  for (int n = tid; n < N; n += nt) {
    if (out.fail[n] != KSS_F_PASS) continue;
    int64_t nm[KSS_NSCORE];
#pragma unroll
    for (int s = 0; s < KSS_NSCORE; s++) nm[s] = out.raw[(size_t)s * NN + n];
    // TaintToleration: DefaultNormalizeScore(100, reverse=true)
    if (max_tt == 0) nm[KSS_S_TAINT_TOLERATION] = 100;
    else nm[KSS_S_TAINT_TOLERATION] = 100 - (100 * nm[KSS_S_TAINT_TOLERATION]) / max_tt;
    // NodeAffinity: DefaultNormalizeScore(100, reverse=false)
    if (max_na != 0) nm[KSS_S_NODE_AFFINITY] = (100 * nm[KSS_S_NODE_AFFINITY]) / max_na;
    // PodTopologySpread.NormalizeScore
    {
      const bool ignored = p.n_soft > 0 && req_all && !has_keys(c, soft, p.n_soft, n);
      int64_t& v = nm[KSS_S_POD_TOPOLOGY_SPREAD];
      if (ignored) v = 0;
      else if (pts_max == 0) v = 100;
      else v = 100 * (pts_max + pts_min - v) / pts_max;
    }
    // InterPodAffinity.NormalizeScore (skipped when topologyScore is empty)
    if (ipa_norm) {
      double f = 0.0;
      if (ipa_diff > 0) f = 100.0 * ((double)(nm[KSS_S_INTER_POD_AFFINITY] - ipa_min) / (double)ipa_diff);
      nm[KSS_S_INTER_POD_AFFINITY] = (int64_t)f;
    }
    int64_t total = 0;
#pragma unroll
    for (int s = 0; s < KSS_NSCORE; s++)
      if ((prof.score_enabled >> s) & 1u) total += nm[s] * (int64_t)prof.weight[s];
    if (keep_norm) {
#pragma unroll
      for (int s = 0; s < KSS_NSCORE; s++) out.norm[(size_t)s * NN + n] = nm[s];
      out.total[n] = total;
    }
    const uint32_t g = (uint32_t)(c.node_base + n);
    const unsigned long long key = ((unsigned long long)(uint32_t)total << 32) | (0xFFFFFFFFull - g);
    best = key > best ? key : best;
  }
  {
    long long v[1] = {(long long)best};
    int op[1] = {1};
    // totals are >= 0 and < 2^31, so the packed key's sign bit is clear and signed max == unsigned max
    block_reduce(sh, v, op);
    best = (unsigned long long)v[0];
  }
  meta.chosen = (int)(0xFFFFFFFFull - (best & 0xFFFFFFFFull));
  meta.best_total = (int64_t)(best >> 32);
}

// Cache.AssumePod -> NodeInfo.AddPod; executed by one lane.
__device__ __forceinline__ void commit_pod(const DevCluster& c, const DevPods& P, const kss_pod& p, int local, int sign) {
  const size_t N = (size_t)c.N;
  for (int r = 0; r < KSS_NRES; r++) c.requested[(size_t)r * N + local] += sign * p.commit_req[r];
  c.nonzero[local] += sign * p.commit_nz[0];
  c.nonzero[N + local] += sign * p.commit_nz[1];
  c.pod_count[local] += sign;
  if (p.cls >= 0) c.class_count[(size_t)p.cls * N + local] += sign;
  for (int i = 0; i < p.own_terms_len; i++) c.term_count[(size_t)P.ints[p.own_terms_off + i] * N + local] += sign;
}

}  // namespace kss
