// kss_preempt.cuh — DefaultPreemption PostFilter dry run of one pod (k_preempt).
//
// Restates, for a pod whose filters left no feasible node, Evaluator.Preempt of upstream
// k8s.io/kubernetes v1.26.2 (pkg/scheduler/framework/preemption/preemption.go) with the
// DefaultPreemption plugin (plugins/defaultpreemption/default_preemption.go), as the
// simulator runs it through wrappedPlugin.PostFilter (simulator/scheduler/plugin/
// wrappedplugin.go:550-577).  The object-level restatement it is tested against is
// oracle/k8s_preemption.py.
//
// Three launches per pod (the PostFilter call is a per-pod latency path):
//   1. PreFilter state of PodTopologySpread / InterPodAffinity (the same LDS histograms
//      as k_schedule, kss_sched.cuh stats_node), plus per hard-spread key the two
//      smallest pair counts with the smallest pair's id (criticalPaths) and the
//      affinity-count total (len(affinityCounts) == 0);
//   2. the filter chain per node; nodesWherePreemptionMightHelp keeps the nodes whose
//      first failure is Unschedulable (NodeResourcesFit, the spread skew, pod
//      anti-affinity and existing pods' anti-affinity), not UnschedulableAndUnresolvable;
//   3. SelectVictimsOnNode on each of them, one lane per node over the grid: remove every
//      lower-priority pod (NodeInfo.RemovePod + the RemovePod extensions: the node's own
//      pair counts move, the spread minimum becomes min(min over the other pairs, the
//      node's pair) — criticalPaths.update keeps exactly that minimum when one pair
//      changes), run the filters, then reprieve in MoreImportantPod order (priority
//      descending, start time ascending, NodeInfo order on ties: sorted per node on the host
//      when the bound-pod table is uploaded), keeping each pod whose return still lets the
//      pod fit;
//   4. pickOneNodeForPreemption as a lexicographic reduction over the candidates'
//      (highest victim priority min, Σ(priority + 2^31) min, #victims min, earliest
//      start of the highest-priority victims max, node index min) — the last criterion
//      replaces the Go map order upstream leaves to chance — per k_preempt_nodes workgroup,
//      then over the workgroups' tuples;
//   5. one lane re-runs the nominated node's reprieve loop and writes the victims' ids in
//      eviction order.
// No PodDisruptionBudgets (every victim is non-violating).  Every filter call is
// RunFilterPluginsWithNominatedPods: the nominator's pods of priority >= the preemptor's on the
// node take part in a first pass (kss_sched.cuh NomView); they are never victims.
#pragma once
#include "kss_sched.cuh"

namespace kss {

constexpr int PRE_THREADS = 512;
constexpr int PRE_WAVES = PRE_THREADS / 64;
constexpr int PRE_NODE_THREADS = 64;  // k_preempt_nodes: one lane per node, many small workgroups

// Bound pods on the device: CSR by node, each node's pods in MoreImportantPod order (the host
// sorts them when it uploads the table: priority descending, start ascending, NodeInfo order
// on ties).
struct DevBound {
  const int32_t* ptr;    // [N + 1]
  const int64_t* id;     // [nb] caller ids
  const int32_t* prio;   // [nb]
  const int64_t* start;  // [nb]
  const int32_t* cls;    // [nb]
  const int64_t* req;    // [nb][KSS_NRES]
  const int32_t* toff;   // [nb] into ints
  const int32_t* tlen;   // [nb]
  const int32_t* ints;
};

struct PreemptOut {
  int32_t status, nominated, n_potential, n_candidates, n_victims, highest_priority;
  int64_t sum_priority, earliest_start;
};

// PreFilter state and counters shared by the three launches (HBM)
struct PreGlobal {
  long long m0[MAXH], id0[MAXH], m1[MAXH];
  long long aff_total, flags;
  int plan_ok, prefilter;
  int n_potential, n_candidates, feasible, pad;
  unsigned ticket;   // k_preempt_stats workgroups done (the last one finishes the criticalPaths)
  unsigned nticket;  // k_preempt_nodes workgroups done (the last one picks the node)
};
constexpr int PRE_STATS_MAX_BLOCKS = 64;

struct PreemptJob {
  DevCluster c;
  DevPods P;
  DevBound B;
  kss_profile prof;
  int32_t pi;        // the preemptor's index in P
  int32_t bins_cap;  // LDS histogram + presence bins
  int32_t victims_cap;
  int32_t n_blocks;  // k_preempt_nodes workgroups
  int64_t* key;      // [5][n_blocks] HBM scratch: each workgroup's best candidate (hp, sum, cnt, start, node)
  int64_t* victims;  // [victims_cap]
  Plan plan;         // the pod's bin plan (make_plan on the host)
  int32_t plan_ok;
  int64_t* vscratch; // [bound pods]: each candidate node's victims in eviction order, at the
                     // node's CSR offset (k_preempt_nodes; a node's victims are among its pods)
  long long* stop2;  // [n_sblocks][MAXH][2]: per stats workgroup and node-valued hard owner, its
                     // smallest (count << 24 | node) and the next smallest count
  PreemptOut* out;
  PreGlobal* G;
  long long* gbins;  // [bins_cap] the PreFilter histograms and presence bins
  const DevNom* nom; // the nominator (kss_nominate): RunFilterPluginsWithNominatedPods' first pass
  int32_t n_nom;
  int32_t pod_id;    // the preemptor's identity (its podset index: it is never its own nominee)
};

struct PreHdr {
  NomPts npts;  // nominees: the pairs at each hard owner's minimum and the next count (from m0 / m1)
  long long red[PRE_WAVES];
  kss_pod pod;
  Plan plan;
  long long m0[MAXH], id0[MAXH], m1[MAXH];  // per hard owner: smallest pair count, its pair, the next one
  long long aff_total;
  long long flags;
  int plan_ok;
  int pad[3];
};

__device__ __forceinline__ long long* pre_bins(long long* smem) { return smem + sizeof(PreHdr) / 8; }

// workgroup reduction (every lane gets the result)
__device__ __forceinline__ long long block_op(long long v, int op, long long* red) {
  v = wave_reduce(v, op);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  long long r = red[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); i++) r = op_apply(op, r, red[i]);
  return r;
}

__device__ __forceinline__ bool in_list(const int32_t* ints, int off, int len, int v) {
  for (int i = 0; i < len; i++)
    if (ints[off + i] == v) return true;
  return false;
}

// tpCounts[pair] of node n for hard group owner i: the count of the group's last member
// admitting n (calPreFilterState), -1 when no member admits n or n lacks a hard key
__device__ __forceinline__ int64_t group_count(const DevCluster& c, const DevPods& P, const kss_pod& p, const Plan& pl,
                                               int i, int n) {
  const kss_spread* sp = P.spreads + p.spread_off;
  if (!has_keys(c, sp, p.n_hard, n)) return -1;
  int64_t cnt = -1;
  for (int j = i; j < p.n_hard; j++)
    if (pl.hard_own[j] == i && spread_policy_ok(c, P, p, sp[j], n)) cnt = spread_count(c, P, sp[j], n);
  return cnt;
}

// The node-local view SelectVictimsOnNode mutates: NodeInfo.Requested / len(Pods), the
// spread pair count of the node's pair per hard owner, the inter-pod-affinity counts of
// the node's pairs per (key slot, x|a|b), and the affinity-count total.
struct DryState {
  int64_t req[KSS_NRES];
  int64_t pods;
  int32_t M[MAXH];     // pod counts (32 bits: the state stays in registers, k_preempt_nodes
  int32_t A[MAXK][3];  // spilled 80 B per lane with 64-bit counts)
  int32_t T;
};

// RemovePod (sign = -1) / AddPod (+1) of bound pod e on node n, with the RemovePod /
// AddPod extensions (podtopologyspread / interpodaffinity preFilterState.updateWithPod)
// A bound pod's request row and class, loaded ahead of its turn (select_victims' reprieve loop
// issues pod k+1's loads before it evaluates pod k: one memory round trip per victim less)
struct VRow {
  int64_t req[KSS_NRES];
  int32_t cls;
};
__device__ __forceinline__ VRow load_vrow(const PreemptJob& J, int e) {
  VRow v;
  const int nr = 3 + J.c.n_scalar;
#pragma unroll
  for (int r = 0; r < KSS_NRES; r++) v.req[r] = r < nr ? J.B.req[(size_t)e * KSS_NRES + r] : 0;
  v.cls = J.B.cls[e];
  return v;
}

__device__ __forceinline__ void apply_row(const PreemptJob& J, const kss_pod& p, const Plan& pl, const VRow& v, int e,
                                          int n, int sign, DryState& s);
__device__ __forceinline__ void apply_pod(const PreemptJob& J, const kss_pod& p, const Plan& pl, int e, int n, int sign,
                                          DryState& s) {
  apply_row(J, p, pl, load_vrow(J, e), e, n, sign, s);
}
__device__ __forceinline__ void apply_row(const PreemptJob& J, const kss_pod& p, const Plan& pl, const VRow& v, int e,
                                          int n, int sign, DryState& s) {
  const DevCluster& c = J.c;
  const DevPods& P = J.P;
#pragma unroll
  for (int r = 0; r < KSS_NRES; r++) s.req[r] += sign * v.req[r];
  s.pods += sign;
  const int cls = v.cls;
  const kss_spread* sp = P.spreads + p.spread_off;
  // the DryState arrays are indexed by compile-time constants only (selects), so they stay in
  // registers: a runtime index would put the whole state in scratch
  for (int j = 0; j < p.n_hard; j++) {  // each matching constraint moves the shared pair counter
    if (!in_list(P.ints, sp[j].cls_off, sp[j].cls_len, cls)) continue;
    const int o = pl.hard_own[j];
#pragma unroll
    for (int x = 0; x < MAXH; x++) s.M[x] += x == o ? sign : 0;
  }
  const kss_ipa* ip = P.ipa + p.ipa_off;
  for (int q = 0; q < p.ipa_len; q++) {
    const kss_ipa& en = ip[q];
    if (en.kind > KSS_IPA_REQ_ANTI) continue;
    if (label_of(c, en.key, n) < 0) continue;  // topologyToMatchedTermCount.update: node lacks the key
    const int k = slot_of(pl, en.key);
    int d = 0, h = 0;
    if (en.kind == KSS_IPA_EXISTING_ANTI) {
      const int t0 = J.B.toff[e], tl = J.B.tlen[e];
      for (int t = 0; t < tl; t++) d += in_list(P.ints, en.row_off, en.row_len, J.B.ints[t0 + t]) ? sign : 0;
    } else if (in_list(P.ints, en.row_off, en.row_len, cls)) {
      d = sign;
      h = en.kind == KSS_IPA_REQ_AFFINITY ? 1 : 2;
      if (en.kind == KSS_IPA_REQ_AFFINITY) s.T += sign;
    }
#pragma unroll
    for (int x = 0; x < MAXK; x++)
#pragma unroll
      for (int y = 0; y < 3; y++) s.A[x][y] += (x == k && y == h) ? d : 0;
  }
}

// AddPod of nominee q on node n (addNominatedPods: NodeInfo.AddPodInfo and the AddPod extensions),
// the same updates apply_pod makes for a bound pod
__device__ __forceinline__ void apply_nom(const PreemptJob& J, const kss_pod& p, const Plan& pl, const DevNom& q, int n,
                                          DryState& s) {
  const DevCluster& c = J.c;
  const DevPods& P = J.P;
  const int nr = 3 + c.n_scalar;
#pragma unroll
  for (int r = 0; r < KSS_NRES; r++)
    if (r < nr) s.req[r] += q.req[r];
  s.pods += 1;
  const kss_spread* sp = P.spreads + p.spread_off;
  for (int j = 0; j < p.n_hard; j++) {
    if (!in_list(P.ints, sp[j].cls_off, sp[j].cls_len, q.cls)) continue;
    const int o = pl.hard_own[j];
#pragma unroll
    for (int x = 0; x < MAXH; x++) s.M[x] += x == o ? 1 : 0;
  }
  const kss_ipa* ip = P.ipa + p.ipa_off;
  for (int e = 0; e < p.ipa_len; e++) {
    const kss_ipa& en = ip[e];
    if (en.kind > KSS_IPA_REQ_ANTI) continue;
    if (label_of(c, en.key, n) < 0) continue;
    const int k = slot_of(pl, en.key);
    int d = 0, h = 0;
    if (en.kind == KSS_IPA_EXISTING_ANTI) {
      for (int t = 0; t < q.n_terms; t++) d += in_list(P.ints, en.row_off, en.row_len, q.terms[t]) ? 1 : 0;
    } else if (in_list(P.ints, en.row_off, en.row_len, q.cls)) {
      d = 1;
      h = en.kind == KSS_IPA_REQ_AFFINITY ? 1 : 2;
      if (en.kind == KSS_IPA_REQ_AFFINITY) s.T += 1;
    }
#pragma unroll
    for (int x = 0; x < MAXK; x++)
#pragma unroll
      for (int y = 0; y < 3; y++) s.A[x][y] += (x == k && y == h) ? d : 0;
  }
}

// s.M[o] / s.A[k][h] for runtime o, k (selects over the unrolled indices: no scratch)
__device__ __forceinline__ int64_t dry_m(const DryState& s, int o) {
  int64_t v = 0;
#pragma unroll
  for (int x = 0; x < MAXH; x++) v = x == o ? s.M[x] : v;
  return v;
}
__device__ __forceinline__ int64_t dry_a(const DryState& s, int k, int h) {
  int64_t v = 0;
#pragma unroll
  for (int x = 0; x < MAXK; x++)
#pragma unroll
    for (int y = 0; y < 3; y++) v = (x == k && y == h) ? s.A[x][y] : v;
  return v;
}

// The node's allocatable row and pod limit, loaded once per dry run of the node (not per victim)
struct NodeCap {
  int64_t alloc[KSS_NRES];
  int64_t allowed;
};
__device__ __forceinline__ NodeCap load_cap(const DevCluster& c, int n) {
  NodeCap k;
  const size_t N = (size_t)c.N;
  const int nr = 3 + c.n_scalar;
#pragma unroll
  for (int r = 0; r < KSS_NRES; r++) k.alloc[r] = r < nr ? c.alloc[(size_t)r * N + n] : 0;
  k.allowed = c.allowed_pods[n];
  return k;
}

// RunFilterPluginsWithNominatedPods on the modified node: NodeResourcesFit, PodTopologySpread,
// InterPodAffinity (the node-level filters before them passed: the node is potential)
__device__ __forceinline__ bool dry_fits(const PreemptJob& J, const kss_pod& p, const Plan& pl, const PreHdr& H,
                                         const DryState& s, int n, const NodeCap& nc) {
  const DevCluster& c = J.c;
  const DevPods& P = J.P;
  const uint32_t en = J.prof.filter_enabled;
  if ((en >> KSS_F_NODE_RESOURCES_FIT) & 1u) {
    if (s.pods + 1 > nc.allowed) return false;
    const int nr = 3 + c.n_scalar;
    bool all_zero = true, bad = false;
#pragma unroll
    for (int r = 0; r < KSS_NRES; r++) {
      if (r >= nr) continue;
      const int64_t q = p.fit_request[r];
      all_zero &= q == 0;
      if (r >= KSS_RES_SCALAR0 && q == 0) continue;
      bad |= q > nc.alloc[r] - s.req[r];
    }
    if (!all_zero && bad) return false;
  }
  if (((en >> KSS_F_POD_TOPOLOGY_SPREAD) & 1u) && p.n_hard > 0) {
    const kss_spread* sp = P.spreads + p.spread_off;
    for (int i = 0; i < p.n_hard; i++) {
      const int d = label_of(c, sp[i].key, n);
      if (d < 0) return false;
      const int o = pl.hard_own[i];
      const int64_t my = pl.hard_off[o] >= 0 ? (int64_t)d : (int64_t)n;
      const int64_t others = H.id0[o] == my ? H.m1[o] : H.m0[o];
      const int64_t mo = dry_m(s, o);
      const int64_t mn = mo < others ? mo : others;
      if (mo + (int64_t)sp[i].self_match - mn > (int64_t)sp[i].max_skew) return false;
    }
  }
  if (((en >> KSS_F_INTER_POD_AFFINITY) & 1u) && p.ipa_len > 0) {
    const kss_ipa* ip = P.ipa + p.ipa_off;
    bool have = false, exist = true;
    for (int q = 0; q < p.ipa_len; q++) {
      if (ip[q].kind != KSS_IPA_REQ_AFFINITY) continue;
      have = true;
      if (label_of(c, ip[q].key, n) < 0) return false;
      if (dry_a(s, slot_of(pl, ip[q].key), 1) <= 0) exist = false;
    }
    if (have && !exist && !(s.T == 0 && (p.flags & KSS_POD_IPA_SELF_MATCH))) return false;
    for (int q = 0; q < p.ipa_len; q++) {
      const int kind = ip[q].kind;
      if (kind != KSS_IPA_REQ_ANTI && kind != KSS_IPA_EXISTING_ANTI) continue;
      if (label_of(c, ip[q].key, n) < 0) continue;
      if (dry_a(s, slot_of(pl, ip[q].key), kind == KSS_IPA_REQ_ANTI ? 2 : 0) > 0) return false;
    }
  }
  return true;
}

// RunFilterPluginsWithNominatedPods over the dry-run view: with nominees on the node (here) the
// first pass runs with them added, the plain pass decides when it passes
__device__ __forceinline__ bool dry_fits_nom(const PreemptJob& J, const kss_pod& p, const Plan& pl, const PreHdr& H,
                                             const DryState& s, int n, uint64_t here, const NodeCap& nc) {
  if (here) {
    DryState s1 = s;
    for (uint64_t m = here; m; m &= m - 1) apply_nom(J, p, pl, J.nom[__ffsll((unsigned long long)m) - 1], n, s1);
    if (!dry_fits(J, p, pl, H, s1, n, nc)) return false;
  }
  return dry_fits(J, p, pl, H, s, n, nc);
}

struct DryResult {
  int64_t hp, sum, cnt, start;  // hp = INT64_MAX: not a candidate
};

// SelectVictimsOnNode for node n; ids (optional): the victims' ids in eviction order
__device__ __forceinline__ DryResult select_victims(const PreemptJob& J, const kss_pod& p, const Plan& pl,
                                                    const PreHdr& H, const long long* bins, int n, int64_t* ids,
                                                    int ids_cap, uint64_t here) {
  const DevCluster& c = J.c;
  const DevPods& P = J.P;
  const DevBound& B = J.B;
  DryResult res{INT64_MAX, 0, 0, 0};
  const int e0 = B.ptr[n], e1 = B.ptr[n + 1];
  const int prio = p.priority;
  // the potential victims (priority below the preemptor's) are the suffix [p0, e1) of the
  // node's importance order, visited in reprieve order
  int below = 0;  // independent loads (a scan from the end would wait on each one in turn)
  for (int k = e0; k < e1; k++) below += B.prio[k] < prio ? 1 : 0;
  const int p0 = e1 - below;
  if (p0 == e1) return res;  // "No preemption victims found for incoming pod"
  // the node's view, then every lower-priority pod removed
  DryState s;
  const size_t N = (size_t)c.N;
#pragma unroll
  for (int r = 0; r < KSS_NRES; r++) s.req[r] = r < 3 + c.n_scalar ? c.requested[(size_t)r * N + n] : 0;
  s.pods = c.pod_count[n];
  const kss_spread* sp = P.spreads + p.spread_off;
#pragma unroll
  for (int i = 0; i < MAXH; i++) s.M[i] = 0;
#pragma unroll
  for (int i = 0; i < MAXH; i++) {
    if (i >= p.n_hard || pl.hard_own[i] != i) continue;
    if (pl.hard_off[i] >= 0) {
      const int d = label_of(c, sp[i].key, n);
      s.M[i] = d >= 0 ? (int32_t)bins[pl.hard_off[i] + d] : 0;
    } else {
      const int64_t g = group_count(c, P, p, pl, i, n);
      s.M[i] = g > 0 ? (int32_t)g : 0;
    }
  }
#pragma unroll
  for (int k = 0; k < MAXK; k++)
#pragma unroll
    for (int h = 0; h < 3; h++) s.A[k][h] = 0;
#pragma unroll
  for (int k = 0; k < MAXK; k++) {
    if (k >= pl.n_keys) continue;
    const int d = label_of(c, pl.key[k], n);
    if (d < 0) continue;
#pragma unroll
    for (int h = 0; h < 3; h++) s.A[k][h] = (int32_t)ipa_value(c, P, p, pl, bins, k, h, d, n);
  }
  s.T = (int32_t)H.aff_total;
  const NodeCap nc = load_cap(c, n);
  for (int k = p0; k < e1; k++) apply_pod(J, p, pl, k, n, -1, s);
  if (!dry_fits_nom(J, p, pl, H, s, n, here, nc)) return res;
  // reprieve in importance order (MoreImportantPod, NodeInfo order on ties); the next pod's row is
  // loaded while this one is evaluated
  int victims = 0;
  int64_t hp = 0, sum = 0, st = 0;
  VRow cur = load_vrow(J, p0);
  for (int k = p0; k < e1; k++) {
    const int best = k;
    const VRow nxt = load_vrow(J, min(k + 1, e1 - 1));
    apply_row(J, p, pl, cur, best, n, 1, s);
    if (!dry_fits_nom(J, p, pl, H, s, n, here, nc)) {
      apply_row(J, p, pl, cur, best, n, -1, s);
      if (victims == 0) {
        hp = B.prio[best];
        st = B.start[best];  // the earliest start among the highest-priority victims
      }
      if (ids && victims < ids_cap) ids[victims] = B.id[best];
      sum += (int64_t)B.prio[best] + 2147483648ll;
      victims++;
    }
    cur = nxt;
  }
  if (victims == 0) return res;  // upstream: an error status ("expected at least one victim")
  res.hp = hp;
  res.sum = sum;
  res.cnt = victims;
  res.start = st;
  return res;
}

__device__ __forceinline__ bool resolvable(int f, int detail) {
  if (f == KSS_F_NODE_RESOURCES_FIT || f == KSS_F_NODE_PORTS) return true;
  if (f == KSS_F_POD_TOPOLOGY_SPREAD) return detail == KSS_PTS_CONSTRAINTS_NOT_MATCH;
  if (f == KSS_F_INTER_POD_AFFINITY) return detail != KSS_IPA_AFFINITY;
  return false;
}

// ---------------------------------------------------------------------------
// Two launches on one stream: k_preempt_stats (node ranges over a few workgroups:
// PreFilter state into HBM), k_preempt_nodes (one lane per node over the whole grid:
// filters, potential nodes, SelectVictimsOnNode, each workgroup's best candidate; the last
// workgroup to finish runs pickOneNodeForPreemption and copies the nominated node's victims).
// ---------------------------------------------------------------------------

// pod record and its plan (built on the host, in the job) -> LDS, word-parallel
__device__ __forceinline__ void pre_load_pod(const PreemptJob& J, PreHdr& H) {
  const int tid = threadIdx.x, nt = blockDim.x;
  constexpr int PD = (int)(sizeof(kss_pod) / 4), PL = (int)(sizeof(Plan) / 4);
  static_assert(sizeof(kss_pod) % 4 == 0 && sizeof(Plan) % 4 == 0, "word copies");
  const uint32_t* src = reinterpret_cast<const uint32_t*>(J.P.pods + J.pi);
  uint32_t* dst = reinterpret_cast<uint32_t*>(&H.pod);
  for (int i = tid; i < PD; i += nt) dst[i] = src[i];
  const uint32_t* ps = reinterpret_cast<const uint32_t*>(&J.plan);
  uint32_t* pd = reinterpret_cast<uint32_t*>(&H.plan);
  for (int i = tid; i < PL; i += nt) pd[i] = ps[i];
  if (tid == 0) H.plan_ok = J.plan_ok;
  __syncthreads();
}

// k_preempt_stats over n_sblocks workgroups, each a contiguous node range: the PreFilter
// histograms in LDS, added into the zeroed HBM bins (presence bins as counts: only non-zero
// matters), flags / affinity total by atomics, and per node-valued hard owner the range's two
// smallest counts.  The last workgroup to finish (a ticket after a release fence) reads the
// final bins and writes criticalPaths per hard owner: its smallest pair count, that pair, the next.
// Only the Filter's state is built (no ScheduleAnyway or InterPodAffinity score bins).
__device__ void preempt_stats(const PreemptJob& J, long long* smem) {
  const int tid = threadIdx.x, nt = blockDim.x;
  PreHdr& H = *reinterpret_cast<PreHdr*>(smem);
  const DevCluster& c = J.c;
  const DevPods& P = J.P;
  pre_load_pod(J, H);
  const kss_pod& p = H.pod;
  const Plan& pl = H.plan;
  PreGlobal& G = *J.G;
  const int B = (int)blockIdx.x, NB = (int)gridDim.x;
  if (B == 0 && tid == 0) {
    G.plan_ok = H.plan_ok;
    G.prefilter = p.prefilter_status;
  }
  if (!H.plan_ok || p.prefilter_status != 0) return;  // every workgroup leaves: no criticalPaths to build
  long long* bins = pre_bins(smem);
  long long* pres = bins + pl.total_bins;
  const int N = c.N;
  const int per = (N + NB - 1) / NB, lo = min(N, B * per), hi = min(N, lo + per);
  long long hard_min[MAXH];
#pragma unroll
  for (int i = 0; i < MAXH; i++) hard_min[i] = INT32_MAX;
  long long flags = 0, aff = 0;
  const int nbins = pl.total_bins + pl.total_pbins;
  for (int b = tid; b < nbins; b += nt) bins[b] = 0;
  __syncthreads();
  const kss_ipa* ip = P.ipa + p.ipa_off;
  if (pl.need_stats) {
    for (int n = lo + tid; n < hi; n += nt) {
      stats_node(c, P, p, pl, bins, pres, n, hard_min, flags, /*scoring=*/false);
      for (int q = 0; q < p.ipa_len; q++)
        if (ip[q].kind == KSS_IPA_REQ_AFFINITY && label_of(c, ip[q].key, n) >= 0)
          aff += sum_rows(c.class_count, (size_t)N, P.ints + ip[q].row_off, ip[q].row_len, n);
    }
  }
  flags = block_op(flags, OP_OR, H.red);
  aff = block_op(aff, OP_SUM, H.red);
  // this range's histograms into the cluster's
  for (int b = tid; b < nbins; b += nt) {
    const long long v = bins[b];
    if (v) atomicAdd((unsigned long long*)&J.gbins[b], (unsigned long long)v);
  }
  if (tid == 0) {
    if (flags) atomicOr((unsigned long long*)&G.flags, (unsigned long long)flags);
    if (aff) atomicAdd((unsigned long long*)&G.aff_total, (unsigned long long)aff);
  }
  // node-valued hard owners: the range's smallest (count << 24 | node) and the next smallest count
  for (int i = 0; i < p.n_hard; i++) {
    if (pl.hard_own[i] != i || pl.hard_off[i] >= 0) continue;
    long long best = INT64_MAX;
    for (int x = lo + tid; x < hi; x += nt) {
      const long long v = (long long)group_count(c, P, p, pl, i, x);
      if (v >= 0) best = min(best, (v << 24) | x);
    }
    best = block_op(best, OP_MIN, H.red);
    const long long id0 = best == INT64_MAX ? -1 : (best & 0xFFFFFF);
    long long second = INT64_MAX;
    for (int x = lo + tid; x < hi; x += nt) {
      if (x == id0) continue;
      const long long v = (long long)group_count(c, P, p, pl, i, x);
      if (v >= 0) second = min(second, v);
    }
    second = block_op(second, OP_MIN, H.red);
    if (tid == 0) {
      J.stop2[((size_t)B * MAXH + i) * 2] = best;
      J.stop2[((size_t)B * MAXH + i) * 2 + 1] = second;
    }
  }
  // the last workgroup (ticket after a release) builds the criticalPaths from the final state
  __threadfence();
  __syncthreads();
  if (tid == 0) H.plan_ok = (int)(atomicAdd(&G.ticket, 1u) == (unsigned)(NB - 1)) + 1;  // 2: last
  __syncthreads();
  if (H.plan_ok != 2) return;
  __threadfence();
  const kss_spread* sp = P.spreads + p.spread_off;
  for (int i = 0; i < p.n_hard; i++) {
    if (pl.hard_own[i] != i) continue;
    long long best = INT64_MAX, second = INT64_MAX;
    if (pl.hard_off[i] >= 0) {  // histogram key: the smallest present pair and the next
      const int span = c.key_card[sp[i].key] + 1;
      auto val = [&](int x) -> long long {
        const long long pr = __hip_atomic_load(&J.gbins[pl.total_bins + pl.hard_poff[i] + x], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
        return pr ? __hip_atomic_load(&J.gbins[pl.hard_off[i] + x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : -1;
      };
      for (int x = tid; x < span; x += nt) {
        const long long v = val(x);
        if (v >= 0) best = min(best, (v << 24) | x);
      }
      best = block_op(best, OP_MIN, H.red);
      const long long id0 = best == INT64_MAX ? -1 : (best & 0xFFFFFF);
      for (int x = tid; x < span; x += nt) {
        if (x == id0) continue;
        const long long v = val(x);
        if (v >= 0) second = min(second, v);
      }
      second = block_op(second, OP_MIN, H.red);
    } else {  // node-valued key: merge the workgroups' two smallest
      long long b = INT64_MAX;
      int owner = -1;
      for (int q = 0; q < NB; q++) {
        const long long v = __hip_atomic_load(&J.stop2[((size_t)q * MAXH + i) * 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v < b) b = v, owner = q;
      }
      best = b;
      for (int q = 0; q < NB; q++) {
        const long long v = q == owner ? __hip_atomic_load(&J.stop2[((size_t)q * MAXH + i) * 2 + 1], __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT)
                                       : __hip_atomic_load(&J.stop2[((size_t)q * MAXH + i) * 2], __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
        const long long cnt = (q == owner || v == INT64_MAX) ? v : (v >> 24);
        second = min(second, cnt);
      }
    }
    if (tid == 0) {
      G.m0[i] = best == INT64_MAX ? INT32_MAX : (best >> 24);
      G.id0[i] = best == INT64_MAX ? -1 : (best & 0xFFFFFF);
      G.m1[i] = second == INT64_MAX ? INT32_MAX : second;
    }
  }
}

// pickOneNodeForPreemption, by the last k_preempt_nodes workgroup (pod and plan already in
// LDS); the other workgroups' counts and tuples through agent-scope loads (their release
// fences wrote them back).
__device__ __forceinline__ long long ld_agent(const long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_agent(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

__device__ void preempt_pick_last(const PreemptJob& J, long long* smem) {
  const int tid = threadIdx.x, nt = blockDim.x;
  PreHdr& H = *reinterpret_cast<PreHdr*>(smem);
  const DevCluster& c = J.c;
  const PreGlobal& G = *J.G;
  PreemptOut& out = *J.out;
  const int feasible = ld_agent(&G.feasible), n_pot = ld_agent(&G.n_potential), n_cand = ld_agent(&G.n_candidates);
  if (feasible || n_cand == 0) {
    if (tid == 0) {
      out.status = feasible ? KSS_PREEMPT_SCHEDULABLE : KSS_PREEMPT_NO_CANDIDATE;
      out.nominated = -1;
      out.n_potential = n_pot;
      out.n_candidates = n_cand;
      out.n_victims = 0;
    }
    return;
  }
  const int nb = J.n_blocks;
  const long long* K = reinterpret_cast<const long long*>(J.key);
  // over the workgroups' best tuples (each lane folds its share lexicographically, then the
  // same successive reductions over the lanes)
  long long hp = INT64_MAX, sum = INT64_MAX, cnt = INT64_MAX, st = INT64_MIN, nn = INT64_MAX;
  for (int b = tid; b < nb; b += nt) {
    const long long h = ld_agent(K + b), s2 = ld_agent(K + nb + b), c2 = ld_agent(K + 2 * nb + b),
                    t2 = ld_agent(K + 3 * nb + b), n2 = ld_agent(K + 4 * nb + b);
    const bool better = h != hp ? h < hp : (s2 != sum ? s2 < sum : (c2 != cnt ? c2 < cnt : (t2 != st ? t2 > st : n2 < nn)));
    if (better) hp = h, sum = s2, cnt = c2, st = t2, nn = n2;
  }
  const long long bhp = block_op(hp, OP_MIN, H.red);
  bool eq = hp == bhp;
  const long long bsum = block_op(eq ? sum : INT64_MAX, OP_MIN, H.red);
  eq &= sum == bsum;
  const long long bcnt = block_op(eq ? cnt : INT64_MAX, OP_MIN, H.red);
  eq &= cnt == bcnt;
  const long long bst = block_op(eq ? st : INT64_MIN, OP_MAX, H.red);
  eq &= st == bst;
  const long long best = block_op(eq ? nn : INT64_MAX, OP_MIN, H.red);
  // the nominated node's victims, kept by its dry run
  const int nv = (int)bcnt;
  const long long* vs = reinterpret_cast<const long long*>(J.vscratch + J.B.ptr[best]);
  for (int i = tid; i < min(nv, J.victims_cap); i += nt) J.victims[i] = ld_agent(vs + i);
  if (tid == 0) {
    out.status = KSS_PREEMPT_NOMINATED;
    out.nominated = (int32_t)(c.node_base + best);
    out.n_potential = n_pot;
    out.n_candidates = n_cand;
    out.n_victims = nv;
    out.highest_priority = (int32_t)bhp;
    out.sum_priority = bsum;
    out.earliest_start = bst;
  }
}

__device__ void preempt_nodes(const PreemptJob& J, long long* smem) {
  const int tid = threadIdx.x;
  PreHdr& H = *reinterpret_cast<PreHdr*>(smem);
  const DevCluster& c = J.c;
  const DevPods& P = J.P;
  const PreGlobal& G = *J.G;
  if (!G.plan_ok || G.prefilter != 0) {
    // a PreFilter failure gives every node UnschedulableAndUnresolvable: nothing to dry-run
    if (blockIdx.x == 0 && tid == 0) {
      PreemptOut& out = *J.out;
      out.status = !G.plan_ok ? -1 : KSS_PREEMPT_NO_CANDIDATE;
      out.nominated = -1;
      out.n_potential = out.n_candidates = out.n_victims = 0;
    }
    return;
  }
  pre_load_pod(J, H);
  if (tid == 0) {
    for (int i = 0; i < MAXH; i++) {
      H.m0[i] = G.m0[i];
      H.id0[i] = G.id0[i];
      H.m1[i] = G.m1[i];
    }
    H.aff_total = G.aff_total;
    H.flags = G.flags;
    for (int i = 0; i < MAXH; i++) {  // criticalPaths' two smallest: another pair at the minimum, or the next count
      H.npts.cnt[i] = G.m1[i] == G.m0[i] ? 2 : 1;
      H.npts.gt[i] = G.m1[i];
    }
  }
  __syncthreads();
  const kss_pod& p = H.pod;
  const Plan& pl = H.plan;
  const long long* bins = J.gbins;
  long long hard_min[MAXH];
#pragma unroll
  for (int i = 0; i < MAXH; i++) hard_min[i] = i < p.n_hard ? H.m0[pl.hard_own[i]] : INT32_MAX;
  const uint32_t en = J.prof.filter_enabled;
  const int N = c.N;
  const int n = (int)(blockIdx.x * blockDim.x) + tid;
  long long n_pot = 0, n_cand = 0, feasible = 0;
  DryResult best{INT64_MAX, INT64_MAX, INT64_MAX, INT64_MIN};
  if (n < N) {
    if (p.names_len >= 0 && !in_names(P, p, (int64_t)c.node_base + n)) {
      n_pot = 1;  // no status in the map: potential, but NodeAffinity rejects it in the dry run
    } else {
      // the scheduling cycle's status of the node: RunFilterPluginsWithNominatedPods
      const NomView nv{J.nom, J.n_nom, J.pod_id, J.n_nom >= 64 ? ~0ull : ((1ull << J.n_nom) - 1ull)};
      const uint64_t here = J.n_nom ? nom_here(nv, n, p.priority) : 0;
      const NodeRow row = load_row(c, n);
      int f = 0;
      uint16_t detail = 0;
      for (int pass = here ? 0 : 1; pass < 2; pass++) {  // pass 0: the nominees added
        const NomView* v = pass == 0 ? &nv : nullptr;
        uint16_t dd = 0;
        int ff = filter_local(c, P, p, en, n, row, &dd, v ? J.nom : nullptr, pass == 0 ? here : 0);
        if (!ff && ((en >> KSS_F_POD_TOPOLOGY_SPREAD) & 1u) && p.n_hard > 0) {
          const int r = filter_pts(c, P, p, pl, bins, hard_min, n, v, here, &H.npts);
          if (r) {
            ff = KSS_F_POD_TOPOLOGY_SPREAD;
            dd = (uint16_t)(r - 1);
          }
        }
        if (!ff && ((en >> KSS_F_INTER_POD_AFFINITY) & 1u) && p.ipa_len > 0) {
          const int r = filter_ipa(c, P, p, pl, bins, H.flags, n, v, here);
          if (r) {
            ff = KSS_F_INTER_POD_AFFINITY;
            dd = (uint16_t)(r - 1);
          }
        }
        f = ff;
        detail = dd;
        if (ff) break;  // a first-pass failure is the node's status
      }
      if (!f) {
        feasible = 1;
      } else if (resolvable(f, detail)) {
        n_pot = 1;
        const DryResult d = select_victims(J, p, pl, H, bins, n, J.vscratch + J.B.ptr[n], INT32_MAX, here);
        if (d.hp != INT64_MAX) {
          n_cand = 1;
          best = d;
        }
      }
    }
  }
  n_pot = block_op(n_pot, OP_SUM, H.red);
  n_cand = block_op(n_cand, OP_SUM, H.red);
  feasible = block_op(feasible, OP_SUM, H.red);
  // pickOneNodeForPreemption over this workgroup's candidates (lexicographic: highest victim
  // priority min, priority sum min, victims min, start max, node min): k_preempt_pick then
  // reduces one tuple per workgroup instead of re-reading every node's keys
  {
    const long long hp = block_op(best.hp, OP_MIN, H.red);
    bool eq = best.hp == hp;
    const long long sum = block_op(eq ? best.sum : INT64_MAX, OP_MIN, H.red);
    eq &= best.sum == sum;
    const long long cnt = block_op(eq ? best.cnt : INT64_MAX, OP_MIN, H.red);
    eq &= best.cnt == cnt;
    const long long st = block_op(eq ? best.start : INT64_MIN, OP_MAX, H.red);
    eq &= best.start == st;
    const long long nn = block_op(eq && hp != INT64_MAX ? (long long)n : INT64_MAX, OP_MIN, H.red);
    if (tid == 0) {
      const int b = (int)blockIdx.x, nb = J.n_blocks;
      int64_t* K = J.key;
      K[b] = hp;
      K[nb + b] = sum;
      K[2 * nb + b] = cnt;
      K[3 * nb + b] = st;
      K[4 * nb + b] = nn;
    }
  }
  // the last workgroup to finish (a ticket after every lane's release fence: the victims'
  // ids, the tuple and the counts) picks the node
  if (tid == 0) {
    PreGlobal& Gw = *J.G;
    if (n_pot) atomicAdd(&Gw.n_potential, (int)n_pot);
    if (n_cand) atomicAdd(&Gw.n_candidates, (int)n_cand);
    if (feasible) atomicAdd(&Gw.feasible, (int)feasible);
  }
  __threadfence();
  __syncthreads();
  if (tid == 0) H.plan_ok = (int)(atomicAdd(&J.G->nticket, 1u) == (unsigned)(gridDim.x - 1)) + 1;  // 2: last
  __syncthreads();
  if (H.plan_ok != 2) return;
  __threadfence();
  preempt_pick_last(J, smem);
}

}  // namespace kss
