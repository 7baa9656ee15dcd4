// kss_spread.cuh — the sequential scheduling loop for staged batches WITH
// PodTopologySpread / InterPodAffinity programs (BASELINE C3, and C4's recipe on one GPU),
// without a per-node result record.  Same semantics as schedule_pod<true> (kss_sched.cuh),
// organised like k_simple (kss_simple.cuh):
//
//   * the commit-invariant part of every (pod, node) evaluation comes from k_static's
//     static words, which also carry the inclusion-policy bits (NodeAffinityPolicy /
//     NodeTaintsPolicy) the PodTopologySpread counts need;
//   * each pod's program is resolved on the host into a fixed GPod record: the plan
//     (histogram / presence bin offsets, key slots), and every constraint / entry as a
//     list of (count row, coefficient) references; InterPodAffinity score entries of one
//     topology key are merged into one weighted list (kss_lib.hip build_gpods);
//   * the batch's read set of class_count / term_count rows is resident in LDS for the
//     launch as 16-bit counts (host-checked), with the shard's node rows and label ids;
//     commits update them in place (rows outside the read set: HBM atomics) and the
//     resident rows are written back when the launch ends;
//   * records and static words of the next pods are prefetched by every wave but wave 0
//     (wave 0 runs the exchanges and never waits on an HBM access); the outcome stores and
//     HBM commits are issued by a prefetch wave too;
//   * exchanges carry 32-bit values, one {epoch, value} granule each; a pod with a single
//     ScheduleAnyway constraint folds the PodTopologySpread score extrema into the filter
//     exchange (the raw score is monotone in the count), so it needs no third exchange.
//
// Per pod: [stats pass + exchange E1 if the pod needs cluster-wide counts] -> filter +
// raw scores + E2 -> [PodTopologySpread score pass + E3 for > 1 soft constraint] ->
// NormalizeScore + weights + selectHost key + E4 -> commit by the winner's shard.
#pragma once
#include "kss_simple.cuh"

#include <type_traits>

namespace kss {

constexpr int G_QMAX = 128;  // uint4 per record (header + references; host-checked)
constexpr int G_IPA = 16;    // inter-pod-affinity entries per pod (score entries merged per key)
constexpr int G_CMT = 8;     // count rows a pod's commit adds to (its class, its own term rows)
constexpr int G_PF = 4;      // static words per prefetch lane (host-checked)
constexpr int G_XW = 512;    // 32-bit values per shard per exchange (host-checked; the inbox is sized for it)
// A shard's granules of one exchange sit `gs` 8-byte words after the previous shard's: the
// batch's longest exchange rounded up to a 128-byte line (GpodNeeds::gs).  At the fixed
// 4 KiB stride (G_XW) every shard's value j shared one page offset, so the whole grid's
// polls and publishes went to one memory channel.
constexpr int G_NS = 16;     // scalar slots of an exchange
constexpr int G_PAY = 32;    // payload values of the argmax exchange (spread_argmax_pay)
constexpr int G_SCORE = 3;   // GIpa.kind of a merged InterPodAffinity score entry (KSS_IPA_SCORE_CLASS)
constexpr int G_NSTAMP = KSS_NSTAMP_PODS / 2;  // pods with diagnostic phase stamps, 16 per pod

// Diagnostic trace, experiment builds only (make -C csrc exp EXP=trace
// EXP_FLAGS=-DKSS_SPREAD_TRACE=1, or =2 for the light form without the per-pod statistics
// and staged-input checks; tools/split_trace_test.py reads it): per (pod, shard)
// G_TW words (GT_* below), and a list of every nonzero resident count a shard loads in its
// prologue and writes back in its epilogue.  Light on purpose (no extra barrier, a few
// stores per pod): the failure it hunts is timing-dependent.  The product build compiles
// none of it.
#ifndef KSS_SPREAD_TRACE
#define KSS_SPREAD_TRACE 0
#endif
constexpr int G_TW = 128;
enum : int {
  GT_LOCAL = 0,      // [32] the shard's bins after its statistics pass
  GT_XBINS = 32,     // [32] the bins after the statistics exchange
  GT_MINIMA = 64,    // [5] critical-path minima and flags after the exchange
  GT_EPOCH = 69,
  GT_REREAD = 71,    // nodes whose first-group count differs between two reads around the pass
  GT_BAD_ST = 72,    // staged static words that differ from HBM
  GT_BAD_REC = 73,   // staged record words that differ from HBM (every pod, at its commit)
  GT_BAD_LBL = 74,   // staged label ids that differ from HBM
  GT_KEY = 75,       // [3] selectHost key lo, hi, seen
  GT_NF = 78,
  GT_CHOSEN = 79,
  GT_CMT = 80,       // [8] the winner shard's commit: n_cmt, then (resident row, count before) pairs
  GT_PRO = 88,       // nonzero bins of the first pod's range right after the prologue zeroed them
  GT_XCC = 89,       // (first pod of a launch) the XCD the shard's workgroup runs on
  GT_WIN = 90,       // [9] window: shard count, before-start count, exchanged before count, parts a before,
                     // all parts a, parts b before, stopping node + 1, kept nodes, start node
};
constexpr int G_TLIST = 1 << 20;  // entries of the count list: {tag, row, node, value}; tag = k0 (load) or -1 - k1 (store)
struct GTrace {
  int32_t* words;  // [n][W][G_TW]
  int32_t* list;   // [0]: entries used, then G_TLIST entries of 4 words
};

// One topology spread constraint.  v1.26 keys PodTopologySpread's counts by topology pair,
// not by constraint: constraints of one kind on one key form a group led by its first member
// (`own`), which holds the group's histogram (members share off / poff).  DoNotSchedule: per
// node the count of the group's LAST member admitting the node (calPreFilterState's
// tpCounts[pair] = count overwrites).  ScheduleAnyway, non-hostname keys: the pair counter
// sums every admitting member's count, and the domain count (topoSize) belongs to the
// leader, the others weigh log(0 + 2) (initPreScoreState).  Hostname soft constraints are
// never grouped (their counts are per node and per constraint in Score).
struct GSpread {
  int32_t max_skew;
  int16_t key, flags, self_match, mode;  // kss_spread; mode: SOFT_HOST / SOFT_DIRECT / SOFT_HIST
  int16_t ri_off, ri_len;                // references ri[ri_off .. +ri_len)
  int16_t off, poff;                     // histogram / presence bin offsets (-1: node-valued key)
  int16_t empty;                         // key_empty: domain of a node without the key
  int16_t nb;                            // domains of the key + 1
  int16_t own;                           // the group leader's index in GPod::sp
  int16_t pad[3];
};
struct GIpa {
  int16_t kind, key, ri_off, ri_len, slot, pad;  // kind: KSS_IPA_* (score entries: G_SCORE)
};
// Host-resolved program of one pod (build_gpods): this header, then its references as
// uint32 (resident row index | coefficient << 16), the record padded to the batch's stride
// of `gq` uint4 (the longest reference list decides it).  Per IPA key slot k, histogram h (0
// existing anti-affinity, 1 required affinity, 2 required anti-affinity, 3 score) lives at
// hoff[k][h]; -1 for a node-valued (unique) key, whose value is the node's own sum, and
// for a histogram no entry of the pod feeds (never read).
struct alignas(16) GPod {
  SPod dyn;
  int32_t pflags, n_hard, n_soft, n_ipa;
  int32_t n_keys, total_bins, hard_pbins, total_pbins;
  int32_t need_stats, n_cmt;
  int32_t fold;  // the statistics may ride with the previous pod's exchanges (spread_argmax_pay)
  int32_t pad1;
  int32_t key[MAXK];
  int32_t hoff[MAXK][4];
  int32_t cmt[G_CMT];   // resident row index, or -(1 + class row) / -(1 + n_classes + term row) in HBM
  GSpread sp[MAXH + MAXS];
  GIpa ipa[G_IPA];
};
static_assert(sizeof(GPod) % 16 == 0 && sizeof(GPod) / 16 < G_QMAX, "record header");
// the references of a record
__host__ __device__ inline const uint32_t* grefs(const GPod& q) { return reinterpret_cast<const uint32_t*>(&q + 1); }

// Go math.Log (src/math/log.go), the same IEEE operation sequence as the host port
// (kss_host.cpp kss_go_log; both compiled with -ffp-contract=off):
// PodTopologySpread's topologyNormalizingWeight = math.Log(float64(size + 2)).
// tests/test_gpu_spread.py checks it bit for bit against the host port.
__device__ __forceinline__ double go_log_dev(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
               L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  int ki;
  double f1 = frexp(x, &ki);
  if (f1 < 0.70710678118654752440 /* math.Sqrt2 / 2 */) {
    f1 *= 2;
    ki--;
  }
  const double f = f1 - 1;
  const double k = (double)ki;
  const double s = f / (2 + f);
  const double s2 = s * s;
  const double s4 = s2 * s2;
  const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  const double R = t1 + t2;
  const double hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

// LDS image: header, the exchange vector, then the shard arrays.
struct alignas(16) SpreadHdr {
  int32_t red[MAXWAVES][G_NS];
  long long kred[2][MAXWAVES];
  long long kx[MAXWAVES];  // multi-wave argmax sweep: each wave's maximum
  long long kres;
  kss_profile prof;  // a runtime (non-default) profile, staged word by word (as SimpleHdr)
  unsigned long long pay[G_PAY];  // fused exchange: {key, payload} of the best shard per payload value
  int32_t payv[G_PAY];            // ... this shard's payloads, as published
  int32_t fmin[MAXH];             // ... the next pod's critical-path minima and flags
  int32_t fflags;
  int32_t abort;
  int32_t pad[2];
  int32_t tl_x, tl_s, tl_n;  // two-level exchange (X.tl): the shard's XCD, its rank there, the XCD's shards
  uint32_t tl_mask;          // ... the XCDs holding shards
  int32_t wc[G_PF][MAXWAVES];  // window: feasible slots per (loop iteration, wave)
  int32_t wb[G_PF][MAXWAVES];  // ... of them, nodes before the start node
  int32_t wsum[4];             // ... parts a before this shard, all parts a, parts b before this shard
};

struct SpreadShard {
  int32_t* xs;     // [G_NS + bins_cap]: exchange scalars, then histogram / presence bins
  uint4* ring;     // [3][gq] pod programs (slot = pod % 3)
  uint32_t* st;    // [2][cap] static words (slot = pod & 1)
  uint16_t* cnt;   // [n_res][cap] resident count rows (snapshot + this launch's commits)
  double* r64;     // [8][cap] allocatable, requested (cpu, mem, eph), non-zero requested (cpu, mem)
  double* inv;     // [3][cap]
  long long* sipa; // [cap] InterPodAffinity raw
  long long* spts; // [cap] PodTopologySpread raw (> 1 soft constraint)
  int32_t* r32;    // [3][cap] pod count, allowed pods, node flags
  int32_t* lbl;    // [n_keys][cap] label value ids
  int32_t* sf;     // [cap] verdict | ignored << 16
  int32_t* stt;    // [cap] TaintToleration raw
  int32_t* sna;    // [cap] NodeAffinity raw
  int32_t* sfit;   // [cap]
  int32_t* sba;    // [cap]
  int32_t* scnt;   // [cap] single soft constraint: the node's count (-1 lacks the key)
  int64_t* sc;     // [2 nsc][cap] allocatable, then requested, of each extended (scalar) resource
  int cap, nsc;
};

// fold (k_spread<., true>): two bins areas (pod k and pod k + 1, by parity) and three static-word
// slots (pods k .. k + 2: the early statistics pass of pod k + 1 reads its words during pod k)
__host__ __device__ inline size_t spread_lds_bytes(int cap, int bins_cap, int n_keys, int n_res, int gq, int nsc = 0,
                                                   bool fold = false) {
  const size_t C = (size_t)cap;
  const size_t nb = (size_t)bins_cap * (fold ? 2 : 1), nst = fold ? 3 : 2;
  size_t b = (sizeof(SpreadHdr) + 4 * ((size_t)G_NS + nb) + 15) / 16 * 16;
  b += 3 * 16 * (size_t)gq + 4 * nst * C + ((size_t)n_res * C * 2 + 15) / 16 * 16;
  b += 8 * 8 * C + 8 * 3 * C + 8 * 2 * C + 4 * 3 * C + 4 * (size_t)n_keys * C + 4 * 6 * C;
  b += 16 * (size_t)nsc * C;
  return b;
}

__device__ __forceinline__ SpreadShard spread_view(long long* smem, int cap, int bins_cap, int n_keys, int n_res,
                                                   int gq, int nsc, bool fold = false) {
  SpreadShard L;
  const size_t C = (size_t)cap;
  L.nsc = nsc;
  uint8_t* b = reinterpret_cast<uint8_t*>(smem);
  size_t o = sizeof(SpreadHdr);
  L.xs = reinterpret_cast<int32_t*>(b + o);
  o = (o + 4 * ((size_t)G_NS + (size_t)bins_cap * (fold ? 2 : 1)) + 15) / 16 * 16;
  L.ring = reinterpret_cast<uint4*>(b + o);
  o += 3 * 16 * (size_t)gq;
  L.st = reinterpret_cast<uint32_t*>(b + o);
  o += 4 * (fold ? 3 : 2) * C;
  L.cnt = reinterpret_cast<uint16_t*>(b + o);
  o += ((size_t)n_res * C * 2 + 15) / 16 * 16;
  L.r64 = reinterpret_cast<double*>(b + o);
  o += 8 * 8 * C;
  L.sc = reinterpret_cast<int64_t*>(b + o);
  o += 16 * (size_t)nsc * C;
  L.inv = reinterpret_cast<double*>(b + o);
  o += 8 * 3 * C;
  L.sipa = reinterpret_cast<long long*>(b + o);
  o += 8 * C;
  L.spts = reinterpret_cast<long long*>(b + o);
  o += 8 * C;
  L.r32 = reinterpret_cast<int32_t*>(b + o);
  o += 4 * 3 * C;
  L.lbl = reinterpret_cast<int32_t*>(b + o);
  o += 4 * (size_t)n_keys * C;
  L.sf = reinterpret_cast<int32_t*>(b + o);
  L.stt = L.sf + C;
  L.sna = L.sf + 2 * C;
  L.sfit = L.sf + 3 * C;
  L.sba = L.sf + 4 * C;
  L.scnt = L.sf + 5 * C;
  L.cap = cap;
  return L;
}

// Σ coefficient x count over references [off, off + len) at slot s (sum_rows of
// class_count / term_count; a merged score entry's Σ coef_e x Σ rows_e).
__device__ __forceinline__ int32_t g_sum(const SpreadShard& L, const GPod& q, int off, int len, int s) {
  const uint32_t* R = grefs(q);
  int32_t v = 0;
  for (int i = 0; i < len; i++) {
    const uint32_t r = R[off + i];
    v += (int32_t)(int16_t)(r >> 16) * (int32_t)L.cnt[(int)(r & 0xFFFFu) * L.cap + s];
  }
  return v;
}

// some referenced row counts a pod at slot s (the "topologyScore is non-empty" test of a
// score entry: every count is >= 0, so a weighted sum can cancel but this cannot)
__device__ __forceinline__ bool g_any(const SpreadShard& L, const GPod& q, int off, int len, int s) {
  const uint32_t* R = grefs(q);
  bool a = false;
  for (int i = 0; i < len; i++) a |= L.cnt[(int)(R[off + i] & 0xFFFFu) * L.cap + s] != 0;
  return a;
}

__device__ __forceinline__ bool g_policy(const GSpread& sp, uint32_t w) {
  if ((sp.flags & KSS_SPREAD_POLICY_AFFINITY_HONOR) && !(w & SW_AFF_OK)) return false;
  if ((sp.flags & KSS_SPREAD_POLICY_TAINTS_HONOR) && !(w & SW_TAINT_OK)) return false;
  return true;
}

__device__ __forceinline__ bool g_has_keys(const SpreadShard& L, const GSpread* sp, int cnt, int s) {
  for (int i = 0; i < cnt; i++)
    if (L.lbl[sp[i].key * L.cap + s] < 0) return false;
  return true;
}

__device__ __forceinline__ int32_t op32(int op, int32_t a, int32_t b) {
  if (op == OP_SUM) return (int32_t)((uint32_t)a + (uint32_t)b);
  if (op == OP_MAX) return b > a ? b : a;
  if (op == OP_MIN) return b < a ? b : a;
  return a | b;
}
__device__ __forceinline__ int32_t ident32(int op) { return op == OP_MAX ? INT32_MIN : (op == OP_MIN ? INT32_MAX : 0); }

// op32 for an operator that differs between lanes: every operator computed, one picked by
// selects (a per-lane `op` in op32 compiles to nested exec-mask branches)
__device__ __forceinline__ int32_t op32_lane(int op, int32_t a, int32_t b) {
  const int32_t s = (int32_t)((uint32_t)a + (uint32_t)b), mx = max(a, b), mn = min(a, b), o = a | b;
  return op == OP_SUM ? s : (op == OP_MAX ? mx : (op == OP_MIN ? mn : o));
}

// K 32-bit wave reductions on the DPP network, interleaved: each step issues every value's
// move before combining any (kss_simple.cuh wave_red's sequence); lane 63 holds the results.
template <int CTRL, int ROWS, int K>
__device__ __forceinline__ void dpp32_step(int32_t (&v)[K], const int (&ops)[K]) {
  int32_t t[K];
#pragma unroll
  for (int k = 0; k < K; k++) t[k] = __builtin_amdgcn_update_dpp(ident32(ops[k]), v[k], CTRL, ROWS, 0xF, false);
#pragma unroll
  for (int k = 0; k < K; k++) v[k] = op32(ops[k], v[k], t[k]);
}

template <int K>
__device__ __forceinline__ void wave_red32(int32_t (&v)[K], const int (&ops)[K]) {
  dpp32_step<0xB1, 0xF>(v, ops);   // quad_perm [1,0,3,2]
  dpp32_step<0x4E, 0xF>(v, ops);   // quad_perm [2,3,0,1]
  dpp32_step<0x141, 0xF>(v, ops);  // row_half_mirror
  dpp32_step<0x140, 0xF>(v, ops);  // row_mirror
  dpp32_step<0x142, 0xA>(v, ops);  // row_bcast:15 -> rows 1, 3
  dpp32_step<0x143, 0xC>(v, ops);  // row_bcast:31 -> rows 2, 3
#pragma unroll
  for (int k = 0; k < K; k++) v[k] = __builtin_amdgcn_readlane(v[k], 63);
}

// Cross-shard part of a 32-bit exchange, wave 0 only: publish M = K + ns + no values
// (scalars xs[0..K), SUM bins xs[G_NS + sum_lo ..), OR bins xs[G_NS + or_lo ..)) as
// {epoch, value} granules, then sweep every shard's.  The sweep gives each value
// T = 64 / M lanes; lane (j, t) polls value j of shards t, t + T, ... (up to XS at once, all
// in flight), folds them in registers, and one LDS atomic per lane combines the T partials
// (the slot holds the operator's identity since the publish; the own contribution comes
// back through the sweep).  A matched granule is final: it can only change at epoch + 2.
// The scalars are combined over the workgroup's waves here (H.red), by the lanes that
// publish them.  Granules are accessed through address-space-1 pointers: flat accesses would
// also count in lgkmcnt and make every following LDS wait on the HBM stores.
// phase bit 0: publish (wave 0), bit 1: sweep by wave gw of nsw sweeping waves (lanes of
// every sweeping wave share the values: T = 64 nsw / M lanes per value).
#ifndef KSS_LANE_RED
#define KSS_LANE_RED 0  // spread_reduce: the waves' partials written by K lanes (r7g A/B: C4 -0.5 %, C3 -1.4 %: off)
#endif
constexpr int G_XS = 16;  // at most this many shards polled per lane at once (4 / 8 / 16 by need)
#ifndef KSS_SPREAD_SAFE
#define KSS_SPREAD_SAFE 0  // experiment builds: extra barriers around the exchanges
#endif
#ifndef KSS_SPREAD_SWEEP_WAVES
#define KSS_SPREAD_SWEEP_WAVES 4  // at most this many waves sweep one exchange (512-lane shards: half)
#endif
#ifndef KSS_SPREAD_MW_MIN
#define KSS_SPREAD_MW_MIN (64 * 4)  // W x values above which every wave sweeps a share (C3: 40 x 13)
#endif
__device__ __forceinline__ bool spread_exchange(SpreadHdr& H, int32_t* xs, unsigned long long* gran_, const XPeers& X,
                                                int W, int wself, int gs,
                                                unsigned epoch, int* err, int K, unsigned opbits, int sum_lo, int ns,
                                                int or_lo, int no, unsigned long long* sp, int gw = 0, int nsw = 1,
                                                int phase = 3, int np = 0, int or2_lo = 0, int no2 = 0) {
  constexpr int XS = G_XS;
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  // np > 0 (spread_argmax_pay): after the bins, np payload values H.payv[] whose fold keeps
  // the value of the shard with the largest key (scalar 0, a compressed key with its top bit
  // flipped so that the signed MAX orders it), into H.pay[] as {key, payload}.
  // no2: a second OR range [or2_lo, + no2) after the first (the fold's early statistics of the
  // next pod ride with this pod's filter exchange: its hard presence in the other bins area)
  const int M0 = K + ns + no + no2, M = M0 + np;
  KSS_GLOBAL unsigned long long* gran = gp(gran_);
  auto slot = [&](int j) -> int32_t* {
    if (j < K) return xs + j;
    if (j < K + ns) return xs + G_NS + sum_lo + (j - K);
    if (j < K + ns + no) return xs + G_NS + or_lo + (j - K - ns);
    if (j < M0) return xs + G_NS + or2_lo + (j - K - ns - no);
    return H.payv + (j - M0);
  };
  auto opof = [&](int j) { return j < K ? (int)((opbits >> (2 * j)) & 3u) : (j < K + ns ? OP_SUM : OP_OR); };
  const unsigned long long tag = (unsigned long long)epoch << 32;
  const size_t mine = ((size_t)(epoch & 1) * W + wself) * gs;
  for (int j = lane; (phase & 1) && j < M; j += 64) {
    int32_t* sl = slot(j);
    const int op = opof(j);
    int32_t v = *sl;
    if (j < K) {  // workgroup value of scalar j: its waves' partials
      v = H.red[0][j];
      for (int x = 1; x < nw; x++) v = op32_lane(op, v, H.red[x][j]);
    }
    xpub(X, gran_, mine + j, tag | (uint32_t)v);
    if (j < M0) *sl = ident32(op);
    else H.pay[j - M0] = 0ull;
  }
  if (sp && lane == 0) sp[2] = wall_clock64();
  if (!(phase & 2)) return true;
  KSS_GLOBAL const unsigned long long* base = gran + (size_t)(epoch & 1) * W * gs;
  const int NL = 64 * nsw, gl = gw * 64 + lane;
  for (int j0 = 0; j0 < M; j0 += NL) {
    const int mc = min(NL, M - j0);
    const int T = NL / mc;  // lanes per value in this chunk
    const int t = gl / mc, j = j0 + (gl - t * mc);
    const bool act = t < T;
    const int op = opof(min(j, M - 1));
    const bool payl = j >= M0;
    // the operator differs between lanes: fold all four, branch-free, and pick one at the end
    int32_t a_sum = 0, a_max = INT32_MIN, a_min = INT32_MAX, a_or = 0;
    uint32_t a_key = 0, a_pay = 0;  // payload lanes: the largest key seen and its shard's payload
    // loads per lane sized to the shards this lane polls (4, 8 or 16), every load issued
    // unconditionally from a clamped address (no exec-mask region per load), the lanes and
    // shards past the end masked in the tag test and the fold
    auto sweep = [&](auto xs_c) -> bool {
      constexpr int XSN = decltype(xs_c)::value;
      const int jc = min(j, M - 1);
      for (int w0 = 0; w0 < W; w0 += T * XSN) {
        unsigned long long g[XSN], gk[XSN];
        long long t0_ = 0;
        for (unsigned spins = 0;; ++spins) {
          bool ok = true;
#pragma unroll
          for (int b = 0; b < XSN; b++) {
            const int w = w0 + t + T * b;
            g[b] = __hip_atomic_load(base + (size_t)min(w, W - 1) * gs + jc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok &= !(act && w < W) || (g[b] >> 32) == epoch;
          }
          if (np && payl) {  // the key granule of the same shards, for the payload lanes
#pragma unroll
            for (int b = 0; b < XSN; b++) {
              const int w = w0 + t + T * b;
              gk[b] = __hip_atomic_load(base + (size_t)min(w, W - 1) * gs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              ok &= !(act && payl && w < W) || (gk[b] >> 32) == epoch;
            }
          }
          if (__all(ok)) break;
          if (spread_spin_over(spins, t0_, err)) {
            if (lane == 0) {
              H.abort = 1;
              err_raise(err, 1);
            }
            return false;
          }
          spin_pause();
        }
        if (sp && lane == 0) sp[3] = wall_clock64();
#pragma unroll
        for (int b = 0; b < XSN; b++) {
          const bool in = w0 + t + T * b < W;
          const int32_t x = (int32_t)(uint32_t)g[b];
          a_sum += in ? x : 0;
          a_max = max(a_max, in ? x : INT32_MIN);
          a_min = min(a_min, in ? x : INT32_MAX);
          a_or |= in ? x : 0;
          if (np) {
            const uint32_t kk = in ? ((uint32_t)gk[b] ^ 0x80000000u) : 0u;
            a_pay = kk > a_key ? (uint32_t)g[b] : a_pay;
            a_key = kk > a_key ? kk : a_key;
          }
        }
      }
      return true;
    };
    const int need = (W + T - 1) / T;  // shards per lane
    const bool swept = need <= 4   ? sweep(std::integral_constant<int, 4>{})
                       : need <= 8 ? sweep(std::integral_constant<int, 8>{})
                                   : sweep(std::integral_constant<int, XS>{});
    if (!swept) return false;
    const int32_t acc = op == OP_SUM ? a_sum : (op == OP_MAX ? a_max : (op == OP_MIN ? a_min : a_or));
    if (act && payl) {
      if (a_key) atomicMax(&H.pay[j - M0], ((unsigned long long)a_key << 32) | a_pay);
    } else if (act) {
      int32_t* sl = slot(j);
      switch (op) {
        case OP_SUM: atomicAdd(sl, acc); break;
        case OP_MAX: atomicMax(sl, acc); break;
        case OP_MIN: atomicMin(sl, acc); break;
        default: atomicOr(sl, acc); break;
      }
    }
  }
  return true;
}

// Wave 0, once the cluster bins are final: criticalPaths[0] of pod q's histogram-valued
// DoNotSchedule groups — the minimum over the present domains, into the scalar xs[i].
__device__ __forceinline__ void hard_minima(const GPod& q, int32_t* xs, const int32_t* bins) {
  const int lane = threadIdx.x & 63;
  for (int i = 0; i < q.n_hard; i++) {
    const GSpread& sp = q.sp[i];
    if (sp.off < 0 || sp.own != i) continue;
    int32_t m[1] = {INT32_MAX};
    for (int b = lane; b < sp.nb; b += 64)
      if (bins[q.total_bins + sp.poff + b]) m[0] = min(m[0], bins[sp.off + b]);
    const int op[1] = {OP_MIN};
    wave_red32(m, op);
    if (lane == 0) xs[i] = min(xs[i], m[0]);
  }
}

// ---- Two-level selectHost exchange (one part, W > 64 shards over the chip's XCDs) -------------
// The flat exchange has every shard poll every shard's granule across XCDs: at C4's 256 shards
// a 3.2 us step (four waves sweep, then an LDS combine).  Two levels instead: each shard stores
// its key with a PLAIN store into its XCD's area (the line stays in that XCD's L2, which the
// polls read: tools/xcd_exchange_probe.hip, 0.41 against 1.23 us a round); the XCD's rank-0
// shard polls its XCD's <= 64 keys with one load per lane, stores their maximum write-through
// (agent scope) into one line per XCD, and every shard polls the <= 16 XCD maxima.  Which XCD
// a shard runs on is read from XCC_ID at the start of the launch (tl_register), never assumed.
// The statistics and filter exchanges (spread_reduce) can take the same two levels when they carry
// at most TL_M values (spread_exchange_tl, option spread_two_level = 2).  Measured slower at C4
// (x_stats 2.17 -> 2.36, x_filter 2.79 -> 3.01 us, 95.7k -> 90.8k pods/s, profiles/r8j_c4_bench.json):
// the flat sweep spreads those values over four waves, the two levels put two dependent hops on
// one wave; off by default.
// Area (8-byte words, X.tl): [0, 16) counters (shards per XCD, [TL_G] all); the argmax: per parity
// TL_G x tl_ls(W) XCD slots, then per parity TL_G lines of 16 words (one XCD maximum each); the
// reductions: per parity TL_G x tl_ls(W) lines of TL_M values (one line per shard), then per
// parity TL_G lines of TL_M values.
constexpr int TL_G = 16;  // XCC ids 0..15
constexpr int TL_M = 16;  // values of a two-level reduction (one 128-byte line)
__host__ __device__ inline int tl_ls(int W) { return (W + 15) / 16 * 16; }
__host__ __device__ inline size_t tl_o_rloc(int W) { return 16 + 2 * (size_t)TL_G * tl_ls(W) + 2 * (size_t)TL_G * 16; }
__host__ __device__ inline size_t tl_o_rglob(int W) { return tl_o_rloc(W) + 2 * (size_t)TL_G * tl_ls(W) * TL_M; }
__host__ __device__ inline size_t tl_words(int W) { return tl_o_rglob(W) + 2 * (size_t)TL_G * TL_M; }

// Thread 0: the shard's XCD and rank there; every shard of the launch registered (bounded wait).
__device__ __forceinline__ void tl_register(SpreadHdr& H, unsigned long long* tl, int W, int* err) {
  int* cnt = reinterpret_cast<int*>(tl);  // [0, TL_G) per XCD, [TL_G] all
  const int x = xcc_id() & (TL_G - 1);
  const int s = atomicAdd(&cnt[x], 1);
  atomicAdd(&cnt[TL_G], 1);
  long long t0 = 0;
  bool ok = false;
  for (unsigned spins = 0;; ++spins) {
    if (__hip_atomic_load(&cnt[TL_G], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= W) {
      ok = true;
      break;
    }
    if (spin_expired(spins, t0)) break;
    __builtin_amdgcn_s_sleep(1);
  }
  uint32_t mask = 0;
  for (int g = 0; g < TL_G; g++)
    mask |= (ok && __hip_atomic_load(&cnt[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > 0) ? 1u << g : 0u;
  H.tl_x = x;
  H.tl_s = s;
  H.tl_n = ok ? __hip_atomic_load(&cnt[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  H.tl_mask = mask;
  if (!ok) err_raise(err, 1);
}

// Wave 0: the cluster maximum of the shards' 32-bit compressed keys (kc) through the two levels.
// False on a timed-out wait (H.abort set).
__device__ __forceinline__ bool tl_argmax(SpreadHdr& H, const XPeers& X, int W, unsigned epoch, uint32_t kc, int* err,
                                          uint32_t& out) {
  const int lane = threadIdx.x & 63;
  const int ls = tl_ls(W);
  const unsigned long long tag = (unsigned long long)epoch << 32;
  unsigned long long* loc = X.tl + 16 + ((size_t)(epoch & 1) * TL_G + H.tl_x) * ls;
  unsigned long long* glob = X.tl + 16 + 2 * (size_t)TL_G * ls + (size_t)(epoch & 1) * TL_G * 16;
  if (lane == 0) asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(loc + H.tl_s), "v"(tag | kc) : "memory");
  if (H.tl_s == 0) {  // the XCD's maximum: its shards' keys from this XCD's L2
    uint32_t m = 0;
    const int n = H.tl_n;
    for (int c0 = 0; c0 < n; c0 += 64) {
      const int s = c0 + lane;
      unsigned long long v = tag;
      long long t0 = 0;
      for (unsigned spins = 0;; ++spins) {
        if (s < n) v = __hip_atomic_load(gp(loc) + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__all((v >> 32) == epoch)) break;
        if (spread_spin_over(spins, t0, err)) {
          if (lane == 0) {
            H.abort = 1;
            err_raise(err, 1);
          }
          return false;
        }
        spin_pause();
      }
      m = max(m, s < n ? (uint32_t)v : 0u);
    }
    m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0xB1, 0xF, 0xF, false));
    m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x4E, 0xF, 0xF, false));
    m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x141, 0xF, 0xF, false));
    m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x140, 0xF, 0xF, false));
    m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x142, 0xA, 0xF, false));
    m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x143, 0xC, 0xF, false));
    m = (uint32_t)__builtin_amdgcn_readlane((int)m, 63);
    if (lane == 0) __hip_atomic_store(gp(glob) + 16 * (size_t)H.tl_x, tag | m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // the XCDs' maxima: lane g polls XCD g's line
  const bool in = lane < TL_G && ((H.tl_mask >> lane) & 1u);
  unsigned long long v = tag;
  long long t0 = 0;
  for (unsigned spins = 0;; ++spins) {
    if (in) v = __hip_atomic_load(gp(glob) + 16 * (size_t)lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__all((v >> 32) == epoch)) break;
    if (spread_spin_over(spins, t0, err)) {
      if (lane == 0) {
        H.abort = 1;
        err_raise(err, 1);
      }
      return false;
    }
    spin_pause();
  }
  uint32_t m = in ? (uint32_t)v : 0u;
  m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0xB1, 0xF, 0xF, false));
  m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x4E, 0xF, 0xF, false));
  m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x141, 0xF, 0xF, false));
  m = max(m, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x140, 0xF, 0xF, false));
  out = (uint32_t)__builtin_amdgcn_readlane((int)m, 15);
  return true;
}

// tl_argmax with payloads (spread_argmax_pay at W > 64, X.tl): wave 0.  Each shard stores one
// line into its XCD's reduction area: word 0 its compressed key kc (0: no candidate), words
// 1..np its payloads H.payv[]; the XCD's rank-0 shard keeps, per word, the value of its shards'
// largest key and stores that line write-through; every shard does the same over the XCDs'
// lines.  Out: the cluster's largest key, H.pay[j] = {key, payload j} of its shard.  The line
// area is the two-level reductions' (tl_o_rloc / tl_o_rglob), on the same epoch sequence.
__device__ __forceinline__ bool tl_argmax_pay(SpreadHdr& H, const XPeers& X, int W, unsigned epoch, uint32_t kc,
                                              int np, int* err, uint32_t& out) {
  const int lane = threadIdx.x & 63;
  const int M = 1 + np;
  const int MP = M <= 4 ? 4 : (M <= 8 ? 8 : 16);
  const int ls = tl_ls(W);
  const unsigned long long tag = (unsigned long long)epoch << 32;
  unsigned long long* loc = X.tl + tl_o_rloc(W) + ((size_t)(epoch & 1) * TL_G + H.tl_x) * ls * TL_M;
  unsigned long long* glob = X.tl + tl_o_rglob(W) + (size_t)(epoch & 1) * TL_G * TL_M;
  const int j = lane & (MP - 1), t = lane / MP, T = 64 / MP;
  const bool jv = j < M;
  if (lane < M) {
    const uint32_t v = lane == 0 ? kc : (uint32_t)H.payv[lane - 1];
    asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(loc + (size_t)H.tl_s * TL_M + lane), "v"(tag | v) : "memory");
  }
  // (key, value) pairs of up to 4 lines per lane, the value of the largest key kept
  auto fold_lines = [&](auto&& addr, auto&& in_of, int n0, int n, uint32_t& a_key, uint32_t& a_val) -> bool {
    for (int s0 = n0; s0 < n; s0 += 4 * T) {
      unsigned long long g[4], gk[4];
      bool in[4];
#pragma unroll
      for (int b = 0; b < 4; b++) in[b] = jv && in_of(s0 + t + T * b);
      long long t0 = 0;
      for (unsigned spins = 0;; ++spins) {
        bool ok = true;
#pragma unroll
        for (int b = 0; b < 4; b++) {
          g[b] = gk[b] = tag;
          if (in[b]) {
            g[b] = __hip_atomic_load(addr(s0 + t + T * b) + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            gk[b] = __hip_atomic_load(addr(s0 + t + T * b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          ok &= ((g[b] >> 32) == epoch) & ((gk[b] >> 32) == epoch);
        }
        if (__all(ok)) break;
        if (spread_spin_over(spins, t0, err)) {
          if (lane == 0) {
            H.abort = 1;
            err_raise(err, 1);
          }
          return false;
        }
        spin_pause();
      }
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const uint32_t k = in[b] ? (uint32_t)gk[b] : 0u;
        a_val = k > a_key ? (uint32_t)g[b] : a_val;
        a_key = k > a_key ? k : a_key;
      }
    }
    for (int o = MP; o < 64; o <<= 1) {
      const uint32_t ok_ = (uint32_t)__shfl_xor((int)a_key, o, 64), ov = (uint32_t)__shfl_xor((int)a_val, o, 64);
      a_val = ok_ > a_key ? ov : a_val;
      a_key = ok_ > a_key ? ok_ : a_key;
    }
    return true;
  };
  if (H.tl_s == 0) {  // the XCD's line: its shards' lines from this XCD's L2
    uint32_t a_key = 0, a_val = 0;
    const int n = H.tl_n;
    if (!fold_lines([&](int s) { return gp(loc) + (size_t)s * TL_M; }, [&](int s) { return s < n; }, 0, n, a_key, a_val))
      return false;
    if (t == 0 && jv)
      __hip_atomic_store(gp(glob) + (size_t)H.tl_x * TL_M + j, tag | (j == 0 ? a_key : a_val), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  uint32_t a_key = 0, a_val = 0;  // every shard: the XCDs' lines
  if (!fold_lines([&](int x) { return gp(glob) + (size_t)x * TL_M; },
                  [&](int x) { return x < TL_G && ((H.tl_mask >> x) & 1u); }, 0, TL_G, a_key, a_val))
    return false;
  if (t == 0 && j >= 1 && jv) H.pay[j - 1] = ((unsigned long long)a_key << 32) | a_val;
  out = (uint32_t)__builtin_amdgcn_readfirstlane((int)a_key);
  return true;
}

// spread_exchange's two-level form (X.tl, M = K + ns + no <= TL_M values, no payload): wave 0.
// Every shard stores its M values as one line into its XCD's area (plain stores: that XCD's L2);
// the XCD's rank-0 shard folds its shards' lines (MP = M rounded up to a power of two lanes per
// shard, 64 / MP shards per load round) and stores the XCD's M values write-through into one
// line; every shard folds the XCDs' lines into xs.  False on a timed-out wait (H.abort set).
__device__ __forceinline__ bool spread_exchange_tl(SpreadHdr& H, int32_t* xs, const XPeers& X, int W, unsigned epoch,
                                                   int* err, int K, unsigned opbits, int sum_lo, int ns, int or_lo,
                                                   int no) {
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const int M = K + ns + no;
  const int MP = M <= 4 ? 4 : (M <= 8 ? 8 : 16);
  auto slot = [&](int j) -> int32_t* {
    if (j < K) return xs + j;
    if (j < K + ns) return xs + G_NS + sum_lo + (j - K);
    return xs + G_NS + or_lo + (j - K - ns);
  };
  auto opof = [&](int j) { return j < K ? (int)((opbits >> (2 * j)) & 3u) : (j < K + ns ? OP_SUM : OP_OR); };
  const int ls = tl_ls(W);
  const unsigned long long tag = (unsigned long long)epoch << 32;
  unsigned long long* loc = X.tl + tl_o_rloc(W) + ((size_t)(epoch & 1) * TL_G + H.tl_x) * ls * TL_M;
  unsigned long long* glob = X.tl + tl_o_rglob(W) + (size_t)(epoch & 1) * TL_G * TL_M;
  const int j = lane & (MP - 1), t = lane / MP, T = 64 / MP;
  const bool jv = j < M;
  const int op = opof(jv ? j : 0);
  if (lane < M) {  // this shard's values (scalars: its waves' partials)
    int32_t v = *slot(lane);
    if (lane < K) {
      v = H.red[0][lane];
      for (int x = 1; x < nw; x++) v = op32_lane(op, v, H.red[x][lane]);
    }
    asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(loc + (size_t)H.tl_s * TL_M + lane), "v"(tag | (uint32_t)v)
                 : "memory");
  }
  auto wait_all = [&](auto&& load, unsigned long long (&g)[4], bool (&in)[4]) -> bool {
    long long t0 = 0;
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int b = 0; b < 4; b++) {
        g[b] = in[b] ? load(b) : tag;
        ok &= (g[b] >> 32) == epoch;
      }
      if (__all(ok)) return true;
      if (spread_spin_over(spins, t0, err)) {
        if (lane == 0) {
          H.abort = 1;
          err_raise(err, 1);
        }
        return false;
      }
      spin_pause();
    }
  };
  if (H.tl_s == 0) {  // the XCD's values: its shards' lines from this XCD's L2
    int32_t acc = ident32(op);
    const int n = H.tl_n;
    for (int s0 = 0; s0 < n; s0 += 4 * T) {
      unsigned long long g[4];
      bool in[4];
#pragma unroll
      for (int b = 0; b < 4; b++) in[b] = jv && s0 + t + T * b < n;
      if (!wait_all([&](int b) { return __hip_atomic_load(gp(loc) + (size_t)(s0 + t + T * b) * TL_M + j, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT); },
                    g, in))
        return false;
#pragma unroll
      for (int b = 0; b < 4; b++)
        if (in[b]) acc = op32_lane(op, acc, (int32_t)(uint32_t)g[b]);
    }
    for (int o = MP; o < 64; o <<= 1) acc = op32_lane(op, acc, __shfl_xor(acc, o, 64));
    if (t == 0 && jv)
      __hip_atomic_store(gp(glob) + (size_t)H.tl_x * TL_M + j, tag | (uint32_t)acc, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  // every shard: the XCDs' lines, 4 * T of them per load round
  int32_t acc = ident32(op);
  for (int g0 = 0; g0 < TL_G; g0 += 4 * T) {
    const uint32_t span = (4 * T >= 32) ? 0xFFFFFFFFu : ((1u << (4 * T)) - 1u);
    if (((H.tl_mask >> g0) & span) == 0) continue;
    unsigned long long g[4];
    bool in[4];
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const int x = g0 + t + T * b;
      in[b] = jv && x < TL_G && ((H.tl_mask >> x) & 1u);
    }
    if (!wait_all([&](int b) { return __hip_atomic_load(gp(glob) + (size_t)(g0 + t + T * b) * TL_M + j, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT); },
                  g, in))
      return false;
#pragma unroll
    for (int b = 0; b < 4; b++)
      if (in[b]) acc = op32_lane(op, acc, (int32_t)(uint32_t)g[b]);
  }
  for (int o = MP; o < 64; o <<= 1) acc = op32_lane(op, acc, __shfl_xor(acc, o, 64));
  if (t == 0 && jv) *slot(j) = acc;
  return true;
}

// Cluster reduction of K int32 scalars v[] (ops[]), plus (W > 1) the cross-shard SUM of
// bins [sum_lo, sum_lo + ns) and OR of [or_lo, or_lo + no) of xs.  local: workgroup only.
// minima_q: the exchange wave then folds pod minima_q's critical-path minima into v (the
// statistics exchange).  LDS-only barriers (the prefetch waves' HBM loads stay in flight).
// False on abort.
template <int K>
__device__ __forceinline__ bool spread_reduce(SpreadHdr& H, int32_t* xs, int W, int w, int gs, unsigned& epoch,
                                              unsigned long long* gran, const XPeers& X, int* err, int32_t (&v)[K],
                                              const int (&ops)[K], int sum_lo = 0, int ns = 0, int or_lo = 0,
                                              int no = 0, bool local = false, unsigned long long* sp = nullptr,
                                              const GPod* minima_q = nullptr, int or2_lo = 0, int no2 = 0, int kx = K) {
  // kx <= K: the scalars exchanged across shards (the pod needs only its first kx; the others hold
  // their operators' identities, which hard_minima then folds into)
  static_assert(K <= G_NS, "too many values");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int32_t r[K];
#pragma unroll
  for (int k = 0; k < K; k++) r[k] = v[k];
  wave_red32(r, ops);
  if (KSS_LANE_RED) {  // lane k writes value k: one LDS store instruction instead of K on lane 0
    if (lane < K) {
      int32_t x = r[0];
#pragma unroll
      for (int k = 1; k < K; k++) x = lane == k ? r[k] : x;
      H.red[wave][lane] = x;
    }
  } else if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; k++) H.red[wave][k] = r[k];
  }
  if (kx < K && threadIdx.x >= kx && threadIdx.x < K) {
    int op = OP_SUM;
#pragma unroll
    for (int q = 0; q < K; q++)
      if (q == (int)threadIdx.x) op = ops[q];
    xs[threadIdx.x] = ident32(op);
  }
  lds_barrier();
  if (sp && threadIdx.x == 0) sp[0] = wall_clock64();
  const bool xchg = W > 1 && !local;
  if (!xchg) {
    if (threadIdx.x < K) {
      const int k = threadIdx.x;
      int op = OP_SUM;
#pragma unroll
      for (int q = 0; q < K; q++)
        if (q == k) op = ops[q];
      int32_t r = H.red[0][k];
      for (int x = 1; x < nw; x++) r = op32(op, r, H.red[x][k]);
      xs[k] = r;
    }
    if (minima_q && wave == 0) hard_minima(*minima_q, xs, xs + G_NS + sum_lo);
    lds_barrier();
  } else {
    unsigned opbits = 0;
#pragma unroll
    for (int k = 0; k < K; k++) opbits |= (unsigned)ops[k] << (2 * k);
    ++epoch;
    if (sp && threadIdx.x == 0) sp[1] = wall_clock64();
    const int KX = W > 1 && !local ? kx : K;
    const int M = KX + ns + no + no2;
    if (X.tl_red && M <= TL_M && no2 == 0) {  // two levels (spread_exchange_tl; option spread_two_level = 2), wave 0
      if (wave == 0 && spread_exchange_tl(H, xs, X, W, epoch, err, KX, opbits, sum_lo, ns, or_lo, no) && minima_q)
        hard_minima(*minima_q, xs, xs + G_NS + sum_lo);
      if (sp && threadIdx.x == 0) sp[4] = wall_clock64();
      lds_barrier();
      if (H.abort) return false;
    } else if (nw == 1 || (long long)W * M <= (long long)KSS_SPREAD_MW_MIN) {  // one polling round for one wave: wave 0 alone
      if (wave == 0 && spread_exchange(H, xs, gran, X, W, w, gs, epoch, err, KX, opbits, sum_lo, ns, or_lo, no, sp, 0, 1, 3,
                                       0, or2_lo, no2) &&
          minima_q)
        hard_minima(*minima_q, xs, xs + G_NS + sum_lo);
      if (sp && threadIdx.x == 0) sp[4] = wall_clock64();
      lds_barrier();
      if (H.abort) return false;
    } else {  // many shards: wave 0 publishes, every wave sweeps a share (fewer polling rounds)
      if (wave == 0)
        spread_exchange(H, xs, gran, X, W, w, gs, epoch, err, KX, opbits, sum_lo, ns, or_lo, no, sp, 0, 1, 1, 0, or2_lo, no2);
      lds_barrier();  // the slots hold the operators' identities before any wave folds into them
      const int nsw = min(nw, KSS_SPREAD_SWEEP_WAVES);  // the sweeping waves (the rest wait)
      if (wave < nsw)
        spread_exchange(H, xs, gran, X, W, w, gs, epoch, err, KX, opbits, sum_lo, ns, or_lo, no, nullptr, wave, nsw, 2, 0,
                        or2_lo, no2);
      lds_barrier();
      if (H.abort) return false;
      if (minima_q && wave == 0) hard_minima(*minima_q, xs, xs + G_NS + sum_lo);
      if (sp && threadIdx.x == 0) sp[4] = wall_clock64();
      lds_barrier();
    }
  }
#pragma unroll
  for (int k = 0; k < K; k++) v[k] = xs[k];  // (k >= kx: the identity, or the folded minimum)
  // no barrier here: the next reduction rewrites xs[0..K) (publish resets, or the local
  // path's stores) only behind its own first barrier, which every wave reaches after reading
  if (KSS_SPREAD_SAFE) lds_barrier();  // experiment: a trailing barrier after every exchange
  return true;
}

// Cluster MAX of the packed selectHost key: one granule {epoch, 32-bit key} per shard when the
// key fits 32 bits (kb > 0, key_bits), else two (lo, hi).
__device__ __forceinline__ bool spread_argmax(SpreadHdr& H, int W, int w, int gs, unsigned& epoch, unsigned long long* gran,
                                              const XPeers& X,
                                              int* err, int parity, long long& key, int kb, int node_base) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const long long r = wave_max_key(key, kb, node_base);
  if (lane == 0) H.kred[parity][wave] = r;
  lds_barrier();
  long long best = H.kred[parity][0];
  for (int x = 1; x < nw; x++) best = H.kred[parity][x] > best ? H.kred[parity][x] : best;
  if (W == 1) {
    key = best;
    return true;
  }
  ++epoch;
  const int ng = kb ? 1 : 2;  // granules per shard
  const uint32_t kc = kb ? key_compress(best, kb, node_base) : 0u;
  if (X.tl && kb) {  // two levels (tl_argmax): wave 0, the other waves wait at the barrier
    if (wave == 0) {
      uint32_t m = 0;
      if (tl_argmax(H, X, W, epoch, kc, err, m) && lane == 0) H.kres = m ? key_expand(m, kb, node_base) : 0;
    }
    lds_barrier();
    if (H.abort) return false;
    key = H.kres;
    return true;
  }
  if (nw > 1 && W > 64) {  // every wave polls a share of the shards, 4 per lane in flight
    const unsigned long long tag = (unsigned long long)epoch << 32;
    if (wave == 0 && lane < ng)
      xpub(X, gran, ((size_t)(epoch & 1) * W + w) * gs + lane,
           tag | (kb ? kc : (lane ? (uint32_t)((unsigned long long)best >> 32) : (uint32_t)best)));
    KSS_GLOBAL const unsigned long long* base = gp(gran) + (size_t)(epoch & 1) * W * gs;
    long long m = 0;
    const int nsw = min(nw, KSS_SPREAD_SWEEP_WAVES);  // the polling waves (the rest add 0)
    const int stride = 64 * nsw;
    for (int c0 = wave * 64; wave < nsw && c0 < W; c0 += 4 * stride) {
      unsigned long long lo[4], hi[4];
      long long t0_ = 0;
      for (unsigned spins = 0;; ++spins) {
        bool ok = true;
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const int s = c0 + lane + b * stride;
          lo[b] = hi[b] = tag;
          if (s < W) {
            lo[b] = __hip_atomic_load(base + (size_t)s * gs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (!kb) hi[b] = __hip_atomic_load(base + (size_t)s * gs + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
#pragma unroll
        for (int b = 0; b < 4; b++) ok &= ((lo[b] >> 32) == epoch) & ((hi[b] >> 32) == epoch);
        if (__all(ok)) break;
        if (spread_spin_over(spins, t0_, err)) {
          if (lane == 0) {
            H.abort = 1;
            err_raise(err, 1);
          }
          break;
        }
        spin_pause();
      }
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const int s = c0 + lane + b * stride;
        const long long k = s >= W ? 0
                            : kb ? (long long)(uint32_t)lo[b]
                                 : (long long)(((hi[b] & 0xFFFFFFFFull) << 32) | (lo[b] & 0xFFFFFFFFull));
        m = k > m ? k : m;
      }
    }
    if (kb) {  // 32-bit keys: one DPP max per step, expanded once
      uint32_t k32 = (uint32_t)m;
      k32 = max(k32, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)k32, 0xB1, 0xF, 0xF, false));
      k32 = max(k32, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)k32, 0x4E, 0xF, 0xF, false));
      k32 = max(k32, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)k32, 0x141, 0xF, 0xF, false));
      k32 = max(k32, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)k32, 0x140, 0xF, 0xF, false));
      k32 = max(k32, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)k32, 0x142, 0xA, 0xF, false));
      k32 = max(k32, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)k32, 0x143, 0xC, 0xF, false));
      m = key_expand((uint32_t)__builtin_amdgcn_readlane((int)k32, 63), kb, node_base);
    } else {
      m = wave_red<OP_MAX>(m);
    }
    if (lane == 0) H.kx[wave] = m;
    lds_barrier();
    if (H.abort) return false;
    long long k = H.kx[0];
    for (int x = 1; x < nw; x++) k = H.kx[x] > k ? H.kx[x] : k;
    key = k;
    return true;
  }
  if (wave == 0) {
    const unsigned long long tag = (unsigned long long)epoch << 32;
    if (lane < ng)
      xpub(X, gran, ((size_t)(epoch & 1) * W + w) * gs + lane,
           tag | (kb ? kc : (lane ? (uint32_t)((unsigned long long)best >> 32) : (uint32_t)best)));
    KSS_GLOBAL const unsigned long long* base = gp(gran) + (size_t)(epoch & 1) * W * gs;
    long long m = 0;
    for (int c0 = 0; c0 < W; c0 += 64) {
      const int s = c0 + lane;
      unsigned long long lo = tag, hi = tag;
      long long t0_ = 0;
      for (unsigned spins = 0;; ++spins) {
        if (s < W) {
          lo = __hip_atomic_load(base + (size_t)s * gs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (!kb) hi = __hip_atomic_load(base + (size_t)s * gs + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (__all(((lo >> 32) == epoch) & ((hi >> 32) == epoch))) break;
        if (spread_spin_over(spins, t0_, err)) {
          if (lane == 0) {
            H.abort = 1;
            err_raise(err, 1);
          }
          break;
        }
        spin_pause();
      }
      const long long k = s >= W ? 0
                          : kb ? key_expand((uint32_t)lo, kb, node_base)
                               : (long long)(((hi & 0xFFFFFFFFull) << 32) | (lo & 0xFFFFFFFFull));
      m = k > m ? k : m;
    }
    m = wave_max_key(m, kb, node_base);
    if (lane == 0) H.kres = m;
  }
  lds_barrier();
  if (H.abort) return false;
  key = H.kres;
  return true;
}

// ---- The statistics exchange of pod k+1 folded into pod k's argmax ----
// Pod k+1's statistics (its PreFilter / PreScore histograms and InterPodAffinity flags) need the
// node state after pod k's AssumePod, which only the argmax decides.  Every shard computes them on
// the state before it (H0) and publishes them with its selectHost key, plus the change its own
// candidate would make if it won (the candidate node's contribution after pod k's commit minus
// before: one (bin, delta) per constraint / entry, and the candidate's flags after the commit);
// the fused sweep sums H0 over the shards and keeps the payloads of the shard with the largest key
// (the winner), which every shard then applies.  Counts only grow on a commit, so the flags are an
// OR.  One exchange per pod fewer on the chain; pods whose DoNotSchedule group is node-valued
// (a critical path over nodes) keep their own exchange (GPod::fold, build_gpods).

// g_sum at slot s as if pod q had been committed there (its resident count rows + 1 each)
__device__ __forceinline__ int32_t g_sum_post(const SpreadShard& L, const GPod& qn, int off, int len, int s, const GPod& q) {
  const uint32_t* R = grefs(qn);
  int32_t v = 0;
  for (int i = 0; i < len; i++) {
    const uint32_t r = R[off + i];
    const int row = (int)(r & 0xFFFFu);
    int32_t c = (int32_t)L.cnt[row * L.cap + s];
    for (int m = 0; m < q.n_cmt; m++) c += q.cmt[m] == row ? 1 : 0;
    v += (int32_t)(int16_t)(r >> 16) * c;
  }
  return v;
}
__device__ __forceinline__ bool g_any_post(const SpreadShard& L, const GPod& qn, int off, int len, int s, const GPod& q) {
  const uint32_t* R = grefs(qn);
  bool a = false;
  for (int i = 0; i < len; i++) {
    const int row = (int)(R[off + i] & 0xFFFFu);
    bool hit = L.cnt[row * L.cap + s] != 0;
    for (int m = 0; m < q.n_cmt; m++) hit |= q.cmt[m] == row;
    a |= hit;
  }
  return a;
}
__device__ __forceinline__ int32_t pay_of(int bin, int32_t delta) {
  return delta == 0 || bin < 0 ? 0 : (int32_t)(((uint32_t)(bin + 1) << 16) | (uint32_t)(uint16_t)(int16_t)delta);
}

// Payload j of candidate slot s (static word wd of pod qn): j < n_hard + n_soft the constraint
// j's histogram delta (stats_node's accumulation), then one per inter-pod entry, the last the
// candidate's InterPodAffinity flags after the commit (only when the pod has inter-pod entries).
__device__ __forceinline__ int32_t fold_payload(const SpreadShard& L, const GPod& q, const GPod& qn, int j, int s,
                                                uint32_t wd) {
  const int cap = L.cap;
  const int nc = qn.n_hard + qn.n_soft;
  if (j < qn.n_hard) {
    const GSpread& sp = qn.sp[j];
    if (sp.own != j || sp.off < 0 || !g_has_keys(L, qn.sp, qn.n_hard, s)) return 0;
    int32_t pre = -1, post = -1;  // the group's last admitting member
    for (int m = j; m < qn.n_hard; m++) {
      const GSpread& mm = qn.sp[m];
      if (mm.own == j && g_policy(mm, wd)) {
        pre = g_sum(L, qn, mm.ri_off, mm.ri_len, s);
        post = g_sum_post(L, qn, mm.ri_off, mm.ri_len, s, q);
      }
    }
    if (pre < 0) return 0;
    return pay_of(sp.off + L.lbl[sp.key * cap + s], post - pre);
  }
  if (j < nc) {
    const GSpread* so = qn.sp + qn.n_hard;
    const GSpread& sp = qn.sp[j];
    if (sp.mode != SOFT_HIST || !g_policy(sp, wd)) return 0;
    if ((qn.pflags & KSS_POD_PTS_REQUIRE_ALL) && !g_has_keys(L, so, qn.n_soft, s)) return 0;
    int d = L.lbl[sp.key * cap + s];
    if (d < 0) d = sp.empty;
    return pay_of(sp.off + d, g_sum_post(L, qn, sp.ri_off, sp.ri_len, s, q) - g_sum(L, qn, sp.ri_off, sp.ri_len, s));
  }
  const bool has_labels = (L.r32[2 * cap + s] & KSS_NODE_HAS_LABELS) != 0;
  if (j < nc + qn.n_ipa) {
    const GIpa& en = qn.ipa[j - nc];
    const int d = L.lbl[en.key * cap + s];
    if (d < 0) return 0;
    int ho;
    if (en.kind == G_SCORE) {
      if (!has_labels) return 0;
      ho = qn.hoff[en.slot][3];
    } else {
      ho = qn.hoff[en.slot][en.kind == KSS_IPA_EXISTING_ANTI ? 0 : (en.kind == KSS_IPA_REQ_AFFINITY ? 1 : 2)];
    }
    if (ho < 0) return 0;
    return pay_of(ho + d, g_sum_post(L, qn, en.ri_off, en.ri_len, s, q) - g_sum(L, qn, en.ri_off, en.ri_len, s));
  }
  int32_t f = 0;  // the flags stats_node would give the candidate after the commit
  for (int e = 0; e < qn.n_ipa; e++) {
    const GIpa& en = qn.ipa[e];
    if (L.lbl[en.key * cap + s] < 0) continue;
    if (en.kind == G_SCORE) {
      if (has_labels && g_any_post(L, qn, en.ri_off, en.ri_len, s, q)) f |= 8;
    } else {
      const int h = en.kind == KSS_IPA_EXISTING_ANTI ? 0 : (en.kind == KSS_IPA_REQ_AFFINITY ? 1 : 2);
      if (g_sum_post(L, qn, en.ri_off, en.ri_len, s, q) > 0) f |= 1 << h;
    }
  }
  return f;
}

// Wave 0, pod qn's statistics final in bins (its cluster histograms after pod q's AssumePod):
// its critical-path minima into H.fmin, its flags into H.fflags (read after the next barrier).
__device__ __forceinline__ void fold_minima(SpreadHdr& H, const GPod& qn, const int32_t* bins, int32_t flags) {
  const int lane = threadIdx.x & 63;
  for (int i = 0; i < qn.n_hard; i++) {
    const GSpread& sp = qn.sp[i];
    int32_t m[1] = {INT32_MAX};
    if (sp.off >= 0 && sp.own == i)
      for (int b = lane; b < sp.nb; b += 64)
        if (bins[qn.total_bins + sp.poff + b]) m[0] = min(m[0], bins[sp.off + b]);
    const int op[1] = {OP_MIN};
    wave_red32(m, op);
    if (lane == 0) H.fmin[i] = m[0];
  }
  if (lane == 0) H.fflags = flags;
}

// spread_argmax for pod q, with the change its winner makes to pod qn's statistics riding along
// (every wave calls it).  qn's statistics on the state before q's AssumePod (H0) were exchanged
// with q's filter exchange into bins_n (flags_n their flags); each shard publishes, beside its
// key, the payloads its candidate would add to them if it won (fold_payload: one (bin, delta) per
// constraint / entry, then the candidate's InterPodAffinity flags after the commit); the sweep
// keeps, per payload value, the value of the shard with the largest key.  On return: key = the
// cluster's best key of q, bins_n hold qn's cluster statistics after q's AssumePod, H.fmin /
// H.fflags qn's critical-path minima and flags.  False on abort.
__device__ __forceinline__ bool spread_argmax_pay(SpreadHdr& H, const SpreadShard& L, int W, int w, int gs,
                                                  unsigned& epoch, unsigned long long* gran, const XPeers& X, int* err,
                                                  int parity, long long& key, int kb, int node_base, int lo,
                                                  const GPod& q, const GPod& qn, int32_t* bins_n, int32_t flags_n,
                                                  const uint32_t* sw1) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int32_t* xs = L.xs;
  const long long r = wave_max_key(key, kb, node_base);
  if (lane == 0) {
    H.kred[parity][wave] = r;
    H.red[wave][0] = (int32_t)(key_compress(r, kb, node_base) ^ 0x80000000u);
  }
  lds_barrier();
  long long best = H.kred[parity][0];
  for (int x = 1; x < nw; x++) best = H.kred[parity][x] > best ? H.kred[parity][x] : best;
  const int np = qn.n_hard + qn.n_soft + qn.n_ipa + (qn.n_ipa > 0 ? 1 : 0);  // + the flags slot
  if (wave == 0) {  // this shard's candidate's payloads (read back by the publishing lanes of this wave)
    const int cs = best ? (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)best) - node_base - lo : -1;
    for (int j = lane; j < np; j += 64) H.payv[j] = cs >= 0 ? fold_payload(L, q, qn, j, cs, sw1[cs]) : 0;
  }
  ++epoch;
  const int K = 1;
  const unsigned opbits = (unsigned)OP_MAX;
  const int M = K + np;
  if (X.tl && M <= TL_M) {  // two levels (tl_argmax_pay): wave 0, the other waves wait at the barrier
    if (wave == 0) {
      uint32_t m = 0;
      if (tl_argmax_pay(H, X, W, epoch, key_compress(best, kb, node_base), np, err, m) && lane == 0)
        xs[0] = (int32_t)(m ^ 0x80000000u);
    }
  } else if (nw == 1 || (long long)W * M <= (long long)KSS_SPREAD_MW_MIN) {
    if (wave == 0) spread_exchange(H, xs, gran, X, W, w, gs, epoch, err, K, opbits, 0, 0, 0, 0, nullptr, 0, 1, 3, np);
  } else {
    if (wave == 0) spread_exchange(H, xs, gran, X, W, w, gs, epoch, err, K, opbits, 0, 0, 0, 0, nullptr, 0, 1, 1, np);
    lds_barrier();  // identities in the slots before any wave folds into them
    const int nsw = min(nw, KSS_SPREAD_SWEEP_WAVES);
    if (wave < nsw) spread_exchange(H, xs, gran, X, W, w, gs, epoch, err, K, opbits, 0, 0, 0, 0, nullptr, wave, nsw, 2, np);
  }
  lds_barrier();
  if (H.abort) return false;
  const uint32_t kc = (uint32_t)xs[0] ^ 0x80000000u;
  if (wave == 0) {  // the winner's payloads, then qn's critical paths over the final bins
    int32_t fl = 0;
    for (int j = lane; j < np; j += 64) {
      const unsigned long long P = H.pay[j];
      const uint32_t p = (uint32_t)P;
      if (!(P >> 32) || !p) continue;
      if (qn.n_ipa > 0 && j == np - 1) fl |= (int32_t)p;
      else atomicAdd(&bins_n[(p >> 16) - 1], (int32_t)(int16_t)(p & 0xFFFFu));
    }
    int32_t f[1] = {fl};
    const int op[1] = {OP_OR};
    wave_red32(f, op);
    fold_minima(H, qn, bins_n, flags_n | f[0]);
  }
  lds_barrier();
  key = key_expand(kc, kb, node_base);
  return true;
}

// A checked hand-off of a shard's node state from one chunk launch to the next: the epilogue
// stores, beside the state, a position-mixed sum of every word it wrote and a tag (the chunk
// sequence number), and a second copy of the state (the shadow); the next chunk's prologue sums
// what it loaded and, while the sums disagree, loads again, alternating between the state and
// its shadow (a bounded number of times, then the launch fails with err = 2 instead of
// scheduling on a wrong state).  The first disagreement of a launch also lists, per differing
// word, the state as a plain agent load, as an atomic and as a nontemporal load sees it, the
// shadow's value and the XCCs of the storing and loading shards (kss_last_handoff_diag).
// hc.sum: [2 W] words {sum, tag} per shard.
constexpr int HANDOFF_DIAG = 64;   // differing words listed per run
constexpr int HANDOFF_DIAG_W = 10;  // words per listed entry
struct HandoffCheck {
  unsigned long long* sum;    // null: no check
  unsigned long long expect;  // tag the previous chunk wrote (0: the first chunk of the call)
  unsigned long long write;   // tag this chunk writes
  int* retries;               // [0] loads repeated because the sums disagreed, [1] loads the shadow answered,
                              // [2] shards whose last write-back failed the final check
  long long* shadow;          // [(6 + n_res) N]: requested x3, nonzero x2, pod count, resident count rows
  int* xcc;                   // [W]: the XCC that ran each shard's last epilogue
  long long* diag;            // [1 + HANDOFF_DIAG * HANDOFF_DIAG_W]: count, then the differing words
};
__device__ __forceinline__ unsigned long long handoff_mix(unsigned long long v, size_t pos) {
  return (v + 0x9E3779B97F4A7C15ull) * (2ull * (unsigned long long)pos + 1ull);
}
// Sum h over the workgroup (scratch: one slot per wave); thread 0 gets it.
__device__ __forceinline__ unsigned long long handoff_sum(unsigned long long h, long long* scratch) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  h = (unsigned long long)wave_red<OP_SUM>((long long)h);
  if (lane == 0) scratch[wave] = (long long)h;
  __syncthreads();
  unsigned long long t = 0;
  for (int x = 0; x < nw; x++) t += (unsigned long long)scratch[x];
  __syncthreads();
  return t;
}
__device__ __forceinline__ void handoff_publish(const HandoffCheck& hc, int w, unsigned long long h, long long* scratch) {
  const unsigned long long t = handoff_sum(h, scratch);
  if (threadIdx.x == 0) {
    st_ag(&hc.sum[2 * (size_t)w], t);
    st_ag(&hc.sum[2 * (size_t)w + 1], hc.write);
    if (hc.xcc) st_ag(&hc.xcc[w], xcc_id());
  }
}
// True when the loaded state matches the previous chunk's sum (or there is nothing to check).
__device__ __forceinline__ bool handoff_verify(const HandoffCheck& hc, int w, unsigned long long h, int attempt,
                                               long long* scratch, int* abort_flag, int* err) {
  const unsigned long long t = handoff_sum(h, scratch);
  if (hc.expect == 0) return true;
  if (threadIdx.x == 0) {
    const unsigned long long tag = ld_ag(&hc.sum[2 * (size_t)w + 1]);
    const bool ok = tag == hc.expect && ld_ag(&hc.sum[2 * (size_t)w]) == t;
    scratch[0] = ok ? 1 : 0;
    if (!ok) {
      __hip_atomic_fetch_add(hc.retries, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (attempt >= 64) {
        *abort_flag = 1;
        err_raise(err, 2);
      }
    }
  }
  __syncthreads();
  const bool ok = scratch[0] != 0;
  __syncthreads();
  if (!ok && !*abort_flag) {
    __builtin_amdgcn_s_sleep(127);
    handoff_acquire();
  }
  return ok;
}
// One differing word of the hand-off (first disagreement of a launch): array a (0-2 requested,
// 3-4 nonzero, 5 pod count, 6 + r resident count row r), node n, and the views of it.
__device__ __forceinline__ void handoff_note(const HandoffCheck& hc, int w, int a, int n, long long plain,
                                             long long atomic_v, long long nt, long long shadow, const void* addr) {
  const long long e = __hip_atomic_fetch_add(hc.diag, 1ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (e >= HANDOFF_DIAG) return;
  long long* d = hc.diag + 1 + e * HANDOFF_DIAG_W;
  st_ag(&d[0], (long long)w | ((long long)xcc_id() << 32) | ((long long)ld_ag(&hc.xcc[w]) << 40));
  st_ag(&d[1], (long long)a);
  st_ag(&d[2], (long long)n);
  st_ag(&d[3], plain);
  st_ag(&d[4], atomic_v);
  st_ag(&d[5], nt);
  st_ag(&d[6], shadow);
  st_ag(&d[7], (long long)hc.expect);
  st_ag(&d[8], (long long)(uintptr_t)addr);
  st_ag(&d[9], (long long)(unsigned)wall_clock64());
}

// The last chunk's write-back, checked after the loop launch has ended (a next chunk's
// prologue checks every other hand-off): shard w's node state in HBM summed as the prologue
// sums it, against the sum and tag its epilogue stored.  A disagreement fails the run (err = 2)
// and counts in retries[2]; nothing is repaired, so no corrupted write-back passes silently.
__device__ __forceinline__ void handoff_final_check(const DevCluster& c, const int32_t* __restrict__ res_rows, int n_res,
                                                    int W, int w, const HandoffCheck& hc, int* err, long long* scratch) {
  const size_t N = (size_t)c.N;
  const int per = (c.N + W - 1) / W;
  const int lo = min(c.N, w * per), hi = min(c.N, lo + per), own = hi - lo, nsc = c.n_scalar;
  // a launch that failed (an exchange timeout) left without its epilogue: nothing to check, and
  // the run already reports why it failed
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  handoff_acquire();
  unsigned long long h = 0;
  for (int s = threadIdx.x; s < own; s += blockDim.x) {
    const int n = lo + s;
#pragma unroll
    for (int k = 0; k < 3; k++) h += handoff_mix((unsigned long long)ld_ag(&c.requested[k * N + n]), (size_t)k * N + n);
    h += handoff_mix((unsigned long long)ld_ag(&c.nonzero[n]), 3 * N + n) +
         handoff_mix((unsigned long long)ld_ag(&c.nonzero[N + n]), 4 * N + n) +
         handoff_mix((unsigned long long)(uint32_t)ld_ag(&c.pod_count[n]), 5 * N + n);
    for (int i = 0; i < nsc; i++)
      h += handoff_mix((unsigned long long)ld_ag(&c.requested[(size_t)(3 + i) * N + n]), (6 + (size_t)n_res + i) * N + n);
  }
  for (int i = threadIdx.x; i < n_res * own; i += blockDim.x) {
    const int r = i / own, s = i - r * own, row = res_rows[r];
    const int32_t v = row < c.n_classes ? ld_ag(&c.class_count[(size_t)row * N + lo + s])
                                        : ld_ag(&c.term_count[(size_t)(row - c.n_classes) * N + lo + s]);
    h += handoff_mix((unsigned long long)(uint32_t)v, (6 + (size_t)r) * N + lo + s);
  }
  const unsigned long long t = handoff_sum(h, scratch);
  if (threadIdx.x == 0) {
    const bool ok = ld_ag(&hc.sum[2 * (size_t)w + 1]) == hc.expect && ld_ag(&hc.sum[2 * (size_t)w]) == t;
    scratch[0] = ok ? 1 : 0;
    if (!ok) {
      __hip_atomic_fetch_add(hc.retries + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      err_raise(err, 2);
      if (hc.diag)  // array -1: {stored tag, stored sum, the sum of the state, the expected tag}
        handoff_note(hc, w, -1, lo, (long long)ld_ag(&hc.sum[2 * (size_t)w + 1]), (long long)ld_ag(&hc.sum[2 * (size_t)w]),
                     (long long)t, (long long)hc.expect, &hc.sum[2 * (size_t)w]);
    }
  }
  __syncthreads();
  if (scratch[0] || !hc.shadow || !hc.diag) return;
  // the words where the state differs from the shadow the epilogue stored beside it
  // (kss_last_handoff_diag), as the prologue's first disagreement lists them
  for (int s = threadIdx.x; s < own; s += blockDim.x) {
    const int n = lo + s;
    for (int a = 0; a < 6; a++) {
      const long long sv = ld_ag(&hc.shadow[(size_t)a * N + n]);
      if (a < 5) {
        int64_t* p = a < 3 ? &c.requested[(size_t)a * N + n] : &c.nonzero[(size_t)(a - 3) * N + n];
        const long long pv = ld_ag(p);
        if (pv != sv)
          handoff_note(hc, w, a, n, pv, __hip_atomic_fetch_add(p, (int64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __builtin_nontemporal_load(p), sv, p);
      } else {
        int32_t* p = &c.pod_count[n];
        const long long pv = ld_ag(p);
        if (pv != sv)
          handoff_note(hc, w, a, n, pv, __hip_atomic_fetch_add(p, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __builtin_nontemporal_load(p), sv, p);
      }
    }
  }
  for (int i = threadIdx.x; i < n_res * own; i += blockDim.x) {
    const int r = i / own, s = i - r * own, row = res_rows[r];
    int32_t* p = row < c.n_classes ? &c.class_count[(size_t)row * N + lo + s]
                                   : &c.term_count[(size_t)(row - c.n_classes) * N + lo + s];
    const long long sv = ld_ag(&hc.shadow[(6 + (size_t)r) * N + lo + s]), pv = ld_ag(p);
    if (pv != sv)
      handoff_note(hc, w, 6 + r, lo + s, pv, __hip_atomic_fetch_add(p, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                   __builtin_nontemporal_load(p), sv, p);
  }
}

// The statistics of node slot s for pod q, accumulated into bins (SUM) / bins + total_bins
// (presence) and hmin / flags: PodTopologySpread calPreFilterState over the DoNotSchedule
// groups, the ScheduleAnyway pair counters (PreScore processAllNode), InterPodAffinity
// PreFilter counts (flags bit0 existing anti, bit1 affinity, bit2 anti) and PreScore
// topologyScore (bit3 non-empty).
__device__ __forceinline__ void stats_node(const SpreadShard& L, const GPod& q, int s, uint32_t wd, int32_t* bins,
                                           int32_t (&hmin)[MAXH], int32_t& flags) {
  const int cap = L.cap;
  if (q.n_hard > 0 && g_has_keys(L, q.sp, q.n_hard, s)) {  // nodeLabelsMatchSpreadConstraints
    for (int i = 0; i < q.n_hard; i++) {
      const GSpread& sp = q.sp[i];
      if (sp.own != i) continue;
      int32_t eff = -1;  // tpCounts[pair]: the count of the group's last member admitting s
      for (int j = i; j < q.n_hard; j++) {
        const GSpread& m = q.sp[j];
        if (m.own == i && g_policy(m, wd)) eff = g_sum(L, q, m.ri_off, m.ri_len, s);
      }
      if (eff < 0) continue;
      if (sp.off < 0) {
        hmin[i] = min(hmin[i], eff);
      } else {
        const int d = L.lbl[sp.key * cap + s];
        atomicAdd(&bins[sp.off + d], eff);
        bins[q.total_bins + sp.poff + d] = 1;  // the pair (key, value) exists
      }
    }
  }
  if (q.n_soft > 0) {
    const GSpread* so = q.sp + q.n_hard;
    if (!(q.pflags & KSS_POD_PTS_REQUIRE_ALL) || g_has_keys(L, so, q.n_soft, s)) {
      for (int i = 0; i < q.n_soft; i++) {
        const GSpread& sp = so[i];
        if (sp.mode != SOFT_HIST || !g_policy(sp, wd)) continue;
        int d = L.lbl[sp.key * cap + s];
        if (d < 0) d = sp.empty;
        const int32_t cnt = g_sum(L, q, sp.ri_off, sp.ri_len, s);  // a group's members share the bins
        if (cnt) atomicAdd(&bins[sp.off + d], cnt);
      }
    }
  }
  if (q.n_ipa > 0) {
    const bool has_labels = (L.r32[2 * cap + s] & KSS_NODE_HAS_LABELS) != 0;
    for (int e = 0; e < q.n_ipa; e++) {
      const GIpa& en = q.ipa[e];
      const int d = L.lbl[en.key * cap + s];
      if (d < 0) continue;
      if (en.kind == G_SCORE) {
        if (!has_labels) continue;
        if (g_any(L, q, en.ri_off, en.ri_len, s)) flags |= 8;
        const int ho = q.hoff[en.slot][3];
        if (ho >= 0) {
          const int32_t v = g_sum(L, q, en.ri_off, en.ri_len, s);
          if (v) atomicAdd(&bins[ho + d], v);
        }
      } else {
        const int32_t v = g_sum(L, q, en.ri_off, en.ri_len, s);
        const int h = en.kind == KSS_IPA_EXISTING_ANTI ? 0 : (en.kind == KSS_IPA_REQ_AFFINITY ? 1 : 2);
        if (v > 0) flags |= 1 << h;
        const int ho = q.hoff[en.slot][h];
        if (ho >= 0 && v) atomicAdd(&bins[ho + d], v);
      }
    }
  }
}

// filter_pts / filter_ipa / ipa_score of kss_sched.cuh over the GPod and the LDS caches.
__device__ __forceinline__ int g_filter_pts(const SpreadShard& L, const GPod& q, const int32_t* bins,
                                            const int32_t (&hard_min)[MAXH], int s, uint32_t w) {
  for (int i = 0; i < q.n_hard; i++) {
    const GSpread& sp = q.sp[i];
    const int d = L.lbl[sp.key * L.cap + s];
    if (d < 0) return 1 + KSS_PTS_MISSING_LABEL;
    int64_t match = 0;  // TpPairToMatchNum[(key, value)]
    if (sp.off >= 0) {
      match = bins[sp.off + d];
    } else if (g_has_keys(L, q.sp, q.n_hard, s)) {  // a node-valued key: the node's own group count
      for (int j = sp.own; j < q.n_hard; j++) {
        const GSpread& m = q.sp[j];
        if (m.own == sp.own && g_policy(m, w)) match = g_sum(L, q, m.ri_off, m.ri_len, s);
      }
    }
    const int64_t skew = match + (int64_t)sp.self_match - (int64_t)hard_min[sp.own];
    if (skew > (int64_t)sp.max_skew) return 1 + KSS_PTS_CONSTRAINTS_NOT_MATCH;
  }
  return 0;
}

// histogram h of key slot k at domain d, or the node's own value for a node-valued key
__device__ __forceinline__ int64_t g_ipa_value(const SpreadShard& L, const GPod& q, const int32_t* bins, int k, int h,
                                               int d, int s) {
  if (q.hoff[k][h] >= 0) return bins[q.hoff[k][h] + d];
  const int kind = h == 0 ? KSS_IPA_EXISTING_ANTI : (h == 1 ? KSS_IPA_REQ_AFFINITY : KSS_IPA_REQ_ANTI);
  int64_t v = 0;
  for (int e = 0; e < q.n_ipa; e++)
    if (q.ipa[e].kind == kind && q.ipa[e].slot == k) v += g_sum(L, q, q.ipa[e].ri_off, q.ipa[e].ri_len, s);
  return v;
}

__device__ __forceinline__ int g_filter_ipa(const SpreadShard& L, const GPod& q, const int32_t* bins, int32_t flags,
                                            int s) {
  // satisfyPodAffinity
  bool have = false, exist = true;
  for (int e = 0; e < q.n_ipa; e++) {
    const GIpa& en = q.ipa[e];
    if (en.kind != KSS_IPA_REQ_AFFINITY) continue;
    have = true;
    const int d = L.lbl[en.key * L.cap + s];
    if (d < 0) return 1 + KSS_IPA_AFFINITY;
    if (g_ipa_value(L, q, bins, en.slot, 1, d, s) <= 0) exist = false;
  }
  if (have && !exist && !(!(flags & 2) && (q.pflags & KSS_POD_IPA_SELF_MATCH))) return 1 + KSS_IPA_AFFINITY;
  // satisfyPodAntiAffinity
  if (flags & 4) {
    for (int e = 0; e < q.n_ipa; e++) {
      const GIpa& en = q.ipa[e];
      if (en.kind != KSS_IPA_REQ_ANTI) continue;
      const int d = L.lbl[en.key * L.cap + s];
      if (d < 0) continue;
      if (g_ipa_value(L, q, bins, en.slot, 2, d, s) > 0) return 1 + KSS_IPA_ANTI_AFFINITY;
    }
  }
  // satisfyExistingPodsAntiAffinity
  if (flags & 1) {
    for (int e = 0; e < q.n_ipa; e++) {
      const GIpa& en = q.ipa[e];
      if (en.kind != KSS_IPA_EXISTING_ANTI) continue;
      const int d = L.lbl[en.key * L.cap + s];
      if (d < 0) continue;
      if (g_ipa_value(L, q, bins, en.slot, 0, d, s) > 0) return 1 + KSS_IPA_EXISTING_ANTI_AFFINITY;
    }
  }
  return 0;
}

// InterPodAffinity.Score: Σ topologyScore[key][node value] over the keys the node has
__device__ __forceinline__ int64_t g_ipa_score(const SpreadShard& L, const GPod& q, const int32_t* bins, int s) {
  int64_t v = 0;
  const bool has_labels = (L.r32[2 * L.cap + s] & KSS_NODE_HAS_LABELS) != 0;
  for (int k = 0; k < q.n_keys; k++) {
    const int d = L.lbl[q.key[k] * L.cap + s];
    if (d < 0) continue;
    if (q.hoff[k][3] >= 0) {
      v += bins[q.hoff[k][3] + d];
    } else if (has_labels) {
      for (int e = 0; e < q.n_ipa; e++) {
        const GIpa& en = q.ipa[e];
        if (en.slot == k && en.kind == G_SCORE) v += g_sum(L, q, en.ri_off, en.ri_len, s);
      }
    }
  }
  return v;
}

#if KSS_SPREAD_TRACE
// trace: stats_node's count of the first hard group at slot s (-1: not counted)
__device__ __forceinline__ int32_t trace_eff(const SpreadShard& L, const GPod& q, int s, uint32_t wd) {
  if (q.n_hard <= 0 || !g_has_keys(L, q.sp, q.n_hard, s)) return -1;
  int32_t eff = -1;
  for (int j = 0; j < q.n_hard; j++)
    if (q.sp[j].own == 0 && g_policy(q.sp[j], wd)) eff = g_sum(L, q, q.sp[j].ri_off, q.sp[j].ri_len, s);
  return eff;
}
#endif

// The batch for shard w of one cluster, pods [k0, k1).  res_rows: the resident count rows
// (class r as r, term r as n_classes + r), n_res of them.  FOLD: the next pod's statistics ride with
// this pod's filter exchange and argmax (spread_argmax_pay).
template <bool DEF, bool FOLD, bool WIN>
__device__ __forceinline__ void spread_schedule(const GTrace& tr, DevCluster c, const GPod* __restrict__ gpods,
                                                const uint32_t* __restrict__ stat, const int32_t* __restrict__ res_rows,
                                                int n_res, int k0, int k1, int32_t* chosen, PodMeta* meta,
                                                const kss_profile& prof, int W, int w, int cap, int bins_cap, int gq, int gs,
                                                unsigned long long* gran, const XPeers& X, unsigned epoch0, int* err,
                                                unsigned long long* stamps, int nst, const HandoffCheck& hc,
                                                long long* smem, int k_find = 0, int32_t* cursor = nullptr) {
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wave = tid >> 6;
  // WIN: nextStartNodeIndex for the launch (every shard holds the same value; shard 0 writes it back)
  int wstart = WIN && cursor && c.N > 0 ? (int)(((long long)ld_ag(cursor) % c.N + c.N) % c.N) : 0;
  SpreadHdr& H = *reinterpret_cast<SpreadHdr*>(smem);
  const SpreadShard L = spread_view(smem, cap, bins_cap, c.n_keys, n_res, gq, c.n_scalar, FOLD);
  const int nsc = c.n_scalar;
  // FOLD: pod j's static words in slot j % 3 (its early statistics pass reads pod k + 1's during
  // pod k) and its bins in area j & 1; otherwise slot j & 1 and one area
  auto st_slot = [](int j) { return FOLD ? j % 3 : j & 1; };
  const int bstride = FOLD ? bins_cap : 0;
  const int kb = key_bits(prof, c.N);  // 32-bit selectHost keys when they fit (0: 64-bit, two granules)
  const size_t N = (size_t)c.N;
  const int per = (c.N + W - 1) / W;
  const int lo = min(c.N, w * per), hi = min(c.N, lo + per), own = hi - lo;
  if (k1 <= k0) return;
  // diagnostic phase stamps (KSS_STAMPS_FILE): s_memrealtime into LDS, copied out at the end
  // (no HBM store on the exchange wave while the loop runs)
  unsigned long long* stl =
      stamps ? reinterpret_cast<unsigned long long*>(reinterpret_cast<uint8_t*>(smem) +
                                                     spread_lds_bytes(cap, bins_cap, c.n_keys, n_res, gq, c.n_scalar, FOLD))
             : nullptr;
  if (stl)
    for (int i = tid; i < 16 * nst; i += nt) stl[i] = 0;
  // shard state -> LDS: node rows, label ids, resident count rows, static words of pod k0,
  // records of pods k0 and k0 + 1
  handoff_acquire();
  for (int s = tid; s < own; s += nt) {  // the rows that never change
    const int n = lo + s;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const int64_t A = c.alloc[k * N + n];
      L.r64[k * cap + s] = (double)A;
      L.inv[k * cap + s] = A > 0 ? 1.0 / (double)A : 0.0;
    }
    L.r32[cap + s] = c.allowed_pods[n];
    L.r32[2 * cap + s] = (int32_t)c.node_flags[n];
    for (int k = 0; k < c.n_keys; k++) L.lbl[k * cap + s] = c.label_value[(size_t)k * N + n];
    for (int i = 0; i < nsc; i++) L.sc[(size_t)i * cap + s] = c.alloc[(size_t)(3 + i) * N + n];
    L.st[st_slot(k0) * cap + s] = ld_ag(&stat[(size_t)lo + s]);
    if (FOLD && k0 + 1 < k1) L.st[st_slot(k0 + 1) * cap + s] = ld_ag(&stat[N + (size_t)lo + s]);
  }
  // node state handed over by the previous chunk: loaded, then checked against the sum its
  // epilogue stored (HandoffCheck); loaded again until they agree, a bounded number of times,
  // odd attempts from the shadow copy
  for (int attempt = 0;; attempt++) {
    const bool shd = hc.shadow && (attempt & 1);
    unsigned long long h = 0;
    for (int s = tid; s < own; s += nt) {
      const int n = lo + s;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        const int64_t R = shd ? ld_ag(&hc.shadow[k * N + n]) : ld_ag(&c.requested[k * N + n]);
        L.r64[(3 + k) * cap + s] = (double)R;
        h += handoff_mix((unsigned long long)R, (size_t)k * N + n);
      }
      const int64_t z0 = shd ? ld_ag(&hc.shadow[3 * N + n]) : ld_ag(&c.nonzero[n]);
      const int64_t z1 = shd ? ld_ag(&hc.shadow[4 * N + n]) : ld_ag(&c.nonzero[N + n]);
      const int32_t pc = shd ? (int32_t)ld_ag(&hc.shadow[5 * N + n]) : ld_ag(&c.pod_count[n]);
      L.r64[6 * cap + s] = (double)z0;
      L.r64[7 * cap + s] = (double)z1;
      L.r32[s] = pc;
      h += handoff_mix((unsigned long long)z0, 3 * N + n) + handoff_mix((unsigned long long)z1, 4 * N + n) +
           handoff_mix((unsigned long long)(uint32_t)pc, 5 * N + n);
      for (int i = 0; i < nsc; i++) {  // extended resources: shadow rows after the count rows
        const size_t a = 6 + (size_t)n_res + i;
        const int64_t v = shd ? ld_ag(&hc.shadow[a * N + n]) : ld_ag(&c.requested[(size_t)(3 + i) * N + n]);
        L.sc[(size_t)(nsc + i) * cap + s] = v;
        h += handoff_mix((unsigned long long)v, a * N + n);
      }
    }
    for (int i = tid; i < n_res * own; i += nt) {
      const int r = i / own, s = i - r * own, row = res_rows[r];
      const int32_t v = shd ? (int32_t)ld_ag(&hc.shadow[(6 + (size_t)r) * N + lo + s])
                            : (row < c.n_classes ? ld_ag(&c.class_count[(size_t)row * N + lo + s])
                                                 : ld_ag(&c.term_count[(size_t)(row - c.n_classes) * N + lo + s]));
      L.cnt[r * cap + s] = (uint16_t)v;
      h += handoff_mix((unsigned long long)(uint32_t)v, (6 + (size_t)r) * N + lo + s);
#if KSS_SPREAD_TRACE
      if (v && tr.list) {
        const int e = atomicAdd(tr.list, 1);
        if (e < G_TLIST) {
          int32_t* E = tr.list + 4 + 4 * (size_t)e;
          E[0] = k0;
          E[1] = row;
          E[2] = lo + s;
          E[3] = v;
        }
      }
#endif
    }
    if (!hc.sum) break;
    if (handoff_verify(hc, w, h, attempt, H.kx, &H.abort, err)) {
      if (shd && tid == 0) __hip_atomic_fetch_add(hc.retries + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    if (H.abort) return;
    if (attempt == 0 && hc.shadow && hc.diag) {  // the words where the state and its shadow differ
      for (int s = tid; s < own; s += nt) {
        const int n = lo + s;
        for (int a = 0; a < 6; a++) {
          const long long sv = ld_ag(&hc.shadow[(size_t)a * N + n]);
          if (a < 5) {
            int64_t* p = a < 3 ? &c.requested[(size_t)a * N + n] : &c.nonzero[(size_t)(a - 3) * N + n];
            const long long pv = ld_ag(p);
            if (pv != sv)
              handoff_note(hc, w, a, n, pv, __hip_atomic_fetch_add(p, (int64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __builtin_nontemporal_load(p), sv, p);
          } else {
            int32_t* p = &c.pod_count[n];
            const long long pv = ld_ag(p);
            if (pv != sv)
              handoff_note(hc, w, a, n, pv, __hip_atomic_fetch_add(p, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __builtin_nontemporal_load(p), sv, p);
          }
        }
      }
      for (int i = tid; i < n_res * own; i += nt) {
        const int r = i / own, s = i - r * own, row = res_rows[r];
        int32_t* p = row < c.n_classes ? &c.class_count[(size_t)row * N + lo + s]
                                       : &c.term_count[(size_t)(row - c.n_classes) * N + lo + s];
        const long long sv = ld_ag(&hc.shadow[(6 + (size_t)r) * N + lo + s]), pv = ld_ag(p);
        if (pv != sv)
          handoff_note(hc, w, 6 + r, lo + s, pv, __hip_atomic_fetch_add(p, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __builtin_nontemporal_load(p), sv, p);
      }
    }
  }
  const uint4* grec = reinterpret_cast<const uint4*>(gpods);
  for (int i = tid; i < min(k1 - k0, 2) * gq; i += nt) {
    const int j = k0 + i / gq;
    L.ring[(j % 3) * gq + i % gq] = grec[(size_t)j * gq + i % gq];
  }
  if (tid == 0) H.abort = 0;
  __syncthreads();  // the first record is in the ring: zero its statistics bins
  if (FOLD) {  // both areas (pods k0 and k0 + 1)
    for (int b = tid; b < 2 * bins_cap; b += nt) L.xs[G_NS + b] = 0;
  } else {
    const GPod& q0 = *reinterpret_cast<const GPod*>(L.ring + (k0 % 3) * gq);
    if (q0.dyn.status == 0 && q0.need_stats)
      for (int b = tid; b < q0.total_bins + q0.total_pbins; b += nt) L.xs[G_NS + b] = 0;
  }
  __syncthreads();
#if KSS_SPREAD_TRACE
  if (tid == 0) {
    int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    tr.words[((size_t)k0 * W + w) * G_TW + GT_XCC] = 16 + (xcc & 0xF);
  }
  {
    const GPod& q0 = *reinterpret_cast<const GPod*>(L.ring + (k0 % 3) * gq);
    int nz = 0;
    if (q0.dyn.status == 0 && q0.need_stats)
      for (int b = tid; b < q0.total_bins + q0.total_pbins; b += nt) nz += L.xs[G_NS + (k0 & 1) * bstride + b] != 0 ? 1 : 0;
    if (nz) atomicAdd(&tr.words[((size_t)k0 * W + w) * G_TW + GT_PRO], nz);
  }
#endif

  KSS_GLOBAL const uint32_t* gstat = gp(stat);
  KSS_GLOBAL const uint4* ggq = gp(grec);
  KSS_GLOBAL int32_t* gchosen = gp(chosen);
  KSS_GLOBAL PodMeta* gmeta = gp(meta);
  KSS_GLOBAL int32_t* gcc = gp(c.class_count);
  KSS_GLOBAL int32_t* gtc = gp(c.term_count);
  const int nwave = nt >> 6;
  const bool pf_wave = nwave == 1 || __builtin_amdgcn_readfirstlane(tid >> 6) >= 1;
  const int pf_lane = nwave == 1 ? tid : tid - 64, pf_n = nwave == 1 ? nt : nt - 64;
  const int pf_per = (own + pf_n - 1) / pf_n;  // <= G_PF (host-checked)
  const int out_tid = nwave == 1 ? 0 : 64;     // the lane that writes outcomes and HBM commits
  uint4 pfq0 = make_uint4(0, 0, 0, 0), pfq1 = pfq0;  // record of pod k+2: uint4 pf_lane and pf_lane + pf_n
  uint32_t pfw[G_PF];
#pragma unroll
  for (int j = 0; j < G_PF; j++) pfw[j] = 0;
  unsigned epoch = epoch0;  // granule tags above every tag an earlier launch left (split grids)
  int kparity = 0;
  bool folded = false;  // this pod's statistics came with the previous pod's exchanges (spread_argmax_pay)
  for (int k = k0; k < k1; k++) {
#define GSTAMP(i)                                                                      \
  do {                                                                                 \
    if (stl && tid == 0 && k - k0 < nst) stl[(k - k0) * 16 + (i)] = wall_clock64();      \
  } while (0)
    GSTAMP(0);
    const GPod& q = *reinterpret_cast<const GPod*>(L.ring + (k % 3) * gq);
    const uint32_t* sw = L.st + st_slot(k) * cap;
    int32_t* bins = L.xs + G_NS + (k & 1) * bstride;  // this pod's histogram / presence bins
    const int boff = (k & 1) * bstride;                // ... as spread_reduce's offsets
    // prefetch (every wave but wave 0): record of pod k+2, static words of pod k+1 (FOLD: k+2).
    // The branch is wave-uniform and the loads inside it unconditional (clamped indices).  A
    // shard without nodes still takes every record: its exchanges follow the programs.
    const int pfs = FOLD ? k + 2 : k + 1;  // the pod whose static words this pod prefetches
    const bool pf_on = pf_wave && k + 1 < k1;
    const bool pfs_on = pf_wave && pfs < k1;
    if (pf_on) {
      if (k + 2 < k1) {
        KSS_GLOBAL const uint4* src = ggq + (size_t)(k + 2) * gq;
        KSS_GLOBAL const uint4& a = src[min(pf_lane, gq - 1)];
        KSS_GLOBAL const uint4& b = src[min(pf_lane + pf_n, gq - 1)];
        pfq0 = make_uint4(a.x, a.y, a.z, a.w);
        pfq1 = make_uint4(b.x, b.y, b.z, b.w);
      }
    }
    if (pfs_on) {
#pragma unroll
      for (int j = 0; j < G_PF; j++)
        if (j < pf_per) pfw[j] = ld_ag(&gstat[(size_t)(pfs - k0) * N + lo + min(j * pf_n + pf_lane, own - 1)]);
    }
    PodMeta m;
    m.chosen = -1;
    m.n_feasible = 0;
    m.scored = 0;
    m.status = 0;
    m.best_total = 0;
    long long best = 0;
    bool evaluated = q.dyn.status == 0;
    if (!evaluated) m.status = q.dyn.status == KSS_PF_ERROR ? 3 : 2;
    int32_t flags = 0, hard_min[MAXH];
#pragma unroll
    for (int i = 0; i < MAXH; i++) hard_min[i] = INT32_MAX;
#if KSS_SPREAD_TRACE
    int32_t* tw = tr.words + ((size_t)k * W + w) * G_TW;
#endif
    // ---- stats: PodTopologySpread PreFilter, InterPodAffinity PreFilter / PreScore ----
    if (KSS_SPREAD_SAFE) lds_barrier();
    if (FOLD && evaluated && folded) {  // the bins already hold the cluster statistics
#pragma unroll
      for (int i = 0; i < MAXH; i++) hard_min[i] = i < q.n_hard ? H.fmin[i] : INT32_MAX;
      flags = H.fflags;
    } else if (evaluated && q.need_stats) {
#if KSS_SPREAD_TRACE == 1
      uint32_t th0 = 0;  // a hash of the first hard group's count per node, read before the pass
      for (int s = tid; s < own; s += nt) th0 = th0 * 31u + (uint32_t)trace_eff(L, q, s, sw[s]) + 7u * (uint32_t)s;
#endif
      // bins zeroed at the end of the previous pod (or in the prologue), behind its barrier
      for (int s = tid; s < own; s += nt) stats_node(L, q, s, sw[s], bins, hard_min, flags);
      GSTAMP(1);
#if KSS_SPREAD_TRACE == 1
      {  // this shard's bins before the exchange; staged inputs against their HBM sources
        lds_barrier();
        const int nbd = min(32, q.total_bins + q.hard_pbins);
        for (int b = tid; b < nbd; b += nt) tw[GT_LOCAL + b] = bins[b];
        int bad_w = 0, bad_r = 0, bad_l = 0;
        uint32_t th1 = 0;
        for (int s2 = tid; s2 < own; s2 += nt) {
          bad_w += sw[s2] != ld_ag(&stat[(size_t)(k - k0) * N + lo + s2]) ? 1 : 0;
          for (int x = 0; x < c.n_keys; x++) bad_l += L.lbl[x * cap + s2] != ld_ag(&c.label_value[(size_t)x * N + lo + s2]) ? 1 : 0;
          th1 = th1 * 31u + (uint32_t)trace_eff(L, q, s2, sw[s2]) + 7u * (uint32_t)s2;
        }
        const uint32_t* rl = reinterpret_cast<const uint32_t*>(L.ring + (k % 3) * gq);
        const uint32_t* rg = reinterpret_cast<const uint32_t*>(grec + (size_t)k * gq);
        for (int i = tid; i < 4 * gq; i += nt) bad_r += rl[i] != ld_ag(&rg[i]) ? 1 : 0;
        if (bad_w) atomicAdd(&tw[GT_BAD_ST], bad_w);
        if (bad_r) atomicAdd(&tw[GT_BAD_REC], bad_r);
        if (bad_l) atomicAdd(&tw[GT_BAD_LBL], bad_l);
        if (th0 != th1) atomicAdd(&tw[GT_REREAD], 1);
      }
#endif
      int32_t v[MAXH + 1];
      const int op[MAXH + 1] = {OP_MIN, OP_MIN, OP_MIN, OP_MIN, OP_OR};
#pragma unroll
      for (int i = 0; i < MAXH; i++) v[i] = hard_min[i];
      v[MAXH] = flags;
      // histogram SUM over every bin, hard-pair presence OR (soft presence, still zero, is
      // filled by the filter pass), then the critical-path minima
      // at more than 64 shards the scalars cross shards only for node-valued DoNotSchedule groups
      // (their minimum over nodes) or inter-pod entries (the flags); histogram groups' minima come
      // from the bins.  C4 (256 shards, zone spread): 8 granules per shard instead of 13, 93.4-94.2k
      // -> 98.4-98.9k pods/s; C3 (32 shards) keeps all five (67.3k against 68.4k in the same A/B,
      // profiles/r9l_stats_scalars_ab.txt)
      bool node_valued = false;
      for (int i = 0; i < q.n_hard; i++) node_valued |= q.sp[i].off < 0;
      if (!spread_reduce(H, L.xs, W, w, gs, epoch, gran, X, err, v, op, boff, q.total_bins, boff + q.total_bins, q.hard_pbins,
                         false, nullptr, &q, 0, 0, W <= 64 || node_valued || q.n_ipa > 0 ? MAXH + 1 : 0))
        return;
#pragma unroll
      for (int i = 0; i < MAXH; i++) hard_min[i] = v[i];
      flags = v[MAXH];
#if KSS_SPREAD_TRACE == 1
      {  // ... and the exchanged bins, minima and flags
        const int nbd = min(32, q.total_bins + q.hard_pbins);
        for (int b = tid; b < nbd; b += nt) tw[GT_XBINS + b] = bins[b];
        if (tid < MAXH + 1) tw[GT_MINIMA + tid] = v[tid];
        if (tid == 0) tw[GT_EPOCH] = (int32_t)epoch;
      }
#endif
      GSTAMP(2);
    }
    // pod k+1: its record, static words and bins area (FOLD: its statistics ride with this pod)
    const GPod& qn = *reinterpret_cast<const GPod*>(L.ring + ((k + 1) % 3) * gq);
    const uint32_t* sw1 = L.st + st_slot(k + 1) * cap;
    int32_t* bins_n = L.xs + G_NS + ((k + 1) & 1) * bstride;
    const int boffn = ((k + 1) & 1) * bstride;
    bool fold_next = false;
    int32_t flags_n = 0;
    // ---- filter + raw scores ----
    const bool has_soft = q.n_soft > 0, has_ipa = q.n_ipa > 0;
    const bool one_soft = q.n_soft == 1;
    const GSpread* soft = q.sp + q.n_hard;
    const uint32_t en = prof.filter_enabled;
    int32_t nf = 0, nign = 0, max_tt = 0, max_na = 0, ipa_min = INT32_MAX, ipa_max = INT32_MIN, smissing = 0;
    int32_t sdirect[MAXS] = {0, 0, 0, 0};
    int32_t cmin = INT32_MAX, cmax = INT32_MIN, lacks = 0;
    // a kept feasible node's part of the filter exchange's statistics (every feasible node; under
    // the window the nodes the search keeps, after the count exchange); returns the node's
    // "ignored" bit (PodTopologySpread PreScore IgnoredNodes)
    auto keep = [&](int s, uint32_t wd, int32_t tt, int32_t na, int64_t ipa) -> int {
      nf++;
      max_tt = tt > max_tt ? tt : max_tt;
      max_na = na > max_na ? na : max_na;
      if (has_ipa) {
        ipa_min = (int32_t)min((int64_t)ipa_min, ipa);
        ipa_max = (int32_t)max((int64_t)ipa_max, ipa);
      }
      if (!has_soft) return 0;
      if ((q.pflags & KSS_POD_PTS_REQUIRE_ALL) && !g_has_keys(L, soft, q.n_soft, s)) {
        nign++;
        return 1;
      }
      for (int i = 0; i < q.n_soft; i++) {
        const GSpread& sp = soft[i];
        int d = L.lbl[sp.key * cap + s];
        if (sp.mode == SOFT_DIRECT) {
          if (d >= 0) sdirect[i]++;
          else smissing |= 1 << i;
        } else if (sp.mode == SOFT_HIST) {
          if (d < 0) d = sp.empty;
          bins[q.total_bins + sp.poff + d] = 1;
        }
      }
      if (one_soft) {  // the count the node's PodTopologySpread raw score is monotone in
        const GSpread& sp = soft[0];
        const int d = L.lbl[sp.key * cap + s];
        int32_t cnt = -1;
        if (d >= 0) {
          if (sp.mode == SOFT_HOST) cnt = g_sum(L, q, sp.ri_off, sp.ri_len, s);
          else if (sp.mode == SOFT_DIRECT) cnt = g_policy(sp, wd) ? g_sum(L, q, sp.ri_off, sp.ri_len, s) : 0;
          else cnt = bins[sp.off + d];
        }
        L.scnt[s] = cnt;
        if (cnt < 0) {
          lacks = 1;
        } else {
          cmin = min(cmin, cnt);
          cmax = max(cmax, cnt);
        }
      }
      return 0;
    };
    // WIN: percentageOfNodesToScore < 100 (findNodesThatPassFilters' window, Parallelism = 1 order
    // from nextStartNodeIndex wstart): the statistics cover the first k_find feasible nodes only
    const bool win = WIN && evaluated && k_find < c.N;
    int it = 0, wstop = -1;  // window: loop iteration; the stopping node (the (k_find + 1)-th feasible)
    if (WIN && win && lane == 0)
      for (int i = 0; i < G_PF; i++) H.wc[i][wave] = H.wb[i][wave] = 0;
    if (evaluated) {
      const SPod qd = q.dyn;  // in registers: the loop's LDS stores would make every field a reload
      for (int s = tid; s < own; s += nt) {
        const uint32_t wd = sw[s];
        DynRow r;
#pragma unroll
        for (int x = 0; x < 3; x++) {
          r.alloc[x] = L.r64[x * cap + s];
          r.req[x] = L.r64[(3 + x) * cap + s];
          r.inv[x] = L.inv[x * cap + s];
        }
        r.nz[0] = L.r64[6 * cap + s];
        r.nz[1] = L.r64[7 * cap + s];
        r.pods = L.r32[s];
        r.allowed = L.r32[cap + s];
        SVal e = DEF ? dyn_eval_def(qd, wd, r) : dyn_eval(prof, qd, wd, r);
        if (nsc && e.f == 0 && ((en >> KSS_F_NODE_RESOURCES_FIT) & 1u) && scalar_short(L.sc, nsc, cap, s, q.dyn, false, q.dyn))
          e.f = KSS_F_NODE_RESOURCES_FIT;
        if (e.f == 0 && ((en >> KSS_F_POD_TOPOLOGY_SPREAD) & 1u) && q.n_hard > 0 &&
            g_filter_pts(L, q, bins, hard_min, s, wd))
          e.f = KSS_F_POD_TOPOLOGY_SPREAD;
        if (e.f == 0 && ((en >> KSS_F_INTER_POD_AFFINITY) & 1u) && has_ipa && g_filter_ipa(L, q, bins, flags, s))
          e.f = KSS_F_INTER_POD_AFFINITY;
        int ign = 0;
        if (WIN && win && e.f == 0) {  // the window: stored, accumulated by the kept pass
          L.stt[s] = e.tt;
          L.sna[s] = e.na;
          L.sfit[s] = e.fit;
          L.sba[s] = e.ba;
          L.sipa[s] = has_ipa ? g_ipa_score(L, q, bins, s) : 0;
        } else if (e.f == 0) {  // (keep()'s accumulation, written out: the default kernel's registers)
          nf++;
          max_tt = e.tt > max_tt ? e.tt : max_tt;
          max_na = e.na > max_na ? e.na : max_na;
          int64_t ipa = 0;
          if (has_ipa) {
            ipa = g_ipa_score(L, q, bins, s);
            ipa_min = (int32_t)min((int64_t)ipa_min, ipa);
            ipa_max = (int32_t)max((int64_t)ipa_max, ipa);
          }
          L.stt[s] = e.tt;
          L.sna[s] = e.na;
          L.sfit[s] = e.fit;
          L.sba[s] = e.ba;
          L.sipa[s] = ipa;
          if (has_soft) {
            if ((q.pflags & KSS_POD_PTS_REQUIRE_ALL) && !g_has_keys(L, soft, q.n_soft, s)) {
              nign++;
              ign = 1;
            } else {
              for (int i = 0; i < q.n_soft; i++) {
                const GSpread& sp = soft[i];
                int d = L.lbl[sp.key * cap + s];
                if (sp.mode == SOFT_DIRECT) {
                  if (d >= 0) sdirect[i]++;
                  else smissing |= 1 << i;
                } else if (sp.mode == SOFT_HIST) {
                  if (d < 0) d = sp.empty;
                  bins[q.total_bins + sp.poff + d] = 1;
                }
              }
              if (one_soft) {  // the count the node's PodTopologySpread raw score is monotone in
                const GSpread& sp = soft[0];
                const int d = L.lbl[sp.key * cap + s];
                int32_t cnt = -1;
                if (d >= 0) {
                  if (sp.mode == SOFT_HOST) cnt = g_sum(L, q, sp.ri_off, sp.ri_len, s);
                  else if (sp.mode == SOFT_DIRECT) cnt = g_policy(sp, wd) ? g_sum(L, q, sp.ri_off, sp.ri_len, s) : 0;
                  else cnt = bins[sp.off + d];
                }
                L.scnt[s] = cnt;
                if (cnt < 0) {
                  lacks = 1;
                } else {
                  cmin = min(cmin, cnt);
                  cmax = max(cmax, cnt);
                }
              }
            }
          }
        }
        L.sf[s] = e.f | (ign << 16);
        if (WIN && win) {  // the window's shard-local prefix: feasible slots per (iteration, wave)
          const unsigned long long bf = __ballot(e.f == 0), bb = __ballot(e.f == 0 && lo + s < wstart);
          if (lane == 0) {
            H.wc[it][wave] = __popcll(bf);
            H.wb[it][wave] = __popcll(bb);
          }
          ++it;
        }
      }
      GSTAMP(3);
      if (WIN && win) {
        // the count exchange: every shard's feasible count (W SUM values behind the pod's bins:
        // this shard's at index w) and the feasible nodes of the start shard before the start node
        lds_barrier();  // the (iteration, wave) counts
        const int nwv = nt >> 6, nit = (own + nt - 1) / nt;
        int32_t cw = 0, cb = 0;
        for (int i = 0; i < nit; i++)
          for (int x = 0; x < nwv; x++) {
            cw += H.wc[i][x];
            cb += H.wb[i][x];
          }
        const int wo = boff + q.total_bins + q.total_pbins;
        for (int x = tid; x < W; x += nt) L.xs[G_NS + wo + x] = x == w ? cw : 0;
        // (only the start shard's: the shards wholly before the start node are parts b entirely)
        int32_t vb[1] = {tid == 0 && w == min(wstart / max(per, 1), W - 1) ? cb : 0};
        const int opb[1] = {OP_SUM};
        if (!spread_reduce(H, L.xs, W, w, gs, epoch, gran, X, err, vb, opb, wo, W, 0, 0, false, nullptr)) return;
        // visiting order: the shards' parts a (nodes >= wstart) in shard order, then their parts b
        if (tid < 64) {
          const int per_ = max(per, 1), ws = min(wstart / per_, W - 1);
          int32_t acc[3] = {0, 0, 0};  // parts a before this shard, all parts a, parts b before this shard
          for (int v = lane; v < W; v += 64) {
            const int32_t cv = L.xs[G_NS + wo + v];
            const int32_t av = v < ws ? 0 : (v == ws ? cv - vb[0] : cv), bv = v < ws ? cv : (v == ws ? vb[0] : 0);
            acc[0] += v < w ? av : 0;
            acc[1] += av;
            acc[2] += v < w ? bv : 0;
          }
          const int op3[3] = {OP_SUM, OP_SUM, OP_SUM};
          wave_red32(acc, op3);
          if (lane == 0) {
            H.wsum[0] = acc[0];
            H.wsum[1] = acc[1];
            H.wsum[2] = acc[2];
          }
        }
        lds_barrier();
        const int32_t a_before = H.wsum[0], a_tot = H.wsum[1], b_before = H.wsum[2];
        // kept pass: Fb(n) = the feasible nodes before n in visiting order; kept iff Fb < k_find,
        // the feasible node with Fb = k_find stops the search (filtered, not kept)
        int pre_w = 0;  // feasible slots of this shard before iteration i's wave
        for (int i = 0; i < nit; i++) {
          int before_i = 0;
          for (int x = 0; x < nwv; x++) before_i += (x < wave ? H.wc[i][x] : 0);
          const int s = tid + i * nt;
          const bool f = s < own && (L.sf[s] & 0xFFFF) == KSS_F_PASS;
          const unsigned long long bf = __ballot(f);
          const int g = pre_w + before_i + __popcll(bf & ((1ull << lane) - 1ull));
          if (f) {
            const int n = lo + s;
            const int fb = n < wstart ? a_tot + b_before + g : a_before + g - cb;
            if (fb < k_find) {
              if (keep(s, sw[s], L.stt[s], L.sna[s], L.sipa[s])) L.sf[s] |= 1 << 16;
            } else {
              L.sf[s] = 0xFFFF;  // filtered and passed, but not in the feasible list
              if (fb == k_find) wstop = n;
            }
          }
          for (int x = 0; x < nwv; x++) pre_w += H.wc[i][x];
        }
#if KSS_SPREAD_TRACE
        if (tid == 0) {
          tw[GT_WIN] = cw;
          tw[GT_WIN + 1] = cb;
          tw[GT_WIN + 2] = vb[0];
          tw[GT_WIN + 3] = a_before;
          tw[GT_WIN + 4] = a_tot;
          tw[GT_WIN + 5] = b_before;
          tw[GT_WIN + 8] = wstart;
        }
        if (wstop >= 0) atomicMax(&tw[GT_WIN + 6], wstop + 1);
        atomicAdd(&tw[GT_WIN + 7], nf);
#endif
      }
      // FOLD: pod k+1's statistics pass on the state before this pod's AssumePod (H0), into its
      // own bins area; they ride with this pod's filter exchange, and the winner's change to them
      // with the argmax (spread_argmax_pay).  Pods whose DoNotSchedule group is node-valued keep
      // their own statistics exchange (GPod::fold, build_gpods).
      if (FOLD) {
        fold_next = W > 1 && kb > 0 && k + 1 < k1 && qn.dyn.status == 0 && qn.need_stats && qn.fold;
        if (fold_next) {
          int32_t hmin_n[MAXH];
#pragma unroll
          for (int i = 0; i < MAXH; i++) hmin_n[i] = INT32_MAX;
          for (int s = tid; s < own; s += nt) stats_node(L, qn, s, sw1[s], bins_n, hmin_n, flags_n);
        }
      }
      // one exchange: feasible count, normalisation maxima, IPA extrema, PTS sizes / extrema.
      // A pod without ScheduleAnyway constraints and inter-pod terms (C4's zone spread) needs
      // only the first three: the other ten stay at their identities on every shard, so they
      // are not exchanged (a quarter of the granules each shard sweeps).
      unsigned long long* est = stl && k - k0 < nst ? stl + (k - k0) * 16 + 10 : nullptr;
      const int nsn = fold_next ? qn.total_bins : 0, non = fold_next ? qn.hard_pbins : 0;  // pod k+1's H0
      if (WIN && !has_soft && !has_ipa) {
        int32_t v[4] = {nf, max_tt, max_na, wstop};
        const int op[4] = {OP_SUM, OP_MAX, OP_MAX, OP_MAX};
        if (!spread_reduce(H, L.xs, W, w, gs, epoch, gran, X, err, v, op, 0, 0, 0, 0, false, est)) return;
        nf = v[0];
        max_tt = v[1];
        max_na = v[2];
        wstop = v[3];
      } else if (!has_soft && !has_ipa) {
        if constexpr (FOLD) {
          int32_t v[4] = {nf, max_tt, max_na, flags_n};
          const int op[4] = {OP_SUM, OP_MAX, OP_MAX, OP_OR};
          if (!spread_reduce(H, L.xs, W, w, gs, epoch, gran, X, err, v, op, boffn, nsn, boffn + qn.total_bins, non, false,
                             est))
            return;
          nf = v[0];
          max_tt = v[1];
          max_na = v[2];
          flags_n = v[3];
        } else {
          int32_t v[3] = {nf, max_tt, max_na};
          const int op[3] = {OP_SUM, OP_MAX, OP_MAX};
          if (!spread_reduce(H, L.xs, W, w, gs, epoch, gran, X, err, v, op, 0, 0, 0, 0, false, est)) return;
          nf = v[0];
          max_tt = v[1];
          max_na = v[2];
        }
      } else {
        constexpr int KV = FOLD || WIN ? 14 : 13;
        int32_t v[KV] = {nf, nign, max_tt, max_na, ipa_min, ipa_max, smissing | (lacks << 30), sdirect[0], sdirect[1],
                         sdirect[2], sdirect[3], cmin, cmax};
        // the 14th scalar: pod k+1's flags (FOLD) or the window's stopping node (WIN; never both);
        // the operators stay a constant array (a written one is a private array in scratch)
        const int op14[14] = {OP_SUM, OP_SUM, OP_MAX, OP_MAX, OP_MIN, OP_MAX, OP_OR, OP_SUM, OP_SUM, OP_SUM, OP_SUM,
                              OP_MIN, OP_MAX, FOLD ? OP_OR : OP_MAX};
        const int(&op)[KV] = *reinterpret_cast<const int(*)[KV]>(op14);
        if (FOLD) v[KV - 1] = flags_n;
        if (WIN) v[KV - 1] = wstop;
        if (!spread_reduce(H, L.xs, W, w, gs, epoch, gran, X, err, v, op, boffn, nsn, boff + q.total_bins + q.hard_pbins,
                           q.total_pbins - q.hard_pbins, false, est, nullptr, boffn + qn.total_bins, non))
          return;
        nf = v[0];
        nign = v[1];
        max_tt = v[2];
        max_na = v[3];
        ipa_min = v[4];
        ipa_max = v[5];
        lacks = (v[6] >> 30) & 1;
        smissing = v[6] & 0xF;
#pragma unroll
        for (int i = 0; i < MAXS; i++) sdirect[i] = v[7 + i];
        cmin = v[11];
        cmax = v[12];
        if (FOLD) flags_n = v[KV - 1];
        if (WIN) wstop = v[KV - 1];
      }
      // nextStartNodeIndex: the stopping node, or unchanged when every node was processed
      if (WIN && win && wstop >= 0) wstart = wstop;
      GSTAMP(4);
      m.n_feasible = nf;
      if (nf == 0) {
        m.status = 1;
        evaluated = false;
        // no AssumePod: pod k+1's exchanged statistics are final
        if (FOLD && fold_next && tid < 64) fold_minima(H, qn, bins_n, flags_n);
      }
    }
    if (evaluated) {
      const bool scored = nf > 1;  // a single feasible node is selected without scoring
      // ---- PodTopologySpread PreScore sizes + Score ----
      long long pts_min = 0, pts_max = 0;
      double wts[MAXS] = {0.0, 0.0, 0.0, 0.0};
      if (scored && has_soft) {
        int32_t sz[MAXS] = {0, 0, 0, 0};
        for (int i = 0; i < q.n_soft; i++) {
          const GSpread& sp = soft[i];
          if (sp.mode != SOFT_HIST || sp.own != q.n_hard + i) continue;
          for (int b = tid; b < sp.nb; b += nt) sz[i] += bins[q.total_bins + sp.poff + b] ? 1 : 0;
        }
        const int ops4[MAXS] = {OP_SUM, OP_SUM, OP_SUM, OP_SUM};
        spread_reduce(H, L.xs, W, w, gs, epoch, gran, X, err, sz, ops4, 0, 0, 0, 0, /*local=*/true);
        for (int i = 0; i < q.n_soft; i++) {
          const GSpread& sp = soft[i];
          long long size;  // topoSize: a group's domains count for its leader only
          if (sp.mode == SOFT_HOST) size = nf - nign;
          else if (sp.own != q.n_hard + i) size = 0;
          else if (sp.mode == SOFT_DIRECT) size = sdirect[i] + ((smissing >> i) & 1);
          else size = sz[i];
          wts[i] = go_log_dev((double)(size + 2));  // topologyNormalizingWeight
        }
        if (one_soft) {  // scoreForCount(cnt) = round(cnt * w + maxSkew - 1) is monotone in cnt
          const double c1 = (double)(soft[0].max_skew - 1);
          pts_min = INT64_MAX;
          if (cmin != INT32_MAX) {
            pts_min = (long long)round((double)cmin * wts[0] + c1);
            pts_max = (long long)round((double)cmax * wts[0] + c1);
          }
          if (lacks) {  // a counted node without the key: raw round(0.0) = 0
            pts_min = pts_min < 0 ? pts_min : 0;
            pts_max = pts_max > 0 ? pts_max : 0;
          }
        } else {
          long long pmin = INT64_MAX, pmax = 0;
          for (int s = tid; s < own; s += nt) {
            const int fi = L.sf[s];
            if ((fi & 0xFFFF) != KSS_F_PASS) continue;
            long long raw = 0;
            if (!(fi >> 16)) {
              double sc = 0.0;
              for (int i = 0; i < q.n_soft; i++) {
                const GSpread& sp = soft[i];
                const int d = L.lbl[sp.key * cap + s];
                if (d < 0) continue;
                int64_t cnt = 0;
                if (sp.mode == SOFT_HOST) {
                  cnt = g_sum(L, q, sp.ri_off, sp.ri_len, s);
                } else if (sp.mode == SOFT_DIRECT) {  // the node's pair counter: every admitting member
                  for (int j = 0; j < q.n_soft; j++)
                    if (soft[j].own == sp.own && g_policy(soft[j], sw[s]))
                      cnt += g_sum(L, q, soft[j].ri_off, soft[j].ri_len, s);
                } else {
                  cnt = bins[sp.off + d];
                }
                const double a = (double)cnt * wts[i];
                sc = sc + (a + (double)(sp.max_skew - 1));  // scoreForCount
              }
              raw = (long long)round(sc);
              pmin = raw < pmin ? raw : pmin;
              pmax = raw > pmax ? raw : pmax;
            }
            L.spts[s] = raw;
          }
          GSTAMP(5);
          // 32-bit extrema: raw scores are host-bounded (spread_bounds_ok)
          int32_t v2[2] = {(int32_t)min(pmin, (long long)INT32_MAX), (int32_t)pmax};
          const int op2[2] = {OP_MIN, OP_MAX};
          if (!spread_reduce(H, L.xs, W, w, gs, epoch, gran, X, err, v2, op2)) return;
          pts_min = v2[0] == INT32_MAX ? INT64_MAX : v2[0];
          pts_max = v2[1];
          GSTAMP(6);
        }
      }
      // ---- NormalizeScore + weights + selectHost ----
      const bool ipa_norm = (flags & 8) != 0;
      const int64_t ipa_diff = (int64_t)ipa_max - (int64_t)ipa_min;
      const float rtt = __builtin_amdgcn_rcpf((float)max(max_tt, 1));
      const float rna = __builtin_amdgcn_rcpf((float)max(max_na, 1));
      for (int s = tid; s < own; s += nt) {
        const int fi = L.sf[s];
        if ((fi & 0xFFFF) != KSS_F_PASS) continue;
        int64_t total = 0;
        if (scored) {
          int64_t nm[KSS_NSCORE];
          // DefaultNormalizeScore(100, reverse=true) / (100, reverse=false); quotients <= 100
          nm[KSS_S_TAINT_TOLERATION] = max_tt == 0 ? 100 : 100 - small_div(100 * L.stt[s], max_tt, rtt);
          nm[KSS_S_NODE_AFFINITY] = max_na != 0 ? small_div(100 * L.sna[s], max_na, rna) : L.sna[s];
          nm[KSS_S_NODE_RESOURCES_FIT] = L.sfit[s];
          nm[KSS_S_VOLUME_BINDING] = 0;
          {  // PodTopologySpread.NormalizeScore
            int64_t raw = 0;
            if (has_soft && !(fi >> 16)) {
              if (one_soft) {
                const int32_t cnt = L.scnt[s];
                raw = cnt < 0 ? 0 : (long long)round((double)cnt * wts[0] + (double)(soft[0].max_skew - 1));
              } else {
                raw = L.spts[s];
              }
            }
            int64_t& pv = nm[KSS_S_POD_TOPOLOGY_SPREAD];
            if (has_soft && (fi >> 16)) pv = 0;
            else if (pts_max == 0) pv = 100;
            else pv = div_i64(100 * (pts_max + pts_min - raw), pts_max);
          }
          nm[KSS_S_INTER_POD_AFFINITY] = L.sipa[s];
          if (ipa_norm) {  // InterPodAffinity.NormalizeScore (skipped when topologyScore is empty)
            double f = 0.0;
            if (ipa_diff > 0) f = 100.0 * ((double)(L.sipa[s] - ipa_min) / (double)ipa_diff);
            nm[KSS_S_INTER_POD_AFFINITY] = (int64_t)f;
          }
          nm[KSS_S_BALANCED_ALLOCATION] = L.sba[s];
          nm[KSS_S_IMAGE_LOCALITY] = 0;
#pragma unroll
          for (int x = 0; x < KSS_NSCORE; x++)
            if ((prof.score_enabled >> x) & 1u) total += nm[x] * (int64_t)prof.weight[x];
        }
        const uint32_t g = (uint32_t)(c.node_base + lo + s);
        const long long key = (long long)(((unsigned long long)(uint32_t)total << 32) | (0xFFFFFFFFull - g));
        best = key > best ? key : best;
      }
      GSTAMP(7);
      if (fold_next ? !spread_argmax_pay(H, L, W, w, gs, epoch, gran, X, err, kparity, best, kb, c.node_base, lo, q, qn,
                                         bins_n, flags_n, sw1)
                    : !spread_argmax(H, W, w, gs, epoch, gran, X, err, kparity, best, kb, c.node_base))
        return;
      GSTAMP(8);
      kparity ^= 1;
#if KSS_SPREAD_TRACE
      if (tid == 0) {  // this shard's view of the selectHost key
        tw[GT_KEY] = (int32_t)(uint32_t)(unsigned long long)best;
        tw[GT_KEY + 1] = (int32_t)(uint32_t)((unsigned long long)best >> 32);
        tw[GT_KEY + 2] = 1;
        tw[GT_NF] = nf;
      }
#endif
      const unsigned long long ub = (unsigned long long)best;
      m.chosen = best ? (int)(0xFFFFFFFFull - (ub & 0xFFFFFFFFull)) : -1;
      m.scored = scored ? 1 : 0;
      m.best_total = scored ? (int64_t)(ub >> 32) : 0;
    }
#if KSS_SPREAD_TRACE
    if (tid == 0) tw[GT_CHOSEN] = m.chosen;
#endif
    // ---- outcome (shard 0) and AssumePod on the winner's shard ----
    const int x = m.chosen >= 0 ? m.chosen - c.node_base : -1;
    const bool won = x >= lo && x < hi;
    if (tid == out_tid) {  // HBM stores off wave 0 (its vmcnt stays free for the exchanges)
      if (w == X.w_off) {  // every part keeps the outcomes
        if (chosen) gchosen[k] = m.chosen;
        if (meta) {
          gmeta[k].chosen = m.chosen;
          gmeta[k].n_feasible = m.n_feasible;
          gmeta[k].scored = m.scored;
          gmeta[k].status = m.status;
          gmeta[k].best_total = m.best_total;
        }
      }
      if (won)
        for (int i = 0; i < q.n_cmt; i++) {
          const int cm = q.cmt[i];
          if (cm >= 0) continue;
          const int row = -1 - cm;
          KSS_GLOBAL int32_t* a = row < c.n_classes ? gcc + (size_t)row * N + x : gtc + (size_t)(row - c.n_classes) * N + x;
          __hip_atomic_fetch_add(a, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
#if KSS_SPREAD_TRACE
    {  // this pod's staged record against HBM (every pod), and the winner's commit
#if KSS_SPREAD_TRACE == 1
      int bad_r = 0;
      const uint32_t* rl = reinterpret_cast<const uint32_t*>(L.ring + (k % 3) * gq);
      const uint32_t* rg = reinterpret_cast<const uint32_t*>(grec + (size_t)k * gq);
      for (int i = tid; i < 4 * gq; i += nt) bad_r += rl[i] != ld_ag(&rg[i]) ? 1 : 0;
      if (bad_r) atomicAdd(&tw[GT_BAD_REC], bad_r);
#endif
      if (won && tid == 0) {
        tw[GT_CMT] = q.n_cmt;
        for (int i = 0; i < q.n_cmt && i < 3; i++) {
          tw[GT_CMT + 1 + 2 * i] = q.cmt[i];
          tw[GT_CMT + 2 + 2 * i] = q.cmt[i] >= 0 ? (int32_t)L.cnt[q.cmt[i] * cap + (x - lo)] : -1;
        }
      }
    }
#endif
    if (KSS_LANE_COMMIT && won && tid < 64) {  // the rows over wave 0's lanes (simple_commit_lanes)
      const int s = x - lo;
      const SPod& pk = q.dyn;
      if (tid < 5) L.r64[(3 + tid) * cap + s] += (&pk.creq[0])[tid];
      if (tid == 5) L.r32[s] += 1;
      if (tid >= 8 && tid < 8 + nsc) L.sc[(size_t)(nsc + tid - 8) * cap + s] += pk.sc_req[tid - 8];
      if (tid == 32)
        for (int i = 0; i < q.n_cmt; i++)
          if (q.cmt[i] >= 0) L.cnt[q.cmt[i] * cap + s] += 1;
    }
    if (!KSS_LANE_COMMIT && won && tid == 0) {
      const int s = x - lo;
      const SPod& pk = q.dyn;
#pragma unroll
      for (int r = 0; r < 3; r++) L.r64[(3 + r) * cap + s] += pk.creq[r];
      L.r64[6 * cap + s] += pk.cnz[0];
      L.r64[7 * cap + s] += pk.cnz[1];
      L.r32[s] += 1;
      for (int i = 0; i < nsc; i++) L.sc[(size_t)(nsc + i) * cap + s] += pk.sc_req[i];
      for (int i = 0; i < q.n_cmt; i++)
        if (q.cmt[i] >= 0) L.cnt[q.cmt[i] * cap + s] += 1;
    }
    // ---- prefetched data of pods k+1 / k+2 -> their LDS slots ----
    if (pf_on && k + 2 < k1) {  // lanes past the end rewrite the last uint4 with its own value
      uint4* dst = L.ring + ((k + 2) % 3) * gq;
      dst[min(pf_lane, gq - 1)] = pfq0;
      dst[min(pf_lane + pf_n, gq - 1)] = pfq1;
    }
    if (pfs_on) {
#pragma unroll
      for (int j = 0; j < G_PF; j++)
        if (j < pf_per) L.st[st_slot(pfs) * cap + min(j * pf_n + pf_lane, own - 1)] = pfw[j];
    }
    // the statistics bins of pod k+1, zeroed ahead of the barrier that ends this pod (its
    // passes no longer read them): its stats pass then starts without a barrier of its own
    // (FOLD: this pod's own area, for pod k+2; pod k+1's area holds its statistics when folded,
    // and was zeroed at the end of pod k-1 when not)
    if (FOLD) {
      for (int b = tid; b < bins_cap; b += nt) bins[b] = 0;
    } else if (k + 1 < k1) {  // (the record again, not qn: a pointer live across the pod costs registers)
      const GPod& qz = *reinterpret_cast<const GPod*>(L.ring + ((k + 1) % 3) * gq);
      if (qz.dyn.status == 0 && qz.need_stats)
        for (int b = tid; b < qz.total_bins + qz.total_pbins; b += nt) bins[b] = 0;
    }
    folded = fold_next;
    lds_barrier();
    GSTAMP(9);
#undef GSTAMP
  }
  // node state and the resident count rows back to HBM
  if (WIN && cursor && w == 0 && tid == 0) *cursor = wstart;  // stream order: the next launch reads it
  __syncthreads();
  if (stl)
    for (int i = tid; i < 16 * nst; i += nt) stamps[(size_t)w * 8 * KSS_NSTAMP_PODS + i] = stl[i];
  for (int s = tid; s < own; s += nt) {
    const int n = lo + s;
#pragma unroll
    for (int r = 0; r < 3; r++) st_ag(&c.requested[(size_t)r * N + n], (int64_t)L.r64[(3 + r) * cap + s]);
    st_ag(&c.nonzero[n], (int64_t)L.r64[6 * cap + s]);
    st_ag(&c.nonzero[N + n], (int64_t)L.r64[7 * cap + s]);
    st_ag(&c.pod_count[n], L.r32[s]);
    if (hc.shadow) {
#pragma unroll
      for (int r = 0; r < 3; r++) st_ag(&hc.shadow[(size_t)r * N + n], (long long)L.r64[(3 + r) * cap + s]);
      st_ag(&hc.shadow[3 * N + n], (long long)L.r64[6 * cap + s]);
      st_ag(&hc.shadow[4 * N + n], (long long)L.r64[7 * cap + s]);
      st_ag(&hc.shadow[5 * N + n], (long long)L.r32[s]);
    }
    for (int i = 0; i < nsc; i++) {
      const int64_t v = L.sc[(size_t)(nsc + i) * cap + s];
      st_ag(&c.requested[(size_t)(3 + i) * N + n], v);
      if (hc.shadow) st_ag(&hc.shadow[(6 + (size_t)n_res + i) * N + n], (long long)v);
    }
  }
  unsigned long long h = 0;
  if (hc.sum)
    for (int s = tid; s < own; s += nt) {
      const int n = lo + s;
#pragma unroll
      for (int k = 0; k < 3; k++) h += handoff_mix((unsigned long long)(int64_t)L.r64[(3 + k) * cap + s], (size_t)k * N + n);
      h += handoff_mix((unsigned long long)(int64_t)L.r64[6 * cap + s], 3 * N + n) +
           handoff_mix((unsigned long long)(int64_t)L.r64[7 * cap + s], 4 * N + n) +
           handoff_mix((unsigned long long)(uint32_t)L.r32[s], 5 * N + n);
      for (int i = 0; i < nsc; i++)
        h += handoff_mix((unsigned long long)L.sc[(size_t)(nsc + i) * cap + s], (6 + (size_t)n_res + i) * N + n);
    }
  for (int i = tid; i < n_res * own; i += nt) {
    const int r = i / own, s = i - r * own, row = res_rows[r];
    const int32_t v = L.cnt[r * cap + s];
    if (row < c.n_classes) st_ag(&c.class_count[(size_t)row * N + lo + s], v);
    else st_ag(&c.term_count[(size_t)(row - c.n_classes) * N + lo + s], v);
    if (hc.shadow) st_ag(&hc.shadow[(6 + (size_t)r) * N + lo + s], (long long)v);
    h += handoff_mix((unsigned long long)(uint32_t)v, (6 + (size_t)r) * N + lo + s);
#if KSS_SPREAD_TRACE
    if (v && tr.list) {
      const int e = atomicAdd(tr.list, 1);
      if (e < G_TLIST) {
        int32_t* E = tr.list + 4 + 4 * (size_t)e;
        E[0] = -1 - k1;
        E[1] = row;
        E[2] = lo + s;
        E[3] = v;
      }
    }
#endif
  }
  if (hc.sum) handoff_publish(hc, w, h, H.kx);
  handoff_release();
}

}  // namespace kss
