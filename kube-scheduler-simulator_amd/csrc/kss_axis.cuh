// kss_axis.cuh — node-axis sharding of one cluster over several GPUs.
//
// Each GPU's context holds a contiguous canonical row range [node_base, node_base + N)
// of the cluster.  One pod is scheduled in three launches on the caller's stream, with
// two small collectives between them that the host issues on the same stream (RCCL
// over xGMI, no host synchronisation):
//
//   k_axis_eval    first the pending AssumePod of the previous pod (the lane owning the
//                  winner row applies it, then reads the row), then the filter chain + the
//                  four raw scores of every local row (HBM-streamed, one lane per row);
//                  folds {feasible count, max TT raw, max NA raw} of the local rows into
//                  stats[0..3) with device atomics.
//   -- all_gather(stats) -> gathered[world][4]
//   k_axis_select  global statistics (Σ feasible, max, max) from gathered, NormalizeScore
//                  + weights + the packed selectHost key (total << 32 | ~global index) of
//                  every local feasible row; the rank's best key is max-folded into key[].
//   -- all_reduce(key, MAX)
//   k_axis_commit  only after the last pod of a batch: its pending AssumePod.
//
// Two launches per pod.  The fold buffers are double-buffered by pod parity: eval(i)
// clears key[i & 1] (select(i) folds into it) and select(i) clears stats[(i + 1) & 1]
// (eval(i + 1) folds into it), so no launch clears a buffer another reads.
//
// The per-row arithmetic is the one k_schedule / k_simple use (kss_eval.cuh, references
// there: fit.go fitsRequest, resource_allocation.go, balanced_allocation.go,
// taint_toleration.go, node_affinity.go); NormalizeScore and the weighted sum follow
// simple_key (framework.go RunScorePlugins, helper/normalize_score.go), and the
// deterministic selectHost tie-break (scheduler/scheduler.go:323-344 with the lowest
// canonical index winning) falls out of the packed key: the MAX over ranks of the
// per-rank maxima is the global maximum.
#pragma once

#include "kss_eval.cuh"
#include "kss_sched.cuh"
#include "kss_simple.cuh"

namespace kss {

constexpr int AXIS_THREADS = 256;
constexpr int AXIS_MAX_KEYS = 8;  // label key columns cached in LDS per tile (more: read from HBM)
constexpr int AXIS_STATS = 4;  // int64 per slot: feasible count, max TT raw, max NA raw, (reserved)
// Fold slots: block b folds into slot b % AXIS_SLOTS, so device-scope atomics on one
// address are AXIS_SLOTS times less contended (one address for the whole grid cost
// ~8 us per launch at 100k rows); readers reduce over the slots.  Per rank the
// statistics are [AXIS_SLOTS][AXIS_STATS] and the key is [AXIS_SLOTS] (MAX all-reduced
// elementwise).
constexpr int AXIS_SLOTS = 32;
static_assert(AXIS_SLOTS == KSS_AXIS_SLOTS && AXIS_STATS == KSS_AXIS_STATS, "kss.h fold layout");
static_assert(AXIS_SLOTS * AXIS_STATS <= AXIS_THREADS, "one block clears a fold buffer");

// per-row results of the current pod, [5][N] int32: verdict, TT, NA, Fit, BA raw
struct AxisRows {
  int32_t* cv;
};

__device__ __forceinline__ long long axis_key(const kss_profile& prof, const int32_t* cv, size_t N, int n, bool scored,
                                              long long max_tt, long long max_na, uint32_t g) {
  int64_t total = 0;
  if (scored) {
    const int64_t rt = cv[N + n], rn = cv[2 * N + n], rf = cv[3 * N + n], rb = cv[4 * N + n];
    const int64_t tt = max_tt == 0 ? 100 : 100 - div_i64(100 * rt, max_tt);
    const int64_t na = max_na != 0 ? div_i64(100 * rn, max_na) : rn;
    const uint32_t se = prof.score_enabled;
    if ((se >> KSS_S_TAINT_TOLERATION) & 1u) total += tt * prof.weight[KSS_S_TAINT_TOLERATION];
    if ((se >> KSS_S_NODE_AFFINITY) & 1u) total += na * prof.weight[KSS_S_NODE_AFFINITY];
    if ((se >> KSS_S_NODE_RESOURCES_FIT) & 1u) total += rf * prof.weight[KSS_S_NODE_RESOURCES_FIT];
    if ((se >> KSS_S_POD_TOPOLOGY_SPREAD) & 1u) total += 100 * (int64_t)prof.weight[KSS_S_POD_TOPOLOGY_SPREAD];
    if ((se >> KSS_S_BALANCED_ALLOCATION) & 1u) total += rb * prof.weight[KSS_S_BALANCED_ALLOCATION];
  }
  return (long long)(((unsigned long long)(uint32_t)total << 32) | (0xFFFFFFFFull - g));
}

// Copy a small record into LDS with all lanes (4-byte words); the caller synchronises.
template <class T>
__device__ __forceinline__ void axis_stage(T* dst, const T* src) {
  static_assert(sizeof(T) % 4 == 0, "record not word-sized");
  const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
  uint32_t* d = reinterpret_cast<uint32_t*>(dst);
  for (int i = threadIdx.x; i < (int)(sizeof(T) / 4); i += blockDim.x) d[i] = s[i];
}

template <int OP>  // 0 sum, 1 max
__device__ __forceinline__ long long axis_block_reduce(long long v, long long* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const long long u = __shfl_xor(v, o, 64);
    v = OP == 0 ? v + u : (u > v ? u : v);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < nw; i++) v = OP == 0 ? v + red[i] : (red[i] > v ? red[i] : v);
  }
  return v;  // valid in thread 0
}

// Wave-cooperative reductions over the fold slots: every lane loads a strided share, then
// a butterfly; all 64 lanes of the wave must be active, and every lane gets the result.
__device__ __forceinline__ long long axis_key_max(const long long* key) {
  const int lane = threadIdx.x & 63;
  long long K = lane < AXIS_SLOTS ? key[lane] : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const long long u = __shfl_xor(K, o, 64);
    K = u > K ? u : K;
  }
  return K;
}

__device__ __forceinline__ int axis_winner(long long K) {
  return K ? (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)K) : -1;
}

__device__ __forceinline__ void axis_global(const long long* gathered, int world, long long& nf, long long& tt,
                                            long long& na) {
  const int lane = threadIdx.x & 63;
  nf = 0;
  tt = 0;
  na = 0;
  for (int r = lane; r < world * AXIS_SLOTS; r += 64) {
    nf += gathered[r * AXIS_STATS];
    tt = gathered[r * AXIS_STATS + 1] > tt ? gathered[r * AXIS_STATS + 1] : tt;
    na = gathered[r * AXIS_STATS + 2] > na ? gathered[r * AXIS_STATS + 2] : na;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    nf += __shfl_xor(nf, o, 64);
    const long long t = __shfl_xor(tt, o, 64), a = __shfl_xor(na, o, 64);
    tt = t > tt ? t : tt;
    na = a > na ? a : na;
  }
}

// chosen[pi] and the PodMeta of pod pi from its reduced key and gathered statistics.
__device__ __forceinline__ void axis_record(const DevPods& P, int pi, long long K, long long nf, int32_t* chosen,
                                            PodMeta* meta) {
  const int g = axis_winner(K);
  if (chosen) chosen[pi] = g;
  if (meta) {
    const kss_pod& p = P.pods[pi];
    PodMeta m;
    m.chosen = g;
    m.n_feasible = (int32_t)nf;
    m.scored = (K && nf > 1) ? 1 : 0;
    m.status = p.prefilter_status != 0 ? (p.prefilter_status == KSS_PF_ERROR ? 3 : 2) : (nf == 0 ? 1 : 0);
    m.best_total = m.scored ? (int64_t)((unsigned long long)K >> 32) : 0;
    meta[pi] = m;
  }
}

// The pod record is indexed with runtime resource ids: staged in LDS, not copied per lane
// (a by-value copy lands in scratch, 392 B per lane).  DEF: the v1.26 default profile is
// folded into the code (no scratch); otherwise the profile is staged in LDS too.
template <bool DEF>
__global__ __launch_bounds__(AXIS_THREADS) void k_axis_eval(DevCluster c, DevPods P, kss_profile prof_arg, int pi,
                                                            int32_t* __restrict__ cv, long long* __restrict__ stats,
                                                            const long long* __restrict__ prev_key,
                                                            const long long* __restrict__ prev_gathered, int world,
                                                            long long* __restrict__ key_zero,
                                                            int32_t* __restrict__ chosen, PodMeta* __restrict__ meta,
                                                            int no_fold) {
  // pending commit of pod pi - 1 (its key was all-reduced after the previous select)
  const long long prevK = prev_key ? axis_key_max(prev_key) : 0;
  const int win = prev_key ? axis_winner(prevK) - c.node_base : -1;
  if (blockIdx.x == 0) {
    if (prev_key && threadIdx.x < 64) {
      long long pnf, ptt, pna;
      axis_global(prev_gathered, world, pnf, ptt, pna);
      if (threadIdx.x == 0) axis_record(P, pi - 1, prevK, pnf, chosen, meta);
    }
    if (threadIdx.x < AXIS_SLOTS) key_zero[threadIdx.x] = 0;  // the buffer k_axis_select folds pod pi's key into
  }
  __shared__ long long red[AXIS_THREADS / 64];
  __shared__ kss_pod p;
  __shared__ kss_profile prof_lds;
  __shared__ int32_t lbl[AXIS_MAX_KEYS * AXIS_THREADS];  // label value ids of the tile's rows
  constexpr kss_profile prof_def = default_profile_c();
  const kss_profile& prof = DEF ? prof_def : prof_lds;
  const size_t N = (size_t)c.N;
  const bool lcache = c.n_keys <= AXIS_MAX_KEYS;
  bool staged = false;
  long long nf = 0, tt = 0, na = 0;
  // one row per lane per tile; the row, its labels and the pod record are all requested
  // before the barrier, so the launch pays one memory round trip before the arithmetic
  for (int base = blockIdx.x * AXIS_THREADS; base < c.N; base += gridDim.x * AXIS_THREADS) {
    const int n = base + (int)threadIdx.x;
    const bool valid = n < c.N;
    NodeRow row{};
    if (valid) row = row_from_hbm(c, n);
    if (lcache)
      for (int k = 0; k < c.n_keys; k++) lbl[k * AXIS_THREADS + threadIdx.x] = valid ? c.label_value[k * N + n] : -1;
    if (!staged) {
      axis_stage(&p, &P.pods[pi]);
      if (!DEF) axis_stage(&prof_lds, &prof_arg);
      staged = true;
    }
    __syncthreads();
    DevCluster cc = c;  // label_of reads the tile's LDS copy
    if (lcache) {
      cc.ncl = lbl;
      cc.nc_cap = AXIS_THREADS;
      cc.nc_lo = base;
    }
    if (valid) {
      int f = KSS_F_NOT_EVALUATED, rt = 0, rn = 0, rf = 0, rb = 0;
      const int64_t g = (int64_t)c.node_base + n;
      bool in = p.prefilter_status == 0;
      if (in && p.names_len >= 0) {  // NodeAffinity PreFilterResult: rows outside the set are not evaluated
        bool hit = false;
        for (int i = 0; i < p.names_len; i++) hit |= (int64_t)P.ints[p.names_off + i] == g;
        in = hit;
      }
      if (n == win) {  // AssumePod of the previous pod, then this lane re-reads its row
        commit_pod(c, P, P.pods[pi - 1], n, 1);
        row = row_from_hbm(c, n);
      }
      if (in) {
        uint16_t detail = 0;
        f = filter_local(cc, P, p, prof.filter_enabled, n, row, &detail);
        if (f == 0) {
          rt = (int)tt_score(row, p);
          rn = (int)na_score(cc, P, p, n);
          rf = (int)fit_score(cc, prof, p, n, row);
          rb = (int)ba_score(cc, prof, p, n, row);
          nf++;
          tt = rt > tt ? rt : tt;
          na = rn > na ? rn : na;
        }
      }
      cv[n] = f;
      cv[N + n] = rt;
      cv[2 * N + n] = rn;
      cv[3 * N + n] = rf;
      cv[4 * N + n] = rb;
    }
    __syncthreads();  // the next tile overwrites lbl
  }
  nf = axis_block_reduce<0>(nf, red);
  tt = axis_block_reduce<1>(tt, red);
  na = axis_block_reduce<1>(na, red);
  if (threadIdx.x == 0 && !no_fold) {
    long long* sl = stats + (blockIdx.x % AXIS_SLOTS) * AXIS_STATS;
    if (nf) atomicAdd((unsigned long long*)&sl[0], (unsigned long long)nf);
    if (tt) atomicMax(&sl[1], tt);
    if (na) atomicMax(&sl[2], na);
  }
}

__global__ __launch_bounds__(AXIS_THREADS) void k_axis_select(DevCluster c, kss_profile prof_arg,
                                                              const int32_t* __restrict__ cv,
                                                              const long long* __restrict__ gathered, int world,
                                                              long long* __restrict__ key,
                                                              long long* __restrict__ stats_zero) {
  if (blockIdx.x == 0 && threadIdx.x < AXIS_SLOTS * AXIS_STATS) stats_zero[threadIdx.x] = 0;  // the next pod's fold buffer
  __shared__ long long red[AXIS_THREADS / 64];
  __shared__ kss_profile prof;
  axis_stage(&prof, &prof_arg);
  __syncthreads();
  long long nf, tt, na;
  axis_global(gathered, world, nf, tt, na);
  const size_t N = (size_t)c.N;
  long long best = 0;
  for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < c.N; n += gridDim.x * blockDim.x) {
    if (cv[n] != 0) continue;
    const long long k = axis_key(prof, cv, N, n, nf > 1, tt, na, (uint32_t)(c.node_base + n));
    best = k > best ? k : best;
  }
  best = axis_block_reduce<1>(best, red);
  if (threadIdx.x == 0 && best) atomicMax(&key[blockIdx.x % AXIS_SLOTS], best);
}

// One lane: the pending commit of the last pod of a batch (k_axis_eval applies every
// other pod's commit at the start of the next pod) and its outcome.
__global__ void k_axis_commit(DevCluster c, DevPods P, int pi, const long long* key, const long long* gathered,
                              int world, int32_t* chosen, PodMeta* meta) {
  if (blockIdx.x != 0) return;
  const long long K = axis_key_max(key);  // the whole wave
  long long nf, tt, na;
  axis_global(gathered, world, nf, tt, na);
  if (threadIdx.x != 0) return;
  const int local = axis_winner(K) - c.node_base;
  if (K && local >= 0 && local < c.N) commit_pod(c, P, P.pods[pi], local, 1);
  axis_record(P, pi, K, nf, chosen, meta);
}

}  // namespace kss
