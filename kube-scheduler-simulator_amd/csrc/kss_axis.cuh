// kss_axis.cuh — node-axis sharding of one cluster over several GPUs.
//
// Each GPU's context holds a contiguous canonical row range [node_base, node_base + N)
// of the cluster.  One pod is scheduled in three launches on the caller's stream, with
// two small collectives between them that the host issues on the same stream (RCCL
// over xGMI, no host synchronisation):
//
//   k_axis_eval    filter chain + the four raw scores of every local row (HBM-streamed,
//                  one lane per row); folds {feasible count, max TT raw, max NA raw} of
//                  the local rows into stats[0..3) with device atomics.
//   -- all_gather(stats) -> gathered[world][4]
//   k_axis_select  global statistics (Σ feasible, max, max) from gathered, NormalizeScore
//                  + weights + the packed selectHost key (total << 32 | ~global index) of
//                  every local feasible row; the rank's best key is max-folded into key[0].
//   -- all_reduce(key, MAX)
//   k_axis_commit  the owning rank applies AssumePod (commit_pod) to the winner row; every
//                  rank writes chosen[pod] and clears stats / key for the next pod.
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

namespace kss {

constexpr int AXIS_THREADS = 256;
constexpr int AXIS_STATS = 4;  // int64 per rank: feasible count, max TT raw, max NA raw, (reserved)

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

__global__ __launch_bounds__(AXIS_THREADS) void k_axis_eval(DevCluster c, DevPods P, kss_profile prof, int pi,
                                                            int32_t* __restrict__ cv, long long* __restrict__ stats) {
  __shared__ long long red[AXIS_THREADS / 64];
  const kss_pod p = P.pods[pi];
  const size_t N = (size_t)c.N;
  long long nf = 0, tt = 0, na = 0;
  for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < c.N; n += gridDim.x * blockDim.x) {
    int f = KSS_F_NOT_EVALUATED, rt = 0, rn = 0, rf = 0, rb = 0;
    const int64_t g = (int64_t)c.node_base + n;
    bool in = p.prefilter_status == 0;
    if (in && p.names_len >= 0) {  // NodeAffinity PreFilterResult: rows outside the set are not evaluated
      bool hit = false;
      for (int i = 0; i < p.names_len; i++) hit |= (int64_t)P.ints[p.names_off + i] == g;
      in = hit;
    }
    if (in) {
      const NodeRow row = row_from_hbm(c, n);
      uint16_t detail = 0;
      f = filter_local(c, P, p, prof.filter_enabled, n, row, &detail);
      if (f == 0) {
        rt = (int)tt_score(row, p);
        rn = (int)na_score(c, P, p, n);
        rf = (int)fit_score(c, prof, p, n, row);
        rb = (int)ba_score(c, prof, p, n, row);
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
  nf = axis_block_reduce<0>(nf, red);
  tt = axis_block_reduce<1>(tt, red);
  na = axis_block_reduce<1>(na, red);
  if (threadIdx.x == 0) {
    if (nf) atomicAdd((unsigned long long*)&stats[0], (unsigned long long)nf);
    if (tt) atomicMax(&stats[1], tt);
    if (na) atomicMax(&stats[2], na);
  }
}

__device__ __forceinline__ void axis_global(const long long* gathered, int world, long long& nf, long long& tt,
                                            long long& na) {
  nf = 0;
  tt = 0;
  na = 0;
  for (int r = 0; r < world; r++) {
    nf += gathered[r * AXIS_STATS];
    tt = gathered[r * AXIS_STATS + 1] > tt ? gathered[r * AXIS_STATS + 1] : tt;
    na = gathered[r * AXIS_STATS + 2] > na ? gathered[r * AXIS_STATS + 2] : na;
  }
}

__global__ __launch_bounds__(AXIS_THREADS) void k_axis_select(DevCluster c, kss_profile prof,
                                                              const int32_t* __restrict__ cv,
                                                              const long long* __restrict__ gathered, int world,
                                                              long long* __restrict__ key) {
  __shared__ long long red[AXIS_THREADS / 64];
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
  if (threadIdx.x == 0 && best) atomicMax(key, best);
}

// One lane: decode the global winner, commit it on the owning rank, record the outcome,
// clear the fold buffers for the next pod.  meta (optional) receives PodMeta of the pod.
__global__ void k_axis_commit(DevCluster c, DevPods P, int pi, long long* key, const long long* gathered, int world,
                              long long* stats, int32_t* chosen, PodMeta* meta) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const long long K = key[0];
  long long nf, tt, na;
  axis_global(gathered, world, nf, tt, na);
  const int g = K ? (int)(0xFFFFFFFFu - (uint32_t)(unsigned long long)K) : -1;
  const int local = g - c.node_base;
  if (g >= 0 && local >= 0 && local < c.N) commit_pod(c, P, P.pods[pi], local, 1);
  if (chosen) chosen[pi] = g;
  if (meta) {
    const kss_pod& p = P.pods[pi];
    PodMeta m;
    m.chosen = g;
    m.n_feasible = (int32_t)nf;
    m.scored = (K && nf > 1) ? 1 : 0;
    m.status = p.prefilter_status != 0 ? (p.prefilter_status == 1 ? 2 : 3) : (nf == 0 ? 1 : 0);
    m.best_total = m.scored ? (int64_t)((unsigned long long)K >> 32) : 0;
    meta[pi] = m;
  }
  key[0] = 0;
#pragma unroll
  for (int i = 0; i < AXIS_STATS; i++) stats[i] = 0;
}

}  // namespace kss
