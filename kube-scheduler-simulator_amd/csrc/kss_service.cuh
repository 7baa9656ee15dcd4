// kss_service.cuh — the per-pod drop-in path as a persistent service grid (kss_service_*).
//
// The Go plugin drives the evaluator one pod at a time (wrappedPlugin.PreFilter ->
// evaluate, Reserve -> AssumePod, Unreserve -> ForgetPod: simulator/scheduler/plugin/
// wrappedplugin.go:491-518, 616-645).  A launch per call costs a kernel dispatch, an
// occupancy query and a stream synchronisation; here one k_schedule-shaped grid stays
// resident and takes commands from a ring in pinned host memory instead:
//
//   host: writes command k into ring[k % SVC_RING] as two 64-bit words, each tagged k + 1
//         in its upper half (the data is the flag: no separate head word to read)
//   shard 0: polls ring[k] (system scope, both words in flight), relays command k into a
//            tagged device-memory slot (agent scope, same format) and reports consumed = k + 1
//   every shard: polls the relay slot, runs the command:
//     EVAL      schedule_pod (kss_sched.cuh) into the HBM record slot, then copies its own
//               node range of the requested record fields into the pinned host record,
//               fences at system scope and stores done[w] = k + 1 (| SVC_DONE_OVF when a
//               compact record value did not fit); a SIMPLE grid (staged default-profile
//               pods) runs svc_simple_eval instead: the k_simple chain, record rows stored
//               from registers
//     COMMIT / ROLLBACK   the owning shard applies AssumePod / ForgetPod (commit_pod)
//     STOP      leave (after writing the LDS node cache back)
//
// Every wait is bounded by wall time: shard 0 relays STOP after SVC_IDLE_TICKS without a
// command (the grid drains by itself; the host restarts it on the next call from
// `consumed`), the other shards leave after 4x that without a relay, and an exchange
// timeout inside a pod aborts with the error word set.
#pragma once
#include <type_traits>

#include "kss_sched.cuh"

namespace kss {

constexpr int SVC_RING = 1024;                                 // host command ring (entries)
constexpr int SVC_DRING = 64;                                  // device relay ring (entries)
constexpr int SVC_MAX_SHARDS = 256;
constexpr unsigned long long SVC_IDLE_TICKS = 100000000ull;    // 1 s of s_memrealtime (100 MHz)
constexpr unsigned long long SVC_DONE_OVF = 1ull << 62;         // done word: a compact value overflowed
enum { SVC_NONE = 0, SVC_EVAL = 1, SVC_COMMIT = 2, SVC_ROLLBACK = 3, SVC_STOP = 4 };

// A command as two tagged words: w0 = (k+1) << 32 | pod << 8 | fields << 3 | op,
// w1 = (k+1) << 32 | node.
struct SvcCmd {
  unsigned long long w0, w1;
};
__host__ __device__ inline unsigned long long svc_w0(unsigned long long k, int op, int fields, int pod) {
  return ((k + 1) << 32) | ((unsigned long long)(uint32_t)pod << 8) | ((unsigned long long)(fields & 31) << 3) |
         (unsigned long long)(op & 7);
}
__host__ __device__ inline unsigned long long svc_w1(unsigned long long k, int node) {
  return ((k + 1) << 32) | (unsigned long long)(uint32_t)node;
}

// Pinned, coherent host memory shared with the grid.
struct SvcBox {
  SvcCmd cmd[SVC_RING];
  unsigned long long consumed;  // commands relayed by shard 0 (device)
  unsigned long long stamp[8];  // diagnostics (kss_service stamps): shard 0's clock at each phase of the last EVAL
  unsigned long long done[SVC_MAX_SHARDS];  // per shard: 1 + the last EVAL finished
  PodMeta meta;                 // outcome of the last EVAL (shard 0)
  int32_t err;                  // an exchange timed out
  int32_t running;              // 1 while the grid runs (shard 0)
  int32_t xcd_fail;             // an XCD-local launch found fewer workgroups on XCD 0 than shards
  int32_t pad;
};

// Every access to the pinned box and to the relay goes through address-space-1 pointers
// (global loads / stores: no flat address-space test on the polled words).
__device__ __forceinline__ void st_sys(KSS_GLOBAL unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The record as SVC_ROWS rows of one element per node: fail, detail, total, raw[KSS_NSCORE],
// norm[KSS_NSCORE].
constexpr int SVC_ROWS = 3 + 2 * KSS_NSCORE;
__device__ __forceinline__ int svc_row_field(int r) {
  return r == 0 ? KSS_FIELD_FAIL : r == 1 ? KSS_FIELD_DETAIL : r == 2 ? KSS_FIELD_TOTAL : r < 3 + KSS_NSCORE ? KSS_FIELD_RAW
                                                                                                           : KSS_FIELD_NORM;
}
// record row r: its field's byte offset in a record of N nodes, the row within the field and
// the element size
__device__ __forceinline__ size_t svc_field(const SlotLayout& L, int r, int& fr, int& es) {
  fr = 0;
  if (r == 0) return es = 1, L.fail;
  if (r == 1) return es = 2, L.detail;
  es = 8;
  if (r == 2) return L.total;
  if (r < 3 + KSS_NSCORE) return fr = r - 3, L.raw;
  return fr = r - 3 - KSS_NSCORE, L.norm;
}
__device__ __forceinline__ size_t svc_row_off(const SlotLayout& L, size_t N, int r, int& es) {
  int fr = 0;
  const size_t o = svc_field(L, r, fr, es);
  return o + (size_t)es * (size_t)fr * N;
}

// Row r of the record as one copy job: source (HBM slot, int64 score rows) and destination
// (pinned host record, full or compact) element sizes, field byte offsets and the row's first
// element (row r of a field starts at element fr * N).  Destination stores carry V elements:
// 16 bytes, except the compact uint8 rows (4 bytes: V = 4, so that a store's source is at
// most 32 bytes — two 16-byte loads — for every row).
struct SvcRow {
  size_t so, dof, e0;
  int es, ed, V;
};
template <bool COMPACT>
__device__ __forceinline__ SvcRow svc_row(const SlotLayout& L, const CompactLayout& CL, size_t N, int r) {
  int fr = 0, es = 0;
  SvcRow x;
  x.so = svc_field(L, r, fr, es);
  x.es = es;
  x.e0 = (size_t)fr * N;
  if (!COMPACT) {
    x.dof = x.so;
    x.ed = es;
  } else {
    x.dof = r == 0 ? CL.fail : r == 1 ? CL.detail : r == 2 ? CL.total : r < 3 + KSS_NSCORE ? CL.raw : CL.norm;
    x.ed = r == 0 ? 1 : r == 1 ? 2 : r < 3 + KSS_NSCORE ? 4 : 1;
  }
  x.V = (COMPACT && r >= 3 + KSS_NSCORE) ? 4 : 16 / x.ed;
  return x;
}

// One element of row x: source value (zero-extended) -> destination (narrowed when compact)
__device__ __forceinline__ uint64_t svc_ld(const uint8_t* src, const SvcRow& x, size_t e) {
  KSS_GLOBAL const uint8_t* p = gp(src) + x.so + e * (size_t)x.es;
  return x.es == 1 ? *p : x.es == 2 ? *reinterpret_cast<KSS_GLOBAL const uint16_t*>(p)
                                    : *reinterpret_cast<KSS_GLOBAL const uint64_t*>(p);
}
__device__ __forceinline__ void svc_st(uint8_t* dst, const SvcRow& x, size_t e, uint64_t v, bool& ovf) {
  KSS_GLOBAL uint8_t* p = gp(dst) + x.dof + e * (size_t)x.ed;
  if (x.ed == x.es) {  // same width: a copy
    if (x.ed == 1) *p = (uint8_t)v;
    else if (x.ed == 2) *reinterpret_cast<KSS_GLOBAL uint16_t*>(p) = (uint16_t)v;
    else *reinterpret_cast<KSS_GLOBAL uint64_t*>(p) = v;
  } else if (x.ed == 4) {
    const int64_t s = (int64_t)v;
    ovf |= s < INT32_MIN || s > INT32_MAX;
    *reinterpret_cast<KSS_GLOBAL int32_t*>(p) = (int32_t)s;
  } else {
    const int64_t s = (int64_t)v;
    ovf |= s < 0 || s > 255;
    *p = (uint8_t)s;
  }
}

// The rows in `send` of this shard's node range [lo, hi): slot -> pinned host record.  The
// record's HBM loads are the latency here (a few hundred ns to ~1 us each), so every lane
// first issues its loads for a batch of rows (at most one destination store per row and
// round), then converts and stores: one load round trip per batch of 10 rows instead of one
// per row.  Interior stores are 16-byte (4-byte for compact uint8 rows); the unaligned ends
// of each row segment go element by element.
#ifndef KSS_SVC_RB
#define KSS_SVC_RB 4  // 10 held 2.1 KB of scratch per lane in the general chain's kernel (r6n A/B: general chain 54.7 -> 47.3 us full, 40.9 -> 31.5 slim)
#endif
template <bool COMPACT>
__device__ __forceinline__ void svc_send(const uint8_t* slot, uint8_t* host, const SlotLayout& L,
                                         const CompactLayout& CL, size_t N, unsigned send, int lo, int hi, bool& ovf) {
  // rows go to the waves in turn (row r to wave r mod waves), a row's chunks to the wave's
  // lanes: a wave's stores to host memory complete one instruction at a time, so the rows
  // are spread over every wave of the shard rather than the lanes of one
  const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6, nw = (int)blockDim.x >> 6;
  constexpr int RB = KSS_SVC_RB;  // rows per batch (registers: RB x 2 x 16 bytes)
  // interior chunks of a row: at most (hi - lo) / 2 + 1 (16-byte stores of 8-byte elements)
  const int rounds = ((hi - lo) / 2 + 1 + 63) / 64;
  for (int rb = 0; rb < SVC_ROWS; rb += RB) {
    for (int k = 0; k < rounds; k++) {
      uint4 v[RB][2];
      bool have[RB];
#pragma unroll
      for (int q = 0; q < RB; q++) {
        const int r = rb + q;
        have[q] = false;
        if (r >= SVC_ROWS || !((send >> r) & 1u) || r % nw != wave) continue;
        const SvcRow x = svc_row<COMPACT>(L, CL, N, r);
        const size_t a0 = x.e0 + (size_t)lo, b0 = x.e0 + (size_t)hi;
        const size_t a = (a0 + x.V - 1) / x.V * x.V, b = b0 / x.V * x.V;
        const size_t i = (size_t)(lane + k * 64);
        if (a >= b || i >= (b - a) / x.V) continue;
        have[q] = true;
        KSS_GLOBAL const uint4* s4 = reinterpret_cast<KSS_GLOBAL const uint4*>(gp(slot) + x.so + (a + i * x.V) * x.es);
        v[q][0] = make_uint4(s4[0].x, s4[0].y, s4[0].z, s4[0].w);
        if (x.V * x.es > 16) v[q][1] = make_uint4(s4[1].x, s4[1].y, s4[1].z, s4[1].w);
      }
#pragma unroll
      for (int q = 0; q < RB; q++) {
        if (!have[q]) continue;
        const int r = rb + q;
        const SvcRow x = svc_row<COMPACT>(L, CL, N, r);
        const size_t a0 = x.e0 + (size_t)lo;
        const size_t a = (a0 + x.V - 1) / x.V * x.V;
        const size_t i = (size_t)(lane + k * 64);
        KSS_GLOBAL uint8_t* dp = gp(host) + x.dof + (a + i * x.V) * x.ed;
        if (x.ed == x.es) {  // a 16-byte copy: member stores, merged into one dwordx4
          KSS_GLOBAL uint4* d4 = reinterpret_cast<KSS_GLOBAL uint4*>(dp);
          d4->x = v[q][0].x;
          d4->y = v[q][0].y;
          d4->z = v[q][0].z;
          d4->w = v[q][0].w;
        } else if (x.ed == 4) {  // 4 int64 -> 4 int32
          const uint32_t w[8] = {v[q][0].x, v[q][0].y, v[q][0].z, v[q][0].w, v[q][1].x, v[q][1].y, v[q][1].z, v[q][1].w};
          uint32_t o[4];
#pragma unroll
          for (int e = 0; e < 4; e++) {
            const int64_t sv = (int64_t)(((uint64_t)w[2 * e + 1] << 32) | w[2 * e]);
            ovf |= sv < INT32_MIN || sv > INT32_MAX;
            o[e] = (uint32_t)(int32_t)sv;
          }
          KSS_GLOBAL uint4* d4 = reinterpret_cast<KSS_GLOBAL uint4*>(dp);
          d4->x = o[0];
          d4->y = o[1];
          d4->z = o[2];
          d4->w = o[3];
        } else {  // 4 int64 -> 4 uint8, one 4-byte store
          const uint32_t w[8] = {v[q][0].x, v[q][0].y, v[q][0].z, v[q][0].w, v[q][1].x, v[q][1].y, v[q][1].z, v[q][1].w};
          uint32_t o = 0;
#pragma unroll
          for (int e = 0; e < 4; e++) {
            const int64_t sv = (int64_t)(((uint64_t)w[2 * e + 1] << 32) | w[2 * e]);
            ovf |= sv < 0 || sv > 255;
            o |= ((uint32_t)sv & 0xFFu) << (8 * e);
          }
          *reinterpret_cast<KSS_GLOBAL uint32_t*>(dp) = o;
        }
      }
    }
  }
  // the unaligned ends: at most V - 1 elements at each end of each row segment, loads first
  for (int rb = 0; rb < SVC_ROWS; rb += RB) {
    {  // a segment has at most 31 such elements: one per lane of the row's wave
      uint64_t ev[RB];
      size_t ee[RB];
      bool have[RB];
#pragma unroll
      for (int q = 0; q < RB; q++) {
        const int r = rb + q;
        have[q] = false;
        if (r >= SVC_ROWS || !((send >> r) & 1u) || r % nw != wave) continue;
        const SvcRow x = svc_row<COMPACT>(L, CL, N, r);
        const size_t a0 = x.e0 + (size_t)lo, b0 = x.e0 + (size_t)hi;
        size_t a = (a0 + x.V - 1) / x.V * x.V, b = b0 / x.V * x.V;
        if (a >= b) a = b = b0;  // no interior: the whole segment is a "head"
        const int nh = (int)(a - a0), ntl = (int)(b0 - b);
        const int i = lane;
        if (i >= nh + ntl) continue;
        ee[q] = i < nh ? a0 + (size_t)i : b + (size_t)(i - nh);
        ev[q] = svc_ld(slot, x, ee[q]);
        have[q] = true;
      }
#pragma unroll
      for (int q = 0; q < RB; q++)
        if (have[q]) svc_st(host, svc_row<COMPACT>(L, CL, N, rb + q), ee[q], ev[q], ovf);
    }
  }
}

// The rows (bit r) whose elements [lo, hi) differ between two records; every lane of the
// workgroup gets the mask (one LDS word, two barriers).
__device__ __forceinline__ unsigned svc_changed_rows(const uint8_t* a, const uint8_t* b, const SlotLayout& L, size_t N,
                                                     unsigned rows, int lo, int hi, unsigned& word) {
  if (threadIdx.x == 0) word = 0;
  __syncthreads();
  unsigned mine = 0;
  for (int r = 0; r < SVC_ROWS; r++) {
    if (!((rows >> r) & 1u)) continue;
    int es = 0;
    const size_t o = svc_row_off(L, N, r, es);
    bool d = false;
    for (int i = lo + (int)threadIdx.x; i < hi; i += (int)blockDim.x) {
      if (es == 1) d |= gp(a + o)[i] != gp(b + o)[i];
      else if (es == 2) d |= gp(reinterpret_cast<const uint16_t*>(a + o))[i] != gp(reinterpret_cast<const uint16_t*>(b + o))[i];
      else d |= gp(reinterpret_cast<const uint64_t*>(a + o))[i] != gp(reinterpret_cast<const uint64_t*>(b + o))[i];
    }
    mine |= d ? 1u << r : 0u;
  }
  if (mine) atomicOr(&word, mine);
  __syncthreads();
  return word;
}

// ---------------------------------------------------------------------------
// The k_simple-shaped evaluation (SIMPLE grids: staged default-profile pods -- no spread /
// inter-pod programs, host ports, node-cached images, volumes or extended resources -- at
// percentageOfNodesToScore 100).  Per node, from the shard's LDS node rows: the static part of
// the cycle (static_word: NodeUnschedulable, NodeName, TaintToleration, NodeAffinity and their raw
// scores) and the state-dependent part (dyn_eval: NodeResourcesFit, the Fit and
// BalancedAllocation scores) as k_simple computes them, one statistics exchange {feasible, max
// TaintToleration, max NodeAffinity}, NormalizeScore and the weighted total, one key exchange.
// The record rows asked for go from registers straight into the pinned host record (the HBM
// slot and its copy are skipped).  Entries equal schedule_pod<false>'s canonical record.
// ---------------------------------------------------------------------------
// The SIMPLE grid's exchange (W <= 64 shards): K 64-bit values per shard, ops[k] OP_SUM / OP_MAX.
// The workgroup folds its waves in LDS, lane 0 of wave 0 publishes 2K granules {epoch, half}
// (a plain store when every shard runs on one XCD: the line stays in its L2; else agent scope),
// lane l < W of wave 0 polls shard l's granules (agent-scope loads, bounded) and the wave folds
// them; every lane gets the result.  One round trip per exchange, no LDS atomics.
constexpr int SVC_XG = 8;  // granules per shard row (64 bytes)

// Wave 0's part (out of line: the caller's registers stay free): publish xv[0..K) as 2K granules
// {epoch, half}, poll every shard's row (lane l: shard l), fold with the operators (opbits: 2 bits
// per value) and leave the result in xv.  False (abort set, error raised) after the wait bound.
__device__ __noinline__ bool svc_sweep(long long* smem, unsigned long long* gran, int W, int wself, unsigned ep, int* err,
                                       int K, unsigned opbits, bool plain) {
  long long* xv = xvec(smem);
  const int lane = threadIdx.x & 63;
  const unsigned long long tag = (unsigned long long)ep << 32;
  unsigned long long* row = gran + ((size_t)(ep & 1) * W) * SVC_XG;
  if (lane < 2 * K) {  // lane 2k / 2k+1: value k's low / high half
    const unsigned long long u = (unsigned long long)xv[lane >> 1];
    const unsigned long long g = tag | ((lane & 1) ? (u >> 32) : (u & 0xFFFFFFFFull));
    unsigned long long* p = row + (size_t)wself * SVC_XG + lane;
    if (plain) asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(g) : "memory");
    else __hip_atomic_store(gp(p), g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  unsigned long long w2[SVC_XG];
  long long t0 = 0;
  for (unsigned spins = 0;; ++spins) {
    bool ok = true;
    if (lane < W) {
      KSS_GLOBAL const unsigned long long* g = gp(row) + (size_t)lane * SVC_XG;
#pragma unroll
      for (int i = 0; i < SVC_XG; i++)
        if (i < 2 * K) w2[i] = __hip_atomic_load(g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int i = 0; i < SVC_XG; i++)
        if (i < 2 * K) ok &= (w2[i] >> 32) == ep;
    }
    if (__all(ok)) break;
    if (spin_expired(spins, t0)) {
      if (lane == 0) err_raise(err, 1);
      return false;
    }
  }
#pragma unroll
  for (int k = 0; k < SVC_XG / 2; k++) {
    if (k >= K) break;
    const int op = (int)((opbits >> (2 * k)) & 3u);
    long long v = lane < W ? (long long)((w2[2 * k + 1] << 32) | (w2[2 * k] & 0xFFFFFFFFull)) : op_identity(op);
    v = wave_reduce(v, op);
    if (lane == 0) xv[k] = v;
  }
  return true;
}

// the same, inlined (KSS_SVC_INLINE_SWEEP=1 selects the kernel built with it: an A/B of the call)
__device__ __forceinline__ bool svc_sweep_inl(long long* smem, unsigned long long* gran, int W, int wself, unsigned ep, int* err,
                                       int K, unsigned opbits, bool plain) {
  long long* xv = xvec(smem);
  const int lane = threadIdx.x & 63;
  const unsigned long long tag = (unsigned long long)ep << 32;
  unsigned long long* row = gran + ((size_t)(ep & 1) * W) * SVC_XG;
  if (lane < 2 * K) {  // lane 2k / 2k+1: value k's low / high half
    const unsigned long long u = (unsigned long long)xv[lane >> 1];
    const unsigned long long g = tag | ((lane & 1) ? (u >> 32) : (u & 0xFFFFFFFFull));
    unsigned long long* p = row + (size_t)wself * SVC_XG + lane;
    if (plain) asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(g) : "memory");
    else __hip_atomic_store(gp(p), g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  unsigned long long w2[SVC_XG];
  long long t0 = 0;
  for (unsigned spins = 0;; ++spins) {
    bool ok = true;
    if (lane < W) {
      KSS_GLOBAL const unsigned long long* g = gp(row) + (size_t)lane * SVC_XG;
#pragma unroll
      for (int i = 0; i < SVC_XG; i++)
        if (i < 2 * K) w2[i] = __hip_atomic_load(g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int i = 0; i < SVC_XG; i++)
        if (i < 2 * K) ok &= (w2[i] >> 32) == ep;
    }
    if (__all(ok)) break;
    if (spin_expired(spins, t0)) {
      if (lane == 0) err_raise(err, 1);
      return false;
    }
  }
#pragma unroll
  for (int k = 0; k < SVC_XG / 2; k++) {
    if (k >= K) break;
    const int op = (int)((opbits >> (2 * k)) & 3u);
    long long v = lane < W ? (long long)((w2[2 * k + 1] << 32) | (w2[2 * k] & 0xFFFFFFFFull)) : op_identity(op);
    v = wave_reduce(v, op);
    if (lane == 0) xv[k] = v;
  }
  return true;
}

// The SIMPLE grid's exchange (W <= 64 shards): K 64-bit values per shard, ops[k] OP_SUM / OP_MAX.
// The workgroup folds its waves in LDS, wave 0 publishes 2K granules {epoch, half} (a plain store
// when every shard runs on one XCD: the line stays in its L2; else agent scope) and polls shard
// l's row on lane l (agent-scope loads, bounded); every lane gets the result.  One round trip per
// exchange, no LDS atomics.
template <int K, bool INL = false>
__device__ __forceinline__ bool svc_xchg(long long* smem, Shard& S, bool plain, long long (&v)[K], const int (&ops)[K]) {
  static_assert(2 * K <= SVC_XG, "granule row");
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
    for (int x = 1; x < nw; x++) r = op_apply(op, r, h.red[x][k]);
    xv[k] = r;
  }
  __syncthreads();
  if (S.W > 1) {
    unsigned opbits = 0;
#pragma unroll
    for (int k = 0; k < K; k++) opbits |= (unsigned)ops[k] << (2 * k);
    ++S.epoch;
    if (wave == 0) {
      const bool ok = INL ? svc_sweep_inl(smem, S.gran, S.W, S.w, S.epoch, S.err, K, opbits, plain)
                          : svc_sweep(smem, S.gran, S.W, S.w, S.epoch, S.err, K, opbits, plain);
      if (!ok && lane == 0) h.abort = 1;
    }
    __syncthreads();
    if (h.abort) return false;
  }
#pragma unroll
  for (int k = 0; k < K; k++) v[k] = xv[k];
  __syncthreads();  // xv may be rewritten by the next exchange
  return true;
}

template <bool COMPACT>
__device__ __forceinline__ void svc_put(uint8_t* host, size_t off, size_t e, int es, int64_t v) {
  KSS_GLOBAL uint8_t* p = gp(host) + off + e * (size_t)es;
  if (es == 1) *p = (uint8_t)v;
  else if (es == 2) *reinterpret_cast<KSS_GLOBAL uint16_t*>(p) = (uint16_t)v;
  else if (es == 4) *reinterpret_cast<KSS_GLOBAL int32_t*>(p) = (int32_t)v;
  else *reinterpret_cast<KSS_GLOBAL int64_t*>(p) = v;
}

// Speculative prefetch for the next evaluation (the plugin evaluates the staged pods in order):
// pod k's static words of this shard's nodes into the slot array the simple evaluation does not
// use (ipa), its compact record into the header's pod area, tagged svc_pf = k.  Issued after an
// evaluation's done flag, it completes while the host reads the record and posts the next command;
// an evaluation of another pod loads from HBM as before.
static_assert(sizeof(SPod) <= sizeof(kss_pod), "the compact record fits the header's pod area");
__device__ __forceinline__ void svc_prefetch(const DevJob& job, long long* smem, const Shard& S, int bins_cap, int npt,
                                             int k) {
  SharedHdr& H = shdr(smem);
  const int tid = threadIdx.x, nt = blockDim.x;
  const size_t N = (size_t)job.c.N;
  if (!job.stat || k < 0 || k >= job.n_pods) {
    if (tid == 0) H.svc_pf = -1;
    __syncthreads();
    return;
  }
  const SlotArrays sa = slot_arrays(smem, bins_cap, npt * nt);
  for (int j = 0; j < npt; j++) {
    const int n = S.lo + j * nt + tid;
    if (n < S.hi) sa.ipa[j * nt + tid] = ld_ag(gp(job.stat) + (size_t)k * N + n);
  }
  constexpr int SW = (int)(sizeof(SPod) / 4);
  const uint32_t* src = reinterpret_cast<const uint32_t*>(job.spods + k);
  uint32_t* dst = reinterpret_cast<uint32_t*>(&H.pod);
  for (int i = tid; i < SW; i += nt) dst[i] = src[i];
  if (tid == 0) H.svc_pf = k;
  __syncthreads();
}

// The findNodesThatPassFilters window on the SIMPLE evaluation (percentageOfNodesToScore < 100,
// no PreFilterResult node lists): k_simple's simple_sync_win for one pod, without
// the speculative halves.  The node list is visited from the cursor s0 in canonical order,
// wrapping: segments a_0 .. a_{W-1} (each shard's nodes >= s0), then b_0 .. b_{W-1} (< s0).  One
// exchange gathers every shard's {feasible count, max raw TaintToleration, max raw NodeAffinity}
// per part (lane l of wave 0 <- shard l: W <= 64); every shard finds the segment holding the
// (K+1)-th feasible node and the maxima of the segments wholly before it; the cut segment's
// shard ranks its feasible nodes for the stopping node d and the maxima over the first j, and a
// second exchange hands {d, TT, NA} to every shard (the cursor moves to d everywhere).
// u = this lane's {Fa, TTa, NAa, Fb, TTb, NAb}.  Out: nf (kept feasible nodes), the maxima over
// them, wd (d, -1 when fewer than K + 1 nodes are feasible).  False on abort.
__device__ bool svc_window(long long* smem, Shard& S, bool plain, int K, int s0, const SlotArrays& sa, int npt,
                           const uint32_t (&u)[6], long long& nf, long long& mtt, long long& mna, int& wd) {
  SharedHdr& h = shdr(smem);
  long long* xv = xvec(smem);
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wave = tid >> 6, nw = nt >> 6;
#pragma unroll
  for (int i = 0; i < 6; i++) {
    const long long r = wave_reduce((long long)u[i], i % 3 == 0 ? OP_SUM : OP_MAX);
    if (lane == 0) h.red[wave][i] = r;
  }
  __syncthreads();
  const unsigned ep = S.W > 1 ? ++S.epoch : S.epoch;
  if (wave == 0) {
    long long v[6];
#pragma unroll
    for (int i = 0; i < 6; i++) {
      v[i] = h.red[0][i];
      for (int x = 1; x < nw; x++) v[i] = op_apply(i % 3 == 0 ? OP_SUM : OP_MAX, v[i], h.red[x][i]);
    }
    // every shard's row in the lane of that shard: {Fa << 16 | TTa, NAa, Fb << 16 | TTb, NAb}
    const uint32_t mine[4] = {(uint32_t)((v[0] << 16) | v[1]), (uint32_t)v[2], (uint32_t)((v[3] << 16) | v[4]),
                              (uint32_t)v[5]};
    uint32_t g4[4] = {0, 0, 0, 0};
    bool ok = true;
    if (S.W == 1) {
#pragma unroll
      for (int i = 0; i < 4; i++) g4[i] = lane == 0 ? mine[i] : 0u;
    } else {
      const unsigned long long tag = (unsigned long long)ep << 32;
      unsigned long long* row = S.gran + (size_t)(ep & 1) * S.W * SVC_XG;
      if (lane < 4) {
        uint32_t x = mine[0];
        x = lane == 1 ? mine[1] : x;
        x = lane == 2 ? mine[2] : x;
        x = lane == 3 ? mine[3] : x;
        unsigned long long* q = row + (size_t)S.w * SVC_XG + lane;
        if (plain) asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(q), "v"(tag | x) : "memory");
        else __hip_atomic_store(gp(q), tag | x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      long long t0 = 0;
      for (unsigned spins = 0;; ++spins) {
        bool got = true;
        unsigned long long w4[4] = {tag, tag, tag, tag};
        if (lane < S.W) {
          KSS_GLOBAL const unsigned long long* g = gp(row) + (size_t)lane * SVC_XG;
#pragma unroll
          for (int i = 0; i < 4; i++) w4[i] = __hip_atomic_load(g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int i = 0; i < 4; i++) got &= (w4[i] >> 32) == ep;
        if (__all(got)) {
#pragma unroll
          for (int i = 0; i < 4; i++) g4[i] = lane < S.W ? (uint32_t)w4[i] : 0u;
          break;
        }
        if (spin_expired(spins, t0)) {
          if (lane == 0) err_raise(S.err, 1);
          ok = false;
          break;
        }
      }
    }
    const uint32_t Fa = g4[0] >> 16, ta = g4[0] & 0xFFFFu, na = g4[1], Fb = g4[2] >> 16, tb = g4[2] & 0xFFFFu, nb = g4[3];
    const uint32_t A = (uint32_t)wave_reduce((long long)Fa, OP_SUM), B = (uint32_t)wave_reduce((long long)Fb, OP_SUM);
    const uint32_t F = A + B;
    long long ftt, fna;
    int cut = -1, part = 0, j = 0;
    if (F <= (uint32_t)K) {
      ftt = wave_reduce((long long)max(ta, tb), OP_MAX);
      fna = wave_reduce((long long)max(na, nb), OP_MAX);
    } else {
      const uint32_t pa = wave_incl_scan(Fa) - Fa, pb = A + wave_incl_scan(Fb) - Fb, Ku = (uint32_t)K;
      ftt = wave_reduce((long long)max(pa + Fa <= Ku ? ta : 0u, pb + Fb <= Ku ? tb : 0u), OP_MAX);
      fna = wave_reduce((long long)max(pa + Fa <= Ku ? na : 0u, pb + Fb <= Ku ? nb : 0u), OP_MAX);
      const unsigned long long ba = __ballot(pa <= Ku && Ku < pa + Fa), bb = __ballot(pb <= Ku && Ku < pb + Fb);
      const int l = __ffsll((long long)(ba ? ba : bb)) - 1;
      cut = l;
      part = ba ? 0 : 1;
      j = (int)(Ku - (uint32_t)__builtin_amdgcn_readlane((int)(ba ? pa : pb), l));
    }
    if (lane == 0) {
      xv[0] = F;
      xv[1] = ftt;
      xv[2] = fna;
      xv[3] = cut;
      xv[4] = part;
      xv[5] = j;
      xv[6] = -1;  // d, written by the cut shard's scan
      if (!ok) h.abort = 1;
    }
  }
  __syncthreads();
  if (h.abort) return false;
  nf = xv[0];
  mtt = xv[1];
  mna = xv[2];
  wd = -1;
  const int cut = (int)xv[3], part = (int)xv[4], j = (int)xv[5];
  if (cut < 0) return true;
  nf = K;
  int ctt = 0, cna = 0;
  if (cut == S.w) {  // rank the part's feasible nodes in canonical order (slot k-major): d = rank j
    int carry = 0;
    for (int k = 0; k < npt; k++) {
      const int n = S.lo + k * nt + tid, si = k * nt + tid;
      const bool f = n < S.hi && (sa.fail[si] & 0xFF) == KSS_F_PASS && (part == 0 ? n >= s0 : n < s0);
      const unsigned long long b = __ballot(f);
      if (lane == 0) h.red[wave][8 + (k & 1)] = (long long)__popcll(b);
      __syncthreads();
      int before = 0, tot = 0;
      for (int x = 0; x < nw; x++) {
        const int cx = (int)h.red[x][8 + (k & 1)];
        before += x < wave ? cx : 0;
        tot += cx;
      }
      const int rank = carry + before + (int)__popcll(b & ((1ull << lane) - 1ull));
      if (f && rank == j) xv[6] = n;
      ctt = max(ctt, (f && rank < j) ? sa.tt[si] : 0);
      cna = max(cna, (f && rank < j) ? (int)sa.na[si] : 0);
      carry += tot;
    }
    ctt = (int)wave_reduce((long long)ctt, OP_MAX);
    cna = (int)wave_reduce((long long)cna, OP_MAX);
    if (lane == 0) {
      h.red[wave][10] = ctt;
      h.red[wave][11] = cna;
    }
    __syncthreads();
    for (int x = 0; x < nw; x++) {
      ctt = max(ctt, (int)h.red[x][10]);
      cna = max(cna, (int)h.red[x][11]);
    }
  }
  if (S.W == 1) {
    wd = (int)xv[6];
    mtt = max(mtt, (long long)ctt);
    mna = max(mna, (long long)cna);
    __syncthreads();  // xv is rewritten by the next exchange
    return true;
  }
  // the second exchange keeps the first one's epoch, in an area of its own (parity ep & 1): the
  // next exchange's tag is ep + 1, so no shard can overwrite a row another still polls
  const unsigned ep2 = ep;
  unsigned long long* e2 = S.gran + 2 * (size_t)S.W * SVC_XG + (size_t)(ep2 & 1) * 4;
  const unsigned long long tag2 = (unsigned long long)ep2 << 32;
  if (cut == S.w && tid < 3) {
    const uint32_t x = tid == 0 ? (uint32_t)xv[6] : (tid == 1 ? (uint32_t)ctt : (uint32_t)cna);
    if (plain) asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(e2 + tid), "v"(tag2 | x) : "memory");
    else __hip_atomic_store(gp(e2) + tid, tag2 | x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();  // the cut shard's xv[6] read before any lane rewrites it below
  if (wave == 0) {
    long long t0 = 0;
    for (unsigned spins = 0;; ++spins) {
      const unsigned long long g = __hip_atomic_load(gp(e2) + min(lane, 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__all((g >> 32) == ep2)) {
        if (lane < 3) xv[8 + lane] = (long long)(uint32_t)g;
        break;
      }
      if (spin_expired(spins, t0)) {
        if (lane == 0) {
          err_raise(S.err, 1);
          h.abort = 1;
        }
        break;
      }
    }
  }
  __syncthreads();
  if (h.abort) return false;
  wd = (int)xv[8];
  mtt = max(mtt, xv[9]);
  mna = max(mna, xv[10]);
  __syncthreads();  // xv is rewritten by the next exchange
  return true;
}

template <bool COMPACT, bool INL>
__device__ bool svc_simple_eval(const DevCluster& c, const DevJob& job, const kss_profile& prof, int pi, long long* smem,
                                Shard& S, int bins_cap, int npt, unsigned want, uint8_t* host, PodMeta& meta, bool plain,
                                unsigned long long* st3) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const size_t N = (size_t)c.N;
  const SlotLayout L(N);
  const CompactLayout CL(N);
  const kss_pod& p = job.P.pods[pi];
  SharedHdr& H = shdr(smem);
  const bool hit = H.svc_pf == pi;  // the prefetch guessed this pod: words and record already in LDS
  const SPod& q = hit ? *reinterpret_cast<const SPod*>(&H.pod) : job.spods[pi];
  const SlotArrays sa = slot_arrays(smem, bins_cap, npt * nt);
  // every HBM load of the evaluation first, in flight together: the static words of this lane's
  // nodes (the table k_static filled) -- no branch between them and the command
  // (staged through the slot array the simple evaluation leaves unused: a register array indexed
  // in the node loop would live in scratch)
  if (job.stat && !hit) {
    uint32_t wpre[KSS_MAX_NPT];
#pragma unroll
    for (int k = 0; k < KSS_MAX_NPT; k++) {
      const int n = S.lo + k * nt + tid;
      wpre[k] = (k < npt && n < S.hi) ? ld_ag(gp(job.stat) + (size_t)pi * N + n) : 0u;
    }
#pragma unroll
    for (int k = 0; k < KSS_MAX_NPT; k++)
      if (k < npt) sa.pts[k * nt + tid] = wpre[k];
  }
  meta.chosen = -1;
  meta.n_feasible = 0;
  meta.scored = 0;
  meta.status = 0;
  meta.best_total = 0;
  // row offsets in the host record: fail, detail, total, raw x, norm x
  const size_t o_fail = COMPACT ? CL.fail : L.fail, o_det = COMPACT ? CL.detail : L.detail;
  const size_t o_tot = COMPACT ? CL.total : L.total, o_raw = COMPACT ? CL.raw : L.raw, o_norm = COMPACT ? CL.norm : L.norm;
  const int es_tot = COMPACT ? 4 : 8, es_raw = COMPACT ? 4 : 8, es_norm = COMPACT ? 1 : 8;
  const bool w_fail = want & 1u, w_det = (want >> 1) & 1u, w_tot = (want >> 2) & 1u;
  const bool w_raw = (want >> 3) & 1u, w_norm = (want >> (3 + KSS_NSCORE)) & 1u;  // every raw / norm row or none
  if (q.status != 0) {  // PreFilter failure (kss_pod.prefilter_status): no node evaluated
    for (int k = 0; k < npt; k++) {
      const int n = S.lo + k * nt + tid;
      if (n >= S.hi) continue;
      if (w_fail) svc_put<COMPACT>(host, o_fail, (size_t)n, 1, KSS_F_NOT_EVALUATED);
      if (w_det) svc_put<COMPACT>(host, o_det, (size_t)n, 2, 0);
      if (w_tot) svc_put<COMPACT>(host, o_tot, (size_t)n, es_tot, 0);
#pragma unroll
      for (int x = 0; x < KSS_NSCORE; x++) {
        if (w_raw) svc_put<COMPACT>(host, o_raw, (size_t)x * N + n, es_raw, 0);
        if (w_norm) svc_put<COMPACT>(host, o_norm, (size_t)x * N + n, es_norm, 0);
      }
    }
    meta.status = q.status == KSS_PF_ERROR ? 3 : 2;
    return true;
  }
  const uint32_t en = prof.filter_enabled;
  // percentageOfNodesToScore < 100: the window from the cursor (svc_window)
  const int k_find = num_feasible_to_find(c.N, prof.pct_nodes_to_score);
  const bool win = k_find < c.N;
  const int s0 = win ? (int)(((long long)S.cursor % c.N + c.N) % c.N) : 0;
  uint32_t wu[6] = {0, 0, 0, 0, 0, 0};  // this lane's {Fa, TTa, NAa, Fb, TTb, NAb}
  long long nf = 0, max_tt = 0, max_na = 0;
  for (int k = 0; k < npt; k++) {
    const int n = S.lo + k * nt + tid;
    const int si = k * nt + tid;
    if (n >= S.hi) {
      sa.fail[si] = KSS_F_NOT_EVALUATED;
      continue;
    }
    const NodeRow row = load_row(c, n);
    // the static word: precomputed for every staged pod at the grid's start (k_static into
    // job.stat, loaded above) or, without that table, evaluated here
    const uint32_t w = !job.stat ? static_word(c, job.P, p, prof, n, row.flags, row.th, row.ts)
                                 : (uint32_t)(hit ? sa.ipa[si] : sa.pts[si]);
    DynRow dr;
#pragma unroll
    for (int r = 0; r < 3; r++) {
      dr.alloc[r] = (double)row.alloc[r];
      dr.req[r] = (double)row.req[r];
      dr.inv[r] = row.alloc[r] > 0 ? 1.0 / (double)row.alloc[r] : 0.0;
    }
    dr.nz[0] = (double)row.nz[0];
    dr.nz[1] = (double)row.nz[1];
    dr.pods = row.pods;
    dr.allowed = row.allowed;
    const SVal e = dyn_eval(prof, q, w, dr);
    uint16_t detail = 0;
    if (e.f == KSS_F_TAINT_TOLERATION || e.f == KSS_F_NODE_RESOURCES_FIT)
      (void)filter_local(c, job.P, p, en, n, row, &detail);  // the failure's detail (taint id, fit bits)
    sa.fail[si] = e.f | ((int)detail << 8);
    sa.tt[si] = e.tt;
    sa.na[si] = e.na;
    sa.fit[si] = e.fit;
    sa.ba[si] = e.ba;
    if (e.f == KSS_F_PASS) {
      nf++;
      max_tt = e.tt > max_tt ? e.tt : max_tt;
      max_na = e.na > max_na ? e.na : max_na;
      const int o = n >= s0 ? 0 : 3;
      wu[o] += 1;
      wu[o + 1] = max(wu[o + 1], (uint32_t)e.tt);
      wu[o + 2] = max(wu[o + 2], (uint32_t)e.na);
    }
  }
  if (st3) st3[0] = wall_clock64();
  int wd = -1;  // the window's stopping node (-1: every node visited)
  if (win) {
    if (!svc_window(smem, S, plain, k_find, s0, sa, npt, wu, nf, max_tt, max_na, wd)) return false;
    if (st3) st3[1] = wall_clock64();
  } else {
    long long v[3] = {nf, max_tt, max_na};
    const int op[3] = {OP_SUM, OP_MAX, OP_MAX};
    if (!svc_xchg<3, INL>(smem, S, plain, v, op)) return false;
    if (st3) st3[1] = wall_clock64();
    nf = v[0];
    max_tt = v[1];
    max_na = v[2];
  }
  // visiting position from the cursor: n was filtered iff pos(n) <= pos(d), kept iff also feasible
  // and pos(n) < pos(d) (d passed every filter but the framework dropped it)
  const int pd = wd >= 0 ? (wd - s0 + c.N) % c.N : c.N;
  const bool scored = nf > 1;
  const float rtt = max_tt ? __builtin_amdgcn_rcpf((float)max_tt) : 0.f, rna = max_na ? __builtin_amdgcn_rcpf((float)max_na) : 0.f;
  // the selectHost key first (its exchange is the chain), then the record rows
  long long best = 0;
  for (int k = 0; k < npt; k++) {
    const int n = S.lo + k * nt + tid;
    const int si = k * nt + tid;
    if (n >= S.hi || (sa.fail[si] & 0xFF) != KSS_F_PASS || (n - s0 + c.N) % c.N >= pd) continue;
    const SVal e{KSS_F_PASS, sa.tt[si], (int)sa.na[si], sa.fit[si], sa.ba[si]};
    const long long key = simple_key(prof, e, scored, (int)max_tt, rtt, (int)max_na, rna, (uint32_t)(c.node_base + n));
    best = key > best ? key : best;
  }
  if (st3) st3[2] = wall_clock64();
  if (nf > 0) {
    long long v[1] = {best};
    const int op[1] = {OP_MAX};
    if (!svc_xchg<1, INL>(smem, S, plain, v, op)) return false;
    best = v[0];
  }
  for (int k = 0; k < npt; k++) {
    const int n = S.lo + k * nt + tid;
    const int si = k * nt + tid;
    if (n >= S.hi) continue;
    int fw = sa.fail[si];
    const int pos = (n - s0 + c.N) % c.N;
    if (pos > pd) fw = KSS_F_NOT_EVALUATED;  // the search stopped before this node
    else if (pos == pd) fw = KSS_F_PASS | (KSS_PASS_NOT_KEPT << 8);  // the stopping node: filtered, dropped
    const int f = fw & 0xFF;
    SVal e{f, sa.tt[si], (int)sa.na[si], sa.fit[si], sa.ba[si]};
    const bool pass = f == KSS_F_PASS && pos < pd;
    // the row values as scalars (a local array indexed in the store loop would go to scratch)
    const int64_t r_tt = pass ? e.tt : 0, r_na = pass ? e.na : 0, r_fit = pass ? e.fit : 0, r_ba = pass ? e.ba : 0;
    int64_t n_tt = 0, n_na = 0, n_fit = 0, n_pts = 0, n_ba = 0, total = 0;
    if (pass && scored) {
      const long long key = simple_key(prof, e, scored, (int)max_tt, rtt, (int)max_na, rna, (uint32_t)(c.node_base + n));
      n_tt = max_tt == 0 ? 100 : 100 - small_div(100 * e.tt, (int)max_tt, rtt);
      n_na = max_na != 0 ? small_div(100 * e.na, (int)max_na, rna) : e.na;
      n_fit = e.fit;
      n_pts = 100;
      n_ba = e.ba;
      total = (int64_t)(((unsigned long long)key) >> 32);
    }
    if (w_fail) svc_put<COMPACT>(host, o_fail, (size_t)n, 1, f);
    if (w_det) svc_put<COMPACT>(host, o_det, (size_t)n, 2, (uint16_t)(fw >> 8));
    if (w_tot) svc_put<COMPACT>(host, o_tot, (size_t)n, es_tot, total);
    if (w_raw) {
      svc_put<COMPACT>(host, o_raw, (size_t)KSS_S_TAINT_TOLERATION * N + n, es_raw, r_tt);
      svc_put<COMPACT>(host, o_raw, (size_t)KSS_S_NODE_AFFINITY * N + n, es_raw, r_na);
      svc_put<COMPACT>(host, o_raw, (size_t)KSS_S_NODE_RESOURCES_FIT * N + n, es_raw, r_fit);
      svc_put<COMPACT>(host, o_raw, (size_t)KSS_S_VOLUME_BINDING * N + n, es_raw, 0);
      svc_put<COMPACT>(host, o_raw, (size_t)KSS_S_POD_TOPOLOGY_SPREAD * N + n, es_raw, 0);
      svc_put<COMPACT>(host, o_raw, (size_t)KSS_S_INTER_POD_AFFINITY * N + n, es_raw, 0);
      svc_put<COMPACT>(host, o_raw, (size_t)KSS_S_BALANCED_ALLOCATION * N + n, es_raw, r_ba);
      svc_put<COMPACT>(host, o_raw, (size_t)KSS_S_IMAGE_LOCALITY * N + n, es_raw, 0);
    }
    if (w_norm) {
      svc_put<COMPACT>(host, o_norm, (size_t)KSS_S_TAINT_TOLERATION * N + n, es_norm, n_tt);
      svc_put<COMPACT>(host, o_norm, (size_t)KSS_S_NODE_AFFINITY * N + n, es_norm, n_na);
      svc_put<COMPACT>(host, o_norm, (size_t)KSS_S_NODE_RESOURCES_FIT * N + n, es_norm, n_fit);
      svc_put<COMPACT>(host, o_norm, (size_t)KSS_S_VOLUME_BINDING * N + n, es_norm, 0);
      svc_put<COMPACT>(host, o_norm, (size_t)KSS_S_POD_TOPOLOGY_SPREAD * N + n, es_norm, n_pts);
      svc_put<COMPACT>(host, o_norm, (size_t)KSS_S_INTER_POD_AFFINITY * N + n, es_norm, 0);
      svc_put<COMPACT>(host, o_norm, (size_t)KSS_S_BALANCED_ALLOCATION * N + n, es_norm, n_ba);
      svc_put<COMPACT>(host, o_norm, (size_t)KSS_S_IMAGE_LOCALITY * N + n, es_norm, 0);
    }
  }
  if (wd >= 0) S.cursor = wd;  // nextStartNodeIndex: the stopping node (every shard knows it)
  meta.n_feasible = (int)nf;
  if (nf == 0) {
    meta.status = 1;
    return true;
  }
  const unsigned long long ub = (unsigned long long)best;
  meta.chosen = (int)(0xFFFFFFFFull - (ub & 0xFFFFFFFFull));
  meta.scored = scored ? 1 : 0;
  meta.best_total = scored ? (int64_t)(ub >> 32) : 0;
  return true;
}

template <bool GEN, bool SIMPLE, bool INL = false>
__device__ void service_loop(DevCluster c, const DevJob& job, const kss_profile& prof, int W, int npt, int bins_cap,
                             int cache_keys, unsigned long long* gran, int* err, SvcBox* box_flat,
                             unsigned long long* relay_flat, unsigned long long* seen_flat, uint8_t* rec_host,
                             unsigned long long seq, unsigned epoch0, int stamps, long long* smem, int xcd) {
  KSS_GLOBAL SvcBox* box = gp(box_flat);
  KSS_GLOBAL unsigned long long* relay = gp(relay_flat);
  KSS_GLOBAL unsigned long long* seen = gp(seen_flat);
  int w = blockIdx.x;
  if (SIMPLE && xcd) {
    // XCD-local grid (xcd_slot): the first W workgroups that run on XCD 0 become the shards, the
    // others leave; the exchanges and the relay then stay in that XCD's L2.  Too few on XCD 0:
    // every workgroup leaves before taking a command and the host relaunches unrestricted.
    if (threadIdx.x == 0) shdr(smem).cmd[0] = xcd_slot(err + 2, W, (int)gridDim.x, err);
    __syncthreads();
    w = shdr(smem).cmd[0];
    __syncthreads();
    if (w == -2 && threadIdx.x == 0) __hip_atomic_store(&box->xcd_fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (w < 0) return;
  }
  const bool plain = SIMPLE && xcd;  // XCD-local granule and relay stores
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
  S.epoch = epoch0;
  S.gran = gran;
  S.err = err;
  S.stamps = nullptr;
  S.cursor = job.cursor ? *job.cursor : 0;  // nextStartNodeIndex, kept across evaluations and relaunches
  int cursor_prev = S.cursor;               // before the last evaluation (a repeated cycle starts from it)
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
  if (threadIdx.x == 0) shdr(smem).svc_pf = -1;  // no prefetched pod (LDS holds garbage until written)
  __syncthreads();
  if (SIMPLE) svc_prefetch(job, smem, S, bins_cap, npt, 0);
  int* cmd = shdr(smem).cmd;
  if (w == 0 && threadIdx.x == 0) __hip_atomic_store(&box->running, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  unsigned long long st0 = 0, st1 = 0, st2 = 0, st4 = 0;  // diagnostic clocks of shard 0's lane 0 (stamps)
  unsigned long long seen_min = seq;              // shard 0: every shard has taken the commands below this
  int parity = 0;                                 // the record slot of the next evaluation
  // rows (bit r) whose host segment equals the last evaluation's slot: full / compact record
  unsigned host_valid = 0, host_valid_c = 0;
  uint8_t* crec_host = rec_host + SlotLayout(N).bytes;  // the compact record behind the full one
  const CompactLayout CL(N);
  for (;; ++seq) {
    if (threadIdx.x == 0) {
      int op = SVC_STOP, pod = 0, node = 0, fields = 0;
      KSS_GLOBAL unsigned long long* slot = relay + 2 * (seq % SVC_DRING);
      if (w == 0) {
        const unsigned long long t0 = wall_clock64();
        bool got = false;
        KSS_GLOBAL const unsigned long long* hc = &box->cmd[seq % SVC_RING].w0;
        unsigned long long a = 0, b = 0;
        for (;;) {  // the host's next command (both tagged words), or STOP after the idle time
          a = __hip_atomic_load(hc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          b = __hip_atomic_load(hc + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if ((a >> 32) == seq + 1 && (b >> 32) == seq + 1) {
            got = true;
            break;
          }
          if (wall_clock64() - t0 > SVC_IDLE_TICKS) break;
        }
        st0 = wall_clock64();
        if (got) {
          op = (int)(a & 7);
          fields = (int)((a >> 3) & 31);
          pod = (int)((a >> 8) & 0xFFFFFF);
          node = (int)(uint32_t)b;
          if (op < SVC_EVAL || op > SVC_STOP) op = SVC_STOP;
        }
        // the relay slot is reused every SVC_DRING commands: every shard must have taken
        // command seq - SVC_DRING first (bounded: a shard that left ends the wait).  The
        // smallest `seen` is cached and re-read (every shard's word in one pass of independent
        // loads) only when the cached value no longer covers this slot: about once per
        // SVC_DRING commands instead of W dependent loads per command.
        if (seq >= (unsigned long long)SVC_DRING && seen_min < seq - SVC_DRING + 1) {
          const unsigned long long need = seq - SVC_DRING + 1, t1 = wall_clock64();
          for (;;) {
            unsigned long long m = ~0ull;
            for (int q = 1; q < W; q++) m = min(m, __hip_atomic_load(seen + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            seen_min = W > 1 ? m : ~0ull;
            if (seen_min >= need || wall_clock64() - t1 > 4 * SVC_IDLE_TICKS) break;
            __builtin_amdgcn_s_sleep(1);
          }
        }
        if (plain) {  // both words in one 16-byte plain store (XCD 0's L2; the shards poll it there)
          const unsigned long long w0 = svc_w0(seq, op, fields, pod), w1 = svc_w1(seq, node);
          typedef unsigned int svc_u32x4 __attribute__((ext_vector_type(4)));
          const svc_u32x4 q = {(unsigned)w0, (unsigned)(w0 >> 32), (unsigned)w1, (unsigned)(w1 >> 32)};
          asm volatile("global_store_dwordx4 %0, %1, off" ::"v"((unsigned long long*)slot), "v"(q) : "memory");
        } else {
          __hip_atomic_store(slot + 1, svc_w1(seq, node), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(slot, svc_w0(seq, op, fields, pod), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (got) __hip_atomic_store(&box->consumed, seq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        st1 = wall_clock64();
      } else {
        const unsigned long long t0 = wall_clock64();
        for (;;) {
          const unsigned long long a = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const unsigned long long b = __hip_atomic_load(slot + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((a >> 32) == (seq + 1) && (b >> 32) == (seq + 1)) {
            op = (int)(a & 7);
            fields = (int)((a >> 3) & 31);
            pod = (int)((a >> 8) & 0xFFFFFF);
            node = (int)(uint32_t)b;
            break;
          }
          if (wall_clock64() - t0 > 4 * SVC_IDLE_TICKS) break;  // shard 0 is gone: leave
          __builtin_amdgcn_s_sleep(1);
        }
      }
      cmd[0] = op;
      cmd[1] = pod;
      cmd[2] = node;
      cmd[3] = fields;
    }
    __syncthreads();
    const int op = cmd[0], pi = cmd[1], node = cmd[2], fields = cmd[3];
    __syncthreads();  // the command words may be rewritten by the next iteration's lane 0
    if (op == SVC_STOP) break;
    if (SIMPLE && op == SVC_EVAL) {
      PodMeta m;
      const bool compact = (node & 1) != 0;
      unsigned want = 0;
      for (int r = 0; r < SVC_ROWS; r++) want |= (fields & svc_row_field(r)) ? 1u << r : 0u;
      unsigned long long st3[3] = {0, 0, 0};
      unsigned long long* sp3 = ((stamps & 1) && w == 0 && threadIdx.x == 0) ? st3 : nullptr;
      if (node & 2) S.cursor = cursor_prev;  // the same scheduling cycle again
      cursor_prev = S.cursor;
      const bool ok = compact
                          ? svc_simple_eval<true, INL>(c, job, prof, pi, smem, S, bins_cap, npt, want, crec_host, m, plain, sp3)
                          : svc_simple_eval<false, INL>(c, job, prof, pi, smem, S, bins_cap, npt, want, rec_host, m, plain, sp3);
      if (!ok) {
        if (threadIdx.x == 0) __hip_atomic_store(&box->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      if ((stamps & 1) && w == 0 && threadIdx.x == 0) st2 = st4 = wall_clock64();
      if (w == 0 && threadIdx.x == 0) {
        if (job.cursor) *job.cursor = S.cursor;  // read by the next launch on this context
        KSS_GLOBAL int32_t* mm = reinterpret_cast<KSS_GLOBAL int32_t*>(&box->meta);
        mm[0] = m.chosen;
        mm[1] = m.n_feasible;
        mm[2] = m.scored;
        mm[3] = m.status;
        *reinterpret_cast<KSS_GLOBAL int64_t*>(mm + 4) = m.best_total;
      }
      if (stamps & 4) {
        __threadfence_system();  // (KSS_SVC_FULL_FENCE: every lane's fence, as the general chain)
      } else {
        // the record went to coherent (uncached) host memory: each wave waits for its own stores'
        // completion; after the barrier lane 0's system-scope release store of done[w] orders them
        // all before the flag (one L2 write-back per shard instead of one per wave)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      if ((stamps & 1) && w == 0 && threadIdx.x == 0) {
        KSS_GLOBAL long long* sp = reinterpret_cast<KSS_GLOBAL long long*>(&box->stamp[0]);
        sp[0] = (long long)st0;
        sp[1] = (long long)st1;
        sp[2] = (long long)st2;
        sp[3] = wall_clock64();
        sp[4] = (long long)st4;
        sp[5] = (long long)st3[0];  // node pass done
        sp[6] = (long long)st3[1];  // statistics exchange done
        sp[7] = (long long)st3[2];  // normalise + record stores issued, before the key exchange
      }
      if (threadIdx.x == 0) st_sys(&box->done[w], seq + 1);
      svc_prefetch(job, smem, S, bins_cap, npt, pi + 1);  // the next staged pod, in LDS before its command
    } else if (op == SVC_EVAL) {
      // two HBM record slots used in turn: a row segment equal to the previous evaluation's,
      // which the host record already holds, is not sent over PCIe again
      uint8_t* base = job.slots + (size_t)parity * job.slot_bytes;
      const uint8_t* prev = job.slots + (size_t)(parity ^ 1) * job.slot_bytes;
      parity ^= 1;
      Slot s;
      s.canon = true;
      s.fail = base + L.fail;
      s.detail = (uint16_t*)(base + L.detail);
      s.raw = (int64_t*)(base + L.raw);
      s.norm = (int64_t*)(base + L.norm);
      s.total = (int64_t*)(base + L.total);
      PodMeta m;
      if (node & 2) S.cursor = cursor_prev;  // the same scheduling cycle again (the full record of a compact one)
      cursor_prev = S.cursor;
      if (!schedule_pod<GEN>(c, job.P, prof, pi, smem, S, bins_cap, npt, &s, /*keep_norm=*/true, m,
                             NomView{nullptr, 0, -1, 0})) {  // the host refuses the service while pods are nominated
        if (threadIdx.x == 0) __hip_atomic_store(&box->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      if ((stamps & 1) && w == 0 && threadIdx.x == 0) st2 = wall_clock64();
      // this shard's node range of the requested rows -> the pinned host record, skipping the
      // segments the host already holds (equal to the previous evaluation's, which it copied)
      // (node bit 0 of an EVAL: the compact record, scores narrowed; else the full one)
      const bool compact = (node & 1) != 0;
      unsigned want = 0;
      for (int r = 0; r < SVC_ROWS; r++) want |= (fields & svc_row_field(r)) ? 1u << r : 0u;
      unsigned& hv = compact ? host_valid_c : host_valid;
      if (threadIdx.x == 0) shdr(smem).svc_ovf = 0;
      __syncthreads();  // the reset before any lane's overflow report
      const unsigned send = (stamps & 2) ? want  // experiment (KSS_SERVICE_NO_DIFF): every requested row
                                         : (want & ~hv) | svc_changed_rows(base, prev, L, N, want & hv, S.lo, S.hi,
                                                                           shdr(smem).svc_dirty);
      bool ovf = false;
      if (compact) svc_send<true>(base, crec_host, L, CL, N, send, S.lo, S.hi, ovf);
      else svc_send<false>(base, rec_host, L, CL, N, send, S.lo, S.hi, ovf);
      if (ovf) atomicOr(&shdr(smem).svc_ovf, 1u);
      if ((stamps & 1) && w == 0 && threadIdx.x == 0) st4 = wall_clock64();
      hv = want;  // the host's rows not asked for now no longer mirror the newest slot
      (compact ? host_valid : host_valid_c) = 0;  // nor does the other record
      if (w == 0 && threadIdx.x == 0) {
        if (job.cursor) *job.cursor = S.cursor;  // read by the next launch on this context
        KSS_GLOBAL int32_t* mm = reinterpret_cast<KSS_GLOBAL int32_t*>(&box->meta);
        mm[0] = m.chosen;
        mm[1] = m.n_feasible;
        mm[2] = m.scored;
        mm[3] = m.status;
        *reinterpret_cast<KSS_GLOBAL int64_t*>(mm + 4) = m.best_total;
      }
      __threadfence_system();  // this lane's record stores are visible to the host
      __syncthreads();
      if ((stamps & 1) && w == 0 && threadIdx.x == 0) {
        KSS_GLOBAL long long* sp = reinterpret_cast<KSS_GLOBAL long long*>(&box->stamp[0]);
        sp[0] = (long long)st0;
        sp[1] = (long long)st1;
        sp[2] = (long long)st2;
        sp[3] = wall_clock64();
        sp[4] = (long long)st4;
      }
      if (threadIdx.x == 0) {
        const unsigned long long dv = (seq + 1) | (shdr(smem).svc_ovf ? SVC_DONE_OVF : 0ull);
        st_sys(&box->done[w], dv);
      }
    } else if (op == SVC_COMMIT || op == SVC_ROLLBACK) {
      const int local = node - c.node_base;
      if (threadIdx.x == 0 && local >= S.lo && local < S.hi)
        commit_pod(c, job.P, job.P.pods[pi], local, op == SVC_COMMIT ? 1 : -1);
      if (threadIdx.x == 0 && job.P.pods[pi].vol_len > 0)  // the assume cache is global: every shard
        wffc_commit(c, job.P.reqs, job.P.terms, job.P.ints, job.P.vols, job.P.pods[pi], local,
                    op == SVC_COMMIT ? 1 : -1, [&](int key) { return c.label_value[(size_t)key * (size_t)c.N + local]; });
      __syncthreads();
    }
    if (threadIdx.x == 0) __hip_atomic_store(seen + w, seq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (c.nc64) {
    __syncthreads();
    cache_writeback(c, S.hi);
  }
  __threadfence_system();
  __syncthreads();
  if (w == 0 && threadIdx.x == 0) __hip_atomic_store(&box->running, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace kss
