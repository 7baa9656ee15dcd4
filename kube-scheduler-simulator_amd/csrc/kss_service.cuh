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
//               fences at system scope and stores done[w] = k + 1
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
};

// Every access to the pinned box and to the relay goes through address-space-1 pointers
// (global loads / stores: no flat address-space test on the polled words).
__device__ __forceinline__ void st_sys(KSS_GLOBAL unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Copy elements [lo, hi) of `rows` rows of ES-byte elements (row stride N) from the HBM
// record to the pinned host record (same layout).  Every row segment goes as 16-byte stores
// over its aligned interior (each narrower store to host memory is one fabric write of its own:
// MI355X_MICROARCH.md, 8-byte ones cost 2.7x and 2-byte ones 12.5x a 16-byte store per byte),
// and element stores for the at most 15 bytes at either end.  Both buffers are 16-byte
// aligned row blocks of the same layout (SlotLayout).
template <int ES>
__device__ __forceinline__ void svc_copy(const uint8_t* src, uint8_t* dst, size_t N, int r0, int rows, int lo, int hi) {
  using T = typename std::conditional<ES == 8, uint64_t, typename std::conditional<ES == 2, uint16_t, uint8_t>::type>::type;
  constexpr int V = 16 / ES;  // elements per 16-byte store
  const int tid = (int)threadIdx.x, nt = (int)blockDim.x;
  for (int r = r0; r < r0 + rows; r++) {
    const size_t base = (size_t)r * N;  // element offset of the row from the field's (16-byte aligned) start
    // elements [a, b) of the row start 16-byte aligned chunks: base + a is a multiple of V
    const size_t a0 = base + (size_t)lo, b0 = base + (size_t)hi;
    const size_t a = (a0 + V - 1) / V * V, b = b0 / V * V;
    KSS_GLOBAL const T* s = gp(reinterpret_cast<const T*>(src));
    KSS_GLOBAL T* d = gp(reinterpret_cast<T*>(dst));
    if (a < b) {
      KSS_GLOBAL const uint4* s4 = gp(reinterpret_cast<const uint4*>(src)) + a / V;
      KSS_GLOBAL uint4* d4 = gp(reinterpret_cast<uint4*>(dst)) + a / V;
      for (int i = tid; i < (int)((b - a) / V); i += nt) {
        const uint4 x = make_uint4(s4[i].x, s4[i].y, s4[i].z, s4[i].w);
        d4[i].x = x.x;  // member stores of one 16-byte value: the compiler merges them into one dwordx4
        d4[i].y = x.y;
        d4[i].z = x.z;
        d4[i].w = x.w;
      }
      for (int i = tid; i < (int)(a - a0); i += nt) d[a0 + i] = s[a0 + i];  // head
      for (int i = tid; i < (int)(b0 - b); i += nt) d[b + i] = s[b + i];    // tail
    } else {
      for (int i = tid; i < (int)(b0 - a0); i += nt) d[a0 + i] = s[a0 + i];
    }
  }
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

template <bool GEN>
__device__ void service_loop(DevCluster c, const DevJob& job, const kss_profile& prof, int W, int npt, int bins_cap,
                             int cache_keys, unsigned long long* gran, int* err, SvcBox* box_flat,
                             unsigned long long* relay_flat, unsigned long long* seen_flat, uint8_t* rec_host,
                             unsigned long long seq, unsigned epoch0, int stamps, long long* smem) {
  KSS_GLOBAL SvcBox* box = gp(box_flat);
  KSS_GLOBAL unsigned long long* relay = gp(relay_flat);
  KSS_GLOBAL unsigned long long* seen = gp(seen_flat);
  const int w = blockIdx.x;
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
  int* cmd = shdr(smem).cmd;
  if (w == 0 && threadIdx.x == 0) __hip_atomic_store(&box->running, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  unsigned long long st0 = 0, st1 = 0, st2 = 0;  // diagnostic clocks of shard 0's lane 0 (stamps)
  unsigned long long seen_min = seq;              // shard 0: every shard has taken the commands below this
  int parity = 0;                                 // the record slot of the next evaluation
  unsigned host_valid = 0;  // rows (bit r) whose host segment equals the last evaluation's slot
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
        __hip_atomic_store(slot + 1, svc_w1(seq, node), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(slot, svc_w0(seq, op, fields, pod), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    if (op == SVC_EVAL) {
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
      if (!schedule_pod<GEN>(c, job.P, prof, pi, smem, S, bins_cap, npt, &s, /*keep_norm=*/true, m)) {
        if (threadIdx.x == 0) __hip_atomic_store(&box->err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      if (stamps && w == 0 && threadIdx.x == 0) st2 = wall_clock64();
      // this shard's node range of the requested rows -> the pinned host record, skipping the
      // segments the host already holds (equal to the previous evaluation's, which it copied)
      unsigned want = 0;
      for (int r = 0; r < SVC_ROWS; r++) want |= (fields & svc_row_field(r)) ? 1u << r : 0u;
      const unsigned send = (want & ~host_valid) | svc_changed_rows(base, prev, L, N, want & host_valid, S.lo, S.hi,
                                                                    shdr(smem).svc_dirty);
      for (int r = 0; r < SVC_ROWS; r++) {
        if (!((send >> r) & 1u)) continue;
        int es = 0, fr = 0;
        const size_t o = svc_field(L, r, fr, es);
        if (es == 1) svc_copy<1>(base + o, rec_host + o, N, fr, 1, S.lo, S.hi);
        else if (es == 2) svc_copy<2>(base + o, rec_host + o, N, fr, 1, S.lo, S.hi);
        else svc_copy<8>(base + o, rec_host + o, N, fr, 1, S.lo, S.hi);
      }
      host_valid = want;  // the host's rows not asked for now no longer mirror the newest slot
      if (w == 0 && threadIdx.x == 0) {
        KSS_GLOBAL int32_t* mm = reinterpret_cast<KSS_GLOBAL int32_t*>(&box->meta);
        mm[0] = m.chosen;
        mm[1] = m.n_feasible;
        mm[2] = m.scored;
        mm[3] = m.status;
        *reinterpret_cast<KSS_GLOBAL int64_t*>(mm + 4) = m.best_total;
      }
      __threadfence_system();  // this lane's record stores are visible to the host
      __syncthreads();
      if (stamps && w == 0 && threadIdx.x == 0) {
        KSS_GLOBAL long long* sp = reinterpret_cast<KSS_GLOBAL long long*>(&box->stamp[0]);
        sp[0] = (long long)st0;
        sp[1] = (long long)st1;
        sp[2] = (long long)st2;
        sp[3] = wall_clock64();
      }
      if (threadIdx.x == 0) st_sys(&box->done[w], seq + 1);
    } else if (op == SVC_COMMIT || op == SVC_ROLLBACK) {
      const int local = node - c.node_base;
      if (threadIdx.x == 0 && local >= S.lo && local < S.hi)
        commit_pod(c, job.P, job.P.pods[pi], local, op == SVC_COMMIT ? 1 : -1);
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
