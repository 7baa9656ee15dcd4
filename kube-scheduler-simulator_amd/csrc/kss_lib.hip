// kss_lib.hip — C ABI of libkss.so (include/kss.h): device context, snapshot upload,
// and the launches of the gfx950 scheduling kernels.
//
// Kernel map:
//   k_schedule   one workgroup per cluster; sequential pods; every phase of the
//                scheduling cycle in the workgroup (kss_sched.cuh).  Used for the
//                sequential batch (kss_schedule_batch), the drop-in per-pod call
//                (kss_eval_pod, no commit) and the what-if scenario sweep
//                (kss_schedule_scenarios, grid = #scenarios).
//   k_simple     batches without PodTopologySpread / InterPodAffinity programs and
//                without a result record: node rows in registers, pod programs as
//                LDS blobs, one exchange per pod (kss_simple.cuh).
//   k_commit     one lane: AssumePod / ForgetPod delta on one node row.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "kss_host.h"
#include "kss_sched.cuh"
#include "kss_simple.cuh"
#include "kss_axis.cuh"

using namespace kss;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                        \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) return fail(KSS_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// per-pod output slot layout (record format), N nodes
struct SlotLayout {
  size_t fail, detail, raw, norm, total, bytes;
  __host__ __device__ explicit SlotLayout(size_t N) {
    fail = 0;
    detail = align_up(N, 256);
    raw = align_up(detail + 2 * N, 256);
    norm = raw + 8 * KSS_NSCORE * N;
    total = norm + 8 * KSS_NSCORE * N;
    bytes = align_up(total + 8 * N, 256);
  }
};

// one workgroup's job
struct DevJob {
  DevCluster c;
  DevPods P;
  int32_t n_pods;
  int32_t commit;     // apply AssumePod after each pod
  int32_t keep_norm;  // write norm/total into the slot(s)
  int32_t record;     // one slot per pod (else slot 0 reused)
  uint8_t* slots;
  size_t slot_bytes;
  int32_t* chosen;
  PodMeta* meta;
  const uint8_t* blobs;  // k_simple: serialized pod programs, blob_stride bytes each
  int32_t blob_stride;
};

}  // namespace

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
// grid = n_jobs * W; workgroup b serves shard (b % W) of cluster (b / W); each lane
// owns npt node slots.
template <bool GEN>
__global__ __launch_bounds__(KSS_MAX_THREADS) void k_schedule(const DevJob* __restrict__ jobs, kss_profile prof,
                                                              int W, int npt, int bins_cap, int cache_keys,
                                                              unsigned long long* gran, int* err,
                                                              unsigned long long* stamps) {
  extern __shared__ __attribute__((aligned(16))) long long smem[];
  const int ji = blockIdx.x / W, w = blockIdx.x % W;
  const DevJob job = jobs[ji];  // by value: the descriptors stay in registers for the whole launch
  DevCluster c = job.c;
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
  S.epoch = 0;
  S.gran = gran ? gran + (size_t)ji * 2 * W * 2 * XW_MAX : nullptr;
  S.err = err;
  S.stamps = nullptr;
  const bool want_out = job.record || job.keep_norm;
  // shard node cache: the hot node columns stay in LDS for the whole launch
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
  for (int pi = 0; pi < job.n_pods; pi++) {
    uint8_t* base = job.slots + (job.record ? (size_t)pi * job.slot_bytes : 0);
    Slot s;
    s.fail = base + L.fail;
    s.detail = (uint16_t*)(base + L.detail);
    s.raw = (int64_t*)(base + L.raw);
    s.norm = (int64_t*)(base + L.norm);
    s.total = (int64_t*)(base + L.total);
    PodMeta m;
    S.stamps = (stamps && ji == 0 && w == 0 && pi < KSS_NSTAMP_PODS) ? stamps + (size_t)pi * 8 : nullptr;
    KSS_STAMP(S, 0);
    if (!schedule_pod<GEN>(c, job.P, prof, pi, smem, S, bins_cap, npt, want_out ? &s : nullptr, job.keep_norm != 0, m))
      return;  // exchange timeout: the error word is set, leave the launch
    if (threadIdx.x == 0) {
      if (w == 0) {
        if (job.chosen) job.chosen[pi] = m.chosen;
        if (job.meta) job.meta[pi] = m;
      }
      const int local = m.chosen - c.node_base;
      if (job.commit && m.chosen >= 0 && local >= S.lo && local < S.hi) commit_pod(c, job.P, job.P.pods[pi], local, 1);
    }
    __syncthreads();
    KSS_STAMP(S, 6);
  }
  if (c.nc64 && job.commit) cache_writeback(c, S.hi);
}

// grid = n_jobs * W, as k_schedule; each shard's nodes live in LDS (cap slots).
// DEF: the profile is the v1.26 default, folded into the code.
template <bool DEF>
__global__ __launch_bounds__(KSS_MAX_THREADS) void k_simple(const DevJob* __restrict__ jobs, kss_profile prof, int W,
                                                            int cap, unsigned long long* gran, int* err,
                                                            unsigned long long* stamps) {
  extern __shared__ __attribute__((aligned(16))) long long smem[];
  const int ji = blockIdx.x / W, w = blockIdx.x % W;
  const DevJob job = jobs[ji];
  const kss_profile P = DEF ? default_profile_c() : prof;
  simple_schedule(job.c, job.blobs, job.blob_stride, job.n_pods, job.chosen, job.meta, P, W, w, cap,
                  gran ? gran + (size_t)ji * 2 * W * SX_VALS : nullptr, err, ji == 0 ? stamps : nullptr, smem);
}

__global__ void k_commit(DevCluster c, DevPods P, int pi, int local, int sign) {
  if (threadIdx.x == 0 && blockIdx.x == 0) commit_pod(c, P, P.pods[pi], local, sign);
}

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    size_t nb = std::max(bytes, (size_t)4096);
    if (hipMalloc(&p, nb) != hipSuccess) return fail(KSS_E_NOMEM, "hipMalloc failed");
    cap = nb;
    return 0;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Per-batch LDS / exchange sizing: the host restatement of make_plan's bin counts.
struct PlanNeeds {
  int bins_cap = 0;  // max over pods of histogram + presence bins
  int xw = 0;        // max exchange payload length (values) over pods and exchanges
  bool general = false;  // some pod carries spread / inter-pod-affinity programs
};

struct kss_ctx {
  kss_config cfg{};
  kss_profile prof{};
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::mutex mu;  // rollback may arrive from the binding goroutine
  // cluster
  bool loaded = false;
  kss_cluster host{};  // sizes only (pointers not retained)
  DevCluster dc{};
  DevBuf cluster_buf;
  DevBuf pristine_buf;  // load-time copy of the mutable columns (kss_reset_node_state)
  size_t mut_bytes[5] = {0, 0, 0, 0, 0};
  size_t pristine_off[5] = {0, 0, 0, 0, 0};
  // pods
  DevBuf pod_buf;      // staged pod programs (kss_stage_pods / kss_schedule_batch)
  DevPods dp{};
  int staged_n = -1;   // pods staged in pod_buf (-1: none)
  DevBuf tmp_pod_buf;  // eval / commit / rollback uploads (never clobber the staged batch)
  DevPods tdp{};
  // outputs
  DevBuf slot_buf, meta_buf, chosen_buf, job_buf;
  size_t slot_bytes = 0;
  int recorded = 0;
  std::vector<PodMeta> meta_host;
  double last_ms = 0;
  int last_launches = 0;
  kss_host_names names;
  // host copies of the per-key tables (plan sizing), and the exchange buffers
  std::vector<int32_t> key_card_h;
  std::vector<uint32_t> key_flags_h;
  DevBuf gran_buf, err_buf;
  int n_cu = 0;
  int force_w = 0;            // KSS_SHARDS env override (tuning / tests)
  int nodes_per_shard = 128;  // KSS_NODES_PER_SHARD (C2 sweep: 128 > 256 > 512 nodes per shard)
  int pref_threads = 256;     // KSS_THREADS
  PlanNeeds staged_need;
  int last_geom[3] = {0, 0, 0};
  const char* stamps_file = nullptr;  // KSS_STAMPS_FILE: dump per-phase timestamps of each launch
  DevBuf stamp_buf;
  // staged pod programs serialized for k_simple (blob_stride 0: some pod needs k_schedule)
  DevBuf blob_buf;
  std::vector<uint8_t> blob_host;
  int blob_stride = 0;
  bool no_simple = false;  // KSS_NO_SIMPLE: always launch k_schedule
  int last_kernel = 0;     // 0 k_schedule, 1 k_simple
  int meta_n = 0;          // pods with an outcome in meta_host
  bool small_values = false;  // every allocatable cpu/mem/eph < 2^46: k_simple's divisions stay below 2^53
  bool axis_meta_dirty = false;  // meta_buf holds node-axis outcomes not yet copied to meta_host
  DevBuf axis_cv;
  int axis_max_blocks = 0;  // KSS_AXIS_BLOCKS: cap on the node-axis grid (tuning)
  int axis_no_fold = 0;     // KSS_AXIS_NO_FOLD: timing experiment only, statistics not folded (wrong results)             // node-axis sharding: [5][N] per-row verdict + raw scores of the current pod
};

namespace {

// Copy a host podset into a device buffer; fills dp with device pointers.
int upload_podset(hipStream_t st, DevBuf& buf, const kss_podset* ps, DevPods& dp) {
  const size_t sz_pods = sizeof(kss_pod) * (size_t)std::max(ps->n_pods, 1);
  const size_t sz_reqs = sizeof(kss_req) * (size_t)std::max(ps->n_reqs, 1);
  const size_t sz_terms = sizeof(kss_term) * (size_t)std::max(ps->n_terms, 1);
  const size_t sz_spr = sizeof(kss_spread) * (size_t)std::max(ps->n_spreads, 1);
  const size_t sz_ipa = sizeof(kss_ipa) * (size_t)std::max(ps->n_ipa, 1);
  const size_t sz_ints = sizeof(int32_t) * (size_t)std::max(ps->n_ints, 1);
  size_t o_pods = 0, o_reqs = align_up(o_pods + sz_pods, 256), o_terms = align_up(o_reqs + sz_reqs, 256),
         o_spr = align_up(o_terms + sz_terms, 256), o_ipa = align_up(o_spr + sz_spr, 256),
         o_ints = align_up(o_ipa + sz_ipa, 256), total = align_up(o_ints + sz_ints, 256);
  int rc = buf.ensure(total);
  if (rc) return rc;
  char* b = (char*)buf.p;
  if (ps->n_pods) HIP_TRY(hipMemcpyAsync(b + o_pods, ps->pods, sizeof(kss_pod) * ps->n_pods, hipMemcpyHostToDevice, st));
  if (ps->n_reqs) HIP_TRY(hipMemcpyAsync(b + o_reqs, ps->reqs, sizeof(kss_req) * ps->n_reqs, hipMemcpyHostToDevice, st));
  if (ps->n_terms) HIP_TRY(hipMemcpyAsync(b + o_terms, ps->terms, sizeof(kss_term) * ps->n_terms, hipMemcpyHostToDevice, st));
  if (ps->n_spreads) HIP_TRY(hipMemcpyAsync(b + o_spr, ps->spreads, sizeof(kss_spread) * ps->n_spreads, hipMemcpyHostToDevice, st));
  if (ps->n_ipa) HIP_TRY(hipMemcpyAsync(b + o_ipa, ps->ipa, sizeof(kss_ipa) * ps->n_ipa, hipMemcpyHostToDevice, st));
  if (ps->n_ints) HIP_TRY(hipMemcpyAsync(b + o_ints, ps->ints, sizeof(int32_t) * ps->n_ints, hipMemcpyHostToDevice, st));
  dp.pods = (const kss_pod*)(b + o_pods);
  dp.reqs = (const kss_req*)(b + o_reqs);
  dp.terms = (const kss_term*)(b + o_terms);
  dp.spreads = (const kss_spread*)(b + o_spr);
  dp.ipa = (const kss_ipa*)(b + o_ipa);
  dp.ints = (const int32_t*)(b + o_ints);
  return 0;
}

// Validate podset references against the cluster shape (a malformed program must
// never reach the kernel: out-of-range ids would fault the device).
int validate(const kss_cluster* cl, const kss_podset* ps, int n) {
  if (n < 0 || n > ps->n_pods) return fail(KSS_E_INVAL, "pod count out of range");
  auto in = [](int64_t off, int64_t len, int64_t cap) { return off >= 0 && len >= 0 && off + len <= cap; };
  for (int i = 0; i < ps->n_reqs; i++) {
    const kss_req& r = ps->reqs[i];
    const bool keyed = r.op >= KSS_OP_MASK && r.op <= KSS_OP_LT;
    if (r.op < KSS_OP_FALSE || r.op > KSS_OP_NAME_NOTIN) return fail(KSS_E_INVAL, "bad requirement op");
    if (keyed && (r.key < 0 || r.key >= cl->n_label_keys)) return fail(KSS_E_INVAL, "requirement key out of range");
    if ((r.op == KSS_OP_IN || r.op == KSS_OP_NOTIN) && !in(r.list_off, r.list_len, ps->n_ints))
      return fail(KSS_E_INVAL, "requirement list out of range");
  }
  for (int i = 0; i < ps->n_terms; i++)
    if (!in(ps->terms[i].req_off, ps->terms[i].req_len, ps->n_reqs)) return fail(KSS_E_INVAL, "term out of range");
  for (int i = 0; i < ps->n_spreads; i++) {
    const kss_spread& s = ps->spreads[i];
    if (s.key < 0 || s.key >= cl->n_label_keys) return fail(KSS_E_INVAL, "spread key out of range");
    if (!in(s.cls_off, s.cls_len, ps->n_ints)) return fail(KSS_E_INVAL, "spread class list out of range");
    for (int j = 0; j < s.cls_len; j++)
      if (ps->ints[s.cls_off + j] < 0 || ps->ints[s.cls_off + j] >= cl->n_classes) return fail(KSS_E_INVAL, "class id out of range");
    if (!(cl->key_flags[s.key] & (KSS_KEY_UNIQUE | KSS_KEY_HOSTNAME)) && cl->key_card[s.key] + 1 > KSS_MAX_BINS)
      return fail(KSS_E_UNSUPPORTED, "non-unique topology key with more than KSS_MAX_BINS domains");
  }
  for (int i = 0; i < ps->n_ipa; i++) {
    const kss_ipa& e = ps->ipa[i];
    if (e.key < 0 || e.key >= cl->n_label_keys) return fail(KSS_E_INVAL, "ipa key out of range");
    if (!in(e.row_off, e.row_len, ps->n_ints)) return fail(KSS_E_INVAL, "ipa rows out of range");
    const bool terms = e.kind == KSS_IPA_EXISTING_ANTI || e.kind == KSS_IPA_SCORE_TERM;
    const int cap = terms ? cl->n_terms : cl->n_classes;
    for (int j = 0; j < e.row_len; j++)
      if (ps->ints[e.row_off + j] < 0 || ps->ints[e.row_off + j] >= cap) return fail(KSS_E_INVAL, "ipa row id out of range");
    if (!(cl->key_flags[e.key] & KSS_KEY_UNIQUE) && cl->key_card[e.key] + 1 > KSS_MAX_BINS)
      return fail(KSS_E_UNSUPPORTED, "non-unique topology key with more than KSS_MAX_BINS domains");
  }
  for (int i = 0; i < n; i++) {
    const kss_pod& p = ps->pods[i];
    if (!in(p.sel_off, p.sel_len, ps->n_reqs) || !in(p.aff_off, p.aff_len, ps->n_terms) ||
        !in(p.pref_off, p.pref_len, ps->n_terms) || !in(p.spread_off, (int64_t)p.n_hard + p.n_soft, ps->n_spreads) ||
        !in(p.ipa_off, p.ipa_len, ps->n_ipa) || !in(p.own_terms_off, p.own_terms_len, ps->n_ints))
      return fail(KSS_E_INVAL, "pod program out of range");
    if (p.names_len >= 0 && !in(p.names_off, p.names_len, ps->n_ints)) return fail(KSS_E_INVAL, "pod names out of range");
    if (p.cls >= cl->n_classes) return fail(KSS_E_INVAL, "pod class out of range");
    for (int j = 0; j < p.own_terms_len; j++)
      if (ps->ints[p.own_terms_off + j] < 0 || ps->ints[p.own_terms_off + j] >= cl->n_terms)
        return fail(KSS_E_INVAL, "own term id out of range");
    if (p.n_hard > MAXH || p.n_soft > MAXS) return fail(KSS_E_UNSUPPORTED, "too many spread constraints for the device path");
  }
  return 0;
}

// One pod program as a position-independent blob for k_simple (kss_simple.cuh): the pod
// record, then only the requirements / terms / ints it references, every offset rebased
// into the blob.  Writes to dst when given; returns the blob size.
size_t serialize_pod(const kss_podset* ps, int i, uint8_t* dst) {
  const kss_pod& src = ps->pods[i];
  kss_pod q = src;
  std::vector<kss_req> R;
  std::vector<kss_term> T;
  std::vector<int32_t> I;
  auto add_req = [&](const kss_req& r0) {
    kss_req r = r0;
    if (r.op == KSS_OP_IN || r.op == KSS_OP_NOTIN) {
      r.list_off = (int32_t)I.size();
      I.insert(I.end(), ps->ints + r0.list_off, ps->ints + r0.list_off + r0.list_len);
    }
    R.push_back(r);
  };
  auto add_terms = [&](int off, int len) {
    const int first = (int)T.size();
    T.insert(T.end(), ps->terms + off, ps->terms + off + len);
    for (int t = 0; t < len; t++) {
      const kss_term& s0 = ps->terms[off + t];
      T[first + t].req_off = (int32_t)R.size();
      for (int k = 0; k < s0.req_len; k++) add_req(ps->reqs[s0.req_off + k]);
    }
    return first;
  };
  q.sel_off = 0;
  for (int k = 0; k < src.sel_len; k++) add_req(ps->reqs[src.sel_off + k]);
  q.aff_off = add_terms(src.aff_off, src.aff_len);
  q.pref_off = add_terms(src.pref_off, src.pref_len);
  if (src.names_len >= 0) {
    q.names_off = (int32_t)I.size();
    I.insert(I.end(), ps->ints + src.names_off, ps->ints + src.names_off + src.names_len);
  }
  q.own_terms_off = (int32_t)I.size();
  I.insert(I.end(), ps->ints + src.own_terms_off, ps->ints + src.own_terms_off + src.own_terms_len);
  q.spread_off = 0;
  q.ipa_off = 0;
  BlobHdr h{};
  const size_t ro = blob_body_off(), to = ro + align_up(R.size() * sizeof(kss_req), 16),
               io = to + align_up(T.size() * sizeof(kss_term), 16), end = io + align_up(I.size() * sizeof(int32_t), 16);
  h.req_off = (int32_t)ro;
  h.term_off = (int32_t)to;
  h.ints_off = (int32_t)io;
  h.n_reqs = (int32_t)R.size();
  h.n_terms = (int32_t)T.size();
  h.n_ints = (int32_t)I.size();
  if (dst) {
    memcpy(dst, &q, sizeof(q));
    memcpy(dst + blob_hdr_off(), &h, sizeof(h));
    if (!R.empty()) memcpy(dst + ro, R.data(), R.size() * sizeof(kss_req));
    if (!T.empty()) memcpy(dst + to, T.data(), T.size() * sizeof(kss_term));
    if (!I.empty()) memcpy(dst + io, I.data(), I.size() * sizeof(int32_t));
  }
  return end;
}

// Blobs of every pod of a (validated) podset at one stride; returns the stride, or 0 when
// some pod needs k_schedule (spread / inter-pod programs, or a program over BLOB_MAX).
int build_blobs(const kss_podset* ps, std::vector<uint8_t>& out) {
  size_t mx = 16;
  for (int i = 0; i < ps->n_pods; i++) {
    const kss_pod& p = ps->pods[i];
    if (p.n_hard | p.n_soft | p.ipa_len) return 0;
    mx = std::max(mx, serialize_pod(ps, i, nullptr));
  }
  const size_t stride = align_up(mx, 64);
  if (stride > (size_t)BLOB_MAX) return 0;
  out.assign(stride * (size_t)std::max(ps->n_pods, 1), 0);
  for (int i = 0; i < ps->n_pods; i++) serialize_pod(ps, i, out.data() + stride * (size_t)i);
  return (int)stride;
}

struct ClusterLayout {
  size_t o_alloc, o_req, o_nz, o_allowed, o_podc, o_flags, o_th, o_ts, o_to, o_lv, o_kb, o_kc, o_kf, o_ke, o_vi, o_vii,
      o_cc, o_tc, o_log, total;
  ClusterLayout(const kss_cluster* cl, int class_cap, int term_cap) {
    const size_t N = (size_t)cl->n_nodes;
    size_t o = 0;
    auto take = [&](size_t bytes) {
      size_t r = o;
      o = align_up(o + std::max(bytes, (size_t)8), 256);
      return r;
    };
    o_alloc = take(8 * KSS_NRES * N);
    o_req = take(8 * KSS_NRES * N);
    o_nz = take(8 * 2 * N);
    o_allowed = take(4 * N);
    o_podc = take(4 * N);
    o_flags = take(4 * N);
    o_th = take(8 * N);
    o_ts = take(8 * N);
    o_to = take((size_t)KSS_TAINT_ORDER * N);
    o_lv = take(4 * (size_t)cl->n_label_keys * N);
    o_kb = take(4 * (size_t)cl->n_label_keys);
    o_kc = take(4 * (size_t)cl->n_label_keys);
    o_kf = take(4 * (size_t)cl->n_label_keys);
    o_ke = take(4 * (size_t)cl->n_label_keys);
    o_vi = take(8 * (size_t)cl->n_label_values);
    o_vii = take((size_t)cl->n_label_values);
    o_cc = take(4 * (size_t)class_cap * N);
    o_tc = take(4 * (size_t)term_cap * N);
    o_log = take(8 * (N + 3));
    total = o;
  }
};

int fill_cluster(hipStream_t st, const kss_cluster* cl, int class_cap, int term_cap, char* b, const ClusterLayout& L,
                 DevCluster& dc, std::vector<double>& logtab) {
  const size_t N = (size_t)cl->n_nodes;
  auto cp = [&](size_t off, const void* src, size_t bytes) -> int {
    if (bytes && src) HIP_TRY(hipMemcpyAsync(b + off, src, bytes, hipMemcpyHostToDevice, st));
    return 0;
  };
  int rc = 0;
  rc |= cp(L.o_alloc, cl->alloc, 8 * KSS_NRES * N);
  rc |= cp(L.o_req, cl->requested, 8 * KSS_NRES * N);
  rc |= cp(L.o_nz, cl->nonzero, 8 * 2 * N);
  rc |= cp(L.o_allowed, cl->allowed_pods, 4 * N);
  rc |= cp(L.o_podc, cl->pod_count, 4 * N);
  rc |= cp(L.o_flags, cl->node_flags, 4 * N);
  rc |= cp(L.o_th, cl->taint_hard, 8 * N);
  rc |= cp(L.o_ts, cl->taint_soft, 8 * N);
  rc |= cp(L.o_to, cl->taint_order, (size_t)KSS_TAINT_ORDER * N);
  rc |= cp(L.o_lv, cl->label_value, 4 * (size_t)cl->n_label_keys * N);
  rc |= cp(L.o_kb, cl->key_base, 4 * (size_t)cl->n_label_keys);
  rc |= cp(L.o_kc, cl->key_card, 4 * (size_t)cl->n_label_keys);
  rc |= cp(L.o_kf, cl->key_flags, 4 * (size_t)cl->n_label_keys);
  rc |= cp(L.o_ke, cl->key_empty, 4 * (size_t)cl->n_label_keys);
  rc |= cp(L.o_vi, cl->value_int, 8 * (size_t)cl->n_label_values);
  rc |= cp(L.o_vii, cl->value_is_int, (size_t)cl->n_label_values);
  if (class_cap) HIP_TRY(hipMemsetAsync(b + L.o_cc, 0, 4 * (size_t)class_cap * N, st));
  if (term_cap) HIP_TRY(hipMemsetAsync(b + L.o_tc, 0, 4 * (size_t)term_cap * N, st));
  rc |= cp(L.o_cc, cl->class_count, 4 * (size_t)cl->n_classes * N);
  rc |= cp(L.o_tc, cl->term_count, 4 * (size_t)cl->n_terms * N);
  logtab.resize(N + 3);
  for (size_t k = 0; k < N + 3; k++) logtab[k] = kss_go_log((double)(k + 2));
  rc |= cp(L.o_log, logtab.data(), 8 * (N + 3));
  if (rc) return rc;
  dc.N = cl->n_nodes;
  dc.n_scalar = cl->n_scalar;
  dc.n_keys = cl->n_label_keys;
  dc.n_classes = cl->n_classes;
  dc.n_terms = cl->n_terms;
  dc.node_base = cl->node_base;
  dc.class_cap = class_cap;
  dc.term_cap = term_cap;
  dc.alloc = (const int64_t*)(b + L.o_alloc);
  dc.requested = (int64_t*)(b + L.o_req);
  dc.nonzero = (int64_t*)(b + L.o_nz);
  dc.allowed_pods = (const int32_t*)(b + L.o_allowed);
  dc.pod_count = (int32_t*)(b + L.o_podc);
  dc.node_flags = (const uint32_t*)(b + L.o_flags);
  dc.taint_hard = (const uint64_t*)(b + L.o_th);
  dc.taint_soft = (const uint64_t*)(b + L.o_ts);
  dc.taint_order = (const uint8_t*)(b + L.o_to);
  dc.label_value = (const int32_t*)(b + L.o_lv);
  dc.key_base = (const int32_t*)(b + L.o_kb);
  dc.key_card = (const int32_t*)(b + L.o_kc);
  dc.key_flags = (const uint32_t*)(b + L.o_kf);
  dc.key_empty = (const int32_t*)(b + L.o_ke);
  dc.value_int = (const int64_t*)(b + L.o_vi);
  dc.value_is_int = (const uint8_t*)(b + L.o_vii);
  dc.class_count = (int32_t*)(b + L.o_cc);
  dc.term_count = (int32_t*)(b + L.o_tc);
  dc.log_table = (const double*)(b + L.o_log);
  return 0;
}

int check_cluster(const kss_cluster* cl) {
  if (!cl || cl->n_nodes < 0) return fail(KSS_E_INVAL, "null cluster");
  if (cl->n_scalar < 0 || cl->n_scalar > KSS_MAX_SCALAR) return fail(KSS_E_INVAL, "n_scalar out of range");
  if (cl->n_taints < 0 || cl->n_taints > KSS_MAX_TAINTS) return fail(KSS_E_INVAL, "n_taints out of range");
  if (cl->n_nodes > 0 && (!cl->alloc || !cl->requested || !cl->nonzero || !cl->allowed_pods || !cl->pod_count ||
                          !cl->node_flags || !cl->taint_hard || !cl->taint_soft || !cl->taint_order))
    return fail(KSS_E_INVAL, "missing node column");
  for (int k = 0; k < cl->n_label_keys; k++) {
    if (cl->key_base[k] < 0 || cl->key_base[k] + cl->key_card[k] > cl->n_label_values)
      return fail(KSS_E_INVAL, "key value table out of range");
    if (cl->key_empty[k] < 0 || cl->key_empty[k] > cl->key_card[k]) return fail(KSS_E_INVAL, "key_empty out of range");
  }
  const size_t N = (size_t)cl->n_nodes;
  for (size_t i = 0; i < (size_t)cl->n_label_keys * N; i++) {
    const int k = (int)(i / (N ? N : 1));
    if (cl->label_value[i] < -1 || cl->label_value[i] >= cl->key_card[k]) return fail(KSS_E_INVAL, "label value id out of range");
  }
  for (size_t i = 0; i < N * KSS_TAINT_ORDER; i++)
    if (cl->taint_order[i] != 0xFF && cl->taint_order[i] >= cl->n_taints) return fail(KSS_E_INVAL, "taint id out of range");
  return 0;
}

// Profile limits of the device path.  percentageOfNodesToScore must be 100 (SURVEY 8a
// a1).  The selectHost key packs TotalScore into the upper 32 bits of a signed 64-bit
// key, so Σ weight·MaxNodeScore over the enabled score plugins must stay below 2^31; the
// reference accepts any positive int32 weight whose sum fits int64 (framework.go
// MaxTotalScore), so larger profiles are refused here rather than mis-ranked.
int check_profile(const kss_profile* prof) {
  if (prof->pct_nodes_to_score != 100 && prof->pct_nodes_to_score != 0)
    return fail(KSS_E_UNSUPPORTED, "percentageOfNodesToScore must be 100 (SURVEY 8a a1)");
  int64_t sum = 0;
  for (int s = 0; s < KSS_NSCORE; s++) {
    if (!((prof->score_enabled >> s) & 1u)) continue;
    if (prof->weight[s] < 0) return fail(KSS_E_INVAL, "negative score plugin weight");
    sum += (int64_t)prof->weight[s] * 100;
  }
  if (sum >= (1ll << 31)) return fail(KSS_E_UNSUPPORTED, "sum of score weights x 100 must be below 2^31 on the device path");
  if (prof->fit_n < 0 || prof->fit_n > 4 || prof->ba_n < 0 || prof->ba_n > 4)
    return fail(KSS_E_INVAL, "scoring resource count out of range");
  for (int i = 0; i < prof->fit_n; i++)
    if (prof->fit_res[i] < 0 || prof->fit_res[i] >= KSS_NRES || prof->fit_weight[i] < 0)
      return fail(KSS_E_INVAL, "NodeResourcesFit scoring resource out of range");
  for (int i = 0; i < prof->ba_n; i++)
    if (prof->ba_res[i] < 0 || prof->ba_res[i] >= KSS_NRES)
      return fail(KSS_E_INVAL, "BalancedAllocation resource out of range");
  return 0;
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

int kss_abi_version(void) { return KSS_ABI_VERSION; }
const char* kss_last_error(void) { return g_err.c_str(); }

int kss_abi_sizes(int32_t* out, int32_t n) {
  const int32_t s[] = {(int32_t)sizeof(kss_cluster), (int32_t)sizeof(kss_req),     (int32_t)sizeof(kss_term),
                       (int32_t)sizeof(kss_spread),  (int32_t)sizeof(kss_ipa),     (int32_t)sizeof(kss_pod),
                       (int32_t)sizeof(kss_podset),  (int32_t)sizeof(kss_profile), (int32_t)sizeof(kss_pod_result),
                       (int32_t)sizeof(kss_config),  (int32_t)sizeof(kss_names),   (int32_t)sizeof(kss_synth)};
  const int32_t k = (int32_t)(sizeof(s) / sizeof(s[0]));
  for (int i = 0; i < n && i < k; i++) out[i] = s[i];
  return k;
}

kss_ctx* kss_create(const kss_config* cfg, const kss_profile* prof) {
  if (!cfg || !prof) {
    fail(KSS_E_INVAL, "null config/profile");
    return nullptr;
  }
  if (check_profile(prof)) return nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    fail(KSS_E_DEVICE, "no HIP device visible");
    return nullptr;
  }
  if (cfg->device < 0 || cfg->device >= ndev) {
    fail(KSS_E_INVAL, "device ordinal out of range");
    return nullptr;
  }
  kss_ctx* ctx = new kss_ctx();
  ctx->cfg = *cfg;
  ctx->prof = *prof;
  hipDeviceProp_t dp{};
  if (hipGetDeviceProperties(&dp, cfg->device) == hipSuccess) ctx->n_cu = dp.multiProcessorCount;
  if (ctx->n_cu <= 0) ctx->n_cu = 1;
  if (const char* e = getenv("KSS_SHARDS")) ctx->force_w = std::max(0, atoi(e));
  ctx->stamps_file = getenv("KSS_STAMPS_FILE");
  ctx->no_simple = getenv("KSS_NO_SIMPLE") != nullptr;
  if (const char* e = getenv("KSS_AXIS_BLOCKS")) ctx->axis_max_blocks = std::max(0, atoi(e));
  ctx->axis_no_fold = getenv("KSS_AXIS_NO_FOLD") != nullptr;
  if (const char* e = getenv("KSS_NODES_PER_SHARD")) ctx->nodes_per_shard = std::max(1, atoi(e));
  if (const char* e = getenv("KSS_THREADS")) ctx->pref_threads = std::min(KSS_MAX_THREADS, std::max(64, atoi(e)));
  if (hipSetDevice(cfg->device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess) {
    fail(KSS_E_DEVICE, "stream/event creation failed");
    delete ctx;
    return nullptr;
  }
  return ctx;
}

void kss_destroy(kss_ctx* ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->cfg.device);
  if (ctx->stream) hipStreamSynchronize(ctx->stream);
  ctx->cluster_buf.release();
  ctx->pristine_buf.release();
  ctx->pod_buf.release();
  ctx->tmp_pod_buf.release();
  ctx->slot_buf.release();
  ctx->meta_buf.release();
  ctx->chosen_buf.release();
  ctx->job_buf.release();
  ctx->blob_buf.release();
  ctx->stamp_buf.release();
  ctx->gran_buf.release();
  ctx->err_buf.release();
  ctx->axis_cv.release();
  if (ctx->ev0) hipEventDestroy(ctx->ev0);
  if (ctx->ev1) hipEventDestroy(ctx->ev1);
  if (ctx->stream) hipStreamDestroy(ctx->stream);
  delete ctx;
}

int kss_load_cluster(kss_ctx* ctx, const kss_cluster* cl) {
  if (!ctx) return fail(KSS_E_INVAL, "null ctx");
  int rc = check_cluster(cl);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  const int class_cap = std::max(cl->n_classes, ctx->cfg.class_capacity);
  const int term_cap = std::max(cl->n_terms, ctx->cfg.term_capacity);
  ClusterLayout L(cl, class_cap, term_cap);
  rc = ctx->cluster_buf.ensure(L.total);
  if (rc) return rc;
  std::vector<double> logtab;
  rc = fill_cluster(ctx->stream, cl, class_cap, term_cap, (char*)ctx->cluster_buf.p, L, ctx->dc, logtab);
  if (rc) return rc;
  // pristine copy of the mutable columns
  const size_t N = (size_t)cl->n_nodes;
  const size_t mb[5] = {8 * KSS_NRES * N, 8 * 2 * N, 4 * N, 4 * (size_t)class_cap * N, 4 * (size_t)term_cap * N};
  size_t tot = 0;
  for (int i = 0; i < 5; i++) {
    ctx->mut_bytes[i] = mb[i];
    ctx->pristine_off[i] = tot;
    tot = align_up(tot + mb[i], 256);
  }
  rc = ctx->pristine_buf.ensure(tot);
  if (rc) return rc;
  void* src[5] = {ctx->dc.requested, ctx->dc.nonzero, ctx->dc.pod_count, ctx->dc.class_count, ctx->dc.term_count};
  for (int i = 0; i < 5; i++)
    if (mb[i])
      HIP_TRY(hipMemcpyAsync((char*)ctx->pristine_buf.p + ctx->pristine_off[i], src[i], mb[i], hipMemcpyDeviceToDevice,
                             ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  ctx->host = *cl;
  {
    bool small = true;
    for (size_t i = 0; i < 3 * N && small; i++) small = cl->alloc[i] >= 0 && cl->alloc[i] < (1ll << 46);
    for (int i = 0; i < ctx->prof.fit_n && small; i++) small = ctx->prof.fit_weight[i] >= 0 && ctx->prof.fit_weight[i] < (1ll << 20);
    ctx->small_values = small;
  }
  ctx->key_card_h.assign(cl->key_card, cl->key_card + cl->n_label_keys);
  ctx->key_flags_h.assign(cl->key_flags, cl->key_flags + cl->n_label_keys);
  ctx->loaded = true;
  ctx->recorded = 0;
  ctx->meta_n = 0;
  ctx->axis_meta_dirty = false;
  ctx->staged_n = -1;
  return 0;
}

static bool same_profile(const kss_profile& a, const kss_profile& b);

int kss_load_cluster_rows(kss_ctx* ctx, const kss_cluster* cl, int32_t lo, int32_t hi) {
  if (!ctx) return fail(KSS_E_INVAL, "null ctx");
  int rc = check_cluster(cl);
  if (rc) return rc;
  if (lo < 0 || hi < lo || hi > cl->n_nodes) return fail(KSS_E_INVAL, "row range out of range");
  const size_t N = (size_t)cl->n_nodes, M = (size_t)(hi - lo);
  // column-blocked [attr][N] matrices: take columns [lo, hi) of every attribute row
  auto rows64 = [&](const int64_t* src, int nrow, std::vector<int64_t>& dst) {
    dst.resize(std::max<size_t>(nrow * M, 1));
    for (int r = 0; r < nrow; r++) std::copy(src + r * N + lo, src + r * N + hi, dst.begin() + r * M);
  };
  auto rows32 = [&](const int32_t* src, int nrow, std::vector<int32_t>& dst) {
    dst.resize(std::max<size_t>(nrow * M, 1));
    if (src)
      for (int r = 0; r < nrow; r++) std::copy(src + r * N + lo, src + r * N + hi, dst.begin() + r * M);
  };
  std::vector<int64_t> alloc, req, nz;
  std::vector<int32_t> allowed, podc, lv, cc, tc;
  rows64(cl->alloc, KSS_NRES, alloc);
  rows64(cl->requested, KSS_NRES, req);
  rows64(cl->nonzero, 2, nz);
  rows32(cl->allowed_pods, 1, allowed);
  rows32(cl->pod_count, 1, podc);
  rows32(cl->label_value, cl->n_label_keys, lv);
  rows32(cl->class_count, cl->n_classes, cc);
  rows32(cl->term_count, cl->n_terms, tc);
  std::vector<uint32_t> flags(cl->node_flags + lo, cl->node_flags + hi);
  std::vector<uint64_t> th(cl->taint_hard + lo, cl->taint_hard + hi), ts(cl->taint_soft + lo, cl->taint_soft + hi);
  std::vector<uint8_t> to(cl->taint_order + (size_t)lo * KSS_TAINT_ORDER, cl->taint_order + (size_t)hi * KSS_TAINT_ORDER);
  kss_cluster s = *cl;
  s.n_nodes = (int32_t)M;
  s.node_base = cl->node_base + lo;
  s.alloc = alloc.data();
  s.requested = req.data();
  s.nonzero = nz.data();
  s.allowed_pods = allowed.data();
  s.pod_count = podc.data();
  s.node_flags = flags.data();
  s.taint_hard = th.data();
  s.taint_soft = ts.data();
  s.taint_order = to.data();
  s.label_value = lv.data();
  s.class_count = cl->class_count ? cc.data() : nullptr;
  s.term_count = cl->term_count ? tc.data() : nullptr;
  return kss_load_cluster(ctx, &s);  // synchronous: the temporaries outlive the upload
}

static hipStream_t axis_stream(kss_ctx* ctx, void* stream) { return stream ? (hipStream_t)stream : ctx->stream; }

static int axis_check(kss_ctx* ctx, int32_t pod_index) {
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  if (pod_index < 0 || pod_index >= ctx->staged_n) return fail(KSS_E_INVAL, "pod index outside the staged pods");
  if (ctx->staged_need.general)
    return fail(KSS_E_UNSUPPORTED, "node-axis path: spread / inter-pod programs need the replicated domain histograms");
  return ctx->axis_cv.ensure(sizeof(int32_t) * 5 * (size_t)std::max(ctx->dc.N, 1));
}

static dim3 axis_grid(kss_ctx* ctx) {
  const int blocks = (ctx->dc.N + AXIS_THREADS - 1) / AXIS_THREADS;
  return dim3((unsigned)std::max(1, std::min(blocks, ctx->axis_max_blocks > 0 ? ctx->axis_max_blocks : 4 * ctx->n_cu)));
}

int kss_axis_eval(kss_ctx* ctx, int32_t pod_index, int64_t* stats_dev, const int64_t* prev_key_dev,
                  const int64_t* prev_gathered_dev, int32_t world, int64_t* key_zero_dev, int32_t* chosen_dev,
                  void* stream) {
  int rc = axis_check(ctx, pod_index);
  if (rc) return rc;
  if (!stats_dev || !key_zero_dev || world < 1) return fail(KSS_E_INVAL, "bad eval arguments");
  if (prev_key_dev && (pod_index < 1 || !prev_gathered_dev)) return fail(KSS_E_INVAL, "pending commit without a previous pod");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  rc = ctx->meta_buf.ensure(sizeof(PodMeta) * (size_t)std::max(ctx->staged_n, 1));
  if (rc) return rc;
  auto fn = same_profile(ctx->prof, default_profile_c()) ? k_axis_eval<true> : k_axis_eval<false>;
  hipLaunchKernelGGL(fn, axis_grid(ctx), dim3(AXIS_THREADS), 0, axis_stream(ctx, stream), ctx->dc, ctx->dp, ctx->prof,
                     pod_index, (int32_t*)ctx->axis_cv.p, (long long*)stats_dev, (const long long*)prev_key_dev,
                     (const long long*)prev_gathered_dev, world, (long long*)key_zero_dev, chosen_dev,
                     (PodMeta*)ctx->meta_buf.p, ctx->axis_no_fold);
  HIP_TRY(hipGetLastError());
  if (prev_key_dev) {
    ctx->meta_n = std::max(ctx->meta_n, (int)pod_index);
    ctx->axis_meta_dirty = true;
  }
  return 0;
}

int kss_axis_select(kss_ctx* ctx, const int64_t* gathered_dev, int32_t world, int64_t* key_dev, int64_t* stats_zero_dev,
                    void* stream) {
  int rc = axis_check(ctx, 0);
  if (rc) return rc;
  if (!gathered_dev || !key_dev || !stats_zero_dev || world < 1) return fail(KSS_E_INVAL, "bad select arguments");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  hipLaunchKernelGGL(k_axis_select, axis_grid(ctx), dim3(AXIS_THREADS), 0, axis_stream(ctx, stream), ctx->dc, ctx->prof,
                     (const int32_t*)ctx->axis_cv.p, (const long long*)gathered_dev, world, (long long*)key_dev,
                     (long long*)stats_zero_dev);
  HIP_TRY(hipGetLastError());
  return 0;
}

int kss_axis_commit(kss_ctx* ctx, int32_t pod_index, const int64_t* key_dev, const int64_t* gathered_dev, int32_t world,
                    int32_t* chosen_dev, void* stream) {
  int rc = axis_check(ctx, pod_index);
  if (rc) return rc;
  if (!key_dev || !gathered_dev || world < 1) return fail(KSS_E_INVAL, "bad commit arguments");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  rc = ctx->meta_buf.ensure(sizeof(PodMeta) * (size_t)std::max(ctx->staged_n, 1));
  if (rc) return rc;
  hipLaunchKernelGGL(k_axis_commit, dim3(1), dim3(64), 0, axis_stream(ctx, stream), ctx->dc, ctx->dp, pod_index,
                     (const long long*)key_dev, (const long long*)gathered_dev, world, chosen_dev,
                     (PodMeta*)ctx->meta_buf.p);
  HIP_TRY(hipGetLastError());
  ctx->meta_n = std::max(ctx->meta_n, pod_index + 1);
  ctx->axis_meta_dirty = true;
  return 0;
}

int kss_reset_node_state(kss_ctx* ctx) {
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  void* dst[5] = {ctx->dc.requested, ctx->dc.nonzero, ctx->dc.pod_count, ctx->dc.class_count, ctx->dc.term_count};
  for (int i = 0; i < 5; i++)
    if (ctx->mut_bytes[i])
      HIP_TRY(hipMemcpyAsync(dst[i], (char*)ctx->pristine_buf.p + ctx->pristine_off[i], ctx->mut_bytes[i],
                             hipMemcpyDeviceToDevice, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int kss_apply_node_delta(kss_ctx* ctx, const int32_t* idx, int32_t n, const int64_t* requested, const int64_t* nonzero,
                         const int32_t* pod_count) {
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  const size_t N = (size_t)ctx->dc.N;
  for (int i = 0; i < n; i++) {
    const int r0 = idx[i];
    if (r0 < 0 || (size_t)r0 >= N) return fail(KSS_E_INVAL, "delta row out of range");
    for (int r = 0; r < KSS_NRES; r++)
      HIP_TRY(hipMemcpyAsync(ctx->dc.requested + (size_t)r * N + r0, requested + (size_t)i * KSS_NRES + r, 8,
                             hipMemcpyHostToDevice, ctx->stream));
    for (int r = 0; r < 2; r++)
      HIP_TRY(hipMemcpyAsync(ctx->dc.nonzero + (size_t)r * N + r0, nonzero + (size_t)i * 2 + r, 8, hipMemcpyHostToDevice,
                             ctx->stream));
    HIP_TRY(hipMemcpyAsync(ctx->dc.pod_count + r0, pod_count + i, 4, hipMemcpyHostToDevice, ctx->stream));
  }
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int kss_read_node_state(kss_ctx* ctx, int64_t* requested, int64_t* nonzero, int32_t* pod_count, int32_t* class_count,
                        int32_t* term_count) {
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  const size_t N = (size_t)ctx->dc.N;
  if (requested) HIP_TRY(hipMemcpyAsync(requested, ctx->dc.requested, 8 * KSS_NRES * N, hipMemcpyDeviceToHost, ctx->stream));
  if (nonzero) HIP_TRY(hipMemcpyAsync(nonzero, ctx->dc.nonzero, 8 * 2 * N, hipMemcpyDeviceToHost, ctx->stream));
  if (pod_count) HIP_TRY(hipMemcpyAsync(pod_count, ctx->dc.pod_count, 4 * N, hipMemcpyDeviceToHost, ctx->stream));
  if (class_count && ctx->host.n_classes)
    HIP_TRY(hipMemcpyAsync(class_count, ctx->dc.class_count, 4 * (size_t)ctx->host.n_classes * N, hipMemcpyDeviceToHost, ctx->stream));
  if (term_count && ctx->host.n_terms)
    HIP_TRY(hipMemcpyAsync(term_count, ctx->dc.term_count, 4 * (size_t)ctx->host.n_terms * N, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

static PlanNeeds plan_needs(const int32_t* key_card, const uint32_t* key_flags, const kss_podset* ps, int n) {
  PlanNeeds r;
  r.xw = 12;  // the filter exchange's scalars
  for (int i = 0; i < n; i++) {
    const kss_pod& p = ps->pods[i];
    int bins = 0, hp = 0, sp = 0;
    if (p.n_hard | p.n_soft | p.ipa_len) r.general = true;
    for (int h = 0; h < p.n_hard && h < MAXH; h++) {
      const int key = ps->spreads[p.spread_off + h].key;
      if (!(key_flags[key] & KSS_KEY_UNIQUE)) {
        bins += key_card[key] + 1;
        hp += key_card[key] + 1;
      }
    }
    for (int q = 0; q < p.n_soft && q < MAXS; q++) {
      const int key = ps->spreads[p.spread_off + p.n_hard + q].key;
      if (!(key_flags[key] & (KSS_KEY_HOSTNAME | KSS_KEY_UNIQUE))) {
        bins += key_card[key] + 1;
        sp += key_card[key] + 1;
      }
    }
    int keys[MAXK + 1], nk = 0;
    for (int e = 0; e < p.ipa_len; e++) {
      const int key = ps->ipa[p.ipa_off + e].key;
      bool seen = false;
      for (int j = 0; j < nk; j++) seen |= keys[j] == key;
      if (seen) continue;
      if (nk <= MAXK) keys[nk++] = key;
      if (!(key_flags[key] & KSS_KEY_UNIQUE)) bins += 4 * (key_card[key] + 1);
    }
    r.bins_cap = std::max(r.bins_cap, bins + hp + sp);
    r.xw = std::max(r.xw, std::max(MAXH + 1 + bins + hp, 12 + sp));
  }
  r.bins_cap = std::min(r.bins_cap, LDS_BINS);
  return r;
}

static size_t lds_bytes(int bins_cap, int slots) {
  return sizeof(SharedHdr) + 8 * (size_t)(NSCAL + bins_cap) + slot_arrays_bytes(slots);
}

// Geometry for clusters of at most maxN nodes split in W shards.
struct Geometry {
  int W = 1, threads = 64, npt = 1;
};

static bool pick_geometry(int maxN, int W, int pref_threads, Geometry& g) {
  g.W = W;
  const int per = (std::max(maxN, 1) + W - 1) / W;
  int t = std::min(KSS_MAX_THREADS, std::max(pref_threads, 64));
  if (per < t) t = std::max(64, (per + 63) / 64 * 64);
  int npt = (per + t - 1) / t;
  const char* ft = getenv("KSS_FORCE_THREADS");  // tuning / diagnosis: exact workgroup size
  if (ft) {
    t = std::min(KSS_MAX_THREADS, std::max(64, atoi(ft) / 64 * 64));
    npt = (per + t - 1) / t;
  }
  while (!ft && npt > 4 && t < KSS_MAX_THREADS) {
    t = std::min(KSS_MAX_THREADS, t * 2);
    npt = (per + t - 1) / t;
  }
  g.threads = t;
  g.npt = npt;
  return npt <= KSS_MAX_NPT;
}

// Launch of a sharded (W > 1) grid whose workgroups must all be resident at once: the
// host checks the occupancy (one workgroup per CU at this LDS / register footprint, and
// no more workgroups than CUs) and launches plainly.  KSS_COOP_LAUNCH=1 uses the
// cooperative launch instead (same residency, runtime-checked).
static int launch_resident(const void* fn, dim3 grid, dim3 block, void** args, size_t shmem, hipStream_t st) {
  static const bool coop = getenv("KSS_COOP_LAUNCH") != nullptr;
  if (coop) {
    HIP_TRY(hipLaunchCooperativeKernel(fn, grid, block, args, (unsigned)shmem, st));
    return 0;
  }
  int dev = 0, n_cu = 0, per_cu = 0;
  HIP_TRY(hipGetDevice(&dev));
  HIP_TRY(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, (int)(block.x * block.y * block.z), shmem));
  if (per_cu < 1 || (long long)grid.x > (long long)per_cu * n_cu)
    return fail(KSS_E_UNSUPPORTED, "sharded grid cannot be co-resident on this device");
  HIP_TRY(hipLaunchKernel(fn, grid, block, args, shmem, st));
  return 0;
}

// Launch k_schedule over n_jobs clusters (jobs already in device memory).  W > 1 needs
// every workgroup resident: cooperative launch (the runtime checks the grid fits).
static int launch_schedule(hipStream_t st, const Geometry& g, int n_jobs, int bins_cap, bool need_general, int n_keys,
                           const DevJob* jobs, const kss_profile& prof, unsigned long long* gran, int* err,
                           unsigned long long* stamps = nullptr) {
  const int cap = g.threads * g.npt;
  const size_t base = lds_bytes(bins_cap, cap);
  if (base > KSS_LDS_BUDGET) return fail(KSS_E_UNSUPPORTED, "per-workgroup LDS budget exceeded (too many nodes per shard)");
  // node cache with every label key, without labels, or none, whatever fits
  int cache_keys = -1;
  if (!getenv("KSS_NO_CACHE")) {
    if (base + node_cache_bytes(cap, n_keys) <= KSS_LDS_BUDGET) cache_keys = n_keys;
    else if (base + node_cache_bytes(cap, 0) <= KSS_LDS_BUDGET) cache_keys = 0;
  }
  const size_t shmem = base + (cache_keys >= 0 ? node_cache_bytes(cap, cache_keys) : 0);
  const bool gen = bins_cap > 0 || need_general;
  const void* fn = gen ? (const void*)k_schedule<true> : (const void*)k_schedule<false>;
  HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
  const dim3 grid((unsigned)(n_jobs * g.W)), block((unsigned)g.threads);
  kss_profile pr = prof;
  int W = g.W, npt = g.npt;
  if (g.W > 1) {
    void* args[] = {(void*)&jobs, (void*)&pr,   (void*)&W,   (void*)&npt,   (void*)&bins_cap,
                    (void*)&cache_keys, (void*)&gran, (void*)&err, (void*)&stamps};
    if (int rc = launch_resident(fn, grid, block, args, shmem, st)) return rc;
  } else {
    if (gen)
      hipLaunchKernelGGL(k_schedule<true>, grid, block, shmem, st, jobs, pr, W, npt, bins_cap, cache_keys, gran, err, stamps);
    else
      hipLaunchKernelGGL(k_schedule<false>, grid, block, shmem, st, jobs, pr, W, npt, bins_cap, cache_keys, gran, err, stamps);
    HIP_TRY(hipGetLastError());
  }
  return 0;
}

// Field-wise profile equality (padding excluded).
static bool same_profile(const kss_profile& a, const kss_profile& b) {
  bool eq = a.filter_enabled == b.filter_enabled && a.score_enabled == b.score_enabled &&
            a.fit_strategy == b.fit_strategy && a.fit_n == b.fit_n && a.ba_n == b.ba_n &&
            a.hard_pod_affinity_weight == b.hard_pod_affinity_weight && a.system_defaulted == b.system_defaulted;
  for (int i = 0; i < KSS_NSCORE; i++) eq &= a.weight[i] == b.weight[i];
  for (int i = 0; i < 4; i++) eq &= a.fit_res[i] == b.fit_res[i] && a.fit_weight[i] == b.fit_weight[i] && a.ba_res[i] == b.ba_res[i];
  return eq;
}

// Node slots per shard for k_simple: every lane's share, plus one spare slot when it
// fits (the spare slot re-evaluates the candidate node in the same pass).
static int simple_cap(const Geometry& g) { return g.npt * g.threads; }

// Launch k_simple (same grid and co-residency rule as k_schedule).
static int launch_simple(hipStream_t st, const Geometry& g, int n_jobs, int stride, int n_keys, const DevJob* jobs,
                         const kss_profile& prof, unsigned long long* gran, int* err,
                         unsigned long long* stamps = nullptr) {
  int cap = simple_cap(g);
  const size_t shmem = simple_lds_bytes(stride, n_keys, cap);
  const bool def = same_profile(prof, default_profile_c());
  const void* fn = def ? (const void*)k_simple<true> : (const void*)k_simple<false>;
  HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
  const dim3 grid((unsigned)(n_jobs * g.W)), block((unsigned)g.threads);
  kss_profile pr = prof;
  int W = g.W;
  void* args[] = {(void*)&jobs, (void*)&pr, (void*)&W, (void*)&cap, (void*)&gran, (void*)&err, (void*)&stamps};
  if (g.W > 1) {
    if (int rc = launch_resident(fn, grid, block, args, shmem, st)) return rc;
  }
  else HIP_TRY(hipLaunchKernel(fn, grid, block, args, shmem, st));
  return 0;
}

static bool simple_fits(const Geometry& g, int stride, int n_keys) {
  return stride > 0 && stride <= 32 * g.threads && g.W <= 64 * SX_CHUNKS &&
         simple_lds_bytes(stride, n_keys, simple_cap(g)) <= KSS_LDS_BUDGET;
}

// run k_schedule / k_simple on the loaded cluster for pods [0, n); results stay on the device
static int run_single(kss_ctx* ctx, const PlanNeeds& need, const DevPods& dp, int n, bool commit, bool record,
                      bool keep_norm, uint32_t flags, int32_t* chosen_out, bool staged = false) {
  const size_t N = (size_t)ctx->dc.N;
  const SlotLayout SL(N);
  const int nslots = record ? std::max(n, 1) : 1;
  int rc = ctx->slot_buf.ensure(SL.bytes * (size_t)nslots);
  if (rc) return rc;
  rc = ctx->meta_buf.ensure(sizeof(PodMeta) * (size_t)std::max(n, 1));
  if (rc) return rc;
  rc = ctx->chosen_buf.ensure(sizeof(int32_t) * (size_t)std::max(n, 1));
  if (rc) return rc;
  // shard count: ~nodes_per_shard nodes per workgroup, at most one workgroup per CU
  int W = std::max(1, std::min(ctx->n_cu, (int)((N + ctx->nodes_per_shard - 1) / ctx->nodes_per_shard)));
  if (ctx->force_w > 0) W = std::min(ctx->force_w, ctx->n_cu);
  if (flags & KSS_SCHED_FORCE_SINGLE_WG) W = 1;
  if (flags & KSS_SCHED_FORCE_MULTI_WG) W = std::max(W, std::min(4, ctx->n_cu));
  W = std::max(1, std::min(W, std::max(1, (int)N)));
  // a k_simple-eligible batch keeps W within k_simple's exchange sweep (64 * SX_CHUNKS
  // shards): at 100k nodes, 98-128 k_simple shards beat 256 k_schedule shards (69.8k
  // against 44.2k pods/s)
  const bool simple_ok = staged && ctx->blob_stride && commit && !record && !keep_norm && !need.general &&
                         ctx->dc.n_scalar == 0 && ctx->small_values && !ctx->no_simple && !(flags & KSS_SCHED_GENERAL_KERNEL);
  if (simple_ok && ctx->force_w <= 0) W = std::min(W, 64 * SX_CHUNKS);
  const int w_min = (int)((N + KSS_MAX_NPT * KSS_MAX_THREADS - 1) / (KSS_MAX_NPT * KSS_MAX_THREADS));
  W = std::max(W, w_min);
  if (W > 1 && need.xw > XW_MAX) {
    if (w_min > 1) return fail(KSS_E_UNSUPPORTED, "topology histograms too large for a sharded cluster");
    W = 1;  // exchange payload too large for granules: one workgroup
  }
  if (W > ctx->n_cu) return fail(KSS_E_UNSUPPORTED, "cluster too large for one device");
  Geometry g;
  if (!pick_geometry((int)N, W, ctx->pref_threads, g)) return fail(KSS_E_UNSUPPORTED, "no geometry for this cluster");
  DevJob job{};
  job.c = ctx->dc;
  job.P = dp;
  job.n_pods = n;
  job.commit = commit ? 1 : 0;
  job.keep_norm = keep_norm ? 1 : 0;
  job.record = record ? 1 : 0;
  job.slots = (uint8_t*)ctx->slot_buf.p;
  job.slot_bytes = SL.bytes;
  job.chosen = (int32_t*)ctx->chosen_buf.p;
  job.meta = (PodMeta*)ctx->meta_buf.p;
  job.blobs = staged && ctx->blob_stride ? (const uint8_t*)ctx->blob_buf.p : nullptr;
  job.blob_stride = ctx->blob_stride;
  const bool simple = job.blobs && simple_ok && simple_fits(g, ctx->blob_stride, ctx->dc.n_keys);
  rc = ctx->job_buf.ensure(sizeof(DevJob));
  if (rc) return rc;
  rc = ctx->err_buf.ensure(16);
  if (rc) return rc;
  unsigned long long* gran = nullptr;
  if (g.W > 1) {
    const size_t gb = sizeof(unsigned long long) * 2 * (size_t)g.W * 2 * XW_MAX;
    rc = ctx->gran_buf.ensure(gb);
    if (rc) return rc;
    gran = (unsigned long long*)ctx->gran_buf.p;
    HIP_TRY(hipMemsetAsync(gran, 0, gb, ctx->stream));  // every polled word zeroed before every launch
  }
  HIP_TRY(hipMemsetAsync(ctx->err_buf.p, 0, 16, ctx->stream));
  HIP_TRY(hipMemcpyAsync(ctx->job_buf.p, &job, sizeof(DevJob), hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
  unsigned long long* stamps = nullptr;
  const size_t stamp_bytes = sizeof(unsigned long long) * 8 * KSS_NSTAMP_PODS;
  if (ctx->stamps_file) {
    if ((rc = ctx->stamp_buf.ensure(stamp_bytes))) return rc;
    stamps = (unsigned long long*)ctx->stamp_buf.p;
    HIP_TRY(hipMemsetAsync(stamps, 0, stamp_bytes, ctx->stream));
  }
  if (simple)
    rc = launch_simple(ctx->stream, g, 1, ctx->blob_stride, ctx->dc.n_keys, (const DevJob*)ctx->job_buf.p, ctx->prof, gran,
                       (int*)ctx->err_buf.p, stamps);
  else
    rc = launch_schedule(ctx->stream, g, 1, std::max(need.bins_cap, 0), need.general, ctx->dc.n_keys,
                         (const DevJob*)ctx->job_buf.p, ctx->prof, gran, (int*)ctx->err_buf.p, stamps);
  if (rc) return rc;
  ctx->last_kernel = simple ? 1 : 0;
  HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  ctx->last_ms = ms;
  ctx->last_launches = 1;
  ctx->last_geom[0] = g.W;
  ctx->last_geom[1] = g.threads;
  ctx->last_geom[2] = g.npt;
  int errw = 0;
  HIP_TRY(hipMemcpy(&errw, ctx->err_buf.p, sizeof(int), hipMemcpyDeviceToHost));
  if (errw) return fail(KSS_E_DEVICE, "shard exchange timed out (workgroups not co-resident?)");
  ctx->meta_host.resize((size_t)std::max(n, 1));
  HIP_TRY(hipMemcpy(ctx->meta_host.data(), ctx->meta_buf.p, sizeof(PodMeta) * (size_t)std::max(n, 1), hipMemcpyDeviceToHost));
  if (chosen_out && n) HIP_TRY(hipMemcpy(chosen_out, ctx->chosen_buf.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
  ctx->recorded = record ? n : (n > 0 && !simple ? 1 : 0);
  ctx->meta_n = n;
  ctx->axis_meta_dirty = false;
  if (stamps) {
    std::vector<unsigned long long> h(8 * KSS_NSTAMP_PODS);
    HIP_TRY(hipMemcpy(h.data(), stamps, stamp_bytes, hipMemcpyDeviceToHost));
    if (FILE* f = fopen(ctx->stamps_file, "ab")) {
      fwrite(h.data(), 8, h.size(), f);
      fclose(f);
    }
  }
  return 0;
}

// serialize the staged podset for k_simple (host copy kept alive for the async upload)
static int stage_blobs(kss_ctx* ctx, const kss_podset* ps) {
  ctx->blob_stride = build_blobs(ps, ctx->blob_host);
  if (!ctx->blob_stride) return 0;
  int rc = ctx->blob_buf.ensure(ctx->blob_host.size());
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(ctx->blob_buf.p, ctx->blob_host.data(), ctx->blob_host.size(), hipMemcpyHostToDevice, ctx->stream));
  return 0;
}

static int copy_slot(kss_ctx* ctx, int slot, const PodMeta& m, kss_pod_result* out) {
  const size_t N = (size_t)ctx->dc.N;
  const SlotLayout SL(N);
  const char* base = (const char*)ctx->slot_buf.p + (size_t)slot * SL.bytes;
  if (out->fail_plugin) HIP_TRY(hipMemcpy(out->fail_plugin, base + SL.fail, N, hipMemcpyDeviceToHost));
  if (out->fail_detail) HIP_TRY(hipMemcpy(out->fail_detail, base + SL.detail, 2 * N, hipMemcpyDeviceToHost));
  if (out->raw) HIP_TRY(hipMemcpy(out->raw, base + SL.raw, 8 * KSS_NSCORE * N, hipMemcpyDeviceToHost));
  if (out->norm) HIP_TRY(hipMemcpy(out->norm, base + SL.norm, 8 * KSS_NSCORE * N, hipMemcpyDeviceToHost));
  if (out->total) HIP_TRY(hipMemcpy(out->total, base + SL.total, 8 * N, hipMemcpyDeviceToHost));
  out->n_feasible = m.n_feasible;
  out->chosen = m.chosen;
  out->best_total = m.best_total;
  out->scored = m.scored;
  out->status = m.status;
  if (m.status == 4) return fail(KSS_E_UNSUPPORTED, "pod program exceeds the device path's per-pod limits");
  return 0;
}

int kss_eval_pod(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, kss_pod_result* out) {
  if (!ctx || !ctx->loaded || !ps || !out) return fail(KSS_E_INVAL, "bad arguments");
  if (pod_index < 0 || pod_index >= ps->n_pods) return fail(KSS_E_INVAL, "pod index out of range");
  int rc = validate(&ctx->host, ps, ps->n_pods);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  // evaluate exactly one pod: view the podset from pod_index
  kss_podset one = *ps;
  one.pods = ps->pods + pod_index;
  one.n_pods = 1;
  rc = upload_podset(ctx->stream, ctx->tmp_pod_buf, &one, ctx->tdp);
  if (rc) return rc;
  const PlanNeeds need = plan_needs(ctx->key_card_h.data(), ctx->key_flags_h.data(), &one, 1);
  rc = run_single(ctx, need, ctx->tdp, 1, /*commit=*/false, /*record=*/false, /*keep_norm=*/true, 0, nullptr);
  if (rc) return rc;
  return copy_slot(ctx, 0, ctx->meta_host[0], out);
}

int kss_commit(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, int32_t node) {
  if (!ctx || !ctx->loaded || !ps) return fail(KSS_E_INVAL, "bad arguments");
  if (pod_index < 0 || pod_index >= ps->n_pods) return fail(KSS_E_INVAL, "pod index out of range");
  const int local = node - ctx->dc.node_base;
  if (local < 0 || local >= ctx->dc.N) return fail(KSS_E_INVAL, "node out of range");
  int rc = validate(&ctx->host, ps, ps->n_pods);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  rc = upload_podset(ctx->stream, ctx->tmp_pod_buf, ps, ctx->tdp);
  if (rc) return rc;
  hipLaunchKernelGGL(k_commit, dim3(1), dim3(64), 0, ctx->stream, ctx->dc, ctx->tdp, pod_index, local, 1);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int kss_rollback(kss_ctx* ctx, const kss_podset* ps, int32_t pod_index, int32_t node) {
  if (!ctx || !ctx->loaded || !ps) return fail(KSS_E_INVAL, "bad arguments");
  if (pod_index < 0 || pod_index >= ps->n_pods) return fail(KSS_E_INVAL, "pod index out of range");
  const int local = node - ctx->dc.node_base;
  if (local < 0 || local >= ctx->dc.N) return fail(KSS_E_INVAL, "node out of range");
  int rc = validate(&ctx->host, ps, ps->n_pods);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  rc = upload_podset(ctx->stream, ctx->tmp_pod_buf, ps, ctx->tdp);
  if (rc) return rc;
  hipLaunchKernelGGL(k_commit, dim3(1), dim3(64), 0, ctx->stream, ctx->dc, ctx->tdp, pod_index, local, -1);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return 0;
}

int kss_schedule_batch(kss_ctx* ctx, const kss_podset* ps, int32_t n, uint32_t flags, int32_t* chosen_out) {
  if (!ctx || !ctx->loaded || !ps) return fail(KSS_E_INVAL, "bad arguments");
  if (n < 0 || n > ps->n_pods) return fail(KSS_E_INVAL, "pod count out of range");
  // every pod is staged (and may be run later by kss_run_staged / the node axis): all of
  // them are validated, not only the first n
  int rc = validate(&ctx->host, ps, ps->n_pods);
  if (rc) return rc;
  const bool record = (flags & KSS_SCHED_RECORD) != 0;
  if (record && n > ctx->cfg.max_pods_record) return fail(KSS_E_INVAL, "record capacity (max_pods_record) exceeded");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  rc = upload_podset(ctx->stream, ctx->pod_buf, ps, ctx->dp);
  if (rc) return rc;
  if ((rc = stage_blobs(ctx, ps))) return rc;
  ctx->staged_n = ps->n_pods;
  ctx->staged_need = plan_needs(ctx->key_card_h.data(), ctx->key_flags_h.data(), ps, ps->n_pods);
  rc = run_single(ctx, ctx->staged_need, ctx->dp, n, /*commit=*/true, record, /*keep_norm=*/record, flags, chosen_out,
                  /*staged=*/true);
  if (rc) return rc;
  for (int i = 0; i < n; i++)
    if (ctx->meta_host[i].status == 4) return fail(KSS_E_UNSUPPORTED, "pod program exceeds the device path's per-pod limits");
  return 0;
}

int kss_stage_pods(kss_ctx* ctx, const kss_podset* ps) {
  if (!ctx || !ctx->loaded || !ps) return fail(KSS_E_INVAL, "bad arguments");
  int rc = validate(&ctx->host, ps, ps->n_pods);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  rc = upload_podset(ctx->stream, ctx->pod_buf, ps, ctx->dp);
  if (rc) return rc;
  if ((rc = stage_blobs(ctx, ps))) return rc;
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  ctx->staged_n = ps->n_pods;
  ctx->staged_need = plan_needs(ctx->key_card_h.data(), ctx->key_flags_h.data(), ps, ps->n_pods);
  return 0;
}

int kss_run_staged(kss_ctx* ctx, int32_t n, uint32_t flags, int32_t* chosen_out) {
  if (!ctx || !ctx->loaded) return fail(KSS_E_INVAL, "no cluster loaded");
  if (n < 0 || n > ctx->staged_n) return fail(KSS_E_INVAL, "n exceeds the staged pods");
  const bool record = (flags & KSS_SCHED_RECORD) != 0;
  if (record && n > ctx->cfg.max_pods_record) return fail(KSS_E_INVAL, "record capacity (max_pods_record) exceeded");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  int rc = run_single(ctx, ctx->staged_need, ctx->dp, n, /*commit=*/true, record, /*keep_norm=*/record, flags, chosen_out,
                      /*staged=*/true);
  if (rc) return rc;
  for (int i = 0; i < n; i++)
    if (ctx->meta_host[i].status == 4) return fail(KSS_E_UNSUPPORTED, "pod program exceeds the device path's per-pod limits");
  return 0;
}

int kss_fetch_record(kss_ctx* ctx, int32_t pod_index, kss_pod_result* out) {
  if (!ctx || !out) return fail(KSS_E_INVAL, "bad arguments");
  if (pod_index < 0 || pod_index >= ctx->recorded) return fail(KSS_E_NOTFOUND, "pod not recorded");
  std::lock_guard<std::mutex> lk(ctx->mu);
  HIP_TRY(hipSetDevice(ctx->cfg.device));
  return copy_slot(ctx, pod_index, ctx->meta_host[pod_index], out);
}

int kss_last_timing(kss_ctx* ctx, double* device_ms, int32_t* launches) {
  if (!ctx) return fail(KSS_E_INVAL, "null ctx");
  if (device_ms) *device_ms = ctx->last_ms;
  if (launches) *launches = ctx->last_launches;
  return 0;
}

int kss_last_geometry(kss_ctx* ctx, int32_t* out3) {
  if (!ctx || !out3) return fail(KSS_E_INVAL, "bad arguments");
  for (int i = 0; i < 3; i++) out3[i] = ctx->last_geom[i];
  return 0;
}

int kss_last_kernel(kss_ctx* ctx) {
  if (!ctx) return fail(KSS_E_INVAL, "null ctx");
  return ctx->last_kernel;
}

int kss_fetch_meta(kss_ctx* ctx, int32_t first, int32_t n, int64_t* out) {
  if (!ctx || (n > 0 && !out)) return fail(KSS_E_INVAL, "bad arguments");
  if (first < 0 || n < 0 || first + n > ctx->meta_n) return fail(KSS_E_NOTFOUND, "pod outcome not available");
  if (ctx->axis_meta_dirty) {  // node-axis outcomes were written on the caller's stream
    HIP_TRY(hipSetDevice(ctx->cfg.device));
    HIP_TRY(hipDeviceSynchronize());
    ctx->meta_host.resize((size_t)ctx->meta_n);
    HIP_TRY(hipMemcpy(ctx->meta_host.data(), ctx->meta_buf.p, sizeof(PodMeta) * (size_t)ctx->meta_n, hipMemcpyDeviceToHost));
    ctx->axis_meta_dirty = false;
  }
  for (int i = 0; i < n; i++) {
    const PodMeta& m = ctx->meta_host[first + i];
    int64_t* o = out + 5 * (size_t)i;
    o[0] = m.chosen;
    o[1] = m.n_feasible;
    o[2] = m.scored;
    o[3] = m.status;
    o[4] = m.best_total;
  }
  return 0;
}

int kss_schedule_scenarios(int32_t device, const kss_profile* prof, int32_t n_scen, const kss_cluster* clusters,
                           const kss_podset* podsets, int32_t* chosen_out, double* device_ms) {
  if (!prof || n_scen < 0 || (n_scen && (!clusters || !podsets || !chosen_out))) return fail(KSS_E_INVAL, "bad arguments");
  int rc = check_profile(prof);
  if (rc) return rc;
  if (n_scen == 0) return 0;
  for (int s = 0; s < n_scen; s++) {
    if ((rc = check_cluster(&clusters[s]))) return rc;
    if ((rc = validate(&clusters[s], &podsets[s], podsets[s].n_pods))) return rc;
  }
  HIP_TRY(hipSetDevice(device));
  hipStream_t st;
  HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  // one device arena: clusters, podsets, scratch slots, chosen, jobs
  std::vector<size_t> c_off(n_scen), p_off(n_scen), s_off(n_scen), ch_off(n_scen);
  std::vector<ClusterLayout> layouts;
  layouts.reserve(n_scen);
  size_t total = 0;
  for (int s = 0; s < n_scen; s++) {
    layouts.emplace_back(&clusters[s], clusters[s].n_classes, clusters[s].n_terms);
    c_off[s] = total;
    total = align_up(total + layouts[s].total, 256);
  }
  std::vector<size_t> pod_bytes(n_scen);
  for (int s = 0; s < n_scen; s++) {
    const kss_podset& ps = podsets[s];
    size_t b = 0;
    b = align_up(b + sizeof(kss_pod) * std::max(ps.n_pods, 1), 256);
    b = align_up(b + sizeof(kss_req) * std::max(ps.n_reqs, 1), 256);
    b = align_up(b + sizeof(kss_term) * std::max(ps.n_terms, 1), 256);
    b = align_up(b + sizeof(kss_spread) * std::max(ps.n_spreads, 1), 256);
    b = align_up(b + sizeof(kss_ipa) * std::max(ps.n_ipa, 1), 256);
    b = align_up(b + sizeof(int32_t) * std::max(ps.n_ints, 1), 256);
    pod_bytes[s] = b;
    p_off[s] = total;
    total = align_up(total + b, 256);
  }
  for (int s = 0; s < n_scen; s++) {
    s_off[s] = total;
    total = align_up(total + SlotLayout((size_t)clusters[s].n_nodes).bytes, 256);
  }
  for (int s = 0; s < n_scen; s++) {
    ch_off[s] = total;
    total = align_up(total + sizeof(int32_t) * std::max(podsets[s].n_pods, 1), 256);
  }
  // per-pod outcomes: a pod whose program exceeds the device limits (status 4) fails the
  // call with KSS_E_UNSUPPORTED instead of looking unschedulable
  std::vector<size_t> m_off(n_scen);
  for (int s = 0; s < n_scen; s++) {
    m_off[s] = total;
    total = align_up(total + sizeof(PodMeta) * std::max(podsets[s].n_pods, 1), 256);
  }
  const size_t job_off = total;
  total = align_up(total + sizeof(DevJob) * n_scen, 256);
  // k_simple for the whole sweep when every scenario qualifies (no spread / inter-pod
  // programs, no scalar resources, values inside the exact f64 envelope): pod programs
  // as blobs at one common stride, one workgroup per scenario
  bool simple = getenv("KSS_NO_SIMPLE") == nullptr;
  for (int i = 0; i < prof->fit_n && simple; i++) simple = prof->fit_weight[i] >= 0 && prof->fit_weight[i] < (1ll << 20);
  size_t blob_mx = 16;
  for (int sc = 0; sc < n_scen && simple; sc++) {
    const kss_cluster& cl = clusters[sc];
    simple = cl.n_scalar == 0;
    for (size_t i = 0; i < 3 * (size_t)cl.n_nodes && simple; i++) simple = cl.alloc[i] >= 0 && cl.alloc[i] < (1ll << 46);
    for (int i = 0; i < podsets[sc].n_pods && simple; i++) {
      const kss_pod& q = podsets[sc].pods[i];
      simple = !(q.n_hard | q.n_soft | q.ipa_len);
      if (simple) blob_mx = std::max(blob_mx, serialize_pod(&podsets[sc], i, nullptr));
    }
  }
  const int blob_stride = simple && align_up(blob_mx, 64) <= (size_t)BLOB_MAX ? (int)align_up(blob_mx, 64) : 0;
  std::vector<size_t> b_off(n_scen, 0);
  if (blob_stride)
    for (int sc = 0; sc < n_scen; sc++) {
      b_off[sc] = total;
      total = align_up(total + (size_t)blob_stride * std::max(podsets[sc].n_pods, 1), 256);
    }
  char* arena = nullptr;
  if (hipMalloc(&arena, total) != hipSuccess) {
    hipStreamDestroy(st);
    return fail(KSS_E_NOMEM, "scenario arena allocation failed");
  }
  std::vector<DevJob> jobs(n_scen);
  std::vector<std::vector<double>> logtabs(n_scen);
  rc = 0;
  for (int s = 0; s < n_scen && !rc; s++) {
    DevJob& j = jobs[s];
    rc = fill_cluster(st, &clusters[s], clusters[s].n_classes, clusters[s].n_terms, arena + c_off[s], layouts[s], j.c, logtabs[s]);
    if (rc) break;
    DevBuf view;
    view.p = arena + p_off[s];
    view.cap = pod_bytes[s];
    rc = upload_podset(st, view, &podsets[s], j.P);
    view.p = nullptr;
    j.n_pods = podsets[s].n_pods;
    j.commit = 1;
    j.keep_norm = 0;
    j.record = 0;
    j.slots = (uint8_t*)(arena + s_off[s]);
    j.slot_bytes = SlotLayout((size_t)clusters[s].n_nodes).bytes;
    j.chosen = (int32_t*)(arena + ch_off[s]);
    j.meta = (PodMeta*)(arena + m_off[s]);
    j.blobs = nullptr;
    j.blob_stride = 0;
    if (blob_stride) {
      std::vector<uint8_t> bl((size_t)blob_stride * std::max(podsets[s].n_pods, 1), 0);
      for (int i = 0; i < podsets[s].n_pods; i++) serialize_pod(&podsets[s], i, bl.data() + (size_t)blob_stride * i);
      if (hipMemcpy(arena + b_off[s], bl.data(), bl.size(), hipMemcpyHostToDevice) != hipSuccess)
        rc = fail(KSS_E_DEVICE, "blob upload failed");
      j.blobs = (const uint8_t*)(arena + b_off[s]);
      j.blob_stride = blob_stride;
    }
    // the host-side log tables must stay alive until the copies finish
    if (s % 256 == 255) {
      if (hipStreamSynchronize(st) != hipSuccess) rc = fail(KSS_E_DEVICE, "upload failed");
      for (int t = s - 255; t <= s; t++) std::vector<double>().swap(logtabs[t]);
    }
  }
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (!rc) {
    if (hipMemcpyAsync(arena + job_off, jobs.data(), sizeof(DevJob) * n_scen, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      rc = fail(KSS_E_DEVICE, "job upload failed");
  }
  PlanNeeds need;
  for (int sc = 0; sc < n_scen; sc++) {
    const PlanNeeds q = plan_needs(clusters[sc].key_card, clusters[sc].key_flags, &podsets[sc], podsets[sc].n_pods);
    need.bins_cap = std::max(need.bins_cap, q.bins_cap);
    need.general |= q.general;
  }
  int maxN = 0;
  for (int sc = 0; sc < n_scen; sc++) maxN = std::max(maxN, clusters[sc].n_nodes);
  // one workgroup per scenario: at most two node slots per lane (C5, 1,000 nodes: 512
  // threads ran the 512-scenario sweep in 16.5 ms against 23.7 ms at 256)
  int pref = maxN > 512 ? 512 : 256;
  if (const char* e = getenv("KSS_THREADS")) pref = std::min(KSS_MAX_THREADS, std::max(64, atoi(e)));
  Geometry g;
  if (!rc && !pick_geometry(maxN, 1, pref, g)) rc = fail(KSS_E_UNSUPPORTED, "scenario cluster too large for one workgroup");
  int* err = nullptr;
  if (!rc && hipMalloc(&err, 16) != hipSuccess) rc = fail(KSS_E_NOMEM, "error word allocation failed");
  if (!rc) {
    hipMemsetAsync(err, 0, 16, st);
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, st);
    int max_keys = 0;
    for (int sc = 0; sc < n_scen; sc++) max_keys = std::max(max_keys, clusters[sc].n_label_keys);
    if (blob_stride && !need.general && simple_fits(g, blob_stride, max_keys))
      rc = launch_simple(st, g, n_scen, blob_stride, max_keys, (const DevJob*)(arena + job_off), *prof, nullptr, err);
    else
      rc = launch_schedule(st, g, n_scen, need.bins_cap, need.general, max_keys, (const DevJob*)(arena + job_off), *prof,
                           nullptr, err);
    hipEventRecord(e1, st);
    if (hipStreamSynchronize(st) != hipSuccess && !rc) rc = fail(KSS_E_DEVICE, "k_schedule failed");
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    if (device_ms) *device_ms = ms;
  }
  if (err) hipFree(err);
  if (!rc) {
    size_t o = 0;
    for (int s = 0; s < n_scen && !rc; s++) {
      if (podsets[s].n_pods &&
          hipMemcpy(chosen_out + o, arena + ch_off[s], sizeof(int32_t) * podsets[s].n_pods, hipMemcpyDeviceToHost) != hipSuccess)
        rc = fail(KSS_E_DEVICE, "chosen copy failed");
      o += (size_t)podsets[s].n_pods;
    }
    std::vector<PodMeta> m;
    for (int s = 0; s < n_scen && !rc; s++) {
      m.resize((size_t)std::max(podsets[s].n_pods, 1));
      if (podsets[s].n_pods &&
          hipMemcpy(m.data(), arena + m_off[s], sizeof(PodMeta) * podsets[s].n_pods, hipMemcpyDeviceToHost) != hipSuccess)
        rc = fail(KSS_E_DEVICE, "outcome copy failed");
      for (int i = 0; i < podsets[s].n_pods && !rc; i++)
        if (m[i].status == 4) rc = fail(KSS_E_UNSUPPORTED, "pod program exceeds the device path's per-pod limits");
    }
  }
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  hipFree(arena);
  hipStreamDestroy(st);
  return rc;
}

int kss_set_names(kss_ctx* ctx, const kss_names* names) {
  if (!ctx || !names) return fail(KSS_E_INVAL, "bad arguments");
  return kss_host_set_names(&ctx->names, names, ctx->host.n_nodes, ctx->host.n_taints, ctx->host.n_scalar);
}

int kss_format_annotations(kss_ctx* ctx, const kss_pod_result* res, int32_t n_nodes, char* buf, size_t cap, size_t* need) {
  if (!ctx || !res || !need) return fail(KSS_E_INVAL, "bad arguments");
  return kss_host_format(&ctx->names, &ctx->prof, res, n_nodes, buf, cap, need);
}

}  // extern "C"
