// kss_synth.cpp — seeded synthetic clusters emitted directly as the
// struct-of-arrays of include/kss.h.  Draw-for-draw identical to kss/synth.py (which
// emits Kubernetes objects for the host compiler and the object-level oracle);
// tests/test_synth.py checks both produce the same schedule through the oracle.
#include <cstdint>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "../../include/kss.h"

namespace {

struct SplitMix64 {
  uint64_t s;
  explicit SplitMix64(uint64_t seed) : s(seed) {}
  uint64_t next() {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  uint64_t rnd(uint64_t n) { return next() % n; }
};

struct Owner {
  std::vector<int64_t> alloc, requested, nonzero, value_int;
  std::vector<int32_t> allowed, podc, label_value, key_base, key_card, key_empty, class_count, term_count;
  std::vector<uint32_t> flags, key_flags;
  std::vector<uint64_t> th, ts;
  std::vector<uint8_t> taint_order, value_is_int;
  std::vector<kss_pod> pods;
  std::vector<kss_req> reqs;
  std::vector<kss_term> terms;
  std::vector<kss_spread> spreads;
  std::vector<kss_ipa> ipa;
  std::vector<int32_t> ints;
};

// label key columns (fixed for every config)
enum { K_GEN = 0, K_HOST = 1, K_ITYPE = 2, K_ZONE = 3, NKEYS = 4 };
const int64_t GI = 1ll << 30, MI = 1ll << 20;
const int64_t POD_CPU[5] = {100, 250, 500, 1000, 2000};
const int64_t POD_MEM[6] = {128 * MI, 256 * MI, 512 * MI, 1024 * MI, 2048 * MI, 4096 * MI};

int cores_of(uint64_t c) { return c < 1 ? 4 : c < 4 ? 8 : c < 7 ? 16 : c < 9 ? 32 : 64; }

int32_t push_list(Owner& o, std::initializer_list<int32_t> v) {
  const int32_t off = (int32_t)o.ints.size();
  o.ints.insert(o.ints.end(), v.begin(), v.end());
  return off;
}

kss_req mask_req(int key, uint64_t mask) {
  kss_req r;
  std::memset(&r, 0, sizeof(r));
  r.key = key;
  r.op = KSS_OP_MASK;
  r.mask = mask;
  return r;
}

void push_term(Owner& o, const kss_req& r, int weight) {
  kss_term t;
  t.req_off = (int32_t)o.reqs.size();
  t.req_len = 1;
  t.weight = weight;
  t.flags = 0;
  o.reqs.push_back(r);
  o.terms.push_back(t);
}

}  // namespace

extern "C" int kss_synth_make(int32_t config, uint64_t seed, int32_t n_nodes, int32_t n_pods, kss_synth* out) {
  static const int def_nodes[6] = {0, 100, 5000, 5000, 100000, 1000};
  static const int def_pods[6] = {0, 1000, 10000, 10000, 20000, 1000};
  if (!out || config < 1 || config > 5) return KSS_E_INVAL;
  const int N = n_nodes > 0 ? n_nodes : def_nodes[config];
  const int NP = n_pods > 0 ? n_pods : def_pods[config];
  if (seed == 0) seed = 0x5EED0000ull + (uint64_t)config;
  Owner* o = new (std::nothrow) Owner();
  if (!o) return KSS_E_NOMEM;
  SplitMix64 r(seed);
  const size_t NN = (size_t)N;
  o->alloc.assign(KSS_NRES * NN, 0);
  o->requested.assign(KSS_NRES * NN, 0);
  o->nonzero.assign(2 * NN, 0);
  o->allowed.assign(NN, 110);
  o->podc.assign(NN, 0);
  o->flags.assign(NN, KSS_NODE_HAS_LABELS);
  o->th.assign(NN, 0);
  o->ts.assign(NN, 0);
  o->taint_order.assign(NN * KSS_TAINT_ORDER, 0xFF);
  o->label_value.assign(NKEYS * NN, -1);
  // value tables: gen "1".."5", hostname (N names), instance type (4), zone (3)
  const int card[NKEYS] = {5, N, 4, 3};
  int base = 0;
  for (int k = 0; k < NKEYS; k++) {
    o->key_base.push_back(base);
    o->key_card.push_back(card[k]);
    o->key_empty.push_back(card[k]);
    base += card[k];
  }
  o->key_flags = {0u, (uint32_t)(KSS_KEY_UNIQUE | KSS_KEY_HOSTNAME), 0u, 0u};
  o->value_int.assign(base, 0);
  o->value_is_int.assign(base, 0);
  for (int v = 0; v < 5; v++) {
    o->value_int[v] = v + 1;
    o->value_is_int[v] = 1;
  }
  for (int i = 0; i < N; i++) {
    const uint64_t c = r.rnd(10), mm = r.rnd(2), it = r.rnd(4), gen = 1 + r.rnd(5);
    const bool ded = r.rnd(100) < 10, spot = r.rnd(100) < 5, uns = r.rnd(100) < 2;
    const int cores = cores_of(c);
    const int64_t mult = mm ? 8 : 4;
    o->alloc[KSS_RES_CPU * NN + i] = (int64_t)cores * 1000;
    o->alloc[KSS_RES_MEMORY * NN + i] = (int64_t)cores * mult * GI;
    o->alloc[KSS_RES_EPHEMERAL * NN + i] = 100 * GI;
    int ti = 0;
    if (ded) {
      o->th[i] |= 1ull;
      o->taint_order[(size_t)i * KSS_TAINT_ORDER + ti++] = 0;
    }
    if (spot) o->ts[i] |= 2ull;
    if (uns) o->flags[i] |= KSS_NODE_UNSCHEDULABLE;
    o->label_value[K_GEN * NN + i] = (int32_t)(gen - 1);
    o->label_value[K_HOST * NN + i] = i;
    o->label_value[K_ITYPE * NN + i] = (int32_t)it;
    o->label_value[K_ZONE * NN + i] = i % 3;
  }
  const int n_classes = (config == 3 || config == 4) ? 100 : 1;
  const int n_terms = config == 3 ? 300 : 0;
  o->class_count.assign((size_t)n_classes * NN, 0);
  o->term_count.assign((size_t)n_terms * NN + 1, 0);
  if (config == 3) {
    for (int i = 0; i < N; i++) {
      for (int k = 0; k < 2; k++) {
        const int app = (int)r.rnd(100);
        o->class_count[(size_t)app * NN + i] += 1;
        o->requested[KSS_RES_CPU * NN + i] += 100;
        o->requested[KSS_RES_MEMORY * NN + i] += 128 * MI;
        o->nonzero[0 * NN + i] += 100;
        o->nonzero[1 * NN + i] += 128 * MI;
        o->podc[i] += 1;
      }
    }
  }
  o->pods.resize((size_t)NP);
  for (int j = 0; j < NP; j++) {
    const bool noreq = r.rnd(100) < 5;
    const uint64_t ci = r.rnd(5), mi = r.rnd(6);
    const bool tded = r.rnd(100) < 10, tspot = r.rnd(100) < 30;
    const bool sel = r.rnd(100) < 20;
    const uint64_t sit = r.rnd(4);
    const bool raff = r.rnd(100) < 20;
    const uint64_t rk = r.rnd(2), z1 = r.rnd(3), z2o = r.rnd(2);
    const bool has_pref = r.rnd(100) < 30;
    const uint64_t npref = 1 + r.rnd(3);
    uint64_t pw[3], pk[3], pv[3];
    for (int t = 0; t < 3; t++) {
      pw[t] = 1 + r.rnd(100);
      pk[t] = r.rnd(3);
      pv[t] = r.rnd(5);
    }
    int app = -1;
    bool pz = false, ph = false, anti = false, pref = false, selfaff = false;
    if (config == 3) {
      app = (int)r.rnd(100);
      pz = r.rnd(100) < 50;
      ph = r.rnd(100) < 50;
      anti = r.rnd(100) < 30;
      pref = r.rnd(100) < 30;
      selfaff = r.rnd(100) < 10;
    } else if (config == 4) {
      app = (int)r.rnd(100);
      pz = r.rnd(100) < 50;
    }
    kss_pod& p = o->pods[(size_t)j];
    std::memset(&p, 0, sizeof(p));
    const int64_t cpu = noreq ? 0 : POD_CPU[ci], mem = noreq ? 0 : POD_MEM[mi];
    p.fit_request[KSS_RES_CPU] = cpu;
    p.fit_request[KSS_RES_MEMORY] = mem;
    p.score_req_nz[KSS_RES_CPU] = noreq ? 100 : cpu;
    p.score_req_nz[KSS_RES_MEMORY] = noreq ? 200 * MI : mem;
    p.score_req[KSS_RES_CPU] = cpu;
    p.score_req[KSS_RES_MEMORY] = mem;
    std::memcpy(p.commit_req, p.fit_request, sizeof(p.commit_req));
    p.commit_nz[0] = p.score_req_nz[KSS_RES_CPU];
    p.commit_nz[1] = p.score_req_nz[KSS_RES_MEMORY];
    p.tol_hard = tded ? 1ull : 0ull;
    p.tol_soft = tspot ? 2ull : 0ull;
    p.node_name = -1;
    p.names_len = -1;
    uint32_t flags = KSS_POD_PTS_SCORE_STATE;
    p.sel_off = (int32_t)o->reqs.size();
    if (sel) o->reqs.push_back(mask_req(K_ITYPE, 1ull << sit));
    p.sel_len = (int32_t)o->reqs.size() - p.sel_off;
    p.aff_off = (int32_t)o->terms.size();
    if (raff) {
      flags |= KSS_POD_HAS_REQ_AFFINITY;
      if (rk == 0)
        push_term(*o, mask_req(K_ZONE, (1ull << z1) | (1ull << ((z1 + 1 + z2o) % 3))), 0);
      else
        push_term(*o, mask_req(K_GEN, (1ull << 2) | (1ull << 3) | (1ull << 4)), 0);  // gen Gt 2
    }
    p.aff_len = (int32_t)o->terms.size() - p.aff_off;
    p.pref_off = (int32_t)o->terms.size();
    if (has_pref) {
      for (uint64_t t = 0; t < npref; t++) {
        const uint64_t v = pv[t];
        if (pk[t] == 0)
          push_term(*o, mask_req(K_ITYPE, 1ull << (v % 4)), (int)pw[t]);
        else if (pk[t] == 1)
          push_term(*o, mask_req(K_ZONE, 1ull << (v % 3)), (int)pw[t]);
        else
          push_term(*o, mask_req(K_GEN, (1ull << v) - 1), (int)pw[t]);  // gen Lt 1+v
      }
    }
    p.pref_len = (int32_t)o->terms.size() - p.pref_off;
    p.spread_off = (int32_t)o->spreads.size();
    if (pz || ph) flags |= KSS_POD_PTS_REQUIRE_ALL;
    if (pz) {
      kss_spread s{K_ZONE, 1, 1, (int32_t)KSS_SPREAD_POLICY_AFFINITY_HONOR, push_list(*o, {app}), 1, 1, 0};
      o->spreads.push_back(s);
      p.n_hard = 1;
    }
    if (ph) {
      kss_spread s{K_HOST, 1, 1, (int32_t)KSS_SPREAD_POLICY_AFFINITY_HONOR, push_list(*o, {app}), 1, 1, 0};
      o->spreads.push_back(s);
      p.n_soft = 1;
    }
    p.ipa_off = (int32_t)o->ipa.size();
    if (config == 3) {
      o->ipa.push_back(kss_ipa{KSS_IPA_EXISTING_ANTI, K_HOST, push_list(*o, {app}), 1, 0, 0});
      if (selfaff) {
        o->ipa.push_back(kss_ipa{KSS_IPA_REQ_AFFINITY, K_ZONE, push_list(*o, {app}), 1, 0, 0});
        flags |= KSS_POD_IPA_SELF_MATCH;
      }
      if (anti) o->ipa.push_back(kss_ipa{KSS_IPA_REQ_ANTI, K_HOST, push_list(*o, {app}), 1, 0, 0});
      if (pref) {
        o->ipa.push_back(kss_ipa{KSS_IPA_SCORE_CLASS, K_ZONE, push_list(*o, {(app + 1) % 100}), 1, 50, 0});
        flags |= KSS_POD_IPA_HAS_PREFERRED;
      }
      o->ipa.push_back(kss_ipa{KSS_IPA_SCORE_TERM, K_ZONE, push_list(*o, {200 + app}), 1, 1, 0});
      o->ipa.push_back(kss_ipa{KSS_IPA_SCORE_TERM, K_ZONE, push_list(*o, {100 + app}), 1, 50, 0});
    }
    p.ipa_len = (int32_t)o->ipa.size() - p.ipa_off;
    p.cls = app >= 0 ? app : 0;
    p.own_terms_off = (int32_t)o->ints.size();
    if (selfaff) o->ints.push_back(200 + app);
    if (anti) o->ints.push_back(app);
    if (pref) o->ints.push_back(100 + (app + 1) % 100);
    p.own_terms_len = (int32_t)o->ints.size() - p.own_terms_off;
    p.flags = flags;
  }
  if (o->reqs.empty()) o->reqs.push_back(kss_req{});
  if (o->terms.empty()) o->terms.push_back(kss_term{});
  if (o->spreads.empty()) o->spreads.push_back(kss_spread{});
  if (o->ipa.empty()) o->ipa.push_back(kss_ipa{});
  if (o->ints.empty()) o->ints.push_back(0);

  std::memset(out, 0, sizeof(*out));
  kss_cluster& cl = out->cluster;
  cl.n_nodes = N;
  cl.n_scalar = 0;
  cl.n_label_keys = NKEYS;
  cl.n_label_values = base;
  cl.n_classes = n_classes;
  cl.n_terms = n_terms;
  cl.n_taints = 2;
  cl.node_base = 0;
  cl.alloc = o->alloc.data();
  cl.requested = o->requested.data();
  cl.nonzero = o->nonzero.data();
  cl.allowed_pods = o->allowed.data();
  cl.pod_count = o->podc.data();
  cl.node_flags = o->flags.data();
  cl.taint_hard = o->th.data();
  cl.taint_soft = o->ts.data();
  cl.taint_order = o->taint_order.data();
  cl.label_value = o->label_value.data();
  cl.key_base = o->key_base.data();
  cl.key_card = o->key_card.data();
  cl.key_flags = o->key_flags.data();
  cl.key_empty = o->key_empty.data();
  cl.value_int = o->value_int.data();
  cl.value_is_int = o->value_is_int.data();
  cl.class_count = o->class_count.data();
  cl.term_count = o->term_count.data();
  kss_podset& ps = out->pods;
  ps.n_pods = NP;
  ps.n_reqs = (int32_t)o->reqs.size();
  ps.n_terms = (int32_t)o->terms.size();
  ps.n_spreads = (int32_t)o->spreads.size();
  ps.n_ipa = (int32_t)o->ipa.size();
  ps.n_ints = (int32_t)o->ints.size();
  ps.pods = o->pods.data();
  ps.reqs = o->reqs.data();
  ps.terms = o->terms.data();
  ps.spreads = o->spreads.data();
  ps.ipa = o->ipa.data();
  ps.ints = o->ints.data();
  out->owner = o;
  return 0;
}

extern "C" void kss_synth_free(kss_synth* s) {
  if (!s || !s->owner) return;
  delete (Owner*)s->owner;
  s->owner = nullptr;
}
