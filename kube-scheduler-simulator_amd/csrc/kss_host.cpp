// kss_host.cpp — host-side parts of the boundary: the default profile, Go's math.Log,
// and lazy annotation formatting identical to the simulator's result store.
//
// Formatting restates simulator/scheduler/plugin/resultstore/store.go:133-198
// (GetStoredResult: json.Marshal of the per-node maps, sorted keys, "{}" for an
// empty map, "" for an empty selected node) and the messages the wrapped plugins
// record (wrappedplugin.go:523-548: "passed" or status.Message()).  It runs off the
// timed scheduling path, from result matrices kept in HBM.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <numeric>
#include <string>
#include <vector>

#include "kss_host.h"

double kss_go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
               L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (std::isnan(x) || x == INFINITY) return x;
  if (x < 0) return NAN;
  if (x == 0) return -INFINITY;
  int ki;
  double f1 = std::frexp(x, &ki);
  if (f1 < M_SQRT2 / 2) {
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

extern "C" double kss_go_log_c(double x) { return kss_go_log(x); }

extern "C" void kss_default_profile(kss_profile* p) {
  std::memset(p, 0, sizeof(*p));
  // simulator/scheduler/plugin/plugins_test.go:184-204 (weights); :878-1096 (args)
  p->weight[KSS_S_TAINT_TOLERATION] = 3;
  p->weight[KSS_S_NODE_AFFINITY] = 2;
  p->weight[KSS_S_NODE_RESOURCES_FIT] = 1;
  p->weight[KSS_S_VOLUME_BINDING] = 1;  // no weight in MultiPoint -> 1 (plugins.go:293-299)
  p->weight[KSS_S_POD_TOPOLOGY_SPREAD] = 2;
  p->weight[KSS_S_INTER_POD_AFFINITY] = 2;
  p->weight[KSS_S_BALANCED_ALLOCATION] = 1;
  p->weight[KSS_S_IMAGE_LOCALITY] = 1;
  for (int i = 1; i <= KSS_NFILTER; i++) p->filter_enabled |= 1u << i;
  p->score_enabled = (1u << KSS_NSCORE) - 1;
  p->fit_strategy = KSS_FIT_LEAST_ALLOCATED;
  p->fit_n = 2;
  p->fit_res[0] = KSS_RES_CPU;
  p->fit_res[1] = KSS_RES_MEMORY;
  p->fit_weight[0] = 1;
  p->fit_weight[1] = 1;
  p->ba_n = 2;
  p->ba_res[0] = KSS_RES_CPU;
  p->ba_res[1] = KSS_RES_MEMORY;
  p->hard_pod_affinity_weight = 1;
  p->pct_nodes_to_score = 100;
  p->system_defaulted = 1;
}

int kss_host_set_names(kss_host_names* dst, const kss_names* src, int n_nodes, int n_taints, int n_scalar) {
  dst->node.clear();
  dst->taint_key.clear();
  dst->taint_value.clear();
  dst->scalar.clear();
  dst->message.clear();
  if (src->node_names)
    for (int i = 0; i < n_nodes; i++) dst->node.emplace_back(src->node_names[i] ? src->node_names[i] : "");
  for (int i = 0; i < n_taints; i++) {
    dst->taint_key.emplace_back(src->taint_keys && src->taint_keys[i] ? src->taint_keys[i] : "");
    dst->taint_value.emplace_back(src->taint_values && src->taint_values[i] ? src->taint_values[i] : "");
  }
  for (int i = 0; i < n_scalar; i++) dst->scalar.emplace_back(src->scalar_names && src->scalar_names[i] ? src->scalar_names[i] : "");
  for (int i = 0; i < src->n_messages; i++) dst->message.emplace_back(src->messages && src->messages[i] ? src->messages[i] : "");
  return 0;
}

namespace {

const char* kFilterNames[KSS_NFILTER + 1] = {nullptr,           "NodeUnschedulable", "NodeName",         "TaintToleration",
                                             "NodeAffinity",    "NodePorts",         "NodeResourcesFit", "VolumeRestrictions",
                                             "EBSLimits",       "GCEPDLimits",       "NodeVolumeLimits", "AzureDiskLimits",
                                             "VolumeBinding",   "VolumeZone",        "PodTopologySpread", "InterPodAffinity"};
const char* kScoreNames[KSS_NSCORE] = {"TaintToleration",   "NodeAffinity",     "NodeResourcesFit",
                                       "VolumeBinding",     "PodTopologySpread", "InterPodAffinity",
                                       "NodeResourcesBalancedAllocation", "ImageLocality"};

// encoding/json string encoding with the default HTML escaping
void json_str(std::string& o, const std::string& s) {
  static const char* hex = "0123456789abcdef";
  o.push_back('"');
  for (size_t i = 0; i < s.size(); i++) {
    const unsigned char ch = (unsigned char)s[i];
    if (ch == '"') {
      o += "\\\"";
    } else if (ch == '\\') {
      o += "\\\\";
    } else if (ch == '\n') {
      o += "\\n";
    } else if (ch == '\r') {
      o += "\\r";
    } else if (ch == '\t') {
      o += "\\t";
    } else if (ch < 0x20 || ch == '<' || ch == '>' || ch == '&') {
      o += "\\u00";
      o.push_back(hex[ch >> 4]);
      o.push_back(hex[ch & 15]);
    } else if (ch == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
               ((unsigned char)s[i + 2] == 0xA8 || (unsigned char)s[i + 2] == 0xA9)) {
      o += (unsigned char)s[i + 2] == 0xA8 ? "\\u2028" : "\\u2029";
      i += 2;
    } else {
      o.push_back((char)ch);
    }
  }
  o.push_back('"');
}

struct KV {
  std::string k, v;
};

// json.Marshal(map[string]string) with keys sorted
std::string json_map(std::vector<KV> kv) {
  std::sort(kv.begin(), kv.end(), [](const KV& a, const KV& b) { return a.k < b.k; });
  std::string o = "{";
  for (size_t i = 0; i < kv.size(); i++) {
    if (i) o.push_back(',');
    json_str(o, kv[i].k);
    o.push_back(':');
    json_str(o, kv[i].v);
  }
  o.push_back('}');
  return o;
}

std::string fail_message(const kss_host_names* nm, int plugin, unsigned detail) {
  switch (plugin) {
    case KSS_F_NODE_UNSCHEDULABLE:
      return "node(s) were unschedulable";
    case KSS_F_NODE_NAME:
      return "node(s) didn't match the requested node name";
    case KSS_F_TAINT_TOLERATION: {
      std::string k = detail < nm->taint_key.size() ? nm->taint_key[detail] : "";
      std::string v = detail < nm->taint_value.size() ? nm->taint_value[detail] : "";
      return "node(s) had untolerated taint {" + k + ": " + v + "}";
    }
    case KSS_F_NODE_AFFINITY:
      return "node(s) didn't match Pod's node affinity/selector";
    case KSS_F_NODE_PORTS:
      return "node(s) didn't have free ports for the requested pod ports";
    case KSS_F_NODE_RESOURCES_FIT: {
      std::vector<std::string> r;
      if (detail & KSS_FIT_TOO_MANY_PODS) r.push_back("Too many pods");
      if (detail & KSS_FIT_CPU) r.push_back("Insufficient cpu");
      if (detail & KSS_FIT_MEMORY) r.push_back("Insufficient memory");
      if (detail & KSS_FIT_EPHEMERAL) r.push_back("Insufficient ephemeral-storage");
      for (int s = 0; s < KSS_MAX_SCALAR; s++)
        if (detail & (KSS_FIT_SCALAR0 << s)) r.push_back("Insufficient " + (s < (int)nm->scalar.size() ? nm->scalar[s] : std::string("?")));
      std::string o;
      for (size_t i = 0; i < r.size(); i++) o += (i ? ", " : "") + r[i];
      return o;
    }
    // volume plugins (v1.26 reason strings: volume_restrictions.go ErrReasonDiskConflict,
    // nodevolumelimits ErrReasonMaxVolumeCountExceeded, volumebinding ErrReasonNodeConflict /
    // ErrReasonPVNotExist, volume_zone.go ErrReasonConflict)
    case KSS_F_VOLUME_RESTRICTIONS:
      return "node(s) had no available disk";
    case KSS_F_EBS_LIMITS:
    case KSS_F_GCEPD_LIMITS:
    case KSS_F_NODE_VOLUME_LIMITS:
    case KSS_F_AZURE_DISK_LIMITS:
      return "node(s) exceed max volume count";
    case KSS_F_VOLUME_BINDING: {  // FindPodVolumes' reasons, joined by Status.Message()
      static const char* const kNode = "node(s) had volume node affinity conflict";
      static const char* const kBind = "node(s) didn't find available persistent volumes to bind";
      static const char* const kNoPV = "node(s) unavailable due to one or more pvc(s) bound to non-existent pv(s)";
      switch (detail) {
        case KSS_VB_PV_NOT_EXIST:
          return kNoPV;
        case KSS_VB_BIND_CONFLICT:
          return kBind;
        case KSS_VB_NODE_BIND:
          return std::string(kNode) + ", " + kBind;
        case KSS_VB_BIND_PV_NOT_EXIST:
          return std::string(kBind) + ", " + kNoPV;
        default:
          return kNode;
      }
    }
    case KSS_F_VOLUME_ZONE:
      if (detail == 0) return "node(s) had no available volume zone";
      return detail - 1 < nm->message.size() ? nm->message[detail - 1] : std::string();
    case KSS_F_POD_TOPOLOGY_SPREAD:
      return detail == KSS_PTS_MISSING_LABEL ? "node(s) didn't match pod topology spread constraints (missing required label)"
                                             : "node(s) didn't match pod topology spread constraints";
    case KSS_F_INTER_POD_AFFINITY:
      return detail == KSS_IPA_AFFINITY      ? "node(s) didn't match pod affinity rules"
             : detail == KSS_IPA_ANTI_AFFINITY ? "node(s) didn't match pod anti-affinity rules"
                                               : "node(s) didn't satisfy existing pods anti-affinity rules";
    default:
      return "";
  }
}

}  // namespace

int kss_host_prefilter_nodes(const kss_podset* ps, int32_t i, int n_nodes, std::vector<int>* out, int* has) {
  *has = 0;
  out->clear();
  if (!ps || i < 0 || i >= ps->n_pods || !ps->pods) return KSS_E_INVAL;
  const kss_pod& p = ps->pods[i];
  if (p.names_len < 0) return 0;
  if (p.names_off < 0 || p.names_off + p.names_len > ps->n_ints || (p.names_len && !ps->ints)) return KSS_E_INVAL;
  for (int k = 0; k < p.names_len; k++) {
    const int n = ps->ints[p.names_off + k];
    if (n < 0 || n >= n_nodes) return KSS_E_INVAL;
    out->push_back(n);
  }
  *has = 1;
  return 0;
}

int kss_host_format(const kss_host_names* nm, const kss_profile* prof, const kss_pod_result* res, int n_nodes, char* buf,
                    size_t cap, size_t* need, const std::vector<int>* prefilter_nodes, const kss_pod* pod) {
  if ((int)nm->node.size() < n_nodes) return KSS_E_INVAL;
  std::vector<int> order(n_nodes);
  std::iota(order.begin(), order.end(), 0);
  std::sort(order.begin(), order.end(), [&](int a, int b) { return nm->node[a] < nm->node[b]; });
  const bool scheduled = res->chosen >= 0;
  const bool prefilter_fail = res->status == 2 || res->status == 3;
  // a VolumeBinding PreFilter rejection (the pod's program says which PreFilter failed)
  const bool vb_reject = res->status == 2 && pod && pod->prefilter_status == KSS_PF_VOLUME_BINDING;
  std::vector<KV> out;
  // prefilter
  // store.go:522-534: PreFilterResult.NodeNames.List() (sorted) under the plugin's name; none on a
  // NodeAffinity conflict (a later PreFilter's rejection keeps NodeAffinity's recorded result)
  if (prefilter_nodes && (res->status != 2 || vb_reject)) {
    std::vector<std::string> names;
    for (int n : *prefilter_nodes)
      if (n >= 0 && n < n_nodes) names.push_back(nm->node[n]);
    std::sort(names.begin(), names.end());
    names.erase(std::unique(names.begin(), names.end()), names.end());
    std::string o = "{\"NodeAffinity\":[";
    for (size_t i = 0; i < names.size(); i++) {
      if (i) o.push_back(',');
      json_str(o, names[i]);
    }
    o += "]}";
    out.push_back({"scheduler-simulator/prefilter-result", o});
  } else {
    out.push_back({"scheduler-simulator/prefilter-result", "{}"});
  }
  if (vb_reject) {  // RunPreFilterPlugins stops at VolumeBinding: the ones before it succeeded
    const int m = pod->prefilter_msg;
    out.push_back({"scheduler-simulator/prefilter-result-status",
                   json_map({{"NodeAffinity", "success"}, {"NodePorts", "success"}, {"NodeResourcesFit", "success"},
                             {"VolumeRestrictions", "success"},
                             {"VolumeBinding", m >= 0 && m < (int)nm->message.size() ? nm->message[m] : std::string()}})});
  } else if (res->status == 2) {
    out.push_back({"scheduler-simulator/prefilter-result-status", json_map({{"NodeAffinity", "pod affinity terms conflict"}})});
  } else {
    out.push_back({"scheduler-simulator/prefilter-result-status",
                   json_map({{"InterPodAffinity", "success"}, {"NodeAffinity", "success"}, {"NodePorts", "success"},
                             {"NodeResourcesFit", "success"}, {"PodTopologySpread", "success"},
                             {"VolumeBinding", "success"}, {"VolumeRestrictions", "success"}})});
  }
  // filter-result: plugins up to and including the first failure, per evaluated node
  {
    std::string o = "{";
    bool firstn = true;
    for (int n : order) {
      const int fp = res->fail_plugin ? res->fail_plugin[n] : KSS_F_NOT_EVALUATED;
      if (fp == KSS_F_NOT_EVALUATED || prefilter_fail) continue;
      std::vector<KV> kv;
      for (int f = 1; f <= KSS_NFILTER; f++) {
        if (!((prof->filter_enabled >> f) & 1u)) continue;
        if (f == fp) {
          kv.push_back({kFilterNames[f], fail_message(nm, f, res->fail_detail ? res->fail_detail[n] : 0)});
          break;
        }
        kv.push_back({kFilterNames[f], "passed"});
      }
      if (!firstn) o.push_back(',');
      firstn = false;
      json_str(o, nm->node[n]);
      o.push_back(':');
      o += json_map(kv);
    }
    o.push_back('}');
    out.push_back({"scheduler-simulator/filter-result", o});
  }
  // postfilter-result: DefaultPreemption records every node of the status map (no victims -> {})
  {
    std::string o = "{";
    if (!scheduled) {
      bool firstn = true;
      for (int n : order) {
        const int fp = res->fail_plugin ? res->fail_plugin[n] : KSS_F_NOT_EVALUATED;
        if (!prefilter_fail && fp == KSS_F_NOT_EVALUATED) continue;
        if (!firstn) o.push_back(',');
        firstn = false;
        json_str(o, nm->node[n]);
        o += ":{}";
      }
    }
    o.push_back('}');
    out.push_back({"scheduler-simulator/postfilter-result", o});
  }
  const bool scored = res->scored != 0;
  out.push_back({"scheduler-simulator/prescore-result",
                 scored ? json_map({{"InterPodAffinity", "success"}, {"NodeAffinity", "success"},
                                    {"PodTopologySpread", "success"}, {"TaintToleration", "success"}})
                        : "{}"});
  for (int which = 0; which < 2; which++) {
    std::string o = "{";
    if (scored) {
      bool firstn = true;
      for (int n : order) {
        if (!res->fail_plugin || res->fail_plugin[n] != KSS_F_PASS) continue;
        if (res->fail_detail && res->fail_detail[n] == KSS_PASS_NOT_KEPT) continue;  // filtered, not in the feasible list
        std::vector<KV> kv;
        for (int s = 0; s < KSS_NSCORE; s++) {
          if (!((prof->score_enabled >> s) & 1u)) continue;
          long long v = which == 0 ? res->raw[(size_t)s * n_nodes + n] : res->norm[(size_t)s * n_nodes + n] * prof->weight[s];
          kv.push_back({kScoreNames[s], std::to_string(v)});
        }
        if (!firstn) o.push_back(',');
        firstn = false;
        json_str(o, nm->node[n]);
        o.push_back(':');
        o += json_map(kv);
      }
    }
    o.push_back('}');
    out.push_back({which == 0 ? "scheduler-simulator/score-result" : "scheduler-simulator/finalscore-result", o});
  }
  out.push_back({"scheduler-simulator/reserve-result", scheduled ? json_map({{"VolumeBinding", "success"}}) : "{}"});
  out.push_back({"scheduler-simulator/permit-result", "{}"});
  out.push_back({"scheduler-simulator/permit-result-timeout", "{}"});
  out.push_back({"scheduler-simulator/prebind-result", scheduled ? json_map({{"VolumeBinding", "success"}}) : "{}"});
  out.push_back({"scheduler-simulator/bind-result", scheduled ? json_map({{"DefaultBinder", "success"}}) : "{}"});
  out.push_back({"scheduler-simulator/selected-node",
                 scheduled && res->chosen < n_nodes ? nm->node[res->chosen] : std::string()});
  size_t total = 1;
  for (auto& kv : out) total += kv.k.size() + 1 + kv.v.size() + 1;
  *need = total;
  if (cap < total || !buf) return cap == 0 ? 0 : KSS_E_RANGE;
  char* p = buf;
  for (auto& kv : out) {
    std::memcpy(p, kv.k.data(), kv.k.size());
    p += kv.k.size();
    *p++ = 0;
    std::memcpy(p, kv.v.data(), kv.v.size());
    p += kv.v.size();
    *p++ = 0;
  }
  *p = 0;
  return 0;
}

extern "C" int kss_format_annotations_ex(const kss_names* names, const kss_profile* prof, const kss_pod_result* res,
                                         int32_t n_nodes, int32_t n_taints, int32_t n_scalar, char* buf, size_t cap,
                                         size_t* need) {
  if (!names || !prof || !res || !need || n_nodes < 0) return KSS_E_INVAL;
  kss_host_names nm;
  kss_host_set_names(&nm, names, n_nodes, n_taints, n_scalar);
  return kss_host_format(&nm, prof, res, n_nodes, buf, cap, need);
}

extern "C" int kss_format_pod_annotations_ex(const kss_names* names, const kss_profile* prof, const kss_podset* ps,
                                             int32_t pod_index, const kss_pod_result* res, int32_t n_nodes,
                                             int32_t n_taints, int32_t n_scalar, char* buf, size_t cap, size_t* need) {
  if (!names || !prof || !res || !need || n_nodes < 0) return KSS_E_INVAL;
  std::vector<int> pf;
  int has = 0;
  int rc = kss_host_prefilter_nodes(ps, pod_index, n_nodes, &pf, &has);
  if (rc) return rc;
  kss_host_names nm;
  kss_host_set_names(&nm, names, n_nodes, n_taints, n_scalar);
  return kss_host_format(&nm, prof, res, n_nodes, buf, cap, need, has ? &pf : nullptr, &ps->pods[pod_index]);
}
