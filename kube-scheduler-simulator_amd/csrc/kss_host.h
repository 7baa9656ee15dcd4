// kss_host.h — host-side helpers of libkss.so (no device code).
#pragma once
#include <string>
#include <vector>

#include "../../include/kss.h"

struct kss_host_names {
  std::vector<std::string> node, taint_key, taint_value, scalar, message;
};

// Go math.Log restated (src/math/log.go); used for the PodTopologySpread weight table.
double kss_go_log(double x);

int kss_host_set_names(kss_host_names* dst, const kss_names* src, int n_nodes, int n_taints, int n_scalar);

// resultstore.Store.GetStoredResult formatting (store.go:133-198) of one pod result.
// prefilter_nodes: the NodeAffinity PreFilterResult node set (global indices) or null for none;
// pod: the pod's program (its PreFilter status and message), or null.
int kss_host_format(const kss_host_names* names, const kss_profile* prof, const kss_pod_result* res, int n_nodes,
                    char* buf, size_t cap, size_t* need, const std::vector<int>* prefilter_nodes = nullptr,
                    const kss_pod* pod = nullptr);

// The PreFilterResult node set of ps->pods[i] (KSS_E_INVAL on a bad index or list); *has = 0 when
// the pod's PreFilter returned none.
int kss_host_prefilter_nodes(const kss_podset* ps, int32_t i, int n_nodes, std::vector<int>* out, int* has);
