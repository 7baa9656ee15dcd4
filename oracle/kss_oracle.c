/*
 * kss_oracle.c — CPU ORACLE (TEST INFRASTRUCTURE ONLY).
 *
 * Plain-C restatement, in reference operation order, of the scheduling-cycle hot
 * path of kube-scheduler-simulator (upstream k8s.io/kubernetes v1.26.2, pinned at
 * /root/reference/simulator/go.mod:56; the module is not vendored and cannot be
 * fetched here, so every ⟨k8s⟩ citation below names the upstream function).
 * It works on the same struct-of-arrays input (include/kss.h) as the HIP path and
 * is used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
 * as the checker.  Nothing in the product links against it.
 *
 * Parity status: the restatement is pinned by the reference's own known-answer
 * vector (README.md:61-79 / simulator/docs/debuggable-scheduler.md:17-35: Fit 73,
 * BalancedAllocation 76, TaintToleration 0->300, PodTopologySpread 0->200) and is
 * cross-checked against the independent object-level Python restatement
 * (oracle/k8s_oracle.py).  Everything else is "parity vs the restated spec"
 * (the Go reference is unbuildable in this container).
 *
 * Selection tie-break: max TotalScore, then LOWEST canonical node index (the
 * reference's selectHost, scheduler/scheduler.go:323-344, samples ties with
 * math/rand; north_star fixes a deterministic rule).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/kss.h"

#define MAXKEYS_PER_POD 16

/* ---------------------------------------------------------------------------
 * Go's math.Log restated (src/math/log.go, FreeBSD e_log.c): used for the
 * PodTopologySpread normalizing weight math.Log(float64(size+2)).
 * Compiled with -ffp-contract=off so no FMA is formed (Go amd64, GOAMD64=v1).
 * ------------------------------------------------------------------------- */
static double go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
               L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (x != x || x == INFINITY) return x;
  if (x < 0) return NAN;
  if (x == 0) return -INFINITY;
  int ki;
  double f1 = frexp(x, &ki);
  if (f1 < M_SQRT2 / 2) {
    f1 *= 2;
    ki--;
  }
  double f = f1 - 1;
  double k = (double)ki;
  double s = f / (2 + f);
  double s2 = s * s;
  double s4 = s2 * s2;
  double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  double R = t1 + t2;
  double hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

double kss_oracle_go_log(double x) { return go_log(x); }

/* Go math.Round: half away from zero (src/math/floor.go Round) == C round(). */
static int64_t go_round_to_i64(double x) { return (int64_t)round(x); }

/* ---------------------------------------------------------------------------
 * mutable oracle state: a private copy of the node columns that commits change
 * ------------------------------------------------------------------------- */
typedef struct {
  kss_cluster c; /* pointers below point into owned arrays */
  int64_t* requested;
  int64_t* nonzero;
  int32_t* pod_count;
  int32_t* class_count;
  int32_t* term_count;
  uint64_t* port_used;
  int32_t* vol_count;
  int32_t* vol_attached;
  int32_t* pv_owner;   /* the binder's assume cache (kss_cluster pv_owner / claim_node) */
  int32_t* claim_node;
  int32_t cursor; /* the scheduler's nextStartNodeIndex (schedule_one.go findNodesThatPassFilters) */
  /* the scheduling queue's nominator (PodNominator): pods of ps nominated to a node by an earlier
     preemption; a nomination leaves when its pod is assumed (DeleteNominatedPodIfExists) */
  int n_nom;
  const int32_t* nom_pod;  /* [n_nom] index in ps */
  const int32_t* nom_node; /* [n_nom] local node */
  uint8_t* nom_active;     /* [n_nom] */
} ostate;

static int ostate_init(ostate* s, const kss_cluster* cl) {
  size_t N = (size_t)cl->n_nodes;
  s->c = *cl;
  s->cursor = 0;
  s->n_nom = 0;
  s->nom_pod = s->nom_node = NULL;
  s->nom_active = NULL;
  s->requested = (int64_t*)malloc(sizeof(int64_t) * KSS_NRES * (N ? N : 1));
  s->nonzero = (int64_t*)malloc(sizeof(int64_t) * 2 * (N ? N : 1));
  s->pod_count = (int32_t*)malloc(sizeof(int32_t) * (N ? N : 1));
  s->class_count = (int32_t*)malloc(sizeof(int32_t) * ((size_t)cl->n_classes * N + 1));
  s->term_count = (int32_t*)malloc(sizeof(int32_t) * ((size_t)cl->n_terms * N + 1));
  s->port_used = (uint64_t*)calloc(N ? N : 1, sizeof(uint64_t));
  s->vol_count = (int32_t*)calloc((size_t)cl->n_vol_rows * N + 1, sizeof(int32_t));
  s->vol_attached = (int32_t*)calloc((size_t)cl->n_vol_keys * N + 1, sizeof(int32_t));
  s->pv_owner = (int32_t*)calloc((size_t)cl->n_pvs + 1, sizeof(int32_t));
  s->claim_node = (int32_t*)calloc((size_t)cl->n_wclaims + 1, sizeof(int32_t));
  if (!s->requested || !s->nonzero || !s->pod_count || !s->class_count || !s->term_count || !s->port_used ||
      !s->vol_count || !s->vol_attached || !s->pv_owner || !s->claim_node)
    return -1;
  if (cl->n_pvs) memcpy(s->pv_owner, cl->pv_owner, sizeof(int32_t) * (size_t)cl->n_pvs);
  if (cl->n_wclaims) memcpy(s->claim_node, cl->claim_node, sizeof(int32_t) * (size_t)cl->n_wclaims);
  if (cl->n_vol_rows) memcpy(s->vol_count, cl->vol_count, sizeof(int32_t) * (size_t)cl->n_vol_rows * N);
  if (cl->n_vol_keys) memcpy(s->vol_attached, cl->vol_attached, sizeof(int32_t) * (size_t)cl->n_vol_keys * N);
  if (cl->port_used) memcpy(s->port_used, cl->port_used, sizeof(uint64_t) * N);
  memcpy(s->requested, cl->requested, sizeof(int64_t) * KSS_NRES * N);
  memcpy(s->nonzero, cl->nonzero, sizeof(int64_t) * 2 * N);
  memcpy(s->pod_count, cl->pod_count, sizeof(int32_t) * N);
  if (cl->n_classes) memcpy(s->class_count, cl->class_count, sizeof(int32_t) * (size_t)cl->n_classes * N);
  if (cl->n_terms) memcpy(s->term_count, cl->term_count, sizeof(int32_t) * (size_t)cl->n_terms * N);
  s->c.requested = s->requested;
  s->c.nonzero = s->nonzero;
  s->c.pod_count = s->pod_count;
  s->c.class_count = s->class_count;
  s->c.term_count = s->term_count;
  s->c.port_used = s->port_used;
  s->c.vol_count = s->vol_count;
  s->c.vol_attached = s->vol_attached;
  s->c.pv_owner = s->pv_owner;
  s->c.claim_node = s->claim_node;
  return 0;
}

static void ostate_free(ostate* s) {
  free(s->requested);
  free(s->nonzero);
  free(s->pod_count);
  free(s->class_count);
  free(s->term_count);
  free(s->port_used);
  free(s->vol_count);
  free(s->vol_attached);
  free(s->pv_owner);
  free(s->claim_node);
  free(s->nom_active);
}

#define LV(cl, key, n) ((cl)->label_value[(size_t)(key) * (size_t)(cl)->n_nodes + (size_t)(n)])

/* labels.Requirement.Matches (apimachinery labels/selector.go) over interned ids,
 * plus the metadata.name field selector (component-helpers nodeaffinity). */
static int req_matches(const kss_cluster* cl, const kss_podset* ps, const kss_req* r, int n) {
  int64_t gidx = (int64_t)cl->node_base + n;
  switch (r->op) {
    case KSS_OP_FALSE:
      return 0;
    case KSS_OP_TRUE:
      return 1;
    case KSS_OP_NAME_IN:
      return r->ival >= 0 && gidx == r->ival;
    case KSS_OP_NAME_NOTIN:
      return !(r->ival >= 0 && gidx == r->ival);
    default:
      break;
  }
  int32_t v = LV(cl, r->key, n);
  switch (r->op) {
    case KSS_OP_MASK:
      if (v < 0) return (int)((r->mask >> 63) & 1u);
      return v < 63 ? (int)((r->mask >> v) & 1u) : 0;
    case KSS_OP_IN:
      if (v < 0) return 0;
      for (int i = 0; i < r->list_len; i++)
        if (ps->ints[r->list_off + i] == v) return 1;
      return 0;
    case KSS_OP_NOTIN:
      if (v < 0) return 1;
      for (int i = 0; i < r->list_len; i++)
        if (ps->ints[r->list_off + i] == v) return 0;
      return 1;
    case KSS_OP_EXISTS:
      return v >= 0;
    case KSS_OP_DNE:
      return v < 0;
    case KSS_OP_GT:
    case KSS_OP_LT: {
      if (v < 0) return 0;
      int32_t g = cl->key_base[r->key] + v;
      if (!cl->value_is_int[g]) return 0;
      return r->op == KSS_OP_GT ? cl->value_int[g] > r->ival : cl->value_int[g] < r->ival;
    }
    default:
      return 0;
  }
}

/* nodeSelectorTerm.match: AND over its requirements */
static int term_matches(const kss_cluster* cl, const kss_podset* ps, const kss_term* t, int n) {
  for (int i = 0; i < t->req_len; i++)
    if (!req_matches(cl, ps, &ps->reqs[t->req_off + i], n)) return 0;
  return 1;
}

/* nodeaffinity.RequiredNodeAffinity.Match (component-helpers):
 * nodeSelector labels AND (OR over parsed NodeSelectorTerms). */
static int required_node_affinity(const kss_cluster* cl, const kss_podset* ps, const kss_pod* p, int n) {
  for (int i = 0; i < p->sel_len; i++)
    if (!req_matches(cl, ps, &ps->reqs[p->sel_off + i], n)) return 0;
  if (p->flags & KSS_POD_HAS_REQ_AFFINITY) {
    for (int t = 0; t < p->aff_len; t++)
      if (term_matches(cl, ps, &ps->terms[p->aff_off + t], n)) return 1;
    return 0;
  }
  return 1;
}

/* v1helper.FindMatchingUntoleratedTaint(node.Spec.Taints, tolerations, DoNotScheduleTaintsFilterFunc) */
static int first_untolerated_taint(const kss_cluster* cl, const kss_pod* p, int n) {
  uint64_t untol = cl->taint_hard[n] & ~p->tol_hard;
  if (!untol) return -1;
  const uint8_t* ord = cl->taint_order + (size_t)n * KSS_TAINT_ORDER;
  for (int i = 0; i < KSS_TAINT_ORDER && ord[i] != 0xFF; i++)
    if ((untol >> ord[i]) & 1u) return ord[i];
  return 63 - __builtin_clzll(untol); /* unreachable for well-formed input */
}

static int64_t sum_rows(const int32_t* mat, size_t N, const int32_t* rows, int len, int n) {
  int64_t s = 0;
  for (int i = 0; i < len; i++) s += mat[(size_t)rows[i] * N + (size_t)n];
  return s;
}

/* per-pod PreFilter / PreScore state for PodTopologySpread and InterPodAffinity */
typedef struct {
  /* PTS hard: per topology key (v1.26 keys TpPairToMatchNum by pair): the histogram and the
     critical-path minimum live at the key's first constraint hard_own[i]; bins = card+1 */
  int hard_own[8];
  int64_t* hard_cnt[8];
  uint8_t* hard_present[8];
  int64_t hard_min[8];
  /* IPA: per (entry kind, key) histograms */
  int nkeys;
  int keys[MAXKEYS_PER_POD];
  int64_t* hx[MAXKEYS_PER_POD]; /* existing anti-affinity */
  int64_t* ha[MAXKEYS_PER_POD]; /* incoming affinity */
  int64_t* hb[MAXKEYS_PER_POD]; /* incoming anti-affinity */
  int64_t* hs[MAXKEYS_PER_POD]; /* score topologyScore */
  int ex_nonempty, aff_nonempty, anti_nonempty, score_nonempty;
} podstate;

static int key_slot(podstate* st, int key) {
  for (int i = 0; i < st->nkeys; i++)
    if (st->keys[i] == key) return i;
  return -1;
}

static int spread_policy_ok(const kss_cluster* cl, const kss_podset* ps, const kss_pod* p, const kss_spread* sp,
                            int n) {
  /* topologySpreadConstraint.matchNodeInclusionPolicies (NodeInclusionPolicy beta, on in v1.26) */
  if ((sp->flags & KSS_SPREAD_POLICY_AFFINITY_HONOR) && !required_node_affinity(cl, ps, p, n)) return 0;
  if ((sp->flags & KSS_SPREAD_POLICY_TAINTS_HONOR) && first_untolerated_taint(cl, p, n) >= 0) return 0;
  return 1;
}

static int has_all_keys(const kss_cluster* cl, const kss_spread* sp, int cnt, int n) {
  for (int i = 0; i < cnt; i++)
    if (LV(cl, sp[i].key, n) < 0) return 0;
  return 1;
}

static void podstate_free(podstate* st) {
  for (int i = 0; i < 8; i++) {
    free(st->hard_cnt[i]);
    free(st->hard_present[i]);
  }
  for (int i = 0; i < st->nkeys; i++) {
    free(st->hx[i]);
    free(st->ha[i]);
    free(st->hb[i]);
    free(st->hs[i]);
  }
}

/* PodTopologySpread PreFilter (calPreFilterState) and InterPodAffinity PreFilter
 * (getExistingAntiAffinityCounts, getIncomingAffinityAntiAffinityCounts) and
 * InterPodAffinity PreScore (processExistingPod) — all scan every node. */
static int podstate_build(podstate* st, const kss_cluster* cl, const kss_podset* ps, const kss_pod* p,
                          int hard_pod_affinity_weight) {
  memset(st, 0, sizeof(*st));
  size_t N = (size_t)cl->n_nodes;
  const kss_spread* hard = ps->spreads + p->spread_off;
  if (p->n_hard > 8 || p->n_soft > 8) return KSS_E_UNSUPPORTED;
  for (int i = 0; i < p->n_hard; i++) {
    st->hard_own[i] = i;
    for (int j = 0; j < i; j++)
      if (hard[j].key == hard[i].key) {
        st->hard_own[i] = j;
        break;
      }
    if (st->hard_own[i] != i) continue;
    int bins = cl->key_card[hard[i].key] + 1;
    st->hard_cnt[i] = (int64_t*)calloc((size_t)bins, sizeof(int64_t));
    st->hard_present[i] = (uint8_t*)calloc((size_t)bins, 1);
  }
  for (size_t n = 0; n < N; n++) {
    if (!has_all_keys(cl, hard, p->n_hard, (int)n)) continue; /* nodeLabelsMatchSpreadConstraints */
    /* tpCounts[pair] = count for each admitting constraint in order: per key, the count of the
       key's LAST constraint that admits the node (matchNodeInclusionPolicies) */
    for (int i = 0; i < p->n_hard; i++) {
      if (st->hard_own[i] != i) continue;
      int64_t eff = -1;
      for (int j = i; j < p->n_hard; j++) {
        if (st->hard_own[j] != i || !spread_policy_ok(cl, ps, p, &hard[j], (int)n)) continue;
        /* countPodsMatchSelector(nodeInfo.Pods, selector, pod.Namespace) */
        eff = sum_rows(cl->class_count, N, ps->ints + hard[j].cls_off, hard[j].cls_len, (int)n);
      }
      if (eff < 0) continue;
      int d = LV(cl, hard[i].key, n);
      st->hard_cnt[i][d] += eff; /* TpPairToMatchNum[tp] += count */
      st->hard_present[i][d] = 1;
    }
  }
  for (int i = 0; i < p->n_hard; i++) {
    if (st->hard_own[i] != i) continue;
    /* TpKeyToCriticalPaths[key] paths[0].MatchNum: minimum over the key's pairs, MaxInt32 if none */
    int64_t mn = INT32_MAX;
    int bins = cl->key_card[hard[i].key] + 1;
    for (int d = 0; d < bins; d++)
      if (st->hard_present[i][d] && st->hard_cnt[i][d] < mn) mn = st->hard_cnt[i][d];
    st->hard_min[i] = mn;
  }

  /* inter-pod affinity histograms, per distinct topology key */
  const kss_ipa* ipa = ps->ipa + p->ipa_off;
  for (int e = 0; e < p->ipa_len; e++) {
    if (ipa[e].kind == KSS_IPA_SCORE_TERM && hard_pod_affinity_weight == 0 && ipa[e].coef == 0) continue;
    if (key_slot(st, ipa[e].key) < 0) {
      if (st->nkeys >= MAXKEYS_PER_POD) return KSS_E_UNSUPPORTED;
      int k = st->nkeys++;
      int bins = cl->key_card[ipa[e].key] + 1;
      st->keys[k] = ipa[e].key;
      st->hx[k] = (int64_t*)calloc((size_t)bins, sizeof(int64_t));
      st->ha[k] = (int64_t*)calloc((size_t)bins, sizeof(int64_t));
      st->hb[k] = (int64_t*)calloc((size_t)bins, sizeof(int64_t));
      st->hs[k] = (int64_t*)calloc((size_t)bins, sizeof(int64_t));
    }
  }
  for (size_t n = 0; n < N; n++) {
    int has_labels = (cl->node_flags[n] & KSS_NODE_HAS_LABELS) != 0;
    for (int e = 0; e < p->ipa_len; e++) {
      const kss_ipa* en = &ipa[e];
      int d = LV(cl, en->key, n);
      if (d < 0) continue; /* topologyToMatchedTermCount.update / scoreMap.processTerm: node lacks key */
      int k = key_slot(st, en->key);
      const int32_t* rows = ps->ints + en->row_off;
      switch (en->kind) {
        case KSS_IPA_EXISTING_ANTI: {
          int64_t c = sum_rows(cl->term_count, N, rows, en->row_len, (int)n);
          st->hx[k][d] += c;
          break;
        }
        case KSS_IPA_REQ_AFFINITY: {
          int64_t c = sum_rows(cl->class_count, N, rows, en->row_len, (int)n);
          st->ha[k][d] += c;
          break;
        }
        case KSS_IPA_REQ_ANTI: {
          int64_t c = sum_rows(cl->class_count, N, rows, en->row_len, (int)n);
          st->hb[k][d] += c;
          break;
        }
        case KSS_IPA_SCORE_CLASS:
        case KSS_IPA_SCORE_TERM: {
          if (!has_labels) break; /* processExistingPod: len(existingPodNode.Labels) == 0 -> return */
          const int32_t* mat = en->kind == KSS_IPA_SCORE_CLASS ? cl->class_count : cl->term_count;
          int64_t c = sum_rows(mat, N, rows, en->row_len, (int)n);
          if (c > 0) st->score_nonempty = 1;
          st->hs[k][d] += c * (int64_t)en->coef;
          break;
        }
      }
    }
  }
  for (int k = 0; k < st->nkeys; k++) {
    int bins = cl->key_card[st->keys[k]] + 1;
    for (int d = 0; d < bins; d++) {
      if (st->hx[k][d] > 0) st->ex_nonempty = 1;
      if (st->ha[k][d] > 0) st->aff_nonempty = 1;
      if (st->hb[k][d] > 0) st->anti_nonempty = 1;
    }
  }
  return 0;
}

/* ---------------------------------------------------------------------------
 * Volume filters over the pod's volume program (include/kss.h kss_vol; the host resolved
 * the objects into rows, keys and requirements, kss/volumes.py).  Restated per plugin:
 *   VolumeRestrictions  volume_restrictions.go satisfyVolumeConflicts: some pod on the node
 *                       uses a disk one of the pod's volumes conflicts with (isVolumeConflict);
 *   EBSLimits / GCEPDLimits / AzureDiskLimits  non_csi.go nonCSILimits.Filter:
 *                       len(existingVolumes) + len(newVolumes \ existingVolumes) > maxAttachLimit,
 *                       whenever the pod has a volume of the plugin, unless migrated (limit -1);
 *   NodeVolumeLimits    csi.go CSILimits.Filter: per limit key with new volumes,
 *                       attachedVolumeCount + newVolumeCount > the node's limit for the key;
 *   VolumeBinding       binder.go checkBoundClaims: bound claims in order, the first missing
 *                       PV or PV node-affinity mismatch decides;
 *   VolumeZone          volume_zone.go Filter: nodes without zone labels pass; otherwise every
 *                       zone label of the pod's PVs must contain the node's value (volume order).
 * Returns the plugin id or 0.
 * ------------------------------------------------------------------------- */
static int limit_check(const kss_cluster* cl, uint32_t en, int key, int n, int64_t newc) {
  size_t N = (size_t)cl->n_nodes;
  int pl = cl->vol_key_plugin[key];
  int32_t lim = cl->vol_limit[(size_t)key * N + n];
  if (!((en >> pl) & 1u) || lim < 0) return 0;
  if (pl == KSS_F_NODE_VOLUME_LIMITS && newc == 0) return 0; /* only keys in newVolumeCount */
  return (int64_t)cl->vol_attached[(size_t)key * N + n] + newc > (int64_t)lim ? pl : 0;
}

static int is_vb(int k) { return k == KSS_VOL_BIND_AFFINITY || k == KSS_VOL_BIND_PV_MISSING || k == KSS_VOL_BIND_WFFC; }

/* pv_helpers.go FindMatchingVolume (delayBinding, scheduler path) for delayed claim entry v on node
   n over its candidates (ints triplets {pv, term_off, term_len}, smallest capacity first, then
   name; the host applied every node-independent check): the PV bound to the claim (claimRef or
   assumed: pv_owner == key + 1) answers wherever it comes -- itself if its node affinity holds,
   else nothing; otherwise the first available candidate not among chosen[0, nch) whose node
   affinity holds.  -1: no match. */
static int pv_affinity_ok(const kss_cluster* cl, const kss_podset* ps, const kss_vol* v, int i, int n) {
  int ta = ps->ints[v->a + 3 * i + 1], tb = ps->ints[v->a + 3 * i + 2];
  if (tb < 0) return 1; /* CheckNodeAffinity: no required node affinity */
  for (int t = 0; t < tb; t++)
    if (term_matches(cl, ps, &ps->terms[ta + t], n)) return 1;
  return 0;
}
static int find_matching_volume(const kss_cluster* cl, const kss_podset* ps, const kss_vol* v, const int* chosen, int nch,
                                int n) {
  for (int i = 0; i < v->b; i++) { /* excludedVolumes come first: a PV an earlier claim took is skipped */
    int pv = ps->ints[v->a + 3 * i], taken = 0;
    for (int k = 0; k < nch; k++) taken |= chosen[k] == pv;
    if (!taken && cl->pv_owner[pv] == v->key + 1) return pv_affinity_ok(cl, ps, v, i, n) ? pv : -1;
  }
  for (int i = 0; i < v->b; i++) {
    int pv = ps->ints[v->a + 3 * i], taken = 0;
    if (cl->pv_owner[pv] != 0) continue; /* claimRef set to another claim */
    for (int k = 0; k < nch; k++) taken |= chosen[k] == pv;
    if (!taken && pv_affinity_ok(cl, ps, v, i, n)) return pv;
  }
  return -1;
}

/* binder.go FindPodVolumes over VolumeBinding entries [e0, e1) of the pod on node n: -1 when
   satisfied, else the KSS_VB_* detail.  pick (optional, one per BIND_WFFC entry): the static
   binding's PV, -1 for a claim to provision. */
static int find_pod_volumes(const kss_cluster* cl, const kss_podset* ps, int e0, int e1, int n, int* pick) {
  int bound = 0; /* checkBoundClaims: 1 node conflict, 2 PV not found; the first failure ends it */
  for (int e = e0; e < e1 && !bound; e++) {
    const kss_vol* v = &ps->vols[e];
    if (v->kind == KSS_VOL_BIND_PV_MISSING) {
      bound = 2;
    } else if (v->kind == KSS_VOL_BIND_AFFINITY) {
      int ok = 0;
      for (int t = 0; t < v->b && !ok; t++) ok = term_matches(cl, ps, &ps->terms[v->a + t], n);
      if (!ok) bound = 1;
    }
  }
  int unbound_ok = 1;
  for (int e = e0; e < e1 && unbound_ok; e++) /* claims whose selected-node annotation names another node */
    if (ps->vols[e].kind == KSS_VOL_BIND_WFFC) {
      int sel = cl->claim_node[ps->vols[e].key];
      if (sel != -1 && sel != n) unbound_ok = 0;
    }
  if (unbound_ok) {
    int chosen[KSS_MAX_WFFC], nch = 0, wi = 0, to_prov[KSS_MAX_WFFC] = {0, 0, 0, 0}, any = 0;
    for (int e = e0; e < e1; e++) { /* findMatchingVolumes: entries come by increasing request */
      const kss_vol* v = &ps->vols[e];
      if (v->kind != KSS_VOL_BIND_WFFC) continue;
      int m = -1;
      if (cl->claim_node[v->key] == -1) {
        m = find_matching_volume(cl, ps, v, chosen, nch, n);
        if (m >= 0) chosen[nch++] = m;
        else unbound_ok = 0;
      }
      if (m < 0) to_prov[wi] = any = 1;
      if (pick) pick[wi] = m;
      wi++;
    }
    if (any) { /* checkVolumeProvisions: a provisioner whose class's allowedTopologies admit the node */
      unbound_ok = 1;
      wi = 0;
      for (int e = e0; e < e1 && unbound_ok; e++) {
        const kss_vol* v = &ps->vols[e];
        if (v->kind != KSS_VOL_BIND_WFFC) continue;
        if (to_prov[wi]) {
          if (!(v->count & 1)) {
            unbound_ok = 0;
          } else if ((v->count >> 1) > 0) {
            int ok = 0;
            for (int t = 0; t < (v->count >> 1) && !ok; t++) ok = term_matches(cl, ps, &ps->terms[v->row + t], n);
            unbound_ok = ok;
          }
        }
        wi++;
      }
    }
  }
  if (!unbound_ok) return bound == 1 ? KSS_VB_NODE_BIND : (bound == 2 ? KSS_VB_BIND_PV_NOT_EXIST : KSS_VB_BIND_CONFLICT);
  return bound == 1 ? KSS_VB_NODE_CONFLICT : (bound == 2 ? KSS_VB_PV_NOT_EXIST : -1);
}

static int volume_filters(const kss_cluster* cl, const kss_podset* ps, const kss_pod* p, uint32_t en, int n,
                          uint16_t* detail) {
  size_t N = (size_t)cl->n_nodes;
  int zone_node = (cl->node_flags[n] & KSS_NODE_VOLUME_ZONE) != 0;
  int cur = -1, r;
  int64_t newc = 0;
  for (int e = 0; e < p->vol_len; e++) {
    const kss_vol* v = &ps->vols[p->vol_off + e];
    if (v->kind != KSS_VOL_LIMIT && cur >= 0) {
      if ((r = limit_check(cl, en, cur, n, newc))) return r;
      cur = -1;
    }
    if (v->kind == KSS_VOL_CONFLICT) {
      if (((en >> KSS_F_VOLUME_RESTRICTIONS) & 1u) && cl->vol_count[(size_t)v->row * N + n] > 0)
        return KSS_F_VOLUME_RESTRICTIONS;
    } else if (v->kind == KSS_VOL_LIMIT) {
      if (v->key != cur) {
        if (cur >= 0 && (r = limit_check(cl, en, cur, n, newc))) return r;
        cur = v->key;
        newc = 0;
      }
      if (v->row >= 0)
        newc += cl->vol_count[(size_t)v->row * N + n] == 0 ? 1 : 0; /* delete(newVolumes, attached) */
      else
        newc += v->count;
    } else if (is_vb(v->kind)) { /* VolumeBinding: its consecutive entries as one FindPodVolumes */
      int e1 = e + 1;
      while (e1 < p->vol_len && is_vb(ps->vols[p->vol_off + e1].kind)) e1++;
      if ((en >> KSS_F_VOLUME_BINDING) & 1u) {
        int d = find_pod_volumes(cl, ps, p->vol_off + e, p->vol_off + e1, n, NULL);
        if (d >= 0) {
          *detail = (uint16_t)d;
          return KSS_F_VOLUME_BINDING;
        }
      }
      e = e1 - 1;
    } else if (v->kind == KSS_VOL_ZONE) {
      if (((en >> KSS_F_VOLUME_ZONE) & 1u) && zone_node)
        for (int k = 0; k < v->b; k++)
          if (!req_matches(cl, ps, &ps->reqs[v->a + k], n)) {
            *detail = 0;
            return KSS_F_VOLUME_ZONE;
          }
    } else if (v->kind == KSS_VOL_ZONE_ERROR) {
      if (((en >> KSS_F_VOLUME_ZONE) & 1u) && zone_node) {
        *detail = (uint16_t)(1 + v->a);
        return KSS_F_VOLUME_ZONE;
      }
    } else {
      break; /* AssumePod entries */
    }
  }
  if (cur >= 0) return limit_check(cl, en, cur, n, newc);
  return 0;
}

/* ---------------------------------------------------------------------------
 * Filter chain for one node (RunFilterPlugins, first failure wins).
 * Returns the failing plugin id (0 = pass) and sets *detail.
 * ------------------------------------------------------------------------- */
static int filter_node(const kss_profile* prof, const kss_cluster* cl, const kss_podset* ps, const kss_pod* p,
                       const podstate* st, int n, uint16_t* detail) {
  uint32_t en = prof->filter_enabled;
  *detail = 0;
  /* NodeUnschedulable.Filter */
  if ((en >> KSS_F_NODE_UNSCHEDULABLE) & 1u) {
    if ((cl->node_flags[n] & KSS_NODE_UNSCHEDULABLE) && !(p->flags & KSS_POD_TOL_UNSCHEDULABLE))
      return KSS_F_NODE_UNSCHEDULABLE;
  }
  /* NodeName.Filter: len(pod.Spec.NodeName)==0 || == node.Name */
  if ((en >> KSS_F_NODE_NAME) & 1u) {
    if (p->node_name != -1 && (int64_t)p->node_name != (int64_t)cl->node_base + n) return KSS_F_NODE_NAME;
  }
  /* TaintToleration.Filter */
  if ((en >> KSS_F_TAINT_TOLERATION) & 1u) {
    int t = first_untolerated_taint(cl, p, n);
    if (t >= 0) {
      *detail = (uint16_t)t;
      return KSS_F_TAINT_TOLERATION;
    }
  }
  /* NodeAffinity.Filter */
  if ((en >> KSS_F_NODE_AFFINITY) & 1u) {
    if (!required_node_affinity(cl, ps, p, n)) return KSS_F_NODE_AFFINITY;
  }
  /* NodePorts.Filter -> fitsPorts: any wanted (ip, protocol, port) in conflict with
   * NodeInfo.UsedPorts (HostPortInfo.CheckConflict; the host resolves the conflict set) */
  if ((en >> KSS_F_NODE_PORTS) & 1u) {
    if (p->port_conflict & cl->port_used[n]) return KSS_F_NODE_PORTS;
  }
  /* NodeResourcesFit.Filter -> fitsRequest */
  if ((en >> KSS_F_NODE_RESOURCES_FIT) & 1u) {
    size_t N = (size_t)cl->n_nodes;
    uint16_t bits = 0;
    if ((int64_t)cl->pod_count[n] + 1 > (int64_t)cl->allowed_pods[n]) bits |= KSS_FIT_TOO_MANY_PODS;
    int all_zero = 1;
    for (int r = 0; r < 3 + cl->n_scalar; r++)
      if (p->fit_request[r] != 0) all_zero = 0;
    /* len(podRequest.ScalarResources)==0: a zero-valued scalar entry still counts as present; the host
       encodes "present with zero" as-is, so treat any scalar request slot flagged by the host as present */
    if (!all_zero) {
      for (int r = 0; r < 3 + cl->n_scalar; r++) {
        int64_t req = p->fit_request[r];
        if (r >= KSS_RES_SCALAR0 && req == 0) continue; /* Skip in case request quantity is zero */
        int64_t freev = cl->alloc[(size_t)r * N + n] - cl->requested[(size_t)r * N + n];
        if (req > freev) bits |= (uint16_t)(1u << (r + 1));
      }
    }
    if (bits) {
      *detail = bits;
      return KSS_F_NODE_RESOURCES_FIT;
    }
  }
  /* VolumeRestrictions, EBSLimits, GCEPDLimits, NodeVolumeLimits, AzureDiskLimits, VolumeBinding,
     VolumeZone: volume-less pods pass. */
  if (p->vol_len > 0) {
    int r = volume_filters(cl, ps, p, en, n, detail);
    if (r) return r;
  }
  /* PodTopologySpread.Filter */
  if (((en >> KSS_F_POD_TOPOLOGY_SPREAD) & 1u) && p->n_hard > 0) {
    const kss_spread* hard = ps->spreads + p->spread_off;
    for (int i = 0; i < p->n_hard; i++) {
      int d = LV(cl, hard[i].key, n);
      if (d < 0) {
        *detail = KSS_PTS_MISSING_LABEL;
        return KSS_F_POD_TOPOLOGY_SPREAD;
      }
      const int o = st->hard_own[i];
      int64_t match = st->hard_present[o][d] ? st->hard_cnt[o][d] : 0;
      int64_t skew = match + (int64_t)hard[i].self_match - st->hard_min[o];
      if (skew > (int64_t)hard[i].max_skew) {
        *detail = KSS_PTS_CONSTRAINTS_NOT_MATCH;
        return KSS_F_POD_TOPOLOGY_SPREAD;
      }
    }
  }
  /* InterPodAffinity.Filter */
  if ((en >> KSS_F_INTER_POD_AFFINITY) & 1u) {
    const kss_ipa* ipa = ps->ipa + p->ipa_off;
    /* satisfyPodAffinity */
    int pods_exist = 1, have_aff = 0;
    for (int e = 0; e < p->ipa_len; e++) {
      if (ipa[e].kind != KSS_IPA_REQ_AFFINITY) continue;
      have_aff = 1;
      int d = LV(cl, ipa[e].key, n);
      if (d < 0) {
        *detail = KSS_IPA_AFFINITY;
        return KSS_F_INTER_POD_AFFINITY;
      }
      int k = key_slot((podstate*)st, ipa[e].key);
      if (st->ha[k][d] <= 0) pods_exist = 0;
    }
    if (have_aff && !pods_exist) {
      if (!(!st->aff_nonempty && (p->flags & KSS_POD_IPA_SELF_MATCH))) {
        *detail = KSS_IPA_AFFINITY;
        return KSS_F_INTER_POD_AFFINITY;
      }
    }
    /* satisfyPodAntiAffinity */
    if (st->anti_nonempty) {
      for (int e = 0; e < p->ipa_len; e++) {
        if (ipa[e].kind != KSS_IPA_REQ_ANTI) continue;
        int d = LV(cl, ipa[e].key, n);
        if (d < 0) continue;
        int k = key_slot((podstate*)st, ipa[e].key);
        if (st->hb[k][d] > 0) {
          *detail = KSS_IPA_ANTI_AFFINITY;
          return KSS_F_INTER_POD_AFFINITY;
        }
      }
    }
    /* satisfyExistingPodsAntiAffinity */
    if (st->ex_nonempty) {
      for (int e = 0; e < p->ipa_len; e++) {
        if (ipa[e].kind != KSS_IPA_EXISTING_ANTI) continue;
        int d = LV(cl, ipa[e].key, n);
        if (d < 0) continue;
        int k = key_slot((podstate*)st, ipa[e].key);
        if (st->hx[k][d] > 0) {
          *detail = KSS_IPA_EXISTING_ANTI_AFFINITY;
          return KSS_F_INTER_POD_AFFINITY;
        }
      }
    }
  }
  return KSS_F_PASS;
}

static int in_ints(const int32_t* ints, int off, int len, int v) {
  for (int i = 0; i < len; i++)
    if (ints[off + i] == v) return 1;
  return 0;
}

/* ---------------------------------------------------------------------------
 * RunFilterPluginsWithNominatedPods (v1.26 runtime/framework.go) for node n: the first pass
 * runs with every nominated pod of priority >= the pod's (other than the pod itself) added to
 * the node (addNominatedPods: NodeInfo.AddPodInfo plus the AddPod PreFilter extensions --
 * podtopologyspread / interpodaffinity preFilterState.updateWithPod on the node's pairs); when
 * it passes, the second pass on the unmodified node decides (*added = 1).  The state is changed
 * in place and restored, so the caller runs it serially.  Nominees carry no volumes (the
 * device refuses them).  The PodTopologySpread minimum after the update is the minimum over
 * the present pairs: criticalPaths.update keeps exactly that when one pair changes.
 * ------------------------------------------------------------------------- */
static int filter_with_nominated(const kss_profile* prof, ostate* s, const kss_podset* ps, int pi, podstate* st,
                                 int n, uint16_t* detail, int* added) {
  const kss_cluster* cl = &s->c;
  const kss_pod* p = &ps->pods[pi];
  const size_t N = (size_t)cl->n_nodes;
  int q[64], nq = 0;
  *added = 0;
  for (int j = 0; j < s->n_nom && nq < 64; j++)
    if (s->nom_active[j] && s->nom_node[j] == n && s->nom_pod[j] != pi && ps->pods[s->nom_pod[j]].priority >= p->priority)
      q[nq++] = s->nom_pod[j];
  if (nq == 0) return filter_node(prof, cl, ps, p, st, n, detail);
  int64_t save_req[KSS_NRES];
  for (int r = 0; r < KSS_NRES; r++) save_req[r] = s->requested[(size_t)r * N + n];
  const int32_t save_pods = s->pod_count[n];
  const uint64_t save_ports = s->port_used[n];
  for (int k = 0; k < nq; k++) {
    const kss_pod* a = &ps->pods[q[k]];
    for (int r = 0; r < KSS_NRES; r++) s->requested[(size_t)r * N + n] += a->commit_req[r];
    s->pod_count[n] += 1;
    s->port_used[n] |= a->port_add;
  }
  /* podtopologyspread updateWithPod: same namespace (the selectors' class lists hold only the
     pod's namespace), the node carries every constraint key, the pod's required node affinity
     matches it; each matching constraint adds one to the node's pair of its key */
  const kss_spread* hard = ps->spreads + p->spread_off;
  int64_t save_cnt[8] = {0}, save_min[8] = {0};
  uint8_t save_pres[8] = {0};
  int pts_on = p->n_hard > 0 && has_all_keys(cl, hard, p->n_hard, n) && required_node_affinity(cl, ps, p, n);
  if (pts_on) {
    for (int i = 0; i < p->n_hard; i++) {
      if (st->hard_own[i] != i) continue;
      const int d = LV(cl, hard[i].key, n);
      save_cnt[i] = st->hard_cnt[i][d];
      save_pres[i] = st->hard_present[i][d];
      save_min[i] = st->hard_min[i];
      int64_t delta = 0;
      for (int k = 0; k < nq; k++)
        for (int j = i; j < p->n_hard; j++)
          if (st->hard_own[j] == i) delta += in_ints(ps->ints, hard[j].cls_off, hard[j].cls_len, ps->pods[q[k]].cls);
      if (delta == 0) continue;
      st->hard_cnt[i][d] += delta;
      st->hard_present[i][d] = 1;
      int64_t mn = INT32_MAX;
      const int bins = cl->key_card[hard[i].key] + 1;
      for (int b = 0; b < bins; b++)
        if (st->hard_present[i][b] && st->hard_cnt[i][b] < mn) mn = st->hard_cnt[i][b];
      st->hard_min[i] = mn;
    }
  }
  /* interpodaffinity updateWithPod on the node's pairs: the nominee's required anti-affinity
     terms matching the pod (existing anti), the pod's required affinity terms when the nominee
     matches all of them, the pod's required anti-affinity terms the nominee matches */
  const kss_ipa* ipa = ps->ipa + p->ipa_off;
  int64_t ipa_delta[64];
  const int ne = p->ipa_len < 64 ? p->ipa_len : 64;
  const int save_ex = st->ex_nonempty, save_aff = st->aff_nonempty, save_anti = st->anti_nonempty;
  for (int e = 0; e < ne; e++) {
    ipa_delta[e] = 0;
    const kss_ipa* en = &ipa[e];
    if (en->kind > KSS_IPA_REQ_ANTI) continue;
    const int d = LV(cl, en->key, n);
    if (d < 0) continue;
    for (int k = 0; k < nq; k++) {
      const kss_pod* a = &ps->pods[q[k]];
      if (en->kind == KSS_IPA_EXISTING_ANTI) {
        for (int t = 0; t < a->own_terms_len; t++)
          ipa_delta[e] += in_ints(ps->ints, en->row_off, en->row_len, ps->ints[a->own_terms_off + t]);
      } else {
        ipa_delta[e] += in_ints(ps->ints, en->row_off, en->row_len, a->cls);
      }
    }
    if (!ipa_delta[e]) continue;
    const int ks = key_slot(st, en->key);
    int64_t* h = en->kind == KSS_IPA_EXISTING_ANTI ? st->hx[ks] : (en->kind == KSS_IPA_REQ_AFFINITY ? st->ha[ks] : st->hb[ks]);
    h[d] += ipa_delta[e];
    if (en->kind == KSS_IPA_EXISTING_ANTI) st->ex_nonempty = 1;
    else if (en->kind == KSS_IPA_REQ_AFFINITY) st->aff_nonempty = 1;
    else st->anti_nonempty = 1;
  }
  int f = filter_node(prof, cl, ps, p, st, n, detail);
  /* restore */
  for (int e = 0; e < ne; e++) {
    const kss_ipa* en = &ipa[e];
    if (en->kind > KSS_IPA_REQ_ANTI || !ipa_delta[e]) continue;
    const int ks = key_slot(st, en->key);
    int64_t* h = en->kind == KSS_IPA_EXISTING_ANTI ? st->hx[ks] : (en->kind == KSS_IPA_REQ_AFFINITY ? st->ha[ks] : st->hb[ks]);
    h[LV(cl, en->key, n)] -= ipa_delta[e];
  }
  st->ex_nonempty = save_ex;
  st->aff_nonempty = save_aff;
  st->anti_nonempty = save_anti;
  if (pts_on) {
    for (int i = 0; i < p->n_hard; i++) {
      if (st->hard_own[i] != i) continue;
      const int d = LV(cl, hard[i].key, n);
      st->hard_cnt[i][d] = save_cnt[i];
      st->hard_present[i][d] = save_pres[i];
      st->hard_min[i] = save_min[i];
    }
  }
  for (int r = 0; r < KSS_NRES; r++) s->requested[(size_t)r * N + n] = save_req[r];
  s->pod_count[n] = save_pods;
  s->port_used[n] = save_ports;
  *added = 1;
  if (f != KSS_F_PASS) return f;
  /* the second pass: the unmodified node (a failure here can only be InterPodAffinity's
     required affinity, the last filter plugin: its record is the whole story) */
  return filter_node(prof, cl, ps, p, st, n, detail);
}

/* the node of pod pi's active nomination (status.nominatedNodeName), or -1 */
static int nomination_of(const ostate* s, int pi) {
  for (int j = 0; j < s->n_nom; j++)
    if (s->nom_active[j] && s->nom_pod[j] == pi) return s->nom_node[j];
  return -1;
}

/* ---------------------------------------------------------------------------
 * raw scores (Score extension point) for one feasible node
 * ------------------------------------------------------------------------- */
static int64_t least_or_most(const kss_profile* prof, int64_t requested, int64_t capacity) {
  if (prof->fit_strategy == KSS_FIT_MOST_ALLOCATED) {
    /* mostRequestedScore (noderesources/most_allocated.go) */
    if (capacity == 0) return 0;
    if (requested > capacity) requested = capacity;
    return (requested * 100) / capacity;
  }
  /* leastRequestedScore (noderesources/least_allocated.go) */
  if (capacity == 0) return 0;
  if (requested > capacity) return 0;
  return ((capacity - requested) * 100) / capacity;
}

/* NodeResourcesFit Score: resourceAllocationScorer.score with useRequested=false */
static int64_t fit_score(const kss_profile* prof, const kss_cluster* cl, const kss_pod* p, int n) {
  size_t N = (size_t)cl->n_nodes;
  int64_t node_score = 0, weight_sum = 0;
  for (int i = 0; i < prof->fit_n; i++) {
    int r = prof->fit_res[i];
    int64_t preq = p->score_req_nz[r];
    int64_t alloc, req;
    /* calculateResourceAllocatableRequest */
    if (r >= KSS_RES_SCALAR0 && preq == 0) continue;
    if (r == KSS_RES_CPU || r == KSS_RES_MEMORY) {
      alloc = cl->alloc[(size_t)r * N + n];
      req = cl->nonzero[(size_t)r * N + n] + preq;
    } else {
      alloc = cl->alloc[(size_t)r * N + n];
      req = cl->requested[(size_t)r * N + n] + preq;
    }
    if (alloc == 0) continue; /* score(): only fill entries with alloc != 0; scorer skips allocable==0 */
    node_score += least_or_most(prof, req, alloc) * prof->fit_weight[i];
    weight_sum += prof->fit_weight[i];
  }
  if (weight_sum == 0) return 0;
  return node_score / weight_sum;
}

/* NodeResourcesBalancedAllocation Score: balancedResourceScorer, useRequested=true */
static int64_t ba_score(const kss_profile* prof, const kss_cluster* cl, const kss_pod* p, int n) {
  size_t N = (size_t)cl->n_nodes;
  double fr[4];
  int nf = 0;
  double total = 0;
  for (int i = 0; i < prof->ba_n; i++) {
    int r = prof->ba_res[i];
    int64_t preq = p->score_req[r];
    if (r >= KSS_RES_SCALAR0 && preq == 0) continue;
    int64_t alloc = cl->alloc[(size_t)r * N + n];
    int64_t req = cl->requested[(size_t)r * N + n] + preq;
    if (alloc == 0) continue;
    double f = (double)req / (double)alloc;
    if (f > 1) f = 1;
    total += f;
    fr[nf++] = f;
  }
  double sd = 0.0;
  if (nf == 2) {
    sd = fabs((fr[0] - fr[1]) / 2);
  } else if (nf > 2) {
    double mean = total / (double)nf;
    double sum = 0;
    for (int i = 0; i < nf; i++) sum = sum + (fr[i] - mean) * (fr[i] - mean);
    sd = sqrt(sum / (double)nf);
  }
  return (int64_t)((1 - sd) * (double)100);
}

/* TaintToleration Score: countIntolerableTaintsPreferNoSchedule */
static int64_t tt_score(const kss_cluster* cl, const kss_pod* p, int n) {
  return (int64_t)__builtin_popcountll(cl->taint_soft[n] & ~p->tol_soft);
}

/* NodeAffinity Score: PreferredSchedulingTerms.Score */
static int64_t na_score(const kss_cluster* cl, const kss_podset* ps, const kss_pod* p, int n) {
  int64_t s = 0;
  for (int t = 0; t < p->pref_len; t++) {
    const kss_term* term = &ps->terms[p->pref_off + t];
    if (term_matches(cl, ps, term, n)) s += term->weight;
  }
  return s;
}

/* helper.DefaultNormalizeScore */
/* ImageLocality.Score (image_locality.go): calculatePriority(sumImageScores(nodeInfo,
 * pod.Spec.Containers, totalNumNodes), len(pod.Spec.Containers)); scaledImageScore per (image,
 * node) is resolved on the host (the v1.26 cache's ImageStateSummary). */
static int64_t il_score(const kss_cluster* cl, const kss_podset* ps, const kss_pod* p, int n) {
  if (p->img_len <= 0) return 0;
  int64_t sum = 0;
  for (int i = 0; i < p->img_len; i++) sum += cl->image_score[(size_t)ps->ints[p->img_off + i] * (size_t)cl->n_nodes + n];
  const int64_t max_t = KSS_IMAGE_MAX_CONTAINER_THRESHOLD * (int64_t)p->n_containers;
  if (sum < KSS_IMAGE_MIN_THRESHOLD) sum = KSS_IMAGE_MIN_THRESHOLD;
  else if (sum > max_t) sum = max_t;
  return (int64_t)100 * (sum - KSS_IMAGE_MIN_THRESHOLD) / (max_t - KSS_IMAGE_MIN_THRESHOLD);
}

static void default_normalize(int64_t* scores, const int32_t* idx, int nf, int reverse) {
  int64_t mx = 0;
  for (int i = 0; i < nf; i++)
    if (scores[idx[i]] > mx) mx = scores[idx[i]];
  if (mx == 0) {
    if (reverse)
      for (int i = 0; i < nf; i++) scores[idx[i]] = 100;
    return;
  }
  for (int i = 0; i < nf; i++) {
    int64_t s = 100 * scores[idx[i]] / mx;
    if (reverse) s = 100 - s;
    scores[idx[i]] = s;
  }
}

typedef struct {
  int threads;
} oracle_opts;

/* numFeasibleNodesToFind (v1.26 pkg/scheduler/schedule_one.go): all nodes when the list is shorter
   than minFeasibleNodesToFind (100) or percentageOfNodesToScore >= 100; pct <= 0 means the adaptive
   50 - numAllNodes/125 percent, at least minFeasibleNodesPercentageToFind (5); at least 100 nodes. */
static int num_feasible_to_find(int m, int pct) {
  if (m < 100 || pct >= 100) return m;
  int a = pct;
  if (a <= 0) {
    a = 50 - m / 125;
    if (a < 5) a = 5;
  }
  long long k = (long long)m * a / 100;
  return k < 100 ? 100 : (int)k;
}

/* one scheduling cycle (schedulePod) for pod p against state s; fills out (arrays sized N) */
static int schedule_one(const kss_profile* prof, ostate* s, const kss_podset* ps, int pi, kss_pod_result* out,
                        int threads) {
  const kss_cluster* cl = &s->c;
  const kss_pod* p = &ps->pods[pi];
  int N = cl->n_nodes;
  uint8_t* fp = (uint8_t*)malloc((size_t)(N ? N : 1));
  uint16_t* fd = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)(N ? N : 1));
  int64_t* raw = (int64_t*)calloc((size_t)KSS_NSCORE * (size_t)(N ? N : 1), sizeof(int64_t));
  int64_t* norm = (int64_t*)calloc((size_t)KSS_NSCORE * (size_t)(N ? N : 1), sizeof(int64_t));
  int64_t* total = (int64_t*)calloc((size_t)(N ? N : 1), sizeof(int64_t));
  int32_t* feas = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N ? N : 1));
  int rc = 0;
  podstate st;
  memset(&st, 0, sizeof(st));
  out->chosen = -1;
  out->n_feasible = 0;
  out->best_total = 0;
  out->scored = 0;
  out->status = 0;
  for (int n = 0; n < N; n++) {
    fp[n] = KSS_F_NOT_EVALUATED;
    fd[n] = 0;
  }

  if (p->prefilter_status != 0) {
    out->status = p->prefilter_status == KSS_PF_ERROR ? 3 : 2;
    goto done;
  }
  rc = podstate_build(&st, cl, ps, p, prof->hard_pod_affinity_weight);
  if (rc) goto done;

  /* PreferNominatedNode (findNodesThatFitPod -> evaluateNominatedNode): a nominated pod first
     runs findNodesThatPassFilters on [its node] alone (whatever the PreFilterResult); the
     one-node list resets nextStartNodeIndex to 0.  A feasible node is chosen without scoring;
     otherwise its status stays in the diagnosis and its record stands. */
  int nom_m = nomination_of(s, pi), nom_f = 0;
  uint16_t nom_d = 0;
  if (nom_m >= 0) {
    int added;
    nom_f = filter_with_nominated(prof, s, ps, pi, &st, nom_m, &nom_d, &added);
    s->cursor = 0;
    if (nom_f == KSS_F_PASS) {
      fp[nom_m] = KSS_F_PASS;
      out->n_feasible = 1;
      out->chosen = cl->node_base + nom_m;
      goto done;
    }
  }

  /* HOT LOOP 1: findNodesThatPassFilters over the (PreFilterResult-restricted) node list */
  {
    uint8_t* inset = NULL;
    if (p->names_len >= 0) {
      inset = (uint8_t*)calloc((size_t)(N ? N : 1), 1);
      for (int i = 0; i < p->names_len; i++) {
        int64_t g = ps->ints[p->names_off + i] - cl->node_base;
        if (g >= 0 && g < N) inset[g] = 1;
      }
    }
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int n = 0; n < N; n++) {
      if (inset && !inset[n]) continue;
      fp[n] = (uint8_t)filter_node(prof, cl, ps, p, &st, n, &fd[n]);
    }
    /* nodes holding nominated pods: RunFilterPluginsWithNominatedPods' first pass (serial: it
       changes the state in place) -- a failure there is the node's status */
    for (int j = 0; j < s->n_nom; j++) {
      const int n = s->nom_node[j];
      if (!s->nom_active[j] || n < 0 || n >= N || (inset && !inset[n])) continue;
      int dup = 0;
      for (int k = 0; k < j; k++) dup |= s->nom_active[k] && s->nom_node[k] == n;
      if (dup) continue;
      uint16_t d;
      int added;
      const int f = filter_with_nominated(prof, s, ps, pi, &st, n, &d, &added);
      fp[n] = (uint8_t)f;
      fd[n] = d;
    }
    /* findNodesThatPassFilters with Parallelism = 1: the node list (all nodes, or the
       PreFilterResult set in canonical order) is visited from nextStartNodeIndex until one
       feasible node more than numFeasibleNodesToFind has been found.  That node passed every
       filter (recorded) but is not in the feasible list; nodes after it were never filtered.
       nextStartNodeIndex advances by the nodes processed: the feasible ones kept plus the
       infeasible ones visited (schedule_one.go: processedNodes = feasibleNodesLen +
       len(diagnosis.NodeToStatusMap)). */
    int m = 0;
    int32_t* list = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N ? N : 1));
    for (int n = 0; n < N; n++)
      if (!inset || inset[n]) list[m++] = n;
    if (m > 0) {
      const int K = num_feasible_to_find(m, prof->pct_nodes_to_score);
      const int start = (int)((int64_t)s->cursor % m);
      int found = 0, processed = m, i = 0;
      for (; i < m; i++) {
        const int n = list[(start + i) % m];
        if (fp[n] != KSS_F_PASS) continue;
        if (++found > K) { /* the context is cancelled after this node: it is dropped */
          fd[n] = KSS_PASS_NOT_KEPT;
          processed = i;
          break;
        }
      }
      for (int j = i + 1; j < m; j++) { /* never visited */
        const int n = list[(start + j) % m];
        fp[n] = KSS_F_NOT_EVALUATED;
        fd[n] = 0;
      }
      /* the diagnosis map already holds evaluateNominatedNode's failure: one node more unless
         the search visited that node again (outside the list, or after the stopping node) */
      if (nom_m >= 0 && ((inset && !inset[nom_m]) || fp[nom_m] == KSS_F_NOT_EVALUATED)) processed++;
      s->cursor = (int32_t)(((int64_t)s->cursor + processed) % m);
    }
    free(list);
    free(inset);
    if (nom_m >= 0) { /* the nominated node's status from evaluateNominatedNode (the same if revisited) */
      fp[nom_m] = (uint8_t)nom_f;
      fd[nom_m] = nom_d;
    }
  }
  int nf = 0;
  for (int n = 0; n < N; n++)
    if (fp[n] == KSS_F_PASS && fd[n] != KSS_PASS_NOT_KEPT) feas[nf++] = n;
  out->n_feasible = nf;
  if (nf == 0) {
    out->status = 1;
    goto done;
  }
  if (nf == 1) { /* "When only one node after predicate, just use it." */
    out->chosen = cl->node_base + feas[0];
    goto done;
  }
  out->scored = 1;

  /* PreScore PodTopologySpread: initPreScoreState + processAllNode */
  const kss_spread* soft = ps->spreads + p->spread_off + p->n_hard;
  int require_all = (p->flags & KSS_POD_PTS_REQUIRE_ALL) != 0;
  double w[8];
  int64_t* soft_cnt[8] = {0};
  uint8_t* soft_present[8] = {0};
  uint8_t* ignored = (uint8_t*)calloc((size_t)(N ? N : 1), 1);
  int nignored = 0;
  for (int i = 0; i < nf; i++) {
    int n = feas[i];
    if (require_all && !has_all_keys(cl, soft, p->n_soft, n)) {
      ignored[n] = 1;
      nignored++;
    }
  }
  /* TopologyPairToPodCounts is keyed by pair: constraints on one (non-hostname) key share the
     counters of the key's first constraint sown[c], which also owns every pair in topoSize
     (the later ones find the pair created and count 0 domains) */
  int sown[8];
  for (int c = 0; c < p->n_soft; c++) {
    int key = soft[c].key;
    sown[c] = c;
    if (!(cl->key_flags[key] & KSS_KEY_HOSTNAME))
      for (int j = 0; j < c; j++)
        if (soft[j].key == key) {
          sown[c] = j;
          break;
        }
    int size = 0;
    if (cl->key_flags[key] & KSS_KEY_HOSTNAME) {
      size = nf - nignored;
    } else if (sown[c] == c) {
      int bins = cl->key_card[key] + 1;
      soft_cnt[c] = (int64_t*)calloc((size_t)bins, sizeof(int64_t));
      soft_present[c] = (uint8_t*)calloc((size_t)bins, 1);
      for (int i = 0; i < nf; i++) {
        int n = feas[i];
        if (ignored[n]) continue;
        int d = LV(cl, key, n);
        if (d < 0) d = cl->key_empty[key]; /* node.Labels[key] == "" for a missing key */
        if (!soft_present[c][d]) {
          soft_present[c][d] = 1;
          size++;
        }
      }
    }
    w[c] = go_log((double)(size + 2)); /* topologyNormalizingWeight */
  }
  if (p->n_soft > 0) {
    for (int n = 0; n < N; n++) {
      if (require_all && !has_all_keys(cl, soft, p->n_soft, n)) continue;
      for (int c = 0; c < p->n_soft; c++) {
        int key = soft[c].key;
        if (cl->key_flags[key] & KSS_KEY_HOSTNAME) continue; /* per-node counts computed in Score */
        if (!spread_policy_ok(cl, ps, p, &soft[c], n)) continue;
        int d = LV(cl, key, n);
        if (d < 0) d = cl->key_empty[key];
        int o = sown[c];
        if (!soft_present[o][d]) continue; /* pair not associated with any candidate node */
        soft_cnt[o][d] += sum_rows(cl->class_count, (size_t)N, ps->ints + soft[c].cls_off, soft[c].cls_len, n);
      }
    }
  }

  /* HOT LOOP 2: RunScorePlugins raw scores */
#pragma omp parallel for num_threads(threads) schedule(static)
  for (int i = 0; i < nf; i++) {
    int n = feas[i];
    size_t NN = (size_t)N;
    raw[KSS_S_TAINT_TOLERATION * NN + n] = tt_score(cl, p, n);
    raw[KSS_S_NODE_AFFINITY * NN + n] = na_score(cl, ps, p, n);
    raw[KSS_S_NODE_RESOURCES_FIT * NN + n] = fit_score(prof, cl, p, n);
    raw[KSS_S_VOLUME_BINDING * NN + n] = 0;
    raw[KSS_S_BALANCED_ALLOCATION * NN + n] = ba_score(prof, cl, p, n);
    raw[KSS_S_IMAGE_LOCALITY * NN + n] = il_score(cl, ps, p, n);
    /* PodTopologySpread.Score */
    int64_t pts = 0;
    if (!ignored[n]) {
      double sc = 0;
      for (int c = 0; c < p->n_soft; c++) {
        int key = soft[c].key;
        int d = LV(cl, key, n);
        if (d < 0) continue;
        int64_t cnt;
        if (cl->key_flags[key] & KSS_KEY_HOSTNAME)
          cnt = sum_rows(cl->class_count, NN, ps->ints + soft[c].cls_off, soft[c].cls_len, n);
        else
          cnt = soft_cnt[sown[c]][d];
        sc += (double)cnt * w[c] + (double)(soft[c].max_skew - 1); /* scoreForCount */
      }
      pts = go_round_to_i64(sc);
    }
    raw[KSS_S_POD_TOPOLOGY_SPREAD * NN + n] = pts;
    /* InterPodAffinity.Score: Σ over topology keys present on the node */
    int64_t ipa = 0;
    for (int k = 0; k < st.nkeys; k++) {
      int d = LV(cl, st.keys[k], n);
      if (d >= 0) ipa += st.hs[k][d];
    }
    raw[KSS_S_INTER_POD_AFFINITY * NN + n] = ipa;
  }
  memcpy(norm, raw, sizeof(int64_t) * KSS_NSCORE * (size_t)N);

  /* HOT LOOP 3: NormalizeScore per plugin over the feasible list */
  default_normalize(norm + (size_t)KSS_S_TAINT_TOLERATION * N, feas, nf, 1);
  default_normalize(norm + (size_t)KSS_S_NODE_AFFINITY * N, feas, nf, 0);
  { /* PodTopologySpread.NormalizeScore */
    int64_t* sc = norm + (size_t)KSS_S_POD_TOPOLOGY_SPREAD * N;
    int64_t mn = INT64_MAX, mx = 0;
    for (int i = 0; i < nf; i++) {
      int n = feas[i];
      if (ignored[n]) continue;
      if (sc[n] < mn) mn = sc[n];
      if (sc[n] > mx) mx = sc[n];
    }
    for (int i = 0; i < nf; i++) {
      int n = feas[i];
      if (ignored[n]) {
        sc[n] = 0;
        continue;
      }
      if (mx == 0) {
        sc[n] = 100;
        continue;
      }
      sc[n] = 100 * (mx + mn - sc[n]) / mx;
    }
  }
  if (st.score_nonempty) { /* InterPodAffinity.NormalizeScore (skipped when topologyScore is empty) */
    int64_t* sc = norm + (size_t)KSS_S_INTER_POD_AFFINITY * N;
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    for (int i = 0; i < nf; i++) {
      int n = feas[i];
      if (sc[n] > mx) mx = sc[n];
      if (sc[n] < mn) mn = sc[n];
    }
    int64_t diff = mx - mn;
    for (int i = 0; i < nf; i++) {
      int n = feas[i];
      double f = 0;
      if (diff > 0) f = (double)100 * ((double)(sc[n] - mn) / (double)diff);
      sc[n] = (int64_t)f;
    }
  }

  /* HOT LOOP 4: weights + TotalScore, then selectHost (deterministic tie-break) */
  {
    int64_t best = INT64_MIN;
    int bi = -1;
    for (int i = 0; i < nf; i++) {
      int n = feas[i];
      int64_t t = 0;
      for (int sp = 0; sp < KSS_NSCORE; sp++) {
        if (!((prof->score_enabled >> sp) & 1u)) continue;
        int64_t v = norm[(size_t)sp * N + n];
        if (v > 100 || v < 0) {
          out->status = 3; /* "plugin returns an invalid score" -> framework Error */
        }
        t += v * (int64_t)prof->weight[sp];
      }
      total[n] = t;
      if (t > best) {
        best = t;
        bi = n;
      }
    }
    if (out->status == 3) {
      bi = -1;
    }
    out->best_total = best;
    out->chosen = bi >= 0 ? cl->node_base + bi : -1;
  }
  for (int c = 0; c < p->n_soft; c++) {
    free(soft_cnt[c]);
    free(soft_present[c]);
  }
  free(ignored);

done:
  podstate_free(&st);
  if (out->fail_plugin) memcpy(out->fail_plugin, fp, (size_t)N);
  if (out->fail_detail) memcpy(out->fail_detail, fd, sizeof(uint16_t) * (size_t)N);
  if (out->raw) memcpy(out->raw, raw, sizeof(int64_t) * KSS_NSCORE * (size_t)N);
  if (out->norm) memcpy(out->norm, norm, sizeof(int64_t) * KSS_NSCORE * (size_t)N);
  if (out->total) memcpy(out->total, total, sizeof(int64_t) * (size_t)N);
  free(fp);
  free(fd);
  free(raw);
  free(norm);
  free(total);
  free(feas);
  return rc;
}

/* Cache.AssumePod -> NodeInfo.AddPod (framework/types.go calculateResource) */
static void commit(ostate* s, const kss_podset* ps, int pi, int node_local) {
  const kss_pod* p = &ps->pods[pi];
  size_t N = (size_t)s->c.n_nodes;
  for (int j = 0; j < s->n_nom; j++) /* SchedulingQueue.DeleteNominatedPodIfExists(assumed pod) */
    if (s->nom_pod[j] == pi) s->nom_active[j] = 0;
  for (int r = 0; r < KSS_NRES; r++) s->requested[(size_t)r * N + node_local] += p->commit_req[r];
  s->nonzero[node_local] += p->commit_nz[0];
  s->nonzero[N + node_local] += p->commit_nz[1];
  s->pod_count[node_local] += 1;
  if (p->cls >= 0) s->class_count[(size_t)p->cls * N + node_local] += 1;
  for (int i = 0; i < p->own_terms_len; i++) s->term_count[(size_t)ps->ints[p->own_terms_off + i] * N + node_local] += 1;
  s->port_used[node_local] |= p->port_add; /* NodeInfo.AddPod updateUsedPorts */
  /* the pod's volumes join NodeInfo.Pods: a row counts the pod; its key counts the volume once */
  for (int e = 0; e < p->vol_len; e++) {
    const kss_vol* v = &ps->vols[p->vol_off + e];
    if (v->kind == KSS_VOL_OWN) {
      int key = s->c.vol_row_key[v->row];
      int32_t* cnt = &s->vol_count[(size_t)v->row * N + node_local];
      if (key >= 0 && *cnt == 0) s->vol_attached[(size_t)key * N + node_local] += 1;
      *cnt += 1;
    } else if (v->kind == KSS_VOL_OWN_PRIVATE) {
      s->vol_attached[(size_t)v->key * N + node_local] += v->count;
    }
  }
  /* Reserve's AssumePodVolumes: the delayed claims' static bindings and provisioning on this node */
  int e0 = -1, e1 = -1;
  for (int e = 0; e < p->vol_len; e++)
    if (is_vb(ps->vols[p->vol_off + e].kind)) {
      if (e0 < 0) e0 = p->vol_off + e;
      e1 = p->vol_off + e + 1;
    }
  if (e0 >= 0) {
    int pick[KSS_MAX_WFFC] = {-1, -1, -1, -1}, wi = 0;
    find_pod_volumes(&s->c, ps, e0, e1, node_local, pick);
    for (int e = e0; e < e1; e++) {
      const kss_vol* v = &ps->vols[e];
      if (v->kind != KSS_VOL_BIND_WFFC) continue;
      if (pick[wi] >= 0) s->pv_owner[pick[wi]] = v->key + 1;
      else s->claim_node[v->key] = node_local;
      wi++;
    }
  }
}

/* ---------------------------------------------------------------------------
 * exported entry points (ctypes)
 * ------------------------------------------------------------------------- */

/* Evaluate pod pi against cl without committing. */
int kss_oracle_eval_pod(const kss_profile* prof, const kss_cluster* cl, const kss_podset* ps, int pi,
                        kss_pod_result* out, int threads) {
  ostate s;
  if (ostate_init(&s, cl)) return KSS_E_NOMEM;
  int rc = schedule_one(prof, &s, ps, pi, out, threads > 0 ? threads : 1);
  ostate_free(&s);
  return rc;
}

/* kss_oracle_schedule_v with the scheduler's nextStartNodeIndex in and out (NULL: starts at 0). */
int kss_oracle_schedule_c(const kss_profile* prof, const kss_cluster* cl, const kss_podset* ps, int n,
                          int32_t* chosen, kss_pod_result* results, int threads, int64_t* out_requested,
                          int64_t* out_nonzero, int32_t* out_pod_count, int32_t* out_class_count,
                          int32_t* out_term_count, uint64_t* out_port_used, int32_t* out_vol_count,
                          int32_t* out_vol_attached, int32_t* cursor);

/* Sequentially schedule pods [0, n): each pod sees the previous commits.
 * results (optional) is an array of n kss_pod_result whose arrays the caller
 * allocated (any NULL array is skipped).  Final node state is written back to
 * the optional out_* arrays. */
int kss_oracle_schedule_v(const kss_profile* prof, const kss_cluster* cl, const kss_podset* ps, int n,
                          int32_t* chosen, kss_pod_result* results, int threads, int64_t* out_requested,
                          int64_t* out_nonzero, int32_t* out_pod_count, int32_t* out_class_count,
                          int32_t* out_term_count, uint64_t* out_port_used, int32_t* out_vol_count,
                          int32_t* out_vol_attached) {
  return kss_oracle_schedule_c(prof, cl, ps, n, chosen, results, threads, out_requested, out_nonzero, out_pod_count,
                               out_class_count, out_term_count, out_port_used, out_vol_count, out_vol_attached, NULL);
}

/* kss_oracle_schedule_c with the scheduling queue's nominator: pods ps.pods[nom_pod[j]] nominated
   to global node nom_node[j] (PodNominator.AddNominatedPod order); a pod of the batch that is
   assumed leaves it.  *nom_left (optional) receives the nominations still active per entry. */
int kss_oracle_schedule_n(const kss_profile* prof, const kss_cluster* cl, const kss_podset* ps, int n,
                          int32_t* chosen, kss_pod_result* results, int threads, int64_t* out_requested,
                          int64_t* out_nonzero, int32_t* out_pod_count, int32_t* out_class_count,
                          int32_t* out_term_count, uint64_t* out_port_used, int32_t* out_vol_count,
                          int32_t* out_vol_attached, int32_t* cursor, const int32_t* nom_pod,
                          const int32_t* nom_node, int32_t n_nom, uint8_t* nom_left);

int kss_oracle_schedule_c(const kss_profile* prof, const kss_cluster* cl, const kss_podset* ps, int n,
                          int32_t* chosen, kss_pod_result* results, int threads, int64_t* out_requested,
                          int64_t* out_nonzero, int32_t* out_pod_count, int32_t* out_class_count,
                          int32_t* out_term_count, uint64_t* out_port_used, int32_t* out_vol_count,
                          int32_t* out_vol_attached, int32_t* cursor) {
  return kss_oracle_schedule_n(prof, cl, ps, n, chosen, results, threads, out_requested, out_nonzero, out_pod_count,
                               out_class_count, out_term_count, out_port_used, out_vol_count, out_vol_attached, cursor,
                               NULL, NULL, 0, NULL);
}

/* kss_oracle_schedule_n with the binder's assume cache after the batch (out_pv_owner [n_pvs],
   out_claim_node [n_wclaims]; NULL: not wanted). */
int kss_oracle_schedule_w(const kss_profile* prof, const kss_cluster* cl, const kss_podset* ps, int n,
                          int32_t* chosen, kss_pod_result* results, int threads, int64_t* out_requested,
                          int64_t* out_nonzero, int32_t* out_pod_count, int32_t* out_class_count,
                          int32_t* out_term_count, uint64_t* out_port_used, int32_t* out_vol_count,
                          int32_t* out_vol_attached, int32_t* cursor, const int32_t* nom_pod,
                          const int32_t* nom_node, int32_t n_nom, uint8_t* nom_left, int32_t* out_pv_owner,
                          int32_t* out_claim_node);

int kss_oracle_schedule_n(const kss_profile* prof, const kss_cluster* cl, const kss_podset* ps, int n,
                          int32_t* chosen, kss_pod_result* results, int threads, int64_t* out_requested,
                          int64_t* out_nonzero, int32_t* out_pod_count, int32_t* out_class_count,
                          int32_t* out_term_count, uint64_t* out_port_used, int32_t* out_vol_count,
                          int32_t* out_vol_attached, int32_t* cursor, const int32_t* nom_pod,
                          const int32_t* nom_node, int32_t n_nom, uint8_t* nom_left) {
  return kss_oracle_schedule_w(prof, cl, ps, n, chosen, results, threads, out_requested, out_nonzero, out_pod_count,
                               out_class_count, out_term_count, out_port_used, out_vol_count, out_vol_attached, cursor,
                               nom_pod, nom_node, n_nom, nom_left, NULL, NULL);
}

/* kss_oracle_schedule_w where pods with skip_commit[i] != 0 are evaluated but not assumed: the
   per-pod API's commit followed by a rollback of the same pod (Reserve then Unreserve leave the
   node state as it was; tests/test_gpu_service.py replays a service sequence with it). */
int kss_oracle_schedule_wm(const kss_profile* prof, const kss_cluster* cl, const kss_podset* ps, int n,
                           int32_t* chosen, kss_pod_result* results, int threads, int64_t* out_requested,
                           int64_t* out_nonzero, int32_t* out_pod_count, int32_t* out_class_count,
                           int32_t* out_term_count, uint64_t* out_port_used, int32_t* out_vol_count,
                           int32_t* out_vol_attached, int32_t* cursor, const int32_t* nom_pod,
                           const int32_t* nom_node, int32_t n_nom, uint8_t* nom_left, int32_t* out_pv_owner,
                           int32_t* out_claim_node, const uint8_t* skip_commit);

int kss_oracle_schedule_w(const kss_profile* prof, const kss_cluster* cl, const kss_podset* ps, int n,
                          int32_t* chosen, kss_pod_result* results, int threads, int64_t* out_requested,
                          int64_t* out_nonzero, int32_t* out_pod_count, int32_t* out_class_count,
                          int32_t* out_term_count, uint64_t* out_port_used, int32_t* out_vol_count,
                          int32_t* out_vol_attached, int32_t* cursor, const int32_t* nom_pod,
                          const int32_t* nom_node, int32_t n_nom, uint8_t* nom_left, int32_t* out_pv_owner,
                          int32_t* out_claim_node) {
  return kss_oracle_schedule_wm(prof, cl, ps, n, chosen, results, threads, out_requested, out_nonzero, out_pod_count,
                                out_class_count, out_term_count, out_port_used, out_vol_count, out_vol_attached,
                                cursor, nom_pod, nom_node, n_nom, nom_left, out_pv_owner, out_claim_node, NULL);
}

int kss_oracle_schedule_wm(const kss_profile* prof, const kss_cluster* cl, const kss_podset* ps, int n,
                           int32_t* chosen, kss_pod_result* results, int threads, int64_t* out_requested,
                           int64_t* out_nonzero, int32_t* out_pod_count, int32_t* out_class_count,
                           int32_t* out_term_count, uint64_t* out_port_used, int32_t* out_vol_count,
                           int32_t* out_vol_attached, int32_t* cursor, const int32_t* nom_pod,
                           const int32_t* nom_node, int32_t n_nom, uint8_t* nom_left, int32_t* out_pv_owner,
                           int32_t* out_claim_node, const uint8_t* skip_commit) {
  ostate s;
  if (ostate_init(&s, cl)) return KSS_E_NOMEM;
  if (cursor) s.cursor = *cursor;
  int32_t* nn_local = NULL;
  if (n_nom > 0) {
    s.n_nom = n_nom;
    s.nom_pod = nom_pod;
    nn_local = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_nom);
    s.nom_active = (uint8_t*)malloc((size_t)n_nom);
    for (int j = 0; j < n_nom; j++) {
      nn_local[j] = nom_node[j] - cl->node_base;
      s.nom_active[j] = nom_pod[j] >= 0 && nom_pod[j] < ps->n_pods && nn_local[j] >= 0 && nn_local[j] < cl->n_nodes;
    }
    s.nom_node = nn_local;
  }
  int th = threads > 0 ? threads : 1;
  int rc = 0;
  for (int i = 0; i < n; i++) {
    kss_pod_result tmp;
    memset(&tmp, 0, sizeof(tmp));
    kss_pod_result* out = results ? &results[i] : &tmp;
    rc = schedule_one(prof, &s, ps, i, out, th);
    if (rc) break;
    chosen[i] = out->chosen;
    if (out->chosen >= 0 && !(skip_commit && skip_commit[i])) commit(&s, ps, i, out->chosen - cl->node_base);
  }
  size_t N = (size_t)cl->n_nodes;
  if (out_requested) memcpy(out_requested, s.requested, sizeof(int64_t) * KSS_NRES * N);
  if (out_nonzero) memcpy(out_nonzero, s.nonzero, sizeof(int64_t) * 2 * N);
  if (out_pod_count) memcpy(out_pod_count, s.pod_count, sizeof(int32_t) * N);
  if (out_class_count && cl->n_classes)
    memcpy(out_class_count, s.class_count, sizeof(int32_t) * (size_t)cl->n_classes * N);
  if (out_term_count && cl->n_terms) memcpy(out_term_count, s.term_count, sizeof(int32_t) * (size_t)cl->n_terms * N);
  if (out_port_used) memcpy(out_port_used, s.port_used, sizeof(uint64_t) * N);
  if (out_vol_count && cl->n_vol_rows) memcpy(out_vol_count, s.vol_count, sizeof(int32_t) * (size_t)cl->n_vol_rows * N);
  if (out_vol_attached && cl->n_vol_keys)
    memcpy(out_vol_attached, s.vol_attached, sizeof(int32_t) * (size_t)cl->n_vol_keys * N);
  if (cursor) *cursor = s.cursor;
  if (out_pv_owner && cl->n_pvs) memcpy(out_pv_owner, s.pv_owner, sizeof(int32_t) * (size_t)cl->n_pvs);
  if (out_claim_node && cl->n_wclaims) memcpy(out_claim_node, s.claim_node, sizeof(int32_t) * (size_t)cl->n_wclaims);
  if (nom_left)
    for (int j = 0; j < n_nom; j++) nom_left[j] = s.nom_active[j];
  free(nn_local);
  ostate_free(&s);
  return rc;
}

int kss_oracle_schedule(const kss_profile* prof, const kss_cluster* cl, const kss_podset* ps, int n,
                        int32_t* chosen, kss_pod_result* results, int threads, int64_t* out_requested,
                        int64_t* out_nonzero, int32_t* out_pod_count, int32_t* out_class_count,
                        int32_t* out_term_count, uint64_t* out_port_used) {
  return kss_oracle_schedule_v(prof, cl, ps, n, chosen, results, threads, out_requested, out_nonzero, out_pod_count,
                               out_class_count, out_term_count, out_port_used, NULL, NULL);
}

int kss_oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* ===========================================================================
 * DefaultPreemption PostFilter dry run (ORACLE / CPU BASELINE) — Evaluator.Preempt of
 * ⟨k8s⟩ pkg/scheduler/framework/preemption/preemption.go with the DefaultPreemption plugin
 * (plugins/defaultpreemption/default_preemption.go), as the simulator wraps it in
 * wrappedPlugin.PostFilter (/root/reference/simulator/scheduler/plugin/wrappedplugin.go:550-577).
 * The same restatement as oracle/k8s_preemption.py, over the struct-of-arrays snapshot and the
 * bound-pod table (include/kss.h kss_boundset), with the same deterministic choices (DESIGN
 * §3.4): every potential node is dry-run, unset start times sort last, sort ties keep NodeInfo
 * order (the boundset's order of a node's pods), full ties go to the lowest node index.
 * SelectVictimsOnNode runs node-parallel (OpenMP), the way DryRunPreemption fans out with
 * parallelize.Until.
 * ========================================================================= */

/* The node-local view SelectVictimsOnNode mutates: NodeInfo.Requested / len(Pods), the hard
 * spread pair count of the node's pair per hard owner, the inter-pod-affinity counts of the
 * node's pairs per (key slot, existing anti | affinity | anti), and the affinity-count total
 * (len(affinityCounts) == 0 <=> total 0: counts never go negative). */
typedef struct {
  int64_t req[KSS_NRES];
  int64_t pods;
  int64_t M[8];
  int64_t A[MAXKEYS_PER_POD][3];
  int64_t T;
} drystate;

typedef struct {
  const kss_profile* prof;
  const kss_cluster* cl;
  const kss_podset* ps;
  const kss_pod* p;
  const podstate* st;
  const kss_boundset* bs;
  const int32_t* ptr;  /* [N + 1] CSR of bound pods by local node */
  const int32_t* ord;  /* per node, its pods in MoreImportantPod order (boundset indices) */
  int64_t m0[8], m1[8];
  int32_t id0[8];
  int64_t aff_total;
  int n_nom; /* the nominator: ps pod indices and local nodes (RunFilterPluginsWithNominatedPods) */
  const int32_t* nom_pod;
  const int32_t* nom_node;
  int pi;    /* the preemptor (never its own nominee) */
} dryctx;

static int in_list32(const int32_t* ints, int off, int len, int v) {
  for (int i = 0; i < len; i++)
    if (ints[off + i] == v) return 1;
  return 0;
}

/* NodeInfo.RemovePod (sign -1) / AddPod (+1) of bound pod e on node n with the RemovePod /
 * AddPod extensions: ⟨k8s⟩ podtopologyspread preFilterState.updateWithPod (each matching
 * constraint moves the node's pair counter), interpodaffinity preFilterState.updateWithPod
 * (topologyToMatchedTermCount.update of the node's pairs). */
static void dry_apply(const dryctx* D, int e, int n, int sign, drystate* s) {
  const kss_cluster* cl = D->cl;
  const kss_podset* ps = D->ps;
  const kss_pod* p = D->p;
  const kss_boundset* bs = D->bs;
  for (int r = 0; r < 3 + cl->n_scalar; r++) s->req[r] += sign * bs->req[(size_t)r * bs->n + e];
  s->pods += sign;
  const int cls = bs->cls[e];
  const kss_spread* hard = ps->spreads + p->spread_off;
  for (int j = 0; j < p->n_hard; j++)
    if (in_list32(ps->ints, hard[j].cls_off, hard[j].cls_len, cls)) s->M[D->st->hard_own[j]] += sign;
  const kss_ipa* ipa = ps->ipa + p->ipa_off;
  for (int q = 0; q < p->ipa_len; q++) {
    const kss_ipa* en = &ipa[q];
    if (en->kind > KSS_IPA_REQ_ANTI) continue;
    if (LV(cl, en->key, n) < 0) continue; /* the node lacks the key: no pair to update */
    const int k = key_slot((podstate*)D->st, en->key);
    if (en->kind == KSS_IPA_EXISTING_ANTI) {
      for (int t = 0; t < bs->terms_len[e]; t++)
        if (in_list32(ps->ints, en->row_off, en->row_len, bs->ints[bs->terms_off[e] + t])) s->A[k][0] += sign;
    } else if (in_list32(ps->ints, en->row_off, en->row_len, cls)) {
      s->A[k][en->kind == KSS_IPA_REQ_AFFINITY ? 1 : 2] += sign;
      if (en->kind == KSS_IPA_REQ_AFFINITY) s->T += sign;
    }
  }
}

/* RunFilterPluginsWithNominatedPods on the modified node: NodeResourcesFit, PodTopologySpread,
 * InterPodAffinity (the filters before them passed: the node is a potential node). */
static int dry_fits(const dryctx* D, const drystate* s, int n) {
  const kss_cluster* cl = D->cl;
  const kss_podset* ps = D->ps;
  const kss_pod* p = D->p;
  const uint32_t en = D->prof->filter_enabled;
  const size_t N = (size_t)cl->n_nodes;
  if ((en >> KSS_F_NODE_RESOURCES_FIT) & 1u) {
    if (s->pods + 1 > (int64_t)cl->allowed_pods[n]) return 0;
    int all_zero = 1;
    for (int r = 0; r < 3 + cl->n_scalar; r++) all_zero &= p->fit_request[r] == 0;
    if (!all_zero)
      for (int r = 0; r < 3 + cl->n_scalar; r++) {
        const int64_t q = p->fit_request[r];
        if (r >= KSS_RES_SCALAR0 && q == 0) continue;
        if (q > cl->alloc[(size_t)r * N + n] - s->req[r]) return 0;
      }
  }
  if (((en >> KSS_F_POD_TOPOLOGY_SPREAD) & 1u) && p->n_hard > 0) {
    const kss_spread* hard = ps->spreads + p->spread_off;
    for (int i = 0; i < p->n_hard; i++) {
      const int d = LV(cl, hard[i].key, n);
      if (d < 0) return 0;
      const int o = D->st->hard_own[i];
      /* criticalPaths after the node's pair changed: min(min over the other pairs, this pair) */
      const int64_t others = D->id0[o] == d ? D->m1[o] : D->m0[o];
      const int64_t mn = s->M[o] < others ? s->M[o] : others;
      if (s->M[o] + (int64_t)hard[i].self_match - mn > (int64_t)hard[i].max_skew) return 0;
    }
  }
  if (((en >> KSS_F_INTER_POD_AFFINITY) & 1u) && p->ipa_len > 0) {
    const kss_ipa* ipa = ps->ipa + p->ipa_off;
    int have = 0, exist = 1;
    for (int q = 0; q < p->ipa_len; q++) {
      if (ipa[q].kind != KSS_IPA_REQ_AFFINITY) continue;
      have = 1;
      if (LV(cl, ipa[q].key, n) < 0) return 0;
      if (s->A[key_slot((podstate*)D->st, ipa[q].key)][1] <= 0) exist = 0;
    }
    if (have && !exist && !(s->T == 0 && (p->flags & KSS_POD_IPA_SELF_MATCH))) return 0;
    for (int q = 0; q < p->ipa_len; q++) {
      const int kind = ipa[q].kind;
      if (kind != KSS_IPA_REQ_ANTI && kind != KSS_IPA_EXISTING_ANTI) continue;
      if (LV(cl, ipa[q].key, n) < 0) continue;
      if (s->A[key_slot((podstate*)D->st, ipa[q].key)][kind == KSS_IPA_REQ_ANTI ? 2 : 0] > 0) return 0;
    }
  }
  return 1;
}

/* AddPod of nominee ps->pods[q] on node n (addNominatedPods): the same updates as dry_apply */
static void dry_apply_nominee(const dryctx* D, int q, int n, drystate* s) {
  const kss_cluster* cl = D->cl;
  const kss_podset* ps = D->ps;
  const kss_pod* p = D->p;
  const kss_pod* a = &ps->pods[q];
  for (int r = 0; r < 3 + cl->n_scalar; r++) s->req[r] += a->commit_req[r];
  s->pods += 1;
  const kss_spread* hard = ps->spreads + p->spread_off;
  for (int j = 0; j < p->n_hard; j++)
    if (in_list32(ps->ints, hard[j].cls_off, hard[j].cls_len, a->cls)) s->M[D->st->hard_own[j]] += 1;
  const kss_ipa* ipa = ps->ipa + p->ipa_off;
  for (int e = 0; e < p->ipa_len; e++) {
    const kss_ipa* en = &ipa[e];
    if (en->kind > KSS_IPA_REQ_ANTI) continue;
    if (LV(cl, en->key, n) < 0) continue;
    const int k = key_slot((podstate*)D->st, en->key);
    if (en->kind == KSS_IPA_EXISTING_ANTI) {
      for (int t = 0; t < a->own_terms_len; t++)
        if (in_list32(ps->ints, en->row_off, en->row_len, ps->ints[a->own_terms_off + t])) s->A[k][0] += 1;
    } else if (in_list32(ps->ints, en->row_off, en->row_len, a->cls)) {
      s->A[k][en->kind == KSS_IPA_REQ_AFFINITY ? 1 : 2] += 1;
      if (en->kind == KSS_IPA_REQ_AFFINITY) s->T += 1;
    }
  }
}

/* RunFilterPluginsWithNominatedPods over the dry-run view: the nominees of priority >= the
   preemptor's on node n added first; the plain view decides when that passes */
static int dry_fits_nom(const dryctx* D, const drystate* s, int n) {
  drystate s1;
  int added = 0;
  for (int j = 0; j < D->n_nom; j++) {
    const int q = D->nom_pod[j];
    if (D->nom_node[j] != n || q == D->pi || D->ps->pods[q].priority < D->p->priority) continue;
    if (!added) s1 = *s;
    added = 1;
    dry_apply_nominee(D, q, n, &s1);
  }
  if (added && !dry_fits(D, &s1, n)) return 0;
  return dry_fits(D, s, n);
}

typedef struct {
  int64_t hp, sum, cnt, start; /* hp == INT64_MAX: not a candidate */
} dryres;

/* ⟨k8s⟩ default_preemption.go SelectVictimsOnNode: remove every lower-priority pod, filter,
 * then reprieve in MoreImportantPod order (no PodDisruptionBudgets: every pod is
 * non-violating); victims (optional, cap) receive the boundset ids in eviction order. */
static dryres dry_select(const dryctx* D, int n, int64_t* victims, int cap) {
  const kss_cluster* cl = D->cl;
  const kss_pod* p = D->p;
  const kss_boundset* bs = D->bs;
  const podstate* st = D->st;
  dryres res = {INT64_MAX, 0, 0, 0};
  const int e0 = D->ptr[n], e1 = D->ptr[n + 1];
  int p0 = e1; /* the pods below the preemptor's priority: a suffix of the importance order */
  while (p0 > e0 && bs->priority[D->ord[p0 - 1]] < p->priority) p0--;
  if (p0 == e1) return res; /* "No preemption victims found for incoming pod" */
  drystate s;
  memset(&s, 0, sizeof(s));
  const size_t N = (size_t)cl->n_nodes;
  for (int r = 0; r < 3 + cl->n_scalar; r++) s.req[r] = cl->requested[(size_t)r * N + n];
  s.pods = cl->pod_count[n];
  const kss_spread* hard = D->ps->spreads + p->spread_off;
  for (int i = 0; i < p->n_hard; i++) {
    if (st->hard_own[i] != i) continue;
    const int d = LV(cl, hard[i].key, n);
    s.M[i] = d >= 0 ? st->hard_cnt[i][d] : 0;
  }
  for (int k = 0; k < st->nkeys; k++) {
    const int d = LV(cl, st->keys[k], n);
    if (d < 0) continue;
    s.A[k][0] = st->hx[k][d];
    s.A[k][1] = st->ha[k][d];
    s.A[k][2] = st->hb[k][d];
  }
  s.T = D->aff_total;
  for (int k = p0; k < e1; k++) dry_apply(D, D->ord[k], n, -1, &s);
  if (!dry_fits_nom(D, &s, n)) return res;
  int nv = 0;
  int64_t hp = 0, sum = 0, stt = 0;
  for (int k = p0; k < e1; k++) {
    const int e = D->ord[k];
    dry_apply(D, e, n, 1, &s);
    if (!dry_fits_nom(D, &s, n)) {
      dry_apply(D, e, n, -1, &s);
      if (nv == 0) {
        hp = bs->priority[e];
        stt = bs->start[e]; /* GetEarliestPodStartTime among the highest-priority victims */
      }
      if (victims && nv < cap) victims[nv] = bs->id[e];
      sum += (int64_t)bs->priority[e] + 2147483648ll;
      nv++;
    }
  }
  if (nv == 0) return res; /* upstream: an error status ("expected at least one victim") */
  res.hp = hp;
  res.sum = sum;
  res.cnt = nv;
  res.start = stt;
  return res;
}

/* nodesWherePreemptionMightHelp: UnschedulableAndUnresolvable statuses are skipped */
static int resolvable_status(int f, int detail) {
  if (f == KSS_F_NODE_RESOURCES_FIT || f == KSS_F_NODE_PORTS) return 1;
  if (f == KSS_F_POD_TOPOLOGY_SPREAD) return detail == KSS_PTS_CONSTRAINTS_NOT_MATCH;
  if (f == KSS_F_INTER_POD_AFFINITY) return detail != KSS_IPA_AFFINITY;
  return 0;
}

static int imp_before(const kss_boundset* bs, int a, int b) { /* MoreImportantPod, NodeInfo order on ties */
  if (bs->priority[a] != bs->priority[b]) return bs->priority[a] > bs->priority[b];
  if (bs->start[a] != bs->start[b]) return bs->start[a] < bs->start[b];
  return a < b;
}

/* PostFilter dry run of ps->pods[pi] against cl and the bound pods bs (the state its filters
 * saw).  out->victims / victims_cap as kss_postfilter_pod. */
int kss_oracle_postfilter_n(const kss_profile* prof, const kss_cluster* cl, const kss_podset* ps, int pi,
                            const kss_boundset* bs, int threads, kss_preempt_result* out, const int32_t* nom_pod,
                            const int32_t* nom_node, int32_t n_nom);

int kss_oracle_postfilter(const kss_profile* prof, const kss_cluster* cl, const kss_podset* ps, int pi,
                          const kss_boundset* bs, int threads, kss_preempt_result* out) {
  return kss_oracle_postfilter_n(prof, cl, ps, pi, bs, threads, out, NULL, NULL, 0);
}

/* kss_oracle_postfilter with the scheduling queue's nominator (ps pod indices nominated to global
   nodes): every filter call is RunFilterPluginsWithNominatedPods. */
int kss_oracle_postfilter_n(const kss_profile* prof, const kss_cluster* cl, const kss_podset* ps, int pi,
                            const kss_boundset* bs, int threads, kss_preempt_result* out, const int32_t* nom_pod,
                            const int32_t* nom_node, int32_t n_nom) {
  const kss_pod* p = &ps->pods[pi];
  const int N = cl->n_nodes;
  const int th = threads > 0 ? threads : 1;
  int32_t* nn_local = NULL;
  out->status = KSS_PREEMPT_NO_CANDIDATE;
  out->nominated = -1;
  out->n_potential = out->n_candidates = out->n_victims = 0;
  out->highest_priority = 0;
  out->sum_priority = out->earliest_start = 0;
  if (p->flags & KSS_POD_PREEMPT_NEVER) { /* PodEligibleToPreemptOthers */
    out->status = KSS_PREEMPT_NOT_ELIGIBLE;
    return 0;
  }
  if (p->prefilter_status != 0) return 0; /* every node UnschedulableAndUnresolvable */
  podstate st;
  int rc = podstate_build(&st, cl, ps, p, prof->hard_pod_affinity_weight);
  if (rc) {
    podstate_free(&st);
    return rc;
  }
  int32_t* ptr = (int32_t*)calloc((size_t)N + 1, sizeof(int32_t));
  int32_t* ord = (int32_t*)malloc(sizeof(int32_t) * (size_t)(bs->n > 0 ? bs->n : 1));
  uint8_t* fp = (uint8_t*)malloc((size_t)(N ? N : 1));
  uint16_t* fd = (uint16_t*)malloc(sizeof(uint16_t) * (size_t)(N ? N : 1));
  dryres* dr = (dryres*)malloc(sizeof(dryres) * (size_t)(N ? N : 1));
  uint8_t* inset = NULL;
  if (!ptr || !ord || !fp || !fd || !dr) {
    rc = KSS_E_NOMEM;
    goto done;
  }
  /* NodeInfo.Pods per node (the boundset's order), then each node's MoreImportantPod order
   * (insertion sort: stable, NodeInfo order on ties) */
  for (int i = 0; i < bs->n; i++) {
    const int n = bs->node[i] - cl->node_base;
    if (n >= 0 && n < N) ptr[n + 1]++;
  }
  for (int n = 0; n < N; n++) ptr[n + 1] += ptr[n];
  {
    int32_t* fill = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N ? N : 1));
    for (int n = 0; n < N; n++) fill[n] = ptr[n];
    for (int i = 0; i < bs->n; i++) {
      const int n = bs->node[i] - cl->node_base;
      if (n >= 0 && n < N) ord[fill[n]++] = i;
    }
    free(fill);
  }
  for (int n = 0; n < N; n++)
    for (int a = ptr[n] + 1; a < ptr[n + 1]; a++)
      for (int b = a; b > ptr[n] && imp_before(bs, ord[b], ord[b - 1]); b--) {
        const int32_t t = ord[b];
        ord[b] = ord[b - 1];
        ord[b - 1] = t;
      }
  /* the pod's filter statuses (findNodesThatPassFilters over the PreFilterResult node set) */
  if (p->names_len >= 0) {
    inset = (uint8_t*)calloc((size_t)(N ? N : 1), 1);
    for (int i = 0; i < p->names_len; i++) {
      const int64_t g = ps->ints[p->names_off + i] - cl->node_base;
      if (g >= 0 && g < N) inset[g] = 1;
    }
  }
  int feasible = 0;
#pragma omp parallel for num_threads(th) schedule(static) reduction(+ : feasible)
  for (int n = 0; n < N; n++) {
    fd[n] = 0;
    if (inset && !inset[n]) {
      fp[n] = KSS_F_NOT_EVALUATED; /* no status: potential, the dry run's NodeAffinity rejects it */
      continue;
    }
    fp[n] = (uint8_t)filter_node(prof, cl, ps, p, &st, n, &fd[n]);
    feasible += fp[n] == KSS_F_PASS;
  }
  if (n_nom > 0) { /* the scheduling cycle's statuses on nodes holding nominees (serial: in place) */
    ostate os;
    if (ostate_init(&os, cl)) {
      rc = KSS_E_NOMEM;
      goto done;
    }
    nn_local = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_nom);
    os.nom_active = (uint8_t*)malloc((size_t)n_nom);
    for (int j = 0; j < n_nom; j++) {
      nn_local[j] = nom_node[j] - cl->node_base;
      os.nom_active[j] = nom_pod[j] >= 0 && nom_pod[j] < ps->n_pods && nn_local[j] >= 0 && nn_local[j] < N;
    }
    os.n_nom = n_nom;
    os.nom_pod = nom_pod;
    os.nom_node = nn_local;
    for (int j = 0; j < n_nom; j++) {
      const int n = nn_local[j];
      if (!os.nom_active[j] || (inset && !inset[n])) continue;
      int added;
      const int was = fp[n] == KSS_F_PASS;
      fp[n] = (uint8_t)filter_with_nominated(prof, &os, ps, pi, &st, n, &fd[n], &added);
      feasible += (fp[n] == KSS_F_PASS) - was;
    }
    ostate_free(&os);
  }
  if (feasible) {
    out->status = KSS_PREEMPT_SCHEDULABLE;
    goto done;
  }
  dryctx D;
  memset(&D, 0, sizeof(D));
  D.prof = prof;
  D.cl = cl;
  D.ps = ps;
  D.p = p;
  D.st = &st;
  D.bs = bs;
  D.ptr = ptr;
  D.ord = ord;
  D.n_nom = n_nom;
  D.nom_pod = nom_pod;
  D.nom_node = nn_local;
  D.pi = pi;
  /* criticalPaths per hard owner: the smallest pair count, its pair, the next smallest */
  {
    const kss_spread* hard = ps->spreads + p->spread_off;
    for (int i = 0; i < p->n_hard; i++) {
      D.m0[i] = D.m1[i] = INT32_MAX;
      D.id0[i] = -1;
      if (st.hard_own[i] != i) continue;
      const int bins = cl->key_card[hard[i].key] + 1;
      for (int d = 0; d < bins; d++) {
        if (!st.hard_present[i][d]) continue;
        const int64_t v = st.hard_cnt[i][d];
        if (v < D.m0[i]) {
          D.m1[i] = D.m0[i];
          D.m0[i] = v;
          D.id0[i] = d;
        } else if (v < D.m1[i]) {
          D.m1[i] = v;
        }
      }
    }
    for (int k = 0; k < st.nkeys; k++) {
      const int bins = cl->key_card[st.keys[k]] + 1;
      for (int d = 0; d < bins; d++) D.aff_total += st.ha[k][d];
    }
  }
  /* DryRunPreemption: SelectVictimsOnNode on every potential node, node-parallel */
  int n_pot = 0, n_cand = 0;
#pragma omp parallel for num_threads(th) schedule(dynamic, 16) reduction(+ : n_pot, n_cand)
  for (int n = 0; n < N; n++) {
    dr[n].hp = INT64_MAX;
    const int f = fp[n];
    if (f != KSS_F_NOT_EVALUATED && !resolvable_status(f, fd[n])) continue;
    n_pot++;
    if (f == KSS_F_NOT_EVALUATED) continue;
    dr[n] = dry_select(&D, n, NULL, 0);
    n_cand += dr[n].hp != INT64_MAX;
  }
  out->n_potential = n_pot;
  out->n_candidates = n_cand;
  if (!n_cand) goto done;
  /* pickOneNodeForPreemption in canonical node order: highest victim priority min, priority
   * sum min, victims min, earliest start (of the highest-priority victims) max, then the
   * lowest node index */
  int best = -1;
  for (int n = 0; n < N; n++) {
    if (dr[n].hp == INT64_MAX) continue;
    if (best < 0) {
      best = n;
      continue;
    }
    const dryres* a = &dr[n];
    const dryres* b = &dr[best];
    const int better = a->hp != b->hp ? a->hp < b->hp
                       : a->sum != b->sum ? a->sum < b->sum
                       : a->cnt != b->cnt ? a->cnt < b->cnt
                                          : a->start > b->start;
    if (better) best = n;
  }
  {
    const dryres d = dry_select(&D, best, out->victims, out->victims_cap);
    out->status = KSS_PREEMPT_NOMINATED;
    out->nominated = cl->node_base + best;
    out->n_victims = (int32_t)d.cnt;
    out->highest_priority = (int32_t)d.hp;
    out->sum_priority = d.sum;
    out->earliest_start = d.start;
  }
done:
  podstate_free(&st);
  free(nn_local);
  free(ptr);
  free(ord);
  free(fp);
  free(fd);
  free(dr);
  free(inset);
  return rc;
}
