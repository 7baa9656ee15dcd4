"""Object-level ORACLE for the volume plugins (TEST INFRASTRUCTURE ONLY) — pure Python.

An independent restatement, on Kubernetes-shaped objects, of the v1.26.2 volume plugins of
the default MultiPoint set (simulator/scheduler/config/plugin_test.go:15-36; upstream
k8s.io/kubernetes v1.26.2, simulator/go.mod:56 — not vendored, so every rule below is
restated from the upstream function it names):

  VolumeRestrictions  volumerestrictions/volume_restrictions.go  Filter: satisfyVolumeConflicts /
                      isVolumeConflict (GCE PD, AWS EBS, iSCSI, RBD).  ReadWriteOncePod is an
                      alpha feature gate in v1.26 (beta, on by default, from v1.27): off, so
                      PreFilter returns success and Filter checks disk conflicts only.
  EBSLimits / GCEPDLimits / AzureDiskLimits
                      nodevolumelimits/non_csi.go  nonCSILimits.Filter / filterVolumes /
                      getMaxVolumeFunc (KUBE_MAX_PD_VOLS unset)
  NodeVolumeLimits    nodevolumelimits/csi.go  CSILimits.Filter / filterAttachableVolumes /
                      getCSIDriverInfo(FromSC) / getVolumeLimits; volumeutil.GetCSIAttachLimitKey
  VolumeBinding       volumebinding/volume_binding.go PreFilter (podHasPVCs,
                      GetPodVolumeClaims) / Filter -> binder.go FindPodVolumes: checkBoundClaims,
                      findMatchingVolumes (pv_helpers.go FindMatchingVolume) and
                      checkVolumeProvisions for unbound WaitForFirstConsumer claims; Reserve ->
                      AssumePodVolumes (the assume cache), Unreserve -> RevertAssumedPodVolumes;
                      Score returns 0 (VolumeCapacityPriority is alpha, off)
  VolumeZone          volumezone/volume_zone.go  Filter

Determinism decisions (upstream is random here): FindMatchingVolume walks pvCache.ListPVs(class),
a map-backed list, and keeps the first of equally small PVs -- here the PVs go by name.  Storage
capacity (hasEnoughCapacity) is not checked: it applies only to CSIDriver objects with
storageCapacity set, and the simulator's snapshot (ResourcesForSnap) carries no CSIDrivers.

Refused (Unsupported), each with its reason: a StorageClass without volumeBindingMode (a PreFilter
Error), in-tree volumes of a plugin some CSINode lists as migrated
(storage.alpha.kubernetes.io/migrated-plugins: CSI translation), an unbound WaitForFirstConsumer
claim without a class name or whose class is missing at provisioning (Filter Errors), and two PVs
pre-bound (spec.claimRef) to one claim (which FindMatchingVolume returns depends on list order).

Used only by tests/ (checker), never by the product.
"""
from __future__ import annotations

import hashlib
import re
from typing import Dict, List, Optional, Tuple

ANN_BIND_COMPLETED = "pv.kubernetes.io/bind-completed"
ANN_BETA_STORAGE_CLASS = "volume.beta.kubernetes.io/storage-class"
ANN_MIGRATED_PLUGINS = "storage.alpha.kubernetes.io/migrated-plugins"
VOLUME_ZONE_LABELS = ("failure-domain.beta.kubernetes.io/zone", "failure-domain.beta.kubernetes.io/region",
                      "topology.kubernetes.io/zone", "topology.kubernetes.io/region")
INSTANCE_TYPE_LABELS = ("beta.kubernetes.io/instance-type", "node.kubernetes.io/instance-type")

MSG_DISK_CONFLICT = "node(s) had no available disk"
MSG_MAX_VOLUME_COUNT = "node(s) exceed max volume count"
MSG_NODE_CONFLICT = "node(s) had volume node affinity conflict"
MSG_PV_NOT_EXIST = "node(s) unavailable due to one or more pvc(s) bound to non-existent pv(s)"
MSG_ZONE_CONFLICT = "node(s) had no available volume zone"
MSG_UNBOUND_IMMEDIATE = "pod has unbound immediate PersistentVolumeClaims"
MSG_BIND_CONFLICT = "node(s) didn't find available persistent volumes to bind"
ANN_SELECTED_NODE = "volume.kubernetes.io/selected-node"
NOT_SUPPORTED_PROVISIONER = "kubernetes.io/no-provisioner"

# the in-tree limit plugins: (plugin, inline/PV source field, id field, provisioner, limit key, default max)
NON_CSI = {
    "EBSLimits": ("awsElasticBlockStore", "volumeID", "kubernetes.io/aws-ebs", "attachable-volumes-aws-ebs", None),
    "GCEPDLimits": ("gcePersistentDisk", "pdName", "kubernetes.io/gce-pd", "attachable-volumes-gce-pd", 16),
    "AzureDiskLimits": ("azureDisk", "diskName", "kubernetes.io/azure-disk", "attachable-volumes-azure-disk", 16),
}
# in-tree plugins CSI migration can translate (csi-translation-lib, v1.26), by PV/inline source field
MIGRATABLE = {"awsElasticBlockStore": "kubernetes.io/aws-ebs", "gcePersistentDisk": "kubernetes.io/gce-pd",
              "azureDisk": "kubernetes.io/azure-disk", "azureFile": "kubernetes.io/azure-file",
              "cinder": "kubernetes.io/cinder", "vsphereVolume": "kubernetes.io/vsphere-volume",
              "portworxVolume": "kubernetes.io/portworx-volume", "rbd": "kubernetes.io/rbd"}
RANDOM_PREFIX = "kss"  # each plugin's randomVolumeIDPrefix: only equality of the ids matters


class Unsupported(Exception):
    pass


def _meta(o):
    return o.get("metadata") or {}


def _spec(o):
    return o.get("spec") or {}


def csi_attach_limit_key(driver: str) -> str:
    """volumeutil.GetCSIAttachLimitKey: 'attachable-volumes-csi-' + driver, or for names
    that would reach 63 characters the first 23 characters + 16 hex of sha1(driver)."""
    prefix = "attachable-volumes-csi-"
    if len(prefix) + len(driver) >= 63:
        return prefix + driver[:23] + hashlib.sha1(driver.encode()).hexdigest()[:16]
    return prefix + driver


def max_ebs_volumes(instance_type: str) -> int:
    """getMaxEBSVolume: regexp.MatchString("^[cmr]5.*|t3|z1d", type) -> 25 (Nitro), else 39."""
    return 25 if re.search(r"^[cmr]5.*|t3|z1d", instance_type) else 39


def instance_type(node) -> str:
    """getMaxVolumeFunc's label loop (the first of the two instance-type labels in map order;
    the restatement refuses nodes carrying both with different values)."""
    lb = _meta(node).get("labels") or {}
    vals = {lb[k] for k in INSTANCE_TYPE_LABELS if k in lb}
    if len(vals) > 1:
        raise Unsupported("node carries both instance-type labels with different values (Go map order)")
    return vals.pop() if vals else ""


def label_zones_to_set(v: str):
    """volumehelpers.LabelZonesToSet: split on "__", trim; an empty element is an error (None)."""
    out = set()
    for z in v.split("__"):
        z = z.strip()
        if not z:
            return None
        out.add(z)
    return out


def storage_bytes(q) -> int:
    """resource.Quantity of a storage request / capacity, in bytes (0 when absent)."""
    if q is None:
        return 0
    from k8s_oracle import qvalue
    return qvalue(q)


class VBClaims:
    """GetPodVolumeClaims: the pod's bound claims and its unbound WaitForFirstConsumer claims
    (pod volume order)."""

    def __init__(self, bound, delayed):
        self.bound = bound
        self.delayed = delayed


class Storage:
    """The snapshot's PVs, PVCs, StorageClasses and CSINodes (listers), plus the binder's assume
    cache for WaitForFirstConsumer claims: PVs assumed bound to a claim (spec.claimRef) and claims
    assumed provisioned on a node (the selected-node annotation)."""

    def __init__(self, pvs=(), pvcs=(), storage_classes=(), csinodes=()):
        self.pv = {_meta(p)["name"]: p for p in pvs}
        self.pvc = {(_meta(p).get("namespace") or "default", _meta(p)["name"]): p for p in pvcs}
        self.sc = {_meta(s)["name"]: s for s in storage_classes}
        self.csinode = {_meta(c)["name"]: c for c in csinodes}
        # the assume cache: pv name -> (namespace, claim name, uid) of its claimRef; claim key -> node name
        self.pv_ref0 = {}
        for name, pv in self.pv.items():
            ref = _spec(pv).get("claimRef")
            if ref:
                self.pv_ref0[name] = (ref.get("namespace") or "", ref.get("name") or "", ref.get("uid") or "")
        self.pv_ref = dict(self.pv_ref0)
        self.selected0 = {}
        for key, pvc in self.pvc.items():
            sel = (_meta(pvc).get("annotations") or {}).get(ANN_SELECTED_NODE)
            if sel is not None:
                self.selected0[key] = sel
        self.selected = dict(self.selected0)

    # ------------------------------------------------------------ helpers
    @staticmethod
    def claim_name(pod, vol) -> Tuple[Optional[str], bool]:
        """(pvcName, isEphemeral) of a PVC-backed volume (ephemeral.VolumeClaimName), else (None, False)."""
        if vol.get("persistentVolumeClaim") is not None:
            return vol["persistentVolumeClaim"].get("claimName") or "", False
        if vol.get("ephemeral") is not None:
            return _meta(pod)["name"] + "-" + vol.get("name", ""), True
        return None, False

    def get_pvc(self, pod, name):
        return self.pvc.get((_meta(pod).get("namespace") or "default", name))

    @staticmethod
    def pvc_class(pvc) -> str:
        """storagehelpers.GetPersistentVolumeClaimClass."""
        ann = _meta(pvc).get("annotations") or {}
        if ANN_BETA_STORAGE_CLASS in ann:
            return ann[ANN_BETA_STORAGE_CLASS]
        return _spec(pvc).get("storageClassName") or ""

    @staticmethod
    def volume_is_for_pod(pod, pvc) -> Optional[str]:
        """ephemeral.VolumeIsForPod: the error message, or None."""
        pm, cm = _meta(pod), _meta(pvc)
        pns, cns = pm.get("namespace") or "default", cm.get("namespace") or "default"
        owned = any(r.get("controller") and (r.get("uid") or "") == (pm.get("uid") or "")
                    for r in cm.get("ownerReferences") or [])
        if pns != cns or not owned:
            return f"PVC {cns}/{cm['name']} was not created for pod {pns}/{pm['name']} (pod is not owner)"
        return None

    def migrated(self, node_name: str, plugin: str) -> bool:
        """isCSIMigrationOn: the CSINode's migrated-plugins annotation lists the plugin."""
        c = self.csinode.get(node_name)
        if c is None:
            return False
        mpa = (_meta(c).get("annotations") or {}).get(ANN_MIGRATED_PLUGINS) or ""
        return plugin in (mpa.split(",") if mpa else [])

    def check_migration(self, nodes, pods):
        """Refuse in-tree volumes (inline, PV sources, unbound PVCs' in-tree provisioners) of a
        plugin some CSINode lists as migrated: their CSI translation is not restated."""
        migrated = set()
        for n in nodes:
            c = self.csinode.get(_meta(n)["name"])
            mpa = (_meta(c).get("annotations") or {}).get(ANN_MIGRATED_PLUGINS) if c else None
            if mpa:
                migrated.update(mpa.split(","))
        if not migrated:
            return
        for pod in pods:
            for vol in _spec(pod).get("volumes") or []:
                for f, pl in MIGRATABLE.items():
                    if vol.get(f) is not None and pl in migrated:
                        raise Unsupported(f"in-tree {f} volume with {pl} migrated to CSI")
                name, _ = self.claim_name(pod, vol)
                pvc = self.get_pvc(pod, name) if name is not None else None
                if pvc is None:
                    continue
                pv = self.pv.get(_spec(pvc).get("volumeName") or "")
                for f, pl in MIGRATABLE.items():
                    if pv is not None and _spec(pv).get(f) is not None and pl in migrated:
                        raise Unsupported(f"in-tree {f} PV with {pl} migrated to CSI")
                sc = self.sc.get(self.pvc_class(pvc))
                if sc is not None and sc.get("provisioner") in migrated:
                    raise Unsupported(f"StorageClass provisioner {sc.get('provisioner')} migrated to CSI")

    # ------------------------------------------------------------ VolumeBinding
    def binding_prefilter(self, pod):
        """VolumeBinding.PreFilter: (None, bound claims) on success (claims None: skip), or
        (message, None) for an UnschedulableAndUnresolvable status."""
        has = False
        for vol in _spec(pod).get("volumes") or []:  # podHasPVCs
            name, eph = self.claim_name(pod, vol)
            if name is None:
                continue
            has = True
            pvc = self.get_pvc(pod, name)
            if pvc is None:
                if eph:
                    return f'waiting for ephemeral volume controller to create the persistentvolumeclaim "{name}"', None
                return f'persistentvolumeclaim "{name}" not found', None
            if ((pvc.get("status") or {}).get("phase")) == "Lost":
                return (f'persistentvolumeclaim "{name}" bound to non-existent persistentvolume '
                        f'"{_spec(pvc).get("volumeName") or ""}"'), None
            if _meta(pvc).get("deletionTimestamp"):
                return f'persistentvolumeclaim "{name}" is being deleted', None
            if eph:
                err = self.volume_is_for_pod(pod, pvc)
                if err:
                    return err, None
        if not has:
            return None, None
        bound, delayed, immediate = [], [], False
        for vol in _spec(pod).get("volumes") or []:  # GetPodVolumeClaims
            name, _ = self.claim_name(pod, vol)
            if name is None:
                continue
            pvc = self.get_pvc(pod, name)
            if _spec(pvc).get("volumeName") and ANN_BIND_COMPLETED in (_meta(pvc).get("annotations") or {}):
                bound.append(pvc)
                continue
            cls = self.pvc_class(pvc)
            delay = False
            if cls and cls in self.sc:  # IsDelayBindingMode (a missing class: not delayed)
                mode = self.sc[cls].get("volumeBindingMode")
                if mode is None:
                    raise Unsupported(f'VolumeBindingMode not set for StorageClass "{cls}" (a PreFilter Error)')
                delay = mode == "WaitForFirstConsumer"
            if delay and not _spec(pvc).get("volumeName"):
                delayed.append(pvc)  # unboundClaimsDelayBinding
                continue
            immediate = True  # "Prebound PVCs are treated as unbound immediate binding"
        if immediate:
            return MSG_UNBOUND_IMMEDIATE, None
        return None, VBClaims(bound, delayed)

    @staticmethod
    def _pv_node_ok(pv, node, node_selector_terms) -> bool:
        """volumeutil.CheckNodeAffinity(pv, node.Labels): the PV's required node selector over a
        node that carries only the labels."""
        req = ((_spec(pv).get("nodeAffinity") or {}).get("required"))
        if req is None:
            return True
        labels_only = {"metadata": {"labels": dict(_meta(node).get("labels") or {})}}
        return node_selector_terms(req.get("nodeSelectorTerms") or []).match(labels_only)

    @staticmethod
    def _claim_key(pvc):
        return (_meta(pvc).get("namespace") or "default", _meta(pvc)["name"])

    def _bound_to(self, pv_name, pvc) -> bool:
        """IsVolumeBoundToClaim against the assume cache's claimRef."""
        ref = self.pv_ref.get(pv_name)
        if ref is None:
            return False
        ns, name = self._claim_key(pvc)
        uid = _meta(pvc).get("uid") or ""
        return ref[0] == ns and ref[1] == name and (ref[2] == "" or ref[2] == uid)

    def find_matching_volume(self, pvc, node, excluded, node_selector_terms) -> Optional[str]:
        """pv_helpers.go FindMatchingVolume(claim, pvCache.ListPVs(class), node, chosenPVs,
        delayBinding=true): a PV bound to the claim is returned (or nothing, if its node
        affinity fails) wherever it comes; otherwise the smallest available PV that passes every
        check (ties: the first by name)."""
        cls = self.pvc_class(pvc)
        req = storage_bytes(((_spec(pvc).get("resources") or {}).get("requests") or {}).get("storage"))
        sel = _spec(pvc).get("selector")
        claim_mode = _spec(pvc).get("volumeMode") or "Filesystem"
        modes = set(_spec(pvc).get("accessModes") or [])
        best, best_q = None, None
        for name in sorted(self.pv):
            pv = self.pv[name]
            if self.pv_class(pv) != cls or name in excluded:  # ListPVs(class); excludedVolumes
                continue
            if name in self.pv_ref and not self._bound_to(name, pvc):
                continue
            q = storage_bytes((_spec(pv).get("capacity") or {}).get("storage"))
            if q < req:
                continue
            if (_spec(pv).get("volumeMode") or "Filesystem") != claim_mode:  # CheckVolumeModeMismatches
                continue
            if _meta(pv).get("deletionTimestamp"):
                continue
            ok = self._pv_node_ok(pv, node, node_selector_terms)
            if self._bound_to(name, pvc):
                return name if ok else None
            if ((pv.get("status") or {}).get("phase")) != "Available":
                continue
            if sel is not None and not self._selector_matches(sel, _meta(pv).get("labels") or {}):
                continue
            if not ok:
                continue
            if not modes <= set(_spec(pv).get("accessModes") or []):  # CheckAccessModes
                continue
            if best is None or q < best_q:
                best, best_q = name, q
        return best

    @staticmethod
    def pv_class(pv) -> str:
        """storagehelpers.GetPersistentVolumeClass."""
        ann = _meta(pv).get("annotations") or {}
        if ANN_BETA_STORAGE_CLASS in ann:
            return ann[ANN_BETA_STORAGE_CLASS]
        return _spec(pv).get("storageClassName") or ""

    @staticmethod
    def _selector_matches(sel, labels) -> bool:
        """metav1.LabelSelectorAsSelector(...).Matches (a selector that does not parse is a
        FindMatchingVolume error: a Filter Error status, refused)."""
        from k8s_oracle import LSel
        ls = LSel(sel)
        if getattr(ls, "error", False):
            raise Unsupported("a claim selector that does not parse (a Filter Error)")
        return ls.matches(labels)

    def _provisionable(self, pvc, node) -> bool:
        """checkVolumeProvisions for one claim: a class with a provisioner whose allowedTopologies
        admit the node (MatchTopologySelectorTerms over the node's labels)."""
        cls = self.pvc_class(pvc)
        if not cls or cls not in self.sc:
            raise Unsupported("an unbound WaitForFirstConsumer claim without a (known) class: a Filter Error")
        sc = self.sc[cls]
        prov = sc.get("provisioner") or ""
        if prov == "" or prov == NOT_SUPPORTED_PROVISIONER:
            return False
        terms = sc.get("allowedTopologies") or []
        if not terms:
            return True
        lb = _meta(node).get("labels") or {}
        return any(all(e.get("key") in lb and lb[e.get("key")] in (e.get("values") or [])
                       for e in t.get("matchLabelExpressions") or []) for t in terms)

    def find_pod_volumes(self, claims, node, node_selector_terms):
        """binder.go FindPodVolumes: (reasons, static bindings [(pvc, pv name)], claims to provision)."""
        bound_ok, pvs_found, unbound_ok = True, True, True
        bindings, provision = [], []
        for pvc in claims.bound:  # checkBoundClaims: the first failure ends the walk
            pv = self.pv.get(_spec(pvc).get("volumeName"))
            if pv is None:
                pvs_found = False
                break
            if not self._pv_node_ok(pv, node, node_selector_terms):
                bound_ok = False
                break
        if claims.delayed:
            to_match, fast_fail = [], False
            for pvc in claims.delayed:
                sel = self.selected.get(self._claim_key(pvc))
                if sel is not None:
                    if sel != _meta(node).get("name"):
                        unbound_ok, fast_fail = False, True
                        break
                    provision.append(pvc)
                else:
                    to_match.append(pvc)
            if not fast_fail:
                if to_match:  # findMatchingVolumes: claims by increasing request (stable)
                    chosen = set()
                    for pvc in sorted(to_match, key=lambda c: storage_bytes(
                            ((_spec(c).get("resources") or {}).get("requests") or {}).get("storage"))):
                        pv = self.find_matching_volume(pvc, node, chosen, node_selector_terms)
                        if pv is None:
                            provision.append(pvc)
                            unbound_ok = False
                        else:
                            chosen.add(pv)
                            bindings.append((pvc, pv))
                if provision:  # checkVolumeProvisions: the first claim that cannot be provisioned ends it
                    unbound_ok = all(self._provisionable(pvc, node) for pvc in provision)
        reasons = []
        if not bound_ok:
            reasons.append(MSG_NODE_CONFLICT)
        if not unbound_ok:
            reasons.append(MSG_BIND_CONFLICT)
        if not pvs_found:
            reasons.append(MSG_PV_NOT_EXIST)
        return reasons, bindings, provision

    def binding_filter(self, claims, node, node_selector_terms) -> Optional[str]:
        """VolumeBinding.Filter -> FindPodVolumes: the status message (the reasons joined with
        ", "), or None."""
        if claims is None:
            return None
        reasons, _, _ = self.find_pod_volumes(claims, node, node_selector_terms)
        return ", ".join(reasons) if reasons else None

    def assume(self, claims, node, node_selector_terms):
        """Reserve -> AssumePodVolumes on the chosen node: the static bindings' PVs get the
        claim as claimRef, the provisioned claims the node as selected-node."""
        if claims is None or not claims.delayed:
            return
        _, bindings, provision = self.find_pod_volumes(claims, node, node_selector_terms)
        for pvc, pv in bindings:
            ns, name = self._claim_key(pvc)
            self.pv_ref[pv] = (ns, name, _meta(pvc).get("uid") or "")
        for pvc in provision:
            self.selected[self._claim_key(pvc)] = _meta(node).get("name")

    def revert(self, claims):
        """Unreserve -> RevertAssumedPodVolumes: the claims' PVs and the claims back to the
        informer's (snapshot) objects."""
        if claims is None:
            return
        for pvc in claims.delayed:
            key = self._claim_key(pvc)
            for pv, ref in list(self.pv_ref.items()):
                if (ref[0], ref[1]) == key and self.pv_ref0.get(pv) != ref:
                    if pv in self.pv_ref0:
                        self.pv_ref[pv] = self.pv_ref0[pv]
                    else:
                        del self.pv_ref[pv]
            if key in self.selected0:
                self.selected[key] = self.selected0[key]
            else:
                self.selected.pop(key, None)

    # ------------------------------------------------------------ VolumeRestrictions
    @staticmethod
    def is_volume_conflict(v, pod) -> bool:
        """isVolumeConflict(volume, existing pod)."""
        for ev in _spec(pod).get("volumes") or []:
            a, b = v.get("gcePersistentDisk"), ev.get("gcePersistentDisk")
            if a is not None and b is not None:
                if a.get("pdName") == b.get("pdName") and not (a.get("readOnly") and b.get("readOnly")):
                    return True
            a, b = v.get("awsElasticBlockStore"), ev.get("awsElasticBlockStore")
            if a is not None and b is not None and a.get("volumeID") == b.get("volumeID"):
                return True
            a, b = v.get("iscsi"), ev.get("iscsi")
            if a is not None and b is not None:
                if a.get("iqn") == b.get("iqn") and not (a.get("readOnly") and b.get("readOnly")):
                    return True
            a, b = v.get("rbd"), ev.get("rbd")
            if a is not None and b is not None:
                if (set(a.get("monitors") or []) & set(b.get("monitors") or [])
                        and (a.get("pool") or "rbd") == (b.get("pool") or "rbd")
                        and a.get("image") == b.get("image") and not (a.get("readOnly") and b.get("readOnly"))):
                    return True
        return False

    def restrictions_filter(self, pod, node_pods) -> Optional[str]:
        for v in _spec(pod).get("volumes") or []:
            if not any(v.get(f) is not None for f in ("gcePersistentDisk", "awsElasticBlockStore", "rbd", "iscsi")):
                continue  # needsRestrictionsCheck
            for ep in node_pods:
                if self.is_volume_conflict(v, ep):
                    return MSG_DISK_CONFLICT
        return None

    # ------------------------------------------------------------ non-CSI limits
    def _non_csi_ids(self, plugin, pod, new_pod) -> set:
        """nonCSILimits.filterVolumes."""
        field, idf, prov, _, _ = NON_CSI[plugin]
        out = set()
        ns = _meta(pod).get("namespace") or "default"
        for vol in _spec(pod).get("volumes") or []:
            if vol.get(field) is not None:  # FilterVolume
                out.add(vol[field].get(idf))
                continue
            name, eph = self.claim_name(pod, vol)
            if name is None:
                continue
            pv_id = f"{RANDOM_PREFIX}-{ns}/{name}"
            pvc = self.get_pvc(pod, name)
            if pvc is None:
                if new_pod:
                    raise Unsupported("new pod's PVC missing (VolumeBinding PreFilter rejects it first)")
                continue
            if eph and self.volume_is_for_pod(pod, pvc):
                raise Unsupported("ephemeral PVC not owned by the pod (an Error status)")
            pv_name = _spec(pvc).get("volumeName") or ""
            sc = _spec(pvc).get("storageClassName")
            match_prov = sc is not None and sc in self.sc and self.sc[sc].get("provisioner") == prov
            if not pv_name:
                if match_prov:
                    out.add(pv_id)
                continue
            pv = self.pv.get(pv_name)
            if pv is None:
                if match_prov:
                    out.add(pv_id)
                continue
            if _spec(pv).get(field) is not None:  # FilterPersistentVolume
                out.add(_spec(pv)[field].get(idf))
        return out

    def non_csi_filter(self, plugin, pod, ni) -> Optional[str]:
        if not (_spec(pod).get("volumes") or []):
            return None
        new = self._non_csi_ids(plugin, pod, True)
        if not new:
            return None
        node = ni.node
        if self.migrated(_meta(node)["name"], NON_CSI[plugin][2]):
            return None
        existing = set()
        for pi in ni.pods:
            existing |= self._non_csi_ids(plugin, pi.pod, False)
        new -= existing
        _, _, _, key, dflt = NON_CSI[plugin]
        limit = max_ebs_volumes(instance_type(node)) if dflt is None else dflt
        alloc = (node.get("status") or {}).get("allocatable") or {}
        if key in alloc:
            limit = int(alloc[key])
        return MSG_MAX_VOLUME_COUNT if len(existing) + len(new) > limit else None

    # ------------------------------------------------------------ CSI limits
    def _csi_driver_info(self, pvc, ns) -> Tuple[str, str]:
        """getCSIDriverInfo / getCSIDriverInfoFromSC (no migration: refused up front)."""
        pv_name = _spec(pvc).get("volumeName") or ""
        pv = self.pv.get(pv_name) if pv_name else None
        if pv is None:
            cls = self.pvc_class(pvc)
            if not cls or cls not in self.sc:
                return "", ""
            prov = self.sc[cls].get("provisioner") or ""
            if not prov or prov in MIGRATABLE.values():  # in-tree provisioner, migration off
                return "", ""
            return prov, f"{RANDOM_PREFIX}-{ns}/{_meta(pvc)['name']}"
        csi = _spec(pv).get("csi")
        if csi is None:
            return "", ""
        return csi.get("driver") or "", csi.get("volumeHandle") or ""

    def _csi_volumes(self, pod, new_pod) -> Dict[str, str]:
        """CSILimits.filterAttachableVolumes: unique name -> limit key."""
        out = {}
        ns = _meta(pod).get("namespace") or "default"
        for vol in _spec(pod).get("volumes") or []:
            name, eph = self.claim_name(pod, vol)
            if name is None:
                continue
            pvc = self.get_pvc(pod, name)
            if pvc is None:
                if new_pod:
                    raise Unsupported("new pod's PVC missing (VolumeBinding PreFilter rejects it first)")
                continue
            if eph and self.volume_is_for_pod(pod, pvc):
                raise Unsupported("ephemeral PVC not owned by the pod (an Error status)")
            drv, handle = self._csi_driver_info(pvc, ns)
            if not drv or not handle:
                continue
            out[f"{drv}/{handle}"] = csi_attach_limit_key(drv)
        return out

    def csi_limits(self, node) -> Dict[str, int]:
        """getVolumeLimits: attachable-volumes-* allocatable, then the CSINode drivers' counts."""
        out = {}
        for k, v in ((node.get("status") or {}).get("allocatable") or {}).items():
            if k.startswith("attachable-volumes-"):
                out[k] = int(v)
        c = self.csinode.get(_meta(node)["name"])
        for d in ((_spec(c).get("drivers") or []) if c else []):
            cnt = (d.get("allocatable") or {}).get("count")
            if cnt is not None:
                out[csi_attach_limit_key(d.get("name") or "")] = int(cnt)
        return out

    def csi_filter(self, pod, ni) -> Optional[str]:
        if not (_spec(pod).get("volumes") or []):
            return None
        new = self._csi_volumes(pod, True)
        if not new:
            return None
        limits = self.csi_limits(ni.node)
        if not limits:
            return None
        attached = {}
        for pi in ni.pods:
            attached.update(self._csi_volumes(pi.pod, False))
        att_count: Dict[str, int] = {}
        for uname, key in attached.items():
            new.pop(uname, None)
            att_count[key] = att_count.get(key, 0) + 1
        new_count: Dict[str, int] = {}
        for key in new.values():
            new_count[key] = new_count.get(key, 0) + 1
        for key, cnt in new_count.items():
            if key in limits and att_count.get(key, 0) + cnt > limits[key]:
                return MSG_MAX_VOLUME_COUNT
        return None

    # ------------------------------------------------------------ VolumeZone
    def zone_filter(self, pod, node) -> Optional[str]:
        vols = _spec(pod).get("volumes") or []
        if not vols:
            return None
        lb = _meta(node).get("labels") or {}
        cons = {k: v for k, v in lb.items() if k in VOLUME_ZONE_LABELS}
        if not cons:
            return None
        for vol in vols:
            pvcv = vol.get("persistentVolumeClaim")
            if pvcv is None:
                continue
            name = pvcv.get("claimName") or ""
            if not name:
                return "PersistentVolumeClaim had no name"
            pvc = self.get_pvc(pod, name)
            if pvc is None:
                return f'persistentvolumeclaim "{name}" not found'
            pv_name = _spec(pvc).get("volumeName") or ""
            if not pv_name:
                cls = self.pvc_class(pvc)
                if not cls:
                    return "PersistentVolumeClaim had no pv name and storageClass name"
                if cls not in self.sc:
                    return f'storageclass.storage.k8s.io "{cls}" not found'
                mode = self.sc[cls].get("volumeBindingMode")
                if mode is None:
                    return f'VolumeBindingMode not set for StorageClass "{cls}"'
                if mode == "WaitForFirstConsumer":
                    continue
                return "PersistentVolume had no name"
            pv = self.pv.get(pv_name)
            if pv is None:
                return f'persistentvolume "{pv_name}" not found'
            for k, v in (_meta(pv).get("labels") or {}).items():
                if k not in VOLUME_ZONE_LABELS:
                    continue
                s = label_zones_to_set(v)
                if s is None:
                    continue  # a parse error: the label is ignored
                if cons.get(k, "") not in s:
                    return MSG_ZONE_CONFLICT
        return None
