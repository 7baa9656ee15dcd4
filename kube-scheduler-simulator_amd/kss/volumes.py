"""Volume programs: PersistentVolumes, claims, StorageClasses and CSINodes -> the volume
columns of kss_cluster and each pending pod's kss_vol entries (include/kss.h).

Restates the v1.26.2 volume plugins of the default MultiPoint set
(simulator/scheduler/config/plugin_test.go:15-36) as integer state the device filters read:

  VolumeRestrictions   volumerestrictions/volume_restrictions.go isVolumeConflict (GCE PD,
                       AWS EBS, iSCSI, RBD) -> disk-usage rows; ReadWriteOncePod is an alpha
                       feature gate in v1.26 (off), so only disk conflicts filter.
  EBSLimits, GCEPDLimits, AzureDiskLimits
                       nodevolumelimits/non_csi.go filterVolumes / getMaxVolumeFunc
                       (KUBE_MAX_PD_VOLS unset) -> one attach-limit key per plugin
  NodeVolumeLimits     nodevolumelimits/csi.go filterAttachableVolumes / getCSIDriverInfo /
                       getVolumeLimits, volumeutil.GetCSIAttachLimitKey -> a key per CSI driver
  VolumeBinding        volumebinding/volume_binding.go PreFilter (podHasPVCs,
                       GetPodVolumeClaims) -> KSS_PF_VOLUME_BINDING; Filter -> binder.go
                       FindPodVolumes: checkBoundClaims -> KSS_VOL_BIND_AFFINITY / _PV_MISSING
                       entries (PV node affinity as node-selector terms over the node's labels
                       alone); unbound WaitForFirstConsumer claims -> KSS_VOL_BIND_WFFC entries
                       (findMatchingVolumes / FindMatchingVolume's static checks resolved here into
                       each claim's candidate PVs, smallest first; checkVolumeProvisions' class
                       provisioner and allowedTopologies) over the binder's assume cache, which
                       the cluster carries as pv_owner / claim_node
  VolumeZone           volumezone/volume_zone.go Filter -> KSS_VOL_ZONE requirements

The device never sees a volume object.  A volume that a pending pod uses is either
*private* (no other pod uses it: it is new on every node, counted on the chosen node at
AssumePod) or *shared*, in which case it gets a vol_count row so the filter can find it
already attached on a node.  Disk usages a pending pod's volumes conflict with get rows too.

Refused (kss.compile.Unsupported), each naming why: a StorageClass without volumeBindingMode (a
PreFilter Error), in-tree volumes of a plugin a CSINode lists as migrated (CSI translation), nodes
whose two instance-type labels disagree (getMaxVolumeFunc reads whichever Go map order yields
first), more than KSS_MAX_WFFC delayed claims in one pod, and two PVs pre-bound to one delayed
claim (which FindMatchingVolume returns depends on pvCache list order).  Determinism decision:
ListPVs is map-backed, so equally small PVs go by name.  Storage capacity (hasEnoughCapacity) is
not checked: it applies only to CSIDrivers with storageCapacity set, and the snapshot
(ResourcesForSnap) carries none.
"""
from __future__ import annotations

import hashlib
import re
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .quantity import value

ANN_BIND_COMPLETED = "pv.kubernetes.io/bind-completed"
ANN_BETA_STORAGE_CLASS = "volume.beta.kubernetes.io/storage-class"
ANN_MIGRATED_PLUGINS = "storage.alpha.kubernetes.io/migrated-plugins"
VOLUME_ZONE_LABELS = ("failure-domain.beta.kubernetes.io/zone", "failure-domain.beta.kubernetes.io/region",
                      "topology.kubernetes.io/zone", "topology.kubernetes.io/region")
INSTANCE_TYPE_LABELS = ("beta.kubernetes.io/instance-type", "node.kubernetes.io/instance-type")
UNBOUND_IMMEDIATE = "pod has unbound immediate PersistentVolumeClaims"
ANN_SELECTED_NODE = "volume.kubernetes.io/selected-node"
NOT_SUPPORTED_PROVISIONER = "kubernetes.io/no-provisioner"

# plugin -> (pod / PV volume source, id field, provisioner = in-tree plugin name, limit key, default max)
NON_CSI = {
    abi.KSS_F_EBS_LIMITS: ("awsElasticBlockStore", "volumeID", "kubernetes.io/aws-ebs", "attachable-volumes-aws-ebs", None),
    abi.KSS_F_GCEPD_LIMITS: ("gcePersistentDisk", "pdName", "kubernetes.io/gce-pd", "attachable-volumes-gce-pd", 16),
    abi.KSS_F_AZURE_DISK_LIMITS: ("azureDisk", "diskName", "kubernetes.io/azure-disk", "attachable-volumes-azure-disk",
                                  16),
}
# in-tree sources csi-translation-lib (v1.26) can migrate, by source field -> in-tree plugin name
MIGRATABLE = {"awsElasticBlockStore": "kubernetes.io/aws-ebs", "gcePersistentDisk": "kubernetes.io/gce-pd",
              "azureDisk": "kubernetes.io/azure-disk", "azureFile": "kubernetes.io/azure-file",
              "cinder": "kubernetes.io/cinder", "vsphereVolume": "kubernetes.io/vsphere-volume",
              "portworxVolume": "kubernetes.io/portworx-volume", "rbd": "kubernetes.io/rbd"}
ID_PREFIX = "kss-vol"  # the plugins' randomVolumeIDPrefix: only equality of ids matters


def _meta(o):
    return (o or {}).get("metadata") or {}


def _spec(o):
    return (o or {}).get("spec") or {}


def _ns(o):
    return _meta(o).get("namespace") or "default"


def csi_attach_limit_key(driver: str) -> str:
    """volumeutil.GetCSIAttachLimitKey."""
    prefix = "attachable-volumes-csi-"
    if len(prefix) + len(driver) >= 63:  # ResourceNameLengthLimit
        return prefix + driver[:23] + hashlib.sha1(driver.encode()).hexdigest()[:16]
    return prefix + driver


def default_max_ebs(instance_type: str) -> int:
    """getMaxEBSVolume: EBSNitroLimitRegex "^[cmr]5.*|t3|z1d" -> 25, otherwise 39."""
    return 25 if re.search(r"^[cmr]5.*|t3|z1d", instance_type) else 39


def disk_usages(pod) -> List[tuple]:
    """The pod's volumes VolumeRestrictions checks (needsRestrictionsCheck), as usage
    entries (kind, identity, readOnly); RBD's pool defaults to "rbd" (API defaulting)."""
    out = []
    for v in _spec(pod).get("volumes") or []:
        if v.get("gcePersistentDisk") is not None:
            d = v["gcePersistentDisk"]
            out.append(("gce", d.get("pdName"), bool(d.get("readOnly"))))
        elif v.get("awsElasticBlockStore") is not None:
            d = v["awsElasticBlockStore"]
            out.append(("ebs", d.get("volumeID"), bool(d.get("readOnly"))))
        elif v.get("iscsi") is not None:
            d = v["iscsi"]
            out.append(("iscsi", d.get("iqn"), bool(d.get("readOnly"))))
        elif v.get("rbd") is not None:
            d = v["rbd"]
            out.append(("rbd", (tuple(sorted(set(d.get("monitors") or []))), d.get("pool") or "rbd", d.get("image")),
                        bool(d.get("readOnly"))))
    return out


def usages_conflict(a: tuple, b: tuple) -> bool:
    """isVolumeConflict for one pair of usage entries."""
    if a[0] != b[0]:
        return False
    kind, ia, ra = a
    _, ib, rb = b
    if kind == "ebs":
        return ia == ib
    if kind in ("gce", "iscsi"):
        return ia == ib and not (ra and rb)
    return bool(set(ia[0]) & set(ib[0])) and ia[1:] == ib[1:] and not (ra and rb)  # rbd: monitors overlap


class VolumeCompiler:
    """Storage objects + nodes (canonical order) + bound / pending pods -> volume columns
    and per-pod volume facts.  Construct, then read: label_keys (for the compiler's key
    dictionary), arrays(), program(pod index) and prefilter(pod index)."""

    def __init__(self, storage: Optional[dict], nodes: Sequence[dict], bound_on: Sequence[Tuple[dict, int]],
                 pending: Sequence[dict]):
        st = storage or {}
        self.pv = {_meta(p)["name"]: p for p in st.get("pvs") or []}
        self.pvc = {(_ns(p), _meta(p)["name"]): p for p in st.get("pvcs") or []}
        self.sc = {_meta(s)["name"]: s for s in st.get("storage_classes") or st.get("storageClasses") or []}
        self.csinode = {_meta(c)["name"]: c for c in st.get("csinodes") or []}
        self.nodes = list(nodes)
        self.bound_on = list(bound_on)      # (pod, canonical node index) of NodeInfo pods
        self.pending = list(pending)
        self.N = len(self.nodes)
        self.messages: List[str] = []
        self._msg_index: Dict[str, int] = {}
        self._check_migration()
        self._prefilter = [self._binding_prefilter(p) for p in self.pending]
        self._build()

    # ---------------------------------------------------------------- objects
    @staticmethod
    def claim_name(pod, vol) -> Tuple[Optional[str], bool]:
        if vol.get("persistentVolumeClaim") is not None:
            return vol["persistentVolumeClaim"].get("claimName") or "", False
        if vol.get("ephemeral") is not None:  # ephemeral.VolumeClaimName
            return _meta(pod).get("name", "") + "-" + (vol.get("name") or ""), True
        return None, False

    def get_pvc(self, pod, name):
        return self.pvc.get((_ns(pod), name))

    @staticmethod
    def pvc_class(pvc) -> str:
        """storagehelpers.GetPersistentVolumeClaimClass."""
        ann = _meta(pvc).get("annotations") or {}
        if ANN_BETA_STORAGE_CLASS in ann:
            return ann[ANN_BETA_STORAGE_CLASS]
        return _spec(pvc).get("storageClassName") or ""

    @staticmethod
    def not_for_pod(pod, pvc) -> Optional[str]:
        """ephemeral.VolumeIsForPod's error message, or None."""
        pm, cm = _meta(pod), _meta(pvc)
        owned = any(r.get("controller") and (r.get("uid") or "") == (pm.get("uid") or "")
                    for r in cm.get("ownerReferences") or [])
        if _ns(pod) != _ns(pvc) or not owned:
            return f"PVC {_ns(pvc)}/{cm.get('name')} was not created for pod {_ns(pod)}/{pm.get('name')} (pod is not owner)"
        return None

    def _migrated_plugins(self, node) -> List[str]:
        c = self.csinode.get(_meta(node).get("name"))
        mpa = (_meta(c).get("annotations") or {}).get(ANN_MIGRATED_PLUGINS) if c else None
        return mpa.split(",") if mpa else []

    def _check_migration(self):
        migrated = set()
        for n in self.nodes:
            migrated.update(self._migrated_plugins(n))
        if not migrated:
            return
        from .compile import Unsupported
        for pod in [p for p, _ in self.bound_on] + self.pending:
            for vol in _spec(pod).get("volumes") or []:
                for f, plugin in MIGRATABLE.items():
                    if vol.get(f) is not None and plugin in migrated:
                        raise Unsupported(f"in-tree {f} volume of a plugin migrated to CSI ({plugin}): CSI translation")
                name, _ = self.claim_name(pod, vol)
                pvc = self.get_pvc(pod, name) if name is not None else None
                if pvc is None:
                    continue
                pv = self.pv.get(_spec(pvc).get("volumeName") or "")
                for f, plugin in MIGRATABLE.items():
                    if pv is not None and _spec(pv).get(f) is not None and plugin in migrated:
                        raise Unsupported(f"in-tree {f} PV of a plugin migrated to CSI ({plugin}): CSI translation")
                sc = self.sc.get(self.pvc_class(pvc))
                if sc is not None and sc.get("provisioner") in migrated:
                    raise Unsupported(f"provisioner {sc.get('provisioner')} migrated to CSI: CSI translation")

    def message(self, m: str) -> int:
        if m not in self._msg_index:
            self._msg_index[m] = len(self.messages)
            self.messages.append(m)
        return self._msg_index[m]

    # ---------------------------------------------------------------- VolumeBinding PreFilter
    def _binding_prefilter(self, pod):
        """(message or None, bound claims or None): podHasPVCs then GetPodVolumeClaims."""
        from .compile import Unsupported
        has = False
        for vol in _spec(pod).get("volumes") or []:
            name, eph = self.claim_name(pod, vol)
            if name is None:
                continue
            has = True
            pvc = self.get_pvc(pod, name)
            if pvc is None:
                if eph:
                    return f'waiting for ephemeral volume controller to create the persistentvolumeclaim "{name}"', None
                return f'persistentvolumeclaim "{name}" not found', None
            if (pvc.get("status") or {}).get("phase") == "Lost":
                return (f'persistentvolumeclaim "{name}" bound to non-existent persistentvolume '
                        f'"{_spec(pvc).get("volumeName") or ""}"'), None
            if _meta(pvc).get("deletionTimestamp"):
                return f'persistentvolumeclaim "{name}" is being deleted', None
            if eph:
                err = self.not_for_pod(pod, pvc)
                if err:
                    return err, None
        if not has:
            return None, None
        bound, delayed, immediate = [], [], False
        for vol in _spec(pod).get("volumes") or []:
            name, _ = self.claim_name(pod, vol)
            if name is None:
                continue
            pvc = self.get_pvc(pod, name)
            if _spec(pvc).get("volumeName") and ANN_BIND_COMPLETED in (_meta(pvc).get("annotations") or {}):
                bound.append(pvc)  # isPVCFullyBound
                continue
            cls, delay = self.pvc_class(pvc), False
            if cls and cls in self.sc:  # volume.IsDelayBindingMode (an unknown class: not delayed)
                mode = self.sc[cls].get("volumeBindingMode")
                if mode is None:
                    raise Unsupported(f'VolumeBindingMode not set for StorageClass "{cls}" (a PreFilter Error)')
                delay = mode == "WaitForFirstConsumer"
            if delay and not _spec(pvc).get("volumeName"):
                delayed.append(pvc)  # unboundClaimsDelayBinding
                continue
            immediate = True  # "Prebound PVCs are treated as unbound immediate binding"
        if immediate:
            return UNBOUND_IMMEDIATE, None
        if len(delayed) > abi.KSS_MAX_WFFC:
            raise Unsupported(f"more than {abi.KSS_MAX_WFFC} unbound WaitForFirstConsumer claims in one pod")
        return None, (bound, delayed)

    # ---------------------------------------------------------------- limit plugins
    def _non_csi_ids(self, plugin, pod, new_pod) -> set:
        """nonCSILimits.filterVolumes."""
        from .compile import Unsupported
        field, idf, prov, _, _ = NON_CSI[plugin]
        out = set()
        for vol in _spec(pod).get("volumes") or []:
            if vol.get(field) is not None:
                out.add(vol[field].get(idf))
                continue
            name, eph = self.claim_name(pod, vol)
            if name is None:
                continue
            pvc = self.get_pvc(pod, name)
            if pvc is None:
                if new_pod:
                    raise Unsupported("a pending pod's claim is missing")  # VolumeBinding PreFilter rejects it first
                continue
            if eph and self.not_for_pod(pod, pvc):
                raise Unsupported("ephemeral claim not owned by its pod (a filter Error)")
            sc = _spec(pvc).get("storageClassName")
            match_prov = sc is not None and sc in self.sc and self.sc[sc].get("provisioner") == prov
            pv_id = f"{ID_PREFIX}-{_ns(pod)}/{name}"
            pv_name = _spec(pvc).get("volumeName") or ""
            pv = self.pv.get(pv_name) if pv_name else None
            if pv is None:
                if match_prov:
                    out.add(pv_id)
                continue
            if _spec(pv).get(field) is not None:
                out.add(_spec(pv)[field].get(idf))
        return out

    def _csi_volumes(self, pod, new_pod) -> Dict[str, str]:
        """CSILimits.filterAttachableVolumes: unique name -> limit key."""
        from .compile import Unsupported
        out = {}
        for vol in _spec(pod).get("volumes") or []:
            name, eph = self.claim_name(pod, vol)
            if name is None:
                continue  # inline in-tree volumes: counted by CSILimits only when migrated (refused)
            pvc = self.get_pvc(pod, name)
            if pvc is None:
                if new_pod:
                    raise Unsupported("a pending pod's claim is missing")
                continue
            if eph and self.not_for_pod(pod, pvc):
                raise Unsupported("ephemeral claim not owned by its pod (a filter Error)")
            drv, handle = self._csi_driver_info(pvc)
            if drv and handle:
                out[f"{drv}/{handle}"] = csi_attach_limit_key(drv)
        return out

    def _csi_driver_info(self, pvc) -> Tuple[str, str]:
        pv_name = _spec(pvc).get("volumeName") or ""
        pv = self.pv.get(pv_name) if pv_name else None
        if pv is None:  # getCSIDriverInfoFromSC
            cls = self.pvc_class(pvc)
            sc = self.sc.get(cls) if cls else None
            prov = (sc or {}).get("provisioner") or ""
            if not prov or prov in MIGRATABLE.values():
                return "", ""
            return prov, f"{ID_PREFIX}-{_ns(pvc)}/{_meta(pvc).get('name')}"
        csi = _spec(pv).get("csi")
        if csi is None:
            return "", ""  # in-tree PV, migration off: the non-CSI plugins count it
        return csi.get("driver") or "", csi.get("volumeHandle") or ""

    def _csi_limits(self, node) -> Dict[str, int]:
        """getVolumeLimits: attachable-volumes-* allocatable, then the CSINode drivers' counts."""
        out = {}
        for k, v in ((node.get("status") or {}).get("allocatable") or {}).items():
            if k.startswith("attachable-volumes-"):
                out[k] = value(v)
        c = self.csinode.get(_meta(node).get("name"))
        for d in (_spec(c).get("drivers") or []) if c else []:
            cnt = (d.get("allocatable") or {}).get("count")
            if cnt is not None:
                out[csi_attach_limit_key(d.get("name") or "")] = int(cnt)
        return out

    def _non_csi_limit(self, plugin, node) -> int:
        from .compile import Unsupported
        _, _, prov, key, dflt = NON_CSI[plugin]
        if prov in self._migrated_plugins(node):
            return -1  # IsMigrated: defer to the CSI plugin
        if dflt is None:
            lb = _meta(node).get("labels") or {}
            vals = {lb[k] for k in INSTANCE_TYPE_LABELS if k in lb}
            if len(vals) > 1:
                raise Unsupported("node with two different instance-type labels (getMaxVolumeFunc takes Go map order)")
            dflt = default_max_ebs(vals.pop() if vals else "")
        alloc = (node.get("status") or {}).get("allocatable") or {}
        return value(alloc[key]) if key in alloc else dflt

    # ---------------------------------------------------------------- VolumeZone
    def zone_constraints(self, pod) -> Tuple[List[List[Tuple[str, List[str]]]], Optional[str]]:
        """Per PVC volume in order, its PV's zone labels as (key, allowed values); the first
        per-volume status error ends the list (the message)."""
        out: List[List[Tuple[str, List[str]]]] = []
        for vol in _spec(pod).get("volumes") or []:
            pvcv = vol.get("persistentVolumeClaim")
            if pvcv is None:
                continue
            name = pvcv.get("claimName") or ""
            if not name:
                return out, "PersistentVolumeClaim had no name"
            pvc = self.get_pvc(pod, name)
            if pvc is None:
                return out, f'persistentvolumeclaim "{name}" not found'
            pv_name = _spec(pvc).get("volumeName") or ""
            if not pv_name:
                cls = self.pvc_class(pvc)
                if not cls:
                    return out, "PersistentVolumeClaim had no pv name and storageClass name"
                if cls not in self.sc:
                    return out, f'storageclass.storage.k8s.io "{cls}" not found'
                mode = self.sc[cls].get("volumeBindingMode")
                if mode is None:
                    return out, f'VolumeBindingMode not set for StorageClass "{cls}"'
                if mode == "WaitForFirstConsumer":
                    continue
                return out, "PersistentVolume had no name"
            pv = self.pv.get(pv_name)
            if pv is None:
                return out, f'persistentvolume "{pv_name}" not found'
            cons = []
            for k, v in sorted((_meta(pv).get("labels") or {}).items()):
                if k not in VOLUME_ZONE_LABELS:
                    continue
                zs = []
                for z in v.split("__"):  # volumehelpers.LabelZonesToSet
                    z = z.strip()
                    if not z:
                        zs = None
                        break
                    zs.append(z)
                if zs is not None:  # a parse error ignores the label
                    cons.append((k, sorted(set(zs))))
            if cons:
                out.append(cons)
        return out, None

    def label_keys(self) -> set:
        """Label keys the volume programs read: the PVs' node-affinity keys and zone keys."""
        keys = set()
        for j, pod in enumerate(self.pending):
            msg, claims = self._prefilter[j]
            bound, delayed = claims or ([], [])
            pvs = [self.pv.get(_spec(pvc).get("volumeName")) for pvc in bound]
            for pvc in delayed:
                c = self.wclaim_index[self.claim_key(pvc)]
                pvs += [self.pv[self.pv_names[v]] for v in self.wclaim_cands[c]]
                sc = self.sc.get(self.pvc_class(pvc)) or {}
                for t in sc.get("allowedTopologies") or []:
                    for e in t.get("matchLabelExpressions") or []:
                        keys.add(e.get("key", ""))
            for pv in pvs:
                req = ((_spec(pv).get("nodeAffinity") or {}).get("required")) if pv else None
                for t in (req or {}).get("nodeSelectorTerms") or []:
                    for e in t.get("matchExpressions") or []:
                        keys.add(e.get("key", ""))
            if msg is None and (_spec(pod).get("volumes") or []):
                cons, _ = self.zone_constraints(pod)
                for c in cons:
                    keys.update(k for k, _ in c)
        return keys

    # ---------------------------------------------------------------- rows and keys
    def _build(self):
        N = self.N
        nb = len(self.bound_on)
        pods = [p for p, _ in self.bound_on] + self.pending  # pod id: bound first, then pending
        pend = range(nb, nb + len(self.pending))
        live = [j for j in range(len(self.pending)) if self._prefilter[j][0] is None]
        # --- disk usage rows
        usages = [sorted(set(disk_usages(p))) for p in pods]
        wanted = [usages[nb + j] for j in live]
        rows: List[tuple] = []
        row_index: Dict[tuple, int] = {}
        for u in sorted({e for us in usages for e in us}, key=repr):
            if any(usages_conflict(w, u) for ws in wanted for w in ws):
                row_index[("disk", u)] = len(rows)
                rows.append(("disk", u))
        # --- attach-limit volumes per key: key name -> (plugin, {pod id: set of unique names})
        per_key: Dict[str, Tuple[int, Dict[int, set]]] = {}
        for i, pod in enumerate(pods):
            new = i >= nb
            if new and self._prefilter[i - nb][0] is not None:
                continue  # rejected at PreFilter: never filtered, never committed
            for plugin in NON_CSI:
                ids = self._non_csi_ids(plugin, pod, new)
                if ids:
                    per_key.setdefault(NON_CSI[plugin][3], (plugin, {}))[1][i] = ids
            for uname, key in self._csi_volumes(pod, new).items():
                per_key.setdefault(key, (abi.KSS_F_NODE_VOLUME_LIMITS, {}))[1].setdefault(i, set()).add(uname)
        # keys the pending pods use, in filter order (EBS, GCE PD, CSI drivers, Azure Disk)
        order = {abi.KSS_F_EBS_LIMITS: 0, abi.KSS_F_GCEPD_LIMITS: 1, abi.KSS_F_NODE_VOLUME_LIMITS: 2,
                 abi.KSS_F_AZURE_DISK_LIMITS: 3}
        keys = sorted((k for k, (_, by) in per_key.items() if any(i in by for i in pend)),
                      key=lambda k: (order[per_key[k][0]], k))
        if len(keys) > abi.KSS_MAX_VOL_KEYS:
            from .compile import Unsupported
            raise Unsupported(f"more than {abi.KSS_MAX_VOL_KEYS} attach-limit keys")
        self.keys = keys
        key_index = {k: i for i, k in enumerate(keys)}
        users: Dict[Tuple[int, str], set] = {}  # (key, unique name) -> pod ids using it
        for k in keys:
            for i, names in per_key[k][1].items():
                for u in names:
                    users.setdefault((key_index[k], u), set()).add(i)
        shared = sorted((ku for ku, us in users.items() if len(us) > 1 and any(i in pend for i in us)),
                        key=lambda ku: (ku[0], ku[1]))
        for ku in shared:
            row_index[("vol", ku)] = len(rows)
            rows.append(("vol", ku))
        self.rows = rows
        R, K = len(rows), len(keys)
        vol_count = np.zeros((R, N), np.int32)
        vol_attached = np.zeros((K, N), np.int32)
        vol_row_key = np.array([ku[0] if kind == "vol" else -1 for kind, ku in rows], np.int32)
        for i, (pod, n) in enumerate(self.bound_on):
            for u in usages[i]:
                r = row_index.get(("disk", u))
                if r is not None:
                    vol_count[r, n] += 1
        attached_names: Dict[Tuple[int, int], set] = {}
        for (k, u), us in users.items():
            for i in us:
                if i < nb:
                    n = self.bound_on[i][1]
                    attached_names.setdefault((k, n), set()).add(u)
                    r = row_index.get(("vol", (k, u)))
                    if r is not None:
                        vol_count[r, n] += 1
        for (k, n), names in attached_names.items():
            vol_attached[k, n] = len(names)
        vol_limit = np.full((K, N), -1, np.int32)
        vol_key_plugin = np.array([per_key[k][0] for k in keys], np.int32)
        for n, node in enumerate(self.nodes):
            csi = None
            for k, key in enumerate(keys):
                plugin = per_key[key][0]
                if plugin == abi.KSS_F_NODE_VOLUME_LIMITS:
                    csi = self._csi_limits(node) if csi is None else csi
                    vol_limit[k, n] = csi.get(key, -1)
                else:
                    vol_limit[k, n] = self._non_csi_limit(plugin, node)
        self.vol_count, self.vol_attached, self.vol_limit = vol_count, vol_attached, vol_limit
        self.vol_row_key, self.vol_key_plugin = vol_row_key, vol_key_plugin
        self._build_wffc(live)
        # --- per pending pod: conflict rows, limit entries, own rows
        self._conflict, self._limits, self._own, self._private = {}, {}, {}, {}
        for j in live:
            i = nb + j
            mine = usages[i]
            self._conflict[j] = sorted({r for (kind, u), r in row_index.items() if kind == "disk"
                                        and any(usages_conflict(w, u) for w in mine)})
            own = {row_index[("disk", u)] for u in mine if ("disk", u) in row_index}
            lim: List[Tuple[int, int, int]] = []  # (key, row, count)
            priv: Dict[int, int] = {}
            for k, key in enumerate(keys):
                names = per_key[key][1].get(i)
                if not names:
                    continue
                n_priv = 0
                for u in sorted(names):
                    r = row_index.get(("vol", (k, u)))
                    if r is None:
                        n_priv += 1
                    else:
                        lim.append((k, r, 0))
                        own.add(r)
                if n_priv:
                    lim.append((k, -1, n_priv))
                    priv[k] = n_priv
            self._limits[j] = lim
            self._own[j] = sorted(own)
            self._private[j] = priv

    # ---------------------------------------------------------------- WaitForFirstConsumer
    @staticmethod
    def claim_key(pvc) -> Tuple[str, str]:
        return _ns(pvc), _meta(pvc).get("name") or ""

    @staticmethod
    def claim_request(pvc) -> int:
        return value(((_spec(pvc).get("resources") or {}).get("requests") or {}).get("storage", "0"))

    @staticmethod
    def pv_class(pv) -> str:
        """storagehelpers.GetPersistentVolumeClass."""
        ann = _meta(pv).get("annotations") or {}
        if ANN_BETA_STORAGE_CLASS in ann:
            return ann[ANN_BETA_STORAGE_CLASS]
        return _spec(pv).get("storageClassName") or ""

    @staticmethod
    def bound_to(pv, pvc) -> bool:
        """IsVolumeBoundToClaim: claimRef name / namespace, and uid when the ref has one."""
        ref = _spec(pv).get("claimRef")
        if not ref:
            return False
        return ((ref.get("name") or "") == (_meta(pvc).get("name") or "") and (ref.get("namespace") or "") == _ns(pvc)
                and (not ref.get("uid") or ref.get("uid") == (_meta(pvc).get("uid") or "")))

    def _candidates(self, pvc) -> Tuple[List[str], Optional[str]]:
        """FindMatchingVolume's node-independent checks over ListPVs(class): the PVs the claim may
        bind in increasing capacity, then name, and the PV pre-bound to it (claimRef) if any."""
        from .compile import Unsupported
        from .selectors import SelectorError, label_selector_as_selector
        cls = self.pvc_class(pvc)
        req = self.claim_request(pvc)
        mode = _spec(pvc).get("volumeMode") or "Filesystem"
        modes = set(_spec(pvc).get("accessModes") or [])
        sel = _spec(pvc).get("selector")
        try:
            selector = label_selector_as_selector(sel) if sel is not None else None
        except SelectorError:
            raise Unsupported("a WaitForFirstConsumer claim's selector does not parse (a Filter Error)")
        out, pre = [], []
        for name in sorted(self.pv):
            pv = self.pv[name]
            if self.pv_class(pv) != cls:
                continue
            ref = _spec(pv).get("claimRef")
            if ref and not self.bound_to(pv, pvc):
                continue
            cap = value((_spec(pv).get("capacity") or {}).get("storage", "0"))
            if cap < req or (_spec(pv).get("volumeMode") or "Filesystem") != mode or _meta(pv).get("deletionTimestamp"):
                continue
            if ref:
                pre.append(name)  # returned whenever its node affinity holds (phase / selector / modes unchecked)
                out.append((cap, name))
                continue
            if ((pv.get("status") or {}).get("phase")) != "Available":
                continue
            if selector is not None and not selector.matches(_meta(pv).get("labels") or {}):
                continue
            if not modes <= set(_spec(pv).get("accessModes") or []):
                continue
            out.append((cap, name))
        if len(pre) > 1:
            raise Unsupported("two PVs pre-bound (claimRef) to one WaitForFirstConsumer claim: "
                              "FindMatchingVolume's answer depends on pvCache list order")
        return [nm for _, nm in sorted(out)], (pre[0] if pre else None)

    def _build_wffc(self, live):
        """The delayed claims of the live pending pods (ids in first-use order), their candidate
        PVs (ids in order of first appearance) and the assume cache's initial state."""
        claims: List[dict] = []
        self.wclaim_index: Dict[Tuple[str, str], int] = {}
        for j in live:
            _, cl = self._prefilter[j]
            for pvc in (cl or ([], []))[1]:
                k = self.claim_key(pvc)
                if k not in self.wclaim_index:
                    self.wclaim_index[k] = len(claims)
                    claims.append(pvc)
        self.pv_names: List[str] = []
        pv_index: Dict[str, int] = {}
        self.wclaim_cands: List[List[int]] = []
        owner: Dict[int, int] = {}
        for c, pvc in enumerate(claims):
            names, pre = self._candidates(pvc)
            ids = []
            for nm in names:
                if nm not in pv_index:
                    pv_index[nm] = len(self.pv_names)
                    self.pv_names.append(nm)
                ids.append(pv_index[nm])
            self.wclaim_cands.append(ids)
            if pre is not None:
                owner[pv_index[pre]] = c + 1
        self.wclaims = claims
        self.pv_owner = np.array([owner.get(v, 0) for v in range(len(self.pv_names))], np.int32)
        node_index = {(_meta(n).get("name") or ""): i for i, n in enumerate(self.nodes)}
        sel = []
        for pvc in claims:
            s = (_meta(pvc).get("annotations") or {}).get(ANN_SELECTED_NODE)
            sel.append(-1 if s is None else node_index.get(s, -2))
        self.claim_node = np.array(sel, np.int32)

    # ---------------------------------------------------------------- results
    def node_zone_flags(self) -> np.ndarray:
        f = np.zeros(self.N, np.uint32)
        for n, node in enumerate(self.nodes):
            lb = _meta(node).get("labels") or {}
            if any(k in lb for k in VOLUME_ZONE_LABELS):
                f[n] = abi.KSS_NODE_VOLUME_ZONE
        return f

    def prefilter(self, j: int) -> Tuple[Optional[str], Optional[list]]:
        return self._prefilter[j]

    def program(self, j: int, pv_terms, zone_reqs, int_list=None) -> List[tuple]:
        """kss_vol rows (kind, key, row, count, a, b) of pending pod j, in filter order.
        pv_terms(required node selector) -> (term_off, term_len); zone_reqs([(key, values)])
        -> (req_off, req_len); int_list(values) -> (off, len): the compiler's pools."""
        msg, claims = self._prefilter[j]
        if msg is not None:
            return []
        pod = self.pending[j]
        out = [(abi.KSS_VOL_CONFLICT, -1, r, 0, 0, 0) for r in self._conflict[j]]
        out += [(abi.KSS_VOL_LIMIT, k, r, c, 0, 0) for k, r, c in self._limits[j]]
        bound, delayed = claims or ([], [])
        for pvc in bound:  # checkBoundClaims, in claim order
            pv = self.pv.get(_spec(pvc).get("volumeName"))
            if pv is None:
                out.append((abi.KSS_VOL_BIND_PV_MISSING, -1, -1, 0, 0, 0))
                break
            req = (_spec(pv).get("nodeAffinity") or {}).get("required")
            if req is not None:
                a, b = pv_terms(req.get("nodeSelectorTerms") or [])
                out.append((abi.KSS_VOL_BIND_AFFINITY, -1, -1, 0, a, b))
        # unbound WaitForFirstConsumer claims: findMatchingVolumes' order (byPVCSize, stable)
        for pvc in sorted(delayed, key=self.claim_request):
            c = self.wclaim_index[self.claim_key(pvc)]
            trip = []
            for v in self.wclaim_cands[c]:
                req = (_spec(self.pv[self.pv_names[v]]).get("nodeAffinity") or {}).get("required")
                ta, tb = pv_terms(req.get("nodeSelectorTerms") or []) if req is not None else (0, -1)
                trip += [v, ta, tb]
            a, _ = int_list(trip)
            sc = self.sc[self.pvc_class(pvc)]
            prov = (sc.get("provisioner") or "") not in ("", NOT_SUPPORTED_PROVISIONER)
            topo = [{"matchExpressions": [{"key": e.get("key", ""), "operator": "In", "values": list(e.get("values") or [])}
                                          for e in t.get("matchLabelExpressions") or []]}
                    for t in sc.get("allowedTopologies") or []]
            ta, tb = pv_terms(topo) if topo else (0, 0)
            if topo and tb == 0:  # every term empty: "nil or empty term selects no objects"
                prov = False
            out.append((abi.KSS_VOL_BIND_WFFC, c, ta, (tb << 1) | (1 if prov else 0), a, len(trip) // 3))
        if _spec(pod).get("volumes") or []:
            cons, err = self.zone_constraints(pod)
            for c in cons:
                a, b = zone_reqs(c)
                out.append((abi.KSS_VOL_ZONE, -1, -1, 0, a, b))
            if err is not None:
                out.append((abi.KSS_VOL_ZONE_ERROR, -1, -1, 0, self.message(err), 0))
        out += [(abi.KSS_VOL_OWN, -1, r, 0, 0, 0) for r in self._own[j]]
        out += [(abi.KSS_VOL_OWN_PRIVATE, k, -1, c, 0, 0) for k, c in sorted(self._private[j].items())]
        return out
