"""ctypes loader for the C oracle (oracle/build/libkss_oracle.so) — test infrastructure."""
import ctypes as C
import os
import subprocess

import numpy as np

from kss import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "build", "libkss_oracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        _lib = C.CDLL(LIB)
        P = C.POINTER
        _lib.kss_oracle_schedule.argtypes = [P(abi.Profile), P(abi.Cluster), P(abi.PodSet), C.c_int,
                                             P(C.c_int32), P(abi.PodResult), C.c_int, P(C.c_int64), P(C.c_int64),
                                             P(C.c_int32), P(C.c_int32), P(C.c_int32), P(C.c_uint64)]
        _lib.kss_oracle_schedule.restype = C.c_int
        _lib.kss_oracle_schedule_v.argtypes = _lib.kss_oracle_schedule.argtypes + [P(C.c_int32), P(C.c_int32)]
        _lib.kss_oracle_schedule_v.restype = C.c_int
        _lib.kss_oracle_schedule_c.argtypes = _lib.kss_oracle_schedule_v.argtypes + [P(C.c_int32)]
        _lib.kss_oracle_schedule_c.restype = C.c_int
        _lib.kss_oracle_schedule_n.argtypes = _lib.kss_oracle_schedule_c.argtypes + [
            P(C.c_int32), P(C.c_int32), C.c_int32, P(C.c_uint8)]
        _lib.kss_oracle_schedule_n.restype = C.c_int
        _lib.kss_oracle_schedule_w.argtypes = _lib.kss_oracle_schedule_n.argtypes + [P(C.c_int32), P(C.c_int32)]
        _lib.kss_oracle_schedule_w.restype = C.c_int
        _lib.kss_oracle_schedule_wm.argtypes = _lib.kss_oracle_schedule_w.argtypes + [P(C.c_uint8)]
        _lib.kss_oracle_schedule_wm.restype = C.c_int
        _lib.kss_oracle_eval_pod.argtypes = [P(abi.Profile), P(abi.Cluster), P(abi.PodSet), C.c_int,
                                             P(abi.PodResult), C.c_int]
        _lib.kss_oracle_eval_pod.restype = C.c_int
        _lib.kss_oracle_go_log.argtypes = [C.c_double]
        _lib.kss_oracle_go_log.restype = C.c_double
        _lib.kss_oracle_max_threads.restype = C.c_int
        _lib.kss_oracle_postfilter.argtypes = [P(abi.Profile), P(abi.Cluster), P(abi.PodSet), C.c_int,
                                               P(abi.Boundset), C.c_int, P(abi.PreemptResult)]
        _lib.kss_oracle_postfilter.restype = C.c_int
        _lib.kss_oracle_postfilter_n.argtypes = _lib.kss_oracle_postfilter.argtypes + [P(C.c_int32), P(C.c_int32),
                                                                                        C.c_int32]
        _lib.kss_oracle_postfilter_n.restype = C.c_int
    return _lib


def postfilter(profile, cluster_struct, podset_struct, i, boundset_struct, threads=1, victims_cap=1024,
               nominations=()):
    """kss_oracle_postfilter(_n): the C PostFilter dry run of pod i (the same dict as
    native.Context.postfilter_pod); nominations: [(pod index, global node)]."""
    vic = np.zeros(max(victims_cap, 1), np.int64)
    r = abi.PreemptResult()
    r.victims_cap = victims_cap
    r.victims = vic.ctypes.data_as(C.POINTER(C.c_int64))
    nominations = list(nominations)
    nom_pod = np.array([a for a, _ in nominations] or [0], dtype=np.int32)
    nom_node = np.array([b for _, b in nominations] or [0], dtype=np.int32)
    rc = lib().kss_oracle_postfilter_n(C.byref(profile), C.byref(cluster_struct), C.byref(podset_struct), i,
                                       C.byref(boundset_struct), threads, C.byref(r),
                                       nom_pod.ctypes.data_as(C.POINTER(C.c_int32)),
                                       nom_node.ctypes.data_as(C.POINTER(C.c_int32)), len(nominations))
    if rc:
        raise RuntimeError(f"kss_oracle_postfilter: {rc}")
    return dict(status=r.status, nominated=r.nominated, n_potential=r.n_potential, n_candidates=r.n_candidates,
                victims=[int(v) for v in vic[:min(r.n_victims, victims_cap)]], n_victims=r.n_victims,
                highest_priority=r.highest_priority, sum_priority=r.sum_priority, earliest_start=r.earliest_start)


class Results:
    """Per-pod result arrays (numpy) for n pods x N nodes."""

    def __init__(self, n_pods, n_nodes, arrays=True):
        N = max(n_nodes, 1)
        self.structs = (abi.PodResult * max(n_pods, 1))()
        if not arrays:  # per-pod outcomes only (chosen, n_feasible, scored, status, best_total)
            return
        self.fail_plugin = np.zeros((n_pods, N), dtype=np.uint8)
        self.fail_detail = np.zeros((n_pods, N), dtype=np.uint16)
        self.raw = np.zeros((n_pods, abi.KSS_NSCORE, N), dtype=np.int64)
        self.norm = np.zeros((n_pods, abi.KSS_NSCORE, N), dtype=np.int64)
        self.total = np.zeros((n_pods, N), dtype=np.int64)
        for i in range(n_pods):
            s = self.structs[i]
            s.fail_plugin = self.fail_plugin[i].ctypes.data_as(C.POINTER(C.c_uint8))
            s.fail_detail = self.fail_detail[i].ctypes.data_as(C.POINTER(C.c_uint16))
            s.raw = self.raw[i].ctypes.data_as(C.POINTER(C.c_int64))
            s.norm = self.norm[i].ctypes.data_as(C.POINTER(C.c_int64))
            s.total = self.total[i].ctypes.data_as(C.POINTER(C.c_int64))

    def meta(self, i):
        s = self.structs[i]
        return dict(n_feasible=s.n_feasible, chosen=s.chosen, best_total=s.best_total, scored=s.scored,
                    status=s.status)


def schedule(profile, cluster_struct, podset_struct, n_pods, n_nodes, threads=1, record=True, n_classes=0,
             n_terms=0, cursor=0, nominations=(), skip_commit=None):
    """Run the C oracle sequentially; returns (chosen, Results|None, final_state dict).
    record=True keeps every per-node array, record="meta" only the per-pod outcomes.
    cursor: the scheduler's nextStartNodeIndex at the first pod; the final value is
    final_state["next_start"].  nominations: [(pod index, global node)] in the nominator's
    order; final_state["nominations"] lists those still active afterwards.  skip_commit: per pod,
    evaluated but not assumed (a commit the caller rolled back)."""
    L = lib()
    chosen = np.full(max(n_pods, 1), -2, dtype=np.int32)
    res = Results(n_pods, n_nodes, arrays=record is True) if record else None
    N = max(n_nodes, 1)
    st = dict(requested=np.zeros((abi.KSS_NRES, N), np.int64), nonzero=np.zeros((2, N), np.int64),
              pod_count=np.zeros(N, np.int32), class_count=np.zeros((max(n_classes, 1), N), np.int32),
              term_count=np.zeros((max(n_terms, 1), N), np.int32), port_used=np.zeros(N, np.uint64),
              vol_count=np.zeros((max(cluster_struct.n_vol_rows, 1), N), np.int32),
              vol_attached=np.zeros((max(cluster_struct.n_vol_keys, 1), N), np.int32),
              pv_owner=np.zeros(max(cluster_struct.n_pvs, 1), np.int32),
              claim_node=np.zeros(max(cluster_struct.n_wclaims, 1), np.int32))
    P = C.POINTER
    cur = C.c_int32(cursor)
    nominations = list(nominations)
    nom_pod = np.array([a for a, _ in nominations] or [0], dtype=np.int32)
    nom_node = np.array([b for _, b in nominations] or [0], dtype=np.int32)
    nom_left = np.zeros(max(len(nominations), 1), dtype=np.uint8)
    skip = np.zeros(max(n_pods, 1), np.uint8)
    if skip_commit is not None:
        skip[:n_pods] = np.asarray(skip_commit, np.uint8)[:n_pods]
    rc = L.kss_oracle_schedule_wm(C.byref(profile), C.byref(cluster_struct), C.byref(podset_struct), n_pods,
                               chosen.ctypes.data_as(P(C.c_int32)), res.structs if res else None, threads,
                               st["requested"].ctypes.data_as(P(C.c_int64)), st["nonzero"].ctypes.data_as(P(C.c_int64)),
                               st["pod_count"].ctypes.data_as(P(C.c_int32)),
                               st["class_count"].ctypes.data_as(P(C.c_int32)),
                               st["term_count"].ctypes.data_as(P(C.c_int32)),
                               st["port_used"].ctypes.data_as(P(C.c_uint64)),
                               st["vol_count"].ctypes.data_as(P(C.c_int32)),
                               st["vol_attached"].ctypes.data_as(P(C.c_int32)), C.byref(cur),
                               nom_pod.ctypes.data_as(P(C.c_int32)), nom_node.ctypes.data_as(P(C.c_int32)),
                               len(nominations), nom_left.ctypes.data_as(P(C.c_uint8)),
                               st["pv_owner"].ctypes.data_as(P(C.c_int32)), st["claim_node"].ctypes.data_as(P(C.c_int32)),
                               skip.ctypes.data_as(P(C.c_uint8)))
    assert rc == 0, f"oracle rc={rc}"
    st["pv_owner"] = st["pv_owner"][:cluster_struct.n_pvs]
    st["claim_node"] = st["claim_node"][:cluster_struct.n_wclaims]
    st["next_start"] = cur.value
    st["nominations"] = [e for e, keep in zip(nominations, nom_left) if keep]
    st["vol_count"] = st["vol_count"][:cluster_struct.n_vol_rows, :n_nodes]
    st["vol_attached"] = st["vol_attached"][:cluster_struct.n_vol_keys, :n_nodes]
    return chosen[:n_pods], res, st
