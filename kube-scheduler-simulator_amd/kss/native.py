"""ctypes binding of libkss.so (include/kss.h).

The HIP library is the only compute path: importing this module fails loudly if
the shared object is missing, and every device call raises ``KssError`` with
the library's own message on failure.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi

# KSS_LIB=dbg selects the bounds-checked diagnostic build (make -C csrc debug), KSS_LIB=<tag>
# an experiment build (make -C csrc exp EXP=<tag> EXP_FLAGS=...)
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        f"libkss_{os.environ['KSS_LIB']}.so" if os.environ.get("KSS_LIB", "base") != "base"
                        else "libkss.so")
P = C.POINTER


class KssError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(f"libkss error {rc}: {msg}")
        self.rc = rc


_lib: Optional[C.CDLL] = None

# (name, restype, argtypes) for every entry point declared in include/kss.h
SIGNATURES = [
    ("kss_abi_version", C.c_int, []),
    ("kss_last_error", C.c_char_p, []),
    ("kss_set_option", C.c_int, [C.c_char_p, C.c_int64]),
    ("kss_get_option", C.c_int, [C.c_char_p, P(C.c_int64)]),
    ("kss_reset_options", C.c_int, []),
    ("kss_set_stamps_file", C.c_int, [C.c_char_p]),
    ("kss_abi_sizes", C.c_int, [P(C.c_int32), C.c_int32]),
    ("kss_default_profile", None, [P(abi.Profile)]),
    ("kss_create", C.c_void_p, [P(abi.Config), P(abi.Profile)]),
    ("kss_destroy", None, [C.c_void_p]),
    ("kss_load_cluster", C.c_int, [C.c_void_p, P(abi.Cluster)]),
    ("kss_apply_node_delta", C.c_int, [C.c_void_p, P(C.c_int32), C.c_int32, P(C.c_int64), P(C.c_int64), P(C.c_int32)]),
    ("kss_apply_count_delta", C.c_int, [C.c_void_p, P(C.c_int32), P(C.c_int32), P(C.c_int32), C.c_int32, C.c_int32]),
    ("kss_read_node_state", C.c_int, [C.c_void_p, P(C.c_int64), P(C.c_int64), P(C.c_int32), P(C.c_int32), P(C.c_int32)]),
    ("kss_read_port_state", C.c_int, [C.c_void_p, P(C.c_uint64)]),
    ("kss_read_volume_state", C.c_int, [C.c_void_p, P(C.c_int32), P(C.c_int32)]),
    ("kss_read_binding_state", C.c_int, [C.c_void_p, P(C.c_int32), P(C.c_int32)]),
    ("kss_apply_volume_delta", C.c_int, [C.c_void_p, P(C.c_int32), P(C.c_int32), P(C.c_int32), C.c_int32, C.c_int32]),
    ("kss_apply_port_delta", C.c_int, [C.c_void_p, P(C.c_int32), C.c_int32, P(C.c_uint64)]),
    ("kss_eval_pod", C.c_int, [C.c_void_p, P(abi.PodSet), C.c_int32, P(abi.PodResult)]),
    ("kss_eval_pod_view", C.c_int, [C.c_void_p, P(abi.PodSet), C.c_int32, C.c_uint32, P(abi.PodView)]),
    ("kss_service_start", C.c_int, [C.c_void_p]),
    ("kss_service_stop", C.c_int, [C.c_void_p]),
    ("kss_service_eval", C.c_int, [C.c_void_p, C.c_int32, C.c_uint32, P(abi.PodView)]),
    ("kss_service_eval_compact", C.c_int, [C.c_void_p, C.c_int32, C.c_uint32, P(abi.PodCView)]),
    ("kss_service_commit", C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
    ("kss_service_rollback", C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
    ("kss_service_mode", C.c_int, [C.c_void_p, P(C.c_int32)]),
    ("kss_service_stamps", C.c_int, [C.c_void_p, P(C.c_uint64)]),
    ("kss_commit", C.c_int, [C.c_void_p, P(abi.PodSet), C.c_int32, C.c_int32]),
    ("kss_rollback", C.c_int, [C.c_void_p, P(abi.PodSet), C.c_int32, C.c_int32]),
    ("kss_schedule_batch", C.c_int, [C.c_void_p, P(abi.PodSet), C.c_int32, C.c_uint32, P(C.c_int32)]),
    ("kss_fetch_record", C.c_int, [C.c_void_p, C.c_int32, P(abi.PodResult)]),
    ("kss_schedule_scenarios", C.c_int, [C.c_int32, P(abi.Profile), C.c_int32, P(abi.Cluster), P(abi.PodSet),
                                         P(C.c_int32), P(C.c_double)]),
    ("kss_sweep_create", C.c_void_p, [C.c_int32, P(abi.Profile), C.c_int32, P(abi.Cluster), P(abi.PodSet)]),
    ("kss_sweep_run", C.c_int, [C.c_void_p, P(C.c_int32), P(C.c_double)]),
    ("kss_sweep_info", C.c_int, [C.c_void_p, P(C.c_double), P(C.c_int32), P(C.c_int64)]),
    ("kss_sweep_destroy", None, [C.c_void_p]),
    ("kss_last_timing", C.c_int, [C.c_void_p, P(C.c_double), P(C.c_int32)]),
    ("kss_last_loop_timing", C.c_int, [C.c_void_p, P(C.c_double)]),
    ("kss_last_handoff_retries", C.c_int, [C.c_void_p, P(C.c_int32)]),
    ("kss_last_handoff_diag", C.c_int, [C.c_void_p, P(C.c_int32), P(C.c_int64), C.c_int32, P(C.c_int32)]),
    ("kss_last_handoff_status", C.c_int, [C.c_void_p, P(C.c_int32)]),
    ("kss_buffer_map", C.c_int, [C.c_void_p, P(C.c_uint64), P(C.c_uint64), C.c_int32, P(C.c_int32)]),
    ("kss_last_geometry", C.c_int, [C.c_void_p, P(C.c_int32)]),
    ("kss_last_kernel", C.c_int, [C.c_void_p]),
    ("kss_last_xcd_local", C.c_int, [C.c_void_p, P(C.c_int32)]),
    ("kss_device_go_log", C.c_int, [C.c_int32, C.c_void_p, C.c_void_p, C.c_int32]),
    ("kss_plan_podset", C.c_int, [C.POINTER(abi.Cluster), C.POINTER(abi.PodSet), C.c_void_p]),
    ("kss_plan_podset_ex", C.c_int, [C.POINTER(abi.Cluster), C.POINTER(abi.PodSet), C.POINTER(abi.Profile),
                                     C.c_void_p]),
    ("kss_plan_reason", C.c_char_p, [C.c_int32]),
    ("kss_next_start_node_index", C.c_int, [C.c_void_p, P(C.c_int32)]),
    ("kss_set_next_start_node_index", C.c_int, [C.c_void_p, C.c_int32]),
    ("kss_nominate", C.c_int, [C.c_void_p, P(abi.PodSet), C.c_int32, C.c_int32]),
    ("kss_clear_nomination", C.c_int, [C.c_void_p, P(abi.PodSet), C.c_int32]),
    ("kss_nominations", C.c_int, [C.c_void_p, P(C.c_int32), P(C.c_int32), C.c_int32, P(C.c_int32)]),
    ("kss_fetch_meta", C.c_int, [C.c_void_p, C.c_int32, C.c_int32, P(C.c_int64)]),
    ("kss_set_names", C.c_int, [C.c_void_p, P(abi.Names)]),
    ("kss_format_annotations", C.c_int, [C.c_void_p, P(abi.PodResult), C.c_int32, C.c_char_p, C.c_size_t,
                                         P(C.c_size_t)]),
    ("kss_format_annotations_ex", C.c_int, [P(abi.Names), P(abi.Profile), P(abi.PodResult), C.c_int32, C.c_int32,
                                            C.c_int32, C.c_char_p, C.c_size_t, P(C.c_size_t)]),
    ("kss_format_pod_annotations", C.c_int, [C.c_void_p, P(abi.PodSet), C.c_int32, P(abi.PodResult), C.c_int32,
                                             C.c_char_p, C.c_size_t, P(C.c_size_t)]),
    ("kss_format_pod_annotations_ex", C.c_int, [P(abi.Names), P(abi.Profile), P(abi.PodSet), C.c_int32,
                                                P(abi.PodResult), C.c_int32, C.c_int32, C.c_int32, C.c_char_p,
                                                C.c_size_t, P(C.c_size_t)]),
    ("kss_load_bound", C.c_int, [C.c_void_p, P(abi.Boundset)]),
    ("kss_remove_bound", C.c_int, [C.c_void_p, P(C.c_int64), C.c_int32]),
    ("kss_postfilter_pod", C.c_int, [C.c_void_p, P(abi.PodSet), C.c_int32, P(abi.PreemptResult)]),
    ("kss_stage_pods", C.c_int, [C.c_void_p, P(abi.PodSet)]),
    ("kss_run_staged", C.c_int, [C.c_void_p, C.c_int32, C.c_uint32, P(C.c_int32)]),
    ("kss_reset_node_state", C.c_int, [C.c_void_p]),
    ("kss_load_cluster_rows", C.c_int, [C.c_void_p, P(abi.Cluster), C.c_int32, C.c_int32]),
    ("kss_axis_eval", C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p,
                                C.c_void_p, C.c_void_p]),
    ("kss_axis_select", C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("kss_axis_commit", C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
    ("kss_split_config", C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32]),
    ("kss_split_inbox", C.c_int, [C.c_void_p, P(C.c_void_p), P(C.c_size_t), C.c_void_p]),
    ("kss_split_peers", C.c_int, [C.c_void_p, P(C.c_void_p)]),
    ("kss_split_open", C.c_int, [C.c_void_p, C.c_void_p]),
    ("kss_synth_make", C.c_int, [C.c_int32, C.c_uint64, C.c_int32, C.c_int32, P(abi.Synth)]),
    ("kss_synth_free", None, [P(abi.Synth)]),
]


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libkss.so not built at {LIB_PATH} (run __graft_entry__.build()); "
                              "there is no CPU fallback for the device path")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.kss_abi_version() != 5:
            raise ImportError("libkss ABI version mismatch")
        _lib = L
    return _lib


def check(rc: int):
    if rc != 0:
        raise KssError(rc, (lib().kss_last_error() or b"").decode())


def set_option(name: str, value: int):
    """kss_set_option: a process-wide tuning / diagnosis option (the library reads no environment)."""
    check(lib().kss_set_option(name.encode(), int(value)))


def get_option(name: str) -> int:
    v = C.c_int64()
    check(lib().kss_get_option(name.encode(), C.byref(v)))
    return v.value


def reset_options():
    """Every option back to its default, stamps off (kss_reset_options)."""
    check(lib().kss_reset_options())


def set_stamps_file(path: Optional[str]):
    """kss_set_stamps_file: phase stamps of contexts created afterwards go to `path` (None: off)."""
    check(lib().kss_set_stamps_file(path.encode() if path else None))


class options:
    """with native.options(shards=9, static_bytes=...): set, then restore the previous values."""

    def __init__(self, **kw):
        self.kw = kw
        self.old = {}

    def __enter__(self):
        for k, v in self.kw.items():
            self.old[k] = get_option(k)
            set_option(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.old.items():
            set_option(k, v)
        return False


class PodView:
    """kss_pod_view as numpy arrays aliasing the library's staging (read-only, zero-copy);
    unrequested fields are None.  Copy what must outlive the next call on the context."""

    def __init__(self, v: "abi.PodView", n_nodes: int):
        N = n_nodes

        def arr(ptr, shape):
            if not ptr:
                return None
            a = np.ctypeslib.as_array(ptr, shape=shape)
            a.flags.writeable = False
            return a

        self.fail_plugin = arr(v.fail_plugin, (N,))
        self.fail_detail = arr(v.fail_detail, (N,))
        self.raw = arr(v.raw, (abi.KSS_NSCORE, N))
        self.norm = arr(v.norm, (abi.KSS_NSCORE, N))
        self.total = arr(v.total, (N,))
        self.n_feasible, self.chosen, self.best_total = v.n_feasible, v.chosen, v.best_total
        self.scored, self.status = v.scored, v.status


class PodCView(PodView):
    """kss_pod_cview as read-only numpy views: raw / total int32, norm uint8 (or, when a value
    did not fit, is_wide and the full record's int64 views)."""

    def __init__(self, v: "abi.PodCView", n_nodes: int):
        self.is_wide = bool(v.is_wide)
        if self.is_wide:
            super().__init__(v.wide, n_nodes)
            return
        N = n_nodes

        def arr(ptr, shape):
            if not ptr:
                return None
            a = np.ctypeslib.as_array(ptr, shape=shape)
            a.flags.writeable = False
            return a

        self.fail_plugin = arr(v.fail_plugin, (N,))
        self.fail_detail = arr(v.fail_detail, (N,))
        self.raw = arr(v.raw, (abi.KSS_NSCORE, N))
        self.norm = arr(v.norm, (abi.KSS_NSCORE, N))
        self.total = arr(v.total, (N,))
        self.n_feasible, self.chosen, self.best_total = v.n_feasible, v.chosen, v.best_total
        self.scored, self.status = v.scored, v.status


class PodResult:
    """Host arrays for one pod's result (kss_pod_result).  `fields` limits which per-node
    arrays the library fills (the others are passed as NULL and not copied back): e.g.
    ("fail_plugin", "fail_detail", "total") for a plugin that answers Filter from the
    verdicts and Score from the weighted totals."""

    ALL = ("fail_plugin", "fail_detail", "raw", "norm", "total")

    def __init__(self, n_nodes: int, fields=ALL):
        N = max(n_nodes, 1)
        self.n_nodes = n_nodes
        self.fail_plugin = np.zeros(N, np.uint8)
        self.fail_detail = np.zeros(N, np.uint16)
        self.raw = np.zeros((abi.KSS_NSCORE, N), np.int64)
        self.norm = np.zeros((abi.KSS_NSCORE, N), np.int64)
        self.total = np.zeros(N, np.int64)
        s = abi.PodResult()
        s.fail_plugin = self.fail_plugin.ctypes.data_as(P(C.c_uint8))
        s.fail_detail = self.fail_detail.ctypes.data_as(P(C.c_uint16))
        s.raw = self.raw.ctypes.data_as(P(C.c_int64))
        s.norm = self.norm.ctypes.data_as(P(C.c_int64))
        s.total = self.total.ctypes.data_as(P(C.c_int64))
        for f in self.ALL:
            if f not in fields:
                setattr(s, f, None)
        self.s = s

    @property
    def chosen(self):
        return self.s.chosen

    @property
    def n_feasible(self):
        return self.s.n_feasible

    @property
    def scored(self):
        return self.s.scored

    @property
    def status(self):
        return self.s.status


def _cstrs(items: Sequence[str]):
    arr = (C.c_char_p * max(len(items), 1))()
    for i, s in enumerate(items):
        arr[i] = s.encode()
    return arr


def make_names(node_names, taints, scalars, messages=()):
    """Build a kss_names struct; returns (struct, keepalive).  messages: the podset's status
    messages (CompiledPods.messages: VolumeBinding PreFilter, VolumeZone errors)."""
    nn = _cstrs(node_names)
    tk = _cstrs([t[0] for t in taints])
    tv = _cstrs([t[1] for t in taints])
    sc = _cstrs(scalars)
    ms = _cstrs(list(messages))
    n = abi.Names(C.cast(nn, P(C.c_char_p)), C.cast(tk, P(C.c_char_p)), C.cast(tv, P(C.c_char_p)),
                  C.cast(sc, P(C.c_char_p)), len(messages), 0, C.cast(ms, P(C.c_char_p)))
    return n, (nn, tk, tv, sc, ms)


def parse_annotations(buf: bytes) -> Dict[str, str]:
    parts = buf.split(b"\0")
    out = {}
    i = 0
    while i + 1 < len(parts) and parts[i]:
        out[parts[i].decode()] = parts[i + 1].decode()
        i += 2
    return out


def _format(call) -> Dict[str, str]:
    need = C.c_size_t(0)
    check(call(None, 0, C.byref(need)))
    buf = C.create_string_buffer(need.value)
    check(call(buf, need.value, C.byref(need)))
    return parse_annotations(buf.raw[:need.value])


def format_annotations_ex(names_struct, profile, result: PodResult, n_nodes, n_taints, n_scalar,
                          podset_struct: Optional[abi.PodSet] = None, pod_index: int = -1) -> Dict[str, str]:
    """Context-free formatting; with (podset_struct, pod_index) the pod's NodeAffinity
    PreFilterResult is recorded too (store.go:522-534)."""
    L = lib()
    if podset_struct is None:
        return _format(lambda b, c, n: L.kss_format_annotations_ex(C.byref(names_struct), C.byref(profile),
                                                                   C.byref(result.s), n_nodes, n_taints, n_scalar,
                                                                   b, c, n))
    return _format(lambda b, c, n: L.kss_format_pod_annotations_ex(
        C.byref(names_struct), C.byref(profile), C.byref(podset_struct), pod_index, C.byref(result.s), n_nodes,
        n_taints, n_scalar, b, c, n))


class Context:
    """One device context (kss_ctx): a loaded cluster snapshot on one GPU."""

    def __init__(self, profile: Optional[abi.Profile] = None, device: int = 0, max_pods_record: int = 0,
                 class_capacity: int = 0, term_capacity: int = 0):
        L = lib()
        self.profile = profile if profile is not None else abi.default_profile()
        cfg = abi.Config(device, max_pods_record, class_capacity, term_capacity)
        h = L.kss_create(C.byref(cfg), C.byref(self.profile))
        if not h:
            raise KssError(-1, (L.kss_last_error() or b"").decode())
        self.h = C.c_void_p(h)
        self.n_nodes = 0
        self._keep = []

    def close(self):
        if getattr(self, "h", None):
            lib().kss_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load(self, cluster_struct: abi.Cluster, names=None):
        check(lib().kss_load_cluster(self.h, C.byref(cluster_struct)))
        self.n_nodes = cluster_struct.n_nodes
        self.n_classes = cluster_struct.n_classes
        self.n_terms = cluster_struct.n_terms
        self.n_taints = cluster_struct.n_taints
        self.n_scalar = cluster_struct.n_scalar
        self.n_vol_rows = cluster_struct.n_vol_rows
        self.n_vol_keys = cluster_struct.n_vol_keys
        self.n_pvs = cluster_struct.n_pvs
        self.n_wclaims = cluster_struct.n_wclaims
        if names is not None:
            st, keep = names
            self._keep = keep
            check(lib().kss_set_names(self.h, C.byref(st)))

    def load_rows(self, cluster_struct: abi.Cluster, lo: int, hi: int):
        """Load canonical rows [lo, hi) of the cluster (node-axis sharding; node_base = lo)."""
        check(lib().kss_load_cluster_rows(self.h, C.byref(cluster_struct), lo, hi))
        self.n_nodes = hi - lo
        self.n_classes = cluster_struct.n_classes
        self.n_terms = cluster_struct.n_terms
        self.n_taints = cluster_struct.n_taints
        self.n_scalar = cluster_struct.n_scalar

    # node-axis launches (kss.h): device pointers and a hipStream_t handle as ints
    def axis_eval(self, i: int, stats_ptr: int, prev_key_ptr: int, prev_gathered_ptr: int, world: int,
                  key_zero_ptr: int, chosen_ptr: int, stream: int):
        check(lib().kss_axis_eval(self.h, i, stats_ptr, prev_key_ptr or None, prev_gathered_ptr or None, world,
                                  key_zero_ptr, chosen_ptr, stream))

    def axis_select(self, gathered_ptr: int, world: int, key_ptr: int, stats_zero_ptr: int, stream: int):
        check(lib().kss_axis_select(self.h, gathered_ptr, world, key_ptr, stats_zero_ptr, stream))

    def axis_commit(self, i: int, key_ptr: int, gathered_ptr: int, world: int, chosen_ptr: int, stream: int):
        check(lib().kss_axis_commit(self.h, i, key_ptr, gathered_ptr, world, chosen_ptr, stream))

    # split grid (kss.h kss_split_*): this context runs one part of a grid spread over GPUs
    def split_config(self, n_parts: int, part: int, shards_per_part: int):
        check(lib().kss_split_config(self.h, n_parts, part, shards_per_part))

    def split_inbox(self, with_handle: bool = False):
        """(device pointer, bytes, IPC handle bytes or None) of this part's exchange inbox."""
        ptr, nb = C.c_void_p(0), C.c_size_t(0)
        h = C.create_string_buffer(abi.KSS_IPC_HANDLE_BYTES) if with_handle else None
        check(lib().kss_split_inbox(self.h, C.byref(ptr), C.byref(nb), h))
        return ptr.value, nb.value, (h.raw if h is not None else None)

    def split_peers(self, inboxes: Sequence[int]):
        arr = (C.c_void_p * len(inboxes))(*inboxes)
        check(lib().kss_split_peers(self.h, arr))

    def split_open(self, handles: Sequence[bytes]):
        buf = C.create_string_buffer(b"".join(handles), abi.KSS_IPC_HANDLE_BYTES * len(handles))
        check(lib().kss_split_open(self.h, buf))

    def schedule_batch(self, podset_struct: abi.PodSet, n: int, record=False, flags=0) -> np.ndarray:
        chosen = np.full(max(n, 1), -2, np.int32)
        fl = flags | (abi.KSS_SCHED_RECORD if record else 0)
        check(lib().kss_schedule_batch(self.h, C.byref(podset_struct), n, fl, chosen.ctypes.data_as(P(C.c_int32))))
        return chosen[:n]

    def stage(self, podset_struct: abi.PodSet):
        check(lib().kss_stage_pods(self.h, C.byref(podset_struct)))

    def run_staged(self, n: int, record=False, out: Optional[np.ndarray] = None, flags: int = 0) -> np.ndarray:
        chosen = out if out is not None else np.full(max(n, 1), -2, np.int32)
        fl = (abi.KSS_SCHED_RECORD if record else 0) | flags
        check(lib().kss_run_staged(self.h, n, fl, chosen.ctypes.data_as(P(C.c_int32))))
        return chosen[:n]

    def reset(self):
        check(lib().kss_reset_node_state(self.h))

    def eval_pod(self, podset_struct: abi.PodSet, i: int, out: Optional[PodResult] = None) -> PodResult:
        """kss_eval_pod into `out` (a reusable PodResult, as a plugin keeps its buffers) or a new one."""
        r = out if out is not None else PodResult(self.n_nodes)
        check(lib().kss_eval_pod(self.h, C.byref(podset_struct), i, C.byref(r.s)))
        return r

    def eval_pod_view(self, podset_struct: abi.PodSet, i: int, fields: int = abi.KSS_FIELD_ALL) -> "PodView":
        """kss_eval_pod_view: the result's arrays as read-only numpy views of the context's
        pinned read-back staging (no host copy); valid until the next call on this context."""
        v = abi.PodView()
        check(lib().kss_eval_pod_view(self.h, C.byref(podset_struct), i, fields, C.byref(v)))
        return PodView(v, self.n_nodes)

    # the per-pod service grid (kss_service_*): staged pods by index, no launch per call
    def service_start(self):
        check(lib().kss_service_start(self.h))

    def service_mode(self) -> int:
        """1: the k_simple-shaped service evaluation, 0: the general chain, -1: not started."""
        v = C.c_int32(-1)
        check(lib().kss_service_mode(self.h, C.byref(v)))
        return v.value

    def service_stop(self):
        check(lib().kss_service_stop(self.h))

    def service_eval(self, i: int, fields: int = abi.KSS_FIELD_ALL, view: Optional[abi.PodView] = None) -> "PodView":
        """kss_service_eval of staged pod i: the record as read-only views of the pinned
        service buffer (valid until the next service call)."""
        v = view if view is not None else abi.PodView()
        check(lib().kss_service_eval(self.h, i, fields, C.byref(v)))
        return PodView(v, self.n_nodes)

    def service_eval_compact(self, i: int, fields: int = abi.KSS_FIELD_ALL,
                             view: Optional[abi.PodCView] = None) -> "PodCView":
        """kss_service_eval_compact of staged pod i: the record with the scores narrowed on the
        device (int32 raw / total, uint8 normalised), or the full record when is_wide."""
        v = view if view is not None else abi.PodCView()
        check(lib().kss_service_eval_compact(self.h, i, fields, C.byref(v)))
        return PodCView(v, self.n_nodes)

    def service_commit(self, i: int, node: int):
        check(lib().kss_service_commit(self.h, i, node))

    def service_rollback(self, i: int, node: int):
        check(lib().kss_service_rollback(self.h, i, node))

    def service_stamps(self):
        """Shard 0's clock (100 MHz ticks) at command taken / relayed / pod done / record
        visible / record stores issued (before the system fence), and for the k_simple-shaped
        evaluation node pass / statistics exchange / record stores before the key exchange."""
        out = (C.c_uint64 * 8)()
        check(lib().kss_service_stamps(self.h, out))
        return list(out)

    def load_bound(self, boundset_struct: abi.Boundset):
        """The bound pods the PostFilter dry run may evict (CompiledCluster.as_boundset())."""
        check(lib().kss_load_bound(self.h, C.byref(boundset_struct)))

    def remove_bound(self, ids):
        """The informer's RemovePod for bound-table pods (victims deleted after a PostFilter):
        kss_remove_bound."""
        arr = np.array(list(ids) or [0], dtype=np.int64)
        check(lib().kss_remove_bound(self.h, arr.ctypes.data_as(P(C.c_int64)), len(ids)))

    def postfilter_pod(self, podset_struct: abi.PodSet, i: int, victims_cap: int = 1024) -> dict:
        """DefaultPreemption PostFilter dry run of pod i on the current snapshot: status
        (KSS_PREEMPT_*), the nominated node (-1), the victims' bound ids in eviction order and
        the pickOneNodeForPreemption criteria of the nominated node."""
        vic = np.zeros(max(victims_cap, 1), np.int64)
        r = abi.PreemptResult()
        r.victims_cap = victims_cap
        r.victims = vic.ctypes.data_as(P(C.c_int64))
        check(lib().kss_postfilter_pod(self.h, C.byref(podset_struct), i, C.byref(r)))
        return dict(status=r.status, nominated=r.nominated, n_potential=r.n_potential, n_candidates=r.n_candidates,
                    victims=[int(v) for v in vic[:min(r.n_victims, victims_cap)]], n_victims=r.n_victims,
                    highest_priority=r.highest_priority, sum_priority=r.sum_priority, earliest_start=r.earliest_start)

    def fetch_record(self, i: int) -> PodResult:
        r = PodResult(self.n_nodes)
        check(lib().kss_fetch_record(self.h, i, C.byref(r.s)))
        return r

    def commit(self, podset_struct, i, node):
        check(lib().kss_commit(self.h, C.byref(podset_struct), i, node))

    def rollback(self, podset_struct, i, node):
        check(lib().kss_rollback(self.h, C.byref(podset_struct), i, node))

    def apply_node_delta(self, idx, requested, nonzero, pod_count):
        """Overwrite node rows idx (kss_apply_node_delta): requested [n][KSS_NRES], nonzero [n][2]."""
        idx = np.ascontiguousarray(idx, np.int32)
        req = np.ascontiguousarray(requested, np.int64).reshape(len(idx), abi.KSS_NRES)
        nz = np.ascontiguousarray(nonzero, np.int64).reshape(len(idx), 2)
        pc = np.ascontiguousarray(pod_count, np.int32)
        check(lib().kss_apply_node_delta(self.h, idx.ctypes.data_as(P(C.c_int32)), len(idx),
                                         req.ctypes.data_as(P(C.c_int64)), nz.ctypes.data_as(P(C.c_int64)),
                                         pc.ctypes.data_as(P(C.c_int32))))

    def apply_count_delta(self, node, row, value, overwrite=False):
        """class / term counts (kss_apply_count_delta): row < n_classes is a class row, else a
        term row (row - n_classes); add value, or overwrite with it."""
        node = np.ascontiguousarray(node, np.int32)
        row = np.ascontiguousarray(row, np.int32)
        value = np.ascontiguousarray(value, np.int32)
        check(lib().kss_apply_count_delta(self.h, node.ctypes.data_as(P(C.c_int32)), row.ctypes.data_as(P(C.c_int32)),
                                          value.ctypes.data_as(P(C.c_int32)), len(node), 1 if overwrite else 0))

    def node_state(self):
        N = max(self.n_nodes, 1)
        st = dict(requested=np.zeros((abi.KSS_NRES, N), np.int64), nonzero=np.zeros((2, N), np.int64),
                  pod_count=np.zeros(N, np.int32), class_count=np.zeros((max(self.n_classes, 1), N), np.int32),
                  term_count=np.zeros((max(self.n_terms, 1), N), np.int32))
        check(lib().kss_read_node_state(self.h, st["requested"].ctypes.data_as(P(C.c_int64)),
                                        st["nonzero"].ctypes.data_as(P(C.c_int64)),
                                        st["pod_count"].ctypes.data_as(P(C.c_int32)),
                                        st["class_count"].ctypes.data_as(P(C.c_int32)),
                                        st["term_count"].ctypes.data_as(P(C.c_int32))))
        return st

    def port_state(self) -> np.ndarray:
        """NodeInfo.UsedPorts of every row as port-dictionary bits (kss_read_port_state)."""
        out = np.zeros(max(self.n_nodes, 1), np.uint64)
        check(lib().kss_read_port_state(self.h, out.ctypes.data_as(P(C.c_uint64))))
        return out[:self.n_nodes]

    def apply_port_delta(self, idx, used):
        """Overwrite the UsedPorts bits of rows idx (kss_apply_port_delta)."""
        idx = np.ascontiguousarray(idx, np.int32)
        used = np.ascontiguousarray(used, np.uint64)
        check(lib().kss_apply_port_delta(self.h, idx.ctypes.data_as(P(C.c_int32)), len(idx),
                                         used.ctypes.data_as(P(C.c_uint64))))

    def volume_state(self):
        """(vol_count [rows][N], vol_attached [keys][N]) read back (kss_read_volume_state)."""
        N = max(self.n_nodes, 1)
        vc = np.zeros((max(self.n_vol_rows, 1), N), np.int32)
        va = np.zeros((max(self.n_vol_keys, 1), N), np.int32)
        check(lib().kss_read_volume_state(self.h, vc.ctypes.data_as(P(C.c_int32)), va.ctypes.data_as(P(C.c_int32))))
        return vc[:self.n_vol_rows, :self.n_nodes], va[:self.n_vol_keys, :self.n_nodes]

    def binding_state(self):
        """(pv_owner [n_pvs], claim_node [n_wclaims]): the binder's assume cache (kss_read_binding_state)."""
        po = np.zeros(max(self.n_pvs, 1), np.int32)
        cn = np.zeros(max(self.n_wclaims, 1), np.int32)
        check(lib().kss_read_binding_state(self.h, po.ctypes.data_as(P(C.c_int32)), cn.ctypes.data_as(P(C.c_int32))))
        return po[:self.n_pvs], cn[:self.n_wclaims]

    def apply_volume_delta(self, node, row, value, overwrite=False):
        """vol_count / vol_attached sync (kss_apply_volume_delta): row r < n_vol_rows is a vol_count
        row, r >= n_vol_rows the vol_attached key r - n_vol_rows."""
        node = np.ascontiguousarray(node, np.int32)
        row = np.ascontiguousarray(row, np.int32)
        value = np.ascontiguousarray(value, np.int32)
        check(lib().kss_apply_volume_delta(self.h, node.ctypes.data_as(P(C.c_int32)), row.ctypes.data_as(P(C.c_int32)),
                                           value.ctypes.data_as(P(C.c_int32)), len(node), 1 if overwrite else 0))

    def last_timing(self):
        ms = C.c_double(0)
        n = C.c_int32(0)
        check(lib().kss_last_timing(self.h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def last_loop_ms(self) -> float:
        """Device ms of the sequential-loop kernel(s) alone in the last batch."""
        ms = C.c_double(0)
        check(lib().kss_last_loop_timing(self.h, C.byref(ms)))
        return ms.value

    def last_handoff_retries(self) -> int:
        """Prologue loads of node state the last run repeated (kss_last_handoff_retries)."""
        n = C.c_int32(0)
        check(lib().kss_last_handoff_retries(self.h, C.byref(n)))
        return n.value

    def next_start_node_index(self) -> int:
        """nextStartNodeIndex (kss_next_start_node_index)."""
        v = C.c_int32(0)
        check(lib().kss_next_start_node_index(self.h, C.byref(v)))
        return v.value

    def set_next_start_node_index(self, v: int):
        check(lib().kss_set_next_start_node_index(self.h, int(v)))

    def nominate(self, ps, i: int, node: int):
        """PodNominator.AddNominatedPod of ps.pods[i] on global node `node` (kss_nominate)."""
        check(lib().kss_nominate(self.h, C.byref(ps), int(i), int(node)))

    def clear_nomination(self, ps, i: int):
        """DeleteNominatedPodIfExists of ps.pods[i] (kss_clear_nomination)."""
        check(lib().kss_clear_nomination(self.h, C.byref(ps), int(i)))

    def nominations(self) -> List[Tuple[int, int]]:
        """[(pod, global node)] in AddNominatedPod order (kss_nominations): pod = the podset index
        of a pod without uid (identity -1 - index), else its uid."""
        pods = (C.c_int32 * 64)()
        nodes = (C.c_int32 * 64)()
        n = C.c_int32(0)
        check(lib().kss_nominations(self.h, pods, nodes, 64, C.byref(n)))
        return [(-1 - int(pods[i]) if pods[i] < 0 else int(pods[i]), int(nodes[i])) for i in range(min(n.value, 64))]

    def last_handoff_status(self) -> Dict[str, int]:
        """{reloads, shadow, final} of the last k_spread run (kss_last_handoff_status): all 0
        when every hand-off between chunk launches and the last write-back were clean."""
        out = (C.c_int32 * 3)()
        check(lib().kss_last_handoff_status(self.h, out))
        return {"reloads": out[0], "shadow": out[1], "final": out[2]}

    def last_handoff_diag(self):
        """(shadow recoveries, [entry dicts]) of the last run (kss_last_handoff_diag)."""
        rec, n = C.c_int32(0), C.c_int32(0)
        W = 10  # KSS_HANDOFF_DIAG_WORDS
        buf = (C.c_int64 * (64 * W))()
        check(lib().kss_last_handoff_diag(self.h, C.byref(rec), buf, 64, C.byref(n)))
        out = []
        for i in range(min(n.value, 64)):
            e = buf[W * i:W * i + W]
            out.append({"shard": e[0] & 0xFFFFFFFF, "xcc_load": (e[0] >> 32) & 0xFF, "xcc_store": (e[0] >> 40) & 0xFF,
                        "array": e[1], "node": e[2], "state": e[3], "atomic": e[4], "nontemporal": e[5],
                        "shadow": e[6], "tag": e[7], "addr": e[8] & 0xFFFFFFFFFFFFFFFF, "t": e[9]})
        return rec.value, out

    BUFFER_NAMES = ("cluster", "pristine", "pods", "tmp_pods", "slot", "meta", "chosen", "job", "gran", "err", "ck",
                    "stamps", "spods", "stat", "gpods", "res", "delta", "axis_cv", "bound", "pre", "split_inbox")

    def buffer_map(self):
        """{name: (device base, bytes)} of the context's device buffers (kss_buffer_map)."""
        base, size, n = (C.c_uint64 * 32)(), (C.c_uint64 * 32)(), C.c_int32(0)
        check(lib().kss_buffer_map(self.h, base, size, 32, C.byref(n)))
        return {nm: (base[i], size[i]) for i, nm in enumerate(self.BUFFER_NAMES[:n.value])}

    def last_geometry(self):
        out = (C.c_int32 * 3)()
        check(lib().kss_last_geometry(self.h, out))
        return {"shards": out[0], "threads": out[1], "nodes_per_lane": out[2]}

    def last_xcd_local(self) -> Dict[str, int]:
        """{used, fallbacks} of the last run's XCD-local k_simple grid (kss_last_xcd_local)."""
        out = (C.c_int32 * 2)()
        check(lib().kss_last_xcd_local(self.h, out))
        return {"used": out[0], "fallbacks": out[1]}

    def last_kernel(self) -> str:
        k = lib().kss_last_kernel(self.h)
        if k < 0:
            check(k)
        return {1: "k_simple", 2: "k_spread", 3: "k_preempt"}.get(k, "k_schedule")

    def fetch_meta(self, n: int, first: int = 0) -> np.ndarray:
        """(n, 5) int64: chosen, n_feasible, scored, status, best_total of pods [first, first+n)."""
        out = np.zeros((max(n, 1), 5), np.int64)
        check(lib().kss_fetch_meta(self.h, first, n, out.ctypes.data_as(P(C.c_int64))))
        return out[:n]

    def format_annotations(self, result: PodResult, podset_struct: Optional[abi.PodSet] = None,
                           pod_index: int = -1) -> Dict[str, str]:
        """store.go GetStoredResult for one result; pass the pod's podset and index to have its
        NodeAffinity PreFilterResult recorded (store.go:522-534)."""
        L = lib()
        if podset_struct is None:
            return _format(lambda b, c, n: L.kss_format_annotations(self.h, C.byref(result.s), self.n_nodes, b, c, n))
        return _format(lambda b, c, n: L.kss_format_pod_annotations(self.h, C.byref(podset_struct), pod_index,
                                                                    C.byref(result.s), self.n_nodes, b, c, n))


class Synth:
    """A C++-generated synthetic cluster (kss_synth_make); owns its arrays until close()."""

    def __init__(self, config: int, seed: int = 0, n_nodes: int = 0, n_pods: int = 0):
        self.s = abi.Synth()
        check(lib().kss_synth_make(config, seed, n_nodes, n_pods, C.byref(self.s)))
        self.cluster = self.s.cluster
        self.pods = self.s.pods

    @property
    def n_nodes(self):
        return self.s.cluster.n_nodes

    @property
    def n_pods(self):
        return self.s.pods.n_pods

    def close(self):
        if self.s.owner:
            lib().kss_synth_free(C.byref(self.s))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def schedule_scenarios(profile, clusters: List[abi.Cluster], podsets: List[abi.PodSet], device=0):
    n = len(clusters)
    carr = (abi.Cluster * max(n, 1))(*clusters)
    parr = (abi.PodSet * max(n, 1))(*podsets)
    total = sum(p.n_pods for p in podsets)
    chosen = np.full(max(total, 1), -2, np.int32)
    ms = C.c_double(0)
    check(lib().kss_schedule_scenarios(device, C.byref(profile), n, carr, parr, chosen.ctypes.data_as(P(C.c_int32)),
                                       C.byref(ms)))
    return chosen[:total], ms.value


class Sweep:
    """A resident what-if sweep (kss_sweep): every scenario staged once, run many times."""

    def __init__(self, profile, clusters: List[abi.Cluster], podsets: List[abi.PodSet], device=0):
        L = lib()
        n = len(clusters)
        carr = (abi.Cluster * max(n, 1))(*clusters)
        parr = (abi.PodSet * max(n, 1))(*podsets)
        h = L.kss_sweep_create(device, C.byref(profile), n, carr, parr)
        if not h:
            raise KssError(-1, (L.kss_last_error() or b"").decode())
        self.h = C.c_void_p(h)
        self.total = sum(p.n_pods for p in podsets)

    def run(self):
        """(chosen [sum n_pods], device ms of reset + launches)."""
        chosen = np.full(max(self.total, 1), -2, np.int32)
        ms = C.c_double(0)
        check(lib().kss_sweep_run(self.h, chosen.ctypes.data_as(P(C.c_int32)), C.byref(ms)))
        return chosen[:self.total], ms.value

    def info(self):
        ms, k, b = C.c_double(0), C.c_int32(0), C.c_int64(0)
        check(lib().kss_sweep_info(self.h, C.byref(ms), C.byref(k), C.byref(b)))
        return {"stage_ms": ms.value, "kernel": "k_simple" if k.value == 1 else "k_schedule", "upload_bytes": b.value}

    def close(self):
        if getattr(self, "h", None):
            lib().kss_sweep_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def device_go_log(x, device: int = 0) -> np.ndarray:
    """Go math.Log of every x as k_spread evaluates it on the device (kss_device_go_log)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    check(lib().kss_device_go_log(device, x.ctypes.data, y.ctypes.data, len(x)))
    return y


def plan_podset(cluster: abi.Cluster, podset: abi.PodSet, profile: Optional[abi.Profile] = None) -> dict:
    """Host-only: the sequential-loop kernel a staged batch can take (kss_plan_podset; with the
    profile: kss_plan_podset_ex, which also sees percentageOfNodesToScore and scored extended
    resources)."""
    out = (C.c_int32 * 3)()
    if profile is None:
        check(lib().kss_plan_podset(C.byref(cluster), C.byref(podset), out))
    else:
        check(lib().kss_plan_podset_ex(C.byref(cluster), C.byref(podset), C.byref(profile), out))
    kernel = {1: "k_simple", 2: "k_spread"}.get(out[0], "k_schedule")
    return {"kernel": kernel, "pod": out[1], "reason": lib().kss_plan_reason(out[2]).decode()}
