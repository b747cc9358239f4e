"""ctypes binding of libupe_gpu.so (the C ABI of include/upe_gpu.h).

This is host plumbing above the C ABI, mirroring the reference worker's interface: a
`GpuWorker` plays the role of one worker_t (reference include/worker.h:23-69) — it owns the
counters, rule_stats and L1 neighbour caches, borrows a rule table and neighbour-table snapshots,
and processes batches.  Device buffers may be torch tensors (data_ptr) or raw device pointers;
streams are hipStream_t handles (torch.cuda.current_stream().cuda_stream).

There is no CPU fallback: if libupe_gpu.so is missing or fails to load, importing this module
raises.  Build it with `make -C upe_amd/csrc` (or __graft_entry__.build()).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .layout import (ARP_DTYPE, BATCH_INFO_DTYPE, COUNTERS_DTYPE, FLOW_KEY_DTYPE, L1_DTYPE,
                     LAUNCH_INFO_DTYPE, NDP_DTYPE, RULE_DTYPE, RULE_INDEX_INFO_DTYPE,
                     RULE_STAT_DTYPE)

LIB_PATH = os.environ.get("UPE_GPU_LIB_DIAG") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "libupe_gpu.so")  # override: diagnostic builds only


# launch_info variant bits (upe_gpu.hip classify_var)
VAR_NOLB = 8    # the kernel without look-back
VAR_RING = 16   # a ring launch whose batches are stamped
VAR_HOST = 32   # a host path's launch (mapped host memory, host round trip)
VAR_FAM = 64    # a linear-scan table past 64 rules, scanned through per-family rule lists
VAR_GLB = 128   # the same scanned whole (a family's list is a single catch-all)
VAR_TREE = 192  # the same matched through the decision tree over the family lists
VAR_SCAN = 192  # the bits of the three above


# upe_tx_batch_fn: int (*)(void *user, const uint8_t *const *frames, const size_t *lens, int count)
TX_BATCH_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p,
                               ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                               ctypes.c_int)


# upe_worker_ops_t callbacks (include/upe_gpu.h): the callees of the reference's worker_main
_VP, _U8P = ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8)
POP_FN = ctypes.CFUNCTYPE(ctypes.c_uint, _VP, ctypes.POINTER(_VP), ctypes.c_uint)
STOP_FN = ctypes.CFUNCTYPE(ctypes.c_int, _VP)
DATA_FN = ctypes.CFUNCTYPE(_VP, _VP, _VP)
LEN_FN = ctypes.CFUNCTYPE(ctypes.c_size_t, _VP, _VP)
FREE_FN = ctypes.CFUNCTYPE(None, _VP, _VP)
TX_SEND_FN = ctypes.CFUNCTYPE(ctypes.c_int, _VP, _VP, ctypes.c_size_t)
ARP_UPDATE_FN = ctypes.CFUNCTYPE(None, _VP, ctypes.c_uint32, _U8P)
NDP_UPDATE_FN = ctypes.CFUNCTYPE(None, _VP, _U8P, _U8P)
CTX_FN = ctypes.CFUNCTYPE(ctypes.c_int, _VP, _VP)
POLL_FN = ctypes.CFUNCTYPE(ctypes.c_int, _VP)
PUBLISH_FN = ctypes.CFUNCTYPE(None, _VP, _VP, _VP)
FREE_BURST_FN = ctypes.CFUNCTYPE(None, _VP, _VP, ctypes.c_uint)


class WorkerOps(ctypes.Structure):
    """upe_worker_ops_t."""
    _fields_ = [("pop_burst", POP_FN), ("stop", STOP_FN), ("data", DATA_FN), ("len", LEN_FN),
                ("free_buf", FREE_FN), ("tx_send", TX_SEND_FN), ("tx_send_batch", TX_BATCH_FN),
                ("arp_update", ARP_UPDATE_FN), ("ndp_update", NDP_UPDATE_FN),
                ("load_neigh", CTX_FN), ("poll", POLL_FN), ("sync", CTX_FN),
                ("publish", PUBLISH_FN), ("free_burst", FREE_BURST_FN)]


class WorkerCfg(ctypes.Structure):
    """upe_worker_cfg_t."""
    _fields_ = [("batch", ctypes.c_size_t), ("burst", ctypes.c_uint), ("pool_base", _VP),
                ("idle_ns", ctypes.c_uint), ("pool_bytes", ctypes.c_size_t)]


class QueueBatch(ctypes.Structure):
    """upe_gpu_batch_t (include/upe_gpu.h)."""
    _fields_ = [("frames", ctypes.c_void_p), ("desc", ctypes.c_void_p),
                ("verdict", ctypes.c_void_p), ("hdr", ctypes.c_void_p), ("n", ctypes.c_size_t)]


class UpeGpuError(RuntimeError):
    pass


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is not built; run `make -C upe_amd/csrc` "
                          "(the MI355X path has no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    P, SZ, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    sig = {
        "upe_gpu_last_error": (ctypes.c_char_p, []),
        "upe_gpu_device_count": (I, []),
        "upe_gpu_local_cpus": (I, [I, P, SZ, P]),
        "upe_gpu_pin_self": (I, [I, I]),
        "upe_gpu_open": (P, [I, SZ]),
        "upe_gpu_close": (None, [P]),
        "upe_gpu_load_rules": (I, [P, P, SZ]),
        "upe_gpu_reload_rules": (I, [P, P, SZ, SZ, P, SZ]),
        "upe_gpu_load_neigh": (I, [P, P, SZ, P, SZ]),
        "upe_gpu_rule_index_kind": (I, [P]),
        "upe_gpu_rule_index_info": (I, [P, P]),
        "upe_gpu_set_port": (I, [P, P, ctypes.c_uint32]),
        "upe_gpu_set_l1": (I, [P, P]),
        "upe_gpu_get_l1": (I, [P, P]),
        "upe_gpu_process": (I, [P, P, P, P, SZ, P]),
        "upe_gpu_sync": (I, [P, P]),
        "upe_gpu_batch_info": (I, [P, P]),
        "upe_gpu_launch_info": (I, [P, P]),
        "upe_gpu_get_stats": (I, [P, P, P, SZ]),
        "upe_gpu_reset_stats": (I, [P]),
        "upe_gpu_timing_enable": (I, [P, I]),
        "upe_gpu_timing_span": (I, [P, I, I]),
        "upe_gpu_timing_read": (I, [P, P, P, P]),
        "upe_gpu_malloc": (P, [P, SZ]),
        "upe_gpu_free": (I, [P, P]),
        "upe_gpu_memcpy_h2d": (I, [P, P, P, SZ, P]),
        "upe_gpu_memcpy_d2h": (I, [P, P, P, SZ, P]),
        "upe_gpu_process_host": (I, [P, P, SZ, P, P, SZ, SZ]),
        "upe_gpu_process_host_emit": (I, [P, P, SZ, P, P, P, SZ, SZ, I]),
        "upe_gpu_process_batches": (I, [P, P, P, P, SZ, SZ, P]),
        "upe_gpu_process_rss": (I, [P, P, P, P, P, SZ, P]),
        "upe_gpu_compact": (I, [P, P, SZ, ctypes.c_uint32, P, P, P]),
        "upe_gpu_process_segmented": (I, [P, P, P, P, SZ, P, SZ, P, SZ, ctypes.c_int64, P, P]),
        "upe_gpu_process_emit": (I, [P, P, P, P, P, SZ, P]),
        "upe_gpu_process_emit_tx": (I, [P, P, P, P, P, P, P, SZ, P]),
        "upe_gpu_process_batches_emit": (I, [P, P, P, P, P, SZ, SZ, P]),
        "upe_gpu_process_ring_emit": (I, [P, P, P, P, P, SZ, SZ, P, P]),
        "upe_gpu_process_queue_emit": (I, [P, P, SZ, P]),
        "upe_hdr_apply": (None, [P, P]),
        "upe_gpu_host_alloc": (P, [SZ]),
        "upe_gpu_host_free": (I, [P]),
        "upe_gpu_host_register": (I, [P, SZ]),
        "upe_gpu_host_unregister": (I, [P]),
        "upe_gpu_process_mapped": (I, [P, P, P, P, SZ, P]),
        "upe_gpu_process_mapped_emit": (I, [P, P, P, P, P, SZ, P]),
        "upe_tx_flush": (I, [P, P, P, SZ, SZ, TX_BATCH_FN, P, P, P]),
        "upe_tx_flush_groups": (I, [P, P, P, P, SZ, SZ, TX_BATCH_FN, P, P, P]),
        "upe_gpu_hdr_layout": (I, []),
        "upe_rules_compile": (P, [P, SZ, SZ]),
        "upe_gpu_reload_image": (I, [P, P, P, SZ]),
        "upe_rules_image_free": (None, [P]),
        "upe_gpu_worker_run": (I, [P, ctypes.POINTER(WorkerOps), P, ctypes.POINTER(WorkerCfg),
                                   P]),
    }
    sig.update({
        "upe_rules_load_ini": (I, [ctypes.c_char_p, P, SZ, P]),
        "upe_rules_match_host": (I, [P, SZ, P, SZ, P, P]),
        "upe_pcap_read": (I, [ctypes.c_char_p, P, SZ, P, SZ, P]),
        "upe_host_last_error": (ctypes.c_char_p, []),
    })
    for name, (res, args) in sig.items():
        if os.environ.get("UPE_GPU_LIB_DIAG") and not hasattr(lib, name):
            continue   # an older diagnostic build (A/B timing) may lack newer entry points
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


LIB = _load()

# every symbol include/upe_gpu.h declares (checked by tests/test_abi.py)
EXPORTED = ("upe_gpu_last_error", "upe_gpu_device_count", "upe_gpu_local_cpus", "upe_gpu_pin_self",
            "upe_gpu_open", "upe_gpu_close",
            "upe_gpu_load_rules", "upe_gpu_reload_rules", "upe_gpu_load_neigh",
            "upe_gpu_rule_index_kind", "upe_gpu_rule_index_info", "upe_gpu_set_port",
            "upe_gpu_set_l1", "upe_gpu_get_l1", "upe_gpu_process", "upe_gpu_sync", "upe_gpu_batch_info",
            "upe_gpu_launch_info",
            "upe_gpu_get_stats", "upe_gpu_reset_stats", "upe_gpu_timing_enable",
            "upe_gpu_timing_span",
            "upe_gpu_timing_read", "upe_gpu_malloc", "upe_gpu_free",
            "upe_gpu_memcpy_h2d", "upe_gpu_memcpy_d2h", "upe_gpu_process_host",
            "upe_gpu_process_host_emit",
            "upe_gpu_process_batches", "upe_gpu_process_rss", "upe_gpu_compact",
            "upe_gpu_process_segmented", "upe_gpu_process_emit", "upe_gpu_process_batches_emit",
            "upe_gpu_process_ring_emit", "upe_gpu_process_queue_emit",
            "upe_hdr_apply",
            "upe_rules_load_ini", "upe_rules_match_host", "upe_pcap_read",
            "upe_host_last_error",
            "upe_gpu_host_alloc", "upe_gpu_host_free", "upe_gpu_host_register",
            "upe_gpu_host_unregister", "upe_gpu_process_mapped", "upe_gpu_process_mapped_emit",
            "upe_tx_flush", "upe_tx_flush_groups", "upe_gpu_process_emit_tx", "upe_gpu_hdr_layout",
            "upe_rules_compile", "upe_gpu_reload_image", "upe_rules_image_free",
            "upe_gpu_worker_run")


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise UpeGpuError(f"{what}: {LIB.upe_gpu_last_error().decode()}")


def _np_ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


def _dev_ptr(x) -> int:
    if x is None:
        return 0
    if isinstance(x, int):
        return x
    return int(x.data_ptr())  # torch tensor


def device_count() -> int:
    return LIB.upe_gpu_device_count()


def local_cpus(device: int):
    """(CPUs local to the GPU that this thread may use, NUMA node) — upe_gpu_local_cpus."""
    buf = np.zeros(4096, np.int32)
    node = ctypes.c_int(-1)
    n = LIB.upe_gpu_local_cpus(device, _np_ptr(buf), buf.size, ctypes.byref(node))
    if n < 0:
        raise UpeGpuError(f"upe_gpu_local_cpus: {LIB.upe_gpu_last_error().decode()}")
    return [int(x) for x in buf[:min(n, buf.size)]], node.value


def pin_self(device: int, slot: int = 0) -> int:
    """Pin the calling thread to a CPU local to the GPU (upe_gpu_pin_self); returns the CPU."""
    cpu = LIB.upe_gpu_pin_self(device, slot)
    if cpu < 0:
        raise UpeGpuError(f"upe_gpu_pin_self: {LIB.upe_gpu_last_error().decode()}")
    return cpu


class GpuWorker:
    """One GPU-backed worker context (include/upe_gpu.h upe_gpu_ctx_t)."""

    def __init__(self, device: int = 0, rule_capacity: int = 1024):
        self._ctx = LIB.upe_gpu_open(device, rule_capacity)
        if not self._ctx:
            raise UpeGpuError(f"upe_gpu_open: {LIB.upe_gpu_last_error().decode()}")
        self.device = device
        self.capacity = rule_capacity

    # ---- lifetime ----
    def close(self) -> None:
        if self._ctx:
            LIB.upe_gpu_close(self._ctx)
            self._ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- tables and identity ----
    def load_rules(self, rules_sorted: np.ndarray) -> None:
        r = np.ascontiguousarray(rules_sorted, dtype=RULE_DTYPE)
        _check(LIB.upe_gpu_load_rules(self._ctx, _np_ptr(r) if len(r) else None, len(r)),
               "upe_gpu_load_rules")

    def reload_rules(self, rules_sorted: np.ndarray, capacity: int | None = None,
                     want_old: bool = True):
        """upe_gpu_reload_rules: the SIGHUP reload (src/main.c:216-282) — new table, fresh zero
        rule_stats of `capacity` entries (default: unchanged), counters and L1 kept.  Returns the
        old rule_stats (old capacity) when want_old."""
        cap = self.capacity if capacity is None else int(capacity)
        r = np.ascontiguousarray(rules_sorted, dtype=RULE_DTYPE)
        old = np.zeros(self.capacity, RULE_STAT_DTYPE) if want_old else None
        _check(LIB.upe_gpu_reload_rules(self._ctx, _np_ptr(r) if len(r) else None, len(r), cap,
                                        _np_ptr(old) if want_old else None,
                                        self.capacity if want_old else 0),
               "upe_gpu_reload_rules")
        self.capacity = cap
        return old

    def reload_image(self, image: "RuleImage", want_old: bool = True):
        """upe_gpu_reload_image: reload_rules with a table compiled beforehand (RuleImage, e.g. on
        another thread); the capacity is the image's.  Returns the old rule_stats when want_old."""
        old = np.zeros(self.capacity, RULE_STAT_DTYPE) if want_old else None
        _check(LIB.upe_gpu_reload_image(self._ctx, image.ptr, _np_ptr(old) if want_old else None,
                                        self.capacity if want_old else 0), "upe_gpu_reload_image")
        self.capacity = image.capacity
        return old

    def rule_index_kind(self) -> int:
        """0: linear scan, 1: tuple-space index, 2: decision tree."""
        k = LIB.upe_gpu_rule_index_kind(self._ctx)
        if k < 0:
            raise UpeGpuError(LIB.upe_gpu_last_error().decode())
        return k

    def rule_index_info(self) -> np.ndarray:
        out = np.zeros(1, RULE_INDEX_INFO_DTYPE)
        _check(LIB.upe_gpu_rule_index_info(self._ctx, _np_ptr(out)), "upe_gpu_rule_index_info")
        return out[0]

    def load_neigh(self, arp: np.ndarray | None, ndp: np.ndarray | None) -> None:
        a = np.ascontiguousarray(arp if arp is not None else np.zeros(0, ARP_DTYPE), ARP_DTYPE)
        b = np.ascontiguousarray(ndp if ndp is not None else np.zeros(0, NDP_DTYPE), NDP_DTYPE)
        _check(LIB.upe_gpu_load_neigh(self._ctx, _np_ptr(a) if len(a) else None, len(a),
                                      _np_ptr(b) if len(b) else None, len(b)),
               "upe_gpu_load_neigh")

    def set_port(self, eth_addr: bytes, ip4_addr: int) -> None:
        mac = np.frombuffer(bytes(eth_addr), np.uint8).copy()
        _check(LIB.upe_gpu_set_port(self._ctx, _np_ptr(mac), ip4_addr), "upe_gpu_set_port")

    def set_l1(self, l1: np.ndarray) -> None:
        x = np.ascontiguousarray(l1, L1_DTYPE).reshape(1)
        _check(LIB.upe_gpu_set_l1(self._ctx, _np_ptr(x)), "upe_gpu_set_l1")

    def get_l1(self) -> np.ndarray:
        x = np.zeros(1, L1_DTYPE)
        _check(LIB.upe_gpu_get_l1(self._ctx, _np_ptr(x)), "upe_gpu_get_l1")
        return x

    def configure(self, wl) -> None:
        """Load a synth.Workload's tables, port identity and starting L1 state."""
        self.load_rules(wl.rules_sorted)
        self.load_neigh(wl.arp, wl.ndp)
        self.set_port(wl.eth_addr, wl.ip4_addr)
        self.set_l1(wl.l1)

    # ---- the hot path ----
    def process(self, frames, desc, verdict, n: int, stream=None) -> None:
        """Queue one batch (device buffers) on `stream` (hipStream_t handle or None)."""
        _check(LIB.upe_gpu_process(self._ctx, _dev_ptr(frames), _dev_ptr(desc),
                                   _dev_ptr(verdict), n, stream or None),
               "upe_gpu_process")

    def process_mapped(self, frames: np.ndarray, desc: np.ndarray, verdict: np.ndarray,
                       stream=None) -> None:
        """upe_gpu_process_mapped: the batch classified where it lies in pinned host memory
        (PinnedArray views or registered buffers), frames rewritten in place; asynchronous, read
        the outputs after sync()."""
        _check(LIB.upe_gpu_process_mapped(self._ctx, _np_ptr(frames), _np_ptr(desc),
                                          _np_ptr(verdict), int(desc.shape[0]), stream or None),
               "upe_gpu_process_mapped")

    def process_mapped_emit(self, frames: np.ndarray, desc: np.ndarray, verdict: np.ndarray,
                            hdr: np.ndarray, stream=None) -> None:
        """upe_gpu_process_mapped_emit: the same with 16-byte records into `hdr` (host), frames
        read only."""
        _check(LIB.upe_gpu_process_mapped_emit(self._ctx, _np_ptr(frames), _np_ptr(desc),
                                               _np_ptr(verdict), _np_ptr(hdr),
                                               int(desc.shape[0]), stream or None),
               "upe_gpu_process_mapped_emit")

    def process_emit(self, frames, desc, verdict, hdr, n: int, stream=None) -> None:
        """Emit mode: rewritten header bytes into `hdr` (n 16-byte records), frames read only."""
        _check(LIB.upe_gpu_process_emit(self._ctx, _dev_ptr(frames), _dev_ptr(desc),
                                        _dev_ptr(verdict), _dev_ptr(hdr), n, stream or None),
               "upe_gpu_process_emit")

    @staticmethod
    def frames_list(frames_ptrs):
        """A native array of batch pointers for process_batches[_emit] (build it once, outside a
        timed region, and pass it instead of a Python list)."""
        if isinstance(frames_ptrs, ctypes.Array):
            return frames_ptrs
        return (ctypes.c_void_p * len(frames_ptrs))(*[int(x) for x in frames_ptrs])

    def process_batches_emit(self, frames_ptrs, desc, verdict, hdr, n: int, stream=None) -> None:
        """process_batches in emit mode (every batch writes its records to `hdr`)."""
        arr = self.frames_list(frames_ptrs)
        _check(LIB.upe_gpu_process_batches_emit(self._ctx, arr, _dev_ptr(desc), _dev_ptr(verdict),
                                                _dev_ptr(hdr), n, len(frames_ptrs),
                                                stream or None),
               "upe_gpu_process_batches_emit")

    def process_queue_emit(self, batches, stream=None) -> None:
        """upe_gpu_process_queue_emit over a list of (frames, desc, verdict, hdr, n) device
        buffers (pointers or tensors): the worker loop's resident batches, one launch each on the
        context's stream, in order (the overlapped form was removed in round 4)."""
        arr = (QueueBatch * len(batches))(*[QueueBatch(_dev_ptr(f), _dev_ptr(d), _dev_ptr(v),
                                                       _dev_ptr(h), int(n))
                                            for f, d, v, h, n in batches])
        _check(LIB.upe_gpu_process_queue_emit(self._ctx, arr, len(batches), stream or None),
               "upe_gpu_process_queue_emit")

    def process_ring_emit(self, frames, desc, verdict, hdr, n: int, count: int, done_ns=None,
                          stream=None) -> None:
        """upe_gpu_process_ring_emit: `count` batches of n packets laid out back to back, one
        launch; done_ns (device uint64[count] or None) receives per-batch completion times."""
        _check(LIB.upe_gpu_process_ring_emit(self._ctx, _dev_ptr(frames), _dev_ptr(desc),
                                             _dev_ptr(verdict), _dev_ptr(hdr), n, count,
                                             _dev_ptr(done_ns) or None, stream or None),
               "upe_gpu_process_ring_emit")

    def process_batches(self, frames_ptrs, desc, verdict, n: int, stream=None) -> None:
        """Queue len(frames_ptrs) batches (device pointers) back to back from native code."""
        arr = self.frames_list(frames_ptrs)
        _check(LIB.upe_gpu_process_batches(self._ctx, arr, _dev_ptr(desc), _dev_ptr(verdict), n,
                                           len(frames_ptrs), stream or None),
               "upe_gpu_process_batches")

    def process_rss(self, frames, desc, verdict, flow_hash, n: int, stream=None) -> None:
        """process() plus per-packet flow_hash (software RSS) into a device uint32 array."""
        _check(LIB.upe_gpu_process_rss(self._ctx, _dev_ptr(frames), _dev_ptr(desc),
                                       _dev_ptr(verdict), _dev_ptr(flow_hash), n, stream or None),
               "upe_gpu_process_rss")

    def process_segmented(self, frames, desc, verdict, n: int, arp: np.ndarray,
                          ndp: np.ndarray, now: int = 0, stream=None) -> int:
        """A device batch with exact control-packet semantics: cut after every table-writing
        ARP / NS / NA packet, apply the write to `arp` / `ndp` (host slot arrays, updated in
        place) and upload them again.  Returns the number of table writes."""
        assert arp.dtype == ARP_DTYPE and ndp.dtype == NDP_DTYPE
        assert arp.flags.c_contiguous and ndp.flags.c_contiguous
        nw = ctypes.c_size_t(0)
        _check(LIB.upe_gpu_process_segmented(
            self._ctx, _dev_ptr(frames), _dev_ptr(desc), _dev_ptr(verdict), n,
            _np_ptr(arp) if len(arp) else None, len(arp), _np_ptr(ndp) if len(ndp) else None,
            len(ndp), now, ctypes.byref(nw), stream or None), "upe_gpu_process_segmented")
        return nw.value

    def process_emit_tx(self, frames, desc, verdict, hdr, tx, tx_count, n: int,
                        stream=None) -> None:
        """upe_gpu_process_emit plus the egress list by 64-packet group (device buffers)."""
        _check(LIB.upe_gpu_process_emit_tx(self._ctx, _dev_ptr(frames), _dev_ptr(desc),
                                           _dev_ptr(verdict), _dev_ptr(hdr), _dev_ptr(tx),
                                           _dev_ptr(tx_count), n, stream or None),
               "upe_gpu_process_emit_tx")

    def compact(self, verdict, n: int, code: int, index, count, stream=None) -> None:
        """Indexes of the packets with verdict code `code`, in packet order (device buffers)."""
        _check(LIB.upe_gpu_compact(self._ctx, _dev_ptr(verdict), n, code, _dev_ptr(index),
                                   _dev_ptr(count), stream or None), "upe_gpu_compact")

    def sync(self, stream=None) -> None:
        _check(LIB.upe_gpu_sync(self._ctx, stream or None), "upe_gpu_sync")

    def batch_info(self) -> np.ndarray:
        x = np.zeros(1, BATCH_INFO_DTYPE)
        _check(LIB.upe_gpu_batch_info(self._ctx, _np_ptr(x)), "upe_gpu_batch_info")
        return x

    def launch_info(self) -> dict:
        """upe_gpu_launch_info: the last classify launch's kernel variant (bit 3 = no look-back),
        grid, deferred look-back entries, and the context's launch count."""
        x = np.zeros(1, LAUNCH_INFO_DTYPE)
        _check(LIB.upe_gpu_launch_info(self._ctx, _np_ptr(x)), "upe_gpu_launch_info")
        return {k: int(x[k][0]) for k in LAUNCH_INFO_DTYPE.names}

    def get_stats(self):
        c = np.zeros(1, COUNTERS_DTYPE)
        s = np.zeros(self.capacity, RULE_STAT_DTYPE)
        _check(LIB.upe_gpu_get_stats(self._ctx, _np_ptr(c), _np_ptr(s), self.capacity),
               "upe_gpu_get_stats")
        return c, s

    def reset_stats(self) -> None:
        _check(LIB.upe_gpu_reset_stats(self._ctx), "upe_gpu_reset_stats")

    # ---- kernel timing (HIP events on the launch stream) ----
    def timing_enable(self, every: int = 1) -> None:
        """Record kernel events on every ``every``-th process() call (0 / False: off)."""
        _check(LIB.upe_gpu_timing_enable(self._ctx, int(every)), "upe_gpu_timing_enable")

    def timing_span(self, every: int, span: int) -> None:
        """Each sample's event pair brackets ``span`` consecutive calls, one sample opened on
        every ``every``-th call."""
        _check(LIB.upe_gpu_timing_span(self._ctx, int(every), int(span)), "upe_gpu_timing_span")

    def timing_read(self):
        a, b = ctypes.c_double(), ctypes.c_double()
        n = ctypes.c_uint64()
        _check(LIB.upe_gpu_timing_read(self._ctx, ctypes.byref(a), ctypes.byref(b),
                                       ctypes.byref(n)), "upe_gpu_timing_read")
        return a.value, b.value, n.value

    # ---- host round trip (pinned host batch in, verdicts and rewritten headers out) ----
    def process_host(self, frames: np.ndarray, desc: np.ndarray, verdict: np.ndarray,
                     chunk: int = 0) -> None:
        """upe_gpu_process_host over host arrays (frames rewritten in place)."""
        assert frames.dtype == np.uint8 and desc.dtype == np.uint64 and verdict.dtype == np.uint32
        assert verdict.shape[0] >= desc.shape[0]
        _check(LIB.upe_gpu_process_host(self._ctx, _np_ptr(frames), frames.nbytes,
                                        _np_ptr(desc) if desc.size else None,
                                        _np_ptr(verdict) if verdict.size else None,
                                        int(desc.shape[0]), int(chunk)),
               "upe_gpu_process_host")

    def process_host_emit(self, frames: np.ndarray, desc: np.ndarray, verdict: np.ndarray,
                          hdr: np.ndarray, chunk: int = 0, apply_threads: int = 0) -> None:
        """upe_gpu_process_host_emit: verdicts + records (hdr, (n, 16) uint8) back; with
        apply_threads >= 0 the records are applied to `frames` on the host."""
        assert frames.dtype == np.uint8 and desc.dtype == np.uint64 and verdict.dtype == np.uint32
        assert hdr.dtype == np.uint8 and hdr.size >= 16 * desc.shape[0]
        assert verdict.shape[0] >= desc.shape[0]
        _check(LIB.upe_gpu_process_host_emit(self._ctx, _np_ptr(frames), frames.nbytes,
                                             _np_ptr(desc) if desc.size else None,
                                             _np_ptr(verdict) if verdict.size else None,
                                             _np_ptr(hdr) if hdr.size else None,
                                             int(desc.shape[0]), int(chunk), int(apply_threads)),
               "upe_gpu_process_host_emit")

    # ---- device memory without torch ----
    def malloc(self, nbytes: int) -> int:
        p = LIB.upe_gpu_malloc(self._ctx, nbytes)
        if not p:
            raise UpeGpuError(f"upe_gpu_malloc: {LIB.upe_gpu_last_error().decode()}")
        return p

    def free(self, ptr: int) -> None:
        _check(LIB.upe_gpu_free(self._ctx, ptr), "upe_gpu_free")

    def h2d(self, dptr: int, host: np.ndarray, stream=None) -> None:
        _check(LIB.upe_gpu_memcpy_h2d(self._ctx, dptr, _np_ptr(host), host.nbytes, stream or None),
               "upe_gpu_memcpy_h2d")

    def d2h(self, host: np.ndarray, dptr: int, stream=None) -> None:
        _check(LIB.upe_gpu_memcpy_d2h(self._ctx, _np_ptr(host), dptr, host.nbytes, stream or None),
               "upe_gpu_memcpy_d2h")


# ---- host-side batch builders (upe_host.c; no GPU needed) ----------------------------------

PCAP_INFO_DTYPE = np.dtype([("records", "<u8"), ("packets", "<u8"), ("dropped_oversize", "<u8"),
                            ("frames_bytes", "<u8")])


def rules_load_ini(path: str, capacity: int = 1024) -> np.ndarray:
    """upe_rules_load_ini: rt->rules after rule_table_init(capacity) + rule_config_load."""
    out = np.zeros(capacity, RULE_DTYPE)
    count = np.zeros(1, np.uint64)
    rc = LIB.upe_rules_load_ini(os.fsencode(path), _np_ptr(out), capacity, _np_ptr(count))
    if rc != 0:
        raise UpeGpuError(LIB.upe_host_last_error().decode())
    return out[: int(count[0])].copy()


def rules_match_host(rules_sorted: np.ndarray, keys: np.ndarray):
    """upe_rules_match_host: the first match of each key (FLOW_KEY_DTYPE) through the decision
    tree the GPU path builds for the table, walked on the host.  Returns (sorted index or -1 per
    key, the tree's RULE_INDEX_INFO_DTYPE record; all zero when the table gets no tree)."""
    r = np.ascontiguousarray(rules_sorted, dtype=RULE_DTYPE)
    k = np.ascontiguousarray(keys, dtype=FLOW_KEY_DTYPE)
    out = np.zeros(len(k), np.int64)
    info = np.zeros(1, RULE_INDEX_INFO_DTYPE)
    _check(LIB.upe_rules_match_host(_np_ptr(r) if len(r) else None, len(r),
                                    _np_ptr(k) if len(k) else None, len(k),
                                    _np_ptr(out) if len(k) else None, _np_ptr(info)),
           "upe_rules_match_host")
    return out, info[0]


def pcap_read(path: str):
    """upe_pcap_read: a pcap capture -> (frames, desc, info) in the batch layout."""
    info = np.zeros(1, PCAP_INFO_DTYPE)
    if LIB.upe_pcap_read(os.fsencode(path), None, 0, None, 0, _np_ptr(info)) != 0:
        raise UpeGpuError(LIB.upe_host_last_error().decode())
    frames = np.zeros(int(info["frames_bytes"][0]) + 128, np.uint8)
    desc = np.zeros(max(int(info["packets"][0]), 1), np.uint64)
    if LIB.upe_pcap_read(os.fsencode(path), _np_ptr(frames), frames.nbytes, _np_ptr(desc),
                         desc.shape[0], _np_ptr(info)) != 0:
        raise UpeGpuError(LIB.upe_host_last_error().decode())
    return frames, desc[: int(info["packets"][0])].copy(), info


class PinnedArray:
    """A numpy view of page-locked host memory (upe_gpu_host_alloc); freed by free()."""

    def __init__(self, shape, dtype):
        dtype = np.dtype(dtype)
        nbytes = int(np.prod(shape)) * dtype.itemsize
        self.ptr = LIB.upe_gpu_host_alloc(max(nbytes, 1))
        if not self.ptr:
            raise UpeGpuError(f"upe_gpu_host_alloc: {LIB.upe_gpu_last_error().decode()}")
        buf = (ctypes.c_uint8 * max(nbytes, 1)).from_address(self.ptr)
        self.array = np.frombuffer(buf, dtype=np.uint8, count=nbytes).view(dtype).reshape(shape)

    def free(self) -> None:
        if self.ptr:
            self.array = None
            LIB.upe_gpu_host_free(self.ptr)
            self.ptr = None


def tx_flush(frames: np.ndarray, desc: np.ndarray, verdict: np.ndarray, burst: int = 32,
             sent_of=None, groups=None):
    """upe_tx_flush over a host batch: returns (batches, forwarded, dropped), batches = one
    (packet indexes, frame bytes) pair per TX call in call order.  sent_of(count) -> frames the
    stand-in for sendmmsg reports sent (default: all).  groups = (tx, tx_count): the grouped
    egress list of upe_gpu_process_emit_tx instead of the verdicts (upe_tx_flush_groups)."""
    frames = np.ascontiguousarray(frames)
    desc = np.ascontiguousarray(desc, dtype=np.uint64)
    verdict = None if verdict is None else np.ascontiguousarray(verdict, dtype=np.uint32)
    base = frames.ctypes.data
    index_of = {int(o): i for i, o in enumerate((desc >> np.uint64(16)).tolist())}
    batches = []

    def cb(user, fr, lens, count):
        idx, data = [], []
        for k in range(count):
            off = fr[k] - base
            idx.append(index_of[off])
            data.append(bytes(frames[off:off + lens[k]]))
        batches.append((np.array(idx, np.int64), data))
        return count if sent_of is None else int(sent_of(count))

    fn = TX_BATCH_FN(cb)
    fwd = ctypes.c_uint64(0)
    drp = ctypes.c_uint64(0)
    if groups is not None:
        tx = np.ascontiguousarray(groups[0], dtype=np.uint32)
        cnt = np.ascontiguousarray(groups[1], dtype=np.uint32)
        rc = LIB.upe_tx_flush_groups(_np_ptr(frames), _np_ptr(desc), _np_ptr(tx), _np_ptr(cnt),
                                     int(desc.shape[0]), int(burst), fn, None, ctypes.byref(fwd),
                                     ctypes.byref(drp))
    else:
        rc = LIB.upe_tx_flush(_np_ptr(frames), _np_ptr(desc), _np_ptr(verdict),
                              int(desc.shape[0]), int(burst), fn, None, ctypes.byref(fwd),
                              ctypes.byref(drp))
    if rc != 0:
        raise UpeGpuError(f"upe_tx_flush: {LIB.upe_host_last_error().decode()}")
    return batches, int(fwd.value), int(drp.value)


class RuleImage:
    """upe_rules_compile: a sorted rule table compiled for the GPU path on the host, with no
    context or GPU (the reference's stats thread builds its new table before the swap the same
    way, src/main.c:222-257); free() (or garbage collection) releases it."""

    def __init__(self, rules_sorted: np.ndarray, capacity: int):
        r = np.ascontiguousarray(rules_sorted, dtype=RULE_DTYPE)
        self.capacity = int(capacity)
        self.ptr = LIB.upe_rules_compile(_np_ptr(r) if len(r) else None, len(r), self.capacity)
        if not self.ptr:
            raise UpeGpuError(LIB.upe_gpu_last_error().decode())

    def free(self) -> None:
        if self.ptr:
            LIB.upe_rules_image_free(self.ptr)
            self.ptr = None

    def __del__(self):
        self.free()


class RegisteredArray:
    """An existing numpy array page-locked and mapped for the GPU (upe_gpu_host_register) until
    free()."""

    def __init__(self, array: np.ndarray):
        assert array.flags["C_CONTIGUOUS"]
        self.array = array
        self.ptr = array.ctypes.data
        _check(LIB.upe_gpu_host_register(self.ptr, max(int(array.nbytes), 1)),
               "upe_gpu_host_register")

    def free(self) -> None:
        if self.ptr:
            _check(LIB.upe_gpu_host_unregister(self.ptr), "upe_gpu_host_unregister")
            self.ptr = None


class DeviceBatch:
    """A workload's batch copied into device memory owned by a GpuWorker."""

    def __init__(self, worker: GpuWorker, frames: np.ndarray, desc: np.ndarray):
        self.worker = worker
        self.n = int(desc.shape[0])
        self.frames_nbytes = int(frames.nbytes)
        self.frames = worker.malloc(frames.nbytes)
        self.desc = worker.malloc(max(desc.nbytes, 8))
        self.verdict = worker.malloc(max(4 * self.n, 4))
        worker.h2d(self.frames, np.ascontiguousarray(frames))
        if self.n:
            worker.h2d(self.desc, np.ascontiguousarray(desc))
        worker.sync()

        self.hdr = 0

    def run(self, stream=None) -> None:
        self.worker.process(self.frames, self.desc, self.verdict, self.n, stream)

    def run_emit(self, stream=None) -> None:
        """Emit mode: records into a device array owned by this batch."""
        if not self.hdr:
            self.hdr = self.worker.malloc(max(16 * self.n, 16))
        self.worker.process_emit(self.frames, self.desc, self.verdict, self.hdr, self.n, stream)

    def fetch(self):
        """(frames, verdict) back to the host (synchronises)."""
        self.worker.sync()
        frames = np.empty(self.frames_nbytes, np.uint8)
        verdict = np.empty(self.n, np.uint32)
        self.worker.d2h(frames, self.frames)
        if self.n:
            self.worker.d2h(verdict, self.verdict)
        self.worker.sync()
        return frames, verdict

    def fetch_hdr(self, raw: bool = False) -> np.ndarray:
        """The emit-mode records (synchronises): one per packet, (n, 16) uint8, zero for a packet
        not forwarded (expand_records); raw=True: the device array as the kernel left it (records
        of forwarded packets compacted per 64-packet group, the other slots unwritten)."""
        self.worker.sync()
        rec = np.zeros((self.n, 16), np.uint8)
        verdict = np.empty(self.n, np.uint32)
        if self.n:
            self.worker.d2h(rec, self.hdr)
            self.worker.d2h(verdict, self.verdict)
        self.worker.sync()
        return rec if raw else expand_records(rec, verdict)

    def free(self) -> None:
        for p in (self.frames, self.desc, self.verdict, self.hdr):
            if p:
                self.worker.free(p)
        self.frames = self.desc = self.verdict = self.hdr = 0


def record_slots(verdict: np.ndarray) -> np.ndarray:
    """Emit mode's record layout (include/upe_gpu.h): forwarded packet i's record sits at
    64 * (i // 64) + the number of forwarded packets before it in its 64-packet group.  Returns
    that slot for every packet (meaningful for forwarded ones)."""
    from .layout import V_FWD

    v = np.asarray(verdict, np.uint32)
    fwd = ((v & 0xF) == V_FWD).astype(np.int64)
    excl = np.cumsum(fwd) - fwd
    idx = np.arange(len(v), dtype=np.int64)
    grp = idx & ~np.int64(63)
    return grp + excl - excl[grp] if len(v) else idx


def expand_records(rec_raw: np.ndarray, verdict: np.ndarray) -> np.ndarray:
    """Per-packet records, (n, 16) uint8, zero for packets not forwarded, from the compacted
    array the emit-mode kernel writes (record_slots)."""
    from .layout import V_FWD

    raw = np.ascontiguousarray(rec_raw, np.uint8).reshape(-1, 16)
    v = np.asarray(verdict, np.uint32)
    out = np.zeros((len(v), 16), np.uint8)
    fwd = (v & 0xF) == V_FWD
    out[fwd] = raw[record_slots(v)[fwd]]
    return out


def hdr_apply(frames: np.ndarray, desc: np.ndarray, rec: np.ndarray) -> np.ndarray:
    """upe_hdr_apply over a batch (through the C helper), returns the rewritten frames."""
    from .layout import desc_offsets

    out = np.ascontiguousarray(frames).copy()
    rec = np.ascontiguousarray(rec, np.uint8).reshape(-1, 16)
    base = out.ctypes.data
    offs = desc_offsets(desc)
    for i in np.nonzero(rec[:, 15] != 0)[0]:
        LIB.upe_hdr_apply(ctypes.c_void_p(base + int(offs[i])), _np_ptr(rec[i]))
    return out


def run_workload(wl, device: int = 0, worker: GpuWorker | None = None, emit: bool = False):
    """Process a synth.Workload once on the GPU; returns (frames, verdict, counters,
    rule_stats, l1) like oracle.Result.  emit: run in emit mode and return the frames with the
    records applied by upe_hdr_apply."""
    own = worker is None
    w = worker or GpuWorker(device, wl.capacity)
    try:
        if own:
            w.configure(wl)
        b = DeviceBatch(w, wl.frames, wl.desc)
        if emit:
            b.run_emit()
            frames, verdict = b.fetch()
            frames = hdr_apply(frames, wl.desc, b.fetch_hdr())
        else:
            b.run()
            frames, verdict = b.fetch()
        b.free()
        counters, stats = w.get_stats()
        l1 = w.get_l1()
        return frames, verdict, counters, stats, l1
    finally:
        if own:
            w.close()
