"""oracle — CHECKERS for the UPE hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package.
Nothing under upe_amd/ imports it; the product path has no CPU fallback.

  restated  build/libupe_oracle.so — our C restatement (oracle/cpu_ref.c)
  reference _ref/libupe_ref.so     — the reference worker itself (oracle/ref_harness.c), built
                                     only where /root/reference exists; prebuilt copies travel
                                     to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from upe_amd.layout import (ARP_DTYPE, COUNTERS_DTYPE, L1_DTYPE, NDP_DTYPE, RULE_DTYPE,
                            RULE_STAT_DTYPE)

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "build", "libupe_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "libupe_ref.so")

_P = ctypes.c_void_p
_SZ = ctypes.c_size_t


def _ptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_P)


def _load(path: str) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built (run `make -C oracle`)")
    return ctypes.CDLL(path)


_oracle = None
_ref = None


def oracle_lib() -> ctypes.CDLL:
    global _oracle
    if _oracle is None:
        lib = _load(ORACLE_SO)
        lib.upe_ref_process.restype = ctypes.c_int
        lib.upe_ref_process.argtypes = [_P, _SZ, _P, _SZ, _P, _SZ, _P, ctypes.c_uint32, ctypes.c_int,
                                        _P, _P, _P, _SZ, _P, _P, _P, _SZ]
        lib.upe_ref_parse.restype = ctypes.c_int
        lib.upe_ref_parse.argtypes = [_P, _SZ, _P]
        lib.upe_ref_flow_hash.restype = ctypes.c_uint32
        lib.upe_ref_flow_hash.argtypes = [_P]
        lib.upe_ref_ipv4_checksum.restype = ctypes.c_uint16
        lib.upe_ref_ipv4_checksum.argtypes = [_P, _SZ]
        lib.upe_ref_ipv4_mask.restype = ctypes.c_bool
        lib.upe_ref_ipv4_mask.argtypes = [ctypes.c_uint8, _P]
        lib.upe_ref_ipv6_mask.restype = ctypes.c_bool
        lib.upe_ref_ipv6_mask.argtypes = [ctypes.c_uint8, _P]
        lib.upe_ref_rules_build.restype = ctypes.c_int
        lib.upe_ref_rules_build.argtypes = [_P, _SZ, _P]
        lib.upe_ref_match.restype = ctypes.c_long
        lib.upe_ref_match.argtypes = [_P, _SZ, _P]
        lib.upe_ref_arp_lookup.restype = ctypes.c_bool
        lib.upe_ref_arp_lookup.argtypes = [_P, _SZ, ctypes.c_uint32, _P]
        lib.upe_ref_ndp_lookup.restype = ctypes.c_bool
        lib.upe_ref_ndp_lookup.argtypes = [_P, _SZ, _P, _P]
        _oracle = lib
    return _oracle


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def ref_lib() -> ctypes.CDLL:
    global _ref
    if _ref is None:
        lib = _load(REF_SO)
        lib.upe_refh_process.restype = ctypes.c_int
        lib.upe_refh_process.argtypes = [_P, _SZ, _SZ, ctypes.c_int, _P, _P, _SZ, _P, _SZ, _P,
                                         ctypes.c_uint32, _P, _P, _P, _SZ, _P, _P, _P]
        lib.upe_refh_process_reload.restype = ctypes.c_int
        lib.upe_refh_process_reload.argtypes = [_P, _SZ, _SZ, _P, _SZ, _SZ, _P, _SZ, _P, _SZ, _P,
                                                _SZ, _P, ctypes.c_uint32, _P, _P, _P, _SZ, _P, _P,
                                                _P, _P]
        lib.upe_refh_tx_log.restype = ctypes.c_int
        lib.upe_refh_tx_log.argtypes = [_P, _SZ, _P, _SZ, _P, _P]
        lib.upe_refh_time.restype = ctypes.c_double
        lib.upe_refh_time.argtypes = [_P, _SZ, _SZ, _P, _SZ, _P, _SZ, _P, ctypes.c_uint32, _P, _P,
                                      _SZ, ctypes.c_int, _P, ctypes.c_int, _P]
        _ref = lib
    return _ref


class Result:
    """Outputs of one batch through a checker."""

    def __init__(self, frames, verdict, counters, rule_stats, l1, arp=None, ndp=None,
                 rules_sorted=None):
        self.frames = frames
        self.verdict = verdict
        self.counters = counters
        self.rule_stats = rule_stats
        self.l1 = l1
        self.arp = arp
        self.ndp = ndp
        self.rules_sorted = rules_sorted


def _eth(wl) -> np.ndarray:
    return np.frombuffer(bytes(wl.eth_addr), dtype=np.uint8).copy()


def run_restated(wl, rules_sorted=None, apply_control: bool = False, l1=None,
                 counters=None, rule_stats=None) -> Result:
    """Our C restatement over the workload (frames copied, not modified)."""
    lib = oracle_lib()
    rs = wl.rules_sorted if rules_sorted is None else rules_sorted
    rs = np.ascontiguousarray(rs, dtype=RULE_DTYPE)
    frames = wl.frames.copy()
    arp = wl.arp.copy()
    ndp = wl.ndp.copy()
    l1 = (wl.l1 if l1 is None else l1).copy()
    verdict = np.zeros(wl.n, dtype=np.uint32)
    cnt = np.zeros(1, COUNTERS_DTYPE) if counters is None else counters.copy()
    st = np.zeros(wl.capacity, RULE_STAT_DTYPE) if rule_stats is None else rule_stats.copy()
    eth = _eth(wl)
    rc = lib.upe_ref_process(_ptr(rs), len(rs), _ptr(arp), len(arp), _ptr(ndp), len(ndp),
                             _ptr(eth), wl.ip4_addr, int(apply_control), _ptr(l1), _ptr(frames),
                             _ptr(wl.desc), wl.n, _ptr(verdict), _ptr(cnt), _ptr(st), wl.capacity)
    if rc != 0:
        raise RuntimeError("upe_ref_process failed")
    return Result(frames, verdict, cnt, st, l1, arp, ndp, rs)


def run_reference(wl, presorted: bool = False, l1=None) -> Result:
    """The reference worker (src/worker.c process_packet) over the workload."""
    lib = ref_lib()
    rules = wl.rules_sorted if presorted else wl.rules
    rules = np.ascontiguousarray(rules, dtype=RULE_DTYPE)
    sorted_out = np.zeros(len(rules), RULE_DTYPE)
    frames = wl.frames.copy()
    arp = wl.arp.copy()
    ndp = wl.ndp.copy()
    l1 = (wl.l1 if l1 is None else l1).copy()
    verdict = np.zeros(wl.n, dtype=np.uint32)
    cnt = np.zeros(1, COUNTERS_DTYPE)
    st = np.zeros(wl.capacity, RULE_STAT_DTYPE)
    eth = _eth(wl)
    rc = lib.upe_refh_process(_ptr(rules), len(rules), wl.capacity, int(presorted),
                              _ptr(sorted_out), _ptr(arp), len(arp), _ptr(ndp), len(ndp), _ptr(eth),
                              wl.ip4_addr, _ptr(l1), _ptr(frames), _ptr(wl.desc), wl.n,
                              _ptr(verdict), _ptr(cnt), _ptr(st))
    if rc != 0:
        raise RuntimeError("upe_refh_process failed")
    return Result(frames, verdict, cnt, st, l1, arp, ndp, sorted_out)


def run_reference_reload(wl, rules_b, capacity_b: int, at: int, l1=None):
    """The reference worker with the stats thread's SIGHUP reload (src/main.c:216-282) between
    packets at-1 and at: table A = wl.rules (insertion order), then table B = rules_b (insertion
    order) with a fresh rule_stats[capacity_b].  Returns (Result with rule_stats = the new array
    and rules_sorted = table B as built, the old array as it stood at the swap)."""
    lib = ref_lib()
    ra = np.ascontiguousarray(wl.rules, dtype=RULE_DTYPE)
    rb = np.ascontiguousarray(rules_b, dtype=RULE_DTYPE)
    sorted_b = np.zeros(len(rb), RULE_DTYPE)
    frames = wl.frames.copy()
    arp = wl.arp.copy()
    ndp = wl.ndp.copy()
    l1 = (wl.l1 if l1 is None else l1).copy()
    verdict = np.zeros(wl.n, dtype=np.uint32)
    cnt = np.zeros(1, COUNTERS_DTYPE)
    st_a = np.zeros(wl.capacity, RULE_STAT_DTYPE)
    st_b = np.zeros(capacity_b, RULE_STAT_DTYPE)
    eth = _eth(wl)
    rc = lib.upe_refh_process_reload(_ptr(ra), len(ra), wl.capacity, _ptr(rb), len(rb), capacity_b,
                                     _ptr(sorted_b), at, _ptr(arp), len(arp), _ptr(ndp), len(ndp),
                                     _ptr(eth), wl.ip4_addr, _ptr(l1), _ptr(frames), _ptr(wl.desc),
                                     wl.n, _ptr(verdict), _ptr(cnt), _ptr(st_a), _ptr(st_b))
    if rc != 0:
        raise RuntimeError("upe_refh_process_reload failed")
    return Result(frames, verdict, cnt, st_b, l1, arp, ndp, sorted_b), st_a


def tx_log():
    """The TX calls of the last run_reference on this thread (reference src/worker.c:287-303
    over the harness's tx_send_batch stub): (sizes per call, packet index of every frame in call
    order)."""
    lib = ref_lib()
    nb, nf = ctypes.c_size_t(0), ctypes.c_size_t(0)
    lib.upe_refh_tx_log(None, 0, None, 0, ctypes.byref(nb), ctypes.byref(nf))
    sizes = np.zeros(max(nb.value, 1), np.uint32)
    frames = np.zeros(max(nf.value, 1), np.uint32)
    lib.upe_refh_tx_log(_ptr(sizes), sizes.size, _ptr(frames), frames.size, ctypes.byref(nb),
                        ctypes.byref(nf))
    return sizes[:nb.value].copy(), frames[:nf.value].copy()


def time_reference(wl, threads: int = 1, cpus=None, reps: int = 5, rates=None) -> float:
    """Median packets/s of the reference worker over the workload (see upe_refh_time); `rates`
    (a list) receives every rep's rate, ascending."""
    lib = ref_lib()
    out = np.zeros(reps, np.float64)
    rs = np.ascontiguousarray(wl.rules_sorted, dtype=RULE_DTYPE)
    eth = _eth(wl)
    cpu_arr = None if cpus is None else np.ascontiguousarray(np.asarray(cpus, dtype=np.int32))
    med = lib.upe_refh_time(_ptr(rs), len(rs), wl.capacity, _ptr(wl.arp), len(wl.arp),
                             _ptr(wl.ndp), len(wl.ndp), _ptr(eth), wl.ip4_addr, _ptr(wl.frames),
                             _ptr(wl.desc), wl.n, threads, _ptr(cpu_arr), reps, _ptr(out))
    if rates is not None:
        rates.extend(float(x) for x in out)
    return med


def parse(frame: bytes, length: int | None = None):
    """upe_ref_parse on one frame -> (rc, key bytes as flow_key_t)."""
    lib = oracle_lib()
    buf = np.zeros(max(len(frame), 128), np.uint8)
    buf[: len(frame)] = np.frombuffer(frame, np.uint8)
    key = np.zeros(44, np.uint8)
    rc = lib.upe_ref_parse(_ptr(buf), len(frame) if length is None else length, _ptr(key))
    return rc, key
