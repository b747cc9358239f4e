"""GPU: the product worker loop (upe_gpu_worker_run, upe_amd/csrc/upe_worker.c) driven from
Python callbacks — a list of handles as the ring, a pinned packet pool, recorded TX calls — with
no reference build involved.  Against the restated worker (oracle/cpu_ref.c, in-order control
writes): the counters worker_main keeps, rule_stats, every packet's bytes, the neighbour tables
after the learning packets, and the calls worker_main makes per popped burst (tx_send of answered
ARP requests, one tx_send_batch of the burst's forwarded frames in packet order,
src/worker.c:40-52, 240-243, 287-303); in both batch paths (header windows staged in pinned memory,
read there by the kernel; frames classified where they lie in registered memory) and with bursts cut across GPU
batches.  Also the loop's argument checks."""
from __future__ import annotations

import ctypes
from collections import deque

import numpy as np
import pytest

import oracle
from upe_amd import gpu, synth
from upe_amd.layout import V_FWD, desc_lens, desc_offsets

pytestmark = pytest.mark.gpu

STRIDE = 2064   # the reference pktbuf_t stride: frames at 16-byte aligned offsets


class Pipeline:
    """Python stand-ins for worker_main's callees over a workload: handle h = packet index + 1."""

    def __init__(self, wl, burst_sizes, mapped, reload=None):
        self.wl = wl
        n = wl.n
        self.pool = gpu.PinnedArray((n * STRIDE + 2 * STRIDE,), np.uint8)
        self.base = self.pool.ptr
        self.off = 16 + STRIDE * np.arange(n, dtype=np.int64)   # data[] 16 bytes into each slot
        self.lens = desc_lens(wl.desc).astype(np.int64)
        src = desc_offsets(wl.desc)
        for i in range(n):
            self.pool.array[self.off[i]:self.off[i] + self.lens[i]] = \
                wl.frames[src[i]:src[i] + self.lens[i]]
        self.ring = deque(range(1, n + 1))
        self.sizes = list(burst_sizes)
        self.pops, self.tx, self.replies, self.freed = [], [], [], []
        self.arp, self.ndp = wl.arp.copy(), wl.ndp.copy()
        self.mapped = mapped
        self.published = 0
        # publishes with the context (nothing in flight): (pkts_matched, rule_stats packets)
        self.points = []
        self.in_flight_publishes = 0
        self.stats_cap = wl.capacity
        # reload = (sorted table B, capacity B, at): the program swaps the table between the
        # burst that ends before packet `at` and the one that starts there
        self.reload = reload
        self.reloaded = False
        self.popped = 0
        self.last_start = -1
        lib = oracle.oracle_lib()
        lib.upe_ref_arp_update.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                           ctypes.c_void_p]
        lib.upe_ref_ndp_update.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                           ctypes.c_void_p]
        self.olib = lib

        def pop(user, bufs, m):
            k = min(m, len(self.ring), self.sizes[len(self.pops) % len(self.sizes)])
            if self.reload and self.popped < self.reload[2]:
                k = min(k, self.reload[2] - self.popped)   # a burst boundary at the reload
            for j in range(k):
                bufs[j] = self.ring.popleft()
            if k:
                self.pops.append(k)
                self.last_start = self.popped
                self.popped += k
            return k

        def poll(user):
            return int(self.reload is not None and not self.reloaded and
                       self.last_start == self.reload[2])

        def sync(user, ctx):
            self.reloaded = True
            rs, cap, _ = self.reload
            return gpu.LIB.upe_gpu_reload_rules(ctx, rs.ctypes.data, len(rs), cap, None, 0)

        def index(b):
            return int(b) - 1

        def data(user, b):
            return self.base + int(self.off[index(b)])

        def length(user, b):
            return int(self.lens[index(b)])

        def free(user, b):
            self.freed.append(index(b))

        def to_index(ptr):
            return int((ptr - self.base - 16) // STRIDE)

        def tx_send(user, frame, ln):
            self.replies.append(to_index(frame))
            return 0

        def tx_batch(user, frames, lens, count):
            self.tx.append([to_index(frames[k]) for k in range(count)])
            return count

        def arp_update(user, ip, mac):
            self.olib.upe_ref_arp_update(self.arp.ctypes.data, len(self.arp), ip,
                                         ctypes.cast(mac, ctypes.c_void_p))

        def ndp_update(user, ip, mac):
            self.olib.upe_ref_ndp_update(self.ndp.ctypes.data, len(self.ndp),
                                         ctypes.cast(ip, ctypes.c_void_p),
                                         ctypes.cast(mac, ctypes.c_void_p))

        def load_neigh(user, ctx):
            return gpu.LIB.upe_gpu_load_neigh(ctx, self.arp.ctypes.data, len(self.arp),
                                              self.ndp.ctypes.data, len(self.ndp))

        def publish(user, ctx, counters):
            from upe_amd.layout import RULE_STAT_DTYPE

            self.published += 1
            c = np.frombuffer(ctypes.string_at(counters, gpu.COUNTERS_DTYPE.itemsize),
                              gpu.COUNTERS_DTYPE)
            if not ctx:
                self.in_flight_publishes += 1
                return
            st = np.zeros(self.stats_cap, RULE_STAT_DTYPE)
            if gpu.LIB.upe_gpu_get_stats(ctx, None, st.ctypes.data, self.stats_cap) == 0:
                self.points.append((int(c["pkts_matched"][0]), int(st["packets"].sum())))

        self.ops = gpu.WorkerOps(
            gpu.POP_FN(pop), gpu.STOP_FN(lambda u: 1), gpu.DATA_FN(data), gpu.LEN_FN(length),
            gpu.FREE_FN(free), gpu.TX_SEND_FN(tx_send), gpu.TX_BATCH_FN(tx_batch),
            gpu.ARP_UPDATE_FN(arp_update), gpu.NDP_UPDATE_FN(ndp_update), gpu.CTX_FN(load_neigh),
            gpu.POLL_FN(poll) if reload else gpu.POLL_FN(),
            gpu.CTX_FN(sync) if reload else gpu.CTX_FN(), gpu.PUBLISH_FN(publish))

    def run(self, w, batch):
        # (PinnedArray memory is mapped for the GPU already: no registration needed)
        cfg = gpu.WorkerCfg(batch, 32, self.base if self.mapped else None, 0,
                            self.pool.array.nbytes if self.mapped else 0)
        counters = np.zeros(1, gpu.COUNTERS_DTYPE)
        rc = gpu.LIB.upe_gpu_worker_run(w._ctx, ctypes.byref(self.ops), None, ctypes.byref(cfg),
                                        counters.ctypes.data)
        if rc != 0:
            raise gpu.UpeGpuError(gpu.LIB.upe_gpu_last_error().decode())
        return counters

    def frames(self):
        out = self.wl.frames.copy()
        src = desc_offsets(self.wl.desc)
        for i in range(self.wl.n):
            out[src[i]:src[i] + self.lens[i]] = \
                self.pool.array[self.off[i]:self.off[i] + self.lens[i]]
        return out


def _workload(kind):
    if kind == "B":
        return synth.config_b(n=20_000, seed=81)
    from test_gpu_control import with_control

    return with_control(synth.config_c(n=12_000, seed=82), 40, 82)


@pytest.mark.parametrize("mapped", [False, True], ids=["windows", "mapped"])
@pytest.mark.parametrize("kind,bursts,batch", [("B", [32], 4096), ("B", [7, 32, 1, 19], 1000),
                                               ("C+control", [32, 5], 65536),
                                               ("C+control", [13], 777)])
def test_worker_loop_equals_restated_worker(gpu_worker_factory, kind, bursts, batch, mapped):
    wl = _workload(kind)
    p = Pipeline(wl, bursts, mapped)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        counters = p.run(w, batch)
        _, stats = w.get_stats()
    finally:
        w.close()
    r = oracle.run_restated(wl, apply_control=True)
    for f in ("pkts_in", "pkts_parsed", "pkts_matched", "pkts_forwarded", "pkts_dropped",
              "pkts_consumed", "arp_learn", "arp_reply"):
        assert int(counters[f][0]) == int(r.counters[f][0]), f
    assert np.array_equal(stats, r.rule_stats)
    got = p.frames()
    assert np.array_equal(got, r.frames), "packet bytes differ from the restated worker's"
    keep = ["ip", "mac", "valid"]
    assert np.array_equal(p.arp[keep], r.arp[keep]) and np.array_equal(p.ndp[keep], r.ndp[keep])
    # the calls worker_main makes for the bursts popped
    assert sum(p.pops) == wl.n and sorted(p.freed) == list(range(wl.n))
    fwd = (r.verdict & 0xF) == V_FWD
    want, s = [], 0
    for k in p.pops:
        idx = (np.nonzero(fwd[s:s + k])[0] + s).tolist()
        if idx:
            want.append(idx)
        s += k
    assert p.tx == want
    assert p.replies == np.nonzero(r.verdict & 0x40)[0].tolist()
    assert p.published >= 1
    p.pool.free()


@pytest.mark.parametrize("mapped", [False, True], ids=["windows", "mapped"])
@pytest.mark.parametrize("name", ["B", "C"])
def test_worker_loop_rule_reload(gpu_worker_factory, name, mapped):
    """poll / sync: the program's rule swap seen between two bursts; the loop finishes the
    packets it holds with the old table, the context reloads (upe_gpu_reload_rules), and the
    rest of the stream runs with the new one — as the restated worker does in two segments
    (the reference-harness equivalence is tests/test_oracle.py)."""
    import dataclasses

    import reload_util
    from upe_amd.layout import RULE_STAT_DTYPE

    wl, rules_b, at, cap_b = reload_util.case(name)
    wl = dataclasses.replace(wl, desc=wl.desc[:60_000])
    at = 31_111
    rs_b = synth.build_rule_table(rules_b)
    p = Pipeline(wl, [32], mapped, reload=(rs_b, cap_b, at))
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        counters = p.run(w, 4096)
        st = np.zeros(cap_b, RULE_STAT_DTYPE)
        gpu._check(gpu.LIB.upe_gpu_get_stats(w._ctx, None, st.ctypes.data, cap_b), "stats")
    finally:
        w.close()
    assert p.reloaded
    ra = oracle.run_restated(dataclasses.replace(wl, desc=wl.desc[:at]))
    rb = oracle.run_restated(dataclasses.replace(wl, frames=ra.frames, desc=wl.desc[at:],
                                                 arp=ra.arp, ndp=ra.ndp, capacity=cap_b),
                             rules_sorted=rs_b, l1=ra.l1, counters=ra.counters,
                             rule_stats=np.zeros(cap_b, RULE_STAT_DTYPE))
    got = {f: int(counters[f][0]) for f in ("pkts_in", "pkts_parsed", "pkts_matched",
                                            "pkts_forwarded", "pkts_dropped")}
    want = {f: int(rb.counters[f][0]) for f in got}
    assert got == want
    assert np.array_equal(st, rb.rule_stats)
    assert np.array_equal(p.frames(), rb.frames)
    p.pool.free()


@pytest.mark.parametrize("mapped", [False, True], ids=["windows", "mapped"])
def test_worker_loop_publish_points(gpu_worker_factory, mapped):
    """with two batches in flight the loop publishes the counters alone (NULL
    context) and never calls into the context then; at points with nothing in flight (at least
    every 32 batches of a stream that never drains, and at the final drain) it passes the context,
    and the rule_stats read there sum exactly to the published pkts_matched."""
    wl = synth.config_b(n=20_000, seed=84)
    p = Pipeline(wl, [32], mapped)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        counters = p.run(w, 64)          # 313 batches of 64 packets, the ring never empty
    finally:
        w.close()
    batches = -(-wl.n // 64)
    assert p.in_flight_publishes >= batches // 2
    assert len(p.points) >= batches // 32
    assert all(m == s for m, s in p.points), p.points[:8]
    assert p.points[-1][0] == int(counters["pkts_matched"][0])
    assert sorted(p.freed) == list(range(wl.n))
    p.pool.free()


def test_worker_loop_failure_with_batches_in_flight(gpu_worker_factory):
    """a frame the loop must refuse (not 16-byte aligned inside the registered pool)
    several batches into a mapped stream of 4-packet batches, with two batches in flight: the call
    fails, and every popped handle is freed exactly once (the in-flight batches after the GPU is
    done with them, the rest of the burst, the TX queue)."""
    wl = synth.config_b(n=2_000, seed=85)
    p = Pipeline(wl, [7, 32, 5], True)
    bad = 301
    p.off[bad] += 8                   # its frame moves 8 bytes: no longer 16-byte aligned
    p.pool.array[p.off[bad]:p.off[bad] + p.lens[bad]] = \
        wl.frames[desc_offsets(wl.desc)[bad]:desc_offsets(wl.desc)[bad] + p.lens[bad]]
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        with pytest.raises(gpu.UpeGpuError, match="16-byte aligned"):
            p.run(w, 4)
    finally:
        w.close()
    popped = sum(p.pops)
    assert popped > bad
    assert sorted(p.freed) == list(range(popped)), "a popped handle freed twice or never"
    p.pool.free()


def test_worker_loop_argument_checks(gpu_worker_factory):
    wl = synth.config_b(n=64, seed=83)
    p = Pipeline(wl, [32], False)
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        bad = gpu.WorkerCfg(0, 65, None, 0, 0)   # bursts above UPE_TX_BATCH_MAX
        assert gpu.LIB.upe_gpu_worker_run(w._ctx, ctypes.byref(p.ops), None, ctypes.byref(bad),
                                          None) == -1
        assert b"burst" in gpu.LIB.upe_gpu_last_error()
        # mapped mode: the region's size is required, and a frame outside it never reaches the GPU
        small = gpu.WorkerCfg(0, 32, p.base, 0, 32)
        assert gpu.LIB.upe_gpu_worker_run(w._ctx, ctypes.byref(p.ops), None, ctypes.byref(small),
                                          None) == -1
        assert b"pool_bytes" in gpu.LIB.upe_gpu_last_error()
        short = gpu.WorkerCfg(0, 32, p.base, 0, 4 * STRIDE)   # the 5th frame lies past the end
        assert gpu.LIB.upe_gpu_worker_run(w._ctx, ctypes.byref(p.ops), None, ctypes.byref(short),
                                          None) == -1
        assert b"inside the registered pool" in gpu.LIB.upe_gpu_last_error()
        assert sorted(p.freed) == list(range(len(p.freed))) and len(p.freed) == sum(p.pops)
        ops = gpu.WorkerOps.from_buffer_copy(p.ops)
        ops.tx_send_batch = gpu.TX_BATCH_FN()
        pops = len(p.pops)
        assert gpu.LIB.upe_gpu_worker_run(w._ctx, ctypes.byref(ops), None, None, None) == -1
        assert len(p.pops) == pops, "nothing may be popped when the call is refused"
    finally:
        w.close()
        p.pool.free()
