"""Error behaviour of the C ABI, as the reference's C interfaces behave:
-1 plus a message (upe_gpu_last_error), no exception across the ABI, and the context stays
usable afterwards — a refused call changes nothing (rule_table_add failing at capacity,
src/rule_table.c:133-136; arp_table_init requiring a power of two, src/arp_table.c:8-11)."""
from __future__ import annotations

import numpy as np
import pytest

import golden_io
from test_gpu_parity import _assert_same
from upe_amd import gpu, synth
from upe_amd.layout import ARP_DTYPE, NDP_DTYPE

pytestmark = pytest.mark.gpu


def _message(fn, *args):
    with pytest.raises(gpu.UpeGpuError) as e:
        fn(*args)
    return str(e.value)


def test_refused_calls_leave_the_context_usable(gpu_worker_factory):
    wl, ref = golden_io.load("config_b_small")
    w = gpu_worker_factory(wl.capacity)
    try:
        w.configure(wl)
        # more rules than the capacity given at open
        big = synth.rules_array([synth.make_rule(i, 0) for i in range(wl.capacity + 1)])
        assert "capacity" in _message(w.load_rules, synth.build_rule_table(big))
        # neighbour tables must have power-of-two capacities
        assert "power of two" in _message(w.load_neigh, np.zeros(12, ARP_DTYPE),
                                          np.zeros(16, NDP_DTYPE))
        # frames must be 16-byte aligned
        dev = w.malloc(4096)
        assert "16-byte aligned" in _message(w.process, dev + 4, dev, dev, 1)
        # verdict codes are 4 bits
        assert "out of range" in _message(w.compact, dev, 1, 16, dev, dev)
        # a timing span of zero calls
        assert "span" in _message(w.timing_span, 1, 0)
        # segmented batches need power-of-two tables too
        assert "powers of two" in _message(w.process_segmented, dev, dev, dev, 1,
                                           np.zeros(12, ARP_DTYPE), np.zeros(16, NDP_DTYPE))
        w.free(dev)
        # nothing above changed the context: the golden batch still comes out bit-exact
        _assert_same(gpu.run_workload(wl, worker=w), ref, "after refused calls")
    finally:
        w.close()
