"""numpy mirrors of the C ABI structs in include/upe_gpu.h (themselves ABI mirrors of the
reference layouts: rule_t include/rule_table.h:19-35, arp_entry_t include/arp_table.h:13-18,
ndp_entry_t include/ndp_table.h:13-18, rule_stat_t include/worker.h:18-21).

Plain data only; used by the ctypes bindings, the synthetic-workload generators and the tests.
"""
from __future__ import annotations

import numpy as np

RULE_DTYPE = np.dtype(
    {
        "names": ["priority", "ip_ver", "src_ip", "src_mask", "dst_ip", "dst_mask",
                  "src_port", "dst_port", "protocol", "action", "out_ifindex", "rule_id"],
        "formats": ["<u4", "u1", ("u1", 16), ("u1", 16), ("u1", 16), ("u1", 16),
                    "<u2", "<u2", "u1", "<i4", "<i4", "<u4"],
        "offsets": [0, 4, 8, 24, 40, 56, 72, 74, 76, 80, 84, 88],
        "itemsize": 92,
    }
)

ARP_DTYPE = np.dtype(
    {
        "names": ["ip", "mac", "update_at", "valid"],
        "formats": ["<u4", ("u1", 6), "<i8", "u1"],
        "offsets": [0, 4, 16, 24],
        "itemsize": 32,
    }
)

NDP_DTYPE = np.dtype(
    {
        "names": ["ip", "mac", "update_at", "valid"],
        "formats": [("u1", 16), ("u1", 6), "<i8", "u1"],
        "offsets": [0, 16, 24, 32],
        "itemsize": 40,
    }
)

RULE_STAT_DTYPE = np.dtype([("packets", "<u8"), ("bytes", "<u8")])

COUNTER_NAMES = ("pkts_in", "pkts_parsed", "pkts_matched", "pkts_forwarded", "pkts_dropped",
                 "pkts_consumed", "arp_learn", "arp_reply")
COUNTERS_DTYPE = np.dtype([(n, "<u8") for n in COUNTER_NAMES])

L1_DTYPE = np.dtype(
    {
        "names": ["last_arp_ip", "last_arp_mac", "last_ndp_ip", "last_ndp_mac"],
        "formats": ["<u4", ("u1", 6), ("u1", 16), ("u1", 6)],
        "offsets": [0, 4, 10, 26],
        "itemsize": 32,
    }
)

BATCH_INFO_DTYPE = np.dtype([("counters", COUNTERS_DTYPE), ("n_ctrl", "<u8"),
                             ("first_ctrl", "<u8")])
# upe_launch_info_t (include/upe_gpu.h)
LAUNCH_INFO_DTYPE = np.dtype({"names": ["variant", "grid", "deferred", "launches"],
                              "formats": ["<u4", "<u4", "<u4", "<u8"],
                              "offsets": [0, 4, 8, 16], "itemsize": 24})

# flow_key_t (reference include/parser.h:134-141; upe_flow_key_t, 44 bytes)
FLOW_KEY_DTYPE = np.dtype({"names": ["ip_ver", "src_ip", "dst_ip", "src_port", "dst_port",
                                     "protocol"],
                           "formats": ["u1", ("u1", 16), ("u1", 16), "<u2", "<u2", "u1"],
                           "offsets": [0, 4, 20, 36, 38, 40], "itemsize": 44})
# upe_rule_index_info_t (include/upe_gpu.h)
RULE_INDEX_INFO_DTYPE = np.dtype([("nodes", "<u8"), ("leaf_entries", "<u8"), ("depth4", "<u4"),
                                  ("depth6", "<u4"), ("max_leaf", "<u4"), ("trees", "<u4")])

# verdict word (include/upe_gpu.h)
V_DROP_PARSE, V_DROP_NOMATCH, V_DROP_RULE, V_DROP_TTL, V_FWD, V_CONSUMED, V_DROP_ACTION = range(7)
VERDICT_NAMES = ("DROP_PARSE", "DROP_NOMATCH", "DROP_RULE", "DROP_TTL", "FWD", "CONSUMED",
                 "DROP_ACTION")
VF_NEIGH_HIT, VF_ARP_LEARN, VF_ARP_REPLY, VF_L1_INIT = 0x10, 0x20, 0x40, 0x80

ACT_DROP, ACT_FWD = 0, 1

HDR_WINDOW = 96
FRAME_TAIL = 96
REWRITE_EXTENT = 48


def verdict_code(v: np.ndarray) -> np.ndarray:
    return v & 0xF


def verdict_rule(v: np.ndarray) -> np.ndarray:
    return (v >> 8).astype(np.int64) - 1


def make_desc(offsets: np.ndarray, lens: np.ndarray) -> np.ndarray:
    offsets = np.asarray(offsets, dtype=np.uint64)
    lens = np.asarray(lens, dtype=np.uint64)
    if np.any(lens > 0xFFFF):
        raise ValueError("frame length > 65535")
    return (offsets << np.uint64(16)) | lens


def desc_offsets(desc: np.ndarray) -> np.ndarray:
    return (desc >> np.uint64(16)).astype(np.int64)


def desc_lens(desc: np.ndarray) -> np.ndarray:
    return (desc & np.uint64(0xFFFF)).astype(np.int64)


def l1_zero() -> np.ndarray:
    """The L1 caches of a calloc'd worker_t (reference src/main.c:444)."""
    return np.zeros(1, dtype=L1_DTYPE)
