"""Segmented replay of a packet stream through a GpuWorker, the way a GPU-backed worker thread
drives the batch ABI when control packets are present: the batch is
cut after every control packet, the control packet's table write is applied to the host copy of
the neighbour tables (restating arp_update / ndp_update, reference src/arp_table.c:26-53,
src/ndp_table.c:39-65, and the NDP option walk of src/worker.c:68-95), the new snapshot is
uploaded, and the next segment runs.  The L1 caches and counters stay on the device throughout.

Test helper only: the reference's own control plane owns these table writes in a deployment.
"""
from __future__ import annotations

import numpy as np

from upe_amd import gpu
from upe_amd.layout import desc_lens, desc_offsets
from upe_amd.synth import ndp_hash


def control_kind(frame: np.ndarray, ln: int):
    """('arp', spa, sha) | ('ndp', ip16, mac) | ('ndp', None, None) | None."""
    b = np.zeros(2048 + 128, np.uint8)
    k = min(ln, 2048)
    b[:k] = frame[:k]
    et = (int(b[12]) << 8) | int(b[13])
    if et == 0x0806:
        if b[14] == 0 and b[15] == 1 and b[16] == 8 and b[17] == 0 and b[18] == 6 and b[19] == 4:
            spa = int.from_bytes(bytes(b[28:32]), "big")
            return ("arp", spa, bytes(b[22:28]))
        return None
    if et == 0x86DD and ln >= 78 and b[20] == 58 and b[54] in (135, 136):
        typ = int(b[54])
        off = 78
        while off + 2 <= ln:
            ot, ol = int(b[off]), (int(b[off + 1]) * 8) & 0xFF   # uint8_t opt_len, src/worker.c:73
            if ol == 0 or off + ol > ln:
                break
            if typ == 135 and ot == 1 and ol >= 8:
                return ("ndp", bytes(b[22:38]), bytes(b[off + 2:off + 8]))
            if typ == 136 and ot == 2 and ol >= 8:
                return ("ndp", bytes(b[62:78]), bytes(b[off + 2:off + 8]))
            off += ol
        return ("ndp", None, None)
    return None


def arp_update(t, ip, mac):
    cap = len(t)
    idx = ip & (cap - 1)
    for i in range(cap):
        s = (idx + i) & (cap - 1)
        if not t["valid"][s] or t["ip"][s] == ip:
            t["valid"][s] = 1
            t["ip"][s] = ip
            t["mac"][s] = np.frombuffer(mac, np.uint8)
            return


def ndp_update(t, ip16, mac):
    cap = len(t)
    idx = ndp_hash(ip16, cap)
    ipa = np.frombuffer(ip16, np.uint8)
    for i in range(cap):
        s = (idx + i) & (cap - 1)
        if not t["valid"][s] or np.array_equal(t["ip"][s], ipa):
            t["valid"][s] = 1
            t["ip"][s] = ipa
            t["mac"][s] = np.frombuffer(mac, np.uint8)
            return


def run_stream(worker: gpu.GpuWorker, wl):
    """Process wl as a stream with exact control-packet semantics.  Returns
    (frames, verdict, arp, ndp) after the whole stream; counters/stats/L1 stay in `worker`."""
    offs = desc_offsets(wl.desc)
    lens = desc_lens(wl.desc)
    arp, ndp = wl.arp.copy(), wl.ndp.copy()
    ctrl = {}
    for i in range(wl.n):
        kind = control_kind(wl.frames[offs[i]:offs[i] + max(lens[i], 0) + 128], int(lens[i]))
        if kind is not None:
            ctrl[i] = kind
    cuts = sorted(ctrl) + [wl.n - 1]
    frames_out = wl.frames.copy()
    verdict = np.zeros(wl.n, np.uint32)
    start = 0
    for c in cuts:
        end = c + 1
        if end <= start:
            continue
        seg_desc = wl.desc[start:end]
        b = gpu.DeviceBatch(worker, frames_out, seg_desc)
        b.run()
        fr, v = b.fetch()
        b.free()
        frames_out = fr
        verdict[start:end] = v
        if c in ctrl:
            kind, ip, mac = ctrl[c]
            if kind == "arp":
                arp_update(arp, ip, mac)
            elif ip is not None:
                ndp_update(ndp, ip, mac)
            worker.load_neigh(arp, ndp)
        start = end
    return frames_out, verdict, arp, ndp
