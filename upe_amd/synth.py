"""Seeded synthetic workloads for the BASELINE.json configurations.

Everything here is deterministic given the seed (numpy PCG64), so the GPU box regenerates
byte-identical batches and the committed golden digests stay valid.  Frames are built in wire
order into a 2-D header matrix and then packed into the batch layout of include/upe_gpu.h
(16-byte aligned starts, uint64 descriptors, FRAME_TAIL bytes of tail padding).

Config names follow BASELINE.json "configs":
  A  10k x 64 B Eth/IPv4/UDP, rules.example (reference rules.example:3-25), CPU replay
  B  1M x 64 B IPv4/UDP, 8 rules (every field type), ARP 240/256 hit
  C  IMIX 64/570/1518 (7:4:1), 70 % IPv4 / 30 % IPv6, 1k 5-tuple rules, ARP+NDP ~600 each
  D  16M packets, 64k rules, IHL/doff 5-15, 10 % malformed, v4/v6 interleaved
"""
from __future__ import annotations

import dataclasses

import os

import numpy as np

from .layout import (ACT_DROP, ACT_FWD, ARP_DTYPE, FRAME_TAIL, HDR_WINDOW, NDP_DTYPE,
                     RULE_DTYPE, desc_lens, desc_offsets, l1_zero, make_desc)

PORT_MAC = bytes([0x02, 0x00, 0x00, 0x00, 0x00, 0x01])
PORT_IP4 = 0x0A8000FE  # 10.128.0.254


@dataclasses.dataclass
class Workload:
    name: str
    frames: np.ndarray        # uint8, packed batch + FRAME_TAIL padding
    desc: np.ndarray          # uint64 (offset << 16 | len)
    rules: np.ndarray         # RULE_DTYPE in insertion order (what rule_table_add receives)
    capacity: int             # rule table capacity (rule_stats size)
    arp: np.ndarray           # ARP_DTYPE slot array (power-of-two length)
    ndp: np.ndarray           # NDP_DTYPE slot array
    eth_addr: bytes = PORT_MAC
    ip4_addr: int = PORT_IP4
    l1: np.ndarray = dataclasses.field(default_factory=l1_zero)

    @property
    def n(self) -> int:
        return int(self.desc.shape[0])

    @property
    def rules_sorted(self) -> np.ndarray:
        return build_rule_table(self.rules)

    def copy(self) -> "Workload":
        return dataclasses.replace(self, frames=self.frames.copy(), desc=self.desc.copy(),
                                   arp=self.arp.copy(), ndp=self.ndp.copy(), l1=self.l1.copy())


# ---------------------------------------------------------------------------------------------
# rule table: rule_table_add semantics (reference src/rule_table.c:130-161), one sort at the end
# ---------------------------------------------------------------------------------------------

def ipv4_mask(prefix: int) -> int:
    """ipv4_mask_from_prefix, reference src/rule_table.c:14-30 (host-order value)."""
    if not 0 <= prefix <= 32:
        raise ValueError("prefix > 32")
    return 0 if prefix == 0 else (0xFFFFFFFF << (32 - prefix)) & 0xFFFFFFFF


def ipv6_mask(prefix: int) -> bytes:
    """ipv6_mask_from_prefix, reference src/rule_table.c:32-50."""
    if not 0 <= prefix <= 128:
        raise ValueError("prefix > 128")
    out = bytearray(16)
    for i in range(16):
        bits = prefix - 8 * i
        out[i] = 0xFF if bits >= 8 else (0 if bits <= 0 else (0xFF << (8 - bits)) & 0xFF)
    return bytes(out)


def build_rule_table(rules: np.ndarray) -> np.ndarray:
    """Final rt->rules after rule_table_add() of `rules` in order: rule_id = insertion index,
    wildcard (all-zero mask) addresses zeroed for ip_ver 4/6, sorted by (priority, rule_id)."""
    r = np.ascontiguousarray(rules).astype(RULE_DTYPE)   # (the 92-byte rule_t layout, padded)
    r["rule_id"] = np.arange(len(r), dtype=np.uint32)
    v4 = r["ip_ver"] == 4
    v6 = r["ip_ver"] == 6
    for a, m in (("src_ip", "src_mask"), ("dst_ip", "dst_mask")):
        mask_v4 = r[m][:, :4].copy().view("<u4").ravel()
        z4 = v4 & (mask_v4 == 0)
        r[a][z4, :4] = 0
        z6 = v6 & ~r[m].any(axis=1)
        r[a][z6] = 0
    order = np.lexsort((r["rule_id"], r["priority"]))
    return r[order]


def _set_v4(field: np.ndarray, value: int) -> None:
    field[:4] = np.frombuffer(np.uint32(value).astype("<u4").tobytes(), np.uint8)


def make_rule(priority: int, action: int, *, ip_ver: int | None = None, proto: int = 0,
              sport: int = 0, dport: int = 0, src=None, dst=None, out_ifindex: int = 1):
    """One rule_t.  src/dst: (int_v4, prefix) or (bytes16, prefix), like rule_config's
    parse_ip_prefix (reference src/rule_config.c:38-91): v4 host order, v6 wire bytes.
    ip_ver=None infers the version from the first address as rule_config_load does
    (src/rule_config.c:213-227); an explicit 0 keeps a version-agnostic rule (API-only)."""
    r = np.zeros(1, dtype=RULE_DTYPE)[0]
    r["priority"] = priority
    infer = ip_ver is None
    r["ip_ver"] = 0 if infer else ip_ver
    r["protocol"] = proto
    r["src_port"] = sport
    r["dst_port"] = dport
    r["action"] = action
    r["out_ifindex"] = out_ifindex if action == ACT_FWD else 0
    for name, spec in (("src", src), ("dst", dst)):
        if spec is None:
            continue
        addr, prefix = spec
        if isinstance(addr, (bytes, bytearray)):
            r[name + "_ip"][:] = np.frombuffer(bytes(addr), np.uint8)
            r[name + "_mask"][:] = np.frombuffer(ipv6_mask(prefix), np.uint8)
            if infer and r["ip_ver"] == 0:
                r["ip_ver"] = 6
        else:
            _set_v4(r[name + "_ip"], addr)
            _set_v4(r[name + "_mask"], ipv4_mask(prefix))
            if infer and r["ip_ver"] == 0:
                r["ip_ver"] = 4
    return r


def rules_array(rules) -> np.ndarray:
    out = np.zeros(len(rules), dtype=RULE_DTYPE)
    for i, r in enumerate(rules):
        out[i] = r
    return out


# ---------------------------------------------------------------------------------------------
# neighbour tables: arp_update / ndp_update insertion (reference src/arp_table.c:26-53,
# src/ndp_table.c:39-65), so slot placement (and probe chains) match a learned table.
# ---------------------------------------------------------------------------------------------

def ndp_hash(ip16: bytes, cap: int) -> int:
    w = np.frombuffer(bytes(ip16), "<u4")
    return int(w[0] ^ w[1] ^ w[2] ^ w[3]) & (cap - 1)


def arp_table(cap: int, entries) -> np.ndarray:
    t = np.zeros(cap, dtype=ARP_DTYPE)
    for ip, mac in entries:
        idx = ip & (cap - 1)
        for i in range(cap):
            s = (idx + i) & (cap - 1)
            if not t["valid"][s] or t["ip"][s] == ip:
                t["valid"][s] = 1
                t["ip"][s] = ip
                t["mac"][s] = np.frombuffer(bytes(mac), np.uint8)
                break
    return t


def ndp_table(cap: int, entries) -> np.ndarray:
    t = np.zeros(cap, dtype=NDP_DTYPE)
    for ip, mac in entries:
        idx = ndp_hash(ip, cap)
        ipa = np.frombuffer(bytes(ip), np.uint8)
        for i in range(cap):
            s = (idx + i) & (cap - 1)
            if not t["valid"][s] or np.array_equal(t["ip"][s], ipa):
                t["valid"][s] = 1
                t["ip"][s] = ipa
                t["mac"][s] = np.frombuffer(bytes(mac), np.uint8)
                break
    return t


# ---------------------------------------------------------------------------------------------
# vectorised frame building
# ---------------------------------------------------------------------------------------------

def _be16(h: np.ndarray, off, val) -> None:
    val = np.asarray(val, dtype=np.uint32)
    h[:, off] = (val >> 8) & 0xFF
    h[:, off + 1] = val & 0xFF


def _be32(h: np.ndarray, off, val) -> None:
    val = np.asarray(val, dtype=np.uint64)
    for k in range(4):
        h[:, off + k] = (val >> np.uint64(24 - 8 * k)) & np.uint64(0xFF)


def ipv4_header_checksum(h: np.ndarray, ihl: np.ndarray) -> np.ndarray:
    """Wire checksum of the IPv4 header at byte 14 (RFC 1071), for realistic input frames."""
    n = h.shape[0]
    if h.shape[1] < 76:
        h = np.concatenate([h, np.zeros((n, 76 - h.shape[1]), h.dtype)], axis=1)
    words = (h[:, 14:74:2].astype(np.uint32) << 8) | h[:, 15:75:2].astype(np.uint32)
    valid = np.arange(30)[None, :] < (ihl[:, None] * 2)
    words = np.where(valid, words, 0)
    words[:, 5] = 0  # checksum field
    s = words.sum(axis=1)
    while np.any(s >> 16):
        s = (s & 0xFFFF) + (s >> 16)
    return (~s & 0xFFFF).astype(np.uint32).reshape(n)


def pack_frames(hdr: np.ndarray, lens: np.ndarray, stride: int | None = None,
                align: int = 16, line_aligned: bool = False) -> tuple[np.ndarray, np.ndarray]:
    """Pack header rows (first hdr.shape[1] bytes of each frame; the rest of a frame is zero
    payload) into one buffer.  Fixed `stride` or variable (len rounded up to `align`)."""
    n, w = hdr.shape
    lens = np.asarray(lens, dtype=np.int64)
    if stride is not None:
        if np.any(lens > stride):
            raise ValueError("frame longer than stride")
        offs = np.arange(n, dtype=np.int64) * stride
        total = n * stride
    elif line_aligned:
        # every frame's header window inside one 128-byte line: frames of up to 64 bytes start
        # on a 64-byte boundary, longer ones on a 128-byte boundary
        sizes = np.maximum((lens + 15) // 16 * 16, 16)
        aligns = np.where(lens <= 64, 64, 128)
        offs = np.zeros(n, dtype=np.int64)
        end = 0
        for i in range(n):
            a = int(aligns[i])
            o = (end + a - 1) // a * a
            offs[i] = o
            end = o + int(sizes[i])
        total = end
    else:
        sizes = (lens + align - 1) // align * align
        sizes = np.maximum(sizes, align)
        offs = np.zeros(n, dtype=np.int64)
        np.cumsum(sizes[:-1], out=offs[1:])
        total = int(offs[-1] + sizes[-1]) if n else 0
    buf = np.zeros(total + FRAME_TAIL + 128, dtype=np.uint8)
    keep = np.minimum(lens, w)
    if stride is not None and stride >= w:
        view = buf[: n * stride].reshape(n, stride)
        cols = np.arange(w, dtype=np.int64)[None, :]
        for s in range(0, n, 1 << 18):   # chunks: no full-size mask or temporary
            e = min(n, s + (1 << 18))
            np.multiply(hdr[s:e], cols < keep[s:e, None], out=view[s:e, :w], casting="unsafe")
    else:
        chunk = 1 << 16
        cols = np.arange(w)
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            m = cols[None, :] < keep[s:e, None]
            idx = offs[s:e, None] + cols[None, :]
            buf[idx[m]] = hdr[s:e][m]
    return buf, make_desc(offs, lens)


def _macs(h: np.ndarray, rng: np.random.Generator) -> None:
    n = h.shape[0]
    h[:, 0:6] = rng.integers(0, 256, size=(n, 6), dtype=np.uint8)
    h[:, 0] &= 0xFE
    h[:, 6:12] = rng.integers(0, 256, size=(n, 6), dtype=np.uint8)
    h[:, 6] &= 0xFE


def build_ipv4(h, rows, *, src, dst, proto, ttl, ihl, total_len, l4_ports, tcp_doff=None,
               icmp=None, rng=None):
    """Fill IPv4 frames in rows of h (wire order)."""
    hh = h[rows]
    _be16(hh, 12, 0x0800)
    hh[:, 14] = 0x40 | ihl
    hh[:, 15] = 0
    _be16(hh, 16, total_len)
    if rng is not None:
        _be16(hh, 18, rng.integers(0, 65536, size=len(rows)))
    _be16(hh, 20, 0x4000)
    hh[:, 22] = ttl
    hh[:, 23] = proto
    _be32(hh, 26, src)
    _be32(hh, 30, dst)
    # options: NOP padding (0x01) then EOL, as a real stack would emit
    for extra in np.unique(ihl[ihl > 5]):
        sel = ihl == extra
        hh[np.ix_(sel, np.arange(34, 14 + int(extra) * 4))] = 1
    l4 = 14 + ihl.astype(np.int64) * 4
    sport, dport = l4_ports
    r = np.arange(len(rows))
    for k, val in ((0, sport >> 8), (1, sport & 0xFF), (2, dport >> 8), (3, dport & 0xFF)):
        hh[r, l4 + k] = val
    if tcp_doff is not None:
        hh[r, l4 + 12] = np.where(proto == 6, tcp_doff << 4, hh[r, l4 + 12])
        hh[r, l4 + 13] = np.where(proto == 6, 0x10, hh[r, l4 + 13])
    if icmp is not None:
        itype, icode, iid = icmp
        isi = proto == 1
        hh[r[isi], l4[isi]] = itype[isi]
        hh[r[isi], l4[isi] + 1] = icode[isi]
        hh[r[isi], l4[isi] + 2] = 0
        hh[r[isi], l4[isi] + 3] = 0
        hh[r[isi], l4[isi] + 4] = iid[isi] >> 8
        hh[r[isi], l4[isi] + 5] = iid[isi] & 0xFF
    cs = ipv4_header_checksum(hh, ihl.astype(np.int64))
    _be16(hh, 24, cs)
    h[rows] = hh


def build_ipv6(h, rows, *, src16, dst16, nh, hop, payload_len, sport, dport, tcp_doff=None):
    hh = h[rows]
    _be16(hh, 12, 0x86DD)
    _be32(hh, 14, np.full(len(rows), 0x60000000, dtype=np.uint64))
    _be16(hh, 18, payload_len)
    hh[:, 20] = nh
    hh[:, 21] = hop
    hh[:, 22:38] = src16
    hh[:, 38:54] = dst16
    _be16(hh, 54, sport)
    _be16(hh, 56, dport)
    if tcp_doff is not None:
        hh[:, 66] = np.where(nh == 6, tcp_doff << 4, hh[:, 66])
        hh[:, 67] = np.where(nh == 6, 0x10, hh[:, 67])
    h[rows] = hh


def _rand_macs(rng, k):
    m = rng.integers(0, 256, size=(k, 6), dtype=np.uint8)
    m[:, 0] = (m[:, 0] & 0xFE) | 0x02
    return m


# ---------------------------------------------------------------------------------------------
# config A — reference rules.example over 64 B UDP/IPv4
# ---------------------------------------------------------------------------------------------

def rules_example() -> np.ndarray:
    """reference rules.example:3-25 as rule_config_load would add them (out_iface = lo -> 1)."""
    return rules_array([
        make_rule(5, ACT_DROP, proto=6, dport=22),
        make_rule(1000, ACT_FWD, ip_ver=4, proto=6, src=(0xC0A80000, 16)),
        make_rule(1200, ACT_FWD, ip_ver=6, src=(bytes.fromhex("20010db8") + bytes(12), 32)),
        make_rule(9999, ACT_DROP),
    ])


def _udp64(n, rng, dst_pool):
    h = np.zeros((n, 64), dtype=np.uint8)
    _macs(h, rng)
    src = (np.uint64(0x0A000000) + rng.integers(0, 1 << 24, size=n).astype(np.uint64))
    dst = dst_pool[rng.integers(0, len(dst_pool), size=n)].astype(np.uint64)
    sport = rng.integers(1, 65536, size=n).astype(np.uint32)
    dport = rng.integers(1, 65536, size=n).astype(np.uint32)
    return h, src, dst, sport, dport


def config_a(n: int = 10_000, seed: int = 1) -> Workload:
    rng = np.random.default_rng(seed)
    dst_pool = np.uint64(0x0A800000) + np.arange(256, dtype=np.uint64)
    h, src, dst, sport, dport = _udp64(n, rng, dst_pool)
    rows = np.arange(n)
    build_ipv4(h, rows, src=src, dst=dst, proto=np.full(n, 17), ttl=np.full(n, 64),
               ihl=np.full(n, 5), total_len=np.full(n, 50), l4_ports=(sport, dport), rng=rng)
    _be16(h, 38, np.full(n, 30))
    frames, desc = pack_frames(h, np.full(n, 64), stride=64)
    return Workload("A", frames, desc, rules_example(), 1024,
                    np.zeros(1024, ARP_DTYPE), np.zeros(1024, NDP_DTYPE))


# ---------------------------------------------------------------------------------------------
# config B — 1M x 64 B UDP/IPv4, 8 rules exercising every field type
# ---------------------------------------------------------------------------------------------

def rules_b() -> np.ndarray:
    """Eight rules, inserted out of priority order so the (priority, rule_id) sort matters."""
    return rules_array([
        make_rule(9999, ACT_DROP),                                            # catch-all
        make_rule(40, ACT_FWD, dst=(0x0A800000, 25)),                         # v4 dst /25
        make_rule(10, ACT_FWD, dport=53),                                     # port only
        make_rule(20, ACT_DROP, src=(0x0A010000, 16)),                        # v4 src /16
        make_rule(30, ACT_DROP, proto=6, dport=22),                           # never (all UDP)
        make_rule(50, ACT_FWD, src=(bytes.fromhex("20010db8") + bytes(12), 32)),  # v6 only
        make_rule(60, ACT_DROP, sport=1234),                                  # port only
        make_rule(70, ACT_DROP, proto=1),                                     # icmp
    ])


def neigh_b(rng) -> np.ndarray:
    """ARP: 240 of the 256 hosts of 10.128.0.0/24, after 64 colliding hosts of 10.129.0.0/24
    (same low 10 bits, so lookups walk probe chains as in a learned table)."""
    ents = []
    for x in rng.permutation(256)[:64]:
        ents.append((0x0A810000 + int(x), _rand_macs(rng, 1)[0].tobytes()))
    for x in rng.permutation(256)[:240]:
        ents.append((0x0A800000 + int(x), _rand_macs(rng, 1)[0].tobytes()))
    return arp_table(1024, ents)


def config_b(n: int = 1 << 20, seed: int = 2) -> Workload:
    rng = np.random.default_rng(seed)
    arp = neigh_b(rng)
    dst_pool = np.uint64(0x0A800000) + np.arange(256, dtype=np.uint64)
    h, src, dst, sport, dport = _udp64(n, rng, dst_pool)
    dport = np.where(rng.integers(0, 8, size=n) == 0, 53, dport).astype(np.uint32)
    sport = np.where(rng.integers(0, 64, size=n) == 0, 1234, sport).astype(np.uint32)
    ttl = rng.integers(1, 65, size=n)
    rows = np.arange(n)
    build_ipv4(h, rows, src=src, dst=dst, proto=np.full(n, 17), ttl=ttl, ihl=np.full(n, 5),
               total_len=np.full(n, 50), l4_ports=(sport, dport), rng=rng)
    _be16(h, 38, np.full(n, 30))
    frames, desc = pack_frames(h, np.full(n, 64), stride=64)
    return Workload("B", frames, desc, rules_b(), 1024, arp, np.zeros(1024, NDP_DTYPE))


# ---------------------------------------------------------------------------------------------
# config C — IMIX, v4+v6, 1k 5-tuple rules, ARP + NDP
# ---------------------------------------------------------------------------------------------

def _v6_pool(rng, k, prefix=bytes.fromhex("20010db8")):
    tail = rng.integers(0, 256, size=(k, 12), dtype=np.uint8)
    tail[:, :6] = rng.integers(0, 4, size=(k, 6), dtype=np.uint8)  # clustered subnets
    pre = np.frombuffer(prefix, np.uint8)[None, :].repeat(k, axis=0)
    return np.concatenate([pre, tail], axis=1)


def _mixed_rules(rng, n_rules, v4_src, v4_dst, v6_src, v6_dst, protos4, protos6, ports,
                 exact_frac=0.0, wildcards_last=False):
    """Random 5-tuple rules drawn from the traffic's own pools so they match at spread-out
    positions; last rule is the catch-all.  wildcards_last: a draw that constrains nothing but
    the IP version (a catch-all for its family) goes after every constraining rule — config C's
    seed-3 draw has an IPv6 one at priority 1, DROP, which takes every IPv6 packet (so C as
    SURVEY.md pins it forwards IPv4 only); with it last, IPv6 packets reach the NDP lookup."""
    rules = []
    prios = rng.permutation(n_rules - 1) + 1
    for i in range(n_rules - 1):
        is6 = rng.random() < 0.3
        act = ACT_FWD if rng.random() < 0.5 else ACT_DROP
        exact = rng.random() < exact_frac
        kw = {}
        if is6:
            kw["ip_ver"] = 6
            if exact or rng.random() < 0.7:
                kw["src"] = (bytes(v6_src[rng.integers(len(v6_src))]),
                             128 if exact else int(rng.integers(32, 129)))
            if exact or rng.random() < 0.7:
                kw["dst"] = (bytes(v6_dst[rng.integers(len(v6_dst))]),
                             128 if exact else int(rng.integers(32, 129)))
            if exact or rng.random() < 0.5:
                kw["proto"] = int(rng.choice(protos6))
        else:
            kw["ip_ver"] = 4
            if exact or rng.random() < 0.7:
                kw["src"] = (int(v4_src[rng.integers(len(v4_src))]),
                             32 if exact else int(rng.integers(8, 33)))
            if exact or rng.random() < 0.7:
                kw["dst"] = (int(v4_dst[rng.integers(len(v4_dst))]),
                             32 if exact else int(rng.integers(8, 33)))
            if exact or rng.random() < 0.5:
                kw["proto"] = int(rng.choice(protos4))
        if exact or rng.random() < 0.3:
            kw["sport"] = int(ports[rng.integers(len(ports))])
        if exact or rng.random() < 0.4:
            kw["dport"] = int(ports[rng.integers(len(ports))])
        if rng.random() < 0.1 and not exact:
            kw["ip_ver"] = 0  # version-agnostic: address bytes apply under both views
        if wildcards_last and not any(k in kw for k in ("src", "dst", "proto", "sport", "dport")):
            prios[i] += n_rules
        rules.append(make_rule(int(prios[i]), act, **kw))
    rules.append(make_rule(1 << 30, ACT_DROP))
    return rules_array(rules)


def mixed_table(n_rules: int, seed: int) -> np.ndarray:
    """A config-C-style table of n_rules random rules (_mixed_rules: prefixes /8-/32 and /32-/128
    drawn from config C's host pools, ports exact or 0, 10 % version-agnostic): thousands of mask
    signatures, so neither the tuple-space index nor an LDS copy applies (the 64k-rule parity test
    and its timing probe)."""
    rng = np.random.default_rng(seed)
    n_hosts = 1000
    v4_src = (0x0A000000 + rng.integers(0, 1 << 16, size=n_hosts) * 7).astype(np.uint64)
    v4_dst = (0xAC100000 + rng.integers(0, 1 << 12, size=n_hosts)).astype(np.uint64)
    v6_src = _v6_pool(rng, n_hosts)
    v6_dst = _v6_pool(rng, n_hosts, prefix=bytes.fromhex("2001db80"))
    ports = np.concatenate([np.array([53, 80, 443, 22, 123, 8080]),
                            rng.integers(1024, 65536, size=200)])
    return _mixed_rules(rng, n_rules, v4_src, v4_dst, v6_src, v6_dst, [17, 6, 1], [17, 6], ports)


def config_c(n: int = 1 << 20, seed: int = 3, n_rules: int = 1024,
             v6_forwarding: bool = False) -> Workload:
    """BASELINE configs[2] as SURVEY.md §5 pins it (seed 3).  v6_forwarding: the same traffic
    and rules with the family-wide wildcards moved last (`_mixed_rules` wildcards_last), so
    that IPv6 packets are forwarded through the NDP lookup (the "C6" variant)."""
    rng = np.random.default_rng(seed)
    n_hosts = 1000
    v4_src = (0x0A000000 + rng.integers(0, 1 << 16, size=n_hosts) * 7).astype(np.uint64)
    v4_dst = (0xAC100000 + rng.integers(0, 1 << 12, size=n_hosts)).astype(np.uint64)
    v6_src = _v6_pool(rng, n_hosts)
    v6_dst = _v6_pool(rng, n_hosts, prefix=bytes.fromhex("2001db80"))
    ports = np.concatenate([np.array([53, 80, 443, 22, 123, 8080]),
                            rng.integers(1024, 65536, size=200)])
    arp = arp_table(1024, [(int(ip), _rand_macs(rng, 1)[0].tobytes())
                           for ip in v4_dst[rng.permutation(n_hosts)[:600]]])
    ndp = ndp_table(1024, [(bytes(ip), _rand_macs(rng, 1)[0].tobytes())
                           for ip in v6_dst[rng.permutation(n_hosts)[:600]]])
    rules = _mixed_rules(rng, n_rules, v4_src, v4_dst, v6_src, v6_dst, [17, 6, 1], [17, 6], ports,
                         wildcards_last=v6_forwarding)

    size = rng.choice(np.array([64, 570, 1518]), size=n, p=[7 / 12, 4 / 12, 1 / 12])
    is6 = rng.random(n) < 0.3
    h = np.zeros((n, 128), dtype=np.uint8)
    _macs(h, rng)
    sport = ports[rng.integers(0, len(ports), size=n)].astype(np.uint32)
    dport = ports[rng.integers(0, len(ports), size=n)].astype(np.uint32)
    r4 = np.nonzero(~is6)[0]
    r6 = np.nonzero(is6)[0]
    p4 = rng.choice(np.array([17, 6, 1]), size=len(r4), p=[0.5, 0.4, 0.1])
    itype = rng.choice(np.array([0, 8, 3, 11]), size=len(r4)).astype(np.uint32)
    icode = rng.integers(0, 4, size=len(r4)).astype(np.uint32)
    build_ipv4(h, r4, src=v4_src[rng.integers(0, n_hosts, size=len(r4))],
               dst=v4_dst[rng.integers(0, n_hosts, size=len(r4))], proto=p4,
               ttl=rng.integers(1, 129, size=len(r4)), ihl=np.full(len(r4), 5),
               total_len=size[r4] - 14, l4_ports=(sport[r4], dport[r4]),
               tcp_doff=np.full(len(r4), 5), icmp=(itype, icode, sport[r4]), rng=rng)
    p6 = rng.choice(np.array([17, 6]), size=len(r6))
    build_ipv6(h, r6, src16=v6_src[rng.integers(0, n_hosts, size=len(r6))],
               dst16=v6_dst[rng.integers(0, n_hosts, size=len(r6))], nh=p6,
               hop=rng.integers(1, 129, size=len(r6)), payload_len=size[r6] - 54,
               sport=sport[r6], dport=dport[r6], tcp_doff=np.full(len(r6), 5))
    frames, desc = pack_frames(h, size,
                               line_aligned=os.environ.get("UPE_SYNTH_LAYOUT") == "line")
    return Workload("C", frames, desc, rules, n_rules, arp, ndp)


# ---------------------------------------------------------------------------------------------
# config C, flow-derived (round 5): the same IMIX traffic mix and rule shape as config_c, but every
# rule is cut from a flow of the traffic and kept selective, so that first-match positions spread
# over the whole 1k table for BOTH families (seed-3 config_c stops every IPv4 packet at sorted
# rule 11 and every IPv6 packet at rule 0, a priority-1 IPv6 wildcard DROP)
# ---------------------------------------------------------------------------------------------

V4_SRC_BASE = 0x0A000000     # IPv4 sources: 10.0.0.0/8
V4_DST_BASE = 0xAC100000     # IPv4 destinations: a pool of hosts in 172.16.0.0/12
V6_SRC_PRE = bytes.fromhex("20010db8")
V6_DST_PRE = bytes.fromhex("2001db80")
C_PROTO4 = (np.array([17, 6, 1]), np.array([0.5, 0.4, 0.1]))
C_PROTO6 = (np.array([17, 6]), np.array([0.5, 0.5]))


def _v6_mask_arr(prefix: int) -> np.ndarray:
    return np.frombuffer(ipv6_mask(prefix), np.uint8)


def _flow_rules(rng, n_rules, dst4, dst6, ports, max_cover):
    """Rules 0..n_rules-2 (the catch-all is appended by the caller), each cut from a random flow:
    prefixes /8-/32 (IPv4) and /32-/128 (IPv6) or wildcards, protocol and ports exact or 0, 50/50
    FWD / DROP, 5 % version-agnostic.  A draw whose estimated share of its family's traffic
    exceeds max_cover is tightened (a longer prefix, or one more exact field) until it does not,
    so that no rule covers the traffic pool: a packet cut from rule j's flow first matches rule j
    (or, rarely, an earlier rule that happens to cover it)."""
    specs = []
    prios = rng.permutation(n_rules - 1) + 1
    for i in range(n_rules - 1):
        fam = 6 if rng.random() < 0.3 else 4
        agnostic = rng.random() < 0.05
        if fam == 4:
            src = V4_SRC_BASE | int(rng.integers(0, 1 << 24))
            di = int(rng.integers(len(dst4)))
            proto = int(rng.choice(C_PROTO4[0], p=C_PROTO4[1]))
            lo_len, hi_len = 8, 32
        else:
            src = V6_SRC_PRE + bytes(rng.integers(0, 256, size=12, dtype=np.uint8))
            di = int(rng.integers(len(dst6)))
            proto = int(rng.choice(C_PROTO6[0], p=C_PROTO6[1]))
            lo_len, hi_len = 32, 128
        ls = int(rng.integers(lo_len, hi_len + 1)) if rng.random() < 0.7 else None
        ld = int(rng.integers(lo_len, hi_len + 1)) if rng.random() < 0.7 else None
        has = {"proto": rng.random() < 0.5, "sport": rng.random() < 0.3,
               "dport": rng.random() < 0.4}
        if agnostic and rng.random() < 0.5:
            ls = ld = None   # ports / protocol only: the rule applies to both families
        sport = int(ports[rng.integers(len(ports))])
        dport = int(ports[rng.integers(len(ports))])

        def dst_pool_in(l):
            if l is None:
                return None
            if fam == 4:
                m = ipv4_mask(l)
                return np.nonzero((dst4.astype(np.uint64) & m) == (int(dst4[di]) & m))[0]
            m = _v6_mask_arr(l)
            return np.nonzero(np.all((dst6 & m) == (dst6[di] & m), axis=1))[0]

        def cover():
            c = 1.0
            if ls is not None:
                c *= 2.0 ** -(max(ls, lo_len) - lo_len)
            if ld is not None:
                c *= len(dst_pool_in(ld)) / (len(dst4) if fam == 4 else len(dst6))
            if has["proto"]:
                tab = C_PROTO4 if fam == 4 else C_PROTO6
                c *= float(tab[1][list(tab[0]).index(proto)])
            c *= (1.0 / len(ports)) ** (int(has["sport"]) + int(has["dport"]))
            return c

        tries = 0
        while cover() > max_cover:
            k = int(rng.integers(0, 5))
            tries += 1
            # (a ports-only version-agnostic rule gets an address too once its ports and
            # protocol alone cannot reach max_cover)
            if k == 0 and not (agnostic and ls is None and tries < 16):
                ls = lo_len if ls is None else min(hi_len, ls + 4)
            elif k == 1 and not (agnostic and ld is None and tries < 16):
                ld = lo_len if ld is None else min(hi_len, ld + 4)
            elif k == 2:
                has["proto"] = True
            elif k == 3:
                has["sport"] = True
            elif k == 4:
                has["dport"] = True
        specs.append(dict(fam=fam, ver=0 if agnostic else fam, src=src, ls=ls, di=di, ld=ld,
                          proto=proto if has["proto"] else 0,
                          sport=sport if has["sport"] else 0,
                          dport=dport if has["dport"] else 0,
                          act=ACT_FWD if rng.random() < 0.5 else ACT_DROP,
                          prio=int(prios[i]), pool=dst_pool_in(ld)))
    rules = []
    for s in specs:
        dst = (int(dst4[s["di"]]) if s["fam"] == 4 else bytes(dst6[s["di"]]))
        rules.append(make_rule(s["prio"], s["act"], ip_ver=s["ver"], proto=s["proto"],
                               sport=s["sport"], dport=s["dport"],
                               src=None if s["ls"] is None else (s["src"], s["ls"]),
                               dst=None if s["ld"] is None else (dst, s["ld"])))
    rules.append(make_rule(1 << 30, ACT_DROP))
    return specs, rules_array(rules)


def config_c_flows(n: int = 1 << 20, seed: int = 3, n_rules: int = 1024,
                   max_cover: float = 2.0 ** -14, stray: float = 0.05) -> Workload:
    """BASELINE configs[2] with first-match positions spread over the table (the bench's `imix`
    leg from round 5; `config_c` seed 3 is kept as `imix_seed3`).  Traffic as SURVEY.md §8(d)
    row C: IMIX 64/570/1518 (7:4:1; a frame is never shorter than its headers), 70 % IPv4 (UDP 50 /
    TCP 40 / ICMP 10 %), 30 % IPv6 (UDP / TCP); 1k rules (`_flow_rules`) + the catch-all; ARP and
    NDP hold 600 of the 1000 destination hosts of each family.  Each packet is cut from a random
    rule's flow (fields the rule constrains by prefix randomised inside the prefix, the
    destination drawn from the pool hosts inside it; wildcard fields drawn from the traffic's
    distributions), except `stray` of them drawn with no rule in mind (the catch-all, after a
    scan of the whole table)."""
    rng = np.random.default_rng(seed + 7000)
    n_hosts = 1000
    dst4 = (V4_DST_BASE + rng.choice(1 << 20, size=n_hosts, replace=False)).astype(np.uint64)
    dst6 = _v6_pool(rng, n_hosts, prefix=V6_DST_PRE)
    ports = np.concatenate([np.array([53, 80, 443, 22, 123, 8080]),
                            rng.integers(1024, 65536, size=200)])
    arp = arp_table(1024, [(int(ip), _rand_macs(rng, 1)[0].tobytes())
                           for ip in dst4[rng.permutation(n_hosts)[:600]]])
    ndp = ndp_table(1024, [(bytes(ip), _rand_macs(rng, 1)[0].tobytes())
                           for ip in dst6[rng.permutation(n_hosts)[:600]]])
    specs, rules = _flow_rules(rng, n_rules, dst4, dst6, ports, max_cover)

    # per-rule arrays, and a last pseudo-rule with every field a wildcard (the strays)
    R = len(specs) + 1
    fam = np.array([s["fam"] for s in specs] + [4])
    agn = np.array([s["ver"] == 0 and s["ls"] is None and s["ld"] is None for s in specs] + [True])
    src4 = np.array([s["src"] if s["fam"] == 4 else V4_SRC_BASE for s in specs] + [V4_SRC_BASE],
                    dtype=np.uint64)
    m4s = np.array([ipv4_mask(s["ls"]) if s["fam"] == 4 and s["ls"] is not None else
                    ipv4_mask(8) for s in specs] + [ipv4_mask(8)], dtype=np.uint64)
    src6 = np.stack([np.frombuffer(s["src"], np.uint8) if s["fam"] == 6 else
                     np.frombuffer(V6_SRC_PRE + bytes(12), np.uint8) for s in specs] +
                    [np.frombuffer(V6_SRC_PRE + bytes(12), np.uint8)])
    m6s = np.stack([_v6_mask_arr(s["ls"] if s["fam"] == 6 and s["ls"] is not None else 32)
                    for s in specs] + [_v6_mask_arr(32)])
    pools = [s["pool"] if s["pool"] is not None else None for s in specs] + [None]
    cnt = np.array([len(p) if p is not None else 0 for p in pools])
    off = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    flat = np.concatenate([p for p in pools if p is not None] + [np.zeros(1, np.int64)])
    r_proto = np.array([s["proto"] for s in specs] + [0])
    r_sport = np.array([s["sport"] for s in specs] + [0])
    r_dport = np.array([s["dport"] for s in specs] + [0])

    j = rng.integers(0, R - 1, size=n)
    j = np.where(rng.random(n) < stray, R - 1, j)
    # family: the rule's, or 70/30 for rules that constrain no address (and strays)
    is6 = np.where(agn[j], rng.random(n) < 0.3, fam[j] == 6)
    r4 = np.nonzero(~is6)[0]
    r6 = np.nonzero(is6)[0]
    # protocol, ports
    p4 = rng.choice(C_PROTO4[0], size=n, p=C_PROTO4[1])
    p6 = rng.choice(C_PROTO6[0], size=n, p=C_PROTO6[1])
    proto = np.where(r_proto[j] != 0, r_proto[j], np.where(is6, p6, p4))
    proto = np.where(is6 & (proto == 1), 17, proto)   # (an ICMP rule of a version-0 draw)
    sport = np.where(r_sport[j] != 0, r_sport[j], ports[rng.integers(0, len(ports), size=n)])
    dport = np.where(r_dport[j] != 0, r_dport[j], ports[rng.integers(0, len(ports), size=n)])
    sport = sport.astype(np.uint32)
    dport = dport.astype(np.uint32)
    # destinations: a pool host inside the rule's prefix, or any pool host
    inside = flat[off[j] + (rng.random(n) * np.maximum(cnt[j], 1)).astype(np.int64)]
    pick = np.where(cnt[j] > 0, inside, rng.integers(0, n_hosts, size=n))
    # sources: random bits below the rule's prefix
    s4 = (src4[j] & m4s[j]) | (rng.integers(0, 1 << 32, size=n, dtype=np.uint64) & ~m4s[j]
                               & np.uint64(0xFFFFFFFF))
    s6 = (src6[j] & m6s[j]) | (rng.integers(0, 256, size=(n, 16), dtype=np.uint8) & ~m6s[j])

    imix = rng.choice(np.array([64, 570, 1518]), size=n, p=[7 / 12, 4 / 12, 1 / 12])
    hdr_len = np.where(is6, 54, 34) + np.where(proto == 6, 20, 8)
    size = np.maximum(imix, hdr_len)
    h = np.zeros((n, 128), dtype=np.uint8)
    _macs(h, rng)
    ttl = rng.integers(1, 129, size=n)
    build_ipv4(h, r4, src=s4[r4], dst=dst4[pick[r4]], proto=proto[r4], ttl=ttl[r4],
               ihl=np.full(len(r4), 5), total_len=size[r4] - 14,
               l4_ports=(sport[r4], dport[r4]), tcp_doff=np.full(len(r4), 5),
               icmp=(dport[r4] >> 8, dport[r4] & 0xFF, sport[r4]), rng=rng)
    build_ipv6(h, r6, src16=s6[r6], dst16=dst6[pick[r6]], nh=proto[r6], hop=ttl[r6],
               payload_len=size[r6] - 54, sport=sport[r6], dport=dport[r6],
               tcp_doff=np.full(len(r6), 5))
    frames, desc = pack_frames(h, size)
    return Workload("C", frames, desc, rules, n_rules, arp, ndp)


# ---------------------------------------------------------------------------------------------
# config D — 64k rules, variable-length headers, malformed traffic, v4/v6 interleaved
# ---------------------------------------------------------------------------------------------

def config_d(n: int = 1 << 24, seed: int = 4, n_rules: int = 1 << 16) -> Workload:
    rng = np.random.default_rng(seed)
    n_flows = n_rules - 1
    # one exact flow per rule so first-match positions spread uniformly over the table
    f6 = rng.random(n_flows) < 0.3
    f_src4 = (0x0B000000 + rng.integers(0, 1 << 24, size=n_flows)).astype(np.uint64)
    f_dst4 = (0xAC100000 + rng.integers(0, 1 << 12, size=n_flows)).astype(np.uint64)
    f_src6 = _v6_pool(rng, n_flows)
    f_dst6 = _v6_pool(rng, n_flows, prefix=bytes.fromhex("2001db80"))
    f_proto = np.where(f6, rng.choice(np.array([17, 6]), size=n_flows),
                       rng.choice(np.array([17, 6, 1]), size=n_flows))
    f_sport = rng.integers(1, 65536, size=n_flows).astype(np.uint32)
    f_dport = rng.integers(1, 65536, size=n_flows).astype(np.uint32)
    f_dport = np.where(f_proto == 1, (8 << 8) | 0, f_dport)  # echo request type/code
    prios = rng.permutation(n_flows) + 1
    acts = np.where(rng.random(n_flows) < 0.5, ACT_FWD, ACT_DROP)

    rules = np.zeros(n_rules, dtype=RULE_DTYPE)
    rules["priority"][:n_flows] = prios
    rules["ip_ver"][:n_flows] = np.where(f6, 6, 4)
    rules["protocol"][:n_flows] = f_proto
    rules["src_port"][:n_flows] = f_sport
    rules["dst_port"][:n_flows] = f_dport
    rules["action"][:n_flows] = acts
    rules["out_ifindex"][:n_flows] = np.where(acts == ACT_FWD, 1, 0)
    v4r = np.nonzero(~f6)[0]
    v6r = np.nonzero(f6)[0]
    rules["src_ip"][v4r, :4] = f_src4[v4r].astype("<u4").view(np.uint8).reshape(-1, 4)
    rules["dst_ip"][v4r, :4] = f_dst4[v4r].astype("<u4").view(np.uint8).reshape(-1, 4)
    rules["src_mask"][v4r, :4] = 0xFF
    rules["dst_mask"][v4r, :4] = 0xFF
    rules["src_ip"][v6r] = f_src6[v6r]
    rules["dst_ip"][v6r] = f_dst6[v6r]
    rules["src_mask"][v6r] = 0xFF
    rules["dst_mask"][v6r] = 0xFF
    # ~1 % wildcard rules (port-only / prefix) sprinkled in, they shadow some flows
    wild = rng.permutation(n_flows)[: n_flows // 100]
    rules["src_port"][wild] = 0
    rules["src_mask"][wild, 2:] = 0
    rules["src_ip"][wild, 2:] = 0
    rules["priority"][n_rules - 1] = 1 << 30
    rules["action"][n_rules - 1] = ACT_DROP

    arp = arp_table(1024, [(int(ip), _rand_macs(rng, 1)[0].tobytes())
                           for ip in np.unique(f_dst4[v4r])[:600]])
    ndp = ndp_table(1024, [(bytes(f_dst6[i]), _rand_macs(rng, 1)[0].tobytes())
                           for i in v6r[:600]])

    flow = rng.integers(0, n_flows, size=n)
    # 5 % of packets hit no specific rule (random 5-tuple -> catch-all, the longest scans)
    stray = rng.random(n) < 0.05
    is6 = f6[flow]
    h = np.zeros((n, 128), dtype=np.uint8)
    _macs(h, rng)
    proto = f_proto[flow].copy()
    sport = np.where(stray, rng.integers(1, 65536, size=n), f_sport[flow]).astype(np.uint32)
    dport = f_dport[flow].astype(np.uint32)
    r4 = np.nonzero(~is6)[0]
    r6 = np.nonzero(is6)[0]
    ihl = np.where(rng.random(len(r4)) < 0.5, 5, rng.integers(6, 16, size=len(r4)))
    doff4 = np.where(rng.random(len(r4)) < 0.5, 5, rng.integers(6, 16, size=len(r4)))
    l4len4 = np.where(proto[r4] == 6, doff4 * 4, 8)
    len4 = 14 + ihl * 4 + l4len4 + rng.integers(0, 8, size=len(r4))
    build_ipv4(h, r4, src=f_src4[flow[r4]], dst=f_dst4[flow[r4]], proto=proto[r4],
               ttl=rng.integers(1, 65, size=len(r4)), ihl=ihl, total_len=len4 - 14,
               l4_ports=(sport[r4], dport[r4]), tcp_doff=doff4,
               icmp=(np.full(len(r4), 8), np.zeros(len(r4), dtype=np.int64), sport[r4]),
               rng=rng)
    doff6 = np.where(rng.random(len(r6)) < 0.5, 5, rng.integers(6, 15, size=len(r6)))
    l4len6 = np.where(proto[r6] == 6, doff6 * 4, 8)
    len6 = 54 + l4len6 + rng.integers(0, 8, size=len(r6))
    build_ipv6(h, r6, src16=f_src6[flow[r6]], dst16=f_dst6[flow[r6]], nh=proto[r6],
               hop=rng.integers(1, 65, size=len(r6)), payload_len=len6 - 54,
               sport=sport[r6], dport=dport[r6], tcp_doff=doff6)
    lens = np.zeros(n, dtype=np.int64)
    lens[r4] = len4
    lens[r6] = len6
    lens = np.minimum(lens, 128)
    # 10 % malformed, one of several failure modes each
    bad = np.nonzero(rng.random(n) < 0.10)[0]
    mode = rng.integers(0, 8, size=len(bad))
    for m in range(8):
        rows = bad[mode == m]
        if m == 0:    # truncated somewhere inside the headers
            lens[rows] = rng.integers(0, np.maximum(lens[rows] - 1, 1))
        elif m == 1:  # wrong IPv4 version nibble
            h[rows, 14] = np.where(h[rows, 12] == 0x08, (h[rows, 14] & 0x0F) | 0x50, h[rows, 14])
        elif m == 2:  # VLAN tag ethertype
            h[rows, 12] = 0x81
            h[rows, 13] = 0x00
        elif m == 3:  # GRE / ESP
            h[rows, 23] = np.where(h[rows, 12] == 0x08, rng.choice([47, 50], size=len(rows)),
                                   h[rows, 23])
            h[rows, 20] = np.where(h[rows, 12] == 0x86, rng.choice([47, 50], size=len(rows)),
                                   h[rows, 20])
        elif m == 4:  # ICMPv6 (not NS/NA) on IPv6 rows, IHL < 5 on IPv4 rows
            h[rows, 20] = np.where(h[rows, 12] == 0x86, 58, h[rows, 20])
            h[rows, 54] = np.where(h[rows, 12] == 0x86, 128, h[rows, 54])
            h[rows, 14] = np.where(h[rows, 12] == 0x08, 0x44, h[rows, 14])
        elif m == 5:  # TCP data offset < 5
            sel4 = (h[rows, 12] == 0x08) & (h[rows, 23] == 6)
            l4 = 14 + (h[rows, 14] & 0x0F).astype(np.int64) * 4
            h[rows[sel4], l4[sel4] + 12] = 0x30
            sel6 = (h[rows, 12] == 0x86) & (h[rows, 20] == 6)
            h[rows[sel6], 66] = 0x20
        elif m == 6:  # TTL / hop limit 0
            h[rows, 22] = np.where(h[rows, 12] == 0x08, 0, h[rows, 22])
            h[rows, 21] = np.where(h[rows, 12] == 0x86, 0, h[rows, 21])
        else:         # IHL larger than the frame
            h[rows, 14] = np.where(h[rows, 12] == 0x08, 0x4F, h[rows, 14])
            lens[rows] = np.where(h[rows, 12] == 0x08, np.minimum(lens[rows], 60), lens[rows])
    frames, desc = pack_frames(h, lens, stride=128)
    return Workload("D", frames, desc, rules, n_rules, arp, ndp)


def header_windows(wl: Workload, window: int = HDR_WINDOW) -> Workload:
    """The same packets as header windows: frame i becomes its first min(len, window) bytes at
    offset i * window (descriptor lengths stay the real lengths, so rule_stats bytes are
    unchanged).  What a host-side batch builder ships instead of whole frames: the path reads at
    most UPE_HDR_WINDOW bytes of a frame and rewrites at most UPE_REWRITE_EXTENT."""
    offs = desc_offsets(wl.desc)
    lens = desc_lens(wl.desc)
    n = wl.n
    out = np.zeros(n * window + FRAME_TAIL + 128, dtype=np.uint8)
    cols = np.arange(window)
    chunk = 1 << 16
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        keep = np.minimum(lens[s:e], window)
        m = cols[None, :] < keep[:, None]
        src = offs[s:e, None] + cols[None, :]
        dst = (np.arange(s, e, dtype=np.int64) * window)[:, None] + cols[None, :]
        out[dst[m]] = wl.frames[src[m]]
    desc = make_desc(np.arange(n, dtype=np.int64) * window, lens)
    return dataclasses.replace(wl, frames=out, desc=desc, arp=wl.arp.copy(), ndp=wl.ndp.copy(),
                               l1=wl.l1.copy())


CONFIGS = {"A": config_a, "B": config_b, "C": config_c, "D": config_d}


def make(name: str, n: int | None = None, seed: int | None = None, **kw) -> Workload:
    fn = CONFIGS[name]
    args = {}
    if n is not None:
        args["n"] = n
    if seed is not None:
        args["seed"] = seed
    args.update(kw)
    return fn(**args)


# ---------------------------------------------------------------------------------------------
# edge cases — every parse gate, control packet kind and quirk of SURVEY.md §8.1
# ---------------------------------------------------------------------------------------------

def _frame(*parts) -> bytes:
    return b"".join(parts)


def _eth(et: int, dst=b"\x00\x11\x22\x33\x44\x55", src=b"\x66\x77\x88\x99\xaa\xbb") -> bytes:
    return dst + src + et.to_bytes(2, "big")


def _ip4(proto, src, dst, ttl=64, ihl=5, ver=4, total=0, opts=None) -> bytes:
    opt = bytes(opts) if opts is not None else b"\x01" * (ihl * 4 - 20)
    hdr = bytes([(ver << 4) | ihl, 0]) + total.to_bytes(2, "big") + b"\x12\x34\x40\x00" + \
        bytes([ttl, proto]) + b"\x00\x00" + src.to_bytes(4, "big") + dst.to_bytes(4, "big") + opt
    return hdr


def _ip6(nh, src16, dst16, hop=64, plen=0) -> bytes:
    return (0x60000000).to_bytes(4, "big") + plen.to_bytes(2, "big") + bytes([nh, hop]) + \
        bytes(src16) + bytes(dst16)


def _udp(sp, dp) -> bytes:
    return sp.to_bytes(2, "big") + dp.to_bytes(2, "big") + b"\x00\x08\x00\x00"


def _tcp(sp, dp, doff=5) -> bytes:
    return sp.to_bytes(2, "big") + dp.to_bytes(2, "big") + b"\x00" * 8 + bytes([doff << 4, 0x10]) + \
        b"\xff\xff\x00\x00\x00\x00" + b"\x00" * max(0, doff * 4 - 20)


def _icmp(t, c, ident) -> bytes:
    return bytes([t, c, 0, 0]) + ident.to_bytes(2, "big") + b"\x00\x01"


def _arp(op, sha, spa, tha, tpa, htype=1, ptype=0x0800, hlen=6, plen=4) -> bytes:
    return htype.to_bytes(2, "big") + ptype.to_bytes(2, "big") + bytes([hlen, plen]) + \
        op.to_bytes(2, "big") + bytes(sha) + spa.to_bytes(4, "big") + bytes(tha) + \
        tpa.to_bytes(4, "big")


def edge_frames():
    """(frame bytes, length) pairs; length may cut the frame short (truncation gates)."""
    V6A = bytes.fromhex("20010db8000000000000000000000001")
    V6B = bytes.fromhex("20010db8000000000000000000000002")
    V6N = bytes.fromhex("2001db80000000000000000000000abc")  # in NDP table
    ZERO6 = bytes(16)
    MAC = bytes.fromhex("0a0b0c0d0e0f")
    out = []

    def add(fr, ln=None):
        out.append((fr, len(fr) if ln is None else ln))

    v4u = _frame(_eth(0x0800), _ip4(17, 0x0A000001, 0x0A800005), _udp(1000, 53))
    for ln in range(0, len(v4u) + 1):                       # every truncation of a UDP frame
        add(v4u, ln)
    v4t = _frame(_eth(0x0800), _ip4(6, 0x0A000001, 0x0A800006), _tcp(2000, 22))
    for ln in (53, 54, 60):
        add(v4t, ln)
    for doff in (0, 4, 5, 6, 15):                            # TCP data offset gates
        add(_frame(_eth(0x0800), _ip4(6, 0x0A000002, 0x0A800007), _tcp(2000, 80, doff=max(doff, 5))[:12] +
                   bytes([doff << 4]) + b"\x10" + b"\x00" * 6 + b"\x00" * 40), 14 + 20 + 20 + 16)
    for ihl in (0, 4, 5, 6, 10, 15):                         # IHL gates and options
        ih = max(ihl, 5)
        f = _frame(_eth(0x0800), _ip4(17, 0x0A000003, 0x0A800008, ihl=ih), _udp(7, 8))
        f = f[:14] + bytes([0x40 | ihl]) + f[15:]
        add(f)
        add(f, 14 + ih * 4 + 4)
    add(_frame(_eth(0x0800), _ip4(17, 0x0A000003, 0x0A800008, ver=6), _udp(7, 8)))  # ver != 4
    for t, c in ((8, 0), (0, 0), (3, 1), (11, 0)):            # ICMP: id->sport, type<<8|code
        add(_frame(_eth(0x0800), _ip4(1, 0x0A000004, 0x0A800009), _icmp(t, c, 0x1234)))
    add(_frame(_eth(0x0800), _ip4(1, 0x0A000004, 0x0A800009), _icmp(8, 0, 1)), 38)
    for proto in (47, 50, 58, 0, 255):                        # unknown L4 protocols
        add(_frame(_eth(0x0800), _ip4(proto, 0x0A000005, 0x0A80000A), _udp(1, 2)))
    for ttl in (0, 1, 2, 255):                                # TTL edge cases on FWD
        add(_frame(_eth(0x0800), _ip4(17, 0x0A000006, 0x0A800005, ttl=ttl), _udp(5, 53)))
    add(_frame(_eth(0x0800), _ip4(17, 0x0A000006, 0x0A8000C8), _udp(5, 53)))  # ARP miss -> FWD
    add(_frame(_eth(0x0800), _ip4(17, 0x0A000006, 0x00000000), _udp(5, 53)))  # dst 0.0.0.0
    add(_frame(_eth(0x0800), _ip4(6, 0xC0A80101, 0x0A800005, ihl=7), _tcp(5, 443, doff=8)))
    # IPv6
    v6u = _frame(_eth(0x86DD), _ip6(17, V6A, V6N), _udp(3000, 53))
    for ln in (53, 54, 61, 62, 70):
        add(v6u, ln)
    add(_frame(_eth(0x86DD), _ip6(6, V6A, V6B), _tcp(4000, 443)))
    add(_frame(_eth(0x86DD), _ip6(6, V6A, V6B), _tcp(4000, 443)), 73)
    add(_frame(_eth(0x86DD), _ip6(6, V6A, V6B), _tcp(4000, 443, doff=6)), 78)
    for hop in (0, 1, 2):
        add(_frame(_eth(0x86DD), _ip6(17, V6A, V6N, hop=hop), _udp(9, 53)))
    add(_frame(_eth(0x86DD), _ip6(17, V6A, ZERO6), _udp(9, 53)))        # dst :: (quirk 15)
    add(_frame(_eth(0x86DD), _ip6(17, V6B, ZERO6), _udp(9, 53)))
    add(_frame(_eth(0x86DD), _ip6(1, V6A, V6B), _icmp(128, 0, 7)))      # ICMP (proto 1) in v6
    v6n = _frame(_eth(0x86DD), _ip6(17, V6A, V6N), _udp(3000, 53))
    add(v6n[:14] + bytes([0x40]) + v6n[15:])                            # v6 version not checked
    add(_frame(_eth(0x86DD), _ip6(58, V6A, V6B), bytes([128, 0, 0, 0]) + b"\x00" * 20))  # echo
    # NDP: NS with SLLA, NA with TLLA, short ones (dropped as parse failures), no option
    ns = _frame(_eth(0x86DD), _ip6(58, V6A, V6B), bytes([135, 0, 0, 0, 0, 0, 0, 0]) + V6B,
                bytes([1, 1]) + MAC)
    na = _frame(_eth(0x86DD), _ip6(58, V6B, V6A), bytes([136, 0, 0, 0, 0x60, 0, 0, 0]) + V6N,
                bytes([2, 1]) + bytes.fromhex("a1a2a3a4a5a6"))
    add(ns)
    add(na)
    add(ns, 77)
    add(ns, 78)
    add(_frame(_eth(0x86DD), _ip6(58, V6A, V6B), bytes([136, 0, 0, 0, 0, 0, 0, 0]) + V6N,
               bytes([5, 0]) + b"\x00" * 6))                            # zero-length option
    # ARP: request for our IP (reply in place), request for another IP, reply, malformed
    add(_frame(_eth(0x0806, dst=b"\xff" * 6), _arp(1, MAC, 0x0A800063, bytes(6), PORT_IP4)))
    add(_frame(_eth(0x0806, dst=b"\xff" * 6), _arp(1, MAC, 0x0A800064, bytes(6), 0x0A800001)))
    add(_frame(_eth(0x0806), _arp(2, bytes.fromhex("0c0c0c0c0c0c"), 0x0A800005, MAC, PORT_IP4)))
    add(_frame(_eth(0x0806), _arp(1, MAC, 0x0A800065, bytes(6), PORT_IP4, hlen=8)))
    add(_frame(_eth(0x0806), _arp(1, MAC, 0x0A800066, bytes(6), PORT_IP4)), 30)  # short ARP
    add(_frame(_eth(0x0806), _arp(1, MAC, 0x0A800067, bytes(6), PORT_IP4 & 0xFFFF0000)), 40)
    add(_frame(_eth(0x0806)), 14)
    # other ethertypes
    add(_frame(_eth(0x8100), b"\x00\x01\x08\x00", _ip4(17, 1, 2), _udp(1, 2)))
    add(_frame(_eth(0x88CC), b"\x00" * 40))
    add(b"\x00" * 12 + b"\x08", 13)
    add(b"", 0)
    return out


def edge_rules() -> np.ndarray:
    V6P = bytes.fromhex("20010db8") + bytes(12)
    return rules_array([
        make_rule(9999, ACT_DROP),
        make_rule(10, ACT_FWD, dport=53),
        make_rule(20, ACT_DROP, proto=6, dport=22),
        make_rule(30, ACT_FWD, ip_ver=4, proto=6, src=(0xC0A80000, 16)),
        make_rule(40, ACT_DROP, proto=1, sport=0x1234, dport=0x0800),
        make_rule(50, 2, proto=1),                                   # unknown action type
        make_rule(60, ACT_FWD, ip_ver=6, src=(V6P, 32)),
        # version-0 rule with a v6 address: its bytes 0-3 also apply to v4 packets
        make_rule(70, ACT_DROP, ip_ver=0, dst=(bytes.fromhex("0a800008") + bytes(12), 40)),
        make_rule(15, ACT_FWD, ip_ver=4, dst=(bytes.fromhex("2001db80") + bytes(12), 128)),
        make_rule(80, ACT_FWD, proto=6),
    ])


def config_edge(repeat: int = 4, seed: int = 5) -> Workload:
    """The edge frames, repeated in a shuffled order, with tables that make both neighbour
    cache paths (hit, miss, starting-entry disagreement) reachable."""
    rng = np.random.default_rng(seed)
    fr = edge_frames()
    order = np.concatenate([np.arange(len(fr))] + [rng.permutation(len(fr)) for _ in range(repeat - 1)])
    frames_b = [fr[i] for i in order]
    lens = np.array([ln for _, ln in frames_b], dtype=np.int64)
    h = np.zeros((len(frames_b), 128), dtype=np.uint8)
    for i, (f, _) in enumerate(frames_b):
        b = np.frombuffer(f[:128], np.uint8)
        h[i, : len(b)] = b
    # store the whole frame bytes (not just `len`): bytes past len must be ignored
    frames, desc = pack_frames(h, np.maximum(lens, 0))
    arp = arp_table(16, [(0x0A800005, bytes.fromhex("aabbccdd0005")),
                         (0x0A800015, bytes.fromhex("aabbccdd0015")),   # same slot as .5
                         (0x0A800006, bytes.fromhex("aabbccdd0006")),
                         (0x00000000, bytes.fromhex("aabbccdd0000"))])
    ndp = ndp_table(16, [(bytes.fromhex("2001db80000000000000000000000abc"),
                          bytes.fromhex("bbccddee0abc")),
                         (bytes.fromhex("20010db8000000000000000000000002"),
                          bytes.fromhex("bbccddee0002"))])
    return Workload("edge", frames, desc, edge_rules(), 64, arp, ndp)


def config_ndp_walk(repeat: int = 3) -> Workload:
    """Long NS / NA frames (up to 400 bytes) whose option walk crosses the uint8_t width of
    reference src/worker.c:73 (`uint8_t opt_len = data[off + 1] * 8`): a length byte of 32 or 64
    wraps to 0 (the walk stops, nothing is learned), 33 wraps to 8 (the walk advances 8 bytes,
    not 264).  Each control frame is followed by IPv6 packets to the address it teaches, so a
    wrong walk shows up in the forwarded bytes and in the final NDP table.  Used by the
    control-packet and drop-in tests."""
    V6S = bytes.fromhex("20010db8000000000000000000000001")
    tgt = [bytes.fromhex("20010db80000000000000000000001%02x" % k) for k in range(8)]
    MA, MB = bytes.fromhex("0a0000000a0a"), bytes.fromhex("0b0000000b0b")

    def opts(first_len: int, typ: int, total: int) -> bytes:
        # option 0: unknown type 5 with length byte first_len; an SLLA / TLLA (MAC A) 8 bytes
        # later and another (MAC B) where the un-wrapped length would land
        o = bytearray(total - 78)
        o[0], o[1] = 5, first_len
        o[8:16] = bytes([typ, 1]) + MA
        far = (first_len * 8) & 0xFFFF
        if 0 < far and far + 8 <= len(o):
            o[far:far + 8] = bytes([typ, 1]) + MB
        return bytes(o)

    frames = []
    for k, (first, total) in enumerate([(32, 350), (33, 360), (64, 400), (31, 300),
                                        (33, 290), (1, 120), (32, 250), (0, 200)]):
        ns = k % 2 == 0
        ip = tgt[k]
        if ns:   # NS: learns (ip6.src, SLLA)
            f = _frame(_eth(0x86DD), _ip6(58, ip, V6S), bytes([135, 0, 0, 0, 0, 0, 0, 0]) + ip,
                       opts(first, 1, total))
        else:    # NA: learns (target, TLLA)
            f = _frame(_eth(0x86DD), _ip6(58, V6S, ip), bytes([136, 0, 0, 0, 0x60, 0, 0, 0]) + ip,
                       opts(first, 2, total))
        probe = _frame(_eth(0x86DD), _ip6(17, V6S, ip), _udp(4000 + k, 53))
        frames += [(probe, len(probe)), (f, len(f)), (probe, len(probe)), (probe, len(probe))]
    frames = frames * repeat
    lens = np.array([ln for _, ln in frames], dtype=np.int64)
    h = np.zeros((len(frames), 512), dtype=np.uint8)
    for i, (f, _) in enumerate(frames):
        h[i, :len(f)] = np.frombuffer(f, np.uint8)
    fr, desc = pack_frames(h, lens)
    ndp = ndp_table(16, [(tgt[7], bytes.fromhex("0c0000000c0c"))])
    return Workload("ndp_walk", fr, desc, edge_rules(), 64, arp_table(16, []), ndp)
