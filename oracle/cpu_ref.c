/*
 * oracle/cpu_ref.c — CPU restatement of UPE's per-packet worker hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this library, and only as the checker (or the timed CPU baseline) — never as part of
 * the product path, which lives in upe_amd/csrc and has no CPU fallback.
 *
 * Parity pinning: this restatement is checked against
 *   (1) golden vectors produced by the reference worker itself (oracle/ref_harness.c, which
 *       #includes /root/reference/src/worker.c) — tests/golden/ fixtures, and
 *   (2) the known-answer tests of reference tests/test_suite.c:132-242, 245-299, 332-362,
 *       365-437, 523-590 (restated in tests/test_oracle.py).
 *
 * It processes packets strictly one after another, with the worker's one-entry L1 neighbour
 * caches updated sequentially (reference src/worker.c:186-195, 218-225) — deliberately NOT the
 * GPU's first-index/last-index emulation, so it checks that emulation independently.
 *
 * Frames are read as if they sat in a zero-filled pktbuf: bytes at or
 * beyond a frame's length read as 0, and writes at or beyond it are discarded (tx_send transmits
 * only b->len bytes, reference src/tx_afpacket.c:60-76).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/upe_gpu.h"

#define PKTBUF_DATA 2048 /* reference include/pktbuf.h:8 */

/* ---- byte helpers (wire order is big-endian) ---------------------------------------------- */
static inline uint16_t rd_be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
static inline uint32_t rd_be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static inline uint32_t rd_le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* ---- parse_flow_key, reference src/parser.c:6-111 ------------------------------------------ */
int upe_ref_parse(const uint8_t *pkt, size_t len, upe_flow_key_t *out) {
    if (len < 14) return -1;                         /* parser.c:8-10 */
    uint16_t et = rd_be16(pkt + 12);
    size_t l4_off, l4_len;
    if (et == 0x0800) {                              /* parser.c:18-44 */
        size_t ip_len = len - 14;
        if (ip_len < 20) return -1;
        uint8_t vihl = pkt[14];
        size_t hl = (size_t)(vihl & 0x0F) * 4;
        if ((vihl >> 4) != 4 || hl < 20 || ip_len < hl) return -1;
        out->ip_ver = 4;
        out->src_ip.v4 = rd_be32(pkt + 26);
        out->dst_ip.v4 = rd_be32(pkt + 30);
        out->protocol = pkt[23];
        l4_off = 14 + hl;
        l4_len = ip_len - hl;
    } else if (et == 0x86DD) {                       /* parser.c:46-64 */
        size_t ip_len = len - 14;
        if (ip_len < 40) return -1;
        out->ip_ver = 6;
        memcpy(out->src_ip.v6, pkt + 22, 16);
        memcpy(out->dst_ip.v6, pkt + 38, 16);
        out->protocol = pkt[20];
        l4_off = 54;
        l4_len = ip_len - 40;
    } else {
        return -1;                                   /* parser.c:66-68 */
    }
    const uint8_t *l4 = pkt + l4_off;
    if (out->protocol == 17) {                       /* UDP, parser.c:70-78 */
        if (l4_len < 8) return -1;
        out->src_port = rd_be16(l4);
        out->dst_port = rd_be16(l4 + 2);
    } else if (out->protocol == 6) {                 /* TCP, parser.c:79-94 */
        if (l4_len < 20) return -1;
        size_t thl = (size_t)(l4[12] >> 4) * 4;
        if (thl < 20 || l4_len < thl) return -1;
        out->src_port = rd_be16(l4);
        out->dst_port = rd_be16(l4 + 2);
    } else if (out->protocol == 1) {                 /* ICMP, parser.c:95-105 */
        if (l4_len < 8) return -1;
        out->src_port = rd_be16(l4 + 4);
        out->dst_port = (uint16_t)((l4[0] << 8) | l4[1]);
    } else {
        return -1;                                   /* parser.c:106-108 */
    }
    return 0;
}

/* ---- flow_hash, reference src/parser.c:113-135 --------------------------------------------- */
uint32_t upe_ref_flow_hash(const upe_flow_key_t *k) {
    if (!k) return 0;
    uint32_t h = (uint32_t)k->src_port ^ k->dst_port ^ k->protocol;
    if (k->ip_ver == 4) {
        h ^= k->src_ip.v4 ^ k->dst_ip.v4;
    } else if (k->ip_ver == 6) {
        for (int i = 0; i < 4; i++) h ^= rd_le32(k->src_ip.v6 + 4 * i) ^ rd_le32(k->dst_ip.v6 + 4 * i);
    }
    return h;
}

/* ---- ipv4_checksum, reference src/parser.c:137-169: native-LE u16 sum, fold, invert ------- */
uint16_t upe_ref_ipv4_checksum(const uint8_t *p, size_t len) {
    uint32_t sum = 0;
    size_t i = 0;
    for (; i + 1 < len; i += 2) sum += (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8);
    if (i < len) sum += p[i];
    while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
    return (uint16_t)~sum;
}

/* ---- mask helpers, reference src/rule_table.c:14-50 ---------------------------------------- */
bool upe_ref_ipv4_mask(uint8_t prefix, uint32_t *out) {
    if (!out || prefix > 32) return false;
    *out = prefix == 0 ? 0u : (uint32_t)(0xFFFFFFFFu << (32 - prefix));
    return true;
}
bool upe_ref_ipv6_mask(uint8_t prefix, uint8_t out[16]) {
    if (!out || prefix > 128) return false;
    for (int i = 0; i < 16; i++) {
        int bits = (int)prefix - 8 * i;
        out[i] = bits >= 8 ? 0xFF : bits <= 0 ? 0 : (uint8_t)(0xFF << (8 - bits));
    }
    return true;
}

/* ---- rule table build: rule_table_add semantics, reference src/rule_table.c:130-161 --------- */
/* Appends rules in insertion order (rule_id = insertion index, canonicalise wildcard addresses),
 * then sorts once by (priority, rule_id) — the same final order as a qsort after every add since
 * the comparator (src/rule_table.c:96-109) is a total order over unique rule_ids. */
static int rule_cmp(const void *a, const void *b) {
    const upe_rule_t *x = a, *y = b;
    if (x->priority != y->priority) return x->priority < y->priority ? -1 : 1;
    if (x->rule_id != y->rule_id) return x->rule_id < y->rule_id ? -1 : 1;
    return 0;
}
int upe_ref_rules_build(const upe_rule_t *in, size_t n, upe_rule_t *out) {
    static const uint8_t zero16[16];
    for (size_t i = 0; i < n; i++) {
        upe_rule_t r = in[i];
        r.rule_id = (uint32_t)i;
        if (r.ip_ver == 4 && r.src_mask.v4 == 0) r.src_ip.v4 = 0;
        if (r.ip_ver == 4 && r.dst_mask.v4 == 0) r.dst_ip.v4 = 0;
        if (r.ip_ver == 6) {
            if (memcmp(r.src_mask.v6, zero16, 16) == 0) memset(r.src_ip.v6, 0, 16);
            if (memcmp(r.dst_mask.v6, zero16, 16) == 0) memset(r.dst_ip.v6, 0, 16);
        }
        out[i] = r;
    }
    qsort(out, n, sizeof(upe_rule_t), rule_cmp);
    return 0;
}

/* ---- match_rule + rule_table_match, reference src/rule_table.c:53-91,163-176 ---------------- */
static bool match_rule(const upe_rule_t *r, const upe_flow_key_t *k) {
    if (r->ip_ver != 0 && r->ip_ver != k->ip_ver) return false;
    if (r->protocol && r->protocol != k->protocol) return false;
    if (r->src_port && r->src_port != k->src_port) return false;
    if (r->dst_port && r->dst_port != k->dst_port) return false;
    if (k->ip_ver == 4) {
        if ((k->src_ip.v4 & r->src_mask.v4) != (r->src_ip.v4 & r->src_mask.v4)) return false;
        if ((k->dst_ip.v4 & r->dst_mask.v4) != (r->dst_ip.v4 & r->dst_mask.v4)) return false;
    } else if (k->ip_ver == 6) {
        for (int i = 0; i < 16; i++) {
            if ((k->src_ip.v6[i] & r->src_mask.v6[i]) != (r->src_ip.v6[i] & r->src_mask.v6[i]))
                return false;
            if ((k->dst_ip.v6[i] & r->dst_mask.v6[i]) != (r->dst_ip.v6[i] & r->dst_mask.v6[i]))
                return false;
        }
    }
    return true;
}
long upe_ref_match(const upe_rule_t *rules, size_t n, const upe_flow_key_t *k) {
    for (size_t i = 0; i < n; i++)
        if (match_rule(&rules[i], k)) return (long)i;
    return -1;
}

/* ---- neighbour lookups: arp_get_mac (src/arp_table.c:55-80), ndp_get_mac + hash_ipv6
 *      (src/ndp_table.c:6-17,67-86) --------------------------------------------------------- */
bool upe_ref_arp_lookup(const upe_arp_entry_t *t, size_t cap, uint32_t ip, uint8_t mac[6]) {
    if (!t || cap == 0) return false;
    size_t idx = ip & (cap - 1);
    for (size_t i = 0; i < cap; i++) {
        const upe_arp_entry_t *e = &t[(idx + i) & (cap - 1)];
        if (e->valid && e->ip == ip) {
            memcpy(mac, e->mac, 6);
            return true;
        }
        if (!e->valid) break;
    }
    return false;
}
static size_t ndp_hash(const uint8_t ip[16], size_t cap) {
    uint32_t h = rd_le32(ip) ^ rd_le32(ip + 4) ^ rd_le32(ip + 8) ^ rd_le32(ip + 12);
    return h & (cap - 1);
}
bool upe_ref_ndp_lookup(const upe_ndp_entry_t *t, size_t cap, const uint8_t ip[16], uint8_t mac[6]) {
    if (!t || cap == 0) return false;
    size_t idx = ndp_hash(ip, cap);
    for (size_t i = 0; i < cap; i++) {
        const upe_ndp_entry_t *e = &t[(idx + i) & (cap - 1)];
        if (e->valid && memcmp(e->ip, ip, 16) == 0) {
            memcpy(mac, e->mac, 6);
            return true;
        }
        if (!e->valid) break;
    }
    return false;
}

/* ---- neighbour updates (control plane; used to replay control packets between segments):
 *      arp_update src/arp_table.c:26-53, ndp_update src/ndp_table.c:39-65 ------------------- */
void upe_ref_arp_update(upe_arp_entry_t *t, size_t cap, uint32_t ip, const uint8_t mac[6]) {
    if (!t || cap == 0) return;
    size_t idx = ip & (cap - 1);
    for (size_t i = 0; i < cap; i++) {
        upe_arp_entry_t *e = &t[(idx + i) & (cap - 1)];
        if (!e->valid || e->ip == ip) {
            e->valid = true;
            e->ip = ip;
            memcpy(e->mac, mac, 6);
            return;
        }
    }
}
void upe_ref_ndp_update(upe_ndp_entry_t *t, size_t cap, const uint8_t ip[16], const uint8_t mac[6]) {
    if (!t || cap == 0) return;
    size_t idx = ndp_hash(ip, cap);
    for (size_t i = 0; i < cap; i++) {
        upe_ndp_entry_t *e = &t[(idx + i) & (cap - 1)];
        if (!e->valid || memcmp(e->ip, ip, 16) == 0) {
            e->valid = true;
            memcpy(e->ip, ip, 16);
            memcpy(e->mac, mac, 6);
            return;
        }
    }
}

/* ---- the worker context the oracle carries between calls ----------------------------------- */
typedef struct {
    const upe_rule_t *rules;
    size_t nrules;
    upe_arp_entry_t *arp;
    size_t arp_cap;
    upe_ndp_entry_t *ndp;
    size_t ndp_cap;
    uint8_t eth_addr[6];
    uint32_t ip4_addr;
    int apply_control; /* replay arp_update / ndp_update as the reference does (sequential) */
} upe_ref_env_t;

/* handle_control_packet, reference src/worker.c:23-104.  Returns 1 if the packet was consumed
 * (NDP NS/NA), 0 otherwise; sets *flags (ARP_LEARN / ARP_REPLY). */
static int control_packet(const upe_ref_env_t *env, uint8_t *d, size_t len, uint32_t *flags) {
    uint16_t et = rd_be16(d + 12);
    if (et == 0x0806) {
        uint8_t *a = d + 14;
        if (rd_be16(a) == 1 && rd_be16(a + 2) == 0x0800 && a[4] == 6 && a[5] == 4) {
            *flags |= UPE_VF_ARP_LEARN;
            if (env->apply_control) upe_ref_arp_update(env->arp, env->arp_cap, rd_be32(a + 14), a + 8);
            if (rd_be16(a + 6) == 1 && env->ip4_addr != 0 && rd_be32(a + 24) == env->ip4_addr) {
                memcpy(d, d + 6, 6);               /* eth.dst = eth.src */
                memcpy(d + 6, env->eth_addr, 6);   /* eth.src = port MAC */
                a[6] = 0; a[7] = 2;                /* op = REPLY */
                memcpy(a + 18, a + 8, 6);          /* tha = sha */
                memcpy(a + 24, a + 14, 4);         /* tpa = spa */
                memcpy(a + 8, env->eth_addr, 6);   /* sha = port MAC */
                a[14] = (uint8_t)(env->ip4_addr >> 24); a[15] = (uint8_t)(env->ip4_addr >> 16);
                a[16] = (uint8_t)(env->ip4_addr >> 8);  a[17] = (uint8_t)env->ip4_addr;
                *flags |= UPE_VF_ARP_REPLY;
            }
        }
    }
    if (et == 0x86DD && len >= 14 + 40 + 24 && d[20] == 58) {
        uint8_t type = d[54];
        if (type == 135 || type == 136) {
            if (env->apply_control) {
                size_t off = 78;
                while (off + 2 <= len) {
                    uint8_t ot = d[off];
                    /* uint8_t, as reference src/worker.c:73: the length wraps at 256 (32 -> 0, 33 -> 8) */
                    size_t ol = (uint8_t)(d[off + 1] * 8);
                    if (ol == 0 || off + ol > len) break;
                    if (type == 135 && ot == 1 && ol >= 8) {
                        upe_ref_ndp_update(env->ndp, env->ndp_cap, d + 22, d + off + 2);
                        break;
                    }
                    if (type == 136 && ot == 2 && ol >= 8) {
                        upe_ref_ndp_update(env->ndp, env->ndp_cap, d + 62, d + off + 2);
                        break;
                    }
                    off += ol;
                }
            }
            return 1;
        }
    }
    return 0;
}

/* process_packet, reference src/worker.c:106-253, for one packet in a zero-filled buffer. */
static uint32_t process_one(const upe_ref_env_t *env, upe_l1_state_t *l1, const upe_l1_state_t *l1_start,
                            uint8_t *d, size_t len, upe_counters_t *c, upe_rule_stat_t *stats,
                            size_t cap) {
    uint32_t flags = 0;
    if (control_packet(env, d, len, &flags)) {
        c->pkts_consumed++;
        return UPE_V_CONSUMED | flags;
    }
    if (flags & UPE_VF_ARP_LEARN) c->arp_learn++;
    if (flags & UPE_VF_ARP_REPLY) c->arp_reply++;

    upe_flow_key_t k;
    memset(&k, 0, sizeof k);
    if (upe_ref_parse(d, len, &k) != 0) {            /* worker.c:117-125 */
        c->pkts_dropped++;
        return UPE_V_DROP_PARSE | flags;
    }
    c->pkts_parsed++;
    long ri = upe_ref_match(env->rules, env->nrules, &k);
    if (ri < 0) {                                    /* worker.c:130-137 */
        c->pkts_dropped++;
        return UPE_V_DROP_NOMATCH | flags;
    }
    c->pkts_matched++;
    const upe_rule_t *r = &env->rules[ri];
    uint32_t rbits = (uint32_t)(ri + 1) << 8;
    if (stats && r->rule_id < cap) {                 /* worker.c:141-144 */
        stats[r->rule_id].packets++;
        stats[r->rule_id].bytes += len;
    }
    if (r->action.type == UPE_ACT_DROP) {            /* worker.c:146-153 */
        c->pkts_dropped++;
        return UPE_V_DROP_RULE | flags | rbits;
    }
    if (r->action.type != UPE_ACT_FWD) {             /* worker.c:247-252 */
        c->pkts_dropped++;
        return UPE_V_DROP_ACTION | flags | rbits;
    }
    uint8_t mac[6];
    bool found = false;
    if (k.ip_ver == 4) {                             /* worker.c:162-200 */
        if (d[22] <= 1) {
            c->pkts_dropped++;
            return UPE_V_DROP_TTL | flags | rbits;
        }
        d[22]--;
        d[24] = d[25] = 0;
        size_t hl = (size_t)(d[14] & 0x0F) * 4;
        uint16_t cs = upe_ref_ipv4_checksum(d + 14, hl);
        d[24] = (uint8_t)cs;                         /* stored natively (LE) */
        d[25] = (uint8_t)(cs >> 8);
        if (l1_start->last_arp_ip != 0 && k.dst_ip.v4 == l1_start->last_arp_ip) flags |= UPE_VF_L1_INIT;
        if (l1->last_arp_ip != 0 && k.dst_ip.v4 == l1->last_arp_ip) {
            memcpy(mac, l1->last_arp_mac, 6);
            found = true;
        } else if (upe_ref_arp_lookup(env->arp, env->arp_cap, k.dst_ip.v4, mac)) {
            l1->last_arp_ip = k.dst_ip.v4;
            memcpy(l1->last_arp_mac, mac, 6);
            found = true;
        }
    } else {                                         /* worker.c:201-231 */
        if (d[21] <= 1) {
            c->pkts_dropped++;
            return UPE_V_DROP_TTL | flags | rbits;
        }
        d[21]--;
        if (memcmp(k.dst_ip.v6, l1_start->last_ndp_ip, 16) == 0) flags |= UPE_VF_L1_INIT;
        if (memcmp(k.dst_ip.v6, l1->last_ndp_ip, 16) == 0) {
            memcpy(mac, l1->last_ndp_mac, 6);
            found = true;
        } else if (upe_ref_ndp_lookup(env->ndp, env->ndp_cap, k.dst_ip.v6, mac)) {
            memcpy(l1->last_ndp_ip, k.dst_ip.v6, 16);
            memcpy(l1->last_ndp_mac, mac, 6);
            found = true;
        }
    }
    if (found) {
        memcpy(d, mac, 6);
        memcpy(d + 6, env->eth_addr, 6);
        flags |= UPE_VF_NEIGH_HIT;
    }
    c->pkts_forwarded++;
    return UPE_V_FWD | flags | rbits;
}

/*
 * Process a batch laid out as the GPU ABI lays it out (include/upe_gpu.h "Batch layout"), in
 * order.  frames are modified in place (bytes [0, len) of each frame only).  counters,
 * rule_stats and *l1 accumulate, as worker_t's do.  pkts_in counts the whole batch.
 */
int upe_ref_process(const upe_rule_t *rules, size_t nrules, upe_arp_entry_t *arp, size_t arp_cap,
                    upe_ndp_entry_t *ndp, size_t ndp_cap, const uint8_t eth_addr[6],
                    uint32_t ip4_addr, int apply_control, upe_l1_state_t *l1, uint8_t *frames,
                    const uint64_t *desc, size_t n, uint32_t *verdict, upe_counters_t *counters,
                    upe_rule_stat_t *rule_stats, size_t capacity) {
    upe_ref_env_t env = {rules, nrules, arp, arp_cap, ndp, ndp_cap, {0}, ip4_addr, apply_control};
    memcpy(env.eth_addr, eth_addr, 6);
    upe_l1_state_t l1_start = *l1;
    uint8_t buf[PKTBUF_DATA + 128];
    counters->pkts_in += n;
    for (size_t i = 0; i < n; i++) {
        size_t off = (size_t)(desc[i] >> 16), len = (size_t)(desc[i] & 0xFFFF);
        size_t keep = len < PKTBUF_DATA ? len : PKTBUF_DATA;
        memset(buf, 0, 128); /* every read past len stays below byte 128 */
        memcpy(buf, frames + off, keep);
        verdict[i] = process_one(&env, l1, &l1_start, buf, len, counters, rule_stats, capacity);
        size_t wb = keep < 64 ? keep : 64; /* the worker writes only bytes 0..41 */
        memcpy(frames + off, buf, wb);
    }
    return 0;
}
