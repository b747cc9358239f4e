/*
 * upe_host.c — host-side batch builders around the MI355X path (C, linked into libupe_gpu.so).
 *
 * These are the two rows SURVEY.md §8(f) ranks next to the kernel: the rule-file loader that
 * fills the table the kernel classifies against, and the ingress batch builder that turns a
 * capture into the packed batch layout of include/upe_gpu.h.  Both restate the reference's
 * behaviour from its sources (no reference code is compiled in):
 *
 *   upe_rules_load_ini  reference src/rule_config.c:129-282 (rule_config_load) into a table of
 *                       rule_table_init(capacity) with rule_table_add semantics
 *                       (src/rule_table.c:130-161): rule_id = insertion index, wildcard addresses
 *                       zeroed, sorted by (priority, rule_id).
 *   upe_pcap_read       the capture side of reference src/rx_pcap.c:42-93 / 95-167 for a pcap
 *                       file: every record in file order, caplen > PKTBUF_DATA_SIZE (2048)
 *                       dropped (src/rx_pcap.c:53-57), the rest packed at 16-byte aligned offsets.
 *   upe_hdr_apply       an emit-mode record (upe_hdr_rec_t) applied to its frame: the rewrite of
 *                       src/worker.c:162-244 as bytes.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <ctype.h>
#include <errno.h>
#include <net/if.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/upe_gpu.h"

static __thread char g_host_err[256];

static int host_fail(const char *fmt, int line, const char *what) {
    snprintf(g_host_err, sizeof g_host_err, fmt, line, what ? what : "");
    return -1;
}

const char *upe_host_last_error(void) { return g_host_err; }

/* ---- rule file (INI) -------------------------------------------------------------------- */

#define UPE_MAX_LINE 512 /* src/rule_config.c:18: longer lines are read in pieces, as fgets does */

static char *strip(char *s) { /* src/rule_config.c:20-32 */
    while (*s && isspace((unsigned char)*s)) s++;
    char *end = s + strlen(s);
    while (end > s && isspace((unsigned char)end[-1])) end--;
    *end = '\0';
    return s;
}

static int mask4(uint8_t prefix, uint32_t *out) { /* src/rule_table.c:14-30 */
    if (prefix > 32) return 0;
    *out = prefix == 0 ? 0u : (uint32_t)(0xFFFFFFFFu << (32 - prefix));
    return 1;
}

static int mask6(uint8_t prefix, uint8_t out[16]) { /* src/rule_table.c:32-50 */
    if (prefix > 128) return 0;
    for (int i = 0; i < 16; i++) {
        int bits = (int)prefix - 8 * i;
        out[i] = bits >= 8 ? 0xFF : bits <= 0 ? 0 : (uint8_t)(0xFF << (8 - bits));
    }
    return 1;
}

/* "addr[/prefix]" -> address + mask, src/rule_config.c:38-91 (the prefix is taken modulo 256,
 * as the reference's uint8_t cast does; no prefix means a host route). */
static int parse_ip_prefix(const char *str, uint8_t *ver, upe_ip_addr_t *ip, upe_ip_addr_t *mask) {
    char buf[INET6_ADDRSTRLEN + 4];
    strncpy(buf, str, sizeof buf - 1);
    buf[sizeof buf - 1] = '\0';
    char *slash = strchr(buf, '/');
    uint8_t plen = 255;
    if (slash) {
        *slash = '\0';
        errno = 0;
        char *end = NULL;
        long pl = strtol(slash + 1, &end, 10);
        if (errno != 0 || end == slash + 1 || *end != '\0' || pl < 0) return -1;
        plen = (uint8_t)pl;
    }
    memset(ip, 0, sizeof *ip);
    memset(mask, 0, sizeof *mask);
    struct in_addr a4;
    if (inet_pton(AF_INET, buf, &a4) == 1) {
        *ver = 4;
        ip->v4 = ntohl(a4.s_addr);
        return mask4(plen == 255 ? 32 : plen, &mask->v4) ? 0 : -1;
    }
    struct in6_addr a6;
    if (inet_pton(AF_INET6, buf, &a6) == 1) {
        *ver = 6;
        memcpy(ip->v6, a6.s6_addr, 16);
        return mask6(plen == 255 ? 128 : plen, mask->v6) ? 0 : -1;
    }
    return -1;
}

static uint8_t parse_protocol(const char *v) { /* src/rule_config.c:93-106 */
    if (strcmp(v, "tcp") == 0) return 6;
    if (strcmp(v, "udp") == 0) return 17;
    if (strcmp(v, "icmp") == 0) return 1;
    if (strcmp(v, "icmpv6") == 0) return 58;
    errno = 0;
    char *end = NULL;
    long x = strtol(v, &end, 10);
    if (errno == 0 && end != v && *end == '\0' && x >= 0 && x <= 255) return (uint8_t)x;
    return 0;
}

static int parse_long(const char *v, long lo, long hi, long *out) {
    errno = 0;
    char *end = NULL;
    long x = strtol(v, &end, 10);
    if (errno != 0 || end == v || *end != '\0' || x < lo || x > hi) return -1;
    *out = x;
    return 0;
}

/* rule_table_add, src/rule_table.c:130-161 (the sort happens once, at the end: the comparator
 * is a total order over unique rule_ids, so the result is the same). */
static int table_add(upe_rule_t *rules, size_t capacity, size_t *count, const upe_rule_t *in) {
    if (*count >= capacity) return -1;
    upe_rule_t r = *in;
    r.rule_id = (uint32_t)*count;
    static const uint8_t zero16[16];
    if (r.ip_ver == 4 && r.src_mask.v4 == 0) r.src_ip.v4 = 0;
    if (r.ip_ver == 4 && r.dst_mask.v4 == 0) r.dst_ip.v4 = 0;
    if (r.ip_ver == 6) {
        if (memcmp(r.src_mask.v6, zero16, 16) == 0) memset(r.src_ip.v6, 0, 16);
        if (memcmp(r.dst_mask.v6, zero16, 16) == 0) memset(r.dst_ip.v6, 0, 16);
    }
    rules[(*count)++] = r;
    return 0;
}

static int rule_cmp(const void *a, const void *b) { /* src/rule_table.c:96-109 */
    const upe_rule_t *x = a, *y = b;
    if (x->priority != y->priority) return x->priority < y->priority ? -1 : 1;
    if (x->rule_id != y->rule_id) return x->rule_id < y->rule_id ? -1 : 1;
    return 0;
}

static int flush_rule(upe_rule_t *r, int *active, upe_rule_t *rules, size_t capacity,
                      size_t *count, int line) { /* src/rule_config.c:112-127 */
    if (!*active) return 0;
    *active = 0;
    if (r->action.type == UPE_ACT_FWD && r->action.out_ifindex == 0)
        return host_fail("rules:%d: fwd rule missing out_iface%s", line, "");
    if (table_add(rules, capacity, count, r) != 0)
        return host_fail("rules:%d: failed to add rule (table may be full)%s", line, "");
    return 0;
}

int upe_rules_load_ini(const char *path, upe_rule_t *rules, size_t capacity, size_t *count) {
    if (!path || !rules || !count || capacity == 0) return host_fail("rules:%d: bad argument%s", 0, "");
    FILE *f = fopen(path, "r");
    if (!f) return host_fail("rules:%d: unable to open %s", 0, path);
    *count = 0;
    char line[UPE_MAX_LINE];
    int ln = 0, active = 0, rc = 0;
    upe_rule_t cur;
    memset(&cur, 0, sizeof cur);
    while (rc == 0 && fgets(line, UPE_MAX_LINE, f)) {
        ln++;
        line[strcspn(line, "\r\n")] = '\0';
        char *s = strip(line);
        if (*s == '\0' || *s == '#' || *s == ';') continue;
        if (*s == '[') {
            if ((rc = flush_rule(&cur, &active, rules, capacity, count, ln)) != 0) break;
            if (strncmp(s, "[rule]", 6) != 0) {
                rc = host_fail("rules:%d: unknown section header: %s", ln, s);
                break;
            }
            memset(&cur, 0, sizeof cur);
            active = 1;
            continue;
        }
        if (!active) {
            rc = host_fail("rules:%d: key=value outside [rule] section%s", ln, "");
            break;
        }
        char *eq = strchr(s, '=');
        if (!eq) {
            rc = host_fail("rules:%d: expected key = value%s", ln, "");
            break;
        }
        *eq = '\0';
        char *key = strip(s), *val = strip(eq + 1);
        long x;
        uint8_t ver = 0;
        if (strcmp(key, "priority") == 0) {
            if (parse_long(val, 0, __LONG_MAX__, &x) != 0) rc = host_fail("rules:%d: invalid priority: %s", ln, val);
            else cur.priority = (uint32_t)x;
        } else if (strcmp(key, "ip_version") == 0) {
            if (strcmp(val, "4") == 0) cur.ip_ver = 4;
            else if (strcmp(val, "6") == 0) cur.ip_ver = 6;
            else rc = host_fail("rules:%d: invalid ip_version: %s", ln, val);
        } else if (strcmp(key, "protocol") == 0) {
            cur.protocol = parse_protocol(val);
        } else if (strcmp(key, "src") == 0 || strcmp(key, "dst") == 0) {
            const int src = key[0] == 's';
            if (parse_ip_prefix(val, &ver, src ? &cur.src_ip : &cur.dst_ip,
                                src ? &cur.src_mask : &cur.dst_mask) != 0)
                rc = host_fail(src ? "rules:%d: invalid src address: %s"
                                   : "rules:%d: invalid dst address: %s", ln, val);
            else if (cur.ip_ver == 0)
                cur.ip_ver = ver;
        } else if (strcmp(key, "src_port") == 0 || strcmp(key, "dst_port") == 0) {
            if (parse_long(val, 0, 65535, &x) != 0)
                rc = host_fail("rules:%d: invalid port: %s", ln, val);
            else if (key[0] == 's')
                cur.src_port = (uint16_t)x;
            else
                cur.dst_port = (uint16_t)x;
        } else if (strcmp(key, "action") == 0) {
            if (strcmp(val, "drop") == 0) cur.action.type = UPE_ACT_DROP;
            else if (strcmp(val, "fwd") == 0) cur.action.type = UPE_ACT_FWD;
            else rc = host_fail("rules:%d: invalid action: %s", ln, val);
        } else if (strcmp(key, "out_iface") == 0) {
            unsigned idx = if_nametoindex(val);
            if (idx == 0) rc = host_fail("rules:%d: unknown interface: %s", ln, val);
            else cur.action.out_ifindex = (int32_t)idx;
        } else {
            rc = host_fail("rules:%d: unknown key: %s", ln, key);
        }
    }
    if (rc == 0) rc = flush_rule(&cur, &active, rules, capacity, count, ln);
    fclose(f);
    if (rc != 0) return -1;
    qsort(rules, *count, sizeof(upe_rule_t), rule_cmp);
    return 0;
}

/* ---- pcap capture -> packed batch --------------------------------------------------------- */

#define PKTBUF_DATA_SIZE 2048 /* reference include/pktbuf.h:8 */

static uint32_t rd32(const uint8_t *p, int swap) {
    uint32_t v;
    memcpy(&v, p, 4);
    return swap ? __builtin_bswap32(v) : v;
}

int upe_pcap_read(const char *path, uint8_t *frames, size_t frames_cap, uint64_t *desc,
                  size_t desc_cap, upe_pcap_info_t *info) {
    if (!path || !info) return host_fail("pcap:%d: bad argument%s", 0, "");
    memset(info, 0, sizeof *info);
    FILE *f = fopen(path, "rb");
    if (!f) return host_fail("pcap:%d: unable to open %s", 0, path);
    uint8_t gh[24];
    if (fread(gh, 1, 24, f) != 24) {
        fclose(f);
        return host_fail("pcap:%d: short global header%s", 0, "");
    }
    uint32_t magic;
    memcpy(&magic, gh, 4);
    int swap;
    if (magic == 0xa1b2c3d4u || magic == 0xa1b23c4du) swap = 0;
    else if (magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u) swap = 1;
    else {
        fclose(f);
        return host_fail("pcap:%d: not a pcap file (magic)%s", 0, "");
    }
    if (rd32(gh + 20, swap) != 1) {
        fclose(f);
        return host_fail("pcap:%d: link type is not Ethernet%s", 0, "");
    }
    const int fill = frames && desc;
    size_t cursor = 0, n = 0;
    uint8_t rh[16];
    uint8_t *buf = malloc(65536 * 4);
    if (!buf) {
        fclose(f);
        return host_fail("pcap:%d: out of memory%s", 0, "");
    }
    int rc = 0;
    for (;;) {
        size_t got = fread(rh, 1, 16, f);
        if (got == 0) break;
        if (got != 16) {
            rc = host_fail("pcap:%d: truncated record header%s", (int)info->records, "");
            break;
        }
        const uint32_t caplen = rd32(rh + 8, swap);
        if (caplen > 65536u * 4) {
            rc = host_fail("pcap:%d: record too large%s", (int)info->records, "");
            break;
        }
        if (fread(buf, 1, caplen, f) != caplen) {
            rc = host_fail("pcap:%d: truncated record%s", (int)info->records, "");
            break;
        }
        info->records++;
        if (caplen > PKTBUF_DATA_SIZE) { /* src/rx_pcap.c:53-57 */
            info->dropped_oversize++;
            continue;
        }
        const size_t sz = caplen ? (caplen + 15u) & ~(size_t)15u : 16u;
        if (fill) {
            if (n >= desc_cap || cursor + sz + UPE_FRAME_TAIL > frames_cap) {
                rc = host_fail("pcap:%d: batch buffers too small%s", (int)info->records, "");
                break;
            }
            memcpy(frames + cursor, buf, caplen);
            memset(frames + cursor + caplen, 0, sz - caplen);
            desc[n] = UPE_DESC(cursor, caplen);
        }
        cursor += sz;
        n++;
    }
    free(buf);
    fclose(f);
    info->packets = n;
    info->frames_bytes = cursor + UPE_FRAME_TAIL;
    if (rc == 0 && fill) memset(frames + cursor, 0, UPE_FRAME_TAIL);
    return rc;
}

/* ---- emit-mode records ------------------------------------------------------------------- */

/* The bytes process_packet leaves in a forwarded frame (reference src/worker.c:174-176 TTL and
 * checksum, :197-200 / :227-230 MACs, :213 hop limit), from a upe_hdr_rec_t. */
void upe_hdr_apply(uint8_t *frame, const upe_hdr_rec_t *rec) {
    const uint8_t fam = rec->b[15];
    if (fam != 4 && fam != 6) return;
    memcpy(frame, rec->b, 12);
    if (fam == 4) {
        frame[22] = rec->b[12];
        frame[24] = rec->b[13];
        frame[25] = rec->b[14];
    } else {
        frame[21] = rec->b[12];
    }
}

/* ---- egress ------------------------------------------------------------------------------ */

/* The TX side of the worker loop (src/worker.c:240-243 queue, :287-303 flush): per input burst,
 * the forwarded frames in packet order go to one tx_send_batch-like call. */
int upe_tx_flush(const uint8_t *h_frames, const uint64_t *h_desc, const uint32_t *h_verdict,
                 size_t n, size_t burst, upe_tx_batch_fn send, void *user, uint64_t *forwarded,
                 uint64_t *dropped) {
    if (burst == 0 || burst > UPE_TX_BATCH_MAX)
        return host_fail("upe_tx_flush: burst %d must be 1..UPE_TX_BATCH_MAX", (int)burst, "");
    if (n && (!h_frames || !h_desc || !h_verdict || !send))
        return host_fail("upe_tx_flush: null argument%.0d%s", 0, "");
    const uint8_t *frames[UPE_TX_BATCH_MAX];
    size_t lens[UPE_TX_BATCH_MAX];
    for (size_t base = 0; base < n; base += burst) {
        const size_t end = n - base < burst ? n : base + burst;
        int count = 0;
        for (size_t i = base; i < end; i++) {
            if (UPE_VERDICT_CODE(h_verdict[i]) != UPE_V_FWD) continue;
            frames[count] = h_frames + (h_desc[i] >> 16);
            lens[count++] = (size_t)(h_desc[i] & 0xFFFFu);
        }
        if (count == 0) continue;   /* src/worker.c:287: no call for an all-dropped burst */
        int sent = send(user, frames, lens, count);
        if (sent < 0) sent = 0;
        if (sent > count) sent = count;
        if (forwarded) *forwarded += (uint64_t)sent;
        if (dropped) *dropped += (uint64_t)(count - sent);
    }
    return 0;
}

int upe_tx_flush_groups(const uint8_t *h_frames, const uint64_t *h_desc, const uint32_t *h_tx,
                        const uint32_t *h_tx_count, size_t n, size_t burst, upe_tx_batch_fn send,
                        void *user, uint64_t *forwarded, uint64_t *dropped) {
    if (burst == 0 || burst > UPE_TX_BATCH_MAX)
        return host_fail("upe_tx_flush_groups: burst %d must be 1..UPE_TX_BATCH_MAX", (int)burst, "");
    if (n && (!h_frames || !h_desc || !h_tx || !h_tx_count || !send))
        return host_fail("upe_tx_flush_groups: null argument%.0d%s", 0, "");
    const uint8_t *frames[UPE_TX_BATCH_MAX];
    size_t lens[UPE_TX_BATCH_MAX];
    size_t g = 0, k = 0; /* the next list entry: group g, its k-th forwarded packet */
    for (size_t base = 0; base < n; base += burst) {
        const size_t end = n - base < burst ? n : base + burst;
        int count = 0;
        for (;;) {
            if (g * 64 >= end || g * 64 >= n) break;
            const uint32_t cnt = h_tx_count[g];
            if (cnt > 64) return host_fail("upe_tx_flush_groups: group count %d above 64", (int)cnt, "");
            if (k >= cnt) { g++; k = 0; continue; }
            const uint32_t i = h_tx[g * 64 + k];
            if (i >= end) break; /* the next burst's */
            if (i < base || count == (int)burst)
                return host_fail("upe_tx_flush_groups: list entry %d out of packet order%s", (int)i, "");
            frames[count] = h_frames + (h_desc[i] >> 16);
            lens[count++] = (size_t)(h_desc[i] & 0xFFFFu);
            k++;
        }
        if (count == 0) continue; /* src/worker.c:287: no call for an all-dropped burst */
        int sent = send(user, frames, lens, count);
        if (sent < 0) sent = 0;
        if (sent > count) sent = count;
        if (forwarded) *forwarded += (uint64_t)sent;
        if (dropped) *dropped += (uint64_t)(count - sent);
    }
    return 0;
}

int upe_gpu_hdr_layout(void) { return UPE_HDR_LAYOUT; }
