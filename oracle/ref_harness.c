/*
 * oracle/ref_harness.c — drives the REFERENCE worker's own process_packet() over a batch.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle/cpu_ref.c header).  Built by oracle/Makefile straight from
 * the reference sources where they lie (the reference src/ directory, never copied), into
 * oracle/_ref/libupe_ref.so (git-ignored).  It is the ground truth the golden vectors in
 * tests/golden/ are generated from, and the timed CPU baseline ("kind": "reference") of bench.py.
 *
 * process_packet() is static in reference src/worker.c:106, so this file #includes that .c (the
 * technique reference router/bench/test_forwarding.c:8 uses for rx_lcore.c).  Around it the
 * harness reproduces worker_main's burst loop (src/worker.c:267-303) minus the ring pop:
 * bursts of WORKER_BURST_SIZE packets, process_packet on each, then the TX flush.  TX is stubbed
 * like reference tests/benchmark_throughput.c:30-42 (tx_send_batch returns count) and tx_send
 * records ARP replies.  The worker_t is calloc'd (as src/main.c:444), buffers are zero-filled
 *  and timestamps are 0 so no latency sample is taken.
 *
 * The verdict word (include/upe_gpu.h) is derived from what process_packet observably did:
 * counter deltas, whether the buffer reached w->tx_bufs, the rule rule_table_match() returns for
 * the original bytes, and the worker's L1 cache / arp_get_mac / ndp_get_mac answers just before.
 */
#define _GNU_SOURCE
#include "worker.c" /* reference src/worker.c, via -I<reference>/src */

#include <pthread.h>
#include <stdio.h>
#include <time.h>

#include "../include/upe_gpu.h"

volatile sig_atomic_t g_stop = 0; /* defined by the program, src/main.c:27 */

static __thread int t_replies; /* tx_send calls seen by this thread */

int tx_send(const tx_ctx_t *ctx, const uint8_t *frame, size_t len) {
    (void)ctx; (void)frame; (void)len;
    t_replies++;
    return 0;
}

/* The TX log of the last upe_refh_process run on this thread: per tx_send_batch call its frame
 * count, and per frame the packet index (t_tx_idx maps the worker's tx slots to packet indexes). */
static __thread size_t t_tx_idx[TX_BATCH_MAX];
static __thread uint32_t *t_log_sizes, *t_log_frames;
static __thread size_t t_log_nb, t_log_nf, t_log_cap_b, t_log_cap_f;

int tx_send_batch(const tx_ctx_t *ctx, const uint8_t *const *frames, const size_t *lens, int count) {
    (void)ctx; (void)frames; (void)lens;
    if (t_log_nb == t_log_cap_b) {
        t_log_cap_b = t_log_cap_b ? 2 * t_log_cap_b : 1024;
        t_log_sizes = realloc(t_log_sizes, t_log_cap_b * sizeof(uint32_t));
    }
    if (t_log_nf + (size_t)count > t_log_cap_f) {
        while (t_log_nf + (size_t)count > t_log_cap_f) t_log_cap_f = t_log_cap_f ? 2 * t_log_cap_f : 4096;
        t_log_frames = realloc(t_log_frames, t_log_cap_f * sizeof(uint32_t));
    }
    if (!t_log_sizes || !t_log_frames) return count;
    t_log_sizes[t_log_nb++] = (uint32_t)count;
    for (int k = 0; k < count; k++) t_log_frames[t_log_nf++] = (uint32_t)t_tx_idx[k];
    return count;
}

/* The last run's TX log (upe_refh_process): *nb batches, sizes[0..nb), and the packet index of
 * every frame handed to tx_send_batch in call order, frames[0..nf).  Either array may be NULL to
 * ask for the counts. */
int upe_refh_tx_log(uint32_t *sizes, size_t cap_b, uint32_t *frames, size_t cap_f, size_t *nb,
                    size_t *nf) {
    *nb = t_log_nb;
    *nf = t_log_nf;
    if (sizes && cap_b >= t_log_nb) memcpy(sizes, t_log_sizes, t_log_nb * sizeof(uint32_t));
    if (frames && cap_f >= t_log_nf) memcpy(frames, t_log_frames, t_log_nf * sizeof(uint32_t));
    return 0;
}

/* The TX flush of worker_main, src/worker.c:286-303. */
static void flush_tx(worker_t *w) {
    if (w->tx_count > 0) {
        int sent = tx_send_batch(w->tx, w->tx_frames, w->tx_lens, w->tx_count);
        if (sent < 0) sent = 0;
        w->pkts_forwarded += (uint64_t)sent;
        w->pkts_dropped += (uint64_t)(w->tx_count - sent);
        for (int i = 0; i < w->tx_count; i++) pktbuf_free(w->pool, w->tx_bufs[i]);
        w->tx_count = 0;
    }
}

static int build_rules(rule_table_t *rt, const upe_rule_t *rules, size_t nrules, size_t capacity,
                       int presorted) {
    if (rule_table_init(rt, capacity) != 0) return -1;
    if (presorted) {
        /* Large tables: the caller passes the final sorted array (checked equal to repeated
         * rule_table_add on smaller tables by the tests); avoids O(n^2 log n) qsorts. */
        if (nrules > capacity) return -1;
        memcpy(rt->rules, rules, nrules * sizeof(rule_t));
        rt->count = nrules;
        return 0;
    }
    for (size_t i = 0; i < nrules; i++)
        if (rule_table_add(rt, (const rule_t *)&rules[i]) != 0) return -1;
    return 0;
}

static void put_l1(worker_t *w, const upe_l1_state_t *l1) {
    w->last_arp_ip = l1->last_arp_ip;
    memcpy(w->last_arp_mac, l1->last_arp_mac, 6);
    memcpy(w->last_ndp_ip, l1->last_ndp_ip, 16);
    memcpy(w->last_ndp_mac, l1->last_ndp_mac, 6);
}

static void get_l1(const worker_t *w, upe_l1_state_t *l1) {
    l1->last_arp_ip = w->last_arp_ip;
    memcpy(l1->last_arp_mac, w->last_arp_mac, 6);
    memcpy(l1->last_ndp_ip, w->last_ndp_ip, 16);
    memcpy(l1->last_ndp_mac, w->last_ndp_mac, 6);
}

/* One pass of worker_main's burst loop (src/worker.c:267-303, minus the ring pop) over packets
 * [i0, i1): bursts of WORKER_BURST_SIZE, process_packet on each packet with the worker's current
 * w->rt, then the TX flush; the verdict word of each packet read back from what process_packet
 * observably did (file header). */
static pktbuf_pool_t g_pool;
static int g_pool_ready;

static int run_range(worker_t *w, const upe_l1_state_t *l1_start, uint8_t *frames,
                     const uint64_t *desc, size_t i0, size_t i1, uint32_t *verdict,
                     upe_counters_t *counters) {
    const rule_table_t *rt = w->rt;
    uint8_t orig[PKTBUF_DATA_SIZE];
    int rc = 0;
    for (size_t base = i0; base < i1; base += WORKER_BURST_SIZE) {
        size_t cnt = i1 - base < WORKER_BURST_SIZE ? i1 - base : WORKER_BURST_SIZE;
        w->pkts_in += cnt; /* src/worker.c:280 */
        for (size_t j = 0; j < cnt; j++) {
            size_t i = base + j;
            size_t off = (size_t)(desc[i] >> 16), len = (size_t)(desc[i] & 0xFFFF);
            if (len > PKTBUF_DATA_SIZE) { rc = -1; len = PKTBUF_DATA_SIZE; }
            pktbuf_t *b = pktbuf_alloc(&g_pool);
            if (!b) return -1;
            memset(b->data, 0, PKTBUF_DATA_SIZE);
            memcpy(b->data, frames + off, len);
            b->len = len;
            b->timestamp = 0;
            memcpy(orig, b->data, 128);

            /* State just before the call, to read back the verdict. */
            uint64_t d0 = w->pkts_dropped, p0 = w->pkts_parsed, m0 = w->pkts_matched;
            int tx0 = w->tx_count, rep0 = t_replies;
            uint32_t flags = 0;
            uint16_t et = (uint16_t)((orig[12] << 8) | orig[13]);
            if (et == ETH_TYPE_ARP && orig[14] == 0 && orig[15] == 1 && orig[16] == 0x08 &&
                orig[17] == 0x00 && orig[18] == 6 && orig[19] == 4) {
                flags |= UPE_VF_ARP_LEARN;
                counters->arp_learn++;
            }
            flow_key_t key;
            memset(&key, 0, sizeof key);
            int parsed = parse_flow_key(orig, len, &key) == 0;
            bool hit = false, l1_init = false;
            if (parsed && key.ip_ver == 4) {
                uint8_t mac[6];
                hit = (w->last_arp_ip != 0 && key.dst_ip.v4 == w->last_arp_ip) ||
                      arp_get_mac(w->arpt, key.dst_ip.v4, mac);
                l1_init = l1_start->last_arp_ip != 0 && key.dst_ip.v4 == l1_start->last_arp_ip;
            } else if (parsed && key.ip_ver == 6) {
                uint8_t mac[6];
                hit = memcmp(key.dst_ip.v6, w->last_ndp_ip, 16) == 0 ||
                      ndp_get_mac(w->ndpt, key.dst_ip.v6, mac);
                l1_init = memcmp(key.dst_ip.v6, l1_start->last_ndp_ip, 16) == 0;
            }

            process_packet(w, b);

            if (t_replies != rep0) {
                flags |= UPE_VF_ARP_REPLY;
                counters->arp_reply++;
            }
            uint32_t v;
            if (w->tx_count != tx0) t_tx_idx[tx0] = i;   /* the TX log's packet index */
            if (w->tx_count != tx0) {
                v = UPE_V_FWD | (hit ? UPE_VF_NEIGH_HIT : 0) | (l1_init ? UPE_VF_L1_INIT : 0);
            } else if (w->pkts_dropped == d0) {
                v = UPE_V_CONSUMED; /* handle_control_packet ate it, src/worker.c:96-98 */
                counters->pkts_consumed++;
            } else if (w->pkts_parsed == p0) {
                v = UPE_V_DROP_PARSE;
            } else if (w->pkts_matched == m0) {
                v = UPE_V_DROP_NOMATCH;
            } else {
                const rule_t *r = rule_table_match(rt, &key);
                v = r->action.type == ACT_DROP  ? UPE_V_DROP_RULE
                    : r->action.type == ACT_FWD ? UPE_V_DROP_TTL
                                                : UPE_V_DROP_ACTION;
            }
            if (w->pkts_matched != m0) {
                const rule_t *r = rule_table_match(rt, &key);
                v |= (uint32_t)(r - rt->rules + 1) << 8;
            }
            verdict[i] = v | flags;
            size_t wb = len < 64 ? len : 64;
            memcpy(frames + off, b->data, wb);
        }
        flush_tx(w);
    }
    return rc;
}

/* A calloc'd worker_t (src/main.c:444) over the given tables, with the caller's L1 state,
 * counters and rule_stats[capacity]. */
static worker_t *new_worker(const rule_table_t *rt, const tx_ctx_t *tx, arp_table_t *arpt,
                            ndp_table_t *ndpt, const upe_l1_state_t *l1,
                            const upe_counters_t *counters, const upe_rule_stat_t *rule_stats,
                            size_t capacity) {
    /* One pool for the process lifetime: pktbuf.c's thread-local cache remembers the pool by
     * address (src/pktbuf.c:298-303), so a destroyed pool must never be followed by a new one
     * on the same thread. */
    if (!g_pool_ready) {
        if (pktbuf_pool_init(&g_pool, 256) != 0) return NULL;
        g_pool_ready = 1;
    }
    worker_t *w = calloc(1, sizeof(worker_t));
    if (!w || worker_init(w, 0, -1, NULL, &g_pool, rt, tx, arpt, ndpt) != 0) return NULL;
    put_l1(w, l1);
    if (rule_stats) memcpy(w->rule_stats, rule_stats, capacity * sizeof(rule_stat_t));
    w->pkts_in = counters->pkts_in;
    w->pkts_parsed = counters->pkts_parsed;
    w->pkts_matched = counters->pkts_matched;
    w->pkts_forwarded = counters->pkts_forwarded;
    w->pkts_dropped = counters->pkts_dropped;
    return w;
}

static void worker_out(const worker_t *w, upe_l1_state_t *l1, upe_counters_t *counters) {
    get_l1(w, l1);
    counters->pkts_in = w->pkts_in;
    counters->pkts_parsed = w->pkts_parsed;
    counters->pkts_matched = w->pkts_matched;
    counters->pkts_forwarded = w->pkts_forwarded;
    counters->pkts_dropped = w->pkts_dropped;
}

typedef struct {
    arp_table_t arpt;
    ndp_table_t ndpt;
    tx_ctx_t tx;
} env_t;

static int env_init(env_t *e, const upe_arp_entry_t *arp, size_t arp_cap,
                    const upe_ndp_entry_t *ndp, size_t ndp_cap, const uint8_t eth_addr[6],
                    uint32_t ip4_addr) {
    size_t acap = arp_cap ? arp_cap : 1, ncap = ndp_cap ? ndp_cap : 1;
    if (arp_table_init(&e->arpt, acap) != 0 || ndp_table_init(&e->ndpt, ncap) != 0) return -1;
    if (arp_cap) memcpy(e->arpt.entries, arp, arp_cap * sizeof(arp_entry_t));
    if (ndp_cap) memcpy(e->ndpt.entries, ndp, ndp_cap * sizeof(ndp_entry_t));
    memset(&e->tx, 0, sizeof e->tx);
    memcpy(e->tx.eth_addr, eth_addr, 6);
    e->tx.ip4_addr = ip4_addr;
    return 0;
}

static void env_out(env_t *e, upe_arp_entry_t *arp, size_t arp_cap, upe_ndp_entry_t *ndp,
                    size_t ndp_cap) {
    if (arp_cap) memcpy(arp, e->arpt.entries, arp_cap * sizeof(arp_entry_t));
    if (ndp_cap) memcpy(ndp, e->ndpt.entries, ndp_cap * sizeof(ndp_entry_t));
    arp_table_destroy(&e->arpt);
    ndp_table_destroy(&e->ndpt);
}

/*
 * Process a batch (include/upe_gpu.h "Batch layout") through the reference worker.
 * rules: insertion order (rule_table_add assigns rule_id and sorts) unless presorted.
 * sorted_out (optional): rt->rules after the build.
 * arp/ndp: slot arrays, updated in place by control packets exactly as the reference does.
 * l1, counters, rule_stats[capacity]: in/out, accumulate.
 */
int upe_refh_process(const upe_rule_t *rules, size_t nrules, size_t capacity, int presorted,
                     upe_rule_t *sorted_out, upe_arp_entry_t *arp, size_t arp_cap,
                     upe_ndp_entry_t *ndp, size_t ndp_cap, const uint8_t eth_addr[6],
                     uint32_t ip4_addr, upe_l1_state_t *l1, uint8_t *frames, const uint64_t *desc,
                     size_t n, uint32_t *verdict, upe_counters_t *counters,
                     upe_rule_stat_t *rule_stats) {
    rule_table_t rt;
    if (build_rules(&rt, rules, nrules, capacity, presorted) != 0) return -1;
    if (sorted_out) memcpy(sorted_out, rt.rules, rt.count * sizeof(rule_t));
    env_t e;
    if (env_init(&e, arp, arp_cap, ndp, ndp_cap, eth_addr, ip4_addr) != 0) return -1;
    worker_t *w = new_worker(&rt, &e.tx, &e.arpt, &e.ndpt, l1, counters, rule_stats, capacity);
    if (!w) return -1;
    const upe_l1_state_t l1_start = *l1;
    t_log_nb = t_log_nf = 0;
    int rc = run_range(w, &l1_start, frames, desc, 0, n, verdict, counters);
    worker_out(w, l1, counters);
    if (rule_stats) memcpy(rule_stats, w->rule_stats, capacity * sizeof(rule_stat_t));
    env_out(&e, arp, arp_cap, ndp, ndp_cap);
    worker_destroy(w);
    free(w);
    rule_table_destroy(&rt);
    return rc;
}

/*
 * The same with the stats thread's SIGHUP reload (src/main.c:216-282) between packets at-1 and
 * at: packets [0, at) run with table A (rules_a, capacity cap_a), then — between two bursts, as
 * the stats thread's plain pointer stores land between the worker's bursts — w->rt becomes table
 * B (rules_b in insertion order, rule_table_init(cap_b) + rule_table_add) and w->rule_stats a
 * fresh calloc(cap_b) array; pkts_* and the L1 caches carry on.  Outputs: sorted_b (table B as
 * built), stats_a[cap_a] (the old array as it was at the swap), stats_b[cap_b], and as
 * upe_refh_process the rest.  Verdict rule indexes refer to the table each packet ran with.
 */
int upe_refh_process_reload(const upe_rule_t *rules_a, size_t n_a, size_t cap_a,
                            const upe_rule_t *rules_b, size_t n_b, size_t cap_b,
                            upe_rule_t *sorted_b, size_t at, upe_arp_entry_t *arp, size_t arp_cap,
                            upe_ndp_entry_t *ndp, size_t ndp_cap, const uint8_t eth_addr[6],
                            uint32_t ip4_addr, upe_l1_state_t *l1, uint8_t *frames,
                            const uint64_t *desc, size_t n, uint32_t *verdict,
                            upe_counters_t *counters, upe_rule_stat_t *stats_a,
                            upe_rule_stat_t *stats_b) {
    if (at > n) return -1;
    rule_table_t *rt_a = malloc(sizeof *rt_a), *rt_b = malloc(sizeof *rt_b);
    if (!rt_a || !rt_b || build_rules(rt_a, rules_a, n_a, cap_a, 0) != 0 ||
        build_rules(rt_b, rules_b, n_b, cap_b, 0) != 0)
        return -1;
    if (sorted_b) memcpy(sorted_b, rt_b->rules, rt_b->count * sizeof(rule_t));
    env_t e;
    if (env_init(&e, arp, arp_cap, ndp, ndp_cap, eth_addr, ip4_addr) != 0) return -1;
    worker_t *w = new_worker(rt_a, &e.tx, &e.arpt, &e.ndpt, l1, counters, NULL, cap_a);
    if (!w) return -1;
    const upe_l1_state_t l1_start = *l1;
    t_log_nb = t_log_nf = 0;
    int rc = run_range(w, &l1_start, frames, desc, 0, at, verdict, counters);
    /* the stats thread's swap (src/main.c:237-265) */
    rule_stat_t *new_stats = calloc(rt_b->capacity, sizeof(rule_stat_t));
    if (!new_stats) return -1;
    rule_stat_t *old_stats = w->rule_stats;
    w->rule_stats = new_stats;
    w->rt = rt_b;
    memcpy(stats_a, old_stats, cap_a * sizeof(rule_stat_t));
    free(old_stats); /* after the grace period, src/main.c:270-275 */
    rule_table_destroy(rt_a);
    free(rt_a);
    if (rc == 0) rc = run_range(w, &l1_start, frames, desc, at, n, verdict, counters);
    worker_out(w, l1, counters);
    memcpy(stats_b, w->rule_stats, cap_b * sizeof(rule_stat_t));
    env_out(&e, arp, arp_cap, ndp, ndp_cap);
    worker_destroy(w);
    free(w);
    rule_table_destroy(rt_b);
    free(rt_b);
    return rc;
}

/* ---- the reference's rule-file loader (src/rule_config.c:129-282) into a fresh table -------- */
#include "rule_config.h"

int upe_refh_rules_load(const char *path, size_t capacity, upe_rule_t *out, size_t *count) {
    rule_table_t rt;
    if (rule_table_init(&rt, capacity) != 0) return -2;
    log_set_level(LOG_ERROR); /* only the reference's error lines */
    int rc = rule_config_load(path, &rt);
    memcpy(out, rt.rules, rt.count * sizeof(rule_t));
    *count = rt.count;
    rule_table_destroy(&rt);
    return rc;
}

/* ---- timed CPU baseline ------------------------------------------------------------------- */

typedef struct {
    pthread_barrier_t *bar;
    int cpu;
    const rule_table_t *rt;
    const tx_ctx_t *tx;
    arp_table_t *arpt;
    ndp_table_t *ndpt;
    const uint8_t *frames;
    const uint64_t *desc;
    size_t begin, end;
    int reps;
    double *secs; /* [reps] */
    uint64_t fwd;
} tshard_t;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC_RAW, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void *shard_main(void *arg) {
    tshard_t *s = arg;
    if (s->cpu >= 0) affinity_pin_self(s->cpu);
    size_t n = s->end - s->begin;
    pktbuf_pool_t pool;
    pktbuf_pool_init(&pool, n + 64);
    pktbuf_t **bufs = malloc(n * sizeof(*bufs));
    worker_t *w = calloc(1, sizeof(worker_t));
    worker_init(w, 0, -1, NULL, &pool, s->rt, s->tx, s->arpt, s->ndpt);

    for (int r = -1; r < s->reps; r++) { /* r = -1 is the warm-up */
        /* untimed: allocate and fill, as the RX thread would; the worker frees every buffer
         * (drops at once, forwards after the TX flush), so the pool is full again after a pass */
        for (size_t i = 0; i < n; i++) {
            bufs[i] = pktbuf_alloc(&pool);
            if (!bufs[i]) abort();
            size_t off = (size_t)(s->desc[s->begin + i] >> 16);
            size_t len = (size_t)(s->desc[s->begin + i] & 0xFFFF);
            if (len > PKTBUF_DATA_SIZE) len = PKTBUF_DATA_SIZE;
            memset(bufs[i]->data, 0, 128);
            memcpy(bufs[i]->data, s->frames + off, len);
            bufs[i]->len = len;
            bufs[i]->timestamp = 0;
        }
        const upe_l1_state_t zero_l1 = {0};
        put_l1(w, &zero_l1); /* every rep starts from a calloc'd worker's caches */
        pthread_barrier_wait(s->bar);
        double t0 = now_s();
        for (size_t base = 0; base < n; base += WORKER_BURST_SIZE) {
            size_t cnt = n - base < WORKER_BURST_SIZE ? n - base : WORKER_BURST_SIZE;
            w->pkts_in += cnt;
            for (size_t j = 0; j < cnt; j++) process_packet(w, bufs[base + j]);
            flush_tx(w);
        }
        double t1 = now_s();
        if (r >= 0) s->secs[r] = t1 - t0;
        pthread_barrier_wait(s->bar);
    }
    s->fwd = w->pkts_forwarded;
    worker_destroy(w);
    free(w);
    free(bufs);
    pktbuf_pool_destroy(&pool);
    return NULL;
}

/*
 * Time the reference worker over a batch: `threads` workers, each pinned to cpus[t] (or
 * unpinned when cpus is NULL), one contiguous shard each, own calloc'd worker_t, shared rule
 * table and neighbour tables (as src/main.c:444-456).  rules are final sorted rt->rules.
 * Returns the median over `reps` of (n / max-over-threads seconds) in packets/s, or -1;
 * rates_out (optional, `reps` doubles) receives every rep's rate, ascending.
 */
double upe_refh_time(const upe_rule_t *rules, size_t nrules, size_t capacity,
                     const upe_arp_entry_t *arp, size_t arp_cap, const upe_ndp_entry_t *ndp,
                     size_t ndp_cap, const uint8_t eth_addr[6], uint32_t ip4_addr,
                     const uint8_t *frames, const uint64_t *desc, size_t n, int threads,
                     const int *cpus, int reps, double *rates_out) {
    if (threads < 1 || reps < 1 || n == 0) return -1;
    rule_table_t rt;
    if (build_rules(&rt, rules, nrules, capacity, 1) != 0) return -1;
    arp_table_t arpt;
    ndp_table_t ndpt;
    arp_table_init(&arpt, arp_cap ? arp_cap : 1);
    ndp_table_init(&ndpt, ndp_cap ? ndp_cap : 1);
    if (arp_cap) memcpy(arpt.entries, arp, arp_cap * sizeof(arp_entry_t));
    if (ndp_cap) memcpy(ndpt.entries, ndp, ndp_cap * sizeof(ndp_entry_t));
    tx_ctx_t tx;
    memset(&tx, 0, sizeof tx);
    memcpy(tx.eth_addr, eth_addr, 6);
    tx.ip4_addr = ip4_addr;

    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)threads);
    tshard_t *sh = calloc((size_t)threads, sizeof(tshard_t));
    pthread_t *th = calloc((size_t)threads, sizeof(pthread_t));
    double *secs = calloc((size_t)threads * (size_t)reps, sizeof(double));
    for (int t = 0; t < threads; t++) {
        sh[t] = (tshard_t){&bar, cpus ? cpus[t] : -1, &rt, &tx, &arpt, &ndpt, frames, desc,
                           n * (size_t)t / (size_t)threads, n * (size_t)(t + 1) / (size_t)threads,
                           reps, secs + (size_t)t * (size_t)reps, 0};
        pthread_create(&th[t], NULL, shard_main, &sh[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);

    double *rate = calloc((size_t)reps, sizeof(double));
    for (int r = 0; r < reps; r++) {
        double mx = 0;
        for (int t = 0; t < threads; t++) mx = secs[t * reps + r] > mx ? secs[t * reps + r] : mx;
        rate[r] = mx > 0 ? (double)n / mx : 0;
    }
    for (int i = 1; i < reps; i++) /* insertion sort for the median */
        for (int j = i; j > 0 && rate[j - 1] > rate[j]; j--) {
            double x = rate[j]; rate[j] = rate[j - 1]; rate[j - 1] = x;
        }
    double med = rate[reps / 2];
    if (rates_out) memcpy(rates_out, rate, (size_t)reps * sizeof(double));
    free(rate); free(secs); free(th); free(sh);
    pthread_barrier_destroy(&bar);
    arp_table_destroy(&arpt);
    ndp_table_destroy(&ndpt);
    rule_table_destroy(&rt);
    return med;
}

/* ---- the RX thread's software RSS (reference src/rx_pcap.c:71-77) -------------------------- */
/* Per packet: the reference's own parse_flow_key() over a zero-filled pktbuf copy of the frame
 * and, when it succeeds, the reference's flow_hash() (src/parser.c:113-135); 0 when the parse
 * fails (the RX thread then falls back to round robin).  ok[i] = 1 where the parse succeeded. */
int upe_refh_flow_hash(const uint8_t *frames, const uint64_t *desc, size_t n, uint32_t *out,
                       uint8_t *ok) {
    static uint8_t buf[PKTBUF_DATA_SIZE];
    for (size_t i = 0; i < n; i++) {
        size_t off = (size_t)(desc[i] >> 16), len = (size_t)(desc[i] & 0xFFFF);
        if (len > PKTBUF_DATA_SIZE) return -1;
        memset(buf, 0, sizeof buf);
        memcpy(buf, frames + off, len);
        flow_key_t k;
        memset(&k, 0, sizeof k);
        const int rc = parse_flow_key(buf, len, &k);
        out[i] = rc == 0 ? flow_hash(&k) : 0u;
        if (ok) ok[i] = rc == 0;
    }
    return 0;
}
