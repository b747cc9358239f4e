/*
 * oracle/dropin_worker.c — the MI355X worker loop dropped into the REFERENCE pipeline
 * (INTEGRATION.md §1).
 *
 * TEST INFRASTRUCTURE ONLY.  Built by oracle/Makefile against the reference's own headers and
 * sources where they lie (ring, pktbuf pool, rule table, neighbour tables, worker.c), into
 * oracle/_ref/libupe_dropin.so (git-ignored), linked to this repo's libupe_gpu.so.
 *
 * The first part is the binding a maintainer adds to the reference (INTEGRATION.md §1 shows it):
 * the callbacks of upe_gpu_worker_run (include/upe_gpu.h, the product loop in
 * upe_amd/csrc/upe_worker.c) over a reference worker_t — ring_pop_burst on its rx_ring,
 * pktbuf_t data / len / pktbuf_free, tx_send / tx_send_batch on its tx, arp_update / ndp_update
 * on its tables, the SIGHUP rule swap picked up between bursts (src/main.c:258-265), and the
 * counters and rule_stats published into the worker_t fields the stats thread reads
 * (src/main.c:284-315).  gpu_worker_start() is the GPU counterpart of worker_start().
 *
 * The rest drives it: upe_dropin_run() feeds a stream through an RX-like producer -> reference
 * SPSC ring -> reference worker_t -> GPU loop, optionally with a rule reload in the middle,
 * for tests/test_gpu_dropin.py to compare with the reference worker; upe_dropin_bench() is the
 * reference's own throughput benchmark (tests/benchmark_throughput.c: synthetic NIC producer ->
 * rings -> workers -> stubbed TX, consumer Mpps = pkts_in / producer time) run with reference
 * worker threads or with GPU workers, for bench.py.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <execinfo.h>
#include <unistd.h>
#include <pthread.h>
#include <sched.h>
#include <signal.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "arp_table.h"
#include "ndp_table.h"
#include "pktbuf.h"
#include "ring.h"
#include "rule_table.h"
#include "tx.h"
#include "worker.h"

#include "../include/upe_gpu.h"

volatile sig_atomic_t g_stop = 0; /* defined by the program, reference src/main.c:27 */

/* ---- TX stubs (as reference tests/benchmark_throughput.c:30-42), with a call log ---------- */
/* The log (tests): per tx_send_batch call its size and each frame's pktbuf; tx_send frames. */
static pktbuf_t **g_log_frames, **g_log_replies;
static uint32_t *g_log_sizes;
static size_t g_log_nf, g_log_nb, g_log_nr, g_log_cap;

static pktbuf_t *buf_of(const uint8_t *data) {
    return (pktbuf_t *)(data - offsetof(pktbuf_t, data));
}
int tx_send(const tx_ctx_t *ctx, const uint8_t *frame, size_t len) {
    (void)ctx; (void)len;
    if (g_log_replies && g_log_nr < g_log_cap) g_log_replies[g_log_nr++] = buf_of(frame);
    return 0;
}
int tx_send_batch(const tx_ctx_t *ctx, const uint8_t *const *frames, const size_t *lens, int count) {
    (void)ctx; (void)lens;
    if (g_log_frames && g_log_nb < g_log_cap && g_log_nf + (size_t)count <= g_log_cap) {
        g_log_sizes[g_log_nb++] = (uint32_t)count;
        for (int i = 0; i < count; i++) g_log_frames[g_log_nf++] = buf_of(frames[i]);
    }
    return count;
}

/* =========================================================================================== */
/* The binding: upe_gpu_worker_run over a reference worker_t                                    */
/* =========================================================================================== */
typedef struct {
    worker_t *w;
    int device;
    const upe_worker_ops_t *ops;    /* NULL: g_ops */
    upe_worker_cfg_t cfg;
    const rule_table_t *rt_loaded;  /* the table the context holds */
    rule_stat_t *stats_loaded;      /* the rule_stats array that goes with it */
    uint64_t stats_every_ns;        /* rule_stats published at most this often (0: every batch) */
    uint64_t stats_last_ns;
    upe_counters_t counters;        /* the loop's, at the end */
    uint64_t consumed;              /* published: NS / NA consumed (no worker_t field) */
    /* the stats thread's precompiled image of the next table (upe_rules_compile) and the table
     * it belongs to, stored before the swap (round 6): the worker thread then only uploads it */
    const rule_table_t *image_rt;
    upe_rule_image_t *image;
    int rc;
} gpu_worker_t;

static uint64_t now_ns(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

#define GW(u) ((gpu_worker_t *)(u))
static unsigned op_pop(void *u, void **b, unsigned m) { return ring_pop_burst(GW(u)->w->rx_ring, b, m); }
static int op_stop(void *u) { (void)u; return g_stop != 0; }
static uint8_t *op_data(void *u, void *b) { (void)u; return ((pktbuf_t *)b)->data; }
static size_t op_len(void *u, void *b) { (void)u; return ((pktbuf_t *)b)->len; }
static void op_free(void *u, void *b) { pktbuf_free(GW(u)->w->pool, (pktbuf_t *)b); }
static void op_free_burst(void *u, void *const *b, unsigned n) {
    pktbuf_pool_t *pool = GW(u)->w->pool;
    for (unsigned i = 0; i < n; i++) pktbuf_free(pool, (pktbuf_t *)b[i]);
}
static int op_tx_send(void *u, const uint8_t *f, size_t len) { return tx_send(GW(u)->w->tx, f, len); }
static int op_tx_send_batch(void *u, const uint8_t *const *f, const size_t *lens, int count) {
    return tx_send_batch(GW(u)->w->tx, f, lens, count);
}
static void op_arp_update(void *u, uint32_t ip, const uint8_t mac[6]) { arp_update(GW(u)->w->arpt, ip, mac); }
static void op_ndp_update(void *u, const uint8_t ip[16], const uint8_t mac[6]) {
    ndp_update(GW(u)->w->ndpt, ip, mac);
}
static int op_load_neigh(void *u, upe_gpu_ctx_t *ctx) {
    worker_t *w = GW(u)->w;
    pthread_rwlock_rdlock(&w->arpt->lock);
    pthread_rwlock_rdlock(&w->ndpt->lock);
    int rc = upe_gpu_load_neigh(ctx, (const upe_arp_entry_t *)w->arpt->entries, w->arpt->capacity,
                                (const upe_ndp_entry_t *)w->ndpt->entries, w->ndpt->capacity);
    pthread_rwlock_unlock(&w->ndpt->lock);
    pthread_rwlock_unlock(&w->arpt->lock);
    return rc;
}
/* the stats thread swapped w->rt (and w->rule_stats) since the context's table was loaded */
static int op_poll(void *u) { return GW(u)->w->rt != GW(u)->rt_loaded; }
static int op_sync(void *u, upe_gpu_ctx_t *ctx) {
    /* the stats thread stored rule_stats before rt (src/main.c:261-263): with the new rt seen,
     * the new rule_stats is the one to publish into from now on */
    const rule_table_t *rt = __atomic_load_n(&GW(u)->w->rt, __ATOMIC_ACQUIRE);
    GW(u)->rt_loaded = rt;
    GW(u)->stats_loaded = __atomic_load_n(&GW(u)->w->rule_stats, __ATOMIC_ACQUIRE);
    /* old rule_stats are not handed back: the stats thread frees the old array.  The table's
     * image, when the stats thread compiled it before the swap (stored before rt: acquire) */
    if (__atomic_load_n(&GW(u)->image_rt, __ATOMIC_ACQUIRE) == rt && GW(u)->image)
        return upe_gpu_reload_image(ctx, GW(u)->image, NULL, 0);
    return upe_gpu_reload_rules(ctx, (const upe_rule_t *)rt->rules, rt->count, rt->capacity, NULL, 0);
}
static void op_publish(void *u, upe_gpu_ctx_t *ctx, const upe_counters_t *c) {
    gpu_worker_t *g = GW(u);
    worker_t *w = g->w;
    /* rule_stats into the array the stats thread reads — unless a swap has begun: the packets
     * just classified ran with the old table, and w->rule_stats may already be the new array
     * (swapped before rt, src/main.c:261-263), so both pointers must still be the loaded ones */
    /* (ctx NULL: a batch is still on the GPU and the context's statistics run ahead of these
     * counters — counters only; the loop publishes with the context at least every 32 batches) */
    const uint64_t t = now_ns();
    rule_stat_t *rs = __atomic_load_n(&w->rule_stats, __ATOMIC_ACQUIRE);
    if (ctx && rs == g->stats_loaded && __atomic_load_n(&w->rt, __ATOMIC_ACQUIRE) == g->rt_loaded &&
        t - g->stats_last_ns >= g->stats_every_ns) {
        g->stats_last_ns = t;
        (void)upe_gpu_get_stats(ctx, NULL, (upe_rule_stat_t *)rs, g->rt_loaded->capacity);
    }
    /* then the counters (release: a reader that sees them sees the rule_stats above) */
    __atomic_store_n(&w->pkts_in, c->pkts_in, __ATOMIC_RELEASE);
    __atomic_store_n(&w->pkts_parsed, c->pkts_parsed, __ATOMIC_RELEASE);
    __atomic_store_n(&w->pkts_matched, c->pkts_matched, __ATOMIC_RELEASE);
    __atomic_store_n(&w->pkts_forwarded, c->pkts_forwarded, __ATOMIC_RELEASE);
    __atomic_store_n(&g->consumed, c->pkts_consumed, __ATOMIC_RELEASE);
    __atomic_store_n(&w->pkts_dropped, c->pkts_dropped, __ATOMIC_RELEASE);
}

static const upe_worker_ops_t g_ops = {
    op_pop, op_stop, op_data, op_len, op_free, op_tx_send, op_tx_send_batch,
    op_arp_update, op_ndp_update, op_load_neigh, op_poll, op_sync, op_publish, op_free_burst,
};

/* The GPU worker thread: what worker_main is for a CPU worker. */
static void *gpu_worker_main(void *arg) {
    gpu_worker_t *g = arg;
    worker_t *w = g->w;
    g->rc = -1;
    if (w->core_id >= 0) {
        cpu_set_t one;
        CPU_ZERO(&one);
        CPU_SET(w->core_id, &one);
        (void)pthread_setaffinity_np(pthread_self(), sizeof one, &one);
    }
    upe_gpu_ctx_t *ctx = upe_gpu_open(g->device, w->rt->capacity);
    if (!ctx) {
        fprintf(stderr, "dropin: %s\n", upe_gpu_last_error());
        return NULL;
    }
    g->rt_loaded = w->rt;
    g->stats_loaded = w->rule_stats;
    if (upe_gpu_load_rules(ctx, (const upe_rule_t *)w->rt->rules, w->rt->count) != 0 ||
        op_load_neigh(g, ctx) != 0 || upe_gpu_set_port(ctx, w->tx->eth_addr, w->tx->ip4_addr) != 0 ||
        upe_gpu_worker_run(ctx, g->ops ? g->ops : &g_ops, g, &g->cfg, &g->counters) != 0) {
        fprintf(stderr, "dropin: %s\n", upe_gpu_last_error());
        upe_gpu_close(ctx);
        return NULL;
    }
    g->stats_every_ns = 0;
    op_publish(g, ctx, &g->counters); /* the final counters and rule_stats */
    upe_gpu_close(ctx);
    g->rc = 0;
    return NULL;
}

/* worker_start() for a GPU worker (reference src/worker.c:336-339). */
static int gpu_worker_start(gpu_worker_t *g, pthread_t *th) {
    return pthread_create(th, NULL, gpu_worker_main, g);
}

/* =========================================================================================== */
/* Tests: a stream through the reference pipeline with the GPU worker                           */
/* =========================================================================================== */
static int g_mapped = 0;
void upe_dropin_set_mapped(int mapped) { g_mapped = mapped; }

/* Burst sizes the worker popped (tests): wraps ring_pop_burst. */
static uint32_t *g_log_pops;
static size_t g_log_np;
static unsigned op_pop_logged(void *u, void **b, unsigned m) {
    unsigned k = op_pop(u, b, m);
    if (k && g_log_pops && g_log_np < g_log_cap) g_log_pops[g_log_np++] = k;
    return k;
}

/* Packet index of each buffer of a run: `all` holds the run's buffers in packet order (distinct
 * pool slots); built once per run, after the worker is done (a cache keyed on the array's address
 * could outlive it: the next run's malloc may hand back the same address with other buffers). */
typedef struct {
    size_t lo, span, *idx;
} buf_index_t;
static int buf_index_build(buf_index_t *x, pktbuf_t *const *all, size_t n) {
    size_t lo = (size_t)-1, hi = 0;
    for (size_t i = 0; i < n; i++) {
        const size_t a = (size_t)all[i];
        lo = a < lo ? a : lo;
        hi = a > hi ? a : hi;
    }
    x->lo = lo;
    x->span = n ? (hi - lo) / sizeof(pktbuf_t) + 1 : 0;
    x->idx = malloc((x->span ? x->span : 1) * sizeof(size_t));
    if (!x->idx) return -1;
    for (size_t i = 0; i < n; i++) x->idx[((size_t)all[i] - lo) / sizeof(pktbuf_t)] = i;
    return 0;
}
static size_t index_of(const buf_index_t *x, const pktbuf_t *b) {
    return x->idx[((size_t)b - x->lo) / sizeof(pktbuf_t)];
}

/*
 * Run `n` packets (batch layout of include/upe_gpu.h) through: an RX-like producer thread ->
 * reference SPSC ring -> reference worker_t driven by the GPU worker loop.  rules in insertion
 * order (rule_table_add), neighbour slot arrays copied into reference tables.  Outputs the
 * worker's counters (pkts_in, parsed, matched, forwarded, dropped), rule_stats[capacity], each
 * packet's bytes as the worker left them in its pktbuf (out_frames, the input's layout), the
 * final neighbour slot arrays (out_arp / out_ndp, the input capacities), and the TX / ring log
 * (optional, `log_cap` entries each): pops[] = burst sizes popped, sizes[] = tx_send_batch call
 * sizes, tx[] = packet index of each frame sent, replies[] = packet index of each tx_send;
 * log_n[4] = their lengths.
 * Reload (rules_b != NULL): after the first `at` packets have been processed, the driver does
 * what the stats thread does on SIGHUP (src/main.c:237-265: new table of capacity cap_b from
 * rules_b in insertion order, fresh calloc'd rule_stats, both swapped into the worker_t) and
 * pushes the rest; stats_a receives the old rule_stats array as it was at the swap, and
 * rule_stats the new one (cap_b entries).
 */
/* UPE_DROPIN_BACKTRACE=1: a fault inside the harness prints the native frames (addresses map to
 * the in-tree .so files with addr2line) before the process dies */
static void on_fault(int sig) {
    void *fr[48];
    const int k = backtrace(fr, 48);
    static const char msg[] = "upe_dropin: fatal signal, native frames:\n";
    (void)!write(2, msg, sizeof msg - 1);
    backtrace_symbols_fd(fr, k, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

int upe_dropin_run(const upe_rule_t *rules, size_t nrules, size_t capacity,
                   const upe_arp_entry_t *arp, size_t arp_cap, const upe_ndp_entry_t *ndp,
                   size_t ndp_cap, const uint8_t eth_addr[6], uint32_t ip4_addr,
                   const uint8_t *frames, const uint64_t *in_desc, size_t n, int device,
                   uint64_t counters[5], upe_rule_stat_t *rule_stats, uint8_t *out_frames,
                   upe_arp_entry_t *out_arp, upe_ndp_entry_t *out_ndp,
                   const upe_rule_t *rules_b, size_t nrules_b, size_t cap_b, size_t at,
                   upe_rule_stat_t *stats_a, size_t log_cap, uint32_t *pops, uint32_t *sizes,
                   uint32_t *tx, uint32_t *replies, uint64_t log_n[4]) {
    if (getenv("UPE_DROPIN_BACKTRACE")) {
        signal(SIGSEGV, on_fault);
        signal(SIGBUS, on_fault);
    }
    rule_table_t *rt = malloc(sizeof *rt);
    if (!rt || rule_table_init(rt, capacity) != 0) return -1;
    for (size_t i = 0; i < nrules; i++)
        if (rule_table_add(rt, (const rule_t *)&rules[i]) != 0) return -1;
    arp_table_t arpt;
    ndp_table_t ndpt;
    if (arp_table_init(&arpt, arp_cap ? arp_cap : 1) != 0 ||
        ndp_table_init(&ndpt, ndp_cap ? ndp_cap : 1) != 0)
        return -1;
    if (arp_cap) memcpy(arpt.entries, arp, arp_cap * sizeof(arp_entry_t));
    if (ndp_cap) memcpy(ndpt.entries, ndp, ndp_cap * sizeof(ndp_entry_t));
    tx_ctx_t txc;
    memset(&txc, 0, sizeof txc);
    memcpy(txc.eth_addr, eth_addr, 6);
    txc.ip4_addr = ip4_addr;
    /* One pool per process (the pool's thread-local caches remember it), sized so that every
     * packet of the run gets its own buffer: the producer allocates all of them before the
     * worker frees any, so the test does not lean on concurrent alloc/free in the pool. */
    static pktbuf_pool_t pool;
    static size_t pool_cap;
    /* (slack: every finished worker thread takes up to LOCAL_CACHE_SIZE buffers with it in its
     * thread-local cache, reference src/pktbuf.c:10) */
    if (pool_cap < n + 256) {
        if (pool_cap) return -1; /* one size per process: room for the largest test stream */
        const size_t want = n + 8192 > ((size_t)1 << 19) ? n + 8192 : (size_t)1 << 19;
        if (pktbuf_pool_init(&pool, want) != 0) return -1;
        pool_cap = want;
    }
    /* mapped mode: the pool's buffers page-locked and mapped for the GPU once */
    static int pool_registered;
    if (g_mapped && !pool_registered) {
        if (upe_gpu_host_register(pool.buffers, pool.capacity * sizeof(pktbuf_t)) != 0) return -1;
        pool_registered = 1;
    }
    pktbuf_t **all = malloc((n ? n : 1) * sizeof(*all));
    if (!all) return -1;
    for (size_t i = 0; i < n; i++) {
        pktbuf_t *b = pktbuf_alloc(&pool);
        if (!b) return -1;
        size_t off = (size_t)(in_desc[i] >> 16), len = (size_t)(in_desc[i] & 0xFFFF);
        memset(b->data, 0, 128);
        memcpy(b->data, frames + off, len);
        b->len = len;
        b->timestamp = 0;
        all[i] = b;
    }
    spsc_ring_t ring;
    if (ring_init(&ring, 1024) != 0) return -1;
    worker_t *w = calloc(1, sizeof(worker_t)); /* src/main.c:444 */
    if (!w || worker_init(w, 0, -1, &ring, &pool, rt, &txc, &arpt, &ndpt) != 0) return -1;

    /* the TX / ring log */
    g_log_cap = log_cap;
    g_log_nb = g_log_nf = g_log_nr = g_log_np = 0;
    pktbuf_t **lf = log_cap ? malloc(log_cap * sizeof(*lf)) : NULL;
    pktbuf_t **lr = log_cap ? malloc(log_cap * sizeof(*lr)) : NULL;
    g_log_frames = lf;
    g_log_replies = lr;
    g_log_sizes = log_cap ? sizes : NULL;
    g_log_pops = log_cap ? pops : NULL;

    g_stop = 0;
    gpu_worker_t g;
    memset(&g, 0, sizeof g);
    g.w = w;
    g.device = device;
    g.cfg.pool_base = g_mapped ? (uint8_t *)pool.buffers : NULL;
    g.cfg.pool_bytes = g_mapped ? pool.capacity * sizeof(pktbuf_t) : 0;
    g.cfg.batch = 65536;
    /* (rule_stats published whenever nothing is in flight: at the drain the ring empties into
     * before the reload below, so the array swapped out holds exactly the counts up to the swap) */
    static upe_worker_ops_t ops;
    ops = g_ops;
    ops.pop_burst = op_pop_logged;
    g.ops = &ops;
    pthread_t th;
    if (gpu_worker_start(&g, &th) != 0) return -1;
    /* producer: the RX thread's staged bursts of 32 into the ring, src/rx_pcap.c:80-92 */
    rule_stat_t *old_stats = NULL;
    rule_table_t *rt_b = NULL;
    const size_t first = rules_b && at < n ? at : n;
    for (size_t i = 0; i < first; i += 32) {
        unsigned ns = (unsigned)(first - i < 32 ? first - i : 32), done = 0;
        while (done < ns) done += ring_push_burst(&ring, (void **)(all + i) + done, ns - done);
    }
    if (rules_b) {
        /* wait until the first part is processed: every packet forwarded, dropped or consumed
         * (the counters the loop publishes after each batch) */
        for (;;) {
            const uint64_t done = __atomic_load_n(&w->pkts_dropped, __ATOMIC_ACQUIRE) +
                                  __atomic_load_n(&w->pkts_forwarded, __ATOMIC_ACQUIRE) +
                                  __atomic_load_n(&g.consumed, __ATOMIC_ACQUIRE);
            if (done >= first) break;
            struct timespec ts = {0, 100000};
            nanosleep(&ts, NULL);
        }
        /* the stats thread's reload, src/main.c:222-265 */
        rt_b = malloc(sizeof *rt_b);
        if (!rt_b || rule_table_init(rt_b, cap_b) != 0) return -1;
        for (size_t i = 0; i < nrules_b; i++)
            if (rule_table_add(rt_b, (const rule_t *)&rules_b[i]) != 0) return -1;
        rule_stat_t *new_stats = calloc(rt_b->capacity, sizeof(rule_stat_t));
        if (!new_stats) return -1;
        /* the GPU worker's image of the new table, built here on the stats thread while the
         * worker keeps forwarding (NULL: the worker compiles it at the swap instead) */
        g.image = upe_rules_compile((const upe_rule_t *)rt_b->rules, rt_b->count, rt_b->capacity);
        __atomic_store_n(&g.image_rt, rt_b, __ATOMIC_RELEASE);
        old_stats = w->rule_stats;
        memcpy(stats_a, old_stats, capacity * sizeof(rule_stat_t));
        __atomic_store_n(&w->rule_stats, new_stats, __ATOMIC_RELEASE);
        __atomic_store_n(&w->rt, rt_b, __ATOMIC_RELEASE);
        for (size_t i = first; i < n; i += 32) {
            unsigned ns = (unsigned)(n - i < 32 ? n - i : 32), done = 0;
            while (done < ns) done += ring_push_burst(&ring, (void **)(all + i) + done, ns - done);
        }
    }
    g_stop = 1;
    pthread_join(th, NULL);
    upe_rules_image_free(g.image);
    counters[0] = w->pkts_in;
    counters[1] = w->pkts_parsed;
    counters[2] = w->pkts_matched;
    counters[3] = w->pkts_forwarded;
    counters[4] = w->pkts_dropped;
    if (rule_stats) memcpy(rule_stats, w->rule_stats, w->rt->capacity * sizeof(rule_stat_t));
    if (out_frames)
        for (size_t i = 0; i < n; i++)
            memcpy(out_frames + (size_t)(in_desc[i] >> 16), all[i]->data, (size_t)(in_desc[i] & 0xFFFF));
    if (out_arp && arp_cap) memcpy(out_arp, arpt.entries, arp_cap * sizeof(arp_entry_t));
    if (out_ndp && ndp_cap) memcpy(out_ndp, ndpt.entries, ndp_cap * sizeof(ndp_entry_t));
    if (log_cap) {
        buf_index_t bx;
        if (buf_index_build(&bx, all, n) != 0) return -1;
        for (size_t k = 0; k < g_log_nf; k++) tx[k] = (uint32_t)index_of(&bx, lf[k]);
        for (size_t k = 0; k < g_log_nr; k++) replies[k] = (uint32_t)index_of(&bx, lr[k]);
        free(bx.idx);
        log_n[0] = g_log_np;
        log_n[1] = g_log_nb;
        log_n[2] = g_log_nf;
        log_n[3] = g_log_nr;
    }
    g_log_frames = g_log_replies = NULL;
    g_log_sizes = g_log_pops = NULL;
    free(lf);
    free(lr);
    worker_destroy(w);
    free(w);
    free(old_stats);
    free(all);
    ring_destroy(&ring);
    arp_table_destroy(&arpt);
    ndp_table_destroy(&ndpt);
    rule_table_destroy(rt);
    free(rt);
    if (rt_b) {
        rule_table_destroy(rt_b);
        free(rt_b);
    }
    return g.rc;
}

/* =========================================================================================== */
/* The reference's throughput benchmark with CPU or GPU workers                                 */
/* =========================================================================================== */
/* The reference benchmark's own packet builder and producer (tests/benchmark_throughput.c:
 * 138-238: build_dummy_packet, run_producer), included where they lie; its g_stop, TX stubs and
 * main are renamed out of the way (this file defines the program's g_stop and logging stubs). */
#define g_stop upe_refbench_g_stop
#define tx_send upe_refbench_tx_send
#define tx_send_batch upe_refbench_tx_send_batch
#define main upe_refbench_main
#include "benchmark_throughput.c"
#undef g_stop
#undef tx_send
#undef tx_send_batch
#undef main

/*
 * The reference benchmark's setup (tests/benchmark_throughput.c:87-116: one TCP FWD rule, one ARP
 * entry for 10.128.0.2, tx MAC ..:bb) with `workers` workers: gpu = 0 the reference's own
 * worker threads (worker_start -> src/worker.c worker_main), gpu = 1 GPU workers (one context
 * each on `device`, gpu_worker_start -> upe_gpu_worker_run; mapped = 1 classifies the pool's
 * pktbufs where they lie, else header windows through the DMA round trip).  The calling thread
 * is the producer, pinned to cpus[0]; worker t is pinned to cpus[1 + t] (cpus may be NULL).
 * warmup then `seconds` of measurement.  out[0] = consumer Mpps (pkts_in delta over the
 * producer's time, as output_json reports it), out[1] = producer Mpps, out[2] = ring-full
 * events, out[3] = seconds, out[4] = packets consumed.  0 / -1.
 */
int upe_dropin_bench(int gpu, int mapped, int workers, int device, size_t pool_cap,
                     size_t ring_size, int batch, int packet_size, double warmup, double seconds,
                     size_t gpu_batch, const int *cpus, double out[5]) {
    if (workers < 1 || workers > 16 || batch < 1 || batch > 256) return -1;
    if (cpus) {
        cpu_set_t one;
        CPU_ZERO(&one);
        CPU_SET(cpus[0], &one);
        (void)pthread_setaffinity_np(pthread_self(), sizeof one, &one);
    }
    /* one pool per capacity, kept for the process's life: a thread's pktbuf cache remembers
     * its pool (src/pktbuf.c:298-303) and flushes into it when the thread switches pools */
    static pktbuf_pool_t pools[4];
    static size_t caps[4];
    static int registered[4];
    int pi = 0;
    while (pi < 4 && caps[pi] && caps[pi] != pool_cap) pi++;
    if (pi == 4) return -1;
    if (!caps[pi]) {
        if (pktbuf_pool_init(&pools[pi], pool_cap) != 0) return -1;
        caps[pi] = pool_cap;
    }
    pktbuf_pool_t *const poolp = &pools[pi];
#define pool (*poolp)
    if (gpu && mapped && !registered[pi]) {
        if (upe_gpu_host_register(pool.buffers, pool.capacity * sizeof(pktbuf_t)) != 0) return -1;
        registered[pi] = 1;
    }
    spsc_ring_t *rings = calloc((size_t)workers, sizeof(spsc_ring_t));
    for (int i = 0; i < workers; i++)
        if (ring_init(&rings[i], ring_size) != 0) return -1;
    rule_table_t rt;
    rule_table_init(&rt, 1024);
    rule_t r = {.priority = 10, .protocol = 6, .action = {.type = ACT_FWD, .out_ifindex = 1}};
    rule_table_add(&rt, &r);
    arp_table_t arpt;
    ndp_table_t ndpt;
    arp_table_init(&arpt, 1024);
    const uint32_t dst_ip = (10U << 24) | (128U << 16) | (0U << 8) | 2U;
    const uint8_t dst_mac[6] = {0xaa, 0x00, 0x00, 0x00, 0x00, 0xbb};
    arp_update(&arpt, dst_ip, dst_mac);
    ndp_table_init(&ndpt, 1024);
    tx_ctx_t txc;
    memset(&txc, 0, sizeof txc);
    txc.eth_addr[5] = 0xbb;
    worker_t *ws = calloc((size_t)workers, sizeof(worker_t));
    gpu_worker_t *gs = calloc((size_t)workers, sizeof(gpu_worker_t));
    pthread_t *th = calloc((size_t)workers, sizeof(pthread_t));
    g_stop = 0;
    for (int i = 0; i < workers; i++) {
        worker_init(&ws[i], i, cpus ? cpus[1 + i] : -1, &rings[i], &pool, &rt, &txc, &arpt, &ndpt);
        if (gpu) {
            gs[i].w = &ws[i];
            gs[i].device = device;
            gs[i].cfg.pool_base = mapped ? (uint8_t *)pool.buffers : NULL;
            gs[i].cfg.pool_bytes = mapped ? pool.capacity * sizeof(pktbuf_t) : 0;
            /* a batch the pool can fill: two batches in flight per GPU worker plus the ring's
             * share stay under the pool (else every batch ends at an empty ring) */
            {
                size_t cap = pool.capacity / (4u * (unsigned)workers);
                if (cap < 256) cap = 256;
                gs[i].cfg.batch = gpu_batch < cap ? gpu_batch : cap;
            }
            gs[i].stats_every_ns = 100000000ull; /* rule_stats for the stats thread: 10 Hz */
            if (gpu_worker_start(&gs[i], &th[i]) != 0) return -1;
        } else if (worker_start(&ws[i]) != 0) {
            return -1;
        }
    }
    bench_config_t bcfg = default_config();
    bcfg.num_workers = workers;
    bcfg.batch_size = batch;
    bcfg.packet_size = packet_size;
    if (warmup > 0) (void)run_producer(&bcfg, &pool, rings, warmup);
    uint64_t before[16];
    for (int i = 0; i < workers; i++) before[i] = __atomic_load_n(&ws[i].pkts_in, __ATOMIC_ACQUIRE);
    const producer_result_t pr = run_producer(&bcfg, &pool, rings, seconds);
    const uint64_t pushed = pr.packets_pushed, full = pr.ring_full_events;
    const double dur = pr.duration_sec;
    uint64_t consumed = 0;
    for (int i = 0; i < workers; i++)
        consumed += __atomic_load_n(&ws[i].pkts_in, __ATOMIC_ACQUIRE) - before[i];
    g_stop = 1;
    int rc = 0;
    for (int i = 0; i < workers; i++) {
        if (gpu) {
            pthread_join(th[i], NULL);
            rc |= gs[i].rc;
        } else {
            worker_join(&ws[i]);
        }
    }
    out[0] = (double)consumed / dur / 1e6;
    out[1] = (double)pushed / dur / 1e6;
    out[2] = (double)full;
    out[3] = dur;
    out[4] = (double)consumed;
    for (int i = 0; i < workers; i++) worker_destroy(&ws[i]);
    for (int i = 0; i < workers; i++) ring_destroy(&rings[i]);
    free(ws);
    free(gs);
    free(th);
    free(rings);
    rule_table_destroy(&rt);
    arp_table_destroy(&arpt);
    ndp_table_destroy(&ndpt);
    return rc;
#undef pool
}
