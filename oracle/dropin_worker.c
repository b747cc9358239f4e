/*
 * oracle/dropin_worker.c — the MI355X path dropped into the REFERENCE pipeline.
 *
 * TEST INFRASTRUCTURE ONLY.  Built by oracle/Makefile against the reference's own headers and
 * sources where they lie (ring, pktbuf pool, rule table, neighbour tables, worker_init), into
 * oracle/_ref/libupe_dropin.so (git-ignored), linked to this repo's libupe_gpu.so.
 *
 * What it shows: a reference worker_t, fed through the reference SPSC ring by an RX-like
 * producer thread exactly as src/rx_pcap.c feeds it (pktbuf_alloc, memcpy, ring_push_burst),
 * runs a GPU-backed worker loop instead of src/worker.c:255-307 — ring_pop_burst bursts
 * aggregated into a pinned batch of header windows, one upe_gpu_process_host() per batch (or, in
 * mapped mode, upe_dropin_set_mapped(1): the pool registered once with upe_gpu_host_register and
 * each batch's pktbufs classified where they lie by upe_gpu_process_mapped, nothing copied) (cut
 * after every packet that writes a neighbour table, whose write is then applied with the
 * reference's own arp_update / ndp_update and the snapshot re-uploaded), then the reference's TX
 * accounting (tx_send_batch, pkts_forwarded / pkts_dropped, pktbuf_free, tx_send of ARP
 * replies) — and ends with the same counters and rule_stats in the same worker_t fields the
 * reference's stats thread reads (src/main.c:293-315).  tests/test_gpu_dropin.py compares
 * them, every packet's bytes and the final neighbour tables with the reference worker itself
 * (oracle/_ref/libupe_ref.so) on the same packets, control packets included.
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <pthread.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "arp_table.h"
#include "ndp_table.h"
#include "pktbuf.h"
#include "ring.h"
#include "rule_table.h"
#include "tx.h"
#include "worker.h"

#include "../include/upe_gpu.h"

volatile sig_atomic_t g_stop = 0; /* defined by the program, reference src/main.c:27 */

/* TX stubs, as reference tests/benchmark_throughput.c:30-42 */
int tx_send(const tx_ctx_t *ctx, const uint8_t *frame, size_t len) {
    (void)ctx; (void)frame; (void)len;
    return 0;
}
int tx_send_batch(const tx_ctx_t *ctx, const uint8_t *const *frames, const size_t *lens, int count) {
    (void)ctx; (void)frames; (void)lens;
    return count;
}

#define GPU_BATCH 65536u
#define WIN UPE_HDR_WINDOW

typedef struct {
    worker_t *w;
    int device;
    int rc;
    uint8_t *pool_base; /* mapped mode: the registered pktbuf array (frames classified in place) */
} gpu_arg_t;

/* 0: header windows through upe_gpu_process_host (copies); 1: the pktbufs classified where they
 * lie in the registered pool (upe_gpu_process_mapped, nothing copied). */
static int g_mapped = 0;
void upe_dropin_set_mapped(int mapped) { g_mapped = mapped; }

/* The TX flush of the reference worker loop, src/worker.c:286-303. */
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

/* Byte k of a frame as a zero-filled pktbuf holds it (the reference reads the ethertype and the
 * ARP header without a length check, src/worker.c:24-35). */
static uint8_t at(const pktbuf_t *b, size_t k) { return k < b->len ? b->data[k] : 0; }

/* A packet handle_control_packet may write a neighbour table for (src/worker.c:28-39, 57-100):
 * ARP with the Ethernet/IPv4 header shape, or an IPv6 NS/NA of at least 78 bytes.  The batch is
 * cut after it, so every later packet sees the table write, as in the reference's burst loop. */
static int is_table_write(const pktbuf_t *b) {
    const unsigned et = (unsigned)at(b, 12) << 8 | at(b, 13);
    if (et == 0x0806)
        return at(b, 14) == 0 && at(b, 15) == 1 && at(b, 16) == 8 && at(b, 17) == 0 &&
               at(b, 18) == 6 && at(b, 19) == 4;
    return et == 0x86DD && b->len >= 78 && at(b, 20) == 58 && (at(b, 54) == 135 || at(b, 54) == 136);
}

/* handle_control_packet's table writes and ARP reply (src/worker.c:30-52, 64-95) for a packet the
 * GPU classified: v is its verdict, b->data the frame as the GPU left it (an answered ARP request
 * already rewritten into the reply, whose tha / tpa now hold the request's sha / spa). */
static void control_writes(worker_t *w, pktbuf_t *b, uint32_t v) {
    const uint8_t *d = b->data;
    if (v & UPE_VF_ARP_LEARN) {
        const int replied = (v & UPE_VF_ARP_REPLY) != 0;
        uint32_t spa_be;
        memcpy(&spa_be, d + (replied ? 38 : 28), 4);
        arp_update(w->arpt, ntohl(spa_be), d + (replied ? 32 : 22));
        if (replied) tx_send(w->tx, b->data, b->len);
    } else if (UPE_VERDICT_CODE(v) == UPE_V_CONSUMED) {
        const int ns = d[54] == 135;
        for (size_t off = 78; off + 2 <= b->len;) {
            const uint8_t type = d[off];
            const size_t olen = (uint8_t)(d[off + 1] * 8); /* uint8_t, src/worker.c:73 */
            if (olen == 0 || off + olen > b->len) break;
            if (olen >= 8 && ((ns && type == 1) || (!ns && type == 2))) {
                ndp_update(w->ndpt, ns ? d + 22 : d + 62, d + off + 2);
                break;
            }
            off += olen;
        }
    }
}

static int load_tables(upe_gpu_ctx_t *ctx, worker_t *w) {
    pthread_rwlock_rdlock(&w->arpt->lock);
    pthread_rwlock_rdlock(&w->ndpt->lock);
    int rc = upe_gpu_load_neigh(ctx, (const upe_arp_entry_t *)w->arpt->entries, w->arpt->capacity,
                                (const upe_ndp_entry_t *)w->ndpt->entries, w->ndpt->capacity);
    pthread_rwlock_unlock(&w->ndpt->lock);
    pthread_rwlock_unlock(&w->arpt->lock);
    return rc;
}

typedef struct {
    upe_gpu_ctx_t *ctx;
    uint8_t *win;
    uint64_t *desc;
    uint32_t *verdict;
    pktbuf_t **bufs;
    size_t n;
    uint8_t *pool_base; /* mapped mode */
} gpu_batch_t;

/* One GPU batch through the host round trip, then the reference's per-verdict handling
 * (src/worker.c:146-153 drops, :240-243 TX queue, :96-98 consumed) and, when the batch ends with
 * a table-writing control packet, that packet's writes and the new table snapshot. */
static int run_batch(worker_t *w, gpu_batch_t *g, int cut) {
    if (g->n == 0) return 0;
    if (g->pool_base) {
        /* the frames rewritten in place in the pool, where tx_send reads them */
        if (upe_gpu_process_mapped(g->ctx, g->pool_base, g->desc, g->verdict, g->n, NULL) != 0 ||
            upe_gpu_sync(g->ctx, NULL) != 0) {
            fprintf(stderr, "dropin: %s\n", upe_gpu_last_error());
            return -1;
        }
    } else if (upe_gpu_process_host(g->ctx, g->win, g->n * WIN + UPE_FRAME_TAIL, g->desc,
                                    g->verdict, g->n, 0) != 0) {
        fprintf(stderr, "dropin: %s\n", upe_gpu_last_error());
        return -1;
    }
    for (size_t i = 0; i < g->n; i++) {
        pktbuf_t *b = g->bufs[i];
        const uint32_t v = g->verdict[i];
        if (!g->pool_base)
            memcpy(b->data, g->win + i * WIN, b->len < UPE_REWRITE_EXTENT ? b->len : UPE_REWRITE_EXTENT);
        if (cut && i + 1 == g->n) control_writes(w, b, v);
        if (UPE_VERDICT_CODE(v) == UPE_V_FWD) {
            w->tx_frames[w->tx_count] = b->data; /* worker.c:240-243 */
            w->tx_lens[w->tx_count] = b->len;
            w->tx_bufs[w->tx_count++] = b;
            if (w->tx_count == WORKER_BURST_SIZE) flush_tx(w);
        } else if (UPE_VERDICT_CODE(v) == UPE_V_CONSUMED) {
            pktbuf_free(w->pool, b); /* consumed control packet: no counter */
        } else {
            w->pkts_dropped++; /* every drop path of process_packet counts one */
            pktbuf_free(w->pool, b);
        }
    }
    flush_tx(w);
    g->n = 0;
    return cut ? load_tables(g->ctx, w) : 0;
}

/* GPU-backed replacement of worker_main (reference src/worker.c:255-307). */
static void *gpu_worker_main(void *arg) {
    gpu_arg_t *ga = arg;
    worker_t *w = ga->w;
    ga->rc = -1;
    gpu_batch_t g;
    memset(&g, 0, sizeof g);
    g.ctx = upe_gpu_open(ga->device, w->rt->capacity);
    g.win = upe_gpu_host_alloc((size_t)GPU_BATCH * WIN + UPE_FRAME_TAIL);
    g.desc = upe_gpu_host_alloc(GPU_BATCH * sizeof(uint64_t));
    g.verdict = upe_gpu_host_alloc(GPU_BATCH * sizeof(uint32_t));
    g.bufs = malloc(GPU_BATCH * sizeof(*g.bufs));
    g.pool_base = ga->pool_base;
    if (!g.ctx || !g.win || !g.desc || !g.verdict || !g.bufs) return NULL;
    if (upe_gpu_load_rules(g.ctx, (const upe_rule_t *)w->rt->rules, w->rt->count) != 0 ||
        load_tables(g.ctx, w) != 0 || upe_gpu_set_port(g.ctx, w->tx->eth_addr, w->tx->ip4_addr) != 0)
        return NULL;
    void *burst[WORKER_BURST_SIZE];
    for (;;) {
        unsigned k = ring_pop_burst(w->rx_ring, burst, WORKER_BURST_SIZE); /* worker.c:268 */
        w->pkts_in += k;                                                   /* worker.c:280 */
        for (unsigned j = 0; j < k; j++) {
            pktbuf_t *b = burst[j];
            if (g.pool_base) {
                /* the pktbuf's data where it lies: offset into the registered pool */
                g.desc[g.n] = UPE_DESC((uint64_t)(b->data - g.pool_base), b->len);
            } else {
                size_t c = b->len < WIN ? b->len : WIN;
                memcpy(g.win + g.n * WIN, b->data, c);
                memset(g.win + g.n * WIN + c, 0, WIN - c);
                g.desc[g.n] = UPE_DESC((uint64_t)g.n * WIN, b->len);
            }
            g.bufs[g.n++] = b;
            const int cut = is_table_write(b);
            if ((cut || g.n == GPU_BATCH) && run_batch(w, &g, cut) != 0) return NULL;
        }
        const int stop = k == 0 && g_stop;
        if (k == 0 && g.n > 0 && run_batch(w, &g, 0) != 0) return NULL;
        if (stop) break;
    }
    /* the counters the GPU keeps, into the reference's own worker_t fields */
    upe_counters_t c;
    if (upe_gpu_get_stats(g.ctx, &c, (upe_rule_stat_t *)w->rule_stats, w->rt->capacity) != 0)
        return NULL;
    w->pkts_parsed = c.pkts_parsed;
    w->pkts_matched = c.pkts_matched;
    upe_gpu_host_free(g.win);
    upe_gpu_host_free(g.desc);
    upe_gpu_host_free(g.verdict);
    free(g.bufs);
    upe_gpu_close(g.ctx);
    ga->rc = 0;
    return NULL;
}

/*
 * Run `n` packets (batch layout of include/upe_gpu.h) through: an RX-like producer thread ->
 * reference SPSC ring -> reference worker_t driven by gpu_worker_main.  rules in insertion order
 * (rule_table_add), neighbour slot arrays copied into reference tables.  Outputs the worker's
 * counters (pkts_in, parsed, matched, forwarded, dropped), rule_stats[capacity], each packet's
 * bytes as the worker left them in its pktbuf (out_frames, the input's layout) and the final
 * neighbour slot arrays (out_arp / out_ndp, the input capacities).
 */
int upe_dropin_run(const upe_rule_t *rules, size_t nrules, size_t capacity,
                   const upe_arp_entry_t *arp, size_t arp_cap, const upe_ndp_entry_t *ndp,
                   size_t ndp_cap, const uint8_t eth_addr[6], uint32_t ip4_addr,
                   const uint8_t *frames, const uint64_t *in_desc, size_t n, int device,
                   uint64_t counters[5], upe_rule_stat_t *rule_stats, uint8_t *out_frames,
                   upe_arp_entry_t *out_arp, upe_ndp_entry_t *out_ndp) {
    rule_table_t rt;
    if (rule_table_init(&rt, capacity) != 0) return -1;
    for (size_t i = 0; i < nrules; i++)
        if (rule_table_add(&rt, (const rule_t *)&rules[i]) != 0) return -1;
    arp_table_t arpt;
    ndp_table_t ndpt;
    if (arp_table_init(&arpt, arp_cap ? arp_cap : 1) != 0 ||
        ndp_table_init(&ndpt, ndp_cap ? ndp_cap : 1) != 0)
        return -1;
    if (arp_cap) memcpy(arpt.entries, arp, arp_cap * sizeof(arp_entry_t));
    if (ndp_cap) memcpy(ndpt.entries, ndp, ndp_cap * sizeof(ndp_entry_t));
    tx_ctx_t tx;
    memset(&tx, 0, sizeof tx);
    memcpy(tx.eth_addr, eth_addr, 6);
    tx.ip4_addr = ip4_addr;
    /* One pool per process (the pool's thread-local caches remember it), sized so that every
     * packet of the run gets its own buffer: the producer allocates all of them before the
     * worker frees any, so the test does not lean on concurrent alloc/free in the pool. */
    static pktbuf_pool_t pool;
    static size_t pool_cap;
    /* (slack: every finished worker thread takes up to LOCAL_CACHE_SIZE buffers with it in its
     * thread-local cache, reference src/pktbuf.c:10) */
    if (pool_cap < n + 256) {
        if (pool_cap) return -1; /* one size per process */
        if (pktbuf_pool_init(&pool, n + 8192) != 0) return -1;
        pool_cap = n + 8192;
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
    if (!w || worker_init(w, 0, -1, &ring, &pool, &rt, &tx, &arpt, &ndpt) != 0) return -1;

    g_stop = 0;
    gpu_arg_t ga = {w, device, -1, g_mapped ? (uint8_t *)pool.buffers : NULL};
    pthread_t th;
    pthread_create(&th, NULL, gpu_worker_main, &ga);
    /* producer: the RX thread's staged bursts of 32 into the ring, src/rx_pcap.c:80-92 */
    for (size_t i = 0; i < n; i += 32) {
        unsigned ns = (unsigned)(n - i < 32 ? n - i : 32), done = 0;
        while (done < ns) done += ring_push_burst(&ring, (void **)(all + i) + done, ns - done);
    }
    g_stop = 1;
    pthread_join(th, NULL);
    counters[0] = w->pkts_in;
    counters[1] = w->pkts_parsed;
    counters[2] = w->pkts_matched;
    counters[3] = w->pkts_forwarded;
    counters[4] = w->pkts_dropped;
    if (rule_stats) memcpy(rule_stats, w->rule_stats, capacity * sizeof(rule_stat_t));
    if (out_frames)
        for (size_t i = 0; i < n; i++)
            memcpy(out_frames + (size_t)(in_desc[i] >> 16), all[i]->data, (size_t)(in_desc[i] & 0xFFFF));
    if (out_arp && arp_cap) memcpy(out_arp, arpt.entries, arp_cap * sizeof(arp_entry_t));
    if (out_ndp && ndp_cap) memcpy(out_ndp, ndpt.entries, ndp_cap * sizeof(ndp_entry_t));
    worker_destroy(w);
    free(w);
    free(all);
    ring_destroy(&ring);
    arp_table_destroy(&arpt);
    ndp_table_destroy(&ndpt);
    rule_table_destroy(&rt);
    return ga.rc;
}
