/*
 * upe_worker.c — the GPU-backed worker loop (include/upe_gpu.h upe_gpu_worker_run), host C above
 * the C ABI.
 *
 * It replaces reference worker_main (src/worker.c:255-307) for a worker whose packets are
 * classified by the MI355X path: the same ring pops, the same per-burst TX flush, the same
 * counters, with process_packet (src/worker.c:106-253) run by the GPU over batches gathered from
 * many bursts.  What it must preserve of the reference's sequential loop:
 *
 *  - the order of table writes: handle_control_packet (src/worker.c:23-104) writes the ARP / NDP
 *    table in the middle of a burst and every later packet sees the write, so a batch is cut
 *    right after each packet that can write a table, the write is applied through the caller's
 *    arp_update / ndp_update and the snapshot re-uploaded before the next packet is classified
 *    (the one-entry L1 caches carry across batches inside the context);
 *  - the external calls per burst and their order: tx_send of an answered ARP request while the
 *    burst is processed (src/worker.c:40-52), then one tx_send_batch of the burst's forwarded
 *    frames (src/worker.c:287-303), forwarded += sent, dropped += count - sent, every TX buffer
 *    freed whether sent or not;
 *  - the counters the stats thread reads (src/main.c:284-315): pkts_in per pop
 *    (src/worker.c:280), parsed / matched / dropped per packet (src/worker.c:119-153), the TX
 *    accounting above.
 *
 * Two ways to get a batch to the GPU (cfg->pool_base): copy each frame's header window into
 * pinned staging and run the DMA round trip in emit mode (the 16-byte records are then applied to
 * the caller's buffers, upe_hdr_apply), or leave the frames where they are in a registered pool and
 * let the kernel classify and rewrite them there (upe_gpu_process_mapped).
 */
#define _GNU_SOURCE
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/upe_gpu.h"

/* upe_gpu.hip: sets the calling thread's upe_gpu_last_error() message (not part of the ABI) */
int upe_gpu_set_last_error(const char *msg);

#define WIN UPE_HDR_WINDOW

typedef struct {
    upe_gpu_ctx_t *ctx;
    const upe_worker_ops_t *ops;
    void *user;
    size_t cap;        /* packets per batch */
    unsigned burst;
    uint8_t *pool;     /* mapped mode: registered region the frames lie in */
    size_t pool_bytes;
    /* the batch being gathered: handles in arrival order, and the pinned arrays the GPU reads */
    void **bufs;
    size_t n;
    uint64_t *desc;
    uint32_t *verdict;
    uint8_t *win;          /* window mode: cap header windows + UPE_FRAME_TAIL */
    upe_hdr_rec_t *rec;    /* window mode: records */
    /* sizes of the bursts popped and not yet flushed, oldest first (a ring) */
    unsigned *bq;
    size_t bq_cap, bq_head, bq_len;
    unsigned left;     /* packets of the oldest burst still to be walked */
    /* the TX queue of the burst being walked (worker_t tx_frames / tx_lens / tx_bufs) */
    const uint8_t *tx_frames[UPE_TX_BATCH_MAX];
    size_t tx_lens[UPE_TX_BATCH_MAX];
    void *tx_bufs[UPE_TX_BATCH_MAX];
    int tx_count;
    upe_counters_t c;
} loop_t;

static uint8_t at(const uint8_t *d, size_t len, size_t k) { return k < len ? d[k] : 0; }

/* A packet handle_control_packet may write a neighbour table for (src/worker.c:28-39, 57-100):
 * ARP with the Ethernet/IPv4 header shape (its learn does not look at len), or an IPv6 NS/NA of
 * at least 78 bytes.  Bytes at or past len read as zero (a zero-filled pktbuf). */
static int is_table_write(const uint8_t *d, size_t len) {
    const unsigned et = (unsigned)at(d, len, 12) << 8 | at(d, len, 13);
    if (et == 0x0806)
        return at(d, len, 14) == 0 && at(d, len, 15) == 1 && at(d, len, 16) == 8 &&
               at(d, len, 17) == 0 && at(d, len, 18) == 6 && at(d, len, 19) == 4;
    return et == 0x86DD && len >= 78 && d[20] == 58 && (d[54] == 135 || d[54] == 136);
}

/* handle_control_packet's table writes (src/worker.c:30-39, 64-95) for a classified packet: v
 * its verdict, d the frame as the GPU left it (an answered ARP request is already the reply,
 * whose tha / tpa hold the request's sha / spa, src/worker.c:42-51). */
static void control_writes(loop_t *L, const uint8_t *d, size_t len, uint32_t v) {
    if (v & UPE_VF_ARP_LEARN) {
        const int replied = (v & UPE_VF_ARP_REPLY) != 0;
        const uint8_t *spa = d + (replied ? 38 : 28);
        const uint32_t ip = (uint32_t)spa[0] << 24 | (uint32_t)spa[1] << 16 |
                            (uint32_t)spa[2] << 8 | (uint32_t)spa[3];
        L->ops->arp_update(L->user, ip, d + (replied ? 32 : 22));
    } else if (UPE_VERDICT_CODE(v) == UPE_V_CONSUMED) {
        const int ns = d[54] == 135;
        for (size_t off = 78; off + 2 <= len;) {
            const uint8_t type = d[off];
            const size_t olen = (uint8_t)(d[off + 1] * 8u); /* uint8_t, src/worker.c:73 */
            if (olen == 0 || off + olen > len) break;
            if (olen >= 8 && ((ns && type == 1) || (!ns && type == 2))) {
                L->ops->ndp_update(L->user, ns ? d + 22 : d + 62, d + off + 2);
                break;
            }
            off += olen;
        }
    }
}

/* The TX flush of worker_main, src/worker.c:286-303. */
static void flush_tx(loop_t *L) {
    if (L->tx_count > 0) {
        int sent = L->ops->tx_send_batch(L->user, L->tx_frames, L->tx_lens, L->tx_count);
        if (sent < 0) sent = 0;
        if (sent > L->tx_count) sent = L->tx_count;
        L->c.pkts_forwarded += (uint64_t)sent;
        L->c.pkts_dropped += (uint64_t)(L->tx_count - sent);
        for (int i = 0; i < L->tx_count; i++) L->ops->free_buf(L->user, L->tx_bufs[i]);
        L->tx_count = 0;
    }
}

/* Classify the gathered batch on the GPU, then walk it in packet order doing what
 * process_packet's exits and worker_main's flush do.  cut: the batch ends with a table-writing
 * control packet, whose write is applied and uploaded before anything else is classified. */
static int run_batch(loop_t *L, int cut) {
    const size_t n = L->n;
    if (n == 0) return 0;
    int rc;
    if (L->pool) {
        rc = upe_gpu_process_mapped(L->ctx, L->pool, L->desc, L->verdict, n, NULL);
        if (rc == 0) rc = upe_gpu_sync(L->ctx, NULL);
    } else {
        rc = upe_gpu_process_host_emit(L->ctx, L->win, n * WIN + UPE_FRAME_TAIL, L->desc,
                                       L->verdict, L->rec, n, 0, -1);
    }
    if (rc != 0) return -1;
    for (size_t i = 0; i < n; i++) {
        void *b = L->bufs[i];
        uint8_t *d = L->ops->data(L->user, b);
        const size_t len = L->ops->len(L->user, b);
        const uint32_t v = L->verdict[i];
        const uint32_t code = UPE_VERDICT_CODE(v);
        if (!L->pool) {
            /* window mode: the rewritten bytes into the caller's buffer */
            if (code == UPE_V_FWD)
                upe_hdr_apply(d, &L->rec[i]);
            else if (v & UPE_VF_ARP_REPLY)
                memcpy(d, L->win + i * WIN, len < UPE_REWRITE_EXTENT ? len : UPE_REWRITE_EXTENT);
        }
        if (L->left == 0) { /* the next burst starts here */
            L->left = L->bq[L->bq_head];
            L->bq_head = (L->bq_head + 1) % L->bq_cap;
            L->bq_len--;
        }
        if (v & UPE_VF_ARP_LEARN) L->c.arp_learn++;
        if (cut && i + 1 == n) control_writes(L, d, len, v); /* arp_update before the reply */
        if (v & UPE_VF_ARP_REPLY) {
            L->c.arp_reply++;
            (void)L->ops->tx_send(L->user, d, len); /* src/worker.c:52 */
        }
        if (code != UPE_V_DROP_PARSE && code != UPE_V_CONSUMED) L->c.pkts_parsed++;
        if (code == UPE_V_DROP_RULE || code == UPE_V_DROP_TTL || code == UPE_V_FWD ||
            code == UPE_V_DROP_ACTION)
            L->c.pkts_matched++;
        if (code == UPE_V_FWD) {
            L->tx_frames[L->tx_count] = d; /* src/worker.c:240-243 */
            L->tx_lens[L->tx_count] = len;
            L->tx_bufs[L->tx_count++] = b;
        } else if (code == UPE_V_CONSUMED) {
            L->c.pkts_consumed++;
            L->ops->free_buf(L->user, b); /* src/worker.c:96-98: no counter */
        } else {
            L->c.pkts_dropped++; /* every drop exit of process_packet counts one */
            L->ops->free_buf(L->user, b);
        }
        if (--L->left == 0) flush_tx(L); /* the burst is complete */
    }
    L->n = 0;
    if (cut && L->ops->load_neigh(L->user, L->ctx) != 0) return -1;
    if (L->ops->publish) L->ops->publish(L->user, L->ctx, &L->c);
    return 0;
}

/* Drop everything the loop holds after an error (the reference would have freed it). */
static void drain(loop_t *L) {
    for (size_t i = 0; i < L->n; i++) L->ops->free_buf(L->user, L->bufs[i]);
    L->n = 0;
    for (int i = 0; i < L->tx_count; i++) L->ops->free_buf(L->user, L->tx_bufs[i]);
    L->tx_count = 0;
}

int upe_gpu_worker_run(upe_gpu_ctx_t *ctx, const upe_worker_ops_t *ops, void *user,
                       const upe_worker_cfg_t *cfg, upe_counters_t *counters) {
    if (!ctx || !ops) return upe_gpu_set_last_error("null context or ops");
    if (!ops->pop_burst || !ops->stop || !ops->data || !ops->len || !ops->free_buf ||
        !ops->tx_send || !ops->tx_send_batch || !ops->arp_update || !ops->ndp_update ||
        !ops->load_neigh || (ops->poll && !ops->sync))
        return upe_gpu_set_last_error("a required worker callback is missing");
    loop_t L;
    memset(&L, 0, sizeof L);
    L.ctx = ctx;
    L.ops = ops;
    L.user = user;
    L.cap = cfg && cfg->batch ? cfg->batch : 65536;
    L.burst = cfg && cfg->burst ? cfg->burst : 32;
    L.pool = cfg ? cfg->pool_base : NULL;
    L.pool_bytes = cfg ? cfg->pool_bytes : 0;
    const long idle = cfg && cfg->idle_ns ? (long)cfg->idle_ns : 1000;
    if (L.burst > UPE_TX_BATCH_MAX) return upe_gpu_set_last_error("burst exceeds UPE_TX_BATCH_MAX");
    if (L.cap > ((size_t)1 << 24)) return upe_gpu_set_last_error("batch exceeds 2^24 packets");
    if (L.pool && ((uintptr_t)L.pool & 15u))
        return upe_gpu_set_last_error("pool_base must be 16-byte aligned");
    if (L.pool && L.pool_bytes < UPE_FRAME_TAIL)
        return upe_gpu_set_last_error("pool_bytes must give the registered region's size");
    L.bufs = malloc((L.cap + L.burst) * sizeof(void *));
    L.bq_cap = L.cap + 2;
    L.bq = malloc(L.bq_cap * sizeof(unsigned));
    L.desc = upe_gpu_host_alloc(L.cap * sizeof(uint64_t));
    L.verdict = upe_gpu_host_alloc(L.cap * sizeof(uint32_t));
    if (!L.pool) {
        L.win = upe_gpu_host_alloc(L.cap * WIN + UPE_FRAME_TAIL);
        L.rec = upe_gpu_host_alloc(L.cap * sizeof(upe_hdr_rec_t));
    }
    int rc = 0;
    if (!L.bufs || !L.bq || !L.desc || !L.verdict || (!L.pool && (!L.win || !L.rec))) {
        rc = upe_gpu_set_last_error("out of memory (worker loop buffers)");
        goto out;
    }
    void *burst[UPE_TX_BATCH_MAX];
    for (;;) {
        const unsigned k = ops->pop_burst(user, burst, L.burst); /* src/worker.c:268 */
        /* a change between bursts (polled after the pop: a burst pushed after the change was
         * made is classified with it): the packets held finish with the old state first */
        if (ops->poll && ops->poll(user) &&
            (run_batch(&L, 0) != 0 || ops->sync(user, ctx) != 0)) {
            for (unsigned r = 0; r < k; r++) L.bufs[L.n++] = burst[r];
            goto fail;
        }
        if (k == 0) {
            if (L.n > 0) { /* the ring is empty: classify what is held now */
                if (run_batch(&L, 0) != 0) goto fail;
                continue;
            }
            if (ops->stop(user)) break; /* stop signal + ring empty, src/worker.c:270-273 */
            struct timespec ts = {0, idle};
            nanosleep(&ts, NULL);
            continue;
        }
        L.c.pkts_in += k; /* src/worker.c:280 */
        L.bq[(L.bq_head + L.bq_len) % L.bq_cap] = k;
        L.bq_len++;
        for (unsigned j = 0; j < k; j++) {
            void *b = burst[j];
            uint8_t *d = ops->data(user, b);
            const size_t len = ops->len(user, b);
            if (L.pool) {
                const size_t off = (size_t)(d - L.pool);
                const size_t span = len > UPE_FRAME_TAIL ? len : UPE_FRAME_TAIL;
                if (d < L.pool || off > L.pool_bytes || span > L.pool_bytes - off || (off & 15u) ||
                    len > 0xFFFFu) {
                    upe_gpu_set_last_error(
                        "a frame is not 16-byte aligned inside the registered pool");
                    for (unsigned r = j; r < k; r++) L.bufs[L.n++] = burst[r];
                    goto fail;
                }
                L.desc[L.n] = UPE_DESC(off, len);
            } else {
                const size_t c = len < WIN ? len : WIN;
                memcpy(L.win + L.n * WIN, d, c);
                L.desc[L.n] = UPE_DESC(L.n * WIN, len);
            }
            L.bufs[L.n++] = b;
            const int cut = is_table_write(d, len);
            if ((cut || L.n == L.cap) && run_batch(&L, cut) != 0) {
                /* the rest of this burst is held by nobody else: keep it for the drain */
                for (unsigned r = j + 1; r < k; r++) L.bufs[L.n++] = burst[r];
                goto fail;
            }
        }
    }
    goto out;
fail:
    rc = -1;
    drain(&L);
out:
    if (counters) *counters = L.c;
    free(L.bufs);
    free(L.bq);
    if (L.desc) upe_gpu_host_free(L.desc);
    if (L.verdict) upe_gpu_host_free(L.verdict);
    if (L.win) upe_gpu_host_free(L.win);
    if (L.rec) upe_gpu_host_free(L.rec);
    return rc;
}
