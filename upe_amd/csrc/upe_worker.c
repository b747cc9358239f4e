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
 * Two batches are in flight (round 5): batch k is launched and, while the GPU classifies it, the
 * loop walks batch k - 1's verdicts (the TX calls, the frees) and then gathers batch k + 1 into
 * the slot k - 1 used — the GPU's share of a batch hides behind the host's.  A batch cut at a
 * table-writing packet drains the pipeline instead (walk k - 1, wait for k, walk it, apply the
 * write, upload the tables) before anything later is launched, and so does a change polled
 * between bursts: the order of every call is the sequential loop's.  An empty ring launches the
 * partial batch gathered so far like a full one (round 6: with the reference's 8192-buffer pool
 * a 65536-packet batch never fills, and draining at every empty ring serialised the GPU and the
 * host), and drains only when the ring is still empty on the next pop.  The walk
 * reads nothing of a frame it does not rewrite: the handle's data pointer and length are kept
 * from the gather.
 *
 * Two ways to get a batch to the GPU (cfg->pool_base): copy each frame's header window into
 * pinned staging and let the kernel read the windows there over the link (round 6: until round 5
 * the windows and descriptors went over by DMA and the verdicts and records came back the same
 * way, four copies per batch whose fixed cost bound the loop at the reference's small pool), or
 * leave the frames where they are in a registered pool and let the kernel read them there.
 * Either way the verdicts and 16-byte records are written into pinned host memory
 * (upe_gpu_process_mapped_emit, nothing copied) and the records applied in the walk.  (Rewriting the frames in the pool from the GPU
 * instead, upe_gpu_process_mapped, measured 50 vs 66 Mpps for one worker thread on the reference
 * benchmark: the link writes evict the frame lines the walk and pktbuf_free then touch.)
 */
#define _GNU_SOURCE
#include <stdlib.h>
#include <stdio.h>
#include <string.h>
#include <time.h>
#include <emmintrin.h>

#include "../../include/upe_gpu.h"

/* upe_gpu.hip, not part of the ABI: the calling thread's upe_gpu_last_error() message, and
 * completion marks on the context's stream */
int upe_gpu_set_last_error(const char *msg);
int upe_gpu_mark(upe_gpu_ctx_t *ctx, int slot);
int upe_gpu_mark_wait(upe_gpu_ctx_t *ctx, int slot);
int upe_gpu_tag_host(upe_gpu_ctx_t *ctx, int on);

#define WIN UPE_HDR_WINDOW
#define NSLOT 2
/* a batch boundary with nothing on the GPU (device statistics equal to the counters) at least
 * this often in a stream that never drains: see advance() */
#define STATS_POINT_EVERY 32

/* One batch: gathered, then launched (busy), then walked. */
typedef struct {
    void **bufs;           /* handles in arrival order */
    uint8_t **data;        /* their frames, as data() gave them at the gather */
    size_t n;
    int cut;               /* ends with a table-writing control packet */
    int busy;              /* launched, not walked yet */
    uint64_t *desc;        /* pinned: offset << 16 | len */
    uint32_t *verdict;     /* pinned (mapped mode: written by the kernel over the link) */
    uint8_t *win;          /* window mode: pinned header windows (read by the kernel there) */
    upe_hdr_rec_t *rec;    /* pinned records (written by the kernel over the link) */
} slot_t;

typedef struct {
    upe_gpu_ctx_t *ctx;
    const upe_worker_ops_t *ops;
    void *user;
    size_t cap;        /* packets per batch */
    unsigned burst;
    uint8_t *pool;     /* mapped mode: registered region the frames lie in */
    size_t pool_bytes;
    slot_t s[NSLOT];
    int g;             /* the slot being gathered */
    int o;             /* the busy slot launched before it, or -1 */
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
    /* UPE_WORKER_PROFILE=1 (diagnostic): where the loop's time goes, printed at the end */
    int inplace;       /* mapped mode, UPE_WORKER_MAPPED_INPLACE=1 (diagnostic): the kernel
                          rewrites the frames in the pool instead of emitting records */
    int prof;
    uint64_t t_wait, t_walk, t_launch, n_batches, t_flush;
    uint64_t t_gather, n_empty, n_sleep, n_partial;   /* (profile) gather time, empty pops,
                                                         idle naps, launches of a partial batch */
    unsigned since_point;  /* batches walked since the last publish with nothing in flight */
} loop_t;

static uint64_t mono_ns(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

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
        const uint64_t t0 = L->prof ? mono_ns() : 0;
        int sent = L->ops->tx_send_batch(L->user, L->tx_frames, L->tx_lens, L->tx_count);
        if (sent < 0) sent = 0;
        if (sent > L->tx_count) sent = L->tx_count;
        L->c.pkts_forwarded += (uint64_t)sent;
        L->c.pkts_dropped += (uint64_t)(L->tx_count - sent);
        if (L->ops->free_burst)
            L->ops->free_burst(L->user, L->tx_bufs, (unsigned)L->tx_count);
        else
            for (int i = 0; i < L->tx_count; i++) L->ops->free_buf(L->user, L->tx_bufs[i]);
        L->tx_count = 0;
        if (L->prof) L->t_flush += mono_ns() - t0;
    }
}

/* A frame's header window into the pinned staging the kernel reads over the link, with
 * streaming (non-temporal) stores: the lines go to memory without being read for ownership, and
 * the GPU's read finds them there instead of snooping them out of this core's cache.  (With
 * cached stores into staging the GPU had just read, the gather cost 57 ns per packet at the
 * reference's 8192-buffer pool — 2048-packet batches, staging that stays cache-resident — against
 * 8 ns with 65536-packet batches.)  16-byte pieces; the last one zero-padded past len (the
 * kernel never reads those bytes).  `win` is 16-byte aligned. */
static inline void stage_window(uint8_t *win, const uint8_t *d, size_t len) {
    const size_t c = len < WIN ? len : WIN;
    size_t o = 0;
    for (; o + 16 <= c; o += 16)
        _mm_stream_si128((__m128i *)(win + o), _mm_loadu_si128((const __m128i *)(d + o)));
    if (o < c) {   /* the last piece: only the frame's own bytes are read */
        uint8_t t[16] = {0};
        memcpy(t, d + o, c - o);
        _mm_stream_si128((__m128i *)(win + o), _mm_loadu_si128((const __m128i *)t));
    }
}

/* upe_hdr_apply (upe_host.c) inlined into the walk: one record into its frame. */
static inline void rec_apply(uint8_t *frame, const upe_hdr_rec_t *rec) {
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

/* Queue slot k's batch on the GPU (asynchronously) and mark its completion. */
static int launch(loop_t *L, int k) {
    slot_t *S = &L->s[k];
    const size_t n = S->n;
    const uint64_t t0 = L->prof ? mono_ns() : 0;
    int rc;
    if (L->pool && !L->inplace) {
        rc = upe_gpu_process_mapped_emit(L->ctx, L->pool, S->desc, S->verdict, S->rec, n, NULL);
    } else if (L->pool) {
        rc = upe_gpu_process_mapped(L->ctx, L->pool, S->desc, S->verdict, n, NULL);
    } else {
        /* the header windows in pinned staging, classified where they lie (the kernel reads them
         * over the link, writes verdicts and records back): one launch, no DMA copies; the
         * streaming stores of the gather drained to memory first */
        _mm_sfence();
        rc = upe_gpu_process_mapped_emit(L->ctx, S->win, S->desc, S->verdict, S->rec, n, NULL);
    }
    if (rc == 0) rc = upe_gpu_mark(L->ctx, k);
    S->busy = rc == 0;
    if (L->prof) {
        L->t_launch += mono_ns() - t0;
        L->n_batches++;
    }
    return rc;
}

/* Wait for slot k's batch, then walk it in packet order doing what process_packet's exits and
 * worker_main's flush do.  A cut batch's last packet writes the tables, which are re-uploaded
 * before anything else is launched. */
static int walk(loop_t *L, int k) {
    slot_t *S = &L->s[k];
    const uint64_t t0 = L->prof ? mono_ns() : 0;
    if (upe_gpu_mark_wait(L->ctx, k) != 0) return -1;
    const uint64_t t1 = L->prof ? mono_ns() : 0;
    const size_t n = S->n;
    size_t rec = 0; /* window mode: the next forwarded packet's record (compacted per 64) */
    for (size_t i = 0; i < n; i++) {
        void *b = S->bufs[i];
        uint8_t *d = S->data[i];
        /* the first line of a frame a few packets ahead, for the record's writes and the
         * handle's release (the line left this core's caches since the gather) */
        if (i + 16 < n) __builtin_prefetch(S->data[i + 16], 1);
        const size_t len = (size_t)(S->desc[i] & 0xFFFFu);
        const uint32_t v = S->verdict[i];
        const uint32_t code = UPE_VERDICT_CODE(v);
        if (L->pool && !L->inplace) {
            /* mapped mode: the forwarded frames' records applied here, where the frame's first
             * line is still in this core's cache from the gather (the kernel only reads the pool;
             * an answered ARP request it rewrote in place) */
            if ((i & 63u) == 0) rec = i;
            if (code == UPE_V_FWD) rec_apply(d, &S->rec[rec++]);
        } else if (!L->pool) {
            /* window mode: the rewritten bytes into the caller's buffer (an answered ARP
             * request was rewritten by the kernel in its staged window) */
            if ((i & 63u) == 0) rec = i;
            if (code == UPE_V_FWD) {
                rec_apply(d, &S->rec[rec++]);
            } else if (v & UPE_VF_ARP_REPLY) {
                const size_t c = len < UPE_REWRITE_EXTENT ? len : UPE_REWRITE_EXTENT;
                memcpy(d, S->win + i * WIN, c);
            }
        }
        if (L->left == 0) { /* the next burst starts here */
            L->left = L->bq[L->bq_head];
            L->bq_head = (L->bq_head + 1) % L->bq_cap;
            L->bq_len--;
        }
        if (v & UPE_VF_ARP_LEARN) L->c.arp_learn++;
        if (S->cut && i + 1 == n) control_writes(L, d, len, v); /* arp_update before the reply */
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
    const int cut = S->cut;
    S->n = 0;
    S->cut = 0;
    S->busy = 0;
    if (L->prof) {
        const uint64_t t2 = mono_ns();
        L->t_wait += t1 - t0;
        L->t_walk += t2 - t1;
    }
    if (cut && L->ops->load_neigh(L->user, L->ctx) != 0) return -1;
    L->since_point++;
    return 0;
}

/* The counters so far to the program.  With a batch still on the GPU the context's statistics
 * already hold some of its packets, which the counters do not: publish gets a NULL context then
 * (counters only).  With nothing in flight it gets the context, whose upe_gpu_get_stats then
 * matches the counters packet for packet. */
static void publish(loop_t *L, int in_flight) {
    if (!L->ops->publish) return;
    L->ops->publish(L->user, in_flight ? NULL : L->ctx, &L->c);
    if (!in_flight) L->since_point = 0;
}

/* Every batch held to completion, oldest first: the gathering slot's is launched first if it
 * holds packets.  Afterwards nothing is on the GPU. */
static int finish_all(loop_t *L) {
    slot_t *G = &L->s[L->g];
    const int any = G->n > 0 || L->o >= 0;
    if (G->n > 0 && !G->busy && launch(L, L->g) != 0) return -1;
    if (L->o >= 0 && walk(L, L->o) != 0) return -1;
    L->o = -1;
    if (G->busy && walk(L, L->g) != 0) return -1;
    if (any) publish(L, 0);
    return 0;
}

/* The gathering slot is complete (full, or cut): launch it; walk the older batch meanwhile and
 * gather the next one into its slot — or, after a cut, drain everything.  Every
 * STATS_POINT_EVERY batches the older batch is walked BEFORE the launch instead, so that the
 * program sees its statistics and counters agree at least that often (one batch's GPU time not
 * hidden, once per STATS_POINT_EVERY). */
static int advance(loop_t *L) {
    if (L->s[L->g].cut) return finish_all(L);
    if (L->o >= 0 && L->since_point + 1 >= STATS_POINT_EVERY) {
        if (walk(L, L->o) != 0) return -1;
        L->o = -1;
        publish(L, 0);
    }
    if (launch(L, L->g) != 0) return -1;
    if (L->o >= 0) {
        if (walk(L, L->o) != 0) return -1;
        publish(L, 1);
    }
    L->o = L->g;
    L->g = (L->g + 1) % NSLOT;
    return 0;
}

/* Drop everything the loop holds after an error (the reference would have freed it). */
static void drain(loop_t *L) {
    if (L->o >= 0) (void)upe_gpu_mark_wait(L->ctx, L->o);   /* the GPU is done with them */
    if (L->s[L->g].busy) (void)upe_gpu_mark_wait(L->ctx, L->g);
    for (int k = 0; k < NSLOT; k++) {
        for (size_t i = 0; i < L->s[k].n; i++) L->ops->free_buf(L->user, L->s[k].bufs[i]);
        L->s[k].n = 0;
    }
    for (int i = 0; i < L->tx_count; i++) L->ops->free_buf(L->user, L->tx_bufs[i]);
    L->tx_count = 0;
}

static void free_slots(loop_t *L) {
    for (int k = 0; k < NSLOT; k++) {
        slot_t *S = &L->s[k];
        free(S->bufs);
        free(S->data);
        if (S->desc) upe_gpu_host_free(S->desc);
        if (S->verdict) upe_gpu_host_free(S->verdict);
        if (S->win) upe_gpu_host_free(S->win);
        if (S->rec) upe_gpu_host_free(S->rec);
    }
}

static int alloc_slots(loop_t *L) {
    for (int k = 0; k < NSLOT; k++) {
        slot_t *S = &L->s[k];
        S->bufs = malloc((L->cap + L->burst) * sizeof(void *));
        S->data = malloc((L->cap + L->burst) * sizeof(uint8_t *));
        S->desc = upe_gpu_host_alloc(L->cap * sizeof(uint64_t));
        S->verdict = upe_gpu_host_alloc(L->cap * sizeof(uint32_t));
        if (!S->bufs || !S->data || !S->desc || !S->verdict) return -1;
        if (L->pool && !L->inplace) {
            S->rec = upe_gpu_host_alloc(L->cap * sizeof(upe_hdr_rec_t));
            if (!S->rec) return -1;
        }
        if (!L->pool) {
            S->win = upe_gpu_host_alloc(L->cap * WIN + UPE_FRAME_TAIL);
            S->rec = upe_gpu_host_alloc(L->cap * sizeof(upe_hdr_rec_t));
            if (!S->win || !S->rec) return -1;
            /* (the tail past the last window is read as zero by the kernel's window loads) */
            memset(S->win, 0, L->cap * WIN + UPE_FRAME_TAIL);
        }
    }
    return 0;
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
    L.o = -1;
    const char *pe = getenv("UPE_WORKER_PROFILE");
    L.prof = pe && pe[0] == '1';
    const char *pi = getenv("UPE_WORKER_MAPPED_INPLACE");
    L.inplace = pi && pi[0] == '1';
    const uint64_t t_start = L.prof ? mono_ns() : 0;
    const unsigned idle = cfg && cfg->idle_ns ? cfg->idle_ns : 1000;
    const struct timespec nap = {(time_t)(idle / 1000000000u), (long)(idle % 1000000000u)};
    if (L.burst > UPE_TX_BATCH_MAX) return upe_gpu_set_last_error("burst exceeds UPE_TX_BATCH_MAX");
    if (L.cap > ((size_t)1 << 24)) return upe_gpu_set_last_error("batch exceeds 2^24 packets");
    if (L.pool && ((uintptr_t)L.pool & 15u))
        return upe_gpu_set_last_error("pool_base must be 16-byte aligned");
    if (L.pool && L.pool_bytes < UPE_FRAME_TAIL)
        return upe_gpu_set_last_error("pool_bytes must give the registered region's size");
    /* every burst popped and not yet flushed: those of two batches in flight and a partial one */
    L.bq_cap = NSLOT * (L.cap + L.burst) + 4;
    L.bq = malloc(L.bq_cap * sizeof(unsigned));
    int rc = 0;
    /* (this loop's launches run the host-path kernel instantiation: profiles keep them apart from
     * device-resident batches of the same process) */
    (void)upe_gpu_tag_host(ctx, 1);
    if (!L.bq || alloc_slots(&L) != 0) {
        rc = upe_gpu_set_last_error("out of memory (worker loop buffers)");
        goto out;
    }
    void *burst[UPE_TX_BATCH_MAX];
    for (;;) {
        const unsigned k = ops->pop_burst(user, burst, L.burst); /* src/worker.c:268 */
        slot_t *G = &L.s[L.g];
        /* a change between bursts (polled after the pop: a burst pushed after the change was
         * made is classified with it): the packets held finish with the old state first */
        if (ops->poll && ops->poll(user)) {
            if (finish_all(&L) != 0 || ops->sync(user, ctx) != 0) {
                G = &L.s[L.g];
                for (unsigned r = 0; r < k; r++) G->bufs[G->n++] = burst[r];
                goto fail;
            }
            /* the counters (and statistics) as they stand under the new state, even if no
             * batch follows for a while */
            publish(&L, 0);
        }
        if (k == 0) {
            /* the ring is empty: classify what is gathered now, keeping it in flight while the
             * older batch is walked (a pool too small to fill a batch still overlaps), and walk
             * the last batch in flight once the ring is still empty after that */
            L.n_empty++;
            if (G->n > 0) {
                L.n_partial++;
                if (advance(&L) != 0) goto fail;
                continue;
            }
            if (L.o >= 0) {
                if (finish_all(&L) != 0) goto fail;
                continue;
            }
            if (ops->stop(user)) break; /* stop signal + ring empty, src/worker.c:270-273 */
            L.n_sleep++;
            nanosleep(&nap, NULL);
            continue;
        }
        L.c.pkts_in += k; /* src/worker.c:280 */
        L.bq[(L.bq_head + L.bq_len) % L.bq_cap] = k;
        L.bq_len++;
        /* the burst's frames first, their first lines requested together (the producer wrote
         * them on another core: one cross-core transfer each, overlapped) */
        const uint64_t tg0 = L.prof ? mono_ns() : 0;
        uint64_t t_adv = 0;   /* (profile) time inside advance() during this burst */
        uint8_t *bd[UPE_TX_BATCH_MAX];
        for (unsigned j = 0; j < k; j++) {
            bd[j] = ops->data(user, burst[j]);
            __builtin_prefetch(bd[j]);
        }
        for (unsigned j = 0; j < k; j++) {
            G = &L.s[L.g];
            void *b = burst[j];
            uint8_t *d = bd[j];
            const size_t len = ops->len(user, b);
            if (L.pool) {
                const size_t off = (size_t)(d - L.pool);
                const size_t span = len > UPE_FRAME_TAIL ? len : UPE_FRAME_TAIL;
                if (d < L.pool || off > L.pool_bytes || span > L.pool_bytes - off || (off & 15u) ||
                    len > 0xFFFFu) {
                    upe_gpu_set_last_error(
                        "a frame is not 16-byte aligned inside the registered pool");
                    for (unsigned r = j; r < k; r++) G->bufs[G->n++] = burst[r];
                    goto fail;
                }
                G->desc[G->n] = UPE_DESC(off, len);
            } else {
                /* (bytes of the window past len are never read: stale ones may stay) */
                stage_window(G->win + G->n * WIN, d, len);
                G->desc[G->n] = UPE_DESC(G->n * WIN, len);
            }
            G->data[G->n] = d;
            G->bufs[G->n++] = b;
            G->cut = is_table_write(d, len);
            if (G->cut || G->n == L.cap) {
                const uint64_t ta = L.prof ? mono_ns() : 0;
                if (advance(&L) != 0) {
                    /* the rest of this burst is held by nobody else: keep it for the drain */
                    G = &L.s[L.g];
                    for (unsigned r = j + 1; r < k; r++) G->bufs[G->n++] = burst[r];
                    goto fail;
                }
                if (L.prof) t_adv += mono_ns() - ta;
            }
        }
        if (L.prof) L.t_gather += mono_ns() - tg0 - t_adv;
    }
    goto out;
fail:
    rc = -1;
    drain(&L);
out:
    if (L.prof)
        fprintf(stderr, "upe_worker: %.3f s total, %llu batches (%.0f packets each): launch %.3f s, "
                "GPU wait %.3f s, walk %.3f s (of which TX flushes %.3f s), rest (pop + gather + idle) %.3f s "
                "(gather %.3f s; empty pops %llu, partial launches %llu, naps %llu)\n",
                (mono_ns() - t_start) * 1e-9, (unsigned long long)L.n_batches,
                L.n_batches ? (double)L.c.pkts_in / (double)L.n_batches : 0.0, L.t_launch * 1e-9,
                L.t_wait * 1e-9, L.t_walk * 1e-9, L.t_flush * 1e-9,
                (mono_ns() - t_start - L.t_launch - L.t_wait - L.t_walk) * 1e-9, L.t_gather * 1e-9,
                (unsigned long long)L.n_empty, (unsigned long long)L.n_partial,
                (unsigned long long)L.n_sleep);
    if (counters) *counters = L.c;
    (void)upe_gpu_tag_host(ctx, 0);
    free(L.bq);
    free_slots(&L);
    return rc;
}
