/*
 * upe_gpu.h — C ABI of the MI355X batch dataplane for UPE's per-packet worker hot path.
 *
 * This is the drop-in boundary.  The reference runs the path one packet at a
 * time inside process_packet() (reference src/worker.c:106-253): parse_flow_key()
 * (src/parser.c:6-111) -> rule_table_match() (src/rule_table.c:163-176) -> counters and
 * rule_stats (src/worker.c:119-153) -> L3 forward rewrite with the one-entry L1 neighbour caches
 * and arp_get_mac()/ndp_get_mac() (src/worker.c:155-244, src/arp_table.c:55-80,
 * src/ndp_table.c:67-86).  This library runs the same semantics over a whole batch of packets
 * resident in GPU memory with one HIP kernel, bit-exact per packet.
 *
 * The reference surface is kept as plain data: every struct below is an ABI mirror of the
 * reference layout (same size, same offsets, checked by _Static_assert), so a C caller passes
 * rt->rules / arpt->entries / ndpt->entries / tx->eth_addr straight through without conversion.
 *
 * Conventions follow the reference (SURVEY.md §8(b) "Errors"): int 0 on success / -1 on failure,
 * NULL for a failed constructor, and upe_gpu_last_error() for a message (thread-local).  No C++
 * exception crosses this ABI.  A context is owned by one worker thread (one HIP stream); it is
 * not internally locked, exactly like a reference worker_t.
 */
#ifndef UPE_GPU_H
#define UPE_GPU_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------------------------ */
/* ABI mirrors of the reference layouts                                                        */
/* ------------------------------------------------------------------------------------------ */

/* Mirrors ip_addr_t, reference include/parser.h:129-132.  IPv4 is host order in .v4 (ntohl),
 * IPv6 is wire-order bytes. */
typedef union {
    uint32_t v4;
    uint8_t v6[16];
} upe_ip_addr_t;

/* Mirrors flow_key_t, reference include/parser.h:134-141 (44 bytes). */
typedef struct {
    uint8_t ip_ver;
    upe_ip_addr_t src_ip;
    upe_ip_addr_t dst_ip;
    uint16_t src_port;
    uint16_t dst_port;
    uint8_t protocol;
} upe_flow_key_t;

/* Mirrors action_type_t / flow_action_t, reference include/rule_table.h:9-17. */
enum { UPE_ACT_DROP = 0, UPE_ACT_FWD = 1 };
typedef struct {
    int32_t type;        /* action_type_t is an int-sized enum */
    int32_t out_ifindex; /* never read by the worker (all TX goes to tx->ifindex) */
} upe_flow_action_t;

/* Mirrors rule_t, reference include/rule_table.h:19-35 (92 bytes). */
typedef struct {
    uint32_t priority;
    uint8_t ip_ver;
    upe_ip_addr_t src_ip;
    upe_ip_addr_t src_mask;
    upe_ip_addr_t dst_ip;
    upe_ip_addr_t dst_mask;
    uint16_t src_port;
    uint16_t dst_port;
    uint8_t protocol;
    upe_flow_action_t action;
    uint32_t rule_id;
} upe_rule_t;

/* Mirrors arp_entry_t, reference include/arp_table.h:13-18 (32 bytes on LP64). */
typedef struct {
    uint32_t ip;
    uint8_t mac[6];
    int64_t update_at; /* time_t */
    bool valid;
} upe_arp_entry_t;

/* Mirrors ndp_entry_t, reference include/ndp_table.h:13-18 (40 bytes on LP64). */
typedef struct {
    uint8_t ip[16];
    uint8_t mac[6];
    int64_t update_at; /* time_t */
    bool valid;
} upe_ndp_entry_t;

/* Mirrors rule_stat_t, reference include/worker.h:18-21. */
typedef struct {
    uint64_t packets;
    uint64_t bytes;
} upe_rule_stat_t;

/* The worker's one-entry neighbour caches, reference include/worker.h:56-63 (worker_t fields
 * last_arp_ip / last_arp_mac / last_ndp_ip / last_ndp_mac).  A calloc'd worker starts all-zero. */
typedef struct {
    uint32_t last_arp_ip;
    uint8_t last_arp_mac[6];
    uint8_t last_ndp_ip[16];
    uint8_t last_ndp_mac[6];
} upe_l1_state_t;

/* Per-worker counters, reference include/worker.h:37-41 plus the control-path tallies the
 * reference does not keep separately.  pkts_forwarded counts FWD verdicts (queued for TX); with
 * the reference's TX stub (tests/benchmark_throughput.c:37-42) that equals its forwarded count. */
typedef struct {
    uint64_t pkts_in;
    uint64_t pkts_parsed;
    uint64_t pkts_matched;
    uint64_t pkts_forwarded;
    uint64_t pkts_dropped;
    uint64_t pkts_consumed; /* NDP NS/NA eaten by handle_control_packet (src/worker.c:96-98) */
    uint64_t arp_learn;     /* ARP packets that reach arp_update (src/worker.c:31-35) */
    uint64_t arp_reply;     /* ARP requests answered in place (src/worker.c:40-52) */
} upe_counters_t;

/* ------------------------------------------------------------------------------------------ */
/* Per-packet verdict word                                                                     */
/* ------------------------------------------------------------------------------------------ */
/* bits 0-3  : verdict code (which exit of process_packet the packet took)
 * bits 4-7  : flags
 * bits 8-31 : index of the matched rule in the caller's sorted rules[] array, plus one
 *             (0 = no rule matched).  rules[idx].rule_id indexes rule_stats. */
enum {
    UPE_V_DROP_PARSE = 0,   /* parse_flow_key failed   src/worker.c:117-125 */
    UPE_V_DROP_NOMATCH = 1, /* no rule                 src/worker.c:130-137 */
    UPE_V_DROP_RULE = 2,    /* ACT_DROP                src/worker.c:146-153 */
    UPE_V_DROP_TTL = 3,     /* TTL / hop limit <= 1    src/worker.c:165-172, 204-211 */
    UPE_V_FWD = 4,          /* queued for TX           src/worker.c:155-244 */
    UPE_V_CONSUMED = 5,     /* NDP NS/NA consumed      src/worker.c:57-100 */
    UPE_V_DROP_ACTION = 6   /* unknown action type     src/worker.c:247-252 */
};
enum {
    UPE_VF_NEIGH_HIT = 0x10, /* MACs rewritten: dst = neighbour MAC, src = port MAC */
    UPE_VF_ARP_LEARN = 0x20, /* well-formed ARP: caller must arp_update(spa, sha) */
    UPE_VF_ARP_REPLY = 0x40, /* ARP request for our IPv4: frame rewritten in place into the
                                reply; caller must tx_send it */
    UPE_VF_L1_INIT = 0x80    /* forwarded v4/v6 packet whose destination equals the L1 cache
                                address the batch started with (ARP: and that address != 0) */
};
#define UPE_VERDICT_CODE(v) ((v) & 0xFu)
#define UPE_VERDICT_RULE(v) ((int64_t)((v) >> 8) - 1)

/* ------------------------------------------------------------------------------------------ */
/* Batch layout in GPU memory                                                                  */
/* ------------------------------------------------------------------------------------------ */
/* frames : one device buffer holding the frames back to back.  Every frame starts on a 16-byte
 *          boundary, and at least UPE_FRAME_TAIL readable bytes must follow each frame start
 *          (pad the buffer end).  Bytes at or beyond a frame's length are never used.
 * desc[i]: (byte_offset << 16) | len, len <= 65535, byte_offset a multiple of 16 below 2^36.
 *          A frame may be a header window shorter than len as long as it holds the first
 *          min(len, UPE_HDR_WINDOW) bytes.
 * verdict: n uint32 words, written by the kernel.
 * A batch is one constant-table segment: control packets (ARP, NDP NS/NA) in it are classified
 * exactly, but their table updates are applied by the caller after the batch (split batches at
 * control packets for exact sequential semantics). */
#define UPE_HDR_WINDOW 96
#define UPE_FRAME_TAIL 96
#define UPE_DESC(off, len) ((((uint64_t)(off)) << 16) | ((uint64_t)(len) & 0xFFFFu))

/* Result summary of the last processed batch. */
typedef struct {
    upe_counters_t counters; /* this batch only */
    uint64_t n_ctrl;         /* control packets (ARP + NDP NS/NA) in the batch */
    uint64_t first_ctrl;     /* index of the first one, or UINT64_MAX */
} upe_batch_info_t;

typedef struct upe_gpu_ctx upe_gpu_ctx_t;

/* ------------------------------------------------------------------------------------------ */
/* Entry points                                                                                */
/* ------------------------------------------------------------------------------------------ */

/* Last error message of the calling thread ("" if none). */
const char *upe_gpu_last_error(void);

/* Number of visible GPUs, or -1. */
int upe_gpu_device_count(void);

/* Host CPUs local to a GPU (its PCI function's NUMA node, sysfs local_cpulist) that the process
 * may run on (its affinity when the library was loaded): up to `cap` of them into cpus (may be
 * NULL), *numa_node (may be NULL) = the node or -1.  Returns how many there are, or -1. */
int upe_gpu_local_cpus(int device, int *cpus, size_t cap, int *numa_node);

/* Pin the calling thread to the slot-th CPU local to `device` (modulo their number), as the
 * reference pins each worker thread (affinity_pin_self, src/affinity.c:48; assign_cores,
 * src/main.c:143-175).  Pinned host buffers allocated afterwards by this thread come from the
 * GPU's NUMA node.  Returns the CPU, or -1. */
int upe_gpu_pin_self(int device, int slot);

/* Open a context on `device`, with its own HIP stream.  Replaces the per-worker state set up by
 * worker_init() (reference src/worker.c:309-330): counters, rule_stats sized by
 * rule_capacity (= rt->capacity, src/worker.c:326), calloc'd L1 caches. */
upe_gpu_ctx_t *upe_gpu_open(int device, size_t rule_capacity);
void upe_gpu_close(upe_gpu_ctx_t *ctx);

/* Upload the rule table: rules[0..count) in the order rule_table_t keeps them (sorted by
 * (priority, rule_id), reference src/rule_table.c:96-109,158).  Replaces the read-only borrow of
 * w->rt (src/worker.c:129).  count <= rule capacity given at open, every rule_id < capacity. */
int upe_gpu_load_rules(upe_gpu_ctx_t *ctx, const upe_rule_t *rules, size_t count);

/* Rule reload with the reference's SIGHUP semantics (src/main.c:216-282: a new table, a fresh
 * calloc'd rule_stats of the new table's capacity per worker, w->rt and w->rule_stats swapped
 * between two bursts; pkts_* and the L1 neighbour caches untouched).  The batches queued so far
 * finish with the old table; if old_stats is given, rule_stats[0..old_capacity) as they stand
 * then (indexed by the OLD table's rule_ids, what the stats thread last printed) are copied out
 * — the reference frees them after its grace period.  The next batch runs with rules[0..count)
 * (sorted, as for upe_gpu_load_rules; rule_id < rule_capacity) and rule_stats all zero, sized
 * rule_capacity (upe_gpu_get_stats reads that many from now on).  Counters and the L1 state
 * carry on.  Arguments are checked before anything changes.  Synchronous; 0 / -1. */
int upe_gpu_reload_rules(upe_gpu_ctx_t *ctx, const upe_rule_t *rules, size_t count,
                         size_t rule_capacity, upe_rule_stat_t *old_stats, size_t old_capacity);

/* The same reload in two halves (round 6), so that the table is built where the reference
 * builds it — in the stats thread, before the swap, while the workers keep forwarding
 * (src/main.c:222-257) — and the worker thread only uploads it between two bursts.
 * upe_rules_compile: the compiled table (rule words, family lists, tuple-space index or decision
 * tree) of `count` sorted rules for a rule_stats of rule_capacity entries; host only (no
 * context, no GPU), any thread; NULL on error (upe_gpu_last_error() on the calling thread).  The
 * build is what dominates a reload of a large table: 0.4 ms (1k rules, scanned) to ~300 ms
 * (16k flow rules, decision tree) on the GPU box's host.
 * upe_gpu_reload_image: upe_gpu_reload_rules() with that image (the capacity is the image's);
 * the image is not consumed.  upe_rules_image_free: NULL is a no-op. */
typedef struct upe_rule_image upe_rule_image_t;
upe_rule_image_t *upe_rules_compile(const upe_rule_t *rules, size_t count, size_t rule_capacity);
int upe_gpu_reload_image(upe_gpu_ctx_t *ctx, const upe_rule_image_t *image,
                         upe_rule_stat_t *old_stats, size_t old_capacity);
void upe_rules_image_free(upe_rule_image_t *image);

/* How the loaded table is classified: 0 = linear first-match scan (tables of up to 64 rules, or
 * a table whose tree outgrew its node budget), 1 = tuple-space index (large tables whose rules
 * fall into few mask signatures: one hash probe per signature, visited in order of each
 * signature's first rule), 2 = decision tree over the per-family rule lists (every other table
 * past 64 rules: a walk to a leaf, then the few rules listed there in order).  Each gives the
 * first match in (priority, rule_id) order (reference src/rule_table.c:163-176).  -1 on error. */
int upe_gpu_rule_index_kind(upe_gpu_ctx_t *ctx);

/* The decision tree of the loaded table (all zero when it has none). */
typedef struct {
    uint64_t nodes;        /* nodes of both families' trees */
    uint64_t leaf_entries; /* rule positions listed in the leaves */
    uint32_t depth4;       /* deepest leaf of the IPv4 tree */
    uint32_t depth6;       /* deepest leaf of the IPv6 tree */
    uint32_t max_leaf;     /* longest leaf list */
    uint32_t trees;        /* trees of the IPv4 forest | trees of the IPv6 forest << 16 */
} upe_rule_index_info_t;
int upe_gpu_rule_index_info(upe_gpu_ctx_t *ctx, upe_rule_index_info_t *info);

/* rule_table_match (reference src/rule_table.c:163-176) over n keys on the host, through the
 * decision tree the GPU path builds for rules[0..count) (sorted as for upe_gpu_load_rules; the
 * walk is the device's, bit for bit), or the per-family linear first match when the table gets
 * no tree.  out[i] = the sorted index of keys[i]'s first matching rule, or -1 (no match, or an
 * ip_ver other than 4 / 6).  info (optional): the tree's shape.  No GPU needed.  0 / -1. */
int upe_rules_match_host(const upe_rule_t *rules, size_t count, const upe_flow_key_t *keys,
                         size_t n, int64_t *out, upe_rule_index_info_t *info);

/* Upload a snapshot of the neighbour tables' slot arrays (arpt->entries / ndpt->entries with
 * their power-of-two capacities).  Lookups probe exactly as arp_get_mac/ndp_get_mac do.
 * Either table may be NULL with capacity 0 (every lookup misses). */
int upe_gpu_load_neigh(upe_gpu_ctx_t *ctx, const upe_arp_entry_t *arp, size_t arp_capacity,
                       const upe_ndp_entry_t *ndp, size_t ndp_capacity);

/* The TX port identity the worker reads from tx_ctx_t (include/tx.h:9-14): own MAC (source MAC of
 * forwarded frames, src/worker.c:199,229) and own IPv4 (ARP replies, src/worker.c:40). */
int upe_gpu_set_port(upe_gpu_ctx_t *ctx, const uint8_t eth_addr[6], uint32_t ip4_addr);

/* L1 neighbour-cache state (kept on the device between batches). */
int upe_gpu_set_l1(upe_gpu_ctx_t *ctx, const upe_l1_state_t *l1);
int upe_gpu_get_l1(upe_gpu_ctx_t *ctx, upe_l1_state_t *l1);

/* Process one batch resident in GPU memory (see "Batch layout").  Asynchronous on `stream`
 * (a hipStream_t; NULL = the context's own stream).  Frames are rewritten in place exactly as
 * process_packet rewrites b->data.  Counters, rule stats and the L1 state accumulate in the
 * context, as they do in worker_t. */
int upe_gpu_process(upe_gpu_ctx_t *ctx, uint8_t *d_frames, const uint64_t *d_desc,
                    uint32_t *d_verdict, size_t n, void *stream);

/* Rewritten-header record (emit mode), 16 bytes per packet.  process_packet rewrites at most
 * three places of a forwarded frame (src/worker.c:162-244): bytes 0..11 (dst MAC = the next-hop
 * MAC and src MAC = tx->eth_addr on a neighbour hit), the TTL (IPv4 byte 22) with the header
 * checksum (bytes 24..25), or the hop limit (IPv6 byte 21).  Emit mode leaves the frame alone
 * and writes those bytes here instead, one coalesced 16-byte store per packet:
 *   b[0..11]  bytes 0..11 of the forwarded frame (the original MACs when the lookup missed)
 *   b[12]     new TTL (IPv4) or hop limit (IPv6)
 *   b[13..14] new IPv4 header checksum as stored at frame bytes 24..25 (0 for IPv6)
 *   b[15]     4 or 6: the packet was forwarded (verdict code UPE_V_FWD) as that family
 * upe_hdr_apply(frame, rec) turns a frame into exactly the bytes process_packet leaves in
 * b->data; it does nothing when b[15] == 0.
 *
 * Layout of a launch's records (round 5): only forwarded packets get one, compacted per 64-packet
 * group in packet order — forwarded packet i's record is rec[64 * (i / 64) + k], k = the number
 * of forwarded packets before it among packets 64 * (i / 64) .. i - 1 (the kernel's ballot and
 * lane count; a reader walking the verdicts in order keeps a cursor, reset to i at every multiple
 * of 64).  The other slots are not written.  UPE_HDR_SLOT gives the slot from that count.
 *
 * BREAKING CHANGE in layout 2 (round 5): layout 1 (rounds 1-4) wrote one record per packet at
 * rec[i], zero for packets not forwarded.  A caller that reads rec[i] per packet applies wrong or
 * stale records under layout 2 without any error: it must walk with the cursor above (or
 * UPE_HDR_SLOT), or check UPE_HDR_LAYOUT at compile time and upe_gpu_hdr_layout() at run time
 * (the library it actually loaded) before trusting either form. */
#define UPE_HDR_LAYOUT 2
#define UPE_HDR_SLOT(i, k) ((((size_t)(i)) & ~(size_t)63) + (size_t)(k))
int upe_gpu_hdr_layout(void);   /* UPE_HDR_LAYOUT of the loaded library */
typedef struct {
    uint8_t b[16];
} upe_hdr_rec_t;

/* upe_gpu_process() in emit mode: d_hdr (device, room for n records, 16-byte aligned) receives
 * the forwarded packets' rewritten header bytes (the record layout above) and the frames are not
 * written — except the ARP requests answered
 * in place (UPE_VF_ARP_REPLY), which the reference transmits at once (src/worker.c:40-52).
 * Verdicts, counters, rule_stats and the L1 state are exactly those of upe_gpu_process().  This
 * is the layout for a TX path that sends header and payload as separate pieces (sendmmsg
 * iovecs, or a NIC gather list) and for host round trips, which then copy back 16 bytes per
 * packet instead of the header span; in-place rewriting of 64-byte frames costs the path the
 * partial 128-byte lines it dirties. */
int upe_gpu_process_emit(upe_gpu_ctx_t *ctx, uint8_t *d_frames, const uint64_t *d_desc,
                         uint32_t *d_verdict, upe_hdr_rec_t *d_hdr, size_t n, void *stream);

/* A ring of `count` resident batches of n packets each in ONE launch (throughput mode): the
 * batches lie back to back in the "Batch layout" (batch j = descriptors, verdicts and records
 * [j*n, (j+1)*n), frames anywhere in d_frames) and are classified in ring order by one
 * persistent launch in emit mode, so the per-launch cost (dispatch, the first windows' round
 * trip, the tail, the boundary) is paid once per ring, not once per batch.  Counters,
 * rule_stats, the L1 state, every verdict code and every record equal those of `count`
 * back-to-back upe_gpu_process_emit() calls over the batches (record slots are counted from the
 * ring's first packet; n is a multiple of 64, so each batch's records stay in its own range);
 * UPE_VF_L1_INIT is relative to the ring's start.  n a multiple of 1024, n * count <= 2^24.  d_done_ns (optional, device or
 * host-mapped, count entries): for each batch, the time (ns) from the launch's first workgroup
 * to the moment its last workgroup had issued the batch's last stores — per-batch completion
 * latency — or 0 where not stamped (stamps need a linear-scan table, batches of at least
 * one tile per persistent workgroup, 256k packets on MI355X, and at most 64 batches per
 * workgroup's share).  A stamp excludes the launch's final repair of look-back candidates that
 * waves deferred (launch_info().deferred > 0, only when another kernel holds CUs): such a
 * batch's last verdicts and records are final when the launch completes, not at its stamp.
 * Asynchronous on `stream`. */
int upe_gpu_process_ring_emit(upe_gpu_ctx_t *ctx, uint8_t *d_frames, const uint64_t *d_desc,
                              uint32_t *d_verdict, upe_hdr_rec_t *d_hdr, size_t n, size_t count,
                              uint64_t *d_done_ns, void *stream);

/* Apply one record to its frame (host; src/worker.c:174-176,197-200,213,227-230 as bytes). */
void upe_hdr_apply(uint8_t *frame, const upe_hdr_rec_t *rec);

/* Host round trip: process n packets that live in HOST memory, the way the path runs between
 * libpcap (reference src/rx_pcap.c:42-93 fills pktbufs in host memory) and AF_PACKET TX
 * (src/tx_afpacket.c:78-118 sends from host memory).  The batch is cut into chunks of `chunk`
 * packets (0 = 256k) pipelined through a ring of device slots (4; UPE_GPU_HOST_SLOTS): chunk k+1's frames and descriptors go
 * host->device on a copy stream while chunk k is classified on the context's stream and chunk
 * k-1's verdicts and rewritten header bytes go device->host on a second copy stream.  Chunks are
 * classified in order, so counters, rule_stats and the L1 state evolve exactly as for
 * back-to-back upe_gpu_process() batches of `chunk` packets (upe_gpu_batch_info() describes the
 * last chunk).  h_frames / h_desc follow the "Batch layout" (offsets relative to h_frames,
 * frames_bytes covering UPE_FRAME_TAIL bytes past every frame start); a frame may be a header
 * window (UPE_HDR_WINDOW), which is how a caller avoids shipping payloads.  Only the first
 * min(len, UPE_REWRITE_EXTENT) bytes of a frame can change; those are copied back in place.
 * Synchronous.  Buffers from upe_gpu_host_alloc() (pinned) give the full PCIe rate; pageable
 * buffers work at the staged-copy rate. */
#define UPE_REWRITE_EXTENT 48
int upe_gpu_process_host(upe_gpu_ctx_t *ctx, uint8_t *h_frames, size_t frames_bytes,
                         const uint64_t *h_desc, uint32_t *h_verdict, size_t n, size_t chunk);

/* The host round trip in emit mode (chunk 0 = 128k packets): the same pipeline, but only the verdicts and the 16-byte
 * rewritten-header records come back (h_hdr, room for n records in the layout above, counted
 * from the batch's first packet; chunks are whole 64-packet groups; pinned for the full rate: 20 bytes per
 * packet over the link instead of the frames' rewritten span — the link's two directions share
 * its bandwidth, so fewer bytes back let the frames go in faster).  apply_threads >= 0: the
 * records are applied to h_frames on the host (upe_hdr_apply, answered ARP requests copied back)
 * by the calling thread plus `apply_threads` pool threads pinned near the GPU, two chunks behind
 * the copies, so that on return h_frames, h_verdict, counters, rule_stats and the L1 state are
 * exactly those of upe_gpu_process_host(); apply_threads = -1 leaves the frames as they were
 * except the answered ARP requests (as upe_gpu_process_emit does; a TX path that sends each
 * record as its own iovec).  Synchronous.  0 / -1. */
int upe_gpu_process_host_emit(upe_gpu_ctx_t *ctx, uint8_t *h_frames, size_t frames_bytes,
                              const uint64_t *h_desc, uint32_t *h_verdict, upe_hdr_rec_t *h_hdr,
                              size_t n, size_t chunk, int apply_threads);

/* Egress (reference src/worker.c:240-243, 287-303 and src/tx_afpacket.c:78-118): the forwarded
 * frames of a classified host batch (verdict code UPE_V_FWD, frames as the path left them —
 * rewritten in place, or with the emit records applied by upe_hdr_apply), in packet order, handed
 * to `send` the way the reference's worker loop flushes them: one call per input burst of `burst`
 * packets that forwarded anything (WORKER_BURST_SIZE = 32 in the reference; at most
 * UPE_TX_BATCH_MAX = 64 frames per call, the sendmmsg cap of src/tx_afpacket.c:82-84).  `send` has
 * tx_send_batch's contract with a user pointer first: it returns the frames it sent (negative
 * counts as 0).  *forwarded += sent and *dropped += count - sent, as the worker counts them
 * (src/worker.c:290-294); the caller then frees every buffer of the batch.  0, or -1 for a bad
 * argument (burst 0 or above UPE_TX_BATCH_MAX). */
#define UPE_TX_BATCH_MAX 64
typedef int (*upe_tx_batch_fn)(void *user, const uint8_t *const *frames, const size_t *lens,
                               int count);
int upe_tx_flush(const uint8_t *h_frames, const uint64_t *h_desc, const uint32_t *h_verdict,
                 size_t n, size_t burst, upe_tx_batch_fn send, void *user, uint64_t *forwarded,
                 uint64_t *dropped);
/* The same TX calls from the grouped egress list of upe_gpu_process_emit_tx (h_tx, h_tx_count
 * copied to the host) instead of the verdicts: no per-packet verdict scan; the same calls,
 * arguments and accounting as upe_tx_flush. */
int upe_tx_flush_groups(const uint8_t *h_frames, const uint64_t *h_desc, const uint32_t *h_tx,
                        const uint32_t *h_tx_count, size_t n, size_t burst, upe_tx_batch_fn send,
                        void *user, uint64_t *forwarded, uint64_t *dropped);

/* ------------------------------------------------------------------------------------------ */
/* The GPU-backed worker loop (upe_amd/csrc/upe_worker.c, C)                                   */
/* ------------------------------------------------------------------------------------------ */
/* What the loop needs from the program around it: the callees of reference worker_main /
 * process_packet (SURVEY.md §8(b) "Callees"), as callbacks with a user pointer first.  A packet
 * buffer is an opaque handle (a pktbuf_t *). */
typedef struct upe_worker_ops {
    /* ring_pop_burst (src/ring.c:53): up to `max` handles into bufs, returns how many */
    unsigned (*pop_burst)(void *user, void **bufs, unsigned max);
    /* g_stop (src/worker.c:18), read only when the ring is empty, as src/worker.c:270-273 */
    int (*stop)(void *user);
    /* a handle's frame: b->data and b->len (include/pktbuf.h:10-14) */
    uint8_t *(*data)(void *user, void *buf);
    size_t (*len)(void *user, void *buf);
    /* pktbuf_free (src/pktbuf.c:324) */
    void (*free_buf)(void *user, void *buf);
    /* tx_send / tx_send_batch (src/tx_afpacket.c:60-118) */
    int (*tx_send)(void *user, const uint8_t *frame, size_t len);
    int (*tx_send_batch)(void *user, const uint8_t *const *frames, const size_t *lens, int count);
    /* handle_control_packet's table writes (src/worker.c:30-39, 64-95): arp_update(ip host
     * order, mac), ndp_update(ip, mac); then the loop calls load_neigh so that the next packet
     * sees the write: the callee uploads the tables (upe_gpu_load_neigh under its locks) */
    void (*arp_update)(void *user, uint32_t ip, const uint8_t mac[6]);
    void (*ndp_update)(void *user, const uint8_t ip[16], const uint8_t mac[6]);
    int (*load_neigh)(void *user, upe_gpu_ctx_t *ctx);
    /* optional: polled after every pop; nonzero = the program changed something the context
     * holds (a SIGHUP rule swap, src/main.c:258-265; neighbour expiry, src/main.c:205-214): the
     * loop finishes the packets popped before with the old state, then calls sync(), which
     * makes the change (upe_gpu_reload_rules, upe_gpu_load_neigh), and classifies the burst just
     * popped with the new state.  A nonzero return of sync() ends the loop with -1. */
    int (*poll)(void *user);
    int (*sync)(void *user, upe_gpu_ctx_t *ctx);
    /* optional: after every GPU batch walked, and after every sync(), the loop's counters so far
     * (the worker_t fields the stats thread reads, src/main.c:284-315: pkts_in, pkts_parsed,
     * pkts_matched, pkts_forwarded, pkts_dropped; the rest as upe_counters_t defines them).
     * ctx is NULL while a later batch is still on the GPU: the context's statistics then already
     * hold some packets the counters do not, so publish the counters only (and never call into
     * the context, which would wait for that batch).  ctx is the context when nothing is in
     * flight — after a drain (empty ring, a table-writing packet, a polled change) and at least
     * every 32 batches of a stream that never drains — and upe_gpu_get_stats(ctx, ...) then
     * matches the counters packet for packet (rule_stats packets sum to pkts_matched). */
    void (*publish)(void *user, upe_gpu_ctx_t *ctx, const upe_counters_t *counters);
    /* optional: the handles of a burst's forwarded frames after its tx_send_batch, in one call
     * (else free_buf on each; src/worker.c:300-302 frees them one by one) */
    void (*free_burst)(void *user, void *const *bufs, unsigned count);
} upe_worker_ops_t;

typedef struct {
    size_t batch;       /* most packets per GPU batch (0 = 65536) */
    unsigned burst;     /* most handles per pop (0 = 32, WORKER_BURST_SIZE; at most 64) */
    /* NULL: each packet's first UPE_HDR_WINDOW bytes are copied into pinned staging and
     * classified there by upe_gpu_process_mapped_emit (the kernel reads the windows over the
     * link; no DMA copies), the verdicts and records written to pinned host memory (records
     * applied to the buffers in the walk).  Non-NULL: every buffer's frame lies at
     * pool_base + a multiple of 16, inside memory registered with upe_gpu_host_register (e.g.
     * the reference's pktbuf pool), and each batch is classified where it lies by
     * upe_gpu_process_mapped_emit (nothing copied; the records, written to pinned host memory,
     * applied to the buffers in the walk). */
    uint8_t *pool_base;
    unsigned idle_ns;   /* sleep when the ring is empty and nothing is held (0 = 1000, as
                           src/worker.c:274-277) */
    size_t pool_bytes;  /* with pool_base: the registered region's size; a frame whose bytes
                           (at least UPE_FRAME_TAIL of them, what the kernel may read) do not lie
                           inside it stops the loop with an error instead of reaching the GPU */
} upe_worker_cfg_t;

/* The GPU-backed replacement of worker_main (reference src/worker.c:255-307), on the calling
 * thread, until the ring is empty with ops->stop() set.  Pops bursts and gathers them into GPU
 * batches, classified by the context's tables; a batch is cut after every packet that writes a
 * neighbour table (ARP, NS/NA), whose write is applied through ops before the next packet is
 * classified, and also run at once whenever the ring is empty.  Then, per popped burst and in
 * packet order, exactly the calls worker_main makes: tx_send of each answered ARP request,
 * free_buf of each dropped or consumed packet (pkts_dropped += 1 for a drop), and one
 * tx_send_batch of the burst's forwarded frames (rewritten as process_packet leaves them) with
 * pkts_forwarded += sent, pkts_dropped += count - sent, and free_buf of each.  *counters
 * (optional) receives the loop's counters at the end (they start from zero).  0, or -1 on a
 * GPU, callback or argument error (upe_gpu_last_error()). */
int upe_gpu_worker_run(upe_gpu_ctx_t *ctx, const upe_worker_ops_t *ops, void *user,
                       const upe_worker_cfg_t *cfg, upe_counters_t *counters);

/* Pinned (page-locked) host memory for upe_gpu_process_host() batches; the GPU can also read and
 * write it directly (upe_gpu_process_mapped). */
void *upe_gpu_host_alloc(size_t bytes);
int upe_gpu_host_free(void *ptr);

/* Page-lock an existing host buffer and map it for the GPU (e.g. the reference's pktbuf pool,
 * src/pktbuf.c: pool->mem), so that upe_gpu_process_mapped() can classify its frames where they
 * lie.  `ptr` and `bytes` need no alignment.  0 / -1. */
int upe_gpu_host_register(void *ptr, size_t bytes);
int upe_gpu_host_unregister(void *ptr);

/* The batch in host memory, classified by the kernel's own loads over the link: no DMA copies and
 * no staging slots.  The kernel reads each frame's header window and its descriptor from host
 * memory and writes the verdicts (and in place: the rewritten header bytes, exactly as
 * upe_gpu_process() does in HBM; emit: the 16-byte records) straight into host memory, so only
 * the bytes the path touches cross the link — for long frames a fraction of the frame span the
 * DMA round trip must copy.  Every pointer is host memory from upe_gpu_host_alloc() or
 * upe_gpu_host_register() (checked: -1 otherwise); layout and UPE_FRAME_TAIL rule as for
 * upe_gpu_process().  Asynchronous on `stream` like upe_gpu_process(): the outputs are the
 * host's to read after upe_gpu_sync().  This replaces the worker's burst loop over pktbufs in the
 * pool (src/worker.c:255-307) with nothing copied: the frames are rewritten where tx_send reads
 * them (src/tx_afpacket.c:60-76). */
int upe_gpu_process_mapped(upe_gpu_ctx_t *ctx, uint8_t *h_frames, const uint64_t *h_desc,
                           uint32_t *h_verdict, size_t n, void *stream);
int upe_gpu_process_mapped_emit(upe_gpu_ctx_t *ctx, uint8_t *h_frames, const uint64_t *h_desc,
                                uint32_t *h_verdict, upe_hdr_rec_t *h_hdr, size_t n,
                                void *stream);

/* Queue `count` batches back to back from native code: batch k is d_frames_list[k] (a host
 * array of device pointers), all sharing one descriptor array and one verdict array (each batch
 * overwrites the verdicts of the one before).  Equivalent to `count` upe_gpu_process() calls,
 * without a caller round trip per batch; what a GPU-backed worker thread does with a ring of
 * resident batch buffers. */
int upe_gpu_process_batches(upe_gpu_ctx_t *ctx, uint8_t *const *d_frames_list,
                            const uint64_t *d_desc, uint32_t *d_verdict, size_t n, size_t count,
                            void *stream);
/* The same in emit mode (every batch writes its records to d_hdr): upe_gpu_process_queue_emit()
 * over `count` batches that share d_desc, d_verdict and d_hdr. */
int upe_gpu_process_batches_emit(upe_gpu_ctx_t *ctx, uint8_t *const *d_frames_list,
                                 const uint64_t *d_desc, uint32_t *d_verdict,
                                 upe_hdr_rec_t *d_hdr, size_t n, size_t count, void *stream);

/* One resident batch of a queue: device frames, descriptors, verdicts and records, n packets. */
typedef struct upe_gpu_batch {
    uint8_t *frames;
    const uint64_t *desc;
    uint32_t *verdict;
    upe_hdr_rec_t *hdr;
    size_t n;
} upe_gpu_batch_t;

/* The worker loop (reference src/worker.c:255-307: burst after burst, the worker's state carried
 * from one to the next) over `count` resident batches in emit mode, one launch per batch queued
 * from native code on `stream`.  Results — every verdict, record, counter, rule_stats word and
 * the L1 state — equal `count` upe_gpu_process_emit() calls in order; batches may differ in size
 * (an empty one is a no-op) and may share descriptor and output buffers.  Every batch is
 * checked (a batch of n > 0 packets needs its records) before any is queued.  0 / -1. */
int upe_gpu_process_queue_emit(upe_gpu_ctx_t *ctx, const upe_gpu_batch_t *batches, size_t count,
                               void *stream);

/* upe_gpu_process() plus software RSS in the same pass (reference src/rx_pcap.c:67-77 parses
 * every packet a second time on the RX thread for this): d_flow_hash[i] (device, n uint32) =
 * flow_hash() of the packet's flow key (src/parser.c:113-135) when parse_flow_key succeeds, 0
 * otherwise (verdict code DROP_PARSE or CONSUMED says which).  A caller spreading a capture over
 * workers takes hash & (workers - 1), as the reference's RX thread does. */
int upe_gpu_process_rss(upe_gpu_ctx_t *ctx, uint8_t *d_frames, const uint64_t *d_desc,
                        uint32_t *d_verdict, uint32_t *d_flow_hash, size_t n, void *stream);

/* Egress list: d_index[0..*d_count) = the indexes i < n whose verdict code is `code` (e.g.
 * UPE_V_FWD), in packet order — the order process_packet queues frames for tx_send_batch
 * (reference src/worker.c:240-243, 287-303).  Device buffers; d_index holds n entries. */
int upe_gpu_compact(upe_gpu_ctx_t *ctx, const uint32_t *d_verdict, size_t n, uint32_t code,
                    uint32_t *d_index, uint64_t *d_count, void *stream);

/* upe_gpu_process_emit() plus the egress list in the same pass, with no second kernel (round 6):
 * the forwarded packets of group g (packets 64g .. 64g + 63) are d_tx[64g .. 64g + d_tx_count[g])
 * in packet order — the order process_packet queues frames for tx_send_batch (reference
 * src/worker.c:240-243, 287-303) — and d_tx[64g + k] is the packet whose record is d_hdr[64g + k]
 * (the records' UPE_HDR_SLOT layout).  The groups concatenated are exactly upe_gpu_compact(...,
 * UPE_V_FWD, ...)'s list; upe_tx_flush_groups() makes the reference worker's TX calls from it
 * directly.  Device buffers: d_tx holds n entries, d_tx_count (n + 63) / 64; slots past a group's
 * count are not written.  0 / -1. */
int upe_gpu_process_emit_tx(upe_gpu_ctx_t *ctx, uint8_t *d_frames, const uint64_t *d_desc,
                            uint32_t *d_verdict, upe_hdr_rec_t *d_hdr, uint32_t *d_tx,
                            uint32_t *d_tx_count, size_t n, void *stream);

/* A batch with exact control-packet semantics, as the reference's burst loop runs it
 * (src/worker.c:23-104 inside process_packet): an ARP packet with the Ethernet/IPv4 header, or
 * an NDP NS/NA carrying a link-layer address option, writes a neighbour table, and every later
 * packet sees the new entry.  The batch is cut after each such packet: the segment up to and
 * including it runs as upe_gpu_process(), its write — arp_update(spa, sha)
 * (src/arp_table.c:26-53) or ndp_update(src | target, lladdr) (src/ndp_table.c:39-65, option
 * walk src/worker.c:68-95) — is applied to the caller's host slot arrays `arp` / `ndp` (the
 * ones last given to upe_gpu_load_neigh; updated in place, update_at = now, as the reference's
 * tables are), the new snapshot is uploaded, and the next segment runs.  Control packets are
 * found on the device (one marking pass plus an ordered compaction), so a batch without them
 * costs one extra pass.  Synchronous; *n_writes (optional) = table writes applied.  Capacities
 * are powers of two, as arp_table_init / ndp_table_init require.  The NS/NA option walk reads
 * the whole frame (len bytes), so this call needs FULL frames: a batch of UPE_FRAME_TAIL-byte
 * header windows (upe_gpu_process_host's window form) is not valid here — an NS/NA longer than
 * its window would have its options read from the bytes that follow the window. */
int upe_gpu_process_segmented(upe_gpu_ctx_t *ctx, uint8_t *d_frames, const uint64_t *d_desc,
                              uint32_t *d_verdict, size_t n, upe_arp_entry_t *arp,
                              size_t arp_capacity, upe_ndp_entry_t *ndp, size_t ndp_capacity,
                              int64_t now, size_t *n_writes, void *stream);

/* Wait for all work queued on the context's stream (or `stream`). */
int upe_gpu_sync(upe_gpu_ctx_t *ctx, void *stream);

/* Summary of the most recent upe_gpu_process() (synchronises). */
int upe_gpu_batch_info(upe_gpu_ctx_t *ctx, upe_batch_info_t *info);

/* How the most recent classify launch ran (synchronises; diagnostics and tests).  A launch that
 * starts from an L1 entry disagreeing with its table resolves the packets aimed at that entry by
 * a bounded look-back; a wave that stops waiting (a workgroup it needs is not resident yet)
 * defers them, and the launch's last workgroup answers them. */
typedef struct {
    uint32_t variant;  /* kernel variant: bit 0 emit, 1 tuple space, 2 lean, 3 no look-back,
                          4 ring (stamped), 5 a host path (upe_gpu_process_mapped / _host),
                          6 a linear-scan table past 64 rules (per-family rule lists),
                          7 the same scanned whole */
    uint32_t grid;     /* workgroups of the launch */
    uint32_t deferred; /* (chunk, family) entries whose look-back was deferred to the last
                          workgroup (0 when the look-back was not live) */
    uint64_t launches; /* classify launches of this context so far */
} upe_launch_info_t;
int upe_gpu_launch_info(upe_gpu_ctx_t *ctx, upe_launch_info_t *info);

/* Accumulated worker counters and rule_stats[0..capacity) (synchronises). */
int upe_gpu_get_stats(upe_gpu_ctx_t *ctx, upe_counters_t *counters, upe_rule_stat_t *rule_stats,
                      size_t capacity);
int upe_gpu_reset_stats(upe_gpu_ctx_t *ctx);

/* Kernel timing.  enable = k > 0: every k-th upe_gpu_process() call (calls k/2, k/2 + k, ...
 * after enabling: not the first, which starts from an idle queue) records HIP events on its
 * stream around its launches (classify, plus the rule_stats group-by
 * pass of tables over 4096 rules); sampling keeps the events' own queue cost out of a throughput
 * run.  enable = 0 turns timing off.  upe_gpu_timing_span(ctx, every, span): each sample's
 * event pair brackets `span` consecutive calls instead of one, so the events' own latency is
 * spread over `span` launches (the time then includes the gaps between those launches).
 * upe_gpu_timing_read() synchronises and returns the summed time (ms) of the closed samples and
 * the number of calls they cover: classify_ms up to the end of each sample's last classify
 * launch, finalize_ms from there to the end of its rule_stats group-by (0 for tables of up to
 * 4096 rules, which have none). */
int upe_gpu_timing_enable(upe_gpu_ctx_t *ctx, int enable);
int upe_gpu_timing_span(upe_gpu_ctx_t *ctx, int every, int span);
int upe_gpu_timing_read(upe_gpu_ctx_t *ctx, double *classify_ms, double *finalize_ms,
                        uint64_t *launches);

/* Device memory helpers so a C caller needs no HIP headers. */
void *upe_gpu_malloc(upe_gpu_ctx_t *ctx, size_t bytes);
int upe_gpu_free(upe_gpu_ctx_t *ctx, void *dptr);
int upe_gpu_memcpy_h2d(upe_gpu_ctx_t *ctx, void *dst, const void *src, size_t bytes, void *stream);
int upe_gpu_memcpy_d2h(upe_gpu_ctx_t *ctx, void *dst, const void *src, size_t bytes, void *stream);

/* ------------------------------------------------------------------------------------------ */
/* Host-side batch builders (upe_amd/csrc/upe_host.c, C)                                      */
/* ------------------------------------------------------------------------------------------ */

/* Load a rule file in the reference's INI format (reference src/rule_config.c:129-282,
 * rules.example) into rules[0..capacity) as rule_table_init(capacity) + rule_config_load would
 * leave rt->rules: rule_id = insertion index, wildcard addresses zeroed, sorted by
 * (priority, rule_id) (src/rule_table.c:130-161).  *count = rules loaded.  0 / -1 (the message,
 * with the reference's "rules:<line>: ..." wording, in upe_host_last_error()). */
int upe_rules_load_ini(const char *path, upe_rule_t *rules, size_t capacity, size_t *count);

/* A pcap capture (LE/BE, usec/nsec, link type Ethernet) -> the packed batch layout above, in
 * record order, as reference src/rx_pcap.c:42-93 admits packets: records with caplen > 2048
 * (PKTBUF_DATA_SIZE) are dropped.  Call with frames = desc = NULL to size the buffers
 * (info->packets descriptors, info->frames_bytes bytes including the UPE_FRAME_TAIL), then again
 * to fill them.  0 / -1. */
typedef struct {
    uint64_t records;          /* records in the file */
    uint64_t packets;          /* packets in the batch */
    uint64_t dropped_oversize; /* caplen > 2048: dropped by RX, never reach the worker */
    uint64_t frames_bytes;     /* frames buffer size needed */
} upe_pcap_info_t;
int upe_pcap_read(const char *path, uint8_t *frames, size_t frames_cap, uint64_t *desc,
                  size_t desc_cap, upe_pcap_info_t *info);

/* Last error of the host-side builders on this thread ("" if none). */
const char *upe_host_last_error(void);

#ifdef __cplusplus
}
#endif

/* Layout checks against the reference (LP64). */
#ifdef __cplusplus
#define UPE_STATIC_ASSERT static_assert
#else
#define UPE_STATIC_ASSERT _Static_assert
#endif
UPE_STATIC_ASSERT(sizeof(upe_gpu_batch_t) == 40, "upe_gpu_batch_t layout");
UPE_STATIC_ASSERT(sizeof(upe_flow_key_t) == 44, "flow_key_t layout");
UPE_STATIC_ASSERT(offsetof(upe_flow_key_t, dst_ip) == 20, "flow_key_t.dst_ip");
UPE_STATIC_ASSERT(offsetof(upe_flow_key_t, protocol) == 40, "flow_key_t.protocol");
UPE_STATIC_ASSERT(sizeof(upe_rule_t) == 92, "rule_t layout");
UPE_STATIC_ASSERT(offsetof(upe_rule_t, src_ip) == 8, "rule_t.src_ip");
UPE_STATIC_ASSERT(offsetof(upe_rule_t, dst_mask) == 56, "rule_t.dst_mask");
UPE_STATIC_ASSERT(offsetof(upe_rule_t, src_port) == 72, "rule_t.src_port");
UPE_STATIC_ASSERT(offsetof(upe_rule_t, protocol) == 76, "rule_t.protocol");
UPE_STATIC_ASSERT(offsetof(upe_rule_t, action) == 80, "rule_t.action");
UPE_STATIC_ASSERT(offsetof(upe_rule_t, rule_id) == 88, "rule_t.rule_id");
UPE_STATIC_ASSERT(sizeof(upe_arp_entry_t) == 32, "arp_entry_t layout");
UPE_STATIC_ASSERT(offsetof(upe_arp_entry_t, valid) == 24, "arp_entry_t.valid");
UPE_STATIC_ASSERT(sizeof(upe_ndp_entry_t) == 40, "ndp_entry_t layout");
UPE_STATIC_ASSERT(offsetof(upe_ndp_entry_t, valid) == 32, "ndp_entry_t.valid");
UPE_STATIC_ASSERT(sizeof(upe_rule_stat_t) == 16, "rule_stat_t layout");
UPE_STATIC_ASSERT(sizeof(upe_hdr_rec_t) == 16, "upe_hdr_rec_t layout");
UPE_STATIC_ASSERT(sizeof(upe_launch_info_t) == 24, "upe_launch_info_t layout");

#endif /* UPE_GPU_H */
