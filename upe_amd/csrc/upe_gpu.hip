// upe_gpu.hip — MI355X (gfx950 / CDNA4) batch dataplane for UPE's per-packet worker hot path,
// and the extern "C" ABI declared in include/upe_gpu.h.
//
// One lane owns one packet.  Per packet the kernel does what reference process_packet() does
// (src/worker.c:106-253): control-packet classification (src/worker.c:23-104), the fixed-format
// parse (src/parser.c:6-111), first-match over the priority-sorted rule table
// (src/rule_table.c:76-91,163-176), counters and rule_stats (src/worker.c:119-153), and the
// L3-forward rewrite: TTL / hop-limit decrement, RFC 1071 checksum (src/parser.c:137-169), and the
// next-hop MAC that arp_get_mac / ndp_get_mac would return (src/arp_table.c:55-80,
// src/ndp_table.c:6-17,67-86).  The rewritten header bytes go either to a 16-byte record per
// packet (emit mode, frames only read) or into the frames in place.
//
// Data layout: frames packed back to back at 16-byte aligned starts, one uint64
// descriptor per packet (offset << 16 | len), one uint32 verdict per packet, and in emit mode one
// upe_hdr_rec_t per packet.  A lane loads the first 80 bytes of its frame as 16-byte vector
// loads issued together (chunks past len are not loaded; the batch buffer carries a 96-byte
// tail, so the last frame's window is readable).
//
// Fast path: option-less IPv4 (first byte 0x45, len >= 34) and IPv6 (len >= 54), which covers
// every well-formed packet of the benchmark configurations, is parsed branch-free from those
// registers; everything else (ARP, IPv4 options, truncated or foreign frames) takes the general
// path, entered only by waves that hold such a packet.
//
// The rule table is compiled into structure-of-arrays streams that a wave scans with
// wave-uniform loads (LDS for small tables, the scalar unit otherwise), so rule operands arrive
// in SGPRs; the per-rule work is a few VALU xor / and-or against them, with an early exit as soon
// as every lane of the wave has its first match (ballot).  Large tables go through a tuple-space
// index instead.
//
// One launch per batch, one persistent 1024-thread workgroup per CU (the grid is what a
// residency census finds the chip holds at once).  Workgroup b owns 1024-packet tiles b,
// b + grid, ...; its 16 waves claim the tiles' 64-packet chunks from an LDS counter, so they
// finish together.  A wave loads its next chunk's descriptors as it starts a chunk and (emit
// mode) issues that chunk's window loads halfway through, after the rule match.  Counters, the rule_stats histogram and the L1 bookkeeping accumulate in LDS
// (ballots per chunk) and leave once per workgroup, as one device-atomic instruction per kind,
// into replicated per-batch accumulators.  Nothing waits for anything at the end of a launch:
// the next launch folds this batch's accumulators (lazy fold), the host reads them after a
// synchronisation (upe_l1_sync folds the last one).
//
// Neighbour lookups answer arp_get_mac / ndp_get_mac exactly without walking the reference's
// linear-probe chains: at upload the host keeps only the entries a reference probe can reach
// (probe from the home slot, first valid match before the first invalid slot) and places them
// by three-choice cuckoo hashing; every answer equals the reference's for the snapshot and a
// lookup is three independent LDS reads (indexes of up to 2048 slots are staged) or one memory
// round trip.
//
// The worker's one-entry L1 neighbour caches are sequential state (src/worker.c:186-195,
// 218-225), emulated exactly.  If the starting L1 entry agrees with the
// table (the steady state), every packet's answer is the table's and the only sequential output
// is the final L1 entry: the last table hit, if any packet missed the starting entry and hit the
// table.  If it disagrees (after a table change, or the calloc'd NDP entry for ::), a packet
// whose destination equals the starting entry takes the entry's MAC iff no earlier packet missed
// the entry and hit the table: each 64-packet chunk publishes whether it holds such a packet,
// and a chunk with candidates looks back over the chunks before it (decoupled look-back).
#include <hip/hip_runtime.h>
#include <ctype.h>
#include <pthread.h>
#include <sched.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <deque>
#include <map>
#include <atomic>
#include <new>
#include <string>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/upe_gpu.h"

namespace {

#ifndef UPE_BLOCK
#define UPE_BLOCK 1024
#endif
constexpr int kBlock = UPE_BLOCK;      // threads per workgroup = packets per tile
constexpr int kWaves = kBlock / 64;    // 64-packet chunks per tile
constexpr int kTile = kBlock;

#ifndef UPE_WAVES_PER_SIMD
#define UPE_WAVES_PER_SIMD 4
#endif
constexpr int kWavesPerSimd = UPE_WAVES_PER_SIMD;   // 4 -> VGPR budget 128, 8 -> 64
constexpr int kUnroll = 4;             // rules per early-exit check (rule table padding unit)
constexpr uint32_t kNone = 0xFFFFFFFFu;
#ifndef UPE_LDS_STATS_MAX
#define UPE_LDS_STATS_MAX 4096
#endif
constexpr int kLdsStatsMax = UPE_LDS_STATS_MAX;   // rule_stats in the classify kernel's LDS up to here
constexpr int kStatReps = 8;   // replicas of the per-sorted-index rule_stats (summed on the host)
// Claim the next chunk after finishing the current one once this few chunks are unclaimed.
#ifndef UPE_LATE_CLAIM
#define UPE_LATE_CLAIM 16
#endif
constexpr uint32_t kLateClaim = UPE_LATE_CLAIM;
// Issue the next chunk's window loads in the middle of the current chunk (after its rule
// match), so that they fly during the rest of it: bit 0 emit-mode linear-scan kernel, bit 1 also
// the in-place one, bit 2 also the tuple-space ones (config B emit 26.2 -> 25.4 us per 1M batch;
// C unchanged; in place +0.3 % with a VGPR spilled, so off; tuple space: D unchanged, with twice
// the SGPR spills, so off; issued right after the parse instead: B no gain, C 39.0 -> 40.5).
#ifndef UPE_MID_PREFETCH
#define UPE_MID_PREFETCH 1
#endif
// Neighbour indexes staged in LDS (one workgroup per CU, so a CU reads them once per launch):
// ARP up to 2048 slots (32 KB), NDP up to 2048 slots (64 KB), within kLdsDynMax of dynamic LDS.
#ifndef UPE_ARP_LDS_SLOTS
#define UPE_ARP_LDS_SLOTS 2048
#endif
#ifndef UPE_NDP_LDS_SLOTS
#define UPE_NDP_LDS_SLOTS 2048
#endif
constexpr uint32_t kArpLdsSlots = UPE_ARP_LDS_SLOTS;
constexpr uint32_t kNdpLdsSlots = UPE_NDP_LDS_SLOTS;
constexpr size_t kLdsDynMax = 152 * 1024;   // 160 KB per CU less the static LDS (7 KB at most)
// kernels for linear tables past kSmallRules (family lists, whole-table scan, decision tree) keep
// no small-table copy in static LDS (~1 KB static): 158 KB for their dynamic LDS
constexpr size_t kLdsDynMaxLarge = 158 * 1024;
constexpr int kSmallRules = 64;        // up to here rule_stats go through replicated accumulators
constexpr int kReps = 32;              // replicas of the per-batch accumulators
constexpr int kRingMax = 64;           // batches of a ring launch whose completion is stamped
// Cache policy of the emit-mode record store: sc1 (buffer aux 16) writes the records through
// and drops their lines from the XCD's L2, so the end of a launch has ~16 MB less dirty data to
// write back at the kernel boundary (config B 24.5 -> 24.1 us per 1M batch; nt 24.5, sc0 sc1
// 24.2).  The verdict words are written through too (B 24.25 -> 24.1 us); the in-place 16-byte
// header stores are not (written through they were slower: 33.7 -> 35.4 us, partial lines).
constexpr int kRecAux = 16;

// ---- compiled rule table (built by upe_gpu_load_rules) --------------------------------------
// rv4[i]: header + first address word, used for every packet:
//   x0 = ip_ver | proto << 8 | src_port << 16 and its wildcard mask m0
//   x1 = dst_port and mask m1; m1 bit 31 (x1 bit 31 clear, so it never decides a match) marks a
//   rule with IPv6 address words, the only rules an IPv6 key must test against rv6; x1 bits
//   16-17 (m1 bits 16-30 clear) carry the action code (0 drop, 1 forward, 2 any other type),
//   so the scan hands the matched rule's action over with its index
//   s0/sm0, d0/dm0: union bytes 0-3 of src/dst as LE u32 (the v4 view, rule_t.src_ip.v4),
//   pre-masked so a match is ((key ^ x) & m) == 0 for every pair.
// rv6[i]: union words 1-3 of src/dst (pre-masked) and masks, used only by IPv6 packets.
// rinfo[i]: (action.type, rule_id).
struct __attribute__((aligned(16))) RuleV4 {
    uint32_t x0, m0, x1, m1, s0, sm0, d0, dm0;
};
constexpr uint32_t kRuleV6Words = 0x80000000u;
struct __attribute__((aligned(16))) RuleV6 {
    uint32_t s[3], sm[3], d[3], dm[3], pad[4];
};
// FamTable (linear-scan tables past the LDS size): the rules an IPv4 key can match (ip_ver 4 or
// 0) and those an IPv6 key can match (6 or 0), each list in priority order, so that a lane walks
// only its own family's list — a wave's scan lasts as long as its deepest lane's position in its
// family's list, not in the whole table.  Image: fam4 RuleV4, then fam6 (RuleV4, RuleV6) pairs,
// then the lists' sorted indexes (u32, fam4 then fam6); padding entries never match.  An IPv6
// entry is 80 bytes: the RuleV4 words, then RuleV6's s[3] sm[3] d[3] dm[3].  When the IPv6 list
// fits beside the launch's other LDS data it is staged there (Args::fam6_lds): an IPv6 lane's
// scan, the deep one in mixed tables, then reads LDS instead of the scalar cache.
constexpr uint32_t kFamV6Stride = 5;   // uint4 per IPv6 entry
#ifndef UPE_FAM_LDS
#define UPE_FAM_LDS 1
#endif
constexpr bool kFamLds = UPE_FAM_LDS;

// L1 state in word form + whether each entry agrees with the current neighbour snapshot.
// DevState keeps two, by batch parity (see "Sequential state between batches").
struct DevL1 {
    uint32_t arp_ip, arp_mac_lo, arp_mac_hi;
    uint32_t ndp_ip[4];
    uint32_t ndp_mac_lo, ndp_mac_hi;
    uint32_t arp_ok, ndp_ok;
    uint32_t pad[5];
};

// ---- Sequential state between batches ------------------------------------------------------
// Nothing is folded at the end of a launch (no last-workgroup fold, no grid-wide wait): every
// workgroup adds what it saw into replicated accumulators (replica = workgroup % kReps) and the
// NEXT launch, in its first instructions, folds the previous batch's L1 outcome into the state
// it starts from.  Batch k (the context's k-th launch) uses
//   l1[k % 2]       the L1 state after batch k - 2 (read)
//   acc[(k - 1) % 3] batch k - 1's minima / maxima and pay[(k - 1) % 2] its last-hit payloads
//                    (read: every workgroup folds them into its own starting L1 entry)
//   l1[(k + 1) % 2] the state after batch k - 1 (written by workgroup 0, for batch k + 1)
//   acc[k % 3]      this batch's accumulators, pay[k % 2] its payloads (written)
//   acc[(k + 1) % 3] re-armed by workgroup 0 for batch k + 1
// Host calls that read or replace the L1 state first fold the pending batch the same way
// (upe_l1_sync).  Batch k's counters are folded into the cumulative totals by batch k + 1
// (workgroups 0..7, one counter each); rule_stats go straight into replicated per-sorted-index
// totals, which the host sums when it reads them.  No workgroup ever waits for another.
enum { C_PARSED, C_MATCHED, C_FWD, C_DROPPED, C_CONSUMED, C_ARP_LEARN, C_ARP_REPLY, C_CTRL, C_N };
// l1r words, all combined with atomicMax (minima stored as kNone - x, so "none" is 0)
enum { R_F4, R_F6, R_M4, R_M6, R_N };
struct __attribute__((aligned(128))) BatchAcc {
    uint32_t cnt[kReps][C_N];              // this batch's counters
    unsigned long long l1r[kReps][R_N];    // R_F4 / R_F6: kNone - first miss-then-hit index
                                           // v4 / v6; R_M4 / R_M6: last table hit v4 / v6 as
                                           // (index + 1) << 32 | the workgroup holding its payload
    uint32_t ctrl[kReps];                  // kNone - first control packet (max)
    uint32_t grid;                         // the batch's grid
    uint32_t n;                            // the batch's size
    uint32_t pad0[30];
    // look-back give-ups (a launch that started from a disagreeing L1 entry): workgroups that have
    // finished, deferred (chunk, family) entries, and "some wave gave up" (later waves then wait
    // only briefly for an unpublished flag).  A line of their own: the launch polls them.
    uint32_t done, ndefer, giveup;
    uint32_t pad[29];
};
// Payload of a workgroup's last table hit per family; the next batch reads the one the batch
// maximum points at.
struct __attribute__((aligned(64))) TilePay {
    uint32_t m4_dst, m4_mac_lo, m4_mac_hi;
    uint32_t m6_dst[4], m6_mac_lo, m6_mac_hi;
    uint32_t pad[7];
};
constexpr int kPayWords = 9;
// Look-back flags (one word per 64-packet chunk: a wave's share of a tile), written only while
// a starting L1 entry disagrees with the table: launch tag << 6 | bits.  A packet the starting
// entry may answer needs to know whether any earlier packet of its family missed the entry and
// hit the table; its wave looks back over the earlier chunks' flags (decoupled look-back).
enum { LB_FP4 = 1, LB_FP6 = 2, LB_KNOWN4 = 4, LB_INCL4 = 8, LB_KNOWN6 = 16, LB_INCL6 = 32 };
constexpr uint32_t kLbTagMod = 0x3FFFFFFu;   // tags 1 .. kLbTagMod

// Everything a batch reads or writes besides the packets and the tables, in one device
// allocation.  One L1 state slot per 128-byte line.
struct __attribute__((aligned(128))) L1Slot {
    DevL1 s;
};
struct DevState {
    L1Slot l1[2];
    BatchAcc acc[3];
    unsigned long long totals[8];                           // cumulative, upe_counters_t order
    unsigned long long acc_stats[kReps][2 * kSmallRules];   // small tables, per sorted index
    uint32_t census[32];                                     // residency census (census_probe)
    TilePay* pay;                    // [grid]
    uint32_t* lb;                    // look-back flags, one per 64-packet chunk
    unsigned long long* stats;       // [cap][2] worker rule_stats (mid-size and large tables)
    unsigned long long* stats_idx;   // [kStatReps][nrules_pad][2] totals per sorted index
};

// Neighbour index (built by upe_gpu_load_neigh): the entries a reference probe reaches, placed
// by three-choice cuckoo hashing, so that every key sits in one of its three candidate slots.
//   ARP slot: uint4 {ip, mac0..3, mac4..5 | used << 16, 0}
//   NDP slot: 2 x uint4 {ip words 0..3}, {mac0..3, mac4..5 | used << 16, 0, 0}
struct NeighIndex {
    const uint4* t;
    uint32_t bits;   // log2(slots); 0 = empty
    uint32_t seed;
};

// Tuple-space index of a large rule table (built by upe_gpu_load_rules when it pays): the rules
// a packet family can match are grouped by mask signature; a group's cuckoo table maps the
// masked key to the smallest sorted index with that key.  Group descriptor words:
//   [0] m0 (proto, src_port masks)  [1] m1 (dst_port mask)  [2] src word-0 mask
//   [3] dst word-0 mask  [4..6] src words 1-3 masks  [7..9] dst words 1-3 masks (family 6)
//   [10] smallest sorted index in the group  [11] log2(slots)  [12] seed  [13] first slot
//   [14] 1 | action << 8 when every mask word is zero (a catch-all group: every packet of the
//        family matches its one key, so the probe needs no memory access), else 0
//   [15] 1 + offset of the group's fingerprints in the staged image (tfs), 0 = not staged
// Slots: family 4 = 2 x uint4 {k0, k1, s0, d0}, {index, used, -, -};
//        family 6 = 3 x uint4 {k0, k1, s0, s1}, {s2, s3, d0, d1}, {d2, d3, index, used}.
struct __attribute__((aligned(16))) TssGroup {
    uint32_t w[16];
};
// An IPv4 slot is one uint4: the masked key's free bits carry the rest — k0's low byte (the IP
// version, never part of a group's mask) and k1's high half (above the 16-bit destination port)
// hold v = (index + 1) | action << 22 (0 = empty slot), so a probe is one 16-byte load, one
// memory request (two loads into one line were two requests: tools/fetch_calib), and the IPv4
// slot array takes half the L2 (config D 755 -> 716 us per 16M against 32-byte slots).
constexpr int kTssSlot4 = 1, kTssSlot6 = 3;   // uint4 per slot
constexpr uint32_t kTssMaxRules = 1u << 22;   // index + 1 in 22 bits, the action above it
// Fingerprints of small groups staged in LDS (word [15] of such a group: 1 + its offset in the
// staged image): their probes then wait for no fingerprint round trip.
constexpr uint32_t kFpStageMax = 8192;     // staged fingerprints (2 bytes each)
constexpr uint32_t kFpStageGroup = 4096;   // largest group (slots) staged
// Groups whose fingerprints are not staged are probed without them: slot t1 (where cuckoo
// placement leaves ~80 % of the keys at this load), then t2 if t1 holds another key.  One round
// trip for most hits instead of a fingerprint trip followed by a slot trip (config D 808 -> 775
// us); a miss takes two slot reads.
constexpr uint32_t kTssRatioX2 = 5;   // tuple-space slots >= ratio / 2 x keys

// Decision-tree index of a linear-scan table past kSmallRules (round 5; built by
// upe_gpu_load_rules when the tuple-space index does not apply).  The family lists (FamTable)
// stay the rules; each list gets a binary tree over the key's words, HyperSplit-style: an inner
// node compares one key word with a threshold, a leaf lists the positions of the rules whose
// conservative range meets the leaf's box (lo = x & m, hi = x | ~m per word), in list order, cut
// after the first one that matches every key of the box (flagged: it needs no test).  A key's
// first match in (priority, rule_id) order is therefore the first of its leaf's rules that
// matches it (reference src/rule_table.c:163-176): a rule that can match the key meets the box,
// so it is listed, or the flagged rule precedes it and matches the key too.  A lane walks its
// family's tree (one node load per level) and tests a handful of rules, however deep its first
// match lies in the table — the wave-uniform scan lasted as long as the wave's deepest lane.
// Key words: 0-3 source address, 4-7 destination address (IPv6: the wire bytes as big-endian
// words, so that a prefix is a range; IPv4: word 0 host order as parse_flow_key stores it, the
// other words 0), 8 source port, 9 destination port, 10 protocol.
// The binary tree is built (build_tree_family), then packed two levels to a node, so that a walk
// step resolves two levels with one 16-byte load (the walk is a chain of dependent LDS loads):
//   node (uint4): {x, y, z, w}: x = dim P | dim L << 4 | dim R << 8 | P leaf << 12 | L leaf << 13 |
//                 R leaf << 14 | base << 15; y = P's threshold (P leaf: its leaf word); z / w =
//                 the threshold of P's left / right child L / R, or its leaf word.  A key word <
//                 threshold goes left.  L's children are nodes base, base + 1; R's follow them
//                 (base, base + 1 when L is a leaf).
//   leaf word: count << 21 | first entry
//   leaf entry (u32): list position | 0x80000000 when the rule matches every key of the leaf
// Each family's rules are split into groups by the key field on which each is narrowest, one
// tree per group (a rule narrow only in a port is then not copied into every leaf of a tree cut on
// addresses); a key's first match is the smallest of its first matches over its family's trees,
// else the family's rule that matches every key (build_forest_family).
// Image: a directory (node 0 = {IPv4 trees, IPv6 trees | byte orders << 16, IPv4 default answer,
// IPv6 default answer}), each tree's root node (IPv4 first), the other nodes, then the leaf
// entries; staged in LDS when it fits beside the launch's other LDS data.
constexpr int kTreeDims = 11;
constexpr int kTreeFields = 5;   // field trees per family (build_forest_family)
constexpr uint32_t kTreeBinth = 4;   // a node with more rules than this is split (if it can be)
constexpr size_t kTreeMinReach = 64;   // (load_rules_impl: tree or scan)

struct Args {
    uint8_t* frames;
    const uint64_t* desc;
    uint32_t* verdict;
    uint32_t n;
    const RuleV4* rv4;
    const RuleV6* rv6;
    const int2* rinfo;
    uint32_t nrules_pad;           // multiple of kUnroll, padding rules never match
    // per-family rule lists of a linear-scan table past the LDS size (FamTable comment)
    const uint4* fam;
    uint32_t fam4, fam6;           // entries per list, multiples of kUnroll
    uint32_t fam6_lds;             // the IPv6 list is staged in LDS (after the neighbour indexes)
    uint32_t fam4_lds;             // (tree kernels) the IPv4 list too, after the IPv6 one
    uint32_t fam_x1idx;            // tables below 8192 rules: each entry's x1 bits 18-30 carry its
                                   // sorted index (no index-array load after a match)
    // decision-tree index over the family lists (kTreeDims comment)
    const uint2* tree;             // nodes, then the leaf entries (u32) from word tree_loff
    uint32_t tree_loff;            // leaf entries' offset in u32 words
    uint32_t tree_lds;             // the image is staged in LDS (uint4 count), 0 = read from memory
    uint32_t port_mac_lo, port_mac_hi, port_ip4;
    NeighIndex arp, ndp;
    DevState* st;
    // tuple-space index (tss != 0): replaces the linear scan for large tables
    const TssGroup* tg4;
    const TssGroup* tg6;
    const uint4* tt4;
    const uint4* tt6;
    const uint4* tfs;              // staged fingerprint image (Args::fp_lds uint4 go to LDS)
    uint32_t ng4, ng6, tss;
    // the context's arrays, passed by value so that no kernel waits on a pointer load
    TilePay* pay;                    // [grid]
    unsigned long long* stats;       // [cap][2]
    unsigned long long* stats_idx;   // [kStatReps][nrules_pad][2]
    uint32_t arp_lds;                // ARP index staged in LDS (slots), 0 = read from memory
    uint32_t ndp_lds;                // NDP index staged in LDS (slots, 2 x uint4 each), 0 = not
    uint32_t fp_lds;                 // staged fingerprints in LDS (uint4 of tfs), 0 = none
    uint32_t* flow_hash;             // optional [n]: flow_hash of each parsed packet (RSS)
    void* gb;                        // optional [n]: what the rule_stats group-by reads beside
                                     // the verdicts (gb_packed: u32 keys, else u16 lengths)
    uint32_t gb_packed;              // 1: gb[i] = matched ? sorted rule index << 16 | len : 0
    uint4* hdr;                      // emit mode: [n] rewritten-header records (upe_hdr_rec_t)
    uint32_t* tx;                    // the egress-list kernels (kTx): group g's forwarded
    uint32_t* tx_cnt;                // packets tx[64g .. 64g + tx_cnt[g])
    uint32_t tx_base;                // the launch's first packet in the caller's batch (a batch
                                     // past kMaxLaunch runs as several launches)
    // this batch's slots of the between-batch state (DevState comment) follow from k6 = k % 6
    // (pointers computed where they are used: the kernel's scalar registers are scarce)
    uint32_t k6;
    uint32_t paycap;                 // a.pay[(k % 2) * paycap + workgroup]
    uint32_t census;                 // non-zero: a residency census launch (census_probe) only
    uint32_t* lb;                    // look-back flags, one per 64-packet chunk
    uint32_t lb_tag;                 // this launch's flag tag
    uint32_t tw;                     // chunks per tile (kWaves; fewer for small batches)
    uint32_t ntiles;                 // tiles of tw chunks
    unsigned long long* agree_out;   // host-mapped: (launch + 1) << 2 | start-state agreement bits
    unsigned long long launch_tag;   // this launch's index + 1
    uint32_t* defer;                 // deferred look-back candidates: (index | family << 31,
                                     // record slot) pairs
    uint32_t lb_spin;                // longest look-back wait, 100 MHz ticks (then defer)
    // ring launch (upe_gpu_process_ring_emit): batches of ring_cpb chunks each; per batch the
    // workgroups that have finished it, and the clock (10 ns) at which the last one did,
    // relative to the first workgroup's start (ring_t0)
    uint32_t ring_cpb, ring_mine;    // chunks per batch, and per batch and workgroup
    uint32_t* ring_wg;
    unsigned long long* ring_done;
    unsigned long long* ring_t0;
};
// Batch k's state slots, from Args (DevState comment).
__device__ __forceinline__ const DevL1* l1_in(const Args& a) { return &a.st->l1[a.k6 % 2].s; }
__device__ __forceinline__ DevL1* l1_out(const Args& a) { return &a.st->l1[(a.k6 + 1) % 2].s; }
__device__ __forceinline__ BatchAcc* acc_cur(const Args& a) { return &a.st->acc[a.k6 % 3]; }
__device__ __forceinline__ const BatchAcc* acc_prev(const Args& a) { return &a.st->acc[(a.k6 + 2) % 3]; }
__device__ __forceinline__ BatchAcc* acc_next(const Args& a) { return &a.st->acc[(a.k6 + 1) % 3]; }
__device__ __forceinline__ TilePay* pay_cur(const Args& a) {
    return a.pay + (size_t)(a.k6 % 2) * a.paycap;
}
__device__ __forceinline__ const TilePay* pay_prev(const Args& a) {
    return a.pay + (size_t)((a.k6 + 1) % 2) * a.paycap;
}

// ---- diagnostic timestamps (UPE_STAMPS builds only; never in the product build) ------------
#ifndef UPE_STAMPS
#define UPE_STAMPS 0
#endif
#if UPE_STAMPS
__device__ unsigned long long g_stamps[8192 * 16];
#define STAMP(k)                                                                              \
    do {                                                                                      \
        if (threadIdx.x == 0) {                                                               \
            unsigned long long t_;                                                            \
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");  \
            g_stamps[(blockIdx.x + ((a.lb_tag - 1u) % 4u) * 2048u) * 16 + (k)] = t_;                                             \
        }                                                                                     \
    } while (0)
#define STAMP_VM(k)                                                                           \
    do {                                                                                      \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                      \
        STAMP(k);                                                                             \
    } while (0)
// where the workgroup runs: slot 11 = XCC id, slot 12 = HW_ID (CU, SE, ...)
#define STAMP_WHERE()                                                                         \
    do {                                                                                      \
        if (threadIdx.x == 0) {                                                               \
            uint32_t x_, h_;                                                                  \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x_));                 \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(h_));                  \
            g_stamps[(blockIdx.x + ((a.lb_tag - 1u) % 4u) * 2048u) * 16 + 11] = x_;                                              \
            g_stamps[(blockIdx.x + ((a.lb_tag - 1u) % 4u) * 2048u) * 16 + 12] = h_;                                              \
        }                                                                                     \
    } while (0)
#else
#define STAMP_WHERE() do {} while (0)
#define STAMP(k) do {} while (0)
#define STAMP_VM(k) do {} while (0)
#endif

// ---- small helpers ------------------------------------------------------------------------
// Wave-wide reduction (K = 0 sum, 1 min, 2 max): DPP rotations inside each 16-lane row, then the
// four row results through scalar registers (no LDS, no shuffle round trips).
template <int K>
__device__ __forceinline__ uint32_t dpp_op(uint32_t x, uint32_t y) {
    return K == 0 ? x + y : K == 1 ? min(x, y) : max(x, y);
}
template <int K>
__device__ __forceinline__ uint32_t wave_reduce(uint32_t x) {
    x = dpp_op<K>(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xF, 0xF, false));
    x = dpp_op<K>(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x124, 0xF, 0xF, false));
    x = dpp_op<K>(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x122, 0xF, 0xF, false));
    x = dpp_op<K>(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x121, 0xF, 0xF, false));
    const uint32_t r0 = __builtin_amdgcn_readlane(x, 0), r1 = __builtin_amdgcn_readlane(x, 16);
    const uint32_t r2 = __builtin_amdgcn_readlane(x, 32), r3 = __builtin_amdgcn_readlane(x, 48);
    return dpp_op<K>(dpp_op<K>(r0, r1), dpp_op<K>(r2, r3));
}

__device__ __forceinline__ uint32_t byte_of(uint32_t w, int k) { return (w >> (8 * k)) & 0xFFu; }
__device__ __forceinline__ uint32_t at2(uint32_t hi, uint32_t lo) {   // dword at byte 4q+2
    return __builtin_amdgcn_alignbit(hi, lo, 16);
}
__host__ __device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
// Mask of the bytes of dword j that lie below len (a zero-filled pktbuf reads 0 past len).
__device__ __forceinline__ uint32_t len_mask(uint32_t len, int j) {
    const uint32_t lo = 4u * (uint32_t)j;
    return len >= lo + 4 ? 0xFFFFFFFFu : len <= lo ? 0u : (1u << (8 * (len - lo))) - 1u;
}
__device__ __forceinline__ uint32_t be16_lo(uint32_t x) {             // BE u16 in bytes 0,1
    return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu);
}
// RFC 1071 fold of a sum of native-LE u16 words held as a sum of u32 (u32 = lo + hi * 2^16,
// and 2^16 == 1 in one's-complement arithmetic), complemented: src/parser.c:137-169.
// v_bfi_b32 with a per-lane all-ones / all-zeros mask in a VGPR: a where m is set, else b (a
// select the compiler cannot turn into an indexed load of the array a and b come from, and one
// that needs no SGPR lane mask)
__device__ __forceinline__ uint32_t vsel(uint32_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ uint32_t csum_fold(unsigned long long sum) {
    uint32_t f = (uint32_t)(sum & 0xFFFFFFFFull) + (uint32_t)(sum >> 32);
    f += (uint32_t)(sum & 0xFFFFFFFFull) > f ? 1u : 0u;            // end-around carry
    f = (f & 0xFFFFu) + (f >> 16);
    f = (f & 0xFFFFu) + (f >> 16);
    f = (f & 0xFFFFu) + (f >> 16);
    return (~f) & 0xFFFFu;
}
__device__ __forceinline__ void store16(uint4* p, uint4 v) { *p = v; }
// Frame windows and descriptors are plain (cached) loads: non-temporal ones measured slower for
// device batches (C +12 us, B +6.5 us per 1M) and for host-memory batches (config B mapped 537
// vs 666-680 Mpps in place, C 214 vs 319; profiles/r03/v5_host_nt_ab.txt).

// ---- neighbour lookups ----------------------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t fold_v6(const uint32_t ip[4]) {
    return (ip[0] * 0x9E3779B1u) ^ (ip[1] * 0x85EBCA77u) ^ (ip[2] * 0xC2B2AE3Du) ^
           (ip[3] * 0x27D4EB2Fu);
}
__host__ __device__ __forceinline__ uint32_t slot1(uint32_t k, uint32_t seed, uint32_t bits) {
    return ((k ^ seed) * 0x9E3779B1u) >> (32 - bits);
}
__host__ __device__ __forceinline__ uint32_t slot2(uint32_t k, uint32_t seed, uint32_t bits) {
    const uint32_t x = (k ^ seed) * 0x85EBCA77u;
    return ((x ^ (x >> 16)) * 0xC2B2AE3Du) >> (32 - bits);
}
// The neighbour indexes' third choice (round 5: three-choice cuckoo placement fills the slots to
// ~0.6-0.8 instead of two-choice's < 0.5, so an index takes half the LDS: config C's ARP and NDP
// indexes 96 -> 48 KB, config B's ARP index 16 -> 8 KB)
__host__ __device__ __forceinline__ uint32_t slot3(uint32_t k, uint32_t seed, uint32_t bits) {
    const uint32_t x = (k ^ (seed * 0x9E3779B9u)) * 0x27D4EB2Fu;
    return ((x ^ (x >> 15)) * 0x165667B1u) >> (32 - bits);
}
__device__ __forceinline__ bool arp_slot_hit(const uint4& e, uint32_t ip) {
    return ((e.z >> 16) & 1u) && e.x == ip;
}
__device__ __forceinline__ bool arp_lookup(const NeighIndex& x, uint32_t ip, uint32_t& lo,
                                           uint32_t& hi) {
    if (x.bits == 0) return false;
    const uint4 e1 = x.t[slot1(ip, x.seed, x.bits)];
    const uint4 e2 = x.t[slot2(ip, x.seed, x.bits)];
    const uint4 e3 = x.t[slot3(ip, x.seed, x.bits)];
    const bool h1 = arp_slot_hit(e1, ip), h2 = arp_slot_hit(e2, ip), h3 = arp_slot_hit(e3, ip);
    const uint4 e = h1 ? e1 : h2 ? e2 : e3;
    lo = e.y;
    hi = e.z & 0xFFFFu;
    return h1 || h2 || h3;
}
// The same lookup against an LDS copy of the slot array.
__device__ __forceinline__ bool arp_lookup_lds(const uint4* t, uint32_t bits, uint32_t seed,
                                               uint32_t ip, uint32_t& lo, uint32_t& hi) {
    const uint4 e1 = t[slot1(ip, seed, bits)];
    const uint4 e2 = t[slot2(ip, seed, bits)];
    const uint4 e3 = t[slot3(ip, seed, bits)];
    const bool h1 = arp_slot_hit(e1, ip), h2 = arp_slot_hit(e2, ip), h3 = arp_slot_hit(e3, ip);
    const uint4 e = h1 ? e1 : h2 ? e2 : e3;
    lo = e.y;
    hi = e.z & 0xFFFFu;
    return h1 || h2 || h3;
}
__device__ __forceinline__ bool ndp_slot_hit(const uint4& a, const uint4& m, const uint32_t ip[4]) {
    return ((m.y >> 16) & 1u) && a.x == ip[0] && a.y == ip[1] && a.z == ip[2] && a.w == ip[3];
}
__device__ __forceinline__ bool ndp_lookup_lds(const uint4* t, uint32_t bits, uint32_t seed,
                                               const uint32_t ip[4], uint32_t& lo, uint32_t& hi) {
    const uint32_t k = fold_v6(ip);
    const uint32_t t1 = slot1(k, seed, bits), t2 = slot2(k, seed, bits), t3 = slot3(k, seed, bits);
    const uint4 a1 = t[2 * t1], m1 = t[2 * t1 + 1];
    const uint4 a2 = t[2 * t2], m2 = t[2 * t2 + 1];
    const uint4 a3 = t[2 * t3], m3 = t[2 * t3 + 1];
    const bool h1 = ndp_slot_hit(a1, m1, ip), h2 = ndp_slot_hit(a2, m2, ip),
               h3 = ndp_slot_hit(a3, m3, ip);
    const uint4 m = h1 ? m1 : h2 ? m2 : m3;
    lo = m.x;
    hi = m.y & 0xFFFFu;
    return h1 || h2 || h3;
}
__device__ __forceinline__ bool ndp_lookup(const NeighIndex& x, const uint32_t ip[4], uint32_t& lo,
                                           uint32_t& hi) {
    if (x.bits == 0) return false;
    return ndp_lookup_lds(x.t, x.bits, x.seed, ip, lo, hi);
}

// Both families in one lookup: the IPv4 (ARP) and IPv6 (NDP) lanes of a wave issue their slot
// loads together, so a mixed wave waits for one memory round trip, not one per family.
__device__ __forceinline__ bool neigh_lookup(const NeighIndex& arp, const NeighIndex& ndp,
                                             bool v6, const uint32_t d[4], uint32_t& lo,
                                             uint32_t& hi) {
    const uint4* t = v6 ? ndp.t : arp.t;
    const uint32_t bits = v6 ? ndp.bits : arp.bits;
    const uint32_t seed = v6 ? ndp.seed : arp.seed;
    if (bits == 0) return false;
    const uint32_t k = v6 ? fold_v6(d) : d[0];
    const uint32_t t1 = slot1(k, seed, bits), t2 = slot2(k, seed, bits), t3 = slot3(k, seed, bits);
    const uint32_t sh = v6 ? 1u : 0u;   // an NDP slot is two uint4: address, then MAC
    const uint4 a1 = t[t1 << sh], a2 = t[t2 << sh], a3 = t[t3 << sh];
    uint4 m1 = a1, m2 = a2, m3 = a3;
    if (v6) {
        m1 = t[2 * t1 + 1];
        m2 = t[2 * t2 + 1];
        m3 = t[2 * t3 + 1];
    }
    const bool h1 = v6 ? ndp_slot_hit(a1, m1, d) : arp_slot_hit(a1, d[0]);
    const bool h2 = v6 ? ndp_slot_hit(a2, m2, d) : arp_slot_hit(a2, d[0]);
    const bool h3 = v6 ? ndp_slot_hit(a3, m3, d) : arp_slot_hit(a3, d[0]);
    const uint4 e = h1 ? (v6 ? m1 : a1) : h2 ? (v6 ? m2 : a2) : (v6 ? m3 : a3);
    lo = v6 ? e.x : e.y;
    hi = (v6 ? e.y : e.z) & 0xFFFFu;
    return h1 || h2 || h3;
}

// Does each L1 entry agree with the table?  (ARP: an entry for 0.0.0.0 is never consulted,
// src/worker.c:186, so it always "agrees".)
__device__ void refresh_ok(DevL1* l1, const NeighIndex& arp, const NeighIndex& ndp) {
    uint32_t lo = 0, hi = 0;
    bool arp_ok = true;
    if (l1->arp_ip != 0)
        arp_ok = arp_lookup(arp, l1->arp_ip, lo, hi) && lo == l1->arp_mac_lo &&
                 hi == l1->arp_mac_hi;
    const uint32_t ip6[4] = {l1->ndp_ip[0], l1->ndp_ip[1], l1->ndp_ip[2], l1->ndp_ip[3]};
    const bool ndp_ok = ndp_lookup(ndp, ip6, lo, hi) && lo == l1->ndp_mac_lo &&
                        hi == l1->ndp_mac_hi;
    l1->arp_ok = arp_ok;
    l1->ndp_ok = ndp_ok;
}

__global__ void upe_refresh(DevL1* l1, NeighIndex arp, NeighIndex ndp) {
    if (threadIdx.x == 0 && blockIdx.x == 0) refresh_ok(l1, arp, ndp);
}

// Rule words are read through the constant address space: the compiler may then use scalar
// (s_load) loads, which it will not do through a generic pointer it cannot prove unwritten.
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
// A write-through (sc1) store: the line leaves this XCD's L2, so a reader on another XCD that
// has not cached it sees the value once the storing wave's stores have drained.
template <typename T>
__device__ __forceinline__ void st_wt(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename V, typename T>
__device__ __forceinline__ const __attribute__((address_space(4))) V* as_const(const T* p) {
    return (const __attribute__((address_space(4))) V*)p;
}

// The L1 state after a batch (src/worker.c:186-195, 218-225): the state
// before it, unless some forwarded packet missed the starting entry and hit the table — then
// the batch's last table hit, whose MAC is the table's (so the entry agrees with the table).
// in: DevL1 words before the batch; f4 / f6: first miss-then-hit (kNone = none); m4 / m6: last
// table hit + 1 (0 = none); wg4 / wg6: the workgroups holding those hits' payloads in pay.
// All arguments wave-uniform.  L: DevL1 words 0..10 after the batch.
__device__ __forceinline__ void fold_l1(const u32x16& in, uint32_t f4, uint32_t f6, uint32_t m4,
                                        uint32_t m6, uint32_t wg4, uint32_t wg6,
                                        const TilePay* pay, uint32_t (&L)[11]) {
#pragma unroll
    for (int j = 0; j < 11; ++j) L[j] = in[j];
    if (f4 != kNone && m4 != 0) {
        const u32x16 P = *as_const<u32x16>(pay + wg4);
        L[0] = P[0]; L[1] = P[1]; L[2] = P[2];
        L[9] = 1;
    }
    if (f6 != kNone && m6 != 0) {
        const u32x16 P = *as_const<u32x16>(pay + wg6);
        L[3] = P[3]; L[4] = P[4]; L[5] = P[5]; L[6] = P[6]; L[7] = P[7]; L[8] = P[8];
        L[10] = 1;
    }
}

// The batch's L1 outcome from its replicated l1r words: lane r < kReps holds replica r (lo/hi
// 32-bit halves of the 64-bit words), the rest zero.  Results wave-uniform.
struct L1Out {
    uint32_t f4, f6, m4, m6, wg4, wg6;
};
__device__ __forceinline__ L1Out reduce_l1r(const unsigned long long (&w)[R_N]) {
    L1Out o;
    o.f4 = kNone - wave_reduce<2>((uint32_t)w[R_F4]);
    o.f6 = kNone - wave_reduce<2>((uint32_t)w[R_F6]);
    const uint32_t h4 = (uint32_t)(w[R_M4] >> 32), h6 = (uint32_t)(w[R_M6] >> 32);
    o.m4 = wave_reduce<2>(h4);
    o.m6 = wave_reduce<2>(h6);
    // one packet index, one workgroup: the lanes holding the maximum agree on it
    o.wg4 = wave_reduce<2>(h4 == o.m4 && o.m4 ? (uint32_t)w[R_M4] : 0u);
    o.wg6 = wave_reduce<2>(h6 == o.m6 && o.m6 ? (uint32_t)w[R_M6] : 0u);
    return o;
}

// Fold a finished batch into the state the next one starts from, on the host's request (before
// the L1 state is read or replaced, or a neighbour table changes): l1 = fold(l1, acc, pay), and
// acc's L1 fields back to "nothing happened", so the next launch's own fold is the identity.
__global__ void upe_l1_sync(DevL1* l1, BatchAcc* acc, const TilePay* pay) {
    const int lane = threadIdx.x;
    unsigned long long w[R_N] = {0, 0, 0, 0};
    if (lane < kReps)
        for (int j = 0; j < R_N; ++j) w[j] = acc->l1r[lane][j];
    const L1Out o = reduce_l1r(w);
    const u32x16 in = *as_const<u32x16>(l1);
    uint32_t L[11];
    fold_l1(in, o.f4, o.f6, o.m4, o.m6, o.wg4, o.wg6, pay, L);
    __syncthreads();
    if (lane < kReps)
        for (int j = 0; j < R_N; ++j) acc->l1r[lane][j] = 0ull;
    if (lane == 0) {
        uint32_t* w = reinterpret_cast<uint32_t*>(l1);
#pragma unroll
        for (int j = 0; j < 11; ++j) w[j] = L[j];
    }
}

// First-match scan (reference src/rule_table.c:163-176 over match_rule :76-91).  Every lane of
// the wave walks the same rules in sorted order; rule words are wave-uniform loads.  `done`
// lanes (already matched, or not scanning) are ignored.  V6 = some lane holds an IPv6 key; rules
// without IPv6 address words skip the rv6 test (a scalar branch).
// Small tables are read from an LDS copy (staged at kernel entry, broadcast reads of a
// wave-uniform address: no scalar-cache round trip in the dependent chain); larger ones through
// the scalar unit from the constant address space.  (Staging the first 64 rules of larger
// tables in LDS too measured slower, profiles/r03/v8_rule_prefix_ab.txt: C's rule words already
// hit in the scalar cache.)
template <bool V6, bool kLdsRules>
__device__ __forceinline__ uint32_t scan_rules(const Args& a, bool done, bool is6, uint32_t k0,
                                               uint32_t k1, const uint32_t s[4],
                                               const uint32_t d[4], uint32_t& act,
                                               const u32x8* l4, const u32x16* l6,
                                               uint32_t b0, uint32_t b1) {
    uint32_t hit = kNone;
    static_assert(sizeof(RuleV4) == 32 && sizeof(RuleV6) == 64, "rule stream strides");
    const auto* rv4 = as_const<u32x8>(a.rv4);
    const auto* rv6 = as_const<u32x16>(a.rv6);
    for (uint32_t b = b0; b < b1; b += kUnroll) {
        // the rule index is wave-uniform: say so, so rule words come through the scalar unit
        const uint32_t base = __builtin_amdgcn_readfirstlane(b);
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            // RuleV4 words: x0 m0 x1 m1 s0 sm0 d0 dm0
            const u32x8 r = kLdsRules ? l4[base + u] : rv4[base + u];
            uint32_t x = ((k0 ^ r[0]) & r[1]) | ((k1 ^ r[2]) & r[3]) | ((s[0] ^ r[4]) & r[5]) |
                         ((d[0] ^ r[6]) & r[7]);
            if (V6 && (__builtin_amdgcn_readfirstlane(r[3]) & kRuleV6Words)) {
                // RuleV6 words: s[3] sm[3] d[3] dm[3]
                const u32x16 q = kLdsRules ? l6[base + u] : rv6[base + u];
                const uint32_t y = ((s[1] ^ q[0]) & q[3]) | ((s[2] ^ q[1]) & q[4]) |
                                   ((s[3] ^ q[2]) & q[5]) | ((d[1] ^ q[6]) & q[9]) |
                                   ((d[2] ^ q[7]) & q[10]) | ((d[3] ^ q[8]) & q[11]);
                if (is6) x |= y;
            }
            if (!done && x == 0) {
                hit = base + u;
                act = r[2];   // the action code rides in x1 bits 16-17 (see RuleV4)
                done = true;
            }
        }
        if (__all(done)) break;
    }
    return hit;
}

// First match over the per-family lists (FamTable): the same rule tests as scan_rules, each lane
// against its own family's list; `pos` is the lane's position in its list, turned into the
// sorted index after the loop (reference src/rule_table.c:163-176: the first match in (priority,
// rule_id) order — a rule of the other family cannot match, so it is skipped, not reordered).
template <bool V6>
__device__ __forceinline__ uint32_t scan_fam(const Args& a, bool done, bool is6, uint32_t k0,
                                             uint32_t k1, const uint32_t s[4], const uint32_t d[4],
                                             uint32_t& act, const uint4* l6) {
    // the IPv4 lanes' list, then the IPv6 lanes' list (one loop after the other: interleaving
    // both in one loop held twice the rule words in SGPRs and spilled)
    const auto* f4 = as_const<u32x8>(a.fam);
    const uint4* f6 = a.fam + 2 * (size_t)a.fam4;
    uint32_t pos = kNone;
    bool dn = done || is6;
    for (uint32_t b = 0; b < a.fam4; b += kUnroll) {
        if (!__any(!dn)) break;
        const uint32_t base = __builtin_amdgcn_readfirstlane(b);
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const u32x8 r = f4[base + u];
            const uint32_t x = ((k0 ^ r[0]) & r[1]) | ((k1 ^ r[2]) & r[3]) |
                               ((s[0] ^ r[4]) & r[5]) | ((d[0] ^ r[6]) & r[7]);
            if (!dn && x == 0) {
                pos = base + u;
                act = r[2];
                dn = true;
            }
        }
    }
    if (V6 && a.fam6_lds) {
        dn = done || !is6;
        for (uint32_t b = 0; b < a.fam6; b += kUnroll) {
            if (!__any(!dn)) break;
            const uint32_t base = __builtin_amdgcn_readfirstlane(b);
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint4* e = l6 + kFamV6Stride * (base + u);
                const uint4 e0 = e[0], e1 = e[1];
                uint32_t x = ((k0 ^ e0.x) & e0.y) | ((k1 ^ e0.z) & e0.w) |
                             ((s[0] ^ e1.x) & e1.y) | ((d[0] ^ e1.z) & e1.w);
                // (the IPv6 words only when some lane still looking passes the rest of the rule:
                // C6 136.6 -> 126.9 us; in the whole-table scan the same test cost C 0.5 us)
                if ((__builtin_amdgcn_readfirstlane(e0.w) & kRuleV6Words) && __any(!dn && x == 0)) {
                    const uint4 e2 = e[2], e3 = e[3], e4 = e[4];
                    // s1 s2 s3 sm1 | sm2 sm3 d1 d2 | d3 dm1 dm2 dm3
                    x |= ((s[1] ^ e2.x) & e2.w) | ((s[2] ^ e2.y) & e3.x) | ((s[3] ^ e2.z) & e3.y) |
                         ((d[1] ^ e3.z) & e4.y) | ((d[2] ^ e3.w) & e4.z) | ((d[3] ^ e4.x) & e4.w);
                }
                if (!dn && x == 0) {
                    pos = base + u;
                    act = e0.z;
                    dn = true;
                }
            }
        }
    } else if (V6) {
        // (two entries per step: four held 96 rule words in SGPRs and spilled)
        dn = done || !is6;
        for (uint32_t b = 0; b < a.fam6; b += 2) {
            if (!__any(!dn)) break;
            const uint32_t base = __builtin_amdgcn_readfirstlane(b);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const uint4* e = f6 + (size_t)kFamV6Stride * (base + u);
                const u32x8 r = *as_const<u32x8>(e);
                uint32_t x = ((k0 ^ r[0]) & r[1]) | ((k1 ^ r[2]) & r[3]) |
                             ((s[0] ^ r[4]) & r[5]) | ((d[0] ^ r[6]) & r[7]);
                if ((__builtin_amdgcn_readfirstlane(r[3]) & kRuleV6Words) && __any(!dn && x == 0)) {
                    const u32x16 q = *as_const<u32x16>(e + 2);
                    x |= ((s[1] ^ q[0]) & q[3]) | ((s[2] ^ q[1]) & q[4]) | ((s[3] ^ q[2]) & q[5]) |
                         ((d[1] ^ q[6]) & q[9]) | ((d[2] ^ q[7]) & q[10]) | ((d[3] ^ q[8]) & q[11]);
                }
                if (!dn && x == 0) {
                    pos = base + u;
                    act = r[2];
                    dn = true;
                }
            }
        }
    }
    // the lane's entry in the lists' index array (fam4 + position for the IPv6 list); the caller
    // loads the sorted index from it late, so the round trip overlaps the rest of the chunk
    return pos == kNone ? kNone : (is6 ? a.fam4 : 0u) + pos;
}

// First match through the decision-tree index (kTreeDims comment): for each of its family's five
// field trees a lane walks to a leaf, then tests the leaf's rules in list order against their
// FamTable entries (the flagged one without a test), stopping at its first match or at a
// position no better than the best so far.  A field's tree splits on that field's words only (an
// address tree also on the ports and the protocol), so each level compares one of a few key words
// prepared before the walk (an address tree: one of its field's four words or a port word, by
// the node's dimension bits).  Walks are per lane (divergent loads: LDS when
// the image is staged, else memory), two levels per 16-byte node load, the deep trees together
// (source and destination address, destination port), then the shallow ones (source port,
// protocol), node loads in flight together; the wave iterates as long as its deepest walk and
// its longest leaf, tree by tree.  Returns the
// lane's FamTable index-array entry, as scan_fam.
template <bool kLdsTree>
__device__ __forceinline__ uint32_t tree_match(const Args& a, bool active, bool is6, uint32_t k0,
                                               uint32_t k1, const uint32_t s[4], const uint32_t d[4],
                                               uint32_t& act, const uint2* lnodes, const uint4* l6,
                                               const uint4* l4) {
    const uint2* N = kLdsTree ? lnodes : a.tree;
    const uint32_t* E = reinterpret_cast<const uint32_t*>(N) + a.tree_loff;
    const uint2 dir = N[0];
    const uint32_t nt = active ? (is6 ? dir.y & 0xFFFFu : dir.x) : 0u, first = 1u + (is6 ? dir.x : 0u);
    const uint32_t sp = k0 >> 16, dp = k1, pr = (k0 >> 8) & 0xFFu;
    const uint4* g6 = a.fam + 2 * (size_t)a.fam4;
    uint32_t best = kNone, bact = 0;
    const bool fam_lds = (a.fam4_lds || a.fam4 == 0u) && (a.fam6_lds || a.fam6 == 0u);
    // The leaf of one tree: its rules in list order until a match or a position >= best.
    auto leaf_tests = [&](const uint32_t lw) {
        const uint32_t cnt = lw >> 21, off = lw & 0x1FFFFFu;
        bool look = cnt != 0u;
        for (uint32_t j = 0; __any(look); ++j) {
            if (look) {
                const uint32_t e = E[off + j];
                const uint32_t p = e & 0x7FFFFFFFu;
                if (p >= best) {
                    look = false;   // the lists ascend: nothing later in this leaf can win
                } else {
                    const bool cov = (e >> 31) != 0u;
                    if (fam_lds) {
                        // both lists in LDS (the usual case): one address, the first two words
                        // read for every lane, an IPv6 entry's other words in a masked block
                        // that updates x in place (no zeroed registers to merge)
                        const uint4* f = is6 ? l6 + kFamV6Stride * p : l4 + 2 * p;
                        const uint4 e0 = f[0], e1 = f[1];
                        uint32_t x6 = 0;
                        if (is6) {   // (issued with the first two reads: no second round trip)
                            const uint4 e2 = f[2], e3 = f[3], e4 = f[4];
                            x6 = ((s[1] ^ e2.x) & e2.w) | ((s[2] ^ e2.y) & e3.x) |
                                 ((s[3] ^ e2.z) & e3.y) | ((d[1] ^ e3.z) & e4.y) |
                                 ((d[2] ^ e3.w) & e4.z) | ((d[3] ^ e4.x) & e4.w);
                        }
                        const uint32_t x = ((k0 ^ e0.x) & e0.y) | ((k1 ^ e0.z) & e0.w) |
                                           ((s[0] ^ e1.x) & e1.y) | ((d[0] ^ e1.z) & e1.w) | x6;
                        if (cov || x == 0u) {
                            best = p;
                            bact = e0.z;
                            look = false;
                        } else if (j + 1u >= cnt) {
                            look = false;
                        }
                        continue;
                    }
                    uint4 e0, e1 = make_uint4(0, 0, 0, 0), e2 = e1, e3 = e1, e4 = e1;
                    if (is6 && a.fam6_lds) {
                        const uint4* f = l6 + kFamV6Stride * p;
                        e0 = f[0];
                        if (!cov) { e1 = f[1]; e2 = f[2]; e3 = f[3]; e4 = f[4]; }
                    } else if (is6) {
                        const uint4* f = g6 + (size_t)kFamV6Stride * p;
                        e0 = f[0];
                        if (!cov) { e1 = f[1]; e2 = f[2]; e3 = f[3]; e4 = f[4]; }
                    } else if (a.fam4_lds) {
                        const uint4* f = l4 + 2 * p;
                        e0 = f[0];
                        if (!cov) e1 = f[1];
                    } else {
                        const uint4* f = a.fam + 2 * (size_t)p;
                        e0 = f[0];
                        if (!cov) e1 = f[1];
                    }
                    uint32_t x = ((k0 ^ e0.x) & e0.y) | ((k1 ^ e0.z) & e0.w) |
                                 ((s[0] ^ e1.x) & e1.y) | ((d[0] ^ e1.z) & e1.w);
                    // s1 s2 s3 sm1 | sm2 sm3 d1 d2 | d3 dm1 dm2 dm3 (zero words for IPv4 entries)
                    x |= ((s[1] ^ e2.x) & e2.w) | ((s[2] ^ e2.y) & e3.x) | ((s[3] ^ e2.z) & e3.y) |
                         ((d[1] ^ e3.z) & e4.y) | ((d[2] ^ e3.w) & e4.z) | ((d[3] ^ e4.x) & e4.w);
                    if (cov || x == 0u) {
                        best = p;
                        bact = e0.z;
                        look = false;
                    } else if (j + 1u >= cnt) {
                        look = false;
                    }
                }
            }
        }
    };
    // an address tree's key word for a dimension: one of its field's words (big-endian for IPv6
    // where the image says so, so that a prefix is a range; IPv4's host-order word 0 and zeros),
    // or a port or the protocol (dimensions 8-10); bit selects keep them in registers
    auto addr_word = [&](const uint32_t dm, const uint32_t (&w)[4]) -> uint32_t {
        const uint32_t m1 = 0u - (dm & 1u), m2 = 0u - ((dm >> 1) & 1u);
        const uint32_t m8 = 0u - ((dm >> 3) & 1u);
        const uint32_t aw = vsel(m2, vsel(m1, w[3], w[2]), vsel(m1, w[1], w[0]));
        return vsel(m8, vsel(m2, pr, vsel(m1, dp, sp)), aw);
    };
    // one walk step (two levels, Args::tree comment): the next node, or the leaf (live = false)
    auto step = [](const uint4 q, uint32_t& idx, uint32_t& leaf, bool& live, auto key) {
        const bool c1 = key(q.x & 15u) >= q.y;
        const uint32_t lleaf = (q.x >> 13) & 1u;
        const bool cl = c1 ? ((q.x >> 14) & 1u) != 0u : lleaf != 0u;
        const uint32_t ct = c1 ? q.w : q.z;
        const uint32_t c2 = key(c1 ? (q.x >> 8) & 15u : (q.x >> 4) & 15u) >= ct ? 1u : 0u;
        if (live) {
            if (q.x & 0x1000u) {
                leaf = q.y;
                live = false;
            } else if (cl) {
                leaf = ct;
                live = false;
            } else {
                idx = (q.x >> 15) + ((c1 && !lleaf) ? 2u : 0u) + c2;
            }
        }
    };
    const uint4* S = reinterpret_cast<const uint4*>(N);
    {
        // the deep trees together (source and destination address, destination port), then the
        // shallow ones (source port, protocol: few distinct values); node loads in flight together
        const uint32_t sw6 = is6 ? dir.y >> 16 : 0u;
        uint32_t ws[4], wd[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            ws[q] = (sw6 >> q & 1u) ? bswap32(s[q]) : (is6 || q == 0) ? s[q] : 0u;
            wd[q] = (sw6 >> (4 + q) & 1u) ? bswap32(d[q]) : (is6 || q == 0) ? d[q] : 0u;
        }
        uint32_t ia = first, ib = first + 1u, ic = first + 3u, la = 0, lb = 0, lc = 0;
        bool va = nt != 0u, vb = va, vc = va;
        while (__any(va || vb || vc)) {
            const uint4 qa = S[ia], qb = S[ib], qc = S[ic];
            step(qa, ia, la, va, [&](uint32_t dm) { return addr_word(dm, ws); });
            step(qb, ib, lb, vb, [&](uint32_t dm) { return addr_word(dm, wd); });
            step(qc, ic, lc, vc, [&](uint32_t) { return dp; });
        }
        leaf_tests(la);
        leaf_tests(lb);
        leaf_tests(lc);
    }
    {
        uint32_t ia = first + 2u, ib = first + 4u, la = 0, lb = 0;
        bool va = nt != 0u, vb = va;
        while (__any(va || vb)) {
            const uint4 qa = S[ia], qb = S[ib];
            step(qa, ia, la, va, [&](uint32_t) { return sp; });
            step(qb, ib, lb, vb, [&](uint32_t) { return pr; });
        }
        leaf_tests(la);
        leaf_tests(lb);
    }
    if (__any(active && best == kNone)) {
        // no tree's rule: the family's rule that matches every key, if it has one
        const uint2 dflt = N[1];
        const uint32_t dv = is6 ? dflt.y : dflt.x;
        if (active && best == kNone && dv != kNone) {
            best = dv;
            bact = (is6 ? g6[(size_t)kFamV6Stride * dv] : a.fam[2 * (size_t)dv]).z;
        }
    }
    act = bact;
    return best == kNone ? kNone : (is6 ? a.fam4 : 0u) + best;
}

// Key hash of the tuple-space index (host and device agree bit for bit).
__host__ __device__ __forceinline__ uint32_t tss_hash(const uint32_t* k, int nw, uint32_t seed) {
    uint32_t h = seed ^ 0x9E3779B9u;
    for (int j = 0; j < nw; ++j) {
        h = (h ^ k[j]) * 0x01000193u;
        h ^= h >> 15;
    }
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}
// A slot's 16-bit fingerprint (never 0, which marks an empty slot).  The slot positions come
// from the high bits of products of the hash, the tag from its low bits.
__host__ __device__ __forceinline__ uint16_t tss_tag(uint32_t h) {
    return (uint16_t)((h & 0xFFFFu) | 1u);
}

// First match through the tuple-space index.  Groups are visited in order of their smallest
// sorted index, so once a lane's best index is below the next group's smallest, nothing later
// can precede it: the result is exactly the first match of the linear scan (reference
// src/rule_table.c:163-176).  Both families share one probe loop: each lane takes its own
// family's group descriptor, fingerprint array and slot table, so a wave that mixes IPv4 and
// IPv6 packets waits for one fingerprint and one slot round trip per group index, not one per
// family (one loop per family measured 1024 vs 940 us per config-D batch).  At most one
// slot per lane and group is read — the first whose fingerprint matches; a lane whose two
// fingerprints both match and whose first slot holds another key reads the second one in a
// (rare) extra step.
__device__ __forceinline__ uint32_t tss_fmix(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}
__device__ __forceinline__ uint32_t tss_match_both(const Args& a, bool active, bool is6,
                                                   uint32_t k0, uint32_t k1, const uint32_t s[4],
                                                   const uint32_t d[4], uint32_t& act,
                                                   const uint16_t* sfp) {
    uint32_t best = kNone;
    const uint32_t ng = a.ng4 > a.ng6 ? a.ng4 : a.ng6;
    const uint32_t ngf = is6 ? a.ng6 : a.ng4;
    const auto* G4 = as_const<u32x16>(a.tg4);
    const auto* G6 = as_const<u32x16>(a.tg6);
    const uint4* T = is6 ? a.tt6 : a.tt4;
    const uint32_t st = is6 ? (uint32_t)kTssSlot6 : (uint32_t)kTssSlot4;   // slot stride in uint4
    for (uint32_t g = 0; g < ng; ++g) {
        const uint32_t gu = __builtin_amdgcn_readfirstlane(g);
        u32x16 q4 = {}, q6 = {};
        if (gu < a.ng4) q4 = G4[gu];
        if (gu < a.ng6) q6 = G6[gu];
        // groups ascend by smallest sorted index within each family: once no lane wants group
        // g, no lane wants a later one
        const bool want = active && g < ngf && best > (is6 ? q6[10] : q4[10]);
        if (!__any(want)) break;
        const uint32_t cw = is6 ? q6[14] : q4[14];
        if (want && (cw & 1u)) {
            // catch-all group: the key matches (every mask is zero), its index is the group's
            if ((is6 ? q6[10] : q4[10]) < best) {
                best = is6 ? q6[10] : q4[10];
                act = (cw >> 8) << 16;
            }
        } else if (want) {
            uint32_t q[14];
#pragma unroll
            for (int j = 0; j < 14; ++j) q[j] = is6 ? q6[j] : q4[j];
            uint32_t kw[10];
            kw[0] = k0 & q[0];
            kw[1] = k1 & q[1];
            kw[2] = s[0] & q[2];
            kw[3] = is6 ? (s[1] & q[4]) : (d[0] & q[3]);
            kw[4] = s[2] & q[5]; kw[5] = s[3] & q[6]; kw[6] = d[0] & q[3];
            kw[7] = d[1] & q[7]; kw[8] = d[2] & q[8]; kw[9] = d[3] & q[9];
            // tss_hash over 4 words (IPv4) or 10 (IPv6), bit for bit
            uint32_t h = q[12] ^ 0x9E3779B9u;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                h = (h ^ kw[j]) * 0x01000193u;
                h ^= h >> 15;
            }
            uint32_t h6 = h;
#pragma unroll
            for (int j = 4; j < 10; ++j) {
                h6 = (h6 ^ kw[j]) * 0x01000193u;
                h6 ^= h6 >> 15;
            }
            h = tss_fmix(is6 ? h6 : h);
            const uint32_t t1 = q[13] + slot1(h, q[12], q[11]);
            const uint32_t t2 = q[13] + slot2(h, q[12], q[11]);
            const uint32_t tag = tss_tag(h);
            // fingerprints from LDS when the group's are staged; otherwise none: slot t1, then t2
            const uint32_t so = sfp ? (is6 ? q6[15] : q4[15]) : 0u;
            uint32_t f1 = tag, f2 = tag;
            if (so) {
                const uint32_t b = so - 1u - q[13];
                f1 = sfp[b + t1];
                f2 = sfp[b + t2];
            }
            const bool m1 = f1 == tag, m2 = f2 == tag;
            uint32_t idx = kNone, ac = 0;
            auto probe = [&](uint32_t t) {
                const uint4 A = T[st * t];
                uint4 B = make_uint4(0, 0, 0, 0), C = B;
                if (is6) {
                    B = T[st * t + 1];
                    C = T[st * t + 2];
                }
                const bool k4 = A.x == kw[0] && A.y == kw[1] && A.z == kw[2] && A.w == kw[3];
                // the compact IPv4 slot: v = (index + 1) | action << 22 in the key's free bits
                const uint32_t v = (A.x & 0xFFu) | ((A.y >> 16) << 8);
                const bool k4c = (A.x & ~0xFFu) == kw[0] && (A.y & 0xFFFFu) == kw[1] &&
                                 A.z == kw[2] && A.w == kw[3];
                const bool hit = is6 ? ((C.w & 1u) && k4 && B.x == kw[4] && B.y == kw[5] &&
                                        B.z == kw[6] && B.w == kw[7] && C.x == kw[8] &&
                                        C.y == kw[9])
                                     : (v != 0u && k4c);
                if (hit) {
                    idx = is6 ? C.z : (v & (kTssMaxRules - 1u)) - 1u;
                    ac = is6 ? (C.w >> 8) : v >> 22;
                }
                return hit;
            };
            if (m1 || m2) {
                const bool hit = probe(m1 ? t1 : t2);
                if (!hit && m1 && m2) probe(t2);
            }
            if (idx < best) {
                best = idx;
                act = ac << 16;
            }
        }
    }
    return best;
}

// ------------------------------------------------------------------------------------------
// General path: every live packet the fast path does not cover (ARP and NDP control frames,
// IPv4 with options, truncated, foreign or malformed frames).  Same outputs as the fast path.
// ------------------------------------------------------------------------------------------
struct Parsed {
    bool ok, consumed, v6;
    uint32_t flags;                // UPE_VF_ARP_LEARN / UPE_VF_ARP_REPLY
    uint32_t proto, sport, dport;
    uint32_t s[4], d[4];
    uint32_t ttl, c1w1, c1w2;      // TTL / hop, and bytes 20..27 as they are forwarded
};

// Inlined (only waves holding such a packet run it).  An out-of-line call (measured in round 2)
// saved the caller's live registers to scratch, ~100 bytes of private-memory traffic per slow
// packet (config D: 1.7 GB written per 16M batch); inlined, the classify kernels run without
// scratch at the 128-VGPR budget.  The path reuses the fast path's window (bytes 0..79, chunks
// at or past len zero) and loads bytes 80..95 only for frames that have them: it reads no byte
// at or past len except the ARP header, which masks them (len_mask), and its ARP reply stores
// bytes 0..47, which the window always holds as loaded.
struct Port {
    uint32_t mac_lo, mac_hi, ip4;
};
template <bool kBarrel>
__device__ __forceinline__ void general_path(Port a, uint8_t* p, uint32_t len, Parsed& r,
                                             const uint32_t (&win)[24]) {
    r.ok = false; r.consumed = false; r.v6 = false; r.flags = 0;
    r.proto = r.sport = r.dport = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) r.s[j] = r.d[j] = 0;
    r.ttl = 0;
    // bytes 0..95 (IPv4 options reach 94): the window, and bytes 80..95 when the frame has them
    uint32_t w[24];
#pragma unroll
    for (int j = 0; j < 24; ++j) w[j] = win[j];
    // Bytes 80..95 matter only to an IPv4 TCP header behind 52 or more bytes of IPv4 header (its
    // data-offset byte is byte 14 + 4 * IHL + 12): loaded here, for such frames only (loading
    // them with every window instead measured no faster for config D, 713 vs 715 us per 16M,
    // and slower for C in place, 57.3 vs 59.0 us: profiles/r04/v3_win6_ab.txt).
    if (len > 80u && (w[3] & 0xFFFFu) == 0x0008u && (byte_of(w[3], 2) & 0xFu) >= 14u &&
        byte_of(w[5], 3) == 6u) {
        const uint4 v = reinterpret_cast<const uint4*>(p)[5];
        w[20] = v.x; w[21] = v.y; w[22] = v.z; w[23] = v.w;
    }
    r.c1w1 = w[5];
    r.c1w2 = w[6];
    // Bytes 12/13 as a zero-filled pktbuf would hold them (the ethertype is read before any
    // length gate, src/worker.c:24-25).
    const uint32_t b12 = len > 12 ? byte_of(w[3], 0) : 0u;
    const uint32_t b13 = len > 13 ? byte_of(w[3], 1) : 0u;
    const uint32_t et = (b12 << 8) | b13;
    const bool is_v4 = et == 0x0800u;
    const bool is_v6 = et == 0x86DDu;
    const uint32_t ihl = byte_of(w[3], 2) & 0xFu;
    r.v6 = is_v6;

    // ---- handle_control_packet, reference src/worker.c:23-104 ----
    if (et == 0x0806u) {
        // The ARP header (bytes 14..41) is read without a length check: bytes at or past len
        // read as zero, as in a zero-filled pktbuf.
        uint32_t z[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) z[j] = w[j] & len_mask(len, j);
        const bool wellformed = (z[3] >> 16) == 0x0100u && z[4] == 0x04060008u;
        if (wellformed) {
            r.flags |= UPE_VF_ARP_LEARN;
            const bool request = (z[5] & 0xFFFFu) == 0x0100u;
            const uint32_t tpa = bswap32(at2(z[10], z[9]));
            if (request && a.ip4 != 0 && tpa == a.ip4) {
                // In-place reply, src/worker.c:42-51, assembled a dword at a time.
                uint32_t nw[12];
                nw[0] = at2(z[2], z[1]);                                  // eth.dst = eth.src
                nw[1] = (z[2] >> 16) | (a.mac_lo << 16);                  // eth.src = port MAC
                nw[2] = (a.mac_lo >> 16) | (a.mac_hi << 16);
                nw[3] = z[3];
                nw[4] = z[4];
                nw[5] = 0x0200u | (a.mac_lo << 16);                       // op = REPLY, sha
                nw[6] = (a.mac_lo >> 16) | (a.mac_hi << 16);
                nw[7] = bswap32(a.ip4);                                   // spa = port IPv4
                nw[8] = at2(z[6], z[5]);                                  // tha = old sha
                nw[9] = (z[6] >> 16) | (z[7] << 16);                      // tpa = old spa
                nw[10] = (z[7] >> 16) | (z[10] & 0xFFFF0000u);
                nw[11] = z[11];
                // bytes at or past len keep the buffer's own (never transmitted) bytes
#pragma unroll
                for (int j = 0; j < 12; ++j) {
                    const uint32_t m = len_mask(len, j);
                    w[j] = (nw[j] & m) | (w[j] & ~m);
                }
                {
                    uint4* q = reinterpret_cast<uint4*>(p);
                    store16(&q[0], make_uint4(w[0], w[1], w[2], w[3]));
                    store16(&q[1], make_uint4(w[4], w[5], w[6], w[7]));
                    store16(&q[2], make_uint4(w[8], w[9], w[10], w[11]));
                }
                r.flags |= UPE_VF_ARP_REPLY;
            }
        }
    }
    if (is_v6 && len >= 78u && byte_of(w[5], 0) == 58u) {               // src/worker.c:58-100
        const uint32_t type = byte_of(w[13], 2);                        // byte 54
        if (type == 135u || type == 136u) r.consumed = true;
    }

    // ---- parse_flow_key, reference src/parser.c:6-111 ----
    if (!r.consumed && len >= 14u) {
        if (is_v4) {
            const uint32_t ver = byte_of(w[3], 2) >> 4;
            const uint32_t hl = ihl * 4;
            if (len - 14 >= 20u && ver == 4 && hl >= 20 && len - 14 >= hl) {
                r.proto = byte_of(w[5], 3);                                  // byte 23
                r.s[0] = bswap32(at2(w[7], w[6]));                           // bytes 26..29
                r.d[0] = bswap32(at2(w[8], w[7]));                           // bytes 30..33
                const uint32_t l4len = len - 14 - hl;
                // L4 starts at byte 14 + 4 * ihl = 4 * (ihl + 3) + 2, i.e. in word ihl + 3, and
                // registers are not indexable: l4 words from w[ihl + 3 .. ihl + 7], and x0 =
                // w[ihl + 3] (the checksum's last half word), selected by IHL
                uint32_t l4w0 = 0, l4w1 = 0, l4w3 = 0, x0 = 0;
                if constexpr (kBarrel) {
                    // a four-stage barrel shift by ihl - 5 (31 selects; ihl < 5 fails the parse
                    // above, so only shifts 0..10 matter).  Tuple-space kernels only: in the scan
                    // kernels it measured slower for config B, whose waves never run this path
                    // (24.5 -> 26.7 us, an allocation effect; profiles/r04/v4_wave_general_ab.txt)
                    const uint32_t sh = ihl - 5u;
                    const uint32_t m8 = (uint32_t)((int32_t)(sh << 28) >> 31);
                    const uint32_t m4 = (uint32_t)((int32_t)(sh << 29) >> 31);
                    const uint32_t m2 = (uint32_t)((int32_t)(sh << 30) >> 31);
                    const uint32_t m1 = (uint32_t)((int32_t)(sh << 31) >> 31);
                    uint32_t y[12], z[8], u[6], x[5];
#pragma unroll
                    for (int k = 0; k < 12; ++k)
                        y[k] = 16 + k < 24 ? vsel(m8, w[16 + k < 24 ? 16 + k : 0], w[8 + k]) : w[8 + k];
#pragma unroll
                    for (int k = 0; k < 8; ++k) z[k] = vsel(m4, y[k + 4], y[k]);
#pragma unroll
                    for (int k = 0; k < 6; ++k) u[k] = vsel(m2, z[k + 2], z[k]);
#pragma unroll
                    for (int k = 0; k < 5; ++k) x[k] = vsel(m1, u[k + 1], u[k]);
                    l4w0 = at2(x[1], x[0]);
                    l4w1 = at2(x[2], x[1]);
                    l4w3 = at2(x[4], x[3]);
                    x0 = x[0];
                } else {
#pragma unroll
                    for (int h = 5; h <= 15; ++h) {
                        if ((int)ihl == h) {
                            l4w0 = at2(w[h + 4], w[h + 3]);
                            l4w1 = at2(w[h + 5], w[h + 4]);
                            l4w3 = at2(w[h + 7], w[h + 6]);
                            x0 = w[h + 3];
                        }
                    }
                }
                if (r.proto == 17u) {
                    r.ok = l4len >= 8u;
                    r.sport = be16_lo(l4w0);
                    r.dport = be16_lo(l4w0 >> 16);
                } else if (r.proto == 6u) {
                    const uint32_t thl = (byte_of(l4w3, 0) >> 4) * 4;
                    r.ok = l4len >= 20u && thl >= 20u && l4len >= thl;
                    r.sport = be16_lo(l4w0);
                    r.dport = be16_lo(l4w0 >> 16);
                } else if (r.proto == 1u) {
                    r.ok = l4len >= 8u;
                    r.sport = be16_lo(l4w1);                                 // icmp id
                    r.dport = be16_lo(l4w0);                                 // type << 8 | code
                }
                // checksum over IHL*4 bytes with the TTL decremented and the field zeroed:
                // sum of u16 words = (w3 >> 16) + w4 + ... + w[2 + ihl] + (w[3 + ihl] & 0xFFFF);
                // words 7..2+ihl as the sum of their 16-bit halves (v_dot2_u32_u16 with a 0/1
                // pair: congruent mod 0xFFFF, which is all the fold needs), w[3 + ihl] = x0
                r.ttl = byte_of(w[5], 2);
                const uint32_t w5n = (w[5] & 0xFF00FFFFu) | (((r.ttl - 1) & 0xFFu) << 16);
                const uint32_t w6z = w[6] & 0xFFFF0000u;
                typedef unsigned short ushort2_t __attribute__((ext_vector_type(2)));
                uint32_t hs = x0 & 0xFFFFu;
#pragma unroll
                for (int k = 7; k <= 17; ++k) {
                    const ushort2_t one = {1, 1}, none = {0, 0};
                    hs = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, w[k]),
                                                (uint32_t)k <= 2 + ihl ? one : none, hs, false);
                }
                const unsigned long long sum = (w[3] >> 16) + (unsigned long long)w[4] + w5n + w6z + hs;
                r.c1w1 = w5n;
                r.c1w2 = w6z | csum_fold(sum);
            }
        } else if (is_v6 && len - 14 >= 40u) {
            // as the fast path: next header byte 20, addresses 22..53, L4 at byte 54
            r.proto = byte_of(w[5], 0);
            r.s[0] = at2(w[6], w[5]);   r.s[1] = at2(w[7], w[6]);
            r.s[2] = at2(w[8], w[7]);   r.s[3] = at2(w[9], w[8]);
            r.d[0] = at2(w[10], w[9]);  r.d[1] = at2(w[11], w[10]);
            r.d[2] = at2(w[12], w[11]); r.d[3] = at2(w[13], w[12]);
            const uint32_t l4a = at2(w[14], w[13]), l4b = at2(w[15], w[14]);
            const uint32_t l4c = at2(w[17], w[16]);
            const uint32_t l4len = len - 54u;
            const uint32_t thl = (byte_of(l4c, 0) >> 4) * 4;
            const bool udp = r.proto == 17u, tcp = r.proto == 6u, icmp = r.proto == 1u;
            r.ok = (udp || icmp) ? l4len >= 8u : tcp && l4len >= 20u && thl >= 20u && l4len >= thl;
            r.sport = icmp ? be16_lo(l4b) : be16_lo(l4a);
            r.dport = icmp ? be16_lo(l4a) : be16_lo(l4a >> 16);
            r.ttl = byte_of(w[5], 1);
            r.c1w1 = (w[5] & 0xFFFF00FFu) | (((r.ttl - 1) & 0xFFu) << 8);
        }
    }
}

// ------------------------------------------------------------------------------------------
// Decoupled look-back (only while a starting L1 entry disagrees with the table).  A packet whose
// destination is the starting entry took the entry's MAC in the reference (src/worker.c:186-188,
// 218-220) iff no earlier packet of its family missed the entry and hit the table.  Every chunk
// (a wave's 64 packets of a tile) publishes whether it holds such a packet; a wave holding
// candidates reads the flags of the chunks before it, nearest first, until one holds such a
// packet or one already knows the answer for everything up to it (LB_KNOWN*), waiting for any
// chunk that has not published yet — but only for `spin` ticks of the 100 MHz clock.  The wait
// must be bounded: a chunk it waits for may belong to a workgroup that is not resident (another
// kernel holds CUs, or another context's grid on the same GPU) and can only start once a
// resident one exits.  A wave that gives up defers its candidates (upe_classify: they keep the
// table's answer for now, and the launch's last workgroup repairs them once every chunk has
// published), so no workgroup ever waits on one that has not started.  Returns the families of
// `need` (bit 0 v4, bit 1 v6) still unresolved (0 = all resolved); `got` = for the resolved
// ones, whether an earlier chunk holds a miss-then-hit packet.
// ------------------------------------------------------------------------------------------
__device__ uint32_t lookback(const uint32_t* lb, uint32_t chunk, uint32_t tag, uint32_t need,
                             int lane, uint32_t spin, uint32_t& got) {
    got = 0;
    int64_t base = chunk;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz
    while (need && base > 0) {
        const int64_t j = base - 64 + lane;
        uint32_t f = 0;
        bool ready = j < 0;
        for (;;) {
            if (!ready) {
                f = __hip_atomic_load(&lb[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ready = (f >> 6) == tag;
            }
            if (__all(ready)) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 >= spin) return need;   // defer
            __builtin_amdgcn_s_sleep(2);
        }
#pragma unroll
        for (int F = 0; F < 2; ++F) {
            const uint32_t fb = F ? LB_FP6 : LB_FP4;
            const uint32_t kb = F ? LB_KNOWN6 : LB_KNOWN4, ib = F ? LB_INCL6 : LB_INCL4;
            if (!(need & fb)) continue;
            const unsigned long long info = __ballot(j >= 0 && (f & (fb | kb)));
            if (info) {
                const int hl = 63 - __builtin_clzll(info);   // the nearest chunk that knows
                const uint32_t fh = (uint32_t)__shfl((int)f, hl, 64);
                if (fh & (fb | ib)) got |= fb;
                need &= ~fb;
            }
        }
        base -= 64;
    }
    return 0;   // walked to chunk 0: what is still needed has no earlier miss-then-hit packet
}

// The launch's last workgroup (wave 0) answers the candidates that waves deferred: every chunk
// has been processed by now, so every flag word of this launch is written or about to land.  F4 /
// F6 = the first chunk holding a miss-then-hit packet of each family; a deferred candidate of
// chunk c takes the starting entry's MAC iff F >= c (the earlier lanes of its own chunk were
// checked when it deferred).  entries[e] = packet index | family << 31 (1 = IPv6).  Plain
// stores suffice: launches on a context are ordered (no launch of the context starts before this
// one's end-of-kernel writeback), and nothing else in this launch writes these words after the
// deferring wave did.
constexpr int kRepairUnroll = 4;
struct Repair {
    uint32_t mac4_lo, mac4_hi, mac6_lo, mac6_hi;   // the batch's starting L1 entries' MACs
};
template <bool kEmit>
__device__ void repair_deferred(const Args& a, uint32_t nd, int lane, Repair m) {
    const uint32_t nchunks = (a.n + 63u) / 64u;
    uint32_t last = 0;   // the highest chunk with a deferred candidate: F beyond it does not matter
    for (uint32_t e = lane; e < nd; e += 64) last = max(last, (a.defer[2 * e] & 0x7FFFFFFFu) / 64u);
    last = wave_reduce<2>(last);
    uint32_t F4 = kNone, F6 = kNone;
    for (uint32_t b = 0; b <= last && b < nchunks && (F4 == kNone || F6 == kNone); b += 64) {
        const uint32_t j = b + (uint32_t)lane;
        uint32_t f = 0;
        if (j < nchunks && j <= last) {
            do {
                f = __hip_atomic_load(&a.lb[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } while ((f >> 6) != a.lb_tag);
        }
        const unsigned long long b4 = __ballot(f & LB_FP4), b6 = __ballot(f & LB_FP6);
        if (F4 == kNone && b4) F4 = b + (uint32_t)__builtin_ctzll(b4);
        if (F6 == kNone && b6) F6 = b + (uint32_t)__builtin_ctzll(b6);
    }
    const uint32_t w1_4 = m.mac4_hi | (a.port_mac_lo << 16), w1_6 = m.mac6_hi | (a.port_mac_lo << 16);
    const uint32_t w2 = (a.port_mac_lo >> 16) | (a.port_mac_hi << 16);
    // kRepairUnroll entries per lane at a time, their loads issued together (one wave does this)
    constexpr int U = kRepairUnroll;
    for (uint32_t e0 = 0; e0 < nd; e0 += U * 64) {
        uint32_t x[U], v[U], rs[U];
        uint4 q[U];
        bool p[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const uint32_t e = e0 + 64u * k + (uint32_t)lane;
            x[k] = e < nd ? a.defer[2 * e] : kNone;
            rs[k] = e < nd ? a.defer[2 * e + 1] : 0u;   // the record slot (emit mode)
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const uint32_t i = x[k] & 0x7FFFFFFFu;
            const bool v6 = (x[k] >> 31) != 0;
            // an earlier chunk's packet took the table: the provisional answer stands
            p[k] = x[k] != kNone && (v6 ? F6 : F4) >= i / 64u;
            if (p[k]) {
                v[k] = a.verdict[i];
                q[k] = kEmit ? a.hdr[rs[k]]
                             : *reinterpret_cast<const uint4*>(a.frames + ((size_t)(a.desc[i] >> 20) << 4));
            }
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (!p[k]) continue;
            const uint32_t i = x[k] & 0x7FFFFFFFu;
            const bool v6 = (x[k] >> 31) != 0;
            a.verdict[i] = v[k] | UPE_VF_NEIGH_HIT;
            const uint4 o = make_uint4(v6 ? m.mac6_lo : m.mac4_lo, v6 ? w1_6 : w1_4, w2, q[k].w);
            if (kEmit)
                a.hdr[rs[k]] = o;
            else
                *reinterpret_cast<uint4*>(a.frames + ((size_t)(a.desc[i] >> 20) << 4)) = o;
        }
    }
}

// ------------------------------------------------------------------------------------------
// Residency census (one launch per kernel configuration, before its first batch): how many
// workgroups of this kernel, with this much dynamic LDS, the chip really holds at once.  The
// occupancy API can answer one workgroup per CU too many (MI355X_MICROARCH.md, "Residency and
// cooperative launch"), and a persistent grid larger than what is resident runs its surplus
// workgroups after the others, doubling the tail.  Each workgroup arrives on w[0] and waits (at
// most ~60 us) for the whole grid; a workgroup that gives up records how many had arrived
// when it gave up (w[1], min).  Resident workgroups all arrive within a few microseconds of
// the first one and give up together, seeing every resident arrival and no other (the rest
// can only start once a resident one has exited); nobody gives up when the whole grid is
// resident.
// ------------------------------------------------------------------------------------------
__device__ void census_probe(uint32_t* w, uint32_t grid) {
    uint32_t v = __hip_atomic_fetch_add(&w[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz
    while (v < grid) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 6000) {
            v = __hip_atomic_load(&w[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_min(&w[1], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        __builtin_amdgcn_s_sleep(8);
        v = __hip_atomic_load(&w[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ------------------------------------------------------------------------------------------
// classify: persistent workgroups over 256-packet tiles
// ------------------------------------------------------------------------------------------
// kEmit: the rewritten header bytes of forwarded packets go to a record per packet (a.hdr,
// upe_hdr_rec_t, one coalesced 16-byte store per lane) and the frames are only read; otherwise
// frames are rewritten in place (bytes 0..31 of each forwarded frame).
// kLean: the launch has no flow_hash output, every non-empty neighbour index staged in LDS and
// (linear scan) no length side array, so those paths are not compiled in (fewer live kernel
// arguments: config B/C emit kernels spill 70 SGPRs instead of 96, ~1 % faster).
// kNoLB (lean only): chosen once the host has seen a launch start from L1 entries that agree with
// the tables (agreement then holds until the host changes the tables or the L1 state) or whose
// family's index is empty; the look-back is not compiled in, and an entry that disagrees with an
// empty index answers its candidates itself (no packet can hit that table first).
// kRing && kHost (emit only): the egress-list kernels (kTx, upe_gpu_process_emit_tx) — that bit
// pair is otherwise unused (a ring is never a host launch), so the list costs no variant bit.
// kRing (lean emit only): a ring launch — a batch of a.ring_cpb chunks completes when every
// workgroup owning part of it has finished its chunks of it; the last one stamps the time.
template <bool kTssMode, bool kEmit, bool kLean = false, bool kNoLB = false, bool kRing = false,
          bool kHost = false, int kScan = 0>
__global__ void __launch_bounds__(kBlock, kWavesPerSimd) upe_classify(Args a) {
    // rule match of a linear-scan table (kScan; the host picks the instantiation, so no kernel
    // carries another flavour's code): 0 small table from its LDS copy, 1 family lists, 2 whole
    // table through the scalar unit, 3 decision tree over the family lists
    constexpr bool kFam = kScan == 1, kGlb = kScan == 2, kTree = kScan == 3;
    constexpr bool kTx = kRing && kHost;          // the egress list (see above), not a ring
    constexpr bool kRingL = kRing && !kHost;      // a ring launch
    constexpr bool kFamIdx = kFam || kTree;   // the match is a FamTable index-array entry
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_hist[]; // [nrules_pad][2]
    // per wave: 8 counters, first f4 / f6 / ctrl, last m4 / m6
    __shared__ uint32_t s_tot[C_N + 3];   // the workgroup's counters; first f4 / f6 / ctrl (min)
    __shared__ uint32_t s_wm[kWaves][2];  // per wave: its last table hit per family (index + 1)
    __shared__ uint32_t s_pay[kWaves][kPayWords];   // ... and that hit's (ip, MAC)
    __shared__ u32x8 s_rv4[kTssMode || kScan ? 1 : kSmallRules];   // small tables: RuleV4 / RuleV6
    __shared__ u32x16 s_rv6[kTssMode || kScan ? 1 : kSmallRules];  // words (only kScan 0 has them)
    __shared__ uint32_t s_claim;   // the workgroup's next unclaimed chunk (workgroup-local index)
    __shared__ uint32_t s_bdone[kRingL ? kRingMax : 1];   // ring: the workgroup's chunks done per batch

    if (a.census) {
        if (threadIdx.x == 0) census_probe(a.st->census, gridDim.x);
        return;
    }
    STAMP(0);
    STAMP_WHERE();
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const bool lds_stats = a.nrules_pad <= (uint32_t)kLdsStatsMax;
    // (kGlb is chosen when a family's list is a single catch-all: there the family split
    // measured slower, config C 39.8 vs 41.9 us)
    const bool small_stats = kScan == 0 && a.nrules_pad <= (uint32_t)kSmallRules;

    if (lds_stats)
        for (uint32_t r = tid; r < 2 * a.nrules_pad; r += kBlock) lds_hist[r] = 0;

    // The next chunk's window issued in the middle of the current chunk (after its rule match),
    // so that its loads fly during the rest of it: into named registers carried into the next
    // iteration (not an array the compiler might place in scratch).  Only the linear-scan
    // kernels: the tuple-space ones have no registers to spare.
    constexpr bool kMid = (UPE_MID_PREFETCH & 1) && (!kTssMode || (UPE_MID_PREFETCH & 4)) &&
                          (kEmit || (UPE_MID_PREFETCH & 2));
    // ---- header window: bytes 0..79 as 16-byte loads issued together.  Chunks at or past len
    // are not loaded (they read as zero, as in a zero-filled pktbuf): a 64-byte frame costs
    // four loads, not five.  Frames shorter than 49 bytes never take the fast path.
    auto load_window = [&](uint64_t dsc, bool live, uint32_t (&w)[24]) {
#pragma unroll
        for (int j = 0; j < 24; ++j) w[j] = 0;
        if (live) {
            const uint32_t len = (uint32_t)(dsc & 0xFFFFu);
            const uint4* q = reinterpret_cast<const uint4*>(a.frames + ((size_t)(dsc >> 20) << 4));
#pragma unroll
            for (int c = 0; c < 5; ++c) {
                if (c < 3 || len > 16u * c) {
                    const uint4 v = q[c];
                    w[4 * c + 0] = v.x; w[4 * c + 1] = v.y; w[4 * c + 2] = v.z; w[4 * c + 3] = v.w;
                }
            }
        }
    };
    struct Win { uint4 c0, c1, c2, c3, c4; };
    auto fetch_window = [&](uint64_t dsc, bool live) -> Win {
        const uint4 z = make_uint4(0, 0, 0, 0);
        Win v{z, z, z, z, z};
        if (live) {
            const uint32_t len = (uint32_t)(dsc & 0xFFFFu);
            const uint4* q = reinterpret_cast<const uint4*>(a.frames + ((size_t)(dsc >> 20) << 4));
            v.c0 = q[0]; v.c1 = q[1]; v.c2 = q[2];
            if (len > 48u) v.c3 = q[3];
            if (len > 64u) v.c4 = q[4];
        }
        return v;
    };
    Win nw;
    bool have_nw = false;   // nw holds the window of the wave's next chunk
    // Work: the workgroup owns tiles blockIdx, blockIdx + grid, ... (one per CU at a time, so a
    // CU's tiles are one workgroup's), and each wave takes 64-packet chunks of them in order:
    // workgroup-local chunk k is chunk k % kWaves of the workgroup's tile k / kWaves.  Waves
    // claim k from an LDS counter, so the workgroup's waves finish together however unevenly
    // the CU schedules them (with several workgroups per CU and static tiles, the last one to
    // finish ran alone for ~4 us after the first: the CU favours older waves).  Global chunk
    // numbers ascend with k, and a wave's claims ascend.
    auto chunk_of = [&](uint32_t k) -> uint32_t {
        const uint32_t t = blockIdx.x + (k / a.tw) * gridDim.x;
        const uint32_t c = t * a.tw + k % a.tw;
        return t < a.ntiles && c * 64u < a.n ? c : kNone;
    };
    if (tid == 0) s_claim = kWaves;
    if (kRingL)
        for (uint32_t k = tid; k < (uint32_t)kRingMax; k += kBlock) s_bdone[k] = 0u;
    if (kRingL && tid == 0)   // the ring's time origin: the first workgroup to start
        __hip_atomic_fetch_min(a.ring_t0, (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid < C_N + 3) s_tot[tid] = tid < C_N ? 0u : kNone;
    if (tid < 2 * kWaves) s_wm[tid / 2][tid % 2] = 0u;
    uint32_t ch = chunk_of((uint32_t)wave);   // this wave's chunk
    // The first descriptor (its round trip runs under the table staging below), then small
    // rule tables into LDS, before the entry barrier.  (Issuing the first chunk's window loads
    // here too queues the staging loads behind them: B 26.3 -> 27.6 us, C 40.1 -> 43.8 us.)
    uint64_t dsc_next = 0;
    if (ch != kNone && ch * 64u + (uint32_t)lane < a.n) dsc_next = a.desc[ch * 64u + lane];
    if (!kTssMode && small_stats) {
        // small tables: the whole table
        const uint32_t nst = a.nrules_pad;
        const uint4* g4 = reinterpret_cast<const uint4*>(a.rv4);
        const uint4* g6 = reinterpret_cast<const uint4*>(a.rv6);
        uint4* d4 = reinterpret_cast<uint4*>(s_rv4);
        uint4* d6 = reinterpret_cast<uint4*>(s_rv6);
        for (uint32_t k = tid; k < 2 * nst; k += kBlock) d4[k] = g4[k];
        for (uint32_t k = tid; k < 4 * nst; k += kBlock) d6[k] = g6[k];
    }
    // The starting L1 entries: the state after batch k - 2 (one scalar load) with batch k - 1's
    // outcome folded in (its replicated minima / maxima, then at most two payload loads).
    // DevL1 words: arp_ip, arp_mac_lo/hi, ndp_ip[4], ndp_mac_lo/hi, arp_ok, ndp_ok.
    static_assert(sizeof(DevL1) == 64, "DevL1 is one scalar load");
    const u32x16 lin = *as_const<u32x16>(l1_in(a));
    unsigned long long pr[R_N] = {0, 0, 0, 0};
    if (lane < kReps)
        for (int j = 0; j < R_N; ++j) pr[j] = acc_prev(a)->l1r[lane][j];
    // small neighbour indexes into LDS after the rule-stats bins: a lookup is then an LDS read,
    // not a memory round trip queued behind the batch's frame traffic
    uint4* s_arp = reinterpret_cast<uint4*>(lds_hist + (lds_stats ? 2 * a.nrules_pad : 0u));
    uint4* s_ndp = s_arp + a.arp_lds;
    for (uint32_t k = tid; k < a.arp_lds; k += kBlock) s_arp[k] = a.arp.t[k];
    for (uint32_t k = tid; k < 2 * a.ndp_lds; k += kBlock) s_ndp[k] = a.ndp.t[k];
    uint4* s_fp4 = s_ndp + 2 * a.ndp_lds;
    if (kTssMode)
        for (uint32_t k = tid; k < a.fp_lds; k += kBlock) s_fp4[k] = a.tfs[k];
    // the decision tree's image, when the host found room for it
    uint4* s_tree = s_fp4;
    if (kTree) {
        const uint4* g = reinterpret_cast<const uint4*>(a.tree);
        for (uint32_t k = tid; k < a.tree_lds; k += kBlock) s_tree[k] = g[k];
    }
    // linear-scan tables past kSmallRules: the IPv6 family list, when the host found room
    // (staging the lists' sorted indexes as well measured slower: config C 41.6 -> 42.7 us)
    uint4* s_fam6 = s_fp4 + (kTree ? a.tree_lds : 0u);
    if (kFamIdx && a.fam6_lds) {
        const uint4* g = a.fam + 2 * (size_t)a.fam4;
        for (uint32_t k = tid; k < kFamV6Stride * a.fam6; k += kBlock) s_fam6[k] = g[k];
    }
    // (tree kernels) the IPv4 list as well, for the leaves' rule tests
    uint4* s_fam4 = s_fam6 + (a.fam6_lds ? kFamV6Stride * a.fam6 : 0u);
    if (kTree && a.fam4_lds)
        for (uint32_t k = tid; k < 2 * a.fam4; k += kBlock) s_fam4[k] = a.fam[k];
    const uint16_t* s_fps = kTssMode && a.fp_lds ? reinterpret_cast<const uint16_t*>(s_fp4) : nullptr;
    __syncthreads();
    STAMP(1);
    // The fold itself waits on those loads (and then on at most two payload loads), so it runs
    // after the first tile's frame loads are issued (or after the loop if there is no tile),
    // off the path to the first frames.
    uint32_t L1[11];
    bool look4 = false, look6 = false, folded = false;
    // Bookkeeping between batches, done by wave 0 of workgroups 0..7 before its first chunk (so
    // that it is off the end of the launch: their other waves take more chunks meanwhile).
    // Nothing else in this launch touches what it writes.
    auto books = [&]() {
        // batch k - 1's counters into the cumulative totals (upe_counters_t order): total j by
        // workgroup j % grid (j = 0 the batch size, pkts_in; j >= 1 counter j - 1)
        if (blockIdx.x < 8) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if ((uint32_t)j % gridDim.x != blockIdx.x) continue;
                const uint32_t v =
                    j == 0 ? __builtin_amdgcn_readfirstlane(__hip_atomic_load(
                                 &acc_prev(a)->n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                           : wave_reduce<0>(lane < kReps ? __hip_atomic_load(&acc_prev(a)->cnt[lane][j - 1],
                                                                             __ATOMIC_RELAXED,
                                                                             __HIP_MEMORY_SCOPE_AGENT)
                                                         : 0u);
                if (lane == 0 && v) atomicAdd(&a.st->totals[j], (unsigned long long)v);
            }
        }
        if (blockIdx.x == 0) {
            // workgroup 0: this batch's grid and size, batch k + 1's accumulators re-armed
            // (batch k - 2's, folded by batch k - 1)
            if (lane == 0) {
                st_wt(&acc_cur(a)->grid, gridDim.x);
                st_wt(&acc_cur(a)->n, a.n);
            }
            uint32_t* nc = &acc_next(a)->cnt[0][0];
            unsigned long long* nr = &acc_next(a)->l1r[0][0];
            for (uint32_t k = lane; k < (uint32_t)(kReps * C_N); k += 64) st_wt(&nc[k], 0u);
            for (uint32_t k = lane; k < (uint32_t)(kReps * R_N); k += 64) st_wt(&nr[k], 0ull);
            if (lane < kReps) st_wt(&acc_next(a)->ctrl[lane], 0u);
            if (lane < 3) st_wt(&(&acc_next(a)->done)[lane], 0u);   // done, ndefer, giveup
        }
    };
    auto fold_start = [&]() {
        const L1Out o = reduce_l1r(pr);
        fold_l1(lin, o.f4, o.f6, o.m4, o.m6, o.wg4, o.wg6, pay_prev(a), L1);
        look4 = L1[9] == 0u;    // the ARP entry disagrees with the table
        look6 = L1[10] == 0u;   // the NDP entry disagrees with the table
        folded = true;
    };
    if (wave == 0 && blockIdx.x < 8) books();

    // Persistent workgroups: the grid is what the chip holds at once, so the per-workgroup
    // flush happens once per workgroup, at the very end of its life.  (Per-wave claims from
    // device-scope counters shared by many workgroups cost 2.5 us per 1M batch: every claim
    // serialised on a few hot lines; the LDS counter is private to the workgroup.)
    // Descriptors run one chunk ahead of the frames they point at.
    // The workgroup's number of chunks: a wave claims its next chunk one ahead (so that its
    // descriptors arrive while it works) only while more than kLateClaim chunks are unclaimed;
    // after that it claims when it has finished its chunk, so that near the end no wave holds
    // an unstarted chunk while another waits with nothing.
    uint32_t nloc = 0;
    if (blockIdx.x < a.ntiles) {
        const uint32_t own = (a.ntiles - 1u - blockIdx.x) / gridDim.x + 1u;
        const uint32_t tl = blockIdx.x + (own - 1u) * gridDim.x;
        const uint32_t lc = min(a.tw, (a.n - tl * a.tw * 64u + 63u) / 64u);
        nloc = (own - 1u) * a.tw + lc;
    }
    auto claim = [&]() {
        uint32_t kn = 0;
        if (lane == 0) kn = atomicAdd(&s_claim, 1u);
        return chunk_of(__builtin_amdgcn_readfirstlane(kn));
    };
    uint32_t chn = kNone;   // this wave's next chunk
    // The descriptors a wave loads are consumed where they were loaded (this one, and the late
    // claim's at the end of the loop body), so that no descriptor is still pending at the loop
    // header: the wait for it would be a vmcnt(0) every iteration shares, which also waits for
    // the previous chunk's stores.
    asm volatile("" : "+v"(dsc_next));
    for (bool first = true; ch != kNone; first = false, ch = chn) {
        bool late;
        {
            uint32_t cur = 0;
            if (lane == 0)
                cur = __hip_atomic_load(&s_claim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            late = __builtin_amdgcn_readfirstlane(cur) + kLateClaim >= nloc;
            chn = late ? kNone : claim();
        }
        const uint32_t i = ch * 64u + (uint32_t)lane;
        const bool live = i < a.n;
        const uint64_t dsc = dsc_next;
        const uint32_t len = (uint32_t)(dsc & 0xFFFFu);
        // frames are 16-byte aligned: the offset in 16-byte units fits one register
        const uint32_t off16 = (uint32_t)(dsc >> 20);
        uint8_t* p = a.frames + ((size_t)off16 << 4);
        uint32_t w[24];
        if (kMid && have_nw) {
            const uint4 c[5] = {nw.c0, nw.c1, nw.c2, nw.c3, nw.c4};
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                w[4 * j + 0] = c[j].x; w[4 * j + 1] = c[j].y; w[4 * j + 2] = c[j].z; w[4 * j + 3] = c[j].w;
            }
            w[20] = w[21] = w[22] = w[23] = 0;
        } else {
            load_window(dsc, live, w);
        }
        have_nw = false;
        dsc_next = 0;
        if (chn != kNone && chn * 64u + (uint32_t)lane < a.n) dsc_next = a.desc[chn * 64u + lane];
        if (!folded) fold_start();

        if (first) STAMP_VM(2);
        // ---- fast path (option-less IPv4 / IPv6) or general path, chosen per wave ----
        const uint32_t e12 = w[3] & 0xFFFFu;          // bytes 12,13 (ethertype, byte-swapped)
        const bool fast4 = live && len >= 34u && e12 == 0x0008u && byte_of(w[3], 2) == 0x45u;
        const bool fast6 = live && len >= 54u && e12 == 0xDD86u;
        const bool slow = live && !fast4 && !fast6;
        Parsed r;
        // Tuple-space kernels (large tables): a wave holding any other frame parses all 64 on
        // the general path, which gives the fast path's results for the fast path's frames — one
        // parse per wave instead of both (config D: IPv4 options, VLAN tags and malformed headers
        // put such a frame in nearly every wave; classify 651 -> 641 us per 16M).  The scan
        // kernels keep the fast path for every wave and the general path for the lanes that need
        // it: there the merged form costs registers (C's emit kernel spilled 12 VGPRs to scratch,
        // 39.9 -> 44.3 us; B 24.7 -> 25.1; profiles/r04/v4_wave_general_ab.txt).
        constexpr bool kWaveGeneral = kTssMode;
        const bool wave_general = kWaveGeneral && __any(slow);
        if (wave_general) {
            general_path<kTssMode>(Port{a.port_mac_lo, a.port_mac_hi, a.port_ip4}, p, len, r, w);
        } else {
            r.ok = false; r.consumed = false; r.v6 = fast6; r.flags = 0;
            r.proto = fast6 ? byte_of(w[5], 0) : byte_of(w[5], 3);              // byte 20 / 23
            // addresses: v4 host order in word 0 (src/parser.c:40-41); v6 wire bytes
            r.s[0] = fast6 ? at2(w[6], w[5]) : bswap32(at2(w[7], w[6]));
            r.d[0] = fast6 ? at2(w[10], w[9]) : bswap32(at2(w[8], w[7]));
            r.s[1] = at2(w[7], w[6]);  r.s[2] = at2(w[8], w[7]);  r.s[3] = at2(w[9], w[8]);
            r.d[1] = at2(w[11], w[10]); r.d[2] = at2(w[12], w[11]); r.d[3] = at2(w[13], w[12]);
            {
                // L4 at byte 34 (v4) or 54 (v6), both 2 mod 4
                const uint32_t l4a = fast6 ? at2(w[14], w[13]) : at2(w[9], w[8]);     // L4 0..3
                const uint32_t l4b = fast6 ? at2(w[15], w[14]) : at2(w[10], w[9]);    // L4 4..7
                const uint32_t l4c = fast6 ? at2(w[17], w[16]) : at2(w[12], w[11]);   // L4 12..15
                const uint32_t l4len = len - (fast6 ? 54u : 34u);
                const uint32_t thl = (byte_of(l4c, 0) >> 4) * 4;
                const bool udp = r.proto == 17u, tcp = r.proto == 6u, icmp = r.proto == 1u;
                r.ok = (fast4 || fast6) &&
                       ((udp || icmp) ? l4len >= 8u
                                      : tcp && l4len >= 20u && thl >= 20u && l4len >= thl);
                r.sport = icmp ? be16_lo(l4b) : be16_lo(l4a);                  // icmp: id
                r.dport = icmp ? be16_lo(l4a) : be16_lo(l4a >> 16);            // type << 8 | code
                // NDP NS / NA, consumed by handle_control_packet (src/worker.c:57-100)
                r.consumed = fast6 && len >= 78u && r.proto == 58u &&
                             ((l4a & 0xFFu) == 135u || (l4a & 0xFFu) == 136u);
            }
            // forward rewrite of bytes 20..27: v4 ttl-- and checksum over the 20-byte header
            // (src/worker.c:174-176, src/parser.c:137-169, stored LE), v6 hop-- (src/worker.c:213)
            r.ttl = fast6 ? byte_of(w[5], 1) : byte_of(w[5], 2);               // byte 21 / 22
            if (fast6) {
                r.c1w1 = (w[5] & 0xFFFF00FFu) | (((r.ttl - 1) & 0xFFu) << 8);
                r.c1w2 = w[6];
            } else {
                const uint32_t w5n = (w[5] & 0xFF00FFFFu) | (((r.ttl - 1) & 0xFFu) << 16);
                const uint32_t w6z = w[6] & 0xFFFF0000u;
                const unsigned long long sum = (unsigned long long)(w[3] >> 16) + w[4] + w5n + w6z +
                                               w[7] + (w[8] & 0xFFFFu);
                r.c1w1 = w5n;
                r.c1w2 = w6z | csum_fold(sum);
            }

        }
        if (!kWaveGeneral && __any(slow) && slow) {
            Parsed g;
            general_path<kTssMode>(Port{a.port_mac_lo, a.port_mac_hi, a.port_ip4}, p, len, g, w);
            r = g;
        }

        const bool ctrl = live && (r.consumed || (r.flags & UPE_VF_ARP_LEARN));
        const bool ok = live && r.ok && !r.consumed;

        // ---- next hop, looked up before the rule scan: it needs only the destination, so its
        // latency hides behind the scan (the answer is unused unless the packet is forwarded) ----
        uint32_t mlo = 0, mhi = 0;
        bool nhit = false;
        if (ok && r.ttl > 1u) {
            if (!r.v6 && a.arp_lds)
                nhit = arp_lookup_lds(s_arp, a.arp.bits, a.arp.seed, r.d[0], mlo, mhi);
            else if (r.v6 && a.ndp_lds)
                nhit = ndp_lookup_lds(s_ndp, a.ndp.bits, a.ndp.seed, r.d, mlo, mhi);
            else if (!kLean)
                nhit = neigh_lookup(a.arp, a.ndp, r.v6, r.d, mlo, mhi);
        }

        // ---- rule_table_match ----
        const uint32_t k0 = (r.v6 ? 6u : 4u) | (r.proto << 8) | (r.sport << 16);
        const uint32_t k1 = r.dport;
        const bool need_v6 = __any(ok && r.v6);
        uint32_t ri, act = 0;   // act: the matched rule's x1 word (action code in bits 16-17)
        if (kTssMode) {
            ri = tss_match_both(a, ok, r.v6, k0, k1, r.s, r.d, act, s_fps);
        } else {
            // small tables from their LDS copy, larger ones through the scalar unit
            const uint32_t nr = a.nrules_pad;
            if (kTree)
                ri = a.tree_lds ? tree_match<true>(a, ok, r.v6, k0, k1, r.s, r.d, act,
                                                   reinterpret_cast<const uint2*>(s_tree), s_fam6,
                                                   s_fam4)
                                : tree_match<false>(a, ok, r.v6, k0, k1, r.s, r.d, act, nullptr,
                                                    s_fam6, s_fam4);
            else if (kFam)
                ri = need_v6 ? scan_fam<true>(a, !ok, r.v6, k0, k1, r.s, r.d, act, s_fam6)
                             : scan_fam<false>(a, !ok, r.v6, k0, k1, r.s, r.d, act, s_fam6);
            else if (kGlb)
                ri = need_v6 ? scan_rules<true, false>(a, !ok, r.v6, k0, k1, r.s, r.d, act, s_rv4, s_rv6, 0u, nr)
                             : scan_rules<false, false>(a, !ok, r.v6, k0, k1, r.s, r.d, act, s_rv4, s_rv6, 0u, nr);
            else
                ri = need_v6 ? scan_rules<true, true>(a, !ok, r.v6, k0, k1, r.s, r.d, act, s_rv4, s_rv6, 0u, nr)
                             : scan_rules<false, true>(a, !ok, r.v6, k0, k1, r.s, r.d, act, s_rv4, s_rv6, 0u, nr);
        }
        // kFam: ri is the lane's entry in the FamTable index array; the sorted index it holds is
        // loaded now and first used at the verdict store
        uint32_t rsi = ri;
        if (kFamIdx && ri != kNone)
            rsi = a.fam_x1idx ? (act >> 18) & 0x1FFFu
                              : reinterpret_cast<const uint32_t*>(a.fam + 2 * (size_t)a.fam4 +
                                                                  (size_t)kFamV6Stride * a.fam6)[ri];

        // ---- verdict, counters, rule_stats (src/worker.c:117-153) ----
        uint32_t code = 0, rbits = 0;
        if (r.consumed) {
            code = UPE_V_CONSUMED;
        } else if (!ok) {
            code = UPE_V_DROP_PARSE;
        } else if (ri == kNone) {
            code = UPE_V_DROP_NOMATCH;
        } else {
            const uint32_t ac = (act >> 16) & 3u;
            if (!kFamIdx) rbits = (ri + 1) << 8;
            // rule_stats[rule_id] += {1, len}, src/worker.c:141-144: an LDS histogram below for
            // LDS-resident tables; for larger ones upe_rule_hist folds the verdict words after
            // the launch (one scattered device atomic per packet would cost more than the
            // whole classification)
            code = ac == 0u ? UPE_V_DROP_RULE : ac == 1u ? UPE_V_FWD : UPE_V_DROP_ACTION;
        }
        uint32_t flags = r.flags;
        if (first) STAMP_VM(3);
        // the next chunk's window (its descriptor has been back since early in this chunk):
        // issued here, it arrives while this chunk finishes
        if (kMid && chn != kNone) {
            nw = fetch_window(dsc_next, chn * 64u + (uint32_t)lane < a.n);
            have_nw = true;
        }

        // ---- L3 forward (src/worker.c:155-244) ----
        bool fp4 = false, fp6 = false;       // this packet misses the start entry, hits table
        bool thit4 = false, thit6 = false;   // the table answered this packet
        bool hit = false;      // the packet gets a MAC: the table's (or the starting entry's)
        bool cand = false;     // destination == starting L1 entry (ARP: and != 0)
        bool wrote1 = false;
        bool deferred = false;   // this wave deferred candidates (wave-uniform)
        if (code == UPE_V_FWD) {
            if (r.ttl <= 1u) {                         // src/worker.c:165-172, 204-211
                code = UPE_V_DROP_TTL;
            } else if (!r.v6) {
                wrote1 = true;
                hit = nhit;
                cand = L1[0] != 0 && r.d[0] == L1[0];
                fp4 = !cand && hit;
                thit4 = hit;
            } else {
                wrote1 = true;
                hit = nhit;
                cand = r.d[0] == L1[3] && r.d[1] == L1[4] && r.d[2] == L1[5] &&
                       r.d[3] == L1[6];
                fp6 = !cand && hit;
                thit6 = hit;
            }
            if (cand) flags |= UPE_VF_L1_INIT;
        }
        // emit mode: a record for each forwarded packet only, compacted per 64-packet group in
        // packet order (the wave's chunk is one group): a ballot and a lane count give its slot,
        // 64 * (i / 64) + the forwarded packets before it in the group.  No record is written for
        // the other packets (config B: 7.5 MB of zero records per 1M batch before round 5).
        uint32_t rslot = 0;
        if (kEmit) {
            const unsigned long long fm = __ballot(live && code == UPE_V_FWD);
            rslot = ch * 64u + __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
        }
        if (kNoLB) {
            // a disagreeing entry here belongs to a family whose index is empty
            if (cand && (r.v6 ? look6 : look4)) {
                hit = true;
                mlo = r.v6 ? L1[7] : L1[1];
                mhi = r.v6 ? L1[8] : L1[2];
            }
        } else if (look4 || look6) {
            // The starting entry disagrees with the table: publish this chunk's miss-then-hit
            // packets, and give the packets aimed at the entry the entry's MAC unless an earlier
            // packet of their family missed it and hit the table (lookback).
            const uint32_t chunk = ch;
            const unsigned long long b4 = __ballot(fp4), b6 = __ballot(fp6);
            const uint32_t fpb = (b4 ? (uint32_t)LB_FP4 : 0u) | (b6 ? (uint32_t)LB_FP6 : 0u);
            const uint32_t tag = a.lb_tag << 6;
            if (lane == 0)
                __hip_atomic_store(&a.lb[chunk], tag | fpb, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            const bool c4 = cand && !r.v6 && look4, c6 = cand && r.v6 && look6;
            const uint32_t need = (__ballot(c4) ? (uint32_t)LB_FP4 : 0u) |
                                  (__ballot(c6) ? (uint32_t)LB_FP6 : 0u);
            if (need) {
                // once any wave of the launch has given up, wait only briefly (1/16 of the bound)
                // for an unpublished flag: the workgroup it belongs to is likely not resident,
                // but a short wait still resolves the flags that are merely in flight, so that
                // the give-up does not cascade into a long serial repair
                const uint32_t spin = __hip_atomic_load(&acc_cur(a)->giveup, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT) ? a.lb_spin / 16u : a.lb_spin;
                uint32_t before = 0;
                const uint32_t left = lookback(a.lb, chunk, a.lb_tag, need, lane, spin, before);
                const unsigned long long lt = (1ull << lane) - 1ull;
                const bool prior4 = (before & LB_FP4) || (b4 & lt);
                const bool prior6 = (before & LB_FP6) || (b6 & lt);
                const bool r4 = c4 && !(left & LB_FP4), r6 = c6 && !(left & LB_FP6);
                if ((r4 && !prior4) || (r6 && !prior6)) {
                    hit = true;
                    mlo = r.v6 ? L1[7] : L1[1];
                    mhi = r.v6 ? L1[8] : L1[2];
                }
                // what this chunk now knows about everything up to it (resolved families only)
                const uint32_t res = need & ~left;
                uint32_t kn = 0;
                if (res & LB_FP4)
                    kn |= LB_KNOWN4 | (((before & LB_FP4) || b4) ? (uint32_t)LB_INCL4 : 0u);
                if (res & LB_FP6)
                    kn |= LB_KNOWN6 | (((before & LB_FP6) || b6) ? (uint32_t)LB_INCL6 : 0u);
                if (lane == 0 && kn)
                    __hip_atomic_store(&a.lb[chunk], tag | fpb | kn, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                if (left) {
                    // Gave up: the candidates an earlier packet of this chunk does not answer keep
                    // the table's answer for now and list themselves (index | family << 31); the
                    // launch's last workgroup repairs them (repair_deferred) once every chunk has
                    // published.
                    const bool dl = (c4 && (left & LB_FP4) && !(b4 & lt)) ||
                                    (c6 && (left & LB_FP6) && !(b6 & lt));
                    const unsigned long long dm = __ballot(dl);
                    uint32_t base = 0;
                    if (lane == 0) {
                        __hip_atomic_store(&acc_cur(a)->giveup, 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                        if (dm) base = atomicAdd(&acc_cur(a)->ndefer, (uint32_t)__popcll(dm));
                    }
                    base = __builtin_amdgcn_readfirstlane(base);
                    if (dl) {   // (index | family, and the packet's record slot in emit mode)
                        const uint32_t e = base + (uint32_t)__popcll(dm & lt);
                        a.defer[2 * e] = i | (r.v6 ? 0x80000000u : 0u);
                        a.defer[2 * e + 1] = rslot;
                    }
                    deferred = dm != 0;
                }
            }
        }
        if (hit) flags |= UPE_VF_NEIGH_HIT;

        // ---- write back ----
        if (kEmit && live && code == UPE_V_FWD) {
            // record: bytes 0..11 as forwarded (neighbour + port MAC on a hit, else unchanged),
            // the new TTL / hop limit, the new IPv4 checksum, the family
            uint4 rec;
            rec.x = hit ? mlo : w[0];
            rec.y = hit ? (mhi | (a.port_mac_lo << 16)) : w[1];
            rec.z = hit ? ((a.port_mac_lo >> 16) | (a.port_mac_hi << 16)) : w[2];
            rec.w = r.v6 ? (((r.c1w1 >> 8) & 0xFFu) | (6u << 24))
                         : (((r.c1w1 >> 16) & 0xFFu) | ((r.c1w2 & 0xFFFFu) << 8) | (4u << 24));
            {   // a buffer store with the write-through cache policy (kRecAux)
                typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.hdr, 0, 0x7FFFFFF0, 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b128(v4u{rec.x, rec.y, rec.z, rec.w}, rs,
                                                       rslot * 16u, 0, kRecAux);
            }
        } else if (!kEmit && live) {
            uint4* q = reinterpret_cast<uint4*>(a.frames + ((size_t)off16 << 4));
            if (hit)
                store16(&q[0], make_uint4(mlo, mhi | (a.port_mac_lo << 16),
                                                (a.port_mac_lo >> 16) | (a.port_mac_hi << 16), w[3]));
            if (wrote1) store16(&q[1], make_uint4(w[4], r.c1w1, r.c1w2, w[7]));
        }
        if (kFamIdx && ok && !r.consumed && ri != kNone) rbits = (rsi + 1) << 8;
        if (live)   // written through (sc1): no dirty lines left for the boundary
            __hip_atomic_store(&a.verdict[i], code | flags | rbits, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        // the egress list in the same pass (upe_gpu_process_emit_tx): each forwarded packet's
        // index in its record's slot, and the group's count (src/worker.c:240-243 queues the
        // forwarded frames in packet order).  Its own kernel instantiations (kTx), so that no
        // other launch carries the code or its registers.
        if (kTx) {
            const unsigned long long fm = __ballot(live && code == UPE_V_FWD);
            if (live && code == UPE_V_FWD)
                a.tx[ch * 64u + __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u))] =
                    a.tx_base + i;
            if (lane == 0) a.tx_cnt[ch] = (uint32_t)__popcll(fm);
        }
        // the side array upe_rule_hist reads (lean linear-scan launches never have it; the
        // tuple-space tables it serves always do)
        if ((kTssMode || !kLean) && a.gb && live) {
            // tables of up to 64k rules: the rule and the length in one 4-byte key, so that the
            // group-by reads 4 bytes per packet per rule range instead of verdict + length (6)
            if (a.gb_packed)
                static_cast<uint32_t*>(a.gb)[i] = rbits ? ((rbits << 8) - 0x10000u) | len : 0u;
            else
                static_cast<uint16_t*>(a.gb)[i] = (uint16_t)len;
        }
        if (!kLean && a.flow_hash && live) {
            // software RSS in the same pass: flow_hash (reference src/parser.c:113-135) of the
            // key parse_flow_key gives the RX thread (src/rx_pcap.c:71-72), 0 if it fails
            uint32_t h = r.sport ^ r.dport ^ r.proto;
            h ^= r.v6 ? (r.s[0] ^ r.s[1] ^ r.s[2] ^ r.s[3] ^ r.d[0] ^ r.d[1] ^ r.d[2] ^ r.d[3])
                      : (r.s[0] ^ r.d[0]);
            a.flow_hash[i] = ok ? h : 0u;
        }
        // a deferring wave's outputs and entries are complete before its workgroup counts itself
        // done (the repair reads and patches them)
        if (!kNoLB && deferred) __threadfence();

        // ---- rule_stats: LDS histogram (same-address lanes serialise in the LDS atomic unit,
        // cheaper than a cross-lane reduction per distinct rule).  One 64-bit atomic per packet:
        // the bin's low word counts packets, the high word bytes; neither carries into the other
        // (a workgroup's packets and bytes each fit 32 bits, as the u32 views below assume) ----
        if (lds_stats && ok && ri != kNone)
            atomicAdd(reinterpret_cast<unsigned long long*>(&lds_hist[2 * rsi]),
                      ((unsigned long long)len << 32) | 1ull);

        // ---- counters and L1 bookkeeping: ballots, added by one lane into the workgroup's LDS
        // totals (no per-lane accumulators to reduce at the end).  A wave's chunks ascend, so its
        // latest table hit per family is the highest such lane of its latest chunk with one, and
        // that lane leaves the hit's payload in the wave's slot. ----
        {
            const bool nc = live && !r.consumed;
            const unsigned long long bm[C_N] = {
                __ballot(ok), __ballot(ok && ri != kNone), __ballot(live && code == UPE_V_FWD),
                __ballot(live && code != UPE_V_FWD && code != UPE_V_CONSUMED),
                __ballot(live && r.consumed), __ballot(nc && (r.flags & UPE_VF_ARP_LEARN)),
                __ballot(nc && (r.flags & UPE_VF_ARP_REPLY)), __ballot(ctrl)};
            const unsigned long long q4 = __ballot(fp4), q6 = __ballot(fp6);
            const unsigned long long h4 = __ballot(thit4), h6 = __ballot(thit6);
            const uint32_t base = ch * 64u;
            if (lane == 0) {
#pragma unroll
                for (int c = 0; c < C_N; ++c)
                    if (bm[c]) atomicAdd(&s_tot[c], (uint32_t)__popcll(bm[c]));
                if (q4) atomicMin(&s_tot[C_N + 0], base + (uint32_t)__builtin_ctzll(q4));
                if (q6) atomicMin(&s_tot[C_N + 1], base + (uint32_t)__builtin_ctzll(q6));
                if (bm[C_CTRL])
                    atomicMin(&s_tot[C_N + 2], base + (uint32_t)__builtin_ctzll(bm[C_CTRL]));
                if (h4) s_wm[wave][0] = base + 64u - (uint32_t)__builtin_clzll(h4);   // index + 1
                if (h6) s_wm[wave][1] = base + 64u - (uint32_t)__builtin_clzll(h6);
            }
            if (h4 && lane == 63 - __builtin_clzll(h4)) {
                s_pay[wave][0] = r.d[0]; s_pay[wave][1] = mlo; s_pay[wave][2] = mhi;
            }
            if (h6 && lane == 63 - __builtin_clzll(h6)) {
                s_pay[wave][3] = r.d[0]; s_pay[wave][4] = r.d[1]; s_pay[wave][5] = r.d[2];
                s_pay[wave][6] = r.d[3]; s_pay[wave][7] = mlo; s_pay[wave][8] = mhi;
            }
        }
        if (kRingL) {
            // every workgroup owns ring_mine chunks of each batch (the host launches the ring
            // kernel only when a batch's tiles divide evenly over the grid, and for at most
            // kRingMax batches: one LDS counter per batch, however far apart the workgroup's
            // waves are)
            const uint32_t j = ch / a.ring_cpb, mine = a.ring_mine;
            uint32_t d = 0;
            if (lane == 0) d = atomicAdd(&s_bdone[j], 1u) + 1u;
            d = __builtin_amdgcn_readfirstlane(d);
            if (d == mine) {   // the workgroup is done with batch j
                uint32_t t = 0;
                if (lane == 0) t = atomicAdd(&a.ring_wg[j], 1u) + 1u;
                t = __builtin_amdgcn_readfirstlane(t);
                if (lane == 0 && t == gridDim.x) {
                    const unsigned long long t0 = __hip_atomic_load(a.ring_t0, __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&a.ring_done[j],
                                       ((unsigned long long)__builtin_amdgcn_s_memrealtime() - t0) * 10ull,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
        if (late) {
            chn = claim();
            dsc_next = 0;
            if (chn != kNone && chn * 64u + (uint32_t)lane < a.n) dsc_next = a.desc[chn * 64u + lane];
            asm volatile("" : "+v"(dsc_next));   // consumed here (see before the loop)
        }
    }
    STAMP(4);
    if (!folded) fold_start();
    STAMP(9);
    // A bare barrier: LDS drained (lgkmcnt), global stores left in flight (nothing in this launch
    // reads what this workgroup wrote; __syncthreads() would make every wave wait for its write
    // acknowledgements).
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    STAMP(10);

    // A look-back-live launch counts its finished workgroups; the last one answers whatever the
    // waves deferred (nobody waits for that: a workgroup that is not resident yet delays only the
    // count).  Wave 1 counts, with one atomic whose return it waits for, issued before anything
    // else it has to send, while wave 0 flushes the accumulators and the other waves the
    // mid-size rule_stats, so the round trip overlaps those.
    constexpr int kCounter = kWaves > 1 ? 1 : 0;
    const bool counting = !kNoLB && (look4 || look6);
    if (counting && wave == kCounter) {
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(&acc_cur(a)->done, 1u);
        t = __builtin_amdgcn_readfirstlane(t);
        if (t + 1u == gridDim.x) {
            const uint32_t nd = __hip_atomic_load(&acc_cur(a)->ndefer, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
            if (nd) {
                __threadfence();   // acquire: the deferring waves' entries and outputs
                repair_deferred<kEmit>(a, nd, lane, Repair{L1[1], L1[2], L1[7], L1[8]});
            }
        }
    }

    // ---- rule_stats of mid-size tables: into one of kStatReps replicas of the per-sorted-index
    // totals (the host sums them and credits rule_id; nothing in this launch reads them), so
    // that the hot rules' counters take 1/kStatReps of the workgroups' atomics each (by every
    // wave but the counting one) ----
    if (lds_stats && !small_stats && !(counting && kWaves > 1 && wave == kCounter)) {
        unsigned long long* rep = a.stats_idx + (size_t)(blockIdx.x % kStatReps) * 2 * a.nrules_pad;
        const uint32_t skip = counting && kWaves > 1 ? 64u : 0u;
        const uint32_t t0 = (uint32_t)tid - (counting && kWaves > 1 && wave > kCounter ? 64u : 0u);
        for (uint32_t k = t0; k < 2 * a.nrules_pad; k += kBlock - skip) {
            const uint32_t v = lds_hist[k];
            if (v) atomicAdd(&rep[k], (unsigned long long)v);
        }
    }
    if (wave != 0) return;
    // ---- wave 0: flush the workgroup into the replicated accumulators ----
    // Device atomics are priced per wave-instruction (~50 ns per CU, whatever the lane count),
    // so every accumulator kind goes out as ONE instruction, lane k carrying field k.  Nothing
    // waits for them: the next launch reads them (kernel boundary), the host after a
    // synchronisation.
    const uint32_t rep = blockIdx.x % kReps;
    const uint32_t f4 = s_tot[C_N + 0], f6 = s_tot[C_N + 1], fc = s_tot[C_N + 2];
    // the workgroup's last table hit per family and the wave holding its payload: lane v reads
    // wave v's (index + 1) << 4 | v, and the maximum names both (index + 1 < 2^25)
    static_assert(kWaves <= 16, "the wave index is packed in 4 bits");
    const uint32_t m4 = wave_reduce<2>(lane < kWaves ? s_wm[lane][0] << 4 | (uint32_t)lane : 0u);
    const uint32_t m6 = wave_reduce<2>(lane < kWaves ? s_wm[lane][1] << 4 | (uint32_t)lane : 0u);
    const uint32_t x4 = m4 >> 4, x6 = m6 >> 4;
    const int w4 = (int)(m4 & 15u), w6 = (int)(m6 & 15u);
    {
        const uint32_t cv = lane < C_N ? s_tot[lane] : 0u;   // lane c < C_N: counter c
        if (lane < C_N && cv) atomicAdd(&acc_cur(a)->cnt[rep][lane], cv);
        // the L1 outcome, one atomicMax instruction: minima as kNone - x, the last table hits
        // with the workgroup whose payload describes them
        const unsigned long long rv =
            lane == R_F4 ? (unsigned long long)(kNone - f4)
          : lane == R_F6 ? (unsigned long long)(kNone - f6)
          : lane == R_M4 ? (x4 ? (unsigned long long)x4 << 32 | blockIdx.x : 0ull)
                         : (x6 ? (unsigned long long)x6 << 32 | blockIdx.x : 0ull);
        if (lane < R_N && rv) atomicMax(&acc_cur(a)->l1r[rep][lane], rv);
        if (lane == 0 && fc != kNone) atomicMax(&acc_cur(a)->ctrl[rep], kNone - fc);
        if (lds_stats && small_stats) {
            for (uint32_t k = lane; k < 2 * a.nrules_pad; k += 64) {
                const uint32_t v = lds_hist[k];
                if (v) atomicAdd(&a.st->acc_stats[rep][k], (unsigned long long)v);
            }
        }
    }
    // the workgroup's last table hit per family (the next launch reads the one the batch
    // maximum points at)
    if ((lane < 3 && x4) || (lane >= 3 && lane < kPayWords && x6))
        st_wt(&reinterpret_cast<uint32_t*>(&pay_cur(a)[blockIdx.x])[lane], s_pay[lane < 3 ? w4 : w6][lane]);
    // workgroup 0: the folded starting state for batch k + 1 (which folds this batch's outcome
    // into it)
    if (blockIdx.x == 0 && lane < 16) {
        // lane j: word j (written through, as the payloads)
        uint32_t v = 0u;
#pragma unroll
        for (int j = 0; j < 11; ++j) v = lane == j ? L1[j] : v;
        st_wt(&reinterpret_cast<uint32_t*>(l1_out(a))[lane], v);
    }
    if (blockIdx.x == 0 && lane == 0) {
        // tell the host whether this batch started from agreeing entries (upe_gpu_process picks
        // the kernel without look-back once one has)
        if (!kNoLB && a.agree_out)
            __hip_atomic_store(a.agree_out,
                               a.launch_tag << 2 | (L1[9] ? 1ull : 0ull) | (L1[10] ? 2ull : 0ull),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    STAMP(5);
}


// ------------------------------------------------------------------------------------------
// rule_stats of large tables (more rules than an LDS histogram holds): a group-by of the
// batch's verdict words by matched rule.  Workgroup (x, y) counts the packets of chunk x whose
// rule falls in range y in LDS bins (packets << 40 | bytes, which cannot overflow: a chunk holds
// at most 2^24 packets of at most 65535 bytes), then writes the bins densely into per-chunk
// partials that upe_hist_reduce sums (device atomics per nonzero bin, measured in round 2, were
// no faster and needed a packed staging array).  Every range re-reads its chunk (for tables of up
// to 64k rules the 4-byte key the classify pass left — rule << 16 | length, round 4: 6 -> 4 bytes
// per packet per range; larger ones the verdict word + a 2-byte length), so ranges are as wide
// as LDS allows; 1024-thread workgroups with sixteen packets
// per thread per round keep enough loads in flight (config D: 256-thread workgroups with four
// packets a round spent ~300 us per 16M batch waiting on them; eight a round 69.5 us, sixteen
// 62.6 us, thirty-two slower again).
// ------------------------------------------------------------------------------------------
#ifndef UPE_HIST_RANGE
#define UPE_HIST_RANGE 16384
#endif
constexpr uint32_t kHistRange = UPE_HIST_RANGE;   // most rules per workgroup: 128 KB of LDS
constexpr uint32_t kHistChunk = 1u << 24;   // most packets per workgroup
constexpr uint32_t kHistChunkMin = 8192;
#ifndef UPE_HIST_TARGET
#define UPE_HIST_TARGET 256
#endif
constexpr uint32_t kHistTarget = UPE_HIST_TARGET;   // workgroups per group-by launch
constexpr int kHistBlock = 1024;
#ifndef UPE_HIST_PER
#define UPE_HIST_PER 16
#endif
constexpr int kHistPer = UPE_HIST_PER;   // packets per thread per round (a multiple of 8)
static_assert(kHistPer % 8 == 0 && 8192 % (kHistPer * 1) == 0, "group-by rounds stay 16-byte aligned");

template <bool kPacked>
__global__ void __launch_bounds__(kHistBlock) upe_rule_hist(const uint32_t* verdict,
                                                            const void* gb, uint32_t n,
                                                            uint32_t nrules,
                                                            unsigned long long* part,
                                                            uint32_t chunk, uint32_t range) {
    extern __shared__ unsigned long long h[];   // [range]: packets << 40 | bytes
    const uint32_t r0 = blockIdx.y * range;
    const uint32_t p0 = blockIdx.x * chunk;
    for (uint32_t k = threadIdx.x; k < range; k += kHistBlock) h[k] = 0;
    __syncthreads();
    const uint32_t pend = n - p0 < chunk ? n : p0 + chunk;
    // kHistPer packets per thread per round, all loads issued before the first bin update
    // (chunks start at multiples of 8192, so full groups are 16-byte aligned).  Packed keys:
    // kHistPer / 4 16-byte key loads (rule index << 16 | len, 0 = not counted); otherwise
    // kHistPer / 4 verdict loads and kHistPer / 8 length loads.
    const uint32_t* keys = static_cast<const uint32_t*>(gb);
    const uint16_t* lens = static_cast<const uint16_t*>(gb);
    for (uint32_t i = p0 + kHistPer * threadIdx.x; i < pend; i += kHistPer * kHistBlock) {
        uint32_t rb[kHistPer], len[kHistPer];   // rule index + 1 (0 = none), length
        if (i + kHistPer <= pend) {
#pragma unroll
            for (int q = 0; q < kHistPer / 4; ++q) {
                const uint4 a0 = *reinterpret_cast<const uint4*>((kPacked ? keys : verdict) + i + 4 * q);
                rb[4 * q + 0] = a0.x; rb[4 * q + 1] = a0.y; rb[4 * q + 2] = a0.z; rb[4 * q + 3] = a0.w;
            }
            if (!kPacked) {
#pragma unroll
                for (int q = 0; q < kHistPer / 8; ++q) {
                    const uint4 l = *reinterpret_cast<const uint4*>(lens + i + 8 * q);
                    len[8 * q + 0] = l.x & 0xFFFFu; len[8 * q + 1] = l.x >> 16;
                    len[8 * q + 2] = l.y & 0xFFFFu; len[8 * q + 3] = l.y >> 16;
                    len[8 * q + 4] = l.z & 0xFFFFu; len[8 * q + 5] = l.z >> 16;
                    len[8 * q + 6] = l.w & 0xFFFFu; len[8 * q + 7] = l.w >> 16;
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < kHistPer; ++j) {
                rb[j] = i + j < pend ? (kPacked ? keys : verdict)[i + j] : 0u;
                if (!kPacked) len[j] = i + j < pend ? (uint32_t)lens[i + j] : 0u;
            }
        }
#pragma unroll
        for (int j = 0; j < kHistPer; ++j) {
            if (kPacked) {
                len[j] = rb[j] & 0xFFFFu;
                rb[j] = len[j] ? (rb[j] >> 16) + 1u : 0u;
            } else {
                rb[j] >>= 8;   // matched rule's sorted index + 1, 0 = none
            }
            if (rb[j] != 0 && rb[j] - 1u - r0 < range) atomicAdd(&h[rb[j] - 1u - r0], (1ull << 40) | len[j]);
        }
    }
    __syncthreads();
    // this chunk's bins, zeros included, as plain coalesced stores (upe_hist_reduce sums them
    // over the chunks; no device atomics)
    const uint32_t rend = nrules - r0 < range ? nrules : r0 + range;
    unsigned long long* o = part + (size_t)blockIdx.x * nrules + r0;
    for (uint32_t k = threadIdx.x; k < rend - r0; k += kHistBlock) o[k] = h[k];
}

// The dense group-by partials ([nchunks][nrules], packets << 40 | bytes) summed over the chunks:
// slice y of the grid sums chunks y, y + S, ... for rule r = blockIdx.x * 256 + thread and adds
// the unpacked totals to replica y % kStatReps of stats_idx; with S = kStatReps every replica
// word has exactly one writer in the launch, so the adds are plain.
__global__ void __launch_bounds__(256) upe_hist_reduce(const unsigned long long* part,
                                                       uint32_t nchunks, uint32_t nrules,
                                                       uint32_t nrules_pad,
                                                       unsigned long long* stats_idx) {
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= nrules) return;
    unsigned long long pk = 0, by = 0;
    uint32_t c = blockIdx.y;
    for (; c + 7 * gridDim.y < nchunks; c += 8 * gridDim.y) {
        unsigned long long b[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = part[(size_t)(c + j * gridDim.y) * nrules + r];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            pk += b[j] >> 40;
            by += b[j] & ((1ull << 40) - 1);
        }
    }
    for (; c < nchunks; c += gridDim.y) {
        const unsigned long long b = part[(size_t)c * nrules + r];
        pk += b >> 40;
        by += b & ((1ull << 40) - 1);
    }
    if (pk) {
        unsigned long long* o = stats_idx + (size_t)(blockIdx.y % kStatReps) * 2 * nrules_pad + 2 * (size_t)r;
        o[0] += pk;
        o[1] += by;
    }
}

// ------------------------------------------------------------------------------------------
// Egress list: the indexes of the packets with a given verdict code, in packet order (the order
// process_packet queues frames for tx_send_batch, reference src/worker.c:240-243).  Pass 1
// counts per block; pass 2 gives each block its offset (sum of the counts before it) and writes
// its indexes with wave ballots.
// ------------------------------------------------------------------------------------------
constexpr uint32_t kCompactBlock = 4096;   // packets per workgroup (256 threads x 16)

__global__ void __launch_bounds__(256) upe_compact_count(const uint32_t* verdict, uint32_t n,
                                                         uint32_t code, uint32_t* counts) {
    __shared__ uint32_t s_c;
    if (threadIdx.x == 0) s_c = 0;
    __syncthreads();
    const uint32_t p0 = blockIdx.x * kCompactBlock;
    uint32_t c = 0;
    for (uint32_t k = threadIdx.x; k < kCompactBlock; k += 256) {
        const uint32_t i = p0 + k;
        c += (i < n && (verdict[i] & 0xFu) == code) ? 1u : 0u;
    }
    c = wave_reduce<0>(c);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(&s_c, c);
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = s_c;
}

__global__ void __launch_bounds__(256) upe_compact_write(const uint32_t* verdict, uint32_t n,
                                                         uint32_t code, const uint32_t* counts,
                                                         uint32_t nblocks, uint32_t* index,
                                                         unsigned long long* total) {
    __shared__ uint32_t s_base;
    __shared__ uint32_t s_wave[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t pre = 0;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += 256) pre += counts[b];
    pre = wave_reduce<0>(pre);
    if (threadIdx.x == 0) s_base = 0;
    __syncthreads();
    if (lane == 0 && pre) atomicAdd(&s_base, pre);
    __syncthreads();
    uint32_t base = s_base;
    const uint32_t p0 = blockIdx.x * kCompactBlock;
    for (uint32_t k = 0; k < kCompactBlock; k += 256) {
        const uint32_t i = p0 + k + threadIdx.x;
        const bool m = i < n && (verdict[i] & 0xFu) == code;
        const unsigned long long bal = __ballot(m);
        if (lane == 0) s_wave[wave] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t off = base;
        for (int v = 0; v < wave; ++v) off += s_wave[v];
        const uint32_t rank = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        if (m) index[off + rank] = i;
        const uint32_t tot = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
        __syncthreads();
        base += tot;
    }
    if (blockIdx.x == nblocks - 1 && threadIdx.x == 0) *total = base;
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
thread_local std::string g_err;

int fail(const std::string& msg) {
    g_err = msg;
    return -1;
}

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail(std::string(#expr) + ": " + hipGetErrorString(e_));                  \
    } while (0)

// Makes the context's device current for the duration of an ABI call and restores the caller's
// current device on return (the ABI must not move the calling thread to another device).
struct DevScope {
    int prev = -1;
    hipError_t e;
    explicit DevScope(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        e = prev == d ? hipSuccess : hipSetDevice(d);
    }
    ~DevScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DevScope(const DevScope&) = delete;
    DevScope& operator=(const DevScope&) = delete;
};
#define DEV_SCOPE(dev)                                                                       \
    DevScope dev_scope_(dev);                                                                \
    HIP_TRY(dev_scope_.e)

uint32_t act_code(int32_t type) { return type == UPE_ACT_DROP ? 0u : type == UPE_ACT_FWD ? 1u : 2u; }
uint32_t mac_lo(const uint8_t* m) {
    return (uint32_t)m[0] | ((uint32_t)m[1] << 8) | ((uint32_t)m[2] << 16) | ((uint32_t)m[3] << 24);
}
uint32_t mac_hi(const uint8_t* m) { return (uint32_t)m[4] | ((uint32_t)m[5] << 8); }
uint32_t le32(const uint8_t* p) { return mac_lo(p); }

// ------------------------------------------------------------------------------------------
// Control packets that write a neighbour table (upe_gpu_process_segmented).  A packet is
// marked when handle_control_packet (reference src/worker.c:23-104) may call arp_update or
// ndp_update for it: ARP with the Ethernet/IPv4 header (the learn does not look at len), or an
// IPv6 NS/NA of at least 78 bytes (whether an option carries the address is decided on the
// host, from the gathered bytes).  Bytes at or past len read as zero (zero-filled pktbuf).
// Marks are verdict-shaped words (code 1 = marked) so upe_compact_* lists them in order.
// ------------------------------------------------------------------------------------------
constexpr uint32_t kCtrlWin = 256;   // bytes of each marked frame gathered for the host

__global__ void __launch_bounds__(256) upe_ctrl_mark(const uint8_t* frames, const uint64_t* desc,
                                                     uint32_t n, uint32_t* marks) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint64_t d = desc[i];
    const uint32_t len = (uint32_t)(d & 0xFFFFu);
    const uint8_t* p = frames + (d >> 16);
    auto at = [&](uint32_t k) -> uint32_t { return k < len ? (uint32_t)p[k] : 0u; };
    const uint32_t et = at(12) << 8 | at(13);
    uint32_t m = 0;
    if (et == 0x0806)
        m = at(14) == 0 && at(15) == 1 && at(16) == 8 && at(17) == 0 && at(18) == 6 && at(19) == 4;
    else if (et == 0x86DD && len >= 78u && at(20) == 58u && (at(54) == 135u || at(54) == 136u))
        m = 1;
    marks[i] = m;
}

// One workgroup per marked packet: its first kCtrlWin bytes (zero past len) and its length.
__global__ void __launch_bounds__(256) upe_ctrl_gather(const uint8_t* frames, const uint64_t* desc,
                                                       const uint32_t* index, uint8_t* win,
                                                       uint32_t* lens) {
    const uint32_t i = index[blockIdx.x];
    const uint64_t d = desc[i];
    const uint32_t len = (uint32_t)(d & 0xFFFFu);
    const uint32_t k = threadIdx.x;
    win[(size_t)blockIdx.x * kCtrlWin + k] = k < len ? frames[(d >> 16) + k] : (uint8_t)0;
    if (k == 0) lens[blockIdx.x] = len;
}

}  // namespace

// A small pool of host threads that run one job over slices: job(slice, slices), the caller
// being slice 0 (upe_gpu_process_host_emit applies the returned records to the caller's frames
// with it while later chunks are on the link).  Threads are pinned to the GPU's NUMA-local CPUs.
struct ApplyPool {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable go, done;
    std::function<void(unsigned, unsigned)> job;
    uint64_t gen = 0;
    unsigned left = 0;
    bool stop = false;

    ApplyPool(unsigned n, const std::vector<int>& cpus) {
        for (unsigned t = 0; t < n; ++t)
            th.emplace_back([this, t, n, cpus] {
                if (!cpus.empty()) {   // after the caller's CPU (local slot 0)
                    cpu_set_t one;
                    CPU_ZERO(&one);
                    CPU_SET(cpus[(1 + t) % cpus.size()], &one);
                    (void)pthread_setaffinity_np(pthread_self(), sizeof one, &one);
                }
                uint64_t seen = 0;
                for (;;) {
                    std::function<void(unsigned, unsigned)> f;
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        go.wait(lk, [&] { return stop || gen != seen; });
                        if (stop) return;
                        seen = gen;
                        f = job;
                    }
                    f(t + 1, n + 1);
                    std::lock_guard<std::mutex> lk(mu);
                    if (--left == 0) done.notify_one();
                }
            });
    }
    ~ApplyPool() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        go.notify_all();
        for (auto& t : th) t.join();
    }
    void run(const std::function<void(unsigned, unsigned)>& f) {
        {
            std::lock_guard<std::mutex> lk(mu);
            job = f;
            left = (unsigned)th.size();
            ++gen;
        }
        go.notify_all();
        f(0, (unsigned)th.size() + 1);
        std::unique_lock<std::mutex> lk(mu);
        done.wait(lk, [&] { return left == 0; });
    }
};

struct upe_gpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    size_t cap = 0;                // rule_stats capacity
    // rules
    RuleV4* rv4 = nullptr;
    RuleV6* rv6 = nullptr;
    int2* rinfo = nullptr;
    uint4* fam = nullptr;                      // FamTable image (linear-scan tables > kSmallRules)
    size_t fam_alloc = 0;                      // bytes
    uint32_t fam4 = 0, fam6 = 0;
    uint32_t fam_all = 0;
    // whether a packet of each family can be forwarded at all under the current table: some
    // rule it can reach first (up to its family's first catch-all) forwards
    bool fwd4 = true, fwd6 = true;
    uint32_t fam_x1idx = 0;
    // decision-tree index over the family lists (null / tree_ok false when not used)
    uint4* tree = nullptr;
    uint32_t tree_words = 0, tree_loff = 0;
    bool tree_ok = false;
    bool tree_stage = true;                    // stage the image in LDS when it fits
    upe_rule_index_info_t tree_info = {};
    size_t rules_alloc = 0;
    uint32_t nrules = 0, nrules_pad = 0;
    unsigned long long* stats_idx = nullptr;   // [rules_alloc][2] totals per sorted index
    bool host_tag = false;   // launches on behalf of a host-side loop (upe_gpu_tag_host)
    unsigned long long* hist_part = nullptr;   // [chunks][nrules_pad] dense group-by partials
    size_t hist_part_alloc = 0;
    void* gb = nullptr;                        // [gb_alloc] u32: group-by keys or u16 lengths
    size_t gb_alloc = 0;
    std::vector<int2> rinfo_host;              // (action, rule_id) per sorted index
    // tuple-space index of large tables (null when the linear scan is used)
    TssGroup* tg4 = nullptr;
    TssGroup* tg6 = nullptr;
    uint4* tt4 = nullptr;
    uint4* tt6 = nullptr;
    uint16_t* tfs = nullptr;          // staged fingerprint image
    uint32_t nfs = 0;                 // its length in uint4
    uint32_t ng4 = 0, ng6 = 0;
    bool tss = false;
    uint32_t* compact_counts = nullptr;   // upe_gpu_compact: per-block counts
    size_t compact_alloc = 0;
    // upe_gpu_process_segmented scratch: marks / index [ctrl_alloc], gathered windows
    uint32_t* ctrl_marks = nullptr;
    uint32_t* ctrl_index = nullptr;
    uint64_t* ctrl_count = nullptr;
    size_t ctrl_alloc = 0;
    uint8_t* ctrl_win = nullptr;
    uint32_t* ctrl_lens = nullptr;
    size_t ctrl_win_alloc = 0;
    // neighbour tables (reachable-entry indexes)
    uint4* arp = nullptr;
    uint32_t arp_bits = 0, arp_seed = 0;
    uint4* ndp = nullptr;
    uint32_t ndp_bits = 0, ndp_seed = 0;
    // state: one DevState allocation (see "Sequential state between batches")
    DevState* st = nullptr;
    uint64_t k = 0;                // launches so far: the next batch is batch k
    uint32_t last_n = 0;           // the last batch's size (batch_info)
    unsigned long long* stats = nullptr;   // [cap][2]
    TilePay* pay = nullptr;        // [2][paycap] per-workgroup last-hit payloads, by batch parity
    uint32_t paycap = 0;           // largest grid
    // per-batch scratch
    uint32_t* lb = nullptr;        // [tiles_alloc * kWaves] look-back flags (zeroed at allocation)
    uint32_t* defer = nullptr;     // [64 * tiles_alloc * kWaves] deferred look-back candidates
    size_t tiles_alloc = 0;
    uint32_t lb_spin = 5000;       // look-back wait before deferring (UPE_GPU_LB_SPIN, 100 MHz ticks)
    bool lb_sync = false;          // UPE_GPU_LB_SYNC=1: wait for each launch's agreement report
    bool allow_nolb = true;        // UPE_GPU_NOLB=0: never use the kernels without look-back
    int last_var = -1;             // kernel variant of the last classify launch
    uint32_t last_grid = 0;
    unsigned long long* ring_wg = nullptr;   // ring launches: per-batch counters + time origin
    size_t ring_alloc = 0;
    // every launch and state upload is ordered after the previous one, whatever its stream
    hipStream_t last_stream = nullptr;
    hipEvent_t order_ev = nullptr;
    int cus = 256;
    std::map<uint64_t, uint32_t> resident;   // persistent grid per (lds, tss, emit) (census)
    int blocks_per_cu_override = 0;   // UPE_GPU_BLOCKS_PER_CU (diagnostic)
    uint32_t port_mac_lo = 0, port_mac_hi = 0, port_ip4 = 0;
    bool have_batch = false;
    // kernel timing (upe_gpu_timing_*)
    bool timing = false;
    uint32_t timing_every = 1, timing_calls = 0;   // sample every n-th process() call
    uint32_t timing_phase = 0;     // samples open at calls c with c % timing_every == phase
    uint32_t timing_span = 1;      // calls one sample's event pair brackets
    uint32_t t_left = 0;           // calls left in the open sample (0: none open)
    uint64_t timing_launches = 0;  // calls covered by closed samples
    std::vector<hipEvent_t> ev;   // event pool, 2 per timed process() call
    size_t ev_used = 0;            // 3 per closed sample: start, after the classify, end
    std::vector<bool> ev_mid;      // per closed sample: the middle event was recorded
    // host round trip (upe_gpu_process_host): copy streams and three device slots
    hipStream_t s_in = nullptr, s_out = nullptr;
    struct HostSlot {
        uint8_t* frames = nullptr;
        size_t frames_cap = 0;
        uint64_t* desc = nullptr;
        uint32_t* verdict = nullptr;
        upe_hdr_rec_t* hdr = nullptr;   // emit-mode records (upe_gpu_process_host_emit)
        size_t pk_cap = 0;
        hipEvent_t in_done = nullptr, k_done = nullptr, out_done = nullptr;
        bool busy = false;
        uint64_t lo = 0, wb = 0;   // host byte range the slot's copy-back writes
    };
    HostSlot hs[8];
    // host threads applying emit-mode records to the caller's frames (upe_gpu_process_host_emit)
    std::unique_ptr<struct ApplyPool> pool;
    uint32_t host_slots = 4;       // device slots of the host round trip (UPE_GPU_HOST_SLOTS, 2..8)
    // the kernel without look-back (kNoLB): the launches' start-state agreement, written by the
    // device into host-mapped memory, and the first launch whose report counts
    hipEvent_t marks[4] = {};      // worker loop completion marks (upe_gpu_mark)
    unsigned long long* agree_h = nullptr;
    unsigned long long* agree_d = nullptr;
    uint64_t lb_reset_k = 0;
    bool no_lb = false;
};

namespace {

NeighIndex arp_index(const upe_gpu_ctx* c) { return NeighIndex{c->arp, c->arp_bits, c->arp_seed}; }
NeighIndex ndp_index(const upe_gpu_ctx* c) { return NeighIndex{c->ndp, c->ndp_bits, c->ndp_seed}; }

// Two-choice cuckoo placement of distinct keys (by their 32-bit hash key; different entries may
// share a hash key, the device compares the full address).  Starts at 2^bits >= 2.5 n slots and
// tries seeds, then doubles, until every key sits in slot1 or slot2.  bits = 0 for no keys.
template <class H>
int cuckoo_place_fn(size_t n, H hfn, uint32_t& bits, uint32_t& seed, std::vector<int32_t>& slot,
                    uint32_t ratio_x2 = 5);

// Three-choice cuckoo placement of the neighbour indexes' keys (slot1 / slot2 / slot3): starts at
// 2^bits >= 1.25 n slots, random-walk eviction, seeds tried, then doubles.  bits = 0 for no keys.
int cuckoo3_place(const std::vector<uint32_t>& key, uint32_t& bits, uint32_t& seed,
                  std::vector<int32_t>& slot) {
    const size_t n = key.size();
    slot.clear();
    bits = 0;
    seed = 0;
    if (n == 0) return 0;
    bits = 1;
    while (((size_t)1 << bits) * 4 < n * 5) ++bits;
    for (; bits <= 31; ++bits) {
        const size_t m = (size_t)1 << bits;
        for (uint32_t attempt = 0; attempt < 64; ++attempt) {
            const uint32_t sd = attempt * 0x6D2B79F5u + bits;
            slot.assign(m, -1);
            uint32_t rnd = sd | 1u;
            bool ok = true;
            for (size_t j = 0; j < n && ok; ++j) {
                int32_t cur = (int32_t)j;
                uint32_t from = ~0u;
                for (int kick = 0;; ++kick) {
                    const uint32_t c[3] = {slot1(key[cur], sd, bits), slot2(key[cur], sd, bits),
                                           slot3(key[cur], sd, bits)};
                    int placed = -1;
                    for (int q = 0; q < 3 && placed < 0; ++q)
                        if (slot[c[q]] < 0) placed = q;
                    if (placed >= 0) {
                        slot[c[placed]] = cur;
                        break;
                    }
                    if (kick >= 1000) {
                        ok = false;
                        break;
                    }
                    // evict a random choice other than the slot the key was just evicted from
                    rnd ^= rnd << 13; rnd ^= rnd >> 17; rnd ^= rnd << 5;
                    uint32_t q = rnd % 3u;
                    if (c[q] == from) q = (q + 1) % 3u;
                    std::swap(cur, slot[c[q]]);
                    from = c[q];
                }
            }
            if (ok) {
                seed = sd;
                return 0;
            }
        }
    }
    return -1;
}

// Same, with a seed-dependent 32-bit hash per key: hfn(j, seed).
template <class H>
int cuckoo_place_fn(size_t n, H hfn, uint32_t& bits, uint32_t& seed, std::vector<int32_t>& slot,
                    uint32_t ratio_x2) {
    std::vector<uint32_t> key(n);
    slot.clear();
    bits = 0;
    seed = 0;
    if (n == 0) return 0;
    bits = 1;
    while (((size_t)1 << bits) * 2 < n * ratio_x2) ++bits;
    for (; bits <= 31; ++bits) {
        const size_t m = (size_t)1 << bits;
        for (uint32_t attempt = 0; attempt < 64; ++attempt) {
            const uint32_t sd = attempt * 0x6D2B79F5u + bits;
            for (size_t j = 0; j < n; ++j) key[j] = hfn(j, sd);
            slot.assign(m, -1);
            bool ok = true;
            for (size_t j = 0; j < n && ok; ++j) {
                int32_t cur = (int32_t)j;
                uint32_t t = slot1(key[cur], sd, bits);
                for (int kick = 0;; ++kick) {
                    if (slot[t] < 0) {
                        slot[t] = cur;
                        break;
                    }
                    if (kick >= 500) {
                        ok = false;
                        break;
                    }
                    std::swap(cur, slot[t]);   // evict; the evicted key moves to its other slot
                    const uint32_t s1 = slot1(key[cur], sd, bits), s2 = slot2(key[cur], sd, bits);
                    t = t == s1 ? s2 : s1;
                }
            }
            if (ok) {
                seed = sd;
                return 0;
            }
        }
    }
    return -1;
}

// Point the DevState at the separately allocated arrays (after any of them is reallocated).
int publish(upe_gpu_ctx* c) {
    struct {
        TilePay* pay;
        uint32_t* lb;
        unsigned long long* stats;
        unsigned long long* stats_idx;
    } p = {c->pay, c->lb, c->stats, c->stats_idx};
    static_assert(offsetof(DevState, stats_idx) - offsetof(DevState, pay) == 3 * sizeof(void*),
                  "DevState pointer block");
    HIP_TRY(hipMemcpy(reinterpret_cast<char*>(c->st) + offsetof(DevState, pay), &p, sizeof p,
                      hipMemcpyHostToDevice));
    return 0;
}

int ensure_scratch(upe_gpu_ctx* c, size_t ntiles) {
    if (ntiles > c->tiles_alloc) {
        if (c->lb) (void)hipFree(c->lb);
        if (c->defer) (void)hipFree(c->defer);
        c->lb = nullptr;
        c->defer = nullptr;
        c->tiles_alloc = 0;
        size_t want = ntiles + ntiles / 4 + 16;
        HIP_TRY(hipMalloc(&c->lb, want * kWaves * sizeof(uint32_t)));
        HIP_TRY(hipMemset(c->lb, 0, want * kWaves * sizeof(uint32_t)));
        HIP_TRY(hipMalloc(&c->defer, 2 * 64 * want * kWaves * sizeof(uint32_t)));
        c->tiles_alloc = want;
        if (publish(c) != 0) return -1;
    }
    return 0;
}

// Order work about to be queued on `s` after everything queued so far on the context's state
// (the last launch, or a state upload), whatever stream that went to.
int order_on(upe_gpu_ctx* c, hipStream_t s) {
    if (c->last_stream && c->last_stream != s) {
        HIP_TRY(hipEventRecord(c->order_ev, c->last_stream));
        HIP_TRY(hipStreamWaitEvent(s, c->order_ev, 0));
    }
    c->last_stream = s;
    return 0;
}

// The state slots of batch k (DevState comment).
DevL1* l1_slot(upe_gpu_ctx* c, uint64_t k) { return &c->st->l1[k % 2].s; }
BatchAcc* acc_slot(upe_gpu_ctx* c, uint64_t k) { return &c->st->acc[k % 3]; }
TilePay* pay_slot(upe_gpu_ctx* c, uint64_t k) { return c->pay + (size_t)(k % 2) * c->paycap; }

// Does the L1 state the next batch starts from agree with the tables?  (After l1_sync.)
int refresh(upe_gpu_ctx* c) {
    if (order_on(c, c->stream) != 0) return -1;
    c->no_lb = false;   // the entries may disagree with the new tables until a launch says not
    c->lb_reset_k = c->k;
    hipLaunchKernelGGL(upe_refresh, dim3(1), dim3(64), 0, c->stream, l1_slot(c, c->k),
                       arp_index(c), ndp_index(c));
    HIP_TRY(hipGetLastError());
    return 0;
}

// Fold the last batch's L1 outcome into l1[k % 2], the state the next batch starts from (and
// clear it from that batch's accumulators, so the next launch does not fold it again).
int l1_sync(upe_gpu_ctx* c) {
    if (c->k == 0) return 0;
    if (order_on(c, c->stream) != 0) return -1;
    hipLaunchKernelGGL(upe_l1_sync, dim3(1), dim3(64), 0, c->stream, l1_slot(c, c->k),
                       acc_slot(c, c->k + 2), pay_slot(c, c->k + 1));
    HIP_TRY(hipGetLastError());
    return 0;
}

// The between-batch state of a fresh context (a calloc'd worker_t): L1 all zero, accumulators
// armed (nothing happened), totals zero.
int arm_state(upe_gpu_ctx* c) {
    if (order_on(c, c->stream) != 0) return -1;
    static DevState init;   // zero, then the armed accumulator fields
    for (auto& acc : init.acc) acc.grid = 1;   // every other word zero: nothing happened
    HIP_TRY(hipMemcpyAsync(c->st, &init, offsetof(DevState, pay), hipMemcpyHostToDevice,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->k = 0;
    c->last_n = 0;
    c->no_lb = false;
    c->lb_reset_k = 0;
    return 0;
}


hipStream_t pick(upe_gpu_ctx* c, void* s) { return s ? (hipStream_t)s : c->stream; }

constexpr int kVarCount = 256;
// Kernel variants: bit 0 emit, bit 1 tuple space, bit 2 lean, bit 3 no look-back (lean only),
// bit 4 ring (lean emit linear scan only), bit 5 a host path's launch (upe_gpu_process_mapped /
// upe_gpu_process_host; not ring), bits 4 and 5 together the egress-list kernels (emit, device
// batches; upe_gpu_process_emit_tx), bits 6-7 how a linear-scan table past kSmallRules is matched
// (never with tuple space): 1 its family lists (FamTable), 2 the whole table through the scalar
// unit, 3 the decision tree over the family lists.
enum { VAR_EMIT = 1, VAR_TSS = 2, VAR_LEAN = 4, VAR_NOLB = 8, VAR_RING = 16, VAR_HOST = 32,
       VAR_FAM = 64, VAR_GLB = 128, VAR_TREE = 192, VAR_SCAN = 192 };
// scan: 0 small table (LDS copy), 1 family lists, 2 whole table through the scalar unit, 3 tree
int classify_var(bool tss, bool emit, bool lean, bool nolb, bool ring = false, bool host = false,
                 int scan = 0, bool tx = false) {
    return (!tss ? (scan & 3) * VAR_FAM : 0) |
           (tx ? VAR_RING | VAR_HOST : (host && !ring ? VAR_HOST : 0) | (ring ? VAR_RING : 0)) |
           (lean && nolb ? VAR_NOLB : 0) | (lean ? VAR_LEAN : 0) | (tss ? VAR_TSS : 0) |
           (emit ? VAR_EMIT : 0);
}
// The instantiated variants (every combination classify_var can return for a launch).
constexpr bool var_built(int v) {
    const bool emit = v & VAR_EMIT, lean = v & VAR_LEAN, nolb = v & VAR_NOLB, ring = v & VAR_RING,
               host = v & VAR_HOST;
    if (nolb && !lean) return false;
    if ((v & VAR_SCAN) && (v & VAR_TSS)) return false;
    if (ring && host) return emit;   // the egress-list kernels
    if (ring) return emit && lean && !(v & VAR_TSS);
    return true;
}
template <int V>
const void* classify_fn_of() {
    if constexpr (var_built(V))
        return reinterpret_cast<const void*>(
            &upe_classify<(V & VAR_TSS) != 0, (V & VAR_EMIT) != 0, (V & VAR_LEAN) != 0,
                          (V & VAR_NOLB) != 0, (V & VAR_RING) != 0, (V & VAR_HOST) != 0,
                          (V & VAR_SCAN) / VAR_FAM>);
    else
        return nullptr;
}
template <int... V>
constexpr std::array<const void* (*)(), sizeof...(V)> classify_table(std::integer_sequence<int, V...>) {
    return {{&classify_fn_of<V>...}};
}
const void* classify_fn(int var) {
    static const auto fns = classify_table(std::make_integer_sequence<int, kVarCount>{});
    return var >= 0 && var < kVarCount ? fns[var]() : nullptr;
}

void launch_classify(int var, uint32_t grid, size_t lds, hipStream_t s, const Args& a) {
    // dynamic LDS beyond 64 KB must be allowed per kernel and device (once per device)
    static std::atomic<uint64_t> lds_attr{0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    const uint64_t bit = 1ull << (dev & 63);
    if (!(lds_attr.fetch_or(bit) & bit))
        for (int v = 0; v < kVarCount; ++v)
            if (classify_fn(v))
                (void)hipFuncSetAttribute(classify_fn(v), hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)((v & VAR_SCAN) && !(v & VAR_TSS) ? kLdsDynMaxLarge
                                                                                 : kLdsDynMax));
    Args arg = a;
    void* args[] = {&arg};
    (void)hipLaunchKernel(classify_fn(var), dim3(grid), dim3(kBlock), args, lds, s);
}

// The persistent grid of a kernel configuration: the occupancy API's answer, checked by a census
// launch the first time the configuration is used (census_probe).  0 on error.
uint32_t resident_grid(upe_gpu_ctx* c, int var, size_t lds, hipStream_t s) {
    static_assert(kVarCount <= 256, "the variant takes the key's low 8 bits");
    const uint64_t key = (uint64_t)lds << 8 | (uint64_t)var;
    auto it = c->resident.find(key);
    if (it != c->resident.end()) return it->second;
    int per_cu = 0;
    hipError_t e;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, classify_fn(var), kBlock, lds);
    if (e != hipSuccess) {
        fail(std::string("hipOccupancyMaxActiveBlocksPerMultiprocessor: ") + hipGetErrorString(e));
        return 0;
    }
    if (per_cu < 1) per_cu = 1;
    uint32_t grid = (uint32_t)per_cu * (uint32_t)c->cus;
    if (c->blocks_per_cu_override > 0) {
        grid = (uint32_t)c->blocks_per_cu_override * (uint32_t)c->cus;   // diagnostic
    } else {
        if (grid > c->paycap) grid = c->paycap;
        Args a;
        memset(&a, 0, sizeof a);
        a.census = 1;
        a.st = c->st;
        uint32_t* w = &c->st->census[0];
        const uint32_t init[2] = {0u, kNone};
        if (hipMemcpyAsync(w, init, sizeof init, hipMemcpyHostToDevice, s) != hipSuccess) {
            fail("census upload failed");
            return 0;
        }
        launch_classify(var, grid, lds, s, a);
        uint32_t out[2] = {0u, 0u};
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(out, w, sizeof out, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            fail("census launch failed");
            return 0;
        }
        if (out[1] != kNone && out[1] < grid) {
            // round down to whole workgroups per CU
            const uint32_t per = out[1] / (uint32_t)c->cus;
            grid = (per ? per : 1u) * (uint32_t)c->cus;
        }
    }
    if (grid > c->paycap) grid = c->paycap;
    c->resident[key] = grid;
    if (getenv("UPE_GPU_VERBOSE"))
        fprintf(stderr, "upe_gpu: persistent grid %u (occupancy API %d per CU, lds %zu, kernel "
                "variant %d)\n", grid, per_cu, lds, var);
    return grid;
}

}  // namespace

extern "C" {

const char* upe_gpu_last_error(void) { return g_err.c_str(); }

// For the library's C parts (upe_worker.c): set the calling thread's message, return -1.  Not
// declared in include/upe_gpu.h and not exported.
__attribute__((visibility("hidden"))) int upe_gpu_set_last_error(const char* msg) {
    return fail(msg ? msg : "");
}

int upe_gpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return -1;
    return n;
}

// The process's allowed CPUs as they were when the library was loaded (before any thread of it
// was pinned: a pinned thread's own mask is one CPU).
static cpu_set_t g_process_cpus;
__attribute__((constructor)) static void upe_capture_cpus() {
    CPU_ZERO(&g_process_cpus);
    if (sched_getaffinity(0, sizeof g_process_cpus, &g_process_cpus) != 0)
        for (int c = 0; c < CPU_SETSIZE; ++c) CPU_SET(c, &g_process_cpus);
}

// The host CPUs local to a GPU: the device's PCI function in sysfs names its NUMA node and the
// CPUs attached to it (local_cpulist), kept in the process's allowed set.
int upe_gpu_local_cpus(int device, int* cpus, size_t cap, int* numa_node) {
    char bus[64] = {0};
    HIP_TRY(hipDeviceGetPCIBusId(bus, (int)sizeof bus, device));
    for (char* p = bus; *p; ++p) *p = (char)tolower((unsigned char)*p);
    const std::string dir = std::string("/sys/bus/pci/devices/") + bus;
    int node = -1;
    if (FILE* f = fopen((dir + "/numa_node").c_str(), "r")) {
        if (fscanf(f, "%d", &node) != 1) node = -1;
        fclose(f);
    }
    if (numa_node) *numa_node = node;
    std::string list;
    if (FILE* f = fopen((dir + "/local_cpulist").c_str(), "r")) {
        char buf[4096];
        if (fgets(buf, sizeof buf, f)) list = buf;
        fclose(f);
    }
    if (list.empty()) return fail("no local_cpulist for PCI device " + std::string(bus));
    const cpu_set_t& allowed = g_process_cpus;
    size_t n = 0;
    const char* p = list.c_str();
    while (*p) {   // "0-63,128-191"
        char* e = nullptr;
        const long lo = strtol(p, &e, 10);
        if (e == p) break;
        long hi = lo;
        p = e;
        if (*p == '-') {
            hi = strtol(p + 1, &e, 10);
            p = e;
        }
        for (long c = lo; c <= hi; ++c)
            if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &allowed)) {
                if (cpus && n < cap) cpus[n] = (int)c;
                ++n;
            }
        while (*p == ',' || *p == '\n' || *p == ' ') ++p;
    }
    return (int)n;
}

// Pin the calling thread to one CPU local to `device` (the slot-th of them, modulo their
// number) — the reference pins each worker thread with affinity_pin_self (src/affinity.c:48,
// cores from assign_cores, src/main.c:143-175); a GPU worker's host thread belongs on the GPU's
// NUMA node, where its pinned buffers are then allocated.  Returns the CPU.
int upe_gpu_pin_self(int device, int slot) {
    std::vector<int> cpus(CPU_SETSIZE);
    const int n = upe_gpu_local_cpus(device, cpus.data(), cpus.size(), nullptr);
    if (n <= 0) return n == 0 ? fail("no allowed CPU is local to the device") : -1;
    const int cpu = cpus[(size_t)(slot < 0 ? 0 : slot) % (size_t)n];
    cpu_set_t one;
    CPU_ZERO(&one);
    CPU_SET(cpu, &one);
    if (pthread_setaffinity_np(pthread_self(), sizeof one, &one) != 0)
        return fail("pthread_setaffinity_np failed");
    return cpu;
}

upe_gpu_ctx_t* upe_gpu_open(int device, size_t rule_capacity) {
    if (rule_capacity == 0 || rule_capacity > (1u << 24)) {
        fail("rule_capacity must be in [1, 2^24]");
        return nullptr;
    }
    upe_gpu_ctx* c = new (std::nothrow) upe_gpu_ctx();
    if (!c) {
        fail("out of memory");
        return nullptr;
    }
    c->device = device;
    c->cap = rule_capacity;
    auto bad = [&](hipError_t e, const char* what) {
        fail(std::string(what) + ": " + hipGetErrorString(e));
        upe_gpu_close(c);
        return nullptr;
    };
    DevScope dg(device);
    hipError_t e;
    if ((e = dg.e) != hipSuccess) return bad(e, "hipSetDevice");
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess)
        return bad(e, "hipStreamCreate");
    if ((e = hipEventCreateWithFlags(&c->order_ev, hipEventDisableTiming)) != hipSuccess)
        return bad(e, "hipEventCreate");
    if ((e = hipMalloc(&c->st, sizeof(DevState))) != hipSuccess) return bad(e, "hipMalloc state");
    if ((e = hipMemset(c->st, 0, sizeof(DevState))) != hipSuccess) return bad(e, "hipMemset");
    if ((e = hipMalloc(&c->stats, rule_capacity * 2 * sizeof(unsigned long long))) != hipSuccess)
        return bad(e, "hipMalloc stats");
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) ==
                hipSuccess && cus > 0)
            c->cus = cus;
        if (const char* v = getenv("UPE_GPU_BLOCKS_PER_CU")) c->blocks_per_cu_override = atoi(v);
        // diagnostics: the look-back wait before deferring (0 = defer whenever a flag is not yet
        // published), a synchronous agreement report per launch (the switch to the kernel without
        // look-back then happens at a deterministic launch), no kernel without look-back
        if (const char* v = getenv("UPE_GPU_LB_SPIN")) c->lb_spin = (uint32_t)strtoul(v, nullptr, 10);
        if (const char* v = getenv("UPE_GPU_LB_SYNC")) c->lb_sync = v[0] == '1';
        if (const char* v = getenv("UPE_GPU_NOLB")) c->allow_nolb = v[0] != '0';
        if (const char* v = getenv("UPE_GPU_HOST_SLOTS"))
            c->host_slots = std::min(8u, std::max(2u, (uint32_t)strtoul(v, nullptr, 10)));
    }
    // payload slots for the largest grid a launch uses (at most 8 workgroups per CU)
    c->paycap = 8u * (uint32_t)c->cus;
    if ((e = hipMalloc(&c->pay, 2 * (size_t)c->paycap * sizeof(TilePay))) != hipSuccess)
        return bad(e, "hipMalloc payloads");
    if ((e = hipMemset(c->pay, 0, 2 * (size_t)c->paycap * sizeof(TilePay))) != hipSuccess)
        return bad(e, "hipMemset");
    // host-mapped report of each launch's start-state agreement (the kernel without look-back
    // is used once one arrives; without it, every launch keeps the look-back)
    if (hipHostMalloc(reinterpret_cast<void**>(&c->agree_h), sizeof(unsigned long long),
                      hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
        *c->agree_h = 0;
        if (hipHostGetDevicePointer(reinterpret_cast<void**>(&c->agree_d), c->agree_h, 0) !=
            hipSuccess) {
            (void)hipHostFree(c->agree_h);
            c->agree_h = nullptr;
            c->agree_d = nullptr;
        }
    } else {
        c->agree_h = nullptr;
    }
    if (arm_state(c) != 0) {
        std::string m = g_err;
        upe_gpu_close(c);
        g_err = m;
        return nullptr;
    }
    if ((e = hipMemsetAsync(c->stats, 0, rule_capacity * 2 * sizeof(unsigned long long),
                            c->stream)) != hipSuccess)
        return bad(e, "hipMemsetAsync");
    // An empty rule table: one padding block of never-matching rules.
    if (upe_gpu_load_rules(c, nullptr, 0) != 0) {
        std::string m = g_err;
        upe_gpu_close(c);
        g_err = m;
        return nullptr;
    }
    if (upe_gpu_load_neigh(c, nullptr, 0, nullptr, 0) != 0 || refresh(c) != 0) {
        std::string m = g_err;
        upe_gpu_close(c);
        g_err = m;
        return nullptr;
    }
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return bad(e, "sync");
    return c;
}

void upe_gpu_close(upe_gpu_ctx_t* c) {
    if (!c) return;
    DevScope dg(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    void* bufs[] = {c->rv4, c->rv6, c->rinfo, c->stats_idx, c->gb, c->arp, c->ndp, c->st, c->stats,
                    c->pay, c->lb, c->tg4, c->tg6, c->tt4, c->tt6, c->tfs, c->fam, c->tree,
                    c->compact_counts,
                    c->ctrl_marks, c->ctrl_index, c->ctrl_count, c->ctrl_win, c->ctrl_lens,
                    c->hist_part};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (c->defer) (void)hipFree(c->defer);
    if (c->ring_wg) (void)hipFree(c->ring_wg);
    for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
    if (c->order_ev) (void)hipEventDestroy(c->order_ev);
    for (hipEvent_t e : c->marks)
        if (e) (void)hipEventDestroy(e);
    for (auto& sl : c->hs) {
        for (void* b : {(void*)sl.frames, (void*)sl.desc, (void*)sl.verdict, (void*)sl.hdr})
            if (b) (void)hipFree(b);
        for (hipEvent_t e : {sl.in_done, sl.k_done, sl.out_done})
            if (e) (void)hipEventDestroy(e);
    }
    if (c->s_in) (void)hipStreamSynchronize(c->s_in), (void)hipStreamDestroy(c->s_in);
    if (c->s_out) (void)hipStreamSynchronize(c->s_out), (void)hipStreamDestroy(c->s_out);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->agree_h) (void)hipHostFree(c->agree_h);
    delete c;
}

namespace {
// Credit the sorted-index totals of the current table to rule_stats[rule_id] (device) and clear
// them: called before upe_gpu_load_rules changes the table, so the counts carry over by rule_id
// (upe_gpu_reload_rules instead starts a fresh rule_stats, as the reference's SIGHUP reload does).
// Every table size keeps its counts per sorted index: small tables in the per-batch replicated
// accumulators (acc_stats, added here), mid-size ones in kStatReps replicas (each workgroup's LDS
// bins) and large ones too (upe_rule_hist).  The host sums the replicas and credits rule_id.
int read_stats_idx(upe_gpu_ctx* c, std::vector<unsigned long long>& idx) {
    const size_t E = 2 * (size_t)c->nrules_pad;
    std::vector<unsigned long long> all(E * kStatReps);
    HIP_TRY(hipMemcpy(all.data(), c->stats_idx, all.size() * sizeof(unsigned long long),
                      hipMemcpyDeviceToHost));
    idx.assign(E, 0);
    for (size_t r = 0; r < (size_t)kStatReps; ++r)
        for (size_t e = 0; e < E; ++e) idx[e] += all[r * E + e];
    if (E <= 2 * (size_t)kSmallRules) {
        // small tables: the classify kernel's replicated per-sorted-index totals
        std::vector<unsigned long long> sm((size_t)kReps * 2 * kSmallRules);
        HIP_TRY(hipMemcpy(sm.data(), &c->st->acc_stats[0][0], sm.size() * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost));
        for (size_t r = 0; r < (size_t)kReps; ++r)
            for (size_t e = 0; e < E; ++e) idx[e] += sm[r * 2 * kSmallRules + e];
    }
    return 0;
}

int fold_stats_idx(upe_gpu_ctx* c) {
    if (!c->stats_idx || c->rinfo_host.empty()) return 0;
    const size_t E = 2 * (size_t)c->nrules_pad;
    std::vector<unsigned long long> idx, st(2 * c->cap);
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (read_stats_idx(c, idx) != 0) return -1;
    bool any = false;
    for (unsigned long long v : idx) any |= v != 0;
    if (!any) return 0;
    HIP_TRY(hipMemcpy(st.data(), c->stats, st.size() * sizeof(unsigned long long),
                      hipMemcpyDeviceToHost));
    for (size_t e = 0; e < E; ++e)
        if (idx[e]) st[2 * (size_t)(uint32_t)c->rinfo_host[e >> 1].y + (e & 1)] += idx[e];
    HIP_TRY(hipMemcpy(c->stats, st.data(), st.size() * sizeof(unsigned long long),
                      hipMemcpyHostToDevice));
    HIP_TRY(hipMemset(c->stats_idx, 0, E * kStatReps * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(&c->st->acc_stats[0][0], 0, sizeof(c->st->acc_stats)));
    return 0;
}

// rule_stats[0..capacity) as the worker holds them: the per-rule_id array plus the current
// table's per-sorted-index totals credited to their rule_id (after a device synchronisation).
int read_rule_stats(upe_gpu_ctx* c, upe_rule_stat_t* rule_stats, size_t capacity) {
    const size_t k = capacity < c->cap ? capacity : c->cap;
    memset(rule_stats, 0, capacity * sizeof(upe_rule_stat_t));
    HIP_TRY(hipMemcpy(rule_stats, c->stats, k * sizeof(upe_rule_stat_t), hipMemcpyDeviceToHost));
    if (c->stats_idx && !c->rinfo_host.empty()) {
        const size_t E = 2 * (size_t)c->nrules_pad;
        std::vector<unsigned long long> idx;
        if (read_stats_idx(c, idx) != 0) return -1;
        for (size_t e = 0; e < E; ++e) {
            const uint32_t rid = (uint32_t)c->rinfo_host[e >> 1].y;
            if (!idx[e] || rid >= k) continue;
            if (e & 1) rule_stats[rid].bytes += idx[e];
            else rule_stats[rid].packets += idx[e];
        }
    }
    return 0;
}
}  // namespace

}  // extern "C"

namespace {
// Tuple-space index of the compiled rules (see TssGroup).  Returns false when the table is
// better served by the linear scan: small tables, or too many distinct mask signatures.
struct TssFamily {
    std::vector<TssGroup> groups;
    std::vector<uint4> slots;
    std::vector<uint16_t> fp;   // one per slot
};

bool build_tss_family(int F, const std::vector<RuleV4>& v4, const std::vector<RuleV6>& v6,
                      const upe_rule_t* rules, size_t count, TssFamily& out) {
    const int nw = F == 4 ? 4 : 10;
    using Sig = std::array<uint32_t, 10>;
    using Key = std::array<uint32_t, 10>;
    struct Grp {
        uint32_t minidx = kNone;
        std::map<Key, uint32_t> keys;   // masked key -> smallest sorted index
    };
    std::map<Sig, Grp> groups;
    for (size_t i = 0; i < count; ++i) {
        const uint8_t ver = rules[i].ip_ver;
        if (ver != 0 && ver != F) continue;
        const RuleV4& r = v4[i];
        const RuleV6& q = v6[i];
        Sig sg{};
        Key k{};
        sg[0] = r.m0 & ~0xFFu;
        sg[1] = r.m1 & 0xFFFFu;
        sg[2] = r.sm0;
        sg[3] = r.dm0;
        k[0] = r.x0 & sg[0];
        k[1] = r.x1 & sg[1];
        k[2] = r.s0;
        if (F == 4) {
            k[3] = r.d0;
        } else {
            for (int j = 0; j < 3; ++j) {
                sg[4 + j] = q.sm[j];
                sg[7 + j] = q.dm[j];
            }
            k[3] = q.s[0]; k[4] = q.s[1]; k[5] = q.s[2];
            k[6] = r.d0;
            k[7] = q.d[0]; k[8] = q.d[1]; k[9] = q.d[2];
        }
        Grp& g = groups[sg];
        if (g.minidx == kNone) g.minidx = (uint32_t)i;
        g.keys.emplace(k, (uint32_t)i);   // first insertion = smallest sorted index
    }
    std::vector<std::pair<uint32_t, const std::pair<const Sig, Grp>*>> order;
    for (const auto& kv : groups) order.push_back({kv.second.minidx, &kv});
    std::sort(order.begin(), order.end(),
              [](const auto& x, const auto& y) { return x.first < y.first; });
    const int per = F == 4 ? kTssSlot4 : kTssSlot6;
    out.groups.clear();
    out.slots.clear();
    for (const auto& o : order) {
        const Sig& sg = o.second->first;
        const Grp& g = o.second->second;
        std::vector<Key> keys;
        std::vector<uint32_t> idx;
        for (const auto& kv : g.keys) {
            keys.push_back(kv.first);
            idx.push_back(kv.second);
        }
        uint32_t bits = 0, seed = 0;
        std::vector<int32_t> slot;
        if (cuckoo_place_fn(keys.size(),
                            [&](size_t j, uint32_t sd) { return tss_hash(keys[j].data(), nw, sd); },
                            bits, seed, slot, kTssRatioX2) != 0)
            return false;
        TssGroup d;
        memset(&d, 0, sizeof d);
        for (int j = 0; j < 10; ++j) d.w[j] = sg[j];
        d.w[10] = g.minidx;
        d.w[11] = bits;
        d.w[12] = seed;
        d.w[13] = (uint32_t)(out.slots.size() / per);
        bool wild = true;
        for (int j = 0; j < 10; ++j) wild = wild && sg[j] == 0;
        if (wild && idx.size() == 1)
            d.w[14] = 1u | (act_code(rules[idx[0]].action.type) << 8);
        out.groups.push_back(d);
        const size_t base = out.slots.size();
        out.slots.resize(base + slot.size() * per, make_uint4(0, 0, 0, 0));
        const size_t fbase = out.fp.size();
        out.fp.resize(fbase + slot.size(), 0);
        for (size_t t = 0; t < slot.size(); ++t) {
            if (slot[t] < 0) continue;
            const Key& k = keys[slot[t]];
            out.fp[fbase + t] = tss_tag(tss_hash(k.data(), nw, seed));
            uint4* e = &out.slots[base + t * per];
            const uint32_t act = act_code(rules[idx[slot[t]]].action.type);
            if (F == 4) {
                const uint32_t v = (idx[slot[t]] + 1u) | act << 22;
                e[0] = make_uint4(k[0] | (v & 0xFFu), k[1] | ((v >> 8) << 16), k[2], k[3]);
            } else {
                e[0] = make_uint4(k[0], k[1], k[2], k[3]);
                e[1] = make_uint4(k[4], k[5], k[6], k[7]);
                e[2] = make_uint4(k[8], k[9], idx[slot[t]], 1u | (act << 8));
            }
        }
    }
    return true;
}

// ---- decision-tree index (round 5; TreeNode comment) ----------------------------------------
// The conservative range of one rule of a family list on one key word: lo = x & m, hi = x | ~m
// (within the word's width); `exact` when ~m is a run of low bits (prefix, exact value or
// wildcard), so that the range is exactly the set of values the rule accepts on that word.
struct TreeRule {
    uint32_t lo[kTreeDims], hi[kTreeDims];
    uint16_t exact;   // bit d: word d's range is exact
};
constexpr uint32_t kTreeWidth[kTreeDims] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                            0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                            0xFFFFu, 0xFFFFu, 0xFFu};
// A family list entry (RuleV4 words, plus the IPv6 words for family 6) as key-word ranges.  IPv4
// word 0 is host order already (src/parser.c:40-41) and its other address words are 0 in the key.
// An IPv6 address word is compared big-endian (a prefix is then a range) when bit j (source word
// j) or 4 + j (destination word j) of swap6 is set, else as loaded: a version-agnostic rule's
// IPv4 prefix (host order, src/rule_config.c:60-66) is a range only that way (tree_swap6).
uint32_t word_of(uint32_t v, uint32_t swap6, int j) { return (swap6 >> j & 1u) ? bswap32(v) : v; }
TreeRule tree_rule(int F, const RuleV4& r, const RuleV6* q, uint32_t swap6 = 0xFFu) {
    TreeRule t;
    uint32_t x[kTreeDims] = {}, m[kTreeDims] = {};
    if (F == 4) {
        x[0] = r.s0; m[0] = r.sm0;
        x[4] = r.d0; m[4] = r.dm0;
    } else {
        for (int j = 0; j < 4; ++j) {
            const uint32_t xs = j ? q->s[j - 1] : r.s0, ms = j ? q->sm[j - 1] : r.sm0;
            const uint32_t xd = j ? q->d[j - 1] : r.d0, md = j ? q->dm[j - 1] : r.dm0;
            x[j] = word_of(xs, swap6, j); m[j] = word_of(ms, swap6, j);
            x[4 + j] = word_of(xd, swap6, 4 + j); m[4 + j] = word_of(md, swap6, 4 + j);
        }
    }
    x[8] = r.x0 >> 16; m[8] = r.m0 >> 16;
    x[9] = r.x1 & 0xFFFFu; m[9] = r.m1 & 0xFFFFu;
    x[10] = (r.x0 >> 8) & 0xFFu; m[10] = (r.m0 >> 8) & 0xFFu;
    t.exact = 0;
    for (int d = 0; d < kTreeDims; ++d) {
        const uint32_t w = kTreeWidth[d], inv = ~m[d] & w;
        t.lo[d] = x[d] & m[d] & w;
        t.hi[d] = (x[d] & w) | inv;
        if ((inv & (inv + 1u)) == 0) t.exact |= (uint16_t)(1u << d);
    }
    return t;
}

struct TreeImage {
    std::vector<uint2> nodes;
    std::vector<uint32_t> leaves;
    uint32_t trees[2] = {0, 0};      // trees per family
    uint32_t depth[2] = {0, 0};      // deepest leaf per family
    uint32_t max_leaf = 0;           // longest leaf list
    uint32_t swap6 = 0xFFu;          // IPv6 address words compared big-endian (tree_rule)
};

// The byte order of each IPv6 address word under which more of the family's rules are ranges
// (exact): big-endian for IPv6 prefixes, as loaded for version-agnostic IPv4 prefixes in the
// IPv6 list (config C's 10 %); ties big-endian.
uint32_t tree_swap6(const std::vector<RuleV4>& v4, const std::vector<RuleV6>& v6,
                    const std::vector<uint32_t>& l6) {
    auto exact = [](uint32_t m) { const uint32_t inv = ~m; return (inv & (inv + 1u)) == 0; };
    uint32_t swap6 = 0;
    for (int w = 0; w < 8; ++w) {
        const int j = w & 3;
        long votes = 0;
        for (uint32_t i : l6) {
            const uint32_t m = w < 4 ? (j ? v6[i].sm[j - 1] : v4[i].sm0)
                                     : (j ? v6[i].dm[j - 1] : v4[i].dm0);
            votes += (long)exact(bswap32(m)) - (long)exact(m);
        }
        if (votes >= 0) swap6 |= 1u << w;
    }
    return swap6;
}

// HyperSplit-style build of one family's tree into img (breadth first, so the top levels are
// contiguous).  rules: the family list's entries in list order.  Returns false when the node
// budget or the leaf-length limit is exceeded (the table then keeps the linear scan).
bool build_tree_family(const std::vector<TreeRule>& R, const std::vector<uint32_t>& members,
                       int fam_slot, uint32_t binth, size_t node_budget, TreeImage& img,
                       uint32_t dims = (1u << kTreeDims) - 1u) {
    struct Task {
        uint32_t node;
        uint32_t depth;
        std::array<uint32_t, kTreeDims> lo, hi;
        std::vector<uint32_t> list;
    };
    const uint32_t root = (uint32_t)img.nodes.size();
    img.nodes.push_back(make_uint2(0, 0));
    std::deque<Task> q;
    Task t0;
    t0.node = root;
    t0.depth = 0;
    for (int d = 0; d < kTreeDims; ++d) {
        t0.lo[d] = 0;
        t0.hi[d] = kTreeWidth[d];
    }
    t0.list = members;
    q.push_back(std::move(t0));
    std::vector<uint32_t> los, his, cand;
    while (!q.empty()) {
        Task t = std::move(q.front());
        q.pop_front();
        // keep the rules up to the first one that matches every key of the box
        std::vector<uint32_t>& L = t.list;
        std::vector<uint8_t> covers(L.size(), 0);
        for (size_t j = 0; j < L.size(); ++j) {
            const TreeRule& r = R[L[j]];
            bool cov = true;
            for (int d = 0; d < kTreeDims && cov; ++d)
                cov = (r.exact >> d & 1u) && r.lo[d] <= t.lo[d] && r.hi[d] >= t.hi[d];
            if (cov) {
                covers[j] = 1;
                L.resize(j + 1);
                covers.resize(j + 1);
                break;
            }
        }
        const uint32_t n = (uint32_t)L.size();
        int best_d = -1;
        uint32_t best_t = 0, best_max = n, best_sum = 2 * n;
        if (n > binth && !covers[0]) {
            for (int d = 0; d < kTreeDims; ++d) {
                if (!(dims >> d & 1u)) continue;
                los.clear();
                his.clear();
                bool split = false;
                for (uint32_t j : L) {
                    const uint32_t lo = std::max(R[j].lo[d], t.lo[d]);
                    const uint32_t hi = std::min(R[j].hi[d], t.hi[d]);
                    los.push_back(lo);
                    his.push_back(hi);
                    split |= lo > t.lo[d] || hi < t.hi[d];
                }
                if (!split) continue;
                std::sort(los.begin(), los.end());
                std::sort(his.begin(), his.end());
                cand.clear();
                for (uint32_t v : los)
                    if (v > t.lo[d]) cand.push_back(v);
                for (uint32_t v : his)
                    if (v < t.hi[d]) cand.push_back(v + 1u);
                std::sort(cand.begin(), cand.end());
                cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
                size_t il = 0, ih = 0;
                for (uint32_t c : cand) {
                    while (il < los.size() && los[il] < c) ++il;   // rules reaching below c
                    while (ih < his.size() && his[ih] < c) ++ih;   // rules ending below c
                    const uint32_t nl = (uint32_t)il, nr = n - (uint32_t)ih;
                    const uint32_t mx = std::max(nl, nr), sm = nl + nr;
                    if (mx < best_max || (mx == best_max && sm < best_sum)) {
                        best_max = mx;
                        best_sum = sm;
                        best_d = d;
                        best_t = c;
                    }
                }
            }
        }
        if (best_d < 0 || best_max >= n) {
            // a leaf: its rules in list order, the covering one flagged
            if (n >= (1u << 11)) return false;
            img.nodes[t.node] = make_uint2(16u | n << 5, (uint32_t)img.leaves.size());
            for (uint32_t j = 0; j < n; ++j)
                img.leaves.push_back(L[j] | (covers[j] ? 0x80000000u : 0u));
            img.max_leaf = std::max(img.max_leaf, n);
            img.depth[fam_slot] = std::max(img.depth[fam_slot], t.depth);
            std::vector<uint32_t>().swap(L);
            continue;
        }
        if (img.nodes.size() + 2 > node_budget || img.nodes.size() + 2 >= (1u << 27)) return false;
        const uint32_t child = (uint32_t)img.nodes.size();
        img.nodes.push_back(make_uint2(0, 0));
        img.nodes.push_back(make_uint2(0, 0));
        img.nodes[t.node] = make_uint2((uint32_t)best_d | child << 5, best_t);
        Task a, b;
        a.node = child;
        b.node = child + 1;
        a.depth = b.depth = t.depth + 1;
        a.lo = b.lo = t.lo;
        a.hi = b.hi = t.hi;
        a.hi[best_d] = best_t - 1u;
        b.lo[best_d] = best_t;
        for (uint32_t j : L) {
            if (std::max(R[j].lo[best_d], t.lo[best_d]) < best_t) a.list.push_back(j);
            if (std::min(R[j].hi[best_d], t.hi[best_d]) >= best_t) b.list.push_back(j);
        }
        std::vector<uint32_t>().swap(L);
        q.push_back(std::move(a));
        q.push_back(std::move(b));
    }
    return true;
}

// One family's forest: its rules grouped by the key field (source address, destination address,
// source port, destination port, protocol) whose range overlaps the fewest other rules of the
// list (EffiCuts-style separation: a rule narrow only in its destination port is not copied into
// every leaf of a tree that splits on addresses), one tree per field, each split on its own field's
// words (an address tree also on the ports and the protocol) only, so that a walk level selects
// among few key words prepared before the walk (tree_match), every tree's
// rules in list order; a field no rule is narrowest in gets an empty tree.  A key's first match
// is the smallest of its first matches in the trees (the groups partition the list).  The
// family's first rule that matches every key is no tree's, nor is any rule after it: it is the
// answer when no tree has one (*def, its list position, else kNone).  roots: kTreeFields entries.
int tree_field(int d) { return d < 4 ? 0 : d < 8 ? 1 : d - 6; }
constexpr uint32_t kTreeFieldDims[kTreeFields] = {0x70Fu, 0x7F0u, 1u << 8, 1u << 9, 1u << 10};
bool build_forest_family(const std::vector<TreeRule>& R, int fam_slot, uint32_t binth,
                         size_t node_budget, TreeImage& img, std::vector<uint32_t>& roots,
                         uint32_t* def, const std::vector<TreeRule>* RG = nullptr) {
    const size_t n = R.size();
    const std::vector<TreeRule>& G = RG ? *RG : R;
    roots.clear();
    *def = kNone;
    std::vector<int> grp(n, -1);
    std::vector<uint32_t> best(n, 0xFFFFFFFFu);
    std::vector<uint32_t> los(n), his(n);
    for (int d = 0; d < kTreeDims && n > 0; ++d) {
        for (size_t i = 0; i < n; ++i) {
            los[i] = G[i].lo[d];
            his[i] = G[i].hi[d];
        }
        std::sort(los.begin(), los.end());
        std::sort(his.begin(), his.end());
        for (size_t i = 0; i < n; ++i) {
            // rules whose range meets rule i's on word d: lo <= hi_i, minus those ending below lo_i
            const size_t a = (size_t)(std::upper_bound(los.begin(), los.end(), G[i].hi[d]) - los.begin());
            const size_t b = (size_t)(std::lower_bound(his.begin(), his.end(), G[i].lo[d]) - his.begin());
            const uint32_t ov = (uint32_t)(a - b);
            if (ov < best[i]) {
                best[i] = ov;
                grp[i] = tree_field(d);
            }
        }
    }
    for (size_t i = 0; i < n; ++i) {
        bool all = true;
        for (int d = 0; d < kTreeDims && all; ++d)
            all = (R[i].exact >> d & 1u) && R[i].lo[d] == 0 && R[i].hi[d] == kTreeWidth[d];
        if (all) {   // matches every key of the family
            grp[i] = -1;
            if (*def == kNone) *def = (uint32_t)i;
        }
    }
    // rules after the family's first catch-all are never a first match: no tree's
    std::vector<std::vector<uint32_t>> groups(kTreeFields);
    for (size_t i = 0; i < n && i < *def; ++i)
        if (grp[i] >= 0) groups[grp[i]].push_back((uint32_t)i);
    for (int g = 0; g < kTreeFields; ++g) {
        const std::vector<uint32_t>& members = groups[g];
        roots.push_back((uint32_t)img.nodes.size());
        if (members.empty()) {   // an empty leaf
            img.nodes.push_back(make_uint2(16u, 0u));
            continue;
        }
        const size_t n0 = img.nodes.size(), e0 = img.leaves.size();
        // (large groups: longer leaves, or nested prefixes multiply the leaves)
        const uint32_t bt = members.size() > 4096 ? std::max(binth, 16u) : binth;
        const bool ok = build_tree_family(R, members, fam_slot, bt, node_budget, img,
                                          kTreeFieldDims[g]);
        if (getenv("UPE_GPU_VERBOSE"))
            fprintf(stderr, "upe_gpu: tree family %d field %d: %zu rules, %zu nodes, %zu leaf entries%s\n",
                    fam_slot ? 6 : 4, g, members.size(), img.nodes.size() - n0,
                    img.leaves.size() - e0, ok ? "" : " (over budget)");
        if (!ok) return false;
    }
    return true;
}

// Binary nodes (build_tree_family: inner {dim | child << 5, threshold}, leaf {16 | count << 5,
// first entry}) -> the walk's two-level nodes (Args::tree comment), breadth first from the roots
// (roots[k] -> node first + k).  False when an index outgrows its bits.
bool pack_two_level(const std::vector<uint2>& bin, const std::vector<uint32_t>& roots,
                    uint32_t first, std::vector<uint4>& out) {
    auto is_leaf = [&](uint32_t b) { return (bin[b].x & 16u) != 0u; };
    auto leaf_word = [&](uint32_t b, bool& ok) {
        const uint32_t cnt = bin[b].x >> 5, off = bin[b].y;
        ok = ok && cnt < (1u << 11) && off < (1u << 21);
        return cnt << 21 | off;
    };
    out.resize(first + roots.size(), make_uint4(0, 0, 0, 0));
    std::deque<std::pair<uint32_t, uint32_t>> q;   // (binary node, packed node)
    for (size_t k = 0; k < roots.size(); ++k) q.emplace_back(roots[k], first + (uint32_t)k);
    bool ok = true;
    while (!q.empty() && ok) {
        const auto [b, o] = q.front();
        q.pop_front();
        if (is_leaf(b)) {
            out[o] = make_uint4(1u << 12, leaf_word(b, ok), 0, 0);
            continue;
        }
        const uint32_t l = bin[b].x >> 5, r = l + 1;
        const bool ll = is_leaf(l), rl = is_leaf(r);
        const uint32_t base = (ll && rl) ? 0u : (uint32_t)out.size();
        ok = ok && base < (1u << 17);
        uint4 nd;
        nd.x = (bin[b].x & 15u) | (bin[l].x & 15u) << 4 | (bin[r].x & 15u) << 8 |
               (ll ? 1u : 0u) << 13 | (rl ? 1u : 0u) << 14 | base << 15;
        nd.y = bin[b].y;
        nd.z = ll ? leaf_word(l, ok) : bin[l].y;
        nd.w = rl ? leaf_word(r, ok) : bin[r].y;
        out[o] = nd;
        uint32_t next = base;
        for (const uint32_t c : {l, r}) {
            if (is_leaf(c)) continue;
            out.resize(out.size() + 2, make_uint4(0, 0, 0, 0));
            q.emplace_back(bin[c].x >> 5, next);
            q.emplace_back((bin[c].x >> 5) + 1u, next + 1u);
            next += 2;
        }
    }
    return ok;
}

// The forests of both family lists (l4 / l6: sorted indexes of the list entries), packed two
// levels to a node after the directory (Args::tree comment: node 0 = {trees of family 4, trees
// of family 6 | IPv6 byte orders << 16, the families' default answers (list positions, kNone =
// none)}, then the trees' roots, family 4's first, so that a walk starts without an indirection).
// group_be: the IPv6 rules grouped by their big-endian ranges whatever the words' byte order
// (build_tree's choice).
bool build_tree_as(const std::vector<RuleV4>& v4, const std::vector<RuleV6>& v6,
                   const std::vector<uint32_t>& l4, const std::vector<uint32_t>& l6, uint32_t binth,
                   size_t node_budget, bool group_be, TreeImage& img) {
    img = TreeImage();
    TreeImage body;
    std::vector<TreeRule> R;
    std::vector<uint32_t> r4, r6;
    uint32_t def4 = kNone, def6 = kNone;
    for (uint32_t i : l4) R.push_back(tree_rule(4, v4[i], nullptr));
    if (!build_forest_family(R, 0, binth, node_budget, body, r4, &def4)) return false;
    R.clear();
    const uint32_t swap6 = tree_swap6(v4, v6, l6);
    for (uint32_t i : l6) R.push_back(tree_rule(6, v4[i], &v6[i], swap6));
    std::vector<TreeRule> RG;
    if (group_be)
        for (uint32_t i : l6) RG.push_back(tree_rule(6, v4[i], &v6[i], 0xFFu));
    if (!build_forest_family(R, 1, binth, node_budget, body, r6, &def6, group_be ? &RG : nullptr))
        return false;
    std::vector<uint32_t> roots = r4;
    roots.insert(roots.end(), r6.begin(), r6.end());
    std::vector<uint4> packed;
    if (!pack_two_level(body.nodes, roots, 1u, packed)) return false;
    packed[0] = make_uint4((uint32_t)r4.size(), (uint32_t)r6.size() | swap6 << 16, def4, def6);
    img.nodes.resize(2 * packed.size());
    memcpy(img.nodes.data(), packed.data(), packed.size() * sizeof(uint4));
    img.leaves = std::move(body.leaves);
    img.depth[0] = body.depth[0];
    img.depth[1] = body.depth[1];
    img.max_leaf = body.max_leaf;
    img.trees[0] = (uint32_t)r4.size();
    img.trees[1] = (uint32_t)r6.size();
    img.swap6 = swap6;
    return true;
}

uint32_t tree_walk_host(const TreeImage& img, const std::vector<RuleV4>& v4,
                        const std::vector<RuleV6>& v6, const std::vector<uint32_t>& list, bool is6,
                        const uint32_t kv[kTreeDims], uint32_t k0, uint32_t k1, const uint32_t s[4],
                        const uint32_t d[4], uint8_t* prof_depth, uint8_t* prof_steps);

// Sampled walk cost of an image's IPv6 forest: nodes loaded plus leaf entries read (tree_walk_host's
// profile) over keys whose fields are drawn from the IPv6 rules' own constrained fields, a stand-in
// for traffic from the pools the rules were written for.
uint64_t tree_sample_cost6(const TreeImage& img, const std::vector<RuleV4>& v4,
                           const std::vector<RuleV6>& v6, const std::vector<uint32_t>& l6) {
    static constexpr int kFieldDims[5][2] = {{0, 4}, {4, 8}, {8, 9}, {9, 10}, {10, 11}};
    std::vector<TreeRule> R;
    for (uint32_t i : l6) R.push_back(tree_rule(6, v4[i], &v6[i], img.swap6));
    std::vector<uint32_t> by_field[5];
    for (uint32_t i = 0; i < (uint32_t)R.size(); ++i)
        for (int f = 0; f < 5; ++f)
            for (int dm = kFieldDims[f][0]; dm < kFieldDims[f][1]; ++dm)
                if (R[i].lo[dm] != 0 || R[i].hi[dm] != kTreeWidth[dm]) {
                    by_field[f].push_back(i);
                    break;
                }
    uint64_t x = 0x9E3779B97F4A7C15ull, cost = 0;
    auto rnd = [&]() {   // splitmix64
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return (uint32_t)(z ^ (z >> 31));
    };
    const size_t n = std::min<size_t>(4096, 4 * R.size());
    for (size_t k = 0; k < n; ++k) {
        uint32_t kv[kTreeDims] = {};
        for (int f = 0; f < 5; ++f) {
            const TreeRule* r = by_field[f].empty() ? nullptr : &R[by_field[f][rnd() % by_field[f].size()]];
            for (int dm = kFieldDims[f][0]; dm < kFieldDims[f][1]; ++dm) {
                const uint32_t lo = r ? r->lo[dm] : 0u, hi = r ? r->hi[dm] : kTreeWidth[dm];
                const uint64_t span = (uint64_t)hi - lo + 1u;
                kv[dm] = lo + (uint32_t)(rnd() % span);
            }
        }
        uint32_t sw[4], dw[4];
        for (int j = 0; j < 4; ++j) {
            sw[j] = word_of(kv[j], img.swap6, j);
            dw[j] = word_of(kv[4 + j], img.swap6, 4 + j);
        }
        const uint32_t k0 = 6u | kv[10] << 8 | kv[8] << 16, k1 = kv[9];
        uint8_t dep[16] = {}, stp[16] = {};
        tree_walk_host(img, v4, v6, l6, true, kv, k0, k1, sw, dw, dep, stp);
        for (int t = 0; t < 16; ++t) cost += dep[t] + stp[t];
    }
    return cost;
}

// build_tree_as, and when the IPv6 words' byte orders differ from big-endian, also with the
// grouping by big-endian ranges: the one of lower sampled cost (tree_sample_cost6).  The byte
// order makes a version-agnostic IPv4 prefix a range (config C6: 75 -> 63 us per 1M), but the
// grouping its ranges imply can move rules into port and protocol trees with long leaves (the
// 16k-rule flow table: 269 -> 332 us; the big-endian grouping 260).
bool build_tree(const std::vector<RuleV4>& v4, const std::vector<RuleV6>& v6,
                const std::vector<uint32_t>& l4, const std::vector<uint32_t>& l6, uint32_t binth,
                size_t node_budget, TreeImage& img) {
    const bool ok = build_tree_as(v4, v6, l4, l6, binth, node_budget, false, img);
    if (!ok || img.swap6 == 0xFFu) return ok;
    TreeImage alt;
    if (!build_tree_as(v4, v6, l4, l6, binth, node_budget, true, alt)) return true;
    const uint64_t ca = tree_sample_cost6(img, v4, v6, l6), cb = tree_sample_cost6(alt, v4, v6, l6);
    if (getenv("UPE_GPU_VERBOSE"))
        fprintf(stderr, "upe_gpu: tree IPv6 byte orders %02x, sampled cost %llu (grouped as such) / %llu (grouped big-endian)\n",
                img.swap6, (unsigned long long)ca, (unsigned long long)cb);
    if (cb < ca) img = std::move(alt);
    return true;
}

// The tree of a table: the shortest leaves (at most 1, 2, 3, then kTreeBinth rules before a
// split) whose image still leaves room in LDS for both family lists (list_bytes), a 1k-rule
// rule_stats histogram and two 1k-slot neighbour indexes — the leaf tests read the lists from
// LDS, and a list left in memory costs more than longer leaves (round 5: CF 73.8 / 71.0 / 87.6 us
// at 4 / 3 / 2, whose image no longer fit; C6 83.7 / 79.2 / 76.6).  Tables whose lists cannot be
// staged anyway get kTreeBinth.  forced: UPE_GPU_TREE_BINTH (diagnostic), 0 = choose.
constexpr size_t kTreeLdsReserve = 56 * 1024;
// The list entries a scan of family F's list can reach: up to and including its first rule that
// matches every key of the family (build_forest_family's default answer), else the whole list.
size_t scan_reach(int F, const std::vector<RuleV4>& v4, const std::vector<RuleV6>& v6,
                  const std::vector<uint32_t>& list) {
    for (size_t j = 0; j < list.size(); ++j) {
        const TreeRule r = tree_rule(F, v4[list[j]], F == 6 ? &v6[list[j]] : nullptr);
        bool all = true;
        for (int d = 0; d < kTreeDims && all; ++d)
            all = (r.exact >> d & 1u) && r.lo[d] == 0 && r.hi[d] == kTreeWidth[d];
        if (all) return j + 1;
    }
    return list.size();
}
size_t tree_node_budget(size_t count);
bool choose_tree(const std::vector<RuleV4>& v4, const std::vector<RuleV6>& v6,
                 const std::vector<uint32_t>& l4, const std::vector<uint32_t>& l6, size_t count,
                 uint32_t forced, TreeImage& t) {
    const size_t budget = tree_node_budget(count);
    if (forced) return build_tree(v4, v6, l4, l6, forced, budget, t);
    const size_t list_bytes = (2 * l4.size() + kFamV6Stride * l6.size()) * sizeof(uint4);
    if (list_bytes + kTreeLdsReserve >= kLdsDynMaxLarge) return build_tree(v4, v6, l4, l6, kTreeBinth, budget, t);
    for (uint32_t b : {1u, 2u, 3u}) {
        if (!build_tree(v4, v6, l4, l6, b, budget, t)) continue;
        const size_t img = 8 * t.nodes.size() + 4 * t.leaves.size();
        if (img + list_bytes + kTreeLdsReserve <= kLdsDynMaxLarge) return true;
    }
    return build_tree(v4, v6, l4, l6, kTreeBinth, budget, t);
}

// Host walk of the image, bit for bit what tree_match does on the device: the list position of
// the key's first match (kNone = none).  kv: the key words (kTreeDims comment).
uint32_t tree_walk_host(const TreeImage& img, const std::vector<RuleV4>& v4,
                        const std::vector<RuleV6>& v6, const std::vector<uint32_t>& list, bool is6,
                        const uint32_t kv[kTreeDims], uint32_t k0, uint32_t k1, const uint32_t s[4],
                        const uint32_t d[4], uint8_t* prof_depth, uint8_t* prof_steps) {
    const uint2 dir = img.nodes[0], dflt = img.nodes[1];
    const uint32_t nt = is6 ? dir.y & 0xFFFFu : dir.x, first = 1u + (is6 ? dir.x : 0u);
    const uint4* S = reinterpret_cast<const uint4*>(img.nodes.data());
    uint32_t best = kNone;
    for (uint32_t t = 0; t < nt; ++t) {
        uint32_t idx = first + t, lw = 0, depth = 0;
        for (;;) {   // tree_match's step, two levels per node
            const uint4 q = S[idx];
            ++depth;
            if (q.x & 0x1000u) {
                lw = q.y;
                break;
            }
            const bool c1 = kv[q.x & 15u] >= q.y;
            const bool lleaf = (q.x >> 13) & 1u;
            const bool cl = c1 ? ((q.x >> 14) & 1u) != 0u : lleaf;
            const uint32_t ct = c1 ? q.w : q.z;
            if (cl) {
                lw = ct;
                break;
            }
            const uint32_t c2 = kv[c1 ? (q.x >> 8) & 15u : (q.x >> 4) & 15u] >= ct ? 1u : 0u;
            idx = (q.x >> 15) + ((c1 && !lleaf) ? 2u : 0u) + c2;
        }
        const uint32_t cnt = lw >> 21, off = lw & 0x1FFFFFu;
        if (prof_depth && t < 16) {
            prof_depth[t] = (uint8_t)std::min(depth, 255u);
            prof_steps[t] = 0;
        }
        for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t e = img.leaves[off + j];
            const uint32_t pos = e & 0x7FFFFFFFu;
            if (prof_steps && t < 16 && prof_steps[t] < 255) ++prof_steps[t];
            if (pos >= best) break;
            bool hit = (e >> 31) != 0;
            if (!hit) {
                const RuleV4& r = v4[list[pos]];
                uint32_t x = ((k0 ^ r.x0) & r.m0) | ((k1 ^ r.x1) & r.m1 & 0xFFFFu) |
                             ((s[0] ^ r.s0) & r.sm0) | ((d[0] ^ r.d0) & r.dm0);
                if (is6) {
                    const RuleV6& q6 = v6[list[pos]];
                    for (int w = 0; w < 3; ++w)
                        x |= ((s[w + 1] ^ q6.s[w]) & q6.sm[w]) | ((d[w + 1] ^ q6.d[w]) & q6.dm[w]);
                }
                hit = x == 0;
            }
            if (hit) {
                best = pos;
                break;
            }
        }
    }
    return best != kNone ? best : is6 ? dflt.y : dflt.x;
}

// rule_t -> the compiled words: RuleV4 / RuleV6 (pre-masked) and rinfo, pad >= count entries (the
// padding never matches).  -1 (message set) on a rule_id outside [0, cap).
int compile_rules(const upe_rule_t* rules, size_t count, size_t cap, size_t pad,
                  std::vector<RuleV4>& v4, std::vector<RuleV6>& v6, std::vector<int2>& info) {
    v4.assign(pad, RuleV4{});
    v6.assign(pad, RuleV6{});
    info.assign(pad, make_int2(0, 0));
    for (size_t i = 0; i < pad; ++i) {
        RuleV4& a = v4[i];
        RuleV6& b = v6[i];
        memset(&a, 0, sizeof a);
        memset(&b, 0, sizeof b);
        if (i >= count) {
            // never matches: ip_ver byte 0xFF against a key version of 4 or 6
            a.x0 = 0xFF;
            a.m0 = 0xFF;
            continue;
        }
        const upe_rule_t& r = rules[i];
        if (r.rule_id >= cap) return fail("rule_id >= capacity (rule_stats index)");
        a.x0 = (uint32_t)r.ip_ver | ((uint32_t)r.protocol << 8) | ((uint32_t)r.src_port << 16);
        a.m0 = (r.ip_ver ? 0xFFu : 0u) | (r.protocol ? 0xFF00u : 0u) |
               (r.src_port ? 0xFFFF0000u : 0u);
        a.x1 = (uint32_t)r.dst_port | (act_code(r.action.type) << 16);
        a.m1 = r.dst_port ? 0xFFFFu : 0u;
        const uint8_t* si = r.src_ip.v6;
        const uint8_t* sm = r.src_mask.v6;
        const uint8_t* di = r.dst_ip.v6;
        const uint8_t* dm = r.dst_mask.v6;
        a.sm0 = le32(sm);
        a.s0 = le32(si) & a.sm0;
        a.dm0 = le32(dm);
        a.d0 = le32(di) & a.dm0;
        bool v6w = false;
        for (int j = 0; j < 3; ++j) {
            b.sm[j] = le32(sm + 4 * (j + 1));
            b.s[j] = le32(si + 4 * (j + 1)) & b.sm[j];
            b.dm[j] = le32(dm + 4 * (j + 1));
            b.d[j] = le32(di + 4 * (j + 1)) & b.dm[j];
            v6w |= b.sm[j] != 0 || b.dm[j] != 0;
        }
        if (v6w) a.m1 |= kRuleV6Words;   // IPv6 keys must test this rule's rv6 words
        info[i] = make_int2(r.action.type, (int)r.rule_id);
    }
    return 0;
}

// Does compiled rule i match every key of family 4 / 6?
bool matches_all4(const RuleV4& e) {
    return (e.m0 & 0xFFFFFF00u) == 0 && (e.m1 & 0xFFFFu) == 0 && e.sm0 == 0 && e.dm0 == 0;
}
bool matches_all6(const RuleV4& e, const RuleV6& q) {
    bool all = matches_all4(e);
    for (int j = 0; j < 3; ++j) all = all && q.sm[j] == 0 && q.dm[j] == 0;
    return all;
}

// The family lists (FamTable): the sorted indexes of the rules a key of each family can match
// (ip_ver 4 or 0, 6 or 0), each ending at its family's first rule that matches every key of the
// family (nothing after it can be a first match: seed-3 config C's IPv6 list is one entry long).
void family_lists(const upe_rule_t* rules, size_t count, const std::vector<RuleV4>& v4,
                  const std::vector<RuleV6>& v6, std::vector<uint32_t>& l4,
                  std::vector<uint32_t>& l6, bool& end4, bool& end6) {
    l4.clear();
    l6.clear();
    end4 = end6 = false;
    for (size_t i = 0; i < count; ++i) {
        const uint8_t ver = rules[i].ip_ver;
        if (!end4 && (ver == 0 || ver == 4)) {
            l4.push_back((uint32_t)i);
            end4 = matches_all4(v4[i]);
        }
        if (!end6 && (ver == 0 || ver == 6)) {
            l6.push_back((uint32_t)i);
            end6 = matches_all6(v4[i], v6[i]);
        }
    }
}

size_t tree_node_budget(size_t count) {
    const char* e = getenv("UPE_GPU_TREE_BUDGET");   // diagnostic override
    if (e) return (size_t)strtoull(e, nullptr, 10);
    return std::max<size_t>(1u << 16, 64 * count);
}
}  // namespace
extern "C" {

}  // extern "C"

namespace {
// A device allocation that frees itself unless taken: load_rules uploads every image of the new
// table first and changes the context only once all of them are on the device.
struct DevBuf {
    void* p = nullptr;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    int put(const void* src, size_t bytes) {
        if (bytes == 0) return 0;
        HIP_TRY(hipMalloc(&p, bytes));
        HIP_TRY(hipMemcpy(p, src, bytes, hipMemcpyHostToDevice));
        return 0;
    }
    template <class T>
    T* take() {
        T* q = static_cast<T*>(p);
        p = nullptr;
        return q;
    }
};
template <class T>
void replace(T*& field, DevBuf& b) {
    if (field) (void)hipFree(field);
    field = b.take<T>();
}

}  // namespace

// The compiled table a context classifies with (round 6: built apart from any context, so that
// a program's stats thread can build it while the workers keep forwarding, as the reference's
// does before its SIGHUP swap, src/main.c:222-257): the rule words, the family lists, the
// tuple-space index or the decision tree, and the flags the launches need.  Host memory only.
struct upe_rule_image {
    size_t count = 0, cap = 0, pad = 0;
    std::vector<RuleV4> v4;
    std::vector<RuleV6> v6;
    std::vector<int2> info;
    bool fwd4 = false, fwd6 = false;
    uint32_t fam4 = 0, fam6 = 0, fam_all = 0, fam_x1idx = 0;
    std::vector<uint4> fimg;
    bool tss = false;
    TssFamily f4, f6;
    std::vector<uint16_t> fps;
    bool tree_ok = false;
    std::vector<uint4> timg;
    TreeImage t;
};

namespace {
// Compile a sorted table of `count` rules for a context whose rule_stats hold `cap` entries
// (host only: no context, no GPU; any thread).  0, or -1 (upe_gpu_last_error()).
int build_image(const upe_rule_t* rules, size_t count, size_t cap, upe_rule_image& im) {
    im.count = count;
    im.cap = cap;
    const size_t pad = ((count + kUnroll - 1) / kUnroll + 1) * kUnroll;  // >= 1 padding block
    im.pad = pad;
    std::vector<RuleV4>& v4 = im.v4;
    std::vector<RuleV6>& v6 = im.v6;
    std::vector<int2>& info = im.info;
    if (compile_rules(rules, count, cap, pad, v4, v6, info) != 0) return -1;
    // a family none of whose reachable rules forwards never consults or updates its L1 entry
    // (src/worker.c:155-244 run only for forwarded packets): its entry's agreement is moot
    bool& fwd4 = im.fwd4;
    bool& fwd6 = im.fwd6;
    {
        bool e4 = false, e6 = false;
        for (size_t i = 0; i < count && !(e4 && e6); ++i) {
            const uint8_t ver = rules[i].ip_ver;
            const bool all4 = matches_all4(v4[i]), all6 = matches_all6(v4[i], v6[i]);
            const bool fwd = rules[i].action.type == UPE_ACT_FWD;
            if (!e4 && (ver == 0 || ver == 4)) { fwd4 = fwd4 || fwd; e4 = all4; }
            if (!e6 && (ver == 0 || ver == 6)) { fwd6 = fwd6 || fwd; e6 = all6; }
        }
    }
    // linear-scan tables past the LDS copy: the per-family lists (FamTable)
    uint32_t& fam4 = im.fam4;
    uint32_t& fam6 = im.fam6;
    uint32_t& fam_all = im.fam_all;
    uint32_t& fam_x1idx = im.fam_x1idx;
    std::vector<uint32_t> l4, l6;   // the family lists' sorted indexes
    std::vector<uint4>& fimg = im.fimg;
    if (pad > (size_t)kSmallRules) {
        bool end4 = false, end6 = false;
        family_lists(rules, count, v4, v6, l4, l6, end4, end6);
        const size_t n4 = (l4.size() + kUnroll - 1) / kUnroll * kUnroll;
        const size_t n6 = (l6.size() + kUnroll - 1) / kUnroll * kUnroll;
        // (+1: the scalar scan loads an IPv6 entry's last 48 bytes as 64)
        fimg.assign(2 * n4 + kFamV6Stride * n6 + (n4 + n6 + 3) / 4 + 1, make_uint4(0, 0, 0, 0));
        RuleV4 never;
        memset(&never, 0, sizeof never);
        never.x0 = 0xFF;   // ip_ver byte 0xFF against a key version of 4 or 6
        never.m0 = 0xFF;
        uint32_t* idx = reinterpret_cast<uint32_t*>(fimg.data() + 2 * n4 + kFamV6Stride * n6);
        // tables below 8192 rules: the sorted index rides in x1 bits 18-30 (m1 keeps them clear,
        // so the match is unchanged) and comes back with the matched rule's words
        const bool x1idx = count < 8192;
        for (size_t j = 0; j < n4; ++j) {
            RuleV4 e = j < l4.size() ? v4[l4[j]] : never;
            if (x1idx && j < l4.size()) e.x1 |= l4[j] << 18;
            memcpy(&fimg[2 * j], &e, sizeof e);
            idx[j] = j < l4.size() ? l4[j] : 0u;
        }
        for (size_t j = 0; j < n6; ++j) {
            uint4* o = &fimg[2 * n4 + kFamV6Stride * j];
            if (j < l6.size()) {
                RuleV4 e = v4[l6[j]];
                if (x1idx) e.x1 |= l6[j] << 18;
                memcpy(o, &e, sizeof(RuleV4));
                memcpy(o + 2, &v6[l6[j]], 3 * sizeof(uint4));   // s, sm, d, dm (12 words)
            } else {
                memcpy(o, &never, sizeof never);
            }
            idx[n4 + j] = j < l6.size() ? l6[j] : 0u;
        }
        fam4 = (uint32_t)n4;
        fam6 = (uint32_t)n6;
        fam_all = (l4.size() == 1 && end4 ? 1u : 0u) | (l6.size() == 1 && end6 ? 2u : 0u);
        fam_x1idx = x1idx ? 1u : 0u;
    }
    // Large tables: a tuple-space index when the rules fall into few mask signatures (one hash
    // probe per signature instead of a test per rule).
    bool& tss = im.tss;
    TssFamily& f4 = im.f4;
    TssFamily& f6 = im.f6;
    std::vector<uint16_t>& fps = im.fps;   // the staged fingerprint image
    const char* force = getenv("UPE_GPU_TSS");   // diagnostic: 0 = never, 1 = always
    if (count > 0 && count < kTssMaxRules && !(force && force[0] == '0') &&
        build_tss_family(4, v4, v6, rules, count, f4) && build_tss_family(6, v4, v6, rules, count, f6)) {
        const size_t ng = f4.groups.size() + f6.groups.size();
        if ((force && force[0] == '1') || (count >= 1024 && ng * 16 <= count)) {
            // the staged fingerprint image: small groups, in probe order, while it fits
            const char* st = getenv("UPE_GPU_FP_STAGE");   // diagnostic: 0 = stage none
            for (TssFamily* f : {&f4, &f6})
                for (TssGroup& g : f->groups) {
                    if (st && st[0] == '0') break;
                    const uint32_t slots = 1u << g.w[11];
                    if ((g.w[14] & 1u) || slots > kFpStageGroup || fps.size() + slots > kFpStageMax)
                        continue;
                    g.w[15] = 1u + (uint32_t)fps.size();
                    fps.insert(fps.end(), f->fp.begin() + g.w[13], f->fp.begin() + g.w[13] + slots);
                }
            fps.resize((fps.size() + 7) & ~(size_t)7, 0);
            tss = true;
        }
    }
    // Linear-scan tables past kSmallRules without a tuple-space index: the decision tree over the
    // family lists (kTreeDims comment), unless it outgrows its node budget, or a scan never gets
    // far: both families' lists reach their first catch-all within kTreeMinReach entries (the
    // scan's cost is then bounded by that, and its wave-uniform scalar loads beat the walk:
    // seed-3 config C 38.1 vs 46.5 us).  UPE_GPU_TREE: 0 = never, 1 = whenever it builds
    // (diagnostics); UPE_GPU_TREE_BINTH: rules per leaf before a split.
    bool& tree_ok = im.tree_ok;
    std::vector<uint4>& timg = im.timg;
    TreeImage& t = im.t;
    const char* tf = getenv("UPE_GPU_TREE");
    // (the reach first, from the lists alone: a table a scan never walks far into is not built a
    // tree only to throw it away — ADVICE r05; a reload then costs the lists, not the forest)
    const size_t reach0 = std::max(scan_reach(4, v4, v6, l4), scan_reach(6, v4, v6, l6));
    if (!tss && pad > (size_t)kSmallRules && !(tf && tf[0] == '0') &&
        (reach0 > kTreeMinReach || (tf && tf[0] == '1'))) {
        const char* bt = getenv("UPE_GPU_TREE_BINTH");
        const uint32_t binth = bt ? (uint32_t)std::max(1, atoi(bt)) : 0u;
        if (choose_tree(v4, v6, l4, l6, count, binth, t)) {
            const size_t nw = 2 * t.nodes.size() + t.leaves.size();
            timg.assign((nw + 3) / 4, make_uint4(0, 0, 0, 0));
            memcpy(timg.data(), t.nodes.data(), t.nodes.size() * sizeof(uint2));
            memcpy(reinterpret_cast<uint32_t*>(timg.data()) + 2 * t.nodes.size(), t.leaves.data(),
                   t.leaves.size() * sizeof(uint32_t));
            // the list entries a scan can reach: up to the family's first catch-all (node 1)
            const uint2 dflt = t.nodes[1];
            const size_t reach = std::max(dflt.x == kNone ? l4.size() : (size_t)dflt.x + 1,
                                          dflt.y == kNone ? l6.size() : (size_t)dflt.y + 1);
            tree_ok = reach > kTreeMinReach || (tf && tf[0] == '1');
        }
    }
    return 0;
}

// upe_gpu_load_rules / upe_gpu_reload_rules[_image] with a compiled image: `fresh` (a zeroed
// rule_stats of fresh_cap entries) replaces the context's statistics on a reload, the old
// per-index totals dropped instead of credited.  Everything the new table needs is uploaded
// before the context changes: on an error the context keeps classifying with the old table and
// its statistics.
int install_image(upe_gpu_ctx_t* c, const upe_rule_image& im, DevBuf* fresh, size_t fresh_cap) {
    const size_t count = im.count, pad = im.pad;
    const std::vector<RuleV4>& v4 = im.v4;
    const std::vector<RuleV6>& v6 = im.v6;
    const std::vector<int2>& info = im.info;
    const std::vector<uint4>& fimg = im.fimg;
    const bool tss = im.tss, tree_ok = im.tree_ok;
    const TssFamily& f4 = im.f4;
    const TssFamily& f6 = im.f6;
    const std::vector<uint16_t>& fps = im.fps;
    const std::vector<uint4>& timg = im.timg;
    const TreeImage& t = im.t;
    const uint32_t fam4 = im.fam4, fam6 = im.fam6, fam_all = im.fam_all, fam_x1idx = im.fam_x1idx;
    const bool fwd4 = im.fwd4, fwd6 = im.fwd6;
    // every image on the device before anything of the context changes
    DevBuf b_rv4, b_rv6, b_rinfo, b_idx, b_fam, b_tfs, b_tg4, b_tg6, b_tt4, b_tt6, b_tree;
    if (b_rv4.put(v4.data(), pad * sizeof(RuleV4)) || b_rv6.put(v6.data(), pad * sizeof(RuleV6)) ||
        b_rinfo.put(info.data(), pad * sizeof(int2)) ||
        b_fam.put(fimg.data(), fimg.size() * sizeof(uint4)) ||
        (tss && (b_tfs.put(fps.data(), fps.size() * sizeof(uint16_t)) ||
                 b_tg4.put(f4.groups.data(), f4.groups.size() * sizeof(TssGroup)) ||
                 b_tg6.put(f6.groups.data(), f6.groups.size() * sizeof(TssGroup)) ||
                 b_tt4.put(f4.slots.data(), f4.slots.size() * sizeof(uint4)) ||
                 b_tt6.put(f6.slots.data(), f6.slots.size() * sizeof(uint4)))) ||
        (tree_ok && b_tree.put(timg.data(), timg.size() * sizeof(uint4))))
        return -1;
    const bool grow = pad > c->rules_alloc;
    if (grow) {
        const size_t bytes = pad * 2 * kStatReps * sizeof(unsigned long long);
        HIP_TRY(hipMalloc(&b_idx.p, bytes));
        HIP_TRY(hipMemset(b_idx.p, 0, bytes));
    }
    // previous batches may still read the table, on whichever stream they went
    if (c->last_stream) HIP_TRY(hipStreamSynchronize(c->last_stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (fresh) {
        // the reload's fresh statistics: the old table's per-index totals are dropped
        if (c->stats_idx)
            HIP_TRY(hipMemset(c->stats_idx, 0,
                              (size_t)c->rules_alloc * 2 * kStatReps * sizeof(unsigned long long)));
        HIP_TRY(hipMemset(&c->st->acc_stats[0][0], 0, sizeof(c->st->acc_stats)));
        if (c->stats) (void)hipFree(c->stats);
        c->stats = fresh->take<unsigned long long>();
        c->cap = fresh_cap;
        c->rinfo_host.clear();
    } else if (fold_stats_idx(c) != 0) {   // the old table's counts credited to their rule_ids
        return -1;
    }
    // the swap
    replace(c->rv4, b_rv4);
    replace(c->rv6, b_rv6);
    replace(c->rinfo, b_rinfo);
    if (grow) {
        replace(c->stats_idx, b_idx);
        c->rules_alloc = pad;
    }
    replace(c->fam, b_fam);
    c->fam_alloc = fimg.size() * sizeof(uint4);
    c->fam4 = fam4;
    c->fam6 = fam6;
    c->fam_all = fam_all;
    c->fam_x1idx = fam_x1idx;
    c->fwd4 = fwd4;
    c->fwd6 = fwd6;
    // the kernel without look-back may have been chosen because a family could not forward
    // under the old table: back to the full kernel until a launch under this one reports
    c->no_lb = false;
    c->lb_reset_k = c->k;
    c->nrules = (uint32_t)count;
    c->nrules_pad = (uint32_t)pad;
    c->rinfo_host = info;
    replace(c->tfs, b_tfs);
    replace(c->tg4, b_tg4);
    replace(c->tg6, b_tg6);
    replace(c->tt4, b_tt4);
    replace(c->tt6, b_tt6);
    c->tss = tss;
    c->nfs = tss ? (uint32_t)(fps.size() / 8) : 0u;
    c->ng4 = tss ? (uint32_t)f4.groups.size() : 0u;
    c->ng6 = tss ? (uint32_t)f6.groups.size() : 0u;
    replace(c->tree, b_tree);
    c->tree_ok = tree_ok;
    const char* tl = getenv("UPE_GPU_TREE_LDS");   // diagnostic: 0 = the image stays in memory
    c->tree_stage = !(tl && tl[0] == '0');
    c->tree_words = tree_ok ? (uint32_t)timg.size() : 0u;
    c->tree_loff = tree_ok ? (uint32_t)(2 * t.nodes.size()) : 0u;
    c->tree_info = tree_ok ? upe_rule_index_info_t{(uint64_t)t.nodes.size(), (uint64_t)t.leaves.size(),
                                                   t.depth[0], t.depth[1], t.max_leaf,
                                                   t.trees[0] | t.trees[1] << 16}
                           : upe_rule_index_info_t{};
    return publish(c);   // the DevState's pointers (stats, stats_idx)
}

int load_rules_impl(upe_gpu_ctx_t* c, const upe_rule_t* rules, size_t count,
                    DevBuf* fresh, size_t fresh_cap) {
    upe_rule_image im;
    if (build_image(rules, count, fresh ? fresh_cap : c->cap, im) != 0) return -1;
    return install_image(c, im, fresh, fresh_cap);
}
}  // namespace

extern "C" {

extern "C" int upe_gpu_load_rules(upe_gpu_ctx_t* c, const upe_rule_t* rules, size_t count) {
    if (!c) return fail("null context");
    if (count > c->cap) return fail("rule count exceeds the capacity given at open");
    if (count && !rules) return fail("null rules");
    DEV_SCOPE(c->device);
    return load_rules_impl(c, rules, count, nullptr, 0);
}

// The reference's SIGHUP reload (src/main.c:216-282): the stats thread builds a new table
// (rule_table_init(1024) + rule_config_load), gives every worker a fresh calloc'd rule_stats of
// the new table's capacity, swaps w->rt and w->rule_stats between two of the worker's bursts and
// frees the old ones after a grace period.  The worker's pkts_* counters and its one-entry L1
// neighbour caches are untouched.  Here: the batches queued so far finish with the old table,
// their rule_stats (credited to the old rule_ids) are handed back in old_stats if asked for,
// and the next batch runs with the new table and an all-zero rule_stats[rule_capacity].  All or
// nothing: on an error the old table and its statistics stay (as the reference keeps both when
// rule_config_load fails, src/main.c:229-255).
extern "C" int upe_gpu_reload_rules(upe_gpu_ctx_t* c, const upe_rule_t* rules, size_t count,
                                    size_t rule_capacity, upe_rule_stat_t* old_stats,
                                    size_t old_capacity) {
    if (!c) return fail("null context");
    if (rule_capacity == 0 || rule_capacity > (1u << 24)) return fail("rule_capacity must be in [1, 2^24]");
    if (count > rule_capacity) return fail("rule count exceeds the new capacity");
    if (count && !rules) return fail("null rules");
    if (old_capacity && !old_stats) return fail("null old_stats");
    for (size_t i = 0; i < count; ++i)
        if (rules[i].rule_id >= rule_capacity) return fail("rule_id >= capacity (rule_stats index)");
    DEV_SCOPE(c->device);
    // the batches queued with the old table finish first (on whichever stream they went)
    if (c->last_stream) HIP_TRY(hipStreamSynchronize(c->last_stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (old_capacity && read_rule_stats(c, old_stats, old_capacity) != 0) return -1;
    DevBuf fresh;   // a zeroed rule_stats of the new capacity (freed unless the reload succeeds)
    HIP_TRY(hipMalloc(&fresh.p, rule_capacity * 2 * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(fresh.p, 0, rule_capacity * 2 * sizeof(unsigned long long)));
    return load_rules_impl(c, rules, count, &fresh, rule_capacity);
}

extern "C" upe_rule_image_t* upe_rules_compile(const upe_rule_t* rules, size_t count,
                                               size_t rule_capacity) {
    if (rule_capacity == 0 || rule_capacity > (1u << 24)) {
        fail("rule_capacity must be in [1, 2^24]");
        return nullptr;
    }
    if (count > rule_capacity || (count && !rules)) {
        fail(count > rule_capacity ? "rule count exceeds the capacity" : "null rules");
        return nullptr;
    }
    try {
        auto* im = new upe_rule_image;
        if (build_image(rules, count, rule_capacity, *im) != 0) {
            delete im;
            return nullptr;
        }
        return im;
    } catch (const std::bad_alloc&) {
        fail("out of memory (rule image)");
        return nullptr;
    }
}

extern "C" void upe_rules_image_free(upe_rule_image_t* im) { delete im; }

extern "C" int upe_gpu_reload_image(upe_gpu_ctx_t* c, const upe_rule_image_t* im,
                                    upe_rule_stat_t* old_stats, size_t old_capacity) {
    if (!c || !im) return fail("null context or image");
    if (old_capacity && !old_stats) return fail("null old_stats");
    DEV_SCOPE(c->device);
    if (c->last_stream) HIP_TRY(hipStreamSynchronize(c->last_stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (old_capacity && read_rule_stats(c, old_stats, old_capacity) != 0) return -1;
    DevBuf fresh;
    HIP_TRY(hipMalloc(&fresh.p, im->cap * 2 * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(fresh.p, 0, im->cap * 2 * sizeof(unsigned long long)));
    return install_image(c, *im, &fresh, im->cap);
}

// (not part of the ABI; upe_worker.c) tag this context's launches as a host-side loop's: they
// run the host-path kernel instantiation (the same code), so that a profile of a process that
// also classifies device-resident batches keeps the two kinds of launch apart
extern "C" int upe_gpu_tag_host(upe_gpu_ctx_t* c, int on) {
    if (!c) return fail("null context");
    c->host_tag = on != 0;
    return 0;
}

extern "C" int upe_gpu_rule_index_kind(upe_gpu_ctx_t* c) {
    if (!c) return fail("null context");
    return c->tss ? 1 : c->tree_ok ? 2 : 0;
}

extern "C" int upe_gpu_rule_index_info(upe_gpu_ctx_t* c, upe_rule_index_info_t* info) {
    if (!c || !info) return fail("null argument");
    *info = c->tree_ok ? c->tree_info : upe_rule_index_info_t{};
    return 0;
}

extern "C" int upe_tree_profile_host(const upe_rule_t* rules, size_t count,
                                     const upe_flow_key_t* keys, size_t n, int64_t* out,
                                     upe_rule_index_info_t* info, uint8_t* prof_depth,
                                     uint8_t* prof_steps);

// rule_table_match (reference src/rule_table.c:163-176) for a batch of keys on the host, through
// the decision tree the GPU path builds for the same table (tree_walk_host: the device's walk bit
// for bit), or the family lists' linear first match when the table gets no tree.
extern "C" int upe_rules_match_host(const upe_rule_t* rules, size_t count,
                                    const upe_flow_key_t* keys, size_t n, int64_t* out,
                                    upe_rule_index_info_t* info) {
    return upe_tree_profile_host(rules, count, keys, n, out, info, nullptr, nullptr);
}

// (diagnostic, not part of the ABI) the same, and per key and tree of its family (first 16):
// levels walked (prof_depth[16 * i + t]) and leaf entries read (prof_steps[16 * i + t])
extern "C" int upe_tree_profile_host(const upe_rule_t* rules, size_t count,
                                     const upe_flow_key_t* keys, size_t n, int64_t* out,
                                     upe_rule_index_info_t* info, uint8_t* prof_depth,
                                     uint8_t* prof_steps) {
    if ((count && !rules) || (n && (!keys || !out))) return fail("null argument");
    const size_t pad = ((count + kUnroll - 1) / kUnroll + 1) * kUnroll;
    std::vector<RuleV4> v4;
    std::vector<RuleV6> v6;
    std::vector<int2> rinfo;
    if (compile_rules(rules, count, 0xFFFFFFFFu, pad, v4, v6, rinfo) != 0) return -1;
    std::vector<uint32_t> l4, l6;
    bool end4 = false, end6 = false;
    family_lists(rules, count, v4, v6, l4, l6, end4, end6);
    const char* bt = getenv("UPE_GPU_TREE_BINTH");
    const uint32_t binth = bt ? (uint32_t)std::max(1, atoi(bt)) : 0u;
    TreeImage t;
    const bool tree = choose_tree(v4, v6, l4, l6, count, binth, t);
    if (info)
        *info = tree ? upe_rule_index_info_t{(uint64_t)t.nodes.size(), (uint64_t)t.leaves.size(),
                                             t.depth[0], t.depth[1], t.max_leaf,
                                             t.trees[0] | t.trees[1] << 16}
                     : upe_rule_index_info_t{};
    for (size_t i = 0; i < n; ++i) {
        const upe_flow_key_t& k = keys[i];
        if (k.ip_ver != 4 && k.ip_ver != 6) {
            out[i] = -1;
            continue;
        }
        const bool is6 = k.ip_ver == 6;
        const uint32_t k0 = (uint32_t)k.ip_ver | ((uint32_t)k.protocol << 8) |
                            ((uint32_t)k.src_port << 16);
        const uint32_t k1 = k.dst_port;
        uint32_t sw[4], dw[4], kv[kTreeDims] = {};
        for (int j = 0; j < 4; ++j) {
            sw[j] = le32(k.src_ip.v6 + 4 * j);
            dw[j] = le32(k.dst_ip.v6 + 4 * j);
        }
        if (is6) {
            for (int j = 0; j < 4; ++j) {
                kv[j] = word_of(sw[j], t.swap6, j);
                kv[4 + j] = word_of(dw[j], t.swap6, 4 + j);
            }
        } else {
            kv[0] = sw[0];
            kv[4] = dw[0];
        }
        kv[8] = k.src_port;
        kv[9] = k.dst_port;
        kv[10] = k.protocol;
        const std::vector<uint32_t>& list = is6 ? l6 : l4;
        uint32_t pos = kNone;
        if (tree) {
            pos = tree_walk_host(t, v4, v6, list, is6, kv, k0, k1, sw, dw,
                                 prof_depth ? prof_depth + 16 * i : nullptr,
                                 prof_steps ? prof_steps + 16 * i : nullptr);
        } else {
            for (size_t j = 0; j < list.size() && pos == kNone; ++j) {
                const RuleV4& r = v4[list[j]];
                uint32_t x = ((k0 ^ r.x0) & r.m0) | ((k1 ^ r.x1) & r.m1 & 0xFFFFu) |
                             ((sw[0] ^ r.s0) & r.sm0) | ((dw[0] ^ r.d0) & r.dm0);
                if (is6)
                    for (int w = 0; w < 3; ++w)
                        x |= ((sw[w + 1] ^ v6[list[j]].s[w]) & v6[list[j]].sm[w]) |
                             ((dw[w + 1] ^ v6[list[j]].d[w]) & v6[list[j]].dm[w]);
                if (x == 0) pos = (uint32_t)j;
            }
        }
        out[i] = pos == kNone ? -1 : (int64_t)list[pos];
    }
    return 0;
}

int upe_gpu_load_neigh(upe_gpu_ctx_t* c, const upe_arp_entry_t* arp, size_t arp_capacity,
                       const upe_ndp_entry_t* ndp, size_t ndp_capacity) {
    if (!c) return fail("null context");
    auto pow2 = [](size_t x) { return x == 0 || (x & (x - 1)) == 0; };
    if (!pow2(arp_capacity) || !pow2(ndp_capacity))
        return fail("neighbour table capacity must be a power of two (arp_table_init)");
    if ((arp_capacity && !arp) || (ndp_capacity && !ndp)) return fail("null table");
    if (arp_capacity > (1u << 30) || ndp_capacity > (1u << 30)) return fail("table too large");
    DEV_SCOPE(c->device);
    // Keep only the entries a reference probe reaches (arp_get_mac, src/arp_table.c:55-80:
    // home slot ip & (cap-1), linear probe, first valid match, stop at the first invalid slot).
    std::vector<uint32_t> arp_keep;
    for (size_t s0 = 0; s0 < arp_capacity; ++s0) {
        if (!arp[s0].valid) continue;
        const uint32_t ip = arp[s0].ip;
        const size_t mask = arp_capacity - 1;
        for (size_t i = 0, t = ip & mask; i < arp_capacity; ++i, t = (t + 1) & mask) {
            if (!arp[t].valid) break;
            if (arp[t].ip == ip) {
                if (t == s0) arp_keep.push_back((uint32_t)s0);
                break;
            }
        }
    }
    // Same for ndp_get_mac (src/ndp_table.c:6-17,67-86): home slot = XOR of the LE words.
    std::vector<uint32_t> ndp_keep;
    for (size_t s0 = 0; s0 < ndp_capacity; ++s0) {
        if (!ndp[s0].valid) continue;
        const uint8_t* ip = ndp[s0].ip;
        const size_t mask = ndp_capacity - 1;
        const size_t h = (le32(ip) ^ le32(ip + 4) ^ le32(ip + 8) ^ le32(ip + 12)) & mask;
        for (size_t i = 0, t = h; i < ndp_capacity; ++i, t = (t + 1) & mask) {
            if (!ndp[t].valid) break;
            if (memcmp(ndp[t].ip, ip, 16) == 0) {
                if (t == s0) ndp_keep.push_back((uint32_t)s0);
                break;
            }
        }
    }
    // Place the reachable entries by three-choice cuckoo hashing at load factor <= 0.8.
    std::vector<uint32_t> akey(arp_keep.size()), nkey(ndp_keep.size());
    for (size_t j = 0; j < arp_keep.size(); ++j) akey[j] = arp[arp_keep[j]].ip;
    std::vector<std::array<uint32_t, 4>> nwords(ndp_keep.size());
    for (size_t j = 0; j < ndp_keep.size(); ++j) {
        const uint8_t* ip = ndp[ndp_keep[j]].ip;
        nwords[j] = {le32(ip), le32(ip + 4), le32(ip + 8), le32(ip + 12)};
        nkey[j] = fold_v6(nwords[j].data());
    }
    uint32_t abits = 0, aseed = 0, nbits = 0, nseed = 0;
    std::vector<int32_t> aslot, nslot;   // slot -> entry (index into *_keep), -1 empty
    if (cuckoo3_place(akey, abits, aseed, aslot) != 0 || cuckoo3_place(nkey, nbits, nseed, nslot) != 0)
        return fail("neighbour index: cuckoo placement failed");
    std::vector<uint4> a(aslot.size(), make_uint4(0, 0, 0, 0));
    for (size_t t = 0; t < aslot.size(); ++t) {
        if (aslot[t] < 0) continue;
        const upe_arp_entry_t& e = arp[arp_keep[aslot[t]]];
        a[t] = make_uint4(e.ip, mac_lo(e.mac), mac_hi(e.mac) | (1u << 16), 0);
    }
    std::vector<uint4> b(2 * nslot.size(), make_uint4(0, 0, 0, 0));
    for (size_t t = 0; t < nslot.size(); ++t) {
        if (nslot[t] < 0) continue;
        const upe_ndp_entry_t& e = ndp[ndp_keep[nslot[t]]];
        const auto& w = nwords[nslot[t]];
        b[2 * t] = make_uint4(w[0], w[1], w[2], w[3]);
        b[2 * t + 1] = make_uint4(mac_lo(e.mac), mac_hi(e.mac) | (1u << 16), 0, 0);
    }
    if (a.empty()) a.push_back(make_uint4(0, 0, 0, 0));   // keep a valid allocation
    if (b.empty()) b.resize(2, make_uint4(0, 0, 0, 0));
    // the last batch's L1 outcome into the starting state before the tables change
    if (c->st && l1_sync(c) != 0) return -1;
    if (c->last_stream) HIP_TRY(hipStreamSynchronize(c->last_stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->arp) (void)hipFree(c->arp);
    if (c->ndp) (void)hipFree(c->ndp);
    c->arp = nullptr; c->ndp = nullptr;
    HIP_TRY(hipMalloc(&c->arp, a.size() * sizeof(uint4)));
    HIP_TRY(hipMalloc(&c->ndp, b.size() * sizeof(uint4)));
    HIP_TRY(hipMemcpy(c->arp, a.data(), a.size() * sizeof(uint4), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->ndp, b.data(), b.size() * sizeof(uint4), hipMemcpyHostToDevice));
    c->arp_bits = abits;
    c->arp_seed = aseed;
    c->ndp_bits = nbits;
    c->ndp_seed = nseed;
    if (c->st && refresh(c) != 0) return -1;   // does the L1 state agree with the new tables?
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

int upe_gpu_set_port(upe_gpu_ctx_t* c, const uint8_t eth_addr[6], uint32_t ip4_addr) {
    if (!c || !eth_addr) return fail("null argument");
    c->port_mac_lo = mac_lo(eth_addr);
    c->port_mac_hi = mac_hi(eth_addr);
    c->port_ip4 = ip4_addr;
    return 0;
}

int upe_gpu_set_l1(upe_gpu_ctx_t* c, const upe_l1_state_t* l1) {
    if (!c || !l1) return fail("null argument");
    DEV_SCOPE(c->device);
    DevL1 d;
    memset(&d, 0, sizeof d);
    d.arp_ip = l1->last_arp_ip;
    d.arp_mac_lo = mac_lo(l1->last_arp_mac);
    d.arp_mac_hi = mac_hi(l1->last_arp_mac);
    for (int j = 0; j < 4; ++j) d.ndp_ip[j] = le32(l1->last_ndp_ip + 4 * j);
    d.ndp_mac_lo = mac_lo(l1->last_ndp_mac);
    d.ndp_mac_hi = mac_hi(l1->last_ndp_mac);
    // the pending batch's outcome is replaced, not folded in later: fold (clears it), overwrite
    if (l1_sync(c) != 0) return -1;
    HIP_TRY(hipMemcpyAsync(l1_slot(c, c->k), &d, sizeof d, hipMemcpyHostToDevice, c->stream));
    if (refresh(c) != 0) return -1;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

int upe_gpu_get_l1(upe_gpu_ctx_t* c, upe_l1_state_t* l1) {
    if (!c || !l1) return fail("null argument");
    DEV_SCOPE(c->device);
    if (l1_sync(c) != 0) return -1;
    HIP_TRY(hipDeviceSynchronize());
    DevL1 d;
    HIP_TRY(hipMemcpy(&d, l1_slot(c, c->k), sizeof d, hipMemcpyDeviceToHost));
    memset(l1, 0, sizeof *l1);
    l1->last_arp_ip = d.arp_ip;
    memcpy(l1->last_arp_mac, &d.arp_mac_lo, 4);
    memcpy(l1->last_arp_mac + 4, &d.arp_mac_hi, 2);
    memcpy(l1->last_ndp_ip, d.ndp_ip, 16);
    memcpy(l1->last_ndp_mac, &d.ndp_mac_lo, 4);
    memcpy(l1->last_ndp_mac + 4, &d.ndp_mac_hi, 2);
    return 0;
}

}  // extern "C"

namespace {
// One batch: the classify launch (in place, or emit mode when d_hdr is given), plus the
// rule_stats group-by for tables over kLdsStatsMax rules.  A launch takes at most kMaxLaunch
// packets (the kernel's per-lane counters are 16-bit halves; a lane sees at most one packet
// per tile).
constexpr size_t kMaxLaunch = (size_t)1 << 24;
static_assert(kMaxLaunch % 64 == 0, "a split launch starts on a 64-packet group (egress list)");
// A ring launch's completion stamps (upe_gpu_process_ring_emit): batches of `per` packets.
struct RingReq {
    size_t per;
    unsigned long long* done;   // [count] ns after the first workgroup's start, 0 = not stamped
};
int process_impl(upe_gpu_ctx_t* c, uint8_t* d_frames, const uint64_t* d_desc, uint32_t* d_verdict,
                 uint32_t* d_flow_hash, upe_hdr_rec_t* d_hdr, size_t n, void* stream,
                 const RingReq* ring = nullptr, bool host = false, uint32_t* d_tx = nullptr,
                 uint32_t* d_tx_cnt = nullptr, size_t tx_base = 0) {
    if (!c) return fail("null context");
    host = host || c->host_tag;
    if (n > 0xFFFFFFFFull - kTile) return fail("batch too large (n must fit in 32 bits)");
    if (n && (!d_frames || !d_desc || !d_verdict)) return fail("null batch buffer");
    if (((uintptr_t)d_frames & 15u) != 0) return fail("frames buffer must be 16-byte aligned");
    if (((uintptr_t)d_hdr & 15u) != 0) return fail("header records must be 16-byte aligned");
    if (ring && n > kMaxLaunch) return fail("a ring holds at most 2^24 packets");
    if (n > kMaxLaunch) {
        // consecutive launches of at most kMaxLaunch packets: the worker's stream semantics are
        // those of one batch (batch_info describes the last launch)
        for (size_t s0 = 0; s0 < n; s0 += kMaxLaunch) {
            const size_t m = n - s0 < kMaxLaunch ? n - s0 : kMaxLaunch;
            if (process_impl(c, d_frames, d_desc + s0, d_verdict + s0,
                             d_flow_hash ? d_flow_hash + s0 : nullptr, d_hdr ? d_hdr + s0 : nullptr,
                             m, stream, nullptr, host, d_tx ? d_tx + s0 : nullptr,
                             d_tx_cnt ? d_tx_cnt + s0 / 64 : nullptr, tx_base + s0) != 0)
                return -1;
        }
        return 0;
    }
    DEV_SCOPE(c->device);
    hipStream_t s = pick(c, stream);
    const uint32_t ntiles = (uint32_t)((n + kTile - 1) / kTile);
    if (ensure_scratch(c, ntiles ? ntiles : 1) != 0) return -1;
    // after the context's previous launch and its own uploads (tables, L1), on whichever stream
    // they went: a batch starts from the state the one before it left
    if (order_on(c, s) != 0) return -1;
    // timing sample: an event pair around `timing_span` consecutive calls, opened on every
    // timing_every-th call (samples never overlap)
    const bool open = c->timing && c->t_left == 0 &&
                      (c->timing_calls % c->timing_every) == c->timing_phase;
    if (c->timing) ++c->timing_calls;
    if (open) {
        while (c->ev.size() < c->ev_used + 3) {
            hipEvent_t e;
            HIP_TRY(hipEventCreate(&e));
            c->ev.push_back(e);
        }
        HIP_TRY(hipEventRecord(c->ev[c->ev_used], s));
        c->t_left = c->timing_span;
    }
    Args a;
    memset(&a, 0, sizeof a);   // every field a launch does not set stays null / zero
    a.frames = d_frames;
    a.desc = d_desc;
    a.verdict = d_verdict;
    a.n = (uint32_t)n;
    a.tx = d_tx;
    a.tx_cnt = d_tx_cnt;
    a.tx_base = (uint32_t)tx_base;
    a.rv4 = c->rv4;
    a.rv6 = c->rv6;
    a.fam = c->fam;
    a.fam4 = c->fam4;
    a.fam6 = c->fam6;
    a.fam_x1idx = c->fam_x1idx;
    a.tree = reinterpret_cast<const uint2*>(c->tree);
    a.tree_loff = c->tree_loff;
    a.rinfo = c->rinfo;
    a.nrules_pad = c->nrules_pad;
    a.arp = arp_index(c);
    a.ndp = ndp_index(c);
    a.st = c->st;
    a.port_mac_lo = c->port_mac_lo;
    a.port_mac_hi = c->port_mac_hi;
    a.port_ip4 = c->port_ip4;
    a.tg4 = c->tg4;
    a.tg6 = c->tg6;
    a.tt4 = c->tt4;
    a.tt6 = c->tt6;
    a.tfs = reinterpret_cast<const uint4*>(c->tfs);
    a.ng4 = c->ng4;
    a.ng6 = c->ng6;
    a.tss = c->tss ? 1u : 0u;
    a.pay = c->pay;
    a.paycap = c->paycap;
    a.k6 = (uint32_t)(c->k % 6);
    a.lb = c->lb;
    a.defer = c->defer;
    a.lb_spin = c->lb_spin;
    a.lb_tag = (uint32_t)(c->k % kLbTagMod) + 1u;
    if (c->k > 0 && c->k % kLbTagMod == 0)   // tags wrap: no flag may carry this launch's tag
        HIP_TRY(hipMemsetAsync(c->lb, 0, c->tiles_alloc * kWaves * sizeof(uint32_t), s));
    a.stats = c->stats;
    a.stats_idx = c->stats_idx;
    a.flow_hash = d_flow_hash;
    a.hdr = reinterpret_cast<uint4*>(d_hdr);
    const bool emit = d_hdr != nullptr && n > 0;
    const bool lds_stats = c->nrules_pad <= (uint32_t)kLdsStatsMax;
    a.gb = nullptr;
    a.gb_packed = c->nrules <= 65536u ? 1u : 0u;   // sorted indexes of matches < nrules
    if (!lds_stats && n > 0) {
        if (n > c->gb_alloc) {
            if (c->gb) (void)hipFree(c->gb);
            c->gb = nullptr;
            c->gb_alloc = 0;
            const size_t want = (n + n / 4 + 64) & ~(size_t)3;
            HIP_TRY(hipMalloc(&c->gb, want * sizeof(uint32_t)));   // room for either form
            c->gb_alloc = want;
        }
        a.gb = c->gb;
    }
    const size_t hist = lds_stats ? 2 * (size_t)c->nrules_pad * sizeof(uint32_t) : 0;
    // large linear tables: the decision tree (when built), else family lists, unless a family's
    // list is a single catch-all (then the split gains that family nothing and measured slower
    // for the other)
    const int scan = c->tss || c->nrules_pad <= (uint32_t)kSmallRules ? 0
                   : c->tree_ok ? 3 : c->fam_all ? 2 : 1;
    const size_t lds_max = scan ? kLdsDynMaxLarge : kLdsDynMax;
    // stage the ARP index in LDS when it is small (the nrules_pad multiple of 4 keeps the slot
    // array 16-byte aligned after the bins)
    const uint32_t arp_slots = c->arp_bits ? (1u << c->arp_bits) : 0u;
    const uint32_t ndp_slots = c->ndp_bits ? (1u << c->ndp_bits) : 0u;
    size_t lds = hist;
    a.arp_lds = a.ndp_lds = 0u;
    if (arp_slots && arp_slots <= kArpLdsSlots && lds + arp_slots * sizeof(uint4) <= lds_max) {
        a.arp_lds = arp_slots;
        lds += arp_slots * sizeof(uint4);
    }
    if (ndp_slots && ndp_slots <= kNdpLdsSlots && lds + 2 * ndp_slots * sizeof(uint4) <= lds_max) {
        a.ndp_lds = ndp_slots;
        lds += 2 * ndp_slots * sizeof(uint4);
    }
    a.fp_lds = 0u;
    if (c->tss && c->nfs && lds + c->nfs * sizeof(uint4) <= lds_max) {
        a.fp_lds = c->nfs;
        lds += c->nfs * sizeof(uint4);
    }
    // the tree's image in LDS first (every lane reads a node per level), then the IPv6 list
    a.tree_lds = 0u;
    if (scan == 3 && c->tree_stage && lds + c->tree_words * sizeof(uint4) <= lds_max) {
        a.tree_lds = c->tree_words;
        lds += c->tree_words * sizeof(uint4);
    }
    a.fam6_lds = 0u;
    if (kFamLds && !c->tss && (scan == 3 || !c->fam_all) && c->fam6 &&
        lds + kFamV6Stride * c->fam6 * sizeof(uint4) <= lds_max) {
        a.fam6_lds = 1u;
        lds += kFamV6Stride * c->fam6 * sizeof(uint4);
    }
    // the tree kernels' leaf tests read the IPv4 list's rule words too: from LDS when it fits
    a.fam4_lds = 0u;
    if (scan == 3 && c->tree_stage && c->fam4 && lds + 2 * c->fam4 * sizeof(uint4) <= lds_max) {
        a.fam4_lds = 1u;
        lds += 2 * c->fam4 * sizeof(uint4);
    }
    // the lean emit kernel when nothing it leaves out is needed (non-empty neighbour indexes
    // all in LDS, no flow_hash, no length side array)
    const bool lean = !d_flow_hash && (c->tss || !a.gb) &&
                      (arp_slots == 0 || a.arp_lds != 0) && (ndp_slots == 0 || a.ndp_lds != 0);
    // once a launch has been seen starting from agreeing L1 entries (or from an entry whose
    // family's index is empty), every later one does until the host changes tables or entries
    if (!c->no_lb && c->agree_h && c->allow_nolb) {
        if (c->lb_sync && c->k > c->lb_reset_k && c->last_stream)
            HIP_TRY(hipStreamSynchronize(c->last_stream));   // the previous launch's report
        const unsigned long long v = __atomic_load_n(c->agree_h, __ATOMIC_ACQUIRE);
        const unsigned long long tag = v >> 2;
        if (tag != 0 && tag - 1 >= c->lb_reset_k && ((v & 1) || c->arp_bits == 0 || !c->fwd4) &&
            ((v & 2) || c->ndp_bits == 0 || !c->fwd6))
            c->no_lb = true;
    }
    a.agree_out = c->no_lb ? nullptr : c->agree_d;
    a.launch_tag = c->k + 1;
    // a ring launch stamps its batches' completion with the ring kernels (lean emit linear scan)
    // (at most kRingMax batches: one LDS counter each)
    bool stamp = ring && ring->done && emit && lean && !c->tss && n / ring->per <= (size_t)kRingMax;
    const bool tx = d_tx != nullptr;   // (emit, device batches: upe_gpu_process_emit_tx)
    if (tx) stamp = host = false;
    int var = classify_var(c->tss, emit, lean, c->no_lb, stamp, host, scan, tx);
    // persistent grid: the workgroups the chip holds at once (or one per tile if fewer)
    uint32_t grid_cap = resident_grid(c, var, lds, s);
    if (grid_cap == 0) return -1;
    // the census of the no-look-back counterpart now as well, so that the switch to it (a few
    // launches later) does not put a synchronous census launch in the middle of a batch stream
    if (lean && !c->no_lb &&
        resident_grid(c, classify_var(c->tss, emit, true, true, stamp, host, scan, tx), lds, s) == 0)
        return -1;
    // Tiles of kWaves chunks (one per wave of a workgroup); a batch too small to give every
    // resident workgroup a tile gets narrower tiles, down to one chunk, so that it spreads over
    // more CUs (a 10k-packet batch on ten CUs, four waves per SIMD, took 9.2 us; spread, 7.9).
    const uint32_t nchunks = (uint32_t)((n + 63) / 64);
    uint32_t tw = (uint32_t)kWaves;
    while (tw > 1 && (nchunks + tw - 1) / tw < grid_cap) tw >>= 1;
    a.tw = tw;
    a.ntiles = (nchunks + tw - 1) / tw;
    const uint32_t grid = a.ntiles == 0 ? 1u : a.ntiles < grid_cap ? a.ntiles : grid_cap;
    if (ring && ring->done) {
        HIP_TRY(hipMemsetAsync(ring->done, 0, (n / ring->per) * sizeof(unsigned long long), s));
        // every workgroup must own the same number of tiles of every batch (at least one)
        const size_t tpb = (ring->per / 64) / tw;
        if (stamp && (tpb < grid || tpb % grid != 0)) stamp = false;
        if (!stamp) {
            var = classify_var(c->tss, emit, lean, c->no_lb, false, false, scan);
            if (resident_grid(c, var, lds, s) == 0) return -1;
        } else {
            const size_t nb = n / ring->per;
            if (nb > c->ring_alloc) {
                if (c->ring_wg) HIP_TRY(hipFree(c->ring_wg));
                c->ring_wg = nullptr;
                c->ring_alloc = 0;
                HIP_TRY(hipMalloc(&c->ring_wg, (nb + 2) * sizeof(unsigned long long)));
                c->ring_alloc = nb;
            }
            HIP_TRY(hipMemsetAsync(c->ring_wg, 0, nb * sizeof(unsigned long long), s));
            HIP_TRY(hipMemsetAsync(c->ring_wg + nb, 0xFF, sizeof(unsigned long long), s));
            a.ring_cpb = (uint32_t)(ring->per / 64);
            a.ring_mine = (uint32_t)(tpb / grid * tw);
            a.ring_wg = reinterpret_cast<uint32_t*>(c->ring_wg);
            a.ring_done = ring->done;
            a.ring_t0 = c->ring_wg + nb;
        }
    }
    launch_classify(var, grid, lds, s, a);
    HIP_TRY(hipGetLastError());
    c->last_var = var;
    c->last_grid = grid;
    const bool group_by = !lds_stats && n > 0;
    // the sample's middle event, between the classify launch and the group-by (last call of the
    // sample only; launches without a group-by have none)
    const bool mid = c->t_left == 1 && group_by;
    if (mid) HIP_TRY(hipEventRecord(c->ev[c->ev_used + 1], s));
    if (group_by) {
        // bins for up to kHistRange rules per workgroup; packet chunks halved (down to
        // kHistChunkMin) while the grid has fewer than about kHistTarget workgroups
        // (over the rules that can match, sorted indexes 0..nrules-1: the padding block never
        // does, and counting it cost config D a fifth range pass over the batch)
        const uint32_t nrules = c->nrules ? c->nrules : 1u;
        const uint32_t range = nrules < kHistRange ? nrules : kHistRange;
        const uint32_t nr = (nrules + range - 1) / range;
        uint32_t chunk = kHistChunk;
        while (chunk > kHistChunkMin && ((n + chunk / 2 - 1) / (chunk / 2)) * nr <= kHistTarget)
            chunk >>= 1;
        const dim3 hg((uint32_t)((n + chunk - 1) / chunk), nr);
        // dense partials: one 8-byte bin per chunk and rule, summed by upe_hist_reduce
        const size_t part_words = (size_t)hg.x * nrules;
        if (part_words > c->hist_part_alloc) {
            if (c->hist_part) (void)hipFree(c->hist_part);
            c->hist_part = nullptr;
            c->hist_part_alloc = 0;
            HIP_TRY(hipMalloc(&c->hist_part, part_words * sizeof(unsigned long long)));
            c->hist_part_alloc = part_words;
        }
        static std::atomic<uint64_t> hist_attr{0};   // 128 KB of dynamic LDS, once per device
        if (!(hist_attr.fetch_or(1ull << (c->device & 63)) & (1ull << (c->device & 63)))) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&upe_rule_hist<true>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)(kHistRange * sizeof(unsigned long long)));
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&upe_rule_hist<false>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)(kHistRange * sizeof(unsigned long long)));
        }
        if (a.gb_packed)
            hipLaunchKernelGGL(upe_rule_hist<true>, hg, dim3(kHistBlock), range * sizeof(unsigned long long), s,
                               d_verdict, c->gb, (uint32_t)n, nrules, c->hist_part, chunk, range);
        else
            hipLaunchKernelGGL(upe_rule_hist<false>, hg, dim3(kHistBlock), range * sizeof(unsigned long long), s,
                               d_verdict, c->gb, (uint32_t)n, nrules, c->hist_part, chunk, range);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(upe_hist_reduce, dim3((nrules + 255) / 256, kStatReps),
                           dim3(256), 0, s, c->hist_part, hg.x, nrules, c->nrules_pad, c->stats_idx);
        HIP_TRY(hipGetLastError());
    }
    if (c->t_left && --c->t_left == 0) {
        HIP_TRY(hipEventRecord(c->ev[c->ev_used + 2], s));
        c->ev_mid.push_back(mid);
        c->ev_used += 3;
        c->timing_launches += c->timing_span;
    }
    ++c->k;
    c->last_n = (uint32_t)n;
    c->have_batch = true;
    return 0;
}
}  // namespace

extern "C" {

int upe_gpu_process(upe_gpu_ctx_t* c, uint8_t* d_frames, const uint64_t* d_desc,
                    uint32_t* d_verdict, size_t n, void* stream) {
    return process_impl(c, d_frames, d_desc, d_verdict, nullptr, nullptr, n, stream);
}

int upe_gpu_process_rss(upe_gpu_ctx_t* c, uint8_t* d_frames, const uint64_t* d_desc,
                        uint32_t* d_verdict, uint32_t* d_flow_hash, size_t n, void* stream) {
    return process_impl(c, d_frames, d_desc, d_verdict, d_flow_hash, nullptr, n, stream);
}

int upe_gpu_process_emit(upe_gpu_ctx_t* c, uint8_t* d_frames, const uint64_t* d_desc,
                         uint32_t* d_verdict, upe_hdr_rec_t* d_hdr, size_t n, void* stream) {
    if (n && !d_hdr) return fail("null header records");
    return process_impl(c, d_frames, d_desc, d_verdict, nullptr, d_hdr, n, stream);
}

int upe_gpu_process_emit_tx(upe_gpu_ctx_t* c, uint8_t* d_frames, const uint64_t* d_desc,
                            uint32_t* d_verdict, upe_hdr_rec_t* d_hdr, uint32_t* d_tx,
                            uint32_t* d_tx_count, size_t n, void* stream) {
    if (n && (!d_hdr || !d_tx || !d_tx_count)) return fail("null header records or egress list");
    return process_impl(c, d_frames, d_desc, d_verdict, nullptr, d_hdr, n, stream, nullptr, false,
                        d_tx, d_tx_count);
}

int upe_gpu_process_ring_emit(upe_gpu_ctx_t* c, uint8_t* d_frames, const uint64_t* d_desc,
                              uint32_t* d_verdict, upe_hdr_rec_t* d_hdr, size_t n, size_t count,
                              uint64_t* d_done_ns, void* stream) {
    if (!c) return fail("null context");
    if (count == 0 || n == 0) return 0;
    if (!d_hdr) return fail("null header records");
    if (n % 1024 != 0) return fail("a ring batch must hold a multiple of 1024 packets");
    if (n * count > kMaxLaunch) return fail("a ring holds at most 2^24 packets");
    const RingReq r{n, reinterpret_cast<unsigned long long*>(d_done_ns)};
    return process_impl(c, d_frames, d_desc, d_verdict, nullptr, d_hdr, n * count, stream, &r);
}

}  // extern "C"

namespace {
// The host round trip (upe_gpu_process_host / _emit): chunks of the caller's host batch through
// a ring of device slots, H2D on one copy stream, classify on the context's stream, D2H on a
// second copy stream.  In place: the rewritten span [lo, wb) of each chunk comes back.  Emit:
// the verdicts and the 16-byte records come back (20 B per packet instead of the span: the
// link's two directions share its bandwidth, so fewer bytes back let more go in), and when
// apply_threads >= 0 the records are applied to the caller's frames on the host two chunks
// behind, by the calling thread and `apply_threads` pool threads, while later chunks move.
int host_roundtrip(upe_gpu_ctx_t* c, uint8_t* h_frames, size_t frames_bytes,
                   const uint64_t* h_desc, uint32_t* h_verdict, upe_hdr_rec_t* h_hdr, size_t n,
                   size_t chunk, bool emit, int apply_threads) {
    if (!c) return fail("null context");
    if (n && (!h_frames || !h_desc || !h_verdict || (emit && !h_hdr))) return fail("null host buffer");
    DEV_SCOPE(c->device);
    // default chunks (round-3 sweep, config B 1M): in place 256k (479 Mpps; 128k 406, 64k 359),
    // emit 128k (559 Mpps; 256k 534, 64k 529)
    if (chunk == 0) chunk = emit ? (size_t)1 << 17 : (size_t)1 << 18;
    // emit: whole 64-packet groups per chunk, so that each chunk's compacted records (relative to
    // its first packet) land where the batch's own layout puts them
    if (emit) chunk = std::max<size_t>(64, chunk & ~(size_t)63);
    if (!c->s_in) {
        HIP_TRY(hipStreamCreateWithFlags(&c->s_in, hipStreamNonBlocking));
        HIP_TRY(hipStreamCreateWithFlags(&c->s_out, hipStreamNonBlocking));
        for (auto& sl : c->hs) {
            HIP_TRY(hipEventCreateWithFlags(&sl.in_done, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&sl.k_done, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&sl.out_done, hipEventDisableTiming));
        }
    }
    if (n == 0) {
        if (upe_gpu_process(c, nullptr, nullptr, nullptr, 0, nullptr) != 0) return -1;
        HIP_TRY(hipStreamSynchronize(c->stream));
        return 0;
    }
    const bool apply = emit && apply_threads >= 0;
    if (apply && apply_threads > 0 && (!c->pool || c->pool->th.size() != (size_t)apply_threads)) {
        std::vector<int> cpus(CPU_SETSIZE);
        const int k = upe_gpu_local_cpus(c->device, cpus.data(), cpus.size(), nullptr);
        cpus.resize(k > 0 ? (size_t)k : 0);
        c->pool.reset();
        c->pool.reset(new ApplyPool((unsigned)apply_threads, cpus));
    }
    // Whatever happens below, no copy into the caller's buffers is left in flight on return.
    struct Drain {
        upe_gpu_ctx* c;
        ~Drain() {
            (void)hipStreamSynchronize(c->s_in);
            (void)hipStreamSynchronize(c->stream);
            (void)hipStreamSynchronize(c->s_out);
            for (auto& sl : c->hs) sl.busy = false;
        }
    } drain{c};
    const size_t nslots = c->host_slots;
    // copies back on their own stream: both link directions at once (issuing them on the copy-in
    // stream after the next chunk's copy-in measured slower: B 332-344 vs 480 Mpps in place)
    hipStream_t s_back = c->s_out;
    const size_t lag = 2;   // emit: chunk k - lag is applied while chunk k is issued
    struct Done {
        size_t s, e, slot;
        uint64_t lo;
    };
    std::vector<Done> pending;
    // apply chunk d's records (and copy back its answered ARP requests, rewritten in place in
    // the device slot, which the reference transmits from b->data, src/worker.c:40-52)
    auto finish = [&](const Done& d) -> int {
        auto& sl = c->hs[d.slot];
        HIP_TRY(hipEventSynchronize(sl.out_done));
        std::atomic<bool> replies{false};
        auto job = [&](unsigned t, unsigned T) {
            const size_t m = d.e - d.s, a0 = d.s + m * t / T, a1 = d.s + m * (t + 1) / T;
            bool r = false;
            // the compacted record of the range's first forwarded packet
            size_t rec = a0 & ~(size_t)63;
            for (size_t j = rec; j < a0; ++j) rec += UPE_VERDICT_CODE(h_verdict[j]) == UPE_V_FWD;
            for (size_t i = a0; i < a1; ++i) {
                r |= (h_verdict[i] & UPE_VF_ARP_REPLY) != 0;
                if ((i & 63u) == 0) rec = i;
                if (UPE_VERDICT_CODE(h_verdict[i]) == UPE_V_FWD) {
                    if (apply) upe_hdr_apply(h_frames + (h_desc[i] >> 16), &h_hdr[rec]);
                    ++rec;
                }
            }
            if (r) replies.store(true, std::memory_order_relaxed);
        };
        if (c->pool && apply && apply_threads > 0) c->pool->run(job);
        else job(0, 1);
        if (replies.load())
            for (size_t i = d.s; i < d.e; ++i)
                if (h_verdict[i] & UPE_VF_ARP_REPLY) {
                    const uint64_t off = h_desc[i] >> 16, len = h_desc[i] & 0xFFFFu;
                    HIP_TRY(hipMemcpy(h_frames + off, sl.frames + (off - d.lo),
                                      len < UPE_REWRITE_EXTENT ? len : UPE_REWRITE_EXTENT,
                                      hipMemcpyDeviceToHost));
                }
        return 0;
    };
    // a chunk's copy-back (verdicts + records, or verdicts + the rewritten span), once its kernel
    // is queued
    auto issue_back = [&](size_t s, size_t e, size_t slot, uint64_t lo, uint64_t wb) -> int {
        auto& sb = c->hs[slot];
        const size_t m = e - s;
        HIP_TRY(hipStreamWaitEvent(s_back, sb.k_done, 0));
        HIP_TRY(hipMemcpyAsync(h_verdict + s, sb.verdict, m * sizeof(uint32_t),
                               hipMemcpyDeviceToHost, s_back));
        if (emit)
            HIP_TRY(hipMemcpyAsync(h_hdr + s, sb.hdr, m * sizeof(upe_hdr_rec_t),
                                   hipMemcpyDeviceToHost, s_back));
        else
            HIP_TRY(hipMemcpyAsync(h_frames + lo, sb.frames, (size_t)(wb - lo),
                                   hipMemcpyDeviceToHost, s_back));
        HIP_TRY(hipEventRecord(sb.out_done, s_back));
        sb.busy = true;
        sb.lo = lo;
        sb.wb = wb;
        return 0;
    };
    size_t k = 0;
    for (size_t s = 0; s < n; s += chunk, ++k) {
        const size_t e = n - s < chunk ? n : s + chunk, m = e - s;
        // The chunk's byte ranges: [lo, hi) holds every frame's window (the kernel reads up to
        // UPE_FRAME_TAIL bytes from a frame start), [lo, wb) every byte the kernel may rewrite.
        // The scan of chunk k+1 overlaps the copies and kernel of chunk k.
        uint64_t lo = ~0ull, hi = 0, wb = 0;
        for (size_t i = s; i < e; ++i) {
            const uint64_t off = h_desc[i] >> 16, len = h_desc[i] & 0xFFFFu;
            if (off & 15u) return fail("frame offsets must be multiples of 16 (include/upe_gpu.h)");
            lo = off < lo ? off : lo;
            hi = off + UPE_FRAME_TAIL > hi ? off + UPE_FRAME_TAIL : hi;
            const uint64_t w = off + (len < UPE_REWRITE_EXTENT ? len : UPE_REWRITE_EXTENT);
            wb = w > wb ? w : wb;
        }
        if (hi > frames_bytes)
            return fail("a frame window runs past frames_bytes (UPE_FRAME_TAIL bytes must follow "
                        "every frame start)");
        const size_t si = k % nslots;
        auto& sl = c->hs[si];
        if (emit && pending.size() >= lag) {   // the oldest finished before its slot is reused
            if (finish(pending.front()) != 0) return -1;
            pending.erase(pending.begin());
        }
        if (sl.busy) HIP_TRY(hipEventSynchronize(sl.out_done));   // the slot's last D2H is done
        sl.busy = false;
        const size_t span = (size_t)(hi - lo);
        if (span > sl.frames_cap) {
            if (sl.frames) HIP_TRY(hipFree(sl.frames));
            sl.frames = nullptr;
            sl.frames_cap = 0;
            const size_t want = span + span / 4;
            HIP_TRY(hipMalloc(&sl.frames, want));
            sl.frames_cap = want;
        }
        if (m > sl.pk_cap || (emit && !sl.hdr)) {
            for (void* b : {(void*)sl.desc, (void*)sl.verdict, (void*)sl.hdr})
                if (b) HIP_TRY(hipFree(b));
            sl.desc = nullptr;
            sl.verdict = nullptr;
            sl.hdr = nullptr;
            const size_t cap = std::max(m, sl.pk_cap);
            sl.pk_cap = 0;
            HIP_TRY(hipMalloc(&sl.desc, cap * sizeof(uint64_t)));
            HIP_TRY(hipMalloc(&sl.verdict, cap * sizeof(uint32_t)));
            if (emit) HIP_TRY(hipMalloc(&sl.hdr, cap * sizeof(upe_hdr_rec_t)));
            sl.pk_cap = cap;
        }
        // In place: a chunk whose bytes interleave with an earlier chunk's (descriptors in any
        // order, e.g. pool addresses) must read them only after that chunk's copy-back has
        // landed: its own copy-back rewrites its whole span, and would otherwise put back the
        // earlier chunk's frames as they were before they were processed.  (Emit mode copies
        // no frame bytes back.)
        if (!emit)
            for (auto& other : c->hs)
                if (&other != &sl && other.busy && other.lo < hi && lo < other.wb)
                    HIP_TRY(hipStreamWaitEvent(c->s_in, other.out_done, 0));
        HIP_TRY(hipMemcpyAsync(sl.frames, h_frames + lo, span, hipMemcpyHostToDevice, c->s_in));
        HIP_TRY(hipMemcpyAsync(sl.desc, h_desc + s, m * sizeof(uint64_t), hipMemcpyHostToDevice,
                               c->s_in));
        HIP_TRY(hipEventRecord(sl.in_done, c->s_in));
        HIP_TRY(hipStreamWaitEvent(c->stream, sl.in_done, 0));
        // the descriptors keep their offsets relative to h_frames: hand the kernel a base that
        // maps offset lo onto the slot (lo is a multiple of 16, so the base stays aligned)
        uint8_t* base = reinterpret_cast<uint8_t*>(reinterpret_cast<uintptr_t>(sl.frames) - lo);
        // (the host-path kernel instantiation: profiles keep these launches apart)
        if (process_impl(c, base, sl.desc, sl.verdict, nullptr, emit ? sl.hdr : nullptr, m,
                         nullptr, nullptr, true) != 0)
            return -1;
        HIP_TRY(hipEventRecord(sl.k_done, c->stream));
        if (issue_back(s, e, si, lo, wb) != 0) return -1;
        if (emit) pending.push_back(Done{s, e, si, lo});
    }
    for (const Done& d : pending)
        if (finish(d) != 0) return -1;
    HIP_TRY(hipStreamSynchronize(s_back));
    return 0;
}
}  // namespace

extern "C" {

int upe_gpu_process_host(upe_gpu_ctx_t* c, uint8_t* h_frames, size_t frames_bytes,
                         const uint64_t* h_desc, uint32_t* h_verdict, size_t n, size_t chunk) {
    return host_roundtrip(c, h_frames, frames_bytes, h_desc, h_verdict, nullptr, n, chunk, false,
                          -1);
}

int upe_gpu_process_host_emit(upe_gpu_ctx_t* c, uint8_t* h_frames, size_t frames_bytes,
                              const uint64_t* h_desc, uint32_t* h_verdict, upe_hdr_rec_t* h_hdr,
                              size_t n, size_t chunk, int apply_threads) {
    if (apply_threads > 64) return fail("apply_threads must be at most 64");
    return host_roundtrip(c, h_frames, frames_bytes, h_desc, h_verdict, h_hdr, n, chunk, true,
                          apply_threads);
}

void* upe_gpu_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
        fail("hipHostMalloc failed");
        return nullptr;
    }
    return p;
}

int upe_gpu_host_free(void* p) {
    if (p) HIP_TRY(hipHostFree(p));
    return 0;
}

int upe_gpu_host_register(void* p, size_t bytes) {
    if (!p || !bytes) return fail("null or empty host buffer");
    HIP_TRY(hipHostRegister(p, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    return 0;
}

int upe_gpu_host_unregister(void* p) {
    if (!p) return fail("null host buffer");
    HIP_TRY(hipHostUnregister(p));
    return 0;
}

}  // extern "C"

namespace {
// The device address of page-locked, mapped host memory; nullptr (and an error) for anything
// else, so that a kernel never dereferences an unmapped host address.
template <typename T>
T* mapped(T* h, const char* what) {
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, const_cast<void*>(static_cast<const void*>(h)), 0) != hipSuccess ||
        !d) {
        (void)hipGetLastError();
        fail(std::string(what) + " is not pinned, mapped host memory (upe_gpu_host_alloc / "
             "upe_gpu_host_register)");
        return nullptr;
    }
    return static_cast<T*>(d);
}
}  // namespace

extern "C" {

int upe_gpu_process_mapped(upe_gpu_ctx_t* c, uint8_t* h_frames, const uint64_t* h_desc,
                           uint32_t* h_verdict, size_t n, void* stream) {
    if (!c) return fail("null context");
    DEV_SCOPE(c->device);
    if (n == 0) return upe_gpu_process(c, nullptr, nullptr, nullptr, 0, stream);
    if (!h_frames || !h_desc || !h_verdict) return fail("null host buffer");
    uint8_t* f = mapped(h_frames, "h_frames");
    const uint64_t* d = f ? mapped(h_desc, "h_desc") : nullptr;
    uint32_t* v = d ? mapped(h_verdict, "h_verdict") : nullptr;
    if (!v) return -1;
    return process_impl(c, f, d, v, nullptr, nullptr, n, stream, nullptr, true);
}

int upe_gpu_process_mapped_emit(upe_gpu_ctx_t* c, uint8_t* h_frames, const uint64_t* h_desc,
                                uint32_t* h_verdict, upe_hdr_rec_t* h_hdr, size_t n,
                                void* stream) {
    if (!c) return fail("null context");
    DEV_SCOPE(c->device);
    if (n == 0) return upe_gpu_process(c, nullptr, nullptr, nullptr, 0, stream);
    if (!h_frames || !h_desc || !h_verdict || !h_hdr) return fail("null host buffer");
    uint8_t* f = mapped(h_frames, "h_frames");
    const uint64_t* d = f ? mapped(h_desc, "h_desc") : nullptr;
    uint32_t* v = d ? mapped(h_verdict, "h_verdict") : nullptr;
    upe_hdr_rec_t* h = v ? mapped(h_hdr, "h_hdr") : nullptr;
    if (!h) return -1;
    return process_impl(c, f, d, v, nullptr, h, n, stream, nullptr, true);
}

int upe_gpu_process_batches(upe_gpu_ctx_t* c, uint8_t* const* d_frames_list, const uint64_t* d_desc,
                            uint32_t* d_verdict, size_t n, size_t count, void* stream) {
    if (!c) return fail("null context");
    if (count && !d_frames_list) return fail("null frames list");
    for (size_t k = 0; k < count; ++k)
        if (upe_gpu_process(c, d_frames_list[k], d_desc, d_verdict, n, stream) != 0) return -1;
    return 0;
}

int upe_gpu_process_queue_emit(upe_gpu_ctx_t* c, const upe_gpu_batch_t* batches, size_t count,
                               void* stream) {
    if (!c) return fail("null context");
    if (count && !batches) return fail("null batch list");
    // one launch after another (overlapping consecutive launches on two streams measured slower
    // on MI355X: DESIGN.md §8, round 3); every batch is checked before any is queued
    for (size_t k = 0; k < count; ++k)
        if (batches[k].n && !batches[k].hdr) return fail("null header records in a queued batch");
    for (size_t k = 0; k < count; ++k)
        if (process_impl(c, batches[k].frames, batches[k].desc, batches[k].verdict, nullptr,
                         batches[k].hdr, batches[k].n, stream) != 0)
            return -1;
    return 0;
}

int upe_gpu_process_batches_emit(upe_gpu_ctx_t* c, uint8_t* const* d_frames_list,
                                 const uint64_t* d_desc, uint32_t* d_verdict, upe_hdr_rec_t* d_hdr,
                                 size_t n, size_t count, void* stream) {
    if (!c) return fail("null context");
    if (count && !d_frames_list) return fail("null frames list");
    std::vector<upe_gpu_batch_t> q(count);
    for (size_t k = 0; k < count; ++k) q[k] = upe_gpu_batch_t{d_frames_list[k], d_desc, d_verdict, d_hdr, n};
    return upe_gpu_process_queue_emit(c, q.data(), count, stream);
}

#if UPE_STAMPS
int upe_gpu_diag_stamps(void* host, size_t bytes) {
    HIP_TRY(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), bytes, 0, hipMemcpyDeviceToHost));
    return 0;
}
#endif

int upe_gpu_compact(upe_gpu_ctx_t* c, const uint32_t* d_verdict, size_t n, uint32_t code,
                    uint32_t* d_index, uint64_t* d_count, void* stream) {
    if (!c) return fail("null context");
    if (!d_count || (n && (!d_verdict || !d_index))) return fail("null buffer");
    if (n > 0xFFFFFFFFull - kCompactBlock) return fail("n must fit in 32 bits");
    if (code > 15) return fail("verdict code out of range");
    DEV_SCOPE(c->device);
    hipStream_t s = pick(c, stream);
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(d_count, 0, sizeof(uint64_t), s));
        return 0;
    }
    const uint32_t nb = (uint32_t)((n + kCompactBlock - 1) / kCompactBlock);
    if (nb > c->compact_alloc) {
        if (c->compact_counts) HIP_TRY(hipFree(c->compact_counts));
        c->compact_counts = nullptr;
        c->compact_alloc = 0;
        HIP_TRY(hipMalloc(&c->compact_counts, nb * sizeof(uint32_t)));
        c->compact_alloc = nb;
    }
    hipLaunchKernelGGL(upe_compact_count, dim3(nb), dim3(256), 0, s, d_verdict, (uint32_t)n, code,
                       c->compact_counts);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(upe_compact_write, dim3(nb), dim3(256), 0, s, d_verdict, (uint32_t)n, code,
                       c->compact_counts, nb, d_index,
                       reinterpret_cast<unsigned long long*>(d_count));
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // extern "C"

namespace {

// The table writes of handle_control_packet, restated on the caller's host slot arrays.
// arp_update, reference src/arp_table.c:26-53: home slot ip & (cap-1), linear probe, insert at
// the first free slot or update the slot holding ip, at most cap probes.
void host_arp_update(upe_arp_entry_t* t, size_t cap, uint32_t ip, const uint8_t* mac,
                     int64_t now) {
    const size_t idx = ip & (cap - 1);
    for (size_t k = 0; k < cap; ++k) {
        upe_arp_entry_t& e = t[(idx + k) & (cap - 1)];
        if (!e.valid || e.ip == ip) {
            if (!e.valid) {
                e.valid = true;
                e.ip = ip;
            }
            memcpy(e.mac, mac, 6);
            e.update_at = now;
            return;
        }
    }
}

// ndp_update, reference src/ndp_table.c:39-65 (hash_ipv6 :6-17: XOR of the address's four
// native-endian words, & (cap-1)).
void host_ndp_update(upe_ndp_entry_t* t, size_t cap, const uint8_t* ip, const uint8_t* mac,
                     int64_t now) {
    const uint32_t h = le32(ip) ^ le32(ip + 4) ^ le32(ip + 8) ^ le32(ip + 12);
    const size_t idx = h & (cap - 1);
    for (size_t k = 0; k < cap; ++k) {
        upe_ndp_entry_t& e = t[(idx + k) & (cap - 1)];
        if (!e.valid || memcmp(e.ip, ip, 16) == 0) {
            if (!e.valid) {
                e.valid = true;
                memcpy(e.ip, ip, 16);
            }
            memcpy(e.mac, mac, 6);
            e.update_at = now;
            return;
        }
    }
}

}  // namespace

extern "C" {

int upe_gpu_process_segmented(upe_gpu_ctx_t* c, uint8_t* d_frames, const uint64_t* d_desc,
                              uint32_t* d_verdict, size_t n, upe_arp_entry_t* arp,
                              size_t arp_capacity, upe_ndp_entry_t* ndp, size_t ndp_capacity,
                              int64_t now, size_t* n_writes, void* stream) {
    if (!c) return fail("null context");
    if (n_writes) *n_writes = 0;
    if (n > 0xFFFFFFFFull - kCompactBlock) return fail("batch too large (n must fit in 32 bits)");
    if (n && (!d_frames || !d_desc || !d_verdict)) return fail("null batch buffer");
    if ((arp_capacity && !arp) || (ndp_capacity && !ndp)) return fail("null neighbour table");
    if ((arp_capacity & (arp_capacity - 1)) || (ndp_capacity & (ndp_capacity - 1)))
        return fail("neighbour table capacities must be powers of two");
    if (n == 0) return upe_gpu_process(c, d_frames, d_desc, d_verdict, 0, stream);
    DEV_SCOPE(c->device);
    hipStream_t s = pick(c, stream);
    // 1. mark and list the table-writing control packets, in packet order
    if (n > c->ctrl_alloc) {
        for (void* b : {(void*)c->ctrl_marks, (void*)c->ctrl_index})
            if (b) HIP_TRY(hipFree(b));
        c->ctrl_marks = c->ctrl_index = nullptr;
        c->ctrl_alloc = 0;
        HIP_TRY(hipMalloc(&c->ctrl_marks, n * sizeof(uint32_t)));
        HIP_TRY(hipMalloc(&c->ctrl_index, n * sizeof(uint32_t)));
        if (!c->ctrl_count) HIP_TRY(hipMalloc(&c->ctrl_count, sizeof(uint64_t)));
        c->ctrl_alloc = n;
    }
    hipLaunchKernelGGL(upe_ctrl_mark, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s,
                       d_frames, d_desc, (uint32_t)n, c->ctrl_marks);
    HIP_TRY(hipGetLastError());
    if (upe_gpu_compact(c, c->ctrl_marks, n, 1u, c->ctrl_index, c->ctrl_count, s) != 0) return -1;
    uint64_t cnt = 0;
    HIP_TRY(hipMemcpyAsync(&cnt, c->ctrl_count, sizeof cnt, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (cnt == 0) return upe_gpu_process(c, d_frames, d_desc, d_verdict, n, stream);
    // 2. their bytes, gathered before any segment runs (the ARP reply is built in place)
    if (cnt > c->ctrl_win_alloc) {
        for (void* b : {(void*)c->ctrl_win, (void*)c->ctrl_lens})
            if (b) HIP_TRY(hipFree(b));
        c->ctrl_win = nullptr;
        c->ctrl_lens = nullptr;
        c->ctrl_win_alloc = 0;
        HIP_TRY(hipMalloc(&c->ctrl_win, cnt * kCtrlWin));
        HIP_TRY(hipMalloc(&c->ctrl_lens, cnt * sizeof(uint32_t)));
        c->ctrl_win_alloc = cnt;
    }
    hipLaunchKernelGGL(upe_ctrl_gather, dim3((uint32_t)cnt), dim3(kCtrlWin), 0, s, d_frames,
                       d_desc, c->ctrl_index, c->ctrl_win, c->ctrl_lens);
    HIP_TRY(hipGetLastError());
    std::vector<uint32_t> idx(cnt), lens(cnt);
    std::vector<uint8_t> win(cnt * kCtrlWin);
    HIP_TRY(hipMemcpyAsync(idx.data(), c->ctrl_index, cnt * sizeof(uint32_t),
                           hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(lens.data(), c->ctrl_lens, cnt * sizeof(uint32_t),
                           hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(win.data(), c->ctrl_win, win.size(), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    // 3. segments: up to and including each control packet, then its table write
    size_t start = 0, writes = 0;
    std::vector<uint8_t> full;
    for (uint64_t j = 0; j < cnt; ++j) {
        const size_t k = idx[j];
        if (upe_gpu_process(c, d_frames, d_desc + start, d_verdict + start, k + 1 - start,
                            stream) != 0)
            return -1;
        start = k + 1;
        const uint8_t* b = win.data() + j * kCtrlWin;
        const uint32_t len = lens[j];
        bool wrote = false;
        if (b[12] == 0x08 && b[13] == 0x06) {
            // ARP learn, src/worker.c:30-39: spa (network order) -> host order, sha
            if (arp_capacity) {
                const uint32_t spa = (uint32_t)b[28] << 24 | (uint32_t)b[29] << 16 |
                                     (uint32_t)b[30] << 8 | (uint32_t)b[31];
                host_arp_update(arp, arp_capacity, spa, b + 22, now);
                wrote = true;
            }
        } else {
            // NS / NA option walk, src/worker.c:64-95, over the whole frame when it is long.
            // This reads len bytes at the frame start: the call takes full frames only
            // (include/upe_gpu.h), never the UPE_FRAME_TAIL-byte header windows of the host path.
            const uint8_t* f = b;
            if (len > kCtrlWin) {
                uint64_t d = 0;
                HIP_TRY(hipMemcpy(&d, d_desc + k, sizeof d, hipMemcpyDeviceToHost));
                full.assign(len, 0);
                HIP_TRY(hipMemcpy(full.data(), d_frames + (d >> 16), len, hipMemcpyDeviceToHost));
                f = full.data();
            }
            const bool ns = f[54] == 135;
            for (size_t off = 78; off + 2 <= len;) {
                // uint8_t opt_len, as the reference's (src/worker.c:73): 32 wraps to 0, 33 to 8
                const uint32_t ot = f[off], ol = (uint8_t)(f[off + 1] * 8u);
                if (ol == 0 || off + ol > len) break;
                if (ol >= 8 && ((ns && ot == 1) || (!ns && ot == 2))) {
                    if (ndp_capacity) {
                        host_ndp_update(ndp, ndp_capacity, ns ? f + 22 : f + 62, f + off + 2, now);
                        wrote = true;
                    }
                    break;
                }
                off += ol;
            }
        }
        if (wrote) {
            ++writes;
            // the next segment reads the new snapshot (load_neigh waits for the context's
            // stream; a caller stream is drained first)
            if (s != c->stream) HIP_TRY(hipStreamSynchronize(s));
            if (upe_gpu_load_neigh(c, arp, arp_capacity, ndp, ndp_capacity) != 0) return -1;
        }
    }
    if (start < n &&
        upe_gpu_process(c, d_frames, d_desc + start, d_verdict + start, n - start, stream) != 0)
        return -1;
    HIP_TRY(hipStreamSynchronize(s));
    if (n_writes) *n_writes = writes;
    return 0;
}

// For the worker loop (upe_worker.c), not part of the ABI: a completion mark after everything
// queued so far on the context's stream, and a wait for it, so that the loop walks batch k - 1
// while batch k is on the GPU.
__attribute__((visibility("hidden"))) int upe_gpu_mark(upe_gpu_ctx_t* c, int slot) {
    if (!c || slot < 0 || slot >= 4) return fail("bad mark");
    DEV_SCOPE(c->device);
    if (!c->marks[slot]) HIP_TRY(hipEventCreateWithFlags(&c->marks[slot], hipEventDisableTiming));
    HIP_TRY(hipEventRecord(c->marks[slot], c->stream));
    return 0;
}
__attribute__((visibility("hidden"))) int upe_gpu_mark_wait(upe_gpu_ctx_t* c, int slot) {
    if (!c || slot < 0 || slot >= 4 || !c->marks[slot]) return fail("bad mark");
    DEV_SCOPE(c->device);
    HIP_TRY(hipEventSynchronize(c->marks[slot]));
    return 0;
}

int upe_gpu_sync(upe_gpu_ctx_t* c, void* stream) {
    if (!c) return fail("null context");
    DEV_SCOPE(c->device);
    HIP_TRY(hipStreamSynchronize(pick(c, stream)));
    return 0;
}

int upe_gpu_batch_info(upe_gpu_ctx_t* c, upe_batch_info_t* info) {
    if (!c || !info) return fail("null argument");
    DEV_SCOPE(c->device);
    HIP_TRY(hipDeviceSynchronize());
    memset(info, 0, sizeof *info);
    info->first_ctrl = ~0ull;
    if (!c->have_batch || c->k == 0) return 0;
    BatchAcc b;   // the last batch's accumulators
    HIP_TRY(hipMemcpy(&b, acc_slot(c, c->k + 2), sizeof b, hipMemcpyDeviceToHost));
    uint64_t* dst = &info->counters.pkts_in;
    dst[0] = b.n;
    uint32_t cm = 0;
    for (int r = 0; r < kReps; ++r) {
        for (int j = 0; j < 7; ++j) dst[1 + j] += b.cnt[r][j];
        info->n_ctrl += b.cnt[r][C_CTRL];
        cm = std::max(cm, b.ctrl[r]);
    }
    if (cm) info->first_ctrl = kNone - cm;
    return 0;
}

int upe_gpu_launch_info(upe_gpu_ctx_t* c, upe_launch_info_t* info) {
    if (!c || !info) return fail("null argument");
    DEV_SCOPE(c->device);
    HIP_TRY(hipDeviceSynchronize());
    memset(info, 0, sizeof *info);
    info->launches = c->k;
    if (c->k == 0 || c->last_var < 0) return 0;
    info->variant = (uint32_t)c->last_var;
    info->grid = c->last_grid;
    HIP_TRY(hipMemcpy(&info->deferred, &acc_slot(c, c->k + 2)->ndefer, sizeof(uint32_t),
                      hipMemcpyDeviceToHost));
    return 0;
}

int upe_gpu_get_stats(upe_gpu_ctx_t* c, upe_counters_t* counters, upe_rule_stat_t* rule_stats,
                      size_t capacity) {
    if (!c) return fail("null context");
    DEV_SCOPE(c->device);
    HIP_TRY(hipDeviceSynchronize());
    if (counters) {
        // the totals up to batch k - 2, plus batch k - 1 (folded in by the next launch)
        unsigned long long t[8];
        HIP_TRY(hipMemcpy(t, &c->st->totals[0], sizeof t, hipMemcpyDeviceToHost));
        uint64_t* dst = &counters->pkts_in;
        for (int j = 0; j < 8; ++j) dst[j] = t[j];
        if (c->k > 0) {
            BatchAcc b;
            HIP_TRY(hipMemcpy(&b, acc_slot(c, c->k + 2), sizeof b, hipMemcpyDeviceToHost));
            dst[0] += b.n;
            for (int r = 0; r < kReps; ++r)
                for (int j = 0; j < 7; ++j) dst[1 + j] += b.cnt[r][j];
        }
    }
    if (rule_stats && read_rule_stats(c, rule_stats, capacity) != 0) return -1;
    return 0;
}

int upe_gpu_reset_stats(upe_gpu_ctx_t* c) {
    if (!c) return fail("null context");
    DEV_SCOPE(c->device);
    if (order_on(c, c->stream) != 0) return -1;
    HIP_TRY(hipMemsetAsync(&c->st->totals[0], 0, sizeof(c->st->totals), c->stream));
    if (c->k > 0) {   // the last batch's counters, not yet folded into the totals
        BatchAcc* b = acc_slot(c, c->k + 2);
        HIP_TRY(hipMemsetAsync(&b->cnt[0][0], 0, sizeof(b->cnt), c->stream));
        HIP_TRY(hipMemsetAsync(&b->n, 0, sizeof(b->n), c->stream));
    }
    HIP_TRY(hipMemsetAsync(&c->st->acc_stats[0][0], 0, sizeof(c->st->acc_stats), c->stream));
    HIP_TRY(hipMemsetAsync(c->stats, 0, c->cap * 2 * sizeof(unsigned long long), c->stream));
    if (c->stats_idx)
        HIP_TRY(hipMemsetAsync(c->stats_idx, 0,
                               (size_t)c->rules_alloc * 2 * kStatReps * sizeof(unsigned long long),
                               c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->have_batch = false;
    return 0;
}

int upe_gpu_timing_span(upe_gpu_ctx_t* c, int every, int span) {
    if (!c) return fail("null context");
    if (span < 1) return fail("span must be at least 1");
    DEV_SCOPE(c->device);
    HIP_TRY(hipDeviceSynchronize());
    c->ev_used = 0;   // the pool is kept for reuse
    c->ev_mid.clear();
    c->timing = every > 0;
    c->timing_every = every > 0 ? (uint32_t)every : 1u;
    c->timing_phase = c->timing_every / 2;   // not the first call: it starts from an idle queue
    c->timing_span = (uint32_t)span;
    c->timing_calls = 0;
    c->t_left = 0;
    c->timing_launches = 0;
    return 0;
}

int upe_gpu_timing_enable(upe_gpu_ctx_t* c, int enable) {
    return upe_gpu_timing_span(c, enable, 1);
}

int upe_gpu_timing_read(upe_gpu_ctx_t* c, double* classify_ms, double* finalize_ms,
                        uint64_t* launches) {
    if (!c) return fail("null context");
    DEV_SCOPE(c->device);
    double a = 0, b = 0;
    for (size_t j = 0, k = 0; j + 3 <= c->ev_used; j += 3, ++k) {
        HIP_TRY(hipEventSynchronize(c->ev[j + 2]));
        float x = 0, y = 0;
        if (c->ev_mid[k]) {
            HIP_TRY(hipEventElapsedTime(&x, c->ev[j], c->ev[j + 1]));
            HIP_TRY(hipEventElapsedTime(&y, c->ev[j + 1], c->ev[j + 2]));
        } else {
            HIP_TRY(hipEventElapsedTime(&x, c->ev[j], c->ev[j + 2]));
        }
        a += x;
        b += y;
    }
    if (classify_ms) *classify_ms = a;
    if (finalize_ms) *finalize_ms = b;
    if (launches) *launches = c->timing_launches;
    return 0;
}

void* upe_gpu_malloc(upe_gpu_ctx_t* c, size_t bytes) {
    if (!c) {
        fail("null context");
        return nullptr;
    }
    void* p = nullptr;
    DevScope dg(c->device);
    if (dg.e != hipSuccess || hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) {
        fail("hipMalloc failed");
        return nullptr;
    }
    return p;
}

int upe_gpu_free(upe_gpu_ctx_t* c, void* p) {
    if (!c) return fail("null context");
    DEV_SCOPE(c->device);
    if (p) HIP_TRY(hipFree(p));
    return 0;
}

int upe_gpu_memcpy_h2d(upe_gpu_ctx_t* c, void* dst, const void* src, size_t bytes, void* stream) {
    if (!c) return fail("null context");
    DEV_SCOPE(c->device);
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, pick(c, stream)));
    return 0;
}

int upe_gpu_memcpy_d2h(upe_gpu_ctx_t* c, void* dst, const void* src, size_t bytes, void* stream) {
    if (!c) return fail("null context");
    DEV_SCOPE(c->device);
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, pick(c, stream)));
    return 0;
}

}  // extern "C"
