// upe_gpu.hip — MI355X (gfx950 / CDNA4) batch dataplane for UPE's per-packet worker hot path,
// and the extern "C" ABI declared in include/upe_gpu.h.
//
// One lane owns one packet.  Per packet the kernel does what reference process_packet() does
// (src/worker.c:106-253): control-packet classification (src/worker.c:23-104), the fixed-format
// parse (src/parser.c:6-111), first-match over the priority-sorted rule table
// (src/rule_table.c:76-91,163-176), counters and rule_stats (src/worker.c:119-153), and the
// L3-forward rewrite: TTL / hop-limit decrement, RFC 1071 checksum (src/parser.c:137-169), and the
// next-hop MAC that arp_get_mac / ndp_get_mac would return (src/arp_table.c:55-80,
// src/ndp_table.c:6-17,67-86).  Frames are rewritten in place in HBM.
//
// Data layout (DESIGN.md "HBM layout"): frames packed back to back at 16-byte aligned starts,
// one uint64 descriptor per packet (offset << 16 | len), one uint32 verdict per packet.  A lane
// reads at most the first UPE_HDR_WINDOW bytes of its frame as 16-byte vector loads (48 bytes for
// an option-less IPv4 header).  The rule table is compiled into structure-of-arrays streams that
// a wave scans with wave-uniform (scalar-unit) loads, so rule operands arrive in SGPRs; the
// per-rule work is a few VALU xor/and-or against them, with an early exit as soon as every lane
// of the wave has its first match (ballot).
//
// Two launches per batch.  classify runs one 256-packet tile per workgroup and keeps the tile's
// counters, rule_stats histogram (LDS) and L1 bookkeeping on chip, flushing them with device
// atomics into replicated per-batch accumulators (replica = tile % 32, so no address sees more
// than a few dozen adders).  finalize folds the accumulators into the worker totals and updates
// the L1 state.  The accumulators are double-buffered by batch parity, so finalize only reads.
//
// Neighbour lookups answer arp_get_mac / ndp_get_mac exactly without walking the reference's
// linear-probe chains: at upload the host keeps only the entries a reference probe can reach
// (probe from the home slot, first valid match before the first invalid slot) and re-hashes
// them into a half-empty multiplicative-hash table; every answer equals the reference's for the
// snapshot and a lookup costs ~1-2 probes.
//
// The worker's one-entry L1 neighbour caches are sequential state (src/worker.c:186-195,
// 218-225), emulated exactly.  If the starting L1 entry agrees with the
// table (the steady state), every packet's answer is the table's and the only sequential output
// is the final L1 entry: the last table hit, if any packet missed the starting entry and hit the
// table.  If it disagrees (after a table change, or the calloc'd NDP entry for ::), a packet
// whose destination equals the starting entry takes the entry's MAC iff no earlier packet missed
// the entry and hit the table: classify flags the tiles that hold such packets and finalize,
// which knows the batch's first miss-then-hit index, rewrites them after the kernel boundary.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <array>
#include <new>
#include <string>
#include <vector>

#include "../../include/upe_gpu.h"

namespace {

#ifndef UPE_BLOCK
#define UPE_BLOCK 256
#endif
constexpr int kBlock = UPE_BLOCK;      // threads per workgroup = packets per tile
constexpr int kWaves = kBlock / 64;
constexpr int kTile = kBlock;
#ifndef UPE_WAVES_PER_SIMD
#define UPE_WAVES_PER_SIMD 8
#endif
constexpr int kWavesPerSimd = UPE_WAVES_PER_SIMD;   // 8 -> VGPR budget 64
constexpr int kUnroll = 4;             // rules per early-exit check
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kLdsStatsMax = 4096;     // rule_stats histogrammed in LDS up to this many rules
constexpr int kSmallRules = 64;        // up to here rule_stats go through replicated accumulators
constexpr int kReps = 32;              // replicas of the per-batch accumulators
#ifndef UPE_ABLATE
#define UPE_ABLATE 0   // diagnostic builds only (make ablate); results are wrong when != 0
#endif
// 1 scan, 2 neighbour lookup, 4 stats/atomics, 8 stores, 16 empty finalize, 32 no finalize
// launch, 64 empty classify
constexpr unsigned kAblate = UPE_ABLATE;

// ---- compiled rule table (built by upe_gpu_load_rules) --------------------------------------
// rv4[i]: header + first address word, used for every packet:
//   x0 = ip_ver | proto << 8 | src_port << 16 and its wildcard mask m0
//   x1 = dst_port and mask m1
//   s0/sm0, d0/dm0: union bytes 0-3 of src/dst as LE u32 (the v4 view, rule_t.src_ip.v4),
//   pre-masked so a match is ((key ^ x) & m) == 0 for every pair.
// rv6[i]: union words 1-3 of src/dst (pre-masked) and masks, used only by IPv6 packets.
// rinfo[i]: (action.type, rule_id).
struct __attribute__((aligned(16))) RuleV4 {
    uint32_t x0, m0, x1, m1, s0, sm0, d0, dm0;
};
struct __attribute__((aligned(16))) RuleV6 {
    uint32_t s[3], sm[3], d[3], dm[3], pad[4];
};

// L1 state in word form (device resident between batches) + whether each entry agrees with the
// current neighbour snapshot (maintained by the last workgroup of every batch and by
// upe_refresh after every table / L1 upload).
struct DevL1 {
    uint32_t arp_ip, arp_mac_lo, arp_mac_hi;
    uint32_t ndp_ip[4];
    uint32_t ndp_mac_lo, ndp_mac_hi;
    uint32_t arp_ok, ndp_ok;
    uint32_t pad[5];
};

// Per-batch accumulators, double-buffered by batch parity: classify(e) adds into acc[e & 1] with
// device atomics and clears acc[(e + 1) & 1] for the next batch; finalize(e) only reads acc[e & 1],
// so any number of finalize workgroups can read it without a re-arm race.
enum { C_PARSED, C_MATCHED, C_FWD, C_DROPPED, C_CONSUMED, C_ARP_LEARN, C_ARP_REPLY, C_CTRL,
       C_CAND, C_N };   // C_CAND: tiles holding packets a disagreeing starting entry may answer
enum { M_F4, M_F6, M_CTRL, M_N };  // minima: first miss-then-hit per family, first control packet
enum { X_M4, X_M6, X_N };          // maxima: last table hit per family (index + 1, 0 = none)
struct BatchAcc {
    uint32_t cnt[kReps][C_N];
    uint32_t mins[kReps][M_N];
    uint32_t maxs[kReps][X_N];
    // the starting L1 entries' MACs and whether each disagreed with the table (copied by
    // classify, read by finalize, which itself rewrites the live L1 state)
    uint32_t start_arp_lo, start_arp_hi, start_ndp_lo, start_ndp_hi, look4, look6, pad[2];
};
// Payload of the last table hit of a 64-packet chunk (one wave's share of a tile), written by the
// lane that holds it; finalize reads the one chunk the batch maximum points at.
struct __attribute__((aligned(16))) ChunkPay {
    uint32_t m4_dst, m4_mac_lo, m4_mac_hi, pad0;
    uint32_t m6_dst[4];
    uint32_t m6_mac_lo, m6_mac_hi, pad1[2];
};

// Accumulated worker state (device resident).
struct DevTotals {
    unsigned long long cnt[8];     // upe_counters_t order
    unsigned long long n_ctrl, first_ctrl;
    unsigned long long batch[8];
    unsigned long long error;
};

struct NeighIndex {
    const uint4* t;
    uint32_t bits;   // log2(slots); 0 = empty
    uint32_t seed;
};

struct Args {
    uint8_t* frames;
    const uint64_t* desc;
    uint32_t* verdict;
    uint32_t n;
    uint32_t ntiles;
    uint32_t parity;               // batch sequence number & 1
    const RuleV4* rv4;
    const RuleV6* rv6;
    const int2* rinfo;
    uint32_t nrules_pad;           // multiple of kUnroll, padding rules never match
    NeighIndex arp, ndp;           // reachable-entry indexes (two-choice cuckoo)
    DevL1* l1;
    BatchAcc* acc;                 // [2]
    ChunkPay* pay;                 // [ntiles * kWaves]
    uint32_t* cand_tile;           // [ntiles] families with packets the starting entry may answer
    unsigned long long* acc_stats; // [2][kReps][nrules_pad][2] when nrules_pad <= kSmallRules
    unsigned long long* stats;     // [cap][2] worker totals (rule_stat_t), large tables
    unsigned long long* stats_idx; // [nrules_pad][2] totals per sorted index, small tables
    DevTotals* totals;
    uint32_t port_mac_lo, port_mac_hi, port_ip4;
};

// ---- small helpers ------------------------------------------------------------------------
__device__ __forceinline__ uint32_t byte_of(uint32_t w, int k) { return (w >> (8 * k)) & 0xFFu; }
__device__ __forceinline__ uint32_t at2(uint32_t hi, uint32_t lo) {   // dword at byte 4q+2
    return __builtin_amdgcn_alignbit(hi, lo, 16);
}
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
// Mask of the bytes of dword j that lie below len (a zero-filled pktbuf reads 0 past len).
__device__ __forceinline__ uint32_t len_mask(uint32_t len, int j) {
    const uint32_t lo = 4u * (uint32_t)j;
    return len >= lo + 4 ? 0xFFFFFFFFu : len <= lo ? 0u : (1u << (8 * (len - lo))) - 1u;
}
__device__ __forceinline__ uint32_t be16_lo(uint32_t x) {             // BE u16 in bytes 0,1
    return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu);
}
// Neighbour index (built by upe_gpu_load_neigh): the entries a reference probe reaches, placed
// by two-choice cuckoo hashing, so that every key sits in one of its two candidate slots.  A
// lookup loads both slots at once: one memory round trip for every packet, no probe loop (a
// linear-probe walk costs the longest chain of the wave, one dependent load per step).
//   ARP slot: uint4 {ip, mac0..3, mac4..5 | used << 16, 0}
//   NDP slot: 2 x uint4 {ip words 0..3}, {mac0..3, mac4..5 | used << 16, 0, 0}
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
__device__ __forceinline__ bool arp_lookup(const NeighIndex& x, uint32_t ip, uint32_t& lo,
                                           uint32_t& hi) {
    if (x.bits == 0) return false;
    const uint4 e1 = x.t[slot1(ip, x.seed, x.bits)];
    const uint4 e2 = x.t[slot2(ip, x.seed, x.bits)];
    const bool h1 = ((e1.z >> 16) & 1u) && e1.x == ip;
    const bool h2 = ((e2.z >> 16) & 1u) && e2.x == ip;
    lo = h1 ? e1.y : e2.y;
    hi = (h1 ? e1.z : e2.z) & 0xFFFFu;
    return h1 || h2;
}
__device__ __forceinline__ bool ndp_lookup(const NeighIndex& x, const uint32_t ip[4], uint32_t& lo,
                                           uint32_t& hi) {
    if (x.bits == 0) return false;
    const uint32_t k = fold_v6(ip);
    const uint32_t t1 = slot1(k, x.seed, x.bits), t2 = slot2(k, x.seed, x.bits);
    const uint4 a1 = x.t[2 * t1], m1 = x.t[2 * t1 + 1];
    const uint4 a2 = x.t[2 * t2], m2 = x.t[2 * t2 + 1];
    const bool h1 = ((m1.y >> 16) & 1u) && a1.x == ip[0] && a1.y == ip[1] && a1.z == ip[2] &&
                    a1.w == ip[3];
    const bool h2 = ((m2.y >> 16) & 1u) && a2.x == ip[0] && a2.y == ip[1] && a2.z == ip[2] &&
                    a2.w == ip[3];
    lo = h1 ? m1.x : m2.x;
    hi = (h1 ? m1.y : m2.y) & 0xFFFFu;
    return h1 || h2;
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

// First-match scan (reference src/rule_table.c:163-176 over match_rule :76-91).  Every lane of
// the wave walks the same rules in sorted order; rule words are wave-uniform loads.  `done`
// lanes (already matched, or not scanning) are ignored.  V6 = some lane holds an IPv6 key.
template <bool V6>
__device__ __forceinline__ uint32_t scan_rules(const Args& a, bool done, bool is6, uint32_t k0,
                                               uint32_t k1, const uint32_t s[4],
                                               const uint32_t d[4]) {
    uint32_t hit = kNone;
    const uint32_t m6 = is6 ? 0xFFFFFFFFu : 0u;
    for (uint32_t base = 0; base < a.nrules_pad; base += kUnroll) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const RuleV4 r = a.rv4[base + u];
            uint32_t x = ((k0 ^ r.x0) & r.m0) | ((k1 ^ r.x1) & r.m1) | ((s[0] ^ r.s0) & r.sm0) |
                         ((d[0] ^ r.d0) & r.dm0);
            if (V6) {
                const RuleV6 q = a.rv6[base + u];
                uint32_t y = ((s[1] ^ q.s[0]) & q.sm[0]) | ((s[2] ^ q.s[1]) & q.sm[1]) |
                             ((s[3] ^ q.s[2]) & q.sm[2]) | ((d[1] ^ q.d[0]) & q.dm[0]) |
                             ((d[2] ^ q.d[1]) & q.dm[1]) | ((d[3] ^ q.d[2]) & q.dm[2]);
                x |= y & m6;
            }
            if (!done && x == 0) {
                hit = base + u;
                done = true;
            }
        }
        if (__all(done)) break;
    }
    return hit;
}

// ------------------------------------------------------------------------------------------
// classify: one 256-packet tile per workgroup
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock, kWavesPerSimd) upe_classify(Args a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_hist[]; // [nrules_pad][2]
    __shared__ uint32_t s_cnt[C_N];
    __shared__ uint32_t s_red[kWaves][8];

    if (kAblate & 64) return;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const uint32_t tile = blockIdx.x;
    const uint32_t rep = tile % kReps;
    const bool lds_stats = a.nrules_pad <= (uint32_t)kLdsStatsMax;
    const bool small_stats = a.nrules_pad <= (uint32_t)kSmallRules;
    BatchAcc* A = &a.acc[a.parity];

    if (lds_stats)
        for (uint32_t r = tid; r < 2 * a.nrules_pad; r += kBlock) lds_hist[r] = 0;
    if (tid < C_N) s_cnt[tid] = 0;

    // L1 state at batch start (uniform).
    const DevL1* l1 = a.l1;
    const uint32_t l1_arp_ip = l1->arp_ip;
    uint32_t l1_ndp[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) l1_ndp[j] = l1->ndp_ip[j];
    const bool look4 = !l1->arp_ok;
    const bool look6 = !l1->ndp_ok;

    if (tile == 0) {
        // clear the other parity's accumulators for the next batch; record the starting
        // entries for this batch's finalize
        BatchAcc* N = &a.acc[a.parity ^ 1];
        uint32_t* nw = reinterpret_cast<uint32_t*>(N);
        for (uint32_t k = tid; k < sizeof(BatchAcc) / 4; k += kBlock) {
            const uint32_t off = k * 4;
            const bool is_min = off >= offsetof(BatchAcc, mins) && off < offsetof(BatchAcc, maxs);
            nw[k] = is_min ? kNone : 0u;
        }
        if (small_stats) {
            unsigned long long* ns = a.acc_stats + (size_t)(a.parity ^ 1) * kReps * 2 * a.nrules_pad;
            for (uint32_t k = tid; k < kReps * 2 * a.nrules_pad; k += kBlock) ns[k] = 0;
        }
        if (tid == 0) {
            A->start_arp_lo = l1->arp_mac_lo;
            A->start_arp_hi = l1->arp_mac_hi;
            A->start_ndp_lo = l1->ndp_mac_lo;
            A->start_ndp_hi = l1->ndp_mac_hi;
            A->look4 = look4;
            A->look6 = look6;
        }
    }
    __syncthreads();

    {
        const uint32_t i = tile * kTile + (uint32_t)tid;
        const bool live = i < a.n;
        const uint64_t dsc = live ? a.desc[i] : 0;
        const uint32_t len = (uint32_t)(dsc & 0xFFFFu);
        uint8_t* p = a.frames + (dsc >> 16);

        // ---- header window: chunks 0-2 (bytes 0..47) for every live lane ----
        uint32_t w[24];
#pragma unroll
        for (int j = 0; j < 24; ++j) w[j] = 0;
        if (live) {
            const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const uint4 v = q[c];
                w[4 * c + 0] = v.x; w[4 * c + 1] = v.y; w[4 * c + 2] = v.z; w[4 * c + 3] = v.w;
            }
        }
        // Bytes 12/13 as a zero-filled pktbuf would hold them (the ethertype is read before
        // any length gate, src/worker.c:24-25).
        const uint32_t b12 = len > 12 ? byte_of(w[3], 0) : 0u;
        const uint32_t b13 = len > 13 ? byte_of(w[3], 1) : 0u;
        const uint32_t et = (b12 << 8) | b13;
        const bool is_v4 = et == 0x0800u;
        const bool is_v6 = et == 0x86DDu;
        const uint32_t ihl = byte_of(w[3], 2) & 0xFu;
        // chunks 3-5 only for IPv6 and IPv4 with options
        if (live && (is_v6 || (is_v4 && ihl > 5))) {
            const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
            for (int c = 3; c < 6; ++c) {
                const uint4 v = q[c];
                w[4 * c + 0] = v.x; w[4 * c + 1] = v.y; w[4 * c + 2] = v.z; w[4 * c + 3] = v.w;
            }
        }

        uint32_t flags = 0;
        bool consumed = false;
        bool wrote0 = false;  // chunk 0 (bytes 0..15) modified
        bool wrote1 = false;  // chunk 1

        // ---- handle_control_packet, reference src/worker.c:23-104 ----
        if (live && et == 0x0806u) {
            // The ARP header (bytes 14..41) is read without a length check: bytes at or past
            // len read as zero, as in a zero-filled pktbuf.
            uint32_t z[12];
#pragma unroll
            for (int j = 0; j < 12; ++j) z[j] = w[j] & len_mask(len, j);
            const bool wellformed = (z[3] >> 16) == 0x0100u && z[4] == 0x04060008u;
            if (wellformed) {
                flags |= UPE_VF_ARP_LEARN;
                const bool request = (z[5] & 0xFFFFu) == 0x0100u;
                const uint32_t tpa = bswap32(at2(z[10], z[9]));
                if (request && a.port_ip4 != 0 && tpa == a.port_ip4) {
                    // In-place reply, src/worker.c:42-51, assembled a dword at a time.
                    uint32_t nw[12];
                    nw[0] = at2(z[2], z[1]);                                  // eth.dst = eth.src
                    nw[1] = (z[2] >> 16) | (a.port_mac_lo << 16);             // eth.src = port MAC
                    nw[2] = (a.port_mac_lo >> 16) | (a.port_mac_hi << 16);
                    nw[3] = z[3];
                    nw[4] = z[4];
                    nw[5] = 0x0200u | (a.port_mac_lo << 16);                  // op = REPLY, sha
                    nw[6] = (a.port_mac_lo >> 16) | (a.port_mac_hi << 16);
                    nw[7] = bswap32(a.port_ip4);                              // spa = port IPv4
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
                    if (!(kAblate & 8)) {
                        uint4* q = reinterpret_cast<uint4*>(p);
                        q[0] = make_uint4(w[0], w[1], w[2], w[3]);
                        q[1] = make_uint4(w[4], w[5], w[6], w[7]);
                        q[2] = make_uint4(w[8], w[9], w[10], w[11]);
                    }
                    flags |= UPE_VF_ARP_REPLY;
                }
            }
        }
        if (live && is_v6 && len >= 78u && byte_of(w[5], 0) == 58u) {   // src/worker.c:58-100
            const uint32_t type = byte_of(w[13], 2);                     // byte 54
            if (type == 135u || type == 136u) consumed = true;
        }
        const bool ctrl = live && (consumed || (flags & UPE_VF_ARP_LEARN));

        // ---- parse_flow_key, reference src/parser.c:6-111 ----
        bool ok = false;
        uint32_t proto = 0, sport = 0, dport = 0;
        uint32_t s[4] = {0, 0, 0, 0}, d[4] = {0, 0, 0, 0};
        if (live && !consumed && len >= 14u) {
            if (is_v4) {
                const uint32_t ver = byte_of(w[3], 2) >> 4;
                const uint32_t hl = ihl * 4;
                if (len - 14 >= 20u && ver == 4 && hl >= 20 && len - 14 >= hl) {
                    proto = byte_of(w[5], 3);                                // byte 23
                    s[0] = bswap32(at2(w[7], w[6]));                         // bytes 26..29
                    d[0] = bswap32(at2(w[8], w[7]));                         // bytes 30..33
                    const uint32_t l4len = len - 14 - hl;
                    uint32_t l4w0, l4w1, l4w3;
                    if (ihl == 5) {
                        l4w0 = at2(w[9], w[8]);    // L4 bytes 0..3  (byte 34)
                        l4w1 = at2(w[10], w[9]);   // L4 bytes 4..7
                        l4w3 = at2(w[12], w[11]);  // L4 bytes 12..15
                    } else {
                        l4w0 = l4w1 = l4w3 = 0;
#pragma unroll
                        for (int h = 6; h <= 15; ++h) {
                            if ((int)ihl == h) {
                                l4w0 = at2(w[h + 4], w[h + 3]);
                                l4w1 = at2(w[h + 5], w[h + 4]);
                                l4w3 = at2(w[h + 7], w[h + 6]);
                            }
                        }
                    }
                    if (proto == 17u) {
                        ok = l4len >= 8u;
                        sport = be16_lo(l4w0);
                        dport = be16_lo(l4w0 >> 16);
                    } else if (proto == 6u) {
                        const uint32_t thl = (byte_of(l4w3, 0) >> 4) * 4;
                        ok = l4len >= 20u && thl >= 20u && l4len >= thl;
                        sport = be16_lo(l4w0);
                        dport = be16_lo(l4w0 >> 16);
                    } else if (proto == 1u) {
                        ok = l4len >= 8u;
                        sport = be16_lo(l4w1);                               // icmp id
                        dport = (byte_of(l4w0, 0) << 8) | byte_of(l4w0, 1);  // type << 8 | code
                    }
                }
            } else if (is_v6) {
                if (len - 14 >= 40u) {
                    proto = byte_of(w[5], 0);                                // byte 20
                    s[0] = at2(w[6], w[5]);  s[1] = at2(w[7], w[6]);
                    s[2] = at2(w[8], w[7]);  s[3] = at2(w[9], w[8]);
                    d[0] = at2(w[10], w[9]); d[1] = at2(w[11], w[10]);
                    d[2] = at2(w[12], w[11]); d[3] = at2(w[13], w[12]);
                    const uint32_t l4len = len - 54;
                    const uint32_t l4w0 = at2(w[14], w[13]);                 // byte 54
                    const uint32_t l4w1 = at2(w[15], w[14]);
                    const uint32_t l4w3 = at2(w[17], w[16]);                 // byte 66
                    if (proto == 17u) {
                        ok = l4len >= 8u;
                        sport = be16_lo(l4w0);
                        dport = be16_lo(l4w0 >> 16);
                    } else if (proto == 6u) {
                        const uint32_t thl = (byte_of(l4w3, 0) >> 4) * 4;
                        ok = l4len >= 20u && thl >= 20u && l4len >= thl;
                        sport = be16_lo(l4w0);
                        dport = be16_lo(l4w0 >> 16);
                    } else if (proto == 1u) {
                        ok = l4len >= 8u;
                        sport = be16_lo(l4w1);
                        dport = (byte_of(l4w0, 0) << 8) | byte_of(l4w0, 1);
                    }
                }
            }
        }

        // ---- the forward rewrite of bytes 16..31, computed now so that the header dwords are
        // dead before the rule scan: IPv4 ttl-- and checksum over IHL*4 bytes
        // (src/worker.c:174-176, src/parser.c:137-169, stored LE), IPv6 hop-- (src/worker.c:213)
        const uint32_t ttl = is_v6 ? byte_of(w[5], 1) : byte_of(w[5], 2);   // byte 21 / 22
        uint32_t c1w1 = w[5], c1w2 = w[6];
        if (ok && !is_v6 && ttl > 1u) {
            const uint32_t hw2 = (ttl - 1) | (byte_of(w[5], 3) << 8);       // bytes 22..25
            unsigned long long sum = 0;
#pragma unroll
            for (int j = 0; j < 15; ++j) {
                const uint32_t dw = j == 2 ? hw2 : at2(w[4 + j], w[3 + j]);
                if ((uint32_t)j < ihl) sum += dw;
            }
            uint32_t f = (uint32_t)(sum & 0xFFFFFFFFull) + (uint32_t)(sum >> 32);
            f += (uint32_t)(sum & 0xFFFFFFFFull) > f ? 1u : 0u;            // end-around carry
            f = (f & 0xFFFFu) + (f >> 16);
            f = (f & 0xFFFFu) + (f >> 16);
            f = (f & 0xFFFFu) + (f >> 16);
            const uint32_t cs = (~f) & 0xFFFFu;
            // bytes 22..25 live in w[5] bytes 2,3 and w[6] bytes 0,1
            c1w1 = (w[5] & 0x0000FFFFu) | ((ttl - 1) << 16) | (byte_of(w[5], 3) << 24);
            c1w2 = (w[6] & 0xFFFF0000u) | cs;
        } else if (ok && is_v6 && ttl > 1u) {
            c1w1 = (w[5] & 0xFFFF00FFu) | ((ttl - 1) << 8);
        }

        // ---- rule_table_match ----
        const uint32_t ver = is_v6 ? 6u : 4u;
        const uint32_t k0 = ver | (proto << 8) | (sport << 16);
        const uint32_t k1 = dport;
        const bool need_v6 = __any(ok && is_v6);
        const uint32_t ri = (kAblate & 1) ? (ok ? 0u : kNone)
                            : need_v6 ? scan_rules<true>(a, !ok, is_v6, k0, k1, s, d)
                                      : scan_rules<false>(a, !ok, is_v6, k0, k1, s, d);

        // ---- verdict, counters, rule_stats (src/worker.c:117-153) ----
        uint32_t code = 0;
        uint32_t rbits = 0;
        if (!live) {
            code = 0;
        } else if (consumed) {
            code = UPE_V_CONSUMED;
        } else if (!ok) {
            code = UPE_V_DROP_PARSE;
        } else if (ri == kNone) {
            code = UPE_V_DROP_NOMATCH;
        } else {
            const int2 info = a.rinfo[ri];
            rbits = (ri + 1) << 8;
            // rule_stats[rule_id] += {1, len}, src/worker.c:141-144: aggregated per wave below
            // for LDS-resident tables, direct device atomics for very large ones
            if (!(kAblate & 4) && !lds_stats) {
                atomicAdd(&a.stats[2 * (uint32_t)info.y], 1ull);
                atomicAdd(&a.stats[2 * (uint32_t)info.y + 1], (unsigned long long)len);
            }
            code = info.x == UPE_ACT_DROP ? UPE_V_DROP_RULE
                 : info.x == UPE_ACT_FWD  ? UPE_V_FWD
                                          : UPE_V_DROP_ACTION;
        }

        // ---- L3 forward (src/worker.c:155-244) ----
        bool fp4 = false, fp6 = false;       // this packet misses the start entry, hits table
        bool thit4 = false, thit6 = false;   // the table answered this packet
        bool hit = false;      // the packet gets a MAC: the table's (or the starting entry's)
        bool cand = false;     // destination == starting L1 entry (ARP: and != 0)
        uint32_t mlo = 0, mhi = 0;
        if (code == UPE_V_FWD) {
            if (ttl <= 1u) {                           // src/worker.c:165-172, 204-211
                code = UPE_V_DROP_TTL;
            } else if (!is_v6) {
                w[5] = c1w1;
                w[6] = c1w2;
                wrote1 = true;
                hit = !(kAblate & 2) && arp_lookup(a.arp, d[0], mlo, mhi);
                cand = l1_arp_ip != 0 && d[0] == l1_arp_ip;
                fp4 = !cand && hit;
                thit4 = hit;
            } else {
                w[5] = c1w1;
                wrote1 = true;
                hit = !(kAblate & 2) && ndp_lookup(a.ndp, d, mlo, mhi);
                cand = d[0] == l1_ndp[0] && d[1] == l1_ndp[1] && d[2] == l1_ndp[2] &&
                       d[3] == l1_ndp[3];
                fp6 = !cand && hit;
                thit6 = hit;
            }
            if (cand) flags |= UPE_VF_L1_INIT;
        }


        if (hit) {
            w[0] = mlo;
            w[1] = mhi | (a.port_mac_lo << 16);
            w[2] = (a.port_mac_lo >> 16) | (a.port_mac_hi << 16);
            wrote0 = true;
            flags |= UPE_VF_NEIGH_HIT;
        }

        // ---- write back ----
        if (live) {
            uint4* q = reinterpret_cast<uint4*>(p);
            if (kAblate & 8) wrote0 = wrote1 = false;
            if (wrote0) q[0] = make_uint4(w[0], w[1], w[2], w[3]);
            if (wrote1) q[1] = make_uint4(w[4], w[5], w[6], w[7]);
            a.verdict[i] = code | flags | rbits;
        }

        // ---- rule_stats: LDS histogram (same-address lanes serialise in the LDS atomic unit,
        // cheaper than a cross-lane reduction per distinct rule) ----
        if (lds_stats && !(kAblate & 4) && live && !consumed && ok && ri != kNone) {
            atomicAdd(&lds_hist[2 * ri], 1u);
            atomicAdd(&lds_hist[2 * ri + 1], len);
        }

        // ---- per-wave totals and L1 bookkeeping ----
        const uint32_t wc[C_N] = {
            (uint32_t)__popcll(__ballot(live && !consumed && ok)),
            (uint32_t)__popcll(__ballot(live && !consumed && ok && ri != kNone)),
            (uint32_t)__popcll(__ballot(live && code == UPE_V_FWD)),
            (uint32_t)__popcll(__ballot(live && code != UPE_V_FWD && code != UPE_V_CONSUMED)),
            (uint32_t)__popcll(__ballot(live && consumed)),
            (uint32_t)__popcll(__ballot(live && !consumed && (flags & UPE_VF_ARP_LEARN))),
            (uint32_t)__popcll(__ballot(live && !consumed && (flags & UPE_VF_ARP_REPLY))),
            (uint32_t)__popcll(__ballot(ctrl)), 0u};
#pragma unroll
        for (int c = 0; c < C_N; ++c)
            if (lane == 0 && wc[c]) atomicAdd(&s_cnt[c], wc[c]);
        // lane order is packet order, so first / last qualifying packets are ballot bit scans
        const uint32_t i0 = i - (uint32_t)lane;
        const unsigned long long bf4 = __ballot(fp4), bf6 = __ballot(fp6), bfc = __ballot(ctrl);
        const unsigned long long bm4 = __ballot(thit4), bm6 = __ballot(thit6);
        const uint32_t f4 = bf4 ? i0 + (uint32_t)__ffsll((long long)bf4) - 1 : kNone;
        const uint32_t f6 = bf6 ? i0 + (uint32_t)__ffsll((long long)bf6) - 1 : kNone;
        const uint32_t fc = bfc ? i0 + (uint32_t)__ffsll((long long)bfc) - 1 : kNone;
        const uint32_t m4 = bm4 ? i0 + 64u - (uint32_t)__clzll((long long)bm4) : 0u;   // index + 1
        const uint32_t m6 = bm6 ? i0 + 64u - (uint32_t)__clzll((long long)bm6) : 0u;
        // packets the starting entry answers if nothing before them missed it and hit the table
        const uint32_t cbits = (__ballot(cand && !is_v6 && look4) ? 1u : 0u) |
                               (__ballot(cand && is_v6 && look6) ? 2u : 0u);
        if (m4 && i + 1 == m4) {
            ChunkPay* P = &a.pay[i / 64];
            P->m4_dst = d[0]; P->m4_mac_lo = mlo; P->m4_mac_hi = mhi;
        }
        if (m6 && i + 1 == m6) {
            ChunkPay* P = &a.pay[i / 64];
            P->m6_dst[0] = d[0]; P->m6_dst[1] = d[1]; P->m6_dst[2] = d[2]; P->m6_dst[3] = d[3];
            P->m6_mac_lo = mlo; P->m6_mac_hi = mhi;
        }
        if (lane == 0) {
            s_red[wave][0] = f4; s_red[wave][1] = f6; s_red[wave][2] = m4;
            s_red[wave][3] = m6; s_red[wave][4] = fc; s_red[wave][5] = cbits;
        }
    }
    __syncthreads();

    // ---- workgroup flush into the replicated accumulators ----
    // Device atomics are priced per wave-instruction (~50 ns per CU, whatever the lane count),
    // so every accumulator kind goes out as ONE instruction, lane k carrying field k.
    if (wave == 0 && !(kAblate & 4)) {
        uint32_t cb = 0;
#pragma unroll
        for (int v = 0; v < kWaves; ++v) cb |= s_red[v][5];
        const bool flag = (look4 || look6) && cb;
        if (lane < C_N) {
            const uint32_t cv = lane == C_CAND ? (flag ? 1u : 0u) : s_cnt[lane];
            if (cv) atomicAdd(&A->cnt[rep][lane], cv);
        }
        if (lane < M_N) {
            const int src = lane == M_F4 ? 0 : lane == M_F6 ? 1 : 4;
            uint32_t mv = kNone;
#pragma unroll
            for (int v = 0; v < kWaves; ++v) mv = min(mv, s_red[v][src]);
            if (mv != kNone) atomicMin(&A->mins[rep][lane], mv);
        }
        if (lane < X_N) {
            const int src = lane == X_M4 ? 2 : 3;
            uint32_t xv = 0;
#pragma unroll
            for (int v = 0; v < kWaves; ++v) xv = max(xv, s_red[v][src]);
            if (xv) atomicMax(&A->maxs[rep][lane], xv);
        }
        if (lane == 0 && (look4 || look6)) a.cand_tile[tile] = cb;
    }
    if (lds_stats && !(kAblate & 4)) {
        if (small_stats) {
            unsigned long long* out =
                a.acc_stats + ((size_t)a.parity * kReps + rep) * 2 * a.nrules_pad;
            for (uint32_t r = tid; r < 2 * a.nrules_pad; r += kBlock) {
                const uint32_t v = lds_hist[r];
                if (v) atomicAdd(&out[r], (unsigned long long)v);
            }
        } else {
            for (uint32_t r = tid; r < 2 * a.nrules_pad; r += kBlock) {
                const uint32_t v = lds_hist[r];
                if (v)
                    atomicAdd(&a.stats[2 * (uint32_t)a.rinfo[r >> 1].y + (r & 1)],
                              (unsigned long long)v);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// finalize: fold the batch's accumulators (workgroup 0) and give the starting L1 entry's answer
// to the packets it answered in the reference (every workgroup, over flagged tiles).
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) upe_finalize(Args a) {
    if (kAblate & 16) return;
    // Every global load below is issued in one round before anything waits on it; the running
    // totals are no-return atomics, so the only dependent round is the L1 payload (and the rare
    // candidate repair).
    const int tid = threadIdx.x;
    const BatchAcc* A = &a.acc[a.parity];
    const bool blk0 = blockIdx.x == 0;
    const bool small = blk0 && a.nrules_pad <= (uint32_t)kSmallRules;
    const uint32_t E = 2 * a.nrules_pad;
    __shared__ uint32_t s_min[M_N], s_max[X_N];
    __shared__ unsigned long long s_cnt[C_N];
    __shared__ unsigned long long s_st[2 * kSmallRules];

    uint32_t mn[M_N], mx[X_N], c[C_N];
    if (tid < kReps) {
#pragma unroll
        for (int j = 0; j < M_N; ++j) mn[j] = A->mins[tid][j];
#pragma unroll
        for (int j = 0; j < X_N; ++j) mx[j] = A->maxs[tid][j];
#pragma unroll
        for (int j = 0; j < C_N; ++j) c[j] = A->cnt[tid][j];
    }
    // small tables: replica r of entry e at acc_stats[parity][r][e]; thread t owns entries
    // (t + k * kBlock) of the flattened [kReps][E] array
    constexpr int kStatLoads = kReps * 2 * kSmallRules / kBlock;
    unsigned long long sv[kStatLoads];
    const unsigned long long* src = a.acc_stats + (size_t)a.parity * kReps * E;
#pragma unroll
    for (int k = 0; k < kStatLoads; ++k) {
        const uint32_t f = (uint32_t)tid + (uint32_t)k * kBlock;
        sv[k] = small && f < E * kReps ? src[f] : 0ull;
    }
    const uint32_t look = (A->look4 ? 1u : 0u) | (A->look6 ? 2u : 0u);

    if (tid < M_N) s_min[tid] = kNone;
    if (tid < X_N) s_max[tid] = 0;
    if (tid < C_N) s_cnt[tid] = 0;
    if ((uint32_t)tid < 2 * kSmallRules) s_st[tid] = 0;
    __syncthreads();
    if (tid < kReps) {
#pragma unroll
        for (int j = 0; j < M_N; ++j) atomicMin(&s_min[j], mn[j]);
#pragma unroll
        for (int j = 0; j < X_N; ++j) atomicMax(&s_max[j], mx[j]);
#pragma unroll
        for (int j = 0; j < C_N; ++j)
            if (c[j]) atomicAdd(&s_cnt[j], (unsigned long long)c[j]);
    }
#pragma unroll
    for (int k = 0; k < kStatLoads; ++k)
        if (sv[k]) atomicAdd(&s_st[((uint32_t)tid + (uint32_t)k * kBlock) % E], sv[k]);
    __syncthreads();

    // Packets whose destination is the starting entry, before the first miss-then-hit packet of
    // their family, took the entry's MAC (found) in the reference: src/worker.c:186-188, 218-220.
    if (look && s_cnt[C_CAND] != 0) {
        const uint32_t f[2] = {s_min[M_F4], s_min[M_F6]};
        const uint32_t lo[2] = {A->start_arp_lo, A->start_ndp_lo};
        const uint32_t hi[2] = {A->start_arp_hi, A->start_ndp_hi};
        __shared__ uint32_t s_list[kBlock];
        __shared__ uint32_t s_nl;
        for (uint32_t base = blockIdx.x * kBlock; base < a.ntiles; base += gridDim.x * kBlock) {
            if (tid == 0) s_nl = 0;
            __syncthreads();
            const uint32_t t = base + (uint32_t)tid;
            const uint32_t cb = t < a.ntiles ? a.cand_tile[t] : 0u;   // flags read in parallel
            if (cb) s_list[atomicAdd(&s_nl, 1u)] = t;
            __syncthreads();
            for (uint32_t k = 0; k < s_nl; ++k) {
                const uint32_t tt = s_list[k];
                const uint32_t i = tt * kTile + (uint32_t)tid;
                if (i >= a.n) continue;
                const uint32_t v = a.verdict[i];
                if ((v & 0xFu) != UPE_V_FWD || !(v & UPE_VF_L1_INIT)) continue;
                uint8_t* p = a.frames + (a.desc[i] >> 16);
                const int fam = (p[12] == 0x86 && p[13] == 0xDD) ? 1 : 0;
                if (!((a.cand_tile[tt] >> fam) & 1u) || i >= f[fam]) continue;
                uint32_t* q = reinterpret_cast<uint32_t*>(p);
                q[0] = lo[fam];
                q[1] = hi[fam] | (a.port_mac_lo << 16);
                q[2] = (a.port_mac_lo >> 16) | (a.port_mac_hi << 16);
                a.verdict[i] = v | UPE_VF_NEIGH_HIT;
            }
            __syncthreads();
        }
    }
    if (!blk0) return;

    // rule_stats of small tables, in sorted-index space (the host maps index -> rule_id)
    if (small && (uint32_t)tid < E && s_st[tid]) atomicAdd(&a.stats_idx[tid], s_st[tid]);
    DevTotals* T = a.totals;
    if (tid < 8) {
        const unsigned long long b =
            tid == 0 ? (unsigned long long)a.n : s_cnt[tid == 1 ? C_PARSED : tid == 2 ? C_MATCHED
                                                     : tid == 3 ? C_FWD : tid == 4 ? C_DROPPED
                                                     : tid == 5 ? C_CONSUMED : tid == 6 ? C_ARP_LEARN
                                                                                : C_ARP_REPLY];
        if (b) atomicAdd(&T->cnt[tid], b);
        T->batch[tid] = b;
    }
    if (tid == 8) T->n_ctrl = s_cnt[C_CTRL];
    if (tid == 9)
        T->first_ctrl = s_min[M_CTRL] == kNone ? ~0ull : (unsigned long long)s_min[M_CTRL];
    // New L1 state: the last table hit, if some packet missed the starting entry and hit the
    // table (from then on the cache only ever holds table answers, so it agrees with the
    // table); otherwise unchanged.
    DevL1* L = a.l1;
    if (tid == 16 && s_min[M_F4] != kNone && s_max[X_M4] != 0) {
        const ChunkPay* P = &a.pay[(s_max[X_M4] - 1) / 64];
        const uint32_t ip = P->m4_dst, lo = P->m4_mac_lo, hi = P->m4_mac_hi;
        L->arp_ip = ip;
        L->arp_mac_lo = lo;
        L->arp_mac_hi = hi;
        L->arp_ok = 1;
    }
    if (tid == 17 && s_min[M_F6] != kNone && s_max[X_M6] != 0) {
        const ChunkPay* P = &a.pay[(s_max[X_M6] - 1) / 64];
        uint32_t ip[4];
        for (int j = 0; j < 4; ++j) ip[j] = P->m6_dst[j];
        const uint32_t lo = P->m6_mac_lo, hi = P->m6_mac_hi;
        for (int j = 0; j < 4; ++j) L->ndp_ip[j] = ip[j];
        L->ndp_mac_lo = lo;
        L->ndp_mac_hi = hi;
        L->ndp_ok = 1;
    }
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

uint32_t mac_lo(const uint8_t* m) {
    return (uint32_t)m[0] | ((uint32_t)m[1] << 8) | ((uint32_t)m[2] << 16) | ((uint32_t)m[3] << 24);
}
uint32_t mac_hi(const uint8_t* m) { return (uint32_t)m[4] | ((uint32_t)m[5] << 8); }
uint32_t le32(const uint8_t* p) { return mac_lo(p); }

}  // namespace

struct upe_gpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    size_t cap = 0;                // rule_stats capacity
    // rules
    RuleV4* rv4 = nullptr;
    RuleV6* rv6 = nullptr;
    int2* rinfo = nullptr;
    size_t rules_alloc = 0;
    uint32_t nrules = 0, nrules_pad = 0;
    unsigned long long* acc_stats = nullptr;   // [2][kReps][rules_alloc][2] (small tables)
    unsigned long long* stats_idx = nullptr;   // [rules_alloc][2] totals per sorted index
    std::vector<int2> rinfo_host;              // (action, rule_id) per sorted index
    // neighbour tables (reachable-entry indexes)
    uint4* arp = nullptr;
    uint32_t arp_bits = 0, arp_seed = 0;
    uint4* ndp = nullptr;
    uint32_t ndp_bits = 0, ndp_seed = 0;
    // state
    DevL1* l1 = nullptr;
    DevTotals* totals = nullptr;
    unsigned long long* stats = nullptr;   // [cap][2]
    BatchAcc* acc = nullptr;
    // per-batch scratch
    ChunkPay* pay = nullptr;       // [ntiles * kWaves]
    uint32_t* cand_tile = nullptr; // [ntiles]
    size_t tiles_alloc = 0;
    uint32_t epoch = 0;
    int cus = 256;
    uint32_t port_mac_lo = 0, port_mac_hi = 0, port_ip4 = 0;
    bool have_batch = false;
    // kernel timing (upe_gpu_timing_*)
    bool timing = false;
    uint32_t timing_every = 1, timing_calls = 0;   // sample every n-th process() call
    std::vector<hipEvent_t> ev;   // event pool, 3 per process() call: start, mid, end
    size_t ev_used = 0;
};

namespace {

NeighIndex arp_index(const upe_gpu_ctx* c) { return NeighIndex{c->arp, c->arp_bits, c->arp_seed}; }
NeighIndex ndp_index(const upe_gpu_ctx* c) { return NeighIndex{c->ndp, c->ndp_bits, c->ndp_seed}; }

// Two-choice cuckoo placement of distinct keys (by their 32-bit hash key; different entries may
// share a hash key, the device compares the full address).  Starts at 2^bits >= 2.5 n slots and
// tries seeds, then doubles, until every key sits in slot1 or slot2.  bits = 0 for no keys.
int cuckoo_place(const std::vector<uint32_t>& key, uint32_t& bits, uint32_t& seed,
                 std::vector<int32_t>& slot) {
    const size_t n = key.size();
    slot.clear();
    bits = 0;
    seed = 0;
    if (n == 0) return 0;
    bits = 1;
    while (((size_t)1 << bits) * 2 < n * 5) ++bits;
    for (; bits <= 31; ++bits) {
        const size_t m = (size_t)1 << bits;
        for (uint32_t attempt = 0; attempt < 64; ++attempt) {
            const uint32_t sd = attempt * 0x6D2B79F5u + bits;
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

int ensure_scratch(upe_gpu_ctx* c, size_t ntiles) {
    if (ntiles > c->tiles_alloc) {
        if (c->pay) (void)hipFree(c->pay);
        if (c->cand_tile) (void)hipFree(c->cand_tile);
        c->pay = nullptr;
        c->cand_tile = nullptr;
        c->tiles_alloc = 0;
        size_t want = ntiles + ntiles / 4 + 16;
        HIP_TRY(hipMalloc(&c->pay, want * kWaves * sizeof(ChunkPay)));
        HIP_TRY(hipMalloc(&c->cand_tile, want * sizeof(uint32_t)));
        c->tiles_alloc = want;
    }
    return 0;
}

int refresh(upe_gpu_ctx* c) {
    hipLaunchKernelGGL(upe_refresh, dim3(1), dim3(64), 0, c->stream, c->l1, arp_index(c),
                       ndp_index(c));
    HIP_TRY(hipGetLastError());
    return 0;
}

int arm_acc(upe_gpu_ctx* c) {
    HIP_TRY(hipMemsetAsync(c->acc, 0, 2 * sizeof(BatchAcc), c->stream));
    HIP_TRY(hipMemsetAsync(reinterpret_cast<char*>(c->acc + 1) + offsetof(BatchAcc, mins), 0xFF,
                           sizeof(((BatchAcc*)nullptr)->mins), c->stream));
    HIP_TRY(hipMemsetAsync(reinterpret_cast<char*>(c->acc) + offsetof(BatchAcc, mins), 0xFF,
                           sizeof(((BatchAcc*)nullptr)->mins), c->stream));
    return 0;
}


hipStream_t pick(upe_gpu_ctx* c, void* s) { return s ? (hipStream_t)s : c->stream; }

}  // namespace

extern "C" {

const char* upe_gpu_last_error(void) { return g_err.c_str(); }

int upe_gpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return -1;
    return n;
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
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return bad(e, "hipSetDevice");
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess)
        return bad(e, "hipStreamCreate");
    if ((e = hipMalloc(&c->l1, sizeof(DevL1))) != hipSuccess) return bad(e, "hipMalloc l1");
    if ((e = hipMalloc(&c->totals, sizeof(DevTotals))) != hipSuccess) return bad(e, "hipMalloc");
    if ((e = hipMalloc(&c->stats, rule_capacity * 2 * sizeof(unsigned long long))) != hipSuccess)
        return bad(e, "hipMalloc stats");
    if ((e = hipMalloc(&c->acc, 2 * sizeof(BatchAcc))) != hipSuccess) return bad(e, "hipMalloc acc");
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) ==
                hipSuccess && cus > 0)
            c->cus = cus;
    }
    if (arm_acc(c) != 0) {
        std::string m = g_err;
        upe_gpu_close(c);
        g_err = m;
        return nullptr;
    }
    if ((e = hipMemsetAsync(c->l1, 0, sizeof(DevL1), c->stream)) != hipSuccess ||
        (e = hipMemsetAsync(c->totals, 0, sizeof(DevTotals), c->stream)) != hipSuccess ||
        (e = hipMemsetAsync(c->stats, 0, rule_capacity * 2 * sizeof(unsigned long long),
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
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    void* bufs[] = {c->rv4, c->rv6, c->rinfo, c->acc_stats, c->stats_idx, c->arp, c->ndp, c->l1,
                    c->totals, c->stats, c->acc, c->pay, c->cand_tile};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

namespace {
// Credit the sorted-index totals of the current table to rule_stats[rule_id] (device) and clear
// them: called before the table changes, so a reload keeps every count (src/main.c:216-282
// swaps rule_stats with the table; here the counts simply carry over by rule_id).
int fold_stats_idx(upe_gpu_ctx* c) {
    if (!c->stats_idx || c->rinfo_host.empty() || c->nrules_pad > (uint32_t)kSmallRules) return 0;
    const size_t E = 2 * (size_t)c->nrules_pad;
    std::vector<unsigned long long> idx(E), st(2 * c->cap);
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(idx.data(), c->stats_idx, E * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    bool any = false;
    for (unsigned long long v : idx) any |= v != 0;
    if (!any) return 0;
    HIP_TRY(hipMemcpy(st.data(), c->stats, st.size() * sizeof(unsigned long long),
                      hipMemcpyDeviceToHost));
    for (size_t e = 0; e < E; ++e)
        if (idx[e]) st[2 * (size_t)(uint32_t)c->rinfo_host[e >> 1].y + (e & 1)] += idx[e];
    HIP_TRY(hipMemcpy(c->stats, st.data(), st.size() * sizeof(unsigned long long),
                      hipMemcpyHostToDevice));
    HIP_TRY(hipMemset(c->stats_idx, 0, E * sizeof(unsigned long long)));
    return 0;
}
}  // namespace

extern "C" int upe_gpu_load_rules(upe_gpu_ctx_t* c, const upe_rule_t* rules, size_t count) {
    if (!c) return fail("null context");
    if (count > c->cap) return fail("rule count exceeds the capacity given at open");
    if (count && !rules) return fail("null rules");
    HIP_TRY(hipSetDevice(c->device));
    const size_t pad = ((count + kUnroll - 1) / kUnroll + 1) * kUnroll;  // >= 1 padding block
    std::vector<RuleV4> v4(pad);
    std::vector<RuleV6> v6(pad);
    std::vector<int2> info(pad);
    for (size_t i = 0; i < pad; ++i) {
        RuleV4& a = v4[i];
        RuleV6& b = v6[i];
        memset(&a, 0, sizeof a);
        memset(&b, 0, sizeof b);
        if (i >= count) {
            // never matches: ip_ver byte 0xFF against a key version of 4 or 6
            a.x0 = 0xFF;
            a.m0 = 0xFF;
            info[i] = make_int2(0, 0);
            continue;
        }
        const upe_rule_t& r = rules[i];
        if (r.rule_id >= c->cap) return fail("rule_id >= capacity (rule_stats index)");
        a.x0 = (uint32_t)r.ip_ver | ((uint32_t)r.protocol << 8) | ((uint32_t)r.src_port << 16);
        a.m0 = (r.ip_ver ? 0xFFu : 0u) | (r.protocol ? 0xFF00u : 0u) |
               (r.src_port ? 0xFFFF0000u : 0u);
        a.x1 = r.dst_port;
        a.m1 = r.dst_port ? 0xFFFFu : 0u;
        const uint8_t* si = r.src_ip.v6;
        const uint8_t* sm = r.src_mask.v6;
        const uint8_t* di = r.dst_ip.v6;
        const uint8_t* dm = r.dst_mask.v6;
        a.sm0 = le32(sm);
        a.s0 = le32(si) & a.sm0;
        a.dm0 = le32(dm);
        a.d0 = le32(di) & a.dm0;
        for (int j = 0; j < 3; ++j) {
            b.sm[j] = le32(sm + 4 * (j + 1));
            b.s[j] = le32(si + 4 * (j + 1)) & b.sm[j];
            b.dm[j] = le32(dm + 4 * (j + 1));
            b.d[j] = le32(di + 4 * (j + 1)) & b.dm[j];
        }
        info[i] = make_int2(r.action.type, (int)r.rule_id);
    }
    HIP_TRY(hipStreamSynchronize(c->stream));   // previous batches may still read the table
    if (fold_stats_idx(c) != 0) return -1;
    if (pad > c->rules_alloc) {
        if (c->rv4) (void)hipFree(c->rv4);
        if (c->rv6) (void)hipFree(c->rv6);
        if (c->rinfo) (void)hipFree(c->rinfo);
        if (c->acc_stats) (void)hipFree(c->acc_stats);
        c->rv4 = nullptr; c->rv6 = nullptr; c->rinfo = nullptr; c->acc_stats = nullptr;
        c->rules_alloc = 0;
        HIP_TRY(hipMalloc(&c->rv4, pad * sizeof(RuleV4)));
        HIP_TRY(hipMalloc(&c->rv6, pad * sizeof(RuleV6)));
        HIP_TRY(hipMalloc(&c->rinfo, pad * sizeof(int2)));
        const size_t acc_words = pad <= (size_t)kSmallRules ? 2 * (size_t)kReps * pad * 2 : 2;
        HIP_TRY(hipMalloc(&c->acc_stats, acc_words * sizeof(unsigned long long)));
        HIP_TRY(hipMemset(c->acc_stats, 0, acc_words * sizeof(unsigned long long)));
        if (c->stats_idx) (void)hipFree(c->stats_idx);
        c->stats_idx = nullptr;
        HIP_TRY(hipMalloc(&c->stats_idx, pad * 2 * sizeof(unsigned long long)));
        HIP_TRY(hipMemset(c->stats_idx, 0, pad * 2 * sizeof(unsigned long long)));
        c->rules_alloc = pad;
    }
    HIP_TRY(hipMemcpy(c->rv4, v4.data(), pad * sizeof(RuleV4), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->rv6, v6.data(), pad * sizeof(RuleV6), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->rinfo, info.data(), pad * sizeof(int2), hipMemcpyHostToDevice));
    if (pad <= (size_t)kSmallRules && c->nrules_pad != (uint32_t)pad) {
        // accumulator rows are indexed with the padded count: clear them for the new layout
        HIP_TRY(hipMemset(c->acc_stats, 0, 2 * (size_t)kReps * pad * 2 * sizeof(unsigned long long)));
    }
    c->nrules = (uint32_t)count;
    c->nrules_pad = (uint32_t)pad;
    c->rinfo_host = info;
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
    HIP_TRY(hipSetDevice(c->device));
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
    // Place the reachable entries by two-choice cuckoo hashing at load factor <= 0.4.
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
    if (cuckoo_place(akey, abits, aseed, aslot) != 0 || cuckoo_place(nkey, nbits, nseed, nslot) != 0)
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
    if (c->l1 && refresh(c) != 0) return -1;   // does the L1 state agree with the new tables?
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
    HIP_TRY(hipSetDevice(c->device));
    DevL1 d;
    memset(&d, 0, sizeof d);
    d.arp_ip = l1->last_arp_ip;
    d.arp_mac_lo = mac_lo(l1->last_arp_mac);
    d.arp_mac_hi = mac_hi(l1->last_arp_mac);
    for (int j = 0; j < 4; ++j) d.ndp_ip[j] = le32(l1->last_ndp_ip + 4 * j);
    d.ndp_mac_lo = mac_lo(l1->last_ndp_mac);
    d.ndp_mac_hi = mac_hi(l1->last_ndp_mac);
    HIP_TRY(hipMemcpyAsync(c->l1, &d, sizeof d, hipMemcpyHostToDevice, c->stream));
    if (refresh(c) != 0) return -1;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

int upe_gpu_get_l1(upe_gpu_ctx_t* c, upe_l1_state_t* l1) {
    if (!c || !l1) return fail("null argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    DevL1 d;
    HIP_TRY(hipMemcpy(&d, c->l1, sizeof d, hipMemcpyDeviceToHost));
    memset(l1, 0, sizeof *l1);
    l1->last_arp_ip = d.arp_ip;
    memcpy(l1->last_arp_mac, &d.arp_mac_lo, 4);
    memcpy(l1->last_arp_mac + 4, &d.arp_mac_hi, 2);
    memcpy(l1->last_ndp_ip, d.ndp_ip, 16);
    memcpy(l1->last_ndp_mac, &d.ndp_mac_lo, 4);
    memcpy(l1->last_ndp_mac + 4, &d.ndp_mac_hi, 2);
    return 0;
}

int upe_gpu_process(upe_gpu_ctx_t* c, uint8_t* d_frames, const uint64_t* d_desc,
                    uint32_t* d_verdict, size_t n, void* stream) {
    if (!c) return fail("null context");
    if (n > 0xFFFFFFFFull - kTile) return fail("batch too large (n must fit in 32 bits)");
    if (n && (!d_frames || !d_desc || !d_verdict)) return fail("null batch buffer");
    if (((uintptr_t)d_frames & 15u) != 0) return fail("frames buffer must be 16-byte aligned");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    const uint32_t ntiles = (uint32_t)((n + kTile - 1) / kTile);
    if (ensure_scratch(c, ntiles ? ntiles : 1) != 0) return -1;
    if (s != c->stream) {
        // the context's own uploads (tables, L1) were queued on its stream: order after them
        hipEvent_t dep;
        HIP_TRY(hipEventCreateWithFlags(&dep, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(dep, c->stream));
        HIP_TRY(hipStreamWaitEvent(s, dep, 0));
        HIP_TRY(hipEventDestroy(dep));
    }
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    const bool timed = c->timing && (c->timing_calls++ % c->timing_every) == 0;
    if (timed) {
        while (c->ev.size() < c->ev_used + 3) {
            hipEvent_t e;
            HIP_TRY(hipEventCreate(&e));
            c->ev.push_back(e);
        }
        for (int j = 0; j < 3; ++j) ev[j] = c->ev[c->ev_used + j];
        c->ev_used += 3;
        HIP_TRY(hipEventRecord(ev[0], s));
    }
    Args a;
    a.frames = d_frames;
    a.desc = d_desc;
    a.verdict = d_verdict;
    a.n = (uint32_t)n;
    a.ntiles = ntiles;
    a.parity = (++c->epoch) & 1u;
    a.rv4 = c->rv4;
    a.rv6 = c->rv6;
    a.rinfo = c->rinfo;
    a.nrules_pad = c->nrules_pad;
    a.arp = arp_index(c);
    a.ndp = ndp_index(c);
    a.l1 = c->l1;
    a.acc = c->acc;
    a.pay = c->pay;
    a.cand_tile = c->cand_tile;
    a.acc_stats = c->acc_stats;
    a.stats = c->stats;
    a.stats_idx = c->stats_idx;
    a.totals = c->totals;
    a.port_mac_lo = c->port_mac_lo;
    a.port_mac_hi = c->port_mac_hi;
    a.port_ip4 = c->port_ip4;
    const bool lds_stats = c->nrules_pad <= (uint32_t)kLdsStatsMax;
    const size_t lds = lds_stats ? 2 * (size_t)c->nrules_pad * sizeof(uint32_t) : 0;
    const uint32_t grid = ntiles ? ntiles : 1;
    hipLaunchKernelGGL(upe_classify, dim3(grid), dim3(kBlock), lds, s, a);
    HIP_TRY(hipGetLastError());
    if (timed) HIP_TRY(hipEventRecord(ev[1], s));
    const uint32_t fgrid = grid < 256 ? grid : 256;
    if (!(kAblate & 32)) {
        hipLaunchKernelGGL(upe_finalize, dim3(fgrid), dim3(kBlock), 0, s, a);
        HIP_TRY(hipGetLastError());
    }
    if (timed) HIP_TRY(hipEventRecord(ev[2], s));
    c->have_batch = true;
    return 0;
}

int upe_gpu_sync(upe_gpu_ctx_t* c, void* stream) {
    if (!c) return fail("null context");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(pick(c, stream)));
    return 0;
}

int upe_gpu_batch_info(upe_gpu_ctx_t* c, upe_batch_info_t* info) {
    if (!c || !info) return fail("null argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    DevTotals t;
    HIP_TRY(hipMemcpy(&t, c->totals, sizeof t, hipMemcpyDeviceToHost));
    memset(info, 0, sizeof *info);
    if (!c->have_batch) {
        info->first_ctrl = ~0ull;
        return 0;
    }
    uint64_t* dst = &info->counters.pkts_in;
    for (int j = 0; j < 8; ++j) dst[j] = t.batch[j];
    info->n_ctrl = t.n_ctrl;
    info->first_ctrl = t.first_ctrl;
    if (t.error) return fail("a tile look-back gave up waiting (results of a batch are invalid)");
    return 0;
}

int upe_gpu_get_stats(upe_gpu_ctx_t* c, upe_counters_t* counters, upe_rule_stat_t* rule_stats,
                      size_t capacity) {
    if (!c) return fail("null context");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    if (counters) {
        DevTotals t;
        HIP_TRY(hipMemcpy(&t, c->totals, sizeof t, hipMemcpyDeviceToHost));
        uint64_t* dst = &counters->pkts_in;
        for (int j = 0; j < 8; ++j) dst[j] = t.cnt[j];
    }
    if (rule_stats) {
        const size_t k = capacity < c->cap ? capacity : c->cap;
        HIP_TRY(hipMemcpy(rule_stats, c->stats, k * sizeof(upe_rule_stat_t), hipMemcpyDeviceToHost));
        if (c->nrules_pad <= (uint32_t)kSmallRules && c->stats_idx) {
            // small tables keep this table's counts per sorted index: credit them to rule_id
            const size_t E = 2 * (size_t)c->nrules_pad;
            std::vector<unsigned long long> idx(E);
            HIP_TRY(hipMemcpy(idx.data(), c->stats_idx, E * sizeof(unsigned long long),
                              hipMemcpyDeviceToHost));
            for (size_t e = 0; e < E; ++e) {
                const uint32_t rid = (uint32_t)c->rinfo_host[e >> 1].y;
                if (!idx[e] || rid >= k) continue;
                if (e & 1) rule_stats[rid].bytes += idx[e];
                else rule_stats[rid].packets += idx[e];
            }
        }
    }
    return 0;
}

int upe_gpu_reset_stats(upe_gpu_ctx_t* c) {
    if (!c) return fail("null context");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemsetAsync(c->totals, 0, sizeof(DevTotals), c->stream));
    HIP_TRY(hipMemsetAsync(c->stats, 0, c->cap * 2 * sizeof(unsigned long long), c->stream));
    if (c->stats_idx)
        HIP_TRY(hipMemsetAsync(c->stats_idx, 0, (size_t)c->rules_alloc * 2 * sizeof(unsigned long long),
                               c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->have_batch = false;
    return 0;
}

int upe_gpu_timing_enable(upe_gpu_ctx_t* c, int enable) {
    if (!c) return fail("null context");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    c->ev_used = 0;   // the pool is kept for reuse
    c->timing = enable > 0;
    c->timing_every = enable > 0 ? (uint32_t)enable : 1u;
    c->timing_calls = 0;
    return 0;
}

int upe_gpu_timing_read(upe_gpu_ctx_t* c, double* classify_ms, double* finalize_ms,
                        uint64_t* launches) {
    if (!c) return fail("null context");
    HIP_TRY(hipSetDevice(c->device));
    double a = 0, b = 0;
    for (size_t j = 0; j + 3 <= c->ev_used; j += 3) {
        HIP_TRY(hipEventSynchronize(c->ev[j + 2]));
        float x = 0, y = 0;
        HIP_TRY(hipEventElapsedTime(&x, c->ev[j], c->ev[j + 1]));
        HIP_TRY(hipEventElapsedTime(&y, c->ev[j + 1], c->ev[j + 2]));
        a += x;
        b += y;
    }
    if (classify_ms) *classify_ms = a;
    if (finalize_ms) *finalize_ms = b;
    if (launches) *launches = c->ev_used / 3;
    return 0;
}

void* upe_gpu_malloc(upe_gpu_ctx_t* c, size_t bytes) {
    if (!c) {
        fail("null context");
        return nullptr;
    }
    void* p = nullptr;
    if (hipSetDevice(c->device) != hipSuccess || hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) {
        fail("hipMalloc failed");
        return nullptr;
    }
    return p;
}

int upe_gpu_free(upe_gpu_ctx_t* c, void* p) {
    if (!c) return fail("null context");
    HIP_TRY(hipSetDevice(c->device));
    if (p) HIP_TRY(hipFree(p));
    return 0;
}

int upe_gpu_memcpy_h2d(upe_gpu_ctx_t* c, void* dst, const void* src, size_t bytes, void* stream) {
    if (!c) return fail("null context");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, pick(c, stream)));
    return 0;
}

int upe_gpu_memcpy_d2h(upe_gpu_ctx_t* c, void* dst, const void* src, size_t bytes, void* stream) {
    if (!c) return fail("null context");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, pick(c, stream)));
    return 0;
}

}  // extern "C"
