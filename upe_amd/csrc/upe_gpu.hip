// upe_gpu.hip — MI355X (gfx950 / CDNA4) batch dataplane for UPE's per-packet worker hot path,
// and the extern "C" ABI declared in include/upe_gpu.h.
//
// One lane owns one packet.  Per packet the classify kernel does what reference process_packet()
// does (src/worker.c:106-253): control-packet classification (src/worker.c:23-104), the
// fixed-format parse (src/parser.c:6-111), first-match over the priority-sorted rule table
// (src/rule_table.c:76-91,163-176), counters and rule_stats (src/worker.c:119-153), and the
// L3-forward rewrite: TTL / hop-limit decrement, RFC 1071 checksum (src/parser.c:137-169), next-hop
// MAC from arp_get_mac / ndp_get_mac probing the reference slot layout (src/arp_table.c:55-80,
// src/ndp_table.c:6-17,67-86).  Frames are rewritten in place in HBM.
//
// Data layout (DESIGN.md "HBM layout"): frames packed back to back at 16-byte aligned starts,
// one uint64 descriptor per packet (offset << 16 | len), one uint32 verdict per packet.  A lane
// reads at most the first UPE_HDR_WINDOW bytes of its frame as 16-byte vector loads.  The rule
// table is compiled into three structure-of-arrays streams that the wave scans with wave-uniform
// (scalar-unit) loads, so rule operands arrive in SGPRs and cost no VGPR or LDS bandwidth; the
// per-rule work is a handful of VALU xor/and against them, with an early exit once every lane
// of the wave has its first match (ballot).  Rule stats are histogrammed in LDS per tile.
//
// The worker's one-entry L1 neighbour caches are sequential state (src/worker.c:186-195,
// 218-225).  They are emulated exactly with first-index / last-index reductions
// (SURVEY.md §8.1 item 16): classify resolves every forwarded packet through the table and
// records, per tile, the first packet that misses the starting L1 entry and hits the table and
// the last packet that hits the table; finalize combines the tiles, repairs the packets that the
// starting entry would have answered differently (only possible when that entry disagrees with
// the table), and writes the new L1 state for the next batch.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/upe_gpu.h"

namespace {

constexpr int kBlock = 256;            // 4 waves of 64
constexpr int kWaves = kBlock / 64;
constexpr int kPPT = 4;                // packets per thread per tile
constexpr int kTile = kBlock * kPPT;   // packets per workgroup
constexpr int kUnroll = 4;             // rules per early-exit check
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kSlabMaxCap = 4096;      // rule_stats histogrammed in LDS up to this capacity

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

// L1 state in word form (device resident between batches).
struct DevL1 {
    uint32_t arp_ip, arp_mac_lo, arp_mac_hi;
    uint32_t ndp_ip[4];
    uint32_t ndp_mac_lo, ndp_mac_hi;
    uint32_t pad[7];
};

// Per-tile partial results written by classify, combined by finalize.
enum { C_PARSED, C_MATCHED, C_FWD, C_DROPPED, C_CONSUMED, C_ARP_LEARN, C_ARP_REPLY, C_CTRL, C_N };
struct __attribute__((aligned(16))) TileRec {
    uint32_t cnt[C_N];
    uint32_t first_ctrl;
    uint32_t f4, m4, c4, f6, m6, c6; // first miss-then-hit, last hit (index+1, 0 = none), first L1_INIT
    uint32_t m4_dst, m4_mac_lo, m4_mac_hi;
    uint32_t m6_dst[4], m6_mac_lo, m6_mac_hi;
    uint32_t pad[3];
};

// Accumulated worker state (device resident).
struct DevTotals {
    unsigned long long cnt[8]; // upe_counters_t order
    unsigned long long n_ctrl, first_ctrl;
    unsigned long long batch[8];
};

struct ClassifyArgs {
    uint8_t* frames;
    const uint64_t* desc;
    uint32_t* verdict;
    uint32_t n;
    const RuleV4* rv4;
    const RuleV6* rv6;
    const int2* rinfo;
    uint32_t nrules_pad;      // multiple of kUnroll, padding rules never match
    const uint4* arp;         // {ip, mac0..3, mac4..5 | valid << 16, 0}
    uint32_t arp_cap;
    const uint4* ndp;         // 2 x uint4 per slot: {ip w0..w3}, {mac0..3, mac4..5 | valid<<16, 0, 0}
    uint32_t ndp_cap;
    const DevL1* l1;
    TileRec* tiles;
    uint32_t* slab;           // [ntiles][cap][2] when cap <= kSlabMaxCap
    unsigned long long* stats; // [cap][2] totals (direct atomics when cap > kSlabMaxCap)
    uint32_t cap;
    uint32_t port_mac_lo, port_mac_hi, port_ip4;
};

// ---- small helpers ------------------------------------------------------------------------
__device__ __forceinline__ uint32_t byte_of(uint32_t w, int k) { return (w >> (8 * k)) & 0xFFu; }
__device__ __forceinline__ uint32_t at2(uint32_t hi, uint32_t lo) {   // dword at byte 4q+2
    return __builtin_amdgcn_alignbit(hi, lo, 16);
}
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint32_t be16_lo(uint32_t x) {             // BE u16 in bytes 0,1
    return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu);
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}

// arp_get_mac (reference src/arp_table.c:55-80): idx = ip & (cap-1), linear probe, stop at the
// first invalid slot, at most cap probes.
__device__ __forceinline__ bool arp_lookup(const uint4* __restrict__ t, uint32_t cap, uint32_t ip,
                                           uint32_t& lo, uint32_t& hi) {
    if (cap == 0) return false;
    const uint32_t mask = cap - 1;
    uint32_t idx = ip & mask;
    for (uint32_t i = 0; i < cap; ++i) {
        const uint4 e = t[(idx + i) & mask];
        const bool valid = (e.z >> 16) & 1u;
        if (valid && e.x == ip) {
            lo = e.y;
            hi = e.z & 0xFFFFu;
            return true;
        }
        if (!valid) break;
    }
    return false;
}

// ndp_get_mac + hash_ipv6 (reference src/ndp_table.c:6-17,67-86): hash = XOR of the four LE
// u32 words of the address.
__device__ __forceinline__ bool ndp_lookup(const uint4* __restrict__ t, uint32_t cap,
                                           const uint32_t ip[4], uint32_t& lo, uint32_t& hi) {
    if (cap == 0) return false;
    const uint32_t mask = cap - 1;
    uint32_t idx = (ip[0] ^ ip[1] ^ ip[2] ^ ip[3]) & mask;
    for (uint32_t i = 0; i < cap; ++i) {
        const uint32_t s = (idx + i) & mask;
        const uint4 meta = t[2 * s + 1];
        const bool valid = (meta.y >> 16) & 1u;
        if (valid) {
            const uint4 a = t[2 * s];
            if (a.x == ip[0] && a.y == ip[1] && a.z == ip[2] && a.w == ip[3]) {
                lo = meta.x;
                hi = meta.y & 0xFFFFu;
                return true;
            }
        } else {
            break;
        }
    }
    return false;
}

// First-match scan (reference src/rule_table.c:163-176 over match_rule :76-91).  Every lane of
// the wave walks the same rules in sorted order; rule words are wave-uniform loads.  `done`
// lanes (already matched, or not scanning) are ignored.  V6 = some lane holds an IPv6 key.
template <bool V6>
__device__ __forceinline__ uint32_t scan_rules(const ClassifyArgs& a, bool done, bool is6,
                                               uint32_t k0, uint32_t k1, const uint32_t s[4],
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
// classify: one tile of kTile packets per workgroup
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) upe_classify(ClassifyArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_hist[]; // [cap][2] (slab mode)
    __shared__ uint32_t s_cnt[C_N];
    __shared__ uint32_t s_red[kWaves][16];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const uint32_t tile = blockIdx.x;
    const bool slab_mode = a.cap <= (uint32_t)kSlabMaxCap;

    if (slab_mode)
        for (uint32_t r = tid; r < 2 * a.cap; r += kBlock) lds_hist[r] = 0;
    if (tid < C_N) s_cnt[tid] = 0;
    __syncthreads();

    // L1 state at batch start (uniform).
    const uint32_t l1_arp_ip = a.l1->arp_ip;
    uint32_t l1_ndp[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) l1_ndp[j] = a.l1->ndp_ip[j];

    // Per-lane running L1 bookkeeping; indices increase with k so first/last are trivial.
    uint32_t f4 = kNone, c4 = kNone, m4 = 0, m4_dst = 0, m4_lo = 0, m4_hi = 0;
    uint32_t f6 = kNone, c6 = kNone, m6 = 0, m6_lo = 0, m6_hi = 0;
    uint32_t m6_dst[4] = {0, 0, 0, 0};
    uint32_t first_ctrl = kNone;
    uint32_t cnt_parsed = 0, cnt_matched = 0, cnt_fwd = 0, cnt_dropped = 0, cnt_consumed = 0,
             cnt_learn = 0, cnt_reply = 0, cnt_ctrl = 0;

    for (int k = 0; k < kPPT; ++k) {
        const uint32_t i = tile * kTile + (uint32_t)(k * kBlock + tid);
        const bool live = i < a.n;
        uint64_t dsc = live ? a.desc[i] : 0;
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
        const bool ext = live && (is_v6 || (is_v4 && ihl > 5));
        if (ext) {
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
        bool wrote2 = false;  // chunk 2

        // ---- handle_control_packet, reference src/worker.c:23-104 ----
        if (live && et == 0x0806u) {
            // ARP header bytes 14..41, read without a length check (zero beyond len).
            auto mb = [&](int b) -> uint32_t {
                return (uint32_t)b < len ? byte_of(w[b >> 2], b & 3) : 0u;
            };
            const bool wellformed = mb(14) == 0 && mb(15) == 1 && mb(16) == 0x08 && mb(17) == 0 &&
                                    mb(18) == 6 && mb(19) == 4;
            if (wellformed) {
                flags |= UPE_VF_ARP_LEARN;
                const uint32_t op = (mb(20) << 8) | mb(21);
                const uint32_t tpa = (mb(38) << 24) | (mb(39) << 16) | (mb(40) << 8) | mb(41);
                if (op == 1 && a.port_ip4 != 0 && tpa == a.port_ip4) {
                    // In-place reply, src/worker.c:42-51.  Build the new bytes 0..41, keep the
                    // original beyond len (writes past b->len are never transmitted).
                    uint8_t nb[48];
#pragma unroll
                    for (int b = 0; b < 48; ++b) nb[b] = (uint8_t)mb(b);
                    uint8_t ob[48];
#pragma unroll
                    for (int b = 0; b < 48; ++b) ob[b] = nb[b];
#pragma unroll
                    for (int b = 0; b < 6; ++b) {
                        nb[b] = ob[6 + b];                                   // eth.dst = eth.src
                        nb[6 + b] = (uint8_t)((b < 4 ? a.port_mac_lo >> (8 * b)
                                                     : a.port_mac_hi >> (8 * (b - 4))) & 0xFF);
                        nb[32 + b] = ob[22 + b];                             // tha = sha
                        nb[22 + b] = nb[6 + b];                              // sha = port MAC
                    }
                    nb[20] = 0; nb[21] = 2;                                  // op = REPLY
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        nb[38 + b] = ob[28 + b];                             // tpa = spa
                        nb[28 + b] = (uint8_t)(a.port_ip4 >> (24 - 8 * b));  // spa = port IPv4
                    }
#pragma unroll
                    for (int j = 0; j < 12; ++j) {
                        uint32_t v = 0;
#pragma unroll
                        for (int b = 0; b < 4; ++b) {
                            const int bi = 4 * j + b;
                            const uint32_t nv = (uint32_t)bi < len ? nb[bi] : byte_of(w[j], b);
                            v |= nv << (8 * b);
                        }
                        w[j] = v;
                    }
                    wrote0 = wrote1 = wrote2 = true;
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

        // ---- rule_table_match ----
        const uint32_t ver = is_v6 ? 6u : 4u;
        const uint32_t k0 = ver | (proto << 8) | (sport << 16);
        const uint32_t k1 = dport;
        const bool need_v6 = __any(ok && is_v6);
        uint32_t ri = need_v6 ? scan_rules<true>(a, !ok, is_v6, k0, k1, s, d)
                              : scan_rules<false>(a, !ok, is_v6, k0, k1, s, d);

        // ---- verdict, counters, rule_stats (src/worker.c:117-153) ----
        uint32_t code;
        uint32_t rbits = 0;
        int act = 0;
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
            act = info.x;
            rbits = (ri + 1) << 8;
            const uint32_t rid = (uint32_t)info.y;
            if (slab_mode) {
                atomicAdd(&lds_hist[2 * rid], 1u);
                atomicAdd(&lds_hist[2 * rid + 1], len);
            } else {
                atomicAdd(&a.stats[2 * rid], 1ull);
                atomicAdd(&a.stats[2 * rid + 1], (unsigned long long)len);
            }
            code = act == UPE_ACT_DROP ? UPE_V_DROP_RULE
                 : act == UPE_ACT_FWD  ? UPE_V_FWD
                                       : UPE_V_DROP_ACTION;
        }

        // ---- L3 forward (src/worker.c:155-244) ----
        if (code == UPE_V_FWD) {
            if (!is_v6) {
                const uint32_t ttl = byte_of(w[5], 2);                       // byte 22
                if (ttl <= 1u) {
                    code = UPE_V_DROP_TTL;
                } else {
                    // ttl--, checksum = 0, checksum = ipv4_checksum(ip, IHL*4), stored LE.
                    const uint32_t hw2 = (ttl - 1) | (byte_of(w[5], 3) << 8); // bytes 22..25
                    unsigned long long sum = 0;
#pragma unroll
                    for (int j = 0; j < 15; ++j) {
                        const uint32_t dw = j == 2 ? hw2 : at2(w[4 + j], w[3 + j]);
                        if ((uint32_t)j < ihl) sum += dw;
                    }
                    uint32_t f = (uint32_t)(sum & 0xFFFFFFFFull) + (uint32_t)(sum >> 32);
                    f += (uint32_t)(sum & 0xFFFFFFFFull) > f ? 1u : 0u; // carry of the add
                    f = (f & 0xFFFFu) + (f >> 16);
                    f = (f & 0xFFFFu) + (f >> 16);
                    f = (f & 0xFFFFu) + (f >> 16);
                    const uint32_t cs = (~f) & 0xFFFFu;
                    // bytes 22..25 live in w[5] bytes 2,3 and w[6] bytes 0,1
                    w[5] = (w[5] & 0x0000FFFFu) | ((ttl - 1) << 16) | (byte_of(w[5], 3) << 24);
                    w[6] = (w[6] & 0xFFFF0000u) | cs;
                    wrote1 = true;
                    uint32_t lo, hi;
                    const bool hit = arp_lookup(a.arp, a.arp_cap, d[0], lo, hi);
                    if (l1_arp_ip != 0 && d[0] == l1_arp_ip) {
                        flags |= UPE_VF_L1_INIT;
                        c4 = min(c4, i);
                    } else if (hit) {
                        f4 = min(f4, i);
                    }
                    if (hit) {
                        m4 = i + 1; m4_dst = d[0]; m4_lo = lo; m4_hi = hi;
                        w[0] = lo;
                        w[1] = hi | (a.port_mac_lo << 16);
                        w[2] = (a.port_mac_lo >> 16) | (a.port_mac_hi << 16);
                        wrote0 = true;
                        flags |= UPE_VF_NEIGH_HIT;
                    }
                }
            } else {
                const uint32_t hop = byte_of(w[5], 1);                       // byte 21
                if (hop <= 1u) {
                    code = UPE_V_DROP_TTL;
                } else {
                    w[5] = (w[5] & 0xFFFF00FFu) | ((hop - 1) << 8);
                    wrote1 = true;
                    uint32_t lo, hi;
                    const bool hit = ndp_lookup(a.ndp, a.ndp_cap, d, lo, hi);
                    if (d[0] == l1_ndp[0] && d[1] == l1_ndp[1] && d[2] == l1_ndp[2] &&
                        d[3] == l1_ndp[3]) {
                        flags |= UPE_VF_L1_INIT;
                        c6 = min(c6, i);
                    } else if (hit) {
                        f6 = min(f6, i);
                    }
                    if (hit) {
                        m6 = i + 1; m6_lo = lo; m6_hi = hi;
                        m6_dst[0] = d[0]; m6_dst[1] = d[1]; m6_dst[2] = d[2]; m6_dst[3] = d[3];
                        w[0] = lo;
                        w[1] = hi | (a.port_mac_lo << 16);
                        w[2] = (a.port_mac_lo >> 16) | (a.port_mac_hi << 16);
                        wrote0 = true;
                        flags |= UPE_VF_NEIGH_HIT;
                    }
                }
            }
        }

        // ---- write back ----
        if (live) {
            uint4* q = reinterpret_cast<uint4*>(p);
            if (wrote0) q[0] = make_uint4(w[0], w[1], w[2], w[3]);
            if (wrote1) q[1] = make_uint4(w[4], w[5], w[6], w[7]);
            if (wrote2) q[2] = make_uint4(w[8], w[9], w[10], w[11]);
            a.verdict[i] = code | flags | rbits;
            if (ctrl) first_ctrl = min(first_ctrl, i);
        }
        cnt_parsed += live && !consumed && ok;
        cnt_matched += live && !consumed && ok && ri != kNone;
        cnt_fwd += live && code == UPE_V_FWD;
        cnt_dropped += live && code != UPE_V_FWD && code != UPE_V_CONSUMED;
        cnt_consumed += live && consumed;
        cnt_learn += live && !consumed && (flags & UPE_VF_ARP_LEARN);
        cnt_reply += live && !consumed && (flags & UPE_VF_ARP_REPLY);
        cnt_ctrl += ctrl;
    }

    // ---- tile reduction ----
    auto wsum = [](uint32_t v) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
        return v;
    };
    const uint32_t cs[C_N] = {cnt_parsed, cnt_matched, cnt_fwd, cnt_dropped,
                              cnt_consumed, cnt_learn, cnt_reply, cnt_ctrl};
#pragma unroll
    for (int c = 0; c < C_N; ++c) {
        const uint32_t v = wsum(cs[c]);
        if (lane == 0 && v) atomicAdd(&s_cnt[c], v);
    }
    // min / max reductions and the payload of the last table hit of each family
    const uint32_t wf4 = wave_min(f4), wc4 = wave_min(c4), wm4 = wave_max(m4);
    const uint32_t wf6 = wave_min(f6), wc6 = wave_min(c6), wm6 = wave_max(m6);
    const uint32_t wfc = wave_min(first_ctrl);
    if (lane == 0) {
        s_red[wave][0] = wf4; s_red[wave][1] = wc4; s_red[wave][2] = wm4;
        s_red[wave][3] = wf6; s_red[wave][4] = wc6; s_red[wave][5] = wm6;
        s_red[wave][6] = wfc;
    }
    if (wm4 != 0 && m4 == wm4) {
        s_red[wave][7] = m4_dst; s_red[wave][8] = m4_lo; s_red[wave][9] = m4_hi;
    }
    if (wm6 != 0 && m6 == wm6) {
        s_red[wave][10] = m6_dst[0]; s_red[wave][11] = m6_dst[1];
        s_red[wave][12] = m6_dst[2]; s_red[wave][13] = m6_dst[3];
        s_red[wave][14] = m6_lo; s_red[wave][15] = m6_hi;
    }
    __syncthreads();

    TileRec* rec = &a.tiles[tile];
    if (tid == 0) {
        TileRec r;
        for (int c = 0; c < C_N; ++c) r.cnt[c] = s_cnt[c];
        r.f4 = r.c4 = r.f6 = r.c6 = r.first_ctrl = kNone;
        r.m4 = r.m6 = 0;
        r.m4_dst = r.m4_mac_lo = r.m4_mac_hi = 0;
        r.m6_dst[0] = r.m6_dst[1] = r.m6_dst[2] = r.m6_dst[3] = r.m6_mac_lo = r.m6_mac_hi = 0;
        r.pad[0] = r.pad[1] = r.pad[2] = 0;
        for (int v = 0; v < kWaves; ++v) {
            r.f4 = min(r.f4, s_red[v][0]);
            r.c4 = min(r.c4, s_red[v][1]);
            r.f6 = min(r.f6, s_red[v][3]);
            r.c6 = min(r.c6, s_red[v][4]);
            r.first_ctrl = min(r.first_ctrl, s_red[v][6]);
            if (s_red[v][2] > r.m4) {
                r.m4 = s_red[v][2];
                r.m4_dst = s_red[v][7]; r.m4_mac_lo = s_red[v][8]; r.m4_mac_hi = s_red[v][9];
            }
            if (s_red[v][5] > r.m6) {
                r.m6 = s_red[v][5];
                r.m6_dst[0] = s_red[v][10]; r.m6_dst[1] = s_red[v][11];
                r.m6_dst[2] = s_red[v][12]; r.m6_dst[3] = s_red[v][13];
                r.m6_mac_lo = s_red[v][14]; r.m6_mac_hi = s_red[v][15];
            }
        }
        *rec = r;
    }
    if (slab_mode) {
        uint32_t* out = a.slab + (size_t)tile * 2 * a.cap;
        for (uint32_t r = tid; r < 2 * a.cap; r += kBlock) out[r] = lds_hist[r];
    }
}

// ------------------------------------------------------------------------------------------
// finalize: combine tiles, repair L1-start answers, update L1 + totals.  Grid: block 0 does the
// sequential-state work; every block reduces a slice of the rule_stats slab.
// ------------------------------------------------------------------------------------------
struct FinalizeArgs {
    uint8_t* frames;
    const uint64_t* desc;
    uint32_t* verdict;
    uint32_t n;
    const TileRec* tiles;
    uint32_t ntiles;
    const uint32_t* slab;
    unsigned long long* stats;
    uint32_t cap;
    const uint4* arp;
    uint32_t arp_cap;
    const uint4* ndp;
    uint32_t ndp_cap;
    DevL1* l1;
    DevTotals* totals;
    uint32_t port_mac_lo, port_mac_hi;
};

__global__ void __launch_bounds__(kBlock) upe_finalize(FinalizeArgs a) {
    const int tid = threadIdx.x;
    // rule_stats slab: one thread per (rule, field)
    if (a.cap <= (uint32_t)kSlabMaxCap) {
        for (uint32_t e = blockIdx.x * kBlock + tid; e < 2 * a.cap; e += gridDim.x * kBlock) {
            unsigned long long acc = 0;
            for (uint32_t t = 0; t < a.ntiles; ++t) acc += a.slab[(size_t)t * 2 * a.cap + e];
            if (acc) a.stats[e] += acc;
        }
    }
    if (blockIdx.x != 0) return;

    __shared__ unsigned long long s_cnt[C_N];
    __shared__ uint32_t s_min[5];        // f4, c4, f6, c6, first_ctrl
    __shared__ uint32_t s_m4, s_m6;      // max (index+1)
    __shared__ uint32_t s_rep[4];        // repair ranges: [lo4, hi4), [lo6, hi6)
    __shared__ uint32_t s_mac[4];        // mac0 (arp lo/hi, ndp lo/hi) for repairs
    if (tid < C_N) s_cnt[tid] = 0;
    if (tid < 5) s_min[tid] = kNone;
    if (tid == 0) { s_m4 = 0; s_m6 = 0; }
    __syncthreads();

    unsigned long long c[C_N];
#pragma unroll
    for (int j = 0; j < C_N; ++j) c[j] = 0;
    uint32_t f4 = kNone, c4 = kNone, f6 = kNone, c6 = kNone, fc = kNone, m4 = 0, m6 = 0;
    for (uint32_t t = tid; t < a.ntiles; t += kBlock) {
        const TileRec& r = a.tiles[t];
#pragma unroll
        for (int j = 0; j < C_N; ++j) c[j] += r.cnt[j];
        f4 = min(f4, r.f4); c4 = min(c4, r.c4); f6 = min(f6, r.f6); c6 = min(c6, r.c6);
        fc = min(fc, r.first_ctrl);
        m4 = max(m4, r.m4); m6 = max(m6, r.m6);
    }
#pragma unroll
    for (int j = 0; j < C_N; ++j) {
        unsigned long long v = c[j];
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if ((tid & 63) == 0 && v) atomicAdd(&s_cnt[j], v);
    }
    f4 = wave_min(f4); c4 = wave_min(c4); f6 = wave_min(f6); c6 = wave_min(c6); fc = wave_min(fc);
    m4 = wave_max(m4); m6 = wave_max(m6);
    if ((tid & 63) == 0) {
        atomicMin(&s_min[0], f4); atomicMin(&s_min[1], c4);
        atomicMin(&s_min[2], f6); atomicMin(&s_min[3], c6); atomicMin(&s_min[4], fc);
        atomicMax(&s_m4, m4); atomicMax(&s_m6, m6);
    }
    __syncthreads();

    DevL1* l1 = a.l1;
    if (tid == 0) {
        // Is the starting L1 entry what the table would answer?  If so, every packet's answer
        // is the table's and nothing needs repair.
        uint32_t lo = 0, hi = 0;
        bool arp_ok = true;
        if (l1->arp_ip != 0) {
            const bool hit = arp_lookup(a.arp, a.arp_cap, l1->arp_ip, lo, hi);
            arp_ok = hit && lo == l1->arp_mac_lo && hi == l1->arp_mac_hi;
        }
        const bool ndp_hit = ndp_lookup(a.ndp, a.ndp_cap, l1->ndp_ip, lo, hi);
        const bool ndp_ok = ndp_hit && lo == l1->ndp_mac_lo && hi == l1->ndp_mac_hi;
        // Packets answered by the starting entry: L1_INIT ones before the first miss-then-hit.
        s_rep[0] = arp_ok ? 0 : s_min[1];
        s_rep[1] = arp_ok ? 0 : min(s_min[0], a.n);
        s_rep[2] = ndp_ok ? 0 : s_min[3];
        s_rep[3] = ndp_ok ? 0 : min(s_min[2], a.n);
        s_mac[0] = l1->arp_mac_lo; s_mac[1] = l1->arp_mac_hi;
        s_mac[2] = l1->ndp_mac_lo; s_mac[3] = l1->ndp_mac_hi;

        DevTotals* T = a.totals;
        const unsigned long long in = a.n;
        T->cnt[0] += in;
        T->cnt[1] += s_cnt[C_PARSED];
        T->cnt[2] += s_cnt[C_MATCHED];
        T->cnt[3] += s_cnt[C_FWD];
        T->cnt[4] += s_cnt[C_DROPPED];
        T->cnt[5] += s_cnt[C_CONSUMED];
        T->cnt[6] += s_cnt[C_ARP_LEARN];
        T->cnt[7] += s_cnt[C_ARP_REPLY];
        T->batch[0] = in;
        T->batch[1] = s_cnt[C_PARSED];
        T->batch[2] = s_cnt[C_MATCHED];
        T->batch[3] = s_cnt[C_FWD];
        T->batch[4] = s_cnt[C_DROPPED];
        T->batch[5] = s_cnt[C_CONSUMED];
        T->batch[6] = s_cnt[C_ARP_LEARN];
        T->batch[7] = s_cnt[C_ARP_REPLY];
        T->n_ctrl = s_cnt[C_CTRL];
        T->first_ctrl = s_min[4] == kNone ? ~0ull : (unsigned long long)s_min[4];
    }
    __syncthreads();

    // Repairs (rare): a forwarded packet flagged L1_INIT before the first miss-then-hit packet
    // took the starting entry's MAC in the reference, found = true (src/worker.c:186-188,218-220).
    for (int fam = 0; fam < 2; ++fam) {
        const uint32_t lo = s_rep[2 * fam], hi = s_rep[2 * fam + 1];
        for (uint32_t i = lo + tid; i < hi; i += kBlock) {
            const uint32_t v = a.verdict[i];
            if ((v & 0xFu) != UPE_V_FWD || !(v & UPE_VF_L1_INIT)) continue;
            const uint64_t dsc = a.desc[i];
            uint8_t* p = a.frames + (dsc >> 16);
            const bool six = p[12] == 0x86 && p[13] == 0xDD;
            if (six != (fam == 1)) continue;
            uint4* q = reinterpret_cast<uint4*>(p);
            uint4 c0 = q[0];
            c0.x = s_mac[2 * fam];
            c0.y = s_mac[2 * fam + 1] | (a.port_mac_lo << 16);
            c0.z = (a.port_mac_lo >> 16) | (a.port_mac_hi << 16);
            q[0] = c0;
            a.verdict[i] = v | UPE_VF_NEIGH_HIT;
        }
    }

    // New L1 state: the last table hit, if any packet missed the starting entry and hit the
    // table; otherwise unchanged.
    if (tid == 0) {
        if (s_min[0] != kNone && s_m4 != 0) {
            const uint32_t t = (s_m4 - 1) / kTile;
            const TileRec& r = a.tiles[t];
            l1->arp_ip = r.m4_dst;
            l1->arp_mac_lo = r.m4_mac_lo;
            l1->arp_mac_hi = r.m4_mac_hi;
        }
        if (s_min[2] != kNone && s_m6 != 0) {
            const uint32_t t = (s_m6 - 1) / kTile;
            const TileRec& r = a.tiles[t];
            for (int j = 0; j < 4; ++j) l1->ndp_ip[j] = r.m6_dst[j];
            l1->ndp_mac_lo = r.m6_mac_lo;
            l1->ndp_mac_hi = r.m6_mac_hi;
        }
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
    // neighbour tables
    uint4* arp = nullptr;
    uint32_t arp_cap = 0;
    uint4* ndp = nullptr;
    uint32_t ndp_cap = 0;
    // state
    DevL1* l1 = nullptr;
    DevTotals* totals = nullptr;
    unsigned long long* stats = nullptr;   // [cap][2]
    // per-batch scratch
    TileRec* tiles = nullptr;
    size_t tiles_alloc = 0;
    uint32_t* slab = nullptr;
    size_t slab_alloc = 0;
    uint32_t port_mac_lo = 0, port_mac_hi = 0, port_ip4 = 0;
    bool have_batch = false;
    // kernel timing (upe_gpu_timing_*)
    bool timing = false;
    std::vector<hipEvent_t> ev;   // 3 per process() call: before classify, between, after
};

namespace {

int ensure_scratch(upe_gpu_ctx* c, size_t ntiles) {
    if (ntiles > c->tiles_alloc) {
        if (c->tiles) (void)hipFree(c->tiles);
        c->tiles = nullptr;
        size_t want = ntiles + ntiles / 4 + 16;
        HIP_TRY(hipMalloc(&c->tiles, want * sizeof(TileRec)));
        c->tiles_alloc = want;
    }
    if (c->cap <= (size_t)kSlabMaxCap) {
        size_t words = ntiles * 2 * c->cap;
        if (words > c->slab_alloc) {
            if (c->slab) (void)hipFree(c->slab);
            c->slab = nullptr;
            size_t want = words + words / 4 + 64;
            HIP_TRY(hipMalloc(&c->slab, want * sizeof(uint32_t)));
            c->slab_alloc = want;
        }
    }
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
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return bad(e, "sync");
    return c;
}

void upe_gpu_close(upe_gpu_ctx_t* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    void* bufs[] = {c->rv4, c->rv6, c->rinfo, c->arp, c->ndp, c->l1, c->totals, c->stats,
                    c->tiles, c->slab};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int upe_gpu_load_rules(upe_gpu_ctx_t* c, const upe_rule_t* rules, size_t count) {
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
    if (pad > c->rules_alloc) {
        if (c->rv4) (void)hipFree(c->rv4);
        if (c->rv6) (void)hipFree(c->rv6);
        if (c->rinfo) (void)hipFree(c->rinfo);
        c->rv4 = nullptr; c->rv6 = nullptr; c->rinfo = nullptr;
        c->rules_alloc = 0;
        HIP_TRY(hipMalloc(&c->rv4, pad * sizeof(RuleV4)));
        HIP_TRY(hipMalloc(&c->rv6, pad * sizeof(RuleV6)));
        HIP_TRY(hipMalloc(&c->rinfo, pad * sizeof(int2)));
        c->rules_alloc = pad;
    }
    HIP_TRY(hipStreamSynchronize(c->stream));   // previous batches may still read the table
    HIP_TRY(hipMemcpy(c->rv4, v4.data(), pad * sizeof(RuleV4), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->rv6, v6.data(), pad * sizeof(RuleV6), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->rinfo, info.data(), pad * sizeof(int2), hipMemcpyHostToDevice));
    c->nrules = (uint32_t)count;
    c->nrules_pad = (uint32_t)pad;
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
    std::vector<uint4> a(arp_capacity ? arp_capacity : 1);
    for (size_t i = 0; i < arp_capacity; ++i) {
        const upe_arp_entry_t& e = arp[i];
        a[i] = make_uint4(e.ip, mac_lo(e.mac), mac_hi(e.mac) | ((e.valid ? 1u : 0u) << 16), 0);
    }
    std::vector<uint4> b(2 * (ndp_capacity ? ndp_capacity : 1));
    for (size_t i = 0; i < ndp_capacity; ++i) {
        const upe_ndp_entry_t& e = ndp[i];
        b[2 * i] = make_uint4(le32(e.ip), le32(e.ip + 4), le32(e.ip + 8), le32(e.ip + 12));
        b[2 * i + 1] = make_uint4(mac_lo(e.mac), mac_hi(e.mac) | ((e.valid ? 1u : 0u) << 16), 0, 0);
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->arp) (void)hipFree(c->arp);
    if (c->ndp) (void)hipFree(c->ndp);
    c->arp = nullptr; c->ndp = nullptr;
    HIP_TRY(hipMalloc(&c->arp, a.size() * sizeof(uint4)));
    HIP_TRY(hipMalloc(&c->ndp, b.size() * sizeof(uint4)));
    HIP_TRY(hipMemcpy(c->arp, a.data(), a.size() * sizeof(uint4), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->ndp, b.data(), b.size() * sizeof(uint4), hipMemcpyHostToDevice));
    c->arp_cap = (uint32_t)arp_capacity;
    c->ndp_cap = (uint32_t)ndp_capacity;
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

    const bool slab_mode = c->cap <= (size_t)kSlabMaxCap;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    if (c->timing) {
        for (int j = 0; j < 3; ++j) HIP_TRY(hipEventCreate(&ev[j]));
        for (int j = 0; j < 3; ++j) c->ev.push_back(ev[j]);
        HIP_TRY(hipEventRecord(ev[0], s));
    }
    if (ntiles) {
        ClassifyArgs a;
        a.frames = d_frames;
        a.desc = d_desc;
        a.verdict = d_verdict;
        a.n = (uint32_t)n;
        a.rv4 = c->rv4;
        a.rv6 = c->rv6;
        a.rinfo = c->rinfo;
        a.nrules_pad = c->nrules_pad;
        a.arp = c->arp;
        a.arp_cap = c->arp_cap;
        a.ndp = c->ndp;
        a.ndp_cap = c->ndp_cap;
        a.l1 = c->l1;
        a.tiles = c->tiles;
        a.slab = c->slab;
        a.stats = c->stats;
        a.cap = (uint32_t)c->cap;
        a.port_mac_lo = c->port_mac_lo;
        a.port_mac_hi = c->port_mac_hi;
        a.port_ip4 = c->port_ip4;
        const size_t lds = slab_mode ? 2 * c->cap * sizeof(uint32_t) : 0;
        hipLaunchKernelGGL(upe_classify, dim3(ntiles), dim3(kBlock), lds, s, a);
        HIP_TRY(hipGetLastError());
    }
    FinalizeArgs f;
    f.frames = d_frames;
    f.desc = d_desc;
    f.verdict = d_verdict;
    f.n = (uint32_t)n;
    f.tiles = c->tiles;
    f.ntiles = ntiles;
    f.slab = c->slab;
    f.stats = c->stats;
    f.cap = ntiles ? (uint32_t)c->cap : 0xFFFFFFFFu;  // no slab to reduce for an empty batch
    f.arp = c->arp;
    f.arp_cap = c->arp_cap;
    f.ndp = c->ndp;
    f.ndp_cap = c->ndp_cap;
    f.l1 = c->l1;
    f.totals = c->totals;
    f.port_mac_lo = c->port_mac_lo;
    f.port_mac_hi = c->port_mac_hi;
    uint32_t fblocks = 1;
    if (slab_mode && ntiles) fblocks = (uint32_t)((2 * c->cap + kBlock - 1) / kBlock);
    if (c->timing) HIP_TRY(hipEventRecord(ev[1], s));
    hipLaunchKernelGGL(upe_finalize, dim3(fblocks), dim3(kBlock), 0, s, f);
    HIP_TRY(hipGetLastError());
    if (c->timing) HIP_TRY(hipEventRecord(ev[2], s));
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
    }
    return 0;
}

int upe_gpu_reset_stats(upe_gpu_ctx_t* c) {
    if (!c) return fail("null context");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemsetAsync(c->totals, 0, sizeof(DevTotals), c->stream));
    HIP_TRY(hipMemsetAsync(c->stats, 0, c->cap * 2 * sizeof(unsigned long long), c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->have_batch = false;
    return 0;
}

int upe_gpu_timing_enable(upe_gpu_ctx_t* c, int enable) {
    if (!c) return fail("null context");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
    c->ev.clear();
    c->timing = enable != 0;
    return 0;
}

int upe_gpu_timing_read(upe_gpu_ctx_t* c, double* classify_ms, double* finalize_ms,
                        uint64_t* launches) {
    if (!c) return fail("null context");
    HIP_TRY(hipSetDevice(c->device));
    double a = 0, b = 0;
    for (size_t j = 0; j + 2 < c->ev.size(); j += 3) {
        HIP_TRY(hipEventSynchronize(c->ev[j + 2]));
        float x = 0, y = 0;
        HIP_TRY(hipEventElapsedTime(&x, c->ev[j], c->ev[j + 1]));
        HIP_TRY(hipEventElapsedTime(&y, c->ev[j + 1], c->ev[j + 2]));
        a += x;
        b += y;
    }
    if (classify_ms) *classify_ms = a;
    if (finalize_ms) *finalize_ms = b;
    if (launches) *launches = c->ev.size() / 3;
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
