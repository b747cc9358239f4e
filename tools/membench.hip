// tools/membench.hip — diagnostic microbenchmarks of the config-B data movement alone (no parse,
// no classify): how fast can one launch move 1M descriptors + 64-byte frames + verdicts (+ the
// in-place header stores) on this GPU, and which launch structure gets there.  Not product
// code; results go to profiles/r02/.  Build: hipcc --offload-arch=gfx950 -O3 -o build/membench
// tools/membench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,          \
                    hipGetErrorString(e_));                                    \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

// store modes: 0 none, 1 two 16-B stores (bytes 0..31) for even packets, 2 one 64-B frame
// (four 16-B stores) for even packets, 3 two 16-B stores for every packet, 4 the whole frame for
// every packet (every 128-B line written whole), 5 the whole frame for packets i with (i >> 1)
// even (half of the lines written whole, half untouched), 6 bytes 0..31 to a separate packed
// array for every packet, 7 the same for even packets only, 8 16 bytes to a packed array, every
// packet
__device__ uint4* g_out;
template <int kStore>
__device__ __forceinline__ uint32_t body(uint8_t* frames, const uint64_t* desc, uint32_t i) {
    const uint64_t d = desc[i];
    const uint4* q = reinterpret_cast<const uint4*>(frames + ((d >> 20) << 4));
    const uint32_t len = (uint32_t)(d & 0xFFFF);
    uint4 v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = (c < 3 || len > 48u) ? q[c] : make_uint4(0, 0, 0, 0);
    uint32_t h = v[0].x ^ v[1].y ^ v[2].z ^ v[3].w ^ v[0].w ^ v[1].x;
    uint4* o = const_cast<uint4*>(q);
    const bool fw = kStore == 3 || (i & 1) == 0;
    if (kStore == 1 || kStore == 3) {
        if (fw) {
            o[0] = make_uint4(v[0].x + 1, v[0].y, v[0].z, v[0].w);
            o[1] = make_uint4(v[1].x, v[1].y + 1, v[1].z, v[1].w);
        }
    } else if (kStore == 4 || (kStore == 5 && ((i >> 1) & 1) == 0)) {
        o[0] = make_uint4(v[0].x + 1, v[0].y, v[0].z, v[0].w);
        o[1] = make_uint4(v[1].x, v[1].y + 1, v[1].z, v[1].w);
        o[2] = v[2];
        o[3] = v[3];
    } else if (kStore == 6 || (kStore == 7 && fw)) {
        g_out[2 * (size_t)i] = make_uint4(v[0].x + 1, v[0].y, v[0].z, v[0].w);
        g_out[2 * (size_t)i + 1] = make_uint4(v[1].x, v[1].y + 1, v[1].z, v[1].w);
    } else if (kStore == 8) {
        g_out[i] = make_uint4(v[0].x + 1, v[0].y, v[0].z, v[1].w);
    } else if (kStore == 2) {
        if (fw) {
            o[0] = make_uint4(v[0].x + 1, v[0].y, v[0].z, v[0].w);
            o[1] = make_uint4(v[1].x, v[1].y + 1, v[1].z, v[1].w);
            o[2] = v[2];
            o[3] = v[3];
        }
    }
    return h;
}

// one packet per lane, one tile per workgroup
template <int kStore>
__global__ void __launch_bounds__(256) flat(uint8_t* frames, const uint64_t* desc, uint32_t* verdict,
                                            uint32_t n) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    verdict[i] = body<kStore>(frames, desc, i);
}

// persistent: workgroup b takes tiles b, b + grid, ...
template <int kStore>
__global__ void __launch_bounds__(256) persist(uint8_t* frames, const uint64_t* desc,
                                               uint32_t* verdict, uint32_t n) {
    const uint32_t nt = (n + 255) / 256;
    for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
        const uint32_t i = t * 256 + threadIdx.x;
        if (i < n) verdict[i] = body<kStore>(frames, desc, i);
    }
}

// persistent with the next tile's descriptor and frame loaded while the current one is used
template <int kStore>
__global__ void __launch_bounds__(256) persist_pf(uint8_t* frames, const uint64_t* desc,
                                                  uint32_t* verdict, uint32_t n) {
    const uint32_t nt = (n + 255) / 256;
    uint32_t t = blockIdx.x;
    if (t >= nt) return;
    uint32_t i = t * 256 + threadIdx.x;
    uint64_t d = i < n ? desc[i] : 0;
    uint4 v[4];
    {
        const uint4* q = reinterpret_cast<const uint4*>(frames + ((d >> 20) << 4));
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = i < n ? q[c] : make_uint4(0, 0, 0, 0);
    }
    for (;;) {
        const uint32_t tn = t + gridDim.x;
        const uint32_t in = tn * 256 + threadIdx.x;
        uint64_t dn = 0;
        uint4 w[4];
        if (tn < nt) {
            dn = in < n ? desc[in] : 0;
            const uint4* qn = reinterpret_cast<const uint4*>(frames + ((dn >> 20) << 4));
#pragma unroll
            for (int c = 0; c < 4; ++c) w[c] = in < n ? qn[c] : make_uint4(0, 0, 0, 0);
        }
        if (i < n) {
            uint32_t h = v[0].x ^ v[1].y ^ v[2].z ^ v[3].w ^ v[0].w ^ v[1].x;
            uint4* o = reinterpret_cast<uint4*>(frames + ((d >> 20) << 4));
            const bool fw = kStore == 3 || (i & 1) == 0;
            if (kStore && fw) {
                o[0] = make_uint4(v[0].x + 1, v[0].y, v[0].z, v[0].w);
                o[1] = make_uint4(v[1].x, v[1].y + 1, v[1].z, v[1].w);
                if (kStore == 2) { o[2] = v[2]; o[3] = v[3]; }
            }
            verdict[i] = h;
        }
        if (tn >= nt) break;
        t = tn; i = in; d = dn;
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = w[c];
    }
}

// the read floor: the same bytes as one contiguous coalesced stream (16 B per lane)
__global__ void __launch_bounds__(256) coalesced(const uint4* frames, const uint4* desc,
                                                 uint32_t* verdict, uint32_t n) {
    // frames: n * 4 uint4, desc: n / 2 uint4; one thread = 4 frame chunks + half a desc uint4
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t nf = n * 4;
    uint32_t h = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint4 v = frames[(uint32_t)c * n + i];   // coalesced sweeps
        h ^= v.x ^ v.w;
    }
    if (i < n / 2) h ^= desc[i].x;
    (void)nf;
    verdict[i] = h;
}


// ---- compute + record store variants: every packet also costs ~kWork VALU ops (4 chains) and
// stores a 16-byte record plus its verdict, as the classify kernel does in emit mode ----------
constexpr int kWork = 48;
__device__ __forceinline__ uint4 crunch(const uint4 (&v)[4], uint32_t i) {
    uint32_t a = v[0].x ^ i, b = v[1].y, c = v[2].z, d = v[3].w;
#pragma unroll
    for (int k = 0; k < kWork; ++k) {
        a = a * 0x9E3779B1u + v[k & 3].x;
        b = (b ^ (b >> 7)) + v[(k + 1) & 3].y;
        c = c * 0x85EBCA77u + v[(k + 2) & 3].z;
        d = (d << 3) ^ v[(k + 3) & 3].w;
    }
    return make_uint4(a, b, c, d);
}

template <bool kFlat>
__global__ void __launch_bounds__(256) work_plain(const uint8_t* frames, const uint64_t* desc,
                                                  uint32_t* verdict, uint4* rec, uint32_t n) {
    const uint32_t nt = (n + 255) / 256;
    for (uint32_t t = blockIdx.x; t < nt; t += kFlat ? nt : gridDim.x) {
        const uint32_t i = t * 256 + threadIdx.x;
        if (i >= n) break;
        const uint64_t d = desc[i];
        const uint4* q = reinterpret_cast<const uint4*>(frames + ((d >> 20) << 4));
        uint4 v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = q[c];
        const uint4 r = crunch(v, i);
        rec[i] = r;
        verdict[i] = r.x ^ r.w;
    }
}

// one-deep software pipeline, branch-free loads (dead lanes load the buffer's first bytes), two
// register sets used in turn (a copy between them would wait for the loads)
__global__ void __launch_bounds__(256) work_pipe(const uint8_t* frames, const uint64_t* desc,
                                                 uint32_t* verdict, uint4* rec, uint32_t n) {
    const uint32_t nt = (n + 255) / 256;
    const uint32_t G = gridDim.x;
    uint32_t t = blockIdx.x;
    if (t >= nt) return;
    auto idx = [&](uint32_t tt) {
        const uint32_t i = tt * 256 + threadIdx.x;
        return tt < nt && i < n ? i : 0u;
    };
    auto load = [&](uint64_t d, uint4 (&w)[4]) {
        const uint4* q = reinterpret_cast<const uint4*>(frames + ((d >> 20) << 4));
#pragma unroll
        for (int c = 0; c < 4; ++c) w[c] = q[c];
    };
    auto work = [&](uint32_t tt, const uint4 (&w)[4]) {
        const uint32_t i = tt * 256 + threadIdx.x;
        const uint4 r = crunch(w, i);
        if (i < n) {
            rec[i] = r;
            verdict[i] = r.x ^ r.w;
        }
    };
    uint4 A[4], B[4];
    uint64_t dB = desc[idx(t + G)];
    load(desc[idx(t)], A);
    for (;;) {
        const uint64_t dA = desc[idx(t + 2 * G)];
        load(dB, B);
        work(t, A);
        t += G;
        if (t >= nt) break;
        dB = desc[idx(t + 2 * G)];
        load(dA, A);
        work(t, B);
        t += G;
        if (t >= nt) break;
    }
}

struct Case {
    const char* name;
    void (*launch)(uint8_t*, const uint64_t*, uint32_t*, uint32_t, int, hipStream_t);
};

template <int S>
void L_flat(uint8_t* f, const uint64_t* d, uint32_t* v, uint32_t n, int, hipStream_t s) {
    hipLaunchKernelGGL(flat<S>, dim3((n + 255) / 256), dim3(256), 0, s, f, d, v, n);
}
template <int S>
void L_persist(uint8_t* f, const uint64_t* d, uint32_t* v, uint32_t n, int g, hipStream_t s) {
    hipLaunchKernelGGL(persist<S>, dim3(g), dim3(256), 0, s, f, d, v, n);
}
template <int S>
void L_persist_pf(uint8_t* f, const uint64_t* d, uint32_t* v, uint32_t n, int g, hipStream_t s) {
    hipLaunchKernelGGL(persist_pf<S>, dim3(g), dim3(256), 0, s, f, d, v, n);
}
uint4* g_rec_host;
void L_work_flat(uint8_t* f, const uint64_t* d, uint32_t* v, uint32_t n, int, hipStream_t s) {
    hipLaunchKernelGGL(work_plain<true>, dim3((n + 255) / 256), dim3(256), 0, s, f, d, v, g_rec_host, n);
}
void L_work_persist(uint8_t* f, const uint64_t* d, uint32_t* v, uint32_t n, int g, hipStream_t s) {
    hipLaunchKernelGGL(work_plain<false>, dim3(g), dim3(256), 0, s, f, d, v, g_rec_host, n);
}
void L_work_pipe(uint8_t* f, const uint64_t* d, uint32_t* v, uint32_t n, int g, hipStream_t s) {
    hipLaunchKernelGGL(work_pipe, dim3(g), dim3(256), 0, s, f, d, v, g_rec_host, n);
}
void L_coal(uint8_t* f, const uint64_t* d, uint32_t* v, uint32_t n, int, hipStream_t s) {
    hipLaunchKernelGGL(coalesced, dim3((n + 255) / 256), dim3(256), 0, s, (const uint4*)f,
                       (const uint4*)d, v, n);
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
    const int reps = argc > 2 ? atoi(argv[2]) : 100;
    const char* only = argc > 3 ? argv[3] : nullptr;   // substring filter of case names
    const size_t fb = (size_t)n * 64 + 256;
    int copies = (int)((12ull << 30) / fb);
    if (copies > 220) copies = 220;
    if (copies < 2) copies = 2;
    uint8_t* pool;
    uint64_t* desc;
    uint32_t* verdict;
    CK(hipMalloc(&pool, fb * copies));
    CK(hipMalloc(&desc, (size_t)n * 8));
    CK(hipMalloc(&verdict, (size_t)n * 4));
    CK(hipMemset(pool, 0x45, fb * copies));
    uint4* outp;
    CK(hipMalloc(&outp, (size_t)n * 32));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_out), &outp, sizeof outp));
    g_rec_host = outp;
    std::vector<uint64_t> hd(n);
    for (uint32_t i = 0; i < n; ++i) hd[i] = ((uint64_t)i * 64) << 16 | 64;
    CK(hipMemcpy(desc, hd.data(), (size_t)n * 8, hipMemcpyHostToDevice));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const Case cases[] = {
        {"flat_out16_all", L_flat<8>},
        {"work_flat", L_work_flat},
        {"pwork_plain", L_work_persist},
        {"pwork_pipe", L_work_pipe},
        {"coalesced_read", L_coal},
        {"flat_read", L_flat<0>},
        {"flat_st32_half", L_flat<1>},
        {"flat_st64_half", L_flat<2>},
        {"flat_st32_all", L_flat<3>},
        {"flat_stfull_all", L_flat<4>},
        {"flat_stfull_pairs", L_flat<5>},
        {"flat_out32_all", L_flat<6>},
        {"flat_out32_half", L_flat<7>},
        {"flat_out16_all", L_flat<8>},
        {"persist_read", L_persist<0>},
        {"persist_st32_half", L_persist<1>},
        {"persist_pf_read", L_persist_pf<0>},
        {"persist_pf_st32_half", L_persist_pf<1>},
        {"persist_pf_st64_half", L_persist_pf<2>},
    };
    const int grids[] = {1024, 1280};
    printf("n=%u copies=%d reps=%d (us per launch; GB/s of desc+frames+verdict)\n", n, copies,
           reps);
    for (const Case& c : cases) {
        const bool per = c.name[0] == 'p';
        if (only && !strstr(c.name, only)) continue;
        for (int gi = 0; gi < (per ? 2 : 1); ++gi) {
            const int g = grids[gi];
            for (int k = 0; k < 5; ++k) c.launch(pool + (size_t)(k % copies) * fb, desc, verdict, n, g, s);
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(e0, s));
            for (int k = 0; k < reps; ++k)
                c.launch(pool + (size_t)((k + 5) % copies) * fb, desc, verdict, n, g, s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            CK(hipGetLastError());
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / reps;
            printf("%-22s grid %5d  %8.2f us  %7.1f GB/s  %7.1f Gpps\n", c.name, per ? g : (int)((n + 255) / 256),
                   us, (double)n * 76 / us / 1e3, n / us / 1e3);
        }
    }
    return 0;
}
