// tools/winbench.hip — diagnostic: is config C's window load bound by the number of distinct
// lines each load instruction touches?  (Not product code.)  1M IMIX-like frames (64 / 570 / 1518
// bytes in a 7:4:1 mix, back to back at 16-byte-aligned offsets, as upe_amd.synth lays config C
// out), one persistent 1024-thread workgroup per CU whose waves take 64-packet chunks; per packet
// the 80-byte header window (16-byte pieces at or past len not loaded) is folded into a checksum
// and one 4-byte word is written.  Modes:
//   0  per-lane loads: lane i loads the five pieces of frame i (the classify kernels' scheme:
//      every load instruction touches up to 64 distinct lines)
//   1  cooperative loads: the wave's 320 pieces are loaded as 5 instructions in which five
//      neighbouring lanes take the pieces of one frame (each instruction touches ~13 frames'
//      lines), staged in LDS (5 KB per wave) and read back per lane
//   2  per-lane loads of bytes 0..47 only (three pieces; a lower bound)
//   3  a dense side array of each frame's bytes 0..63 (64-byte stride, four pieces, every line
//      used whole) plus bytes 64..79 from the frame for the 30 % of frames (IPv6) that need them
// Build: hipcc --offload-arch=gfx950 -O3 -o build/winbench tools/winbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

constexpr int kBlock = 1024, kWaves = kBlock / 64;

template <int kMode>
__global__ void __launch_bounds__(kBlock) win(const uint8_t* frames, const uint64_t* desc,
                                              uint32_t* out, uint32_t n, const uint4* side) {
    __shared__ uint4 stage[kMode == 1 ? kWaves * 320 : 1];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t nch = (n + 63) / 64;
    for (uint32_t ch = blockIdx.x * kWaves + wave; ch < nch; ch += gridDim.x * kWaves) {
        const uint32_t i = ch * 64 + lane;
        const bool live = i < n;
        uint4 w[5];
        for (int c = 0; c < 5; ++c) w[c] = make_uint4(0, 0, 0, 0);
        if (kMode == 1) {
            const uint64_t dsc = live ? desc[i] : 0;
            uint4* st = stage + wave * 320;
            for (int k = 0; k < 5; ++k) {
                const int p = 64 * k + lane, f = p / 5, c = p % 5;
                const uint64_t df = __shfl(dsc, f);
                const uint32_t len = (uint32_t)(df & 0xFFFF);
                uint4 v = make_uint4(0, 0, 0, 0);
                if (ch * 64 + f < n && (c < 3 || len > 16u * c))
                    v = reinterpret_cast<const uint4*>(frames + (df >> 16))[c];
                st[p] = v;
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (int c = 0; c < 5; ++c) w[c] = st[5 * lane + c];
            __builtin_amdgcn_wave_barrier();
        } else if (kMode == 3 && live) {
            const uint64_t dsc = desc[i];
            const uint32_t len = (uint32_t)(dsc & 0xFFFF);
            for (int c = 0; c < 4; ++c) w[c] = side[4 * (size_t)i + c];
            if (len > 64u && (i * 2654435761u) % 10u < 3u)   // the IPv6 share
                w[4] = reinterpret_cast<const uint4*>(frames + (dsc >> 16))[4];
        } else if (live) {
            const uint64_t dsc = desc[i];
            const uint32_t len = (uint32_t)(dsc & 0xFFFF);
            const uint4* q = reinterpret_cast<const uint4*>(frames + (dsc >> 16));
            const int nc = kMode == 2 ? 3 : 5;
            for (int c = 0; c < nc; ++c)
                if (c < 3 || len > 16u * c) w[c] = q[c];
        }
        uint32_t x = 0;
        for (int c = 0; c < 5; ++c) x ^= w[c].x + w[c].y * 3u + w[c].z * 5u + w[c].w * 7u;
        if (live) out[i] = x;
    }
}

__global__ void fill(uint32_t* p, size_t words) {
    for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < words;
         k += (size_t)gridDim.x * blockDim.x)
        p[k] = (uint32_t)(k * 2654435761u) ^ (uint32_t)(k >> 7);
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
    const int copies = 16;
    // IMIX sizes 7:4:1, frames back to back at 16-byte alignment, 96 readable bytes after each
    // layout 0: packed (16-byte aligned); layout 1 (argv[2] = 1): line-aligned, frames of up to 64
    // bytes on 64-byte boundaries and longer ones on 128-byte boundaries (every window in one line)
    const int aligned = argc > 2 ? atoi(argv[2]) : 0;
    std::vector<uint64_t> desc(n);
    uint64_t off = 0;
    uint64_t r = 88172645463325252ull;
    for (uint32_t i = 0; i < n; ++i) {
        r ^= r << 13; r ^= r >> 7; r ^= r << 17;
        const uint32_t k = (uint32_t)(r % 12);
        const uint32_t len = k < 7 ? 64 : k < 11 ? 570 : 1518;
        if (aligned) off = len <= 64 ? (off + 63) & ~63ull : (off + 127) & ~127ull;
        desc[i] = off << 16 | len;
        off += (len + 15) & ~15u;
    }
    const size_t fbytes = off + 96;
    const size_t stride = (fbytes + 4095) & ~(size_t)4095;
    uint8_t* frames;
    uint64_t* d_desc;
    uint32_t* out;
    CK(hipMalloc(&frames, stride * copies));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(frames),
                       stride * copies / 4);
    CK(hipDeviceSynchronize());
    CK(hipMalloc(&d_desc, n * 8));
    CK(hipMemcpy(d_desc, desc.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&out, n * 4));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("winbench: %u IMIX frames (%s), %.1f MB per copy, %d copies, grid %d x %d\n", n,
           aligned ? "line-aligned" : "packed", fbytes / 1e6, copies, cus, kBlock);
    uint4* side;
    CK(hipMalloc(&side, (size_t)n * 64 * copies));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(side),
                       (size_t)n * 16 * copies);
    CK(hipDeviceSynchronize());
    for (int mode = 0; mode < 4; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            const int launches = 48;
            CK(hipEventRecord(e0));
            for (int k = 0; k < launches; ++k) {
                const uint8_t* f = frames + (size_t)(k % copies) * stride;
                const uint4* sd = side + (size_t)(k % copies) * n * 4;
                if (mode == 0) hipLaunchKernelGGL(win<0>, dim3(cus), dim3(kBlock), 0, 0, f, d_desc, out, n, sd);
                if (mode == 1) hipLaunchKernelGGL(win<1>, dim3(cus), dim3(kBlock), 0, 0, f, d_desc, out, n, sd);
                if (mode == 2) hipLaunchKernelGGL(win<2>, dim3(cus), dim3(kBlock), 0, 0, f, d_desc, out, n, sd);
                if (mode == 3) hipLaunchKernelGGL(win<3>, dim3(cus), dim3(kBlock), 0, 0, f, d_desc, out, n, sd);
            }
            CK(hipGetLastError());
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::vector<uint32_t> h(n);
            CK(hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost));
            uint64_t sum = 0;
            for (uint32_t i = 0; i < n; ++i) sum += h[i];
            if (rep == 1)
                printf("mode %d: %.2f us per launch (%.1f Mpps), checksum %llu\n", mode,
                       1e3 * ms / launches, n / (1e3 * ms / launches), (unsigned long long)sum);
        }
    }
    return 0;
}
