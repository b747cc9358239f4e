// tools/hostwrite_probe.hip — diagnostic: the in-place header stores of the mapped host path
// (upe_gpu_process_mapped) go over the link as the kernel issues them.  Does the shape of those
// stores matter?  (Not product code.)  1M 64-byte frames in pinned host memory, 55 % of them
// "forwarded"; per forwarded frame bytes 0..31 are rewritten.  Modes:
//   0  per lane: two 16-byte stores (bytes 0..15, then 16..31), as the classify kernel does
//   1  lane pairs: in each of two store instructions the two lanes of a pair write one frame's
//      32 bytes (contiguous 32-byte pieces per instruction)
//   2  per lane: one 16-byte store (bytes 16..31 only; a lower bound)
//   3  per lane: the whole 64-byte frame as four 16-byte stores (full lines)
// Build: hipcc --offload-arch=gfx950 -O3 -o build/hostwrite_probe tools/hostwrite_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

__device__ __forceinline__ bool fwd_of(uint32_t i) {
    uint32_t h = i * 2654435761u;
    h ^= h >> 15;
    return (h % 100u) < 55u;
}

template <int kMode>
__global__ void __launch_bounds__(1024) wr(uint4* frames, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t base = (blockIdx.x * 1024 + (threadIdx.x & ~63u)); base < n;
         base += gridDim.x * 1024) {
        const uint32_t i = base + lane;
        const bool live = i < n;
        const uint4 v0 = make_uint4(i, i + 1, i + 2, i + 3), v1 = make_uint4(~i, i ^ 5, i * 3, 7);
        if (kMode == 0) {
            if (live && fwd_of(i)) {
                frames[4 * i] = v0;
                frames[4 * i + 1] = v1;
            }
        } else if (kMode == 1) {
            // pair (2j, 2j+1): first instruction writes frame 2j, second frame 2j+1
            const uint32_t even = base + (lane & ~1u), odd = even + 1;
            const uint32_t half = lane & 1u;
            const uint32_t fa = even, fb = odd;
            const uint4 a = half ? make_uint4(~fa, fa ^ 5, fa * 3, 7) : make_uint4(fa, fa + 1, fa + 2, fa + 3);
            const uint4 b = half ? make_uint4(~fb, fb ^ 5, fb * 3, 7) : make_uint4(fb, fb + 1, fb + 2, fb + 3);
            if (fa < n && fwd_of(fa)) frames[4 * fa + half] = a;
            if (fb < n && fwd_of(fb)) frames[4 * fb + half] = b;
        } else if (kMode == 2) {
            if (live && fwd_of(i)) frames[4 * i + 1] = v1;
        } else {
            if (live && fwd_of(i)) {
                frames[4 * i] = v0;
                frames[4 * i + 1] = v1;
                frames[4 * i + 2] = v0;
                frames[4 * i + 3] = v1;
            }
        }
    }
}

int main() {
    const uint32_t n = 1u << 20;
    uint4* h;
    CK(hipHostMalloc(reinterpret_cast<void**>(&h), (size_t)n * 64, hipHostMallocDefault));
    uint4* d = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int mode = 0; mode < 4; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            const int launches = 20;
            CK(hipEventRecord(e0));
            for (int k = 0; k < launches; ++k) {
                if (mode == 0) hipLaunchKernelGGL(wr<0>, dim3(cus), dim3(1024), 0, 0, d, n);
                if (mode == 1) hipLaunchKernelGGL(wr<1>, dim3(cus), dim3(1024), 0, 0, d, n);
                if (mode == 2) hipLaunchKernelGGL(wr<2>, dim3(cus), dim3(1024), 0, 0, d, n);
                if (mode == 3) hipLaunchKernelGGL(wr<3>, dim3(cus), dim3(1024), 0, 0, d, n);
            }
            CK(hipGetLastError());
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            // check: frame 2's first word (mode 0/1/3 write it when frame 2 is forwarded)
            if (rep == 1)
                printf("mode %d: %.1f us per launch (1M frames, 55 %% rewritten)\n", mode,
                       1e3 * ms / launches);
        }
    }
    uint64_t bad = 0;
    for (uint32_t i = 0; i < 1024; ++i) {
        uint32_t hh = i * 2654435761u;
        hh ^= hh >> 15;
        if ((hh % 100u) < 55u && (h[4 * i].x != i || h[4 * i + 1].x != ~i)) ++bad;
    }
    printf("check (last mode wrote frames whole): %llu bad of the first 1024\n", (unsigned long long)bad);
    CK(hipHostFree(h));
    return 0;
}
