// tools/fetch_calib.hip — calibration of rocprofv3's FETCH_SIZE on gfx950 for the access shapes
// the classify kernels make (diagnostic, not product code).  MI355X_MICROARCH.md §HBM validates
// "read bytes = 2 x FETCH_SIZE" only for wide coalesced streaming reads; config D's windows and
// tuple-space slots are gathers.  Each mode reads a known set of addresses from a 4 GiB buffer
// (16x the Infinity Cache, so nothing is re-served on-die) once; the program prints, per mode,
// the bytes the lanes asked for, the distinct 64-B sectors and 128-B lines they touch, and
// tools/fetch_calib.sh sets FETCH_SIZE per dispatch beside them.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

constexpr uint64_t kBuf = 4ull << 30;
constexpr uint32_t kLanes = 1u << 22;

__host__ __device__ inline uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
    return x ^ (x >> 33);
}

// mode 0 streaming 16 B per lane; 1 one 16-B load per random 128-B line; 2 two 16-B loads in one
// random line; 3 64 B at a random 64-aligned offset; 4 32 B at a random 32-aligned offset (a
// tuple-space IPv4 slot); 5 80 B at a random 16-aligned offset (a header window); 6 and 7 one
// 16-B load per random line of a 64 MiB region (Infinity-Cache resident: 6 fills, 7 re-reads)
__host__ __device__ inline void shape(int mode, uint32_t i, uint64_t& off, int& n16) {
    const uint64_t r = mix(i + 0x9e3779b97f4a7c15ull * (uint64_t)(mode + 1));
    switch (mode) {
        case 0: off = 16ull * i; n16 = 1; break;
        case 1: off = (r % (kBuf / 128)) * 128; n16 = 1; break;
        case 2: off = (r % (kBuf / 128)) * 128; n16 = 2; break;
        case 3: off = (r % (kBuf / 64)) * 64; n16 = 4; break;
        case 4: off = (r % (kBuf / 32)) * 32; n16 = 2; break;
        case 5: off = (r % (kBuf / 16 - 8)) * 16; n16 = 5; break;
        default: {
            const uint64_t r6 = mix(i + 0x9e3779b97f4a7c15ull * 7);   // modes 6, 7: same lines
            off = (r6 % ((64ull << 20) / 128)) * 128; n16 = 1; break;
        }
    }
}

__global__ void __launch_bounds__(256) gather(const uint4* buf, int mode, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint64_t off;
    int n16;
    shape(mode, i, off, n16);
    const uint4* q = buf + off / 16;
    uint32_t h = 0;
    for (int c = 0; c < n16; ++c) {
        const uint4 v = q[c];
        h ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (h == 0x12345678u) out[i] = h;   // keeps the loads; never true for the zero buffer
}

int main() {
    uint4* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, kBuf));
    CK(hipMemset(buf, 0, kBuf));
    CK(hipMalloc(&out, kLanes * sizeof(uint32_t)));
    static const char* names[] = {"stream16", "line128_16B", "line128_2x16B", "sector64_64B",
                                  "slot32_32B", "window80_16align", "mall_fill", "mall_reread"};
    for (int mode = 0; mode < 8; ++mode) {
        std::vector<uint64_t> sec, lin;
        uint64_t bytes = 0;
        for (uint32_t i = 0; i < kLanes; ++i) {
            uint64_t off;
            int n16;
            shape(mode, i, off, n16);
            bytes += 16ull * n16;
            for (uint64_t b = off; b < off + 16ull * n16; b += 16) {
                sec.push_back(b / 64);
                lin.push_back(b / 128);
            }
        }
        std::sort(sec.begin(), sec.end());
        std::sort(lin.begin(), lin.end());
        const size_t ns = std::unique(sec.begin(), sec.end()) - sec.begin();
        const size_t nl = std::unique(lin.begin(), lin.end()) - lin.begin();
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(gather, dim3(kLanes / 256), dim3(256), 0, 0, buf, mode, out);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        printf("mode %d %-18s lanes %u asked %.1f MB  sectors64 %.1f MB  lines128 %.1f MB\n", mode,
               names[mode], kLanes, bytes / 1e6, ns * 64.0 / 1e6, nl * 128.0 / 1e6);
        fflush(stdout);
    }
    return 0;
}
