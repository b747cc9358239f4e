// tools/waitvalue_probe.hip — does hipStreamWaitValue32 on signal memory written by a running
// kernel release a second stream's kernel while the first still runs, and how fast?  (diagnostic)
// Kernel A (stream X): its workgroups count themselves started; the last one stores 1 into the
// signal word; every workgroup then runs ~200 us.  Stream Y: WaitValue32(sig >= 1), then kernel
// B, which records its start.  Prints B's start relative to A's signal store and A's end.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/waitvalue_probe tools/waitvalue_probe.hip
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

__global__ void kernel_a(uint32_t* started, uint64_t* sig, unsigned long long* t, uint32_t grid) {
    if (threadIdx.x == 0) {
        const uint32_t old = atomicAdd(started, 1u);
        if (old + 1 == grid) {
            t[0] = __builtin_amdgcn_s_memrealtime();
            __hip_atomic_store(sig, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 20000) __builtin_amdgcn_s_sleep(8);  // 200 us
    if (threadIdx.x == 0) atomicMax(&t[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

__global__ void kernel_b(unsigned long long* t) {
    if (threadIdx.x == 0) atomicMin(&t[2], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

int main() {
    int can = 0;
    CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0));
    printf("hipDeviceAttributeCanUseStreamWaitValue = %d\n", can);
    if (!can) return 0;
    uint64_t* sig;
    CK(hipExtMallocWithFlags((void**)&sig, 8, hipMallocSignalMemory));
    uint32_t* started;
    unsigned long long* t;
    CK(hipMalloc(&started, 4));
    CK(hipMallocManaged(&t, 3 * sizeof(unsigned long long)));
    hipStream_t x, y;
    CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&y, hipStreamNonBlocking));
    for (int rep = 0; rep < 5; ++rep) {
        CK(hipMemset(sig, 0, 8));
        CK(hipMemset(started, 0, 4));
        t[0] = 0; t[1] = 0; t[2] = ~0ull;
        CK(hipDeviceSynchronize());
        const uint32_t grid = 128;   // half the CUs: B's workgroups have room
        hipLaunchKernelGGL(kernel_a, dim3(grid), dim3(256), 0, x, started, sig, t, grid);
        CK(hipStreamWaitValue32(y, sig, 1, hipStreamWaitValueGte, 0xFFFFFFFFu));
        hipLaunchKernelGGL(kernel_b, dim3(1), dim3(64), 0, y, t);
        CK(hipDeviceSynchronize());
        printf("rep %d: B started %.2f us after A's signal, %.2f us before A's end\n", rep,
               (double)(t[2] - t[0]) / 100.0, ((double)t[1] - (double)t[2]) / 100.0);
    }
    return 0;
}
