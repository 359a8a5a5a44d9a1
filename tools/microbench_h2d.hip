// Host-to-device rates on MI355X for the headline's input path (prepare bodies in host memory):
//   copy     hipMemcpyAsync from pinned host memory (the runtime's engine choice), one stream
//   copy2    the same buffer split over two streams
//   pull<W>  a kernel on W workgroups reading mapped host memory (16 B per lane per load, 8 loads in
//            flight per lane) and storing to HBM
//   reg      hipMemcpyAsync from malloc'd memory registered with hipHostRegister (the engine's case)
//   d2h, d2h_8m, duplex_d2h / duplex_h2d: the other direction, sliced, and both at once
//   busy     `copy` while a kernel holding every CU spins on another stream: a copy engine (SDMA)
//            keeps its rate, a blit kernel waits for CUs
// usage: microbench_h2d [MiB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <utility>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void pull(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256 * 8;
    for (size_t base = (size_t)blockIdx.x * 256 * 8 + threadIdx.x; base < n; base += stride) {
        u32x4 v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const size_t i = base + (size_t)k * 256;
            v[k] = i < n ? __builtin_nontemporal_load(&src[i]) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const size_t i = base + (size_t)k * 256;
            if (i < n) dst[i] = v[k];
        }
    }
}

__global__ __launch_bounds__(256) void spin(unsigned long long cycles, unsigned* sink) {
    const unsigned long long t0 = clock64();
    unsigned x = threadIdx.x;
    while (clock64() - t0 < cycles) x = x * 1664525u + 1013904223u;
    if (x == 0x12345678u) *sink = x;
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? (size_t)atol(argv[1]) : 1024;
    const size_t bytes = mib << 20;
    void* h = nullptr;
    CK(hipHostMalloc(&h, bytes, hipHostMallocMapped));
    memset(h, 1, bytes);
    void* hd = nullptr;
    CK(hipHostGetDevicePointer(&hd, h, 0));
    void* d = nullptr;
    CK(hipMalloc(&d, bytes));
    hipStream_t s[2];
    CK(hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s[1], hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int reps = 5;
    auto report = [&](const char* name) {
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("%-10s %8.2f GB/s  (%zu MiB x %d in %.2f ms)\n", name, (double)bytes * reps / (ms * 1e-3) / 1e9, mib, reps,
               ms);
    };
    for (int warm = 0; warm < 2; warm++) {
        CK(hipEventRecord(a, s[0]));
        for (int r = 0; r < reps; r++) CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s[0]));
        CK(hipEventRecord(b, s[0]));
        CK(hipEventSynchronize(b));
    }
    report("copy");
    CK(hipEventRecord(a, s[0]));
    CK(hipStreamWaitEvent(s[1], a, 0));
    for (int r = 0; r < reps; r++) {
        CK(hipMemcpyAsync(d, h, bytes / 2, hipMemcpyHostToDevice, s[0]));
        CK(hipMemcpyAsync((char*)d + bytes / 2, (char*)h + bytes / 2, bytes / 2, hipMemcpyHostToDevice, s[1]));
    }
    hipEvent_t c;
    CK(hipEventCreate(&c));
    CK(hipEventRecord(c, s[1]));
    CK(hipStreamWaitEvent(s[0], c, 0));
    CK(hipEventRecord(b, s[0]));
    CK(hipEventSynchronize(b));
    report("copy2");
    const size_t n = bytes / 16;
    for (int w : {16, 32, 64, 128, 256, 512}) {
        for (int warm = 0; warm < 2; warm++) {
            CK(hipEventRecord(a, s[0]));
            for (int r = 0; r < reps; r++) hipLaunchKernelGGL(pull, dim3(w), dim3(256), 0, s[0], (const u32x4*)hd, (u32x4*)d, n);
            CK(hipEventRecord(b, s[0]));
            CK(hipEventSynchronize(b));
        }
        char name[32];
        snprintf(name, sizeof name, "pull%d", w);
        report(name);
    }
    {
        void* r = malloc(bytes);
        memset(r, 1, bytes);
        CK(hipHostRegister(r, bytes, hipHostRegisterDefault));
        for (int warm = 0; warm < 2; warm++) {
            CK(hipEventRecord(a, s[0]));
            for (int r2 = 0; r2 < reps; r2++) CK(hipMemcpyAsync(d, r, bytes, hipMemcpyHostToDevice, s[0]));
            CK(hipEventRecord(b, s[0]));
            CK(hipEventSynchronize(b));
        }
        report("reg");
        // busy: a spinning grid of 8 workgroups per CU on stream 1, the copy on stream 0
        unsigned* sink = nullptr;
        CK(hipMalloc(&sink, 4));
        int cus = 0;
        CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
        hipLaunchKernelGGL(spin, dim3(cus * 8), dim3(256), 0, s[1], 2000000000ULL, sink);  // ~1 s at 2 GHz
        CK(hipEventRecord(a, s[0]));
        for (int r2 = 0; r2 < reps; r2++) CK(hipMemcpyAsync(d, r, bytes, hipMemcpyHostToDevice, s[0]));
        CK(hipEventRecord(b, s[0]));
        CK(hipEventSynchronize(b));
        report("busy");
        CK(hipStreamSynchronize(s[1]));
        // d2h: the write-back's direction (device -> registered host memory), whole and in 8-MiB
        // slices; duplex: d2h on stream 0 while the same bytes go h2d on stream 1 (the replica's
        // copy-out beside the next prepares' bodies).
        for (int warm = 0; warm < 2; warm++) {
            CK(hipEventRecord(a, s[0]));
            for (int r2 = 0; r2 < reps; r2++) CK(hipMemcpyAsync(r, d, bytes, hipMemcpyDeviceToHost, s[0]));
            CK(hipEventRecord(b, s[0]));
            CK(hipEventSynchronize(b));
        }
        report("d2h");
        const size_t sl = std::min<size_t>(bytes, 8 << 20);
        CK(hipEventRecord(a, s[0]));
        for (int r2 = 0; r2 < reps; r2++)
            for (size_t o = 0; o < bytes; o += sl)
                CK(hipMemcpyAsync((char*)r + o, (char*)d + o, std::min(sl, bytes - o), hipMemcpyDeviceToHost, s[0]));
        CK(hipEventRecord(b, s[0]));
        CK(hipEventSynchronize(b));
        report("d2h_8m");
        void* r3 = malloc(bytes);
        memset(r3, 2, bytes);
        CK(hipHostRegister(r3, bytes, hipHostRegisterDefault));
        void* d3 = nullptr;
        CK(hipMalloc(&d3, bytes));
        hipEvent_t a1, b1;
        CK(hipEventCreate(&a1));
        CK(hipEventCreate(&b1));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, s[0]));
        CK(hipEventRecord(a1, s[1]));
        for (int r2 = 0; r2 < reps; r2++) {
            CK(hipMemcpyAsync(r, d, bytes, hipMemcpyDeviceToHost, s[0]));
            CK(hipMemcpyAsync(d3, r3, bytes, hipMemcpyHostToDevice, s[1]));
        }
        CK(hipEventRecord(b, s[0]));
        CK(hipEventRecord(b1, s[1]));
        CK(hipEventSynchronize(b));
        CK(hipEventSynchronize(b1));
        report("duplex_d2h");
        std::swap(a, a1);
        std::swap(b, b1);
        report("duplex_h2d");
        std::swap(a, a1);
        std::swap(b, b1);
        CK(hipHostUnregister(r3));
        free(r3);
        CK(hipFree(d3));
        CK(hipHostUnregister(r));
        free(r);
    }
    unsigned char probe[16];
    CK(hipMemcpy(probe, (char*)d + bytes - 16, 16, hipMemcpyDeviceToHost));
    printf("check %s\n", probe[0] == 1 && probe[15] == 1 ? "ok" : "BAD");
    return 0;
}
