// microbench_random.hip — random small-access rates on MI355X (tooling, not product).
//
// Measures, for a table of `bytes` bytes, the rate of: random 16-B loads, random 32-B loads,
// random 8-B CAS (returning), random 8-B atomicAdd (no return), random 128-B stores, and a
// coalesced 16-B/lane stream read, so the commit engine's per-transfer random-op budget can be
// priced.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mb tools/microbench_random.hip && /tmp/mb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                    \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef unsigned long long u64;

__device__ inline u64 mix(u64 x) {
    x ^= x >> 31;
    x *= 0x7fb5d329728ea185ULL;
    x ^= x >> 27;
    x *= 0x81dadef4bc2dd44dULL;
    x ^= x >> 33;
    return x;
}

template <int MODE>
__global__ void k(u64* table, u64 mask16, u64 n_ops, u64* sink) {
    u64 acc = 0;
    const u64 stride = (u64)gridDim.x * blockDim.x;
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n_ops; i += stride) {
        const u64 h = mix(i * 0x9e3779b97f4a7c15ULL + 12345);
        const u64 slot = h & mask16;  // 16-B granule index
        if (MODE == 0) {  // random 16-B load
            const uint4 v = *(const uint4*)(table + 2 * slot);
            acc += v.x ^ v.w;
        } else if (MODE == 1) {  // random 32-B load (aligned)
            const uint4* p = (const uint4*)(table + 2 * (slot & ~1ULL));
            const uint4 a = p[0], b = p[1];
            acc += a.x ^ b.w;
        } else if (MODE == 2) {  // random CAS 8 B (returning)
            acc += atomicCAS(table + 2 * slot, 0ULL, h | 1);
        } else if (MODE == 3) {  // random no-return add 8 B
            __hip_atomic_fetch_add(table + 2 * slot, 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (MODE == 4) {  // random 128-B store (one lane writes a whole line)
            uint4* p = (uint4*)(table + 2 * (slot & ~7ULL));
            const uint4 v = make_uint4((unsigned)h, (unsigned)(h >> 32), 1, 2);
#pragma unroll
            for (int w = 0; w < 8; w++) p[w] = v;
        } else if (MODE == 5) {  // coalesced stream read, 16 B per lane
            const uint4 v = *(const uint4*)(table + 2 * (i & mask16));
            acc += v.x;
        } else if (MODE == 6) {  // two independent random 16-B loads per op
            const u64 s2 = mix(h) & mask16;
            const uint4 v = *(const uint4*)(table + 2 * slot);
            const uint4 w = *(const uint4*)(table + 2 * s2);
            acc += v.x ^ w.y;
        }
    }
    if (acc == 0x123456789ULL) sink[0] = acc;
}

template <int MODE>
static double run(u64* table, u64 mask16, u64 n_ops, u64* sink) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k<MODE>, dim3(2048), dim3(256), 0, 0, table, mask16, n_ops / 8, sink);  // warm
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k<MODE>, dim3(8192), dim3(256), 0, 0, table, mask16, n_ops, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return n_ops / (ms * 1e-3) / 1e9;  // G ops/s
}

int main(int argc, char** argv) {
    const u64 sizes_mb[] = {16, 64, 256, 4096, 16384};
    const u64 n_ops = 1ULL << 27;
    u64* sink;
    CK(hipMalloc(&sink, 64));
    printf("%10s %10s %10s %10s %10s %10s %10s %10s  (G ops/s)\n", "table_MB", "rd16", "rd32", "cas8", "add8_nr",
           "st128", "stream16", "2xrd16");
    for (u64 mb : sizes_mb) {
        const u64 bytes = mb << 20;
        u64* table;
        CK(hipMalloc(&table, bytes));
        CK(hipMemset(table, 0, bytes));
        const u64 mask16 = bytes / 16 - 1;
        const double r0 = run<0>(table, mask16, n_ops, sink);
        const double r1 = run<1>(table, mask16, n_ops, sink);
        const double r2 = run<2>(table, mask16, n_ops, sink);
        const double r3 = run<3>(table, mask16, n_ops, sink);
        const double r4 = run<4>(table, mask16, n_ops / 4, sink);
        const double r5 = run<5>(table, mask16, n_ops, sink);
        const double r6 = run<6>(table, mask16, n_ops, sink);
        printf("%10llu %10.2f %10.2f %10.2f %10.2f %10.2f %10.2f %10.2f\n", mb, r0, r1, r2, r3, r4, r5, r6);
        CK(hipFree(table));
    }
    return 0;
}
