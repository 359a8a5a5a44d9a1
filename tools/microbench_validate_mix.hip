// microbench_validate_mix.hip — the memory-access mix of tb_transfers_validate, without its logic
// (tooling, not product): the achievable time of one C2 pass's worth of accesses on MI355X, so the
// kernel can be priced against what the hardware does for THIS pattern, not only
// against the streaming HBM peak.
//
// Per transfer (one lane, 4,193,280 lanes = one 512-prepare pass):
//   stream  read the 128-B event, write the 128-B record and 42 B of per-event scratch (SoA)
//   probe   two random 32-B reads of a 64-MB account table (1M accounts at load 1/2)
//   cas     one random 8-B CAS into the transfer index (sized like the bench's)
// Each component alone and together; `sum` = the components' times added, `mix` = measured.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/microbench_validate_mix tools/microbench_validate_mix.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

typedef unsigned long long u64;
typedef unsigned int u32;

__device__ inline u64 mix(u64 x) {
    x ^= x >> 31;
    x *= 0x7fb5d329728ea185ULL;
    x ^= x >> 27;
    x *= 0x81dadef4bc2dd44dULL;
    x ^= x >> 33;
    return x;
}

struct Bufs {
    const uint4* events;  // n * 128 B
    uint4* records;       // n * 128 B
    u32* s4[4];           // info, dr, cr, rs
    unsigned short* s2;   // flags
    u64* s8[3];           // amt lo, amt hi, kid
    const uint4* accounts;  // account rows, 32 B each
    u64 acct_mask;          // rows - 1
    u64* index;             // 8-B entries
    u64 index_mask;
    u64 n;
    u64* sink;
};

enum : u32 { STREAM = 1, PROBE = 2, CAS = 4 };

template <u32 M>
__global__ __launch_bounds__(256) void k(Bufs B) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i >= B.n) return;
    u64 acc = 0;
    uint4 ev[8];
    const u64 h = mix(i * 0x9e3779b97f4a7c15ULL + 7);
    if (M & STREAM) {
#pragma unroll
        for (int w = 0; w < 8; w++) ev[w] = B.events[8 * i + w];
        acc ^= ev[0].x ^ ev[7].w;
    }
    if (M & PROBE) {
        const u64 d = mix(h ^ 1) & B.acct_mask, c = mix(h ^ 2) & B.acct_mask;
        const uint4 a0 = B.accounts[2 * d], a1 = B.accounts[2 * d + 1];
        const uint4 b0 = B.accounts[2 * c], b1 = B.accounts[2 * c + 1];
        acc ^= a0.x ^ a1.w ^ b0.y ^ b1.z;
    }
    if (M & CAS) {
        acc ^= atomicCAS(B.index + (h & B.index_mask), 0ULL, i + 1);
    }
    if (M & STREAM) {
#pragma unroll
        for (int w = 0; w < 8; w++) B.records[8 * i + w] = ev[w];
        B.s4[0][i] = (u32)acc;
        B.s4[1][i] = (u32)h;
        B.s4[2][i] = (u32)(h >> 8);
        B.s4[3][i] = (u32)(h >> 16);
        B.s2[i] = (unsigned short)h;
        B.s8[0][i] = h;
        B.s8[1][i] = 0;
        B.s8[2][i] = acc;
    } else if (acc == 0x123456789ULL) {
        B.sink[0] = acc;
    }
}

template <u32 M>
static float run(Bufs B, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const dim3 grid((unsigned)((B.n + 255) / 256));
    hipLaunchKernelGGL(k<M>, grid, dim3(256), 0, 0, B);
    CK(hipDeviceSynchronize());
    float total = 0;
    for (int r = 0; r < reps; r++) {
        CK(hipMemsetAsync(B.index, 0, (B.index_mask + 1) * 8, 0));  // every CAS finds its slot empty
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k<M>, grid, dim3(256), 0, 0, B);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        total += ms;
    }
    return total / reps;
}

int main(int argc, char** argv) {
    const u64 n = 4193280;
    const u64 index_mb = argc > 1 ? strtoull(argv[1], nullptr, 10) : 4096;
    Bufs B = {};
    B.n = n;
    void* p;
    CK(hipMalloc(&p, n * 128));
    CK(hipMemset(p, 1, n * 128));
    B.events = (const uint4*)p;
    CK(hipMalloc(&p, n * 128));
    B.records = (uint4*)p;
    for (int k = 0; k < 4; k++) CK(hipMalloc((void**)&B.s4[k], n * 4));
    CK(hipMalloc((void**)&B.s2, n * 2));
    for (int k = 0; k < 3; k++) CK(hipMalloc((void**)&B.s8[k], n * 8));
    const u64 rows = 1ULL << 21;
    CK(hipMalloc(&p, rows * 32));
    CK(hipMemset(p, 2, rows * 32));
    B.accounts = (const uint4*)p;
    B.acct_mask = rows - 1;
    const u64 entries = (index_mb << 20) / 8;
    CK(hipMalloc((void**)&B.index, entries * 8));
    B.index_mask = entries - 1;
    CK(hipMalloc((void**)&B.sink, 8));

    const int reps = 10;
    const float ts = run<STREAM>(B, reps), tp = run<PROBE>(B, reps), tc = run<CAS>(B, reps);
    const float tsp = run<STREAM | PROBE>(B, reps), tsc = run<STREAM | CAS>(B, reps), tpc = run<PROBE | CAS>(B, reps);
    const float tall = run<STREAM | PROBE | CAS>(B, reps);
    printf("transfers %llu, account table 64 MB, index %llu MB (ms per pass)\n", n, index_mb);
    printf("stream (128 B in, 128 B + 42 B out)  %.4f  (%.0f GB/s)\n", ts, n * 298.0 / ts / 1e6);
    printf("probe  (2 random 32-B reads)          %.4f  (%.1f G reads/s)\n", tp, 2.0 * n / tp / 1e6);
    printf("cas    (1 random 8-B CAS)             %.4f  (%.1f G CAS/s)\n", tc, n / tc / 1e6);
    printf("stream+probe %.4f  stream+cas %.4f  probe+cas %.4f\n", tsp, tsc, tpc);
    printf("mix (all three) %.4f   sum of parts %.4f   max of parts %.4f\n", tall, ts + tp + tc,
           ts > tp ? (ts > tc ? ts : tc) : (tp > tc ? tp : tc));
    return 0;
}
