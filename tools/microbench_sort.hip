// microbench_sort.hip — what a sort-merge join of a pass's account legs would cost on MI355X,
// against the hash probes tb_transfers_validate issues instead ("Why hash probes").
//
// A C2 pass of 512 prepares has T = 4,193,280 transfers = 2T legs; a sort-merge join orders the
// legs by account (key = the account's table slot, 20 bits for 1M accounts, or its 64-bit id hash),
// then reads each touched account once in key order.  This times rocPRIM's device radix sort of
// (key, leg index) pairs at those sizes, and the gather of one 32-B account row per leg in sorted
// order versus in random (hash-probe) order.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/microbench_sort tools/microbench_sort.hip
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

__global__ void fill_keys32(uint32_t* k, uint32_t* v, uint64_t n, uint32_t mask, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t x = (i + seed) * 0x9E3779B97F4A7C15ULL;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ULL;
    x ^= x >> 29;
    k[i] = (uint32_t)x & mask;
    v[i] = (uint32_t)i;
}
__global__ void fill_keys64(uint64_t* k, uint32_t* v, uint64_t n, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t x = (i + seed) * 0x9E3779B97F4A7C15ULL;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ULL;
    x ^= x >> 29;
    k[i] = x;
    v[i] = (uint32_t)i;
}
struct Row {
    uint64_t w[4];
};
// One 32-B row per leg, the key naming the row; the sum keeps the loads alive.
__global__ void gather(const uint32_t* keys, const Row* rows, uint64_t n, uint64_t* out) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t s = 0;
    if (i < n) {
        const Row r = rows[keys[i]];
        s = r.w[0] ^ r.w[1] ^ r.w[2] ^ r.w[3];
    }
    if (s == 0x123456789ULL) out[0] = s;
}

template <typename F>
static float time_ms(F f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < reps; r++) f();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms / reps;
}

int main() {
    const uint64_t T = 4193280, n = 2 * T;  // legs of one 512-prepare C2 pass
    const uint32_t slots = 1u << 21;        // 1M accounts at load 1/2
    uint32_t *k32, *k32o, *v, *vo;
    uint64_t *k64, *k64o, *sink;
    Row* rows;
    CK(hipMalloc(&k32, n * 4));
    CK(hipMalloc(&k32o, n * 4));
    CK(hipMalloc(&v, n * 4));
    CK(hipMalloc(&vo, n * 4));
    CK(hipMalloc(&k64, n * 8));
    CK(hipMalloc(&k64o, n * 8));
    CK(hipMalloc(&sink, 8));
    CK(hipMalloc(&rows, (uint64_t)slots * sizeof(Row)));
    CK(hipMemset(rows, 1, (uint64_t)slots * sizeof(Row)));
    const unsigned g = (unsigned)((n + 255) / 256);
    fill_keys32<<<g, 256>>>(k32, v, n, slots - 1, 1);
    fill_keys64<<<g, 256>>>(k64, v, n, 2);
    CK(hipDeviceSynchronize());

    size_t tmp_bytes = 0, t2 = 0;
    CK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, k64, k64o, v, vo, n, 0, 64));
    CK(rocprim::radix_sort_pairs(nullptr, t2, k32, k32o, v, vo, n, 0, 21));
    if (t2 > tmp_bytes) tmp_bytes = t2;
    void* tmp;
    CK(hipMalloc(&tmp, tmp_bytes));

    const int reps = 20;
    const float s21 = time_ms([&] { (void)rocprim::radix_sort_pairs(tmp, tmp_bytes, k32, k32o, v, vo, n, 0, 21); }, reps);
    const float s32 = time_ms([&] { (void)rocprim::radix_sort_pairs(tmp, tmp_bytes, k32, k32o, v, vo, n, 0, 32); }, reps);
    const float s64 = time_ms([&] { (void)rocprim::radix_sort_pairs(tmp, tmp_bytes, k64, k64o, v, vo, n, 0, 64); }, reps);
    const float g_rand = time_ms([&] { gather<<<g, 256>>>(k32, rows, n, sink); }, reps);
    const float g_sort = time_ms([&] { gather<<<g, 256>>>(k32o, rows, n, sink); }, reps);
    CK(hipDeviceSynchronize());
    printf("legs %llu (one 512-prepare C2 pass), account rows %u x 32 B\n", (unsigned long long)n, slots);
    printf("radix_sort_pairs  key 21 bit (table slot): %.4f ms  (%.2f G pairs/s)\n", s21, n / s21 / 1e6);
    printf("radix_sort_pairs  key 32 bit:              %.4f ms  (%.2f G pairs/s)\n", s32, n / s32 / 1e6);
    printf("radix_sort_pairs  key 64 bit (id hash):    %.4f ms  (%.2f G pairs/s)\n", s64, n / s64 / 1e6);
    printf("gather 32-B rows, random order (probe):    %.4f ms  (%.2f G rows/s)\n", g_rand, n / g_rand / 1e6);
    printf("gather 32-B rows, sorted order (join):     %.4f ms  (%.2f G rows/s)\n", g_sort, n / g_sort / 1e6);
    return 0;
}
