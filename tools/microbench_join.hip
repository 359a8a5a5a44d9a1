// microbench_join.hip — north-star (b)'s sort + merge-join for the transfer-id exists check,
// priced against the engine's hash-index claim on MI355X (tooling, not product).
//
// One 512-prepare C2 pass: N = 4,166,667 new transfer ids (64-bit id hashes, 0.1 % same-pass
// duplicates) against an index holding R = 100M ids (the end of a 100M-transfer step).
//   cas        the engine's claim: one random 8-B CAS per id into a 2^28-entry (2-GB) hash index
//   sort       a hand-written device sort of the pass's (hash, event) pairs: one partition pass by
//              the top 12 hash bits (LDS histograms of 128 workgroups, a three-kernel scan, a scatter
//              ranked per workgroup so each workgroup's run of a bucket is contiguous), then every
//              bucket (~1K pairs) sorted in LDS (bitonic, 2048 slots)
//   dups       same-pass duplicates: adjacent equal hashes in sorted order
//   probe_sorted / probe_random
//              the sorted runs' exists filter: a blocked Bloom filter of the R ids (2^22 64-B
//              blocks = 256 MB, 4 bits per id in its block, ~20 bits per id), probed by the pass's
//              hashes in sorted order (block indices ascend: near-streaming) and in event order
//   append     the pass's sorted run (8-B hashes + 4-B positions) and its filter bits set in
//              sorted order — the inserts a sorted-run index makes instead of the CAS
// The exact lookup behind a filter hit (a binary search in a run's fence index) is not timed:
// at ~0.2 % false positives it is ~8K searches a pass.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mbj tools/microbench_join.hip && /tmp/mbj
#include <hip/hip_runtime.h>

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

__host__ __device__ inline u64 mix(u64 x) {
    x ^= x >> 31;
    x *= 0x7fb5d329728ea185ULL;
    x ^= x >> 27;
    x *= 0x81dadef4bc2dd44dULL;
    x ^= x >> 33;
    return x;
}

#define BUCKET_BITS 12
#define NBUCKETS (1u << BUCKET_BITS)
#define BUCKET_CAP 2048
#define FILTER_BLOCK_BITS 22

__global__ void gen_keys(u64* keys, u32* vals, u64 n, u64 seed, u64 dup_every) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 j = (dup_every && i % dup_every == dup_every - 1) ? i / 2 : i;  // a same-pass duplicate
        keys[i] = mix(j * 0x9e3779b97f4a7c15ULL + seed);
        vals[i] = (u32)i;
    }
}

__device__ inline void filter_bits(u64 h, u64* block, u64* bit) {
    *block = h >> (64 - FILTER_BLOCK_BITS);
    *bit = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) *bit |= 1ULL << ((h >> (6 * k)) & 63);
}

// The 4 bits of a hash sit in one 8-B word of its 64-B block (word chosen by more hash bits).
__global__ void filter_build(u64* filter, u64 n, u64 seed) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 h = mix((i + (1ULL << 40)) * 0x9e3779b97f4a7c15ULL + seed);
        u64 b, bit;
        filter_bits(h, &b, &bit);
        atomicOr(filter + b * 8 + ((h >> 24) & 7), bit);
    }
}

__global__ void cas_claim(u64* table, u64 mask, const u64* keys, u64 n, u32* out) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 h = keys[i];
        out[i] = (u32)atomicCAS(table + (h & mask), 0ULL, (h | 1) + i);
    }
}

__global__ void hist(const u64* keys, u64 n, u32* counts) {
    __shared__ u32 s[NBUCKETS];
    for (u32 k = threadIdx.x; k < NBUCKETS; k += blockDim.x) s[k] = 0;
    __syncthreads();
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        atomicAdd(&s[keys[i] >> (64 - BUCKET_BITS)], 1u);
    }
    __syncthreads();
    // per-workgroup counts: [bucket][workgroup], scanned bucket-major so each workgroup's run of a
    // bucket is contiguous
    for (u32 k = threadIdx.x; k < NBUCKETS; k += blockDim.x) counts[(u64)k * gridDim.x + blockIdx.x] = s[k];
}

// The exclusive scan of the [bucket][workgroup] counts in three short kernels: each bucket's total
// (one thread per bucket), the scan of the 4096 totals (one workgroup), each bucket's run rewritten.
__global__ void bucket_totals(const u32* counts, u32 nwg, u32* totals) {
    const u32 k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= NBUCKETS) return;
    u32 t = 0;
    for (u32 w = 0; w < nwg; w++) t += counts[(u64)k * nwg + w];
    totals[k] = t;
}

__global__ void scan_totals(u32* totals) {  // one workgroup of 1024, 4 buckets per thread
    __shared__ u32 s_part[1024];
    u32 v[4], sum = 0;
    for (u32 q = 0; q < 4; q++) {
        v[q] = totals[threadIdx.x * 4 + q];
        sum += v[q];
    }
    s_part[threadIdx.x] = sum;
    __syncthreads();
    for (u32 off = 1; off < 1024; off <<= 1) {
        const u32 x = threadIdx.x >= off ? s_part[threadIdx.x - off] : 0;
        __syncthreads();
        s_part[threadIdx.x] += x;
        __syncthreads();
    }
    u32 run = s_part[threadIdx.x] - sum;
    for (u32 q = 0; q < 4; q++) {
        totals[threadIdx.x * 4 + q] = run;
        run += v[q];
    }
}

__global__ void bucket_runs(u32* counts, u32 nwg, const u32* starts) {
    const u32 k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= NBUCKETS) return;
    u32 run = starts[k];
    for (u32 w = 0; w < nwg; w++) {
        const u32 c = counts[(u64)k * nwg + w];
        counts[(u64)k * nwg + w] = run;
        run += c;
    }
}

__global__ void scatter(const u64* keys, const u32* vals, u64 n, const u32* base, u64* okeys, u32* ovals) {
    __shared__ u32 s[NBUCKETS];
    for (u32 k = threadIdx.x; k < NBUCKETS; k += blockDim.x) s[k] = base[(u64)k * gridDim.x + blockIdx.x];
    __syncthreads();
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 key = keys[i];
        const u32 p = atomicAdd(&s[key >> (64 - BUCKET_BITS)], 1u);
        okeys[p] = key;
        ovals[p] = vals[i];
    }
}

// One workgroup per bucket: its pairs sorted in LDS (bitonic over 2048 slots, padding = ~0).
__global__ __launch_bounds__(1024) void bucket_sort(u64* keys, u32* vals, const u32* counts, u32 nwg, u64 n) {
    __shared__ u64 sk[BUCKET_CAP];
    __shared__ u32 sv[BUCKET_CAP];
    const u32 bkt = blockIdx.x;
    const u64 a = counts[(u64)bkt * nwg];
    const u64 b = bkt + 1 < NBUCKETS ? counts[(u64)(bkt + 1) * nwg] : n;
    const u32 m = (u32)(b - a);
    for (u32 t = threadIdx.x; t < BUCKET_CAP; t += blockDim.x) {
        sk[t] = t < m ? keys[a + t] : ~0ULL;
        sv[t] = t < m ? vals[a + t] : 0;
    }
    __syncthreads();
    for (u32 size = 2; size <= BUCKET_CAP; size <<= 1) {
        for (u32 stride = size >> 1; stride > 0; stride >>= 1) {
            for (u32 t = threadIdx.x; t < BUCKET_CAP / 2; t += blockDim.x) {
                const u32 lo = 2 * t - (t & (stride - 1));
                const u32 hi = lo + stride;
                const bool up = (lo & size) == 0;
                const u64 x = sk[lo], y = sk[hi];
                if ((x > y) == up) {
                    sk[lo] = y;
                    sk[hi] = x;
                    const u32 v = sv[lo];
                    sv[lo] = sv[hi];
                    sv[hi] = v;
                }
            }
            __syncthreads();
        }
    }
    for (u32 t = threadIdx.x; t < m; t += blockDim.x) {
        keys[a + t] = sk[t];
        vals[a + t] = sv[t];
    }
}

__global__ void dups(const u64* keys, u64 n, unsigned char* flag) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        flag[i] = (i > 0 && keys[i] == keys[i - 1]) || (i + 1 < n && keys[i] == keys[i + 1]);
    }
}

__global__ void probe(const u64* filter, const u64* keys, u64 n, unsigned char* out) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 h = keys[i];
        u64 b, bit;
        filter_bits(h, &b, &bit);
        out[i] = (filter[b * 8 + ((h >> 24) & 7)] & bit) == bit;
    }
}

__global__ void append(const u64* keys, const u32* vals, u64 n, u64* run_keys, u32* run_pos, u64* filter) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 h = keys[i];
        run_keys[i] = h;
        run_pos[i] = vals[i];
        u64 b, bit;
        filter_bits(h, &b, &bit);
        atomicOr(filter + b * 8 + ((h >> 24) & 7), bit);
    }
}

int main() {
    const u64 N = 4166667, R = 100000000;
    const u64 table_n = 1ULL << 28, filter_words = (1ULL << FILTER_BLOCK_BITS) * 8;
    const u32 grid = 2048, nwg = 128;
    u64 *keys, *keys2, *table, *filter, *run_keys;
    u32 *vals, *vals2, *counts, *totals, *run_pos, *cas_out;
    unsigned char *flag, *hit;
    CK(hipMalloc(&keys, N * 8));
    CK(hipMalloc(&keys2, N * 8));
    CK(hipMalloc(&vals, N * 4));
    CK(hipMalloc(&vals2, N * 4));
    CK(hipMalloc(&table, table_n * 8));
    CK(hipMalloc(&filter, filter_words * 8));
    CK(hipMalloc(&run_keys, N * 8));
    CK(hipMalloc(&run_pos, N * 4));
    CK(hipMalloc(&cas_out, N * 4));
    CK(hipMalloc(&counts, (u64)NBUCKETS * nwg * 4));
    CK(hipMalloc(&totals, NBUCKETS * 4));
    CK(hipMalloc(&flag, N));
    CK(hipMalloc(&hit, N));
    CK(hipMemset(filter, 0, filter_words * 8));
    hipLaunchKernelGGL(filter_build, dim3(4096), dim3(256), 0, 0, filter, R, 7);
    hipLaunchKernelGGL(gen_keys, dim3(grid), dim3(256), 0, 0, keys, vals, N, 11, 1000);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 10;
    double t_cas = 0, t_sort = 0, t_dups = 0, t_ps = 0, t_pr = 0, t_app = 0;
    for (int it = 0; it < iters + 1; it++) {
        float ms;
        CK(hipMemset(table, 0, table_n * 8));  // (an empty index: the CAS's cost without probe chains)
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(cas_claim, dim3(grid), dim3(256), 0, 0, table, table_n - 1, keys, N, cas_out);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it) t_cas += ms;

        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(hist, dim3(nwg), dim3(256), 0, 0, keys, N, counts);
        hipLaunchKernelGGL(bucket_totals, dim3(NBUCKETS / 256), dim3(256), 0, 0, counts, nwg, totals);
        hipLaunchKernelGGL(scan_totals, dim3(1), dim3(1024), 0, 0, totals);
        hipLaunchKernelGGL(bucket_runs, dim3(NBUCKETS / 256), dim3(256), 0, 0, counts, nwg, totals);
        hipLaunchKernelGGL(scatter, dim3(nwg), dim3(256), 0, 0, keys, vals, N, counts, keys2, vals2);
        hipLaunchKernelGGL(bucket_sort, dim3(NBUCKETS), dim3(1024), 0, 0, keys2, vals2, counts, nwg, N);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it) t_sort += ms;

        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(dups, dim3(grid), dim3(256), 0, 0, keys2, N, flag);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it) t_dups += ms;

        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(probe, dim3(grid), dim3(256), 0, 0, filter, keys2, N, hit);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it) t_ps += ms;

        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(probe, dim3(grid), dim3(256), 0, 0, filter, keys, N, hit);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it) t_pr += ms;

        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(append, dim3(grid), dim3(256), 0, 0, keys2, vals2, N, run_keys, run_pos, filter);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it) t_app += ms;
    }
    // Check the sort: ascending, and the duplicates found.
    u64* h = (u64*)malloc(N * 8);
    unsigned char* f = (unsigned char*)malloc(N);
    CK(hipMemcpy(h, keys2, N * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(f, flag, N, hipMemcpyDeviceToHost));
    u64 bad = 0, nd = 0;
    for (u64 i = 1; i < N; i++) bad += h[i] < h[i - 1];
    for (u64 i = 0; i < N; i++) nd += f[i];
    printf("{\"pass_ids\": %llu, \"index_ids\": %llu, \"ms\": {\"cas\": %.4f, \"sort\": %.4f, \"dups\": %.4f, "
           "\"probe_sorted\": %.4f, \"probe_random\": %.4f, \"append\": %.4f}, \"sort_join_total_ms\": %.4f, "
           "\"sorted_ok\": %s, \"dup_events\": %llu}\n",
           (unsigned long long)N, (unsigned long long)R, t_cas / iters, t_sort / iters, t_dups / iters, t_ps / iters,
           t_pr / iters, t_app / iters, (t_sort + t_dups + t_ps + t_app) / iters, bad ? "false" : "true",
           (unsigned long long)nd);
    return 0;
}
