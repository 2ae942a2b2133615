// Micro-benchmark: random reads of G bytes per probe from a table of T bytes,
// the access shape of a hash-join probe.  G = 8 (one lane, one 8-byte load),
// 64 (4 lanes x 16 B of one aligned 64-B bucket) or 128 (8 lanes x 16 B of a
// 128-B bucket).  Prints ms and probes/s per variant.  `xcd` rows: the table
// is split into 8 slices and workgroup b reads only slice b % 8 (under the
// round-robin dispatch of workgroups over the 8 XCDs, each slice is read by
// one XCD, so a slice <= 4 MiB can stay in that XCD's L2: the access shape
// of an XCD-partitioned probe).
//   hipcc -O3 --offload-arch=gfx950 tools/randread_bench.hip -o tools/_randread
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

// LANES lanes cooperate on one probe; each reads 16 B (LANES = 1: 8 B).
template <int LANES, int UNROLL, bool XCD = false>
__global__ __launch_bounds__(256) void probe_kernel(const uint4* __restrict__ tab, uint64_t nbuckets, int64_t nprobe,
                                                    uint64_t* __restrict__ out) {
    const uint64_t slice = XCD ? nbuckets / 8 : nbuckets;
    const uint64_t base = XCD ? (uint64_t)(blockIdx.x % 8) * slice : 0;
    const int lane = threadIdx.x % LANES;
    const int64_t groups = (int64_t)gridDim.x * blockDim.x / LANES;
    int64_t g = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / LANES;
    uint64_t acc = 0;
    for (int64_t p0 = g * UNROLL; p0 < nprobe; p0 += groups * UNROLL) {
        uint64_t v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const int64_t p = p0 + u;
            const uint64_t b = base + mix((uint64_t)p) % slice;
            if (LANES == 1) {
                v[u] = p < nprobe ? ((const uint64_t*)tab)[b] : 0;
            } else {
                const uint4 x = p < nprobe ? tab[b * LANES + lane] : make_uint4(0, 0, 0, 0);
                v[u] = x.x ^ x.z;
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc += v[u];
    }
    if (acc == 0x1234567) out[0] = acc;
}

template <int LANES, int UNROLL, bool XCD = false>
float run(const uint4* tab, size_t tbytes, int64_t nprobe, uint64_t* out, int grid) {
    const uint64_t bucket_bytes = LANES == 1 ? 8 : 16 * LANES;
    const uint64_t nb = tbytes / bucket_bytes;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    probe_kernel<LANES, UNROLL, XCD><<<grid, 256>>>(tab, nb, nprobe, out);
    hipEventRecord(a);
    for (int i = 0; i < 3; ++i) probe_kernel<LANES, UNROLL, XCD><<<grid, 256>>>(tab, nb, nprobe, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 3;
}

int main(int argc, char** argv) {
    const int64_t nprobe = argc > 1 ? atoll(argv[1]) : 1000000000ll;
    const size_t sizes[] = {size_t(16) << 20, size_t(128) << 20, size_t(256) << 20, size_t(512) << 20,
                            size_t(2) << 30};
    uint4* tab;
    uint64_t* out;
    hipMalloc(&tab, sizes[4]);
    hipMalloc(&out, 64);
    hipMemset(tab, 1, sizes[4]);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (size_t tb : sizes) {
        for (int gm : {8, 32}) {
            const int grid = cus * gm;
            float m8 = run<1, 16>(tab, tb, nprobe, out, grid);
            float m64 = run<4, 8>(tab, tb, nprobe, out, grid);
            float m128 = run<8, 8>(tab, tb, nprobe, out, grid);
            printf("table %5zu MiB grid %5d: 8B %7.2f ms (%.1f Gprobe/s) | 64B %7.2f ms (%.1f) | 128B %7.2f ms (%.1f)\n",
                   tb >> 20, grid, m8, nprobe / m8 / 1e6, m64, nprobe / m64 / 1e6, m128, nprobe / m128 / 1e6);
            fflush(stdout);
        }
    }
    // XCD-sliced tables: 8 slices of 0.5 .. 8 MiB
    for (size_t tb : {size_t(4) << 20, size_t(8) << 20, size_t(16) << 20, size_t(32) << 20, size_t(64) << 20}) {
        const int grid = cus * 8;
        float m8 = run<1, 16, true>(tab, tb, nprobe, out, grid);
        float m128 = run<8, 8, true>(tab, tb, nprobe, out, grid);
        printf("xcd table %5zu MiB (slice %4zu KiB) grid %5d: 8B %7.2f ms (%.1f Gprobe/s) | 128B %7.2f ms (%.1f)\n",
               tb >> 20, tb >> 13, grid, m8, nprobe / m8 / 1e6, m128, nprobe / m128 / 1e6);
        fflush(stdout);
    }
    return 0;
}
