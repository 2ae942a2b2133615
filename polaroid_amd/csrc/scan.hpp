// Device-wide exclusive scan (reduce -> scan of block totals -> apply) and
// a block-level exclusive scan helper, shared by join.hip and sort.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

namespace plgpu {
namespace {  // internal linkage: included by several translation units

// Exclusive scan of n u64 values: out[i] = sum(in[0..i)), out[n] = total.
constexpr int kScanThreads = 256;
constexpr int kScanPer = 16;  // values per thread per block chunk
constexpr int64_t kScanChunk = (int64_t)kScanThreads * kScanPer;

__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t* wsum, uint64_t& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint64_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint64_t base = 0;
    total = 0;
    const int nw = blockDim.x >> 6;
    for (int w = 0; w < nw; ++w) {
        if (w < wid) base += wsum[w];
        total += wsum[w];
    }
    __syncthreads();
    return base + x - v;
}

template <typename T>
__global__ __launch_bounds__(kScanThreads) void scan_reduce_kernel(const T* __restrict__ in, int64_t n,
                                                                   uint64_t* __restrict__ part) {
    __shared__ uint64_t wsum[kScanThreads / 64];
    const int64_t base = (int64_t)blockIdx.x * kScanChunk;
    uint64_t s = 0;
    for (int k = 0; k < kScanPer; ++k) {
        const int64_t i = base + (int64_t)k * kScanThreads + threadIdx.x;
        if (i < n) s += (uint64_t)in[i];
    }
    uint64_t total;
    (void)block_excl_scan(s, wsum, total);
    if (threadIdx.x == 0) part[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void scan_parts_kernel(uint64_t* __restrict__ part, int64_t nparts,
                                                          uint64_t* __restrict__ total_out) {
    __shared__ uint64_t wsum[16];
    const int64_t per = (nparts + 1023) / 1024;
    const int64_t lo = threadIdx.x * per;
    const int64_t hi = lo + per < nparts ? lo + per : nparts;
    uint64_t s = 0;
    for (int64_t i = lo; i < hi; ++i) s += part[i];
    uint64_t total;
    uint64_t run = block_excl_scan(s, wsum, total);
    for (int64_t i = lo; i < hi; ++i) {
        const uint64_t v = part[i];
        part[i] = run;
        run += v;
    }
    if (threadIdx.x == 0) *total_out = total;
}

template <typename T, typename O = uint64_t>
__global__ __launch_bounds__(kScanThreads) void scan_apply_kernel(const T* in, int64_t n,
                                                                  const uint64_t* __restrict__ part, O* out) {
    __shared__ uint64_t wsum[kScanThreads / 64];
    // thread owns kScanPer consecutive values so the chunk scans in order
    const int64_t base = (int64_t)blockIdx.x * kScanChunk + (int64_t)threadIdx.x * kScanPer;
    uint64_t v[kScanPer];
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        const int64_t i = base + k;
        v[k] = i < n ? (uint64_t)in[i] : 0;
        s += v[k];
    }
    uint64_t total;
    uint64_t run = block_excl_scan(s, wsum, total) + part[blockIdx.x];
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
        const int64_t i = base + k;
        if (i < n) out[i] = (O)run;
        run += v[k];
    }
}

// out: n + 1 u64 (out[n] = total).  part: scratch of ceil(n / chunk) + 1.
template <typename T>
static hipError_t scan_exclusive(const T* in, int64_t n, uint64_t* out, uint64_t* part, hipStream_t s) {
    const int64_t nb = std::max<int64_t>(1, (n + kScanChunk - 1) / kScanChunk);
    scan_reduce_kernel<T><<<(unsigned)nb, kScanThreads, 0, s>>>(in, n, part);
    scan_parts_kernel<<<1, 1024, 0, s>>>(part, nb, out + n);
    scan_apply_kernel<T><<<(unsigned)nb, kScanThreads, 0, s>>>(in, n, part, out);
    return hipGetLastError();
}

// In-place exclusive scan of n u32 values whose total stays below 2^32 (the
// sort's digit counts: n < 2^32 rows): cnt[i] = sum(cnt[0..i)); the total
// lands in part[nb].  part: scratch of ceil(n / chunk) + 1.
static hipError_t scan_exclusive32_inplace(uint32_t* cnt, int64_t n, uint64_t* part, hipStream_t s) {
    const int64_t nb = std::max<int64_t>(1, (n + kScanChunk - 1) / kScanChunk);
    scan_reduce_kernel<uint32_t><<<(unsigned)nb, kScanThreads, 0, s>>>(cnt, n, part);
    scan_parts_kernel<<<1, 1024, 0, s>>>(part, nb, part + nb);
    scan_apply_kernel<uint32_t, uint32_t><<<(unsigned)nb, kScanThreads, 0, s>>>(cnt, n, part, cnt);
    return hipGetLastError();
}

}  // namespace
}  // namespace plgpu
