// Row shuffles for the multi-GPU operators: hash partitioning of a frame's
// rows by key, packing the partitioned rows into flat send buffers, and
// re-packing received byte masks into Arrow bitmaps.
//
// Reference (paths under /root/reference/crates):
//   polars-utils/src/hashing.rs:101 HashPartitioner::hash_to_partition (a
//     multiply-high of the key hash by the partition count) and :113
//     null_partition (nulls go to partition 0);
//   polars-stream/src/nodes/joins/equi_join.rs:445 BuildState::
//     partition_and_sink and :740 ProbeState::partition_and_probe (both
//     join sides are split by that partitioner, and partition p of the build
//     side only ever meets partition p of the probe side);
//   polars-stream/src/nodes/group_by.rs:509 (the group-by's use of it).
// Here a partition is a GPU: rows are routed to rank hash(key) * world >> 64
// and exchanged with one RCCL all-to-all per buffer (polaroid_amd/
// distributed.py).
//
// MI355X design:
//   count   - one wave owns 1024 consecutive rows (a "wave tile"), counts
//             its rows per destination in LDS;
//   scan    - device-wide exclusive scan of the [partition][wave tile] count
//             matrix gives every wave tile its output base per partition;
//   scatter - the wave re-reads its rows and ranks them per destination with
//             peer masks from log2(P) ballots (no atomics, no barriers), so
//             the permutation is stable: partition-major, row order within
//             a partition, as the reference's partitioner keeps morsel order;
//   pack    - values gathered by the permutation into caller-owned buffers
//             (torch tensors handed to RCCL), validity and Boolean values as
//             one byte per row so every per-rank segment starts on a byte.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "plgpu_internal.hpp"
#include "scan.hpp"
#include "tuplehash.hpp"

namespace plgpu {

constexpr int kShThreads = 256;
constexpr int kShWaveRows = 1024;  // rows per wave tile
constexpr int kShWaves = kShThreads / 64;
constexpr int kShMaxParts = 1024;
// fixed seed: every rank must route a key to the same partition
constexpr uint64_t kShSeed = 0x5851F42D4C957F2Dull;

// Destination of row r: [0, nparts), or nparts for a row that is dropped
// (a key tuple holding a null when nulls do not join); with nulls joining,
// such tuples go to partition 0 (hashing.rs:113 null_partition).
__device__ __forceinline__ uint32_t sh_dest(const MkKeys& k, int64_t r, uint32_t nparts, bool drop_nulls) {
    if (mk_any_null(k, r)) return drop_nulls ? nparts : 0u;
    const uint64_t h = mk_row_hash(k, r, kShSeed);
    return (uint32_t)__umul64hi(h, (uint64_t)nparts);
}

// counts[p * nwt + wt] = rows of wave tile wt routed to partition p.
__global__ __launch_bounds__(kShThreads) void sh_count_kernel(MkKeys k, int64_t n, uint32_t nparts, bool drop_nulls,
                                                              int64_t nwt, uint32_t* __restrict__ counts) {
    extern __shared__ uint32_t sh_cnt[];  // [kShWaves][nparts]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t* cnt = sh_cnt + w * nparts;
    for (int64_t wt0 = (int64_t)blockIdx.x * kShWaves; wt0 < nwt; wt0 += (int64_t)gridDim.x * kShWaves) {
        const int64_t wt = wt0 + w;
        for (uint32_t p = lane; p < nparts; p += 64) cnt[p] = 0;
        __builtin_amdgcn_wave_barrier();
        if (wt < nwt) {
            for (int i = 0; i < kShWaveRows / 64; ++i) {
                const int64_t r = wt * kShWaveRows + i * 64 + lane;
                if (r < n) {
                    const uint32_t d = sh_dest(k, r, nparts, drop_nulls);
                    if (d < nparts) atomicAdd(&cnt[d], 1u);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(0);
        if (wt < nwt)
            for (uint32_t p = lane; p < nparts; p += 64) counts[(int64_t)p * nwt + wt] = cnt[p];
        __builtin_amdgcn_wave_barrier();
    }
}

// perm[off[d * nwt + wt] + rank] = r, rank = the row's position among the
// wave tile's rows of destination d (stable).
__global__ __launch_bounds__(kShThreads) void sh_scatter_kernel(MkKeys k, int64_t n, uint32_t nparts, int dbits,
                                                                bool drop_nulls, int64_t nwt,
                                                                const uint64_t* __restrict__ off,
                                                                uint32_t* __restrict__ perm) {
    extern __shared__ uint32_t sh_run[];  // [kShWaves][nparts]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t* run = sh_run + w * nparts;
    const uint64_t lt = (1ull << lane) - 1;
    for (int64_t wt0 = (int64_t)blockIdx.x * kShWaves; wt0 < nwt; wt0 += (int64_t)gridDim.x * kShWaves) {
        const int64_t wt = wt0 + w;
        if (wt >= nwt) continue;  // wave-uniform; no block barriers below
        for (uint32_t p = lane; p < nparts; p += 64) run[p] = (uint32_t)off[(int64_t)p * nwt + wt];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(0);
        for (int i = 0; i < kShWaveRows / 64; ++i) {
            const int64_t r = wt * kShWaveRows + i * 64 + lane;
            const bool in = r < n;
            const uint32_t d = in ? sh_dest(k, r, nparts, drop_nulls) : nparts;
            // peers: lanes of this wave with the same destination
            uint64_t peers = __ballot(in);
            for (int b = 0; b < dbits; ++b) {
                const uint64_t bb = __ballot((d >> b) & 1u);
                peers &= ((d >> b) & 1u) ? bb : ~bb;
            }
            const bool live = in && d < nparts;
            const uint32_t base = live ? run[d] : 0u;
            __builtin_amdgcn_wave_barrier();
            if (live) {
                perm[base + (uint32_t)__popcll(peers & lt)] = (uint32_t)r;
                if ((peers & lt) == 0) run[d] = base + (uint32_t)__popcll(peers);
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}

__global__ void sh_totals_kernel(const uint64_t* __restrict__ off, uint32_t nparts, int64_t nwt,
                                 int64_t* __restrict__ totals) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < nparts; p += gridDim.x * blockDim.x)
        totals[p] = (int64_t)(off[(int64_t)(p + 1) * nwt] - off[(int64_t)p * nwt]);
}

// dst[o] = values[idx[o]] (idx == nullptr: identity); Boolean values and
// validity as one byte per row.
template <int EB>
__global__ __launch_bounds__(256) void sh_gather_kernel(DevCol c, const uint32_t* __restrict__ idx, int64_t n,
                                                        void* __restrict__ dst, uint8_t* __restrict__ dvalid) {
    for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < n; o += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = idx ? (int64_t)idx[o] : o;
        if (EB == 8) ((uint64_t*)dst)[o] = ((const uint64_t*)c.values)[c.offset + r];
        else if (EB == 4) ((uint32_t*)dst)[o] = ((const uint32_t*)c.values)[c.offset + r];
        else if (EB == 2) ((uint16_t*)dst)[o] = ((const uint16_t*)c.values)[c.offset + r];
        else ((uint8_t*)dst)[o] = (uint8_t)dev_load(c, r);  // 1-byte ints, Booleans as 0 / 1
        if (dvalid) dvalid[o] = dev_valid(c, r) ? 1 : 0;
    }
}

// bytes -> LSB-first bitmap (one ballot per 64 rows), zero bytes counted.
__global__ __launch_bounds__(256) void sh_pack_bits_kernel(const uint8_t* __restrict__ bytes, int64_t n,
                                                           uint64_t* __restrict__ bits,
                                                           unsigned long long* __restrict__ zeros) {
    uint32_t z = 0;
    for (int64_t r0 = (int64_t)blockIdx.x * blockDim.x; r0 < n; r0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = r0 + threadIdx.x;
        const bool in = r < n;
        const bool v = in && bytes[r] != 0;
        z += (in && !v) ? 1u : 0u;
        const uint64_t b = __ballot(v);
        const int64_t w0 = r - (threadIdx.x & 63);
        if ((threadIdx.x & 63) == 0 && w0 < n) bits[w0 >> 6] = b;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) z += __shfl_xor(z, o, 64);
    if ((threadIdx.x & 63) == 0 && z) atomicAdd(zeros, (unsigned long long)z);
}

static int num_cus_sh() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        hipDeviceProp_t prop;
        n = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
                ? prop.multiProcessorCount
                : 256;
    }
    return n;
}

static DevCol sh_dev(const plgpu_column& c) {
    DevCol d;
    std::memset(&d, 0, sizeof d);
    d.dtype = c.dtype;
    d.offset = c.offset;
    d.values = c.values;
    d.validity = c.validity;
    d.data = c.data;  // PLGPU_STR: the bytes (hashed, mk_row_hash)
    return d;
}

}  // namespace plgpu

using namespace plgpu;

PLGPU_API int plgpu_hash_partition(const plgpu_column* keys, int32_t nkeys, int32_t nparts, int32_t nulls_equal,
                                   plgpu_column* out_perm, int64_t* out_counts, void* stream) {
    hipStream_t s = as_stream(stream);
    if (keys == nullptr || out_perm == nullptr || out_counts == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    if (nkeys < 1 || nkeys > kMaxKeys) return fail(PLGPU_ERR_INVALID, "number of partition keys must be 1..8");
    if (nparts < 1 || nparts > kShMaxParts) return fail(PLGPU_ERR_INVALID, "number of partitions must be 1..1024");
    std::memset(out_perm, 0, sizeof *out_perm);
    MkKeys k;
    std::memset(&k, 0, sizeof k);
    k.n = nkeys;
    const int64_t n = keys[0].length;
    for (int i = 0; i < nkeys; ++i) {
        const int32_t dt = keys[i].dtype;
        if (!dtype_is_int(dt) && !dtype_is_float(dt) && dt != PLGPU_BOOL && dt != PLGPU_STR)
            return fail(PLGPU_ERR_SCHEMA, "partition keys must be integer, float, Boolean or String columns");
        if (keys[i].length != n) return fail(PLGPU_ERR_SHAPE, "partition key columns must have equal lengths");
        k.c[i] = sh_dev(keys[i]);
    }
    if (n >= 0xFFFFFFFFll) return fail(PLGPU_ERR_CAPACITY, "partition input exceeds the u32 index space");
    const bool drop = nulls_equal == 0;
    const uint32_t P = (uint32_t)nparts;
    int dbits = 0;
    while ((1u << dbits) < P + 1) ++dbits;  // destination codes 0..P (P = dropped)
    const int64_t nwt = std::max<int64_t>(1, (n + kShWaveRows - 1) / kShWaveRows);
    const int64_t ncnt = (int64_t)P * nwt;
    uint32_t* counts = nullptr;
    uint64_t* off = nullptr;
    uint64_t* part = nullptr;
    int64_t* totals = nullptr;
    int rc = dev_alloc((void**)&counts, ncnt * 4, s);
    if (!rc) rc = dev_alloc((void**)&off, (ncnt + 1) * 8, s);
    if (!rc) rc = dev_alloc((void**)&part, ((ncnt + kScanChunk - 1) / kScanChunk + 1) * 8, s);
    if (!rc) rc = dev_alloc((void**)&totals, (int64_t)P * 8, s);
    const size_t lds = (size_t)kShWaves * P * 4;
    const int g = (int)std::min<int64_t>((nwt + kShWaves - 1) / kShWaves, (int64_t)num_cus_sh() * 8);
    int64_t total = 0;
    if (!rc) {
        sh_count_kernel<<<g, kShThreads, lds, s>>>(k, n, P, drop, nwt, counts);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = scan_exclusive<uint32_t>(counts, ncnt, off, part, s);
        if (e == hipSuccess) {
            sh_totals_kernel<<<(P + 255) / 256, 256, 0, s>>>(off, P, nwt, totals);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(out_counts, totals, (size_t)P * 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "hash partition count");
    }
    if (!rc) {
        for (uint32_t p = 0; p < P; ++p) total += out_counts[p];
        rc = make_owned_column(out_perm, PLGPU_U32, total, false, s);
    }
    if (!rc && total > 0) {
        sh_scatter_kernel<<<g, kShThreads, lds, s>>>(k, n, P, dbits, drop, nwt, off, (uint32_t*)out_perm->values);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "hash partition scatter");
    }
    dev_free(counts, s);
    dev_free(off, s);
    dev_free(part, s);
    dev_free(totals, s);
    if (rc) plgpu_column_release(out_perm);
    return rc;
}

PLGPU_API int plgpu_gather_rows(const plgpu_column* cols, int32_t ncols, const plgpu_column* idx,
                                void* const* dst_values, uint8_t* const* dst_valid, void* stream) {
    hipStream_t s = as_stream(stream);
    if (ncols < 0 || (ncols > 0 && (cols == nullptr || dst_values == nullptr)))
        return fail(PLGPU_ERR_INVALID, "NULL argument");
    const uint32_t* ix = nullptr;
    int64_t n = ncols > 0 ? cols[0].length : 0;
    if (idx != nullptr) {
        if (idx->dtype != PLGPU_U32 || idx->validity != nullptr)
            return fail(PLGPU_ERR_SCHEMA, "row indices must be a UInt32 column without nulls");
        ix = (const uint32_t*)idx->values + idx->offset;
        n = idx->length;
    }
    for (int i = 0; i < ncols; ++i) {
        if (idx == nullptr && cols[i].length != n) return fail(PLGPU_ERR_SHAPE, "columns must have equal lengths");
        if (n > 0 && dst_values[i] == nullptr) return fail(PLGPU_ERR_INVALID, "NULL destination buffer");
    }
    if (n == 0) return PLGPU_OK;
    const int g = (int)std::min<int64_t>((n + 255) / 256, (int64_t)num_cus_sh() * 16);
    for (int i = 0; i < ncols; ++i) {
        const DevCol c = sh_dev(cols[i]);
        uint8_t* dv = dst_valid ? dst_valid[i] : nullptr;
        const int eb = cols[i].dtype == PLGPU_BOOL ? 1 : dtype_bytes(cols[i].dtype);
        switch (eb) {
        case 8: sh_gather_kernel<8><<<g, 256, 0, s>>>(c, ix, n, dst_values[i], dv); break;
        case 4: sh_gather_kernel<4><<<g, 256, 0, s>>>(c, ix, n, dst_values[i], dv); break;
        case 2: sh_gather_kernel<2><<<g, 256, 0, s>>>(c, ix, n, dst_values[i], dv); break;
        case 1: sh_gather_kernel<1><<<g, 256, 0, s>>>(c, ix, n, dst_values[i], dv); break;
        default: return fail(PLGPU_ERR_SCHEMA, "unsupported column dtype");
        }
    }
    PLGPU_HIP(hipGetLastError());
    PLGPU_HIP(hipStreamSynchronize(s));
    return PLGPU_OK;
}

PLGPU_API int plgpu_pack_bits(const uint8_t* bytes, int64_t n, uint8_t* out_bits, int64_t* out_zero_count,
                              void* stream) {
    hipStream_t s = as_stream(stream);
    if (n < 0) return fail(PLGPU_ERR_INVALID, "negative length");
    if (n > 0 && (bytes == nullptr || out_bits == nullptr)) return fail(PLGPU_ERR_INVALID, "NULL argument");
    unsigned long long* z = nullptr;
    int rc = dev_alloc((void**)&z, 8, s);
    if (rc) return rc;
    unsigned long long hz = 0;
    hipError_t e = hipMemsetAsync(z, 0, 8, s);
    if (e == hipSuccess && n > 0) {
        const int g = (int)std::min<int64_t>((n + 255) / 256, (int64_t)num_cus_sh() * 16);
        sh_pack_bits_kernel<<<g, 256, 0, s>>>(bytes, n, (uint64_t*)out_bits, z);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(&hz, z, 8, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    dev_free(z, s);
    if (e != hipSuccess) return hip_fail(e, "pack bits");
    if (out_zero_count) *out_zero_count = (int64_t)hz;
    return PLGPU_OK;
}
