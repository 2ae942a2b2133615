// Stable LSD radix arg-sort of one column (the sort_by / arg_sort hot path).
//
// Reference (paths under /root/reference/crates):
//   polars-core/src/chunked_array/ops/sort/arg_sort.rs:7 sort_impl /
//     arg_sort: stable sort of (idx, value) pairs by TotalOrd
//     (polars-utils/src/total_ord.rs: NaN == NaN and greatest, -0.0 == 0.0),
//     descending by a reversed comparator (equal values keep their order),
//     nulls gathered first or last (SortOptions, options.rs:32);
//   DataFrame::sort -> arg_sort then take (gather.rs).
//
// MI355X design:
//   prep     - nulls are split off in order; keys become order-preserving
//              u64 codes (descending = complement), carried with u32 row ids;
//   bits     - one read of the codes gives their OR and AND, so bytes that
//              are constant over the column cost no pass;
//   per pass - upsweep (per-tile digit counts) -> device scan (digit-major)
//              -> downsweep: a tile of 4096 codes is ranked stably in LDS
//              (wave64 ballot peer masks per digit) and written out in
//              digit runs, so global writes are coalesced.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>

#include "plgpu_internal.hpp"
#include "scan.hpp"

namespace plgpu {

constexpr int kSrtThreads = 256;                  // upsweep / stats workgroups
constexpr int kSrtPer = 16;
constexpr int kSrtTile = kSrtThreads * kSrtPer;  // 4096 codes per tile

__device__ __forceinline__ uint64_t sort_code(const DevCol& c, int64_t r, bool descending) {
    uint64_t b = dev_load(c, r);
    uint64_t k;
    if (c.dtype == PLGPU_F64 || c.dtype == PLGPU_F32) {  // Float32 in register form (f64 bits)
        if ((b & 0x7fffffffffffffffull) == 0) b = 0;                      // -0.0 == 0.0
        else if ((b & 0x7fffffffffffffffull) > 0x7ff0000000000000ull) b = 0x7ff8000000000000ull;  // one NaN
        k = ord_f64(b);
    } else if (c.dtype == PLGPU_U8 || c.dtype == PLGPU_U16 || c.dtype == PLGPU_U32 || c.dtype == PLGPU_U64) {
        k = b;
    } else if (c.dtype == PLGPU_I8 || c.dtype == PLGPU_I16 || c.dtype == PLGPU_I32) {
        k = (uint64_t)((uint32_t)b ^ 0x80000000u);  // upper bytes constant: their passes are skipped
    } else {
        k = b ^ 0x8000000000000000ull;  // I64
    }
    return descending ? ~k : k;
}

// Per 1024-row block: valid-row counts (for the null split).
__global__ __launch_bounds__(256) void srt_count_valid_kernel(DevCol c, int64_t n, uint32_t* __restrict__ cnt) {
    __shared__ uint32_t s;
    const int64_t base = (int64_t)blockIdx.x * 1024;
    if (threadIdx.x == 0) s = 0;
    __syncthreads();
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
        const int64_t r = base + k * 256 + threadIdx.x;
        v += (r < n && dev_valid(c, r)) ? 1u : 0u;
    }
    atomicAdd(&s, v);
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = s;
}

// Codes + row ids of the valid rows (in row order) and the null row ids (in
// row order) -- block b's valid rows start at voff[b], its nulls at
// b*1024 - voff[b].
__global__ __launch_bounds__(256) void srt_prep_kernel(DevCol c, int64_t n, bool descending,
                                                       const uint64_t* __restrict__ voff, uint64_t* __restrict__ keys,
                                                       uint32_t* __restrict__ idx, uint32_t* __restrict__ nulls) {
    __shared__ uint32_t wv[4], wn[4];
    const int64_t base = (int64_t)blockIdx.x * 1024;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t vpos = voff[blockIdx.x];
    uint64_t npos = (uint64_t)base - vpos;
    for (int k = 0; k < 4; ++k) {
        const int64_t r = base + k * 256 + threadIdx.x;
        const bool in = r < n;
        const bool valid = in && dev_valid(c, r);
        const uint64_t bv = __ballot(valid), bn = __ballot(in && !valid);
        const uint64_t lt = (1ull << lane) - 1;
        if (lane == 0) {
            wv[wid] = (uint32_t)__popcll(bv);
            wn[wid] = (uint32_t)__popcll(bn);
        }
        __syncthreads();
        uint64_t pv = vpos, pn = npos;
        uint32_t tv = 0, tn = 0;
        for (int w = 0; w < 4; ++w) {
            if (w < wid) {
                pv += wv[w];
                pn += wn[w];
            }
            tv += wv[w];
            tn += wn[w];
        }
        if (valid) {
            const uint64_t p = pv + __popcll(bv & lt);
            keys[p] = sort_code(c, r, descending);
            idx[p] = (uint32_t)r;
        } else if (in) {
            nulls[pn + __popcll(bn & lt)] = (uint32_t)r;
        }
        vpos += tv;
        npos += tn;
        __syncthreads();
    }
}

__global__ void srt_codes_kernel(DevCol c, int64_t n, bool descending, uint64_t* __restrict__ keys,
                                 uint32_t* __restrict__ idx) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        keys[r] = sort_code(c, r, descending);
        if (idx) idx[r] = (uint32_t)r;
    }
}

// OR and AND of all codes in one read: a byte whose bits agree over the
// column ((OR ^ AND) byte == 0) is constant, and its pass is skipped.
__global__ __launch_bounds__(256) void srt_bits_kernel(const uint64_t* __restrict__ keys, int64_t n,
                                                       unsigned long long* __restrict__ bits) {
    uint64_t o = 0, a = ~0ull;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[i];
        o |= k;
        a &= k;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        o |= __shfl_xor(o, off, 64);
        a &= __shfl_xor(a, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicOr(&bits[0], (unsigned long long)o);
        atomicAnd(&bits[1], (unsigned long long)a);
    }
}

// Null-free column, first read: each 4096-row tile writes its codes, its
// OR / AND of them (reduced over the tiles by srt_tbits_kernel: constant
// bytes) and its byte-0 digit counts, digit-major like the upsweep's -- the
// first pass's upsweep whenever byte 0 varies.  Replaces codes + bits +
// first upsweep (three reads of the column) by one.
__global__ __launch_bounds__(kSrtThreads) void srt_codes_stats_kernel(DevCol c, int64_t n, bool descending,
                                                                      int64_t ntiles, uint64_t* __restrict__ keys,
                                                                      uint32_t* __restrict__ cnt,
                                                                      uint64_t* __restrict__ tbits) {
    __shared__ uint32_t h[256];
    __shared__ uint64_t wo[kSrtThreads / 64], wa[kSrtThreads / 64];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t tile = xcd_tile(blockIdx.x, ntiles);
    const int64_t base = tile * kSrtTile;
    uint64_t o = 0, a = ~0ull;
    uint64_t k[kSrtPer];
#pragma unroll
    for (int j = 0; j < kSrtPer; ++j) {
        const int64_t i = base + j * kSrtThreads + threadIdx.x;
        k[j] = i < n ? sort_code(c, i, descending) : 0;
    }
#pragma unroll
    for (int j = 0; j < kSrtPer; ++j) {
        const int64_t i = base + j * kSrtThreads + threadIdx.x;
        if (i < n) {
            keys[i] = k[j];
            o |= k[j];
            a &= k[j];
            atomicAdd(&h[k[j] & 0xFF], 1u);
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        o |= __shfl_xor(o, off, 64);
        a &= __shfl_xor(a, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        wo[threadIdx.x >> 6] = o;
        wa[threadIdx.x >> 6] = a;
    }
    __syncthreads();
    cnt[(int64_t)threadIdx.x * ntiles + tile] = h[threadIdx.x];
    if (threadIdx.x == 0) {
        for (int w = 1; w < kSrtThreads / 64; ++w) {
            o |= wo[w];
            a &= wa[w];
        }
        tbits[2 * tile] = o;
        tbits[2 * tile + 1] = a;
    }
}

__global__ __launch_bounds__(256) void srt_tbits_kernel(const uint64_t* __restrict__ tbits, int64_t nt,
                                                        unsigned long long* __restrict__ bits) {
    uint64_t o = 0, a = ~0ull;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nt; i += (int64_t)gridDim.x * blockDim.x) {
        o |= tbits[2 * i];
        a &= tbits[2 * i + 1];
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        o |= __shfl_xor(o, off, 64);
        a &= __shfl_xor(a, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicOr(&bits[0], (unsigned long long)o);
        atomicAnd(&bits[1], (unsigned long long)a);
    }
}

// Representations of the (code, row id) stream between passes:
//   SEP    - codes u64 + row ids u32 in two buffers (12 B per row);
//   PACKED - one u64 word (remaining code bits << 32 | row id) once the
//            code bits still to be sorted fit 32 bits (LSD: the bytes below
//            the current pass are never looked at again), 8 B per row;
//   IDX    - the last pass writes the row ids only (4 B per row).
// For 40-bit timestamps the traffic per pass drops from 24 to 16 B per row
// after the first pass, and the last pass writes 4 B instead of 12.
enum SrtOut { SRT_SEP = 0, SRT_PACK = 1, SRT_IDX = 2 };

// Upsweep: digit counts of every tile, digit-major (cnt[d * ntiles + t]).
// (A resident grid looping over the tiles, the next tile's keys loaded
// before this one's counts, measured no faster: 1.63 against 1.56 ms; the
// same loop made the downsweep slower, 3.9 -> 5.5-6.0 ms: not kept.)
// tpw tiles per workgroup (option srt_up_tiles; 1: one tile per workgroup,
// XCD-remapped): each tile's histogram is written on its own, the next
// tile's codes already in flight while this one's are counted.
__global__ __launch_bounds__(kSrtThreads) void srt_upsweep_kernel(const uint64_t* __restrict__ keys, int64_t n,
                                                                  int shift, int64_t ntiles,
                                                                  uint32_t* __restrict__ cnt, int tpw) {
    __shared__ uint32_t h[256];
    const int64_t nwg = (ntiles + tpw - 1) / tpw;
    const int64_t t0 = xcd_tile(blockIdx.x, nwg) * tpw;
    const int64_t t1 = t0 + tpw < ntiles ? t0 + tpw : ntiles;
    uint64_t v[kSrtPer];
    auto load = [&](int64_t tile) {
        const int64_t base = tile * kSrtTile;
#pragma unroll
        for (int k = 0; k < kSrtPer; ++k) {
            const int64_t i = base + k * kSrtThreads + threadIdx.x;
            v[k] = i < n ? __builtin_nontemporal_load(keys + i) : ~0ull;
        }
    };
    if (t0 < t1) load(t0);
    for (int64_t tile = t0; tile < t1; ++tile) {
        h[threadIdx.x] = 0;
        __syncthreads();
        const int64_t base = tile * kSrtTile;
        uint32_t d[kSrtPer];
        bool in[kSrtPer];
#pragma unroll
        for (int k = 0; k < kSrtPer; ++k) {
            d[k] = (uint32_t)(v[k] >> shift) & 0xFF;
            in[k] = base + k * kSrtThreads + threadIdx.x < n;
        }
        if (tile + 1 < t1) load(tile + 1);
#pragma unroll
        for (int k = 0; k < kSrtPer; ++k)
            if (in[k]) atomicAdd(&h[d[k]], 1u);
        __syncthreads();
        cnt[(int64_t)threadIdx.x * ntiles + tile] = h[threadIdx.x];
        __syncthreads();
    }
}

// Downsweep: stable scatter of one tile by the digit at `shift` (of the
// input representation).  Wave w ranks its own contiguous 1024 codes row by
// row (64 codes per row, peer masks from 8 ballots, per-wave digit counters
// in LDS -- no barriers), then one block-wide combine turns (wave, digit)
// counts into local positions; the tile is staged in LDS in digit order and
// written out in runs.  IN_P: input is PACKED.  OUT: SrtOut; a SEP -> PACK
// transition keeps (code >> cons) & kmask as the remaining code.  off: the
// scanned digit-major counts (u32, n < 2^32; scanned in place).  (A side
// array of the next pass's digit bytes, written here so the next upsweep
// reads 1 B instead of 8 per code, cut the upsweep 1.78 -> 0.38 ms but cost
// every downsweep 1.2 ms of scattered byte stores: not kept.)
// WPE: the occupancy the register allocation targets (waves per SIMD; 1 =
// the compiler's choice, 142 VGPRs for the packed passes: 3 workgroups per
// CU; 4 = 128 VGPRs with a few spilled words: 4 workgroups per CU, which the
// LDS allows), option srt_w4 (A/B)
template <bool IN_P, int OUT, int WPE = 1>
__global__ __launch_bounds__(kSrtThreads) __attribute__((amdgpu_waves_per_eu(WPE))) void srt_downsweep_kernel(const uint64_t* __restrict__ keys_in,
                                                                    const uint32_t* __restrict__ idx_in, int64_t n,
                                                                    int shift, int64_t ntiles,
                                                                    const uint32_t* __restrict__ off,
                                                                    uint64_t* __restrict__ keys_out,
                                                                    uint32_t* __restrict__ idx_out, int cons,
                                                                    uint64_t kmask) {
    constexpr int TH = kSrtThreads;
    constexpr int NW = TH / 64;
    constexpr int ROWS = kSrtTile / TH;  // rows of 64 per wave (16)
    __shared__ uint64_t skey[OUT == SRT_IDX ? 1 : kSrtTile];
    __shared__ uint32_t sidx[OUT == SRT_PACK ? 1 : kSrtTile];
    // packed in and out: a staged code's digit is re-read from the code, so
    // the digit array is not staged (4 KiB less LDS: 4 workgroups per CU
    // instead of 3)
    constexpr bool DIG_FROM_KEY = IN_P && OUT == SRT_PACK;
    __shared__ uint8_t sdig[DIG_FROM_KEY ? 1 : kSrtTile];
    __shared__ uint32_t dstart[256];
    __shared__ uint64_t gbase[256];  // global position of local slot 0 of each digit run
    __shared__ uint32_t cnt[NW][256];
    __shared__ uint64_t wsum[NW];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // consecutive tiles on one XCD (bijective remap of the round-robin
    // dispatch), so the digit runs that neighbouring tiles write into the
    // same output lines meet in one L2 instead of leaving it as two partial
    // line write-backs
    const int64_t tile = xcd_tile(blockIdx.x, ntiles);
    const int64_t base = tile * kSrtTile;
    const int m = n - base < kSrtTile ? (int)(n - base) : kSrtTile;
    // this tile's digit offsets (256 scattered words): issued first so their
    // latency hides behind the key loads and the ranking
    const uint64_t my_off = tid < 256 ? (uint64_t)off[(int64_t)tid * ntiles + tile] : 0;
    for (int i = tid; i < NW * 256; i += TH) cnt[i >> 8][i & 255] = 0;
    uint64_t k[ROWS];
    uint32_t rk[ROWS];
    const int c0 = wid * (kSrtTile / NW);  // this wave's chunk
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
        const int i = c0 + r * 64 + lane;
        k[r] = i < m ? __builtin_nontemporal_load(keys_in + base + i) : 0;
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
        const int i = c0 + r * 64 + lane;
        const bool valid = i < m;
        const uint32_t d = (uint32_t)(k[r] >> shift) & 0xFF;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint64_t bb = __ballot((d >> b) & 1);
            peers &= ((d >> b) & 1) ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        const uint32_t old = cnt[wid][d];
        rk[r] = old + rank;
        // the group's leader bumps the counter (program order within the wave
        // keeps every peer's read before this write)
        if (valid && rank == 0) cnt[wid][d] = old + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    {
        // thread = digit (threads >= 256 add nothing): wave prefixes and the
        // tile's digit starts
        uint32_t t = 0;
        if (tid < 256) {
            for (int w = 0; w < NW; ++w) {
                const uint32_t c = cnt[w][tid];
                cnt[w][tid] = t;
                t += c;
            }
        }
        uint64_t total;
        const uint32_t ds = (uint32_t)block_excl_scan(t, wsum, total);
        if (tid < 256) {
            dstart[tid] = ds;
            gbase[tid] = my_off - ds;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
        const int i = c0 + r * 64 + lane;
        if (i < m) {
            const uint32_t d = (uint32_t)(k[r] >> shift) & 0xFF;
            const uint32_t pos = dstart[d] + cnt[wid][d] + rk[r];
            if (!DIG_FROM_KEY) sdig[pos] = (uint8_t)d;
            if (IN_P) {
                if (OUT == SRT_IDX) sidx[pos] = (uint32_t)k[r];
                else skey[pos] = k[r];
            } else {
                const uint32_t id = idx_in ? __builtin_nontemporal_load(idx_in + base + i) : (uint32_t)(base + i);
                if (OUT == SRT_PACK) skey[pos] = (((k[r] >> cons) & kmask) << 32) | id;
                else {
                    if (OUT == SRT_SEP) skey[pos] = k[r];
                    sidx[pos] = id;
                }
            }
        }
    }
    __syncthreads();
    // coalesced write-out: consecutive threads, consecutive slots of a digit run
    for (int p = tid; p < m; p += TH) {
        const uint32_t d = DIG_FROM_KEY ? (uint32_t)(skey[p] >> shift) & 0xFF : sdig[p];
        const uint64_t o = gbase[d] + (uint64_t)p;
        if (OUT != SRT_IDX) keys_out[o] = skey[p];
        if (OUT != SRT_PACK) idx_out[o] = sidx[p];
    }
}

// Multi-column sort: the codes of column c at the rows of the current
// permutation (null rows get code 0; their place comes from the null pass).
__global__ void srt_perm_codes_kernel(DevCol c, int64_t n, bool descending, const uint32_t* __restrict__ perm,
                                      uint64_t* __restrict__ keys) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = perm[i];
        keys[i] = dev_valid(c, r) ? sort_code(c, r, descending) : 0ull;
    }
}

// String sort keys (polars orders strings by their UTF-8 bytes): the key of
// a string is the tuple (8-byte chunk 0, chunk 1, ..., length) with chunks
// big-endian and zero-padded -- a proper prefix sorts first through the
// length.  LSD over the tuple: the length pass, then the chunks from last
// to first, each a stable radix sort of one u64 code per row.
// part < 0: the length; part = k: chunk k.  Null rows get code 0 (placed by
// the null pass afterwards, their order kept).
__global__ void srt_str_codes_kernel(DevCol c, int64_t n, bool descending, int part,
                                     const uint32_t* __restrict__ perm, uint64_t* __restrict__ keys) {
    const int64_t* off = (const int64_t*)c.values;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = perm[i];
        uint64_t k = 0;
        if (dev_valid(c, r)) {
            const int64_t b = off[c.offset + r], len = off[c.offset + r + 1] - b;
            if (part < 0) {
                k = (uint64_t)len;
            } else {
                const int64_t lo = (int64_t)part * 8;
                for (int j = 0; j < 8; ++j) {
                    const uint64_t byte = lo + j < len ? c.data[b + lo + j] : 0u;
                    k |= byte << (56 - 8 * j);
                }
            }
            if (descending) k = ~k;
        }
        keys[i] = k;
    }
}

__global__ void srt_str_maxlen_kernel(DevCol c, int64_t n, unsigned long long* __restrict__ mx) {
    const int64_t* off = (const int64_t*)c.values;
    uint64_t m = 0;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        if (dev_valid(c, r)) {
            const uint64_t len = (uint64_t)(off[c.offset + r + 1] - off[c.offset + r]);
            m = len > m ? len : m;
        }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint64_t y = __shfl_xor(m, o, 64);
        m = y > m ? y : m;
    }
    if ((threadIdx.x & 63) == 0 && m) atomicMax(mx, (unsigned long long)m);
}

// Null placement of column c as a one-byte code: 0 sorts first.
__global__ void srt_null_codes_kernel(DevCol c, int64_t n, bool nulls_last, const uint32_t* __restrict__ perm,
                                      uint64_t* __restrict__ keys) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        keys[i] = (dev_valid(c, perm[i]) == nulls_last) ? 0ull : 1ull;
}

__global__ void srt_iota_kernel(int64_t n, uint32_t* __restrict__ idx) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        idx[i] = (uint32_t)i;
}

__global__ void srt_place_nulls_kernel(const uint32_t* __restrict__ nulls, int64_t nn, uint32_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nn; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = nulls[i];
}

}  // namespace plgpu

using namespace plgpu;

// Scratch of the radix passes over n codes.
struct SrtScratch {
    uint32_t* cnt = nullptr;  // per-tile digit counts, scanned in place into offsets
    uint64_t* part = nullptr;
    unsigned long long* hist = nullptr;
    uint64_t* tbits = nullptr;  // per-tile OR / AND (srt_codes_stats_kernel)
    int alloc(int64_t n, hipStream_t s, bool stats = false) {
        const int64_t ntiles = (n + kSrtTile - 1) / kSrtTile;
        int rc = dev_alloc((void**)&hist, 16, s);
        if (!rc && n > 0 && stats) rc = dev_alloc((void**)&tbits, ntiles * 16, s);
        if (!rc && n > 0) rc = dev_alloc((void**)&cnt, ntiles * 256 * 4, s);
        if (!rc && n > 0) rc = dev_alloc((void**)&part, ((ntiles * 256 + kScanChunk - 1) / kScanChunk + 1) * 8, s);
        return rc;
    }
    void release(hipStream_t s) {
        dev_free(cnt, s);
        dev_free(part, s);
        dev_free(hist, s);
        dev_free(tbits, s);
        tbits = nullptr;
        cnt = nullptr;
        part = nullptr;
        hist = nullptr;
    }
};

// Stable LSD passes over the bytes of keys[cur] that vary (one OR/AND read
// finds them), carrying idx[cur] (nullptr in idx[cur]: row ids are the
// positions); the result (row ids) ends in idx[cur].  Codes and ids switch
// to the PACKED representation as soon as the remaining code bits fit 32.
template <bool IN_P, int OUT>
static void srt_down(const uint64_t* ki, const uint32_t* ii, int64_t nv, int shift, int64_t ntiles,
                     const uint32_t* off, uint64_t* ko, uint32_t* io, int cons, uint64_t kmask, hipStream_t s) {
    // XCD-aware tiles (round-robin tiles measured slower, profiles/r02_sort_xcd_ab.log)
    KtScope kt("srt_downsweep_kernel", s);
    if constexpr (IN_P && OUT != SRT_SEP) {
        if (options().srt_w4) {
            srt_downsweep_kernel<IN_P, OUT, 4>
                <<<(unsigned)ntiles, kSrtThreads, 0, s>>>(ki, ii, nv, shift, ntiles, off, ko, io, cons, kmask);
            return;
        }
    }
    srt_downsweep_kernel<IN_P, OUT>
        <<<(unsigned)ntiles, kSrtThreads, 0, s>>>(ki, ii, nv, shift, ntiles, off, ko, io, cons, kmask);
}

// pre: srt_codes_stats_kernel produced keys[cur], the per-tile OR / AND in
// sc.tbits and the byte-0 digit counts in sc.cnt.  final_out (optional): the
// last pass writes the sorted row ids there (*wrote_final = true) instead of
// into idx[cur].
static int radix_passes(uint64_t* keys[2], uint32_t* idx[2], int64_t nv, int& cur, SrtScratch& sc, hipStream_t s,
                        bool ids_implicit = false, bool pre = false, uint32_t* final_out = nullptr,
                        bool* wrote_final = nullptr) {
    if (wrote_final) *wrote_final = false;
    if (nv <= 0) return PLGPU_OK;
    const int cus = 256;
    unsigned long long h[2] = {0ull, ~0ull};
    hipError_t e = hipMemcpyAsync(sc.hist, h, 16, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) {
        const int64_t nt = (nv + kSrtTile - 1) / kSrtTile;
        if (pre)
            srt_tbits_kernel<<<(unsigned)std::min<int64_t>((nt + 255) / 256, cus * 4), 256, 0, s>>>(sc.tbits, nt,
                                                                                                    sc.hist);
        else
            srt_bits_kernel<<<(unsigned)std::min<int64_t>((nv + 255) / 256, cus * 8), 256, 0, s>>>(keys[cur], nv,
                                                                                                   sc.hist);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h, sc.hist, 16, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "sort key bits");
    const int64_t ntiles = (nv + kSrtTile - 1) / kSrtTile;
    int bytes[8], nb = 0;
    for (int byte = 0; byte < 8; ++byte)
        if ((((h[0] ^ h[1]) >> (8 * byte)) & 0xFF) != 0) bytes[nb++] = byte;  // constant bytes: identity passes
    if (nb == 0) {
        if (ids_implicit) {
            srt_iota_kernel<<<(unsigned)std::min<int64_t>((nv + 255) / 256, cus * 16), 256, 0, s>>>(nv, idx[cur]);
            e = hipGetLastError();
            if (e != hipSuccess) return hip_fail(e, "sort iota");
        }
        return PLGPU_OK;
    }
    const int hi_bits = 8 * (bytes[nb - 1] + 1);
    bool packed = false;
    int cons = 0;  // code bits dropped by the packing
    for (int j = 0; j < nb; ++j) {
        const int S = 8 * bytes[j];
        const int shift = packed ? 32 + S - cons : S;
        const uint32_t* ii = (ids_implicit && j == 0) ? nullptr : idx[cur];
        if (!(pre && j == 0 && S == 0)) {  // byte-0 counts already in sc.cnt
            KtScope kt("srt_upsweep_kernel", s);
        {
            const int tpw = std::max<int>(1, (int)options().srt_up_tiles);
            srt_upsweep_kernel<<<(unsigned)((ntiles + tpw - 1) / tpw), kSrtThreads, 0, s>>>(keys[cur], nv, shift,
                                                                                           ntiles, sc.cnt, tpw);
        }
        }
        e = scan_exclusive32_inplace(sc.cnt, ntiles * 256, sc.part, s);
        if (e != hipSuccess) return hip_fail(e, "sort scan");
        const bool last = j == nb - 1;
        const int ncons = S + 8;
        const bool to_pack = !packed && !last && hi_bits - ncons <= 32;
        const uint64_t kmask = hi_bits - ncons >= 64 ? ~0ull : ((1ull << (hi_bits - ncons)) - 1);
        uint64_t* ko = keys[cur ^ 1];
        uint32_t* io = idx[cur ^ 1];
        if (last && final_out) {
            io = final_out;
            *wrote_final = true;
        }
        const uint32_t* off = sc.cnt;
        if (packed) {
            if (last) srt_down<true, SRT_IDX>(keys[cur], ii, nv, shift, ntiles, off, ko, io, 0, 0, s);
            else srt_down<true, SRT_PACK>(keys[cur], ii, nv, shift, ntiles, off, ko, io, 0, 0, s);
        } else if (last) {
            srt_down<false, SRT_IDX>(keys[cur], ii, nv, shift, ntiles, off, ko, io, 0, 0, s);
        } else if (to_pack) {
            srt_down<false, SRT_PACK>(keys[cur], ii, nv, shift, ntiles, off, ko, io, ncons, kmask, s);
            packed = true;
            cons = ncons;
        } else {
            srt_down<false, SRT_SEP>(keys[cur], ii, nv, shift, ntiles, off, ko, io, 0, 0, s);
        }
        e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(e, "sort pass");
        cur ^= 1;
    }
    return PLGPU_OK;
}

PLGPU_API int plgpu_arg_sort(const plgpu_column* key, int32_t descending, int32_t nulls_last, plgpu_column* out_idx,
                             void* stream) {
    hipStream_t s = as_stream(stream);
    if (key == nullptr || out_idx == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    std::memset(out_idx, 0, sizeof *out_idx);
    if (!dtype_is_int(key->dtype) && !dtype_is_float(key->dtype))
        return fail(PLGPU_ERR_SCHEMA, "sort key must be an integer or float column");
    const int64_t n = key->length;
    if (n >= 0xFFFFFFFFll) return fail(PLGPU_ERR_CAPACITY, "sort input exceeds the u32 index space");
    DevCol c;
    std::memset(&c, 0, sizeof c);
    c.dtype = key->dtype;
    c.offset = key->offset;
    c.values = key->values;
    c.validity = key->validity;
    int rc = make_owned_column(out_idx, PLGPU_U32, n, false, s);
    if (rc || n == 0) return rc;
    uint64_t* keys[2] = {nullptr, nullptr};
    uint32_t* idx[2] = {nullptr, nullptr};
    uint32_t* nulls = nullptr;
    uint64_t* part = nullptr;
    const int64_t nblk = (n + 1023) / 1024;
    for (int i = 0; i < 2 && !rc; ++i) {
        rc = dev_alloc((void**)&keys[i], n * 8, s);
        if (!rc) rc = dev_alloc((void**)&idx[i], n * 4, s);
    }
    int64_t nv = n;  // valid rows
    if (!rc && c.validity) {
        uint64_t* voff = nullptr;
        uint32_t* vcnt = nullptr;
        rc = dev_alloc((void**)&vcnt, nblk * 4, s);
        if (!rc) rc = dev_alloc((void**)&voff, (nblk + 1) * 8, s);
        if (!rc) rc = dev_alloc((void**)&part, ((nblk + kScanChunk - 1) / kScanChunk + 1) * 8, s);
        if (!rc) rc = dev_alloc((void**)&nulls, n * 4, s);
        if (!rc) {
            srt_count_valid_kernel<<<(unsigned)nblk, 256, 0, s>>>(c, n, vcnt);
            hipError_t e = scan_exclusive<uint32_t>(vcnt, nblk, voff, part, s);
            uint64_t tv = 0;
            if (e == hipSuccess) {
                srt_prep_kernel<<<(unsigned)nblk, 256, 0, s>>>(c, n, descending != 0, voff, keys[0], idx[0], nulls);
                e = hipGetLastError();
            }
            if (e == hipSuccess) e = hipMemcpyAsync(&tv, voff + nblk, 8, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) rc = hip_fail(e, "sort prep");
            nv = (int64_t)tv;
        }
        dev_free(vcnt, s);
        dev_free(voff, s);
        dev_free(part, s);
        part = nullptr;
    }
    int cur = 0;
    SrtScratch sc;
    const bool stats = c.validity == nullptr;
    if (!rc) rc = sc.alloc(nv, s, stats);
    if (!rc && stats) {
        // row ids stay implicit (= positions) until the first pass writes them
        const int64_t ntiles = (n + kSrtTile - 1) / kSrtTile;
        KtScope kt("srt_codes_stats_kernel", s);
        srt_codes_stats_kernel<<<(unsigned)ntiles, kSrtThreads, 0, s>>>(c, n, descending != 0, ntiles, keys[0],
                                                                         sc.cnt, sc.tbits);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) rc = hip_fail(e, "sort codes");
    }
    uint32_t* out = (uint32_t*)out_idx->values;
    const int64_t nn = n - nv;
    // nulls first (default) or last, each group in row order
    uint32_t* vdst = nulls_last ? out : out + nn;
    uint32_t* ndst = nulls_last ? out + nv : out;
    bool wrote = false;
    if (!rc) rc = radix_passes(keys, idx, nv, cur, sc, s, stats, stats, vdst, &wrote);
    sc.release(s);
    if (!rc) {
        hipError_t e = hipSuccess;
        if (nv > 0 && !wrote) e = hipMemcpyAsync(vdst, idx[cur], nv * 4, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess && nn > 0) e = hipMemcpyAsync(ndst, nulls, nn * 4, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "sort output");
    }
    for (int i = 0; i < 2; ++i) {
        dev_free(keys[i], s);
        dev_free(idx[i], s);
    }
    dev_free(nulls, s);
    if (rc) plgpu_column_release(out_idx);
    return rc;
}

// Multi-column arg_sort: LSD over the columns (last column first), each
// column one stable radix sort of its codes gathered through the current
// permutation, then -- if it has nulls -- one stable pass placing them.
PLGPU_API int plgpu_arg_sort_multi(const plgpu_column* keys_in, int32_t nkeys, const int32_t* descending,
                                   const int32_t* nulls_last, plgpu_column* out_idx, void* stream) {
    hipStream_t s = as_stream(stream);
    if (keys_in == nullptr || out_idx == nullptr || descending == nullptr || nulls_last == nullptr)
        return fail(PLGPU_ERR_INVALID, "NULL argument");
    std::memset(out_idx, 0, sizeof *out_idx);
    if (nkeys < 1 || nkeys > 8) return fail(PLGPU_ERR_INVALID, "number of sort columns must be 1..8");
    const int64_t n = keys_in[0].length;
    for (int j = 0; j < nkeys; ++j) {
        const int32_t dt = keys_in[j].dtype;
        if (!dtype_is_int(dt) && !dtype_is_float(dt) && dt != PLGPU_BOOL && dt != PLGPU_STR)
            return fail(PLGPU_ERR_SCHEMA, "sort keys must be integer, float, Boolean or String columns");
        if (keys_in[j].length != n) return fail(PLGPU_ERR_SHAPE, "sort columns must have equal lengths");
    }
    if (n >= 0xFFFFFFFFll) return fail(PLGPU_ERR_CAPACITY, "sort input exceeds the u32 index space");
    int rc = make_owned_column(out_idx, PLGPU_U32, n, false, s);
    if (rc || n == 0) return rc;
    uint64_t* keys[2] = {nullptr, nullptr};
    uint32_t* idx[2] = {nullptr, nullptr};
    for (int i = 0; i < 2 && !rc; ++i) {
        rc = dev_alloc((void**)&keys[i], n * 8, s);
        if (!rc) rc = dev_alloc((void**)&idx[i], n * 4, s);
    }
    SrtScratch sc;
    if (!rc) rc = sc.alloc(n, s);
    int cur = 0;
    const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 256 * 16);
    if (!rc) {
        srt_iota_kernel<<<g, 256, 0, s>>>(n, idx[0]);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) rc = hip_fail(e, "sort iota");
    }
    unsigned long long* maxlen = nullptr;
    for (int j = nkeys - 1; j >= 0 && !rc; --j) {
        const DevCol c = dev_col(keys_in[j]);
        hipError_t e = hipSuccess;
        if (c.dtype == PLGPU_STR) {
            unsigned long long ml = 0;
            if (maxlen == nullptr && (rc = dev_alloc((void**)&maxlen, 8, s))) break;
            e = hipMemsetAsync(maxlen, 0, 8, s);
            if (e == hipSuccess) {
                srt_str_maxlen_kernel<<<g, 256, 0, s>>>(c, n, maxlen);
                e = hipGetLastError();
            }
            if (e == hipSuccess) e = hipMemcpyAsync(&ml, maxlen, 8, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            const int chunks = (int)((ml + 7) / 8);
            for (int part = -1; part < chunks && e == hipSuccess && !rc; ++part) {
                // LSD order: the length first, then the chunks from the last
                const int pk = part < 0 ? -1 : chunks - 1 - part;
                srt_str_codes_kernel<<<g, 256, 0, s>>>(c, n, descending[j] != 0, pk, idx[cur], keys[cur]);
                e = hipGetLastError();
                if (e == hipSuccess) rc = radix_passes(keys, idx, n, cur, sc, s);
            }
        } else {
            srt_perm_codes_kernel<<<g, 256, 0, s>>>(c, n, descending[j] != 0, idx[cur], keys[cur]);
            e = hipGetLastError();
            if (e == hipSuccess) rc = radix_passes(keys, idx, n, cur, sc, s);
        }
        if (e != hipSuccess) {
            rc = hip_fail(e, "sort codes");
            break;
        }
        if (!rc && c.validity && keys_in[j].null_count != 0) {
            srt_null_codes_kernel<<<g, 256, 0, s>>>(c, n, nulls_last[j] != 0, idx[cur], keys[cur]);
            e = hipGetLastError();
            if (e != hipSuccess) rc = hip_fail(e, "sort null codes");
            if (!rc) rc = radix_passes(keys, idx, n, cur, sc, s);
        }
    }
    if (!rc) {
        hipError_t e = hipMemcpyAsync((void*)out_idx->values, idx[cur], n * 4, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "sort output");
    }
    sc.release(s);
    dev_free(maxlen, s);
    for (int i = 0; i < 2; ++i) {
        dev_free(keys[i], s);
        dev_free(idx[i], s);
    }
    if (rc) plgpu_column_release(out_idx);
    return rc;
}
