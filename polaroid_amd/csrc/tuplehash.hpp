// Key tuples of several columns (multi-key group-by / join): a 64-bit hash
// per row and tuple equality.  The reference row-encodes the key columns
// (polars-core/src/chunked_array/ops/row_encode.rs:11) and compares the
// encoded bytes: a null equals only a null, f64 keys compare by TotalOrd
// (-0.0 == 0.0, every NaN equal).  Equal tuples hash equally; unequal ones
// collide with probability ~2^-64 per pair, and every user of the hash
// verifies tuples afterwards.
#pragma once

#include <cstdlib>
#include <cstring>

#include "plgpu_internal.hpp"

namespace plgpu {

constexpr int kMaxKeys = 8;

struct MkKeys {
    DevCol c[kMaxKeys];
    int32_t n;
    int32_t _pad;
};

__device__ __forceinline__ uint64_t mk_fmix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 33;
    x *= 0xC4CEB9FE1A85EC53ull;
    x ^= x >> 33;
    return x;
}

// Partition hash of the many-groups group-by and the partitioned join (its
// top bits pick the partition; independent of the table hashes, which
// multiply by the golden ratio).  A bijection of the key (fmix64 is
// invertible), so distinct keys never share all 64 bits.
__device__ __forceinline__ uint64_t part_hash(uint64_t key) { return mk_fmix(key ^ 0x2545F4914F6CDD1Dull); }

// 64-bit hash of a string's bytes (8-byte little-endian words, then the
// tail; the length is mixed in, so "" and "\0" differ).
__device__ __forceinline__ uint64_t str_hash(const DevCol& c, int64_t r, uint64_t seed = 0) {
    const int64_t* off = (const int64_t*)c.values;
    const int64_t b = off[c.offset + r], len = off[c.offset + r + 1] - b;
    const uint8_t* p = c.data + b;
    uint64_t h = (0x9E3779B97F4A7C15ull + seed) ^ (uint64_t)len;
    int64_t i = 0;
    for (; i + 8 <= len; i += 8) {
        uint64_t w = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) w |= (uint64_t)p[i + j] << (8 * j);
        h = mk_fmix(h ^ w) + 0xD6E8FEB86659FD93ull;
    }
    uint64_t w = 0;
    for (int j = 0; i + j < len; ++j) w |= (uint64_t)p[i + j] << (8 * j);
    return mk_fmix(h ^ w ^ 0xA0761D6478BD642Full);
}

// Byte equality of row ra of string column a and row rb of b.
__device__ __forceinline__ bool str_equal(const DevCol& a, int64_t ra, const DevCol& b, int64_t rb) {
    const int64_t* oa = (const int64_t*)a.values;
    const int64_t* ob = (const int64_t*)b.values;
    const int64_t sa = oa[a.offset + ra], la = oa[a.offset + ra + 1] - sa;
    const int64_t sb = ob[b.offset + rb], lb = ob[b.offset + rb + 1] - sb;
    if (la != lb) return false;
    for (int64_t i = 0; i < la; ++i)
        if (a.data[sa + i] != b.data[sb + i]) return false;
    return true;
}

// Canonical key word: f64 keys compare by TotalOrd (-0 == 0, NaN == NaN);
// a string key's word is its hash (equality is checked on the bytes).
__device__ __forceinline__ uint64_t mk_word(const DevCol& c, int64_t r) {
    if (c.dtype == PLGPU_STR) return str_hash(c, r);
    uint64_t x = dev_load(c, r);
    if (c.dtype == PLGPU_F64 || c.dtype == PLGPU_F32) {
        if ((x & 0x7FFFFFFFFFFFFFFFull) == 0) x = 0;
        else if ((x & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull) x = 0x7FF8000000000000ull;
    }
    return x;
}

__device__ __forceinline__ uint64_t mk_row_hash(const MkKeys& k, int64_t r, uint64_t seed) {
    uint64_t h = seed;
    for (int i = 0; i < k.n; ++i) {
        const DevCol& c = k.c[i];
        // strings hash with the seed, so a re-seed also separates two strings
        // whose unseeded hashes collide
        const uint64_t w = dev_valid(c, r) ? mk_fmix((c.dtype == PLGPU_STR ? str_hash(c, r, seed) : mk_word(c, r)) ^ seed)
                                           : 0x6A09E667F3BCC909ull + (uint64_t)i;
        h = mk_fmix(h * 0x9E3779B97F4A7C15ull + w + (uint64_t)i);
    }
    return h;
}

__device__ __forceinline__ bool mk_any_null(const MkKeys& k, int64_t r) {
    bool any = false;
    for (int i = 0; i < k.n; ++i) any |= !dev_valid(k.c[i], r);
    return any;
}

// Tuple of row ra in `a` equals tuple of row rb in `b` (same dtypes).
__device__ __forceinline__ bool mk_equal(const MkKeys& a, int64_t ra, const MkKeys& b, int64_t rb) {
    bool eq = true;
    for (int i = 0; i < a.n; ++i) {
        const bool va = dev_valid(a.c[i], ra), vb = dev_valid(b.c[i], rb);
        if (a.c[i].dtype == PLGPU_STR) eq &= va == vb && (!va || str_equal(a.c[i], ra, b.c[i], rb));
        else eq &= va == vb && (!va || mk_word(a.c[i], ra) == mk_word(b.c[i], rb));
    }
    return eq;
}

}  // namespace plgpu

// ---------------------------------------------------------------------------
// Exact packing: when every key is an integer (or Boolean) column whose value
// range, plus a null code, fits next to the others in 63 bits, a tuple is
// encoded injectively as one Int64 -- the multi-key operators then run as
// single-key ones with no hashing, no verification and no collision path.
// Field i = null ? 0 : v - min_i + (nullable_i ? 1 : 0), at bit shift_i.
namespace plgpu {
namespace {  // internal linkage: included by several translation units

struct MkPack {
    int32_t n;
    int32_t ok;
    int64_t minv[kMaxKeys];
    int32_t shift[kMaxKeys];
    int32_t bits[kMaxKeys];
    int32_t nullable[kMaxKeys];
};

// Per key column: [ord(min), ord(max), any null] at stats[3 * i ...]; ord(x)
// = x ^ 2^63 so unsigned atomics order signed values.
__global__ __launch_bounds__(256) void mk_range_kernel(MkKeys k, int64_t n, unsigned long long* __restrict__ stats) {
    for (int i = 0; i < k.n; ++i) {
        const DevCol& c = k.c[i];
        uint64_t mn = ~0ull, mx = 0, nul = 0;
        for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
            if (!dev_valid(c, r)) {
                nul = 1;
                continue;
            }
            const uint64_t o = dev_load(c, r) ^ 0x8000000000000000ull;
            mn = o < mn ? o : mn;
            mx = o > mx ? o : mx;
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint64_t a = __shfl_xor(mn, off, 64), b = __shfl_xor(mx, off, 64);
            mn = a < mn ? a : mn;
            mx = b > mx ? b : mx;
            nul |= __shfl_xor(nul, off, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            if (mn != ~0ull) atomicMin(&stats[3 * i], (unsigned long long)mn);
            if (mx != 0) atomicMax(&stats[3 * i + 1], (unsigned long long)mx);
            if (nul) atomicOr(&stats[3 * i + 2], 1ull);
        }
    }
}

// Sampled key ranges (the group-by's optimistic packing): `samples` rows in
// clusters of 16 consecutive rows spread evenly over the column, per key
// [ord(min), ord(max), any null] into stats as mk_range_kernel does.
__global__ __launch_bounds__(256) void mk_sample_range_kernel(MkKeys k, int64_t n, int64_t samples,
                                                              unsigned long long* __restrict__ stats) {
    const int64_t m = n < samples ? n : samples;
    const int64_t cstep = n <= samples ? 16 : n / (samples >> 4);
    for (int i = 0; i < k.n; ++i) {
        const DevCol& c = k.c[i];
        uint64_t mn = ~0ull, mx = 0, nul = 0;
        for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
            const int64_t r = n <= samples ? j : (j >> 4) * cstep + (j & 15);
            if (r >= n) continue;
            if (!dev_valid(c, r)) {
                nul = 1;
                continue;
            }
            const uint64_t o = dev_load(c, r) ^ 0x8000000000000000ull;
            mn = o < mn ? o : mn;
            mx = o > mx ? o : mx;
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint64_t a = __shfl_xor(mn, off, 64), b = __shfl_xor(mx, off, 64);
            mn = a < mn ? a : mn;
            mx = b > mx ? b : mx;
            nul |= __shfl_xor(nul, off, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            if (mn != ~0ull) atomicMin(&stats[3 * i], (unsigned long long)mn);
            if (mx != 0) atomicMax(&stats[3 * i + 1], (unsigned long long)mx);
            if (nul) atomicOr(&stats[3 * i + 2], 1ull);
        }
    }
}

// Packed Int64 code per row; `valid_words` (optional): one bit per row, 0
// when the tuple holds a null and nulls are not values (join without
// nulls_equal).  `outside` (optional, a plan from sampled ranges): set when
// some row's field does not fit its bits (the code would be wrong; the
// caller repacks with exact ranges).
// Largest field value of key i that is a packed value: v - base <= span
// holds exactly for base <= v < base + 2^bits (a v below base wraps past
// 2^64 - 1 - ord(base), ord(x) = x ^ 2^63), base = minv - nullable.
__device__ __forceinline__ uint64_t mk_span(const MkPack& pk, int i) {
    // a 64-bit field (the identity plan of one key: the sign- or
    // zero-extended value is the code) holds every value
    if (pk.bits[i] >= 64) return ~0ull;
    const uint64_t mask = pk.bits[i] >= 64 ? ~0ull : (1ull << pk.bits[i]) - 1;
    const uint64_t ordb = ((uint64_t)pk.minv[i] - (pk.nullable[i] ? 1u : 0u)) ^ 0x8000000000000000ull;
    return mask < ~0ull - ordb ? mask : ~0ull - ordb;
}

__global__ __launch_bounds__(256) void mk_pack_kernel(MkKeys k, MkPack pk, int64_t n, uint64_t* __restrict__ out,
                                                      uint64_t* __restrict__ valid_words,
                                                      unsigned int* __restrict__ outside = nullptr) {
    bool bad = false;
    for (int64_t r0 = (int64_t)blockIdx.x * blockDim.x; r0 < n; r0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = r0 + threadIdx.x;
        const bool in = r < n;
        bool anynull = false;
        uint64_t code = 0;
        if (in) {
            for (int i = 0; i < k.n; ++i) {
                const DevCol& c = k.c[i];
                uint64_t f;
                if (dev_valid(c, r)) f = (uint64_t)((int64_t)dev_load(c, r) - pk.minv[i]) + (pk.nullable[i] ? 1u : 0u);
                else {
                    f = 0;
                    anynull = true;
                    bad |= !pk.nullable[i];
                }
                if (outside) bad |= f > mk_span(pk, i);
                code |= f << pk.shift[i];
            }
            out[r] = code;
        }
        if (valid_words) {
            const uint64_t b = __ballot(in && !anynull);
            if ((threadIdx.x & 63) == 0 && r - (threadIdx.x & 63) < n) valid_words[(r - (threadIdx.x & 63)) >> 6] = b;
        }
    }
    if (outside && __any(bad) && (threadIdx.x & 63) == 0) atomicOr(outside, 1u);
}

// Two consecutive rows (r, r + 1) of a null-free 4- or 8-byte integer key
// column: one 16-byte (8-byte) load when both are in range and the pair is
// aligned, register-form loads otherwise.
__device__ __forceinline__ void mk_load_pair(const DevCol& c, int64_t r, int64_t n, uint64_t& a, uint64_t& b) {
    const int64_t p = c.offset + r;
    if (r + 1 < n && (p & 1) == 0) {
        if (c.dtype == PLGPU_I64) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2*>((const uint64_t*)c.values + p);
            a = v.x;
            b = v.y;
            return;
        }
        const uint2 v = *reinterpret_cast<const uint2*>((const uint32_t*)c.values + p);
        a = c.dtype == PLGPU_U32 ? (uint64_t)v.x : (uint64_t)(int64_t)(int32_t)v.x;
        b = c.dtype == PLGPU_U32 ? (uint64_t)v.y : (uint64_t)(int64_t)(int32_t)v.y;
        return;
    }
    a = r < n ? dev_load(c, r) : 0ull;
    b = r + 1 < n ? dev_load(c, r + 1) : 0ull;
}

// mk_pack_kernel for null-free I64 / I32 / U32 keys and no validity output:
// each thread packs U pairs of consecutive rows per step, every key column
// read with pair loads and the codes stored as 16-byte pairs.
template <int U>
__global__ __launch_bounds__(256) void mk_pack_vec_kernel(MkKeys k, MkPack pk, int64_t n, uint64_t* __restrict__ out,
                                                          unsigned int* __restrict__ outside) {
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    bool bad = false;
    for (int64_t base = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2; base < n; base += T * 2 * U) {
        uint64_t code[U][2];
#pragma unroll
        for (int u = 0; u < U; ++u) code[u][0] = code[u][1] = 0;
#pragma unroll
        for (int i = 0; i < kMaxKeys; ++i) {
            if (i >= k.n) break;
            uint64_t v[U][2];
#pragma unroll
            for (int u = 0; u < U; ++u) mk_load_pair(k.c[i], base + (int64_t)u * T * 2, n, v[u][0], v[u][1]);
            const uint64_t noff = pk.nullable[i] ? 1u : 0u;
            const uint64_t span = mk_span(pk, i);
#pragma unroll
            for (int u = 0; u < U; ++u) {
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const uint64_t f = (uint64_t)((int64_t)v[u][e] - pk.minv[i]) + noff;
                    if (outside) bad |= base + (int64_t)u * T * 2 + e < n && f > span;
                    code[u][e] |= f << pk.shift[i];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t r = base + (int64_t)u * T * 2;
            if (r + 1 < n) {
                *reinterpret_cast<ulonglong2*>(out + r) = make_ulonglong2(code[u][0], code[u][1]);
            } else if (r < n) {
                out[r] = code[u][0];
            }
        }
    }
    if (outside && __any(bad) && (threadIdx.x & 63) == 0) atomicOr(outside, 1u);
}

// Launch the packing pass: the vector form when it applies.
inline void mk_pack_launch(const MkKeys& k, const MkPack& pk, int64_t n, uint64_t* out, uint64_t* valid_words,
                           unsigned int* outside, int grid, hipStream_t s) {
    if (n <= 0) return;
    bool vec = ((uintptr_t)out & 15) == 0;
    for (int i = 0; i < k.n; ++i)
        vec = vec && k.c[i].validity == nullptr &&
              (k.c[i].dtype == PLGPU_I64 || k.c[i].dtype == PLGPU_I32 || k.c[i].dtype == PLGPU_U32) &&
              ((uintptr_t)k.c[i].values & 15) == 0;
    if (vec) {
        // null-free keys: every tuple is valid
        if (valid_words) (void)hipMemsetAsync(valid_words, 0xFF, (size_t)((n + 63) / 64) * 8, s);
        const int64_t pairs = (n + 1) / 2;
        const int g = (int)std::max<int64_t>(1, std::min<int64_t>((pairs + 255) / 256, (int64_t)grid));
        {
            KtScope kt("mk_pack_vec_kernel", s);
            mk_pack_vec_kernel<2><<<g, 256, 0, s>>>(k, pk, n, out, outside);
        }
    } else {
        mk_pack_kernel<<<grid, 256, 0, s>>>(k, pk, n, out, valid_words, outside);
    }
}

// Packed codes -> key column i (dtype of the input key; validity zeroed
// beforehand; Boolean values bit-packed, zeroed beforehand).
__global__ __launch_bounds__(256) void mk_unpack_kernel(const int64_t* __restrict__ codes, const uint32_t* code_valid,
                                                        int64_t g_n, MkPack pk, int i, int32_t dtype, void* out,
                                                        uint32_t* out_valid) {
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < g_n; g += (int64_t)gridDim.x * blockDim.x) {
        const bool cv = code_valid == nullptr || ((code_valid[g >> 5] >> (g & 31)) & 1u);
        const uint64_t mask = pk.bits[i] >= 64 ? ~0ull : ((1ull << pk.bits[i]) - 1);
        const uint64_t f = ((uint64_t)codes[g] >> pk.shift[i]) & mask;
        const bool valid = cv && !(pk.nullable[i] && f == 0);
        const int64_t v = valid ? pk.minv[i] + (int64_t)(f - (pk.nullable[i] ? 1u : 0u)) : 0;
        if (dtype == PLGPU_BOOL) {
            if (v & 1) atomicOr(&((uint32_t*)out)[g >> 5], 1u << (g & 31));
        } else {
            dev_store(out, dtype, g, (uint64_t)v);
        }
        if (out_valid && valid) atomicOr(&out_valid[g >> 5], 1u << (g & 31));
    }
}

// Packing plan from per-key [ord(min), ord(max), any null] ranges (min >
// max: no valid value); pk->ok = 0 when the fields need more than 63 bits.
inline void mk_plan_from_ranges(const uint64_t* h, int n, MkPack* pk) {
    int shift = 0;
    pk->ok = 0;
    for (int i = 0; i < n; ++i) {
        uint64_t mn = h[3 * i], mx = h[3 * i + 1];
        const bool nul = h[3 * i + 2] != 0;
        if (mn > mx) {  // no valid value anywhere: one code (null or 0)
            mn = mx = 0x8000000000000000ull;
        }
        const uint64_t span = mx - mn;  // of ord values == of the signed values
        const uint64_t codes = span + (nul ? 2u : 1u);
        if (span >= (1ull << 62)) return;
        int b = 0;
        while (b < 63 && (1ull << b) < codes) ++b;
        pk->minv[i] = (int64_t)(mn ^ 0x8000000000000000ull);
        pk->shift[i] = shift;
        pk->bits[i] = b;
        pk->nullable[i] = nul ? 1 : 0;
        shift += b;
        if (shift > 63) return;
    }
    pk->ok = 1;
}

// Packing plan from sampled ranges, widened by each key's sampled span (and
// a null code reserved for every key), so that values the sample missed
// near its ends still fit; mk_pack_kernel's `outside` flag catches the rest
// and the caller repacks with the exact ranges.  pk->ok = 0 when a key is not
// packable or the widened fields need > 63 bits.
inline int mk_plan_pack_sampled(const MkKeys& ka, int64_t na, MkPack* pk, hipStream_t s) {
    std::memset(pk, 0, sizeof *pk);
    pk->n = ka.n;
    for (int i = 0; i < ka.n; ++i)
        if (dtype_is_float(ka.c[i].dtype) || ka.c[i].dtype == PLGPU_U64 || ka.c[i].dtype == PLGPU_STR)
            return PLGPU_OK;
    if (options().no_pack) return PLGPU_OK;
    unsigned long long* st = nullptr;
    const size_t bytes = 3 * kMaxKeys * 8;
    int rc = dev_alloc((void**)&st, bytes, s);
    if (rc) return rc;
    unsigned long long h[3 * kMaxKeys];
    for (int j = 0; j < kMaxKeys; ++j) h[3 * j] = ~0ull, h[3 * j + 1] = 0, h[3 * j + 2] = 0;
    hipError_t e = hipMemcpyAsync(st, h, bytes, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && na > 0) {
        {
            KtScope kt("mk_sample_range_kernel", s);
            mk_sample_range_kernel<<<16, 256, 0, s>>>(ka, na, 65536, st);
        }
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h, st, bytes, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    dev_free(st, s);
    if (e != hipSuccess) return hip_fail(e, "sampled key range pass");
    uint64_t r[3 * kMaxKeys];
    for (int i = 0; i < ka.n; ++i) {
        uint64_t mn = h[3 * i], mx = h[3 * i + 1];
        if (mn > mx) mn = mx = 0x8000000000000000ull;
        const uint64_t span = (mx - mn) + 1024;
        mn = mn > span ? mn - span : 0;
        mx = mx < ~0ull - span ? mx + span : ~0ull;
        // the dtype's own range bounds the widened one
        const int b = dtype_bytes(ka.c[i].dtype) * 8;
        if (ka.c[i].dtype == PLGPU_BOOL) {
            mn = 0x8000000000000000ull;
            mx = mn + 1;
        } else if (b > 0 && b < 64) {
            const bool uns = ka.c[i].dtype == PLGPU_U8 || ka.c[i].dtype == PLGPU_U16 || ka.c[i].dtype == PLGPU_U32;
            const int64_t lo = uns ? 0 : -(int64_t(1) << (b - 1));
            const int64_t hi = uns ? (int64_t(1) << b) - 1 : (int64_t(1) << (b - 1)) - 1;
            const uint64_t olo = (uint64_t)lo ^ 0x8000000000000000ull, ohi = (uint64_t)hi ^ 0x8000000000000000ull;
            mn = mn < olo ? olo : mn;
            mx = mx > ohi ? ohi : mx;
        }
        r[3 * i] = mn;
        r[3 * i + 1] = mx;
        r[3 * i + 2] = 1;
    }
    mk_plan_from_ranges(r, ka.n, pk);
    return PLGPU_OK;
}

// Range pass over `ka` (and `kb`, the other join side, when non-null) and the
// packing plan; pk->ok = 0 when a key is Float64 or the fields need > 63 bits.
inline int mk_plan_pack(const MkKeys& ka, int64_t na, const MkKeys* kb, int64_t nb, int grid, MkPack* pk,
                        hipStream_t s) {
    std::memset(pk, 0, sizeof *pk);
    pk->n = ka.n;
    for (int i = 0; i < ka.n; ++i)
        if (dtype_is_float(ka.c[i].dtype) || ka.c[i].dtype == PLGPU_U64 || ka.c[i].dtype == PLGPU_STR)
            return PLGPU_OK;  // hashed path (UInt64 ranges do not fit the signed range pass)
    if (options().no_pack) return PLGPU_OK;  // tests: force the hashed path
    unsigned long long* st = nullptr;
    const size_t bytes = 2 * 3 * kMaxKeys * 8;
    int rc = dev_alloc((void**)&st, bytes, s);
    if (rc) return rc;
    unsigned long long h[2 * 3 * kMaxKeys];
    for (int j = 0; j < 2 * kMaxKeys; ++j) {
        h[3 * j] = ~0ull;
        h[3 * j + 1] = 0;
        h[3 * j + 2] = 0;
    }
    hipError_t e = hipMemcpyAsync(st, h, bytes, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && na > 0) {
        mk_range_kernel<<<grid, 256, 0, s>>>(ka, na, st);
        e = hipGetLastError();
    }
    if (e == hipSuccess && kb && nb > 0) {
        mk_range_kernel<<<grid, 256, 0, s>>>(*kb, nb, st + 3 * kMaxKeys);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h, st, bytes, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    dev_free(st, s);
    if (e != hipSuccess) return hip_fail(e, "key range pass");
    uint64_t r[3 * kMaxKeys];
    for (int i = 0; i < ka.n; ++i) {
        uint64_t mn = h[3 * i], mx = h[3 * i + 1];
        bool nul = h[3 * i + 2] != 0;
        if (kb) {
            const uint64_t mn2 = h[3 * (kMaxKeys + i)], mx2 = h[3 * (kMaxKeys + i) + 1];
            mn = mn2 < mn ? mn2 : mn;
            mx = mx2 > mx ? mx2 : mx;
            nul = nul || h[3 * (kMaxKeys + i) + 2] != 0;
        }
        r[3 * i] = mn;
        r[3 * i + 1] = mx;
        r[3 * i + 2] = nul ? 1 : 0;
    }
    mk_plan_from_ranges(r, ka.n, pk);
    return PLGPU_OK;
}

}  // namespace
}  // namespace plgpu
