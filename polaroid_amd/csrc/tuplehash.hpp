// Key tuples of several columns (multi-key group-by / join): a 64-bit hash
// per row and tuple equality.  The reference row-encodes the key columns
// (polars-core/src/chunked_array/ops/row_encode.rs:11) and compares the
// encoded bytes: a null equals only a null, f64 keys compare by TotalOrd
// (-0.0 == 0.0, every NaN equal).  Equal tuples hash equally; unequal ones
// collide with probability ~2^-64 per pair, and every user of the hash
// verifies tuples afterwards.
#pragma once

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

// Canonical key word: f64 keys compare by TotalOrd (-0 == 0, NaN == NaN).
__device__ __forceinline__ uint64_t mk_word(const DevCol& c, int64_t r) {
    uint64_t x = dev_load(c, r);
    if (c.dtype == PLGPU_F64) {
        if ((x & 0x7FFFFFFFFFFFFFFFull) == 0) x = 0;
        else if ((x & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull) x = 0x7FF8000000000000ull;
    }
    return x;
}

__device__ __forceinline__ uint64_t mk_row_hash(const MkKeys& k, int64_t r, uint64_t seed) {
    uint64_t h = seed;
    for (int i = 0; i < k.n; ++i) {
        const DevCol& c = k.c[i];
        const uint64_t w = dev_valid(c, r) ? mk_fmix(mk_word(c, r) ^ seed) : 0x6A09E667F3BCC909ull + (uint64_t)i;
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
        eq &= va == vb && (!va || mk_word(a.c[i], ra) == mk_word(b.c[i], rb));
    }
    return eq;
}

}  // namespace plgpu
