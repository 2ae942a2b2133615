// Fixed-window rolling sum / mean of one column.
//
// Reference (paths under /root/reference/crates):
//   polars-compute/src/rolling/no_nulls/mean.rs:6 rolling_mean,
//   no_nulls/sum.rs:5 rolling_sum, nulls/{mean,sum}.rs, over
//   rolling/sum.rs:7 SumWindow (Kahan add / subtract of the values entering
//   and leaving the window, inf / NaN counted apart) and mean.rs:6
//   MeanWindow (sum / number of non-null values); window bounds
//   rolling/mod.rs:68 det_offsets / :71 det_offsets_center; validity
//   mod.rs:79 create_validity and sum.rs:203 is_valid (non-null count >=
//   min_periods).
//
// MI355X design: a workgroup owns 1024 consecutive
// outputs.  It stages the inputs their windows cover (<= 2048 or 4096
// values) in LDS as exact 120-bit fixed-point integers (three carry-free
// 40-bit limbs) relative to the tile's own exponent window, plus packed
// non-null / +inf / -inf / NaN counts, and prefix-scans them.  Every output
// is then two prefix reads: the exact window sum, rounded once.  A tile
// whose values span more binades than one window (or a window wider than
// the LDS stage) takes the per-output exact path (Shewchuk partials, as
// math.fsum).  f64 results are therefore the correctly rounded window sums
// (the reference's Kahan fold agrees within 1 ULP); integer sums wrap like
// the reference's integer SumWindow.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>

#include "plgpu_internal.hpp"
#include "scan.hpp"

namespace plgpu {

constexpr int kRlThreads = 256;
constexpr int kRlOut = 1024;  // outputs per workgroup (4 per thread)

struct RlParams {
    DevCol c;
    int64_t n;
    int64_t w;
    int64_t min_periods;
    int32_t center;
    int32_t mean;
    int32_t isf;      // f64 input (else integer)
    int32_t out_int;  // integer sum output (I64 / I32)
    void* out;
    uint64_t* out_valid;  // always written (one word per 64 outputs)
};

__device__ __forceinline__ void rl_bounds(const RlParams& p, int64_t i, int64_t& s, int64_t& e) {
    if (p.center) {
        const int64_t right = (p.w + 1) / 2;
        const int64_t left = p.w - right;
        s = i > left ? i - left : 0;
        e = i + right < p.n ? i + right : p.n;
    } else {
        s = i + 1 > p.w ? i + 1 - p.w : 0;
        e = i + 1;
    }
}

__device__ __forceinline__ uint64_t rl_bits(const RlParams& p, int64_t r) {
    const uint64_t b = dev_load(p.c, r);
    return p.isf ? b : f64_bits((double)(int64_t)b);
}

// Exact sum of the finite values of [s, e) (Shewchuk partials + the
// half-way correction of CPython's math.fsum).
__device__ double rl_exact_sum(const RlParams& p, int64_t s, int64_t e) {
    double part[64];
    int np = 0;
    for (int64_t r = s; r < e; ++r) {
        if (!dev_valid(p.c, r)) continue;
        double x = as_f64(rl_bits(p, r));
        if (!__builtin_isfinite(x)) continue;
        int i = 0;
        for (int j = 0; j < np; ++j) {
            double y = part[j];
            if (fabs(x) < fabs(y)) {
                const double t = x;
                x = y;
                y = t;
            }
            const double hi = x + y;
            const double lo = y - (hi - x);
            if (lo != 0.0) part[i++] = lo;
            x = hi;
        }
        if (i < 64) part[i++] = x;
        np = i;
    }
    double hi = 0.0;
    if (np > 0) {
        int n = np - 1;
        hi = part[n];
        double lo = 0.0;
        while (n > 0) {
            const double x = hi;
            const double y = part[--n];
            hi = x + y;
            const double yr = hi - x;
            lo = y - yr;
            if (lo != 0.0) break;
        }
        if (n > 0 && ((lo < 0.0 && part[n - 1] < 0.0) || (lo > 0.0 && part[n - 1] > 0.0))) {
            const double y = lo * 2.0;
            const double x = hi + y;
            const double yr = x - hi;
            if (y == yr) hi = x;
        }
    }
    return hi;
}

// Packed counts: non-null | +inf << 16 | -inf << 32 | NaN << 48 (each < 2^16).
constexpr uint64_t kC1 = 1ull, kCPinf = 1ull << 16, kCNinf = 1ull << 32, kCNan = 1ull << 48;

struct RlCounts {
    int64_t nn, pinf, ninf, nan;  // non-null, +inf, -inf, NaN values of the window
};

__device__ __forceinline__ RlCounts rl_unpack(uint64_t c) {
    return {(int64_t)(c & 0xFFFF), (int64_t)((c >> 16) & 0xFFFF), (int64_t)((c >> 32) & 0xFFFF),
            (int64_t)(c >> 48)};
}

__device__ __forceinline__ void rl_count(const RlParams& p, int64_t r, RlCounts& k) {
    if (!dev_valid(p.c, r)) return;
    ++k.nn;
    if (p.out_int) return;
    const uint64_t b = rl_bits(p, r);
    const uint64_t ab = b & 0x7fffffffffffffffull;
    if (ab > 0x7ff0000000000000ull) ++k.nan;
    else if (ab == 0x7ff0000000000000ull) ++((b >> 63) ? k.ninf : k.pinf);
}

__device__ __forceinline__ void rl_write(const RlParams& p, int64_t i, double sum, int64_t isum, const RlCounts& k,
                                         int64_t len, bool& valid) {
    const int64_t nn = k.nn, pinf = k.pinf, ninf = k.ninf, nan = k.nan;
    valid = (int64_t)nn >= p.min_periods && len > 0;
    if (p.mean && nn == 0) valid = false;
    if (p.out_int) {
        if (p.out_int == PLGPU_I64) ((int64_t*)p.out)[i] = valid ? isum : 0;
        else ((int32_t*)p.out)[i] = valid ? (int32_t)isum : 0;
        return;
    }
    double r = sum;
    if (nan || (pinf && ninf)) r = __builtin_nan("");
    else if (pinf) r = __builtin_inf();
    else if (ninf) r = -__builtin_inf();
    if (p.mean) r = r / (double)nn;
    ((double*)p.out)[i] = valid ? r : 0.0;
}

// One workgroup = kRlOut outputs; ELEMS = LDS stage size.
template <int ELEMS>
__global__ __launch_bounds__(kRlThreads) void rl_tile_kernel(RlParams p) {
    constexpr int PER = ELEMS / kRlThreads;
    __shared__ uint64_t L0[ELEMS], L1[ELEMS], L2[ELEMS];  // wrapping prefix sums
    __shared__ uint64_t CN[ELEMS];
    __shared__ uint64_t wsum[kRlThreads / 64];
    __shared__ uint32_t red[2];
    const int tid = threadIdx.x;
    const int64_t o0 = (int64_t)blockIdx.x * kRlOut;
    const int64_t o1 = o0 + kRlOut < p.n ? o0 + kRlOut : p.n;
    int64_t lo, hi, tmp;
    rl_bounds(p, o0, lo, tmp);
    rl_bounds(p, o1 - 1, tmp, hi);
    const int m = (int)(hi - lo);  // staged values (<= ELEMS by the host's choice)
    // pass 1: exponent range of the finite nonzero values
    if (tid == 0) {
        red[0] = 0;
        red[1] = 0;
    }
    __syncthreads();
    uint32_t mx = 0, inv_mn = 0;
    {
        for (int j = tid; j < m; j += kRlThreads) {
            const int64_t r = lo + j;
            if (!dev_valid(p.c, r)) continue;
            const uint64_t b = rl_bits(p, r);
            const uint32_t ex = (uint32_t)(b >> 52) & 0x7FF;
            if (ex == 0x7FF || (b << 1) == 0) continue;
            const uint32_t e1 = ex ? ex : 1;
            mx = e1 > mx ? e1 : mx;
            inv_mn = 0x7FF - e1 > inv_mn ? 0x7FF - e1 : inv_mn;
        }
    }
    atomicMax(&red[0], mx);
    atomicMax(&red[1], inv_mn);
    __syncthreads();
    const int tmax = (int)red[0], tmin = 0x7FF - (int)red[1];
    const bool exact_path = !p.out_int && tmax > 0 && tmax - tmin > kSumWindowBits - 53;
    if (exact_path) {
        // values too far apart for one window: exact per-output summation
        for (int64_t i = o0 + tid; i < o1; i += kRlThreads) {
            int64_t s, e;
            rl_bounds(p, i, s, e);
            RlCounts k = {0, 0, 0, 0};
            for (int64_t r = s; r < e; ++r) rl_count(p, r, k);
            bool valid;
            rl_write(p, i, rl_exact_sum(p, s, e), 0, k, e - s, valid);
            const uint64_t wv = __ballot(valid);
            if ((tid & 63) == 0) p.out_valid[i >> 6] = wv;  // i of lane 0 is a multiple of 64
        }
        return;
    }
    const int bottom = (tmax > 0 ? tmax : 1) - 1075 - (kSumWindowBits - 53);
    // pass 2: stage limbs / counts, thread-contiguous chunks
    const int j0 = tid * PER;
    uint64_t a0 = 0, a1 = 0, a2 = 0, ac = 0;
#pragma unroll 4
    for (int k = 0; k < PER; ++k) {
        const int j = j0 + k;
        uint64_t l0 = 0, l1 = 0, l2 = 0, c = 0;
        if (j < m) {
            const int64_t r = lo + j;
            if (dev_valid(p.c, r)) {
                c = kC1;
                if (p.out_int) {
                    l0 = dev_load(p.c, r);
                } else {
                    const uint64_t b = rl_bits(p, r);
                    const uint64_t ab = b & 0x7fffffffffffffffull;
                    if (ab > 0x7ff0000000000000ull) c += kCNan;
                    else if (ab == 0x7ff0000000000000ull) c += (b >> 63) ? kCNinf : kCPinf;
                    else {
                        uint64_t x0, x1, x2;
                        uint32_t fl = 0, ex = 0;
                        if (fx_limbs<kSumWindowBits>(b, bottom, x0, x1, x2, fl, ex)) {
                            l0 = x0;
                            l1 = x1;
                            l2 = x2;
                        }
                    }
                }
            }
        }
        a0 += l0;
        a1 += l1;
        a2 += l2;
        ac += c;
        if (j < ELEMS) {
            L0[j] = a0;
            L1[j] = a1;
            L2[j] = a2;
            CN[j] = ac;
        }
    }
    // block scan of the thread totals, added to each chunk
    uint64_t t0, t1, t2, tc;
    const uint64_t b0 = block_excl_scan(a0, wsum, t0);
    const uint64_t b1 = block_excl_scan(a1, wsum, t1);
    const uint64_t b2 = block_excl_scan(a2, wsum, t2);
    const uint64_t bc = block_excl_scan(ac, wsum, tc);
    for (int k = 0; k < PER; ++k) {
        const int j = j0 + k;
        L0[j] += b0;
        L1[j] += b1;
        L2[j] += b2;
        CN[j] += bc;
    }
    __syncthreads();
    // outputs: window [s, e) -> inclusive prefixes at e-1 and s-1
    for (int64_t i = o0 + tid; i < o1 + ((o1 - o0) % 64 ? 64 - (o1 - o0) % 64 : 0); i += kRlThreads) {
        bool valid = false;
        if (i < o1) {
            int64_t s, e;
            rl_bounds(p, i, s, e);
            const int je = (int)(e - lo) - 1, js = (int)(s - lo) - 1;
            uint64_t s0 = 0, s1 = 0, s2 = 0, cnt = 0;
            if (je >= 0) {
                s0 = L0[je];
                s1 = L1[je];
                s2 = L2[je];
                cnt = CN[je];
            }
            if (js >= 0) {
                s0 -= L0[js];
                s1 -= L1[js];
                s2 -= L2[js];
                cnt -= CN[js];
            }
            double sum = 0.0;
            if (!p.out_int) {
                uint64_t w0, w1, w2;
                limbs_to_192((int64_t)s0, (int64_t)s1, (int64_t)s2, w0, w1, w2);
                sum = fx_to_double(w0, w1, w2, bottom);
            }
            rl_write(p, i, sum, (int64_t)s0, rl_unpack(cnt), e - s, valid);
        }
        const uint64_t wv = __ballot(valid);
        if ((tid & 63) == 0 && i < o1) p.out_valid[i >> 6] = wv;
    }
}

// Small windows (w <= kSlideMaxW): a workgroup stages 4096 outputs' inputs
// in LDS (coalesced), then each thread slides an exact fixed-point window
// over 16 consecutive outputs: per output, the limbs of the value entering
// are added and those of the value leaving subtracted (integer arithmetic,
// so no drift), and the sum is rounded once.  Outputs go back through LDS
// so the global stores are coalesced.
constexpr int kSlideMaxW = 64;
constexpr int kSlideRun = 8;
constexpr int kSlideOut = kRlThreads * kSlideRun;  // 2048

struct RlAcc {
    int64_t l0, l1, l2, isum;
    int32_t nn, pinf, ninf, nan;
};

// Limbs of a finite value known to lie in the tile's window (zero allowed):
// t = +-m * 2^sh split as l0 + l1 * 2^40 + l2 * 2^80 (low limbs >= 0, top
// limb signed), branch-free.
__device__ __forceinline__ void rl_limbs(uint64_t b, int bottom, int64_t& l0, int64_t& l1, int64_t& l2) {
    constexpr uint64_t M40 = (1ull << 40) - 1;
    const uint32_t ex = (uint32_t)(b >> 52) & 0x7FF;
    const uint64_t m = (b & 0x000FFFFFFFFFFFFFull) | ((uint64_t)(ex != 0) << 52);
    const int sh0 = (int)(ex ? ex : 1) - 1075 - bottom;
    const uint32_t sh = sh0 < 0 ? 0u : (uint32_t)sh0;  // only zero can fall below (m == 0)
    const int64_t sm = (int64_t)b < 0 ? -(int64_t)m : (int64_t)m;
    l0 = sh < 40 ? (int64_t)(((uint64_t)sm << sh) & M40) : 0;
    l1 = (int64_t)((sh <= 40 ? (uint64_t)(sm >> (40 - sh)) : ((uint64_t)sm << (sh - 40))) & M40);
    l2 = sm >> (sh > 16 ? 80 - sh : 63);
}

// Correctly rounded double of (l0 + l1*2^40 + l2*2^80) * 2^bottom for limb
// sums of at most a few thousand values (|total| < 2^126): the magnitude is
// normalised, its top 64 bits carry a sticky bit for the rest (round to
// odd), and one u64 -> f64 conversion rounds.  Results that would be
// subnormal take fx_to_double.
__device__ __forceinline__ double rl_to_double(int64_t l0, int64_t l1, int64_t l2, int bottom) {
    const __int128 t = (__int128)l0 + ((__int128)l1 << 40) + ((__int128)l2 << 80);
    if (t == 0) return 0.0;
    const bool neg = t < 0;
    unsigned __int128 u = neg ? (unsigned __int128)(-t) : (unsigned __int128)t;
    const uint64_t hi = (uint64_t)(u >> 64);
    const int lz = hi ? __clzll(hi) : 64 + __clzll((uint64_t)u);
    u <<= lz;
    const uint64_t top = (uint64_t)(u >> 64) | (((uint64_t)u) != 0 ? 1ull : 0ull);
    const int e = 64 - lz + bottom;  // value ~= top * 2^e, leading bit at 2^(63 + e)
    if (63 + e < -1021) {
        uint64_t w0, w1, w2;
        limbs_to_192(l0, l1, l2, w0, w1, w2);
        return fx_to_double(w0, w1, w2, bottom);
    }
    const double r = __builtin_ldexp((double)top, e);
    return neg ? -r : r;
}

template <bool NULLABLE>
__device__ __forceinline__ void rl_acc(const RlParams& p, const uint64_t* vals, const uint8_t* vld, int j, int bottom,
                                       int sign, RlAcc& a) {
    if (NULLABLE && !vld[j]) return;
    a.nn += sign;
    const uint64_t b = vals[j];
    if (p.out_int) {
        a.isum = (int64_t)((uint64_t)a.isum + (uint64_t)(sign > 0 ? b : 0ull - b));
        return;
    }
    const uint64_t ab = b & 0x7fffffffffffffffull;
    if (ab >= 0x7ff0000000000000ull) {
        if (ab > 0x7ff0000000000000ull) a.nan += sign;
        else if (b >> 63) a.ninf += sign;
        else a.pinf += sign;
        return;
    }
    int64_t x0, x1, x2;
    rl_limbs(b, bottom, x0, x1, x2);
    if (sign > 0) {
        a.l0 += x0;
        a.l1 += x1;
        a.l2 += x2;
    } else {
        a.l0 -= x0;
        a.l1 -= x1;
        a.l2 -= x2;
    }
}

template <bool NULLABLE>
__global__ __launch_bounds__(kRlThreads) void rl_slide_kernel(RlParams p) {
    __shared__ uint64_t vals[kSlideOut + kSlideMaxW];
    __shared__ uint8_t vld[NULLABLE ? kSlideOut + kSlideMaxW : 1];
    __shared__ uint64_t outv[kSlideOut];
    __shared__ uint64_t outm[kSlideOut / 64];
    __shared__ uint32_t red[2];
    const int tid = threadIdx.x;
    const int64_t o0 = (int64_t)blockIdx.x * kSlideOut;
    const int64_t o1 = o0 + kSlideOut < p.n ? o0 + kSlideOut : p.n;
    int64_t lo, hi, tmp;
    rl_bounds(p, o0, lo, tmp);
    rl_bounds(p, o1 - 1, tmp, hi);
    const int m = (int)(hi - lo);
    if (tid < 2) red[tid] = 0;
    if (tid < kSlideOut / 64) outm[tid] = 0;
    __syncthreads();
    uint32_t mx = 0, inv_mn = 0;
    for (int j = tid; j < m; j += kRlThreads) {
        const int64_t r = lo + j;
        const bool v = !NULLABLE || dev_valid(p.c, r);
        const uint64_t b = p.out_int ? dev_load(p.c, r) : rl_bits(p, r);
        vals[j] = b;
        if (NULLABLE) vld[j] = v;
        if (!p.out_int && v) {
            const uint32_t ex = (uint32_t)(b >> 52) & 0x7FF;
            if (ex != 0x7FF && (b << 1) != 0) {
                const uint32_t e1 = ex ? ex : 1;
                mx = e1 > mx ? e1 : mx;
                inv_mn = 0x7FF - e1 > inv_mn ? 0x7FF - e1 : inv_mn;
            }
        }
    }
    atomicMax(&red[0], mx);
    atomicMax(&red[1], inv_mn);
    __syncthreads();
    const int tmax = (int)red[0], tmin = 0x7FF - (int)red[1];
    const bool exact_path = !p.out_int && tmax > 0 && tmax - tmin > kSumWindowBits - 53;
    const int bottom = (tmax > 0 ? tmax : 1) - 1075 - (kSumWindowBits - 53);
    const int64_t i0 = o0 + (int64_t)tid * kSlideRun;
    RlAcc a = {0, 0, 0, 0, 0, 0, 0, 0};
    int64_t ps = 0, pe = 0;
    for (int k = 0; k < kSlideRun; ++k) {
        const int64_t i = i0 + k;
        if (i >= o1) break;
        int64_t s, e;
        rl_bounds(p, i, s, e);
        double sum = 0.0;
        RlCounts cnt;
        if (exact_path) {
            cnt = {0, 0, 0, 0};
            for (int64_t r = s; r < e; ++r) rl_count(p, r, cnt);
            sum = rl_exact_sum(p, s, e);
        } else {
            if (k == 0) {
                for (int64_t r = s; r < e; ++r) rl_acc<NULLABLE>(p, vals, vld, (int)(r - lo), bottom, 1, a);
            } else {
                for (int64_t r = ps; r < s; ++r) rl_acc<NULLABLE>(p, vals, vld, (int)(r - lo), bottom, -1, a);
                for (int64_t r = pe; r < e; ++r) rl_acc<NULLABLE>(p, vals, vld, (int)(r - lo), bottom, 1, a);
            }
            cnt = {a.nn, a.pinf, a.ninf, a.nan};
            if (!p.out_int) sum = rl_to_double(a.l0, a.l1, a.l2, bottom);
        }
        ps = s;
        pe = e;
        bool valid;
        RlParams q = p;  // write into the LDS staging buffer (index i - o0)
        q.out = outv;
        q.out_int = p.out_int ? PLGPU_I64 : 0;
        rl_write(q, i - o0, sum, a.isum, cnt, e - s, valid);
        if (valid) atomicOr((unsigned long long*)&outm[(i - o0) >> 6], 1ull << ((i - o0) & 63));
    }
    __syncthreads();
    // coalesced write-out of values and validity words
    for (int j = tid; j < (int)(o1 - o0); j += kRlThreads) {
        const int64_t i = o0 + j;
        if (!p.out_int) ((double*)p.out)[i] = __longlong_as_double((long long)outv[j]);
        else if (p.out_int == PLGPU_I64) ((int64_t*)p.out)[i] = (int64_t)outv[j];
        else ((int32_t*)p.out)[i] = (int32_t)(int64_t)outv[j];
    }
    for (int j = tid; j < (int)((o1 - o0 + 63) / 64); j += kRlThreads) p.out_valid[(o0 >> 6) + j] = outm[j];
}

// Windows too wide for the LDS stage: per-output direct summation.
__global__ void rl_direct_kernel(RlParams p) {
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < p.n; base += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = base + threadIdx.x;
        bool valid = false;
        if (i < p.n) {
            int64_t s, e;
            rl_bounds(p, i, s, e);
            RlCounts k = {0, 0, 0, 0};
            uint64_t isum = 0;
            for (int64_t r = s; r < e; ++r) {
                rl_count(p, r, k);
                if (p.out_int && dev_valid(p.c, r)) isum += dev_load(p.c, r);  // wrapping, like SumWindow<int>
            }
            const double sum = p.out_int ? 0.0 : rl_exact_sum(p, s, e);
            rl_write(p, i, sum, (int64_t)isum, k, e - s, valid);
        }
        const uint64_t wv = __ballot(valid);
        if ((threadIdx.x & 63) == 0 && i < p.n) p.out_valid[i >> 6] = wv;
    }
}

}  // namespace plgpu

using namespace plgpu;

// ------------------------------------------------------- rolling min / max
// polars-compute/src/rolling/{no_nulls,nulls}/min_max.rs (MinMaxWindow with
// MinPropagateNan / MaxPropagateNan): a NaN in the window gives NaN, nulls
// are skipped, fewer than min_periods values (or none) give null.
// Values become order-preserving u64 codes in which NaN is the extreme that
// wins (0 for min, ~0 for max) and a null is the identity, so a window's
// answer is one unsigned min / max.  Windows of up to kMmDirect rows scan
// their rows directly (neighbouring outputs share cached lines); longer
// ones use van Herk / Gil-Werman: per aligned block of w rows, prefix and
// suffix extrema, so every window -- full length w, or clipped at either end
// of the column -- is min(suffix[s], prefix[e - 1]) in O(1).
constexpr int64_t kMmDirect = 64;

struct MmParams {
    DevCol c;
    int64_t n;
    int64_t w;
    int64_t min_periods;
    int32_t center;
    int32_t is_max;
    int32_t isf;
    int32_t out_dtype;
    void* out;
    uint64_t* out_valid;
    uint64_t* pre;           // van Herk prefix codes (or null)
    uint64_t* suf;           // van Herk suffix codes
    const uint64_t* vcount;  // exclusive prefix counts of valid rows (nulls only), n + 1
};

__device__ __forceinline__ uint64_t mm_code(const MmParams& p, int64_t r) {
    if (!dev_valid(p.c, r)) return p.is_max ? 0ull : ~0ull;
    const uint64_t b = dev_load(p.c, r);
    if (p.isf) {
        if ((b & 0x7fffffffffffffffull) > 0x7ff0000000000000ull) return p.is_max ? ~0ull : 0ull;  // NaN wins
        return ord_f64(b);
    }
    return b ^ 0x8000000000000000ull;  // ord_i64 of the sign-extended value
}

__device__ __forceinline__ uint64_t mm_best(const MmParams& p, uint64_t a, uint64_t b) {
    return p.is_max ? (a > b ? a : b) : (a < b ? a : b);
}

__device__ __forceinline__ void mm_bounds(const MmParams& p, int64_t i, int64_t& s, int64_t& e) {
    if (p.center) {
        const int64_t right = (p.w + 1) / 2;
        const int64_t left = p.w - right;
        s = i > left ? i - left : 0;
        e = i + right < p.n ? i + right : p.n;
    } else {
        s = i + 1 > p.w ? i + 1 - p.w : 0;
        e = i + 1;
    }
}

// One wave per aligned block of w rows: prefix and suffix extrema, 64 rows
// at a time with a wave scan and a carried running extreme (coalesced).
__global__ __launch_bounds__(256) void mm_blocks_kernel(MmParams p) {
    const int64_t nb = (p.n + p.w - 1) / p.w;
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t ident = p.is_max ? 0ull : ~0ull;
    for (int64_t b = wave; b < nb; b += waves) {
        const int64_t lo = b * p.w, hi = lo + p.w < p.n ? lo + p.w : p.n;
        uint64_t carry = ident;
        for (int64_t c0 = lo; c0 < hi; c0 += 64) {
            const int64_t r = c0 + lane;
            uint64_t x = r < hi ? mm_code(p, r) : ident;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint64_t y = __shfl_up(x, off, 64);
                if (lane >= off) x = mm_best(p, x, y);
            }
            x = mm_best(p, x, carry);
            if (r < hi) p.pre[r] = x;
            carry = __shfl(x, 63, 64);
        }
        carry = ident;
        for (int64_t c1 = hi; c1 > lo; c1 -= 64) {
            const int64_t r = c1 - 64 + lane;  // lanes below lo are outside the block
            uint64_t x = r >= lo ? mm_code(p, r) : ident;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint64_t y = __shfl_down(x, off, 64);
                if (lane + off < 64) x = mm_best(p, x, y);
            }
            x = mm_best(p, x, carry);
            if (r >= lo) p.suf[r] = x;
            carry = __shfl(x, 0, 64);
        }
    }
}

// Windows of up to kMmDirect rows: a workgroup stages the codes of its 1024
// outputs' input span in LDS once (coalesced), then every output scans its
// window there.
constexpr int kMmTile = 1024;
__global__ __launch_bounds__(256) void mm_direct_kernel(MmParams p) {
    __shared__ uint64_t codes[kMmTile + kMmDirect];
    const uint64_t ident = p.is_max ? 0ull : ~0ull;
    const int64_t left = p.center ? p.w - (p.w + 1) / 2 : p.w - 1;  // rows before the output row
    for (int64_t base = (int64_t)blockIdx.x * kMmTile; base < p.n; base += (int64_t)gridDim.x * kMmTile) {
        const int64_t lo = base - left;  // may be negative
        const int span = kMmTile + (int)p.w - 1;
        for (int k = threadIdx.x; k < span; k += blockDim.x) {
            const int64_t r = lo + k;
            codes[k] = (r >= 0 && r < p.n) ? mm_code(p, r) : ident;
        }
        __syncthreads();
        for (int k = threadIdx.x; k < kMmTile; k += blockDim.x) {
            const int64_t i = base + k;
            bool valid = false;
            uint64_t v = 0;
            if (i < p.n) {
                int64_t s, e;
                mm_bounds(p, i, s, e);
                uint64_t best = ident;
                for (int64_t r = s; r < e; ++r) best = mm_best(p, best, codes[r - lo]);
                const int64_t cnt = p.vcount ? (int64_t)(p.vcount[e] - p.vcount[s]) : e - s;
                valid = cnt >= p.min_periods && cnt > 0;
                if (valid) {
                    if (p.isf) v = best == (p.is_max ? ~0ull : 0ull) ? 0x7ff8000000000000ull : unord_f64(best);
                    else v = best ^ 0x8000000000000000ull;
                }
                if (p.out_dtype == PLGPU_I32) ((int32_t*)p.out)[i] = (int32_t)v;
                else ((uint64_t*)p.out)[i] = v;
            }
            const uint64_t wv = __ballot(valid);
            if ((threadIdx.x & 63) == 0 && i < p.n) p.out_valid[i >> 6] = wv;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void mm_out_kernel(MmParams p) {
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < p.n; i0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = i0 + threadIdx.x;
        bool valid = false;
        if (i < p.n) {
            int64_t s, e;
            mm_bounds(p, i, s, e);
            uint64_t best;
            if (p.pre) {
                // [s, e) lies in one block, or spans two adjacent ones
                best = (s / p.w == (e - 1) / p.w && s % p.w != 0) ? p.suf[s]
                       : (s % p.w == 0 ? p.pre[e - 1] : mm_best(p, p.suf[s], p.pre[e - 1]));
            } else {
                best = p.is_max ? 0ull : ~0ull;
                for (int64_t r = s; r < e; ++r) best = mm_best(p, best, mm_code(p, r));
            }
            const int64_t cnt = p.vcount ? (int64_t)(p.vcount[e] - p.vcount[s]) : e - s;
            valid = cnt >= p.min_periods && cnt > 0;
            uint64_t v = 0;
            if (valid) {
                if (p.isf) v = best == (p.is_max ? ~0ull : 0ull) ? 0x7ff8000000000000ull : unord_f64(best);
                else v = best ^ 0x8000000000000000ull;
            }
            if (p.out_dtype == PLGPU_I32) ((int32_t*)p.out)[i] = (int32_t)v;
            else ((uint64_t*)p.out)[i] = v;
        }
        const uint64_t wv = __ballot(valid);
        if ((threadIdx.x & 63) == 0 && i < p.n) p.out_valid[i >> 6] = wv;
    }
}

__global__ __launch_bounds__(256) void mm_valid_flags_kernel(DevCol c, int64_t n, uint8_t* __restrict__ f) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        f[r] = dev_valid(c, r) ? 1 : 0;
}

static int rolling_minmax(const plgpu_column* values, bool is_max, int64_t w, int64_t min_periods, bool center,
                          plgpu_column* out, hipStream_t s) {
    MmParams p;
    std::memset(&p, 0, sizeof p);
    p.c = dev_col(*values);
    p.n = values->length;
    p.w = w;
    p.min_periods = min_periods;
    p.center = center ? 1 : 0;
    p.is_max = is_max ? 1 : 0;
    p.isf = values->dtype == PLGPU_F64;
    p.out_dtype = values->dtype;
    int rc = make_owned_column(out, values->dtype, p.n, true, s);
    if (rc || p.n == 0) return rc;
    p.out = (void*)out->values;
    p.out_valid = (uint64_t*)out->validity;
    uint8_t* flags = nullptr;
    uint64_t* vcount = nullptr;
    uint64_t* part = nullptr;
    hipError_t e = hipSuccess;
    const unsigned g = (unsigned)std::min<int64_t>((p.n + 255) / 256, 256 * 32);
    if (values->validity != nullptr) {
        rc = dev_alloc((void**)&flags, p.n, s);
        if (!rc) rc = dev_alloc((void**)&vcount, (p.n + 1) * 8, s);
        if (!rc) rc = dev_alloc((void**)&part, ((p.n + kScanChunk - 1) / kScanChunk + 2) * 8, s);
        if (!rc) {
            mm_valid_flags_kernel<<<g, 256, 0, s>>>(p.c, p.n, flags);
            e = hipGetLastError();
            if (e == hipSuccess) e = scan_exclusive<uint8_t>(flags, p.n, vcount, part, s);
            p.vcount = vcount;
        }
    }
    if (!rc && e == hipSuccess && w > kMmDirect) {
        rc = dev_alloc((void**)&p.pre, p.n * 8, s);
        if (!rc) rc = dev_alloc((void**)&p.suf, p.n * 8, s);
        if (!rc) {
            const int64_t nb = (p.n + w - 1) / w;  // one wave (of 4 per workgroup) per block
            mm_blocks_kernel<<<(unsigned)std::min<int64_t>((nb + 3) / 4, 256 * 64), 256, 0, s>>>(p);
            e = hipGetLastError();
        }
        if (!rc && e == hipSuccess) {
            mm_out_kernel<<<g, 256, 0, s>>>(p);
            e = hipGetLastError();
        }
    } else if (!rc && e == hipSuccess) {
        mm_direct_kernel<<<(unsigned)std::min<int64_t>((p.n + kMmTile - 1) / kMmTile, 256 * 64), 256, 0, s>>>(p);
        e = hipGetLastError();
    }
    if (!rc && e == hipSuccess) e = hipStreamSynchronize(s);
    if (!rc && e != hipSuccess) rc = hip_fail(e, "rolling min / max");
    dev_free(flags, s);
    dev_free(vcount, s);
    dev_free(part, s);
    dev_free(p.pre, s);
    dev_free(p.suf, s);
    if (rc) plgpu_column_release(out);
    else out->null_count = -1;
    return rc;
}

PLGPU_API int plgpu_rolling(const plgpu_column* values, int32_t kind, int64_t window_size, int64_t min_periods,
                            int32_t center, plgpu_column* out, void* stream) {
    hipStream_t s = as_stream(stream);
    if (values == nullptr || out == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    std::memset(out, 0, sizeof *out);
    if (kind < PLGPU_ROLLING_SUM || kind > PLGPU_ROLLING_MAX) return fail(PLGPU_ERR_INVALID, "unknown rolling kind");
    if (values->dtype != PLGPU_F64 && values->dtype != PLGPU_I64 && values->dtype != PLGPU_I32)
        return fail(PLGPU_ERR_SCHEMA, "rolling input must be Float64 / Int64 / Int32");
    if (window_size < 1) return fail(PLGPU_ERR_INVALID, "window_size must be >= 1");
    if (min_periods < 0) return fail(PLGPU_ERR_INVALID, "min_periods must be >= 0");
    if (min_periods > window_size)
        return fail(PLGPU_ERR_INVALID, "`min_periods` should be <= `window_size`");
    if (kind == PLGPU_ROLLING_MIN || kind == PLGPU_ROLLING_MAX)
        return rolling_minmax(values, kind == PLGPU_ROLLING_MAX, window_size, min_periods, center != 0, out, s);
    RlParams p;
    std::memset(&p, 0, sizeof p);
    p.c.dtype = values->dtype;
    p.c.offset = values->offset;
    p.c.values = values->values;
    p.c.validity = values->validity;
    p.n = values->length;
    p.w = window_size;
    p.min_periods = min_periods;
    p.center = center != 0;
    p.mean = kind == PLGPU_ROLLING_MEAN;
    p.isf = values->dtype == PLGPU_F64;
    p.out_int = (!p.mean && !p.isf) ? values->dtype : 0;
    const int32_t odt = p.out_int ? values->dtype : PLGPU_F64;
    int rc = make_owned_column(out, odt, p.n, true, s);
    if (rc || p.n == 0) return rc;
    p.out = (void*)out->values;
    p.out_valid = (uint64_t*)out->validity;
    const int64_t tiles = (p.n + kRlOut - 1) / kRlOut;
    if (window_size <= kSlideMaxW) {
        const int64_t g = (p.n + kSlideOut - 1) / kSlideOut;
        if (p.c.validity) rl_slide_kernel<true><<<(unsigned)g, kRlThreads, 0, s>>>(p);
        else rl_slide_kernel<false><<<(unsigned)g, kRlThreads, 0, s>>>(p);
    } else if (window_size - 1 + kRlOut <= 2048)
        rl_tile_kernel<2048><<<(unsigned)tiles, kRlThreads, 0, s>>>(p);
    else if (window_size - 1 + kRlOut <= 4096)
        rl_tile_kernel<4096><<<(unsigned)tiles, kRlThreads, 0, s>>>(p);
    else
        rl_direct_kernel<<<(unsigned)std::min<int64_t>((p.n + 255) / 256, 256 * 64), 256, 0, s>>>(p);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        plgpu_column_release(out);
        return hip_fail(e, "rolling");
    }
    out->null_count = -1;
    return PLGPU_OK;
}
