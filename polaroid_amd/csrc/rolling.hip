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

PLGPU_API int plgpu_rolling(const plgpu_column* values, int32_t kind, int64_t window_size, int64_t min_periods,
                            int32_t center, plgpu_column* out, void* stream) {
    hipStream_t s = as_stream(stream);
    if (values == nullptr || out == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    std::memset(out, 0, sizeof *out);
    if (kind != PLGPU_ROLLING_SUM && kind != PLGPU_ROLLING_MEAN) return fail(PLGPU_ERR_INVALID, "unknown rolling kind");
    if (values->dtype != PLGPU_F64 && values->dtype != PLGPU_I64 && values->dtype != PLGPU_I32)
        return fail(PLGPU_ERR_SCHEMA, "rolling input must be Float64 / Int64 / Int32");
    if (window_size < 1) return fail(PLGPU_ERR_INVALID, "window_size must be >= 1");
    if (min_periods < 0) return fail(PLGPU_ERR_INVALID, "min_periods must be >= 0");
    if (min_periods > window_size)
        return fail(PLGPU_ERR_INVALID, "`min_periods` should be <= `window_size`");
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
    if (window_size - 1 + kRlOut <= 2048)
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
