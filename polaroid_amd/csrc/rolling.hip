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
    int32_t var;          // 0: sum / mean; 1: rolling_var; 2: rolling_std
    int32_t ddof;
    int32_t var_f32;      // std of a Float32 column: sqrt of the variance rounded to f32
    int32_t fast_div;     // option rl_div: full windows' means by rw_div
    int32_t var128;       // option rl_var128: rw_var_scan_full's numerators modulo 2^128 where they fit
    int32_t full;         // option rl_full: interior int64-form waves by rw_scan_full
    double rw;            // RN(1 / w)
    double wd;            // w as an f64
    double rw2;           // var / std: RN(1 / (w - ddof)) (w > ddof)
    double wd2;           // var / std: w - ddof as an f64
    uint32_t* rest;       // rl_var_hot_kernel: blocks for rl_var_rest_kernel (word 0: count)
};

// RN(a / w) for a full window (count w) without a division: q0 = RN(a y),
// the exact remainder r = a - w q0 (one fma), q = RN(q0 + r y) with y =
// RN(1 / w) -- correctly rounded for every a and w whose quotient and
// remainder stay normal (Markstein's one-correction theorem; w an integer
// < 2^53, so its significand is never all ones; checked against exact
// rational division over 1.3e6 random (a, w), w = 1 ... 4096 and beyond,
// |a| from 2^-1000 to 2^1000).  Other values take the division.
__device__ __forceinline__ double rw_div(double a, uint64_t cnt, const RlParams& p) {
    const uint32_t ex = (uint32_t)(f64_bits(a) >> 52) & 0x7FF;
    if (cnt == (uint64_t)p.w && ex >= 1023 - 900 && ex <= 1023 + 990) {
        const double y = p.rw, w = p.wd;
        const double q0 = a * y;
        const double r = __builtin_fma(-q0, w, a);
        return __builtin_fma(r, y, q0);
    }
    return a / (double)cnt;
}

__device__ __forceinline__ double rv_std(const RlParams& p, double v) {
    return __builtin_sqrt(p.var_f32 ? (double)(float)v : v);
}

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
    return hi == 0.0 ? 0.0 : hi;  // +0.0, as SumWindow's S::zeroed() start (sum.rs:31)
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

// Small windows (w <= kRwMaxW): wave-scan kernel.  A wave owns kRwOut
// consecutive outputs.  It loads the rows their windows cover once
// (coalesced, held in registers), finds their exponent range, and turns
// every finite value into an exact fixed-point integer relative to the
// smallest exponent: one int64 when the range is narrow enough that any
// window's sum fits 63 bits (prices, volumes: a few binades), else a
// 128-bit integer.  A wave64 prefix scan (DPP row shifts + row broadcasts)
// gives wrapping prefix sums P; every window is P[e-1] - P[s-1], exact
// modulo 2^64 / 2^128 and therefore exact, and it is rounded to f64 once.
// Non-null / +inf / -inf / NaN counts run the same scan only when the
// wave's rows hold a null or a non-finite value.  Prefixes of the last four
// 64-row chunks sit in a per-wave LDS ring, so clipped and centred windows
// read their two prefixes the same way.
constexpr int kRwMaxW = 64;
constexpr int kRwChunks = 8;               // output chunks of 64 per wave
constexpr int kRwWaves = 4;                // waves per workgroup
constexpr int kRwOut = 64 * kRwChunks;     // outputs per wave
constexpr int kRwRing = 256;               // 4 chunks of prefixes

// Inclusive wave64 prefix sum, wrapping: row_shr 1/2/4/8 within rows of 16
// lanes, then row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3), with
// the DPP moves folded into the adds (round 5: 4.0 -> 3.6 ms for
// rolling_mean(20) at 1e9 rows against separate v_mov_b32_dpp + 64-bit
// adds): one 32-bit add with carry-out and one add-with-carry per step,
// src0 read across lanes
// (a lane without a source, or outside the row mask, is not written and
// keeps its value -- x + 0).  s_nop 1: a VALU write read through DPP by the
// next instruction needs two wait states.
__device__ __forceinline__ uint64_t wave_scan64_fused(uint64_t x) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    asm volatile(
        "s_nop 1\n"
        "v_add_co_u32_dpp %0, vcc, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n"
        "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc row_shr:1 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n"
        "v_add_co_u32_dpp %0, vcc, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n"
        "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc row_shr:2 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n"
        "v_add_co_u32_dpp %0, vcc, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n"
        "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc row_shr:4 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n"
        "v_add_co_u32_dpp %0, vcc, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n"
        "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc row_shr:8 row_mask:0xf bank_mask:0xf\n"
        "s_nop 1\n"
        "v_add_co_u32_dpp %0, vcc, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
        "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc row_bcast:15 row_mask:0xa bank_mask:0xf\n"
        "s_nop 1\n"
        "v_add_co_u32_dpp %0, vcc, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
        "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc row_bcast:31 row_mask:0xc bank_mask:0xf\n"
        "s_nop 1\n"
        : "+v"(lo), "+v"(hi)
        :
        : "vcc");
    return ((uint64_t)hi << 32) | lo;
}

// 128-bit form: the carry runs through four 32-bit words.
#define PLGPU_DPP128(CTRL, RM)                                                                    \
    "s_nop 1\n"                                                                                  \
    "v_add_co_u32_dpp %0, vcc, %0, %0 " CTRL " row_mask:" RM " bank_mask:0xf\n"                 \
    "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc " CTRL " row_mask:" RM " bank_mask:0xf\n"           \
    "v_addc_co_u32_dpp %2, vcc, %2, %2, vcc " CTRL " row_mask:" RM " bank_mask:0xf\n"           \
    "v_addc_co_u32_dpp %3, vcc, %3, %3, vcc " CTRL " row_mask:" RM " bank_mask:0xf\n"
__device__ __forceinline__ void wave_scan128_fused(uint64_t& lo, uint64_t& hi) {
    uint32_t w0 = (uint32_t)lo, w1 = (uint32_t)(lo >> 32), w2 = (uint32_t)hi, w3 = (uint32_t)(hi >> 32);
    asm volatile(PLGPU_DPP128("row_shr:1", "0xf") PLGPU_DPP128("row_shr:2", "0xf") PLGPU_DPP128("row_shr:4", "0xf")
                     PLGPU_DPP128("row_shr:8", "0xf") PLGPU_DPP128("row_bcast:15", "0xa")
                         PLGPU_DPP128("row_bcast:31", "0xc") "s_nop 1\n"
                 : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3)
                 :
                 : "vcc");
    lo = ((uint64_t)w1 << 32) | w0;
    hi = ((uint64_t)w3 << 32) | w2;
}
#undef PLGPU_DPP128

__device__ __forceinline__ void add128(uint64_t& lo, uint64_t& hi, uint64_t blo, uint64_t bhi) {
    const uint64_t l = lo + blo;
    hi = hi + bhi + (l < lo ? 1ull : 0ull);
    lo = l;
}


__device__ __forceinline__ uint64_t lane63(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 128-bit two's complement fixed-point value * 2^bottom -> f64, rounded once:
// the magnitude's top 64 bits with a sticky bit for the rest, one u64 -> f64
// conversion, an exact scaling.  Subnormal results take fx_to_double.
__device__ __forceinline__ double i128_to_double(uint64_t lo, uint64_t hi, int bottom) {
    const bool neg = (int64_t)hi < 0;
    uint64_t ml = lo, mh = hi;
    if (neg) {
        ml = ~lo + 1;
        mh = ~hi + (ml == 0 ? 1ull : 0ull);
    }
    if ((ml | mh) == 0) return 0.0;
    const int lz = mh ? __clzll(mh) : 64 + __clzll(ml);
    uint64_t top;
    if (lz >= 64) top = ml << (lz - 64);
    else if (lz == 0) top = mh | (ml != 0 ? 1ull : 0ull);
    else top = (mh << lz) | (ml >> (64 - lz)) | ((ml << lz) != 0 ? 1ull : 0ull);
    const int e = 64 - lz + bottom;
    if (63 + e < -1021) return fx_to_double(lo, hi, neg ? ~0ull : 0ull, bottom);
    const double r = __builtin_ldexp((double)top, e);
    return neg ? -r : r;
}

// One row of a rolling input, as loaded (DT: F64 bits, I64, or I32
// sign-extended); `tof` converts an integer to the bits of its f64 value.
template <int DT>
__device__ __forceinline__ uint64_t rw_load(const RlParams& p, int64_t r, bool tof) {
    const int64_t q = p.c.offset + r;
    if (DT == PLGPU_F64) return ((const uint64_t*)p.c.values)[q];
    const int64_t v = DT == PLGPU_I64 ? ((const int64_t*)p.c.values)[q] : (int64_t)((const int32_t*)p.c.values)[q];
    return tof ? f64_bits((double)v) : (uint64_t)v;
}

// Scan + emit phase of rl_wave_kernel for one number format.  MODE 0:
// integer sums (wrapping, like SumWindow<int>); 1: int64 fixed point;
// 2: 128-bit fixed point.  COUNTS: the wave's rows hold a null or a
// non-finite value, so non-null / inf / NaN counts are scanned too (else a
// window's non-null count is its length).  Straight-line per chunk: every
// branch below is uniform and resolved at compile time or once per wave.
template <int MODE, bool COUNTS, bool MEAN>
__device__ __forceinline__ void rw_scan(const RlParams& p, const uint64_t (&x)[kRwChunks + 1],
                                        const uint64_t (&vm)[kRwChunks + 1], int64_t o_first, int64_t o_end,
                                        int64_t s_first, int tmin, uint64_t* rlo, uint64_t* rhi, uint64_t* rcn) {
    const int lane = threadIdx.x & 63;
    const int bottom = tmin - 1075;
    // interior waves: every window is unclipped, [i - left, i + right)
    const int64_t right = p.center ? (p.w + 1) / 2 : 1;
    const int64_t left = p.w - right;
    const bool interior = o_first - left >= 0 && o_end + right - 1 <= p.n;
    uint64_t carry_lo = 0, carry_hi = 0, carry_cn = 0;
#pragma unroll
    for (int k = 0; k <= kRwChunks; ++k) {
        const uint64_t b = x[k];
        uint64_t flo, fhi = 0, code = 0;
        if (MODE == 0) {
            flo = b;
            if (COUNTS) code = (vm[k] >> lane) & 1;
        } else {
            const uint64_t ab = b & 0x7fffffffffffffffull;
            const bool fin = ab < 0x7ff0000000000000ull;
            if (COUNTS) {
                const bool v = (vm[k] >> lane) & 1;
                code = !v ? 0 : (fin ? kC1 : ab > 0x7ff0000000000000ull ? kC1 + kCNan
                                            : kC1 + ((b >> 63) ? kCNinf : kCPinf));
            }
            const uint32_t ex = (uint32_t)(b >> 52) & 0x7FF;
            const uint64_t m = fin ? ((b & 0x000FFFFFFFFFFFFFull) | ((uint64_t)(ex != 0) << 52)) : 0ull;
            const int sh0 = (int)(ex ? ex : 1) - tmin;
            const uint32_t sh = sh0 < 0 ? 0u : (uint32_t)sh0;  // only zero lies below tmin
            const bool neg = (b >> 63) != 0;
            if (MODE == 1) {
                const uint64_t t = m << sh;
                flo = neg ? 0ull - t : t;
            } else {
                flo = sh < 64 ? m << sh : 0ull;
                fhi = sh == 0 ? 0ull : sh < 64 ? m >> (64 - sh) : m << (sh - 64);
                if (neg) {
                    flo = ~flo + 1;
                    fhi = ~fhi + (flo == 0 ? 1ull : 0ull);
                }
            }
        }
        const int slot = ((k & 3) << 6) | lane;
        if (MODE == 2) {
            wave_scan128_fused(flo, fhi);
            add128(flo, fhi, carry_lo, carry_hi);
            carry_lo = lane63(flo);
            carry_hi = lane63(fhi);
            rhi[slot] = fhi;
        } else {
            flo = wave_scan64_fused(flo) + carry_lo;
            carry_lo = lane63(flo);
        }
        rlo[slot] = flo;
        if (COUNTS) {
            code = wave_scan64_fused(code) + carry_cn;
            carry_cn = lane63(code);
            rcn[slot] = code;
        }
        wave_sync();
        if (k == 0) continue;
        // outputs of chunk q = k - 1: their prefixes lie in row chunks q-1..q+1
        const int q = k - 1;
        if (o_first + 64 * q >= o_end) break;
        const int64_t i = o_first + 64 * q + lane;
        int64_t s, e;
        if (interior) {
            s = i - left;
            e = i + right;
        } else {
            rl_bounds(p, i, s, e);
        }
        const int je = (int)(e - 1 - s_first), js = (int)(s - 1 - s_first);
        const int ie = je & (kRwRing - 1), is = js & (kRwRing - 1);
        uint64_t slo = rlo[ie];
        const uint64_t plo = js >= 0 ? rlo[is] : 0ull;
        double sum = 0.0;
        int64_t isum = 0;
        if (MODE == 2) {
            uint64_t shi = rhi[ie];
            const uint64_t phi = js >= 0 ? rhi[is] : 0ull;
            add128(slo, shi, ~plo, ~phi);
            add128(slo, shi, 1, 0);
            sum = i128_to_double(slo, shi, bottom);
        } else if (MODE == 1) {
            sum = __builtin_ldexp((double)(int64_t)(slo - plo), bottom);
        } else {
            isum = (int64_t)(slo - plo);
        }
        RlCounts c;
        if (COUNTS) c = rl_unpack(rcn[ie] - (js >= 0 ? rcn[is] : 0ull));
        else c = RlCounts{e - s, 0, 0, 0};
        bool valid = i < o_end && c.nn >= p.min_periods && (!MEAN || c.nn > 0);
        if (i < o_end) {
            if (MODE == 0) {
                if (p.out_int == PLGPU_I64) ((int64_t*)p.out)[i] = valid ? isum : 0;
                else ((int32_t*)p.out)[i] = valid ? (int32_t)isum : 0;
            } else {
                double r = sum;
                if (COUNTS) {
                    if (c.nan || (c.pinf && c.ninf)) r = __builtin_nan("");
                    else if (c.pinf) r = __builtin_inf();
                    else if (c.ninf) r = -__builtin_inf();
                }
                if (MEAN) r = p.fast_div ? rw_div(r, c.nn, p) : r / (double)c.nn;
                ((double*)p.out)[i] = valid ? r : 0.0;
            }
        }
        const uint64_t bits = __ballot(valid);
        if (lane == 0) p.out_valid[(o_first >> 6) + q] = bits;
        wave_sync();
    }
}

// rw_scan's common case, an interior wave (every window full, [i - left,
// i + right)) in the int64 form with no null or non-finite row.  Its
// prefixes are not kept in a ring: all kRwChunks + 1 chunks' prefixes fit
// the wave's three rings as one array (rw_block's rlo, 3 * kRwRing words),
// prefix r at word r + 1 and word 0 = 0 for prefix -1, so each output's two
// reads are a per-lane base plus a per-chunk immediate offset, as are the
// stores; the mean is the one-correction quotient with no per-lane range
// test when the wave's exponents keep every window's quotient normal (DIV1,
// rw_block).  Round 5: the general scan's emit took about 60 VALU
// instructions per 64 outputs (64-bit bounds, clipping and count tests,
// ring wrap, store addresses, `1 / w` read back from a spilled SGPR lane).
static_assert(kRwChunks * 64 + 64 + 1 <= 3 * kRwRing, "rw_scan_full: the prefixes in the wave's rings");
template <bool MEAN>
__device__ __forceinline__ void rw_scan_full(const RlParams& p, const uint64_t (&x)[kRwChunks + 1],
                                             int64_t o_first, int64_t o_end, int64_t s_first, int tmin, bool div1,
                                             uint64_t* pre) {
    const int lane = threadIdx.x & 63;
    const int bottom = tmin - 1075;
    const int w = (int)p.w;
    const int right = p.center ? (w + 1) / 2 : 1;
    // the output's window ends at row e0 + j of the wave's rows (j = its index)
    const int e0 = (int)(o_first - s_first) + right - 1;
    const int nout = (int)(o_end - o_first);
    const bool ok = p.w >= p.min_periods;  // (w >= 1: a mean's count is never 0)
    double* ol = (double*)p.out + o_first + lane;
    uint64_t* ov = p.out_valid + (o_first >> 6);
    const uint64_t* pe = pre + 1 + e0 + lane;
    const uint64_t* ps = pe - w;
    uint64_t* pw = pre + 1 + lane;
    // 1 / w and w in VGPRs (as uniform values they spill to VGPR lanes and
    // are read back every chunk)
    double y = p.rw, wd = p.wd;
    asm volatile("" : "+v"(y), "+v"(wd));
    if (lane == 0) pre[0] = 0ull;  // prefix -1
    uint64_t carry = 0;
#pragma unroll
    for (int k = 0; k <= kRwChunks; ++k) {
        // finite, normal or zero (the int64 form has tmin >= 128): m << (ex - tmin)
        const uint64_t b = x[k];
        const uint32_t ex = (uint32_t)(b >> 52) & 0x7FF;
        const uint64_t m = (b & 0x000FFFFFFFFFFFFFull) | (1ull << 52);
        const uint64_t t = ex ? m << (ex - (uint32_t)tmin) : 0ull;
        uint64_t flo = (int64_t)b < 0 ? 0ull - t : t;
        flo = wave_scan64_fused(flo) + carry;
        carry = lane63(flo);
        pw[64 * k] = flo;
        wave_sync();
        if (k == 0) continue;
        const int q = k - 1;
        if (64 * q >= nout) break;
        const uint64_t d = pe[64 * q] - ps[64 * q];
        double r = __builtin_ldexp((double)(int64_t)d, bottom);
        if (MEAN) {
            if (div1) {
                const double q0 = r * y;
                r = __builtin_fma(__builtin_fma(-q0, wd, r), y, q0);
            } else {
                r = r / wd;
            }
        }
        const bool in = 64 * q + lane < nout;
        if (in) ol[64 * q] = ok ? r : 0.0;
        const uint64_t bits = __ballot(in && ok);
        if (lane == 0) ov[q] = bits;
    }
}

// A wave's outputs summed exactly one by one (values spanning more binades
// than 128 bits hold).  Out of line, with its own copy of the parameters, so
// the kernel's parameters never have their address taken.
__device__ __noinline__ void rw_exact_outputs(RlParams p, int64_t o_first, int64_t o_end) {
    const int lane = threadIdx.x & 63;
    for (int q = 0; q < kRwChunks; ++q) {
        const int64_t i = o_first + 64 * q + lane;
        if (o_first + 64 * q >= o_end) break;
        bool valid = false;
        if (i < o_end) {
            int64_t s, e;
            rl_bounds(p, i, s, e);
            RlCounts k = {0, 0, 0, 0};
            for (int64_t r = s; r < e; ++r) rl_count(p, r, k);
            rl_write(p, i, rl_exact_sum(p, s, e), 0, k, e - s, valid);
        }
        const uint64_t bits = __ballot(valid);
        if (lane == 0) p.out_valid[(o_first >> 6) + q] = bits;
    }
}

// ----------------------------------------------------- rolling var / std
// polars-compute/src/rolling/moment.rs:138 MomentWindow<VarianceMoment>
// slides a Welford VarState (polars-compute/src/moment.rs:87,99,126) over
// the window; a non-finite value enters as 0.0 and makes the result NaN,
// nulls are skipped, and the result is null below min_periods non-null
// values or at a count <= ddof.  Here every window's variance is formed
// from exact sums: with c the non-null count and the values x = t * 2^b
// (t integers over the wave's smallest exponent),
//   var = (RN(c * sum t^2 - (sum t)^2) * 2^(2b) / c) / (c - ddof),
// the numerator exact and rounded once -- the group-by's fused variance
// (groupby.hip var_exact) per window -- and std its square root.
// Fast form (the wave's values within a few binades, none tiny): wave
// prefix scans of t (int64) and t^2 (128-bit), as the window sums.  Other
// waves: each output summed exactly in big integers (rw_var_exact_outputs).
constexpr int kRvL = 68;  // 4352-bit integers: c * sum t^2 for any finite f64 window of <= 2^16 values

// a += (neg ? -1 : 1) * (v << sh), two's complement over kRvL words.
__device__ __forceinline__ void rv_add(uint64_t* a, unsigned __int128 v, int sh, bool neg) {
    const int ws = sh >> 6, bs = sh & 63;
    const uint64_t lo = (uint64_t)v, hi = (uint64_t)(v >> 64);
    const uint64_t d0 = bs ? lo << bs : lo;
    const uint64_t d1 = bs ? (hi << bs) | (lo >> (64 - bs)) : hi;
    const uint64_t d2 = bs ? hi >> (64 - bs) : 0ull;
    uint64_t c = 0;
    for (int i = ws; i < kRvL; ++i) {
        const int k = i - ws;
        const uint64_t d = k == 0 ? d0 : (k == 1 ? d1 : (k == 2 ? d2 : 0ull));
        if (k >= 3 && c == 0) break;
        if (!neg) {
            const unsigned __int128 t = (unsigned __int128)a[i] + d + c;
            a[i] = (uint64_t)t;
            c = (uint64_t)(t >> 64);
        } else {
            const unsigned __int128 t = (unsigned __int128)a[i] - d - c;
            a[i] = (uint64_t)t;
            c = (uint64_t)(t >> 64) ? 1ull : 0ull;
        }
    }
}

// a (>= 0) * 2^e rounded to nearest-even f64, subnormal results included.
__device__ double rv_round(const uint64_t* a, int e) {
    int top = kRvL - 1;
    while (top >= 0 && a[top] == 0) --top;
    if (top < 0) return 0.0;
    const int pl = top * 64 + 63 - __clzll(a[top]);
    int q = pl - 52;
    if (q + e < -1074) q = -1074 - e;
    if (q <= 0) return __builtin_ldexp((double)a[0], e);  // < 2^53: exact
    auto bit = [&](int b) -> uint64_t { return (a[b >> 6] >> (b & 63)) & 1ull; };
    uint64_t keep = 0;
    for (int b = pl; b >= q; --b) keep = (keep << 1) | bit(b);
    const bool rnd = bit(q - 1) != 0;
    bool sticky = false;
    for (int b = 0; b < q - 1 && !sticky; ++b) sticky = bit(b) != 0;
    if (rnd && (sticky || (keep & 1))) ++keep;
    return __builtin_ldexp((double)keep, q + e);
}

// Exact variance of the non-null values of [s, e) (any finite values).
__device__ double rv_window_exact(const RlParams& p, int64_t s, int64_t e, int64_t c) {
    int emin = 1 << 20;
    for (int64_t r = s; r < e; ++r) {
        if (!dev_valid(p.c, r)) continue;
        const uint64_t b = rl_bits(p, r);
        const uint32_t ex = (uint32_t)(b >> 52) & 0x7FF;
        if (ex == 0x7FF || (b << 1) == 0) continue;
        const int e0 = (int)(ex ? ex : 1) - 1075;  // x = t * 2^e0, t < 2^53
        emin = e0 < emin ? e0 : emin;
    }
    if (emin == 1 << 20) return 0.0;
    uint64_t sq[kRvL], s1[kRvL], num[kRvL];
    for (int i = 0; i < kRvL; ++i) sq[i] = s1[i] = num[i] = 0;
    for (int64_t r = s; r < e; ++r) {
        if (!dev_valid(p.c, r)) continue;
        const uint64_t b = rl_bits(p, r);
        const uint32_t ex = (uint32_t)(b >> 52) & 0x7FF;
        if (ex == 0x7FF || (b << 1) == 0) continue;
        const uint64_t t = (b & 0x000FFFFFFFFFFFFFull) | ((uint64_t)(ex != 0) << 52);
        const int sh = (int)(ex ? ex : 1) - 1075 - emin;
        rv_add(sq, (unsigned __int128)t * t, 2 * sh, false);
        rv_add(s1, t, sh, (b >> 63) != 0);
    }
    for (int i = 0; i < kRvL; ++i)
        if (sq[i]) rv_add(num, (unsigned __int128)sq[i] * (uint64_t)c, 64 * i, false);
    if ((int64_t)s1[kRvL - 1] < 0) {  // |sum t|
        uint64_t cy = 1;
        for (int i = 0; i < kRvL; ++i) {
            const unsigned __int128 t = (unsigned __int128)(~s1[i]) + cy;
            s1[i] = (uint64_t)t;
            cy = (uint64_t)(t >> 64);
        }
    }
    for (int i = 0; i < kRvL; ++i) {
        if (!s1[i]) continue;
        for (int j = 0; i + j < kRvL; ++j)
            if (s1[j]) rv_add(num, (unsigned __int128)s1[i] * s1[j], 64 * (i + j), true);
    }
    if ((int64_t)num[kRvL - 1] < 0) return 0.0;  // (c sum t^2 >= (sum t)^2: unreachable)
    const double nr = rv_round(num, 2 * emin);
    return (nr / (double)c) / (double)(c - p.ddof);
}

// A wave's outputs one by one, exactly (out of line: its big integers live
// in private memory; only waves whose values the fast form cannot hold).
__device__ __noinline__ void rw_var_exact_outputs(RlParams p, int64_t o_first, int64_t o_end) {
    const int lane = threadIdx.x & 63;
    for (int q = 0; q < kRwChunks; ++q) {
        const int64_t i = o_first + 64 * q + lane;
        if (o_first + 64 * q >= o_end) break;
        bool valid = false;
        if (i < o_end) {
            int64_t s, e;
            rl_bounds(p, i, s, e);
            RlCounts k = {0, 0, 0, 0};
            for (int64_t r = s; r < e; ++r) rl_count(p, r, k);
            valid = k.nn >= p.min_periods && k.nn > p.ddof;
            double v = 0.0;
            if (valid) {
                v = (k.nan || k.pinf || k.ninf) ? __builtin_nan("") : rv_window_exact(p, s, e, k.nn);
                if (p.var == 2) v = rv_std(p, v);
            }
            ((double*)p.out)[i] = valid ? v : 0.0;
        }
        const uint64_t bits = __ballot(valid);
        if (lane == 0) p.out_valid[(o_first >> 6) + q] = bits;
    }
}

// |v| of a 192-bit value's... (w2:w1:w0, >= 0) * 2^e as f64, rounded once
// (no subnormal results: the fast form's values are not tiny).
__device__ __forceinline__ double u192_to_double(uint64_t w0, uint64_t w1, uint64_t w2, int e) {
    if ((w0 | w1 | w2) == 0) return 0.0;
    uint64_t top, rest;
    int sh;
    if (w2) {
        const int lz = __clzll(w2);
        top = lz ? (w2 << lz) | (w1 >> (64 - lz)) : w2;
        rest = (lz ? w1 << lz : w1) | w0;
        sh = 128 - lz;
    } else if (w1) {
        const int lz = __clzll(w1);
        top = lz ? (w1 << lz) | (w0 >> (64 - lz)) : w1;
        rest = lz ? w0 << lz : w0;
        sh = 64 - lz;
    } else {
        const int lz = __clzll(w0);
        top = w0 << lz;
        rest = 0;
        sh = -lz;
    }
    top |= rest != 0 ? 1ull : 0ull;  // sticky: one u64 -> f64 rounding is then exact-once
    return __builtin_ldexp((double)top, sh + e);
}

// Scan + emit of the fast form: prefix sums of t (int64), t^2 (128-bit)
// and, with COUNTS, the non-null / inf / NaN counts; per output the exact
// window sums S1, S2 give num = c * S2 - S1^2 (192-bit, exact).
template <bool COUNTS>
__device__ __forceinline__ void rw_var_scan(const RlParams& p, const uint64_t (&x)[kRwChunks + 1],
                                            const uint64_t (&vm)[kRwChunks + 1], int64_t o_first, int64_t o_end,
                                            int64_t s_first, int tmin, uint64_t* r1, uint64_t* r2l, uint64_t* r2h,
                                            uint64_t* rcn) {
    const int lane = threadIdx.x & 63;
    const int bottom = tmin - 1075;
    const int64_t right = p.center ? (p.w + 1) / 2 : 1;
    const int64_t left = p.w - right;
    const bool interior = o_first - left >= 0 && o_end + right - 1 <= p.n;
    uint64_t c1 = 0, c2l = 0, c2h = 0, ccn = 0;
#pragma unroll
    for (int k = 0; k <= kRwChunks; ++k) {
        const uint64_t b = x[k];
        const uint64_t ab = b & 0x7fffffffffffffffull;
        const bool fin = ab < 0x7ff0000000000000ull;
        uint64_t code = 0;
        if (COUNTS) {
            const bool v = (vm[k] >> lane) & 1;
            code = !v ? 0 : (fin ? kC1 : ab > 0x7ff0000000000000ull ? kC1 + kCNan
                                        : kC1 + ((b >> 63) ? kCNinf : kCPinf));
        }
        const uint32_t ex = (uint32_t)(b >> 52) & 0x7FF;
        const uint64_t m = fin ? ((b & 0x000FFFFFFFFFFFFFull) | ((uint64_t)(ex != 0) << 52)) : 0ull;
        const int sh0 = (int)(ex ? ex : 1) - tmin;
        const uint32_t sh = sh0 < 0 ? 0u : (uint32_t)sh0;
        const uint64_t t = m << sh;  // |t| < 2^63
        const unsigned __int128 u = (unsigned __int128)t * t;
        uint64_t f1 = (b >> 63) ? 0ull - t : t;
        uint64_t f2l = (uint64_t)u, f2h = (uint64_t)(u >> 64);
        f1 = wave_scan64_fused(f1) + c1;
        c1 = lane63(f1);
        wave_scan128_fused(f2l, f2h);
        add128(f2l, f2h, c2l, c2h);
        c2l = lane63(f2l);
        c2h = lane63(f2h);
        const int slot = ((k & 3) << 6) | lane;
        r1[slot] = f1;
        r2l[slot] = f2l;
        r2h[slot] = f2h;
        if (COUNTS) {
            code = wave_scan64_fused(code) + ccn;
            ccn = lane63(code);
            rcn[slot] = code;
        }
        wave_sync();
        if (k == 0) continue;
        const int q = k - 1;
        if (o_first + 64 * q >= o_end) break;
        const int64_t i = o_first + 64 * q + lane;
        int64_t s, e;
        if (interior) {
            s = i - left;
            e = i + right;
        } else {
            rl_bounds(p, i, s, e);
        }
        const int je = (int)(e - 1 - s_first), js = (int)(s - 1 - s_first);
        const int ie = je & (kRwRing - 1), is = js & (kRwRing - 1);
        const int64_t S1 = (int64_t)(r1[ie] - (js >= 0 ? r1[is] : 0ull));
        uint64_t s2l = r2l[ie], s2h = r2h[ie];
        if (js >= 0) {
            add128(s2l, s2h, ~r2l[is], ~r2h[is]);
            add128(s2l, s2h, 1, 0);
        }
        RlCounts cn;
        if (COUNTS) cn = rl_unpack(rcn[ie] - (js >= 0 ? rcn[is] : 0ull));
        else cn = RlCounts{e - s, 0, 0, 0};
        const uint64_t c = (uint64_t)cn.nn;
        const bool valid = i < o_end && cn.nn >= p.min_periods && cn.nn > p.ddof;
        if (i < o_end) {
            // num = c * S2 - S1^2, exact in 192 bits
            const unsigned __int128 lo = (unsigned __int128)s2l * c;
            const unsigned __int128 hi = (unsigned __int128)s2h * c + (uint64_t)(lo >> 64);
            uint64_t w0 = (uint64_t)lo, w1 = (uint64_t)hi, w2 = (uint64_t)(hi >> 64);
            const uint64_t a1 = (uint64_t)(S1 < 0 ? -S1 : S1);
            const unsigned __int128 q2 = (unsigned __int128)a1 * a1;
            const uint64_t q0 = (uint64_t)q2, q1 = (uint64_t)(q2 >> 64);
            const uint64_t b0 = w0 < q0 ? 1ull : 0ull;
            w0 -= q0;
            const unsigned __int128 d1 = (unsigned __int128)w1 - q1 - b0;
            w1 = (uint64_t)d1;
            w2 -= (uint64_t)(d1 >> 64) ? 1ull : 0ull;
            double v = 0.0;
            if (valid) {
                if (COUNTS && (cn.nan || cn.pinf || cn.ninf)) {
                    v = __builtin_nan("");
                } else {
                    const double nr = (int64_t)w2 < 0 ? 0.0 : u192_to_double(w0, w1, w2, 2 * bottom);
                    v = (nr / (double)c) / (double)(c - (uint64_t)p.ddof);
                }
                if (p.var == 2) v = rv_std(p, v);
            }
            ((double*)p.out)[i] = valid ? v : 0.0;
        }
        const uint64_t bits = __ballot(valid);
        if (lane == 0) p.out_valid[(o_first >> 6) + q] = bits;
        wave_sync();
    }
}

// rw_var_scan's common case, as rw_scan_full for the sum: an interior wave
// (every window full, count w) with no null or non-finite row.  Its three
// prefix rings sit at fixed distances in the wave's ring array (t, t^2 low
// and high words at words 0, kRwRing, 2 kRwRing), indexed in 32 bits
// relative to the wave, ring slot kRwRing - 1 zeroed for prefix -1 (read
// only by the wave's first output; chunk 3 overwrites it afterwards).  The
// two quotients num / w / (w - ddof) take the one-correction form when the
// wave's exponents keep them normal (DIV1, rw_block).
// A nonnegative 128-bit integer (nh:nl) * 2^e as f64, rounded once (no
// subnormal results), without branches: the leading word and the bits
// below it as one sticky bit, then the one u64 -> f64 rounding.
__device__ __forceinline__ double u128_to_double(uint64_t nl, uint64_t nh, int e) {
    const bool hi = nh != 0;
    const uint64_t w = hi ? nh : nl;
    const int lz = __clzll(w | 1ull) - (w == 0 ? 1 : 0);  // (w == 0: nl == nh == 0, result 0)
    const uint64_t below = hi ? nl : 0ull;
    uint64_t top = lz ? (w << lz) | (below >> (64 - lz)) : w;
    const uint64_t rest = lz ? below << lz : below;
    top |= rest != 0 ? 1ull : 0ull;
    return __builtin_ldexp((double)top, (hi ? 128 : 64) - 64 - lz + e);
}

// sqrt(x), correctly rounded, for x == 0 or 2^-767 <= x < 2^1024: the
// compiler's f64 square root sequence (v_rsq_f64, then two Newton steps on
// the root and its half-reciprocal) without its small-input scaling and its
// class test, which such inputs never take.
__device__ __forceinline__ double sqrt_rn_scaled_free(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    return x == 0.0 ? x : g;
}

// N128: the wave's numerators are below 2^128 (rw_block: 2 (54 + span) +
// 2 lw <= 129, so w S2 - S1^2 = sum over pairs (t_i - t_j)^2 < 2^128), so
// w S2 and S1^2 are formed modulo 2^128 and their difference is exact.
// EMIT: 0 p.var / p.var_f32 decide (rv_std); 1 the variance; 2 its square
// root by sqrt_rn_scaled_free (the caller bounds nonzero variances >= 2^-767)
template <bool DIV1, bool N128, int EMIT = 0>
__device__ __forceinline__ void rw_var_scan_full(const RlParams& p, const uint64_t (&x)[kRwChunks + 1],
                                                 int64_t o_first, int64_t o_end, int64_t s_first, int tmin,
                                                 uint64_t* ring) {
    const int lane = threadIdx.x & 63;
    const int bottom = tmin - 1075;
    const int w = (int)p.w;
    const int right = p.center ? (w + 1) / 2 : 1;
    const int e0 = (int)(o_first - s_first) + right - 1;
    const int nout = (int)(o_end - o_first);
    const bool ok = p.w >= p.min_periods && p.w > p.ddof;
    double* ol = (double*)p.out + o_first + lane;
    uint64_t* ov = p.out_valid + (o_first >> 6);
    double y = p.rw, wd = p.wd, y2 = p.rw2, wd2 = p.wd2;
    asm volatile("" : "+v"(y), "+v"(wd), "+v"(y2), "+v"(wd2));
    const uint32_t cw = (uint32_t)w;
    if (lane == 63) ring[kRwRing - 1] = ring[2 * kRwRing - 1] = ring[3 * kRwRing - 1] = 0ull;
    uint64_t c1 = 0, c2l = 0, c2h = 0;
#pragma unroll
    for (int k = 0; k <= kRwChunks; ++k) {
        // finite, normal or zero (the fast form has tmin >= 600)
        const uint64_t b = x[k];
        const uint32_t ex = (uint32_t)(b >> 52) & 0x7FF;
        const uint64_t m = (b & 0x000FFFFFFFFFFFFFull) | (1ull << 52);
        const uint64_t t = ex ? m << (ex - (uint32_t)tmin) : 0ull;  // |t| < 2^63
        const unsigned __int128 u = (unsigned __int128)t * t;
        uint64_t f1 = (int64_t)b < 0 ? 0ull - t : t;
        uint64_t f2l = (uint64_t)u, f2h = (uint64_t)(u >> 64);
        f1 = wave_scan64_fused(f1) + c1;
        c1 = lane63(f1);
        wave_scan128_fused(f2l, f2h);
        add128(f2l, f2h, c2l, c2h);
        c2l = lane63(f2l);
        c2h = lane63(f2h);
        const int slot = ((k & 3) << 6) | lane;
        ring[slot] = f1;
        ring[kRwRing + slot] = f2l;
        ring[2 * kRwRing + slot] = f2h;
        wave_sync();
        if (k == 0) continue;
        const int q = k - 1;
        if (64 * q >= nout) break;
        const int je = e0 + 64 * q + lane;
        const int ie = je & (kRwRing - 1), is = (je - w) & (kRwRing - 1);
        const int64_t S1 = (int64_t)(ring[ie] - ring[is]);
        uint64_t s2l = ring[kRwRing + ie], s2h = ring[2 * kRwRing + ie];
        add128(s2l, s2h, ~ring[kRwRing + is], ~ring[2 * kRwRing + is]);
        add128(s2l, s2h, 1, 0);
        double nr;
        const uint64_t a1 = (uint64_t)(S1 < 0 ? -S1 : S1);
        const unsigned __int128 q2 = (unsigned __int128)a1 * a1;
        if (N128) {
            // num = w * S2 - S1^2 modulo 2^128 (exact: it is below 2^128)
            const unsigned __int128 lo = (unsigned __int128)s2l * cw;
            const unsigned __int128 num = (((unsigned __int128)(s2h * cw + (uint64_t)(lo >> 64))) << 64 |
                                           (uint64_t)lo) - q2;
            nr = u128_to_double((uint64_t)num, (uint64_t)(num >> 64), 2 * bottom);
        } else {
            // num = w * S2 - S1^2, exact in 192 bits
            const unsigned __int128 lo = (unsigned __int128)s2l * cw;
            const unsigned __int128 hi = (unsigned __int128)s2h * cw + (uint64_t)(lo >> 64);
            uint64_t w0 = (uint64_t)lo, w1 = (uint64_t)hi, w2 = (uint64_t)(hi >> 64);
            const uint64_t q0 = (uint64_t)q2, q1 = (uint64_t)(q2 >> 64);
            const uint64_t b0 = w0 < q0 ? 1ull : 0ull;
            w0 -= q0;
            const unsigned __int128 d1 = (unsigned __int128)w1 - q1 - b0;
            w1 = (uint64_t)d1;
            w2 -= (uint64_t)(d1 >> 64) ? 1ull : 0ull;
            nr = (int64_t)w2 < 0 ? 0.0 : u192_to_double(w0, w1, w2, 2 * bottom);
        }
        double v;
        if (DIV1) {
            const double a0 = nr * y;
            const double v1 = __builtin_fma(__builtin_fma(-a0, wd, nr), y, a0);
            const double a2 = v1 * y2;
            v = __builtin_fma(__builtin_fma(-a2, wd2, v1), y2, a2);
        } else {
            v = (nr / wd) / wd2;
        }
        if (EMIT == 0 && p.var == 2) v = rv_std(p, v);
        if (EMIT == 2) v = sqrt_rn_scaled_free(v);
        const bool in = 64 * q + lane < nout;
        if (in) ol[64 * q] = ok ? v : 0.0;
        const uint64_t bits = __ballot(in && ok);
        if (lane == 0) ov[q] = bits;
        wave_sync();
    }
}

// The rows [s_first, s_first + 64 (kRwChunks + 1)) of one wave's block as
// loaded (the row index clamped to the column, so the loads are
// branch-free and all in flight together; rows past n are masked by
// rw_block).  4-byte integers sign-extended.
template <int DT>
__device__ __forceinline__ void rw_load_block(const RlParams& p, int64_t s_first, uint64_t (&x)[kRwChunks + 1]) {
    const int lane = threadIdx.x & 63;
    const int64_t last = p.n - 1;
#pragma unroll
    for (int k = 0; k <= kRwChunks; ++k) {
        int64_t r = s_first + 64 * k + lane;
        r = r < last ? r : last;
        const int64_t q = p.c.offset + r;
        if (DT == PLGPU_F64 || DT == PLGPU_I64) x[k] = __builtin_nontemporal_load((const uint64_t*)p.c.values + q);
        else x[k] = (uint64_t)(int64_t)__builtin_nontemporal_load((const int32_t*)p.c.values + q);
    }
}

// One wave's block of kRwOut outputs from its loaded rows: validity, the
// exponent range and the number format, then the scan + emit.
template <int DT, bool NULLABLE, bool VAR>
__device__ __forceinline__ void rw_block(const RlParams& p, uint64_t (&x)[kRwChunks + 1], int64_t o_first,
                                         int64_t s_first, uint64_t* rlo, uint64_t* rhi, uint64_t* rcn,
                                         uint64_t* rv2) {
    const int lane = threadIdx.x & 63;
    const int64_t o_end = o_first + kRwOut < p.n ? o_first + kRwOut : p.n;
    const bool isint = p.out_int != 0;  // (var / std: integers enter as their f64 values)
    uint64_t vm[kRwChunks + 1];
    uint32_t mx = 0, inv_mn = 0;
    bool odd = false;  // a null (in range) or a non-finite value
#pragma unroll
    for (int k = 0; k <= kRwChunks; ++k) {
        const int64_t r = s_first + 64 * k + lane;
        const bool in = r < p.n;
        const bool v = in && (!NULLABLE || dev_valid(p.c, r));
        const uint64_t b = (DT == PLGPU_F64 || isint) ? x[k] : f64_bits((double)(int64_t)x[k]);
        vm[k] = __ballot(v);
        x[k] = v ? b : 0ull;
        if (NULLABLE) odd |= in && !v;
        if (v) {
            const uint32_t ex = (uint32_t)(b >> 52) & 0x7FF;
            odd |= ex == 0x7FF;
            if (ex != 0x7FF && (b << 1) != 0) {
                const uint32_t e1 = ex ? ex : 1;
                mx = e1 > mx ? e1 : mx;
                inv_mn = 0x7FF - e1 > inv_mn ? 0x7FF - e1 : inv_mn;
            }
        }
    }
    const bool counts = __ballot(odd) != 0;
    if (isint) {
        // (the exponent fields of integers mean nothing; only nulls count)
        if (__ballot(NULLABLE && odd) != 0) rw_scan<0, true, false>(p, x, vm, o_first, o_end, s_first, 0, rlo, rhi, rcn);
        else rw_scan<0, false, false>(p, x, vm, o_first, o_end, s_first, 0, rlo, rhi, rcn);
        return;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t a = __shfl_xor(mx, off, 64), c = __shfl_xor(inv_mn, off, 64);
        mx = a > mx ? a : mx;
        inv_mn = c > inv_mn ? c : inv_mn;
    }
    const int tmax = (int)mx, tmin = mx ? 0x7FF - (int)inv_mn : 1024;
    int lw = 0;
    while ((int64_t(1) << lw) <= p.w) ++lw;  // p.w < 2^lw
    const int span = tmax - tmin;
    if (VAR) {
        // fast form: t < 2^63 with window sums in 64 bits, t^2's window
        // sums in 127 bits, and no result near the subnormal range
        const bool vfast = mx == 0 || (tmin >= 600 && lw + 53 + span <= 63 && 2 * (53 + span) + lw <= 126);
        if (!vfast) {
            rw_var_exact_outputs(p, o_first, o_end);
            return;
        }
        const int64_t right = p.center ? (p.w + 1) / 2 : 1;
        if (!counts && p.full && o_first - (p.w - right) >= 0 && o_end + right - 1 <= p.n) {
            // nonzero numerators lie in [2^(2 bottom), 2^(2 (tmax - 1022) + 2 lw)):
            // both quotients inside rw_div's exponent range
            const int b2 = 2 * (tmin - 1075), top = 2 * (tmax - 1022) + 2 * lw;
            const bool div1 = p.fast_div && b2 - 2 * lw >= -900 && top <= 990;
            const bool n128 = p.var128 && 2 * (54 + span) + 2 * lw <= 129;
            if (div1 && n128) rw_var_scan_full<true, true>(p, x, o_first, o_end, s_first, tmin, rlo);
            else if (div1) rw_var_scan_full<true, false>(p, x, o_first, o_end, s_first, tmin, rlo);
            else rw_var_scan_full<false, false>(p, x, o_first, o_end, s_first, tmin, rlo);
            return;
        }
        if (counts) rw_var_scan<true>(p, x, vm, o_first, o_end, s_first, tmin, rlo, rhi, rv2, rcn);
        else rw_var_scan<false>(p, x, vm, o_first, o_end, s_first, tmin, rlo, rhi, rv2, rcn);
        return;
    }
    // int64 when any window's sum fits 63 bits and results cannot be subnormal
    const bool narrow = mx == 0 || (tmin >= 128 && lw + 53 + span <= 63);
    if (!narrow && lw + 53 + span > 127) {
        rw_exact_outputs(p, o_first, o_end);  // beyond 128 bits
        return;
    }
    if (narrow && !counts && p.full) {
        const int64_t right = p.center ? (p.w + 1) / 2 : 1;
        if (o_first - (p.w - right) >= 0 && o_end + right - 1 <= p.n) {
            // the one-correction mean without its per-lane test: nonzero
            // window sums lie in [2^(tmin - 1075), 2^(tmax - 1022 + lw)),
            // inside rw_div's exponent range
            const bool div1 = p.fast_div && tmin - 1075 >= -900 && tmax - 1022 + lw <= 990;
            if (p.mean) rw_scan_full<true>(p, x, o_first, o_end, s_first, tmin, div1, rlo);
            else rw_scan_full<false>(p, x, o_first, o_end, s_first, tmin, div1, rlo);
            return;
        }
    }
#define PLGPU_RW(M, C)                                                                                   \
    (p.mean ? rw_scan<M, C, true>(p, x, vm, o_first, o_end, s_first, tmin, rlo, rhi, rcn)               \
            : rw_scan<M, C, false>(p, x, vm, o_first, o_end, s_first, tmin, rlo, rhi, rcn))
    if (narrow) {
        if (counts) PLGPU_RW(1, true);
        else PLGPU_RW(1, false);
    } else {
        if (counts) PLGPU_RW(2, true);
        else PLGPU_RW(2, false);
    }
#undef PLGPU_RW
}

// One block of kRwOut outputs per wave.  (A register cap for 6 waves per
// SIMD, __launch_bounds__(256, 6), spilled 6 VGPRs and still ended at 5
// waves: not kept.)
template <int DT, bool NULLABLE, bool VAR = false>
__global__ __launch_bounds__(256) void rl_wave_kernel(RlParams p) {
    // each wave's three rings, adjacent (rw_scan_full uses them as one array)
    __shared__ uint64_t ring[kRwWaves][3 * kRwRing];
    __shared__ uint64_t ring_v2[VAR ? kRwWaves : 1][VAR ? kRwRing : 1];  // var: the t^2 prefixes' high words
    const int wv = threadIdx.x >> 6;
    const int64_t o_first = ((int64_t)blockIdx.x * kRwWaves + wv) * kRwOut;
    if (o_first >= p.n) return;  // (no workgroup barriers below)
    int64_t s_first, tmp;
    rl_bounds(p, o_first, s_first, tmp);
    uint64_t x[kRwChunks + 1];
    rw_load_block<DT>(p, s_first, x);
    rw_block<DT, NULLABLE, VAR>(p, x, o_first, s_first, ring[wv], ring[wv] + kRwRing, ring[wv] + 2 * kRwRing,
                                VAR ? ring_v2[wv] : nullptr);
}

// Resident waves, each over blocks b, b + stride, ...: the next block's
// rows are loaded before this block is scanned, so every wave keeps its
// loads in flight while it computes (the one-block form waits for them).
template <int DT, bool VAR = false>
__global__ __launch_bounds__(256) void rl_stream_kernel(RlParams p) {
    // each wave's three rings, adjacent (rw_scan_full uses them as one array)
    __shared__ uint64_t ring[kRwWaves][3 * kRwRing];
    __shared__ uint64_t ring_v2[VAR ? kRwWaves : 1][VAR ? kRwRing : 1];
    const int wv = threadIdx.x >> 6;
    const int64_t nblocks = (p.n + kRwOut - 1) / kRwOut;
    const int64_t stride = (int64_t)gridDim.x * kRwWaves;
    int64_t b = (int64_t)blockIdx.x * kRwWaves + wv;
    if (b >= nblocks) return;  // (no workgroup barriers below)
    int64_t s_first, tmp;
    rl_bounds(p, b * kRwOut, s_first, tmp);
    uint64_t x[kRwChunks + 1];
    rw_load_block<DT>(p, s_first, x);
    for (; b < nblocks; b += stride) {
        const int64_t bn = b + stride;
        int64_t sn = 0;
        uint64_t xn[kRwChunks + 1];
        if (bn < nblocks) {
            rl_bounds(p, bn * kRwOut, sn, tmp);
            rw_load_block<DT>(p, sn, xn);
        }
        rw_block<DT, false, VAR>(p, x, b * kRwOut, s_first, ring[wv], ring[wv] + kRwRing, ring[wv] + 2 * kRwRing,
                                 VAR ? ring_v2[wv] : nullptr);
#pragma unroll
        for (int k = 0; k <= kRwChunks; ++k) x[k] = xn[k];
        s_first = sn;
    }
}

// rolling var / std, its common block alone (option rl_var_hot): a
// null-free interior block whose values are finite and fit the fast form
// with both one-correction quotients and the numerators modulo 2^128
// (rw_block's conditions for rw_var_scan_full<true, true>).  Without the
// general paths inlined the kernel holds fewer registers (more waves per
// SIMD, no scalar spills in the loop).  Any other block goes to
// p.rest (count in word 0, then block indices) for rl_var_rest_kernel.
template <int DT, bool STD>
__device__ __forceinline__ bool rw_var_hot_block(const RlParams& p, uint64_t (&x)[kRwChunks + 1], int64_t o_first,
                                                 int64_t s_first, uint64_t* ring, int lw, int64_t right) {
    const int64_t o_end = o_first + kRwOut < p.n ? o_first + kRwOut : p.n;
    if (!(o_first - (p.w - right) >= 0 && o_end + right - 1 <= p.n)) return false;
    uint32_t mx = 0, inv_mn = 0;
    bool odd = false;
#pragma unroll
    for (int k = 0; k <= kRwChunks; ++k) {
        const int64_t r = s_first + 64 * k + (threadIdx.x & 63);
        const uint64_t b = r >= p.n ? 0ull : DT == PLGPU_F64 ? x[k] : f64_bits((double)(int64_t)x[k]);
        x[k] = b;
        const uint32_t ex = (uint32_t)(b >> 52) & 0x7FF;
        odd |= ex == 0x7FF;
        if ((b << 1) != 0) {
            const uint32_t e1 = ex ? ex : 1;
            mx = e1 > mx ? e1 : mx;
            inv_mn = 0x7FF - e1 > inv_mn ? 0x7FF - e1 : inv_mn;
        }
    }
    if (__ballot(odd) != 0) return false;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t a = __shfl_xor(mx, off, 64), c = __shfl_xor(inv_mn, off, 64);
        mx = a > mx ? a : mx;
        inv_mn = c > inv_mn ? c : inv_mn;
    }
    const int tmax = (int)mx, tmin = mx ? 0x7FF - (int)inv_mn : 1024;
    const int span = tmax - tmin;
    const bool vfast = mx == 0 || (tmin >= 600 && lw + 53 + span <= 63 && 2 * (53 + span) + lw <= 126);
    const int b2 = 2 * (tmin - 1075), top = 2 * (tmax - 1022) + 2 * lw;
    // (nonzero variances >= 2^(b2 - 2 lw) >= 2^-760: sqrt_rn_scaled_free's range)
    const bool div1 = b2 - 2 * lw >= -760 && top <= 990;
    const bool n128 = 2 * (54 + span) + 2 * lw <= 129;
    if (!(vfast && div1 && n128)) return false;
    rw_var_scan_full<true, true, STD ? 2 : 1>(p, x, o_first, o_end, s_first, tmin, ring);
    return true;
}

// rolling sum / mean, the same split (option rl_mean_hot): an interior,
// finite block in the int64 form (rw_block's conditions for rw_scan_full).
template <int DT>
__device__ __forceinline__ bool rw_mean_hot_block(const RlParams& p, uint64_t (&x)[kRwChunks + 1], int64_t o_first,
                                                  int64_t s_first, uint64_t* ring, int lw, int64_t right) {
    const int64_t o_end = o_first + kRwOut < p.n ? o_first + kRwOut : p.n;
    if (!(o_first - (p.w - right) >= 0 && o_end + right - 1 <= p.n)) return false;
    uint32_t mx = 0, inv_mn = 0;
    bool odd = false;
#pragma unroll
    for (int k = 0; k <= kRwChunks; ++k) {
        const int64_t r = s_first + 64 * k + (threadIdx.x & 63);
        const uint64_t b = r >= p.n ? 0ull : DT == PLGPU_F64 ? x[k] : f64_bits((double)(int64_t)x[k]);
        x[k] = b;
        const uint32_t ex = (uint32_t)(b >> 52) & 0x7FF;
        odd |= ex == 0x7FF;
        if ((b << 1) != 0) {
            const uint32_t e1 = ex ? ex : 1;
            mx = e1 > mx ? e1 : mx;
            inv_mn = 0x7FF - e1 > inv_mn ? 0x7FF - e1 : inv_mn;
        }
    }
    if (__ballot(odd) != 0) return false;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t a = __shfl_xor(mx, off, 64), c = __shfl_xor(inv_mn, off, 64);
        mx = a > mx ? a : mx;
        inv_mn = c > inv_mn ? c : inv_mn;
    }
    const int tmax = (int)mx, tmin = mx ? 0x7FF - (int)inv_mn : 1024;
    const int span = tmax - tmin;
    if (!(mx == 0 || (tmin >= 128 && lw + 53 + span <= 63))) return false;
    const bool div1 = p.fast_div && tmin - 1075 >= -900 && tmax - 1022 + lw <= 990;
    if (p.mean) rw_scan_full<true>(p, x, o_first, o_end, s_first, tmin, div1, ring);
    else rw_scan_full<false>(p, x, o_first, o_end, s_first, tmin, div1, ring);
    return true;
}

template <int DT>
__global__ __launch_bounds__(256) void rl_mean_hot_kernel(RlParams p) {
    __shared__ uint64_t ring[kRwWaves][kRwChunks * 64 + 64 + 1];  // rw_scan_full's prefixes
    const int wv = threadIdx.x >> 6;
    const int64_t nblocks = (p.n + kRwOut - 1) / kRwOut;
    const int64_t b = (int64_t)blockIdx.x * kRwWaves + wv;
    if (b >= nblocks) return;  // (no workgroup barriers below)
    int lw = 0;
    while ((int64_t(1) << lw) <= p.w) ++lw;  // p.w < 2^lw
    const int64_t right = p.center ? (p.w + 1) / 2 : 1;
    int64_t s_first, tmp;
    rl_bounds(p, b * kRwOut, s_first, tmp);
    uint64_t x[kRwChunks + 1];
    rw_load_block<DT>(p, s_first, x);
    if (!rw_mean_hot_block<DT>(p, x, b * kRwOut, s_first, ring[wv], lw, right) && (threadIdx.x & 63) == 0)
        p.rest[1 + atomicAdd(&p.rest[0], 1u)] = (uint32_t)b;
}

template <int DT, bool STREAM, bool STD>
__global__ __launch_bounds__(256) void rl_var_hot_kernel(RlParams p) {
    __shared__ uint64_t ring[kRwWaves][3 * kRwRing];
    const int wv = threadIdx.x >> 6;
    const int64_t nblocks = (p.n + kRwOut - 1) / kRwOut;
    const int64_t stride = STREAM ? (int64_t)gridDim.x * kRwWaves : nblocks;
    int64_t b = (int64_t)blockIdx.x * kRwWaves + wv;
    if (b >= nblocks) return;  // (no workgroup barriers below)
    int lw = 0;
    while ((int64_t(1) << lw) <= p.w) ++lw;  // p.w < 2^lw
    const int64_t right = p.center ? (p.w + 1) / 2 : 1;
    int64_t s_first, tmp;
    rl_bounds(p, b * kRwOut, s_first, tmp);
    uint64_t x[kRwChunks + 1];
    rw_load_block<DT>(p, s_first, x);
    for (; b < nblocks; b += stride) {
        // (STREAM: resident waves, the next block's rows in flight while
        // this one is scanned)
        const int64_t bn = b + stride;
        int64_t sn = 0;
        uint64_t xn[kRwChunks + 1];
        if constexpr (STREAM) {
            if (bn < nblocks) {
                rl_bounds(p, bn * kRwOut, sn, tmp);
                rw_load_block<DT>(p, sn, xn);
            }
        }
        if (!rw_var_hot_block<DT, STD>(p, x, b * kRwOut, s_first, ring[wv], lw, right) && (threadIdx.x & 63) == 0)
            p.rest[1 + atomicAdd(&p.rest[0], 1u)] = (uint32_t)b;
        if constexpr (STREAM) {
#pragma unroll
            for (int k = 0; k <= kRwChunks; ++k) x[k] = xn[k];
            s_first = sn;
        }
    }
}

// The blocks rl_var_hot_kernel / rl_mean_hot_kernel left, one per wave, by rw_block.
template <int DT, bool VAR = true>
__global__ __launch_bounds__(256) void rl_var_rest_kernel(RlParams p) {
    __shared__ uint64_t ring[kRwWaves][3 * kRwRing];
    __shared__ uint64_t ring_v2[VAR ? kRwWaves : 1][VAR ? kRwRing : 1];
    const int wv = threadIdx.x >> 6;
    const uint32_t cnt = __builtin_nontemporal_load(&p.rest[0]);
    for (uint32_t j = blockIdx.x * kRwWaves + wv; j < cnt; j += gridDim.x * kRwWaves) {
        const int64_t b = p.rest[1 + j];
        int64_t s_first, tmp;
        rl_bounds(p, b * kRwOut, s_first, tmp);
        uint64_t x[kRwChunks + 1];
        rw_load_block<DT>(p, s_first, x);
        rw_block<DT, false, VAR>(p, x, b * kRwOut, s_first, ring[wv], ring[wv] + kRwRing, ring[wv] + 2 * kRwRing,
                                 VAR ? ring_v2[wv] : nullptr);
    }
}

// rolling var / std over windows wider than the wave kernel's: each output
// from its exact window sums (rv_window_exact; O(window) per output).
__global__ void rl_direct_var_kernel(RlParams p) {
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < p.n; base += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = base + threadIdx.x;
        bool valid = false;
        if (i < p.n) {
            int64_t s, e;
            rl_bounds(p, i, s, e);
            RlCounts k = {0, 0, 0, 0};
            for (int64_t r = s; r < e; ++r) rl_count(p, r, k);
            valid = k.nn >= p.min_periods && k.nn > p.ddof;
            double v = 0.0;
            if (valid) {
                v = (k.nan || k.pinf || k.ninf) ? __builtin_nan("") : rv_window_exact(p, s, e, k.nn);
                if (p.var == 2) v = rv_std(p, v);
            }
            ((double*)p.out)[i] = valid ? v : 0.0;
        }
        const uint64_t wv = __ballot(valid);
        if ((threadIdx.x & 63) == 0 && i < p.n) p.out_valid[i >> 6] = wv;
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

static int num_cus_rl() {
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

PLGPU_API int plgpu_rolling(const plgpu_column* values, int32_t kind, int64_t window_size, int64_t min_periods,
                            int32_t center, plgpu_column* out, void* stream) {
    hipStream_t s = as_stream(stream);
    if (values == nullptr || out == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    std::memset(out, 0, sizeof *out);
    // bits 8..15: ddof; bit 16 (std of a Float32 column): the variance is
    // rounded to Float32 before the square root, as the reference's f32 sqrt
    const int32_t base = kind & 0xFF, ddof = (kind >> 8) & 0xFF, var_f32 = (kind >> 16) & 1;
    if (base < PLGPU_ROLLING_SUM || base > PLGPU_ROLLING_STD) return fail(PLGPU_ERR_INVALID, "unknown rolling kind");
    const bool var = base == PLGPU_ROLLING_VAR || base == PLGPU_ROLLING_STD;
    if (!var && ddof != 0) return fail(PLGPU_ERR_INVALID, "ddof applies to rolling var / std only");
    kind = base;
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
    p.rw = 1.0 / (double)std::max<int64_t>(window_size, 1);
    p.fast_div = options().rl_div;
    p.var128 = options().rl_var128;
    p.full = options().rl_full;
    p.wd = (double)window_size;
    p.wd2 = (double)std::max<int64_t>(window_size - ddof, 1);
    p.rw2 = 1.0 / p.wd2;
    p.var = var ? (kind == PLGPU_ROLLING_STD ? 2 : 1) : 0;
    p.ddof = ddof;
    p.var_f32 = var_f32;
    p.isf = values->dtype == PLGPU_F64;
    p.out_int = (!p.mean && !var && !p.isf) ? values->dtype : 0;
    const int32_t odt = p.out_int ? values->dtype : PLGPU_F64;
    int rc = make_owned_column(out, odt, p.n, true, s);
    if (rc || p.n == 0) return rc;
    p.out = (void*)out->values;
    p.out_valid = (uint64_t*)out->validity;
    const int64_t tiles = (p.n + kRlOut - 1) / kRlOut;
    if (window_size <= kRwMaxW) {
        const unsigned g = (unsigned)((p.n + (int64_t)kRwOut * kRwWaves - 1) / ((int64_t)kRwOut * kRwWaves));
        const bool nl = p.c.validity != nullptr;
        KtScope kt(var ? "rl_wave_var_kernel" : "rl_wave_kernel", s);
        const bool hot = var && !nl && !p.var_f32 && options().rl_var_hot && p.full && p.fast_div && p.var128;
        const bool mhot = !var && !nl && !p.out_int && options().rl_mean_hot && p.full;
        if (hot || mhot) {
            // the common blocks by rl_var_hot_kernel, the rest listed for
            // rl_var_rest_kernel (stream-ordered; the count read on the device)
            const int64_t nblocks = (p.n + kRwOut - 1) / kRwOut;
            int arc = dev_alloc((void**)&p.rest, (size_t)(nblocks + 1) * 4, s);
            if (!arc && hipMemsetAsync(p.rest, 0, 4, s) != hipSuccess) arc = PLGPU_ERR_HIP;
            if (arc) {
                if (p.rest) dev_free(p.rest, s);
                plgpu_column_release(out);
                return arc == PLGPU_ERR_HIP ? hip_fail(hipGetLastError(), "rolling") : arc;
            }
            const bool st = options().rl_stream != 0;
            const int per_cu = options().rl_grid > 0 ? options().rl_grid : 4;
            const unsigned gs = (unsigned)std::max<int64_t>(1, std::min<int64_t>((int64_t)g, (int64_t)num_cus_rl() * per_cu));
            const unsigned gr = (unsigned)std::max<int64_t>(1, std::min<int64_t>((int64_t)g, (int64_t)num_cus_rl()));
#define PLGPU_RLHOT(DT)                                                      \
    do {                                                                     \
        if (mhot) {                                                          \
            rl_mean_hot_kernel<DT><<<g, 64 * kRwWaves, 0, s>>>(p);           \
            rl_var_rest_kernel<DT, false><<<gr, 64 * kRwWaves, 0, s>>>(p);   \
            break;                                                           \
        }                                                                    \
        if (st && p.var == 2) rl_var_hot_kernel<DT, true, true><<<gs, 64 * kRwWaves, 0, s>>>(p);    \
        else if (st) rl_var_hot_kernel<DT, true, false><<<gs, 64 * kRwWaves, 0, s>>>(p);       \
        else if (p.var == 2) rl_var_hot_kernel<DT, false, true><<<g, 64 * kRwWaves, 0, s>>>(p); \
        else rl_var_hot_kernel<DT, false, false><<<g, 64 * kRwWaves, 0, s>>>(p);               \
        rl_var_rest_kernel<DT><<<gr, 64 * kRwWaves, 0, s>>>(p);              \
    } while (0)
            if (values->dtype == PLGPU_F64) PLGPU_RLHOT(PLGPU_F64);
            else if (values->dtype == PLGPU_I64) PLGPU_RLHOT(PLGPU_I64);
            else PLGPU_RLHOT(PLGPU_I32);
#undef PLGPU_RLHOT
        } else if (!nl && options().rl_stream != 0) {
            // null-free: resident waves streaming their blocks
            const int per_cu = options().rl_grid > 0 ? options().rl_grid : 4;
            const unsigned gs = (unsigned)std::max<int64_t>(1, std::min<int64_t>((int64_t)g, (int64_t)num_cus_rl() * per_cu));
            if (values->dtype == PLGPU_F64) {
                if (var) rl_stream_kernel<PLGPU_F64, true><<<gs, 64 * kRwWaves, 0, s>>>(p);
                else rl_stream_kernel<PLGPU_F64, false><<<gs, 64 * kRwWaves, 0, s>>>(p);
            } else if (values->dtype == PLGPU_I64) {
                if (var) rl_stream_kernel<PLGPU_I64, true><<<gs, 64 * kRwWaves, 0, s>>>(p);
                else rl_stream_kernel<PLGPU_I64, false><<<gs, 64 * kRwWaves, 0, s>>>(p);
            } else {
                if (var) rl_stream_kernel<PLGPU_I32, true><<<gs, 64 * kRwWaves, 0, s>>>(p);
                else rl_stream_kernel<PLGPU_I32, false><<<gs, 64 * kRwWaves, 0, s>>>(p);
            }
        } else if (var) {
            if (values->dtype == PLGPU_F64) {
                if (nl) rl_wave_kernel<PLGPU_F64, true, true><<<g, 64 * kRwWaves, 0, s>>>(p);
                else rl_wave_kernel<PLGPU_F64, false, true><<<g, 64 * kRwWaves, 0, s>>>(p);
            } else if (values->dtype == PLGPU_I64) {
                if (nl) rl_wave_kernel<PLGPU_I64, true, true><<<g, 64 * kRwWaves, 0, s>>>(p);
                else rl_wave_kernel<PLGPU_I64, false, true><<<g, 64 * kRwWaves, 0, s>>>(p);
            } else {
                if (nl) rl_wave_kernel<PLGPU_I32, true, true><<<g, 64 * kRwWaves, 0, s>>>(p);
                else rl_wave_kernel<PLGPU_I32, false, true><<<g, 64 * kRwWaves, 0, s>>>(p);
            }
        } else if (values->dtype == PLGPU_F64) {
            if (nl) rl_wave_kernel<PLGPU_F64, true><<<g, 64 * kRwWaves, 0, s>>>(p);
            else rl_wave_kernel<PLGPU_F64, false><<<g, 64 * kRwWaves, 0, s>>>(p);
        } else if (values->dtype == PLGPU_I64) {
            if (nl) rl_wave_kernel<PLGPU_I64, true><<<g, 64 * kRwWaves, 0, s>>>(p);
            else rl_wave_kernel<PLGPU_I64, false><<<g, 64 * kRwWaves, 0, s>>>(p);
        } else {
            if (nl) rl_wave_kernel<PLGPU_I32, true><<<g, 64 * kRwWaves, 0, s>>>(p);
            else rl_wave_kernel<PLGPU_I32, false><<<g, 64 * kRwWaves, 0, s>>>(p);
        }
    } else if (var)
        rl_direct_var_kernel<<<(unsigned)std::min<int64_t>((p.n + 255) / 256, 256 * 64), 256, 0, s>>>(p);
    else if (window_size - 1 + kRlOut <= 2048)
        rl_tile_kernel<2048><<<(unsigned)tiles, kRlThreads, 0, s>>>(p);
    else if (window_size - 1 + kRlOut <= 4096)
        rl_tile_kernel<4096><<<(unsigned)tiles, kRlThreads, 0, s>>>(p);
    else
        rl_direct_kernel<<<(unsigned)std::min<int64_t>((p.n + 255) / 256, 256 * 64), 256, 0, s>>>(p);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (p.rest) dev_free(p.rest, s);
    if (e != hipSuccess) {
        plgpu_column_release(out);
        return hip_fail(e, "rolling");
    }
    out->null_count = -1;
    return PLGPU_OK;
}
