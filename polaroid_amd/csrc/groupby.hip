// groupby.hip — fused predicate + hash group-by + aggregation on gfx950.
//
// Reference path (Rust): FilterExec (polars-mem-engine/src/executors/
// filter.rs:51) feeding GroupByStreamingExec / GroupByExec (group_by.rs:117,
// chosen at polars-mem-engine/src/planner/lp.rs:648), whose per-group folds
// are polars-expr/src/reduce/{sum,mean,min_max,count,len}.rs and
// polars-core/src/frame/group_by/aggregations/mod.rs:581 (agg_sum).
//
// Design:
//  * one persistent launch streams the key + referenced columns once,
//    coalesced, evaluating the predicate in registers (no mask column);
//  * each workgroup owns an LDS open-addressing table (key -> slot) whose
//    accumulators are updated with LDS atomics; rows whose key does not fit
//    the LDS table go straight to the global table (device-scope atomics);
//  * at the end each workgroup folds its LDS table into the global table;
//  * f64 sums are exact: every value is converted to a 120-bit fixed-point
//    integer (3 carry-free 40-bit limbs in LDS, one 192-bit two's-complement
//    integer per group in HBM) and rounded once at the end, so the result is
//    the correctly rounded sum, independent of the order of arrival — the
//    deterministic answer that Kahan / naive row-order folds approximate.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "plgpu_internal.hpp"

namespace plgpu {

constexpr int kGbThreads = 512;
constexpr int kMaxAcc = 6;
constexpr int kMaxFields = 48;
constexpr int kLdsProbe = 32;
constexpr int kGlobalProbe = 4096;
constexpr int kSumWindowBits = 120;   // fixed-point window of one value
constexpr int kHeadroomBinades = 8;   // above the sampled max exponent
constexpr int64_t kMaxRowsPerWg = int64_t(1) << 22;  // keeps 40-bit limbs exact in int64

// Acc flags
enum : int32_t { A_FSUM = 1, A_FSUMCAST = 2, A_ISUM = 4, A_CNT = 8, A_MIN = 16, A_MAX = 32, A_FLAGS = 64 };
// Special-value flags (f64)
enum : uint32_t { FL_NAN = 1, FL_PINF = 2, FL_NINF = 4 };
// Status words
enum : int {
    ST_NEWKEYS = 0,
    ST_GLOBAL_ROWS = 1,
    ST_TABLE_FULL = 2,
    ST_SELECTED = 3,
    ST_SPECIAL = 4,      // bit0 null group present, bit1 INT64_MIN group present
    ST_GROUPS_OUT = 5,   // finalize counter
    ST_MAXEX = 8,        // + acc
    ST_FXFLAGS = 16,     // + acc: bit0 overflow, bit1 inexact
    ST_WORDS = 24
};

struct AccSpec {
    int32_t col;
    int32_t flags;
    int32_t f_sum;    // FSUM/FSUMCAST: 3 limb fields; ISUM: 1 field
    int32_t f_isum;
    int32_t f_cnt;
    int32_t f_min;
    int32_t f_max;
    int32_t f_flags;
};

struct GbParams {
    DevCol key;
    DevCol cols[PLGPU_MAX_COLS];
    int64_t n;
    int32_t nacc;
    int32_t nfields;
    AccSpec acc[kMaxAcc];
    int32_t f_len;
    int32_t f_first;        // -1 unless maintain_order
    uint64_t min_init_mask; // fields initialised to ~0
    int32_t lbits;
    int32_t lcap;
    int32_t gbits;
    int32_t _pad;
    int64_t gcap;
    uint64_t* gtab;         // nfields regions of (gcap + 2) words; field 0 = keys
    const int32_t* bottoms; // [kMaxAcc]
    uint64_t* status;       // [ST_WORDS]
};

// ------------------------------------------------------------ helpers
__device__ __forceinline__ uint64_t lds_load(uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// LDS probe: slot index or -1 (table saturated along the probe window).
__device__ __forceinline__ int lds_find(uint64_t* lkeys, int lbits, int lcap, uint64_t key) {
    const uint32_t h = hash_slot(key, lbits);
    const uint32_t mask = (uint32_t)lcap - 1;
    for (int p = 0; p < kLdsProbe; ++p) {
        const uint32_t s = (h + (uint32_t)p) & mask;
        uint64_t k = lds_load(&lkeys[s]);
        if (k == key) return (int)s;
        if (k == kEmptyKey) {
            k = atomicCAS((unsigned long long*)&lkeys[s], (unsigned long long)kEmptyKey, (unsigned long long)key);
            if (k == kEmptyKey || k == key) return (int)s;
        }
    }
    return -1;
}

// Global probe: slot index or -1.  A plain load may return a stale EMPTY
// (another CU inserted since); the CAS then returns the true key, so the
// protocol never needs an acquire: keys only ever go EMPTY -> key.
__device__ __forceinline__ int64_t g_find(const GbParams& p, uint64_t key) {
    uint64_t* gkeys = p.gtab;
    const uint64_t mask = (uint64_t)p.gcap - 1;
    const uint64_t h = p.gbits == 0 ? 0 : ((key * 0x9E3779B97F4A7C15ull) >> (64 - p.gbits));
    const int lim = p.gcap < kGlobalProbe ? (int)p.gcap : kGlobalProbe;
    for (int i = 0; i < lim; ++i) {
        const uint64_t s = (h + (uint64_t)i) & mask;
        uint64_t k = __hip_atomic_load(&gkeys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == key) return (int64_t)s;
        if (k == kEmptyKey) {
            k = atomicCAS((unsigned long long*)&gkeys[s], (unsigned long long)kEmptyKey, (unsigned long long)key);
            if (k == kEmptyKey) {
                atomicAdd((unsigned long long*)&p.status[ST_NEWKEYS], 1ull);
                return (int64_t)s;
            }
            if (k == key) return (int64_t)s;
        }
    }
    return -1;
}

// f64 bits -> three carry-free 40-bit limbs of the fixed-point value
// x / 2^bottom (rounded half-even below the window).  Returns false for
// zero / rounded-away values; sets FX overflow (1) / inexact (2) in fl.
__device__ __forceinline__ bool fx_limbs(uint64_t b, int bottom, uint64_t& l0, uint64_t& l1, uint64_t& l2,
                                         uint32_t& fl, uint32_t& ex_out) {
    uint32_t ex = (uint32_t)(b >> 52) & 0x7FF;
    uint64_t m = b & 0x000FFFFFFFFFFFFFull;
    if (ex == 0) {
        if (m == 0) return false;
        ex = 1;
    } else {
        m |= 0x0010000000000000ull;
    }
    ex_out = ex;
    const int sh = (int)ex - 1075 - bottom;
    uint64_t lo, hi;
    if (sh >= 0) {
        if (sh + 53 > kSumWindowBits) {
            fl |= 1u;
            return false;
        }
        if (sh == 0) { lo = m; hi = 0; }
        else if (sh < 64) { lo = m << sh; hi = m >> (64 - sh); }
        else { lo = 0; hi = m << (sh - 64); }
    } else {
        const int k = -sh;
        if (k > 53) {
            fl |= 2u;
            return false;
        }
        uint64_t q = m >> k;
        const uint64_t rem = m & ((1ull << k) - 1);
        const uint64_t half = 1ull << (k - 1);
        if (rem) fl |= 2u;
        if (rem > half || (rem == half && (q & 1))) ++q;
        if (q == 0) return false;
        lo = q;
        hi = 0;
    }
    constexpr uint64_t M40 = (1ull << 40) - 1;
    l0 = lo & M40;
    l1 = ((lo >> 40) | (hi << 24)) & M40;
    l2 = hi >> 16;
    if (b >> 63) {
        l0 = 0ull - l0;
        l1 = 0ull - l1;
        l2 = 0ull - l2;
    }
    return true;
}

// Signed limb sums -> 192-bit two's complement words.
__device__ __forceinline__ void limbs_to_192(int64_t L0, int64_t L1, int64_t L2, uint64_t& w0, uint64_t& w1,
                                             uint64_t& w2) {
    const __int128 A = (__int128)L0 + ((__int128)L1 << 40);
    const uint64_t a0 = (uint64_t)A;
    const uint64_t a1 = (uint64_t)(A >> 64);
    const uint64_t a2 = A < 0 ? ~0ull : 0ull;
    const uint64_t b1 = (uint64_t)L2 << 16;
    const uint64_t b2 = (uint64_t)(L2 >> 48);
    w0 = a0;
    w1 = a1 + b1;
    const uint64_t c = w1 < a1 ? 1ull : 0ull;
    w2 = a2 + b2 + c;
}

// Exact 192-bit atomic accumulate (mod 2^192) with explicit carries.
__device__ __forceinline__ void g_add192(uint64_t* p0, uint64_t* p1, uint64_t* p2, uint64_t w0, uint64_t w1,
                                         uint64_t w2) {
    uint64_t c0 = 0;
    if (w0) {
        const uint64_t o0 = atomicAdd((unsigned long long*)p0, (unsigned long long)w0);
        c0 = (o0 + w0) < o0 ? 1ull : 0ull;
    }
    const uint64_t a1 = w1 + c0;
    uint64_t c1 = (a1 < w1) ? 1ull : 0ull;
    if (a1) {
        const uint64_t o1 = atomicAdd((unsigned long long*)p1, (unsigned long long)a1);
        c1 += (o1 + a1) < o1 ? 1ull : 0ull;
    }
    const uint64_t a2 = w2 + c1;
    if (a2) atomicAdd((unsigned long long*)p2, (unsigned long long)a2);
}

__device__ __forceinline__ uint64_t* gfield(const GbParams& p, int f, int64_t s) {
    return p.gtab + (int64_t)f * (p.gcap + 2) + s;
}

// Per-thread running diagnostics, reduced once per workgroup.
struct ThreadDiag {
    uint32_t maxex[kMaxAcc];
    uint32_t fxfl[kMaxAcc];
    uint32_t nsel;
    uint32_t nglobal;
};

// Apply one selected row to an LDS slot (LDS=true) or a global slot.
template <bool LDS>
__device__ __forceinline__ void apply_row(const GbParams& p, uint64_t* lds, int L, int64_t s, int64_t row,
                                          const uint64_t* vals, uint32_t validmask, ThreadDiag& d) {
    auto F = [&](int f) -> unsigned long long* {
        if (LDS) return (unsigned long long*)&lds[f * L + s];
        return (unsigned long long*)gfield(p, f, s);
    };
    atomicAdd(F(p.f_len), 1ull);
    if (p.f_first >= 0) atomicMin(F(p.f_first), (unsigned long long)row);
#pragma unroll
    for (int a = 0; a < kMaxAcc; ++a) {
        if (a >= p.nacc) break;
        if (!((validmask >> a) & 1u)) continue;
        const AccSpec& ac = p.acc[a];
        const uint64_t x = vals[a];
        if (ac.f_cnt >= 0) atomicAdd(F(ac.f_cnt), 1ull);
        if (ac.flags & (A_FSUM | A_FSUMCAST | A_MIN | A_MAX)) {
            const bool isf = (ac.flags & A_FSUMCAST) == 0 && p.cols[ac.col].dtype == PLGPU_F64;
            bool is_nan = false;
            if (isf) {
                const uint64_t ab = x & 0x7fffffffffffffffull;
                if (ab >= 0x7ff0000000000000ull) {
                    uint32_t fl = ab > 0x7ff0000000000000ull ? FL_NAN : ((x >> 63) ? FL_NINF : FL_PINF);
                    is_nan = fl == FL_NAN;
                    atomicOr(F(ac.f_flags), (unsigned long long)fl);
                } else if (ac.flags & A_FSUM) {
                    uint64_t l0, l1, l2;
                    uint32_t ex;
                    if (fx_limbs(x, p.bottoms[a], l0, l1, l2, d.fxfl[a], ex)) {
                        d.maxex[a] = d.maxex[a] > ex ? d.maxex[a] : ex;
                        if (LDS) {
                            if (l0) atomicAdd(F(ac.f_sum), (unsigned long long)l0);
                            if (l1) atomicAdd(F(ac.f_sum + 1), (unsigned long long)l1);
                            if (l2) atomicAdd(F(ac.f_sum + 2), (unsigned long long)l2);
                        } else {
                            uint64_t w0, w1, w2;
                            limbs_to_192((int64_t)l0, (int64_t)l1, (int64_t)l2, w0, w1, w2);
                            g_add192((uint64_t*)F(ac.f_sum), (uint64_t*)F(ac.f_sum + 1), (uint64_t*)F(ac.f_sum + 2),
                                     w0, w1, w2);
                        }
                    }
                }
            }
            if (ac.flags & A_FSUMCAST) {
                uint64_t l0, l1, l2;
                uint32_t ex;
                const uint64_t xb = f64_bits((double)(int64_t)x);
                if (fx_limbs(xb, p.bottoms[a], l0, l1, l2, d.fxfl[a], ex)) {
                    d.maxex[a] = d.maxex[a] > ex ? d.maxex[a] : ex;
                    if (LDS) {
                        if (l0) atomicAdd(F(ac.f_sum), (unsigned long long)l0);
                        if (l1) atomicAdd(F(ac.f_sum + 1), (unsigned long long)l1);
                        if (l2) atomicAdd(F(ac.f_sum + 2), (unsigned long long)l2);
                    } else {
                        uint64_t w0, w1, w2;
                        limbs_to_192((int64_t)l0, (int64_t)l1, (int64_t)l2, w0, w1, w2);
                        g_add192((uint64_t*)F(ac.f_sum), (uint64_t*)F(ac.f_sum + 1), (uint64_t*)F(ac.f_sum + 2), w0,
                                 w1, w2);
                    }
                }
            }
            if ((ac.flags & (A_MIN | A_MAX)) && !is_nan) {
                const uint64_t o = isf ? ord_f64(x) : ord_i64(x);
                if (ac.flags & A_MIN) atomicMin(F(ac.f_min), (unsigned long long)o);
                if (ac.flags & A_MAX) atomicMax(F(ac.f_max), (unsigned long long)o);
            }
        }
        if (ac.flags & A_ISUM) atomicAdd(F(ac.f_isum), (unsigned long long)x);
    }
}

template <int PRED, int KEYW>  // PRED: 0 none, 1 simple, 2 program; KEYW: 4 / 8 bytes
__global__ __launch_bounds__(kGbThreads) void gb_kernel(GbParams p, DevProgram prog) {
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const int L = p.lcap + 2;
    for (int i = threadIdx.x; i < p.nfields * L; i += blockDim.x) {
        const int f = i / L;
        lds[i] = f == 0 ? kEmptyKey : (((p.min_init_mask >> f) & 1ull) ? ~0ull : 0ull);
    }
    ThreadDiag d;
#pragma unroll
    for (int a = 0; a < kMaxAcc; ++a) { d.maxex[a] = 0; d.fxfl[a] = 0; }
    d.nsel = 0;
    d.nglobal = 0;
    __syncthreads();

    const int64_t n = p.n;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += stride) {
        // ---- predicate
        bool sel = true;
        if (PRED == 1) {
            const DevCol& c = p.cols[prog.simple_col];
            sel = dev_valid(c, r) && simple_pred(prog.simple_isf, prog.simple_op, dev_load(c, r), prog.simple_imm);
        } else if (PRED == 2) {
            RowVal rv = eval_row(prog.code, prog.n, p.cols, r);
            sel = rv.valid && (rv.v & 1);
        }
        if (!sel) continue;
        // ---- loads (key + aggregated columns)
        const int64_t kp = p.key.offset + r;
        const uint64_t key = KEYW == 8 ? ((const uint64_t*)p.key.values)[kp]
                                       : (uint64_t)(int64_t)((const int32_t*)p.key.values)[kp];
        const bool kvalid = dev_valid(p.key, r);
        uint64_t vals[kMaxAcc];
        uint32_t vmask = 0;
#pragma unroll
        for (int a = 0; a < kMaxAcc; ++a) {
            vals[a] = 0;
            if (a < p.nacc) {
                const DevCol& c = p.cols[p.acc[a].col];
                vals[a] = dev_load(c, r);
                vmask |= dev_valid(c, r) ? (1u << a) : 0u;
            }
        }
        ++d.nsel;
        int s;
        if (!kvalid) s = p.lcap;
        else if (key == kEmptyKey) s = p.lcap + 1;
        else s = lds_find(lds, p.lbits, p.lcap, key);
        if (s >= 0) {
            apply_row<true>(p, lds, L, s, r, vals, vmask, d);
        } else {
            ++d.nglobal;
            const int64_t gs = g_find(p, key);
            if (gs < 0) {
                atomicAdd((unsigned long long*)&p.status[ST_TABLE_FULL], 1ull);
            } else {
                apply_row<false>(p, lds, L, gs, r, vals, vmask, d);
            }
        }
    }
    __syncthreads();

    // ---- fold the LDS table into the global table
    for (int s = threadIdx.x; s < L; s += blockDim.x) {
        const uint64_t len = lds[p.f_len * L + s];
        if (len == 0) continue;
        int64_t gs;
        if (s == p.lcap) {
            gs = p.gcap;
            atomicOr((unsigned long long*)&p.status[ST_SPECIAL], 1ull);
        } else if (s == p.lcap + 1) {
            gs = p.gcap + 1;
            atomicOr((unsigned long long*)&p.status[ST_SPECIAL], 2ull);
        } else {
            gs = g_find(p, lds[s]);
            if (gs < 0) {
                atomicAdd((unsigned long long*)&p.status[ST_TABLE_FULL], 1ull);
                continue;
            }
        }
        atomicAdd((unsigned long long*)gfield(p, p.f_len, gs), (unsigned long long)len);
        if (p.f_first >= 0)
            atomicMin((unsigned long long*)gfield(p, p.f_first, gs), (unsigned long long)lds[p.f_first * L + s]);
        for (int a = 0; a < p.nacc; ++a) {
            const AccSpec& ac = p.acc[a];
            if (ac.f_cnt >= 0) {
                const uint64_t v = lds[ac.f_cnt * L + s];
                if (v) atomicAdd((unsigned long long*)gfield(p, ac.f_cnt, gs), (unsigned long long)v);
            }
            if (ac.flags & (A_FSUM | A_FSUMCAST)) {
                uint64_t w0, w1, w2;
                limbs_to_192((int64_t)lds[ac.f_sum * L + s], (int64_t)lds[(ac.f_sum + 1) * L + s],
                             (int64_t)lds[(ac.f_sum + 2) * L + s], w0, w1, w2);
                g_add192(gfield(p, ac.f_sum, gs), gfield(p, ac.f_sum + 1, gs), gfield(p, ac.f_sum + 2, gs), w0, w1,
                         w2);
            }
            if (ac.flags & A_ISUM) {
                const uint64_t v = lds[ac.f_isum * L + s];
                if (v) atomicAdd((unsigned long long*)gfield(p, ac.f_isum, gs), (unsigned long long)v);
            }
            if (ac.flags & A_MIN) {
                const uint64_t v = lds[ac.f_min * L + s];
                if (v != ~0ull) atomicMin((unsigned long long*)gfield(p, ac.f_min, gs), (unsigned long long)v);
            }
            if (ac.flags & A_MAX) {
                const uint64_t v = lds[ac.f_max * L + s];
                if (v) atomicMax((unsigned long long*)gfield(p, ac.f_max, gs), (unsigned long long)v);
            }
            if (ac.f_flags >= 0) {
                const uint64_t v = lds[ac.f_flags * L + s];
                if (v) atomicOr((unsigned long long*)gfield(p, ac.f_flags, gs), (unsigned long long)v);
            }
        }
    }

    // ---- diagnostics: one atomic per wave
    uint64_t nsel = d.nsel, nglob = d.nglobal;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        nsel += __shfl_xor(nsel, off, 64);
        nglob += __shfl_xor(nglob, off, 64);
    }
    const int lane = threadIdx.x & 63;
    if (lane == 0) {
        if (nsel) atomicAdd((unsigned long long*)&p.status[ST_SELECTED], (unsigned long long)nsel);
        if (nglob) atomicAdd((unsigned long long*)&p.status[ST_GLOBAL_ROWS], (unsigned long long)nglob);
    }
#pragma unroll
    for (int a = 0; a < kMaxAcc; ++a) {
        uint32_t mx = d.maxex[a], fl = d.fxfl[a];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint32_t o = __shfl_xor(mx, off, 64);
            mx = mx > o ? mx : o;
            fl |= __shfl_xor(fl, off, 64);
        }
        if (lane == 0 && a < p.nacc) {
            if (mx) atomicMax((unsigned long long*)&p.status[ST_MAXEX + a], (unsigned long long)mx);
            if (fl) atomicOr((unsigned long long*)&p.status[ST_FXFLAGS + a], (unsigned long long)fl);
        }
    }
}

// Sampled max exponent -> fixed-point bottom, one workgroup per acc.
__global__ __launch_bounds__(256) void gb_sample_kernel(GbParams p, int32_t* bottoms, int64_t samples) {
    __shared__ uint32_t red[256];
    const int a = blockIdx.x;
    const AccSpec& ac = p.acc[a];
    uint32_t mx = 0;
    if (ac.flags & (A_FSUM | A_FSUMCAST)) {
        const DevCol& c = p.cols[ac.col];
        const int64_t n = p.n;
        const int64_t step = n > samples ? n / samples : 1;
        for (int64_t i = threadIdx.x; i * step < n && i < samples; i += blockDim.x) {
            const int64_t r = i * step;
            if (!dev_valid(c, r)) continue;
            uint64_t x = dev_load(c, r);
            if (ac.flags & A_FSUMCAST) x = f64_bits((double)(int64_t)x);
            const uint32_t ex = (uint32_t)(x >> 52) & 0x7FF;
            if (ex != 0x7FF && ex > mx) mx = ex;
        }
    }
    red[threadIdx.x] = mx;
    __syncthreads();
    for (int off = 128; off >= 1; off >>= 1) {
        if (threadIdx.x < off) red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + off]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        int e = red[0] == 0 ? 2046 : (int)red[0] + kHeadroomBinades;
        if (e > 2046) e = 2046;
        // fits iff ex <= bottom + 1075 + (window - 53)
        bottoms[a] = e - 1075 - (kSumWindowBits - 53);
    }
}

__global__ void gb_init_table_kernel(uint64_t* gtab, int64_t words_per_field, int nfields, uint64_t min_init_mask) {
    const int64_t total = words_per_field * nfields;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int f = (int)(i / words_per_field);
        gtab[i] = f == 0 ? kEmptyKey : (((min_init_mask >> f) & 1ull) ? ~0ull : 0ull);
    }
}

// 192-bit two's complement * 2^bottom -> correctly rounded double.
__device__ double fx_to_double(uint64_t w0, uint64_t w1, uint64_t w2, int bottom) {
    const bool neg = (int64_t)w2 < 0;
    if (neg) {
        w0 = ~w0; w1 = ~w1; w2 = ~w2;
        w0 += 1;
        const uint64_t c0 = w0 == 0;
        w1 += c0;
        const uint64_t c1 = c0 && w1 == 0;
        w2 += c1;
    }
    if ((w0 | w1 | w2) == 0) return 0.0;
    int p;
    if (w2) p = 128 + 63 - __clzll(w2);
    else if (w1) p = 64 + 63 - __clzll(w1);
    else p = 63 - __clzll(w0);
    uint64_t mant;
    int e = bottom;
    if (p <= 52) {
        mant = w0;
    } else {
        const int sh = p - 52;
        // mant = (W >> sh) & (2^53 - 1 | 2^52)
        auto shr = [&](int k) -> uint64_t {  // low 64 bits of W >> k
            if (k >= 128) return w2 >> (k - 128);
            if (k >= 64) {
                const int j = k - 64;
                return j == 0 ? w1 : (w1 >> j) | (w2 << (64 - j));
            }
            return k == 0 ? w0 : (w0 >> k) | (w1 << (64 - k));
        };
        mant = shr(sh) & ((1ull << 53) - 1);
        const uint64_t halfbit = (shr(sh - 1) & 1ull);
        // sticky: any bit below sh - 1
        bool sticky = false;
        const int sb = sh - 1;  // bits [0, sb) must be checked
        if (sb > 0) {
            if (sb >= 128) sticky = w0 || w1 || (sb > 128 && (w2 & ((sb - 128 >= 64) ? ~0ull : ((1ull << (sb - 128)) - 1))));
            else if (sb >= 64) sticky = w0 || (w1 & ((sb - 64 == 0) ? 0ull : ((1ull << (sb - 64)) - 1)));
            else sticky = (w0 & ((1ull << sb) - 1)) != 0;
        }
        if (halfbit && (sticky || (mant & 1))) {
            ++mant;
            if (mant == (1ull << 53)) {
                mant >>= 1;
                ++e;
            }
        }
        e += sh;
    }
    const double r = ldexp((double)mant, e);
    return neg ? -r : r;
}

struct OutSpec {
    int32_t kind;
    int32_t acc;
    int32_t out_dtype;
    int32_t in_isf;
    void* values;
    uint32_t* validity;
};

struct FinParams {
    OutSpec out[PLGPU_MAX_COLS * 2];
    int32_t nout;
    int32_t _pad;
    int64_t* out_keys;
    uint32_t* out_key_valid;
    uint64_t* out_first;  // optional
    int64_t cap;          // allocated output rows (guards against a miscount)
};

__global__ void gb_finalize_kernel(GbParams p, FinParams fp) {
    const int64_t total = p.gcap + 2;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < total;
         s += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t len = *gfield(p, p.f_len, s);
        if (len == 0) continue;
        const int64_t g = (int64_t)atomicAdd((unsigned long long*)&p.status[ST_GROUPS_OUT], 1ull);
        if (g >= fp.cap) continue;
        const bool null_key = s == p.gcap;
        fp.out_keys[g] = null_key ? 0 : (int64_t)(s == p.gcap + 1 ? kEmptyKey : *gfield(p, 0, s));
        if (!null_key) atomicOr(&fp.out_key_valid[g >> 5], 1u << (g & 31));
        if (fp.out_first) fp.out_first[g] = *gfield(p, p.f_first, s);
        for (int o = 0; o < fp.nout; ++o) {
            const OutSpec& os = fp.out[o];
            const AccSpec& ac = p.acc[os.acc];
            bool valid = true;
            const uint64_t cnt = ac.f_cnt >= 0 ? *gfield(p, ac.f_cnt, s) : len;
            const uint64_t flags = ac.f_flags >= 0 ? *gfield(p, ac.f_flags, s) : 0;
            switch (os.kind) {
            case PLGPU_AGG_LEN: ((uint32_t*)os.values)[g] = (uint32_t)len; break;
            case PLGPU_AGG_COUNT: ((uint32_t*)os.values)[g] = (uint32_t)cnt; break;
            case PLGPU_AGG_SUM:
            case PLGPU_AGG_MEAN: {
                if (os.kind == PLGPU_AGG_SUM && !os.in_isf) {
                    const uint64_t v = *gfield(p, ac.f_isum, s);
                    if (os.out_dtype == PLGPU_I64) ((uint64_t*)os.values)[g] = v;
                    else ((uint32_t*)os.values)[g] = (uint32_t)v;
                    break;
                }
                double sum;
                if (flags & FL_NAN || ((flags & FL_PINF) && (flags & FL_NINF))) sum = __builtin_nan("");
                else if (flags & FL_PINF) sum = __builtin_inf();
                else if (flags & FL_NINF) sum = -__builtin_inf();
                else sum = fx_to_double(*gfield(p, ac.f_sum, s), *gfield(p, ac.f_sum + 1, s),
                                        *gfield(p, ac.f_sum + 2, s), p.bottoms[os.acc]);
                if (os.kind == PLGPU_AGG_MEAN) {
                    if (cnt == 0) { valid = false; sum = 0.0; }
                    else sum = sum / (double)cnt;
                }
                ((double*)os.values)[g] = sum;
                break;
            }
            case PLGPU_AGG_MIN:
            case PLGPU_AGG_MAX: {
                const uint64_t o = *gfield(p, os.kind == PLGPU_AGG_MIN ? ac.f_min : ac.f_max, s);
                const bool none = os.kind == PLGPU_AGG_MIN ? (o == ~0ull) : (o == 0ull);
                if (os.in_isf) {
                    double v;
                    if (cnt == 0) { valid = false; v = 0.0; }
                    else if (none) v = __builtin_nan("");  // every valid value was NaN
                    else v = as_f64(unord_f64(o));
                    ((double*)os.values)[g] = v;
                } else {
                    const int64_t v = (cnt == 0 || none) ? 0 : (int64_t)(o ^ 0x8000000000000000ull);
                    if (cnt == 0) valid = false;
                    if (os.out_dtype == PLGPU_I64) ((int64_t*)os.values)[g] = v;
                    else ((int32_t*)os.values)[g] = (int32_t)v;
                }
                break;
            }
            default: break;
            }
            if (os.validity && valid) atomicOr(&os.validity[g >> 5], 1u << (g & 31));
        }
    }
}

// Gather rows of fixed-width buffers by a permutation (maintain_order).
template <typename T>
__global__ void gather_kernel(const T* __restrict__ src, const int64_t* __restrict__ perm, T* __restrict__ dst,
                              int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[perm[i]];
}
__global__ void narrow_i64_kernel(const int64_t* __restrict__ a, int32_t* __restrict__ b, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        b[i] = (int32_t)a[i];
}
__global__ void gather_bits_kernel(const uint32_t* __restrict__ src, const int64_t* __restrict__ perm,
                                   uint32_t* __restrict__ dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = perm[i];
        if ((src[j >> 5] >> (j & 31)) & 1u) atomicOr(&dst[i >> 5], 1u << (i & 31));
    }
}

// ------------------------------------------------------------- host
static int g_num_cus = 0;
static int num_cus() {
    if (g_num_cus == 0) {
        int dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
            g_num_cus = prop.multiProcessorCount;
        else
            g_num_cus = 256;
    }
    return g_num_cus;
}

struct Plan {
    GbParams p;
    std::vector<OutSpec> outs;
    int acc_of_agg[64];
    size_t lds_bytes;
    int grid;
};

static int plan_groupby(const plgpu_column* key, const plgpu_column* cols, int32_t ncols, const plgpu_agg* aggs,
                        int32_t naggs, bool maintain_order, Plan* pl) {
    GbParams& p = pl->p;
    std::memset(&p, 0, sizeof p);
    p.key.values = key->values;
    p.key.validity = key->validity;
    p.key.offset = key->offset;
    p.key.dtype = key->dtype;
    for (int i = 0; i < ncols; ++i) {
        p.cols[i].values = cols[i].values;
        p.cols[i].validity = cols[i].validity;
        p.cols[i].offset = cols[i].offset;
        p.cols[i].dtype = cols[i].dtype;
    }
    p.n = key->length;
    int nf = 1;  // field 0: keys
    p.f_len = nf++;
    p.f_first = maintain_order ? nf++ : -1;
    if (maintain_order) p.min_init_mask |= 1ull << p.f_first;
    int acc_of_col[PLGPU_MAX_COLS];
    for (int i = 0; i < PLGPU_MAX_COLS; ++i) acc_of_col[i] = -1;
    p.nacc = 0;
    // pass 1: flags per column
    for (int i = 0; i < naggs; ++i) {
        const int c = aggs[i].col;
        if (c < 0 || c >= ncols) return fail(PLGPU_ERR_INVALID, "aggregation column index out of range");
        const int32_t dt = cols[c].dtype;
        if (dt != PLGPU_F64 && dt != PLGPU_I64 && dt != PLGPU_I32 && dt != PLGPU_U32)
            return fail(PLGPU_ERR_INVALID, "aggregation not supported for this dtype");
        if (acc_of_col[c] < 0) {
            if (p.nacc == kMaxAcc) return fail(PLGPU_ERR_INVALID, "too many aggregated columns (max 6)");
            acc_of_col[c] = p.nacc;
            AccSpec& ac = p.acc[p.nacc++];
            std::memset(&ac, 0xff, sizeof ac);
            ac.col = c;
            ac.flags = 0;
        }
        AccSpec& ac = p.acc[acc_of_col[c]];
        const bool isf = dt == PLGPU_F64;
        const bool nullable = cols[c].validity != nullptr;
        switch (aggs[i].kind) {
        case PLGPU_AGG_SUM: ac.flags |= isf ? (A_FSUM | A_FLAGS) : A_ISUM; break;
        case PLGPU_AGG_MEAN: ac.flags |= isf ? (A_FSUM | A_FLAGS) : A_FSUMCAST; if (nullable) ac.flags |= A_CNT; break;
        case PLGPU_AGG_MIN: ac.flags |= A_MIN | (isf ? A_FLAGS : 0) | A_CNT; break;
        case PLGPU_AGG_MAX: ac.flags |= A_MAX | (isf ? A_FLAGS : 0) | A_CNT; break;
        case PLGPU_AGG_COUNT: if (nullable) ac.flags |= A_CNT; break;
        case PLGPU_AGG_LEN: break;
        default: return fail(PLGPU_ERR_INVALID, "unknown aggregation kind");
        }
        pl->acc_of_agg[i] = acc_of_col[c];
    }
    // MIN/MAX validity needs a non-null count only when the column is nullable
    for (int a = 0; a < p.nacc; ++a) {
        AccSpec& ac = p.acc[a];
        if ((ac.flags & A_CNT) && cols[ac.col].validity == nullptr) ac.flags &= ~A_CNT;
        if (ac.flags & (A_FSUM | A_FSUMCAST)) { ac.f_sum = nf; nf += 3; }
        if (ac.flags & A_ISUM) ac.f_isum = nf++;
        if (ac.flags & A_CNT) ac.f_cnt = nf++;
        if (ac.flags & A_MIN) { ac.f_min = nf++; p.min_init_mask |= 1ull << ac.f_min; }
        if (ac.flags & A_MAX) ac.f_max = nf++;
        if (ac.flags & A_FLAGS) ac.f_flags = nf++;
    }
    if (nf > kMaxFields) return fail(PLGPU_ERR_INVALID, "too many accumulator fields");
    p.nfields = nf;
    // outputs
    pl->outs.clear();
    for (int i = 0; i < naggs; ++i) {
        OutSpec o;
        std::memset(&o, 0, sizeof o);
        o.kind = aggs[i].kind;
        o.acc = pl->acc_of_agg[i];
        const int32_t dt = cols[aggs[i].col].dtype;
        o.in_isf = dt == PLGPU_F64;
        switch (o.kind) {
        case PLGPU_AGG_LEN:
        case PLGPU_AGG_COUNT: o.out_dtype = PLGPU_U32; break;
        case PLGPU_AGG_MEAN: o.out_dtype = PLGPU_F64; break;
        default: o.out_dtype = dt == PLGPU_F64 ? PLGPU_F64 : (dt == PLGPU_I64 ? PLGPU_I64 : dt); break;
        }
        pl->outs.push_back(o);
    }
    // LDS sizing: as many slots as fit 80 KiB (two 512-thread workgroups per CU)
    const size_t budget = 80 * 1024;
    int lbits = 12;
    while (lbits > 6 && (size_t)nf * ((1u << lbits) + 2) * 8 > budget) --lbits;
    p.lbits = lbits;
    p.lcap = 1 << lbits;
    pl->lds_bytes = (size_t)nf * (p.lcap + 2) * 8;
    const int per_cu = pl->lds_bytes <= 80 * 1024 ? 2 : 1;
    int64_t grid = (int64_t)num_cus() * per_cu;
    const int64_t need = (p.n + kMaxRowsPerWg - 1) / kMaxRowsPerWg;
    if (grid < need) grid = need;
    const int64_t useful = (p.n + kGbThreads - 1) / kGbThreads;
    if (grid > useful) grid = useful < 1 ? 1 : useful;
    pl->grid = (int)grid;
    return PLGPU_OK;
}

template <int PRED, int KEYW>
static hipError_t launch_main(const Plan& pl, const DevProgram& dp, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)gb_kernel<PRED, KEYW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr_set = true;
    }
    gb_kernel<PRED, KEYW><<<pl.grid, kGbThreads, pl.lds_bytes, s>>>(pl.p, dp);
    return hipGetLastError();
}

static hipError_t launch_main_dispatch(const Plan& pl, const DevProgram& dp, int pred, int keyw, hipStream_t s) {
    if (keyw == 8) {
        if (pred == 0) return launch_main<0, 8>(pl, dp, s);
        if (pred == 1) return launch_main<1, 8>(pl, dp, s);
        return launch_main<2, 8>(pl, dp, s);
    }
    if (pred == 0) return launch_main<0, 4>(pl, dp, s);
    if (pred == 1) return launch_main<1, 4>(pl, dp, s);
    return launch_main<2, 4>(pl, dp, s);
}

static int log2_ceil(int64_t x) {
    int b = 0;
    while ((int64_t(1) << b) < x) ++b;
    return b;
}

}  // namespace plgpu

using namespace plgpu;

PLGPU_API int plgpu_group_by_agg(const plgpu_column* key, const plgpu_column* cols, int32_t ncols,
                                 const plgpu_instr* program, int32_t n_instr, const plgpu_agg* aggs, int32_t naggs,
                                 int32_t maintain_order, plgpu_column* out_key, plgpu_column* out_aggs,
                                 plgpu_groupby_info* info, void* stream) {
    hipStream_t s = as_stream(stream);
    if (key == nullptr || out_key == nullptr) return fail(PLGPU_ERR_INVALID, "key / out_key is NULL");
    if (ncols < 0 || ncols > PLGPU_MAX_COLS) return fail(PLGPU_ERR_INVALID, "too many columns (max 8)");
    if (naggs < 0 || naggs > PLGPU_MAX_COLS * 2) return fail(PLGPU_ERR_INVALID, "too many aggregations (max 16)");
    if (key->dtype != PLGPU_I64 && key->dtype != PLGPU_I32)
        return fail(PLGPU_ERR_SCHEMA, "group-by key must be Int64 or Int32");
    for (int i = 0; i < ncols; ++i)
        if (cols[i].length != key->length) return fail(PLGPU_ERR_SHAPE, "columns must match the key length");
    std::memset(out_key, 0, sizeof *out_key);
    for (int i = 0; i < naggs; ++i) std::memset(&out_aggs[i], 0, sizeof(plgpu_column));
    plgpu_groupby_info local_info;
    if (info == nullptr) info = &local_info;
    std::memset(info, 0, sizeof *info);

    DevProgram dp;
    std::memset(&dp, 0, sizeof dp);
    int pred = 0;
    int rc;
    if (program != nullptr && n_instr > 0) {
        if ((rc = lower_program(cols, ncols, program, n_instr, &dp))) return rc;
        if (dp.out_dtype != PLGPU_BOOL) return fail(PLGPU_ERR_SCHEMA, "filter predicate must be of type `Boolean`");
        pred = dp.simple ? 1 : 2;
    }
    Plan pl;
    if ((rc = plan_groupby(key, cols, ncols, aggs, naggs, maintain_order != 0, &pl))) return rc;
    GbParams& p = pl.p;
    const int64_t n = p.n;

    // device scratch: status + bottoms
    uint64_t* status = nullptr;
    if ((rc = dev_alloc((void**)&status, ST_WORDS * 8 + kMaxAcc * 4, s))) return rc;
    int32_t* bottoms = (int32_t*)(status + ST_WORDS);
    p.status = status;
    p.bottoms = bottoms;

    int64_t cap_hint = n < (int64_t(1) << 20) ? n : (int64_t(1) << 20);
    int gbits = log2_ceil(cap_hint * 2 < 1024 ? 1024 : cap_hint * 2);
    uint64_t* gtab = nullptr;
    int32_t host_bottoms[kMaxAcc] = {0};
    bool bottoms_from_host = false;
    uint64_t st[ST_WORDS];
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    PLGPU_HIP(hipEventCreate(&ev0));
    PLGPU_HIP(hipEventCreate(&ev1));
    int attempt = 0;
    for (;; ++attempt) {
        p.gbits = gbits;
        p.gcap = int64_t(1) << gbits;
        const size_t gwords = (size_t)p.nfields * (p.gcap + 2);
        if ((rc = dev_alloc((void**)&gtab, gwords * 8, s))) break;
        p.gtab = gtab;
        const int ig = (int)std::min<int64_t>((int64_t)(gwords + 255) / 256, 256 * 16);
        if (getenv("PLGPU_MEMSET_INIT")) {
            for (int f = 0; f < p.nfields; ++f) {
                const int byte = f == 0 ? 0 : (((p.min_init_mask >> f) & 1ull) ? 0xFF : 0);
                PLGPU_HIP(hipMemsetAsync(gtab + (size_t)f * (p.gcap + 2), byte, (size_t)(p.gcap + 2) * 8, s));
            }
            gb_init_table_kernel<<<ig, 256, 0, s>>>(gtab, p.gcap + 2, 1, 0);
        } else {
            gb_init_table_kernel<<<ig, 256, 0, s>>>(gtab, p.gcap + 2, p.nfields, p.min_init_mask);
        }
        if (getenv("PLGPU_DEBUG")) {
            std::vector<uint64_t> chk(gwords);
            PLGPU_HIP(hipMemcpyAsync(chk.data(), gtab, gwords * 8, hipMemcpyDeviceToHost, s));
            PLGPU_HIP(hipStreamSynchronize(s));
            size_t bad = 0;
            for (size_t i = 0; i < gwords; ++i) {
                const int f = (int)(i / (size_t)(p.gcap + 2));
                const uint64_t want = f == 0 ? kEmptyKey : (((p.min_init_mask >> f) & 1ull) ? ~0ull : 0ull);
                bad += chk[i] != want;
            }
            size_t firstbad = gwords;
            for (size_t i = 0; i < gwords && firstbad == gwords; ++i) {
                const int f = (int)(i / (size_t)(p.gcap + 2));
                const uint64_t want = f == 0 ? kEmptyKey : (((p.min_init_mask >> f) & 1ull) ? ~0ull : 0ull);
                if (chk[i] != want) firstbad = i;
            }
            fprintf(stderr, "[plgpu] init check: %zu bad words of %zu (gtab=%p) first bad %zu field %zu val %llx mask %llx\n",
                    bad, gwords, (void*)gtab, firstbad, firstbad / (size_t)(p.gcap + 2),
                    firstbad < gwords ? (unsigned long long)chk[firstbad] : 0ull, (unsigned long long)p.min_init_mask);
        }
        PLGPU_HIP(hipMemsetAsync(status, 0, ST_WORDS * 8, s));
        if (bottoms_from_host) {
            PLGPU_HIP(hipMemcpyAsync(bottoms, host_bottoms, sizeof host_bottoms, hipMemcpyHostToDevice, s));
        } else if (p.nacc > 0) {
            gb_sample_kernel<<<p.nacc, 256, 0, s>>>(p, bottoms, 65536);
        }
        PLGPU_HIP(hipGetLastError());
        PLGPU_HIP(hipEventRecord(ev0, s));
        if (n > 0) PLGPU_HIP(launch_main_dispatch(pl, dp, pred, key->dtype == PLGPU_I64 ? 8 : 4, s));
        PLGPU_HIP(hipEventRecord(ev1, s));
        PLGPU_HIP(hipMemcpyAsync(st, status, sizeof st, hipMemcpyDeviceToHost, s));
        PLGPU_HIP(hipMemcpyAsync(host_bottoms, bottoms, sizeof host_bottoms, hipMemcpyDeviceToHost, s));
        PLGPU_HIP(hipStreamSynchronize(s));
        if (getenv("PLGPU_DEBUG")) {
            fprintf(stderr,
                    "[plgpu] gb attempt %d: n=%lld grid=%d lcap=%d gcap=%lld nfields=%d lds=%zu newkeys=%llu "
                    "special=%llu global_rows=%llu full=%llu selected=%llu\n",
                    attempt, (long long)n, pl.grid, p.lcap, (long long)p.gcap, p.nfields, pl.lds_bytes,
                    (unsigned long long)st[ST_NEWKEYS], (unsigned long long)st[ST_SPECIAL],
                    (unsigned long long)st[ST_GLOBAL_ROWS], (unsigned long long)st[ST_TABLE_FULL],
                    (unsigned long long)st[ST_SELECTED]);
            for (int a = 0; a < p.nacc; ++a)
                fprintf(stderr, "[plgpu]   acc %d flags=%d bottom=%d maxex=%llu fx=%llu\n", a, p.acc[a].flags,
                        host_bottoms[a], (unsigned long long)st[ST_MAXEX + a], (unsigned long long)st[ST_FXFLAGS + a]);
        }
        bool again = false;
        if (st[ST_TABLE_FULL] > 0) {
            gbits = log2_ceil(std::max<int64_t>((int64_t)st[ST_NEWKEYS] * 4, p.gcap * 8));
            again = true;
        }
        for (int a = 0; a < p.nacc; ++a) {
            if (!(p.acc[a].flags & (A_FSUM | A_FSUMCAST))) continue;
            const int tmax = (int)st[ST_MAXEX + a];
            const int allowed = host_bottoms[a] + 1075 + (kSumWindowBits - 53);
            const uint64_t fl = st[ST_FXFLAGS + a];
            if ((fl & 1u) || ((fl & 2u) && tmax > 0 && tmax < allowed)) {
                // refit the window to the true max exponent
                const int e = (fl & 1u) ? std::max(tmax, allowed + 1) : tmax;
                host_bottoms[a] = e - 1075 - (kSumWindowBits - 53);
                again = true;
            }
        }
        if (!again || attempt >= 3) {
            if (again) rc = fail(PLGPU_ERR_CAPACITY, "group-by did not converge after retries");
            break;
        }
        // overflowed values were dropped: the whole pass must rerun
        bottoms_from_host = true;
        dev_free(gtab, s);
        gtab = nullptr;
    }
    float ms = 0.f;
    if (rc == PLGPU_OK) (void)hipEventElapsedTime(&ms, ev0, ev1);
    (void)hipEventDestroy(ev0);
    (void)hipEventDestroy(ev1);
    if (rc) {
        dev_free(gtab, s);
        dev_free(status, s);
        return rc;
    }
    // overflow that persisted means the window could not hold a value: the
    // max exponent pass above already refit it, so only inexact remains.
    int64_t groups = (int64_t)st[ST_NEWKEYS] + ((st[ST_SPECIAL] & 1) ? 1 : 0) + ((st[ST_SPECIAL] & 2) ? 1 : 0);
    info->rows_in = n;
    info->rows_selected = (int64_t)st[ST_SELECTED];
    info->groups = groups;
    info->global_path_rows = (int64_t)st[ST_GLOBAL_ROWS];
    info->reruns = attempt;
    info->lds_slots = p.lcap;
    info->grid = pl.grid;
    info->table_capacity = p.gcap;
    info->main_kernel_ms = ms;
    for (int a = 0; a < p.nacc; ++a)
        if (st[ST_FXFLAGS + a] & 2u) info->sum_inexact |= 1 << a;

    // ---- outputs
    FinParams fp;
    std::memset(&fp, 0, sizeof fp);
    rc = make_owned_column(out_key, key->dtype == PLGPU_I32 ? PLGPU_I32 : PLGPU_I64, groups, true, s);
    if (rc == PLGPU_OK && key->dtype == PLGPU_I32) {
        // keys are materialised as i64 first, then narrowed below
        plgpu_column_release(out_key);
        rc = make_owned_column(out_key, PLGPU_I64, groups, true, s);
    }
    for (int i = 0; i < naggs && rc == PLGPU_OK; ++i) {
        const OutSpec& o = pl.outs[i];
        const bool nullable = o.kind == PLGPU_AGG_MEAN || o.kind == PLGPU_AGG_MIN || o.kind == PLGPU_AGG_MAX;
        rc = make_owned_column(&out_aggs[i], o.out_dtype, groups, nullable, s);
    }
    uint64_t* first = nullptr;
    if (rc == PLGPU_OK && maintain_order && groups > 0) rc = dev_alloc((void**)&first, groups * 8, s);
    if (rc == PLGPU_OK && groups > 0) {
        fp.nout = naggs;
        for (int i = 0; i < naggs; ++i) {
            fp.out[i] = pl.outs[i];
            fp.out[i].values = (void*)out_aggs[i].values;
            fp.out[i].validity = (uint32_t*)out_aggs[i].validity;
            if (fp.out[i].validity) (void)hipMemsetAsync(fp.out[i].validity, 0, ((groups + 63) / 64) * 8, s);
        }
        fp.out_keys = (int64_t*)out_key->values;
        fp.out_key_valid = (uint32_t*)out_key->validity;
        (void)hipMemsetAsync((void*)out_key->validity, 0, ((groups + 63) / 64) * 8, s);
        fp.out_first = first;
        fp.cap = groups;
        const int fg = (int)std::min<int64_t>((p.gcap + 2 + 255) / 256, 256 * 16);
        gb_finalize_kernel<<<fg, 256, 0, s>>>(p, fp);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) rc = hip_fail(e, "gb_finalize_kernel");
        uint64_t produced = 0;
        if (rc == PLGPU_OK) {
            e = hipMemcpyAsync(&produced, status + ST_GROUPS_OUT, 8, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) rc = hip_fail(e, "finalize count");
        }
        if (rc == PLGPU_OK && (int64_t)produced != groups) {
            char buf[256];
            snprintf(buf, sizeof buf,
                     "internal: group count mismatch (inserted %llu + specials %llu, finalized %llu, "
                     "global rows %llu, table_full %llu)",
                     (unsigned long long)st[ST_NEWKEYS], (unsigned long long)st[ST_SPECIAL],
                     (unsigned long long)produced, (unsigned long long)st[ST_GLOBAL_ROWS],
                     (unsigned long long)st[ST_TABLE_FULL]);
            rc = fail(PLGPU_ERR_CAPACITY, buf);
        }
    }
    if (rc == PLGPU_OK && maintain_order && groups > 1) {
        // order groups by first occurrence (host argsort of `groups` row ids)
        std::vector<uint64_t> hf(groups);
        std::vector<int64_t> perm(groups);
        hipError_t e = hipMemcpyAsync(hf.data(), first, groups * 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "copy first rows");
        if (rc == PLGPU_OK) {
            std::iota(perm.begin(), perm.end(), 0);
            std::sort(perm.begin(), perm.end(), [&](int64_t a, int64_t b) { return hf[a] < hf[b]; });
            int64_t* dperm = nullptr;
            rc = dev_alloc((void**)&dperm, groups * 8, s);
            if (rc == PLGPU_OK) {
                (void)hipMemcpyAsync(dperm, perm.data(), groups * 8, hipMemcpyHostToDevice, s);
                const int gg = (int)std::min<int64_t>((groups + 255) / 256, 4096);
                auto permute = [&](plgpu_column* c) -> int {
                    plgpu_column nc;
                    int r2 = make_owned_column(&nc, c->dtype, groups, c->validity != nullptr, s);
                    if (r2) return r2;
                    if (dtype_bytes(c->dtype) == 8)
                        gather_kernel<uint64_t><<<gg, 256, 0, s>>>((const uint64_t*)c->values, dperm,
                                                                   (uint64_t*)nc.values, groups);
                    else
                        gather_kernel<uint32_t><<<gg, 256, 0, s>>>((const uint32_t*)c->values, dperm,
                                                                   (uint32_t*)nc.values, groups);
                    if (c->validity) {
                        (void)hipMemsetAsync((void*)nc.validity, 0, ((groups + 63) / 64) * 8, s);
                        gather_bits_kernel<<<gg, 256, 0, s>>>((const uint32_t*)c->validity, dperm,
                                                              (uint32_t*)nc.validity, groups);
                    }
                    plgpu_column_release(c);
                    *c = nc;
                    return PLGPU_OK;
                };
                rc = permute(out_key);
                for (int i = 0; i < naggs && rc == PLGPU_OK; ++i) rc = permute(&out_aggs[i]);
                dev_free(dperm, s);
                if (rc == PLGPU_OK) {
                    e = hipStreamSynchronize(s);  // keep `perm` alive until the copy ran
                    if (e != hipSuccess) rc = hip_fail(e, "permute");
                }
            }
        }
    }
    if (rc == PLGPU_OK && key->dtype == PLGPU_I32 && groups > 0) {
        // narrow the key back to Int32 (the reference keeps the key dtype)
        plgpu_column nk;
        rc = make_owned_column(&nk, PLGPU_I32, groups, true, s);
        if (rc == PLGPU_OK) {
            const int gg = (int)std::min<int64_t>((groups + 255) / 256, 4096);
            narrow_i64_kernel<<<gg, 256, 0, s>>>((const int64_t*)out_key->values, (int32_t*)nk.values, groups);
            (void)hipMemcpyAsync((void*)nk.validity, out_key->validity, ((groups + 63) / 64) * 8,
                                 hipMemcpyDeviceToDevice, s);
            plgpu_column_release(out_key);
            *out_key = nk;
        }
    } else if (rc == PLGPU_OK && key->dtype == PLGPU_I32) {
        out_key->dtype = PLGPU_I32;
    }
    if (rc == PLGPU_OK) {
        out_key->null_count = (st[ST_SPECIAL] & 1) ? 1 : 0;
        PLGPU_HIP(hipStreamSynchronize(s));
    }
    dev_free(first, s);
    dev_free(gtab, s);
    dev_free(status, s);
    if (rc) {
        plgpu_column_release(out_key);
        for (int i = 0; i < naggs; ++i) plgpu_column_release(&out_aggs[i]);
    }
    return rc;
}
