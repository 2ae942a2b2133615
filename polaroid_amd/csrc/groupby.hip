// groupby.hip — fused predicate + hash group-by + aggregation on gfx950.
//
// Reference path (Rust): FilterExec (polars-mem-engine/src/executors/
// filter.rs:51) feeding GroupByStreamingExec / GroupByExec (group_by.rs:117,
// chosen at polars-mem-engine/src/planner/lp.rs:648), whose per-group folds
// are polars-expr/src/reduce/{sum,mean,min_max,count,len}.rs and
// polars-core/src/frame/group_by/aggregations/mod.rs:581 (agg_sum).
//
// Design:
//  * a planning launch samples the key column (distinct-key estimate, sizes
//    the LDS and global tables) and the summed f64 columns (max exponent ->
//    fixed-point window);
//  * one persistent launch streams the key + referenced columns once with
//    16-byte loads, four rows per thread issued before any is consumed,
//    evaluating the predicate in registers (no mask column);
//  * each workgroup owns an LDS open-addressing table (key -> slot) whose
//    accumulators are updated with LDS atomics; rows whose key does not fit
//    go straight to the global table (device-scope atomics); when the key
//    sample says the groups cannot fit LDS at all, the LDS stage is skipped;
//  * at the end each workgroup folds its LDS table into the global table;
//  * f64 sums are exact: every value becomes a 120-bit fixed-point integer
//    (3 carry-free 40-bit limbs in LDS, one 192-bit two's-complement integer
//    per group in HBM), rounded once at the end: the correctly rounded sum,
//    independent of arrival order — the deterministic answer the reference's
//    Kahan / naive row-order folds approximate.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <numeric>
#include <string>
#include <tuple>
#include <vector>

#include "groupby_kernels.hpp"

namespace plgpu {

// A small device -> host download (status words) through the runtime's
// pinned stage: the copy is queued and one synchronisation waits for it (a
// copy into pageable memory is staged and blocking, then a second wait).
static int d2h_stage(int n, void* const* dst, const void* const* src, const size_t* bytes, hipStream_t s) {
    return plgpu_memcpy_d2h_many(n, dst, src, bytes, (void*)s);
}


#ifdef PLGPU_CHECKS
static std::vector<GbChecksTake>& gb_checks_takers() {
    static std::vector<GbChecksTake> v;
    return v;
}
void gb_checks_register(GbChecksTake f) { gb_checks_takers().push_back(f); }
#endif

// ------------------------------------------------------ partitioned path
// Keys with more groups than one LDS table holds (DESIGN.md "Group-by for
// many groups"): the selected rows are radix-partitioned by a hash of the
// key into 2^B partitions of raw 8-byte words (the key, each aggregated
// column in register form and, for the first / last row fields, the input
// row id), so that every partition's groups fit the LDS table of the
// workgroup(s) that then aggregate it.  Up to kPartOneLevel bits take one
// scatter pass; more take two: B1 = B / 2 bits over the input rows, then
// B2 = B - B1 bits within each level-1 partition, so each pass keeps runs of
// >= ~16 rows per partition and column (the reference partitions by
// polars-utils/src/hashing.rs:72 HashPartitioner before its per-partition
// hash tables, polars-stream/src/nodes/group_by.rs:85).  The partition hash
// is independent of the table hashes (hash_slot / g_find take the top bits
// of a multiplicative hash).  Order inside a partition is irrelevant: every
// aggregate is order-independent (exact sums, min / max, counts, min / max
// row).
//
// Each pass is a radix-sort pass over (tile, digit) (sort.hip's downsweep
// structure): a count kernel writes every 4096-row tile's digit counts
// digit-major, one device scan turns them into output positions, and the
// scatter kernel ranks its tile's selected rows per wave with ballots (no
// atomics, no barriers), stages each column in LDS in digit order and
// writes one run per digit.  Level 2 tiles never straddle a level-1
// partition: the count matrix is laid out (level-1 partition, digit, tile),
// so the same one scan places every level-2 run after the runs of the
// partitions before it.
constexpr int kPartMaxBits = 16;   // partitions in all
constexpr int kPartOneLevel = 8;   // up to this many bits: one scatter pass
constexpr int kPsDigitBits = 8;    // digit bits per scatter pass
constexpr int kPsThreads = 256;
constexpr int kPsPer = 16;
constexpr int kPsTile = kPsThreads * kPsPer;  // 4096 rows; a wave ranks 1024 consecutive rows

struct PartOut {
    uint64_t* key;
    uint64_t* acc[kMaxAcc];
    uint32_t* rows;  // null unless the first / last row fields are in use
    uint8_t* nulls;  // null unless an input column is nullable: GbParams::part_nulls bits per row
    int64_t cap;     // rows each buffer holds
};

// Tile geometry of one scatter pass.  Level 1 (range == null): tile t is
// input rows [t * kPsTile, ...).  Level 2: the tiles of each level-1
// partition q are tstart[q] .. tstart[q + 1] - 1 (tpart maps a tile back
// to q), over the partition's rows [range[q], range[q + 1]) of the level-1
// buffers.  The digit of a key: (part_hash(key) >> sh) & (2^dbits - 1).
constexpr int kKeyRangeSlots = 256;  // PsGeom::keyrange pairs
struct PsGeom {
    int64_t n;
    int64_t ntiles;
    const uint64_t* range;
    const uint32_t* tstart;
    const uint32_t* tpart;
    int32_t sh;
    int32_t dbits;
    // null-key sentinel (sum-only runs with a nullable Int64 key): the level-1
    // count pass reduces the non-null keys' range into keyrange[0 .. 1]
    // (signed min, max pairs, kKeyRangeSlots of them by tile); the level-1
    // scatter then writes a null key as
    // `sentinel`, a value no row holds, so no null-bits column is needed
    int64_t* keyrange;
    int64_t sentinel;
    int32_t has_sentinel;
    int32_t _pad;
};

struct PsTile {
    int64_t base;    // the tile's kPsTile-aligned block of rows (its loads)
    int64_t lo, hi;  // rows of the tile (within the block)
    int64_t mbase;   // count matrix entry of (tile, digit d): mbase + d * ntq + tl
    int64_t ntq, tl;
};

__device__ __forceinline__ PsTile ps_tile(const PsGeom& g, int64_t t) {
    PsTile x;
    if (g.range == nullptr) {
        x.base = x.lo = t * kPsTile;
        x.hi = std::min<int64_t>(g.n, x.lo + kPsTile);
        x.mbase = 0;
        x.ntq = g.ntiles;
        x.tl = t;
    } else {
        // level 2: the aligned blocks of the level-1 buffers that level-1
        // partition q touches, each cut to the partition's rows (aligned
        // loads: a partition starts anywhere)
        const uint32_t q = g.tpart[t];
        const uint32_t t0 = g.tstart[q];
        x.ntq = (int64_t)(g.tstart[q + 1] - t0);
        x.tl = t - t0;
        x.mbase = (int64_t)t0 << g.dbits;
        const int64_t r0 = (int64_t)g.range[q], r1 = (int64_t)g.range[q + 1];
        x.base = (r0 & ~(int64_t)(kPsTile - 1)) + x.tl * kPsTile;
        x.lo = std::max<int64_t>(r0, x.base);
        x.hi = std::min<int64_t>(r1, x.base + kPsTile);
    }
    return x;
}

// Row k of this thread within its tile's block (c0 + k * 64 + lane,
// clamped to the tile's rows [lo, hi)): f(k, i) for k = 0 .. kPsPer - 1, i
// relative to the block.  A full tile takes the unclamped form, whose
// offsets are one register plus immediates (with a uniform base pointer:
// saddr loads, no 64-bit address per row).
template <typename F>
__device__ __forceinline__ void ps_rows(const PsTile& tl, int c0, F&& f) {
    const uint32_t i0 = (uint32_t)(c0 + (int)(threadIdx.x & 63));
    if (tl.lo == tl.base && tl.hi - tl.base == kPsTile) {
#pragma unroll
        for (int k = 0; k < kPsPer; ++k) f(k, i0 + (uint32_t)(k * 64));
    } else {
        const uint32_t first = (uint32_t)(tl.lo - tl.base), last = (uint32_t)(tl.hi - tl.base - 1);
#pragma unroll
        for (int k = 0; k < kPsPer; ++k) f(k, min(max(i0 + (uint32_t)(k * 64), first), last));
    }
}

// One column's values at this thread's rows of the tile: the level-1
// buffers (L2), a null-free 8-byte column (F8) or any column in register
// form (dev_load).
template <bool L2, bool F8>
__device__ __forceinline__ void ps_col(const DevCol& c, const uint64_t* buf, const PsTile& tl, int c0,
                                       uint64_t (&v)[kPsPer]) {
    if (L2 || F8) {
        const uint64_t* b = (L2 ? buf : (const uint64_t*)c.values + c.offset) + tl.base;
        ps_rows(tl, c0, [&](int k, uint32_t i) { v[k] = __builtin_nontemporal_load(b + i); });
    } else {
        ps_rows(tl, c0, [&](int k, uint32_t i) { v[k] = dev_load(c, tl.base + (int64_t)i); });
    }
}

// The tile's keys (and a simple predicate's column) for this thread's rows,
// and which rows are selected.  L2: the level-1 buffers (every row
// selected).  F8: the key and predicate columns are null-free 8-byte
// columns.
// NUL: some key / aggregated / predicate column has a validity bitmap (or,
// at level 2, the level-1 buffers carry null bits): nb[k] gets the row's
// GbParams::part_nulls bits, a null predicate value drops the row, and a
// null-key row is spread over the partitions by its position (ps_digit):
// it aggregates into the null group wherever it lands.
template <int PRED, bool L2, bool F8, bool NUL = false, bool ACCS = true>
__device__ __forceinline__ void ps_keys(const GbParams& p, const DevProgram& prog, const PartOut& in, const PsTile& tl,
                                        int c0, uint64_t (&key)[kPsPer], uint64_t (&pv)[kPsPer],
                                        bool (&sel)[kPsPer], uint32_t (&nb)[kPsPer]) {
    const int lane = threadIdx.x & 63;
    ps_col<L2, F8>(p.key, in.key, tl, c0, key);
    if (!L2 && PRED == 1) ps_col<false, F8>(p.pred_col, nullptr, tl, c0, pv);
    // full level-1 tile and word-aligned bitmaps: a wave's 64 rows' bits are
    // one word per column (ACCS: the aggregated columns' bits too -- the
    // count pass needs only the key's and the predicate's)
    const bool words = NUL && !L2 && p.vwords && tl.lo == tl.base && tl.hi - tl.base == kPsTile;
    // words: every column's validity word of each of the wave's kPsPer row
    // blocks, loaded first and together (uniform loads with no dependence
    // between them), the bits taken afterwards; ~0 (all valid) for a column
    // without a bitmap
    uint64_t wk[kPsPer], wp[kPsPer], wa[kMaxAcc][kPsPer];
    if (NUL && !L2 && words) {
        auto word = [&](const DevCol& c, int64_t rb) -> uint64_t {
            return c.validity ? ((const uint64_t*)c.validity)[(uint64_t)(c.offset + rb) >> 6] : ~0ull;
        };
#pragma unroll
        for (int k = 0; k < kPsPer; ++k) {
            const int64_t rb = tl.base + c0 + k * 64;
            wk[k] = word(p.key, rb);
            wp[k] = PRED == 1 ? word(p.pred_col, rb) : ~0ull;
#pragma unroll
            for (int a = 0; a < kMaxAcc; ++a) wa[a][k] = ACCS && a < p.nacc ? word(p.acc[a].c, rb) : ~0ull;
        }
    }
#pragma unroll
    for (int k = 0; k < kPsPer; ++k) {
        const int64_t r = tl.base + c0 + k * 64 + lane;
        bool s = r >= tl.lo && r < tl.hi;
        nb[k] = 0;
        bool pvalid = true;
        if (NUL && L2) {
            nb[k] = in.nulls && s ? in.nulls[r] : 0u;
        } else if (NUL && words) {
            uint32_t m = ((uint32_t)(~wk[k] >> lane) & 1u) << 6;
#pragma unroll
            for (int a = 0; a < kMaxAcc; ++a) m |= ((uint32_t)(~wa[a][k] >> lane) & 1u) << a;
            nb[k] = m;
            if (PRED == 1) pvalid = ((wp[k] >> lane) & 1u) != 0;
        } else if (NUL && s) {
            uint32_t m = dev_valid(p.key, r) ? 0u : 0x40u;
            if (ACCS)
                for (int a = 0; a < p.nacc; ++a)
                    if (!dev_valid(p.acc[a].c, r)) m |= 1u << a;
            nb[k] = m;
            if (PRED == 1) pvalid = dev_valid(p.pred_col, r);
        }
        if (!L2 && PRED == 1)
            s = s && ((F8 && !NUL) || (NUL ? pvalid : dev_valid(p.pred_col, r))) &&
                simple_pred(prog.simple_isf, prog.simple_op, pv[k], prog.simple_imm);
        if (!L2 && PRED == 2 && s) {
            const RowVal rv = eval_row(prog.code, prog.n, p.cols, r);
            s = rv.valid && (rv.v & 1);
        }
        sel[k] = s;
    }
}

// The partition hash of row r (its input row at level 1, its position in
// the level-1 buffers at level 2): its key's, or for a null key (nb bit 6)
// one of its position, so the null group's rows spread over the partitions.
__device__ __forceinline__ uint64_t ps_hash(uint64_t key, uint32_t nb, int64_t r) {
    return part_hash((nb & 0x40u) ? (uint64_t)r * 0x9E3779B97F4A7C15ull : key);
}

// Count pass: the selected rows of each tile per digit, written digit-major
// per level-1 partition (cnt[mbase + d * ntq + tl]).
template <int PRED, bool L2, bool F8, bool NUL = false>
__global__ __launch_bounds__(kPsThreads) void gbp_count_kernel(GbParams p, DevProgram prog, PsGeom g, PartOut in,
                                                               uint32_t* __restrict__ cnt) {
    __shared__ uint32_t h[1 << kPsDigitBits];
    const int P = 1 << g.dbits;
    const int64_t t = xcd_tile(blockIdx.x, g.ntiles);
    const PsTile tl = ps_tile(g, t);
    if (threadIdx.x < P) h[threadIdx.x] = 0;
    uint64_t key[kPsPer], pv[kPsPer];
    bool sel[kPsPer];
    uint32_t nb[kPsPer];
    const int c0 = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) * (kPsTile / (kPsThreads / 64));
    ps_keys<PRED, L2, F8, NUL, false>(p, prog, in, tl, c0, key, pv, sel, nb);
    if (NUL && !L2 && g.keyrange) {
        // the non-null keys' signed range (every row in the tile, selected
        // or not: a superset is enough for a sentinel outside it)
        int64_t lo = INT64_MAX, hi = INT64_MIN;
#pragma unroll
        for (int k = 0; k < kPsPer; ++k) {
            const int64_t r = tl.base + c0 + k * 64 + (threadIdx.x & 63);
            if (r >= tl.lo && r < tl.hi && !((nb[k] >> 6) & 1u)) {
                lo = min(lo, (int64_t)key[k]);
                hi = max(hi, (int64_t)key[k]);
            }
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            lo = min(lo, (int64_t)__shfl_xor(lo, off, 64));
            hi = max(hi, (int64_t)__shfl_xor(hi, off, 64));
        }
        // one of kKeyRangeSlots pairs by tile (same-address atomics serialise;
        // the host folds the slots)
        if ((threadIdx.x & 63) == 0 && lo <= hi) {
            int64_t* kr = g.keyrange + 2 * (t % kKeyRangeSlots);
            atomicMin((long long*)&kr[0], (long long)lo);
            atomicMax((long long*)&kr[1], (long long)hi);
        }
    }
    __syncthreads();
    const uint32_t mask = (uint32_t)P - 1;
#pragma unroll
    for (int k = 0; k < kPsPer; ++k) {
        const int64_t r = tl.base + c0 + k * 64 + (threadIdx.x & 63);
        // (level 2 of a sentinel run: the null group's rows spread by position
        // again, as the null bit spreads them at level 1)
        const uint64_t hh = NUL ? ps_hash(key[k], nb[k], r)
                                : ps_hash(key[k], (L2 && g.has_sentinel && key[k] == (uint64_t)g.sentinel) ? 0x40u : 0u, r);
        if (sel[k]) atomicAdd(&h[(uint32_t)(hh >> g.sh) & mask], 1u);
    }
    __syncthreads();
    if (threadIdx.x < P) cnt[tl.mbase + (int64_t)threadIdx.x * tl.ntq + tl.tl] = h[threadIdx.x];
}

// Scatter pass: wave w ranks its 1024 rows of the tile row by row (peer
// masks from dbits ballots, per-wave digit counters in LDS, no barriers),
// one block-wide combine turns (wave, digit) counts into tile positions,
// then column by column the values are staged in LDS in digit order and
// written out as one run per digit (the next column's loads are issued
// before this column's write-out).  off: the scanned count matrix.
template <int PRED, bool L2, bool F8, bool NUL = false>
__global__ __launch_bounds__(kPsThreads) void gbp_scatter_kernel(GbParams p, DevProgram prog, PsGeom g, PartOut in,
                                                                 const uint32_t* __restrict__ off, PartOut o) {
    constexpr int NW = kPsThreads / 64;
    constexpr int ND = 1 << kPsDigitBits;
    __shared__ uint64_t sval[kPsTile];
    __shared__ uint8_t sdig[kPsTile];
    __shared__ uint32_t cw[NW][ND];
    __shared__ uint32_t dstart[ND];
    __shared__ uint64_t gbase[ND];
    __shared__ uint64_t wsum[NW];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int P = 1 << g.dbits;
    const int64_t t = xcd_tile(blockIdx.x, g.ntiles);
    const PsTile tl = ps_tile(g, t);
    // this tile's digit offsets (P scattered words): issued first, so their
    // latency hides behind the key loads and the ranking
    const uint64_t my_off = tid < P ? (uint64_t)off[tl.mbase + (int64_t)tid * tl.ntq + tl.tl] : 0ull;
    for (int i = tid; i < NW * ND; i += kPsThreads) cw[i / ND][i % ND] = 0;
    const int c0 = __builtin_amdgcn_readfirstlane(wid) * (kPsTile / NW);
    uint64_t key[kPsPer], pv[kPsPer];
    bool sel[kPsPer];
    uint32_t nb[kPsPer];
    ps_keys<PRED, L2, F8, NUL>(p, prog, in, tl, c0, key, pv, sel, nb);
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1;
    const uint32_t mask = (uint32_t)P - 1;
    uint32_t rk[kPsPer];  // rank | digit << 16 (then the LDS slot); ~0: not selected
#pragma unroll
    for (int k = 0; k < kPsPer; ++k) {
        const int64_t r = tl.base + c0 + k * 64 + lane;
        // (level 2 of a sentinel run: the null group's rows spread by position
        // again, as the null bit spreads them at level 1)
        const uint64_t hh = NUL ? ps_hash(key[k], nb[k], r)
                                : ps_hash(key[k], (L2 && g.has_sentinel && key[k] == (uint64_t)g.sentinel) ? 0x40u : 0u, r);
        const uint32_t d = (uint32_t)(hh >> g.sh) & mask;
        uint64_t peers = __ballot(sel[k]);
#pragma unroll
        for (int b = 0; b < kPsDigitBits; ++b) {
            if (b >= g.dbits) break;
            const uint64_t bb = __ballot((d >> b) & 1);
            peers &= ((d >> b) & 1) ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        const uint32_t old = cw[wid][d];
        rk[k] = sel[k] ? ((old + rank) | (d << 16)) : ~0u;
        // the group's leader bumps the counter (program order within the
        // wave keeps every peer's read before this write)
        if (sel[k] && rank == 0) cw[wid][d] = old + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    uint64_t m;  // selected rows of the tile
    {
        uint32_t ts = 0;
        if (tid < P) {
            for (int w = 0; w < NW; ++w) {
                const uint32_t c = cw[w][tid];
                cw[w][tid] = ts;
                ts += c;
            }
        }
        const uint32_t ds = (uint32_t)block_excl_scan(ts, wsum, m);
        if (tid < P) {
            dstart[tid] = ds;
            gbase[tid] = my_off - ds;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPsPer; ++k) {
        if (rk[k] == ~0u) continue;
        const uint32_t d = rk[k] >> 16;
        const uint32_t pos = dstart[d] + cw[wid][d] + (rk[k] & 0xFFFFu);
        sdig[pos] = (uint8_t)d;
        rk[k] = pos;
    }
    // columns: key 0, aggregated 1 .. nacc, then row ids (if kept), then
    // null bits (NUL, if kept)
    const int rows_col = o.rows ? p.nacc + 1 : -1;
    const int nulls_col = NUL && o.nulls ? p.nacc + 1 + (o.rows ? 1 : 0) : -1;
    const int ncols = 1 + p.nacc + (o.rows ? 1 : 0) + (nulls_col >= 0 ? 1 : 0);
    // column order: the key, then the predicate's column when it is an
    // aggregated one (its registers die first), then the rest
    const int pa = (!L2 && PRED == 1) ? p.pred_acc : -1;
    auto col_at = [&](int i) -> int {
        if (pa < 0 || i == 0 || i > p.nacc) return i;
        if (i == 1) return pa + 1;
        return i - 1 <= pa ? i - 1 : i;
    };
    uint64_t cv[kPsPer];
#pragma unroll
    for (int k = 0; k < kPsPer; ++k) cv[k] = key[k];
    if (NUL && !L2 && g.has_sentinel) {
#pragma unroll
        for (int k = 0; k < kPsPer; ++k) cv[k] = ((nb[k] >> 6) & 1u) ? (uint64_t)g.sentinel : cv[k];
    }
#pragma unroll 1
    for (int ci = 0; ci < ncols; ++ci) {
        // col 0: key; 1..nacc: aggregated columns; nacc + 1: row ids
        const int col = col_at(ci);
#pragma unroll
        for (int k = 0; k < kPsPer; ++k)
            if (rk[k] != ~0u) sval[rk[k]] = cv[k];
        __syncthreads();
        if (ci + 1 < ncols) {
            const int nc = col_at(ci + 1);
            const int a = nc - 1;
            const bool rows = nc == rows_col;
            const bool use_pv = !L2 && PRED == 1 && nc <= p.nacc && a == p.pred_acc;
            if (nc == nulls_col) {
#pragma unroll
                for (int k = 0; k < kPsPer; ++k) cv[k] = nb[k];
            } else if (use_pv) {
#pragma unroll
                for (int k = 0; k < kPsPer; ++k) cv[k] = pv[k];
                if (NUL && !L2) {
#pragma unroll
                    for (int k = 0; k < kPsPer; ++k) cv[k] = ((nb[k] >> a) & 1u) ? 0ull : cv[k];
                }
            } else if (rows && L2) {
                const uint32_t* b = in.rows + tl.base;
                ps_rows(tl, c0, [&](int k, uint32_t i) { cv[k] = (uint64_t)__builtin_nontemporal_load(b + i); });
            } else if (rows) {
                ps_rows(tl, c0, [&](int k, uint32_t i) { cv[k] = (uint64_t)(tl.base + (int64_t)i); });
            } else {
                ps_col<L2, F8>(p.acc[a].c, L2 ? in.acc[a] : nullptr, tl, c0, cv);
                // level 1: a null value is written as 0 (+0.0), which a sum
                // adds as nothing; the other aggregations read its null bit
                if (NUL && !L2) {
#pragma unroll
                    for (int k = 0; k < kPsPer; ++k) cv[k] = ((nb[k] >> a) & 1u) ? 0ull : cv[k];
                }
            }
        }
        if (col <= p.nacc) {
            uint64_t* dst = col == 0 ? o.key : o.acc[col - 1];
            for (int q = tid; q < (int)m; q += kPsThreads) {
                const uint64_t pos = gbase[sdig[q]] + (uint64_t)q;
                if (gb_ok(pos < (uint64_t)o.cap, CK_PART_POS)) dst[pos] = sval[q];
            }
        } else if (col == nulls_col) {
            for (int q = tid; q < (int)m; q += kPsThreads) {
                const uint64_t pos = gbase[sdig[q]] + (uint64_t)q;
                if (gb_ok(pos < (uint64_t)o.cap, CK_PART_POS)) o.nulls[pos] = (uint8_t)sval[q];
            }
        } else {
            for (int q = tid; q < (int)m; q += kPsThreads) {
                const uint64_t pos = gbase[sdig[q]] + (uint64_t)q;
                if (gb_ok(pos < (uint64_t)o.cap, CK_PART_POS)) o.rows[pos] = (uint32_t)sval[q];
            }
        }
        __syncthreads();
    }
}

// Level-1 partition of each level-2 tile (tstart: first tile of each of
// the P1 level-1 partitions, tstart[P1] = tiles).
__global__ void gbp_tpart_kernel(const uint32_t* __restrict__ tstart, int P1, int64_t ntiles,
                                 uint32_t* __restrict__ tpart) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += (int64_t)gridDim.x * blockDim.x) {
        int lo = 0, hi = P1;  // the last q with tstart[q] <= t
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (tstart[mid] <= (uint32_t)t) lo = mid;
            else hi = mid;
        }
        tpart[t] = (uint32_t)lo;
    }
}

// Partition bounds from a scanned count matrix (in place, u32; total =
// selected rows).  Level 1: range[d] = off[d * ntiles].  Level 2: range[q *
// P2 + d] = off[tstart[q] * P2 + d * ntq], or the level-1 partition's start
// when it has no tile.
__global__ void gbp_bounds_kernel(const uint32_t* __restrict__ off, const uint64_t* __restrict__ total, int P,
                                  int64_t ntiles, uint64_t* __restrict__ range) {
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q <= P; q += gridDim.x * blockDim.x)
        range[q] = q < P ? (uint64_t)off[(int64_t)q * ntiles] : *total;
}
__global__ void gbp_bounds2_kernel(const uint32_t* __restrict__ off, const uint64_t* __restrict__ range1,
                                   const uint32_t* __restrict__ tstart, int P1, int b2, uint64_t* __restrict__ range) {
    const int P = P1 << b2;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j <= P; j += gridDim.x * blockDim.x) {
        if (j == P) {
            range[j] = range1[P1];
            continue;
        }
        const int q = j >> b2, d = j & ((1 << b2) - 1);
        const int64_t ntq = (int64_t)(tstart[q + 1] - tstart[q]);
        range[j] = ntq > 0 ? (uint64_t)off[((int64_t)tstart[q] << b2) + (int64_t)d * ntq] : range1[q];
    }
}

// Exact max exponent of a summed column (rerun path only: refits the
// fixed-point window after an overflow / inexact flag).
__global__ __launch_bounds__(256) void gb_maxexp_kernel(GbParams p, int a) {
    const AccSpec& ac = p.acc[a];
    uint32_t mx = 0, inv_mn = 0;  // inv_mn = 0x7FF - (smallest exponent of a nonzero finite value)
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < p.n; r += (int64_t)gridDim.x * blockDim.x) {
        bool valid;
        uint64_t x = acc_value(ac, r, valid);
        if (!valid) continue;
        if (ac.flags & A_FSUMCAST) x = f64_bits((double)(int64_t)x);
        const uint32_t ex = (uint32_t)(x >> 52) & 0x7FF;
        if (ex != 0x7FF && ex > mx) mx = ex;
        if (ex != 0x7FF && (x & 0x7fffffffffffffffull) != 0 && 0x7FF - ex > inv_mn) inv_mn = 0x7FF - ex;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint32_t o = __shfl_xor(mx, off, 64);
        mx = mx > o ? mx : o;
        const uint32_t q = __shfl_xor(inv_mn, off, 64);
        inv_mn = inv_mn > q ? inv_mn : q;
    }
    if ((threadIdx.x & 63) == 0 && mx) atomicMax((unsigned long long*)&p.status[ST_MAXEX + a], (unsigned long long)mx);
    if ((threadIdx.x & 63) == 0 && inv_mn)
        atomicMax((unsigned long long*)&p.status[ST_MINEX + a], (unsigned long long)inv_mn);
}

// ------------------------------------------------------------ wide sums
// Exact fallback for an f64 sum whose values span more binades than one
// fixed-point window holds (e.g. 1e300 in one group, 1e3 in another): a
// second pass adds every selected value, as its 53-bit mantissa, into a
// per-group big integer of 24-bit digits held in int64 words (carry-free
// for 2^39 additions per word) from the column's exact smallest exponent
// upwards.  gb_wide_round_kernel then normalises the digits and rounds once
// (half-even), so the sum is still the correctly rounded exact sum.
constexpr int kWideDigit = 24;

// Digit words per group of a wide sum whose values' biased exponents lie in
// [exmin, exmax] (six words of headroom for the carries of the group's sum).
static inline int wide_nwords(int exmin, int exmax) { return (exmax - exmin) / kWideDigit + 6; }

// Wide f64 sums in the multi-GPU partial-state records: per wide acc (acc
// order) the group's digit words over the ranks' agreed exponent range,
// appended after the record's fields.  `digits`: the table's digit arrays
// (slots x nwords).
struct WideRec {
    int32_t n;
    int32_t acc[kMaxAcc];
    int32_t nwords[kMaxAcc];
    int32_t off[kMaxAcc];  // word offset of acc i's digits from the record start
    int64_t* digits[kMaxAcc];
};

template <int PRED>
__global__ __launch_bounds__(256) void gb_wide_kernel(GbParams p, DevProgram prog, int a, int exmin, int nwords,
                                                      int64_t* __restrict__ wide) {
    const AccSpec& ac = p.acc[a];
    constexpr uint64_t M24 = (1ull << kWideDigit) - 1;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < p.n; r += (int64_t)gridDim.x * blockDim.x) {
        bool valid;
        uint64_t x = acc_value(ac, r, valid);
        if (!valid) continue;
        if (PRED == 1) {
            if (!dev_valid(p.pred_col, r)) continue;
            if (!simple_pred(prog.simple_isf, prog.simple_op, dev_load(p.pred_col, r), prog.simple_imm)) continue;
        } else if (PRED == 2) {
            const RowVal rv = eval_row(prog.code, prog.n, p.cols, r);
            if (!(rv.valid && (rv.v & 1))) continue;
        }
        if (ac.flags & A_FSUMCAST) x = f64_bits((double)(int64_t)x);
        uint32_t ex = (uint32_t)(x >> 52) & 0x7FF;
        uint64_t m = x & 0x000FFFFFFFFFFFFFull;
        if (ex == 0x7FF || (ex == 0 && m == 0)) continue;  // inf / NaN flags come from the main pass
        if (ex == 0) ex = 1;
        else m |= 1ull << 52;
        int64_t gs;
        if (!gb_key_valid(p, r)) {
            gs = p.gcap;
        } else {
            const uint64_t k = gb_key(p, r);
            gs = k == kEmptyKey ? p.gcap + 1 : g_find(p, k);
        }
        if (gs < 0) continue;
        const int pos = (int)ex - exmin;
        const unsigned __int128 v = (unsigned __int128)m << (pos % kWideDigit);
        int64_t* q = wide + gs * nwords + pos / kWideDigit;
        const bool neg = (int64_t)x < 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t dg = (int64_t)((uint64_t)(v >> (kWideDigit * k)) & M24);
            if (dg) atomicAdd((unsigned long long*)&q[k], (unsigned long long)(neg ? -dg : dg));
        }
    }
}

__global__ void gb_wide_round_kernel(GbParams p, int exmin, int nwords, int64_t* __restrict__ wide,
                                     double* __restrict__ out) {
    constexpr int64_t M24 = (1ll << kWideDigit) - 1;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < p.gcap + 2;
         s += (int64_t)gridDim.x * blockDim.x) {
        if (*gfield(p, p.f_len, s) == 0) continue;
        int64_t* d = wide + s * nwords;
        // normalise to digits in [0, 2^24) and a signed carry out of the top
        int64_t c = 0;
        for (int k = 0; k < nwords; ++k) {
            const int64_t t = d[k] + c;
            c = t >> kWideDigit;
            d[k] = t & M24;
        }
        const bool neg = c < 0;
        if (neg) {  // magnitude of a negative number: negate and renormalise
            c = 0;
            for (int k = 0; k < nwords; ++k) {
                const int64_t t = -d[k] + c;
                c = t >> kWideDigit;
                d[k] = t & M24;
            }
        }
        int top = nwords - 1;
        while (top >= 0 && d[top] == 0) --top;
        if (top < 0) {
            out[s] = 0.0;
            continue;
        }
        // the top (up to) 96 bits of the magnitude, plus a sticky bit
        unsigned __int128 acc = 0;
        int k = top;
        for (int taken = 0; k >= 0 && taken < 4; --k, ++taken) acc = (acc << kWideDigit) | (uint64_t)d[k];
        bool sticky = false;
        for (int j = k; j >= 0; --j) sticky |= d[j] != 0;
        const int low = k + 1;  // lowest digit inside acc
        const uint64_t hi64 = (uint64_t)(acc >> 64);
        const int lz = hi64 ? __clzll(hi64) : 64 + __clzll((uint64_t)acc);
        acc <<= lz;  // leading one at bit 127
        // value = acc * 2^(kWideDigit*low + E0 - lz), E0 = exmin - 1075
        const int e2 = 127 + kWideDigit * low + (exmin - 1075) - lz;  // exponent of the leading bit
        int kept = 53;
        if (e2 < -1022) kept = 53 - (-1022 - e2);
        double r;
        if (kept <= 0) {
            // below half the smallest subnormal unless exactly representable rounding up
            const bool above_half = kept == 0 && (((uint64_t)(acc >> 64) << 1) != 0 || (uint64_t)acc != 0 || sticky);
            r = (kept == 0 && above_half) ? __builtin_ldexp(1.0, -1074) : 0.0;
        } else {
            uint64_t mant = (uint64_t)(acc >> (128 - kept));
            const unsigned __int128 rest = acc << kept;  // bits below the kept ones, leading first
            const bool half = (uint64_t)(rest >> 127) & 1;
            const bool below = (rest << 1) != 0 || sticky;
            if (half && (below || (mant & 1))) ++mant;
            r = __builtin_ldexp((double)mant, e2 - kept + 1);
        }
        out[s] = neg ? -r : r;
    }
}

constexpr int kPlanBatch = 16;
constexpr int kPlanThreads = 256;

// Sample i of the plan: clusters of 16 consecutive rows (one 128-B line) spread
// evenly over the column, so 65,536 samples touch 4,096 pages per column
// instead of 65,536 (each a TLB miss: 208 us per plan with single rows).
__device__ __forceinline__ int64_t plan_row(int64_t i, int64_t n, int64_t samples) {
    if (n <= samples) return i;
    const int64_t cstep = n / (samples >> 4);
    return (i >> 4) * cstep + (i & 15);
}

// Planning launch, kPlanBlocks workgroups per task, each sampling its
// 1/kPlanBlocks share of the samples in one batch (one memory round trip per
// thread).  Tasks [0, nacc): the summed columns' largest and smallest
// exponents (atomic max into ST_MAXEX / ST_MINEX; the host derives the
// fixed-point bottoms).  Task nacc: distinct keys of the sample -- each
// workgroup dedups its share in an LDS set and inserts its new keys into a
// global set (`gset`, kPlanSetSlots words, zeroed, holding key ^ kEmptyKey
// so 0 means empty), counting successful inserts in ST_DISTINCT.
// (One workgroup per task took 147 us per plan at 1e9 rows: 16 dependent
// rounds of strided loads.)
constexpr int kPlanBlocks = 16;
// The key task runs kPlanKeyBlocks workgroups, each over the samples of one
// contiguous 1/kPlanKeyBlocks of the rows, and reports the most distinct
// keys any one of them saw (ST_LOCAL): keys that are clustered in row order
// (time-ordered (symbol, day), frames sorted by a key) show few per range
// even when the column holds many.
constexpr int kPlanKeyBlocks = 128;

__global__ __launch_bounds__(kPlanThreads) void gb_plan_kernel(GbParams p, uint64_t* __restrict__ gset,
                                                               int64_t samples, int32_t psimple, int32_t pisf,
                                                               int32_t pop, uint64_t pimm) {
    __shared__ uint64_t set[kPlanSetSlots];
    __shared__ uint32_t red[2][kPlanThreads / 64];
    const bool key_task = (int)blockIdx.x >= p.nacc * kPlanBlocks;
    const int a = key_task ? p.nacc : (int)blockIdx.x / kPlanBlocks;
    const int nb = key_task ? kPlanKeyBlocks : kPlanBlocks;
    const int bi = key_task ? (int)blockIdx.x - p.nacc * kPlanBlocks : (int)blockIdx.x % kPlanBlocks;
    const int64_t per = (samples + nb - 1) / nb;
    const int64_t s0 = (int64_t)bi * per;
    const int64_t s1 = s0 + per < samples ? s0 + per : samples;
    const int64_t n = p.n;
    if (key_task) {
        for (int i = threadIdx.x; i < kPlanSetSlots; i += blockDim.x) set[i] = kEmptyKey;
        __syncthreads();
        const int bits = __builtin_ctz(kPlanSetSlots);
        unsigned long long runs = 0;  // samples whose next row holds the same key
        uint32_t nlocal = 0;          // distinct keys new to this workgroup's set
        // kPlanBatch strided samples per thread are loaded before any is
        // inserted: one memory round trip per batch, not per sample
        for (int64_t i0 = s0 + threadIdx.x; i0 < s1; i0 += (int64_t)blockDim.x * kPlanBatch) {
          uint64_t kb[kPlanBatch];
          bool okb[kPlanBatch];
#pragma unroll
          for (int u = 0; u < kPlanBatch; ++u) {
            const int64_t i = i0 + (int64_t)u * blockDim.x;
            const int64_t r = plan_row(i, n, samples);
            okb[u] = i < s1 && r < n && gb_key_valid(p, r);
            kb[u] = okb[u] ? gb_key(p, r) : 0;
            const bool nx = okb[u] && r + 1 < n && gb_key_valid(p, r + 1);
            runs += (nx && gb_key(p, r + 1) == kb[u]) ? 1u : 0u;
          }
#pragma unroll 1
          for (int u = 0; u < kPlanBatch; ++u) {
            if (!okb[u]) continue;
            const uint64_t k = kb[u];
            if (k == kEmptyKey) continue;
            const uint32_t h = hash_slot(k, bits);
            bool fresh = false;
            for (int q = 0; q < 64; ++q) {
                const uint32_t s = (h + q) & (kPlanSetSlots - 1);
                uint64_t o = lds_load(&set[s]);
                if (o == k) break;
                if (o == kEmptyKey) {
                    o = atomicCAS((unsigned long long*)&set[s], (unsigned long long)kEmptyKey, (unsigned long long)k);
                    if (o == kEmptyKey) {
                        fresh = true;
                        break;
                    }
                    if (o == k) break;
                }
            }
            if (!fresh) continue;
            ++nlocal;
            // new to this workgroup: into the global set, unless the count
            // already reached the saturation mark (then only the HLL pass
            // can size the table, and more inserts would only probe a full set)
            if (__hip_atomic_load(&p.status[ST_DISTINCT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >=
                (uint64_t)kPlanSetSlots / 2)
                continue;
            const unsigned long long w = (unsigned long long)(k ^ kEmptyKey);
            for (int q = 0; q < 64; ++q) {
                const uint32_t s = (h + q) & (kPlanSetSlots - 1);
                const unsigned long long o = atomicCAS((unsigned long long*)&gset[s], 0ull, w);
                if (o == 0ull) {
                    atomicAdd((unsigned long long*)&p.status[ST_DISTINCT], 1ull);
                    break;
                }
                if (o == w) break;
            }
          }
        }
        if (runs) atomicAdd((unsigned long long*)&p.status[ST_RUNS], runs);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) nlocal += __shfl_xor(nlocal, off, 64);
        if ((threadIdx.x & 63) == 0) red[0][threadIdx.x >> 6] = nlocal;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t t = 0;
            for (int w = 0; w < kPlanThreads / 64; ++w) t += red[0][w];
            atomicMax((unsigned long long*)&p.status[ST_LOCAL], (unsigned long long)t);
        }
        return;
    }
    const AccSpec& ac = p.acc[a];
    uint32_t mx = 0, mn = 0x7FF;
    const bool sqlo = ac.dop != DOP_NONE && (ac.dop & DOP_OPMASK) == DOP_SQLO;
    if (ac.flags & (A_FSUM | A_FSUMCAST)) {
        for (int64_t i0 = s0 + threadIdx.x; i0 < s1; i0 += (int64_t)blockDim.x * kPlanBatch) {
            uint64_t xb[kPlanBatch];
            bool okb[kPlanBatch];
#pragma unroll
            for (int u = 0; u < kPlanBatch; ++u) {
                const int64_t i = i0 + (int64_t)u * blockDim.x;
                const int64_t r = plan_row(i, n, samples);
                bool v = false;
                xb[u] = (i < s1 && r < n) ? acc_value(ac, r, v) : 0;
                // a simple predicate (col <cmp> literal): only the rows the
                // sums will take shape their windows
                if (psimple && i < s1 && r < n)
                    v = v && dev_valid(p.pred_col, r) && simple_pred(pisf, pop, dev_load(p.pred_col, r), pimm);
                okb[u] = i < s1 && r < n && v;
            }
#pragma unroll
            for (int u = 0; u < kPlanBatch; ++u) {
                if (!okb[u]) continue;
                uint64_t x = xb[u];
                if (ac.flags & A_FSUMCAST) x = f64_bits((double)(int64_t)x);
                const uint32_t ex = (uint32_t)(x >> 52) & 0x7FF;
                if (ex != 0x7FF && ex > mx) mx = ex;
                // smallest exponent of a nonzero finite value (subnormals: 0)
                uint32_t el = ex;
                if (sqlo && ex != 0) {
                    // the error term l = fma(x, x, -x * x) of a fused
                    // variance: its set bits end at the lowest bit of x * x,
                    // wherever its leading bit falls (its magnitude spreads
                    // over ~20 binades below ulp(x * x) / 2), so the 2-limb
                    // test takes the exponent its lowest set bit implies
                    const uint64_t m = (x & 0x000FFFFFFFFFFFFFull) | (1ull << 52);
                    el = ex + (uint32_t)__builtin_ctzll(m);
                }
                if ((x & 0x7fffffffffffffffull) != 0 && ex != 0x7FF && el < mn) mn = el;
            }
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint32_t o = __shfl_xor(mx, off, 64);
        mx = mx > o ? mx : o;
        const uint32_t q = __shfl_xor(mn, off, 64);
        mn = mn < q ? mn : q;
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = mx;
        red[1][threadIdx.x >> 6] = mn;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kPlanThreads / 64; ++w) {
            mx = red[0][w] > mx ? red[0][w] : mx;
            mn = red[1][w] < mn ? red[1][w] : mn;
        }
        if (mx) atomicMax((unsigned long long*)&p.status[ST_MAXEX + a], (unsigned long long)mx);
        if (mn != 0x7FF) atomicMax((unsigned long long*)&p.status[ST_MINEX + a], (unsigned long long)(0x7FF - mn));
    }
}

// Fixed-point bottom of a summed column from its largest sampled exponent
// (0: none sampled): kHeadroomBinades above it, so a value fits iff
// ex <= bottom + 1075 + (window - 53).
static int32_t plan_bottom(uint64_t maxex) {
    int e = maxex == 0 ? 2046 : (int)maxex + kHeadroomBinades;
    if (e > 2046) e = 2046;
    return e - 1075 - (kSumWindowBits - 53);
}

__global__ void gb_init_table_kernel(uint64_t* gtab, int64_t words_per_field, int nfields, uint64_t min_init_mask) {
    for (int f = 0; f < nfields; ++f) {
        const uint64_t v = f == 0 ? kEmptyKey : (((min_init_mask >> f) & 1ull) ? ~0ull : 0ull);
        uint64_t* q = gtab + (int64_t)f * words_per_field;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words_per_field;
             i += (int64_t)gridDim.x * blockDim.x)
            q[i] = v;
    }
}

// 192-bit two's complement * 2^bottom -> correctly rounded double.

// ---- fused variance: exact second moment from exact sums
// With S1 = sum x = W1 * 2^b1, and x * x = h + l exactly (DOP_SQHI / SQLO,
// |x| in [2^-484, 2^511)) summed exactly as W2 * 2^b2 and W3 * 2^b3:
//   n * sum((x - mean)^2) = n * (W2 * 2^b2 + W3 * 2^b3) - W1^2 * 2^(2 b1),
// an integer times 2^e, e = min(b2, b3, 2 b1), formed exactly in a 1024-bit
// two's complement accumulator and rounded once to f64.
constexpr int kVarWords = 16;

// |W| of a 192-bit two's complement word triple; returns the sign.
__device__ __forceinline__ bool abs192(uint64_t& w0, uint64_t& w1, uint64_t& w2) {
    const bool neg = (int64_t)w2 < 0;
    if (neg) {
        w0 = ~w0; w1 = ~w1; w2 = ~w2;
        w0 += 1;
        const uint64_t c0 = w0 == 0;
        w1 += c0;
        w2 += (c0 && w1 == 0) ? 1 : 0;
    }
    return neg;
}

// acc += (negate ? -1 : 1) * (m[0..k) << sh) over the full width; false when
// the shifted value would not fit (the caller falls back).
__device__ bool big_add_shifted(uint64_t (&acc)[kVarWords], const uint64_t* m, int k, int sh, bool negate) {
    int top = k - 1;
    while (top >= 0 && m[top] == 0) --top;
    if (top < 0) return true;
    const int bitlen = top * 64 + 64 - __clzll(m[top]);
    if (sh < 0 || bitlen + sh > kVarWords * 64 - 2) return false;
    const int ws = sh >> 6, bs = sh & 63;
    uint64_t carry = negate ? 1 : 0;
    for (int i = 0; i < kVarWords; ++i) {
        const int j = i - ws;
        uint64_t t = 0;
        if (j >= 0 && j <= k) {
            const uint64_t lo = j < k ? m[j] : 0ull;
            const uint64_t hi = (j >= 1 && j - 1 < k) ? m[j - 1] : 0ull;
            t = bs ? (lo << bs) | (hi >> (64 - bs)) : lo;
        }
        if (negate) t = ~t;
        const uint64_t s1 = acc[i] + t;
        const uint64_t c1 = s1 < t ? 1ull : 0ull;
        const uint64_t s2 = s1 + carry;
        const uint64_t c2 = s2 < s1 ? 1ull : 0ull;
        acc[i] = s2;
        carry = c1 | c2;
    }
    return true;
}

// acc * 2^e2 as f64, rounded once (half-even); acc >= 0 (a negative value
// cannot occur for an exact sum of squares, and is clamped to 0).
__device__ double big_to_double(const uint64_t (&acc)[kVarWords], int e2) {
    if ((int64_t)acc[kVarWords - 1] < 0) return 0.0;
    int t = kVarWords - 1;
    while (t >= 0 && acc[t] == 0) --t;
    if (t < 0) return 0.0;
    const int p = t * 64 + 63 - __clzll(acc[t]);  // leading bit
    const int q = p - 63;                           // bit offset of the 64-bit window
    uint64_t x;
    bool sticky = false;
    if (q <= 0) {
        x = acc[0] << (-q);
    } else {
        const int w = q >> 6, b = q & 63;
        x = b ? (acc[w] >> b) | (acc[w + 1] << (64 - b)) : acc[w];
        sticky = b ? (acc[w] & ((1ull << b) - 1)) != 0 : false;
        for (int i = 0; i < w && !sticky; ++i) sticky = acc[i] != 0;
    }
    uint64_t keep = x >> 11;
    const uint64_t rem = x & 0x7FF;
    if (rem > 0x400 || (rem == 0x400 && (sticky || (keep & 1)))) ++keep;
    int ex = p - 52 + e2;
    if (keep == (1ull << 53)) {
        keep >>= 1;
        ++ex;
    }
    return ldexp((double)keep, ex);
}

// The variance of one group from its exact states; false: out of range.
__device__ bool var_exact(uint64_t a0, uint64_t a1, uint64_t a2, int b1, uint64_t h0, uint64_t h1, uint64_t h2,
                          int b2, uint64_t l0, uint64_t l1, uint64_t l2, int b3, uint64_t n, double& num) {
    (void)abs192(a0, a1, a2);  // W1^2 only
    const bool hneg = abs192(h0, h1, h2), lneg = abs192(l0, l1, l2);
    const uint64_t W1[3] = {a0, a1, a2};
    uint64_t sq[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 3; ++i) {
        unsigned __int128 c = 0;
        for (int j = 0; j < 3; ++j) {
            c += (unsigned __int128)W1[i] * W1[j] + sq[i + j];
            sq[i + j] = (uint64_t)c;
            c >>= 64;
        }
        sq[i + 3] = (uint64_t)c;
    }
    auto times_n = [&](uint64_t w0, uint64_t w1, uint64_t w2, uint64_t (&o)[4]) {
        unsigned __int128 c = (unsigned __int128)w0 * n;
        o[0] = (uint64_t)c;
        c = (c >> 64) + (unsigned __int128)w1 * n;
        o[1] = (uint64_t)c;
        c = (c >> 64) + (unsigned __int128)w2 * n;
        o[2] = (uint64_t)c;
        o[3] = (uint64_t)(c >> 64);
    };
    uint64_t nh[4], nl[4];
    times_n(h0, h1, h2, nh);
    times_n(l0, l1, l2, nl);
    const int e = min(min(b2, b3), 2 * b1);
    uint64_t acc[kVarWords];
    for (int i = 0; i < kVarWords; ++i) acc[i] = 0;
    if (!big_add_shifted(acc, nh, 4, b2 - e, hneg)) return false;
    if (!big_add_shifted(acc, nl, 4, b3 - e, lneg)) return false;
    if (!big_add_shifted(acc, sq, 6, 2 * b1 - e, true)) return false;
    num = big_to_double(acc, e);
    return true;
}

struct FinParams {
    OutSpec out[PLGPU_MAX_COLS * 2];
    int32_t nout;
    int32_t _pad;
    int64_t* out_keys;
    uint32_t* out_key_valid;
    uint64_t* out_first;  // optional
    int64_t cap;          // allocated output rows (guards against a miscount)
    const double* wide[kMaxAcc];  // per acc: rounded wide sums per slot, or null
    // validity as one byte per output row (row 0: the key, row 1 + o:
    // output o; stride cap), packed into the bitmaps afterwards
    // (gb_pack_valid_kernel): no per-group atomics on shared words
    uint8_t* vbytes;
};

// Table slot s (len selected rows) -> output row g: the key, its validity
// byte, the first row, and every output's value and validity byte.
__device__ void fin_slot(const GbParams& p, const FinParams& fp, const uint64_t* tab, int64_t stride, int64_t s,
                         int special, int64_t g, uint64_t len) {
    if (g >= fp.cap) return;
    auto F = [&](int f) { return tab + (int64_t)f * stride + s; };
    const bool null_key = special == 1;
    fp.out_keys[g] = null_key ? 0 : (int64_t)(special == 2 ? kEmptyKey : *F(0));
    fp.vbytes[g] = null_key ? 0 : 1;
    if (fp.out_first) fp.out_first[g] = *F(p.f_first);
    for (int o = 0; o < fp.nout; ++o) {
        const OutSpec& os = fp.out[o];
        const AccSpec& ac = p.acc[os.acc];
        bool valid = true;
        const uint64_t cnt = ac.f_cnt >= 0 ? *F(ac.f_cnt) : len;
        const uint64_t flags = ac.f_flags >= 0 ? *F(ac.f_flags) : 0;
        switch (os.kind) {
        case PLGPU_AGG_LEN: ((uint32_t*)os.values)[g] = (uint32_t)len; break;
        case PLGPU_AGG_COUNT: ((uint32_t*)os.values)[g] = (uint32_t)cnt; break;
        case PLGPU_AGG_SUM:
        case PLGPU_AGG_MEAN: {
            if (os.kind == PLGPU_AGG_SUM && !os.in_isf) {
                // wrapping integer sum, stored at the output width
                dev_store(os.values, os.out_dtype, g, *F(ac.f_isum));
                break;
            }
            double sum;
            if (flags & FL_NAN || ((flags & FL_PINF) && (flags & FL_NINF))) sum = __builtin_nan("");
            else if (flags & FL_PINF) sum = __builtin_inf();
            else if (flags & FL_NINF) sum = -__builtin_inf();
            else if (fp.wide[os.acc]) sum = fp.wide[os.acc][s];
            else sum = fx_to_double(*F(ac.f_sum), *F(ac.f_sum + 1),
                                    *F(ac.f_sum + 2), p.bottoms[os.acc]);
            if (os.kind == PLGPU_AGG_MEAN) {
                if (cnt == 0) { valid = false; sum = 0.0; }
                else sum = sum / (double)cnt;
            }
            dev_store(os.values, os.out_dtype, g, f64_bits(sum));  // Float32: rounded once more
            break;
        }
        case PLGPU_AGG_VAR:
        case PLGPU_AGG_STD: {
            // moment.rs:126 VarState::finalize: null when count <= ddof;
            // an inf / NaN value makes it NaN
            double v = 0.0;
            if (cnt <= (uint64_t)os.ddof) {
                valid = false;
            } else if (flags) {
                v = __builtin_nan("");
            } else {
                const AccSpec& ah = p.acc[os.acc_hi];
                const AccSpec& al = p.acc[os.acc_lo];
                const uint64_t hf = *F(ah.f_flags) | *F(al.f_flags);
                double num = 0.0;
                const bool ok = hf == 0 &&
                                var_exact(*F(ac.f_sum), *F(ac.f_sum + 1),
                                          *F(ac.f_sum + 2), p.bottoms[os.acc],
                                          *F(ah.f_sum), *F(ah.f_sum + 1),
                                          *F(ah.f_sum + 2), p.bottoms[os.acc_hi],
                                          *F(al.f_sum), *F(al.f_sum + 1),
                                          *F(al.f_sum + 2), p.bottoms[os.acc_lo], cnt, num);
                if (!ok) {
                    // x * x overflowed, or the exact state left the accumulator
                    atomicOr((unsigned long long*)&p.status[ST_VAR_OUT], 1ull);
                } else {
                    v = (num / (double)cnt) / (double)(cnt - (uint64_t)os.ddof);
                    if (os.kind == PLGPU_AGG_STD) v = __builtin_sqrt(v);
                }
            }
            ((double*)os.values)[g] = v;
            break;
        }
        case PLGPU_AGG_MIN:
        case PLGPU_AGG_MAX: {
            const uint64_t o = *F(os.kind == PLGPU_AGG_MIN ? ac.f_min : ac.f_max);
            const bool none = os.kind == PLGPU_AGG_MIN ? (o == ~0ull) : (o == 0ull);
            if (os.in_isf) {
                double v;
                if (cnt == 0) { valid = false; v = 0.0; }
                else if (none) v = __builtin_nan("");  // every valid value was NaN
                else v = as_f64(unord_f64(o));
                dev_store(os.values, os.out_dtype, g, f64_bits(v));
            } else {
                // (the all-ones / all-zeros "none" encodings are real
                // values here: an integer group with cnt > 0 has one)
                const uint64_t v = cnt == 0 ? 0ull : (os.in_uns ? o : (o ^ 0x8000000000000000ull));
                if (cnt == 0) valid = false;
                dev_store(os.values, os.out_dtype, g, v);
            }
            break;
        }
        case PLGPU_AGG_FIRST:
        case PLGPU_AGG_LAST: {
            // the value (null included) of the group's first / last
            // selected row (polars-expr/src/reduce/first_last.rs)
            const int64_t row = (int64_t)*F(os.kind == PLGPU_AGG_FIRST ? p.f_first : p.f_last);
            if (!gb_ok(row >= 0 && row < p.n, CK_FIRST_ROW)) {
                valid = false;
                break;
            }
            const uint64_t v0 = acc_value(ac, row, valid);
            const uint64_t v = valid ? v0 : 0ull;
            dev_store(os.values, os.out_dtype, g, v);
            break;
        }
        default: break;
        }
        if (os.validity) fp.vbytes[(int64_t)(1 + o) * fp.cap + g] = valid ? 1 : 0;
    }
}

__global__ __launch_bounds__(256) void gb_finalize_kernel(GbParams p, FinParams fp) {
    const int64_t total = p.gcap + 2;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    // output positions: each workgroup owns one contiguous range of slots,
    // counts its live groups, and takes its output range with ONE counter
    // add (one add per wave on the single status word serialised: ~6 ms at
    // 2^25 slots); then each 256-slot chunk's live groups are ranked by
    // wave ballots and a block prefix
    __shared__ uint64_t wcnt[4];
    __shared__ unsigned long long gbase;
    const int64_t per = (((total + gridDim.x - 1) / gridDim.x) + 255) & ~int64_t(255);
    const int64_t lo = std::min<int64_t>(total, (int64_t)blockIdx.x * per), hi = std::min<int64_t>(total, lo + per);
    uint64_t mine = 0;
    for (int64_t s = lo + threadIdx.x; s < hi; s += blockDim.x) mine += *gfield(p, p.f_len, s) != 0 ? 1 : 0;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) mine += __shfl_xor(mine, off, 64);
    if (lane == 0) wcnt[wid] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t t = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
        gbase = t ? atomicAdd((unsigned long long*)&p.status[ST_GROUPS_OUT], (unsigned long long)t) : 0ull;
    }
    __syncthreads();
    uint64_t run = gbase;
    for (int64_t s0 = lo; s0 < hi; s0 += blockDim.x) {
        const int64_t s = s0 + threadIdx.x;
        const uint64_t len = s < hi ? *gfield(p, p.f_len, s) : 0ull;
        const uint64_t live = __ballot(len != 0);
        __syncthreads();  // the previous chunk's readers of wcnt are done
        if (lane == 0) wcnt[wid] = (uint64_t)__popcll(live);
        __syncthreads();
        uint64_t before = 0, chunk = 0;
        for (int w = 0; w < 4; ++w) {
            before += w < wid ? wcnt[w] : 0;
            chunk += wcnt[w];
        }
        const uint64_t base = run + before;
        run += chunk;
        if (len == 0) continue;
        const int64_t g = (int64_t)base + __popcll(live & lt);
        fin_slot(p, fp, p.gtab, p.gcap + 2, s, s == p.gcap ? 1 : (s == p.gcap + 1 ? 2 : 0), g, len);
    }
}

// The groups of a compact-region run (GbParams::region_cnt): block q
// finalizes region q's dense prefix of the region table into outputs
// [off[q], off[q + 1]) (off: the exclusive scan of the region counts) and
// adds its count to ST_GROUPS_OUT, so the overflow table's finalize
// (gb_finalize_kernel, launched next) places its groups after them.
__global__ __launch_bounds__(256) void gb_finalize_regions_kernel(GbParams p, FinParams fp,
                                                                  const uint64_t* __restrict__ off, int lbits) {
    const int q = blockIdx.x;
    const uint64_t b = off[q], c = off[q + 1] - b;
    const int64_t t0 = (int64_t)q << lbits;  // region q: the partition's LDS table size
    for (uint64_t i = threadIdx.x; i < c; i += blockDim.x) {
        const int64_t s = t0 + (int64_t)i;
        fin_slot(p, fp, p.rtab, p.rcap, s, 0, (int64_t)(b + i), p.rtab[(int64_t)p.f_len * p.rcap + s]);
    }
    if (threadIdx.x == 0 && c) atomicAdd((unsigned long long*)&p.status[ST_GROUPS_OUT], (unsigned long long)c);
}

// Validity bytes (FinParams::vbytes) -> Arrow bitmaps: one 32-bit word per
// thread per column.
struct PackValid {
    uint32_t* dst[PLGPU_MAX_COLS * 2 + 1];  // null: no bitmap for that row of bytes
    int32_t n;
};
__global__ void gb_pack_valid_kernel(const uint8_t* __restrict__ vb, int64_t cap, PackValid pv) {
    const int64_t words = ((cap + 63) / 64) * 2;  // the bitmap's whole 64-bit words (bits past cap: 0)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words * pv.n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i / words);
        const int64_t w = i - (int64_t)c * words;
        if (pv.dst[c] == nullptr) continue;
        const uint8_t* b = vb + (int64_t)c * cap + w * 32;
        const int m = (int)std::max<int64_t>(0, std::min<int64_t>(32, cap - w * 32));
        uint32_t bits = 0;
        for (int j = 0; j < m; ++j) bits |= (uint32_t)(b[j] != 0) << j;
        pv.dst[c][w] = bits;
    }
}

__global__ void widen_u32_kernel(const uint32_t* __restrict__ a, int64_t* __restrict__ b, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        b[i] = (int64_t)a[i];
}

// Gather rows of fixed-width buffers by a permutation (maintain_order).
template <typename T>
__global__ void gather_kernel(const T* __restrict__ src, const int64_t* __restrict__ perm, T* __restrict__ dst,
                              int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (gb_ok(perm[i] >= 0 && perm[i] < n, CK_PERM)) dst[i] = src[perm[i]];
}
__global__ void narrow_i64_kernel(const int64_t* __restrict__ a, void* __restrict__ b, int32_t dt, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dev_store(b, dt, i, (uint64_t)a[i]);
}
// One destination bitmap word per thread (bits past n: 0), no atomics.
__global__ void gather_bits_kernel(const uint32_t* __restrict__ src, const int64_t* __restrict__ perm,
                                   uint32_t* __restrict__ dst, int64_t n) {
    const int64_t words = (n + 31) / 32;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words;
         w += (int64_t)gridDim.x * blockDim.x) {
        uint32_t bits = 0;
        const int m = (int)std::min<int64_t>(32, n - w * 32);
        for (int k = 0; k < m; ++k) {
            const int64_t j = perm[w * 32 + k];
            bits |= ((src[j >> 5] >> (j & 31)) & 1u) << k;
        }
        dst[w] = bits;
    }
}

// --------------------------------------------- partial states (multi-GPU)
// Record of one group: [kind (0 key, 1 null, 2 INT64_MIN), key, fields
// 1..nfields-1 in table representation]; record_words = nfields + 1.
__device__ __forceinline__ int dest_rank(uint64_t kind, uint64_t key, int world) {
    if (kind != 0 || world <= 1) return 0;
    const uint64_t h = (key ^ (key >> 31)) * 0xC2B2AE3D27D4EB4Full;
    return (int)((h >> 33) % (uint64_t)world);
}

__device__ __forceinline__ bool slot_record(const GbParams& p, int64_t s, uint64_t& kind, uint64_t& key) {
    if (*gfield(p, p.f_len, s) == 0) return false;
    kind = s == p.gcap ? 1 : (s == p.gcap + 1 ? 2 : 0);
    key = kind == 0 ? *gfield(p, 0, s) : (kind == 2 ? kEmptyKey : 0);
    return true;
}

__global__ void gb_export_count_kernel(GbParams p, int world, uint64_t* counts) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < p.gcap + 2;
         s += (int64_t)gridDim.x * blockDim.x) {
        uint64_t kind, key;
        if (!slot_record(p, s, kind, key)) continue;
        atomicAdd((unsigned long long*)&counts[dest_rank(kind, key, world)], 1ull);
    }
}

__global__ void gb_export_kernel(GbParams p, int world, uint64_t* cursor, uint64_t* out, WideRec wr, int rw) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < p.gcap + 2;
         s += (int64_t)gridDim.x * blockDim.x) {
        uint64_t kind, key;
        if (!slot_record(p, s, kind, key)) continue;
        const uint64_t idx = atomicAdd((unsigned long long*)&cursor[dest_rank(kind, key, world)], 1ull);
        uint64_t* r = out + idx * rw;
        r[0] = kind;
        r[1] = key;
        for (int f = 1; f < p.nfields; ++f) r[1 + f] = *gfield(p, f, s);
        for (int i = 0; i < wr.n; ++i) {
            const int64_t* d = wr.digits[i] + s * wr.nwords[i];
            for (int k = 0; k < wr.nwords[i]; ++k) r[wr.off[i] + k] = (uint64_t)d[k];
        }
    }
}

// (w2:w1:w0) <<= d as a two's-complement 192-bit integer, 0 <= d; false
// (value unchanged) when the result would not fit with `guard` bits to
// spare (so that 2^guard such values still add without wrapping).
__device__ __forceinline__ bool shl192(uint64_t& w0, uint64_t& w1, uint64_t& w2, int d, int guard = 0) {
    if (d == 0 && guard == 0) return true;
    const uint64_t sign = (uint64_t)((int64_t)w2 >> 63);
    const int top = d + guard;
    if (top >= 191) return (w0 | w1 | w2) == 0;
    // the top d + guard + 1 bits must all equal the sign
    const uint64_t x[3] = {w0, w1, w2};
    for (int b = 191 - top; b < 192; b += 64) {
        const int lo = b, hi = b + 64 < 192 ? b + 64 : 192;  // bits [lo, hi) of this chunk
        const int wi = lo >> 6, sh = lo & 63;
        uint64_t chunk = x[wi] >> sh;
        if (sh && wi + 1 < 3) chunk |= x[wi + 1] << (64 - sh);
        const int nb = hi - lo;
        const uint64_t m = nb == 64 ? ~0ull : ((1ull << nb) - 1);
        if ((chunk & m) != (sign & m)) return false;
    }
    if (d == 0) return true;
    const int q = d >> 6, r = d & 63;
    uint64_t o[3];
    for (int i = 0; i < 3; ++i) {
        const int j = i - q;
        uint64_t v = j >= 0 ? (r ? x[j] << r : x[j]) : 0ull;
        if (r && j - 1 >= 0) v |= x[j - 1] >> (64 - r);
        o[i] = v;
    }
    w0 = o[0];
    w1 = o[1];
    w2 = o[2];
    return true;
}

// Fold records (from any rank) into the global table.  With nsrc > 0 the
// records come from nsrc sources in order (source j: records
// [src_start[j], src_start[j + 1])), each aggregated with its own
// fixed-point windows; an f64 sum state of acc a is shifted left by
// src_shift[j * kMaxAcc + a] bits onto the table's window (exact).
__global__ void gb_merge_kernel(GbParams p, const uint64_t* __restrict__ rec, int64_t nrec, int nsrc,
                                const int64_t* __restrict__ src_start, const int32_t* __restrict__ src_shift,
                                WideRec wr, int rw) {
    // the 192-bit states of wide accs are not merged (their digits are)
    uint64_t skip = 0;
    for (int i = 0; i < wr.n; ++i) skip |= 1ull << p.acc[wr.acc[i]].f_sum;
    uint32_t special = 0;
    bool ovf = false;
    // up to nsrc states fold into one cell: each must leave ceil(log2 nsrc)
    // sign bits to spare, so their sum cannot wrap the 192-bit cell
    const int guard = nsrc > 1 ? 32 - __clz((unsigned)(nsrc - 1)) : 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nrec; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t* r = rec + i * rw;
        const uint64_t kind = r[0];
        int src = 0;
        while (src + 1 < nsrc && i >= src_start[src + 1]) ++src;
        int64_t gs;
        if (kind == 1) {
            gs = p.gcap;
            special |= 1u;
        } else if (kind == 2) {
            gs = p.gcap + 1;
            special |= 2u;
        } else {
            gs = g_find(p, r[1]);
        }
        if (gs < 0) {
            atomicAdd((unsigned long long*)&p.status[ST_TABLE_FULL], 1ull);
            continue;
        }
        if (!gb_ok(gs < p.gcap + 2, CK_MERGE_SLOT)) continue;
        for (int f = 1; f < p.nfields; ++f) {
            const uint64_t v = r[1 + f];
            unsigned long long* q = (unsigned long long*)gfield(p, f, gs);
            switch (p.fop[f]) {
            case FOP_ADD: if (v) atomicAdd(q, (unsigned long long)v); break;
            case FOP_MIN: if (v != ~0ull) atomicMin(q, (unsigned long long)v); break;
            case FOP_MAX: if (v) atomicMax(q, (unsigned long long)v); break;
            case FOP_OR: if (v) atomicOr(q, (unsigned long long)v); break;
            case FOP_ADD192: {
                if ((skip >> f) & 1ull) break;
                uint64_t w0 = v, w1 = r[2 + f], w2 = r[3 + f];
                if (nsrc > 0) {
                    int d = 0;
                    for (int a = 0; a < p.nacc; ++a)
                        if (p.acc[a].f_sum == f) d = src_shift[src * kMaxAcc + a];
                    if (!shl192(w0, w1, w2, d, guard)) {
                        ovf = true;
                        break;
                    }
                }
                g_add192(gfield(p, f, gs), gfield(p, f + 1, gs), gfield(p, f + 2, gs), w0, w1, w2);
                break;
            }
            default: break;
            }
        }
        for (int w = 0; w < wr.n; ++w) {
            int64_t* d = wr.digits[w] + gs * wr.nwords[w];
            for (int k = 0; k < wr.nwords[w]; ++k) {
                const uint64_t v = r[wr.off[w] + k];
                if (v) atomicAdd((unsigned long long*)&d[k], (unsigned long long)v);
            }
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) special |= __shfl_xor(special, off, 64);
    if ((threadIdx.x & 63) == 0 && special) atomicOr((unsigned long long*)&p.status[ST_SPECIAL], (unsigned long long)special);
    if (__any(ovf) && (threadIdx.x & 63) == 0) atomicOr((unsigned long long*)&p.status[ST_SHIFT_OVF], 1ull);
}

// ------------------------------------------------------------- host
static DevCol to_dev(const plgpu_column& c) { return dev_col(c); }


// One aggregation input (plan_groupby): a column, or a derived value x op y
// computed in registers (DOP_*, both operands Float64).
struct InSpec {
    plgpu_column col;   // the column (derived: the first operand)
    plgpu_column col2;  // derived: the second operand column (unless DOP_LIT)
    int32_t dtype;      // dtype of the input (derived: Float64)
    int32_t dop;        // DOP_NONE: the column itself
    uint64_t imm;       // DOP_LIT: the literal's f64 bits
};

static std::vector<InSpec> column_inputs(const plgpu_column* cols, int32_t ncols) {
    std::vector<InSpec> v((size_t)std::max(ncols, 0));
    for (int i = 0; i < ncols; ++i) {
        std::memset(&v[i], 0, sizeof v[i]);
        v[i].col = cols[i];
        v[i].dtype = cols[i].dtype;
    }
    return v;
}

// Aggregations `aggs` (agg.col indexes `ins`) -> accumulators, table fields
// and output specs.  `cols` are the columns the predicate program reads.
static int plan_groupby(const plgpu_column* key, const plgpu_column* cols, int32_t ncols, const InSpec* ins,
                        int32_t nins, const plgpu_agg* aggs, int32_t naggs, bool maintain_order, const DevProgram& dp,
                        Plan* pl, bool force_counts = false) {
    GbParams& p = pl->p;
    std::memset(&p, 0, sizeof p);
    p.key = to_dev(*key);
    for (int i = 0; i < ncols; ++i) p.cols[i] = to_dev(cols[i]);
    p.n = key->length;
    int nf = 1;  // field 0: keys
    p.f_len = nf++;
    bool any_first = false, any_last = false;
    for (int i = 0; i < naggs; ++i) {
        any_first |= (aggs[i].kind & 0xFF) == PLGPU_AGG_FIRST;
        any_last |= (aggs[i].kind & 0xFF) == PLGPU_AGG_LAST;
    }
    p.f_first = (maintain_order || any_first) ? nf++ : -1;
    if (p.f_first >= 0) p.min_init_mask |= 1ull << p.f_first;
    p.f_last = any_last ? nf++ : -1;
    std::vector<int> acc_of_col((size_t)std::max(nins, 1), -1);
    p.nacc = 0;
    // the acc of input c (created on first use); -1 with the error set
    auto acc_for = [&](int c) -> int {
        if (c < 0 || c >= nins) return fail(PLGPU_ERR_INVALID, "aggregation column index out of range"), -1;
        const InSpec& in = ins[c];
        const int32_t dt = in.dtype;
        if (!dtype_is_int(dt) && !dtype_is_float(dt))
            return fail(PLGPU_ERR_INVALID, "aggregation not supported for this dtype"), -1;
        if (acc_of_col[c] < 0) {
            if (p.nacc == kMaxAcc) return fail(PLGPU_ERR_INVALID, "too many aggregated columns (max 6)"), -1;
            acc_of_col[c] = p.nacc;
            pl->acc_in[p.nacc] = c;
            AccSpec& ac = p.acc[p.nacc++];
            std::memset(&ac, 0xff, sizeof ac);
            ac.c = to_dev(in.col);
            ac.flags = 0;
            ac.isf = dtype_is_float(dt);  // Float32 in register form (f64 bits): exact sums, TotalOrd min / max
            ac.uns = dt == PLGPU_U64;
            ac.dop = in.dop;
            std::memset(&ac.c2, 0, sizeof ac.c2);
            if (in.dop != DOP_NONE && !(in.dop & DOP_LIT)) ac.c2 = to_dev(in.col2);
            ac.dimm = in.imm;
        }
        return acc_of_col[c];
    };
    std::vector<int> var_hi((size_t)std::max(naggs, 1), -1), var_lo((size_t)std::max(naggs, 1), -1);
    for (int i = 0; i < naggs; ++i) {
        const int c = aggs[i].col;
        const int a = acc_for(c);
        if (a < 0) return PLGPU_ERR_INVALID;
        const InSpec& in = ins[c];
        const int32_t dt = in.dtype;
        AccSpec& ac = p.acc[a];
        const bool isf = dtype_is_float(dt);
        // partial / merge mode keeps the record layout schema-only (the same on
        // every rank whatever its validity bitmaps): counts always present
        const bool nullable = in.col.validity != nullptr || (ac.c2.validity != nullptr) || force_counts;
        switch (aggs[i].kind & 0xFF) {
        case PLGPU_AGG_VAR:
        case PLGPU_AGG_STD: {
            // exact sum and count of x; exact sums of x * x's two parts
            // (derived inputs hi, hi + 1, plgpu_group_by_agg_ex)
            const int hi = (aggs[i].kind >> 16) & 0xFFF;
            if (!isf || hi == 0) return fail(PLGPU_ERR_INVALID, "var / std in one pass take a Float64 column");
            ac.flags |= A_FSUM | A_FLAGS;
            if (nullable) ac.flags |= A_CNT;
            const int ah = acc_for(hi), al = ah < 0 ? -1 : acc_for(hi + 1);
            if (ah < 0 || al < 0) return PLGPU_ERR_INVALID;
            p.acc[ah].flags |= A_FSUM | A_FLAGS;
            p.acc[al].flags |= A_FSUM | A_FLAGS;
            var_hi[i] = ah;
            var_lo[i] = al;
            break;
        }
        case PLGPU_AGG_SUM: ac.flags |= isf ? (A_FSUM | A_FLAGS) : A_ISUM; break;
        case PLGPU_AGG_MEAN:
            ac.flags |= isf ? (A_FSUM | A_FLAGS) : A_FSUMCAST;
            if (nullable) ac.flags |= A_CNT;
            break;
        case PLGPU_AGG_MIN: ac.flags |= A_MIN | (isf ? A_FLAGS : 0) | A_CNT; break;
        case PLGPU_AGG_MAX: ac.flags |= A_MAX | (isf ? A_FLAGS : 0) | A_CNT; break;
        case PLGPU_AGG_COUNT: if (nullable) ac.flags |= A_CNT; break;
        case PLGPU_AGG_LEN:
        case PLGPU_AGG_FIRST:
        case PLGPU_AGG_LAST: break;
        default: return fail(PLGPU_ERR_INVALID, "unknown aggregation kind");
        }
        pl->acc_of_agg[i] = a;
    }
    // operand columns shared between accs ((close * volume).sum() next to
    // volume.sum()) are loaded once by the fused kernel
    auto same_col = [](const DevCol& x, const DevCol& y) {
        return x.values == y.values && x.offset == y.offset && x.dtype == y.dtype;
    };
    for (int a = 0; a < p.nacc; ++a) {
        AccSpec& ac = p.acc[a];
        ac.v_from = ac.w_from = -1;
        for (int b = 0; b < a && ac.v_from < 0; ++b)
            if (same_col(p.acc[b].c, ac.c)) ac.v_from = b;
        if (ac.dop != DOP_NONE && !(ac.dop & DOP_LIT))
            for (int b = 0; b < p.nacc && ac.w_from < 0; ++b)
                if (same_col(p.acc[b].c, ac.c2) && p.acc[b].v_from < 0 && b != a) ac.w_from = b;
    }
    for (int a = 0; a < p.nacc; ++a) {
        AccSpec& ac = p.acc[a];
        // an inf / NaN row of an f64 acc always ORs the flags word
        if (ac.isf) ac.flags |= A_FLAGS;
        if ((ac.flags & A_CNT) && ac.c.validity == nullptr && ac.c2.validity == nullptr && !force_counts)
            ac.flags &= ~A_CNT;
        if (ac.flags & (A_FSUM | A_FSUMCAST)) {
            ac.f_sum = nf;
            nf += 3;
        }
        if (ac.flags & A_ISUM) ac.f_isum = nf++;
        if (ac.flags & A_CNT) ac.f_cnt = nf++;
        if (ac.flags & A_MIN) {
            ac.f_min = nf++;
            p.min_init_mask |= 1ull << ac.f_min;
        }
        if (ac.flags & A_MAX) ac.f_max = nf++;
        if (ac.flags & A_FLAGS) ac.f_flags = nf++;
    }
    if (nf > kMaxFields) return fail(PLGPU_ERR_INVALID, "too many accumulator fields");
    if (nf > 255) return fail(PLGPU_ERR_INVALID, "too many accumulator fields");
    p.nfields = nf;
    std::memset(p.fop, 0, sizeof p.fop);
    p.fop[p.f_len] = FOP_ADD;
    if (p.f_first >= 0) p.fop[p.f_first] = FOP_MIN;
    if (p.f_last >= 0) p.fop[p.f_last] = FOP_MAX;
    for (int a = 0; a < p.nacc; ++a) {
        const AccSpec& ac = p.acc[a];
        if (ac.f_sum >= 0) {
            p.fop[ac.f_sum] = FOP_ADD192;
            p.fop[ac.f_sum + 1] = FOP_SKIP;
            p.fop[ac.f_sum + 2] = FOP_SKIP;
        }
        if (ac.f_isum >= 0) p.fop[ac.f_isum] = FOP_ADD;
        if (ac.f_cnt >= 0) p.fop[ac.f_cnt] = FOP_ADD;
        if (ac.f_min >= 0) p.fop[ac.f_min] = FOP_MIN;
        if (ac.f_max >= 0) p.fop[ac.f_max] = FOP_MAX;
        if (ac.f_flags >= 0) p.fop[ac.f_flags] = FOP_OR;
    }
    for (int a = 0; a < p.nacc; ++a) {
        const AccSpec& ac = p.acc[a];
        auto fb = [](int f) -> uint64_t { return f < 0 ? (uint64_t)kNoField : (uint64_t)f; };
        p.desc[a] = (uint64_t)(ac.flags & 0xFF) | (fb(ac.f_sum) << 8) | (fb(ac.f_isum) << 16) | (fb(ac.f_cnt) << 24) |
                    (fb(ac.f_min) << 32) | (fb(ac.f_max) << 40) | (fb(ac.f_flags) << 48) |
                    ((uint64_t)(ac.isf ? 1 : 0) << 56) | ((uint64_t)(ac.uns ? 1 : 0) << 57);
    }
    // simple predicate: reuse an aggregated column's registers when possible
    // (an acc reading that column as it is)
    p.pred_acc = -1;
    if (dp.simple) {
        p.pred_col = to_dev(cols[dp.simple_col]);
        for (int a = 0; a < p.nacc && p.pred_acc < 0; ++a)
            if (p.acc[a].c.values == p.pred_col.values && p.acc[a].c.offset == p.pred_col.offset &&
                p.acc[a].c.dtype == p.pred_col.dtype && p.acc[a].c.validity == p.pred_col.validity)
                p.pred_acc = a;
    }
    pl->outs.clear();
    for (int i = 0; i < naggs; ++i) {
        OutSpec o;
        std::memset(&o, 0, sizeof o);
        o.kind = aggs[i].kind & 0xFF;
        o.acc = pl->acc_of_agg[i];
        o.ddof = (aggs[i].kind >> 8) & 0xFF;
        o.acc_hi = var_hi[i];
        o.acc_lo = var_lo[i];
        const int32_t dt = ins[aggs[i].col].dtype;
        o.in_isf = dtype_is_float(dt);
        o.in_uns = dt == PLGPU_U64;
        switch (o.kind) {
        case PLGPU_AGG_VAR:
        case PLGPU_AGG_STD: o.out_dtype = PLGPU_F64; break;
        case PLGPU_AGG_LEN:
        case PLGPU_AGG_COUNT: o.out_dtype = PLGPU_U32; break;
        case PLGPU_AGG_MEAN: o.out_dtype = dt == PLGPU_F32 ? PLGPU_F32 : PLGPU_F64; break;  // reduce/mean.rs:29
        case PLGPU_AGG_SUM:  // reduce/sum.rs:40 out_dtype: small ints sum as Int64
            o.out_dtype = (dt == PLGPU_I8 || dt == PLGPU_I16 || dt == PLGPU_U8 || dt == PLGPU_U16) ? PLGPU_I64 : dt;
            break;
        default: o.out_dtype = dt; break;
        }
        pl->outs.push_back(o);
    }
    return PLGPU_OK;
}

static int log2_ceil(int64_t x) {
    int b = 0;
    while ((int64_t(1) << b) < x) ++b;
    return b;
}

// Size the LDS table / grid from the distinct-key sample of the plan kernel.
static void size_tables(Plan* pl, uint64_t distinct, uint64_t sampled, int* gbits_out, int64_t hll_est = -1,
                        int64_t* est_out = nullptr) {
    GbParams& p = pl->p;
    const int64_t n = p.n;
    const int nf = p.nfields;
    // Max LDS slots at one workgroup per CU (160 KiB), power of two.
    int lmax_bits = 12;
    while (lmax_bits > 6 && (size_t)nf * ((1u << lmax_bits) + 2) * 8 + kWgScratch > 160 * 1024) --lmax_bits;
    const bool saturated = distinct >= (uint64_t)kPlanSetSlots / 2;
    int want_bits = log2_ceil(std::max<int64_t>(64, (int64_t)distinct * 2));
    pl->use_lds = !saturated && want_bits <= lmax_bits;
    if (!pl->use_lds) want_bits = 6;  // keep a tiny (unused) table
    p.lbits = want_bits;
    p.lcap = 1 << want_bits;
    pl->lds_bytes = pl->use_lds ? (size_t)nf * (p.lcap + 2) * 8 : 0;
    // Global table: the sample saw most keys if distinct << sampled.
    int64_t est;
    if ((saturated || sampled == 0) && hll_est >= 0) est = std::min<int64_t>(n, hll_est + hll_est / 4 + 1024);
    else if (saturated || sampled == 0) est = n;
    else if ((int64_t)distinct * 4 < (int64_t)sampled) est = (int64_t)distinct * 2 + 64;
    else est = std::min<int64_t>(n, (int64_t)((double)distinct * (double)n / (double)sampled) + 64);
    *gbits_out = log2_ceil(std::max<int64_t>(1024, est * 2));
    if (est_out) *est_out = est;
    // Grid: fill the chip (LDS permitting), rows per workgroup bounded for
    // the limb headroom.
    int per_cu = 4;
    if (pl->lds_bytes > 0) per_cu = (int)std::max<size_t>(1, std::min<size_t>(4, (160 * 1024) / pl->lds_bytes));
    int64_t grid = (int64_t)num_cus() * per_cu;
    const int64_t need = (n + kMaxRowsPerWg - 1) / kMaxRowsPerWg;
    if (grid < need) grid = need;
    const int64_t useful = (n + 4 * kGbThreads - 1) / (4 * kGbThreads);
    if (grid > useful) grid = useful < 1 ? 1 : useful;
    pl->grid = (int)grid;
}

template <int PRED, bool LDS>
static hipError_t launch_main(const Plan& pl, const DevProgram& dp, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)gb_kernel<PRED, LDS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr_set = true;
    }
    gb_kernel<PRED, LDS><<<pl.grid, kGbThreads, pl.lds_bytes, s>>>(pl.p, dp);
    return hipGetLastError();
}

static hipError_t launch_fast_dispatch(const Plan& pl, const DevProgram& dp, int pred, hipStream_t s) {
    if (pl.nulls) {
        // validity bitmaps on the key, aggregated or predicate columns
        switch (pl.p.nacc) {
        case 0: return launch_fast_nulls<0>(pl, dp, pred, s);
        case 1: return launch_fast_nulls<1>(pl, dp, pred, s);
        case 2: return launch_fast_nulls<2>(pl, dp, pred, s);
        case 3: return launch_fast_nulls<3>(pl, dp, pred, s);
        case 4: return launch_fast_nulls<4>(pl, dp, pred, s);
        case 5: return launch_fast_nulls<5>(pl, dp, pred, s);
        default: return launch_fast_nulls<6>(pl, dp, pred, s);
        }
    }
    bool dv = false;
    for (int a = 0; a < pl.p.nacc; ++a) dv = dv || pl.p.acc[a].dop != DOP_NONE;
    if (pl.p.kp.n > 0) {
        // fused key packing: plain (non-derived) inputs only (gb_plan
        // guarantees it, falling back to a code column otherwise)
        if (dv || pl.p.kp.n > kKpFast) return hipErrorInvalidValue;
        if (pl.p.kp.c[0].dtype == PLGPU_STR) {
            switch (pl.p.nacc) {
            case 0: return hipErrorInvalidValue;
            case 1: return launch_fast_nacc<1, false, 2>(pl, dp, pred, s);
            case 2: return launch_fast_nacc<2, false, 2>(pl, dp, pred, s);
            case 3: return launch_fast_nacc<3, false, 2>(pl, dp, pred, s);
            case 4: return launch_fast_nacc<4, false, 2>(pl, dp, pred, s);
            case 5: return launch_fast_nacc<5, false, 2>(pl, dp, pred, s);
            default: return launch_fast_nacc<6, false, 2>(pl, dp, pred, s);
            }
        }
        switch (pl.p.nacc) {
        case 0: return launch_fast_nacc<0, false, 1>(pl, dp, pred, s);
        case 1: return launch_fast_nacc<1, false, 1>(pl, dp, pred, s);
        case 2: return launch_fast_nacc<2, false, 1>(pl, dp, pred, s);
        case 3: return launch_fast_nacc<3, false, 1>(pl, dp, pred, s);
        case 4: return launch_fast_nacc<4, false, 1>(pl, dp, pred, s);
        case 5: return launch_fast_nacc<5, false, 1>(pl, dp, pred, s);
        default: return launch_fast_nacc<6, false, 1>(pl, dp, pred, s);
        }
    }
    if (dv && var_triple(pl) && !pl.runs)
        return pred == 0 ? launch_fast_var<0>(pl, dp, s) : launch_fast_var<1>(pl, dp, s);
    const int pair = dv && options().gb_pair ? product_pair(pl) : -1;
    if (pair == 0) return pred == 0 ? launch_fast_pair<0, 2>(pl, dp, s) : launch_fast_pair<1, 2>(pl, dp, s);
    if (pair == 1) return pred == 0 ? launch_fast_pair<0, 3>(pl, dp, s) : launch_fast_pair<1, 3>(pl, dp, s);
    if (dv) {
        switch (pl.p.nacc) {
        case 1: return launch_fast_nacc<1, true>(pl, dp, pred, s);
        case 2: return launch_fast_nacc<2, true>(pl, dp, pred, s);
        case 3: return launch_fast_nacc<3, true>(pl, dp, pred, s);
        case 4: return launch_fast_nacc<4, true>(pl, dp, pred, s);
        case 5: return launch_fast_nacc<5, true>(pl, dp, pred, s);
        default: return launch_fast_nacc<6, true>(pl, dp, pred, s);
        }
    }
    switch (pl.p.nacc) {
    case 0: return launch_fast_nacc<0, false>(pl, dp, pred, s);
    case 1: return launch_fast_nacc<1, false>(pl, dp, pred, s);
    case 2: return launch_fast_nacc<2, false>(pl, dp, pred, s);
    case 3: return launch_fast_nacc<3, false>(pl, dp, pred, s);
    case 4: return launch_fast_nacc<4, false>(pl, dp, pred, s);
    case 5: return launch_fast_nacc<5, false>(pl, dp, pred, s);
    default: return launch_fast_nacc<6, false>(pl, dp, pred, s);
    }
}

static hipError_t launch_main_dispatch(const Plan& pl, const DevProgram& dp, int pred, hipStream_t s) {
    if (pl.p.kp.n > 0) return hipErrorInvalidValue;  // the generic kernel reads a key column
    if (pl.use_lds) {
        if (pred == 0) return launch_main<0, true>(pl, dp, s);
        if (pred == 1) return launch_main<1, true>(pl, dp, s);
        return launch_main<2, true>(pl, dp, s);
    }
    if (pred == 0) return launch_main<0, false>(pl, dp, s);
    if (pred == 1) return launch_main<1, false>(pl, dp, s);
    return launch_main<2, false>(pl, dp, s);
}

// One group-by execution: plan, sampled windows, table, main launches,
// finalize.  Shared by plgpu_group_by_agg (single GPU) and the partial /
// merge entry points of the hash-partitioned multi-GPU group-by.

// Aggregation inputs given as programs over the columns (plgpu_agg_input):
// agg.col >= ncols names input agg.col - ncols.  Each is classified once:
//   a single column                        -> that column;
//   x op y, x / y Float64 columns or one a literal, op + - * / (one IEEE
//   rounding, the lowering's own typing)    -> fused: computed in registers
//                                              by the fused kernel (DOP_*);
//   anything else                          -> materialised by plgpu_eval
//                                              before the pass.
// A fused input is materialised as well when the pass does not run the
// fused kernel (generic kernel, partitioned many-groups path).
__global__ void sq_split_kernel(DevCol x, int64_t n, int32_t dop, uint64_t* __restrict__ out) {
    const uint64_t* v = (const uint64_t*)x.values;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[x.offset + i] = derive(dop, v[x.offset + i], 0ull);
}

struct DerivIn {
    const plgpu_instr* prog;
    int32_t n;
    int32_t kind;    // 1 column, 2 fused, 0 materialise, 3 a var column's x * x split (DOP_SQHI / DOP_SQLO)
    int32_t ca, cb;  // column operands (cb -1: literal)
    int32_t dop;
    uint64_t imm;
    int32_t out_dtype;
};

struct Deriv {
    std::vector<DerivIn> in;
};

static int classify_inputs(const plgpu_column* cols, int32_t ncols, const plgpu_agg_input* inputs, int32_t ninputs,
                           Deriv* d) {
    d->in.assign((size_t)std::max(ninputs, 0), DerivIn{});
    for (int j = 0; j < ninputs; ++j) {
        DerivIn& di = d->in[j];
        di.prog = inputs[j].program;
        di.n = inputs[j].n_instr;
        DevProgram lp;
        int rc = lower_program(cols, ncols, di.prog, di.n, &lp);
        if (rc) return rc;
        di.out_dtype = lp.out_dtype;
        di.kind = 0;
        di.cb = -1;
        if (lp.n == 1 && lp.code[0].op == D_COL) {
            di.kind = 1;
            di.ca = lp.code[0].arg;
            continue;
        }
        if (lp.n != 3 || lp.code[2].arg != PLGPU_F64) continue;
        int32_t op;
        switch (lp.code[2].op) {
        case D_ADD_F: op = DOP_ADD; break;
        case D_SUB_F: op = DOP_SUB; break;
        case D_MUL_F: op = DOP_MUL; break;
        case D_DIV_F: op = DOP_DIV; break;
        case D_DIV_FS: op = DOP_DIVS; break;
        default: continue;
        }
        const DevInstr &i0 = lp.code[0], &i1 = lp.code[1];
        auto f64col = [&](const DevInstr& i) { return i.op == D_COL && cols[i.arg].dtype == PLGPU_F64; };
        if (f64col(i0) && f64col(i1)) {
            di.kind = 2, di.ca = i0.arg, di.cb = i1.arg, di.dop = op;
        } else if (f64col(i0) && i1.op == D_LIT) {
            di.kind = 2, di.ca = i0.arg, di.dop = op | DOP_LIT, di.imm = i1.imm;
        } else if (i0.op == D_LIT && f64col(i1)) {
            di.kind = 2, di.ca = i1.arg, di.dop = op | DOP_LIT | DOP_SWAP, di.imm = i0.imm;
        }
    }
    return PLGPU_OK;
}

struct GbRun {
    Plan pl;
    DevProgram dp;
    int pred = 0;
    hipStream_t s = nullptr;
    uint64_t* status = nullptr;  // ST_WORDS words + kMaxAcc int32 bottoms
    int32_t* bottoms = nullptr;
    uint64_t* gtab = nullptr;
    uint64_t st[ST_WORDS];
    int32_t hb[kMaxAcc];         // host copy of the fixed-point bottoms
    int gbits = 10;
    int attempts = 0;
    float ms = 0.f;
    int32_t key_dtype = PLGPU_I64;
    bool maintain = false;
    bool want_first = false;                 // keep each group's first selected row (multi-key)
    int world = 1;
    uint32_t wide = 0;                       // accs summed by the wide fallback
    int wide_exmin[kMaxAcc] = {0};
    int wide_exmax[kMaxAcc] = {0};
    int64_t* wide_digits[kMaxAcc] = {nullptr};
    double* wide_sum[kMaxAcc] = {nullptr};
    int64_t est_groups = -1;                 // plan's group estimate (sampled / HLL)
    bool wide_round = true;                  // gb_wide rounds (false: multi-GPU partial digits)
    std::string plan_ckey;                   // plan-cache key when the statistics came from the cache
    // fused key packing (p.kp.n > 0): the plan found the fused kernel does
    // not apply (kp_fallback), or a selected row left the packing plan
    // (kp_bad); the caller then writes a code column / repacks
    bool kp_fallback = false;
    bool kp_bad = false;
    // partitioned path (gb_partition): buffers, ranges, launch shape
    bool part = false;
    int pbits = 0;
    int part_lbits = 0;
    int part_blocks = 1;
    int part_levels = 0;                     // scatter passes taken (info)
    int rbits = 0;                           // global-table region bits (GbParams::rbits)
    // compact regions (GbParams::region_cnt): allowed by the caller (a result
    // read only through gb_finalize), on for this attempt (compact_now)
    bool compact_ok = false;
    bool compact_now = false;
    uint32_t* region_cnt = nullptr;
    uint64_t* rtab = nullptr;                // compact regions' table (GbParams::rtab)
    bool has_null_key = false;               // partitioned: null keys written as null_key (GbParams)
    int64_t null_key = 0;
    uint64_t* pbuf = nullptr;
    uint64_t* prange = nullptr;              // scan of the count matrix + partition bounds
    const uint64_t* part_range = nullptr;    // P + 1 partition boundaries (inside prange)
    int64_t part_rows_total = 0;
    std::vector<uint64_t> part_hrange;       // host copy of the P + 1 bounds
    PartOut pout;
    // aggregation inputs: the predicate's columns, the derived inputs and
    // the columns materialised for them (owned)
    const plgpu_column* cols = nullptr;
    int32_t ncols = 0;
    const Deriv* deriv = nullptr;
    std::vector<InSpec> ins;
    std::vector<plgpu_column> mat;
    std::vector<int> acc_input;  // input index of each acc

    GbRun() {
        std::memset(st, 0, sizeof st);
        std::memset(hb, 0, sizeof hb);
        std::memset(&pout, 0, sizeof pout);
    }
    ~GbRun() {
        for (int a = 0; a < kMaxAcc; ++a) {
            dev_free(wide_digits[a], s);
            dev_free(wide_sum[a], s);
        }
        dev_free(gtab, s);
        dev_free(status, s);
        dev_free(pbuf, s);
        dev_free(region_cnt, s);
        dev_free(rtab, s);
        dev_free(prange, s);
        for (auto& c : mat) plgpu_column_release(&c);
    }
};

// The run's status words into R.st (host), one synchronisation.
static int d2h_status(GbRun& R) {
    void* d[1] = {R.st};
    const void* src[1] = {R.status};
    const size_t b[1] = {sizeof R.st};
    return d2h_stage(1, d, src, b, R.s);
}

// Materialise aggregation input j (plgpu_eval of its program) into R.mat.
static int gb_materialize(GbRun& R, int j, plgpu_column* out) {
    if (R.deriv == nullptr || j < 0 || j >= (int)R.deriv->in.size())
        return fail(PLGPU_ERR_INVALID, "internal: derived input index out of range");
    const DerivIn& di = R.deriv->in[j];
    plgpu_column c;
    std::memset(&c, 0, sizeof c);
    int rc;
    if (di.kind == 3) {
        // x * x or its exact error, rows at the column's own offset so its
        // validity bitmap is shared as it is
        const plgpu_column& x = R.cols[di.ca];
        if ((rc = make_owned_column(&c, PLGPU_F64, x.offset + x.length, false, R.s))) return rc;
        c.offset = x.offset;
        c.length = x.length;
        c.validity = x.validity;
        c.null_count = x.null_count;
        const int g = (int)std::min<int64_t>((x.length + 255) / 256, 256 * 32);
        if (x.length > 0) sq_split_kernel<<<g, 256, 0, R.s>>>(to_dev(x), x.length, di.dop, (uint64_t*)c.values);
        if (hipGetLastError() != hipSuccess) {
            plgpu_column_release(&c);
            return fail(PLGPU_ERR_HIP, "var square split");
        }
    } else {
        rc = plgpu_eval(R.cols, R.ncols, di.prog, di.n, &c, R.s);
        if (rc) return rc;
    }
    R.mat.push_back(c);
    *out = c;
    return PLGPU_OK;
}

// The fused derived accs as plain columns: when the pass will not run the
// fused kernel.  (Their sampled exponents stay valid: same values.)
static int gb_unfuse(GbRun& R) {
    GbParams& p = R.pl.p;
    for (int a = 0; a < p.nacc; ++a) {
        if (p.acc[a].dop == DOP_NONE) continue;
        plgpu_column c;
        int rc = gb_materialize(R, R.acc_input[a] - R.ncols, &c);
        if (rc) return rc;
        p.acc[a].c = to_dev(c);
        p.acc[a].dop = DOP_NONE;
        std::memset(&p.acc[a].c2, 0, sizeof p.acc[a].c2);
        // the predicate no longer shares this acc's registers
        if (p.pred_acc == a) p.pred_acc = -1;
    }
    return PLGPU_OK;
}

static bool gb_has_fused(const GbRun& R) {
    for (int a = 0; a < R.pl.p.nacc; ++a)
        if (R.pl.p.acc[a].dop != DOP_NONE) return true;
    return false;
}

static int gb_prepare(GbRun& R, const plgpu_column* key, const plgpu_column* cols, int32_t ncols,
                      const plgpu_instr* program, int32_t n_instr, const plgpu_agg* aggs, int32_t naggs,
                      bool maintain_order, bool force_counts, void* stream, const Deriv* deriv = nullptr) {
    R.s = as_stream(stream);
    if (key == nullptr) return fail(PLGPU_ERR_INVALID, "key is NULL");
    if (ncols < 0 || ncols > PLGPU_MAX_COLS) return fail(PLGPU_ERR_INVALID, "too many columns (max 8)");
    if (naggs < 0 || naggs > PLGPU_MAX_COLS * 2) return fail(PLGPU_ERR_INVALID, "too many aggregations (max 16)");
    if (!dtype_is_int(key->dtype)) return fail(PLGPU_ERR_SCHEMA, "group-by key must be an integer column");
    for (int i = 0; i < ncols; ++i)
        if (cols[i].length != key->length) return fail(PLGPU_ERR_SHAPE, "columns must match the key length");
    R.key_dtype = key->dtype;
    R.maintain = maintain_order;
    R.cols = cols;
    R.ncols = ncols;
    R.deriv = deriv;
    std::memset(&R.dp, 0, sizeof R.dp);
    int rc;
    if (program != nullptr && n_instr > 0) {
        if ((rc = lower_program(cols, ncols, program, n_instr, &R.dp))) return rc;
        if (R.dp.out_dtype != PLGPU_BOOL) return fail(PLGPU_ERR_SCHEMA, "filter predicate must be of type `Boolean`");
        R.pred = R.dp.simple ? 1 : 2;
    }
    // aggregation inputs: the columns, then the derived inputs (a column,
    // a fused x op y, or materialised now)
    R.ins = column_inputs(cols, ncols);
    if (deriv) {
        for (size_t j = 0; j < deriv->in.size(); ++j) {
            const DerivIn& di = deriv->in[j];
            InSpec in;
            std::memset(&in, 0, sizeof in);
            if (di.kind == 1) {
                in = R.ins[di.ca];
            } else if (di.kind == 2 || di.kind == 3) {
                in.col = cols[di.ca];
                if (di.cb >= 0) in.col2 = cols[di.cb];
                in.dtype = PLGPU_F64;
                in.dop = di.dop;
                in.imm = di.imm;
            } else {
                if ((rc = gb_materialize(R, (int)j, &in.col))) return rc;
                in.dtype = in.col.dtype;
            }
            R.ins.push_back(in);
        }
    }
    if ((rc = plan_groupby(key, cols, ncols, R.ins.data(), (int32_t)R.ins.size(), aggs, naggs,
                           maintain_order || R.want_first, R.dp, &R.pl, force_counts)))
        return rc;
    // the input index of each acc (also the var / std accs of x * x's parts,
    // which no aggregation names directly)
    R.acc_input.assign(kMaxAcc, -1);
    for (int a = 0; a < R.pl.p.nacc; ++a) R.acc_input[a] = R.pl.acc_in[a];
    // status words, the bottoms, then (at word kPlanSetWord) the plan's
    // global distinct-key set; one allocation, one memset
    static_assert(ST_WORDS * 8 + kMaxAcc * 4 <= kPlanSetWord * 8, "status layout");
    const size_t bytes = (size_t)(kPlanSetWord + kPlanSetSlots) * 8;
    if ((rc = dev_alloc((void**)&R.status, bytes, R.s))) return rc;
    R.bottoms = (int32_t*)(R.status + ST_WORDS);
    R.pl.p.status = R.status;
    R.pl.p.bottoms = R.bottoms;
    PLGPU_HIP(hipMemsetAsync(R.status, 0, bytes, R.s));
    return PLGPU_OK;
}

// HyperLogLog distinct-key count over the whole key column (2^12 registers,
// ~1.6 % standard error), run only when the plan's sample saturates: it
// sizes the global table for high-cardinality keys instead of assuming every
// row is a new group.
constexpr int kHllBits = 12;

__device__ __forceinline__ void hll_add(uint32_t* r, uint64_t k) {
    const uint64_t h = mk_fmix(k ^ 0x5851F42D4C957F2Dull);
    const uint32_t j = (uint32_t)(h >> (64 - kHllBits));
    const uint32_t rho = (uint32_t)__clzll((h << kHllBits) | (1ull << (kHllBits - 1))) + 1;
    if (rho > r[j]) atomicMax(&r[j], rho);
}

__global__ __launch_bounds__(256) void gb_hll_kernel(DevCol key, int64_t n, uint32_t* __restrict__ regs) {
    __shared__ uint32_t r[1 << kHllBits];
    for (int i = threadIdx.x; i < (1 << kHllBits); i += blockDim.x) r[i] = 0;
    __syncthreads();
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (key.validity == nullptr && dtype_bytes(key.dtype) == 8) {
        // null-free 8-byte keys: 8 branch-free streamed loads in flight
        const uint64_t* kp = (const uint64_t*)key.values + key.offset;
        constexpr int U = 8;
        for (; i0 < n; i0 += T * U) {
            uint64_t k[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = i0 + u * T;
                k[u] = __builtin_nontemporal_load(kp + (i < n ? i : n - 1));
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (i0 + u * T < n) hll_add(r, k[u]);
        }
    } else {
        for (int64_t i = i0; i < n; i += T)
            if (dev_valid(key, i)) hll_add(r, dev_load(key, i));
    }
    __syncthreads();
    for (int i = threadIdx.x; i < (1 << kHllBits); i += blockDim.x)
        if (r[i]) atomicMax(&regs[i], r[i]);
}

static double hll_estimate(const uint32_t* regs) {
    const double m = (double)(1 << kHllBits);
    double sum = 0;
    int zeros = 0;
    for (int i = 0; i < (1 << kHllBits); ++i) {
        sum += std::ldexp(1.0, -(int)regs[i]);
        zeros += regs[i] == 0;
    }
    double e = (0.7213 / (1.0 + 1.079 / m)) * m * m / sum;
    if (e <= 2.5 * m && zeros > 0) e = m * std::log(m / zeros);  // linear counting
    return e;
}

// Plan statistics of recent group-bys (the plan kernels' status words and
// the HLL estimate), keyed by the plan's inputs: the key / packed-key
// columns, the accumulators (columns, derived operands, field layout), the
// row count and the simple predicate.  A repeated query over resident
// columns (the plugin's warm path) skips the sampling launches and their
// round trip.  The statistics only steer table sizes and kernel choice:
// every pass still checks its own results (table full, window flags,
// packed-key fit) and reruns, so a stale entry -- a freed column's address
// reused by other data -- costs speed, never exactness.  Option
// plan_cache = 0 disables it.
namespace {
struct PlanStats {
    uint64_t st[ST_WORDS];
    int64_t hll;
};
std::mutex g_plan_mu;
std::vector<std::pair<std::string, PlanStats>> g_plan_cache;  // most recent last
constexpr size_t kPlanCacheEntries = 32;

std::string plan_key(const GbRun& R) {
    const GbParams& p = R.pl.p;
    std::string k;
    auto put = [&k](const void* x, size_t nb) { k.append((const char*)x, nb); };
    put(&p.n, sizeof p.n);
    put(&p.key, sizeof p.key);
    put(&p.kp, sizeof p.kp);
    put(&p.nacc, sizeof p.nacc);
    for (int a = 0; a < p.nacc; ++a) put(&p.acc[a], sizeof p.acc[a]);
    put(&R.pred, sizeof R.pred);
    if (R.pred == 1) {
        put(&R.dp.simple_isf, sizeof R.dp.simple_isf);
        put(&R.dp.simple_op, sizeof R.dp.simple_op);
        put(&R.dp.simple_imm, sizeof R.dp.simple_imm);
        put(&p.pred_col, sizeof p.pred_col);
        put(&p.pred_acc, sizeof p.pred_acc);
    }
    return k;
}

bool plan_cache_get(const std::string& key, PlanStats* out) {
    std::lock_guard<std::mutex> g(g_plan_mu);
    for (size_t i = g_plan_cache.size(); i-- > 0;) {
        if (g_plan_cache[i].first != key) continue;
        *out = g_plan_cache[i].second;
        std::rotate(g_plan_cache.begin() + (ptrdiff_t)i, g_plan_cache.begin() + (ptrdiff_t)i + 1, g_plan_cache.end());
        return true;
    }
    return false;
}

void plan_cache_erase(const std::string& key) {
    std::lock_guard<std::mutex> g(g_plan_mu);
    for (size_t i = 0; i < g_plan_cache.size(); ++i)
        if (g_plan_cache[i].first == key) {
            g_plan_cache.erase(g_plan_cache.begin() + (ptrdiff_t)i);
            return;
        }
}

void plan_cache_put(const std::string& key, const PlanStats& v) {
    std::lock_guard<std::mutex> g(g_plan_mu);
    for (auto& e : g_plan_cache)
        if (e.first == key) {
            e.second = v;
            return;
        }
    if (g_plan_cache.size() >= kPlanCacheEntries) g_plan_cache.erase(g_plan_cache.begin());
    g_plan_cache.emplace_back(key, v);
}
}  // namespace

// The same for the multi-key packing plan (the sampled key ranges of
// mk_plan_pack_sampled, or the exact ranges once a row left them): the
// fused kernel flags any row outside the plan and the caller repacks, so a
// stale plan costs a repack, never exactness.
namespace {
std::vector<std::pair<std::string, MkPack>> g_pack_cache;  // most recent last

std::string pack_key(const MkKeys& mk, int64_t n) {
    std::string k((const char*)&mk, sizeof mk);
    k.append((const char*)&n, sizeof n);
    return k;
}

bool pack_cache_get(const std::string& key, MkPack* out) {
    std::lock_guard<std::mutex> g(g_plan_mu);
    for (auto& e : g_pack_cache)
        if (e.first == key) {
            *out = e.second;
            return true;
        }
    return false;
}

void pack_cache_put(const std::string& key, const MkPack& v) {
    std::lock_guard<std::mutex> g(g_plan_mu);
    for (auto& e : g_pack_cache)
        if (e.first == key) {
            e.second = v;
            return;
        }
    if (g_pack_cache.size() >= kPlanCacheEntries) g_pack_cache.erase(g_pack_cache.begin());
    g_pack_cache.emplace_back(key, v);
}
}  // namespace

void gb_plan_cache_clear() {
    std::lock_guard<std::mutex> g(g_plan_mu);
    g_plan_cache.clear();
    g_pack_cache.clear();
}

// Distinct keys of the key column by HyperLogLog (gb_hll_kernel, ~1.6 %).
static int gb_hll_count(GbRun& R, int64_t* out) {
    uint32_t* regs = nullptr;
    std::vector<uint32_t> h(1 << kHllBits);
    int rc = dev_alloc((void**)&regs, h.size() * 4, R.s);
    if (rc) return rc;
    hipError_t e = hipMemsetAsync(regs, 0, h.size() * 4, R.s);
    if (e == hipSuccess) {
        KtScope kt("gb_hll_kernel", R.s);
        gb_hll_kernel<<<num_cus() * 4, 256, 0, R.s>>>(R.pl.p.key, R.pl.p.n, regs);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h.data(), regs, h.size() * 4, hipMemcpyDeviceToHost, R.s);
    if (e == hipSuccess) e = hipStreamSynchronize(R.s);
    dev_free(regs, R.s);
    if (e != hipSuccess) return hip_fail(e, "gb_hll_kernel");
    *out = (int64_t)hll_estimate(h.data());
    return PLGPU_OK;
}

// Planning launch -> distinct-key estimate, fixed-point bottoms, table
// sizes, kernel choice.  `fixed` (nullable) overrides the sampled bottoms.
static int gb_plan(GbRun& R, const int32_t* fixed) {
    Plan& pl = R.pl;
    GbParams& p = pl.p;
    const int64_t n = p.n;
    // a simple predicate filters the sampled values, so the windows (and
    // the 2-limb choice) follow the rows the sums take; when some summed
    // column has no selected nonzero value in the sample, its acc tasks run
    // again unfiltered (the key task is not repeated)
    const bool ps = R.pred == 1;
    // (large inputs only: below 2^24 rows the sampling is a small share)
    const bool use_cache = fixed == nullptr && options().plan_cache != 0 && n >= (int64_t(1) << 24);
    const std::string ckey = use_cache ? plan_key(R) : std::string();
    PlanStats cached;
    const bool hit = use_cache && plan_cache_get(ckey, &cached);
    if (hit) {
        std::memcpy(R.st, cached.st, sizeof R.st);
        R.plan_ckey = ckey;
    } else {
        {
            KtScope kt("gb_plan_kernel", R.s);
            gb_plan_kernel<<<p.nacc * kPlanBlocks + kPlanKeyBlocks, kPlanThreads, 0, R.s>>>(
                p, R.status + kPlanSetWord, kPlanSamples, ps ? 1 : 0, ps ? R.dp.simple_isf : 0,
                ps ? R.dp.simple_op : 0, ps ? R.dp.simple_imm : 0ull);
        }
        PLGPU_HIP(hipGetLastError());
        if (int rs = d2h_status(R)) return rs;
        bool unsampled = false;
        for (int a = 0; a < p.nacc; ++a)
            if ((p.acc[a].flags & (A_FSUM | A_FSUMCAST)) && R.st[ST_MAXEX + a] == 0) unsampled = true;
        if (ps && unsampled) {
            gb_plan_kernel<<<p.nacc * kPlanBlocks, kPlanThreads, 0, R.s>>>(p, R.status + kPlanSetWord, kPlanSamples,
                                                                           0, 0, 0, 0ull);
            PLGPU_HIP(hipGetLastError());
            if (int rs = d2h_status(R)) return rs;
        }
        if (use_cache) {
            std::memcpy(cached.st, R.st, sizeof R.st);
            cached.hll = -1;
            plan_cache_put(ckey, cached);
        }
    }
    R.st[ST_SAMPLED] = (uint64_t)std::min<int64_t>(n, kPlanSamples);
    // sorted / clustered keys: the fused kernel's lanes keep a register
    // accumulator (option "runs" = 0 / 1 forces the choice in tests)
    pl.runs = options().runs >= 0 ? options().runs != 0 : R.st[ST_RUNS] * 2 > R.st[ST_SAMPLED];
    for (int a = 0; a < kMaxAcc; ++a) R.hb[a] = a < p.nacc ? plan_bottom(R.st[ST_MAXEX + a]) : 0;
    if (fixed)
        for (int a = 0; a < kMaxAcc; ++a) R.hb[a] = fixed[a];
    int64_t hll = -1;
    // clustered keys (the range-local test below): every row range's keys
    // showed in its samples, so the column holds at most ~kPlanKeyBlocks x
    // that many; twice that sizes the global table without the HLL pass
    // (a miss only costs a table-size rerun)
    const uint64_t local = R.st[ST_LOCAL];
    const uint64_t per_range = (uint64_t)std::min<int64_t>(n, kPlanSamples) / kPlanKeyBlocks;
    const bool clustered = n >= (int64_t(1) << 22) && local > 0 && local * 4 <= per_range * 3 && options().local != 0;
    if (clustered && R.st[ST_DISTINCT] >= (uint64_t)kPlanSetSlots / 2)
        hll = std::min<int64_t>(n, (int64_t)local * kPlanKeyBlocks * 2);
    if (hll < 0 && R.st[ST_DISTINCT] >= (uint64_t)kPlanSetSlots / 2 && n > 4 * (int64_t)kPlanSamples) {
        if (p.kp.n > 0) {
            // many groups: not the fused single-table kernel's case
            if (options().debug)
                fprintf(stderr, "[plgpu] key pack fallback: %llu distinct of %llu sampled\n",
                        (unsigned long long)R.st[ST_DISTINCT], (unsigned long long)R.st[ST_SAMPLED]);
            R.kp_fallback = true;
            return PLGPU_OK;
        }
        if (hit && cached.hll >= 0) {
            hll = cached.hll;
        } else {
            int rc = gb_hll_count(R, &hll);
            if (rc) return rc;
            if (use_cache) {
                cached.hll = hll;
                plan_cache_put(ckey, cached);
            }
        }
    }
    size_tables(&pl, R.st[ST_DISTINCT], R.st[ST_SAMPLED], &R.gbits, hll, &R.est_groups);
    // forced paths (option gb_path, tests): LDS tables on or off; the
    // fused-kernel and partitioned choices follow below
    const int gpath = options().gb_path;
    if (gpath == 0) {
        pl.use_lds = false;
        pl.lds_bytes = 0;
    } else if ((gpath == 1 || gpath == 2) && !pl.use_lds) {
        // the largest table one workgroup per CU holds; keys beyond it take
        // the global table
        int lb = 12;
        while (lb > 6 && (size_t)p.nfields * ((1u << lb) + 2) * 8 + kWgScratch > 160 * 1024) --lb;
        pl.use_lds = true;
        p.lbits = lb;
        p.lcap = 1 << lb;
        pl.lds_bytes = (size_t)p.nfields * (p.lcap + 2) * 8;
    }
    // range-local mode: too many keys for one LDS table over the column, but
    // few within each contiguous row range (the plan's per-range sample
    // count ST_LOCAL: a range's samples repeat their keys); the fused kernel
    // then gives each workgroup one contiguous run of tiles and an LDS table
    // sized for about twice the keys one range showed.  Keys beyond it take
    // the global table, so the choice only changes speed.
    pl.local = false;
    const int lbits0 = p.lbits, lcap0 = p.lcap;
    const size_t lds0 = pl.lds_bytes;
    {
        if (!pl.use_lds && clustered && gpath < 0) {
            const int lb = log2_ceil(std::max<int64_t>(64, 2 * (int64_t)local));
            const size_t bytes = (size_t)p.nfields * ((1u << lb) + 2) * 8;
            if (bytes + kWgScratch <= (size_t)160 * 1024) {
                pl.local = pl.use_lds = true;
                p.lbits = lb;
                p.lcap = 1 << lb;
                pl.lds_bytes = bytes;
            }
        }
    }
    // fast path eligibility: no nulls, 8-byte columns
    // at even offsets of 16-byte aligned buffers, simple or no predicate,
    // LDS table in use
    // (validity bitmaps allowed: the NULLS variant reads one validity byte
    // per row pair and column beside the values; plain inputs only)
    auto ok = [](const DevCol& c) {
        return (c.dtype == PLGPU_I64 || c.dtype == PLGPU_F64) && (c.offset & 1) == 0 &&
               ((uintptr_t)c.values & 15) == 0;
    };
    auto ok_kp = [](const KeyPack& k) {
        if (k.n == 1 && k.c[0].dtype == PLGPU_STR)
            return k.c[0].validity == nullptr && (k.c[0].offset & 1) == 0 && ((uintptr_t)k.c[0].values & 15) == 0 &&
                   ((uintptr_t)k.c[0].data & 7) == 0;
        bool good = k.n > 0 && k.n <= kKpFast;
        for (int i = 0; i < k.n && good; ++i) {
            const DevCol& c = k.c[i];
            const bool w8 = c.dtype == PLGPU_I64, w4 = c.dtype == PLGPU_I32 || c.dtype == PLGPU_U32;
            good = (w8 || w4) && c.validity == nullptr && (c.offset & 1) == 0 &&
                   ((uintptr_t)c.values & (w8 ? 15 : 7)) == 0;
        }
        return good;
    };
    bool fast = pl.use_lds && R.pred != 2 && (p.kp.n > 0 ? ok_kp(p.kp) : ok(p.key));
    for (int a = 0; a < p.nacc; ++a) {
        fast = fast && ok(p.acc[a].c);
        if (p.acc[a].dop != DOP_NONE && !(p.acc[a].dop & DOP_LIT)) fast = fast && ok(p.acc[a].c2);
    }
    if (R.pred == 1 && p.pred_acc < 0) fast = fast && ok(p.pred_col);
    {
        bool nul = p.key.validity != nullptr || (R.pred == 1 && p.pred_col.validity != nullptr);
        bool dv = false;
        for (int a = 0; a < p.nacc; ++a) {
            nul = nul || p.acc[a].c.validity != nullptr || p.acc[a].c2.validity != nullptr;
            dv = dv || p.acc[a].dop != DOP_NONE;
        }
        // nullable inputs: the NULLS variant takes plain inputs and a key
        // column (derived operands or a packed key take the generic kernel /
        // the code column)
        if (nul && (p.kp.n > 0 || dv)) fast = false;
        pl.nulls = nul;
        // whole-word validity reads (GbParams::vwords): every bitmap at a
        // column offset that is a multiple of 64 in an 8-byte aligned buffer
        auto wa = [](const DevCol& c) {
            return c.validity == nullptr || ((c.offset & 63) == 0 && ((uintptr_t)c.validity & 7) == 0);
        };
        bool vw = wa(p.key) && (R.pred != 1 || wa(p.pred_col));
        for (int a = 0; a < p.nacc; ++a) vw = vw && wa(p.acc[a].c);
        p.vwords = vw ? 1 : 0;
    }
    if (gpath == 0 || gpath == 1 || gpath == 3 || gpath == 5) fast = false;
    if (pl.local && !fast) {
        // the generic kernel walks the rows grid-strided: no range-local table
        pl.local = pl.use_lds = false;
        p.lbits = lbits0;
        p.lcap = lcap0;
        pl.lds_bytes = lds0;
    }
    const int64_t tile = (int64_t)2 * kGbThreads;
    p.n_full = fast ? (n / tile) * tile : 0;
    {
        // as many workgroups as the LDS budget allows per CU (up to 8)
        const int per_cu =
            (int)std::max<size_t>(1, std::min<size_t>(8, pl.lds_bytes ? (160 * 1024) / pl.lds_bytes : 8));
        int64_t g = (int64_t)num_cus() * per_cu;
        const int64_t need = (p.n_full + kMaxRowsPerWg - 1) / kMaxRowsPerWg;
        if (g < need) g = need;
        const int64_t useful = p.n_full / tile;
        if (g > useful) g = useful < 1 ? 1 : useful;
        pl.fast_grid = (int)g;
    }
    // sum-only signature with the compile-time field layout
    bool so = p.f_first < 0 && p.f_last < 0 && p.f_len == 1 && p.nacc > 0;
    for (int a = 0; a < p.nacc; ++a) {
        const AccSpec& ac = p.acc[a];
        so = so && ac.isf && ac.flags == (A_FSUM | A_FLAGS) && ac.f_sum == 2 + 4 * a && ac.f_flags == 5 + 4 * a &&
             ac.f_cnt < 0;
    }
    pl.sum_only = so;
    // two LDS limbs when every sampled nonzero value of every summed column
    // sits at least kLimb2Margin binades above the 2-limb window's bottom
    // (the register-run kernel for mixed aggregations holds two limbs the
    // same way, for f64 sums; integer columns summed as f64 keep it off)
    pl.limbs = 3;
    {
        bool two = true;
        for (int a = 0; a < p.nacc; ++a) {
            const AccSpec& ac = p.acc[a];
            if (ac.flags & A_FSUMCAST) two = false;
            if (!(ac.flags & A_FSUM)) continue;
            const int mn = 0x7FF - (int)R.st[ST_MINEX + a];
            if (mn != 0x7FF && mn < R.hb[a] + 40 + 1075 + kLimb2Margin) two = false;
        }
        if (two) pl.limbs = 2;
    }
    // the fused kernel covers every row (its last tile is masked); below one
    // tile, or off the fast path, the generic kernel takes them all
    p.row_begin = p.n_full > 0 ? n : 0;
    // partitioned path: too many groups for one LDS table, but few enough
    // that 2^kPartMaxBits partitions of LDS tables hold them; the key and
    // aggregated columns are copied as raw words (their null bits beside
    // them); the u32 count matrix and row ids bound n below 2^32
    R.part = false;
    // (a keyless reduction has no key column to partition by)
    // (validity bitmaps travel with the rows as the null-bits column)
    bool part_ok = n > 0 && n < 0xFFFFFFFFll && R.est_groups > 0 && p.key.values != nullptr &&
                   p.key.dtype != PLGPU_STR;
    // gb_path 5 (tests): the partitioned path with the checks above skipped,
    // so that the partition launchers' own preconditions must refuse
    if (gpath == 5) part_ok = true;
    if (part_ok && ((gpath < 0 && !pl.use_lds && n >= (int64_t(1) << 20)) || gpath == 3 || gpath == 5)) {
        // LDS table of the partition workgroups: two per CU, or one when
        // 2^kPartMaxBits partitions of the smaller table are not enough
        const int64_t want = R.est_groups + (R.est_groups >> 3);
        // sum-only on the 2-limb window: the fast kernel's slim table
        // (2 + 3 nacc fields); the full layout must still fit one workgroup
        // per CU for a 3-limb rerun through the generic kernel
        const int fields = (pl.sum_only && pl.limbs == 2) ? slim_words(p.nacc) : p.nfields;
        // Fewer, larger partition tables first (160 KB, one workgroup per
        // CU): measured 2-7 % faster than 80 KB tables at 14k-100k groups
        // (profiles/r02_ab_part.log)
        const int min_pb = std::min(kPartMaxBits, std::max(0, options().part_bits));
        const size_t b0 = options().part_lds_kb > 0 ? (size_t)options().part_lds_kb * 1024 : (size_t)160 * 1024;
        for (size_t budget : {b0, (size_t)80 * 1024}) {
            int lb = 13;
            // (+ 256 B: the fast kernel's static LDS, compact regions' wave counts)
            while (lb > 6 && ((size_t)fields * ((1u << lb) + 2) * 8 + 256 > budget ||
                              (size_t)p.nfields * ((1u << lb) + 2) * 8 > (size_t)160 * 1024))
                --lb;
            const int64_t per = (int64_t(1) << lb) / 2;  // groups per partition at load 1/2
            int pb = min_pb;
            while (pb < kPartMaxBits && want > (per << pb)) ++pb;
            if (want <= (per << pb)) {
                R.part = true;
                R.pbits = pb;
                R.part_lbits = lb;
                break;
            }
        }
    }
    if (R.part) p.n_full = 0, p.row_begin = 0;
    // the partition kernel's register accumulators pay when the rows of a
    // partition repeat their groups nearby (sorted or clustered keys)
    pl.part_racc = R.part && (pl.runs || clustered);
    if (p.kp.n > 0 && (p.n_full == 0 || R.part || gb_has_fused(R) ||
                       (p.kp.c[0].dtype == PLGPU_STR && (!pl.sum_only || p.nacc == 0)))) {
        // the packed key lives only in the fused kernel's registers
        if (options().debug)
            fprintf(stderr, "[plgpu] key pack fallback: n_full=%lld part=%d fused=%d use_lds=%d pred=%d\n",
                    (long long)p.n_full, (int)R.part, (int)gb_has_fused(R), (int)pl.use_lds, R.pred);
        R.kp_fallback = true;
        return PLGPU_OK;
    }
    // fused derived inputs run in the fused kernel only; any other pass
    // reads them materialised
    if (gb_has_fused(R) && (p.n_full == 0 || R.part)) return gb_unfuse(R);
    return PLGPU_OK;
}

// Scatter the selected rows into the hash partitions (once per run; the
// attempts of gb_main reuse them): one pass of 2^pbits digits, or two
// (level 1 over the input rows, level 2 within each level-1 partition).
template <int PRED, bool L2, bool F8, bool NUL = false>
static hipError_t gbp_pass(const GbRun& R, const PsGeom& g, const PartOut& in, uint32_t* cnt, uint64_t* part,
                           bool scatter, const PartOut& out) {
    hipStream_t s = R.s;
    const unsigned grid = (unsigned)g.ntiles;
    if (!scatter) {
        {
            KtScope kt("gbp_count_kernel", s);
            gbp_count_kernel<PRED, L2, F8, NUL><<<grid, kPsThreads, 0, s>>>(R.pl.p, R.dp, g, in, cnt);
        }
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = scan_exclusive32_inplace(cnt, g.ntiles << g.dbits, part, s);
        return e;
    }
    {
        KtScope kt("gbp_scatter_kernel", s);
        gbp_scatter_kernel<PRED, L2, F8, NUL><<<grid, kPsThreads, 0, s>>>(R.pl.p, R.dp, g, in, cnt, out);
    }
    return hipGetLastError();
}

template <bool NUL>
static hipError_t gbp_pass1_nul(const GbRun& R, bool f8, const PsGeom& g, uint32_t* cnt, uint64_t* part,
                                bool scatter, const PartOut& out) {
    PartOut none;
    std::memset(&none, 0, sizeof none);
    if (f8 && R.pred == 0) return gbp_pass<0, false, true, NUL>(R, g, none, cnt, part, scatter, out);
    if (f8 && R.pred == 1) return gbp_pass<1, false, true, NUL>(R, g, none, cnt, part, scatter, out);
    switch (R.pred) {
    case 0: return gbp_pass<0, false, false, NUL>(R, g, none, cnt, part, scatter, out);
    case 1: return gbp_pass<1, false, false, NUL>(R, g, none, cnt, part, scatter, out);
    default: return gbp_pass<2, false, false, NUL>(R, g, none, cnt, part, scatter, out);
    }
}
static hipError_t gbp_pass1(const GbRun& R, bool f8, bool nul, const PsGeom& g, uint32_t* cnt, uint64_t* part,
                            bool scatter, const PartOut& out) {
    return nul ? gbp_pass1_nul<true>(R, f8, g, cnt, part, scatter, out)
               : gbp_pass1_nul<false>(R, f8, g, cnt, part, scatter, out);
}

// Partition buffers for `rows` selected rows: key, nacc columns, row ids,
// null bits (nul).
static int gbp_alloc(GbRun& R, int64_t sel, bool nul, uint64_t** buf, PartOut* o) {
    const GbParams& p = R.pl.p;
    // a multiple of 16 rows, so every column's buffer starts on a 128-B line
    // (pair loads; the level-2 tiles' aligned block loads)
    const int64_t rows = ((int64_t)std::max<int64_t>(sel, 2) + 17) & ~int64_t(15);
    const bool want_rows = p.f_first >= 0 || p.f_last >= 0;
    const size_t rwords = want_rows ? ((size_t)rows + 1) / 2 : 0;
    const size_t words = (size_t)rows * (1 + p.nacc) + rwords + (nul ? ((size_t)rows + 7) / 8 : 0);
    int rc = dev_alloc((void**)buf, words * 8, R.s);
    if (rc) return rc;
    std::memset(o, 0, sizeof *o);
    o->key = *buf;
    for (int a = 0; a < p.nacc; ++a) o->acc[a] = *buf + (size_t)rows * (1 + a);
    o->rows = want_rows ? (uint32_t*)(*buf + (size_t)rows * (1 + p.nacc)) : nullptr;
    o->nulls = nul ? (uint8_t*)(*buf + (size_t)rows * (1 + p.nacc) + rwords) : nullptr;
    o->cap = rows;
    return PLGPU_OK;
}

static int gb_partition(GbRun& R) {
    GbParams& p = R.pl.p;
    hipStream_t s = R.s;
    // the count / scatter kernels read the key column at every row and copy
    // the key and aggregated columns as raw words: a keyless reduction must
    // never reach them (the plan refuses it; this holds for every caller)
    if (p.key.values == nullptr || p.key.dtype == PLGPU_STR || p.n <= 0 || p.n >= 0xFFFFFFFFll)
        return fail(PLGPU_ERR_INVALID, "partitioned group-by: needs a key column and 1 .. 2^32 - 1 rows");
    for (int a = 0; a < p.nacc; ++a)
        if (p.acc[a].c.values == nullptr)
            return fail(PLGPU_ERR_INVALID, "partitioned group-by: an aggregated column without values");
    const int B = R.pbits;
    const int lv = options().part_levels;
    const bool two = B >= 2 && (B > kPartOneLevel || lv == 2) && !(lv == 1 && B <= kPartOneLevel);
    const int b1 = two ? B / 2 : B, b2 = B - b1;
    const int P1 = 1 << b1, P = 1 << B;
    // the fast forms: 8-byte key, aggregated and predicate columns (plain
    // loads); nul: some of them has a validity bitmap (its bits travel with
    // the rows as the null-bits column)
    auto c8 = [](const DevCol& c) { return dtype_bytes(c.dtype) == 8 && c.dtype != PLGPU_STR; };
    bool f8 = c8(p.key) && R.pred <= 1 && (R.pred == 0 || c8(p.pred_col));
    for (int a = 0; a < p.nacc; ++a) f8 = f8 && c8(p.acc[a].c);
    bool nul = p.key.validity != nullptr || (R.pred == 1 && p.pred_col.validity != nullptr);
    // the count pass reads only the key's and the predicate's bits
    const bool nul_cnt = nul;
    for (int a = 0; a < p.nacc; ++a) nul = nul || p.acc[a].c.validity != nullptr;
    // sum-only accs (every one an f64 sum): the level-1 scatter writes a null
    // value as +0.0, which the exact sum adds as nothing, so the partition
    // buffers carry null bits only for a nullable key (nul_out); other
    // aggregations keep every value's bit
    bool nul_out = R.pl.sum_only ? p.key.validity != nullptr : nul;
    // sum-only with a nullable Int64 key: the level-1 count pass finds the
    // non-null keys' range and a null key is written as a value outside it
    // (GbParams::null_key), so the partition buffers carry no null bits
    const bool want_sent = R.pl.sum_only && p.key.validity != nullptr && p.key.dtype == PLGPU_I64 && f8 &&
                           options().part_null_sentinel != 0;
    PsGeom g1;
    std::memset(&g1, 0, sizeof g1);
    g1.n = p.n;
    g1.ntiles = (p.n + kPsTile - 1) / kPsTile;
    g1.sh = b1 ? 64 - b1 : 0;
    g1.dbits = b1;
    const int64_t ncnt1 = g1.ntiles << b1;
    uint32_t* cnt = nullptr;
    uint64_t* part = nullptr;
    // final bounds (P + 1), then the level-1 bounds (P1 + 1) of a two-pass run
    int rc = dev_alloc((void**)&R.prange, (size_t)(P + 1 + (two ? P1 + 1 : 0)) * 8, s);
    uint64_t* range = R.prange;
    uint64_t* range1 = two ? R.prange + P + 1 : range;
    if (!rc) rc = dev_alloc((void**)&cnt, (size_t)ncnt1 * 4, s);
    // (+ the key range slots of a sentinel run)
    if (!rc)
        rc = dev_alloc((void**)&part, (size_t)((ncnt1 + kScanChunk - 1) / kScanChunk + 2 + 2 * kKeyRangeSlots) * 8,
                       s);
    std::vector<uint64_t> hr1((size_t)P1 + 1);
    std::vector<int64_t> krange(2 * kKeyRangeSlots);
    for (int i = 0; i < kKeyRangeSlots; ++i) krange[2 * i] = INT64_MAX, krange[2 * i + 1] = INT64_MIN;
    if (!rc && want_sent) {
        g1.keyrange = (int64_t*)(part + (ncnt1 + kScanChunk - 1) / kScanChunk + 2);
        if (hipMemcpyAsync(g1.keyrange, krange.data(), krange.size() * 8, hipMemcpyHostToDevice, s) != hipSuccess)
            rc = fail(PLGPU_ERR_HIP, "key range init");
    }
    if (!rc) {
        hipError_t e = gbp_pass1(R, f8, nul_cnt, g1, cnt, part, false, R.pout);
        const int64_t nb = std::max<int64_t>(1, (ncnt1 + kScanChunk - 1) / kScanChunk);
        if (e == hipSuccess) {
            gbp_bounds_kernel<<<(P1 + 256) / 256, 256, 0, s>>>(cnt, part + nb, P1, g1.ntiles, range1);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(hr1.data(), range1, (size_t)(P1 + 1) * 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && g1.keyrange)
            e = hipMemcpyAsync(krange.data(), g1.keyrange, krange.size() * 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "gbp_count_kernel");
    }
    R.has_null_key = false;
    if (!rc && g1.keyrange) {
        // a value outside [min, max] of the non-null keys, never kEmptyKey
        // (INT64_MIN: the key that has a special slot of its own)
        int64_t lo = INT64_MAX, hi = INT64_MIN;
        for (int i = 0; i < kKeyRangeSlots; ++i) lo = std::min(lo, krange[2 * i]), hi = std::max(hi, krange[2 * i + 1]);
        if (lo > hi) R.null_key = 0, R.has_null_key = true;
        else if (hi < INT64_MAX) R.null_key = hi + 1, R.has_null_key = true;
        else if (lo > INT64_MIN + 1) R.null_key = lo - 1, R.has_null_key = true;
        g1.keyrange = nullptr;
        if (R.has_null_key) {
            g1.has_sentinel = 1;
            g1.sentinel = R.null_key;
            nul_out = false;
        }
    }
    uint64_t* buf1 = nullptr;
    PartOut out1;
    if (!rc) rc = gbp_alloc(R, (int64_t)hr1[P1], nul_out, &buf1, &out1);
    if (!rc) {
        const hipError_t e = gbp_pass1(R, f8, nul, g1, cnt, part, true, out1);
        if (e != hipSuccess) rc = hip_fail(e, "gbp_scatter_kernel");
    }
    dev_free(cnt, s);
    dev_free(part, s);
    cnt = nullptr;
    part = nullptr;
    if (rc) {
        dev_free(buf1, s);
        return rc;
    }
    std::vector<uint64_t> hr;
    if (!two) {
        R.pbuf = buf1;
        R.pout = out1;
        hr = hr1;
    } else {
        // level 2: the tiles of each level-1 partition
        std::vector<uint32_t> ts((size_t)P1 + 1);
        uint64_t t = 0;
        for (int q = 0; q < P1; ++q) {
            ts[q] = (uint32_t)t;
            // the aligned blocks this partition's rows touch (ps_tile)
            if (hr1[q + 1] > hr1[q]) t += ((hr1[q + 1] - 1) / kPsTile) - (hr1[q] / kPsTile) + 1;
        }
        ts[P1] = (uint32_t)t;
        PsGeom g2;
        std::memset(&g2, 0, sizeof g2);
        g2.ntiles = (int64_t)t;
        g2.range = range1;
        g2.sh = 64 - B;
        g2.dbits = b2;
        g2.has_sentinel = g1.has_sentinel;
        g2.sentinel = g1.sentinel;
        const int64_t ncnt2 = g2.ntiles << b2;
        uint32_t* meta = nullptr;
        rc = dev_alloc((void**)&meta, (size_t)(P1 + 1 + std::max<int64_t>(g2.ntiles, 1)) * 4, s);
        if (!rc) rc = dev_alloc((void**)&cnt, (size_t)std::max<int64_t>(ncnt2, 1) * 4, s);
        if (!rc) rc = dev_alloc((void**)&part, (size_t)((ncnt2 + kScanChunk - 1) / kScanChunk + 2) * 8, s);
        hr.resize((size_t)P + 1);
        if (!rc) {
            g2.tstart = meta;
            g2.tpart = meta + P1 + 1;
            hipError_t e = hipMemcpyAsync(meta, ts.data(), ts.size() * 4, hipMemcpyHostToDevice, s);
            if (e == hipSuccess && g2.ntiles > 0) {
                gbp_tpart_kernel<<<(unsigned)std::min<int64_t>((g2.ntiles + 255) / 256, 4096), 256, 0, s>>>(
                    meta, P1, g2.ntiles, meta + P1 + 1);
                e = hipGetLastError();
            }
            if (e == hipSuccess && g2.ntiles > 0)
                e = nul_out ? gbp_pass<0, true, true, true>(R, g2, out1, cnt, part, false, out1)
                            : gbp_pass<0, true, true>(R, g2, out1, cnt, part, false, out1);
            if (e == hipSuccess) {
                gbp_bounds2_kernel<<<(P + 256) / 256, 256, 0, s>>>(cnt, range1, meta, P1, b2, range);
                e = hipGetLastError();
            }
            if (e == hipSuccess) e = hipMemcpyAsync(hr.data(), range, (size_t)(P + 1) * 8, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) rc = hip_fail(e, "gbp_count_kernel (level 2)");
        }
        if (!rc) rc = gbp_alloc(R, (int64_t)hr[P], nul_out, &R.pbuf, &R.pout);
        if (!rc && g2.ntiles > 0) {
            const hipError_t e = nul_out ? gbp_pass<0, true, true, true>(R, g2, out1, cnt, part, true, R.pout)
                                         : gbp_pass<0, true, true>(R, g2, out1, cnt, part, true, R.pout);
            if (e != hipSuccess) rc = hip_fail(e, "gbp_scatter_kernel (level 2)");
        }
        dev_free(cnt, s);
        dev_free(part, s);
        dev_free(meta, s);
        dev_free(buf1, s);
        if (rc) return rc;
    }
    uint64_t maxpart = 0;
    for (int q = 0; q < P; ++q) maxpart = std::max<uint64_t>(maxpart, hr[q + 1] - hr[q]);
    R.part_hrange = hr;
    R.part_rows_total = (int64_t)hr[P];
    R.part_range = range;
    R.part_levels = two ? 2 : 1;
    // workgroups per partition: fill the chip (4 per CU over all partitions,
    // profiles/r02_ab_part.log), bound rows per workgroup
    const int64_t wpc = 4;
    int nb = (int)std::max<int64_t>(1, (wpc * (int64_t)num_cus() + P - 1) / P);
    while ((int64_t)maxpart > (int64_t)nb * (kMaxRowsPerWg / 2)) nb *= 2;
    R.part_blocks = nb;
    // one workgroup per partition: its groups get a region of the global
    // table that it fills slot for slot from its LDS table (plain stores,
    // no probing, no atomics), 2^(pbits + lbits) slots in all
    if (nb == 1 && options().part_direct != 0) {
        R.rbits = R.part_lbits;
        R.gbits = R.pbits + R.part_lbits;
    }
    return PLGPU_OK;
}

// The partition passes of the many-groups path, reused by the join's
// partitioned probe (join.hip jn_radix_take): every row selected, the key
// and up to kMaxAcc carried columns scattered as raw 8-byte words.
int radix_partition8(const DevCol& key, const DevCol* cols, int ncols, int64_t n, int bits, hipStream_t s,
                     RadixParts* out) {
    if (ncols < 0 || ncols > kMaxAcc || bits < 0 || bits > kPartMaxBits || n <= 0 || n >= 0xFFFFFFFFll)
        return fail(PLGPU_ERR_INVALID, "radix partition: 0..6 columns, 0..16 bits, 1 .. 2^32 - 1 rows");
    auto c8 = [](const DevCol& c) {
        return c.values != nullptr && c.validity == nullptr && dtype_bytes(c.dtype) == 8 && c.dtype != PLGPU_STR;
    };
    if (!c8(key)) return fail(PLGPU_ERR_INVALID, "radix partition: null-free 8-byte columns");
    for (int i = 0; i < ncols; ++i)
        if (!c8(cols[i])) return fail(PLGPU_ERR_INVALID, "radix partition: null-free 8-byte columns");
    GbRun R;
    R.s = s;
    GbParams& p = R.pl.p;
    std::memset(&p, 0, sizeof p);
    p.key = key;
    p.n = n;
    p.nacc = ncols;
    for (int i = 0; i < ncols; ++i) p.acc[i].c = cols[i];
    p.pred_acc = -1;
    p.f_first = p.f_last = -1;
    R.pred = 0;
    R.pbits = bits;
    const int rc = gb_partition(R);
    if (rc) return rc;
    out->buf = R.pbuf;
    out->key = R.pout.key;
    for (int i = 0; i < ncols; ++i) out->col[i] = R.pout.acc[i];
    out->range = R.prange;
    out->bounds = R.part_range;
    out->hrange = R.part_hrange;
    out->levels = R.part_levels;
    R.pbuf = nullptr;  // owned by the caller now
    R.prange = nullptr;
    return PLGPU_OK;
}

// The main pass over the partition buffers.
static hipError_t launch_partitioned(const GbRun& R) {
    Plan pp = R.pl;
    GbParams& q = pp.p;
    const GbParams& p = R.pl.p;
    std::memset(&q.key, 0, sizeof q.key);
    q.key.values = R.pout.key;
    q.key.dtype = PLGPU_I64;
    for (int a = 0; a < p.nacc; ++a) {
        DevCol c;
        std::memset(&c, 0, sizeof c);
        c.values = R.pout.acc[a];
        c.dtype = p.acc[a].isf ? PLGPU_F64 : PLGPU_I64;
        q.acc[a].c = c;
    }
    q.n = R.part_rows_total;
    q.row_begin = 0;
    q.n_full = 0;
    q.part_range = R.part_range;
    // (compact regions: p's rtab / rcap / region_cnt and the overflow table
    // from gb_alloc_table)
    q.part_rows = R.pout.rows;
    q.part_nulls = R.pout.nulls;
    q.has_null_key = R.has_null_key ? 1 : 0;
    q.null_key = R.null_key;
    q.part_blocks = R.part_blocks;
    q.lbits = R.part_lbits;
    q.lcap = 1 << R.part_lbits;
    if (pp.sum_only && p.nacc >= 1 && p.nacc <= 6) {
        // sum-only accs: the fast kernel over the partition buffers (the
        // slim layout on the 2-limb window)
        const int grid = (1 << R.pbits) * R.part_blocks;
        switch (p.nacc) {
        case 1: return launch_part_fast_limbs<1>(pp, grid, R.s);
        case 2: return launch_part_fast_limbs<2>(pp, grid, R.s);
        case 3: return launch_part_fast_limbs<3>(pp, grid, R.s);
        case 4: return launch_part_fast_limbs<4>(pp, grid, R.s);
        case 5: return launch_part_fast_limbs<5>(pp, grid, R.s);
        default: return launch_part_fast_limbs<6>(pp, grid, R.s);
        }
    }
    const size_t lds = (size_t)p.nfields * (q.lcap + 2) * 8;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)gb_kernel<0, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr_set = true;
    }
    DevProgram none;
    std::memset(&none, 0, sizeof none);
    gb_kernel<0, true, true><<<(1 << R.pbits) * R.part_blocks, kGbThreads, lds, R.s>>>(q, none);
    return hipGetLastError();
}

static int gb_alloc_table(GbRun& R) {
    GbParams& p = R.pl.p;
    dev_free(R.gtab, R.s);
    dev_free(R.rtab, R.s);
    R.gtab = nullptr;
    R.rtab = nullptr;
    p.rtab = nullptr;
    p.rcap = 0;
    p.region_cnt = nullptr;
    p.gbits = R.gbits;
    p.rbits = R.rbits;
    if (R.compact_now) {
        // compact regions: the region table (2^(pbits + lbits) slots, written
        // whole where read, never initialised) and a small hashed overflow
        // table (plain probing) for the keys that find no LDS slot
        p.rcap = int64_t(1) << (R.pbits + R.part_lbits);
        int rc = dev_alloc((void**)&R.rtab, (size_t)p.rcap * p.nfields * 8, R.s);
        if (rc) return rc;
        p.rtab = R.rtab;
        p.region_cnt = R.region_cnt;
        p.gbits = std::max(16, R.pbits + 2);
        p.rbits = 0;
    }
    p.gcap = int64_t(1) << p.gbits;
    const size_t wpf = (size_t)(p.gcap + 2);
    int rc = dev_alloc((void**)&R.gtab, wpf * p.nfields * 8, R.s);
    if (rc) return rc;
    p.gtab = R.gtab;
    const int ig = (int)std::min<int64_t>((int64_t)(wpf + 255) / 256, 256 * 8);
    gb_init_table_kernel<<<ig, 256, 0, R.s>>>(R.gtab, (int64_t)wpf, p.nfields, p.min_init_mask);
    // keep the plan words (distinct / sampled), clear the run words
    PLGPU_HIP(hipMemsetAsync(R.status, 0, 6 * 8, R.s));
    PLGPU_HIP(hipMemsetAsync(R.status + ST_MAXEX, 0, (ST_WORDS - ST_MAXEX) * 8, R.s));
    PLGPU_HIP(hipGetLastError());
    return PLGPU_OK;
}

// Exact max exponents of the flagged accs -> refit bottoms in `hint`.
// Returns true when some window changes.
static int gb_refit(GbRun& R, uint32_t flagged, int32_t* hint, bool* changed, uint32_t* wide) {
    GbParams& p = R.pl.p;
    *changed = false;
    *wide = 0;
    for (int a = 0; a < kMaxAcc; ++a) hint[a] = R.hb[a];
    if (!flagged) return PLGPU_OK;
    for (int a = 0; a < p.nacc; ++a)
        if ((flagged >> a) & 1u) gb_maxexp_kernel<<<std::max(1, num_cus() * 4), 256, 0, R.s>>>(p, a);
    PLGPU_HIP(hipGetLastError());
    if (int rs = d2h_status(R)) return rs;
    for (int a = 0; a < p.nacc; ++a) {
        if (!((flagged >> a) & 1u)) continue;
        const int tmax = std::max((int)R.st[ST_MAXEX + a], 1);
        const int tmin = std::max(0x7FF - (int)R.st[ST_MINEX + a], 1);
        if (tmax - tmin <= kSumWindowBits - 53) {
            // one window holds every value exactly: put its top at the max
            hint[a] = tmax - 1075 - (kSumWindowBits - 53);
            *changed = *changed || hint[a] != R.hb[a];
        } else {
            // wider than a window: exact big-integer pass for this column
            *wide |= 1u << a;
            R.wide_exmin[a] = std::min(tmin, tmax);
            R.wide_exmax[a] = tmax;
        }
    }
    return PLGPU_OK;
}

// Exact wide sums for the accs in R.wide (see gb_wide_kernel): the digit
// pass over the rows, then (round) the rounding into R.wide_sum, which
// normalises the digits in place.  Multi-GPU partial states export the
// digits unrounded (round = false).
static int gb_wide(GbRun& R, bool round = true) {
    GbParams& p = R.pl.p;
    for (int a = 0; a < p.nacc; ++a) {
        if (!((R.wide >> a) & 1u)) continue;
        dev_free(R.wide_digits[a], R.s);
        dev_free(R.wide_sum[a], R.s);
        R.wide_digits[a] = nullptr;
        R.wide_sum[a] = nullptr;
        const int exmin = R.wide_exmin[a];
        const int nwords = wide_nwords(exmin, R.wide_exmax[a]);
        const size_t slots = (size_t)(p.gcap + 2);
        int rc = dev_alloc((void**)&R.wide_digits[a], slots * nwords * 8, R.s);
        if (!rc && round) rc = dev_alloc((void**)&R.wide_sum[a], slots * 8, R.s);
        if (rc) return rc;
        PLGPU_HIP(hipMemsetAsync(R.wide_digits[a], 0, slots * nwords * 8, R.s));
        const int g = std::max(1, num_cus() * 8);
        if (R.pred == 0) gb_wide_kernel<0><<<g, 256, 0, R.s>>>(p, R.dp, a, exmin, nwords, R.wide_digits[a]);
        else if (R.pred == 1) gb_wide_kernel<1><<<g, 256, 0, R.s>>>(p, R.dp, a, exmin, nwords, R.wide_digits[a]);
        else gb_wide_kernel<2><<<g, 256, 0, R.s>>>(p, R.dp, a, exmin, nwords, R.wide_digits[a]);
        if (round) {
            const int fg = (int)std::min<int64_t>((p.gcap + 2 + 255) / 256, 256 * 16);
            gb_wide_round_kernel<<<fg, 256, 0, R.s>>>(p, exmin, nwords, R.wide_digits[a], R.wide_sum[a]);
        }
        PLGPU_HIP(hipGetLastError());
    }
    return PLGPU_OK;
}

// The record layout's wide part for the accs in R.wide over R.wide_exmin /
// exmax; returns the record's words.
static int wide_layout(const GbRun& R, WideRec& wr) {
    std::memset(&wr, 0, sizeof wr);
    int w = R.pl.p.nfields + 1;
    for (int a = 0; a < R.pl.p.nacc; ++a) {
        if (!((R.wide >> a) & 1u)) continue;
        wr.acc[wr.n] = a;
        wr.nwords[wr.n] = wide_nwords(R.wide_exmin[a], R.wide_exmax[a]);
        wr.off[wr.n] = w;
        wr.digits[wr.n] = R.wide_digits[a];
        w += wr.nwords[wr.n];
        ++wr.n;
    }
    return w;
}

// Main launches with table-size reruns; window refits too when auto_refit.
// Without auto_refit a needed refit is reported in *refit / hint.
static int gb_main(GbRun& R, bool auto_refit, bool* refit, int32_t* hint) {
    Plan& pl = R.pl;
    GbParams& p = pl.p;
    const int64_t n = p.n;
    const bool debug = options().debug != 0;
    if (refit) *refit = false;
    hipEvent_t ev0 = ev_acquire(), ev1 = ev_acquire();
    if (ev0 == nullptr || ev1 == nullptr) {
        ev_release(ev0);
        ev_release(ev1);
        return fail(PLGPU_ERR_HIP, "hipEventCreate failed");
    }
    int rc = PLGPU_OK;
    if (R.part && n > 0 && R.pbuf == nullptr) rc = gb_partition(R);
    for (R.attempts = 0; rc == PLGPU_OK; ++R.attempts) {
        R.compact_now = R.compact_ok && R.part && n > 0 && pl.sum_only && pl.limbs == 2 && R.rbits > 0 &&
                        R.part_blocks == 1 && R.wide == 0 && options().part_compact != 0;
        if (R.compact_now && R.region_cnt == nullptr &&
            (rc = dev_alloc((void**)&R.region_cnt, ((size_t)1 << R.pbits) * 4, R.s)))
            break;
        if ((rc = gb_alloc_table(R))) break;
        PLGPU_HIP(hipMemcpyAsync(R.bottoms, R.hb, sizeof R.hb, hipMemcpyHostToDevice, R.s));
        for (int a = 0; a < kMaxAcc; ++a) p.bottom[a] = R.hb[a];
        PLGPU_HIP(hipEventRecord(ev0, R.s));
        if (n > 0 && R.part) {
            KtScope kt("gb_part_agg_kernel", R.s);
            PLGPU_HIP(launch_partitioned(R));
        } else if (n > 0) {
            // the fused kernel covers every row (its last tile masked); off
            // the fast path, or below one tile, the generic kernel does
            if (p.n_full > 0) {
                PLGPU_HIP(launch_fast_dispatch(pl, R.dp, R.pred, R.s));
            } else {
                PLGPU_HIP(launch_main_dispatch(pl, R.dp, R.pred, R.s));
            }
        }
        PLGPU_HIP(hipEventRecord(ev1, R.s));
        if (int rs = d2h_status(R)) return rs;
        if (debug) {
            fprintf(stderr,
                    "[plgpu] gb attempt %d: n=%lld grid=%d/%d lds=%d lcap=%d gcap=%lld nfields=%d lds_bytes=%zu "
                    "fast=%lld sumonly=%d distinct=%llu/%llu newkeys=%llu special=%llu global_rows=%llu full=%llu "
                    "selected=%llu fx=%llx limbs=%d runs=%d nacc=%d\n",
                    R.attempts, (long long)n, pl.grid, pl.fast_grid, (int)pl.use_lds, p.lcap, (long long)p.gcap,
                    p.nfields, pl.lds_bytes, (long long)p.n_full, (int)pl.sum_only,
                    (unsigned long long)R.st[ST_DISTINCT], (unsigned long long)R.st[ST_SAMPLED],
                    (unsigned long long)R.st[ST_NEWKEYS], (unsigned long long)R.st[ST_SPECIAL],
                    (unsigned long long)R.st[ST_GLOBAL_ROWS], (unsigned long long)R.st[ST_TABLE_FULL],
                    (unsigned long long)R.st[ST_SELECTED], (unsigned long long)R.st[ST_FXFLAGS], pl.limbs, (int)pl.runs,
                    p.nacc);
        }
        if (R.st[ST_KPACK]) {
            // a selected row's key left the sampled packing plan: the caller
            // repacks with the exact ranges (this pass's result is dropped)
            R.kp_bad = true;
            break;
        }
        bool again = false;
        if (R.st[ST_TABLE_FULL] > 0 && R.compact_now) {
            // the compact run's overflow table filled: rerun on the probed
            // regions of the whole table
            R.compact_ok = false;
            again = true;
        } else if (R.st[ST_TABLE_FULL] > 0) {
            // (a full partition region: the rerun takes the plain hashed table)
            R.rbits = 0;
            R.gbits = std::max(R.gbits + 3, log2_ceil((int64_t)R.st[ST_NEWKEYS] * 4));
            if (R.attempts == 0 && p.key.values != nullptr && p.kp.n == 0) {
                // the plan's estimate was far off (stale plan statistics, a
                // skewed sample): count the key column's distinct values once
                // so the next table holds them all
                int64_t hll = 0;
                if ((rc = gb_hll_count(R, &hll))) break;
                R.gbits = std::max(R.gbits, log2_ceil(std::min<int64_t>(n, hll + hll / 4 + 1024) * 2));
            }
            again = true;
        }
        uint32_t flagged = 0;
        for (int a = 0; a < p.nacc; ++a)
            if ((p.acc[a].flags & (A_FSUM | A_FSUMCAST)) && ((R.st[ST_FXFLAGS] >> (2 * a)) & 3u)) flagged |= 1u << a;
        flagged &= ~R.wide;
        if (flagged && pl.limbs == 2 && (p.n_full > 0 || R.part) && pl.sum_only) {
            // a value fell below the 2-limb window (or out of the top): redo
            // the pass with the full 3-limb window before any refit
            pl.limbs = 3;
            again = true;
            uint32_t over = 0;
            for (int a = 0; a < p.nacc; ++a)
                if ((R.st[ST_FXFLAGS] >> (2 * a)) & 1u) over |= 1u << a;
            flagged = over;
        }
        if (flagged) {
            int32_t h[kMaxAcc];
            bool changed = false;
            uint32_t wide = 0;
            if ((rc = gb_refit(R, flagged, h, &changed, &wide))) break;
            if (wide && !auto_refit) {
                rc = fail(PLGPU_ERR_CAPACITY,
                          "f64 sum: the values of one column span more binades than the partitioned "
                          "group-by's fixed-point window; use the single-GPU group-by for this column");
                break;
            }
            R.wide |= wide;
            // the wide pass finds each row's slot by probing: no compact regions
            if (wide && R.compact_now) again = true;
            if (changed) {
                if (auto_refit) {
                    for (int a = 0; a < kMaxAcc; ++a)
                        if (!((R.wide >> a) & 1u)) R.hb[a] = h[a];
                    again = true;
                } else {
                    if (refit) *refit = true;
                    if (hint)
                        for (int a = 0; a < kMaxAcc; ++a) hint[a] = h[a];
                }
            }
        }
        if (!again) break;
        if (R.attempts >= 3) {
            rc = fail(PLGPU_ERR_CAPACITY, "group-by did not converge after retries");
            break;
        }
    }
    if (rc == PLGPU_OK) (void)hipEventElapsedTime(&R.ms, ev0, ev1);
    ev_release(ev0);
    ev_release(ev1);
    // cached statistics the run contradicted (a table-size or window rerun,
    // or several times the estimated groups: the columns' addresses now hold
    // other data) are dropped, so the next query samples afresh
    if (!R.plan_ckey.empty() &&
        (rc != PLGPU_OK || R.attempts > 0 || R.kp_bad ||
         (int64_t)R.st[ST_NEWKEYS] > 2 * std::max<int64_t>(R.est_groups, 4096)))
        plan_cache_erase(R.plan_ckey);
    if (rc == PLGPU_OK && R.wide && !R.kp_bad) rc = gb_wide(R, R.wide_round);
    return rc;
}

static int64_t gb_groups(const GbRun& R) {
    return (int64_t)R.st[ST_NEWKEYS] + ((R.st[ST_SPECIAL] & 1) ? 1 : 0) + ((R.st[ST_SPECIAL] & 2) ? 1 : 0);
}

static void gb_fill_info(const GbRun& R, plgpu_groupby_info* info) {
    const GbParams& p = R.pl.p;
    std::memset(info, 0, sizeof *info);
    info->rows_in = p.n;
    info->rows_selected = (int64_t)R.st[ST_SELECTED];
    info->groups = gb_groups(R);
    info->global_path_rows = (int64_t)R.st[ST_GLOBAL_ROWS];
    info->reruns = R.attempts;
    info->lds_slots = R.pl.use_lds ? p.lcap : 0;
    info->grid = p.n_full > 0 ? R.pl.launched_grid : R.pl.grid;
    info->table_capacity = p.gcap;
    info->main_kernel_ms = R.ms;
    info->path = R.part ? 3 : (p.n_full > 0 ? (R.pl.launched_var ? 4 : (R.pl.sum_only ? 2 : 1)) : 0);
    info->sum_limbs = (p.n_full > 0 || R.part) && R.pl.sum_only ? R.pl.limbs : 3;
    info->local_range = R.pl.local ? 1 : 0;
    info->register_runs = p.n_full > 0 && !R.part && R.pl.launched_runs ? 1 : 0;
    info->key_pack = p.kp.n;
    info->part_layout = R.part ? (R.pbits | (R.part_levels << 8)) : 0;
    for (int a = 0; a < p.nacc; ++a)
        if (((R.st[ST_FXFLAGS] >> (2 * a)) & 2u) && !((R.wide >> a) & 1u)) info->sum_inexact |= 1 << a;
}

// Global table -> output columns (+ first-occurrence order, key narrowing).
// `keep_first` (R.want_first): receives each output group's first selected
// row, in output order (device buffer, caller frees).
static int gb_finalize(GbRun& R, int32_t naggs, plgpu_column* out_key, plgpu_column* out_aggs,
                       uint64_t** keep_first = nullptr) {
    Plan& pl = R.pl;
    GbParams& p = pl.p;
    hipStream_t s = R.s;
    const int64_t groups = gb_groups(R);
    FinParams fp;
    std::memset(&fp, 0, sizeof fp);
    int rc = make_owned_column(out_key, PLGPU_I64, groups, true, s);
    for (int i = 0; i < naggs && rc == PLGPU_OK; ++i) {
        const OutSpec& o = pl.outs[i];
        const bool nullable = o.kind == PLGPU_AGG_MEAN || o.kind == PLGPU_AGG_MIN || o.kind == PLGPU_AGG_MAX ||
                              o.kind == PLGPU_AGG_FIRST || o.kind == PLGPU_AGG_LAST || o.kind == PLGPU_AGG_VAR ||
                              o.kind == PLGPU_AGG_STD;
        if (o.kind == PLGPU_AGG_VAR || o.kind == PLGPU_AGG_STD) {
            // exactness of the fused second moment: no wide (multi-window)
            // sum among its three, and |x| >= 2^-484 for every nonzero x
            // (the window bottom), so x * x splits exactly into h + l
            const bool wide = ((R.wide >> o.acc) | (R.wide >> o.acc_hi) | (R.wide >> o.acc_lo)) & 1u;
            if (wide || R.hb[o.acc] < -484)
                rc = fail(PLGPU_ERR_CAPACITY, "var: the fused second moment is out of its exact range");
        }
        if (rc == PLGPU_OK) rc = make_owned_column(&out_aggs[i], o.out_dtype, groups, nullable, s);
    }
    uint64_t* first = nullptr;
    if (rc == PLGPU_OK && (R.maintain || keep_first) && groups > 0) rc = dev_alloc((void**)&first, groups * 8, s);
    if (rc == PLGPU_OK && groups > 0) {
        fp.nout = naggs;
        for (int i = 0; i < naggs; ++i) {
            fp.out[i] = pl.outs[i];
            fp.out[i].values = (void*)out_aggs[i].values;
            fp.out[i].validity = (uint32_t*)out_aggs[i].validity;
        }
        fp.out_keys = (int64_t*)out_key->values;
        fp.out_key_valid = (uint32_t*)out_key->validity;
        fp.out_first = first;
        fp.cap = groups;
        for (int a = 0; a < kMaxAcc; ++a) fp.wide[a] = R.wide_sum[a];
        uint8_t* vbytes = nullptr;
        rc = dev_alloc((void**)&vbytes, (size_t)(1 + naggs) * groups, s);
        if (rc) {
            dev_free(first, s);
            plgpu_column_release(out_key);
            for (int i = 0; i < naggs; ++i) plgpu_column_release(&out_aggs[i]);
            return rc;
        }
        fp.vbytes = vbytes;
        const int fg = (int)std::min<int64_t>((p.gcap + 2 + 255) / 256, 256 * 16);
        uint64_t* roff = nullptr;  // compact regions: scan of the region counts + scratch
        const int nreg = R.compact_now ? 1 << R.pbits : 0;
        if (nreg) {
            const int64_t nb = std::max<int64_t>(1, (nreg + kScanChunk - 1) / kScanChunk);
            rc = dev_alloc((void**)&roff, (size_t)(nreg + 1 + nb + 2) * 8, s);
            if (!rc && scan_exclusive<uint32_t>(R.region_cnt, nreg, roff, roff + nreg + 1, s) != hipSuccess)
                rc = fail(PLGPU_ERR_HIP, "region count scan");
            if (rc) {
                dev_free(roff, s);
                dev_free(vbytes, s);
                dev_free(first, s);
                plgpu_column_release(out_key);
                for (int i = 0; i < naggs; ++i) plgpu_column_release(&out_aggs[i]);
                return rc;
            }
        }
        {
            KtScope kt("gb_finalize_kernel", s);
            // compact regions: the regions first, then the overflow table
            // (its groups and the two special ones) after them
            if (nreg) gb_finalize_regions_kernel<<<nreg, 256, 0, s>>>(p, fp, roff, R.part_lbits);
            gb_finalize_kernel<<<fg, 256, 0, s>>>(p, fp);
            PackValid pv;
            std::memset(&pv, 0, sizeof pv);
            pv.n = 1 + naggs;
            pv.dst[0] = (uint32_t*)out_key->validity;
            for (int i = 0; i < naggs; ++i) pv.dst[1 + i] = (uint32_t*)out_aggs[i].validity;
            const int64_t work = ((groups + 63) / 64) * 2 * pv.n;
            gb_pack_valid_kernel<<<(unsigned)std::min<int64_t>((work + 255) / 256, 4096), 256, 0, s>>>(vbytes, groups,
                                                                                                       pv);
        }
        dev_free(vbytes, s);
        dev_free(roff, s);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) rc = hip_fail(e, "gb_finalize_kernel");
        uint64_t produced = 0, var_out = 0;
        if (rc == PLGPU_OK) {
            void* d[2] = {&produced, &var_out};
            const void* src[2] = {R.status + ST_GROUPS_OUT, R.status + ST_VAR_OUT};
            const size_t b[2] = {8, 8};
            rc = d2h_stage(2, d, src, b, s);
        }
        if (rc == PLGPU_OK && var_out)
            rc = fail(PLGPU_ERR_CAPACITY, "var: the fused second moment is out of its exact range");
        if (rc == PLGPU_OK && (int64_t)produced != groups) {
            char buf[256];
            snprintf(buf, sizeof buf,
                     "internal: group count mismatch (inserted %llu + specials %llu, finalized %llu, "
                     "global rows %llu, table_full %llu)",
                     (unsigned long long)R.st[ST_NEWKEYS], (unsigned long long)R.st[ST_SPECIAL],
                     (unsigned long long)produced, (unsigned long long)R.st[ST_GLOBAL_ROWS],
                     (unsigned long long)R.st[ST_TABLE_FULL]);
            rc = fail(PLGPU_ERR_CAPACITY, buf);
        }
    }
    if (rc == PLGPU_OK && R.maintain && groups > 1) {
        // order groups by first occurrence: a stable radix arg_sort of the
        // groups' first rows on the device (sort.hip), then every output
        // column gathered by it
        plgpu_column fc, pidx;
        std::memset(&fc, 0, sizeof fc);
        std::memset(&pidx, 0, sizeof pidx);
        fc.dtype = PLGPU_I64;
        fc.length = groups;
        fc.values = first;
        rc = plgpu_arg_sort(&fc, 0, 0, &pidx, s);
        int64_t* dperm = nullptr;
        if (rc == PLGPU_OK) rc = dev_alloc((void**)&dperm, groups * 8, s);
        if (rc == PLGPU_OK) {
            const int gg = (int)std::min<int64_t>((groups + 255) / 256, 4096);
            widen_u32_kernel<<<gg, 256, 0, s>>>((const uint32_t*)pidx.values, dperm, groups);
            auto permute = [&](plgpu_column* c) -> int {
                plgpu_column nc;
                int r2 = make_owned_column(&nc, c->dtype, groups, c->validity != nullptr, s);
                if (r2) return r2;
                switch (dtype_bytes(c->dtype)) {
                case 8:
                    gather_kernel<uint64_t><<<gg, 256, 0, s>>>((const uint64_t*)c->values, dperm,
                                                               (uint64_t*)nc.values, groups);
                    break;
                case 4:
                    gather_kernel<uint32_t><<<gg, 256, 0, s>>>((const uint32_t*)c->values, dperm,
                                                               (uint32_t*)nc.values, groups);
                    break;
                case 2:
                    gather_kernel<uint16_t><<<gg, 256, 0, s>>>((const uint16_t*)c->values, dperm,
                                                               (uint16_t*)nc.values, groups);
                    break;
                case 1:
                    gather_kernel<uint8_t><<<gg, 256, 0, s>>>((const uint8_t*)c->values, dperm,
                                                              (uint8_t*)nc.values, groups);
                    break;
                default:
                    plgpu_column_release(&nc);
                    return fail(PLGPU_ERR_SCHEMA, "group order: unsupported output dtype");
                }
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
            if (rc == PLGPU_OK && keep_first) {
                // first rows in output order
                uint64_t* sf = nullptr;
                rc = dev_alloc((void**)&sf, groups * 8, s);
                if (rc == PLGPU_OK) {
                    gather_kernel<uint64_t><<<gg, 256, 0, s>>>(first, dperm, sf, groups);
                    dev_free(first, s);
                    first = sf;
                }
            }
            hipError_t e = hipGetLastError();
            if (rc == PLGPU_OK && e != hipSuccess) rc = hip_fail(e, "permute");
        }
        dev_free(dperm, s);
        plgpu_column_release(&pidx);
    }
    if (rc == PLGPU_OK && R.key_dtype != PLGPU_I64 && dtype_bytes(R.key_dtype) > 0) {
        // the key back in its own dtype (the reference keeps the key dtype)
        plgpu_column nk;
        rc = make_owned_column(&nk, R.key_dtype, groups, true, s);
        if (rc == PLGPU_OK && groups > 0) {
            const int gg = (int)std::min<int64_t>((groups + 255) / 256, 4096);
            narrow_i64_kernel<<<gg, 256, 0, s>>>((const int64_t*)out_key->values, (void*)nk.values, R.key_dtype,
                                                 groups);
            (void)hipMemcpyAsync((void*)nk.validity, out_key->validity, ((groups + 63) / 64) * 8,
                                 hipMemcpyDeviceToDevice, s);
        }
        if (rc == PLGPU_OK) {
            plgpu_column_release(out_key);
            *out_key = nk;
        }
    }
    if (rc == PLGPU_OK) {
        out_key->null_count = (R.st[ST_SPECIAL] & 1) ? 1 : 0;
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "finalize sync");
    }
    if (rc == PLGPU_OK && keep_first) {
        *keep_first = first;
        first = nullptr;
    }
    dev_free(first, s);
    if (rc) {
        plgpu_column_release(out_key);
        for (int i = 0; i < naggs; ++i) plgpu_column_release(&out_aggs[i]);
    }
    return rc;
}

// ------------------------------------------------------ multi-key group-by
// The reference groups several key columns by row-encoding them
// (polars-core/src/frame/group_by/mod.rs:91 encode_rows_vertical_par_unordered
// -> chunked_array/ops/row_encode.rs:11) and grouping the encoded rows:
// tuple equality, a null distinct from every value.  Here each row's tuple is
// hashed to 64 bits in one pass, the single-key kernels group the hashes
// (keeping each group's first row), and a verify pass checks every row's
// tuple against its group's first row; a collision re-runs with a new seed.
__global__ void mk_hash_kernel(MkKeys k, int64_t n, uint64_t seed, uint64_t mask, uint64_t* __restrict__ out) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        out[r] = mk_row_hash(k, r, seed) & mask;
    }
}

// Read-only probe of the global table: slot of `key`, or -1.
__device__ __forceinline__ int64_t g_lookup(const GbParams& p, uint64_t key) {
    if (key == kEmptyKey) return p.gcap + 1;
    const int lim = g_probe_limit(p);
    for (int i = 0; i < lim; ++i) {
        const uint64_t s = g_slot(p, key, (uint64_t)i);
        const uint64_t k = p.gtab[s];
        if (k == key) return (int64_t)s;
        if (k == kEmptyKey) return -1;
    }
    return -1;
}

// Every group's representative tuple (its first row), slot-aligned with the
// table: vw[i * (gcap + 2) + s] = canonical word of key i (0 for a null),
// vm[s] = validity bits.  The verify pass then reads these L2-resident
// arrays instead of the representative rows themselves.
__global__ __launch_bounds__(256) void mk_rep_kernel(GbParams p, MkKeys k, uint64_t* __restrict__ vw,
                                                     uint32_t* __restrict__ vm) {
    const int64_t total = p.gcap + 2;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < total; s += (int64_t)gridDim.x * blockDim.x) {
        if (*gfield(p, p.f_len, s) == 0) continue;
        const int64_t rep = (int64_t)*gfield(p, p.f_first, s);
        if (!gb_ok(rep >= 0 && rep < p.n, CK_REP_ROW)) continue;
        uint32_t m = 0;
        for (int i = 0; i < k.n; ++i) {
            const bool v = dev_valid(k.c[i], rep);
            m |= (v ? 1u : 0u) << i;
            vw[(int64_t)i * total + s] = v ? mk_word(k.c[i], rep) : 0ull;
        }
        vm[s] = m;
    }
}

// Every row whose hash names a group must hold that group's tuple.  (Rows the
// predicate dropped are checked too: a differing tuple there is a genuine
// 64-bit collision as well, and only costs a re-run.)
__global__ __launch_bounds__(256) void mk_verify_kernel(GbParams p, MkKeys k, const uint64_t* __restrict__ hashes,
                                                        int64_t n, const uint64_t* __restrict__ vw,
                                                        const uint32_t* __restrict__ vm,
                                                        uint32_t* __restrict__ collision) {
    const int64_t total = p.gcap + 2;
    bool bad = false;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = g_lookup(p, hashes[r]);
        if (s < 0 || !gb_ok(s < total, CK_VERIFY_SLOT) || *gfield(p, p.f_len, s) == 0) continue;
        const uint32_t m = vm[s];
        for (int i = 0; i < k.n; ++i) {
            const bool v = dev_valid(k.c[i], r);
            bad |= v != (bool)((m >> i) & 1u);
            if (!v) continue;
            if (k.c[i].dtype == PLGPU_STR)  // bytes against the group's first row
                bad |= !str_equal(k.c[i], r, k.c[i], (int64_t)*gfield(p, p.f_first, s));
            else
                bad |= mk_word(k.c[i], r) != vw[(int64_t)i * total + s];
        }
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(collision, 1u);
}

// out[g] = key column c at row rows[g] (validity bit-packed, zeroed first).
__global__ void mk_gather_key_kernel(DevCol c, const uint64_t* __restrict__ rows, int64_t g_n, int64_t n, void* out,
                                     uint32_t* out_valid) {
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < g_n; g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = (int64_t)rows[g];
        if (!gb_ok(r >= 0 && r < n, CK_KEY_ROW)) continue;
        const bool v = dev_valid(c, r);
        const uint64_t x = dev_load(c, r);
        if (c.dtype == PLGPU_BOOL) {
            if (x & 1) atomicOr(&((uint32_t*)out)[g >> 5], 1u << (g & 31));
        } else {
            dev_store(out, c.dtype, g, x);
        }
        if (out_valid && v) atomicOr(&out_valid[g >> 5], 1u << (g & 31));
    }
}

}  // namespace plgpu

using namespace plgpu;

static int gb_single_impl(const plgpu_column* key, const plgpu_column* cols, int32_t ncols, const Deriv* deriv,
                          const plgpu_instr* program, int32_t n_instr, const plgpu_agg* aggs, int32_t naggs,
                          int32_t maintain_order, plgpu_column* out_key, plgpu_column* out_aggs,
                          plgpu_groupby_info* info, void* stream) {
    if (out_key == nullptr) return fail(PLGPU_ERR_INVALID, "out_key is NULL");
    std::memset(out_key, 0, sizeof *out_key);
    for (int i = 0; i < naggs && out_aggs; ++i) std::memset(&out_aggs[i], 0, sizeof(plgpu_column));
    GbRun R;
    int rc = gb_prepare(R, key, cols, ncols, program, n_instr, aggs, naggs, maintain_order != 0, false, stream,
                        deriv);
    R.compact_ok = maintain_order == 0;  // the table is read only by gb_finalize below
    if (!rc) rc = gb_plan(R, nullptr);
    if (!rc) rc = gb_main(R, true, nullptr, nullptr);
    if (rc) return rc;
    if (info) gb_fill_info(R, info);
    return gb_finalize(R, naggs, out_key, out_aggs);
}

PLGPU_API int plgpu_group_by_agg(const plgpu_column* key, const plgpu_column* cols, int32_t ncols,
                                 const plgpu_instr* program, int32_t n_instr, const plgpu_agg* aggs, int32_t naggs,
                                 int32_t maintain_order, plgpu_column* out_key, plgpu_column* out_aggs,
                                 plgpu_groupby_info* info, void* stream) {
    return gb_single_impl(key, cols, ncols, nullptr, program, n_instr, aggs, naggs, maintain_order, out_key,
                          out_aggs, info, stream);
}

PLGPU_API int plgpu_debug_checks(uint32_t* out) {
    if (out == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    *out = 0;
#ifdef PLGPU_CHECKS
    PLGPU_HIP(hipDeviceSynchronize());
    // every translation unit's bits (groupby.hip and groupby_fast*.hip)
    for (GbChecksTake f : gb_checks_takers()) *out |= f();
    return PLGPU_OK;
#else
    return PLGPU_OK;
#endif
}

// ------------------------------------------------------- multi-GPU partials
struct plgpu_gb_partial {
    GbRun run;
};

PLGPU_API int plgpu_gb_record_words(const plgpu_column* cols, int32_t ncols, const plgpu_agg* aggs, int32_t naggs,
                                    int32_t* out_words) {
    if (out_words == nullptr || (cols == nullptr && ncols > 0)) return fail(PLGPU_ERR_INVALID, "NULL argument");
    if (ncols < 0 || ncols > PLGPU_MAX_COLS) return fail(PLGPU_ERR_INVALID, "too many columns (max 8)");
    std::vector<plgpu_column> c2(cols, cols + ncols);
    for (auto& c : c2) c.length = 0;
    plgpu_column k;
    std::memset(&k, 0, sizeof k);
    k.dtype = PLGPU_I64;
    Plan pl;
    DevProgram dp;
    std::memset(&dp, 0, sizeof dp);
    const std::vector<InSpec> ins = column_inputs(c2.data(), ncols);
    const int rc = plan_groupby(&k, c2.data(), ncols, ins.data(), ncols, aggs, naggs, false, dp, &pl, true);
    if (rc) return rc;
    *out_words = pl.p.nfields + 1;
    return PLGPU_OK;
}

PLGPU_API int plgpu_gb_plan_bottoms(const plgpu_column* key, const plgpu_column* cols, int32_t ncols,
                                    const plgpu_agg* aggs, int32_t naggs, int32_t* out_bottoms, void* stream) {
    if (out_bottoms == nullptr) return fail(PLGPU_ERR_INVALID, "out_bottoms is NULL");
    GbRun R;
    int rc = gb_prepare(R, key, cols, ncols, nullptr, 0, aggs, naggs, false, true, stream);
    if (!rc) rc = gb_plan(R, nullptr);
    if (rc) return rc;
    for (int a = 0; a < kMaxAcc; ++a) out_bottoms[a] = R.hb[a];
    return PLGPU_OK;
}

PLGPU_API int plgpu_gb_partial_begin(const plgpu_column* key, const plgpu_column* cols, int32_t ncols,
                                     const plgpu_instr* program, int32_t n_instr, const plgpu_agg* aggs,
                                     int32_t naggs, const int32_t* bottoms, int32_t world, plgpu_gb_partial** out,
                                     int64_t* out_records, int32_t* out_bottoms_used, int32_t* out_refit,
                                     int32_t* out_bottoms_hint, plgpu_groupby_info* info, void* stream) {
    if (out == nullptr || out_records == nullptr || out_bottoms_used == nullptr || out_refit == nullptr ||
        out_bottoms_hint == nullptr)
        return fail(PLGPU_ERR_INVALID, "NULL argument");
    if (world < 1) return fail(PLGPU_ERR_INVALID, "world must be >= 1");
    *out = nullptr;
    for (int i = 0; i < naggs && aggs; ++i)
        if (aggs[i].kind == PLGPU_AGG_FIRST || aggs[i].kind == PLGPU_AGG_LAST)
            // partial states hold rank-local row ids; merging first / last
            // across ranks needs global row order, which is not exchanged
            return fail(PLGPU_ERR_INVALID, "first / last aggregations are not supported on the partitioned path");
    plgpu_gb_partial* h = new plgpu_gb_partial();
    GbRun& R = h->run;
    R.world = world;
    R.wide_round = false;  // a wide sum's digits travel in the records
    bool refit = false;
    int rc = gb_prepare(R, key, cols, ncols, program, n_instr, aggs, naggs, false, true, stream);
    if (!rc) rc = gb_plan(R, bottoms);
    // own windows (bottoms NULL): refits happen here, since each source's
    // windows travel with its records (plgpu_gb_merge_sources); fixed
    // windows: a needed refit is reported.  A column wider than one window
    // keeps exact per-group digits (gb_wide); the ranks agree on one digit
    // range (plgpu_gb_partial_wide / _set_wide) before the export.
    if (!rc) rc = gb_main(R, bottoms == nullptr, &refit, out_bottoms_hint);
    if (rc) {
        delete h;
        return rc;
    }
    for (int a = 0; a < kMaxAcc; ++a) {
        out_bottoms_used[a] = R.hb[a];
        if (!refit) out_bottoms_hint[a] = R.hb[a];
    }
    *out_refit = refit ? 1 : 0;
    *out_records = gb_groups(R);
    if (info) gb_fill_info(R, info);
    *out = h;
    return PLGPU_OK;
}

PLGPU_API int plgpu_gb_partial_wide(const plgpu_gb_partial* h, int32_t* out_wide, int32_t* out_exmin,
                                    int32_t* out_exmax) {
    if (h == nullptr || out_wide == nullptr || out_exmin == nullptr || out_exmax == nullptr)
        return fail(PLGPU_ERR_INVALID, "NULL argument");
    const GbRun& R = h->run;
    const GbParams& p = R.pl.p;
    for (int a = 0; a < kMaxAcc; ++a) {
        out_wide[a] = 0;
        out_exmin[a] = 0x7FF;  // neutral for the ranks' min / max
        out_exmax[a] = 0;
        if (a >= p.nacc || !(p.acc[a].flags & (A_FSUM | A_FSUMCAST))) continue;
        if ((R.wide >> a) & 1u) {
            out_wide[a] = 1;
            out_exmin[a] = R.wide_exmin[a];
            out_exmax[a] = R.wide_exmax[a];
        } else {
            // every value of an exact fixed-point state has its bits in
            // [bottom, bottom + kSumWindowBits): biased exponents (mantissa
            // LSB at ex - 1075, subnormals as ex 1) in this range
            out_exmin[a] = std::max(1, R.hb[a] + 1075);
            out_exmax[a] = std::min(0x7FE, std::max(out_exmin[a], R.hb[a] + 1075 + kSumWindowBits - 53));
        }
    }
    return PLGPU_OK;
}

PLGPU_API int plgpu_gb_partial_set_wide(plgpu_gb_partial* h, const int32_t* wide, const int32_t* exmin,
                                        const int32_t* exmax) {
    if (h == nullptr || wide == nullptr || exmin == nullptr || exmax == nullptr)
        return fail(PLGPU_ERR_INVALID, "NULL argument");
    GbRun& R = h->run;
    const GbParams& p = R.pl.p;
    uint32_t mask = 0;
    for (int a = 0; a < kMaxAcc; ++a) {
        if (!wide[a]) continue;
        if (a >= p.nacc || !(p.acc[a].flags & (A_FSUM | A_FSUMCAST)))
            return fail(PLGPU_ERR_INVALID, "wide: only f64 sums take digit states");
        if (exmin[a] < 1 || exmax[a] > 0x7FE || exmin[a] > exmax[a])
            return fail(PLGPU_ERR_INVALID, "wide: bad exponent range");
        if (((R.wide >> a) & 1u) && (exmin[a] > R.wide_exmin[a] || exmax[a] < R.wide_exmax[a]))
            return fail(PLGPU_ERR_INVALID, "wide: the agreed range must cover this rank's");
        mask |= 1u << a;
    }
    if (mask == 0) return R.wide ? fail(PLGPU_ERR_INVALID, "wide: this rank holds a wide sum") : PLGPU_OK;
    if ((R.wide & ~mask) != 0) return fail(PLGPU_ERR_INVALID, "wide: this rank holds a wide sum");
    R.wide = mask;
    for (int a = 0; a < kMaxAcc; ++a)
        if ((mask >> a) & 1u) {
            R.wide_exmin[a] = exmin[a];
            R.wide_exmax[a] = exmax[a];
        }
    int rc = gb_wide(R, false);
    if (rc == PLGPU_OK) {
        hipError_t e = hipStreamSynchronize(R.s);
        if (e != hipSuccess) rc = hip_fail(e, "gb_wide_kernel");
    }
    return rc;
}

PLGPU_API int plgpu_gb_partial_record_words(const plgpu_gb_partial* h, int32_t* out_words) {
    if (h == nullptr || out_words == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    WideRec wr;
    *out_words = wide_layout(h->run, wr);
    return PLGPU_OK;
}

PLGPU_API int plgpu_gb_partial_export(plgpu_gb_partial* h, void* dst_records, int64_t* out_counts, void* stream) {
    if (h == nullptr || out_counts == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    GbRun& R = h->run;
    hipStream_t s = stream ? as_stream(stream) : R.s;
    const GbParams& p = R.pl.p;
    const int W = R.world;
    WideRec wr;
    const int rw = wide_layout(R, wr);
    for (int i = 0; i < wr.n; ++i)
        if (wr.digits[i] == nullptr) return fail(PLGPU_ERR_INVALID, "wide: digits missing");
    uint64_t* counts = nullptr;  // [W] counts, [W] cursors
    int rc = dev_alloc((void**)&counts, (size_t)W * 16, s);
    if (rc) return rc;
    PLGPU_HIP(hipMemsetAsync(counts, 0, (size_t)W * 16, s));
    const int fg = (int)std::min<int64_t>((p.gcap + 2 + 255) / 256, 256 * 16);
    gb_export_count_kernel<<<fg, 256, 0, s>>>(p, W, counts);
    std::vector<uint64_t> hc(W), cur(W);
    PLGPU_HIP(hipMemcpyAsync(hc.data(), counts, (size_t)W * 8, hipMemcpyDeviceToHost, s));
    PLGPU_HIP(hipStreamSynchronize(s));
    uint64_t run = 0;
    for (int w = 0; w < W; ++w) {
        cur[w] = run;
        run += hc[w];
        out_counts[w] = (int64_t)hc[w];
    }
    if (run > 0) {
        if (dst_records == nullptr) {
            dev_free(counts, s);
            return fail(PLGPU_ERR_INVALID, "dst_records is NULL");
        }
        PLGPU_HIP(hipMemcpyAsync(counts + W, cur.data(), (size_t)W * 8, hipMemcpyHostToDevice, s));
        gb_export_kernel<<<fg, 256, 0, s>>>(p, W, counts + W, (uint64_t*)dst_records, wr, rw);
        PLGPU_HIP(hipGetLastError());
    }
    PLGPU_HIP(hipStreamSynchronize(s));
    dev_free(counts, s);
    return PLGPU_OK;
}

PLGPU_API void plgpu_gb_partial_free(plgpu_gb_partial* h) { delete h; }

// Route rows by the partial states' owner rank (dest_rank of the row's key,
// as gb_export_kernel routes records): pass 0 counts per rank, pass 1 writes
// each row's index at its rank's cursor.  Order inside a rank is unspecified.
__device__ __forceinline__ int route_rank(const DevCol& key, int64_t r, int world) {
    if (!dev_valid(key, r)) return dest_rank(1, 0, world);
    const uint64_t k = dev_load(key, r);
    return dest_rank(k == kEmptyKey ? 2 : 0, k, world);
}

__global__ void gb_route_kernel(DevCol key, int64_t n, int world, int pass, unsigned long long* ctr,
                                uint32_t* __restrict__ perm) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        const int d = route_rank(key, r, world);
        const unsigned long long at = atomicAdd(&ctr[d], 1ull);
        if (pass) perm[at] = (uint32_t)r;
    }
}

PLGPU_API int plgpu_gb_route(const plgpu_column* key, int32_t world, plgpu_column* out_perm, int64_t* out_counts,
                             void* stream) {
    if (key == nullptr || out_perm == nullptr || out_counts == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    if (world < 1 || world > 1024) return fail(PLGPU_ERR_INVALID, "world must be 1..1024");
    if (!dtype_is_int(key->dtype) || dtype_bytes(key->dtype) > 8 || key->dtype == PLGPU_U64)
        return fail(PLGPU_ERR_SCHEMA, "route key must be a signed or 32-bit integer column");
    const int64_t n = key->length;
    if (n < 0 || n >= 0xFFFFFFFFll) return fail(PLGPU_ERR_CAPACITY, "route input exceeds the u32 index space");
    std::memset(out_perm, 0, sizeof *out_perm);
    hipStream_t s = as_stream(stream);
    int rc = make_owned_column(out_perm, PLGPU_U32, n, false, s);
    if (rc) return rc;
    unsigned long long* ctr = nullptr;  // [world] counts, then [world] cursors
    if ((rc = dev_alloc((void**)&ctr, (size_t)world * 16, s))) {
        plgpu_column_release(out_perm);
        return rc;
    }
    const DevCol k = to_dev(*key);
    const int g = (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096));
    std::vector<unsigned long long> hc(world), cur(world);
    hipError_t e = hipMemsetAsync(ctr, 0, (size_t)world * 8, s);
    if (e == hipSuccess && n > 0) {
        gb_route_kernel<<<g, 256, 0, s>>>(k, n, world, 0, ctr, nullptr);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(hc.data(), ctr, (size_t)world * 8, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    unsigned long long run = 0;
    for (int w = 0; w < world; ++w) {
        cur[w] = run;
        run += hc[w];
        out_counts[w] = (int64_t)hc[w];
    }
    if (e == hipSuccess && n > 0) {
        e = hipMemcpyAsync(ctr + world, cur.data(), (size_t)world * 8, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) {
            gb_route_kernel<<<g, 256, 0, s>>>(k, n, world, 1, ctr + world, (uint32_t*)out_perm->values);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipStreamSynchronize(s);  // `cur` is a host temporary
    }
    dev_free(ctr, s);
    if (e != hipSuccess) {
        plgpu_column_release(out_perm);
        return hip_fail(e, "gb_route_kernel");
    }
    return PLGPU_OK;
}

// ---------------------------------------- packed tuple keys across ranks
// The multi-key group-by packs integer / Boolean key tuples into one exact
// Int64 code (mk_plan_pack).  Across GPUs every rank must pack with the same
// plan, so the ranges are exported, reduced over the ranks by the caller
// (min / max / or), and the agreed ranges drive the packing and decoding.
static bool mk_packable(const plgpu_column* keys, int32_t nkeys) {
    for (int i = 0; i < nkeys; ++i) {
        const int32_t dt = keys[i].dtype;
        if ((!dtype_is_int(dt) && dt != PLGPU_BOOL) || dt == PLGPU_U64) return false;
    }
    return true;
}

static void mk_ranges_to_ord(const int64_t* ranges, int32_t nkeys, uint64_t* h) {
    for (int i = 0; i < nkeys; ++i) {
        h[3 * i] = (uint64_t)ranges[3 * i] ^ 0x8000000000000000ull;
        h[3 * i + 1] = (uint64_t)ranges[3 * i + 1] ^ 0x8000000000000000ull;
        h[3 * i + 2] = ranges[3 * i + 2] != 0;
    }
}

PLGPU_API int plgpu_key_ranges(const plgpu_column* keys, int32_t nkeys, int64_t* out_ranges, void* stream) {
    if (keys == nullptr || out_ranges == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    if (nkeys < 1 || nkeys > kMaxKeys) return fail(PLGPU_ERR_INVALID, "number of key columns must be 1..8");
    if (!mk_packable(keys, nkeys)) return fail(PLGPU_ERR_SCHEMA, "packed keys must be integer or Boolean columns");
    MkKeys mk;
    std::memset(&mk, 0, sizeof mk);
    mk.n = nkeys;
    const int64_t n = keys[0].length;
    for (int i = 0; i < nkeys; ++i) {
        if (keys[i].length != n) return fail(PLGPU_ERR_SHAPE, "key columns must have equal lengths");
        mk.c[i] = to_dev(keys[i]);
    }
    hipStream_t s = as_stream(stream);
    unsigned long long* st = nullptr;
    int rc = dev_alloc((void**)&st, 3 * kMaxKeys * 8, s);
    if (rc) return rc;
    unsigned long long h[3 * kMaxKeys];
    for (int i = 0; i < kMaxKeys; ++i) h[3 * i] = ~0ull, h[3 * i + 1] = 0, h[3 * i + 2] = 0;
    hipError_t e = hipMemcpyAsync(st, h, sizeof h, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && n > 0) {
        const int g = (int)std::min<int64_t>((n + 255) / 256, (int64_t)num_cus() * 16);
        mk_range_kernel<<<g, 256, 0, s>>>(mk, n, st);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h, st, sizeof h, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    dev_free(st, s);
    if (e != hipSuccess) return hip_fail(e, "key range pass");
    // signed min / max (no valid value: min = INT64_MAX > max = INT64_MIN)
    for (int i = 0; i < nkeys; ++i) {
        out_ranges[3 * i] = (int64_t)(h[3 * i] ^ 0x8000000000000000ull);
        out_ranges[3 * i + 1] = (int64_t)(h[3 * i + 1] ^ 0x8000000000000000ull);
        out_ranges[3 * i + 2] = h[3 * i + 2] ? 1 : 0;
    }
    return PLGPU_OK;
}

PLGPU_API int plgpu_key_pack(const plgpu_column* keys, int32_t nkeys, const int64_t* ranges, plgpu_column* out_codes,
                             int32_t* out_ok, void* stream) {
    if (keys == nullptr || ranges == nullptr || out_codes == nullptr || out_ok == nullptr)
        return fail(PLGPU_ERR_INVALID, "NULL argument");
    if (nkeys < 1 || nkeys > kMaxKeys) return fail(PLGPU_ERR_INVALID, "number of key columns must be 1..8");
    if (!mk_packable(keys, nkeys)) return fail(PLGPU_ERR_SCHEMA, "packed keys must be integer or Boolean columns");
    std::memset(out_codes, 0, sizeof *out_codes);
    *out_ok = 0;
    MkKeys mk;
    std::memset(&mk, 0, sizeof mk);
    mk.n = nkeys;
    const int64_t n = keys[0].length;
    for (int i = 0; i < nkeys; ++i) {
        if (keys[i].length != n) return fail(PLGPU_ERR_SHAPE, "key columns must have equal lengths");
        mk.c[i] = to_dev(keys[i]);
    }
    uint64_t h[3 * kMaxKeys];
    mk_ranges_to_ord(ranges, nkeys, h);
    MkPack pk;
    std::memset(&pk, 0, sizeof pk);
    pk.n = nkeys;
    mk_plan_from_ranges(h, nkeys, &pk);
    if (!pk.ok) return PLGPU_OK;
    hipStream_t s = as_stream(stream);
    int rc = make_owned_column(out_codes, PLGPU_I64, n, false, s);
    if (rc) return rc;
    if (n > 0) {
        const int g = (int)std::min<int64_t>((n + 255) / 256, (int64_t)num_cus() * 16);
        mk_pack_launch(mk, pk, n, (uint64_t*)out_codes->values, nullptr, nullptr, g, s);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            plgpu_column_release(out_codes);
            return hip_fail(e, "mk_pack_kernel");
        }
    }
    *out_ok = 1;
    return PLGPU_OK;
}

PLGPU_API int plgpu_key_unpack(const plgpu_column* codes, const int32_t* dtypes, int32_t nkeys, const int64_t* ranges,
                               plgpu_column* out_keys, void* stream) {
    if (codes == nullptr || dtypes == nullptr || ranges == nullptr || out_keys == nullptr)
        return fail(PLGPU_ERR_INVALID, "NULL argument");
    if (nkeys < 1 || nkeys > kMaxKeys) return fail(PLGPU_ERR_INVALID, "number of key columns must be 1..8");
    if (codes->dtype != PLGPU_I64) return fail(PLGPU_ERR_SCHEMA, "packed codes must be an Int64 column");
    for (int i = 0; i < nkeys; ++i) std::memset(&out_keys[i], 0, sizeof(plgpu_column));
    uint64_t h[3 * kMaxKeys];
    mk_ranges_to_ord(ranges, nkeys, h);
    MkPack pk;
    std::memset(&pk, 0, sizeof pk);
    pk.n = nkeys;
    mk_plan_from_ranges(h, nkeys, &pk);
    if (!pk.ok) return fail(PLGPU_ERR_INVALID, "these key ranges do not pack into 63 bits");
    hipStream_t s = as_stream(stream);
    const int64_t groups = codes->length;
    const int gg = (int)std::max<int64_t>(1, std::min<int64_t>((groups + 255) / 256, 4096));
    const int64_t* cv = (const int64_t*)codes->values + codes->offset;
    int rc = PLGPU_OK;
    for (int i = 0; i < nkeys && !rc; ++i) {
        const bool nullable = pk.nullable[i] != 0;
        rc = make_owned_column(&out_keys[i], dtypes[i], groups, nullable, s);
        if (rc || groups == 0) continue;
        if (dtypes[i] == PLGPU_BOOL) (void)hipMemsetAsync((void*)out_keys[i].values, 0, ((groups + 63) / 64) * 8, s);
        if (nullable) (void)hipMemsetAsync((void*)out_keys[i].validity, 0, ((groups + 63) / 64) * 8, s);
        mk_unpack_kernel<<<gg, 256, 0, s>>>(cv, nullptr, groups, pk, i, dtypes[i], (void*)out_keys[i].values,
                                            (uint32_t*)out_keys[i].validity);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) rc = hip_fail(e, "mk_unpack_kernel");
    }
    if (!rc) {
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "key unpack");
    }
    if (rc)
        for (int i = 0; i < nkeys; ++i) plgpu_column_release(&out_keys[i]);
    return rc;
}

// Float keys across ranks: a Float64 / Float32 key as the Int64 of its
// canonical bits (mk_word: -0.0 -> 0.0, every NaN -> one NaN), equal exactly
// when the reference's TotalEq groups them together.  The canonical bits
// are never INT64_MIN (that is -0.0's pattern).
__global__ __launch_bounds__(256) void float_code_kernel(DevCol c, int64_t n, int64_t* __restrict__ out,
                                                         uint64_t* __restrict__ valid_words) {
    for (int64_t r0 = (int64_t)blockIdx.x * blockDim.x; r0 < n; r0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = r0 + threadIdx.x;
        const bool in = r < n;
        const bool v = in && dev_valid(c, r);
        if (in) out[r] = v ? (int64_t)mk_word(c, r) : 0;
        const uint64_t b = __ballot(v);
        if (valid_words && (threadIdx.x & 63) == 0 && r < n) valid_words[r >> 6] = b;
    }
}

PLGPU_API int plgpu_float_key_encode(const plgpu_column* keys, plgpu_column* out_codes, void* stream) {
    if (keys == nullptr || out_codes == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    std::memset(out_codes, 0, sizeof *out_codes);
    if (keys->dtype != PLGPU_F64 && keys->dtype != PLGPU_F32)
        return fail(PLGPU_ERR_SCHEMA, "float key codes of a non-float column");
    hipStream_t s = as_stream(stream);
    const int64_t n = keys->length;
    // validity only when the keys have nulls: a null-free key keeps the
    // group-by's fast kernels
    int rc = make_owned_column(out_codes, PLGPU_I64, n, keys->validity != nullptr, s);
    if (rc) return rc;
    if (n > 0) {
        const int g = (int)std::min<int64_t>((n + 255) / 256, (int64_t)num_cus() * 16);
        float_code_kernel<<<g, 256, 0, s>>>(to_dev(*keys), n, (int64_t*)out_codes->values,
                                            (uint64_t*)out_codes->validity);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            plgpu_column_release(out_codes);
            return hip_fail(e, "float key codes");
        }
    }
    return PLGPU_OK;
}

// Merge of records from `nsrc` sources (nsrc 0: one source already on the
// table's windows `bottoms`).  With sources, the table takes, per acc, the
// lowest window of any source holding records, and each source's sum
// states are shifted onto it.
static int gb_merge_impl(const void* records, int64_t n_records, int32_t nsrc, const int64_t* src_records,
                         const int32_t* src_bottoms, const plgpu_column* cols, int32_t ncols, const plgpu_agg* aggs,
                         int32_t naggs, const int32_t* bottoms, int32_t key_dtype, plgpu_column* out_key,
                         plgpu_column* out_aggs, plgpu_groupby_info* info, void* stream,
                         const int32_t* wide = nullptr, const int32_t* wide_exmin = nullptr,
                         const int32_t* wide_exmax = nullptr) {
    if (out_key == nullptr || (cols == nullptr && ncols > 0)) return fail(PLGPU_ERR_INVALID, "NULL argument");
    if (ncols < 0 || ncols > PLGPU_MAX_COLS) return fail(PLGPU_ERR_INVALID, "too many columns (max 8)");
    if (n_records < 0 || (n_records > 0 && records == nullptr)) return fail(PLGPU_ERR_INVALID, "bad records");
    int32_t tb[kMaxAcc];
    std::vector<int64_t> start;
    std::vector<int32_t> shift;
    if (nsrc > 0) {
        start.assign(nsrc + 1, 0);
        for (int j = 0; j < nsrc; ++j) {
            if (src_records[j] < 0) return fail(PLGPU_ERR_INVALID, "bad source record count");
            start[j + 1] = start[j] + src_records[j];
        }
        if (start[nsrc] != n_records) return fail(PLGPU_ERR_INVALID, "source record counts do not add up");
        for (int a = 0; a < kMaxAcc; ++a) {
            bool any = false;
            tb[a] = 0;
            for (int j = 0; j < nsrc; ++j) {
                if (src_records[j] == 0) continue;
                const int32_t b = src_bottoms[j * kMaxAcc + a];
                tb[a] = any ? std::min(tb[a], b) : b;
                any = true;
            }
            if (!any) tb[a] = src_bottoms[a];
        }
        shift.assign((size_t)nsrc * kMaxAcc, 0);
        for (int j = 0; j < nsrc; ++j)
            for (int a = 0; a < kMaxAcc; ++a)
                if (src_records[j] > 0) shift[j * kMaxAcc + a] = src_bottoms[j * kMaxAcc + a] - tb[a];
    } else {
        if (bottoms == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
        for (int a = 0; a < kMaxAcc; ++a) tb[a] = bottoms[a];
    }
    std::memset(out_key, 0, sizeof *out_key);
    for (int i = 0; i < naggs && out_aggs; ++i) std::memset(&out_aggs[i], 0, sizeof(plgpu_column));
    // the schema alone fixes the record layout: a length-0 key of the right
    // dtype and the columns' dtypes (their buffers are not read)
    std::vector<plgpu_column> c2(cols, cols + ncols);
    for (auto& c : c2) c.length = 0;
    plgpu_column k;
    std::memset(&k, 0, sizeof k);
    k.dtype = dtype_is_int(key_dtype) ? key_dtype : PLGPU_I64;
    GbRun R;
    int rc = gb_prepare(R, &k, c2.data(), ncols, nullptr, 0, aggs, naggs, false, true, stream);
    if (rc) return rc;
    for (int a = 0; a < kMaxAcc; ++a) {
        R.hb[a] = tb[a];
        R.pl.p.bottom[a] = tb[a];
    }
    R.gbits = log2_ceil(std::max<int64_t>(1024, n_records * 2));
    GbParams& p = R.pl.p;
    if (wide) {
        for (int a = 0; a < kMaxAcc; ++a) {
            if (!wide[a]) continue;
            if (a >= p.nacc || !(p.acc[a].flags & (A_FSUM | A_FSUMCAST)))
                return fail(PLGPU_ERR_INVALID, "wide: only f64 sums take digit states");
            if (wide_exmin[a] < 1 || wide_exmax[a] > 0x7FE || wide_exmin[a] > wide_exmax[a])
                return fail(PLGPU_ERR_INVALID, "wide: bad exponent range");
            R.wide |= 1u << a;
            R.wide_exmin[a] = wide_exmin[a];
            R.wide_exmax[a] = wide_exmax[a];
        }
    }
    // source table on the device: nsrc + 1 starts, then nsrc x kMaxAcc shifts
    int64_t* dsrc = nullptr;
    if (nsrc > 0) {
        const size_t bytes = (size_t)(nsrc + 1) * 8 + shift.size() * 4;
        if ((rc = dev_alloc((void**)&dsrc, bytes, R.s))) return rc;
        std::vector<uint8_t> h(bytes);
        std::memcpy(h.data(), start.data(), (size_t)(nsrc + 1) * 8);
        std::memcpy(h.data() + (size_t)(nsrc + 1) * 8, shift.data(), shift.size() * 4);
        hipError_t e = hipMemcpyAsync(dsrc, h.data(), bytes, hipMemcpyHostToDevice, R.s);
        if (e == hipSuccess) e = hipStreamSynchronize(R.s);  // `h` is a host temporary
        if (e != hipSuccess) {
            dev_free(dsrc, R.s);
            return hip_fail(e, "merge sources");
        }
    }
    for (R.attempts = 0;; ++R.attempts) {
        if ((rc = gb_alloc_table(R))) break;
        // wide sums: zeroed digit arrays for this table
        for (int a = 0; a < kMaxAcc && !rc; ++a) {
            if (!((R.wide >> a) & 1u)) continue;
            dev_free(R.wide_digits[a], R.s);
            R.wide_digits[a] = nullptr;
            const size_t words = (size_t)(p.gcap + 2) * wide_nwords(R.wide_exmin[a], R.wide_exmax[a]);
            rc = dev_alloc((void**)&R.wide_digits[a], words * 8, R.s);
            if (!rc && hipMemsetAsync(R.wide_digits[a], 0, words * 8, R.s) != hipSuccess)
                rc = fail(PLGPU_ERR_HIP, "wide digits");
        }
        if (rc) break;
        WideRec wr;
        const int rw = wide_layout(R, wr);
        hipError_t e = hipMemcpyAsync(R.bottoms, R.hb, sizeof R.hb, hipMemcpyHostToDevice, R.s);
        if (e == hipSuccess && n_records > 0) {
            const int g = (int)std::min<int64_t>((n_records + 255) / 256, 256 * 16);
            gb_merge_kernel<<<g, 256, 0, R.s>>>(p, (const uint64_t*)records, n_records, nsrc, dsrc,
                                                dsrc ? (const int32_t*)(dsrc + nsrc + 1) : nullptr, wr, rw);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(R.st, R.status, sizeof R.st, hipMemcpyDeviceToHost, R.s);
        if (e == hipSuccess) e = hipStreamSynchronize(R.s);
        if (e != hipSuccess) {
            rc = hip_fail(e, "gb_merge_kernel");
            break;
        }
        if (R.st[ST_SHIFT_OVF]) {
            rc = fail(PLGPU_ERR_CAPACITY,
                      "multi-GPU group-by: the ranks' f64 sums span more binades than one 192-bit state holds");
            break;
        }
        if (R.st[ST_TABLE_FULL] == 0) break;
        if (R.attempts >= 3) {
            rc = fail(PLGPU_ERR_CAPACITY, "merge did not converge");
            break;
        }
        R.gbits += 3;
    }
    dev_free(dsrc, R.s);
    for (int a = 0; a < kMaxAcc && !rc; ++a) {
        // the merged digits, rounded once per group
        if (!((R.wide >> a) & 1u)) continue;
        rc = dev_alloc((void**)&R.wide_sum[a], (size_t)(p.gcap + 2) * 8, R.s);
        if (rc) break;
        const int fg = (int)std::min<int64_t>((p.gcap + 2 + 255) / 256, 256 * 16);
        gb_wide_round_kernel<<<fg, 256, 0, R.s>>>(p, R.wide_exmin[a], wide_nwords(R.wide_exmin[a], R.wide_exmax[a]),
                                                  R.wide_digits[a], R.wide_sum[a]);
        if (hipGetLastError() != hipSuccess) rc = fail(PLGPU_ERR_HIP, "gb_wide_round_kernel");
    }
    if (rc) return rc;
    if (info) gb_fill_info(R, info);
    return gb_finalize(R, naggs, out_key, out_aggs);
}

PLGPU_API int plgpu_gb_merge(const void* records, int64_t n_records, const plgpu_column* cols, int32_t ncols,
                             const plgpu_agg* aggs, int32_t naggs, const int32_t* bottoms, int32_t key_dtype,
                             plgpu_column* out_key, plgpu_column* out_aggs, plgpu_groupby_info* info, void* stream) {
    return gb_merge_impl(records, n_records, 0, nullptr, nullptr, cols, ncols, aggs, naggs, bottoms, key_dtype,
                         out_key, out_aggs, info, stream);
}

PLGPU_API int plgpu_gb_merge_sources(const void* records, int32_t n_sources, const int64_t* src_records,
                                     const int32_t* src_bottoms, const plgpu_column* cols, int32_t ncols,
                                     const plgpu_agg* aggs, int32_t naggs, int32_t key_dtype, plgpu_column* out_key,
                                     plgpu_column* out_aggs, plgpu_groupby_info* info, void* stream) {
    if (n_sources < 1 || src_records == nullptr || src_bottoms == nullptr)
        return fail(PLGPU_ERR_INVALID, "merge: need >= 1 source with its record count and windows");
    int64_t n = 0;
    for (int j = 0; j < n_sources; ++j) n += src_records[j];
    return gb_merge_impl(records, n, n_sources, src_records, src_bottoms, cols, ncols, aggs, naggs, nullptr,
                         key_dtype, out_key, out_aggs, info, stream);
}

PLGPU_API int plgpu_gb_merge_sources_wide(const void* records, int32_t n_sources, const int64_t* src_records,
                                          const int32_t* src_bottoms, const int32_t* wide, const int32_t* wide_exmin,
                                          const int32_t* wide_exmax, const plgpu_column* cols, int32_t ncols,
                                          const plgpu_agg* aggs, int32_t naggs, int32_t key_dtype,
                                          plgpu_column* out_key, plgpu_column* out_aggs, plgpu_groupby_info* info,
                                          void* stream) {
    if (n_sources < 1 || src_records == nullptr || src_bottoms == nullptr)
        return fail(PLGPU_ERR_INVALID, "merge: need >= 1 source with its record count and windows");
    if (wide == nullptr || wide_exmin == nullptr || wide_exmax == nullptr)
        return fail(PLGPU_ERR_INVALID, "NULL argument");
    int64_t n = 0;
    for (int j = 0; j < n_sources; ++j) n += src_records[j];
    return gb_merge_impl(records, n, n_sources, src_records, src_bottoms, cols, ncols, aggs, naggs, nullptr,
                         key_dtype, out_key, out_aggs, info, stream, wide, wide_exmin, wide_exmax);
}

// ------------------------------------------------------ multi-key group-by
// Packed path: group by the exact Int64 code, then decode the output codes
// into the key columns.
// `checked`: pk comes from sampled ranges (mk_plan_pack_sampled); a row
// outside them sets *repack (nothing else done) and the caller repacks
// with the exact ranges.
// Field i's fit test (KeyPack::span): v - base <= min(2^bits - 1, 2^64 - 1 -
// ord(base)) holds exactly for base <= v < base + 2^bits (signed): a v below
// base wraps to more than 2^64 - 1 - ord(base).  Same on 32 bits for a 4-byte
// column whose base is a value of its type.
static void kp_span(KeyPack& k, int i) {
    const int bits = k.bits[i];
    if (bits >= 64) {
        // identity field (one key whose extended value is the code): every
        // value fits, whatever its sign
        k.span[i] = ~0ull;
        k.mode[i] = (k.c[i].dtype == PLGPU_I32 || k.c[i].dtype == PLGPU_U32) ? 2 : 0;  // widened
        k.span32[i] = 0xFFFFFFFFu;
        return;
    }
    const uint64_t mask = bits >= 64 ? ~0ull : (1ull << bits) - 1;
    const uint64_t ordb = k.base[i] ^ 0x8000000000000000ull;
    k.span[i] = std::min<uint64_t>(mask, ~0ull - ordb);
    const int32_t dt = k.c[i].dtype;
    const int64_t b = (int64_t)k.base[i];
    k.mode[i] = 0;
    if (dt == PLGPU_I32 || dt == PLGPU_U32) {
        const bool in_range = dt == PLGPU_I32 ? (b >= INT32_MIN && b <= INT32_MAX) : (b >= 0 && b <= (int64_t)UINT32_MAX);
        k.mode[i] = in_range ? 1 : 2;
        k.x32[i] = dt == PLGPU_I32 ? 0x80000000u : 0u;
        k.b32[i] = (uint32_t)b ^ k.x32[i];
        const uint32_t m32 = bits >= 32 ? 0xFFFFFFFFu : (1u << bits) - 1;
        k.span32[i] = std::min<uint32_t>(m32, 0xFFFFFFFFu - k.b32[i]);
    }
}

// The packing plan as the fused kernel's KeyPack, or n = 0 when the key
// columns do not qualify (more than kKpFast, nullable, not Int64 / Int32 /
// UInt32, misaligned, or a small input).
static KeyPack kp_from_plan(const MkKeys& mk, const MkPack& pk, int64_t n) {
    KeyPack k;
    std::memset(&k, 0, sizeof k);
    if (!options().fuse_keys || mk.n < 1 || mk.n > kKpFast || n < (int64_t(1) << 20)) return k;
    for (int i = 0; i < mk.n; ++i) {
        const DevCol& c = mk.c[i];
        const bool w8 = c.dtype == PLGPU_I64, w4 = c.dtype == PLGPU_I32 || c.dtype == PLGPU_U32;
        if (!(w8 || w4) || c.validity != nullptr || (c.offset & 1) != 0 ||
            ((uintptr_t)c.values & (w8 ? 15 : 7)) != 0)
            return k;
    }
    for (int i = 0; i < mk.n; ++i) {
        k.c[i] = mk.c[i];
        k.base[i] = (uint64_t)pk.minv[i] - (pk.nullable[i] ? 1u : 0u);
        k.shift[i] = pk.shift[i];
        k.bits[i] = pk.bits[i];
        kp_span(k, i);
    }
    k.n = mk.n;
    return k;
}

// Decode the group-by's output codes (hout) into the key columns.
static int gb_multi_decode(const MkPack& pk, const plgpu_column* keys, int32_t nkeys, plgpu_column& hout,
                           plgpu_column* out_keys, plgpu_column* out_aggs, int32_t naggs, hipStream_t s) {
    int rc = PLGPU_OK;
    const int64_t groups = hout.length;
    const int gg = (int)std::max<int64_t>(1, std::min<int64_t>((groups + 255) / 256, 4096));
    for (int i = 0; i < nkeys && !rc; ++i) {
        const bool nullable = pk.nullable[i] != 0;
        rc = make_owned_column(&out_keys[i], keys[i].dtype, groups, nullable, s);
        if (rc || groups == 0) continue;
        if (keys[i].dtype == PLGPU_BOOL) (void)hipMemsetAsync((void*)out_keys[i].values, 0, ((groups + 63) / 64) * 8, s);
        if (nullable) (void)hipMemsetAsync((void*)out_keys[i].validity, 0, ((groups + 63) / 64) * 8, s);
        {
            KtScope kt("mk_unpack_kernel", s);
            mk_unpack_kernel<<<gg, 256, 0, s>>>((const int64_t*)hout.values, nullptr, groups, pk, i, keys[i].dtype,
                                                (void*)out_keys[i].values, (uint32_t*)out_keys[i].validity);
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) rc = hip_fail(e, "mk_unpack_kernel");
    }
    // (no synchronisation: the key columns are ready in the caller's stream
    // order, and hout's block is reused only by work enqueued after these
    // kernels)
    plgpu_column_release(&hout);
    if (rc) {
        for (int i = 0; i < nkeys; ++i) plgpu_column_release(&out_keys[i]);
        for (int i = 0; i < naggs; ++i) plgpu_column_release(&out_aggs[i]);
    }
    return rc;
}

static int gb_multi_packed(const MkKeys& mk, MkPack pk, int64_t n, const plgpu_column* keys, int32_t nkeys,
                           const plgpu_column* cols, int32_t ncols, const Deriv* deriv, const plgpu_instr* program,
                           int32_t n_instr, const plgpu_agg* aggs, int32_t naggs, int32_t maintain_order,
                           plgpu_column* out_keys, plgpu_column* out_aggs, plgpu_groupby_info* info, void* stream,
                           bool checked = false, bool* repack = nullptr) {
    hipStream_t s = as_stream(stream);
    if (repack) *repack = false;
    const KeyPack kp = kp_from_plan(mk, pk, n);
    if (options().debug)
        fprintf(stderr, "[plgpu] gb_multi_packed: n=%lld keys=%d fused key pack=%d checked=%d\n", (long long)n, mk.n,
                kp.n, (int)checked);
    if (kp.n > 0) {
        // fused key packing: the fused kernel forms each row's code from the
        // key columns it loads (no code column written or read).  Off the
        // fused kernel (many groups, derived inputs, ...) the plan says so
        // and the code column below is used instead.
        plgpu_column ck;
        std::memset(&ck, 0, sizeof ck);
        ck.dtype = PLGPU_I64;
        ck.length = n;
        ck.values = keys[0].values;  // never read as a key column while p.kp.n > 0
        plgpu_column hout;
        std::memset(&hout, 0, sizeof hout);
        GbRun R;
        int rc = gb_prepare(R, &ck, cols, ncols, program, n_instr, aggs, naggs, maintain_order != 0, false, stream,
                            deriv);
        if (!rc) {
            R.pl.p.kp = kp;
            rc = gb_plan(R, nullptr);
        }
        if (!rc && !R.kp_fallback) {
            rc = gb_main(R, true, nullptr, nullptr);
            if (!rc && R.kp_bad) {
                if (!checked) return fail(PLGPU_ERR_HIP, "fused key packing: a row outside the exact packing plan");
                *repack = true;
                return PLGPU_OK;
            }
            if (!rc && info) gb_fill_info(R, info);
            if (!rc) rc = gb_finalize(R, naggs, &hout, out_aggs);
            if (rc) return rc;
            return gb_multi_decode(pk, keys, nkeys, hout, out_keys, out_aggs, naggs, s);
        }
        if (rc) return rc;
    }
    uint64_t* codes = nullptr;
    int rc = dev_alloc((void**)&codes, (size_t)std::max<int64_t>(n, 1) * 8 + (checked ? 8 : 0), s);
    if (rc) return rc;
    if (n > 0) {
        unsigned int* outside = checked ? (unsigned int*)(codes + std::max<int64_t>(n, 1)) : nullptr;
        hipError_t e = hipSuccess;
        if (outside) e = hipMemsetAsync(outside, 0, 4, s);
        const int g = (int)std::min<int64_t>((n + 255) / 256, (int64_t)num_cus() * 16);
        if (e == hipSuccess) {
            mk_pack_launch(mk, pk, n, codes, nullptr, outside, g, s);
            e = hipGetLastError();
        }
        unsigned int bad = 0;
        if (e == hipSuccess && outside) e = hipMemcpyAsync(&bad, outside, 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && outside) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "mk_pack_kernel");
        if (!rc && bad) {
            dev_free(codes, s);
            *repack = true;
            return PLGPU_OK;
        }
    }
    plgpu_column ck;
    std::memset(&ck, 0, sizeof ck);
    ck.dtype = PLGPU_I64;
    ck.length = n;
    ck.values = codes;
    plgpu_column hout;
    std::memset(&hout, 0, sizeof hout);
    {
        GbRun R;
        if (!rc)
            rc = gb_prepare(R, &ck, cols, ncols, program, n_instr, aggs, naggs, maintain_order != 0, false, stream,
                            deriv);
        if (!rc) rc = gb_plan(R, nullptr);
        if (!rc) rc = gb_main(R, true, nullptr, nullptr);
        if (!rc && info) gb_fill_info(R, info);
        if (!rc) rc = gb_finalize(R, naggs, &hout, out_aggs);
    }
    dev_free(codes, s);
    if (rc) return rc;
    return gb_multi_decode(pk, keys, nkeys, hout, out_keys, out_aggs, naggs, s);
}

// A single null-free String key grouped on short-string codes formed in the
// fused kernel (KeyPack with a String column).  *done = false (nothing
// produced) when the fused kernel does not apply or a selected string is
// longer than 7 bytes.
static int gb_str_fused(const plgpu_column& key, const plgpu_column* cols, int32_t ncols, const Deriv* deriv,
                        const plgpu_instr* program, int32_t n_instr, const plgpu_agg* aggs, int32_t naggs,
                        int32_t maintain_order, plgpu_column* out_keys, plgpu_column* out_aggs,
                        plgpu_groupby_info* info, hipStream_t s, bool* done) {
    *done = false;
    const int64_t n = key.length;
    int64_t data_end = 0;
    PLGPU_HIP(hipMemcpyAsync(&data_end, (const int64_t*)key.values + key.offset + n, 8, hipMemcpyDeviceToHost, s));
    PLGPU_HIP(hipStreamSynchronize(s));
    KeyPack kp;
    std::memset(&kp, 0, sizeof kp);
    kp.n = 1;
    kp.c[0] = dev_col(key);
    kp.bits[0] = 64;
    kp.span[0] = ~0ull;
    kp.data_end = data_end;
    plgpu_column ck;
    std::memset(&ck, 0, sizeof ck);
    ck.dtype = PLGPU_I64;
    ck.length = n;
    ck.values = key.values;  // never read as a key column while p.kp.n > 0
    GbRun R;
    int rc = gb_prepare(R, &ck, cols, ncols, program, n_instr, aggs, naggs, maintain_order != 0, false, s, deriv);
    if (!rc) {
        R.pl.p.kp = kp;
        rc = gb_plan(R, nullptr);
    }
    if (rc || R.kp_fallback) return rc;
    rc = gb_main(R, true, nullptr, nullptr);
    if (rc || R.kp_bad) return rc;  // a long string: the hashed path
    plgpu_column hout;
    std::memset(&hout, 0, sizeof hout);
    if (info) gb_fill_info(R, info);
    if ((rc = gb_finalize(R, naggs, &hout, out_aggs))) return rc;
    rc = str_from_codes(hout, &out_keys[0], s);
    plgpu_column_release(&hout);
    if (rc) {
        for (int i = 0; i < naggs; ++i) plgpu_column_release(&out_aggs[i]);
        return rc;
    }
    *done = true;
    return PLGPU_OK;
}

static int gb_multi_impl(const plgpu_column* keys, int32_t nkeys, const plgpu_column* cols, int32_t ncols,
                         const Deriv* deriv, const plgpu_instr* program, int32_t n_instr, const plgpu_agg* aggs,
                         int32_t naggs, int32_t maintain_order, plgpu_column* out_keys, plgpu_column* out_aggs,
                         plgpu_groupby_info* info, void* stream) {
    if (keys == nullptr || out_keys == nullptr) return fail(PLGPU_ERR_INVALID, "keys / out_keys is NULL");
    if (nkeys < 1 || nkeys > kMaxKeys) return fail(PLGPU_ERR_INVALID, "number of key columns must be 1..8");
    for (int i = 0; i < nkeys; ++i) std::memset(&out_keys[i], 0, sizeof(plgpu_column));
    for (int i = 0; i < naggs && out_aggs; ++i) std::memset(&out_aggs[i], 0, sizeof(plgpu_column));
    const int64_t n = keys[0].length;
    MkKeys mk;
    std::memset(&mk, 0, sizeof mk);
    mk.n = nkeys;
    for (int i = 0; i < nkeys; ++i) {
        const int32_t dt = keys[i].dtype;
        if (!dtype_is_int(dt) && !dtype_is_float(dt) && dt != PLGPU_BOOL && dt != PLGPU_STR)
            return fail(PLGPU_ERR_SCHEMA, "group-by keys must be integer, float, Boolean or String columns");
        if (keys[i].length != n) return fail(PLGPU_ERR_SHAPE, "key columns must have equal lengths");
        mk.c[i] = to_dev(keys[i]);
    }
    hipStream_t s = as_stream(stream);
    if (nkeys == 1 && keys[0].dtype == PLGPU_STR && keys[0].validity == nullptr && n >= (int64_t(1) << 20) &&
        options().fuse_keys) {
        // one null-free String key: its short-string codes formed inside the
        // fused kernel (no code column); a string longer than 7 bytes, or a
        // plan off the fused kernel, falls through to the passes below
        bool done = false;
        const int rc = gb_str_fused(keys[0], cols, ncols, deriv, program, n_instr, aggs, naggs, maintain_order,
                                    out_keys, out_aggs, info, s, &done);
        if (rc || done) return rc;
    }
    {
        // String keys whose strings are all <= 7 bytes: exact Int64 codes,
        // grouped as integer keys; the output codes turn back into strings
        bool any_str = false, short_all = true;
        plgpu_column ck[kMaxKeys];
        std::memset(ck, 0, sizeof ck);
        int rc = PLGPU_OK;
        for (int i = 0; i < nkeys; ++i) {
            ck[i] = keys[i];
            if (keys[i].dtype != PLGPU_STR || !short_all || rc) continue;
            any_str = true;
            bool sh = false;
            rc = str_short_codes(keys[i], &ck[i], &sh, s);
            short_all = short_all && sh;
        }
        if (any_str && !rc && short_all) {
            // one key: the single-key group-by takes the Int64 codes (and
            // their validity) directly, no tuple packing pass
            if (nkeys == 1)
                rc = gb_single_impl(&ck[0], cols, ncols, deriv, program, n_instr, aggs, naggs, maintain_order,
                                    &out_keys[0], out_aggs, info, stream);
            else
                rc = gb_multi_impl(ck, nkeys, cols, ncols, deriv, program, n_instr, aggs, naggs, maintain_order,
                                   out_keys, out_aggs, info, stream);
            for (int i = 0; i < nkeys && !rc; ++i) {
                if (keys[i].dtype != PLGPU_STR) continue;
                plgpu_column strs;
                rc = str_from_codes(out_keys[i], &strs, s);
                plgpu_column_release(&out_keys[i]);
                if (!rc) out_keys[i] = strs;
            }
            if (rc) {
                for (int i = 0; i < nkeys; ++i) plgpu_column_release(&out_keys[i]);
                for (int i = 0; i < naggs && out_aggs; ++i) plgpu_column_release(&out_aggs[i]);
            }
        }
        for (int i = 0; i < nkeys; ++i)
            if (keys[i].dtype == PLGPU_STR && ck[i].dtype == PLGPU_I64) str_codes_free(&ck[i], s);
        if (rc || (any_str && short_all)) return rc;
    }
    if (nkeys == 1 && (keys[0].dtype == PLGPU_I32 || keys[0].dtype == PLGPU_U32) && keys[0].validity == nullptr &&
        n >= (int64_t(1) << 20) && options().fuse_keys) {
        // one null-free 4-byte key (dates, Categorical codes): its extended
        // value is the code (identity plan: no sample, no range check); the
        // fused kernel reads the 4-byte column itself
        MkPack pk;
        std::memset(&pk, 0, sizeof pk);
        pk.n = 1;
        pk.ok = 1;
        pk.bits[0] = 64;
        // (nothing lies outside a 64-bit identity field, so no repack; if
        // one were ever reported, the exact packing below takes over)
        bool repack = false;
        const int rc = gb_multi_packed(mk, pk, n, keys, nkeys, cols, ncols, deriv, program, n_instr, aggs, naggs,
                                       maintain_order, out_keys, out_aggs, info, stream, true, &repack);
        if (rc || !repack) return rc;
    }
    const int hg = (int)std::min<int64_t>((n + 255) / 256, (int64_t)num_cus() * 16);
    {
        // integer keys whose ranges fit 63 bits together: one exact packed
        // Int64 key, grouped by the single-key paths (no hash, no verify)
        // The plan comes from a sample of the key columns first (no full
        // range pass); a row outside the sampled (widened) ranges sends it
        // to the exact range pass and a repack.
        MkPack pk;
        int rc = PLGPU_OK;
        // a repeated query over the same resident key columns reuses the
        // last packing plan (large inputs; option plan_cache)
        const bool reuse = options().plan_cache != 0 && n >= (int64_t(1) << 24);
        const std::string pkey = reuse ? pack_key(mk, n) : std::string();
        if (n >= (int64_t(1) << 20)) {
            if (!(reuse && pack_cache_get(pkey, &pk))) {
                if ((rc = mk_plan_pack_sampled(mk, n, &pk, s))) return rc;
                if (reuse && pk.ok) pack_cache_put(pkey, pk);
            }
            if (pk.ok) {
                bool repack = false;
                rc = gb_multi_packed(mk, pk, n, keys, nkeys, cols, ncols, deriv, program, n_instr, aggs, naggs,
                                     maintain_order, out_keys, out_aggs, info, stream, true, &repack);
                if (rc || !repack) return rc;
            }
        }
        rc = mk_plan_pack(mk, n, nullptr, 0, std::max(hg, 1), &pk, s);
        if (rc) return rc;
        if (reuse && pk.ok) pack_cache_put(pkey, pk);  // the exact ranges: no repack next time
        if (pk.ok) return gb_multi_packed(mk, pk, n, keys, nkeys, cols, ncols, deriv, program, n_instr, aggs, naggs,
                                          maintain_order, out_keys, out_aggs, info, stream);
    }
    uint64_t* hashes = nullptr;
    uint32_t* collision = nullptr;
    int rc = dev_alloc((void**)&hashes, (size_t)std::max<int64_t>(n, 1) * 8, s);
    if (!rc) rc = dev_alloc((void**)&collision, 4, s);
    plgpu_column hk;
    std::memset(&hk, 0, sizeof hk);
    hk.dtype = PLGPU_I64;
    hk.length = n;
    hk.values = hashes;
    bool done = false;
    for (int attempt = 0; attempt < 4 && !rc && !done; ++attempt) {
        const uint64_t seed = 0x243F6A8885A308D3ull * (uint64_t)(2 * attempt + 1);
        // PLGPU_MK_COLLIDE (tests only): a 3-bit first hash forces the
        // collision -> re-seed path
        const uint64_t mask = attempt == 0 && options().mk_collide ? 7ull : ~0ull;
        if (n > 0) mk_hash_kernel<<<std::max(hg, 1), 256, 0, s>>>(mk, n, seed, mask, hashes);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) { rc = hip_fail(e, "mk_hash_kernel"); break; }
        GbRun R;
        R.want_first = true;
        rc = gb_prepare(R, &hk, cols, ncols, program, n_instr, aggs, naggs, maintain_order != 0, false, stream, deriv);
        if (!rc) rc = gb_plan(R, nullptr);
        if (!rc) rc = gb_main(R, true, nullptr, nullptr);
        if (rc) break;
        plgpu_column hout;
        uint64_t* first = nullptr;
        if ((rc = gb_finalize(R, naggs, &hout, out_aggs, &first))) break;
        const int64_t groups = hout.length;
        plgpu_column_release(&hout);
        uint32_t coll = 0;
        if (n > 0 && groups > 0) {
            const int64_t total = R.pl.p.gcap + 2;
            uint64_t* vw = nullptr;
            if ((rc = dev_alloc((void**)&vw, (size_t)total * (nkeys * 8 + 4), s))) break;
            uint32_t* vmask = (uint32_t*)(vw + (size_t)total * nkeys);
            (void)hipMemsetAsync(collision, 0, 4, s);
            mk_rep_kernel<<<(unsigned)std::min<int64_t>((total + 255) / 256, 4096), 256, 0, s>>>(R.pl.p, mk, vw,
                                                                                               vmask);
            mk_verify_kernel<<<std::max(hg, 1), 256, 0, s>>>(R.pl.p, mk, hashes, n, vw, vmask, collision);
            dev_free(vw, s);
            e = hipGetLastError();
            if (e == hipSuccess) e = hipMemcpyAsync(&coll, collision, 4, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) rc = hip_fail(e, "mk_verify_kernel");
        }
        if (!rc && !coll) {
            const int gg = (int)std::min<int64_t>((groups + 255) / 256, 4096);
            for (int i = 0; i < nkeys && !rc; ++i) {
                const bool nullable = keys[i].validity != nullptr;
                if (keys[i].dtype == PLGPU_STR) {  // each group's key string from its first row
                    rc = str_gather(mk.c[i], nullptr, (const int64_t*)first, nullptr, 0, groups, nullable,
                                    &out_keys[i], s);
                    continue;
                }
                rc = make_owned_column(&out_keys[i], keys[i].dtype, groups, nullable, s);
                if (rc || groups == 0) continue;
                if (keys[i].dtype == PLGPU_BOOL) (void)hipMemsetAsync((void*)out_keys[i].values, 0, ((groups + 63) / 64) * 8, s);
                if (nullable) (void)hipMemsetAsync((void*)out_keys[i].validity, 0, ((groups + 63) / 64) * 8, s);
                mk_gather_key_kernel<<<gg, 256, 0, s>>>(mk.c[i], first, groups, n, (void*)out_keys[i].values,
                                                        (uint32_t*)out_keys[i].validity);
                e = hipGetLastError();
                if (e != hipSuccess) rc = hip_fail(e, "mk_gather_key_kernel");
            }
            if (!rc) {
                e = hipStreamSynchronize(s);
                if (e != hipSuccess) rc = hip_fail(e, "multi-key gather");
            }
            if (!rc && info) {
                gb_fill_info(R, info);
                info->reruns += attempt;
            }
            done = !rc;
        }
        dev_free(first, s);
        if (!done)
            for (int i = 0; i < naggs; ++i) plgpu_column_release(&out_aggs[i]);
    }
    dev_free(collision, s);
    dev_free(hashes, s);
    if (!rc && !done) rc = fail(PLGPU_ERR_CAPACITY, "multi-key group-by: unresolved 64-bit hash collisions");
    if (rc)
        for (int i = 0; i < nkeys; ++i) plgpu_column_release(&out_keys[i]);
    return rc;
}

PLGPU_API int plgpu_group_by_agg_multi(const plgpu_column* keys, int32_t nkeys, const plgpu_column* cols,
                                       int32_t ncols, const plgpu_instr* program, int32_t n_instr,
                                       const plgpu_agg* aggs, int32_t naggs, int32_t maintain_order,
                                       plgpu_column* out_keys, plgpu_column* out_aggs, plgpu_groupby_info* info,
                                       void* stream) {
    return gb_multi_impl(keys, nkeys, cols, ncols, nullptr, program, n_instr, aggs, naggs, maintain_order, out_keys,
                         out_aggs, info, stream);
}

// Global reduction: every selected row in one group (the keyless key
// column, key_at), then the one output row -- or, with no row selected, the
// reference's empty reductions (sum / len / count 0, the rest null).
static int gb_keyless(const plgpu_column* cols, int32_t ncols, const Deriv* deriv, const plgpu_instr* program,
                      int32_t n_instr, const plgpu_agg* aggs, int32_t naggs, plgpu_column* out_aggs,
                      plgpu_groupby_info* info, void* stream) {
    if (ncols < 1) return fail(PLGPU_ERR_INVALID, "a global reduction needs at least one column (the length)");
    plgpu_column k;
    std::memset(&k, 0, sizeof k);
    k.dtype = PLGPU_I64;
    k.length = cols[0].length;
    k.device_id = cols[0].device_id;
    plgpu_column out_key;
    int rc = gb_single_impl(&k, cols, ncols, deriv, program, n_instr, aggs, naggs, 0, &out_key, out_aggs, info,
                            stream);
    if (rc) return rc;
    const int64_t groups = out_key.length;
    plgpu_column_release(&out_key);
    if (groups == 1) return PLGPU_OK;
    if (groups != 0) return fail(PLGPU_ERR_CAPACITY, "internal: a global reduction produced several groups");
    hipStream_t s = as_stream(stream);
    for (int i = 0; i < naggs && rc == PLGPU_OK; ++i) {
        const int32_t dt = out_aggs[i].dtype;
        const bool has_valid = out_aggs[i].validity != nullptr;
        plgpu_column_release(&out_aggs[i]);
        rc = make_owned_column(&out_aggs[i], dt, 1, has_valid, s);
        if (rc) break;
        const int32_t kind = aggs[i].kind & 0xFF;
        const bool valid = kind == PLGPU_AGG_SUM || kind == PLGPU_AGG_LEN || kind == PLGPU_AGG_COUNT;
        const size_t vb = dt == PLGPU_BOOL ? 8 : (size_t)std::max(dtype_bytes(dt), 1);
        hipError_t e = hipMemsetAsync((void*)out_aggs[i].values, 0, vb, s);
        if (e == hipSuccess && has_valid) e = hipMemsetAsync((void*)out_aggs[i].validity, valid ? 0x01 : 0x00, 1, s);
        if (e == hipSuccess && has_valid) e = hipMemsetAsync((uint8_t*)out_aggs[i].validity + 1, 0, 7, s);
        if (e != hipSuccess) rc = hip_fail(e, "empty reduction");
        out_aggs[i].null_count = (has_valid && !valid) ? 1 : 0;
    }
    if (rc == PLGPU_OK) {
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "empty reduction");
    }
    if (rc)
        for (int i = 0; i < naggs; ++i) plgpu_column_release(&out_aggs[i]);
    return rc;
}

PLGPU_API int plgpu_group_by_agg_ex(const plgpu_column* keys, int32_t nkeys, const plgpu_column* cols, int32_t ncols,
                                    const plgpu_agg_input* inputs, int32_t ninputs, const plgpu_instr* program,
                                    int32_t n_instr, const plgpu_agg* aggs, int32_t naggs, int32_t maintain_order,
                                    plgpu_column* out_keys, plgpu_column* out_aggs, plgpu_groupby_info* info,
                                    void* stream) {
    if (nkeys < 0 || nkeys > kMaxKeys) return fail(PLGPU_ERR_INVALID, "number of key columns must be 0..8");
    if (nkeys > 0 && (keys == nullptr || out_keys == nullptr)) return fail(PLGPU_ERR_INVALID, "keys / out_keys is NULL");
    if (ninputs < 0 || (ninputs > 0 && inputs == nullptr)) return fail(PLGPU_ERR_INVALID, "bad aggregation inputs");
    if (ncols < 0 || ncols > PLGPU_MAX_COLS) return fail(PLGPU_ERR_INVALID, "too many columns (max 8)");
    if (naggs > 0 && out_aggs == nullptr) return fail(PLGPU_ERR_INVALID, "out_aggs is NULL");
    for (int i = 0; i < naggs; ++i) std::memset(&out_aggs[i], 0, sizeof(plgpu_column));
    for (int i = 0; i < nkeys; ++i) std::memset(&out_keys[i], 0, sizeof(plgpu_column));
    Deriv d;
    int rc = classify_inputs(cols, ncols, inputs, ninputs, &d);
    if (rc) return rc;
    // var / std (fused second moment, DESIGN.md "var / std in one pass"):
    // every var column x adds two derived inputs, x * x rounded and its exact
    // error, whose exact sums next to x's give n * sum(x^2) - (sum x)^2
    // exactly; the rewritten kind carries the first of them in bits 16..27
    std::vector<plgpu_agg> ag(aggs, aggs + std::max(naggs, 0));
    int hi_of[PLGPU_MAX_COLS];
    for (int c = 0; c < PLGPU_MAX_COLS; ++c) hi_of[c] = -1;
    bool any_var = false;
    for (int i = 0; i < naggs; ++i) {
        const int base = aggs[i].kind & 0xFF;
        if (base != PLGPU_AGG_VAR && base != PLGPU_AGG_STD) continue;
        const int c = aggs[i].col;
        if (c < 0 || c >= ncols || cols[c].dtype != PLGPU_F64)
            return fail(PLGPU_ERR_INVALID, "var / std in one pass take a Float64 column");
        if (hi_of[c] < 0) {
            hi_of[c] = ncols + (int)d.in.size();
            for (int q = 0; q < 2; ++q) {
                DerivIn di;
                std::memset(&di, 0, sizeof di);
                di.kind = 3;
                di.ca = c;
                di.cb = -1;
                di.dop = (q == 0 ? DOP_SQHI : DOP_SQLO) | DOP_LIT;
                di.out_dtype = PLGPU_F64;
                d.in.push_back(di);
            }
        }
        ag[i].kind = (aggs[i].kind & 0xFFFF) | (hi_of[c] << 16);
        any_var = true;
    }
    const Deriv* dv = (ninputs > 0 || any_var) ? &d : nullptr;
    const plgpu_agg* ap = naggs > 0 ? ag.data() : aggs;
    if (nkeys == 0) return gb_keyless(cols, ncols, dv, program, n_instr, ap, naggs, out_aggs, info, stream);
    // one null-free 4-byte key (Int32 / UInt32: dates, Categorical codes)
    // of a large input: the packed path, whose fused kernel reads the 4-byte
    // key itself (fused key packing) instead of the generic kernel
    const bool narrow = nkeys == 1 && (keys[0].dtype == PLGPU_I32 || keys[0].dtype == PLGPU_U32) &&
                        keys[0].validity == nullptr && keys[0].length >= (int64_t(1) << 20) && options().fuse_keys;
    if (nkeys == 1 && dtype_is_int(keys[0].dtype) && !narrow)
        return gb_single_impl(&keys[0], cols, ncols, dv, program, n_instr, ap, naggs, maintain_order, &out_keys[0],
                              out_aggs, info, stream);
    return gb_multi_impl(keys, nkeys, cols, ncols, dv, program, n_instr, ap, naggs, maintain_order, out_keys,
                         out_aggs, info, stream);
}

// ------------------------------------------------------- var / std finalize
// polars-compute/src/moment.rs:126 VarState::finalize (used by
// polars-expr/src/reduce/var_std.rs): null when the non-null count is <=
// ddof, else sum of squared deviations / (count - ddof), a negative value
// clamped to 0 (NaN propagates); std takes the square root.
__global__ __launch_bounds__(256) void var_finalize_kernel(DevCol ss, DevCol cnt, int64_t n, int32_t ddof,
                                                           int32_t take_sqrt, double* __restrict__ out,
                                                           uint64_t* __restrict__ out_valid) {
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < n; i0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = i0 + threadIdx.x;
        bool valid = false;
        if (i < n) {
            const uint64_t c = dev_valid(cnt, i) ? dev_load(cnt, i) : 0;
            double v = 0.0;
            if (c > (uint64_t)ddof && dev_valid(ss, i)) {
                v = as_f64(dev_load(ss, i)) / (double)(c - (uint64_t)ddof);
                if (v < 0.0) v = 0.0;
                if (take_sqrt) v = __builtin_sqrt(v);
                valid = true;
            }
            out[i] = v;
        }
        const uint64_t w = __ballot(valid);
        if ((threadIdx.x & 63) == 0 && i < n) out_valid[i >> 6] = w;
    }
}

PLGPU_API int plgpu_var_finalize(const plgpu_column* sum_sq, const plgpu_column* count, int32_t ddof,
                                 int32_t take_sqrt, plgpu_column* out, void* stream) {
    hipStream_t s = as_stream(stream);
    if (sum_sq == nullptr || count == nullptr || out == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    std::memset(out, 0, sizeof *out);
    if (sum_sq->dtype != PLGPU_F64 || (count->dtype != PLGPU_U32 && count->dtype != PLGPU_I64))
        return fail(PLGPU_ERR_SCHEMA, "var finalize takes Float64 sums and UInt32 / Int64 counts");
    if (sum_sq->length != count->length) return fail(PLGPU_ERR_SHAPE, "columns differ in length");
    if (ddof < 0 || ddof > 255) return fail(PLGPU_ERR_INVALID, "ddof must be 0..255");
    const int64_t n = sum_sq->length;
    int rc = make_owned_column(out, PLGPU_F64, n, true, s);
    if (rc || n == 0) return rc;
    const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    var_finalize_kernel<<<g, 256, 0, s>>>(to_dev(*sum_sq), to_dev(*count), n, ddof, take_sqrt,
                                          (double*)out->values, (uint64_t*)out->validity);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        plgpu_column_release(out);
        return hip_fail(e, "var finalize");
    }
    return PLGPU_OK;
}

// ------------------------------------------------- per-row squared deviation
// Second pass of var / std for one fixed-width key column: every row's
// d = (x - mean[group(row)])^2, the group found in a small open-addressing
// table of the (unique) group keys; the null key is its own group.  Null
// when x is null, the row's key is not a group (rows the predicate dropped)
// or the mean is null.  Same arithmetic as x.cast(f64) - mean, squared.
constexpr uint32_t kSqEmpty = 0xFFFFFFFFu;

// Table slot: key, mean bits, group index | kSqNoMean when the mean is null.
constexpr uint32_t kSqNoMean = 0x80000000u;
constexpr int kSqLdsBits = 11;  // tables up to 2048 slots (40 KB) are staged in LDS per block

__global__ __launch_bounds__(256) void sq_build_kernel(DevCol gk, DevCol mean, int64_t ng, int bits,
                                                       uint64_t* __restrict__ tkey, uint64_t* __restrict__ tval,
                                                       uint32_t* __restrict__ tidx, uint32_t* __restrict__ null_g) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ng) return;
    const uint32_t tag = (uint32_t)g | (dev_valid(mean, g) ? 0u : kSqNoMean);
    if (!dev_valid(gk, g)) {
        null_g[0] = tag;
        null_g[1] = (uint32_t)dev_load(mean, g);
        null_g[2] = (uint32_t)(dev_load(mean, g) >> 32);
        return;
    }
    const uint64_t k = dev_load(gk, g);
    const uint32_t mask = (1u << bits) - 1;
    for (uint32_t h = hash_slot(k, bits);; h = (h + 1) & mask) {
        if (atomicCAS(&tidx[h], kSqEmpty, tag) == kSqEmpty) {
            tkey[h] = k;
            tval[h] = dev_load(mean, g);
            return;
        }
    }
}

__device__ __forceinline__ double sq_as_f64(const DevCol& c, int64_t r) {
    const uint64_t b = dev_load(c, r);
    switch (c.dtype) {
    case PLGPU_F64:
    case PLGPU_F32: return as_f64(b);  // register form
    case PLGPU_U64: return (double)b;
    default: return (double)(int64_t)b;  // signed ints sign-extended, unsigned / Boolean zero-extended
    }
}

// Four rows per thread per step (loads issued before the probes); the key
// table in LDS when it fits (kSqLdsBits), else read through the caches.
template <bool LDS>
__global__ __launch_bounds__(256) void sq_dev_kernel(DevCol rk, DevCol x, int64_t n, int bits,
                                                     const uint64_t* __restrict__ gkey,
                                                     const uint64_t* __restrict__ gval,
                                                     const uint32_t* __restrict__ gidx,
                                                     const uint32_t* __restrict__ null_g,
                                                     double* __restrict__ out, uint64_t* __restrict__ out_valid) {
    extern __shared__ uint64_t sq_lds[];
    const uint32_t slots = 1u << bits, mask = slots - 1;
    const uint64_t* tkey = gkey;
    const uint64_t* tval = gval;
    const uint32_t* tidx = gidx;
    if (LDS) {
        uint64_t* k = sq_lds;
        uint64_t* v = sq_lds + slots;
        uint32_t* t = (uint32_t*)(sq_lds + 2 * slots);
        for (uint32_t h = threadIdx.x; h < slots; h += blockDim.x) {
            k[h] = gkey[h];
            v[h] = gval[h];
            t[h] = gidx[h];
        }
        __syncthreads();
        tkey = k;
        tval = v;
        tidx = t;
    }
    const uint32_t null_tag = null_g[0];
    const uint64_t null_mean = (uint64_t)null_g[1] | ((uint64_t)null_g[2] << 32);
    constexpr int R = 4;
    for (int64_t base = (int64_t)blockIdx.x * 256 * R; base < n; base += (int64_t)gridDim.x * 256 * R) {
        uint64_t kk[R];
        double xv[R];
        bool kv[R], xok[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int64_t i = base + j * 256 + threadIdx.x;
            xok[j] = i < n && dev_valid(x, i);
            kv[j] = i < n && dev_valid(rk, i);
            kk[j] = i < n ? dev_load(rk, i) : 0;
            xv[j] = i < n ? sq_as_f64(x, i) : 0.0;
        }
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const int64_t i = base + j * 256 + threadIdx.x;
            uint32_t tag = kSqEmpty;
            uint64_t m = 0;
            if (xok[j]) {
                if (!kv[j]) {
                    tag = null_tag;
                    m = null_mean;
                } else {
                    for (uint32_t h = hash_slot(kk[j], bits);; h = (h + 1) & mask) {
                        const uint32_t t = tidx[h];
                        if (t == kSqEmpty) break;
                        if (tkey[h] == kk[j]) {
                            tag = t;
                            m = tval[h];
                            break;
                        }
                    }
                }
            }
            const bool valid = xok[j] && tag != kSqEmpty && !(tag & kSqNoMean);
            const double d = xv[j] - as_f64(m);
            if (i < n) out[i] = valid ? d * d : 0.0;
            const uint64_t w = __ballot(valid);
            if ((threadIdx.x & 63) == 0 && i < n) out_valid[i >> 6] = w;
        }
    }
}

PLGPU_API int plgpu_group_sq_dev(const plgpu_column* row_key, const plgpu_column* x, const plgpu_column* group_key,
                                 const plgpu_column* group_mean, plgpu_column* out, void* stream) {
    hipStream_t s = as_stream(stream);
    if (!row_key || !x || !group_key || !group_mean || !out) return fail(PLGPU_ERR_INVALID, "NULL argument");
    std::memset(out, 0, sizeof *out);
    const int32_t kt = row_key->dtype;
    if (kt != group_key->dtype || (!dtype_is_int(kt) && kt != PLGPU_BOOL))
        return fail(PLGPU_ERR_SCHEMA, "squared deviations take one integer / Boolean key of one dtype");
    if (x->dtype == PLGPU_STR || group_mean->dtype != PLGPU_F64)
        return fail(PLGPU_ERR_SCHEMA, "squared deviations take a numeric x and Float64 means");
    if (row_key->length != x->length || group_key->length != group_mean->length)
        return fail(PLGPU_ERR_SHAPE, "columns differ in length");
    const int64_t n = x->length, ng = group_key->length;
    if (ng >= (int64_t)1 << 30) return fail(PLGPU_ERR_SHAPE, "too many groups");
    int rc = make_owned_column(out, PLGPU_F64, n, true, s);
    if (rc || n == 0) return rc;
    int bits = 6;
    while (((int64_t)1 << bits) < 2 * ng) ++bits;
    const size_t slots = (size_t)1 << bits;
    uint64_t* tkey = nullptr;
    uint32_t* tidx = nullptr;
    // the library's stream-ordered cache, like every other scratch buffer
    if ((rc = dev_alloc((void**)&tkey, slots * 16, s)) || (rc = dev_alloc((void**)&tidx, slots * 4 + 12, s))) {
        dev_free(tkey, s);
        plgpu_column_release(out);
        return rc;
    }
    hipError_t e = hipMemsetAsync(tidx, 0xFF, slots * 4 + 12, s);
    uint64_t* tval = tkey + slots;
    uint32_t* null_g = tidx + slots;
    if (e == hipSuccess && ng > 0)
        sq_build_kernel<<<(unsigned)((ng + 255) / 256), 256, 0, s>>>(dev_col(*group_key), dev_col(*group_mean), ng,
                                                                     bits, tkey, tval, tidx, null_g);
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) {
        const int64_t steps = (n + 1023) / 1024;
        if (bits <= kSqLdsBits) {
            const unsigned g = (unsigned)std::min<int64_t>(steps, (int64_t)num_cus() * 8);
            sq_dev_kernel<true><<<g, 256, slots * 20, s>>>(dev_col(*row_key), dev_col(*x), n, bits, tkey, tval, tidx,
                                                            null_g, (double*)out->values, (uint64_t*)out->validity);
        } else {
            const unsigned g = (unsigned)std::min<int64_t>(steps, (int64_t)1 << 30);
            sq_dev_kernel<false><<<g, 256, 0, s>>>(dev_col(*row_key), dev_col(*x), n, bits, tkey, tval, tidx, null_g,
                                                   (double*)out->values, (uint64_t*)out->validity);
        }
        e = hipGetLastError();
    }
    dev_free(tkey, s);
    dev_free(tidx, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        plgpu_column_release(out);
        return hip_fail(e, "squared deviations");
    }
    return PLGPU_OK;
}
