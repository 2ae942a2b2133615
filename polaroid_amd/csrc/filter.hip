// filter.hip — expression evaluation and filter compaction on gfx950.
//
// plgpu_eval:        PhysicalExpr::evaluate for column / literal / binary
//                    expressions; Boolean results are bit-packed with one
//                    wave64 ballot per 64 rows (Arrow LSB-first layout).
// plgpu_filter*:     polars-compute/src/filter/mod.rs:18 (null mask = false),
//                    three launches: mask+tile counts -> tile scan -> stable
//                    scatter.  Each wave owns whole 64-row mask words, so the
//                    in-word rank is one popcount of (word & lanemask_lt).
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "plgpu_internal.hpp"
#include "scan.hpp"

namespace plgpu {

constexpr int kEvalThreads = 256;
constexpr int kTileRows = 4096;                 // rows per filter tile
constexpr int kTileWords = kTileRows / 64;      // 64 mask words per tile
constexpr int kFilterThreads = 256;             // 4 waves; 16 words per wave per tile

struct ColArgs {
    DevCol c[PLGPU_MAX_COLS];
};

static int grid_for(int64_t items, int threads, int max_blocks = 256 * 16) {
    int64_t b = (items + threads - 1) / threads;
    if (b < 1) b = 1;
    if (b > max_blocks) b = max_blocks;
    return (int)b;
}

// ---------------------------------------------------------------- eval
template <int SIMPLE>
__global__ __launch_bounds__(kEvalThreads) void eval_kernel(ColArgs cols, DevProgram prog, int64_t n,
                                                            void* __restrict__ out_values,
                                                            uint64_t* __restrict__ out_validity) {
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += stride) {
        const int64_t r = base + threadIdx.x;
        uint64_t v = 0;
        bool ok = false;
        if (r < n) {
            if (SIMPLE) {
                const DevCol& c = cols.c[prog.simple_col];
                ok = dev_valid(c, r);
                v = simple_pred(prog.simple_isf, prog.simple_op, dev_load(c, r), prog.simple_imm) ? 1 : 0;
            } else {
                RowVal rv = eval_row(prog.code, prog.n, cols.c, r);
                v = rv.v;
                ok = rv.valid;
            }
        }
        const uint64_t vbits = __ballot(ok);
        const int64_t word = r >> 6;
        if (prog.out_dtype == PLGPU_BOOL) {
            const uint64_t bbits = __ballot(ok && (v & 1));
            if (lane == 0 && base + (threadIdx.x & ~63) < n) {
                ((uint64_t*)out_values)[word] = bbits;
                out_validity[word] = vbits;
            }
        } else {
            if (r < n) dev_store(out_values, prog.out_dtype, r, ok ? v : 0ull);
            if (lane == 0 && base + (threadIdx.x & ~63) < n) out_validity[word] = vbits;
        }
    }
}

// ------------------------------------------------------------- filter
// Mask source: either a BOOL column (values & validity, null = false) or a
// lowered program.  Writes one u64 per 64 rows and one count per tile.  A
// thread owns rows it * 256 + tid (it < 16) of its tile: the simple-predicate
// form loads all 16 before the first ballot, so each wave keeps 16 loads in
// flight.
template <int SRC>  // 0 = bool column, 1 = simple predicate, 2 = program, 3 = simple on a null-free 8-byte column
__global__ __launch_bounds__(kFilterThreads) void filter_mask_kernel(ColArgs cols, DevProgram prog, DevCol mask,
                                                                     int64_t n, int64_t ntiles,
                                                                     uint64_t* __restrict__ mask_words,
                                                                     uint32_t* __restrict__ tile_counts) {
    constexpr int IT = kTileRows / kFilterThreads;
    __shared__ uint32_t wave_cnt[kFilterThreads / 64];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        uint32_t cnt = 0;
        bool sel[IT];
        if (SRC == 3) {
            // simple predicate over a null-free 8-byte column: 16 branch-free
            // loads (row index clamped at the end), then the compares
            const DevCol c = cols.c[prog.simple_col];
            const uint64_t* __restrict__ v = (const uint64_t*)c.values + c.offset;
            uint64_t x[IT];
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int64_t r = t * kTileRows + it * kFilterThreads + threadIdx.x;
                x[it] = __builtin_nontemporal_load(v + (r < n ? r : n - 1));
            }
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int64_t r = t * kTileRows + it * kFilterThreads + threadIdx.x;
                sel[it] = r < n && simple_pred(prog.simple_isf, prog.simple_op, x[it], prog.simple_imm);
            }
        } else {
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int64_t r = t * kTileRows + it * kFilterThreads + threadIdx.x;
                sel[it] = false;
                if (r < n) {
                    if (SRC == 0) {
                        sel[it] = dev_valid(mask, r) && (dev_load(mask, r) & 1);
                    } else if (SRC == 1) {
                        const DevCol& c = cols.c[prog.simple_col];
                        sel[it] = dev_valid(c, r) &&
                                  simple_pred(prog.simple_isf, prog.simple_op, dev_load(c, r), prog.simple_imm);
                    } else {
                        RowVal rv = eval_row(prog.code, prog.n, cols.c, r);
                        sel[it] = rv.valid && (rv.v & 1);
                    }
                }
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const uint64_t w = __ballot(sel[it]);
            if (lane == 0) mask_words[t * kTileWords + it * (kFilterThreads / 64) + wave] = w;
            cnt += (uint32_t)__popcll(w);
        }
        if (lane == 0) wave_cnt[wave] = cnt;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t s = 0;
            for (int w = 0; w < kFilterThreads / 64; ++w) s += wave_cnt[w];
            tile_counts[t] = s;
        }
        __syncthreads();
    }
}

__device__ __forceinline__ uint64_t wave_or64(uint64_t x) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x |= __shfl_xor(x, off, 64);
    return x;
}

// Stable scatter of one column by the mask words.
template <int EB>  // element bytes (1, 2, 4 or 8); 0 = bit-packed bool; 16 = the selected row ids
__global__ __launch_bounds__(kFilterThreads) void filter_scatter_kernel(DevCol col, int64_t n, int64_t ntiles,
                                                                        const uint64_t* __restrict__ mask_words,
                                                                        const uint64_t* __restrict__ tile_off,
                                                                        void* __restrict__ out_values,
                                                                        uint64_t* __restrict__ out_validity) {
    __shared__ uint64_t words[kTileWords];
    __shared__ uint32_t prefix[kTileWords];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const uint64_t lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        if (threadIdx.x < kTileWords) {
            uint64_t w = mask_words[t * kTileWords + threadIdx.x];
            words[threadIdx.x] = w;
            prefix[threadIdx.x] = (uint32_t)__popcll(w);
        }
        __syncthreads();
        if (threadIdx.x < 64) {  // inclusive scan of 64 counts in one wave
            uint32_t x = prefix[threadIdx.x];
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                uint32_t y = __shfl_up(x, off, 64);
                if (lane >= off) x += y;
            }
            prefix[threadIdx.x] = x - (uint32_t)__popcll(words[threadIdx.x]);
        }
        __syncthreads();
        const uint64_t base_off = tile_off[t];
        for (int it = 0; it < kTileRows / kFilterThreads; ++it) {
            const int wi = it * (kFilterThreads / 64) + wave;
            const uint64_t w = words[wi];
            if (w == 0) continue;  // wave-uniform
            const int64_t r = t * kTileRows + it * kFilterThreads + threadIdx.x;
            const bool sel = (w >> lane) & 1;
            const uint32_t rank = (uint32_t)__popcll(w & lt_mask);
            const uint64_t pos = base_off + prefix[wi] + rank;
            if (sel) {
                const int64_t p = col.offset + r;
                if (EB == 8) ((uint64_t*)out_values)[pos] = ((const uint64_t*)col.values)[p];
                else if (EB == 4) ((uint32_t*)out_values)[pos] = ((const uint32_t*)col.values)[p];
                else if (EB == 2) ((uint16_t*)out_values)[pos] = ((const uint16_t*)col.values)[p];
                else if (EB == 1) ((uint8_t*)out_values)[pos] = ((const uint8_t*)col.values)[p];
                else if (EB == 16) ((int64_t*)out_values)[pos] = r;  // row ids (string columns)
            }
            if (EB == 0 || col.validity != nullptr) {
                // Pack bits of the selected rows at their output ranks, then
                // OR the (<=64-bit) run into the output bitmap.
                const uint64_t wpos = base_off + prefix[wi];
                uint64_t vb = 0, bb = 0;
                if (sel) {
                    if (col.validity != nullptr && dev_valid(col, r)) vb = 1ull << rank;
                    if (col.validity == nullptr) vb = 1ull << rank;
                    if (EB == 0 && (dev_load(col, r) & 1)) bb = 1ull << rank;
                }
                vb = wave_or64(vb);
                if (EB == 0) bb = wave_or64(bb);
                if (lane == 0) {
                    const uint64_t word = wpos >> 6;
                    const int sh = (int)(wpos & 63);
                    const int cntw = __popcll(w);
                    (void)cntw;
                    atomicOr((unsigned long long*)&out_validity[word], (unsigned long long)(vb << sh));
                    if (sh != 0 && (vb >> (64 - sh)) != 0)
                        atomicOr((unsigned long long*)&out_validity[word + 1], (unsigned long long)(vb >> (64 - sh)));
                    if (EB == 0) {
                        uint64_t* ov = (uint64_t*)out_values;
                        atomicOr((unsigned long long*)&ov[word], (unsigned long long)(bb << sh));
                        if (sh != 0 && (bb >> (64 - sh)) != 0)
                            atomicOr((unsigned long long*)&ov[word + 1], (unsigned long long)(bb >> (64 - sh)));
                    }
                }
            }
        }
        __syncthreads();
    }
}

// Stable scatter of up to 8 null-free 8-byte columns in one launch: the
// tile's mask words and their prefix are read once, then every column's
// selected rows are copied (each thread's 16 loads of a column issued
// together).
struct Scatter8Args {
    const uint64_t* src[PLGPU_MAX_COLS];
    uint64_t* dst[PLGPU_MAX_COLS];
    int32_t ncols;
};

template <bool PIPE>
__global__ __launch_bounds__(kFilterThreads) void filter_scatter8_kernel(Scatter8Args a, int64_t n, int64_t ntiles,
                                                                         const uint64_t* __restrict__ mask_words,
                                                                         const uint64_t* __restrict__ tile_off) {
    constexpr int IT = kTileRows / kFilterThreads;
    __shared__ uint64_t words[kTileWords];
    __shared__ uint32_t prefix[kTileWords];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const uint64_t lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        if (threadIdx.x < kTileWords) {
            const uint64_t w = mask_words[t * kTileWords + threadIdx.x];
            words[threadIdx.x] = w;
            uint32_t x = (uint32_t)__popcll(w), c = x;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(x, off, 64);
                if (lane >= off) x += y;
            }
            prefix[threadIdx.x] = x - c;
        }
        __syncthreads();
        const uint64_t base_off = tile_off[t];
        uint64_t pos[IT];
        bool sel[IT];
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int wi = it * (kFilterThreads / 64) + wave;
            const uint64_t w = words[wi];
            sel[it] = (w >> lane) & 1;
            pos[it] = base_off + prefix[wi] + (uint32_t)__popcll(w & lt_mask);
        }
        // branch-free loads (row clamped at the end of the column): the
        // lines are fetched whole anyway; only the stores are predicated
        auto load_col = [&](int j, uint64_t (&v)[IT]) {
            const uint64_t* __restrict__ src = a.src[j];
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int64_t r = t * kTileRows + it * kFilterThreads + threadIdx.x;
                v[it] = __builtin_nontemporal_load(src + (r < n ? r : n - 1));
            }
        };
        if (PIPE) {
            // column j + 1's loads go out before column j's stores, so the
            // wave always has a column's lines in flight
            uint64_t v[IT], w[IT];
            load_col(0, v);
            for (int j = 0; j < a.ncols; ++j) {
                if (j + 1 < a.ncols) load_col(j + 1, w);
                uint64_t* __restrict__ dst = a.dst[j];
#pragma unroll
                for (int it = 0; it < IT; ++it)
                    if (sel[it]) dst[pos[it]] = v[it];
#pragma unroll
                for (int it = 0; it < IT; ++it) v[it] = w[it];
            }
        } else {
            for (int j = 0; j < a.ncols; ++j) {
                uint64_t v[IT];
                load_col(j, v);
                uint64_t* __restrict__ dst = a.dst[j];
#pragma unroll
                for (int it = 0; it < IT; ++it)
                    if (sel[it]) dst[pos[it]] = v[it];
            }
        }
        __syncthreads();
    }
}

// One pass for the common filter (a simple predicate over a null-free
// 8-byte column, every output column null-free and 8 bytes wide): each
// workgroup takes the next tile by ticket (tiles start in order), forms its
// mask words from the predicate column's registers, publishes its count,
// looks back over its predecessors' published counts for its output offset
// (decoupled look-back: a tile's word holds its count, flag kFtAgg, or its
// inclusive prefix, flag kFtIncl), publishes its inclusive prefix and
// scatters its selected rows as filter_scatter8_kernel does.  The predicate
// column is read once (its registers serve the scatter when it is an output
// column), and no mask words, tile scan or host round trip sit between the
// passes.  Every tile waits only on tiles with earlier tickets, which are
// already running, and tile 0 publishes its prefix without waiting, so every
// wave reaches its exit.
constexpr uint64_t kFtAgg = 1ull << 62, kFtIncl = 2ull << 62, kFtValue = (1ull << 62) - 1;

__device__ __forceinline__ uint64_t ft_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ft_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool PIPE>
__global__ __launch_bounds__(kFilterThreads) void filter_fused8_kernel(Scatter8Args a, const uint64_t* __restrict__ pcol,
                                                                       int32_t pj, DevProgram prog, int64_t n,
                                                                       uint64_t* __restrict__ status,
                                                                       uint32_t* __restrict__ ticket) {
    constexpr int IT = kTileRows / kFilterThreads;
    constexpr int NW = kFilterThreads / 64;
    __shared__ uint64_t words[kTileWords];
    __shared__ uint32_t prefix[kTileWords];
    __shared__ uint32_t wave_cnt[NW];
    __shared__ int64_t tile_sh;
    __shared__ uint64_t base_sh;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const uint64_t lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    if (threadIdx.x == 0) tile_sh = (int64_t)atomicAdd(ticket, 1u);
    __syncthreads();
    const int64_t t = tile_sh;
    // the columns in scatter order: the predicate column first (its rows are
    // already in registers), then the others
    auto col_at = [&](int k) { return k == 0 ? pj : (k - 1 < pj ? k - 1 : k); };
    auto load_col = [&](int j, uint64_t (&v)[IT]) {
        const uint64_t* __restrict__ src = a.src[j];
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int64_t r = t * kTileRows + it * kFilterThreads + threadIdx.x;
            v[it] = __builtin_nontemporal_load(src + (r < n ? r : n - 1));
        }
    };
    // the predicate column's rows of the tile (clamped at the end; rows
    // >= n are never selected)
    uint64_t v[IT], w[IT];
    bool sel[IT];
    {
        const uint64_t* __restrict__ src = pcol;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int64_t r = t * kTileRows + it * kFilterThreads + threadIdx.x;
            v[it] = __builtin_nontemporal_load(src + (r < n ? r : n - 1));
        }
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int64_t r = t * kTileRows + it * kFilterThreads + threadIdx.x;
        sel[it] = r < n && simple_pred(prog.simple_isf, prog.simple_op, v[it], prog.simple_imm);
        const uint64_t bw = __ballot(sel[it]);
        if (lane == 0) words[it * NW + wave] = bw;
        cnt += (uint32_t)__popcll(bw);
    }
    if (lane == 0) wave_cnt[wave] = cnt;
    __syncthreads();
    // the next column's loads go out before the look-back (they do not
    // depend on the tile's output offset)
    if (PIPE && a.ncols > 1) load_col(col_at(1), w);
    if (wave == 0) {
        uint64_t total = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) total += wave_cnt[q];
        // publish the count (tile 0: its inclusive prefix), then look back
        if (lane == 0) ft_store(&status[t], (t == 0 ? kFtIncl : kFtAgg) | total);
        uint64_t excl = 0;
        int64_t j0 = t - 1;
        while (j0 >= 0) {
            const int64_t j = j0 - lane;
            const uint64_t st = j >= 0 ? ft_load(&status[j]) : kFtIncl;
            const uint64_t flag = st & ~kFtValue;
            const uint64_t incl = __ballot(flag == kFtIncl);
            const uint64_t ready = __ballot(flag != 0);
            const int first = incl ? __builtin_ctzll(incl) : 64;  // nearest inclusive predecessor
            const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1);
            if ((ready & need) != need) {
                __builtin_amdgcn_s_sleep(1);
                continue;  // a predecessor in the window has not published yet
            }
            uint64_t x = lane <= first ? (st & kFtValue) : 0ull;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
            excl += x;
            if (first < 64) break;
            j0 -= 64;
        }
        if (lane == 0) {
            if (t > 0) ft_store(&status[t], kFtIncl | (excl + total));
            base_sh = excl;
        }
        // the tile's 64 mask words' exclusive prefix
        const uint64_t mw = words[lane];
        uint32_t px = (uint32_t)__popcll(mw), c = px;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(px, off, 64);
            if (lane >= off) px += y;
        }
        prefix[lane] = px - c;
    }
    __syncthreads();
    uint64_t* const* dsts = a.dst;
    const uint64_t base_off = base_sh;
    uint32_t lp[IT];  // output position within the tile's selected rows
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int wi = it * NW + wave;
        lp[it] = prefix[wi] + (uint32_t)__popcll(words[wi] & lt_mask);
    }
    for (int k = 0; k < a.ncols; ++k) {
        if (!PIPE && k > 0) load_col(col_at(k), v);
        uint64_t* __restrict__ dst = dsts[col_at(k)] + base_off;
#pragma unroll
        for (int it = 0; it < IT; ++it)
            if (sel[it]) dst[lp[it]] = v[it];
        if (PIPE && k + 1 < a.ncols) {
#pragma unroll
            for (int it = 0; it < IT; ++it) v[it] = w[it];
            if (k + 2 < a.ncols) load_col(col_at(k + 2), w);
        }
    }
}

static ColArgs pack_cols(const plgpu_column* cols, int32_t ncols) {
    ColArgs a;
    std::memset(&a, 0, sizeof a);
    for (int i = 0; i < ncols && i < PLGPU_MAX_COLS; ++i) {
        a.c[i].values = cols[i].values;
        a.c[i].validity = cols[i].validity;
        a.c[i].offset = cols[i].offset;
        a.c[i].dtype = cols[i].dtype;
    }
    return a;
}

static int check_cols(const plgpu_column* cols, int32_t ncols, int64_t* n) {
    if (ncols < 0 || ncols > PLGPU_MAX_COLS) return fail(PLGPU_ERR_INVALID, "too many columns (max 8)");
    if (ncols == 0) { *n = 0; return PLGPU_OK; }
    *n = cols[0].length;
    for (int i = 0; i < ncols; ++i) {
        if (cols[i].length != *n)
            return fail(PLGPU_ERR_SHAPE, "all columns must have the same length");
        if (cols[i].values == nullptr && cols[i].length > 0)
            return fail(PLGPU_ERR_INVALID, "column has no values buffer");
    }
    return PLGPU_OK;
}

// Shared body of plgpu_filter / plgpu_filter_expr.
static int run_filter(const plgpu_column* cols, int32_t ncols, int src, const DevProgram* prog,
                      const plgpu_column* mask, plgpu_column* out_cols, int64_t* out_len, hipStream_t s) {
    int64_t n = 0;
    int rc = check_cols(cols, ncols, &n);
    if (rc) return rc;
    if (src == 0) {
        if (mask->dtype != PLGPU_BOOL) {
            return fail(PLGPU_ERR_SCHEMA, "filter predicate must be of type `Boolean`");
        }
        if (ncols > 0 && mask->length != n) return fail(PLGPU_ERR_SHAPE, "filter's length differs from that of the mask");
        if (ncols == 0) n = mask->length;
    }
    for (int i = 0; i < ncols; ++i) std::memset(&out_cols[i], 0, sizeof(plgpu_column));
    const int64_t ntiles = (n + kTileRows - 1) / kTileRows;
    ColArgs ca = pack_cols(cols, ncols);
    DevCol md;
    std::memset(&md, 0, sizeof md);
    if (src == 0) {
        md.values = mask->values;
        md.validity = mask->validity;
        md.offset = mask->offset;
        md.dtype = PLGPU_BOOL;
    }
    DevProgram dp;
    if (prog) dp = *prog;
    else std::memset(&dp, 0, sizeof dp);

    // the one-pass form (filter_fused8_kernel): a simple predicate over a
    // null-free 8-byte column, every column null-free and 8 bytes wide, and
    // output columns allocated at the input's length (their length set to
    // the selected count afterwards) within a quarter of the free memory.
    // Off by default (measured slower, DESIGN "Filter compaction"): it
    // OVER-ALLOCATES -- each output keeps n * 8 bytes for the result's
    // lifetime -- and the free/4 guard makes the choice depend on memory
    // pressure; size the outputs from a count before turning it on.
    bool all8 = ncols > 0 && src != 0 && dp.simple && options().filt_fused != 0 && n > 0;
    for (int i = 0; i < ncols && all8; ++i)
        all8 = cols[i].dtype != PLGPU_STR && cols[i].dtype != PLGPU_BOOL && cols[i].validity == nullptr &&
               dtype_bytes(cols[i].dtype) == 8;
    if (all8) {
        size_t fr = 0, tot = 0;
        all8 = hipMemGetInfo(&fr, &tot) == hipSuccess && (uint64_t)ncols * (uint64_t)n * 8 <= fr / 4;
    }
    if (all8) {
        uint64_t* status = nullptr;  // ntiles words + the ticket
        if ((rc = dev_alloc((void**)&status, (ntiles + 1) * 8, s))) return rc;
        Scatter8Args sa;
        std::memset(&sa, 0, sizeof sa);
        for (int i = 0; i < ncols && !rc; ++i) {
            rc = make_owned_column(&out_cols[i], cols[i].dtype, n, false, s);
            sa.src[i] = (const uint64_t*)cols[i].values + cols[i].offset;
            sa.dst[i] = rc ? nullptr : (uint64_t*)out_cols[i].values;
        }
        sa.ncols = ncols;
        uint64_t last = 0;
        if (!rc) {
            hipError_t e = hipMemsetAsync(status, 0, (ntiles + 1) * 8, s);
            const plgpu_column& pc = cols[dp.simple_col];
            const uint64_t* pcol = (const uint64_t*)pc.values + pc.offset;
            if (e == hipSuccess) {
                KtScope kt("filter_fused8_kernel", s);
                if (options().filt_pipe != 0)
                    filter_fused8_kernel<true><<<(unsigned)ntiles, kFilterThreads, 0, s>>>(
                        sa, pcol, dp.simple_col, dp, n, status, (uint32_t*)(status + ntiles));
                else
                    filter_fused8_kernel<false><<<(unsigned)ntiles, kFilterThreads, 0, s>>>(
                        sa, pcol, dp.simple_col, dp, n, status, (uint32_t*)(status + ntiles));
                e = hipGetLastError();
            }
            if (e == hipSuccess) e = hipMemcpyAsync(&last, status + ntiles - 1, 8, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) rc = hip_fail(e, "filter_fused8_kernel");
            if (!rc && (last & ~kFtValue) != kFtIncl) rc = fail(PLGPU_ERR_CAPACITY, "internal: filter prefix not published");
        }
        dev_free(status, s);
        if (rc) {
            for (int i = 0; i < ncols; ++i) plgpu_column_release(&out_cols[i]);
            return rc;
        }
        const int64_t total = (int64_t)(last & kFtValue);
        for (int i = 0; i < ncols; ++i) out_cols[i].length = total;
        *out_len = total;
        return PLGPU_OK;
    }

    uint64_t* mask_words = nullptr;
    uint32_t* counts = nullptr;
    uint64_t* offs = nullptr;  // ntiles offsets + 1 total
    uint64_t* scan_part = nullptr;
    uint64_t total = 0;
    if (ntiles > 0) {
        if ((rc = dev_alloc((void**)&mask_words, ntiles * kTileWords * 8, s))) return rc;
        if ((rc = dev_alloc((void**)&counts, ntiles * 4, s))) { dev_free(mask_words, s); return rc; }
        if ((rc = dev_alloc((void**)&offs, (ntiles + 1) * 8, s)) ||
            (rc = dev_alloc((void**)&scan_part, ((ntiles + kScanChunk - 1) / kScanChunk + 1) * 8, s))) {
            dev_free(mask_words, s);
            dev_free(counts, s);
            dev_free(offs, s);
            return rc;
        }
        const int g = grid_for(ntiles, 1, 256 * 8);
        {
            KtScope kt("filter_mask_kernel", s);
            if (src == 0)
                filter_mask_kernel<0><<<g, kFilterThreads, 0, s>>>(ca, dp, md, n, ntiles, mask_words, counts);
            else if (dp.simple && cols[dp.simple_col].validity == nullptr &&
                     dtype_bytes(cols[dp.simple_col].dtype) == 8)
                filter_mask_kernel<3><<<g, kFilterThreads, 0, s>>>(ca, dp, md, n, ntiles, mask_words, counts);
            else if (dp.simple)
                filter_mask_kernel<1><<<g, kFilterThreads, 0, s>>>(ca, dp, md, n, ntiles, mask_words, counts);
            else
                filter_mask_kernel<2><<<g, kFilterThreads, 0, s>>>(ca, dp, md, n, ntiles, mask_words, counts);
        }
        {
            KtScope kt("filter_tile_scan", s);
            PLGPU_HIP(scan_exclusive<uint32_t>(counts, ntiles, offs, scan_part, s));
        }
        PLGPU_HIP(hipMemcpyAsync(&total, offs + ntiles, 8, hipMemcpyDeviceToHost, s));
        PLGPU_HIP(hipStreamSynchronize(s));
    }
    int64_t* sel_rows = nullptr;  // selected row ids, for string columns
    for (int i = 0; i < ncols && !rc; ++i) {
        if (cols[i].dtype != PLGPU_STR) continue;
        if (sel_rows == nullptr) {
            if ((rc = dev_alloc((void**)&sel_rows, std::max<uint64_t>(total, 1) * 8, s))) break;
            if (total > 0) {
                DevCol rows;
                std::memset(&rows, 0, sizeof rows);
                filter_scatter_kernel<16><<<grid_for(ntiles, 1, 256 * 8), kFilterThreads, 0, s>>>(
                    rows, n, ntiles, mask_words, offs, (void*)sel_rows, nullptr);
                PLGPU_HIP(hipGetLastError());
            }
        }
        rc = str_gather(dev_col(cols[i]), nullptr, sel_rows, nullptr, 0, (int64_t)total, cols[i].validity != nullptr,
                        &out_cols[i], s);
    }
    // null-free 8-byte columns: one multi-column scatter launch
    auto wide8 = [&](int i) {
        return cols[i].dtype != PLGPU_STR && cols[i].dtype != PLGPU_BOOL && cols[i].validity == nullptr &&
               dtype_bytes(cols[i].dtype) == 8;
    };
    Scatter8Args sa;
    std::memset(&sa, 0, sizeof sa);
    for (int i = 0; i < ncols && !rc; ++i) {
        if (!wide8(i)) continue;
        rc = make_owned_column(&out_cols[i], cols[i].dtype, (int64_t)total, false, s);
        if (rc) break;
        sa.src[sa.ncols] = (const uint64_t*)cols[i].values + cols[i].offset;
        sa.dst[sa.ncols] = (uint64_t*)out_cols[i].values;
        ++sa.ncols;
    }
    if (!rc && sa.ncols > 0 && total > 0) {
        KtScope kt("filter_scatter8_kernel", s);
        if (options().filt_pipe != 0)
            filter_scatter8_kernel<true><<<grid_for(ntiles, 1, 256 * 8), kFilterThreads, 0, s>>>(sa, n, ntiles,
                                                                                               mask_words, offs);
        else
            filter_scatter8_kernel<false><<<grid_for(ntiles, 1, 256 * 8), kFilterThreads, 0, s>>>(sa, n, ntiles,
                                                                                                mask_words, offs);
        PLGPU_HIP(hipGetLastError());
    }
    for (int i = 0; i < ncols && !rc; ++i) {
        if (cols[i].dtype == PLGPU_STR || wide8(i)) continue;
        const bool need_valid = cols[i].validity != nullptr;
        rc = make_owned_column(&out_cols[i], cols[i].dtype, (int64_t)total,
                               need_valid || cols[i].dtype == PLGPU_BOOL, s);
        if (rc) break;
        if (total == 0) continue;
        if (out_cols[i].validity)
            PLGPU_HIP(hipMemsetAsync((void*)out_cols[i].validity, 0, ((total + 63) / 64) * 8, s));
        if (cols[i].dtype == PLGPU_BOOL) {
            PLGPU_HIP(hipMemsetAsync((void*)out_cols[i].values, 0, ((total + 63) / 64) * 8, s));
        }
        DevCol dc = ca.c[i];
        const int g = grid_for(ntiles, 1, 256 * 8);
        uint64_t* ovalid = (uint64_t*)out_cols[i].validity;
        if (cols[i].dtype == PLGPU_BOOL)
            filter_scatter_kernel<0><<<g, kFilterThreads, 0, s>>>(dc, n, ntiles, mask_words, offs,
                                                                  (void*)out_cols[i].values, ovalid);
        else if (dtype_bytes(cols[i].dtype) == 8)
            filter_scatter_kernel<8><<<g, kFilterThreads, 0, s>>>(dc, n, ntiles, mask_words, offs,
                                                                  (void*)out_cols[i].values, ovalid);
        else if (dtype_bytes(cols[i].dtype) == 4)
            filter_scatter_kernel<4><<<g, kFilterThreads, 0, s>>>(dc, n, ntiles, mask_words, offs,
                                                                  (void*)out_cols[i].values, ovalid);
        else if (dtype_bytes(cols[i].dtype) == 2)
            filter_scatter_kernel<2><<<g, kFilterThreads, 0, s>>>(dc, n, ntiles, mask_words, offs,
                                                                  (void*)out_cols[i].values, ovalid);
        else
            filter_scatter_kernel<1><<<g, kFilterThreads, 0, s>>>(dc, n, ntiles, mask_words, offs,
                                                                  (void*)out_cols[i].values, ovalid);
        PLGPU_HIP(hipGetLastError());
        if (!need_valid && cols[i].dtype == PLGPU_BOOL) out_cols[i].null_count = 0;
    }
    dev_free(mask_words, s);
    dev_free(counts, s);
    dev_free(offs, s);
    dev_free(scan_part, s);
    dev_free(sel_rows, s);
    if (rc) {
        for (int i = 0; i < ncols; ++i) plgpu_column_release(&out_cols[i]);
        return rc;
    }
    *out_len = (int64_t)total;
    return PLGPU_OK;
}

}  // namespace plgpu

using namespace plgpu;

PLGPU_API int plgpu_eval(const plgpu_column* cols, int32_t ncols, const plgpu_instr* program, int32_t n_instr,
                         plgpu_column* out, void* stream) {
    hipStream_t s = as_stream(stream);
    int64_t n = 0;
    int rc = check_cols(cols, ncols, &n);
    if (rc) return rc;
    DevProgram dp;
    if ((rc = lower_program(cols, ncols, program, n_instr, &dp))) return rc;
    if (ncols == 0) return fail(PLGPU_ERR_INVALID, "eval needs at least one column to define the length");
    if ((rc = make_owned_column(out, dp.out_dtype, n, true, s))) return rc;
    if (n == 0) return PLGPU_OK;
    ColArgs ca = pack_cols(cols, ncols);
    const int g = grid_for(n, kEvalThreads);
    if (dp.simple)
        eval_kernel<1><<<g, kEvalThreads, 0, s>>>(ca, dp, n, (void*)out->values, (uint64_t*)out->validity);
    else
        eval_kernel<0><<<g, kEvalThreads, 0, s>>>(ca, dp, n, (void*)out->values, (uint64_t*)out->validity);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        plgpu_column_release(out);
        return hip_fail(e, "eval_kernel launch");
    }
    return PLGPU_OK;
}

PLGPU_API int plgpu_filter(const plgpu_column* cols, int32_t ncols, const plgpu_column* mask,
                           plgpu_column* out_cols, int64_t* out_len, void* stream) {
    if (mask == nullptr) return fail(PLGPU_ERR_INVALID, "mask is NULL");
    return run_filter(cols, ncols, 0, nullptr, mask, out_cols, out_len, as_stream(stream));
}

PLGPU_API int plgpu_filter_expr(const plgpu_column* cols, int32_t ncols, const plgpu_instr* program,
                                int32_t n_instr, plgpu_column* out_cols, int64_t* out_len, void* stream) {
    DevProgram dp;
    int rc = lower_program(cols, ncols, program, n_instr, &dp);
    if (rc) return rc;
    if (dp.out_dtype != PLGPU_BOOL) {
        return fail(PLGPU_ERR_SCHEMA, "filter predicate must be of type `Boolean`");
    }
    return run_filter(cols, ncols, dp.simple ? 1 : 2, &dp, nullptr, out_cols, out_len, as_stream(stream));
}
