/*
 * polaroid_gpu.h — C-ABI of the MI355X columnar executor backend.
 *
 * This is the drop-in boundary a Polars host (Rust, via `extern "C"` +
 * bindgen, or Python via ctypes) binds to run the filter / arithmetic /
 * comparison / hash-group-by-aggregation hot path on gfx950.  Only plain C
 * types cross it: device pointers, lengths, Arrow bit-packed validity
 * bitmaps (LSB-first, Arrow offset semantics), status codes.  No torch or
 * HIP types appear in any signature; `stream` is an opaque hipStream_t
 * (NULL = the library's default stream).
 *
 * Each entry point names the reference interface it replaces
 * (paths relative to /root/reference/crates).
 *
 * Column ownership follows the Arrow C data interface: a column produced by
 * the library carries a non-NULL `release` callback that the consumer must
 * call exactly once; borrowed input columns have `release == NULL`.
 */
#ifndef POLAROID_GPU_H
#define POLAROID_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PLGPU_ABI_VERSION 1

/* ---------------------------------------------------------------- status */
/* Error classes mirror polars_error::PolarsError variants
 * (polars-error/src/lib.rs) so the host can map them 1:1. */
enum plgpu_status {
    PLGPU_OK = 0,
    PLGPU_ERR_INVALID = -1,        /* InvalidOperation                      */
    PLGPU_ERR_SCHEMA = -2,         /* SchemaMismatch / ComputeError (dtype)  */
    PLGPU_ERR_SHAPE = -3,          /* ShapeMismatch (column lengths differ)  */
    PLGPU_ERR_OOM = -4,            /* device allocation failed               */
    PLGPU_ERR_HIP = -5,            /* HIP runtime error                      */
    PLGPU_ERR_NO_DEVICE = -6,      /* no gfx950 device visible               */
    PLGPU_ERR_CAPACITY = -7        /* internal table overflow (retry failed) */
};

/* ---------------------------------------------------------------- dtypes */
/* Physical types of the path; Arrow format string in the comment. */
enum plgpu_dtype {
    PLGPU_BOOL = 1, /* "b"  bit-packed values, LSB first               */
    PLGPU_I32 = 2,  /* "i"                                             */
    PLGPU_I64 = 3,  /* "l"                                             */
    PLGPU_F64 = 4,  /* "g"                                             */
    PLGPU_U32 = 5,  /* "I"  polars IdxSize (count / len outputs)       */
    PLGPU_STR = 6,  /* "U"  large_string: int64 offsets in `values`,
                       UTF-8 bytes in `data` (polars String / Binary)   */
    PLGPU_I8 = 7,   /* "c"                                             */
    PLGPU_I16 = 8,  /* "s"                                             */
    PLGPU_U8 = 9,   /* "C"                                             */
    PLGPU_U16 = 10, /* "S"                                             */
    PLGPU_U64 = 11, /* "L"                                             */
    PLGPU_F32 = 12  /* "f"                                             */
    /* polars' temporal types travel as their physical integers: Datetime /
     * Duration as PLGPU_I64, Date as PLGPU_I32 (the host keeps the unit). */
};

/* One Arrow array in device memory (Arrow C Device Data Interface,
 * ARROW_DEVICE_ROCM = 10, flattened to the two buffers the path uses). */
typedef struct plgpu_column {
    int32_t dtype;            /* enum plgpu_dtype                                  */
    int32_t device_id;        /* HIP device ordinal                                */
    int64_t length;           /* logical length                                    */
    int64_t offset;           /* Arrow offset (elements; bits for PLGPU_BOOL)      */
    int64_t null_count;       /* -1 = unknown                                      */
    const void* values;       /* device ptr, Arrow buffers[1]                      */
    const uint8_t* validity;  /* device ptr, Arrow buffers[0]; NULL = all valid    */
    void (*release)(struct plgpu_column*); /* NULL for borrowed columns             */
    void* private_data;
    const uint8_t* data;      /* device ptr, Arrow buffers[2] of PLGPU_STR (bytes); */
                              /* NULL for fixed-width columns                       */
} plgpu_column;

/* ------------------------------------------------------- expression ISA */
/* A physical expression (polars-expr/src/expressions/{binary,column,
 * literal}.rs) is lowered to a postfix program evaluated per row on the
 * GPU.  Semantics per op follow the reference kernels cited below. */
enum plgpu_opcode {
    PLGPU_OP_COL = 1,       /* push column[arg]                                 */
    PLGPU_OP_LIT_F64 = 2,   /* push f64 literal imm.f64                         */
    PLGPU_OP_LIT_I64 = 3,   /* push i64 literal imm.i64                         */
    PLGPU_OP_LIT_BOOL = 4,  /* push bool literal imm.i64 != 0                   */
    PLGPU_OP_LIT_NULL = 5,  /* push typed null (arg = plgpu_dtype)              */
    /* arithmetic: polars-compute/src/arithmetic/{signed,unsigned,float}.rs.
     * Operands are coerced to their supertype first
     * (polars-core/src/utils/supertype.rs, dynamic literals included: an
     * integer literal takes the smallest type that holds it, a float
     * literal takes the float column's type or Float64), and integer
     * results wrap at the supertype's width.  LIT_I64 / LIT_F64 are the
     * dynamic (untyped) literals; CAST gives a literal a concrete type. */
    PLGPU_OP_ADD = 10,
    PLGPU_OP_SUB = 11,
    PLGPU_OP_MUL = 12,
    PLGPU_OP_TRUEDIV = 13,  /* ints -> Float64; float / literal = x * (1 / lit)
                               (true_div_scalar, arithmetic/float.rs:113)    */
    PLGPU_OP_NEG = 14,
    PLGPU_OP_ABS = 15,
    PLGPU_OP_CAST_F64 = 16,
    PLGPU_OP_FLOORDIV = 17, /* ints: floor division, x // 0 = null
                               (floor_divmod.rs:39); floats: floor(a / b)    */
    PLGPU_OP_MOD = 18,      /* ints: remainder with the divisor's sign, x % 0
                               = null; floats: a - b * floor(a / b)          */
    PLGPU_OP_DIVIDE = 19,   /* Operator::Divide (legacy_div, arithmetic/mod.rs:40):
                               floor division for ints, true division for floats */
    PLGPU_OP_CAST = 50,     /* cast to dtype `arg`; imm.i64: 0 = non-strict
                               (a value that does not fit -> null), 1 =
                               overflowing (integers wrap)                   */
    PLGPU_OP_XOR = 51,      /* Boolean xor (null if either is null); bitwise on ints */
    PLGPU_OP_FILL_NULL = 52,/* [x, fill] -> x where valid, else fill         */
    PLGPU_OP_IF_ELSE = 53,  /* [cond, then, otherwise] -> when(cond).then().otherwise();
                               a null condition selects `otherwise`
                               (polars-compute/src/if_then_else)             */
    /* comparisons: TotalOrd semantics, polars-utils/src/total_ord.rs:317-368
     * (NaN == NaN, NaN greatest); null in -> null out. */
    PLGPU_OP_EQ = 20,
    PLGPU_OP_NE = 21,
    PLGPU_OP_LT = 22,
    PLGPU_OP_LE = 23,
    PLGPU_OP_GT = 24,
    PLGPU_OP_GE = 25,
    PLGPU_OP_EQ_MISSING = 26, /* null == null, never null out */
    PLGPU_OP_NE_MISSING = 27,
    /* boolean: Kleene logic, polars-compute/src/bitwise + ops::and/or;
     * AND / OR / XOR of integers are bitwise */
    PLGPU_OP_AND = 30,
    PLGPU_OP_OR = 31,
    PLGPU_OP_NOT = 32,
    PLGPU_OP_IS_NULL = 33,
    PLGPU_OP_IS_NOT_NULL = 34,
    PLGPU_OP_IS_NAN = 35,
    PLGPU_OP_IS_FINITE = 36,
    /* String literal pattern tests (plgpu_str_compare only):
     * polars-ops/src/chunked_array/binary/namespace.rs:85 starts_with, :78
     * ends_with, strings/namespace.rs:332 contains_literal */
    PLGPU_OP_STR_STARTS_WITH = 40,
    PLGPU_OP_STR_ENDS_WITH = 41,
    PLGPU_OP_STR_CONTAINS = 42
};

typedef struct plgpu_instr {
    int32_t op;   /* enum plgpu_opcode */
    int32_t arg;  /* column index / dtype */
    union {
        double f64;
        int64_t i64;
    } imm;
} plgpu_instr;

#define PLGPU_MAX_STACK 8
#define PLGPU_MAX_PROGRAM 64
#define PLGPU_MAX_COLS 8

/* -------------------------------------------------------- aggregations */
/* polars-core/src/frame/group_by/aggregations/mod.rs (agg_sum :581,
 * agg_mean :659, agg_min/agg_max) and the streaming reductions the lazy
 * engine actually runs for a partitionable group-by
 * (polars-mem-engine/src/planner/lp.rs:648 -> polars-expr/src/reduce/
 * {sum,mean,min_max,count,len}.rs). */
enum plgpu_agg_kind {
    PLGPU_AGG_SUM = 1,   /* f64: correctly-rounded exact sum; i64: wrapping  */
    PLGPU_AGG_MEAN = 2,  /* f64 out, null if no non-null values              */
    PLGPU_AGG_MIN = 3,   /* NaN ignored unless all NaN (min_ignore_nan)      */
    PLGPU_AGG_MAX = 4,
    PLGPU_AGG_COUNT = 5, /* non-null count, u32 (IdxSize)                    */
    PLGPU_AGG_LEN = 6,   /* group length incl. nulls, u32                    */
    PLGPU_AGG_FIRST = 7, /* value of the group's first row, null included    */
    PLGPU_AGG_LAST = 8,  /* ... last row (reduce/first_last.rs First / Last) */
    PLGPU_AGG_VAR = 9,   /* variance of a Float64 column, f64 out; ddof in bits */
                         /* 8..15 of the kind (plgpu_group_by_agg_ex only)      */
    PLGPU_AGG_STD = 10   /* its square root                                    */
};

typedef struct plgpu_agg {
    int32_t kind; /* enum plgpu_agg_kind */
    int32_t col;  /* input column index */
} plgpu_agg;

/* An aggregation input computed from the columns: the elementwise
 * expression under an aggregation (`(close * volume).sum()`), which the
 * reference's partitionable group-by pre-aggregates directly
 * (polars-plan/src/plans/aexpr/properties/general.rs:335 can_pre_agg).
 * `program` is an expression program over the call's columns. */
typedef struct plgpu_agg_input {
    const plgpu_instr* program;
    int32_t n_instr;
    int32_t _pad;
} plgpu_agg_input;

/* Diagnostics of one group-by call (for tests / bench / rocprof cross-check). */
typedef struct plgpu_groupby_info {
    int64_t rows_in;
    int64_t rows_selected;       /* rows passing the fused predicate            */
    int64_t groups;
    int64_t global_path_rows;    /* rows that missed the LDS table             */
    int32_t reruns;              /* fixed-point window / table-size retries    */
    int32_t lds_slots;           /* per-workgroup LDS hash-table capacity      */
    int32_t grid;                /* workgroups in the main launch              */
    int32_t sum_inexact;         /* bit i: f64 sum acc i rounded below window  */
    int64_t table_capacity;      /* global hash-table slots                    */
    double main_kernel_ms;       /* device time of the aggregation kernel(s)   */
    int32_t path;                /* 0 generic, 1 fast, 2 fast sum-only, 3 partitioned,
                                    4 fast variance triple (one var / std column)   */
    int32_t sum_limbs;           /* 40-bit LDS limbs per f64 sum (2 or 3)      */
    int32_t local_range;         /* 1: range-local fused kernel (clustered keys) */
    int32_t register_runs;       /* 1: fused kernel with per-lane register runs (sorted keys) */
    int32_t key_pack;            /* key columns packed in the fused kernel's registers (0: a key / code column) */
    int32_t part_layout;         /* partitioned path: partition bits | scatter passes << 8 (0: not partitioned) */
} plgpu_groupby_info;

/* ---------------------------------------------------------------- basics */
int plgpu_abi_version(void);
const char* plgpu_last_error(void);           /* thread-local message        */
int plgpu_device_count(int* out);
int plgpu_set_device(int device);
int plgpu_synchronize(void* stream);

/* Stream-ordered device allocator (native caching pool). */
int plgpu_alloc(void** out_ptr, size_t bytes, void* stream);
int plgpu_free(void* ptr, void* stream);
int plgpu_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream);
int plgpu_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream);
/* n device -> host copies (dst[i] <- src[i], bytes[i]) with one
 * synchronisation: small ranges go through a library-owned pinned buffer.
 * Returns when every dst holds its bytes (a query's result columns). */
int plgpu_memcpy_d2h_many(int32_t n, void* const* dst, const void* const* src, const size_t* bytes, void* stream);
int plgpu_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream);

/* Test hooks and diagnostics, each read once from the environment variable
 * PLGPU_<NAME> (upper case) when the library loads and settable here:
 *   "ktime"       1: time the named kernels with HIP events (plgpu_ktime_read)
 *   "fuse_keys"   0: multi-key / Categorical group-bys write their packed
 *                 code column instead of forming the codes in the fused kernel
 *   "plan_cache"  0: every group-by samples its inputs (no reuse of the plan
 *                 statistics of a recent group-by over the same columns)
 *   "grid_rounds" > 0: the fused group-by grid in that many rounds of resident
 *                 workgroups (A/B; 0: scaled with the input)
 *   "debug"       per-attempt group-by diagnostics on stderr
 *   "no_pack"     multi-key operators hash their key tuples even when the
 *                 tuples would pack into one Int64 (exercises the hashed path)
 *   "mk_collide"  a 3-bit first tuple hash (forces the collision / re-seed path)
 *   "runs"        -1: the plan decides; 0 / 1 force the sorted-key variant of
 *                 the fused group-by kernel
 *   "local"       -1: the plan decides; 0 keeps the group-by off the
 *                 range-local fused kernel (clustered keys)
 *   "gb_path"     -1: the plan decides; forces the single-key group-by's
 *                 path where its inputs allow it: 0 generic kernel on the
 *                 global table, 1 generic kernel with LDS tables, 2 fused
 *                 kernel, 3 partitioned (results never depend on it)
 *   "part_bits"   partitioned group-by: at least this many partition bits
 *   "part_levels" partitioned group-by: 1 / 2 scatter passes (-1: by the
 *                 partition bits, two above 8)
 * A / B switches of measured kernel variants (results never depend on them):
 *   "part_direct"  1: one-workgroup partitions flush into their own region
 *   "part_lds_kb"  partitioned aggregation's LDS table budget (0: 160 KiB)
 *   "part_threads" partitioned aggregation's threads per workgroup (0: by
 *                  the rows per workgroup)
 *   "rl_stream"    1: rolling windows <= 64 by resident streaming waves
 *   "rl_grid"      the streaming rolling kernel's workgroups per CU
 *   "rl_div"       1: full windows' means by the one-correction quotient
 *   "rl_full"      1: interior null-free rolling waves by the specialised
 *                  scans (sum / mean / var / std)
 *   "filt_pipe"    1: the filter scatter issues the next column's loads
 *                  before this column's stores
 *   "gb_pair"      1: (x * y).sum() next to y.sum() by the fused kernel's
 *                  product-pair variant
 *   "var_pos"      1: the fused variance's x limbs unsigned when the fused
 *                  predicate keeps only x >= 0
 *   "sum_pos"      1: the fused 4-sum kernel's limbs of the predicate's own
 *                  column unsigned when the predicate keeps only x >= 0
 *   "filt_fused"   1: a simple-predicate filter of null-free 8-byte columns
 *                  in one pass (decoupled look-back; off: measured slower)
 *   "part_compact" 1: sum-only one-workgroup partitions write their groups
 *                  densely into a region table, misses go to a small hashed
 *                  overflow table, the finalize reads only the dense runs
 *   "part_null_sentinel" 1: sum-only partitioned runs write a null Int64 key
 *                  as a value outside the non-null keys' range (no null-bits
 *                  column in the partition buffers)
 *   "rl_var128"    1: rolling var / std interior waves form their numerators
 *                  modulo 2^128 where the wave's exponent span bounds them
 *   "rl_var_hot"   1: rolling var / std run their common blocks (interior,
 *                  finite, 128-bit numerators) in a kernel of their own and
 *                  the other blocks from a device-side list afterwards
 *   "rl_mean_hot"  1: the same split for rolling sum / mean (interior,
 *                  finite blocks in the 64-bit form)
 *   "wave_report"  1: the slim fused kernels publish their diagnostics per
 *                  wave instead of once per workgroup
 *   "alloc_skew"   1: device blocks of 256 MiB and more start at rotating
 *                  64 KiB offsets (placement probe; off)
 *   "alloc_contig" 1: device blocks of 256 MiB and more physically
 *                  contiguous where the driver grants it (placement probe; off)
 *   "srt_w4"       1: the sort's packed downsweeps compiled for 4 waves per
 *                  SIMD (off: measured slower)
 *   "srt_up_tiles" tiles per sort upsweep workgroup (1; more measured slower)
 *   "part_rows4"   1: 512-thread partition workgroups take 4 rows per thread
 * An unknown name is PLGPU_ERR_INVALID. */
int plgpu_set_option(const char* name, int64_t value);
int plgpu_get_option(const char* name, int64_t* out);
/* Kernel timer (option "ktime" = 1): HIP-event times of the library's named
 * kernels since the last reset, one "name\tms_total\tlaunches\n" line per
 * kernel into buf (NUL-terminated); waits for pending launches.  reset != 0
 * clears the sums.  Measurement support (no reference counterpart; the
 * reference's equivalent is its profiling via `should_time`,
 * crates/polars-mem-engine/src/executors/scan/python_scan.rs:91). */
int plgpu_ktime_read(char* buf, int64_t cap, int32_t reset);
/* Return the allocator's cached free blocks on the current device to the HIP
 * runtime (waits for the device first), e.g. before another allocator in the
 * process needs the memory.  Live columns are untouched. */
int plgpu_release_cached(void);

/* Checked build only (make CHECKS=1, libpolaroid_gpu_checked.so): the bits of
 * the group-by kernels' index invariants violated since the last call (the
 * violating accesses were skipped), then cleared.  Always 0 in the product
 * build. */
int plgpu_debug_checks(uint32_t* out);

/* Release a library-produced column (no-op for borrowed ones). */
void plgpu_column_release(plgpu_column* col);

/* ---- ingestion: Arrow RecordBatches in host memory -> device columns -------
 * The reference hands a DataFrame to an engine as one Arrow RecordBatch per
 * chunk: crates/polars-python/src/dataframe/export.rs:80 PyDataFrame.to_arrow
 * (what a GPU-engine scan calls on DataFrameScan.df, visitor/nodes.rs:190).
 * plgpu_column_alloc makes an owning column for the concatenated chunks
 * (PLGPU_STR: `str_bytes` bytes of string data).  plgpu_ingest_chunk copies
 * rows [src_offset, src_offset + length) of one chunk's Arrow buffers, as they
 * lie in host memory, into rows [dst_row, dst_row + length) of `dst`:
 *   values    Arrow buffers[1] (fixed width; bit-packed for PLGPU_BOOL;
 *             int64 offsets for PLGPU_STR, rebased so the chunk's first byte
 *             lands at `dst_byte` of dst->data)
 *   validity  Arrow buffers[0] or NULL (all valid; required NULL when dst has
 *             no validity)
 *   str_data  Arrow buffers[2] of a PLGPU_STR chunk
 * Copies are the runtime's staged copies of the pageable buffers,
 * asynchronously on `stream`; bits at any offset are placed by a device
 * kernel.  The host buffers may be reused on return; the device data is
 * complete after plgpu_synchronize. */
int plgpu_column_alloc(int32_t dtype, int64_t length, int32_t with_validity, int64_t str_bytes,
                       plgpu_column* out, void* stream);
int plgpu_ingest_chunk(plgpu_column* dst, int64_t dst_row, int64_t dst_byte, const void* values,
                       const uint8_t* validity, const uint8_t* str_data, int64_t src_offset, int64_t length,
                       void* stream);

/* Result dtype of a program over columns of the given dtypes (only the
 * columns' dtype fields are read; nothing runs on the device): the static
 * typing of polars' type coercion (polars-plan/src/plans/conversion/
 * type_coercion, polars-core/src/utils/supertype.rs) as the executor applies
 * it. */
int plgpu_expr_dtype(const plgpu_column* cols, int32_t ncols, const plgpu_instr* program, int32_t n_instr,
                     int32_t* out_dtype);

/* ------------------------------------------------------------ hot path */

/* Evaluate a physical expression over `ncols` input columns of equal length
 * into a new column (BOOL / I64 / F64).  Replaces PhysicalExpr::evaluate for
 * column/literal/binary expressions (polars-expr/src/expressions/binary.rs)
 * and the broadcast comparison kernels TotalOrdKernel::tot_*_kernel_broadcast
 * (polars-compute/src/comparisons/{scalar,simd}.rs). */
int plgpu_eval(const plgpu_column* cols, int32_t ncols, const plgpu_instr* program,
               int32_t n_instr, plgpu_column* out, void* stream);

/* Filter `ncols` columns by a BOOL mask (null = false) into new columns.
 * Replaces polars-compute/src/filter/mod.rs:18 `filter` (and
 * DataFrame::filter, polars-core/src/frame/mod.rs:2012, which FilterExec
 * calls in polars-mem-engine/src/executors/filter.rs:51). */
int plgpu_filter(const plgpu_column* cols, int32_t ncols, const plgpu_column* mask,
                 plgpu_column* out_cols, int64_t* out_len, void* stream);

/* Fused FilterExec + predicate: evaluate `program` (must yield BOOL) and
 * compact the columns in one pipeline (no materialised mask column). */
int plgpu_filter_expr(const plgpu_column* cols, int32_t ncols, const plgpu_instr* program,
                      int32_t n_instr, plgpu_column* out_cols, int64_t* out_len,
                      void* stream);

/* Hash group-by on one integer key column with aggregations, optionally
 * fused with a filter predicate (`program` may be NULL / n_instr 0).
 * Replaces GroupByExec / GroupByStreamingExec
 * (polars-mem-engine/src/executors/group_by.rs:117,
 * group_by_streaming.rs) for keys = [col(k)], aggs over plain columns.
 * Output: `out_key` (I64, null group allowed) and `out_aggs[naggs]`.
 * maintain_order != 0 orders groups by first occurrence (the reference's
 * `maintain_order=True`); otherwise group order is unspecified, as in the
 * reference. */
int plgpu_group_by_agg(const plgpu_column* key, const plgpu_column* cols, int32_t ncols,
                       const plgpu_instr* program, int32_t n_instr, const plgpu_agg* aggs,
                       int32_t naggs, int32_t maintain_order, plgpu_column* out_key,
                       plgpu_column* out_aggs, plgpu_groupby_info* info, void* stream);

/* Group-by on 1..8 key columns (I64 / I32 / U32 / F64 / BOOL, nullable).
 * Replaces the multi-key branch of DataFrame::group_by_with_series
 * (polars-core/src/frame/group_by/mod.rs:91): the reference row-encodes the
 * keys (chunked_array/ops/row_encode.rs:11) and groups the encoded rows, so
 * groups are distinct key tuples, a null equal only to a null and f64 keys
 * compared by TotalOrd.  Here the tuples are hashed to 64 bits, grouped by
 * the single-key kernels, and every row is verified against its group's first
 * row (a hash collision re-runs with another seed; PLGPU_ERR_CAPACITY after 4
 * seeds).  `out_keys[nkeys]` take the key columns' dtypes and hold each
 * group's first-row tuple; `maintain_order`, aggregations and the fused
 * predicate are as for plgpu_group_by_agg. */
int plgpu_group_by_agg_multi(const plgpu_column* keys, int32_t nkeys, const plgpu_column* cols,
                             int32_t ncols, const plgpu_instr* program, int32_t n_instr,
                             const plgpu_agg* aggs, int32_t naggs, int32_t maintain_order,
                             plgpu_column* out_keys, plgpu_column* out_aggs,
                             plgpu_groupby_info* info, void* stream);

/* The general form of both: 0..8 key columns, and aggregations over the
 * columns or over computed inputs.  An agg.col >= ncols names
 * inputs[agg.col - ncols], an elementwise expression over the columns (see
 * plgpu_agg_input): `x op y` of two Float64 columns or a column and a
 * literal (+ - * /) is computed in registers by the fused kernel; any other
 * expression is evaluated once into a column first.
 * nkeys == 0 is a global reduction, `lf.filter(p).select(aggs)`
 * (polars-expr/src/reduce/sum.rs:112 reduce_ca and its siblings): every
 * selected row in one group, and one output row even when no row is
 * selected (sum / len / count 0, the other aggregations null, as the
 * reference's empty reductions); `out_keys` is not written.  `ncols` must be
 * >= 1 then, to give the length. */
int plgpu_group_by_agg_ex(const plgpu_column* keys, int32_t nkeys, const plgpu_column* cols, int32_t ncols,
                          const plgpu_agg_input* inputs, int32_t ninputs, const plgpu_instr* program,
                          int32_t n_instr, const plgpu_agg* aggs, int32_t naggs, int32_t maintain_order,
                          plgpu_column* out_keys, plgpu_column* out_aggs, plgpu_groupby_info* info,
                          void* stream);


/* ---- hash-partitioned group-by (one process per GPU) ----------------------
 * Mirrors the partitioned sink of the streaming group-by
 * (polars-stream/src/nodes/group_by.rs:216 `combine_locals`): each local
 * builder pre-aggregates, splits its pre-aggregates by a hash partitioner
 * (group_by.rs:85 `add_pre_agg`, :509 HashPartitioner) and each partition
 * folds the pre-aggregates routed to it (group_by.rs:378 `combine_subset`).
 * Here a "local" is one GPU's shard, partitions are ranks, and the
 * pre-aggregates are exact partial states (records) moved by one RCCL
 * all-to-all.  A record is `record_words` u64 words:
 * [kind (0 key, 1 null key, 2 INT64_MIN key), key, state fields...].
 * Each rank aggregates with its own f64 fixed-point windows (`bottoms`,
 * PLGPU_GB_MAX_ACC int32, refitted locally as needed); the windows travel
 * with the record counts, and plgpu_gb_merge_sources shifts every source's
 * exact sum states onto the lowest window before folding them
 * (polaroid_amd/distributed.py).  No collective precedes the exchange. */
typedef struct plgpu_gb_partial plgpu_gb_partial;

#define PLGPU_GB_MAX_ACC 6

/* Words per exported record for this aggregation schema (lengths ignored). */
int plgpu_gb_record_words(const plgpu_column* cols, int32_t ncols, const plgpu_agg* aggs,
                          int32_t naggs, int32_t* out_words);

/* Sampled fixed-point windows of this shard (out_bottoms[PLGPU_GB_MAX_ACC]). */
int plgpu_gb_plan_bottoms(const plgpu_column* key, const plgpu_column* cols, int32_t ncols,
                          const plgpu_agg* aggs, int32_t naggs, int32_t* out_bottoms,
                          void* stream);

/* Filter + pre-aggregate this shard.  `bottoms` NULL: this shard's own
 * windows (sampled, refitted here when a value does not fit); otherwise the
 * fixed windows to use, and whether one must move for an exact sum is
 * reported (*out_refit, new windows in out_bottoms_hint[6]; without a refit
 * the hint equals the used windows).  The windows used come back in
 * out_bottoms_used[6].  Returns a handle holding the partial table and the
 * number of groups (*out_records).  A column whose values need the wide
 * (multi-window) sum keeps exact per-group digit states instead: the ranks
 * agree one digit range per column (plgpu_gb_partial_wide, a max all-reduce,
 * plgpu_gb_partial_set_wide) before the export. */
int plgpu_gb_partial_begin(const plgpu_column* key, const plgpu_column* cols, int32_t ncols,
                           const plgpu_instr* program, int32_t n_instr, const plgpu_agg* aggs,
                           int32_t naggs, const int32_t* bottoms, int32_t world,
                           plgpu_gb_partial** out, int64_t* out_records, int32_t* out_bottoms_used,
                           int32_t* out_refit, int32_t* out_bottoms_hint,
                           plgpu_groupby_info* info, void* stream);

/* Wide f64 sums across ranks (round 5; polars-stream/src/nodes/group_by.rs:85
 * add_pre_agg ships fixed-size pre-aggregates whatever the values): per acc
 * a, out_wide[a] = 1 when this shard's values of that f64 sum span more
 * binades than one fixed-point window, and [out_exmin[a], out_exmax[a]] the
 * biased exponents its values take (the window's range for a non-wide f64
 * sum; 0x7FF / 0 for other accs).  The ranks reduce (max of wide, min of
 * exmin, max of exmax); when any wide[a] is set, every rank calls
 * plgpu_gb_partial_set_wide with the reduced arrays: those columns' states
 * become per-group digit words (24-bit digits in int64 words, the single-GPU
 * wide sum's form) over the agreed range, appended to every record, and
 * plgpu_gb_merge_sources_wide adds them and rounds each group once.  The
 * result is bit-identical to the single-GPU group-by.  Record words then
 * come from plgpu_gb_partial_record_words. */
int plgpu_gb_partial_wide(const plgpu_gb_partial* h, int32_t* out_wide, int32_t* out_exmin,
                          int32_t* out_exmax);
int plgpu_gb_partial_set_wide(plgpu_gb_partial* h, const int32_t* wide, const int32_t* exmin,
                              const int32_t* exmax);
int plgpu_gb_partial_record_words(const plgpu_gb_partial* h, int32_t* out_words);

/* Write the partial groups as records into device buffer `dst_records`
 * (out_records * record_words u64), grouped by destination rank in rank
 * order; out_counts[world] receives the records per destination. */
int plgpu_gb_partial_export(plgpu_gb_partial* h, void* dst_records, int64_t* out_counts,
                            void* stream);

void plgpu_gb_partial_free(plgpu_gb_partial* h);

/* Rows of a key column routed to the rank that owns their key's partial
 * states (the partition function plgpu_gb_partial_export routes records by;
 * the null key and the INT64_MIN key go to rank 0): *out_perm receives a
 * UInt32 row-index column grouped by rank in rank order, out_counts[world]
 * the rows per rank.  Used to move per-rank first() / last() results to the
 * owner of their groups (the partitioned sink's `combine_subset` for
 * reduce/first_last.rs, polars-stream/src/nodes/group_by.rs:378). */
int plgpu_gb_route(const plgpu_column* key, int32_t world, plgpu_column* out_perm,
                   int64_t* out_counts, void* stream);

/* Packed tuple keys agreed across ranks (the multi-key group-by's exact
 * Int64 packing, row_encode.rs:11 semantics: tuple equality, a null distinct
 * from every value).  plgpu_key_ranges writes per key column [min, max,
 * any null] (signed; no valid value: min = INT64_MAX > max = INT64_MIN) into
 * out_ranges[3 * nkeys]; the caller reduces them over the ranks (min / max /
 * max).  plgpu_key_pack packs every row's tuple with the plan those ranges
 * give into *out_codes (Int64, no nulls; *out_ok = 0 and no column when the
 * fields need more than 63 bits); plgpu_key_unpack turns codes back into
 * key columns of `dtypes`.  Keys: integer (not UInt64) or Boolean. */
int plgpu_key_ranges(const plgpu_column* keys, int32_t nkeys, int64_t* out_ranges, void* stream);
int plgpu_key_pack(const plgpu_column* keys, int32_t nkeys, const int64_t* ranges,
                   plgpu_column* out_codes, int32_t* out_ok, void* stream);
int plgpu_key_unpack(const plgpu_column* codes, const int32_t* dtypes, int32_t nkeys,
                     const int64_t* ranges, plgpu_column* out_keys, void* stream);

/* Float64 / Float32 keys across ranks: each key as the Int64 of its
 * canonical bits (-0.0 as 0.0, every NaN as one NaN; polars-utils/src/
 * total_ord.rs TotalEq groups exactly these together), validity carried, so
 * a float key crosses the integer-keyed partitioned group-by (the output
 * key is each group's first value, carried by a first() aggregation). */
int plgpu_float_key_encode(const plgpu_column* keys, plgpu_column* out_codes, void* stream);

/* Fold `n_records` received records (device memory) into this rank's
 * partition and finalize it like plgpu_group_by_agg (`cols` supplies the
 * dtypes only; `key_dtype` is the original key dtype). */
int plgpu_gb_merge(const void* records, int64_t n_records, const plgpu_column* cols,
                   int32_t ncols, const plgpu_agg* aggs, int32_t naggs, const int32_t* bottoms,
                   int32_t key_dtype, plgpu_column* out_key, plgpu_column* out_aggs,
                   plgpu_groupby_info* info, void* stream);

/* Fold the records received from `n_sources` ranks: source j's
 * src_records[j] records lie consecutively, in source order (the layout of
 * an all-to-all's receive buffer), aggregated with that source's windows
 * src_bottoms[j * PLGPU_GB_MAX_ACC + a].  Per column, the sums are shifted
 * onto the lowest window of any source that sent records (exact); a state
 * that would leave the 192-bit range fails with PLGPU_ERR_CAPACITY.  Then
 * finalized like plgpu_gb_merge.  Replaces the window agreement before the
 * partial stage (polars-stream/src/nodes/group_by.rs:378 combine_subset
 * folds pre-aggregates of any origin). */
int plgpu_gb_merge_sources(const void* records, int32_t n_sources, const int64_t* src_records,
                           const int32_t* src_bottoms, const plgpu_column* cols, int32_t ncols,
                           const plgpu_agg* aggs, int32_t naggs, int32_t key_dtype,
                           plgpu_column* out_key, plgpu_column* out_aggs, plgpu_groupby_info* info,
                           void* stream);

/* plgpu_gb_merge_sources for records carrying wide digit states (the
 * reduced wide / exmin / exmax of plgpu_gb_partial_set_wide). */
int plgpu_gb_merge_sources_wide(const void* records, int32_t n_sources, const int64_t* src_records,
                                const int32_t* src_bottoms, const int32_t* wide,
                                const int32_t* wide_exmin, const int32_t* wide_exmax,
                                const plgpu_column* cols, int32_t ncols, const plgpu_agg* aggs,
                                int32_t naggs, int32_t key_dtype, plgpu_column* out_key,
                                plgpu_column* out_aggs, plgpu_groupby_info* info, void* stream);

/* ---- hash join ------------------------------------------------------------
 * maintain_order (polars-ops/src/frame/join/args.rs:100 MaintainOrderJoin)
 * and validate (args.rs JoinValidation). */
enum plgpu_join_order {
    PLGPU_JOIN_ORDER_NONE = 0,        /* unspecified (build on the shorter side) */
    PLGPU_JOIN_ORDER_LEFT = 1,        /* left row order (then right row order)   */
    PLGPU_JOIN_ORDER_RIGHT = 2,       /* right row order (then left row order)   */
    PLGPU_JOIN_ORDER_LEFT_RIGHT = 3,
    PLGPU_JOIN_ORDER_RIGHT_LEFT = 4
};
enum plgpu_join_validate {
    PLGPU_JOIN_VALIDATE_M_M = 0,
    PLGPU_JOIN_VALIDATE_1_M = 1,      /* left keys unique  */
    PLGPU_JOIN_VALIDATE_M_1 = 2,      /* right keys unique */
    PLGPU_JOIN_VALIDATE_1_1 = 3
};

/* Join type (polars-ops/src/frame/join/args.rs JoinType; cross / as-of /
 * IE joins are not on the GPU path). */
enum plgpu_join_how {
    PLGPU_JOIN_INNER = 0,
    PLGPU_JOIN_LEFT = 1,
    PLGPU_JOIN_RIGHT = 2,
    PLGPU_JOIN_FULL = 3,
    PLGPU_JOIN_SEMI = 4,
    PLGPU_JOIN_ANTI = 5
};

/* Equi-join of any type on one integer key (I64 / I32 / U32).  Produces the
 * row pairs as two UInt32 index columns; a row without a partner has a null
 * partner index (left / right / full joins: the reference's
 * NullableIdxSize / ChunkJoinOptIds), and such an index column carries an
 * Arrow validity bitmap.  Semi / anti joins produce the kept left rows in
 * `out_left_idx` (in left-row order) and an empty `out_right_idx`.  Pair
 * order is the reference's for every maintain_order mode (left joins are
 * always in left order; full joins with maintain_order "none" leave the
 * order unspecified, as the reference's hash-table drain does).  Replaces
 *   inner  single_keys_inner.rs:45 hash_join_tuples_inner,
 *   left   single_keys_left.rs:106 hash_join_tuples_left (+ the ordering of
 *          dispatch_left_right.rs:143 maintain_order_idx),
 *   right  dispatch_left_right.rs:19 right_join_from_series,
 *   full   single_keys_outer.rs:181 hash_join_tuples_outer (+ the ordering of
 *          hash_join/mod.rs:164 _full_join_from_series),
 *   semi / anti  single_keys_semi_anti.rs:111 / :95
 * (paths under polars-ops/src/frame/join/). */
int plgpu_join(const plgpu_column* left_key, const plgpu_column* right_key, int32_t how, int32_t nulls_equal,
               int32_t maintain_order, int32_t validate, plgpu_column* out_left_idx, plgpu_column* out_right_idx,
               void* stream);

/* plgpu_join on 1..8 key columns per side (pairwise equal dtypes: I64 / I32
 * / U32 / F64 / BOOL; join/mod.rs:625 prepare_keys_multiple). */
int plgpu_join_multi(const plgpu_column* left_keys, const plgpu_column* right_keys, int32_t nkeys, int32_t how,
                     int32_t nulls_equal, int32_t maintain_order, int32_t validate, plgpu_column* out_left_idx,
                     plgpu_column* out_right_idx, void* stream);

/* Boolean column of a comparison of String column `a` with String column
 * `b`, or (b == NULL) with the literal `lit` (lit_len bytes, host memory):
 * op = PLGPU_OP_EQ .. PLGPU_OP_NE_MISSING; or IS_NULL / IS_NOT_NULL of `a`;
 * or PLGPU_OP_STR_{STARTS_WITH,ENDS_WITH,CONTAINS} against the literal.
 * Bytes compare lexicographically (a proper prefix first); a null operand
 * gives null except for the *_MISSING ops.  Replaces
 * polars-compute/src/comparisons/view.rs TotalEqKernel / TotalOrdKernel for
 * BinaryViewArray (and their _broadcast scalar forms). */
int plgpu_str_compare(const plgpu_column* a, const plgpu_column* b, const uint8_t* lit, int64_t lit_len, int32_t op,
                      plgpu_column* out, void* stream);

/* Group variance / standard deviation from per-group sums of squared
 * deviations (Float64) and non-null counts (UInt32 / Int64): null when
 * count <= ddof, else sum_sq / (count - ddof) (negative clamped to 0), the
 * square root when take_sqrt.  Replaces polars-compute/src/moment.rs:126
 * VarState::finalize as used by polars-expr/src/reduce/var_std.rs.  The
 * executor computes the sums with two exact group-by passes around the
 * per-row group mean (polaroid_amd/frame.py:_group_by_var). */
int plgpu_var_finalize(const plgpu_column* sum_sq, const plgpu_column* count, int32_t ddof, int32_t take_sqrt,
                       plgpu_column* out, void* stream);

/* Per-row squared deviation from the row's group mean, the second pass of
 * var / std for one integer / Boolean key: out[i] = (x[i] - mean[g])^2 with
 * g the row of group_key equal to row_key[i] (group keys unique; a null
 * row key matches the null group).  Null where x is null, the key is not a
 * group or the mean is null.  Same values as the composed join path
 * (x.cast(f64) - mean)^2, without materialising the joined frame. */
int plgpu_group_sq_dev(const plgpu_column* row_key, const plgpu_column* x, const plgpu_column* group_key,
                       const plgpu_column* group_mean, plgpu_column* out, void* stream);

/* Short-string codes: each string of at most 7 bytes as the Int64
 * (length << 56) | bytes (little-endian), exact and injective, so String
 * keys can cross the integer-keyed paths (the multi-GPU group-by's partial
 * states and exchange); *all_short = 0 if some string is longer (its code
 * is then 0).  Validity is carried.  plgpu_str_decode_short is the inverse. */
int plgpu_str_encode_short(const plgpu_column* strs, plgpu_column* out_codes, int32_t* all_short, void* stream);
int plgpu_str_decode_short(const plgpu_column* codes, plgpu_column* out, void* stream);

/* out[i] = a[i] if valid, else b[i] (same dtype and length); the coalesced
 * key columns of a full join with coalesce=True
 * (polars-ops/src/frame/join/general.rs:52 _coalesce_full_join). */
int plgpu_coalesce(const plgpu_column* a, const plgpu_column* b, plgpu_column* out, void* stream);

/* Inner equi-join on one integer key (I64 / I32 / U32; the two sides may
 * differ, values compare as integers).  Produces the matching row pairs as
 * two UInt32 index columns (the reference's IdxSize pairs).  Null keys match
 * only when nulls_equal != 0.  Replaces
 * polars-ops/src/frame/join/hash_join/single_keys_inner.rs:45
 * hash_join_tuples_inner (via _inner_join / JoinDispatch). */
int plgpu_join_inner(const plgpu_column* left_key, const plgpu_column* right_key,
                     int32_t nulls_equal, int32_t maintain_order, int32_t validate,
                     plgpu_column* out_left_idx, plgpu_column* out_right_idx, void* stream);

/* Inner join on one integer key plus the take of both frames' columns: the
 * left frame's `left_cols` and the right frame's `right_cols` (0..8 each,
 * every one as long as its side's key) at the matching pairs, in the pair
 * order of plgpu_join_inner; *out_len rows.  The fused form of
 * polars-ops/src/frame/join/hash_join/single_keys_inner.rs:45
 * hash_join_tuples_inner followed by _finish_join's takes
 * (polars-ops/src/frame/join/general.rs:17).  With one right column, unique
 * right keys and a null-free 8-byte right column the hash table is
 * row-format (each cell {key, payload}) and the emit pass writes the
 * payload and the null-free 8-byte left columns straight to their output
 * rows; other inputs take the pairs + gather route with the same result.
 * With maintain_order "none" (the reference's default), null-free 8-byte
 * integer keys and columns, a long probe side and a build side beyond the
 * L2s, the join is radix-partitioned (round 6): per-partition L2-resident
 * sub-tables (polars-ops/src/frame/join/hash_join/single_keys.rs:16
 * build_tables), the probe rows scattered by partition, rows out in
 * partition order. */
int plgpu_join_inner_take(const plgpu_column* left_key, const plgpu_column* right_key,
                          const plgpu_column* left_cols, int32_t nleft,
                          const plgpu_column* right_cols, int32_t nright, int32_t nulls_equal,
                          int32_t maintain_order, int32_t validate, plgpu_column* out_left,
                          plgpu_column* out_right, int64_t* out_len, void* stream);

/* plgpu_join_inner_take on 1..8 key columns per side (as plgpu_join_inner_multi):
 * integer / Boolean keys whose ranges pack into one exact Int64 take the
 * single-key route on the packed keys (row-format table included); other
 * keys compute the verified pairs and gather. */
int plgpu_join_inner_take_multi(const plgpu_column* left_keys, const plgpu_column* right_keys,
                                int32_t nkeys, const plgpu_column* left_cols, int32_t nleft,
                                const plgpu_column* right_cols, int32_t nright, int32_t nulls_equal,
                                int32_t maintain_order, int32_t validate, plgpu_column* out_left,
                                plgpu_column* out_right, int64_t* out_len, void* stream);

/* Inner join on 1..8 key columns per side (pairwise equal dtypes: I64 / I32 /
 * U32 / F64 / BOOL).  Replaces the multi-key branch of the reference's join
 * (polars-ops/src/frame/join/mod.rs:625 prepare_keys_multiple: both sides'
 * keys row-encoded, then hash-joined as binary keys; a tuple holding a null
 * joins only when nulls_equal).  Here tuples are hashed to 64 bits
 * (tuplehash.hpp), joined with the single-key kernels, and every output pair
 * is verified tuple by tuple (a collision re-runs with another seed).
 * Arguments, output and order modes as plgpu_join_inner. */
int plgpu_join_inner_multi(const plgpu_column* left_keys, const plgpu_column* right_keys,
                           int32_t nkeys, int32_t nulls_equal, int32_t maintain_order,
                           int32_t validate, plgpu_column* out_left_idx,
                           plgpu_column* out_right_idx, void* stream);

/* out_cols[i] = cols[i][idx] (UInt32 indices), validity carried; a null
 * index gathers a null.  Replaces the join materialisation take
 * (polars-core/src/chunked_array/ops/gather.rs, DataFrame::take_unchecked;
 * IdxCa::with_nullable_idx for the outer joins' nullable indices). */
int plgpu_gather(const plgpu_column* cols, int32_t ncols, const plgpu_column* idx,
                 plgpu_column* out_cols, void* stream);

/* ---- row shuffles (multi-GPU join / group-by) -------------------------------
 * Stable hash partitioning of rows by 1..8 key columns into nparts (1..1024)
 * partitions: out_perm (UInt32, library-owned) lists the rows partition by
 * partition, in row order within each; out_counts[p] = rows of partition p.
 * A key tuple holding a null is dropped when nulls_equal == 0 (it cannot
 * join) and routed to partition 0 otherwise.  The partition of a row depends
 * only on its key values, so every rank routes equal keys alike (floats by
 * TotalEq class, -0.0 with 0.0 and every NaN together; String keys by a hash
 * of their bytes).  Replaces
 * polars-utils/src/hashing.rs:101 HashPartitioner::hash_to_partition as
 * used by polars-stream/src/nodes/joins/equi_join.rs:445 / :740
 * (partition_and_sink / partition_and_probe). */
int plgpu_hash_partition(const plgpu_column* keys, int32_t nkeys, int32_t nparts,
                         int32_t nulls_equal, plgpu_column* out_perm, int64_t* out_counts,
                         void* stream);

/* Pack rows into caller-owned flat buffers (e.g. RCCL send tensors):
 * dst_values[i][o] = cols[i][idx[o]] (idx NULL: o), 8 / 4 bytes per value,
 * one byte (0/1) per Boolean value; dst_valid[i] (when dst_valid and
 * dst_valid[i] are non-NULL) gets one validity byte per row.  The
 * send-side half of the reference's per-partition DataFrame::take. */
int plgpu_gather_rows(const plgpu_column* cols, int32_t ncols, const plgpu_column* idx,
                      void* const* dst_values, uint8_t* const* dst_valid, void* stream);

/* Bytes (0 / non-zero) -> Arrow LSB-first bitmap of ceil(n / 64) 8-byte
 * words; *out_zero_count (optional) = number of zero bytes (the null count
 * of a validity mask).  The receive-side inverse of plgpu_gather_rows. */
int plgpu_pack_bits(const uint8_t* bytes, int64_t n, uint8_t* out_bits, int64_t* out_zero_count,
                    void* stream);

/* ---- sort ------------------------------------------------------------------
 * Stable arg-sort of one column (I64 / I32 / U32 / F64) into a UInt32
 * permutation: TotalOrd order (NaN greatest, -0.0 == 0.0), descending
 * reverses the order of distinct values while equal values keep their row
 * order, nulls first unless nulls_last.  Replaces
 * polars-core/src/chunked_array/ops/sort/arg_sort.rs arg_sort with
 * SortOptions { maintain_order: true } (options.rs:32); DataFrame.sort is
 * this permutation followed by plgpu_gather. */
int plgpu_arg_sort(const plgpu_column* key, int32_t descending, int32_t nulls_last,
                   plgpu_column* out_idx, void* stream);

/* Stable arg-sort by 1..8 columns (I64 / I32 / U32 / F64 / BOOL), each with
 * its own `descending[j]` and `nulls_last[j]`.  Replaces
 * polars-core/src/chunked_array/ops/sort/arg_sort_multiple.rs:24
 * arg_sort_multiple_impl (lexicographic compare, column by column, nulls
 * placed per column independently of `descending`; maintain_order = a stable
 * result, which this always is).  LSD over the columns: each column is one
 * stable radix sort of its codes through the running permutation, plus one
 * pass placing its nulls. */
int plgpu_arg_sort_multi(const plgpu_column* keys, int32_t nkeys, const int32_t* descending,
                         const int32_t* nulls_last, plgpu_column* out_idx, void* stream);

/* ---- rolling windows ---------------------------------------------------------
 * Fixed-size window sum / mean (window_size rows, min_periods non-null rows
 * for a valid output, optionally centred), like Series.rolling_sum /
 * rolling_mean.  Float64 (and integer mean) results are the correctly
 * rounded window sums (divided by the non-null count); integer sums wrap.
 * Replaces polars-compute/src/rolling/no_nulls/{sum,mean}.rs rolling_sum /
 * rolling_mean and nulls/{sum,mean}.rs (rolling/sum.rs:7 SumWindow).
 * VAR / STD (ddof in bits 8..15 of kind): Series.rolling_var / rolling_std,
 * replacing polars-compute/src/rolling/{no_nulls,nulls}/moment.rs
 * rolling_var (rolling/moment.rs:138 MomentWindow<VarianceMoment>) and
 * polars-time/src/chunkedarray/rolling_window/dispatch.rs:526 (std = its
 * square root): Float64 output, (RN(c sum x^2 - (sum x)^2) / c) / (c - ddof)
 * with the numerator exact; a non-finite value gives NaN; null below
 * min_periods non-null values or at c <= ddof. */
enum plgpu_rolling_kind {
    PLGPU_ROLLING_SUM = 1,
    PLGPU_ROLLING_MEAN = 2,
    PLGPU_ROLLING_MIN = 3,  /* rolling/no_nulls/min_max.rs MinWindow (NaN propagates) */
    PLGPU_ROLLING_MAX = 4,  /* ... MaxWindow; output dtype = input dtype            */
    PLGPU_ROLLING_VAR = 5,
    PLGPU_ROLLING_STD = 6
};

int plgpu_rolling(const plgpu_column* values, int32_t kind, int64_t window_size,
                  int64_t min_periods, int32_t center, plgpu_column* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* POLAROID_GPU_H */
