// plgpu_internal.hpp — shared internals of the gfx950 executor backend.
//
// Device side: Arrow column access, polars TotalOrd comparisons, the typed
// row interpreter for lowered expression programs, orderable encodings and
// the exact fixed-point representation used by f64 sums.
// Host side: error plumbing, the stream-ordered allocator, program lowering.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstring>

#include <string>
#include <vector>

#include "../../include/polaroid_gpu.h"

#define PLGPU_API extern "C" __attribute__((visibility("default")))

namespace plgpu {

// ------------------------------------------------------------------ host
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

#define PLGPU_HIP(expr)                                   \
    do {                                                  \
        hipError_t _e = (expr);                           \
        if (_e != hipSuccess) return plgpu::hip_fail(_e, #expr); \
    } while (0)

hipStream_t as_stream(void* s);

// Test hooks / diagnostics (runtime.cpp): read once from PLGPU_<NAME> at
// load, settable with plgpu_set_option.
struct Options {
    int debug = 0;       // per-attempt group-by diagnostics on stderr
    int no_pack = 0;     // multi-key operators hash tuples even when they would pack (tests)
    int mk_collide = 0;  // 3-bit first tuple hash: forces the collision / re-seed path (tests)
    int runs = -1;       // -1: the plan picks the sorted-key variant; 0 / 1 force it (tests)
    int local = -1;      // -1: the plan picks the range-local kernel; 0 keeps it off (tests)
    int ktime = 0;       // 1: time the named kernels with HIP events (plgpu_ktime_read)
    int fuse_keys = 1;   // 0: packed multi-key codes go through a code column (tests / A-B)
    int plan_cache = 1;  // 0: every group-by samples its inputs (no reuse of recent plan statistics)
    int grid_rounds = 0; // fused group-by grid in rounds of resident workgroups (0: kGridRounds; A-B)
    // group-by path hooks (tests: the forced-path parity sweep, DESIGN.md
    // "Group-by paths"): -1 lets the plan choose
    int gb_path = -1;     // 0 generic kernel on the global table, 1 generic with LDS tables,
                          // 2 fused kernel, 3 partitioned (where the inputs allow it),
                          // 5 partitioned without the plan's input checks (the launchers refuse)
    int part_bits = -1;   // partitioned path: at least this many partition bits
    int part_levels = -1; // partitioned path: 1 / 2 scatter passes (-1: by the partition bits)
    int part_direct = 1;  // partitioned path: one-workgroup partitions flush into their own table region
    int part_lds_kb = 0;  // partitioned path: LDS table budget per workgroup (0: 160 KiB)
    int part_compact = 1; // partitioned path, slim sum-only layout: compact regions + region finalize (A/B)
    int rl_stream = 0;    // rolling windows <= 64, null-free: resident streaming waves (0: one block per wave; A/B)
    int rl_grid = 0;      // rolling stream kernel: workgroups per CU (0: 4)
    int filt_pipe = 1;    // filter scatter: next column's loads before this column's stores (A/B)
    int part_threads = 0; // partitioned aggregation: threads per workgroup (0: 1024; A/B)
    int rl_div = 1;       // rolling mean of full windows by one correction step instead of a division (A/B)
    int rl_full = 1;      // rolling sum / mean: interior int64-form waves by the specialised scan (A/B)
    int rl_mean_hot = 1;  // rolling sum / mean: common blocks by a kernel of their own, the rest listed (A/B)
    int rl_var_hot = 1;   // rolling var / std: common blocks by a kernel of their own, the rest listed (A/B)
    int rl_var128 = 1;    // rolling var / std, interior waves: 128-bit modular numerators where they fit (A/B)
    int alloc_skew = 0;   // device pool: blocks >= 256 MiB at rotating 64 KiB offsets (A/B)
    int alloc_contig = 0; // device pool: blocks >= 256 MiB physically contiguous where the driver can (A/B)
    int srt_w4 = 0;       // sort: packed downsweeps compiled for 4 waves per SIMD (A/B)
    int srt_up_tiles = 1; // sort: tiles per upsweep workgroup, the next tile's codes prefetched (A/B)
    int part_rows4 = 0;   // partitioned aggregation, 512-thread workgroups: 4 rows per thread (A/B)
    int wave_report = 0;  // fused kernels: publish diagnostics per wave instead of per workgroup (A/B)
    int part_null_sentinel = 1; // partitioned sum-only runs: null Int64 keys as an unused key value (A/B)
    int filt_fused = 0;   // filter: the one-pass look-back kernel where it applies (A/B; measured slower)
    int var_pos = 1;      // fused variance: x's limbs unsigned when the predicate keeps x >= 0 (A/B)
    int sum_pos = 1;      // fused 4-sum kernel: the predicate column's limbs unsigned when it keeps x >= 0 (A/B)
    int gb_pair = 1;      // (x * y).sum() next to y.sum(): the product-pair fused variant (A/B)
    // order-free inner join + take by radix partitions with L2-resident
    // sub-tables (join.hip "partitioned join"): 1 where it pays (large probe
    // and build sides), 2 forced wherever it applies (tests), 0 off (A/B)
    int join_radix = 1;
    int join_radix_keys = 0;  // build keys per partition target (0: 2^15)
    int join_radix_load = 0;  // sub-table load factor in percent (0: 35)
    int join_radix_batch = 0; // match pass: probe steps with bucket reads in flight together, 4 or 8 (0: 4)
};
Options& options();

// Kernel timer (option "ktime", runtime.cpp): HIP events recorded on the
// launching stream immediately before and after one named kernel launch,
// summed per name and read back by plgpu_ktime_read.  The bench reports
// these live per-kernel times next to its step times, and they are the same
// quantity a rocprofv3 kernel trace reports.  Off (the default), a scope
// costs one load and a branch.
// Recycled HIP events (hipEventCreate / Destroy per query cost more than
// the query's host work at 1e8 rows); ev_acquire returns nullptr on failure.
// Forget the group-by plan statistics kept for repeated queries (groupby.hip).
void gb_plan_cache_clear();
hipEvent_t ev_acquire();
void ev_release(hipEvent_t e);
// A scope owns its event pair until it ends; only then does the pair join
// the pending list that plgpu_ktime_read drains, so a read from another
// thread never sees (or recycles) a scope that is still open.
bool kt_begin(hipStream_t s, hipEvent_t* a, hipEvent_t* b);
void kt_end(const char* name, hipEvent_t a, hipEvent_t b, hipStream_t s);
struct KtScope {
    const char* name;
    hipEvent_t a = nullptr, b = nullptr;
    hipStream_t s;
    KtScope(const char* nm, hipStream_t st) : name(nm), s(st) {
        if (options().ktime && !kt_begin(st, &a, &b)) a = b = nullptr;
    }
    ~KtScope() {
        if (a) kt_end(name, a, b, s);
    }
    KtScope(const KtScope&) = delete;
    KtScope& operator=(const KtScope&) = delete;
};
int dev_alloc(void** p, size_t bytes, hipStream_t s);
void dev_free(void* p, hipStream_t s);

// A library-owned device column buffer set (released via plgpu_column.release).
struct OwnedBuffers {
    void* values = nullptr;
    void* validity = nullptr;
    void* data = nullptr;
    hipStream_t stream = nullptr;
};
// Fill `out` as an owning column over freshly allocated buffers.
int make_owned_column(plgpu_column* out, int32_t dtype, int64_t length, bool with_validity,
                      hipStream_t s);

__host__ __device__ inline int dtype_bytes(int32_t dt) {
    switch (dt) {
    case PLGPU_I8:
    case PLGPU_U8: return 1;
    case PLGPU_I16:
    case PLGPU_U16: return 2;
    case PLGPU_I32:
    case PLGPU_U32:
    case PLGPU_F32: return 4;
    case PLGPU_I64:
    case PLGPU_U64:
    case PLGPU_F64: return 8;
    default: return 0;  // BOOL is bit-packed, STR has offsets + bytes
    }
}

// Numeric classes of the physical dtypes.
__host__ __device__ inline bool dtype_is_int(int32_t dt) {
    return dt == PLGPU_I8 || dt == PLGPU_I16 || dt == PLGPU_I32 || dt == PLGPU_I64 || dt == PLGPU_U8 ||
           dt == PLGPU_U16 || dt == PLGPU_U32 || dt == PLGPU_U64;
}
__host__ __device__ inline bool dtype_is_float(int32_t dt) { return dt == PLGPU_F32 || dt == PLGPU_F64; }

// --------------------------------------------------------- device columns
struct DevCol {
    const void* values;       // PLGPU_STR: int64 offsets
    const uint8_t* validity;
    int64_t offset;
    int32_t dtype;
    int32_t _pad;
    const uint8_t* data;      // PLGPU_STR: string bytes
};

// Radix partition of null-free 8-byte columns by the top `bits` bits of
// part_hash(key) (groupby.hip gb_partition: count, scan and LDS-staged
// scatter passes; one pass up to 2^8 partitions, two above): partition q
// holds rows [hrange[q], hrange[q + 1]) of `key` and of each col[i].  `buf`
// and `range` (the P + 1 bounds on the device, at `bounds`) are owned by the
// caller (dev_free).  Used by the join's partitioned probe.
struct RadixParts {
    uint64_t* buf = nullptr;
    uint64_t* key = nullptr;
    uint64_t* col[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    uint64_t* range = nullptr;
    const uint64_t* bounds = nullptr;
    std::vector<uint64_t> hrange;
    int levels = 0;
};
int radix_partition8(const DevCol& key, const DevCol* cols, int ncols, int64_t n, int bits, hipStream_t s,
                     RadixParts* out);

inline DevCol dev_col(const plgpu_column& c) {
    DevCol d;
    std::memset(&d, 0, sizeof d);
    d.values = c.values;
    d.validity = c.validity;
    d.offset = c.offset;
    d.dtype = c.dtype;
    d.data = c.data;
    return d;
}

// Owning PLGPU_STR column: n + 1 offsets, `bytes` of string data.
int make_owned_string_column(plgpu_column* out, int64_t length, int64_t bytes, bool with_validity, hipStream_t s);
// An owned I64 column of length + 1 offsets -> a PLGPU_STR column of
// `length` strings with a `bytes` data buffer.
int owned_attach_data(plgpu_column* out, int64_t bytes, hipStream_t s);
// out = src[idx] of a PLGPU_STR column (strings.hip); idx32 / idx64 row ids,
// iv / ioff optional index validity (a null index gathers a null).
int str_gather(const DevCol& src, const uint32_t* idx32, const int64_t* idx64, const uint8_t* iv, int64_t ioff,
               int64_t n, bool nullable, plgpu_column* out, hipStream_t s);
// Short-string key codes (strings.hip): a borrowed-style I64 column over
// codes[(length << 56) | bytes] sharing the strings' validity / offset, or
// *all_short = false when some string is longer than 7 bytes.  Free with
// str_codes_free.  str_from_codes turns a code column back into strings.
int str_short_codes(const plgpu_column& src, plgpu_column* out, bool* all_short, hipStream_t s);
void str_codes_free(plgpu_column* c, hipStream_t s);
int str_from_codes(const plgpu_column& codes, plgpu_column* out, hipStream_t s);

// Lowered (typed) program: the host resolves every operand type, inserts
// casts, and emits one micro-op per step so the device interpreter does no
// type dispatch of its own.
// Operand widths: an `arg` of F32 on a float op computes in single
// precision; D_WRAP / D_CAST take physical dtype codes.
enum DevOp : int32_t {
    D_COL_F64 = 1, D_COL_I64, D_COL_I32, D_COL_U32, D_COL_BOOL,
    D_LIT, D_NULL,
    D_ADD_I, D_SUB_I, D_MUL_I, D_NEG_I, D_ABS_I,
    D_ADD_F, D_SUB_F, D_MUL_F, D_DIV_F, D_NEG_F, D_ABS_F,
    D_I2F_0, D_I2F_1,  // cast top / second-from-top i64 -> f64
    D_EQ_F, D_NE_F, D_LT_F, D_LE_F, D_GT_F, D_GE_F,
    D_EQ_I, D_NE_I, D_LT_I, D_LE_I, D_GT_I, D_GE_I,
    D_EQM_F, D_NEM_F, D_EQM_I, D_NEM_I, D_EQM_B, D_NEM_B,
    D_EQ_B, D_NE_B,
    D_AND, D_OR, D_NOT, D_ISNULL, D_ISNOTNULL, D_ISNAN_F, D_ISFINITE_F, D_FALSE_VALID,
    // round 2: widths, division, casts, bitwise, selection
    D_COL,            // any dtype (dev_load register form)
    D_WRAP,           // s0 = s0 wrapped to integer dtype arg
    D_CAST,           // s0 = cast(s0) from dtype imm>>8 & 0xff to arg; imm & 1 = overflowing
    D_EQ_U, D_NE_U, D_LT_U, D_LE_U, D_GT_U, D_GE_U,   // UInt64 compares
    D_FLOORDIV_I, D_MOD_I,      // arg: 1 = UInt64 (unsigned); x / 0 -> null
    D_FLOORDIV_F, D_MOD_F,      // floor(a / b), a - b * floor(a / b)
    D_DIV_FS, D_FLOORDIV_FS, D_MOD_FS,  // scalar divisor: a * (1 / b) forms (float.rs:78-98, :113)
    D_BAND, D_BOR, D_BXOR,      // bitwise on integers
    D_XOR,                      // Boolean xor, null if either is null
    D_FILL_NULL,                // [x, fill]
    D_IF_ELSE                   // [cond, then, otherwise]
};

struct DevInstr {
    int32_t op;
    int32_t arg;
    uint64_t imm;
};

struct DevProgram {
    DevInstr code[PLGPU_MAX_PROGRAM];
    int32_t n;
    int32_t out_dtype;  // PLGPU_BOOL / PLGPU_I64 / PLGPU_F64
    // Fast path: program is exactly `col(c) <cmp> literal` (c numeric).
    int32_t simple;     // 0 = no, 1 = yes
    int32_t simple_col;
    int32_t simple_op;  // D_*_F or D_*_I compare op
    int32_t simple_isf; // compare in f64
    uint64_t simple_imm;
};

// Type-check and lower a user program over `cols`.  Returns PLGPU_OK or an
// error code (message set).
int lower_program(const plgpu_column* cols, int32_t ncols, const plgpu_instr* prog, int32_t n,
                  DevProgram* out);

// ------------------------------------------------------------ device code
constexpr uint64_t kEmptyKey = 0x8000000000000000ull;  // INT64_MIN sentinel

__device__ __forceinline__ double as_f64(uint64_t b) { return __longlong_as_double((long long)b); }
__device__ __forceinline__ uint64_t f64_bits(double d) { return (uint64_t)__double_as_longlong(d); }

__device__ __forceinline__ bool dev_valid(const DevCol& c, int64_t r) {
    if (c.validity == nullptr) return true;
    int64_t p = c.offset + r;
    return (c.validity[p >> 3] >> (p & 7)) & 1;
}

// Register form of column c at row r: signed ints sign-extended, unsigned
// ints zero-extended (UInt64 as its bits), Float64 as its bits, Float32 as
// the bits of the (exactly equal) double, Boolean as 0 / 1.
__device__ __forceinline__ uint64_t dev_load(const DevCol& c, int64_t r) {
    int64_t p = c.offset + r;
    switch (c.dtype) {
    case PLGPU_F64:
    case PLGPU_I64:
    case PLGPU_U64: return ((const uint64_t*)c.values)[p];
    case PLGPU_I32: return (uint64_t)(int64_t)((const int32_t*)c.values)[p];
    case PLGPU_U32: return (uint64_t)((const uint32_t*)c.values)[p];
    case PLGPU_F32: return (uint64_t)__double_as_longlong((double)((const float*)c.values)[p]);
    case PLGPU_I16: return (uint64_t)(int64_t)((const int16_t*)c.values)[p];
    case PLGPU_U16: return (uint64_t)((const uint16_t*)c.values)[p];
    case PLGPU_I8: return (uint64_t)(int64_t)((const int8_t*)c.values)[p];
    case PLGPU_U8: return (uint64_t)((const uint8_t*)c.values)[p];
    default: return (((const uint8_t*)c.values)[p >> 3] >> (p & 7)) & 1;
    }
}

// Store the register form v as one element of dtype dt at out[i].
__device__ __forceinline__ void dev_store(void* out, int32_t dt, int64_t i, uint64_t v) {
    switch (dt) {
    case PLGPU_I8:
    case PLGPU_U8: ((uint8_t*)out)[i] = (uint8_t)v; break;
    case PLGPU_I16:
    case PLGPU_U16: ((uint16_t*)out)[i] = (uint16_t)v; break;
    case PLGPU_I32:
    case PLGPU_U32: ((uint32_t*)out)[i] = (uint32_t)v; break;
    case PLGPU_F32: ((float*)out)[i] = (float)__longlong_as_double((long long)v); break;
    default: ((uint64_t*)out)[i] = v; break;
    }
}

// polars-utils/src/total_ord.rs:317-368 for f64: NaN == NaN, NaN greatest.
__device__ __forceinline__ bool tot_ge_f(double a, double b) { return __builtin_isnan(a) | (a >= b); }
__device__ __forceinline__ bool tot_eq_f(double a, double b) {
    return __builtin_isnan(a) ? __builtin_isnan(b) : (a == b);
}
// op encoded as 0..5 = eq, ne, lt, le, gt, ge
__device__ __forceinline__ bool cmp_f(int op, double a, double b) {
    switch (op) {
    case 0: return tot_eq_f(a, b);
    case 1: return !tot_eq_f(a, b);
    case 2: return !tot_ge_f(a, b);
    case 3: return tot_ge_f(b, a);
    case 4: return !tot_ge_f(b, a);
    default: return tot_ge_f(a, b);
    }
}
__device__ __forceinline__ bool cmp_i(int op, int64_t a, int64_t b) {
    switch (op) {
    case 0: return a == b;
    case 1: return a != b;
    case 2: return a < b;
    case 3: return a <= b;
    case 4: return a > b;
    default: return a >= b;
    }
}

// Integer register value wrapped to integer dtype dt (two's complement).
__device__ __forceinline__ uint64_t wrap_to(uint64_t v, int dt) {
    switch (dt) {
    case PLGPU_I8: return (uint64_t)(int64_t)(int8_t)v;
    case PLGPU_I16: return (uint64_t)(int64_t)(int16_t)v;
    case PLGPU_I32: return (uint64_t)(int64_t)(int32_t)v;
    case PLGPU_U8: return v & 0xFFull;
    case PLGPU_U16: return v & 0xFFFFull;
    case PLGPU_U32: return v & 0xFFFFFFFFull;
    default: return v;
    }
}

// Does the integer register value v (of dtype from) hold a value of dtype to?
__device__ __forceinline__ bool int_fits(uint64_t v, int from, int to) {
    const bool neg = from != PLGPU_U64 && (int64_t)v < 0;
    const bool big = from == PLGPU_U64 && (int64_t)v < 0;  // >= 2^63
    const int64_t x = (int64_t)v;
    switch (to) {
    case PLGPU_I8: return !big && x >= -128 && x <= 127;
    case PLGPU_I16: return !big && x >= -32768 && x <= 32767;
    case PLGPU_I32: return !big && x >= INT32_MIN && x <= INT32_MAX;
    case PLGPU_I64: return !big;
    case PLGPU_U8: return !neg && !big && x <= 255;
    case PLGPU_U16: return !neg && !big && x <= 65535;
    case PLGPU_U32: return !neg && !big && x <= 4294967295ll;
    case PLGPU_U64: return !neg;
    default: return true;
    }
}

// cast(v: from) -> to (polars non-strict cast: a value that does not fit
// gives null; `overflowing`: integers wrap).  Floats are in register form.
__device__ __forceinline__ uint64_t cast_value(uint64_t v, int from, int to, bool overflowing, bool& ok) {
    const bool fi = from == PLGPU_F32 || from == PLGPU_F64, ti = to == PLGPU_F32 || to == PLGPU_F64;
    if (to == PLGPU_BOOL) return fi ? (as_f64(v) != 0.0 ? 1ull : 0ull) : (v != 0 ? 1ull : 0ull);
    if (from == PLGPU_BOOL) return ti ? f64_bits(v ? 1.0 : 0.0) : v;
    if (!fi && !ti) {
        if (int_fits(v, from, to)) return v;
        if (overflowing) return wrap_to(v, to);
        ok = false;
        return 0;
    }
    if (!fi && ti) {
        if (to == PLGPU_F32) {
            const float f = from == PLGPU_U64 ? (float)v : (float)(int64_t)v;
            return f64_bits((double)f);
        }
        return f64_bits(from == PLGPU_U64 ? (double)v : (double)(int64_t)v);
    }
    const double d = as_f64(v);
    if (ti) return to == PLGPU_F32 ? f64_bits((double)(float)d) : v;
    // float -> int: truncate; NaN / out of range -> null
    const double t = trunc(d);
    bool in;
    switch (to) {
    case PLGPU_I8: in = t >= -128.0 && t <= 127.0; break;
    case PLGPU_I16: in = t >= -32768.0 && t <= 32767.0; break;
    case PLGPU_I32: in = t >= -2147483648.0 && t <= 2147483647.0; break;
    case PLGPU_I64: in = t >= -9223372036854775808.0 && t < 9223372036854775808.0; break;
    case PLGPU_U8: in = t >= 0.0 && t <= 255.0; break;
    case PLGPU_U16: in = t >= 0.0 && t <= 65535.0; break;
    case PLGPU_U32: in = t >= 0.0 && t <= 4294967295.0; break;
    default: in = t >= 0.0 && t < 18446744073709551616.0; break;
    }
    if (!in) {  // also NaN
        ok = false;
        return 0;
    }
    return to == PLGPU_U64 ? (uint64_t)t : (uint64_t)(int64_t)t;
}

// Evaluate a lowered program for one row.  The stack lives in eight named
// registers shifted by static moves (no runtime-indexed arrays -> no
// scratch); the validity of stack entry j is bit j of `vm`.
struct RowVal {
    uint64_t v;
    bool valid;
};

__device__ __forceinline__ RowVal eval_row(const DevInstr* __restrict__ code, int n, const DevCol* cols,
                                           int64_t r) {
    uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0, s6 = 0, s7 = 0;
    uint32_t vm = 0;
#define PUSH(x, ok)                                                        \
    do {                                                                   \
        s7 = s6; s6 = s5; s5 = s4; s4 = s3; s3 = s2; s2 = s1; s1 = s0;     \
        s0 = (x);                                                          \
        vm = (vm << 1) | ((ok) ? 1u : 0u);                                 \
    } while (0)
#define POP1()                                                             \
    do {                                                                   \
        s0 = s1; s1 = s2; s2 = s3; s3 = s4; s4 = s5; s5 = s6; s6 = s7;     \
        vm >>= 1;                                                          \
    } while (0)
    for (int k = 0; k < n; ++k) {
        const int op = code[k].op;
        const int arg = code[k].arg;
        const uint64_t imm = code[k].imm;
        switch (op) {
        case D_COL:
        case D_COL_F64:
        case D_COL_I64:
        case D_COL_I32:
        case D_COL_U32:
        case D_COL_BOOL: {
            const DevCol& c = cols[arg];
            bool ok = dev_valid(c, r);
            uint64_t x = dev_load(c, r);
            PUSH(x, ok);
            break;
        }
        case D_LIT: PUSH(imm, true); break;
        case D_NULL: PUSH(0ull, false); break;
        case D_NEG_I: s0 = 0ull - s0; break;
        case D_ABS_I: s0 = ((int64_t)s0 < 0) ? 0ull - s0 : s0; break;
        case D_NEG_F: s0 ^= 0x8000000000000000ull; break;
        case D_ABS_F: s0 &= 0x7fffffffffffffffull; break;
        case D_I2F_0: s0 = f64_bits((double)(int64_t)s0); break;
        case D_I2F_1: s1 = f64_bits((double)(int64_t)s1); break;
        case D_NOT: s0 = s0 ^ 1ull; break;
        case D_ISNULL: s0 = (vm & 1u) ? 0ull : 1ull; vm |= 1u; break;
        case D_ISNOTNULL: s0 = (vm & 1u) ? 1ull : 0ull; vm |= 1u; break;
        case D_ISNAN_F: s0 = __builtin_isnan(as_f64(s0)) ? 1ull : 0ull; break;
        case D_ISFINITE_F: s0 = __builtin_isfinite(as_f64(s0)) ? 1ull : 0ull; break;
        case D_FALSE_VALID: s0 = 0ull; vm |= 1u; break;
        case D_WRAP: s0 = wrap_to(s0, arg); break;
        case D_CAST: {
            // imm bits 8..15: source dtype; bit 0: overflowing; bit 16: cast
            // the second entry (s1) instead of the top
            bool ok = true;
            if (imm & 0x10000ull) {
                s1 = cast_value(s1, (int)((imm >> 8) & 0xFF), arg, (imm & 1) != 0, ok);
                if (!ok) vm &= ~2u;
            } else {
                s0 = cast_value(s0, (int)((imm >> 8) & 0xFF), arg, (imm & 1) != 0, ok);
                if (!ok) vm &= ~1u;
            }
            break;
        }
        case D_IF_ELSE: {
            // [cond = s2, then = s1, otherwise = s0]; a null condition is false
            const bool take = ((vm >> 2) & 1u) && (s2 & 1);
            const uint64_t v = take ? s1 : s0;
            const bool ok = take ? ((vm >> 1) & 1u) : (vm & 1u);
            POP1();
            POP1();
            s0 = v;
            vm = (vm & ~1u) | (ok ? 1u : 0u);
            break;
        }
        default: {
            // binary: a = s1, b = s0
            const uint64_t a = s1, b = s0;
            const bool va = (vm >> 1) & 1u, vb = vm & 1u;
            uint64_t res = 0;
            bool ok = va & vb;
            const bool f32 = arg == PLGPU_F32;
            const double fa = as_f64(a), fb = as_f64(b);
            const float ga = (float)fa, gb = (float)fb;  // exact for Float32 operands
            switch (op) {
            case D_ADD_I: res = a + b; break;
            case D_SUB_I: res = a - b; break;
            case D_MUL_I: res = a * b; break;
            case D_ADD_F: res = f64_bits(f32 ? (double)(ga + gb) : fa + fb); break;
            case D_SUB_F: res = f64_bits(f32 ? (double)(ga - gb) : fa - fb); break;
            case D_MUL_F: res = f64_bits(f32 ? (double)(ga * gb) : fa * fb); break;
            case D_DIV_F: res = f64_bits(f32 ? (double)(ga / gb) : fa / fb); break;
            case D_DIV_FS: res = f64_bits(f32 ? (double)(ga * (1.0f / gb)) : fa * (1.0 / fb)); break;
            case D_FLOORDIV_F: res = f64_bits(f32 ? (double)floorf(ga / gb) : floor(fa / fb)); break;
            case D_FLOORDIV_FS:
                res = f64_bits(f32 ? (double)floorf(ga * (1.0f / gb)) : floor(fa * (1.0 / fb)));
                break;
            case D_MOD_F: {
                if (f32) {
                    const float q = floorf(ga / gb);
                    const float bq = gb * q;
                    res = f64_bits((double)(ga - bq));
                } else {
                    const double q = floor(fa / fb);
                    const double bq = fb * q;
                    res = f64_bits(fa - bq);
                }
                break;
            }
            case D_MOD_FS: {
                if (f32) {
                    const float q = floorf(ga * (1.0f / gb));
                    const float bq = gb * q;
                    res = f64_bits((double)(ga - bq));
                } else {
                    const double q = floor(fa * (1.0 / fb));
                    const double bq = fb * q;
                    res = f64_bits(fa - bq);
                }
                break;
            }
            case D_FLOORDIV_I:
            case D_MOD_I: {
                // polars-utils/src/floor_divmod.rs: floor division, remainder
                // with the divisor's sign; x / 0 -> null (arithmetic/signed.rs:35)
                if (b == 0) {
                    ok = false;
                    break;
                }
                uint64_t q, rm;
                if (arg == 1) {
                    q = a / b;
                    rm = a % b;
                } else {
                    const int64_t x = (int64_t)a, y = (int64_t)b;
                    if (x == INT64_MIN && y == -1) {
                        q = (uint64_t)INT64_MIN;
                        rm = 0;
                    } else {
                        int64_t qq = x / y, rr = x % y;
                        if (rr != 0 && ((x < 0) != (y < 0))) {
                            qq -= 1;
                            rr += y;
                        }
                        q = (uint64_t)qq;
                        rm = (uint64_t)rr;
                    }
                }
                res = op == D_FLOORDIV_I ? q : rm;
                break;
            }
            case D_EQ_U: case D_NE_U: case D_LT_U: case D_LE_U: case D_GT_U: case D_GE_U: {
                const int c = op - D_EQ_U;
                res = (c == 0 ? a == b : c == 1 ? a != b : c == 2 ? a < b : c == 3 ? a <= b : c == 4 ? a > b : a >= b)
                          ? 1ull : 0ull;
                break;
            }
            case D_BAND: res = a & b; break;
            case D_BOR: res = a | b; break;
            case D_BXOR: res = a ^ b; break;
            case D_XOR: res = (a ^ b) & 1ull; break;
            case D_FILL_NULL:
                res = va ? a : b;
                ok = va | vb;
                break;
            case D_EQ_F: case D_NE_F: case D_LT_F: case D_LE_F: case D_GT_F: case D_GE_F:
                res = cmp_f(op - D_EQ_F, as_f64(a), as_f64(b)) ? 1ull : 0ull;
                break;
            case D_EQ_I: case D_NE_I: case D_LT_I: case D_LE_I: case D_GT_I: case D_GE_I:
                res = cmp_i(op - D_EQ_I, (int64_t)a, (int64_t)b) ? 1ull : 0ull;
                break;
            case D_EQ_B: res = (a == b) ? 1ull : 0ull; break;
            case D_NE_B: res = (a != b) ? 1ull : 0ull; break;
            case D_EQM_F: case D_NEM_F: case D_EQM_I: case D_NEM_I: case D_EQM_B: case D_NEM_B: {
                bool eq;
                if (va & vb) {
                    eq = (op == D_EQM_F || op == D_NEM_F) ? tot_eq_f(as_f64(a), as_f64(b)) : (a == b);
                } else {
                    eq = !va && !vb;
                }
                bool ne_op = (op == D_NEM_F || op == D_NEM_I || op == D_NEM_B);
                res = (ne_op ? !eq : eq) ? 1ull : 0ull;
                ok = true;
                break;
            }
            case D_AND: {
                // Kleene: false dominates nulls.
                bool fa = va && !(a & 1), fb = vb && !(b & 1);
                if (fa || fb) { res = 0; ok = true; }
                else { res = 1; ok = va & vb; }
                break;
            }
            case D_OR: {
                bool ta = va && (a & 1), tb = vb && (b & 1);
                if (ta || tb) { res = 1; ok = true; }
                else { res = 0; ok = va & vb; }
                break;
            }
            default: break;
            }
            POP1();
            s0 = res;
            vm = (vm & ~1u) | (ok ? 1u : 0u);
            break;
        }
        }
    }
#undef PUSH
#undef POP1
    (void)s7;
    return RowVal{s0, (vm & 1u) != 0};
}

// Fast-path predicate `col <cmp> imm` (null handled by the caller),
// branch-free: classify the pair as lt / eq / gt under the total order
// (trichotomy holds with NaN greatest, NaN == NaN) and test the class
// against the op's accept mask.  op 0..5 = eq, ne, lt, le, gt, ge with
// masks (lt=1, eq=2, gt=4) 2, 5, 1, 3, 4, 6 packed one nibble per op.
__device__ __forceinline__ bool simple_pred(bool isf, int op, uint64_t x, uint64_t imm) {
    const uint32_t accept = (0x643152u >> (4 * op)) & 0xFu;
    uint32_t cls;
    if (isf) {
        const double a = as_f64(x), b = as_f64(imm);
        const bool an = __builtin_isnan(a), bn = __builtin_isnan(b);
        const bool eq = (an & bn) | (a == b);
        const bool lt = !an & (bn | (a < b));
        cls = eq ? 2u : (lt ? 1u : 4u);
    } else {
        const int64_t a = (int64_t)x, b = (int64_t)imm;
        cls = a == b ? 2u : (a < b ? 1u : 4u);
    }
    return (cls & accept) != 0u;
}

// Fibonacci hashing of a 64-bit key into `bits` bits.
__device__ __forceinline__ uint32_t hash_slot(uint64_t key, int bits) {
    return bits == 0 ? 0u : (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - bits));
}

// Orderable unsigned encodings: unsigned compare == total order.
__device__ __forceinline__ uint64_t ord_f64(uint64_t b) {
    return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ uint64_t unord_f64(uint64_t u) {
    return (u & 0x8000000000000000ull) ? (u & 0x7fffffffffffffffull) : ~u;
}
__device__ __forceinline__ uint64_t ord_i64(uint64_t b) { return b ^ 0x8000000000000000ull; }

inline int wave_size() { return 64; }


constexpr int kSumWindowBits = 120;  // fixed-point window of one value (exact f64 sums)

// f64 bits -> three carry-free 40-bit limbs of the fixed-point value
// x / 2^bottom (rounded half-even below the window).  Returns false for
// zero / rounded-away values; sets FX overflow (1) / inexact (2) in fl.
template <int WBITS = kSumWindowBits>
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
    unsigned __int128 F;
    if (sh >= 0) {
        if (sh > WBITS - 53) {
            fl |= 1u;
            return false;
        }
        F = (unsigned __int128)m << sh;
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
        F = q;
    }
    constexpr uint64_t M40 = (1ull << 40) - 1;
    l0 = (uint64_t)F & M40;
    if (WBITS > 80) {
        l1 = (uint64_t)(F >> 40) & M40;
        l2 = (uint64_t)(F >> 80);
    } else {
        l1 = (uint64_t)(F >> 40);
        l2 = 0;
    }
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

// 192-bit two's complement fixed-point value * 2^bottom -> f64, rounded
// once (half-even).
__device__ __forceinline__ double fx_to_double(uint64_t w0, uint64_t w1, uint64_t w2, int bottom) {
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


// Bijective XCD-aware remap of a 1-D grid (cdna_hip_programming.md T1):
// blocks that share an XCD (same blockIdx % 8) take consecutive tiles, so
// output lines that neighbouring tiles share (the sort's digit runs and
// digit-major count words, the partition runs of the many-groups scatter)
// are completed in one L2 instead of being written back as partial lines
// from several.
__device__ __forceinline__ int64_t xcd_tile(int64_t bid, int64_t nwg) {
    const int64_t q = nwg / 8, r = nwg % 8, x = bid % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

}  // namespace plgpu
