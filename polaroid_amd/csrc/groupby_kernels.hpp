// groupby_kernels.hpp -- the group-by's shared device code and the fused
// kernel (gb_fast_kernel) with its launch templates.  The fused kernel has
// ~300 instantiations (aggregated-column count x predicate x layout x
// variant); they are compiled in six translation units, groupby_fast1..6.hip
// (explicit instantiations by aggregated-column count), so the library
// builds in parallel; groupby.hip declares them extern.  Design notes are in
// groupby.hip and DESIGN.md.
#pragma once
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

#include "plgpu_internal.hpp"
#include "scan.hpp"
#include "tuplehash.hpp"

namespace plgpu {

constexpr int kGbThreads = 512;
constexpr int kMaxAcc = 6;
constexpr int kMaxFields = 48;
constexpr int kLdsProbe = 16;
constexpr int kGlobalProbe = 4096;
constexpr int kLimb2Margin = 4;
// SLIM table (sum-only, 2 limbs) of NACC sums: the keys (L words), then per
// slot its len and each acc's two limbs and flags word, slot-major, padded
// to an odd word count (two LDS banks per word: an odd stride spreads the
// slots over 32 bank pairs).  LDS words per slot:
constexpr int slim_vwords(int nacc) { return (1 + 3 * nacc) | 1; }
constexpr int slim_words(int nacc) { return 1 + slim_vwords(nacc); }
constexpr int kMinTilesPerWg = 160;  // fast kernel: fewer rounds below this many tiles per workgroup
constexpr int kGridRounds = 8;        // fast kernel grid = rounds x resident workgroups       // binades below the smallest sampled exponent kept by 2 limbs
constexpr int kHeadroomBinades = 8;   // above the sampled max exponent
constexpr int64_t kMaxRowsPerWg = int64_t(1) << 22;  // keeps 40-bit limbs exact in int64
constexpr int kPlanSamples = 65536;
constexpr int kPlanSetSlots = 4096;   // LDS hash set of the distinct-key sample (32 KiB)
constexpr int kPlanSetWord = 32;      // the plan's global key set, in words after the status block

// Acc flags
enum : int32_t { A_FSUM = 1, A_FSUMCAST = 2, A_ISUM = 4, A_CNT = 8, A_MIN = 16, A_MAX = 32, A_FLAGS = 64 };
// Per-field merge ops of partial states
enum : uint8_t { FOP_NONE = 0, FOP_ADD = 1, FOP_MIN = 2, FOP_MAX = 3, FOP_OR = 4, FOP_ADD192 = 5, FOP_SKIP = 6 };
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
    ST_DISTINCT = 6,     // plan: distinct keys in the sample (saturates at kPlanSetSlots/2)
    ST_SAMPLED = 7,      // plan: keys sampled
    ST_MAXEX = 8,        // + acc
    ST_FXFLAGS = 16,     // + acc: bit0 overflow, bit1 inexact
    ST_SHIFT_OVF = 14,   // merge: a shifted f64 sum state left the 192-bit range
    ST_MINEX = 17,       // + acc: 0x7FF - smallest exponent of a nonzero finite value (plan / maxexp)
    ST_RUNS = 23,        // plan: sampled adjacent row pairs with equal keys (sorted / clustered keys)
    ST_LOCAL = 24,       // plan: most distinct keys among the samples of one 1/kPlanKeyBlocks row range
    ST_VAR_OUT = 25,     // finalize: a fused variance whose exact state left its range (caller reruns)
    ST_KPACK = 26,       // fused key packing: a selected row's key field left its planned bits (caller repacks)
    ST_WORDS = 27
};

// An aggregation input derived from the columns in registers (an
// elementwise expression under the aggregation, polars-plan/src/plans/
// aexpr/properties/general.rs:335 can_pre_agg): value = x op y with x the
// acc's column, y a second Float64 column (c2) or a literal (dimm); every
// other expression is materialised by the host before the pass.
// DOP_SQHI / DOP_SQLO (unary, with DOP_LIT): x * x rounded, and its exact
// error fma(x, x, -(x * x)) -- the fused variance's second-moment inputs.
enum : int32_t { DOP_NONE = 0, DOP_ADD = 1, DOP_SUB = 2, DOP_MUL = 3, DOP_DIV = 4, DOP_DIVS = 5, DOP_SQHI = 6,
                 DOP_SQLO = 7, DOP_OPMASK = 7, DOP_SWAP = 8, DOP_LIT = 16 };

struct AccSpec {
    DevCol c;         // the aggregated column (derived: the first operand column)
    int32_t flags;
    int32_t isf;      // column is f64 (compared / summed as f64)
    int32_t f_sum;    // FSUM/FSUMCAST: 3 limb fields
    int32_t f_isum;
    int32_t f_cnt;
    int32_t f_min;
    int32_t f_max;
    int32_t f_flags;
    int32_t uns;      // UInt64 column: min / max order and f64 conversion are unsigned
    int32_t dop;      // DOP_*: derived input (0: the column itself)
    DevCol c2;        // derived: the second operand column (unless DOP_LIT)
    uint64_t dimm;    // derived: the literal operand's f64 bits (DOP_LIT)
    int32_t v_from;   // fused kernel (DERIV): c is acc v_from's column too (-1: own load)
    int32_t w_from;   // fused kernel (DERIV): c2 is acc w_from's column (-1: own load)
};

// Fused key packing (round 4): the group key of row r is the exact Int64
// code of the tuple of up to kKpMax null-free Int64 / Int32 / UInt32 key
// columns in mk_plan_pack's layout (field i = v - minv[i] + nul[i] at bit
// shift[i], polars-core/src/chunked_array/ops/row_encode.rs:189 encodes
// the same tuple as bytes), formed in registers from the key columns as the
// tile arrives -- no code column is written or read.  n = 0: the key is
// GbParams::key itself.  A selected row whose field leaves its bits sets
// ST_KPACK and the caller repacks with the exact ranges.
// A String key (n = 1, c[0].dtype PLGPU_STR, null-free) is formed the same
// way as its exact short-string code (len << 56) | bytes (strings.hip
// str_code_kernel) from the offsets and one or two aligned data words; a
// selected string longer than 7 bytes sets ST_KPACK (the caller takes the
// hashed long-string path).
constexpr int kKpMax = 4;
struct KeyPack {
    int32_t n;
    int32_t _pad;
    DevCol c[kKpMax];
    uint64_t base[kKpMax];  // minv[i] - nul[i] (wrapping): field i = v - base[i]
    // field i fits iff v - base[i] (wrapping) <= span[i] = min(2^bits - 1,
    // 2^64 - 1 - ord(base)), ord(x) = x ^ 2^63: one unsigned compare that is
    // false for every v < base too (kp_span)
    uint64_t span[kKpMax];
    // 4-byte columns whose base lies in the column type's range: the same
    // test on 32-bit ordered values (ord32(v) - b32 <= span32, ord32 = v ^ x32)
    uint32_t b32[kKpMax];
    uint32_t span32[kKpMax];
    uint32_t x32[kKpMax];
    int32_t mode[kKpMax];   // 0: 8-byte column, 1: 4-byte on 32-bit values, 2: 4-byte widened to 64 bits
    int32_t shift[kKpMax];
    int32_t bits[kKpMax];
    int64_t data_end;       // String key: bytes in the data buffer (bounds the word loads)
};

struct GbParams {
    DevCol key;
    DevCol cols[PLGPU_MAX_COLS];  // all input columns (program predicates)
    DevCol pred_col;              // simple predicate column
    int64_t n;
    int64_t row_begin;            // generic kernel: first row it owns
    int64_t n_full;               // fast kernel: rows [0, n_full), a multiple of its tile
    int32_t _pad1;
    int32_t _pad2;
    int32_t nacc;
    int32_t nfields;
    AccSpec acc[kMaxAcc];
    uint64_t desc[kMaxAcc];  // packed per-acc descriptors (see dfield)
    int32_t bottom[kMaxAcc]; // fixed-point bottoms of the main launch (by value)
    uint8_t fop[kMaxFields]; // per-field merge op (partial-state merge)
    int32_t pred_acc;       // acc whose column is the simple predicate's, or -1
    int32_t f_len;
    int32_t f_first;        // min selected row per group: maintain_order / first(); else -1
    int32_t f_last;         // max selected row per group: last(); else -1
    int32_t lbits;
    uint64_t min_init_mask; // fields initialised to ~0
    int32_t lcap;
    int32_t gbits;
    int64_t gcap;
    uint64_t* gtab;         // nfields regions of (gcap + 2) words; field 0 = keys
    const int32_t* bottoms; // [kMaxAcc]
    uint64_t* status;       // [ST_WORDS]
    // partitioned launches (gb_kernel<.., PART>): partition q = b / part_blocks
    // owns rows [part_range[q], part_range[q + 1]) of the partition buffers;
    // part_rows maps them back to input rows (first-row field)
    const uint64_t* part_range;
    const uint32_t* part_rows;
    // null bits of each partitioned row (null unless an input column has a
    // validity bitmap): bit a = acc a's value is null, bit 6 = the key is
    // null (the row belongs to the null group)
    const uint8_t* part_nulls;
    int32_t part_blocks;
    // fast kernel, range-local mode (clustered keys): workgroup b takes the
    // contiguous tiles [b * tiles_per_wg, (b + 1) * tiles_per_wg); 0 = the
    // grid-strided tile order
    int32_t tiles_per_wg;
    // partitioned run with one workgroup per partition: each partition's
    // groups live in a region of 2^rbits global slots (g_slot); 0 = off
    int32_t rbits;
    // every validity bitmap of the key / aggregated / predicate columns has a
    // column offset that is a multiple of 64 and an 8-byte aligned buffer:
    // a wave's validity bits come as whole 64-bit words (fast_nulls,
    // ps_keys) instead of one byte load per lane
    int32_t vwords;
    KeyPack kp;             // fused key packing (kp.n > 0): the key is the packed tuple code
    // compact regions (one workgroup per partition, the slim sum-only
    // layout; null = off): the workgroup of partition q writes its LDS
    // groups densely, in slot order, to slots [q lcap, q lcap +
    // region_cnt[q]) of the region table rtab (field f of slot t at
    // rtab[f * rcap + t], never initialised) and stores that count.  gtab
    // is then a small hashed overflow table (rbits = 0, initialised): the
    // rows of keys that found no LDS slot (a key's rows all miss, or none
    // do: one workgroup sees every row of its partition) and the two
    // special groups.  The finalize reads the regions' dense prefixes, then
    // the overflow table.
    uint32_t* region_cnt;
    uint64_t* rtab;
    int64_t rcap;
    int32_t wave_report;    // option wave_report: per-wave status atomics (A/B of report_wg)
    // partition buffers of a sum-only run whose null keys were written as
    // null_key (a value no non-null key holds): those rows are the null group
    int32_t has_null_key;
    int64_t null_key;
};

// ------------------------------------------------------ invariant checks
// Checked build (make CHECKS=1: -DPLGPU_CHECKS, libpolaroid_gpu_checked.so):
// a violated index invariant sets its bit in g_gb_checks and the access is
// skipped, never performed; plgpu_debug_checks returns and clears the bits.
// The product build compiles every check away (gb_ok is constant true).
enum : uint32_t {
    CK_LDS_SLOT = 1,      // LDS table slot outside [0, lcap + 2)
    CK_GLOBAL_SLOT = 2,   // global table slot outside [0, gcap + 2)
    CK_FAST_SLOT = 4,     // fused kernel LDS slot outside [0, lcap + 2)
    CK_FIRST_ROW = 8,     // first / last row id outside [0, n)
    CK_MERGE_SLOT = 16,   // merge slot outside the table
    CK_REP_ROW = 32,      // multi-key representative row outside [0, n)
    CK_VERIFY_SLOT = 64,  // multi-key verify slot outside the table
    CK_PART_POS = 128,    // partition scatter position outside the buffers
    CK_KEY_ROW = 256,     // multi-key output key row outside [0, n)
    CK_PERM = 512,        // group-order permutation entry outside [0, groups)
    CK_REGION = 1024,     // compact region slot outside its partition's region / the region table
    CK_FIELD = 1024       // apply_row: table field outside [0, nfields)
};
#ifdef PLGPU_CHECKS
// one copy per translation unit (the fused kernels are compiled in
// groupby_fast*.hip): each registers its reader with groupby.hip
using GbChecksTake = uint32_t (*)();
void gb_checks_register(GbChecksTake f);
static __device__ unsigned int g_gb_checks;
static __device__ unsigned long long g_gb_sink;  // target of a skipped field access
static uint32_t gb_checks_take_local() {
    uint32_t v = 0, z = 0;
    (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_gb_checks), sizeof v);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_gb_checks), &z, sizeof z);
    return v;
}
static const bool g_gb_checks_registered = (gb_checks_register(&gb_checks_take_local), true);
__device__ __forceinline__ bool gb_ok(bool c, uint32_t bit) {
    if (!c) atomicOr(&g_gb_checks, bit);
    return c;
}
__device__ __forceinline__ unsigned long long* gb_sink() { return &g_gb_sink; }
#else
__device__ __forceinline__ constexpr bool gb_ok(bool, uint32_t) { return true; }
__device__ __forceinline__ unsigned long long* gb_sink() { return nullptr; }
#endif

// ------------------------------------------------------------ helpers
// Derived input: x op y in f64 (DOP_SWAP: y op x; DOP_DIVS: a * (1 / b), the
// scalar-divisor form, polars-compute/src/arithmetic/float.rs:78).  The
// library is built with -ffp-contract=off: one IEEE rounding per operation,
// as the reference's elementwise kernel.
__device__ __forceinline__ uint64_t derive(int32_t dop, uint64_t x, uint64_t y) {
    const double xa = as_f64(x), ya = as_f64(y);
    const double a = (dop & DOP_SWAP) ? ya : xa, b = (dop & DOP_SWAP) ? xa : ya;
    double r;
    switch (dop & DOP_OPMASK) {
    case DOP_ADD: r = a + b; break;
    case DOP_SUB: r = a - b; break;
    case DOP_MUL: r = a * b; break;
    case DOP_DIV: r = a / b; break;
    case DOP_DIVS: r = a * (1.0 / b); break;
    case DOP_SQHI: r = xa * xa; break;
    default: {
        const double h = xa * xa;
        r = __builtin_fma(xa, xa, -h);  // exact: x * x == h + r for 2^-484 <= |x| < 2^511
        break;
    }
    }
    return f64_bits(r);
}

// Aggregation input of row r (register form) and its validity.
__device__ __forceinline__ uint64_t acc_value(const AccSpec& ac, int64_t r, bool& valid) {
    valid = dev_valid(ac.c, r);
    const uint64_t x = dev_load(ac.c, r);
    if (ac.dop == DOP_NONE) return x;
    if (ac.dop & DOP_LIT) return derive(ac.dop, x, ac.dimm);
    valid = valid && dev_valid(ac.c2, r);
    return derive(ac.dop, x, dev_load(ac.c2, r));
}

// Group key of row r: `values` NULL is the keyless form (a global
// reduction, select(agg...)): every row in the one group 0.
__device__ __forceinline__ uint64_t key_at(const DevCol& k, int64_t r) {
    return k.values ? dev_load(k, r) : 0ull;
}

// Field i of a packed key from the column's loaded word (`raw`: the 8-byte
// value, or a 4-byte value in the low half), OR-ing into `bad` when it does
// not fit its planned bits.
__device__ __forceinline__ uint64_t kp_field(const KeyPack& k, int i, uint64_t raw, bool& bad) {
    const int32_t dt = k.c[i].dtype;
    const uint64_t v = dt == PLGPU_I32 ? (uint64_t)(int64_t)(int32_t)(uint32_t)raw
                                       : (dt == PLGPU_U32 ? (uint64_t)(uint32_t)raw : raw);
    const uint64_t f = v - k.base[i];
    bad |= f > k.span[i];
    return f << k.shift[i];
}

// Short-string code of the string [b, b + len) of a String column's data
// (len <= 7; `bad` when longer): aligned word loads within data_end, bytes
// otherwise.
__device__ __forceinline__ uint64_t kp_str_code(const uint8_t* data, int64_t data_end, uint64_t b, uint64_t len,
                                                bool& bad) {
    if (len > 7) {
        bad = true;
        return 0;
    }
    if (len == 0) return 0;
    const uint64_t* dw = (const uint64_t*)data;
    const uint64_t w = b >> 3;
    const int sh = (int)(b & 7) * 8;
    uint64_t x;
    if ((int64_t)b + 16 <= data_end) {
        // both words inside the buffer (every row but the last few): a
        // funnel shift of the pair, no per-row branch on the word boundary
        const uint64_t lo = dw[w], hi = dw[w + 1];
        x = (lo >> sh) | ((hi << 1) << (63 - sh));
    } else if ((int64_t)((w + 1) * 8) <= data_end && (sh + 8 * (int)len <= 64 || (int64_t)((w + 2) * 8) <= data_end)) {
        x = dw[w] >> sh;
        if (sh + 8 * (int)len > 64) x |= dw[w + 1] << (64 - sh);
    } else {
        x = 0;
        for (uint64_t j = 0; j < len; ++j) x |= (uint64_t)data[b + j] << (8 * j);
    }
    return (len << 56) | (x & ((1ull << (8 * len)) - 1));
}

// The group key of row r as every pass but the fused kernel's tile loads
// reads it: the key column, or the packed code of the key columns.
__device__ __forceinline__ uint64_t gb_key(const GbParams& p, int64_t r) {
    if (p.kp.n == 0) return key_at(p.key, r);
    if (p.kp.c[0].dtype == PLGPU_STR) {
        const int64_t* o = (const int64_t*)p.kp.c[0].values + p.kp.c[0].offset + r;
        bool bad = false;
        return kp_str_code(p.kp.c[0].data, p.kp.data_end, (uint64_t)o[0], (uint64_t)(o[1] - o[0]), bad);
    }
    uint64_t code = 0;
    bool bad = false;
    for (int i = 0; i < p.kp.n; ++i) code |= kp_field(p.kp, i, dev_load(p.kp.c[i], r), bad);
    return code;
}
__device__ __forceinline__ bool gb_key_valid(const GbParams& p, int64_t r) {
    return p.kp.n > 0 || dev_valid(p.key, r);
}

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

// (part_hash, the many-groups path's partition hash: tuplehash.hpp)

// Probe i of `key` in the global table.  A partitioned run whose partitions
// each have one workgroup (p.rbits > 0) keeps every partition's groups in a
// region of its own, 2^rbits slots at region index = the partition (the
// partition hash's top gbits - rbits bits), probed with the LDS table's hash:
// the partition's workgroup then writes its LDS table into the region slot
// for slot (DESIGN.md "Group-by for many groups").
__device__ __forceinline__ uint64_t g_slot(const GbParams& p, uint64_t key, uint64_t i) {
    if (p.rbits > 0) {
        const int qb = p.gbits - p.rbits;
        const uint64_t q = qb > 0 ? part_hash(key) >> (64 - qb) : 0ull;
        const uint64_t rm = (1ull << p.rbits) - 1;
        return (q << p.rbits) | (((uint64_t)hash_slot(key, p.rbits) + i) & rm);
    }
    const uint64_t h = p.gbits == 0 ? 0 : ((key * 0x9E3779B97F4A7C15ull) >> (64 - p.gbits));
    return (h + i) & ((uint64_t)p.gcap - 1);
}
__device__ __forceinline__ int g_probe_limit(const GbParams& p) {
    const int64_t span = p.rbits > 0 ? (int64_t(1) << p.rbits) : p.gcap;
    return span < kGlobalProbe ? (int)span : kGlobalProbe;
}

// Global probe: slot index or -1; `inserted` when this call claimed the
// slot (the caller counts new keys, one atomic per wave: a per-key add to
// one status word serialises).  A plain load may return a stale EMPTY
// (another CU inserted since); the CAS then returns the true key, so the
// protocol never needs an acquire: keys only ever go EMPTY -> key.
__device__ __forceinline__ int64_t g_find_ins(const GbParams& p, uint64_t key, bool& inserted) {
    uint64_t* gkeys = p.gtab;
    const int lim = g_probe_limit(p);
    for (int i = 0; i < lim; ++i) {
        const uint64_t s = g_slot(p, key, (uint64_t)i);
        uint64_t k = __hip_atomic_load(&gkeys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == key) return (int64_t)s;
        if (k == kEmptyKey) {
            k = atomicCAS((unsigned long long*)&gkeys[s], (unsigned long long)kEmptyKey, (unsigned long long)key);
            if (k == kEmptyKey) {
                inserted = true;
                return (int64_t)s;
            }
            if (k == key) return (int64_t)s;
        }
    }
    return -1;
}
__device__ __forceinline__ int64_t g_find(const GbParams& p, uint64_t key) {
    bool ins = false;
    const int64_t s = g_find_ins(p, key, ins);
    if (ins) atomicAdd((unsigned long long*)&p.status[ST_NEWKEYS], 1ull);
    return s;
}

// Branch-free conversion for the common case: a finite value whose bits all
// fall inside the window (no rounding, no overflow), or zero.  LIMBS 3: the
// 120-bit window at `bottom`; LIMBS 2: its top 80 bits (bottom + 40), limbs
// returned in l0, l1 (l2 = 0).  Returns false (limbs 0) when the value needs
// fx_limbs (inf / NaN, bits below the window, overflow).
template <int LIMBS>
__device__ __forceinline__ bool fx_limbs_fast(uint64_t x, int bottom, uint64_t& l0, uint64_t& l1, uint64_t& l2,
                                              bool nonneg = false) {
    if (LIMBS == 2) {
        // The 2-limb form with the least VALU work (the fused kernels are
        // issue-bound): the mantissa keeps its implicit bit only for ex != 0,
        // so a zero gives zero limbs whatever the shift, and nothing is
        // zeroed for values outside the window -- their limbs are garbage
        // and the callers use limbs only on a true return.  Shift amounts
        // are taken mod 64 (the hardware's own masking).
        constexpr uint64_t M40 = (1ull << 40) - 1;
        constexpr int W = kSumWindowBits - 40;
        const uint32_t hi = (uint32_t)(x >> 32), lo = (uint32_t)x;
        const uint32_t ex = (hi >> 20) & 0x7FF;
        const uint32_t sh = ex - (uint32_t)(1075 + bottom + 40);
        const bool inrange = sh <= (uint32_t)(W - 53) && ex != 0;
        const bool zero = ((hi << 1) | lo) == 0;
        const uint64_t m = (x & 0x000FFFFFFFFFFFFFull) | ((uint64_t)(ex != 0 ? 1u : 0u) << 52);
        // nonneg: the caller knows x >= 0 (the variance triple's x * x), no
        // sign to apply (a NaN's sign does not matter: it fails the window)
        const int64_t sm = (!nonneg && (int32_t)hi < 0) ? -(int64_t)m : (int64_t)m;
        l0 = ((uint64_t)sm << (sh & 63)) & M40;
        l1 = (uint64_t)(sm >> ((40 - sh) & 63));  // sh <= 27 when used
        l2 = 0;
        return inrange || zero;
    }
    // The signed value t = +-m * 2^sh (sh >= 0, t < 2^W) is split as
    // t = l0 + l1 * 2^40 (+ l2 * 2^80) with l0 (and l1 in the 3-limb case)
    // taken as the low 40 bits (>= 0) and the top limb as the arithmetic
    // shift (signed): carry-free, exact, and no per-limb negation.
    // Subnormals take the slow path (ex == 0 is only accepted for zero);
    // inf / NaN exceed the window for every reachable bottom.
    constexpr uint64_t M40 = (1ull << 40) - 1;
    constexpr int W = LIMBS == 3 ? kSumWindowBits : kSumWindowBits - 40;
    const uint32_t hi = (uint32_t)(x >> 32);
    const uint32_t ex = (hi >> 20) & 0x7FF;
    const int sh = (int)ex - 1075 - (LIMBS == 3 ? bottom : bottom + 40);
    const bool inrange = (uint32_t)sh <= (uint32_t)(W - 53) && ex != 0;
    const bool zero = (x & 0x7fffffffffffffffull) == 0;
    const uint64_t m = inrange ? ((x & 0x000FFFFFFFFFFFFFull) | (1ull << 52)) : 0ull;
    const int64_t sm = (int64_t)x < 0 ? -(int64_t)m : (int64_t)m;
    const uint32_t s = inrange ? (uint32_t)sh : 0u;
    if (LIMBS == 3) {
        l0 = s < 40 ? ((uint64_t)sm << s) & M40 : 0ull;
        l1 = (s <= 40 ? (uint64_t)(sm >> (40 - s)) : ((uint64_t)sm << (s - 40))) & M40;
        l2 = (uint64_t)(sm >> (s > 16 ? 80 - s : 63));
    } else {
        l0 = ((uint64_t)sm << s) & M40;
        l1 = (uint64_t)(sm >> (40 - s));  // s <= 27
        l2 = 0;
    }
    return inrange || zero;
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

__device__ __forceinline__ uint64_t widen32(uint32_t v, int32_t dtype) {
    return dtype == PLGPU_U32 ? (uint64_t)v : (uint64_t)(int64_t)(int32_t)v;
}

// Two consecutive rows (r0, r0+1) of a column; one 16-byte (8-byte for
// 32-bit types) load when both are in range and the pair is aligned.
__device__ __forceinline__ void load_pair(const DevCol& c, int64_t r0, int64_t n, uint64_t& a, uint64_t& b) {
    const int64_t p = c.offset + r0;
    const bool wide = c.dtype == PLGPU_F64 || c.dtype == PLGPU_I64 || c.dtype == PLGPU_U64;
    const bool w32 = c.dtype == PLGPU_I32 || c.dtype == PLGPU_U32;
    if (r0 + 1 < n && (p & 1) == 0 && (wide || w32)) {
        if (wide) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2*>((const uint64_t*)c.values + p);
            a = v.x;
            b = v.y;
        } else {
            const uint2 v = *reinterpret_cast<const uint2*>((const uint32_t*)c.values + p);
            a = widen32(v.x, c.dtype);
            b = widen32(v.y, c.dtype);
        }
    } else {  // unaligned pair, tail, or a 1 / 2-byte / Float32 column: register-form loads
        a = r0 < n ? dev_load(c, r0) : 0ull;
        b = r0 + 1 < n ? dev_load(c, r0 + 1) : 0ull;
    }
}

// Per-thread running diagnostics, reduced once per wave.
struct ThreadDiag {
    uint32_t fxbits;   // 2 bits per acc: overflow (1), inexact (2)
    uint32_t nsel;
    uint32_t nglobal;
    uint32_t special;
    uint32_t kbad;     // fused key packing: a selected row's field left its bits
    uint32_t newkeys;  // global-table slots this thread claimed
};

// Packed per-acc descriptor word (uniform): field indices and flags, so the
// per-row code walks the accs in a rolled loop with one copy of the logic
// and only two scalar registers per acc live.
//   [0,8) flags  [8,16) f_sum  [16,24) f_isum  [24,32) f_cnt
//   [32,40) f_min  [40,48) f_max  [48,56) f_flags  [56] isf  [57] unsigned (UInt64)
// Absent fields are 0xFF.
__device__ __forceinline__ int dfield(uint64_t d, int sh) { return (int)((d >> sh) & 0xFF); }
constexpr int kNoField = 0xFF;

// Apply one selected row's aggregated values to slot s of the LDS table
// (LDS=true) or of the global table.  `v` / `dd` / `bot` are consumed
// (rotated) in place.
template <bool LDS, int NA>
__device__ __forceinline__ void apply_row(const GbParams& p, uint64_t* lds, int L, int64_t s, int64_t row,
                                          uint64_t (&v)[NA], uint32_t vm, uint64_t (&dd)[NA], int (&bot)[NA],
                                          int nacc, ThreadDiag& diag) {
    auto F = [&](int f) -> unsigned long long* {
        if (!gb_ok(f >= 0 && f < p.nfields, CK_FIELD)) return gb_sink();
        if (LDS) return (unsigned long long*)&lds[f * L + s];
        return (unsigned long long*)gfield(p, f, s);
    };
    if (!gb_ok(s >= 0 && s < (LDS ? (int64_t)L : p.gcap + 2), LDS ? CK_LDS_SLOT : CK_GLOBAL_SLOT)) return;
    atomicAdd(F(p.f_len), 1ull);
    if (p.f_first >= 0) atomicMin(F(p.f_first), (unsigned long long)row);
    if (p.f_last >= 0) atomicMax(F(p.f_last), (unsigned long long)row);
#pragma unroll 1
    for (int k = 0; k < nacc; ++k) {
        const uint64_t d = dd[0];
        const uint32_t flags = (uint32_t)d & 0xFF;
        const uint64_t x = v[0];
        if (vm & 1u) {
            const int f_cnt = dfield(d, 24);
            if (f_cnt != kNoField) atomicAdd(F(f_cnt), 1ull);
            const bool isf = (d >> 56) & 1;
            bool is_nan = false;
            bool fsum_ok = false;
            uint64_t sb = x;  // bits summed as f64
            if (isf) {
                const uint64_t ab = x & 0x7fffffffffffffffull;
                if (ab >= 0x7ff0000000000000ull) {
                    const uint32_t fl = ab > 0x7ff0000000000000ull ? FL_NAN : ((x >> 63) ? FL_NINF : FL_PINF);
                    is_nan = fl == FL_NAN;
                    // every f64 acc has a flags field (plan_groupby), also
                    // one aggregated only by len / count / first / last: its
                    // absence was round 2's out-of-table write (DESIGN.md
                    // "GPU fault audit")
                    atomicOr(F(dfield(d, 48)), (unsigned long long)fl);
                } else {
                    fsum_ok = (flags & A_FSUM) != 0;
                }
            } else if (flags & A_FSUMCAST) {
                sb = f64_bits(((d >> 57) & 1) ? (double)x : (double)(int64_t)x);
                fsum_ok = true;
            }
            if (fsum_ok) {
                uint64_t l0, l1, l2;
                uint32_t ex = 0, fl = 0;
                const bool ok = fx_limbs(sb, bot[0], l0, l1, l2, fl, ex);
                diag.fxbits |= fl << (2 * k);
                if (ok) {
                    const int f = dfield(d, 8);
                    if (LDS) {
                        atomicAdd(F(f), (unsigned long long)l0);
                        atomicAdd(F(f + 1), (unsigned long long)l1);
                        atomicAdd(F(f + 2), (unsigned long long)l2);
                    } else {
                        uint64_t w0, w1, w2;
                        limbs_to_192((int64_t)l0, (int64_t)l1, (int64_t)l2, w0, w1, w2);
                        g_add192((uint64_t*)F(f), (uint64_t*)F(f + 1), (uint64_t*)F(f + 2), w0, w1, w2);
                    }
                }
            }
            if ((flags & (A_MIN | A_MAX)) && !is_nan) {
                const uint64_t o = isf ? ord_f64(x) : (((d >> 57) & 1) ? x : ord_i64(x));
                if (flags & A_MIN) atomicMin(F(dfield(d, 32)), (unsigned long long)o);
                if (flags & A_MAX) atomicMax(F(dfield(d, 40)), (unsigned long long)o);
            }
            if (flags & A_ISUM) atomicAdd(F(dfield(d, 16)), (unsigned long long)x);
        }
        // rotate the per-acc registers (static moves, no indexed access)
#pragma unroll
        for (int i = 0; i + 1 < NA; ++i) {
            v[i] = v[i + 1];
            dd[i] = dd[i + 1];
            bot[i] = bot[i + 1];
        }
        vm >>= 1;
    }
}

// Row on the global table.  kvalid=false -> null group slot.
template <int NA>
__device__ __forceinline__ void global_row(const GbParams& p, uint64_t key, bool kvalid, int64_t row,
                                           uint64_t (&v)[NA], uint32_t vm, uint64_t (&dd)[NA], int (&bot)[NA],
                                           int nacc, ThreadDiag& diag) {
    int64_t gs;
    if (!kvalid) gs = p.gcap;
    else if (key == kEmptyKey) gs = p.gcap + 1;
    else {
        bool ins = false;
        gs = g_find_ins(p, key, ins);
        diag.newkeys += ins ? 1u : 0u;
    }
    if (gs < 0) {
        atomicAdd((unsigned long long*)&p.status[ST_TABLE_FULL], 1ull);
        return;
    }
    if (gs >= p.gcap) diag.special |= gs == p.gcap ? 1u : 2u;
    apply_row<false, NA>(p, nullptr, 0, gs, row, v, vm, dd, bot, nacc, diag);
}

// Partition region of a one-workgroup-per-partition run (p.rbits > 0):
// claim LDS slot s's own global slot for `key` -- region q (this
// workgroup's partition), slot s -- or -1 when an overflow row's key took it
// first (the caller then probes with g_find).  A claimed slot belongs to this
// thread alone: its fields are written with plain stores.
__device__ __forceinline__ int64_t g_direct_claim(const GbParams& p, int s, uint64_t key) {
    const int64_t t = ((int64_t)(blockIdx.x / p.part_blocks) << p.rbits) + s;
    return atomicCAS((unsigned long long*)&p.gtab[t], (unsigned long long)kEmptyKey, (unsigned long long)key) ==
                   kEmptyKey
               ? t
               : -1;
}

// End of a main launch: fold the workgroup's LDS table into the global
// table, then publish the per-thread diagnostics (one atomic per wave).
template <bool USE_LDS>
__device__ __forceinline__ void flush_and_report(const GbParams& p, uint64_t* lds, int L, ThreadDiag& d) {
    if (USE_LDS) {
        __syncthreads();
        for (int s = threadIdx.x; s < L; s += blockDim.x) {
            const uint64_t len = lds[p.f_len * L + s];
            if (len == 0) continue;
            int64_t gs;
            if (s == p.lcap) {
                gs = p.gcap;
                d.special |= 1u;
            } else if (s == p.lcap + 1) {
                gs = p.gcap + 1;
                d.special |= 2u;
            } else {
                const int64_t t = p.rbits > 0 ? g_direct_claim(p, s, lds[s]) : -1;
                if (t >= 0) {
                    // the partition's own region slot: plain stores of the
                    // LDS state (the global fields start at the same initial
                    // values as the LDS ones)
                    ++d.newkeys;
                    *gfield(p, p.f_len, t) = len;
                    if (p.f_first >= 0) *gfield(p, p.f_first, t) = lds[p.f_first * L + s];
                    if (p.f_last >= 0) *gfield(p, p.f_last, t) = lds[p.f_last * L + s];
                    for (int a = 0; a < p.nacc; ++a) {
                        const AccSpec& ac = p.acc[a];
                        if (ac.f_cnt >= 0) *gfield(p, ac.f_cnt, t) = lds[ac.f_cnt * L + s];
                        if (ac.flags & (A_FSUM | A_FSUMCAST)) {
                            uint64_t w0, w1, w2;
                            limbs_to_192((int64_t)lds[ac.f_sum * L + s], (int64_t)lds[(ac.f_sum + 1) * L + s],
                                         (int64_t)lds[(ac.f_sum + 2) * L + s], w0, w1, w2);
                            *gfield(p, ac.f_sum, t) = w0;
                            *gfield(p, ac.f_sum + 1, t) = w1;
                            *gfield(p, ac.f_sum + 2, t) = w2;
                        }
                        if (ac.flags & A_ISUM) *gfield(p, ac.f_isum, t) = lds[ac.f_isum * L + s];
                        if (ac.flags & A_MIN) *gfield(p, ac.f_min, t) = lds[ac.f_min * L + s];
                        if (ac.flags & A_MAX) *gfield(p, ac.f_max, t) = lds[ac.f_max * L + s];
                        if (ac.f_flags >= 0) *gfield(p, ac.f_flags, t) = lds[ac.f_flags * L + s];
                    }
                    continue;
                }
                bool ins = false;
                gs = g_find_ins(p, lds[s], ins);
                d.newkeys += ins ? 1u : 0u;
                if (gs < 0) {
                    atomicAdd((unsigned long long*)&p.status[ST_TABLE_FULL], 1ull);
                    continue;
                }
            }
            atomicAdd((unsigned long long*)gfield(p, p.f_len, gs), (unsigned long long)len);
            if (p.f_first >= 0)
                atomicMin((unsigned long long*)gfield(p, p.f_first, gs), (unsigned long long)lds[p.f_first * L + s]);
            if (p.f_last >= 0)
                atomicMax((unsigned long long*)gfield(p, p.f_last, gs), (unsigned long long)lds[p.f_last * L + s]);
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
                    g_add192(gfield(p, ac.f_sum, gs), gfield(p, ac.f_sum + 1, gs), gfield(p, ac.f_sum + 2, gs), w0,
                             w1, w2);
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
    }
    uint64_t nsel = d.nsel, nglob = d.nglobal, nk = d.newkeys;
    uint32_t special = d.special, fx = d.fxbits;
    const bool kbad = __any(d.kbad != 0);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        nsel += __shfl_xor(nsel, off, 64);
        nglob += __shfl_xor(nglob, off, 64);
        nk += __shfl_xor(nk, off, 64);
        special |= __shfl_xor(special, off, 64);
        fx |= __shfl_xor(fx, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (kbad) atomicOr((unsigned long long*)&p.status[ST_KPACK], 1ull);
        if (nsel) atomicAdd((unsigned long long*)&p.status[ST_SELECTED], (unsigned long long)nsel);
        if (nglob) atomicAdd((unsigned long long*)&p.status[ST_GLOBAL_ROWS], (unsigned long long)nglob);
        if (nk) atomicAdd((unsigned long long*)&p.status[ST_NEWKEYS], (unsigned long long)nk);
        if (special) atomicOr((unsigned long long*)&p.status[ST_SPECIAL], (unsigned long long)special);
        if (fx) atomicOr((unsigned long long*)&p.status[ST_FXFLAGS], (unsigned long long)fx);
    }
}

// The end of a fused launch whose dynamic LDS has kWgScratch bytes after
// its table (`sc`): the diagnostics summed per wave, then per workgroup
// through `sc`, and published with one atomic per status word and
// workgroup.  Same-address atomics serialise (about 11 ns each on one
// status word, measured on the finalize's counter), so per-wave publication
// costs ~0.7 ms at the headline's 32,768 waves and most of the many-groups
// aggregation at 2^15 workgroups of 8 waves.
constexpr int kWgScratch = 256;  // 16 waves x 4 words
__device__ __forceinline__ void report_wg(const GbParams& p, const ThreadDiag& d, uint32_t* sc) {
    uint64_t nsel = d.nsel, nglob = d.nglobal, nk = d.newkeys;
    uint32_t special = d.special, fx = d.fxbits;
    const bool kbad = __any(d.kbad != 0);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        nsel += __shfl_xor(nsel, off, 64);
        nglob += __shfl_xor(nglob, off, 64);
        nk += __shfl_xor(nk, off, 64);
        special |= __shfl_xor(special, off, 64);
        fx |= __shfl_xor(fx, off, 64);
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();  // (the scratch's earlier use is over)
    if (lane == 0) {
        // a workgroup's rows stay below kMaxRowsPerWg: 32-bit counts
        sc[4 * wid] = (uint32_t)nsel;
        sc[4 * wid + 1] = (uint32_t)nglob;
        sc[4 * wid + 2] = (uint32_t)nk;
        sc[4 * wid + 3] = special | (fx << 2) | (kbad ? 0x80000000u : 0u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t a = 0, b = 0, c = 0;
        uint32_t o = 0;
        for (int w = 0; w < nw; ++w) {
            a += sc[4 * w];
            b += sc[4 * w + 1];
            c += sc[4 * w + 2];
            o |= sc[4 * w + 3];
        }
        if (o >> 31) atomicOr((unsigned long long*)&p.status[ST_KPACK], 1ull);
        if (a) atomicAdd((unsigned long long*)&p.status[ST_SELECTED], (unsigned long long)a);
        if (b) atomicAdd((unsigned long long*)&p.status[ST_GLOBAL_ROWS], (unsigned long long)b);
        if (c) atomicAdd((unsigned long long*)&p.status[ST_NEWKEYS], (unsigned long long)c);
        if (o & 3u) atomicOr((unsigned long long*)&p.status[ST_SPECIAL], (unsigned long long)(o & 3u));
        if ((o >> 2) & 0xFFFu)
            atomicOr((unsigned long long*)&p.status[ST_FXFLAGS], (unsigned long long)((o >> 2) & 0xFFFu));
    }
}

template <int NA>
__device__ __forceinline__ void load_descs(const GbParams& p, uint64_t (&dd)[NA], int (&bot)[NA]) {
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        // kernel-argument values: no memory access inside the row loop (a
        // load there would wait for the prefetched tile / LDS atomics)
        dd[a] = a < p.nacc ? p.desc[a] : 0ull;
        bot[a] = a < p.nacc ? p.bottom[a] : 0;
    }
}

__device__ __forceinline__ void init_lds(const GbParams& p, uint64_t* lds, int L) {
    for (int f = 0; f < p.nfields; ++f) {
        const uint64_t v = f == 0 ? kEmptyKey : (((p.min_init_mask >> f) & 1ull) ? ~0ull : 0ull);
        for (int i = threadIdx.x; i < L; i += blockDim.x) lds[f * L + i] = v;
    }
}

// slot codes of a row within a tile
constexpr int kNotSelected = -2;
constexpr int kGlobalKey = -1;
constexpr int kGlobalNull = -3;

// Generic kernel: any dtype / validity / offset / predicate, rows
// [row_begin, n) in tiles of four rows per thread.
template <int PRED, bool USE_LDS, bool PART = false>  // PRED: 0 none, 1 simple, 2 program
__global__ __launch_bounds__(kGbThreads) void gb_kernel(GbParams p, DevProgram prog) {
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const int L = p.lcap + 2;
    if (USE_LDS) init_lds(p, lds, L);
    ThreadDiag d = {0u, 0u, 0u, 0u, 0u};
    const int nacc = p.nacc;
    uint64_t dd0[kMaxAcc];
    int bot0[kMaxAcc];
    load_descs(p, dd0, bot0);
    if (USE_LDS) __syncthreads();

    int64_t n = p.n;
    const int T = blockDim.x;
    const int64_t tile = (int64_t)T * 4;
    int64_t first = p.row_begin + (int64_t)blockIdx.x * tile, stride = (int64_t)gridDim.x * tile;
    int64_t lo = 0;
    if (PART) {
        // this block's share of its partition (PRED is 0: rows are selected);
        // tiles start at an even row for the 16-byte pair loads, rows below
        // the partition's first are masked
        const int q = blockIdx.x / p.part_blocks, sub = blockIdx.x % p.part_blocks;
        lo = (int64_t)p.part_range[q];
        first = (lo & ~int64_t(1)) + (int64_t)sub * tile;
        n = (int64_t)p.part_range[q + 1];
        stride = (int64_t)p.part_blocks * tile;
    }
    for (int64_t base = first; base < n; base += stride) {
        const int64_t r0 = base + 2 * threadIdx.x;
        const int64_t r2 = r0 + 2 * T;
        uint64_t key[4], pv[4];
        uint64_t v[kMaxAcc][4];
        if (p.key.values) {
            load_pair(p.key, r0, n, key[0], key[1]);
            load_pair(p.key, r2, n, key[2], key[3]);
        } else {
            key[0] = key[1] = key[2] = key[3] = 0;  // keyless: one group
        }
#pragma unroll
        for (int a = 0; a < kMaxAcc; ++a) {
            if (a < nacc) {
                load_pair(p.acc[a].c, r0, n, v[a][0], v[a][1]);
                load_pair(p.acc[a].c, r2, n, v[a][2], v[a][3]);
            } else {
                v[a][0] = v[a][1] = v[a][2] = v[a][3] = 0;
            }
        }
        if (PRED == 1 && p.pred_acc < 0) {
            load_pair(p.pred_col, r0, n, pv[0], pv[1]);
            load_pair(p.pred_col, r2, n, pv[2], pv[3]);
        }
        int slot[4];
        uint32_t vm[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t r = (j < 2 ? r0 : r2) + (j & 1);
            bool sel = r < n && (!PART || r >= lo);
            if (sel && PRED == 1) {
                uint64_t x = pv[j];
#pragma unroll
                for (int a = 0; a < kMaxAcc; ++a)
                    if (a == p.pred_acc) x = v[a][j];
                sel = dev_valid(p.pred_col, r) && simple_pred(prog.simple_isf, prog.simple_op, x, prog.simple_imm);
            } else if (sel && PRED == 2) {
                const RowVal rv = eval_row(prog.code, prog.n, p.cols, r);
                sel = rv.valid && (rv.v & 1);
            }
            vm[j] = 0;
            slot[j] = kNotSelected;
            if (sel) {
                bool kval;
                if (PART && p.part_nulls) {
                    // the partition buffers' null bits (bit a: acc a, bit 6: key)
                    const uint32_t nb = p.part_nulls[r];
                    vm[j] = ((1u << nacc) - 1u) & ~nb;
                    kval = !((nb >> 6) & 1u);
                } else {
#pragma unroll
                    for (int a = 0; a < kMaxAcc; ++a)
                        if (a < nacc && dev_valid(p.acc[a].c, r)) vm[j] |= 1u << a;
                    kval = dev_valid(p.key, r);
                }
                if (!kval) slot[j] = USE_LDS ? p.lcap : kGlobalNull;
                else if (USE_LDS && key[j] == kEmptyKey) slot[j] = p.lcap + 1;
                else slot[j] = kGlobalKey;
            }
        }
#pragma unroll 1
        for (int j = 0; j < 4; ++j) {
            const int64_t r = (j < 2 ? r0 : r2) + (j & 1);
            int s = slot[0];
            if (s != kNotSelected) {
                ++d.nsel;
                const int64_t row = PART ? (int64_t)(p.part_rows ? p.part_rows[r] : 0) : r;
                uint64_t rv[kMaxAcc], dd[kMaxAcc];
                int bot[kMaxAcc];
#pragma unroll
                for (int a = 0; a < kMaxAcc; ++a) {
                    rv[a] = v[a][0];
                    dd[a] = dd0[a];
                    bot[a] = bot0[a];
                }
                if (USE_LDS && s == kGlobalKey) s = lds_find(lds, p.lbits, p.lcap, key[0]);
                if (s >= 0) {
                    apply_row<true, kMaxAcc>(p, lds, L, s, row, rv, vm[0], dd, bot, nacc, d);
                } else {
                    ++d.nglobal;
                    global_row<kMaxAcc>(p, key[0], s != kGlobalNull, row, rv, vm[0], dd, bot, nacc, d);
                }
            }
            slot[0] = slot[1]; slot[1] = slot[2]; slot[2] = slot[3];
            vm[0] = vm[1]; vm[1] = vm[2]; vm[2] = vm[3];
            key[0] = key[1]; key[1] = key[2]; key[2] = key[3];
#pragma unroll
            for (int a = 0; a < kMaxAcc; ++a) {
                v[a][0] = v[a][1];
                v[a][1] = v[a][2];
                v[a][2] = v[a][3];
            }
        }
    }
    flush_and_report<USE_LDS>(p, lds, L, d);
}

// ------------------------------------------------------------- fast path
// Common case: no validity bitmaps, 8-byte key and aggregated columns at
// even offsets of 16-byte aligned buffers, no predicate or `col <cmp> lit`,
// LDS table in use.  Rows [0, n_full) in tiles of 4 rows per thread; the
// tail and every other case go through gb_kernel.  Loads of the next tile
// are issued before the current tile's LDS atomics, so HBM reads overlap
// the aggregation.
// PACK: the key is formed from up to kKpFast packed key columns (KeyPack),
// whose raw words the tile holds until its rows are consumed.
constexpr int kKpFast = 2;
template <int NACC, int ROWS, bool DERIV = false, int PACK = 0, bool NUL = false>
struct FastTile {
    uint64_t key[ROWS];
    uint64_t kr[PACK ? kKpFast : 1][ROWS];
    uint64_t v[NACC > 0 ? NACC : 1][ROWS];
    uint64_t w[DERIV && NACC > 0 ? NACC : 1][ROWS];  // DERIV: second operand columns
    uint64_t pv[ROWS];
    // NUL: null bits of each row pair, row 2q in bits 0-7 and row 2q + 1 in
    // bits 8-15 of nv[q] (the part_nulls layout: bit a acc a, 6 the key, 7
    // the predicate's own column).  fast_nulls leaves the loaded validity
    // words raw in nr[q][column] (column NACC the key, NACC + 1 the
    // predicate's own) and fast_nulls_finish turns them into nv when the
    // tile is consumed: a shift of a loaded word at prefetch time would make
    // the next tile's loads wait for it (one HBM latency per tile).
    uint32_t nv[NUL ? (ROWS + 1) / 2 : 1];
    uint32_t nr[NUL ? (ROWS + 1) / 2 : 1][NUL ? (NACC > 0 ? NACC : 1) + 2 : 1];
};

// Row j of tile t for this thread: pairs of consecutive rows, pair q at
// t*T*ROWS + q*2*T + 2*tid.
__device__ __forceinline__ int64_t fast_row(int64_t t, int T, int rows, int j) {
    return t * (int64_t)T * rows + (int64_t)(j >> 1) * 2 * T + 2 * threadIdx.x + (j & 1);
}

typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));

// 16-byte load; NT: non-temporal (streamed once, not kept in the caches).
template <bool NT>
__device__ __forceinline__ u64x2_t ld16(const uint64_t* p) {
    if (NT) return __builtin_nontemporal_load(reinterpret_cast<const u64x2_t*>(p));
    return *reinterpret_cast<const u64x2_t*>(p);
}

// The rows after the last full tile (fewer than one tile): one more, masked
// tile of guarded single-row loads (rows >= n read as 0 and are not
// selected), so the fused kernel covers every row in one launch.
template <int NACC, int PRED, int ROWS, bool DERIV, int PACK, bool NUL = false>
__device__ __forceinline__ void fast_load_tail(const GbParams& p, int64_t t,
                                               FastTile<NACC, ROWS, DERIV, PACK, NUL>& x) {
    const int T = blockDim.x;
    const uint64_t* kp = (const uint64_t*)p.key.values + p.key.offset;
#pragma unroll
    for (int j = 0; j < ROWS; ++j) {
        const int64_t r = fast_row(t, T, ROWS, j);
        const bool in = r < p.n;
        if (PACK == 2) {
            // String key: kr[0][j] = offset of row r, kr[1][j] = of row r + 1
            const int64_t* o = (const int64_t*)p.kp.c[0].values + p.kp.c[0].offset;
            x.kr[0][j] = in ? (uint64_t)o[r] : 0ull;
            x.kr[1][j] = in ? (uint64_t)o[r + 1] : 0ull;
        } else if (PACK == 1) {
#pragma unroll
            for (int i = 0; i < kKpFast; ++i) x.kr[i][j] = in && i < p.kp.n ? dev_load(p.kp.c[i], r) : 0ull;
        } else {
            x.key[j] = in && p.key.values ? kp[r] : 0ull;
        }
#pragma unroll
        for (int c = 0; c < NACC; ++c) {
            if (!DERIV || p.acc[c].v_from < 0)
                x.v[c][j] = in ? ((const uint64_t*)p.acc[c].c.values + p.acc[c].c.offset)[r] : 0ull;
            if (DERIV && p.acc[c].dop != DOP_NONE && !(p.acc[c].dop & DOP_LIT) && p.acc[c].w_from < 0)
                x.w[c][j] = in ? ((const uint64_t*)p.acc[c].c2.values + p.acc[c].c2.offset)[r] : 0ull;
        }
        if (PRED == 1 && p.pred_acc < 0) x.pv[j] = in ? ((const uint64_t*)p.pred_col.values + p.pred_col.offset)[r] : 0ull;
    }
}

// rbase: first row of tile 0 (even); rmax >= 0: row pairs beyond it are
// clamped to it (the partitioned buffers end a pair after the last row).
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

template <int NACC, int PRED, int ROWS, bool NT, bool DERIV, int PACK, bool NUL = false>
__device__ __forceinline__ void fast_load(const GbParams& p, int64_t t, FastTile<NACC, ROWS, DERIV, PACK, NUL>& x,
                                          int64_t rbase = 0, int64_t rmax = -1) {
    const int T = blockDim.x;
    const uint64_t* kp = (const uint64_t*)p.key.values + p.key.offset;
#pragma unroll
    for (int q = 0; q < ROWS / 2; ++q) {
        int64_t r = rbase + fast_row(t, T, ROWS, 2 * q);
        if (rmax >= 0) r = r < rmax ? r : rmax;
        if (PACK == 2) {
            // String key: the pair's offsets (16 B) and the next row's (8 B):
            // kr[0][j] = start, kr[1][j] = end of row 2q + j
            const int64_t* o = (const int64_t*)p.kp.c[0].values + p.kp.c[0].offset + r;
            const u64x2_t a = ld16<NT>((const uint64_t*)o);
            const uint64_t e = NT ? __builtin_nontemporal_load((const uint64_t*)o + 2) : ((const uint64_t*)o)[2];
            x.kr[0][2 * q] = a.x;
            x.kr[0][2 * q + 1] = a.y;
            x.kr[1][2 * q] = a.y;
            x.kr[1][2 * q + 1] = e;
        } else if (PACK == 1) {
            // each packed key column: one 16-byte (Int64) or 8-byte (Int32 /
            // UInt32) load per row pair, kept raw until the rows are consumed
#pragma unroll
            for (int i = 0; i < kKpFast; ++i) {
                if (i >= p.kp.n) {
                    x.kr[i][2 * q] = x.kr[i][2 * q + 1] = 0;
                    continue;
                }
                const DevCol& kc = p.kp.c[i];
                if (kc.dtype == PLGPU_I64) {
                    const u64x2_t a = ld16<NT>((const uint64_t*)kc.values + kc.offset + r);
                    x.kr[i][2 * q] = a.x;
                    x.kr[i][2 * q + 1] = a.y;
                } else {
                    const u32x2_t* ap = reinterpret_cast<const u32x2_t*>((const uint32_t*)kc.values + kc.offset + r);
                    const u32x2_t a = NT ? __builtin_nontemporal_load(ap) : *ap;
                    x.kr[i][2 * q] = a.x;
                    x.kr[i][2 * q + 1] = a.y;
                }
            }
        } else if (p.key.values) {
            const u64x2_t a = ld16<NT>(kp + r);
            x.key[2 * q] = a.x;
            x.key[2 * q + 1] = a.y;
        } else {
            x.key[2 * q] = x.key[2 * q + 1] = 0;  // keyless: one group
        }
#pragma unroll
        for (int c = 0; c < NACC; ++c) {
            if (!DERIV || p.acc[c].v_from < 0) {
                const uint64_t* vp = (const uint64_t*)p.acc[c].c.values + p.acc[c].c.offset;
                const u64x2_t b = ld16<NT>(vp + r);
                x.v[c][2 * q] = b.x;
                x.v[c][2 * q + 1] = b.y;
            }
            if (DERIV && p.acc[c].dop != DOP_NONE && !(p.acc[c].dop & DOP_LIT) && p.acc[c].w_from < 0) {
                const uint64_t* wp = (const uint64_t*)p.acc[c].c2.values + p.acc[c].c2.offset;
                const u64x2_t w = ld16<NT>(wp + r);
                x.w[c][2 * q] = w.x;
                x.w[c][2 * q + 1] = w.y;
            }
        }
        if (PRED == 1 && p.pred_acc < 0) {
            const uint64_t* pp = (const uint64_t*)p.pred_col.values + p.pred_col.offset;
            const u64x2_t b = ld16<NT>(pp + r);
            x.pv[2 * q] = b.x;
            x.pv[2 * q + 1] = b.y;
        }
    }
}

// Bit position of row r of a column in 32-bit words counted from the
// bitmap's address rounded down to 4 bytes: a word read there never leaves
// the aligned word of a bitmap byte (no page crossing, any byte alignment).
__device__ __forceinline__ uint64_t pair_bit(const DevCol& c, int64_t r) {
    return ((uint64_t)(uintptr_t)c.validity & 3u) * 8u + (uint64_t)(c.offset + r);
}

// The validity word holding rows r, r + 1 of a column (r and the column
// offset even, so both bits sit in one 32-bit word), raw: set = valid; ~0
// without a bitmap.  Its bits are taken at pair_bit & 31 (fast_nulls_finish).
__device__ __forceinline__ uint32_t pair_word(const DevCol& c, int64_t r) {
    if (!c.validity) return ~0u;
    const uint32_t* w = (const uint32_t*)((uintptr_t)c.validity & ~(uintptr_t)3);
    return __builtin_nontemporal_load(w + (pair_bit(c, r) >> 5));
}

// The 32-bit word of a wave's 128-row window (first row rw, a multiple of
// 128; the column offset a multiple of 64) that holds this lane's row pair
// (rows rw + 2 lane, + 1): 16 lanes share each of the window's four words,
// one request per wave.  The pair's bits are at (2 lane) & 31.
__device__ __forceinline__ uint32_t pair_word_wave(const DevCol& c, int64_t rw) {
    if (!c.validity) return ~0u;
    const int lane = threadIdx.x & 63;
    const uint64_t b = (uint64_t)(c.offset + rw) + 2u * (uint32_t)lane;
    return __builtin_nontemporal_load((const uint32_t*)c.validity + (b >> 5));
}

// NUL: the tile's validity words (FastTile::nr), from the columns' bitmaps
// (whole words per wave when p.vwords, else the word of each pair) or, over
// the partition buffers (PART), part_nulls (two bytes per pair, already in
// nv's layout).  Rows past n (the masked tail tile) read nothing.  Issued
// before the tile's value loads; nothing here waits for them.  (p.vwords:
// 8-byte aligned bitmaps at offsets that are multiples of 64, so the
// wave-window word and pair_bit agree.)
template <int NACC, int PRED, int ROWS, bool PART, bool DERIV, int PACK, bool NUL>
__device__ __forceinline__ void fast_nulls(const GbParams& p, int64_t t, FastTile<NACC, ROWS, DERIV, PACK, NUL>& x,
                                           int64_t rbase, int64_t rmax, bool full) {
    if constexpr (NUL) {
        const int T = blockDim.x;
#pragma unroll
        for (int q = 0; q < ROWS / 2; ++q) {
            int64_t r = rbase + fast_row(t, T, ROWS, 2 * q);
            if (rmax >= 0) r = r < rmax ? r : rmax;
            if (PART) {
                x.nr[q][0] = p.part_nulls ? __builtin_nontemporal_load((const uint16_t*)(p.part_nulls + r)) : 0u;
            } else if (full && p.vwords) {
                // a full tile: the wave's 128 rows end at or below n_full, a
                // multiple of 1024, so the words lie inside the bitmap
                const int64_t rw = r - 2 * (threadIdx.x & 63);
#pragma unroll
                for (int c = 0; c < NACC; ++c) x.nr[q][c] = pair_word_wave(p.acc[c].c, rw);
                x.nr[q][NACC] = pair_word_wave(p.key, rw);
                x.nr[q][NACC + 1] = PRED == 1 && p.pred_acc < 0 ? pair_word_wave(p.pred_col, rw) : ~0u;
            } else if (r < p.n) {
#pragma unroll
                for (int c = 0; c < NACC; ++c) x.nr[q][c] = pair_word(p.acc[c].c, r);
                x.nr[q][NACC] = pair_word(p.key, r);
                x.nr[q][NACC + 1] = PRED == 1 && p.pred_acc < 0 ? pair_word(p.pred_col, r) : ~0u;
            } else {
#pragma unroll
                for (int c = 0; c < NACC + 2; ++c) x.nr[q][c] = ~0u;
            }
        }
    }
}

// NUL: the raw words of fast_nulls as FastTile::nv, once the tile's loads
// have landed.  A pair's bits sit at pair_bit & 31 of its word (with
// p.vwords that is (2 lane) & 31).
template <int NACC, int PRED, int ROWS, bool PART, bool DERIV, int PACK, bool NUL>
__device__ __forceinline__ void fast_nulls_finish(const GbParams& p, int64_t t,
                                                  FastTile<NACC, ROWS, DERIV, PACK, NUL>& x, int64_t rbase,
                                                  int64_t rmax) {
    if constexpr (NUL) {
        const int T = blockDim.x;
#pragma unroll
        for (int q = 0; q < ROWS / 2; ++q) {
            if (PART) {
                x.nv[q] = x.nr[q][0];
                continue;
            }
            int64_t r = rbase + fast_row(t, T, ROWS, 2 * q);
            if (rmax >= 0) r = r < rmax ? r : rmax;
            auto bits = [&](const DevCol& c, uint32_t w) -> uint32_t {
                return ~(w >> ((uint32_t)pair_bit(c, r) & 31u)) & 3u;
            };
            uint32_t m = 0;
#pragma unroll
            for (int c = 0; c < NACC; ++c) {
                const uint32_t b = bits(p.acc[c].c, x.nr[q][c]);
                m |= ((b & 1u) << c) | ((b >> 1) << (8 + c));
            }
            const uint32_t bk = bits(p.key, x.nr[q][NACC]);
            m |= ((bk & 1u) << 6) | ((bk >> 1) << 14);
            if (PRED == 1) {
                const uint32_t bp = bits(p.pred_col, x.nr[q][NACC + 1]);
                m |= ((bp & 1u) << 7) | ((bp >> 1) << 15);
            }
            x.nv[q] = m;
        }
    }
}

// DERIV: fill the operand registers whose column another acc loaded
// (v_from / w_from, uniform), once the tile's loads are being consumed --
// not at prefetch time, where the copy would wait for the loads.
template <int NACC, int ROWS, bool DERIV, int PACK, bool NUL = false>
__device__ __forceinline__ void fast_share(const int32_t (&vf)[NACC > 0 ? NACC : 1],
                                           const int32_t (&wf)[NACC > 0 ? NACC : 1],
                                           FastTile<NACC, ROWS, DERIV, PACK, NUL>& x) {
    if (!DERIV) return;
#pragma unroll
    for (int c = 0; c < NACC; ++c)
#pragma unroll
        for (int b = 0; b < NACC; ++b)
#pragma unroll
            for (int j = 0; j < ROWS; ++j) {
                if (b == vf[c]) x.v[c][j] = x.v[b][j];
                if (b == wf[c]) x.w[c][j] = x.v[b][j];
            }
}

// SUMONLY: every acc is an f64 sum / mean (flags A_FSUM|A_FLAGS, no count /
// min / max), no maintain_order: the field layout is compile-time
// (key 0, len 1, acc a: limbs 2+4a..4+4a, flags 5+4a) and the per-acc code
// is unrolled with no descriptor decode.
// LIMBS (SUMONLY only): 3 = the full 120-bit window; 2 = its top 80 bits
// (bottom + 40), chosen by the plan when the sampled exponents span few
// binades.  A value with bits below the 2-limb window sets the inexact flag
// and the host reruns with 3 limbs, so results never depend on the choice.
// The two limbs land in fields (3+4a, 4+4a): the 3-limb representation with
// a zero low limb, so the flush and finalize are unchanged.
// RUNS (sum-only, 2 limbs): per-lane register accumulators for sorted /
// clustered keys (below).
// PART: the workgroups aggregate the partition buffers of the many-groups
// path (gb_partition): workgroup b takes its share of partition
// b / part_blocks (rows [part_range[q], part_range[q + 1]), already
// selected, so PRED is 0) with an LDS table of lcap slots for that
// partition's groups.
// Without PART the launch covers every row: the full tiles, then the rows
// after the last full tile as one masked tile (fast_load_tail).
// (Measured and removed variants -- no prefetch, default-policy loads,
// 80-VGPR caps, 4 rows per thread -- are logged in DESIGN.md.)
// DERIV: some accs are derived inputs (x op y, AccSpec.dop), computed in
// registers from the loaded operand columns as each row is applied.
// PACK: the key is the fused packed code of p.kp's (at most kKpFast) key
// columns (KeyPack), formed as each tile's rows are consumed.
// (PART without register runs: up to kGbPartThreads per workgroup -- with
// one workgroup per partition and LDS table, more waves share the table;
// the register-run variant keeps kGbThreads, its registers would spill)
constexpr int kGbPartThreads = 1024;
// NULLS: key, aggregated and predicate columns may carry validity bitmaps
// (or, with PART, the partition buffers' part_nulls bytes): a null
// aggregated value takes no part in its acc (a sum adds nothing, counts /
// min / max skip it), a null key row joins the null group (LDS slot lcap ->
// global slot gcap), a null predicate value drops the row.  Bits travel
// with each tile (FastTile::nv: one byte per row pair and column read).
template <int NACC, int PRED, bool SUMONLY, int ROWS, int LIMBS = 3, bool RUNS = false, bool PART = false,
          bool DERIV = false, int VAR = 0, int PACK = 0, bool NULLS = false>
__global__ __launch_bounds__(PART && !RUNS && ROWS == 2 ? kGbPartThreads : kGbThreads) void gb_fast_kernel(GbParams p,
                                                                                               DevProgram prog) {
    static_assert(!PACK || !PART, "PACK: the single-table kernel");
    static_assert(!NULLS || (!RUNS && !DERIV && (VAR == 0 || VAR == 5) && PACK == 0), "NULLS: plain inputs");
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    constexpr int NA = NACC > 0 ? NACC : 1;
    // VAR 1 (sum-only, NACC 3): the fused variance's three sums of one column
    // x -- x, h = x * x and l = fma(x, x, -h) -- with h and l computed from
    // x's registers: one column loaded, no operand registers per acc.
    // VAR 2 / 3 (NACC 2): a product and one of its operands ((close *
    // volume).sum() next to volume.sum()): the tile loads acc 0's and acc
    // 1's columns as plain sums do, acc VAR - 2 sums v[0] * v[1] (the host
    // puts the product's other operand in its column, pair_normalize), with
    // none of the general derived path's operand registers or op switch
    // VAR 4: the triple with x >= 0 (or NaN) on every selected row -- the
    // fused predicate x > c (or >=) with c >= 0 on x's column -- so x's limbs
    // need no sign either (launch_fast_var)
    constexpr bool TRIPLE = VAR == 1 || VAR == 4;
    static_assert(!TRIPLE || (NACC == 3 && !DERIV), "VAR 1 / 4: three sums of one column");
    static_assert((VAR != 2 && VAR != 3) || (NACC == 2 && !DERIV), "VAR 2 / 3: a product and its operand");
    // VAR 5 (sum-only, plain inputs): the last acc's column is the fused
    // predicate's and keeps no value below a literal >= 0, so its limbs need
    // no sign (the headline's close.sum() under close > 250)
    static_assert(VAR != 5 || (SUMONLY && !DERIV && NACC > 0), "VAR 5: plain sums");
    constexpr int NL = TRIPLE ? 1 : NACC;  // accs whose column the tile loads
    // SLIM (sum-only, 2 limbs): fields key 0, len 1, acc a: limbs 2+3a,
    // 3+3a, flags 4+3a (the unused low limb of the 3-limb layout is not
    // stored, so more workgroups fit per CU).  The keys are one array (the
    // probes scan it); a slot's other fields are adjacent (slot-major,
    // slim_vwords per slot), so a row's atomics share one address register
    // and take immediate offsets.  Other layouts: field-major, field f of
    // slot s at f * L + s.
    constexpr bool SLIM = SUMONLY && LIMBS == 2;
    constexpr int FV = slim_vwords(NACC);
    auto so_mid = [](int a) { return SLIM ? 2 + 3 * a : 3 + 4 * a; };
    auto so_top = [](int a) { return SLIM ? 3 + 3 * a : 4 + 4 * a; };
    auto so_flags = [](int a) { return SLIM ? 4 + 3 * a : 5 + 4 * a; };
    const int L = p.lcap + 2;
    // field f (>= 1) of slot s
    auto fld = [&](int s_, int f) -> unsigned long long* {
        return (unsigned long long*)(SLIM ? &lds[L + s_ * FV + (f - 1)] : &lds[f * L + s_]);
    };
    if (SLIM) {
        for (int i = threadIdx.x; i < L; i += blockDim.x) lds[i] = kEmptyKey;
        for (int i = threadIdx.x; i < L * FV; i += blockDim.x) lds[L + i] = 0ull;
    } else {
        init_lds(p, lds, L);
    }
    ThreadDiag d = {0u, 0u, 0u, 0u, 0u};
    uint64_t dd0[NA];
    int bot0[NA];
    load_descs(p, dd0, bot0);
    int32_t dop0[NA], vf0[NA], wf0[NA];
    uint64_t dim0[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        dop0[a] = DERIV && a < NACC ? p.acc[a].dop : DOP_NONE;
        dim0[a] = DERIV && a < NACC ? p.acc[a].dimm : 0ull;
        vf0[a] = DERIV && a < NACC ? p.acc[a].v_from : -1;
        wf0[a] = DERIV && a < NACC ? p.acc[a].w_from : -1;
    }
    __syncthreads();

    const int T = blockDim.x;
    // the tile stream is read once: non-temporal loads (6.60 vs 6.84 ms at
    // 1e9 rows with default-policy loads, tools/ablate.py)
    int64_t ntiles = p.n_full / ((int64_t)T * ROWS);
    int64_t nall = ntiles + (p.n > p.n_full ? 1 : 0);  // + the masked tail tile
    int64_t t = blockIdx.x, tstep = gridDim.x;
    int64_t rbase = 0, rlo = 0, rhi = 0, rmax = -1;
    if (!PART && p.tiles_per_wg > 0) {
        // range-local mode: one contiguous run of tiles per workgroup, so
        // its LDS table holds only the keys of that row range
        t = (int64_t)blockIdx.x * p.tiles_per_wg;
        nall = std::min<int64_t>(nall, t + p.tiles_per_wg);
        tstep = 1;
    }
    if (PART) {
        const int q = blockIdx.x / p.part_blocks;
        rlo = (int64_t)p.part_range[q];
        rhi = (int64_t)p.part_range[q + 1];
        rbase = rlo & ~int64_t(1);
        rmax = p.n & ~int64_t(1);
        ntiles = (rhi - rbase + (int64_t)T * ROWS - 1) / ((int64_t)T * ROWS);
        nall = ntiles;
        t = blockIdx.x % p.part_blocks;
        tstep = p.part_blocks;
    }
    auto load_tile = [&](int64_t tt, FastTile<NL, ROWS, DERIV, PACK, NULLS>& x) {
        fast_nulls<NL, PRED, ROWS, PART, DERIV, PACK, NULLS>(p, tt, x, rbase, rmax, tt < ntiles);
        if (PART || tt < ntiles) fast_load<NL, PRED, ROWS, true, DERIV, PACK, NULLS>(p, tt, x, rbase, rmax);
        else fast_load_tail<NL, PRED, ROWS, DERIV, PACK, NULLS>(p, tt, x);
    };
    // NULLS: the null bit of the predicate's column (its acc's, or its own)
    const int pbit = p.pred_acc >= 0 ? p.pred_acc : 7;
    // PACK: the plan's fields as uniform constants, hoisted.  Field i of a
    // raw word w: an 8-byte column's w - base (mode 0); a 4-byte column's
    // (w ^ x32) - b32 on 32 bits (mode 1), or widened, ((w & kpm) ^ kpx) -
    // kpc with kpx = 2^31 sign-extending an Int32 and kpc = kpx + base (mode
    // 2).  It fits iff it is <= its span (KeyPack::span / span32).
    uint64_t kpm[kKpFast], kpx[kKpFast], kpc[kKpFast];
    int32_t kpsh[kKpFast];
#pragma unroll
    for (int i = 0; i < kKpFast; ++i) {
        const bool on = PACK && i < p.kp.n;
        const int32_t dt = on ? p.kp.c[i].dtype : PLGPU_I64;
        kpm[i] = (dt == PLGPU_I32 || dt == PLGPU_U32) ? 0xFFFFFFFFull : ~0ull;
        kpx[i] = dt == PLGPU_I32 ? 0x80000000ull : 0ull;
        kpc[i] = kpx[i] + (on ? p.kp.base[i] : 0ull);
        kpsh[i] = on ? p.kp.shift[i] : 0;
    }
    // identity plan: one non-String key, base 0, 64 bits (gb_multi_impl's
    // narrow single key)
    const bool kpid = PACK == 1 && p.kp.n == 1 && p.kp.bits[0] >= 64 && p.kp.base[0] == 0 &&
                      p.kp.shift[0] == 0;
    constexpr uint32_t VM = (1u << NACC) - 1u;
    // RACC (partition buffers, sum-only, 2 limbs): each lane keeps KR
    // register accumulators {slot, len, limbs} and adds a row whose group
    // it already holds there instead of in LDS.  Time-ordered keys put only
    // a few groups into a wave at a time, whose same-address LDS atomics
    // serialise (bank-conflict ratio 0.92 measured).  RUNS: the same with
    // one accumulator in the single-table kernel, chosen by the plan for
    // sorted / clustered keys (a frame sorted by symbol gives every lane
    // long runs of one group).
    // (partition buffers: only for clustered / sorted keys, RUNS; random keys
    // would evict on nearly every row)
    constexpr bool RACC = SUMONLY && LIMBS == 2 && RUNS;
    constexpr int KR = RACC ? (PART ? 4 : 1) : 1;
    int rs[KR];
    uint64_t rn[KR], rlo_[KR][NA], rhi_[KR][NA];
#pragma unroll
    for (int k = 0; k < KR; ++k) {
        rs[k] = -1;
        rn[k] = 0;
#pragma unroll
        for (int a = 0; a < NA; ++a) rlo_[k][a] = rhi_[k][a] = 0;
    }
    int rvict = 0;
    auto racc_flush = [&](int k) {
        if (rs[k] < 0) return;
        atomicAdd(fld(rs[k], 1), (unsigned long long)rn[k]);
#pragma unroll
        for (int a = 0; a < NACC; ++a) {
            atomicAdd(fld(rs[k], so_mid(a)), (unsigned long long)rlo_[k][a]);
            atomicAdd(fld(rs[k], so_top(a)), (unsigned long long)rhi_[k][a]);
        }
        rs[k] = -1;
    };
    // GRUNS (RUNS without SUMONLY: min / max / count / first / last next to
    // the sums, sorted / clustered keys): one register run per lane holding
    // the state of the group of LDS slot gs -- len, first / last row, per
    // acc two registers r0 / r1 (an f64 sum's top two limbs of the window,
    // LIMBS == 2; an integer sum in r0) and min / max as ordered bits --
    // folded into the LDS table when the lane meets another group.  A value
    // below the 2-limb window, inf / NaN flags and (rare) an integer column
    // summed both as integers and as f64 go straight to the LDS fields.
    // The plan picks this variant only when its sampled exponents fit the
    // 2-limb window and no acc casts integers to f64 sums.
    constexpr bool GRUNS = RUNS && !SUMONLY;
    constexpr int NG = GRUNS ? NA : 1;
    int gs = -1;
    uint64_t gn = 0, gfirst = 0, glast = 0;
    uint64_t gr0[NG], gr1[NG], gmin[NG], gmax[NG];
    auto grun_flush = [&]() {
        if (!GRUNS || gs < 0) return;
        unsigned long long* q = (unsigned long long*)&lds[gs];
        atomicAdd(q + p.f_len * L, (unsigned long long)gn);
        if (p.f_first >= 0) atomicMin(q + p.f_first * L, (unsigned long long)gfirst);
        if (p.f_last >= 0) atomicMax(q + p.f_last * L, (unsigned long long)glast);
#pragma unroll
        for (int a = 0; a < NG && a < NACC; ++a) {
            const uint64_t dsc = dd0[a];
            const uint32_t flags = (uint32_t)dsc & 0xFF;
            const int f_cnt = dfield(dsc, 24);
            if (f_cnt != kNoField) atomicAdd(q + f_cnt * L, (unsigned long long)gn);
            const bool isf = (dsc >> 56) & 1;
            if (isf && (flags & A_FSUM)) {
                // the top two limbs: 3-limb fields (f + 1, f + 2), low limb 0
                const int f = dfield(dsc, 8);
                if (gr0[a]) atomicAdd(q + (f + 1) * L, (unsigned long long)gr0[a]);
                if (gr1[a]) atomicAdd(q + (f + 2) * L, (unsigned long long)gr1[a]);
            } else if (!isf && (flags & A_ISUM) && gr0[a]) {
                atomicAdd(q + dfield(dsc, 16) * L, (unsigned long long)gr0[a]);
            }
            if (flags & A_MIN) atomicMin(q + dfield(dsc, 32) * L, (unsigned long long)gmin[a]);
            if (flags & A_MAX) atomicMax(q + dfield(dsc, 40) * L, (unsigned long long)gmax[a]);
        }
        gs = -1;
    };
    auto grun_take = [&](int sl, int64_t r, const uint64_t (&x)[NA]) -> bool {
        if (!GRUNS) return false;
        if (gs != sl) {
            grun_flush();
            gs = sl;
            gn = 0;
            gfirst = glast = (uint64_t)r;
#pragma unroll
            for (int a = 0; a < NG; ++a) {
                gr0[a] = gr1[a] = gmax[a] = 0;
                gmin[a] = ~0ull;
            }
        }
        ++gn;
        gfirst = std::min<uint64_t>(gfirst, (uint64_t)r);
        glast = std::max<uint64_t>(glast, (uint64_t)r);
        unsigned long long* q = (unsigned long long*)&lds[sl];
#pragma unroll
        for (int a = 0; a < NG && a < NACC; ++a) {
            const uint64_t dsc = dd0[a];
            const uint32_t flags = (uint32_t)dsc & 0xFF;
            const bool isf = (dsc >> 56) & 1;
            const bool uns = (dsc >> 57) & 1;
            const uint64_t ab = x[a] & 0x7fffffffffffffffull;
            if (isf && ab >= 0x7ff0000000000000ull) {
                // inf / NaN: the flags word (every f64 acc has one)
                atomicOr(q + dfield(dsc, 48) * L, (unsigned long long)(ab > 0x7ff0000000000000ull ? FL_NAN
                                                                     : ((x[a] >> 63) ? FL_NINF : FL_PINF)));
            } else if (isf && (flags & A_FSUM)) {
                uint64_t l0, l1, l2;
                if (fx_limbs_fast<2>(x[a], bot0[a], l0, l1, l2)) {
                    gr0[a] += l0;
                    gr1[a] += l1;
                } else {
                    // below the 2-limb window (or out of the top): exact
                    // conversion straight into the three LDS limb fields
                    uint32_t ex = 0, fl = 0;
                    const bool ok = fx_limbs(x[a], bot0[a], l0, l1, l2, fl, ex);
                    d.fxbits |= fl << (2 * a);
                    if (ok) {
                        const int f = dfield(dsc, 8);
                        atomicAdd(q + f * L, (unsigned long long)l0);
                        atomicAdd(q + (f + 1) * L, (unsigned long long)l1);
                        atomicAdd(q + (f + 2) * L, (unsigned long long)l2);
                    }
                }
            } else if (!isf && (flags & A_ISUM)) {
                gr0[a] += x[a];
            }
            if (!(isf && ab > 0x7ff0000000000000ull)) {  // NaN takes no part in min / max
                const uint64_t o = isf ? ord_f64(x[a]) : (uns ? x[a] : ord_i64(x[a]));
                gmin[a] = std::min(gmin[a], o);
                gmax[a] = std::max(gmax[a], o);
            }
        }
        return true;
    };
    FastTile<NL, ROWS, DERIV, PACK, NULLS> cur;
    if (t < nall) load_tile(t, cur);
    for (; t < nall; t += tstep) {
        if constexpr (!VAR) fast_share<NACC, ROWS, DERIV, PACK, NULLS>(vf0, wf0, cur);
        fast_nulls_finish<NL, PRED, ROWS, PART, DERIV, PACK, NULLS>(p, t, cur, rbase, rmax);
        bool kout[ROWS];
        constexpr bool kstr = PACK == 2;
        if (kstr) {
            // String key: each row's short-string code from its offsets and
            // one or two data words (dependent loads, issued for the tile's
            // rows together)
#pragma unroll
            for (int j = 0; j < ROWS; ++j) {
                kout[j] = false;
                cur.key[j] = kp_str_code(p.kp.c[0].data, p.kp.data_end, cur.kr[0][j], cur.kr[1][j] - cur.kr[0][j],
                                         kout[j]);
            }
        }
        if (PACK == 1 && kpid) {
            // one 4-byte (or 8-byte) key as itself: its sign- or zero-extended
            // value is the code (no range to check)
#pragma unroll
            for (int j = 0; j < ROWS; ++j) {
                kout[j] = false;
                cur.key[j] = ((cur.kr[0][j] & kpm[0]) ^ kpx[0]) - kpx[0];
            }
        }
#pragma unroll
        for (int j = 0; j < ROWS; ++j) {
            if (!kstr) kout[j] = false;
        }
        if (PACK == 1 && !kpid) {
            // the packed codes (mk_plan_pack's layout), field by field; each
            // field's form is uniform, so one branch per field and tile
#pragma unroll
            for (int j = 0; j < ROWS; ++j) cur.key[j] = 0;
#pragma unroll
            for (int i = 0; i < kKpFast; ++i) {
                if (i >= p.kp.n) continue;
                const int md = p.kp.mode[i];
                if (md == 0) {
#pragma unroll
                    for (int j = 0; j < ROWS; ++j) {
                        const uint64_t f = cur.kr[i][j] - kpc[i];
                        kout[j] |= f > p.kp.span[i];
                        cur.key[j] |= f << kpsh[i];
                    }
                } else if (md == 1) {
#pragma unroll
                    for (int j = 0; j < ROWS; ++j) {
                        const uint32_t f = ((uint32_t)cur.kr[i][j] ^ p.kp.x32[i]) - p.kp.b32[i];
                        kout[j] |= f > p.kp.span32[i];
                        cur.key[j] |= (uint64_t)f << kpsh[i];
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < ROWS; ++j) {
                        const uint64_t f = ((cur.kr[i][j] & kpm[i]) ^ kpx[i]) - kpc[i];
                        kout[j] |= f > p.kp.span[i];
                        cur.key[j] |= f << kpsh[i];
                    }
                }
            }
        }
        // ---- predicate + batched LDS probes of the tile's rows
        int slot[ROWS];
        uint64_t probe[ROWS];
        uint32_t h[ROWS];
        uint32_t nrw[ROWS];  // NULLS: the row's null bits
#pragma unroll
        for (int j = 0; j < ROWS; ++j) {
            nrw[j] = NULLS ? (cur.nv[j >> 1] >> (8 * (j & 1))) & 0xFFu : 0u;
            bool sel = true;
            if (PRED == 1) {
                uint64_t x = cur.pv[j];
                if (TRIPLE) {
                    if (p.pred_acc >= 0) x = cur.v[0][j];  // every acc reads x's column
                } else {
#pragma unroll
                    for (int a = 0; a < NACC; ++a)
                        if (a == p.pred_acc) x = cur.v[a][j];
                }
                sel = simple_pred(prog.simple_isf, prog.simple_op, x, prog.simple_imm);
                if (NULLS) sel = sel && !((nrw[j] >> pbit) & 1u);
            }
            if (PART) {
                const int64_t r = rbase + fast_row(t, T, ROWS, j);
                sel = r >= rlo && r < rhi;
            } else if (t >= ntiles) {
                sel = sel && fast_row(t, T, ROWS, j) < p.n;
            }
            if (PACK && sel && kout[j]) d.kbad = 1u;
            const bool knull = (NULLS && ((nrw[j] >> 6) & 1u)) ||
                               (PART && p.has_null_key && cur.key[j] == (uint64_t)p.null_key);
            slot[j] = sel ? (knull ? p.lcap : (cur.key[j] == kEmptyKey ? p.lcap + 1 : kGlobalKey)) : kNotSelected;
            h[j] = hash_slot(cur.key[j], p.lbits);
            probe[j] = lds_load(&lds[h[j]]);
        }
#pragma unroll
        for (int j = 0; j < ROWS; ++j)
            if (slot[j] == kGlobalKey && probe[j] == cur.key[j]) slot[j] = (int)h[j];
        // ---- next tile's loads go out before this tile's atomics
        FastTile<NL, ROWS, DERIV, PACK, NULLS> nxt;
        const int64_t tn = t + tstep;
        if (tn < nall) load_tile(tn, nxt);
        // ---- apply rows one at a time (rolled; arrays shift statically)
#pragma unroll 1
        for (int j = 0; j < ROWS; ++j) {
            const int64_t r = rbase + fast_row(t, T, ROWS, j);
            int s = slot[0];
            if (s != kNotSelected) {
                ++d.nsel;
                uint64_t rv[NA], dd[NA];
                int bot[NA];
#pragma unroll
                for (int a = 0; a < NA; ++a) {
                    if (TRIPLE) {
                        rv[a] = a == 0 ? cur.v[0][0] : derive(a == 1 ? DOP_SQHI : DOP_SQLO, cur.v[0][0], 0ull);
                    } else if (VAR == 2 || VAR == 3) {
                        rv[a] = a == VAR - 2 ? f64_bits(as_f64(cur.v[0][0]) * as_f64(cur.v[1][0])) : cur.v[a][0];
                    } else {
                        rv[a] = cur.v[a][0];
                        if (DERIV && dop0[a] != DOP_NONE)
                            rv[a] = derive(dop0[a], cur.v[a][0], (dop0[a] & DOP_LIT) ? dim0[a] : cur.w[a][0]);
                    }
                    dd[a] = dd0[a];
                    bot[a] = bot0[a];
                    // a null value adds nothing to a sum-only layout's sums
                    if (NULLS && SUMONLY && ((nrw[0] >> a) & 1u)) rv[a] = 0ull;
                }
                const uint32_t vm = NULLS ? VM & ~nrw[0] : VM;
                if (s == kGlobalKey) s = lds_find(lds, p.lbits, p.lcap, cur.key[0]);
                if (s >= 0 && !gb_ok(s < L, CK_FAST_SLOT)) s = -1;
                bool held = false;
                if (RACC && s >= 0) {
                    uint64_t lo[NA], hi[NA];
                    bool ok = true;
#pragma unroll
                    for (int a = 0; a < NACC; ++a) {
                        uint64_t l0, l1, l2;
                        ok = fx_limbs_fast<LIMBS>(rv[a], bot[a], l0, l1, l2) && ok;
                        lo[a] = l0;
                        hi[a] = l1;
                    }
                    if (ok) {
                        // fully in-window row: into the lane's accumulator
                        // for slot s (evicting one round-robin if none holds it)
                        int k = -1;
#pragma unroll
                        for (int i = 0; i < KR; ++i)
                            if (rs[i] == s) k = i;
                        if (k < 0) {
#pragma unroll
                            for (int i = 0; i < KR; ++i)
                                if (k < 0 && rs[i] < 0) k = i;
                        }
                        if (k < 0) {
                            k = rvict;
                            rvict = (rvict + 1) % KR;
#pragma unroll
                            for (int i = 0; i < KR; ++i)
                                if (i == k) racc_flush(i);
                        }
#pragma unroll
                        for (int i = 0; i < KR; ++i) {
                            if (i != k) continue;
                            if (rs[i] < 0) {
                                rs[i] = s;
                                rn[i] = 0;
#pragma unroll
                                for (int a = 0; a < NA; ++a) rlo_[i][a] = rhi_[i][a] = 0;
                            }
                            rn[i] += 1;
#pragma unroll
                            for (int a = 0; a < NACC; ++a) {
                                rlo_[i][a] += lo[a];
                                rhi_[i][a] += hi[a];
                            }
                        }
                        held = true;
                    }
                }
                if (held) {
                } else if (SUMONLY && s >= 0) {
                    atomicAdd(fld(s, 1), 1ull);
                    uint32_t slow = 0;
                    uint64_t fl0[NA], fl1[NA], fl2[NA];
#pragma unroll
                    for (int a = 0; a < NACC; ++a) {
                        const bool ok = fx_limbs_fast<LIMBS>(rv[a], bot[a], fl0[a], fl1[a], fl2[a],
                                                                  (TRIPLE && (a == 1 || (VAR == 4 && a == 0))) ||
                                                                      (VAR == 5 && a == NACC - 1));
                        slow |= (ok ? 0u : 1u) << a;
                    }
                    // the limbs of a slow value are not added here (2 limbs:
                    // they are unspecified; 3 limbs: zero); the common row
                    // has none and takes the unmasked block
                    auto add_limbs = [&](int a) {
                        if (LIMBS == 3) atomicAdd(fld(s, 2 + 4 * a), (unsigned long long)fl0[a]);
                        atomicAdd(fld(s, so_mid(a)), (unsigned long long)(LIMBS == 3 ? fl1[a] : fl0[a]));
                        atomicAdd(fld(s, so_top(a)), (unsigned long long)(LIMBS == 3 ? fl2[a] : fl1[a]));
                    };
                    if (LIMBS == 3 || slow == 0) {
#pragma unroll
                        for (int a = 0; a < NACC; ++a) add_limbs(a);
                    } else {
#pragma unroll
                        for (int a = 0; a < NACC; ++a)
                            if (!((slow >> a) & 1u)) add_limbs(a);
                    }
                    if (slow) {
                        // inf / NaN flags, rounding below the window, overflow
#pragma unroll
                        for (int a = 0; a < NACC; ++a) {
                            if (!((slow >> a) & 1u)) continue;
                            const uint64_t x = rv[a];
                            const uint64_t ab = x & 0x7fffffffffffffffull;
                            if (ab >= 0x7ff0000000000000ull) {
                                atomicOr(fld(s, so_flags(a)),
                                         (unsigned long long)(ab > 0x7ff0000000000000ull ? FL_NAN
                                                              : ((x >> 63) ? FL_NINF : FL_PINF)));
                            } else {
                                uint64_t l0, l1, l2;
                                uint32_t ex = 0, fl = 0;
                                const bool ok = LIMBS == 3
                                                    ? fx_limbs<kSumWindowBits>(x, bot[a], l0, l1, l2, fl, ex)
                                                    : fx_limbs<kSumWindowBits - 40>(x, bot[a] + 40, l0, l1, l2, fl,
                                                                                    ex);
                                d.fxbits |= fl << (2 * a);
                                if (ok) {
                                    if (LIMBS == 3) atomicAdd(fld(s, 2 + 4 * a), (unsigned long long)l0);
                                    atomicAdd(fld(s, so_mid(a)), (unsigned long long)(LIMBS == 3 ? l1 : l0));
                                    atomicAdd(fld(s, so_top(a)), (unsigned long long)(LIMBS == 3 ? l2 : l1));
                                }
                            }
                        }
                    }
                } else if (s >= 0) {
                    if (!grun_take(s, r, rv)) apply_row<true, NA>(p, lds, L, s, r, rv, vm, dd, bot, NACC, d);
                } else {
                    ++d.nglobal;
                    global_row<NA>(p, cur.key[0], true, r, rv, vm, dd, bot, NACC, d);
                }
            }
#pragma unroll
            for (int i = 0; i + 1 < ROWS; ++i) {
                slot[i] = slot[i + 1];
                nrw[i] = nrw[i + 1];
                cur.key[i] = cur.key[i + 1];
#pragma unroll
                for (int a = 0; a < NL; ++a) {
                    cur.v[a][i] = cur.v[a][i + 1];
                    if (DERIV) cur.w[a][i] = cur.w[a][i + 1];
                }
            }
        }
        cur = nxt;
    }
    if (RACC) {
#pragma unroll
        for (int k = 0; k < KR; ++k) racc_flush(k);
    }
    if (SLIM) {
        __syncthreads();
        // kWgScratch bytes after the slim table (every slim launch sizes the
        // dynamic LDS with them; no static LDS, so the kernel's dynamic limit
        // stays the full 160 KiB)
        uint32_t* wsc = (uint32_t*)&lds[(size_t)L * slim_words(NACC)];
        // LDS slot sl's state: plain stores into its own slot t, or added
        // into a shared slot gs
        // (tab, stride: the hashed table, or the compact region table)
        auto store_slot = [&](int sl, uint64_t* tab, int64_t stride, int64_t t, uint64_t len) {
            tab[(int64_t)p.f_len * stride + t] = len;
#pragma unroll
            for (int a = 0; a < NACC; ++a) {
                const int f = p.acc[a].f_sum;
                uint64_t w0, w1, w2;
                limbs_to_192(0, (int64_t)*fld(sl, so_mid(a)), (int64_t)*fld(sl, so_top(a)), w0, w1, w2);
                tab[(int64_t)f * stride + t] = w0;
                tab[(int64_t)(f + 1) * stride + t] = w1;
                tab[(int64_t)(f + 2) * stride + t] = w2;
                tab[(int64_t)p.acc[a].f_flags * stride + t] = *fld(sl, so_flags(a));
            }
        };
        auto add_slot = [&](int sl, int64_t gs, uint64_t len) {
            atomicAdd((unsigned long long*)gfield(p, p.f_len, gs), (unsigned long long)len);
#pragma unroll
            for (int a = 0; a < NACC; ++a) {
                const int f = p.acc[a].f_sum;
                uint64_t w0, w1, w2;
                limbs_to_192(0, (int64_t)*fld(sl, so_mid(a)), (int64_t)*fld(sl, so_top(a)), w0, w1, w2);
                g_add192(gfield(p, f, gs), gfield(p, f + 1, gs), gfield(p, f + 2, gs), w0, w1, w2);
                const uint64_t fl = *fld(sl, so_flags(a));
                if (fl) atomicOr((unsigned long long*)gfield(p, p.acc[a].f_flags, gs), (unsigned long long)fl);
            }
        };
        if (PART && p.region_cnt) {
            // compact regions: the live slots ranked in slot order (wave
            // ballots + the waves' counts), written densely from the
            // region's first slot; the two special groups add into the
            // table's shared special slots
            uint32_t* wcnt = wsc;  // the waves' counts
            const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
            const int64_t t0 = (int64_t)(blockIdx.x / p.part_blocks) << p.lbits;
            uint32_t run = 0;
            for (int s0 = 0; s0 < L; s0 += blockDim.x) {
                const int sl = s0 + threadIdx.x;
                const uint64_t len = sl < L ? *fld(sl, 1) : 0ull;
                const bool live = len != 0 && sl < p.lcap;
                const uint64_t bl = __ballot(live);
                if (lane == 0) wcnt[wid] = (uint32_t)__popcll(bl);
                __syncthreads();
                uint32_t before = 0, tot = 0;
                for (int w = 0; w < nw; ++w) {
                    before += w < wid ? wcnt[w] : 0u;
                    tot += wcnt[w];
                }
                __syncthreads();
                if (live) {
                    const uint32_t idx = run + before + (uint32_t)__popcll(bl & ((1ull << lane) - 1ull));
                    ++d.newkeys;
                    if (gb_ok(idx < (uint32_t)p.lcap && t0 + (int64_t)idx < p.rcap, CK_REGION)) {
                        p.rtab[t0 + idx] = lds[sl];
                        store_slot(sl, p.rtab, p.rcap, t0 + idx, len);
                    }
                } else if (len != 0) {
                    d.special |= sl == p.lcap ? 1u : 2u;
                    add_slot(sl, sl == p.lcap ? p.gcap : p.gcap + 1, len);
                }
                run += tot;
            }
            if (threadIdx.x == 0) p.region_cnt[blockIdx.x / p.part_blocks] = run;
            if (p.wave_report) flush_and_report<false>(p, lds, L, d);
            else report_wg(p, d, wsc);
        } else {
        for (int sl = threadIdx.x; sl < L; sl += blockDim.x) {
            const uint64_t len = *fld(sl, 1);
            if (len == 0) continue;
            int64_t gs;
            if (sl == p.lcap) {
                gs = p.gcap;
                d.special |= 1u;
            } else if (sl == p.lcap + 1) {
                gs = p.gcap + 1;
                d.special |= 2u;
            } else {
                const int64_t t = PART && p.rbits > 0 ? g_direct_claim(p, sl, lds[sl]) : -1;
                if (t >= 0) {
                    // the partition's own region slot: plain stores
                    ++d.newkeys;
                    store_slot(sl, p.gtab, p.gcap + 2, t, len);
                    continue;
                }
                bool ins = false;
                gs = g_find_ins(p, lds[sl], ins);
                d.newkeys += ins ? 1u : 0u;
                if (gs < 0) {
                    atomicAdd((unsigned long long*)&p.status[ST_TABLE_FULL], 1ull);
                    continue;
                }
            }
            add_slot(sl, gs, len);
        }
        if (p.wave_report) flush_and_report<false>(p, lds, L, d);
            else report_wg(p, d, wsc);
        }
    } else {
        grun_flush();
        flush_and_report<true>(p, lds, L, d);
    }
}

struct OutSpec {
    int32_t kind;
    int32_t acc;
    int32_t out_dtype;
    int32_t in_isf;
    int32_t in_uns;
    int32_t ddof;     // VAR / STD
    int32_t acc_hi;   // VAR / STD: the accs of x * x rounded and of its exact error
    int32_t acc_lo;
    void* values;
    uint32_t* validity;
};

inline int num_cus() {
    static int g_num_cus = 0;
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
    int acc_in[kMaxAcc];  // the input index each acc aggregates
    size_t lds_bytes;
    int grid;
    bool use_lds;
    bool sum_only;
    int limbs;         // SUMONLY: 40-bit LDS limbs per f64 sum (3, or 2 for narrow exponent spans)
    int fast_grid;
    bool runs;         // sampled keys mostly equal their next row's (sorted / clustered input)
    bool local;        // range-local mode: contiguous tiles per workgroup, LDS sized by range-local keys
    bool part_racc = false;  // partitioned path: register accumulators (clustered / sorted keys)
    bool nulls = false;      // the fused kernel's NULLS variant (nullable key / values / predicate)
    mutable int launched_grid;  // grid of the last fast launch (info)
    mutable bool launched_runs = false;  // that launch used the register-run variant (info)
    mutable bool launched_var = false;   // that launch was the variance-triple variant (info)
};

// Workgroups of `kern` resident per CU at this LDS size (cached).
inline int resident_per_cu(const void* kern, int threads, size_t lds) {
    static std::vector<std::tuple<const void*, int, size_t, int>> cache;
    for (auto& c : cache)
        if (std::get<0>(c) == kern && std::get<1>(c) == threads && std::get<2>(c) == lds) return std::get<3>(c);
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, threads, lds) != hipSuccess || nb < 1) nb = 1;
    cache.emplace_back(kern, threads, lds, nb);
    return nb;
}

inline bool same_dev_col(const DevCol& x, const DevCol& y) {
    return x.values == y.values && x.offset == y.offset && x.dtype == y.dtype && x.validity == y.validity;
}

// The product pair's launch parameters (gb_fast_kernel VAR 2 / 3): acc pi's
// column becomes the product's operand that is not the other acc's column
// (x * y commutes exactly), and a simple predicate (pred) shares the acc
// whose column it reads.
inline void pair_normalize(GbParams& q, int pi, bool pred) {
    AccSpec& pa = q.acc[pi];
    if (!same_dev_col(pa.c2, q.acc[1 - pi].c)) std::swap(pa.c, pa.c2);
    if (pred) {
        q.pred_acc = -1;
        for (int a = 0; a < 2 && q.pred_acc < 0; ++a)
            if (same_dev_col(q.acc[a].c, q.pred_col)) q.pred_acc = a;
    }
}

template <int NACC, int PRED, bool SUMONLY, int LIMBS = 3, bool RUNS = false, bool DERIV = false, int VAR = 0,
          int PACK = 0, int ROWS = 2, bool NULLS = false>
hipError_t launch_fast_rows(const Plan& pl, const DevProgram& dp, hipStream_t s) {
    const void* kern =
        (const void*)gb_fast_kernel<NACC, PRED, SUMONLY, ROWS, LIMBS, RUNS, false, DERIV, VAR, PACK, NULLS>;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    const size_t lds =
        (SUMONLY && LIMBS == 2) ? (size_t)slim_words(NACC) * (pl.p.lcap + 2) * 8 + kWgScratch : pl.lds_bytes;
    GbParams q = pl.p;
    q.tiles_per_wg = 0;
    q.wave_report = options().wave_report;
    if (VAR == 2 || VAR == 3) pair_normalize(q, VAR - 2, PRED == 1);
    // the plan's n_full is a multiple of the 2-row tile; a wider tile takes
    // its own multiple (the masked last tile covers the rest)
    if (ROWS != 2) q.n_full = (pl.p.n / ((int64_t)kGbThreads * ROWS)) * kGbThreads * ROWS;
    // up to kGridRounds rounds of the workgroups resident per CU (later
    // rounds' table init / flush overlap earlier rounds' streaming), but at
    // least kMinTilesPerWg tiles per workgroup: every workgroup flushes its
    // table to the global one, a fixed cost a short input cannot amortise
    // (1e8 rows: 0.66 ms in one round against 0.84 ms in 8,
    // profiles/r04_grid_rounds_ab.txt)
    const int64_t need = (q.n_full + kMaxRowsPerWg - 1) / kMaxRowsPerWg;
    const int64_t useful = q.n_full / ((int64_t)kGbThreads * ROWS);
    const int64_t resident = (int64_t)num_cus() * resident_per_cu(kern, kGbThreads, lds);
    const int64_t rounds = options().grid_rounds > 0
                               ? options().grid_rounds
                               : std::min<int64_t>(kGridRounds, std::max<int64_t>(1, useful / (resident * kMinTilesPerWg)));
    int64_t g = resident * rounds;
    if (g < need) g = need;
    if (g > useful) g = std::max<int64_t>(1, useful);
    const int grid = (int)g;
    pl.launched_grid = grid;
    pl.launched_runs = RUNS;
    pl.launched_var = VAR == 1 || VAR == 4;
    if (pl.local) {
        const int64_t tile = (int64_t)kGbThreads * ROWS;
        const int64_t nall = q.n_full / tile + (pl.p.n > q.n_full ? 1 : 0);
        q.tiles_per_wg = (int32_t)((nall + grid - 1) / grid);
    }
    KtScope kt("gb_fast_kernel", s);
    gb_fast_kernel<NACC, PRED, SUMONLY, ROWS, LIMBS, RUNS, false, DERIV, VAR, PACK, NULLS>
        <<<grid, kGbThreads, lds, s>>>(q, dp);
    return hipGetLastError();
}

// x >= 0 (or NaN) on every row the fused predicate keeps: a float compare
// on acc `a`'s own column that accepts no value below c (x > c, x >= c,
// x == c) with c >= 0 (NaN compares greatest and fails the limb window
// anyway; -0.0 converts to zero limbs either way).
// pred_acc is the FIRST acc reading the predicate's column (groupby.hip
// gb_plan), so sum_pos (VAR 5, a = NACC - 1) only fires when that column
// feeds the last acc alone; if it also feeds an earlier acc this returns
// false and the signed-limb kernel runs (correct, just not the variant).
inline bool var_x_nonneg(const Plan& pl, const DevProgram& dp, int a = 0) {
    if (!dp.simple || !dp.simple_isf || pl.p.pred_acc != a || dp.simple_op < 0 || dp.simple_op > 5) return false;
    if (pl.p.acc[a].dop != DOP_NONE || pl.p.acc[a].c.dtype != PLGPU_F64) return false;
    const uint32_t accept = (0x643152u >> (4 * dp.simple_op)) & 0xFu;  // simple_pred's classes: 1 lt, 2 eq, 4 gt
    if (accept & 1u) return false;
    double c;
    std::memcpy(&c, &dp.simple_imm, 8);
    return c >= 0.0;
}

// Nullable key / aggregated / predicate columns (gb_plan sends plain inputs
// here: no derived operands, no packed key, no register runs): the sum-only
// 2-limb layout, or the general one (3-limb sums, counts, min / max, first /
// last rows).
template <int NACC>
hipError_t launch_fast_nulls(const Plan& pl, const DevProgram& dp, int pred, hipStream_t s) {
    if constexpr (NACC > 0) {
        // VAR 5 (sum_pos): a null value of the predicate's column drops its
        // row, so the selected values of the last acc are still >= 0
        if (pl.sum_only && pl.limbs == 2 && pred == 1 && options().sum_pos && var_x_nonneg(pl, dp, NACC - 1))
            return launch_fast_rows<NACC, 1, true, 2, false, false, 5, 0, 2, true>(pl, dp, s);
        if (pl.sum_only && pl.limbs == 2)
            return pred == 0 ? launch_fast_rows<NACC, 0, true, 2, false, false, 0, 0, 2, true>(pl, dp, s)
                             : launch_fast_rows<NACC, 1, true, 2, false, false, 0, 0, 2, true>(pl, dp, s);
    }
    return pred == 0 ? launch_fast_rows<NACC, 0, false, 3, false, false, 0, 0, 2, true>(pl, dp, s)
                     : launch_fast_rows<NACC, 1, false, 3, false, false, 0, 0, 2, true>(pl, dp, s);
}

template <int NACC, int PRED, bool SUMONLY, bool DERIV, int PACK = 0>
hipError_t launch_fast(const Plan& pl, const DevProgram& dp, hipStream_t s) {
    if (SUMONLY && pl.limbs == 2 && pl.runs)
        return launch_fast_rows<NACC, PRED, SUMONLY, 2, true, DERIV, false, PACK>(pl, dp, s);
    if constexpr (NACC == 4 && PRED == 1 && SUMONLY && !DERIV) {
        if (pl.limbs == 2 && options().sum_pos && var_x_nonneg(pl, dp, NACC - 1))
            return launch_fast_rows<NACC, PRED, SUMONLY, 2, false, DERIV, 5, PACK>(pl, dp, s);
    }
    if (SUMONLY && pl.limbs == 2) return launch_fast_rows<NACC, PRED, SUMONLY, 2, false, DERIV, false, PACK>(pl, dp, s);
    if (!SUMONLY && NACC > 0 && !DERIV && pl.runs && pl.limbs == 2)
        return launch_fast_rows<NACC, PRED, false, 2, true, false, false, PACK>(pl, dp, s);
    return launch_fast_rows<NACC, PRED, SUMONLY, 3, false, DERIV, false, PACK>(pl, dp, s);
}

template <int NACC, bool DERIV, int PACK = 0>
hipError_t launch_fast_nacc(const Plan& pl, const DevProgram& dp, int pred, hipStream_t s) {
    if constexpr (PACK == 2) {
        // String key codes: sum-only layouts (gb_plan falls back otherwise)
        if (!pl.sum_only) return hipErrorInvalidValue;
        return pred == 0 ? launch_fast<NACC, 0, true, DERIV, 2>(pl, dp, s) : launch_fast<NACC, 1, true, DERIV, 2>(pl, dp, s);
    } else {
    if (pl.sum_only)
        return pred == 0 ? launch_fast<NACC, 0, true, DERIV, PACK>(pl, dp, s)
                         : launch_fast<NACC, 1, true, DERIV, PACK>(pl, dp, s);
    return pred == 0 ? launch_fast<NACC, 0, false, DERIV, PACK>(pl, dp, s)
                     : launch_fast<NACC, 1, false, DERIV, PACK>(pl, dp, s);
    }
}

// The fused variance's triple (x, x * x, its error: three sums of one
// column, the derived two sharing x's load), on the sum-only layout or the
// general one (maintain_order's first-row field, x's count).
inline bool var_triple(const Plan& pl) {
    const GbParams& p = pl.p;
    if (p.nacc != 3) return false;
    const AccSpec& a0 = p.acc[0];
    for (int a = 1; a < 3; ++a) {
        const AccSpec& ac = p.acc[a];
        if (ac.dop != ((a == 1 ? DOP_SQHI : DOP_SQLO) | DOP_LIT) || ac.c.values != a0.c.values ||
            ac.c.offset != a0.c.offset || ac.c.validity != a0.c.validity || ac.c.dtype != a0.c.dtype)
            return false;
    }
    return a0.dop == DOP_NONE && a0.c.dtype == PLGPU_F64;
}

template <int PRED>
hipError_t launch_fast_var(const Plan& pl, const DevProgram& dp, hipStream_t s) {
    if (!pl.sum_only) return launch_fast_rows<3, PRED, false, 3, false, false, 1>(pl, dp, s);
    if (pl.limbs == 2) {
        if (PRED == 1 && options().var_pos && var_x_nonneg(pl, dp))
            return launch_fast_rows<3, PRED, true, 2, false, false, 4>(pl, dp, s);
        return launch_fast_rows<3, PRED, true, 2, false, false, 1>(pl, dp, s);
    }
    return launch_fast_rows<3, PRED, true, 3, false, false, 1>(pl, dp, s);
}


// A product and one of its operands, f64 sums on the sum-only layout:
// (close * volume).sum() next to volume.sum(), in either order.  Returns the
// product's acc index, or -1.
inline int product_pair(const Plan& pl) {
    const GbParams& p = pl.p;
    if (p.nacc != 2 || !pl.sum_only) return -1;
    for (int pi = 0; pi < 2; ++pi) {
        const AccSpec& pa = p.acc[pi];
        const AccSpec& oa = p.acc[1 - pi];
        if ((pa.dop & ~DOP_SWAP) != DOP_MUL || oa.dop != DOP_NONE) continue;
        if (pa.c.dtype != PLGPU_F64 || pa.c2.dtype != PLGPU_F64 || oa.c.dtype != PLGPU_F64) continue;
        if (pa.c.validity || pa.c2.validity || oa.c.validity) continue;
        if (same_dev_col(pa.c2, oa.c) || same_dev_col(pa.c, oa.c)) return pi;
    }
    return -1;
}

template <int PRED, int VAR>
hipError_t launch_fast_pair(const Plan& pl, const DevProgram& dp, hipStream_t s) {
    if (pl.limbs == 2 && pl.runs) return launch_fast_rows<2, PRED, true, 2, true, false, VAR>(pl, dp, s);
    if (pl.limbs == 2) return launch_fast_rows<2, PRED, true, 2, false, false, VAR>(pl, dp, s);
    return launch_fast_rows<2, PRED, true, 3, false, false, VAR>(pl, dp, s);
}

template <int NACC, int LIMBS, bool RACC, bool NULLS = false>
hipError_t launch_part_fast(const Plan& pp, int grid, hipStream_t s) {
    const void* kern = (const void*)gb_fast_kernel<NACC, 0, true, 2, LIMBS, RACC, true, false, 0, 0, NULLS>;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    // (+ the slim flush's workgroup scratch after the table)
    const size_t lds = (size_t)(LIMBS == 2 ? slim_words(NACC) : pp.p.nfields) * (pp.p.lcap + 2) * 8 + kWgScratch;
    DevProgram none;
    std::memset(&none, 0, sizeof none);
    // 1024 threads where each workgroup has many rows to share its table's
    // fixed costs over (2e4 groups: 5.0 -> 3.9 ms, 1e6: 5.0 -> 4.2 ms);
    // with ~17k rows per partition (1e7 groups) 512 (7.7 against 13.7 ms)
    const int64_t per_wg = pp.p.n / std::max(grid, 1);
    int threads = RACC || per_wg < 65536 ? kGbThreads : kGbPartThreads;
    if (!RACC && options().part_threads > 0) threads = std::min(kGbPartThreads, options().part_threads);
    GbParams q = pp.p;
    q.wave_report = options().wave_report;
    if constexpr (LIMBS == 2 && !RACC) {
        // option part_rows4 (A/B): 512-thread workgroups holding 4 rows per
        // thread (two row pairs in flight per tile instead of one), compiled
        // for 512 threads: a partition workgroup owns its CU's LDS, so the
        // extra registers cost no occupancy
        if (threads == kGbThreads && options().part_rows4) {
            const void* k4 = (const void*)gb_fast_kernel<NACC, 0, true, 4, 2, false, true, false, 0, 0, NULLS>;
            static bool attr4 = false;
            if (!attr4) {
                (void)hipFuncSetAttribute(k4, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                attr4 = true;
            }
            gb_fast_kernel<NACC, 0, true, 4, 2, false, true, false, 0, 0, NULLS><<<grid, threads, lds, s>>>(q, none);
            return hipGetLastError();
        }
    }
    gb_fast_kernel<NACC, 0, true, 2, LIMBS, RACC, true, false, 0, 0, NULLS><<<grid, threads, lds, s>>>(q, none);
    return hipGetLastError();
}

// register accumulators (RACC) on the 2-limb window, for clustered keys
template <int NACC>
hipError_t launch_part_fast_limbs(const Plan& pp, int grid, hipStream_t s) {
    // nullable rows (the partition buffers' null bits): no register runs
    if (pp.p.part_nulls)
        return pp.limbs == 2 ? launch_part_fast<NACC, 2, false, true>(pp, grid, s)
                             : launch_part_fast<NACC, 3, false, true>(pp, grid, s);
    if (pp.limbs != 2) return launch_part_fast<NACC, 3, false>(pp, grid, s);
    return pp.part_racc ? launch_part_fast<NACC, 2, true>(pp, grid, s) : launch_part_fast<NACC, 2, false>(pp, grid, s);
}


// fused-kernel launches compiled in groupby_fast1..6.hip
#ifndef PLGPU_GB_FAST_TU
extern template hipError_t launch_fast_nacc<0, false, 0>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<0, false, 1>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<1, false, 0>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<1, false, 1>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<1, true, 0>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<1, false, 2>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_part_fast_limbs<1>(const Plan&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<2, false, 0>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<2, false, 1>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<2, true, 0>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<2, false, 2>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_part_fast_limbs<2>(const Plan&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<3, false, 0>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<3, false, 1>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<3, true, 0>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<3, false, 2>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_part_fast_limbs<3>(const Plan&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<4, false, 0>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<4, false, 1>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<4, true, 0>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<4, false, 2>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_part_fast_limbs<4>(const Plan&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<5, false, 0>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<5, false, 1>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<5, true, 0>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<5, false, 2>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_part_fast_limbs<5>(const Plan&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<6, false, 0>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<6, false, 1>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<6, true, 0>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nacc<6, false, 2>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_part_fast_limbs<6>(const Plan&, int, hipStream_t);
extern template hipError_t launch_fast_nulls<0>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nulls<1>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nulls<2>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nulls<3>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nulls<4>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nulls<5>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_nulls<6>(const Plan&, const DevProgram&, int, hipStream_t);
extern template hipError_t launch_fast_var<0>(const Plan&, const DevProgram&, hipStream_t);
extern template hipError_t launch_fast_var<1>(const Plan&, const DevProgram&, hipStream_t);
extern template hipError_t launch_fast_pair<0, 2>(const Plan&, const DevProgram&, hipStream_t);
extern template hipError_t launch_fast_pair<1, 2>(const Plan&, const DevProgram&, hipStream_t);
extern template hipError_t launch_fast_pair<0, 3>(const Plan&, const DevProgram&, hipStream_t);
extern template hipError_t launch_fast_pair<1, 3>(const Plan&, const DevProgram&, hipStream_t);
#endif

}  // namespace plgpu
