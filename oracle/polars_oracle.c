/*
 * polars_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded (plus one OpenMP baseline entry) restatement of
 * the reference's CPU algorithms for the filter -> group_by -> agg path.  It
 * is the checker the parity tests compare the HIP path against, and the
 * `cpu_baseline` leg of bench.py.  Nothing in the product path (polaroid_amd/)
 * links, imports or calls it.
 *
 * Reference (Rust, /root/reference/crates — unbuildable here: no rustc) is
 * followed function by function; each function cites file:line.
 * Pinned by: the JSON fixtures in tests/golden (truth tables and expected outputs from the
 * reference's own tests, see tests/golden/make_golden.py) and by CPython's
 * math.fsum for the exact-sum leg (tests/test_oracle.py).
 *
 * Host buffers use the same plgpu_column struct as the C-ABI (host pointers).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/polaroid_gpu.h"

#define OR_EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------ helpers */
static inline int bit_get(const uint8_t* bm, int64_t i) { return (bm[i >> 3] >> (i & 7)) & 1; }
static inline void bit_set(uint8_t* bm, int64_t i, int v) {
    if (v) bm[i >> 3] |= (uint8_t)(1u << (i & 7));
    else bm[i >> 3] &= (uint8_t)~(1u << (i & 7));
}
static inline int col_valid(const plgpu_column* c, int64_t r) {
    return c->validity == NULL ? 1 : bit_get(c->validity, c->offset + r);
}

/* A typed scalar as seen by the expression interpreter.
 *   dt     the polars dtype (plgpu_dtype code), or one of the dynamic
 *          literal kinds below (polars' UnknownKind::Int / Float / a bare
 *          null), which take their type from the other operand;
 *   i      signed ints and Boolean (value), unsigned ints (bits);
 *   f      Float64, or a Float32 value widened (exactly) to double;
 *   scalar a literal or an expression of literals: a length-1 column that
 *          the reference broadcasts with the *_scalar kernels. */
#define DYN_INT 100
#define DYN_FLOAT 101
#define DYN_NULL 102
typedef struct {
    int dt;
    int valid;
    int scalar;
    int64_t i;
    double f;
} val_t;

static int is_signed(int dt) { return dt == PLGPU_I8 || dt == PLGPU_I16 || dt == PLGPU_I32 || dt == PLGPU_I64; }
static int is_unsigned(int dt) { return dt == PLGPU_U8 || dt == PLGPU_U16 || dt == PLGPU_U32 || dt == PLGPU_U64; }
static int is_intd(int dt) { return is_signed(dt) || is_unsigned(dt); }
static int is_floatd(int dt) { return dt == PLGPU_F32 || dt == PLGPU_F64; }
static int bits_of(int dt) {
    switch (dt) {
    case PLGPU_I8: case PLGPU_U8: return 8;
    case PLGPU_I16: case PLGPU_U16: return 16;
    case PLGPU_I32: case PLGPU_U32: case PLGPU_F32: return 32;
    default: return 64;
    }
}

static val_t col_get(const plgpu_column* c, int64_t r) {
    val_t v;
    v.valid = col_valid(c, r);
    v.scalar = 0;
    v.i = 0;
    v.f = 0.0;
    v.dt = c->dtype;
    int64_t p = c->offset + r;
    switch (c->dtype) {
    case PLGPU_BOOL: v.i = bit_get((const uint8_t*)c->values, p); break;
    case PLGPU_I8: v.i = ((const int8_t*)c->values)[p]; break;
    case PLGPU_I16: v.i = ((const int16_t*)c->values)[p]; break;
    case PLGPU_I32: v.i = ((const int32_t*)c->values)[p]; break;
    case PLGPU_I64: v.i = ((const int64_t*)c->values)[p]; break;
    case PLGPU_U8: v.i = ((const uint8_t*)c->values)[p]; break;
    case PLGPU_U16: v.i = ((const uint16_t*)c->values)[p]; break;
    case PLGPU_U32: v.i = ((const uint32_t*)c->values)[p]; break;
    case PLGPU_U64: v.i = (int64_t)((const uint64_t*)c->values)[p]; break;
    case PLGPU_F32: v.f = ((const float*)c->values)[p]; break;
    default: v.f = ((const double*)c->values)[p]; break;
    }
    return v;
}

/* TotalOrd for f64: polars-utils/src/total_ord.rs:317-368.
 * tot_ge(a,b) = a.is_nan() | (a >= b); tot_lt = !tot_ge; tot_gt(a,b) = tot_lt(b,a);
 * tot_le(a,b) = tot_ge(b,a); tot_eq: NaN == NaN. */
static int f_tot_ge(double a, double b) { return isnan(a) || a >= b; }
static int f_tot_eq(double a, double b) { return isnan(a) ? isnan(b) : a == b; }
static int f_cmp(int op, double a, double b) {
    switch (op) {
    case PLGPU_OP_EQ: return f_tot_eq(a, b);
    case PLGPU_OP_NE: return !f_tot_eq(a, b);
    case PLGPU_OP_LT: return !f_tot_ge(a, b);
    case PLGPU_OP_LE: return f_tot_ge(b, a);
    case PLGPU_OP_GT: return !f_tot_ge(b, a);
    case PLGPU_OP_GE: return f_tot_ge(a, b);
    }
    return 0;
}
static int i_cmp(int op, int64_t a, int64_t b) {
    switch (op) {
    case PLGPU_OP_EQ: return a == b;
    case PLGPU_OP_NE: return a != b;
    case PLGPU_OP_LT: return a < b;
    case PLGPU_OP_LE: return a <= b;
    case PLGPU_OP_GT: return a > b;
    case PLGPU_OP_GE: return a >= b;
    }
    return 0;
}
static int u_cmp(int op, uint64_t a, uint64_t b) {
    switch (op) {
    case PLGPU_OP_EQ: return a == b;
    case PLGPU_OP_NE: return a != b;
    case PLGPU_OP_LT: return a < b;
    case PLGPU_OP_LE: return a <= b;
    case PLGPU_OP_GT: return a > b;
    case PLGPU_OP_GE: return a >= b;
    }
    return 0;
}

/* polars-core/src/utils/supertype.rs:146 get_supertype, the primitive
 * numeric / Boolean rows (0 = no supertype). */
static int supertype(int l, int r) {
    if (l == r) return l;
    if (l == PLGPU_BOOL) return (is_intd(r) || is_floatd(r)) ? r : 0;  /* (Int8, Boolean) => Int8, ... */
    if (r == PLGPU_BOOL) return (is_intd(l) || is_floatd(l)) ? l : 0;
    if (is_floatd(l) && is_floatd(r)) return PLGPU_F64;                /* (Float32, Float64) => Float64 */
    if (is_floatd(l) || is_floatd(r)) {
        int fl = is_floatd(l) ? l : r, in = is_floatd(l) ? r : l;
        if (fl == PLGPU_F64) return PLGPU_F64;
        return bits_of(in) <= 16 ? PLGPU_F32 : PLGPU_F64;                 /* (Int16, Float32) => Float32,
                                                                           (Int32, Float32) => Float64 */
    }
    if (is_signed(l) == is_signed(r)) return bits_of(l) >= bits_of(r) ? l : r;
    int s = is_signed(l) ? l : r, u = is_signed(l) ? r : l;
    if (u == PLGPU_U64) return PLGPU_F64;                                /* (Int64, UInt64) => Float64 */
    if (bits_of(u) < bits_of(s)) return s;                                /* (Int16, UInt8) => Int16 */
    return bits_of(u) == 8 ? PLGPU_I16 : bits_of(u) == 16 ? PLGPU_I32 : PLGPU_I64; /* (Int8, UInt8) => Int16 */
}

/* supertype.rs:463: a dynamic int v next to dtype dt: the smallest dtype
 * holding v (materialize_dyn_int_pos for an unsigned dt and v >= 0), then
 * the supertype; UInt64 with a signed literal stays integral (Int64). */
static int smallest_fit(int64_t v, int unsigned_ok) {
    if (unsigned_ok && v >= 0) {
        if (v <= 0xFF) return PLGPU_U8;
        if (v <= 0xFFFF) return PLGPU_U16;
        if (v <= 0xFFFFFFFFll) return PLGPU_U32;
        return PLGPU_U64;
    }
    if (v >= INT8_MIN && v <= INT8_MAX) return PLGPU_I8;
    if (v >= INT16_MIN && v <= INT16_MAX) return PLGPU_I16;
    if (v >= INT32_MIN && v <= INT32_MAX) return PLGPU_I32;
    return PLGPU_I64;
}
static int dyn_join(const val_t* lit, int dt) {
    if (lit->dt == DYN_NULL) return dt;
    if (is_floatd(dt)) return dt;                      /* materialize to the float dtype */
    if (lit->dt == DYN_FLOAT) return PLGPU_F64;        /* UnknownKind::Float with an integer */
    if (dt == PLGPU_BOOL) return supertype(PLGPU_BOOL, smallest_fit(lit->i, 0));
    int sm = smallest_fit(lit->i, is_unsigned(dt));
    if (dt == PLGPU_U64 && is_signed(sm)) return PLGPU_I64;
    return supertype(dt, sm);
}
/* A literal on its own materializes as Int32 / Int64 / Float64. */
static int dyn_alone(const val_t* v) {
    if (v->dt == DYN_INT) return (v->i >= INT32_MIN && v->i <= INT32_MAX) ? PLGPU_I32 : PLGPU_I64;
    if (v->dt == DYN_FLOAT) return PLGPU_F64;
    if (v->dt == DYN_NULL) return PLGPU_BOOL;
    return v->dt;
}
static int is_dyn(const val_t* v) { return v->dt == DYN_INT || v->dt == DYN_FLOAT || v->dt == DYN_NULL; }
static int join_types(const val_t* a, const val_t* b) {
    if (is_dyn(a) && is_dyn(b)) {
        if (a->dt == DYN_NULL) return dyn_alone(b);
        if (b->dt == DYN_NULL) return dyn_alone(a);
        if (a->dt == DYN_FLOAT || b->dt == DYN_FLOAT) return PLGPU_F64;
        return supertype(dyn_alone(a), dyn_alone(b));
    }
    if (is_dyn(a)) return dyn_join(a, b->dt);
    if (is_dyn(b)) return dyn_join(b, a->dt);
    return supertype(a->dt, b->dt);
}

/* Two's complement wrap of an integer to dtype dt (Rust `as` / wrapping_*). */
static int64_t wrap_int(int dt, uint64_t x) {
    switch (dt) {
    case PLGPU_I8: return (int8_t)x;
    case PLGPU_I16: return (int16_t)x;
    case PLGPU_I32: return (int32_t)x;
    case PLGPU_U8: return (uint8_t)x;
    case PLGPU_U16: return (uint16_t)x;
    case PLGPU_U32: return (uint32_t)x;
    default: return (int64_t)x;
    }
}

/* Non-strict cast (polars-core/src/chunked_array/cast.rs: a value that does
 * not fit the target is null; `overflowing` wraps integers).  Float -> int
 * truncates (num_traits::NumCast), int -> float rounds to nearest. */
static val_t cast_to(val_t v, int to, int overflowing) {
    val_t z = v;
    z.dt = to;
    if (!v.valid) { z.i = 0; z.f = 0; return z; }
    if (v.dt == DYN_INT) v.dt = PLGPU_I64;
    if (v.dt == DYN_FLOAT) v.dt = PLGPU_F64;
    if (to == PLGPU_BOOL) { z.i = is_floatd(v.dt) ? v.f != 0.0 : v.i != 0; return z; }
    if (v.dt == PLGPU_BOOL) { if (is_floatd(to)) z.f = (double)v.i; else z.i = v.i; return z; }
    if (is_intd(v.dt) && is_intd(to)) {
        /* exact value of the source: signed / unsigned 64-bit */
        int neg = is_signed(v.dt) && v.i < 0;
        uint64_t mag = (uint64_t)v.i;
        int fits;
        if (is_unsigned(to)) {
            fits = !neg && (to == PLGPU_U64 || mag <= (((uint64_t)1 << bits_of(to)) - 1));
        } else {
            int64_t lo = to == PLGPU_I64 ? INT64_MIN : -((int64_t)1 << (bits_of(to) - 1));
            int64_t hi = to == PLGPU_I64 ? INT64_MAX : ((int64_t)1 << (bits_of(to) - 1)) - 1;
            if (v.dt == PLGPU_U64) fits = mag <= (uint64_t)hi;
            else fits = v.i >= lo && v.i <= hi;
        }
        if (fits) z.i = v.i;
        else if (overflowing) z.i = wrap_int(to, (uint64_t)v.i);
        else { z.valid = 0; z.i = 0; }
        return z;
    }
    if (is_intd(v.dt) && is_floatd(to)) {
        if (to == PLGPU_F32) z.f = v.dt == PLGPU_U64 ? (double)(float)(uint64_t)v.i : (double)(float)v.i;
        else z.f = v.dt == PLGPU_U64 ? (double)(uint64_t)v.i : (double)v.i;
        return z;
    }
    if (is_floatd(v.dt) && is_floatd(to)) { z.f = to == PLGPU_F32 ? (double)(float)v.f : v.f; return z; }
    /* float -> int */
    double t = trunc(v.f);
    int ok;
    if (isnan(t)) ok = 0;
    else if (to == PLGPU_U64) ok = t >= 0.0 && t < 18446744073709551616.0;
    else if (to == PLGPU_I64) ok = t >= -9223372036854775808.0 && t < 9223372036854775808.0;
    else if (is_unsigned(to)) ok = t >= 0.0 && t <= (double)((((uint64_t)1) << bits_of(to)) - 1);
    else ok = t >= -(double)((int64_t)1 << (bits_of(to) - 1)) && t <= (double)(((int64_t)1 << (bits_of(to) - 1)) - 1);
    if (!ok) { z.valid = 0; z.i = 0; return z; }
    z.i = to == PLGPU_U64 ? (int64_t)(uint64_t)t : (int64_t)t;
    return z;
}

/* Give an operand the type t (literal materialization or a cast). */
static val_t coerce(val_t v, int t) {
    if (v.dt == DYN_NULL) { v.dt = t; v.i = 0; v.f = 0; return v; }
    if (v.dt == DYN_INT) {
        v.dt = t;
        if (is_floatd(t)) v.f = t == PLGPU_F32 ? (double)(float)v.i : (double)v.i;
        return v;
    }
    if (v.dt == DYN_FLOAT) {
        v.dt = t;
        if (t == PLGPU_F32) v.f = (double)(float)v.f;
        return v;
    }
    if (v.dt == t) return v;
    int s = v.scalar;
    v = cast_to(v, t, 0);
    v.scalar = s;
    return v;
}

/* polars-utils/src/floor_divmod.rs:39 (signed) and :28 (unsigned). */
static void int_floor_divmod(int dt, int64_t a, int64_t b, int64_t* q, int64_t* m) {
    if (dt == PLGPU_U64) {
        *q = (int64_t)((uint64_t)a / (uint64_t)b);
        *m = (int64_t)((uint64_t)a % (uint64_t)b);
        return;
    }
    if (a == INT64_MIN && b == -1) { *q = INT64_MIN; *m = 0; return; }  /* wrapping_div */
    int64_t d = a / b, r = a % b;
    if (r != 0 && ((a < 0) != (b < 0))) { d -= 1; r += b; }
    *q = d;
    *m = r;
}

/* One arithmetic op on two operands of type t.  Integer ops wrap at t's
 * width (polars-compute/src/arithmetic/{signed,unsigned}.rs wrapping_*); a
 * zero divisor gives null (:35, :60); Float32 runs in single precision;
 * a broadcast (scalar) divisor uses the reciprocal forms of
 * arithmetic/float.rs:78-98 and :113 (true_div_scalar: x * (1 / rhs)). */
static val_t arith(int op, val_t a, val_t b, int t) {
    val_t z;
    memset(&z, 0, sizeof z);
    z.dt = t;
    z.scalar = a.scalar && b.scalar;
    z.valid = a.valid && b.valid;
    const int bscalar = b.scalar && !a.scalar;
    if (is_intd(t)) {
        uint64_t x = (uint64_t)a.i, y = (uint64_t)b.i;
        switch (op) {
        case PLGPU_OP_ADD: z.i = wrap_int(t, x + y); break;
        case PLGPU_OP_SUB: z.i = wrap_int(t, x - y); break;
        case PLGPU_OP_MUL: z.i = wrap_int(t, x * y); break;
        default: {  /* FLOORDIV / DIVIDE (legacy_div = floor div for ints) / MOD */
            if (b.i == 0) { z.valid = 0; break; }
            int64_t q, m;
            int_floor_divmod(t, a.i, b.i, &q, &m);
            z.i = wrap_int(t, (uint64_t)(op == PLGPU_OP_MOD ? m : q));
        }
        }
        if (!z.valid) z.i = 0;
        return z;
    }
    if (t == PLGPU_F32) {
        float x = (float)a.f, y = (float)b.f, r;
        switch (op) {
        case PLGPU_OP_ADD: r = x + y; break;
        case PLGPU_OP_SUB: r = x - y; break;
        case PLGPU_OP_MUL: r = x * y; break;
        case PLGPU_OP_FLOORDIV: r = bscalar ? floorf(x * (1.0f / y)) : floorf(x / y); break;
        case PLGPU_OP_MOD: {
            float q = bscalar ? floorf(x * (1.0f / y)) : floorf(x / y);
            float yq = y * q;
            r = x - yq;
            break;
        }
        default: r = bscalar ? x * (1.0f / y) : x / y; break;  /* TRUEDIV / DIVIDE */
        }
        z.f = r;
        return z;
    }
    double x = a.f, y = b.f;
    switch (op) {
    case PLGPU_OP_ADD: z.f = x + y; break;
    case PLGPU_OP_SUB: z.f = x - y; break;
    case PLGPU_OP_MUL: z.f = x * y; break;
    case PLGPU_OP_FLOORDIV: z.f = bscalar ? floor(x * (1.0 / y)) : floor(x / y); break;
    case PLGPU_OP_MOD: {
        double q = bscalar ? floor(x * (1.0 / y)) : floor(x / y);
        double yq = y * q;
        z.f = x - yq;
        break;
    }
    default: z.f = bscalar ? x * (1.0 / y) : x / y; break;
    }
    return z;
}

/* One postfix program, one row.  Returns 0 on success, -1 on type error. */
static int eval_row(const plgpu_column* cols, const plgpu_instr* prog, int n, int64_t r, val_t* out) {
    val_t st[PLGPU_MAX_STACK];
    int sp = 0;
    for (int k = 0; k < n; ++k) {
        const plgpu_instr* in = &prog[k];
        val_t a, b, c, z;
        memset(&z, 0, sizeof z);
        if (sp >= PLGPU_MAX_STACK && (in->op <= PLGPU_OP_LIT_NULL)) return -1;
        switch (in->op) {
        case PLGPU_OP_COL: st[sp++] = col_get(&cols[in->arg], r); break;
        case PLGPU_OP_LIT_F64: z.dt = DYN_FLOAT; z.valid = 1; z.scalar = 1; z.f = in->imm.f64; st[sp++] = z; break;
        case PLGPU_OP_LIT_I64: z.dt = DYN_INT; z.valid = 1; z.scalar = 1; z.i = in->imm.i64; st[sp++] = z; break;
        case PLGPU_OP_LIT_BOOL: z.dt = PLGPU_BOOL; z.valid = 1; z.scalar = 1; z.i = in->imm.i64 != 0; st[sp++] = z; break;
        case PLGPU_OP_LIT_NULL:
            z.dt = in->arg ? in->arg : DYN_NULL;
            z.valid = 0;
            z.scalar = 1;
            st[sp++] = z;
            break;
        case PLGPU_OP_ADD: case PLGPU_OP_SUB: case PLGPU_OP_MUL: case PLGPU_OP_TRUEDIV:
        case PLGPU_OP_FLOORDIV: case PLGPU_OP_MOD: case PLGPU_OP_DIVIDE: {
            if (sp < 2) return -1;
            b = st[--sp]; a = st[--sp];
            if (a.dt == PLGPU_BOOL || b.dt == PLGPU_BOOL) return -1;
            int t = join_types(&a, &b);
            if (!t) return -1;
            if (t == PLGPU_BOOL) t = PLGPU_I32;
            /* TrueDivide: integers are cast to Float64 first
             * (polars-expr/src/expressions/binary.rs:73 apply_operator) */
            if (in->op == PLGPU_OP_TRUEDIV && !is_floatd(t)) t = PLGPU_F64;
            a = coerce(a, t);
            b = coerce(b, t);
            st[sp++] = arith(in->op, a, b, t);
            break;
        }
        case PLGPU_OP_NEG: case PLGPU_OP_ABS:
            if (sp < 1) return -1;
            a = st[--sp];
            if (a.dt == PLGPU_BOOL) return -1;
            if (a.dt == DYN_INT) {
                a.i = in->op == PLGPU_OP_NEG ? (int64_t)(0 - (uint64_t)a.i)
                                             : (a.i < 0 ? (int64_t)(0 - (uint64_t)a.i) : a.i);
            } else if (a.dt == DYN_FLOAT || is_floatd(a.dt)) {
                a.f = in->op == PLGPU_OP_NEG ? -a.f : fabs(a.f);
            } else {
                if (a.dt == DYN_NULL) a.dt = PLGPU_I32;
                if (in->op == PLGPU_OP_NEG && is_unsigned(a.dt)) return -1;  /* `neg` not supported for u8.. */
                uint64_t x = (uint64_t)a.i;
                int64_t v = in->op == PLGPU_OP_NEG ? (int64_t)(0 - x) : (a.i < 0 ? (int64_t)(0 - x) : a.i);
                a.i = wrap_int(a.dt, (uint64_t)v);  /* wrapping_neg / wrapping_abs at the width */
                if (!a.valid) a.i = 0;
            }
            st[sp++] = a;
            break;
        case PLGPU_OP_CAST_F64:
        case PLGPU_OP_CAST: {
            if (sp < 1) return -1;
            a = st[--sp];
            int to = in->op == PLGPU_OP_CAST_F64 ? PLGPU_F64 : in->arg;
            if (is_dyn(&a)) a = coerce(a, a.dt == DYN_NULL ? to : dyn_alone(&a));
            int s = a.scalar;
            a = cast_to(a, to, in->op == PLGPU_OP_CAST && (in->imm.i64 & 1));
            a.scalar = s;
            st[sp++] = a;
            break;
        }
        case PLGPU_OP_EQ: case PLGPU_OP_NE: case PLGPU_OP_LT: case PLGPU_OP_LE:
        case PLGPU_OP_GT: case PLGPU_OP_GE: case PLGPU_OP_EQ_MISSING: case PLGPU_OP_NE_MISSING: {
            if (sp < 2) return -1;
            b = st[--sp]; a = st[--sp];
            int missing = in->op == PLGPU_OP_EQ_MISSING || in->op == PLGPU_OP_NE_MISSING;
            int op = in->op == PLGPU_OP_EQ_MISSING ? PLGPU_OP_EQ
                   : in->op == PLGPU_OP_NE_MISSING ? PLGPU_OP_NE : in->op;
            if ((a.dt == PLGPU_BOOL) != (b.dt == PLGPU_BOOL) && !is_dyn(&a) && !is_dyn(&b)) return -1;
            int t = join_types(&a, &b);
            if (!t) return -1;
            if (a.dt == PLGPU_BOOL || b.dt == PLGPU_BOOL) t = PLGPU_BOOL;
            if (t == PLGPU_BOOL && op != PLGPU_OP_EQ && op != PLGPU_OP_NE) return -1;
            a = coerce(a, t);
            b = coerce(b, t);
            z.dt = PLGPU_BOOL;
            z.scalar = a.scalar && b.scalar;
            if (!(a.valid && b.valid)) {
                if (missing) {
                    /* null == null; null != value (polars eq_missing) */
                    int eq = !a.valid && !b.valid;
                    z.valid = 1;
                    z.i = op == PLGPU_OP_EQ ? eq : !eq;
                } else {
                    z.valid = 0;
                }
            } else {
                z.valid = 1;
                if (is_floatd(t)) z.i = f_cmp(op, a.f, b.f);
                else if (t == PLGPU_U64) z.i = u_cmp(op, (uint64_t)a.i, (uint64_t)b.i);
                else z.i = i_cmp(op, a.i, b.i);
            }
            st[sp++] = z;
            break;
        }
        case PLGPU_OP_AND: case PLGPU_OP_OR: case PLGPU_OP_XOR: {
            if (sp < 2) return -1;
            b = st[--sp]; a = st[--sp];
            int ba = a.dt == PLGPU_BOOL || a.dt == DYN_NULL, bb = b.dt == PLGPU_BOOL || b.dt == DYN_NULL;
            z.scalar = a.scalar && b.scalar;
            if (ba && bb) {
                z.dt = PLGPU_BOOL;
                if (in->op == PLGPU_OP_XOR) {
                    /* BooleanArray ^ (bitxor): null if either is null */
                    z.valid = a.valid && b.valid;
                    z.i = z.valid ? (a.i ^ b.i) : 0;
                } else if (in->op == PLGPU_OP_AND) {
                    /* Kleene logic (polars-arrow/src/compute/boolean_kleene.rs). */
                    if ((a.valid && !a.i) || (b.valid && !b.i)) { z.valid = 1; z.i = 0; }
                    else if (a.valid && b.valid) { z.valid = 1; z.i = 1; }
                    else z.valid = 0;
                } else {
                    if ((a.valid && a.i) || (b.valid && b.i)) { z.valid = 1; z.i = 1; }
                    else if (a.valid && b.valid) { z.valid = 1; z.i = 0; }
                    else z.valid = 0;
                }
            } else {
                /* integers: bitand / bitor / bitxor of the supertype */
                int t = join_types(&a, &b);
                if (!t || !is_intd(t)) return -1;
                a = coerce(a, t);
                b = coerce(b, t);
                z.dt = t;
                z.valid = a.valid && b.valid;
                uint64_t x = (uint64_t)a.i, y = (uint64_t)b.i;
                z.i = z.valid ? wrap_int(t, in->op == PLGPU_OP_AND ? x & y : in->op == PLGPU_OP_OR ? x | y : x ^ y) : 0;
            }
            st[sp++] = z;
            break;
        }
        case PLGPU_OP_FILL_NULL: {
            /* FunctionExpr::FillNull: coalesce(x, fill) in the supertype */
            if (sp < 2) return -1;
            b = st[--sp]; a = st[--sp];
            int t = join_types(&a, &b);
            if (!t) return -1;
            a = coerce(a, t);
            b = coerce(b, t);
            z = a.valid ? a : b;
            z.scalar = a.scalar && b.scalar;
            st[sp++] = z;
            break;
        }
        case PLGPU_OP_IF_ELSE: {
            /* when(c).then(a).otherwise(b): a null condition selects b
             * (polars-core zip_with / if_then_else: mask nulls are false) */
            if (sp < 3) return -1;
            b = st[--sp]; a = st[--sp]; c = st[--sp];
            if (c.dt != PLGPU_BOOL && c.dt != DYN_NULL) return -1;
            int t = join_types(&a, &b);
            if (!t) return -1;
            a = coerce(a, t);
            b = coerce(b, t);
            z = (c.valid && c.i) ? a : b;
            z.scalar = c.scalar && a.scalar && b.scalar;
            st[sp++] = z;
            break;
        }
        case PLGPU_OP_NOT:
            if (sp < 1) return -1;
            a = st[--sp];
            if (a.dt == DYN_NULL) a.dt = PLGPU_BOOL;
            if (a.dt == PLGPU_BOOL) a.i = a.valid ? !a.i : 0;
            else if (is_intd(a.dt)) a.i = a.valid ? wrap_int(a.dt, ~(uint64_t)a.i) : 0;  /* bitwise not */
            else return -1;
            st[sp++] = a;
            break;
        case PLGPU_OP_IS_NULL: case PLGPU_OP_IS_NOT_NULL:
            if (sp < 1) return -1;
            a = st[--sp];
            z.dt = PLGPU_BOOL; z.valid = 1; z.scalar = a.scalar;
            z.i = in->op == PLGPU_OP_IS_NULL ? !a.valid : a.valid;
            st[sp++] = z;
            break;
        case PLGPU_OP_IS_NAN: case PLGPU_OP_IS_FINITE:
            if (sp < 1) return -1;
            a = st[--sp];
            if (a.dt == DYN_FLOAT) a.dt = PLGPU_F64;
            if (!is_floatd(a.dt)) return -1;
            z.dt = PLGPU_BOOL; z.valid = a.valid; z.scalar = a.scalar;
            z.i = a.valid ? (in->op == PLGPU_OP_IS_NAN ? isnan(a.f) : isfinite(a.f)) : 0;
            st[sp++] = z;
            break;
        default:
            return -1;
        }
    }
    if (sp != 1) return -1;
    if (is_dyn(&st[0])) st[0] = coerce(st[0], dyn_alone(&st[0]));
    *out = st[0];
    return 0;
}

/* Evaluate a program for all rows.  out_values: BOOL -> bit-packed bytes,
 * otherwise the result dtype's own width (Float32 as float);
 * out_validity bit-packed (always written).  Returns the output dtype or -1. */
OR_EXPORT int or_eval(const plgpu_column* cols, int32_t ncols, const plgpu_instr* prog, int32_t n,
                      int64_t nrows, void* out_values, uint8_t* out_validity) {
    (void)ncols;
    int dt = -1;
    for (int64_t r = 0; r < nrows; ++r) {
        val_t v;
        if (eval_row(cols, prog, n, r, &v) != 0) return -1;
        dt = v.dt;
        bit_set(out_validity, r, v.valid);
        switch (v.dt) {
        case PLGPU_BOOL: bit_set((uint8_t*)out_values, r, v.valid ? (int)v.i : 0); break;
        case PLGPU_I8: case PLGPU_U8: ((uint8_t*)out_values)[r] = (uint8_t)(v.valid ? v.i : 0); break;
        case PLGPU_I16: case PLGPU_U16: ((uint16_t*)out_values)[r] = (uint16_t)(v.valid ? v.i : 0); break;
        case PLGPU_I32: case PLGPU_U32: ((uint32_t*)out_values)[r] = (uint32_t)(v.valid ? v.i : 0); break;
        case PLGPU_I64: case PLGPU_U64: ((int64_t*)out_values)[r] = v.valid ? v.i : 0; break;
        case PLGPU_F32: ((float*)out_values)[r] = v.valid ? (float)v.f : 0.0f; break;
        default: ((double*)out_values)[r] = v.valid ? v.f : 0.0; break;
        }
    }
    return dt;
}

/* Filter mask from a program: null -> false (polars-compute/src/filter/mod.rs:21-27). */
static int eval_mask(const plgpu_column* cols, const plgpu_instr* prog, int n, int64_t r) {
    if (n <= 0) return 1;
    val_t v;
    if (eval_row(cols, prog, n, r, &v) != 0) return 0;
    return v.dt == PLGPU_BOOL && v.valid && v.i;
}

/* Filter one fixed-width column by a program-derived mask; stable order
 * (polars-compute/src/filter/primitive.rs filter_values_and_validity).
 * any fixed-width column; BOOL columns are not supported by this helper.
 * Returns the number of selected rows. */
OR_EXPORT int64_t or_filter(const plgpu_column* cols, int32_t ncols, const plgpu_instr* prog, int32_t n,
                            int64_t nrows, int32_t which, void* out_values, uint8_t* out_validity) {
    (void)ncols;
    const plgpu_column* c = &cols[which];
    int eb = bits_of(c->dtype) / 8;
    int64_t o = 0;
    for (int64_t r = 0; r < nrows; ++r) {
        if (!eval_mask(cols, prog, n, r)) continue;
        memcpy((char*)out_values + o * eb, (const char*)c->values + (c->offset + r) * eb, eb);
        if (out_validity) bit_set(out_validity, o, col_valid(c, r));
        ++o;
    }
    return o;
}

/* ---------------------------------------------------------- exact sum */
/* Shewchuk's exact-partials summation with a correctly rounded result (the
 * algorithm CPython's math.fsum publishes).  Used as the "exact" leg. */
typedef struct {
    double* p;
    int n, cap;
    double special; /* accumulates inf / nan IEEE-wise */
    int has_special;
} fsum_t;

static void fsum_init(fsum_t* s) { s->p = NULL; s->n = s->cap = 0; s->special = 0.0; s->has_special = 0; }
static void fsum_add(fsum_t* s, double x) {
    if (!isfinite(x)) { s->special += x; s->has_special = 1; return; }
    int i = 0;
    for (int j = 0; j < s->n; ++j) {
        double y = s->p[j];
        if (fabs(x) < fabs(y)) { double t = x; x = y; y = t; }
        double hi = x + y;
        double lo = y - (hi - x);
        if (lo != 0.0) s->p[i++] = lo;
        x = hi;
    }
    if (i + 1 > s->cap) { s->cap = s->cap ? s->cap * 2 : 8; s->p = (double*)realloc(s->p, sizeof(double) * s->cap); }
    s->p[i++] = x;
    s->n = i;
}
static double fsum_result(fsum_t* s) {
    if (s->has_special) return s->special;
    int n = s->n;
    double hi = 0.0, lo = 0.0;
    if (n > 0) {
        hi = s->p[--n];
        while (n > 0) {
            double x = hi, y = s->p[--n];
            hi = x + y;
            double yr = hi - x;
            lo = y - yr;
            if (lo != 0.0) break;
        }
        /* round-half-even correction across the remaining partials */
        if (n > 0 && ((lo < 0.0 && s->p[n - 1] < 0.0) || (lo > 0.0 && s->p[n - 1] > 0.0))) {
            double y = lo * 2.0;
            double x = hi + y;
            double yr = x - hi;
            if (y == yr) hi = x;
        }
    }
    return hi;
}
static void fsum_free(fsum_t* s) { free(s->p); }

/* The correctly rounded sum of finite x[0..n) when the partials above
 * overflow on the way (1.7e308 + 1.7e308 - 1.7e308: `math.fsum` raises
 * there): values of magnitude >= 2^-800 are summed scaled by 2^-128 (exact),
 * the others unscaled, and the two sets of exact partials are added back
 * together at scale; a partial that overflows there means the sum rounds
 * to +-inf. */
static double fsum_overflowing(const double* x, int64_t n) {
    fsum_t big, small, all;
    fsum_init(&big);
    fsum_init(&small);
    for (int64_t i = 0; i < n; ++i) {
        if (fabs(x[i]) >= 0x1p-800) fsum_add(&big, ldexp(x[i], -128));
        else fsum_add(&small, x[i]);
    }
    fsum_init(&all);
    double r = 0.0;
    int inf = 0;
    for (int j = 0; j < big.n && !inf; ++j) {
        const double y = ldexp(big.p[j], 128);
        if (isinf(y)) { r = y; inf = 1; }
        else fsum_add(&all, y);
    }
    for (int j = 0; j < small.n && !inf; ++j) fsum_add(&all, small.p[j]);
    if (!inf) {
        r = fsum_result(&all);
        /* overflow again: the partials' sum is beyond the largest double */
        if (isnan(r)) r = big.n ? copysign(INFINITY, big.p[big.n - 1]) : r;
    }
    fsum_free(&big);
    fsum_free(&small);
    fsum_free(&all);
    return r;
}

/* fsum of finite or special x[0..n), exact through intermediate overflow */
static double fsum_array(const double* x, int64_t n) {
    fsum_t s;
    fsum_init(&s);
    for (int64_t i = 0; i < n; ++i) fsum_add(&s, x[i]);
    double r = fsum_result(&s);
    const int special = s.has_special;
    fsum_free(&s);
    if (!special && !isfinite(r)) r = fsum_overflowing(x, n);
    return r;
}

/* ------------------------------------------------------------ group_by */
/* Row-order hash grouping (polars-core/src/frame/group_by/hashing.rs
 * group_by_threaded_slice / into_groups.rs): groups in order of first
 * occurrence, each group's rows ascending (GroupsIdx {first, all}).
 * Null keys form their own group. */
typedef struct {
    int64_t* keys;
    int64_t* gid;   /* slot -> group id */
    uint8_t* used;
    int64_t cap;
} imap_t;

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}
static void imap_init(imap_t* m, int64_t expect) {
    int64_t cap = 16;
    while (cap < 2 * expect + 16) cap <<= 1;
    m->cap = cap;
    m->keys = (int64_t*)malloc(sizeof(int64_t) * cap);
    m->gid = (int64_t*)malloc(sizeof(int64_t) * cap);
    m->used = (uint8_t*)calloc(cap, 1);
}
static void imap_free(imap_t* m) { free(m->keys); free(m->gid); free(m->used); }
/* returns group id, inserting new_gid if absent */
static int64_t imap_get_or_insert(imap_t* m, int64_t key, int64_t new_gid, int* inserted) {
    uint64_t h = mix64((uint64_t)key) & (uint64_t)(m->cap - 1);
    for (;;) {
        if (!m->used[h]) { m->used[h] = 1; m->keys[h] = key; m->gid[h] = new_gid; *inserted = 1; return new_gid; }
        if (m->keys[h] == key) { *inserted = 0; return m->gid[h]; }
        h = (h + 1) & (uint64_t)(m->cap - 1);
    }
}

typedef struct {
    int64_t ngroups;
    int64_t* first;    /* first row of each group                        */
    int64_t* key;      /* key value                                      */
    uint8_t* key_null; /* 1 if the null group                            */
    int64_t* start;    /* CSR offsets into rows[]                        */
    int64_t* rows;     /* member rows in ascending order                 */
} groups_t;

static void build_groups(const plgpu_column* key, const plgpu_column* cols, const plgpu_instr* prog, int n,
                         int64_t nrows, groups_t* g) {
    imap_t m;
    imap_init(&m, nrows < 1024 ? nrows : 1024);
    int64_t cap = 64, ng = 0, null_gid = -1;
    int64_t* gid_of_row = (int64_t*)malloc(sizeof(int64_t) * (nrows ? nrows : 1));
    g->first = (int64_t*)malloc(sizeof(int64_t) * cap);
    g->key = (int64_t*)malloc(sizeof(int64_t) * cap);
    g->key_null = (uint8_t*)malloc(cap);
    int64_t* cnt = (int64_t*)calloc(cap, sizeof(int64_t));
    for (int64_t r = 0; r < nrows; ++r) {
        gid_of_row[r] = -1;
        if (!eval_mask(cols, prog, n, r)) continue;
        val_t k = col_get(key, r);
        int64_t gi;
        int ins = 0;
        if (!k.valid) {
            if (null_gid < 0) { null_gid = ng; ins = 1; }
            gi = null_gid;
        } else {
            if (m.cap < 2 * (ng + 1)) {
                /* grow */
                imap_t m2;
                imap_init(&m2, 2 * m.cap);
                for (int64_t s = 0; s < m.cap; ++s)
                    if (m.used[s]) { int d; imap_get_or_insert(&m2, m.keys[s], m.gid[s], &d); }
                imap_free(&m);
                m = m2;
            }
            gi = imap_get_or_insert(&m, k.i, ng, &ins);
        }
        if (ins) {
            if (ng == cap) {
                cap *= 2;
                g->first = (int64_t*)realloc(g->first, sizeof(int64_t) * cap);
                g->key = (int64_t*)realloc(g->key, sizeof(int64_t) * cap);
                g->key_null = (uint8_t*)realloc(g->key_null, cap);
                cnt = (int64_t*)realloc(cnt, sizeof(int64_t) * cap);
            }
            g->first[ng] = r;
            g->key[ng] = k.valid ? k.i : 0;
            g->key_null[ng] = !k.valid;
            cnt[ng] = 0;
            ++ng;
        }
        cnt[gi]++;
        gid_of_row[r] = gi;
    }
    g->ngroups = ng;
    g->start = (int64_t*)malloc(sizeof(int64_t) * (ng + 1));
    g->start[0] = 0;
    for (int64_t i = 0; i < ng; ++i) g->start[i + 1] = g->start[i] + cnt[i];
    g->rows = (int64_t*)malloc(sizeof(int64_t) * (g->start[ng] ? g->start[ng] : 1));
    for (int64_t i = 0; i < ng; ++i) cnt[i] = g->start[i];
    for (int64_t r = 0; r < nrows; ++r)
        if (gid_of_row[r] >= 0) g->rows[cnt[gid_of_row[r]]++] = r;
    free(cnt);
    free(gid_of_row);
    imap_free(&m);
}
static void free_groups(groups_t* g) {
    free(g->first); free(g->key); free(g->key_null); free(g->start); free(g->rows);
}

/* sum_mode for f64 SUM / MEAN:
 *   0 = KahanSum in row order   (polars-core .../aggregations/mod.rs:581-610,
 *                                polars-utils/src/kahan_sum.rs)
 *   1 = naive `+=` in row order  (polars-expr/src/reduce/sum.rs:103-110, one thread)
 *   2 = exact, correctly rounded (what the GPU path computes)             */
static double f64_sum_group(const plgpu_column* c, const int64_t* rows, int64_t len, int mode, int64_t* nvalid) {
    int64_t nv = 0;
    if (mode == 0 && len == 1) {
        /* agg_sum: `idx.len() == 1 => arr.get(first).unwrap_or(0)` (:590);
         * the streaming fold (modes 1, 2) starts from +0.0 instead. */
        val_t v = col_get(c, rows[0]);
        *nvalid = v.valid;
        return v.valid ? v.f : 0.0;
    }
    if (mode == 0) {
        double sum = 0.0, err = 0.0;
        for (int64_t i = 0; i < len; ++i) {
            val_t v = col_get(c, rows[i]);
            if (!v.valid) continue;
            ++nv;
            double x = v.f;
            if (isfinite(x)) {
                double y = x - err;
                double t = sum + y;
                err = (t - sum) - y;
                sum = t;
            } else {
                sum += x;
            }
        }
        *nvalid = nv;
        return sum;
    } else if (mode == 1) {
        double sum = 0.0;
        for (int64_t i = 0; i < len; ++i) {
            val_t v = col_get(c, rows[i]);
            if (!v.valid) continue;
            ++nv;
            sum += v.f;
        }
        *nvalid = nv;
        return sum;
    } else {
        double* buf = (double*)malloc(sizeof(double) * (size_t)(len > 0 ? len : 1));
        for (int64_t i = 0; i < len; ++i) {
            val_t v = col_get(c, rows[i]);
            if (!v.valid) continue;
            buf[nv++] = v.f;
        }
        double r = fsum_array(buf, nv);
        free(buf);
        *nvalid = nv;
        return r + 0.0; /* exact zero -> +0.0, as the fold from +0.0 gives */
    }
}

/* Group-by with aggregations, groups in first-occurrence order
 * (maintain_order=True).  For each agg a: out_vals[a] is int64_t[] for I64
 * results, uint32_t[] for COUNT/LEN, double[] otherwise; out_valid[a] is a
 * byte-per-group validity array.  Returns the number of groups, or -1. */
OR_EXPORT int64_t or_group_by_agg(const plgpu_column* key, const plgpu_column* cols, int32_t ncols,
                                  const plgpu_instr* prog, int32_t n, const plgpu_agg* aggs, int32_t naggs,
                                  int64_t nrows, int32_t sum_mode, int64_t max_groups, int64_t* out_keys,
                                  uint8_t* out_key_valid, void** out_vals, uint8_t** out_valid) {
    (void)ncols;
    groups_t g;
    build_groups(key, cols, prog, n, nrows, &g);
    if (g.ngroups > max_groups) { free_groups(&g); return -1; }
    for (int64_t gi = 0; gi < g.ngroups; ++gi) {
        out_keys[gi] = g.key[gi];
        out_key_valid[gi] = !g.key_null[gi];
        const int64_t* rows = g.rows + g.start[gi];
        int64_t len = g.start[gi + 1] - g.start[gi];
        for (int a = 0; a < naggs; ++a) {
            const plgpu_column* c = &cols[aggs[a].col];
            int isf = c->dtype == PLGPU_F64 || c->dtype == PLGPU_F32;  /* Float32 widened exactly */
            int isu64 = c->dtype == PLGPU_U64;
            uint8_t valid = 1;
            switch (aggs[a].kind) {
            case PLGPU_AGG_LEN: ((uint32_t*)out_vals[a])[gi] = (uint32_t)len; break;
            case PLGPU_AGG_COUNT: {
                uint32_t nv = 0;
                for (int64_t i = 0; i < len; ++i) nv += col_valid(c, rows[i]);
                ((uint32_t*)out_vals[a])[gi] = nv;
                break;
            }
            case PLGPU_AGG_SUM:
                if (isf) {
                    int64_t nv;
                    ((double*)out_vals[a])[gi] = f64_sum_group(c, rows, len, sum_mode, &nv);
                } else {
                    /* integer sum wraps (Rust release arithmetic) */
                    uint64_t s = 0;
                    for (int64_t i = 0; i < len; ++i) {
                        val_t v = col_get(c, rows[i]);
                        if (v.valid) s += (uint64_t)v.i;
                    }
                    ((int64_t*)out_vals[a])[gi] = (int64_t)s;
                }
                break;
            case PLGPU_AGG_MEAN: {
                /* agg_mean (mod.rs:659-700): sum / non-null count, null if 0 */
                int64_t nv = 0;
                double s;
                if (isf) {
                    s = f64_sum_group(c, rows, len, sum_mode, &nv);
                } else {
                    fsum_t fs;
                    fsum_init(&fs);
                    double ks = 0.0, ke = 0.0;
                    for (int64_t i = 0; i < len; ++i) {
                        val_t v = col_get(c, rows[i]);
                        if (!v.valid) continue;
                        ++nv;
                        double x = isu64 ? (double)(uint64_t)v.i : (double)v.i;
                        if (sum_mode == 2) fsum_add(&fs, x);
                        else { double y = x - ke; double t = ks + y; ke = (t - ks) - y; ks = t; }
                    }
                    s = sum_mode == 2 ? fsum_result(&fs) : ks;
                    fsum_free(&fs);
                }
                if (nv == 0) { valid = 0; ((double*)out_vals[a])[gi] = 0.0; }
                else ((double*)out_vals[a])[gi] = s / (double)nv;
                break;
            }
            case PLGPU_AGG_MIN: case PLGPU_AGG_MAX: {
                /* min_ignore_nan / max_ignore_nan (polars-utils/src/min_max.rs:91-98,
                 * polars-expr/src/reduce/min_max.rs:100-130): NaN only if every
                 * valid value is NaN; null if no valid value. */
                int is_min = aggs[a].kind == PLGPU_AGG_MIN;
                int any = 0, any_num = 0;
                double bf = 0.0;
                int64_t bi = 0;
                for (int64_t i = 0; i < len; ++i) {
                    val_t v = col_get(c, rows[i]);
                    if (!v.valid) continue;
                    any = 1;
                    if (isf) {
                        if (isnan(v.f)) continue;
                        if (!any_num) bf = v.f;
                        else if (is_min ? (v.f < bf || (v.f == bf && signbit(v.f))) : (v.f > bf || (v.f == bf && !signbit(v.f)))) bf = v.f;
                        any_num = 1;
                    } else {
                        int less = isu64 ? (uint64_t)v.i < (uint64_t)bi : v.i < bi;
                        int more = isu64 ? (uint64_t)v.i > (uint64_t)bi : v.i > bi;
                        if (!any_num || (is_min ? less : more)) bi = v.i;
                        any_num = 1;
                    }
                }
                if (!any) valid = 0;
                if (isf) ((double*)out_vals[a])[gi] = any_num ? bf : (any ? NAN : 0.0);
                else ((int64_t*)out_vals[a])[gi] = bi;
                break;
            }
            case PLGPU_AGG_FIRST: case PLGPU_AGG_LAST: {
                /* polars-expr/src/reduce/first_last.rs First / Last: the value
                 * of the group's first / last row, null included */
                val_t v = col_get(c, rows[aggs[a].kind == PLGPU_AGG_FIRST ? 0 : len - 1]);
                valid = (uint8_t)v.valid;
                if (isf) ((double*)out_vals[a])[gi] = v.valid ? v.f : 0.0;
                else ((int64_t*)out_vals[a])[gi] = v.valid ? v.i : 0;
                break;
            }
            default:
                free_groups(&g);
                return -1;
            }
            out_valid[a][gi] = valid;
        }
    }
    int64_t ng = g.ngroups;
    free_groups(&g);
    return ng;
}

/* Exact, correctly rounded sum of a plain f64 array (pinned to math.fsum
 * in tests/test_oracle.py). */
OR_EXPORT double or_fsum(const double* x, int64_t n) { return fsum_array(x, n); }

/* ------------------------------------------------------ CPU baseline */
/* The bench's cpu_baseline leg: `filter(col(p) > k).group_by(key).agg(
 * [col(c).sum() for c in sums])` over no-null columns, restating the
 * streaming engine's partitioned hash aggregation (polars-stream group_by
 * + polars-expr/src/reduce/sum.rs): each thread folds a contiguous morsel
 * into a private hash table with naive `+=`, then tables are combined
 * (combine_subset).  Returns the number of groups; out_sum_of_sums is a
 * checksum (sum over groups and columns) so the work is not elided. */
#ifdef _OPENMP
#include <omp.h>
#endif
OR_EXPORT int64_t or_baseline_filter_groupby_sum(const int64_t* key, const double* pred, double k,
                                                 const double* const* sums, int32_t nsums, int64_t nrows,
                                                 int32_t threads, double* out_sum_of_sums) {
    int T = threads > 0 ? threads : 1;
    typedef struct { imap_t m; double* acc; int64_t ng, cap; int64_t* keys; } part_t;
    part_t* parts = (part_t*)calloc(T, sizeof(part_t));
#pragma omp parallel num_threads(T)
    {
#ifdef _OPENMP
        int t = omp_get_thread_num();
#else
        int t = 0;
#endif
        part_t* p = &parts[t];
        imap_init(&p->m, 4096);
        p->cap = 4096;
        p->acc = (double*)calloc((size_t)p->cap * nsums, sizeof(double));
        p->keys = (int64_t*)malloc(sizeof(int64_t) * p->cap);
        int64_t lo = nrows * t / T, hi = nrows * (t + 1) / T;
        for (int64_t r = lo; r < hi; ++r) {
            double x = pred[r];
            if (!(isnan(x) || x > k)) continue; /* tot_gt(x, k) with k not NaN */
            if (p->m.cap < 2 * (p->ng + 1)) {
                imap_t m2;
                imap_init(&m2, 2 * p->m.cap);
                for (int64_t s = 0; s < p->m.cap; ++s)
                    if (p->m.used[s]) { int d; imap_get_or_insert(&m2, p->m.keys[s], p->m.gid[s], &d); }
                imap_free(&p->m);
                p->m = m2;
            }
            int ins;
            int64_t gi = imap_get_or_insert(&p->m, key[r], p->ng, &ins);
            if (ins) {
                if (p->ng == p->cap) {
                    p->cap *= 2;
                    p->acc = (double*)realloc(p->acc, sizeof(double) * p->cap * nsums);
                    p->keys = (int64_t*)realloc(p->keys, sizeof(int64_t) * p->cap);
                }
                memset(p->acc + p->ng * nsums, 0, sizeof(double) * nsums);
                p->keys[p->ng] = key[r];
                p->ng++;
            }
            double* a = p->acc + gi * nsums;
            for (int c = 0; c < nsums; ++c) a[c] += sums[c][r];
        }
    }
    /* combine partials into thread 0's table */
    part_t* d = &parts[0];
    for (int t = 1; t < T; ++t) {
        part_t* p = &parts[t];
        for (int64_t i = 0; i < p->ng; ++i) {
            if (d->m.cap < 2 * (d->ng + 1)) {
                imap_t m2;
                imap_init(&m2, 2 * d->m.cap);
                for (int64_t s = 0; s < d->m.cap; ++s)
                    if (d->m.used[s]) { int dd; imap_get_or_insert(&m2, d->m.keys[s], d->m.gid[s], &dd); }
                imap_free(&d->m);
                d->m = m2;
            }
            int ins;
            int64_t gi = imap_get_or_insert(&d->m, p->keys[i], d->ng, &ins);
            if (ins) {
                if (d->ng == d->cap) {
                    d->cap *= 2;
                    d->acc = (double*)realloc(d->acc, sizeof(double) * d->cap * nsums);
                    d->keys = (int64_t*)realloc(d->keys, sizeof(int64_t) * d->cap);
                }
                memset(d->acc + d->ng * nsums, 0, sizeof(double) * nsums);
                d->keys[d->ng] = p->keys[i];
                d->ng++;
            }
            for (int c = 0; c < nsums; ++c) d->acc[gi * nsums + c] += p->acc[i * nsums + c];
        }
    }
    double chk = 0.0;
    for (int64_t i = 0; i < d->ng * nsums; ++i) chk += d->acc[i];
    *out_sum_of_sums = chk;
    int64_t ng = d->ng;
    for (int t = 0; t < T; ++t) { imap_free(&parts[t].m); free(parts[t].acc); free(parts[t].keys); }
    free(parts);
    return ng;
}

/* ------------------------------------------------------------ hash join
 * polars-ops/src/frame/join/hash_join/single_keys_inner.rs:45
 * hash_join_tuples_inner: a hash table key -> IdxVec of build rows (rows in
 * insertion = row order; null keys inserted only when nulls_equal,
 * single_keys.rs build_tables), then every probe row in order looks its key
 * up (probe_inner, :11) and emits (probe_idx, build_idx) for each build row.
 * Restated with the right side as the build side and the left side probed
 * in order, i.e. the pairs in (left, right) order ("left_right"); the
 * reference's other orders are permutations of the same pairs.
 * The "hash table" is a (key, row) array sorted by key then row. */
typedef struct {
    int64_t key;
    int64_t row;
    int is_null;
} jn_item;

static int jn_cmp(const void* a, const void* b) {
    const jn_item* x = (const jn_item*)a;
    const jn_item* y = (const jn_item*)b;
    if (x->is_null != y->is_null) return x->is_null < y->is_null ? -1 : 1;
    if (!x->is_null && x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->row < y->row ? -1 : (x->row > y->row ? 1 : 0);
}

static int64_t col_int(const plgpu_column* c, int64_t r) { return col_get(c, r).i; }  /* UInt64 as its bits */

/* Returns the number of pairs (or -1 if more than cap). */
OR_EXPORT int64_t or_join_inner(const plgpu_column* lk, const plgpu_column* rk, int32_t nulls_equal, int64_t cap,
                                int64_t* out_l, int64_t* out_r) {
    const int64_t nr = rk->length, nl = lk->length;
    jn_item* t = (jn_item*)malloc(sizeof(jn_item) * (size_t)(nr > 0 ? nr : 1));
    int64_t m = 0;
    for (int64_t r = 0; r < nr; ++r) {
        const int v = col_valid(rk, r);
        if (!v && !nulls_equal) continue;
        t[m].is_null = !v;
        t[m].key = v ? col_int(rk, r) : 0;
        t[m].row = r;
        ++m;
    }
    qsort(t, (size_t)m, sizeof(jn_item), jn_cmp);
    int64_t n = 0;
    for (int64_t l = 0; l < nl; ++l) {
        const int v = col_valid(lk, l);
        if (!v && !nulls_equal) continue;
        jn_item q;
        q.is_null = !v;
        q.key = v ? col_int(lk, l) : 0;
        q.row = -1;
        /* first item >= (key, -1) */
        int64_t lo = 0, hi = m;
        while (lo < hi) {
            const int64_t mid = (lo + hi) / 2;
            if (jn_cmp(&t[mid], &q) < 0) lo = mid + 1;
            else hi = mid;
        }
        for (int64_t i = lo; i < m && t[i].is_null == q.is_null && (q.is_null || t[i].key == q.key); ++i) {
            if (n >= cap) {
                free(t);
                return -1;
            }
            out_l[n] = l;
            out_r[n] = t[i].row;
            ++n;
        }
    }
    free(t);
    return n;
}

/* ------------------------------------------------------- other join types
 * The same build (right side, key -> rows in row order) probed by every left
 * row in order; how:
 *   1 left   single_keys_left.rs:106 hash_join_tuples_left: each left row's
 *            matches in right-row order, or (l, null) when it has none;
 *   3 full   single_keys_outer.rs:101 probe_outer: the left join's pairs,
 *            then every right row that no left row matched as (null, r)
 *            (null right keys among them unless nulls_equal) -- the
 *            reference drains these in hash-table order, restated here in
 *            right-row order;
 *   4 semi / 5 anti  single_keys_semi_anti.rs:111 / :95: the left rows with
 *            / without a match, in left-row order (out_r unused).
 * (paths under polars-ops/src/frame/join/hash_join/).  -1 is a null index.
 * The right join and the maintain_order permutations are restated in
 * oracle.py on top of these sequences.  Returns the number of rows, or -1
 * if more than cap. */
OR_EXPORT int64_t or_join(const plgpu_column* lk, const plgpu_column* rk, int32_t how, int32_t nulls_equal,
                          int64_t cap, int64_t* out_l, int64_t* out_r) {
    const int64_t nr = rk->length, nl = lk->length;
    jn_item* t = (jn_item*)malloc(sizeof(jn_item) * (size_t)(nr > 0 ? nr : 1));
    char* hit = (char*)calloc((size_t)(nr > 0 ? nr : 1), 1);
    int64_t m = 0, n = 0;
    for (int64_t r = 0; r < nr; ++r) {
        const int v = col_valid(rk, r);
        if (!v && !nulls_equal) continue;
        t[m].is_null = !v;
        t[m].key = v ? col_int(rk, r) : 0;
        t[m].row = r;
        ++m;
    }
    qsort(t, (size_t)m, sizeof(jn_item), jn_cmp);
#define OR_PUSH(a, b)                    \
    do {                                 \
        if (n >= cap) goto overflow;     \
        out_l[n] = (a);                  \
        if (out_r) out_r[n] = (b);       \
        ++n;                             \
    } while (0)
    for (int64_t l = 0; l < nl; ++l) {
        const int v = col_valid(lk, l);
        int64_t lo = m, hi = m;
        if (v || nulls_equal) {
            jn_item q;
            q.is_null = !v;
            q.key = v ? col_int(lk, l) : 0;
            q.row = -1;
            int64_t a = 0, b = m;
            while (a < b) {
                const int64_t mid = (a + b) / 2;
                if (jn_cmp(&t[mid], &q) < 0) a = mid + 1;
                else b = mid;
            }
            lo = hi = a;
            while (hi < m && t[hi].is_null == q.is_null && (q.is_null || t[hi].key == q.key)) ++hi;
        }
        if (how == 4 || how == 5) {
            if ((hi > lo) == (how == 4)) OR_PUSH(l, -1);
            continue;
        }
        if (hi == lo) {
            OR_PUSH(l, -1);
            continue;
        }
        for (int64_t i = lo; i < hi; ++i) {
            OR_PUSH(l, t[i].row);
            hit[t[i].row] = 1;
        }
    }
    if (how == 3)
        for (int64_t r = 0; r < nr; ++r)
            if (!hit[r]) OR_PUSH(-1, r);
#undef OR_PUSH
    free(t);
    free(hit);
    return n;
overflow:
    free(t);
    free(hit);
    return -1;
}

/* ------------------------------------------------------------------ sort
 * polars-core/src/chunked_array/ops/sort/arg_sort.rs:7 sort_impl: a stable
 * sort of (idx, value) pairs by TotalOrd (total_ord.rs: NaN == NaN and
 * greatest, -0.0 == 0.0); descending reverses the comparator (equal values
 * keep their order); nulls are placed first, or last with nulls_last, in row
 * order.  Restated as a comparison sort with the row index as tie-break. */
typedef struct {
    const plgpu_column* c;
    int descending;
} srt_ctx;
static srt_ctx g_srt;

static int srt_cmp_val(int64_t a, int64_t b) {
    const plgpu_column* c = g_srt.c;
    if (c->dtype == PLGPU_F64 || c->dtype == PLGPU_F32) {
        const double x = col_get(c, a).f, y = col_get(c, b).f;
        const int xn = isnan(x), yn = isnan(y);
        if (xn || yn) return xn == yn ? 0 : (xn ? 1 : -1);
        return x < y ? -1 : (x > y ? 1 : 0); /* -0.0 == 0.0 */
    }
    const int64_t x = col_int(c, a), y = col_int(c, b);
    if (c->dtype == PLGPU_U64) return (uint64_t)x < (uint64_t)y ? -1 : ((uint64_t)x > (uint64_t)y ? 1 : 0);
    return x < y ? -1 : (x > y ? 1 : 0);
}

static int srt_cmp(const void* pa, const void* pb) {
    const int64_t a = *(const int64_t*)pa, b = *(const int64_t*)pb;
    int r = srt_cmp_val(a, b);
    if (g_srt.descending) r = -r;
    if (r) return r;
    return a < b ? -1 : (a > b ? 1 : 0);
}

OR_EXPORT void or_arg_sort(const plgpu_column* c, int32_t descending, int32_t nulls_last, int64_t* out) {
    const int64_t n = c->length;
    int64_t* v = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    int64_t nv = 0, nn = 0;
    for (int64_t r = 0; r < n; ++r)
        if (col_valid(c, r)) v[nv++] = r;
    g_srt.c = c;
    g_srt.descending = descending;
    qsort(v, (size_t)nv, sizeof(int64_t), srt_cmp);
    nn = n - nv;
    int64_t* dv = nulls_last ? out : out + nn;
    int64_t* dn = nulls_last ? out + nv : out;
    memcpy(dv, v, sizeof(int64_t) * (size_t)nv);
    int64_t k = 0;
    for (int64_t r = 0; r < n; ++r)
        if (!col_valid(c, r)) dn[k++] = r;
    free(v);
}

/* --------------------------------------------------------------- rolling
 * polars-compute/src/rolling/sum.rs:7 SumWindow: Kahan add of values
 * entering the window (err_add) and Kahan subtract of values leaving it
 * (err_sub), non-finite values counted apart (finalize: only +inf -> +inf,
 * only -inf -> -inf, else NaN); update() resets when the new window does not
 * overlap the last one.  mean.rs:6 MeanWindow: sum / (len - null_count).
 * Drivers: no_nulls/mod.rs:43 (windows shorter than min_periods are skipped
 * without updating) and nulls/mod.rs:38 (every window updated, valid iff
 * non-null count >= min_periods); bounds mod.rs:68 det_offsets / :71
 * det_offsets_center.  mode 0 restates that arithmetic exactly; mode 1 is
 * the exact window sum (math.fsum of the finite values) used to pin the GPU
 * bit for bit. */
typedef struct {
    double sum, err_add, err_sub;
    int64_t isum;
    int64_t nonfinite, pinf, ninf, null_count, last_start, last_end;
} sw_t;

static void sw_reset(sw_t* w) {
    w->sum = w->err_add = w->err_sub = 0.0;
    w->isum = 0;
    w->nonfinite = w->pinf = w->ninf = w->null_count = 0;
}

static double rl_val(const plgpu_column* c, int64_t r) {
    if (c->dtype == PLGPU_F64) return ((const double*)c->values)[c->offset + r];
    return (double)col_int(c, r);
}

static void sw_add(sw_t* w, const plgpu_column* c, int64_t r, int isint) {
    if (isint) {
        w->isum = (int64_t)((uint64_t)w->isum + (uint64_t)col_int(c, r));
        return;
    }
    const double v = rl_val(c, r);
    if (isfinite(v)) {
        const double y = v - w->err_add;
        const double ns = w->sum + y;
        w->err_add = (ns - w->sum) - y;
        w->sum = ns;
    } else {
        w->nonfinite += 1;
        w->pinf += v > 0.0;
        w->ninf += v < 0.0;
    }
}

static void sw_sub(sw_t* w, const plgpu_column* c, int64_t r, int isint) {
    if (isint) {
        w->isum = (int64_t)((uint64_t)w->isum - (uint64_t)col_int(c, r));
        return;
    }
    const double v = rl_val(c, r);
    if (isfinite(v)) {
        const double val = 0.0 - v;
        const double y = val - w->err_sub;
        const double ns = w->sum + y;
        w->err_sub = (ns - w->sum) - y;
        w->sum = ns;
    } else {
        w->nonfinite -= 1;
        w->pinf -= v > 0.0;
        w->ninf -= v < 0.0;
    }
}

static double sw_update(sw_t* w, const plgpu_column* c, int64_t s, int64_t e, int isint) {
    if (s >= w->last_end) {
        sw_reset(w);
        w->last_start = s;
        w->last_end = s;
    }
    for (int64_t r = w->last_start; r < s; ++r) {
        if (col_valid(c, r)) sw_sub(w, c, r, isint);
        else w->null_count -= 1;
    }
    for (int64_t r = w->last_end; r < e; ++r) {
        if (col_valid(c, r)) sw_add(w, c, r, isint);
        else w->null_count += 1;
    }
    w->last_start = s;
    w->last_end = e;
    if (w->nonfinite == 0) return w->sum;
    if (w->nonfinite == w->pinf) return INFINITY;
    if (w->nonfinite == w->ninf) return -INFINITY;
    return NAN;
}

static void rl_offsets(int64_t i, int64_t ws, int64_t n, int center, int64_t* s, int64_t* e) {
    if (center) {
        const int64_t right = (ws + 1) / 2;
        const int64_t left = ws - right;
        *s = i > left ? i - left : 0;
        *e = i + right < n ? i + right : n;
    } else {
        *s = i + 1 > ws ? i + 1 - ws : 0;
        *e = i + 1;
    }
}

/* Rolling min / max (kind 3 / 4): polars-compute/src/rolling/{no_nulls,
 * nulls}/min_max.rs MinMaxWindow with MinPropagateNan / MaxPropagateNan
 * (polars-utils/src/min_max.rs:144,168): a NaN in the window makes the
 * result NaN; nulls are skipped; the result is null when the window holds
 * fewer than min_periods values (the window length when there are no nulls)
 * or no value at all.  Restated as a direct scan of each window. */
static void or_rolling_minmax(const plgpu_column* c, int32_t kind, int64_t ws, int64_t min_periods, int32_t center,
                              double* out_f64, int64_t* out_i64, uint8_t* out_valid) {
    const int64_t n = c->length;
    const int isf = c->dtype == PLGPU_F64;
    for (int64_t i = 0; i < n; ++i) {
        int64_t s, e;
        rl_offsets(i, ws, n, center, &s, &e);
        int64_t nn = 0;
        int nan = 0;
        double bf = 0.0;
        int64_t bi = 0;
        for (int64_t r = s; r < e; ++r) {
            if (!col_valid(c, r)) continue;
            if (isf) {
                const double x = rl_val(c, r);
                if (isnan(x)) nan = 1;
                else if (nn == 0 || (kind == 3 ? x < bf : x > bf)) bf = x;
            } else {
                const int64_t x = col_int(c, r);
                if (nn == 0 || (kind == 3 ? x < bi : x > bi)) bi = x;
            }
            ++nn;
        }
        const int valid = nn >= min_periods && nn > 0;
        out_valid[i] = (uint8_t)valid;
        if (isf) out_f64[i] = valid ? (nan ? NAN : bf) : 0.0;
        else out_i64[i] = valid ? bi : 0;
    }
}

/* kind 1 sum / 2 mean / 3 min / 4 max; out_f64 or out_i64 (integer sums,
 * integer min / max); out_valid bytes. */
OR_EXPORT void or_rolling(const plgpu_column* c, int32_t kind, int64_t ws, int64_t min_periods, int32_t center,
                          int32_t mode, double* out_f64, int64_t* out_i64, uint8_t* out_valid) {
    if (kind == 3 || kind == 4) {
        or_rolling_minmax(c, kind, ws, min_periods, center, out_f64, out_i64, out_valid);
        return;
    }
    const int64_t n = c->length;
    const int isint = kind == 1 && c->dtype != PLGPU_F64;
    int has_nulls = 0;
    for (int64_t r = 0; r < n && !has_nulls; ++r) has_nulls = !col_valid(c, r);
    sw_t w;
    memset(&w, 0, sizeof w);
    for (int64_t i = 0; i < n; ++i) {
        int64_t s, e;
        rl_offsets(i, ws, n, center, &s, &e);
        double v = 0.0;
        int valid;
        int64_t nn = 0;
        if (mode == 0) {
            if (!has_nulls && e - s < min_periods) {
                out_valid[i] = 0;
                if (isint) out_i64[i] = 0;
                else out_f64[i] = 0.0;
                continue;
            }
            v = sw_update(&w, c, s, e, isint);
            nn = (e - s) - w.null_count;
            valid = nn >= min_periods;
        } else {
            /* exact: fsum of the finite non-null values, specials by count */
            double* buf = (double*)malloc(sizeof(double) * (size_t)(e - s > 0 ? e - s : 1));
            int64_t m = 0, pinf = 0, ninf = 0, nan = 0;
            uint64_t isum = 0;
            for (int64_t r = s; r < e; ++r) {
                if (!col_valid(c, r)) continue;
                ++nn;
                if (isint) {
                    isum += (uint64_t)col_int(c, r);
                    continue;
                }
                const double x = rl_val(c, r);
                if (isnan(x)) ++nan;
                else if (isinf(x)) (x > 0 ? ++pinf : ++ninf);
                else buf[m++] = x;
            }
            v = or_fsum(buf, m);
            /* SumWindow starts from S::zeroed() = +0.0 (rolling/sum.rs:31), so
             * a window whose values cancel (or are all -0.0) sums to +0.0 */
            if (v == 0.0) v = 0.0;
            free(buf);
            if (nan || (pinf && ninf)) v = NAN;
            else if (pinf) v = INFINITY;
            else if (ninf) v = -INFINITY;
            w.isum = (int64_t)isum;
            valid = nn >= min_periods && e > s;
        }
        if (kind == 2) {
            if (nn == 0) valid = 0;
            else v = v / (double)nn;
        }
        out_valid[i] = (uint8_t)valid;
        /* SumWindow<i32, i32> wraps in 32 bits */
        if (isint && c->dtype == PLGPU_I32) w.isum = (int64_t)(int32_t)(uint32_t)(uint64_t)w.isum;
        if (isint) out_i64[i] = valid ? w.isum : 0;
        else out_f64[i] = valid ? v : 0.0;
    }
}

/* ------------------------------------------- CPU baselines: sort, join
 * The bench's cpu_baseline legs for configs[2] and configs[3] (TEST
 * INFRASTRUCTURE: timed beside the GPU, never the product).  Both use every
 * thread they are given, as the reference's rayon POOL does. */

/* configs[2]: `df.sort("ts")` over ncols 8-byte columns, then
 * rolling_mean(ws) of column `roll`.
 *  - arg_sort: polars-core/src/chunked_array/ops/sort/arg_sort.rs:82
 *    arg_sort_no_nulls collects (row, value) pairs and sorts them with
 *    sort_by_branch -> par_sort_by (a parallel stable merge sort).  Restated:
 *    T contiguous runs sorted in parallel (qsort with the row id as the tie
 *    break, i.e. stable), then pairwise merge rounds, each round's merges in
 *    parallel;
 *  - the frame gather: DataFrame::take_unchecked, one take per column, the
 *    columns in parallel (POOL.install over the columns);
 *  - rolling_mean: rolling/no_nulls/mod.rs:43 rolling_apply_agg_window with
 *    mean.rs MeanWindow over sum.rs:7 SumWindow (Kahan add / sub), one
 *    thread (a rolling kernel runs per chunk, sequentially).
 * Returns a checksum of the rolling output so nothing is elided. */
typedef struct { int64_t v; int64_t r; } bl_pair;

static int bl_pair_cmp(const void* a, const void* b) {
    const bl_pair* x = (const bl_pair*)a;
    const bl_pair* y = (const bl_pair*)b;
    if (x->v != y->v) return x->v < y->v ? -1 : 1;
    return x->r < y->r ? -1 : (x->r > y->r ? 1 : 0);
}

static void bl_merge(const bl_pair* a, int64_t na, const bl_pair* b, int64_t nb, bl_pair* out) {
    int64_t i = 0, j = 0, k = 0;
    while (i < na && j < nb) out[k++] = bl_pair_cmp(&b[j], &a[i]) < 0 ? b[j++] : a[i++];
    while (i < na) out[k++] = a[i++];
    while (j < nb) out[k++] = b[j++];
}

OR_EXPORT double or_baseline_sort_rolling(const int64_t* key, const uint64_t* const* cols, int32_t ncols,
                                          int32_t roll, int64_t n, int64_t ws, int32_t threads,
                                          uint64_t* const* out_cols, double* out_roll) {
    int T = threads > 0 ? threads : 1;
    bl_pair* p = (bl_pair*)malloc(sizeof(bl_pair) * (size_t)(n > 0 ? n : 1));
    bl_pair* q = (bl_pair*)malloc(sizeof(bl_pair) * (size_t)(n > 0 ? n : 1));
    int R = 1;
    while (R < T) R <<= 1; /* runs: a power of two >= T */
#pragma omp parallel for num_threads(T) schedule(static)
    for (int t = 0; t < R; ++t) {
        const int64_t lo = n * t / R, hi = n * (t + 1) / R;
        for (int64_t r = lo; r < hi; ++r) { p[r].v = key[r]; p[r].r = r; }
        qsort(p + lo, (size_t)(hi - lo), sizeof(bl_pair), bl_pair_cmp);
    }
    for (int width = 1; width < R; width <<= 1) {
#pragma omp parallel for num_threads(T) schedule(dynamic, 1)
        for (int t = 0; t < R; t += 2 * width) {
            const int64_t lo = n * t / R, mid = n * (t + width) / R, hi = n * (t + 2 * width) / R;
            bl_merge(p + lo, mid - lo, p + mid, hi - mid, q + lo);
        }
        bl_pair* tmp = p; p = q; q = tmp;
    }
#pragma omp parallel for num_threads(T) schedule(static) collapse(2)
    for (int c = 0; c < ncols; ++c)
        for (int t = 0; t < T; ++t) {
            const int64_t lo = n * t / T, hi = n * (t + 1) / T;
            const uint64_t* src = cols[c];
            uint64_t* dst = out_cols[c];
            for (int64_t i = lo; i < hi; ++i) dst[i] = src[p[i].r];
        }
    /* rolling_mean(ws), min_periods = ws: the first ws - 1 outputs are null */
    const double* x = (const double*)out_cols[roll];
    double sum = 0.0, err_add = 0.0, err_sub = 0.0, chk = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        if (i >= ws) {  /* SumWindow::update: Kahan subtract of the leaving value first */
            const double y = (0.0 - x[i - ws]) - err_sub;
            const double ns = sum + y;
            err_sub = (ns - sum) - y;
            sum = ns;
        }
        {   /* then Kahan add of the entering value */
            const double y = x[i] - err_add;
            const double ns = sum + y;
            err_add = (ns - sum) - y;
            sum = ns;
        }
        out_roll[i] = i + 1 >= ws ? sum / (double)ws : 0.0;
        chk += out_roll[i];
    }
    free(p);
    free(q);
    return chk;
}

/* configs[3]: `probe.join(build, on="k")` inner, materialised (probe key,
 * probe payload, build payload).
 *  - build: polars-ops/src/frame/join/hash_join/single_keys.rs build_tables:
 *    the build keys hash-partitioned over the threads; each thread scans
 *    every build key and inserts those of its partition into its own table
 *    (key -> the rows in row order);
 *  - probe: single_keys_inner.rs:40 hash_join_tuples_inner, the probe side
 *    split into one contiguous chunk per thread, each probing in row order
 *    (probe_inner, :11) into a thread-local pair list; the lists are
 *    concatenated in chunk order;
 *  - materialise: general.rs:17 _finish_join, one take per column.
 * Tables are open addressing (the reference's hashbrown maps) over a 64-bit
 * mix of the key.  Returns the number of output rows. */
OR_EXPORT int64_t or_baseline_join_inner(const int64_t* pk, const double* pv, int64_t np, const int64_t* bk,
                                         const double* bv, int64_t nb, int32_t threads, int64_t* out_k,
                                         double* out_pv, double* out_bv, int64_t cap) {
    int T = threads > 0 ? threads : 1;
    int P = 1;
    while (P < T) P <<= 1;
    imap_t* tabs = (imap_t*)calloc((size_t)P, sizeof(imap_t));
    int64_t** heads = (int64_t**)calloc((size_t)P, sizeof(int64_t*));
    int64_t* next = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nb > 0 ? nb : 1));
#pragma omp parallel for num_threads(T) schedule(dynamic, 1)
    for (int part = 0; part < P; ++part) {
        imap_t* m = &tabs[part];
        imap_init(m, nb / P + 16);
        int64_t ng = 0, hcap = nb / P + 16;
        int64_t* head = (int64_t*)malloc(sizeof(int64_t) * (size_t)hcap);
        int64_t* tail = (int64_t*)malloc(sizeof(int64_t) * (size_t)hcap);
        for (int64_t r = 0; r < nb; ++r) {
            const uint64_t h = mix64((uint64_t)bk[r]);
            if ((int)(h >> 58) % P != part) continue;
            if (m->cap < 2 * (ng + 1)) {
                imap_t m2;
                imap_init(&m2, 2 * m->cap);
                for (int64_t s = 0; s < m->cap; ++s)
                    if (m->used[s]) { int d; imap_get_or_insert(&m2, m->keys[s], m->gid[s], &d); }
                imap_free(m);
                *m = m2;
            }
            int ins;
            const int64_t g = imap_get_or_insert(m, bk[r], ng, &ins);
            next[r] = -1;
            if (ins) {
                if (ng == hcap) {
                    hcap *= 2;
                    head = (int64_t*)realloc(head, sizeof(int64_t) * (size_t)hcap);
                    tail = (int64_t*)realloc(tail, sizeof(int64_t) * (size_t)hcap);
                }
                head[ng] = tail[ng] = r;
                ++ng;
            } else {
                next[tail[g]] = r;
                tail[g] = r;
            }
        }
        free(tail);
        heads[part] = head;
    }
    int64_t* cnt = (int64_t*)calloc((size_t)T + 1, sizeof(int64_t));
    int64_t** lp = (int64_t**)calloc((size_t)T, sizeof(int64_t*));
    int64_t** lb = (int64_t**)calloc((size_t)T, sizeof(int64_t*));
#pragma omp parallel for num_threads(T) schedule(static)
    for (int t = 0; t < T; ++t) {
        const int64_t lo = np * t / T, hi = np * (t + 1) / T;
        int64_t c = 0, cp = (hi - lo) / 2 + 16;
        int64_t* a = (int64_t*)malloc(sizeof(int64_t) * (size_t)cp);
        int64_t* b = (int64_t*)malloc(sizeof(int64_t) * (size_t)cp);
        for (int64_t r = lo; r < hi; ++r) {
            const uint64_t h0 = mix64((uint64_t)pk[r]);
            const int part = (int)(h0 >> 58) % P;
            const imap_t* m = &tabs[part];
            uint64_t h = h0 & (uint64_t)(m->cap - 1);
            int64_t g = -1;
            while (m->used[h]) {
                if (m->keys[h] == pk[r]) { g = m->gid[h]; break; }
                h = (h + 1) & (uint64_t)(m->cap - 1);
            }
            if (g < 0) continue;
            for (int64_t br = heads[part][g]; br >= 0; br = next[br]) {
                if (c == cp) {
                    cp *= 2;
                    a = (int64_t*)realloc(a, sizeof(int64_t) * (size_t)cp);
                    b = (int64_t*)realloc(b, sizeof(int64_t) * (size_t)cp);
                }
                a[c] = r;
                b[c] = br;
                ++c;
            }
        }
        lp[t] = a;
        lb[t] = b;
        cnt[t + 1] = c;
    }
    for (int t = 0; t < T; ++t) cnt[t + 1] += cnt[t];
    const int64_t total = cnt[T];
    if (total <= cap) {
#pragma omp parallel for num_threads(T) schedule(static)
        for (int t = 0; t < T; ++t) {
            const int64_t o = cnt[t], c = cnt[t + 1] - cnt[t];
            for (int64_t i = 0; i < c; ++i) {
                out_k[o + i] = pk[lp[t][i]];
                out_pv[o + i] = pv[lp[t][i]];
                out_bv[o + i] = bv[lb[t][i]];
            }
        }
    }
    for (int t = 0; t < T; ++t) { free(lp[t]); free(lb[t]); }
    for (int part = 0; part < P; ++part) { imap_free(&tabs[part]); free(heads[part]); }
    free(lp); free(lb); free(cnt); free(tabs); free(heads); free(next);
    return total <= cap ? total : -1;
}

/* ------------------------------------------ keyless float sum (pairwise)
 * polars-compute/src/float_sum.rs sum_arr_as_f64, the fold of the in-memory
 * engine's keyless `select(x.sum())` / `x.mean()` (ChunkAgg::sum /
 * _sum_as_f64, polars-core/src/chunked_array/ops/aggregate/mod.rs:68,94,
 * one call per chunk):
 *  - the first n % 128 values ("rest") are summed by Iterator::sum; the rest
 *    of the array ("main", a multiple of 128) pairwise: a block of
 *    PAIRWISE_RECURSION_LIMIT = 128 values is summed in STRIPE = 16 lanes
 *    (lane j takes values j, j + 16, ...), the lanes folded 16 -> 8 -> 4 and
 *    then (v0 + v2) + (v1 + v3) (vector_horizontal_sum); a longer run splits
 *    at floor(blocks / 2) * 128 and adds the halves (pairwise_sum);
 *  - masked (null) values contribute +0.0 (a select, not a skip);
 *  - result: mainsum + restsum.
 * Iterator::sum of f64 starts from -0.0 on the reference's toolchain
 * (rust-toolchain.toml: nightly-2025-10-24), so an empty "rest" adds -0.0. */
static double fs_block(const double* x, const uint8_t* valid) {
    double v[16];
    for (int j = 0; j < 16; ++j) v[j] = 0.0;
    for (int c = 0; c < 128; c += 16)
        for (int j = 0; j < 16; ++j) v[j] = v[j] + ((valid == NULL || valid[c + j]) ? x[c + j] : 0.0);
    for (int w = 16; w > 4; w /= 2)
        for (int j = 0; j < w / 2; ++j) v[j] = v[j] + v[w / 2 + j];
    return (v[0] + v[2]) + (v[1] + v[3]);
}

static double fs_pairwise(const double* x, const uint8_t* valid, int64_t n) {
    if (n == 128) return fs_block(x, valid);
    const int64_t left = (n / 128 / 2) * 128;
    return fs_pairwise(x, valid, left) + fs_pairwise(x + left, valid ? valid + left : NULL, n - left);
}

OR_EXPORT double or_float_sum(const double* x, const uint8_t* valid, int64_t n) {
    const int64_t rem = n % 128;
    const double mainsum = n > rem ? fs_pairwise(x + rem, valid ? valid + rem : NULL, n - rem) : 0.0;
    double restsum = -0.0;
    for (int64_t i = 0; i < rem; ++i) restsum = restsum + ((valid == NULL || valid[i]) ? x[i] : 0.0);
    return mainsum + restsum;
}

/* ------------------------------------------------ variance (VarState)
 * polars-compute/src/moment.rs VarState (Schubert & Gertz 2018):
 *  - or_var_welford: the streaming group-by's VarReducer
 *    (polars-expr/src/reduce/var_std.rs:89 reduce_one -> insert_one per row,
 *    :84 combine): one state per partition id part[i] (a thread's or a
 *    morsel's rows), each fed row by row with insert_one, the states combined
 *    in order; finalize(ddof) (negative -> 0).
 *  - or_var_chunked: the in-memory keyless `x.var()` (moment.rs:641 var):
 *    VarState::new over consecutive chunks of CHUNK_SIZE = 128 values (mean
 *    and squared deviations summed with alg_sum_f64, which lets the compiler
 *    reassociate; restated in row order), combined in order.
 * Return NaN for "None" (weight <= ddof). */
typedef struct { double w, mean, dp; } vs_t;

static void vs_zero_nan(vs_t* s) {
    if (s->w == 0.0) { s->mean = 0.0; s->dp = 0.0; }
}
static void vs_insert(vs_t* s, double x) {
    const double nw = s->w + 1.0;
    const double dm = x - s->mean;
    const double nm = s->mean + dm / nw;
    s->dp += (x - nm) * dm;
    s->w = nw;
    s->mean = nm;
    vs_zero_nan(s);
}
static void vs_combine(vs_t* s, const vs_t* o) {
    if (o->w == 0.0) return;
    const double nw = s->w + o->w;
    const double frac = o->w / nw;
    const double dm = o->mean - s->mean;
    const double nm = s->mean + dm * frac;
    s->dp += o->dp + o->w * (o->mean - nm) * dm;
    s->w = nw;
    s->mean = nm;
    vs_zero_nan(s);
}
static double vs_finalize(const vs_t* s, int32_t ddof) {
    if (s->w <= (double)ddof) return NAN;
    const double v = s->dp / (s->w - (double)ddof);
    return v < 0.0 ? 0.0 : v;
}

OR_EXPORT double or_var_welford(const double* x, const int64_t* part, int64_t n, int32_t ddof) {
    vs_t tot = {0.0, 0.0, 0.0}, cur = {0.0, 0.0, 0.0};
    for (int64_t i = 0; i < n; ++i) {
        if (i > 0 && part[i] != part[i - 1]) {
            vs_combine(&tot, &cur);
            cur.w = cur.mean = cur.dp = 0.0;
        }
        vs_insert(&cur, x[i]);
    }
    vs_combine(&tot, &cur);
    return vs_finalize(&tot, ddof);
}

OR_EXPORT double or_var_chunked(const double* x, int64_t n, int32_t ddof) {
    vs_t tot = {0.0, 0.0, 0.0};
    for (int64_t c = 0; c < n; c += 128) {
        const int64_t m = n - c < 128 ? n - c : 128;
        double s = 0.0;
        for (int64_t i = 0; i < m; ++i) s += x[c + i];
        vs_t ch;
        ch.w = (double)m;
        ch.mean = s / ch.w;
        double dp = 0.0;
        for (int64_t i = 0; i < m; ++i) dp += (x[c + i] - ch.mean) * (x[c + i] - ch.mean);
        ch.dp = dp;
        vs_combine(&tot, &ch);
    }
    return vs_finalize(&tot, ddof);
}

/* ------------------------------------------------- CPU baseline: filter */
/* filter(pred > k).collect() of ncols 8-byte columns on the host cores, as
 * the reference's FilterExec runs it (polars-mem-engine/src/executors/
 * filter.rs:70 -> DataFrame::filter, each column by the one mask,
 * polars-compute/src/filter/mod.rs:18 filter with the primitive kernel of
 * filter/primitive.rs): the mask is evaluated per thread chunk with
 * tot_gt (a NaN compares greater), a prefix over the chunks' counts places
 * each chunk's rows, and every column is compacted in row order.  `out`:
 * ncols buffers of nrows words.  Returns the selected rows. */
OR_EXPORT int64_t or_baseline_filter(const double* pred, double k, const uint64_t* const* cols, int32_t ncols,
                                     int64_t nrows, int32_t threads, uint64_t* const* out) {
    int T = threads > 0 ? threads : 1;
    int64_t* cnt = (int64_t*)calloc((size_t)T + 1, sizeof(int64_t));
#pragma omp parallel num_threads(T)
    {
#ifdef _OPENMP
        int t = omp_get_thread_num();
#else
        int t = 0;
#endif
        const int64_t lo = nrows * t / T, hi = nrows * (t + 1) / T;
        int64_t c = 0;
        for (int64_t r = lo; r < hi; ++r) {
            const double x = pred[r];
            c += (isnan(x) || x > k) ? 1 : 0;
        }
        cnt[t + 1] = c;
#pragma omp barrier
#pragma omp single
        for (int i = 0; i < T; ++i) cnt[i + 1] += cnt[i];
        int64_t o = cnt[t];
        for (int64_t r = lo; r < hi; ++r) {
            const double x = pred[r];
            if (!(isnan(x) || x > k)) continue;
            for (int ci = 0; ci < ncols; ++ci) out[ci][o] = cols[ci][r];
            ++o;
        }
    }
    const int64_t total = cnt[T];
    free(cnt);
    return total;
}

/* ------------------------------------------------- rolling var / std */
/* Mode 0 restates the reference: polars-compute/src/rolling/moment.rs:138
 * MomentWindow<VarianceMoment> (:16) -- a VarState (polars-compute/src/
 * moment.rs:87 insert_one, :99 remove_one, :126 finalize) slid over the
 * window (reset when the new window starts past the old one's end, :228);
 * a non-finite value enters as 0.0 and is counted apart, and any makes the
 * result NaN (:196); nulls are skipped (nulls/moment.rs, moment.rs:255);
 * the result is null when fewer than min_periods non-null values are in
 * the window (no_nulls/mod.rs:61, nulls/mod.rs:73) or weight <= ddof
 * (moment.rs:127); rolling_std is its square root (polars-time/src/
 * chunkedarray/rolling_window/dispatch.rs:526).
 *
 * Mode 1 is the exact form the GPU computes: with c the window's non-null
 * count, var = (RN(c * sum x^2 - (sum x)^2) / c) / (c - ddof), the
 * numerator formed exactly (big integer over the window's smallest
 * exponent) and rounded once -- the group-by's fused variance
 * (groupby.hip var_exact) applied to each window. */
static void vs_remove(vs_t* s, double x) {
    const double nw = s->w - 1.0;
    const double dm = x - s->mean;
    const double nm = s->mean - dm / nw;
    s->dp -= (x - nm) * dm;
    s->w = nw;
    s->mean = nm;
    vs_zero_nan(s);
}

#define RV_LIMBS 80 /* 5120 bits: c * sum t^2 for any f64 span, c < 2^16 */
typedef struct { uint64_t w[RV_LIMBS]; } rv_big;

static void rvb_add_shifted(rv_big* a, unsigned __int128 v, int sh, int negate) {
    /* a += (negate ? -1 : 1) * (v << sh), two's complement over RV_LIMBS */
    const int ws = sh / 64, bs = sh % 64;
    const uint64_t lo = (uint64_t)v, hi = (uint64_t)(v >> 64);
    uint64_t parts[3];
    parts[0] = bs ? lo << bs : lo;
    parts[1] = bs ? (hi << bs) | (lo >> (64 - bs)) : hi;
    parts[2] = bs ? hi >> (64 - bs) : 0;
    uint64_t carry = 0;
    for (int i = ws; i < RV_LIMBS; ++i) {
        const int k = i - ws;
        const uint64_t d = k < 3 ? parts[k] : 0;
        if (k >= 3 && carry == 0) break;
        if (!negate) {
            const unsigned __int128 t = (unsigned __int128)a->w[i] + d + carry;
            a->w[i] = (uint64_t)t;
            carry = (uint64_t)(t >> 64);
        } else {
            const unsigned __int128 t = (unsigned __int128)a->w[i] - d - carry;
            a->w[i] = (uint64_t)t;
            carry = (uint64_t)(t >> 64) ? 1 : 0; /* borrow */
        }
    }
}

/* x (>= 0) * 2^e rounded to nearest-even f64 (subnormals included). */
static double rvb_to_double(const rv_big* a, int e) {
    int top = RV_LIMBS - 1;
    while (top >= 0 && a->w[top] == 0) --top;
    if (top < 0) return 0.0;
    const int p = top * 64 + 63 - __builtin_clzll(a->w[top]); /* leading bit */
    /* keep bits down to position q: 53 significant bits, fewer when the
     * result is subnormal (bit q weighs 2^(q + e) >= 2^-1074) */
    int q = p - 52;
    if (q + e < -1074) q = -1074 - e;
    if (q <= 0) return ldexp((double)a->w[0], e); /* exact: < 2^53 */
    uint64_t keep = 0;
    for (int b = p; b >= q; --b) keep = (keep << 1) | ((a->w[b / 64] >> (b % 64)) & 1);
    const int rb = q - 1;
    const int round = (int)((a->w[rb / 64] >> (rb % 64)) & 1);
    int sticky = 0;
    for (int b = 0; b < rb && !sticky; ++b) sticky = (int)((a->w[b / 64] >> (b % 64)) & 1);
    if (round && (sticky || (keep & 1))) ++keep;
    return ldexp((double)keep, q + e);
}

/* Exact variance of the finite values xs[0..m) (c = m + nonfinite is the
 * count), the GPU's rounding: (RN(c sum t^2 - (sum t)^2) / c) / (c - ddof). */
static double rv_exact(const double* xs, int64_t m, int64_t c, int32_t ddof) {
    int emin = 1 << 20;
    for (int64_t i = 0; i < m; ++i) {
        if (xs[i] == 0.0) continue;
        int ex;
        (void)frexp(xs[i], &ex);
        const int e0 = ex - 53; /* xs[i] = t * 2^e0 with |t| < 2^53 */
        if (e0 < emin) emin = e0;
    }
    if (emin < -1074) emin = -1074;
    if (emin == 1 << 20) return 0.0; /* every value zero */
    rv_big sq, s1;
    memset(&sq, 0, sizeof sq);
    memset(&s1, 0, sizeof s1);
    for (int64_t i = 0; i < m; ++i) {
        if (xs[i] == 0.0) continue;
        int ex;
        const double fr = frexp(fabs(xs[i]), &ex);
        const uint64_t t = (uint64_t)ldexp(fr, 53); /* |x| = t * 2^(ex - 53) */
        int sh = ex - 53 - emin;
        uint64_t tt = t;
        if (sh < 0) { tt = t >> (-sh); sh = 0; } /* subnormal: exact (low bits zero) */
        /* t^2 << 2 sh into sq; t << sh into s1 (signed) */
        rvb_add_shifted(&sq, (unsigned __int128)tt * tt, 2 * sh, 0);
        rvb_add_shifted(&s1, tt, sh, xs[i] < 0);
    }
    /* num = c * sq - s1^2 */
    rv_big num;
    memset(&num, 0, sizeof num);
    for (int i = 0; i < RV_LIMBS; ++i) {
        if (sq.w[i] == 0) continue;
        rvb_add_shifted(&num, (unsigned __int128)sq.w[i] * (uint64_t)c, 64 * i, 0);
    }
    const int neg1 = (int64_t)s1.w[RV_LIMBS - 1] < 0;
    if (neg1) { /* |s1| */
        unsigned __int128 carry = 1;
        for (int i = 0; i < RV_LIMBS; ++i) {
            const unsigned __int128 s = (unsigned __int128)(~s1.w[i]) + carry;
            s1.w[i] = (uint64_t)s;
            carry = s >> 64;
        }
    }
    for (int i = 0; i < RV_LIMBS; ++i) {
        if (s1.w[i] == 0) continue;
        for (int j = 0; j < RV_LIMBS && i + j < RV_LIMBS; ++j) {
            if (s1.w[j] == 0) continue;
            rvb_add_shifted(&num, (unsigned __int128)s1.w[i] * s1.w[j], 64 * (i + j), 1);
        }
    }
    if ((int64_t)num.w[RV_LIMBS - 1] < 0) return 0.0; /* cannot happen: c sum t^2 >= (sum t)^2 */
    const double nr = rvb_to_double(&num, 2 * emin);
    return (nr / (double)c) / (double)(c - ddof);
}

OR_EXPORT void or_rolling_var(const plgpu_column* c, int64_t ws, int64_t min_periods, int32_t center, int32_t ddof,
                              int32_t std, int32_t mode, double* out, uint8_t* out_valid) {
    const int64_t n = c->length;
    int has_nulls = 0;
    for (int64_t r = 0; r < n && !has_nulls; ++r) has_nulls = !col_valid(c, r);
    vs_t st;
    memset(&st, 0, sizeof st);
    int64_t nonfinite = 0, nulls = 0, last_start = 0, last_end = 0;
    double* buf = (double*)malloc(sizeof(double) * (size_t)(ws > 0 ? ws : 1));
    for (int64_t i = 0; i < n; ++i) {
        int64_t s, e;
        rl_offsets(i, ws, n, center, &s, &e);
        double v = 0.0;
        int valid = 0;
        if (mode == 0) {
            if (!has_nulls && e - s < min_periods) {
                out[i] = 0.0;
                out_valid[i] = 0;
                continue;
            }
            if (s >= last_end) {
                memset(&st, 0, sizeof st);
                nonfinite = nulls = 0;
                last_start = last_end = s;
            }
            for (int64_t r = last_start; r < s; ++r) {
                if (!col_valid(c, r)) { --nulls; continue; }
                const double x = rl_val(c, r);
                if (isfinite(x)) vs_remove(&st, x);
                else { vs_remove(&st, 0.0); --nonfinite; }
            }
            for (int64_t r = last_end; r < e; ++r) {
                if (!col_valid(c, r)) { ++nulls; continue; }
                const double x = rl_val(c, r);
                if (isfinite(x)) vs_insert(&st, x);
                else { vs_insert(&st, 0.0); ++nonfinite; }
            }
            last_start = s;
            last_end = e;
            const int some = st.w > (double)ddof;
            valid = some && (e - s) - nulls >= min_periods;
            if (valid) v = nonfinite > 0 ? NAN : vs_finalize(&st, ddof);
        } else {
            int64_t m = 0, cnt = 0, nf = 0;
            for (int64_t r = s; r < e; ++r) {
                if (!col_valid(c, r)) continue;
                ++cnt;
                const double x = rl_val(c, r);
                if (isfinite(x)) buf[m++] = x;
                else ++nf;
            }
            valid = cnt >= min_periods && cnt > ddof;
            if (valid) v = nf > 0 ? NAN : rv_exact(buf, m, cnt, ddof);
        }
        if (valid && std) v = sqrt(v);
        out[i] = valid ? v : 0.0;
        out_valid[i] = (uint8_t)valid;
    }
    free(buf);
}
