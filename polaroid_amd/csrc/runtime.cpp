// runtime.cpp — error plumbing, stream-ordered device allocator, copies,
// column ownership and host-side lowering of expression programs.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "plgpu_internal.hpp"

namespace plgpu {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    g_last_error = std::string("HIP error: ") + hipGetErrorString(e) + " at " + what;
    (void)hipGetLastError();
    return e == hipErrorOutOfMemory ? PLGPU_ERR_OOM : PLGPU_ERR_HIP;
}

hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------------------ options
// Test hooks and diagnostics: each read once from the environment
// (PLGPU_<NAME>, an integer) when the library loads, and settable through
// plgpu_set_option.  No measurement variant lives here: losing A/B variants
// leave the product once their numbers are logged.
// name, environment variable and field of every option
namespace {
struct OptField {
    const char* name;
    const char* env;
    int Options::*f;
};
const OptField kOptFields[] = {
    {"debug", "PLGPU_DEBUG", &Options::debug},
    {"no_pack", "PLGPU_NO_PACK", &Options::no_pack},
    {"mk_collide", "PLGPU_MK_COLLIDE", &Options::mk_collide},
    {"runs", "PLGPU_RUNS", &Options::runs},
    {"local", "PLGPU_LOCAL", &Options::local},
    {"ktime", "PLGPU_KTIME", &Options::ktime},
    {"fuse_keys", "PLGPU_FUSE_KEYS", &Options::fuse_keys},
    {"grid_rounds", "PLGPU_GRID_ROUNDS", &Options::grid_rounds},
    {"plan_cache", "PLGPU_PLAN_CACHE", &Options::plan_cache},
    {"gb_path", "PLGPU_GB_PATH", &Options::gb_path},
    {"part_bits", "PLGPU_PART_BITS", &Options::part_bits},
    {"part_levels", "PLGPU_PART_LEVELS", &Options::part_levels},
    {"part_direct", "PLGPU_PART_DIRECT", &Options::part_direct},
    {"part_compact", "PLGPU_PART_COMPACT", &Options::part_compact},
    {"rl_var128", "PLGPU_RL_VAR128", &Options::rl_var128},
    {"rl_var_hot", "PLGPU_RL_VAR_HOT", &Options::rl_var_hot},
    {"rl_mean_hot", "PLGPU_RL_MEAN_HOT", &Options::rl_mean_hot},
    {"alloc_skew", "PLGPU_ALLOC_SKEW", &Options::alloc_skew},
    {"alloc_contig", "PLGPU_ALLOC_CONTIG", &Options::alloc_contig},
    {"srt_w4", "PLGPU_SRT_W4", &Options::srt_w4},
    {"srt_up_tiles", "PLGPU_SRT_UP_TILES", &Options::srt_up_tiles},
    {"part_rows4", "PLGPU_PART_ROWS4", &Options::part_rows4},
    {"wave_report", "PLGPU_WAVE_REPORT", &Options::wave_report},
    {"part_null_sentinel", "PLGPU_PART_NULL_SENTINEL", &Options::part_null_sentinel},
    {"part_lds_kb", "PLGPU_PART_LDS_KB", &Options::part_lds_kb},
    {"rl_stream", "PLGPU_RL_STREAM", &Options::rl_stream},
    {"rl_grid", "PLGPU_RL_GRID", &Options::rl_grid},
    {"filt_pipe", "PLGPU_FILT_PIPE", &Options::filt_pipe},
    {"rl_div", "PLGPU_RL_DIV", &Options::rl_div},
    {"part_threads", "PLGPU_PART_THREADS", &Options::part_threads},
    {"gb_pair", "PLGPU_GB_PAIR", &Options::gb_pair},
    {"rl_full", "PLGPU_RL_FULL", &Options::rl_full},
    {"filt_fused", "PLGPU_FILT_FUSED", &Options::filt_fused},
    {"var_pos", "PLGPU_VAR_POS", &Options::var_pos},
    {"sum_pos", "PLGPU_SUM_POS", &Options::sum_pos},
    {"join_radix", "PLGPU_JOIN_RADIX", &Options::join_radix},
    {"join_radix_keys", "PLGPU_JOIN_RADIX_KEYS", &Options::join_radix_keys},
    {"join_radix_load", "PLGPU_JOIN_RADIX_LOAD", &Options::join_radix_load},
    {"join_radix_batch", "PLGPU_JOIN_RADIX_BATCH", &Options::join_radix_batch},
};
const OptField* opt_field(const char* name) {
    for (const OptField& f : kOptFields)
        if (!strcmp(name, f.name)) return &f;
    return nullptr;
}
}  // namespace

static Options read_env_options() {
    Options o;
    for (const OptField& f : kOptFields) {
        const char* e = getenv(f.env);
        if (e) o.*(f.f) = atoi(e);
    }
    return o;
}

Options& options() {
    static Options o = read_env_options();
    return o;
}

// ------------------------------------------------------------ kernel timer
// Pending (name, start, stop) event pairs; plgpu_ktime_read waits for them
// and folds them into per-name sums.  Events are pooled across reads.
namespace {
struct KtPending {
    const char* name;
    hipEvent_t a, b;
};
struct KtSum {
    std::string name;
    double ms = 0.0;
    int64_t count = 0;
};
std::mutex g_kt_mu;
std::vector<KtPending> g_kt_pending;
std::vector<hipEvent_t> g_kt_pool;
std::vector<KtSum> g_kt_sums;

hipEvent_t kt_event() {
    if (!g_kt_pool.empty()) {
        hipEvent_t e = g_kt_pool.back();
        g_kt_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}
}  // namespace

hipEvent_t ev_acquire() {
    std::lock_guard<std::mutex> g(g_kt_mu);
    return kt_event();
}

void ev_release(hipEvent_t e) {
    if (e == nullptr) return;
    std::lock_guard<std::mutex> g(g_kt_mu);
    g_kt_pool.push_back(e);
}

bool kt_begin(hipStream_t s, hipEvent_t* a, hipEvent_t* b) {
    std::lock_guard<std::mutex> g(g_kt_mu);
    *a = kt_event();
    *b = kt_event();
    if (*a == nullptr || *b == nullptr || hipEventRecord(*a, s) != hipSuccess) {
        if (*a) g_kt_pool.push_back(*a);
        if (*b) g_kt_pool.push_back(*b);
        *a = *b = nullptr;
        return false;
    }
    return true;
}

void kt_end(const char* name, hipEvent_t a, hipEvent_t b, hipStream_t s) {
    std::lock_guard<std::mutex> g(g_kt_mu);
    (void)hipEventRecord(b, s);
    g_kt_pending.push_back({name, a, b});
}

// Caching device allocator.  Blocks come from hipMalloc and are recycled
// through size-keyed free lists instead of being returned with hipFree
// (which synchronises the device).  Every entry point enqueues all of its
// work on the caller's one stream (the library has no stream of its own)
// and frees only after the kernels that use a block were enqueued there, so
// stream order makes reuse safe.  (hipMallocAsync / hipFreeAsync from the
// device's default pool passed the same parity suites, profiles/
// r02_alloc_async_ab.log; the cache stays because it never synchronises.)
namespace {
struct Pool {
    std::mutex mu;
    std::multimap<size_t, void*> free_blocks;        // size -> ptr
    std::unordered_map<void*, size_t> sizes;         // every block we own
    // option alloc_skew: large blocks handed out at base + a rotating
    // multiple of 64 KiB (returned pointer -> base)
    std::unordered_map<void*, void*> skewed;
    uint32_t skew_ctr = 0;
    size_t cached = 0;
};
Pool& pool_for(int dev) {
    static Pool pools[64];
    return pools[(dev >= 0 && dev < 64) ? dev : 0];
}
size_t round_bytes(size_t b) {
    if (b <= (size_t(1) << 20)) return (b + 255) & ~size_t(255);
    return (b + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);  // 2 MiB granules
}
void release_cached(Pool& P) {
    for (auto& kv : P.free_blocks) {
        (void)hipFree(kv.second);
        P.sizes.erase(kv.second);
    }
    P.free_blocks.clear();
    P.cached = 0;
}
}  // namespace

int dev_alloc(void** p, size_t bytes, hipStream_t s) {
    (void)s;
    *p = nullptr;
    // option alloc_skew (A/B): blocks of 256 MiB and more start at one of 16
    // offsets 64 KiB apart inside a block 1 MiB larger, so the concurrent
    // streams of a multi-column kernel land at different offsets modulo the
    // HBM channel interleave whatever their bases
    const bool skew = options().alloc_skew != 0 && bytes >= (size_t(256) << 20);
    const size_t want = round_bytes(bytes == 0 ? 256 : bytes + (skew ? size_t(1) << 20 : 0));
    int dev = 0;
    (void)hipGetDevice(&dev);
    Pool& P = pool_for(dev);
    std::lock_guard<std::mutex> lk(P.mu);
    auto it = P.free_blocks.lower_bound(want);
    auto skew_out = [&]() {
        if (!skew) return;
        char* q = (char*)*p + (size_t)(P.skew_ctr++ % 16) * (size_t(64) << 10);
        P.skewed[q] = *p;
        *p = q;
    };
    if (it != P.free_blocks.end() && it->first <= want + want / 4) {
        *p = it->second;
        P.cached -= it->first;
        P.free_blocks.erase(it);
        skew_out();
        return PLGPU_OK;
    }
    hipError_t e = hipErrorOutOfMemory;
    if (options().alloc_contig != 0 && want >= (size_t(256) << 20)) {
        // (option alloc_contig, A/B: physically contiguous large blocks, for
        // the TLB reach of streams over them; plain hipMalloc when refused)
        e = hipExtMallocWithFlags(p, want, hipDeviceMallocContiguous);
        if (e != hipSuccess) (void)hipGetLastError();
    }
    if (e != hipSuccess) e = hipMalloc(p, want);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        (void)hipDeviceSynchronize();
        release_cached(P);
        e = hipMalloc(p, want);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            *p = nullptr;
            char buf[128];
            snprintf(buf, sizeof buf, "device allocation of %zu bytes failed", bytes);
            return fail(PLGPU_ERR_OOM, buf);
        }
    }
    P.sizes[*p] = want;
    skew_out();
    return PLGPU_OK;
}

void dev_free(void* p, hipStream_t s) {
    (void)s;
    if (p == nullptr) return;
    int dev = 0;
    (void)hipGetDevice(&dev);
    Pool& P = pool_for(dev);
    std::lock_guard<std::mutex> lk(P.mu);
    auto sk = P.skewed.find(p);
    if (sk != P.skewed.end()) {
        p = sk->second;
        P.skewed.erase(sk);
    }
    auto it = P.sizes.find(p);
    if (it == P.sizes.end()) {
        (void)hipFree(p);  // not ours: release directly
        return;
    }
    P.free_blocks.emplace(it->second, p);
    P.cached += it->second;
}

static void release_owned(plgpu_column* c) {
    if (c == nullptr || c->private_data == nullptr) return;
    OwnedBuffers* ob = static_cast<OwnedBuffers*>(c->private_data);
    dev_free(ob->values, ob->stream);
    dev_free(ob->validity, ob->stream);
    dev_free(ob->data, ob->stream);
    delete ob;
    c->private_data = nullptr;
    c->values = nullptr;
    c->validity = nullptr;
    c->data = nullptr;
    c->release = nullptr;
}

int make_owned_column(plgpu_column* out, int32_t dtype, int64_t length, bool with_validity,
                      hipStream_t s) {
    std::memset(out, 0, sizeof *out);
    OwnedBuffers* ob = new OwnedBuffers();
    ob->stream = s;
    size_t vbytes = dtype == PLGPU_BOOL ? (size_t)((length + 63) / 64) * 8
                                        : (size_t)length * dtype_bytes(dtype);
    int rc = dev_alloc(&ob->values, vbytes, s);
    if (rc != PLGPU_OK) { delete ob; return rc; }
    if (with_validity) {
        rc = dev_alloc(&ob->validity, (size_t)((length + 63) / 64) * 8, s);
        if (rc != PLGPU_OK) { dev_free(ob->values, s); delete ob; return rc; }
    }
    int dev = 0;
    (void)hipGetDevice(&dev);
    out->dtype = dtype;
    out->device_id = dev;
    out->length = length;
    out->offset = 0;
    out->null_count = with_validity ? -1 : 0;
    out->values = ob->values;
    out->validity = (const uint8_t*)ob->validity;
    out->release = release_owned;
    out->private_data = ob;
    return PLGPU_OK;
}

int owned_attach_data(plgpu_column* out, int64_t bytes, hipStream_t s) {
    OwnedBuffers* ob = static_cast<OwnedBuffers*>(out->private_data);
    if (ob == nullptr) return fail(PLGPU_ERR_INVALID, "not an owned column");
    const int rc = dev_alloc(&ob->data, (size_t)std::max<int64_t>(bytes, 1), s);
    if (rc != PLGPU_OK) return rc;
    out->dtype = PLGPU_STR;
    out->length -= 1;  // the offsets buffer holds length + 1 entries
    out->data = (const uint8_t*)ob->data;
    return PLGPU_OK;
}

int make_owned_string_column(plgpu_column* out, int64_t length, int64_t bytes, bool with_validity, hipStream_t s) {
    int rc = make_owned_column(out, PLGPU_I64, length + 1, with_validity, s);
    if (rc == PLGPU_OK) rc = owned_attach_data(out, bytes, s);
    if (rc != PLGPU_OK) plgpu_column_release(out);
    return rc;
}

// ------------------------------------------------------ program lowering
// Every operand gets polars' static type: binary operands are coerced to
// their supertype (polars-core/src/utils/supertype.rs) before the op, and
// integer results wrap at the supertype's width.  LIT_I64 / LIT_F64 are
// dynamic literals (UnknownKind::Int / Float): they take the type the other
// operand's supertype rule gives them, and their immediate is rewritten in
// that type (a float literal against a Float32 column is rounded to f32).
namespace {
constexpr int TY_LIT_INT = 100, TY_LIT_FLOAT = 101, TY_NULL = 102;

bool is_int(int t) { return dtype_is_int(t); }
bool is_uint(int t) { return t == PLGPU_U8 || t == PLGPU_U16 || t == PLGPU_U32 || t == PLGPU_U64; }
bool is_float(int t) { return t == PLGPU_F32 || t == PLGPU_F64; }
int int_bits(int t) { return dtype_bytes(t) * 8; }
int sint_of_bits(int b) { return b <= 8 ? PLGPU_I8 : b <= 16 ? PLGPU_I16 : b <= 32 ? PLGPU_I32 : PLGPU_I64; }
int uint_of_bits(int b) { return b <= 8 ? PLGPU_U8 : b <= 16 ? PLGPU_U16 : b <= 32 ? PLGPU_U32 : PLGPU_U64; }

// supertype of two concrete numeric / Boolean types (supertype.rs:146); 0 = none
int supertype(int a, int b) {
    if (a == b) return a;
    if (a == PLGPU_BOOL) return (is_int(b) || is_float(b)) ? b : 0;
    if (b == PLGPU_BOOL) return (is_int(a) || is_float(a)) ? a : 0;
    if (is_float(a) || is_float(b)) {
        if (is_float(a) && is_float(b)) return PLGPU_F64;
        const int f = is_float(a) ? a : b, i = is_float(a) ? b : a;
        if (f == PLGPU_F64) return PLGPU_F64;
        return int_bits(i) <= 16 ? PLGPU_F32 : PLGPU_F64;  // Int8/16, UInt8/16 + Float32 -> Float32
    }
    const bool ua = is_uint(a), ub = is_uint(b);
    if (ua == ub) return int_bits(a) >= int_bits(b) ? a : b;
    const int s = ua ? b : a, u = ua ? a : b;
    if (u == PLGPU_U64) return PLGPU_F64;  // "follow numpy"
    if (int_bits(u) < int_bits(s)) return s;
    return sint_of_bits(2 * int_bits(u));
}

// smallest type holding the dynamic int v (materialize_smallest_dyn_int /
// materialize_dyn_int_pos)
int smallest_int(int64_t v, bool prefer_unsigned) {
    if (prefer_unsigned && v >= 0)
        return v <= 255 ? PLGPU_U8 : v <= 65535 ? PLGPU_U16 : v <= 4294967295ll ? PLGPU_U32 : PLGPU_U64;
    if (v >= -128 && v <= 127) return PLGPU_I8;
    if (v >= -32768 && v <= 32767) return PLGPU_I16;
    if (v >= INT32_MIN && v <= INT32_MAX) return PLGPU_I32;
    return PLGPU_I64;
}

uint64_t bits_of(double d) {
    uint64_t u;
    std::memcpy(&u, &d, 8);
    return u;
}
double dbl_of(uint64_t u) {
    double d;
    std::memcpy(&d, &u, 8);
    return d;
}

struct Ent {
    int ty;          // dtype code, or TY_LIT_INT / TY_LIT_FLOAT / TY_NULL
    int lit_pos;     // index of the D_LIT / D_NULL that pushed a pending literal, else -1
    bool scalar;     // a literal or an expression of literals (broadcast scalar)
    int64_t ival;
    double fval;
};

struct Lowering {
    std::vector<Ent> st;
    std::vector<DevInstr> code;

    void emit(int32_t op, int32_t arg = 0, uint64_t imm = 0) {
        DevInstr d;
        d.op = op;
        d.arg = arg;
        d.imm = imm;
        code.push_back(d);
    }
    static bool pending(const Ent& e) { return e.ty == TY_LIT_INT || e.ty == TY_LIT_FLOAT || e.ty == TY_NULL; }

    // A dynamic literal takes the type `t`: rewrite its immediate in place.
    void settle(Ent& e, int t) {
        if (!pending(e)) return;
        DevInstr& d = code[e.lit_pos];
        if (e.ty == TY_LIT_INT) {
            if (is_float(t)) d.imm = bits_of(t == PLGPU_F32 ? (double)(float)e.ival : (double)e.ival);
            else if (t == PLGPU_BOOL) d.imm = e.ival != 0;
            else d.imm = (uint64_t)e.ival;
        } else if (e.ty == TY_LIT_FLOAT) {
            d.imm = bits_of(t == PLGPU_F32 ? (double)(float)e.fval : e.fval);
        }
        e.ty = t;
        e.lit_pos = -1;
    }

    // Type a dynamic literal takes next to an operand of type t.
    static int lit_join(const Ent& lit, int t) {
        if (t == TY_NULL) return lit.ty == TY_LIT_INT ? smallest_int(lit.ival, false) : PLGPU_F64;
        if (lit.ty == TY_NULL) return t;
        if (lit.ty == TY_LIT_FLOAT) return is_float(t) ? t : PLGPU_F64;
        if (is_float(t)) return t;
        if (t == PLGPU_BOOL) return smallest_int(lit.ival, false) == PLGPU_I8 ? PLGPU_I32 : PLGPU_I64;
        const int sm = smallest_int(lit.ival, is_uint(t));
        if (t == PLGPU_U64 && !is_uint(sm)) return PLGPU_I64;
        return supertype(t, sm);
    }

    // Materialize a literal on its own (Int32 / Int64 / Float64).
    static int lit_alone(const Ent& e) {
        if (e.ty == TY_LIT_INT) return (e.ival >= INT32_MIN && e.ival <= INT32_MAX) ? PLGPU_I32 : PLGPU_I64;
        if (e.ty == TY_LIT_FLOAT) return PLGPU_F64;
        return e.ty == TY_NULL ? PLGPU_BOOL : e.ty;
    }

    // Common type of two operands (0 = incompatible).
    static int join(const Ent& a, const Ent& b) {
        const bool pa = pending(a), pb = pending(b);
        if (pa && pb) {
            if (a.ty == TY_NULL && b.ty == TY_NULL) return PLGPU_BOOL;
            if (a.ty == TY_NULL) return lit_alone(b);
            if (b.ty == TY_NULL) return lit_alone(a);
            if (a.ty == TY_LIT_FLOAT || b.ty == TY_LIT_FLOAT) return PLGPU_F64;
            return supertype(lit_alone(a), lit_alone(b));
        }
        if (pa) return lit_join(a, b.ty);
        if (pb) return lit_join(b, a.ty);
        return supertype(a.ty, b.ty);
    }

    // Bring stack entry `depth` (0 = top) to type t (settle or cast).
    void coerce(int depth, int t) {
        Ent& e = st[st.size() - 1 - depth];
        if (pending(e)) {
            settle(e, t);
            return;
        }
        if (e.ty == t) return;
        emit(D_CAST, t, ((uint64_t)e.ty << 8) | (depth ? 0x10000ull : 0ull));
        e.ty = t;
    }
};

int cmp_index(int32_t op) {
    switch (op) {
    case PLGPU_OP_EQ: return 0;
    case PLGPU_OP_NE: return 1;
    case PLGPU_OP_LT: return 2;
    case PLGPU_OP_LE: return 3;
    case PLGPU_OP_GT: return 4;
    case PLGPU_OP_GE: return 5;
    default: return -1;
    }
}

bool numeric_or_bool(int t) { return t == PLGPU_BOOL || is_int(t) || is_float(t); }
}  // namespace

int lower_program(const plgpu_column* cols, int32_t ncols, const plgpu_instr* prog, int32_t n,
                  DevProgram* out) {
    std::memset(out, 0, sizeof *out);
    if (n <= 0) return fail(PLGPU_ERR_INVALID, "empty expression program");
    if (n > PLGPU_MAX_PROGRAM) return fail(PLGPU_ERR_INVALID, "expression program too long");
    Lowering L;
    auto& st = L.st;
    auto push = [&](int ty, int lit_pos, bool scalar, int64_t iv = 0, double fv = 0) {
        Ent e;
        e.ty = ty;
        e.lit_pos = lit_pos;
        e.scalar = scalar;
        e.ival = iv;
        e.fval = fv;
        st.push_back(e);
    };
    for (int k = 0; k < n; ++k) {
        const plgpu_instr& in = prog[k];
        auto need = [&](size_t m) -> bool { return st.size() >= m; };
        switch (in.op) {
        case PLGPU_OP_COL: {
            if (in.arg < 0 || in.arg >= ncols) return fail(PLGPU_ERR_INVALID, "column index out of range");
            const int t = cols[in.arg].dtype;
            if (!numeric_or_bool(t)) return fail(PLGPU_ERR_SCHEMA, "unsupported column dtype in expression");
            L.emit(D_COL, in.arg);
            push(t, -1, false);
            break;
        }
        case PLGPU_OP_LIT_F64:
            L.emit(D_LIT, 0, bits_of(in.imm.f64));
            push(TY_LIT_FLOAT, (int)L.code.size() - 1, true, 0, in.imm.f64);
            break;
        case PLGPU_OP_LIT_I64:
            L.emit(D_LIT, 0, (uint64_t)in.imm.i64);
            push(TY_LIT_INT, (int)L.code.size() - 1, true, in.imm.i64);
            break;
        case PLGPU_OP_LIT_BOOL:
            L.emit(D_LIT, 0, in.imm.i64 ? 1ull : 0ull);
            push(PLGPU_BOOL, -1, true);
            break;
        case PLGPU_OP_LIT_NULL: {
            L.emit(D_NULL);
            if (in.arg == 0) push(TY_NULL, (int)L.code.size() - 1, true);
            else if (numeric_or_bool(in.arg)) push(in.arg, -1, true);
            else return fail(PLGPU_ERR_SCHEMA, "typed null literal needs a numeric / Boolean dtype");
            break;
        }
        case PLGPU_OP_ADD:
        case PLGPU_OP_SUB:
        case PLGPU_OP_MUL:
        case PLGPU_OP_TRUEDIV:
        case PLGPU_OP_FLOORDIV:
        case PLGPU_OP_MOD:
        case PLGPU_OP_DIVIDE: {
            if (!need(2)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            Ent a = st[st.size() - 2], b = st.back();
            if (a.ty == PLGPU_BOOL || b.ty == PLGPU_BOOL)
                return fail(PLGPU_ERR_INVALID, "arithmetic on Boolean is not supported");
            int t = L.join(a, b);
            if (!t) return fail(PLGPU_ERR_SCHEMA, "arithmetic operands have no common numeric type");
            if (t == PLGPU_BOOL) t = PLGPU_I32;  // null op null
            const bool divide = in.op == PLGPU_OP_TRUEDIV || (in.op == PLGPU_OP_DIVIDE && is_float(t));
            if (in.op == PLGPU_OP_TRUEDIV && !is_float(t)) t = PLGPU_F64;  // ints -> Float64
            L.coerce(1, t);
            L.coerce(0, t);
            const bool bscalar = b.scalar && !a.scalar;  // x op scalar (a broadcast divisor)
            int32_t dop;
            bool wrap = false;
            if (is_float(t)) {
                switch (in.op) {
                case PLGPU_OP_ADD: dop = D_ADD_F; break;
                case PLGPU_OP_SUB: dop = D_SUB_F; break;
                case PLGPU_OP_MUL: dop = D_MUL_F; break;
                case PLGPU_OP_FLOORDIV: dop = bscalar ? D_FLOORDIV_FS : D_FLOORDIV_F; break;
                case PLGPU_OP_MOD: dop = bscalar ? D_MOD_FS : D_MOD_F; break;
                default: dop = bscalar ? D_DIV_FS : D_DIV_F; break;  // true / legacy division
                }
                (void)divide;
                L.emit(dop, t);
            } else {
                wrap = t != PLGPU_I64 && t != PLGPU_U64;
                switch (in.op) {
                case PLGPU_OP_ADD: L.emit(D_ADD_I, t); break;
                case PLGPU_OP_SUB: L.emit(D_SUB_I, t); break;
                case PLGPU_OP_MUL: L.emit(D_MUL_I, t); break;
                case PLGPU_OP_MOD: L.emit(D_MOD_I, t == PLGPU_U64 ? 1 : 0); break;
                default: L.emit(D_FLOORDIV_I, t == PLGPU_U64 ? 1 : 0); break;  // floor / legacy division
                }
                if (wrap) L.emit(D_WRAP, t);
            }
            st.pop_back();
            st.back().ty = t;
            st.back().lit_pos = -1;
            st.back().scalar = a.scalar && b.scalar;
            break;
        }
        case PLGPU_OP_NEG:
        case PLGPU_OP_ABS: {
            if (!need(1)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            Ent& a = st.back();
            if (a.ty == PLGPU_BOOL) return fail(PLGPU_ERR_INVALID, "neg/abs on Boolean is not supported");
            if (Lowering::pending(a) && a.ty != TY_NULL) {
                // fold into the dynamic literal
                DevInstr& d = L.code[a.lit_pos];
                if (a.ty == TY_LIT_INT) {
                    a.ival = in.op == PLGPU_OP_NEG ? (int64_t)(0ull - (uint64_t)a.ival)
                                                   : (a.ival < 0 ? (int64_t)(0ull - (uint64_t)a.ival) : a.ival);
                    d.imm = (uint64_t)a.ival;
                } else {
                    a.fval = in.op == PLGPU_OP_NEG ? -a.fval : std::fabs(a.fval);
                    d.imm = bits_of(a.fval);
                }
                break;
            }
            if (a.ty == TY_NULL) L.settle(a, PLGPU_I32);
            if (in.op == PLGPU_OP_NEG && is_uint(a.ty))  // py-polars test_neg.py:57
                return fail(PLGPU_ERR_INVALID, "`neg` operation not supported for unsigned integer dtypes");
            if (is_float(a.ty)) {
                L.emit(in.op == PLGPU_OP_NEG ? D_NEG_F : D_ABS_F);
            } else {
                L.emit(in.op == PLGPU_OP_NEG ? D_NEG_I : D_ABS_I);
                if (a.ty != PLGPU_I64 && a.ty != PLGPU_U64) L.emit(D_WRAP, a.ty);
            }
            break;
        }
        case PLGPU_OP_CAST_F64:
        case PLGPU_OP_CAST: {
            if (!need(1)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            const int to = in.op == PLGPU_OP_CAST_F64 ? PLGPU_F64 : in.arg;
            const bool overflowing = in.op == PLGPU_OP_CAST && (in.imm.i64 & 1);
            if (!numeric_or_bool(to)) return fail(PLGPU_ERR_SCHEMA, "cast target must be numeric or Boolean");
            Ent& a = st.back();
            if (Lowering::pending(a)) {
                // a literal cast: settle in its own materialized type, then cast
                L.settle(a, a.ty == TY_NULL ? to : Lowering::lit_alone(a));
            }
            if (a.ty != to) L.emit(D_CAST, to, ((uint64_t)a.ty << 8) | (overflowing ? 1ull : 0ull));
            a.ty = to;
            break;
        }
        case PLGPU_OP_EQ: case PLGPU_OP_NE: case PLGPU_OP_LT: case PLGPU_OP_LE: case PLGPU_OP_GT:
        case PLGPU_OP_GE: case PLGPU_OP_EQ_MISSING: case PLGPU_OP_NE_MISSING: {
            if (!need(2)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            Ent a = st[st.size() - 2], b = st.back();
            const bool missing = in.op == PLGPU_OP_EQ_MISSING || in.op == PLGPU_OP_NE_MISSING;
            const int ci = missing ? (in.op == PLGPU_OP_EQ_MISSING ? 0 : 1) : cmp_index(in.op);
            if ((a.ty == PLGPU_BOOL) != (b.ty == PLGPU_BOOL) && !Lowering::pending(a) && !Lowering::pending(b))
                return fail(PLGPU_ERR_SCHEMA, "cannot compare Boolean with numeric");
            int t = L.join(a, b);
            if (!t) return fail(PLGPU_ERR_SCHEMA, "comparison operands have no common type");
            if ((a.ty == PLGPU_BOOL || b.ty == PLGPU_BOOL)) t = PLGPU_BOOL;
            L.coerce(1, t);
            L.coerce(0, t);
            if (t == PLGPU_BOOL) {
                if (ci > 1) return fail(PLGPU_ERR_INVALID, "ordering comparison on Boolean not supported");
                L.emit(missing ? (ci == 0 ? D_EQM_B : D_NEM_B) : (ci == 0 ? D_EQ_B : D_NE_B));
            } else if (is_float(t)) {
                L.emit(missing ? (ci == 0 ? D_EQM_F : D_NEM_F) : D_EQ_F + ci);
            } else if (t == PLGPU_U64) {
                L.emit(missing ? (ci == 0 ? D_EQM_I : D_NEM_I) : D_EQ_U + ci);
            } else {
                L.emit(missing ? (ci == 0 ? D_EQM_I : D_NEM_I) : D_EQ_I + ci);
            }
            st.pop_back();
            st.back().ty = PLGPU_BOOL;
            st.back().lit_pos = -1;
            st.back().scalar = a.scalar && b.scalar;
            break;
        }
        case PLGPU_OP_AND:
        case PLGPU_OP_OR:
        case PLGPU_OP_XOR: {
            if (!need(2)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            Ent a = st[st.size() - 2], b = st.back();
            const bool ba = a.ty == PLGPU_BOOL || a.ty == TY_NULL, bb = b.ty == PLGPU_BOOL || b.ty == TY_NULL;
            if (ba && bb) {
                L.coerce(1, PLGPU_BOOL);
                L.coerce(0, PLGPU_BOOL);
                L.emit(in.op == PLGPU_OP_AND ? D_AND : in.op == PLGPU_OP_OR ? D_OR : D_XOR);
                st.pop_back();
                st.back().ty = PLGPU_BOOL;
            } else {
                int t = L.join(a, b);
                if (!t || !is_int(t)) return fail(PLGPU_ERR_SCHEMA, "and/or/xor need Boolean or integer operands");
                L.coerce(1, t);
                L.coerce(0, t);
                L.emit(in.op == PLGPU_OP_AND ? D_BAND : in.op == PLGPU_OP_OR ? D_BOR : D_BXOR);
                st.pop_back();
                st.back().ty = t;
            }
            st.back().lit_pos = -1;
            st.back().scalar = a.scalar && b.scalar;
            break;
        }
        case PLGPU_OP_FILL_NULL: {
            if (!need(2)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            Ent a = st[st.size() - 2], b = st.back();
            int t = L.join(a, b);
            if (!t) return fail(PLGPU_ERR_SCHEMA, "fill_null: value has no common type with the column");
            L.coerce(1, t);
            L.coerce(0, t);
            L.emit(D_FILL_NULL);
            st.pop_back();
            st.back().ty = t;
            st.back().lit_pos = -1;
            st.back().scalar = a.scalar && b.scalar;
            break;
        }
        case PLGPU_OP_IF_ELSE: {
            if (!need(3)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            Ent c = st[st.size() - 3], a = st[st.size() - 2], b = st.back();
            if (c.ty != PLGPU_BOOL && c.ty != TY_NULL)
                return fail(PLGPU_ERR_SCHEMA, "when() condition must be Boolean");
            if (Lowering::pending(c)) L.settle(st[st.size() - 3], PLGPU_BOOL);
            int t = L.join(a, b);
            if (!t) return fail(PLGPU_ERR_SCHEMA, "then() and otherwise() have no common type");
            L.coerce(1, t);
            L.coerce(0, t);
            L.emit(D_IF_ELSE);
            st.pop_back();
            st.pop_back();
            st.back().ty = t;
            st.back().lit_pos = -1;
            st.back().scalar = c.scalar && a.scalar && b.scalar;
            break;
        }
        case PLGPU_OP_NOT:
            if (!need(1)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            if (st.back().ty == TY_NULL) L.settle(st.back(), PLGPU_BOOL);
            if (st.back().ty == PLGPU_BOOL) {
                L.emit(D_NOT);
            } else if (is_int(st.back().ty)) {  // bitwise not of an integer: x ^ ~0
                L.emit(D_LIT, 0, ~0ull);
                L.emit(D_BXOR);
                if (st.back().ty != PLGPU_I64 && st.back().ty != PLGPU_U64) L.emit(D_WRAP, st.back().ty);
            } else {
                return fail(PLGPU_ERR_SCHEMA, "not needs a Boolean operand");
            }
            break;
        case PLGPU_OP_IS_NULL:
        case PLGPU_OP_IS_NOT_NULL:
            if (!need(1)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            if (Lowering::pending(st.back())) L.settle(st.back(), Lowering::lit_alone(st.back()));
            L.emit(in.op == PLGPU_OP_IS_NULL ? D_ISNULL : D_ISNOTNULL);
            st.back().ty = PLGPU_BOOL;
            break;
        case PLGPU_OP_IS_NAN:
        case PLGPU_OP_IS_FINITE:
            if (!need(1)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            if (st.back().ty == TY_LIT_FLOAT) L.settle(st.back(), PLGPU_F64);
            if (!is_float(st.back().ty))
                return fail(PLGPU_ERR_INVALID, "is_nan/is_finite operation not supported for non-float dtype");
            L.emit(in.op == PLGPU_OP_IS_NAN ? D_ISNAN_F : D_ISFINITE_F);
            st.back().ty = PLGPU_BOOL;
            break;
        default: return fail(PLGPU_ERR_INVALID, "unknown opcode " + std::to_string(in.op));
        }
        if (st.size() > PLGPU_MAX_STACK) return fail(PLGPU_ERR_INVALID, "expression stack too deep");
        if ((int)L.code.size() > PLGPU_MAX_PROGRAM) return fail(PLGPU_ERR_INVALID, "lowered program too long");
    }
    if (st.size() != 1) return fail(PLGPU_ERR_INVALID, "program must leave exactly one value");
    if (Lowering::pending(st[0])) L.settle(st[0], Lowering::lit_alone(st[0]));
    const auto& code = L.code;
    out->n = (int32_t)code.size();
    for (size_t i = 0; i < code.size(); ++i) out->code[i] = code[i];
    out->out_dtype = st[0].ty;
    // Fast path: the lowered program is exactly [COL c, LIT x, CMP] (no
    // casts): the predicate compares the register form with x directly.
    if (code.size() == 3 && code[0].op == D_COL && code[1].op == D_LIT) {
        const int op = code[2].op;
        if (op >= D_EQ_F && op <= D_GE_F) {
            out->simple = 1;
            out->simple_isf = 1;
            out->simple_op = op - D_EQ_F;
        } else if (op >= D_EQ_I && op <= D_GE_I) {
            out->simple = 1;
            out->simple_isf = 0;
            out->simple_op = op - D_EQ_I;
        }
        if (out->simple) {
            out->simple_col = code[0].arg;
            out->simple_imm = code[1].imm;
        }
    }
    return PLGPU_OK;
}

}  // namespace plgpu

using namespace plgpu;

PLGPU_API int plgpu_abi_version(void) { return PLGPU_ABI_VERSION; }

PLGPU_API const char* plgpu_last_error(void) { return g_last_error.c_str(); }

PLGPU_API int plgpu_device_count(int* out) {
    *out = 0;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(PLGPU_ERR_NO_DEVICE, "no HIP device visible");
    }
    *out = n;
    return PLGPU_OK;
}

PLGPU_API int plgpu_set_device(int device) {
    PLGPU_HIP(hipSetDevice(device));
    return PLGPU_OK;
}

PLGPU_API int plgpu_synchronize(void* stream) {
    PLGPU_HIP(hipStreamSynchronize(as_stream(stream)));
    return PLGPU_OK;
}

PLGPU_API int plgpu_alloc(void** out_ptr, size_t bytes, void* stream) {
    return dev_alloc(out_ptr, bytes, as_stream(stream));
}

PLGPU_API int plgpu_free(void* ptr, void* stream) {
    dev_free(ptr, as_stream(stream));
    return PLGPU_OK;
}

PLGPU_API int plgpu_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
    PLGPU_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, as_stream(stream)));
    PLGPU_HIP(hipStreamSynchronize(as_stream(stream)));
    return PLGPU_OK;
}

PLGPU_API int plgpu_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream) {
    PLGPU_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, as_stream(stream)));
    PLGPU_HIP(hipStreamSynchronize(as_stream(stream)));
    return PLGPU_OK;
}

// Small device -> host downloads batched through one pinned staging buffer
// (library-owned, grown on demand up to kD2hStageMax): every range's copy is
// queued on the stream, then one synchronisation and host copies out.  A
// range larger than the cap is copied on its own.  A query's result columns
// (a few KB each) come back in one round trip instead of one per buffer.
namespace {
constexpr size_t kD2hStageMax = size_t(64) << 20;
std::mutex g_stage_mu;
void* g_stage = nullptr;
size_t g_stage_bytes = 0;
}  // namespace

PLGPU_API int plgpu_memcpy_d2h_many(int32_t n, void* const* dst, const void* const* src, const size_t* bytes,
                                    void* stream) {
    if (n < 0 || (n > 0 && (dst == nullptr || src == nullptr || bytes == nullptr)))
        return fail(PLGPU_ERR_INVALID, "memcpy_d2h_many: bad arguments");
    hipStream_t s = as_stream(stream);
    size_t total = 0;
    for (int32_t i = 0; i < n; ++i)
        if (bytes[i] <= kD2hStageMax) total += (bytes[i] + 255) & ~size_t(255);
    std::lock_guard<std::mutex> lk(g_stage_mu);
    if (total > kD2hStageMax) total = 0;  // too much for the stage: direct copies
    if (total > g_stage_bytes) {
        if (g_stage) (void)hipHostFree(g_stage);
        g_stage = nullptr;
        g_stage_bytes = 0;
        const size_t want = std::max<size_t>(total, size_t(1) << 20);
        if (hipHostMalloc(&g_stage, want, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            g_stage = nullptr;
            total = 0;
        } else {
            g_stage_bytes = want;
        }
    }
    size_t off = 0;
    for (int32_t i = 0; i < n; ++i) {
        if (bytes[i] == 0) continue;
        if (total > 0 && bytes[i] <= kD2hStageMax) {
            PLGPU_HIP(hipMemcpyAsync((char*)g_stage + off, src[i], bytes[i], hipMemcpyDeviceToHost, s));
            off += (bytes[i] + 255) & ~size_t(255);
        } else {
            PLGPU_HIP(hipMemcpyAsync(dst[i], src[i], bytes[i], hipMemcpyDeviceToHost, s));
        }
    }
    PLGPU_HIP(hipStreamSynchronize(s));
    off = 0;
    for (int32_t i = 0; i < n; ++i) {
        if (bytes[i] == 0 || !(total > 0 && bytes[i] <= kD2hStageMax)) continue;
        std::memcpy(dst[i], (const char*)g_stage + off, bytes[i]);
        off += (bytes[i] + 255) & ~size_t(255);
    }
    return PLGPU_OK;
}

PLGPU_API int plgpu_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream) {
    PLGPU_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, as_stream(stream)));
    return PLGPU_OK;
}

PLGPU_API int plgpu_expr_dtype(const plgpu_column* cols, int32_t ncols, const plgpu_instr* program, int32_t n_instr,
                               int32_t* out_dtype) {
    if (out_dtype == nullptr || (ncols > 0 && cols == nullptr)) return fail(PLGPU_ERR_INVALID, "NULL argument");
    DevProgram dp;
    const int rc = lower_program(cols, ncols, program, n_instr, &dp);
    if (rc) return rc;
    *out_dtype = dp.out_dtype;
    return PLGPU_OK;
}

PLGPU_API int plgpu_set_option(const char* name, int64_t value) {
    if (name == nullptr) return fail(PLGPU_ERR_INVALID, "option name is NULL");
    const OptField* f = opt_field(name);
    if (f == nullptr) return fail(PLGPU_ERR_INVALID, std::string("unknown option ") + name);
    options().*(f->f) = (int)value;
    return PLGPU_OK;
}

PLGPU_API int plgpu_get_option(const char* name, int64_t* out) {
    if (name == nullptr || out == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    const OptField* f = opt_field(name);
    if (f == nullptr) return fail(PLGPU_ERR_INVALID, std::string("unknown option ") + name);
    *out = options().*(f->f);
    return PLGPU_OK;
}

PLGPU_API int plgpu_release_cached(void) {
    int dev = 0;
    PLGPU_HIP(hipGetDevice(&dev));
    PLGPU_HIP(hipDeviceSynchronize());
    Pool& P = pool_for(dev);
    {
        std::lock_guard<std::mutex> lk(P.mu);
        release_cached(P);
    }
    gb_plan_cache_clear();  // the released addresses will hold other data
    return PLGPU_OK;
}

PLGPU_API int plgpu_ktime_read(char* buf, int64_t cap, int32_t reset) {
    if (buf == nullptr || cap <= 0) return fail(PLGPU_ERR_INVALID, "NULL argument");
    std::lock_guard<std::mutex> g(g_kt_mu);
    for (KtPending& p : g_kt_pending) {
        float ms = 0.f;
        const hipError_t e = hipEventSynchronize(p.b);
        if (e == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            auto it = std::find_if(g_kt_sums.begin(), g_kt_sums.end(), [&](const KtSum& k) { return k.name == p.name; });
            if (it == g_kt_sums.end()) it = g_kt_sums.insert(g_kt_sums.end(), KtSum{p.name, 0.0, 0});
            it->ms += ms;
            it->count += 1;
        }
        g_kt_pool.push_back(p.a);
        g_kt_pool.push_back(p.b);
    }
    g_kt_pending.clear();
    std::string out;
    char line[256];
    for (const KtSum& k : g_kt_sums) {
        snprintf(line, sizeof line, "%s\t%.6f\t%lld\n", k.name.c_str(), k.ms, (long long)k.count);
        out += line;
    }
    if (reset) g_kt_sums.clear();
    if ((int64_t)out.size() + 1 > cap) return fail(PLGPU_ERR_CAPACITY, "ktime buffer too small");
    std::memcpy(buf, out.c_str(), out.size() + 1);
    return PLGPU_OK;
}

PLGPU_API void plgpu_column_release(plgpu_column* col) {
    if (col && col->release) col->release(col);
}
