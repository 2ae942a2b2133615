// runtime.cpp — error plumbing, stream-ordered device allocator, copies,
// column ownership and host-side lowering of expression programs.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
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

// Caching device allocator.  Blocks come from hipMalloc and are recycled
// through size-keyed free lists instead of being returned with hipFree
// (which synchronises the device).  Every entry point enqueues its work on
// one stream and frees only after the kernels that use a block were
// enqueued, so stream order makes reuse safe.  (hipMallocAsync's default
// pool was measured to lose writes into a recycled block on this ROCm
// build, see DESIGN.md "Allocator"; it is not used.)
namespace {
struct Pool {
    std::mutex mu;
    std::multimap<size_t, void*> free_blocks;        // size -> ptr
    std::unordered_map<void*, size_t> sizes;         // every block we own
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
    const size_t want = round_bytes(bytes == 0 ? 256 : bytes);
    int dev = 0;
    (void)hipGetDevice(&dev);
    Pool& P = pool_for(dev);
    std::lock_guard<std::mutex> lk(P.mu);
    auto it = P.free_blocks.lower_bound(want);
    if (it != P.free_blocks.end() && it->first <= want + want / 4) {
        *p = it->second;
        P.cached -= it->first;
        P.free_blocks.erase(it);
        return PLGPU_OK;
    }
    hipError_t e = hipMalloc(p, want);
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
    return PLGPU_OK;
}

void dev_free(void* p, hipStream_t s) {
    (void)s;
    if (p == nullptr) return;
    int dev = 0;
    (void)hipGetDevice(&dev);
    Pool& P = pool_for(dev);
    std::lock_guard<std::mutex> lk(P.mu);
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
namespace {
enum Ty { TB = 1, TI = 2, TF = 3 };

int col_ty(int32_t dt) {
    switch (dt) {
    case PLGPU_BOOL: return TB;
    case PLGPU_I32:
    case PLGPU_I64:
    case PLGPU_U32: return TI;
    case PLGPU_F64: return TF;
    default: return 0;
    }
}
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
uint64_t bits_of(double d) {
    uint64_t u;
    std::memcpy(&u, &d, 8);
    return u;
}
}  // namespace

int lower_program(const plgpu_column* cols, int32_t ncols, const plgpu_instr* prog, int32_t n,
                  DevProgram* out) {
    std::memset(out, 0, sizeof *out);
    if (n <= 0) return fail(PLGPU_ERR_INVALID, "empty expression program");
    if (n > PLGPU_MAX_PROGRAM) return fail(PLGPU_ERR_INVALID, "expression program too long");
    std::vector<int> st;  // type stack
    std::vector<DevInstr> code;
    auto emit = [&](int32_t op, int32_t arg = 0, uint64_t imm = 0) {
        DevInstr d;
        d.op = op;
        d.arg = arg;
        d.imm = imm;
        code.push_back(d);
    };
    for (int k = 0; k < n; ++k) {
        const plgpu_instr& in = prog[k];
        auto need = [&](size_t m) -> bool { return st.size() >= m; };
        switch (in.op) {
        case PLGPU_OP_COL: {
            if (in.arg < 0 || in.arg >= ncols) return fail(PLGPU_ERR_INVALID, "column index out of range");
            int t = col_ty(cols[in.arg].dtype);
            if (!t) return fail(PLGPU_ERR_SCHEMA, "unsupported column dtype in expression");
            int32_t dop = cols[in.arg].dtype == PLGPU_F64   ? D_COL_F64
                          : cols[in.arg].dtype == PLGPU_I64 ? D_COL_I64
                          : cols[in.arg].dtype == PLGPU_I32 ? D_COL_I32
                          : cols[in.arg].dtype == PLGPU_U32 ? D_COL_U32
                                                            : D_COL_BOOL;
            emit(dop, in.arg);
            st.push_back(t);
            break;
        }
        case PLGPU_OP_LIT_F64: emit(D_LIT, 0, bits_of(in.imm.f64)); st.push_back(TF); break;
        case PLGPU_OP_LIT_I64: emit(D_LIT, 0, (uint64_t)in.imm.i64); st.push_back(TI); break;
        case PLGPU_OP_LIT_BOOL: emit(D_LIT, 0, in.imm.i64 ? 1ull : 0ull); st.push_back(TB); break;
        case PLGPU_OP_LIT_NULL: {
            int t = col_ty(in.arg);
            if (!t) return fail(PLGPU_ERR_SCHEMA, "typed null literal needs a dtype");
            emit(D_NULL);
            st.push_back(t);
            break;
        }
        case PLGPU_OP_ADD:
        case PLGPU_OP_SUB:
        case PLGPU_OP_MUL:
        case PLGPU_OP_TRUEDIV: {
            if (!need(2)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            int b = st.back(); st.pop_back();
            int a = st.back(); st.pop_back();
            if (a == TB || b == TB)
                return fail(PLGPU_ERR_INVALID, "arithmetic on Boolean is not supported");
            bool fl = (a == TF || b == TF || in.op == PLGPU_OP_TRUEDIV);
            if (fl) {
                if (b == TI) emit(D_I2F_0);
                if (a == TI) emit(D_I2F_1);
                emit(in.op == PLGPU_OP_ADD ? D_ADD_F : in.op == PLGPU_OP_SUB ? D_SUB_F
                     : in.op == PLGPU_OP_MUL ? D_MUL_F : D_DIV_F);
                st.push_back(TF);
            } else {
                emit(in.op == PLGPU_OP_ADD ? D_ADD_I : in.op == PLGPU_OP_SUB ? D_SUB_I : D_MUL_I);
                st.push_back(TI);
            }
            break;
        }
        case PLGPU_OP_NEG:
        case PLGPU_OP_ABS: {
            if (!need(1)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            int a = st.back();
            if (a == TB) return fail(PLGPU_ERR_INVALID, "neg/abs on Boolean is not supported");
            emit(a == TF ? (in.op == PLGPU_OP_NEG ? D_NEG_F : D_ABS_F)
                         : (in.op == PLGPU_OP_NEG ? D_NEG_I : D_ABS_I));
            break;
        }
        case PLGPU_OP_CAST_F64: {
            if (!need(1)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            if (st.back() == TB) return fail(PLGPU_ERR_INVALID, "cast Boolean -> f64 not supported");
            if (st.back() == TI) emit(D_I2F_0);
            st.back() = TF;
            break;
        }
        case PLGPU_OP_EQ: case PLGPU_OP_NE: case PLGPU_OP_LT: case PLGPU_OP_LE: case PLGPU_OP_GT:
        case PLGPU_OP_GE: case PLGPU_OP_EQ_MISSING: case PLGPU_OP_NE_MISSING: {
            if (!need(2)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            int b = st.back(); st.pop_back();
            int a = st.back(); st.pop_back();
            bool missing = in.op == PLGPU_OP_EQ_MISSING || in.op == PLGPU_OP_NE_MISSING;
            int ci = missing ? (in.op == PLGPU_OP_EQ_MISSING ? 0 : 1) : cmp_index(in.op);
            if (a == TB || b == TB) {
                if (a != b) return fail(PLGPU_ERR_SCHEMA, "cannot compare Boolean with numeric");
                if (ci > 1) return fail(PLGPU_ERR_INVALID, "ordering comparison on Boolean not supported");
                emit(missing ? (ci == 0 ? D_EQM_B : D_NEM_B) : (ci == 0 ? D_EQ_B : D_NE_B));
            } else if (a == TF || b == TF) {
                if (b == TI) emit(D_I2F_0);
                if (a == TI) emit(D_I2F_1);
                emit(missing ? (ci == 0 ? D_EQM_F : D_NEM_F) : D_EQ_F + ci);
            } else {
                emit(missing ? (ci == 0 ? D_EQM_I : D_NEM_I) : D_EQ_I + ci);
            }
            st.push_back(TB);
            break;
        }
        case PLGPU_OP_AND:
        case PLGPU_OP_OR: {
            if (!need(2)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            int b = st.back(); st.pop_back();
            int a = st.back(); st.pop_back();
            if (a != TB || b != TB) return fail(PLGPU_ERR_SCHEMA, "and/or need Boolean operands");
            emit(in.op == PLGPU_OP_AND ? D_AND : D_OR);
            st.push_back(TB);
            break;
        }
        case PLGPU_OP_NOT:
            if (!need(1)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            if (st.back() != TB) return fail(PLGPU_ERR_SCHEMA, "not needs a Boolean operand");
            emit(D_NOT);
            break;
        case PLGPU_OP_IS_NULL:
        case PLGPU_OP_IS_NOT_NULL:
            if (!need(1)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            emit(in.op == PLGPU_OP_IS_NULL ? D_ISNULL : D_ISNOTNULL);
            st.back() = TB;
            break;
        case PLGPU_OP_IS_NAN:
        case PLGPU_OP_IS_FINITE:
            if (!need(1)) return fail(PLGPU_ERR_INVALID, "stack underflow");
            if (st.back() != TF)
                return fail(PLGPU_ERR_INVALID, "is_nan/is_finite operation not supported for non-float dtype");
            emit(in.op == PLGPU_OP_IS_NAN ? D_ISNAN_F : D_ISFINITE_F);
            st.back() = TB;
            break;
        default: return fail(PLGPU_ERR_INVALID, "unknown opcode " + std::to_string(in.op));
        }
        if (st.size() > PLGPU_MAX_STACK) return fail(PLGPU_ERR_INVALID, "expression stack too deep");
        if ((int)code.size() > PLGPU_MAX_PROGRAM) return fail(PLGPU_ERR_INVALID, "lowered program too long");
    }
    if (st.size() != 1) return fail(PLGPU_ERR_INVALID, "program must leave exactly one value");
    out->n = (int32_t)code.size();
    for (size_t i = 0; i < code.size(); ++i) out->code[i] = code[i];
    out->out_dtype = st[0] == TB ? PLGPU_BOOL : st[0] == TI ? PLGPU_I64 : PLGPU_F64;
    // Fast path detection: exactly [COL c, LIT x, CMP] with matching types.
    if (n == 3 && prog[0].op == PLGPU_OP_COL && cmp_index(prog[2].op) >= 0 &&
        (prog[1].op == PLGPU_OP_LIT_F64 || prog[1].op == PLGPU_OP_LIT_I64)) {
        int ct = col_ty(cols[prog[0].arg].dtype);
        if (ct == TF) {
            out->simple = 1;
            out->simple_isf = 1;
            double v = prog[1].op == PLGPU_OP_LIT_F64 ? prog[1].imm.f64 : (double)prog[1].imm.i64;
            out->simple_imm = bits_of(v);
        } else if (ct == TI && prog[1].op == PLGPU_OP_LIT_I64) {
            out->simple = 1;
            out->simple_isf = 0;
            out->simple_imm = (uint64_t)prog[1].imm.i64;
        }
        if (out->simple) {
            out->simple_col = prog[0].arg;
            out->simple_op = cmp_index(prog[2].op);
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

PLGPU_API int plgpu_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream) {
    PLGPU_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, as_stream(stream)));
    return PLGPU_OK;
}

PLGPU_API void plgpu_column_release(plgpu_column* col) {
    if (col && col->release) col->release(col);
}
