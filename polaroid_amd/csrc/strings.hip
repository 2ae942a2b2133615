// String columns (Arrow large_string: int64 offsets + UTF-8 bytes): the
// variable-length gather that materialises them after a join, a sort, a
// filter or as group-by output keys.
//
// Reference: polars-core/src/chunked_array/ops/gather.rs (take on
// BinaryView / Utf8View arrays) and polars-compute/src/filter (filtering the
// same).  The reference stores strings as views; the Arrow interchange the
// GPU executor reads and writes is large_string, so the GPU works on offsets
// and bytes.
//
// MI355X design: three passes over the output rows -- lengths (+ validity
// ballots), an exclusive scan into the output offsets, then the byte copy.
// The copy gives every string one thread for short strings and a whole wave
// for long ones (8-byte lane words when source and destination agree on
// alignment), so symbol-like keys (4..16 bytes) and long payloads both
// stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "plgpu_internal.hpp"
#include "scan.hpp"

namespace plgpu {

constexpr int kStrThreads = 256;
constexpr int64_t kStrLongBytes = 256;  // strings this long are copied by a whole wave

__device__ __forceinline__ bool str_idx(const uint32_t* idx32, const int64_t* idx64, const uint8_t* iv, int64_t ioff,
                                        int64_t i, int64_t* r) {
    if (iv != nullptr && !((iv[(ioff + i) >> 3] >> ((ioff + i) & 7)) & 1)) return false;
    *r = idx32 ? (int64_t)idx32[i] : idx64[i];
    return true;
}

// lens[i] = byte length of output row i (0 for a null); validity ballots.
__global__ __launch_bounds__(kStrThreads) void str_len_kernel(DevCol src, const uint32_t* __restrict__ idx32,
                                                              const int64_t* __restrict__ idx64,
                                                              const uint8_t* __restrict__ iv, int64_t ioff,
                                                              int64_t n, uint64_t* __restrict__ lens,
                                                              uint64_t* __restrict__ out_valid) {
    const int64_t* off = (const int64_t*)src.values;
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < n; i0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = i0 + threadIdx.x;
        bool valid = false;
        uint64_t len = 0;
        int64_t r;
        if (i < n && str_idx(idx32, idx64, iv, ioff, i, &r) && dev_valid(src, r)) {
            valid = true;
            len = (uint64_t)(off[src.offset + r + 1] - off[src.offset + r]);
        }
        if (i < n) lens[i] = len;
        if (out_valid) {
            const uint64_t w = __ballot(valid);
            if ((threadIdx.x & 63) == 0 && i < n) out_valid[i >> 6] = w;
        }
    }
}

__device__ __forceinline__ void copy_bytes_lane(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, int64_t len,
                                                int lane, int lanes) {
    if ((((uintptr_t)s ^ (uintptr_t)d) & 7) == 0) {
        // same alignment: head bytes, 8-byte words, tail bytes
        int64_t head = (int64_t)((8 - ((uintptr_t)s & 7)) & 7);
        if (head > len) head = len;
        for (int64_t j = lane; j < head; j += lanes) d[j] = s[j];
        const int64_t words = (len - head) >> 3;
        const uint64_t* sw = (const uint64_t*)(s + head);
        uint64_t* dw = (uint64_t*)(d + head);
        for (int64_t j = lane; j < words; j += lanes) dw[j] = sw[j];
        for (int64_t j = head + (words << 3) + lane; j < len; j += lanes) d[j] = s[j];
    } else {
        for (int64_t j = lane; j < len; j += lanes) d[j] = s[j];
    }
}

// Short strings: one thread each.  Long ones are queued for the wave copy.
__global__ __launch_bounds__(kStrThreads) void str_copy_kernel(DevCol src, const uint32_t* __restrict__ idx32,
                                                               const int64_t* __restrict__ idx64,
                                                               const uint8_t* __restrict__ iv, int64_t ioff, int64_t n,
                                                               const uint64_t* __restrict__ out_off,
                                                               uint8_t* __restrict__ out_data,
                                                               int64_t* __restrict__ long_rows,
                                                               unsigned long long* __restrict__ nlong) {
    const int64_t* off = (const int64_t*)src.values;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t len = (int64_t)(out_off[i + 1] - out_off[i]);
        if (len == 0) continue;
        if (len >= kStrLongBytes) {
            long_rows[atomicAdd(nlong, 1ull)] = i;
            continue;
        }
        int64_t r;
        (void)str_idx(idx32, idx64, iv, ioff, i, &r);
        copy_bytes_lane(src.data + off[src.offset + r], out_data + out_off[i], len, 0, 1);
    }
}

__global__ __launch_bounds__(kStrThreads) void str_copy_long_kernel(DevCol src, const uint32_t* __restrict__ idx32,
                                                                    const int64_t* __restrict__ idx64,
                                                                    const uint64_t* __restrict__ out_off,
                                                                    uint8_t* __restrict__ out_data,
                                                                    const int64_t* __restrict__ long_rows,
                                                                    int64_t nlong) {
    const int64_t* off = (const int64_t*)src.values;
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t waves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t k = wave; k < nlong; k += waves) {
        const int64_t i = long_rows[k];
        const int64_t r = idx32 ? (int64_t)idx32[i] : idx64[i];
        copy_bytes_lane(src.data + off[src.offset + r], out_data + out_off[i], (int64_t)(out_off[i + 1] - out_off[i]),
                        lane, 64);
    }
}

static int num_cus_str() {
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

// out = src[idx] for a PLGPU_STR column; idx is UInt32 (idx32) or Int64
// (idx64) row ids; `iv` / `ioff`: optional index validity (a null index
// gathers a null).  The output is library-owned.
int str_gather(const DevCol& src, const uint32_t* idx32, const int64_t* idx64, const uint8_t* iv, int64_t ioff,
               int64_t n, bool nullable, plgpu_column* out, hipStream_t s) {
    int rc = make_owned_column(out, PLGPU_I64, n + 1, nullable, s);  // offsets (+ validity)
    if (rc) return rc;
    uint64_t* lens = nullptr;
    uint64_t* part = nullptr;
    int64_t* long_rows = nullptr;
    unsigned long long* nlong = nullptr;
    uint64_t total = 0;
    const int g = (int)std::max<int64_t>(1, std::min<int64_t>((n + kStrThreads - 1) / kStrThreads,
                                                              (int64_t)num_cus_str() * 16));
    rc = dev_alloc((void**)&lens, std::max<int64_t>(n, 1) * 8, s);
    if (!rc) rc = dev_alloc((void**)&part, ((n + kScanChunk - 1) / kScanChunk + 2) * 8, s);
    uint64_t* out_off = (uint64_t*)out->values;
    if (!rc) {
        if (n > 0)
            str_len_kernel<<<g, kStrThreads, 0, s>>>(src, idx32, idx64, iv, ioff, n, lens,
                                                     (uint64_t*)out->validity);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = scan_exclusive<uint64_t>(lens, n, out_off, part, s);
        if (e == hipSuccess) e = hipMemcpyAsync(&total, out_off + n, 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "string gather lengths");
    }
    if (!rc) rc = owned_attach_data(out, (int64_t)total, s);
    if (!rc && total > 0) {
        rc = dev_alloc((void**)&long_rows, n * 8, s);
        if (!rc) rc = dev_alloc((void**)&nlong, 8, s);
        unsigned long long hl = 0;
        hipError_t e = hipSuccess;
        if (!rc) {
            e = hipMemsetAsync(nlong, 0, 8, s);
            if (e == hipSuccess) {
                str_copy_kernel<<<g, kStrThreads, 0, s>>>(src, idx32, idx64, iv, ioff, n, out_off,
                                                          (uint8_t*)out->data, long_rows, nlong);
                e = hipGetLastError();
            }
            if (e == hipSuccess) e = hipMemcpyAsync(&hl, nlong, 8, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e == hipSuccess && hl > 0) {
                const int gl = (int)std::min<int64_t>(((int64_t)hl * 64 + kStrThreads - 1) / kStrThreads,
                                                      (int64_t)num_cus_str() * 16);
                str_copy_long_kernel<<<gl, kStrThreads, 0, s>>>(src, idx32, idx64, out_off, (uint8_t*)out->data,
                                                                long_rows, (int64_t)hl);
                e = hipGetLastError();
            }
            if (e != hipSuccess) rc = hip_fail(e, "string gather copy");
        }
    }
    if (!rc) {
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "string gather");
    }
    dev_free(lens, s);
    dev_free(part, s);
    dev_free(long_rows, s);
    dev_free(nlong, s);
    if (rc) plgpu_column_release(out);
    return rc;
}

// ------------------------------------------------ short-string key codes
// A string of at most 7 bytes is encoded exactly and injectively as one
// integer: (length << 56) | bytes (little-endian).  A key column whose
// strings are all that short is then grouped / joined as an Int64 column --
// exact, with no hashing, no byte verification and no collision path
// (symbols, tickers, country codes).  *any_long reports a longer string.
// `words`: the data buffer is 8-byte aligned and `data_end` (= the last
// offset) bounds the aligned 8-byte word loads, so a string's bytes come in
// one or two word loads and a funnel shift instead of byte loads.
// `out_valid` (optional): the strings' validity re-based to offset 0, one
// ballot word per 64 rows.
__global__ __launch_bounds__(kStrThreads) void str_code_kernel(DevCol src, int64_t n, uint64_t* __restrict__ codes,
                                                               unsigned long long* __restrict__ any_long,
                                                               bool words, int64_t data_end,
                                                               uint64_t* __restrict__ out_valid) {
    const int64_t* off = (const int64_t*)src.values;
    const uint64_t* dw = (const uint64_t*)src.data;
    bool lng = false;
    for (int64_t r0 = (int64_t)blockIdx.x * blockDim.x; r0 < n; r0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = r0 + threadIdx.x;
        const bool vr = r < n && dev_valid(src, r);
        if (out_valid) {
            const uint64_t wv = __ballot(vr);
            if ((threadIdx.x & 63) == 0 && r < n) out_valid[r >> 6] = wv;
        }
        if (r >= n) continue;
        uint64_t code = 0;
        if (vr) {
            const int64_t b = off[src.offset + r], len = off[src.offset + r + 1] - b;
            if (len > 7) {
                lng = true;
            } else if (len > 0) {
                const int64_t w = b >> 3;
                const int sh = (int)(b & 7) * 8;
                uint64_t x;
                if (words && (w + 1) * 8 <= data_end && (sh + 8 * len <= 64 || (w + 2) * 8 <= data_end)) {
                    const uint64_t lo = dw[w];
                    x = lo >> sh;
                    if (sh + 8 * len > 64) x |= dw[w + 1] << (64 - sh);
                } else {
                    x = 0;
                    for (int j = 0; j < len; ++j) x |= (uint64_t)src.data[b + j] << (8 * j);
                }
                code = ((uint64_t)len << 56) | (x & ((1ull << (8 * len)) - 1));
            }
        }
        codes[r] = code;
    }
    if (__any(lng) && (threadIdx.x & 63) == 0) atomicOr(any_long, 1ull);
}

// Codes -> strings: lengths, scan, bytes.
__global__ __launch_bounds__(kStrThreads) void str_code_len_kernel(DevCol codes, int64_t n, uint64_t* __restrict__ lens,
                                                                   uint64_t* __restrict__ out_valid) {
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < n; i0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = i0 + threadIdx.x;
        const bool v = i < n && dev_valid(codes, i);
        if (i < n) lens[i] = v ? (dev_load(codes, i) >> 56) : 0;
        if (out_valid) {
            const uint64_t w = __ballot(v);
            if ((threadIdx.x & 63) == 0 && i < n) out_valid[i >> 6] = w;
        }
    }
}

__global__ __launch_bounds__(kStrThreads) void str_code_bytes_kernel(DevCol codes, int64_t n,
                                                                     const uint64_t* __restrict__ out_off,
                                                                     uint8_t* __restrict__ out_data) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t len = (int64_t)(out_off[i + 1] - out_off[i]);
        if (len == 0) continue;
        const uint64_t c = dev_load(codes, i);
        for (int j = 0; j < len; ++j) out_data[out_off[i] + j] = (uint8_t)(c >> (8 * j));
    }
}

int str_short_codes(const plgpu_column& src, plgpu_column* out, bool* all_short, hipStream_t s) {
    const int64_t n = src.length;
    std::memset(out, 0, sizeof *out);
    uint64_t* codes = nullptr;
    unsigned long long* flag = nullptr;
    int rc = dev_alloc((void**)&codes, std::max<int64_t>(n, 1) * 8, s);
    if (!rc) rc = dev_alloc((void**)&flag, 8, s);
    unsigned long long hf = 0;
    if (!rc) {
        int64_t data_end = 0;
        hipError_t e = hipMemsetAsync(flag, 0, 8, s);
        if (e == hipSuccess && n > 0)
            e = hipMemcpyAsync(&data_end, (const int64_t*)src.values + src.offset + n, 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e == hipSuccess && n > 0) {
            const int g = (int)std::min<int64_t>((n + kStrThreads - 1) / kStrThreads, (int64_t)num_cus_str() * 16);
            const bool words = ((uintptr_t)src.data & 7) == 0;
            {
                KtScope kt("str_code_kernel", s);
                str_code_kernel<<<g, kStrThreads, 0, s>>>(dev_col(src), n, codes, flag, words, data_end, nullptr);
            }
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(&hf, flag, 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "short-string codes");
    }
    dev_free(flag, s);
    if (rc) {
        dev_free(codes, s);
        return rc;
    }
    *all_short = hf == 0;
    // same validity bitmap and offset as the strings: values[offset + r] is
    // the code of row r
    out->dtype = PLGPU_I64;
    out->length = n;
    out->offset = src.offset;
    out->null_count = src.null_count;
    out->validity = src.validity;
    out->values = codes - src.offset;
    out->private_data = codes;  // the allocation (free with str_codes_free)
    return PLGPU_OK;
}

void str_codes_free(plgpu_column* c, hipStream_t s) {
    if (c && c->private_data) dev_free(c->private_data, s);
    if (c) std::memset(c, 0, sizeof *c);
}

int str_from_codes(const plgpu_column& codes, plgpu_column* out, hipStream_t s) {
    const int64_t n = codes.length;
    const bool nullable = codes.validity != nullptr;
    int rc = make_owned_column(out, PLGPU_I64, n + 1, nullable, s);
    if (rc) return rc;
    uint64_t* lens = nullptr;
    uint64_t* part = nullptr;
    uint64_t total = 0;
    const int g = (int)std::max<int64_t>(1, std::min<int64_t>((n + kStrThreads - 1) / kStrThreads,
                                                              (int64_t)num_cus_str() * 16));
    const DevCol dc = dev_col(codes);
    rc = dev_alloc((void**)&lens, std::max<int64_t>(n, 1) * 8, s);
    if (!rc) rc = dev_alloc((void**)&part, ((n + kScanChunk - 1) / kScanChunk + 2) * 8, s);
    uint64_t* out_off = (uint64_t*)out->values;
    if (!rc) {
        if (n > 0) str_code_len_kernel<<<g, kStrThreads, 0, s>>>(dc, n, lens, (uint64_t*)out->validity);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = scan_exclusive<uint64_t>(lens, n, out_off, part, s);
        if (e == hipSuccess) e = hipMemcpyAsync(&total, out_off + n, 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "codes to strings");
    }
    if (!rc) rc = owned_attach_data(out, (int64_t)total, s);
    if (!rc && total > 0) {
        str_code_bytes_kernel<<<g, kStrThreads, 0, s>>>(dc, n, out_off, (uint8_t*)out->data);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "codes to strings");
    }
    dev_free(lens, s);
    dev_free(part, s);
    if (rc) plgpu_column_release(out);
    return rc;
}

// ------------------------------------------------- string comparisons
// polars-compute/src/comparisons/view.rs (TotalEqKernel / TotalOrdKernel for
// BinaryViewArray, and their _broadcast forms against a scalar): strings
// compare by their bytes, lexicographically, a proper prefix first; a null
// operand gives a null result, except eq_missing / ne_missing (null equals
// only null, never null out).  `b` is a second string column, or (b.values
// == nullptr) the literal `lit` of `lit_len` bytes.  IS_NULL / IS_NOT_NULL
// read `a` only.
__device__ __forceinline__ int str_cmp3(const uint8_t* x, int64_t lx, const uint8_t* y, int64_t ly) {
    const int64_t m = lx < ly ? lx : ly;
    for (int64_t i = 0; i < m; ++i)
        if (x[i] != y[i]) return x[i] < y[i] ? -1 : 1;
    return lx < ly ? -1 : (lx > ly ? 1 : 0);
}

__global__ __launch_bounds__(kStrThreads) void str_cmp_kernel(DevCol a, DevCol b, const uint8_t* __restrict__ lit,
                                                              int64_t lit_len, int32_t op, int64_t n,
                                                              uint64_t* __restrict__ out_vals,
                                                              uint64_t* __restrict__ out_valid) {
    const int64_t* oa = (const int64_t*)a.values;
    const int64_t* ob = (const int64_t*)b.values;
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < n; i0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i0 + threadIdx.x;
        bool res = false, valid = false;
        if (r < n) {
            const bool va = dev_valid(a, r);
            if (op == PLGPU_OP_IS_NULL || op == PLGPU_OP_IS_NOT_NULL) {
                res = (op == PLGPU_OP_IS_NULL) ? !va : va;
                valid = true;
            } else if (op >= PLGPU_OP_STR_STARTS_WITH) {
                // literal pattern tests; a null string gives null
                valid = va;
                if (va) {
                    const int64_t sa = oa[a.offset + r], la = oa[a.offset + r + 1] - sa;
                    const uint8_t* x = a.data + sa;
                    if (op == PLGPU_OP_STR_STARTS_WITH || op == PLGPU_OP_STR_ENDS_WITH) {
                        const int64_t base = op == PLGPU_OP_STR_STARTS_WITH ? 0 : la - lit_len;
                        res = lit_len <= la;
                        for (int64_t j = 0; res && j < lit_len; ++j) res = x[base + j] == lit[j];
                    } else {  // contains (literal): naive scan, first-byte filter
                        res = lit_len == 0;
                        for (int64_t p0 = 0; !res && p0 + lit_len <= la; ++p0) {
                            if (x[p0] != lit[0]) continue;
                            bool m = true;
                            for (int64_t j = 1; m && j < lit_len; ++j) m = x[p0 + j] == lit[j];
                            res = m;
                        }
                    }
                }
            } else {
                const bool vb = ob == nullptr || dev_valid(b, r);
                int c = 0;
                if (va && vb) {
                    const int64_t sa = oa[a.offset + r], la = oa[a.offset + r + 1] - sa;
                    const uint8_t* y = lit;
                    int64_t ly = lit_len;
                    if (ob) {
                        const int64_t sb = ob[b.offset + r];
                        ly = ob[b.offset + r + 1] - sb;
                        y = b.data + sb;
                    }
                    c = str_cmp3(a.data + sa, la, y, ly);
                }
                switch (op) {
                case PLGPU_OP_EQ: res = c == 0; break;
                case PLGPU_OP_NE: res = c != 0; break;
                case PLGPU_OP_LT: res = c < 0; break;
                case PLGPU_OP_LE: res = c <= 0; break;
                case PLGPU_OP_GT: res = c > 0; break;
                case PLGPU_OP_GE: res = c >= 0; break;
                case PLGPU_OP_EQ_MISSING: res = (va && vb) ? c == 0 : va == vb; break;
                default: res = (va && vb) ? c != 0 : va != vb; break;  // NE_MISSING
                }
                valid = (op == PLGPU_OP_EQ_MISSING || op == PLGPU_OP_NE_MISSING) ? true : (va && vb);
                if (!valid) res = false;
            }
        }
        const uint64_t wv = __ballot(res), wm = __ballot(valid);
        if ((threadIdx.x & 63) == 0 && r < n) {
            out_vals[r >> 6] = wv;
            out_valid[r >> 6] = wm;
        }
    }
}

}  // namespace plgpu

using namespace plgpu;

PLGPU_API int plgpu_str_compare(const plgpu_column* a, const plgpu_column* b, const uint8_t* lit, int64_t lit_len,
                                int32_t op, plgpu_column* out, void* stream) {
    hipStream_t s = as_stream(stream);
    if (a == nullptr || out == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    std::memset(out, 0, sizeof *out);
    if (a->dtype != PLGPU_STR || (b && b->dtype != PLGPU_STR))
        return fail(PLGPU_ERR_SCHEMA, "string comparison of a non-String column");
    const bool unary = op == PLGPU_OP_IS_NULL || op == PLGPU_OP_IS_NOT_NULL;
    const bool pattern = op >= PLGPU_OP_STR_STARTS_WITH && op <= PLGPU_OP_STR_CONTAINS;
    if (!unary && !pattern && (op < PLGPU_OP_EQ || op > PLGPU_OP_NE_MISSING))
        return fail(PLGPU_ERR_INVALID, "unsupported string comparison");
    if (pattern && b != nullptr) return fail(PLGPU_ERR_INVALID, "string pattern tests take a literal");
    if (!unary && b == nullptr && lit_len > 0 && lit == nullptr) return fail(PLGPU_ERR_INVALID, "NULL literal");
    if (b && b->length != a->length) return fail(PLGPU_ERR_SHAPE, "compared columns differ in length");
    const int64_t n = a->length;
    int rc = make_owned_column(out, PLGPU_BOOL, n, true, s);
    if (rc || n == 0) return rc;
    uint8_t* dlit = nullptr;
    if (!unary && b == nullptr) {
        rc = dev_alloc((void**)&dlit, std::max<int64_t>(lit_len, 1), s);
        if (!rc && lit_len > 0 && hipMemcpyAsync(dlit, lit, lit_len, hipMemcpyHostToDevice, s) != hipSuccess)
            rc = fail(PLGPU_ERR_HIP, "string literal upload");
    }
    if (!rc) {
        DevCol db;
        std::memset(&db, 0, sizeof db);
        if (b) db = dev_col(*b);
        const int g = (int)std::min<int64_t>((n + kStrThreads - 1) / kStrThreads, (int64_t)num_cus_str() * 16);
        str_cmp_kernel<<<g, kStrThreads, 0, s>>>(dev_col(*a), db, dlit, lit_len, op, n, (uint64_t*)out->values,
                                                 (uint64_t*)out->validity);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "string comparison");
    }
    dev_free(dlit, s);
    if (rc) plgpu_column_release(out);
    return rc;
}

PLGPU_API int plgpu_str_encode_short(const plgpu_column* strs, plgpu_column* out_codes, int32_t* all_short,
                                     void* stream) {
    hipStream_t s = as_stream(stream);
    if (strs == nullptr || out_codes == nullptr || all_short == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    std::memset(out_codes, 0, sizeof *out_codes);
    if (strs->dtype != PLGPU_STR) return fail(PLGPU_ERR_SCHEMA, "short-string codes of a non-String column");
    const int64_t n = strs->length;
    int rc = make_owned_column(out_codes, PLGPU_I64, n, strs->validity != nullptr, s);
    if (rc) return rc;
    unsigned long long* flag = nullptr;
    unsigned long long hf = 0;
    rc = dev_alloc((void**)&flag, 8, s);
    if (!rc) {
        int64_t data_end = 0;
        hipError_t e = hipMemsetAsync(flag, 0, 8, s);
        if (e == hipSuccess && n > 0)
            e = hipMemcpyAsync(&data_end, (const int64_t*)strs->values + strs->offset + n, 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e == hipSuccess && n > 0) {
            const int g = (int)std::min<int64_t>((n + kStrThreads - 1) / kStrThreads, (int64_t)num_cus_str() * 16);
            str_code_kernel<<<g, kStrThreads, 0, s>>>(dev_col(*strs), n, (uint64_t*)out_codes->values, flag,
                                                      ((uintptr_t)strs->data & 7) == 0, data_end,
                                                      (uint64_t*)out_codes->validity);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(&hf, flag, 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "short-string codes");
    }
    dev_free(flag, s);
    if (rc) {
        plgpu_column_release(out_codes);
        return rc;
    }
    *all_short = hf == 0 ? 1 : 0;
    return PLGPU_OK;
}

PLGPU_API int plgpu_str_decode_short(const plgpu_column* codes, plgpu_column* out, void* stream) {
    if (codes == nullptr || out == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    std::memset(out, 0, sizeof *out);
    if (codes->dtype != PLGPU_I64) return fail(PLGPU_ERR_SCHEMA, "short-string codes must be Int64");
    return str_from_codes(*codes, out, as_stream(stream));
}
