// ingest.hip — Arrow RecordBatches in host memory -> device columns.
//
// The reference hands a DataFrame to an engine as one Arrow RecordBatch per
// chunk (crates/polars-python/src/dataframe/export.rs:80 PyDataFrame.to_arrow,
// called by the GPU engine's scan).  Each chunk's buffers are copied as they
// lie in host memory: value bytes go straight into their rows of the
// destination column, bitmaps (validity, Boolean values) at any bit offset
// are placed by a device kernel, String offsets are rebased on the device.
//
// Copies are the HIP runtime's own staged copy of the pageable Arrow
// buffer.  Measured with tools/bench_ingest.py on one MI355X box (1e8-row
// OHLCV table, profiles/r02_ingest.jsonl): 49.0 GB/s at 1M-row chunks,
// 55.7 GB/s at 8M-row chunks, the host link's rate (56.6 GB/s for whole
// columns).  Two alternatives were measured and removed: pinning the source
// pages in place (51.2 / 56.6 GB/s, no gain) and a double-buffered pinned
// staging pair filled by host threads (31.6 / 50.7 GB/s: the host memcpy
// into the pinned buffer is the bottleneck).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "plgpu_internal.hpp"

namespace plgpu {

// Host -> device copy, asynchronous on `s`; the runtime stages a pageable
// source before returning, so the source may be reused afterwards.
int h2d_staged(void* dst, const void* src, size_t n, hipStream_t s) {
    if (n == 0) return PLGPU_OK;
    PLGPU_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s));
    return PLGPU_OK;
}

namespace {

// Place n bits of `src` (bit src_bit of byte 0 onward; src padded by >= 8
// bytes) at bit dst_bit of the word array dst (or set them to 1 when src is
// null).  One thread per destination word; the first and last words are
// merged with their other bits, which belong to neighbouring chunks.
__global__ __launch_bounds__(256) void place_bits_kernel(uint64_t* __restrict__ dst, int64_t dst_bit,
                                                         const uint8_t* __restrict__ src, int src_bit, int64_t n) {
    const int64_t w0 = dst_bit >> 6;
    const int64_t w1 = (dst_bit + n - 1) >> 6;
    for (int64_t w = w0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w <= w1;
         w += (int64_t)gridDim.x * blockDim.x) {
        const int64_t lo = std::max(w << 6, dst_bit);                // first dst bit in this word
        const int64_t hi = std::min((w << 6) + 64, dst_bit + n);     // one past the last
        const int nb = (int)(hi - lo);
        const int sh = (int)(lo & 63);
        const uint64_t mask = (nb == 64 ? ~0ull : ((1ull << nb) - 1)) << sh;
        uint64_t bits;
        if (src == nullptr) {
            bits = ~0ull;
        } else {
            const int64_t q = lo - dst_bit + src_bit;  // source bit of `lo`
            const uint8_t* p = src + (q >> 3);
            uint64_t v = 0;
#pragma unroll
            for (int b = 0; b < 8; ++b) v |= (uint64_t)p[b] << (8 * b);
            const int r = (int)(q & 7);
            if (r) v = (v >> r) | ((uint64_t)p[8] << (64 - r));
            bits = v << sh;
        }
        dst[w] = (dst[w] & ~mask) | (bits & mask);
    }
}

int place_bits(uint8_t* dst, int64_t dst_bit, const uint8_t* host_bits, int64_t src_bit, int64_t n, hipStream_t s) {
    if (n <= 0) return PLGPU_OK;
    uint8_t* tmp = nullptr;
    int src_rem = 0;
    if (host_bits) {
        const int64_t b0 = src_bit >> 3;
        const int64_t nbytes = ((src_bit + n + 7) >> 3) - b0;
        int rc = dev_alloc((void**)&tmp, (size_t)nbytes + 16, s);
        if (rc) return rc;
        rc = h2d_staged(tmp, host_bits + b0, (size_t)nbytes, s);
        if (rc) { dev_free(tmp, s); return rc; }
        src_rem = (int)(src_bit & 7);
    }
    const int64_t words = ((dst_bit + n - 1) >> 6) - (dst_bit >> 6) + 1;
    const int g = (int)std::min<int64_t>((words + 255) / 256, 4096);
    place_bits_kernel<<<g, 256, 0, s>>>((uint64_t*)dst, dst_bit, tmp, src_rem, n);
    const hipError_t e = hipGetLastError();
    dev_free(tmp, s);  // stream-ordered: the block is reused only by later work
    if (e != hipSuccess) return hip_fail(e, "place_bits_kernel");
    return PLGPU_OK;
}

// offsets[i] += delta for i in [0, n)
__global__ __launch_bounds__(256) void rebase_offsets_kernel(int64_t* __restrict__ o, int64_t n, int64_t delta) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        o[i] += delta;
}

bool fixed_width(int32_t dt) { return dtype_bytes(dt) > 0; }

}  // namespace
}  // namespace plgpu

using namespace plgpu;

PLGPU_API int plgpu_column_alloc(int32_t dtype, int64_t length, int32_t with_validity, int64_t str_bytes,
                                 plgpu_column* out, void* stream) {
    if (out == nullptr || length < 0) return fail(PLGPU_ERR_INVALID, "column_alloc: bad arguments");
    hipStream_t s = as_stream(stream);
    if (dtype == PLGPU_STR) {
        const int rc = make_owned_string_column(out, length, std::max<int64_t>(str_bytes, 0), with_validity != 0, s);
        if (rc == PLGPU_OK && length == 0) {
            const int64_t zero = 0;
            PLGPU_HIP(hipMemcpyAsync((void*)out->values, &zero, 8, hipMemcpyHostToDevice, s));
            PLGPU_HIP(hipStreamSynchronize(s));
        }
        return rc;
    }
    if (dtype != PLGPU_BOOL && !fixed_width(dtype)) return fail(PLGPU_ERR_SCHEMA, "column_alloc: unsupported dtype");
    return make_owned_column(out, dtype, length, with_validity != 0, s);
}

PLGPU_API int plgpu_ingest_chunk(plgpu_column* dst, int64_t dst_row, int64_t dst_byte, const void* values,
                                 const uint8_t* validity, const uint8_t* str_data, int64_t src_offset,
                                 int64_t length, void* stream) {
    if (dst == nullptr || length < 0 || dst_row < 0 || src_offset < 0 || dst_row + length > dst->length)
        return fail(PLGPU_ERR_SHAPE, "ingest_chunk: rows out of range");
    if (length == 0) return PLGPU_OK;
    hipStream_t s = as_stream(stream);
    const int64_t base = dst->offset + dst_row;
    int rc = PLGPU_OK;
    if (dst->dtype == PLGPU_BOOL) {
        rc = place_bits((uint8_t*)dst->values, base, (const uint8_t*)values, src_offset, length, s);
    } else if (dst->dtype == PLGPU_STR) {
        const int64_t* offs = (const int64_t*)values + src_offset;
        const int64_t b0 = offs[0], b1 = offs[length];
        if (b1 < b0) return fail(PLGPU_ERR_INVALID, "ingest_chunk: string offsets decrease");
        int64_t* dofs = (int64_t*)dst->values + base;
        rc = h2d_staged(dofs, offs, (size_t)(length + 1) * 8, s);
        if (!rc && dst_byte != b0) {
            const int g = (int)std::min<int64_t>((length + 1 + 255) / 256, 2048);
            rebase_offsets_kernel<<<g, 256, 0, s>>>(dofs, length + 1, dst_byte - b0);
            PLGPU_HIP(hipGetLastError());
        }
        if (!rc && b1 > b0) rc = h2d_staged((uint8_t*)dst->data + dst_byte, str_data + b0, (size_t)(b1 - b0), s);
    } else {
        const int eb = dtype_bytes(dst->dtype);
        if (eb == 0) return fail(PLGPU_ERR_SCHEMA, "ingest_chunk: unsupported dtype");
        rc = h2d_staged((char*)dst->values + base * eb, (const char*)values + src_offset * eb, (size_t)length * eb, s);
    }
    if (rc) return rc;
    if (dst->validity) rc = place_bits((uint8_t*)dst->validity, base, validity, src_offset, length, s);
    else if (validity) return fail(PLGPU_ERR_INVALID, "ingest_chunk: chunk has nulls but the column has no validity");
    return rc;
}
