// Hash inner join on one integer key, and multi-column gather (the join's
// materialisation step).
//
// Reference (paths under /root/reference/crates):
//   polars-ops/src/frame/join/hash_join/single_keys_inner.rs:45
//     hash_join_tuples_inner: build hash tables on the shorter relation,
//     probe with the other, emit (left_idx, right_idx) IdxSize pairs;
//   polars-ops/src/frame/join/args.rs:25 JoinArgs (nulls_equal,
//     maintain_order, validate);
//   polars-core/src/chunked_array/ops/gather.rs (take by index) for the
//     materialisation.
//
// MI355X design:
//   build  - open-addressing table of 16-byte entries {key, ref, cnt} in HBM
//            (2^k slots, load <= 0.6, sized to stay resident in the 256 MiB
//            Infinity Cache for 1e7 build rows); one 16-byte load per probe
//            step returns key, count and (unique keys) the build row itself;
//            duplicate keys keep a CSR row list (ref = offset);
//   probe  - count pass (per 4096-row tile) -> scan -> write pass with
//            block-level scans, so pairs come out in probe-row order; rows
//            of one key follow build-row order (segments sorted when needed);
//   gather - one kernel per output column, validity bits re-packed with a
//            wave-wide OR.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "plgpu_internal.hpp"
#include "scan.hpp"
#include "tuplehash.hpp"

namespace plgpu {

constexpr int kJnThreads = 256;
constexpr int kJnTileRows = 4096;          // probe tile (16 rows per thread)
constexpr int kJnProbeLimit = 1 << 16;      // linear-probe bound before "table full"
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

// Table: cap + 2 cells of 16 B {key (EMPTY = INT64_MIN), ref}, 8 cells per
// 128-B bucket (one L2 line).  A key's home bucket is hash_slot(key, bbits)
// and it takes the first free cell from the start of that bucket on
// (linear probing over cells, so a full bucket overflows into the next).
// The ref word:
//   ref < 2^31          the single build row of a unique key;
//   ref == kRefList     duplicate key: rows[off[s] .. off[s + 1]);
//   ref == kRefNone     no build row (special slots only).
// Cells cap / cap + 1 are the null key / INT64_MIN key.  For 1e7 build
// rows the cells take 268 MB.
//
// The probe is bound by random line requests, not bytes: on MI355X about
// 55 G random requests/s whether a request reads 8, 64 or 128 B, from a
// table of 128 MB - 2 GB (tools/randread_bench.hip, profiles/
// r02_randread.txt).  Eight lanes read a probe's home bucket together (one
// 16-B load each, one line request), so a probe costs ~1.1 requests; the
// round-1 layout (8-B keys, then a separate ref array) cost ~1.8.
constexpr uint32_t kRefList = 0x80000000u;
constexpr uint32_t kRefNone = 0xFFFFFFFFu;
constexpr int kBktCells = 8;  // cells per 128-B bucket

struct JnTable {
    uint4* cells;      // cap + 2 cells {key lo, key hi, ref, -}: cap / 8 buckets of 8, then the 2 special slots
    uint32_t* off;     // cap + 3 CSR offsets (duplicate keys only)
    uint32_t* rows;    // CSR row lists
    int bits;          // cap = 2^bits cells
    int bbits;         // 2^bbits buckets
    int64_t cap;
};

// Cell s of the table: its key (8 B) and ref word (4 B); one 16-B load
// returns both.
__device__ __forceinline__ uint64_t& jn_key(const JnTable& t, int64_t s) { return ((uint64_t*)t.cells)[2 * s]; }
__device__ __forceinline__ uint32_t& jn_ref(const JnTable& t, int64_t s) { return ((uint32_t*)t.cells)[4 * s + 2]; }

// ---------------------------------------------------------------- build
__global__ void jn_init_kernel(JnTable t, uint32_t* cnt) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.cap + 2;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (i < t.cap) jn_key(t, i) = kEmptyKey;
        cnt[i] = 0;
    }
}

__global__ void jn_empty_kernel(JnTable t) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.cap; i += (int64_t)gridDim.x * blockDim.x)
        jn_key(t, i) = kEmptyKey;
}

// Insert the build keys; bslot[i] = slot of row i (kNoSlot: a null key that
// never matches).  status[0] counts rows that found no free slot.
__global__ void jn_build_kernel(DevCol bk, int64_t nb, JnTable t, bool nulls_equal, uint32_t* __restrict__ cnt,
                                uint32_t* __restrict__ bslot, unsigned long long* status) {
    const uint64_t mask = (uint64_t)t.cap - 1;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t slot;
        if (!dev_valid(bk, i)) {
            slot = nulls_equal ? t.cap : -1;
        } else {
            const uint64_t key = dev_load(bk, i);
            if (key == kEmptyKey) {
                slot = t.cap + 1;
            } else {
                slot = -2;
                uint64_t s = (uint64_t)hash_slot(key, t.bbits) * kBktCells;
                for (int p = 0; p < kJnProbeLimit; ++p, s = (s + 1) & mask) {
                    uint64_t k = __hip_atomic_load(&jn_key(t, s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (k == kEmptyKey) {
                        k = atomicCAS((unsigned long long*)&jn_key(t, s), (unsigned long long)kEmptyKey,
                                      (unsigned long long)key);
                        if (k == kEmptyKey) k = key;
                    }
                    if (k == key) {
                        slot = (int64_t)s;
                        break;
                    }
                }
                if (slot == -2) {
                    atomicAdd(&status[0], 1ull);
                    slot = -1;
                }
            }
        }
        if (slot >= 0) {
            atomicAdd(&cnt[slot], 1u);
            bslot[i] = (uint32_t)slot;
        } else {
            bslot[i] = kNoSlot;
        }
    }
}

// CSR offsets (u32) and max count (status[1]); ref gets kRefNone / kRefList
// (unique keys are filled in after the scatter).
__global__ void jn_offsets_kernel(JnTable t, const uint32_t* __restrict__ cnt, const uint64_t* __restrict__ off64,
                                  unsigned long long* status) {
    uint32_t mx = 0;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < t.cap + 3;
         s += (int64_t)gridDim.x * blockDim.x) {
        t.off[s] = (uint32_t)off64[s];
        if (s < t.cap + 2) {
            const uint32_t c = cnt[s];
            jn_ref(t, s) = c == 0 ? kRefNone : kRefList;
            mx = c > mx ? c : mx;
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t y = __shfl_xor(mx, o, 64);
        mx = y > mx ? y : mx;
    }
    if ((threadIdx.x & 63) == 0 && mx) atomicMax(&status[1], (unsigned long long)mx);
}

__global__ void jn_scatter_kernel(int64_t nb, JnTable t, const uint32_t* __restrict__ bslot,
                                  uint32_t* __restrict__ cursor) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t s = bslot[i];
        if (s == kNoSlot) continue;
        const uint32_t k = atomicAdd(&cursor[s], 1u);
        t.rows[t.off[s] + k] = (uint32_t)i;
    }
}

__global__ void jn_unique_ref_kernel(JnTable t) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < t.cap + 2;
         s += (int64_t)gridDim.x * blockDim.x) {
        if (t.off[s + 1] - t.off[s] == 1) jn_ref(t, s) = t.rows[t.off[s]];
    }
}

// Sort the row list of every duplicate key (build-row order, as the
// reference's IdxVec is filled in row order).  Short lists: one thread,
// insertion sort; long lists: one workgroup, odd-even transposition.
constexpr uint32_t kShortList = 64;
__global__ void jn_sort_short_kernel(JnTable t, uint32_t* __restrict__ long_slots,
                                     unsigned long long* __restrict__ nlong) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < t.cap + 2;
         s += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t c = t.off[s + 1] - t.off[s];
        if (c <= 1) continue;
        if (c > kShortList) {
            const unsigned long long k = atomicAdd(nlong, 1ull);
            long_slots[k] = (uint32_t)s;
            continue;
        }
        uint32_t* r = t.rows + t.off[s];
        for (uint32_t i = 1; i < c; ++i) {
            const uint32_t x = r[i];
            uint32_t j = i;
            while (j > 0 && r[j - 1] > x) {
                r[j] = r[j - 1];
                --j;
            }
            r[j] = x;
        }
    }
}

__global__ __launch_bounds__(256) void jn_sort_long_kernel(JnTable t, const uint32_t* __restrict__ long_slots) {
    const uint32_t s = long_slots[blockIdx.x];
    const uint32_t c = t.off[s + 1] - t.off[s];
    uint32_t* r = t.rows + t.off[s];
    for (uint32_t phase = 0; phase < c; ++phase) {
        for (uint32_t i = 2 * threadIdx.x + (phase & 1); i + 1 < c; i += 2 * blockDim.x) {
            const uint32_t a = r[i], b = r[i + 1];
            if (a > b) {
                r[i] = b;
                r[i + 1] = a;
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- probe
// Probe modes (one per join type; DESIGN.md §Join types):
//   JM_INNER  matching pairs only (hash_join_tuples_inner);
//   JM_OUTER  matching pairs, and (row, null) for a row without a match
//             (hash_join_tuples_left, probe_outer's no-match arm);
//   JM_SEMI   the rows with a match, once each (hash_join_tuples_left_semi);
//   JM_ANTI   the rows without a match (hash_join_tuples_left_anti);
//   JM_DRAIN  the build side's own rows whose slot was never marked by a
//             probe (probe_outer's drain of untracked build rows).
// MARK: a matched probe row sets flags[slot] (full joins and right-ordered
// left joins drain the unmarked build rows afterwards).
constexpr int JM_INNER = 0, JM_OUTER = 1, JM_SEMI = 2, JM_ANTI = 3, JM_DRAIN = 4;
constexpr uint32_t kNullIdx = 0xFFFFFFFFu;  // null index in an output pair

// Pass A: one lookup per probe row -> match word m[r] (the build row, or
// kRefList | slot for a duplicate key, or kRefNone) and per-tile output
// counts.  The probe keys are streamed with non-temporal loads so they do
// not evict the table from the Infinity Cache.
// Per round k a wave looks up its 64 rows in 8 sub-rounds: in sub-round j
// lane group g = lane / 8 reads the bucket of row (8j + g) of the wave, each
// lane one 16-B cell.  Rows' keys and buckets reach the groups through LDS,
// and the (ref, slot) of a matching cell goes back to the row's lane the
// same way; ballots tell the row's lane whether its bucket held the key or
// an empty cell (a full bucket without the key continues, lane by lane, in
// the next buckets - rare at load <= 0.6).
// INLINE (row-format table, unique build keys): a cell holds {key, payload}
// instead of {key, ref}; each wave writes one 64-bit hit mask into m's
// buffer and its hits' payloads, packed in hit order, at the start of its
// 64-word segment of mp (misses write nothing).
template <bool NULLABLE, int MODE, bool MARK, bool INLINE = false>
__global__ __launch_bounds__(kJnThreads) void jn_probe_match_kernel(DevCol pk, int64_t np, JnTable t,
                                                                  bool nulls_equal, uint32_t* __restrict__ m,
                                                                  uint64_t* __restrict__ tile_counts, int64_t ntiles,
                                                                  uint8_t* __restrict__ flags,
                                                                  uint64_t* __restrict__ mp = nullptr) {
    __shared__ uint64_t wsum[kJnThreads / 64];
    __shared__ uint4 rowbuf[kJnThreads];  // {key lo, key hi, bucket, regular}
    __shared__ uint4 hitbuf[kJnThreads];  // {ref (payload lo), slot, payload hi, -} of the matching cell
    const uint64_t* kp = (const uint64_t*)pk.values + pk.offset;
    const bool wide = pk.dtype == PLGPU_I64 || pk.dtype == PLGPU_U64;
    const int lane = threadIdx.x & 63;
    const int wbase = threadIdx.x & ~63;
    const int g = lane >> 3, e = lane & 7;
    const int bbits = t.bbits;
    const uint4* __restrict__ bkt = t.cells;
    const uint64_t nbm = (uint64_t(1) << bbits) - 1;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        constexpr int R = kJnTileRows / kJnThreads;
        uint64_t key[R];
        bool valid[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int64_t r = tile * kJnTileRows + (int64_t)k * kJnThreads + threadIdx.x;
            valid[k] = r < np;
            key[k] = 0;
            if (valid[k]) {
                key[k] = wide ? __builtin_nontemporal_load(kp + r) : dev_load(pk, r);
                if (NULLABLE) valid[k] = dev_valid(pk, r) ? true : false;
            }
        }
        uint64_t c = 0;
        for (int k = 0; k < R; ++k) {
            const int64_t r = tile * kJnTileRows + (int64_t)k * kJnThreads + threadIdx.x;
            const bool regular = r < np && (!NULLABLE || valid[k]) && key[k] != kEmptyKey;
            const uint32_t b = (uint32_t)hash_slot(key[k], bbits);
            rowbuf[threadIdx.x] = make_uint4((uint32_t)key[k], (uint32_t)(key[k] >> 32), b, regular ? 1u : 0u);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint4 rq[kBktCells];
            uint4 cell[kBktCells];
#pragma unroll
            for (int j = 0; j < kBktCells; ++j) {
                rq[j] = rowbuf[wbase + 8 * j + g];
                cell[j] = rq[j].w ? bkt[(uint64_t)rq[j].z * kBktCells + e] : make_uint4(0u, 0u, 0u, 0u);
            }
            uint64_t beq = 0, bem = 0;
#pragma unroll
            for (int j = 0; j < kBktCells; ++j) {
                const bool live = rq[j].w != 0;
                const bool eq = live && cell[j].x == rq[j].x && cell[j].y == rq[j].y;
                const bool em = live && cell[j].x == 0u && cell[j].y == 0x80000000u;
                const uint64_t eqm = __ballot(eq), emm = __ballot(em);
                if (eq) hitbuf[wbase + 8 * j + g] = make_uint4(cell[j].z, rq[j].z * kBktCells + e, cell[j].w, 0u);
                // this lane's row was served in sub-round lane / 8 by group lane % 8
                if ((lane >> 3) == j) {
                    beq = (eqm >> (8 * (lane & 7))) & 0xFFull;
                    bem = (emm >> (8 * (lane & 7))) & 0xFFull;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            int64_t slot = -1;
            uint32_t ref = kRefNone;
            uint64_t pay = 0;
            if (r >= np || (NULLABLE && !valid[k])) {
                if (r < np && NULLABLE && !valid[k] && nulls_equal) slot = t.cap;
            } else if (key[k] == kEmptyKey) {
                slot = t.cap + 1;
            } else if (beq) {
                const uint4 h = hitbuf[threadIdx.x];
                ref = h.x;
                slot = h.y;
                pay = (uint64_t)h.x | ((uint64_t)h.z << 32);
            } else if (!bem) {
                // the home bucket is full without the key: later buckets
                uint64_t bb = (b + 1) & nbm;
                for (uint64_t i = 0; i < nbm; ++i, bb = (bb + 1) & nbm) {
                    bool stop = false;
                    for (int ee = 0; ee < kBktCells; ++ee) {
                        const uint4 x = bkt[bb * kBktCells + ee];
                        const uint64_t kk = (uint64_t)x.x | ((uint64_t)x.y << 32);
                        if (kk == key[k]) {
                            ref = x.z;
                            pay = (uint64_t)x.z | ((uint64_t)x.w << 32);
                            slot = (int64_t)(bb * kBktCells + ee);
                            stop = true;
                            break;
                        }
                        if (kk == kEmptyKey) {
                            stop = true;
                            break;
                        }
                    }
                    if (stop) break;
                }
            }
            if (slot >= t.cap) {  // null / INT64_MIN key slots
                if (INLINE) {
                    // row-format special cells: key word 1 = occupied
                    const uint4 x = t.cells[slot];
                    ref = (x.x == 1u && x.y == 0u) ? 0u : kRefNone;
                    pay = (uint64_t)x.z | ((uint64_t)x.w << 32);
                } else {
                    ref = jn_ref(t, slot);
                }
            }
            if (INLINE && slot >= 0 && slot < t.cap) ref = 0u;  // a key match: the payload is in the cell
            if (MODE == JM_DRAIN) ref = (slot >= 0 && flags[slot]) ? 0u : kRefNone;
            if (r >= np) continue;
            const bool hit = ref != kRefNone;
            uint32_t w = kRefNone;
            if (MODE == JM_SEMI || MODE == JM_ANTI || MODE == JM_DRAIN) {
                w = hit ? 0u : kRefNone;
                c += (MODE == JM_SEMI) == hit ? 1 : 0;
            } else {
                if (INLINE) {
                    // one hit bit per row (ballot words in m's buffer; no
                    // match word) and the hits' payload words packed at the
                    // start of their wave's 64-word segment of mp (misses
                    // write nothing; the emit reads them back the same way)
                    const uint64_t hw = __ballot(hit);
                    const int ln = threadIdx.x & 63;
                    const uint64_t lt = ln == 0 ? 0ull : (~0ull >> (64 - ln));
                    if (hit) __builtin_nontemporal_store(pay, mp + (r & ~int64_t(63)) + __popcll(hw & lt));
                    if ((threadIdx.x & 63) == 0) reinterpret_cast<uint64_t*>(m)[r >> 6] = hw;
                    c += hit ? 1 : 0;
                    continue;
                } else if (ref == kRefList) {
                    w = kRefList | (uint32_t)slot;
                    c += t.off[slot + 1] - t.off[slot];
                } else if (hit) {
                    w = ref;
                    c += 1;
                } else if (MODE == JM_OUTER) {
                    c += 1;
                }
                if (MARK && hit) flags[slot] = 1;
            }
            __builtin_nontemporal_store(w, m + r);
        }
        uint64_t total;
        (void)block_excl_scan(c, wsum, total);
        if (threadIdx.x == 0) tile_counts[tile] = total;
    }
}

// Row-format build in one pass (no CSR): insert each build key with its
// payload; a key met twice sets status[1] (the caller falls back to the
// general build), a row that finds no free cell status[0].  The two special
// cells (null key, INT64_MIN key) count their rows in status[2] / [3] and
// carry key word 1 once occupied.
__global__ void jn_build_rowformat_kernel(DevCol bk, int64_t nb, JnTable t, bool nulls_equal, DevCol pay,
                                          unsigned long long* status) {
    const uint64_t mask = (uint64_t)t.cap - 1;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t slot = -1;
        if (!dev_valid(bk, i)) {
            if (!nulls_equal) continue;
            slot = t.cap;
        } else {
            const uint64_t key = dev_load(bk, i);
            if (key == kEmptyKey) {
                slot = t.cap + 1;
            } else {
                uint64_t s = (uint64_t)hash_slot(key, t.bbits) * kBktCells;
                bool placed = false;
                for (int p = 0; p < kJnProbeLimit; ++p, s = (s + 1) & mask) {
                    uint64_t k = __hip_atomic_load(&jn_key(t, s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (k == kEmptyKey) {
                        k = atomicCAS((unsigned long long*)&jn_key(t, s), (unsigned long long)kEmptyKey,
                                      (unsigned long long)key);
                        if (k == kEmptyKey) {
                            const uint64_t v = dev_load(pay, i);
                            uint32_t* c = (uint32_t*)&t.cells[s];
                            c[2] = (uint32_t)v;
                            c[3] = (uint32_t)(v >> 32);
                            placed = true;
                            break;
                        }
                    }
                    if (k == key) {
                        atomicOr(&status[1], 1ull);  // duplicate key
                        placed = true;
                        break;
                    }
                }
                if (!placed) atomicAdd(&status[0], 1ull);
                continue;
            }
        }
        // special cell: the first row claims it, a second is a duplicate
        if (atomicAdd(&status[2 + (slot - t.cap)], 1ull) == 0) {
            const uint64_t v = dev_load(pay, i);
            uint32_t* c = (uint32_t*)&t.cells[slot];
            c[0] = 1u;
            c[1] = 0u;
            c[2] = (uint32_t)v;
            c[3] = (uint32_t)(v >> 32);
        } else {
            atomicOr(&status[1], 1ull);
        }
    }
}

// ------------------------------------------------- wide row-format table
// The row-format table for W = 2..3 build payload columns (round 4): 32-B
// cells {key, p0, p1, p2}, four to a 128-B bucket, so one probe still reads
// one line and gets every payload of its build row with the key (a
// row-container hash table; the reference's _finish_join then takes each
// right column at the pairs, polars-ops/src/frame/join/general.rs:17).
// Special cells cap (null key) and cap + 1 (INT64_MIN key): key word 1 once
// occupied.
constexpr int kBktWide = 4;  // 32-B cells per 128-B bucket
struct WideCell {
    uint64_t key;
    uint64_t p[3];
};

__global__ void jn_empty_wide_kernel(WideCell* cells, int64_t cap) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x)
        cells[i].key = kEmptyKey;
}

struct WidePay {
    DevCol c[3];
};

template <int W>
__global__ void jn_build_wide_kernel(DevCol bk, int64_t nb, WideCell* cells, int64_t cap, int bbits, bool nulls_equal,
                                     WidePay pay, unsigned long long* status) {
    const uint64_t mask = (uint64_t)cap - 1;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t slot = -1;
        if (!dev_valid(bk, i)) {
            if (!nulls_equal) continue;
            slot = cap;
        } else {
            const uint64_t key = dev_load(bk, i);
            if (key == kEmptyKey) {
                slot = cap + 1;
            } else {
                uint64_t sl = (uint64_t)hash_slot(key, bbits) * kBktWide;
                bool placed = false;
                for (int q = 0; q < kJnProbeLimit; ++q, sl = (sl + 1) & mask) {
                    uint64_t k = __hip_atomic_load(&cells[sl].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (k == kEmptyKey) {
                        k = atomicCAS((unsigned long long*)&cells[sl].key, (unsigned long long)kEmptyKey,
                                      (unsigned long long)key);
                        if (k == kEmptyKey) {
#pragma unroll
                            for (int w = 0; w < W; ++w) cells[sl].p[w] = dev_load(pay.c[w], i);
                            placed = true;
                            break;
                        }
                    }
                    if (k == key) {
                        atomicOr(&status[1], 1ull);  // duplicate key
                        placed = true;
                        break;
                    }
                }
                if (!placed) atomicAdd(&status[0], 1ull);
                continue;
            }
        }
        if (atomicAdd(&status[2 + (slot - cap)], 1ull) == 0) {
            cells[slot].key = 1ull;
#pragma unroll
            for (int w = 0; w < W; ++w) cells[slot].p[w] = dev_load(pay.c[w], i);
        } else {
            atomicOr(&status[1], 1ull);
        }
    }
}

// Match pass over the wide table (inner join, no marks): per round k a wave
// looks up its 64 rows in 4 sub-rounds, lane group g = lane / 4 reading the
// bucket of row 16 j + g of the wave, each lane one 32-B cell (two 16-B
// loads).  The payloads of a matching cell go back to the row's lane through
// LDS.  Every row writes its W payload words (0 on a miss) to W dense arrays
// and each wave one 64-bit hit mask into `mwords`; a hit row's W payload
// words go to the wave's 64-word segment of W arrays, packed in hit order.
template <bool NULLABLE, int W>
__global__ __launch_bounds__(kJnThreads) void jn_probe_match_wide_kernel(DevCol pk, int64_t np, WideCell* cells,
                                                                       int64_t cap, int bbits, bool nulls_equal,
                                                                       uint64_t* __restrict__ mwords,
                                                                       uint64_t* __restrict__ tile_counts,
                                                                       int64_t ntiles, uint64_t* __restrict__ mp0,
                                                                       uint64_t* __restrict__ mp1,
                                                                       uint64_t* __restrict__ mp2) {
    __shared__ uint64_t wsum[kJnThreads / 64];
    __shared__ uint64_t rkey[kJnThreads];
    __shared__ uint32_t rbkt[kJnThreads];  // home bucket, or ~0: not a regular key
    __shared__ uint64_t hpay[W][kJnThreads];
    const uint64_t* kp = (const uint64_t*)pk.values + pk.offset;
    const bool wide = pk.dtype == PLGPU_I64 || pk.dtype == PLGPU_U64;
    const int lane = threadIdx.x & 63;
    const int wbase = threadIdx.x & ~63;
    const int g = lane >> 2, e = lane & 3;
    const uint64_t nbm = (uint64_t(1) << bbits) - 1;
    uint64_t* mp[3] = {mp0, mp1, mp2};
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        constexpr int R = kJnTileRows / kJnThreads;
        uint64_t key[R];
        bool valid[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int64_t r = tile * kJnTileRows + (int64_t)k * kJnThreads + threadIdx.x;
            valid[k] = r < np;
            key[k] = 0;
            if (valid[k]) {
                key[k] = wide ? __builtin_nontemporal_load(kp + r) : dev_load(pk, r);
                if (NULLABLE) valid[k] = dev_valid(pk, r) ? true : false;
            }
        }
        uint64_t c = 0;
        for (int k = 0; k < R; ++k) {
            const int64_t r = tile * kJnTileRows + (int64_t)k * kJnThreads + threadIdx.x;
            const bool regular = r < np && (!NULLABLE || valid[k]) && key[k] != kEmptyKey;
            const uint32_t b = (uint32_t)hash_slot(key[k], bbits);
            rkey[threadIdx.x] = key[k];
            rbkt[threadIdx.x] = regular ? b : ~0u;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint32_t qb[4];
            uint64_t qk[4];
            uint4 ca[4], cb[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                qb[j] = rbkt[wbase + 16 * j + g];
                qk[j] = rkey[wbase + 16 * j + g];
                const uint4* cp = reinterpret_cast<const uint4*>(cells + (uint64_t)qb[j] * kBktWide + e);
                ca[j] = qb[j] != ~0u ? cp[0] : make_uint4(0u, 0x80000000u, 0u, 0u);
                cb[j] = qb[j] != ~0u && W > 1 ? cp[1] : make_uint4(0u, 0u, 0u, 0u);
            }
            uint64_t beq = 0, bem = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint64_t ck = (uint64_t)ca[j].x | ((uint64_t)ca[j].y << 32);
                const bool live = qb[j] != ~0u;
                const bool eq = live && ck == qk[j];
                const bool em = live && ck == kEmptyKey;
                const uint64_t eqm = __ballot(eq), emm = __ballot(em);
                if (eq) {
                    const int row = wbase + 16 * j + g;
                    hpay[0][row] = (uint64_t)ca[j].z | ((uint64_t)ca[j].w << 32);
                    if (W > 1) hpay[1 % W][row] = (uint64_t)cb[j].x | ((uint64_t)cb[j].y << 32);
                    if (W > 2) hpay[2 % W][row] = (uint64_t)cb[j].z | ((uint64_t)cb[j].w << 32);
                }
                // this lane's row was served in sub-round lane / 16 by group lane % 16
                if ((lane >> 4) == j) {
                    beq = (eqm >> (4 * (lane & 15))) & 0xFull;
                    bem = (emm >> (4 * (lane & 15))) & 0xFull;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            bool hit = false;
            uint64_t pay[W];
#pragma unroll
            for (int w = 0; w < W; ++w) pay[w] = 0;
            if (r >= np || (NULLABLE && !valid[k])) {
                if (r < np && NULLABLE && !valid[k] && nulls_equal && cells[cap].key == 1ull) {
                    hit = true;
#pragma unroll
                    for (int w = 0; w < W; ++w) pay[w] = cells[cap].p[w];
                }
            } else if (key[k] == kEmptyKey) {
                if (cells[cap + 1].key == 1ull) {
                    hit = true;
#pragma unroll
                    for (int w = 0; w < W; ++w) pay[w] = cells[cap + 1].p[w];
                }
            } else if (beq) {
                hit = true;
#pragma unroll
                for (int w = 0; w < W; ++w) pay[w] = hpay[w][threadIdx.x];
            } else if (!bem) {
                // the home bucket is full without the key: later buckets
                uint64_t bb = (b + 1) & nbm;
                for (uint64_t i = 0; i < nbm && !hit; ++i, bb = (bb + 1) & nbm) {
                    bool stop = false;
                    for (int ee = 0; ee < kBktWide; ++ee) {
                        const WideCell& x = cells[bb * kBktWide + ee];
                        if (x.key == key[k]) {
                            hit = true;
#pragma unroll
                            for (int w = 0; w < W; ++w) pay[w] = x.p[w];
                            stop = true;
                            break;
                        }
                        if (x.key == kEmptyKey) {
                            stop = true;
                            break;
                        }
                    }
                    if (stop) break;
                }
            }
            if (r >= np) continue;
            const uint64_t hw = __ballot(hit);
            // the hits' payloads packed at the start of the wave's 64-word
            // segment of each array (as the single-payload match pass)
            const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
            if (hit) {
#pragma unroll
                for (int w = 0; w < W; ++w)
                    __builtin_nontemporal_store(pay[w], mp[w] + (r & ~int64_t(63)) + __popcll(hw & lt));
            }
            if ((threadIdx.x & 63) == 0) mwords[r >> 6] = hw;
            c += hit ? 1 : 0;
        }
        uint64_t total;
        (void)block_excl_scan(c, wsum, total);
        if (threadIdx.x == 0) tile_counts[tile] = total;
    }
}

// Emit of the row-format probe, fused with the take of the left columns:
// every hit row's payload and its null-free 8-byte left columns go straight
// to their output position (probe-row order); the row id too when other
// left columns are gathered afterwards.
struct TakeCols {
    const uint64_t* src[PLGPU_MAX_COLS];
    uint64_t* dst[PLGPU_MAX_COLS];
    int32_t n;
};

struct TakePay {
    const uint64_t* src[3];  // dense payload words of the match pass
    uint64_t* dst[3];        // the right output columns
};

template <int NC, int W = 1>
__global__ __launch_bounds__(kJnThreads) void jn_take_emit_kernel(int64_t np, const uint64_t* __restrict__ mwords,
                                                                  TakePay tp,
                                                                  const uint64_t* __restrict__ tile_off,
                                                                  int64_t ntiles, TakeCols lc,
                                                                  uint32_t* __restrict__ out_idx) {
    // A tile's 64 hit words (row chunk k, wave w -> word 4k + w, row order)
    // are scanned once; a row's output position is then the tile offset +
    // its word's prefix + the hits below it in the word.
    constexpr int R = kJnTileRows / kJnThreads;
    constexpr int NW = kJnThreads / 64;
    constexpr int U = NC <= 2 ? 8 : 4;  // row chunks whose loads are issued together
    __shared__ uint64_t words[kJnTileRows / 64];
    __shared__ uint32_t prefix[kJnTileRows / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        if (threadIdx.x < kJnTileRows / 64) {
            const int64_t wi = tile * (kJnTileRows / 64) + threadIdx.x;
            const uint64_t w = wi * 64 < np ? mwords[wi] : 0ull;
            uint32_t x = (uint32_t)__popcll(w), c = x;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(x, off, 64);
                if (lane >= off) x += y;
            }
            words[threadIdx.x] = w;
            prefix[threadIdx.x] = x - c;
        }
        __syncthreads();
        const uint64_t run = tile_off[tile];
        for (int k0 = 0; k0 < R; k0 += U) {
            uint64_t pv[U][W], v[U][NC > 0 ? NC : 1];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t r = tile * kJnTileRows + (int64_t)(k0 + u) * kJnThreads + threadIdx.x;
                const int64_t rr = r < np ? r : np - 1;
                // a hit's payloads sit packed at the start of its wave's
                // 64-word segment (the match pass's layout): only hits load
                const uint64_t w = words[(k0 + u) * NW + wave];
                const bool h = (w >> lane) & 1;
                const int64_t pq = (r & ~int64_t(63)) + __popcll(w & lt);
#pragma unroll
                for (int q = 0; q < W; ++q) pv[u][q] = h ? __builtin_nontemporal_load(tp.src[q] + pq) : 0ull;
#pragma unroll
                for (int j = 0; j < NC; ++j) v[u][j] = __builtin_nontemporal_load(lc.src[j] + rr);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int wi = (k0 + u) * NW + wave;
                const uint64_t w = words[wi];
                if ((w >> lane) & 1) {
                    const uint64_t pos = run + prefix[wi] + (uint32_t)__popcll(w & lt);
#pragma unroll
                    for (int q = 0; q < W; ++q) tp.dst[q][pos] = pv[u][q];
#pragma unroll
                    for (int j = 0; j < NC; ++j) lc.dst[j][pos] = v[u][j];
                    if (out_idx)
                        out_idx[pos] = (uint32_t)(tile * kJnTileRows + (int64_t)(k0 + u) * kJnThreads + threadIdx.x);
                }
            }
        }
        __syncthreads();
    }
}

// Pass B: pairs in probe-row order.  Row r = base + k*T + tid of a tile is
// ranked k*T + tid; one block scan per k.
// `rowmap` (partitioned probe, semi/anti selection): position r holds probe
// row rowmap[r].
// JM_OUTER writes kNullIdx as the build row of an unmatched probe row;
// JM_SEMI / JM_ANTI / JM_DRAIN write probe rows only (out_b unused).
template <int MODE>
__global__ __launch_bounds__(kJnThreads) void jn_probe_emit_kernel(int64_t np, JnTable t,
                                                                   const uint32_t* __restrict__ m,
                                                                   const uint64_t* __restrict__ tile_off,
                                                                   int64_t ntiles, uint32_t* __restrict__ out_p,
                                                                   uint32_t* __restrict__ out_b,
                                                                   const uint32_t* __restrict__ rowmap) {
    __shared__ uint64_t wsum[kJnThreads / 64];
    constexpr int R = kJnTileRows / kJnThreads;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        uint32_t w[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int64_t r = tile * kJnTileRows + (int64_t)k * kJnThreads + threadIdx.x;
            w[k] = r < np ? __builtin_nontemporal_load(m + r) : kRefNone;
        }
        uint64_t run = tile_off[tile];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int64_t r = tile * kJnTileRows + (int64_t)k * kJnThreads + threadIdx.x;
            uint32_t c = 0, lo = 0;
            if (MODE == JM_SEMI) {
                c = w[k] != kRefNone ? 1u : 0u;
            } else if (MODE == JM_ANTI || MODE == JM_DRAIN) {
                c = (r < np && w[k] == kRefNone) ? 1u : 0u;
            } else if (w[k] != kRefNone) {
                if (w[k] & kRefList) {
                    const uint32_t slot = w[k] & ~kRefList;
                    lo = t.off[slot];
                    c = t.off[slot + 1] - lo;
                } else {
                    c = 1;
                }
            } else if (MODE == JM_OUTER && r < np) {
                c = 1;
            }
            uint64_t total;
            const uint64_t pos = run + block_excl_scan(c, wsum, total);
            const uint32_t pr = c ? (rowmap ? rowmap[r] : (uint32_t)r) : 0u;
            if (MODE == JM_SEMI || MODE == JM_ANTI || MODE == JM_DRAIN) {
                if (c) out_p[pos] = pr;
            } else if (MODE == JM_OUTER && c == 1 && w[k] == kRefNone) {
                out_p[pos] = pr;
                out_b[pos] = kNullIdx;
            } else if (c == 1 && !(w[k] & kRefList)) {
                out_p[pos] = pr;
                out_b[pos] = w[k];
            } else {
                for (uint32_t j = 0; j < c; ++j) {
                    out_p[pos + j] = pr;
                    out_b[pos + j] = t.rows[lo + j];
                }
            }
            run += total;
        }
    }
}


static int num_cus_jn() {
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

// --------------------------------------------------------------- gather
// `iv` (optional): validity of the index column (Arrow bits from `ioff`); a
// null index gathers a null (IdxCa::with_nullable_idx + take in the
// reference's left / full join materialisation).
__device__ __forceinline__ bool idx_null(const uint8_t* iv, int64_t ioff, int64_t o) {
    return iv != nullptr && !((iv[(ioff + o) >> 3] >> ((ioff + o) & 7)) & 1);
}

template <int EB>  // element bytes 1 / 2 / 4 / 8
__global__ __launch_bounds__(256) void gather_col_kernel(DevCol c, const uint32_t* __restrict__ idx, int64_t n,
                                                         void* __restrict__ out, uint64_t* __restrict__ out_valid,
                                                         const uint8_t* __restrict__ iv, int64_t ioff) {
    // 8 outputs per thread (strided by the block), loads issued together and
    // branch-free (a null index reads row 0), so none waits on another
    constexpr int K = 8;
    const int64_t step = (int64_t)gridDim.x * blockDim.x * K;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x * K; base < n; base += step) {
        uint32_t r[K];
        bool in[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t o = base + (int64_t)k * blockDim.x + threadIdx.x;
            r[k] = __builtin_nontemporal_load(idx + (o < n ? o : n - 1));
            in[k] = o < n && !idx_null(iv, ioff, o);
            if (!in[k]) r[k] = 0;
        }
        uint64_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t p = c.offset + r[k];
            v[k] = EB == 8   ? ((const uint64_t*)c.values)[p]
                   : EB == 4 ? ((const uint32_t*)c.values)[p]
                   : EB == 2 ? ((const uint16_t*)c.values)[p]
                             : ((const uint8_t*)c.values)[p];
            if (!in[k]) v[k] = 0;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t o = base + (int64_t)k * blockDim.x + threadIdx.x;
            if (o < n) {
                if (EB == 8) __builtin_nontemporal_store(v[k], (uint64_t*)out + o);
                else if (EB == 4) __builtin_nontemporal_store((uint32_t)v[k], (uint32_t*)out + o);
                else if (EB == 2) ((uint16_t*)out)[o] = (uint16_t)v[k];
                else ((uint8_t*)out)[o] = (uint8_t)v[k];
            }
            if (out_valid) {
                // one validity word per wave and k (o of lane 0 is a multiple of 64)
                const uint64_t w = __ballot(in[k] && dev_valid(c, r[k]));
                if ((threadIdx.x & 63) == 0 && o < n) out_valid[o >> 6] = w;
            }
        }
    }
}

__global__ void gather_bool_kernel(DevCol c, const uint32_t* __restrict__ idx, int64_t n,
                                   uint64_t* __restrict__ out, uint64_t* __restrict__ out_valid,
                                   const uint8_t* __restrict__ iv, int64_t ioff) {
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = base + threadIdx.x;
        bool v = false, valid = false;
        if (o < n && !idx_null(iv, ioff, o)) {
            const int64_t r = idx[o];
            v = dev_load(c, r) & 1;
            valid = dev_valid(c, r);
        }
        const uint64_t wv = __ballot(v), wm = __ballot(valid);
        if ((threadIdx.x & 63) == 0 && o < n) {
            out[o >> 6] = wv;
            if (out_valid) out_valid[o >> 6] = wm;
        }
    }
}

// Many 8-byte columns gathered by one random index: the columns are first
// packed row-major (sequential read, sequential write), so each random row
// fetch brings every column's value in one or two cache lines instead of
// one line per column.
constexpr int kAosMax = 8;

struct AosCols {
    const uint64_t* src[kAosMax];
    uint64_t* dst[kAosMax];
};

template <int NC>
__global__ __launch_bounds__(256) void aos_pack_kernel(AosCols c, int64_t rows, uint64_t* __restrict__ aos) {
    // 256 rows per step: column loads coalesced, rows transposed through LDS
    // (row stride NP + 2 words against bank conflicts), then the block's
    // 256 * NP words stored as consecutive 16-byte chunks
    constexpr int NP = (NC + 1) & ~1;  // row stride in u64 (16-byte aligned rows)
    constexpr int STR = NP + 2;
    __shared__ __attribute__((aligned(16))) uint64_t tile[256 * STR];
    for (int64_t r0 = (int64_t)blockIdx.x * 256; r0 < rows; r0 += (int64_t)gridDim.x * 256) {
        const int64_t r = r0 + threadIdx.x;
        const int64_t rr = r < rows ? r : rows - 1;
        uint64_t v[NP];
#pragma unroll
        for (int k = 0; k < NC; ++k) v[k] = __builtin_nontemporal_load(c.src[k] + rr);
        if (NP != NC) v[NP - 1] = 0;
#pragma unroll
        for (int k = 0; k < NP / 2; ++k)
            *reinterpret_cast<ulonglong2*>(&tile[threadIdx.x * STR + 2 * k]) = make_ulonglong2(v[2 * k], v[2 * k + 1]);
        __syncthreads();
        const int nrows = rows - r0 < 256 ? (int)(rows - r0) : 256;
        const int nchunks = nrows * (NP / 2);
        ulonglong2* dst = reinterpret_cast<ulonglong2*>(aos + r0 * NP);
        for (int j = threadIdx.x; j < nchunks; j += 256) {
            const int row = j / (NP / 2), q = j - row * (NP / 2);
            dst[j] = *reinterpret_cast<const ulonglong2*>(&tile[row * STR + 2 * q]);
        }
        __syncthreads();
    }
}

// Gather of packed rows: a block gathers 256 destination rows per step (NP/2
// lanes per row, each loading 16 bytes = two columns of it, so one load
// instruction of a wave fetches whole contiguous rows; non-temporal, the
// random lines are not reused) into an LDS image held column-major, then
// stores each column's 256 values as 2 KiB of consecutive 16-byte chunks --
// the inverse of aos_pack_kernel.  Against 8-byte stores straight from the
// loading lanes (NC scattered 128-byte segments per store instruction):
// 58.7 -> 54.6 ms for pack + gather of 1e9 rows x 8 columns by a random
// index, 50.7 -> 43.3 ms by the identity (profiles/r03_gather_ab.log).
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

template <int NC>
__global__ __launch_bounds__(256) void aos_gather_kernel(const uint64_t* __restrict__ aos,
                                                           const uint32_t* __restrict__ idx, int64_t n, AosCols c) {
    constexpr int NP = (NC + 1) & ~1;
    constexpr int L = NP / 2;          // lanes per row
    constexpr int PER = L;             // 16-B row pieces per thread per 256-row step
    constexpr int R = 256;             // rows per block step
    constexpr int CS = R + 2;          // LDS column stride in u64
    __shared__ __attribute__((aligned(16))) uint64_t img[NP * CS];
    for (int64_t r0 = (int64_t)blockIdx.x * R; r0 < n; r0 += (int64_t)gridDim.x * R) {
        const int nrows = n - r0 < R ? (int)(n - r0) : R;
        uint32_t r[PER];
        int row[PER], q[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int t = k * 256 + threadIdx.x;
            row[k] = t / L;
            q[k] = t - row[k] * L;
            r[k] = __builtin_nontemporal_load(idx + r0 + (row[k] < nrows ? row[k] : nrows - 1));
        }
        u64x2 x[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const u64x2* src = reinterpret_cast<const u64x2*>(aos + (int64_t)r[k] * NP) + q[k];
            x[k] = __builtin_nontemporal_load(src);
        }
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            img[(2 * q[k]) * CS + row[k]] = x[k].x;
            img[(2 * q[k] + 1) * CS + row[k]] = x[k].y;
        }
        __syncthreads();
        if (nrows == R) {
            // NC columns x R / 2 chunks of two rows
            for (int j = threadIdx.x; j < NC * (R / 2); j += 256) {
                const int col = j / (R / 2), p = (j - col * (R / 2)) * 2;
                const u64x2 v = *reinterpret_cast<const u64x2*>(&img[col * CS + p]);
                __builtin_nontemporal_store(v, reinterpret_cast<u64x2*>(c.dst[col] + r0 + p));
            }
        } else {
            for (int j = threadIdx.x; j < NC * R; j += 256) {
                const int col = j / R, p = j - col * R;
                if (p < nrows) c.dst[col][r0 + p] = img[col * CS + p];
            }
        }
        __syncthreads();
    }
}

template <int NC>
static hipError_t aos_run(const AosCols& c, int64_t rows, const uint32_t* idx, int64_t n, uint64_t* aos,
                          hipStream_t s) {
    const int g = std::max(1, num_cus_jn() * 16);
    {
        KtScope kt("aos_pack_kernel", s);
        aos_pack_kernel<NC><<<g, 256, 0, s>>>(c, rows, aos);
    }
    {
        KtScope kt("aos_gather_kernel", s);
        aos_gather_kernel<NC><<<g, 256, 0, s>>>(aos, idx, n, c);
    }
    return hipGetLastError();
}

static hipError_t aos_dispatch(int nc, const AosCols& c, int64_t rows, const uint32_t* idx, int64_t n,
                               uint64_t* aos, hipStream_t s) {
    switch (nc) {
    case 2: return aos_run<2>(c, rows, idx, n, aos, s);
    case 3: return aos_run<3>(c, rows, idx, n, aos, s);
    case 4: return aos_run<4>(c, rows, idx, n, aos, s);
    case 5: return aos_run<5>(c, rows, idx, n, aos, s);
    case 6: return aos_run<6>(c, rows, idx, n, aos, s);
    case 7: return aos_run<7>(c, rows, idx, n, aos, s);
    default: return aos_run<8>(c, rows, idx, n, aos, s);
    }
}

static int gather_into(const plgpu_column& src, const uint32_t* idx, int64_t n, plgpu_column* out, hipStream_t s,
                       const uint8_t* iv = nullptr, int64_t ioff = 0) {
    const bool nullable = src.validity != nullptr || iv != nullptr;
    if (src.dtype == PLGPU_STR) return str_gather(dev_col(src), idx, nullptr, iv, ioff, n, nullable, out, s);
    int rc = make_owned_column(out, src.dtype, n, nullable, s);
    if (rc) return rc;
    if (n == 0) return PLGPU_OK;
    if (src.length == 0) {
        // every index is null (an empty side of an outer join): all-null
        // output, and the kernels' branch-free row-0 reads must not run
        PLGPU_HIP(hipMemsetAsync((void*)out->values, 0,
                                 src.dtype == PLGPU_BOOL ? ((n + 63) / 64) * 8 : n * dtype_bytes(src.dtype), s));
        if (out->validity) PLGPU_HIP(hipMemsetAsync((void*)out->validity, 0, ((n + 63) / 64) * 8, s));
        out->null_count = n;
        return PLGPU_OK;
    }
    DevCol c;
    std::memset(&c, 0, sizeof c);
    c.dtype = src.dtype;
    c.offset = src.offset;
    c.values = src.values;
    c.validity = src.validity;
    const int g = (int)std::min<int64_t>((n + 1023) / 1024, (int64_t)num_cus_jn() * 16);
    uint64_t* ov = (uint64_t*)out->validity;
    if (src.dtype == PLGPU_BOOL)
        gather_bool_kernel<<<g, 256, 0, s>>>(c, idx, n, (uint64_t*)out->values, ov, iv, ioff);
    else if (dtype_bytes(src.dtype) == 8)
        gather_col_kernel<8><<<g, 256, 0, s>>>(c, idx, n, (void*)out->values, ov, iv, ioff);
    else if (dtype_bytes(src.dtype) == 4)
        gather_col_kernel<4><<<g, 256, 0, s>>>(c, idx, n, (void*)out->values, ov, iv, ioff);
    else if (dtype_bytes(src.dtype) == 2)
        gather_col_kernel<2><<<g, 256, 0, s>>>(c, idx, n, (void*)out->values, ov, iv, ioff);
    else
        gather_col_kernel<1><<<g, 256, 0, s>>>(c, idx, n, (void*)out->values, ov, iv, ioff);
    PLGPU_HIP(hipGetLastError());
    out->null_count = nullable ? -1 : 0;
    return PLGPU_OK;
}

static int log2_ceil64(int64_t x) {
    int b = 0;
    while ((int64_t(1) << b) < x) ++b;
    return b;
}

}  // namespace plgpu

using namespace plgpu;

// Built hash table of one join side (kept for the probe).
struct JnBuilt {
    JnTable t;
    uint64_t max_count = 0;
    int64_t rows = 0;
    JnBuilt() { std::memset(&t, 0, sizeof t); }
};

static void jn_free(JnBuilt& b, hipStream_t s) {
    dev_free(b.t.cells, s);
    dev_free(b.t.off, s);
    dev_free(b.t.rows, s);
    std::memset(&b.t, 0, sizeof b.t);
}

static DevCol as_dev(const plgpu_column* c) { return dev_col(*c); }

// Build the table over `key` (rows [0, n)); sorted row lists if `ordered`.
static int jn_build(const plgpu_column* key, bool nulls_equal, bool ordered, JnBuilt* out, hipStream_t s) {
    const int64_t nb = key->length;
    const DevCol bk = as_dev(key);
    int bits = std::max(10, log2_ceil64((nb * 5 + 2) / 3));  // load <= 0.6
    uint32_t* cnt = nullptr;
    uint32_t* bslot = nullptr;
    uint64_t* off64 = nullptr;
    uint64_t* part = nullptr;
    unsigned long long* status = nullptr;
    int rc = dev_alloc((void**)&status, 16, s);
    if (!rc) rc = dev_alloc((void**)&bslot, std::max<int64_t>(nb, 1) * 4, s);
    JnBuilt b;
    for (int attempt = 0; !rc; ++attempt) {
        b.t.bits = bits;
        b.t.bbits = bits - 3;
        b.t.cap = int64_t(1) << bits;
        const int64_t ne = b.t.cap + 2;
        if ((rc = dev_alloc((void**)&b.t.cells, ne * 16, s))) break;
        if ((rc = dev_alloc((void**)&cnt, ne * 4, s))) break;
        PLGPU_HIP(hipMemsetAsync(status, 0, 16, s));
        const int gi = (int)std::min<int64_t>((ne + 255) / 256, 256 * 32);
        jn_init_kernel<<<gi, 256, 0, s>>>(b.t, cnt);
        if (nb > 0) {
            const int gb = (int)std::min<int64_t>((nb + 255) / 256, 256 * 32);
            jn_build_kernel<<<gb, 256, 0, s>>>(bk, nb, b.t, nulls_equal, cnt, bslot, status);
        }
        PLGPU_HIP(hipGetLastError());
        unsigned long long st[2];
        PLGPU_HIP(hipMemcpyAsync(st, status, 16, hipMemcpyDeviceToHost, s));
        PLGPU_HIP(hipStreamSynchronize(s));
        if (st[0] == 0) break;
        if (attempt >= 3) {
            rc = fail(PLGPU_ERR_CAPACITY, "join build table did not converge");
            break;
        }
        dev_free(b.t.cells, s);
        dev_free(cnt, s);
        b.t.cells = nullptr;
        cnt = nullptr;
        bits += 2;
    }
    const int64_t ne = b.t.cap + 2;
    if (!rc) rc = dev_alloc((void**)&b.t.off, (ne + 1) * 4, s);
    if (!rc) rc = dev_alloc((void**)&off64, (ne + 1) * 8, s);
    if (!rc) rc = dev_alloc((void**)&part, ((ne + kScanChunk - 1) / kScanChunk + 1) * 8, s);
    if (!rc) rc = dev_alloc((void**)&b.t.rows, std::max<int64_t>(nb, 1) * 4, s);
    if (!rc) {
        hipError_t e = scan_exclusive<uint32_t>(cnt, ne, off64, part, s);
        const int ge = (int)std::min<int64_t>((ne + 256) / 256, 256 * 32);
        if (e == hipSuccess) {
            jn_offsets_kernel<<<ge, 256, 0, s>>>(b.t, cnt, off64, status);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, ne * 4, s);  // reused as scatter cursors
        if (e == hipSuccess && nb > 0) {
            const int gb = (int)std::min<int64_t>((nb + 255) / 256, 256 * 32);
            jn_scatter_kernel<<<gb, 256, 0, s>>>(nb, b.t, bslot, cnt);
            e = hipGetLastError();
        }
        unsigned long long st[2] = {0, 0};
        if (e == hipSuccess) e = hipMemcpyAsync(st, status, 16, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "join build");
        b.max_count = st[1];
    }
    if (!rc && ordered && b.max_count > 1) {
        // deterministic build-row order inside each duplicate key
        uint32_t* long_slots = nullptr;
        unsigned long long* nlong = status;  // reuse word 0
        rc = dev_alloc((void**)&long_slots, ne * 4, s);
        if (!rc) {
            (void)hipMemsetAsync(nlong, 0, 8, s);
            const int ge = (int)std::min<int64_t>((ne + 255) / 256, 256 * 32);
            jn_sort_short_kernel<<<ge, 256, 0, s>>>(b.t, long_slots, nlong);
            unsigned long long nl = 0;
            hipError_t e = hipMemcpyAsync(&nl, nlong, 8, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e == hipSuccess && nl > 0) {
                jn_sort_long_kernel<<<(unsigned)nl, 256, 0, s>>>(b.t, long_slots);
                e = hipGetLastError();
            }
            if (e != hipSuccess) rc = hip_fail(e, "join list sort");
        }
        dev_free(long_slots, s);
    }
    if (!rc) {
        const int ge = (int)std::min<int64_t>((ne + 255) / 256, 256 * 32);
        jn_unique_ref_kernel<<<ge, 256, 0, s>>>(b.t);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) rc = hip_fail(e, "join build refs");
    }
    dev_free(cnt, s);
    dev_free(bslot, s);
    dev_free(off64, s);
    dev_free(part, s);
    dev_free(status, s);
    if (rc) {
        jn_free(b, s);
        return rc;
    }
    b.rows = nb;
    *out = b;
    return PLGPU_OK;
}

// Wide row-format table over a unique-keyed build side with W = 2..3
// payload columns (jn_build_wide_kernel); *unique = false (and nothing
// built) when a key repeats.  cells: (cap + 2) 32-B cells.
struct WideBuilt {
    WideCell* cells = nullptr;
    int64_t cap = 0;
    int bbits = 0;
};

static int jn_build_wide(const plgpu_column* key, const plgpu_column* pays, int W, bool nulls_equal, WideBuilt* out,
                         bool* unique, hipStream_t s) {
    const int64_t nb = key->length;
    int bits = std::max(10, log2_ceil64((nb * 5 + 2) / 3));  // load <= 0.6
    unsigned long long* status = nullptr;
    int rc = dev_alloc((void**)&status, 32, s);
    *unique = true;
    WidePay wp;
    std::memset(&wp, 0, sizeof wp);
    for (int w = 0; w < W; ++w) wp.c[w] = dev_col(pays[w]);
    WideBuilt b;
    for (int attempt = 0; !rc; ++attempt) {
        b.cap = int64_t(1) << bits;
        b.bbits = bits - 2;  // 4 cells per bucket
        const int64_t ne = b.cap + 2;
        if ((rc = dev_alloc((void**)&b.cells, ne * sizeof(WideCell), s))) break;
        hipError_t e = hipMemsetAsync(status, 0, 32, s);
        if (e == hipSuccess) e = hipMemsetAsync(b.cells, 0x00, ne * sizeof(WideCell), s);
        if (e == hipSuccess) {
            const int gi = (int)std::min<int64_t>((ne + 255) / 256, 256 * 32);
            jn_empty_wide_kernel<<<gi, 256, 0, s>>>(b.cells, b.cap);
            const int gb = (int)std::min<int64_t>((nb + 255) / 256, 256 * 32);
            if (nb > 0) {
                KtScope kt("jn_build_wide_kernel", s);
                if (W == 2)
                    jn_build_wide_kernel<2><<<gb, 256, 0, s>>>(dev_col(*key), nb, b.cells, b.cap, b.bbits, nulls_equal,
                                                               wp, status);
                else
                    jn_build_wide_kernel<3><<<gb, 256, 0, s>>>(dev_col(*key), nb, b.cells, b.cap, b.bbits, nulls_equal,
                                                               wp, status);
            }
            e = hipGetLastError();
        }
        unsigned long long st[4] = {0, 0, 0, 0};
        if (e == hipSuccess) e = hipMemcpyAsync(st, status, 32, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            rc = hip_fail(e, "join wide row-format build");
            break;
        }
        if (st[1]) {
            *unique = false;
            break;
        }
        if (st[0] == 0) break;
        if (attempt >= 3) {
            rc = fail(PLGPU_ERR_CAPACITY, "join build table did not converge");
            break;
        }
        dev_free(b.cells, s);
        b.cells = nullptr;
        bits += 2;
    }
    dev_free(status, s);
    if (rc || !*unique) {
        dev_free(b.cells, s);
        b.cells = nullptr;
        return rc;
    }
    *out = b;
    return PLGPU_OK;
}

// Row-format table over a unique-keyed build side (jn_build_rowformat_kernel);
// *unique = false (and nothing built) when a key repeats.
static int jn_build_rowformat(const plgpu_column* key, const plgpu_column* pay, bool nulls_equal, JnBuilt* out,
                              bool* unique, hipStream_t s) {
    const int64_t nb = key->length;
    int bits = std::max(10, log2_ceil64((nb * 5 + 2) / 3));  // load <= 0.6
    unsigned long long* status = nullptr;
    int rc = dev_alloc((void**)&status, 32, s);
    *unique = true;
    JnBuilt b;
    for (int attempt = 0; !rc; ++attempt) {
        b.t.bits = bits;
        b.t.bbits = bits - 3;
        b.t.cap = int64_t(1) << bits;
        const int64_t ne = b.t.cap + 2;
        if ((rc = dev_alloc((void**)&b.t.cells, ne * 16, s))) break;
        hipError_t e = hipMemsetAsync(status, 0, 32, s);
        // keys EMPTY everywhere; special cells all zero (unoccupied)
        if (e == hipSuccess) e = hipMemsetAsync(b.t.cells, 0x00, ne * 16, s);
        if (e == hipSuccess) {
            const int gi = (int)std::min<int64_t>((ne + 255) / 256, 256 * 32);
            jn_empty_kernel<<<gi, 256, 0, s>>>(b.t);
            const int gb = (int)std::min<int64_t>((nb + 255) / 256, 256 * 32);
            if (nb > 0) {
                KtScope kt("jn_build_rowformat_kernel", s);
                jn_build_rowformat_kernel<<<gb, 256, 0, s>>>(dev_col(*key), nb, b.t, nulls_equal, dev_col(*pay),
                                                             status);
            }
            e = hipGetLastError();
        }
        unsigned long long st[4] = {0, 0, 0, 0};
        if (e == hipSuccess) e = hipMemcpyAsync(st, status, 32, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            rc = hip_fail(e, "join row-format build");
            break;
        }
        if (st[1]) {
            *unique = false;
            break;
        }
        if (st[0] == 0) break;
        if (attempt >= 3) {
            rc = fail(PLGPU_ERR_CAPACITY, "join build table did not converge");
            break;
        }
        dev_free(b.t.cells, s);
        b.t.cells = nullptr;
        bits += 2;
    }
    dev_free(status, s);
    if (rc || !*unique) {
        jn_free(b, s);
        return rc;
    }
    b.rows = nb;
    *out = b;
    return PLGPU_OK;
}

// One probe pass: per-row match words, per-tile output counts and their
// exclusive scan; `total` output rows.
struct JnPass {
    uint32_t* m = nullptr;
    uint64_t* tcount = nullptr;
    uint64_t* toff = nullptr;
    uint64_t* part = nullptr;
    int64_t np = 0;
    int64_t ntiles = 0;
    uint64_t total = 0;
};

static void jn_pass_free(JnPass& p, hipStream_t s) {
    dev_free(p.m, s);
    dev_free(p.tcount, s);
    dev_free(p.toff, s);
    dev_free(p.part, s);
    p = JnPass();
}

static int jn_pass_alloc(int64_t np, JnPass* p, hipStream_t s) {
    p->np = np;
    p->ntiles = std::max<int64_t>(1, (np + kJnTileRows - 1) / kJnTileRows);
    int rc = dev_alloc((void**)&p->tcount, p->ntiles * 8, s);
    if (!rc) rc = dev_alloc((void**)&p->toff, (p->ntiles + 1) * 8, s);
    if (!rc) rc = dev_alloc((void**)&p->part, ((p->ntiles + kScanChunk - 1) / kScanChunk + 1) * 8, s);
    if (!rc) rc = dev_alloc((void**)&p->m, std::max<int64_t>(np, 1) * 4, s);
    return rc;
}

static int jn_pass_grid(const JnPass& p) { return (int)std::min<int64_t>(p.ntiles, (int64_t)num_cus_jn() * 8); }

// Scan of the tile counts -> p->total (host).
static int jn_pass_scan(JnPass* p, hipStream_t s, const char* what) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = scan_exclusive<uint64_t>(p->tcount, p->ntiles, p->toff, p->part, s);
    if (e == hipSuccess) e = hipMemcpyAsync(&p->total, p->toff + p->ntiles, 8, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return e == hipSuccess ? PLGPU_OK : hip_fail(e, what);
}

template <int MODE, bool MARK>
static void jn_launch_match(const DevCol& pk, const JnPass& p, const JnBuilt& b, bool neq, uint8_t* flags,
                            hipStream_t s) {
    const int g = jn_pass_grid(p);
    KtScope kt("jn_probe_match_kernel", s);
    if (pk.validity)
        jn_probe_match_kernel<true, MODE, MARK><<<g, kJnThreads, 0, s>>>(pk, p.np, b.t, neq, p.m, p.tcount, p.ntiles,
                                                                         flags);
    else
        jn_probe_match_kernel<false, MODE, MARK><<<g, kJnThreads, 0, s>>>(pk, p.np, b.t, neq, p.m, p.tcount, p.ntiles,
                                                                          flags);
}

// Match pass of `key` against the table in `mode` (MARK: set flags[slot] of
// every matched slot; JM_DRAIN reads them).
static int jn_match(const plgpu_column* key, const JnBuilt& b, bool neq, int mode, bool mark, uint8_t* flags,
                    JnPass* p, hipStream_t s) {
    int rc = jn_pass_alloc(key->length, p, s);
    if (rc) return rc;
    const DevCol pk = as_dev(key);
    switch (mode) {
    case JM_INNER:
        if (mark) jn_launch_match<JM_INNER, true>(pk, *p, b, neq, flags, s);
        else jn_launch_match<JM_INNER, false>(pk, *p, b, neq, flags, s);
        break;
    case JM_OUTER:
        if (mark) jn_launch_match<JM_OUTER, true>(pk, *p, b, neq, flags, s);
        else jn_launch_match<JM_OUTER, false>(pk, *p, b, neq, flags, s);
        break;
    case JM_SEMI: jn_launch_match<JM_SEMI, false>(pk, *p, b, neq, flags, s); break;
    case JM_ANTI: jn_launch_match<JM_ANTI, false>(pk, *p, b, neq, flags, s); break;
    default: jn_launch_match<JM_DRAIN, false>(pk, *p, b, neq, flags, s); break;
    }
    return jn_pass_scan(p, s, "join probe match");
}

// Emit pass: rows / pairs of `p` in probe-row order into out_p / out_b.
static int jn_emit(const JnPass& p, const JnBuilt& b, int mode, uint32_t* out_p, uint32_t* out_b,
                   const uint32_t* rowmap, hipStream_t s) {
    if (p.total == 0) return PLGPU_OK;
    const int g = jn_pass_grid(p);
    KtScope kt("jn_probe_emit_kernel", s);
    switch (mode) {
    case JM_INNER:
        jn_probe_emit_kernel<JM_INNER><<<g, kJnThreads, 0, s>>>(p.np, b.t, p.m, p.toff, p.ntiles, out_p, out_b, rowmap);
        break;
    case JM_OUTER:
        jn_probe_emit_kernel<JM_OUTER><<<g, kJnThreads, 0, s>>>(p.np, b.t, p.m, p.toff, p.ntiles, out_p, out_b, rowmap);
        break;
    case JM_SEMI:
        jn_probe_emit_kernel<JM_SEMI><<<g, kJnThreads, 0, s>>>(p.np, b.t, p.m, p.toff, p.ntiles, out_p, out_b, rowmap);
        break;
    default:
        jn_probe_emit_kernel<JM_ANTI><<<g, kJnThreads, 0, s>>>(p.np, b.t, p.m, p.toff, p.ntiles, out_p, out_b, rowmap);
        break;
    }
    PLGPU_HIP(hipGetLastError());
    return PLGPU_OK;
}

// Validity bits of an index column: kNullIdx entries are null.
__global__ __launch_bounds__(256) void jn_idx_validity_kernel(const uint32_t* __restrict__ v, int64_t n,
                                                              uint64_t* __restrict__ words) {
    for (int64_t r0 = (int64_t)blockIdx.x * blockDim.x; r0 < n; r0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = r0 + threadIdx.x;
        const uint64_t w = __ballot(r < n && v[r] != kNullIdx);
        if ((threadIdx.x & 63) == 0 && r < n) words[r >> 6] = w;
    }
}

static int jn_idx_validity(plgpu_column* c, hipStream_t s) {
    if (c->validity == nullptr || c->length == 0) return PLGPU_OK;
    const int g = (int)std::min<int64_t>((c->length + 255) / 256, (int64_t)num_cus_jn() * 16);
    jn_idx_validity_kernel<<<g, 256, 0, s>>>((const uint32_t*)c->values, c->length, (uint64_t*)c->validity);
    PLGPU_HIP(hipGetLastError());
    return PLGPU_OK;
}

// Semi / anti rows out of verified left-join pairs (a ascending, b =
// kNullIdx for a row without a match): semi keeps the first pair of every
// matched left row, anti the unmatched rows.  A kept pair gets the JM_ANTI
// emit mark (kRefNone); the emit writes a[i] through its row map.
__global__ __launch_bounds__(kJnThreads) void jn_select_kernel(const uint32_t* __restrict__ a,
                                                               const uint32_t* __restrict__ b, int64_t n, bool semi,
                                                               uint32_t* __restrict__ m,
                                                               uint64_t* __restrict__ tile_counts, int64_t ntiles) {
    __shared__ uint64_t wsum[kJnThreads / 64];
    constexpr int R = kJnTileRows / kJnThreads;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        uint64_t c = 0;
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int64_t r = tile * kJnTileRows + (int64_t)k * kJnThreads + threadIdx.x;
            if (r >= n) continue;
            const bool keep = semi ? (b[r] != kNullIdx && (r == 0 || a[r - 1] != a[r])) : b[r] == kNullIdx;
            m[r] = keep ? kRefNone : 0u;
            c += keep ? 1 : 0;
        }
        uint64_t total;
        (void)block_excl_scan(c, wsum, total);
        if (threadIdx.x == 0) tile_counts[tile] = total;
    }
}


static int check_key(const plgpu_column* k) {
    if (k == nullptr) return fail(PLGPU_ERR_INVALID, "join key is NULL");
    if (!dtype_is_int(k->dtype)) return fail(PLGPU_ERR_SCHEMA, "join key must be an integer column");
    if (k->length >= 0xFFFFFFFFll) return fail(PLGPU_ERR_CAPACITY, "join side exceeds the u32 index space");
    return PLGPU_OK;
}

// Stable sort of the pairs by the left (or right) index, a null index last.
static int jn_sort_pairs(plgpu_column* li, plgpu_column* ri, bool by_right, hipStream_t s) {
    plgpu_column perm;
    int rc = plgpu_arg_sort(by_right ? ri : li, 0, 1, &perm, s);
    if (rc) {
        plgpu_column_release(li);
        plgpu_column_release(ri);
        return rc;
    }
    plgpu_column in[2] = {*li, *ri};
    plgpu_column out[2];
    rc = plgpu_gather(in, 2, &perm, out, s);
    plgpu_column_release(&perm);
    plgpu_column_release(li);
    plgpu_column_release(ri);
    if (rc) return rc;
    *li = out[0];
    *ri = out[1];
    return PLGPU_OK;
}

// Join of two checked key columns (validation failures return
// PLGPU_ERR_SCHEMA; nothing else does).  How each join type maps onto a
// build side, probe mode and drain (DESIGN.md §Join types):
//   inner  probe the side whose order is kept (else build the shorter side);
//   left   build right, probe left with JM_OUTER -- left order, matches in
//          right-row order, as hash_join_tuples_left; with a right-first
//          order, build left, probe right (JM_INNER, marking) and drain the
//          unmatched left rows, which is what the reference's stable sort by
//          the right index (dispatch_left_right.rs:143) yields;
//   right  the left join with the sides swapped and the order flipped
//          (dispatch_left_right.rs:19);
//   full   probe with JM_OUTER + marks, then drain the unmarked build rows
//          (probe_outer); the build side follows maintain_order so that the
//          pairs come out already in the reference's sorted order
//          (hash_join/mod.rs:164), else the shorter side as
//          det_hash_prone_order;
//   semi / anti  build right, probe left (hash_join_tuples_left_semi/_anti).
static int join_impl(const plgpu_column* left_key, const plgpu_column* right_key, int32_t how, bool neq,
                     int32_t maintain_order, int32_t validate, plgpu_column* out_left_idx,
                     plgpu_column* out_right_idx, hipStream_t s) {
    int rc;
    std::memset(out_left_idx, 0, sizeof *out_left_idx);
    std::memset(out_right_idx, 0, sizeof *out_right_idx);
    if (how == PLGPU_JOIN_RIGHT) {
        static const int32_t flip[5] = {PLGPU_JOIN_ORDER_NONE, PLGPU_JOIN_ORDER_RIGHT, PLGPU_JOIN_ORDER_LEFT,
                                        PLGPU_JOIN_ORDER_RIGHT_LEFT, PLGPU_JOIN_ORDER_LEFT_RIGHT};
        return join_impl(right_key, left_key, PLGPU_JOIN_LEFT, neq, flip[maintain_order], validate, out_right_idx,
                         out_left_idx, s);
    }
    const bool order_left = maintain_order == PLGPU_JOIN_ORDER_LEFT || maintain_order == PLGPU_JOIN_ORDER_LEFT_RIGHT;
    const bool order_right =
        maintain_order == PLGPU_JOIN_ORDER_RIGHT || maintain_order == PLGPU_JOIN_ORDER_RIGHT_LEFT;
    {
        // The ordered plans probe the side whose order is kept, so they build
        // on the other side.  When that side is the much larger one (a 1e9-row
        // table for a 1e7-row probe), build on the small side instead and
        // stably sort the pairs by the kept side's index (nulls last), which
        // is what the reference itself does (dispatch_left_right.rs:143,
        // hash_join/mod.rs:164).  The base order of the swapped plan has the
        // other side's rows ascending within each kept row, as required.
        const int64_t nl = left_key->length, nr = right_key->length;
        const bool swap_right = order_right && (how == PLGPU_JOIN_INNER || how == PLGPU_JOIN_LEFT ||
                                                how == PLGPU_JOIN_FULL) && nl > 2 * nr;
        const bool swap_left = order_left && (how == PLGPU_JOIN_INNER || how == PLGPU_JOIN_FULL) && nr > 2 * nl;
        if (swap_right || swap_left) {
            rc = join_impl(left_key, right_key, how, neq, swap_right ? PLGPU_JOIN_ORDER_LEFT : PLGPU_JOIN_ORDER_RIGHT,
                           validate, out_left_idx, out_right_idx, s);
            if (!rc) rc = jn_sort_pairs(out_left_idx, out_right_idx, swap_right, s);
            return rc;
        }
    }
    bool build_right, ordered = maintain_order != PLGPU_JOIN_ORDER_NONE, drain = false;
    int mode;
    switch (how) {
    case PLGPU_JOIN_LEFT:
        build_right = !order_right;
        mode = order_right ? JM_INNER : JM_OUTER;
        drain = order_right;
        ordered = true;  // the reference's left join is ordered in every mode
        break;
    case PLGPU_JOIN_FULL:
        build_right = order_left || (!order_right && right_key->length <= left_key->length);
        mode = JM_OUTER;
        drain = true;
        break;
    case PLGPU_JOIN_SEMI:
    case PLGPU_JOIN_ANTI:
        build_right = true;
        mode = how == PLGPU_JOIN_SEMI ? JM_SEMI : JM_ANTI;
        ordered = false;
        validate = PLGPU_JOIN_VALIDATE_M_M;  // semi / anti joins do not validate
        break;
    default:
        // the probe order decides the output order: probe the side whose
        // order must be kept; otherwise build on the shorter side as the
        // reference does
        build_right = order_left || (!order_right && right_key->length <= left_key->length);
        mode = JM_INNER;
        break;
    }
    JnBuilt b;
    rc = jn_build(build_right ? right_key : left_key, neq, ordered, &b, s);
    if (rc) return rc;
    // validation (args.rs JoinValidation): "1:m" left unique, "m:1" right
    // unique, "1:1" both; duplicates of the build side are known from the
    // table, the probe side needs its own table
    const bool need_left = validate == PLGPU_JOIN_VALIDATE_1_M || validate == PLGPU_JOIN_VALIDATE_1_1;
    const bool need_right = validate == PLGPU_JOIN_VALIDATE_M_1 || validate == PLGPU_JOIN_VALIDATE_1_1;
    auto unique_side = [&](bool right_side, bool* unique) -> int {
        if (right_side == build_right) {
            *unique = b.max_count <= 1;
            return PLGPU_OK;
        }
        JnBuilt o;
        int r2 = jn_build(right_side ? right_key : left_key, neq, false, &o, s);
        if (r2) return r2;
        *unique = o.max_count <= 1;
        jn_free(o, s);
        return PLGPU_OK;
    };
    bool ok = true;
    if (!rc && need_left) rc = unique_side(false, &ok);
    if (!rc && !ok) rc = fail(PLGPU_ERR_SCHEMA, "join keys did not fulfill 1:m validation");
    if (!rc && need_right) rc = unique_side(true, &ok);
    if (!rc && !ok)
        rc = fail(PLGPU_ERR_SCHEMA, validate == PLGPU_JOIN_VALIDATE_1_1 ? "join keys did not fulfill 1:1 validation"
                                                                        : "join keys did not fulfill m:1 validation");
    if (rc) {
        jn_free(b, s);
        return rc;
    }
    const plgpu_column* pkey = build_right ? left_key : right_key;
    const plgpu_column* bkey = build_right ? right_key : left_key;
    plgpu_column* op = build_right ? out_left_idx : out_right_idx;
    plgpu_column* ob = build_right ? out_right_idx : out_left_idx;
    uint8_t* flags = nullptr;
    JnPass pp, dp;
    if (drain) {
        rc = dev_alloc((void**)&flags, b.t.cap + 2, s);
        if (!rc && hipMemsetAsync(flags, 0, b.t.cap + 2, s) != hipSuccess) rc = fail(PLGPU_ERR_HIP, "join flags");
    }
    if (!rc) rc = jn_match(pkey, b, neq, mode, drain, flags, &pp, s);
    if (!rc && drain) rc = jn_match(bkey, b, neq, JM_DRAIN, false, flags, &dp, s);
    const uint64_t total = pp.total + dp.total;
    const bool rows_only = mode == JM_SEMI || mode == JM_ANTI;
    if (!rc && total >= 0xFFFFFFFFull) rc = fail(PLGPU_ERR_CAPACITY, "join output exceeds the u32 index space");
    // null partners: the probe side's in drained rows, the build side's for
    // unmatched probe rows (JM_OUTER)
    if (!rc) rc = make_owned_column(op, PLGPU_U32, (int64_t)total, drain, s);
    if (!rc) rc = make_owned_column(ob, PLGPU_U32, rows_only ? 0 : (int64_t)total, mode == JM_OUTER, s);
    if (!rc) rc = jn_emit(pp, b, mode, (uint32_t*)op->values, (uint32_t*)ob->values, nullptr, s);
    if (!rc && drain && dp.total > 0) {
        // drained build rows, each with a null probe-side partner
        rc = jn_emit(dp, b, JM_DRAIN, (uint32_t*)ob->values + pp.total, nullptr, nullptr, s);
        if (!rc && hipMemsetAsync((uint32_t*)op->values + pp.total, 0xFF, dp.total * 4, s) != hipSuccess)
            rc = fail(PLGPU_ERR_HIP, "join drain fill");
    }
    if (!rc) rc = jn_idx_validity(op, s);
    if (!rc) rc = jn_idx_validity(ob, s);
    if (!rc) {
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "join emit");
    }
    jn_pass_free(pp, s);
    jn_pass_free(dp, s);
    dev_free(flags, s);
    jn_free(b, s);
    if (rc) {
        plgpu_column_release(out_left_idx);
        plgpu_column_release(out_right_idx);
    }
    (void)hipStreamSynchronize(s);
    return rc;
}

// Semi / anti rows from verified left-join pairs (multi-key hashed path).
static int jn_select_rows(const plgpu_column& li, const plgpu_column& ri, bool semi, plgpu_column* out,
                          hipStream_t s) {
    std::memset(out, 0, sizeof *out);
    JnPass p;
    int rc = jn_pass_alloc(li.length, &p, s);
    if (!rc) {
        jn_select_kernel<<<jn_pass_grid(p), kJnThreads, 0, s>>>((const uint32_t*)li.values, (const uint32_t*)ri.values,
                                                                p.np, semi, p.m, p.tcount, p.ntiles);
        rc = jn_pass_scan(&p, s, "join semi/anti select");
    }
    JnBuilt none;
    if (!rc) rc = make_owned_column(out, PLGPU_U32, (int64_t)p.total, false, s);
    if (!rc) rc = jn_emit(p, none, JM_ANTI, (uint32_t*)out->values, nullptr, (const uint32_t*)li.values, s);
    if (!rc) {
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "join semi/anti select");
    }
    jn_pass_free(p, s);
    if (rc) plgpu_column_release(out);
    return rc;
}

// ------------------------------------------------------- multi-key join
// Key tuples -> 64-bit hashes (tuplehash.hpp); a tuple holding a null is a
// null key unless nulls_equal.  Validity is written one wave ballot per 64
// rows (grid-stride bases are multiples of 64).
__global__ __launch_bounds__(256) void jn_tuple_hash_kernel(MkKeys k, int64_t n, uint64_t seed, uint64_t mask, bool neq,
                                                            uint64_t* __restrict__ hash,
                                                            uint64_t* __restrict__ valid_words) {
    for (int64_t r0 = (int64_t)blockIdx.x * blockDim.x; r0 < n; r0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = r0 + threadIdx.x;
        const bool in = r < n;
        const bool v = in && (neq || !mk_any_null(k, r));
        if (in) hash[r] = mk_row_hash(k, r, seed) & mask;
        const uint64_t b = __ballot(v);
        const int64_t w0 = r - (threadIdx.x & 63);
        if ((threadIdx.x & 63) == 0 && w0 < n) valid_words[w0 >> 6] = b;
    }
}

// Every output pair must join equal tuples (a hash collision otherwise).
__global__ __launch_bounds__(256) void jn_verify_kernel(MkKeys a, MkKeys b, const uint32_t* __restrict__ ia,
                                                        const uint32_t* __restrict__ ib, int64_t n,
                                                        uint32_t* __restrict__ bad) {
    bool x = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (ia[i] != kNullIdx && ib[i] != kNullIdx) x |= !mk_equal(a, ia[i], b, ib[i]);
    if (__any(x) && (threadIdx.x & 63) == 0) atomicOr(bad, 1u);
}

static int check_args(int32_t how, int32_t maintain_order, int32_t validate) {
    if (how < PLGPU_JOIN_INNER || how > PLGPU_JOIN_ANTI) return fail(PLGPU_ERR_INVALID, "invalid join type");
    if (maintain_order < PLGPU_JOIN_ORDER_NONE || maintain_order > PLGPU_JOIN_ORDER_RIGHT_LEFT)
        return fail(PLGPU_ERR_INVALID, "invalid maintain_order");
    if (validate < PLGPU_JOIN_VALIDATE_M_M || validate > PLGPU_JOIN_VALIDATE_1_1)
        return fail(PLGPU_ERR_INVALID, "invalid validate");
    return PLGPU_OK;
}

PLGPU_API int plgpu_join(const plgpu_column* left_key, const plgpu_column* right_key, int32_t how, int32_t nulls_equal,
                         int32_t maintain_order, int32_t validate, plgpu_column* out_left_idx,
                         plgpu_column* out_right_idx, void* stream) {
    int rc;
    if ((rc = check_key(left_key)) || (rc = check_key(right_key))) return rc;
    if (out_left_idx == nullptr || out_right_idx == nullptr) return fail(PLGPU_ERR_INVALID, "NULL output");
    if ((rc = check_args(how, maintain_order, validate))) return rc;
    return join_impl(left_key, right_key, how, nulls_equal != 0, maintain_order, validate, out_left_idx,
                     out_right_idx, as_stream(stream));
}

PLGPU_API int plgpu_join_inner(const plgpu_column* left_key, const plgpu_column* right_key, int32_t nulls_equal,
                               int32_t maintain_order, int32_t validate, plgpu_column* out_left_idx,
                               plgpu_column* out_right_idx, void* stream) {
    return plgpu_join(left_key, right_key, PLGPU_JOIN_INNER, nulls_equal, maintain_order, validate, out_left_idx,
                      out_right_idx, stream);
}

template <int NC>
static void jn_take_emit(const JnPass& pp, const TakeCols& lc, const TakePay& tp, int W, uint32_t* out_idx,
                         hipStream_t s) {
    KtScope kt("jn_take_emit_kernel", s);
    if (W == 1)
        jn_take_emit_kernel<NC, 1><<<jn_pass_grid(pp), kJnThreads, 0, s>>>(pp.np, (const uint64_t*)pp.m, tp, pp.toff,
                                                                           pp.ntiles, lc, out_idx);
    else if (W == 2)
        jn_take_emit_kernel<NC, 2><<<jn_pass_grid(pp), kJnThreads, 0, s>>>(pp.np, (const uint64_t*)pp.m, tp, pp.toff,
                                                                           pp.ntiles, lc, out_idx);
    else
        jn_take_emit_kernel<NC, 3><<<jn_pass_grid(pp), kJnThreads, 0, s>>>(pp.np, (const uint64_t*)pp.m, tp, pp.toff,
                                                                           pp.ntiles, lc, out_idx);
}

// ------------------------------------------------ partitioned join (round 6)
// The order-free inner join + take of BASELINE configs[3] (one unique-keyed
// build payload, null-free 8-byte keys and columns) as a radix join, so that
// every table read is served by an XCD's L2 instead of the ~55 G random
// line requests/s of the HBM / Infinity-Cache-resident row-format table:
//   1. the build keys go into P = 2^pbits sub-tables, one per partition
//      (the top pbits bits of part_hash(key)), each nbk 64-B buckets of four
//      16-B cells {key, payload} at load <= 1/2 (~1.25 MiB for 2^15 keys);
//   2. the probe rows -- key and carried left columns as raw words -- are
//      radix-partitioned by the same bits (radix_partition8: the group-by's
//      count / scan / LDS-staged scatter), so a partition's rows meet only
//      its own sub-table;
//   3. the match pass (rj_match_kernel) walks the partitioned rows in
//      4,096-row tiles, split into eight contiguous ranges, one per
//      workgroup group (blockIdx % 8: the blocks one XCD receives), so an
//      XCD probes one or two sub-tables at a time and holds them in its L2;
//      four lanes read a probe row's home bucket together (one 64-B
//      request); it writes the row-format join's intermediate layout (hit
//      words, packed payloads, tile counts);
//   4. the row-format join's scan and emit (jn_take_emit_kernel) place the
//      rows: the key and carried columns come from the partition buffers,
//      the payloads from the match pass.  Outputs are allocated at the exact
//      result length; no atomics.
// The rows come out in partition order: maintain_order = "none", the
// reference's and this library's default.  The reference builds per-
// partition tables the same way (polars-ops/src/frame/join/hash_join/
// single_keys.rs:16 build_tables) and probes each partition's rows against
// its own table (single_keys_inner.rs:40 probe_inner).
constexpr int kMaxAccCarry = 6;                 // carried left columns besides the key (radix_partition8)
constexpr int kRjGroups = 8;                    // workgroup groups (one XCD each)
constexpr int kRjMaxBits = 12;                  // partitions <= 4,096

struct RjTable {
    const uint4* cells;  // P * nbk buckets of 4 cells {key lo, key hi, payload lo, payload hi}
    uint32_t nbk;        // buckets per sub-table
    int32_t pbits;
};

__device__ __forceinline__ uint32_t rj_part(uint64_t h, int pbits) {
    return pbits ? (uint32_t)(h >> (64 - pbits)) : 0u;
}
// home bucket within the sub-table: the hash's low word scaled to nbk
__device__ __forceinline__ uint32_t rj_bucket(uint64_t h, uint32_t nbk) {
    return (uint32_t)(((uint64_t)(uint32_t)h * nbk) >> 32);
}

__global__ __launch_bounds__(256) void rj_count_kernel(DevCol bk, int64_t nb, int pbits, uint32_t* __restrict__ counts) {
    __shared__ uint32_t h[1 << kRjMaxBits];
    const int P = 1 << pbits;
    for (int i = threadIdx.x; i < P; i += blockDim.x) h[i] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&h[rj_part(part_hash(dev_load(bk, i)), pbits)], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < P; i += blockDim.x)
        if (h[i]) atomicAdd(&counts[i], h[i]);
}

__global__ __launch_bounds__(256) void rj_init_kernel(uint4* __restrict__ cells, int64_t ncells) {
    const uint4 e = make_uint4((uint32_t)kEmptyKey, (uint32_t)(kEmptyKey >> 32), 0u, 0u);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ncells; i += (int64_t)gridDim.x * blockDim.x)
        cells[i] = e;
}

// status[0]: a key found no free cell; [1]: a key met twice; [2]: an
// INT64_MIN key (the empty marker).  The caller falls back for any.
__global__ __launch_bounds__(256) void rj_build_kernel(DevCol bk, DevCol pay, int64_t nb, uint4* __restrict__ cells,
                                                      uint32_t nbk, int pbits, unsigned long long* status) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t key = dev_load(bk, i);
        if (key == kEmptyKey) {
            atomicOr(&status[2], 1ull);
            continue;
        }
        const uint64_t h = part_hash(key);
        uint64_t* sub = (uint64_t*)(cells + (size_t)rj_part(h, pbits) * nbk * 4);
        uint32_t b = rj_bucket(h, nbk);
        bool placed = false;
        for (uint32_t q = 0; q < nbk && !placed; ++q) {
            for (int c = 0; c < 4; ++c) {
                uint64_t* kp = sub + ((size_t)b * 4 + c) * 2;
                uint64_t k = __hip_atomic_load(kp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (k == kEmptyKey) {
                    k = atomicCAS((unsigned long long*)kp, (unsigned long long)kEmptyKey, (unsigned long long)key);
                    if (k == kEmptyKey) {
                        kp[1] = dev_load(pay, i);
                        placed = true;
                        break;
                    }
                }
                if (k == key) {
                    atomicOr(&status[1], 1ull);
                    placed = true;
                    break;
                }
            }
            b = b + 1 == nbk ? 0u : b + 1;
        }
        if (!placed) atomicOr(&status[0], 1ull);
    }
}

// The match pass of the partitioned probe, in the row-format join's
// intermediate layout (jn_probe_match_kernel<.., INLINE>), so that its scan
// and its emit (jn_take_emit_kernel) finish the join: per 64 partitioned rows
// one hit word, the hits' payloads packed in hit order at the start of the
// rows' 64-word segment of mp, and per 4,096-row tile its hit count.  Row r
// of tile t is t * 4096 + k * 256 + tid (k = 0 .. 15).  The tiles are taken
// in partitioned-row order within eight contiguous ranges, one per workgroup
// group (blockIdx % 8: the blocks one XCD receives), so an XCD walks its
// partitions in order and their sub-tables stay in its L2.  Each row is
// hashed once, by its own lane (key and home bucket staged in LDS); the
// wave then probes cooperatively: in a step, lanes 4g .. 4g + 3 read the
// four cells of row g's home bucket (one 64-B request per row), kRjBatch
// steps' reads in flight together.  A workgroup takes half a tile; the two
// halves add their hit counts to the tile's, and the scan of the tile counts
// places the rows.
template <int kRjBatch>
__global__ __launch_bounds__(kJnThreads) void rj_match_kernel(const uint64_t* __restrict__ keys, int64_t np,
                                                             int64_t ntiles, RjTable t, uint64_t* __restrict__ mwords,
                                                             uint64_t* __restrict__ mp,
                                                             unsigned long long* __restrict__ tile_counts) {
    // a workgroup takes half a 4,096-row tile: chunks 8h .. 8h + 7 (row
    // tile * 4096 + k * 256 + tid), its hit count added to the tile's
    constexpr int R = kJnTileRows / kJnThreads / 2;  // 8 rows per thread
    constexpr int NW = kJnThreads / 64;
    constexpr int CB = kRjBatch / 4;                  // 64-row chunks per batch
    __shared__ uint64_t skey[NW][R * 64];             // the wave's keys, then its hits' payloads
    __shared__ uint32_t sgb[NW][R * 64];              // each row's home bucket (~0: no probe)
    __shared__ uint64_t wsum[NW];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t nhalf = 2 * ntiles;
    const int64_t per = (nhalf + kRjGroups - 1) / kRjGroups;
    const int64_t half = (int64_t)(blockIdx.x % kRjGroups) * per + (int64_t)(blockIdx.x / kRjGroups);
    if (half >= nhalf) return;  // (uniform: the whole workgroup)
    const int64_t tile = half >> 1, kb = (half & 1) * R;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const int g = lane >> 2, c4 = lane & 3;
    const uint4 empty_cell = make_uint4((uint32_t)kEmptyKey, (uint32_t)(kEmptyKey >> 32), 0u, 0u);
    const uint32_t nbk = t.nbk;
    // the half tile's keys (all loads out at once), each hashed once by its
    // own lane: the home bucket over the whole table (partition * nbk +
    // bucket), or ~0 for a row past the end or an INT64_MIN key
    uint64_t key[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int64_t r = tile * kJnTileRows + (int64_t)(kb + k) * kJnThreads + threadIdx.x;
        key[k] = __builtin_nontemporal_load(keys + (r < np ? r : np - 1));
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int64_t r = tile * kJnTileRows + (int64_t)(kb + k) * kJnThreads + threadIdx.x;
        const uint64_t h = part_hash(key[k]);
        skey[w][k * 64 + lane] = key[k];
        sgb[w][k * 64 + lane] = r < np && key[k] != kEmptyKey ? rj_part(h, t.pbits) * nbk + rj_bucket(h, nbk) : ~0u;
    }
    uint32_t cnt = 0;
#pragma unroll 1
    for (int k0 = 0; k0 < R; k0 += CB) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // step i: rows i * 16 .. i * 16 + 15 of the batch (chunk i / 4)
        uint64_t kq[kRjBatch];
        uint32_t bq[kRjBatch];
        uint4 cell[kRjBatch];
        bool open[kRjBatch];
#pragma unroll
        for (int i = 0; i < kRjBatch; ++i) {
            const int q = k0 * 64 + i * 16 + g;
            kq[i] = skey[w][q];
            bq[i] = sgb[w][q];
            open[i] = bq[i] != ~0u;
            // (every lane loads: a closed row reads bucket 0 and discards it)
            const uint4 c = t.cells[(size_t)(open[i] ? bq[i] : 0u) * 4 + c4];
            cell[i] = open[i] ? c : empty_cell;
        }
        uint64_t hm[kRjBatch];
#pragma unroll
        for (int i = 0; i < kRjBatch; ++i) hm[i] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // rounds of bucket reads: every step's open rows read their next
        // bucket together (a full home bucket without the key continues;
        // rare at load <= 1/2)
        for (uint32_t rd = 0;; ++rd) {
            bool again = false;
#pragma unroll
            for (int i = 0; i < kRjBatch; ++i) {
                const uint64_t ck = (uint64_t)cell[i].x | ((uint64_t)cell[i].y << 32);
                const bool hit = open[i] && ck == kq[i];
                const uint64_t m = __ballot(hit);
                const uint64_t done = m | __ballot(ck == kEmptyKey);
                if (hit) skey[w][k0 * 64 + i * 16 + g] = (uint64_t)cell[i].z | ((uint64_t)cell[i].w << 32);
                hm[i] |= m;
                open[i] = open[i] && ((done >> (4 * g)) & 0xFull) == 0;
                again = again || open[i];
            }
            if (!__any(again) || rd + 1 >= nbk) break;
#pragma unroll
            for (int i = 0; i < kRjBatch; ++i) {
                if (!open[i]) continue;
                // the next bucket within the row's partition
                const uint32_t q = bq[i] / nbk;
                bq[i] = bq[i] + 1 == (q + 1) * nbk ? q * nbk : bq[i] + 1;
                cell[i] = t.cells[(size_t)bq[i] * 4 + c4];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // each chunk's hit word (16 bits per step) and its packed payloads
#pragma unroll
        for (int c = 0; c < CB; ++c) {
            uint64_t hw = 0;
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const uint64_t x = hm[c * 4 + s4];
                const uint64_t gm = __ballot(lane < 16 && ((x >> (4 * lane)) & 0xFull) != 0) & 0xFFFFull;
                hw |= gm << (16 * s4);
            }
            const int64_t r = tile * kJnTileRows + (int64_t)(kb + k0 + c) * kJnThreads + threadIdx.x;
            const int64_t seg = r - lane;
            if (seg < np) {
                if (lane == 0) mwords[seg >> 6] = hw;
                if ((hw >> lane) & 1ull) mp[seg + __popcll(hw & lt)] = skey[w][(k0 + c) * 64 + lane];
            }
            cnt += (uint32_t)__popcll(hw);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (lane == 0) wsum[w] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t s = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) s += wsum[i];
        if (s) atomicAdd(&tile_counts[tile], (unsigned long long)s);
    }
}

// -> PLGPU_OK with *done = true, or *done = false (the build side has a
// repeated or INT64_MIN key: the caller runs the row-format join instead).
static int jn_radix_take(const plgpu_column* left_key, const plgpu_column* right_key, const plgpu_column* left_cols,
                         int32_t nleft, const plgpu_column* right_pay, plgpu_column* out_left,
                         plgpu_column* out_right, int64_t* out_len, bool* done, hipStream_t s) {
    *done = false;
    const int64_t np = left_key->length, nb = right_key->length;
    // carried left columns (each once; the key is carried as the partition key)
    int carry_of[PLGPU_MAX_COLS];
    DevCol carry[kMaxAccCarry];
    int nc = 0;
    auto same = [](const plgpu_column& a, const plgpu_column& b) {
        return a.values == b.values && a.offset == b.offset && a.dtype == b.dtype;
    };
    for (int i = 0; i < nleft; ++i) {
        carry_of[i] = -1;
        if (same(left_cols[i], *left_key)) continue;
        for (int j = 0; j < i && carry_of[i] < 0; ++j)
            if (carry_of[j] >= 0 && same(left_cols[i], left_cols[j])) carry_of[i] = carry_of[j];
        if (carry_of[i] >= 0) continue;
        if (nc == kMaxAccCarry) return PLGPU_OK;
        carry_of[i] = nc;
        carry[nc++] = as_dev(&left_cols[i]);
    }
    // partitions of ~2^15 build keys (sub-tables of ~1.25 MiB)
    const int64_t per = options().join_radix_keys > 0 ? options().join_radix_keys : (int64_t(1) << 15);
    int pbits = 0;
    while (pbits < kRjMaxBits && (nb >> pbits) > per) ++pbits;
    // one scatter pass (<= 2^8 partitions) while the sub-tables stay under
    // twice the target (~2.5 MiB): a second pass costs more than the L2
    // misses it saves (1e7 keys: 2^8 partitions of ~39k keys)
    if (pbits > 8 && (nb >> 8) <= 2 * per && options().join_radix_keys <= 0) pbits = 8;
    const int P = 1 << pbits;
    const int cus = num_cus_jn();
    const DevCol bk = as_dev(right_key), bp = as_dev(right_pay);
    uint32_t* cnt = nullptr;
    unsigned long long* status = nullptr;  // build flags
    int rc = dev_alloc((void**)&cnt, (size_t)P * 4, s);
    if (!rc) rc = dev_alloc((void**)&status, 4 * 8, s);
    std::vector<uint32_t> hc((size_t)P);
    if (!rc) {
        hipError_t e = hipMemsetAsync(cnt, 0, (size_t)P * 4, s);
        if (e == hipSuccess) e = hipMemsetAsync(status, 0, 4 * 8, s);
        if (e == hipSuccess && nb > 0) {
            rj_count_kernel<<<(unsigned)std::max<int64_t>(1, std::min<int64_t>((nb + 255) / 256, cus * 4)), 256, 0,
                              s>>>(bk, nb, pbits, cnt);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(hc.data(), cnt, (size_t)P * 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "rj_count_kernel");
    }
    dev_free(cnt, s);
    uint32_t maxc = 0;
    for (uint32_t c : hc) maxc = std::max(maxc, c);
    const int load = options().join_radix_load > 0 ? std::min(90, options().join_radix_load) : 35;
    const uint32_t nbk = std::max<uint32_t>(1u, (uint32_t)(((uint64_t)maxc * 100 + 4 * load - 1) / (4 * load)));
    uint4* cells = nullptr;
    const int64_t ncells = (int64_t)P * nbk * 4;
    if (!rc) rc = dev_alloc((void**)&cells, (size_t)ncells * 16, s);
    if (!rc) {
        rj_init_kernel<<<(unsigned)std::min<int64_t>((ncells + 255) / 256, cus * 16), 256, 0, s>>>(cells, ncells);
        if (nb > 0) {
            KtScope kt("rj_build_kernel", s);
            rj_build_kernel<<<(unsigned)std::max<int64_t>(1, std::min<int64_t>((nb + 255) / 256, cus * 16)), 256, 0,
                              s>>>(bk, bp, nb, cells, nbk, pbits, status);
        }
        hipError_t e = hipGetLastError();
        unsigned long long hs[3] = {0, 0, 0};
        if (e == hipSuccess) e = hipMemcpyAsync(hs, status, sizeof hs, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "rj_build_kernel");
        if (!rc && (hs[0] || hs[1] || hs[2])) {
            // duplicate / INT64_MIN build keys: the row-format join decides
            dev_free(cells, s);
            dev_free(status, s);
            return PLGPU_OK;
        }
    }
    dev_free(status, s);
    if (rc) {
        dev_free(cells, s);
        return rc;
    }
    RjTable tab;
    tab.cells = cells;
    tab.nbk = nbk;
    tab.pbits = pbits;
    // the probe rows, partitioned with their carried columns
    RadixParts parts;
    rc = radix_partition8(as_dev(left_key), carry, nc, np, pbits, s, &parts);
    // match pass (hit words, packed payloads, tile counts) and its scan
    JnPass pp;
    uint64_t* mp = nullptr;
    if (!rc) rc = jn_pass_alloc(np, &pp, s);
    if (!rc) rc = dev_alloc((void**)&mp, (size_t)std::max<int64_t>(np, 1) * 8, s);
    if (!rc && hipMemsetAsync(pp.tcount, 0, (size_t)pp.ntiles * 8, s) != hipSuccess)
        rc = fail(PLGPU_ERR_HIP, "rj_match_kernel tile counts");
    if (!rc) {
        KtScope kt("rj_match_kernel", s);
        const unsigned grid = (unsigned)(((2 * pp.ntiles + kRjGroups - 1) / kRjGroups) * kRjGroups);
        unsigned long long* tc = (unsigned long long*)pp.tcount;
        // 4 probe steps in flight per wave: 54 VGPRs, the LDS bound of 6
        // workgroups per CU (7.69 ms against 7.96 for 8 steps at 86 VGPRs,
        // 1e9 x 1e7, gpurun_out/r06i_*)
        if (options().join_radix_batch == 8)
            rj_match_kernel<8><<<grid, kJnThreads, 0, s>>>(parts.key, np, pp.ntiles, tab, (uint64_t*)pp.m, mp, tc);
        else
            rj_match_kernel<4><<<grid, kJnThreads, 0, s>>>(parts.key, np, pp.ntiles, tab, (uint64_t*)pp.m, mp, tc);
    }
    if (!rc) rc = jn_pass_scan(&pp, s, "rj_match_kernel");
    const int64_t total = (int64_t)pp.total;
    // outputs: exact length; the emit writes every left column from the
    // partition buffers (the key listing(s) from the partitioned keys) and
    // the payloads from mp
    TakeCols lc;
    std::memset(&lc, 0, sizeof lc);
    for (int i = 0; i < nleft && !rc; ++i) {
        rc = make_owned_column(&out_left[i], left_cols[i].dtype, total, false, s);
        if (rc) break;
        lc.src[lc.n] = carry_of[i] < 0 ? parts.key : parts.col[carry_of[i]];
        lc.dst[lc.n] = (uint64_t*)out_left[i].values;
        ++lc.n;
    }
    if (!rc) rc = make_owned_column(&out_right[0], right_pay->dtype, total, false, s);
    TakePay tp;
    std::memset(&tp, 0, sizeof tp);
    if (!rc) {
        tp.src[0] = mp;
        tp.dst[0] = (uint64_t*)out_right[0].values;
    }
    if (!rc && total > 0) {
        switch (lc.n) {
        case 0: jn_take_emit<0>(pp, lc, tp, 1, nullptr, s); break;
        case 1: jn_take_emit<1>(pp, lc, tp, 1, nullptr, s); break;
        case 2: jn_take_emit<2>(pp, lc, tp, 1, nullptr, s); break;
        case 3: jn_take_emit<3>(pp, lc, tp, 1, nullptr, s); break;
        case 4: jn_take_emit<4>(pp, lc, tp, 1, nullptr, s); break;
        case 5: jn_take_emit<5>(pp, lc, tp, 1, nullptr, s); break;
        case 6: jn_take_emit<6>(pp, lc, tp, 1, nullptr, s); break;
        case 7: jn_take_emit<7>(pp, lc, tp, 1, nullptr, s); break;
        default: jn_take_emit<8>(pp, lc, tp, 1, nullptr, s); break;
        }
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) rc = hip_fail(e, "join take emit");
    }
    if (!rc) {
        const hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "partitioned join");
    }
    if (!rc) {
        *out_len = total;
        *done = true;
    } else {
        for (int i = 0; i < nleft; ++i) plgpu_column_release(&out_left[i]);
        plgpu_column_release(&out_right[0]);
    }
    dev_free(mp, s);
    jn_pass_free(pp, s);
    dev_free(parts.buf, s);
    dev_free(parts.range, s);
    dev_free(cells, s);
    return rc;
}

// Inner join + take: the left frame's columns and the right frame's columns
// at the matching pairs (pairs and their order as plgpu_join_inner), i.e.
// the reference's hash_join_tuples_inner followed by _finish_join's takes.
// With one right column, unique right keys and a null-free 8-byte right
// column the table is row-format: each cell holds {key, payload}, the
// probe's bucket read returns the payload, and the emit pass writes it and
// the null-free 8-byte left columns straight to their output rows -- no
// index pairs, no random gather of the build side.  Everything else takes
// pairs + gathers.
PLGPU_API int plgpu_join_inner_take(const plgpu_column* left_key, const plgpu_column* right_key,
                                    const plgpu_column* left_cols, int32_t nleft, const plgpu_column* right_cols,
                                    int32_t nright, int32_t nulls_equal, int32_t maintain_order, int32_t validate,
                                    plgpu_column* out_left, plgpu_column* out_right, int64_t* out_len,
                                    void* stream) {
    hipStream_t s = as_stream(stream);
    if (out_len == nullptr || (nleft > 0 && (left_cols == nullptr || out_left == nullptr)) ||
        (nright > 0 && (right_cols == nullptr || out_right == nullptr)))
        return fail(PLGPU_ERR_INVALID, "NULL argument");
    if (nleft < 0 || nleft > PLGPU_MAX_COLS || nright < 0 || nright > PLGPU_MAX_COLS)
        return fail(PLGPU_ERR_INVALID, "0..8 columns per side");
    for (int i = 0; i < nleft; ++i) std::memset(&out_left[i], 0, sizeof out_left[i]);
    for (int i = 0; i < nright; ++i) std::memset(&out_right[i], 0, sizeof out_right[i]);
    *out_len = 0;
    int rc = check_key(left_key);
    if (!rc) rc = check_key(right_key);
    if (!rc) rc = check_args(PLGPU_JOIN_INNER, maintain_order, validate);
    for (int i = 0; i < nleft && !rc; ++i)
        if (left_cols[i].length != left_key->length) rc = fail(PLGPU_ERR_SHAPE, "left column length differs");
    for (int i = 0; i < nright && !rc; ++i)
        if (right_cols[i].length != right_key->length) rc = fail(PLGPU_ERR_SHAPE, "right column length differs");
    if (rc) return rc;
    const bool neq = nulls_equal != 0;
    auto fused8 = [](const plgpu_column& c) {
        return c.validity == nullptr && c.dtype != PLGPU_STR && c.dtype != PLGPU_BOOL && dtype_bytes(c.dtype) == 8;
    };
    // order-free join, one unique-keyed payload, null-free 8-byte integer
    // keys and 8-byte columns: the partitioned join (jn_radix_take) where
    // the build table outgrows the L2s and the probe side is long
    // (option join_radix: 1 there, 2 wherever it applies, 0 off)
    const int jr = options().join_radix;
    if (jr != 0 && maintain_order == PLGPU_JOIN_ORDER_NONE && nright == 1 && fused8(right_cols[0]) &&
        fused8(*left_key) && fused8(*right_key) && dtype_is_int(left_key->dtype) &&
        (validate == PLGPU_JOIN_VALIDATE_M_M || validate == PLGPU_JOIN_VALIDATE_M_1) &&
        right_key->length <= left_key->length && left_key->length < 0xFFFFFFFFll &&
        (jr == 2 ? left_key->length > 0
                 : left_key->length >= (int64_t(1) << 22) && right_key->length >= (int64_t(1) << 17))) {
        bool ok = true;
        for (int i = 0; i < nleft; ++i) ok = ok && fused8(left_cols[i]);
        if (ok) {
            bool done = false;
            rc = jn_radix_take(left_key, right_key, left_cols, nleft, &right_cols[0], out_left, out_right, out_len,
                               &done, s);
            if (rc || done) return rc;
        }
    }
    const bool order_ok = maintain_order == PLGPU_JOIN_ORDER_NONE || maintain_order == PLGPU_JOIN_ORDER_LEFT;
    bool pay8 = nright >= 1 && nright <= 3;
    for (int i = 0; i < nright && pay8; ++i) pay8 = fused8(right_cols[i]);
    const bool inline_ok = order_ok && pay8 &&
                           (validate == PLGPU_JOIN_VALIDATE_M_M || validate == PLGPU_JOIN_VALIDATE_M_1) &&
                           left_key->length >= (int64_t(1) << 16) &&
                           (right_key->length <= left_key->length || maintain_order == PLGPU_JOIN_ORDER_LEFT);
    // W = nright payload words per table cell: 16-B cells for one, 32-B
    // cells (wide table) for two or three
    const int W = nright;
    JnBuilt b;
    WideBuilt wb;
    bool use_inline = false;
    if (inline_ok && W == 1) {
        rc = jn_build_rowformat(right_key, &right_cols[0], neq, &b, &use_inline, s);
        if (rc) return rc;
    } else if (inline_ok) {
        rc = jn_build_wide(right_key, right_cols, W, neq, &wb, &use_inline, s);
        if (rc) return rc;
    }
    auto release_all = [&]() {
        for (int i = 0; i < nleft; ++i) plgpu_column_release(&out_left[i]);
        for (int i = 0; i < nright; ++i) plgpu_column_release(&out_right[i]);
    };
    if (!use_inline) {
        plgpu_column li, ri;
        rc = join_impl(left_key, right_key, PLGPU_JOIN_INNER, neq, maintain_order, validate, &li, &ri, s);
        if (rc) return rc;
        for (int i = 0; i < nleft && !rc; ++i)
            rc = gather_into(left_cols[i], (const uint32_t*)li.values, li.length, &out_left[i], s);
        for (int i = 0; i < nright && !rc; ++i)
            rc = gather_into(right_cols[i], (const uint32_t*)ri.values, ri.length, &out_right[i], s);
        if (!rc) {
            const hipError_t e = hipStreamSynchronize(s);
            if (e != hipSuccess) rc = hip_fail(e, "join take");
        }
        *out_len = li.length;
        plgpu_column_release(&li);
        plgpu_column_release(&ri);
        if (rc) release_all();
        return rc;
    }
    JnPass pp;
    uint64_t* mp = nullptr;  // W dense payload arrays of np words
    uint32_t* idx = nullptr;
    const int64_t npw = std::max<int64_t>(left_key->length, 1);
    rc = jn_pass_alloc(left_key->length, &pp, s);
    if (!rc) rc = dev_alloc((void**)&mp, npw * 8 * W, s);
    if (!rc) {
        const DevCol pk = as_dev(left_key);
        const int g = jn_pass_grid(pp);
        {
            KtScope kt("jn_probe_match_kernel", s);
            uint64_t* mw = reinterpret_cast<uint64_t*>(pp.m);
            uint64_t* m1 = W > 1 ? mp + npw : nullptr;
            uint64_t* m2 = W > 2 ? mp + 2 * npw : nullptr;
            if (W == 1 && pk.validity)
                jn_probe_match_kernel<true, JM_INNER, false, true><<<g, kJnThreads, 0, s>>>(
                    pk, pp.np, b.t, neq, pp.m, pp.tcount, pp.ntiles, nullptr, mp);
            else if (W == 1)
                jn_probe_match_kernel<false, JM_INNER, false, true><<<g, kJnThreads, 0, s>>>(
                    pk, pp.np, b.t, neq, pp.m, pp.tcount, pp.ntiles, nullptr, mp);
            else if (W == 2 && pk.validity)
                jn_probe_match_wide_kernel<true, 2><<<g, kJnThreads, 0, s>>>(
                    pk, pp.np, wb.cells, wb.cap, wb.bbits, neq, mw, pp.tcount, pp.ntiles, mp, m1, m2);
            else if (W == 2)
                jn_probe_match_wide_kernel<false, 2><<<g, kJnThreads, 0, s>>>(
                    pk, pp.np, wb.cells, wb.cap, wb.bbits, neq, mw, pp.tcount, pp.ntiles, mp, m1, m2);
            else if (pk.validity)
                jn_probe_match_wide_kernel<true, 3><<<g, kJnThreads, 0, s>>>(
                    pk, pp.np, wb.cells, wb.cap, wb.bbits, neq, mw, pp.tcount, pp.ntiles, mp, m1, m2);
            else
                jn_probe_match_wide_kernel<false, 3><<<g, kJnThreads, 0, s>>>(
                    pk, pp.np, wb.cells, wb.cap, wb.bbits, neq, mw, pp.tcount, pp.ntiles, mp, m1, m2);
        }
        rc = jn_pass_scan(&pp, s, "join probe match (row-format table)");
    }
    const int64_t total = (int64_t)pp.total;
    if (!rc && pp.total >= 0xFFFFFFFFull) rc = fail(PLGPU_ERR_CAPACITY, "join output exceeds the u32 index space");
    // left columns: fused (null-free 8-byte) or gathered by the row ids
    TakeCols lc;
    std::memset(&lc, 0, sizeof lc);
    bool need_idx = false;
    for (int i = 0; i < nleft && !rc; ++i) {
        if (!fused8(left_cols[i])) {
            need_idx = true;
            continue;
        }
        rc = make_owned_column(&out_left[i], left_cols[i].dtype, total, false, s);
        if (!rc) {
            lc.src[lc.n] = (const uint64_t*)left_cols[i].values + left_cols[i].offset;
            lc.dst[lc.n] = (uint64_t*)out_left[i].values;
            ++lc.n;
        }
    }
    TakePay tp;
    std::memset(&tp, 0, sizeof tp);
    for (int q = 0; q < W && !rc; ++q) {
        rc = make_owned_column(&out_right[q], right_cols[q].dtype, total, false, s);
        if (!rc) {
            tp.src[q] = mp + q * npw;
            tp.dst[q] = (uint64_t*)out_right[q].values;
        }
    }
    if (!rc && need_idx) rc = dev_alloc((void**)&idx, std::max<int64_t>(total, 1) * 4, s);
    if (!rc && total > 0) {
        switch (lc.n) {
        case 0: jn_take_emit<0>(pp, lc, tp, W, idx, s); break;
        case 1: jn_take_emit<1>(pp, lc, tp, W, idx, s); break;
        case 2: jn_take_emit<2>(pp, lc, tp, W, idx, s); break;
        case 3: jn_take_emit<3>(pp, lc, tp, W, idx, s); break;
        case 4: jn_take_emit<4>(pp, lc, tp, W, idx, s); break;
        case 5: jn_take_emit<5>(pp, lc, tp, W, idx, s); break;
        case 6: jn_take_emit<6>(pp, lc, tp, W, idx, s); break;
        case 7: jn_take_emit<7>(pp, lc, tp, W, idx, s); break;
        default: jn_take_emit<8>(pp, lc, tp, W, idx, s); break;
        }
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) rc = hip_fail(e, "join take emit");
    }
    for (int i = 0; i < nleft && !rc && need_idx; ++i)
        if (!fused8(left_cols[i])) rc = gather_into(left_cols[i], idx, total, &out_left[i], s);
    if (!rc) {
        const hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "join (row-format table)");
    }
    dev_free(idx, s);
    dev_free(mp, s);
    jn_pass_free(pp, s);
    jn_free(b, s);
    dev_free(wb.cells, s);
    if (rc) release_all();
    else *out_len = total;
    return rc;
}

PLGPU_API int plgpu_join_inner_multi(const plgpu_column* left_keys, const plgpu_column* right_keys, int32_t nkeys,
                                     int32_t nulls_equal, int32_t maintain_order, int32_t validate,
                                     plgpu_column* out_left_idx, plgpu_column* out_right_idx, void* stream) {
    return plgpu_join_multi(left_keys, right_keys, nkeys, PLGPU_JOIN_INNER, nulls_equal, maintain_order, validate,
                            out_left_idx, out_right_idx, stream);
}

PLGPU_API int plgpu_join_multi(const plgpu_column* left_keys, const plgpu_column* right_keys, int32_t nkeys,
                               int32_t how, int32_t nulls_equal, int32_t maintain_order, int32_t validate,
                               plgpu_column* out_left_idx, plgpu_column* out_right_idx, void* stream) {
    hipStream_t s = as_stream(stream);
    if (left_keys == nullptr || right_keys == nullptr || out_left_idx == nullptr || out_right_idx == nullptr)
        return fail(PLGPU_ERR_INVALID, "NULL argument");
    if (nkeys < 1 || nkeys > kMaxKeys) return fail(PLGPU_ERR_INVALID, "number of join keys must be 1..8");
    {
        const int rc = check_args(how, maintain_order, validate);
        if (rc) return rc;
    }
    std::memset(out_left_idx, 0, sizeof *out_left_idx);
    std::memset(out_right_idx, 0, sizeof *out_right_idx);
    MkKeys ka, kb;
    std::memset(&ka, 0, sizeof ka);
    std::memset(&kb, 0, sizeof kb);
    ka.n = kb.n = nkeys;
    const int64_t nl = left_keys[0].length, nr = right_keys[0].length;
    for (int i = 0; i < nkeys; ++i) {
        const int32_t dt = left_keys[i].dtype;
        if (!dtype_is_int(dt) && !dtype_is_float(dt) && dt != PLGPU_BOOL && dt != PLGPU_STR)
            return fail(PLGPU_ERR_SCHEMA, "join keys must be integer, float, Boolean or String columns");
        if (right_keys[i].dtype != dt) return fail(PLGPU_ERR_SCHEMA, "datatypes of join keys don't match");
        if (left_keys[i].length != nl || right_keys[i].length != nr)
            return fail(PLGPU_ERR_SHAPE, "join key columns of one side must have equal lengths");
        ka.c[i] = as_dev(&left_keys[i]);
        kb.c[i] = as_dev(&right_keys[i]);
    }
    if (nl >= 0xFFFFFFFFll || nr >= 0xFFFFFFFFll) return fail(PLGPU_ERR_CAPACITY, "join side exceeds the u32 index space");
    {
        // String keys whose strings are all <= 7 bytes on both sides: exact
        // Int64 codes, joined as integer keys (no byte verification)
        bool any_str = false, short_all = true;
        plgpu_column cl[kMaxKeys], cr[kMaxKeys];
        std::memset(cl, 0, sizeof cl);
        std::memset(cr, 0, sizeof cr);
        int rc = PLGPU_OK;
        for (int i = 0; i < nkeys; ++i) {
            cl[i] = left_keys[i];
            cr[i] = right_keys[i];
            if (left_keys[i].dtype != PLGPU_STR || !short_all || rc) continue;
            any_str = true;
            bool a = false, b = false;
            rc = str_short_codes(left_keys[i], &cl[i], &a, s);
            if (!rc) rc = str_short_codes(right_keys[i], &cr[i], &b, s);
            short_all = short_all && a && b;
        }
        if (any_str && !rc && short_all)
            rc = plgpu_join_multi(cl, cr, nkeys, how, nulls_equal, maintain_order, validate, out_left_idx,
                                  out_right_idx, stream);
        for (int i = 0; i < nkeys; ++i) {
            if (left_keys[i].dtype == PLGPU_STR && cl[i].dtype == PLGPU_I64) str_codes_free(&cl[i], s);
            if (right_keys[i].dtype == PLGPU_STR && cr[i].dtype == PLGPU_I64) str_codes_free(&cr[i], s);
        }
        if (rc || (any_str && short_all)) return rc;
    }
    const bool neq = nulls_equal != 0;
    const int cus = num_cus_jn();
    {
        // integer keys whose common ranges fit 63 bits: both sides packed into
        // one exact Int64 key (a tuple with a null is a null key unless
        // nulls_equal), joined once, no verification
        MkPack pk;
        int rc = mk_plan_pack(ka, nl, &kb, nr, cus * 16, &pk, s);
        if (rc) return rc;
        if (pk.ok) {
            uint64_t *cl = nullptr, *cr = nullptr;
            rc = dev_alloc((void**)&cl, (std::max<int64_t>(nl, 1) + (nl + 63) / 64 + 1) * 8, s);
            if (!rc) rc = dev_alloc((void**)&cr, (std::max<int64_t>(nr, 1) + (nr + 63) / 64 + 1) * 8, s);
            uint64_t* vl = cl ? cl + std::max<int64_t>(nl, 1) : nullptr;
            uint64_t* vr = cr ? cr + std::max<int64_t>(nr, 1) : nullptr;
            if (!rc)
                mk_pack_launch(ka, pk, nl, cl, neq ? nullptr : vl, nullptr,
                               (int)std::min<int64_t>((nl + 255) / 256, cus * 16), s);
            if (!rc)
                mk_pack_launch(kb, pk, nr, cr, neq ? nullptr : vr, nullptr,
                               (int)std::min<int64_t>((nr + 255) / 256, cus * 16), s);
            if (!rc) {
                hipError_t e = hipGetLastError();
                if (e != hipSuccess) rc = hip_fail(e, "mk_pack_kernel");
            }
            if (!rc) {
                plgpu_column a, b;
                std::memset(&a, 0, sizeof a);
                std::memset(&b, 0, sizeof b);
                a.dtype = b.dtype = PLGPU_I64;
                a.length = nl;
                b.length = nr;
                a.values = cl;
                b.values = cr;
                a.validity = neq ? nullptr : (const uint8_t*)vl;
                b.validity = neq ? nullptr : (const uint8_t*)vr;
                a.null_count = b.null_count = neq ? 0 : -1;
                rc = join_impl(&a, &b, how, neq, maintain_order, validate, out_left_idx, out_right_idx, s);
            }
            dev_free(cl, s);
            dev_free(cr, s);
            (void)hipStreamSynchronize(s);
            return rc;
        }
    }
    uint64_t *hl = nullptr, *hr = nullptr, *vl = nullptr, *vr = nullptr;
    uint32_t* bad = nullptr;
    int rc = dev_alloc((void**)&hl, std::max<int64_t>(nl, 1) * 8, s);
    if (!rc) rc = dev_alloc((void**)&hr, std::max<int64_t>(nr, 1) * 8, s);
    if (!rc) rc = dev_alloc((void**)&vl, ((nl + 63) / 64 + 1) * 8, s);
    if (!rc) rc = dev_alloc((void**)&vr, ((nr + 63) / 64 + 1) * 8, s);
    if (!rc) rc = dev_alloc((void**)&bad, 4, s);
    plgpu_column cl, cr;
    std::memset(&cl, 0, sizeof cl);
    std::memset(&cr, 0, sizeof cr);
    cl.dtype = cr.dtype = PLGPU_I64;
    cl.length = nl;
    cr.length = nr;
    cl.values = hl;
    cr.values = hr;
    // null tuples are dropped through the key validity (nulls_equal: every
    // tuple is a value, nulls included, and no validity is needed)
    cl.validity = neq ? nullptr : (const uint8_t*)vl;
    cr.validity = neq ? nullptr : (const uint8_t*)vr;
    cl.null_count = cr.null_count = neq ? 0 : -1;
    bool done = false;
    int validation_fails = 0;
    // semi / anti on hashed tuples: a left join whose pairs can be verified,
    // then the semi / anti rows selected from it
    const bool rows_only = how == PLGPU_JOIN_SEMI || how == PLGPU_JOIN_ANTI;
    const int32_t how_h = rows_only ? PLGPU_JOIN_LEFT : how;
    const int32_t order_h = rows_only ? PLGPU_JOIN_ORDER_LEFT : maintain_order;
    for (int attempt = 0; attempt < 4 && !rc && !done; ++attempt) {
        const uint64_t seed = 0x243F6A8885A308D3ull * (uint64_t)(2 * attempt + 1);
        // PLGPU_MK_COLLIDE (tests only): a 3-bit first hash forces collisions
        const uint64_t mask = attempt == 0 && options().mk_collide ? 7ull : ~0ull;
        if (nl > 0)
            jn_tuple_hash_kernel<<<(unsigned)std::min<int64_t>((nl + 255) / 256, cus * 16), 256, 0, s>>>(ka, nl, seed,
                                                                                                       mask, neq, hl, vl);
        if (nr > 0)
            jn_tuple_hash_kernel<<<(unsigned)std::min<int64_t>((nr + 255) / 256, cus * 16), 256, 0, s>>>(kb, nr, seed,
                                                                                                       mask, neq, hr, vr);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            rc = hip_fail(e, "join tuple hash");
            break;
        }
        rc = join_impl(&cl, &cr, how_h, neq, order_h, rows_only ? PLGPU_JOIN_VALIDATE_M_M : validate, out_left_idx,
                       out_right_idx, s);
        if (rc == PLGPU_ERR_SCHEMA && ++validation_fails < 2) {
            // a duplicate hash may be a collision of distinct tuples: a second
            // seed tells a real duplicate (fails again) from a collision
            rc = PLGPU_OK;
            continue;
        }
        if (rc) break;
        const int64_t np = out_left_idx->length;
        uint32_t hbad = 0;
        if (np > 0) {
            e = hipMemsetAsync(bad, 0, 4, s);
            if (e == hipSuccess) {
                jn_verify_kernel<<<(unsigned)std::min<int64_t>((np + 255) / 256, cus * 16), 256, 0, s>>>(
                    ka, kb, (const uint32_t*)out_left_idx->values, (const uint32_t*)out_right_idx->values, np, bad);
                e = hipGetLastError();
            }
            if (e == hipSuccess) e = hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) rc = hip_fail(e, "join tuple verify");
        }
        if (!rc && !hbad) done = true;
        else {
            plgpu_column_release(out_left_idx);
            plgpu_column_release(out_right_idx);
        }
    }
    dev_free(hl, s);
    dev_free(hr, s);
    dev_free(vl, s);
    dev_free(vr, s);
    dev_free(bad, s);
    if (!rc && !done) rc = fail(PLGPU_ERR_CAPACITY, "multi-key join: unresolved 64-bit hash collisions");
    if (!rc && rows_only) {
        plgpu_column rows;
        rc = jn_select_rows(*out_left_idx, *out_right_idx, how == PLGPU_JOIN_SEMI, &rows, s);
        plgpu_column_release(out_left_idx);
        plgpu_column_release(out_right_idx);
        if (!rc) {
            *out_left_idx = rows;
            rc = make_owned_column(out_right_idx, PLGPU_U32, 0, false, s);
            if (rc) plgpu_column_release(out_left_idx);
        }
    }
    (void)hipStreamSynchronize(s);
    return rc;
}

PLGPU_API int plgpu_gather(const plgpu_column* cols, int32_t ncols, const plgpu_column* idx, plgpu_column* out_cols,
                           void* stream) {
    hipStream_t s = as_stream(stream);
    if (idx == nullptr || (ncols > 0 && (cols == nullptr || out_cols == nullptr)))
        return fail(PLGPU_ERR_INVALID, "NULL argument");
    if (idx->dtype != PLGPU_U32) return fail(PLGPU_ERR_SCHEMA, "gather indices must be UInt32");
    for (int i = 0; i < ncols; ++i) std::memset(&out_cols[i], 0, sizeof(plgpu_column));
    const uint32_t* ix = (const uint32_t*)idx->values + idx->offset;
    const int64_t n = idx->length;
    int rc = PLGPU_OK;
    // null-free 8-byte columns of one length (and no null indices): row-major
    // packed gather, in groups of up to kAosMax; everything else column by
    // column
    std::vector<int> packed;
    if (n >= (1 << 20) && idx->validity == nullptr) {
        for (int i = 0; i < ncols; ++i)
            if (cols[i].validity == nullptr && dtype_bytes(cols[i].dtype) == 8 && cols[i].dtype != PLGPU_BOOL &&
                cols[i].length == cols[0].length)
                packed.push_back(i);
        // the packing pass costs a sequential read + write of every column, so
        // it only pays when several columns share the random index
        if (packed.size() < 4) packed.clear();
    }
    std::vector<bool> done(ncols, false);
    for (size_t g0 = 0; g0 < packed.size() && rc == PLGPU_OK; g0 += kAosMax) {
        const int nc = (int)std::min<size_t>(kAosMax, packed.size() - g0);
        if (nc < 4) break;  // leftover columns go the per-column way
        const int64_t rows = cols[packed[g0]].length;
        AosCols c;
        std::memset(&c, 0, sizeof c);
        for (int k = 0; k < nc; ++k) {
            const plgpu_column& src = cols[packed[g0 + k]];
            rc = make_owned_column(&out_cols[packed[g0 + k]], src.dtype, n, false, s);
            if (rc) break;
            c.src[k] = (const uint64_t*)src.values + src.offset;
            c.dst[k] = (uint64_t*)out_cols[packed[g0 + k]].values;
            done[packed[g0 + k]] = true;
        }
        uint64_t* aos = nullptr;
        if (!rc) rc = dev_alloc((void**)&aos, (size_t)rows * ((nc + 1) & ~1) * 8, s);
        if (!rc) {
            hipError_t e = aos_dispatch(nc, c, rows, ix, n, aos, s);
            if (e != hipSuccess) rc = hip_fail(e, "packed gather");
        }
        dev_free(aos, s);
    }
    for (int i = 0; i < ncols && rc == PLGPU_OK; ++i)
        if (!done[i]) rc = gather_into(cols[i], ix, n, &out_cols[i], s, idx->validity, idx->offset);
    if (rc == PLGPU_OK) {
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "gather");
    }
    if (rc)
        for (int i = 0; i < ncols; ++i) plgpu_column_release(&out_cols[i]);
    return rc;
}

// out[i] = a[i] when valid, else b[i] (null when both are null).  Bool
// columns are written one ballot word per 64 rows.
__global__ __launch_bounds__(256) void coalesce_kernel(DevCol a, DevCol b, int64_t n, void* __restrict__ out,
                                                       uint64_t* __restrict__ out_valid) {
    for (int64_t r0 = (int64_t)blockIdx.x * blockDim.x; r0 < n; r0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = r0 + threadIdx.x;
        const bool in = r < n;
        const bool va = in && dev_valid(a, r);
        const bool vb = in && !va && dev_valid(b, r);
        const uint64_t v = va ? dev_load(a, r) : (vb ? dev_load(b, r) : 0ull);
        if (a.dtype == PLGPU_BOOL) {
            const uint64_t w = __ballot(in && (v & 1));
            if ((threadIdx.x & 63) == 0 && in) ((uint64_t*)out)[r >> 6] = w;
        } else if (in) {
            dev_store(out, a.dtype, r, v);
        }
        const uint64_t vw = __ballot(va || vb);
        if ((threadIdx.x & 63) == 0 && in) out_valid[r >> 6] = vw;
    }
}

PLGPU_API int plgpu_coalesce(const plgpu_column* a, const plgpu_column* b, plgpu_column* out, void* stream) {
    hipStream_t s = as_stream(stream);
    if (a == nullptr || b == nullptr || out == nullptr) return fail(PLGPU_ERR_INVALID, "NULL argument");
    std::memset(out, 0, sizeof *out);
    if (a->dtype != b->dtype) return fail(PLGPU_ERR_SCHEMA, "coalesce of columns with different dtypes");
    if (a->length != b->length) return fail(PLGPU_ERR_SHAPE, "coalesce of columns with different lengths");
    if (a->dtype != PLGPU_BOOL && dtype_bytes(a->dtype) == 0) return fail(PLGPU_ERR_SCHEMA, "unsupported dtype");
    const int64_t n = a->length;
    int rc = make_owned_column(out, a->dtype, n, true, s);
    if (rc) return rc;
    if (n > 0) {
        const int g = (int)std::min<int64_t>((n + 255) / 256, (int64_t)num_cus_jn() * 16);
        coalesce_kernel<<<g, 256, 0, s>>>(as_dev(a), as_dev(b), n, (void*)out->values, (uint64_t*)out->validity);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            plgpu_column_release(out);
            return hip_fail(e, "coalesce");
        }
    }
    return PLGPU_OK;
}

// plgpu_join_inner_take over 1..8 key columns: integer / Boolean keys whose
// ranges pack into one exact Int64 (mk_plan_pack) run the single-key take on
// the packed keys (a tuple holding a null is a null key unless nulls_equal),
// so the row-format table applies to multi-key joins too; other keys compute
// the pairs (plgpu_join_multi: hashed, verified) and gather.
PLGPU_API int plgpu_join_inner_take_multi(const plgpu_column* left_keys, const plgpu_column* right_keys,
                                          int32_t nkeys, const plgpu_column* left_cols, int32_t nleft,
                                          const plgpu_column* right_cols, int32_t nright, int32_t nulls_equal,
                                          int32_t maintain_order, int32_t validate, plgpu_column* out_left,
                                          plgpu_column* out_right, int64_t* out_len, void* stream) {
    hipStream_t s = as_stream(stream);
    if (left_keys == nullptr || right_keys == nullptr || out_len == nullptr ||
        (nleft > 0 && (left_cols == nullptr || out_left == nullptr)) ||
        (nright > 0 && (right_cols == nullptr || out_right == nullptr)))
        return fail(PLGPU_ERR_INVALID, "NULL argument");
    if (nkeys < 1 || nkeys > kMaxKeys) return fail(PLGPU_ERR_INVALID, "number of join keys must be 1..8");
    if (nleft < 0 || nleft > PLGPU_MAX_COLS || nright < 0 || nright > PLGPU_MAX_COLS)
        return fail(PLGPU_ERR_INVALID, "0..8 columns per side");
    const int64_t nl = left_keys[0].length, nr = right_keys[0].length;
    bool packable = true;
    MkKeys ka, kb;
    std::memset(&ka, 0, sizeof ka);
    std::memset(&kb, 0, sizeof kb);
    ka.n = kb.n = nkeys;
    for (int i = 0; i < nkeys; ++i) {
        const int32_t dt = left_keys[i].dtype;
        if (right_keys[i].dtype != dt) return fail(PLGPU_ERR_SCHEMA, "datatypes of join keys don't match");
        if (left_keys[i].length != nl || right_keys[i].length != nr)
            return fail(PLGPU_ERR_SHAPE, "join key columns of one side must have equal lengths");
        if (!dtype_is_int(dt) && dt != PLGPU_BOOL) packable = false;
        ka.c[i] = as_dev(&left_keys[i]);
        kb.c[i] = as_dev(&right_keys[i]);
    }
    const bool neq = nulls_equal != 0;
    const int cus = num_cus_jn();
    MkPack pk;
    pk.ok = false;
    if (packable && nl < 0xFFFFFFFFll && nr < 0xFFFFFFFFll) {
        const int rc = mk_plan_pack(ka, nl, &kb, nr, cus * 16, &pk, s);
        if (rc) return rc;
    }
    if (pk.ok) {
        uint64_t *cl = nullptr, *cr = nullptr;
        int rc = dev_alloc((void**)&cl, (std::max<int64_t>(nl, 1) + (nl + 63) / 64 + 1) * 8, s);
        if (!rc) rc = dev_alloc((void**)&cr, (std::max<int64_t>(nr, 1) + (nr + 63) / 64 + 1) * 8, s);
        uint64_t* vl = cl ? cl + std::max<int64_t>(nl, 1) : nullptr;
        uint64_t* vr = cr ? cr + std::max<int64_t>(nr, 1) : nullptr;
        if (!rc)
            mk_pack_launch(ka, pk, nl, cl, neq ? nullptr : vl, nullptr,
                           (int)std::min<int64_t>((nl + 255) / 256, cus * 16), s);
        if (!rc)
            mk_pack_launch(kb, pk, nr, cr, neq ? nullptr : vr, nullptr,
                           (int)std::min<int64_t>((nr + 255) / 256, cus * 16), s);
        if (!rc) {
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) rc = hip_fail(e, "mk_pack_kernel");
        }
        if (!rc) {
            plgpu_column a, b;
            std::memset(&a, 0, sizeof a);
            std::memset(&b, 0, sizeof b);
            a.dtype = b.dtype = PLGPU_I64;
            a.length = nl;
            b.length = nr;
            a.values = cl;
            b.values = cr;
            a.validity = neq ? nullptr : (const uint8_t*)vl;
            b.validity = neq ? nullptr : (const uint8_t*)vr;
            a.null_count = b.null_count = neq ? 0 : -1;
            rc = plgpu_join_inner_take(&a, &b, left_cols, nleft, right_cols, nright, nulls_equal, maintain_order,
                                       validate, out_left, out_right, out_len, stream);
        }
        (void)hipStreamSynchronize(s);
        dev_free(cl, s);
        dev_free(cr, s);
        return rc;
    }
    // pairs (hashed and verified), then the takes
    for (int i = 0; i < nleft; ++i) std::memset(&out_left[i], 0, sizeof out_left[i]);
    for (int i = 0; i < nright; ++i) std::memset(&out_right[i], 0, sizeof out_right[i]);
    *out_len = 0;
    plgpu_column li, ri;
    int rc = plgpu_join_multi(left_keys, right_keys, nkeys, PLGPU_JOIN_INNER, nulls_equal, maintain_order, validate,
                              &li, &ri, stream);
    if (rc) return rc;
    for (int i = 0; i < nleft && !rc; ++i)
        rc = gather_into(left_cols[i], (const uint32_t*)li.values, li.length, &out_left[i], s);
    for (int i = 0; i < nright && !rc; ++i)
        rc = gather_into(right_cols[i], (const uint32_t*)ri.values, ri.length, &out_right[i], s);
    if (!rc) {
        const hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) rc = hip_fail(e, "join take");
    }
    *out_len = li.length;
    plgpu_column_release(&li);
    plgpu_column_release(&ri);
    if (rc) {
        for (int i = 0; i < nleft; ++i) plgpu_column_release(&out_left[i]);
        for (int i = 0; i < nright; ++i) plgpu_column_release(&out_right[i]);
    }
    return rc;
}
