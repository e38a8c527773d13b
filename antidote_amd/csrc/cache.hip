// cache.hip — the materializer_vnode snapshot cache as a device table
// (include/antidote_gpu.h agn_ss_cache): batched get_from_snapshot_cache
// (src/materializer_vnode.erl:384-413 + vector_orddict:get_smaller,
// src/vector_orddict.erl:74-87) and the cache half of materialize_snapshot /
// internal_store_ss / snapshot_insert_gc (:341-364, 466-563).
//
// One wave per request, lanes over DCs: every vector-clock predicate (le of
// a cached clock against R or LastOpCt) is one ballot, the vectorclock:min of
// the kept snapshots is a per-lane min, and moving an entry is a
// lane-parallel row copy.  The per-request control flow (cache policy) is
// wave-uniform scalar code.  HBM bytes per request: lookup reads up to
// `n` cached clocks (8D each, stops at the first <= R) + R, writes the SCT
// row; store reads the materialize result row + the head clock and rewrites
// at most SNAPSHOT_MIN + 1 rows.
#include "common.hpp"

namespace agn {
namespace {

__device__ __forceinline__ bool mbit(const uint64_t *m, uint64_t row, uint32_t W, uint32_t d) {
    return m == nullptr || ((m[row * W + (d >> 6)] >> (d & 63)) & 1ull);
}

// vectorclock:le(A, B) with A = cached row `ra` (mask am), B = row `rb` of
// (b, bm); missing entries read 0.  Wave-uniform result.
__device__ __forceinline__ bool wave_le(const uint64_t *a, const uint64_t *am, uint64_t ra,
                                        const uint64_t *b, const uint64_t *bm, uint64_t rb,
                                        uint32_t D, uint32_t W) {
    bool bad = false;
    for (uint32_t d = lane_id(); d < D; d += AGN_WAVE) {
        if (!mbit(am, ra, W, d)) continue;
        const uint64_t bv = mbit(bm, rb, W, d) ? b[rb * D + d] : 0ull;
        bad = bad || a[ra * D + d] > bv;
    }
    return ballot(bad) == 0ull;
}

__device__ __forceinline__ void copy_row(uint64_t *dst, uint64_t rd, const uint64_t *src,
                                         uint64_t rs, uint32_t n) {
    for (uint32_t d = lane_id(); d < n; d += AGN_WAVE) dst[rd * n + d] = src[rs * n + d];
}

__global__ __launch_bounds__(256) void k_ss_lookup(agn_ss_cache c, uint64_t n_req,
                                                   const uint64_t *__restrict__ keys,
                                                   const uint64_t *__restrict__ R,
                                                   const uint64_t *__restrict__ Rm,
                                                   uint64_t *__restrict__ sct,
                                                   uint64_t *__restrict__ sctm,
                                                   uint8_t *__restrict__ sct_ign,
                                                   int64_t *__restrict__ base,
                                                   uint8_t *__restrict__ first,
                                                   uint8_t *__restrict__ status) {
    const uint64_t i = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    if (i >= n_req) return;
    const int lane = lane_id();
    const uint32_t D = c.n_dcs, W = n_words(D), S = c.slots;
    const uint64_t k = keys ? uniform_u64(keys[i]) : i;
    const uint32_t n = __builtin_amdgcn_readfirstlane(c.n[k]);
    if (n == 0) {
        // store_snapshot(.., EmptySnapshot, vectorclock:new(), ..) (:398-402)
        for (uint32_t d = lane; d < D; d += AGN_WAVE) {
            c.clock[(k * S) * D + d] = 0ull;
            sct[i * D + d] = 0ull;
        }
        for (uint32_t x = lane; x < W; x += AGN_WAVE) {
            if (c.clock_mask) c.clock_mask[(k * S) * W + x] = 0ull;
            if (sctm) sctm[i * W + x] = 0ull;
        }
        if (lane == 0) {
            c.last_op[k * S] = 0;
            c.value[k * S] = 0;
            c.n[k] = 1;
            sct_ign[i] = 1;  // base {ignore, Type:new()} (:395-396)
            base[i] = 0;
            first[i] = 1;
            status[i] = AGN_SS_NEW;
        }
        return;
    }
    int found = -1;
    for (uint32_t j = 0; j < n; ++j) {
        if (wave_le(c.clock, c.clock_mask, k * S + j, R, Rm, i, D, W)) {
            found = (int)j;
            break;
        }
    }
    if (found >= 0) {
        const uint64_t row = k * S + (uint64_t)found;
        copy_row(sct, i, c.clock, row, D);
        if (sctm) {
            if (c.clock_mask) copy_row(sctm, i, c.clock_mask, row, W);
            else for (uint32_t x = lane; x < W; x += AGN_WAVE)
                     sctm[i * W + x] = (x + 1 < W || D % 64 == 0) ? ~0ull : ((1ull << (D % 64)) - 1ull);
        }
    }
    if (lane == 0) {
        sct_ign[i] = found >= 0 ? 0 : 1;
        base[i] = found >= 0 ? c.value[k * S + (uint64_t)found] : 0;
        first[i] = found == 0 ? 1 : 0;
        status[i] = found >= 0 ? AGN_SS_HIT : AGN_SS_LOG;
    }
}

__global__ __launch_bounds__(256) void k_ss_store(agn_ss_cache c, const uint64_t *__restrict__ key_off,
                                                  uint64_t n_req, const uint64_t *__restrict__ keys,
                                                  const uint8_t *__restrict__ is_first,
                                                  const uint8_t *__restrict__ status,
                                                  const uint8_t *__restrict__ should_gc,
                                                  agn_result res, const int64_t *__restrict__ handle,
                                                  uint8_t *__restrict__ prune,
                                                  uint64_t *__restrict__ thr,
                                                  uint64_t *__restrict__ thrm) {
    const uint64_t i = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    if (i >= n_req) return;
    const int lane = lane_id();
    const uint32_t D = c.n_dcs, W = n_words(D), S = c.slots;
    const uint64_t k = keys ? uniform_u64(keys[i]) : i;
    if (status[i] == AGN_SS_LOG) return;
    if (key_off[k + 1] == key_off[k]) return;  // number_of_ops = 0 (:468-471)
    const uint32_t fl = res.flags[i];
    if (fl & (AGN_F_ERR_UNEXPECTED | AGN_F_ERR_CORRUPTED | AGN_F_ERR_CAPACITY)) return;
    if (fl & AGN_F_CT_IGNORE) return;  // CommitTime == ignore (:483-484)
    const bool gc = should_gc != nullptr && should_gc[i] != 0;
    const bool refresh = (fl & AGN_F_NEWSS) && is_first[i] && res.count[i] >= AGN_MIN_OP_STORE_SS;
    if (!(refresh || gc)) return;
    const uint32_t n = __builtin_amdgcn_readfirstlane(c.n[k]);
    const int64_t new_op = res.hole[i];
    const int64_t val = handle ? handle[i] : res.value[i];
    // internal_store_ss (:341-364)
    const bool should_insert = n == 0 || new_op - c.last_op[k * S] >= AGN_MIN_OP_STORE_SS;
    if (!(should_insert || gc)) return;
    // insert_bigger: prepend iff not le(LastOpCt, head clock)
    const bool prepend =
        n == 0 || !wave_le(res.lastct, res.lastct_mask, i, c.clock, c.clock_mask, k * S, D, W);
    const uint32_t size1 = n + (prepend ? 1u : 0u);
    const bool collect = size1 >= AGN_SNAPSHOT_THRESHOLD || gc;
    // entries kept from the old list, and the new list size
    uint32_t old_kept = n;
    if (collect) old_kept = prepend ? (n < AGN_SNAPSHOT_MIN - 1 ? n : AGN_SNAPSHOT_MIN - 1)
                                    : (n < AGN_SNAPSHOT_MIN ? n : AGN_SNAPSHOT_MIN);
    const uint32_t new_n = old_kept + (prepend ? 1u : 0u);
    if (prepend) {
        for (int j = (int)old_kept - 1; j >= 0; --j) {  // shift down, newest first
            copy_row(c.clock, k * S + j + 1, c.clock, k * S + j, D);
            if (c.clock_mask) copy_row(c.clock_mask, k * S + j + 1, c.clock_mask, k * S + j, W);
            if (lane == 0) {
                c.last_op[k * S + j + 1] = c.last_op[k * S + j];
                c.value[k * S + j + 1] = c.value[k * S + j];
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        copy_row(c.clock, k * S, res.lastct, i, D);
        if (c.clock_mask) {
            if (res.lastct_mask) copy_row(c.clock_mask, k * S, res.lastct_mask, i, W);
            else for (uint32_t x = lane; x < W; x += AGN_WAVE)
                     c.clock_mask[(k * S) * W + x] =
                         (x + 1 < W || D % 64 == 0) ? ~0ull : ((1ull << (D % 64)) - 1ull);
        }
        if (lane == 0) {
            c.last_op[k * S] = new_op;
            c.value[k * S] = val;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    if (collect) {
        // CommitTime = vectorclock:min of the kept clocks (:523-527), missing = 0
        for (uint32_t d = lane; d < D; d += AGN_WAVE) {
            uint64_t m = ~0ull;
            bool any = false;
            for (uint32_t j = 0; j < new_n; ++j) {
                const bool p = mbit(c.clock_mask, k * S + j, W, d);
                const uint64_t v = p ? c.clock[(k * S + j) * D + d] : 0ull;
                any = any || p;
                m = v < m ? v : m;
            }
            thr[k * D + d] = any ? m : 0ull;
        }
        if (thrm) {
            for (uint32_t x = lane; x < W; x += AGN_WAVE) {
                uint64_t u = 0;
                for (uint32_t j = 0; j < new_n; ++j)
                    u |= c.clock_mask ? c.clock_mask[(k * S + j) * W + x]
                                      : ((x + 1 < W || D % 64 == 0) ? ~0ull
                                                                    : ((1ull << (D % 64)) - 1ull));
                thrm[k * W + x] = u;
            }
        }
        if (lane == 0) prune[k] = 1;
    }
    if (lane == 0) c.n[k] = new_n;
}

}  // namespace

int launch_ss_lookup(const agn_ss_cache &c, uint64_t n_req, const uint64_t *keys,
                     const uint64_t *R, const uint64_t *Rm, uint64_t *sct, uint64_t *sctm,
                     uint8_t *sct_ign, int64_t *base, uint8_t *first, uint8_t *status,
                     hipStream_t st) {
    if (n_req == 0) return AGN_OK;
    hipLaunchKernelGGL(k_ss_lookup, dim3(grid_for(n_req, 4, 0x7fffffffu)), dim3(256), 0, st, c,
                       n_req, keys, R, Rm, sct, sctm, sct_ign, base, first, status);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

int launch_ss_store(const agn_ss_cache &c, const uint64_t *key_off, uint64_t n_req,
                    const uint64_t *keys, const uint8_t *is_first, const uint8_t *status,
                    const uint8_t *should_gc, const agn_result &res, const int64_t *handle,
                    uint8_t *prune, uint64_t *thr, uint64_t *thrm, hipStream_t st) {
    AGN_HIP(hipMemsetAsync(prune, 0, c.n_keys, st));
    if (n_req == 0) return AGN_OK;
    hipLaunchKernelGGL(k_ss_store, dim3(grid_for(n_req, 4, 0x7fffffffu)), dim3(256), 0, st, c,
                       key_off, n_req, keys, is_first, status, should_gc, res, handle, prune, thr,
                       thrm);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

}  // namespace agn
