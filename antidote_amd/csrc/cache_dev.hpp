// cache_dev.hpp -- the snapshot cache's per-request device logic
// (get_from_snapshot_cache and the cache half of materialize_snapshot), on a
// group of G lanes per request; used by the batched kernels (cache.hip) and
// the fused cached read (read6.hip).
#pragma once
#include "common.hpp"

namespace agn {
namespace {

__device__ __forceinline__ bool mbit(const uint64_t *m, uint64_t row, uint32_t W, uint32_t d) {
    return m == nullptr || ((m[row * W + (d >> 6)] >> (d & 63)) & 1ull);
}

__device__ __forceinline__ uint64_t full_word(uint32_t x, uint32_t W, uint32_t D) {
    return (x + 1 < W || D % 64 == 0) ? ~0ull : ((1ull << (D % 64)) - 1ull);
}

template <int G>
struct Grp {
    uint32_t sub;    // lane within the request's group = first DC it handles
    uint64_t gmask;  // the group's lanes in a ballot
    __device__ Grp() {
        const uint32_t lane = (uint32_t)lane_id();
        sub = lane % G;
        gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << (lane - sub);
    }
    __device__ bool all(bool p) const { return (ballot(!p) & gmask) == 0ull; }
};

// vectorclock:le(A, B): A = row ra of (a, am), B = row rb of (b, bm);
// missing entries read 0.  Group-uniform result.
template <int G>
__device__ __forceinline__ bool grp_le(const Grp<G> &g, const uint64_t *a, const uint64_t *am,
                                       uint64_t ra, const uint64_t *b, const uint64_t *bm,
                                       uint64_t rb, uint32_t D, uint32_t W) {
    bool ok = true;
    for (uint32_t d = g.sub; d < D; d += G) {
        if (!mbit(am, ra, W, d)) continue;
        const uint64_t bv = mbit(bm, rb, W, d) ? b[rb * D + d] : 0ull;
        ok = ok && a[ra * D + d] <= bv;
    }
    return g.all(ok);
}

template <int G>
__device__ __forceinline__ void copy_row(const Grp<G> &g, uint64_t *dst, uint64_t rd,
                                         const uint64_t *src, uint64_t rs, uint32_t n) {
    for (uint32_t d = g.sub; d < n; d += G) dst[rd * n + d] = src[rs * n + d];
}

// get_from_snapshot_cache (:384-413) for one request on its group: the
// first cached clock of key k (newest first) <= R (vector_orddict:get_smaller,
// src/vector_orddict.erl:74-87) gives the base; an absent key stores the
// empty snapshot at vectorclock:new() (:398-402).  R_row / Rm_row and
// sct_row / sctm_row are the request's rows (masks may be NULL).  Returns,
// group-uniform: out.ign (SCT = ignore), base, first (IsFirst), status.
struct LookupOut {
    uint8_t ign, first, status;
    int64_t base;
};
template <int G>
__device__ __forceinline__ LookupOut ss_lookup_one(const Grp<G> &g, const agn_ss_cache &c,
                                                   uint64_t k, const uint64_t *R_row,
                                                   const uint64_t *Rm_row, uint64_t *sct_row,
                                                   uint64_t *sctm_row) {
    const uint32_t D = c.n_dcs, W = n_words(D), S = c.slots;
    // Dense rows with D <= G: slot 0 (always in bounds), its value and R are
    // loaded with the entry count, so a hit on the newest snapshot -- the
    // common warm read -- costs no round trip after it.
    const bool dense1 = D <= (uint32_t)G && c.clock_mask == nullptr && Rm_row == nullptr;
    const uint32_t dd = g.sub < D ? g.sub : D - 1u;
    const uint64_t c0 = c.clock[(k * S) * D + dd];
    const uint64_t r0 = R_row[dd];
    const int64_t v0 = c.value[k * S];
    const uint32_t n = c.n[k];
    if (n == 0) {
        for (uint32_t d = g.sub; d < D; d += G) {
            c.clock[(k * S) * D + d] = 0ull;
            sct_row[d] = 0ull;
        }
        for (uint32_t x = g.sub; x < W; x += G) {
            if (c.clock_mask) c.clock_mask[(k * S) * W + x] = 0ull;
            if (sctm_row) sctm_row[x] = 0ull;
        }
        if (g.sub == 0) {
            c.last_op[k * S] = 0;
            c.value[k * S] = 0;
            c.n[k] = 1;
        }
        return LookupOut{1, 1, AGN_SS_NEW, 0};  // base {ignore, Type:new()} (:395-396)
    }
    int found = -1;
    uint32_t j0 = 0;
    if (dense1) {
        if (g.all(g.sub >= D || c0 <= r0)) found = 0;
        else j0 = 1;
    }
    for (uint32_t j = j0; found < 0 && j < n; ++j) {
        if (grp_le<G>(g, c.clock, c.clock_mask, k * S + j, R_row, Rm_row, 0, D, W)) {
            found = (int)j;
            break;
        }
    }
    if (found >= 0) {
        const uint64_t row = k * S + (uint64_t)found;
        if (dense1 && found == 0) {
            if (g.sub < D) sct_row[g.sub] = c0;
        } else {
            copy_row<G>(g, sct_row, 0, c.clock, row, D);
        }
        if (sctm_row) {
            if (c.clock_mask) copy_row<G>(g, sctm_row, 0, c.clock_mask, row, W);
            else for (uint32_t x = g.sub; x < W; x += G) sctm_row[x] = full_word(x, W, D);
        }
    }
    return LookupOut{(uint8_t)(found >= 0 ? 0 : 1), (uint8_t)(found == 0 ? 1 : 0),
                     (uint8_t)(found >= 0 ? AGN_SS_HIT : AGN_SS_LOG),
                     found == 0 && dense1 ? v0
                     : found >= 0         ? c.value[k * S + (uint64_t)found]
                                          : 0};
}

// 64-bit value of the group's first lane
template <int G>
__device__ __forceinline__ uint64_t grp_bcast(const Grp<G> &g, uint64_t v) {
    const int src = lane_id() - (int)g.sub;
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, AGN_WAVE);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, AGN_WAVE);
    return ((uint64_t)hi << 32) | lo;
}

// The cache half of materialize_snapshot for one request on its group
// (internal_store_ss / insert_bigger / snapshot_insert_gc, :341-364, 466-563):
// nops = the key's op count, the materialize result (LastOpCt row + mask row
// or NULL, NewLastOp `hole`, value, count, flags), status / is_first from
// the lookup, gc = a GC read (op_insert_gc, :640).  Writes the GC threshold
// of key k (vectorclock:min of the kept clocks, :523-527) and returns whether
// its ops are to be pruned.  Group-uniform.  A set_aw / register_mv cache
// with a state arena (c.state_tag) stores the result's state (st_tag /
// st_tok, st_n pairs) there and records the pairs of the snapshots it drops;
// dl (optional, the group's first lane): the pairs added to state_ctl[0] and
// [1], and whether the store overflowed the arena.
template <int G>
__device__ __forceinline__ bool ss_store_one(const Grp<G> &g, const agn_ss_cache &c, uint64_t k,
                                             uint64_t nops, uint8_t status, uint8_t is_first,
                                             bool gc, const uint64_t *lastct_row,
                                             const uint64_t *lastct_mask_row, int64_t new_op,
                                             int64_t val, uint32_t count, uint32_t fl,
                                             uint64_t *thr, uint64_t *thrm,
                                             const uint32_t *st_tag = nullptr,
                                             const uint64_t *st_tok = nullptr,
                                             uint32_t st_n = 0, uint64_t *dl = nullptr) {
    const uint32_t D = c.n_dcs, W = n_words(D), S = c.slots;
    if (status == AGN_SS_LOG) return false;
    if (nops == 0) return false;  // number_of_ops = 0 (:468-471)
    if (fl & (AGN_F_ERR_UNEXPECTED | AGN_F_ERR_CORRUPTED | AGN_F_ERR_CAPACITY)) return false;
    if (fl & AGN_F_CT_IGNORE) return false;  // CommitTime == ignore (:483-484)
    const bool refresh = (fl & AGN_F_NEWSS) && is_first && count >= AGN_MIN_OP_STORE_SS;
    if (!(refresh || gc)) return false;
    const uint32_t n = c.n[k];
    // internal_store_ss (:341-364)
    const bool should_insert = n == 0 || new_op - c.last_op[k * S] >= AGN_MIN_OP_STORE_SS;
    if (!(should_insert || gc)) return false;
    // insert_bigger: prepend iff not le(LastOpCt, head clock)
    const bool prepend =
        n == 0 || !grp_le<G>(g, lastct_row, lastct_mask_row, 0, c.clock, c.clock_mask, k * S, D, W);
    const uint32_t size1 = n + (prepend ? 1u : 0u);
    const bool collect = size1 >= AGN_SNAPSHOT_THRESHOLD || gc;
    // entries kept from the old list, and the new list size
    uint32_t old_kept = n;
    if (collect) old_kept = prepend ? (n < AGN_SNAPSHOT_MIN - 1 ? n : AGN_SNAPSHOT_MIN - 1)
                                    : (n < AGN_SNAPSHOT_MIN ? n : AGN_SNAPSHOT_MIN);
    const uint32_t new_n = old_kept + (prepend ? 1u : 0u);
    if (c.state_tag) {
        // the new snapshot's state: appended to the arena (before any change,
        // so a store that does not fit changes nothing); the dropped
        // snapshots' pairs are released
        if (prepend) {
            uint64_t start = 0;
            if (g.sub == 0)
                start = atomicAdd((unsigned long long *)&c.state_ctl[0], (unsigned long long)st_n);
            start = grp_bcast<G>(g, start);
            if (dl) dl[0] = st_n;
            if (start + st_n > c.state_cap || st_n > AGN_SS_STATE_MAX_PAIRS) {
                if (g.sub == 0) {
                    c.state_ctl[2] = 1ull;
                    atomicAdd((unsigned long long *)&c.state_ctl[1], (unsigned long long)st_n);
                }
                if (dl) {
                    dl[1] = st_n;
                    dl[2] = 1;
                }
                return false;
            }
            for (uint32_t x = g.sub; x < st_n; x += G) {
                c.state_tag[start + x] = st_tag[x];
                c.state_tok[start + x] = st_tok[x];
            }
            val = AGN_SS_STATE(start, st_n);
        }
        if (g.sub == 0 && old_kept < n) {
            uint64_t rel = 0;
            for (uint32_t j = old_kept; j < n; ++j) rel += AGN_SS_STATE_PAIRS(c.value[k * S + j]);
            if (rel) atomicAdd((unsigned long long *)&c.state_ctl[1], (unsigned long long)rel);
            if (dl) dl[1] = rel;
        }
    }
    if (prepend) {
        for (int j = (int)old_kept - 1; j >= 0; --j) {  // shift down, newest first
            copy_row<G>(g, c.clock, k * S + j + 1, c.clock, k * S + j, D);
            if (c.clock_mask) copy_row<G>(g, c.clock_mask, k * S + j + 1, c.clock_mask, k * S + j, W);
            if (g.sub == 0) {
                c.last_op[k * S + j + 1] = c.last_op[k * S + j];
                c.value[k * S + j + 1] = c.value[k * S + j];
            }
        }
        copy_row<G>(g, c.clock, k * S, lastct_row, 0, D);
        if (c.clock_mask) {
            if (lastct_mask_row) copy_row<G>(g, c.clock_mask, k * S, lastct_mask_row, 0, W);
            else for (uint32_t x = g.sub; x < W; x += G)
                     c.clock_mask[(k * S) * W + x] = full_word(x, W, D);
        }
        if (g.sub == 0) {
            c.last_op[k * S] = new_op;
            c.value[k * S] = val;
        }
    }
    if (collect) {
        // CommitTime = vectorclock:min of the kept clocks (:523-527), missing = 0
        for (uint32_t d = g.sub; d < D; d += G) {
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
            for (uint32_t x = g.sub; x < W; x += G) {
                uint64_t u = 0;
                for (uint32_t j = 0; j < new_n; ++j)
                    u |= c.clock_mask ? c.clock_mask[(k * S + j) * W + x] : full_word(x, W, D);
                thrm[k * W + x] = u;
            }
        }
    }
    if (g.sub == 0) c.n[k] = new_n;
    return collect;
}

// group width: the power of two >= D, capped at a wave
inline int group_of(uint32_t D) {
    int g = 1;
    while (g < (int)D && g < AGN_WAVE) g <<= 1;
    return g;
}

}  // namespace
}  // namespace agn
