// cache.hip — the materializer_vnode snapshot cache as a device table
// (include/antidote_gpu.h agn_ss_cache): batched get_from_snapshot_cache
// (src/materializer_vnode.erl:384-413 + vector_orddict:get_smaller,
// src/vector_orddict.erl:74-87) and the cache half of materialize_snapshot /
// internal_store_ss / snapshot_insert_gc (:341-364, 466-563).
//
// A group of G lanes per request (G = the power of two >= D, capped at 64;
// 64 / G requests per wave), lanes over DCs: every vector-clock predicate (le
// of a cached clock against R or LastOpCt) is one ballot masked to the group,
// the vectorclock:min of the kept snapshots is a per-lane min, and moving an
// entry is a lane-parallel row copy.  The per-request control flow (cache
// policy) is group-uniform.  HBM bytes per request: lookup reads up to `n`
// cached clocks (8D each, stops at the first <= R) + R and writes the SCT
// row; store reads the materialize result row + the head clock and rewrites
// at most SNAPSHOT_MIN + 1 rows.
#include "serve.hpp"

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

template <int G>
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
    const Grp<G> g;
    const uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    if (i >= n_req) return;
    const uint32_t D = c.n_dcs, W = n_words(D), S = c.slots;
    const uint64_t k = keys ? keys[i] : i;
    const uint32_t n = c.n[k];
    if (n == 0) {
        // store_snapshot(.., EmptySnapshot, vectorclock:new(), ..) (:398-402)
        for (uint32_t d = g.sub; d < D; d += G) {
            c.clock[(k * S) * D + d] = 0ull;
            sct[i * D + d] = 0ull;
        }
        for (uint32_t x = g.sub; x < W; x += G) {
            if (c.clock_mask) c.clock_mask[(k * S) * W + x] = 0ull;
            if (sctm) sctm[i * W + x] = 0ull;
        }
        if (g.sub == 0) {
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
        if (grp_le<G>(g, c.clock, c.clock_mask, k * S + j, R, Rm, i, D, W)) {
            found = (int)j;
            break;
        }
    }
    if (found >= 0) {
        const uint64_t row = k * S + (uint64_t)found;
        copy_row<G>(g, sct, i, c.clock, row, D);
        if (sctm) {
            if (c.clock_mask) copy_row<G>(g, sctm, i, c.clock_mask, row, W);
            else for (uint32_t x = g.sub; x < W; x += G) sctm[i * W + x] = full_word(x, W, D);
        }
    }
    if (g.sub == 0) {
        sct_ign[i] = found >= 0 ? 0 : 1;
        base[i] = found >= 0 ? c.value[k * S + (uint64_t)found] : 0;
        first[i] = found == 0 ? 1 : 0;
        status[i] = found >= 0 ? AGN_SS_HIT : AGN_SS_LOG;
    }
}

template <int G>
__global__ __launch_bounds__(256) void k_ss_store(agn_ss_cache c, const uint64_t *__restrict__ key_off,
                                                  const uint64_t *__restrict__ key_len,
                                                  uint64_t n_req, const uint64_t *__restrict__ keys,
                                                  const uint8_t *__restrict__ is_first,
                                                  const uint8_t *__restrict__ status,
                                                  const uint8_t *__restrict__ should_gc,
                                                  agn_result res, const int64_t *__restrict__ handle,
                                                  uint8_t *__restrict__ prune,
                                                  uint64_t *__restrict__ thr,
                                                  uint64_t *__restrict__ thrm, int by_req) {
    const Grp<G> g;
    const uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    if (i >= n_req) return;
    const uint32_t D = c.n_dcs, W = n_words(D), S = c.slots;
    const uint64_t k = keys ? keys[i] : i;
    // by_req: prune flags per request (prune[i], every request written),
    // otherwise per key (prune[k], the caller cleared the array)
    if (by_req && g.sub == 0) prune[i] = 0;
    if (status[i] == AGN_SS_LOG) return;
    if (key_n(key_off, key_len, k) == 0) return;  // number_of_ops = 0 (:468-471)
    const uint32_t fl = res.flags[i];
    if (fl & (AGN_F_ERR_UNEXPECTED | AGN_F_ERR_CORRUPTED | AGN_F_ERR_CAPACITY)) return;
    if (fl & AGN_F_CT_IGNORE) return;  // CommitTime == ignore (:483-484)
    const bool gc = should_gc != nullptr && should_gc[i] != 0;
    const bool refresh = (fl & AGN_F_NEWSS) && is_first[i] && res.count[i] >= AGN_MIN_OP_STORE_SS;
    if (!(refresh || gc)) return;
    const uint32_t n = c.n[k];
    const int64_t new_op = res.hole[i];
    const int64_t val = handle ? handle[i] : res.value[i];
    // internal_store_ss (:341-364)
    const bool should_insert = n == 0 || new_op - c.last_op[k * S] >= AGN_MIN_OP_STORE_SS;
    if (!(should_insert || gc)) return;
    // insert_bigger: prepend iff not le(LastOpCt, head clock)
    const bool prepend =
        n == 0 || !grp_le<G>(g, res.lastct, res.lastct_mask, i, c.clock, c.clock_mask, k * S, D, W);
    const uint32_t size1 = n + (prepend ? 1u : 0u);
    const bool collect = size1 >= AGN_SNAPSHOT_THRESHOLD || gc;
    // entries kept from the old list, and the new list size
    uint32_t old_kept = n;
    if (collect) old_kept = prepend ? (n < AGN_SNAPSHOT_MIN - 1 ? n : AGN_SNAPSHOT_MIN - 1)
                                    : (n < AGN_SNAPSHOT_MIN ? n : AGN_SNAPSHOT_MIN);
    const uint32_t new_n = old_kept + (prepend ? 1u : 0u);
    if (prepend) {
        for (int j = (int)old_kept - 1; j >= 0; --j) {  // shift down, newest first
            copy_row<G>(g, c.clock, k * S + j + 1, c.clock, k * S + j, D);
            if (c.clock_mask) copy_row<G>(g, c.clock_mask, k * S + j + 1, c.clock_mask, k * S + j, W);
            if (g.sub == 0) {
                c.last_op[k * S + j + 1] = c.last_op[k * S + j];
                c.value[k * S + j + 1] = c.value[k * S + j];
            }
        }
        copy_row<G>(g, c.clock, k * S, res.lastct, i, D);
        if (c.clock_mask) {
            if (res.lastct_mask) copy_row<G>(g, c.clock_mask, k * S, res.lastct_mask, i, W);
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
        if (g.sub == 0) prune[by_req ? i : k] = 1;
    }
    if (g.sub == 0) c.n[k] = new_n;
}

// group width: the power of two >= D, capped at a wave
inline int group_of(uint32_t D) {
    int g = 1;
    while (g < (int)D && g < AGN_WAVE) g <<= 1;
    return g;
}

template <int G>
int lookup_g(const agn_ss_cache &c, uint64_t n_req, const uint64_t *keys, const uint64_t *R,
             const uint64_t *Rm, uint64_t *sct, uint64_t *sctm, uint8_t *sct_ign, int64_t *base,
             uint8_t *first, uint8_t *status, hipStream_t st) {
    hipLaunchKernelGGL((k_ss_lookup<G>), dim3(grid_for(n_req, 256 / G, 0x7fffffffu)), dim3(256), 0,
                       st, c, n_req, keys, R, Rm, sct, sctm, sct_ign, base, first, status);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

template <int G>
int store_g(const agn_ss_cache &c, const uint64_t *key_off, const uint64_t *key_len, uint64_t n_req, const uint64_t *keys,
            const uint8_t *is_first, const uint8_t *status, const uint8_t *should_gc,
            const agn_result &res, const int64_t *handle, uint8_t *prune, uint64_t *thr,
            uint64_t *thrm, int by_req, hipStream_t st) {
    hipLaunchKernelGGL((k_ss_store<G>), dim3(grid_for(n_req, 256 / G, 0x7fffffffu)), dim3(256), 0,
                       st, c, key_off, key_len, n_req, keys, is_first, status, should_gc, res, handle,
                       prune, thr, thrm, by_req);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

}  // namespace

#define AGN_GROUP_DISPATCH(D, CALL)    \
    switch (group_of(D)) {             \
        case 1: return CALL(1);        \
        case 2: return CALL(2);        \
        case 4: return CALL(4);        \
        case 8: return CALL(8);        \
        case 16: return CALL(16);      \
        case 32: return CALL(32);      \
        default: return CALL(64);      \
    }

int launch_ss_lookup(const agn_ss_cache &c, uint64_t n_req, const uint64_t *keys,
                     const uint64_t *R, const uint64_t *Rm, uint64_t *sct, uint64_t *sctm,
                     uint8_t *sct_ign, int64_t *base, uint8_t *first, uint8_t *status,
                     hipStream_t st) {
    if (n_req == 0) return AGN_OK;
#define AGN_C(G) lookup_g<G>(c, n_req, keys, R, Rm, sct, sctm, sct_ign, base, first, status, st)
    AGN_GROUP_DISPATCH(c.n_dcs, AGN_C)
#undef AGN_C
}

int launch_ss_store(const agn_ss_cache &c, const uint64_t *key_off, const uint64_t *key_len,
                    uint64_t n_req,
                    const uint64_t *keys, const uint8_t *is_first, const uint8_t *status,
                    const uint8_t *should_gc, const agn_result &res, const int64_t *handle,
                    uint8_t *prune, uint64_t *thr, uint64_t *thrm, hipStream_t st) {
    AGN_HIP(hipMemsetAsync(prune, 0, c.n_keys, st));
    if (n_req == 0) return AGN_OK;
#define AGN_C(G) \
    store_g<G>(c, key_off, key_len, n_req, keys, is_first, status, should_gc, res, handle, prune, \
               thr, thrm, 0, st)
    AGN_GROUP_DISPATCH(c.n_dcs, AGN_C)
#undef AGN_C
}

// The same store with the prune flags per request (prune_req[n_req], no
// clearing of a per-key array): the cached batcher's form.
int launch_ss_store_req(const agn_ss_cache &c, const uint64_t *key_off, const uint64_t *key_len,
                        uint64_t n_req, const uint64_t *keys, const uint8_t *is_first,
                        const uint8_t *status, const uint8_t *should_gc, const agn_result &res,
                        uint8_t *prune_req, uint64_t *thr, uint64_t *thrm, hipStream_t st) {
    if (n_req == 0) return AGN_OK;
#define AGN_C(G) \
    store_g<G>(c, key_off, key_len, n_req, keys, is_first, status, should_gc, res, nullptr, \
               prune_req, thr, thrm, 1, st)
    AGN_GROUP_DISPATCH(c.n_dcs, AGN_C)
#undef AGN_C
}

}  // namespace agn
