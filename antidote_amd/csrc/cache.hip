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
#include "cache_dev.hpp"
#include "serve.hpp"
#include "tags_serve.hpp"

namespace agn {
namespace {

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
    const uint32_t D = c.n_dcs, W = n_words(D);
    const uint64_t k = keys ? keys[i] : i;
    const LookupOut r = ss_lookup_one<G>(g, c, k, R + i * D, Rm ? Rm + i * W : nullptr, sct + i * D,
                                         sctm ? sctm + i * W : nullptr);
    if (g.sub == 0) {
        sct_ign[i] = r.ign;
        base[i] = r.base;
        first[i] = r.first;
        status[i] = r.status;
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
                                                  uint64_t *__restrict__ thrm, int by_req,
                                                  const uint32_t *__restrict__ list,
                                                  const uint32_t *__restrict__ list_n) {
    const Grp<G> g;
    uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    if (list) {  // a request list (the fused set/register read's hand-ons)
        if (i >= *list_n) return;
        i = list[i];
    }
    if (i >= n_req) return;
    const uint32_t D = c.n_dcs, W = n_words(D);
    const uint64_t k = keys ? keys[i] : i;
    // a state arena stores the result's state pairs (set_aw / register_mv)
    const bool st = c.state_tag != nullptr && res.out_off != nullptr;
    const uint64_t so = st ? res.out_off[i] : 0ull;
    // nops: the key's device op count (number_of_ops of the read's ops list,
    // :468-471); without key_off the caller's snapshot came from a log
    // response whose number_of_ops it checked (agn_batcher_store): not 0
    const uint64_t nops = key_off ? key_n(key_off, key_len, k) : 1ull;
    const bool pr = ss_store_one<G>(
        g, c, k, nops, status[i], is_first[i],
        should_gc != nullptr && should_gc[i] != 0, res.lastct + i * D,
        res.lastct_mask ? res.lastct_mask + i * W : nullptr, res.hole[i],
        (handle && !st) ? handle[i] : st ? 0 : res.value[i], res.count[i], res.flags[i], thr, thrm,
        st ? res.out_tag + so : nullptr, st ? res.out_tok + so : nullptr, st ? res.out_n[i] : 0u);
    // by_req: prune flags per request (prune[i], every request written),
    // otherwise per key (prune[k], the caller cleared the array)
    if (g.sub == 0) {
        if (by_req) prune[i] = pr ? 1 : 0;
        else if (pr) prune[k] = 1;
    }
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
            uint64_t *thrm, int by_req, hipStream_t st, const uint32_t *list = nullptr,
            const uint32_t *list_n = nullptr) {
    hipLaunchKernelGGL((k_ss_store<G>), dim3(grid_for(n_req, 256 / G, 0x7fffffffu)), dim3(256), 0,
                       st, c, key_off, key_len, n_req, keys, is_first, status, should_gc, res, handle,
                       prune, thr, thrm, by_req, list, list_n);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

// agn_ss_state_compact: one wave per key; the key's live slots' states are
// copied into the fresh arena at one atomically reserved range, and their
// references rewritten (into nv when given, else in place).  ctl[0] (reset to
// 0 before) ends as the live pairs.
__global__ __launch_bounds__(256) void k_ss_compact(agn_ss_cache c, uint32_t *__restrict__ nt,
                                                   uint64_t *__restrict__ nk, uint64_t ncap,
                                                   uint64_t *__restrict__ ovf,
                                                   int64_t *__restrict__ nv) {
    int64_t *const out = nv ? nv : c.value;
    const uint64_t k = uniform_u64((uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6));
    if (k >= c.n_keys) return;
    const int lane = lane_id();
    const uint32_t S = c.slots, n = c.n[k];
    uint64_t tot = 0;
    for (uint32_t j = 0; j < n; ++j) tot += AGN_SS_STATE_PAIRS(c.value[k * S + j]);
    if (tot == 0) {
        if (lane == 0)
            for (uint32_t j = 0; j < n; ++j) out[k * S + j] = AGN_SS_STATE(0, 0);
        return;
    }
    uint64_t base = 0;
    if (lane == 0) base = atomicAdd((unsigned long long *)&c.state_ctl[0], (unsigned long long)tot);
    base = uniform_u64(base);  // lane 0's (the first active lane)
    if (base + tot > ncap) {  // the host sized the arena from ctl: cannot happen
        if (lane == 0) *ovf = 1ull;
        return;
    }
    for (uint32_t j = 0; j < n; ++j) {
        const int64_t v = c.value[k * S + j];
        const uint64_t s0 = AGN_SS_STATE_START(v);
        const uint32_t p = AGN_SS_STATE_PAIRS(v);
        for (uint32_t x = lane; x < p; x += AGN_WAVE) {
            nt[base + x] = c.state_tag[s0 + x];
            nk[base + x] = c.state_tok[s0 + x];
        }
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) out[k * S + j] = AGN_SS_STATE(p ? base : 0, p);
        base += p;
    }
}

}  // namespace

int launch_ss_compact(const agn_ss_cache &c, uint32_t *new_tag, uint64_t *new_tok, uint64_t new_cap,
                      uint64_t *ovf, hipStream_t st, int64_t *new_value) {
    AGN_HIP(hipMemsetAsync(c.state_ctl, 0, 4 * sizeof(uint64_t), st));
    if (c.n_keys == 0) return AGN_OK;
    const uint64_t nb = (c.n_keys + 3) / 4;
    if (nb > 0x7fffffffull) return fail(AGN_EINVAL, "ss_state_compact: too many keys");
    hipLaunchKernelGGL(k_ss_compact, dim3((unsigned)nb), dim3(256), 0, st, c, new_tag, new_tok,
                       new_cap, ovf, new_value);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

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

int launch_ss_store_list(const agn_ss_cache &c, const uint64_t *key_off, const uint64_t *key_len,
                         uint64_t n_req, const uint32_t *list, const uint32_t *list_n,
                         const uint64_t *keys, const uint8_t *is_first, const uint8_t *status,
                         const uint8_t *should_gc, const agn_result &res, uint8_t *prune_req,
                         uint64_t *thr, uint64_t *thrm, hipStream_t st) {
    if (n_req == 0) return AGN_OK;
#define AGN_C(G) \
    store_g<G>(c, key_off, key_len, n_req, keys, is_first, status, should_gc, res, nullptr, \
               prune_req, thr, thrm, 1, st, list, list_n)
    AGN_GROUP_DISPATCH(c.n_dcs, AGN_C)
#undef AGN_C
}

}  // namespace agn
