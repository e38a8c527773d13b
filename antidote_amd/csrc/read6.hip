// read6.hip — materializer_vnode:read/6 for a batch of distinct keys in ONE
// kernel (the cached read batcher's path for counter_pn, dense clocks,
// D <= 8).  One wave per request:
//   1. get_from_snapshot_cache (src/materializer_vnode.erl:384-413,
//      vector_orddict:get_smaller src/vector_orddict.erl:74-87) on the
//      request's group of G lanes (cache_dev.hpp), the SCT row into LDS;
//   2. materialize/4 from that base (src/clocksi_materializer.erl:82-268):
//      the dense counter scan (counter_scan.hpp), SCT and R in SGPRs;
//   3. the cache half of materialize_snapshot / internal_store_ss /
//      snapshot_insert_gc (:341-364, 466-563) on the group, LastOpCt from LDS.
// The three steps are the batched kernels k_ss_lookup -> k_counter_key ->
// k_ss_store run back to back per request, so a batch costs one launch
// instead of three kernels and two copies: requests are read from, and
// results written to, device-visible pinned host memory.
#include "cache_dev.hpp"
#include "counter_scan.hpp"
#include "serve.hpp"

namespace agn {
namespace {

template <int D, int G>
__global__ __launch_bounds__(64) void k_read6(agn_ss_cache c, Read6Args a) {
    constexpr int DCP = D <= 1 ? 1 : D <= 2 ? 2 : D <= 4 ? 4 : 8;  // pow2 >= D
    constexpr int V = DCP;                                          // op slots per lane
    static_assert(G == DCP, "group = the power of two >= D");
    __shared__ uint64_t stage[DCP][AGN_WAVE];
    __shared__ uint64_t sct_row[DCP], ct_row[DCP];
    const uint64_t i = blockIdx.x;
    if (i >= a.n_req) return;
    const int lane = lane_id();
    const uint64_t key = uniform_u64(a.keys[i]);

    // 1. the base snapshot <= R
    LookupOut lk{0, 0, 0, 0};
    if (lane < G) {
        const Grp<G> g;
        lk = ss_lookup_one<G>(g, c, key, a.R + i * D, nullptr, sct_row, nullptr);
    }
    const bool sct_ign = __builtin_amdgcn_readfirstlane(lk.ign) != 0;
    const uint32_t st = __builtin_amdgcn_readfirstlane(lk.status);
    const uint32_t is_first = __builtin_amdgcn_readfirstlane(lk.first);
    const int64_t base = (int64_t)uniform_u64((uint64_t)lk.base);
    __syncthreads();  // sct_row

    // 2. materialize/4 from the base (k_counter_key's body)
    uint64_t r[D], s[D], ct[D];
#pragma unroll
    for (int j = 0; j < D; ++j) r[j] = uniform_u64(a.R[i * D + j]);
    const KeyMeta km = key_meta(key, a.key_off, a.key_len, a.key_id0);
    const uint64_t off = km.off, n = km.n;
    if (n != 0 && a.key_type != nullptr && byte_of(a.key_type, key) != (a.req_type & 0xffu)) {
        if (lane == 0) {  // erlang:error(corrupted_ops_cache) (:190-191)
            a.value[i] = 0;
            a.hole[i] = 0;
            a.count[i] = 0;
            a.flags[i] = AGN_F_ERR_CORRUPTED;
            a.err_pos[i] = 0xffffffffu;
            a.status[i] = (uint8_t)st;
            a.prune[i] = 0;
            a.dkeys[i] = key;
            a.dprune[i] = 0;
        }
        if (lane < D) a.lastct[i * D + (uint64_t)lane] = 0ull;
        return;
    }
#pragma unroll
    for (int j = 0; j < D; ++j) {
        s[j] = sct_ign ? 0ull : uniform_u64(sct_row[j]);
        ct[j] = s[j];  // LastOpCt starts as SCT (materialize/4 :94-95)
    }
    const uint64_t txr = a.txid ? uniform_u64(a.txid[i]) : 0ull;
    const uint64_t *tx = (txr != 0ull) ? a.log_txid : nullptr;
    int64_t sum = 0, first_excl = -1, first_err = -1;
    uint32_t cnt = 0;
    if (sct_ign)
        scan_key<D, false>(a.oc, a.eff, tx, txr, off, n, r, s, ct, sum, cnt, first_excl, first_err);
    else
        scan_key<D, true>(a.oc, a.eff, tx, txr, off, n, r, s, ct, sum, cnt, first_excl, first_err);
    int64_t hid;
    {
        const uint64_t pos = first_excl >= 0 ? (uint64_t)first_excl : n - 1;
        if (km.id0 != AGN_ID0_NONE)  // op_id[off + pos] == id0 + pos (agn_log_index_ids)
            hid = n ? (int64_t)((uint64_t)km.id0 + pos) : 0;
        else
            hid = n ? (int64_t)a.op_id[uniform_u64(off + pos)] : 0;
    }
    const int64_t total = wave_sum_dpp(sum);
    // LastOpCt: per-lane maxima -> LDS [DCP][64] -> each lane folds V slots of
    // one DC -> xor-shuffle across the 64/DCP lanes that share it
#pragma unroll
    for (int j = 0; j < D; ++j) stage[j][lane] = ct[j];
    __syncthreads();
    const int cd = lane % DCP, grp = lane / DCP;
    uint64_t m = 0;
    if (cd < D) {
#pragma unroll
        for (int v = 0; v < V; ++v) m = umax64(m, stage[cd][grp * V + v]);
    }
#pragma unroll
    for (int x = DCP; x < AGN_WAVE; x <<= 1) m = umax64(m, shfl_xor_u64(m, x));
    const bool ct_ign = sct_ign && cnt == 0u;
    if (grp == 0 && cd < D) {
        const uint64_t mv = ct_ign ? 0ull : m;
        a.lastct[i * D + (uint64_t)cd] = mv;
        ct_row[cd] = mv;
    }
    // NewLastOp = id(oldest excluded) - 1, else get_first_id (:49-63)
    const int64_t hole = first_excl >= 0 ? hid - 1 : hid;
    uint32_t fl = 0;
    if (cnt) fl |= AGN_F_NEWSS;
    if (ct_ign) fl |= AGN_F_CT_IGNORE;
    if (first_err >= 0) fl |= AGN_F_ERR_UNEXPECTED;
    const int64_t value = (int64_t)((uint64_t)base + (uint64_t)total);
    __syncthreads();  // ct_row

    // 3. internal_store_ss / snapshot_insert_gc's policy
    bool pr = false;
    if (lane < G) {
        const Grp<G> g;
        const bool gc = a.gc != nullptr && a.gc[i] != 0;
        pr = ss_store_one<G>(g, c, key, n, (uint8_t)st, (uint8_t)is_first, gc, ct_row, nullptr,
                             hole, value, cnt, fl, a.thr, nullptr);
    }
    if (lane == 0) {
        a.value[i] = value;
        a.hole[i] = hole;
        a.count[i] = cnt;
        a.flags[i] = fl;
        a.err_pos[i] = first_err >= 0 ? (uint32_t)(off + (uint64_t)first_err) : 0xffffffffu;
        a.status[i] = (uint8_t)st;
        a.prune[i] = pr ? 1 : 0;
        a.dkeys[i] = key;
        a.dprune[i] = pr ? 1 : 0;
    }
}

}  // namespace

bool read6_supported(const agn_log &view, uint32_t D) {
    return view.crdt_type == AGN_COUNTER_PN && view.oc_mask == nullptr && D >= 1 && D <= 8;
}

int launch_read6(const agn_ss_cache &c, const Read6Args &a, hipStream_t st) {
    if (a.n_req == 0) return AGN_OK;
    if (a.n_req > 0x7fffffffull) return fail(AGN_ENOTSUP, "read6: batch too large");
    const dim3 grid((unsigned)a.n_req), block(AGN_WAVE);
    switch (a.n_dcs) {
        case 1: hipLaunchKernelGGL((k_read6<1, 1>), grid, block, 0, st, c, a); break;
        case 2: hipLaunchKernelGGL((k_read6<2, 2>), grid, block, 0, st, c, a); break;
        case 3: hipLaunchKernelGGL((k_read6<3, 4>), grid, block, 0, st, c, a); break;
        case 4: hipLaunchKernelGGL((k_read6<4, 4>), grid, block, 0, st, c, a); break;
        case 5: hipLaunchKernelGGL((k_read6<5, 8>), grid, block, 0, st, c, a); break;
        case 6: hipLaunchKernelGGL((k_read6<6, 8>), grid, block, 0, st, c, a); break;
        case 7: hipLaunchKernelGGL((k_read6<7, 8>), grid, block, 0, st, c, a); break;
        case 8: hipLaunchKernelGGL((k_read6<8, 8>), grid, block, 0, st, c, a); break;
        default: return fail(AGN_ENOTSUP, "read6: n_dcs=%u", a.n_dcs);
    }
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

}  // namespace agn
