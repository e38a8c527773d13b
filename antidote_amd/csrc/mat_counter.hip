// mat_counter.hip — batched clocksi_materializer:materialize/4 for
// antidote_crdt_counter_pn on gfx950 (one wave per key, grid-stride).
//
// Reference: materialize/4 src/clocksi_materializer.erl:89-101,
// apply_operations :113-121 with counter_pn update(E, S) = S + E
// (SURVEY.md §8(a) a5.1).  The snapshot filter is filter.hpp.
//   NewLastOp = id(oldest excluded, not-in-prev op) - 1, else FirstId (:49-63)
//   Count     = popcount of the included ballot
//   value     = base + sum of included effects (wave sum; integer, order-free)
// An included effect equal to AGN_EFFECT_INVALID (an Erlang term that was not
// an integer) yields {error,{unexpected_operation,..}} for the oldest such op
// (src/materializer.erl:53-58).
// HBM bytes per op: 8*D (OpSSCommit) + 8 (effect); per key: 16 (key_off pair)
// + 8*D (R) + 8*D (LastOpCt) + 32 (value, hole, count, flags, err_pos).
#include <cstdlib>

#include "filter.hpp"

namespace agn {
namespace {

template <int DPL, int LPO, bool SPARSE>
__global__ __launch_bounds__(256) void k_counter(agn_log log, agn_read req, agn_result out) {
    using F = KeyFilter<DPL, LPO, SPARSE>;
    __shared__ uint64_t stage[4][DPL][AGN_WAVE];
    const int w = threadIdx.x >> 6;
    const uint64_t nw = (uint64_t)gridDim.x * 4u;

    for (uint64_t i = (uint64_t)blockIdx.x * 4u + (uint64_t)w; i < req.n_req; i += nw) {
        const uint64_t key = req.keys ? uniform_u64(req.keys[i]) : i;
        const uint64_t off = uniform_u64(log.key_off[key]);
        const uint64_t n = uniform_u64(key_n(log.key_off, log.key_len, key));
        const int lane = lane_id();

        if (n != 0 && log.key_type != nullptr && log.key_type[key] != (uint8_t)req.req_type) {
            if (lane == 0) {  // erlang:error(corrupted_ops_cache) (:190-191)
                out.flags[i] = AGN_F_ERR_CORRUPTED;
                out.err_pos[i] = 0xffffffffu;
            }
            continue;
        }

        F f;
        f.init(log, req, i);
        int64_t sum = 0;
        uint32_t cnt = 0;
        int64_t first_err = -1;
        for (uint64_t b = 0; b < n; b += F::S::OPI) {
            bool valid;
            const bool incl = f.step(log, off, n, b, valid);
            const bool lead = incl && f.sub == 0;
            int64_t ev = 0;
            if (lead) ev = log.eff[off + b + (uint64_t)f.slot];
            const bool bad = lead && ev == AGN_EFFECT_INVALID;
            cnt += (uint32_t)__builtin_popcountll(ballot(lead));
            if (first_err < 0) {
                const uint64_t be = ballot(bad);
                if (be) first_err = (int64_t)b + (int64_t)(__builtin_ctzll(be) / LPO);
            }
            sum += bad ? 0 : ev;
        }
        sum = wave_sum_i64(sum);
        const bool ct_ign = f.sct_ign && cnt == 0u;
        f.write_ct(stage[w], out, i, ct_ign);

        if (lane == 0) {
            const int64_t base = req.base_value ? req.base_value[i] : 0;
            int64_t hole;
            if (f.first_excl >= 0) hole = (int64_t)log.op_id[off + (uint64_t)f.first_excl] - 1;
            else hole = n ? (int64_t)log.op_id[off + n - 1] : 0;
            uint32_t fl = 0;
            if (cnt) fl |= AGN_F_NEWSS;
            if (ct_ign) fl |= AGN_F_CT_IGNORE;
            if (first_err >= 0) fl |= AGN_F_ERR_UNEXPECTED;
            out.value[i] = (int64_t)((uint64_t)base + (uint64_t)sum);
            out.hole[i] = hole;
            out.count[i] = cnt;
            out.flags[i] = fl;
            out.err_pos[i] =
                first_err >= 0 ? (uint32_t)(off + (uint64_t)first_err) : 0xffffffffu;
        }
    }
}

template <int DPL, int LPO, bool SPARSE>
int launch_shape(const agn_log &log, const agn_read &req, const agn_result &out,
                 hipStream_t st) {
    const unsigned blocks = grid_for(req.n_req, 4, 0x7fffffffu);  // one wave per request
    hipLaunchKernelGGL((k_counter<DPL, LPO, SPARSE>), dim3(blocks), dim3(256), 0, st, log,
                       req, out);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

template <bool SPARSE>
int dispatch(const agn_log &log, const agn_read &req, const agn_result &out, hipStream_t st) {
#define AGN_L(DPL, LPO) launch_shape<DPL, LPO, SPARSE>(log, req, out, st)
    AGN_DISPATCH_SHAPES(log.n_dcs, AGN_L)
#undef AGN_L
}

}  // namespace

int launch_counter(const agn_log &log, const agn_read &req, const agn_result &out,
                   hipStream_t st) {
    if (req.n_req == 0) return AGN_OK;
    // AGN_COUNTER_IMPL=general forces the general kernel (A/B and tests)
    const bool force_general = [] {
        const char *v = AGN_KNOB("AGN_COUNTER_IMPL");
        return v && v[0] == 'g';
    }();
    if (!force_general) {
        const int rc = launch_counter_dense(log, req, out, st);
        if (rc != AGN_ENOTSUP) return rc;
    }
    const bool sparse = log.oc_mask || req.R_mask || req.sct_mask || out.lastct_mask;
    return sparse ? dispatch<true>(log, req, out, st) : dispatch<false>(log, req, out, st);
}

}  // namespace agn
