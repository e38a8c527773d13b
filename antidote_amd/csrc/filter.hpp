// filter.hpp — the per-key vector-clock snapshot filter shared by every CRDT
// kernel: is_op_in_snapshot/7 + belongs_to_snapshot_op/3 + the NewLastOp /
// LastOpCt bookkeeping of materialize_intern (src/clocksi_materializer.erl:
// 157-268, src/materializer.erl:101-106).
//
// One wave owns one key.  LPO lanes cover one op, DPL DCs per lane
// (D <= DPL*LPO); OPI = 64/LPO ops per iteration, visited oldest first
// (the reference visits newest first; every output it derives is either
// order-free or a min over positions, so the order does not matter).
#pragma once
#include "common.hpp"

namespace agn {

template <int DPL, int LPO>
struct Shape {
    static constexpr int OPI = AGN_WAVE / LPO;
    static constexpr int DC = DPL * LPO;
    static constexpr int DCP = DC <= 1 ? 1 : DC <= 2 ? 2 : DC <= 4 ? 4 : DC <= 8 ? 8 : DC;
    static constexpr int G = DCP <= AGN_WAVE ? AGN_WAVE / DCP : 1;   // lanes per DC
    static constexpr int T = DCP <= AGN_WAVE ? 1 : DCP / AGN_WAVE;   // DCs per lane
    static constexpr int V = DCP <= AGN_WAVE ? DCP / LPO : OPI;      // slots per lane
};

// Presence bits of DCs [d0, d0+DPL) of clock `row` (dense: all d < D).
template <int DPL, bool SPARSE>
__device__ __forceinline__ uint32_t chunk_bits(const uint64_t *mask, uint64_t row, uint32_t W,
                                               int d0, uint32_t D) {
    const int valid = (int)D - d0;
    if (valid <= 0) return 0u;
    const uint32_t full = valid >= DPL ? ((1u << DPL) - 1u) : ((1u << valid) - 1u);
    if (!SPARSE || mask == nullptr) return full;
    const uint64_t w = mask[row * W + ((uint32_t)d0 >> 6)];
    return (uint32_t)(w >> ((uint32_t)d0 & 63u)) & full;
}

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

// One sub-iteration's OpSSCommit slice: DPL DCs of one op per lane.
template <int DPL, bool SPARSE, bool FULL>
__device__ __forceinline__ void load_rows(const agn_log &log, uint64_t e, int d0, uint32_t D,
                                          uint32_t W, uint64_t (&v)[DPL], uint32_t &bits) {
    if constexpr (FULL) {
        const u64x2 *q = reinterpret_cast<const u64x2 *>(log.oc + e * D + (uint32_t)d0);
#pragma unroll
        for (int j = 0; j < DPL / 2; ++j) {
            const u64x2 x = q[j];
            v[2 * j] = x.x;
            v[2 * j + 1] = x.y;
        }
        bits = (1u << DPL) - 1u;
    } else {
        bits = chunk_bits<DPL, SPARSE>(log.oc_mask, e, W, d0, D);
#pragma unroll
        for (int j = 0; j < DPL; ++j)
            v[j] = ((bits >> j) & 1u) ? log.oc[e * D + (uint32_t)(d0 + j)] : 0ull;
    }
}

template <int DPL, int LPO, bool SPARSE>
struct KeyFilter {
    using S = Shape<DPL, LPO>;
    int lane, sub, slot, d0;
    uint32_t D, W;
    uint64_t grp;
    uint64_t r[DPL], s[DPL];
    uint64_t ct[DPL];  // LastOpCt, "+1 encoded": 0 = DC absent from the dict
    uint32_t rbits;
    bool sct_ign, use_tx;
    uint64_t txr;
    int64_t first_excl;  // position of the oldest op with notInPrev && !incl

    __device__ __forceinline__ void init(const agn_log &log, const agn_read &req, uint64_t i) {
        lane = lane_id();
        sub = lane % LPO;
        slot = lane / LPO;
        d0 = sub * DPL;
        D = log.n_dcs;
        W = n_words(D);
        grp = ((1ull << LPO) - 1ull) << (slot * LPO);
        rbits = chunk_bits<DPL, SPARSE>(req.R_mask, i, W, d0, D);
        sct_ign = req.sct == nullptr || (req.sct_ignore && req.sct_ignore[i]);
        const uint32_t sbits =
            sct_ign ? 0u : chunk_bits<DPL, SPARSE>(req.sct_mask, i, W, d0, D);
#pragma unroll
        for (int j = 0; j < DPL; ++j) {
            const uint32_t d = (uint32_t)(d0 + j);
            r[j] = (d < D) ? req.R[i * D + d] : 0ull;
            s[j] = ((sbits >> j) & 1u) ? req.sct[i * D + d] : 0ull;
            // LastOpCt starts as SnapshotCommitTime (materialize/4 :94-95)
            ct[j] = ((sbits >> j) & 1u) ? s[j] + 1ull : 0ull;
        }
        txr = req.txid ? req.txid[i] : 0ull;
        use_tx = (txr != 0ull) && (log.txid != nullptr);
        first_excl = -1;
    }

    // One iteration over ops [b, b+OPI) of the key; returns whether this
    // lane's op is included (identical on the op's LPO lanes).
    __device__ __forceinline__ bool step(const agn_log &log, uint64_t off, uint64_t n,
                                         uint64_t b, bool &valid_out) {
        const uint64_t pos = b + (uint64_t)slot;
        const bool valid = pos < n;
        valid_out = valid;
        const uint64_t e = off + pos;
        const uint32_t obits =
            valid ? chunk_bits<DPL, SPARSE>(log.oc_mask, e, W, d0, D) : 0u;
        uint64_t oc[DPL];
#pragma unroll
        for (int j = 0; j < DPL; ++j)
            oc[j] = ((obits >> j) & 1u) ? log.oc[e * D + (uint32_t)(d0 + j)] : 0ull;

        // dict:fold over OpSSCommit (:235-258) and vectorclock:le(oc, SCT)
        bool okR = true, leS = true;
#pragma unroll
        for (int j = 0; j < DPL; ++j) {
            if ((obits >> j) & 1u) {
                const bool inR = SPARSE ? (((rbits >> j) & 1u) != 0u) : true;
                okR = okR && inR && (oc[j] <= r[j]);  // DC missing in R -> false (:245-247)
                leS = leS && (oc[j] <= s[j]);         // missing SCT entry reads 0
            }
        }
        if (LPO > 1) {
            const uint64_t bR = ballot(!okR), bS = ballot(!leS);
            okR = (bR & grp) == 0ull;
            leS = (bS & grp) == 0ull;
        }
        // belongs_to_snapshot_op(SCT, ...) or (TxId == op.txid)  (:219-220)
        bool not_in_prev = sct_ign || !leS;
        if (use_tx) {
            bool txm = valid && sub == 0 && log.txid[e] == txr;
            if (LPO > 1) txm = (ballot(txm) >> (slot * LPO)) & 1ull;
            not_in_prev = not_in_prev || txm;
        }
        const bool incl = valid && not_in_prev && okR;
        const bool excl = valid && not_in_prev && !okR;
        if (first_excl < 0) {
            const uint64_t bx = ballot(excl && sub == 0);
            if (bx) first_excl = (int64_t)b + (int64_t)(__builtin_ctzll(bx) / LPO);
        }
        if (incl) {
#pragma unroll
            for (int j = 0; j < DPL; ++j)
                if ((obits >> j) & 1u) ct[j] = umax64(ct[j], oc[j] + 1ull);
        }
        return incl;
    }

    // Reduce the per-lane LastOpCt accumulators across the wave (through the
    // wave's LDS stage [DPL][64]) and write lastct / lastct_mask of request i.
    __device__ __forceinline__ void write_ct(uint64_t (*stage)[AGN_WAVE], const agn_result &out,
                                             uint64_t i, bool ct_ign) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
        for (int j = 0; j < DPL; ++j) stage[j][lane] = ct[j];
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int t = 0; t < S::T; ++t) {
            const int c = (S::DCP <= AGN_WAVE) ? (lane % S::DCP) : (lane + AGN_WAVE * t);
            const int g = (S::DCP <= AGN_WAVE) ? (lane / S::DCP) : 0;
            const int csub = c / DPL, cj = c % DPL;
            uint64_t m = 0;
            if (c < S::DC) {
#pragma unroll
                for (int v = 0; v < S::V; ++v) {
                    const int sl = g * S::V + v;
                    m = umax64(m, stage[cj][sl * LPO + csub]);
                }
            }
#pragma unroll
            for (int x = S::DCP; x < AGN_WAVE; x <<= 1) m = umax64(m, shfl_xor_u64(m, x));
            const bool writer = (g == 0) && ((uint32_t)c < D);
            if (writer) out.lastct[i * D + (uint32_t)c] = (m && !ct_ign) ? m - 1ull : 0ull;
            if (SPARSE && out.lastct_mask != nullptr) {
                const uint64_t pm = ballot(writer && m != 0ull && !ct_ign);
                if (lane == 0) out.lastct_mask[i * W + (uint32_t)t] = pm;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
};

// Shape dispatch: D <= 8 exact (DPL = D, one lane per op), wider clocks use
// 8 DCs per lane and LPO = 2..32 lanes per op.
#define AGN_DISPATCH_SHAPES(D, LAUNCH)                       \
    switch (D) {                                             \
        case 1: return LAUNCH(1, 1);                         \
        case 2: return LAUNCH(2, 1);                         \
        case 3: return LAUNCH(3, 1);                         \
        case 4: return LAUNCH(4, 1);                         \
        case 5: return LAUNCH(5, 1);                         \
        case 6: return LAUNCH(6, 1);                         \
        case 7: return LAUNCH(7, 1);                         \
        case 8: return LAUNCH(8, 1);                         \
        default: break;                                      \
    }                                                        \
    if ((D) <= 16) return LAUNCH(8, 2);                      \
    if ((D) <= 32) return LAUNCH(8, 4);                      \
    if ((D) <= 64) return LAUNCH(8, 8);                      \
    if ((D) <= 128) return LAUNCH(8, 16);                    \
    return LAUNCH(8, 32);

}  // namespace agn
