// gen.hpp — deterministic synthetic op logs,
// one SplitMix64 stream per key, compiled for host and device alike so both
// produce bit-identical logs.
//
// Per key (global index gk = key_base + k * key_stride), N ops, D DCs:
//   cut  = U[0,N]   read snapshot covers the ops before `cut`
//   cut2 = U[0,cut] (warm only) base snapshot covers the ops before `cut2`
//   clk[d] = 1.7e15 + U[0,1000]
//   op i: c = U[0,D-1]; lag[d] = U[0,5000] for every d; clk[c] += U[1,1000];
//         OpSSCommit oc[d] = clk[d] - lag[d] (d != c), oc[c] = clk[c]
//         counter_pn : effect U[0,2000] - 1000
//         set_aw     : elem U[0,E-1]; U[0,99] < 70 -> add a fresh token,
//                      observing (removing) the elem's live tokens unless a
//                      concurrent add (U[0,99] < 20 and < 4 live); else remove
//                      every live token of the elem
//         register_mv: value U[0,E-1]; U[0,99] < 5 -> reset(live tokens);
//                      else assign a fresh token overriding the live tokens
//                      unless concurrent (U[0,99] < 20 and < 4 live)
//   R[d]   = max(clk0[d], oc[d] of ops < cut) + U[0,4000] - J, J = min(2000, 16000/D)
//            (J shrinks with D so that wide clocks still include a prefix-ish
//            subset: every one of the op's D entries must be <= R)
//   SCT[d] = max(clk0[d], oc[d] of ops < cut2)     (warm; else ignore)
//   token = (gk << 24) | (i + 1); op_id = i + 1; txid none.
#pragma once
#include <stdint.h>

#include "../../include/antidote_gpu.h"

#ifdef __HIPCC__
#define AGN_HD __host__ __device__
#else
#define AGN_HD
#endif

namespace agn {

struct Rng {
    uint64_t s;
    AGN_HD uint64_t next() {
        s += 0x9E3779B97F4A7C15ull;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    AGN_HD uint64_t uni(uint64_t lo, uint64_t hi) { return lo + next() % (hi - lo + 1ull); }
};

AGN_HD inline Rng key_rng(uint64_t seed, uint64_t gk) {
    Rng r{seed ^ (0x632BE59BD9B4E019ull * (gk + 1ull))};
    r.next();
    return r;
}

constexpr uint64_t GEN_CLOCK_BASE = 1700000000000000ull;
constexpr int GEN_MAX_LIVE = 4;

struct GenOut {
    // per-key views (already offset to this key); counts-only when oc == nullptr
    uint64_t *oc;        // [N * D]
    uint32_t *op_id;     // [N]
    int64_t *eff;        // [N]
    uint32_t *tag;       // [N]
    uint64_t *add_tok;   // [N]
    uint32_t *rem_cnt;   // [N] (counts pass) — rem_off[e+1] before the scan
    const uint32_t *rem_off;  // [N] absolute offsets (write pass)
    uint64_t *rem_tok;   // base of the log's rem_tok
    uint64_t *R;         // [D]
    uint64_t *sct;       // [D] or nullptr
    uint8_t *sct_ignore; // [1] or nullptr
    uint64_t *clk;       // scratch [D]
    uint64_t *live;      // scratch [E * GEN_MAX_LIVE] (set) or [GEN_MAX_LIVE] (register)
    uint32_t *live_n;    // scratch [E] or [1]
};

AGN_HD inline void gen_key(const agn_gen_cfg &cfg, uint64_t k, GenOut &o) {
    const uint32_t D = cfg.n_dcs, N = cfg.ops_per_key, E = cfg.n_elems ? cfg.n_elems : 1;
    const uint64_t gk = cfg.key_base + k * (cfg.key_stride ? cfg.key_stride : 1ull);
    const bool write = o.oc != nullptr;
    Rng rng = key_rng(cfg.seed, gk);
    const uint64_t cut = rng.uni(0, N);
    const uint64_t cut2 = cfg.warm ? rng.uni(0, cut) : 0;
    for (uint32_t d = 0; d < D; ++d) {
        o.clk[d] = GEN_CLOCK_BASE + rng.uni(0, 1000);
        if (write) {
            o.R[d] = o.clk[d];
            if (o.sct) o.sct[d] = o.clk[d];
        }
    }
    const int set = cfg.crdt_type == AGN_SET_AW;
    const int reg = cfg.crdt_type == AGN_REGISTER_MV;
    const uint32_t nl = set ? E : 1;
    for (uint32_t x = 0; x < nl; ++x) o.live_n[x] = 0;

    for (uint32_t i = 0; i < N; ++i) {
        const uint32_t c = (uint32_t)rng.uni(0, D - 1);
        const uint64_t inc = rng.uni(1, 1000);
        uint64_t *oc = write ? o.oc + (uint64_t)i * D : nullptr;
        for (uint32_t d = 0; d < D; ++d) {
            const uint64_t lag = rng.uni(0, 5000);
            if (write) oc[d] = o.clk[d] - lag;
        }
        o.clk[c] += inc;
        if (write) {
            oc[c] = o.clk[c];
            o.op_id[i] = i + 1;
            for (uint32_t d = 0; d < D; ++d) {
                if (i < cut && oc[d] > o.R[d]) o.R[d] = oc[d];
                if (o.sct && i < cut2 && oc[d] > o.sct[d]) o.sct[d] = oc[d];
            }
        }
        if (cfg.crdt_type == AGN_COUNTER_PN) {
            const int64_t eff = (int64_t)rng.uni(0, 2000) - 1000;
            if (write) o.eff[i] = eff;
            continue;
        }
        const uint64_t tok = (gk << 24) | (uint64_t)(i + 1);
        uint32_t tag = 0;
        uint64_t add = 0;
        uint32_t slot = 0;  // which live list
        bool add_op = false, keep = false;
        if (set) {
            tag = (uint32_t)rng.uni(0, E - 1);
            slot = tag;
            add_op = rng.uni(0, 99) < 70;
            if (add_op) keep = rng.uni(0, 99) < 20 && o.live_n[slot] < GEN_MAX_LIVE;
        } else if (reg) {
            tag = (uint32_t)rng.uni(0, E - 1);
            add_op = rng.uni(0, 99) >= 5;
            if (add_op) keep = rng.uni(0, 99) < 20 && o.live_n[0] < GEN_MAX_LIVE;
            if (!add_op) tag = 0;
        }
        uint64_t *lv = o.live + (uint64_t)slot * GEN_MAX_LIVE;
        const uint32_t n_rem = keep ? 0u : o.live_n[slot];
        if (write) {
            o.tag[i] = tag;
            o.add_tok[i] = add_op ? tok : 0ull;
            for (uint32_t x = 0; x < n_rem; ++x) o.rem_tok[o.rem_off[i] + x] = lv[x];
        } else {
            o.rem_cnt[i] = n_rem;
        }
        if (add_op) {
            add = tok;
            if (keep) {
                lv[o.live_n[slot]++] = add;
            } else {
                lv[0] = add;
                o.live_n[slot] = 1;
            }
        } else {
            o.live_n[slot] = 0;
        }
    }
    if (write) {
        const uint64_t J = D >= 8 ? 16000ull / D : 2000ull;
        for (uint32_t d = 0; d < D; ++d) o.R[d] = o.R[d] + rng.uni(0, 4000) - J;
        if (o.sct_ignore) o.sct_ignore[0] = cfg.warm ? 0 : 1;
    }
}

}  // namespace agn
