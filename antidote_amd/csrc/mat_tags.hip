// mat_tags.hip — batched materialize/4 for antidote_crdt_set_aw and
// antidote_crdt_register_mv on gfx950: order-aware tag resolution.
//
// Reference fold (apply_operations, src/clocksi_materializer.erl:113-121,
// antidote_crdt 0.1.2 update/2, restated in SURVEY.md §8(a) a5.2/a5.3):
//   set_aw      entry {Elem, Add, Rem}: Tokens(Elem) := (Tokens -- Rem) ++ Add
//   register_mv entry {V, Tok, Ovr}: drop tokens in Ovr, insert_sorted({V, Tok})
//               entry {reset, Ovr}: drop tokens in Ovr
// applied oldest first.  Sequentially, the pair added at position p (or base
// pair, p < 0) survives iff no INCLUDED entry at a position q > p removes its
// token (set_aw: under the same elem); inside one entry the removal happens
// before the add.  Every pair is judged on its own, so repeated tokens keep
// the fold's multiset semantics.
//
// Kernel structure (one wave per key, one wave per block, grid = batch):
//   * the key is processed in chunks of 64 log entries (lane = entry for the
//     per-entry fields, LPO lanes x DPL DCs per op for the clock rows);
//   * the snapshot filter streams the OpSSCommit rows through a two-deep
//     register ring: the rows of sub-iteration j+1 (and the next chunk's side
//     fields) are in flight while sub-iteration j is compared, and every
//     prefetch is unconditional (clamped address) so the compiler's counted
//     vmcnt waits stay exact;
//   * per chunk, the entry fields (tag, add token, removal range, op id) and
//     the chunk's removal tokens (up to RB*64, prefetched before the filter)
//     are resolved against an LDS candidate list: included adds are appended
//     in position order ({tok, tag, ord}), hashed into per-bucket chains; each
//     included removal token then walks its chain and marks DEAD every
//     candidate with that token (set_aw: and elem) whose ord is older;
//   * the list is compacted in place when full; a key whose live state does
//     not fit CAP - 64 slots is pushed to a worklist and redone by the same
//     kernel with a 4096-slot table (one wave per block), which flags
//     AGN_F_ERR_CAPACITY only beyond that;
//   * live pairs are bitonic-sorted in LDS into the fold's order: set_aw
//     (elem, add order), register_mv (value, token).
//
// HBM bytes per entry: 8*D (OpSSCommit) + 4 (op_id) + 4 (tag) + 8 (add_tok)
// + 4 (rem_off) + 8 per removed token; plus 12 per live output pair.
#include <cstdlib>

#include "cache_dev.hpp"
#include "filter.hpp"
#include "tags_serve.hpp"

namespace agn {
namespace {

constexpr uint32_t DEAD = 0x80000000u;
constexpr uint32_t NIL = 0xffffffffu;


// The candidate table: 5.5 KB per wave at CAP = 256 (CAP hash buckets,
// 16-bit chain links).  The fast pass's occupancy is set by it: at 7 KB
// (2 CAP buckets, 32-bit links) 22 one-wave blocks fit a CU, 5.5 per SIMD,
// below the 7 its 73 VGPRs allow.
template <int CAP>
struct CandLds {
    static_assert(CAP < 0xffff, "16-bit chain links");
    uint64_t tok[CAP];
    uint32_t tag[CAP];
    uint32_t ord[CAP];   // B + position (base pairs: index < B); DEAD bit
    uint32_t head[CAP];  // hash buckets (chain heads, NIL = empty)
    uint16_t nxt[CAP];   // hash chain, 0xffff = end
};

template <int CAP>
__device__ __forceinline__ uint32_t hbucket(uint64_t t) {
    constexpr int LOG = __builtin_ctz(CAP);
    return (uint32_t)((t * 0x9E3779B97F4A7C15ull) >> (64 - LOG));
}

template <int CAP>
__device__ __forceinline__ uint32_t chain_next(const CandLds<CAP> &L, uint32_t x) {
    const uint32_t v = L.nxt[x];
    return v == 0xffffu ? NIL : v;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint64_t lanes_below() {
    const int lane = lane_id();
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

template <int CAP>
__device__ __forceinline__ void heads_clear(CandLds<CAP> &L) {
    for (int s = lane_id(); s < CAP; s += AGN_WAVE) L.head[s] = NIL;
    wave_sync();
}

template <int CAP>
__device__ __forceinline__ void link(CandLds<CAP> &L, uint32_t s, uint64_t t) {
    const uint32_t prev = atomicExch(&L.head[hbucket<CAP>(t)], s);
    L.nxt[s] = (uint16_t)prev;  // NIL -> 0xffff
}

// Stable in-place compaction of the live candidates [0, used); returns the
// live count.  With relink, the hash chains are rebuilt.
template <int CAP>
__device__ __forceinline__ uint32_t compact(CandLds<CAP> &L, uint32_t used, bool relink) {
    const int lane = lane_id();
    const uint64_t lt = lanes_below();
    uint32_t n = 0;
    for (uint32_t s0 = 0; s0 < used; s0 += AGN_WAVE) {
        const uint32_t s = s0 + (uint32_t)lane;
        uint64_t t = 0;
        uint32_t g = 0, o = DEAD;
        if (s < used) {
            t = L.tok[s];
            g = L.tag[s];
            o = L.ord[s];
        }
        const bool live = !(o & DEAD);
        const uint64_t m = ballot(live);
        wave_sync();  // every read of this chunk before any write
        if (live) {
            const uint32_t d = n + (uint32_t)__builtin_popcountll(m & lt);
            L.tok[d] = t;
            L.tag[d] = g;
            L.ord[d] = o;
        }
        n += (uint32_t)__builtin_popcountll(m);
        wave_sync();
    }
    if (relink) {
        heads_clear<CAP>(L);
        for (uint32_t s = lane; s < n; s += AGN_WAVE) link<CAP>(L, s, L.tok[s]);
        wave_sync();
    }
    return n;
}

// (tag, ord) for set_aw, (tag, tok) for register_mv
template <bool SET>
__device__ __forceinline__ bool key_less(uint32_t ta, uint64_t ka, uint32_t oa, uint32_t tb,
                                         uint64_t kb, uint32_t ob) {
    if (ta != tb) return ta < tb;
    if (SET) return oa < ob;
    return ka < kb;
}

template <bool SET, int CAP>
__device__ __forceinline__ void bitonic(CandLds<CAP> &L, uint32_t n) {
    const int lane = lane_id();
    uint32_t M = 1;
    while (M < n) M <<= 1;
    for (uint32_t s = n + lane; s < M; s += AGN_WAVE) {  // pad with +inf
        L.tag[s] = 0xffffffffu;
        L.tok[s] = ~0ull;
        L.ord[s] = 0xffffffffu;
    }
    wave_sync();
    for (uint32_t k = 2; k <= M; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = lane; t < (M >> 1); t += AGN_WAVE) {
                const uint32_t a = 2u * j * (t / j) + (t % j);
                const uint32_t b = a + j;
                const bool up = (a & k) == 0u;
                const uint32_t ta = L.tag[a], tb = L.tag[b];
                const uint64_t ka = L.tok[a], kb = L.tok[b];
                const uint32_t oa = L.ord[a], ob = L.ord[b];
                const bool swap = up ? key_less<SET>(tb, kb, ob, ta, ka, oa)
                                     : key_less<SET>(ta, ka, oa, tb, kb, ob);
                if (swap) {
                    L.tag[a] = tb; L.tok[a] = kb; L.ord[a] = ob;
                    L.tag[b] = ta; L.tok[b] = ka; L.ord[b] = oa;
                }
            }
            wave_sync();
        }
    }
}

// Per-entry fields of one 64-entry chunk (lane = entry).
struct Side {
    uint32_t tag, ro0, ro1, id, id_prev;
    uint64_t add;
};

__device__ __forceinline__ Side load_side(const agn_log &log, uint64_t off, uint64_t n,
                                          uint64_t c0) {
    const uint64_t pos = c0 + (uint64_t)lane_id();
    const uint64_t p = pos < n ? pos : n - 1;  // clamped: unconditional loads
    const uint64_t e = off + p;
    Side s;
    s.tag = log.tag[e];
    s.add = log.add_tok[e];
    s.ro0 = log.rem_off[e];
    s.ro1 = log.rem_off[e + 1];
    s.id = log.op_id[e];
    s.id_prev = log.op_id[p ? e - 1 : e];
    return s;
}


// CT ("contiguous rows", dense clocks with D = 4 LPO): a sub-iteration's OPI
// OpSSCommit rows (2 KiB) are read by two lane-contiguous 16-byte loads, 1 KiB
// each, non-temporal -- every instruction covers whole 128-byte lines, where
// the LPO-lanes-by-4-DCs loads cover half of each line per instruction.  Lane
// l holds DCs 2 (l % P), 2 (l % P) + 1 (P = D / 2 parts per op) of op l / P
// of each half; the per-op verdicts are group-any folds of wave ballots
// (scalar), LastOpCt stays per part until the end of the key.
// Work lists of one launch sequence: `in` (NULL: the batch) the requests this
// launch serves; keys whose live state overflows the fast table go to ovf;
// MSK: keys the dense scan cannot serve exactly go to mix (see MSK below).
struct TagLists {
    const uint32_t *in, *in_n;
    uint32_t *ovf, *ovf_n;
    uint32_t *mix, *mix_n;
};

// MSK (presence masks on a dense-loadable shape, D <= 64): per request the
// key's shared DC set U (agn_log.key_mask), R's and SCT's mask words; a key
// with U known and inside R runs the dense row scan with R and SCT at +inf
// outside U (so those columns never exclude an op nor keep it out of the
// snapshot, is_op_in_snapshot :236-258), SCT's missing DCs at 0, LastOpCt
// outside U kept at SCT's value and its DC set = SCT's | (U if any op was
// included).  Any other key goes to the `mix` list, served by the per-entry-
// mask (SPARSE) kernel in a second launch.
//
// SV (the fused set/register read, tags_serve.hpp; fast pass, WARM): the
// wave runs the snapshot cache's lookup for its request before the pass and
// the store after it; keys the pass hands on are stored by a later launch.
template <int DPL, int LPO, bool SPARSE, bool FULL, bool SET, int CAP, int WPB, int RB,
          bool WARM, bool SLOW, bool CT, bool MSK, bool SV = false>
__global__ __launch_bounds__(64 * WPB) void k_tags(agn_log log, agn_read req, agn_result out,
                                                   TagLists tl, uint32_t xcd, TagServe sv) {
    using S = Shape<DPL, LPO>;
    constexpr int OPI = S::OPI;
    static_assert(!CT || (DPL == 4 && FULL && !SPARSE), "CT: dense rows, 4 DCs per lane");
    static_assert(!MSK || (FULL && !SPARSE), "MSK: the dense row scans");
    static_assert(!SV || (WARM && !SLOW && DPL * LPO <= 64), "SV: the fast pass, D <= 64");
    constexpr int SVD = DPL * LPO;  // SV: the LastOpCt stash's row width (>= D), mask word after it
    constexpr int P = CT ? DPL * LPO / 2 : 1;  // 16-byte parts per op
    constexpr int OPH = AGN_WAVE / P;          // ops per 1 KiB load (OPI / 2)
    __shared__ CandLds<CAP> Lall[WPB];
    __shared__ uint64_t Sct[WPB][SV ? SVD + 1 : 1];  // SV: LastOpCt row + mask word for the store
    const int w = (WPB == 1) ? 0 : (int)(threadIdx.x >> 6);
    CandLds<CAP> &L = Lall[w];
    const int lane = lane_id();
    const int sub = lane % LPO, slot = lane / LPO, d0 = sub * DPL;
    const uint32_t D = log.n_dcs, W = n_words(D);
    const uint64_t lt = lanes_below();
    const uint64_t n_items = tl.in ? (uint64_t)__builtin_amdgcn_readfirstlane(ldc(tl.in_n)) : req.n_req;
    const uint64_t nw = (uint64_t)gridDim.x * WPB;

    const uint32_t blk = block_order(xcd, blockIdx.x, gridDim.x);
    for (uint64_t it = (uint64_t)blk * WPB + (uint64_t)w; it < n_items; it += nw) {
        // the per-request / per-key words below are read through the scalar
        // cache (ldc: arrays this launch never writes); as plain loads in the
        // grid-stride loop, whose stores may alias them, they were vector
        // loads waited for one by one before the rows issued
        const uint64_t i = tl.in ? (uint64_t)__builtin_amdgcn_readfirstlane(ldc(tl.in + it)) : it;
        const uint64_t key = req.keys ? uniform_u64(ldc(req.keys + i)) : i;
        LookupOut lk{};
        if constexpr (SV) {
            // get_from_snapshot_cache (materializer_vnode.erl:384-413) on the
            // whole wave: SCT row (+ mask) and base reference into sv's arrays,
            // which req.sct / sct_mask / base_value name for the reads below
            const Grp<AGN_WAVE> g;
            lk = ss_lookup_one<AGN_WAVE>(g, sv.c, key, req.R + i * D,
                                         req.R_mask ? req.R_mask + i * W : nullptr, sv.sct + i * D,
                                         sv.sctm ? sv.sctm + i * W : nullptr);
            if (lane == 0) {
                sv.ign[i] = lk.ign;
                sv.base[i] = lk.base;
                sv.first[i] = lk.first;
                sv.status[i] = lk.status;
                sv.dkeys[i] = key;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // other lanes read the rows
        }
        // hand-on / no-store outcomes of SV (lane 0): prune[i] and the deltas
        auto sv_mark = [&](uint8_t pf) {
            if (SV && lane == 0) {
                sv.prune[i] = pf;
                sv.dprune[i] = 0;
                sv.delta[2 * i] = 0;
                sv.delta[2 * i + 1] = 0;
            }
        };
        // The key's and the request's side values load together and
        // unconditionally (in-bounds dummies for absent columns): each
        // conditional load was waited for on its own before the next issued.
        const uint64_t *lenp = log.key_len ? log.key_len + key : log.key_off + key + 1;
        const uint64_t off = uniform_u64(ldc(log.key_off + key));
        const uint64_t lv = uniform_u64(ldc(lenp));
        const uint32_t kt = ldc_byte(
            log.key_type ? log.key_type : reinterpret_cast<const uint8_t *>(log.key_off), key);
        const uint32_t si = SV ? (uint32_t)lk.ign : ldc_byte(
            req.sct_ignore ? req.sct_ignore : reinterpret_cast<const uint8_t *>(req.R), i);
        const uint64_t txv = uniform_u64(ldc((req.txid ? req.txid : req.R) + i));
        // base state: CSR base_off, or AGN_SS_STATE(start, pairs) in
        // base_value (a snapshot cache's state arena, agn_ss_lookup)
        const bool packed = req.base_off == nullptr && req.base_value != nullptr;
        const uint64_t *bop = req.base_off ? req.base_off + i
                            : packed        ? reinterpret_cast<const uint64_t *>(req.base_value) + i
                                            : req.R + i;
        // SV: the lookup above wrote base_value (lk.base); otherwise read-only
        const uint64_t b0v = SV ? (uint64_t)lk.base : uniform_u64(ldc(bop));
        const uint64_t b1v = req.base_off ? uniform_u64(ldc(bop + 1)) : 0ull;
        const uint64_t n = log.key_len ? lv : lv - off;

        uint64_t kmw = 0, rmw = 0, smw = 0;
        if constexpr (MSK) {
            kmw = uniform_u64(ldc(log.key_mask ? log.key_mask + key : req.R));
            rmw = uniform_u64(ldc(req.R_mask ? req.R_mask + i : req.R));
            // SV: the lookup above wrote the SCT mask word (sv.sctm)
            const uint64_t *smp = (req.sct && req.sct_mask) ? req.sct_mask + i : req.R;
            smw = uniform_u64(SV ? *smp : ldc(smp));
        }

        if (n != 0 && log.key_type != nullptr && kt != (uint32_t)(uint8_t)req.req_type) {
            if (lane == 0) {  // erlang:error(corrupted_ops_cache) (:190-191)
                out.flags[i] = AGN_F_ERR_CORRUPTED;
                out.err_pos[i] = 0xffffffffu;
                out.out_n[i] = 0;
            }
            sv_mark(0);  // not stored (materialize_snapshot sees the error)
            continue;
        }
        // MSK: the key's DC set U, R's and SCT's (see above)
        const uint64_t FULLW = low_bits(D);
        const uint64_t mU = !MSK ? FULLW : log.oc_mask ? (log.key_mask ? (kmw & FULLW) : 0ull) : FULLW;
        const uint64_t mR = (MSK && req.R_mask) ? (rmw & FULLW) : FULLW;
        const uint64_t mS = (MSK && req.sct && req.sct_mask) ? (smw & FULLW) : FULLW;
        if (MSK && !(n == 0 || (mU != 0ull && (mU & ~mR) == 0ull))) {
            if (lane == 0) {
                const uint32_t at = atomicAdd(tl.mix_n, 1u);
                tl.mix[at] = (uint32_t)i;
            }
            sv_mark(4);
            continue;
        }

        // ---- read snapshot R, base snapshot time SCT, LastOpCt seed
        const bool sct_ign = !WARM || req.sct == nullptr || (req.sct_ignore && si != 0u);
        const uint64_t *sctp = req.sct ? req.sct : req.R;
        const uint32_t rbits = chunk_bits<DPL, SPARSE>(req.R_mask, i, W, d0, D);
        const uint32_t sbits = sct_ign ? 0u : chunk_bits<DPL, SPARSE>(req.sct_mask, i, W, d0, D);
        uint64_t r[DPL], s[DPL], ct[DPL], e[DPL];
#pragma unroll
        for (int j = 0; j < DPL; ++j) {
            const uint32_t d = (uint32_t)(d0 + j);
            const uint32_t dd = d < D ? d : D - 1u;
            const uint64_t rv = req.R[i * D + dd];
            const uint64_t sv = WARM ? sctp[i * D + dd] : 0ull;
            r[j] = (d < D) ? rv : 0ull;
            s[j] = ((sbits >> j) & 1u) ? sv : 0ull;
            // LastOpCt starts as SnapshotCommitTime (materialize/4 :94-95);
            // "+1 encoded" in sparse mode (0 = DC absent from the dict)
            ct[j] = ((sbits >> j) & 1u) ? (SPARSE ? s[j] + 1ull : s[j]) : 0ull;
            if constexpr (MSK) {  // dict read of SCT; +inf outside U
                const bool inU = d < D && ((mU >> (d & 63u)) & 1ull);
                e[j] = (sct_ign || d >= D || !((mS >> (d & 63u)) & 1ull)) ? 0ull : sv;
                ct[j] = e[j];
                s[j] = inU ? e[j] : ~0ull;
                r[j] = inU ? r[j] : ~0ull;
            }
        }
        const uint64_t txr = req.txid ? txv : 0ull;
        const bool use_tx = txr != 0ull && log.txid != nullptr;
        // CT: this lane's parts of R / SCT / LastOpCt (DCs dp, dp + 1)
        uint64_t rA = 0, rB = 0, sA = 0, sB = 0, ctA = 0, ctB = 0, eA = 0, eB = 0;
        bool uA = true, uB = true;  // MSK: this lane's DCs are in U
        if constexpr (CT) {
            const uint32_t dp = 2u * (uint32_t)(lane % P);
            rA = req.R[i * D + dp];
            rB = req.R[i * D + dp + 1];
            if constexpr (WARM) {
                const uint64_t xa = sctp[i * D + dp], xb = sctp[i * D + dp + 1];
                sA = sct_ign ? 0ull : xa;
                sB = sct_ign ? 0ull : xb;
            }
            if constexpr (MSK) {
                uA = ((mU >> (dp & 63u)) & 1ull) != 0ull;
                uB = ((mU >> ((dp + 1u) & 63u)) & 1ull) != 0ull;
                sA = ((mS >> (dp & 63u)) & 1ull) ? sA : 0ull;
                sB = ((mS >> ((dp + 1u) & 63u)) & 1ull) ? sB : 0ull;
                eA = sA;
                eB = sB;
                rA = uA ? rA : ~0ull;
                rB = uB ? rB : ~0ull;
                sA = uA ? sA : ~0ull;
                sB = uB ? sB : ~0ull;
            }
            ctA = MSK ? eA : sA;
            ctB = MSK ? eB : sB;
        }

        // ---- base snapshot state: candidates with ord = index (< B)
        heads_clear<CAP>(L);
        const uint64_t b0 = req.base_off ? b0v : packed ? AGN_SS_STATE_START(b0v) : 0ull;
        const uint32_t B = req.base_off ? (uint32_t)(b1v - b0v)
                         : packed        ? AGN_SS_STATE_PAIRS(b0v)
                                         : 0u;
        bool overflow = B > (uint32_t)(CAP - AGN_WAVE);
        uint32_t used = 0;
        if (!overflow) {
            for (uint32_t x = lane; x < B; x += AGN_WAVE) {
                const uint64_t t = req.base_tok[b0 + x];
                L.tok[x] = t;
                L.tag[x] = req.base_tag[b0 + x];
                L.ord[x] = x;
                link<CAP>(L, x, t);
            }
            used = B;
        }
        wave_sync();

        int64_t first_excl = -1, first_err = -1, hid = 0;
        uint32_t cnt = 0;

        if (n != 0) {
            Side side = load_side(log, off, n, 0);
            uint64_t nx[DPL];
            uint32_t nxbits = 0;
            u64x2 cx0, cx1;  // CT: the next sub-iteration's two 1 KiB halves
            const u64x2 *rows16 = reinterpret_cast<const u64x2 *>(log.oc);
            const uint64_t ue = (off + n) * (uint64_t)P - 1u;  // the key's last 16-byte unit
            auto load_ct = [&](uint64_t sb) {
                const uint64_t u = (off + sb) * (uint64_t)P + (uint64_t)lane;
                cx0 = __builtin_nontemporal_load(rows16 + (u < ue ? u : ue));
                cx1 = __builtin_nontemporal_load(rows16 + (u + AGN_WAVE < ue ? u + AGN_WAVE : ue));
            };
            if constexpr (CT) {
                load_ct(0);
            } else {
                const uint64_t p = (uint64_t)slot < n ? (uint64_t)slot : n - 1;
                load_rows<DPL, SPARSE, FULL>(log, off + p, d0, D, W, nx, nxbits);
            }
            for (uint64_t c0 = 0; c0 < n; c0 += AGN_WAVE) {
                const uint64_t left = n - c0;
                const uint32_t nvalid = left < AGN_WAVE ? (uint32_t)left : (uint32_t)AGN_WAVE;
                const Side cs = side;
                // the chunk's removal tokens, first RB*64 of them
                const uint32_t K0 = __builtin_amdgcn_readfirstlane(cs.ro0);
                const uint32_t K1 = __builtin_amdgcn_readlane(cs.ro1, nvalid - 1);
                uint64_t rt[RB];
#pragma unroll
                for (int q = 0; q < RB; ++q) rt[q] = 0ull;
                if (K1 > K0) {  // rem_tok may be empty (NULL) for a log without removals
#pragma unroll
                    for (int q = 0; q < RB; ++q) {
                        const uint32_t k = K0 + (uint32_t)(q * AGN_WAVE + lane);
                        rt[q] = log.rem_tok[k < K1 ? k : K1 - 1u];
                    }
                }

                // ---- snapshot filter over the chunk's sub-iterations
                const uint32_t nsub = (nvalid + OPI - 1) / OPI;
                bool incl_e = false;
                for (uint32_t j = 0; j < nsub && CT; ++j) {
                    const u64x2 o0 = cx0, o1 = cx1;
                    const uint64_t b = c0 + (uint64_t)j * OPI;
                    const uint64_t nb = (j + 1 < nsub) ? b + OPI : c0 + AGN_WAVE;
                    if (j + 1 == nsub) side = load_side(log, off, n, nb < n ? nb : c0);
                    load_ct(nb < n ? nb : n - 1);
                    const uint64_t vm = low_bits(n - b < (uint64_t)OPI ? n - b : (uint64_t)OPI);
                    const uint64_t bad = group_any<P>(ballot(o0.x > rA || o0.y > rB)) |
                                         (group_any<P>(ballot(o1.x > rA || o1.y > rB)) << OPH);
                    uint64_t nipm = ~0ull;  // belongs_to_snapshot_op(SCT, ...)
                    if (WARM && !sct_ign)
                        nipm = group_any<P>(ballot(o0.x > sA || o0.y > sB)) |
                               (group_any<P>(ballot(o1.x > sA || o1.y > sB)) << OPH);
                    if (use_tx) {  // or (TxId == op.txid)  (:219-220)
                        const bool tv = lane < OPI && b + (uint64_t)lane < n &&
                                        log.txid[off + b + (uint64_t)lane] == txr;
                        nipm |= ballot(tv);
                    }
                    const uint64_t inc = vm & nipm & ~bad, exc = vm & nipm & bad;
                    if (first_excl < 0 && exc) {
                        first_excl = (int64_t)b + (int64_t)__builtin_ctzll(exc);
                        // its op id is in the chunk's side fields: no dependent load
                        hid = (int64_t)(uint32_t)__shfl((int)cs.id, (int)(first_excl - (int64_t)c0));
                    }
                    const int q = lane / P;
                    if ((inc >> q) & 1ull) {
                        ctA = umax64(ctA, o0.x);
                        ctB = umax64(ctB, o0.y);
                    }
                    if ((inc >> (q + OPH)) & 1ull) {
                        ctA = umax64(ctA, o1.x);
                        ctB = umax64(ctB, o1.y);
                    }
                    // per-op verdict -> lane = entry
                    if ((uint32_t)lane / (uint32_t)OPI == j)
                        incl_e = (inc >> ((uint32_t)lane % (uint32_t)OPI)) & 1ull;
                }
                for (uint32_t j = 0; j < nsub && !CT; ++j) {
                    uint64_t o[DPL];
                    const uint32_t obits0 = nxbits;
#pragma unroll
                    for (int x = 0; x < DPL; ++x) o[x] = nx[x];
                    const uint64_t b = c0 + (uint64_t)j * OPI;
                    const uint64_t nb = (j + 1 < nsub) ? b + OPI : c0 + AGN_WAVE;
                    if (j + 1 == nsub) side = load_side(log, off, n, nb < n ? nb : c0);
                    {
                        const uint64_t p = nb + (uint64_t)slot;
                        load_rows<DPL, SPARSE, FULL>(log, off + (p < n ? p : n - 1), d0, D, W,
                                                     nx, nxbits);
                    }
                    const uint64_t pos = b + (uint64_t)slot;
                    const bool valid = pos < n;
                    const uint32_t obits = valid ? obits0 : 0u;
                    bool okR = true, leS = true;
#pragma unroll
                    for (int x = 0; x < DPL; ++x) {
                        if ((obits >> x) & 1u) {
                            const bool inR = SPARSE ? (((rbits >> x) & 1u) != 0u) : true;
                            okR = okR && inR && (o[x] <= r[x]);  // DC missing in R -> false
                            if (WARM) leS = leS && (o[x] <= s[x]);
                        }
                    }
                    if (LPO > 1) {
                        const uint64_t grp = ((1ull << LPO) - 1ull) << (slot * LPO);
                        okR = (ballot(!okR) & grp) == 0ull;
                        if (WARM) leS = (ballot(!leS) & grp) == 0ull;
                    }
                    // belongs_to_snapshot_op(SCT, ...) or (TxId == op.txid)  (:219-220)
                    bool nip = sct_ign || !leS;
                    if (use_tx) {
                        bool txm = valid && sub == 0 && log.txid[off + pos] == txr;
                        if (LPO > 1) txm = (ballot(txm) >> (slot * LPO)) & 1ull;
                        nip = nip || txm;
                    }
                    const bool incl = valid && nip && okR;
                    const bool excl = valid && nip && !okR;
                    if (first_excl < 0) {
                        const uint64_t bx = ballot(excl && sub == 0);
                        if (bx) {
                            first_excl = (int64_t)b + (int64_t)(__builtin_ctzll(bx) / LPO);
                            // its op id is in the chunk's side fields: no dependent load
                            hid = (int64_t)(uint32_t)__shfl((int)cs.id,
                                                            (int)(first_excl - (int64_t)c0));
                        }
                    }
                    if (incl) {
#pragma unroll
                        for (int x = 0; x < DPL; ++x)
                            if ((obits >> x) & 1u)
                                ct[x] = umax64(ct[x], SPARSE ? o[x] + 1ull : o[x]);
                    }
                    // per-op verdict -> lane = entry
                    const uint64_t bi = ballot(incl && sub == 0);
                    if ((uint32_t)lane / (uint32_t)OPI == j)
                        incl_e = (bi >> (((uint32_t)lane % (uint32_t)OPI) * LPO)) & 1ull;
                }

                if (first_excl < 0 && c0 + AGN_WAVE >= n)  // get_first_id (:49-63)
                    hid = (int64_t)(uint32_t)__shfl((int)cs.id, (int)(nvalid - 1u));
                // ---- chunk resolution (lane = entry c0 + lane)
                const uint64_t pos = c0 + (uint64_t)lane;
                const bool opstart = pos == 0 || cs.id_prev != cs.id;
                cnt += (uint32_t)__builtin_popcountll(ballot(incl_e && opstart));
                if (first_err < 0) {
                    const uint64_t be = ballot(incl_e && cs.tag == AGN_TAG_INVALID);
                    if (be) first_err = (int64_t)c0 + (int64_t)__builtin_ctzll(be);
                }
                if (first_err >= 0 || overflow) continue;  // {error,..} / no state kept

                // (1) candidates: the chunk's included adds, in position order
                const bool adds = incl_e && cs.add != 0ull;
                const uint64_t am = ballot(adds);
                const uint32_t n_add = (uint32_t)__builtin_popcountll(am);
                if (used + n_add > (uint32_t)CAP) {
                    used = compact<CAP>(L, used, true);
                    if (used + n_add > (uint32_t)CAP) {
                        overflow = true;
                        continue;
                    }
                }
                if (adds) {
                    const uint32_t sl = used + (uint32_t)__builtin_popcountll(am & lt);
                    L.tok[sl] = cs.add;
                    L.tag[sl] = cs.tag;
                    L.ord[sl] = B + (uint32_t)pos;
                    link<CAP>(L, sl, cs.add);
                }
                used += n_add;
                wave_sync();

                // (2) removals: lane = removal token; owner entry by binary
                // search over the chunk's removal offsets
                const uint64_t im = ballot(incl_e);
                for (uint32_t k0 = K0, q = 0; k0 < K1; k0 += AGN_WAVE, ++q) {
                    const uint32_t k = k0 + (uint32_t)lane;
                    const bool has = k < K1;
                    uint64_t t;
                    if (q < (uint32_t)RB) {
                        t = rt[0];
#pragma unroll
                        for (int z = 1; z < RB; ++z)
                            if (q == (uint32_t)z) t = rt[z];
                    } else {
                        t = has ? log.rem_tok[k] : 0ull;
                    }
                    uint32_t sidx = 0;
#pragma unroll
                    for (uint32_t st = AGN_WAVE / 2; st > 0; st >>= 1) {
                        const uint32_t c = sidx + st;
                        const uint32_t v = (uint32_t)__shfl((int)cs.ro0, (int)(c & 63u));
                        if (c < nvalid && v <= k) sidx = c;
                    }
                    const uint32_t etag = (uint32_t)__shfl((int)cs.tag, (int)sidx);
                    const bool einc = (im >> sidx) & 1ull;
                    if (has && einc) {
                        const uint32_t qpos = B + (uint32_t)(c0 + sidx);
                        for (uint32_t x = L.head[hbucket<CAP>(t)]; x != NIL; x = chain_next(L, x)) {
                            if (L.tok[x] != t) continue;
                            if (SET && L.tag[x] != etag) continue;
                            const uint32_t o = L.ord[x];
                            if (qpos > (o & ~DEAD)) L.ord[x] = o | DEAD;
                        }
                    }
                }
                wave_sync();
            }
        }

        // ---- fast path overflow: hand the key to the 4096-slot pass
        if (!SLOW && overflow && first_err < 0) {
            if (lane == 0) {
                const uint32_t at = atomicAdd(tl.ovf_n, 1u);
                tl.ovf[at] = (uint32_t)i;
            }
            sv_mark(4);
            continue;
        }

        // ---- live state -> sorted pairs
        uint32_t n_live = 0;
        bool cap_err = overflow;
        const uint64_t o = out.out_off[i];
        if (!overflow && first_err < 0) {
            n_live = compact<CAP>(L, used, false);
            if ((uint64_t)n_live > out.out_off[i + 1] - o) {
                cap_err = true;
            } else {
                bitonic<SET, CAP>(L, n_live);
                for (uint32_t x = lane; x < n_live; x += AGN_WAVE) {
                    out.out_tag[o + x] = L.tag[x];
                    out.out_tok[o + x] = L.tok[x];
                }
            }
        }
        wave_sync();

        // ---- LastOpCt: max over the lanes that hold the same DC slice
        const bool ct_ign = sct_ign && cnt == 0u;
        if constexpr (MSK) {  // outside U: SCT's value (an op's row there is not in its dict)
            ctA = uA ? ctA : eA;
            ctB = uB ? ctB : eB;
#pragma unroll
            for (int j = 0; j < DPL; ++j) {
                const uint32_t d = (uint32_t)(d0 + j);
                ct[j] = (d < D && ((mU >> (d & 63u)) & 1ull)) ? ct[j] : e[j];
            }
            const uint64_t ctm = ct_ign ? 0ull : ((sct_ign ? 0ull : mS) | (cnt ? mU : 0ull));
            if (out.lastct_mask != nullptr && lane == 0) out.lastct_mask[i] = ctm;
            if (SV && lane == 0) Sct[w][SV ? SVD : 0] = ctm;
        }
        if constexpr (CT) {
#pragma unroll
            for (int x = P; x < AGN_WAVE; x <<= 1) {
                ctA = umax64(ctA, shfl_xor_u64(ctA, x));
                ctB = umax64(ctB, shfl_xor_u64(ctB, x));
            }
            if (lane < P) {
                u64x2 v;
                v.x = ct_ign ? 0ull : ctA;
                v.y = ct_ign ? 0ull : ctB;
                reinterpret_cast<u64x2 *>(out.lastct + i * D)[lane] = v;
                if (SV) {
                    Sct[w][SV ? 2 * lane : 0] = v.x;
                    Sct[w][SV ? 2 * lane + 1 : 0] = v.y;
                }
            }
        } else {
#pragma unroll
        for (int x = LPO; x < AGN_WAVE; x <<= 1) {
#pragma unroll
            for (int j = 0; j < DPL; ++j) ct[j] = umax64(ct[j], shfl_xor_u64(ct[j], x));
        }
        if (slot == 0) {
#pragma unroll
            for (int j = 0; j < DPL; ++j) {
                const uint32_t d = (uint32_t)(d0 + j);
                if (d < D) {
                    uint64_t v = ct[j];
                    if (SPARSE) v = (v && !ct_ign) ? v - 1ull : 0ull;
                    else if (ct_ign) v = 0ull;
                    out.lastct[i * D + d] = v;
                    if (SV) Sct[w][SV ? d : 0] = v;
                }
            }
        }
        }
        if (SPARSE && out.lastct_mask != nullptr) {
            uint64_t part = 0;
            if (slot == 0 && !ct_ign) {
#pragma unroll
                for (int j = 0; j < DPL; ++j)
                    if ((uint32_t)(d0 + j) < D && ct[j] != 0ull)
                        part |= 1ull << ((uint32_t)(d0 + j) & 63u);
            }
            for (uint32_t wd = 0; wd < W; ++wd) {
                uint64_t v = (((uint32_t)d0 >> 6) == wd) ? part : 0ull;
#pragma unroll
                for (int x = 1; x < AGN_WAVE; x <<= 1) v |= shfl_xor_u64(v, x);
                if (lane == 0) out.lastct_mask[i * W + wd] = v;
                if (SV && lane == 0 && wd == 0) Sct[w][SV ? SVD : 0] = v;
            }
        }

        // wave-uniform
        const int64_t hole = first_excl >= 0 ? hid - 1 : hid;  // hid = 0 for n = 0
        uint32_t fl = 0;
        if (cnt) fl |= AGN_F_NEWSS;
        if (ct_ign) fl |= AGN_F_CT_IGNORE;
        if (first_err >= 0) fl |= AGN_F_ERR_UNEXPECTED;
        if (cap_err) fl |= AGN_F_ERR_CAPACITY;
        if constexpr (SV) {
            // materialize_snapshot's store (:466-509): the state from the LDS
            // table (sorted, [0, n_live)), LastOpCt from its stash
            wave_sync();
            const Grp<AGN_WAVE> g;
            uint64_t dl[3] = {0ull, 0ull, 0ull};
            const bool pr = ss_store_one<AGN_WAVE>(
                g, sv.c, key, n, lk.status, lk.first, sv.gc != nullptr && sv.gc[i] != 0, Sct[w],
                ((MSK || SPARSE) && out.lastct_mask != nullptr) ? &Sct[w][SV ? SVD : 0] : nullptr,
                hole, 0, cnt,
                fl, sv.thr, sv.thrm, L.tag, L.tok, n_live, dl);
            if (lane == 0) {
                sv.prune[i] = (uint8_t)((pr ? 1u : 0u) | (dl[2] ? 2u : 0u));
                sv.dprune[i] = pr ? 1 : 0;
                sv.delta[2 * i] = dl[0];
                sv.delta[2 * i + 1] = dl[1];
            }
        }
        if (lane == 0) {
            out.hole[i] = hole;
            out.count[i] = cnt;
            out.flags[i] = fl;
            out.err_pos[i] =
                first_err >= 0 ? (uint32_t)(off + (uint64_t)first_err) : 0xffffffffu;
            out.out_n[i] = n_live;
        }
    }
}

// The tags pass's block order.  A bulk batch (>= 2^16 keys, one wave per
// block) runs in runs of 128 blocks per XCD: cfg3 6.45 against 6.64 / 6.81
// ms in the XCD-aware order, cfg4 8.87 against 9.07 in the identity order
// (profiles/r06/ab_xcd_chunk.log).  Smaller batches and list passes keep
// the XCD-aware order up to 32 DCs, the identity order for wider clocks
// (cfg4: 9.08 against 9.25 ms, profiles/r06/ab_xcd_remap.log).
// AGN_XCD_REMAP / AGN_XCD_CHUNK override (order_or).
inline uint32_t tags_order(uint32_t D, uint64_t n_req, bool list) {
    return order_or(!list && n_req >= (1ull << 16) ? 128u : D <= 32 ? 1u : 0u);
}

// FAST_WPB: one wave per block measured 0.7-1.4 % faster than 4 (cfg3/cfg4,
// profiles/r01/ab_tags_wpb_unbiased.log)
constexpr int FAST_CAP = 256, SLOW_CAP = 4096, FAST_WPB = 1, RBATCH = 2;

// One fast pass (grid = the batch, or a resident grid over a list) and the
// 4096-slot pass over its overflow list.  `in` / `in_n`: the requests (NULL =
// the batch); lists: the scratch of the launch sequence.
template <int DPL, int LPO, bool SPARSE, bool FULL, bool SET, bool WARM, bool CT, bool MSK>
hipError_t tags_passes(const agn_log &log, const agn_read &req, const agn_result &out,
                       const uint32_t *in, const uint32_t *in_n, uint32_t *ovf, uint32_t *ovf_n,
                       uint32_t *mix, uint32_t *mix_n, hipStream_t st, bool run_fast = true) {
    // one wave per key: the grid is the batch (the wave dispatcher then
    // overlaps keys; AGN_TAGS_GRID=<blocks> caps it for A/B); a list pass
    // grid-strides over a resident grid
    const char *ge = AGN_KNOB("AGN_TAGS_GRID");
    const unsigned cap = in ? 8192u : ge ? (unsigned)atoi(ge) : 0x7fffffffu;
    const unsigned blocks = grid_for(req.n_req, FAST_WPB, cap);
    TagLists fast{in, in_n, ovf, ovf_n, mix, mix_n};
    if (run_fast) {  // (false: the fused read ran it, tags_serve.hpp)
        hipLaunchKernelGGL((k_tags<DPL, LPO, SPARSE, FULL, SET, FAST_CAP, FAST_WPB, RBATCH, WARM,
                                   false, CT, MSK>),
                           dim3(blocks), dim3(64 * FAST_WPB), 0, st, log, req, out, fast,
                           tags_order(log.n_dcs, req.n_req, in != nullptr), TagServe{});
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    // the overflow pass grid-strides over a list of at most n_req keys: a
    // resident grid of up to 256 one-wave blocks (88 KB of LDS each), no
    // more than the batch -- a serving batch of ~10 reads must not occupy
    // every CU's LDS, while other partitions' batches wait, to find the list
    // empty
    TagLists slow{ovf, ovf_n, nullptr, nullptr, mix, mix_n};
    const unsigned sblocks = (unsigned)(req.n_req < 256u ? (req.n_req ? req.n_req : 1u) : 256u);
    hipLaunchKernelGGL((k_tags<DPL, LPO, SPARSE, FULL, SET, SLOW_CAP, 1, RBATCH, WARM, true, CT,
                               MSK>),
                       dim3(sblocks), dim3(64), 0, st, log, req, out, slow, 0u, TagServe{});
    return hipGetLastError();
}

// Scratch of a launch sequence: [0] overflow count, [1] mixed-key count,
// [2] the mixed keys' overflow count, then three lists of n_req entries.
struct TagScratch {
    uint32_t *base = nullptr;
    uint64_t n = 0;
    uint32_t *ovf_n() const { return base; }
    uint32_t *mix_n() const { return base + 1; }
    uint32_t *ovf2_n() const { return base + 2; }
    uint32_t *ovf() const { return base + 4; }
    uint32_t *mix() const { return base + 4 + n; }
    uint32_t *ovf2() const { return base + 4 + 2 * n; }
};

template <int DPL, int LPO, bool SPARSE, bool FULL, bool SET, bool WARM, bool CT>
int launch_shape(const agn_log &log, const agn_read &req, const agn_result &out,
                 hipStream_t st) {
    TagScratch w;
    w.n = req.n_req;
    AGN_HIP(pool_malloc((void **)&w.base, (3 * req.n_req + 4) * sizeof(uint32_t), st));
    hipError_t e = hipMemsetAsync(w.base, 0, 4 * sizeof(uint32_t), st);
    if (e == hipSuccess)
        e = tags_passes<DPL, LPO, SPARSE, FULL, SET, WARM, CT, false>(
            log, req, out, nullptr, nullptr, w.ovf(), w.ovf_n(), w.mix(), w.mix_n(), st);
    const int rc = e == hipSuccess ? AGN_OK : fail(AGN_EHIP, "k_tags launch: %s", hipGetErrorString(e));
    const hipError_t ef = hipFreeAsync(w.base, st);
    if (rc == AGN_OK && ef != hipSuccess)
        return fail(AGN_EHIP, "hipFreeAsync: %s", hipGetErrorString(ef));
    return rc;
}

// Presence masks with a dense-loadable shape: the MSK dense passes, then the
// per-entry-mask (SPARSE) passes over the keys they handed on.
template <int DPL, int LPO, bool SET, bool WARM, bool CT, int SDPL, int SLPO>
int launch_masked(const agn_log &log, const agn_read &req, const agn_result &out, hipStream_t st) {
    TagScratch w;
    w.n = req.n_req;
    AGN_HIP(pool_malloc((void **)&w.base, (3 * req.n_req + 4) * sizeof(uint32_t), st));
    hipError_t e = hipMemsetAsync(w.base, 0, 4 * sizeof(uint32_t), st);
    if (e == hipSuccess)
        e = tags_passes<DPL, LPO, false, true, SET, WARM, CT, true>(
            log, req, out, nullptr, nullptr, w.ovf(), w.ovf_n(), w.mix(), w.mix_n(), st);
    if (e == hipSuccess)
        e = tags_passes<SDPL, SLPO, true, false, SET, WARM, false, false>(
            log, req, out, w.mix(), w.mix_n(), w.ovf2(), w.ovf2_n(), nullptr, nullptr, st);
    const int rc = e == hipSuccess ? AGN_OK : fail(AGN_EHIP, "k_tags launch: %s", hipGetErrorString(e));
    const hipError_t ef = hipFreeAsync(w.base, st);
    if (rc == AGN_OK && ef != hipSuccess)
        return fail(AGN_EHIP, "hipFreeAsync: %s", hipGetErrorString(ef));
    return rc;
}

// Contiguous row loads for dense clocks with 4 DCs per lane (k_tags CT);
// AGN_TAGS_CT=0 (A/B knob) keeps the LPO-lanes-by-4-DCs loads.
inline bool tags_ct() {
    const char *v = AGN_KNOB("AGN_TAGS_CT");
    return !(v && v[0] == '0');
}

template <int DPL, int LPO, bool SPARSE, bool SET>
int launch_full(const agn_log &log, const agn_read &req, const agn_result &out, hipStream_t st) {
    const bool warm = req.sct != nullptr;
    // FULL: dense rows that split exactly into 16-byte loads
    const bool full = !SPARSE && (DPL % 2 == 0) && log.n_dcs == (uint32_t)(DPL * LPO);
    if constexpr (!SPARSE && DPL == 4) {
        if (full && tags_ct())
            return warm ? launch_shape<DPL, LPO, false, true, SET, true, true>(log, req, out, st)
                        : launch_shape<DPL, LPO, false, true, SET, false, true>(log, req, out, st);
    }
    if constexpr (!SPARSE && DPL % 2 == 0) {
        if (full)
            return warm ? launch_shape<DPL, LPO, false, true, SET, true, false>(log, req, out, st)
                        : launch_shape<DPL, LPO, false, true, SET, false, false>(log, req, out, st);
    }
    (void)full;
    return warm ? launch_shape<DPL, LPO, SPARSE, false, SET, true, false>(log, req, out, st)
                : launch_shape<DPL, LPO, SPARSE, false, SET, false, false>(log, req, out, st);
}

// Dense clocks wider than 8 DCs run 4 DCs per lane: 83 VGPRs (5 waves/SIMD)
// against 116 (4 waves/SIMD) with 8 per lane -- cfg3 -3.8/-4.7 %, cfg4
// -0.7/-1.3 % on two boxes; 2 per lane (69 VGPRs, but LDS caps the CU at 22
// waves) lost 12 % / 9 % to the extra sub-iterations
// (profiles/r01/ab_tags_dpl.log).  AGN_TAGS_DPL8=1 (A/B knob) keeps 8.
inline bool tags_dpl8() {
    const char *v = AGN_KNOB("AGN_TAGS_DPL8");
    return v && v[0] == '1';
}

template <bool SPARSE, bool SET>
int dispatch(const agn_log &log, const agn_read &req, const agn_result &out, hipStream_t st) {
    if constexpr (!SPARSE) {
        const uint32_t D = log.n_dcs;
        if (D > 8 && D <= 128 && !tags_dpl8()) {
            if (D <= 16) return launch_full<4, 4, false, SET>(log, req, out, st);
            if (D <= 32) return launch_full<4, 8, false, SET>(log, req, out, st);
            if (D <= 64) return launch_full<4, 16, false, SET>(log, req, out, st);
            return launch_full<4, 32, false, SET>(log, req, out, st);
        }
    }
#define AGN_L(DPL, LPO) launch_full<DPL, LPO, SPARSE, SET>(log, req, out, st)
    AGN_DISPATCH_SHAPES(log.n_dcs, AGN_L)
#undef AGN_L
}

// A sparse batch whose width has a dense-loadable shape (D = 2, 4, 6, 8: one
// lane per op; 16, 32, 64: 4 DCs per lane, contiguous rows): AGN_ENOTSUP
// otherwise (the SPARSE kernel then serves every key).  AGN_TAGS_MSK=0 (A/B
// knob) disables it.
template <bool SET>
int dispatch_masked(const agn_log &log, const agn_read &req, const agn_result &out,
                    hipStream_t st) {
    const char *v = AGN_KNOB("AGN_TAGS_MSK");
    if (v && v[0] == '0') return AGN_ENOTSUP;
    const bool warm = req.sct != nullptr;
#define AGN_M(DPL, LPO, CTV, SD, SL)                                                         \
    return warm ? launch_masked<DPL, LPO, SET, true, CTV, SD, SL>(log, req, out, st)       \
                : launch_masked<DPL, LPO, SET, false, CTV, SD, SL>(log, req, out, st)
    switch (log.n_dcs) {
        case 2: AGN_M(2, 1, false, 2, 1);
        case 4: AGN_M(4, 1, false, 4, 1);
        case 6: AGN_M(6, 1, false, 6, 1);
        case 8: AGN_M(8, 1, false, 8, 1);
        case 16: if (tags_ct()) AGN_M(4, 4, true, 8, 2); break;
        case 32: if (tags_ct()) AGN_M(4, 8, true, 8, 4); break;
        case 64: if (tags_ct()) AGN_M(4, 16, true, 8, 8); break;
        default: break;
    }
#undef AGN_M
    return AGN_ENOTSUP;
}

// The fused set/register read (tags_serve.hpp): the SV fast pass over the
// batch; _rest: the passes and the store for the keys it handed on.
// Shapes (as launch_tags picks them for D <= 8): FULL dense rows (even D;
// D = 4 the CT form), the MSK form (masked, even D), non-FULL dense rows or
// the per-entry-mask (SPARSE) form for odd D.
// DPL x LPO: the pass's shape (D <= 8: one lane per op; 16, 32, 64: 4 DCs
// per lane, the CT rows); SDPL x SLPO: the per-entry-mask pass's for the keys
// the MSK form hands on.
template <int DPL, int LPO, int SDPL, int SLPO, bool SET, bool SPARSE, bool FULL, bool MSK, bool CT>
int serve_fast(const agn_log &log, const agn_read &req, const agn_result &out, const TagServe &sv,
               uint32_t *scr, hipStream_t st) {
    TagScratch w;
    w.base = scr;
    w.n = req.n_req;
    const TagLists fast{nullptr, nullptr, w.ovf(), w.ovf_n(), w.mix(), w.mix_n()};
    hipLaunchKernelGGL((k_tags<DPL, LPO, SPARSE, FULL, SET, FAST_CAP, FAST_WPB, RBATCH, true, false,
                               CT, MSK, true>),
                       dim3(grid_for(req.n_req, FAST_WPB, 0x7fffffffu)), dim3(64 * FAST_WPB), 0, st,
                       log, req, out, fast, 0u, sv);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

template <int DPL, int LPO, int SDPL, int SLPO, bool SET, bool SPARSE, bool FULL, bool MSK, bool CT>
int serve_rest(const agn_log &log, const agn_read &req, const agn_result &out, const TagServe &sv,
               uint32_t *scr, hipStream_t st) {
    TagScratch w;
    w.base = scr;
    w.n = req.n_req;
    hipError_t e = tags_passes<DPL, LPO, SPARSE, FULL, SET, true, CT, MSK>(
        log, req, out, nullptr, nullptr, w.ovf(), w.ovf_n(), w.mix(), w.mix_n(), st, false);
    if (MSK && e == hipSuccess)
        e = tags_passes<SDPL, SLPO, true, false, SET, true, false, false>(
            log, req, out, w.mix(), w.mix_n(), w.ovf2(), w.ovf2_n(), nullptr, nullptr, st);
    if (e != hipSuccess) return fail(AGN_EHIP, "k_tags launch: %s", hipGetErrorString(e));
    // the store for both lists (the mixed keys' overflow list is part of mix)
    for (int l = 0; l < (MSK ? 2 : 1); ++l) {
        const int rc = launch_ss_store_list(
            sv.c, log.key_off, log.key_len, req.n_req, l ? w.mix() : w.ovf(), l ? w.mix_n() : w.ovf_n(),
            sv.dkeys, sv.first, sv.status, sv.gc, out, sv.dprune, sv.thr, sv.thrm, st);
        if (rc) return rc;
    }
    AGN_HIP(hipMemsetAsync(scr, 0, 4 * sizeof(uint32_t), st));
    return AGN_OK;
}

template <bool REST, bool SET>
int serve_dispatch(const agn_log &log, const agn_read &req, const agn_result &out,
                   const TagServe &sv, uint32_t *scr, bool msk, hipStream_t st) {
#define AGN_SW(DPL, LPO, SD, SL, SPV, FULLV, MSKV, CTV)                                              \
    return REST ? serve_rest<DPL, LPO, SD, SL, SET, SPV, FULLV, MSKV, CTV>(log, req, out, sv, scr, st) \
                : serve_fast<DPL, LPO, SD, SL, SET, SPV, FULLV, MSKV, CTV>(log, req, out, sv, scr, st)
#define AGN_S(D, SPV, FULLV, MSKV, CTV) AGN_SW(D, 1, D, 1, SPV, FULLV, MSKV, CTV)
    if (msk) {
        switch (log.n_dcs) {
            case 1: AGN_S(1, true, false, false, false);
            case 2: AGN_S(2, false, true, true, false);
            case 3: AGN_S(3, true, false, false, false);
            case 4: AGN_S(4, false, true, true, false);
            case 5: AGN_S(5, true, false, false, false);
            case 6: AGN_S(6, false, true, true, false);
            case 7: AGN_S(7, true, false, false, false);
            case 8: AGN_S(8, false, true, true, false);
            // the masked shapes launch_tags picks (dispatch_masked): CT rows,
            // the per-entry-mask pass at 8 DCs per lane
            case 16: AGN_SW(4, 4, 8, 2, false, true, true, true);
            case 32: AGN_SW(4, 8, 8, 4, false, true, true, true);
            case 64: AGN_SW(4, 16, 8, 8, false, true, true, true);
            default: break;
        }
    } else {
        switch (log.n_dcs) {
            case 1: AGN_S(1, false, false, false, false);
            case 2: AGN_S(2, false, true, false, false);
            case 3: AGN_S(3, false, false, false, false);
            case 4: AGN_S(4, false, true, false, true);
            case 5: AGN_S(5, false, false, false, false);
            case 6: AGN_S(6, false, true, false, false);
            case 7: AGN_S(7, false, false, false, false);
            case 8: AGN_S(8, false, true, false, false);
            // dense wide clocks: 4 DCs per lane, contiguous (CT) rows (dispatch)
            case 16: AGN_SW(4, 4, 4, 4, false, true, false, true);
            case 32: AGN_SW(4, 8, 4, 8, false, true, false, true);
            case 64: AGN_SW(4, 16, 4, 16, false, true, false, true);
            default: break;
        }
    }
#undef AGN_S
#undef AGN_SW
    return AGN_ENOTSUP;
}

}  // namespace

// D <= 8 in the shape launch_tags picks: even D with the MSK form for masked
// logs (not with AGN_TAGS_MSK=0) and, dense, D = 4 in the CT form (not with
// AGN_TAGS_CT=0); odd D with the per-entry-mask or non-FULL dense rows;
// D = 16, 32, 64 in the CT form (4 DCs per lane), dense or MSK
bool tags_serve_supported(const agn_log &log, bool sparse) {
    const uint32_t D = log.n_dcs;
    if (D == 16 || D == 32 || D == 64) {  // the CT shapes, dense or MSK
        if (!tags_ct()) return false;
        const char *v = AGN_KNOB("AGN_TAGS_MSK");
        return !sparse || !(v && v[0] == '0');
    }
    if (D == 0 || D > 8) return false;
    if (D % 2) return true;
    if (sparse) {
        const char *v = AGN_KNOB("AGN_TAGS_MSK");
        return !(v && v[0] == '0');
    }
    return D != 4 || tags_ct();
}

static bool serve_masked(const agn_log &log, const agn_read &req, const agn_result &out) {
    return log.oc_mask || req.R_mask || req.sct_mask || out.lastct_mask;
}

int launch_tags_serve(const agn_log &log, const agn_read &req, const agn_result &out,
                      const TagServe &sv, uint32_t *scr, hipStream_t st) {
    if (req.n_req == 0) return AGN_OK;
    const bool msk = serve_masked(log, req, out);
    if (!tags_serve_supported(log, msk)) return AGN_ENOTSUP;
    return log.crdt_type == AGN_SET_AW ? serve_dispatch<false, true>(log, req, out, sv, scr, msk, st)
                                       : serve_dispatch<false, false>(log, req, out, sv, scr, msk, st);
}

int launch_tags_serve_rest(const agn_log &log, const agn_read &req, const agn_result &out,
                           const TagServe &sv, uint32_t *scr, hipStream_t st) {
    if (req.n_req == 0) return AGN_OK;
    const bool msk = serve_masked(log, req, out);
    if (!tags_serve_supported(log, msk)) return AGN_ENOTSUP;
    return log.crdt_type == AGN_SET_AW ? serve_dispatch<true, true>(log, req, out, sv, scr, msk, st)
                                       : serve_dispatch<true, false>(log, req, out, sv, scr, msk, st);
}

int launch_tags(const agn_log &log, const agn_read &req, const agn_result &out,
                hipStream_t st) {
    if (req.n_req == 0) return AGN_OK;
    // base_value without base_off names AGN_SS_STATE references into
    // base_tag / base_tok (ABI v4): both arrays are required for them
    if (!req.base_off && req.base_value && (!req.base_tag || !req.base_tok))
        return fail(AGN_EINVAL, "set/register read: base_value (state references) without base_tag/base_tok");
    const bool sparse = log.oc_mask || req.R_mask || req.sct_mask || out.lastct_mask;
    const bool set = log.crdt_type == AGN_SET_AW;
    if (sparse) {
        const int rc = set ? dispatch_masked<true>(log, req, out, st)
                           : dispatch_masked<false>(log, req, out, st);
        if (rc != AGN_ENOTSUP) return rc;
    }
    if (sparse) return set ? dispatch<true, true>(log, req, out, st)
                           : dispatch<true, false>(log, req, out, st);
    return set ? dispatch<false, true>(log, req, out, st) : dispatch<false, false>(log, req, out, st);
}

}  // namespace agn
