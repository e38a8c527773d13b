// mat_tags.hip — batched materialize/4 for antidote_crdt_set_aw and
// antidote_crdt_register_mv on gfx950: order-aware tag resolution.
//
// Reference fold (apply_operations, src/clocksi_materializer.erl:113-121,
// antidote_crdt 0.1.2 update/2, restated in SURVEY.md §8(a) a5.2/a5.3):
//   set_aw      entry {Elem, Add, Rem}: Tokens(Elem) := (Tokens -- Rem) ++ Add
//   register_mv entry {V, Tok, Ovr}: drop tokens in Ovr, insert_sorted({V, Tok})
//               entry {reset, Ovr}: drop tokens in Ovr
// applied oldest first.  Sequentially, a token t added at position p (or
// present in the base snapshot, p = -1) survives iff no INCLUDED op at a
// position q > p removes it (within one entry the removal happens before the
// add).  The kernel evaluates exactly that rule in one streaming pass, in
// position order, with an LDS token table per wave:
//   per iteration of OPI ops: (1) insert every included add as a candidate
//   {tok, tag, ord = B + p}; (2) every included removal (t, q) kills the
//   candidate t if q + B > ord (set_aw: and the elem matches).
// Removals of tokens added later are ignored (q < p), which is what the
// sequential fold does.  Dead candidates are tombstones; the table is
// compacted when 3/4 full (the live state, not the log length, bounds it).
// Output order: set_aw (elem, add order), register_mv (value, token) — the
// order the sequential fold produces; bitonic-sorted in LDS per key.
//
// HBM bytes per entry: 8*D (OpSSCommit) + 4 (op_id) + 4 (tag) + 8 (add_tok)
// + 4 (rem_off) + 8 per removed token; plus 12 per live output pair.
#include "filter.hpp"

namespace agn {
namespace {

constexpr uint32_t DEAD = 0x80000000u;

template <int CAP>
struct TagLds {
    uint64_t tok[CAP];
    uint32_t tag[CAP];
    uint32_t ord[CAP];
    // sort / compaction buffer; also aliased as the LastOpCt stage at the end
    uint64_t btok[CAP];
    uint32_t btag[CAP];
    uint32_t bord[CAP];
};

template <int CAP>
__device__ __forceinline__ uint32_t hslot(uint64_t t) {
    constexpr int LOG = __builtin_ctz(CAP);
    return (uint32_t)((t * 0x9E3779B97F4A7C15ull) >> (64 - LOG));
}

template <int CAP>
__device__ __forceinline__ void tab_insert(TagLds<CAP> &L, uint64_t t, uint32_t tag, uint32_t ord) {
    uint32_t h = hslot<CAP>(t);
    for (int probe = 0; probe < CAP; ++probe) {
        const uint64_t prev = atomicCAS((unsigned long long *)&L.tok[h], 0ull,
                                        (unsigned long long)t);
        if (prev == 0ull || prev == t) {
            L.tag[h] = tag;
            L.ord[h] = ord;  // a repeated token: the later add wins
            return;
        }
        h = (h + 1u) & (CAP - 1);
    }
}

template <int CAP>
__device__ __forceinline__ int tab_find(const TagLds<CAP> &L, uint64_t t) {
    uint32_t h = hslot<CAP>(t);
    for (int probe = 0; probe < CAP; ++probe) {
        const uint64_t k = L.tok[h];
        if (k == t) return (int)h;
        if (k == 0ull) return -1;
        h = (h + 1u) & (CAP - 1);
    }
    return -1;
}

// Gather live slots of the table into the buffer (stable in slot order);
// returns the number gathered (wave-uniform).
template <int CAP>
__device__ __forceinline__ uint32_t gather_live(TagLds<CAP> &L, int lane) {
    uint32_t n = 0;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int s0 = 0; s0 < CAP; s0 += AGN_WAVE) {
        const int s = s0 + lane;
        const uint64_t k = L.tok[s];
        const bool live = k != 0ull && !(L.ord[s] & DEAD);
        const uint64_t m = ballot(live);
        if (live) {
            const uint32_t at = n + (uint32_t)__builtin_popcountll(m & lt);
            L.btok[at] = k;
            L.btag[at] = L.tag[s];
            L.bord[at] = L.ord[s];
        }
        n += (uint32_t)__builtin_popcountll(m);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    return n;
}

template <int CAP>
__device__ __forceinline__ void tab_clear(TagLds<CAP> &L, int lane) {
    for (int s = lane; s < CAP; s += AGN_WAVE) {
        L.tok[s] = 0ull;
        L.ord[s] = 0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
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
__device__ __forceinline__ void bitonic(TagLds<CAP> &L, uint32_t n, int lane) {
    uint32_t M = 1;
    while (M < n) M <<= 1;
    for (uint32_t s = n + lane; s < M; s += AGN_WAVE) {  // pad with +inf
        L.btag[s] = 0xffffffffu;
        L.btok[s] = ~0ull;
        L.bord[s] = 0xffffffffu;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (uint32_t k = 2; k <= M; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = lane; t < (M >> 1); t += AGN_WAVE) {
                const uint32_t a = 2u * j * (t / j) + (t % j);
                const uint32_t b = a + j;
                const bool up = (a & k) == 0u;
                const uint32_t ta = L.btag[a], tb = L.btag[b];
                const uint64_t ka = L.btok[a], kb = L.btok[b];
                const uint32_t oa = L.bord[a], ob = L.bord[b];
                const bool swap = up ? key_less<SET>(tb, kb, ob, ta, ka, oa)
                                     : key_less<SET>(ta, ka, oa, tb, kb, ob);
                if (swap) {
                    L.btag[a] = tb; L.btok[a] = kb; L.bord[a] = ob;
                    L.btag[b] = ta; L.btok[b] = ka; L.bord[b] = oa;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
    }
}

template <int DPL, int LPO, bool SPARSE, bool SET, int CAP>
__global__ __launch_bounds__(64) void k_tags(agn_log log, agn_read req, agn_result out) {
    using F = KeyFilter<DPL, LPO, SPARSE>;
    static_assert(sizeof(uint64_t) * DPL * AGN_WAVE <= sizeof(uint64_t) * CAP * 2,
                  "stage must fit the sort buffer");
    __shared__ TagLds<CAP> L;
    const int lane = lane_id();
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    constexpr uint32_t HIGH = (uint32_t)(CAP * 3 / 4);

    for (uint64_t i = blockIdx.x; i < req.n_req; i += gridDim.x) {
        const uint64_t key = req.keys ? uniform_u64(req.keys[i]) : i;
        const uint64_t off = uniform_u64(log.key_off[key]);
        const uint64_t n = uniform_u64(log.key_off[key + 1]) - off;

        if (n != 0 && log.key_type != nullptr && log.key_type[key] != (uint8_t)req.req_type) {
            if (lane == 0) {
                out.flags[i] = AGN_F_ERR_CORRUPTED;
                out.err_pos[i] = 0xffffffffu;
                out.out_n[i] = 0;
            }
            continue;
        }

        F f;
        f.init(log, req, i);
        tab_clear<CAP>(L, lane);
        bool overflow = false;

        // base snapshot state: candidates with ord = index (< B)
        const uint64_t b0 = req.base_off ? req.base_off[i] : 0ull;
        const uint32_t B = req.base_off ? (uint32_t)(req.base_off[i + 1] - b0) : 0u;
        if (B > (uint32_t)(CAP / 2)) overflow = true;
        uint32_t used = overflow ? 0u : B;
        for (uint32_t x = lane; !overflow && x < B; x += AGN_WAVE)
            tab_insert<CAP>(L, req.base_tok[b0 + x], req.base_tag[b0 + x], x);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();

        uint32_t cnt = 0;
        int64_t first_err = -1;
        for (uint64_t b = 0; b < n; b += F::S::OPI) {
            bool valid;
            const bool incl = f.step(log, off, n, b, valid);
            if (overflow) continue;  // keep the filter outputs exact; state is lost
            const uint64_t pos = b + (uint64_t)f.slot;
            const uint64_t e = off + pos;
            const bool lead = incl && f.sub == 0;
            uint32_t tag = 0;
            uint64_t add = 0;
            bool opstart = false;
            if (lead) {
                tag = log.tag[e];
                add = log.add_tok[e];
                opstart = (pos == 0) || (log.op_id[e - 1] != log.op_id[e]);
            }
            const bool bad = lead && tag == AGN_TAG_INVALID;
            cnt += (uint32_t)__builtin_popcountll(ballot(lead && opstart));
            if (first_err < 0) {
                const uint64_t be = ballot(bad);
                if (be) first_err = (int64_t)b + (int64_t)(__builtin_ctzll(be) / LPO);
            }
            if (first_err >= 0) continue;  // {error, ...}: the state is not returned

            const bool adds = lead && add != 0ull;
            const uint32_t n_add = (uint32_t)__builtin_popcountll(ballot(adds));
            if (used + n_add > HIGH) {  // compact: drop tombstones
                const uint32_t live = gather_live<CAP>(L, lane);
                tab_clear<CAP>(L, lane);
                if (live > (uint32_t)(CAP / 2)) {
                    overflow = true;
                    continue;
                }
                for (uint32_t x = lane; x < live; x += AGN_WAVE)
                    tab_insert<CAP>(L, L.btok[x], L.btag[x], L.bord[x]);
                used = live;
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
            }
            // (1) candidates: included adds of this iteration
            if (adds) tab_insert<CAP>(L, add, tag, B + (uint32_t)pos);
            used += n_add;
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            // (2) removals (set_aw: Rem of the entry's elem; register_mv: Overridden)
            if (lead) {
                const uint32_t r0 = log.rem_off[e], r1 = log.rem_off[e + 1];
                const uint32_t q = B + (uint32_t)pos;
                for (uint32_t k = r0; k < r1; ++k) {
                    const int h = tab_find<CAP>(L, log.rem_tok[k]);
                    if (h >= 0 && (!SET || L.tag[h] == tag) && q > (L.ord[h] & ~DEAD))
                        atomicOr(&L.ord[h], DEAD);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }

        // live state -> sorted pairs
        uint32_t n_live = 0;
        bool cap_err = overflow;
        const uint64_t o = out.out_off[i];
        if (!overflow && first_err < 0) {
            n_live = gather_live<CAP>(L, lane);
            if ((uint64_t)n_live > out.out_off[i + 1] - o) {
                cap_err = true;
            } else {
                bitonic<SET, CAP>(L, n_live, lane);
                for (uint32_t x = lane; x < n_live; x += AGN_WAVE) {
                    out.out_tag[o + x] = L.btag[x];
                    out.out_tok[o + x] = L.btok[x];
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();

        const bool ct_ign = f.sct_ign && cnt == 0u;
        f.write_ct(reinterpret_cast<uint64_t(*)[AGN_WAVE]>(L.btok), out, i, ct_ign);

        if (lane == 0) {
            int64_t hole;
            if (f.first_excl >= 0) hole = (int64_t)log.op_id[off + (uint64_t)f.first_excl] - 1;
            else hole = n ? (int64_t)log.op_id[off + n - 1] : 0;
            uint32_t fl = 0;
            if (cnt) fl |= AGN_F_NEWSS;
            if (ct_ign) fl |= AGN_F_CT_IGNORE;
            if (first_err >= 0) fl |= AGN_F_ERR_UNEXPECTED;
            if (cap_err) fl |= AGN_F_ERR_CAPACITY;
            out.hole[i] = hole;
            out.count[i] = cnt;
            out.flags[i] = fl;
            out.err_pos[i] =
                first_err >= 0 ? (uint32_t)(off + (uint64_t)first_err) : 0xffffffffu;
            out.out_n[i] = n_live;
        }
        (void)lt;
    }
}

constexpr int TAG_CAP = 512;

template <int DPL, int LPO, bool SPARSE, bool SET>
int launch_shape(const agn_log &log, const agn_read &req, const agn_result &out,
                 hipStream_t st) {
    const unsigned blocks = grid_for(req.n_req, 1, 256u * 10u * 4u);
    hipLaunchKernelGGL((k_tags<DPL, LPO, SPARSE, SET, TAG_CAP>), dim3(blocks), dim3(64), 0,
                       st, log, req, out);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

template <bool SPARSE, bool SET>
int dispatch(const agn_log &log, const agn_read &req, const agn_result &out, hipStream_t st) {
#define AGN_L(DPL, LPO) launch_shape<DPL, LPO, SPARSE, SET>(log, req, out, st)
    AGN_DISPATCH_SHAPES(log.n_dcs, AGN_L)
#undef AGN_L
}

}  // namespace

int launch_tags(const agn_log &log, const agn_read &req, const agn_result &out,
                hipStream_t st) {
    if (req.n_req == 0) return AGN_OK;
    const bool sparse = log.oc_mask || req.R_mask || req.sct_mask || out.lastct_mask;
    const bool set = log.crdt_type == AGN_SET_AW;
    if (sparse) return set ? dispatch<true, true>(log, req, out, st)
                           : dispatch<true, false>(log, req, out, st);
    return set ? dispatch<false, true>(log, req, out, st) : dispatch<false, false>(log, req, out, st);
}

}  // namespace agn
