// mat_counter_dense.hip — the counter_pn fast path for dense clocks, D <= 8
// (BASELINE cfg1/cfg2 shapes): the same semantics as k_counter (filter.hpp +
// mat_counter.hip), specialised where the general kernel pays for
// generality:
//   * the read clock R and SCT are wave-uniform: explicit noalias kernel
//     arguments + readfirstlane keep them in SGPRs (s_load, no VGPRs);
//   * no presence masks (every DC present), so "+1 encoding" and per-DC
//     branches disappear; each OpSSCommit row is loaded with 16-byte loads;
//   * cold (SCT = ignore) and warm reads run separate loop bodies, so the
//     cold body does one D-wide compare per op, exactly the reference's
//     VC compare count;
//   * the i64 effect sum is reduced with DPP row ops + 4 readlanes.
// HBM bytes per op: 8*D + 8; per key: 8 + 16*D + 32.
#include <cstdlib>

#include "common.hpp"

namespace agn {
namespace {

__device__ __forceinline__ uint64_t dpp_u64(uint64_t v, int ctrl_id) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    switch (ctrl_id) {
        case 0:
            lo = __builtin_amdgcn_update_dpp(0u, lo, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
            hi = __builtin_amdgcn_update_dpp(0u, hi, 0xB1, 0xF, 0xF, false);
            break;
        case 1:
            lo = __builtin_amdgcn_update_dpp(0u, lo, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
            hi = __builtin_amdgcn_update_dpp(0u, hi, 0x4E, 0xF, 0xF, false);
            break;
        case 2:
            lo = __builtin_amdgcn_update_dpp(0u, lo, 0x141, 0xF, 0xF, false);  // row_half_mirror
            hi = __builtin_amdgcn_update_dpp(0u, hi, 0x141, 0xF, 0xF, false);
            break;
        default:
            lo = __builtin_amdgcn_update_dpp(0u, lo, 0x140, 0xF, 0xF, false);  // row_mirror
            hi = __builtin_amdgcn_update_dpp(0u, hi, 0x140, 0xF, 0xF, false);
            break;
    }
    return ((uint64_t)hi << 32) | lo;
}

// Full-wave i64 sum: 4 DPP steps make every 16-lane row uniform, then the 4
// row totals are read into SGPRs.
__device__ __forceinline__ int64_t wave_sum_dpp(int64_t x) {
    uint64_t v = (uint64_t)x;
    v += dpp_u64(v, 0);
    v += dpp_u64(v, 1);
    v += dpp_u64(v, 2);
    v += dpp_u64(v, 3);
    uint64_t t = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, r * 16);
        const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), r * 16);
        t += ((uint64_t)hi << 32) | lo;
    }
    return (int64_t)t;
}

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

template <bool NT, class T>
__device__ __forceinline__ T ld(const T *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// One OpSSCommit row; 16-byte loads when the row is 16-byte aligned (D even).
// NT: non-temporal (streamed once; keeps the log from thrashing L2/MALL).
template <int D, bool NT>
__device__ __forceinline__ void load_row(const uint64_t *__restrict__ p, uint64_t (&o)[D]) {
    if constexpr (D % 2 == 0) {
        const u64x2 *q = reinterpret_cast<const u64x2 *>(p);
#pragma unroll
        for (int j = 0; j < D / 2; ++j) {
            const u64x2 x = ld<NT>(q + j);
            o[2 * j] = x.x;
            o[2 * j + 1] = x.y;
        }
    } else {
#pragma unroll
        for (int j = 0; j < D; ++j) o[j] = ld<NT>(p + j);
    }
}

// Wave-uniform byte (key_type, sct_ignore) through the scalar cache: an s_load
// of the aligned dword (byte arrays are read in 4-byte units; allocations are
// rounded up far beyond that), so the check never waits on the vector-memory
// queue, where it would drain the cross-key prefetch.
__device__ __forceinline__ uint32_t byte_of(const uint8_t *__restrict__ p, uint64_t idx) {
    const uint32_t w = reinterpret_cast<const uint32_t *>(p)[idx >> 2];
    return (w >> ((uint32_t)(idx & 3u) * 8u)) & 0xffu;
}

struct DenseArgs {
    uint64_t n_req;
    uint64_t n_entries;
    uint32_t req_type;
    uint32_t _pad;
};

// Process the key's ops in chunks of 64 (lane = op).  `pre` holds the first
// chunk's row + effect when the caller prefetched them (software pipelining
// across keys); later chunks are loaded here.
template <int D, bool WARM, bool NT>
__device__ __forceinline__ void scan_key(const uint64_t *__restrict__ oc,
                                         const int64_t *__restrict__ eff,
                                         const uint64_t *__restrict__ txid, uint64_t txr,
                                         uint64_t off, uint64_t n, const uint64_t (&r)[D],
                                         const uint64_t (&s)[D], uint64_t (&ct)[D], int64_t &sum,
                                         uint32_t &cnt, int64_t &first_excl, int64_t &first_err,
                                         const uint64_t (*pre_o)[D], int64_t pre_ev) {
    const int lane = lane_id();
    for (uint64_t b = 0; b < n; b += AGN_WAVE) {
        const uint64_t pos = b + (uint64_t)lane;
        const bool valid = pos < n;
        const uint64_t e = off + (valid ? pos : 0ull);  // in-bounds for idle lanes
        uint64_t o[D];
        int64_t ev;
        if (b == 0 && pre_o != nullptr) {
#pragma unroll
            for (int j = 0; j < D; ++j) o[j] = (*pre_o)[j];
            ev = pre_ev;
        } else {
            load_row<D, NT>(oc + e * D, o);
            ev = ld<NT>(eff + e);
        }
        bool okR = true, leS = true;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            okR = okR && (o[j] <= r[j]);
            if (WARM) leS = leS && (o[j] <= s[j]);
        }
        bool nip = WARM ? !leS : true;  // belongs_to_snapshot_op (ignore -> true)
        if (txid != nullptr) nip = nip || (txid[e] == txr);
        const bool incl = valid && nip && okR;
        const bool excl = valid && nip && !okR;
        if (first_excl < 0) {
            const uint64_t bx = ballot(excl);
            if (bx) first_excl = (int64_t)b + (int64_t)__builtin_ctzll(bx);
        }
#pragma unroll
        for (int j = 0; j < D; ++j) ct[j] = (incl && o[j] > ct[j]) ? o[j] : ct[j];
        const bool bad = incl && ev == AGN_EFFECT_INVALID;
        cnt += (uint32_t)__builtin_popcountll(ballot(incl));
        if (first_err < 0) {
            const uint64_t be = ballot(bad);
            if (be) first_err = (int64_t)b + (int64_t)__builtin_ctzll(be);
        }
        sum += (incl && !bad) ? ev : 0;
    }
}

// ANY_WARM = false when the batch has no SCT at all (cold reads): the SCT
// registers and the warm loop body are compiled out (SGPR pressure).
// VAR: 0 = plain; 1 = prefetch the next key's first 64 rows + effects before
// reducing the current key (keeps HBM requests in flight across the per-key
// reduction).  MINW = launch-bound waves per SIMD (8 caps SGPRs at 80, so 8
// blocks of 256 fit a CU).
template <int D, bool ANY_WARM, int VAR, int MINW>
__global__ __launch_bounds__(256, MINW) void k_counter_dense(
    DenseArgs a, const uint64_t *__restrict__ keys, const uint64_t *__restrict__ key_off,
    const uint8_t *__restrict__ key_type, const uint64_t *__restrict__ oc,
    const uint32_t *__restrict__ op_id, const int64_t *__restrict__ eff,
    const uint64_t *__restrict__ log_txid, const uint64_t *__restrict__ R,
    const uint64_t *__restrict__ sct, const uint8_t *__restrict__ sct_ignore,
    const uint64_t *__restrict__ req_txid, const int64_t *__restrict__ base_value,
    int64_t *__restrict__ o_value, int64_t *__restrict__ o_hole, uint64_t *__restrict__ o_lastct,
    uint32_t *__restrict__ o_count, uint32_t *__restrict__ o_flags,
    uint32_t *__restrict__ o_err) {
    constexpr bool PF = VAR >= 1, NT = false;
    constexpr int DCP = D <= 1 ? 1 : D <= 2 ? 2 : D <= 4 ? 4 : 8;  // pow2 >= D
    constexpr int V = DCP;                                          // op slots per lane
    __shared__ uint64_t stage[4][DCP][AGN_WAVE];
    const int lane = lane_id();
    const int w = threadIdx.x >> 6;
    const uint64_t nw = (uint64_t)gridDim.x * 4u;

    // key meta (uniform) + first-chunk rows of the key this wave handles next
    auto meta = [&](uint64_t i, uint64_t &key, uint64_t &off, uint64_t &n) {
        key = keys ? uniform_u64(keys[i]) : i;
        off = uniform_u64(key_off[key]);
        n = uniform_u64(key_off[key + 1]) - off;
    };
    uint64_t p_o[D];
    int64_t p_ev = 0;
    uint64_t i = uniform_u64((uint64_t)blockIdx.x * 4u + (uint64_t)w);
    uint64_t key = 0, off = 0, n = 0;
    if (i < a.n_req) {
        meta(i, key, off, n);
        if (PF && n) {
            const uint64_t e = off + ((uint64_t)lane < n ? (uint64_t)lane : 0ull);
            load_row<D, NT>(oc + e * D, p_o);
            p_ev = ld<NT>(eff + e);
        }
    }
    for (; i < a.n_req; i += nw) {
        uint64_t c_o[D];
        const int64_t c_ev = p_ev;
#pragma unroll
        for (int j = 0; j < D; ++j) c_o[j] = p_o[j];
        const uint64_t c_key = key, c_off = off, c_n = n;
        const uint64_t inext = i + nw;
        if (inext < a.n_req) {
            meta(inext, key, off, n);
            if (PF && n) {
                const uint64_t e = off + ((uint64_t)lane < n ? (uint64_t)lane : 0ull);
                load_row<D, NT>(oc + e * D, p_o);
                p_ev = ld<NT>(eff + e);
            }
        }
        if (c_n != 0 && key_type != nullptr && byte_of(key_type, c_key) != (a.req_type & 0xffu)) {
            if (lane == 0) {  // erlang:error(corrupted_ops_cache)
                o_flags[i] = AGN_F_ERR_CORRUPTED;
                o_err[i] = 0xffffffffu;
            }
            continue;
        }
        uint64_t r[D], s[D], ct[D];
        const bool sct_ign = !ANY_WARM || sct == nullptr || (sct_ignore && byte_of(sct_ignore, i));
#pragma unroll
        for (int j = 0; j < D; ++j) {
            r[j] = uniform_u64(R[i * D + j]);
            s[j] = sct_ign ? 0ull : uniform_u64(sct[i * D + j]);
            ct[j] = s[j];  // LastOpCt starts as SCT (materialize/4 :94-95)
        }
        const uint64_t txr = req_txid ? uniform_u64(req_txid[i]) : 0ull;
        const uint64_t *tx = (txr != 0ull) ? log_txid : nullptr;
        int64_t sum = 0, first_excl = -1, first_err = -1;
        uint32_t cnt = 0;
        const uint64_t(*pre)[D] = PF ? &c_o : nullptr;
        if (!ANY_WARM || sct_ign)
            scan_key<D, false, NT>(oc, eff, tx, txr, c_off, c_n, r, s, ct, sum, cnt, first_excl,
                                   first_err, pre, c_ev);
        else
            scan_key<D, ANY_WARM, NT>(oc, eff, tx, txr, c_off, c_n, r, s, ct, sum, cnt,
                                      first_excl, first_err, pre, c_ev);

        const int64_t total = wave_sum_dpp(sum);
        // LastOpCt: per-lane maxima -> LDS [DCP][64] -> each lane folds V slots
        // of one DC -> xor-shuffle across the 64/DCP lanes that share it
#pragma unroll
        for (int j = 0; j < D; ++j) stage[w][j][lane] = ct[j];
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const int c = lane % DCP, g = lane / DCP;
        uint64_t m = 0;
        if (c < D) {
#pragma unroll
            for (int v = 0; v < V; ++v) m = umax64(m, stage[w][c][g * V + v]);
        }
#pragma unroll
        for (int x = DCP; x < AGN_WAVE; x <<= 1) m = umax64(m, shfl_xor_u64(m, x));
        const bool ct_ign = sct_ign && cnt == 0u;
        if (g == 0 && c < D) o_lastct[i * D + (uint64_t)c] = ct_ign ? 0ull : m;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();

        // NewLastOp and the base value through scalar loads (uniform addresses)
        const uint64_t hole_e =
            first_excl >= 0 ? c_off + (uint64_t)first_excl : c_off + c_n - 1;
        const int64_t hid = c_n ? (int64_t)op_id[uniform_u64(hole_e)] : 0;
        const int64_t base = base_value ? (int64_t)uniform_u64((uint64_t)base_value[i]) : 0;
        if (lane == 0) {
            // id(oldest excluded) - 1, else get_first_id (:49-63)
            const int64_t hole = first_excl >= 0 ? hid - 1 : hid;
            uint32_t fl = 0;
            if (cnt) fl |= AGN_F_NEWSS;
            if (ct_ign) fl |= AGN_F_CT_IGNORE;
            if (first_err >= 0) fl |= AGN_F_ERR_UNEXPECTED;
            o_value[i] = (int64_t)((uint64_t)base + (uint64_t)total);
            o_hole[i] = hole;
            o_count[i] = cnt;
            o_flags[i] = fl;
            o_err[i] = first_err >= 0 ? (uint32_t)(c_off + (uint64_t)first_err) : 0xffffffffu;
        }
    }
}

// VAR 2 — "meta-ahead" stream: per key only ONE dependent HBM round trip is
// exposed (the OpSSCommit rows).  Everything else a key needs is fetched one
// key AHEAD with a single divergent-address vector load (lane 0/1: key_off
// pair, lanes 2..D+1: R, then SCT, base value, reading TxId; a second load
// carries the key_type / sct_ignore dwords), issued right after the current
// key's rows so the compiler's counted vmcnt waits leave it in flight; and
// the op_id that defines NewLastOp is loaded one key LATE (its hole is
// stored during the next key).  No scalar loads remain in the loop, so the
// LDS waits of the LastOpCt reduction never wait on memory.
template <int D>
struct Meta {
    uint64_t v;  // per-lane slot, see meta_lane()
    uint32_t b;  // lane 0: key_type dword, lane 1: sct_ignore dword
};

template <int D, bool ANY_WARM, int MINW>
__global__ __launch_bounds__(256, MINW) void k_counter_stream(
    DenseArgs a, const uint64_t *__restrict__ keys, const uint64_t *__restrict__ key_off,
    const uint8_t *__restrict__ key_type, const uint64_t *__restrict__ oc,
    const uint32_t *__restrict__ op_id, const int64_t *__restrict__ eff,
    const uint64_t *__restrict__ log_txid, const uint64_t *__restrict__ R,
    const uint64_t *__restrict__ sct, const uint8_t *__restrict__ sct_ignore,
    const uint64_t *__restrict__ req_txid, const int64_t *__restrict__ base_value,
    int64_t *__restrict__ o_value, int64_t *__restrict__ o_hole, uint64_t *__restrict__ o_lastct,
    uint32_t *__restrict__ o_count, uint32_t *__restrict__ o_flags,
    uint32_t *__restrict__ o_err) {
    constexpr int DCP = D <= 1 ? 1 : D <= 2 ? 2 : D <= 4 ? 4 : 8;  // pow2 >= D
    constexpr int V = DCP;
    // lane layout of Meta::v
    constexpr int L_OFF = 0, L_END = 1, L_R = 2, L_S = 2 + D, L_BASE = 2 + 2 * D,
                  L_TX = 3 + 2 * D;
    static_assert(L_TX < AGN_WAVE, "meta lanes");
    __shared__ uint64_t stage[4][DCP][AGN_WAVE];
    const int lane = lane_id();
    const int w = threadIdx.x >> 6;
    const uint64_t nw = (uint64_t)gridDim.x * 4u;
    const uint64_t last_e = a.n_entries - 1;  // n_entries > 0 (checked by the launcher)

    auto fetch_meta = [&](uint64_t i) {
        const uint64_t key = keys ? uniform_u64(keys[i]) : i;
        const uint64_t *p = key_off + key;  // safe default address
        if (lane == L_END) p = key_off + key + 1;
        else if (lane >= L_R && lane < L_R + D) p = R + i * D + (lane - L_R);
        else if (ANY_WARM && sct && lane >= L_S && lane < L_S + D) p = sct + i * D + (lane - L_S);
        else if (base_value && lane == L_BASE) p = reinterpret_cast<const uint64_t *>(base_value + i);
        else if (req_txid && lane == L_TX) p = req_txid + i;
        const uint32_t *q = reinterpret_cast<const uint32_t *>(key_off + key);
        if (key_type && lane == 0) q = reinterpret_cast<const uint32_t *>(key_type) + (key >> 2);
        else if (ANY_WARM && sct_ignore && lane == 1)
            q = reinterpret_cast<const uint32_t *>(sct_ignore) + (i >> 2);
        Meta<D> m;
        m.v = *p;
        m.b = *q;
        return m;
    };
    auto rd = [&](uint64_t v, int l) {
        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
        const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
        return ((uint64_t)hi << 32) | lo;
    };

    uint64_t i = uniform_u64((uint64_t)blockIdx.x * 4u + (uint64_t)w);
    if (i >= a.n_req) return;
    Meta<D> mc = fetch_meta(i);
    // deferred NewLastOp of the previous key: request index, entry, flag
    uint64_t h_i = 0, h_e = 0;
    bool h_pending = false, h_first = false;
    for (;;) {
        const uint64_t off = rd(mc.v, L_OFF), n = rd(mc.v, L_END) - off;
        const uint64_t key = keys ? uniform_u64(keys[i]) : i;
        // (1) this key's first 64 rows + effects: the one exposed round trip
        uint64_t o[D];
        int64_t ev;
        {
            uint64_t e = off + ((uint64_t)lane < n ? (uint64_t)lane : 0ull);
            e = e < last_e ? e : last_e;
            load_row<D, false>(oc + e * D, o);
            ev = eff[e];
        }
        // (2) next key's metadata, one key ahead (clamped to a harmless re-read)
        const uint64_t inext = i + nw;
        const bool more = inext < a.n_req;
        const Meta<D> mn = fetch_meta(more ? inext : i);
        // (3) previous key's NewLastOp id, one key late
        uint32_t hid = 0;
        if (h_pending) hid = op_id[h_e];

        const uint32_t ktw = __builtin_amdgcn_readlane(mc.b, 0);
        const bool corrupted = n != 0 && key_type != nullptr &&
                               ((ktw >> ((uint32_t)(key & 3u) * 8u)) & 0xffu) !=
                                   (a.req_type & 0xffu);
        int64_t first_excl = -1;
        uint32_t cnt = 0;
        if (corrupted) {
            if (lane == 0) {  // erlang:error(corrupted_ops_cache) (:190-191)
                o_flags[i] = AGN_F_ERR_CORRUPTED;
                o_err[i] = 0xffffffffu;
            }
        } else {
            const uint32_t siw = __builtin_amdgcn_readlane(mc.b, 1);
            const bool sct_ign = !ANY_WARM || sct == nullptr ||
                                 (sct_ignore && ((siw >> ((uint32_t)(i & 3u) * 8u)) & 0xffu));
            uint64_t r[D], sv[D], ct[D];
#pragma unroll
            for (int j = 0; j < D; ++j) {
                r[j] = rd(mc.v, L_R + j);
                sv[j] = sct_ign ? 0ull : rd(mc.v, L_S + j);
                ct[j] = sv[j];  // LastOpCt starts as SCT (materialize/4 :94-95)
            }
            const uint64_t txr = req_txid ? rd(mc.v, L_TX) : 0ull;
            const uint64_t *tx = (txr != 0ull) ? log_txid : nullptr;
            int64_t sum = 0, first_err = -1;
            if (sct_ign)
                scan_key<D, false, false>(oc, eff, tx, txr, off, n, r, sv, ct, sum, cnt,
                                          first_excl, first_err, &o, ev);
            else
                scan_key<D, ANY_WARM, false>(oc, eff, tx, txr, off, n, r, sv, ct, sum, cnt,
                                             first_excl, first_err, &o, ev);
            const int64_t base = base_value ? (int64_t)rd(mc.v, L_BASE) : 0;
            const int64_t total = wave_sum_dpp(sum);
#pragma unroll
            for (int j = 0; j < D; ++j) stage[w][j][lane] = ct[j];
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const int c = lane % DCP, g = lane / DCP;
            uint64_t m = 0;
            if (c < D) {
#pragma unroll
                for (int v = 0; v < V; ++v) m = umax64(m, stage[w][c][g * V + v]);
            }
#pragma unroll
            for (int x = DCP; x < AGN_WAVE; x <<= 1) m = umax64(m, shfl_xor_u64(m, x));
            const bool ct_ign = sct_ign && cnt == 0u;
            if (g == 0 && c < D) o_lastct[i * D + (uint64_t)c] = ct_ign ? 0ull : m;
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) {
                uint32_t fl = 0;
                if (cnt) fl |= AGN_F_NEWSS;
                if (ct_ign) fl |= AGN_F_CT_IGNORE;
                if (first_err >= 0) fl |= AGN_F_ERR_UNEXPECTED;
                o_value[i] = (int64_t)((uint64_t)base + (uint64_t)total);
                o_count[i] = cnt;
                o_flags[i] = fl;
                o_err[i] = first_err >= 0 ? (uint32_t)(off + (uint64_t)first_err) : 0xffffffffu;
            }
        }
        // store the previous key's hole: id(oldest excluded) - 1, else get_first_id
        if (h_pending && lane == 0) o_hole[h_i] = h_first ? (int64_t)hid - 1 : (int64_t)hid;
        if (corrupted) {
            h_pending = false;
        } else if (n == 0) {
            if (lane == 0) o_hole[i] = 0;
            h_pending = false;
        } else {
            h_pending = true;
            h_i = i;
            h_first = first_excl >= 0;
            h_e = first_excl >= 0 ? off + (uint64_t)first_excl : off + n - 1;
        }
        if (!more) break;
        mc = mn;
        i = inext;
    }
    if (h_pending) {
        const uint32_t hid = op_id[h_e];
        if (lane == 0) o_hole[h_i] = h_first ? (int64_t)hid - 1 : (int64_t)hid;
    }
}

template <int D, int VAR, int MINW>
int launch_dense_var(const agn_log &log, const agn_read &req, const agn_result &out,
                     hipStream_t st) {
    DenseArgs a{req.n_req, log.n_entries, req.req_type, 0};
    const unsigned blocks = grid_for(req.n_req, 4, 256u * 16u);
    if (VAR == 2) {
        if (req.sct)
            hipLaunchKernelGGL((k_counter_stream<D, true, MINW>), dim3(blocks), dim3(256), 0, st,
                               a, req.keys, log.key_off, log.key_type, log.oc, log.op_id,
                               log.eff, log.txid, req.R, req.sct, req.sct_ignore, req.txid,
                               req.base_value, out.value, out.hole, out.lastct, out.count,
                               out.flags, out.err_pos);
        else
            hipLaunchKernelGGL((k_counter_stream<D, false, MINW>), dim3(blocks), dim3(256), 0, st,
                               a, req.keys, log.key_off, log.key_type, log.oc, log.op_id,
                               log.eff, log.txid, req.R, req.sct, req.sct_ignore, req.txid,
                               req.base_value, out.value, out.hole, out.lastct, out.count,
                               out.flags, out.err_pos);
    } else if (req.sct)
        hipLaunchKernelGGL((k_counter_dense<D, true, VAR, MINW>), dim3(blocks), dim3(256), 0, st, a,
                           req.keys, log.key_off, log.key_type, log.oc, log.op_id, log.eff,
                           log.txid, req.R, req.sct, req.sct_ignore, req.txid, req.base_value,
                           out.value, out.hole, out.lastct, out.count, out.flags, out.err_pos);
    else
        hipLaunchKernelGGL((k_counter_dense<D, false, VAR, MINW>), dim3(blocks), dim3(256), 0, st, a,
                           req.keys, log.key_off, log.key_type, log.oc, log.op_id, log.eff,
                           log.txid, req.R, req.sct, req.sct_ignore, req.txid, req.base_value,
                           out.value, out.hole, out.lastct, out.count, out.flags, out.err_pos);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

// A/B knobs: AGN_COUNTER_VARIANT=0|1|2 (plain / cross-key row prefetch / meta-ahead stream, default 2),
// AGN_COUNTER_MINW=6|8 (launch-bound waves per SIMD, default 6).
int dense_variant() {
    const char *v = getenv("AGN_COUNTER_VARIANT");
    if (v && (v[0] == '0' || v[0] == '1')) return v[0] - '0';
    return 2;
}
int dense_minw() {
    const char *v = getenv("AGN_COUNTER_MINW");
    return (v && v[0] == '8') ? 8 : 6;
}

template <int D>
int launch_dense(const agn_log &log, const agn_read &req, const agn_result &out,
                 hipStream_t st) {
    const int var = dense_variant(), minw = dense_minw();
    if (var == 2) return minw == 6 ? launch_dense_var<D, 2, 6>(log, req, out, st)
                                   : launch_dense_var<D, 2, 8>(log, req, out, st);
    if (var == 1) return minw == 6 ? launch_dense_var<D, 1, 6>(log, req, out, st)
                                   : launch_dense_var<D, 1, 8>(log, req, out, st);
    return minw == 6 ? launch_dense_var<D, 0, 6>(log, req, out, st)
                     : launch_dense_var<D, 0, 8>(log, req, out, st);
}

}  // namespace

// Dense fast path applies when every clock is dense and D <= 8; returns
// AGN_ENOTSUP otherwise so the caller uses the general kernel.
int launch_counter_dense(const agn_log &log, const agn_read &req, const agn_result &out,
                         hipStream_t st) {
    if (log.oc_mask || req.R_mask || req.sct_mask || out.lastct_mask) return AGN_ENOTSUP;
    if (log.n_entries == 0) return AGN_ENOTSUP;  // the clamped row loads need one valid row
    switch (log.n_dcs) {
        case 1: return launch_dense<1>(log, req, out, st);
        case 2: return launch_dense<2>(log, req, out, st);
        case 3: return launch_dense<3>(log, req, out, st);
        case 4: return launch_dense<4>(log, req, out, st);
        case 5: return launch_dense<5>(log, req, out, st);
        case 6: return launch_dense<6>(log, req, out, st);
        case 7: return launch_dense<7>(log, req, out, st);
        case 8: return launch_dense<8>(log, req, out, st);
        default: return AGN_ENOTSUP;
    }
}

}  // namespace agn
