// counter_scan.hpp -- the counter_pn per-key scan shared by the dense
// counter kernel (mat_counter_dense.hip, the batched materialize/4) and the
// fused cached read (read6.hip, read/6 from the snapshot cache): wave
// reductions, row loads, scalar side loads, per-key metadata and the
// newest-to-oldest filter + fold over a key's ops (one wave per key), with
// row-per-lane loads (scan_key) or, for D = 8, lane-contiguous quad rows
// (scan_key_q8).
#pragma once
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
// (ldc: the read-only per-key / per-request arrays load through the scalar
// cache also where the kernel's pointers carry no __restrict__ -- read6.hip,
// k_counter_q8e2's parameter block -- instead of as vector loads each waited
// for before its readfirstlane)
__device__ __forceinline__ uint32_t byte_of(const uint8_t *__restrict__ p, uint64_t idx) {
    const uint32_t w = ldc(reinterpret_cast<const uint32_t *>(p) + (idx >> 2));
    return (w >> ((uint32_t)(idx & 3u) * 8u)) & 0xffu;
}

// Per-key metadata as branch-free scalar loads, so key_off, the segment
// length and the id base share one round trip (a conditional load would be
// scheduled after the previous one's wait): absent arrays are replaced by an
// in-bounds dummy address whose value is discarded.
struct KeyMeta {
    uint64_t off, n;
    uint32_t id0;
};
__device__ __forceinline__ KeyMeta key_meta(uint64_t key, const uint64_t *__restrict__ key_off,
                                            const uint64_t *__restrict__ key_len,
                                            const uint32_t *__restrict__ key_id0) {
    const uint64_t *lp = key_len ? key_len + key : key_off + key + 1;
    const uint32_t *ip = key_id0 ? key_id0 + key : reinterpret_cast<const uint32_t *>(key_off + key);
    const uint64_t off = uniform_u64(ldc(key_off + key));
    const uint64_t l = uniform_u64(ldc(lp));
    const uint32_t id = __builtin_amdgcn_readfirstlane(ldc(ip));
    return KeyMeta{off, key_len ? l : l - off, key_id0 ? id : AGN_ID0_NONE};
}

// Process the key's ops in chunks of 64 (lane = op), rows by 16-byte VGPR
// loads.  The op id that defines NewLastOp is one scalar load after the scan:
// loading every lane's op id with its row instead (+4 B per op, no dependent
// load) measured 2.7 % slower (profiles/r01/ab_counter_ids_wpb.log).
//
// PAIR (small D only, where the registers are free): a key longer than one
// chunk is walked two chunks per step with both chunks' loads issued before
// either is compared (unconditional loads, idle lanes clamped to the key's
// first entry), so a 65..128-op key costs one row round trip instead of two --
// the latency of a small batch (cfg1: 10k keys x 100 ops, one wave per key,
// ~1.2 waves per wave slot) is a few such round trips.
template <int D, bool WARM>
__device__ __forceinline__ void scan_chunk(const uint64_t (&o)[D], int64_t ev, bool valid,
                                           uint64_t b, const uint64_t *__restrict__ txid,
                                           uint64_t txr, uint64_t e, const uint64_t (&r)[D],
                                           const uint64_t (&s)[D], uint64_t (&ct)[D], int64_t &sum,
                                           uint32_t &cnt, int64_t &first_excl,
                                           int64_t &first_err) {
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

template <int D, bool WARM, bool PAIR = false>
__device__ __forceinline__ void scan_key(const uint64_t *__restrict__ oc,
                                         const int64_t *__restrict__ eff,
                                         const uint64_t *__restrict__ txid, uint64_t txr,
                                         uint64_t off, uint64_t n, const uint64_t (&r)[D],
                                         const uint64_t (&s)[D], uint64_t (&ct)[D], int64_t &sum,
                                         uint32_t &cnt, int64_t &first_excl, int64_t &first_err) {
    const int lane = lane_id();
    if constexpr (PAIR) {
        if (n > (uint64_t)AGN_WAVE) {
            for (uint64_t b = 0; b < n; b += 2 * AGN_WAVE) {
                const uint64_t p0 = b + (uint64_t)lane, p1 = p0 + AGN_WAVE;
                const bool v0 = p0 < n, v1 = p1 < n;
                const uint64_t e0 = off + (v0 ? p0 : 0ull), e1 = off + (v1 ? p1 : 0ull);
                uint64_t o0[D], o1[D];
                load_row<D, false>(oc + e0 * D, o0);
                load_row<D, false>(oc + e1 * D, o1);
                const int64_t ev0 = eff[e0], ev1 = eff[e1];
                scan_chunk<D, WARM>(o0, ev0, v0, b, txid, txr, e0, r, s, ct, sum, cnt,
                                    first_excl, first_err);
                scan_chunk<D, WARM>(o1, ev1, v1, b + AGN_WAVE, txid, txr, e1, r, s, ct, sum, cnt,
                                    first_excl, first_err);
            }
            return;
        }
    }
    for (uint64_t b = 0; b < n; b += AGN_WAVE) {
        const uint64_t pos = b + (uint64_t)lane;
        const bool valid = pos < n;
        const uint64_t e = off + (valid ? pos : 0ull);  // in-bounds for idle lanes
        uint64_t o[D];
        load_row<D, false>(oc + e * D, o);
        const int64_t ev = eff[e];
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

// ---- presence masks (D <= 8, one mask word per clock) ---------------------
// A sparse log's key whose entries do not all carry the same DC set, or whose
// DCs are not all in R (agn_log.key_mask), is scanned with its per-entry
// masks: lane = op, the row and its mask word loaded together, and the dict
// fold of is_op_in_snapshot (src/clocksi_materializer.erl:236-258): a DC of
// the op missing from R excludes the op (:245-247), a DC missing from SCT
// reads 0 (vectorclock:le), LastOpCt takes the max over each included op's
// own DCs and unites their DC sets (um, per lane).  s[] is SCT with its
// missing DCs already 0.  Same outputs as scan_key otherwise.
template <int D, bool WARM>
__device__ __forceinline__ void scan_key_msk(const uint64_t *__restrict__ oc,
                                             const uint64_t *__restrict__ oc_mask,
                                             const int64_t *__restrict__ eff,
                                             const uint64_t *__restrict__ txid, uint64_t txr,
                                             uint64_t off, uint64_t n, const uint64_t (&r)[D],
                                             const uint64_t (&s)[D], uint64_t rm, uint64_t (&ct)[D],
                                             uint64_t &um, int64_t &sum, uint32_t &cnt,
                                             int64_t &first_excl, int64_t &first_err) {
    constexpr uint64_t FULL = (1ull << D) - 1ull;
    const int lane = lane_id();
    for (uint64_t b = 0; b < n; b += AGN_WAVE) {
        const uint64_t pos = b + (uint64_t)lane;
        const bool valid = pos < n;
        const uint64_t e = off + (valid ? pos : 0ull);
        uint64_t o[D];
        load_row<D, false>(oc + e * D, o);
        const uint64_t m = (oc_mask ? oc_mask[e] : FULL) & FULL;
        const int64_t ev = eff[e];
        bool okR = (m & ~rm) == 0ull, leS = true;  // a DC of the op missing from R: false
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const bool p = ((m >> j) & 1ull) != 0ull;
            okR = okR && (!p || o[j] <= r[j]);
            if (WARM) leS = leS && (!p || o[j] <= s[j]);
        }
        bool nip = WARM ? !leS : true;
        if (txid != nullptr) nip = nip || (txid[e] == txr);
        const bool incl = valid && nip && okR;
        const bool excl = valid && nip && !okR;
        if (first_excl < 0) {
            const uint64_t bx = ballot(excl);
            if (bx) first_excl = (int64_t)b + (int64_t)__builtin_ctzll(bx);
        }
#pragma unroll
        for (int j = 0; j < D; ++j)
            ct[j] = (incl && ((m >> j) & 1ull) && o[j] > ct[j]) ? o[j] : ct[j];
        um |= incl ? m : 0ull;
        const bool bad = incl && ev == AGN_EFFECT_INVALID;
        cnt += (uint32_t)__builtin_popcountll(ballot(incl));
        if (first_err < 0) {
            const uint64_t be = ballot(bad);
            if (be) first_err = (int64_t)b + (int64_t)__builtin_ctzll(be);
        }
        sum += (incl && !bad) ? ev : 0;
    }
}

// OR of a per-lane DC set over the wave (D <= 8 bits), as a scalar.
template <int D>
__device__ __forceinline__ uint64_t wave_or_bits(uint64_t um) {
    uint64_t r = 0;
#pragma unroll
    for (int j = 0; j < D; ++j) r |= (ballot(((um >> j) & 1ull) != 0ull) != 0ull) ? (1ull << j) : 0ull;
    return r;
}

// scan_key for D = 8 with lane-CONTIGUOUS row loads ("quad rows"): load j of a
// 64-op chunk reads bytes [1 KiB j, 1 KiB (j+1)) of the chunk's rows, so
// every instruction covers 8 whole 128-byte lines -- the row-per-lane loads
// of scan_key touch 32 lines per instruction, 32 bytes of each, and request
// every line four times.  Lane l holds DCs 2p, 2p+1 (p = l & 3) of op
// 16 j + (l >> 2): the per-op verdicts are nibbles of wave ballots folded on
// the scalar unit into 64-bit op masks (incl / excl), and the LastOpCt maxima
// stay per part (ctA, ctB) until one xor-shuffle fold at the end of the key.
// The effect (and TxId) loads stay lane = op.  Same results as scan_key.
// One 64-op chunk of quad rows (load j: lane l holds DCs 2p, 2p+1 of op
// 16 j + (l >> 2)) and its effects (lane = op).
struct Q8Chunk {
    u64x2 x[4];
    int64_t ev;
};

template <bool NT, bool EFF_NT>
__device__ __forceinline__ Q8Chunk q8_load(const uint64_t *__restrict__ oc,
                                           const int64_t *__restrict__ eff, uint64_t off,
                                           uint64_t b, uint64_t n_entries) {
    const int lane = lane_id();
    const u64x2 *rows = reinterpret_cast<const u64x2 *>(oc);
    const uint64_t lim = n_entries * 4u - 1u, lim_e = n_entries - 1u;
    Q8Chunk c;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint64_t u = (off + b) * 4u + (uint64_t)(j * AGN_WAVE + lane);
        u = u < lim ? u : lim;  // past the log's end: clamped, masked in q8_fold
        c.x[j] = ld<NT>(rows + u);
    }
    uint64_t e = off + b + (uint64_t)lane;
    e = e < lim_e ? e : lim_e;
    c.ev = ld<NT && EFF_NT>(eff + e);
    return c;
}

// noR: R lacks one of the DCs every op of the key carries -- every op is
// excluded (is_op_in_snapshot's missing-DC branch, :245-247); the SCT compare
// (notInPrev) still decides which exclusions count.
template <bool WARM>
__device__ __forceinline__ void q8_fold(const Q8Chunk &c, const uint64_t *__restrict__ txid,
                                        uint64_t txr, uint64_t off, uint64_t b, uint64_t n,
                                        uint64_t n_entries, uint64_t rA, uint64_t rB, uint64_t sA,
                                        uint64_t sB, uint64_t &ctA, uint64_t &ctB, int64_t &sum,
                                        uint32_t &cnt, int64_t &first_excl, int64_t &first_err,
                                        bool noR = false) {
    const int lane = lane_id();
    const int q = lane >> 2;
    const uint64_t valid = (n - b >= (uint64_t)AGN_WAVE) ? ~0ull : ((1ull << (n - b)) - 1ull);
    uint64_t bad = 0, gt = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        bad |= nib_any16(ballot(c.x[j].x > rA || c.x[j].y > rB)) << (16 * j);
        if (WARM) gt |= nib_any16(ballot(c.x[j].x > sA || c.x[j].y > sB)) << (16 * j);
    }
    uint64_t nip = WARM ? gt : ~0ull;  // belongs_to_snapshot_op: not covered by SCT
    if (txid != nullptr) {
        uint64_t e = off + b + (uint64_t)lane;
        e = e < n_entries - 1u ? e : n_entries - 1u;
        nip |= ballot(txid[e] == txr);
    }
    if (noR) bad = ~0ull;
    const uint64_t incl = valid & nip & ~bad, excl = valid & nip & bad;
    if (first_excl < 0 && excl) first_excl = (int64_t)b + (int64_t)__builtin_ctzll(excl);
    cnt += (uint32_t)__builtin_popcountll(incl);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool in = ((incl >> (16 * j + q)) & 1ull) != 0ull;
        ctA = (in && c.x[j].x > ctA) ? c.x[j].x : ctA;
        ctB = (in && c.x[j].y > ctB) ? c.x[j].y : ctB;
    }
    const bool mine = ((incl >> lane) & 1ull) != 0ull;
    const bool badv = mine && c.ev == AGN_EFFECT_INVALID;
    if (first_err < 0) {
        const uint64_t be = ballot(badv);
        if (be) first_err = (int64_t)b + (int64_t)__builtin_ctzll(be);
    }
    sum += (mine && !badv) ? c.ev : 0;
}

// scan_key for D = 8 with lane-CONTIGUOUS row loads ("quad rows"): load j of a
// 64-op chunk reads bytes [1 KiB j, 1 KiB (j+1)) of the chunk's rows, so
// every instruction covers 8 whole 128-byte lines -- the row-per-lane loads
// of scan_key touch 32 lines per instruction, 32 bytes of each, and request
// every line four times.  Lane l holds DCs 2p, 2p+1 (p = l & 3) of op
// 16 j + (l >> 2): the per-op verdicts are nibbles of wave ballots folded on
// the scalar unit into 64-bit op masks (incl / excl), and the LastOpCt maxima
// stay per part (ctA, ctB) until one xor-shuffle fold at the end of the key.
// The effect (and TxId) loads stay lane = op.  Same results as scan_key.
// FROM1: the caller has loaded and folded chunk 0 (read6.hip issues it
// before its cache lookup) and the walk starts at op 64.
template <bool WARM, bool NT, bool EFF_NT = false, bool FROM1 = false>
__device__ __forceinline__ void scan_key_q8(
    const uint64_t *__restrict__ oc, const int64_t *__restrict__ eff,
    const uint64_t *__restrict__ txid, uint64_t txr, uint64_t off, uint64_t n,
    uint64_t n_entries, uint64_t rA, uint64_t rB, uint64_t sA, uint64_t sB, uint64_t &ctA,
    uint64_t &ctB, int64_t &sum, uint32_t &cnt, int64_t &first_excl, int64_t &first_err,
    bool noR = false) {
    for (uint64_t b = FROM1 ? AGN_WAVE : 0; b < n; b += AGN_WAVE) {
        const Q8Chunk c = q8_load<NT, EFF_NT>(oc, eff, off, b, n_entries);
        // every load of the chunk is in flight before the first verdict (left
        // alone, the scheduler interleaves the ballots with the loads and
        // waits for each row load in turn)
        __builtin_amdgcn_sched_barrier(0);
        q8_fold<WARM>(c, txid, txr, off, b, n, n_entries, rA, rB, sA, sB, ctA, ctB, sum, cnt,
                      first_excl, first_err, noR);
    }
}

// scan_key_q8 for a key whose entries carry different DC sets (presence
// masks, D = 8): the quad rows as above plus each op's mask word (lane = op,
// loaded with the effects), which the lanes holding its parts read with one
// shuffle per load.  The dict fold of is_op_in_snapshot (:236-258) per part:
// a DC of the op missing from R (rm) excludes it, absent DCs are not
// compared, SCT's absent DCs are 0 in sA / sB; LastOpCt takes each included
// op's present DCs only, and um (lane = op) collects the included ops' sets.
template <bool WARM>
__device__ __forceinline__ void scan_key_q8_msk(
    const uint64_t *__restrict__ oc, const uint64_t *__restrict__ oc_mask,
    const int64_t *__restrict__ eff, const uint64_t *__restrict__ txid, uint64_t txr,
    uint64_t off, uint64_t n, uint64_t n_entries, uint64_t rA, uint64_t rB, uint64_t sA,
    uint64_t sB, uint64_t rm, uint64_t &ctA, uint64_t &ctB, uint64_t &um, int64_t &sum,
    uint32_t &cnt, int64_t &first_excl, int64_t &first_err) {
    const int lane = lane_id();
    const int q = lane >> 2, p = lane & 3;
    const uint64_t lim_e = n_entries - 1u;
    for (uint64_t b = 0; b < n; b += AGN_WAVE) {
        const Q8Chunk c = q8_load<true, false>(oc, eff, off, b, n_entries);
        uint64_t e = off + b + (uint64_t)lane;
        e = e < lim_e ? e : lim_e;
        const uint32_t m = (uint32_t)(oc_mask ? oc_mask[e] : 0xFFull) & 0xFFu;
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t valid = (n - b >= (uint64_t)AGN_WAVE) ? ~0ull : ((1ull << (n - b)) - 1ull);
        // ops with a DC missing from R
        const uint64_t noR = ballot((m & ~(uint32_t)rm) != 0u);
        uint64_t bad = noR, gt = 0, pres[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t mq = (uint32_t)__shfl((int)m, 16 * j + q, AGN_WAVE);
            pres[j] = mq;
            const bool pa = (mq >> (2 * p)) & 1u, pb = (mq >> (2 * p + 1)) & 1u;
            bad |= nib_any16(ballot((pa && c.x[j].x > rA) || (pb && c.x[j].y > rB))) << (16 * j);
            if (WARM)
                gt |= nib_any16(ballot((pa && c.x[j].x > sA) || (pb && c.x[j].y > sB))) << (16 * j);
        }
        uint64_t nip = WARM ? gt : ~0ull;
        if (txid != nullptr) nip |= ballot(txid[e] == txr);
        const uint64_t incl = valid & nip & ~bad, excl = valid & nip & bad;
        if (first_excl < 0 && excl) first_excl = (int64_t)b + (int64_t)__builtin_ctzll(excl);
        cnt += (uint32_t)__builtin_popcountll(incl);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool in = ((incl >> (16 * j + q)) & 1ull) != 0ull;
            const bool pa = (pres[j] >> (2 * p)) & 1u, pb = (pres[j] >> (2 * p + 1)) & 1u;
            ctA = (in && pa && c.x[j].x > ctA) ? c.x[j].x : ctA;
            ctB = (in && pb && c.x[j].y > ctB) ? c.x[j].y : ctB;
        }
        const bool mine = ((incl >> lane) & 1ull) != 0ull;
        um |= mine ? (uint64_t)m : 0ull;
        const bool badv = mine && c.ev == AGN_EFFECT_INVALID;
        if (first_err < 0) {
            const uint64_t be = ballot(badv);
            if (be) first_err = (int64_t)b + (int64_t)__builtin_ctzll(be);
        }
        sum += (mine && !badv) ? c.ev : 0;
    }
}

}  // namespace
}  // namespace agn
