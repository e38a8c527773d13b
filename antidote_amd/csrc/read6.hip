// read6.hip — materializer_vnode:read/6 for a batch of distinct keys in ONE
// kernel (the cached read batcher's path for counter_pn, D <= 8, dense clocks
// or presence-masked ones as the Erlang NIF's partitions carry).  One wave per request, the key's cache slots in registers:
//   1. get_from_snapshot_cache (src/materializer_vnode.erl:384-413,
//      vector_orddict:get_smaller src/vector_orddict.erl:74-87): a ballot of
//      "slot > R" folded per slot on the scalar unit, SCT and the base value
//      read out of the slot registers;
//   2. materialize/4 from that base (src/clocksi_materializer.erl:82-268):
//      the dense counter scan (counter_scan.hpp), SCT and R in SGPRs; D = 8
//      scans quad rows with the first chunk issued with the slot loads;
//   3. the cache half of materialize_snapshot / internal_store_ss /
//      insert_bigger / snapshot_insert_gc (:341-364, 466-563): the shift and
//      the GC threshold from the slot registers.
// Same results as the batched kernels k_ss_lookup -> k_counter_key ->
// k_ss_store (cache_dev.hpp, per-request prune flags), in one launch instead
// of three kernels and two copies: for the read batcher requests are read
// from, and results written to, device-visible pinned host memory;
// agn_read_cached runs it over device arrays (for D < 8 below 2^15 requests).
#include <type_traits>

#include "cache_dev.hpp"
#include "counter_scan.hpp"
#include "filter.hpp"
#include "serve.hpp"

namespace agn {
namespace {

// The key's cache slots in registers, lane l = slot (l / DCP) + SPR r of
// register r, DC l % DCP: every slot the lookup compares and the store
// shifts is read by one batch of loads, issued before the log scan, and
// written back from the lane that read it -- the batched kernels' group loops
// (cache_dev.hpp) walk the slots one dependent load at a time, which a wave
// serving one request cannot hide.  A cache written by these entry points
// holds at most SNAPSHOT_THRESHOLD - 1 entries per key; NSLOT bounds the
// slots read.
constexpr uint32_t NSLOT = 16;

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, AGN_WAVE);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, AGN_WAVE);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// MSK: presence masks (the logs the Erlang NIF builds, one word per clock for
// D <= 8).  The lookup and the store's le / min follow vectorclock on dicts
// (a DC missing from a clock reads 0; cache_dev.hpp grp_le / ss_store_one);
// the scan routes the key as k_counter_key's MSK instantiations do: a key
// whose entries share one DC set U inside R's runs the dense scan with R and
// SCT neutralised (+inf) outside U, a mixed key the per-entry-mask scan.
//
// NP requests per wave (1 or 2).  A request is a chain of dependent round
// trips -- its key, then the key's slot count and segment, then the slots
// and the first chunk of rows.  With NP = 2 each stage's loads are issued
// for both requests before either waits, and the second request's slots and
// rows stay in flight while the first is served.  Stages: r6_meta (scalar:
// slot count, segment, type, presence words, TxId; vector: R), r6_rows (the
// slots, chunk 0), r6_serve.  Measured (10M warm reads at D = 8, one
// process; profiles/r05/ab_read6_*): the pair (127 VGPRs,
// 4 waves per SIMD) gains nothing; what did: R as per-lane vector loads
// instead of 16 uniform words (they sat in SGPRs beside the kernel's
// arguments and spilled), the lookup's first-clear-slot search in spread
// form, the per-key words through the scalar cache, and a 6-wave register
// budget -- 12.2 -> 9.45 ms, under the three batched kernels' 9.70.
template <int D, bool MSK>
struct R6Req {
    static constexpr int DCP = D <= 1 ? 1 : D <= 2 ? 2 : D <= 4 ? 4 : 8;  // pow2 >= D
    static constexpr int SPR = AGN_WAVE / DCP;                             // cache slots per register
    static constexpr int NR = (int)((NSLOT + SPR - 1) / SPR);
    uint64_t i, key, off, n, kmw, rmw, txv;
    uint32_t n0, nv, id0, kty;
    uint64_t r[D < 8 ? D : 1];  // D < 8: R as uniform words (the row-per-lane scan's compare)
    uint64_t rd;                // per lane: R at this lane's DC (the lookup's compare)
    u64x2 rq;                   // D = 8, per lane: R at DCs 2p, 2p+1 (p = lane & 3)
    uint64_t clk[NR], cmk[NR];  // the key's cache slots (lane = slot x DC)
    int64_t lop, val;           // slot lane: its last op and value
    Q8Chunk ch0;                // D = 8: the log's first 64-op chunk
    uint64_t row0[D < 8 ? D : 1];  // D < 8: chunk 0's row of this lane's op (lane = op)
    int64_t ev0;                   // and its effect
};

template <int D, bool MSK, class KA>
__device__ __forceinline__ void r6_meta(R6Req<D, MSK> &q, KA &k) {
    const auto &c = k.c;
    const auto &a = k.a;
    const int lane = lane_id();
    const int dl = lane % R6Req<D, MSK>::DCP;
    const uint64_t i = q.i, key = q.key;
    // the key's slot count through the scalar cache with the segment words
    // (one wait for all): this launch writes c.n, but only key's own wave
    // writes c.n[key], after this read (a batch names distinct keys), and the
    // scalar cache starts every launch empty
    q.n0 = __builtin_amdgcn_readfirstlane(ldc(c.n + key));
    if constexpr (D < 8) {
#pragma unroll
        for (int j = 0; j < D; ++j) q.r[j] = uniform_u64(ldc(a.R + i * D + j));
    }
    q.rd = a.R[i * D + (uint64_t)(dl < D ? dl : D - 1)];
    if constexpr (D == 8) q.rq = *reinterpret_cast<const u64x2 *>(a.R + i * D + 2u * (lane & 3));
    // MSK: the key's DC set and R's, with the metadata (unconditional, from a
    // dummy word when absent: a conditional scalar load waits on its own)
    q.kmw = q.rmw = 0ull;
    if constexpr (MSK) {
        q.kmw = uniform_u64(ldc(a.key_mask ? a.key_mask + key : a.R));
        q.rmw = uniform_u64(ldc(a.R_mask ? a.R_mask + i : a.R));
    }
    const KeyMeta km = key_meta(key, a.key_off, a.key_len, a.key_id0);
    q.off = km.off;
    q.n = km.n;
    q.id0 = km.id0;
    // key_type (corrupted_ops_cache, read before any store) and the TxId:
    // unconditional, from dummy addresses when absent
    q.kty = byte_of(a.key_type ? a.key_type : reinterpret_cast<const uint8_t *>(a.key_off), key);
    q.txv = uniform_u64(ldc((a.txid ? a.txid : a.R) + i));
}

template <int D, bool MSK, class KA>
__device__ __forceinline__ void r6_rows(R6Req<D, MSK> &q, KA &k) {
    const auto &c = k.c;
    const auto &a = k.a;
    using Q = R6Req<D, MSK>;
    constexpr uint64_t FULL = (1ull << D) - 1ull;
    const int lane = lane_id();
    const int dl = lane % Q::DCP, jl = lane / Q::DCP;
    const uint64_t key = q.key;
    const uint32_t S = c.slots;
    const uint32_t nv = q.n0 < NSLOT ? q.n0 : NSLOT;
    q.nv = nv;
    // the key's cache slots (rows past nv re-read slot 0: same lines, unused)
    const int dc = dl < D ? dl : D - 1;
#pragma unroll
    for (int r = 0; r < Q::NR; ++r) {
        const uint32_t j = (uint32_t)(jl + r * Q::SPR);
        q.clk[r] = c.clock[(key * S + (j < nv ? j : 0u)) * D + (uint64_t)dc];
    }
    // MSK: each slot's DC set (one word per slot; the slot's lanes share it)
#pragma unroll
    for (int r = 0; r < Q::NR; ++r) {
        const uint32_t j = (uint32_t)(jl + r * Q::SPR);
        q.cmk[r] = (MSK && c.clock_mask) ? (c.clock_mask[key * S + (j < nv ? j : 0u)] & FULL) : FULL;
    }
    const uint32_t ls = (uint32_t)lane < nv ? (uint32_t)lane : 0u;
    q.lop = c.last_op[key * S + ls];
    q.val = c.value[key * S + ls];
    // D = 8: the log's first chunk is in flight with the slots.  Unconditional
    // (an empty key reads its own slot 0 instead): a load under a branch makes
    // the wait for the slots at the join wait for the chunk too.
    if constexpr (D == 8) {
        const bool has = q.n != 0;
        q.ch0 = q8_load<true, false>(has ? a.oc : c.clock + key * S * D,
                                     has ? a.eff : c.value + key * S, has ? q.off : 0ull, 0,
                                     has ? a.n_entries : 1ull);
    } else {
        // D < 8: chunk 0 row per lane (lane = op; the dense scan's first
        // step), clamped to the key's first entry past its end, or to the
        // key's own slot rows when it has no ops -- one wait with the slots
        // instead of a row round trip after the lookup (D = 3: the batched
        // kernels ran 1.08-1.10x faster in bulk without it)
        const bool has = q.n != 0;
        const uint64_t p = (uint64_t)lane < q.n ? (uint64_t)lane : 0ull;
        const uint64_t *rp = has ? a.oc + (q.off + p) * D : c.clock + key * S * D;
        load_row<D, false>(rp, q.row0);
        q.ev0 = has ? a.eff[q.off + p] : c.value[key * S];
    }
}

template <int D, bool MSK, class KA>
__device__ __forceinline__ void r6_serve(R6Req<D, MSK> &q, KA &k,
                                         uint64_t (&stage)[R6Req<D, MSK>::DCP][AGN_WAVE]) {
    const auto &c = k.c;
    const auto &a = k.a;
    using Q = R6Req<D, MSK>;
    constexpr uint64_t FULL = (1ull << D) - 1ull;
    constexpr int DCP = Q::DCP, V = DCP, SPR = Q::SPR, NR = Q::NR;
    const int lane = lane_id();
    const int dl = lane % DCP, jl = lane / DCP;  // this lane's DC and slot
    const uint64_t i = q.i, key = q.key, off = q.off, n = q.n;
    const uint32_t S = c.slots, n0 = q.n0, nv = q.nv;
    const uint64_t Rm = (MSK && a.R_mask) ? (q.rmw & FULL) : FULL;
    const bool corrupt = n != 0 && a.key_type != nullptr && q.kty != (a.req_type & 0xffu);

    // 1. get_from_snapshot_cache: the first slot <= R (vector_orddict:get_smaller)
    uint64_t rd = q.rd;
    if (MSK && !((Rm >> dl) & 1ull)) rd = 0ull;  // a DC missing from R reads 0
    uint32_t st, is_first;
    bool sct_ign;
    int64_t base = 0;
    // SCT (the hit slot's clock): D < 8 as uniform words, D = 8 this lane's
    // pair of DCs 2p, 2p+1
    uint64_t s[D < 8 ? D : 1];
#pragma unroll
    for (int j = 0; j < (D < 8 ? D : 1); ++j) s[j] = 0ull;
    uint64_t sqA = 0ull, sqB = 0ull;
    // slots of nv with no DC above R, per register in spread form (bit g
    // DCP: slot r SPR + g) -- a first-zero-group search on five scalar
    // operations where the packed fold took ~30; ahead of the branch below,
    // so the wait for the slots is not also the wait for chunk 0's rows
    uint64_t okz[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const bool pres = !MSK || ((q.cmk[r] >> dl) & 1ull) != 0ull;
        const uint64_t gt = group_any_spread<DCP>(ballot(dl < D && pres && q.clk[r] > rd));
        const uint32_t lo = (uint32_t)(r * SPR);
        const uint32_t cv = nv > lo ? (nv - lo < (uint32_t)SPR ? nv - lo : (uint32_t)SPR) : 0u;
        okz[r] = ~gt & group_base<DCP>() & low_bits((uint64_t)cv * DCP);
    }
    uint64_t smw = FULL;  // SCT's DC set (the hit slot's)
    uint32_t n1 = nv;  // the key's entries after the lookup
    if (n0 == 0) {     // absent: store the empty snapshot at vectorclock:new() (:395-402)
        if (lane < D) c.clock[(key * S) * D + (uint64_t)lane] = 0ull;
        if (lane == 0) {
            c.last_op[key * S] = 0;
            c.value[key * S] = 0;
            c.n[key] = 1;
            if (MSK && c.clock_mask) c.clock_mask[key * S] = 0ull;
        }
        q.clk[0] = jl == 0 ? 0ull : q.clk[0];
        if (MSK && c.clock_mask) q.cmk[0] = jl == 0 ? 0ull : q.cmk[0];
        smw = 0ull;
        q.lop = lane == 0 ? 0 : q.lop;
        q.val = lane == 0 ? 0 : q.val;
        n1 = 1;
        st = AGN_SS_NEW;
        is_first = 1;
        sct_ign = true;
    } else {
        int f = -1;  // the first slot <= R
#pragma unroll
        for (int r = NR - 1; r >= 0; --r)
            if (okz[r]) f = r * SPR + __builtin_ctzll(okz[r]) / DCP;
        if (f >= 0) {
            const int fr = f / SPR, l0 = (f % SPR) * DCP;
            if constexpr (D == 8) {
                const int p = lane & 3;
                uint64_t v = q.clk[0];
                if constexpr (NR > 1) v = fr ? q.clk[1] : v;
                sqA = shfl_u64(v, l0 + 2 * p);
                sqB = shfl_u64(v, l0 + 2 * p + 1);
            } else {
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    uint64_t v = readlane_u64(q.clk[0], l0 + j);
                    if constexpr (NR > 1) v = fr ? readlane_u64(q.clk[1], l0 + j) : v;
                    s[j] = v;
                }
            }
            base = (int64_t)readlane_u64((uint64_t)q.val, f);
            if constexpr (MSK) {
                uint64_t mw = readlane_u64(q.cmk[0], l0);
                if constexpr (NR > 1) mw = fr ? readlane_u64(q.cmk[1], l0) : mw;
                smw = mw;
            }
            st = AGN_SS_HIT;
            is_first = f == 0;
            sct_ign = false;
        } else {
            st = AGN_SS_LOG;
            is_first = 0;
            sct_ign = true;
        }
    }

    // 2. materialize/4 from the base (k_counter_key's body)
    if (corrupt) {
        if (lane == 0) {
            a.value[i] = 0;
            a.hole[i] = 0;
            a.count[i] = 0;
            a.flags[i] = AGN_F_ERR_CORRUPTED;
            a.err_pos[i] = 0xffffffffu;
            a.status[i] = (uint8_t)st;
            a.prune[i] = 0;
            if (a.dkeys) a.dkeys[i] = key;
            if (a.dprune) a.dprune[i] = 0;
        }
        if (lane < D) a.lastct[i * D + (uint64_t)lane] = 0ull;
        if (MSK && a.lastct_mask && lane == 0) a.lastct_mask[i] = 0ull;
        return;
    }
    // MSK: U, the DC set every entry of the key carries (0 = they differ), and
    // whether the dense scan serves the key exactly (no ops, or U inside R's)
    uint64_t U = FULL, Sm = FULL;
    bool uni = true;
    if constexpr (MSK) {
        U = a.oc_mask ? (a.key_mask ? (q.kmw & FULL) : 0ull) : FULL;
        Sm = smw & FULL;
        uni = n == 0 || (U != 0ull && (U & ~Rm) == 0ull);
    }
    const uint64_t txr = a.txid ? q.txv : 0ull;
    const uint64_t *tx = (txr != 0ull) ? a.log_txid : nullptr;
    int64_t sum = 0, first_excl = -1, first_err = -1;
    uint32_t cnt = 0;
    uint64_t um = 0;  // MSK, mixed key: DCs of the included ops (per lane)
    uint64_t ct[D < 8 ? D : 1];
    uint64_t ctA = 0, ctB = 0;  // D = 8: quad rows, LastOpCt of DCs 2p, 2p+1 (p = lane & 3)
    if constexpr (D == 8) {
        // e = SCT as a dict read (missing DC = 0), where LastOpCt starts
        // (materialize/4 :94-95); r / s = the compare values: +inf outside U
        // on the dense scan of a masked key
        const int p = lane & 3;
        const bool inA = ((U >> (2 * p)) & 1ull) != 0ull, inB = ((U >> (2 * p + 1)) & 1ull) != 0ull;
        const uint64_t eA = (sct_ign || !((Sm >> (2 * p)) & 1ull)) ? 0ull : sqA;
        const uint64_t eB = (sct_ign || !((Sm >> (2 * p + 1)) & 1ull)) ? 0ull : sqB;
        const uint64_t sA = (MSK && uni && !inA) ? ~0ull : eA;
        const uint64_t sB = (MSK && uni && !inB) ? ~0ull : eB;
        const uint64_t rA = (MSK && uni && !inA) ? ~0ull : q.rq.x;
        const uint64_t rB = (MSK && uni && !inB) ? ~0ull : q.rq.y;
        ctA = eA;
        ctB = eB;
        if (n != 0 && MSK && !uni) {
            // a mixed key: the quad rows with each op's mask word (chunk 0
            // is read again with its masks)
            if (sct_ign)
                scan_key_q8_msk<false>(a.oc, a.oc_mask, a.eff, tx, txr, off, n, a.n_entries, rA, rB,
                                       sA, sB, Rm, ctA, ctB, um, sum, cnt, first_excl, first_err);
            else
                scan_key_q8_msk<true>(a.oc, a.oc_mask, a.eff, tx, txr, off, n, a.n_entries, rA, rB,
                                      sA, sB, Rm, ctA, ctB, um, sum, cnt, first_excl, first_err);
        } else if (n != 0) {
#define AGN_R6Q(W)                                                                             \
    q8_fold<W>(q.ch0, tx, txr, off, 0, n, a.n_entries, rA, rB, sA, sB, ctA, ctB, sum, cnt,     \
               first_excl, first_err);                                                         \
    scan_key_q8<W, true, false, true>(a.oc, a.eff, tx, txr, off, n, a.n_entries, rA, rB, sA, sB, \
                                      ctA, ctB, sum, cnt, first_excl, first_err)
            if (sct_ign) {
                AGN_R6Q(false);
            } else {
                AGN_R6Q(true);
            }
#undef AGN_R6Q
            if (MSK) {  // outside U: SCT's value (an op's row there is not in its dict)
                ctA = inA ? ctA : eA;
                ctB = inB ? ctB : eB;
            }
        }
    } else {
        uint64_t e[D], rc[D], sc[D];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const bool inU = ((U >> j) & 1ull) != 0ull;
            e[j] = (sct_ign || !((Sm >> j) & 1ull)) ? 0ull : s[j];
            sc[j] = (MSK && uni && !inU) ? ~0ull : e[j];
            rc[j] = (MSK && uni && !inU) ? ~0ull : q.r[j];
            ct[j] = e[j];
        }
        if (MSK && !uni) {
            if (sct_ign)
                scan_key_msk<D, false>(a.oc, a.oc_mask, a.eff, tx, txr, off, n, rc, sc, Rm, ct, um,
                                       sum, cnt, first_excl, first_err);
            else
                scan_key_msk<D, true>(a.oc, a.oc_mask, a.eff, tx, txr, off, n, rc, sc, Rm, ct, um,
                                      sum, cnt, first_excl, first_err);
        } else if (n != 0) {
            // chunk 0 from the rows r6_rows issued, then the key's later chunks
            const uint64_t p0 = (uint64_t)lane < n ? (uint64_t)lane : 0ull;
            auto walk = [&](auto warm) {
                constexpr bool WM = decltype(warm)::value;
                scan_chunk<D, WM>(q.row0, q.ev0, (uint64_t)lane < n, 0, tx, txr, off + p0, rc, sc,
                                  ct, sum, cnt, first_excl, first_err);
                for (uint64_t b = AGN_WAVE; b < n; b += AGN_WAVE) {
                    const uint64_t pos = b + (uint64_t)lane;
                    const bool valid = pos < n;
                    const uint64_t e = off + (valid ? pos : 0ull);
                    uint64_t o[D];
                    load_row<D, false>(a.oc + e * D, o);
                    scan_chunk<D, WM>(o, a.eff[e], valid, b, tx, txr, e, rc, sc, ct, sum, cnt,
                                      first_excl, first_err);
                }
            };
            if (sct_ign) walk(std::false_type{});
            else walk(std::true_type{});
            if (MSK) {
#pragma unroll
                for (int j = 0; j < D; ++j) ct[j] = ((U >> j) & 1ull) ? ct[j] : e[j];
            }
        }
    }
    int64_t hid;
    {
        const uint64_t pos = first_excl >= 0 ? (uint64_t)first_excl : n - 1;
        if (q.id0 != AGN_ID0_NONE)  // op_id[off + pos] == id0 + pos (agn_log_index_ids)
            hid = n ? (int64_t)((uint64_t)q.id0 + pos) : 0;
        else
            hid = n ? (int64_t)a.op_id[uniform_u64(off + pos)] : 0;
    }
    const int64_t total = wave_sum_dpp(sum);
    const bool ct_ign = sct_ign && cnt == 0u;
    uint64_t ctl;  // LastOpCt of DC dl on every lane
    if constexpr (D == 8) {
        // the 16 lanes of each part fold by xor-shuffles; lanes 0..3 hold the row
#pragma unroll
        for (int x = 4; x < AGN_WAVE; x <<= 1) {
            ctA = umax64(ctA, shfl_xor_u64(ctA, x));
            ctB = umax64(ctB, shfl_xor_u64(ctB, x));
        }
        if (ct_ign) ctA = ctB = 0ull;
        if (lane < 4) {
            u64x2 v;
            v.x = ctA;
            v.y = ctB;
            reinterpret_cast<u64x2 *>(a.lastct + i * D)[lane] = v;
        }
        const uint64_t xa = shfl_u64(ctA, dl >> 1), xb = shfl_u64(ctB, dl >> 1);
        ctl = (dl & 1) ? xb : xa;
    } else {
        // LastOpCt: per-lane maxima -> LDS [DCP][64] -> each lane folds V slots
        // of one DC -> xor-shuffle across the 64/DCP lanes that share it
#pragma unroll
        for (int j = 0; j < D; ++j) stage[j][lane] = ct[j];
        __syncthreads();
        uint64_t m = 0;
        if (dl < D) {
#pragma unroll
            for (int v = 0; v < V; ++v) m = umax64(m, stage[dl][jl * V + v]);
        }
        __syncthreads();  // NP = 2: the next request writes stage
#pragma unroll
        for (int x = DCP; x < AGN_WAVE; x <<= 1) m = umax64(m, shfl_xor_u64(m, x));
        ctl = ct_ign ? 0ull : m;
        if (jl == 0 && dl < D) a.lastct[i * D + (uint64_t)dl] = ctl;
    }
    // LastOpCt's DC set: SCT's united with the included ops' (U, or the
    // per-lane sets of a mixed key)
    uint64_t mo = FULL;
    if constexpr (MSK) {
        const uint64_t un = uni ? (cnt ? U : 0ull) : wave_or_bits<D>(um);
        mo = ct_ign ? 0ull : ((sct_ign ? 0ull : Sm) | un);
    }
    // NewLastOp = id(oldest excluded) - 1, else get_first_id (:49-63)
    const int64_t hole = first_excl >= 0 ? hid - 1 : hid;
    uint32_t fl = 0;
    if (cnt) fl |= AGN_F_NEWSS;
    if (ct_ign) fl |= AGN_F_CT_IGNORE;
    if (first_err >= 0) fl |= AGN_F_ERR_UNEXPECTED;
    const int64_t value = (int64_t)((uint64_t)base + (uint64_t)total);

    // 3. internal_store_ss / insert_bigger / snapshot_insert_gc (cache_dev.hpp
    //    ss_store_one on the register copy of the slots)
    const bool gc = a.gc != nullptr && a.gc[i] != 0;
    bool pr = false;
    const bool refresh = (fl & AGN_F_NEWSS) && is_first && cnt >= AGN_MIN_OP_STORE_SS;
    const int64_t lop0 = (int64_t)readlane_u64((uint64_t)q.lop, 0);
    if (st != AGN_SS_LOG && n != 0 && !(fl & (AGN_F_ERR_UNEXPECTED | AGN_F_CT_IGNORE)) &&
        (refresh || gc) && (hole - lop0 >= AGN_MIN_OP_STORE_SS || gc)) {
        // insert_bigger: prepend iff not le(LastOpCt, head clock) (dicts: DCs
        // of LastOpCt only, the head's missing ones read 0)
        const bool inct = !MSK || ((mo >> dl) & 1ull) != 0ull;
        const uint64_t hv = (!MSK || ((q.cmk[0] >> dl) & 1ull)) ? q.clk[0] : 0ull;
        const bool prepend = (ballot(jl == 0 && dl < D && inct && ctl > hv) & low_bits(DCP)) != 0ull;
        const uint32_t size1 = n1 + (prepend ? 1u : 0u);
        const bool collect = size1 >= AGN_SNAPSHOT_THRESHOLD || gc;
        uint32_t kept = n1;
        if (collect) kept = prepend ? (n1 < AGN_SNAPSHOT_MIN - 1 ? n1 : AGN_SNAPSHOT_MIN - 1)
                                    : (n1 < AGN_SNAPSHOT_MIN ? n1 : AGN_SNAPSHOT_MIN);
        const uint32_t new_n = kept + (prepend ? 1u : 0u);
        uint64_t m = ~0ull, pm = 0ull;  // CommitTime: min (missing = 0), its DC set
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const uint32_t j = (uint32_t)(jl + r * SPR);
            if (j < kept) {
                if (prepend && dl < D) c.clock[(key * S + j + 1) * D + (uint64_t)dl] = q.clk[r];
                if (MSK && c.clock_mask && prepend && dl == 0) c.clock_mask[key * S + j + 1] = q.cmk[r];
                const uint64_t v = (!MSK || ((q.cmk[r] >> dl) & 1ull)) ? q.clk[r] : 0ull;
                m = v < m ? v : m;
                pm |= q.cmk[r];
            }
        }
        if (prepend) {
            if ((uint32_t)lane < kept) {
                c.last_op[key * S + (uint64_t)lane + 1] = q.lop;
                c.value[key * S + (uint64_t)lane + 1] = q.val;
            }
            if (jl == 0 && dl < D) c.clock[(key * S) * D + (uint64_t)dl] = ctl;
            if (lane == 0) {
                c.last_op[key * S] = hole;
                c.value[key * S] = value;
                if (MSK && c.clock_mask) c.clock_mask[key * S] = mo;
            }
            const uint64_t v = inct ? ctl : 0ull;
            m = v < m ? v : m;
            pm |= mo;
        }
        if (collect) {  // CommitTime = vectorclock:min of the kept clocks (:523-527)
#pragma unroll
            for (int x = DCP; x < AGN_WAVE; x <<= 1) {
                const uint64_t o = shfl_xor_u64(m, x);
                m = o < m ? o : m;
                if (MSK) pm |= shfl_xor_u64(pm, x);
            }
            // a DC no kept clock has: 0 (and absent from the threshold's set)
            if (MSK && !((pm >> dl) & 1ull)) m = 0ull;
            if (jl == 0 && dl < D) a.thr[key * D + (uint64_t)dl] = m;
            if (MSK && a.thrm && lane == 0) a.thrm[key] = pm & FULL;
        }
        if (lane == 0) c.n[key] = new_n;
        pr = collect;
    }
    if (lane == 0) {
        a.value[i] = value;
        a.hole[i] = hole;
        a.count[i] = cnt;
        a.flags[i] = fl;
        a.err_pos[i] = first_err >= 0 ? (uint32_t)(off + (uint64_t)first_err) : 0xffffffffu;
        a.status[i] = (uint8_t)st;
        a.prune[i] = pr ? 1 : 0;
        if (MSK && a.lastct_mask) a.lastct_mask[i] = mo;
        if (a.dkeys) a.dkeys[i] = key;
        if (a.dprune) a.dprune[i] = pr ? 1 : 0;
    }
}

// The kernel's parameters (~400 bytes) are read through the kernarg segment
// pointer at each stage (kp(): an opaque copy, so a stage's loads are
// neither hoisted to the kernel's entry nor shared with another stage's):
// as by-value arguments they were all loaded at the entry and held in SGPRs
// for the whole kernel, which spilled 34 of them to VGPR lanes (now 0; 84
// VGPRs instead of 89; by itself 10.88 vs 10.90 ms for 10M warm reads, but
// it is what lets the 6-wave budget below fit).
struct R6Params {
    agn_ss_cache c;
    Read6Args a;
    uint32_t xcd;
};
using R6K = const __attribute__((address_space(4))) R6Params;
__device__ __forceinline__ R6K &kp() { return kparams<R6Params>(); }

// One request per wave on a dense log: a budget of 6 waves per SIMD (80
// VGPRs, 4 spilled to scratch outside the scan; 84 and 5 waves without it):
// 10M warm reads 9.53 against 10.23 ms, under the batched kernels' 9.68
// (profiles/r05/ab_read6_cfg2_10M_w6.log).  The masked form would spill 38.
template <int D, bool MSK, int NP>
__global__ __launch_bounds__(64, (NP == 1 && !MSK) ? 6 : 1) void k_read6(R6Params) {
    using Q = R6Req<D, MSK>;
    __shared__ uint64_t stage[Q::DCP][AGN_WAVE];
    R6K &k0 = kp();
    const uint32_t blk = block_order(k0.xcd, blockIdx.x, gridDim.x);
    const uint64_t n_req = k0.a.n_req;
    const uint64_t i0 = (uint64_t)blk * NP;
    if (i0 >= n_req) return;
    Q q[NP];
    // a missing second request (odd batch) re-reads the first's and is not served
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        q[p].i = i0 + (uint64_t)p < n_req ? i0 + (uint64_t)p : i0;
        q[p].key = uniform_u64(ldc(k0.a.keys + q[p].i));
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) r6_meta(q[p], kp());
#pragma unroll
    for (int p = 0; p < NP; ++p) r6_rows(q[p], kp());
#pragma unroll
    for (int p = 0; p < NP; ++p)
        if (p == 0 || i0 + (uint64_t)p < n_req) r6_serve(q[p], kp(), stage);
}

// read/6 for clocks of 9 .. 64 DCs (D > 8 has no register-resident dense
// scan): one wave per request runs get_from_snapshot_cache on all 64 lanes
// (cache_dev.hpp ss_lookup_one, the SCT row into device scratch), the general
// per-key filter + counter fold from that base (filter.hpp KeyFilter, as
// mat_counter.hip's k_counter: DPL DCs per lane, LPO lanes per op, per-entry
// masks when SPARSE) and materialize_snapshot's store (ss_store_one) -- one
// launch where the batcher otherwise runs lookup -> materialize -> store as
// three kernels around two copies.  Same results as that sequence.
template <int DPL, int LPO, bool SPARSE>
__global__ __launch_bounds__(64) void k_read6w(agn_ss_cache c, Read6Args a) {
    using F = KeyFilter<DPL, LPO, SPARSE>;
    __shared__ uint64_t stage[DPL][AGN_WAVE];
    const uint64_t i = blockIdx.x;
    if (i >= a.n_req) return;
    const int lane = lane_id();
    const uint32_t D = a.n_dcs, W = n_words(D);
    const uint64_t key = uniform_u64(a.keys[i]);
    agn_log log;
    __builtin_memset(&log, 0, sizeof log);
    log.crdt_type = AGN_COUNTER_PN;
    log.n_dcs = D;
    log.n_entries = a.n_entries;
    log.key_off = a.key_off;
    log.key_len = a.key_len;
    log.key_type = a.key_type;
    log.oc = a.oc;
    log.oc_mask = SPARSE ? a.oc_mask : nullptr;
    log.op_id = a.op_id;
    log.txid = a.log_txid;
    log.eff = a.eff;
    agn_read rq;
    __builtin_memset(&rq, 0, sizeof rq);
    rq.n_req = a.n_req;
    rq.keys = a.keys;
    rq.R = a.R;
    rq.R_mask = SPARSE ? a.R_mask : nullptr;
    rq.sct = a.sct_scr;
    rq.sct_mask = SPARSE ? a.sctm_scr : nullptr;
    rq.sct_ignore = a.ign_scr;
    rq.txid = a.txid;
    rq.req_type = a.req_type;
    // 1. get_from_snapshot_cache (:384-413, vector_orddict:get_smaller)
    const Grp<AGN_WAVE> g;
    const LookupOut lk = ss_lookup_one<AGN_WAVE>(
        g, c, key, a.R + i * D, (SPARSE && a.R_mask) ? a.R_mask + i * W : nullptr,
        a.sct_scr + i * D, (SPARSE && a.sctm_scr) ? a.sctm_scr + i * W : nullptr);
    if (lane == 0) a.ign_scr[i] = lk.ign;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // the filter reads them back
    __builtin_amdgcn_wave_barrier();
    const uint64_t off = uniform_u64(a.key_off[key]);
    const uint64_t n = uniform_u64(key_n(a.key_off, a.key_len, key));
    const uint32_t kty = a.key_type ? __builtin_amdgcn_readfirstlane((uint32_t)a.key_type[key]) : 0u;
    if (n != 0 && a.key_type != nullptr && kty != (a.req_type & 0xffu)) {
        // erlang:error(corrupted_ops_cache) (:190-191): no store
        for (uint32_t d = lane; d < D; d += AGN_WAVE) a.lastct[i * D + d] = 0ull;
        if (lane == 0) {
            a.value[i] = 0;
            a.hole[i] = 0;
            a.count[i] = 0;
            a.flags[i] = AGN_F_ERR_CORRUPTED;
            a.err_pos[i] = 0xffffffffu;
            a.status[i] = (uint8_t)lk.status;
            a.prune[i] = 0;
            if (SPARSE && a.lastct_mask) a.lastct_mask[i] = 0ull;
            if (a.dkeys) a.dkeys[i] = key;
            if (a.dprune) a.dprune[i] = 0;
        }
        return;
    }
    // 2. materialize/4 from the base (mat_counter.hip k_counter's body)
    F f;
    f.init(log, rq, i);
    int64_t sum = 0;
    uint32_t cnt = 0;
    int64_t first_err = -1;
    // the effect is loaded with the rows (not after the verdict: one round
    // trip per iteration)
    for (uint64_t b = 0; b < n; b += F::S::OPI) {
        const uint64_t pos = b + (uint64_t)f.slot;
        int64_t ev = 0;
        if (f.sub == 0 && pos < n) ev = a.eff[off + pos];
        bool valid;
        const bool incl = f.step(log, off, n, b, valid);
        const bool lead = incl && f.sub == 0;
        const bool bad = lead && ev == AGN_EFFECT_INVALID;
        cnt += (uint32_t)__builtin_popcountll(ballot(lead));
        if (first_err < 0) {
            const uint64_t be = ballot(bad);
            if (be) first_err = (int64_t)b + (int64_t)(__builtin_ctzll(be) / LPO);
        }
        sum += (lead && !bad) ? ev : 0;  // ev is loaded for excluded ops too
    }
    const int64_t total = wave_sum_i64(sum);
    const bool ct_ign = f.sct_ign && cnt == 0u;
    agn_result o;
    __builtin_memset(&o, 0, sizeof o);
    o.lastct = a.ct_scr;
    o.lastct_mask = SPARSE ? a.ctm_scr : nullptr;
    f.write_ct(stage, o, i, ct_ign);
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // the store reads the row back
    __builtin_amdgcn_wave_barrier();
    int64_t hid;
    if (f.first_excl >= 0) hid = (int64_t)a.op_id[uniform_u64(off + (uint64_t)f.first_excl)];
    else hid = n ? (int64_t)a.op_id[uniform_u64(off + n - 1)] : 0;
    const int64_t hole = f.first_excl >= 0 ? hid - 1 : hid;
    uint32_t fl = 0;
    if (cnt) fl |= AGN_F_NEWSS;
    if (ct_ign) fl |= AGN_F_CT_IGNORE;
    if (first_err >= 0) fl |= AGN_F_ERR_UNEXPECTED;
    const int64_t value = (int64_t)((uint64_t)lk.base + (uint64_t)total);
    // 3. internal_store_ss / insert_bigger / snapshot_insert_gc (:341-364, 466-563)
    const bool gc = a.gc != nullptr && a.gc[i] != 0;
    const bool pr = ss_store_one<AGN_WAVE>(g, c, key, n, lk.status, lk.first, gc, a.ct_scr + i * D,
                                           SPARSE ? a.ctm_scr + i * W : nullptr, hole, value, cnt,
                                           fl, a.thr, SPARSE ? a.thrm : nullptr);
    for (uint32_t d = lane; d < D; d += AGN_WAVE) a.lastct[i * D + d] = a.ct_scr[i * D + d];
    if (lane == 0) {
        a.value[i] = value;
        a.hole[i] = hole;
        a.count[i] = cnt;
        a.flags[i] = fl;
        a.err_pos[i] = first_err >= 0 ? (uint32_t)(off + (uint64_t)first_err) : 0xffffffffu;
        a.status[i] = (uint8_t)lk.status;
        a.prune[i] = pr ? 1 : 0;
        if (SPARSE && a.lastct_mask) a.lastct_mask[i] = a.ctm_scr[i * W];
        if (a.dkeys) a.dkeys[i] = key;
        if (a.dprune) a.dprune[i] = pr ? 1 : 0;
    }
}

}  // namespace

bool read6_supported(const agn_log &view, uint32_t D) {
    return view.crdt_type == AGN_COUNTER_PN && view.oc_mask == nullptr && D >= 1 && D <= 8;
}

// Requests per wave of k_read6: AGN_READ6_NP=2 takes two (opt-in).  Measured
// against one, in one process (profiles/r05/ab_read6_*): 10M reads at D = 8
// 11.00-11.17 vs 10.88-10.90 ms; 1M at D = 3 0.94-0.96 vs 0.94-0.97 ms.
// AGN_READ6_XCD=1: the XCD-aware block order (xcd_block; 11.59 vs 11.47 ms at
// 10M, off); AGN_READ6_XCD=g >= 2: runs of g blocks per XCD (block_order).
int launch_read6(const agn_ss_cache &c, const Read6Args &a, hipStream_t st) {
    if (a.n_req == 0) return AGN_OK;
    if (a.n_req > 0x7fffffffull) return fail(AGN_ENOTSUP, "read6: batch too large");
    const dim3 grid((unsigned)a.n_req), block(AGN_WAVE);
    const bool msk = a.oc_mask || a.R_mask || c.clock_mask;
    const char *npv = AGN_KNOB("AGN_READ6_NP");
    const bool pair = npv && npv[0] == '2';
    const char *xv = AGN_KNOB("AGN_READ6_XCD");
    const unsigned long xg = xv ? strtoul(xv, nullptr, 10) : 0ul;
    const uint32_t xcd = xg <= 4096ul ? (uint32_t)xg : 0u;
    const dim3 grid2((unsigned)((a.n_req + 1) / 2));
    const R6Params prm{c, a, xcd};
#define AGN_R6(DV)                                                                             \
    if (pair) {                                                                                \
        if (msk) hipLaunchKernelGGL((k_read6<DV, true, 2>), grid2, block, 0, st, prm);          \
        else hipLaunchKernelGGL((k_read6<DV, false, 2>), grid2, block, 0, st, prm);             \
    } else {                                                                                   \
        if (msk) hipLaunchKernelGGL((k_read6<DV, true, 1>), grid, block, 0, st, prm);           \
        else hipLaunchKernelGGL((k_read6<DV, false, 1>), grid, block, 0, st, prm);              \
    }                                                                                          \
    break
#define AGN_R6W(DPL, LPO)                                                                      \
    if (msk) hipLaunchKernelGGL((k_read6w<DPL, LPO, true>), grid, block, 0, st, c, a);          \
    else hipLaunchKernelGGL((k_read6w<DPL, LPO, false>), grid, block, 0, st, c, a);             \
    break
    if (a.n_dcs > 8 && (!a.sct_scr || !a.ign_scr || !a.ct_scr || (msk && (!a.sctm_scr || !a.ctm_scr))))
        return fail(AGN_EINVAL, "read6: D > 8 needs the device scratch");
    switch (a.n_dcs) {
        case 1: AGN_R6(1);
        case 2: AGN_R6(2);
        case 3: AGN_R6(3);
        case 4: AGN_R6(4);
        case 5: AGN_R6(5);
        case 6: AGN_R6(6);
        case 7: AGN_R6(7);
        case 8: AGN_R6(8);
        default:
            if (a.n_dcs <= 16) { AGN_R6W(8, 2); }
            if (a.n_dcs <= 32) { AGN_R6W(8, 4); }
            if (a.n_dcs <= 64) { AGN_R6W(8, 8); }
            return fail(AGN_ENOTSUP, "read6: n_dcs=%u", a.n_dcs);
    }
#undef AGN_R6W
#undef AGN_R6
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

}  // namespace agn
