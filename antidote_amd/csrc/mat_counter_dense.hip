// mat_counter_dense.hip — the counter_pn fast path for dense clocks, D <= 8
// (BASELINE cfg1/cfg2 shapes): the same semantics as k_counter (filter.hpp +
// mat_counter.hip), specialised where the general kernel pays for
// generality:
//   * the read clock R and SCT are wave-uniform: explicit noalias kernel
//     arguments + readfirstlane keep them in SGPRs (s_load, no VGPRs);
//   * no presence masks (every DC present), so "+1 encoding" and per-DC
//     branches disappear;
//   * rows are 16-byte VGPR loads (scan_key); for D = 8 a lane-contiguous
//     "quad rows" variant (scan_key_q8, non-temporal); for even D
//     (scan_key_glds) each chunk of 64 entries is streamed
//     (OpSSCommit rows, effects, op ids) into LDS by non-temporal LDS-DMA
//     (global_load_lds), the fastest pure-read idiom measured (7.1-7.2 TB/s
//     against 6.0 for 16-byte VGPR loads, profiles/r01/ab_read_probe.log),
//     and reads the NewLastOp op id from LDS instead of a dependent load --
//     faster on some boxes, slower on others (counter_variant below);
//   * cold (SCT = ignore) and warm reads run separate loop bodies, so the
//     cold body does one D-wide compare per op, exactly the reference's
//     VC compare count;
//   * the i64 effect sum is reduced with DPP row ops + 4 readlanes;
//   * one wave per request and no loop: the grid is the whole batch, so the
//     wave dispatcher overlaps the dependent round trips of different keys
//     (measured against cross-key software pipelines and grouped streams:
//     profiles/r01/ab_counter_key_per_wave.log, ab_grid_oversubscription.log),
//     in XCD-aware block order (xcd_block: consecutive requests share the
//     lines of the per-request arrays inside one L2);
//   * per-key side values (key_type, sct_ignore, base value) are scalar
//     loads, never vector loads + vmcnt(0).
// HBM bytes per op: 8*D + 8; per key: 8 + 16*D + 32;
// the LDS-DMA path also reads the chunk's 4-byte op ids (+4 per op).
#include <atomic>
#include <cstdlib>
#include <vector>

#include "counter_scan.hpp"

namespace agn {
namespace {

// k_counter_q8e's hand-on sub-lists: count, and the stride of their counters
// (uint32 words: one 128-byte line each)
constexpr uint32_t QL_S = 1024, QL_STRIDE = 32;

// The counter launchers' block order (block_order's mode): the XCD-aware
// order for small batches, else runs of `bulk` blocks per XCD (order_or:
// AGN_XCD_REMAP / AGN_XCD_CHUNK override).  Same-box A/Bs
// (profiles/r06/ab_xcd_chunk.log): dense cfg2 runs of 64 7.57 ms against
// 7.83 identity and 7.92 XCD-aware, warm 7.43 against 7.69; the masked
// q8e in one process 8.02 against 8.18 identity and 8.37 XCD-aware (with
// the bench's hints), its warm two-per-wave form level in every order.
inline uint32_t counter_order(uint64_t n_req, uint32_t bulk) {
    return order_or(n_req < (1ull << 20) ? 1u : bulk);
}
constexpr uint32_t BULK_CHUNK = 64;

struct DenseArgs {
    uint64_t n_req;
    uint64_t n_entries;
    uint32_t req_type;
    uint32_t xcd;  // block_order mode: 0 identity, 1 xcd_block, g >= 2 runs of g per XCD
    uint32_t pair; // 1: D <= 4 keys longer than a chunk walk two chunks per step
    uint32_t qnt;  // quad rows, non-temporal loads: bit 0 rows, bit 1 effects (AGN_COUNTER_QUAD_NT)
    uint32_t hints;  // agn_read.hints (k_counter_q8e / k_counter_quad2)
    uint32_t ql_cap; // k_counter_q8e / q8m: entries per hand-on sub-list
};

// Presence masks of a sparse batch (the MSK instantiations; one word per
// clock, D <= 8): agn_log.key_mask / oc_mask, agn_read.R_mask / sct_mask and
// agn_result.lastct_mask.  Any may be null (= every DC present).
struct MaskArgs {
    const uint64_t *key_mask, *oc_mask, *R_mask, *sct_mask;
    uint64_t *o_mask;
};

// A request of a sparse batch: the DC set U every op of its key carries (0 =
// the entries differ or it is unknown), R's and SCT's DC sets, and whether
// the dense scan serves it exactly (uni: no ops, or U is known and inside R:
// then every compare of is_op_in_snapshot's dict fold is a compare of U's
// columns, src/clocksi_materializer.erl:236-258, and the columns outside U
// are neutralised -- R and SCT read as +inf there, so they never exclude an
// op nor keep it out of the snapshot; LastOpCt keeps SCT's value there).
template <int D>
struct Presence {
    uint64_t U, Rm, Sm;
    bool uni;
};

template <int D, bool MSK>
__device__ __forceinline__ Presence<D> presence(const MaskArgs &m, uint64_t kmw, uint64_t rmw,
                                                uint64_t smw, uint64_t n) {
    constexpr uint64_t FULL = (1ull << D) - 1ull;
    Presence<D> p;
    if constexpr (!MSK) {
        p.U = p.Rm = p.Sm = FULL;
        p.uni = true;
    } else {
        // a log without masks: every entry carries every DC
        p.U = m.oc_mask ? (m.key_mask ? (kmw & FULL) : 0ull) : FULL;
        p.Rm = m.R_mask ? (rmw & FULL) : FULL;
        p.Sm = m.sct_mask ? (smw & FULL) : FULL;
        p.uni = n == 0 || (p.U != 0ull && (p.U & ~p.Rm) == 0ull);
    }
    return p;
}

typedef __attribute__((address_space(3))) void *lds_ptr;

// LDS words per wave of the LDS-DMA path: rows (DCP*64 u64, reused as the
// LastOpCt stage), effects (64 u64), op ids (64 u32).
template <int D>
struct GldsLds {
    static constexpr int DCP = D <= 1 ? 1 : D <= 2 ? 2 : D <= 4 ? 4 : 8;
    static constexpr int ROWS = DCP * AGN_WAVE, EFF = ROWS, OPID = EFF + AGN_WAVE,
                         WORDS = OPID + AGN_WAVE / 2;
};

// scan_key for even D through LDS-DMA: each chunk of 64 log entries is
// fetched by global_load_lds (non-temporal) into the wave's LDS slice --
// D/2 x 1 KiB of OpSSCommit rows (image linear: row of lane l at 8*D*l
// bytes), the effects and the op ids as 4-byte pieces -- then every lane
// reads its row back with ds_read_b128.  Addresses past the end of the log
// are clamped (those lanes are idle).  Returns the op id that defines
// NewLastOp, read from LDS: fetching the chunk's 256 B of op ids with the
// rows (+5.4 % bytes) removes the dependent round trip a scalar load of the
// one id costs after the scan (measured 8.09 -> 7.29 ms on cfg2,
// profiles/r01/ab_counter_glds.log).  Only DMA loads are in flight, so the
// one vmcnt(0) per chunk drains nothing else.
template <int D, bool WARM>
__device__ __forceinline__ int64_t scan_key_glds(
    const uint64_t *__restrict__ oc, const int64_t *__restrict__ eff,
    const uint32_t *__restrict__ op_id, const uint64_t *__restrict__ txid, uint64_t txr,
    uint64_t off, uint64_t n, uint64_t n_entries, const uint64_t (&r)[D],
    const uint64_t (&s)[D], uint64_t (&ct)[D], int64_t &sum, uint32_t &cnt,
    int64_t &first_excl, int64_t &first_err, uint64_t *lds) {
    using L = GldsLds<D>;
    const int lane = lane_id();
    const uint64_t lim_oc = n_entries * D - 2u, lim_e = n_entries * 2u - 1u,
                   lim_id = n_entries - 1u;
    const uint32_t *ids = reinterpret_cast<const uint32_t *>(lds + L::OPID);
    int64_t hid = -1;
    for (uint64_t b = 0; b < n; b += AGN_WAVE) {
        const uint64_t pos = b + (uint64_t)lane;
        const bool valid = pos < n;
        const uint64_t e = off + (valid ? pos : 0ull);
        const uint64_t cb = (off + b) * D;
#pragma unroll
        for (int j = 0; j < D / 2; ++j) {
            uint64_t q = cb + (uint64_t)(j * AGN_WAVE + lane) * 2u;
            q = q < lim_oc ? q : lim_oc;
            __builtin_amdgcn_global_load_lds((const void *)(oc + q), (lds_ptr)(lds + j * 2 * AGN_WAVE),
                                             16, 0, 2 /* nt */);
        }
        const uint32_t *e32 = reinterpret_cast<const uint32_t *>(eff);
#pragma unroll
        for (int j = 0; j < 2; ++j) {  // i64 effects as 2 x 64 dwords
            uint64_t q = (off + b) * 2u + (uint64_t)(j * AGN_WAVE + lane);
            q = q < lim_e ? q : lim_e;
            __builtin_amdgcn_global_load_lds((const void *)(e32 + q),
                                             (lds_ptr)(lds + L::EFF + j * AGN_WAVE / 2), 4, 0, 2);
        }
        {
            uint64_t q = off + b + (uint64_t)lane;
            q = q < lim_id ? q : lim_id;
            __builtin_amdgcn_global_load_lds((const void *)(op_id + q), (lds_ptr)(lds + L::OPID), 4,
                                             0, 2);
        }
        __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0): the DMA has landed
        __builtin_amdgcn_wave_barrier();
        uint64_t o[D];
        const u64x2 *lr = reinterpret_cast<const u64x2 *>(lds + (uint64_t)lane * D);
#pragma unroll
        for (int j = 0; j < D / 2; ++j) {
            const u64x2 x = lr[j];
            o[2 * j] = x.x;
            o[2 * j + 1] = x.y;
        }
        const int64_t ev = (int64_t)lds[L::EFF + lane];
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
            if (bx) {
                first_excl = (int64_t)b + (int64_t)__builtin_ctzll(bx);
                hid = (int64_t)ids[__builtin_ctzll(bx)];
            }
        }
        if (first_excl < 0 && b + AGN_WAVE >= n) hid = (int64_t)ids[(n - 1) - b];  // get_first_id
#pragma unroll
        for (int j = 0; j < D; ++j) ct[j] = (incl && o[j] > ct[j]) ? o[j] : ct[j];
        const bool bad = incl && ev == AGN_EFFECT_INVALID;
        cnt += (uint32_t)__builtin_popcountll(ballot(incl));
        if (first_err < 0) {
            const uint64_t be = ballot(bad);
            if (be) first_err = (int64_t)b + (int64_t)__builtin_ctzll(be);
        }
        sum += (incl && !bad) ? ev : 0;
        __builtin_amdgcn_wave_barrier();  // LDS reads done before the next chunk's DMA
    }
    return hid;
}

// Row-load variants of k_counter_key (bit-identical results; agn_tune picks
// per device): VGPR rows (scan_key), LDS-DMA rows (scan_key_glds, even D),
// quad rows (scan_key_q8, D = 8, non-temporal).
enum { ROWS_VGPR = 0, ROWS_GLDS = 1, ROWS_QUAD = 2, ROWS_QUAD2 = 3 };

// One wave = one request, no loop: the grid is the batch (ceil(n_req / WPB)
// blocks).  Measured on cfg2 this beats every software-pipelined variant
// above: with ~10M short-lived waves the dispatcher keeps every CU's wave
// slots full and the HBM queue deep, while each wave's dependent round trips
// (metadata -> rows -> NewLastOp id) overlap with other waves' instead of
// serialising inside one.  Side values are scalar loads (no vmcnt drains).
// R, key_off, the segment length and the consecutive-id base (key_id0) are
// issued as one group of scalar loads, and with key_id0 the NewLastOp id
// needs no load after the scan: +0.9 % against the previous prologue
// (profiles/r01/ab_counter_prologue.log).  Where the rest of the gap to the
// read ceiling goes (diagnostic builds, scripts/build_diag.sh,
// profiles/r01/ab_counter_attribution.log): not latency -- two requests per
// wave with both keys' rows in flight (2x bytes per wave slot) measured
// +0.2 %, dropping the metadata loads 0.3 % -- but the per-key result
// writes: 92 B per key (1.9 % of the bytes) cost 9 % of the kernel time
// (writing 16 B instead: 8.33 -> 7.57 ms), full 128 B record lines 1 %,
// non-temporal stores +7 % worse.  The HBM read/write turnaround, not the
// instruction stream, is the remaining bound.
template <int D, bool ANY_WARM, int WPB, int VAR, bool KEYS, bool MSK>
__global__ __launch_bounds__(64 * WPB) void k_counter_key(
    DenseArgs a, MaskArgs mk, const uint64_t *__restrict__ keys,
    const uint64_t *__restrict__ key_off, const uint64_t *__restrict__ key_len,
    const uint8_t *__restrict__ key_type, const uint32_t *__restrict__ key_id0,
    const uint64_t *__restrict__ oc, const uint32_t *__restrict__ op_id,
    const int64_t *__restrict__ eff, const uint64_t *__restrict__ log_txid,
    const uint64_t *__restrict__ R, const uint64_t *__restrict__ sct,
    const uint8_t *__restrict__ sct_ignore, const uint64_t *__restrict__ req_txid,
    const int64_t *__restrict__ base_value, int64_t *__restrict__ o_value,
    int64_t *__restrict__ o_hole, uint64_t *__restrict__ o_lastct,
    uint32_t *__restrict__ o_count, uint32_t *__restrict__ o_flags,
    uint32_t *__restrict__ o_err) {
    constexpr int DCP = D <= 1 ? 1 : D <= 2 ? 2 : D <= 4 ? 4 : 8;  // pow2 >= D
    constexpr int V = DCP;                                          // op slots per lane
    constexpr bool GLDS = VAR == ROWS_GLDS;
    constexpr bool QUAD = VAR == ROWS_QUAD && D == 8;
    static_assert(!(MSK && GLDS), "sparse batches use VGPR or quad rows");
    constexpr int LW = GLDS ? GldsLds<D>::WORDS : QUAD ? 1 : DCP * AGN_WAVE;
    __shared__ uint64_t lds_all[WPB][LW];  // GLDS: chunk rows/effects/ids; then the ct stage

    const int lane = lane_id();
    const int w = WPB == 1 ? 0 : (int)(threadIdx.x >> 6);
    // unconditional (as the side loads below): a conditional scalar load is
    // waited for on its own
    const uint32_t blk = block_order(a.xcd, blockIdx.x, gridDim.x);
    const uint64_t i = uniform_u64((uint64_t)blk * WPB + (uint64_t)w);
    if (i >= a.n_req) return;
    uint64_t r[D], s[D], e[D], ct[D];
#pragma unroll
    for (int j = 0; j < D; ++j) r[j] = uniform_u64(R[i * D + j]);  // issued with the key's metadata
    // KEYS = false (identity key map): R and the key's metadata in one round trip
    const uint64_t key = KEYS ? uniform_u64(keys[i]) : i;
    const KeyMeta km = key_meta(key, key_off, key_len, key_id0);
    const uint64_t off = km.off, n = km.n;
    const uint32_t id0 = km.id0;  // consecutive-id base (agn_log_index_ids)
    // The side bytes and rows (key_type, sct_ignore, SCT, TxId) load
    // unconditionally -- from an in-bounds dummy when the column is absent --
    // so they share the metadata's round trip: a conditional scalar load is
    // waited for on its own before the row loads issue.
    const uint32_t kty =
        byte_of(key_type ? key_type : reinterpret_cast<const uint8_t *>(key_off), key);
    const uint64_t *sct_p = (ANY_WARM && sct) ? sct : R;
    const uint32_t sib =
        ANY_WARM ? byte_of(sct_ignore ? sct_ignore : reinterpret_cast<const uint8_t *>(R), i) : 0u;
    const uint64_t txv = uniform_u64((req_txid ? req_txid : R)[i]);
    uint64_t sv[D];
#pragma unroll
    for (int j = 0; j < D; ++j) sv[j] = ANY_WARM ? uniform_u64(sct_p[i * D + j]) : 0ull;
    // sparse batch: the key's DC set and R's / SCT's mask words, same round trip
    uint64_t kmw = 0, rmw = 0, smw = 0;
    if constexpr (MSK) {
        kmw = uniform_u64(*(mk.key_mask ? mk.key_mask + key : R));
        rmw = uniform_u64(*(mk.R_mask ? mk.R_mask + i : R));
        smw = uniform_u64(*((ANY_WARM && mk.sct_mask) ? mk.sct_mask + i : R));
    }
    if (n != 0 && key_type != nullptr && kty != (a.req_type & 0xffu)) {
        if (lane == 0) {  // erlang:error(corrupted_ops_cache) (:190-191)
            o_flags[i] = AGN_F_ERR_CORRUPTED;
            o_err[i] = 0xffffffffu;
        }
        return;
    }
    const bool sct_ign = !ANY_WARM || sct == nullptr || (sct_ignore && sib != 0u);
    const Presence<D> pr = presence<D, MSK>(mk, kmw, rmw, smw, n);
#pragma unroll
    for (int j = 0; j < D; ++j) {
        // e = SCT as a dict read (missing DC = 0); LastOpCt starts as it
        // (materialize/4 :94-95).  s = the compare value: +inf outside U on
        // the dense scan of a sparse key.
        const bool inU = ((pr.U >> j) & 1ull) != 0ull;
        e[j] = (sct_ign || !((pr.Sm >> j) & 1ull)) ? 0ull : sv[j];
        s[j] = (MSK && pr.uni && !inU) ? ~0ull : e[j];
        r[j] = (MSK && pr.uni && !inU) ? ~0ull : r[j];
        ct[j] = e[j];
    }
    const uint64_t txr = req_txid ? txv : 0ull;
    const uint64_t *tx = (txr != 0ull) ? log_txid : nullptr;
    int64_t sum = 0, first_excl = -1, first_err = -1;
    uint32_t cnt = 0;
    int64_t hid = -1;
    uint64_t um = 0;            // MSK, mixed key: DCs of the included ops (per lane)
    uint64_t ctA = 0, ctB = 0;  // QUAD: LastOpCt of DCs 2p, 2p+1 (p = lane & 3)
    const bool warm = ANY_WARM && !sct_ign;
#define AGN_MSK_SCAN()                                                                         \
    do {                                                                                       \
        if (!warm)                                                                             \
            scan_key_msk<D, false>(oc, mk.oc_mask, eff, tx, txr, off, n, r, s, pr.Rm, ct, um,  \
                                   sum, cnt, first_excl, first_err);                           \
        else                                                                                   \
            scan_key_msk<D, ANY_WARM>(oc, mk.oc_mask, eff, tx, txr, off, n, r, s, pr.Rm, ct,   \
                                      um, sum, cnt, first_excl, first_err);                    \
    } while (0)
    if constexpr (QUAD) {
        const int p = lane & 3;
        const uint64_t rA = p == 0 ? r[0] : p == 1 ? r[2 % D] : p == 2 ? r[4 % D] : r[6 % D];
        const uint64_t rB = p == 0 ? r[1 % D] : p == 1 ? r[3 % D] : p == 2 ? r[5 % D] : r[7 % D];
        const uint64_t sA = p == 0 ? s[0] : p == 1 ? s[2 % D] : p == 2 ? s[4 % D] : s[6 % D];
        const uint64_t sB = p == 0 ? s[1 % D] : p == 1 ? s[3 % D] : p == 2 ? s[5 % D] : s[7 % D];
        const uint64_t eA = p == 0 ? e[0] : p == 1 ? e[2 % D] : p == 2 ? e[4 % D] : e[6 % D];
        const uint64_t eB = p == 0 ? e[1 % D] : p == 1 ? e[3 % D] : p == 2 ? e[5 % D] : e[7 % D];
        ctA = eA;
        ctB = eB;
#define AGN_Q8(W, NT, ENT)                                                                     \
    scan_key_q8<W, NT, ENT>(oc, eff, tx, txr, off, n, a.n_entries, rA, rB, sA, sB, ctA, ctB, sum, \
                            cnt, first_excl, first_err)
        if (!MSK || pr.uni) {
            if (!warm) {
                if (a.qnt & 2u) AGN_Q8(false, true, true);
                else if (a.qnt & 1u) AGN_Q8(false, true, false);
                else AGN_Q8(false, false, false);
            } else {
                if (a.qnt & 2u) AGN_Q8(ANY_WARM, true, true);
                else if (a.qnt & 1u) AGN_Q8(ANY_WARM, true, false);
                else AGN_Q8(ANY_WARM, false, false);
            }
            if (MSK) {  // outside U: SCT's value (an op's row there is not in its dict)
                ctA = ((pr.U >> (2 * p)) & 1ull) ? ctA : eA;
                ctB = ((pr.U >> (2 * p + 1)) & 1ull) ? ctB : eB;
            }
        } else if constexpr (MSK) {
            // a mixed key: the quad rows with each op's mask word
            if (!warm)
                scan_key_q8_msk<false>(oc, mk.oc_mask, eff, tx, txr, off, n, a.n_entries, rA, rB,
                                       sA, sB, pr.Rm, ctA, ctB, um, sum, cnt, first_excl,
                                       first_err);
            else
                scan_key_q8_msk<ANY_WARM>(oc, mk.oc_mask, eff, tx, txr, off, n, a.n_entries, rA,
                                          rB, sA, sB, pr.Rm, ctA, ctB, um, sum, cnt, first_excl,
                                          first_err);
        }
#undef AGN_Q8
    } else if constexpr (GLDS && D % 2 == 0) {
        if (!ANY_WARM || sct_ign)
            hid = scan_key_glds<D, false>(oc, eff, op_id, tx, txr, off, n, a.n_entries, r, s, ct,
                                          sum, cnt, first_excl, first_err, lds_all[w]);
        else
            hid = scan_key_glds<D, ANY_WARM>(oc, eff, op_id, tx, txr, off, n, a.n_entries, r, s,
                                             ct, sum, cnt, first_excl, first_err, lds_all[w]);
    } else {
        if (MSK && !pr.uni) {
            if constexpr (MSK) AGN_MSK_SCAN();
        } else if (D <= 4 && a.pair) {
            if (!warm)
                scan_key<D, false, true>(oc, eff, tx, txr, off, n, r, s, ct, sum, cnt, first_excl,
                                         first_err);
            else
                scan_key<D, ANY_WARM, true>(oc, eff, tx, txr, off, n, r, s, ct, sum, cnt,
                                            first_excl, first_err);
        } else {
            if (!warm)
                scan_key<D, false>(oc, eff, tx, txr, off, n, r, s, ct, sum, cnt, first_excl,
                                   first_err);
            else
                scan_key<D, ANY_WARM>(oc, eff, tx, txr, off, n, r, s, ct, sum, cnt, first_excl,
                                      first_err);
        }
        if (MSK && pr.uni) {
#pragma unroll
            for (int j = 0; j < D; ++j) ct[j] = ((pr.U >> j) & 1ull) ? ct[j] : e[j];
        }
    }
#undef AGN_MSK_SCAN
    // NewLastOp id and base value: scalar loads, issued before the reductions
    if (hid < 0) {
        const uint64_t pos = first_excl >= 0 ? (uint64_t)first_excl : n - 1;
        if (id0 != AGN_ID0_NONE)  // op_id[off + pos] == id0 + pos (agn_log_index_ids)
            hid = n ? (int64_t)((uint64_t)id0 + pos) : 0;
        else
            hid = n ? (int64_t)op_id[uniform_u64(off + pos)] : 0;
    }
    const int64_t base = base_value ? (int64_t)uniform_u64((uint64_t)base_value[i]) : 0;

    const int64_t total = wave_sum_dpp(sum);
    const bool ct_ign = sct_ign && cnt == 0u;
    if constexpr (QUAD) {
        // LastOpCt: the 16 lanes of each part fold by xor-shuffles; lanes 0..3
        // write the row's 4 x 16 bytes
#pragma unroll
        for (int x = 4; x < AGN_WAVE; x <<= 1) {
            ctA = umax64(ctA, shfl_xor_u64(ctA, x));
            ctB = umax64(ctB, shfl_xor_u64(ctB, x));
        }
        if (lane < 4) {
            u64x2 v;
            v.x = ct_ign ? 0ull : ctA;
            v.y = ct_ign ? 0ull : ctB;
            reinterpret_cast<u64x2 *>(o_lastct + i * D)[lane] = v;
        }
    } else {
        // LastOpCt: per-lane maxima -> LDS [DCP][64] -> each lane folds V slots
        // of one DC -> xor-shuffle across the 64/DCP lanes that share it
        uint64_t(*stage)[AGN_WAVE] = reinterpret_cast<uint64_t(*)[AGN_WAVE]>(lds_all[w]);
#pragma unroll
        for (int j = 0; j < D; ++j) stage[j][lane] = ct[j];
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const int c = lane % DCP, g = lane / DCP;
        uint64_t m = 0;
        if (c < D) {
#pragma unroll
            for (int v = 0; v < V; ++v) m = umax64(m, stage[c][g * V + v]);
        }
#pragma unroll
        for (int x = DCP; x < AGN_WAVE; x <<= 1) m = umax64(m, shfl_xor_u64(m, x));
        if (g == 0 && c < D) o_lastct[i * D + (uint64_t)c] = ct_ign ? 0ull : m;
    }
    // LastOpCt's DC set: SCT's united with the included ops' (U, or the
    // per-lane sets of a mixed key)
    uint64_t mo = 0;
    if constexpr (MSK) {
        const uint64_t un = pr.uni ? (cnt ? pr.U : 0ull) : wave_or_bits<D>(um);
        mo = ct_ign ? 0ull : ((sct_ign ? 0ull : pr.Sm) | un);
    }
    if (lane == 0) {
        // NewLastOp = id(oldest excluded) - 1, else get_first_id (:49-63)
        const int64_t hole = first_excl >= 0 ? hid - 1 : hid;
        uint32_t fl = 0;
        if (cnt) fl |= AGN_F_NEWSS;
        if (ct_ign) fl |= AGN_F_CT_IGNORE;
        if (first_err >= 0) fl |= AGN_F_ERR_UNEXPECTED;
        o_value[i] = (int64_t)((uint64_t)base + (uint64_t)total);
        o_hole[i] = hole;
        o_count[i] = cnt;
        o_flags[i] = fl;
        o_err[i] = first_err >= 0 ? (uint32_t)(off + (uint64_t)first_err) : 0xffffffffu;
        if (MSK && mk.o_mask) mk.o_mask[i] = mo;
    }
}

// agn_log.key_id0, unless AGN_COUNTER_ID0=0 (A/B knob: always load the op id)
inline const uint32_t *id0_index(const agn_log &log) {
    const char *v = AGN_KNOB("AGN_COUNTER_ID0");
    return (v && v[0] == '0') ? nullptr : log.key_id0;
}

// ROWS_QUAD2 (D = 8): quad rows, TWO requests per wave with both keys'
// first chunks in flight at once (9 KiB of rows per wave slot instead of 4.5).
// Same results as k_counter_key.  The default for warm batches (the SCT
// rows and flags lengthen each request's prologue, which the second key's
// loads cover); cold batches measured no change (56 VGPRs, 8 waves).
// AGN_COUNTER_VARIANT=3 forces it, =2 the one-request form.
struct Q2Key {
    uint64_t i, key, off, n, txr;
    uint32_t id0;
    bool corrupt, sct_ign;
    bool uni;  // the dense scan serves the key: its DC set U is known (MSK) or the batch is dense
    bool noR;  // MSK: U is known but R lacks one of its DCs -- every op excluded (:245-247)
    uint64_t rA, rB, sA, sB, eA, eB;  // per lane: DCs 2p, 2p+1 (p = lane & 3)
    uint64_t U, Sm, Rm;               // MSK (Presence)
};

// agn_log.key_mask of a key (an in-bounds dummy when the log has none).
__device__ __forceinline__ uint64_t key_word(const MaskArgs &mk, uint64_t key,
                                             const uint64_t *__restrict__ key_off) {
    return uniform_u64(ldc(mk.key_mask ? mk.key_mask + key : key_off));
}

// The key's segment (the metadata the row loads depend on).
__device__ __forceinline__ void q2_meta(Q2Key &k, uint64_t i, const uint64_t *__restrict__ keys,
                                        const uint64_t *__restrict__ key_off,
                                        const uint64_t *__restrict__ key_len,
                                        const uint32_t *__restrict__ key_id0) {
    k.i = i;
    k.key = keys ? uniform_u64(ldc(keys + i)) : i;
    const KeyMeta km = key_meta(k.key, key_off, key_len, key_id0);
    k.off = km.off;
    k.n = km.n;
    k.id0 = km.id0;
}

// The rest of a request's prologue: key_type, SCT and its ignore byte, TxId,
// R, the presence words of a sparse batch -- as raw scalar loads (q2_load:
// every address depends only on the request and the key's segment), then the
// values derived from them (q2_apply).  Scalar loads return out of order, so
// the first use of any of them waits for all (lgkmcnt(0)): k_counter_q8e
// issues the whole group under chunk 0's rows and puts a scheduling barrier
// before the first use -- left alone, the scheduler interleaved uses with the
// loads and the warm masked prologue became three dependent scalar round
// trips after the rows (warm masked cfg2 1.23x the dense warm kernel).
// R's and SCT's DCs 2p, 2p+1 (p = lane & 3) -- the pair this lane compares
// -- come as one 16-byte vector load each: as 16 uniform words apiece they
// sat in SGPRs next to the kernel's pointer arguments, and the warm masked
// kernel spilled 17 SGPRs to VGPR lanes (v_writelane / v_readlane, issue
// stalls: SQ_WAIT_INST_ANY 1662 vs 990 quad-cycles per wave, warm masked cfg2
// 1.26x the dense warm kernel).
struct Q2Raw {
    uint64_t kmw, txv, rmw, smw;
    u64x2 rq, sq;        // per lane: R / SCT at DCs 2p, 2p+1
    uint32_t ktw, sibw;  // the dwords holding key_type[key] / sct_ignore[i]
};

template <bool ANY_WARM, bool MSK>
__device__ __forceinline__ Q2Raw q2_load(const Q2Key &k, const DenseArgs &a, const MaskArgs &mk,
                                         bool with_km, const uint64_t *__restrict__ key_off,
                                         const uint8_t *__restrict__ key_type,
                                         const uint64_t *__restrict__ R,
                                         const uint64_t *__restrict__ sct,
                                         const uint8_t *__restrict__ sct_ignore,
                                         const uint64_t *__restrict__ req_txid) {
    constexpr int D = 8;
    const uint64_t i = k.i;
    Q2Raw x;
    const uint8_t *ktp = key_type ? key_type : reinterpret_cast<const uint8_t *>(key_off);
    x.ktw = __builtin_amdgcn_readfirstlane(ldc(reinterpret_cast<const uint32_t *>(ktp) + (k.key >> 2)));
    const uint8_t *sip = sct_ignore ? sct_ignore : reinterpret_cast<const uint8_t *>(R);
    x.sibw = ANY_WARM ? __builtin_amdgcn_readfirstlane(ldc(reinterpret_cast<const uint32_t *>(sip) + (i >> 2)))
                      : 0u;
    x.txv = uniform_u64(ldc((req_txid ? req_txid : R) + i));
    x.kmw = (MSK && with_km) ? key_word(mk, k.key, key_off) : 0ull;
    x.rmw = x.smw = 0ull;
    if constexpr (MSK) {
        // AGN_HINT_R_FULL: every R mask carries all D DCs (not read)
        const bool rfull = (a.hints & AGN_HINT_R_FULL) != 0u;
        x.rmw = uniform_u64(ldc((mk.R_mask && !rfull) ? mk.R_mask + i : R));
        x.smw = uniform_u64(ldc((ANY_WARM && mk.sct_mask) ? mk.sct_mask + i : R));
    }
    const uint64_t *sct_p = (ANY_WARM && sct) ? sct : R;
    const uint64_t pp = 2u * (uint64_t)(lane_id() & 3);
    x.rq = *reinterpret_cast<const u64x2 *>(R + i * D + pp);
    if constexpr (ANY_WARM) x.sq = *reinterpret_cast<const u64x2 *>(sct_p + i * D + pp);
    else x.sq = u64x2{0ull, 0ull};
    return x;
}

// Pins the raw side values behind the scheduling barrier: the IR passes hoist
// a use (kmw & 0xFF) next to its load, where its wait would precede the other
// loads' issue; a use of an asm output cannot move above the asm.
__device__ __forceinline__ void q2_pin(Q2Raw &x) {
    asm volatile("" : "+s"(x.kmw), "+s"(x.txv), "+s"(x.rmw), "+s"(x.smw), "+s"(x.ktw), "+s"(x.sibw));
}

template <bool ANY_WARM, bool MSK>
__device__ __forceinline__ void q2_apply(Q2Key &k, const DenseArgs &a, const MaskArgs &mk,
                                         const Q2Raw &x, uint64_t kmw,
                                         const uint8_t *__restrict__ key_type,
                                         const uint64_t *__restrict__ sct,
                                         const uint8_t *__restrict__ sct_ignore,
                                         const uint64_t *__restrict__ req_txid) {
    constexpr int D = 8;
    const uint32_t kty = (x.ktw >> ((uint32_t)(k.key & 3u) * 8u)) & 0xffu;
    k.corrupt = k.n != 0 && key_type != nullptr && kty != (a.req_type & 0xffu);
    const uint32_t sib = ANY_WARM ? (x.sibw >> ((uint32_t)(k.i & 3u) * 8u)) & 0xffu : 0u;
    k.sct_ign = !ANY_WARM || sct == nullptr || (sct_ignore && sib != 0u);
    k.txr = req_txid ? x.txv : 0ull;
    const uint64_t rmw = (a.hints & AGN_HINT_R_FULL) ? ~0ull : x.rmw;
    const Presence<D> pr = presence<D, MSK>(mk, kmw, rmw, x.smw, k.n);
    k.U = pr.U;
    k.Rm = pr.Rm;
    k.Sm = pr.Sm;
    // a known DC set U is served by the dense scan whether or not R covers it:
    // when R lacks one of U's DCs, every op (all carry U) is excluded
    const bool known = !MSK || pr.uni || pr.U != 0ull;
    k.uni = known;
    k.noR = MSK && known && !pr.uni;
    // this lane's DCs dA = 2p, dB = 2p + 1
    const uint32_t dA = 2u * (uint32_t)(lane_id() & 3), dB = dA + 1u;
    const bool inA = ((pr.U >> dA) & 1ull) != 0ull, inB = ((pr.U >> dB) & 1ull) != 0ull;
    // e = SCT as a dict read (a DC missing from it = 0); s = the compare
    // value, r = R: +inf outside U on the dense scan of a masked key
    k.eA = (k.sct_ign || !((pr.Sm >> dA) & 1ull)) ? 0ull : x.sq.x;
    k.eB = (k.sct_ign || !((pr.Sm >> dB) & 1ull)) ? 0ull : x.sq.y;
    k.sA = (MSK && known && !inA) ? ~0ull : k.eA;
    k.sB = (MSK && known && !inB) ? ~0ull : k.eB;
    k.rA = (MSK && known && !inA) ? ~0ull : x.rq.x;
    k.rB = (MSK && known && !inB) ? ~0ull : x.rq.y;
}

template <bool ANY_WARM, bool MSK>
__device__ __forceinline__ void q2_side(Q2Key &k, const DenseArgs &a, const MaskArgs &mk,
                                        uint64_t kmw, const uint64_t *__restrict__ key_off,
                                        const uint8_t *__restrict__ key_type,
                                        const uint64_t *__restrict__ R,
                                        const uint64_t *__restrict__ sct,
                                        const uint8_t *__restrict__ sct_ignore,
                                        const uint64_t *__restrict__ req_txid) {
    const Q2Raw x = q2_load<ANY_WARM, MSK>(k, a, mk, false, key_off, key_type, R, sct, sct_ignore,
                                           req_txid);
    q2_apply<ANY_WARM, MSK>(k, a, mk, x, kmw, key_type, sct, sct_ignore, req_txid);
}

template <bool ANY_WARM, bool MSK>
__device__ __forceinline__ Q2Key q2_prologue(const DenseArgs &a, const MaskArgs &mk, uint64_t i,
                                             const uint64_t *__restrict__ keys,
                                             const uint64_t *__restrict__ key_off,
                                             const uint64_t *__restrict__ key_len,
                                             const uint8_t *__restrict__ key_type,
                                             const uint32_t *__restrict__ key_id0,
                                             const uint64_t *__restrict__ R,
                                             const uint64_t *__restrict__ sct,
                                             const uint8_t *__restrict__ sct_ignore,
                                             const uint64_t *__restrict__ req_txid) {
    Q2Key k;
    q2_meta(k, i, keys, key_off, key_len, key_id0);
    const uint64_t kmw = MSK ? key_word(mk, k.key, key_off) : 0ull;
    q2_side<ANY_WARM, MSK>(k, a, mk, kmw, key_off, key_type, R, sct, sct_ignore, req_txid);
    return k;
}

struct Q2Acc {
    int64_t sum = 0, first_excl = -1, first_err = -1;
    uint32_t cnt = 0;
    uint64_t ctA, ctB;
    uint64_t um = 0;  // MSK, mixed key: the included ops' DC set
};

template <bool ANY_WARM>
__device__ __forceinline__ void q2_fold(const Q2Key &k, const Q8Chunk &c, uint64_t b,
                                        const uint64_t *__restrict__ log_txid, uint64_t n_entries,
                                        Q2Acc &s) {
    const uint64_t *tx = k.txr ? log_txid : nullptr;
    if (ANY_WARM && !k.sct_ign)
        q8_fold<true>(c, tx, k.txr, k.off, b, k.n, n_entries, k.rA, k.rB, k.sA, k.sB, s.ctA, s.ctB,
                      s.sum, s.cnt, s.first_excl, s.first_err, k.noR);
    else
        q8_fold<false>(c, tx, k.txr, k.off, b, k.n, n_entries, k.rA, k.rB, k.sA, k.sB, s.ctA,
                       s.ctB, s.sum, s.cnt, s.first_excl, s.first_err, k.noR);
}

template <bool ANY_WARM>
__device__ __forceinline__ void q2_rest(const Q2Key &k, const uint64_t *__restrict__ oc,
                                        const int64_t *__restrict__ eff,
                                        const uint64_t *__restrict__ log_txid, uint64_t n_entries,
                                        Q2Acc &s) {
    if (k.n <= (uint64_t)AGN_WAVE) return;
    const uint64_t *tx = k.txr ? log_txid : nullptr;
    if (ANY_WARM && !k.sct_ign)
        scan_key_q8<true, true, false, true>(oc, eff, tx, k.txr, k.off, k.n, n_entries, k.rA, k.rB,
                                             k.sA, k.sB, s.ctA, s.ctB, s.sum, s.cnt, s.first_excl,
                                             s.first_err, k.noR);
    else
        scan_key_q8<false, true, false, true>(oc, eff, tx, k.txr, k.off, k.n, n_entries, k.rA,
                                              k.rB, k.sA, k.sB, s.ctA, s.ctB, s.sum, s.cnt,
                                              s.first_excl, s.first_err, k.noR);
}

// A mixed key of a sparse batch (MSK, !uni): the per-entry-mask scan, lane =
// op, with R / SCT / the LastOpCt seed gathered back from the quad lanes
// (lane p < 4 holds DCs 2p, 2p+1).
template <bool ANY_WARM>
__device__ __forceinline__ void q2_msk(const Q2Key &k, const uint64_t *__restrict__ oc,
                                       const uint64_t *__restrict__ oc_mask,
                                       const int64_t *__restrict__ eff,
                                       const uint64_t *__restrict__ log_txid, uint64_t n_entries,
                                       Q2Acc &s) {
    const uint64_t *tx = k.txr ? log_txid : nullptr;
    if (ANY_WARM && !k.sct_ign)
        scan_key_q8_msk<true>(oc, oc_mask, eff, tx, k.txr, k.off, k.n, n_entries, k.rA, k.rB,
                              k.sA, k.sB, k.Rm, s.ctA, s.ctB, s.um, s.sum, s.cnt, s.first_excl,
                              s.first_err);
    else
        scan_key_q8_msk<false>(oc, oc_mask, eff, tx, k.txr, k.off, k.n, n_entries, k.rA, k.rB,
                               k.sA, k.sB, k.Rm, s.ctA, s.ctB, s.um, s.sum, s.cnt, s.first_excl,
                               s.first_err);
}

template <bool MSK>
__device__ __forceinline__ void q2_epilogue(const Q2Key &k, Q2Acc &s, uint32_t hints,
                                            const uint32_t *__restrict__ op_id,
                                            const int64_t *__restrict__ base_value,
                                            int64_t *__restrict__ o_value,
                                            int64_t *__restrict__ o_hole,
                                            uint64_t *__restrict__ o_lastct,
                                            uint32_t *__restrict__ o_count,
                                            uint32_t *__restrict__ o_flags,
                                            uint32_t *__restrict__ o_err,
                                            uint64_t *__restrict__ o_mask) {
    constexpr int D = 8;
    const int lane = lane_id();
    const uint64_t i = k.i;
    if (k.corrupt) {
        if (lane == 0) {  // erlang:error(corrupted_ops_cache) (:190-191)
            o_flags[i] = AGN_F_ERR_CORRUPTED;
            o_err[i] = 0xffffffffu;
        }
        return;
    }
    int64_t hid;
    const uint64_t pos = s.first_excl >= 0 ? (uint64_t)s.first_excl : k.n - 1;
    if (k.id0 != AGN_ID0_NONE)
        hid = k.n ? (int64_t)((uint64_t)k.id0 + pos) : 0;
    else
        hid = k.n ? (int64_t)__builtin_amdgcn_readfirstlane(ldc(op_id + uniform_u64(k.off + pos))) : 0;
    const int64_t base = base_value ? (int64_t)uniform_u64((uint64_t)ldc(base_value + i)) : 0;
    const int64_t total = wave_sum_dpp(s.sum);
    const bool ct_ign = k.sct_ign && s.cnt == 0u;
    uint64_t mo = 0;
    if constexpr (MSK) {
        if (k.uni) {  // outside U: SCT's value (an op's row there is not in its dict)
            const int p = lane & 3;
            s.ctA = ((k.U >> (2 * p)) & 1ull) ? s.ctA : k.eA;
            s.ctB = ((k.U >> (2 * p + 1)) & 1ull) ? s.ctB : k.eB;
        }
        const uint64_t un = k.uni ? (s.cnt ? k.U : 0ull) : wave_or_bits<D>(s.um);
        mo = ct_ign ? 0ull : ((k.sct_ign ? 0ull : k.Sm) | un);
    }
#pragma unroll
    for (int x = 4; x < AGN_WAVE; x <<= 1) {
        s.ctA = umax64(s.ctA, shfl_xor_u64(s.ctA, x));
        s.ctB = umax64(s.ctB, shfl_xor_u64(s.ctB, x));
    }
    if (lane < 4) {
        u64x2 v;
        v.x = ct_ign ? 0ull : s.ctA;
        v.y = ct_ign ? 0ull : s.ctB;
        reinterpret_cast<u64x2 *>(o_lastct + i * D)[lane] = v;
    }
    if (lane == 0) {
        const int64_t hole = s.first_excl >= 0 ? hid - 1 : hid;
        uint32_t fl = 0;
        if (s.cnt) fl |= AGN_F_NEWSS;
        if (ct_ign) fl |= AGN_F_CT_IGNORE;
        if (s.first_err >= 0) fl |= AGN_F_ERR_UNEXPECTED;
        o_value[i] = (int64_t)((uint64_t)base + (uint64_t)total);
        o_hole[i] = hole;
        o_count[i] = s.cnt;
        o_err[i] = s.first_err >= 0 ? (uint32_t)(k.off + (uint64_t)s.first_err) : 0xffffffffu;
        // AGN_HINT_CT_FLAG: a LastOpCt over every column is a flag bit, not a
        // mask word (one store stream less per request)
        const bool full = MSK && (hints & AGN_HINT_CT_FLAG) && mo == 0xFFull;
        if (full) fl |= AGN_F_CT_FULL;
        o_flags[i] = fl;
        if (MSK && o_mask && !full) o_mask[i] = mo;
    }
}

// k_counter_q8e2's parameters as one block (kparams: each stage reads the
// fields it uses; as 26 separate arguments it spilled 62 SGPRs, 43-47 so).
// k_counter_quad2 keeps its by-value arguments: read this way its dense warm
// form ran 9.47 against 8.32 ms (the parameter loads joined the prologue's
// dependent chain; profiles/r05/ab_masked_warm_quad2_kparams.log).
struct Q2Params {
    DenseArgs a;
    MaskArgs mk;
    const uint64_t *keys, *key_off, *key_len;
    const uint8_t *key_type;
    const uint32_t *key_id0;
    const uint64_t *oc;
    const uint32_t *op_id;
    const int64_t *eff;
    const uint64_t *log_txid, *R, *sct;
    const uint8_t *sct_ignore;
    const uint64_t *req_txid;
    const int64_t *base_value;
    int64_t *o_value, *o_hole;
    uint64_t *o_lastct;
    uint32_t *o_count, *o_flags, *o_err, *list, *list_n;
};

template <class T>
__device__ __forceinline__ DenseArgs dense_of(const T &x) {
    return DenseArgs{x.n_req, x.n_entries, x.req_type, x.xcd, x.pair, x.qnt, x.hints, x.ql_cap};
}
template <class T>
__device__ __forceinline__ MaskArgs mask_of(const T &x) {
    return MaskArgs{x.key_mask, x.oc_mask, x.R_mask, x.sct_mask, x.o_mask};
}

// The dense warm form runs at 6 waves per SIMD: 80 VGPRs and 2 scratch
// spills instead of 84 VGPRs (5 waves) and 24 spilled SGPRs, 8.13 against
// 8.33 ms on warm cfg2 (profiles/r05/ab_quad2_w6.log).  The masked forms spill
// far more under that budget and keep the default.
template <bool ANY_WARM, bool MSK>
__global__ __launch_bounds__(64, (ANY_WARM && !MSK) ? 6 : 1) void k_counter_quad2(
    DenseArgs a, MaskArgs mk, const uint64_t *__restrict__ keys,
    const uint64_t *__restrict__ key_off, const uint64_t *__restrict__ key_len,
    const uint8_t *__restrict__ key_type, const uint32_t *__restrict__ key_id0,
    const uint64_t *__restrict__ oc, const uint32_t *__restrict__ op_id,
    const int64_t *__restrict__ eff, const uint64_t *__restrict__ log_txid,
    const uint64_t *__restrict__ R, const uint64_t *__restrict__ sct,
    const uint8_t *__restrict__ sct_ignore, const uint64_t *__restrict__ req_txid,
    const int64_t *__restrict__ base_value, int64_t *__restrict__ o_value,
    int64_t *__restrict__ o_hole, uint64_t *__restrict__ o_lastct,
    uint32_t *__restrict__ o_count, uint32_t *__restrict__ o_flags,
    uint32_t *__restrict__ o_err) {
    const uint32_t blk = block_order(a.xcd, blockIdx.x, gridDim.x);
    const uint64_t i0 = uniform_u64((uint64_t)blk * 2u);
    if (i0 >= a.n_req) return;
    const bool two = i0 + 1u < a.n_req;
    const uint64_t i1 = two ? i0 + 1u : i0;
    const Q2Key k0 = q2_prologue<ANY_WARM, MSK>(a, mk, i0, keys, key_off, key_len, key_type,
                                                key_id0, R, sct, sct_ignore, req_txid);
    const Q2Key k1 = q2_prologue<ANY_WARM, MSK>(a, mk, i1, keys, key_off, key_len, key_type,
                                                key_id0, R, sct, sct_ignore, req_txid);
    Q2Acc s0, s1;
    s0.ctA = k0.eA;
    s0.ctB = k0.eB;
    s1.ctA = k1.eA;
    s1.ctB = k1.eB;
    if (a.n_entries != 0) {
        const Q8Chunk c0 = q8_load<true, false>(oc, eff, k0.off, 0, a.n_entries);
        const Q8Chunk c1 = q8_load<true, false>(oc, eff, k1.off, 0, a.n_entries);
        __builtin_amdgcn_sched_barrier(0);
        const bool d0 = !k0.corrupt && (!MSK || k0.uni), d1 = !k1.corrupt && (!MSK || k1.uni);
        if (d0) q2_fold<ANY_WARM>(k0, c0, 0, log_txid, a.n_entries, s0);
        if (d1) q2_fold<ANY_WARM>(k1, c1, 0, log_txid, a.n_entries, s1);
        if (d0) q2_rest<ANY_WARM>(k0, oc, eff, log_txid, a.n_entries, s0);
        if (d1) q2_rest<ANY_WARM>(k1, oc, eff, log_txid, a.n_entries, s1);
        if constexpr (MSK) {
            if (!k0.corrupt && !k0.uni)
                q2_msk<ANY_WARM>(k0, oc, mk.oc_mask, eff, log_txid, a.n_entries, s0);
            if (!k1.corrupt && !k1.uni)
                q2_msk<ANY_WARM>(k1, oc, mk.oc_mask, eff, log_txid, a.n_entries, s1);
        }
    }
    q2_epilogue<MSK>(k0, s0, a.hints, op_id, base_value, o_value, o_hole, o_lastct, o_count, o_flags, o_err,
                     mk.o_mask);
    if (two)
        q2_epilogue<MSK>(k1, s1, a.hints, op_id, base_value, o_value, o_hole, o_lastct, o_count, o_flags,
                         o_err, mk.o_mask);
}

// ROWS_QUAD with the first chunk EARLY (D = 8, one request per wave; the
// sparse batches, MSK): the key's segment metadata (key_off, key_len,
// key_id0) is the only scalar round trip before the rows -- chunk 0's quad
// rows and effects are issued as soon as it lands, and R, SCT, the side
// bytes, the TxId and the mask words load under them.  In k_counter_key all
// of those share the metadata's round trip, and scalar loads return out of
// order, so the first row load waits for the slowest of them (lgkmcnt(0)).
// A key whose DC set U is known (agn_log.key_mask) is served by the dense
// scan, also when R lacks one of U's DCs (every op excluded, :245-247); a key
// whose entries carry different DC sets is appended to `list` for
// k_counter_q8m, so this kernel holds no per-entry-mask scan (inlined, it
// cost 73-98 VGPRs: 4-6 waves per SIMD, or spills at a 7-wave cap;
// profiles/r04/ab_masked_*.log).  KM: the key's DC set loads with the
// segment metadata (1) or under the chunk (0).  Same results as
// k_counter_key.
template <bool ANY_WARM, bool KEYS, int KM>
__global__ __launch_bounds__(64) void k_counter_q8e(
    DenseArgs a, MaskArgs mk, const uint64_t *__restrict__ keys,
    const uint64_t *__restrict__ key_off, const uint64_t *__restrict__ key_len,
    const uint8_t *__restrict__ key_type, const uint32_t *__restrict__ key_id0,
    const uint64_t *__restrict__ oc, const uint32_t *__restrict__ op_id,
    const int64_t *__restrict__ eff, const uint64_t *__restrict__ log_txid,
    const uint64_t *__restrict__ R, const uint64_t *__restrict__ sct,
    const uint8_t *__restrict__ sct_ignore, const uint64_t *__restrict__ req_txid,
    const int64_t *__restrict__ base_value, int64_t *__restrict__ o_value,
    int64_t *__restrict__ o_hole, uint64_t *__restrict__ o_lastct,
    uint32_t *__restrict__ o_count, uint32_t *__restrict__ o_flags,
    uint32_t *__restrict__ o_err, uint32_t *__restrict__ list, uint32_t *__restrict__ list_n) {
    const uint32_t blk = block_order(a.xcd, blockIdx.x, gridDim.x);
    const uint64_t i = uniform_u64((uint64_t)blk);
    if (i >= a.n_req) return;
    Q2Key k;
    q2_meta(k, i, KEYS ? keys : nullptr, key_off, key_len, key_id0);
    // a key whose entries carry different DC sets: k_counter_q8m's
    auto mixed = [&](uint64_t kmw) {
        return !(mk.oc_mask == nullptr || (mk.key_mask && (kmw & 0xFFull)) || k.n == 0);
    };
    // QL_S sub-lists (request i -> i mod QL_S), each with its own counter in
    // its own 128-byte line: one shared counter serialised every hand-on of
    // a batch of mixed keys at one L2 channel (10M atomics, 16x the scan)
    auto hand_on = [&]() {
        if (lane_id() == 0) {
            const uint32_t sl = (uint32_t)(i % QL_S);
            list[(uint64_t)sl * a.ql_cap + atomicAdd(list_n + sl * QL_STRIDE, 1u)] = (uint32_t)i;
        }
    };
    uint64_t kmw = 0;
    if constexpr (KM == 1) {
        kmw = key_word(mk, k.key, key_off);
        if (mixed(kmw)) {
            hand_on();
            return;
        }
    }
    const bool any = a.n_entries != 0;
    Q8Chunk c0{};
    if (any) c0 = q8_load<true, false>(oc, eff, k.off, 0, a.n_entries);
    // the request's side values: one group of scalar loads under the rows,
    // used only past the barrier (one lgkmcnt wait, see q2_load)
    Q2Raw x = q2_load<ANY_WARM, true>(k, a, mk, KM == 0, key_off, key_type, R, sct, sct_ignore,
                                      req_txid);
    __builtin_amdgcn_sched_barrier(0);
    q2_pin(x);
    if constexpr (KM == 0) kmw = x.kmw;
    q2_apply<ANY_WARM, true>(k, a, mk, x, kmw, key_type, sct, sct_ignore, req_txid);
    if (KM == 0 && mixed(kmw)) {
        hand_on();
        return;
    }
    Q2Acc s;
    s.ctA = k.eA;
    s.ctB = k.eB;
    if (any && !k.corrupt) {
        q2_fold<ANY_WARM>(k, c0, 0, log_txid, a.n_entries, s);
        q2_rest<ANY_WARM>(k, oc, eff, log_txid, a.n_entries, s);
    }
    q2_epilogue<true>(k, s, a.hints, op_id, base_value, o_value, o_hole, o_lastct, o_count, o_flags,
                      o_err, mk.o_mask);
}

// Sparse batches, cold and warm: k_counter_q8e with two requests per wave,
// as k_counter_quad2 serves dense warm batches -- both keys' segment
// metadata in one scalar round trip, both first chunks issued under it, the
// side loads (R, SCT, the DC sets) under the chunks.  Mixed keys are handed
// on to k_counter_q8m as in q8e.  (Round 3's two-request masked form carried
// the per-entry-mask scan inline: 118 VGPRs, slower than one request.)
template <bool ANY_WARM, bool KEYS>
__global__ __launch_bounds__(64) void k_counter_q8e2(Q2Params) {
    const DenseArgs a = dense_of(kparams<Q2Params>().a);
    const uint32_t blk = block_order(a.xcd, blockIdx.x, gridDim.x);
    const uint64_t i0 = uniform_u64((uint64_t)blk * 2u);
    if (i0 >= a.n_req) return;
    const bool two = i0 + 1u < a.n_req;
    const uint64_t i1 = two ? i0 + 1u : i0;
    Q2Key k0, k1;
    {
        const auto &p = kparams<Q2Params>();
        q2_meta(k0, i0, KEYS ? p.keys : nullptr, p.key_off, p.key_len, p.key_id0);
        q2_meta(k1, i1, KEYS ? p.keys : nullptr, p.key_off, p.key_len, p.key_id0);
    }
    const bool any = a.n_entries != 0;
    Q8Chunk c0{}, c1{};
    if (any) {
        const auto &p = kparams<Q2Params>();
        c0 = q8_load<true, false>(p.oc, p.eff, k0.off, 0, a.n_entries);
        c1 = q8_load<true, false>(p.oc, p.eff, k1.off, 0, a.n_entries);
    }
    __builtin_amdgcn_sched_barrier(0);
    const auto &ps = kparams<Q2Params>();
    const MaskArgs mk = mask_of(ps.mk);
    const uint64_t kmw0 = key_word(mk, k0.key, ps.key_off), kmw1 = key_word(mk, k1.key, ps.key_off);
    q2_side<ANY_WARM, true>(k0, a, mk, kmw0, ps.key_off, ps.key_type, ps.R, ps.sct,
                            ps.sct_ignore, ps.req_txid);
    q2_side<ANY_WARM, true>(k1, a, mk, kmw1, ps.key_off, ps.key_type, ps.R, ps.sct,
                            ps.sct_ignore, ps.req_txid);
    auto mixed = [&](const Q2Key &k, uint64_t kmw) {
        return !(mk.oc_mask == nullptr || (mk.key_mask && (kmw & 0xFFull)) || k.n == 0);
    };
    auto hand_on = [&](uint64_t i) {  // q8e's sub-lists
        if (lane_id() == 0) {
            const auto &p = kparams<Q2Params>();
            const uint32_t sl = (uint32_t)(i % QL_S);
            p.list[(uint64_t)sl * a.ql_cap + atomicAdd(p.list_n + sl * QL_STRIDE, 1u)] = (uint32_t)i;
        }
    };
    const bool m0 = mixed(k0, kmw0), m1 = two && mixed(k1, kmw1);
    if (m0) hand_on(i0);
    if (m1) hand_on(i1);
    Q2Acc s0, s1;
    s0.ctA = k0.eA;
    s0.ctB = k0.eB;
    s1.ctA = k1.eA;
    s1.ctB = k1.eB;
    const bool d0 = any && !k0.corrupt && !m0, d1 = two && any && !k1.corrupt && !m1;
    {
        const auto &p = kparams<Q2Params>();
        if (d0) q2_fold<ANY_WARM>(k0, c0, 0, p.log_txid, a.n_entries, s0);
        if (d1) q2_fold<ANY_WARM>(k1, c1, 0, p.log_txid, a.n_entries, s1);
        if (d0) q2_rest<ANY_WARM>(k0, p.oc, p.eff, p.log_txid, a.n_entries, s0);
        if (d1) q2_rest<ANY_WARM>(k1, p.oc, p.eff, p.log_txid, a.n_entries, s1);
    }
    const auto &pe = kparams<Q2Params>();
    if (!m0)
        q2_epilogue<true>(k0, s0, a.hints, pe.op_id, pe.base_value, pe.o_value, pe.o_hole,
                          pe.o_lastct, pe.o_count, pe.o_flags, pe.o_err, pe.mk.o_mask);
    if (two && !m1)
        q2_epilogue<true>(k1, s1, a.hints, pe.op_id, pe.base_value, pe.o_value, pe.o_hole,
                          pe.o_lastct, pe.o_count, pe.o_flags, pe.o_err, pe.mk.o_mask);
}

// The keys k_counter_q8e handed on (entries with different DC sets): the
// per-entry-mask quad scan (scan_key_q8_msk), one request per wave, the
// waves striding over the sub-lists -- the grid does not know their
// lengths, and empty lists cost one short launch.
template <bool ANY_WARM, bool KEYS>
__global__ __launch_bounds__(64) void k_counter_q8m(
    DenseArgs a, MaskArgs mk, const uint64_t *__restrict__ keys,
    const uint64_t *__restrict__ key_off, const uint64_t *__restrict__ key_len,
    const uint8_t *__restrict__ key_type, const uint32_t *__restrict__ key_id0,
    const uint64_t *__restrict__ oc, const uint32_t *__restrict__ op_id,
    const int64_t *__restrict__ eff, const uint64_t *__restrict__ log_txid,
    const uint64_t *__restrict__ R, const uint64_t *__restrict__ sct,
    const uint8_t *__restrict__ sct_ignore, const uint64_t *__restrict__ req_txid,
    const int64_t *__restrict__ base_value, int64_t *__restrict__ o_value,
    int64_t *__restrict__ o_hole, uint64_t *__restrict__ o_lastct,
    uint32_t *__restrict__ o_count, uint32_t *__restrict__ o_flags,
    uint32_t *__restrict__ o_err, const uint32_t *__restrict__ list,
    const uint32_t *__restrict__ list_n) {
    // block b walks sub-list b mod QL_S, entries b / QL_S, + gridDim.x / QL_S
    const uint32_t sl = blockIdx.x % QL_S, per = gridDim.x / QL_S;
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(list_n[sl * QL_STRIDE]);
    for (uint32_t j = blockIdx.x / QL_S; j < cnt; j += per) {
        const uint64_t i = __builtin_amdgcn_readfirstlane(list[(uint64_t)sl * a.ql_cap + j]);
        const Q2Key k = q2_prologue<ANY_WARM, true>(a, mk, i, KEYS ? keys : nullptr, key_off,
                                                    key_len, key_type, key_id0, R, sct, sct_ignore,
                                                    req_txid);
        Q2Acc s;
        s.ctA = k.eA;
        s.ctB = k.eB;
        if (a.n_entries != 0 && !k.corrupt)
            q2_msk<ANY_WARM>(k, oc, mk.oc_mask, eff, log_txid, a.n_entries, s);
        q2_epilogue<true>(k, s, a.hints, op_id, base_value, o_value, o_hole, o_lastct, o_count,
                          o_flags, o_err, mk.o_mask);
    }
}

MaskArgs mask_args(const agn_log &log, const agn_read &req, const agn_result &out) {
    MaskArgs m;
    m.key_mask = log.oc_mask ? log.key_mask : nullptr;
    m.oc_mask = log.oc_mask;
    m.R_mask = req.R_mask;
    m.sct_mask = req.sct ? req.sct_mask : nullptr;
    m.o_mask = out.lastct_mask;
    return m;
}

inline bool sparse_batch(const agn_log &log, const agn_read &req, const agn_result &out) {
    return log.oc_mask || req.R_mask || (req.sct && req.sct_mask) || out.lastct_mask;
}

int launch_quad2(const agn_log &log, const agn_read &req, const agn_result &out, hipStream_t st) {
    DenseArgs a{req.n_req, log.n_entries, req.req_type, counter_order(req.n_req, BULK_CHUNK), 0u, 1u,
                req.hints};
    const MaskArgs mk = mask_args(log, req, out);
    const uint64_t nb = (req.n_req + 1) / 2;
    if (nb > 0x7fffffffull) return fail(AGN_EINVAL, "batch too large: %llu requests",
                                        (unsigned long long)req.n_req);
#define AGN_Q2L(W, M)                                                                           \
    hipLaunchKernelGGL((k_counter_quad2<W, M>), dim3((unsigned)nb), dim3(64), 0, st, a, mk,     \
                       req.keys, log.key_off, log.key_len, log.key_type, id0_index(log), log.oc, \
                       log.op_id, log.eff, log.txid, req.R, req.sct, req.sct_ignore, req.txid,  \
                       req.base_value, out.value, out.hole, out.lastct, out.count, out.flags,   \
                       out.err_pos)
    const bool msk = sparse_batch(log, req, out);
    if (req.sct) {
        if (msk) AGN_Q2L(true, true);
        else AGN_Q2L(true, false);
    } else {
        if (msk) AGN_Q2L(false, true);
        else AGN_Q2L(false, false);
    }
#undef AGN_Q2L
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

// Sparse batches (D = 8, quad rows) run k_counter_q8e + k_counter_q8m,
// unless AGN_COUNTER_EARLY=0 (A/B knob) or the batch carries AGN_HINT_MIXED:
// k_counter_key, which scans a mixed key in the same pass (cfg2 with one
// entry in 8 lacking a DC: 1.24x dense there, 2.56x through the hand-on,
// whose first pass reads the key's only chunk for nothing;
// profiles/r04/ab_masked_*).  The hint comes from the caller, from the read
// batcher (the op log's host copy of the key DC sets) or from agn_materialize
// itself for a key_mask that agn_log_index_masks built (many_mixed).  By
// default q8e loads the key's DC set under the first chunk; AGN_Q8E_KM=1
// loads it with the segment metadata instead.
inline bool early_chunk() {
    const char *v = AGN_KNOB("AGN_COUNTER_EARLY");
    return !(v && v[0] == '0');
}

int launch_q8e(const agn_log &log, const agn_read &req, const agn_result &out, hipStream_t st) {
    DenseArgs a{req.n_req, log.n_entries, req.req_type, counter_order(req.n_req, BULK_CHUNK), 0u, 1u,
                req.hints};
    const MaskArgs mk = mask_args(log, req, out);
    if (req.n_req > 0x7fffffffull) return fail(AGN_EINVAL, "batch too large: %llu requests",
                                               (unsigned long long)req.n_req);
    // the key's DC set loaded under the first chunk (default; cold masked
    // cfg2 1.047x dense vs 1.107x with the metadata, profiles/r04/), or with
    // the segment metadata (AGN_Q8E_KM=1)
    const char *kv = AGN_KNOB("AGN_Q8E_KM");
    const bool km0 = !(kv && kv[0] == '1');
    // QL_S counters (QL_STRIDE apart), then QL_S sub-lists of ql_cap indices
    a.ql_cap = (uint32_t)((req.n_req + QL_S - 1) / QL_S);
    const size_t hdr = (size_t)QL_S * QL_STRIDE;
    uint32_t *lst = nullptr;
    AGN_HIP(pool_malloc(&lst, (hdr + (size_t)QL_S * a.ql_cap) * sizeof(uint32_t), st));
    int rc = AGN_OK;
    if (hipMemsetAsync(lst, 0, hdr * sizeof(uint32_t), st) != hipSuccess)
        rc = fail(AGN_EHIP, "counter q8e: list reset");
#define AGN_ARGS                                                                                \
    a, mk, req.keys, log.key_off, log.key_len, log.key_type, id0_index(log), log.oc, log.op_id,  \
        log.eff, log.txid, req.R, req.sct, req.sct_ignore, req.txid, req.base_value, out.value,  \
        out.hole, out.lastct, out.count, out.flags, out.err_pos, lst + hdr, lst
#define AGN_Q8E_(W, K, KM)                                                                      \
    hipLaunchKernelGGL((k_counter_q8e<W, K, KM>), dim3((unsigned)req.n_req), dim3(64), 0, st,   \
                       AGN_ARGS)
#define AGN_Q8E(W, K)                                                                           \
    do {                                                                                        \
        if (km0) AGN_Q8E_(W, K, 0);                                                             \
        else AGN_Q8E_(W, K, 1);                                                                 \
    } while (0)
    const unsigned mb = QL_S * 16u;  // a multiple of QL_S
#define AGN_Q8M(W, K)                                                                           \
    hipLaunchKernelGGL((k_counter_q8m<W, K>), dim3(mb), dim3(64), 0, st, AGN_ARGS)
    // two requests per wave (k_counter_q8e2; AGN_Q8E_TWO=0: one).
    // Warm masked cfg2 8.55 ms against q8e's 9.27 and the dense warm
    // kernel's 8.27 (profiles/r05/ab_masked_warm_q8e2_ldc.log)
    // cold batches too since the dense path went two per wave: masked cfg2
    // with the bench's hints 7.36 against 8.00 ms in one process
    // (profiles/r06/ab_masked_cold_two.log); AGN_Q8E_TWO=1: warm batches only
    const char *tv = AGN_KNOB("AGN_Q8E_TWO");
    const bool two = !(tv && tv[0] == '0');
    const bool two_cold = two && !(tv && tv[0] == '1');
    const unsigned nb2 = (unsigned)((req.n_req + 1) / 2);
#define AGN_Q8E2(W, K)                                                                          \
    hipLaunchKernelGGL((k_counter_q8e2<W, K>), dim3(nb2), dim3(64), 0, st, Q2Params{AGN_ARGS})
    if (rc == AGN_OK) {
        if (req.sct && two) {
            if (req.keys) { AGN_Q8E2(true, true); AGN_Q8M(true, true); }
            else { AGN_Q8E2(true, false); AGN_Q8M(true, false); }
        } else if (two_cold) {
            if (req.keys) { AGN_Q8E2(false, true); AGN_Q8M(false, true); }
            else { AGN_Q8E2(false, false); AGN_Q8M(false, false); }
        } else if (req.sct) {
            if (req.keys) { AGN_Q8E(true, true); AGN_Q8M(true, true); }
            else { AGN_Q8E(true, false); AGN_Q8M(true, false); }
        } else {
            if (req.keys) { AGN_Q8E(false, true); AGN_Q8M(false, true); }
            else { AGN_Q8E(false, false); AGN_Q8M(false, false); }
        }
        if (hipGetLastError() != hipSuccess) rc = fail(AGN_EHIP, "counter q8e: launch");
    }
#undef AGN_Q8E2
#undef AGN_Q8M
#undef AGN_Q8E
#undef AGN_Q8E_
#undef AGN_ARGS
    const hipError_t ef = hipFreeAsync(lst, st);
    if (rc == AGN_OK && ef != hipSuccess) rc = fail(AGN_EHIP, "hipFreeAsync: %s", hipGetErrorString(ef));
    return rc;
}

// Two chunks per step for D <= 4 (scan_key PAIR), unless AGN_COUNTER_PAIR=0
// (A/B knob).
inline uint32_t pair_chunks() {
    const char *v = AGN_KNOB("AGN_COUNTER_PAIR");
    return (v && v[0] == '0') ? 0u : 1u;
}

// Row-load variant per device.  LDS-DMA rows (even D) are box-dependent: on
// two MI355X boxes they beat the VGPR-load path by 7-10 % (cfg2 7.29-7.55 vs
// 8.16-8.44 ms), on three others they lost by 6-14 % (8.86-9.28 vs 7.95-8.39
// ms), consistently across processes on one box (profiles/r01/ab_counter_
// glds*.log).  Quad rows (D = 8) beat VGPR rows by 4-6 % on the boxes
// measured (cfg2 7.81 vs 8.24-8.30 ms, warm 8.35 vs 8.68 ms;
// profiles/r02/ab_counter_quad*.log), so they are the untuned default for
// D = 8 and VGPR rows for other D.  agn_tune times the bit-identical variants
// on the caller's batch and keeps another one for the device only when it is
// at least 3 % faster than that default.  AGN_COUNTER_VARIANT=0/1/2 (or the
// older AGN_COUNTER_GLDS=0/1) forces the choice.
constexpr int kMaxDev = 64;
// per device: 0 untuned (the default of the shape), else 1 + ROWS_VGPR /
// ROWS_GLDS / ROWS_QUAD
std::atomic<int> g_rows_choice[kMaxDev];

template <int D>
constexpr int default_variant() { return D == 8 ? ROWS_QUAD : ROWS_VGPR; }

inline int cur_dev() {
    int d = 0;
    (void)hipGetDevice(&d);
    return d >= 0 && d < kMaxDev ? d : 0;
}

inline int forced_variant() {
    const char *v = AGN_KNOB("AGN_COUNTER_VARIANT");
    if (v && v[0] >= '0' && v[0] <= '3') return v[0] - '0';
    v = AGN_KNOB("AGN_COUNTER_GLDS");
    if (v && (v[0] == '0' || v[0] == '1')) return v[0] - '0';
    return -1;
}

inline int tuned_variant() {  // -1 = untuned
    return g_rows_choice[cur_dev()].load(std::memory_order_relaxed) - 1;
}

template <int D>
int counter_variant() {
    const int f = forced_variant();
    if (f >= 0) return f;
    const int t = tuned_variant();
    return t >= 0 ? t : default_variant<D>();
}

template <int D, int WPB, int VAR, bool KEYS, bool MSK>
int launch_key_k(const agn_log &log, const agn_read &req, const agn_result &out, hipStream_t st) {
    const char *qv = AGN_KNOB("AGN_COUNTER_QUAD_NT");
    DenseArgs a{req.n_req, log.n_entries, req.req_type, counter_order(req.n_req, BULK_CHUNK), pair_chunks(),
                (qv && qv[0] >= '0' && qv[0] <= '3') ? (uint32_t)(qv[0] - '0') : 1u};
    const MaskArgs mk = mask_args(log, req, out);
    const uint64_t nb = (req.n_req + WPB - 1) / WPB;
    if (nb > 0x7fffffffull) return fail(AGN_EINVAL, "batch too large: %llu requests",
                                        (unsigned long long)req.n_req);
    if (req.sct)
        hipLaunchKernelGGL((k_counter_key<D, true, WPB, VAR, KEYS, MSK>), dim3((unsigned)nb),
                           dim3(64 * WPB), 0, st, a, mk, req.keys, log.key_off, log.key_len,
                           log.key_type, id0_index(log), log.oc, log.op_id, log.eff, log.txid,
                           req.R, req.sct, req.sct_ignore, req.txid, req.base_value, out.value,
                           out.hole, out.lastct, out.count, out.flags, out.err_pos);
    else
        hipLaunchKernelGGL((k_counter_key<D, false, WPB, VAR, KEYS, MSK>), dim3((unsigned)nb),
                           dim3(64 * WPB), 0, st, a, mk, req.keys, log.key_off, log.key_len,
                           log.key_type, id0_index(log), log.oc, log.op_id, log.eff, log.txid,
                           req.R, req.sct, req.sct_ignore, req.txid, req.base_value, out.value,
                           out.hole, out.lastct, out.count, out.flags, out.err_pos);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

template <int D, int WPB, int VAR, bool MSK>
int launch_key_g(const agn_log &log, const agn_read &req, const agn_result &out, hipStream_t st) {
    return req.keys ? launch_key_k<D, WPB, VAR, true, MSK>(log, req, out, st)
                    : launch_key_k<D, WPB, VAR, false, MSK>(log, req, out, st);
}

// The variants this D has: VGPR rows always, LDS-DMA rows for even D, quad
// rows for D = 8.
template <int D>
constexpr bool has_variant(int v) {
    return v == ROWS_VGPR || (v == ROWS_GLDS && D % 2 == 0) || (v == ROWS_QUAD && D == 8);
}

// A sparse batch (presence masks, MSK) runs VGPR or quad rows: the LDS-DMA
// variant has no per-entry-mask scan for its mixed keys.
template <int D, int WPB, bool MSK>
int launch_var(int v, const agn_log &log, const agn_read &req, const agn_result &out,
               hipStream_t st) {
    if constexpr (D % 2 == 0 && !MSK)
        if (v == ROWS_GLDS) return launch_key_g<D, WPB, ROWS_GLDS, false>(log, req, out, st);
    if constexpr (D == 8)
        if (v == ROWS_QUAD || (MSK && v == ROWS_GLDS)) {
            if (MSK && WPB == 1 && early_chunk() && !(req.hints & AGN_HINT_MIXED))
                return launch_q8e(log, req, out, st);
            return launch_key_g<D, WPB, ROWS_QUAD, MSK>(log, req, out, st);
        }
    return launch_key_g<D, WPB, ROWS_VGPR, MSK>(log, req, out, st);
}

template <int D, int WPB>
int launch_key(const agn_log &log, const agn_read &req, const agn_result &out, hipStream_t st) {
    const int v = counter_variant<D>();
    // quad rows, dense batch, not forced: two requests per wave -- warm cfg2
    // 8.37-8.45 vs 8.83-9.02 ms (profiles/r02/ab_counter_quad2.log); cold
    // batches too since the blocks go to the XCDs in runs (block_order):
    // cold cfg2 7.28 vs 7.46 ms in one process (round 2, identity order: no
    // change; profiles/r06/ab_counter_quad2_cold.log).  A masked batch keeps
    // one request per wave (its two-request form takes 118 VGPRs, 4 waves per
    // SIMD: warm masked cfg2 13.06 vs 11.06 ms, mixed keys 17.32 vs 13.00;
    // profiles/r03/ab_masked_warm_quad{2,1}.log)
    const bool masked = sparse_batch(log, req, out);
    if constexpr (D == 8)
        if (v == ROWS_QUAD2 || (v == ROWS_QUAD && !masked && forced_variant() < 0))
            return launch_quad2(log, req, out, st);
    const int v2 = v == ROWS_QUAD2 ? default_variant<D>() : v;
    return masked ? launch_var<D, WPB, true>(v2, log, req, out, st)
                  : launch_var<D, WPB, false>(v2, log, req, out, st);
}

// Waves (= requests) per block: 1 measured 1.4-3.4 % faster than 2 and
// 0-1.6 % faster than 4 on cfg2 (profiles/r01/ab_counter_wpb.log), so only
// WPB = 1 is instantiated.
template <int D>
int launch_dense(const agn_log &log, const agn_read &req, const agn_result &out,
                 hipStream_t st) {
    return launch_key<D, 1>(log, req, out, st);
}

// agn_log_index_masks: one wave per key; out[k] = the mask word every entry
// of the segment carries (low D bits), 0 when they differ or the key is empty.
// The block's mixed keys (non-empty, entries differ) are added to one of
// IM_CNT counters (IM_STRIDE words apart: one counter per 128-byte line).
constexpr uint32_t IM_CNT = 256, IM_STRIDE = 16;
__global__ __launch_bounds__(256) void k_index_masks(const uint64_t *__restrict__ key_off,
                                                    const uint64_t *__restrict__ key_len,
                                                    const uint64_t *__restrict__ oc_mask,
                                                    uint64_t full, uint64_t n_keys,
                                                    uint64_t *__restrict__ out,
                                                    unsigned long long *__restrict__ mixed) {
    __shared__ uint32_t blk_mixed;
    if (threadIdx.x == 0) blk_mixed = 0;
    __syncthreads();
    const uint64_t k = uniform_u64((uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6));
    const int lane = lane_id();
    if (k < n_keys) {
        const uint64_t off = key_off[k];
        const uint64_t n = key_len ? key_len[k] : key_off[k + 1] - off;
        if (n == 0 || oc_mask == nullptr) {
            if (lane == 0) out[k] = n ? full : 0ull;
        } else {
            const uint64_t m0 = uniform_u64(oc_mask[off]) & full;
            bool ok = true;
            for (uint64_t b = 0; ok && b < n; b += AGN_WAVE) {
                const uint64_t p = b + (uint64_t)lane;
                const bool bad = p < n && (oc_mask[off + p] & full) != m0;
                ok = ballot(bad) == 0;
            }
            if (lane == 0) {
                out[k] = ok ? m0 : 0ull;
                if (!ok) atomicAdd(&blk_mixed, 1u);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && blk_mixed && mixed)
        atomicAdd(&mixed[(blockIdx.x % IM_CNT) * IM_STRIDE], (unsigned long long)blk_mixed);
}

// agn_log_index_ids: one wave per key, lanes over the segment's positions.
__global__ __launch_bounds__(256) void k_index_ids(const uint64_t *__restrict__ key_off,
                                                  const uint64_t *__restrict__ key_len,
                                                  const uint32_t *__restrict__ op_id,
                                                  uint64_t n_keys, uint32_t *__restrict__ out) {
    const uint64_t k = uniform_u64((uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6));
    if (k >= n_keys) return;
    const int lane = lane_id();
    const uint64_t off = key_off[k];
    const uint64_t n = key_len ? key_len[k] : key_off[k + 1] - off;
    if (n == 0) {
        if (lane == 0) out[k] = AGN_ID0_NONE;
        return;
    }
    const uint64_t id0 = op_id[off];
    bool ok = id0 + (n - 1) < (uint64_t)AGN_ID0_NONE;  // id0 + p fits and is never NONE
    for (uint64_t b = 0; ok && b < n; b += AGN_WAVE) {
        const uint64_t p = b + (uint64_t)lane;
        const bool bad = p < n && (uint64_t)op_id[off + p] != id0 + p;
        ok = ballot(bad) == 0;
    }
    if (lane == 0) out[k] = ok ? (uint32_t)id0 : AGN_ID0_NONE;
}

}  // namespace

int launch_index_masks(const agn_log &log, uint64_t *out, uint64_t *mixed, hipStream_t st) {
    const uint64_t nb = (log.n_keys + 3) / 4;
    if (mixed) *mixed = 0;
    if (nb == 0) return AGN_OK;
    if (nb > 0x7fffffffull) return fail(AGN_EINVAL, "index_masks: too many keys");
    if (log.n_dcs > 64) return fail(AGN_ENOTSUP, "index_masks: n_dcs %u > 64", log.n_dcs);
    unsigned long long *cnt = nullptr;
    const size_t cb = (size_t)IM_CNT * IM_STRIDE * sizeof(unsigned long long);
    if (mixed) {
        AGN_HIP(pool_malloc(&cnt, cb, st));
        if (hipMemsetAsync(cnt, 0, cb, st) != hipSuccess) {
            (void)hipFreeAsync(cnt, st);
            return fail(AGN_EHIP, "index_masks: counter reset");
        }
    }
    hipLaunchKernelGGL(k_index_masks, dim3((unsigned)nb), dim3(256), 0, st, log.key_off,
                       log.key_len, log.oc_mask, low_bits(log.n_dcs), log.n_keys, out, cnt);
    int rc = hipGetLastError() == hipSuccess ? AGN_OK : fail(AGN_EHIP, "index_masks: launch");
    if (cnt) {
        // the count is read back here: the call blocks until the index is built
        std::vector<unsigned long long> h((size_t)IM_CNT * IM_STRIDE);
        if (rc == AGN_OK &&
            (hipMemcpyAsync(h.data(), cnt, cb, hipMemcpyDeviceToHost, st) != hipSuccess ||
             hipStreamSynchronize(st) != hipSuccess))
            rc = fail(AGN_EHIP, "index_masks: mixed-key count");
        if (rc == AGN_OK)
            for (uint32_t i = 0; i < IM_CNT; ++i) *mixed += h[(size_t)i * IM_STRIDE];
        (void)hipFreeAsync(cnt, st);
    }
    return rc;
}

int launch_index_ids(const agn_log &log, uint32_t *out, hipStream_t st) {
    const uint64_t nb = (log.n_keys + 3) / 4;
    if (nb == 0) return AGN_OK;
    if (nb > 0x7fffffffull) return fail(AGN_EINVAL, "index_ids: too many keys");
    hipLaunchKernelGGL(k_index_ids, dim3((unsigned)nb), dim3(256), 0, st, log.key_off,
                       log.key_len, log.op_id, log.n_keys, out);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

// agn_tune for the dense counter path: alternate the row-load variants this
// D has over the caller's batch (`rounds` launches each, on `st`), keep each
// variant's fastest launch, and select another variant than the shape's
// default for this device only when it is at least 3 % faster.  All write
// the same results, so `out` holds the batch's results afterwards.  ms[v] =
// fastest launch of variant v (0 when absent).
template <int D>
int tune_dense(const agn_log &log, const agn_read &req, const agn_result &out, hipStream_t st,
               int rounds, int *choice, float *ms) {
    hipEvent_t e0, e1;
    AGN_HIP(hipEventCreate(&e0));
    if (hipEventCreate(&e1) != hipSuccess) {
        (void)hipEventDestroy(e0);
        return fail(AGN_EHIP, "tune: hipEventCreate");
    }
    constexpr int NV = 3;
    float best[NV] = {3.4e38f, 3.4e38f, 3.4e38f};
    int rc = AGN_OK;
    for (int r = 0; r < rounds && rc == AGN_OK; ++r) {
        for (int k = 0; k < NV && rc == AGN_OK; ++k) {
            const int var = (r & 1) ? NV - 1 - k : k;  // alternate which variant goes first
            if (!has_variant<D>(var)) continue;
            if (hipEventRecord(e0, st) != hipSuccess) { rc = fail(AGN_EHIP, "tune: record"); break; }
            // quad rows run two requests per wave on a dense batch (launch_key)
            if constexpr (D == 8)
                rc = var == ROWS_QUAD ? launch_quad2(log, req, out, st)
                                      : launch_var<D, 1, false>(var, log, req, out, st);
            else
                rc = launch_var<D, 1, false>(var, log, req, out, st);
            if (rc) break;
            float t = 0.f;
            if (hipEventRecord(e1, st) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                hipEventElapsedTime(&t, e0, e1) != hipSuccess) {
                rc = fail(AGN_EHIP, "tune: event timing");
                break;
            }
            best[var] = t < best[var] ? t : best[var];
        }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc) return rc;
    const int d0 = default_variant<D>();
    int c = d0;
    for (int v = 0; v < NV; ++v)
        if (v != d0 && has_variant<D>(v) && best[v] < 0.97f * best[d0] && best[v] < best[c]) c = v;
    g_rows_choice[cur_dev()].store(c + 1, std::memory_order_relaxed);
    *choice = c;
    if (ms)
        for (int v = 0; v < NV; ++v) ms[v] = has_variant<D>(v) ? best[v] : 0.f;
    return AGN_OK;
}

// Dense fast path applies when every clock is dense and D <= 8; returns
// AGN_ENOTSUP otherwise so the caller uses the general kernel.
int launch_counter_dense(const agn_log &log, const agn_read &req, const agn_result &out,
                         hipStream_t st) {
    // presence masks (D <= 8: one word per clock) run the MSK instantiations
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

// Tunable only for the dense counter path with even D (the LDS-DMA variant
// exists there); AGN_ENOTSUP otherwise, before anything is launched.
int tune_counter_dense(const agn_log &log, const agn_read &req, const agn_result &out,
                       hipStream_t st, int rounds, int *choice, float *ms) {
    if (log.crdt_type != AGN_COUNTER_PN || log.oc_mask || req.R_mask || req.sct_mask ||
        out.lastct_mask || req.n_req == 0)
        return AGN_ENOTSUP;
    const char *impl = AGN_KNOB("AGN_COUNTER_IMPL");
    if (impl && impl[0] == 'g') return AGN_ENOTSUP;  // general kernel forced
    switch (log.n_dcs) {
        case 2: return tune_dense<2>(log, req, out, st, rounds, choice, ms);
        case 4: return tune_dense<4>(log, req, out, st, rounds, choice, ms);
        case 6: return tune_dense<6>(log, req, out, st, rounds, choice, ms);
        case 8: return tune_dense<8>(log, req, out, st, rounds, choice, ms);
        default: return AGN_ENOTSUP;
    }
}

}  // namespace agn
