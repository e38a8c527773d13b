// gc.hip — garbage collection of the device op log on gfx950:
// materializer_vnode:snapshot_insert_gc -> prune_ops/check_filter
// (src/materializer_vnode.erl:513-604).  For every key selected for GC the
// ops already covered by the pruned snapshot are dropped:
//   keep(op) = belongs_to_snapshot_op(Threshold, op)
//            = not vectorclock:le(OpSSCommit, Threshold)   (src/materializer.erl:101-106)
// in log order (check_filter keeps the survivors' order, :592-604).
//
// Out-of-place stream compaction in three HBM-bound passes:
//   1. k_prune_mark   one wave per key: the VC filter over the key's
//      OpSSCommit rows (filter.hpp shape: LPO lanes x DPL DCs per op) writes
//      one keep byte per entry, the key's kept-entry and kept-token counts;
//   2. two inclusive scans (hipcub) turn the counts into the new key_off and
//      the per-key base of the new removal-token CSR;
//   3. k_prune_scatter one wave per key, 64 entries per step: ballot prefix
//      -> destination slot; the kept OpSSCommit rows are copied
//      cooperatively (kept-rank -> source entry through LDS, so reads and
//      writes are lane-contiguous), the per-entry fields lane = entry, and the
//      removal tokens after a wave scan of the kept list lengths.
// HBM bytes per entry: pass 1 reads 8*D (+4 rem_off for tag logs) and writes
// 1; pass 3 reads 1 + the entry's fields and writes the kept ones.
#include <hipcub/hipcub.hpp>

#include "filter.hpp"
#include "serve.hpp"

namespace agn {
namespace {

template <int DPL, int LPO, bool SPARSE, bool FULL>
__global__ __launch_bounds__(256) void k_prune_mark(agn_log log, const uint8_t *__restrict__ prune,
                                                    const uint64_t *__restrict__ thr,
                                                    const uint64_t *__restrict__ thr_mask,
                                                    uint8_t *__restrict__ keep,
                                                    uint64_t *__restrict__ cnt,
                                                    uint64_t *__restrict__ rcnt) {
    using S = Shape<DPL, LPO>;
    const uint64_t k = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    if (k >= log.n_keys) return;
    const int lane = lane_id();
    const int sub = lane % LPO, slot = lane / LPO, d0 = sub * DPL;
    const uint32_t D = log.n_dcs, W = n_words(D);
    const uint64_t off = uniform_u64(log.key_off[k]);
    const uint64_t n = uniform_u64(key_n(log.key_off, log.key_len, k));
    const bool gc = prune == nullptr || prune[k] != 0;
    // the threshold slice this lane compares (missing entry = 0)
    uint64_t t[DPL];
    const uint32_t tbits = chunk_bits<DPL, SPARSE>(thr_mask, k, W, d0, D);
#pragma unroll
    for (int j = 0; j < DPL; ++j) t[j] = ((tbits >> j) & 1u) ? thr[k * D + (uint32_t)(d0 + j)] : 0ull;
    uint64_t kept = 0, rk = 0;
    for (uint64_t b = 0; b < n; b += S::OPI) {
        const uint64_t pos = b + (uint64_t)slot;
        const bool valid = pos < n;
        const uint64_t e = off + (valid ? pos : 0ull);
        bool le = true;
        if (gc) {
            uint64_t o[DPL];
            uint32_t obits;
            load_rows<DPL, SPARSE, FULL>(log, e, d0, D, W, o, obits);
            if (!valid) obits = 0u;
#pragma unroll
            for (int j = 0; j < DPL; ++j)
                if ((obits >> j) & 1u) le = le && (o[j] <= t[j]);
            if (LPO > 1) {
                const uint64_t grp = ((1ull << LPO) - 1ull) << (slot * LPO);
                le = (ballot(!le) & grp) == 0ull;
            }
        }
        const bool kp = valid && (!gc || !le);  // belongs_to_snapshot_op
        if (valid && sub == 0) keep[e] = kp ? 1 : 0;
        kept += (uint64_t)__builtin_popcountll(ballot(kp && sub == 0));
        if (log.rem_off != nullptr && kp && sub == 0) rk += log.rem_off[e + 1] - log.rem_off[e];
    }
    rk = (uint64_t)wave_sum_i64((int64_t)rk);
    if (lane == 0) {
        cnt[k] = kept;
        rcnt[k] = rk;
    }
}

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
    const int lane = lane_id();
#pragma unroll
    for (int x = 1; x < AGN_WAVE; x <<= 1) {
        const uint32_t o = (uint32_t)__shfl_up((int)v, x, AGN_WAVE);
        if (lane >= x) v += o;
    }
    return v;
}

__global__ __launch_bounds__(256) void k_prune_scatter(agn_log log, agn_log out,
                                                       const uint8_t *__restrict__ prune,
                                                       const uint8_t *__restrict__ keep,
                                                       const uint64_t *__restrict__ rbase,
                                                       uint32_t *__restrict__ flags, int seg) {
    __shared__ uint64_t src[4][AGN_WAVE];
    const int w = threadIdx.x >> 6;
    const uint64_t k = (uint64_t)blockIdx.x * 4u + (uint64_t)w;
    if (k >= log.n_keys) return;
    const int lane = lane_id();
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const uint32_t D = log.n_dcs, W = n_words(D);
    const uint64_t off = uniform_u64(log.key_off[k]);
    const uint64_t n = uniform_u64(key_n(log.key_off, log.key_len, k));
    const uint64_t noff = uniform_u64(out.key_off[k]);
    uint64_t written = 0, rwritten = 0;
    const uint64_t rb = rbase ? uniform_u64(rbase[k]) : 0ull;
    if (seg) {  // segmented output: the key owns [noff, noff + cap + 1), ~0 = none
        if (noff == ~0ull) {
            if (lane == 0 && flags) flags[k] = (prune == nullptr || prune[k] != 0) ? AGN_GC_ALL_PRUNED : 0u;
            return;
        }
        // the segment's first rem_off slot is its own token base (CSR: the
        // previous key's end, written by that key)
        if (lane == 0 && log.rem_off) ((uint32_t *)out.rem_off)[noff] = (uint32_t)rb;
    }
    for (uint64_t b = 0; b < n; b += AGN_WAVE) {
        const uint64_t pos = b + (uint64_t)lane;
        const bool valid = pos < n;
        const uint64_t e = off + (valid ? pos : 0ull);
        const bool kp = valid && keep[e] != 0;
        const uint64_t m = ballot(kp);
        const uint32_t nk = (uint32_t)__builtin_popcountll(m);
        const uint64_t dst = noff + written + (uint64_t)__builtin_popcountll(m & lt);
        if (kp) {
            src[w][__builtin_popcountll(m & lt)] = e;
            ((uint32_t *)out.op_id)[dst] = log.op_id[e];
            if (log.txid) ((uint64_t *)out.txid)[dst] = log.txid[e];
            if (log.eff) ((int64_t *)out.eff)[dst] = log.eff[e];
            if (log.tag) ((uint32_t *)out.tag)[dst] = log.tag[e];
            if (log.add_tok) ((uint64_t *)out.add_tok)[dst] = log.add_tok[e];
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // kept OpSSCommit rows (and masks): rank-major, lane-contiguous copy
        // (16-byte units when D is even)
        uint64_t *ooc = (uint64_t *)out.oc + (noff + written) * D;
        if ((D & 1u) == 0u) {
            const uint32_t H = D / 2;
            u64x2 *o2 = reinterpret_cast<u64x2 *>(ooc);
            const u64x2 *i2 = reinterpret_cast<const u64x2 *>(log.oc);
            for (uint64_t x = (uint64_t)lane; x < (uint64_t)nk * H; x += AGN_WAVE)
                o2[x] = i2[src[w][x / H] * H + x % H];
        } else {
            for (uint64_t x = (uint64_t)lane; x < (uint64_t)nk * D; x += AGN_WAVE)
                ooc[x] = log.oc[src[w][x / D] * D + x % D];
        }
        if (log.oc_mask) {
            uint64_t *om = (uint64_t *)out.oc_mask + (noff + written) * W;
            for (uint64_t x = (uint64_t)lane; x < (uint64_t)nk * W; x += AGN_WAVE)
                om[x] = log.oc_mask[src[w][x / W] * W + x % W];
        }
        // removal tokens: kept lists, concatenated in order
        if (log.rem_off) {
            const uint32_t r0 = kp ? log.rem_off[e] : 0u;
            const uint32_t len = kp ? log.rem_off[e + 1] - r0 : 0u;
            const uint32_t incl = wave_incl_scan_u32(len);
            const uint64_t start = rb + rwritten + (uint64_t)(incl - len);
            if (kp) {
                ((uint32_t *)out.rem_off)[dst + 1] = (uint32_t)(start + len);
                for (uint32_t j = 0; j < len; ++j)
                    ((uint64_t *)out.rem_tok)[start + j] = log.rem_tok[r0 + j];
            }
            rwritten += (uint64_t)__builtin_amdgcn_readlane(incl, 63);
        }
        written += nk;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0 && flags) {
        const bool gc = prune == nullptr || prune[k] != 0;
        // every op covered: the reference stores element(?FIRST_OP+Len) (:580-583)
        flags[k] = (gc && written == 0) ? AGN_GC_ALL_PRUNED : 0u;
    }
}

template <int DPL, int LPO, bool SPARSE>
int mark_shape(const agn_log &log, const uint8_t *prune, const uint64_t *thr,
               const uint64_t *thr_mask, uint8_t *keep, uint64_t *cnt, uint64_t *rcnt,
               hipStream_t st) {
    const unsigned blocks = grid_for(log.n_keys, 4, 0x7fffffffu);
    // FULL: dense rows that split exactly into 16-byte loads
    const bool full = !log.oc_mask && (DPL % 2 == 0) && log.n_dcs == (uint32_t)(DPL * LPO);
    if (full)
        hipLaunchKernelGGL((k_prune_mark<DPL, LPO, SPARSE, (DPL % 2 == 0)>), dim3(blocks),
                           dim3(256), 0, st, log, prune, thr, thr_mask, keep, cnt, rcnt);
    else
        hipLaunchKernelGGL((k_prune_mark<DPL, LPO, SPARSE, false>), dim3(blocks), dim3(256), 0,
                           st, log, prune, thr, thr_mask, keep, cnt, rcnt);
    return hipGetLastError() == hipSuccess ? AGN_OK : fail(AGN_EHIP, "k_prune_mark launch");
}

template <bool SPARSE>
int mark(const agn_log &log, const uint8_t *prune, const uint64_t *thr, const uint64_t *thr_mask,
         uint8_t *keep, uint64_t *cnt, uint64_t *rcnt, hipStream_t st) {
#define AGN_L(DPL, LPO) mark_shape<DPL, LPO, SPARSE>(log, prune, thr, thr_mask, keep, cnt, rcnt, st)
    AGN_DISPATCH_SHAPES(log.n_dcs, AGN_L)
#undef AGN_L
}

}  // namespace

int launch_prune_ops(const agn_log &log, const uint8_t *prune, const uint64_t *thr,
                     const uint64_t *thr_mask, const agn_log &out, uint32_t *flags,
                     uint64_t *totals, hipStream_t st) {
    const uint64_t K = log.n_keys, E = log.n_entries;
    const bool tags = log.rem_off != nullptr;
    size_t scan_bytes = 0, scan_bytes2 = 0;
    AGN_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, scan_bytes, (uint64_t *)nullptr,
                                             (uint64_t *)nullptr, (int)K, st));
    if (tags)
        AGN_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, scan_bytes2, (uint64_t *)nullptr,
                                                 (uint64_t *)nullptr, (int)K, st));
    if (scan_bytes2 > scan_bytes) scan_bytes = scan_bytes2;
    // layout: [scan temp (256-aligned, rocPRIM assumes an aligned base)]
    //         [keep E bytes][cnt K+1][rcnt K+1][rbase K+1]
    const size_t tmp_bytes = (scan_bytes + 255) / 256 * 256;
    const size_t keep_bytes = (E + 255) / 256 * 256;
    const size_t bytes = tmp_bytes + keep_bytes + 3 * (K + 1) * sizeof(uint64_t) + 256;
    uint8_t *scratch = nullptr;
    AGN_HIP(pool_malloc((void **)&scratch, bytes, st));
    void *tmp = scratch;
    uint8_t *keep = scratch + tmp_bytes;
    uint64_t *cnt = (uint64_t *)(keep + keep_bytes);
    uint64_t *rcnt = cnt + (K + 1);
    uint64_t *rbase = rcnt + (K + 1);
    int rc = AGN_OK;
    const bool sparse = log.oc_mask || thr_mask;
    if (K) rc = sparse ? mark<true>(log, prune, thr, thr_mask, keep, cnt, rcnt, st)
                       : mark<false>(log, prune, thr, thr_mask, keep, cnt, rcnt, st);
    hipError_t e = hipSuccess;
    // new key_off = [0, inclusive scan of cnt]; token bases likewise
    if (rc == AGN_OK) e = hipMemsetAsync((void *)out.key_off, 0, sizeof(uint64_t), st);
    if (rc == AGN_OK && e == hipSuccess && K)
        e = hipcub::DeviceScan::InclusiveSum(tmp, scan_bytes, cnt, (uint64_t *)out.key_off + 1,
                                             (int)K, st);
    if (rc == AGN_OK && e == hipSuccess && tags) {
        e = hipMemsetAsync(rbase, 0, sizeof(uint64_t), st);
        if (e == hipSuccess) e = hipMemsetAsync((void *)out.rem_off, 0, sizeof(uint32_t), st);
        if (e == hipSuccess && K)
            e = hipcub::DeviceScan::InclusiveSum(tmp, scan_bytes, rcnt, rbase + 1, (int)K, st);
    }
    if (rc == AGN_OK && e == hipSuccess && K) {
        hipLaunchKernelGGL(k_prune_scatter, dim3(grid_for(K, 4, 0x7fffffffu)), dim3(256), 0, st,
                           log, out, prune, keep, tags ? rbase : nullptr, flags, 0);
        e = hipGetLastError();
    }
    if (rc == AGN_OK && e == hipSuccess && totals) {
        e = hipMemcpyAsync(totals, (const uint64_t *)out.key_off + K, sizeof(uint64_t),
                           hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess)
            e = tags ? hipMemcpyAsync(totals + 1, rbase + K, sizeof(uint64_t),
                                      hipMemcpyDeviceToDevice, st)
                     : hipMemsetAsync(totals + 1, 0, sizeof(uint64_t), st);
    }
    if (rc == AGN_OK && e != hipSuccess) rc = fail(AGN_EHIP, "prune_ops: %s", hipGetErrorString(e));
    const hipError_t ef = hipFreeAsync(scratch, st);
    if (rc == AGN_OK && ef != hipSuccess) rc = fail(AGN_EHIP, "hipFreeAsync: %s", hipGetErrorString(ef));
    return rc;
}

// ---- in-place prune of the engine-owned op log (agn_oplog_prune) -----------
// snapshot_insert_gc -> prune_ops over the segmented arena, in place and in
// ONE pass: each wave owns a key, runs the VC filter over the key's entries
// (the mark loop above) and compacts the kept entries toward the segment
// start while their OpSSCommit slices are still in registers -- every row is
// read once, every kept row written once, unselected keys cost nothing.
// Compaction is safe in place: the destination of an entry is never above
// its source, every load of an iteration precedes its stores in program
// order (one pointer per array, no __restrict__, so the compiler keeps that
// order), and an iteration only writes slots below the next iteration's
// sources.  Removal tokens move the same way; a lane buffers up to PT tokens
// in registers before any lane stores, and an iteration with a longer list
// copies its lists one entry at a time in position order instead.
// Per key it then writes the new key_len, key_id0 (consecutive-id base or
// AGN_ID0_NONE), the ETS ListLen after the resize policy (:540-558, with
// prune_ops' NewLength = 1 when nothing survives, :580-583) and
// meta[4][K] = {len, token len, ListLen, id0} for the host's bookkeeping
// (the engine-owned log: [6][K], the last two rows 0 here -- see k_prune_tail).
//
// The same kernel runs out of place into segmented output (agn_prune_ops
// with out.key_len): every key keeps its input segment start in the output
// arrays and only its length changes -- no prefix scan over the keys, one pass,
// rows still read once and kept rows written once; unselected keys are copied.
namespace {

struct InplaceArgs {
    // source arrays, and the destination arrays (the same pointers in place)
    const uint64_t *oc, *mask, *txid, *add, *tok;
    const uint32_t *op_id, *tag, *rem_off;
    const int64_t *eff;
    uint64_t *d_oc, *d_mask, *d_txid, *d_add, *d_tok;
    uint32_t *d_op_id, *d_tag, *d_rem_off;
    int64_t *d_eff;
    const uint64_t *key_off;
    const uint64_t *key_len;   // input lengths, NULL = CSR (key_off[k+1] - key_off[k])
    uint64_t *d_key_len;       // output lengths
    uint64_t *d_key_off;       // out of place: the output segment starts (= input), or NULL
    uint32_t *key_id0, *key_lcap;  // may be NULL (no index / no ListLen)
    uint64_t n_keys;
    uint32_t D, W;
    int copy_unselected;       // out of place: keys with prune[k] == 0 are copied whole
    uint32_t xcd;              // block_order mode
    int late_fields;           // entry fields loaded after the filter (kept entries only)
    // key-list launch (n_keys = list length): entry i is key key_list[i], GC'd
    // iff list_flags[i] != 0; meta is indexed by i.  NULL = every key, by prune[k].
    const uint64_t *key_list;
    const uint8_t *list_flags;
    // engine-owned log: meta has 6 rows, the last two the key's live range
    // start after the prune (entry slot, token slot; arenas < 2^32 slots)
    int meta6;
};

__device__ __forceinline__ uint32_t resize_list_len_dev(uint32_t new_len, uint32_t list_len) {
    if ((int64_t)new_len > (int64_t)list_len - AGN_RESIZE_THRESHOLD) return list_len * 2u;
    const uint32_t half = list_len / 2u;
    if (half <= AGN_OPS_THRESHOLD) return list_len;
    return ((int64_t)half - AGN_RESIZE_THRESHOLD > (int64_t)new_len) ? half : list_len;
}

constexpr int PT = 4;  // removal tokens a lane buffers per entry

// Staged field stores (k_prune_inplace, set/register): the kept entries' per-entry fields
// (op id, txid, effect or tag + add token + token start) go to a per-wave LDS
// ring and leave it in runs of 33-64 entries whose ends fall on 32-entry
// (128-byte) boundaries, lane = entry: every interior line of the field
// arrays is written whole by one store instruction, where the head lanes of
// an iteration stored <= 32 scattered words each (every other lane at
// LPO = 2) and left partial lines at both ends of every iteration.  Delaying
// a store is safe in place: a destination is never above its source and
// later iterations read only higher sources.  AGN_PRUNE_STAGE=0 at build time
// keeps the direct stores (A/B).
#ifndef AGN_PRUNE_STAGE
#define AGN_PRUNE_STAGE 1
#endif
constexpr bool PRUNE_STAGE = AGN_PRUNE_STAGE != 0;
constexpr uint32_t SRING = 128;  // ring slots: < 64 pending + one iteration's kept

// The kept entries' removal tokens the same way (set/register, lists of <= PT
// tokens): a 512-token ring leaving in runs of 113-128 tokens that end on a
// 16-token (128-byte) boundary; an iteration that copies its lists another
// way (a list longer than PT) first empties the ring.
// AGN_PRUNE_STAGE_TOK=0 at build time keeps the direct token stores (A/B).
#ifndef AGN_PRUNE_STAGE_TOK
#define AGN_PRUNE_STAGE_TOK 1
#endif
constexpr uint32_t TRING = 512;
template <bool ON>
struct TokRing {
    uint64_t t[ON ? TRING : 1];
};

template <bool ON>
struct FieldRing {
    static constexpr uint32_t N = ON ? SRING : 1u;
    uint64_t tx[N];
    uint64_t w64[N];  // add token (set/register) or effect (counter)
    uint32_t id[N];
    uint32_t tg[N];   // set/register: tag
    uint32_t ro[N];   // set/register: the entry's token start
};

// CTL (dense rows, 8 DCs per lane-slice): an iteration's rows are read
// lane-contiguously -- load j covers bytes [1 KiB j, 1 KiB (j+1)), whole
// lines, lane l holding DCs 2p, 2p+1 (p = l mod P, P = D / 2) of op
// j (64 / P) + l / P -- where the row-slice loads touch every line of the
// iteration with each instruction and re-request it (the tags kernel's CT
// rows, k_tags).  Verdicts are group-any folds of wave ballots; a kept row is
// stored from the same registers (its parts' lanes fetch its destination).
template <int DPL, int LPO, bool SPARSE, bool FULL, bool TAGS, int WPB, bool CTL = false,
          int PF = 0, int MINW = 1>
__global__ __launch_bounds__(64 * WPB, PF == 2 ? 5 : MINW) void k_prune_inplace(InplaceArgs a,
                                                       const uint8_t *__restrict__ prune,
                                                       const uint64_t *__restrict__ thr,
                                                       const uint64_t *__restrict__ thr_mask,
                                                       uint32_t *__restrict__ meta,
                                                       uint32_t *__restrict__ flags) {
    using S = Shape<DPL, LPO>;
    static_assert(!CTL || (FULL && !SPARSE && DPL == 8), "CTL: dense 8-DC slices");
    static_assert(PF == 0 || !CTL, "PF: row-slice loads");
    constexpr int P = DPL * LPO >= 2 ? DPL * LPO / 2 : 1;  // CTL: 16-byte parts per op
    constexpr int OPL = AGN_WAVE / P;                      // CTL: ops per 1 KiB load
    constexpr int NQ = DPL >= 2 ? DPL / 2 : 1;             // CTL: loads per lane
    // XCD-aware key order: consecutive keys (whose per-key outputs share lines)
    // run on one XCD's L2
    const uint32_t blk = block_order(a.xcd, blockIdx.x, gridDim.x);
    const uint64_t i = (uint64_t)blk * WPB + (WPB == 1 ? 0u : (threadIdx.x >> 6));
    if (i >= a.n_keys) return;
    const uint64_t K = a.n_keys;   // launch size (meta stride)
    const uint64_t k = a.key_list ? uniform_u64(ldc(a.key_list + i)) : i;
    const int lane = lane_id();
    const int sub = lane % LPO, slot = lane / LPO, d0 = sub * DPL;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const uint32_t D = a.D, W = a.W;
    constexpr bool tags = TAGS;
    // staged stores for set/register (counter_pn: measured 0.7 % slower on
    // cfg2's GC, profiles/r06/ab_gc_staged_cfg2.log)
    constexpr bool STG = PRUNE_STAGE && TAGS && MINW < 6;  // (the register-budget A/B forms: direct)
    __shared__ FieldRing<STG> rings[STG ? WPB : 1];
    FieldRing<STG> &ring = rings[(STG && WPB > 1) ? (threadIdx.x >> 6) : 0];
    constexpr bool STOK = STG && AGN_PRUNE_STAGE_TOK;
    __shared__ TokRing<STOK> trings[STOK ? WPB : 1];
    TokRing<STOK> &tring = trings[(STOK && WPB > 1) ? (threadIdx.x >> 6) : 0];
    // The key's metadata: one group of unconditional scalar loads (absent
    // columns from an in-bounds dummy) through the scalar cache (ldc) -- each
    // of these words is read by the key's own wave before that wave writes
    // it (in place) and written by no other wave.  As plain loads the GC
    // flag byte and the ListLen were vector loads under branches, each waited
    // for on its own: four round trips before the first row load issued.
    const uint64_t off = uniform_u64(ldc(a.key_off + k));
    const uint64_t lraw = uniform_u64(ldc(a.key_len ? a.key_len + k : a.key_off + k + 1));
    const uint8_t *gfp = a.key_list ? a.list_flags
                       : prune      ? prune
                                    : reinterpret_cast<const uint8_t *>(a.key_off);
    const uint32_t gfb = ldc_byte(gfp, a.key_list ? i : k);
    // the ETS ListLen, with the key's metadata: unconditional (a dummy word
    // when there is none), so it shares their round trip instead of costing
    // one of its own after the scan
    const uint32_t lc0 = __builtin_amdgcn_readfirstlane(
        ldc(a.key_lcap ? a.key_lcap + k : reinterpret_cast<const uint32_t *>(a.key_off + k)));
    const uint64_t n = a.key_len ? lraw : lraw - off;
    const bool gc = (a.key_list == nullptr && prune == nullptr) || gfb != 0u;
    const uint32_t tb = tags ? __builtin_amdgcn_readfirstlane(ldc(a.rem_off + off)) : 0u;
    const uint32_t lc_in = a.key_lcap ? lc0 : 0u;
    if (lane == 0 && a.d_key_off) a.d_key_off[k] = off;
    if (!gc && !a.copy_unselected) {
        if (lane == 0) {
            if (meta) {
                meta[i] = (uint32_t)n;
                meta[K + i] = tags ? a.rem_off[off + n] - tb : 0u;
                meta[2 * K + i] = lc_in;
                meta[3 * K + i] = a.key_id0 ? a.key_id0[k] : AGN_ID0_NONE;
                if (a.meta6) {
                    meta[4 * K + i] = (uint32_t)off;
                    meta[5 * K + i] = tb;
                }
            }
            if (flags) flags[k] = 0u;
        }
        return;
    }
    uint64_t t[DPL];
    const uint32_t tbits = chunk_bits<DPL, SPARSE>(thr_mask, k, W, d0, D);
#pragma unroll
    for (int j = 0; j < DPL; ++j) t[j] = ((tbits >> j) & 1u) ? thr[k * D + (uint32_t)(d0 + j)] : 0ull;
    const agn_log rl = [&] {
        agn_log l;
        l.oc = a.oc;
        l.oc_mask = a.mask;
        return l;
    }();
    // CTL: this lane's part of the threshold
    const uint32_t cp = 2u * (uint32_t)(lane % P);
    const uint64_t tA = CTL ? thr[k * D + cp] : 0ull, tB = CTL ? thr[k * D + cp + 1u] : 0ull;
    uint64_t written = 0;
    uint32_t rwritten = 0, first_id = AGN_ID0_NONE, last_id = 0;
    bool consec = true;
    // staged fields: ring head slot, pending entries, destination of the head
    uint32_t sh = 0, sp = 0;
    uint64_t sbase = off;
    // lanes < cnt store the ring's first cnt pending entries (lane = entry)
    auto flush = [&](uint32_t cnt) {
        if ((uint32_t)lane < cnt) {
            const uint32_t q = (sh + (uint32_t)lane) & (SRING - 1u);
            const uint64_t d = sbase + (uint64_t)lane;
            a.d_op_id[d] = ring.id[q];
            if (a.d_txid) a.d_txid[d] = ring.tx[q];
            if constexpr (TAGS) {
                a.d_tag[d] = ring.tg[q];
                a.d_add[d] = ring.w64[q];
                a.d_rem_off[d] = ring.ro[q];
            } else {
                a.d_eff[d] = (int64_t)ring.w64[q];
            }
        }
        sh = (sh + cnt) & (SRING - 1u);
        sp -= cnt;
        sbase += cnt;
    };
    // staged tokens: ring head slot, pending tokens, destination of the head
    uint32_t th = 0, tp = 0, tsbase = tb;
    auto tflush = [&](uint32_t cnt) {
        for (uint32_t c = 0; c < cnt; c += AGN_WAVE)
            if (c + (uint32_t)lane < cnt)
                a.d_tok[tsbase + c + (uint32_t)lane] = tring.t[(th + c + (uint32_t)lane) & (TRING - 1u)];
        th = (th + cnt) & (TRING - 1u);
        tp -= cnt;
        tsbase += cnt;
    };
    // PF: the next iteration's rows are requested once this iteration's
    // filter has decided, so they are in flight while its fields, removal
    // tokens and stores wait (the next rows are above every destination of
    // this iteration: in place, the early load reads them unchanged)
    uint64_t on[DPL];
    uint32_t onb = 0;
    auto load_slice = [&](uint64_t ee, uint64_t (&v)[DPL], uint32_t &bits) {
        if constexpr (FULL) {
            load_rows<DPL, SPARSE, FULL>(rl, ee, d0, D, W, v, bits);
        } else {
            bits = chunk_bits<DPL, SPARSE>(a.mask, ee, W, d0, D);
#pragma unroll
            for (int j = 0; j < DPL; ++j)
                v[j] = ((uint32_t)(d0 + j) < D) ? a.oc[ee * D + (uint32_t)(d0 + j)] : 0ull;
        }
    };
    if constexpr (PF != 0) {
        if (n) load_slice(off + ((uint64_t)slot < n ? (uint64_t)slot : 0ull), on, onb);
    }
    // EF (PF = 3, set/register): when an iteration keeps every entry, the
    // next one most likely does too (a GC threshold covers a prefix of the
    // key's commit-ordered ops), so its entries' fields are requested with
    // its rows instead of after its filter -- one round trip less per kept
    // iteration; a misprediction only reads the fields of dropped entries
    constexpr bool EF = PF == 3 && TAGS;
    bool nf = false;
    uint32_t nid = 0, ntg = 0, nr0 = 0, nr1 = 0;
    uint64_t ntx = 0, nad = 0;
    for (uint64_t b = 0; b < n; b += S::OPI) {
        const uint64_t pos = b + (uint64_t)slot;
        const bool valid = pos < n;
        const uint64_t e = off + (valid ? pos : 0ull);
        // the raw row (absent DCs included: a kept row moves bit for bit)
        uint64_t o[DPL];
        uint32_t obits = 0;
        u64x2 qx[NQ];
        if constexpr (PF != 0) {
#pragma unroll
            for (int j = 0; j < DPL; ++j) o[j] = on[j];
            obits = onb;
        } else if constexpr (CTL) {
            const u64x2 *rows = reinterpret_cast<const u64x2 *>(a.oc);
            const uint64_t lim = (off + n) * (uint64_t)P - 1u;  // the key's last part
#pragma unroll
            for (int j = 0; j < NQ; ++j) {
                uint64_t u = (off + b) * (uint64_t)P + (uint64_t)(j * AGN_WAVE + lane);
                u = u < lim ? u : lim;
                qx[j] = __builtin_nontemporal_load(rows + u);
            }
        } else if constexpr (FULL) {
            load_rows<DPL, SPARSE, FULL>(rl, e, d0, D, W, o, obits);
        } else {
            obits = chunk_bits<DPL, SPARSE>(a.mask, e, W, d0, D);
#pragma unroll
            for (int j = 0; j < DPL; ++j)
                o[j] = ((uint32_t)(d0 + j) < D) ? a.oc[e * D + (uint32_t)(d0 + j)] : 0ull;
        }
        if (!valid) obits = 0u;
        // the entry's fields are loaded with its row, before the filter decides
        // (one memory round trip per iteration instead of two; the fields of
        // dropped entries are read for nothing: 20 B each)
        uint32_t id = 0, tg = 0, r0 = 0, rl_ = 0;
        uint64_t tx = 0, ad = 0;
        int64_t ef = 0;
        auto load_fields = [&]() {
            id = a.op_id[e];
            tx = a.txid ? a.txid[e] : 0ull;
            if constexpr (TAGS) {
                tg = a.tag[e];
                ad = a.add[e];
                r0 = a.rem_off[e];
                rl_ = a.rem_off[e + 1] - r0;
            } else {
                ef = a.eff[e];
            }
        };
        const bool late = a.late_fields < 0 ? TAGS : a.late_fields != 0;
        bool have = false;  // EF: this iteration's fields came with its rows
        if constexpr (EF) {
            if (nf) {
                id = nid;
                tx = ntx;
                tg = ntg;
                ad = nad;
                r0 = nr0;
                rl_ = nr1 - nr0;
                have = true;
            }
        }
        if (!late && !have && valid && sub == 0) load_fields();
        bool le = true;
        if constexpr (CTL) {
            uint64_t gtm = 0;  // ops with a DC above the threshold
#pragma unroll
            for (int j = 0; j < NQ; ++j)
                gtm |= group_any<P>(ballot(qx[j].x > tA || qx[j].y > tB)) << (j * OPL);
            le = ((gtm >> slot) & 1ull) == 0ull;
        } else {
#pragma unroll
            for (int j = 0; j < DPL; ++j)
                if ((obits >> j) & 1u) le = le && (o[j] <= t[j]);
            if (LPO > 1) {
                const uint64_t grp = ((1ull << LPO) - 1ull) << (slot * LPO);
                le = (ballot(!le) & grp) == 0ull;
            }
        }
        const bool kp = valid && (!gc || !le);  // belongs_to_snapshot_op(Threshold, op)
        // set_aw / register_mv: 32 B of fields per entry, loaded for the kept
        // entries only once the filter has decided; counter_pn: 20 B, loaded
        // with the row (one round trip less; measured, scripts/ab_prune.py)
        if (late && !have && kp && sub == 0) load_fields();
        if constexpr (PF != 0) {
            const uint64_t pn = b + (uint64_t)S::OPI + (uint64_t)slot;
            const bool more = b + (uint64_t)S::OPI < n;
            if (more) load_slice(off + (pn < n ? pn : 0ull), on, onb);
            if constexpr (EF) {
                // the next iteration's fields read their source slots, above
                // every destination of this iteration (the one rem_off slot
                // it may rewrite there gets the same value)
                nf = more && ballot(valid && sub == 0 && !kp) == 0ull;
                if (nf && pn < n && sub == 0) {
                    const uint64_t en = off + pn;
                    nid = a.op_id[en];
                    ntx = a.txid ? a.txid[en] : 0ull;
                    ntg = a.tag[en];
                    nad = a.add[en];
                    nr0 = a.rem_off[en];
                    nr1 = a.rem_off[en + 1];
                }
            }
        }
        const uint64_t km = ballot(kp && sub == 0);  // one bit per kept op (its sub-0 lane)
        const uint32_t nk = (uint32_t)__builtin_popcountll(km);
        const uint32_t rank = (uint32_t)__builtin_popcountll(km & ((1ull << (slot * LPO)) - 1ull) &
                                                            ~0ull);
        const uint64_t dst = off + written + rank;
        // per-entry fields and removal lists: loads of the whole iteration first
        uint64_t tk[PT];
        const bool head = kp && sub == 0;
        if (!head) rl_ = 0;
        // token destinations: exclusive scan of the kept list lengths
        uint32_t tincl = 0;
        if (tags) {
            tincl = rl_;
#pragma unroll
            for (int x = 1; x < AGN_WAVE; x <<= 1) {
                const uint32_t v = (uint32_t)__shfl_up((int)tincl, x, AGN_WAVE);
                if (lane >= x) tincl += v;
            }
        }
        const uint32_t tdst = tb + rwritten + (tincl - rl_);
        const uint32_t T = tags ? (uint32_t)__builtin_amdgcn_readlane((int)tincl, 63) : 0u;
        const bool long_list = tags && ballot(head && rl_ > (uint32_t)PT) != 0ull;
        if (tags && !long_list && head) {
#pragma unroll
            for (int x = 0; x < PT; ++x) tk[x] = (uint32_t)x < rl_ ? a.tok[r0 + x] : 0ull;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // stores
        if constexpr (CTL) {
#pragma unroll
            for (int j = 0; j < NQ; ++j) {
                const int hq = (j * OPL + lane / P) * LPO;  // head lane of this part's op
                const uint64_t dq = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(dst >> 32), hq, AGN_WAVE) << 32) |
                                    (uint32_t)__shfl((int)(uint32_t)dst, hq, AGN_WAVE);
                if ((km >> hq) & 1ull)
                    reinterpret_cast<u64x2 *>(a.d_oc)[dq * (uint64_t)P + (uint64_t)(lane % P)] = qx[j];
            }
        } else if (kp) {
            if constexpr (FULL) {
                u64x2 *q = reinterpret_cast<u64x2 *>(a.d_oc + dst * D + (uint32_t)d0);
#pragma unroll
                for (int j = 0; j < DPL / 2; ++j) {
                    u64x2 x;
                    x.x = o[2 * j];
                    x.y = o[2 * j + 1];
                    q[j] = x;
                }
            } else {
#pragma unroll
                for (int j = 0; j < DPL; ++j)
                    if ((uint32_t)(d0 + j) < D) a.d_oc[dst * D + (uint32_t)(d0 + j)] = o[j];
            }
        }
        if (SPARSE && a.mask) {
            // mask words of the kept entries: lane sub < W of each kept op
            const uint64_t mw = (kp && (uint32_t)sub < W) ? a.mask[e * W + (uint32_t)sub] : 0ull;
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (kp && (uint32_t)sub < W) a.d_mask[dst * W + (uint32_t)sub] = mw;
        }
        if (STG) {
            if (head) {
                const uint32_t q = (sh + sp + rank) & (SRING - 1u);
                ring.id[q] = id;
                ring.tx[q] = tx;
                if constexpr (TAGS) {
                    ring.tg[q] = tg;
                    ring.w64[q] = ad;
                    ring.ro[q] = tdst;
                } else {
                    ring.w64[q] = (uint64_t)ef;
                }
            }
        } else if (head) {
            a.d_op_id[dst] = id;
            if (a.d_txid) a.d_txid[dst] = tx;
            if constexpr (TAGS) {
                a.d_tag[dst] = tg;
                a.d_add[dst] = ad;
            } else {
                a.d_eff[dst] = ef;
            }
        }
        if (STOK && long_list && tp) {
            tflush(tp);  // the other copies start right after the ring's range
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        if (tags) {
            if (!long_list) {
                if (STOK) {
                    if (head) {
#pragma unroll
                        for (int x = 0; x < PT; ++x)
                            if ((uint32_t)x < rl_)
                                tring.t[(th + (tdst - tsbase) + (uint32_t)x) & (TRING - 1u)] = tk[x];
                    }
                } else if (head) {
#pragma unroll
                    for (int x = 0; x < PT; ++x)
                        if ((uint32_t)x < rl_) a.d_tok[tdst + x] = tk[x];
                }
            } else {
                // position order, one kept entry at a time, 64 tokens per step
                uint64_t rest = km;
                while (rest) {
                    const int src_lane = __builtin_ctzll(rest);
                    rest &= rest - 1ull;
                    const uint32_t s0 = (uint32_t)__shfl((int)r0, src_lane, AGN_WAVE);
                    const uint32_t sl = (uint32_t)__shfl((int)rl_, src_lane, AGN_WAVE);
                    const uint32_t sd = (uint32_t)__shfl((int)tdst, src_lane, AGN_WAVE);
                    for (uint32_t c = 0; c < sl; c += AGN_WAVE) {
                        const bool in = c + (uint32_t)lane < sl;
                        const uint64_t v = in ? a.tok[s0 + c + (uint32_t)lane] : 0ull;
                        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        if (in) a.d_tok[sd + c + (uint32_t)lane] = v;
                        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                    }
                }
            }
            if (!STG && head) {
                a.d_rem_off[dst] = tdst;
                a.d_rem_off[dst + 1] = tdst + rl_;
            }
            rwritten += (uint32_t)__builtin_amdgcn_readlane((int)tincl, 63);
            if (STOK) {
                if (long_list) tsbase = tb + rwritten;  // copied directly
                else tp += T;
            }
        }
        // consecutive-id index over the kept ids, in position order
        if (nk) {
            const uint64_t prev_m = km & lt;
            const int pl = prev_m ? 63 - __builtin_clzll(prev_m) : lane;
            const uint32_t prev_id = (uint32_t)__shfl((int)id, pl, AGN_WAVE);
            const bool first_of_iter = head && prev_m == 0ull;
            bool ok = true;
            if (head) ok = first_of_iter ? (written == 0 || id == last_id + 1u) : (id == prev_id + 1u);
            consec = consec && (ballot(head && !ok) == 0ull);
            const int lo = __builtin_ctzll(km), hi = 63 - __builtin_clzll(km);
            if (written == 0) first_id = (uint32_t)__shfl((int)id, lo, AGN_WAVE);
            last_id = (uint32_t)__shfl((int)id, hi, AGN_WAVE);
        }
        written += nk;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (STOK) {
            while (tp >= 2u * (uint32_t)AGN_WAVE) {
                tflush(2u * (uint32_t)AGN_WAVE - ((tsbase + 2u * (uint32_t)AGN_WAVE) & 15u));
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
            }
        }
        if (STG) {
            sp += nk;
            // runs ending on a 32-entry boundary: 33..64 entries
            while (sp >= (uint32_t)AGN_WAVE) {
                flush((uint32_t)AGN_WAVE - (uint32_t)((sbase + (uint64_t)AGN_WAVE) & 31u));
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
    if (STOK) tflush(tp);
    if (STG) {
        flush(sp);
        // the token end of the last kept entry (each staged entry carried its start)
        if (tags && lane == 0) a.d_rem_off[off + written] = tb + rwritten;
    }
    if (lane == 0) {
        const uint32_t l = (uint32_t)written;
        const uint32_t id0 = (l && consec && first_id != AGN_ID0_NONE) ? first_id : AGN_ID0_NONE;
        uint32_t lc = lc_in;
        if (lc && gc) {
            lc = resize_list_len_dev(l ? l : 1u, lc);  // prune_ops' NewLength (1 if none kept)
            if (lc < l) lc = l;
        }
        a.d_key_len[k] = written;
        if (a.key_id0) a.key_id0[k] = id0;
        if (a.key_lcap) a.key_lcap[k] = lc;
        if (tags && l == 0 && !STG) a.d_rem_off[off] = tb;  // an empty segment keeps its token base
        if (meta) {
            meta[i] = l;
            meta[K + i] = rwritten;
            meta[2 * K + i] = lc;
            meta[3 * K + i] = id0;
            if (a.meta6) {  // the live range still starts at the segment start
                meta[4 * K + i] = (uint32_t)off;
                meta[5 * K + i] = tb;
            }
        }
        if (flags) flags[k] = (gc && l == 0) ? AGN_GC_ALL_PRUNED : 0u;
    }
}

// ---- in-place prune toward the END of the live range (the engine-owned log) --
// Ops are appended in commit order, so the ops a GC drops (covered by the
// stored snapshot) are, in the common case, a prefix of the key's log.
// Compacting the kept entries toward the END of the key's live range instead
// of its start leaves every kept entry with no dropped entry above it where it
// is: its row, fields and removal tokens are neither read (fields) nor
// written.  The live range then starts later in the key's segment: the kernel
// writes the new key_off, and meta rows 4/5 carry the new live range start
// (entry slot, token slot) to the host; an append that no longer fits behind
// the range moves the key to a fresh segment (oplog.hip).
// Walk: chunks from the newest down; a kept entry's destination is end - 1 -
// (kept entries above it), so no destination is below its source, every load
// of a chunk precedes its stores, and a chunk writes only above the next
// (lower) chunk's sources.  Removal tokens slide the same way (an entry that
// stays has no token that moves); the token end of a chunk's top entry is
// carried from the chunk above, whose stores may have rewritten that rem_off
// slot.  Consecutive-id index: with an index before the GC the kept ids are
// id0 + position, so it survives iff the kept positions are contiguous and no
// id is loaded; without one the kept entries' ids are loaded and checked.
//
// QUAD (dense D = 8, one op per lane): a chunk's 4 KiB of rows are read
// lane-contiguously, non-temporal -- load j covers bytes [1 KiB j, 1 KiB
// (j+1)), 8 whole lines per instruction, lane l holding DCs 2p, 2p+1 (p = l &
// 3) of op 16 j + (l >> 2), the counter kernel's quad rows (counter_scan.hpp)
// -- where the row-per-lane loads touch 32 lines per instruction, a quarter
// of each, and request every line four times.  belongs_to_snapshot_op's
// verdicts are nibbles of wave ballots folded on the scalar unit; a moving
// row is written back from the same registers (its parts' lanes fetch its
// destination).  On a prefix drop nothing moves and the GC is a read pass.
// MINW: waves per SIMD the register allocation must allow (1 = the
// compiler's choice; 8: the counter form fits 8 waves in 59 VGPRs / 78 SGPRs
// where the default allocation takes 104 SGPRs and 7 waves)
template <int DPL, int LPO, bool SPARSE, bool FULL, bool TAGS, int WPB = 1, int MINW = 1>
__global__ __launch_bounds__(64 * WPB, MINW) void k_prune_tail(InplaceArgs a,
                                                   const uint8_t *__restrict__ prune,
                                                   const uint64_t *__restrict__ thr,
                                                   const uint64_t *__restrict__ thr_mask,
                                                   uint32_t *__restrict__ meta,
                                                   uint32_t *__restrict__ flags) {
    using S = Shape<DPL, LPO>;
    constexpr int OPI = S::OPI;
    constexpr bool QUAD = FULL && DPL == 8 && LPO == 1 && !SPARSE;
    const uint32_t blk = block_order(a.xcd, blockIdx.x, gridDim.x);
    const uint64_t i = (uint64_t)blk * WPB + (WPB == 1 ? 0u : (threadIdx.x >> 6));
    if (i >= a.n_keys) return;
    const uint64_t K = a.n_keys;  // launch size (meta stride)
    const uint64_t k = a.key_list ? uniform_u64(a.key_list[i]) : i;
    const int lane = lane_id();
    const int sub = lane % LPO, slot = lane / LPO, d0 = sub * DPL;
    const int hl = slot * LPO;  // the lane holding this op's fields
    const uint32_t D = a.D, W = a.W;
    const uint64_t off = uniform_u64(a.key_off[k]);
    const uint64_t n = uniform_u64(key_n(a.key_off, a.key_len, k));
    const bool gc = a.key_list ? a.list_flags[i] != 0 : (prune == nullptr || prune[k] != 0);
    // token range [tb, te) of the key, read before any store
    const uint32_t tb = TAGS ? __builtin_amdgcn_readfirstlane(a.rem_off[off]) : 0u;
    const uint32_t te = TAGS ? __builtin_amdgcn_readfirstlane(a.rem_off[off + n]) : 0u;
    // the id index and the ETS ListLen, with the key's metadata:
    // unconditional (a dummy word when absent), so they share its round trip
    // instead of costing one of their own (ListLen: after the scan)
    const uint32_t *dummy = reinterpret_cast<const uint32_t *>(a.key_off + k);
    const uint32_t id0_raw = __builtin_amdgcn_readfirstlane(*(a.key_id0 ? a.key_id0 + k : dummy));
    const uint32_t lc0 = __builtin_amdgcn_readfirstlane(*(a.key_lcap ? a.key_lcap + k : dummy));
    const uint32_t id0_old = a.key_id0 ? id0_raw : AGN_ID0_NONE;
    const uint32_t lc_in = a.key_lcap ? lc0 : 0u;
    if (!gc) {
        if (lane == 0) {
            if (meta) {
                meta[i] = (uint32_t)n;
                meta[K + i] = te - tb;
                meta[2 * K + i] = lc_in;
                meta[3 * K + i] = id0_old;
                meta[4 * K + i] = (uint32_t)off;
                meta[5 * K + i] = tb;
            }
            if (flags) flags[k] = 0u;
        }
        return;
    }
    uint64_t t[DPL];
    const uint32_t tbits = chunk_bits<DPL, SPARSE>(thr_mask, k, W, d0, D);
#pragma unroll
    for (int j = 0; j < DPL; ++j) t[j] = ((tbits >> j) & 1u) ? thr[k * D + (uint32_t)(d0 + j)] : 0ull;
    const agn_log rl = [&] {
        agn_log l;
        l.oc = a.oc;
        l.oc_mask = a.mask;
        return l;
    }();
    const bool derive = id0_old != AGN_ID0_NONE;
    // QUAD: this lane's part of the threshold (DCs 2p, 2p+1)
    const int qp = lane & 3;
    const uint64_t tA = qp == 0 ? t[0] : qp == 1 ? t[2 % DPL] : qp == 2 ? t[4 % DPL] : t[6 % DPL];
    const uint64_t tB = qp == 0 ? t[1 % DPL] : qp == 1 ? t[3 % DPL] : qp == 2 ? t[5 % DPL] : t[7 % DPL];
    uint64_t written = 0;             // kept entries above the current chunk
    uint32_t twritten = 0;            // their tokens
    uint32_t rtop = te;               // token start of the entry just above the chunk
    uint32_t low_id = 0;              // id of the lowest kept entry so far (loaded ids)
    bool consec = true;
    int64_t lo_pos = -1, hi_pos = -1;  // lowest / highest kept position (derived ids)
    for (uint64_t c = (n + OPI - 1) / OPI; c-- > 0;) {
        const uint64_t b = c * (uint64_t)OPI;
        const uint64_t pos = b + (uint64_t)slot;
        const bool valid = pos < n;
        const uint64_t e = off + (valid ? pos : 0ull);
        uint64_t o[DPL];
        uint32_t obits = 0;
        u64x2 qx[4];
        uint64_t gtm = 0;  // QUAD: ops with a DC above the threshold
        if constexpr (QUAD) {
            const u64x2 *rows = reinterpret_cast<const u64x2 *>(a.oc);
            const uint64_t lim = (off + n) * 4u - 1u;  // the key's last part
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint64_t u = (off + b) * 4u + (uint64_t)(j * AGN_WAVE + lane);
                u = u < lim ? u : lim;
                qx[j] = __builtin_nontemporal_load(rows + u);
            }
        } else if constexpr (FULL) {
            load_rows<DPL, SPARSE, FULL>(rl, e, d0, D, W, o, obits);
        } else {
            obits = chunk_bits<DPL, SPARSE>(a.mask, e, W, d0, D);
#pragma unroll
            for (int j = 0; j < DPL; ++j)
                o[j] = ((uint32_t)(d0 + j) < D) ? a.oc[e * D + (uint32_t)(d0 + j)] : 0ull;
        }
        uint32_t r0 = 0;
        if constexpr (TAGS) r0 = (valid && sub == 0) ? a.rem_off[e] : 0u;
        bool kp;
        if constexpr (QUAD) {
            __builtin_amdgcn_sched_barrier(0);  // every load of the chunk in flight first
#pragma unroll
            for (int j = 0; j < 4; ++j)
                gtm |= nib_any16(ballot(qx[j].x > tA || qx[j].y > tB)) << (16 * j);
            kp = valid && ((gtm >> lane) & 1ull);  // belongs_to_snapshot_op(Threshold, op)
        } else {
            if (!valid) obits = 0u;
            bool le = true;
#pragma unroll
            for (int j = 0; j < DPL; ++j)
                if ((obits >> j) & 1u) le = le && (o[j] <= t[j]);
            if (LPO > 1) {
                const uint64_t grp = ((1ull << LPO) - 1ull) << hl;
                le = (ballot(!le) & grp) == 0ull;
            }
            kp = valid && !le;  // belongs_to_snapshot_op(Threshold, op)
        }
        const bool head = kp && sub == 0;
        const uint64_t km = ballot(head);  // one bit per kept op (its head lane)
        const uint32_t nk = (uint32_t)__builtin_popcountll(km);
        const uint64_t above = hl >= 63 ? 0ull : (km & (~0ull << (hl + 1)));
        const uint64_t dst = off + n - 1ull - written - (uint64_t)__builtin_popcountll(above);
        const bool mv = kp && dst != e;
        // removal lists: the entry's token end is the start of the entry
        // above it (the next op's head lane), or the carried start of the
        // chunk above for the chunk's top op (te for the key's newest)
        uint32_t rl_ = 0, suf = 0, tdst = 0;
        if constexpr (TAGS) {
            const int nx = hl + LPO;
            uint32_t r1 = (uint32_t)__shfl((int)r0, nx < AGN_WAVE ? nx : 0, AGN_WAVE);
            if (nx >= AGN_WAVE || pos + 1 >= n) r1 = rtop;
            rl_ = head ? r1 - r0 : 0u;
            suf = rl_;  // tokens of the kept entries at or above this lane
#pragma unroll
            for (int x = 1; x < AGN_WAVE; x <<= 1) {
                const uint32_t v = (uint32_t)__shfl_down((int)suf, x, AGN_WAVE);
                if (lane + x < AGN_WAVE) suf += v;
            }
            tdst = te - twritten - suf;
        }
        // fields: only the entries that move (and, without an id index, the
        // ids of every kept entry)
        uint32_t id = 0, tg = 0;
        uint64_t tx = 0, ad = 0;
        int64_t ef = 0;
        const bool mvh = mv && sub == 0;
        if (mvh) {
            id = a.op_id[e];
            tx = a.txid ? a.txid[e] : 0ull;
            if constexpr (TAGS) {
                tg = a.tag[e];
                ad = a.add[e];
            } else {
                ef = a.eff[e];
            }
        } else if (!derive && head) {
            id = a.op_id[e];
        }
        uint64_t tk[PT];
        const bool long_list = TAGS && ballot(mvh && rl_ > (uint32_t)PT) != 0ull;
        if (TAGS && !long_list && mvh) {
#pragma unroll
            for (int x = 0; x < PT; ++x) tk[x] = (uint32_t)x < rl_ ? a.tok[r0 + x] : 0ull;
        }
        const uint64_t mw = (SPARSE && a.mask && mv && (uint32_t)sub < W) ? a.mask[e * W + (uint32_t)sub] : 0ull;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // stores: the moving entries only
        if constexpr (QUAD) {
            const uint64_t mvm = ballot(mv);
            if (mvm) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int q = 16 * j + (lane >> 2);  // the op whose part this lane holds
                    const uint64_t dq = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(dst >> 32), q, AGN_WAVE) << 32) |
                                        (uint32_t)__shfl((int)(uint32_t)dst, q, AGN_WAVE);
                    if ((mvm >> q) & 1ull) reinterpret_cast<u64x2 *>(a.d_oc)[dq * 4u + (uint64_t)qp] = qx[j];
                }
            }
        } else if (mv) {
            if constexpr (FULL) {
                u64x2 *q = reinterpret_cast<u64x2 *>(a.d_oc + dst * D + (uint32_t)d0);
#pragma unroll
                for (int j = 0; j < DPL / 2; ++j) {
                    u64x2 x;
                    x.x = o[2 * j];
                    x.y = o[2 * j + 1];
                    q[j] = x;
                }
            } else {
#pragma unroll
                for (int j = 0; j < DPL; ++j)
                    if ((uint32_t)(d0 + j) < D) a.d_oc[dst * D + (uint32_t)(d0 + j)] = o[j];
            }
            if (SPARSE && a.mask && (uint32_t)sub < W) a.d_mask[dst * W + (uint32_t)sub] = mw;
        }
        if (mvh) {
            a.d_op_id[dst] = id;
            if (a.d_txid) a.d_txid[dst] = tx;
            if constexpr (TAGS) {
                a.d_tag[dst] = tg;
                a.d_add[dst] = ad;
            } else {
                a.d_eff[dst] = ef;
            }
        }
        if constexpr (TAGS) {
            if (!long_list) {
                if (mvh) {
#pragma unroll
                    for (int x = 0; x < PT; ++x)
                        if ((uint32_t)x < rl_) a.d_tok[tdst + x] = tk[x];
                }
            } else {
                // newest moving entry first, each list from its top 64 tokens
                // down: a destination is never below its source
                uint64_t rest = ballot(mvh);
                while (rest) {
                    const int src_lane = 63 - __builtin_clzll(rest);
                    rest &= ~(1ull << src_lane);
                    const uint32_t s0 = (uint32_t)__shfl((int)r0, src_lane, AGN_WAVE);
                    const uint32_t sl = (uint32_t)__shfl((int)rl_, src_lane, AGN_WAVE);
                    const uint32_t sd = (uint32_t)__shfl((int)tdst, src_lane, AGN_WAVE);
                    for (uint32_t cc = (sl + AGN_WAVE - 1) / AGN_WAVE; cc-- > 0;) {
                        const uint32_t j = cc * AGN_WAVE + (uint32_t)lane;
                        const bool in = j < sl;
                        const uint64_t v = in ? a.tok[s0 + j] : 0ull;
                        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        if (in) a.d_tok[sd + j] = v;
                        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                    }
                }
            }
            if (mvh) {
                a.d_rem_off[dst] = tdst;
                a.d_rem_off[dst + 1] = tdst + rl_;
            }
            twritten += (uint32_t)__builtin_amdgcn_readlane((int)suf, 0);
            rtop = (uint32_t)__builtin_amdgcn_readlane((int)r0, 0);
        }
        // consecutive-id index
        if (nk) {
            if (derive) {
                if (hi_pos < 0) hi_pos = (int64_t)b + (63 - __builtin_clzll(km)) / LPO;
                lo_pos = (int64_t)b + __builtin_ctzll(km) / LPO;
            } else {
                // each kept entry's successor (the next kept above it, or the
                // lowest kept entry of the chunks above) carries id + 1
                const int nl = above ? __builtin_ctzll(above) : 0;
                const uint32_t nid = (uint32_t)__shfl((int)id, nl, AGN_WAVE);
                bool ok = true;
                if (head) ok = above ? (nid == id + 1u) : (written == 0 || low_id == id + 1u);
                consec = consec && (ballot(head && !ok) == 0ull);
                low_id = (uint32_t)__shfl((int)id, __builtin_ctzll(km), AGN_WAVE);
            }
        }
        written += nk;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) {
        const uint32_t l = (uint32_t)written;
        uint32_t id0 = AGN_ID0_NONE;
        if (l) {
            if (derive) {
                if (hi_pos - lo_pos + 1 == (int64_t)l) id0 = id0_old + (uint32_t)lo_pos;
            } else if (consec && (uint64_t)low_id + (l - 1u) < (uint64_t)AGN_ID0_NONE) {
                id0 = low_id;
            }
        }
        uint32_t lc = lc_in;
        if (lc) {
            lc = resize_list_len_dev(l ? l : 1u, lc);  // prune_ops' NewLength (1 if none kept)
            if (lc < l) lc = l;
        }
        a.d_key_len[k] = written;
        a.d_key_off[k] = off + n - written;
        if (a.key_id0) a.key_id0[k] = id0;
        if (a.key_lcap) a.key_lcap[k] = lc;
        if (meta) {
            meta[i] = l;
            meta[K + i] = twritten;
            meta[2 * K + i] = lc;
            meta[3 * K + i] = id0;
            meta[4 * K + i] = (uint32_t)(off + n - written);
            meta[5 * K + i] = te - twritten;
        }
        if (flags) flags[k] = l == 0 ? AGN_GC_ALL_PRUNED : 0u;
    }
}

// k_prune_tail for counter_pn with dense 8-DC rows (the engine-owned log the
// bench and a steady counter partition have), KPW keys per wave: every key's
// metadata is requested in one round trip and every key's newest chunk of
// quad rows in the next, before the first key is walked -- KPW x 4 KiB in
// flight per wave slot where the one-key form has 4 KiB and a metadata round
// trip in which nothing streams.  Per key the walk, the moves and the
// records are k_prune_tail's (QUAD, !TAGS) exactly.
struct TailKey {
    uint64_t i, k, off, n;
    uint32_t id0_old, lc_in;
    bool live, gc;
    uint64_t tA, tB;
};

template <int KPW, int MINW>
__global__ __launch_bounds__(64, MINW) void k_prune_tail_q(InplaceArgs a,
                                                         const uint8_t *__restrict__ prune,
                                                         const uint64_t *__restrict__ thr,
                                                         uint32_t *__restrict__ meta,
                                                         uint32_t *__restrict__ flags) {
    const uint32_t blk = block_order(a.xcd, blockIdx.x, gridDim.x);
    const uint64_t K = a.n_keys;  // launch size (meta stride)
    const int lane = lane_id(), qp = lane & 3;
    TailKey s[KPW];
    // 1. every key's metadata (unconditional loads, dummies past the launch)
    uint64_t off_r[KPW], n_r[KPW];
    uint32_t id0_r[KPW], lc_r[KPW], pr_r[KPW];
    u64x2 t_r[KPW];
#pragma unroll
    for (int x = 0; x < KPW; ++x) {
        const uint64_t i = (uint64_t)blk * KPW + (uint64_t)x;
        s[x].i = i;
        s[x].live = i < K;
        const uint64_t ic = s[x].live ? i : 0ull;
        s[x].k = a.key_list ? uniform_u64(a.key_list[ic]) : ic;
        const uint64_t k = s[x].k;
        const uint32_t *dummy = reinterpret_cast<const uint32_t *>(a.key_off + k);
        off_r[x] = a.key_off[k];
        n_r[x] = a.key_len ? a.key_len[k] : a.key_off[k + 1];
        id0_r[x] = *(a.key_id0 ? a.key_id0 + k : dummy);
        lc_r[x] = *(a.key_lcap ? a.key_lcap + k : dummy);
        pr_r[x] = a.key_list ? a.list_flags[ic] : (prune ? prune[k] : 1u);
        t_r[x] = reinterpret_cast<const u64x2 *>(thr + k * 8u)[qp];
    }
    // 2. every key's newest chunk of rows
    u64x2 top[KPW][4];
#pragma unroll
    for (int x = 0; x < KPW; ++x) {
        const uint64_t off = uniform_u64(off_r[x]);
        const uint64_t nn = uniform_u64(n_r[x]);
        const uint64_t n = a.key_len ? nn : nn - off;
        s[x].off = off;
        s[x].n = n;
        s[x].gc = s[x].live && pr_r[x] != 0u;
        s[x].id0_old = a.key_id0 ? (uint32_t)__builtin_amdgcn_readfirstlane(id0_r[x]) : AGN_ID0_NONE;
        s[x].lc_in = a.key_lcap ? (uint32_t)__builtin_amdgcn_readfirstlane(lc_r[x]) : 0u;
        s[x].tA = t_r[x].x;
        s[x].tB = t_r[x].y;
        const uint64_t nc = (n + AGN_WAVE - 1) / AGN_WAVE;
        const uint64_t b = nc ? (nc - 1) * (uint64_t)AGN_WAVE : 0ull;
        // an empty key (possibly without a segment) reads its own key_off word
        const u64x2 *rows = reinterpret_cast<const u64x2 *>(n ? a.oc : a.key_off);
        const uint64_t lim = n ? (off + n) * 4u - 1u : 0ull;  // the key's last part
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint64_t u = (off + b) * 4u + (uint64_t)(j * AGN_WAVE + lane);
            u = (n && u < lim) ? u : lim;
            top[x][j] = __builtin_nontemporal_load(rows + u);
        }
    }
    // 3. each key in turn
#pragma unroll
    for (int x = 0; x < KPW; ++x) {
        if (!s[x].live) continue;
        const uint64_t i = s[x].i, k = s[x].k, off = s[x].off, n = s[x].n;
        if (!s[x].gc) {
            if (lane == 0) {
                if (meta) {
                    meta[i] = (uint32_t)n;
                    meta[K + i] = 0u;
                    meta[2 * K + i] = s[x].lc_in;
                    meta[3 * K + i] = s[x].id0_old;
                    meta[4 * K + i] = (uint32_t)off;
                    meta[5 * K + i] = 0u;
                }
                if (flags) flags[k] = 0u;
            }
            continue;
        }
        const bool derive = s[x].id0_old != AGN_ID0_NONE;
        const uint64_t tA = s[x].tA, tB = s[x].tB;
        uint64_t written = 0;
        uint32_t low_id = 0;
        bool consec = true;
        int64_t lo_pos = -1, hi_pos = -1;
        const uint64_t nc = (n + AGN_WAVE - 1) / AGN_WAVE;
        for (uint64_t c = nc; c-- > 0;) {
            const uint64_t b = c * (uint64_t)AGN_WAVE;
            const uint64_t pos = b + (uint64_t)lane;
            const bool valid = pos < n;
            const uint64_t e = off + (valid ? pos : 0ull);
            u64x2 qx[4];
            if (c == nc - 1) {
#pragma unroll
                for (int j = 0; j < 4; ++j) qx[j] = top[x][j];
            } else {
                const u64x2 *rows = reinterpret_cast<const u64x2 *>(a.oc);
                const uint64_t lim = (off + n) * 4u - 1u;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    uint64_t u = (off + b) * 4u + (uint64_t)(j * AGN_WAVE + lane);
                    u = u < lim ? u : lim;
                    qx[j] = __builtin_nontemporal_load(rows + u);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            uint64_t gtm = 0;  // ops with a DC above the threshold
#pragma unroll
            for (int j = 0; j < 4; ++j)
                gtm |= nib_any16(ballot(qx[j].x > tA || qx[j].y > tB)) << (16 * j);
            const bool kp = valid && ((gtm >> lane) & 1ull);  // belongs_to_snapshot_op(Threshold, op)
            const uint64_t km = ballot(kp);
            const uint32_t nk = (uint32_t)__builtin_popcountll(km);
            const uint64_t above = lane >= 63 ? 0ull : (km & (~0ull << (lane + 1)));
            const uint64_t dst = off + n - 1ull - written - (uint64_t)__builtin_popcountll(above);
            const bool mv = kp && dst != e;
            uint32_t id = 0;
            uint64_t tx = 0;
            int64_t ef = 0;
            if (mv) {
                id = a.op_id[e];
                tx = a.txid ? a.txid[e] : 0ull;
                ef = a.eff[e];
            } else if (!derive && kp) {
                id = a.op_id[e];
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const uint64_t mvm = ballot(mv);
            if (mvm) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int q = 16 * j + (lane >> 2);  // the op whose part this lane holds
                    const uint64_t dq = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(dst >> 32), q, AGN_WAVE) << 32) |
                                        (uint32_t)__shfl((int)(uint32_t)dst, q, AGN_WAVE);
                    if ((mvm >> q) & 1ull) reinterpret_cast<u64x2 *>(a.d_oc)[dq * 4u + (uint64_t)qp] = qx[j];
                }
            }
            if (mv) {
                a.d_op_id[dst] = id;
                if (a.d_txid) a.d_txid[dst] = tx;
                a.d_eff[dst] = ef;
            }
            if (nk) {
                if (derive) {
                    if (hi_pos < 0) hi_pos = (int64_t)b + (63 - __builtin_clzll(km));
                    lo_pos = (int64_t)b + __builtin_ctzll(km);
                } else {
                    const int nl = above ? __builtin_ctzll(above) : 0;
                    const uint32_t nid = (uint32_t)__shfl((int)id, nl, AGN_WAVE);
                    bool ok = true;
                    if (kp) ok = above ? (nid == id + 1u) : (written == 0 || low_id == id + 1u);
                    consec = consec && (ballot(kp && !ok) == 0ull);
                    low_id = (uint32_t)__shfl((int)id, __builtin_ctzll(km), AGN_WAVE);
                }
            }
            written += nk;
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        if (lane == 0) {
            const uint32_t l = (uint32_t)written;
            uint32_t id0 = AGN_ID0_NONE;
            if (l) {
                if (derive) {
                    if (hi_pos - lo_pos + 1 == (int64_t)l) id0 = s[x].id0_old + (uint32_t)lo_pos;
                } else if (consec && (uint64_t)low_id + (l - 1u) < (uint64_t)AGN_ID0_NONE) {
                    id0 = low_id;
                }
            }
            uint32_t lc = s[x].lc_in;
            if (lc) {
                lc = resize_list_len_dev(l ? l : 1u, lc);  // prune_ops' NewLength (1 if none kept)
                if (lc < l) lc = l;
            }
            a.d_key_len[k] = written;
            a.d_key_off[k] = off + n - written;
            if (a.key_id0) a.key_id0[k] = id0;
            if (a.key_lcap) a.key_lcap[k] = lc;
            if (meta) {
                meta[i] = l;
                meta[K + i] = 0u;
                meta[2 * K + i] = lc;
                meta[3 * K + i] = id0;
                meta[4 * K + i] = (uint32_t)(off + n - written);
                meta[5 * K + i] = 0u;
            }
            if (flags) flags[k] = l == 0 ? AGN_GC_ALL_PRUNED : 0u;
        }
    }
}

template <int DPL, int LPO, bool SPARSE>
int inplace_shape(const InplaceArgs &a, const uint8_t *prune, const uint64_t *thr,
                  const uint64_t *thr_mask, uint32_t *meta, uint32_t *flags, hipStream_t st) {
    // waves per block: 1 (default; the grid is the key list, as the counter
    // kernel) or 4 (AGN_PRUNE_WPB=4, A/B knob)
    const char *ev = AGN_KNOB("AGN_PRUNE_WPB");
    const bool w4 = ev && ev[0] == '4';
    const unsigned blocks = grid_for(a.n_keys, w4 ? 4 : 1, 0x7fffffffu);
    const bool full = !a.mask && (DPL % 2 == 0) && a.D == (uint32_t)(DPL * LPO);
    const bool tags = a.rem_off != nullptr;
    // the register budget of MINW waves per SIMD instead of the compiler's
    // choice: AGN_PRUNE_MINW=6|8 (A/B knob; the tail kernel: 8, counter only)
    const char *mw = AGN_KNOB("AGN_PRUNE_MINW");
    const bool mw6 = mw && mw[0] == '6', mw8 = mw && mw[0] == '8';
    if (a.d_key_off && a.meta6) {  // the engine-owned log: toward the end of the live range
        // waves per block: 1 (default) or 4 (AGN_PRUNE_WPB=4, A/B knob).  The
        // counter forms run with the register budget of 8 waves per SIMD
        // (prefix drop, 2M x 64: 2.43 vs 2.53 ms for the GC call, 4 waves
        // per block 2.93; profiles/r03/ab_prune_tail.log); AGN_PRUNE_TAIL_MINW=1
        // gives the compiler's allocation (7 waves)
        const char *tmw = AGN_KNOB("AGN_PRUNE_TAIL_MINW");
        const bool w8 = !(tmw && tmw[0] == '1');
        // counter_pn with dense 8-DC rows: KPW keys per wave, every key's
        // metadata and newest chunk in flight before the first is walked --
        // 2 by default (prefix drop, 2M x 64: 2.31 ms per GC call against
        // 2.43 for one key per wave at 8 waves per SIMD and 2.35 for 4 keys;
        // profiles/r03/ab_prune_tail_kpw.log); AGN_PRUNE_TAIL_KPW=1|2|4
        if constexpr (DPL == 8 && LPO == 1 && !SPARSE) {
            const char *kv = AGN_KNOB("AGN_PRUNE_TAIL_KPW");
            const int kpw = kv ? atoi(kv) : 2;
            if (full && !tags && !w4 && (kpw == 2 || kpw == 4)) {
                if (kpw == 2)
                    hipLaunchKernelGGL((k_prune_tail_q<2, 1>), dim3(grid_for(a.n_keys, 2, 0x7fffffffu)),
                                       dim3(64), 0, st, a, prune, thr, meta, flags);
                else
                    hipLaunchKernelGGL((k_prune_tail_q<4, 1>), dim3(grid_for(a.n_keys, 4, 0x7fffffffu)),
                                       dim3(64), 0, st, a, prune, thr, meta, flags);
                return hipGetLastError() == hipSuccess ? AGN_OK : fail(AGN_EHIP, "k_prune_tail_q launch");
            }
        }
#define AGN_T(FULLV, TAGSV)                                                                    \
    do {                                                                                       \
        if (w4)                                                                                \
            hipLaunchKernelGGL((k_prune_tail<DPL, LPO, SPARSE, FULLV, TAGSV, 4>),               \
                               dim3(grid_for(a.n_keys, 4, 0x7fffffffu)), dim3(256), 0, st, a,  \
                               prune, thr, thr_mask, meta, flags);                             \
        else if (w8 && !(TAGSV))                                                               \
            hipLaunchKernelGGL((k_prune_tail<DPL, LPO, SPARSE, FULLV, TAGSV, 1, 8>),            \
                               dim3(grid_for(a.n_keys, 1, 0x7fffffffu)), dim3(64), 0, st, a,   \
                               prune, thr, thr_mask, meta, flags);                             \
        else                                                                                   \
            hipLaunchKernelGGL((k_prune_tail<DPL, LPO, SPARSE, FULLV, TAGSV, 1>),               \
                               dim3(grid_for(a.n_keys, 1, 0x7fffffffu)), dim3(64), 0, st, a,   \
                               prune, thr, thr_mask, meta, flags);                             \
    } while (0)
        if (full) {
            if (tags) AGN_T((DPL % 2 == 0), true);
            else AGN_T((DPL % 2 == 0), false);
        } else {
            if (tags) AGN_T(false, true);
            else AGN_T(false, false);
        }
#undef AGN_T
        return hipGetLastError() == hipSuccess ? AGN_OK : fail(AGN_EHIP, "k_prune_tail launch");
    }
#define AGN_K(FULLV, TAGSV)                                                                    \
    do {                                                                                       \
        if (w4)                                                                                \
            hipLaunchKernelGGL((k_prune_inplace<DPL, LPO, SPARSE, FULLV, TAGSV, 4>),           \
                               dim3(blocks), dim3(256), 0, st, a, prune, thr, thr_mask, meta,  \
                               flags);                                                         \
        else if (mw6)                                                                          \
            hipLaunchKernelGGL((k_prune_inplace<DPL, LPO, SPARSE, FULLV, TAGSV, 1, false, 0, 6>), \
                               dim3(blocks), dim3(64), 0, st, a, prune, thr, thr_mask, meta,   \
                               flags);                                                         \
        else if (mw8)                                                                          \
            hipLaunchKernelGGL((k_prune_inplace<DPL, LPO, SPARSE, FULLV, TAGSV, 1, false, 0, 8>), \
                               dim3(blocks), dim3(64), 0, st, a, prune, thr, thr_mask, meta,   \
                               flags);                                                         \
        else                                                                                   \
            hipLaunchKernelGGL((k_prune_inplace<DPL, LPO, SPARSE, FULLV, TAGSV, 1>),           \
                               dim3(blocks), dim3(64), 0, st, a, prune, thr, thr_mask, meta,   \
                               flags);                                                         \
    } while (0)
    // contiguous rows (CTL) for dense 8-DC slices: the default for counter_pn
    // (cfg2: 15.37-15.70 vs 15.60-15.97 ms, three boxes), not for set/register
    // (cfg3: 13.79 vs 13.26; profiles/r03/*_abp{2,3}.log); AGN_PRUNE_CT=0|1
    // (A/B knob) overrides
    if constexpr (DPL == 8 && !SPARSE) {
        const char *cv = AGN_KNOB("AGN_PRUNE_CT");
        const bool ct = (cv && (cv[0] == '0' || cv[0] == '1')) ? cv[0] == '1' : !tags;
        if (full && ct && !w4) {
            if (tags)
                hipLaunchKernelGGL((k_prune_inplace<DPL, LPO, false, true, true, 1, true>),
                                   dim3(blocks), dim3(64), 0, st, a, prune, thr, thr_mask, meta,
                                   flags);
            else
                hipLaunchKernelGGL((k_prune_inplace<DPL, LPO, false, true, false, 1, true>),
                                   dim3(blocks), dim3(64), 0, st, a, prune, thr, thr_mask, meta,
                                   flags);
            return hipGetLastError() == hipSuccess ? AGN_OK : fail(AGN_EHIP, "k_prune_inplace launch");
        }
    }
    // next iteration's rows prefetched (PF) for keys that span iterations:
    // the default for set/register (cfg3: 13.13 vs 13.26 and 13.82 vs 13.97
    // ms on two boxes), AGN_PRUNE_PF=0|1|2|3 (A/B knob; 3: with the next
    // iteration's fields predicted (EF); 2: held to 5 waves per
    // SIMD, slower: 14.5)
    const char *pv = AGN_KNOB("AGN_PRUNE_PF");
    const int pf = w4 || mw6 || mw8 ? 0
                   : (pv && pv[0] >= '0' && pv[0] <= '3') ? pv[0] - '0'
                   : (tags ? 1 : 0);
    if (pf) {
#define AGN_P(FULLV, TAGSV)                                                                    \
    do {                                                                                       \
        if (pf == 3)                                                                           \
            hipLaunchKernelGGL((k_prune_inplace<DPL, LPO, SPARSE, FULLV, TAGSV, 1, false, 3>), \
                               dim3(blocks), dim3(64), 0, st, a, prune, thr, thr_mask, meta,   \
                               flags);                                                         \
        else if (pf == 2)                                                                      \
            hipLaunchKernelGGL((k_prune_inplace<DPL, LPO, SPARSE, FULLV, TAGSV, 1, false, 2>), \
                               dim3(blocks), dim3(64), 0, st, a, prune, thr, thr_mask, meta,   \
                               flags);                                                         \
        else                                                                                   \
            hipLaunchKernelGGL((k_prune_inplace<DPL, LPO, SPARSE, FULLV, TAGSV, 1, false, 1>), \
                               dim3(blocks), dim3(64), 0, st, a, prune, thr, thr_mask, meta,   \
                               flags);                                                         \
    } while (0)
        if (full) {
            if (tags) AGN_P((DPL % 2 == 0), true);
            else AGN_P((DPL % 2 == 0), false);
        } else {
            if (tags) AGN_P(false, true);
            else AGN_P(false, false);
        }
#undef AGN_P
        return hipGetLastError() == hipSuccess ? AGN_OK : fail(AGN_EHIP, "k_prune_inplace launch");
    }
    if (full) {
        if (tags) AGN_K((DPL % 2 == 0), true);
        else AGN_K((DPL % 2 == 0), false);
    } else {
        if (tags) AGN_K(false, true);
        else AGN_K(false, false);
    }
#undef AGN_K
    return hipGetLastError() == hipSuccess ? AGN_OK : fail(AGN_EHIP, "k_prune_inplace launch");
}

template <bool SPARSE>
int inplace(const InplaceArgs &a, const uint8_t *prune, const uint64_t *thr,
            const uint64_t *thr_mask, uint32_t *meta, uint32_t *flags, hipStream_t st) {
#define AGN_L(DPL, LPO) inplace_shape<DPL, LPO, SPARSE>(a, prune, thr, thr_mask, meta, flags, st)
    AGN_DISPATCH_SHAPES(a.D, AGN_L)
#undef AGN_L
}

InplaceArgs seg_args(const agn_log &in, const agn_log &out) {
    InplaceArgs a;
    a.oc = in.oc;
    a.mask = in.oc_mask;
    a.txid = in.txid;
    a.add = in.add_tok;
    a.tok = in.rem_tok;
    a.op_id = in.op_id;
    a.tag = in.tag;
    a.rem_off = in.rem_off;
    a.eff = in.eff;
    a.d_oc = (uint64_t *)out.oc;
    a.d_mask = (uint64_t *)out.oc_mask;
    a.d_txid = (uint64_t *)out.txid;
    a.d_add = (uint64_t *)out.add_tok;
    a.d_tok = (uint64_t *)out.rem_tok;
    a.d_op_id = (uint32_t *)out.op_id;
    a.d_tag = (uint32_t *)out.tag;
    a.d_rem_off = (uint32_t *)out.rem_off;
    a.d_eff = (int64_t *)out.eff;
    a.key_off = in.key_off;
    a.key_len = in.key_len;
    a.d_key_len = (uint64_t *)out.key_len;
    a.d_key_off = nullptr;
    a.key_id0 = (uint32_t *)out.key_id0;
    a.key_lcap = nullptr;
    a.n_keys = in.n_keys;
    a.D = in.n_dcs;
    a.W = n_words(in.n_dcs);
    a.copy_unselected = 0;
    a.key_list = nullptr;
    a.list_flags = nullptr;
    a.xcd = order_or(1u);
    const char *lf = AGN_KNOB("AGN_PRUNE_LATE_FIELDS");  // A/B override: 0 | 1
    a.late_fields = (lf && (lf[0] == '0' || lf[0] == '1')) ? lf[0] - '0' : -1;
    a.meta6 = 0;
    return a;
}

// The engine-owned log's prune: toward the end of the live range (k_prune_tail)
// unless AGN_PRUNE_TAIL=0 (A/B knob: the start-anchored k_prune_inplace).
void engine_log_mode(InplaceArgs &a, const agn_log &view) {
    const char *v = AGN_KNOB("AGN_PRUNE_TAIL");
    a.meta6 = 1;
    a.d_key_off = (v && v[0] == '0') ? nullptr : const_cast<uint64_t *>(view.key_off);
}

}  // namespace

int launch_prune_inplace(const agn_log &view, uint64_t *key_len, uint32_t *key_id0,
                         uint32_t *key_lcap, const uint8_t *prune, const uint64_t *thr,
                         const uint64_t *thr_mask, uint32_t *meta, uint32_t *flags,
                         hipStream_t st) {
    if (view.n_keys == 0) return AGN_OK;
    agn_log out = view;  // in place: the destination arrays are the source arrays
    out.key_len = key_len;
    out.key_id0 = key_id0;
    InplaceArgs a = seg_args(view, out);
    a.key_len = key_len;
    a.key_lcap = key_lcap;
    engine_log_mode(a, view);
    const bool sparse = view.oc_mask || thr_mask;
    return sparse ? inplace<true>(a, prune, thr, thr_mask, meta, flags, st)
                  : inplace<false>(a, prune, thr, thr_mask, meta, flags, st);
}

// prune_ops of a key list in place (the cached batcher's GC: the batch's keys,
// flags[i] from the snapshot-cache policy): n waves instead of one per key of
// the log; meta[6][n] per list entry (the engine-owned log's records).
int launch_prune_keys(const agn_log &view, uint64_t *key_len, uint32_t *key_id0,
                      uint32_t *key_lcap, uint64_t n, const uint64_t *keys, const uint8_t *flags,
                      const uint64_t *thr, const uint64_t *thr_mask, uint32_t *meta,
                      hipStream_t st) {
    if (n == 0) return AGN_OK;
    agn_log out = view;
    out.key_len = key_len;
    out.key_id0 = key_id0;
    InplaceArgs a = seg_args(view, out);
    a.key_len = key_len;
    a.key_lcap = key_lcap;
    a.n_keys = n;
    a.key_list = keys;
    a.list_flags = flags;
    a.xcd = 0;
    engine_log_mode(a, view);
    const bool sparse = view.oc_mask || thr_mask;
    return sparse ? inplace<true>(a, nullptr, thr, thr_mask, meta, nullptr, st)
                  : inplace<false>(a, nullptr, thr, thr_mask, meta, nullptr, st);
}

// {kept entries, kept removal tokens} of a segmented output: per-block sums
// into scratch, then one block folds them (no same-address atomics)
constexpr unsigned TOT_BLOCK = 1024;
__global__ __launch_bounds__(TOT_BLOCK) void k_seg_totals(const uint64_t *__restrict__ key_off,
                                                          const uint64_t *__restrict__ key_len,
                                                          const uint32_t *__restrict__ rem_off,
                                                          uint64_t n, uint64_t *__restrict__ part) {
    __shared__ uint64_t se[TOT_BLOCK / 64], st[TOT_BLOCK / 64];
    uint64_t e = 0, t = 0;
    for (uint64_t k = (uint64_t)blockIdx.x * TOT_BLOCK + threadIdx.x; k < n;
         k += (uint64_t)gridDim.x * TOT_BLOCK) {
        const uint64_t l = key_len[k];
        e += l;
        if (rem_off && l) t += rem_off[key_off[k] + l] - rem_off[key_off[k]];
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        e += shfl_xor_u64(e, m);
        t += shfl_xor_u64(t, m);
    }
    const int w = threadIdx.x >> 6;
    if (lane_id() == 0) {
        se[w] = e;
        st[w] = t;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t a = 0, b = 0;
        for (unsigned x = 0; x < TOT_BLOCK / 64; ++x) {
            a += se[x];
            b += st[x];
        }
        part[2 * blockIdx.x] = a;
        part[2 * blockIdx.x + 1] = b;
    }
}

__global__ __launch_bounds__(64) void k_seg_totals_fold(const uint64_t *__restrict__ part,
                                                         unsigned nb, uint64_t *__restrict__ out) {
    uint64_t a = 0, b = 0;
    for (unsigned x = threadIdx.x; x < nb; x += 64) {
        a += part[2 * x];
        b += part[2 * x + 1];
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        a += shfl_xor_u64(a, m);
        b += shfl_xor_u64(b, m);
    }
    if (threadIdx.x == 0) {
        out[0] = a;
        out[1] = b;
    }
}

int launch_seg_totals(const agn_log &out, uint64_t *totals, hipStream_t st) {
    if (out.n_keys == 0) {
        AGN_HIP(hipMemsetAsync(totals, 0, 2 * sizeof(uint64_t), st));
        return AGN_OK;
    }
    const unsigned nb = grid_for(out.n_keys, TOT_BLOCK, 2048);
    uint64_t *part = nullptr;
    AGN_HIP(pool_malloc(&part, (size_t)nb * 2 * sizeof(uint64_t), st));
    hipLaunchKernelGGL(k_seg_totals, dim3(nb), dim3(TOT_BLOCK), 0, st, out.key_off, out.key_len,
                       out.rem_off, out.n_keys, part);
    hipLaunchKernelGGL(k_seg_totals_fold, dim3(1), dim3(64), 0, st, part, nb, totals);
    const hipError_t e = hipGetLastError();
    (void)hipFreeAsync(part, st);
    AGN_HIP(e);
    return AGN_OK;
}

// agn_prune_ops into segmented output (out.key_len != NULL): one pass, every
// key at its input segment start; out.key_off receives the starts.
int launch_prune_segmented(const agn_log &log, const uint8_t *prune, const uint64_t *thr,
                           const uint64_t *thr_mask, const agn_log &out, uint32_t *flags,
                           hipStream_t st) {
    if (log.n_keys == 0) return AGN_OK;
    InplaceArgs a = seg_args(log, out);
    a.d_key_off = (uint64_t *)out.key_off;
    a.copy_unselected = 1;
    const bool sparse = log.oc_mask || thr_mask;
    return sparse ? inplace<true>(a, prune, thr, thr_mask, nullptr, flags, st)
                  : inplace<false>(a, prune, thr, thr_mask, nullptr, flags, st);
}

// Two-phase prune_ops into a fresh segmented arena (agn_oplog_prune): the
// mark pass gives per-key kept entry / token counts, the caller sizes the new
// segments from them (ETS resize policy), then the scatter pass copies the
// kept entries straight into their segments -- no CSR intermediate and no
// re-segmenting copy.  keep: [log.n_entries] bytes, cnt / rcnt: [n_keys].
int launch_prune_mark(const agn_log &log, const uint8_t *prune, const uint64_t *thr,
                      const uint64_t *thr_mask, uint8_t *keep, uint64_t *cnt, uint64_t *rcnt,
                      hipStream_t st) {
    if (log.n_keys == 0) return AGN_OK;
    const bool sparse = log.oc_mask || thr_mask;
    return sparse ? mark<true>(log, prune, thr, thr_mask, keep, cnt, rcnt, st)
                  : mark<false>(log, prune, thr, thr_mask, keep, cnt, rcnt, st);
}

// out.key_off[k] = the key's new segment start (~0: no segment), tstart[k] =
// its token segment start (tag logs); out.rem_off holds absolute token
// positions like the arena's.
int launch_prune_scatter_seg(const agn_log &log, const agn_log &out, const uint8_t *prune,
                             const uint8_t *keep, const uint64_t *tstart, uint32_t *flags,
                             hipStream_t st) {
    if (log.n_keys == 0) return AGN_OK;
    hipLaunchKernelGGL(k_prune_scatter, dim3(grid_for(log.n_keys, 4, 0x7fffffffu)), dim3(256), 0,
                       st, log, out, prune, keep, log.rem_off ? tstart : nullptr, flags, 1);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

}  // namespace agn
