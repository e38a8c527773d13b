// oplog.hip — the engine-owned per-partition op log (include/antidote_gpu.h,
// "engine-owned op log").  It keeps the materializer_vnode ETS ops cache
// (src/materializer_vnode.erl:284-286, 321-338, 621-647) resident in HBM so
// reads never re-upload a key's ops.
//
// Layout in HBM.  Entry arrays (oc rows, masks, op_id, txid, effect fields,
// rem_off) form one arena; key k owns the segment [start[k], start[k] +
// cap[k] + 1) of it — cap slots for its ops, oldest first (the ETS tuple's
// element FIRST_OP.. of ListLen slots), plus one rem_off slot for the end of
// its last token list.  A second arena holds removal tokens, key k owning
// [tstart[k], tstart[k] + tcap[k]).  The flushed view is an agn_log with
// key_off = segment starts and key_len = lengths, which every kernel reads.
//
// Writes.  agn_oplog_append is host-only: it assigns op ids (the per-key
// counter of ets:update_counter, :630) and stages the entries with their
// final slot (key, position).  A key whose segment fills gets a new one of
// twice the size at the arena's end (a "move", copied on the device at the
// next flush, before the staged entries land).  agn_oplog_flush packs
// everything into one pinned buffer, does one H2D copy and three kernels:
// move segments, scatter entries, update key_off/key_len.  The arenas grow by
// doubling with stream-ordered alloc/copy/free.
//
// GC.  agn_oplog_prune is one in-place kernel (gc.hip k_prune_tail): per
// selected key the VC filter and the compaction of the kept entries toward
// the END of the key's live range (kept entries with no dropped entry above
// them -- the common case, GC drops the oldest ops -- are not touched), the
// new key_off / key_len / key_id0 and the ETS ListLen after the resize policy
// (snapshot_insert_gc, :540-558), all on the device; the per-key records come
// back to the host asynchronously (one D2H into the pinned metadata block,
// with the log's totals reduced on the device) and are settled by the next
// host-side call.  A key's live entries are [lstart, lstart + len) of its
// segment [start, start + cap] (tokens [ltstart, ltstart + tlen) of theirs); a
// prune advances lstart, and an append that no longer fits behind the live
// range moves the key to a fresh segment.  Slots are u32 (arenas < 2^32).  The
// physical segments stay where they are; ListLen (`lcap`, what op_insert_gc's
// GC trigger and the resize policy see) is kept apart from the segment's
// physical capacity (`cap`).  When the arenas hold more than twice the slots
// the keys want (segments abandoned by growth moves, halved ListLens), the
// next prune first re-lays the arenas out (relayout: fresh arenas sized
// max(ListLen, length) per key, one copy kernel), allocating everything
// before it changes any state.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <new>
#include <shared_mutex>
#include <vector>

#include "serve.hpp"

namespace agn {
namespace {

struct Arena {  // entry arrays of one log (null when the type lacks them)
    uint64_t *oc = nullptr, *mask = nullptr, *txid = nullptr, *add = nullptr;
    uint32_t *op_id = nullptr, *tag = nullptr, *rem_off = nullptr;
    int64_t *eff = nullptr;
    uint64_t *tok = nullptr;  // token arena
};

struct Move {  // one segment copy: entries [src, src+len) -> dst, tokens likewise
    uint64_t src, dst, tsrc, tdst;
    uint32_t len, tlen;
};

// Copies one key's segment (entries, their rows and fields, the token list)
// and rebases rem_off onto the destination token segment.  One wave.
__device__ void copy_segment(const Arena &a, const Arena &b, uint32_t D, uint32_t W,
                             uint64_t src, uint64_t dst, uint32_t len, uint64_t tsrc,
                             uint64_t tdst, uint32_t tlen, int lane) {
    const bool same = (src == dst) && (a.oc == b.oc);
    if (!same) {
        const uint64_t nw = (uint64_t)len * D;
        for (uint64_t j = lane; j < nw; j += AGN_WAVE) b.oc[dst * D + j] = a.oc[src * D + j];
        if (a.mask) {
            const uint64_t nm = (uint64_t)len * W;
            for (uint64_t j = lane; j < nm; j += AGN_WAVE) b.mask[dst * W + j] = a.mask[src * W + j];
        }
        for (uint32_t j = lane; j < len; j += AGN_WAVE) {
            b.op_id[dst + j] = a.op_id[src + j];
            b.txid[dst + j] = a.txid[src + j];
            if (a.eff) b.eff[dst + j] = a.eff[src + j];
            if (a.tag) {
                b.tag[dst + j] = a.tag[src + j];
                b.add[dst + j] = a.add[src + j];
            }
        }
    }
    if (a.rem_off) {
        if (len == 0 && lane == 0) b.rem_off[dst] = (uint32_t)tdst;
        for (uint32_t j = lane; j < len + (len ? 1u : 0u); j += AGN_WAVE)
            b.rem_off[dst + j] = (uint32_t)(a.rem_off[src + j] - tsrc + tdst);
        if (!(tsrc == tdst && a.tok == b.tok))
            for (uint32_t j = lane; j < tlen; j += AGN_WAVE) b.tok[tdst + j] = a.tok[tsrc + j];
    }
}

// Pending segment moves of a flush.  Source and destination ranges never
// overlap: a destination is always fresh arena space.  Rebase-only moves
// (token segment moved, entry segment not) have src == dst.
__global__ void __launch_bounds__(256) k_move(Arena a, uint32_t D, uint32_t W,
                                              const Move *__restrict__ mv, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const Move m = mv[i];
    copy_segment(a, a, D, W, m.src, m.dst, m.len, m.tsrc, m.tdst, m.tlen, lane_id());
}

// Staged entries: fields and token lists, one thread per entry.
__global__ void __launch_bounds__(256) k_scatter(
    Arena a, uint32_t W, uint64_t n, const uint64_t *__restrict__ dst,
    const uint64_t *__restrict__ tdst, const uint32_t *__restrict__ tlen,
    const uint64_t *__restrict__ toff, const uint32_t *__restrict__ op_id,
    const uint64_t *__restrict__ txid, const int64_t *__restrict__ eff,
    const uint32_t *__restrict__ tag, const uint64_t *__restrict__ add,
    const uint64_t *__restrict__ mask, const uint64_t *__restrict__ tok) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t e = dst[i];
    a.op_id[e] = op_id[i];
    a.txid[e] = txid[i];
    if (a.eff) a.eff[e] = eff[i];
    if (a.tag) {
        a.tag[e] = tag[i];
        a.add[e] = add[i];
    }
    if (a.mask)
        for (uint32_t w = 0; w < W; ++w) a.mask[e * W + w] = mask[i * W + w];
    if (a.rem_off) {
        // The next entry of the key writes the same value into e + 1.
        const uint64_t t = tdst[i];
        const uint32_t l = tlen[i];
        a.rem_off[e] = (uint32_t)t;
        a.rem_off[e + 1] = (uint32_t)(t + l);
        const uint64_t s = toff[i];
        for (uint32_t j = 0; j < l; ++j) a.tok[t + j] = tok[s + j];
    }
}

// Staged oc rows: one thread per clock word, coalesced on the staging side.
__global__ void __launch_bounds__(256) k_scatter_rows(uint64_t *__restrict__ oc, uint32_t D,
                                                      uint64_t n, const uint64_t *__restrict__ dst,
                                                      const uint64_t *__restrict__ rows) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n * D) return;
    const uint64_t i = j / D;
    oc[dst[i] * D + (j - i * D)] = rows[j];
}

constexpr int KV = 6;  // k_keys record: key, start, len, id0, ListLen, DC set (key_mask)
__global__ void __launch_bounds__(256) k_keys(uint64_t *__restrict__ key_off,
                                              uint64_t *__restrict__ key_len,
                                              uint32_t *__restrict__ key_id0,
                                              uint32_t *__restrict__ key_lcap,
                                              uint64_t *__restrict__ key_mask, uint64_t n,
                                              const uint64_t *__restrict__ kv) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = kv[KV * i];
    key_off[k] = kv[KV * i + 1];
    key_len[k] = kv[KV * i + 2];
    key_id0[k] = (uint32_t)kv[KV * i + 3];
    key_lcap[k] = (uint32_t)kv[KV * i + 4];
    if (key_mask) key_mask[k] = kv[KV * i + 5];
}

// relayout: every key's segment from arena a into fresh arena b (one wave per key)
__global__ void __launch_bounds__(256) k_relayout(Arena a, Arena b, uint32_t D, uint32_t W,
                                                  const Move *__restrict__ mv, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const Move m = mv[i];
    copy_segment(a, b, D, W, m.src, m.dst, m.len, m.tsrc, m.tdst, m.tlen, lane_id());
}

// Totals of a whole-log prune's records [6][stride] on the device, so the
// host's settle is O(1): {entries, tokens, slots the keys want = sum over the
// keys with a segment (ListLen != 0) of max(ListLen, length) + 1}.  Per-block
// partials, then one folding block (no same-address atomics).
constexpr unsigned TOT_B = 1024;
__global__ __launch_bounds__(TOT_B) void k_oplog_totals(const uint32_t *__restrict__ meta,
                                                        uint64_t K, uint64_t stride,
                                                        uint64_t *__restrict__ part) {
    __shared__ uint64_t sh[3][TOT_B / 64];
    uint64_t e = 0, t = 0, w = 0;
    for (uint64_t k = (uint64_t)blockIdx.x * TOT_B + threadIdx.x; k < K;
         k += (uint64_t)gridDim.x * TOT_B) {
        const uint32_t l = meta[k], lc = meta[2 * stride + k];
        e += l;
        t += meta[stride + k];
        if (lc) w += (uint64_t)(lc > l ? lc : l) + 1u;
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        e += shfl_xor_u64(e, m);
        t += shfl_xor_u64(t, m);
        w += shfl_xor_u64(w, m);
    }
    const int wv = threadIdx.x >> 6;
    if (lane_id() == 0) {
        sh[0][wv] = e;
        sh[1][wv] = t;
        sh[2][wv] = w;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        uint64_t a = 0;
        for (unsigned x = 0; x < TOT_B / 64; ++x) a += sh[threadIdx.x][x];
        part[3 * blockIdx.x + threadIdx.x] = a;
    }
}

__global__ __launch_bounds__(64) void k_oplog_totals_fold(const uint64_t *__restrict__ part,
                                                          unsigned nb, uint64_t *__restrict__ out) {
    uint64_t v[3] = {0, 0, 0};
    for (unsigned x = threadIdx.x; x < nb; x += 64)
        for (int j = 0; j < 3; ++j) v[j] += part[3 * x + j];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1)
        for (int j = 0; j < 3; ++j) v[j] += shfl_xor_u64(v[j], m);
    if (threadIdx.x == 0)
        for (int j = 0; j < 3; ++j) out[j] = v[j];
}

template <class T>
hipError_t grow_array(T *&p, uint64_t old_n, uint64_t new_n, hipStream_t st) {
    if (!p && old_n) return hipErrorInvalidValue;
    T *q = nullptr;
    hipError_t e = pool_malloc((void **)&q, std::max<uint64_t>(new_n, 1) * sizeof(T), st);
    if (e != hipSuccess) return e;
    if (p && old_n) {
        e = hipMemcpyAsync(q, p, old_n * sizeof(T), hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return e;
    }
    if (p) e = hipFreeAsync(p, st);
    p = q;
    return e;
}

template <class T>
void free_async(T *&p, hipStream_t st) {
    if (p) (void)hipFreeAsync(p, st);
    p = nullptr;
}

inline uint64_t align8(uint64_t b) { return (b + 255) & ~255ull; }

}  // namespace
}  // namespace agn

using namespace agn;

struct agn_oplog {
    agn_ctx *ctx = nullptr;
    uint32_t crdt = 0, D = 0, W = 0, init_slots = AGN_OPS_THRESHOLD;
    bool sparse = false, tags = false;
    uint64_t K = 0;

    // Locking: `wmu` guards the host side (metadata + staging: append),
    // `rw` the device arenas -- shared by readers for the whole of their
    // kernel, exclusive for flush / prune, which move and free segments.
    // Order: wmu before rw.
    mutable std::mutex wmu;
    std::shared_mutex rw;

    // host metadata per key
    std::vector<uint64_t> start, tstart;     // physical segments
    std::vector<uint32_t> cap, tcap, counter;
    std::vector<uint32_t> s_cnt, s_tcnt;     // staged (not yet flushed) entries / tokens
    // sparse logs with D <= 64: the DC set every entry of the key carries, 0
    // when they differ (agn_log.key_mask; set by the first append to an empty
    // key, cleared by an entry with another set; a GC only removes entries,
    // so a shared set stays shared)
    std::vector<uint64_t> umask;
    // pinned [6][K]: length (staged included), token length, ListLen, key_id0,
    // live range start (entry slot, token slot); a prune's D2H lands here
    // directly (settled by the next host call), then [3] u64 totals
    // {entries, tokens, slots wanted} reduced on the device
    uint32_t *meta = nullptr;
    uint32_t *len = nullptr, *tlen = nullptr, *lcap = nullptr, *id0 = nullptr;
    uint32_t *lstart = nullptr, *ltstart = nullptr;
    uint64_t *tot = nullptr;
    std::vector<uint8_t> dirty;
    std::vector<uint64_t> dirty_keys;
    std::vector<int64_t> move_of;  // index into moves, -1 = none pending
    std::vector<Move> moves;
    uint64_t used = 0, tused = 0;  // arena high-water marks (slots)
    uint64_t live = 0, tlive = 0;  // slots of the current segments
    uint64_t n_entries = 0, n_tokens = 0;
    bool relayout_wanted = false;

    // device
    Arena a;
    uint64_t dcap = 0, tdcap = 0;  // allocated slots
    uint64_t *key_off = nullptr, *key_len = nullptr;
    uint32_t *key_id0 = nullptr;   // consecutive-id index, kept with key_off / key_len
    uint32_t *key_lcap = nullptr;  // ListLen (the in-place prune applies the resize policy)
    uint64_t *key_mask = nullptr;  // sparse, D <= 64: umask on the device (agn_log.key_mask)
    uint32_t *d_meta = nullptr;    // [6][K] prune output, copied into `meta`
    hipEvent_t up_done = nullptr, gc_done = nullptr;
    bool up_pending = false, gc_pending = false;
    // key-list prune (oplog_prune_keys): the keys, their [6][n] records
    // (device, and the pinned copy the settle scatters)
    std::vector<uint64_t> gc_list;
    uint32_t *d_lmeta = nullptr, *h_lmeta = nullptr;
    uint64_t lmeta_cap = 0, list_since_sum = 0;
    void *pinned = nullptr;
    size_t pinned_bytes = 0;

    // staging (host)
    std::vector<uint64_t> s_dst, s_tdst, s_toff, s_txid, s_add, s_oc, s_mask, s_tok;
    std::vector<uint32_t> s_tlen, s_opid, s_tag;
    std::vector<int64_t> s_eff;
    // staged entries are stored by key + position and resolved at flush
    std::vector<uint64_t> s_key;
    std::vector<uint32_t> s_pos, s_tpos;
};

namespace {

inline uint32_t dlen_of(const agn_oplog *L, uint64_t k) { return L->len[k] - L->s_cnt[k]; }
inline uint32_t dtlen_of(const agn_oplog *L, uint64_t k) { return L->tlen[k] - L->s_tcnt[k]; }

// The host side of a prune: wait for its kernel and metadata copy, then the
// totals and the relayout check (arenas holding more than twice the slots
// the keys want).
int settle(agn_oplog *L) {
    if (!L->gc_pending) return AGN_OK;
    L->gc_pending = false;
    AGN_HIP(hipEventSynchronize(L->gc_done));
    if (!L->gc_list.empty()) {
        // key-list prune: scatter the listed keys' records, totals by difference
        const uint64_t n = L->gc_list.size();
        const uint32_t *m = L->h_lmeta;
        for (uint64_t i = 0; i < n; ++i) {
            const uint64_t k = L->gc_list[i];
            L->n_entries = L->n_entries - L->len[k] + m[i];
            L->n_tokens = L->n_tokens - L->tlen[k] + m[n + i];
            L->len[k] = m[i];
            L->tlen[k] = m[n + i];
            L->lcap[k] = m[2 * n + i];
            L->id0[k] = m[3 * n + i];
            L->lstart[k] = m[4 * n + i];
            L->ltstart[k] = m[5 * n + i];
        }
        L->gc_list.clear();
        // the relayout check is O(K): once per K/4 listed keys
        L->list_since_sum += n;
        if (L->list_since_sum < L->K / 4 + 1) return AGN_OK;
        L->list_since_sum = 0;
        uint64_t ne = 0, nt = 0, want = 0;
        for (uint64_t k = 0; k < L->K; ++k) {
            ne += L->len[k];
            nt += L->tlen[k];
            if (L->cap[k]) want += (uint64_t)std::max(L->lcap[k], L->len[k]) + 1;
        }
        L->tot[0] = ne;
        L->tot[1] = nt;
        L->tot[2] = want;
    }
    // totals: summed above, or (a whole-log prune) reduced on the device with
    // the records (k_oplog_totals)
    const uint64_t want = L->tot[2], nt = L->tot[1];
    L->n_entries = L->tot[0];
    L->n_tokens = nt;
    L->relayout_wanted = L->used > 2 * want + 1024 || (L->tags && L->tused > 2 * nt + 1024 + 16 * L->K);
    return AGN_OK;
}

void oplog_new_segment(agn_oplog *L, uint64_t k, uint32_t need, uint32_t tneed) {
    // ListLen: the ETS tuple starts with init_slots (OPS_THRESHOLD) and
    // doubles while full (the engine grows instead of forcing the GC read)
    uint32_t lc = L->lcap[k] ? L->lcap[k] : L->init_slots;
    while (lc < need) lc *= 2;
    L->lcap[k] = lc;
    // A key the GC emptied restarts at its segment start (len counts staged
    // entries: none exist, on the device or staged); this append marks it
    // dirty, so the flush writes its key_off.
    if (L->len[k] == 0) {
        L->lstart[k] = (uint32_t)L->start[k];
        L->ltstart[k] = (uint32_t)L->tstart[k];
    }
    // Physical entry segment: a new one at the arena's end when the live
    // range [lstart, lstart + need) does not fit behind the segment start (a
    // prune's advance included); the live entries move to its start.
    if ((uint64_t)L->lstart[k] - L->start[k] + need > L->cap[k]) {
        const uint32_t c = std::max(lc, need);
        const uint64_t old = L->lstart[k];
        L->live += (uint64_t)c + 1 - (L->cap[k] ? (uint64_t)L->cap[k] + 1 : 0);
        L->start[k] = L->used;
        L->used += (uint64_t)c + 1;
        L->cap[k] = c;
        L->lstart[k] = (uint32_t)L->start[k];
        const uint32_t dl = dlen_of(L, k), dt = dtlen_of(L, k);
        if (dl || dt || L->move_of[k] >= 0) {
            if (L->move_of[k] < 0) {
                L->move_of[k] = (int64_t)L->moves.size();
                L->moves.push_back(Move{old, 0, L->ltstart[k], 0, dl, dt});
            }
        }
    }
    if (L->tags && (uint64_t)L->ltstart[k] - L->tstart[k] + tneed > L->tcap[k]) {
        uint32_t c = L->tcap[k] ? L->tcap[k] : 16u;
        while (c < tneed) c *= 2;
        const uint64_t old = L->ltstart[k];
        L->tlive += c - L->tcap[k];
        L->tstart[k] = L->tused;
        L->tused += c;
        L->tcap[k] = c;
        L->ltstart[k] = (uint32_t)L->tstart[k];
        const uint32_t dl = dlen_of(L, k), dt = dtlen_of(L, k);
        if (dl || dt || L->move_of[k] >= 0) {
            if (L->move_of[k] < 0) {
                L->move_of[k] = (int64_t)L->moves.size();
                L->moves.push_back(Move{L->lstart[k], 0, old, 0, dl, dt});
            }
        }
    }
}

int ensure_pinned(agn_oplog *L, size_t bytes) {
    if (L->up_pending) {
        AGN_HIP(hipEventSynchronize(L->up_done));
        L->up_pending = false;
    }
    if (bytes <= L->pinned_bytes) return AGN_OK;
    if (L->pinned) AGN_HIP(hipHostFree(L->pinned));
    L->pinned = nullptr;
    L->pinned_bytes = 0;
    size_t b = std::max<size_t>(bytes, 2 * L->pinned_bytes);
    AGN_HIP(hipHostMalloc(&L->pinned, b, hipHostMallocDefault));
    L->pinned_bytes = b;
    return AGN_OK;
}

int ensure_arena(agn_oplog *L, hipStream_t st) {
    if (L->used >= 0xffffffffull)  // slots are u32 (live starts, rem_off)
        return fail(AGN_ENOTSUP, "oplog: entry arena beyond 2^32 slots");
    if (L->used > L->dcap || !L->a.op_id) {
        uint64_t c = std::max<uint64_t>(L->used, 2 * L->dcap);
        Arena &a = L->a;
        AGN_HIP(grow_array(a.oc, L->dcap * L->D, c * L->D, st));
        if (L->sparse) AGN_HIP(grow_array(a.mask, L->dcap * L->W, c * L->W, st));
        AGN_HIP(grow_array(a.op_id, L->dcap, c, st));
        AGN_HIP(grow_array(a.txid, L->dcap, c, st));
        if (L->tags) {
            AGN_HIP(grow_array(a.tag, L->dcap, c, st));
            AGN_HIP(grow_array(a.add, L->dcap, c, st));
            AGN_HIP(grow_array(a.rem_off, L->dcap, c, st));
        } else {
            AGN_HIP(grow_array(a.eff, L->dcap, c, st));
        }
        L->dcap = c;
    }
    if (L->tags && (L->tused > L->tdcap || !L->a.tok)) {
        if (L->tused >= 0xffffffffull)
            return fail(AGN_ENOTSUP, "oplog: token arena beyond 2^32 slots");
        uint64_t c = std::min<uint64_t>(std::max<uint64_t>(L->tused, 2 * L->tdcap), 0xffffffffull);
        AGN_HIP(grow_array(L->a.tok, L->tdcap, c, st));
        L->tdcap = c;
    }
    return AGN_OK;
}

void fill_view(const agn_oplog *L, agn_log *v) {
    std::memset(v, 0, sizeof *v);
    v->crdt_type = L->crdt;
    v->n_dcs = L->D;
    v->n_keys = L->K;
    v->n_entries = L->used;
    v->key_off = L->key_off;
    v->key_len = L->key_len;
    v->oc = L->a.oc;
    v->oc_mask = L->a.mask;
    v->op_id = L->a.op_id;
    v->txid = L->a.txid;
    v->eff = L->a.eff;
    v->tag = L->a.tag;
    v->add_tok = L->a.add;
    v->rem_off = L->a.rem_off;
    v->rem_tok = L->a.tok;
    v->key_id0 = L->key_id0;
    v->key_mask = L->key_mask;
}

int do_flush(agn_oplog *L, hipStream_t st) {
    const uint64_t n = L->s_key.size(), nm = L->moves.size(), nk = L->dirty_keys.size();
    int rc = ensure_arena(L, st);
    if (rc) return rc;
    if (n == 0 && nm == 0 && nk == 0) return AGN_OK;
    const uint32_t D = L->D, W = L->W;
    // Resolve staged (key, position) to arena slots now that segments are final.
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t k = L->s_key[i];
        L->s_dst[i] = (uint64_t)L->lstart[k] + L->s_pos[i];
        L->s_tdst[i] = (uint64_t)L->ltstart[k] + L->s_tpos[i];
    }
    for (uint64_t k : L->dirty_keys)
        if (L->move_of[k] >= 0) {
            Move &m = L->moves[L->move_of[k]];
            m.dst = L->lstart[k];
            m.tdst = L->ltstart[k];
        }
    // Pack: moves | dst | tdst | toff | txid | add | tlen | opid | tag | eff | oc | mask | tok | keys
    size_t off = 0;
    auto slot = [&](size_t bytes) { size_t o = off; off = align8(off + bytes); return o; };
    const size_t o_mv = slot(nm * sizeof(Move)), o_dst = slot(n * 8), o_tdst = slot(n * 8),
                 o_toff = slot(n * 8), o_txid = slot(n * 8), o_add = slot(L->tags ? n * 8 : 0),
                 o_tlen = slot(n * 4), o_opid = slot(n * 4), o_tag = slot(L->tags ? n * 4 : 0),
                 o_eff = slot(L->tags ? 0 : n * 8), o_oc = slot(n * D * 8),
                 o_mask = slot(L->sparse ? n * W * 8 : 0), o_tok = slot(L->s_tok.size() * 8),
                 o_keys = slot(nk * KV * 8);
    rc = ensure_pinned(L, off);
    if (rc) return rc;
    char *h = (char *)L->pinned;
    auto put = [&](size_t o, const void *src, size_t bytes) { if (bytes) std::memcpy(h + o, src, bytes); };
    put(o_mv, L->moves.data(), nm * sizeof(Move));
    put(o_dst, L->s_dst.data(), n * 8);
    put(o_tdst, L->s_tdst.data(), n * 8);
    put(o_toff, L->s_toff.data(), n * 8);
    put(o_txid, L->s_txid.data(), n * 8);
    if (L->tags) {
        put(o_add, L->s_add.data(), n * 8);
        put(o_tag, L->s_tag.data(), n * 4);
    } else {
        put(o_eff, L->s_eff.data(), n * 8);
    }
    put(o_tlen, L->s_tlen.data(), n * 4);
    put(o_opid, L->s_opid.data(), n * 4);
    put(o_oc, L->s_oc.data(), n * D * 8);
    if (L->sparse) put(o_mask, L->s_mask.data(), n * W * 8);
    put(o_tok, L->s_tok.data(), L->s_tok.size() * 8);
    {
        uint64_t *kv = (uint64_t *)(h + o_keys);
        for (uint64_t j = 0; j < nk; ++j) {
            const uint64_t k = L->dirty_keys[j];
            kv[KV * j] = k;
            kv[KV * j + 1] = L->lstart[k];
            kv[KV * j + 2] = L->len[k];
            kv[KV * j + 3] = L->len[k] ? L->id0[k] : AGN_ID0_NONE;
            kv[KV * j + 4] = L->lcap[k];
            kv[KV * j + 5] = L->umask.empty() ? 0ull : L->umask[k];
        }
    }
    char *d = nullptr;
    AGN_HIP(pool_malloc((void **)&d, off, st));
    AGN_HIP(hipMemcpyAsync(d, h, off, hipMemcpyHostToDevice, st));
    AGN_HIP(hipEventRecord(L->up_done, st));
    L->up_pending = true;
    if (nm)
        k_move<<<(unsigned)((nm + 3) / 4), 256, 0, st>>>(L->a, D, W, (const Move *)(d + o_mv), nm);
    if (n) {
        k_scatter<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(
            L->a, W, n, (const uint64_t *)(d + o_dst), (const uint64_t *)(d + o_tdst),
            (const uint32_t *)(d + o_tlen), (const uint64_t *)(d + o_toff),
            (const uint32_t *)(d + o_opid), (const uint64_t *)(d + o_txid),
            (const int64_t *)(d + o_eff), (const uint32_t *)(d + o_tag),
            (const uint64_t *)(d + o_add), (const uint64_t *)(d + o_mask),
            (const uint64_t *)(d + o_tok));
        k_scatter_rows<<<(unsigned)((n * D + 255) / 256), 256, 0, st>>>(
            L->a.oc, D, n, (const uint64_t *)(d + o_dst), (const uint64_t *)(d + o_oc));
    }
    if (nk)
        k_keys<<<(unsigned)((nk + 255) / 256), 256, 0, st>>>(L->key_off, L->key_len, L->key_id0,
                                                              L->key_lcap, L->key_mask, nk,
                                                              (const uint64_t *)(d + o_keys));
    AGN_HIP(hipGetLastError());
    AGN_HIP(hipFreeAsync(d, st));
    for (uint64_t k : L->dirty_keys) {
        L->s_cnt[k] = 0;
        L->s_tcnt[k] = 0;
        L->dirty[k] = 0;
        L->move_of[k] = -1;
    }
    L->dirty_keys.clear();
    L->moves.clear();
    for (auto *v : {&L->s_dst, &L->s_tdst, &L->s_toff, &L->s_txid, &L->s_add, &L->s_oc, &L->s_mask,
                    &L->s_tok, &L->s_key})
        v->clear();
    for (auto *v : {&L->s_tlen, &L->s_opid, &L->s_tag, &L->s_pos, &L->s_tpos}) v->clear();
    L->s_eff.clear();
    return AGN_OK;
}

// Fresh arenas sized max(ListLen, length) + 1 per key (token segments
// max(16, token length)) and one copy kernel.  Every allocation happens
// before any state changes: on failure the log is left exactly as it was
// (the caller treats relayout as an optimisation).  Requires a flushed,
// settled log.
int relayout(agn_oplog *L, hipStream_t st) {
    const uint64_t K = L->K;
    std::vector<uint64_t> ns(K), nts(K);
    std::vector<uint32_t> nc(K), ntc(K);
    std::vector<Move> mv;
    uint64_t used = 0, tused = 0;
    for (uint64_t k = 0; k < K; ++k) {
        nc[k] = L->cap[k] ? std::max(L->lcap[k], L->len[k]) : 0u;
        if (nc[k] == 0 && L->cap[k]) nc[k] = 1;
        ntc[k] = L->tags && L->tcap[k] ? std::max<uint32_t>(16u, L->tlen[k]) : 0u;
        ns[k] = nc[k] ? used : 0;
        nts[k] = tused;
        if (nc[k]) used += (uint64_t)nc[k] + 1;
        tused += ntc[k];
        if (L->cap[k] || L->tcap[k])
            mv.push_back(Move{L->lstart[k], ns[k], L->ltstart[k], nts[k], L->len[k], L->tlen[k]});
    }
    const uint64_t U = std::max<uint64_t>(used, 1), TU = std::max<uint64_t>(tused, 1);
    Arena b;
    Move *d_mv = nullptr;
    uint64_t *d_kv = nullptr;
    hipError_t e = pool_malloc(&b.oc, U * L->D * 8, st);
    if (e == hipSuccess && L->sparse) e = pool_malloc(&b.mask, U * L->W * 8, st);
    if (e == hipSuccess) e = pool_malloc(&b.op_id, U * 4, st);
    if (e == hipSuccess) e = pool_malloc(&b.txid, U * 8, st);
    if (e == hipSuccess && !L->tags) e = pool_malloc(&b.eff, U * 8, st);
    if (e == hipSuccess && L->tags) e = pool_malloc(&b.tag, U * 4, st);
    if (e == hipSuccess && L->tags) e = pool_malloc(&b.add, U * 8, st);
    if (e == hipSuccess && L->tags) e = pool_malloc(&b.rem_off, U * 4, st);
    if (e == hipSuccess && L->tags) e = pool_malloc(&b.tok, TU * 8, st);
    if (e == hipSuccess) e = pool_malloc(&d_mv, std::max<size_t>(mv.size(), 1) * sizeof(Move), st);
    if (e == hipSuccess) e = pool_malloc(&d_kv, std::max<uint64_t>(K, 1) * KV * 8, st);
    int rc = AGN_OK;
    if (e == hipSuccess) rc = ensure_pinned(L, mv.size() * sizeof(Move) + K * KV * 8);
    auto drop = [&]() {
        for (void *p : {(void *)b.oc, (void *)b.mask, (void *)b.op_id, (void *)b.txid,
                        (void *)b.eff, (void *)b.tag, (void *)b.add, (void *)b.rem_off,
                        (void *)b.tok, (void *)d_mv, (void *)d_kv})
            if (p) (void)hipFreeAsync(p, st);
    };
    if (e != hipSuccess || rc != AGN_OK) {
        drop();
        return fail(AGN_ENOMEM, "oplog relayout: %s", e != hipSuccess ? hipGetErrorString(e) : "staging");
    }
    char *h = (char *)L->pinned;
    std::memcpy(h, mv.data(), mv.size() * sizeof(Move));
    uint64_t *kv = (uint64_t *)(h + mv.size() * sizeof(Move));
    for (uint64_t k = 0; k < K; ++k) {
        kv[KV * k] = k;
        kv[KV * k + 1] = ns[k];
        kv[KV * k + 2] = L->len[k];
        kv[KV * k + 3] = L->len[k] ? L->id0[k] : AGN_ID0_NONE;
        kv[KV * k + 4] = L->lcap[k];
        kv[KV * k + 5] = L->umask.empty() ? 0ull : L->umask[k];
    }
    e = hipMemcpyAsync(d_mv, h, mv.size() * sizeof(Move), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(d_kv, kv, K * KV * 8, hipMemcpyHostToDevice, st);
    if (e == hipSuccess && !mv.empty())
        k_relayout<<<(unsigned)((mv.size() + 3) / 4), 256, 0, st>>>(L->a, b, L->D, L->W, d_mv,
                                                                    mv.size());
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) {
        drop();
        return fail(AGN_EHIP, "oplog relayout: %s", hipGetErrorString(e));
    }
    // commit: the new key_off (the copy above read the old arena first)
    if (K)
        k_keys<<<(unsigned)((K + 255) / 256), 256, 0, st>>>(L->key_off, L->key_len, L->key_id0,
                                                             L->key_lcap, L->key_mask, K, d_kv);
    (void)hipEventRecord(L->up_done, st);
    L->up_pending = true;
    (void)hipFreeAsync(d_mv, st);
    (void)hipFreeAsync(d_kv, st);
    Arena &a = L->a;
    for (void *p : {(void *)a.oc, (void *)a.mask, (void *)a.txid, (void *)a.add, (void *)a.op_id,
                    (void *)a.tag, (void *)a.rem_off, (void *)a.eff, (void *)a.tok})
        if (p) (void)hipFreeAsync(p, st);
    L->a = b;
    L->dcap = U;
    L->tdcap = L->tags ? TU : 0;
    L->used = L->live = used;
    L->tused = L->tlive = tused;
    L->start.swap(ns);
    L->tstart.swap(nts);
    for (uint64_t k = 0; k < K; ++k) {
        L->lstart[k] = (uint32_t)L->start[k];
        L->ltstart[k] = (uint32_t)L->tstart[k];
    }
    L->cap.swap(nc);
    L->tcap.swap(ntc);
    L->relayout_wanted = false;
    return AGN_OK;
}

}  // namespace

extern "C" {

int agn_oplog_create(agn_ctx *ctx, uint32_t crdt_type, uint32_t n_dcs, uint64_t n_keys,
                     int sparse, uint32_t init_slots, agn_oplog **out) {
    if (!out) return fail(AGN_EINVAL, "oplog_create: null out");
    *out = nullptr;
    if (n_dcs == 0 || n_dcs > 256) return fail(AGN_EINVAL, "oplog_create: n_dcs=%u", n_dcs);
    if (crdt_type != AGN_COUNTER_PN && crdt_type != AGN_SET_AW && crdt_type != AGN_REGISTER_MV)
        return fail(AGN_EINVAL, "oplog_create: crdt_type %u", crdt_type);
    if (init_slots > (1u << 30)) return fail(AGN_EINVAL, "oplog_create: init_slots %u", init_slots);
    int rc = use_device(ctx);
    if (rc) return rc;
    agn_oplog *L = new (std::nothrow) agn_oplog;
    if (!L) return fail(AGN_ENOMEM, "oplog_create");
    L->ctx = ctx;
    L->crdt = crdt_type;
    L->D = n_dcs;
    L->W = n_words(n_dcs);
    L->sparse = sparse != 0;
    L->tags = crdt_type != AGN_COUNTER_PN;
    L->init_slots = init_slots ? init_slots : AGN_OPS_THRESHOLD;
    L->K = n_keys;
    try {
        L->start.assign(n_keys, 0);
        L->tstart.assign(n_keys, 0);
        for (auto *v : {&L->cap, &L->tcap, &L->counter, &L->s_cnt, &L->s_tcnt}) v->assign(n_keys, 0);
        L->dirty.assign(n_keys, 0);
        L->move_of.assign(n_keys, -1);
        if (L->sparse && n_dcs <= 64) L->umask.assign(n_keys, 0);
    } catch (...) {
        delete L;
        return fail(AGN_ENOMEM, "oplog_create: host metadata for %llu keys",
                    (unsigned long long)n_keys);
    }
    const uint64_t K1 = std::max<uint64_t>(n_keys, 1);
    // [6][K] u32 rows, then 3 u64 totals (8-byte aligned: K1 * 6 * 4 is)
    hipError_t e = hipHostMalloc((void **)&L->meta, 6 * K1 * 4 + 3 * 8, hipHostMallocDefault);
    if (e == hipSuccess) {
        L->len = L->meta;
        L->tlen = L->meta + K1;
        L->lcap = L->meta + 2 * K1;
        L->id0 = L->meta + 3 * K1;
        L->lstart = L->meta + 4 * K1;
        L->ltstart = L->meta + 5 * K1;
        L->tot = reinterpret_cast<uint64_t *>(L->meta + 6 * K1);
        std::memset(L->meta, 0, 6 * K1 * 4 + 3 * 8);
        for (uint64_t k = 0; k < K1; ++k) L->id0[k] = AGN_ID0_NONE;
    }
    if (e == hipSuccess) e = hipMalloc((void **)&L->key_off, K1 * 8);
    if (e == hipSuccess) e = hipMalloc((void **)&L->key_len, K1 * 8);
    if (e == hipSuccess) e = hipMemset(L->key_off, 0, K1 * 8);
    if (e == hipSuccess) e = hipMemset(L->key_len, 0, K1 * 8);
    if (e == hipSuccess) e = hipMalloc((void **)&L->key_id0, K1 * 4);
    if (e == hipSuccess) e = hipMemset(L->key_id0, 0xff, K1 * 4);
    if (e == hipSuccess) e = hipMalloc((void **)&L->key_lcap, K1 * 4);
    if (e == hipSuccess) e = hipMemset(L->key_lcap, 0, K1 * 4);
    if (e == hipSuccess && !L->umask.empty()) e = hipMalloc((void **)&L->key_mask, K1 * 8);
    if (e == hipSuccess && L->key_mask) e = hipMemset(L->key_mask, 0, K1 * 8);
    if (e == hipSuccess) e = hipMalloc((void **)&L->d_meta, 6 * K1 * 4 + 3 * 8);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&L->up_done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&L->gc_done, hipEventDisableTiming);
    if (e != hipSuccess) {
        agn_oplog_destroy(L);
        return fail(AGN_ENOMEM, "oplog_create: device key arrays");
    }
    *out = L;
    return AGN_OK;
}

int agn_oplog_destroy(agn_oplog *L) {
    if (!L) return AGN_OK;
    if (L->ctx) use_device(L->ctx);
    (void)hipDeviceSynchronize();
    Arena &a = L->a;
    for (void *p : {(void *)a.oc, (void *)a.mask, (void *)a.txid, (void *)a.add, (void *)a.op_id,
                    (void *)a.tag, (void *)a.rem_off, (void *)a.eff, (void *)a.tok,
                    (void *)L->key_off, (void *)L->key_len, (void *)L->key_id0,
                    (void *)L->key_lcap, (void *)L->key_mask, (void *)L->d_meta,
                    (void *)L->d_lmeta})
        if (p) (void)hipFree(p);
    if (L->pinned) (void)hipHostFree(L->pinned);
    if (L->meta) (void)hipHostFree(L->meta);
    if (L->h_lmeta) (void)hipHostFree(L->h_lmeta);
    if (L->up_done) (void)hipEventDestroy(L->up_done);
    if (L->gc_done) (void)hipEventDestroy(L->gc_done);
    delete L;
    return AGN_OK;
}

static int oplog_append_locked(agn_oplog *L, uint64_t n, const uint64_t *keys,
                               const uint8_t *same_op, const uint64_t *oc,
                               const uint64_t *oc_mask, const uint64_t *txid, const int64_t *eff,
                               const uint32_t *tag, const uint64_t *add_tok,
                               const uint32_t *rem_off, const uint64_t *rem_tok,
                               uint32_t *out_op_id, uint8_t *out_gc_due);

int agn_oplog_append(agn_oplog *L, uint64_t n, const uint64_t *keys, const uint8_t *same_op,
                     const uint64_t *oc, const uint64_t *oc_mask, const uint64_t *txid,
                     const int64_t *eff, const uint32_t *tag, const uint64_t *add_tok,
                     const uint32_t *rem_off, const uint64_t *rem_tok, uint32_t *out_op_id,
                     uint8_t *out_gc_due) {
    if (!L) return fail(AGN_EINVAL, "oplog_append: null oplog");
    if (n == 0) return AGN_OK;
    std::lock_guard<std::mutex> g(L->wmu);
    int rc = settle(L);
    if (rc) return rc;
    try {
        return oplog_append_locked(L, n, keys, same_op, oc, oc_mask, txid, eff, tag, add_tok,
                                   rem_off, rem_tok, out_op_id, out_gc_due);
    } catch (const std::bad_alloc &) {
        return fail(AGN_ENOMEM, "oplog_append: host staging");
    }
}

static int oplog_append_locked(agn_oplog *L, uint64_t n, const uint64_t *keys,
                               const uint8_t *same_op, const uint64_t *oc,
                               const uint64_t *oc_mask, const uint64_t *txid, const int64_t *eff,
                               const uint32_t *tag, const uint64_t *add_tok,
                               const uint32_t *rem_off, const uint64_t *rem_tok,
                               uint32_t *out_op_id, uint8_t *out_gc_due) {
    if (!keys || !oc) return fail(AGN_EINVAL, "oplog_append: keys / oc required");
    if (L->sparse && !oc_mask) return fail(AGN_EINVAL, "oplog_append: sparse log needs oc_mask");
    if (L->tags ? (!tag || !add_tok || !rem_off || (rem_off[n] > rem_off[0] && !rem_tok)) : !eff)
        return fail(AGN_EINVAL, "oplog_append: effect arrays missing for type %u", L->crdt);
    // Validate the whole batch before touching any state (all or nothing).
    for (uint64_t i = 0; i < n; ++i) {
        if (keys[i] >= L->K)
            return fail(AGN_EINVAL, "oplog_append: key %llu >= n_keys", (unsigned long long)keys[i]);
        if (same_op && same_op[i] && (i == 0 || keys[i - 1] != keys[i]))
            return fail(AGN_EINVAL, "oplog_append: same_op[%llu] without a preceding entry of its key",
                        (unsigned long long)i);
        if (L->tags && rem_off[i + 1] < rem_off[i])
            return fail(AGN_EINVAL, "oplog_append: rem_off not monotone at %llu",
                        (unsigned long long)i);
    }
    const uint32_t D = L->D, W = L->W;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t k = keys[i];
        if (!(same_op && same_op[i])) ++L->counter[k];
        const uint32_t id = L->counter[k];
        if (out_op_id) out_op_id[i] = id;
        if (out_gc_due)
            out_gc_due[i] = !(same_op && same_op[i]) &&
                            (L->len[k] >= std::max(L->lcap[k], L->init_slots) ||
                             id % AGN_OPS_THRESHOLD == 0);
        const uint32_t tl = L->tags ? rem_off[i + 1] - rem_off[i] : 0u;
        oplog_new_segment(L, k, L->len[k] + 1, L->tlen[k] + tl);
        L->s_key.push_back(k);
        L->s_pos.push_back(L->len[k]);
        L->s_tpos.push_back(L->tlen[k]);
        L->s_opid.push_back(id);
        L->s_txid.push_back(txid ? txid[i] : 0ull);
        L->s_oc.insert(L->s_oc.end(), oc + i * D, oc + (i + 1) * D);
        if (L->sparse) L->s_mask.insert(L->s_mask.end(), oc_mask + i * W, oc_mask + (i + 1) * W);
        if (L->tags) {
            L->s_tag.push_back(tag[i]);
            L->s_add.push_back(add_tok[i]);
            L->s_toff.push_back(L->s_tok.size());
            L->s_tok.insert(L->s_tok.end(), rem_tok + rem_off[i], rem_tok + rem_off[i + 1]);
        } else {
            L->s_eff.push_back(eff[i]);
            L->s_toff.push_back(0);
        }
        L->s_tlen.push_back(tl);
        L->s_dst.push_back(0);
        L->s_tdst.push_back(0);
        // consecutive ids (op_id[p] == id0 + p) survive appends until a
        // same_op entry or a gap; AGN_ID0_NONE itself is never an id base
        const uint32_t p = L->len[k];
        if (!L->umask.empty()) {
            const uint64_t m = oc_mask[i * W] & low_bits(D);
            L->umask[k] = (p == 0) ? m : (L->umask[k] == m ? m : 0ull);
        }
        if (p == 0) L->id0[k] = id;
        else if (L->id0[k] != AGN_ID0_NONE && (uint64_t)id != (uint64_t)L->id0[k] + p)
            L->id0[k] = AGN_ID0_NONE;
        if (id == AGN_ID0_NONE) L->id0[k] = AGN_ID0_NONE;
        ++L->len[k];
        ++L->s_cnt[k];
        L->tlen[k] += tl;
        L->s_tcnt[k] += tl;
        if (!L->dirty[k]) {
            L->dirty[k] = 1;
            L->dirty_keys.push_back(k);
        }
    }
    L->n_entries += n;
    if (L->tags) L->n_tokens += rem_off[n] - rem_off[0];
    return AGN_OK;
}

int agn_oplog_flush(agn_oplog *L, agn_log *view, void *stream) {
    if (!L) return fail(AGN_EINVAL, "oplog_flush: null oplog");
    int rc = use_device(L->ctx);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(L->wmu);
    std::unique_lock<std::shared_mutex> x(L->rw);
    rc = settle(L);
    if (rc) return rc;
    try {
        rc = do_flush(L, (hipStream_t)stream);
    } catch (const std::bad_alloc &) {
        rc = fail(AGN_ENOMEM, "oplog_flush: host staging");
    }
    if (rc) return rc;
    // Readers on other streams must see the scattered entries.
    AGN_HIP(hipStreamSynchronize((hipStream_t)stream));
    if (view) fill_view(L, view);
    return AGN_OK;
}

int agn_oplog_prune(agn_oplog *L, const uint8_t *prune, const uint64_t *threshold,
                    const uint64_t *threshold_mask, uint32_t *out_flags, void *stream) {
    if (!L) return fail(AGN_EINVAL, "oplog_prune: null oplog");
    if (!threshold) return fail(AGN_EINVAL, "oplog_prune: threshold required");
    if (L->sparse && !threshold_mask) return fail(AGN_EINVAL, "oplog_prune: sparse log needs threshold_mask");
    if (misaligned4(prune)) return fail(AGN_EINVAL, "oplog_prune: prune must be 4-byte aligned");
    int rc = use_device(L->ctx);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(L->wmu);
    std::unique_lock<std::shared_mutex> x(L->rw);
    hipStream_t st = (hipStream_t)stream;
    rc = settle(L);
    if (rc) return rc;
    try {
        rc = do_flush(L, st);
        if (rc == AGN_OK && L->relayout_wanted) {
            // an optimisation: on failure the log stays as it is (fragmented)
            const int r2 = relayout(L, st);
            (void)r2;
        }
    } catch (const std::bad_alloc &) {
        rc = fail(AGN_ENOMEM, "oplog_prune: host staging");
    }
    if (rc) return rc;
    if (L->K == 0) return AGN_OK;
    if (L->used > 0xffffffffull) return fail(AGN_ENOTSUP, "oplog_prune: arena beyond 2^32 slots");
    agn_log view;
    fill_view(L, &view);
    rc = launch_prune_inplace(view, L->key_len, L->key_id0, L->key_lcap, prune, threshold,
                              threshold_mask, L->d_meta, out_flags, st);
    if (rc) return rc;
    // the log's totals, then the host's copy of {len, token len, ListLen,
    // id0, live start, token live start} + totals (counter logs: without the
    // token rows), settled by the next call
    const uint64_t K1 = std::max<uint64_t>(L->K, 1);
    {
        const unsigned nb = (unsigned)std::min<uint64_t>((L->K + TOT_B - 1) / TOT_B, 2048);
        uint64_t *part = nullptr;
        AGN_HIP(pool_malloc((void **)&part, (size_t)nb * 3 * 8, st));
        k_oplog_totals<<<nb, TOT_B, 0, st>>>(L->d_meta, L->K, K1, part);
        k_oplog_totals_fold<<<1, 64, 0, st>>>(part, nb, reinterpret_cast<uint64_t *>(L->d_meta + 6 * K1));
        const hipError_t e = hipGetLastError();
        (void)hipFreeAsync(part, st);
        AGN_HIP(e);
    }
    if (L->tags) {
        AGN_HIP(hipMemcpyAsync(L->meta, L->d_meta, 6 * K1 * 4 + 3 * 8, hipMemcpyDeviceToHost, st));
    } else {
        AGN_HIP(hipMemcpyAsync(L->meta, L->d_meta, K1 * 4, hipMemcpyDeviceToHost, st));
        AGN_HIP(hipMemcpyAsync(L->meta + 2 * K1, L->d_meta + 2 * K1, 4 * K1 * 4 + 3 * 8,
                               hipMemcpyDeviceToHost, st));
    }
    AGN_HIP(hipEventRecord(L->gc_done, st));
    L->gc_pending = true;
    return AGN_OK;
}

int agn_oplog_read(agn_oplog *L, const agn_read *req, agn_result *out, void *stream) {
    if (!L) return fail(AGN_EINVAL, "oplog_read: null oplog");
    hipStream_t st = (hipStream_t)stream;
    std::shared_lock<std::shared_mutex> hold;
    int rc = oplog_begin_read(L, st, 0, nullptr, nullptr, hold);
    if (rc) return rc;
    agn_log view;
    fill_view(L, &view);
    rc = agn_materialize(L->ctx, &view, req, out, stream);
    if (rc) return rc;
    AGN_HIP(hipStreamSynchronize(st));
    return AGN_OK;
}

int agn_oplog_stats(const agn_oplog *Lc, uint64_t *entries, uint64_t *slots, uint64_t *tokens) {
    if (!Lc) return fail(AGN_EINVAL, "oplog_stats: null oplog");
    agn_oplog *L = const_cast<agn_oplog *>(Lc);
    std::lock_guard<std::mutex> g(L->wmu);
    int rc = settle(L);
    if (rc) return rc;
    if (entries) *entries = L->n_entries;
    if (slots) *slots = L->used;
    if (tokens) *tokens = L->n_tokens;
    return AGN_OK;
}

int agn_oplog_set_counter(agn_oplog *L, uint64_t n, const uint64_t *keys, const uint32_t *counter) {
    if (!L) return fail(AGN_EINVAL, "oplog_set_counter: null oplog");
    if (n && (!keys || !counter)) return fail(AGN_EINVAL, "oplog_set_counter: null argument");
    std::lock_guard<std::mutex> g(L->wmu);
    for (uint64_t i = 0; i < n; ++i)
        if (keys[i] >= L->K)
            return fail(AGN_EINVAL, "oplog_set_counter: key %llu >= n_keys", (unsigned long long)keys[i]);
    for (uint64_t i = 0; i < n; ++i) L->counter[keys[i]] = counter[i];
    return AGN_OK;
}

int agn_oplog_key_meta(agn_oplog *L, uint64_t n, const uint64_t *keys, uint32_t *out_len,
                       uint32_t *out_list_len, uint32_t *out_counter) {
    if (!L) return fail(AGN_EINVAL, "oplog_key_meta: null oplog");
    if (n && !keys) return fail(AGN_EINVAL, "oplog_key_meta: null keys");
    std::lock_guard<std::mutex> g(L->wmu);
    int rc = settle(L);
    if (rc) return rc;
    for (uint64_t i = 0; i < n; ++i)
        if (keys[i] >= L->K)
            return fail(AGN_EINVAL, "oplog_key_meta: key %llu >= n_keys", (unsigned long long)keys[i]);
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t k = keys[i];
        if (out_len) out_len[i] = L->len[k];
        if (out_list_len) out_list_len[i] = L->lcap[k];
        if (out_counter) out_counter[i] = L->counter[k];
    }
    return AGN_OK;
}

int agn_oplog_gc_due(agn_oplog *L, uint64_t n, const uint64_t *keys, uint8_t *out_due) {
    if (!L) return fail(AGN_EINVAL, "oplog_gc_due: null oplog");
    if (n && (!keys || !out_due)) return fail(AGN_EINVAL, "oplog_gc_due: null argument");
    std::lock_guard<std::mutex> g(L->wmu);
    int rc = settle(L);
    if (rc) return rc;
    for (uint64_t i = 0; i < n; ++i)
        if (keys[i] >= L->K)
            return fail(AGN_EINVAL, "oplog_gc_due: key %llu >= n_keys", (unsigned long long)keys[i]);
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t k = keys[i];
        out_due[i] = L->len[k] >= std::max(L->lcap[k], L->init_slots) ||
                     (L->counter[k] + 1u) % AGN_OPS_THRESHOLD == 0;
    }
    return AGN_OK;
}

}  // extern "C"

namespace agn {
// Start of a read over the resident log: flushes staged appends
// (read-your-writes: update/2 is a sync_command that precedes the read),
// then, still under the writer lock, takes the arena shared in `hold` and
// writes each requested key's length into lens[n] -- so the lengths are
// exactly those of the device log the read's kernel will see (a concurrent
// append only stages on the host; its flush waits for `hold`).
// How many of keys[0..n) hold entries with different DC sets (umask 0, not
// empty): the read batcher's AGN_HINT_MIXED decision, from the host's copy
// of agn_log.key_mask -- no device read.  Caller holds L->wmu.
static uint64_t mixed_keys_locked(const agn_oplog *L, uint64_t n, const uint64_t *keys) {
    if (!L->sparse || L->umask.empty()) return 0;
    uint64_t m = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t k = keys[i];
        m += k < L->K && L->umask[k] == 0 && L->len[k] != 0;
    }
    return m;
}

int oplog_begin_read(agn_oplog *L, hipStream_t st, uint64_t n, const uint64_t *keys,
                     uint32_t *lens, std::shared_lock<std::shared_mutex> &hold,
                     uint64_t nm, const uint64_t *mixed_keys, uint64_t *mixed) {
    int rc = use_device(L->ctx);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(L->wmu);
    rc = settle(L);  // a prune's kernel precedes every later read
    if (rc) return rc;
    if (!L->s_key.empty() || !L->moves.empty() || !L->dirty_keys.empty()) {
        std::unique_lock<std::shared_mutex> x(L->rw);
        try {
            rc = do_flush(L, st);
        } catch (const std::bad_alloc &) {
            rc = fail(AGN_ENOMEM, "oplog read: host staging");
        }
        if (rc) return rc;
        AGN_HIP(hipStreamSynchronize(st));
    }
    if (mixed) *mixed = mixed_keys_locked(L, nm, mixed_keys);
    hold = std::shared_lock<std::shared_mutex>(L->rw);
    for (uint64_t i = 0; i < n; ++i) lens[i] = dlen_of(L, keys[i]);
    return AGN_OK;
}
void oplog_view(const agn_oplog *L, agn_log *v) { fill_view(L, v); }

int oplog_prune_keys(agn_oplog *L, uint64_t n, const uint64_t *h_keys, const uint64_t *d_keys,
                     const uint8_t *d_flags, const uint64_t *thr, const uint64_t *thr_mask,
                     hipStream_t st) {
    if (n == 0) return AGN_OK;
    if (L->sparse && !thr_mask) return fail(AGN_EINVAL, "oplog_prune_keys: sparse log needs threshold_mask");
    int rc = use_device(L->ctx);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(L->wmu);
    std::unique_lock<std::shared_mutex> x(L->rw);
    rc = settle(L);
    if (rc) return rc;
    try {
        rc = do_flush(L, st);
        if (rc == AGN_OK && L->relayout_wanted) (void)relayout(L, st);  // best effort
        if (rc == AGN_OK) L->gc_list.reserve(n);
    } catch (const std::bad_alloc &) {
        rc = fail(AGN_ENOMEM, "oplog_prune_keys: host staging");
    }
    if (rc) return rc;
    if (L->used > 0xffffffffull) return fail(AGN_ENOTSUP, "oplog_prune_keys: arena beyond 2^32 slots");
    if (n > L->lmeta_cap) {
        const uint64_t c = std::max<uint64_t>(n, 2 * L->lmeta_cap);
        if (L->d_lmeta) AGN_HIP(hipFree(L->d_lmeta));
        if (L->h_lmeta) AGN_HIP(hipHostFree(L->h_lmeta));
        L->d_lmeta = L->h_lmeta = nullptr;
        L->lmeta_cap = 0;
        AGN_HIP(hipMalloc((void **)&L->d_lmeta, 6 * c * 4));
        AGN_HIP(hipHostMalloc((void **)&L->h_lmeta, 6 * c * 4, hipHostMallocDefault));
        L->lmeta_cap = c;
    }
    agn_log view;
    fill_view(L, &view);
    rc = launch_prune_keys(view, L->key_len, L->key_id0, L->key_lcap, n, d_keys, d_flags, thr,
                           thr_mask, L->d_lmeta, st);
    if (rc) return rc;
    AGN_HIP(hipMemcpyAsync(L->h_lmeta, L->d_lmeta, 6 * n * 4, hipMemcpyDeviceToHost, st));
    AGN_HIP(hipEventRecord(L->gc_done, st));
    L->gc_list.assign(h_keys, h_keys + n);
    L->gc_pending = true;
    return AGN_OK;
}
void oplog_shape(const agn_oplog *L, uint32_t *crdt, uint32_t *D, int *sparse, uint64_t *K) {
    *crdt = L->crdt;
    *D = L->D;
    *sparse = L->sparse;
    *K = L->K;
}
agn_ctx *oplog_ctx(const agn_oplog *L) { return L->ctx; }
}  // namespace agn
