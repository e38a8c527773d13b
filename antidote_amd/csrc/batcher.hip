// batcher.hip — micro-batching read queue over an agn_oplog
// (include/antidote_gpu.h, "micro-batching read queue").
//
// The reference serves reads per key: each of up to READ_CONCURRENCY = 20
// read servers per partition (include/antidote.hrl:28) calls
// materializer_vnode:read/6 (src/clocksi_readitem_server.erl:272) and runs
// materialize/4 on its own copy of the key's ops.  On the GPU one key is
// 1/4 of a wave of work, so calls are coalesced: callers enqueue a request
// and block; one worker thread per batcher packs up to max_batch requests
// into one pinned buffer, does one H2D copy, one agn_oplog_read (the
// materialize kernel over the resident log, held shared) and one D2H copy,
// then wakes the callers.  Requests that arrive while a batch runs form the
// next batch, so the batch size adapts to the offered load.
//
// Cached mode (agn_batcher_create_cached, counter_pn) runs every batch as the
// whole of materializer_vnode:read/6 on the device: the batcher owns the
// partition's snapshot cache (agn_ss_cache), and a batch is
// get_from_snapshot_cache (agn_ss_lookup: the base snapshot <= R) ->
// materialize/4 from that base -> internal_store_ss / snapshot_insert_gc's
// policy (agn_ss_store, prune flags per request) -> prune_ops of the keys
// the policy selected (in place over the batch's key list, enqueued after the
// batch's results are out; only those keys' segments are visited).
// One batch holds distinct keys only (the cache's per-key state is
// read-modify-write); a second read of a key waits for the next batch, so
// reads of one key are applied in arrival order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_set>
#include <vector>

#include "serve.hpp"
#include "tags_serve.hpp"

using namespace agn;

namespace {

using Clock = std::chrono::steady_clock;

// agn_batcher_store's request: a snapshot the caller materialized itself
struct StoreReq {
    uint64_t key;
    const uint64_t *clock, *clock_mask;  // LastOpCt row [D] (+ [W]) (host)
    int64_t last_op, value;
    uint32_t count, n_pairs, flags;
    const uint32_t *tags;
    const uint64_t *toks;
};

struct Pending {
    const agn_key_read *rd;
    const StoreReq *st = nullptr;  // a store instead of a read (rd is null)
    agn_key_result *out;
    Clock::time_point t;
    int rc = AGN_OK;
    bool done = false;
    std::condition_variable cv;  // this caller's wake-up (no herd of every waiter per batch)
    char err[256] = "";
};

inline size_t al(size_t b) { return (b + 255) & ~size_t(255); }

}  // namespace

struct agn_batcher {
    agn_oplog *log = nullptr;
    agn_ctx *ctx = nullptr;
    uint32_t crdt = 0, D = 0, W = 0;
    int sparse_log = 0;
    uint64_t K = 0;
    uint32_t max_batch = 0, max_wait_us = 0;

    std::mutex mu;
    std::condition_variable cv_work;
    std::deque<Pending *> q;
    bool stop = false;
    std::thread worker;

    hipStream_t stream = nullptr;
    char *dbuf = nullptr, *hbuf = nullptr;  // device / pinned [in | out]
    char *hdev = nullptr;                   // hbuf as the device addresses it (read6)
    size_t cap = 0;
    std::atomic<uint64_t> n_batches{0}, n_reads{0};

    // cached mode: the partition's device snapshot cache + GC scratch
    bool cached = false;
    bool read6 = true;  // the fused one-kernel batch (AGN_READ6=0: the kernel sequence)
    bool tags_fused = true;  // set/register batches too (AGN_TAGS_FUSED=0: their sequence)
    agn_ss_cache ss{};
    uint64_t *thr = nullptr;    // [K][D] prune thresholds
    uint64_t *thrm = nullptr;   // [K][W] (sparse logs)
    // set_aw / register_mv: the cache's state arena (ss.state_*), the host's
    // copy of its state_ctl after the last batch, and per key an upper bound
    // of the pairs of any state the cache holds for it (the largest result
    // seen: every cached state is a result's), which sizes a batch's output
    uint64_t *ctl_h = nullptr;  // pinned [4]
    // written by the worker only; read by agn_batcher_state_bound's callers
    std::unique_ptr<std::atomic<uint32_t>[]> kbound;
    uint32_t bound_of(uint64_t k) const { return kbound[k].load(std::memory_order_relaxed); }
    void raise_bound(uint64_t k, uint32_t m) {
        if (m > bound_of(k)) kbound[k].store(m, std::memory_order_relaxed);
    }
    // the fused set/register read's scratch (tags_serve.hpp): 3 n + 4 words,
    // the first 4 zero between batches
    uint32_t *tscr = nullptr;
    uint64_t tscr_n = 0;
};

namespace {

int grow(agn_batcher *B, size_t bytes) {
    if (bytes <= B->cap) return AGN_OK;
    size_t c = std::max(bytes, 2 * B->cap);
    if (B->dbuf) AGN_HIP(hipFree(B->dbuf));
    if (B->hbuf) AGN_HIP(hipHostFree(B->hbuf));
    B->dbuf = B->hbuf = B->hdev = nullptr;
    B->cap = 0;
    AGN_HIP(hipMalloc((void **)&B->dbuf, c));
    AGN_HIP(hipHostMalloc((void **)&B->hbuf, c, hipHostMallocDefault));
    AGN_HIP(hipHostGetDevicePointer((void **)&B->hdev, B->hbuf, 0));
    B->cap = c;
    return AGN_OK;
}

// Wait for the batch's work on the batcher's stream.  (Polling a completion
// event instead measured the same: 0.955M vs 0.953M reads/s, 8 partitions,
// profiles/r02/serve/.)
int wait_batch(agn_batcher *B) {
    AGN_HIP(hipStreamSynchronize(B->stream));
    return AGN_OK;
}

// agn_key_result.err_pos is the failing op's id (its key's op counter value,
// what the caller's error term names): the kernels report the entry's slot in
// the log, meaningful only while the log is held, so it is translated through
// the log's op_id column here (one 4-byte read per failed read: rare).
int errs_to_op_ids(agn_batcher *B, const agn_log &view, std::vector<Pending *> &b) {
    for (Pending *p : b) {
        agn_key_result *o = p->out;
        if (!(o->flags & AGN_F_ERR_UNEXPECTED) || o->err_pos == 0xffffffffu || !view.op_id)
            continue;
        uint32_t id = 0;
        AGN_HIP(hipMemcpyAsync(&id, view.op_id + o->err_pos, 4, hipMemcpyDeviceToHost, B->stream));
        AGN_HIP(hipStreamSynchronize(B->stream));
        o->err_pos = id;
    }
    return AGN_OK;
}

// Cached mode, counter_pn with D <= 64 (dense clocks, or presence masks: the
// Erlang NIF's partitions): the whole batch is one fused kernel (read6.hip;
// k_read6 for D <= 8, k_read6w above)
// reading the requests from, and writing the results to, the pinned block
// directly; its GC follows in stream order from the batch's device key list.
int run_batch_read6(agn_batcher *B, std::vector<Pending *> &b, bool sparse) {
    const uint64_t n = b.size();
    const uint32_t D = B->D;
    std::vector<uint64_t> keys(n);
    for (uint64_t i = 0; i < n; ++i) keys[i] = b[i]->rd->key;
    size_t d_keys = 0, d_pr = 0;
    {
        std::shared_lock<std::shared_mutex> hold;
        int rc = oplog_begin_read(B->log, B->stream, 0, nullptr, nullptr, hold);
        if (rc) return rc;
        size_t off = 0;
        auto slot = [&](size_t bytes) { size_t o = off; off = al(off + bytes); return o; };
        const size_t o_keys = slot(n * 8), o_R = slot(n * D * 8), o_txid = slot(n * 8),
                     o_gc = slot(n), o_val = slot(n * 8), o_hole = slot(n * 8),
                     o_ct = slot(n * D * 8), o_cnt = slot(n * 4), o_flg = slot(n * 4),
                     o_epos = slot(n * 4), o_st = slot(n), o_pr = slot(n),
                     o_Rm = slot(sparse ? n * 8 : 0), o_ctm = slot(sparse ? n * 8 : 0);
        d_keys = 0;
        d_pr = al(n * 8);
        // D > 8 (k_read6w): the lookup's SCT rows / masks, ignore bytes and the
        // LastOpCt rows / masks, in device memory
        const bool wide = D > 8;
        const size_t d_sct = al(d_pr + n), d_sctm = al(d_sct + (wide ? n * D * 8 : 0)),
                     d_ct = al(d_sctm + (wide ? n * 8 : 0)), d_ctm = al(d_ct + (wide ? n * D * 8 : 0)),
                     d_ign = al(d_ctm + (wide ? n * 8 : 0)), d_end = d_ign + (wide ? n : 0);
        rc = grow(B, std::max(off, d_end));
        if (rc) return rc;
        char *h = B->hbuf;
        bool any_tx = false;
        const uint64_t full = D >= 64 ? ~0ull : (1ull << D) - 1ull;
        for (uint64_t i = 0; i < n; ++i) {
            const agn_key_read *r = b[i]->rd;
            ((uint64_t *)(h + o_keys))[i] = r->key;
            std::memcpy(h + o_R + i * D * 8, r->R, D * 8);
            if (sparse) ((uint64_t *)(h + o_Rm))[i] = r->R_mask ? r->R_mask[0] : full;
            ((uint64_t *)(h + o_txid))[i] = r->txid;
            any_tx = any_tx || r->txid;
            ((uint8_t *)(h + o_gc))[i] = (r->flags & AGN_READ_GC) ? 1 : 0;
        }
        agn_log view;
        oplog_view(B->log, &view);
        char *x = B->hdev;
        Read6Args a;
        std::memset(&a, 0, sizeof a);
        a.key_off = view.key_off;
        a.key_len = view.key_len;
        a.key_id0 = view.key_id0;
        a.key_type = view.key_type;
        a.oc = view.oc;
        a.op_id = view.op_id;
        a.eff = view.eff;
        a.log_txid = view.txid;
        a.n_entries = view.n_entries;
        a.n_dcs = D;
        a.req_type = B->crdt;
        a.n_req = n;
        a.keys = (const uint64_t *)(x + o_keys);
        a.R = (const uint64_t *)(x + o_R);
        a.txid = any_tx ? (const uint64_t *)(x + o_txid) : nullptr;
        a.gc = (const uint8_t *)(x + o_gc);
        a.value = (int64_t *)(x + o_val);
        a.hole = (int64_t *)(x + o_hole);
        a.lastct = (uint64_t *)(x + o_ct);
        a.count = (uint32_t *)(x + o_cnt);
        a.flags = (uint32_t *)(x + o_flg);
        a.err_pos = (uint32_t *)(x + o_epos);
        a.status = (uint8_t *)(x + o_st);
        a.prune = (uint8_t *)(x + o_pr);
        a.dkeys = (uint64_t *)(B->dbuf + d_keys);
        a.dprune = (uint8_t *)(B->dbuf + d_pr);
        a.thr = B->thr;
        if (wide) {
            a.sct_scr = (uint64_t *)(B->dbuf + d_sct);
            a.sctm_scr = (uint64_t *)(B->dbuf + d_sctm);
            a.ct_scr = (uint64_t *)(B->dbuf + d_ct);
            a.ctm_scr = (uint64_t *)(B->dbuf + d_ctm);
            a.ign_scr = (uint8_t *)(B->dbuf + d_ign);
        }
        if (sparse) {
            a.key_mask = view.key_mask;
            a.oc_mask = view.oc_mask;
            a.R_mask = (const uint64_t *)(x + o_Rm);
            a.lastct_mask = (uint64_t *)(x + o_ctm);
            a.thrm = B->thrm;
        }
        rc = launch_read6(B->ss, a, B->stream);
        if (rc) return rc;
        rc = wait_batch(B);
        if (rc) return rc;
        bool any_prune = false;
        for (uint64_t i = 0; i < n; ++i) {
            agn_key_result *o = b[i]->out;
            o->status = ((const uint8_t *)(h + o_st))[i];
            o->value = ((const int64_t *)(h + o_val))[i];
            o->hole = ((const int64_t *)(h + o_hole))[i];
            std::memcpy(o->lastct, h + o_ct + i * D * 8, D * 8);
            if (o->lastct_mask) {
                std::memset(o->lastct_mask, 0, B->W * 8);
                o->lastct_mask[0] = sparse ? ((const uint64_t *)(h + o_ctm))[i] : full;
            }
            o->count = ((const uint32_t *)(h + o_cnt))[i];
            o->flags = ((const uint32_t *)(h + o_flg))[i];
            o->err_pos = ((const uint32_t *)(h + o_epos))[i];
            o->out_n = 0;
            any_prune = any_prune || ((const uint8_t *)(h + o_pr))[i] != 0;
        }
        rc = errs_to_op_ids(B, view, b);
        if (rc) return rc;
        if (!any_prune) return AGN_OK;
    }  // the shared hold ends: the GC takes the log exclusively
    return oplog_prune_keys(B->log, n, keys.data(), (const uint64_t *)(B->dbuf + d_keys),
                            (const uint8_t *)(B->dbuf + d_pr), B->thr, B->thrm, B->stream);
}

// The state arena must hold `need` more pairs: re-pack the live states into a
// fresh arena of max(capacity, 2 x (live + need)) pairs (agn_ss_state_compact's
// kernel) and free the old one.  Between batches, on the batcher's stream.
// A store that did not fit (state_ctl[2]) still advanced state_ctl[0] past
// the capacity (its pairs counted as released), so the room is clamped at 0
// and an overflow always re-packs (which clears it).  The re-pack commits all
// or nothing: the slots' new references go to scratch and replace the cache's
// only when every live state fit; otherwise the old arena, references and
// state_ctl stay as they were.
int ensure_state_room(agn_batcher *B, uint64_t need) {
    const uint64_t used = B->ctl_h[0];
    const uint64_t room = used >= B->ss.state_cap ? 0 : B->ss.state_cap - used;
    if (room >= need && !B->ctl_h[2]) return AGN_OK;
    // the exact counters (the host copy may be a sum of per-store deltas)
    uint64_t ctl[4];
    AGN_HIP(hipMemcpyAsync(ctl, B->ss.state_ctl, sizeof ctl, hipMemcpyDeviceToHost, B->stream));
    AGN_HIP(hipStreamSynchronize(B->stream));
    std::memcpy(B->ctl_h, ctl, sizeof ctl);
    const uint64_t live = ctl[0] - ctl[1];
    const uint64_t cap = std::max<uint64_t>(B->ss.state_cap, 2 * (live + need));
    const uint64_t nval = B->ss.n_keys * B->ss.slots;
    uint32_t *nt = nullptr;
    uint64_t *nk = nullptr;
    int64_t *nv = nullptr;
    if (hipMalloc((void **)&nt, cap * 4) != hipSuccess || hipMalloc((void **)&nk, cap * 8) != hipSuccess ||
        hipMalloc((void **)&nv, std::max<uint64_t>(nval, 1) * 8) != hipSuccess) {
        if (nt) (void)hipFree(nt);
        if (nk) (void)hipFree(nk);
        return fail(AGN_ENOMEM, "batcher: state arena of %llu pairs", (unsigned long long)cap);
    }
    int rc = launch_ss_compact(B->ss, nt, nk, cap, B->ss.state_ctl + 2, B->stream, nv);
    uint64_t after[4] = {0, 0, 0, 0};
    if (rc == AGN_OK && hipMemcpyAsync(after, B->ss.state_ctl, sizeof after, hipMemcpyDeviceToHost,
                                       B->stream) != hipSuccess)
        rc = fail(AGN_EHIP, "batcher: state_ctl copy");
    if (rc == AGN_OK && hipStreamSynchronize(B->stream) != hipSuccess)
        rc = fail(AGN_EHIP, "batcher: state compaction");
    if (rc == AGN_OK && after[2]) {
        // did not fit (the live count disagreed with the slots): keep the old
        // arena and references, restore its counters
        if (hipMemcpyAsync(B->ss.state_ctl, ctl, sizeof ctl, hipMemcpyHostToDevice, B->stream) !=
                hipSuccess ||
            hipStreamSynchronize(B->stream) != hipSuccess)
            rc = fail(AGN_EHIP, "batcher: state_ctl restore");
        else
            rc = fail(AGN_ECAPACITY, "batcher: state re-pack overflowed %llu pairs",
                      (unsigned long long)cap);
    }
    if (rc == AGN_OK && nval &&
        (hipMemcpyAsync(B->ss.value, nv, nval * 8, hipMemcpyDeviceToDevice, B->stream) != hipSuccess ||
         hipStreamSynchronize(B->stream) != hipSuccess))
        rc = fail(AGN_EHIP, "batcher: state references commit");
    (void)hipFree(nv);
    if (rc) {
        (void)hipFree(nt);
        (void)hipFree(nk);
        return rc;
    }
    std::memcpy(B->ctl_h, after, sizeof after);
    (void)hipFree(B->ss.state_tag);
    (void)hipFree(B->ss.state_tok);
    B->ss.state_tag = nt;
    B->ss.state_tok = nk;
    B->ss.state_cap = cap;
    return AGN_OK;
}

// Cached mode, set_aw / register_mv with D <= 8: the fused read
// (tags_serve.hpp) -- one kernel per batch reading the requests from, and
// writing the results to, the pinned block (lookup -> fast tags pass ->
// store, per request on one wave).  The host keeps its copy of state_ctl
// from the stores' reported deltas.  A batch with keys the kernel handed on
// (a state past the fast table, a key not uniform inside R's DC set) runs
// the remaining passes and their store, and reads state_ctl back.
int run_batch_tags_fused(agn_batcher *B, std::vector<Pending *> &b, bool sparse) {
    const uint64_t n = b.size();
    const uint32_t D = B->D, W = B->W;
    std::vector<uint64_t> keys(n);
    std::vector<uint32_t> lens(n);
    for (uint64_t i = 0; i < n; ++i) keys[i] = b[i]->rd->key;
    size_t d_keys = 0, d_pr = 0;
    {
        std::shared_lock<std::shared_mutex> hold;
        int rc = oplog_begin_read(B->log, B->stream, n, keys.data(), lens.data(), hold);
        if (rc) return rc;
        std::vector<uint64_t> co(n + 1);
        co[0] = 0;
        for (uint64_t i = 0; i < n; ++i) co[i + 1] = co[i] + lens[i] + B->bound_of(keys[i]);
        const uint64_t ncap = co[n];
        rc = ensure_state_room(B, ncap);
        if (rc) return rc;
        if (B->tscr_n < n) {
            const uint64_t m = std::max<uint64_t>(n, 2 * B->tscr_n);
            if (B->tscr) AGN_HIP(hipFree(B->tscr));
            B->tscr = nullptr;
            B->tscr_n = 0;
            AGN_HIP(hipMalloc((void **)&B->tscr, (3 * m + 4) * sizeof(uint32_t)));
            AGN_HIP(hipMemsetAsync(B->tscr, 0, 4 * sizeof(uint32_t), B->stream));
            B->tscr_n = m;
        }
        // pinned block (the kernel addresses it through hdev)
        size_t off = 0;
        auto slot = [&](size_t bytes) { size_t o = off; off = al(off + bytes); return o; };
        const size_t o_keys = slot(n * 8), o_R = slot(n * D * 8), o_Rm = slot(sparse ? n * W * 8 : 0),
                     o_txid = slot(n * 8), o_gc = slot(n), o_cap = slot((n + 1) * 8),
                     o_st = slot(n), o_pr = slot(n), o_dl = slot(n * 16), o_hole = slot(n * 8),
                     o_ct = slot(n * D * 8), o_ctm = slot(sparse ? n * W * 8 : 0),
                     o_cnt = slot(n * 4), o_flg = slot(n * 4), o_epos = slot(n * 4),
                     o_outn = slot(n * 4), o_otag = slot(std::max<uint64_t>(ncap, 1) * 4),
                     o_otok = slot(std::max<uint64_t>(ncap, 1) * 8);
        const size_t hbytes = off;
        // device block: the lookup's rows and the GC list
        off = 0;
        const size_t d_sct = slot(n * D * 8), d_sctm = slot(sparse ? n * W * 8 : 0),
                     d_ign = slot(n), d_base = slot(n * 8), d_first = slot(n);
        d_keys = slot(n * 8);
        d_pr = slot(n);
        rc = grow(B, std::max(hbytes, off));
        if (rc) return rc;
        char *h = B->hbuf, *x = B->hdev, *d = B->dbuf;
        auto H = [&](size_t o) { return h + o; };
        uint64_t full[4] = {0, 0, 0, 0};
        for (uint32_t c = 0; c < D; ++c) full[c >> 6] |= 1ull << (c & 63);
        bool any_tx = false;
        for (uint64_t i = 0; i < n; ++i) {
            const agn_key_read *r = b[i]->rd;
            ((uint64_t *)H(o_keys))[i] = r->key;
            std::memcpy(H(o_R) + i * D * 8, r->R, D * 8);
            if (sparse) std::memcpy(H(o_Rm) + i * W * 8, r->R_mask ? r->R_mask : full, W * 8);
            ((uint64_t *)H(o_txid))[i] = r->txid;
            any_tx = any_tx || r->txid;
            ((uint8_t *)H(o_gc))[i] = (r->flags & AGN_READ_GC) ? 1 : 0;
        }
        std::memcpy(H(o_cap), co.data(), (n + 1) * 8);
        agn_log view;
        oplog_view(B->log, &view);
        agn_read req;
        std::memset(&req, 0, sizeof req);
        req.n_req = n;
        req.keys = (const uint64_t *)(x + o_keys);
        req.R = (const uint64_t *)(x + o_R);
        req.R_mask = sparse ? (const uint64_t *)(x + o_Rm) : nullptr;
        req.sct = (const uint64_t *)(d + d_sct);
        req.sct_mask = sparse ? (const uint64_t *)(d + d_sctm) : nullptr;
        req.sct_ignore = (const uint8_t *)(d + d_ign);
        req.txid = any_tx ? (const uint64_t *)(x + o_txid) : nullptr;
        req.req_type = B->crdt;
        req.base_value = (const int64_t *)(d + d_base);  // AGN_SS_STATE into the arena
        req.base_tag = B->ss.state_tag;
        req.base_tok = B->ss.state_tok;
        agn_result res;
        std::memset(&res, 0, sizeof res);
        res.hole = (int64_t *)(x + o_hole);
        res.lastct = (uint64_t *)(x + o_ct);
        res.lastct_mask = sparse ? (uint64_t *)(x + o_ctm) : nullptr;
        res.count = (uint32_t *)(x + o_cnt);
        res.flags = (uint32_t *)(x + o_flg);
        res.err_pos = (uint32_t *)(x + o_epos);
        res.out_off = (const uint64_t *)(x + o_cap);
        res.out_n = (uint32_t *)(x + o_outn);
        res.out_tag = (uint32_t *)(x + o_otag);
        res.out_tok = (uint64_t *)(x + o_otok);
        TagServe sv;
        std::memset(&sv, 0, sizeof sv);
        sv.c = B->ss;
        sv.sct = (uint64_t *)(d + d_sct);
        sv.sctm = sparse ? (uint64_t *)(d + d_sctm) : nullptr;
        sv.ign = (uint8_t *)(d + d_ign);
        sv.first = (uint8_t *)(d + d_first);
        sv.base = (int64_t *)(d + d_base);
        sv.status = (uint8_t *)(x + o_st);
        sv.gc = (const uint8_t *)(x + o_gc);
        sv.prune = (uint8_t *)(x + o_pr);
        sv.delta = (uint64_t *)(x + o_dl);
        sv.dkeys = (uint64_t *)(d + d_keys);
        sv.dprune = (uint8_t *)(d + d_pr);
        sv.thr = B->thr;
        sv.thrm = B->thrm;
        rc = launch_tags_serve(view, req, res, sv, B->tscr, B->stream);
        if (rc) return rc;
        rc = wait_batch(B);
        if (rc) return rc;
        bool handed_on = false;
        for (uint64_t i = 0; i < n; ++i) handed_on = handed_on || (((const uint8_t *)H(o_pr))[i] & 4u);
        if (handed_on) {
            rc = launch_tags_serve_rest(view, req, res, sv, B->tscr, B->stream);
            if (rc) return rc;
            AGN_HIP(hipMemcpyAsync(H(o_pr), d + d_pr, n, hipMemcpyDeviceToHost, B->stream));
            AGN_HIP(hipMemcpyAsync(B->ctl_h, B->ss.state_ctl, 4 * 8, hipMemcpyDeviceToHost, B->stream));
            rc = wait_batch(B);
            if (rc) return rc;
        } else {
            for (uint64_t i = 0; i < n; ++i) {
                const uint64_t *dl = (const uint64_t *)H(o_dl) + 2 * i;
                B->ctl_h[0] += dl[0];
                B->ctl_h[1] += dl[1];
                if (((const uint8_t *)H(o_pr))[i] & 2u) B->ctl_h[2] = 1;
            }
        }
        // ctl_h[2]: a store did not fit the arena and was not made (its
        // snapshot is simply not cached: the results stand); the next batch's
        // ensure_state_room re-packs
        bool any_prune = false;
        for (uint64_t i = 0; i < n; ++i) {
            agn_key_result *o = b[i]->out;
            const uint32_t m = ((const uint32_t *)H(o_outn))[i];
            o->status = ((const uint8_t *)H(o_st))[i];
            o->value = 0;
            o->hole = ((const int64_t *)H(o_hole))[i];
            std::memcpy(o->lastct, H(o_ct) + i * D * 8, D * 8);
            if (o->lastct_mask)
                std::memcpy(o->lastct_mask, sparse ? H(o_ctm) + i * W * 8 : (char *)full, W * 8);
            o->count = ((const uint32_t *)H(o_cnt))[i];
            o->flags = ((const uint32_t *)H(o_flg))[i];
            o->err_pos = ((const uint32_t *)H(o_epos))[i];
            any_prune = any_prune || (((const uint8_t *)H(o_pr))[i] & 1u) != 0;
            const bool ok = !(o->flags & (AGN_F_ERR_CORRUPTED | AGN_F_ERR_UNEXPECTED |
                                          AGN_F_ERR_CAPACITY));
            o->out_n = ok ? m : 0;
            if (ok) B->raise_bound(keys[i], m);
            if (!ok || o->status == AGN_SS_LOG) continue;
            if (m > o->out_cap) {  // the caller retries with out_cap >= out_n
                b[i]->rc = AGN_ECAPACITY;
                std::snprintf(b[i]->err, sizeof b[i]->err, "batcher_read: %u pairs, out_cap %u",
                              m, o->out_cap);
                continue;
            }
            if (m) {
                std::memcpy(o->out_tag, H(o_otag) + co[i] * 4, m * 4);
                std::memcpy(o->out_tok, H(o_otok) + co[i] * 8, m * 8);
            }
        }
        rc = errs_to_op_ids(B, view, b);
        if (rc) return rc;
        if (!any_prune) return AGN_OK;
    }  // the shared hold ends: the GC takes the log exclusively
    return oplog_prune_keys(B->log, n, keys.data(), (const uint64_t *)(B->dbuf + d_keys),
                            (const uint8_t *)(B->dbuf + d_pr), B->thr, B->thrm, B->stream);
}

// Cached mode, set_aw / register_mv: read/6 for a batch with the snapshot
// states on the device.  get_from_snapshot_cache's base is the hit slot's
// state in the arena (agn_ss_lookup writes its AGN_SS_STATE reference), the
// tags kernel folds the key's ops onto it in place of a host-shipped base,
// and materialize_snapshot's store appends the result's state to the arena:
// no state crosses PCIe except the caller's result.
int run_batch_cached_tags(agn_batcher *B, std::vector<Pending *> &b) {
    const uint64_t n = b.size();
    const uint32_t D = B->D, W = B->W;
    bool sparse = B->sparse_log != 0;
    for (Pending *p : b) sparse = sparse || p->rd->R_mask;
    if (B->read6 && B->tags_fused) {
        agn_log v;  // the shape only (the log's view is taken under its hold)
        std::memset(&v, 0, sizeof v);
        v.n_dcs = D;
        if (tags_serve_supported(v, sparse)) return run_batch_tags_fused(B, b, sparse);
    }
    std::vector<uint64_t> keys(n);
    std::vector<uint32_t> lens(n);
    for (uint64_t i = 0; i < n; ++i) keys[i] = b[i]->rd->key;
    size_t o_keys_saved = 0, o_pr_saved = 0;
    {
        std::shared_lock<std::shared_mutex> hold;
        int rc = oplog_begin_read(B->log, B->stream, n, keys.data(), lens.data(), hold);
        if (rc) return rc;
        // result capacity per request: the key's entries (each adds at most
        // one pair) + the bound of its cached states
        std::vector<uint64_t> co(n + 1);
        co[0] = 0;
        for (uint64_t i = 0; i < n; ++i) co[i + 1] = co[i] + lens[i] + B->bound_of(keys[i]);
        const uint64_t ncap = co[n];
        rc = ensure_state_room(B, ncap);
        if (rc) return rc;
        size_t off = 0;
        auto slot = [&](size_t bytes) { size_t o = off; off = al(off + bytes); return o; };
        const size_t o_keys = slot(n * 8), o_R = slot(n * D * 8), o_Rm = slot(sparse ? n * W * 8 : 0),
                     o_txid = slot(n * 8), o_gc = slot(n), o_cap = slot((n + 1) * 8);
        const size_t in_bytes = off;
        const size_t o_sct = slot(n * D * 8), o_sctm = slot(sparse ? n * W * 8 : 0),
                     o_ign = slot(n), o_base = slot(n * 8), o_first = slot(n);
        const size_t out_start = off;
        const size_t o_hole = slot(n * 8), o_ct = slot(n * D * 8),
                     o_ctm = slot(sparse ? n * W * 8 : 0), o_cnt = slot(n * 4), o_flg = slot(n * 4),
                     o_epos = slot(n * 4), o_st = slot(n), o_pr = slot(n), o_outn = slot(n * 4),
                     o_otag = slot(std::max<uint64_t>(ncap, 1) * 4),
                     o_otok = slot(std::max<uint64_t>(ncap, 1) * 8);
        rc = grow(B, off);
        if (rc) return rc;
        o_keys_saved = o_keys;
        o_pr_saved = o_pr;
        char *h = B->hbuf, *d = B->dbuf;
        auto H = [&](size_t o) { return h + o; };
        uint64_t full[4] = {0, 0, 0, 0};
        for (uint32_t x = 0; x < D; ++x) full[x >> 6] |= 1ull << (x & 63);
        for (uint64_t i = 0; i < n; ++i) {
            const agn_key_read *r = b[i]->rd;
            ((uint64_t *)H(o_keys))[i] = r->key;
            std::memcpy(H(o_R) + i * D * 8, r->R, D * 8);
            if (sparse) std::memcpy(H(o_Rm) + i * W * 8, r->R_mask ? r->R_mask : full, W * 8);
            ((uint64_t *)H(o_txid))[i] = r->txid;
            ((uint8_t *)H(o_gc))[i] = (r->flags & AGN_READ_GC) ? 1 : 0;
        }
        std::memcpy(H(o_cap), co.data(), (n + 1) * 8);
        AGN_HIP(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, B->stream));
        agn_log view;
        oplog_view(B->log, &view);
        const uint64_t *dkeys = (const uint64_t *)(d + o_keys);
        rc = launch_ss_lookup(B->ss, n, dkeys, (const uint64_t *)(d + o_R),
                              sparse ? (const uint64_t *)(d + o_Rm) : nullptr,
                              (uint64_t *)(d + o_sct), sparse ? (uint64_t *)(d + o_sctm) : nullptr,
                              (uint8_t *)(d + o_ign), (int64_t *)(d + o_base),
                              (uint8_t *)(d + o_first), (uint8_t *)(d + o_st), B->stream);
        if (rc) return rc;
        agn_read req;
        std::memset(&req, 0, sizeof req);
        req.n_req = n;
        req.keys = dkeys;
        req.R = (const uint64_t *)(d + o_R);
        req.R_mask = sparse ? (const uint64_t *)(d + o_Rm) : nullptr;
        req.sct = (const uint64_t *)(d + o_sct);
        req.sct_mask = sparse ? (const uint64_t *)(d + o_sctm) : nullptr;
        req.sct_ignore = (const uint8_t *)(d + o_ign);
        req.txid = (const uint64_t *)(d + o_txid);
        req.req_type = B->crdt;
        req.base_value = (const int64_t *)(d + o_base);  // AGN_SS_STATE into the arena
        req.base_tag = B->ss.state_tag;
        req.base_tok = B->ss.state_tok;
        agn_result res;
        std::memset(&res, 0, sizeof res);
        res.hole = (int64_t *)(d + o_hole);
        res.lastct = (uint64_t *)(d + o_ct);
        res.lastct_mask = sparse ? (uint64_t *)(d + o_ctm) : nullptr;
        res.count = (uint32_t *)(d + o_cnt);
        res.flags = (uint32_t *)(d + o_flg);
        res.err_pos = (uint32_t *)(d + o_epos);
        res.out_off = (const uint64_t *)(d + o_cap);
        res.out_n = (uint32_t *)(d + o_outn);
        res.out_tag = (uint32_t *)(d + o_otag);
        res.out_tok = (uint64_t *)(d + o_otok);
        rc = launch_tags(view, req, res, B->stream);
        if (rc) return rc;
        rc = launch_ss_store_req(B->ss, view.key_off, view.key_len, n, dkeys,
                                 (const uint8_t *)(d + o_first), (const uint8_t *)(d + o_st),
                                 (const uint8_t *)(d + o_gc), res, (uint8_t *)(d + o_pr), B->thr,
                                 B->thrm, B->stream);
        if (rc) return rc;
        AGN_HIP(hipMemcpyAsync(h + out_start, d + out_start, off - out_start, hipMemcpyDeviceToHost,
                               B->stream));
        AGN_HIP(hipMemcpyAsync(B->ctl_h, B->ss.state_ctl, 4 * 8, hipMemcpyDeviceToHost, B->stream));
        rc = wait_batch(B);
        if (rc) return rc;
        // ctl_h[2]: a store did not fit the arena and was not made (its
        // snapshot is simply not cached: the results stand); the next batch's
        // ensure_state_room re-packs
        bool any_prune = false;
        for (uint64_t i = 0; i < n; ++i) {
            agn_key_result *o = b[i]->out;
            const uint32_t m = ((const uint32_t *)H(o_outn))[i];
            o->status = ((const uint8_t *)H(o_st))[i];
            o->value = 0;
            o->hole = ((const int64_t *)H(o_hole))[i];
            std::memcpy(o->lastct, H(o_ct) + i * D * 8, D * 8);
            if (o->lastct_mask)
                std::memcpy(o->lastct_mask, sparse ? H(o_ctm) + i * W * 8 : (char *)full, W * 8);
            o->count = ((const uint32_t *)H(o_cnt))[i];
            o->flags = ((const uint32_t *)H(o_flg))[i];
            o->err_pos = ((const uint32_t *)H(o_epos))[i];
            any_prune = any_prune || ((const uint8_t *)H(o_pr))[i] != 0;
            const bool ok = !(o->flags & (AGN_F_ERR_CORRUPTED | AGN_F_ERR_UNEXPECTED |
                                          AGN_F_ERR_CAPACITY));
            o->out_n = ok ? m : 0;
            if (ok) B->raise_bound(keys[i], m);
            if (!ok || o->status == AGN_SS_LOG) continue;
            if (m > o->out_cap) {  // the caller retries with out_cap >= out_n
                b[i]->rc = AGN_ECAPACITY;
                std::snprintf(b[i]->err, sizeof b[i]->err, "batcher_read: %u pairs, out_cap %u",
                              m, o->out_cap);
                continue;
            }
            if (m) {
                std::memcpy(o->out_tag, H(o_otag) + co[i] * 4, m * 4);
                std::memcpy(o->out_tok, H(o_otok) + co[i] * 8, m * 8);
            }
        }
        rc = errs_to_op_ids(B, view, b);
        if (rc) return rc;
        if (!any_prune) return AGN_OK;
    }  // the shared hold ends: the GC takes the log exclusively
    return oplog_prune_keys(B->log, n, keys.data(), (const uint64_t *)(B->dbuf + o_keys_saved),
                            (const uint8_t *)(B->dbuf + o_pr_saved), B->thr, B->thrm, B->stream);
}

// Cached mode: read/6 for a batch of distinct keys (see the file comment).
int run_batch_cached(agn_batcher *B, std::vector<Pending *> &b) {
    const uint64_t n = b.size();
    const uint32_t D = B->D, W = B->W;
    if (B->crdt != AGN_COUNTER_PN) return run_batch_cached_tags(B, b);
    bool sparse = B->sparse_log != 0;
    for (Pending *p : b) sparse = sparse || p->rd->R_mask;
    if (D <= 64 && B->read6) return run_batch_read6(B, b, sparse);
    std::vector<uint64_t> keys(n);
    for (uint64_t i = 0; i < n; ++i) keys[i] = b[i]->rd->key;
    int rc;
    size_t o_keys_saved = 0, o_pr_saved = 0;
    {
        std::shared_lock<std::shared_mutex> hold;
        uint64_t n_mixed = 0;
        rc = oplog_begin_read(B->log, B->stream, 0, nullptr, nullptr, hold, sparse ? n : 0,
                              keys.data(), &n_mixed);
        if (rc) return rc;
        // in = keys R Rm txid gc | scratch = sct sctm ign base first
        // out = value hole lastct lastct_mask count flags err_pos status prune
        size_t off = 0;
        auto slot = [&](size_t bytes) { size_t o = off; off = al(off + bytes); return o; };
        const size_t o_keys = slot(n * 8), o_R = slot(n * D * 8), o_Rm = slot(sparse ? n * W * 8 : 0),
                     o_txid = slot(n * 8), o_gc = slot(n);
        const size_t in_bytes = off;
        const size_t o_sct = slot(n * D * 8), o_sctm = slot(sparse ? n * W * 8 : 0),
                     o_ign = slot(n), o_base = slot(n * 8), o_first = slot(n);
        const size_t out_start = off;
        const size_t o_val = slot(n * 8), o_hole = slot(n * 8), o_ct = slot(n * D * 8),
                     o_ctm = slot(sparse ? n * W * 8 : 0), o_cnt = slot(n * 4), o_flg = slot(n * 4),
                     o_epos = slot(n * 4), o_st = slot(n), o_pr = slot(n);
        rc = grow(B, off);
        if (rc) return rc;
        o_keys_saved = o_keys;
        o_pr_saved = o_pr;
        char *h = B->hbuf, *d = B->dbuf;
        auto H = [&](size_t o) { return h + o; };
        uint64_t full[4] = {0, 0, 0, 0};
        for (uint32_t x = 0; x < D; ++x) full[x >> 6] |= 1ull << (x & 63);
        for (uint64_t i = 0; i < n; ++i) {
            const agn_key_read *r = b[i]->rd;
            ((uint64_t *)H(o_keys))[i] = r->key;
            std::memcpy(H(o_R) + i * D * 8, r->R, D * 8);
            if (sparse) std::memcpy(H(o_Rm) + i * W * 8, r->R_mask ? r->R_mask : full, W * 8);
            ((uint64_t *)H(o_txid))[i] = r->txid;
            ((uint8_t *)H(o_gc))[i] = (r->flags & AGN_READ_GC) ? 1 : 0;
        }
        AGN_HIP(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, B->stream));
        agn_log view;
        oplog_view(B->log, &view);
        const uint64_t *dkeys = (const uint64_t *)(d + o_keys);
        rc = agn_ss_lookup(B->ctx, &B->ss, n, dkeys, (const uint64_t *)(d + o_R),
                           sparse ? (const uint64_t *)(d + o_Rm) : nullptr, (uint64_t *)(d + o_sct),
                           sparse ? (uint64_t *)(d + o_sctm) : nullptr, (uint8_t *)(d + o_ign),
                           (int64_t *)(d + o_base), (uint8_t *)(d + o_first),
                           (uint8_t *)(d + o_st), B->stream);
        if (rc) return rc;
        agn_read req;
        std::memset(&req, 0, sizeof req);
        req.n_req = n;
        req.keys = dkeys;
        req.R = (const uint64_t *)(d + o_R);
        req.R_mask = sparse ? (const uint64_t *)(d + o_Rm) : nullptr;
        req.sct = (const uint64_t *)(d + o_sct);
        req.sct_mask = sparse ? (const uint64_t *)(d + o_sctm) : nullptr;
        req.sct_ignore = (const uint8_t *)(d + o_ign);
        req.txid = (const uint64_t *)(d + o_txid);
        req.req_type = B->crdt;
        req.base_value = (const int64_t *)(d + o_base);
        // many of the batch's keys with entries of different DC sets (e.g.
        // soon after a DC joined): the counter kernel scans them in one pass
        if (sparse && many_mixed(n_mixed, n)) req.hints |= AGN_HINT_MIXED;
        agn_result res;
        std::memset(&res, 0, sizeof res);
        res.value = (int64_t *)(d + o_val);
        res.hole = (int64_t *)(d + o_hole);
        res.lastct = (uint64_t *)(d + o_ct);
        res.lastct_mask = sparse ? (uint64_t *)(d + o_ctm) : nullptr;
        res.count = (uint32_t *)(d + o_cnt);
        res.flags = (uint32_t *)(d + o_flg);
        res.err_pos = (uint32_t *)(d + o_epos);
        // a key whose cache has no snapshot <= R (AGN_SS_LOG) still runs
        // through the kernel from the empty base; its result is discarded
        rc = agn_materialize(B->ctx, &view, &req, &res, B->stream);
        if (rc) return rc;
        // internal_store_ss / snapshot_insert_gc's policy; its prune flags go
        // per request straight into the batch's output block
        rc = launch_ss_store_req(B->ss, view.key_off, view.key_len, n, dkeys,
                                 (const uint8_t *)(d + o_first), (const uint8_t *)(d + o_st),
                                 (const uint8_t *)(d + o_gc), res, (uint8_t *)(d + o_pr), B->thr,
                                 B->thrm, B->stream);
        if (rc) return rc;
        AGN_HIP(hipMemcpyAsync(h + out_start, d + out_start, off - out_start, hipMemcpyDeviceToHost,
                               B->stream));
        rc = wait_batch(B);
        if (rc) return rc;
        bool any_prune = false;
        for (uint64_t i = 0; i < n; ++i) {
            agn_key_result *o = b[i]->out;
            o->status = ((const uint8_t *)H(o_st))[i];
            o->value = ((const int64_t *)H(o_val))[i];
            o->hole = ((const int64_t *)H(o_hole))[i];
            std::memcpy(o->lastct, H(o_ct) + i * D * 8, D * 8);
            if (o->lastct_mask)
                std::memcpy(o->lastct_mask, sparse ? H(o_ctm) + i * W * 8 : (char *)full, W * 8);
            o->count = ((const uint32_t *)H(o_cnt))[i];
            o->flags = ((const uint32_t *)H(o_flg))[i];
            o->err_pos = ((const uint32_t *)H(o_epos))[i];
            o->out_n = 0;
            any_prune = any_prune || ((const uint8_t *)H(o_pr))[i] != 0;
        }
        rc = errs_to_op_ids(B, view, b);
        if (rc) return rc;
        if (!any_prune) return AGN_OK;
    }  // the shared hold ends: the GC takes the log exclusively
    // prune_ops of the batch's selected keys (in place, over the batch's key
    // list and flags still in the device block -- stream-ordered before the
    // next batch's copy-in -- asynchronous: the next read of the log waits)
    return oplog_prune_keys(B->log, n, keys.data(), (const uint64_t *)(B->dbuf + o_keys_saved),
                            (const uint8_t *)(B->dbuf + o_pr_saved), B->thr, B->thrm, B->stream);
}

// One batch: pack, copy in, materialize over the resident log, copy out, unpack.
int run_batch(agn_batcher *B, std::vector<Pending *> &b) {
    const uint64_t n = b.size();
    const uint32_t D = B->D, W = B->W;
    const bool tags = B->crdt != AGN_COUNTER_PN;
    bool sparse = B->sparse_log != 0, any_sct = false;
    uint64_t nb = 0;
    for (Pending *p : b) {
        sparse = sparse || p->rd->R_mask || p->rd->sct_mask;
        any_sct = any_sct || p->rd->sct;
        nb += tags ? p->rd->n_base : 0;
    }
    std::vector<uint64_t> keys(n);
    std::vector<uint32_t> lens(n);
    for (uint64_t i = 0; i < n; ++i) keys[i] = b[i]->rd->key;
    // flush + exact key lengths + the arena held shared until the batch is done
    std::shared_lock<std::shared_mutex> hold;
    uint64_t n_mixed = 0;
    int rc = oplog_begin_read(B->log, B->stream, tags ? n : 0, keys.data(), lens.data(), hold,
                              tags ? 0 : n, keys.data(), &n_mixed);
    if (rc) return rc;
    uint64_t ncap = 0;
    if (tags)
        for (uint64_t i = 0; i < n; ++i) ncap += (uint64_t)lens[i] + b[i]->rd->n_base;
    // Layout: in = keys R Rm sct sctm sign txid base_value base_off base_tag base_tok cap_off
    //         out = value hole lastct lastct_mask count flags err_pos out_n out_tag out_tok
    size_t off = 0;
    auto slot = [&](size_t bytes) { size_t o = off; off = al(off + bytes); return o; };
    const size_t o_keys = slot(n * 8), o_R = slot(n * D * 8), o_Rm = slot(sparse ? n * W * 8 : 0),
                 o_sct = slot(any_sct ? n * D * 8 : 0),
                 o_sctm = slot(any_sct && sparse ? n * W * 8 : 0), o_sign = slot(any_sct ? n : 0),
                 o_txid = slot(n * 8), o_bv = slot(tags ? 0 : n * 8),
                 o_boff = slot(tags ? (n + 1) * 8 : 0), o_btag = slot(tags ? nb * 4 : 0),
                 o_btok = slot(tags ? nb * 8 : 0), o_cap = slot(tags ? (n + 1) * 8 : 0);
    const size_t in_bytes = off;
    const size_t o_val = slot(n * 8), o_hole = slot(n * 8), o_ct = slot(n * D * 8),
                 o_ctm = slot(sparse ? n * W * 8 : 0), o_cnt = slot(n * 4), o_flg = slot(n * 4),
                 o_epos = slot(n * 4), o_outn = slot(tags ? n * 4 : 0),
                 o_otag = slot(tags ? ncap * 4 : 0), o_otok = slot(tags ? ncap * 8 : 0);
    rc = grow(B, off);
    if (rc) return rc;
    char *h = B->hbuf, *d = B->dbuf;
    std::memset(h, 0, in_bytes);
    auto H = [&](size_t o) { return h + o; };
    uint64_t full[4] = {0, 0, 0, 0};
    for (uint32_t x = 0; x < D; ++x) full[x >> 6] |= 1ull << (x & 63);
    uint64_t bpos = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const agn_key_read *r = b[i]->rd;
        ((uint64_t *)H(o_keys))[i] = r->key;
        std::memcpy(H(o_R) + i * D * 8, r->R, D * 8);
        if (sparse) std::memcpy(H(o_Rm) + i * W * 8, r->R_mask ? r->R_mask : full, W * 8);
        if (any_sct) {
            if (r->sct) {
                std::memcpy(H(o_sct) + i * D * 8, r->sct, D * 8);
                if (sparse) std::memcpy(H(o_sctm) + i * W * 8, r->sct_mask ? r->sct_mask : full, W * 8);
            } else {
                ((uint8_t *)H(o_sign))[i] = 1;
            }
        }
        ((uint64_t *)H(o_txid))[i] = r->txid;
        if (tags) {
            ((uint64_t *)H(o_boff))[i] = bpos;
            if (r->n_base) {
                std::memcpy(H(o_btag) + bpos * 4, r->base_tag, r->n_base * 4);
                std::memcpy(H(o_btok) + bpos * 8, r->base_tok, r->n_base * 8);
            }
            bpos += r->n_base;
        } else {
            ((int64_t *)H(o_bv))[i] = r->base_value;
        }
    }
    if (tags) {
        ((uint64_t *)H(o_boff))[n] = bpos;
        uint64_t *co = (uint64_t *)H(o_cap);
        co[0] = 0;
        for (uint64_t i = 0; i < n; ++i) co[i + 1] = co[i] + lens[i] + b[i]->rd->n_base;
    }
    AGN_HIP(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, B->stream));

    agn_read req;
    std::memset(&req, 0, sizeof req);
    req.n_req = n;
    req.keys = (const uint64_t *)(d + o_keys);
    req.R = (const uint64_t *)(d + o_R);
    req.R_mask = sparse ? (const uint64_t *)(d + o_Rm) : nullptr;
    if (any_sct) {
        req.sct = (const uint64_t *)(d + o_sct);
        req.sct_mask = sparse ? (const uint64_t *)(d + o_sctm) : nullptr;
        req.sct_ignore = (const uint8_t *)(d + o_sign);
    }
    req.txid = (const uint64_t *)(d + o_txid);
    req.req_type = B->crdt;
    if (sparse) {
        // the batch's promises (agn_read.hints): every R mask carries all D
        // DCs, and LastOpCt masks over every column come back as a flag
        bool rfull = true;
        for (uint64_t i = 0; i < n && rfull; ++i) {
            const uint64_t *m = b[i]->rd->R_mask;
            for (uint32_t x = 0; m && x < W && rfull; ++x) rfull = (m[x] & full[x]) == full[x];
        }
        req.hints = AGN_HINT_CT_FLAG | (rfull ? AGN_HINT_R_FULL : 0u);
        if (!tags && many_mixed(n_mixed, n)) req.hints |= AGN_HINT_MIXED;
    }
    if (tags) {
        req.base_off = (const uint64_t *)(d + o_boff);
        req.base_tag = (const uint32_t *)(d + o_btag);
        req.base_tok = (const uint64_t *)(d + o_btok);
    } else {
        req.base_value = (const int64_t *)(d + o_bv);
    }
    agn_result res;
    std::memset(&res, 0, sizeof res);
    res.value = (int64_t *)(d + o_val);
    res.hole = (int64_t *)(d + o_hole);
    res.lastct = (uint64_t *)(d + o_ct);
    res.lastct_mask = sparse ? (uint64_t *)(d + o_ctm) : nullptr;
    res.count = (uint32_t *)(d + o_cnt);
    res.flags = (uint32_t *)(d + o_flg);
    res.err_pos = (uint32_t *)(d + o_epos);
    if (tags) {
        res.out_off = (const uint64_t *)(d + o_cap);
        res.out_n = (uint32_t *)(d + o_outn);
        res.out_tag = (uint32_t *)(d + o_otag);
        res.out_tok = (uint64_t *)(d + o_otok);
    }
    agn_log view;
    oplog_view(B->log, &view);
    rc = agn_materialize(B->ctx, &view, &req, &res, B->stream);
    if (rc) return rc;
    AGN_HIP(hipMemcpyAsync(h + in_bytes, d + in_bytes, off - in_bytes, hipMemcpyDeviceToHost,
                           B->stream));
    rc = wait_batch(B);
    if (rc) return rc;
    for (uint64_t i = 0; i < n; ++i) {
        agn_key_result *o = b[i]->out;
        o->value = tags ? 0 : ((const int64_t *)H(o_val))[i];
        o->hole = ((const int64_t *)H(o_hole))[i];
        std::memcpy(o->lastct, H(o_ct) + i * D * 8, D * 8);
        o->count = ((const uint32_t *)H(o_cnt))[i];
        o->flags = ((const uint32_t *)H(o_flg))[i];
        const bool ct_full = (o->flags & AGN_F_CT_FULL) != 0u;  // AGN_HINT_CT_FLAG
        o->flags &= ~AGN_F_CT_FULL;
        if (o->lastct_mask)
            std::memcpy(o->lastct_mask, (sparse && !ct_full) ? H(o_ctm) + i * W * 8 : (char *)full,
                        W * 8);
        o->err_pos = ((const uint32_t *)H(o_epos))[i];
        o->status = 0;
        if (tags) {
            const uint32_t m = ((const uint32_t *)H(o_outn))[i];
            const uint64_t s = ((const uint64_t *)H(o_cap))[i];
            o->out_n = m;
            o->status = 0;
            if (m > o->out_cap) {
                b[i]->rc = AGN_ECAPACITY;
                std::snprintf(b[i]->err, sizeof b[i]->err, "batcher_read: %u pairs, out_cap %u", m,
                              o->out_cap);
                continue;
            }
            if (m) {
                std::memcpy(o->out_tag, H(o_otag) + s * 4, m * 4);
                std::memcpy(o->out_tok, H(o_otok) + s * 8, m * 8);
            }
        }
    }
    return errs_to_op_ids(B, view, b);
}

// agn_batcher_store: materialize_snapshot's store (:466-509) of a snapshot
// the caller materialized from get_from_snapshot_log's response (IsNewest =
// false: only a GC read stores it) -> internal_store_ss / insert_bigger /
// snapshot_insert_gc (:341-364, 513-563) on the device cache, then prune_ops
// of the key when the policy collects -- the same kernels a read's store runs.
int run_store(agn_batcher *B, const StoreReq &s) {
    const uint32_t D = B->D, W = B->W;
    const bool tags = B->crdt != AGN_COUNTER_PN;
    const bool msk = B->ss.clock_mask != nullptr;
    uint64_t key = s.key;
    uint32_t len = 0;
    size_t d_keys = 0, d_pr = 0;
    bool collect = false;
    {
        std::shared_lock<std::shared_mutex> hold;
        int rc = oplog_begin_read(B->log, B->stream, 1, &key, &len, hold);
        if (rc) return rc;
        if (tags) {
            rc = ensure_state_room(B, s.n_pairs);
            if (rc) return rc;
        }
        size_t off = 0;
        auto slot = [&](size_t bytes) { size_t o = off; off = al(off + bytes); return o; };
        const size_t o_first = slot(1), o_st = slot(1), o_gc = slot(1), o_ct = slot(D * 8),
                     o_ctm = slot(W * 8), o_hole = slot(8), o_val = slot(8), o_cnt = slot(4),
                     o_flg = slot(4), o_off = slot(16), o_n = slot(4),
                     o_tag = slot(std::max<uint32_t>(s.n_pairs, 1) * 4),
                     o_tok = slot(std::max<uint32_t>(s.n_pairs, 1) * 8), o_pr = slot(1);
        d_keys = 0;
        d_pr = al(8);
        rc = grow(B, std::max(off, d_pr + 1));
        if (rc) return rc;
        char *h = B->hbuf, *x = B->hdev;
        ((uint8_t *)(h + o_first))[0] = 0;            // a log response: not the newest
        ((uint8_t *)(h + o_st))[0] = AGN_SS_HIT;       // (anything but LOG)
        ((uint8_t *)(h + o_gc))[0] = (s.flags & AGN_READ_GC) ? 1 : 0;
        std::memcpy(h + o_ct, s.clock, D * 8);
        uint64_t full[4] = {0, 0, 0, 0};
        for (uint32_t c = 0; c < D; ++c) full[c >> 6] |= 1ull << (c & 63);
        std::memcpy(h + o_ctm, s.clock_mask ? s.clock_mask : full, W * 8);
        ((int64_t *)(h + o_hole))[0] = s.last_op;
        ((int64_t *)(h + o_val))[0] = s.value;
        ((uint32_t *)(h + o_cnt))[0] = s.count;
        ((uint32_t *)(h + o_flg))[0] = s.count ? AGN_F_NEWSS : 0u;
        ((uint64_t *)(h + o_off))[0] = 0;
        ((uint64_t *)(h + o_off))[1] = s.n_pairs;
        ((uint32_t *)(h + o_n))[0] = s.n_pairs;
        if (s.n_pairs) {
            std::memcpy(h + o_tag, s.tags, (size_t)s.n_pairs * 4);
            std::memcpy(h + o_tok, s.toks, (size_t)s.n_pairs * 8);
        }
        AGN_HIP(hipMemcpyAsync(B->dbuf + d_keys, &key, 8, hipMemcpyHostToDevice, B->stream));
        agn_result res;
        std::memset(&res, 0, sizeof res);
        res.lastct = (uint64_t *)(x + o_ct);
        res.lastct_mask = msk ? (uint64_t *)(x + o_ctm) : nullptr;
        res.hole = (int64_t *)(x + o_hole);
        res.value = (int64_t *)(x + o_val);
        res.count = (uint32_t *)(x + o_cnt);
        res.flags = (uint32_t *)(x + o_flg);
        if (tags) {
            res.out_off = (const uint64_t *)(x + o_off);
            res.out_n = (uint32_t *)(x + o_n);
            res.out_tag = (uint32_t *)(x + o_tag);
            res.out_tok = (uint64_t *)(x + o_tok);
        }
        agn_log view;
        oplog_view(B->log, &view);
        // no key_off: the store's op count is the log response's (> 0, the
        // caller's check, :469-475), not the device list's, which a GC may
        // have emptied
        rc = launch_ss_store_req(B->ss, nullptr, nullptr, 1,
                                 (const uint64_t *)(B->dbuf + d_keys), (const uint8_t *)(x + o_first),
                                 (const uint8_t *)(x + o_st), (const uint8_t *)(x + o_gc), res,
                                 (uint8_t *)(B->dbuf + d_pr), B->thr, B->thrm, B->stream);
        if (rc) return rc;
        AGN_HIP(hipMemcpyAsync(h + o_pr, B->dbuf + d_pr, 1, hipMemcpyDeviceToHost, B->stream));
        if (tags)
            AGN_HIP(hipMemcpyAsync(B->ctl_h, B->ss.state_ctl, 4 * 8, hipMemcpyDeviceToHost,
                                   B->stream));
        rc = wait_batch(B);
        if (rc) return rc;
        if (tags && !B->ctl_h[2]) B->raise_bound(key, s.n_pairs);
        collect = ((const uint8_t *)(h + o_pr))[0] != 0;
    }  // the shared hold ends: the GC takes the log exclusively
    if (!collect) return AGN_OK;
    return oplog_prune_keys(B->log, 1, &key, (const uint64_t *)(B->dbuf + d_keys),
                            (const uint8_t *)(B->dbuf + d_pr), B->thr, B->thrm, B->stream);
}

void worker_main(agn_batcher *B) {
    (void)use_device(B->ctx);
    std::unique_lock<std::mutex> lk(B->mu);
    for (;;) {
        B->cv_work.wait(lk, [&] { return B->stop || !B->q.empty(); });
        if (B->q.empty()) break;  // stop requested and drained
        const auto deadline = B->q.front()->t + std::chrono::microseconds(B->max_wait_us);
        while (!B->stop && B->q.size() < B->max_batch && Clock::now() < deadline)
            B->cv_work.wait_until(lk, deadline);
        std::vector<Pending *> batch;
        if (!B->cached) {
            const size_t n = std::min<size_t>(B->q.size(), B->max_batch);
            batch.assign(B->q.begin(), B->q.begin() + n);
            B->q.erase(B->q.begin(), B->q.begin() + n);
        } else if (B->q.front()->st) {
            // a caller-computed snapshot (agn_batcher_store): alone, in order
            batch.push_back(B->q.front());
            B->q.pop_front();
        } else {
            // distinct keys, in arrival order; a repeated key waits for the next
            // batch, and nothing queued after a store joins this one
            std::unordered_set<uint64_t> in;
            std::deque<Pending *> rest;
            bool barrier = false;
            for (Pending *p : B->q) {
                barrier = barrier || p->st != nullptr;
                if (!barrier && batch.size() < B->max_batch && in.insert(p->rd->key).second)
                    batch.push_back(p);
                else
                    rest.push_back(p);
            }
            B->q.swap(rest);
        }
        const size_t n = batch[0]->st ? 0 : batch.size();
        lk.unlock();
        int rc = !B->cached        ? run_batch(B, batch)
                 : batch[0]->st ? run_store(B, *batch[0]->st)
                                : run_batch_cached(B, batch);
        if (rc)
            for (Pending *p : batch) {
                p->rc = rc;
                std::snprintf(p->err, sizeof p->err, "%s", agn_last_error());
            }
        B->n_batches.fetch_add(1, std::memory_order_relaxed);
        B->n_reads.fetch_add(n, std::memory_order_relaxed);
        lk.lock();
        for (Pending *p : batch) {
            p->done = true;
            p->cv.notify_one();
        }
    }
}

}  // namespace

extern "C" {

int agn_batcher_create(agn_oplog *log, uint32_t max_batch, uint32_t max_wait_us,
                       agn_batcher **out) {
    if (!out || !log) return fail(AGN_EINVAL, "batcher_create: null argument");
    *out = nullptr;
    if (max_batch == 0) return fail(AGN_EINVAL, "batcher_create: max_batch = 0");
    agn_batcher *B = new (std::nothrow) agn_batcher;
    if (!B) return fail(AGN_ENOMEM, "batcher_create");
    B->log = log;
    B->ctx = oplog_ctx(log);
    oplog_shape(log, &B->crdt, &B->D, &B->sparse_log, &B->K);
    B->W = n_words(B->D);
    B->max_batch = max_batch;
    B->max_wait_us = max_wait_us;
    int rc = use_device(B->ctx);
    if (rc == AGN_OK && hipStreamCreateWithFlags(&B->stream, hipStreamNonBlocking) != hipSuccess)
        rc = fail(AGN_EHIP, "batcher_create: stream");
    if (rc) {
        if (B->stream) (void)hipStreamDestroy(B->stream);
        delete B;
        return rc;
    }
    try {
        B->worker = std::thread(worker_main, B);
    } catch (...) {
        (void)hipStreamDestroy(B->stream);
        delete B;
        return fail(AGN_ENOMEM, "batcher_create: worker thread");
    }
    *out = B;
    return AGN_OK;
}

int agn_batcher_destroy(agn_batcher *B) {
    if (!B) return AGN_OK;
    {
        std::lock_guard<std::mutex> g(B->mu);
        B->stop = true;
    }
    B->cv_work.notify_all();
    if (B->worker.joinable()) B->worker.join();
    (void)use_device(B->ctx);
    if (B->stream) (void)hipStreamSynchronize(B->stream);
    if (B->dbuf) (void)hipFree(B->dbuf);
    if (B->hbuf) (void)hipHostFree(B->hbuf);
    for (void *p : {(void *)B->ss.n, (void *)B->ss.clock, (void *)B->ss.clock_mask,
                    (void *)B->ss.last_op, (void *)B->ss.value, (void *)B->thr, (void *)B->thrm,
                    (void *)B->ss.state_tag, (void *)B->ss.state_tok, (void *)B->ss.state_ctl})
        if (p) (void)hipFree(p);
    if (B->ctl_h) (void)hipHostFree(B->ctl_h);
    if (B->tscr) (void)hipFree(B->tscr);
    if (B->stream) (void)hipStreamDestroy(B->stream);
    delete B;
    return AGN_OK;
}

int agn_batcher_create_cached(agn_oplog *log, uint32_t slots, uint32_t max_batch,
                              uint32_t max_wait_us, agn_batcher **out) {
    if (!out || !log) return fail(AGN_EINVAL, "batcher_create_cached: null argument");
    *out = nullptr;
    uint32_t crdt, D;
    int sparse;
    uint64_t K;
    oplog_shape(log, &crdt, &D, &sparse, &K);
    if (slots == 0) slots = AGN_SNAPSHOT_THRESHOLD;
    if (slots < AGN_SNAPSHOT_THRESHOLD - 1)
        return fail(AGN_EINVAL, "batcher_create_cached: slots %u < %d", slots,
                    AGN_SNAPSHOT_THRESHOLD - 1);
    int rc = use_device(oplog_ctx(log));
    if (rc) return rc;
    const uint32_t W = n_words(D);
    const uint64_t K1 = std::max<uint64_t>(K, 1);
    agn_ss_cache c{};
    c.n_dcs = D;
    c.slots = slots;
    c.n_keys = K;
    uint64_t *thr = nullptr, *thrm = nullptr;
    hipError_t e = hipMalloc((void **)&c.n, K1 * 4);
    if (e == hipSuccess) e = hipMemset(c.n, 0, K1 * 4);
    if (e == hipSuccess) e = hipMalloc((void **)&c.clock, K1 * slots * D * 8);
    if (e == hipSuccess && sparse) e = hipMalloc((void **)&c.clock_mask, K1 * slots * W * 8);
    if (e == hipSuccess) e = hipMalloc((void **)&c.last_op, K1 * slots * 8);
    if (e == hipSuccess) e = hipMalloc((void **)&c.value, K1 * slots * 8);
    if (e == hipSuccess) e = hipMalloc((void **)&thr, K1 * D * 8);
    if (e == hipSuccess && sparse) e = hipMalloc((void **)&thrm, K1 * W * 8);
    // set_aw / register_mv: the snapshots' states live in a device arena
    // (16 pairs per key to start; re-packed / grown between batches)
    uint64_t *ctl_h = nullptr;
    if (crdt != AGN_COUNTER_PN) {
        c.state_cap = std::max<uint64_t>(16 * K1, 1u << 16);
        // test knob: a small first arena, so re-packs and growth happen early
        const char *ai = AGN_KNOB("AGN_SS_ARENA_INIT");
        if (ai && std::strtoull(ai, nullptr, 10) > 0) c.state_cap = std::strtoull(ai, nullptr, 10);
        if (e == hipSuccess) e = hipMalloc((void **)&c.state_tag, c.state_cap * 4);
        if (e == hipSuccess) e = hipMalloc((void **)&c.state_tok, c.state_cap * 8);
        if (e == hipSuccess) e = hipMalloc((void **)&c.state_ctl, 4 * 8);
        if (e == hipSuccess) e = hipMemset(c.state_ctl, 0, 4 * 8);
        if (e == hipSuccess) e = hipHostMalloc((void **)&ctl_h, 4 * 8, hipHostMallocDefault);
        if (e == hipSuccess) std::memset(ctl_h, 0, 4 * 8);
    }
    std::unique_ptr<std::atomic<uint32_t>[]> kb;  // set/register: per-key state bounds
    if (e == hipSuccess && crdt != AGN_COUNTER_PN) {
        kb.reset(new (std::nothrow) std::atomic<uint32_t>[K1]);
        if (!kb) e = hipErrorOutOfMemory;
        else for (uint64_t k = 0; k < K1; ++k) kb[k].store(0, std::memory_order_relaxed);
    }
    if (e == hipSuccess) rc = agn_batcher_create(log, max_batch, max_wait_us, out);
    if (e != hipSuccess || rc != AGN_OK) {
        for (void *p : {(void *)c.n, (void *)c.clock, (void *)c.clock_mask, (void *)c.last_op,
                        (void *)c.value, (void *)thr, (void *)thrm, (void *)c.state_tag,
                        (void *)c.state_tok, (void *)c.state_ctl})
            if (p) (void)hipFree(p);
        if (ctl_h) (void)hipHostFree(ctl_h);
        return e != hipSuccess ? fail(AGN_ENOMEM, "batcher_create_cached: snapshot cache") : rc;
    }
    // the worker only looks at `cached` under the queue lock, after a read arrives
    std::lock_guard<std::mutex> g((*out)->mu);
    (*out)->cached = true;
    const char *r6 = AGN_KNOB("AGN_READ6");
    (*out)->read6 = !(r6 && r6[0] == '0');
    const char *tf = AGN_KNOB("AGN_TAGS_FUSED");
    (*out)->tags_fused = !(tf && tf[0] == '0');
    (*out)->ss = c;
    (*out)->thr = thr;
    (*out)->thrm = thrm;
    (*out)->ctl_h = ctl_h;
    (*out)->kbound = std::move(kb);
    return AGN_OK;
}

int agn_batcher_read(agn_batcher *B, const agn_key_read *rd, agn_key_result *out) {
    if (!B || !rd || !out) return fail(AGN_EINVAL, "batcher_read: null argument");
    if (rd->key >= B->K) return fail(AGN_EINVAL, "batcher_read: key %llu >= n_keys",
                                     (unsigned long long)rd->key);
    if (!rd->R || !out->lastct) return fail(AGN_EINVAL, "batcher_read: R / lastct required");
    if (rd->flags & ~(uint32_t)AGN_READ_GC) return fail(AGN_EINVAL, "batcher_read: unknown flags");
    if (B->crdt != AGN_COUNTER_PN) {
        if (rd->n_base && (!rd->base_tag || !rd->base_tok))
            return fail(AGN_EINVAL, "batcher_read: base pairs missing");
        if (out->out_cap && (!out->out_tag || !out->out_tok))
            return fail(AGN_EINVAL, "batcher_read: out_tag / out_tok missing");
    }
    Pending p;
    p.rd = rd;
    p.out = out;
    p.t = Clock::now();
    std::unique_lock<std::mutex> lk(B->mu);
    if (B->stop) return fail(AGN_EINVAL, "batcher_read: batcher is shutting down");
    B->q.push_back(&p);
    if (B->q.size() == 1 || B->q.size() >= B->max_batch) B->cv_work.notify_one();
    p.cv.wait(lk, [&] { return p.done; });
    if (p.rc) return fail(p.rc, "%s", p.err);
    return AGN_OK;
}

int agn_batcher_store(agn_batcher *B, uint64_t key, const uint64_t *clock,
                      const uint64_t *clock_mask, int64_t last_op, uint32_t count, int64_t value,
                      uint32_t n_pairs, const uint32_t *tags, const uint64_t *toks, uint32_t flags) {
    if (!B || !clock) return fail(AGN_EINVAL, "batcher_store: null argument");
    if (!B->cached) return fail(AGN_EINVAL, "batcher_store: the batcher has no snapshot cache");
    if (key >= B->K) return fail(AGN_EINVAL, "batcher_store: key %llu >= n_keys",
                                 (unsigned long long)key);
    if (flags & ~(uint32_t)AGN_READ_GC) return fail(AGN_EINVAL, "batcher_store: unknown flags");
    if (B->crdt == AGN_COUNTER_PN ? n_pairs != 0 : (n_pairs && (!tags || !toks)))
        return fail(AGN_EINVAL, "batcher_store: state pairs do not match the type");
    if (n_pairs > AGN_SS_STATE_MAX_PAIRS) return fail(AGN_ECAPACITY, "batcher_store: %u pairs", n_pairs);
    StoreReq s{key, clock, clock_mask, last_op, value, count, n_pairs, flags, tags, toks};
    Pending p;
    p.rd = nullptr;
    p.st = &s;
    p.t = Clock::now();
    std::unique_lock<std::mutex> lk(B->mu);
    if (B->stop) return fail(AGN_EINVAL, "batcher_store: batcher is shutting down");
    B->q.push_back(&p);
    B->cv_work.notify_one();
    p.cv.wait(lk, [&] { return p.done; });
    if (p.rc) return fail(p.rc, "%s", p.err);
    return AGN_OK;
}

int agn_batcher_state_bound(agn_batcher *B, uint64_t key, uint32_t *pairs) {
    if (!B || !pairs) return fail(AGN_EINVAL, "batcher_state_bound: null argument");
    if (key >= B->K) return fail(AGN_EINVAL, "batcher_state_bound: key %llu >= n_keys",
                                 (unsigned long long)key);
    *pairs = B->kbound ? B->bound_of(key) : 0u;
    return AGN_OK;
}

int agn_batcher_stats(agn_batcher *B, uint64_t *batches, uint64_t *reads) {
    if (!B) return fail(AGN_EINVAL, "batcher_stats: null batcher");
    if (batches) *batches = B->n_batches.load();
    if (reads) *reads = B->n_reads.load();
    return AGN_OK;
}

}  // extern "C"
