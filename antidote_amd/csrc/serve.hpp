// serve.hpp -- internals shared by the read batcher (batcher.hip), the op
// log (oplog.hip), the snapshot cache (cache.hip) and the GC kernel (gc.hip)
// for the cached read/6 path.  Kept out of common.hpp, which the streaming
// kernels include.
#pragma once
#include "common.hpp"

namespace agn {

// agn_ss_store with the prune flags per request (prune_req[n_req], every
// request written; no per-key array to clear).
int launch_ss_store_req(const agn_ss_cache &c, const uint64_t *key_off, const uint64_t *key_len,
                        uint64_t n_req, const uint64_t *keys, const uint8_t *is_first,
                        const uint8_t *status, const uint8_t *should_gc, const agn_result &res,
                        uint8_t *prune_req, uint64_t *thr, uint64_t *thrm, hipStream_t st);

// agn_ss_state_compact's kernel: the live states into new_tag / new_tok
// (state_ctl reset, then the live pairs; *ovf = 1 if they do not fit).  The
// slots' rewritten references go to c.value, or -- new_value given, [n_keys
// * slots] -- there, for the caller to commit only when *ovf stayed 0.
int launch_ss_compact(const agn_ss_cache &c, uint32_t *new_tag, uint64_t *new_tok, uint64_t new_cap,
                      uint64_t *ovf, hipStream_t st, int64_t *new_value = nullptr);

// prune_ops in place over a key list (entry i: key keys[i], GC'd iff
// flags[i] != 0); meta[6][n] per entry.
int launch_prune_keys(const agn_log &view, uint64_t *key_len, uint32_t *key_id0,
                      uint32_t *key_lcap, uint64_t n, const uint64_t *keys, const uint8_t *flags,
                      const uint64_t *thr, const uint64_t *thr_mask, uint32_t *meta,
                      hipStream_t st);

// agn_oplog_prune over a key list: h_keys (host) / d_keys, d_flags (device,
// stream-ordered on `st`) name n distinct keys; only those keys' segments are
// visited and only their host metadata is settled.  Asynchronous like
// agn_oplog_prune (the next call on the log waits for it).
int oplog_prune_keys(agn_oplog *L, uint64_t n, const uint64_t *h_keys, const uint64_t *d_keys,
                     const uint8_t *d_flags, const uint64_t *thr, const uint64_t *thr_mask,
                     hipStream_t st);

}  // namespace agn

namespace agn {

// The fused cached read (read6.hip): one kernel per batch runs the whole of
// materializer_vnode:read/6 for counter_pn with dense clocks (D <= 8).
// Requests in and results out live in pinned host memory the kernel reads
// and writes directly (no copy operations); the batch's keys and prune flags
// are also written to device memory for the stream-ordered GC that follows.
struct Read6Args {
    // the partition's log (device view)
    const uint64_t *key_off, *key_len;
    const uint32_t *key_id0;
    const uint8_t *key_type;
    const uint64_t *oc;
    const uint32_t *op_id;
    const int64_t *eff;
    const uint64_t *log_txid;
    uint64_t n_entries;  // entry slots of the log (quad-row loads are clamped below)
    uint32_t n_dcs, req_type;
    // the batch (device-visible pinned host memory)
    uint64_t n_req;
    const uint64_t *keys, *R, *txid;
    const uint8_t *gc;
    int64_t *value, *hole;
    uint64_t *lastct;
    uint32_t *count, *flags, *err_pos;
    uint8_t *status, *prune;
    // device: the batch's keys and prune flags again (the batcher's GC list;
    // either may be null when the caller has no GC list), and the GC
    // thresholds [K][D]
    uint64_t *dkeys;
    uint8_t *dprune;
    uint64_t *thr;
    // presence masks (D <= 8: one word per clock; all null = dense): the
    // log's key_mask / oc_mask, the requests' R_mask, and the results'
    // LastOpCt mask and the GC thresholds' [K] masks (with a cache that
    // carries clock_mask)
    const uint64_t *key_mask, *oc_mask, *R_mask;
    uint64_t *lastct_mask, *thrm;
    // D = 9 .. 64 (k_read6w): device scratch of the batch -- the lookup's SCT
    // rows [n][D] and mask words [n], its ignore bytes [n], and the LastOpCt
    // rows [n][D] / mask words [n] the store reads back
    uint64_t *sct_scr, *sctm_scr, *ct_scr, *ctm_scr;
    uint8_t *ign_scr;
};
// agn_read_cached's fused path: dense logs (its cache has no clock masks)
bool read6_supported(const agn_log &view, uint32_t D);
int launch_read6(const agn_ss_cache &c, const Read6Args &a, hipStream_t st);

}  // namespace agn
