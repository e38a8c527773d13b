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

// prune_ops in place over a key list (entry i: key keys[i], GC'd iff
// flags[i] != 0); meta[4][n] per entry.
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
