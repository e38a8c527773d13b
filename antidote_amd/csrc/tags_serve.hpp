// tags_serve.hpp -- the fused set_aw / register_mv cached read (mat_tags.hip,
// k_tags with SV), shared with the read batcher (batcher.hip) and the
// snapshot cache (cache.hip).
//
// Per request, one wave runs get_from_snapshot_cache (the lookup writes the
// SCT row and the base state's arena reference below, which the agn_read of
// the launch names as its sct / sct_mask / sct_ignore / base_value), the fast
// tags pass from that base, and materialize_snapshot's store of the result
// (the state read from the wave's LDS table, LastOpCt from LDS).  A request
// whose state overflows the fast table, or whose key is not uniform inside
// R's DC set (presence masks), is handed on (prune[i] = 4) and finished by
// launch_tags_serve_rest: the remaining tags passes over the scratch lists,
// then the store over the same lists.
#pragma once
#include "common.hpp"

namespace agn {

struct TagServe {
    agn_ss_cache c;
    uint64_t *sct, *sctm;  // device [n][D], [n][W] (sctm: masked batches)
    uint8_t *ign, *first;  // device [n]
    int64_t *base;         // device [n]: AGN_SS_STATE into c's arena
    uint8_t *status;       // [n] AGN_SS_*
    const uint8_t *gc;     // [n] op_insert_gc's GC read
    uint8_t *prune;        // [n] bit 0: GC the key, bit 1: arena overflow, 4: handed on
    uint64_t *delta;       // [n][2] pairs the store added to state_ctl[0] / [1]
    uint64_t *dkeys;       // device [n] the batch's keys (the GC list)
    uint8_t *dprune;       // device [n] the prune flags (bit 0)
    uint64_t *thr, *thrm;  // GC thresholds [K][D], [K][W]
};

// Fused shapes: D <= 8, dense rows or presence masks.
bool tags_serve_supported(const agn_log &log, bool sparse);
// scr: 3 n + 4 words, the first 4 zero on entry (and again after _rest).
int launch_tags_serve(const agn_log &log, const agn_read &req, const agn_result &out,
                      const TagServe &sv, uint32_t *scr, hipStream_t st);
int launch_tags_serve_rest(const agn_log &log, const agn_read &req, const agn_result &out,
                           const TagServe &sv, uint32_t *scr, hipStream_t st);

// agn_ss_store (prune flags per request) over a device list of request
// indices list[0, *list_n) (cache.hip).
int launch_ss_store_list(const agn_ss_cache &c, const uint64_t *key_off, const uint64_t *key_len,
                         uint64_t n_req, const uint32_t *list, const uint32_t *list_n,
                         const uint64_t *keys, const uint8_t *is_first, const uint8_t *status,
                         const uint8_t *should_gc, const agn_result &res, uint8_t *prune_req,
                         uint64_t *thr, uint64_t *thrm, hipStream_t st);

}  // namespace agn
