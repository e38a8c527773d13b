/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of AntidoteDB's materialization path, used as the parity
 * checker for the HIP engine.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product library never links
 * it (antidote_amd fails loudly instead of falling back to it).
 *
 * Parity is pinned against the reference's own EUnit known answers,
 * transcribed to tests/golden/kats.json (see tests/test_oracle_kats.py).
 * set_aw / register_mv concurrency semantics are only partially pinned
 * (antidote_crdt 0.1.2 is not vendored in the reference).
 */
#ifndef AGN_ORACLE_H
#define AGN_ORACLE_H

#include "../include/antidote_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* clocksi_materializer:materialize/4 for every request (host pointers). */
int oracle_materialize(const agn_log *log, const agn_read *req, agn_result *out,
                       int n_threads);

/* stable_time_functions:get_min_time/1 over [n_epochs][P][D] -> [n_epochs][D+1]
 * (same encoding as agn_gst_min), followed by the finalize rule. */
int oracle_gst_min(uint32_t n_dcs, uint64_t n_parts, uint64_t n_epochs,
                   const uint64_t *clocks, const uint8_t *defined, uint64_t *out,
                   int finalize);

/* meta_data_sender:update_stable/3 */
int oracle_update_stable(uint32_t n_dcs, uint64_t *last, const uint64_t *new_,
                         int *changed);

/* vector_orddict:get_smaller/2 */
int oracle_select_base(uint32_t n_dcs, uint64_t n_req, const uint64_t *cache_off,
                       const uint64_t *clocks, const uint64_t *clock_mask,
                       const uint64_t *R, const uint64_t *R_mask,
                       int32_t *out_idx, uint8_t *out_is_first);

/* logging_vnode filter_terms_for_key / handle_commit over decoded records
 * (host arrays), same contract as agn_log_ingest (out arrays sized >= the
 * update count; out->n_entries is set). */
int oracle_log_ingest(const agn_log_records *recs, uint32_t crdt_type, uint32_t n_dcs,
                      uint64_t n_keys, const uint64_t *max_time, const uint64_t *max_time_mask,
                      uint32_t op_id_base, agn_log *out);

/* materializer_vnode snapshot cache (host arrays), same contracts as
 * agn_ss_lookup / agn_ss_store. */
int oracle_ss_lookup(agn_ss_cache *cache, uint64_t n_req, const uint64_t *keys, const uint64_t *R,
                     const uint64_t *R_mask, uint64_t *sct, uint64_t *sct_mask, uint8_t *sct_ignore,
                     int64_t *base_value, uint8_t *is_first, uint8_t *status);
int oracle_ss_store(agn_ss_cache *cache, const agn_log *log, uint64_t n_req, const uint64_t *keys,
                    const uint8_t *is_first, const uint8_t *status, const uint8_t *should_gc,
                    const agn_result *res, const int64_t *handle, uint8_t *prune,
                    uint64_t *threshold, uint64_t *threshold_mask);

/* materializer_vnode prune_ops/check_filter over the SoA log (host arrays),
 * same contract as agn_prune_ops (out arrays sized like the input). */
int oracle_prune_ops(const agn_log *log, const uint8_t *prune, const uint64_t *threshold,
                     const uint64_t *threshold_mask, agn_log *out, uint32_t *out_flags);

/* dc_utilities gentlerain GST (get_scalar_stable_time/0), same encoding as
 * agn_gst_scalar. */
int oracle_gst_scalar(uint32_t n_dcs, uint64_t n_epochs, uint64_t *vec, uint64_t *out_gst);

/* inter_dc_dep_vnode:try_store/2 dependency check, same encoding as agn_dep_check. */
int oracle_dep_check(uint32_t n_dcs, uint64_t n_txn, const uint64_t *deps,
                     const uint64_t *deps_mask, const uint32_t *origin, const uint32_t *part,
                     uint64_t n_parts, const uint64_t *part_clock, const uint64_t *part_mask,
                     uint8_t *out_ok);

/* vectorclock 0.1.0 predicates on single clocks (missing entry = 0). */
int oracle_vc_le(uint32_t n_dcs, const uint64_t *a, const uint64_t *am,
                 const uint64_t *b, const uint64_t *bm);
int oracle_vc_all_dots_greater(uint32_t n_dcs, const uint64_t *a, const uint64_t *am,
                               const uint64_t *b, const uint64_t *bm);

#ifdef __cplusplus
}
#endif
#endif
