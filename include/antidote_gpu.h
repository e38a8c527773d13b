/*
 * antidote_gpu.h — C ABI of the MI355X snapshot-materialization engine.
 *
 * This is the drop-in boundary for AntidoteDB's materialization hot path.
 * Each entry point names the reference interface it replaces
 * (paths relative to the AntidoteDB tree, snapshot 2025-01-12).  The Erlang
 * side binds these through the thin NIF in nif/antidote_gpu_nif.c (see
 * INTEGRATION.md); every test in this repository drives them directly.
 *
 * Conventions
 *   - plain C, no torch / HIP types in the signatures (streams are void*);
 *   - every function returns int: AGN_OK (0) or a negative AGN_E* code, and
 *     agn_last_error() returns a per-thread message for the last failure;
 *   - "dev" pointers live in HBM (hipMalloc / agn_dev_alloc / torch), "host"
 *     pointers in ordinary memory;
 *   - the library is thread-safe: a context serialises nothing but its own
 *     RCCL communicator, so many reader threads (the reference's 20 read
 *     servers per partition, include/antidote.hrl:28) may call
 *     agn_materialize concurrently on different streams.
 *
 * Data model (the SoA "device op log", mirroring the per-key ETS ops tuple of
 * src/materializer_vnode.erl:621-647 and include/antidote.hrl:81-90):
 *   - a log holds n_keys keys; key k owns entries [key_off[k], key_off[k+1])
 *     stored OLDEST -> NEWEST (tuple slot ?FIRST_OP is the oldest op) — or,
 *     when key_len is given, [key_off[k], key_off[k] + key_len[k]): segments
 *     with slack capacity, like the ETS tuple's Length / ListLen (the
 *     engine-owned agn_oplog below);
 *   - vector clocks are dense rows of n_dcs u64 words (DC index = column) with
 *     an optional presence bitmask of W = ceil(n_dcs/64) words per clock; a
 *     NULL mask means "every DC present" (the dense fast path);
 *   - oc[e] is the op's OpSSCommit: its snapshot_time with the commit DC's
 *     entry replaced by the commit time (src/clocksi_materializer.erl:224,
 *     src/materializer.erl:105) — computed once at ingest;
 *   - an op whose effect has several parts (set_aw add_all) occupies several
 *     consecutive entries with the same op_id.
 */
#ifndef ANTIDOTE_GPU_H
#define ANTIDOTE_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AGN_ABI_VERSION 6

/* ---- status codes ------------------------------------------------------ */
#define AGN_OK 0
#define AGN_EINVAL (-1)     /* malformed argument (enif_make_badarg in the NIF) */
#define AGN_EHIP (-2)       /* HIP runtime error */
#define AGN_ENOMEM (-3)     /* device or host allocation failed */
#define AGN_ECAPACITY (-4)  /* a per-key table exceeded its device capacity */
#define AGN_ENOTSUP (-5)    /* unsupported configuration */
#define AGN_ERCCL (-6)      /* RCCL error */
#define AGN_ENODEV (-7)     /* no GPU / library built without device code */

/* ---- CRDT types (antidote_crdt 0.1.2, rebar.lock:3) --------------------- */
#define AGN_COUNTER_PN 1   /* antidote_crdt_counter_pn */
#define AGN_SET_AW 2       /* antidote_crdt_set_aw     */
#define AGN_REGISTER_MV 3  /* antidote_crdt_register_mv */
#define AGN_TYPE_MIXED 0xFF /* key_type marker: the key's ops have different types */

/* counter_pn effect that the Erlang side could not encode as an i64: applying
 * it yields {error,{unexpected_operation,Op,Type}} (src/materializer.erl:53-58) */
#define AGN_EFFECT_INVALID INT64_MIN
/* set_aw / register_mv entry whose effect could not be encoded */
#define AGN_TAG_INVALID 0xFFFFFFFFu

/* ---- per-key result flags --------------------------------------------- */
#define AGN_F_NEWSS 0x1u          /* IsNewSS: at least one op was included       */
#define AGN_F_CT_IGNORE 0x2u      /* LastOpCt == ignore (nothing included, SCT ignore) */
#define AGN_F_ERR_UNEXPECTED 0x4u /* {error,{unexpected_operation,Op,Type}}      */
#define AGN_F_ERR_CORRUPTED 0x8u  /* erlang:error(corrupted_ops_cache)           */
#define AGN_F_ERR_CAPACITY 0x10u  /* a per-key device table overflowed            */
/* ABI v5: LastOpCt carries every column of the partition (its dict has all n_dcs
 * DCs); set only for requests of a batch with AGN_HINT_CT_FLAG, and then
 * lastct_mask[i] is NOT written (the mask is the n_dcs low bits) */
#define AGN_F_CT_FULL 0x20u

/* ---- op log (device or host pointers, same layout) -------------------- */
typedef struct agn_log {
    uint32_t crdt_type;       /* AGN_COUNTER_PN / AGN_SET_AW / AGN_REGISTER_MV */
    uint32_t n_dcs;           /* D: vector-clock width */
    uint64_t n_keys;
    uint64_t n_entries;
    const uint64_t *key_off;  /* [n_keys+1] CSR, or segment starts when key_len != NULL */
    const uint64_t *key_len;  /* [n_keys] entries in use per segment, or NULL (CSR) */
    const uint8_t *key_type;  /* [n_keys] type of the key's ops or AGN_TYPE_MIXED; NULL: all crdt_type;
                                 4-byte aligned (AGN_EINVAL otherwise) */
    const uint64_t *oc;       /* [n_entries * D] OpSSCommit */
    const uint64_t *oc_mask;  /* [n_entries * W] presence, NULL = dense */
    const uint32_t *op_id;    /* [n_entries] per-key op number (ets update_counter, :630) */
    const uint64_t *txid;     /* [n_entries] writer txid (0 = none) or NULL */
    /* AGN_COUNTER_PN */
    const int64_t *eff;       /* [n_entries] effect = signed increment */
    /* AGN_SET_AW: entry = {Elem, AddTokens, RemoveTokens};
     * AGN_REGISTER_MV: entry = {Value, Token, Overridden} or {reset, Overridden} */
    const uint32_t *tag;      /* [n_entries] elem id (set) / value id (register) */
    const uint64_t *add_tok;  /* [n_entries] token added (0 = none: remove / reset) */
    const uint32_t *rem_off;  /* [n_entries+1] CSR into rem_tok (with key_len: contiguous
                                 within a key, rem_off[key_off[k]+key_len[k]] = end) */
    const uint64_t *rem_tok;  /* removed (set) / overridden (register) tokens */
    /* ABI v3, optional (NULL = read op_id): per key, the op id of the segment's
     * first entry when its ids are consecutive (op_id[off+p] == key_id0 + p
     * for every p < len), else AGN_ID0_NONE.  Ids stay consecutive from
     * op_insert_gc's ets:update_counter (src/materializer_vnode.erl:630) until
     * a GC prune leaves gaps (:576-585); built by agn_log_index_ids.  Lets the
     * counter kernel derive NewLastOp without a dependent op_id load. */
    const uint32_t *key_id0;
    /* ABI v4, optional (NULL = look at the per-entry masks only; D <= 64): per
     * key, the presence word that EVERY entry of its segment carries
     * (oc_mask[e] & low D bits, the same for all e of the key), or 0 when the
     * key's entries differ (or it is not known).  A dict clock carries the
     * DCs the DC knew of when it was taken (include/antidote.hrl:188), so in a
     * steady deployment every op of a key has the same DC set U.  When U is a
     * subset of the read snapshot's DCs, is_op_in_snapshot's dict fold
     * (src/clocksi_materializer.erl:236-258) is a plain element-wise compare
     * over U's columns, and LastOpCt's DC set is SCT's united with U when
     * any op was included -- so the dense row-scan kernels serve the key
     * exactly, without reading a mask per op.  Built by agn_log_index_masks;
     * maintained by the engine-owned agn_oplog. */
    const uint64_t *key_mask;
} agn_log;

#define AGN_ID0_NONE 0xFFFFFFFFu

/* ---- a batch of reads: one materialize/4 per requested key ------------- */
typedef struct agn_read {
    uint64_t n_req;
    const uint64_t *keys;       /* [n_req] key index into the log, NULL = identity (n_req == n_keys) */
    const uint64_t *R;          /* [n_req * D] MinSnapshotTime (read snapshot) */
    const uint64_t *R_mask;     /* [n_req * W] or NULL (dense) */
    const uint64_t *sct;        /* [n_req * D] SnapshotCommitTime of the base snapshot, NULL = all ignore */
    const uint64_t *sct_mask;   /* [n_req * W] or NULL */
    const uint8_t *sct_ignore;  /* [n_req] 1 = ignore (with sct != NULL), NULL = none ignored;
                                   4-byte aligned (AGN_EINVAL otherwise) */
    const uint64_t *txid;       /* [n_req] reading TxId (0 = ignore) or NULL = all ignore */
    uint32_t req_type;          /* Type argument of materialize/4 */
    uint32_t hints;             /* ABI v5 (was padding; 0 = none): AGN_HINT_* promises
                                   about this batch that let a kernel skip loads /
                                   stores of presence words */
    /* base snapshot value (#materialized_snapshot.value) */
    const int64_t *base_value;  /* counter: [n_req] or NULL (= 0, Type:new());
                                   set/register with base_off NULL: [n_req]
                                   AGN_SS_STATE(start, pairs) references into
                                   base_tag / base_tok (a cache's state arena,
                                   as agn_ss_lookup writes them; both arrays
                                   required, else AGN_EINVAL).  Device memory
                                   for the device calls; host memory for the
                                   host helpers agn_state_capacity and
                                   agn_materialize_host, which read the pair
                                   counts out of the references */
    const uint64_t *base_off;   /* set/register: CSR [n_req+1] or NULL (= empty) */
    const uint32_t *base_tag;   /* set: elem, register: value */
    const uint64_t *base_tok;   /* token */
} agn_read;

/* agn_read.hints.  AGN_HINT_R_FULL: every R_mask[i] carries all n_dcs DCs (the
 * caller checked; the masks are then not read).  AGN_HINT_CT_FLAG: the caller
 * reads lastct_mask through AGN_F_CT_FULL (a request whose LastOpCt carries
 * every column gets the flag instead of its mask word; see agn_result).  The
 * read batcher sets both from the requests it packs.  AGN_HINT_MIXED: many of
 * the batch's keys carry entries with different DC sets (agn_log.key_mask 0,
 * e.g. soon after a DC joined): the counter kernel scans them in the same
 * pass instead of handing them on to a second one (which re-reads them).
 * Kernels may ignore a hint (then the mask is loaded / written as without
 * it); no hint changes a result. */
#define AGN_HINT_R_FULL 0x1u
#define AGN_HINT_CT_FLAG 0x2u
#define AGN_HINT_MIXED 0x4u

/* ---- results ----------------------------------------------------------- */
typedef struct agn_result {
    int64_t *value;           /* counter: [n_req] materialized value */
    int64_t *hole;            /* [n_req] NewLastOp (1 - id of the oldest excluded op) */
    uint64_t *lastct;         /* [n_req * D] LastOpCt */
    uint64_t *lastct_mask;    /* [n_req * W] or NULL when inputs are dense; with
                                 AGN_HINT_CT_FLAG not written for a request whose
                                 flags carry AGN_F_CT_FULL */
    uint32_t *count;          /* [n_req] number of effects applied */
    uint32_t *flags;          /* [n_req] AGN_F_* */
    uint32_t *err_pos;        /* [n_req] entry index (global) of the failing op, or UINT32_MAX */
    /* set/register state: pairs written at [out_off[i], out_off[i] + out_n[i]) */
    const uint64_t *out_off;  /* [n_req+1] capacity CSR (input; see agn_state_capacity) */
    uint32_t *out_n;          /* [n_req] live pairs */
    uint32_t *out_tag;        /* elem / value */
    uint64_t *out_tok;        /* token */
} agn_result;

/* ---- context ------------------------------------------------------------ */
typedef struct agn_ctx agn_ctx;

int agn_abi_version(void);
const char *agn_last_error(void);
const char *agn_strerror(int code);
/* The library reads its AGN_* environment knobs (A/B switches, test hooks)
 * once and caches them; after changing one in a running process, call this
 * so the next launch sees it.  Not part of the reference's API. */
int agn_env_reload(void);

/* Open a context on HIP device `device` (riak_core vnode start analogue:
 * src/materializer_vnode.erl:120-131). */
int agn_open(int device, agn_ctx **out);
int agn_close(agn_ctx *ctx);
int agn_device_count(int *out);
/* Stream-ordered scratch and op-log arenas come from the library's own
 * memory pool per device (not the device's default pool, so torch and other
 * hipMallocAsync users in the process are unaffected).  Freed blocks stay
 * cached in it for the next GC / ingest (environment AGN_POOL_KEEP = bytes to
 * keep, default unlimited); agn_pool_trim releases all but keep_bytes of the
 * cached memory back to the device (after synchronizing it), and closing the
 * last context of a device trims to 0.  Not part of the reference's API. */
int agn_pool_trim(agn_ctx *ctx, uint64_t keep_bytes);

/* Device memory helpers (for callers without their own allocator). */
int agn_dev_alloc(agn_ctx *ctx, size_t bytes, void **out);
int agn_dev_free(agn_ctx *ctx, void *ptr);
int agn_memcpy_h2d(agn_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream);
int agn_memcpy_d2h(agn_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream);
int agn_memset_d(agn_ctx *ctx, void *dst, int value, size_t bytes, void *stream);
int agn_stream_sync(agn_ctx *ctx, void *stream);

/* Batched clocksi_materializer:materialize/4 (src/clocksi_materializer.erl:82-101)
 * over a device-resident log: for each requested key, the VC snapshot filter
 * (materialize_intern/is_op_in_snapshot, :145-268) and the CRDT effect fold
 * (apply_operations, :111-121 -> antidote_crdt update/2).  All pointers are
 * device pointers; launched on `stream` (NULL = default stream), asynchronous.
 * Returns AGN_EINVAL for malformed descriptors. */
int agn_materialize(agn_ctx *ctx, const agn_log *log, const agn_read *req,
                    agn_result *out, void *stream);

/* Host-pointer convenience: copies log, request and result through a staged
 * device buffer and blocks.  This is what the NIF calls for a single
 * materialize/4 whose ops list arrives as an Erlang term. */
int agn_materialize_host(agn_ctx *ctx, const agn_log *log, const agn_read *req,
                         agn_result *out);

/* Kernel-variant selection for this process and device: runs the batch
 * (same arguments as agn_materialize) through each bit-identical kernel
 * variant its shape has, `rounds` launches per variant alternated on
 * `stream`, and selects the fastest for later agn_materialize calls of the
 * same path.  Today that is the dense counter_pn path with even D: VGPR row
 * loads vs non-temporal LDS-DMA rows (and, for D = 8, lane-contiguous "quad"
 * rows), whose order differs between MI355X boxes; the
 * environment variable AGN_COUNTER_VARIANT=0/1/2 (or AGN_COUNTER_GLDS=0/1)
 * overrides the selection.  Blocks until done; `out` then holds the batch's
 * results.  *choice: -1 = nothing to tune (the batch ran once), 0 = VGPR
 * rows, 1 = LDS-DMA rows, 2 = quad rows; ms (may be NULL) receives the
 * fastest launch of each variant in milliseconds ([3], 0 for a variant the
 * shape lacks).  Not part of the reference's API: an engine-setup call
 * (INTEGRATION.md), e.g. on the first batch of a partition. */
int agn_tune(agn_ctx *ctx, const agn_log *log, const agn_read *req, agn_result *out,
             void *stream, int rounds, int *choice, float *ms);

/* agn_log.key_id0 for a device log: out[k] = op_id[off_k] when the ids of
 * key k's segment are consecutive, else AGN_ID0_NONE (also for empty keys).
 * The caller owns out ([n_keys] u32, device) and sets log.key_id0 = out; the
 * index must be rebuilt whenever op ids change (append past a gap, prune). */
int agn_log_index_ids(agn_ctx *ctx, const agn_log *log, uint32_t *out, void *stream);

/* agn_log.key_mask for a device log with presence masks and D <= 64:
 * out[k] = the presence word all of key k's entries share (low D bits), or 0
 * when they differ or the key is empty.  The caller owns out ([n_keys] u64,
 * device) and sets log.key_mask = out; rebuild it when entries change.  A
 * log without oc_mask gets every key's full word (all D DCs present).
 * ABI v6: the call also counts the log's mixed keys (non-empty, entries with
 * different DC sets) and blocks until the index is built; the context keeps
 * the count with `out`, and agn_materialize over a log whose key_mask is
 * `out` (same n_keys) routes a counter batch by it as if AGN_HINT_MIXED
 * were passed when more than 1/16 of the log's keys are mixed. */
int agn_log_index_masks(agn_ctx *ctx, const agn_log *log, uint64_t *out, void *stream);

/* Upper bound of live pairs per request for set/register types:
 * writes cap_off[n_req+1] (host pointers): cap = #adding entries of the key
 * + #base pairs.  Host-side helper (the bound is static per log): every
 * array of host_log / host_req it reads -- key_off / key_len, the adding
 * flags, base_off, or base_value's AGN_SS_STATE references when base_off is
 * NULL -- must be host memory (copy a device agn_ss_lookup's base_value
 * back first). */
int agn_state_capacity(const agn_log *host_log, const agn_read *host_req,
                       uint64_t *cap_off);

/* ---- engine-owned op log: one per partition ------------------------------
 * The materializer_vnode ETS ops cache (ops_cache-<P>,
 * src/materializer_vnode.erl:284-286, 321-338) resident in HBM: per key a
 * segment of `cap` slots (the ETS tuple's ListLen: OPS_THRESHOLD = 50 slots
 * at first, doubling) holding its ops oldest first, plus the per-key op
 * counter of ets:update_counter (:630).  update/2 calls are staged on the
 * host and moved to HBM by agn_oplog_flush in one batched transfer + scatter
 * kernel (the micro-batch of a partition's writes); reads then run on the
 * flushed view.  Thread safety (SURVEY §8(b) Threading): one writer (the
 * vnode process: append / flush / prune) and any number of concurrent
 * readers through agn_oplog_read / agn_batcher; the engine holds the device
 * log shared for the duration of each read kernel and exclusive while a
 * flush or prune moves segments.  A view returned by agn_oplog_flush is for
 * single-threaded use and is invalidated by the next flush or prune.  Slots
 * are 32-bit: a log holds fewer than 2^32 entry slots (segments included;
 * e.g. ~370 GB of 8-DC entries, beyond one MI355X) and token slots; past
 * that, flush / prune return AGN_ENOTSUP. */
#define AGN_OPS_THRESHOLD 50 /* src/materializer_vnode.erl:41 */
#define AGN_RESIZE_THRESHOLD 5 /* :44 */
typedef struct agn_oplog agn_oplog;
/* init_slots: a key's first segment (0 = AGN_OPS_THRESHOLD, as :626). */
int agn_oplog_create(agn_ctx *ctx, uint32_t crdt_type, uint32_t n_dcs, uint64_t n_keys,
                     int sparse, uint32_t init_slots, agn_oplog **out);
int agn_oplog_destroy(agn_oplog *log);
/* materializer_vnode:update/2 -> op_insert_gc/3 for n log entries (host
 * arrays).  Entry i belongs to key keys[i]; same_op[i] = 1 (same_op may be
 * NULL) continues the previous entry's op (an effect with several parts,
 * e.g. set_aw add_all), which must be of the same key; every other entry
 * starts an op whose id is ++counter[key] (ets:update_counter(OpsCache, Key,
 * {3, 1}), :630), written to out_op_id[i] (may be NULL).  out_gc_due[i]
 * (may be NULL) = 1 where op_insert_gc would first run its GC read (:635:
 * Length >= ListLen or NewId rem OPS_THRESHOLD == 0, counted in entries
 * before this one is inserted); the engine grows the segment instead of
 * forcing it, the caller may run the GC read (agn_materialize +
 * agn_ss_store(should_gc) + agn_oplog_prune) when it sees the flag.  oc[n][D] is the
 * OpSSCommit row (+ oc_mask[n][W] for a sparse log), txid may be NULL, the
 * effect arrays are those of the log's type, rem_off[n+1] is a CSR into
 * rem_tok. */
int agn_oplog_append(agn_oplog *log, uint64_t n, const uint64_t *keys, const uint8_t *same_op,
                     const uint64_t *oc, const uint64_t *oc_mask, const uint64_t *txid,
                     const int64_t *eff, const uint32_t *tag, const uint64_t *add_tok,
                     const uint32_t *rem_off, const uint64_t *rem_tok, uint32_t *out_op_id,
                     uint8_t *out_gc_due);
/* Moves the staged appends to HBM (ordered on `stream`) and fills *view with
 * the device descriptor (key_off = segment starts, key_len) for
 * agn_materialize / agn_ss_store / agn_prune_ops. */
int agn_oplog_flush(agn_oplog *log, agn_log *view, void *stream);
/* GC of the resident log: snapshot_insert_gc's prune_ops for every key with
 * prune[k] != 0 (device arrays, e.g. from agn_ss_store), then the ETS resize
 * policy (:540-560: ListLen doubles when fewer than RESIZE_THRESHOLD slots
 * stay free, halves when that leaves room and stays above OPS_THRESHOLD;
 * prune_ops' NewLength counts 1 when nothing survives, :580-583).  One
 * in-place kernel on `stream` (unselected keys cost nothing); flushes first,
 * does not block: the new per-key lengths reach the host asynchronously and
 * every later call on this log (append, flush, read, stats) waits for them,
 * so reads on any stream see the pruned log.  When the arenas hold more than
 * twice the slots the keys want, the call first re-lays them out into fresh
 * arenas (allocating everything before changing anything; skipped if memory
 * is short).  out_flags (device, may be NULL) as agn_prune_ops.  prune
 * (device, [n_keys]) must be 4-byte aligned. */
int agn_oplog_prune(agn_oplog *log, const uint8_t *prune, const uint64_t *threshold,
                    const uint64_t *threshold_mask, uint32_t *out_flags, void *stream);
/* Host-side accounting: entries in use, allocated slots, removal tokens. */
int agn_oplog_stats(const agn_oplog *log, uint64_t *entries, uint64_t *slots, uint64_t *tokens);
/* Per key (host arrays, each may be NULL): its entries (staged included) =
 * the ETS tuple's Length, its ListLen (0 = never written; what op_insert_gc's
 * GC trigger and the resize policy see) and its op counter (element 3,
 * :630) -- the {Length, ListLen} / OpId of deconstruct_opscache_entry (:614). */
int agn_oplog_key_meta(agn_oplog *log, uint64_t n, const uint64_t *keys, uint32_t *out_len,
                       uint32_t *out_list_len, uint32_t *out_counter);
/* op_insert_gc's trigger for the NEXT op of each key (:635: Length >= ListLen
 * or NewId rem OPS_THRESHOLD == 0), before it is appended: the reference runs
 * the GC read first and inserts after it, so a caller that wants the ETS
 * list sizes to the slot calls this, runs the GC read (agn_batcher_read with
 * AGN_READ_GC, or agn_oplog_prune) when due, then agn_oplog_append.
 * (agn_oplog_append's out_gc_due reports the same condition, but the entry is
 * then already in the log.) */
int agn_oplog_gc_due(agn_oplog *log, uint64_t n, const uint64_t *keys, uint8_t *out_due);
/* Sets each key's op counter (element 3 of the ETS tuple, :630): the next
 * op appended to the key gets counter + 1.  For a caller that keeps one
 * counter per key across several logs -- the NIF's partition holds one log
 * per CRDT type where the reference keeps ONE tuple per key for every type
 * (:621-647) -- so op ids (and op_insert_gc's NewId rem OPS_THRESHOLD
 * trigger) follow the reference's single counter.  Ids may then have gaps in
 * one log (the consecutive-id index drops such keys by itself). */
int agn_oplog_set_counter(agn_oplog *log, uint64_t n, const uint64_t *keys,
                          const uint32_t *counter);
/* Batched materialize/4 over the oplog's current contents (req / out as
 * agn_materialize, device pointers, req->keys indexing the oplog's keys).
 * Staged appends are flushed first (read-your-writes: update/2 is a
 * sync_command that precedes the read); blocks until the kernel is done. */
int agn_oplog_read(agn_oplog *log, const agn_read *req, agn_result *out, void *stream);

/* ---- micro-batching read queue ------------------------------------------
 * materializer_vnode:read/6 arrives per key from up to 20 read servers per
 * partition (clocksi_readitem_server:return/6, src/clocksi_readitem_server.erl
 * :272; READ_CONCURRENCY, include/antidote.hrl:28).  An agn_batcher
 * coalesces those calls: agn_batcher_read blocks the calling thread until
 * its request has run in a batch of up to max_batch reads, launched when
 * max_batch reads wait or the oldest has waited max_wait_us.  One worker
 * thread and one HIP stream per batcher; any number of calling threads. */
typedef struct agn_batcher agn_batcher;
typedef struct agn_key_read { /* one read/6 (host pointers) */
    uint64_t key;
    const uint64_t *R;          /* [D] */
    const uint64_t *R_mask;     /* [W] or NULL (all DCs present) */
    const uint64_t *sct;        /* [D] base SnapshotCommitTime, NULL = ignore */
    const uint64_t *sct_mask;   /* [W] or NULL */
    uint64_t txid;              /* 0 = ignore */
    int64_t base_value;         /* counter_pn base */
    uint32_t n_base;            /* set/register base pairs */
    uint32_t flags;             /* AGN_READ_GC: op_insert_gc's GC read (ShouldGc = true,
                                   src/materializer_vnode.erl:640; cached mode) */
    const uint32_t *base_tag;
    const uint64_t *base_tok;
} agn_key_read;
#define AGN_READ_GC 0x1u
typedef struct agn_key_result { /* caller-owned host memory */
    int64_t value, hole;
    uint64_t *lastct;           /* [D] */
    uint64_t *lastct_mask;      /* [W] or NULL (then the batch must be dense) */
    uint32_t count, flags;
    uint32_t err_pos;           /* AGN_F_ERR_UNEXPECTED: the op id (agn_oplog_append's
                                   out_op_id) of the failing op -- the op whose effect
                                   {error,{unexpected_operation,Op,Type}} names -- else
                                   UINT32_MAX (ABI v5; was its slot in the log) */
    uint32_t out_cap;           /* set/register: room in out_tag / out_tok */
    uint32_t out_n;             /* live pairs (> out_cap => AGN_ECAPACITY) */
    uint32_t status;            /* cached mode: AGN_SS_HIT / AGN_SS_NEW, or AGN_SS_LOG (no
                                   cached snapshot <= R: the caller reads the log,
                                   get_from_snapshot_log :416-419; the result is void) */
    uint32_t *out_tag;
    uint64_t *out_tok;
} agn_key_result;
int agn_batcher_create(agn_oplog *log, uint32_t max_batch, uint32_t max_wait_us,
                       agn_batcher **out);
int agn_batcher_destroy(agn_batcher *b);
int agn_batcher_read(agn_batcher *b, const agn_key_read *rd, agn_key_result *out);
int agn_batcher_stats(agn_batcher *b, uint64_t *batches, uint64_t *reads);
/* Cached mode (counter_pn): the batcher also owns the partition's device
 * snapshot cache (an agn_ss_cache of n_keys x slots, 0 = SNAPSHOT_THRESHOLD)
 * and serves each batch as the whole of materializer_vnode:read/6
 * (:96-102, 371-509): get_from_snapshot_cache (agn_ss_lookup) -> materialize/4
 * from the cached base -> internal_store_ss / snapshot_insert_gc
 * (agn_ss_store; AGN_READ_GC in agn_key_read.flags forces the GC as
 * op_insert_gc's GC read does) -> prune_ops of the selected keys
 * (agn_oplog_prune, in place).  agn_key_read.sct / base_value are ignored
 * (the base comes from the cache); agn_key_result.status tells HIT / NEW /
 * LOG.  Reads of one key are applied in arrival order. */
int agn_batcher_create_cached(agn_oplog *log, uint32_t slots, uint32_t max_batch,
                              uint32_t max_wait_us, agn_batcher **out);
/* ABI v5, cached set_aw / register_mv batchers: *pairs = an upper bound of the
 * pairs of any state the partition's snapshot cache holds for `key` (the
 * largest state the batcher has returned for it; 0 otherwise).  A read whose
 * out_cap is the key's length (agn_oplog_key_meta) + this bound cannot get
 * AGN_ECAPACITY from its cached base.  Not part of the reference's API (the
 * ETS read copies terms of any size). */
int agn_batcher_state_bound(agn_batcher *b, uint64_t key, uint32_t *pairs);
/* ABI v5, cached batchers: materialize_snapshot's store (:466-509) of a
 * snapshot the caller materialized itself -- the read whose cache held no
 * snapshot <= its clock (agn_key_result.status AGN_SS_LOG) and which the
 * caller served from the log (get_from_snapshot_log :416-419 ->
 * logging_vnode:get_up_to_time -> materialize/4, e.g. agn_materialize_host).
 * Such a response is never the newest snapshot (is_newest_snapshot = false,
 * src/logging_vnode.erl:538-540), so only a GC read stores it: flags =
 * AGN_READ_GC (op_insert_gc's GC read, :640) runs internal_store_ss /
 * insert_bigger / snapshot_insert_gc (:341-364, 513-563) on the device cache
 * and prune_ops of the key when it collects, exactly as a GC read served from
 * the cache does; flags = 0 stores nothing (the reference's ShouldRefreshCache
 * is false for it).  Call it only when the materialize returned ok with a
 * LastOpCt other than ignore and the log response had ops (:466-484).  clock
 * [D] (+ clock_mask [W], NULL = every DC) = LastOpCt, last_op = NewLastOp,
 * count = ops applied, value = counter_pn value, or n_pairs / tags / toks =
 * the set_aw / register_mv state (host arrays, the result layout).  Runs in
 * arrival order with the batcher's reads; blocks. */
int agn_batcher_store(agn_batcher *b, uint64_t key, const uint64_t *clock,
                      const uint64_t *clock_mask, int64_t last_op, uint32_t count, int64_t value,
                      uint32_t n_pairs, const uint32_t *tags, const uint64_t *toks, uint32_t flags);

/* ---- exact term interning (the Erlang binding's term <-> integer maps) ----
 * Host-only.  The device log holds DC ids, keys, TxIds, set elements /
 * register values and tokens as integers; the NIF maps a term through its
 * external term format (enif_term_to_binary) with an interner: equal byte
 * strings <=> equal id (full comparison, no hash shortcut -- exact, as
 * is_op_in_snapshot's TxId == Op#clocksi_payload.txid,
 * src/clocksi_materializer.erl:220, requires), ids dense from first_id, at
 * most max_ids (AGN_ECAPACITY beyond).  agn_intern_bytes returns the stored
 * bytes of an id for decoding (valid until destroy).  Thread-safe. */
typedef struct agn_interner agn_interner;
int agn_interner_create(uint64_t first_id, uint64_t max_ids, agn_interner **out);
int agn_interner_destroy(agn_interner *t);
int agn_intern(agn_interner *t, const void *bytes, size_t n, uint64_t *id, int *is_new);
int agn_intern_find(const agn_interner *t, const void *bytes, size_t n, uint64_t *id,
                    int *found);
int agn_intern_bytes(const agn_interner *t, uint64_t id, const void **bytes, size_t *n);
int agn_interner_size(const agn_interner *t, uint64_t *n);

/* ---- base-snapshot selection: vector_orddict:get_smaller/2 --------------
 * (src/vector_orddict.erl:74-87, called from
 * src/materializer_vnode.erl:400).  cache_off[n_req+1] CSR over cached
 * snapshot clocks (newest first), clocks [n_cached * D] (+ masks).  For each
 * request writes the index (within its list) of the first clock <= R, or -1
 * (= {undefined, _}), and is_first (1 if that index is 0 / list empty). */
int agn_select_base(agn_ctx *ctx, uint32_t n_dcs, uint64_t n_req,
                    const uint64_t *cache_off, const uint64_t *clocks,
                    const uint64_t *clock_mask, const uint64_t *R,
                    const uint64_t *R_mask, int32_t *out_idx,
                    uint8_t *out_is_first, void *stream);

/* ---- global stable time ------------------------------------------------
 * stable_time_functions:get_min_time/1 (src/stable_time_functions.erl:51-85)
 * over P partition clocks [n_epochs][P][D] (device).  Absent DC entries are
 * UINT64_MAX; defined[n_epochs*P] = 0 marks an `undefined` partition
 * (NULL: all defined).  Output out[n_epochs][D+1]: per-DC min (UINT64_MAX =
 * DC absent from every partition), word D = 1 if every partition was defined
 * else 0.  agn_gst_finalize applies the "undefined => 0" rule (:78-84). */
int agn_gst_min(agn_ctx *ctx, uint32_t n_dcs, uint64_t n_parts, uint64_t n_epochs,
                const uint64_t *clocks, const uint8_t *defined, uint64_t *out,
                void *stream);
/* In place on [n_epochs][D+1]: if word D == 0, every present DC becomes 0. */
int agn_gst_finalize(agn_ctx *ctx, uint32_t n_dcs, uint64_t n_epochs, uint64_t *vec,
                     void *stream);

/* meta_data_sender:update_stable/3 with stable_time_functions:update_func_min/2
 * (src/meta_data_sender.erl:341-356, src/stable_time_functions.erl:42-48),
 * host pointers: last[D] is updated in place from new_[D]; UINT64_MAX = absent.
 * *changed = 1 if any DC was stored. */
int agn_update_stable(uint32_t n_dcs, uint64_t *last, const uint64_t *new_,
                      int *changed);

/* ---- device snapshot cache -------------------------------------------------
 * The per-partition ETS snapshot cache of materializer_vnode
 * (src/materializer_vnode.erl:341-413, 466-563) as a device table: per key a
 * vector_orddict (src/vector_orddict.erl:36-146) of at most `slots` entries,
 * newest first, each {commit clock, #materialized_snapshot{last_op_id, value}}
 * (include/antidote.hrl:169-176).  `value` is the counter_pn value; for
 * set_aw / register_mv it is the snapshot's state (the orddict the reference
 * stores) kept on the device: AGN_SS_STATE(start, pairs) into the cache's
 * state arena (state_tag / state_tok), or -- a cache without an arena -- a
 * caller handle (e.g. an index into the caller's state store).  Clocks are
 * dense rows (+ optional presence masks; an empty clock, vectorclock:new(),
 * is all-absent / all-zero). */
#define AGN_SNAPSHOT_THRESHOLD 10 /* src/materializer_vnode.erl:37 */
#define AGN_SNAPSHOT_MIN 3        /* :39 */
#define AGN_MIN_OP_STORE_SS 5     /* :47 */
typedef struct agn_ss_cache {
    uint32_t n_dcs;
    uint32_t slots;        /* >= AGN_SNAPSHOT_THRESHOLD - 1 */
    uint64_t n_keys;
    uint32_t *n;           /* [n_keys] entries in use; 0 = key absent from the cache */
    uint64_t *clock;       /* [n_keys][slots][D] */
    uint64_t *clock_mask;  /* [n_keys][slots][W] or NULL (dense) */
    int64_t *last_op;      /* [n_keys][slots] last_op_id */
    int64_t *value;        /* [n_keys][slots] value / AGN_SS_STATE / state handle */
    /* ABI v4, set_aw / register_mv (NULL = value is a caller handle): the
     * snapshot states as (tag, token) pairs, the layout of agn_result's
     * out_tag / out_tok.  agn_ss_store appends a stored snapshot's state at
     * state_ctl[0] (the next free pair) and adds the pairs of the snapshots
     * it drops to state_ctl[1]; a store that would pass state_cap is not made
     * and sets state_ctl[2] = 1 -- keep state_cap - state_ctl[0] >= the
     * batch's result capacity, re-packing with agn_ss_state_compact. */
    uint32_t *state_tag;   /* [state_cap] elem / value */
    uint64_t *state_tok;   /* [state_cap] token */
    uint64_t state_cap;    /* pairs */
    uint64_t *state_ctl;   /* [4] device: next free pair, pairs released, overflow, 0 */
} agn_ss_cache;
/* a snapshot state in a cache's arena: pairs [start, start + pairs) */
#define AGN_SS_STATE(start, pairs) ((int64_t)(((uint64_t)(start) << 24) | (uint64_t)(pairs)))
#define AGN_SS_STATE_START(v) ((uint64_t)(v) >> 24)
#define AGN_SS_STATE_PAIRS(v) ((uint32_t)((uint64_t)(v) & 0xFFFFFFu))
#define AGN_SS_STATE_MAX_PAIRS 0xFFFFFFu

/* lookup status */
#define AGN_SS_HIT 0 /* a cached snapshot <= R: base = it */
#define AGN_SS_NEW 1 /* key absent: base {ignore, Type:new()}, empty snapshot stored */
#define AGN_SS_LOG 2 /* no cached snapshot <= R: get_from_snapshot_log (:416-419) */

/* get_from_snapshot_cache/5 (:384-413) for a batch of reads (device
 * pointers; writes the agn_read fields of the materialize that follows):
 *  - key absent (n[k] == 0): sct_ignore = 1, base_value = 0, is_first = 1,
 *    status AGN_SS_NEW, and the empty snapshot {last_op_id 0, value 0} is
 *    stored at vectorclock:new() (store_snapshot, :398-402);
 *  - else vector_orddict:get_smaller(R, SD) (src/vector_orddict.erl:74-87):
 *    the newest entry whose clock <= R: sct (+ sct_mask) = its clock,
 *    sct_ignore = 0, base_value = its value, is_first = (it is the head),
 *    status AGN_SS_HIT;
 *  - no entry <= R: status AGN_SS_LOG, is_first = 0 (the caller falls back
 *    to the log; agn_ss_store ignores the request).
 * sct_mask / R_mask may be NULL for dense caches.  Requests of one batch must
 * name distinct keys. */
int agn_ss_lookup(agn_ctx *ctx, agn_ss_cache *cache, uint64_t n_req, const uint64_t *keys,
                  const uint64_t *R, const uint64_t *R_mask, uint64_t *sct, uint64_t *sct_mask,
                  uint8_t *sct_ignore, int64_t *base_value, uint8_t *is_first, uint8_t *status,
                  void *stream);

/* The cache half of materialize_snapshot/7 + internal_store_ss/5 +
 * snapshot_insert_gc/4 (:466-563), after agn_materialize of the same batch
 * (`res`, device): for a request that materialized (no error, status !=
 * AGN_SS_LOG, the key has >= 1 op, LastOpCt != ignore):
 *   refresh = IsNewSS and is_first and Count >= MIN_OP_STORE_SS
 *   if refresh or should_gc:  ShouldInsert = SD empty or
 *        NewLastOp - first.last_op_id >= MIN_OP_STORE_SS
 *     if ShouldInsert or should_gc:  SD1 = insert_bigger(LastOpCt, {NewLastOp,
 *        value}, SD) (prepend iff not le(LastOpCt, first clock));
 *        if size(SD1) >= SNAPSHOT_THRESHOLD or should_gc: SD := first
 *        SNAPSHOT_MIN entries of SD1, prune[k] = 1 and threshold[k] =
 *        vectorclock:min of their clocks (missing entry = 0) — the input of
 *        agn_prune_ops; else SD := SD1.
 * value = handle[i] when handle != NULL, else res->value[i].  should_gc may
 * be NULL (no GC reads).  prune[n_keys] is cleared first; threshold_mask may
 * be NULL for dense caches.  Requests of one batch must name distinct keys. */
int agn_ss_store(agn_ctx *ctx, agn_ss_cache *cache, const agn_log *log, uint64_t n_req,
                 const uint64_t *keys, const uint8_t *is_first, const uint8_t *status,
                 const uint8_t *should_gc, const agn_result *res, const int64_t *handle,
                 uint8_t *prune, uint64_t *threshold, uint64_t *threshold_mask, void *stream);

/* materializer_vnode:read/6 for a batch (:96-102, 371-509) in ONE kernel:
 * agn_ss_lookup -> agn_materialize from the cached base -> agn_ss_store, per
 * request, for counter_pn logs with dense clocks (D <= 8; the read
 * batcher's fused path over device arrays).  For set_aw / register_mv caches
 * with a state arena (and any clock width) the same three steps run as the
 * batched kernels, the base state read from the arena by the tags kernel and
 * the stored state appended to it: out.out_off is the caller's capacity CSR
 * (a request whose state does not fit gets AGN_F_ERR_CAPACITY and no store),
 * out.out_n / out_tag / out_tok receive the states.  keys[n_req] (distinct, device),
 * R[n_req][D], txid[n_req] (NULL: ignore), should_gc[n_req] (NULL: none);
 * results in out (value, hole, lastct, count, flags, err_pos), status[n_req]
 * (AGN_SS_*), prune[n_req] (per request, unlike agn_ss_store's per key) and
 * threshold[n_keys][D].  Same results, cache contents and prune flags as the
 * three calls; AGN_ENOTSUP for another type or shape.  One launch, the
 * key's cache slots held in registers (21 us for 10k keys, cfg1, D = 3, where
 * the three calls take 35 us); in bulk the batched kernels, which are faster
 * there: for D < 8 from 2^15 requests, at D = 8 from 5M (10M keys: 9.05 vs
 * 9.25 ms); AGN_READ_CACHED_SPLIT=<n> sets the switch (0: always one launch).  Reads
 * at most 16 slots of a key (caches written by these entry points hold at
 * most SNAPSHOT_THRESHOLD - 1). */
int agn_read_cached(agn_ctx *ctx, agn_ss_cache *cache, const agn_log *log, uint64_t n_req,
                    const uint64_t *keys, const uint64_t *R, const uint64_t *txid,
                    const uint8_t *should_gc, agn_result *out, uint8_t *status, uint8_t *prune,
                    uint64_t *threshold, void *stream);

/* Re-packs the live snapshot states of a set_aw / register_mv cache into a
 * fresh arena new_tag / new_tok of new_cap pairs (device, caller-owned): every
 * slot's AGN_SS_STATE is rewritten to its new place, state_ctl becomes {live
 * pairs, 0, 0, 0} and cache->state_tag / state_tok / state_cap point to the new
 * arrays (the host struct is updated; the old arrays are free once `stream`
 * has passed this call).  AGN_ECAPACITY (nothing changed) when the live states
 * need more than new_cap pairs -- read state_ctl[0] - state_ctl[1] first.
 * Not part of the reference's API (the ETS table's memory is the runtime's). */
int agn_ss_state_compact(agn_ctx *ctx, agn_ss_cache *cache, uint32_t *new_tag,
                         uint64_t *new_tok, uint64_t new_cap, void *stream);

/* ---- log-read fallback and recovery ingest ------------------------------
 * A partition's logging_vnode disk log, decoded into records in log order
 * (#log_record{} -> #log_operation{tx_id, op_type, log_payload},
 * include/antidote.hrl:120-145).  Update records carry the key and the
 * effect (same encodings as agn_log); commit records the commit
 * {DcId, Time} and the transaction's snapshot_time. */
#define AGN_REC_OTHER 0   /* prepare / abort / noop: ignored */
#define AGN_REC_UPDATE 1
#define AGN_REC_COMMIT 2
typedef struct agn_log_records {
    uint64_t n;
    const uint8_t *kind;         /* [n] AGN_REC_* */
    const uint64_t *txid;        /* [n] */
    const uint64_t *key;         /* [n] update: key index (< n_keys) */
    const uint32_t *commit_dc;   /* [n] commit: DC index of commit_time */
    const uint64_t *commit_time; /* [n] commit */
    const uint64_t *ss;          /* [n][D] commit: snapshot_time rows */
    const uint64_t *ss_mask;     /* [n][W] or NULL (dense) */
    const int64_t *eff;          /* update effects, as in agn_log */
    const uint32_t *tag;
    const uint64_t *add_tok;
    const uint32_t *rem_off;     /* [n+1] */
    const uint64_t *rem_tok;
} agn_log_records;

/* logging_vnode get_ops_from_log / filter_terms_for_key / handle_commit
 * (src/logging_vnode.erl:522-549, 660-779) for every key at once: an update
 * is committed by the first later commit record of its transaction; it is
 * emitted iff check_max_time(CommitSnapshotTime, MaxSnapshotTime) holds
 * (max_time[n_keys][D] + mask per key, NULL = undefined, i.e. recovery
 * get_all); per key the emitted ops keep commit order, then update order
 * (dict:append), and become the device op log `out` (caller-allocated
 * arrays of >= the update count): OpSSCommit = snapshot_time with the commit
 * DC replaced by the commit time (src/clocksi_materializer.erl:224),
 * op_id = op_id_base + rank (0 for the get_up_to_time response of
 * reverse_and_add_op_id, :586-591; 1 for the op_insert_gc ids of
 * load_from_log, src/materializer_vnode.erl:288-319), txid = the
 * transaction id.  out_totals (device, may be NULL) = {ops, removal tokens}.
 * Keys index the partition's key space [0, n_keys): a partition's log holds
 * only its own keys (every update is logged at its key's partition,
 * src/log_utilities.erl:58-68), and a record naming a key outside it is
 * another partition's and is skipped.  Requires n_keys < 2^24 and n < 2^40. */
int agn_log_ingest(agn_ctx *ctx, const agn_log_records *recs, uint32_t crdt_type,
                   uint32_t n_dcs, uint64_t n_keys, const uint64_t *max_time,
                   const uint64_t *max_time_mask, uint32_t op_id_base, agn_log *out,
                   uint64_t *out_totals, void *stream);

/* ---- op-log garbage collection ------------------------------------------
 * materializer_vnode:snapshot_insert_gc -> prune_ops/check_filter
 * (src/materializer_vnode.erl:513-604): for every key k with prune[k] != 0
 * (prune == NULL: every key) drop the entries already covered by the pruned
 * snapshot, keeping exactly those with
 *   belongs_to_snapshot_op(Threshold_k, op) = not vectorclock:le(OpSSCommit, Threshold_k)
 * (src/materializer.erl:101-106) in log order.  threshold[n_keys][D] (+ mask,
 * NULL = dense; missing entries read 0) is vectorclock:min over the kept
 * snapshots' commit times (:523-527), computed by the caller.  Keys with
 * prune[k] == 0 are copied unchanged; prune must be 4-byte aligned.
 * Out-of-place: `out` (host descriptor of device arrays) must provide
 * key_off[n_keys+1], oc, op_id (+ oc_mask, txid, eff, tag, add_tok,
 * rem_off[n_entries+1], rem_tok when `log` has them) with at least the input
 * sizes; n_keys / n_dcs / crdt_type / key_type are taken from `log`.
 * out_flags[n_keys] (device, may be NULL): AGN_GC_ALL_PRUNED when no op of
 * a collected key survives (every op covered, or none to begin with) — the
 * reference then stores element(?FIRST_OP+Len) of the ETS tuple, an empty
 * slot, as a length-1 op list (:580-583); here the key keeps zero entries.
 * out_totals (device, may be NULL) receives {kept entries, kept removal
 * tokens}.  Asynchronous on `stream`.
 * Segmented output (out->key_len != NULL): one pass instead of mark / scan /
 * scatter -- every key keeps its input segment start in the output arrays
 * (out->key_off[n_keys] receives the starts, out->key_len the kept lengths,
 * removal tokens keep their input positions' ranges), unselected keys are
 * copied, and out->key_id0 (if given) receives the consecutive-id index. */
#define AGN_GC_ALL_PRUNED 0x1u
int agn_prune_ops(agn_ctx *ctx, const agn_log *log, const uint8_t *prune,
                  const uint64_t *threshold, const uint64_t *threshold_mask, agn_log *out,
                  uint32_t *out_flags, uint64_t *out_totals, void *stream);

/* ---- gentlerain scalar GST ----------------------------------------------
 * dc_utilities:get_scalar_stable_time/0 and the gr branch of
 * get_stable_snapshot/0 (src/dc_utilities.erl:247-320): GST = the min over
 * the DCs present in the merged stable dict; every present DC is replaced by
 * GST (in place on [n_epochs][D+1] rows as produced by agn_gst_min /
 * agn_gst_finalize; word D is left as is).  out_gst[n_epochs] receives GST,
 * or UINT64_MAX when the dict is empty (the caller then uses
 * now - ?OLD_SS_MICROSEC, :303-309).  Device pointers. */
int agn_gst_scalar(agn_ctx *ctx, uint32_t n_dcs, uint64_t n_epochs, uint64_t *vec,
                   uint64_t *out_gst, void *stream);

/* ---- causal-dependency check ---------------------------------------------
 * inter_dc_dep_vnode:try_store/2 (src/inter_dc_dep_vnode.erl:128-155): a
 * remote transaction is applicable iff vectorclock:ge(CurrentClock, Deps)
 * with the originating DC's entry set to 0 on both sides.  Batched over
 * n_txn transactions: deps[n_txn][D] (+ deps_mask, NULL = dense) is the
 * transaction's snapshot, origin[n_txn] its DC index, part[n_txn] the index
 * of its partition's clock in part_clock[n_parts][D] (+ part_mask).  Each
 * transaction is checked against the given clocks (the caller applies the
 * in-order queue semantics: the first blocked transaction stops its queue).
 * out_ok[n_txn] = 1 if applicable.  Device pointers. */
int agn_dep_check(agn_ctx *ctx, uint32_t n_dcs, uint64_t n_txn, const uint64_t *deps,
                  const uint64_t *deps_mask, const uint32_t *origin, const uint32_t *part,
                  uint64_t n_parts, const uint64_t *part_clock, const uint64_t *part_mask,
                  uint8_t *out_ok, void *stream);

/* ---- multi-GPU: the one collective -------------------------------------
 * The meta_data_sender exchange (src/meta_data_sender.erl:230-255: local min,
 * cast to every node, min again) is one RCCL allreduce(ncclUint64, ncclMin)
 * over xGMI.  The unique id (128 bytes) is produced by rank 0 and
 * distributed by the caller (torch.distributed / the Erlang cluster). */
#define AGN_UNIQUE_ID_BYTES 128
int agn_comm_unique_id(uint8_t *out_id /* [AGN_UNIQUE_ID_BYTES] */);
int agn_comm_init(agn_ctx *ctx, int nranks, int rank, const uint8_t *id);
int agn_comm_destroy(agn_ctx *ctx);
int agn_gst_allreduce(agn_ctx *ctx, uint64_t *dev_vec, uint64_t n_words, void *stream);
/* The same exchange over any other transport (disterl casts, a gloo /
 * host all-gather): the [n_vecs][D+1] vectors agn_gst_min produced on the
 * nodes (host pointers) -> out[D+1] = their element-wise min followed by
 * agn_gst_finalize's rule -- get_min_time over {local_merged, remote...}
 * (src/meta_data_sender.erl:244).  Host-only. */
int agn_gst_merge(uint32_t n_dcs, uint64_t n_vecs, const uint64_t *vecs, uint64_t *out);

/* ---- synthetic op logs (BASELINE.md §3 / SURVEY.md §8(d) generator) -----
 * Deterministic SplitMix64 streams, one per key (global key index
 * key_base + i * key_stride, seed cfg->seed); identical output on host and
 * device.  Used by bench.py and the parity tests only.  The library owns the
 * arrays it fills into *log / *req (host: malloc, device: HBM); release them
 * with the matching agn_gen_free_*.  The request holds one read per key:
 * R = "random snapshot VC" (max OpSSCommit of a random prefix, jittered),
 * SCT = ignore (cold) or, with warm = 1, the max OpSSCommit of a shorter
 * random prefix; base = Type:new(). */
typedef struct agn_gen_cfg {
    uint32_t crdt_type;
    uint32_t n_dcs;
    uint64_t n_keys;
    uint32_t ops_per_key;
    uint32_t n_elems;      /* set_aw elements / register_mv values per key */
    uint64_t seed;
    uint64_t key_base;     /* global index of local key 0 */
    uint64_t key_stride;   /* global key = key_base + i * key_stride (sharding) */
    uint32_t warm;
    uint32_t _pad;
} agn_gen_cfg;

int agn_gen_host(const agn_gen_cfg *cfg, agn_log *log, agn_read *req);
int agn_gen_free_host(agn_log *log, agn_read *req);
int agn_gen_dev(agn_ctx *ctx, const agn_gen_cfg *cfg, agn_log *log, agn_read *req,
                void *stream);
int agn_gen_free_dev(agn_ctx *ctx, agn_log *log, agn_read *req);

#ifdef __cplusplus
}
#endif
#endif /* ANTIDOTE_GPU_H */
