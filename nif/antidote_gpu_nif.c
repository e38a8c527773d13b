/*
 * antidote_gpu_nif.c — thin Erlang NIF over include/antidote_gpu.h.
 *
 * Built only where erl_nif.h exists (not in this image; see nif/Makefile).
 * The Erlang side (nif/antidote_gpu.erl) encodes terms into the SoA binaries
 * of the C ABI (DC index table, OpSSCommit rows, interned tags/tokens); this
 * file only wraps binaries into agn_* descriptors, runs the engine on a dirty
 * scheduler and returns result binaries.  It never crashes the VM: malformed
 * terms -> enif_make_badarg, engine failures -> {error, Atom}.
 *
 * Exports (antidote_gpu_nif):
 *   open(Device) -> {ok, Ctx} | {error, Reason}
 *
 *   Engine-owned partition (the materializer_vnode ETS ops cache in HBM,
 *   one per vnode, holding keys of every CRDT type like ops_cache-<P>; one
 *   device op log per type, created with the type's first op; the resource's
 *   destructor frees them).  Type = a type atom (antidote_crdt_counter_pn,
 *   antidote_crdt_set_aw, antidote_crdt_register_mv) or its id 1..3:
 *   part_open(Ctx, Type, NDcs, NKeys, Cached) -> {ok, Part}
 *       Type: the type whose log is created up front
 *   part_update(Part, Key, Type, OcPairs, TxId, Effect) -> {ok, OpId, GcDue}
 *       update/2 -> op_insert_gc/3 (agn_oplog_append): OcPairs =
 *       [{Dc, Time}] of the op's OpSSCommit, TxId a term or ignore, Effect the
 *       #clocksi_payload.op_param (counter_pn integer, set_aw
 *       [{Elem, AddToks, RemToks}], register_mv {V, Tok, Ovr} | {reset, Ovr})
 *   part_read(Part, Key, Type, RPairs, TxId, Gc) -> {ok, Value, NewLastOp,
 *       LastOpCt, IsNewSS, Count} | {error, no_snapshot} | {error, Reason}
 *       cached partition: the whole read/6 (device snapshot cache + GC);
 *       Gc = true is op_insert_gc's GC read.  Raises corrupted_ops_cache when
 *       the key holds ops of another type (src/clocksi_materializer.erl:191)
 *   part_materialize(Part, Key, Type, RPairs, SctPairs | ignore, TxId, Base) ->
 *       same result: materialize/4 of the resident ops from a caller base
 *       (the reference's own ETS snapshot cache stays in Erlang)
 *   part_gc_due(Part, Key, Type) -> boolean()
 *       op_insert_gc's GC trigger for the key's next op of Type (:635),
 *       checked before the insert as the reference does
 *   part_gc(Part, Key, ThresholdPairs) -> ok
 *       snapshot_insert_gc's prune_ops + resize for one key (agn_oplog_prune),
 *       over its ops of every type
 *   part_store(Part, Key, Type, CommitTimePairs, NewLastOp, Count, Value, Gc) -> ok
 *       materialize_snapshot's store of a snapshot served from the log
 *       (agn_batcher_store; Gc = true: op_insert_gc's GC read)
 *   part_stats(Part) -> {Entries, Slots, Tokens}
 *   part_key_meta(Part, Key, Type) -> {Length, ListLen, OpId}
 *   Keys, DC ids, TxIds, elements / values and tokens are interned exactly
 *   (agn_interner over enif_term_to_binary), never hashed.
 *   materialize(Ctx, Type, NDcs, Log, Read, CapOff) ->
 *       {ok, {Value, Hole, LastCt, LastCtMask, Count, Flags, ErrPos, OutN, OutTag, OutTok}}
 *     Log  = {KeyOff, KeyType, Oc, OcMask, OpId, TxId, Eff, Tag, AddTok, RemOff, RemTok}
 *     Read = {Keys, R, RMask, Sct, SctMask, SctIgnore, TxIds, BaseValue, BaseOff, BaseTag, BaseTok}
 *     every element a binary (<<>> = NULL); result elements are binaries.
 *   gst_min(Ctx, NDcs, NParts, Clocks, Defined) -> {ok, Vec}
 *   select_base(Ctx, NDcs, CacheOff, Clocks, ClockMask, R, RMask) -> {ok, {Idx, IsFirst}}
 */
#include <erl_nif.h>
#include <string.h>

#include "../include/antidote_gpu.h"

#include <pthread.h>
#include <stdlib.h>

static ErlNifResourceType *CTX_RES;
static ErlNifResourceType *PART_RES;

typedef struct {
    agn_ctx *ctx;
} ctx_res;

static ERL_NIF_TERM atom(ErlNifEnv *env, const char *a) { return enif_make_atom(env, a); }

static ERL_NIF_TERM error_tuple(ErlNifEnv *env, int code) {
    const char *a = "engine_error";
    switch (code) {
        case AGN_EINVAL: a = "einval"; break;
        case AGN_EHIP: a = "ehip"; break;
        case AGN_ENOMEM: a = "enomem"; break;
        case AGN_ECAPACITY: a = "ecapacity"; break;
        case AGN_ENOTSUP: a = "enotsup"; break;
        case AGN_ERCCL: a = "erccl"; break;
        case AGN_ENODEV: a = "enodev"; break;
    }
    return enif_make_tuple2(env, atom(env, "error"), atom(env, a));
}

static void ctx_dtor(ErlNifEnv *env, void *obj) {
    (void)env;
    ctx_res *r = (ctx_res *)obj;
    if (r->ctx) agn_close(r->ctx);
    r->ctx = NULL;
}

/* ---- partition resource ------------------------------------------------ */
/* One CRDT type's share of a partition: the device op log of the partition's
 * ops of that type, its read batcher and part_gc's scratch.  The reference's
 * ops_cache-<P> holds keys of any type; a key's ops normally share one type
 * (its bucket's), and a read of another type raises corrupted_ops_cache. */
typedef struct {
    agn_oplog *log;
    agn_batcher *bt;
    /* part_gc scratch (device): prune flags [K], threshold row [K][D] (+ mask) */
    uint8_t *d_prune;
    uint64_t *d_thr, *d_thrm;
    int ready;              /* published (release) once every field is set */
} part_sub;

#define NTYPES 4 /* indexed by AGN_COUNTER_PN .. AGN_REGISTER_MV */
#define NO_HOME 0xFFu

typedef struct {
    ctx_res *ctx;           /* kept alive while the partition lives */
    part_sub sub[NTYPES];
    pthread_mutex_t sub_mu; /* creation of a type's log */
    agn_interner *keys, *dcs, *txids, *tags, *toks;
    uint32_t type, D, W;    /* type: the one part_open created */
    uint64_t K;
    int cached;
    /* The reference keeps ONE ETS tuple per key for every type (:621-647):
     * one op counter (element 3, :630) and one {Length, ListLen}.  Per key:
     * the counter across this partition's per-type logs (set on a log before
     * each append, agn_oplog_set_counter) and the type of the key's first op,
     * whose log's ListLen is the tuple's (only a GC read changes ListLen, and
     * one over ops of two types raises). */
    uint32_t *kcnt;
    uint8_t *khome;         /* NO_HOME until the key's first op */
    pthread_mutex_t gc_mu;
    /* the original effect term (external format) of every op whose effect the
     * engine could not encode (an invalid entry), by (key, type, op id): a read
     * that includes it returns {error, {unexpected_operation, Effect, Type}}
     * with that term, as materializer:update_snapshot/3 (src/materializer.erl:
     * 51-58).  Recorded before the append makes the op visible; a key's
     * records are dropped once a GC leaves it no ops. */
    pthread_mutex_t inv_mu;
    struct inv_op {
        uint64_t key;
        uint32_t type, id;
        ErlNifBinary eff;
    } *inv;
    size_t n_inv, cap_inv;
} part_res;

static const char *type_name(uint32_t type) {
    switch (type) {
        case AGN_COUNTER_PN: return "antidote_crdt_counter_pn";
        case AGN_SET_AW: return "antidote_crdt_set_aw";
        case AGN_REGISTER_MV: return "antidote_crdt_register_mv";
    }
    return "undefined";
}

/* keep the effect term of an invalid op (one writer: the vnode) */
static int inv_put(ErlNifEnv *env, part_res *p, uint64_t key, uint32_t type, uint32_t id,
                   ERL_NIF_TERM eff) {
    ErlNifBinary b;
    if (!enif_term_to_binary(env, eff, &b)) return AGN_ENOMEM;
    pthread_mutex_lock(&p->inv_mu);
    if (p->n_inv == p->cap_inv) {
        const size_t c = p->cap_inv ? 2 * p->cap_inv : 16;
        struct inv_op *n = enif_realloc(p->inv, c * sizeof *n);
        if (!n) {
            pthread_mutex_unlock(&p->inv_mu);
            enif_release_binary(&b);
            return AGN_ENOMEM;
        }
        p->inv = n;
        p->cap_inv = c;
    }
    p->inv[p->n_inv].key = key;
    p->inv[p->n_inv].type = type;
    p->inv[p->n_inv].id = id;
    p->inv[p->n_inv].eff = b;
    p->n_inv++;
    pthread_mutex_unlock(&p->inv_mu);
    return AGN_OK;
}

/* the effect term of op `id` of `key` (type `type`), or 'undefined' */
static ERL_NIF_TERM inv_get(ErlNifEnv *env, part_res *p, uint64_t key, uint32_t type,
                            uint32_t id) {
    ERL_NIF_TERM out = enif_make_atom(env, "undefined");
    pthread_mutex_lock(&p->inv_mu);
    for (size_t i = p->n_inv; i-- > 0;)
        if (p->inv[i].key == key && p->inv[i].type == type && p->inv[i].id == id) {
            if (!enif_binary_to_term(env, p->inv[i].eff.data, p->inv[i].eff.size, &out, 0))
                out = enif_make_atom(env, "undefined");
            break;
        }
    pthread_mutex_unlock(&p->inv_mu);
    return out;
}

/* drop the records of `key`'s ops of `type` with id >= `from` (from = 0: all
 * of them -- a GC left the key no ops of the type) */
static void inv_drop(part_res *p, uint64_t key, uint32_t type, uint32_t from) {
    pthread_mutex_lock(&p->inv_mu);
    size_t j = 0;
    for (size_t i = 0; i < p->n_inv; ++i) {
        if (p->inv[i].key == key && p->inv[i].type == type && p->inv[i].id >= from) {
            enif_release_binary(&p->inv[i].eff);
            continue;
        }
        p->inv[j++] = p->inv[i];
    }
    p->n_inv = j;
    pthread_mutex_unlock(&p->inv_mu);
}

static void part_dtor(ErlNifEnv *env, void *obj) {
    (void)env;
    part_res *p = (part_res *)obj;
    for (int t = 0; t < NTYPES; ++t) {
        part_sub *s = &p->sub[t];
        if (s->bt) agn_batcher_destroy(s->bt);
        if (s->log) agn_oplog_destroy(s->log);
        if (p->ctx) {
            agn_dev_free(p->ctx->ctx, s->d_prune);
            agn_dev_free(p->ctx->ctx, s->d_thr);
            agn_dev_free(p->ctx->ctx, s->d_thrm);
        }
    }
    agn_interner_destroy(p->keys);
    agn_interner_destroy(p->dcs);
    agn_interner_destroy(p->txids);
    agn_interner_destroy(p->tags);
    agn_interner_destroy(p->toks);
    pthread_mutex_destroy(&p->gc_mu);
    pthread_mutex_destroy(&p->sub_mu);
    for (size_t i = 0; i < p->n_inv; ++i) enif_release_binary(&p->inv[i].eff);
    enif_free(p->inv);
    enif_free(p->kcnt);
    enif_free(p->khome);
    pthread_mutex_destroy(&p->inv_mu);
    if (p->ctx) enif_release_resource(p->ctx);
}

static int load(ErlNifEnv *env, void **priv, ERL_NIF_TERM info) {
    (void)priv;
    (void)info;
    CTX_RES = enif_open_resource_type(env, NULL, "agn_ctx", ctx_dtor, ERL_NIF_RT_CREATE, NULL);
    PART_RES = enif_open_resource_type(env, NULL, "agn_part", part_dtor, ERL_NIF_RT_CREATE, NULL);
    return CTX_RES == NULL || PART_RES == NULL;
}

static int get_ctx(ErlNifEnv *env, ERL_NIF_TERM t, agn_ctx **out) {
    ctx_res *r;
    if (!enif_get_resource(env, t, CTX_RES, (void **)&r) || !r->ctx) return 0;
    *out = r->ctx;
    return 1;
}

/* binary -> pointer (empty binary -> NULL) with an element-count check */
static int bin_ptr(ErlNifEnv *env, ERL_NIF_TERM t, size_t elem, size_t want, const void **out) {
    ErlNifBinary b;
    if (!enif_inspect_binary(env, t, &b)) return 0;
    if (b.size == 0) {
        *out = NULL;
        return 1;
    }
    if (b.size % elem) return 0;
    if (want != (size_t)-1 && b.size / elem < want) return 0;
    *out = b.data;
    return 1;
}

static ERL_NIF_TERM nif_open(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    int dev;
    if (argc != 1 || !enif_get_int(env, argv[0], &dev)) return enif_make_badarg(env);
    agn_ctx *c = NULL;
    int rc = agn_open(dev, &c);
    if (rc) return error_tuple(env, rc);
    ctx_res *r = enif_alloc_resource(CTX_RES, sizeof *r);
    r->ctx = c;
    ERL_NIF_TERM t = enif_make_resource(env, r);
    enif_release_resource(r);
    return enif_make_tuple2(env, atom(env, "ok"), t);
}

static ERL_NIF_TERM new_bin(ErlNifEnv *env, size_t bytes, void **data) {
    ERL_NIF_TERM t;
    *data = enif_make_new_binary(env, bytes ? bytes : 1, &t);
    if (!bytes) memset(*data, 0, 1);
    return t;
}

static ERL_NIF_TERM nif_materialize(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    agn_ctx *ctx;
    unsigned type, D;
    int arity;
    const ERL_NIF_TERM *L, *Q;
    if (argc != 6 || !get_ctx(env, argv[0], &ctx) || !enif_get_uint(env, argv[1], &type) ||
        !enif_get_uint(env, argv[2], &D) || D == 0 || D > 256 ||
        !enif_get_tuple(env, argv[3], &arity, &L) || arity != 11 ||
        !enif_get_tuple(env, argv[4], &arity, &Q) || arity != 11)
        return enif_make_badarg(env);
    const size_t W = (D + 63) / 64;
    agn_log log;
    agn_read req;
    memset(&log, 0, sizeof log);
    memset(&req, 0, sizeof req);
    log.crdt_type = type;
    log.n_dcs = D;
    ErlNifBinary ko, ks;
    if (!enif_inspect_binary(env, L[0], &ko) || ko.size < 8 || ko.size % 8)
        return enif_make_badarg(env);
    log.n_keys = ko.size / 8 - 1;
    log.key_off = (const uint64_t *)ko.data;
    log.n_entries = log.key_off[log.n_keys];
    const size_t E = log.n_entries, K = log.n_keys;
    if (!bin_ptr(env, L[1], 1, K, (const void **)&log.key_type) ||
        !bin_ptr(env, L[2], 8, E * D, (const void **)&log.oc) ||
        !bin_ptr(env, L[3], 8, E * W, (const void **)&log.oc_mask) ||
        !bin_ptr(env, L[4], 4, E, (const void **)&log.op_id) ||
        !bin_ptr(env, L[5], 8, E, (const void **)&log.txid) ||
        !bin_ptr(env, L[6], 8, E, (const void **)&log.eff) ||
        !bin_ptr(env, L[7], 4, E, (const void **)&log.tag) ||
        !bin_ptr(env, L[8], 8, E, (const void **)&log.add_tok) ||
        !bin_ptr(env, L[9], 4, E + 1, (const void **)&log.rem_off) ||
        !bin_ptr(env, L[10], 8, (size_t)-1, (const void **)&log.rem_tok))
        return enif_make_badarg(env);
    if (!enif_inspect_binary(env, Q[0], &ks) || ks.size % 8) return enif_make_badarg(env);
    req.n_req = ks.size / 8;
    const size_t N = req.n_req;
    req.keys = (const uint64_t *)ks.data;
    req.req_type = type;
    if (!bin_ptr(env, Q[1], 8, N * D, (const void **)&req.R) ||
        !bin_ptr(env, Q[2], 8, N * W, (const void **)&req.R_mask) ||
        !bin_ptr(env, Q[3], 8, N * D, (const void **)&req.sct) ||
        !bin_ptr(env, Q[4], 8, N * W, (const void **)&req.sct_mask) ||
        !bin_ptr(env, Q[5], 1, N, (const void **)&req.sct_ignore) ||
        !bin_ptr(env, Q[6], 8, N, (const void **)&req.txid) ||
        !bin_ptr(env, Q[7], 8, N, (const void **)&req.base_value) ||
        !bin_ptr(env, Q[8], 8, N + 1, (const void **)&req.base_off) ||
        !bin_ptr(env, Q[9], 4, (size_t)-1, (const void **)&req.base_tag) ||
        !bin_ptr(env, Q[10], 8, (size_t)-1, (const void **)&req.base_tok))
        return enif_make_badarg(env);
    for (size_t i = 0; i < N; ++i)
        if (req.keys[i] >= K) return enif_make_badarg(env);
    agn_result out;
    memset(&out, 0, sizeof out);
    const uint64_t *cap = NULL;
    if (!bin_ptr(env, argv[5], 8, 0, (const void **)&cap)) return enif_make_badarg(env);
    const size_t n_out = cap ? cap[N] : 0;
    out.out_off = cap;
    ERL_NIF_TERM t[10];
    t[0] = new_bin(env, N * 8, (void **)&out.value);
    t[1] = new_bin(env, N * 8, (void **)&out.hole);
    t[2] = new_bin(env, N * D * 8, (void **)&out.lastct);
    t[3] = new_bin(env, N * W * 8, (void **)&out.lastct_mask);
    t[4] = new_bin(env, N * 4, (void **)&out.count);
    t[5] = new_bin(env, N * 4, (void **)&out.flags);
    t[6] = new_bin(env, N * 4, (void **)&out.err_pos);
    t[7] = new_bin(env, N * 4, (void **)&out.out_n);
    t[8] = new_bin(env, n_out * 4, (void **)&out.out_tag);
    t[9] = new_bin(env, n_out * 8, (void **)&out.out_tok);
    if (type == AGN_COUNTER_PN) out.out_off = NULL;
    int rc = agn_materialize_host(ctx, &log, &req, &out);
    if (rc) return error_tuple(env, rc);
    return enif_make_tuple2(env, atom(env, "ok"), enif_make_tuple_from_array(env, t, 10));
}

static ERL_NIF_TERM nif_gst_min(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    agn_ctx *ctx;
    unsigned D;
    ErlNifUInt64 P;
    const uint64_t *clocks;
    const uint8_t *defined;
    if (argc != 5 || !get_ctx(env, argv[0], &ctx) || !enif_get_uint(env, argv[1], &D) ||
        !enif_get_uint64(env, argv[2], &P) ||
        !bin_ptr(env, argv[3], 8, (size_t)P * D, (const void **)&clocks) ||
        !bin_ptr(env, argv[4], 1, (size_t)P, (const void **)&defined))
        return enif_make_badarg(env);
    /* small epochs: stage through device buffers */
    void *dc = NULL, *dd = NULL, *dv = NULL;
    uint64_t *vec;
    ERL_NIF_TERM vt = new_bin(env, (D + 1) * 8, (void **)&vec);
    int rc = agn_dev_alloc(ctx, (size_t)P * D * 8, &dc);
    if (!rc && defined) rc = agn_dev_alloc(ctx, P, &dd);
    if (!rc) rc = agn_dev_alloc(ctx, (D + 1) * 8, &dv);
    if (!rc) rc = agn_memcpy_h2d(ctx, dc, clocks, (size_t)P * D * 8, NULL);
    if (!rc && defined) rc = agn_memcpy_h2d(ctx, dd, defined, P, NULL);
    if (!rc) rc = agn_gst_min(ctx, D, P, 1, (const uint64_t *)dc, (const uint8_t *)dd,
                              (uint64_t *)dv, NULL);
    if (!rc) rc = agn_gst_finalize(ctx, D, 1, (uint64_t *)dv, NULL);
    if (!rc) rc = agn_memcpy_d2h(ctx, vec, dv, (D + 1) * 8, NULL);
    if (!rc) rc = agn_stream_sync(ctx, NULL);
    agn_dev_free(ctx, dc);
    agn_dev_free(ctx, dd);
    agn_dev_free(ctx, dv);
    if (rc) return error_tuple(env, rc);
    return enif_make_tuple2(env, atom(env, "ok"), vt);
}

static ERL_NIF_TERM nif_select_base(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    agn_ctx *ctx;
    unsigned D;
    ErlNifBinary off;
    const uint64_t *clocks, *cmask, *R, *Rm;
    if (argc != 7 || !get_ctx(env, argv[0], &ctx) || !enif_get_uint(env, argv[1], &D) ||
        D == 0 || !enif_inspect_binary(env, argv[2], &off) || off.size < 8 || off.size % 8)
        return enif_make_badarg(env);
    const size_t n = off.size / 8 - 1, W = (D + 63) / 64;
    const uint64_t M = ((const uint64_t *)off.data)[n];
    if (!bin_ptr(env, argv[3], 8, M * D, (const void **)&clocks) ||
        !bin_ptr(env, argv[4], 8, M * W, (const void **)&cmask) ||
        !bin_ptr(env, argv[5], 8, n * D, (const void **)&R) ||
        !bin_ptr(env, argv[6], 8, n * W, (const void **)&Rm))
        return enif_make_badarg(env);
    int32_t *idx;
    uint8_t *first;
    ERL_NIF_TERM ti = new_bin(env, n * 4, (void **)&idx), tf = new_bin(env, n, (void **)&first);
    void *b[7] = {0};
    const size_t sz[5] = {off.size, M * D * 8, cmask ? M * W * 8 : 0, n * D * 8, Rm ? n * W * 8 : 0};
    const void *src[5] = {off.data, clocks, cmask, R, Rm};
    int rc = AGN_OK;
    for (int i = 0; i < 5 && !rc; ++i)
        if (sz[i]) {
            rc = agn_dev_alloc(ctx, sz[i], &b[i]);
            if (!rc) rc = agn_memcpy_h2d(ctx, b[i], src[i], sz[i], NULL);
        }
    if (!rc) rc = agn_dev_alloc(ctx, n * 4 + 4, &b[5]);
    if (!rc) rc = agn_dev_alloc(ctx, n + 1, &b[6]);
    if (!rc) rc = agn_select_base(ctx, D, n, b[0], b[1], b[2], b[3], b[4], b[5], b[6], NULL);
    if (!rc) rc = agn_memcpy_d2h(ctx, idx, b[5], n * 4, NULL);
    if (!rc) rc = agn_memcpy_d2h(ctx, first, b[6], n, NULL);
    if (!rc) rc = agn_stream_sync(ctx, NULL);
    for (int i = 0; i < 7; ++i) agn_dev_free(ctx, b[i]);
    if (rc) return error_tuple(env, rc);
    return enif_make_tuple2(env, atom(env, "ok"), enif_make_tuple2(env, ti, tf));
}

/* ---- partition functions -------------------------------------------------- */
static int get_part(ErlNifEnv *env, ERL_NIF_TERM t, part_res **out) {
    return enif_get_resource(env, t, PART_RES, (void **)out) && (*out)->keys != NULL;
}

/* a CRDT type: its atom or its id */
static int type_of(ErlNifEnv *env, ERL_NIF_TERM t, uint32_t *type) {
    unsigned v;
    if (enif_get_uint(env, t, &v)) {
        *type = v;
        return v >= AGN_COUNTER_PN && v <= AGN_REGISTER_MV;
    }
    for (uint32_t x = AGN_COUNTER_PN; x <= AGN_REGISTER_MV; ++x)
        if (enif_is_identical(t, atom(env, type_name(x)))) {
            *type = x;
            return 1;
        }
    return 0;
}

/* the partition's log of `type`, NULL while it holds no op of that type */
static part_sub *sub_get(part_res *p, uint32_t type) {
    part_sub *s = &p->sub[type];
    return __atomic_load_n(&s->ready, __ATOMIC_ACQUIRE) ? s : NULL;
}

/* the log of `type`, created with the type's first op (op log, read batcher,
 * part_gc scratch); the writer creates, readers see it once published */
static int sub_make(part_res *p, uint32_t type, part_sub **out) {
    part_sub *s = sub_get(p, type);
    if (s) {
        *out = s;
        return AGN_OK;
    }
    pthread_mutex_lock(&p->sub_mu);
    s = &p->sub[type];
    int rc = AGN_OK;
    if (!s->ready) {
        agn_ctx *c = p->ctx->ctx;
        rc = agn_oplog_create(c, type, p->D, p->K, 1, 0, &s->log);
        if (!rc) rc = p->cached ? agn_batcher_create_cached(s->log, 0, 1024, 50, &s->bt)
                                : agn_batcher_create(s->log, 1024, 50, &s->bt);
        if (!rc) rc = agn_dev_alloc(c, p->K, (void **)&s->d_prune);
        if (!rc) rc = agn_dev_alloc(c, p->K * p->D * 8, (void **)&s->d_thr);
        if (!rc) rc = agn_dev_alloc(c, p->K * p->W * 8, (void **)&s->d_thrm);
        if (!rc) __atomic_store_n(&s->ready, 1, __ATOMIC_RELEASE);
        /* on failure the fields stay for the destructor; a later op retries */
    }
    pthread_mutex_unlock(&p->sub_mu);
    *out = rc ? NULL : s;
    return rc;
}

/* does `key` hold ops of a type other than `type` (materialize_intern's
 * type check over the key's ops, src/clocksi_materializer.erl:190-191)? */
static int other_type_ops(part_res *p, uint64_t key, uint32_t type, int *out) {
    *out = 0;
    for (uint32_t t = AGN_COUNTER_PN; t <= AGN_REGISTER_MV && !*out; ++t) {
        part_sub *s = t == type ? NULL : sub_get(p, t);
        uint32_t len = 0;
        if (!s) continue;
        int rc = agn_oplog_key_meta(s->log, 1, &key, &len, NULL, NULL);
        if (rc) return rc;
        *out = len != 0;
    }
    return AGN_OK;
}

/* exact id of a term: its external format through an interner */
static int term_id(ErlNifEnv *env, agn_interner *t, ERL_NIF_TERM term, uint64_t *id) {
    ErlNifBinary b;
    if (!enif_term_to_binary(env, term, &b)) return AGN_ENOMEM;
    int rc = agn_intern(t, b.data, b.size, id, NULL);
    enif_release_binary(&b);
    return rc;
}

static ERL_NIF_TERM id_term(ErlNifEnv *env, agn_interner *t, uint64_t id) {
    const void *data;
    size_t n;
    ERL_NIF_TERM out;
    if (agn_intern_bytes(t, id, &data, &n) != AGN_OK ||
        enif_binary_to_term(env, (const unsigned char *)data, n, &out, 0) == 0)
        return atom(env, "undefined");
    return out;
}

/* [{Dc, Time}] -> dense row + presence mask; columns from the DC interner */
static int clock_row(ErlNifEnv *env, part_res *p, ERL_NIF_TERM pairs, uint64_t *row,
                     uint64_t *mask) {
    memset(row, 0, p->D * 8);
    memset(mask, 0, p->W * 8);
    ERL_NIF_TERM head, tail = pairs;
    while (enif_get_list_cell(env, tail, &head, &tail)) {
        int ar;
        const ERL_NIF_TERM *kv;
        ErlNifUInt64 t;
        uint64_t col;
        if (!enif_get_tuple(env, head, &ar, &kv) || ar != 2 || !enif_get_uint64(env, kv[1], &t))
            return AGN_EINVAL;
        int rc = term_id(env, p->dcs, kv[0], &col);
        if (rc) return rc;
        col -= 1;
        row[col] = t;
        mask[col >> 6] |= 1ull << (col & 63);
    }
    return enif_is_empty_list(env, tail) ? AGN_OK : AGN_EINVAL;
}

static ERL_NIF_TERM clock_pairs(ErlNifEnv *env, part_res *p, const uint64_t *row,
                                const uint64_t *mask) {
    ERL_NIF_TERM l = enif_make_list(env, 0);
    for (uint32_t d = p->D; d-- > 0;)
        if ((mask[d >> 6] >> (d & 63)) & 1ull)
            l = enif_make_list_cell(env, enif_make_tuple2(env, id_term(env, p->dcs, d + 1),
                                                         enif_make_uint64(env, row[d])), l);
    return l;
}

static int key_index(ErlNifEnv *env, part_res *p, ERL_NIF_TERM key, uint64_t *k) {
    uint64_t id;
    int rc = term_id(env, p->keys, key, &id);
    if (rc) return rc;
    *k = id - 1;
    return AGN_OK;
}

static int txid_of(ErlNifEnv *env, part_res *p, ERL_NIF_TERM t, uint64_t *id) {
    if (enif_is_identical(t, atom(env, "ignore"))) {
        *id = 0;
        return AGN_OK;
    }
    return term_id(env, p->txids, t, id);
}

static ERL_NIF_TERM nif_part_open(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    ctx_res *c;
    uint32_t type;
    unsigned D;
    ErlNifUInt64 K;
    if (argc != 5 || !enif_get_resource(env, argv[0], CTX_RES, (void **)&c) || !c->ctx ||
        !type_of(env, argv[1], &type) || !enif_get_uint(env, argv[2], &D) || D == 0 ||
        D > 256 || !enif_get_uint64(env, argv[3], &K) || K == 0)
        return enif_make_badarg(env);
    const int cached = enif_is_identical(argv[4], atom(env, "true"));
    part_res *p = enif_alloc_resource(PART_RES, sizeof *p);
    memset(p, 0, sizeof *p);
    pthread_mutex_init(&p->gc_mu, NULL);
    pthread_mutex_init(&p->sub_mu, NULL);
    pthread_mutex_init(&p->inv_mu, NULL);
    p->type = type;
    p->D = D;
    p->W = (D + 63) / 64;
    p->K = K;
    p->cached = cached;
    p->ctx = c;
    enif_keep_resource(c);
    part_sub *s;
    p->kcnt = enif_alloc(K * sizeof *p->kcnt);
    p->khome = enif_alloc(K);
    if (!p->kcnt || !p->khome) {
        enif_release_resource(p);  /* the destructor frees what was allocated */
        return error_tuple(env, AGN_ENOMEM);
    }
    memset(p->kcnt, 0, K * sizeof *p->kcnt);
    memset(p->khome, NO_HOME, K);
    int rc = agn_interner_create(1, K, &p->keys);
    if (!rc) rc = agn_interner_create(1, D, &p->dcs);
    if (!rc) rc = agn_interner_create(1, UINT64_MAX / 2, &p->txids);
    if (!rc) rc = agn_interner_create(0, 0xFFFFFFFEull, &p->tags);
    if (!rc) rc = agn_interner_create(1, UINT64_MAX / 2, &p->toks);
    if (!rc) rc = sub_make(p, type, &s);
    if (rc) {
        ERL_NIF_TERM e = error_tuple(env, rc);
        enif_release_resource(p);  /* the destructor frees what was created */
        return e;
    }
    ERL_NIF_TERM t = enif_make_resource(env, p);
    enif_release_resource(p);
    return enif_make_tuple2(env, atom(env, "ok"), t);
}

/* Entries of one effect (set_aw: one per {Elem, Add, Rem} part and per extra
 * add token; register_mv: one) into the arrays; returns the entry count or -1
 * when the effect cannot be represented (-> an invalid entry). */
#define MAXE 256
#define MAXT 4096
typedef struct {
    uint32_t n, nrem;
    uint32_t tag[MAXE];
    uint64_t add[MAXE];
    uint32_t rem_off[MAXE + 1];
    uint64_t rem[MAXT];
} entries;

static int push_rems(ErlNifEnv *env, part_res *p, ERL_NIF_TERM list, entries *E) {
    ERL_NIF_TERM h, t = list;
    while (enif_get_list_cell(env, t, &h, &t)) {
        uint64_t id;
        if (E->nrem >= MAXT || term_id(env, p->toks, h, &id)) return -1;
        E->rem[E->nrem++] = id;
    }
    return enif_is_empty_list(env, t) ? 0 : -1;
}

/* one entry {tag, add token, removal tokens of `rems` (or none)} */
static int push_entry(ErlNifEnv *env, part_res *p, entries *E, uint64_t tag, uint64_t add,
                      const ERL_NIF_TERM *rems) {
    if (E->n >= MAXE) return -1;
    E->rem_off[E->n] = E->nrem;
    E->tag[E->n] = (uint32_t)tag;
    E->add[E->n] = add;
    if (rems && push_rems(env, p, *rems, E)) return -1;
    E->n++;
    E->rem_off[E->n] = E->nrem;
    return 0;
}

static int effect_entries(ErlNifEnv *env, part_res *p, uint32_t type, ERL_NIF_TERM eff,
                          entries *E) {
    E->n = E->nrem = 0;
    E->rem_off[0] = 0;
    int ar;
    const ERL_NIF_TERM *tp;
    if (type == AGN_REGISTER_MV) {
        uint64_t tag = 0, tok = 0;
        if (!enif_get_tuple(env, eff, &ar, &tp)) return -1;
        if (ar == 2 && enif_is_identical(tp[0], atom(env, "reset")))
            return push_entry(env, p, E, 0, 0, &tp[1]) ? -1 : 1;   /* {reset, Overridden} */
        if (ar != 3 || term_id(env, p->tags, tp[0], &tag) || term_id(env, p->toks, tp[1], &tok))
            return -1;
        return push_entry(env, p, E, tag, tok, &tp[2]) ? -1 : 1;    /* {Value, Token, Overridden} */
    }
    /* set_aw: [{Elem, AddTokens, RemoveTokens}], one part per element (add_all /
     * remove_all have several); a part with several add tokens becomes several
     * entries, the removals riding on the first, as the Python encoder does */
    ERL_NIF_TERM h, t = eff;
    while (enif_get_list_cell(env, t, &h, &t)) {
        uint64_t tag;
        if (!enif_get_tuple(env, h, &ar, &tp) || ar != 3 || term_id(env, p->tags, tp[0], &tag))
            return -1;
        if (enif_is_empty_list(env, tp[1])) {
            if (push_entry(env, p, E, tag, 0, &tp[2])) return -1;
            continue;
        }
        ERL_NIF_TERM ah, at = tp[1];
        int first = 1;
        while (enif_get_list_cell(env, at, &ah, &at)) {
            uint64_t tok;
            if (term_id(env, p->toks, ah, &tok) ||
                push_entry(env, p, E, tag, tok, first ? &tp[2] : NULL))
                return -1;
            first = 0;
        }
        if (!enif_is_empty_list(env, at)) return -1;
    }
    return enif_is_empty_list(env, t) ? (int)E->n : -1;
}

static ERL_NIF_TERM nif_part_update(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    part_res *p;
    uint32_t type;
    if (argc != 6 || !get_part(env, argv[0], &p) || !type_of(env, argv[2], &type))
        return enif_make_badarg(env);
    uint64_t k, tx, row[256], mask[4];
    int rc = key_index(env, p, argv[1], &k);
    if (!rc) rc = clock_row(env, p, argv[3], row, mask);
    if (!rc) rc = txid_of(env, p, argv[4], &tx);
    if (rc == AGN_EINVAL) return enif_make_badarg(env);
    if (rc) return error_tuple(env, rc);
    part_sub *sb;
    rc = sub_make(p, type, &sb);
    if (rc) return error_tuple(env, rc);
    const uint32_t D = p->D, W = p->W;
    uint64_t keys[MAXE], txids[MAXE];
    uint8_t same[MAXE];
    int64_t eff[MAXE];
    entries *E = enif_alloc(sizeof *E);
    uint64_t *oc = enif_alloc((size_t)MAXE * D * 8), *ocm = enif_alloc((size_t)MAXE * W * 8);
    if (!E || !oc || !ocm) {
        enif_free(E);
        enif_free(oc);
        enif_free(ocm);
        return error_tuple(env, AGN_ENOMEM);
    }
    uint32_t n = 1;
    int invalid = 0;
    if (type == AGN_COUNTER_PN) {
        ErlNifSInt64 v;
        invalid = !enif_get_int64(env, argv[5], &v) || v == AGN_EFFECT_INVALID;
        eff[0] = invalid ? AGN_EFFECT_INVALID : (int64_t)v;
        E->n = 0;
    } else {
        const int ne = effect_entries(env, p, type, argv[5], E);
        if (ne < 0) {  /* not representable: one invalid entry (update/2 raises at read) */
            E->n = 1;
            E->nrem = 0;
            E->tag[0] = AGN_TAG_INVALID;
            E->add[0] = 0;
            E->rem_off[0] = E->rem_off[1] = 0;
            invalid = 1;
        }
        n = E->n;
    }
    uint32_t ids[MAXE];
    uint8_t due[MAXE];
    if (n == 0) {  /* an effect with no parts (add_all of []) changes nothing */
        enif_free(E);
        enif_free(oc);
        enif_free(ocm);
        return enif_make_tuple3(env, atom(env, "ok"), enif_make_uint(env, 0), atom(env, "false"));
    }
    for (uint32_t i = 0; i < n; ++i) {
        keys[i] = k;
        txids[i] = tx;
        same[i] = i > 0;
        memcpy(oc + (size_t)i * D, row, D * 8);
        memcpy(ocm + (size_t)i * W, mask, W * 8);
    }
    /* the key's one counter across the per-type logs (the ETS tuple's) */
    rc = agn_oplog_set_counter(sb->log, 1, &k, &p->kcnt[k]);
    /* an invalid op's effect term is recorded under the id the append gives
     * it (the key's op counter + 1; one writer) before a read can see it */
    const uint32_t next = p->kcnt[k];
    if (!rc && invalid) rc = inv_put(env, p, k, type, next + 1, argv[5]);
    if (!rc)
        rc = agn_oplog_append(sb->log, n, keys, same, oc, ocm, txids,
                              type == AGN_COUNTER_PN ? eff : NULL,
                              type == AGN_COUNTER_PN ? NULL : E->tag,
                              type == AGN_COUNTER_PN ? NULL : E->add,
                              type == AGN_COUNTER_PN ? NULL : E->rem_off,
                              type == AGN_COUNTER_PN ? NULL : E->rem, ids, due);
    if (rc && invalid) inv_drop(p, k, type, next + 1);
    if (!rc) {
        p->kcnt[k] = ids[0];
        if (p->khome[k] == NO_HOME) p->khome[k] = (uint8_t)type;
    }
    enif_free(E);
    enif_free(oc);
    enif_free(ocm);
    if (rc) return error_tuple(env, rc);
    return enif_make_tuple3(env, atom(env, "ok"), enif_make_uint(env, ids[0]),
                            atom(env, due[0] ? "true" : "false"));
}

/* qsort by Erlang term order of `key`: set_aw groups {Elem, [Tok]} by Elem,
 * register_mv pairs {V, Tok} as lists:sort/1 orders them */
typedef struct {
    ERL_NIF_TERM key, term;
} sort_item;
static int cmp_item(const void *a, const void *b) {
    return enif_compare(((const sort_item *)a)->key, ((const sort_item *)b)->key);
}

/* the state pairs of a set/register result -> the reference's value: the
 * set_aw orddict [{Elem, [Tok]}] (sorted by Elem; tokens in fold order) /
 * the register_mv list of {Value, Token}, sorted (decoded through the
 * interners, whose ids do not follow term order); 0 when out of memory */
static ERL_NIF_TERM state_term(ErlNifEnv *env, part_res *p, uint32_t type, uint32_t n,
                               const uint32_t *tag, const uint64_t *tok) {
    sort_item *v = enif_alloc(sizeof(sort_item) * (n + 1));
    if (!v) return 0;
    uint32_t m = 0;
    if (type == AGN_REGISTER_MV) {
        for (uint32_t i = 0; i < n; ++i, ++m) {
            v[m].term = enif_make_tuple2(env, id_term(env, p->tags, tag[i]), id_term(env, p->toks, tok[i]));
            v[m].key = v[m].term;
        }
    } else {
        /* pairs come grouped by element, tokens in fold order */
        for (uint32_t i = 0; i < n;) {
            uint32_t j = i;
            while (j < n && tag[j] == tag[i]) ++j;
            ERL_NIF_TERM toks = enif_make_list(env, 0);
            for (uint32_t x = j; x-- > i;) toks = enif_make_list_cell(env, id_term(env, p->toks, tok[x]), toks);
            v[m].key = id_term(env, p->tags, tag[i]);
            v[m].term = enif_make_tuple2(env, v[m].key, toks);
            ++m;
            i = j;
        }
    }
    qsort(v, m, sizeof *v, cmp_item);
    ERL_NIF_TERM l = enif_make_list(env, 0);
    for (uint32_t i = m; i-- > 0;) l = enif_make_list_cell(env, v[i].term, l);
    enif_free(v);
    return l;
}

static ERL_NIF_TERM read_result(ErlNifEnv *env, part_res *p, uint32_t type, uint64_t key,
                                const agn_key_result *o, const uint64_t *ct, const uint64_t *ctm) {
    /* erlang:error(corrupted_ops_cache) (src/clocksi_materializer.erl:190-191) */
    if (o->flags & AGN_F_ERR_CORRUPTED)
        return enif_raise_exception(env, atom(env, "corrupted_ops_cache"));
    /* {error, {unexpected_operation, Op, Type}} (src/materializer.erl:51-58),
     * Op = the effect term the vnode was given; err_pos = the op's id */
    if (o->flags & AGN_F_ERR_UNEXPECTED)
        return enif_make_tuple2(env, atom(env, "error"),
                                enif_make_tuple3(env, atom(env, "unexpected_operation"),
                                                 inv_get(env, p, key, type, o->err_pos),
                                                 atom(env, type_name(type))));
    ERL_NIF_TERM v = type == AGN_COUNTER_PN
                         ? enif_make_int64(env, o->value)
                         : state_term(env, p, type, o->out_n, o->out_tag, o->out_tok);
    if (!v) return error_tuple(env, AGN_ENOMEM);
    ERL_NIF_TERM lct = (o->flags & AGN_F_CT_IGNORE) ? atom(env, "ignore") : clock_pairs(env, p, ct, ctm);
    ERL_NIF_TERM res[6] = {atom(env, "ok"), v, enif_make_int64(env, o->hole), lct,
                           atom(env, (o->flags & AGN_F_NEWSS) ? "true" : "false"),
                           enif_make_uint(env, o->count)};
    return enif_make_tuple_from_array(env, res, 6);
}

/* a set_aw orddict [{Elem, [Tok]}] / register_mv [{V, Tok}] -> interned
 * (tag, token) pairs in the result layout (enif_alloc'ed; NULL when empty);
 * AGN_EINVAL for a malformed term */
static int state_pairs(ErlNifEnv *env, part_res *p, uint32_t type, ERL_NIF_TERM st,
                       uint32_t *n_out, uint32_t **tags_out, uint64_t **toks_out) {
    unsigned nl = 0;
    *n_out = 0;
    *tags_out = NULL;
    *toks_out = NULL;
    if (!enif_get_list_length(env, st, &nl)) return AGN_EINVAL;
    ERL_NIF_TERM h, t = st;
    uint32_t cap = 0;
    while (enif_get_list_cell(env, t, &h, &t)) {
        int ar;
        const ERL_NIF_TERM *tp;
        unsigned m = 1;
        if (!enif_get_tuple(env, h, &ar, &tp) || ar != 2) return AGN_EINVAL;
        if (type == AGN_SET_AW && !enif_get_list_length(env, tp[1], &m)) return AGN_EINVAL;
        cap += m;
    }
    uint32_t *tg = enif_alloc(4 * (cap + 1));
    uint64_t *tk = enif_alloc(8 * (cap + 1));
    if (!tg || !tk) {
        enif_free(tg);
        enif_free(tk);
        return AGN_ENOMEM;
    }
    uint32_t n = 0;
    for (t = st; enif_get_list_cell(env, t, &h, &t);) {
        int ar;
        const ERL_NIF_TERM *tp;
        uint64_t id_tag, id_tok;
        enif_get_tuple(env, h, &ar, &tp);
        int rc = term_id(env, p->tags, tp[0], &id_tag);
        if (type == AGN_REGISTER_MV) {
            if (!rc) rc = term_id(env, p->toks, tp[1], &id_tok);
            if (!rc) {
                tg[n] = (uint32_t)id_tag;
                tk[n++] = id_tok;
            }
        } else {
            ERL_NIF_TERM th, tt = tp[1];
            while (!rc && enif_get_list_cell(env, tt, &th, &tt)) {
                rc = term_id(env, p->toks, th, &id_tok);
                if (!rc) {
                    tg[n] = (uint32_t)id_tag;
                    tk[n++] = id_tok;
                }
            }
        }
        if (rc) {
            enif_free(tg);
            enif_free(tk);
            return rc;
        }
    }
    *n_out = n;
    *tags_out = tg;
    *toks_out = tk;
    return AGN_OK;
}

/* one read of `type` through the partition's batcher of that type */
static ERL_NIF_TERM part_read_common(ErlNifEnv *env, part_res *p, ERL_NIF_TERM key,
                                     uint32_t type, ERL_NIF_TERM rpairs, ERL_NIF_TERM sct,
                                     ERL_NIF_TERM txid, ERL_NIF_TERM base, int gc) {
    uint64_t k, tx, R[256], Rm[4], S[256], Sm[4], ct[256], ctm[4];
    int rc = key_index(env, p, key, &k);
    if (!rc) rc = clock_row(env, p, rpairs, R, Rm);
    if (!rc) rc = txid_of(env, p, txid, &tx);
    const int has_sct = !enif_is_identical(sct, atom(env, "ignore"));
    if (!rc && has_sct) rc = clock_row(env, p, sct, S, Sm);
    if (rc == AGN_EINVAL) return enif_make_badarg(env);
    if (rc) return error_tuple(env, rc);
    /* erlang:error(corrupted_ops_cache) (src/clocksi_materializer.erl:190-191):
     * the key holds ops of another type than the read's */
    int other = 0;
    rc = other_type_ops(p, k, type, &other);
    if (rc) return error_tuple(env, rc);
    if (other) {
        /* op_insert_gc's GC read: the op's id was taken (ets:update_counter,
         * :630) before the read (:640) raises, so the next op's id is one on */
        if (gc) p->kcnt[k]++;
        return enif_raise_exception(env, atom(env, "corrupted_ops_cache"));
    }
    part_sub *sb = sub_get(p, type);
    if (!sb) {
        /* no op of this type was ever written: materialize/4 of an empty ops
         * list -- the base value, NewLastOp = get_first_id([]) = 0, LastOpCt
         * = SCT (ignore for read/6), nothing new, nothing cached */
        ERL_NIF_TERM v;
        ErlNifSInt64 b = 0;
        if (type == AGN_COUNTER_PN)
            v = (!enif_is_identical(base, atom(env, "undefined")) && enif_get_int64(env, base, &b))
                    ? enif_make_int64(env, b) : enif_make_int64(env, 0);
        else
            v = (!p->cached && enif_is_list(env, base)) ? base : enif_make_list(env, 0);
        ERL_NIF_TERM res[6] = {atom(env, "ok"), v, enif_make_int64(env, 0),
                               has_sct ? sct : atom(env, "ignore"), atom(env, "false"),
                               enif_make_uint(env, 0)};
        return enif_make_tuple_from_array(env, res, 6);
    }
    agn_key_read rd;
    agn_key_result o;
    memset(&rd, 0, sizeof rd);
    memset(&o, 0, sizeof o);
    rd.key = k;
    rd.R = R;
    rd.R_mask = Rm;
    rd.sct = has_sct ? S : NULL;
    rd.sct_mask = has_sct ? Sm : NULL;
    rd.txid = tx;
    rd.flags = gc ? AGN_READ_GC : 0;
    o.lastct = ct;
    o.lastct_mask = ctm;
    uint32_t len = 0, nb = 0;
    uint32_t *btag = NULL, *otag = NULL;
    uint64_t *btok = NULL, *otok = NULL;
    if (type == AGN_COUNTER_PN) {
        ErlNifSInt64 v = 0;
        if (!enif_is_identical(base, atom(env, "undefined")) && !enif_get_int64(env, base, &v))
            return enif_make_badarg(env);
        rd.base_value = v;
    } else if (!p->cached) {
        /* base state pairs: set_aw orddict [{Elem, [Tok]}], register_mv [{V, Tok}]
         * (a cached partition's base state is the device snapshot cache's) */
        const int src = state_pairs(env, p, type, base, &nb, &btag, &btok);
        if (src == AGN_EINVAL) return enif_make_badarg(env);
        if (src) goto oom;
        rd.n_base = nb;
        rd.base_tag = btag;
        rd.base_tok = btok;
    }
    if (type != AGN_COUNTER_PN) {
        /* room for the state: the key's entries + the base (a cached base:
         * the largest state the partition's cache holds for the key) */
        uint32_t bound = 0;
        if (agn_oplog_key_meta(sb->log, 1, &k, &len, NULL, NULL)) goto oom;
        if (p->cached && agn_batcher_state_bound(sb->bt, k, &bound)) goto oom;
        o.out_cap = len + nb + bound + (p->cached ? 16u : 0u);
        otag = enif_alloc(4 * (o.out_cap + 1));
        otok = enif_alloc(8 * (o.out_cap + 1));
        if (!otag || !otok) goto oom;
        o.out_tag = otag;
        o.out_tok = otok;
    }
    rc = agn_batcher_read(sb->bt, &rd, &o);
    if (rc == AGN_ECAPACITY && type != AGN_COUNTER_PN && o.out_n > o.out_cap) {
        /* the state outgrew the buffer (updates landed after key_meta): read
         * again with room for it (a read/6 is repeatable: the second one is
         * served from what the first stored).  The first pass already ran a GC
         * read's store and prune, so the retry is a plain read: running
         * op_insert_gc's GC twice would resize ListLen twice (:540-558). */
        rd.flags &= ~AGN_READ_GC;
        enif_free(otag);
        enif_free(otok);
        o.out_cap = o.out_n + 16u;
        otag = enif_alloc(4 * (o.out_cap + 1));
        otok = enif_alloc(8 * (o.out_cap + 1));
        if (!otag || !otok) goto oom;
        o.out_tag = otag;
        o.out_tok = otok;
        rc = agn_batcher_read(sb->bt, &rd, &o);
    }
    ERL_NIF_TERM r;
    if (rc) r = error_tuple(env, rc);
    else if (p->cached && o.status == AGN_SS_LOG)
        r = enif_make_tuple2(env, atom(env, "error"), atom(env, "no_snapshot"));
    else r = read_result(env, p, type, k, &o, ct, ctm);
    if (!rc && gc && agn_oplog_key_meta(sb->log, 1, &k, &len, NULL, NULL) == AGN_OK && len == 0)
        inv_drop(p, k, type, 0);  /* the GC read pruned every op of the key */
    enif_free(btag);
    enif_free(btok);
    enif_free(otag);
    enif_free(otok);
    return r;
oom:
    enif_free(btag);
    enif_free(btok);
    enif_free(otag);
    enif_free(otok);
    return error_tuple(env, AGN_ENOMEM);
}

static ERL_NIF_TERM nif_part_read(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    part_res *p;
    uint32_t type;
    if (argc != 6 || !get_part(env, argv[0], &p) || !type_of(env, argv[2], &type))
        return enif_make_badarg(env);
    /* read/6 through the device snapshot cache: a partition opened with
     * Cached = false keeps the reference's ETS cache (use part_materialize) */
    if (!p->cached)
        return enif_make_tuple2(env, atom(env, "error"), atom(env, "not_cached"));
    return part_read_common(env, p, argv[1], type, argv[3], atom(env, "ignore"), argv[4],
                            atom(env, "undefined"), enif_is_identical(argv[5], atom(env, "true")));
}

static ERL_NIF_TERM nif_part_materialize(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    part_res *p;
    uint32_t type;
    if (argc != 7 || !get_part(env, argv[0], &p) || p->cached || !type_of(env, argv[2], &type))
        return enif_make_badarg(env);
    return part_read_common(env, p, argv[1], type, argv[3], argv[4], argv[5], argv[6], 0);
}

/* part_store(Part, Key, Type, CommitTimePairs, NewLastOp, Count, Value, Gc) ->
 * ok: materialize_snapshot's store (:466-509) of a snapshot the vnode
 * materialized from the log (get_from_snapshot_log, :416-419), on the
 * partition's device cache (agn_batcher_store); Gc = true for op_insert_gc's
 * GC read (a log response is never the newest, so only it stores) */
static ERL_NIF_TERM nif_part_store(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    part_res *p;
    uint32_t type;
    if (argc != 8 || !get_part(env, argv[0], &p) || !p->cached || !type_of(env, argv[2], &type))
        return enif_make_badarg(env);
    uint64_t k, row[256], mask[4];
    ErlNifSInt64 last_op = 0, value = 0;
    unsigned count = 0;
    int rc = key_index(env, p, argv[1], &k);
    if (!rc) rc = clock_row(env, p, argv[3], row, mask);
    if (rc == AGN_EINVAL || !enif_get_int64(env, argv[4], &last_op) ||
        !enif_get_uint(env, argv[5], &count))
        return enif_make_badarg(env);
    if (rc) return error_tuple(env, rc);
    uint32_t n = 0, *tags = NULL;
    uint64_t *toks = NULL;
    if (type == AGN_COUNTER_PN) {
        if (!enif_get_int64(env, argv[6], &value)) return enif_make_badarg(env);
    } else {
        rc = state_pairs(env, p, type, argv[6], &n, &tags, &toks);
        if (rc == AGN_EINVAL) return enif_make_badarg(env);
        if (rc) return error_tuple(env, rc);
    }
    const int gc = enif_is_identical(argv[7], atom(env, "true"));
    part_sub *sb;
    rc = sub_make(p, type, &sb);
    if (!rc)
        rc = agn_batcher_store(sb->bt, k, row, mask, last_op, count, value, n, tags, toks,
                               gc ? AGN_READ_GC : 0u);
    enif_free(tags);
    enif_free(toks);
    return rc ? error_tuple(env, rc) : atom(env, "ok");
}

/* part_gc(Part, Key, ThresholdPairs): snapshot_insert_gc's prune_ops over the
 * key's ops of every type (prune_ops filters the whole ETS tuple, :566-604) */
static ERL_NIF_TERM nif_part_gc(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    part_res *p;
    if (argc != 3 || !get_part(env, argv[0], &p)) return enif_make_badarg(env);
    uint64_t k, row[256], mask[4];
    int rc = key_index(env, p, argv[1], &k);
    if (!rc) rc = clock_row(env, p, argv[2], row, mask);
    if (rc == AGN_EINVAL) return enif_make_badarg(env);
    if (rc) return error_tuple(env, rc);
    agn_ctx *c = p->ctx->ctx;
    const uint8_t one = 1;
    pthread_mutex_lock(&p->gc_mu);
    for (uint32_t t = AGN_COUNTER_PN; t <= AGN_REGISTER_MV && !rc; ++t) {
        part_sub *s = sub_get(p, t);
        uint32_t len = 0;
        if (!s) continue;
        rc = agn_oplog_key_meta(s->log, 1, &k, &len, NULL, NULL);
        if (rc || len == 0) continue;
        rc = agn_memset_d(c, s->d_prune, 0, p->K, NULL);
        if (!rc) rc = agn_memcpy_h2d(c, s->d_prune + k, &one, 1, NULL);
        if (!rc) rc = agn_memcpy_h2d(c, s->d_thr + k * p->D, row, p->D * 8, NULL);
        if (!rc) rc = agn_memcpy_h2d(c, s->d_thrm + k * p->W, mask, p->W * 8, NULL);
        if (!rc) rc = agn_stream_sync(c, NULL);
        if (!rc) rc = agn_oplog_prune(s->log, s->d_prune, s->d_thr, s->d_thrm, NULL, NULL);
        if (!rc) rc = agn_oplog_key_meta(s->log, 1, &k, &len, NULL, NULL);
        if (!rc && len == 0) inv_drop(p, k, t, 0);
    }
    pthread_mutex_unlock(&p->gc_mu);
    return rc ? error_tuple(env, rc) : atom(env, "ok");
}

static ERL_NIF_TERM nif_part_gc_due(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    part_res *p;
    uint32_t type;
    uint64_t k;
    if (argc != 3 || !get_part(env, argv[0], &p) || !type_of(env, argv[2], &type))
        return enif_make_badarg(env);
    int rc = key_index(env, p, argv[1], &k);
    if (rc) return error_tuple(env, rc);
    /* op_insert_gc's trigger for the key's next op (:635) on the ONE tuple the
     * reference keeps per key: Length = its ops of every type, ListLen = the
     * home type's log's, NewId = the shared counter + 1.  For a key whose ops
     * are all of one type this is that log's own agn_oplog_gc_due.  A key
     * with no op yet (id 1, Length 0 < ListLen) is not due; nor is the op
     * Type's own -- the trigger does not depend on the new op's type. */
    (void)type;
    uint8_t due = 0;
    if (p->khome[k] != NO_HOME) {
        uint32_t total = 0, lcap = 0;
        for (uint32_t t = AGN_COUNTER_PN; t <= AGN_REGISTER_MV && !rc; ++t) {
            part_sub *s = sub_get(p, t);
            uint32_t len = 0, ll = 0;
            if (!s) continue;
            rc = agn_oplog_key_meta(s->log, 1, &k, &len, &ll, NULL);
            total += len;
            if (t == p->khome[k]) lcap = ll;
        }
        if (rc) return error_tuple(env, rc);
        const uint32_t list_len = lcap > AGN_OPS_THRESHOLD ? lcap : AGN_OPS_THRESHOLD;
        due = total >= list_len || (p->kcnt[k] + 1u) % AGN_OPS_THRESHOLD == 0;
    }
    return atom(env, due ? "true" : "false");
}

static ERL_NIF_TERM nif_part_stats(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    part_res *p;
    uint64_t E = 0, S = 0, T = 0;
    if (argc != 1 || !get_part(env, argv[0], &p)) return enif_make_badarg(env);
    for (uint32_t t = AGN_COUNTER_PN; t <= AGN_REGISTER_MV; ++t) {
        part_sub *s = sub_get(p, t);
        uint64_t e, sl, tk;
        if (!s) continue;
        int rc = agn_oplog_stats(s->log, &e, &sl, &tk);
        if (rc) return error_tuple(env, rc);
        E += e;
        S += sl;
        T += tk;
    }
    return enif_make_tuple3(env, enif_make_uint64(env, E), enif_make_uint64(env, S),
                            enif_make_uint64(env, T));
}

static ERL_NIF_TERM nif_part_key_meta(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    part_res *p;
    uint32_t type;
    uint64_t k;
    uint32_t len = 0, ll = 0, ct = 0;
    if (argc != 3 || !get_part(env, argv[0], &p) || !type_of(env, argv[2], &type))
        return enif_make_badarg(env);
    int rc = key_index(env, p, argv[1], &k);
    part_sub *s = sub_get(p, type);
    if (!rc && s) rc = agn_oplog_key_meta(s->log, 1, &k, &len, &ll, &ct);
    if (rc) return error_tuple(env, rc);
    return enif_make_tuple3(env, enif_make_uint(env, len), enif_make_uint(env, ll),
                            enif_make_uint(env, ct));
}

static ErlNifFunc funcs[] = {
    {"open", 1, nif_open, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"part_open", 5, nif_part_open, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"part_update", 6, nif_part_update, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"part_read", 6, nif_part_read, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"part_materialize", 7, nif_part_materialize, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"part_gc", 3, nif_part_gc, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"part_store", 8, nif_part_store, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"part_gc_due", 3, nif_part_gc_due, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"part_stats", 1, nif_part_stats, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"part_key_meta", 3, nif_part_key_meta, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"materialize", 6, nif_materialize, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"gst_min", 5, nif_gst_min, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"select_base", 7, nif_select_base, ERL_NIF_DIRTY_JOB_IO_BOUND},
};

ERL_NIF_INIT(antidote_gpu_nif, funcs, load, NULL, NULL, NULL)
