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

static ErlNifResourceType *CTX_RES;

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

static int load(ErlNifEnv *env, void **priv, ERL_NIF_TERM info) {
    (void)priv;
    (void)info;
    CTX_RES = enif_open_resource_type(env, NULL, "agn_ctx", ctx_dtor, ERL_NIF_RT_CREATE, NULL);
    return CTX_RES == NULL;
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

static ErlNifFunc funcs[] = {
    {"open", 1, nif_open, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"materialize", 6, nif_materialize, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"gst_min", 5, nif_gst_min, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"select_base", 7, nif_select_base, ERL_NIF_DIRTY_JOB_IO_BOUND},
};

ERL_NIF_INIT(antidote_gpu_nif, funcs, load, NULL, NULL, NULL)
