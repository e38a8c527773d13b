/*
 * oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * A deliberately literal, sequential restatement of the reference Erlang
 * code, one key at a time, in the reference's own visiting order:
 *
 *   materialize/4              src/clocksi_materializer.erl:89-101
 *   materialize_intern(_perform) src/clocksi_materializer.erl:157-197
 *   is_op_in_snapshot/7        src/clocksi_materializer.erl:216-268
 *   belongs_to_snapshot_op/3   src/materializer.erl:101-106
 *   apply_operations/4         src/clocksi_materializer.erl:113-121
 *   update_snapshot/3          src/materializer.erl:51-58
 *   antidote_crdt_*:update/2   (antidote_crdt 0.1.2, restated in SURVEY.md §8(a) a5.1-a5.3)
 *   get_min_time/1             src/stable_time_functions.erl:51-85
 *   update_stable/3            src/meta_data_sender.erl:341-356
 *   get_smaller/2              src/vector_orddict.erl:74-87
 *
 * Vector clocks are Erlang dicts in the reference; here a clock is a dense
 * row of D words plus a presence bitmask (NULL = every DC present).  The
 * vectorclock 0.1.0 predicates read a missing entry as 0.
 *
 * CRDT state for set_aw / register_mv is folded SEQUENTIALLY, effect after
 * effect, exactly as apply_operations does; the HIP kernels instead resolve
 * tags order-aware in parallel, and parity proves the two agree.
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define W_OF(d) (((d) + 63u) / 64u)
/* entries of key k: [key_off[k], key_off[k] + KEY_N) (segments with key_len, else CSR) */
#define KEY_N(log, k) ((log)->key_len ? (log)->key_len[k] : (log)->key_off[(k) + 1] - (log)->key_off[k])

static inline int present(const uint64_t *mask, uint32_t d) {
    return mask == NULL || ((mask[d >> 6] >> (d & 63)) & 1u);
}
static inline uint64_t get_clock(const uint64_t *v, const uint64_t *m, uint32_t d) {
    return present(m, d) ? v[d] : 0; /* vectorclock:get_clock_of_dc: missing = 0 */
}

/* vectorclock:le(A, B): for all d in keys(A) U keys(B): A[d] <= B[d] (missing = 0).
 * DCs only in B compare 0 <= B[d], always true. */
int oracle_vc_le(uint32_t D, const uint64_t *a, const uint64_t *am, const uint64_t *b,
                 const uint64_t *bm) {
    for (uint32_t d = 0; d < D; ++d)
        if (present(am, d) && a[d] > get_clock(b, bm, d)) return 0;
    return 1;
}

/* vectorclock:all_dots_greater(A, B): for all d in keys(A) U keys(B): A[d] > B[d]. */
int oracle_vc_all_dots_greater(uint32_t D, const uint64_t *a, const uint64_t *am,
                               const uint64_t *b, const uint64_t *bm) {
    for (uint32_t d = 0; d < D; ++d) {
        if (!present(am, d) && !present(bm, d)) continue;
        if (!(get_clock(a, am, d) > get_clock(b, bm, d))) return 0;
    }
    return 1;
}

/* ------------------------------------------------------------------------ */
/* CRDT states for the sequential fold                                       */

typedef struct {
    uint32_t tag;     /* elem (set_aw) / value (register_mv) */
    uint64_t tok;
} pair_t;

typedef struct {
    pair_t *v;
    size_t n, cap;
} pairvec;

static void pv_push(pairvec *p, uint32_t tag, uint64_t tok) {
    if (p->n == p->cap) {
        p->cap = p->cap ? p->cap * 2 : 16;
        p->v = (pair_t *)realloc(p->v, p->cap * sizeof(pair_t));
    }
    p->v[p->n].tag = tag;
    p->v[p->n].tok = tok;
    p->n++;
}
static void pv_insert_at(pairvec *p, size_t at, uint32_t tag, uint64_t tok) {
    pv_push(p, 0, 0);
    memmove(p->v + at + 1, p->v + at, (p->n - 1 - at) * sizeof(pair_t));
    p->v[at].tag = tag;
    p->v[at].tok = tok;
}

static int tok_in(const uint64_t *list, uint32_t n, uint64_t t) {
    for (uint32_t i = 0; i < n; ++i)
        if (list[i] == t) return 1;
    return 0;
}

/* antidote_crdt_set_aw:update/2 for one effect entry {Elem, AddTokens, RemoveTokens}.
 * The state is the orddict [{Elem, [Token]}] flattened to pairs grouped by
 * elem (elems ascending, tokens in list order).  Per elem:
 * Tokens := (Tokens -- Remove) ++ Add; the elem disappears when empty. */
static void set_aw_apply(pairvec *st, uint32_t elem, uint64_t add_tok,
                         const uint64_t *rem, uint32_t n_rem) {
    size_t w = 0, insert_at = (size_t)-1;
    for (size_t r = 0; r < st->n; ++r) {
        pair_t p = st->v[r];
        if (p.tag == elem && tok_in(rem, n_rem, p.tok)) continue; /* Tokens -- Remove */
        st->v[w++] = p;
    }
    st->n = w;
    if (add_tok == 0) return;
    /* ++ Add: append after the elem's surviving tokens (or create the elem
     * at its sorted position). */
    for (size_t r = 0; r < st->n; ++r) {
        if (st->v[r].tag == elem) insert_at = r + 1;
        else if (st->v[r].tag > elem && insert_at == (size_t)-1) { insert_at = r; break; }
        else if (st->v[r].tag > elem) break;
    }
    if (insert_at == (size_t)-1) insert_at = st->n;
    pv_insert_at(st, insert_at, elem, add_tok);
}

/* antidote_crdt_register_mv:update/2: {Value, Token, Overridden} drops the
 * overridden tokens then insert_sorted({Value, Token}); {reset, Overridden}
 * only drops.  The list stays sorted by (value, token). */
static void register_mv_apply(pairvec *st, uint32_t value, uint64_t add_tok,
                              const uint64_t *ovr, uint32_t n_ovr) {
    size_t w = 0;
    for (size_t r = 0; r < st->n; ++r) {
        pair_t p = st->v[r];
        if (tok_in(ovr, n_ovr, p.tok)) continue;
        st->v[w++] = p;
    }
    st->n = w;
    if (add_tok == 0) return; /* reset */
    size_t at = 0;
    while (at < st->n && (st->v[at].tag < value ||
                          (st->v[at].tag == value && st->v[at].tok < add_tok)))
        ++at;
    pv_insert_at(st, at, value, add_tok);
}

/* ------------------------------------------------------------------------ */

static void materialize_one(const agn_log *log, const agn_read *req, agn_result *out,
                            uint64_t i, uint32_t *incl_buf) {
    const uint32_t D = log->n_dcs, W = W_OF(D);
    const uint64_t key = req->keys ? req->keys[i] : i;
    const uint64_t off = log->key_off[key], n = KEY_N(log, key);
    const uint64_t *R = req->R + i * D;
    const uint64_t *Rm = req->R_mask ? req->R_mask + i * W : NULL;
    int sct_ign = (req->sct == NULL) || (req->sct_ignore && req->sct_ignore[i]);
    const uint64_t *sct = sct_ign ? NULL : req->sct + i * D;
    const uint64_t *sctm = (sct_ign || !req->sct_mask) ? NULL : req->sct_mask + i * W;
    const uint64_t txid = req->txid ? req->txid[i] : 0;
    uint32_t flags = 0;

    /* materialize_intern_perform raises erlang:error(corrupted_ops_cache) on
     * the first visited op whose type differs (:174,190-191).  All ops are
     * visited, so this is "any op of the key has another type". */
    if (n > 0) {
        uint8_t kt = log->key_type ? log->key_type[key] : (uint8_t)log->crdt_type;
        if (kt != (uint8_t)req->req_type) {
            out->flags[i] = AGN_F_ERR_CORRUPTED;
            out->err_pos[i] = UINT32_MAX;
            return;
        }
    }

    /* LastOpCt starts as SnapshotCommitTime (materialize/4 passes it twice, :94-95). */
    uint64_t ct[256], ctm[4];
    int ct_ignore = sct_ign;
    if (!ct_ignore) {
        for (uint32_t d = 0; d < D; ++d) ct[d] = sct[d];
        for (uint32_t w = 0; w < W; ++w) ctm[w] = sctm ? sctm[w] : ~0ull;
    }
    /* FirstHole = get_first_id(Ops): id of the newest op, 0 if none (:49-63). */
    int64_t hole = n ? (int64_t)log->op_id[off + n - 1] : 0;
    int new_ss = 0;
    uint64_t n_incl = 0;

    /* newest -> oldest (tuple form: element(?FIRST_OP+Length-1-Location), :163-171) */
    for (uint64_t pos = n; pos-- > 0;) {
        const uint64_t e = off + pos;
        const uint64_t *oc = log->oc + e * D;
        const uint64_t *ocm = log->oc_mask ? log->oc_mask + e * W : NULL;
        /* belongs_to_snapshot_op(LastSnapshot, ...) or (TxId == op.txid)  (:219-220) */
        int not_in_prev = sct_ign ? 1 : !oracle_vc_le(D, oc, ocm, sct, sctm);
        if (txid != 0 && log->txid && log->txid[e] == txid) not_in_prev = 1;
        if (!not_in_prev) continue; /* {false, true, _}: already in the base snapshot */
        /* dict:fold over OpSSCommit (:235-258): every DC of the op must be in
         * the read snapshot with TimeSS >= TimeOp. */
        int result = 1;
        for (uint32_t d = 0; d < D; ++d) {
            if (!present(ocm, d)) continue;
            if (!present(Rm, d)) { result = 0; continue; } /* logger:error, false (:245-247) */
            if (R[d] < oc[d]) result = 0;
        }
        if (result) {
            /* NewTime: PrevTime2 (= OpSSCommit when PrevTime is ignore) with
             * every DC of the op max-merged in (dict:update, :249-256). */
            if (ct_ignore) {
                for (uint32_t d = 0; d < D; ++d) ct[d] = present(ocm, d) ? oc[d] : 0;
                for (uint32_t w = 0; w < W; ++w) ctm[w] = ocm ? ocm[w] : ~0ull;
                ct_ignore = 0;
            } else {
                for (uint32_t d = 0; d < D; ++d) {
                    if (!present(ocm, d)) continue;
                    int had = (ctm[d >> 6] >> (d & 63)) & 1u;
                    if (!had) { ct[d] = oc[d]; ctm[d >> 6] |= 1ull << (d & 63); }
                    else if (oc[d] > ct[d]) ct[d] = oc[d];
                }
            }
            new_ss = 1;
            incl_buf[n_incl++] = (uint32_t)pos; /* [Op | OpList]: ends oldest-first */
        } else {
            hole = (int64_t)log->op_id[e] - 1; /* {ok, OpList, LastOpCt, NewSS, OpId-1} */
        }
    }

    /* apply_operations over OpList, oldest first (:113-121). */
    uint32_t count = 0;
    uint32_t err = UINT32_MAX;
    if (log->crdt_type == AGN_COUNTER_PN) {
        int64_t v = req->base_value ? req->base_value[i] : 0;
        for (uint64_t j = n_incl; j-- > 0;) {
            const uint64_t e = off + incl_buf[j];
            if (log->eff[e] == AGN_EFFECT_INVALID) { err = (uint32_t)e; break; }
            v = (int64_t)((uint64_t)v + (uint64_t)log->eff[e]); /* S + E */
            ++count;
        }
        if (out->value) out->value[i] = v;
    } else {
        pairvec st = {0};
        if (req->base_off)
            for (uint64_t b = req->base_off[i]; b < req->base_off[i + 1]; ++b)
                pv_push(&st, req->base_tag[b], req->base_tok[b]);
        for (uint64_t j = n_incl; j-- > 0;) {
            const uint64_t e = off + incl_buf[j];
            const uint32_t *ro = log->rem_off;
            if (log->tag[e] == AGN_TAG_INVALID) { err = (uint32_t)e; break; }
            if (log->crdt_type == AGN_SET_AW)
                set_aw_apply(&st, log->tag[e], log->add_tok[e], log->rem_tok + ro[e],
                             ro[e + 1] - ro[e]);
            else
                register_mv_apply(&st, log->tag[e], log->add_tok[e], log->rem_tok + ro[e],
                                  ro[e + 1] - ro[e]);
            /* one Op may span several entries (same op_id): count it once */
            if (incl_buf[j] == 0 || log->op_id[e - 1] != log->op_id[e]) ++count;
        }
        if (err == UINT32_MAX) {
            uint64_t o = out->out_off[i], cap = out->out_off[i + 1] - o;
            if (st.n > cap) {
                flags |= AGN_F_ERR_CAPACITY;
            } else {
                for (size_t r = 0; r < st.n; ++r) {
                    out->out_tag[o + r] = st.v[r].tag;
                    out->out_tok[o + r] = st.v[r].tok;
                }
            }
            out->out_n[i] = (uint32_t)st.n;
        }
        free(st.v);
    }

    if (err != UINT32_MAX) flags |= AGN_F_ERR_UNEXPECTED;
    if (new_ss) flags |= AGN_F_NEWSS;
    if (ct_ignore) flags |= AGN_F_CT_IGNORE;
    out->flags[i] = flags;
    out->err_pos[i] = err;
    out->count[i] = count;
    out->hole[i] = hole;
    uint64_t *oct = out->lastct + i * D;
    for (uint32_t d = 0; d < D; ++d)
        oct[d] = ct_ignore ? 0 : (((ctm[d >> 6] >> (d & 63)) & 1u) ? ct[d] : 0);
    if (out->lastct_mask) {  /* the dict's DCs: bits of columns < D only */
        uint64_t *om = out->lastct_mask + i * W;
        for (uint32_t w = 0; w < W; ++w) {
            const uint32_t left = D - 64u * w;
            const uint64_t cols = left >= 64u ? ~0ull : ((1ull << left) - 1ull);
            om[w] = ct_ignore ? 0 : (ctm[w] & cols);
        }
    }
}

typedef struct {
    const agn_log *log;
    const agn_read *req;
    agn_result *out;
    uint64_t lo, hi;
    uint64_t max_n;
} job_t;

static void *run_job(void *arg) {
    job_t *j = (job_t *)arg;
    uint32_t *buf = (uint32_t *)malloc((j->max_n + 1) * sizeof(uint32_t));
    for (uint64_t i = j->lo; i < j->hi; ++i) materialize_one(j->log, j->req, j->out, i, buf);
    free(buf);
    return NULL;
}

int oracle_materialize(const agn_log *log, const agn_read *req, agn_result *out,
                       int n_threads) {
    if (!log || !req || !out || log->n_dcs == 0 || log->n_dcs > 256) return AGN_EINVAL;
    if (!req->keys && req->n_req != log->n_keys) return AGN_EINVAL;
    uint64_t max_n = 0;
    for (uint64_t k = 0; k < log->n_keys; ++k) {
        uint64_t n = KEY_N(log, k);
        if (n > max_n) max_n = n;
    }
    if (n_threads < 1) n_threads = 1;
    if ((uint64_t)n_threads > req->n_req) n_threads = req->n_req ? (int)req->n_req : 1;
    job_t *jobs = (job_t *)calloc((size_t)n_threads, sizeof(job_t));
    pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
    uint64_t per = (req->n_req + n_threads - 1) / n_threads;
    for (int t = 0; t < n_threads; ++t) {
        jobs[t].log = log;
        jobs[t].req = req;
        jobs[t].out = out;
        jobs[t].lo = per * t < req->n_req ? per * t : req->n_req;
        jobs[t].hi = per * (t + 1) < req->n_req ? per * (t + 1) : req->n_req;
        jobs[t].max_n = max_n;
        if (n_threads == 1) run_job(&jobs[t]);
        else pthread_create(&th[t], NULL, run_job, &jobs[t]);
    }
    if (n_threads > 1)
        for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
    return AGN_OK;
}

/* ------------------------------------------------------------------------ */
/* get_min_time/1 (src/stable_time_functions.erl:51-85): per DC, the min over
 * the partitions whose dict contains it; an `undefined` partition makes
 * every output DC 0.  Absent = UINT64_MAX, output word D = "all defined". */
int oracle_gst_min(uint32_t D, uint64_t P, uint64_t E, const uint64_t *clocks,
                   const uint8_t *defined, uint64_t *out, int finalize) {
    for (uint64_t e = 0; e < E; ++e) {
        uint64_t *o = out + e * (D + 1);
        for (uint32_t d = 0; d < D; ++d) o[d] = UINT64_MAX;
        o[D] = 1;
        for (uint64_t p = 0; p < P; ++p) {
            if (defined && !defined[e * P + p]) { o[D] = 0; continue; }
            const uint64_t *c = clocks + (e * P + p) * D;
            for (uint32_t d = 0; d < D; ++d)
                if (c[d] < o[d]) o[d] = c[d]; /* PrevTime >= Time -> store Time */
        }
        if (finalize && o[D] == 0)
            for (uint32_t d = 0; d < D; ++d)
                if (o[d] != UINT64_MAX) o[d] = 0; /* FoundUndefined (:78-82) */
    }
    return AGN_OK;
}

/* update_stable/3 with update_func_min/2: store Time iff Last is undefined
 * or Time >= Last; DCs absent from NewDict keep their last value. */
int oracle_update_stable(uint32_t D, uint64_t *last, const uint64_t *nw, int *changed) {
    int c = 0;
    for (uint32_t d = 0; d < D; ++d) {
        if (nw[d] == UINT64_MAX) continue;
        if (last[d] == UINT64_MAX || nw[d] >= last[d]) { last[d] = nw[d]; c = 1; }
    }
    if (changed) *changed = c;
    return AGN_OK;
}

/* ---- logging_vnode filter_terms_for_key (src/logging_vnode.erl:722-779) ----
 * Walk the records in log order.  Ops (dict TxId -> buffered updates):
 * handle_update appends the update to its transaction's list; handle_commit
 * takes the list (if any), and for every buffered update, if
 * check_max_time(SnapshotTime, Max) holds, dict:append(Key, #clocksi_payload{})
 * to CommittedOpsDict; then erases the transaction.  Each key's list ends up
 * in append order; op ids are base + position (reverse_and_add_op_id). */
typedef struct { uint64_t txid; int64_t head, tail; int used; } txslot;

int oracle_log_ingest(const agn_log_records *r, uint32_t crdt, uint32_t D, uint64_t K,
                      const uint64_t *max_t, const uint64_t *max_m, uint32_t base, agn_log *out) {
    const uint32_t W = W_OF(D);
    const uint64_t n = r->n;
    uint64_t T = 16;
    while (T < 2 * n + 2) T <<= 1;
    txslot *tab = (txslot *)calloc(T, sizeof(txslot));
    int64_t *next = (int64_t *)malloc((n + 1) * sizeof(int64_t));
    /* committed ops per key as linked lists of (update, commit) in append order */
    int64_t *khead = (int64_t *)malloc((K + 1) * sizeof(int64_t));
    int64_t *ktail = (int64_t *)malloc((K + 1) * sizeof(int64_t));
    int64_t *knext = (int64_t *)malloc((n + 1) * sizeof(int64_t));
    uint64_t *kcommit = (uint64_t *)malloc((n + 1) * sizeof(uint64_t));
    for (uint64_t k = 0; k < K; ++k) khead[k] = ktail[k] = -1;
    for (uint64_t x = 0; x < n; ++x) {
        const uint64_t t = r->txid[x];
        uint64_t s = (t * 0x9E3779B97F4A7C15ull >> 17) & (T - 1);
        while (tab[s].used && tab[s].txid != t) s = (s + 1) & (T - 1);
        if (r->kind[x] == AGN_REC_UPDATE) { /* dict:append(TxId, OpPayload, Ops) */
            if (!tab[s].used) { tab[s].used = 1; tab[s].txid = t; tab[s].head = tab[s].tail = -1; }
            next[x] = -1;
            if (tab[s].tail < 0) tab[s].head = (int64_t)x; else next[tab[s].tail] = (int64_t)x;
            tab[s].tail = (int64_t)x;
        } else if (r->kind[x] == AGN_REC_COMMIT) {
            if (!tab[s].used || tab[s].head < 0) continue; /* dict:find -> error */
            for (int64_t u = tab[s].head; u >= 0; u = next[u]) {
                const uint64_t k = r->key[u];
                /* A partition's log holds only its own keys: logging_vnode writes
                 * every update to the log of its key's partition
                 * (log_utilities:get_key_partition / get_preflist_from_key,
                 * src/log_utilities.erl:58-68; the log id is [Partition],
                 * src/materializer_vnode.erl:289-292), so the partition's key
                 * index space [0, K) covers its log.  A record outside it
                 * belongs to another partition's table and is not loaded here. */
                if (k >= K) continue;
                int ok = 1;
                if (max_t) /* check_max_time: vectorclock:le(SnapshotTime, Max) */
                    ok = oracle_vc_le(D, r->ss + x * D, r->ss_mask ? r->ss_mask + x * W : NULL,
                                      max_t + k * D, max_m ? max_m + k * W : NULL);
                if (!ok) continue;
                knext[u] = -1;
                kcommit[u] = x;
                if (ktail[k] < 0) khead[k] = u; else knext[ktail[k]] = u;
                ktail[k] = u;
            }
            tab[s].head = tab[s].tail = -1; /* dict:erase(TxId, Ops) */
        }
    }
    uint64_t *ko = (uint64_t *)out->key_off, *oc = (uint64_t *)out->oc, *om = (uint64_t *)out->oc_mask;
    uint32_t *id = (uint32_t *)out->op_id;
    uint64_t w = 0, rw = 0;
    ko[0] = 0;
    if (out->rem_off && crdt != AGN_COUNTER_PN) ((uint32_t *)out->rem_off)[0] = 0;
    for (uint64_t k = 0; k < K; ++k) {
        uint32_t rank = 0;
        for (int64_t u = khead[k]; u >= 0; u = knext[u], ++w, ++rank) {
            const uint64_t c = kcommit[u];
            for (uint32_t d = 0; d < D; ++d)
                oc[w * D + d] = d == r->commit_dc[c] ? r->commit_time[c] : r->ss[c * D + d];
            if (om) {
                for (uint32_t x2 = 0; x2 < W; ++x2) om[w * W + x2] = r->ss_mask ? r->ss_mask[c * W + x2] : ~0ull;
                om[w * W + (r->commit_dc[c] >> 6)] |= 1ull << (r->commit_dc[c] & 63);
                if (D % 64) om[w * W + W - 1] &= (1ull << (D % 64)) - 1ull;
            }
            id[w] = base + rank;
            if (out->txid) ((uint64_t *)out->txid)[w] = r->txid[u];
            if (crdt == AGN_COUNTER_PN) {
                ((int64_t *)out->eff)[w] = r->eff[u];
            } else {
                ((uint32_t *)out->tag)[w] = r->tag[u];
                ((uint64_t *)out->add_tok)[w] = r->add_tok[u];
                for (uint32_t q = r->rem_off[u]; q < r->rem_off[u + 1]; ++q)
                    ((uint64_t *)out->rem_tok)[rw++] = r->rem_tok[q];
                ((uint32_t *)out->rem_off)[w + 1] = (uint32_t)rw;
            }
        }
        ko[k + 1] = w;
    }
    out->crdt_type = crdt;
    out->n_dcs = D;
    out->n_keys = K;
    out->n_entries = w;
    free(tab); free(next); free(khead); free(ktail); free(knext); free(kcommit);
    return AGN_OK;
}

/* ---- snapshot cache: a literal walk of the Erlang, one request at a time ---- */
static void row_copy(uint64_t *dst, const uint64_t *src, uint32_t n) {
    for (uint32_t x = 0; x < n; ++x) dst[x] = src[x];
}
static void full_mask(uint64_t *m, uint32_t D) {
    for (uint32_t x = 0; x < W_OF(D); ++x)
        m[x] = (x + 1 < W_OF(D) || D % 64 == 0) ? ~0ull : ((1ull << (D % 64)) - 1ull);
}

/* get_from_snapshot_cache/5 (src/materializer_vnode.erl:384-413) with
 * vector_orddict:get_smaller/2 (src/vector_orddict.erl:74-87). */
int oracle_ss_lookup(agn_ss_cache *c, uint64_t n_req, const uint64_t *keys, const uint64_t *R,
                     const uint64_t *Rm, uint64_t *sct, uint64_t *sctm, uint8_t *sct_ign,
                     int64_t *base, uint8_t *first, uint8_t *status) {
    const uint32_t D = c->n_dcs, W = W_OF(D), S = c->slots;
    for (uint64_t i = 0; i < n_req; ++i) {
        const uint64_t k = keys ? keys[i] : i;
        if (c->n[k] == 0) { /* [] -> store the empty snapshot at vectorclock:new() */
            for (uint32_t d = 0; d < D; ++d) c->clock[k * S * D + d] = 0, sct[i * D + d] = 0;
            for (uint32_t x = 0; x < W; ++x) {
                if (c->clock_mask) c->clock_mask[k * S * W + x] = 0;
                if (sctm) sctm[i * W + x] = 0;
            }
            c->last_op[k * S] = 0;
            c->value[k * S] = 0;
            c->n[k] = 1;
            sct_ign[i] = 1, base[i] = 0, first[i] = 1, status[i] = AGN_SS_NEW;
            continue;
        }
        int found = -1;
        for (uint32_t j = 0; j < c->n[k] && found < 0; ++j) {
            const uint64_t row = k * S + j;
            if (oracle_vc_le(D, c->clock + row * D, c->clock_mask ? c->clock_mask + row * W : NULL,
                             R + i * D, Rm ? Rm + i * W : NULL))
                found = (int)j;
        }
        if (found >= 0) {
            const uint64_t row = k * S + (uint64_t)found;
            row_copy(sct + i * D, c->clock + row * D, D);
            if (sctm) {
                if (c->clock_mask) row_copy(sctm + i * W, c->clock_mask + row * W, W);
                else full_mask(sctm + i * W, D);
            }
        }
        sct_ign[i] = found >= 0 ? 0 : 1;
        base[i] = found >= 0 ? c->value[k * S + (uint64_t)found] : 0;
        first[i] = found == 0;
        status[i] = found >= 0 ? AGN_SS_HIT : AGN_SS_LOG;
    }
    return AGN_OK;
}

/* materialize_snapshot/7 (:466-509) -> internal_store_ss/5 (:341-364) ->
 * vector_orddict:insert_bigger/3 (src/vector_orddict.erl:126-140) ->
 * snapshot_insert_gc/4 (:513-563) up to the prune_ops call, whose threshold
 * (vectorclock:min of the kept clocks, missing = 0) is returned. */
int oracle_ss_store(agn_ss_cache *c, const agn_log *log, uint64_t n_req, const uint64_t *keys,
                    const uint8_t *is_first, const uint8_t *status, const uint8_t *should_gc,
                    const agn_result *res, const int64_t *handle, uint8_t *prune, uint64_t *thr,
                    uint64_t *thrm) {
    const uint32_t D = c->n_dcs, W = W_OF(D), S = c->slots;
    uint64_t *lst = (uint64_t *)malloc((size_t)(S + 1) * (D + W) * sizeof(uint64_t));
    int64_t *lop = (int64_t *)malloc((S + 1) * sizeof(int64_t));
    int64_t *lval = (int64_t *)malloc((S + 1) * sizeof(int64_t));
    for (uint64_t k = 0; k < c->n_keys; ++k) prune[k] = 0;
    for (uint64_t i = 0; i < n_req; ++i) {
        const uint64_t k = keys ? keys[i] : i;
        if (status[i] == AGN_SS_LOG) continue;
        if (KEY_N(log, k) == 0) continue; /* number_of_ops = 0 */
        const uint32_t fl = res->flags[i];
        if (fl & (AGN_F_ERR_UNEXPECTED | AGN_F_ERR_CORRUPTED | AGN_F_ERR_CAPACITY)) continue;
        if (fl & AGN_F_CT_IGNORE) continue; /* CommitTime == ignore */
        const int gc = should_gc && should_gc[i];
        const int refresh = (fl & AGN_F_NEWSS) && is_first[i] && res->count[i] >= AGN_MIN_OP_STORE_SS;
        if (!(refresh || gc)) continue;
        const int64_t new_op = res->hole[i], val = handle ? handle[i] : res->value[i];
        const uint32_t n = c->n[k];
        const int should_insert = n == 0 || new_op - c->last_op[k * S] >= AGN_MIN_OP_STORE_SS;
        if (!(should_insert || gc)) continue;
        /* SD as a list: rows of D clock words + W mask words */
        uint32_t m = 0;
        const uint64_t *ct = res->lastct + i * D;
        const uint64_t *ctm = res->lastct_mask ? res->lastct_mask + i * W : NULL;
        int prepend = n == 0 || !oracle_vc_le(D, ct, ctm, c->clock + k * S * D,
                                              c->clock_mask ? c->clock_mask + k * S * W : NULL);
        if (prepend) {
            row_copy(lst, ct, D);
            if (ctm) row_copy(lst + D, ctm, W); else full_mask(lst + D, D);
            lop[0] = new_op, lval[0] = val, m = 1;
        }
        for (uint32_t j = 0; j < n; ++j, ++m) {
            const uint64_t row = k * S + j;
            row_copy(lst + (size_t)m * (D + W), c->clock + row * D, D);
            if (c->clock_mask) row_copy(lst + (size_t)m * (D + W) + D, c->clock_mask + row * W, W);
            else full_mask(lst + (size_t)m * (D + W) + D, D);
            lop[m] = c->last_op[row], lval[m] = c->value[row];
        }
        if (m >= AGN_SNAPSHOT_THRESHOLD || gc) { /* sublist(SD1, 1, SNAPSHOT_MIN) */
            if (m > AGN_SNAPSHOT_MIN) m = AGN_SNAPSHOT_MIN;
            /* CommitTime = fold of vectorclock:min([CT1, Acc]) from the last entry */
            for (uint32_t d = 0; d < D; ++d) {
                uint64_t mn = UINT64_MAX;
                int any = 0;
                for (uint32_t j = 0; j < m; ++j) {
                    const uint64_t *r = lst + (size_t)j * (D + W);
                    const int p = (int)((r[D + (d >> 6)] >> (d & 63)) & 1u);
                    const uint64_t v = p ? r[d] : 0;
                    any |= p;
                    if (v < mn) mn = v;
                }
                thr[k * D + d] = any ? mn : 0;
                if (thrm) {
                    if (d % 64 == 0) thrm[k * W + (d >> 6)] = 0;
                    if (any) thrm[k * W + (d >> 6)] |= 1ull << (d & 63);
                }
            }
            prune[k] = 1;
        }
        for (uint32_t j = 0; j < m; ++j) {
            const uint64_t row = k * S + j;
            row_copy(c->clock + row * D, lst + (size_t)j * (D + W), D);
            if (c->clock_mask) row_copy(c->clock_mask + row * W, lst + (size_t)j * (D + W) + D, W);
            c->last_op[row] = lop[j];
            c->value[row] = lval[j];
        }
        c->n[k] = m;
    }
    free(lst);
    free(lop);
    free(lval);
    return AGN_OK;
}

/* prune_ops/2 + check_filter/7 (src/materializer_vnode.erl:566-604): walk the
 * key's ops oldest first and keep those for which
 * belongs_to_snapshot_op(Threshold, CommitTime, SnapshotTime) holds, i.e.
 * not le(OpSSCommit, Threshold).  A key whose every op is covered keeps no
 * entry and is flagged (the reference stores the empty slot after the last
 * op, :580-583). */
int oracle_prune_ops(const agn_log *log, const uint8_t *prune, const uint64_t *thr,
                     const uint64_t *thr_mask, agn_log *out, uint32_t *out_flags) {
    const uint32_t D = log->n_dcs, W = W_OF(D);
    uint64_t *ko = (uint64_t *)out->key_off;
    uint64_t *oc = (uint64_t *)out->oc, *om = (uint64_t *)out->oc_mask;
    uint32_t *id = (uint32_t *)out->op_id, *tag = (uint32_t *)out->tag;
    uint64_t *tx = (uint64_t *)out->txid, *add = (uint64_t *)out->add_tok;
    int64_t *eff = (int64_t *)out->eff;
    uint32_t *ro = (uint32_t *)out->rem_off;
    uint64_t *rt = (uint64_t *)out->rem_tok;
    uint64_t w = 0, rw = 0;
    ko[0] = 0;
    if (ro) ro[0] = 0;
    for (uint64_t k = 0; k < log->n_keys; ++k) {
        const int gc = prune == NULL || prune[k] != 0;
        const uint64_t *t = thr + k * D, *tm = thr_mask ? thr_mask + k * W : NULL;
        uint64_t kept = 0;
        for (uint64_t e = log->key_off[k]; e < log->key_off[k] + KEY_N(log, k); ++e) {
            const uint64_t *o = log->oc + e * D, *m = log->oc_mask ? log->oc_mask + e * W : NULL;
            if (gc && oracle_vc_le(D, o, m, t, tm)) continue; /* already in the snapshot */
            for (uint32_t d = 0; d < D; ++d) oc[w * D + d] = o[d];
            if (om) for (uint32_t x = 0; x < W; ++x) om[w * W + x] = m[x];
            id[w] = log->op_id[e];
            if (tx) tx[w] = log->txid[e];
            if (eff) eff[w] = log->eff[e];
            if (tag) tag[w] = log->tag[e];
            if (add) add[w] = log->add_tok[e];
            if (ro) {
                for (uint32_t r = log->rem_off[e]; r < log->rem_off[e + 1]; ++r) rt[rw++] = log->rem_tok[r];
                ro[w + 1] = (uint32_t)rw;
            }
            ++w;
            ++kept;
        }
        ko[k + 1] = w;
        if (out_flags)
            out_flags[k] = (gc && kept == 0) ? AGN_GC_ALL_PRUNED : 0u;
    }
    out->n_entries = w;
    return AGN_OK;
}

/* Gentlerain (src/dc_utilities.erl:287-320): GST = lists:min of the values of
 * the stable dict; get_stable_snapshot's gr branch maps every entry to GST. */
int oracle_gst_scalar(uint32_t D, uint64_t E, uint64_t *vec, uint64_t *out_gst) {
    for (uint64_t e = 0; e < E; ++e) {
        uint64_t *row = vec + e * (D + 1);
        uint64_t gst = UINT64_MAX;
        for (uint32_t d = 0; d < D; ++d)
            if (row[d] != UINT64_MAX && row[d] < gst) gst = row[d];
        if (gst != UINT64_MAX)
            for (uint32_t d = 0; d < D; ++d)
                if (row[d] != UINT64_MAX) row[d] = gst; /* dict:map(fun(_K,_V) -> GST end) */
        if (out_gst) out_gst[e] = gst;
    }
    return AGN_OK;
}

/* try_store/2 (src/inter_dc_dep_vnode.erl:128-155): Deps = set_clock_of_dc(DCID, 0,
 * snapshot), Cur = set_clock_of_dc(DCID, 0, partition clock), ok = ge(Cur, Deps)
 * = le(Deps, Cur): every DC of Deps (except the origin, now 0) <= Cur (missing = 0). */
int oracle_dep_check(uint32_t D, uint64_t n, const uint64_t *deps, const uint64_t *dm,
                     const uint32_t *origin, const uint32_t *part, uint64_t n_parts,
                     const uint64_t *pc, const uint64_t *pm, uint8_t *ok) {
    const uint32_t W = W_OF(D);
    for (uint64_t t = 0; t < n; ++t) {
        const uint64_t p = part[t];
        if (p >= n_parts) return AGN_EINVAL;
        const uint64_t *a = deps + t * D, *am = dm ? dm + t * W : NULL;
        const uint64_t *b = pc + p * D, *bm = pm ? pm + p * W : NULL;
        int r = 1;
        for (uint32_t d = 0; d < D && r; ++d) {
            if (d == origin[t]) continue; /* both sides 0 */
            if (present(am, d) && a[d] > get_clock(b, bm, d)) r = 0;
        }
        ok[t] = (uint8_t)r;
    }
    return AGN_OK;
}

/* get_smaller/2: first (newest) entry whose clock is le the read clock;
 * IsFirst is true until the walk moves past the head (:78-87). */
int oracle_select_base(uint32_t D, uint64_t n_req, const uint64_t *cache_off,
                       const uint64_t *clocks, const uint64_t *clock_mask,
                       const uint64_t *R, const uint64_t *R_mask, int32_t *out_idx,
                       uint8_t *out_is_first) {
    const uint32_t W = W_OF(D);
    for (uint64_t i = 0; i < n_req; ++i) {
        int32_t idx = -1;
        uint8_t first = 1;
        for (uint64_t c = cache_off[i]; c < cache_off[i + 1]; ++c) {
            if (oracle_vc_le(D, clocks + c * D, clock_mask ? clock_mask + c * W : NULL,
                             R + i * D, R_mask ? R_mask + i * W : NULL)) {
                idx = (int32_t)(c - cache_off[i]);
                break;
            }
            first = 0;
        }
        out_idx[i] = idx;
        out_is_first[i] = first;
    }
    return AGN_OK;
}
