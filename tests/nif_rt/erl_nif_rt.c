/*
 * erl_nif_rt.c -- a minimal erl_nif term runtime.  TEST INFRASTRUCTURE ONLY.
 *
 * Links with nif/antidote_gpu_nif.c (against tests/nif_rt/erl_nif.h) into
 * tests/nif_rt/libagn_nif_rt.so so the NIF's own C -- term decoding,
 * interning, error terms, enif_raise_exception, resources and their
 * destructors -- runs in the tests without Erlang/OTP (none in this image).
 *
 * Terms: integers (arbitrary within 128 bits), atoms (interned: one term per
 * name), tuples, proper/improper lists (cons cells + nil), binaries and
 * resource references.  A term lives in the environment that made it (an
 * arena freed with the environment); a resource term holds a reference on
 * its resource, released with the environment, so a resource's destructor
 * runs when the last reference goes (enif_release_resource / rt_release).
 *
 * enif_term_to_binary / enif_binary_to_term use this runtime's own external
 * format -- injective, so the NIF's exact interning of keys, DCs, TxIds,
 * elements and tokens holds as with OTP's -- which is also the ctypes
 * boundary (rt_decode / rt_encode; tests/nif_rt/terms.py mirrors it):
 *   'I' int128 LE | 'A' u32 len, name | 'T' u32 arity, elems | 'N' nil |
 *   'L' head, tail | 'B' u32 len, bytes | 'R' u64 resource
 */
#include <stdarg.h>
#include <stdatomic.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "erl_nif.h"

typedef __int128 i128;

enum { K_INT = 1, K_ATOM, K_TUPLE, K_NIL, K_CONS, K_BIN, K_RES, K_EXC };

struct rt_res;
typedef struct term {
    int k;
    union {
        i128 i;
        struct { size_t n; char *s; } atom;
        struct { unsigned n; ERL_NIF_TERM *e; } tup;
        struct { ERL_NIF_TERM h, t; } cons;
        struct { size_t n; unsigned char *d; } bin;
        struct rt_res *res;
    } u;
} term;

struct enif_resource_type_t {
    char name[64];
    ErlNifResourceDtor *dtor;
};

typedef struct rt_res {
    ErlNifResourceType *type;
    atomic_long refc;
    size_t size;
    _Alignas(16) unsigned char data[];
} rt_res;

static atomic_long g_live_res;

/* ---- environments: arenas of blocks ------------------------------------ */
typedef struct blk {
    struct blk *next;
    _Alignas(16) unsigned char data[];
} blk;

struct enif_environment_t {
    blk *blocks;
    rt_res **held;          /* resource references held by this env's terms */
    size_t n_held, cap_held;
    int exc;                /* 0, 1 = badarg, 2 = raised */
    ERL_NIF_TERM reason;
};

static void *env_alloc(ErlNifEnv *env, size_t n) {
    blk *b = malloc(sizeof(blk) + (n ? n : 1));
    if (!b) abort();
    b->next = env->blocks;
    env->blocks = b;
    return b->data;
}

static term *mk(ErlNifEnv *env, int k) {
    term *t = env_alloc(env, sizeof(term));
    memset(t, 0, sizeof *t);
    t->k = k;
    return t;
}
#define T(x) ((term *)(uintptr_t)(x))
#define H(t) ((ERL_NIF_TERM)(uintptr_t)(t))

static void hold(ErlNifEnv *env, rt_res *r) {
    if (env->n_held == env->cap_held) {
        env->cap_held = env->cap_held ? 2 * env->cap_held : 8;
        env->held = realloc(env->held, env->cap_held * sizeof *env->held);
        if (!env->held) abort();
    }
    atomic_fetch_add(&r->refc, 1);
    env->held[env->n_held++] = r;
}

static void res_release(rt_res *r) {
    if (atomic_fetch_sub(&r->refc, 1) == 1) {
        if (r->type->dtor) r->type->dtor(NULL, r->data);
        atomic_fetch_sub(&g_live_res, 1);
        free(r);
    }
}

/* ---- atoms: one global term per name ----------------------------------- */
static pthread_mutex_t g_atom_mu = PTHREAD_MUTEX_INITIALIZER;
static ErlNifEnv g_atom_env;

static ERL_NIF_TERM atom_n(const char *s, size_t n) {
    pthread_mutex_lock(&g_atom_mu);
    for (blk *b = g_atom_env.blocks; b; b = b->next) {
        term *t = (term *)b->data;
        if (t->k == K_ATOM && t->u.atom.n == n && memcmp(t->u.atom.s, s, n) == 0) {
            pthread_mutex_unlock(&g_atom_mu);
            return H(t);
        }
    }
    blk *b = malloc(sizeof(blk) + sizeof(term) + n + 1);
    if (!b) abort();
    term *t = (term *)b->data;
    memset(t, 0, sizeof *t);
    t->k = K_ATOM;
    t->u.atom.n = n;
    t->u.atom.s = (char *)(t + 1);
    memcpy(t->u.atom.s, s, n);
    t->u.atom.s[n] = 0;
    b->next = g_atom_env.blocks;
    g_atom_env.blocks = b;
    pthread_mutex_unlock(&g_atom_mu);
    return H(t);
}

/* ---- the erl_nif API subset --------------------------------------------- */
ERL_NIF_TERM enif_make_atom(ErlNifEnv *env, const char *name) {
    (void)env;
    return atom_n(name, strlen(name));
}

ERL_NIF_TERM enif_make_badarg(ErlNifEnv *env) {
    env->exc = 1;
    env->reason = enif_make_atom(env, "badarg");
    return H(mk(env, K_EXC));
}

ERL_NIF_TERM enif_raise_exception(ErlNifEnv *env, ERL_NIF_TERM reason) {
    env->exc = 2;
    env->reason = reason;
    return H(mk(env, K_EXC));
}

ERL_NIF_TERM enif_make_tuple_from_array(ErlNifEnv *env, const ERL_NIF_TERM arr[], unsigned cnt) {
    term *t = mk(env, K_TUPLE);
    t->u.tup.n = cnt;
    t->u.tup.e = env_alloc(env, cnt * sizeof(ERL_NIF_TERM));
    memcpy(t->u.tup.e, arr, cnt * sizeof(ERL_NIF_TERM));
    return H(t);
}

ERL_NIF_TERM enif_make_tuple2(ErlNifEnv *env, ERL_NIF_TERM e1, ERL_NIF_TERM e2) {
    const ERL_NIF_TERM a[2] = {e1, e2};
    return enif_make_tuple_from_array(env, a, 2);
}

ERL_NIF_TERM enif_make_tuple3(ErlNifEnv *env, ERL_NIF_TERM e1, ERL_NIF_TERM e2, ERL_NIF_TERM e3) {
    const ERL_NIF_TERM a[3] = {e1, e2, e3};
    return enif_make_tuple_from_array(env, a, 3);
}

ERL_NIF_TERM enif_make_list_cell(ErlNifEnv *env, ERL_NIF_TERM head, ERL_NIF_TERM tail) {
    term *t = mk(env, K_CONS);
    t->u.cons.h = head;
    t->u.cons.t = tail;
    return H(t);
}

ERL_NIF_TERM enif_make_list(ErlNifEnv *env, unsigned cnt, ...) {
    ERL_NIF_TERM *e = cnt ? malloc(cnt * sizeof *e) : NULL;
    va_list ap;
    va_start(ap, cnt);
    for (unsigned i = 0; i < cnt; ++i) e[i] = va_arg(ap, ERL_NIF_TERM);
    va_end(ap);
    ERL_NIF_TERM l = H(mk(env, K_NIL));
    for (unsigned i = cnt; i-- > 0;) l = enif_make_list_cell(env, e[i], l);
    free(e);
    return l;
}

static ERL_NIF_TERM make_int(ErlNifEnv *env, i128 v) {
    term *t = mk(env, K_INT);
    t->u.i = v;
    return H(t);
}
ERL_NIF_TERM enif_make_uint(ErlNifEnv *env, unsigned i) { return make_int(env, i); }
ERL_NIF_TERM enif_make_uint64(ErlNifEnv *env, ErlNifUInt64 i) { return make_int(env, i); }
ERL_NIF_TERM enif_make_int64(ErlNifEnv *env, ErlNifSInt64 i) { return make_int(env, i); }

unsigned char *enif_make_new_binary(ErlNifEnv *env, size_t size, ERL_NIF_TERM *termp) {
    term *t = mk(env, K_BIN);
    t->u.bin.n = size;
    t->u.bin.d = env_alloc(env, size);
    *termp = H(t);
    return t->u.bin.d;
}

ERL_NIF_TERM enif_make_resource(ErlNifEnv *env, void *obj) {
    rt_res *r = (rt_res *)((unsigned char *)obj - offsetof(rt_res, data));
    term *t = mk(env, K_RES);
    t->u.res = r;
    hold(env, r);
    return H(t);
}

static int get_i128(ERL_NIF_TERM x, i128 *v) {
    if (!x || T(x)->k != K_INT) return 0;
    *v = T(x)->u.i;
    return 1;
}
int enif_get_int(ErlNifEnv *env, ERL_NIF_TERM x, int *ip) {
    (void)env;
    i128 v;
    if (!get_i128(x, &v) || v < INT32_MIN || v > INT32_MAX) return 0;
    *ip = (int)v;
    return 1;
}
int enif_get_uint(ErlNifEnv *env, ERL_NIF_TERM x, unsigned *ip) {
    (void)env;
    i128 v;
    if (!get_i128(x, &v) || v < 0 || v > UINT32_MAX) return 0;
    *ip = (unsigned)v;
    return 1;
}
int enif_get_uint64(ErlNifEnv *env, ERL_NIF_TERM x, ErlNifUInt64 *ip) {
    (void)env;
    i128 v;
    if (!get_i128(x, &v) || v < 0 || v > (i128)UINT64_MAX) return 0;
    *ip = (ErlNifUInt64)v;
    return 1;
}
int enif_get_int64(ErlNifEnv *env, ERL_NIF_TERM x, ErlNifSInt64 *ip) {
    (void)env;
    i128 v;
    if (!get_i128(x, &v) || v < INT64_MIN || v > INT64_MAX) return 0;
    *ip = (ErlNifSInt64)v;
    return 1;
}

int enif_get_tuple(ErlNifEnv *env, ERL_NIF_TERM x, int *arity, const ERL_NIF_TERM **array) {
    (void)env;
    if (!x || T(x)->k != K_TUPLE) return 0;
    *arity = (int)T(x)->u.tup.n;
    *array = T(x)->u.tup.e;
    return 1;
}

int enif_get_list_cell(ErlNifEnv *env, ERL_NIF_TERM x, ERL_NIF_TERM *head, ERL_NIF_TERM *tail) {
    (void)env;
    if (!x || T(x)->k != K_CONS) return 0;
    *head = T(x)->u.cons.h;
    *tail = T(x)->u.cons.t;
    return 1;
}

int enif_get_list_length(ErlNifEnv *env, ERL_NIF_TERM x, unsigned *len) {
    (void)env;
    unsigned n = 0;
    while (x && T(x)->k == K_CONS) {
        ++n;
        x = T(x)->u.cons.t;
    }
    if (!x || T(x)->k != K_NIL) return 0;  /* improper */
    *len = n;
    return 1;
}

int enif_is_empty_list(ErlNifEnv *env, ERL_NIF_TERM x) {
    (void)env;
    return x && T(x)->k == K_NIL;
}

int enif_is_list(ErlNifEnv *env, ERL_NIF_TERM x) {
    (void)env;
    return x && (T(x)->k == K_NIL || T(x)->k == K_CONS);
}

int enif_is_identical(ERL_NIF_TERM a, ERL_NIF_TERM b) {
    for (;;) {
        if (a == b) return 1;
        if (!a || !b || T(a)->k != T(b)->k) return 0;
        const term *x = T(a), *y = T(b);
        switch (x->k) {
            case K_INT: return x->u.i == y->u.i;
            case K_ATOM: return 0;  /* interned: equal names share the term */
            case K_NIL: return 1;
            case K_BIN: return x->u.bin.n == y->u.bin.n &&
                               memcmp(x->u.bin.d, y->u.bin.d, x->u.bin.n) == 0;
            case K_RES: return x->u.res == y->u.res;
            case K_TUPLE:
                if (x->u.tup.n != y->u.tup.n) return 0;
                for (unsigned i = 0; i < x->u.tup.n; ++i)
                    if (!enif_is_identical(x->u.tup.e[i], y->u.tup.e[i])) return 0;
                return 1;
            case K_CONS:
                if (!enif_is_identical(x->u.cons.h, y->u.cons.h)) return 0;
                a = x->u.cons.t;
                b = y->u.cons.t;
                continue;
            default: return 0;
        }
    }
}

/* Erlang's standard term order (number < atom < ... < tuple < nil < list <
 * binary, as far as this runtime's kinds go): tuples by size then elements,
 * lists element by element, atoms and binaries bytewise */
static int kind_rank(int k) {
    switch (k) {
        case K_INT: return 0;
        case K_ATOM: return 1;
        case K_RES: return 2;   /* a reference */
        case K_TUPLE: return 3;
        case K_NIL: return 4;
        case K_CONS: return 5;
        case K_BIN: return 6;
    }
    return 7;
}

static int cmp_bytes(const void *a, size_t na, const void *b, size_t nb) {
    const int c = memcmp(a, b, na < nb ? na : nb);
    if (c) return c < 0 ? -1 : 1;
    return na < nb ? -1 : na > nb;
}

int enif_compare(ERL_NIF_TERM a, ERL_NIF_TERM b) {
    for (;;) {
        if (a == b) return 0;
        const term *x = T(a), *y = T(b);
        const int rx = kind_rank(x->k), ry = kind_rank(y->k);
        if (rx != ry) return rx < ry ? -1 : 1;
        switch (x->k) {
            case K_INT: return x->u.i < y->u.i ? -1 : x->u.i > y->u.i;
            case K_ATOM: return cmp_bytes(x->u.atom.s, x->u.atom.n, y->u.atom.s, y->u.atom.n);
            case K_BIN: return cmp_bytes(x->u.bin.d, x->u.bin.n, y->u.bin.d, y->u.bin.n);
            case K_RES: return x->u.res < y->u.res ? -1 : x->u.res > y->u.res;
            case K_NIL: return 0;
            case K_TUPLE:
                if (x->u.tup.n != y->u.tup.n) return x->u.tup.n < y->u.tup.n ? -1 : 1;
                for (unsigned i = 0; i < x->u.tup.n; ++i) {
                    const int c = enif_compare(x->u.tup.e[i], y->u.tup.e[i]);
                    if (c) return c;
                }
                return 0;
            case K_CONS: {
                const int c = enif_compare(x->u.cons.h, y->u.cons.h);
                if (c) return c;
                a = x->u.cons.t;
                b = y->u.cons.t;
                continue;
            }
        }
        return 0;
    }
}

int enif_inspect_binary(ErlNifEnv *env, ERL_NIF_TERM x, ErlNifBinary *bin) {
    (void)env;
    if (!x || T(x)->k != K_BIN) return 0;
    memset(bin, 0, sizeof *bin);
    bin->size = T(x)->u.bin.n;
    bin->data = T(x)->u.bin.d;
    return 1;
}

/* ---- external format ------------------------------------------------------ */
typedef struct {
    unsigned char *d;
    size_t n, cap;
} buf;

static void put(buf *b, const void *p, size_t n) {
    if (b->n + n > b->cap) {
        b->cap = (b->n + n) * 2 + 64;
        b->d = realloc(b->d, b->cap);
        if (!b->d) abort();
    }
    memcpy(b->d + b->n, p, n);
    b->n += n;
}
static void put_u32(buf *b, uint32_t v) { put(b, &v, 4); }

static int enc(buf *b, ERL_NIF_TERM x) {
    while (x && T(x)->k == K_CONS) {  /* lists iteratively */
        put(b, "L", 1);
        if (!enc(b, T(x)->u.cons.h)) return 0;
        x = T(x)->u.cons.t;
    }
    if (!x) return 0;
    const term *t = T(x);
    switch (t->k) {
        case K_INT: put(b, "I", 1); put(b, &t->u.i, 16); return 1;
        case K_ATOM: put(b, "A", 1); put_u32(b, (uint32_t)t->u.atom.n);
                     put(b, t->u.atom.s, t->u.atom.n); return 1;
        case K_NIL: put(b, "N", 1); return 1;
        case K_BIN: put(b, "B", 1); put_u32(b, (uint32_t)t->u.bin.n);
                    put(b, t->u.bin.d, t->u.bin.n); return 1;
        case K_RES: {
            uint64_t p = (uint64_t)(uintptr_t)t->u.res;
            put(b, "R", 1); put(b, &p, 8); return 1;
        }
        case K_TUPLE:
            put(b, "T", 1); put_u32(b, t->u.tup.n);
            for (unsigned i = 0; i < t->u.tup.n; ++i)
                if (!enc(b, t->u.tup.e[i])) return 0;
            return 1;
    }
    return 0;
}

static int get(const unsigned char **p, const unsigned char *end, void *out, size_t n) {
    if ((size_t)(end - *p) < n) return 0;
    memcpy(out, *p, n);
    *p += n;
    return 1;
}

static ERL_NIF_TERM dec(ErlNifEnv *env, const unsigned char **p, const unsigned char *end,
                        int depth) {
    if (depth > 10000) return 0;
    unsigned char tag;
    if (!get(p, end, &tag, 1)) return 0;
    uint32_t n;
    switch (tag) {
        case 'I': {
            i128 v;
            return get(p, end, &v, 16) ? make_int(env, v) : 0;
        }
        case 'A':
            if (!get(p, end, &n, 4) || (size_t)(end - *p) < n) return 0;
            *p += n;
            return atom_n((const char *)*p - n, n);
        case 'N': return H(mk(env, K_NIL));
        case 'B': {
            ERL_NIF_TERM t;
            if (!get(p, end, &n, 4) || (size_t)(end - *p) < n) return 0;
            unsigned char *d = enif_make_new_binary(env, n, &t);
            memcpy(d, *p, n);
            *p += n;
            return t;
        }
        case 'R': {
            uint64_t r;
            if (!get(p, end, &r, 8) || !r) return 0;
            term *t = mk(env, K_RES);
            t->u.res = (rt_res *)(uintptr_t)r;
            hold(env, t->u.res);
            return H(t);
        }
        case 'T': {
            if (!get(p, end, &n, 4)) return 0;
            ERL_NIF_TERM *e = n ? malloc(n * sizeof *e) : NULL;
            for (uint32_t i = 0; i < n; ++i)
                if (!(e[i] = dec(env, p, end, depth + 1))) {
                    free(e);
                    return 0;
                }
            ERL_NIF_TERM t = enif_make_tuple_from_array(env, e, n);
            free(e);
            return t;
        }
        case 'L': {  /* a run of cons cells, iteratively */
            term *first = NULL, *last = NULL;
            --*p;
            while (*p < end && **p == 'L') {
                ++*p;
                ERL_NIF_TERM h = dec(env, p, end, depth + 1);
                if (!h) return 0;
                term *c = mk(env, K_CONS);
                c->u.cons.h = h;
                if (last) last->u.cons.t = H(c); else first = c;
                last = c;
            }
            ERL_NIF_TERM tail = dec(env, p, end, depth + 1);
            if (!tail) return 0;
            last->u.cons.t = tail;
            return H(first);
        }
    }
    return 0;
}

int enif_term_to_binary(ErlNifEnv *env, ERL_NIF_TERM x, ErlNifBinary *bin) {
    (void)env;
    buf b = {0, 0, 0};
    if (!enc(&b, x)) {
        free(b.d);
        return 0;
    }
    memset(bin, 0, sizeof *bin);
    bin->size = b.n;
    bin->data = b.d;
    return 1;
}

size_t enif_binary_to_term(ErlNifEnv *env, const unsigned char *data, size_t size,
                           ERL_NIF_TERM *out, unsigned opts) {
    (void)opts;
    const unsigned char *p = data;
    ERL_NIF_TERM t = dec(env, &p, data + size, 0);
    if (!t) return 0;
    *out = t;
    return (size_t)(p - data);
}

void enif_release_binary(ErlNifBinary *bin) {
    free(bin->data);
    bin->data = NULL;
    bin->size = 0;
}

/* ---- resources ----------------------------------------------------------- */
ErlNifResourceType *enif_open_resource_type(ErlNifEnv *env, const char *module_str,
                                            const char *name, ErlNifResourceDtor *dtor,
                                            ErlNifResourceFlags flags, ErlNifResourceFlags *tried) {
    (void)env;
    (void)module_str;
    if (tried) *tried = flags;
    ErlNifResourceType *t = calloc(1, sizeof *t);
    if (!t) return NULL;
    strncpy(t->name, name, sizeof t->name - 1);
    t->dtor = dtor;
    return t;
}

void *enif_alloc_resource(ErlNifResourceType *type, size_t size) {
    rt_res *r = malloc(sizeof(rt_res) + size);
    if (!r) return NULL;
    r->type = type;
    atomic_init(&r->refc, 1);
    r->size = size;
    atomic_fetch_add(&g_live_res, 1);
    return r->data;
}

int enif_get_resource(ErlNifEnv *env, ERL_NIF_TERM x, ErlNifResourceType *type, void **objp) {
    (void)env;
    if (!x || T(x)->k != K_RES || T(x)->u.res->type != type) return 0;
    *objp = T(x)->u.res->data;
    return 1;
}

void enif_release_resource(void *obj) {
    res_release((rt_res *)((unsigned char *)obj - offsetof(rt_res, data)));
}

void enif_keep_resource(void *obj) {
    rt_res *r = (rt_res *)((unsigned char *)obj - offsetof(rt_res, data));
    atomic_fetch_add(&r->refc, 1);
}

void *enif_alloc(size_t size) { return malloc(size ? size : 1); }
void *enif_realloc(void *ptr, size_t size) { return realloc(ptr, size ? size : 1); }
void enif_free(void *ptr) { free(ptr); }

/* ---- the test-side API (ctypes) ------------------------------------------ */
int rt_nif_entry(const ErlNifFunc **funcs, int *n, int (**load)(ErlNifEnv *, void **, ERL_NIF_TERM));

static const ErlNifFunc *g_funcs;
static int g_n_funcs;
static int g_loaded;
static void *g_priv;

/* the module's load callback, once; 0 = loaded */
int rt_load(void) {
    if (g_loaded) return 0;
    int (*load)(ErlNifEnv *, void **, ERL_NIF_TERM) = NULL;
    rt_nif_entry(&g_funcs, &g_n_funcs, &load);
    ErlNifEnv env;
    memset(&env, 0, sizeof env);
    int rc = load ? load(&env, &g_priv, enif_make_atom(&env, "undefined")) : 0;
    g_loaded = rc == 0;
    return rc;
}

ErlNifEnv *rt_env_new(void) { return calloc(1, sizeof(ErlNifEnv)); }

void rt_env_free(ErlNifEnv *env) {
    for (size_t i = 0; i < env->n_held; ++i) res_release(env->held[i]);
    free(env->held);
    for (blk *b = env->blocks, *nx; b; b = nx) {
        nx = b->next;
        free(b);
    }
    free(env);
}

ERL_NIF_TERM rt_decode(ErlNifEnv *env, const unsigned char *data, size_t n) {
    ERL_NIF_TERM t = 0;
    return enif_binary_to_term(env, data, n, &t, 0) == n ? t : 0;
}

/* the term's external format in a malloc'ed buffer (rt_free_buf); -1 = bad term */
long rt_encode(ERL_NIF_TERM t, unsigned char **out) {
    buf b = {0, 0, 0};
    if (!enc(&b, t)) {
        free(b.d);
        return -1;
    }
    *out = b.d;
    return (long)b.n;
}

void rt_free_buf(void *p) { free(p); }

/* call Name/argc; *exc = 0 (returned normally), 1 (badarg), 2 (raised;
 * rt_exc_reason has the reason), -1 (no such function) */
ERL_NIF_TERM rt_call(ErlNifEnv *env, const char *name, int argc, const ERL_NIF_TERM *argv,
                     int *exc) {
    for (int i = 0; i < g_n_funcs; ++i)
        if ((int)g_funcs[i].arity == argc && strcmp(g_funcs[i].name, name) == 0) {
            env->exc = 0;
            ERL_NIF_TERM r = g_funcs[i].fptr(env, argc, argv);
            *exc = env->exc;
            return r;
        }
    *exc = -1;
    return 0;
}

ERL_NIF_TERM rt_exc_reason(ErlNifEnv *env) { return env->reason; }

/* a test's own reference on a resource term's resource (kept across
 * environments), and its release -- the destructor runs with the last one */
uint64_t rt_keep(ERL_NIF_TERM t) {
    if (!t || T(t)->k != K_RES) return 0;
    atomic_fetch_add(&T(t)->u.res->refc, 1);
    return (uint64_t)(uintptr_t)T(t)->u.res;
}

void rt_release(uint64_t res) { res_release((rt_res *)(uintptr_t)res); }

long rt_live_resources(void) { return atomic_load(&g_live_res); }
