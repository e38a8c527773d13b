/*
 * A minimal, runnable stand-in for <erl_nif.h> -- TEST INFRASTRUCTURE ONLY.
 *
 * This image has no Erlang/OTP.  The NIF (nif/antidote_gpu_nif.c) is
 * compiled against this header twice by the tests:
 *   - `gcc -fsyntax-only -Wall -Wextra -Werror` (tests/test_nif_syntax.py);
 *   - linked with tests/nif_rt/erl_nif_rt.c, a small term runtime (integers,
 *     atoms, tuples, lists, binaries, resources with destructors, exceptions,
 *     enif_term_to_binary as an injective byte encoding), into
 *     tests/nif_rt/libagn_nif_rt.so, whose NIF functions the GPU tests call
 *     through ctypes (tests/test_nif_exec.py) -- so the NIF's C runs.
 * It declares exactly the erl_nif API subset the NIF uses, with the
 * documented signatures (erl_nif(3)).  Where the NIF is built for real
 * (nif/Makefile) OTP's own header is used instead.
 */
#ifndef AGN_ERL_NIF_RT_H
#define AGN_ERL_NIF_RT_H
#include <stddef.h>
#include <stdint.h>

typedef uint64_t ERL_NIF_TERM;
typedef struct enif_environment_t ErlNifEnv;
typedef struct enif_resource_type_t ErlNifResourceType;
typedef uint64_t ErlNifUInt64;
typedef int64_t ErlNifSInt64;
typedef void ErlNifResourceDtor(ErlNifEnv *, void *);
typedef enum { ERL_NIF_RT_CREATE = 1, ERL_NIF_RT_TAKEOVER = 2 } ErlNifResourceFlags;
typedef enum { ERL_NIF_DIRTY_JOB_CPU_BOUND = 1, ERL_NIF_DIRTY_JOB_IO_BOUND = 2 } ErlNifDirtyTaskFlags;
typedef struct {
    size_t size;
    unsigned char *data;
    void *ref_bin;
    void *__spare__[2];
} ErlNifBinary;
typedef struct {
    const char *name;
    unsigned arity;
    ERL_NIF_TERM (*fptr)(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]);
    unsigned flags;
} ErlNifFunc;

ERL_NIF_TERM enif_make_atom(ErlNifEnv *env, const char *name);
ERL_NIF_TERM enif_make_badarg(ErlNifEnv *env);
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv *env, ERL_NIF_TERM e1, ERL_NIF_TERM e2);
ERL_NIF_TERM enif_make_tuple3(ErlNifEnv *env, ERL_NIF_TERM e1, ERL_NIF_TERM e2, ERL_NIF_TERM e3);
ERL_NIF_TERM enif_make_tuple_from_array(ErlNifEnv *env, const ERL_NIF_TERM arr[], unsigned cnt);
ERL_NIF_TERM enif_make_list(ErlNifEnv *env, unsigned cnt, ...);
ERL_NIF_TERM enif_make_list_cell(ErlNifEnv *env, ERL_NIF_TERM head, ERL_NIF_TERM tail);
ERL_NIF_TERM enif_make_uint(ErlNifEnv *env, unsigned i);
ERL_NIF_TERM enif_make_uint64(ErlNifEnv *env, ErlNifUInt64 i);
ERL_NIF_TERM enif_make_int64(ErlNifEnv *env, ErlNifSInt64 i);
ERL_NIF_TERM enif_make_resource(ErlNifEnv *env, void *obj);
unsigned char *enif_make_new_binary(ErlNifEnv *env, size_t size, ERL_NIF_TERM *termp);
int enif_get_int(ErlNifEnv *env, ERL_NIF_TERM term, int *ip);
int enif_get_uint(ErlNifEnv *env, ERL_NIF_TERM term, unsigned *ip);
int enif_get_uint64(ErlNifEnv *env, ERL_NIF_TERM term, ErlNifUInt64 *ip);
int enif_get_int64(ErlNifEnv *env, ERL_NIF_TERM term, ErlNifSInt64 *ip);
int enif_get_tuple(ErlNifEnv *env, ERL_NIF_TERM term, int *arity, const ERL_NIF_TERM **array);
int enif_get_list_cell(ErlNifEnv *env, ERL_NIF_TERM term, ERL_NIF_TERM *head, ERL_NIF_TERM *tail);
int enif_get_list_length(ErlNifEnv *env, ERL_NIF_TERM term, unsigned *len);
int enif_is_empty_list(ErlNifEnv *env, ERL_NIF_TERM term);
int enif_is_list(ErlNifEnv *env, ERL_NIF_TERM term);
int enif_is_identical(ERL_NIF_TERM lhs, ERL_NIF_TERM rhs);
int enif_compare(ERL_NIF_TERM lhs, ERL_NIF_TERM rhs);
int enif_inspect_binary(ErlNifEnv *env, ERL_NIF_TERM bin_term, ErlNifBinary *bin);
int enif_term_to_binary(ErlNifEnv *env, ERL_NIF_TERM term, ErlNifBinary *bin);
size_t enif_binary_to_term(ErlNifEnv *env, const unsigned char *data, size_t size,
                           ERL_NIF_TERM *term, unsigned opts);
void enif_release_binary(ErlNifBinary *bin);
ErlNifResourceType *enif_open_resource_type(ErlNifEnv *env, const char *module_str,
                                            const char *name, ErlNifResourceDtor *dtor,
                                            ErlNifResourceFlags flags, ErlNifResourceFlags *tried);
void *enif_alloc_resource(ErlNifResourceType *type, size_t size);
int enif_get_resource(ErlNifEnv *env, ERL_NIF_TERM term, ErlNifResourceType *type, void **objp);
void enif_release_resource(void *obj);
void enif_keep_resource(void *obj);
void *enif_alloc(size_t size);
void *enif_realloc(void *ptr, size_t size);
void enif_free(void *ptr);
ERL_NIF_TERM enif_raise_exception(ErlNifEnv *env, ERL_NIF_TERM reason);

/* The module's function table and load callback, for the runtime's loader
 * (rt_nif_entry); OTP's macro builds its ErlNifEntry instead. */
#define ERL_NIF_INIT(NAME, FUNCS, LOAD, RELOAD, UPGRADE, UNLOAD)                       \
    int rt_nif_entry(const ErlNifFunc **rt_funcs_, int *rt_n_,                         \
                     int (**rt_load_)(ErlNifEnv *, void **, ERL_NIF_TERM));             \
    int rt_nif_entry(const ErlNifFunc **rt_funcs_, int *rt_n_,                         \
                     int (**rt_load_)(ErlNifEnv *, void **, ERL_NIF_TERM)) {            \
        *rt_funcs_ = FUNCS;                                                            \
        *rt_n_ = (int)(sizeof(FUNCS) / sizeof((FUNCS)[0]));                            \
        *rt_load_ = LOAD;                                                              \
        return 0;                                                                      \
    }
#endif
