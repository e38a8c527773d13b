// api.hip — the C ABI of include/antidote_gpu.h: context, descriptor
// validation, host-staged materialize (the per-key NIF entry), the GST
// collective over RCCL, and the synthetic op-log generator.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"
#include "gen.hpp"
#include "serve.hpp"

namespace agn {
// host-staged materialize (agn_materialize_host): a non-blocking stream plus
// a device buffer and a pinned host buffer that only grow
struct Stager {
    hipStream_t s = nullptr;
    char *d = nullptr, *h = nullptr;
    size_t cap = 0;
};
}  // namespace agn

struct agn_ctx {
    int device = 0;
    std::mutex comm_mu;
    ncclComm_t comm = nullptr;
    // host-staged materialize: stagers (stream + buffers) reused across calls
    std::mutex st_mu;
    std::vector<agn::Stager *> st_all, st_free;
    // agn_log_index_masks' mixed-key count per key_mask buffer it built (the
    // last kMaskIdx): agn_materialize adds AGN_HINT_MIXED to a batch over such
    // a log when enough of its keys are mixed -- a hint changes no result, so
    // a stale entry (a buffer rewritten by the caller) only costs speed
    struct MaskIdx {
        const uint64_t *key_mask;
        uint64_t n_keys, mixed;
    };
    static constexpr int kMaskIdx = 16;
    std::mutex mi_mu;
    MaskIdx mi[kMaskIdx] = {};
    unsigned mi_next = 0;
    std::atomic<bool> mi_any{false};
};

namespace agn {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

int use_device(agn_ctx *ctx) {
    if (!ctx) return fail(AGN_EINVAL, "null context");
    AGN_HIP(hipSetDevice(ctx->device));
    return AGN_OK;
}

// ---- cached environment knobs (common.hpp EnvKnob) -------------------------
std::atomic<uint32_t> g_env_gen{1};
static std::mutex g_env_mu;

void EnvKnob::refresh(uint32_t g) {
    std::lock_guard<std::mutex> lk(g_env_mu);
    if (gen_.load(std::memory_order_relaxed) == g) return;
    const char *v = getenv(name_);
    const char *cur = val_.load(std::memory_order_relaxed);
    // a new snapshot only when the value changed; the old one is kept (leaked
    // on purpose: readers may hold it; reloads happen between test phases)
    if (!v) {
        val_.store(nullptr, std::memory_order_release);
    } else if (!cur || std::strcmp(cur, v) != 0) {
        const char *copy = strdup(v);
        if (copy) val_.store(copy, std::memory_order_release);
    }
    gen_.store(g, std::memory_order_release);
}

// ---- the library's memory pools (one per device) ---------------------------
namespace {
constexpr int kMaxDevices = 64;
std::mutex g_pool_mu;
hipMemPool_t g_pool[kMaxDevices] = {};
int g_pool_users[kMaxDevices] = {};

uint64_t pool_keep_bytes() {
    const char *v = AGN_KNOB("AGN_POOL_KEEP");
    if (!v || !*v) return UINT64_MAX;
    return strtoull(v, nullptr, 10);
}

hipError_t pool_of(int dev, hipMemPool_t *out) {
    if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> g(g_pool_mu);
    if (!g_pool[dev]) {
        hipMemPoolProps props;
        std::memset(&props, 0, sizeof props);
        props.allocType = hipMemAllocationTypePinned;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = dev;
        hipMemPool_t p = nullptr;
        hipError_t e = hipMemPoolCreate(&p, &props);
        if (e != hipSuccess) return e;
        uint64_t keep = pool_keep_bytes();
        (void)hipMemPoolSetAttribute(p, hipMemPoolAttrReleaseThreshold, &keep);
        g_pool[dev] = p;
    }
    *out = g_pool[dev];
    return hipSuccess;
}
}  // namespace

hipError_t pool_malloc(void **p, size_t bytes, hipStream_t st) {
    // test hook: AGN_TEST_POOL_FAIL=n makes the n-th allocation from now fail
    // (tests/test_oplog.py drives the all-or-nothing paths with it)
    // (unset -- every production call -- costs one cached-knob load and no lock)
    static std::atomic<bool> was_armed{false};
    const char *v = AGN_KNOB("AGN_TEST_POOL_FAIL");
    if (v || was_armed.load(std::memory_order_relaxed)) {
        static std::mutex mu;
        static std::string armed;
        static long left = 0;
        std::lock_guard<std::mutex> g(mu);
        was_armed.store(v != nullptr, std::memory_order_relaxed);
        if (!v) {
            armed.clear();
        } else {
            if (armed != v) {
                armed = v;
                left = strtol(v, nullptr, 10);
            }
            if (left > 0 && --left == 0) return hipErrorOutOfMemory;
        }
    }
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    hipMemPool_t pool = nullptr;
    if (e == hipSuccess) e = pool_of(dev, &pool);
    if (e != hipSuccess) return e;
    return hipMallocFromPoolAsync(p, bytes ? bytes : 1, pool, st);
}

static bool is_tag_type(uint32_t t) { return t == AGN_SET_AW || t == AGN_REGISTER_MV; }

// A log whose key_mask agn_log_index_masks built (same buffer, same key
// count) with many mixed keys (many_mixed).
static bool mixed_log(agn_ctx *ctx, const agn_log *log) {
    if (!ctx->mi_any.load(std::memory_order_acquire)) return false;
    std::lock_guard<std::mutex> g(ctx->mi_mu);
    for (const auto &m : ctx->mi)
        if (m.key_mask == log->key_mask && m.n_keys == log->n_keys)
            return many_mixed(m.mixed, m.n_keys);
    return false;
}

static int validate(const agn_log *log, const agn_read *req, const agn_result *out) {
    if (!log || !req || !out) return fail(AGN_EINVAL, "null descriptor");
    // byte arrays are read by the kernels as aligned dwords (scalar loads
    // ignore the address's low two bits)
    if (misaligned4(log->key_type) || misaligned4(req->sct_ignore))
        return fail(AGN_EINVAL, "key_type / sct_ignore must be 4-byte aligned");
    if (log->n_dcs == 0 || log->n_dcs > 256) return fail(AGN_EINVAL, "n_dcs=%u not in [1,256]", log->n_dcs);
    if (log->crdt_type != AGN_COUNTER_PN && !is_tag_type(log->crdt_type))
        return fail(AGN_EINVAL, "unknown crdt_type %u", log->crdt_type);
    if (req->n_req == 0) return AGN_OK;
    if (!log->key_off) return fail(AGN_EINVAL, "log: key_off required");
    if (log->n_entries && (!log->oc || !log->op_id))
        return fail(AGN_EINVAL, "log: oc/op_id required");
    if (!req->keys && req->n_req != log->n_keys)
        return fail(AGN_EINVAL, "identity key map needs n_req == n_keys");
    if (!req->R) return fail(AGN_EINVAL, "read: R required");
    if (!out->hole || !out->lastct || !out->count || !out->flags || !out->err_pos)
        return fail(AGN_EINVAL, "result: hole/lastct/count/flags/err_pos required");
    if (log->crdt_type == AGN_COUNTER_PN) {
        if (log->n_entries && !log->eff) return fail(AGN_EINVAL, "counter_pn log needs eff");
        if (!out->value) return fail(AGN_EINVAL, "counter_pn result needs value");
    } else {
        if (log->n_entries && (!log->tag || !log->add_tok || !log->rem_off))
            return fail(AGN_EINVAL, "set/register log needs tag/add_tok/rem_off");
        if (!out->out_off || !out->out_n || !out->out_tag || !out->out_tok)
            return fail(AGN_EINVAL, "set/register result needs out_off/out_n/out_tag/out_tok");
    }
    return AGN_OK;
}

}  // namespace agn

using namespace agn;

extern "C" {

int agn_abi_version(void) { return AGN_ABI_VERSION; }

const char *agn_last_error(void) { return g_err; }

int agn_env_reload(void) {
    g_env_gen.fetch_add(1, std::memory_order_acq_rel);
    return AGN_OK;
}

const char *agn_strerror(int code) {
    switch (code) {
        case AGN_OK: return "ok";
        case AGN_EINVAL: return "invalid argument";
        case AGN_EHIP: return "HIP runtime error";
        case AGN_ENOMEM: return "out of memory";
        case AGN_ECAPACITY: return "device table capacity exceeded";
        case AGN_ENOTSUP: return "not supported";
        case AGN_ERCCL: return "RCCL error";
        case AGN_ENODEV: return "no device";
        default: return "unknown error";
    }
}

int agn_device_count(int *out) {
    if (!out) return fail(AGN_EINVAL, "null out");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *out = n;
    return AGN_OK;
}

int agn_open(int device, agn_ctx **out) {
    if (!out) return fail(AGN_EINVAL, "null out");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(AGN_ENODEV, "no HIP device");
    if (device < 0 || device >= n) return fail(AGN_EINVAL, "device %d of %d", device, n);
    AGN_HIP(hipSetDevice(device));
    hipDeviceProp_t p;
    AGN_HIP(hipGetDeviceProperties(&p, device));
    if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0)
        return fail(AGN_ENOTSUP, "built for gfx950, device is %s", p.gcnArchName);
    // Stream-ordered scratch (prune, ingest, op-log arenas) comes from the
    // library's own pool of this device (pool_malloc), created here so a
    // failure shows at open; freed blocks stay cached in it (GC and ingest
    // do not remap gigabytes per call) until agn_pool_trim / agn_close.
    hipMemPool_t pool = nullptr;
    if (pool_of(device, &pool) != hipSuccess) return fail(AGN_EHIP, "hipMemPoolCreate");
    agn_ctx *c = new (std::nothrow) agn_ctx;
    if (!c) return fail(AGN_ENOMEM, "ctx");
    c->device = device;
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        ++g_pool_users[device];
    }
    *out = c;
    return AGN_OK;
}

int agn_pool_trim(agn_ctx *ctx, uint64_t keep_bytes) {
    int rc = use_device(ctx);
    if (rc) return rc;
    hipMemPool_t pool = nullptr;
    if (pool_of(ctx->device, &pool) != hipSuccess) return fail(AGN_EHIP, "pool");
    AGN_HIP(hipDeviceSynchronize());  // frees still queued on streams reach the pool
    AGN_HIP(hipMemPoolTrimTo(pool, (size_t)keep_bytes));
    return AGN_OK;
}

int agn_close(agn_ctx *ctx) {
    if (!ctx) return AGN_OK;
    agn_comm_destroy(ctx);
    bool last = false;
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        last = --g_pool_users[ctx->device] == 0;
    }
    for (Stager *S : ctx->st_all) {
        (void)hipStreamSynchronize(S->s);
        if (S->d) (void)hipFree(S->d);
        if (S->h) (void)hipHostFree(S->h);
        (void)hipStreamDestroy(S->s);
        delete S;
    }
    // the last context of a device hands the pool's cached blocks back
    if (last) (void)agn_pool_trim(ctx, 0);
    delete ctx;
    return AGN_OK;
}

int agn_dev_alloc(agn_ctx *ctx, size_t bytes, void **out) {
    int rc = use_device(ctx);
    if (rc) return rc;
    if (!out) return fail(AGN_EINVAL, "null out");
    *out = nullptr;
    if (bytes == 0) return AGN_OK;
    if (hipMalloc(out, bytes) != hipSuccess) return fail(AGN_ENOMEM, "hipMalloc(%zu)", bytes);
    return AGN_OK;
}

int agn_dev_free(agn_ctx *ctx, void *ptr) {
    int rc = use_device(ctx);
    if (rc) return rc;
    if (ptr) AGN_HIP(hipFree(ptr));
    return AGN_OK;
}

int agn_memcpy_h2d(agn_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream) {
    int rc = use_device(ctx);
    if (rc) return rc;
    if (bytes) AGN_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
    return AGN_OK;
}

int agn_memcpy_d2h(agn_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream) {
    int rc = use_device(ctx);
    if (rc) return rc;
    if (bytes) AGN_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
    return AGN_OK;
}

int agn_memset_d(agn_ctx *ctx, void *dst, int value, size_t bytes, void *stream) {
    int rc = use_device(ctx);
    if (rc) return rc;
    if (bytes) AGN_HIP(hipMemsetAsync(dst, value, bytes, (hipStream_t)stream));
    return AGN_OK;
}

int agn_stream_sync(agn_ctx *ctx, void *stream) {
    int rc = use_device(ctx);
    if (rc) return rc;
    AGN_HIP(hipStreamSynchronize((hipStream_t)stream));
    return AGN_OK;
}

int agn_materialize(agn_ctx *ctx, const agn_log *log, const agn_read *req, agn_result *out,
                    void *stream) {
    int rc = validate(log, req, out);  // descriptors first: checkable without a GPU
    if (rc) return rc;
    rc = use_device(ctx);
    if (rc) return rc;
    if (req->n_req == 0) return AGN_OK;
    hipStream_t s = (hipStream_t)stream;
    if (log->crdt_type == AGN_COUNTER_PN) {
        if (log->oc_mask && log->key_mask && !(req->hints & AGN_HINT_MIXED) &&
            mixed_log(ctx, log)) {
            agn_read r = *req;
            r.hints |= AGN_HINT_MIXED;
            return launch_counter(*log, r, *out, s);
        }
        return launch_counter(*log, *req, *out, s);
    }
    return launch_tags(*log, *req, *out, s);
}

int agn_tune(agn_ctx *ctx, const agn_log *log, const agn_read *req, agn_result *out,
             void *stream, int rounds, int *choice, float *ms) {
    if (!choice) return fail(AGN_EINVAL, "tune: null choice");
    *choice = -1;
    int rc = validate(log, req, out);
    if (rc) return rc;
    rc = use_device(ctx);
    if (rc) return rc;
    if (req->n_req == 0) return AGN_OK;
    hipStream_t s = (hipStream_t)stream;
    if (rounds < 1) rounds = 1;
    rc = tune_counter_dense(*log, *req, *out, s, rounds, choice, ms);
    if (rc != AGN_ENOTSUP) return rc;
    *choice = -1;  // one kernel for this shape: plain materialize
    rc = log->crdt_type == AGN_COUNTER_PN ? launch_counter(*log, *req, *out, s)
                                          : launch_tags(*log, *req, *out, s);
    if (rc) return rc;
    AGN_HIP(hipStreamSynchronize(s));
    return AGN_OK;
}

int agn_log_index_ids(agn_ctx *ctx, const agn_log *log, uint32_t *out, void *stream) {
    if (!log || !out) return fail(AGN_EINVAL, "index_ids: null argument");
    if (log->n_keys && !log->key_off) return fail(AGN_EINVAL, "index_ids: key_off required");
    if (log->n_entries && !log->op_id) return fail(AGN_EINVAL, "index_ids: op_id required");
    int rc = use_device(ctx);
    if (rc) return rc;
    return launch_index_ids(*log, out, (hipStream_t)stream);
}

int agn_log_index_masks(agn_ctx *ctx, const agn_log *log, uint64_t *out, void *stream) {
    if (!log || !out) return fail(AGN_EINVAL, "index_masks: null argument");
    if (log->n_keys && !log->key_off) return fail(AGN_EINVAL, "index_masks: key_off required");
    if (log->n_dcs == 0 || log->n_dcs > 64)
        return fail(AGN_EINVAL, "index_masks: n_dcs=%u not in [1,64]", log->n_dcs);
    int rc = use_device(ctx);
    if (rc) return rc;
    // the mixed-key count (a kernel-choice heuristic for later reads of this
    // index; results never depend on it) is read back synchronously -- not
    // inside a stream capture, where the index is then left unregistered
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing((hipStream_t)stream, &cap) != hipSuccess)
        cap = hipStreamCaptureStatusNone;
    const bool count = log->oc_mask && cap == hipStreamCaptureStatusNone;
    uint64_t mixed = 0;
    rc = launch_index_masks(*log, out, count ? &mixed : nullptr, (hipStream_t)stream);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(ctx->mi_mu);
    int slot = -1;
    for (int i = 0; i < agn_ctx::kMaskIdx && slot < 0; ++i)
        if (ctx->mi[i].key_mask == out) slot = i;
    if (!count && log->oc_mask) {  // no count: forget a stale one for this buffer
        if (slot >= 0) ctx->mi[slot] = {};
        return AGN_OK;
    }
    if (slot < 0) slot = (int)(ctx->mi_next++ % agn_ctx::kMaskIdx);
    ctx->mi[slot] = {out, log->n_keys, mixed};
    ctx->mi_any.store(true, std::memory_order_release);
    return AGN_OK;
}

int agn_state_capacity(const agn_log *log, const agn_read *req, uint64_t *cap_off) {
    if (!log || !req || !cap_off) return fail(AGN_EINVAL, "null argument");
    cap_off[0] = 0;
    for (uint64_t i = 0; i < req->n_req; ++i) {
        const uint64_t k = req->keys ? req->keys[i] : i;
        uint64_t c = 0;
        if (log->add_tok)
            for (uint64_t e = log->key_off[k]; e < log->key_off[k] + key_n(log->key_off, log->key_len, k); ++e)
                c += log->add_tok[e] != 0;
        if (req->base_off) c += req->base_off[i + 1] - req->base_off[i];
        else if (req->base_value && is_tag_type(log->crdt_type))
            c += AGN_SS_STATE_PAIRS(req->base_value[i]);
        cap_off[i + 1] = cap_off[i] + c;
    }
    return AGN_OK;
}

}  // extern "C"

// ---- host-staged materialize --------------------------------------------------
// The per-key NIF entry (materialize/4 with the ops list as an Erlang term).
// Each call borrows a stager of its context -- a non-blocking stream plus a
// device buffer and a pinned host buffer that only grow -- packs every input
// array into the pinned buffer, and does one H2D copy, the materialize kernel
// and one D2H copy on that stream, then waits for that stream only.  Calls from
// many threads run on different stagers concurrently; nothing allocates in
// the steady state and nothing synchronizes the device.
namespace {
int stager_grow(Stager *S, size_t bytes) {
    if (bytes <= S->cap) return AGN_OK;
    const size_t c = std::max(bytes, 2 * S->cap);
    if (S->d) (void)hipFree(S->d);
    if (S->h) (void)hipHostFree(S->h);
    S->d = S->h = nullptr;
    S->cap = 0;
    if (hipMalloc((void **)&S->d, c) != hipSuccess) return fail(AGN_ENOMEM, "staging: %zu B", c);
    if (hipHostMalloc((void **)&S->h, c, hipHostMallocDefault) != hipSuccess)
        return fail(AGN_ENOMEM, "staging: %zu B pinned", c);
    S->cap = c;
    return AGN_OK;
}

Stager *stager_get(agn_ctx *ctx) {
    {
        std::lock_guard<std::mutex> g(ctx->st_mu);
        if (!ctx->st_free.empty()) {
            Stager *S = ctx->st_free.back();
            ctx->st_free.pop_back();
            return S;
        }
    }
    Stager *S = new (std::nothrow) Stager;
    if (!S) return nullptr;
    if (hipStreamCreateWithFlags(&S->s, hipStreamNonBlocking) != hipSuccess) {
        delete S;
        return nullptr;
    }
    std::lock_guard<std::mutex> g(ctx->st_mu);
    ctx->st_all.push_back(S);
    return S;
}

void stager_put(agn_ctx *ctx, Stager *S) {
    std::lock_guard<std::mutex> g(ctx->st_mu);
    ctx->st_free.push_back(S);
}

// Packs host arrays into the stager: in(...) reserves an input slot (copied
// H2D), out(...) an output slot (copied back D2H); device pointers are final
// once layout() has sized the buffer.
struct Pack {
    struct In { const void *h; size_t bytes; size_t off; };
    struct Out { void *h; size_t bytes; size_t off; };
    std::vector<In> ins;
    std::vector<Out> outs;
    size_t off = 0, in_end = 0;
    static size_t al(size_t b) { return (b + 255) & ~size_t(255); }
    template <class T>
    size_t in(const T *h, size_t n) {
        if (!h || n == 0) return SIZE_MAX;
        ins.push_back({h, n * sizeof(T), off});
        off = al(off + n * sizeof(T));
        return ins.back().off;
    }
    template <class T>
    size_t out(T *h, size_t n) {
        if (!h) return SIZE_MAX;
        if (in_end == 0) in_end = off;
        outs.push_back({h, std::max<size_t>(n, 1) * sizeof(T), off});
        off = al(off + std::max<size_t>(n, 1) * sizeof(T));
        return outs.back().off;
    }
};

template <class T>
T *at(const Stager *S, size_t o) { return o == SIZE_MAX ? nullptr : (T *)(S->d + o); }
}  // namespace

extern "C" {

int agn_materialize_host(agn_ctx *ctx, const agn_log *log, const agn_read *req, agn_result *out) {
    int rc = validate(log, req, out);
    if (rc) return rc;
    rc = use_device(ctx);
    if (rc) return rc;
    if (req->n_req == 0) return AGN_OK;
    const uint32_t D = log->n_dcs, W = n_words(D);
    const uint64_t E = log->n_entries, K = log->n_keys, Q = req->n_req;
    uint64_t n_rem = log->rem_off ? log->rem_off[E] : 0;
    if (log->rem_off && log->key_len)  // segmented log: the token arena's high-water mark
        for (uint64_t e = 0; e <= E; ++e) n_rem = std::max<uint64_t>(n_rem, log->rem_off[e]);
    uint64_t n_base = req->base_off ? req->base_off[Q] : 0;
    if (!req->base_off && req->base_value && is_tag_type(log->crdt_type))  // arena references
        for (uint64_t i = 0; i < Q; ++i)
            n_base = std::max<uint64_t>(n_base, AGN_SS_STATE_START(req->base_value[i]) +
                                                    AGN_SS_STATE_PAIRS(req->base_value[i]));
    const uint64_t n_out = out->out_off ? out->out_off[Q] : 0;
    // a sparse log without agn_log.key_mask: build it here (one pass over the
    // masks already in host memory), so keys whose entries share one DC set
    // take the dense row scans (D <= 64)
    std::vector<uint64_t> hkm;
    const uint64_t *kmask = log->key_mask;
    if (log->oc_mask && !kmask && D <= 64) {
        const uint64_t full = low_bits(D);
        hkm.assign(K, 0);
        for (uint64_t k = 0; k < K; ++k) {
            const uint64_t o = log->key_off[k], n = key_n(log->key_off, log->key_len, k);
            if (n == 0) continue;
            uint64_t m0 = log->oc_mask[o] & full;
            for (uint64_t x = 1; x < n && m0; ++x)
                if ((log->oc_mask[o + x] & full) != m0) m0 = 0;
            hkm[k] = m0;
        }
        kmask = hkm.data();
    }
    Pack p;
    const size_t l_koff = p.in(log->key_off, K + 1), l_klen = p.in(log->key_len, K),
                 l_ktype = p.in(log->key_type, K), l_oc = p.in(log->oc, E * D),
                 l_ocm = p.in(log->oc_mask, E * W), l_id = p.in(log->op_id, E),
                 l_tx = p.in(log->txid, E), l_eff = p.in(log->eff, E), l_tag = p.in(log->tag, E),
                 l_add = p.in(log->add_tok, E),
                 l_roff = p.in(log->rem_off, log->rem_off ? E + 1 : 0),
                 l_rtok = p.in(log->rem_tok, n_rem), l_id0 = p.in(log->key_id0, K),
                 l_kmask = p.in(kmask, (log->oc_mask && D <= 64) ? K : 0);
    const size_t q_keys = p.in(req->keys, Q), q_R = p.in(req->R, Q * D),
                 q_Rm = p.in(req->R_mask, Q * W), q_sct = p.in(req->sct, Q * D),
                 q_sctm = p.in(req->sct_mask, Q * W), q_sign = p.in(req->sct_ignore, Q),
                 q_tx = p.in(req->txid, Q), q_bv = p.in(req->base_value, Q),
                 q_boff = p.in(req->base_off, req->base_off ? Q + 1 : 0),
                 q_btag = p.in(req->base_tag, n_base), q_btok = p.in(req->base_tok, n_base),
                 o_off = p.in(out->out_off, out->out_off ? Q + 1 : 0);
    const size_t o_val = p.out(out->value, Q), o_hole = p.out(out->hole, Q),
                 o_ct = p.out(out->lastct, Q * D), o_ctm = p.out(out->lastct_mask, Q * W),
                 o_cnt = p.out(out->count, Q), o_flg = p.out(out->flags, Q),
                 o_epos = p.out(out->err_pos, Q), o_n = p.out(out->out_n, Q),
                 o_tag = p.out(out->out_tag, n_out), o_tok = p.out(out->out_tok, n_out);
    if (p.in_end == 0) p.in_end = p.off;
    Stager *S = stager_get(ctx);
    if (!S) return fail(AGN_ENOMEM, "materialize_host: stager");
    rc = stager_grow(S, p.off);
    if (rc) {
        stager_put(ctx, S);
        return rc;
    }
    for (const auto &x : p.ins) std::memcpy(S->h + x.off, x.h, x.bytes);
    agn_log dl = *log;
    dl.key_off = at<const uint64_t>(S, l_koff);
    dl.key_len = at<const uint64_t>(S, l_klen);
    dl.key_type = at<const uint8_t>(S, l_ktype);
    dl.oc = at<const uint64_t>(S, l_oc);
    dl.oc_mask = at<const uint64_t>(S, l_ocm);
    dl.op_id = at<const uint32_t>(S, l_id);
    dl.txid = at<const uint64_t>(S, l_tx);
    dl.eff = at<const int64_t>(S, l_eff);
    dl.tag = at<const uint32_t>(S, l_tag);
    dl.add_tok = at<const uint64_t>(S, l_add);
    dl.rem_off = at<const uint32_t>(S, l_roff);
    dl.rem_tok = at<const uint64_t>(S, l_rtok);
    dl.key_id0 = at<const uint32_t>(S, l_id0);
    dl.key_mask = at<const uint64_t>(S, l_kmask);
    agn_read dr = *req;
    dr.keys = at<const uint64_t>(S, q_keys);
    dr.R = at<const uint64_t>(S, q_R);
    dr.R_mask = at<const uint64_t>(S, q_Rm);
    dr.sct = at<const uint64_t>(S, q_sct);
    dr.sct_mask = at<const uint64_t>(S, q_sctm);
    dr.sct_ignore = at<const uint8_t>(S, q_sign);
    dr.txid = at<const uint64_t>(S, q_tx);
    dr.base_value = at<const int64_t>(S, q_bv);
    dr.base_off = at<const uint64_t>(S, q_boff);
    dr.base_tag = at<const uint32_t>(S, q_btag);
    dr.base_tok = at<const uint64_t>(S, q_btok);
    agn_result dout = *out;
    dout.value = at<int64_t>(S, o_val);
    dout.hole = at<int64_t>(S, o_hole);
    dout.lastct = at<uint64_t>(S, o_ct);
    dout.lastct_mask = at<uint64_t>(S, o_ctm);
    dout.count = at<uint32_t>(S, o_cnt);
    dout.flags = at<uint32_t>(S, o_flg);
    dout.err_pos = at<uint32_t>(S, o_epos);
    dout.out_off = at<const uint64_t>(S, o_off);
    dout.out_n = at<uint32_t>(S, o_n);
    dout.out_tag = at<uint32_t>(S, o_tag);
    dout.out_tok = at<uint64_t>(S, o_tok);
    hipError_t e = hipMemcpyAsync(S->d, S->h, p.in_end, hipMemcpyHostToDevice, S->s);
    if (e == hipSuccess) {
        rc = agn_materialize(ctx, &dl, &dr, &dout, S->s);
        if (rc == AGN_OK && p.off > p.in_end)
            e = hipMemcpyAsync(S->h + p.in_end, S->d + p.in_end, p.off - p.in_end,
                               hipMemcpyDeviceToHost, S->s);
    }
    const hipError_t es = hipStreamSynchronize(S->s);
    if (e == hipSuccess) e = es;
    if (rc == AGN_OK && e != hipSuccess)
        rc = fail(AGN_EHIP, "materialize_host: %s", hipGetErrorString(e));
    if (rc == AGN_OK)
        for (const auto &x : p.outs) {
            // out_tag / out_tok hold n_out elements (at least one slot reserved)
            const size_t b = (x.h == (void *)out->out_tag) ? n_out * 4
                           : (x.h == (void *)out->out_tok) ? n_out * 8 : x.bytes;
            if (b) std::memcpy(x.h, S->h + x.off, b);
        }
    stager_put(ctx, S);
    return rc;
}

}  // extern "C"

extern "C" {

// ---- base selection / GST ---------------------------------------------------------
int agn_select_base(agn_ctx *ctx, uint32_t n_dcs, uint64_t n_req, const uint64_t *cache_off,
                    const uint64_t *clocks, const uint64_t *clock_mask, const uint64_t *R,
                    const uint64_t *R_mask, int32_t *out_idx, uint8_t *out_is_first,
                    void *stream) {
    int rc = use_device(ctx);
    if (rc) return rc;
    if (n_dcs == 0 || !cache_off || !R || !out_idx || !out_is_first)
        return fail(AGN_EINVAL, "select_base: bad arguments");
    return launch_select_base(n_dcs, n_req, cache_off, clocks, clock_mask, R, R_mask, out_idx,
                              out_is_first, (hipStream_t)stream);
}

int agn_gst_min(agn_ctx *ctx, uint32_t n_dcs, uint64_t n_parts, uint64_t n_epochs,
                const uint64_t *clocks, const uint8_t *defined, uint64_t *out, void *stream) {
    int rc = use_device(ctx);
    if (rc) return rc;
    if (!out || (n_parts && n_epochs && !clocks)) return fail(AGN_EINVAL, "gst: null buffer");
    return launch_gst_min(n_dcs, n_parts, n_epochs, clocks, defined, out, (hipStream_t)stream);
}

int agn_gst_finalize(agn_ctx *ctx, uint32_t n_dcs, uint64_t n_epochs, uint64_t *vec,
                     void *stream) {
    int rc = use_device(ctx);
    if (rc) return rc;
    if (!vec) return fail(AGN_EINVAL, "gst: null buffer");
    return launch_gst_finalize(n_dcs, n_epochs, vec, (hipStream_t)stream);
}

int agn_log_ingest(agn_ctx *ctx, const agn_log_records *recs, uint32_t crdt_type,
                   uint32_t n_dcs, uint64_t n_keys, const uint64_t *max_time,
                   const uint64_t *max_time_mask, uint32_t op_id_base, agn_log *out,
                   uint64_t *out_totals, void *stream) {
    if (!recs || !out) return fail(AGN_EINVAL, "log_ingest: null descriptor");
    if (n_dcs == 0 || n_dcs > 256) return fail(AGN_EINVAL, "log_ingest: n_dcs=%u", n_dcs);
    if (crdt_type != AGN_COUNTER_PN && !is_tag_type(crdt_type))
        return fail(AGN_EINVAL, "log_ingest: crdt_type %u", crdt_type);
    if (n_keys >= (1ull << 24)) return fail(AGN_ENOTSUP, "log_ingest: n_keys >= 2^24");
    if (recs->n >= 0x7fffffffull) return fail(AGN_ENOTSUP, "log_ingest: n >= 2^31 records");
    if (recs->n && (!recs->kind || !recs->txid || !recs->key || !recs->commit_dc ||
                    !recs->commit_time || !recs->ss))
        return fail(AGN_EINVAL, "log_ingest: null record array");
    if (crdt_type == AGN_COUNTER_PN ? !recs->eff
                                    : (!recs->tag || !recs->add_tok || !recs->rem_off))
        return fail(AGN_EINVAL, "log_ingest: effect arrays missing for type %u", crdt_type);
    if (!out->key_off || !out->oc || !out->op_id || (recs->ss_mask && !out->oc_mask) ||
        (crdt_type == AGN_COUNTER_PN ? !out->eff
                                     : (!out->tag || !out->add_tok || !out->rem_off)))
        return fail(AGN_EINVAL, "log_ingest: out arrays missing");
    int rc = use_device(ctx);
    if (rc) return rc;
    agn_log_records r = *recs;
    if (crdt_type == AGN_COUNTER_PN) r.tag = nullptr, r.add_tok = nullptr, r.rem_off = nullptr,
                                     r.rem_tok = nullptr;
    else r.eff = nullptr;
    agn_log o = *out;
    if (crdt_type == AGN_COUNTER_PN) o.tag = nullptr, o.add_tok = nullptr, o.rem_off = nullptr,
                                     o.rem_tok = nullptr;
    else o.eff = nullptr;
    out->crdt_type = crdt_type;
    out->n_dcs = n_dcs;
    out->n_keys = n_keys;
    out->key_id0 = nullptr;  // fresh op ids: no index until agn_log_index_ids
    if (recs->n == 0) {
        AGN_HIP(hipMemsetAsync((void *)out->key_off, 0, (n_keys + 1) * 8, (hipStream_t)stream));
        if (out_totals) AGN_HIP(hipMemsetAsync(out_totals, 0, 16, (hipStream_t)stream));
        return AGN_OK;
    }
    return launch_log_ingest(r, n_dcs, n_keys, max_time, max_time_mask, op_id_base, o, out_totals,
                             (hipStream_t)stream);
}

static int check_cache(const agn_ss_cache *c) {
    if (!c) return fail(AGN_EINVAL, "ss cache: null");
    if (c->n_dcs == 0 || c->n_dcs > 256) return fail(AGN_EINVAL, "ss cache: n_dcs=%u", c->n_dcs);
    if (c->slots < AGN_SNAPSHOT_THRESHOLD - 1)
        return fail(AGN_EINVAL, "ss cache: slots=%u < %d", c->slots, AGN_SNAPSHOT_THRESHOLD - 1);
    if (c->n_keys && (!c->n || !c->clock || !c->last_op || !c->value))
        return fail(AGN_EINVAL, "ss cache: null array");
    if ((c->state_tag || c->state_tok || c->state_ctl) &&
        !(c->state_tag && c->state_tok && c->state_ctl))
        return fail(AGN_EINVAL, "ss cache: state arena needs state_tag, state_tok and state_ctl");
    return AGN_OK;
}

int agn_ss_lookup(agn_ctx *ctx, agn_ss_cache *cache, uint64_t n_req, const uint64_t *keys,
                  const uint64_t *R, const uint64_t *R_mask, uint64_t *sct, uint64_t *sct_mask,
                  uint8_t *sct_ignore, int64_t *base_value, uint8_t *is_first, uint8_t *status,
                  void *stream) {
    int rc = check_cache(cache);
    if (rc) return rc;
    if (n_req && (!R || !sct || !sct_ignore || !base_value || !is_first || !status))
        return fail(AGN_EINVAL, "ss_lookup: null argument");
    if (!keys && n_req != cache->n_keys)
        return fail(AGN_EINVAL, "ss_lookup: keys == NULL needs n_req == n_keys");
    rc = use_device(ctx);
    if (rc) return rc;
    return launch_ss_lookup(*cache, n_req, keys, R, R_mask, sct, sct_mask, sct_ignore, base_value,
                            is_first, status, (hipStream_t)stream);
}

int agn_ss_store(agn_ctx *ctx, agn_ss_cache *cache, const agn_log *log, uint64_t n_req,
                 const uint64_t *keys, const uint8_t *is_first, const uint8_t *status,
                 const uint8_t *should_gc, const agn_result *res, const int64_t *handle,
                 uint8_t *prune, uint64_t *threshold, uint64_t *threshold_mask, void *stream) {
    int rc = check_cache(cache);
    if (rc) return rc;
    if (!log || !res || !log->key_off || !prune || !threshold)
        return fail(AGN_EINVAL, "ss_store: null argument");
    if (log->n_keys != cache->n_keys || log->n_dcs != cache->n_dcs)
        return fail(AGN_EINVAL, "ss_store: log and cache disagree on keys / DCs");
    const bool arena = cache->state_tag != nullptr && is_tag_type(log->crdt_type);
    if (n_req && (!is_first || !status || !res->hole || !res->lastct || !res->count ||
                  !res->flags || (!arena && !handle && !res->value) ||
                  (arena && (!res->out_off || !res->out_n || !res->out_tag || !res->out_tok))))
        return fail(AGN_EINVAL, "ss_store: null argument");
    if (!keys && n_req != cache->n_keys)
        return fail(AGN_EINVAL, "ss_store: keys == NULL needs n_req == n_keys");
    rc = use_device(ctx);
    if (rc) return rc;
    return launch_ss_store(*cache, log->key_off, log->key_len, n_req, keys, is_first, status, should_gc, *res,
                           handle, prune, threshold, threshold_mask, (hipStream_t)stream);
}

// agn_read_cached's batch size from which it runs the three batched kernels
// (k_ss_lookup -> the counter kernel -> k_ss_store, per-request prune flags)
// instead of the fused one: same results.  D = 8 (quad rows): from 5M
// requests -- the fused kernel won at every size in round 5 (100k 0.099 vs
// 0.111 ms, 1M 0.97 vs 1.00, 10M 9.45 vs 9.70; profiles/r05/
// ab_read6_sizes.log); since the batched scan runs two requests per wave in
// runs of 64 blocks per XCD it leads from about 5M (warm cfg2 keys, fused vs
// batched: 2M 1.90 vs 1.93 ms, 4M 3.78 vs 3.83, 6M 5.75 vs 5.56, 8M 7.63 vs
// 7.49, 10M 9.25 vs 9.05; profiles/r06/ab_read6_xcd.log).  D < 8: from 2^15 requests, where the
// batched kernels' 8 requests per wave in the cache steps and two per wave in
// the scan win (D = 3: 100k 0.090 vs 0.090 ms, 1M 0.90 vs 0.84, 10M 8.99 vs
// 8.20).  AGN_READ_CACHED_SPLIT=<n> moves the switch (0: never).
static uint64_t read_cached_split(uint32_t D) {
    const char *v = AGN_KNOB("AGN_READ_CACHED_SPLIT");
    if (v && v[0]) {
        const uint64_t n = strtoull(v, nullptr, 10);
        return n ? n : ~0ull;
    }
    return D == 8 ? 5000000ull : 1ull << 15;
}

static int read_cached_seq(agn_ss_cache *cache, const agn_log *log, uint64_t n_req,
                           const uint64_t *keys, const uint64_t *R, const uint64_t *txid,
                           const uint8_t *should_gc, agn_result *out, uint8_t *status,
                           uint8_t *prune, uint64_t *threshold, hipStream_t st) {
    const uint32_t D = log->n_dcs;
    uint8_t *tmp = nullptr;  // sct [n][D] u64 | base [n] i64 | ign [n] | first [n]
    const size_t sz = n_req * (8ull * D + 8ull + 2ull);
    AGN_HIP(pool_malloc((void **)&tmp, sz, st));
    uint64_t *sct = reinterpret_cast<uint64_t *>(tmp);
    int64_t *base = reinterpret_cast<int64_t *>(sct + n_req * D);
    uint8_t *ign = reinterpret_cast<uint8_t *>(base + n_req);
    uint8_t *first = ign + n_req;
    agn_result o = *out;
    o.lastct_mask = nullptr;
    int rc = launch_ss_lookup(*cache, n_req, keys, R, nullptr, sct, nullptr, ign, base, first,
                              status, st);
    if (rc == AGN_OK) {
        agn_read rq{};
        rq.n_req = n_req;
        rq.keys = keys;
        rq.R = R;
        rq.sct = sct;
        rq.sct_ignore = ign;
        rq.txid = txid;
        rq.req_type = AGN_COUNTER_PN;
        rq.base_value = base;
        rc = launch_counter(*log, rq, o, st);
    }
    if (rc == AGN_OK)
        // the store reads LastOpCt as the counter kernel wrote it: dense, so
        // with the (unwritten) caller mask nulled as in the kernel's copy
        rc = launch_ss_store_req(*cache, log->key_off, log->key_len, n_req, keys, first, status,
                                 should_gc, o, prune, threshold, nullptr, st);
    (void)hipFreeAsync(tmp, st);
    return rc;
}

// read/6 of a set_aw / register_mv batch over a cache with a state arena:
// lookup (the hit slot's AGN_SS_STATE as the base) -> the tags kernel reading
// the base state from the arena -> the store appending the new state to it.
static int read_cached_tags(agn_ss_cache *cache, const agn_log *log, uint64_t n_req,
                            const uint64_t *keys, const uint64_t *R, const uint64_t *txid,
                            const uint8_t *should_gc, agn_result *out, uint8_t *status,
                            uint8_t *prune, uint64_t *threshold, hipStream_t st) {
    const uint32_t D = log->n_dcs;
    uint8_t *tmp = nullptr;  // sct [n][D] u64 | base [n] i64 | ign [n] | first [n]
    AGN_HIP(pool_malloc((void **)&tmp, n_req * (8ull * D + 8ull + 2ull), st));
    uint64_t *sct = reinterpret_cast<uint64_t *>(tmp);
    int64_t *base = reinterpret_cast<int64_t *>(sct + n_req * D);
    uint8_t *ign = reinterpret_cast<uint8_t *>(base + n_req);
    uint8_t *first = ign + n_req;
    agn_result o = *out;
    o.lastct_mask = nullptr;
    o.value = nullptr;
    int rc = launch_ss_lookup(*cache, n_req, keys, R, nullptr, sct, nullptr, ign, base, first,
                              status, st);
    if (rc == AGN_OK) {
        agn_read rq{};
        rq.n_req = n_req;
        rq.keys = keys;
        rq.R = R;
        rq.sct = sct;
        rq.sct_ignore = ign;
        rq.txid = txid;
        rq.req_type = log->crdt_type;
        rq.base_value = base;  // AGN_SS_STATE references into the arena
        rq.base_tag = cache->state_tag;
        rq.base_tok = cache->state_tok;
        rc = launch_tags(*log, rq, o, st);
    }
    if (rc == AGN_OK)
        rc = launch_ss_store_req(*cache, log->key_off, log->key_len, n_req, keys, first, status,
                                 should_gc, o, prune, threshold, nullptr, st);
    (void)hipFreeAsync(tmp, st);
    return rc;
}

int agn_ss_state_compact(agn_ctx *ctx, agn_ss_cache *cache, uint32_t *new_tag, uint64_t *new_tok,
                         uint64_t new_cap, void *stream) {
    int rc = check_cache(cache);
    if (rc) return rc;
    if (!cache->state_tag || !cache->state_tok || !cache->state_ctl)
        return fail(AGN_EINVAL, "ss_state_compact: the cache has no state arena");
    if ((!new_tag || !new_tok) && new_cap)
        return fail(AGN_EINVAL, "ss_state_compact: null arena");
    rc = use_device(ctx);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    uint64_t ctl[4];
    AGN_HIP(hipMemcpyAsync(ctl, cache->state_ctl, sizeof ctl, hipMemcpyDeviceToHost, st));
    AGN_HIP(hipStreamSynchronize(st));
    const uint64_t live = ctl[0] - ctl[1];
    if (live > new_cap)
        return fail(AGN_ECAPACITY, "ss_state_compact: %llu live pairs > %llu",
                    (unsigned long long)live, (unsigned long long)new_cap);
    rc = launch_ss_compact(*cache, new_tag, new_tok, new_cap, cache->state_ctl + 2, st);
    if (rc) return rc;
    cache->state_tag = new_tag;
    cache->state_tok = new_tok;
    cache->state_cap = new_cap;
    return AGN_OK;
}

int agn_read_cached(agn_ctx *ctx, agn_ss_cache *cache, const agn_log *log, uint64_t n_req,
                    const uint64_t *keys, const uint64_t *R, const uint64_t *txid,
                    const uint8_t *should_gc, agn_result *out, uint8_t *status, uint8_t *prune,
                    uint64_t *threshold, void *stream) {
    int rc = check_cache(cache);
    if (rc) return rc;
    if (!log || !out || !log->key_off) return fail(AGN_EINVAL, "read_cached: null argument");
    if (log->n_keys != cache->n_keys || log->n_dcs != cache->n_dcs)
        return fail(AGN_EINVAL, "read_cached: log and cache disagree on keys / DCs");
    if (is_tag_type(log->crdt_type)) {
        if (!cache->state_tag || !cache->state_tok || !cache->state_ctl || cache->clock_mask)
            return fail(AGN_ENOTSUP, "read_cached: set/register needs a cache with a state "
                                     "arena and dense clocks");
        if (n_req == 0) return AGN_OK;
        if (!keys || !R || !status || !prune || !threshold || !out->hole || !out->lastct ||
            !out->count || !out->flags || !out->err_pos || !out->out_off || !out->out_n ||
            !out->out_tag || !out->out_tok)
            return fail(AGN_EINVAL, "read_cached: null argument");
        rc = use_device(ctx);
        if (rc) return rc;
        return read_cached_tags(cache, log, n_req, keys, R, txid, should_gc, out, status, prune,
                                threshold, (hipStream_t)stream);
    }
    if (!read6_supported(*log, log->n_dcs) || cache->clock_mask)
        return fail(AGN_ENOTSUP, "read_cached: counter_pn with dense clocks, D <= 8");
    if (n_req == 0) return AGN_OK;
    if (!keys || !R || !status || !prune || !threshold || !out->value || !out->hole ||
        !out->lastct || !out->count || !out->flags || !out->err_pos)
        return fail(AGN_EINVAL, "read_cached: null argument");
    rc = use_device(ctx);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    if (n_req >= read_cached_split(log->n_dcs)) return read_cached_seq(cache, log, n_req, keys, R, txid,
                                                             should_gc, out, status, prune,
                                                             threshold, st);
    Read6Args a{};  // dense: the mask pointers stay null
    a.key_off = log->key_off;
    a.key_len = log->key_len;
    a.key_id0 = log->key_id0;
    a.key_type = log->key_type;
    a.oc = log->oc;
    a.op_id = log->op_id;
    a.eff = log->eff;
    a.log_txid = log->txid;
    a.n_entries = log->n_entries;
    a.n_dcs = log->n_dcs;
    a.req_type = AGN_COUNTER_PN;
    a.n_req = n_req;
    a.keys = keys;
    a.R = R;
    a.txid = txid;
    a.gc = should_gc;
    a.value = out->value;
    a.hole = out->hole;
    a.lastct = out->lastct;
    a.count = out->count;
    a.flags = out->flags;
    a.err_pos = out->err_pos;
    a.status = status;
    a.prune = prune;
    a.dkeys = nullptr;  // the batcher's GC list copies: not needed here
    a.dprune = nullptr;
    a.thr = threshold;
    return launch_read6(*cache, a, st);
}

int agn_prune_ops(agn_ctx *ctx, const agn_log *log, const uint8_t *prune,
                  const uint64_t *threshold, const uint64_t *threshold_mask, agn_log *out,
                  uint32_t *out_flags, uint64_t *out_totals, void *stream) {
    if (!log || !out) return fail(AGN_EINVAL, "prune_ops: null descriptor");
    if (log->n_dcs == 0 || log->n_dcs > 256)
        return fail(AGN_EINVAL, "prune_ops: n_dcs=%u not in [1,256]", log->n_dcs);
    if (log->n_keys == 0) return AGN_OK;
    if (!log->key_off || !threshold || !out->key_off)
        return fail(AGN_EINVAL, "prune_ops: key_off / threshold required");
    if (log->n_entries && (!log->oc || !log->op_id || !out->oc || !out->op_id))
        return fail(AGN_EINVAL, "prune_ops: oc / op_id required");
    if ((log->oc_mask && !out->oc_mask) || (log->txid && !out->txid) ||
        (log->eff && !out->eff) || (log->tag && !out->tag) || (log->add_tok && !out->add_tok) ||
        (log->rem_off && (!out->rem_off || (!out->rem_tok && log->rem_tok))))
        return fail(AGN_EINVAL, "prune_ops: out lacks an array the log has");
    if (log->n_entries > 0x7fffffffull || log->n_keys > 0x7fffffffull)
        return fail(AGN_ENOTSUP, "prune_ops: log too large for one pass");
    if (misaligned4(prune) || misaligned4(log->key_type))
        return fail(AGN_EINVAL, "prune_ops: prune / key_type must be 4-byte aligned");
    int rc = use_device(ctx);
    if (rc) return rc;
    out->crdt_type = log->crdt_type;
    out->n_dcs = log->n_dcs;
    out->n_keys = log->n_keys;
    out->key_type = log->key_type;
    hipStream_t st = (hipStream_t)stream;
    if (out->key_len) {
        // segmented output: one pass, each key at its input segment start
        out->n_entries = log->n_entries;
        rc = launch_prune_segmented(*log, prune, threshold, threshold_mask, *out, out_flags, st);
        if (rc == AGN_OK && out_totals) rc = launch_seg_totals(*out, out_totals, st);
        return rc;
    }
    out->key_id0 = nullptr;  // pruning leaves id gaps: rebuild with agn_log_index_ids
    return launch_prune_ops(*log, prune, threshold, threshold_mask, *out, out_flags, out_totals,
                            st);
}

int agn_gst_scalar(agn_ctx *ctx, uint32_t n_dcs, uint64_t n_epochs, uint64_t *vec,
                   uint64_t *out_gst, void *stream) {
    if (n_dcs == 0) return fail(AGN_EINVAL, "gst_scalar: n_dcs=0");
    if (n_epochs && !vec) return fail(AGN_EINVAL, "gst_scalar: null vec");
    int rc = use_device(ctx);
    if (rc) return rc;
    return launch_gst_scalar(n_dcs, n_epochs, vec, out_gst, (hipStream_t)stream);
}

int agn_dep_check(agn_ctx *ctx, uint32_t n_dcs, uint64_t n_txn, const uint64_t *deps,
                  const uint64_t *deps_mask, const uint32_t *origin, const uint32_t *part,
                  uint64_t n_parts, const uint64_t *part_clock, const uint64_t *part_mask,
                  uint8_t *out_ok, void *stream) {
    if (n_dcs == 0 || n_dcs > 4096) return fail(AGN_EINVAL, "dep_check: n_dcs=%u", n_dcs);
    if (n_txn && (!deps || !origin || !part || !part_clock || !out_ok || n_parts == 0))
        return fail(AGN_EINVAL, "dep_check: null argument");
    int rc = use_device(ctx);
    if (rc) return rc;
    return launch_dep_check(n_dcs, n_txn, deps, deps_mask, origin, part, n_parts, part_clock,
                            part_mask, out_ok, (hipStream_t)stream);
}

int agn_update_stable(uint32_t n_dcs, uint64_t *last, const uint64_t *nw, int *changed) {
    if (!last || !nw) return fail(AGN_EINVAL, "null clock");
    int c = 0;
    for (uint32_t d = 0; d < n_dcs; ++d) {
        if (nw[d] == UINT64_MAX) continue;  // DC absent from NewDict: keep Last
        if (last[d] == UINT64_MAX || nw[d] >= last[d]) {  // update_func_min/2
            last[d] = nw[d];
            c = 1;
        }
    }
    if (changed) *changed = c;
    return AGN_OK;
}

int agn_gst_merge(uint32_t n_dcs, uint64_t n_vecs, const uint64_t *vecs, uint64_t *out) {
    if (!out || (n_vecs && !vecs)) return fail(AGN_EINVAL, "gst_merge: null buffer");
    if (n_dcs == 0) return fail(AGN_EINVAL, "gst_merge: n_dcs = 0");
    const uint64_t W = (uint64_t)n_dcs + 1;
    for (uint64_t j = 0; j < W; ++j) out[j] = UINT64_MAX;
    out[n_dcs] = 1;  // no vector: nothing undefined
    for (uint64_t v = 0; v < n_vecs; ++v)
        for (uint64_t j = 0; j < W; ++j) out[j] = std::min(out[j], vecs[v * W + j]);
    if (out[n_dcs] == 0)  // some partition undefined: every present DC -> 0 (:78-84)
        for (uint32_t d = 0; d < n_dcs; ++d)
            if (out[d] != UINT64_MAX) out[d] = 0;
    return AGN_OK;
}

// ---- RCCL ------------------------------------------------------------------------
int agn_comm_unique_id(uint8_t *out_id) {
    static_assert(sizeof(ncclUniqueId) <= AGN_UNIQUE_ID_BYTES, "unique id size");
    if (!out_id) return fail(AGN_EINVAL, "null id");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return fail(AGN_ERCCL, "ncclGetUniqueId: %s", ncclGetErrorString(r));
    std::memset(out_id, 0, AGN_UNIQUE_ID_BYTES);
    std::memcpy(out_id, &id, sizeof id);
    return AGN_OK;
}

int agn_comm_init(agn_ctx *ctx, int nranks, int rank, const uint8_t *id) {
    int rc = use_device(ctx);
    if (rc) return rc;
    if (!id || nranks < 1 || rank < 0 || rank >= nranks) return fail(AGN_EINVAL, "comm args");
    std::lock_guard<std::mutex> g(ctx->comm_mu);
    if (ctx->comm) return fail(AGN_EINVAL, "communicator already initialised");
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    ncclResult_t r = ncclCommInitRank(&ctx->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        ctx->comm = nullptr;
        return fail(AGN_ERCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
    return AGN_OK;
}

int agn_comm_destroy(agn_ctx *ctx) {
    if (!ctx) return AGN_OK;
    std::lock_guard<std::mutex> g(ctx->comm_mu);
    if (ctx->comm) {
        ncclCommDestroy(ctx->comm);
        ctx->comm = nullptr;
    }
    return AGN_OK;
}

int agn_gst_allreduce(agn_ctx *ctx, uint64_t *dev_vec, uint64_t n_words_, void *stream) {
    int rc = use_device(ctx);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(ctx->comm_mu);
    if (!ctx->comm) return fail(AGN_EINVAL, "no communicator (agn_comm_init)");
    ncclResult_t r = ncclAllReduce(dev_vec, dev_vec, n_words_, ncclUint64, ncclMin, ctx->comm,
                                   (hipStream_t)stream);
    if (r != ncclSuccess) return fail(AGN_ERCCL, "ncclAllReduce: %s", ncclGetErrorString(r));
    return AGN_OK;
}

}  // extern "C"

// ---- synthetic generator ------------------------------------------------------------
namespace agn {
namespace {

uint32_t gen_live_lists(const agn_gen_cfg &c) {
    return c.crdt_type == AGN_SET_AW ? (c.n_elems ? c.n_elems : 1) : 1;
}

int check_cfg(const agn_gen_cfg *c) {
    if (!c) return fail(AGN_EINVAL, "null cfg");
    if (c->n_dcs == 0 || c->n_dcs > 256) return fail(AGN_EINVAL, "gen: n_dcs");
    if (c->ops_per_key >= (1u << 24) - 1) return fail(AGN_EINVAL, "gen: ops_per_key");
    if (c->crdt_type != AGN_COUNTER_PN && !is_tag_type(c->crdt_type))
        return fail(AGN_EINVAL, "gen: crdt_type");
    return AGN_OK;
}

__global__ void k_gen(agn_gen_cfg cfg, agn_log log, agn_read req, int pass, uint64_t *scratch,
                      uint32_t *rem_cnt) {
    const uint32_t D = cfg.n_dcs, N = cfg.ops_per_key;
    const uint32_t nl = cfg.crdt_type == AGN_SET_AW ? (cfg.n_elems ? cfg.n_elems : 1) : 1;
    const uint64_t per = (uint64_t)D + (uint64_t)nl * GEN_MAX_LIVE + nl;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t *my = scratch + tid * per;
    for (uint64_t k = tid; k < cfg.n_keys; k += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e0 = k * N;
        GenOut o{};
        o.clk = my;
        o.live = my + D;
        o.live_n = (uint32_t *)(my + D + (uint64_t)nl * GEN_MAX_LIVE);
        if (pass == 0) {
            o.rem_cnt = rem_cnt + e0;
        } else {
            o.oc = (uint64_t *)log.oc + e0 * D;
            o.op_id = (uint32_t *)log.op_id + e0;
            o.eff = (int64_t *)log.eff + (log.eff ? e0 : 0);
            o.tag = (uint32_t *)log.tag + (log.tag ? e0 : 0);
            o.add_tok = (uint64_t *)log.add_tok + (log.add_tok ? e0 : 0);
            o.rem_off = log.rem_off ? log.rem_off + e0 : nullptr;
            o.rem_tok = (uint64_t *)log.rem_tok;
            o.R = (uint64_t *)req.R + k * D;
            o.sct = req.sct ? (uint64_t *)req.sct + k * D : nullptr;
            o.sct_ignore = req.sct_ignore ? (uint8_t *)req.sct_ignore + k : nullptr;
        }
        gen_key(cfg, k, o);
        if (pass == 1 && k == 0) ((uint64_t *)log.key_off)[0] = 0;
        if (pass == 1) ((uint64_t *)log.key_off)[k + 1] = (k + 1) * (uint64_t)N;
    }
}

template <class T>
T *dmalloc(uint64_t n, int &err) {
    if (err || n == 0) return nullptr;
    void *p = nullptr;
    if (hipMalloc(&p, n * sizeof(T)) != hipSuccess) {
        err = fail(AGN_ENOMEM, "gen: hipMalloc(%llu)", (unsigned long long)(n * sizeof(T)));
        return nullptr;
    }
    return (T *)p;
}

}  // namespace
}  // namespace agn

extern "C" {

int agn_gen_dev(agn_ctx *ctx, const agn_gen_cfg *cfg, agn_log *log, agn_read *req,
                void *stream) {
    int rc = use_device(ctx);
    if (rc) return rc;
    rc = check_cfg(cfg);
    if (rc) return rc;
    if (!log || !req) return fail(AGN_EINVAL, "null out");
    std::memset(log, 0, sizeof *log);
    std::memset(req, 0, sizeof *req);
    hipStream_t s = (hipStream_t)stream;
    const agn_gen_cfg c = *cfg;
    const uint32_t D = c.n_dcs;
    const uint64_t K = c.n_keys, E = K * c.ops_per_key;
    const bool tags = is_tag_type(c.crdt_type);
    int err = AGN_OK;
    log->crdt_type = c.crdt_type;
    log->n_dcs = D;
    log->n_keys = K;
    log->n_entries = E;
    log->key_off = dmalloc<uint64_t>(K + 1, err);
    log->oc = dmalloc<uint64_t>(E * D, err);
    log->op_id = dmalloc<uint32_t>(E, err);
    if (!tags) {
        log->eff = dmalloc<int64_t>(E, err);
    } else {
        log->tag = dmalloc<uint32_t>(E, err);
        log->add_tok = dmalloc<uint64_t>(E, err);
        log->rem_off = dmalloc<uint32_t>(E + 1, err);
    }
    req->n_req = K;
    req->req_type = c.crdt_type;
    req->R = dmalloc<uint64_t>(K * D, err);
    if (c.warm) {
        req->sct = dmalloc<uint64_t>(K * D, err);
        req->sct_ignore = dmalloc<uint8_t>(K, err);
    }
    const uint32_t nl = gen_live_lists(c);
    const uint64_t threads = std::min<uint64_t>(std::max<uint64_t>(K, 1), 256ull * 1024ull);
    const uint64_t per = (uint64_t)D + (uint64_t)nl * GEN_MAX_LIVE + nl;
    uint64_t *scratch = dmalloc<uint64_t>(threads * per, err);
    if (err) { agn_gen_free_dev(ctx, log, req); if (scratch) (void)hipFree(scratch); return err; }
    const unsigned blocks = (unsigned)((threads + 255) / 256);
    if (tags && E) {
        // pass 0: removal counts into rem_off[1..E], inclusive scan, rem_off[0] = 0
        uint32_t *ro = (uint32_t *)log->rem_off;
        hipLaunchKernelGGL(k_gen, dim3(blocks), dim3(256), 0, s, c, *log, *req, 0, scratch, ro + 1);
        size_t tmp_bytes = 0;
        if (hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, ro + 1, ro + 1, (int)E, s) !=
            hipSuccess)
            err = fail(AGN_EHIP, "gen: removal-offset scan sizing failed");
        void *tmp = err ? nullptr : dmalloc<uint8_t>(tmp_bytes ? tmp_bytes : 1, err);
        if (!err && hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, ro + 1, ro + 1, (int)E, s) !=
                        hipSuccess)
            err = fail(AGN_EHIP, "gen: removal-offset scan failed");
        if (!err) (void)hipMemsetAsync(ro, 0, sizeof(uint32_t), s);
        uint32_t total = 0;
        if (!err) (void)hipMemcpyAsync(&total, ro + E, sizeof total, hipMemcpyDeviceToHost, s);
        if (!err) (void)hipStreamSynchronize(s);
        if (tmp) (void)hipFree(tmp);
        log->rem_tok = dmalloc<uint64_t>(total ? total : 1, err);
    } else if (tags) {
        (void)hipMemsetAsync((void *)log->rem_off, 0, sizeof(uint32_t), s);
        log->rem_tok = dmalloc<uint64_t>(1, err);
    }
    if (err) { (void)hipFree(scratch); agn_gen_free_dev(ctx, log, req); return err; }
    if (K == 0) (void)hipMemsetAsync((void *)log->key_off, 0, sizeof(uint64_t), s);
    hipLaunchKernelGGL(k_gen, dim3(blocks), dim3(256), 0, s, c, *log, *req, 1, scratch, nullptr);
    hipError_t he = hipGetLastError();
    // the consecutive-id index (ids 1..N per key), as an engine-built log carries it
    log->key_id0 = dmalloc<uint32_t>(K, err);
    if (!err && he == hipSuccess && K) err = launch_index_ids(*log, (uint32_t *)log->key_id0, s);
    (void)hipStreamSynchronize(s);
    (void)hipFree(scratch);
    if (he != hipSuccess) err = fail(AGN_EHIP, "k_gen: %s", hipGetErrorString(he));
    if (err) agn_gen_free_dev(ctx, log, req);
    return err;
}

int agn_gen_free_dev(agn_ctx *ctx, agn_log *log, agn_read *req) {
    int rc = use_device(ctx);
    if (rc) return rc;
    const void *ptrs[] = {log ? log->key_off : nullptr, log ? log->key_type : nullptr,
                          log ? log->oc : nullptr, log ? log->oc_mask : nullptr,
                          log ? log->op_id : nullptr, log ? log->txid : nullptr,
                          log ? log->eff : nullptr, log ? log->tag : nullptr,
                          log ? log->add_tok : nullptr, log ? log->rem_off : nullptr,
                          log ? log->rem_tok : nullptr, log ? log->key_id0 : nullptr,
                          req ? req->keys : nullptr,
                          req ? req->R : nullptr, req ? req->R_mask : nullptr,
                          req ? req->sct : nullptr, req ? req->sct_mask : nullptr,
                          req ? req->sct_ignore : nullptr, req ? req->txid : nullptr,
                          req ? req->base_value : nullptr, req ? req->base_off : nullptr,
                          req ? req->base_tag : nullptr, req ? req->base_tok : nullptr};
    for (const void *p : ptrs)
        if (p) (void)hipFree((void *)p);
    if (log) std::memset(log, 0, sizeof *log);
    if (req) std::memset(req, 0, sizeof *req);
    return AGN_OK;
}

int agn_gen_host(const agn_gen_cfg *cfg, agn_log *log, agn_read *req) {
    int rc = check_cfg(cfg);
    if (rc) return rc;
    if (!log || !req) return fail(AGN_EINVAL, "null out");
    std::memset(log, 0, sizeof *log);
    std::memset(req, 0, sizeof *req);
    const agn_gen_cfg c = *cfg;
    const uint32_t D = c.n_dcs, N = c.ops_per_key;
    const uint64_t K = c.n_keys, E = K * N;
    const bool tags = is_tag_type(c.crdt_type);
    auto hm = [](uint64_t bytes) { return std::calloc(bytes ? bytes : 1, 1); };
    log->crdt_type = c.crdt_type;
    log->n_dcs = D;
    log->n_keys = K;
    log->n_entries = E;
    uint64_t *key_off = (uint64_t *)hm((K + 1) * 8);
    for (uint64_t k = 0; k <= K; ++k) key_off[k] = k * N;
    log->key_off = key_off;
    log->oc = (uint64_t *)hm(E * D * 8);
    log->op_id = (uint32_t *)hm(E * 4);
    if (!tags) log->eff = (int64_t *)hm(E * 8);
    else {
        log->tag = (uint32_t *)hm(E * 4);
        log->add_tok = (uint64_t *)hm(E * 8);
        log->rem_off = (uint32_t *)hm((E + 1) * 4);
    }
    req->n_req = K;
    req->req_type = c.crdt_type;
    req->R = (uint64_t *)hm(K * D * 8);
    if (c.warm) {
        req->sct = (uint64_t *)hm(K * D * 8);
        req->sct_ignore = (uint8_t *)hm(K);
    }
    const uint32_t nl = gen_live_lists(c);
    unsigned nt = std::thread::hardware_concurrency();
    if (nt < 1) nt = 1;
    if (nt > 32) nt = 32;
    if ((uint64_t)nt > K) nt = K ? (unsigned)K : 1;
    auto run = [&](int pass, unsigned t) {
        std::vector<uint64_t> clk(D), live((size_t)nl * GEN_MAX_LIVE);
        std::vector<uint32_t> live_n(nl);
        for (uint64_t k = t; k < K; k += nt) {
            const uint64_t e0 = k * N;
            GenOut o{};
            o.clk = clk.data();
            o.live = live.data();
            o.live_n = live_n.data();
            if (pass == 0) {
                o.rem_cnt = (uint32_t *)log->rem_off + 1 + e0;
            } else {
                o.oc = (uint64_t *)log->oc + e0 * D;
                o.op_id = (uint32_t *)log->op_id + e0;
                o.eff = log->eff ? (int64_t *)log->eff + e0 : nullptr;
                o.tag = log->tag ? (uint32_t *)log->tag + e0 : nullptr;
                o.add_tok = log->add_tok ? (uint64_t *)log->add_tok + e0 : nullptr;
                o.rem_off = log->rem_off ? log->rem_off + e0 : nullptr;
                o.rem_tok = (uint64_t *)log->rem_tok;
                o.R = (uint64_t *)req->R + k * D;
                o.sct = req->sct ? (uint64_t *)req->sct + k * D : nullptr;
                o.sct_ignore = req->sct_ignore ? (uint8_t *)req->sct_ignore + k : nullptr;
            }
            gen_key(c, k, o);
        }
    };
    auto par = [&](int pass) {
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; ++t) th.emplace_back(run, pass, t);
        for (auto &x : th) x.join();
    };
    if (tags) {
        par(0);
        uint32_t *ro = (uint32_t *)log->rem_off;
        ro[0] = 0;
        for (uint64_t e = 0; e < E; ++e) ro[e + 1] += ro[e];
        log->rem_tok = (uint64_t *)hm((uint64_t)ro[E] * 8);
    }
    par(1);
    return AGN_OK;
}

int agn_gen_free_host(agn_log *log, agn_read *req) {
    if (log) {
        std::free((void *)log->key_off); std::free((void *)log->key_type);
        std::free((void *)log->oc); std::free((void *)log->oc_mask);
        std::free((void *)log->op_id); std::free((void *)log->txid);
        std::free((void *)log->eff); std::free((void *)log->tag);
        std::free((void *)log->add_tok); std::free((void *)log->rem_off);
        std::free((void *)log->rem_tok);
        std::memset(log, 0, sizeof *log);
    }
    if (req) {
        std::free((void *)req->keys); std::free((void *)req->R); std::free((void *)req->R_mask);
        std::free((void *)req->sct); std::free((void *)req->sct_mask);
        std::free((void *)req->sct_ignore); std::free((void *)req->txid);
        std::free((void *)req->base_value); std::free((void *)req->base_off);
        std::free((void *)req->base_tag); std::free((void *)req->base_tok);
        std::memset(req, 0, sizeof *req);
    }
    return AGN_OK;
}

}  // extern "C"
