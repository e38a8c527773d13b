// common.hpp — shared device/host helpers for the gfx950 engine.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <atomic>
#include <shared_mutex>

#include "../../include/antidote_gpu.h"

#define AGN_WAVE 64

namespace agn {

// Environment knobs (A/B switches and test hooks, AGN_*): each is read once
// and cached, so a launch costs one atomic load instead of a getenv walk over
// the environment (serving batches launch every few microseconds).
// agn_env_reload() bumps g_env_gen and every knob re-reads its variable at
// its next use -- the tests and A/B scripts change knobs between launches.
extern std::atomic<uint32_t> g_env_gen;
class EnvKnob {
  public:
    explicit EnvKnob(const char *name) : name_(name) {}
    // the variable's value, nullptr when unset: an immutable snapshot that
    // stays valid for the life of the process (a reload publishes a new one
    // and never frees the old, so a caller may keep the pointer)
    const char *get() {
        const uint32_t g = g_env_gen.load(std::memory_order_acquire);
        if (gen_.load(std::memory_order_acquire) != g) refresh(g);
        return val_.load(std::memory_order_acquire);
    }

  private:
    void refresh(uint32_t g);  // api.hip
    const char *name_;
    std::atomic<uint32_t> gen_{0};
    std::atomic<const char *> val_{nullptr};
};
// getenv(NAME) through a per-call-site cached knob
#define AGN_KNOB(NAME)                     \
    ([]() -> const char * {                \
        static ::agn::EnvKnob knob_(NAME); \
        return knob_.get();                \
    }())

// Thread-local last-error message (agn_last_error).
void set_error(const char *fmt, ...);
int fail(int code, const char *fmt, ...);
// hipSetDevice(ctx's device); AGN_EINVAL for a null context.
int use_device(agn_ctx *ctx);

// Stream-ordered scratch and arenas come from the library's own memory pool
// of the current device (never the device's default pool, which torch and
// other hipMallocAsync users share): freed blocks stay cached in it (release
// threshold AGN_POOL_KEEP bytes, default unlimited), agn_pool_trim and
// agn_close hand them back.
hipError_t pool_malloc(void **p, size_t bytes, hipStream_t st);
template <class T>
inline hipError_t pool_malloc(T **p, size_t bytes, hipStream_t st) {
    return pool_malloc((void **)p, bytes, st);
}

#define AGN_HIP(call)                                                              \
    do {                                                                           \
        hipError_t e_ = (call);                                                    \
        if (e_ != hipSuccess)                                                      \
            return ::agn::fail(AGN_EHIP, "%s:%d %s: %s", __FILE__, __LINE__, #call, \
                               hipGetErrorString(e_));                             \
    } while (0)

__host__ __device__ inline uint32_t n_words(uint32_t d) { return (d + 63u) / 64u; }

// ---- wave-level helpers (wave64) ------------------------------------------
__device__ inline uint64_t ballot(bool p) { return __ballot(p); }

__device__ inline int lane_id() { return threadIdx.x & (AGN_WAVE - 1); }

__device__ inline uint64_t shfl_xor_u64(uint64_t v, int m) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = __shfl_xor(lo, m, AGN_WAVE);
    hi = __shfl_xor(hi, m, AGN_WAVE);
    return ((uint64_t)hi << 32) | lo;
}

__device__ inline int64_t wave_sum_i64(int64_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += (int64_t)shfl_xor_u64((uint64_t)v, m);
    return v;
}

__device__ inline uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

// Bit g of the result = some bit of group g (P consecutive bits) of the wave
// ballot b, on the scalar unit: the per-op verdict of a ballot whose P lanes
// per op hold its P 16-byte parts.
// Runs of r set bits every s bits (r <= s, s divides 64).
__host__ __device__ constexpr uint64_t run_mask(int r, int s) {
    uint64_t m = 0;
    for (int k = 0; k * s < 64; ++k) m |= (r >= 64 ? ~0ull : ((1ull << r) - 1ull)) << (k * s);
    return m;
}
// The fold leaves group g's verdict at bit g P; log2(64 / P) shift-or-mask
// steps then pack them (runs of 2^t bits every P 2^t bits merge pairwise) --
// for P = 8, 16 scalar operations where the per-group extract-and-insert
// loop took about twice that (k_tags' CT filter folds four ballots per
// 16-op sub-iteration).
template <int P>
__device__ __forceinline__ uint64_t group_any(uint64_t b) {
#pragma unroll
    for (int sh = 1; sh < P; sh <<= 1) b |= b >> sh;
    if constexpr (P == 1) return b;
    b &= run_mask(1, P);
#pragma unroll
    for (int t = 0; (P << t) < 64; ++t) {
        const int run = 1 << t, stride = P << t;
        b = (b | (b >> (stride - run))) & run_mask(2 * run, 2 * stride);
    }
    return b;
}

// group_any without the compaction ("spread" form): bit g P of the result =
// some bit of group g of b, the other bits 0 -- five scalar operations for
// P = 4 where the packed form takes ~11 (nib_any16) or ~30 (group_any<8>).
template <int P>
__host__ __device__ constexpr uint64_t group_base() {
    return run_mask(1, P);
}
template <int P>
__device__ __forceinline__ uint64_t group_any_spread(uint64_t b) {
#pragma unroll
    for (int sh = 1; sh < P; sh <<= 1) b |= b >> sh;
    return b & group_base<P>();
}

// Bit q of the result = some bit of nibble q of b (q = 0..15), on the scalar
// unit: the per-op verdict of a ballot whose 4 lanes per op are its 4 parts.
__device__ __forceinline__ uint64_t nib_any16(uint64_t b) {
    b |= b >> 1;
    b |= b >> 2;
    b &= 0x1111111111111111ull;
    b = (b | (b >> 3)) & 0x0303030303030303ull;
    b = (b | (b >> 6)) & 0x000F000F000F000Full;
    b = (b | (b >> 12)) & 0x000000FF000000FFull;
    return (b | (b >> 24)) & 0xFFFFull;
}

__host__ __device__ inline uint64_t low_bits(uint64_t k) { return k >= 64 ? ~0ull : ((1ull << k) - 1ull); }

// Entries of key k: [key_off[k], key_off[k] + key_len[k]) or CSR.
__host__ __device__ inline uint64_t key_n(const uint64_t *key_off, const uint64_t *key_len,
                                          uint64_t k) {
    return key_len ? key_len[k] : key_off[k + 1] - key_off[k];
}

// A load of memory the running kernel never writes, through the constant
// address space: at a wave-uniform address it is a scalar (s_load) load even
// where the kernel stores through other pointers that might alias it (a
// grid-stride loop), which otherwise keeps it a vector load.  Never use it
// on an array the same launch writes.
inline bool misaligned4(const void *p) { return ((uintptr_t)p & 3u) != 0; }
template <class T>
__device__ __forceinline__ T ldc(const T *p) {
    return *(const __attribute__((address_space(4))) T *)p;
}
// A byte of a read-only byte array (key_type, sct_ignore) by ldc of its
// aligned dword (byte arrays are allocated in whole dwords or more; the ABI
// requires them 4-byte aligned and validates it with misaligned4).
__device__ __forceinline__ uint32_t ldc_byte(const uint8_t *p, uint64_t idx) {
    const uint32_t w = ldc(reinterpret_cast<const uint32_t *>(p) + (idx >> 2));
    return (__builtin_amdgcn_readfirstlane(w) >> ((uint32_t)(idx & 3u) * 8u)) & 0xffu;
}

// A kernel's by-value parameter block T (its only parameter), read through
// the kernarg segment pointer.  Each call returns an opaque copy of the
// pointer, so the loads of a field are issued where it is used and are not
// shared with another call's: passed and used as ordinary arguments, every
// field a kernel touches is loaded at its entry and held in SGPRs to the
// end, and the ~100 dwords of this engine's argument structs spill the rest
// of the kernel's scalar state to VGPR lanes (read6.hip, k_counter_q8e2).
template <class T>
__device__ __forceinline__ const __attribute__((address_space(4))) T &kparams() {
    using P = const __attribute__((address_space(4))) T;
    P *p = (P *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *p;
}

// Scalar (wave-uniform) value: lets hipcc keep it in an SGPR.
__device__ inline uint64_t uniform_u64(uint64_t v) {
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// XCD-aware block order.  The dispatcher hands block b to XCD b mod 8, and
// every XCD has its own L2; with the identity order, the 16-32 consecutive
// requests that share one 128-byte line of a per-request array (key_off,
// value, hole, count, flags) are spread over all eight L2s, so each L2 reads
// the line and writes it back partially.  This bijection gives XCD x the
// contiguous logical range [x*q + min(x,r), ...) instead (q = nb/8, r = nb%8).
#define AGN_XCDS 8u
__device__ inline uint32_t xcd_block(uint32_t b, uint32_t nb) {
    const uint32_t q = nb / AGN_XCDS, r = nb % AGN_XCDS;
    const uint32_t x = b % AGN_XCDS, idx = b / AGN_XCDS;
    return x < r ? x * (q + 1u) + idx : r * (q + 1u) + (x - r) * q + idx;
}
// Chunked XCD order: runs of g consecutive logical blocks per XCD, the eight
// XCDs on neighbouring runs (a super-run of 8g blocks), so a per-request
// line stays in one L2 while the chip streams one region at a time; blocks
// past the last whole super-run keep the identity order.
__device__ inline uint32_t xcd_chunk_block(uint32_t b, uint32_t nb, uint32_t g) {
    const uint32_t sup = AGN_XCDS * g;
    if (b >= (nb / sup) * sup) return b;
    const uint32_t x = b % AGN_XCDS, idx = b / AGN_XCDS;
    return ((idx / g) * AGN_XCDS + x) * g + idx % g;
}
// A launch's block order: 0 identity, 1 xcd_block, g >= 2 xcd_chunk_block.
__device__ inline uint32_t block_order(uint32_t mode, uint32_t b, uint32_t nb) {
    return mode == 0u ? b : mode == 1u ? xcd_block(b, nb) : xcd_chunk_block(b, nb, mode);
}

// AGN_HINT_MIXED routing threshold: a masked counter batch with more than
// 1/16 of its keys mixed (entries with different DC sets) is scanned in one
// pass (k_counter_key MSK, 1.11x dense on uniform keys, 1.24x on mixed ones)
// instead of k_counter_q8e + the hand-on (1.04x, and ~2.5x for a mixed
// 64-op key, whose only chunk q8e reads before handing it on): break-even
// near a twentieth of the keys.
inline bool many_mixed(uint64_t mixed, uint64_t n) { return mixed * 16 > n; }

// A/B knob AGN_XCD_REMAP=0|1 (default on).
inline bool xcd_remap() {
    const char *v = AGN_KNOB("AGN_XCD_REMAP");
    return !(v && v[0] == '0');
}
// The XCD-aware block order where a launcher's measured default differs:
// AGN_XCD_REMAP=0|1 set explicitly wins, else `dflt`.
inline bool xcd_remap_or(bool dflt) {
    const char *v = AGN_KNOB("AGN_XCD_REMAP");
    return (v && (v[0] == '0' || v[0] == '1')) ? v[0] == '1' : dflt;
}
// Bulk counter batches (>= 2^20 requests) leave the XCD-aware order: dense
// cfg2 7.65 / 7.70 against 7.85 ms in the identity order, warm 7.97 / 8.05
// against 8.13, masked (k_counter_q8e) 7.83 against 8.04
// (profiles/r06/ab_xcd_remap.log), and the dense / warm kernels faster still
// in runs of 64 blocks per XCD (mat_counter_dense.hip counter_order); small
// batches keep the XCD-aware order (cfg1: 6.5 % faster with it).
inline bool counter_xcd(uint64_t n_req) { return xcd_remap_or(n_req < (1ull << 20)); }
// A launcher's block order (block_order's mode), default `dflt`: an explicit
// AGN_XCD_REMAP=0|1 wins, then AGN_XCD_CHUNK=g (runs of g >= 2 blocks per
// XCD; any other value the identity order) -- A/B knobs.
inline uint32_t order_or(uint32_t dflt) {
    const char *v = AGN_KNOB("AGN_XCD_REMAP");
    if (v && (v[0] == '0' || v[0] == '1')) return (uint32_t)(v[0] - '0');
    const char *c = AGN_KNOB("AGN_XCD_CHUNK");
    if (!c) return dflt;
    const unsigned long g = strtoul(c, nullptr, 10);
    return (g >= 2ul && g <= 4096ul) ? (uint32_t)g : 0u;
}

// Grid sizing for the streaming kernels: enough waves to fill 256 CUs.
inline unsigned grid_for(uint64_t work_items, unsigned items_per_block, unsigned max_blocks) {
    uint64_t b = (work_items + items_per_block - 1) / items_per_block;
    if (b < 1) b = 1;
    if (b > max_blocks) b = max_blocks;
    return (unsigned)b;
}

// Grid of exactly one resident round of `kernel` (blocks per CU from the
// occupancy API x CUs), capped by the work: the streaming kernels grid-stride,
// so a grid of k.33 rounds would leave its last third of a round running at a
// third of the chip.  Cached per kernel instantiation.
template <class K>
inline unsigned resident_grid(K kernel, unsigned threads, uint64_t work_blocks) {
    static int per_cu = -1, cus = -1;
    if (per_cu < 0) {
        int dev = 0, nb = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, (int)threads, 0) !=
                hipSuccess || nb < 1 || c < 1) {
            nb = 2;
            c = 256;
        }
        per_cu = nb;
        cus = c;
    }
    uint64_t b = (uint64_t)per_cu * (uint64_t)cus;
    if (work_blocks < b) b = work_blocks;
    return (unsigned)(b < 1 ? 1 : b);
}

// oplog.hip internals used by the read batcher.
void oplog_shape(const agn_oplog *L, uint32_t *crdt, uint32_t *D, int *sparse, uint64_t *K);
// mixed (optional): how many of mixed_keys[0..nm) hold entries with
// different DC sets, counted under the writer lock before `hold` is taken
// (the lock order is wmu before rw; nothing may take wmu under `hold`).
int oplog_begin_read(agn_oplog *L, hipStream_t st, uint64_t n, const uint64_t *keys,
                     uint32_t *lens, std::shared_lock<std::shared_mutex> &hold,
                     uint64_t nm = 0, const uint64_t *mixed_keys = nullptr,
                     uint64_t *mixed = nullptr);
void oplog_view(const agn_oplog *L, agn_log *v);
agn_ctx *oplog_ctx(const agn_oplog *L);

// Launchers (defined in the .hip files).
int launch_counter(const agn_log &log, const agn_read &req, const agn_result &out,
                   hipStream_t s);
int launch_index_ids(const agn_log &log, uint32_t *out, hipStream_t st);
int launch_index_masks(const agn_log &log, uint64_t *out, uint64_t *mixed, hipStream_t st);
int launch_counter_dense(const agn_log &log, const agn_read &req, const agn_result &out,
                         hipStream_t s);
int tune_counter_dense(const agn_log &log, const agn_read &req, const agn_result &out,
                       hipStream_t st, int rounds, int *choice, float *ms);
int launch_tags(const agn_log &log, const agn_read &req, const agn_result &out,
                hipStream_t s);
int launch_gst_min(uint32_t D, uint64_t P, uint64_t E, const uint64_t *clocks,
                   const uint8_t *defined, uint64_t *out, hipStream_t s);
int launch_gst_finalize(uint32_t D, uint64_t E, uint64_t *vec, hipStream_t s);
int launch_log_ingest(const agn_log_records &r, uint32_t D, uint64_t n_keys,
                      const uint64_t *max_t, const uint64_t *max_m, uint32_t base,
                      const agn_log &out, uint64_t *totals, hipStream_t st);
int launch_ss_lookup(const agn_ss_cache &c, uint64_t n_req, const uint64_t *keys,
                     const uint64_t *R, const uint64_t *Rm, uint64_t *sct, uint64_t *sctm,
                     uint8_t *sct_ign, int64_t *base, uint8_t *first, uint8_t *status,
                     hipStream_t st);
int launch_ss_store(const agn_ss_cache &c, const uint64_t *key_off, const uint64_t *key_len,
                    uint64_t n_req,
                    const uint64_t *keys, const uint8_t *is_first, const uint8_t *status,
                    const uint8_t *should_gc, const agn_result &res, const int64_t *handle,
                    uint8_t *prune, uint64_t *thr, uint64_t *thrm, hipStream_t st);
int launch_prune_mark(const agn_log &log, const uint8_t *prune, const uint64_t *thr,
                      const uint64_t *thr_mask, uint8_t *keep, uint64_t *cnt, uint64_t *rcnt,
                      hipStream_t st);
int launch_prune_scatter_seg(const agn_log &log, const agn_log &out, const uint8_t *prune,
                             const uint8_t *keep, const uint64_t *tstart, uint32_t *flags,
                             hipStream_t st);
int launch_prune_inplace(const agn_log &view, uint64_t *key_len, uint32_t *key_id0,
                         uint32_t *key_lcap, const uint8_t *prune, const uint64_t *thr,
                         const uint64_t *thr_mask, uint32_t *meta, uint32_t *flags,
                         hipStream_t st);
int launch_prune_segmented(const agn_log &log, const uint8_t *prune, const uint64_t *thr,
                           const uint64_t *thr_mask, const agn_log &out, uint32_t *flags,
                           hipStream_t st);
int launch_seg_totals(const agn_log &out, uint64_t *totals, hipStream_t st);
int launch_prune_ops(const agn_log &log, const uint8_t *prune, const uint64_t *thr,
                     const uint64_t *thr_mask, const agn_log &out, uint32_t *flags,
                     uint64_t *totals, hipStream_t st);
int launch_gst_scalar(uint32_t D, uint64_t E, uint64_t *vec, uint64_t *out_gst, hipStream_t s);
int launch_dep_check(uint32_t D, uint64_t n, const uint64_t *deps, const uint64_t *dm,
                     const uint32_t *origin, const uint32_t *part, uint64_t n_parts,
                     const uint64_t *pc, const uint64_t *pm, uint8_t *ok, hipStream_t s);
int launch_select_base(uint32_t D, uint64_t n_req, const uint64_t *cache_off,
                       const uint64_t *clocks, const uint64_t *clock_mask,
                       const uint64_t *R, const uint64_t *R_mask, int32_t *out_idx,
                       uint8_t *out_is_first, hipStream_t s);

}  // namespace agn
