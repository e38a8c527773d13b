// gst.hip — global stable time and base-snapshot selection on gfx950.
//
// get_min_time/1 (src/stable_time_functions.erl:51-85): per DC, the min of
// the partition clocks that contain it; an `undefined` partition zeroes every
// output DC.  Layout [E epochs][P partitions][D] u64, absent = UINT64_MAX, so
// the dict "union of keys" survives an elementwise min; the extra word D of
// each output row carries "every partition defined" (min of 1/0), which is
// also what the RCCL ncclMin allreduce across GPUs combines
// (meta_data_sender merge, src/meta_data_sender.erl:230-255).
//
// k_gst_min: each block reduces a band of partition rows of one epoch into an
// LDS column-min (ds_min_u64), then one global atomicMin per column.  HBM bytes
// per epoch: 8*P*D + P (defined) + 8*(D+1).
//
// k_select_base: vector_orddict:get_smaller/2 (src/vector_orddict.erl:74-87):
// first cached clock (newest first) that is le the read clock.
#include "common.hpp"

namespace agn {
namespace {

__global__ void k_gst_init(uint64_t *out, uint32_t D, uint64_t E) {
    const uint64_t n = E * (uint64_t)(D + 1);
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (uint64_t)gridDim.x * blockDim.x)
        out[x] = ((x % (D + 1)) == D) ? 1ull : ~0ull;
}

constexpr int GST_THREADS = 256;
constexpr uint32_t GST_MAX_LDS_D = 4096;

__global__ __launch_bounds__(GST_THREADS) void k_gst_min(const uint64_t *__restrict__ clocks,
                                                         const uint8_t *__restrict__ defined,
                                                         uint64_t *out, uint32_t D, uint64_t P,
                                                         uint64_t rows_per_block,
                                                         uint64_t bands) {
    __shared__ uint64_t colmin[GST_MAX_LDS_D];
    __shared__ int all_def;
    const uint64_t e = blockIdx.x / bands;
    const uint64_t band = blockIdx.x % bands;
    const uint64_t p0 = band * rows_per_block;
    const uint64_t p1 = p0 + rows_per_block < P ? p0 + rows_per_block : P;
    for (uint32_t d = threadIdx.x; d < D; d += GST_THREADS) colmin[d] = ~0ull;
    if (threadIdx.x == 0) all_def = 1;
    __syncthreads();

    // undefined partitions contribute no clock, only the flag
    if (defined) {
        for (uint64_t p = p0 + threadIdx.x; p < p1; p += GST_THREADS)
            if (!defined[e * P + p]) all_def = 0;
    }
    __syncthreads();
    const uint64_t *base = clocks + (e * P + p0) * D;
    const uint64_t n = (p1 - p0) * D;
    // flat walk of the band; consecutive threads read consecutive words
    uint64_t acc = ~0ull;
    uint32_t acc_d = 0xffffffffu;
    for (uint64_t x = threadIdx.x; x < n; x += GST_THREADS) {
        const uint64_t p = p0 + x / D;
        const uint32_t d = (uint32_t)(x % D);
        if (defined && !defined[e * P + p]) continue;
        const uint64_t v = base[x];
        if (d == acc_d) {
            acc = v < acc ? v : acc;
        } else {
            if (acc_d != 0xffffffffu) atomicMin((unsigned long long *)&colmin[acc_d], acc);
            acc_d = d;
            acc = v;
        }
    }
    if (acc_d != 0xffffffffu) atomicMin((unsigned long long *)&colmin[acc_d], acc);
    __syncthreads();
    uint64_t *o = out + e * (uint64_t)(D + 1);
    for (uint32_t d = threadIdx.x; d < D; d += GST_THREADS)
        if (colmin[d] != ~0ull) atomicMin((unsigned long long *)&o[d], colmin[d]);
    if (threadIdx.x == 0 && !all_def) atomicMin((unsigned long long *)&o[D], 0ull);
}

// Column-resident form for D | 512 (D a power of two <= 512, e.g. the cfg5
// D = 256): thread t owns the DC pair c = 2t mod D of row offset 2t div D,
// so its column never changes; it streams its band's rows with 16-byte loads
// (4 rows in flight) into two running minima held in registers.  The
// RG = 512 / D threads that share a column pair fold through LDS once, and
// the block issues ONE global atomicMin per column (bands blocks per epoch).
// Undefined partitions only clear word D (they contribute no clock).
typedef unsigned long long u64x2g __attribute__((ext_vector_type(2)));

template <bool DEF, int U, bool NT>
__global__ __launch_bounds__(GST_THREADS) void k_gst_cols(const uint64_t *__restrict__ clocks,
                                                          const uint8_t *__restrict__ defined,
                                                          uint64_t *out, uint32_t D, uint64_t P,
                                                          uint64_t rows_per_block,
                                                          uint64_t bands) {
    __shared__ uint64_t red[2 * GST_THREADS];
    __shared__ int all_def;
    const uint32_t t = threadIdx.x;
    const uint32_t RG = (2u * GST_THREADS) / D;        // rows per block step
    const uint32_t c = (2u * t) % D, r0 = (2u * t) / D;
    const uint64_t e = blockIdx.x / bands, band = blockIdx.x % bands;
    const uint64_t p0 = band * rows_per_block;
    const uint64_t p1 = p0 + rows_per_block < P ? p0 + rows_per_block : P;
    if (t == 0) all_def = 1;
    __syncthreads();
    uint64_t m0 = ~0ull, m1 = ~0ull;
    const uint64_t *base = clocks + e * P * D + c;
    uint64_t p = p0 + r0;
    for (; p + (U - 1) * RG < p1; p += U * RG) {
        u64x2g v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const u64x2g *q = reinterpret_cast<const u64x2g *>(base + (p + (uint64_t)k * RG) * D);
            v[k] = NT ? __builtin_nontemporal_load(q) : *q;
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            bool ok = true;
            if (DEF) ok = defined[e * P + p + (uint64_t)k * RG] != 0;
            if (ok) {
                m0 = v[k].x < m0 ? v[k].x : m0;
                m1 = v[k].y < m1 ? v[k].y : m1;
            } else {
                all_def = 0;
            }
        }
    }
    for (; p < p1; p += RG) {
        const u64x2g v = *reinterpret_cast<const u64x2g *>(base + p * D);
        if (!DEF || defined[e * P + p]) {
            m0 = v.x < m0 ? v.x : m0;
            m1 = v.y < m1 ? v.y : m1;
        } else {
            all_def = 0;
        }
    }
    red[2 * t] = m0;
    red[2 * t + 1] = m1;
    __syncthreads();
    uint64_t *o = out + e * (uint64_t)(D + 1);
    for (uint32_t d = t; d < D; d += GST_THREADS) {
        uint64_t m = ~0ull;
        for (uint32_t r = 0; r < RG; ++r) {
            const uint64_t v = red[r * D + d];
            m = v < m ? v : m;
        }
        if (m != ~0ull) {
            if (bands == 1) o[d] = m;
            else atomicMin((unsigned long long *)&o[d], (unsigned long long)m);
        }
    }
    if (t == 0 && !all_def) atomicMin((unsigned long long *)&o[D], 0ull);
}

__global__ void k_gst_finalize(uint64_t *vec, uint32_t D, uint64_t E) {
    const uint64_t n = E * (uint64_t)D;
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e = x / D, d = x % D;
        uint64_t *row = vec + e * (uint64_t)(D + 1);
        if (row[D] == 0ull && row[d] != ~0ull) row[d] = 0ull;  // FoundUndefined (:78-82)
    }
}

// Gentlerain scalar GST: one wave per epoch row, lanes over DCs.
__global__ __launch_bounds__(256) void k_gst_scalar(uint64_t *vec, uint64_t *out_gst,
                                                    uint32_t D, uint64_t E) {
    const uint64_t e = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    if (e >= E) return;
    const int lane = lane_id();
    uint64_t *row = vec + e * (uint64_t)(D + 1);
    uint64_t m = ~0ull;
    for (uint32_t d = lane; d < D; d += AGN_WAVE) m = row[d] < m ? row[d] : m;
#pragma unroll
    for (int x = 1; x < AGN_WAVE; x <<= 1) {
        const uint64_t o = shfl_xor_u64(m, x);
        m = o < m ? o : m;
    }
    if (m != ~0ull)
        for (uint32_t d = lane; d < D; d += AGN_WAVE)
            if (row[d] != ~0ull) row[d] = m;  // dict:map(fun(_K, _V) -> GST end)
    if (lane == 0 && out_gst) out_gst[e] = m;
}

// try_store/2's vectorclock:ge(Cur, Deps) with the origin entry zeroed on
// both sides.  A group of G lanes per transaction (G = pow2 >= D, at most
// 64; 64 / G transactions per wave, so a wave reads 64 consecutive clock
// words), lanes over DCs, one ballot folded per group.  The waves of a
// resident grid stride over tiles of 64 / G transactions, U tiles per step
// with all their loads issued before the first compare, and the partition
// clocks (a few KB: P x D words and masks) are staged in LDS once per block
// when they fit (STAGE), so a tile's only memory round trip is its own
// words.  One wave per transaction (round 4) ran 3.6e9 waves/s against the
// dispatcher: 0.036 of 8 TB/s at D = 8 (profiles/r05/bench_dep_check*.log).
constexpr int DEP_U = 4;
constexpr size_t DEP_LDS = 48u << 10;  // bytes of partition clocks staged per block

template <int G, bool STAGE>
__global__ __launch_bounds__(256) void k_dep_check(uint32_t D, uint64_t n,
                                                   const uint64_t *__restrict__ deps,
                                                   const uint64_t *__restrict__ dm,
                                                   const uint32_t *__restrict__ origin,
                                                   const uint32_t *__restrict__ part,
                                                   uint64_t n_parts,
                                                   const uint64_t *__restrict__ pc,
                                                   const uint64_t *__restrict__ pm,
                                                   uint8_t *__restrict__ ok) {
    extern __shared__ uint64_t sh[];  // STAGE: pc [n_parts][D], then pm [n_parts][W]
    constexpr int TPW = AGN_WAVE / G;  // transactions per tile (one wave)
    const uint32_t W = n_words(D);
    const uint64_t *cpc = pc, *cpm = pm;
    if constexpr (STAGE) {
        const uint64_t nc = n_parts * D, nm = pm ? n_parts * W : 0;
        for (uint64_t x = threadIdx.x; x < nc; x += blockDim.x) sh[x] = pc[x];
        for (uint64_t x = threadIdx.x; x < nm; x += blockDim.x) sh[nc + x] = pm[x];
        __syncthreads();
        cpc = sh;
        cpm = pm ? sh + nc : nullptr;
    }
    const int lane = lane_id();
    const int g = lane / G, gl = lane % G;
    const uint64_t nt = (n + TPW - 1) / TPW;                       // tiles
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    for (uint64_t tile = w; tile < nt; tile += waves * DEP_U) {
        uint64_t t[DEP_U], p[DEP_U], dv[DEP_U], dmw[DEP_U];
        uint32_t o[DEP_U];
        bool live[DEP_U];
        const uint32_t dl = (uint32_t)gl < D ? (uint32_t)gl : D - 1u;  // D <= G: lane gl's DC
#pragma unroll
        for (int u = 0; u < DEP_U; ++u) {  // the step's words, all issued before any compare
            const uint64_t tu = (tile + (uint64_t)u * waves) * TPW + (uint64_t)g;
            live[u] = tu < n;
            t[u] = live[u] ? tu : 0ull;
            p[u] = part[t[u]];
            o[u] = origin[t[u]];
            dv[u] = deps[t[u] * D + dl];
            dmw[u] = dm ? dm[t[u] * W + (dl >> 6)] : ~0ull;
        }
        bool bad[DEP_U];
#pragma unroll
        for (int u = 0; u < DEP_U; ++u) {
            bad[u] = live[u] && p[u] >= n_parts;
            const uint64_t pp = p[u];
            if (!live[u] || bad[u]) continue;  // an unknown partition: not applicable
            if (D <= (uint32_t)G) {  // one DC per lane, its words preloaded above
                const uint32_t d = (uint32_t)gl;
                if (d < D && d != o[u] && ((dmw[u] >> (d & 63)) & 1ull)) {
                    const bool pb = !cpm || ((cpm[pp * W + (d >> 6)] >> (d & 63)) & 1ull);
                    const uint64_t b = pb ? cpc[pp * D + d] : 0ull;
                    if (dv[u] > b) bad[u] = true;
                }
                continue;
            }
            for (uint32_t d = (uint32_t)gl; d < D; d += G) {
                if (d == o[u]) continue;
                const bool pa = !dm || ((dm[t[u] * W + (d >> 6)] >> (d & 63)) & 1ull);
                const bool pb = !cpm || ((cpm[pp * W + (d >> 6)] >> (d & 63)) & 1ull);
                const uint64_t b = pb ? cpc[pp * D + d] : 0ull;
                if (pa && deps[t[u] * D + d] > b) bad[u] = true;
            }
        }
        const uint64_t gm = (G == AGN_WAVE ? ~0ull : ((1ull << G) - 1ull)) << (g * G);
#pragma unroll
        for (int u = 0; u < DEP_U; ++u) {
            const uint64_t any = ballot(bad[u]);
            if (live[u] && gl == 0) ok[t[u]] = (any & gm) ? 0 : 1;
        }
    }
}

__global__ void k_select_base(uint32_t D, uint64_t n_req, const uint64_t *cache_off,
                              const uint64_t *clocks, const uint64_t *clock_mask,
                              const uint64_t *R, const uint64_t *R_mask, int32_t *out_idx,
                              uint8_t *out_is_first) {
    const uint32_t W = n_words(D);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_req;
         i += (uint64_t)gridDim.x * blockDim.x) {
        int32_t idx = -1;
        uint8_t first = 1;
        const uint64_t c0 = cache_off[i], c1 = cache_off[i + 1];
        for (uint64_t c = c0; c < c1; ++c) {
            bool le = true;  // vectorclock:le(Clock, R): missing entries read 0
            for (uint32_t d = 0; d < D && le; ++d) {
                const bool pa = !clock_mask || ((clock_mask[c * W + (d >> 6)] >> (d & 63)) & 1ull);
                if (!pa) continue;
                const bool pb = !R_mask || ((R_mask[i * W + (d >> 6)] >> (d & 63)) & 1ull);
                const uint64_t b = pb ? R[i * D + d] : 0ull;
                le = clocks[c * D + d] <= b;
            }
            if (le) {
                idx = (int32_t)(c - c0);
                break;
            }
            first = 0;
        }
        out_idx[i] = idx;
        out_is_first[i] = first;
    }
}

}  // namespace

int launch_gst_min(uint32_t D, uint64_t P, uint64_t E, const uint64_t *clocks,
                   const uint8_t *defined, uint64_t *out, hipStream_t s) {
    if (D == 0 || D > GST_MAX_LDS_D) return fail(AGN_ENOTSUP, "gst: D=%u unsupported", D);
    hipLaunchKernelGGL(k_gst_init, dim3(grid_for(E * (D + 1), 256, 1024)), dim3(256), 0, s,
                       out, D, E);
    AGN_HIP(hipGetLastError());
    if (P == 0 || E == 0) return AGN_OK;
    if (D <= 2u * GST_THREADS && ((2u * GST_THREADS) % D) == 0 && (D % 2u) == 0 &&
        ((uintptr_t)clocks % 16u) == 0) {
        // column-resident kernel: ~target blocks over all epochs, >= 32 block
        // steps each.  A/B knobs: AGN_GST_BLOCKS (target, default 1024),
        // AGN_GST_UNROLL = 4 | 8 (rows in flight per thread)
        const char *eb = AGN_KNOB("AGN_GST_BLOCKS");
        const char *eu = AGN_KNOB("AGN_GST_UNROLL");
        const uint64_t target = eb ? strtoull(eb, nullptr, 10) : 1024;
        const int unroll = (eu && eu[0] == '8') ? 8 : 4;
        // non-temporal row loads (default; AGN_GST_NT=0 for plain loads): the
        // clocks are streamed once, 0.366 -> 0.311 ms on cfg5 (scripts/ab_gst.py,
        // profiles/r02/ab_gst.log)
        const char *en = AGN_KNOB("AGN_GST_NT");
        const bool nt = !(en && en[0] == '0');
        const uint64_t RG = (2u * GST_THREADS) / D;
        uint64_t bands = ((target ? target : 1024) + E - 1) / E;
        uint64_t rows = (P + bands - 1) / bands;
        const uint64_t min_rows = 32 * RG;
        if (rows < min_rows) rows = min_rows;
        rows = (rows + RG - 1) / RG * RG;  // whole block steps
        bands = (P + rows - 1) / rows;
        const uint64_t blocks = E * bands;
        if (blocks > 0x7fffffffull) return fail(AGN_ENOTSUP, "gst: grid too large");
#define AGN_G(DEFV, UV, NTV)                                                                    \
    hipLaunchKernelGGL((k_gst_cols<DEFV, UV, NTV>), dim3((unsigned)blocks), dim3(GST_THREADS), 0, \
                       s, clocks, defined, out, D, P, rows, bands)
#define AGN_GU(DEFV)                                                                            \
    do {                                                                                        \
        if (unroll == 8) {                                                                      \
            if (nt) AGN_G(DEFV, 8, true);                                                       \
            else AGN_G(DEFV, 8, false);                                                         \
        } else {                                                                                \
            if (nt) AGN_G(DEFV, 4, true);                                                       \
            else AGN_G(DEFV, 4, false);                                                         \
        }                                                                                       \
    } while (0)
        if (defined) AGN_GU(true);
        else AGN_GU(false);
#undef AGN_GU
#undef AGN_G
        AGN_HIP(hipGetLastError());
        return AGN_OK;
    }
    // general D: ~16 KB of clocks per block; at least 1 row
    uint64_t rows = (16384 / 8) / D;
    if (rows < 1) rows = 1;
    const uint64_t bands = (P + rows - 1) / rows;
    const uint64_t blocks = E * bands;
    if (blocks > 0x7fffffffull) return fail(AGN_ENOTSUP, "gst: grid too large");
    hipLaunchKernelGGL(k_gst_min, dim3((unsigned)blocks), dim3(GST_THREADS), 0, s, clocks,
                       defined, out, D, P, rows, bands);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

int launch_gst_finalize(uint32_t D, uint64_t E, uint64_t *vec, hipStream_t s) {
    if (E == 0 || D == 0) return AGN_OK;
    hipLaunchKernelGGL(k_gst_finalize, dim3(grid_for(E * D, 256, 1024)), dim3(256), 0, s, vec,
                       D, E);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

int launch_gst_scalar(uint32_t D, uint64_t E, uint64_t *vec, uint64_t *out_gst, hipStream_t s) {
    if (E == 0) return AGN_OK;
    hipLaunchKernelGGL(k_gst_scalar, dim3((unsigned)((E + 3) / 4)), dim3(256), 0, s, vec, out_gst,
                       D, E);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

int launch_dep_check(uint32_t D, uint64_t n, const uint64_t *deps, const uint64_t *dm,
                     const uint32_t *origin, const uint32_t *part, uint64_t n_parts,
                     const uint64_t *pc, const uint64_t *pm, uint8_t *ok, hipStream_t s) {
    if (n == 0) return AGN_OK;
    const uint32_t G = D <= 1 ? 1 : D <= 2 ? 2 : D <= 4 ? 4 : D <= 8 ? 8 : D <= 16 ? 16
                     : D <= 32 ? 32 : 64;
    const uint64_t W = n_words(D);
    const size_t stage = (size_t)(n_parts * D + (pm ? n_parts * W : 0)) * 8u;
    const bool st = n_parts > 0 && stage <= DEP_LDS;
    // a resident grid: the tiles (64 / G transactions each) over 4-wave
    // blocks, at most 8 blocks per CU
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint64_t tiles = (n + (AGN_WAVE / G) - 1) / (AGN_WAVE / G);
    const uint64_t want = (tiles + 4 * DEP_U - 1) / (4 * DEP_U);
    const uint64_t cap = (uint64_t)(cus > 0 ? cus : 256) * 8u;
    const unsigned nb = (unsigned)(want < cap ? want : cap);
#define AGN_DEP(GV)                                                                             \
    do {                                                                                        \
        if (st) hipLaunchKernelGGL((k_dep_check<GV, true>), dim3(nb), dim3(256), stage, s, D, n, \
                                   deps, dm, origin, part, n_parts, pc, pm, ok);                 \
        else hipLaunchKernelGGL((k_dep_check<GV, false>), dim3(nb), dim3(256), 0, s, D, n, deps, \
                                dm, origin, part, n_parts, pc, pm, ok);                          \
    } while (0)
    switch (G) {
        case 1: AGN_DEP(1); break;
        case 2: AGN_DEP(2); break;
        case 4: AGN_DEP(4); break;
        case 8: AGN_DEP(8); break;
        case 16: AGN_DEP(16); break;
        case 32: AGN_DEP(32); break;
        default: AGN_DEP(64); break;
    }
#undef AGN_DEP
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

int launch_select_base(uint32_t D, uint64_t n_req, const uint64_t *cache_off,
                       const uint64_t *clocks, const uint64_t *clock_mask, const uint64_t *R,
                       const uint64_t *R_mask, int32_t *out_idx, uint8_t *out_is_first,
                       hipStream_t s) {
    if (n_req == 0) return AGN_OK;
    hipLaunchKernelGGL(k_select_base, dim3(grid_for(n_req, 256, 4096)), dim3(256), 0, s, D,
                       n_req, cache_off, clocks, clock_mask, R, R_mask, out_idx, out_is_first);
    AGN_HIP(hipGetLastError());
    return AGN_OK;
}

}  // namespace agn
