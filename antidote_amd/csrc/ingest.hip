// ingest.hip — the logging_vnode read paths as device passes:
// get_ops_from_log / filter_terms_for_key / handle_commit
// (src/logging_vnode.erl:522-549, 660-779) for every key at once, producing a
// device op log (agn_log CSR) — the get_up_to_time fallback read and the
// load_from_log recovery ingest of materializer_vnode (:288-319).
//
// The sequential walk "buffer updates per TxId, emit them at the commit
// record" becomes a hash join + a stable sort:
//   1. k_commit_map  every commit record inserts txid -> record index into an
//                    open-addressing table (one commit per transaction);
//   2. k_join        every update record looks up its transaction's commit c;
//                    it is emitted iff c comes later in the log and
//                    check_max_time(snapshot_time(c), Max[key]) holds; its
//                    sort key is (key << pb) | c with pb = the bits of a
//                    record index (else n_keys << pb, after every key);
//   3. stable radix sort of (sort key, 32-bit record index) over only the
//                    kb + pb bits a key can have — per key: commit order,
//                    then update order, exactly dict:append's order;
//   4. k_bounds      key_off from the sorted keys; k_rows / k_fields gather
//                    the OpSSCommit rows (snapshot_time with the commit DC
//                    set to the commit time) and the per-op fields; removal
//                    lists through a scan of their lengths.
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace agn {
namespace {

constexpr uint64_t EMPTY = ~0ull;

// bits needed for the values 0..v
inline int bits_for(uint64_t v) {
    int b = 0;
    while (b < 64 && (v >> b) != 0) ++b;
    return b ? b : 1;
}

__device__ __forceinline__ uint64_t slot_of(uint64_t t, uint64_t mask) {
    return (t * 0x9E3779B97F4A7C15ull) >> 20 & mask;
}

// The commit table: open addressing over {txid, first commit index} slot
// pairs (one 16-byte access per probe), sized on the device from the number
// of commit records (a power of two >= 1.5x, so a log of 10M commits probes a
// 256 MiB table that the MALL can hold) -- tab[0] of the scratch holds the
// mask, the slots follow.
__global__ void k_count_commits(agn_log_records r, unsigned long long *cnt) {
    uint64_t c = 0;
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < r.n;
         x += (uint64_t)gridDim.x * blockDim.x)
        c += r.kind[x] == AGN_REC_COMMIT;
    if (c) atomicAdd(cnt, (unsigned long long)c);
}

__device__ __forceinline__ uint64_t table_mask(const unsigned long long *cnt) {
    uint64_t T = 16;
    const uint64_t want = *cnt + *cnt / 2 + 1;
    while (T < want) T <<= 1;
    return T - 1;
}

__global__ void k_fill(uint64_t *tab, const unsigned long long *cnt) {
    const uint64_t mask = table_mask(cnt);
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x <= mask;
         x += (uint64_t)gridDim.x * blockDim.x) {
        tab[2 * x] = EMPTY;
        tab[2 * x + 1] = EMPTY;
    }
}

__global__ void k_commit_map(agn_log_records r, uint64_t *tab, const unsigned long long *cnt) {
    const uint64_t mask = table_mask(cnt);
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < r.n;
         x += (uint64_t)gridDim.x * blockDim.x) {
        if (r.kind[x] != AGN_REC_COMMIT) continue;
        const uint64_t t = r.txid[x];
        uint64_t s = slot_of(t, mask);
        for (;;) {
            const uint64_t prev = atomicCAS((unsigned long long *)&tab[2 * s],
                                            (unsigned long long)EMPTY, (unsigned long long)t);
            if (prev == EMPTY || prev == t) {
                atomicMin((unsigned long long *)&tab[2 * s + 1], (unsigned long long)x);
                break;
            }
            s = (s + 1) & mask;
        }
    }
}

typedef unsigned long long u64x2i __attribute__((ext_vector_type(2)));

__global__ void k_join(agn_log_records r, uint32_t D, const uint64_t *__restrict__ tab,
                       const unsigned long long *__restrict__ cnt,
                       const uint64_t *__restrict__ max_t, const uint64_t *__restrict__ max_m,
                       int pb, uint64_t none, uint64_t *__restrict__ skey,
                       uint32_t *__restrict__ sval, unsigned long long *__restrict__ n_out) {
    const uint32_t W = n_words(D);
    const uint64_t mask = table_mask(cnt);
    const u64x2i *slots = reinterpret_cast<const u64x2i *>(tab);
    uint64_t emitted = 0;
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < r.n;
         x += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t key = none;
        if (r.kind[x] == AGN_REC_UPDATE) {
            const uint64_t t = r.txid[x];
            uint64_t s = slot_of(t, mask), c = EMPTY;
            for (;;) {
                const u64x2i h = slots[s];
                if (h.x == EMPTY) break;
                if (h.x == t) {
                    c = h.y;
                    break;
                }
                s = (s + 1) & mask;
            }
            const uint64_t k = r.key[x];
            // the commit follows the update; a key outside the log's key range
            // is not this partition's (never emitted, never indexed)
            bool emit = c != EMPTY && c > x && k < (none >> pb);
            if (emit && max_t) {  // check_max_time: le(SnapshotTime, Max), missing = 0
                for (uint32_t d = 0; d < D && emit; ++d) {
                    const bool pa = !r.ss_mask || ((r.ss_mask[c * W + (d >> 6)] >> (d & 63)) & 1ull);
                    if (!pa) continue;
                    const bool pb = !max_m || ((max_m[k * W + (d >> 6)] >> (d & 63)) & 1ull);
                    emit = r.ss[c * D + d] <= (pb ? max_t[k * D + d] : 0ull);
                }
            }
            if (emit) key = (k << pb) | c;
        }
        emitted += key != none;
        skey[x] = key;
        sval[x] = (uint32_t)x;
    }
    // the emitted count: one same-address atomic per thread after the loop
    // (the compiler folds a wave's into one), not one per record -- per-record
    // atomics, even wave-aggregated, serialised k_join at 5.7 ms for 30M records
    if (emitted) atomicAdd(n_out, (unsigned long long)emitted);
}

// key_off[k] = first sorted position with key >= k; positions [0, E) are
// the emitted ops, sorted by key.
__global__ void k_bounds(const uint64_t *__restrict__ skey, const unsigned long long *__restrict__ n_out,
                         uint64_t n_keys, int pb, uint64_t *__restrict__ key_off) {
    const uint64_t E = *n_out;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p <= E;
         p += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t lo = p == 0 ? 0ull : (skey[p - 1] >> pb) + 1ull;
        const uint64_t hi = p == E ? n_keys : (skey[p] >> pb);
        for (uint64_t k = lo; k <= hi && k <= n_keys; ++k) key_off[k] = p;
    }
}

__global__ void k_rows(agn_log_records r, uint32_t D, const uint64_t *__restrict__ skey,
                       const unsigned long long *__restrict__ n_out, int pb,
                       uint64_t *__restrict__ oc, uint64_t *__restrict__ ocm) {
    const uint64_t E = *n_out;
    const uint32_t W = n_words(D);
    const uint64_t pmask = (1ull << pb) - 1ull;
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < E * D;
         x += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p = x / D, d = x % D;
        const uint64_t c = skey[p] & pmask;
        // OpSSCommit: snapshot_time with the commit DC replaced by the commit time
        oc[x] = (d == r.commit_dc[c]) ? r.commit_time[c] : r.ss[c * D + d];
        if (ocm && d < W) {
            const uint64_t m = r.ss_mask ? r.ss_mask[c * W + d] : ~0ull;
            const uint32_t cd = r.commit_dc[c];
            ocm[p * W + d] = ((cd >> 6) == d ? m | (1ull << (cd & 63)) : m) &
                             ((d + 1 < W || D % 64 == 0) ? ~0ull : ((1ull << (D % 64)) - 1ull));
        }
    }
}

__global__ void k_fields(agn_log_records r, const uint64_t *__restrict__ skey,
                         const uint32_t *__restrict__ sval,
                         const unsigned long long *__restrict__ n_out,
                         const uint64_t *__restrict__ key_off, uint32_t base, int pb, agn_log out,
                         uint32_t *__restrict__ rlen) {
    const uint64_t E = *n_out;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < E;
         p += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t u = sval[p], k = skey[p] >> pb;
        ((uint32_t *)out.op_id)[p] = base + (uint32_t)(p - key_off[k]);
        if (out.txid) ((uint64_t *)out.txid)[p] = r.txid[u];
        if (out.eff) ((int64_t *)out.eff)[p] = r.eff[u];
        if (out.tag) ((uint32_t *)out.tag)[p] = r.tag[u];
        if (out.add_tok) ((uint64_t *)out.add_tok)[p] = r.add_tok[u];
        if (rlen) rlen[p] = r.rem_off[u + 1] - r.rem_off[u];
    }
}

__global__ void k_rem_copy(agn_log_records r, const uint32_t *__restrict__ sval,
                           const unsigned long long *__restrict__ n_out, agn_log out) {
    const uint64_t E = *n_out;
    const uint64_t lane = threadIdx.x & 63u;
    for (uint64_t p = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; p < E;
         p += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
        const uint64_t u = sval[p];
        const uint32_t s = r.rem_off[u], n = r.rem_off[u + 1] - s;
        const uint32_t d = out.rem_off[p];
        for (uint32_t j = (uint32_t)lane; j < n; j += 64) ((uint64_t *)out.rem_tok)[d + j] = r.rem_tok[s + j];
    }
}

__global__ void k_rem_off(const uint32_t *__restrict__ scanned,
                          const unsigned long long *__restrict__ n_out, uint32_t *__restrict__ ro) {
    const uint64_t E = *n_out;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < E;
         p += (uint64_t)gridDim.x * blockDim.x)
        ro[p + 1] = scanned[p];
}

__global__ void k_totals(const unsigned long long *n_out, const uint32_t *rem_off,
                         uint64_t *totals) {
    const uint64_t E = *n_out;
    totals[0] = E;
    totals[1] = rem_off ? rem_off[E] : 0ull;
}

}  // namespace

int launch_log_ingest(const agn_log_records &r, uint32_t D, uint64_t n_keys,
                      const uint64_t *max_t, const uint64_t *max_m, uint32_t base,
                      const agn_log &out, uint64_t *totals, hipStream_t st) {
    const uint64_t n = r.n;
    if (n > 0xffffffffull) return fail(AGN_ENOTSUP, "log_ingest: %llu records (max 2^32 - 1)",
                                       (unsigned long long)n);
    // sort key (key << pb) | commit index: pb bits for a record index, kb for
    // a key or the "not emitted" marker n_keys
    const int pb = bits_for(n ? n - 1 : 0), kb = bits_for(n_keys);
    if (pb + kb > 64) return fail(AGN_ENOTSUP, "log_ingest: %d + %d sort-key bits", pb, kb);
    const uint64_t none = n_keys << pb;
    uint64_t T = 16;  // table slots for the worst case (every record a commit)
    while (T < n + n / 2 + 1) T <<= 1;
    size_t sort_bytes = 0, scan_bytes = 0;
    AGN_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (uint64_t *)nullptr,
                                               (uint64_t *)nullptr, (uint32_t *)nullptr,
                                               (uint32_t *)nullptr, (int)n, 0, pb + kb, st));
    AGN_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, scan_bytes, (uint32_t *)nullptr,
                                             (uint32_t *)nullptr, (int)n, st));
    const size_t tb = ((sort_bytes > scan_bytes ? sort_bytes : scan_bytes) + 255) / 256 * 256;
    const size_t words = 2 * T + 2 * n + 4;  // table k0 k1 n_out cnt (+ v0 v1 as 32-bit)
    const size_t bytes = tb + words * 8 + 2 * ((n + 1) / 2 * 2) * 4 + (n + 1) * 4 + 512;
    uint8_t *scratch = nullptr;
    AGN_HIP(pool_malloc((void **)&scratch, bytes, st));
    void *tmp = scratch;
    uint64_t *tab = (uint64_t *)(scratch + tb);
    uint64_t *k0 = tab + 2 * T, *k1 = k0 + n;
    unsigned long long *n_out = (unsigned long long *)(k1 + n);  // [0] emitted, [2] commits
    uint32_t *v0 = (uint32_t *)(n_out + 4), *v1 = v0 + (n + 1) / 2 * 2;
    uint32_t *rlen = v1 + (n + 1) / 2 * 2;
    const unsigned g = 2048;
    hipError_t e = hipSuccess;
    e = hipMemsetAsync(n_out, 0, 32, st);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_count_commits, dim3(g), dim3(256), 0, st, r, n_out + 2);
        hipLaunchKernelGGL(k_fill, dim3(g), dim3(256), 0, st, tab, n_out + 2);
        hipLaunchKernelGGL(k_commit_map, dim3(g), dim3(256), 0, st, r, tab, n_out + 2);
        hipLaunchKernelGGL(k_join, dim3(g), dim3(256), 0, st, r, D, tab, n_out + 2, max_t, max_m,
                           pb, none, k0, v0, n_out);
        e = hipcub::DeviceRadixSort::SortPairs(tmp, sort_bytes, k0, k1, v0, v1, (int)n, 0, pb + kb,
                                               st);
    }
    if (e == hipSuccess && r.rem_off) e = hipMemsetAsync(rlen, 0, (n + 1) * sizeof(uint32_t), st);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_bounds, dim3(g), dim3(256), 0, st, k1, n_out, n_keys, pb,
                           (uint64_t *)out.key_off);
        hipLaunchKernelGGL(k_rows, dim3(g), dim3(256), 0, st, r, D, k1, n_out, pb,
                           (uint64_t *)out.oc, (uint64_t *)out.oc_mask);
        hipLaunchKernelGGL(k_fields, dim3(g), dim3(256), 0, st, r, k1, v1, n_out,
                           (const uint64_t *)out.key_off, base, pb, out,
                           r.rem_off ? rlen : (uint32_t *)nullptr);
        e = hipGetLastError();
    }
    if (e == hipSuccess && r.rem_off) {
        // removal lists: lengths of the emitted ops (zero beyond E) -> in-place
        // inclusive scan -> out.rem_off[1..E] -> token copy
        e = hipcub::DeviceScan::InclusiveSum(tmp, scan_bytes, rlen, rlen, (int)n, st);
        if (e == hipSuccess) e = hipMemsetAsync((void *)out.rem_off, 0, sizeof(uint32_t), st);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_rem_off, dim3(g), dim3(256), 0, st, rlen, n_out,
                               (uint32_t *)out.rem_off);
            hipLaunchKernelGGL(k_rem_copy, dim3(g), dim3(256), 0, st, r, v1, n_out, out);
            e = hipGetLastError();
        }
    }
    if (e == hipSuccess) e = hipGetLastError();
    if (totals && e == hipSuccess) {
        hipLaunchKernelGGL(k_totals, dim3(1), dim3(1), 0, st, n_out, (const uint32_t *)out.rem_off,
                           totals);
        e = hipGetLastError();
    }
    int rc = e == hipSuccess ? AGN_OK : fail(AGN_EHIP, "log_ingest: %s", hipGetErrorString(e));
    const hipError_t ef = hipFreeAsync(scratch, st);
    if (rc == AGN_OK && ef != hipSuccess) rc = fail(AGN_EHIP, "hipFreeAsync: %s", hipGetErrorString(ef));
    return rc;
}

}  // namespace agn
