// bwprobe.hip — measurement infrastructure (not the product): the practical
// HBM read ceiling of the box the bench runs on.  The fastest read idiom
// measured here (scripts/ab_probe.py over tools/bwprobe_ab.hip,
// profiles/r01/ab_read_probe.log): one-shot waves, each streaming 4 KiB with
// four non-temporal LDS-DMA loads (global_load_lds_dwordx4 nt); every byte is
// read once.  bench.py reports the materialize kernel's bytes/s both against
// the 8 TB/s spec peak and against this probe.
//
// agn_probe_copy: the same one-shot 4 KiB waves, non-temporal 16-B loads and
// stores, the first wq of every four 1 KiB chunks stored to dst (wq = 4: a
// copy; wq = 3: the GC kernel's ~0.7 write:read mix) -- the practical ceiling
// for a kernel that reads and writes, reported beside the GC numbers.  The
// fastest of nine read+write idioms (tools/copyprobe_ab.hip,
// profiles/r02/ab_copy.log): 6.18-6.20 TB/s of bytes read + written against
// 5.76-5.84 with plain loads and stores, 5.24-5.48 in place.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(128) void k_read(const u64x2 *__restrict__ p, uint64_t n,
                                             uint64_t *__restrict__ out) {
    __shared__ u64x2 st[2][256];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * 2 + wv;
    if (w * 256 + 255 >= n) return;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_global_load_lds((const void *)(p + w * 256 + j * 64 + lane),
                                         (__attribute__((address_space(3))) void *)&st[wv][j * 64],
                                         16, 0, 2 /* nt */);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    uint64_t acc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const u64x2 x = st[wv][lane * 4 + j];
        acc ^= x.x ^ x.y;
    }
    if (acc == 0x9E3779B97F4A7C15ull) out[0] = acc;  // practically never taken
}

__global__ __launch_bounds__(128) void k_copy(const u64x2 *__restrict__ p, u64x2 *__restrict__ q,
                                             uint64_t n, int wq) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * 2 + wv;
    if (w * 256 + 255 >= n) return;
    u64x2 x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = __builtin_nontemporal_load(p + w * 256 + j * 64 + lane);
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (j < wq) __builtin_nontemporal_store(x[j], q + w * 256 + j * 64 + lane);
}

extern "C" int agn_probe_copy(const void *src, void *dst, uint64_t bytes, int wq, void *stream) {
    const uint64_t n = bytes / 16;
    const uint64_t nb = n / 512;
    if (nb == 0 || nb > 0x7fffffffull || wq < 0 || wq > 4) return -1;
    hipLaunchKernelGGL(k_copy, dim3((unsigned)nb), dim3(128), 0, (hipStream_t)stream,
                       (const u64x2 *)src, (u64x2 *)dst, n, wq);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int agn_probe_read(const void *buf, uint64_t bytes, void *scratch, void *stream) {
    const uint64_t n = bytes / 16;  // whole 8 KiB blocks; the tail (< 8 KiB) is not read
    const uint64_t nb = n / 512;
    if (nb == 0 || nb > 0x7fffffffull) return -1;
    hipLaunchKernelGGL(k_read, dim3((unsigned)nb), dim3(128), 0, (hipStream_t)stream,
                       (const u64x2 *)buf, n, (uint64_t *)scratch);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
