// copyprobe_ab.hip — measurement infrastructure (not the product): which
// read+write streaming idiom moves HBM bytes fastest on this box, i.e. the
// practical ceiling of a kernel that reads X and writes a fraction of X (the
// GC kernels).  Every variant reads n 16-byte units and stores the first wq
// of every four 1 KiB quarters (wq = 4: a copy, wq = 3: the GC's write mix).
// scripts/ab_copy.py interleaves the variants in one process.
//   0  one-shot wave, 4 KiB, 16-B loads/stores           (bwprobe.hip k_copy)
//   1  as 0, non-temporal loads and stores
//   2  as 0, non-temporal stores only
//   3  one-shot wave, 4 KiB, LDS-DMA nt loads, stores from LDS
//   4  one-shot wave, 8 KiB (8 loads in flight per lane)
//   5  grid-stride, 2048 x 256 threads, 4 x 16 B per lane per step
//   6  one-shot, 4 waves per block (256 threads), 4 KiB per wave
//   7  as 0 but in place (dst == src), the op-log GC's pattern
//   8  as 3 but in place
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void *lds_ptr;

template <bool NTL, bool NTS>
__global__ __launch_bounds__(128) void k_oneshot(const u64x2 *p, u64x2 *q, uint64_t n, int wq) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * 2 + wv;
    if (w * 256 + 255 >= n) return;
    u64x2 x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const u64x2 *a = p + w * 256 + j * 64 + lane;
        x[j] = NTL ? __builtin_nontemporal_load(a) : *a;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (j < wq) {
            u64x2 *a = q + w * 256 + j * 64 + lane;
            if (NTS) __builtin_nontemporal_store(x[j], a);
            else *a = x[j];
        }
}

__global__ __launch_bounds__(128) void k_glds(const u64x2 *p, u64x2 *q, uint64_t n, int wq) {
    __shared__ u64x2 st[2][256];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * 2 + wv;
    if (w * 256 + 255 >= n) return;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_global_load_lds((const void *)(p + w * 256 + j * 64 + lane),
                                         (lds_ptr)&st[wv][j * 64], 16, 0, 2 /* nt */);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (j < wq) q[w * 256 + j * 64 + lane] = st[wv][j * 64 + lane];
}

__global__ __launch_bounds__(64) void k_oneshot8(const u64x2 *p, u64x2 *q, uint64_t n, int wq) {
    const int lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x;
    if (w * 512 + 511 >= n) return;
    u64x2 x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = p[w * 512 + j * 64 + lane];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if ((j & 3) < wq) q[w * 512 + j * 64 + lane] = x[j];
}

__global__ __launch_bounds__(256) void k_gs(const u64x2 *p, u64x2 *q, uint64_t n, int wq) {
    const uint64_t nthr = (uint64_t)gridDim.x * 256u;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t w0 = (uint64_t)blockIdx.x * 4 + wv, nw = nthr / 64;
    for (uint64_t w = w0; w * 256 + 255 < n; w += nw) {
        u64x2 x[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = p[w * 256 + j * 64 + lane];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (j < wq) q[w * 256 + j * 64 + lane] = x[j];
    }
}

__global__ __launch_bounds__(256) void k_oneshot_wpb4(const u64x2 *p, u64x2 *q, uint64_t n, int wq) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + wv;
    if (w * 256 + 255 >= n) return;
    u64x2 x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = p[w * 256 + j * 64 + lane];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (j < wq) q[w * 256 + j * 64 + lane] = x[j];
}

extern "C" int agn_copy_variant(int v, const void *src, void *dst, uint64_t bytes, int wq,
                                void *stream) {
    const uint64_t n = bytes / 16;
    hipStream_t st = (hipStream_t)stream;
    const u64x2 *p = (const u64x2 *)src;
    u64x2 *q = (u64x2 *)dst;
    if (v == 7 || v == 8) q = (u64x2 *)src;
    if (n / 512 == 0 || n / 512 > 0x7fffffffull || wq < 0 || wq > 4) return -1;
    const unsigned nb2 = (unsigned)(n / 512);  // 2 waves x 4 KiB per block
    switch (v) {
        case 0: case 7: hipLaunchKernelGGL((k_oneshot<false, false>), dim3(nb2), dim3(128), 0, st, p, q, n, wq); break;
        case 1: hipLaunchKernelGGL((k_oneshot<true, true>), dim3(nb2), dim3(128), 0, st, p, q, n, wq); break;
        case 2: hipLaunchKernelGGL((k_oneshot<false, true>), dim3(nb2), dim3(128), 0, st, p, q, n, wq); break;
        case 3: case 8: hipLaunchKernelGGL(k_glds, dim3(nb2), dim3(128), 0, st, p, q, n, wq); break;
        case 4: hipLaunchKernelGGL(k_oneshot8, dim3(nb2), dim3(64), 0, st, p, q, n, wq); break;
        case 5: hipLaunchKernelGGL(k_gs, dim3(2048), dim3(256), 0, st, p, q, n, wq); break;
        case 6: hipLaunchKernelGGL(k_oneshot_wpb4, dim3(nb2 / 2), dim3(256), 0, st, p, q, n, wq); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
