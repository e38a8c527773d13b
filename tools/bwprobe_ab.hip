// bwprobe_ab.hip — measurement infrastructure (not the product): read-path
// variants over one large buffer, to find the fastest HBM streaming idiom for
// the materialize kernels (16-byte VGPR loads, non-temporal loads, one-shot
// waves vs grid-stride, LDS-DMA global_load_lds with default / nt policy).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

// v0: grid-stride, 4 x 16 B in flight per lane (tools/bwprobe.hip)
__global__ __launch_bounds__(256) void k_gs(const u64x2 *__restrict__ p, uint64_t n,
                                           uint64_t *__restrict__ out) {
    uint64_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const u64x2 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
        acc ^= a.x ^ a.y ^ b.x ^ b.y ^ c.x ^ c.y ^ d.x ^ d.y;
    }
    for (; i < n; i += stride) acc ^= p[i].x ^ p[i].y;
    if (acc == 0x9E3779B97F4A7C15ull) out[0] = acc;
}

// v1/v2: one-shot waves: each wave reads one 4 KiB chunk (64 lanes x 4 x 16 B,
// lane-contiguous 64-byte rows like the counter kernel's OpSSCommit rows),
// grid = whole buffer; NT = non-temporal loads
template <bool NT, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_chunk(const u64x2 *__restrict__ p, uint64_t n,
                                                    uint64_t *__restrict__ out) {
    const uint64_t w = (uint64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
    const uint64_t base = w * 256 + (uint64_t)(threadIdx.x & 63) * 4;
    if (base + 3 >= n) return;
    u64x2 a, b, c, d;
    if (NT) {
        a = __builtin_nontemporal_load(p + base);
        b = __builtin_nontemporal_load(p + base + 1);
        c = __builtin_nontemporal_load(p + base + 2);
        d = __builtin_nontemporal_load(p + base + 3);
    } else {
        a = p[base]; b = p[base + 1]; c = p[base + 2]; d = p[base + 3];
    }
    const uint64_t acc = a.x ^ a.y ^ b.x ^ b.y ^ c.x ^ c.y ^ d.x ^ d.y;
    if (acc == 0x9E3779B97F4A7C15ull) out[0] = acc;
}

// v3/v4: one-shot waves through LDS-DMA: 4 x global_load_lds_dwordx4 per wave
// (4 KiB into LDS), then each lane reads its 64-byte row back from LDS.
template <int AUX, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_glds(const u64x2 *__restrict__ p, uint64_t n,
                                                   uint64_t *__restrict__ out) {
    __shared__ u64x2 st[WPB][256];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * WPB + wv;
    if (w * 256 + 255 >= n) return;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_global_load_lds((const void *)(p + w * 256 + j * 64 + lane),
                                         (__attribute__((address_space(3))) void *)&st[wv][j * 64],
                                         16, 0, AUX);
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    uint64_t acc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const u64x2 x = st[wv][lane * 4 + j];
        acc ^= x.x ^ x.y;
    }
    if (acc == 0x9E3779B97F4A7C15ull) out[0] = acc;
}

// v10: one-shot waves, 4 KiB each as 16 x global_load_lds_dword (64 lanes x 4 B,
// 256 contiguous bytes per instruction), nt: FETCH_SIZE calibration of the
// 4-byte LDS-DMA width (the counter kernel's effects and op ids)
__global__ __launch_bounds__(128) void k_glds4(const uint32_t *__restrict__ p, uint64_t n16,
                                              uint64_t *__restrict__ out) {
    __shared__ uint32_t st[2][1024];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * 2 + wv;
    if (w * 256 + 255 >= n16) return;
#pragma unroll
    for (int j = 0; j < 16; ++j)
        __builtin_amdgcn_global_load_lds((const void *)(p + w * 1024 + j * 64 + lane),
                                         (__attribute__((address_space(3))) void *)&st[wv][j * 64],
                                         4, 0, 2);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    uint64_t acc = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc ^= st[wv][lane * 16 + j];
    if (acc == 0x9E3779B97F4A7C15ull) out[0] = acc;
}

// v11/v12: one-shot waves, 4 KiB each, lane-CONTIGUOUS 16-byte loads (load j
// covers bytes [1 KiB j, 1 KiB (j+1)) of the chunk: every instruction reads
// 8 whole 128-byte lines), default / non-temporal policy; one wave per block
// like the counter kernel.  v13: the counter kernel's row-per-lane pattern
// (lane l reads the 64-byte row l: every instruction touches 32 lines,
// 32 bytes of each), one wave per block.
template <bool NT, bool ROWS>
__global__ __launch_bounds__(64) void k_chunk1(const u64x2 *__restrict__ p, uint64_t n,
                                              uint64_t *__restrict__ out) {
    const uint64_t w = blockIdx.x;
    const int lane = threadIdx.x & 63;
    if (w * 256 + 255 >= n) return;
    u64x2 x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const u64x2 *a = p + w * 256 + (ROWS ? (uint64_t)lane * 4 + j : (uint64_t)j * 64 + lane);
        x[j] = NT ? __builtin_nontemporal_load(a) : *a;
    }
    const uint64_t acc = x[0].x ^ x[0].y ^ x[1].x ^ x[1].y ^ x[2].x ^ x[2].y ^ x[3].x ^ x[3].y;
    if (acc == 0x9E3779B97F4A7C15ull) out[0] = acc;
}

// v5: grid-stride with non-temporal loads
__global__ __launch_bounds__(256) void k_gs_nt(const u64x2 *__restrict__ p, uint64_t n,
                                              uint64_t *__restrict__ out) {
    uint64_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const u64x2 a = __builtin_nontemporal_load(p + i),
                    b = __builtin_nontemporal_load(p + i + stride),
                    c = __builtin_nontemporal_load(p + i + 2 * stride),
                    d = __builtin_nontemporal_load(p + i + 3 * stride);
        acc ^= a.x ^ a.y ^ b.x ^ b.y ^ c.x ^ c.y ^ d.x ^ d.y;
    }
    for (; i < n; i += stride) acc ^= p[i].x ^ p[i].y;
    if (acc == 0x9E3779B97F4A7C15ull) out[0] = acc;
}

extern "C" int agn_probe_variant(int v, const void *buf, uint64_t bytes, void *scratch,
                                 void *stream) {
    const uint64_t n = bytes / 16;
    hipStream_t s = (hipStream_t)stream;
    const u64x2 *p = (const u64x2 *)buf;
    uint64_t *o = (uint64_t *)scratch;
    const unsigned nw = (unsigned)(n / 256);
    switch (v) {
        case 0: hipLaunchKernelGGL(k_gs, dim3(256 * 16), dim3(256), 0, s, p, n, o); break;
        case 1: hipLaunchKernelGGL((k_chunk<false, 2>), dim3(nw / 2), dim3(128), 0, s, p, n, o); break;
        case 2: hipLaunchKernelGGL((k_chunk<true, 2>), dim3(nw / 2), dim3(128), 0, s, p, n, o); break;
        case 3: hipLaunchKernelGGL((k_glds<0, 2>), dim3(nw / 2), dim3(128), 0, s, p, n, o); break;
        case 4: hipLaunchKernelGGL((k_glds<2, 2>), dim3(nw / 2), dim3(128), 0, s, p, n, o); break;
        case 5: hipLaunchKernelGGL(k_gs_nt, dim3(256 * 16), dim3(256), 0, s, p, n, o); break;
        case 6: hipLaunchKernelGGL((k_glds<0, 4>), dim3(nw / 4), dim3(256), 0, s, p, n, o); break;
        case 7: hipLaunchKernelGGL((k_chunk<false, 4>), dim3(nw / 4), dim3(256), 0, s, p, n, o); break;
        case 8: hipLaunchKernelGGL((k_glds<1, 2>), dim3(nw / 2), dim3(128), 0, s, p, n, o); break;
        case 9: hipLaunchKernelGGL((k_glds<3, 2>), dim3(nw / 2), dim3(128), 0, s, p, n, o); break;
        case 10: hipLaunchKernelGGL(k_glds4, dim3(nw / 2), dim3(128), 0, s, (const uint32_t *)buf, n, o); break;
        case 11: hipLaunchKernelGGL((k_chunk1<false, false>), dim3(nw), dim3(64), 0, s, p, n, o); break;
        case 12: hipLaunchKernelGGL((k_chunk1<true, false>), dim3(nw), dim3(64), 0, s, p, n, o); break;
        case 13: hipLaunchKernelGGL((k_chunk1<false, true>), dim3(nw), dim3(64), 0, s, p, n, o); break;
        case 14: hipLaunchKernelGGL((k_chunk1<true, true>), dim3(nw), dim3(64), 0, s, p, n, o); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
