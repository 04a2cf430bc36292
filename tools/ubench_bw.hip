// Microbenchmark: the HBM ceilings a byte-shuffle kernel works against on MI355X.
// Read-only, write-only and copy streams at the codec's working-set size (350 MB per buffer, four
// rotating sets so no launch finds its data in the 256 MiB Infinity Cache) and at 2 GiB, in the
// shapes that matter: grid-stride with U 16-byte loads in flight per lane, one chunk per thread on
// a grid as large as the data, non-temporal stores.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_bw.hip -o tools/ubench_bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gc_u4;
typedef __attribute__((address_space(1))) u32x4 g_u4;

#define CHECK(x)                                                          \
    do {                                                                  \
        hipError_t e = (x);                                               \
        if (e != hipSuccess) {                                            \
            printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__);    \
            exit(1);                                                      \
        }                                                                 \
    } while (0)

template <int U>
__global__ __launch_bounds__(256) void read_k(const unsigned char* src, u32* sink, size_t nchunks) {
    const size_t stride = (size_t)gridDim.x * 256;
    u32x4 acc = {0, 0, 0, 0};
    size_t c = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; c + (U - 1) * stride < nchunks; c += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = *(gc_u4*)(src + 16 * (c + u * stride));
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u];
    }
    for (; c < nchunks; c += stride) acc ^= *(gc_u4*)(src + 16 * c);
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;  // keeps the loads
}

template <int NT>
__global__ __launch_bounds__(256) void write_k(unsigned char* dst, size_t nchunks) {
    const size_t stride = (size_t)gridDim.x * 256;
    const u32x4 v = {1, 2, 3, 4};
    for (size_t c = (size_t)blockIdx.x * 256 + threadIdx.x; c < nchunks; c += stride) {
        if constexpr (NT) __builtin_nontemporal_store(v, (g_u4*)(dst + 16 * c));
        else *(g_u4*)(dst + 16 * c) = v;
    }
}

template <int U, int NT>
__global__ __launch_bounds__(256) void copy_k(const unsigned char* src, unsigned char* dst, size_t nchunks) {
    const size_t stride = (size_t)gridDim.x * 256;
    size_t c = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; c + (U - 1) * stride < nchunks; c += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = *(gc_u4*)(src + 16 * (c + u * stride));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (NT) __builtin_nontemporal_store(v[u], (g_u4*)(dst + 16 * (c + u * stride)));
            else *(g_u4*)(dst + 16 * (c + u * stride)) = v[u];
        }
    }
    for (; c < nchunks; c += stride) *(g_u4*)(dst + 16 * c) = *(gc_u4*)(src + 16 * c);
}

// each workgroup copies K consecutive 4 KiB blocks (its own contiguous K*4 KiB span), one per step
template <int K>
__global__ __launch_bounds__(256) void copy_blocks_k(const unsigned char* src, unsigned char* dst, size_t nchunks) {
    const size_t c0 = (size_t)blockIdx.x * 256 * K + threadIdx.x;
#pragma unroll 1
    for (int k = 0; k < K; ++k) {
        const size_t c = c0 + (size_t)k * 256;
        if (c < nchunks) *(g_u4*)(dst + 16 * c) = *(gc_u4*)(src + 16 * c);
    }
}

int main() {
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    u32* sink;
    CHECK(hipMalloc(&sink, 64));
    const size_t sizes[3] = {(size_t)350 << 20, (size_t)700 << 20, (size_t)2800 << 20};
    for (size_t bytes : sizes) {
        const int nsets = bytes < ((size_t)1 << 30) ? 4 : 1;
        unsigned char *src[4], *dst[4];
        for (int k = 0; k < nsets; ++k) {
            CHECK(hipMalloc(&src[k], bytes));
            CHECK(hipMalloc(&dst[k], bytes));
            CHECK(hipMemset(src[k], k + 1, bytes));
            CHECK(hipMemset(dst[k], 0, bytes));
        }
        const size_t nch = bytes / 16;
        const unsigned full = (unsigned)((nch + 255) / 256);  // one chunk per thread
        struct Case {
            const char* name;
            int kind;  // 0 read, 1 write, 2 copy
            double mult;
            unsigned grid;
        };
        const Case cases[] = {
            {"read   grid-stride x1, 8 WG/CU", 0, 1, (unsigned)ncu * 8},
            {"read   grid-stride x4, 8 WG/CU", 0, 1, (unsigned)ncu * 8},
            {"read   one chunk per thread", 0, 1, full},
            {"write  grid-stride, 8 WG/CU", 1, 1, (unsigned)ncu * 8},
            {"write  grid-stride nt, 8 WG/CU", 1, 1, (unsigned)ncu * 8},
            {"write  one chunk per thread", 1, 1, full},
            {"copy   grid-stride x1, 8 WG/CU", 2, 2, (unsigned)ncu * 8},
            {"copy   grid-stride x4, 8 WG/CU", 2, 2, (unsigned)ncu * 8},
            {"copy   grid-stride x4 nt, 8 WG/CU", 2, 2, (unsigned)ncu * 8},
            {"copy   grid-stride x4, 32 WG/CU", 2, 2, (unsigned)ncu * 32},
            {"copy   one chunk per thread", 2, 2, full},
            {"copy   4 KiB x4 per WG", 2, 2, (full + 3) / 4},
            {"copy   4 KiB x16 per WG", 2, 2, (full + 15) / 16},
            {"copy   4 KiB x64 per WG", 2, 2, (full + 63) / 64},
        };
        printf("--- %zu MiB per buffer, %d rotating set(s)\n", bytes >> 20, nsets);
        for (int ci = 0; ci < (int)(sizeof(cases) / sizeof(cases[0])); ++ci) {
            const Case& cs = cases[ci];
            auto launch = [&](int k) {
                const dim3 g(cs.grid), b(256);
                switch (ci) {
                    case 0: hipLaunchKernelGGL(read_k<1>, g, b, 0, 0, src[k], sink, nch); break;
                    case 1: hipLaunchKernelGGL(read_k<4>, g, b, 0, 0, src[k], sink, nch); break;
                    case 2: hipLaunchKernelGGL(read_k<1>, g, b, 0, 0, src[k], sink, nch); break;
                    case 3: hipLaunchKernelGGL(write_k<0>, g, b, 0, 0, dst[k], nch); break;
                    case 4: hipLaunchKernelGGL(write_k<1>, g, b, 0, 0, dst[k], nch); break;
                    case 5: hipLaunchKernelGGL(write_k<0>, g, b, 0, 0, dst[k], nch); break;
                    case 6: hipLaunchKernelGGL((copy_k<1, 0>), g, b, 0, 0, src[k], dst[k], nch); break;
                    case 7: hipLaunchKernelGGL((copy_k<4, 0>), g, b, 0, 0, src[k], dst[k], nch); break;
                    case 8: hipLaunchKernelGGL((copy_k<4, 1>), g, b, 0, 0, src[k], dst[k], nch); break;
                    case 9: hipLaunchKernelGGL((copy_k<4, 0>), g, b, 0, 0, src[k], dst[k], nch); break;
                    case 10: hipLaunchKernelGGL((copy_k<1, 0>), g, b, 0, 0, src[k], dst[k], nch); break;
                    case 11: hipLaunchKernelGGL((copy_blocks_k<4>), g, b, 0, 0, src[k], dst[k], nch); break;
                    case 12: hipLaunchKernelGGL((copy_blocks_k<16>), g, b, 0, 0, src[k], dst[k], nch); break;
                    case 13: hipLaunchKernelGGL((copy_blocks_k<64>), g, b, 0, 0, src[k], dst[k], nch); break;
                }
            };
            for (int k = 0; k < nsets; ++k) launch(k);
            CHECK(hipDeviceSynchronize());
            const int reps = 20;
            float tot = 0, best = 1e9f;
            for (int r = 0; r < reps; ++r) {
                CHECK(hipEventRecord(e0));
                launch(r % nsets);
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                tot += ms;
                best = ms < best ? ms : best;
            }
            const double moved = cs.mult * (double)bytes;
            printf("%-36s avg %8.1f us %6.0f GB/s   best %8.1f us %6.0f GB/s\n", cs.name, tot / reps * 1e3,
                   moved / (tot / reps * 1e-3) / 1e9, best * 1e3, moved / (best * 1e-3) / 1e9);
        }
        for (int k = 0; k < nsets; ++k) {
            CHECK(hipFree(src[k]));
            CHECK(hipFree(dst[k]));
        }
    }
    return 0;
}
