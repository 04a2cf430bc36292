// Microbenchmark: what a 350 MB stream copy achieves on MI355X in the shapes the codec uses.
//   0: grid-stride aligned 16 B/lane copy (the roofline reference)
//   1: one 22,400-byte tile per wave, 1 KiB per step (encode's shape), aligned
//   2: as 1, source byte-unaligned (+3)
//   3: as 2, nontemporal stores
//   4: as 2, nontemporal loads and stores
//   5: as 2, two steps per round (loads of both issued before either store)
//   6: as 1, 2 tiles per wave (half the waves)
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_copy.hip -o tools/ubench_copy
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gc_u4;
typedef __attribute__((address_space(1))) u32x4 g_u4;

#define CHECK(x)                                                              \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__);        \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

constexpr size_t kTile = 22400;

__global__ __launch_bounds__(256) void grid_copy(const unsigned char* src, unsigned char* dst, size_t nchunks) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t c = (size_t)blockIdx.x * 256 + threadIdx.x; c < nchunks; c += stride)
        *(g_u4*)(dst + 16 * c) = *(gc_u4*)(src + 16 * c);
}

template <int V>
__global__ __launch_bounds__(256) void tile_copy(const unsigned char* src, unsigned char* dst, size_t ntiles,
                                                 u32 shift) {
    const int lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    constexpr int kPer = V == 6 ? 2 : 1;
    for (int h = 0; h < kPer; ++h) {
        const size_t t = wave * kPer + h;
        if (t >= ntiles) return;
        const unsigned char* s = src + t * kTile + shift;
        unsigned char* d = dst + t * kTile;
        if constexpr (V == 5) {
            for (int B = 0; B < (int)kTile; B += 2048) {
                const int P0 = B + 16 * lane, P1 = P0 + 1024;
                const u32x4 a = *(gc_u4*)(s + (P0 < (int)kTile ? P0 : 0));
                const u32x4 b = *(gc_u4*)(s + (P1 < (int)kTile ? P1 : 0));
                if (P0 + 16 <= (int)kTile) *(g_u4*)(d + P0) = a;
                if (P1 + 16 <= (int)kTile) *(g_u4*)(d + P1) = b;
            }
        } else {
            for (int B = 0; B < (int)kTile; B += 1024) {
                const int P = B + 16 * lane;
                if (P + 16 > (int)kTile) break;
                u32x4 v;
                if constexpr (V == 4) v = __builtin_nontemporal_load((gc_u4*)(s + P));
                else v = *(gc_u4*)(s + P);
                if constexpr (V == 3 || V == 4) __builtin_nontemporal_store(v, (g_u4*)(d + P));
                else *(g_u4*)(d + P) = v;
            }
        }
    }
}

int main() {
    const size_t ntiles = 16384;  // 2^20 records of 350 B
    const size_t bytes = ntiles * kTile;
    const int nsets = 4;
    unsigned char *src[nsets], *dst[nsets];
    for (int k = 0; k < nsets; ++k) {
        CHECK(hipMalloc(&src[k], bytes + 64));
        CHECK(hipMalloc(&dst[k], bytes + 64));
        CHECK(hipMemset(src[k], k + 1, bytes + 64));
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const char* names[] = {"grid-stride aligned", "tile/wave aligned", "tile/wave src+3", "tile/wave src+3 nt-store",
                           "tile/wave src+3 nt-ld+st", "tile/wave src+3 2 steps/round", "2 tiles/wave aligned"};
    for (int V = 0; V < 7; ++V) {
        auto launch = [&](int k) {
            const dim3 tgrid((unsigned)((ntiles + 3) / 4)), block(256);
            switch (V) {
                case 0: hipLaunchKernelGGL(grid_copy, dim3(256 * 8), block, 0, 0, src[k], dst[k], bytes / 16); break;
                case 1: hipLaunchKernelGGL(tile_copy<1>, tgrid, block, 0, 0, src[k], dst[k], ntiles, 0u); break;
                case 2: hipLaunchKernelGGL(tile_copy<2>, tgrid, block, 0, 0, src[k], dst[k], ntiles, 3u); break;
                case 3: hipLaunchKernelGGL(tile_copy<3>, tgrid, block, 0, 0, src[k], dst[k], ntiles, 3u); break;
                case 4: hipLaunchKernelGGL(tile_copy<4>, tgrid, block, 0, 0, src[k], dst[k], ntiles, 3u); break;
                case 5: hipLaunchKernelGGL(tile_copy<5>, tgrid, block, 0, 0, src[k], dst[k], ntiles, 3u); break;
                case 6:
                    hipLaunchKernelGGL(tile_copy<6>, dim3((unsigned)((ntiles / 2 + 3) / 4)), block, 0, 0, src[k], dst[k],
                                       ntiles, 0u);
                    break;
            }
        };
        for (int k = 0; k < nsets; ++k) launch(k);
        CHECK(hipDeviceSynchronize());
        float tot = 0, best = 1e9f;
        const int reps = 20;
        for (int r = 0; r < reps; ++r) {
            CHECK(hipEventRecord(e0));
            launch(r % nsets);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            tot += ms;
            if (ms < best) best = ms;
        }
        printf("%-32s avg %7.1f us  %6.0f GB/s   best %7.1f us  %6.0f GB/s (read+write)\n", names[V],
               tot / reps * 1e3, 2.0 * bytes / (tot / reps * 1e-3) / 1e9, best * 1e3, 2.0 * bytes / (best * 1e-3) / 1e9);
    }
    return 0;
}
