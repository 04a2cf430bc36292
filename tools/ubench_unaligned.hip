// Microbenchmark: byte-unaligned 16-byte loads on gfx950 (correctness + copy bandwidth).
//   variant 0: aligned load + aligned store (baseline copy)
//   variant 1: unaligned global_load_dwordx4 at src+s, aligned store
//   variant 2: two aligned loads + funnel shift (what the codec does), aligned store
//   variant 3: unaligned ds_read_b128 from an LDS staging buffer
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_unaligned.hip -o /tmp/ub
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef unsigned int u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gc_u4;
typedef __attribute__((address_space(1))) u32x4 g_u4;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ u32 alignbyte(u32 hi, u32 lo, u32 sh) { return __builtin_amdgcn_alignbyte(hi, lo, sh); }

__device__ __forceinline__ u32x4 funnel(u32x4 a, u32x4 b, u32 s) {
    const u32 d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const u32 m2 = (s & 8) ? ~0u : 0u, m1 = (s & 4) ? ~0u : 0u;
    u32 e[6], f[5];
#pragma unroll
    for (int k = 0; k < 6; ++k) e[k] = (d[k + 2] & m2) | (d[k] & ~m2);
#pragma unroll
    for (int k = 0; k < 5; ++k) f[k] = (e[k + 1] & m1) | (e[k] & ~m1);
    const u32 sh = s & 3;
    return u32x4{alignbyte(f[1], f[0], sh), alignbyte(f[2], f[1], sh), alignbyte(f[3], f[2], sh), alignbyte(f[4], f[3], sh)};
}

template <int V>
__global__ __launch_bounds__(256) void copy_kernel(const unsigned char* src, unsigned char* dst, size_t nchunks, u32 s) {
    __shared__ u32x4 lds[256 * 2 + 1];
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t c = (size_t)blockIdx.x * 256 + threadIdx.x; c < nchunks; c += stride) {
        u32x4 v;
        if constexpr (V == 0) {
            v = *(gc_u4*)(src + 16 * c);
        } else if constexpr (V == 1) {
            v = *(gc_u4*)(src + 16 * c + s);
        } else if constexpr (V == 2) {
            const unsigned char* X = src + 16 * c + s;
            const uintptr_t B0 = (uintptr_t)X & ~(uintptr_t)15;
            u32x4 a = *(gc_u4*)B0, b = {0, 0, 0, 0};
            if ((uintptr_t)X & 15) b = *(gc_u4*)(B0 + 16);
            v = funnel(a, b, (u32)((uintptr_t)X & 15));
        } else {
            // stage 2 aligned blocks per lane then read unaligned from LDS
            lds[threadIdx.x] = *(gc_u4*)(src + 16 * c);
            __syncthreads();
            const unsigned char* l = (const unsigned char*)lds + 16 * threadIdx.x + s;
            v = *(const u32x4*)l;
            __syncthreads();
        }
        *(g_u4*)(dst + 16 * c) = v;
    }
}

int main() {
    const size_t bytes = (size_t)1 << 30;  // 1 GiB
    const size_t nchunks = bytes / 16 - 2;
    unsigned char *src, *dst;
    CHECK(hipMalloc(&src, bytes + 64));
    CHECK(hipMalloc(&dst, bytes + 64));
    std::vector<unsigned char> h(bytes + 64);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (unsigned char)(i * 2654435761u >> 13);
    CHECK(hipMemcpy(src, h.data(), h.size(), hipMemcpyHostToDevice));
    std::vector<unsigned char> out(4096);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const dim3 grid(256 * 8), block(256);
    for (int V = 0; V < 4; ++V) {
        for (u32 s : {0u, 1u, 3u, 4u, 7u, 8u, 13u}) {
            if (V == 0 && s) continue;
            if (V == 3 && s > 0) {}  // LDS variant reads past lane's block into neighbour: fine for s < 16
            auto launch = [&]() {
                if (V == 0) hipLaunchKernelGGL(copy_kernel<0>, grid, block, 0, 0, src, dst, nchunks, s);
                if (V == 1) hipLaunchKernelGGL(copy_kernel<1>, grid, block, 0, 0, src, dst, nchunks, s);
                if (V == 2) hipLaunchKernelGGL(copy_kernel<2>, grid, block, 0, 0, src, dst, nchunks, s);
                if (V == 3) hipLaunchKernelGGL(copy_kernel<3>, grid, block, 0, 0, src, dst, nchunks, s);
            };
            launch();
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(out.data(), dst, out.size(), hipMemcpyDeviceToHost));
            bool ok = true;
            for (size_t i = 0; i < out.size(); ++i) {
                // LDS variant: lane's neighbour block only within a workgroup; check first 16 chunks only
                const unsigned char want = h[i + s];
                if (V == 3 && (i % 4096) >= 255 * 16) continue;
                if (out[i] != want) { ok = false; break; }
            }
            float best = 1e9f;
            for (int rep = 0; rep < 10; ++rep) {
                CHECK(hipEventRecord(e0));
                launch();
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            printf("variant %d shift %2u: %s  %.3f ms  %.0f GB/s (read+write)\n", V, s, ok ? "correct" : "WRONG", best,
                   2.0 * nchunks * 16 / (best * 1e-3) / 1e9);
        }
    }
    return 0;
}
