// calib_traffic.hip -- what rocprofv3's FETCH_SIZE / WRITE_SIZE report per access width on gfx950,
// on known byte counts (MI355X_MICROARCH.md: "FETCH_SIZE reports exactly half of the bytes of a
// wide coalesced streaming read ... Other access widths are uncalibrated: calibrate on a known byte
// count in your own access pattern").  Each kernel below is one access pattern of the decode
// (decode_pipe.hip) in isolation, over buffers larger than the 256 MiB Infinity Cache where the
// pattern allows:
//   stream16   16 B per lane, coalesced, over 1 GiB                 (the copiers' stream reads)
//   off8       rec_off[i] and rec_off[i+1], 8 B per lane, 2^20+1     (the parsers' record offsets)
//   k0_4       one 4-byte load at record i's byte 22, 2^20 records   (the speculative parser's key
//              of 350 bytes (a 367 MB stream), half of them unaligned  length)
//   parser     off8 and k0_4 together, as parse_tiles_spec does them
//   store16    16 B per lane, coalesced, 256 MiB                      (the copiers' column writes)
//   store8     8 B per lane, 2^20+1                                   (the column offsets)
//   store1     1 B per lane, 2^20                                      (the status bytes)
// Run under rocprofv3 --pmc FETCH_SIZE (one pass) and --pmc WRITE_SIZE (another); each kernel runs
// `reps` times.  Prints each kernel's bytes and its time (HIP events).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

typedef uint32_t __attribute__((aligned(1))) u32u;

__global__ __launch_bounds__(256) void stream16(const uint4* __restrict__ p, uint64_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;  // (never: keeps the loads)
}

__global__ __launch_bounds__(256) void off8(const uint64_t* __restrict__ off, uint64_t n, uint32_t* sink) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t L = off[i + 1] - off[i];
    if (L == 0x12345) sink[threadIdx.x] = (uint32_t)L;
}

__global__ __launch_bounds__(256) void k0_4(const uint8_t* __restrict__ in, uint64_t n, uint32_t* sink) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = *(const u32u*)(in + 350 * i + 22);
    if (k == 0x12345u) sink[threadIdx.x] = k;
}

// the same 4-byte loads with other cache policies (gfx950 sc0 / sc1 / nt bits), aligned to 4 here
__global__ __launch_bounds__(256) void k0_nt(const uint8_t* __restrict__ in, uint64_t n, uint32_t* sink) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = __builtin_nontemporal_load((const uint32_t*)(in + 352 * i + 24));
    if (k == 0x12345u) sink[threadIdx.x] = k;
}
__global__ __launch_bounds__(256) void k0_sc1(const uint8_t* __restrict__ in, uint64_t n, uint32_t* sink) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = __hip_atomic_load((const uint32_t*)(in + 352 * i + 24), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == 0x12345u) sink[threadIdx.x] = k;
}
__global__ __launch_bounds__(256) void k0_sys(const uint8_t* __restrict__ in, uint64_t n, uint32_t* sink) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = __hip_atomic_load((const uint32_t*)(in + 352 * i + 24), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (k == 0x12345u) sink[threadIdx.x] = k;
}
__global__ __launch_bounds__(256) void k0_ntsc(const uint8_t* __restrict__ in, uint64_t n, uint32_t* sink) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t k;
    asm volatile("global_load_dword %0, %1, off sc0 sc1 nt\n s_waitcnt vmcnt(0)" : "=v"(k) : "v"(in + 352 * i + 24) : "memory");
    if (k == 0x12345u) sink[threadIdx.x] = k;
}
__global__ __launch_bounds__(256) void k0_a4(const uint8_t* __restrict__ in, uint64_t n, uint32_t* sink) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = *(const uint32_t*)(in + 352 * i + 24);
    if (k == 0x12345u) sink[threadIdx.x] = k;
}

__global__ __launch_bounds__(256) void parser(const uint8_t* __restrict__ in, const uint64_t* __restrict__ off,
                                               uint64_t n, uint32_t* sink) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t st = off[i], L = off[i + 1] - st;
    const uint32_t k = *(const u32u*)(in + st + 22);
    if (k + L == 0x12345u) sink[threadIdx.x] = k;
}

__global__ __launch_bounds__(256) void store16(uint4* __restrict__ p, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
        p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

__global__ __launch_bounds__(256) void store8(uint64_t* __restrict__ p, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = 350 * i;
}

__global__ __launch_bounds__(256) void store1(uint8_t* __restrict__ p, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = (uint8_t)i;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 3;
    const uint64_t big = 1ull << 30, n = 1ull << 20, rec = 350;
    uint8_t *a, *s;
    uint64_t* off;
    uint32_t* sink;
    CK(hipMalloc(&a, big));
    CK(hipMalloc(&s, 352 * n + 64));
    CK(hipMalloc(&off, 8 * (n + 1)));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(a, 1, big));
    CK(hipMemset(s, 2, 352 * n + 64));
    store8<<<(n + 1 + 255) / 256, 256>>>(off, n + 1);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned g = (unsigned)((n + 255) / 256);
    struct K {
        const char* name;
        double bytes;  // the bytes the pattern names (stream: the whole buffer; scattered: 4 B each)
        int which;
    } ks[] = {{"stream16", (double)big, 0}, {"off8", 8.0 * (n + 1), 1}, {"k0_4", 4.0 * n, 2},
              {"parser", 8.0 * (n + 1) + 4.0 * n, 3}, {"store16", (double)(256ull << 20), 4},
              {"store8", 8.0 * (n + 1), 5}, {"store1", (double)n, 6}, {"k0_a4", 4.0 * n, 7}, {"k0_nt", 4.0 * n, 8},
              {"k0_sc1", 4.0 * n, 9}, {"k0_sys", 4.0 * n, 10}, {"k0_ntsc", 4.0 * n, 11}};
    for (const K& k : ks) {
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CK(hipMemset(a + (256ull << 20), r, 64ull << 20));  // evict: 64 MiB written between reps
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            switch (k.which) {
                case 0: stream16<<<4096, 256>>>((const uint4*)a, big / 16, sink); break;
                case 1: off8<<<g, 256>>>(off, n, sink); break;
                case 2: k0_4<<<g, 256>>>(s, n, sink); break;
                case 3: parser<<<g, 256>>>(s, off, n, sink); break;
                case 4: store16<<<4096, 256>>>((uint4*)a, (256ull << 20) / 16); break;
                case 5: store8<<<(n + 1 + 255) / 256, 256>>>(off, n + 1); break;
                case 6: store1<<<g, 256>>>(s, n); break;
                case 7: k0_a4<<<g, 256>>>(s, n, sink); break;
                case 8: k0_nt<<<g, 256>>>(s, n, sink); break;
                case 9: k0_sc1<<<g, 256>>>(s, n, sink); break;
                case 10: k0_sys<<<g, 256>>>(s, n, sink); break;
                case 11: k0_ntsc<<<g, 256>>>(s, n, sink); break;
            }
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        printf("%-9s pattern_bytes %.0f best_us %.2f\n", k.name, k.bytes, best * 1e3);
    }
    return 0;
}
