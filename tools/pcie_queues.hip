// pcie_queues.hip -- which stream set-ups let H2D and D2H run at once (full duplex) in one process.
//
// tools/pcie_bw.py found the link full-duplex only with ONE stream per direction (97 GB/s both ways;
// two or four streams per direction: 55-80).  With GPU_MAX_HW_QUEUES = 4, HIP deals streams out to
// hardware queues in creation order, so in a process with more streams (sym_ctx slots, the batcher,
// torch) two copy streams may share a queue, or a copy stream a kernel stream.  This measures H2D +
// D2H of `total` bytes each way in `chunk`-byte copies, a kernel stream busy beside them or not, for:
//   plain      two fresh hipStreamNonBlocking streams (after `extra` other streams were created)
//   priority   the two copy streams created with the highest priority
//   cumask     the two copy streams created with hipExtStreamCreateWithCUMask (all CUs)
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/pcie_queues tools/pcie_queues.hip && tools/pcie_queues
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__global__ void spin_kernel(unsigned long long ticks) {  // keeps a kernel stream busy (bounded)
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const size_t total = (size_t)(argc > 1 ? atoi(argv[1]) : 1024) << 20;
    const size_t chunk = (size_t)8 << 20;
    void *h_in, *h_out, *d_in, *d_out;
    CK(hipHostMalloc(&h_in, total, hipHostMallocDefault));
    CK(hipHostMalloc(&h_out, total, hipHostMallocDefault));
    CK(hipMalloc(&d_in, total));
    CK(hipMalloc(&d_out, total));
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    for (int mode = 0; mode < 3; ++mode) {
        for (int extra : {0, 5}) {
            for (int busy : {0, 1}) {
                std::vector<hipStream_t> others(extra);
                for (auto& s : others) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
                hipStream_t a, b, k;
                CK(hipStreamCreateWithFlags(&k, hipStreamNonBlocking));
                if (mode == 0) {
                    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
                    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
                } else if (mode == 1) {
                    CK(hipStreamCreateWithPriority(&a, hipStreamNonBlocking, hi));
                    CK(hipStreamCreateWithPriority(&b, hipStreamNonBlocking, hi));
                } else {
                    uint32_t mask[8];
                    for (auto& m : mask) m = ~0u;
                    CK(hipExtStreamCreateWithCUMask(&a, 8, mask));
                    CK(hipExtStreamCreateWithCUMask(&b, 8, mask));
                }
                double best = 0;
                for (int rep = 0; rep < 3; ++rep) {
                    CK(hipDeviceSynchronize());
                    if (busy) hipLaunchKernelGGL(spin_kernel, dim3(8), dim3(64), 0, k, 3000000ull);  // 30 ms
                    const double t0 = now();
                    for (size_t o = 0; o < total; o += chunk) {
                        CK(hipMemcpyAsync((char*)d_in + o, (char*)h_in + o, chunk, hipMemcpyHostToDevice, a));
                        CK(hipMemcpyAsync((char*)h_out + o, (char*)d_out + o, chunk, hipMemcpyDeviceToHost, b));
                    }
                    CK(hipStreamSynchronize(a));
                    CK(hipStreamSynchronize(b));
                    const double dt = now() - t0;
                    CK(hipStreamSynchronize(k));
                    best = std::max(best, 2.0 * total / dt / 1e9);
                }
                printf("{\"mode\": \"%s\", \"other_streams\": %d, \"kernel_busy\": %d, \"both_gbps\": %.1f}\n",
                       mode == 0 ? "plain" : (mode == 1 ? "priority" : "cumask"), extra, busy, best);
                fflush(stdout);
                CK(hipStreamDestroy(a));
                CK(hipStreamDestroy(b));
                CK(hipStreamDestroy(k));
                for (auto& s : others) CK(hipStreamDestroy(s));
            }
        }
    }
    return 0;
}
