// pcie_pattern.hip -- which part of the host entry points' copy pattern (arpc_amd/csrc/host.cpp) keeps
// H2D and D2H from overlapping.  Each mode moves `total` bytes each way in 8 MB chunks over one stream
// per direction (A: H2D, B: D2H), adding one ingredient of host.cpp at a time:
//   0 plain        no dependencies (tools/pcie_queues: ~92 GB/s both ways)
//   1 events       B's D2H of chunk c waits (hipStreamWaitEvent) for an event A records after H2D(c)
//   2 kernel       + a small kernel on A after H2D(c); the event is recorded after it
//   3 split        + each chunk's H2D as 1 large + 3 small (64 KB) copies, its D2H as 1 large + 1 small
//   4 reuse        + 3 device slots: A waits for the D2H event of chunk c-3 before reusing the slot
//   5 host-wait    like 4, but the host waits (hipEventSynchronize) for chunk c-3's D2H instead
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/pcie_pattern tools/pcie_pattern.hip && tools/pcie_pattern
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

__global__ void touch_kernel(unsigned* p) {  // a small kernel (one wave), standing in for the codec
    if (threadIdx.x == 0) p[blockIdx.x] += 1;
}

// copies as kernels: 16-byte loads and stores, grid-stride (host memory is mapped: hipHostMalloc)
__global__ __launch_bounds__(256) void copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const size_t total = (size_t)(argc > 1 ? atoi(argv[1]) : 1024) << 20;
    const size_t chunk = (size_t)8 << 20, small = 64 << 10;
    const int kSlots = 3;
    char *h_in, *h_out, *d_in_all, *d_out_all;
    unsigned* d_k;
    CK(hipHostMalloc((void**)&h_in, total, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&h_out, total, hipHostMallocDefault));
    CK(hipMalloc((void**)&d_in_all, total));
    CK(hipMalloc((void**)&d_out_all, total));
    CK(hipMalloc((void**)&d_k, 4096));
    const char* names[] = {"plain", "events", "kernel", "split", "reuse", "host-wait"};
    // extra: streams created before the two copy streams; distinct: chunk c at device offset c * chunk
    // (as tools/pcie_queues) instead of one of 3 rotating slot buffers
    // two sweeps: a slow first sweep with a fast second one means warm-up, not the stream set-up
    for (int sweep = 0; sweep < 2; ++sweep)
    for (int extra : {0, 1, 3}) {
        for (int distinct : {1, 0}) {
            std::vector<hipStream_t> others(extra);
            for (auto& s : others) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            hipStream_t a, b;
            CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
            CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
            hipEvent_t ev_in[kSlots], ev_done[kSlots];
            for (int k = 0; k < kSlots; ++k) {
                CK(hipEventCreateWithFlags(&ev_in[k], hipEventDisableTiming));
                CK(hipEventCreateWithFlags(&ev_done[k], hipEventDisableTiming));
            }
            for (int mode = 0; mode < 6; ++mode) {
                double best = 0;
                for (int rep = 0; rep < 3; ++rep) {
                    CK(hipDeviceSynchronize());
                    const double t0 = now();
                    const size_t C = total / chunk;
                    for (size_t c = 0; c < C; ++c) {
                        const int k = (int)(c % kSlots);
                        const size_t o = c * chunk;
                        char* din = d_in_all + (distinct ? o : k * chunk);
                        char* dout = d_out_all + (distinct ? o : k * chunk);
                        if (mode == 4 && c >= (size_t)kSlots) CK(hipStreamWaitEvent(a, ev_done[k], 0));
                        if (mode == 5 && c >= (size_t)kSlots) CK(hipEventSynchronize(ev_done[k]));
                        if (mode >= 3) {
                            CK(hipMemcpyAsync(din, h_in + o, chunk - 3 * small, hipMemcpyHostToDevice, a));
                            for (int s = 0; s < 3; ++s)
                                CK(hipMemcpyAsync(din + chunk - (s + 1) * small, h_in + o + chunk - (s + 1) * small, small,
                                                  hipMemcpyHostToDevice, a));
                        } else {
                            CK(hipMemcpyAsync(din, h_in + o, chunk, hipMemcpyHostToDevice, a));
                        }
                        if (mode >= 2) hipLaunchKernelGGL(touch_kernel, dim3(1), dim3(64), 0, a, d_k);
                        if (mode >= 1) {
                            CK(hipEventRecord(ev_in[k], a));
                            CK(hipStreamWaitEvent(b, ev_in[k], 0));
                        }
                        if (mode >= 3) {
                            CK(hipMemcpyAsync(h_out + o, dout, chunk - small, hipMemcpyDeviceToHost, b));
                            CK(hipMemcpyAsync(h_out + o + chunk - small, dout + chunk - small, small, hipMemcpyDeviceToHost, b));
                        } else {
                            CK(hipMemcpyAsync(h_out + o, dout, chunk, hipMemcpyDeviceToHost, b));
                        }
                        if (mode >= 4) CK(hipEventRecord(ev_done[k], b));
                    }
                    CK(hipStreamSynchronize(a));
                    CK(hipStreamSynchronize(b));
                    const double dt = now() - t0;
                    best = std::max(best, 2.0 * total / dt / 1e9);
                }
                printf("{\"sweep\": %d, \"extra_streams\": %d, \"distinct\": %d, \"mode\": \"%s\", \"both_gbps\": %.1f}\n",
                       sweep, extra, distinct, names[mode], best);
                fflush(stdout);
            }
            CK(hipStreamDestroy(a));
            CK(hipStreamDestroy(b));
            for (auto& s : others) CK(hipStreamDestroy(s));
            for (int k = 0; k < kSlots; ++k) {
                CK(hipEventDestroy(ev_in[k]));
                CK(hipEventDestroy(ev_done[k]));
            }
        }
    }
    // copy engines: 0 SDMA both ways (hipMemcpyAsync, in a process whose runtime picks SDMA), 1 SDMA H2D +
    // kernel D2H (what a torch process's runtime does), 2 kernels both ways; `blocks` workgroups per copy kernel
    for (int eng = 0; eng < 3; ++eng) {
        for (int blocks : {32, 128, 512}) {
            if (eng == 0 && blocks != 32) continue;
            hipStream_t a, b;
            CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
            CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
            hipEvent_t ev[kSlots];
            for (auto& x : ev) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
            double best = 0, best_h = 0, best_d = 0;
            for (int rep = 0; rep < 3; ++rep) {
                for (int dir = 0; dir < 3; ++dir) {  // 0 both, 1 H2D only, 2 D2H only
                    CK(hipDeviceSynchronize());
                    const double t0 = now();
                    const size_t C = total / chunk;
                    for (size_t c = 0; c < C; ++c) {
                        const size_t o = c * chunk;
                        if (dir != 2) {
                            if (eng == 2)
                                hipLaunchKernelGGL(copy_kernel, dim3(blocks), dim3(256), 0, a, (const uint4*)(h_in + o),
                                                   (uint4*)(d_in_all + o), chunk / 16);
                            else
                                CK(hipMemcpyAsync(d_in_all + o, h_in + o, chunk, hipMemcpyHostToDevice, a));
                            CK(hipEventRecord(ev[c % kSlots], a));
                            CK(hipStreamWaitEvent(b, ev[c % kSlots], 0));
                        }
                        if (dir != 1) {
                            if (eng >= 1)
                                hipLaunchKernelGGL(copy_kernel, dim3(blocks), dim3(256), 0, b, (const uint4*)(d_out_all + o),
                                                   (uint4*)(h_out + o), chunk / 16);
                            else
                                CK(hipMemcpyAsync(h_out + o, d_out_all + o, chunk, hipMemcpyDeviceToHost, b));
                        }
                    }
                    CK(hipStreamSynchronize(a));
                    CK(hipStreamSynchronize(b));
                    const double r = (dir == 0 ? 2.0 : 1.0) * total / (now() - t0) / 1e9;
                    double& bst = dir == 0 ? best : dir == 1 ? best_h : best_d;
                    bst = std::max(bst, r);
                }
            }
            printf("{\"engines\": \"%s\", \"blocks\": %d, \"both_gbps\": %.1f, \"h2d_gbps\": %.1f, \"d2h_gbps\": %.1f}\n",
                   eng == 0 ? "sdma/sdma" : eng == 1 ? "sdma/kernel" : "kernel/kernel", blocks, best, best_h, best_d);
            fflush(stdout);
            CK(hipStreamDestroy(a));
            CK(hipStreamDestroy(b));
            for (auto& x : ev) CK(hipEventDestroy(x));
        }
    }
    // host-wait with more slots (host.cpp's kSlots), warm
    for (int slots : {3, 4, 6, 8}) {
        hipStream_t a, b;
        CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
        std::vector<hipEvent_t> ev_in(slots), ev_done(slots);
        for (int k = 0; k < slots; ++k) {
            CK(hipEventCreateWithFlags(&ev_in[k], hipEventDisableTiming));
            CK(hipEventCreateWithFlags(&ev_done[k], hipEventDisableTiming));
        }
        double best = 0;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipDeviceSynchronize());
            const double t0 = now();
            const size_t C = total / chunk;
            for (size_t c = 0; c < C; ++c) {
                const int k = (int)(c % slots);
                const size_t o = c * chunk;
                if (c >= (size_t)slots) CK(hipEventSynchronize(ev_done[k]));
                CK(hipMemcpyAsync(d_in_all + o, h_in + o, chunk - 3 * small, hipMemcpyHostToDevice, a));
                for (int s = 0; s < 3; ++s)
                    CK(hipMemcpyAsync(d_in_all + o + chunk - (s + 1) * small, h_in + o + chunk - (s + 1) * small, small,
                                      hipMemcpyHostToDevice, a));
                hipLaunchKernelGGL(touch_kernel, dim3(1), dim3(64), 0, a, d_k);
                CK(hipEventRecord(ev_in[k], a));
                CK(hipStreamWaitEvent(b, ev_in[k], 0));
                CK(hipMemcpyAsync(h_out + o, d_out_all + o, chunk - small, hipMemcpyDeviceToHost, b));
                CK(hipMemcpyAsync(h_out + o + chunk - small, d_out_all + o + chunk - small, small, hipMemcpyDeviceToHost, b));
                CK(hipEventRecord(ev_done[k], b));
            }
            CK(hipStreamSynchronize(a));
            CK(hipStreamSynchronize(b));
            best = std::max(best, 2.0 * total / (now() - t0) / 1e9);
        }
        printf("{\"host_wait_slots\": %d, \"both_gbps\": %.1f}\n", slots, best);
        fflush(stdout);
        CK(hipStreamDestroy(a));
        CK(hipStreamDestroy(b));
        for (int k = 0; k < slots; ++k) {
            CK(hipEventDestroy(ev_in[k]));
            CK(hipEventDestroy(ev_done[k]));
        }
    }
    return 0;
}
