// host.cpp -- sym_encode_host / sym_decode_host: the codec over host memory.
//
// aRPC hands the codec host buffers: Marshal's output goes to fragmentation and the socket, and
// Unmarshal reads pooled receive buffers (pkg/transport/transport.go:87, pkg/common/bufferpool.go).
// These entry points move a host batch through the GPU in record chunks of about kChunkBytes, chunk c
// in slot c % kSlots (device buffers and pinned staging), over ONE stream per direction:
//   stream A: [wait: the slot's last D2H] H2D inputs -> kernel -> event K(c)
//   stream B: [wait: K(c)] D2H outputs -> event D(c)
// so the next chunks' H2D run on A while earlier chunks' D2H run on B.  PCIe is full duplex, but
// only with one stream per direction: tools/pcie_bw.py measured 97 GB/s both ways that way and
// 48-80 GB/s with two to four streams per direction (profiles/r03_pcie_bw.txt), which is what the
// round-3 form (every slot its own stream doing H2D, kernel and D2H) ran into.  Kernels stay on A,
// in chunk order (they share the ctx's workspaces).  A slot is reused after a HOST wait for its
// last D2H (tools/pcie_pattern.hip, profiles/r04_pcie_pattern.txt: the same dependency as a
// device-side wait of A on B's event ran at half the rate).
// Caller memory that is pinned (hipHostMalloc, sym_host_alloc, a registered range) is read and
// written by DMA in place; pageable memory is staged through the slot's pinned buffer with a host
// memcpy, which overlaps the other slots' transfers.
//
// Decode output sizes are only known after the kernel, and a chunk's column bytes go right after
// the previous chunks' in the caller's columns: after each chunk's decode a small kernel on stream
// A rebases its column offsets by the device's running column totals and writes the chunk's
// (base, total) per column into coherent pinned memory.  The host waits for that (an event on A,
// two chunks behind) and issues all of the chunk's D2H at once on B, so B never waits for A on the
// device and never idles behind a chunk whose kernel has not run.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/symphony_hip.h"
#include "codec.hpp"
#include "ctx.hpp"

using namespace symhip::capi;
using symhip::Layout;
using symhip::host::kSlots;
using symhip::host::Slot;

namespace {

constexpr size_t kChunkBytes = 32u << 20;  // target stream bytes per chunk (fewer, larger copies: each op on a
                                            // stream costs ~10 us of dependency latency, r04e trace)
constexpr uint64_t kMinChunkRecords = 1024;
constexpr uint64_t kLag = 1;  // decode: chunk c's D2H are issued after chunk c + kLag's kernels are queued
static_assert(kLag + 2 <= (uint64_t)kSlots, "a slot is reused only after its D2H were issued");

// Tuning builds: SYMHIP_HOST_TRACE=1 prints, per call, the host time spent inside the copy
// enqueues, the waits and the kernel launches (tools/host_timeline.py).
#ifdef SYMHIP_TUNING
struct HostProbe {
    double t[4] = {};
    long n[4] = {};
    std::chrono::steady_clock::time_point t0;
};
HostProbe g_probe;
bool probe_on() {
    static const bool v = getenv("SYMHIP_HOST_TRACE") != nullptr;
    return v;
}
template <class F>
auto timed(int cat, F&& f) {  // 0 H2D enqueue, 1 D2H enqueue, 2 waits, 3 kernel launches
    if (!probe_on()) return f();
    const auto a = std::chrono::steady_clock::now();
    auto r = f();
    g_probe.t[cat] += std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
    ++g_probe.n[cat];
    return r;
}
void probe_begin() {
    if (probe_on()) g_probe = HostProbe{{}, {}, std::chrono::steady_clock::now()};
}
void probe_end(const char* what) {
    if (!probe_on()) return;
    const double tot = std::chrono::duration<double>(std::chrono::steady_clock::now() - g_probe.t0).count();
    fprintf(stderr, "%s: %.3f ms; h2d enqueue %.3f ms (%ld), d2h enqueue %.3f ms (%ld), waits %.3f ms (%ld), kernels %.3f ms (%ld)\n",
            what, 1e3 * tot, 1e3 * g_probe.t[0], g_probe.n[0], 1e3 * g_probe.t[1], g_probe.n[1], 1e3 * g_probe.t[2],
            g_probe.n[2], 1e3 * g_probe.t[3], g_probe.n[3]);
}
#else
template <class F>
auto timed(int, F&& f) {
    return f();
}
inline void probe_begin() {}
inline void probe_end(const char*) {}
#endif

int slots_init(sym_ctx* ctx) {
    if (ctx->slots_ready) return SYM_OK;
    hipError_t e = hipSuccess;
    for (hipStream_t& st : ctx->host_stream)
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    for (Slot& s : ctx->slots) {
        if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&s.kernel, hipEventDisableTiming);
    }
    if (e == hipSuccess)
        e = hipHostMalloc((void**)&ctx->host_meta, sizeof(uint64_t) * 2 * symhip::kMaxVar * kSlots,
                          hipHostMallocCoherent | hipHostMallocMapped);
    if (e == hipSuccess) e = hipMalloc((void**)&ctx->host_base, sizeof(uint64_t) * 2 * symhip::kMaxVar);
    if (e != hipSuccess) {
        symhip::capi::host_slots_destroy(ctx);
        return hip_fail(e, "host slot streams / events");
    }
    ctx->slots_ready = true;
    return SYM_OK;
}

int ensure_slot(Slot& s, size_t dev_need, size_t pin_need) {
    hipError_t e;
    if (dev_need > s.dev_bytes) {
        if (s.dev) (void)hipFree(s.dev);
        s.dev = nullptr;
        s.dev_bytes = 0;
        if ((e = hipMalloc(&s.dev, dev_need)) != hipSuccess)
            return fail(SYM_ERR_NOMEM, "host staging: %zu device bytes: %s", dev_need, hipGetErrorString(e));
        s.dev_bytes = dev_need;
    }
    if (pin_need > s.pin_bytes) {
        if (s.pin) (void)hipHostFree(s.pin);
        s.pin = nullptr;
        s.pin_bytes = 0;
        if ((e = hipHostMalloc(&s.pin, pin_need, hipHostMallocDefault)) != hipSuccess)
            return fail(SYM_ERR_NOMEM, "host staging: %zu pinned bytes: %s", pin_need, hipGetErrorString(e));
        s.pin_bytes = pin_need;
    }
    return SYM_OK;
}

// Host memory the DMA engines can reach in place (pinned / registered).
bool is_pinned(const void* p) {
    if (!p) return true;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// Bump allocator over a slot buffer.  `bad` latches a size that would wrap (never for validated
// offsets; the sizing pass checks it before anything is allocated or copied).
struct Carve {
    size_t at = 0;
    bool bad = false;
    size_t take(size_t bytes) {
        const size_t o = at;
        if (bytes > (SIZE_MAX >> 2) || at > (SIZE_MAX >> 2)) bad = true;
        else at = align256(at + bytes + 16);  // +16: kernels may read 16 bytes past a column
        return o;
    }
};

// Every offset of a host column is >= the one before it.  The chunk sizes, the pinned copies and
// the kernels' record placement all assume it; one pass over n+1 host words (~1 ms per 2^20
// records), far below the PCIe time of the batch.
bool monotone(const uint64_t* o, uint64_t n) {
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; ++i) bad |= (uint64_t)(o[i + 1] < o[i]);
    return bad == 0;
}

uint64_t records_per_chunk(uint64_t n, uint64_t bytes) {
    const uint64_t avg = std::max<uint64_t>(1, bytes / std::max<uint64_t>(1, n));
    uint64_t r = std::max<uint64_t>(kMinChunkRecords, kChunkBytes / avg);
    r = (r + 63) & ~(uint64_t)63;
    return std::min(r, n);
}

int sync_all(sym_ctx* ctx) {
    for (hipStream_t st : ctx->host_stream) {
        hipError_t e = hipStreamSynchronize(st);
        if (e != hipSuccess) return hip_fail(e, "host staging: hipStreamSynchronize");
    }
    return SYM_OK;
}

// After chunk c's decode (stream A): its column offsets 1..m rebased by the running totals of the
// chunks before it, base[c & 1] (base[(c + 1) & 1] = base[c & 1] + the chunk's totals for the next
// chunk), and (base, total) per column into meta, coherent pinned memory the host reads once the
// kernel's event has completed.
struct RebaseArgs {
    uint64_t* offs[symhip::kMaxVar];  // chunk-local offsets, entries 0..m, [0] = 0
    uint64_t m;
    int nvar;
    uint64_t* base_in;
    uint64_t* base_out;
    uint64_t* meta;  // [2 * kMaxVar]: base, total per column
};

__global__ __launch_bounds__(256) void rebase_kernel(RebaseArgs a) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x + 1;
    if (i > a.m) return;
    for (int f = 0; f < a.nvar; ++f) {
        const uint64_t b = a.base_in[f], v = a.offs[f][i];
        a.offs[f][i] = v + b;
        if (i == a.m) {  // the entry's owner: v is the chunk's total
            a.base_out[f] = b + v;
            a.meta[2 * f] = b;
            a.meta[2 * f + 1] = v;
            __threadfence_system();
        }
    }
}

}  // namespace

void symhip::capi::host_slots_destroy(sym_ctx* ctx) {
    for (hipStream_t& st : ctx->host_stream) {
        if (st) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
        st = nullptr;
    }
    for (Slot& s : ctx->slots) {
        if (s.dev) (void)hipFree(s.dev);
        if (s.pin) (void)hipHostFree(s.pin);
        if (s.done) (void)hipEventDestroy(s.done);
        if (s.kernel) (void)hipEventDestroy(s.kernel);
        s = Slot{};
    }
    if (ctx->host_meta) (void)hipHostFree(ctx->host_meta);
    if (ctx->host_base) (void)hipFree(ctx->host_base);
    ctx->host_meta = nullptr;
    ctx->host_base = nullptr;
    ctx->slots_ready = false;
}

extern "C" {

int sym_host_alloc(sym_ctx* ctx, uint64_t bytes, void** out) {
    if (!ctx || !out) return fail(SYM_ERR_INVALID, "sym_host_alloc: NULL argument");
    *out = nullptr;
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    hipError_t e = hipHostMalloc(out, std::max<uint64_t>(bytes, 1), hipHostMallocDefault);
    return e == hipSuccess ? SYM_OK : fail(SYM_ERR_NOMEM, "sym_host_alloc(%llu): %s", (unsigned long long)bytes,
                                           hipGetErrorString(e));
}

int sym_host_free(sym_ctx* ctx, void* p) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_host_free: ctx is NULL");
    if (!p) return SYM_OK;
    DeviceGuard g(ctx->device);
    hipError_t e = hipHostFree(p);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "hipHostFree");
}

int sym_encode_host(sym_ctx* ctx, int schema, uint64_t n, const int32_t* const* h_fixed,
                    const uint8_t* const* h_bytes, const uint64_t* const* h_offs, uint32_t service_id,
                    uint32_t method_id, uint8_t* h_out, uint64_t* h_out_off) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_encode_host: ctx is NULL");
    if (!schema_ok(schema)) return fail(SYM_ERR_INVALID, "sym_encode_host: unknown schema %d", schema);
    if (!h_out_off) return fail(SYM_ERR_INVALID, "sym_encode_host: h_out_off is NULL");
    const Layout lay = kLayouts[schema];
    if (n == 0) {
        h_out_off[0] = 0;
        return SYM_OK;
    }
    if (!h_out || !h_bytes || !h_offs || (lay.nfixed && !h_fixed))
        return fail(SYM_ERR_INVALID, "sym_encode_host: NULL column");
    for (int f = 0; f < lay.nfixed; ++f)
        if (!h_fixed[f]) return fail(SYM_ERR_INVALID, "sym_encode_host: NULL fixed column %d", f);
    uint64_t var_total = 0;
    for (int f = 0; f < lay.nvar; ++f) {
        if (!h_offs[f] || !h_bytes[f]) return fail(SYM_ERR_INVALID, "sym_encode_host: NULL var column %d", f);
        if (!monotone(h_offs[f], n)) return fail(SYM_ERR_INVALID, "sym_encode_host: offsets of field %d decrease", f);
        var_total += h_offs[f][n] - h_offs[f][0];
    }
    const uint64_t ovh = sym_record_overhead(schema);
    const uint64_t R = records_per_chunk(n, ovh * n + var_total);
    const uint64_t C = (n + R - 1) / R;

    // caller memory: pinned -> DMA in place, else staged through the slot's pinned buffer
    bool direct = is_pinned(h_out) && is_pinned(h_out_off);
    for (int f = 0; f < lay.nfixed; ++f) direct = direct && is_pinned(h_fixed[f]);
    for (int f = 0; f < lay.nvar; ++f) direct = direct && is_pinned(h_offs[f]) && is_pinned(h_bytes[f] + h_offs[f][0]);

    // per-chunk buffer sizes (the largest chunk sizes every slot)
    auto chunk_var = [&](uint64_t a, uint64_t b, int f) { return h_offs[f][b] - h_offs[f][a]; };
    size_t dev_need = 0, pin_need = 0;
    for (uint64_t c = 0; c < C; ++c) {
        const uint64_t a = c * R, b = std::min(n, a + R), m = b - a;
        Carve d;
        uint64_t vb = 0;
        for (int f = 0; f < lay.nfixed; ++f) d.take(4 * m);
        for (int f = 0; f < lay.nvar; ++f) {
            d.take(chunk_var(a, b, f));
            d.take(8 * (m + 1));
            vb += chunk_var(a, b, f);
        }
        d.take(m * ovh + vb);
        d.take(8 * (m + 1));
        if (d.bad) return fail(SYM_ERR_INVALID, "sym_encode_host: chunk %llu does not fit the address space",
                               (unsigned long long)c);
        dev_need = std::max(dev_need, d.at);
        if (!direct) pin_need = std::max(pin_need, d.at);
    }
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    int rc = slots_init(ctx);
    for (int k = 0; k < kSlots && rc == SYM_OK; ++k) rc = ensure_slot(ctx->slots[k], dev_need, pin_need);
    if (rc != SYM_OK) return rc;

    struct Pending {  // a staged chunk's outputs, copied out of pinned memory once its D2H landed
        bool live = false;
        size_t pin_out = 0, pin_off = 0;
        uint64_t out_at = 0, out_bytes = 0, a = 0, m = 0;
    } pend[kSlots];
    auto finish = [&](int k) -> int {
        Pending& P = pend[k];
        if (!P.live) return SYM_OK;
        hipError_t e = timed(2, [&] { return hipEventSynchronize(ctx->slots[k].done); });
        if (e != hipSuccess) return hip_fail(e, "sym_encode_host: chunk");
        char* pin = (char*)ctx->slots[k].pin;
        memcpy(h_out + P.out_at, pin + P.pin_out, P.out_bytes);
        memcpy(h_out_off + P.a, pin + P.pin_off, 8 * (P.m + 1));
        P.live = false;
        return SYM_OK;
    };

    hipError_t e = hipSuccess;
    hipStream_t sa = ctx->host_stream[0], sb = ctx->host_stream[1];  // H2D + kernels, D2H
    probe_begin();
    for (uint64_t c = 0; c < C && rc == SYM_OK; ++c) {
        const int k = (int)(c % kSlots);
        Slot& S = ctx->slots[k];
        if ((rc = finish(k)) != SYM_OK) break;
        // the slot's buffers are free once its last D2H is done: a host wait (tools/pcie_pattern: a
        // device-side wait of the H2D stream on the D2H stream's event halved the duplex rate, 80 -> 40 GB/s)
        if ((e = timed(2, [&] { return hipEventSynchronize(S.done); })) != hipSuccess) break;
        const uint64_t a = c * R, b = std::min(n, a + R), m = b - a;
        char* dev = (char*)S.dev;
        char* pin = (char*)S.pin;
        Carve d;
        // stage one input region: DMA in place, or via the slot's pinned buffer (same offset)
        auto h2d = [&](const void* src, size_t bytes) -> size_t {
            const size_t o = d.take(bytes);
            if (!bytes) return o;
            const void* from = src;
            if (!direct) {
                memcpy(pin + o, src, bytes);
                from = pin + o;
            }
            if (e == hipSuccess) e = timed(0, [&] { return hipMemcpyAsync(dev + o, from, bytes, hipMemcpyHostToDevice, sa); });
            return o;
        };
        const int32_t* d_fixed[symhip::kMaxFixed] = {};
        const uint8_t* d_bytes[symhip::kMaxVar] = {};
        const uint64_t* d_offs[symhip::kMaxVar] = {};
        uint64_t vb = 0;
        for (int f = 0; f < lay.nfixed; ++f) d_fixed[f] = (const int32_t*)(dev + h2d(h_fixed[f] + a, 4 * m));
        for (int f = 0; f < lay.nvar; ++f) {
            const uint64_t lo = h_offs[f][a], len = chunk_var(a, b, f);
            d_bytes[f] = (const uint8_t*)(dev + h2d(h_bytes[f] + lo, len)) - lo;  // absolute offsets stay valid
            d_offs[f] = (const uint64_t*)(dev + h2d(h_offs[f] + a, 8 * (m + 1)));
            vb += len;
        }
        const uint64_t out_at = a * ovh;
        uint64_t base = out_at;
        for (int f = 0; f < lay.nvar; ++f) base += h_offs[f][a] - h_offs[f][0];
        const uint64_t out_bytes = m * ovh + vb;
        const size_t o_out = d.take(out_bytes), o_off = d.take(8 * (m + 1));
        if (e != hipSuccess) break;
        rc = timed(3, [&] {
            return encode_call(ctx, schema, m, d_fixed, d_bytes, d_offs, service_id, method_id, (uint8_t*)(dev + o_out),
                               (uint64_t*)(dev + o_off), base, sa);
        });
        if (rc != SYM_OK) break;
        // output sizes are known on the host: B waits for the kernel on the device (tools/pcie_pattern
        // "kernel": 90 GB/s both ways)
        if ((e = hipEventRecord(S.kernel, sa)) != hipSuccess) break;
        if ((e = hipStreamWaitEvent(sb, S.kernel, 0)) != hipSuccess) break;
        uint8_t* to_out = direct ? h_out + base : (uint8_t*)(pin + o_out);
        uint64_t* to_off = direct ? h_out_off + a : (uint64_t*)(pin + o_off);
        if ((e = timed(1, [&] { return hipMemcpyAsync(to_out, dev + o_out, out_bytes, hipMemcpyDeviceToHost, sb); })) != hipSuccess) break;
        if ((e = timed(1, [&] { return hipMemcpyAsync(to_off, dev + o_off, 8 * (m + 1), hipMemcpyDeviceToHost, sb); })) != hipSuccess) break;
        if ((e = hipEventRecord(S.done, sb)) != hipSuccess) break;
        if (!direct) pend[k] = Pending{true, o_out, o_off, base, out_bytes, a, m};
    }
    if (rc == SYM_OK && e != hipSuccess) rc = hip_fail(e, "sym_encode_host");
    for (int k = 0; k < kSlots; ++k) {  // drain in order (even after an error: nothing may stay in flight)
        const int r2 = finish((int)((C + k) % kSlots));
        if (rc == SYM_OK) rc = r2;
    }
    const int r3 = sync_all(ctx);
    if (rc == SYM_OK) rc = r3;
    const int r4 = sym_ctx_check(ctx, sa);  // the kernels' device error word
    probe_end("sym_encode_host");
    return rc == SYM_OK ? r4 : rc;
}

int sym_decode_host(sym_ctx* ctx, int schema, uint64_t n, const uint8_t* h_in, const uint64_t* h_rec_off,
                    int32_t* const* h_fixed, uint8_t* const* h_bytes, const uint64_t* caps, uint64_t* const* h_offs,
                    uint8_t* h_status) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_decode_host: ctx is NULL");
    if (!schema_ok(schema)) return fail(SYM_ERR_INVALID, "sym_decode_host: unknown schema %d", schema);
    const Layout lay = kLayouts[schema];
    if (!h_offs) return fail(SYM_ERR_INVALID, "sym_decode_host: h_offs is NULL");
    for (int f = 0; f < lay.nvar; ++f)
        if (!h_offs[f]) return fail(SYM_ERR_INVALID, "sym_decode_host: h_offs[%d] is NULL", f);
    if (n == 0) {
        for (int f = 0; f < lay.nvar; ++f) h_offs[f][0] = 0;
        return SYM_OK;
    }
    if (!h_in || !h_rec_off || !h_status || !h_bytes || !caps || (lay.nfixed && !h_fixed))
        return fail(SYM_ERR_INVALID, "sym_decode_host: NULL argument");
    for (int f = 0; f < lay.nfixed; ++f)
        if (!h_fixed[f]) return fail(SYM_ERR_INVALID, "sym_decode_host: NULL fixed column %d", f);
    for (int f = 0; f < lay.nvar; ++f)
        if (!h_bytes[f] && caps[f]) return fail(SYM_ERR_INVALID, "sym_decode_host: NULL byte column %d", f);
    if (!monotone(h_rec_off, n)) return fail(SYM_ERR_INVALID, "sym_decode_host: record offsets decrease");
    const uint64_t R = records_per_chunk(n, h_rec_off[n] - h_rec_off[0]);
    const uint64_t C = (n + R - 1) / R;

    bool direct = is_pinned(h_in + h_rec_off[0]) && is_pinned(h_rec_off) && is_pinned(h_status);
    for (int f = 0; f < lay.nfixed; ++f) direct = direct && is_pinned(h_fixed[f]);
    for (int f = 0; f < lay.nvar; ++f) direct = direct && is_pinned(h_offs[f]) && (!caps[f] || is_pinned(h_bytes[f]));

    // slot layout: in | rec_off | status | fixed... | per column: bytes (<= the chunk's stream) | offsets
    size_t dev_need = 0;
    for (uint64_t c = 0; c < C; ++c) {
        const uint64_t a = c * R, b = std::min(n, a + R), m = b - a, span = h_rec_off[b] - h_rec_off[a];
        Carve d;
        d.take(span);
        d.take(8 * (m + 1));
        d.take(m);
        for (int f = 0; f < lay.nfixed; ++f) d.take(4 * m);
        for (int f = 0; f < lay.nvar; ++f) {
            d.take(span);
            d.take(8 * (m + 1));
        }
        if (d.bad) return fail(SYM_ERR_INVALID, "sym_decode_host: chunk %llu does not fit the address space",
                               (unsigned long long)c);
        dev_need = std::max(dev_need, d.at);
    }
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    int rc = slots_init(ctx);
    if (rc == SYM_OK) rc = sym_ctx_reserve(ctx, R);  // no workspace reallocation while chunks are in flight
    for (int k = 0; k < kSlots && rc == SYM_OK; ++k) rc = ensure_slot(ctx->slots[k], dev_need, direct ? 0 : dev_need);
    if (rc != SYM_OK) return rc;

    struct Chunk {  // a chunk between its kernels and its D2H
        int phase = 0;  // 0 idle, 1 kernels queued (no D2H yet), 2 D2H in flight
        uint64_t a = 0, m = 0;
        size_t o_status = 0, o_fixed[symhip::kMaxFixed] = {}, o_col[symhip::kMaxVar] = {}, o_offs[symhip::kMaxVar] = {};
        uint64_t col_at[symhip::kMaxVar] = {}, col_len[symhip::kMaxVar] = {};
    } ch[kSlots];
    bool overflow = false;
    hipError_t e = hipSuccess;
    hipStream_t sa = ctx->host_stream[0], sb = ctx->host_stream[1];  // H2D + kernels, D2H

    // phase 1 -> 2: the chunk's kernels are done; its column (base, total) pairs are in host_meta:
    // every D2H of the chunk at once (fixed-size outputs, rebased offsets, column bytes)
    auto issue = [&](int k) -> int {
        Chunk& Q = ch[k];
        Slot& S = ctx->slots[k];
        if (Q.phase != 1) return SYM_OK;
        if ((e = timed(2, [&] { return hipEventSynchronize(S.kernel); })) != hipSuccess) return hip_fail(e, "sym_decode_host: chunk");
        const volatile uint64_t* meta = ctx->host_meta + 2 * symhip::kMaxVar * k;
        char* pin = (char*)S.pin;
        const char* dev = (const char*)S.dev;
        auto d2h = [&](void* final_dst, size_t o, size_t bytes) {
            if (e == hipSuccess && bytes)
                e = timed(1, [&] { return hipMemcpyAsync(direct ? final_dst : (void*)(pin + o), dev + o, bytes, hipMemcpyDeviceToHost, sb); });
        };
        d2h(h_status + Q.a, Q.o_status, Q.m);
        for (int f = 0; f < lay.nfixed; ++f) d2h(h_fixed[f] + Q.a, Q.o_fixed[f], 4 * Q.m);
        for (int f = 0; f < lay.nvar; ++f) {
            d2h(h_offs[f] + Q.a + 1, Q.o_offs[f] + 8, 8 * Q.m);  // entries 1..m, rebased on the device
            const uint64_t base = meta[2 * f], total = meta[2 * f + 1];
            Q.col_at[f] = base;
            Q.col_len[f] = total;
            if (base + total > caps[f]) {  // SYM_ERR_CAPACITY; the bytes that fit are kept
                overflow = true;
                Q.col_len[f] = caps[f] > base ? caps[f] - base : 0;
            }
            if (Q.col_len[f]) d2h(h_bytes[f] + Q.col_at[f], Q.o_col[f], Q.col_len[f]);
        }
        if (e == hipSuccess) e = hipEventRecord(S.done, sb);
        if (e != hipSuccess) return hip_fail(e, "sym_decode_host: D2H");
        Q.phase = 2;
        return SYM_OK;
    };
    // phase 2 -> idle: staged outputs copied to the caller's memory
    auto complete = [&](int k) -> int {
        Chunk& Q = ch[k];
        if (Q.phase == 1) {
            const int r = issue(k);
            if (r != SYM_OK) return r;
        }
        if (Q.phase != 2) return SYM_OK;
        Slot& S = ctx->slots[k];
        if ((e = timed(2, [&] { return hipEventSynchronize(S.done); })) != hipSuccess) return hip_fail(e, "sym_decode_host: chunk");
        if (!direct) {
            const char* pin = (const char*)S.pin;
            memcpy(h_status + Q.a, pin + Q.o_status, Q.m);
            for (int f = 0; f < lay.nfixed; ++f) memcpy(h_fixed[f] + Q.a, pin + Q.o_fixed[f], 4 * Q.m);
            for (int f = 0; f < lay.nvar; ++f) {
                memcpy(h_offs[f] + Q.a + 1, pin + Q.o_offs[f] + 8, 8 * Q.m);
                if (Q.col_len[f]) memcpy(h_bytes[f] + Q.col_at[f], pin + Q.o_col[f], Q.col_len[f]);
            }
        }
        Q.phase = 0;
        return SYM_OK;
    };

    for (int f = 0; f < lay.nvar; ++f) h_offs[f][0] = 0;
    probe_begin();
    if ((e = hipMemsetAsync(ctx->host_base, 0, sizeof(uint64_t) * 2 * symhip::kMaxVar, sa)) != hipSuccess)
        rc = hip_fail(e, "sym_decode_host");
    for (uint64_t c = 0; c < C && rc == SYM_OK; ++c) {
        const int k = (int)(c % kSlots);
        Slot& S = ctx->slots[k];
        if ((rc = complete(k)) != SYM_OK) break;  // the slot's previous chunk has landed
        const uint64_t a = c * R, b = std::min(n, a + R), m = b - a;
        const uint64_t lo = h_rec_off[a], span = h_rec_off[b] - lo;
        char* dev = (char*)S.dev;
        char* pin = (char*)S.pin;
        Carve d;
        auto h2d = [&](const void* src, size_t bytes) -> size_t {
            const size_t o = d.take(bytes);
            if (!bytes) return o;
            const void* from = src;
            if (!direct) {
                memcpy(pin + o, src, bytes);
                from = pin + o;
            }
            if (e == hipSuccess) e = timed(0, [&] { return hipMemcpyAsync(dev + o, from, bytes, hipMemcpyHostToDevice, sa); });
            return o;
        };
        Chunk& Q = ch[k];
        Q = Chunk{};
        Q.a = a;
        Q.m = m;
        const uint8_t* d_in = (const uint8_t*)(dev + h2d(h_in + lo, span)) - lo;  // absolute offsets stay valid
        const uint64_t* d_rec = (const uint64_t*)(dev + h2d(h_rec_off + a, 8 * (m + 1)));
        Q.o_status = d.take(m);
        int32_t* d_fixed[symhip::kMaxFixed] = {};
        uint8_t* d_bytes[symhip::kMaxVar] = {};
        uint64_t* d_offs[symhip::kMaxVar] = {};
        uint64_t dcaps[symhip::kMaxVar] = {};
        for (int f = 0; f < lay.nfixed; ++f) d_fixed[f] = (int32_t*)(dev + (Q.o_fixed[f] = d.take(4 * m)));
        for (int f = 0; f < lay.nvar; ++f) {
            d_bytes[f] = (uint8_t*)(dev + (Q.o_col[f] = d.take(span)));
            dcaps[f] = span;  // a column never holds more than the chunk's stream
            d_offs[f] = (uint64_t*)(dev + (Q.o_offs[f] = d.take(8 * (m + 1))));
        }
        if (e != hipSuccess) break;
        rc = timed(3, [&] {
            return decode_call("sym_decode_host", ctx, lay, nullptr, m, d_in, d_rec, d_fixed, d_bytes, dcaps, d_offs,
                               (uint8_t*)(dev + Q.o_status), sa);
        });
        if (rc != SYM_OK) break;
        if (lay.nvar) {
            RebaseArgs ra{};
            for (int f = 0; f < lay.nvar; ++f) ra.offs[f] = d_offs[f];
            ra.m = m;
            ra.nvar = lay.nvar;
            ra.base_in = ctx->host_base + (c & 1) * symhip::kMaxVar;
            ra.base_out = ctx->host_base + ((c + 1) & 1) * symhip::kMaxVar;
            ra.meta = ctx->host_meta + 2 * symhip::kMaxVar * k;
            hipLaunchKernelGGL(rebase_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, sa, ra);
            if ((e = hipGetLastError()) != hipSuccess) break;
        }
        if ((e = hipEventRecord(S.kernel, sa)) != hipSuccess) break;
        Q.phase = 1;
        // chunk c - kLag's D2H: its kernels finished long ago (the H2D of the chunks after it are queued
        // on A), and B still has the chunks before it to copy meanwhile
        if (c >= kLag && (rc = issue((int)((c - kLag) % kSlots))) != SYM_OK) break;
    }
    if (rc == SYM_OK && e != hipSuccess) rc = hip_fail(e, "sym_decode_host");
    for (uint64_t i = 0; i < (uint64_t)kSlots; ++i) {  // drain in chunk order
        const int r2 = complete((int)((C + i) % kSlots));
        if (rc == SYM_OK) rc = r2;
    }
    const int r3 = sync_all(ctx);
    if (rc == SYM_OK) rc = r3;
    const int r4 = sym_ctx_check(ctx, sa);
    probe_end("sym_decode_host");
    if (rc != SYM_OK) return rc;
    if (r4 != SYM_OK) return r4;
    if (overflow) return fail(SYM_ERR_CAPACITY, "sym_decode_host: a decoded column exceeds its capacity");
    return SYM_OK;
}

}  // extern "C"
