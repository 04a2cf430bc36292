// record_worker.hip -- the per-record Serializer path without a launch per record (sym_batcher_*).
//
// The reference calls Marshal / Unmarshal once per record from many goroutines at once
// (pkg/rpc/client.go:233-310, :252; pkg/rpc/server.go:152 / :173; pkg/serializer/symphony.go:10-16).
// A kernel launch plus a synchronisation per call costs ~10 us or more; here one small persistent
// kernel (one workgroup per queue) serves the records in place in a ring of slots in pinned host
// memory that is mapped into the GPU's address space and coherent both ways:
//
//   caller   t = ticket++; wait until slot[t % kRingSlots].turn == t; write the record into the slot;
//            store req = t + 1; posted += 1; if the worker announced that it is quitting, see that
//            one runs (batcher.cpp); spin until done == t + 1; copy the result out; turn = t + kRingSlots
//   worker   poll `posted` (one 8-byte PCIe read); when it passed the records served, every lane looks
//            at one slot of the window [e, e + kRingSlots) and the ready ones are served, one wave per
//            record: the record is read into LDS with system-scope 8-byte loads, encoded or parsed there
//            exactly as MarshalSymphony / UnmarshalSymphony (kv.syn.go:611-745, echo.syn.go:111-263),
//            the result written back with system-scope 8-byte stores, waited for, then done = t + 1
//
// The worker exits when told to (sym_batcher_destroy) or after kIdleTicks without a record; before it
// exits it announces `quit` and looks at `posted` once more (a Dekker hand-shake with the callers,
// who publish before they look at `quit`), so a record posted meanwhile is either served by this
// worker or finds the announcement and has the caller launch the next one.  No wave waits on another
// workgroup, and every wave reaches the exit.
#include <hip/hip_runtime.h>

#include "../../include/symphony_hip.h"
#include "codec.hpp"
#include "device_util.hpp"
#include "record_worker.hpp"

namespace symhip {
namespace rw {

__device__ __forceinline__ u64 ld_sys(const u64* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }
__device__ __forceinline__ void st_sys(u64* p, u64 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }
__device__ __forceinline__ void fence_sys() { __atomic_thread_fence(__ATOMIC_SEQ_CST); }

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

constexpr size_t kOutStage = (kDecData + 2 * (kRingRecordMax + 16) + 15) & ~(size_t)15;  // >= any result
struct alignas(16) WaveBuf {
    uint8_t in[kSlotIn + 16];
    uint8_t out[kOutStage + 16];
};

struct alignas(16) Lds {
    WaveBuf w[kWaves];
    u64 served[kRingSlots];  // served[t % kRingSlots] == t + 1: ticket t was served by a worker
    int list[kRingSlots];    // ready tickets of this pass (offsets from e)
    int nlist;
    int quit;                // 1: leave the loop
};

__device__ __forceinline__ u32 rd32(const uint8_t* b, u64 q) {
    return (u32)b[q] | ((u32)b[q + 1] << 8) | ((u32)b[q + 2] << 16) | ((u32)b[q + 3] << 24);
}

// One wave copies `bytes` (rounded up to 8) from host memory at src (8-byte aligned) into LDS with
// system-scope 8-byte loads: they read the caller's bytes from host memory, never a cached copy.
__device__ __forceinline__ void load_in(uint8_t* dst, const uint8_t* src, u64 bytes, int lane) {
    for (u64 c = 8 * (u64)lane; c < bytes; c += 8 * 64) *(u64*)(dst + c) = ld_sys((const u64*)(src + c));
}
// One wave copies `bytes` (rounded up to 8) from LDS to host memory at dst with system-scope 8-byte
// stores, then waits until they are performed: the done flag that follows cannot overtake them.
__device__ __forceinline__ void store_out(uint8_t* dst, const uint8_t* src, u64 bytes, int lane) {
    for (u64 c = 8 * (u64)lane; c < bytes; c += 8 * 64) st_sys((u64*)(dst + c), *(const u64*)(src + c));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// MarshalSymphony of one record (+ the client's ID patch, pkg/rpc/client.go:267-271) into LDS.
// In area: EncIn header, then the var fields' bytes back to back.  Returns the record size.
__device__ u64 encode_one(const Layout lay, const uint8_t* in, uint8_t* out, int lane) {
    const EncIn* h = (const EncIn*)in;
    const int F = lay.nfixed, V = lay.nvar;
    const u64 tab = 14 + 4 * (u64)(F + V);  // header + private table
    u64 len[kMaxVar] = {0, 0}, pay[kMaxVar] = {0, 0}, src[kMaxVar] = {0, 0};
    u64 p = tab, s = sizeof(EncIn);
#pragma unroll
    for (int f = 0; f < kMaxVar; ++f) {
        if (f < V) {
            len[f] = h->len[f];
            pay[f] = p;  // the field's [u32 len]
            src[f] = s;
            p += 4 + len[f];
            s += len[f];
        }
    }
    const u64 size = p;
    for (u64 q = (u64)lane; q < size; q += 64) {
        u32 b;
        if (q < tab) {
            u32 word = 0;  // the 4-byte word holding byte q (the two version bytes aside)
            const u64 w = q < 13 ? (q - 1) / 4 : (q - 14) / 4;
            if (q == 0 || q == 13) {
                b = 1;  // public / private version
                out[q] = (uint8_t)b;
                continue;
            }
            if (q < 13) word = w == 0 ? 13u : (w == 1 ? h->service_id : h->method_id);
            else if ((int)w < F) word = (u32)h->fixed[w];
            else word = (u32)((w == (u64)F ? pay[0] : pay[1]) - 13);  // offset relative to the private segment
            const u64 k = q < 13 ? (q - 1) % 4 : (q - 14) % 4;
            b = (word >> (8 * k)) & 0xffu;
        } else {
            const bool second = V == 2 && q >= pay[1];
            const u64 r = q - (second ? pay[1] : pay[0]);
            const u64 ln = second ? len[1] : len[0];
            b = r < 4 ? (u32)((ln >> (8 * r)) & 0xffu) : in[(second ? src[1] : src[0]) + (r - 4)];
        }
        out[q] = (uint8_t)b;
    }
    return size;
}

// UnmarshalSymphony of one record (kv.syn.go:680-745, echo.syn.go:186-263) from LDS: the DecOut header
// and the fields' bytes (field f at kDecData + its offset) into LDS.  Returns the out bytes used.
__device__ u64 decode_one(const Layout lay, const uint8_t* in, u64 L, uint8_t* out, int lane) {
    DecOut* o = (DecOut*)out;
    u64 flen[kMaxVar] = {0, 0}, fpos[kMaxVar] = {0, 0};
    u32 st = SYM_STATUS_OK;
    int32_t fx[kMaxFixed] = {0, 0};
    if (L < 13) {
        st = SYM_STATUS_TOO_SHORT;
    } else if (in[0] != 0x01) {
        st = SYM_STATUS_BAD_VERSION;
    } else {
        const u64 off2p = rd32(in, 1);
        if (off2p >= L || in[off2p] != 0x01) {
            st = SYM_STATUS_NO_PRIVATE;
        } else {
            const u64 pts = off2p + 1;
            u64 toff = 0;
#pragma unroll
            for (int f = 0; f < kMaxFixed; ++f) {
                if (f < lay.nfixed) {
                    if (st == 0) {
                        if (L < pts + toff + 4) st = SYM_STATUS_FIELD_TOO_SHORT;
                        else fx[f] = (int32_t)rd32(in, pts + toff);
                    }
                    toff += 4;
                }
            }
            if (st == 0) {
#pragma unroll
                for (int f = 0; f < kMaxVar; ++f, toff += 4) {
                    if (f < lay.nvar && L >= pts + toff + 4) {
                        u64 q = rd32(in, pts + toff);
                        if (q > 0) q += off2p;
                        if (q > 0 && L >= q + 4) {
                            const u64 nb = rd32(in, q);
                            if (L >= q + 4 + nb) {
                                flen[f] = nb;
                                fpos[f] = q + 4;
                            }
                        }
                    }
                }
            }
        }
    }
    const u64 at1 = (flen[0] + 15) & ~(u64)15;  // field 1's bytes start 16-byte aligned after field 0's
    if (lane == 0) {
        o->status = st;
        for (int f = 0; f < kMaxFixed; ++f) o->fixed[f] = fx[f];
        for (int f = 0; f < kMaxVar; ++f) o->len[f] = flen[f];
        o->at1 = at1;
    }
    uint8_t* d = out + kDecData;
    for (u64 q = (u64)lane; q < flen[0]; q += 64) d[q] = in[fpos[0] + q];
    for (u64 q = (u64)lane; q < flen[1]; q += 64) d[at1 + q] = in[fpos[1] + q];
    return kDecData + at1 + flen[1];
}

__global__ __launch_bounds__(kThreads) void worker_kernel(RingCtl* ctl, uint8_t* slots, Layout lay, int dir, u64 gen) {
    __shared__ Lds S;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    u64 e = ld_sys(&ctl->e), nproc = ld_sys(&ctl->nproc);  // where the previous worker stopped
    // tickets of the window the previous worker served out of order
    for (int k = tid; k < kRingSlots; k += kThreads) {
        const u64 t = e + (u64)k;
        const SlotCtl* sc = (const SlotCtl*)(slots + (size_t)(t % kRingSlots) * kSlotBytes);
        const u64 d = ld_sys(&sc->done);
        S.served[t % kRingSlots] = d == t + 1 ? t + 1 : 0;
    }
    if (tid == 0) S.quit = 0;
    __syncthreads();
    u64 progress = __builtin_amdgcn_s_memrealtime();  // lane 0 of wave 0: when a record was last served
    u64 served = tid == 0 ? ld_sys(&ctl->served) : 0, passes = tid == 0 ? ld_sys(&ctl->passes) : 0;
    for (;;) {
        // ---- wave 0, lane 0: is there work, should we stop? ----
        if (tid == 0) {
            S.nlist = 0;
            for (;;) {
                if (ld_sys(&ctl->stop)) {
                    S.quit = 1;
                    break;
                }
                const u64 posted = ld_sys(&ctl->posted);
                if (__builtin_amdgcn_s_memrealtime() - progress > kIdleTicks) {
                    // Nothing served for a while: announce, then look once more.  A caller publishes and
                    // then looks at `quit`, so either we see its record here or it sees the announcement
                    // (batcher.cpp ensure_worker); a caller that still waits later finds `gone`.
                    st_sys(&ctl->quit, gen);
                    fence_sys();
                    if (ld_sys(&ctl->posted) != posted) {
                        st_sys(&ctl->quit, 0);
                        progress = __builtin_amdgcn_s_memrealtime();
                        continue;
                    }
                    S.quit = 1;
                    break;
                }
                if (posted != nproc) break;  // published records not served yet
                __builtin_amdgcn_s_sleep(10);
            }
        }
        __syncthreads();
        if (S.quit) break;
        // ---- the window: which tickets are ready and not served yet ----
        {
            const u64 t = e + (u64)tid;
            const SlotCtl* sc = (const SlotCtl*)(slots + (size_t)(t % kRingSlots) * kSlotBytes);
            const bool ready = S.served[t % kRingSlots] != t + 1 && ld_sys(&sc->req) == t + 1;
            if (ready) S.list[atomicAdd(&S.nlist, 1)] = tid;
        }
        __syncthreads();
        const int nl = S.nlist;
        for (int i = wave; i < nl; i += kWaves) {  // one wave per record
            const u64 t = e + (u64)S.list[i];
            uint8_t* slot = slots + (size_t)(t % kRingSlots) * kSlotBytes;
            SlotCtl* sc = (SlotCtl*)slot;
            WaveBuf& B = S.w[wave];
            const u64 in_len = min(ld_sys(&sc->in_len), (u64)kRingRecordMax);  // (the caller checked it)
            if (dir == 0) {
                load_in(B.in, slot + kSlotInAt, sizeof(EncIn) + in_len, lane);
                wave_sync();
                const u64 size = encode_one(lay, B.in, B.out, lane);
                wave_sync();
                store_out(slot + kSlotOutAt, B.out, size, lane);
            } else {
                load_in(B.in, slot + kSlotInAt, in_len, lane);
                wave_sync();
                const u64 used = decode_one(lay, B.in, in_len, B.out, lane);
                wave_sync();
                store_out(slot + kSlotOutAt, B.out, used, lane);
            }
            if (lane == 0) st_sys(&sc->done, t + 1);  // after the wave's stores were performed
        }
        __syncthreads();
        // ---- served: advance the window over its served prefix ----
        for (int i = tid; i < nl; i += kThreads) {
            const u64 t = e + (u64)S.list[i];
            S.served[t % kRingSlots] = t + 1;
        }
        __syncthreads();
        nproc += (u64)nl;
        while (S.served[e % kRingSlots] == e + 1) ++e;  // (every thread, the same walk)
        if (nl) {
            progress = __builtin_amdgcn_s_memrealtime();
            if (tid == 0) {  // (stores only: the counters of earlier workers were read at the start)
                served += (u64)nl;
                st_sys(&ctl->served, served);
                st_sys(&ctl->passes, ++passes);
            }
        } else {
            __builtin_amdgcn_s_sleep(20);  // published records outside the window: look again shortly
        }
        __syncthreads();
    }
    if (tid == 0) {  // where the next worker starts; then gone (the callers' hand-shake)
        st_sys(&ctl->e, e);
        st_sys(&ctl->nproc, nproc);
        fence_sys();
        st_sys(&ctl->gone, gen);
    }
}

}  // namespace rw

hipError_t launch_record_worker(RingCtl* ctl, uint8_t* slots, Layout lay, int dir, uint64_t gen, hipStream_t stream) {
    hipLaunchKernelGGL(rw::worker_kernel, dim3(1), dim3(rw::kThreads), 0, stream, ctl, slots, lay, dir, (u64)gen);
    return hipGetLastError();
}

}  // namespace symhip
