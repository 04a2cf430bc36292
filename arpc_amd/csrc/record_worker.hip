// record_worker.hip -- the per-record Serializer path without a launch per record (sym_batcher_*).
//
// The reference calls Marshal / Unmarshal once per record from many goroutines at once
// (pkg/rpc/client.go:233-310, :252; pkg/rpc/server.go:152 / :173; pkg/serializer/symphony.go:10-16).
// A kernel launch plus a synchronisation per call costs ~10 us or more; here one small persistent
// kernel per device (kGroups workgroups, shared by every batcher on the device and both directions) serves
// the records in place in a ring of slots in pinned host memory that is mapped into the GPU's address
// space and coherent both ways:
//
//   caller   t = ticket++; wait until slot[t % kRingSlots].turn == t; write the record and its kind
//            (direction, layout, batcher id) into the slot; store req = t + 1; posted += 1; if the worker announced
//            that it is quitting, see that the next one runs (batcher.cpp); spin until done == t + 1;
//            copy the result out; turn = t + kRingSlots
//   worker   poll `posted` (one 8-byte PCIe read) while cold; when it passed the records served -- or
//            at once while hot (a record within the last 50 us) -- each of the first kWin threads
//            (kRingSlots / kGroups = 64) looks at one slot of the group's window (req and
//            in_len|tag|kind in one round trip; the tag is the ticket's low bits, checked against req)
//            and the ready ones are served, one wave per record, 16 at once: the record is read into
//            LDS with system-scope 8-byte loads and encoded or parsed there exactly as MarshalSymphony /
//            UnmarshalSymphony (kv.syn.go:611-745, echo.syn.go:111-263), each 8-byte word of the result
//            built from LDS and written with a system-scope store, waited for, then done = t + 1
//
// The worker exits when told to (the device's last sym_batcher_destroy, sym_batcher_quiesce), after
// kIdleTicks without a record, or after kLifeTicks of life, busy or idle (a persistent kernel holds
// its hardware queue: with more streams than queues, a launch that shares the queue waits behind it,
// so the worker hands over to a fresh launch, which queues behind that launch).  The exit is announced and
// the records owed are served first (worker_kernel), so no caller is left waiting.  No wave waits on
// another workgroup, and every wave reaches the exit.
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
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

constexpr int kThreads = 1024;  // 16 waves: up to 16 records served at once (each latency-bound)
constexpr int kWaves = kThreads / 64;
constexpr u64 kHotTicks = 5000;  // 50 us after the last record the worker polls the slots directly
constexpr int kWin = kRingSlots / kGroups;  // a group's window: tickets e, e + kGroups, ... (one slot each)
static_assert(kRingSlots % kGroups == 0 && kWin <= kThreads, "window");

struct alignas(16) Lds {
    uint8_t in[kWaves][kSlotIn + 16];  // a wave's record (results are built from it word by word)
    u64 served[kWin];        // served[widx(t)] == t + 1: this group's ticket t was served
    int list[kWin];          // ready tickets of this pass (window positions: ticket e + kGroups * k)
    u32 len[kWin];           // and their in_len
    u32 kind[kWin];          // and kind (slot_kind >> 32)
    int nlist;
    int owed;                // draining: ready tickets below t0 in this pass
    int drain;               // 1: the exit is announced (serve what is owed, then leave)
    int hot;                 // 1: records came lately: look at the slots without waiting for `posted`
    u64 t0;                  // draining: the ticket counter read after the announcement
    u64 bp[2 * kMaxBatchers];         // ctl->bpasses, kept here (this worker is their only writer)
    u32 bseen[2 * kMaxBatchers / 32]; // batcher-direction pairs with a record in this pass
};

__device__ __forceinline__ u32 rd32(const uint8_t* b, u64 q) {
    return (u32)b[q] | ((u32)b[q + 1] << 8) | ((u32)b[q + 2] << 16) | ((u32)b[q + 3] << 24);
}
__device__ __forceinline__ u64 rd64(const uint8_t* b) {  // 8 bytes from any LDS byte address
    u64 v = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) v |= (u64)b[i] << (8 * i);
    return v;
}

// One wave copies `bytes` (rounded up to 8) from host memory at src (8-byte aligned) into LDS with
// system-scope 8-byte loads: they read the caller's bytes from host memory, never a cached copy.
__device__ __forceinline__ void load_in(uint8_t* dst, const uint8_t* src, u64 bytes, int lane) {
    for (u64 c = 8 * (u64)lane; c < bytes; c += 8 * 64) *(u64*)(dst + c) = ld_sys((const u64*)(src + c));
}
// One wave writes words [0, words) of a result, word(w) computed from LDS, to host memory at dst
// with system-scope 8-byte stores, then waits until they are performed: the done flag that follows
// cannot overtake them.
template <class W>
__device__ __forceinline__ void store_words(uint8_t* dst, u64 words, int lane, W&& word) {
    for (u64 w = (u64)lane; w < words; w += 64) st_sys((u64*)dst + w, word(w));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// MarshalSymphony of one record (+ the client's ID patch, pkg/rpc/client.go:267-271) from its in
// area (EncIn header, then the var fields' bytes back to back) straight to the slot's out area.
__device__ void encode_one(const Layout lay, const uint8_t* in, uint8_t* dst, int lane) {
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
    // scalars for the lambdas (a captured array would live in scratch)
    const u64 len0 = len[0], len1 = len[1], pay0 = pay[0], pay1 = pay[1], src0 = src[0], src1 = src[1];
    auto byte_at = [&](u64 q) -> u32 {
        if (q >= size) return 0;
        if (q < tab) {
            if (q == 0 || q == 13) return 1;  // public / private version
            const u64 w = q < 13 ? (q - 1) / 4 : (q - 14) / 4;
            u32 word;  // the 4-byte word holding byte q
            if (q < 13) word = w == 0 ? 13u : (w == 1 ? h->service_id : h->method_id);
            else if ((int)w < F) word = (u32)h->fixed[w];
            else word = (u32)((w == (u64)F ? pay0 : pay1) - 13);  // offset relative to the private segment
            const u64 k = q < 13 ? (q - 1) % 4 : (q - 14) % 4;
            return (word >> (8 * k)) & 0xffu;
        }
        const bool second = V == 2 && q >= pay1;
        const u64 r = q - (second ? pay1 : pay0);
        const u64 ln = second ? len1 : len0;
        return r < 4 ? (u32)((ln >> (8 * r)) & 0xffu) : in[(second ? src1 : src0) + (r - 4)];
    };
    store_words(dst, (size + 7) / 8, lane, [&](u64 w) {
        u64 v = 0;
        for (int i = 0; i < 8; ++i) v |= (u64)byte_at(8 * w + i) << (8 * i);
        return v;
    });
}

// UnmarshalSymphony of one record (kv.syn.go:680-745, echo.syn.go:186-263) from its in area straight
// to the slot's out area: the DecOut header, field 0's bytes at kDecData, field 1's at kDecData + at1.
__device__ void decode_one(const Layout lay, const uint8_t* in, u64 L, uint8_t* dst, int lane) {
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
    static_assert(sizeof(DecOut) == 40 && kDecData == 64, "DecOut words: status | fixed[0], fixed[1], len[0], len[1], at1");
    // (a field's last word may read up to 7 bytes past it: inside the in area, never used)
    const u64 flen0 = flen[0], flen1 = flen[1], fpos0 = fpos[0], fpos1 = fpos[1];  // (no captured arrays)
    const u64 w0 = (u64)st | ((u64)(u32)fx[0] << 32), w1 = (u64)(u32)fx[1];
    store_words(dst, (kDecData + at1 + flen1 + 7) / 8, lane, [&](u64 w) -> u64 {
        switch (w) {
            case 0: return w0;
            case 1: return w1;
            case 2: return flen0;
            case 3: return flen1;
            case 4: return at1;
            case 5: case 6: case 7: return 0;
            default: break;
        }
        const u64 p = 8 * w - kDecData;
        return p < at1 ? rd64(in + fpos0 + p) : rd64(in + fpos1 + (p - at1));
    });
}

// The exit (idle for kIdleTicks, busy for kLifeTicks, or told to stop) is announced, not taken at
// once: `quit` = this generation, a system fence, then the callers' ticket counter T0 is read.  A
// caller publishes its record (req, then posted) and only then looks at `quit` (sequentially
// consistent on the host), so for each record either its caller sees the announcement -- and has
// the next generation launched once this one is `gone` (batcher.cpp ring_ensure_worker) -- or this
// worker sees its req in a later window scan, and such a record has a ticket below T0.  So the
// worker keeps scanning until a pass finds no ready ticket below T0 in its window; a ready ticket
// below T0 outside the window waits behind a lower one whose caller published after the
// announcement, and the next generation serves both.
// kGroups (4) workgroups run as one launch, so the worker still holds one hardware queue: group w
// serves the tickets t with t % kGroups == w -- its own window, `posted` word, counters and exit --
// so kGroups passes are in flight at once (a pass is a few PCIe round trips whatever its size: one
// group served both directions at ~0.65 M records/s from 64 threads, four at ~0.86 M).  Each group
// announces and drains as above for its own tickets (all reach kLifeTicks together); the last group
// to leave publishes `gone`.
__device__ __forceinline__ int widx(u64 t) { return (int)((t % kRingSlots) / kGroups); }

__global__ __launch_bounds__(kThreads) void worker_kernel(RingCtl* ctl, uint8_t* slots, unsigned* exits, u64 gen) {
    __shared__ Lds S;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = blockIdx.x;
    u64 e = ld_sys(&ctl->e[grp]), nproc = ld_sys(&ctl->nproc[grp]);  // where the group's previous run stopped
    // tickets of the window the previous worker served out of order
    for (int k = tid; k < kWin; k += kThreads) {
        const u64 t = e + (u64)kGroups * k;
        const SlotCtl* sc = (const SlotCtl*)(slots + (size_t)(t % kRingSlots) * kSlotBytes);
        const u64 d = ld_sys(&sc->done);
        S.served[widx(t)] = d == t + 1 ? t + 1 : 0;
    }
    for (int k = tid; k < 2 * kMaxBatchers; k += kThreads) S.bp[k] = ld_sys(&ctl->bpasses[grp][k >> 1][k & 1]);
    if (tid == 0) {
        S.drain = 0;
        S.t0 = 0;
        S.hot = 0;
    }
    __syncthreads();
    const u64 born = __builtin_amdgcn_s_memrealtime();
    u64 progress = born;  // when a record was last served (every thread)
    u64 served = tid == 0 ? ld_sys(&ctl->served[grp]) : 0, passes = tid == 0 ? ld_sys(&ctl->passes[grp]) : 0;
    auto announce = [&]() {  // (thread 0)
        st_sys(&ctl->quit, gen);
        fence_sys();
        S.t0 = ld_sys(&ctl->ticket);
        S.drain = 1;
    };
    for (;;) {
        // ---- cold: thread 0 waits for work on `posted` (one 8-byte PCIe read per look) ----
        if (tid < 2 * kMaxBatchers / 32) S.bseen[tid] = 0;
        if (tid == 0) {
            S.nlist = 0;
            S.owed = 0;
            while (!S.drain && !S.hot) {
                const u64 posted = ld_sys(&ctl->posted[grp]);
                const u64 now = __builtin_amdgcn_s_memrealtime();
                if (ld_sys(&ctl->stop) || now - progress > kIdleTicks || now - born > kLifeTicks) announce();
                else if (posted != nproc) break;  // published records not served yet
                else __builtin_amdgcn_s_sleep(10);
            }
            if (!S.drain && (__builtin_amdgcn_s_memrealtime() - born > kLifeTicks || (S.hot && ld_sys(&ctl->stop))))
                announce();
        }
        __syncthreads();
        // ---- the window: which tickets are ready and not served yet (req and in_len in one round trip) ----
        const u64 t0 = S.t0;
        const bool drain = S.drain;
        if (tid < kWin) {
            const u64 t = e + (u64)kGroups * tid;
            const SlotCtl* sc = (const SlotCtl*)(slots + (size_t)(t % kRingSlots) * kSlotBytes);
            // req and in_len in one system-coherent 16-byte load (volatile: sc0 sc1, as ld_sys)
            const u64x2 ri = *(const volatile u64x2*)&sc->req;
            const u64 rq = ri.x, il = ri.y;
            // (in_len carries the ticket's low bits: a length and kind left by the slot's previous
            // ticket never pair with this req -- the slot is then simply not ready yet)
            if (S.served[widx(t)] != t + 1 && rq == t + 1 && (il & 0xffff0000ull) == slot_tag(t)) {
                const int k = atomicAdd(&S.nlist, 1);
                S.list[k] = tid;
                S.len[k] = (u32)min(il & kSlotLenMask, (u64)kRingRecordMax);  // (the caller checked it)
                S.kind[k] = (u32)(il >> 32);
                const u32 bd = 2 * ((u32)(il >> 56) & 0xffu) + (u32)((il >> 32) & 1);  // batcher, direction
                atomicOr(&S.bseen[bd >> 5], 1u << (bd & 31));
                if (drain && t < t0) atomicAdd(&S.owed, 1);
            }
        }
        __syncthreads();
        if (drain && S.owed == 0) break;  // every record this generation owes is served
        const int nl = S.nlist;
        ++passes;
        for (int i = wave; i < nl; i += kWaves) {  // one wave per record
            const u64 t = e + (u64)kGroups * S.list[i];
            uint8_t* slot = slots + (size_t)(t % kRingSlots) * kSlotBytes;
            SlotCtl* sc = (SlotCtl*)slot;
            uint8_t* in = S.in[wave];
            const u64 in_len = S.len[i];
            const u32 kind = S.kind[i];
            const Layout lay{(int)((kind >> 8) & 0xff), (int)((kind >> 16) & 0xff)};
            if ((kind & 0xff) == 0) {
                load_in(in, slot + kSlotInAt, sizeof(EncIn) + in_len, lane);
                wave_sync();
                encode_one(lay, in, slot + kSlotOutAt, lane);
            } else {
                load_in(in, slot + kSlotInAt, in_len, lane);
                wave_sync();
                decode_one(lay, in, in_len, slot + kSlotOutAt, lane);
            }
            if (lane == 0) st_sys(&sc->done, t + 1);  // after the wave's stores were performed
            wave_sync();  // the wave's in buffer is read before its next record overwrites it
        }
        // the pass counters of the batchers served in this pass (issued after the records' done flags,
        // not waited for: a caller may see its record done a few microseconds before its pass counts)
        if (tid < 2 * kMaxBatchers && (S.bseen[tid >> 5] >> (tid & 31) & 1u))
            st_sys(&ctl->bpasses[grp][tid >> 1][tid & 1], ++S.bp[tid]);
        __syncthreads();
        // ---- served: advance the window over its served prefix ----
        for (int i = tid; i < nl; i += kThreads) {
            const u64 t = e + (u64)kGroups * S.list[i];
            S.served[widx(t)] = t + 1;
        }
        __syncthreads();
        nproc += (u64)nl;
        while (S.served[widx(e)] == e + 1) e += kGroups;  // (every thread, the same walk)
        const u64 now = __builtin_amdgcn_s_memrealtime();
        if (nl) {
            progress = now;
            if (tid == 0) {  // (stores only: the counters of earlier workers were read at the start)
                served += (u64)nl;
                st_sys(&ctl->served[grp], served);
                st_sys(&ctl->passes[grp], passes);
                S.hot = 1;
            }
        } else {
            --passes;
            if (tid == 0 && now - progress > kHotTicks) S.hot = 0;  // cold again: wait on `posted`
            __builtin_amdgcn_s_sleep(2);
        }
        __syncthreads();
    }
    if (tid == 0) {  // where the group's next run starts; the last group out publishes gone
        st_sys(&ctl->e[grp], e);
        st_sys(&ctl->nproc[grp], nproc);
        st_sys(&ctl->passes[grp], passes);
        fence_sys();
        if (atomicAdd(exits, 1u) == kGroups - 1) {
            __hip_atomic_store(exits, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
            fence_sys();
            st_sys(&ctl->gone, gen);
        }
    }
}

}  // namespace rw

hipError_t launch_record_worker(RingCtl* ctl, uint8_t* slots, unsigned* exits, uint64_t gen, hipStream_t stream) {
    hipLaunchKernelGGL(rw::worker_kernel, dim3(kGroups), dim3(rw::kThreads), 0, stream, ctl, slots, exits, (u64)gen);
    return hipGetLastError();
}

}  // namespace symhip
