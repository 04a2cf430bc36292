// batcher.cpp -- sym_batcher_*: concurrent one-record Marshal / Unmarshal calls coalesced into
// device batches (the per-record Serializer path, SURVEY.md 8b "Threading").
//
// The reference Serializer is called once per record from many goroutines at once
// (pkg/rpc/client.go:233-310 Call, :252 Marshal; pkg/rpc/server.go:152 / :173; the adapter
// pkg/serializer/symphony.go:10-16).  One GPU round trip per record would cost a kernel launch and
// a synchronisation each; here callers append to the open batch of a queue and the batch runs as
// one launch.  There is no flusher thread: the batch is run by one of its own callers (combining),
// which saves two thread hand-offs per batch:
//
//   caller:  lock; append the record to slot[fill] (pinned, mapped); then, until the slot is DONE:
//            if no other caller is launching a batch of this queue and the slot is still the open
//              one, LEAD it: wait (up to max_wait_us from the slot's first record, or until it is
//              full) for more records; point fill at a free slot (later callers append there);
//              unlock; launch the kernel on the slot in place and record the slot's event; hand the
//              queue to one caller of the new open slot (the next leader, whose launch then queues
//              behind this one on the stream); wait for the event; mark the slot DONE; wake its
//              callers
//            else sleep on the slot's condition variable
//            copy its own result out of the slot; the last reader frees the slot
//
// Four slots per queue: one filling, up to two on the GPU, one draining (callers copying out).  The
// kernels read their inputs from and write their outputs to the pinned slot directly (host memory
// allocated with hipHostMalloc is mapped into the device's address space), so a batch is one
// launch plus one hipStreamSynchronize and no copies.  The encode and decode queues each own a
// sym_ctx (only the current leader uses it) and a non-blocking stream.
//
// Records up to kRingRecordMax bytes (every kv / echo request an RPC carries in practice) take the
// ring instead (record_worker.hip): no launch per record or batch, one persistent launch (four
// workgroups) per device -- shared by every batcher on the device and both directions, each slot carrying
// its record's direction and layout -- serving tickets in place in coherent pinned slots; a record is
// published with one store, served within a few microseconds, and read back as soon as its own flag
// is set.  ONE worker per device, however many batchers: a persistent kernel holds the hardware queue
// its stream maps to (GPU_MAX_HW_QUEUES, 4 by default), and a launch of another stream on that queue
// waits behind it -- two persistent workers whose streams share a queue serve in turns of their idle
// timeout (measured: 40 ms per record, DESIGN.md section 4, per-record path).  The worker also hands
// over to a fresh launch every kLifeTicks (2 ms), busy or idle, so such a launch (a batch of large
// records, a caller's own kernels) waits at most that long.  Larger records keep the batched path
// above.  Both give the same bytes and statuses.
#include <hip/hip_runtime.h>

#include <immintrin.h>
#include <sched.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>

#include "../../include/symphony_hip.h"
#include "codec.hpp"
#include "ctx.hpp"
#include "record_worker.hpp"

using namespace symhip::capi;
using symhip::Layout;

namespace {

using Clock = std::chrono::steady_clock;
constexpr int kBSlots = 4;
enum SlotState { kFree = 0, kClosed = 1, kRunning = 2, kDone = 3 };

struct BSlot {
    char* pin = nullptr;  // hipHostMalloc'd: the kernels read and write it in place
    // encode: inputs fixed / offs / bytes, outputs rec (stream) / rec_off (the IDs are patched at copy-out)
    // decode: inputs rec / rec_off, outputs status / fixed / offs / bytes
    int32_t* fixed[symhip::kMaxFixed] = {};
    uint64_t* offs[symhip::kMaxVar] = {};
    uint8_t* bytes[symhip::kMaxVar] = {};
    uint8_t* rec = nullptr;
    uint64_t* rec_off = nullptr;
    uint8_t* status = nullptr;
    uint64_t n = 0;
    uint64_t used = 0;  // record bytes in the batch (encode: encoded sizes; decode: input bytes)
    int state = kFree;
    uint64_t readers = 0;  // callers of the batch still to copy out
    int rc = SYM_OK;
    char msg[256] = "";
    Clock::time_point first;
    hipEvent_t ev = nullptr;     // the slot's batch has finished on the GPU
    std::condition_variable cv;  // the slot's callers: DONE, or "lead me"
};

// The ring of one device and direction (record_worker.hpp): coherent mapped pinned memory (the
// callers' ticket counter in it) and the worker's generation (relaunched under `mu` when one has
// exited).
struct Ring {
    int device = 0;
    symhip::RingCtl* ctl = nullptr;
    uint8_t* slots = nullptr;
    unsigned* exits = nullptr;  // device word: the worker's groups count their exits on it
    std::atomic<uint64_t> gen{0};
    std::mutex mu;
    hipStream_t stream = nullptr;
};

// A device's ring, the batchers using it and their ids.
struct DevRings {
    int refs = 0;
    bool id_used[symhip::kMaxBatchers] = {};
    Ring* ring = nullptr;
};

constexpr int kMaxDevices = 64;
std::mutex g_rings_mu;  // g_rings and every DevRings' refs / id_used
DevRings g_rings[kMaxDevices];

struct Queue {
    sym_ctx* ctx = nullptr;
    hipStream_t stream = nullptr;
    std::mutex mu;
    std::condition_variable cv_space;  // callers waiting for room / a leader waiting for a free slot
    BSlot slot[kBSlots];
    int fill = 0;
    bool busy = false;  // a leader owns the queue (waiting for records or launching a batch)
    uint64_t batches = 0, records = 0;
};

}  // namespace

struct sym_batcher {
    int device = 0;
    int schema = 0;
    Layout lay{};
    uint64_t ovh = 0;
    uint64_t R = 0;  // records per batch
    uint64_t B = 0;  // record bytes per batch
    uint32_t wait_us = 0;
    Queue q[2];      // 0 encode, 1 decode
    Ring* ring[2] = {};    // per direction, the device's ring (the same one): records up to kRingRecordMax bytes
    int bid = -1;          // this batcher's id on the ring (its records' kind; its pass counters)
    uint64_t pass_base[2] = {};  // the ring's pass counters of this id when the batcher took it
    std::atomic<uint64_t> ring_recs[2] = {};  // this batcher's ring records per direction
};

namespace {

size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

// Carve a slot's pinned buffer.  Column and stream regions get 16 bytes of slack: the kernels may
// read up to the 16-byte boundary past a column's last byte.
int slot_alloc(sym_batcher* b, int dir, BSlot& s) {
    const uint64_t R = b->R, B = b->B;
    const Layout& L = b->lay;
    size_t o = 0;
    size_t at_fixed[symhip::kMaxFixed], at_offs[symhip::kMaxVar], at_bytes[symhip::kMaxVar];
    for (int f = 0; f < L.nfixed; ++f) at_fixed[f] = o, o = a256(o + 4 * R);
    for (int f = 0; f < L.nvar; ++f) at_offs[f] = o, o = a256(o + 8 * (R + 1));
    for (int f = 0; f < L.nvar; ++f) at_bytes[f] = o, o = a256(o + B + 16);
    const size_t at_rec = o;
    o = a256(o + B + 16);
    const size_t at_roff = o;
    o = a256(o + 8 * (R + 1));
    const size_t at_status = o;
    o = a256(o + R);
    hipError_t e = hipHostMalloc((void**)&s.pin, o, hipHostMallocDefault);
    if (e != hipSuccess) return fail(SYM_ERR_NOMEM, "sym_batcher_create: %zu pinned bytes: %s", o, hipGetErrorString(e));
    memset(s.pin, 0, o);
    for (int f = 0; f < L.nfixed; ++f) s.fixed[f] = (int32_t*)(s.pin + at_fixed[f]);
    for (int f = 0; f < L.nvar; ++f) {
        s.offs[f] = (uint64_t*)(s.pin + at_offs[f]);
        s.bytes[f] = (uint8_t*)(s.pin + at_bytes[f]);
    }
    s.rec = (uint8_t*)(s.pin + at_rec);
    s.rec_off = (uint64_t*)(s.pin + at_roff);
    s.status = (uint8_t*)(s.pin + at_status);
    (void)dir;
    return SYM_OK;
}

void slot_reset(BSlot& s, int nvar) {
    s.n = 0;
    s.used = 0;
    s.rc = SYM_OK;
    s.msg[0] = 0;
    s.rec_off[0] = 0;
    for (int f = 0; f < nvar; ++f) s.offs[f][0] = 0;
}

// One batch on the GPU, in place in its pinned slot; the slot's event marks its end.
int launch_batch(sym_batcher* b, int dir, BSlot& s) {
    Queue& q = b->q[dir];
    DeviceGuard g(b->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "sym_batcher: hipSetDevice");
    int rc;
    if (dir == 0) {
        const int32_t* fx[symhip::kMaxFixed] = {s.fixed[0], s.fixed[1]};
        const uint8_t* by[symhip::kMaxVar] = {s.bytes[0], s.bytes[1]};
        const uint64_t* of[symhip::kMaxVar] = {s.offs[0], s.offs[1]};
        rc = encode_call(q.ctx, b->schema, s.n, fx, by, of, 0, 0, s.rec, s.rec_off, 0, q.stream);
    } else {
        const uint64_t caps[symhip::kMaxVar] = {s.used, s.used};  // a column never holds more than the stream
        rc = decode_call("sym_batcher_decode_one", q.ctx, b->lay, nullptr, s.n, s.rec, s.rec_off, s.fixed, s.bytes,
                         caps, s.offs, s.status, q.stream);
    }
    if (rc != SYM_OK) return rc;
    // The kernels cannot raise device error bits here: a batch's record bytes are bounded by
    // max_bytes (< 2 GiB per tile) and every decode column's capacity is the batch's stream size.
    hipError_t e = hipEventRecord(s.ev, q.stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "sym_batcher: hipEventRecord");
}

// The calling thread runs the open batch of queue `dir` (q.busy set by the caller).  Entered and
// left with q.mu held.
void lead(sym_batcher* b, int dir, std::unique_lock<std::mutex>& lk) {
    Queue& q = b->q[dir];
    BSlot& s = q.slot[q.fill];
    if (b->wait_us) {  // let the batch grow until full or until its first record has waited long enough
        const Clock::time_point due = s.first + std::chrono::microseconds(b->wait_us);
        while (s.state == kFree && Clock::now() < due) s.cv.wait_until(lk, due);
    }
    int next = -1;  // the next slot to fill: one whose callers have all copied out
    while (next < 0) {
        for (int k = 1; k < kBSlots && next < 0; ++k) {
            const int c = (q.fill + k) % kBSlots;
            if (q.slot[c].state == kFree) next = c;
        }
        if (next < 0) q.cv_space.wait(lk);
    }
    slot_reset(q.slot[next], b->lay.nvar);
    q.fill = next;
    s.state = kRunning;
    q.cv_space.notify_all();
    lk.unlock();
    int rc = launch_batch(b, dir, s);
    lk.lock();
    q.busy = false;  // the next batch may launch now (it queues behind this one on the stream)
    q.slot[q.fill].cv.notify_one();
    lk.unlock();
    if (rc == SYM_OK) {
        DeviceGuard g(b->device);
        const hipError_t e = hipEventSynchronize(s.ev);
        if (e != hipSuccess) rc = hip_fail(e, "sym_batcher: hipEventSynchronize");
    }
    char msg[256] = "";
    if (rc != SYM_OK) snprintf(msg, sizeof(msg), "%s", sym_last_error());
    lk.lock();
    s.rc = rc;
    memcpy(s.msg, msg, sizeof(msg));
    s.readers = s.n;
    s.state = kDone;
    ++q.batches;
    q.records += s.n;
    s.cv.notify_all();
}

// Append under q.mu: wait for room in the open slot (closing a full one), return it.
BSlot* reserve(sym_batcher* b, Queue& q, std::unique_lock<std::mutex>& lk, uint64_t bytes) {
    for (;;) {
        BSlot& s = q.slot[q.fill];
        if (s.state == kFree && s.n < b->R && s.used + bytes <= b->B) return &s;
        if (s.state == kFree && s.n > 0) {  // full for this record: close it (its leader stops waiting)
            s.state = kClosed;
            s.cv.notify_all();
        }
        q.cv_space.wait(lk);
    }
}

// After the append: lead the batch or wait for it; return (q.mu held) with the slot DONE.
void await(sym_batcher* b, int dir, std::unique_lock<std::mutex>& lk, BSlot& s) {
    Queue& q = b->q[dir];
    if (s.n == 1) s.first = Clock::now();
    if (s.n == b->R) {
        s.state = kClosed;
        s.cv.notify_all();
    }
    while (s.state != kDone) {
        if (!q.busy && &q.slot[q.fill] == &s) {
            q.busy = true;
            lead(b, dir, lk);
            continue;
        }
        s.cv.wait(lk);
    }
}

void release(Queue& q, std::unique_lock<std::mutex>& lk, BSlot& s) {
    lk.lock();
    if (--s.readers == 0) {
        s.state = kFree;
        q.cv_space.notify_all();
    }
}

// ---- the ring path (record_worker.hip) ----
int ring_launch(Ring& r, uint64_t gen) {
    DeviceGuard g(r.device);
    if (g.err != hipSuccess) return hip_fail(g.err, "sym_batcher: hipSetDevice");
    hipError_t e = symhip::launch_record_worker(r.ctl, r.slots, r.exits, gen, r.stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "sym_batcher: record worker launch");
}

// Tell the worker to leave and wait until it has (r.mu held or no caller active); the next call
// relaunches it.
void ring_stop(Ring& r) {
    if (!r.ctl || !r.stream) return;
    __atomic_store_n(&r.ctl->stop, 1, __ATOMIC_SEQ_CST);
    {
        DeviceGuard g(r.device);
        (void)hipStreamSynchronize(r.stream);
    }
    __atomic_store_n(&r.ctl->stop, 0, __ATOMIC_SEQ_CST);
}

void ring_destroy(Ring* r) {
    ring_stop(*r);
    DeviceGuard g(r->device);
    if (r->stream) (void)hipStreamDestroy(r->stream);
    if (r->slots) (void)hipHostFree(r->slots);
    if (r->ctl) (void)hipHostFree(r->ctl);
    if (r->exits) (void)hipFree(r->exits);
    delete r;
}

int ring_create(int device, Ring** out) {
    Ring* r = new (std::nothrow) Ring;
    if (!r) return fail(SYM_ERR_NOMEM, "sym_batcher_create: out of host memory");
    r->device = device;
    DeviceGuard g(device);
    if (g.err != hipSuccess) {
        delete r;
        return hip_fail(g.err, "sym_batcher_create: hipSetDevice");
    }
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    hipError_t e = hipHostMalloc((void**)&r->ctl, sizeof(symhip::RingCtl), fl);
    if (e == hipSuccess) e = hipHostMalloc((void**)&r->slots, (size_t)symhip::kRingSlots * symhip::kSlotBytes, fl);
    if (e != hipSuccess) {
        ring_destroy(r);
        return fail(SYM_ERR_NOMEM, "sym_batcher_create: ring of %d slots: %s", symhip::kRingSlots, hipGetErrorString(e));
    }
    if (e == hipSuccess && (e = hipMalloc((void**)&r->exits, sizeof(unsigned))) == hipSuccess)
        e = hipMemset(r->exits, 0, sizeof(unsigned));
    if (e != hipSuccess) {
        ring_destroy(r);
        return hip_fail(e, "sym_batcher_create: worker exit counter");
    }
    memset(r->ctl, 0, sizeof(symhip::RingCtl));
    for (int w = 0; w < symhip::kGroups; ++w) r->ctl->e[w] = (uint64_t)w;  // group w's first ticket
    memset(r->slots, 0, (size_t)symhip::kRingSlots * symhip::kSlotBytes);
    for (int k = 0; k < symhip::kRingSlots; ++k)
        ((symhip::SlotCtl*)(r->slots + (size_t)k * symhip::kSlotBytes))->turn = (uint64_t)k;
    if ((e = hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking)) != hipSuccess) {
        ring_destroy(r);
        return hip_fail(e, "sym_batcher_create: worker stream");
    }
    r->gen = 1;
    const int rc = ring_launch(*r, 1);
    if (rc != SYM_OK) {
        ring_destroy(r);
        return rc;
    }
    *out = r;
    return SYM_OK;
}

// Worker passes that served records of batcher id `bid` in direction `dir` (both groups).
uint64_t ring_passes(const Ring& r, int bid, int dir) {
    uint64_t v = 0;
    for (int w = 0; w < symhip::kGroups; ++w) v += __atomic_load_n(&r.ctl->bpasses[w][bid][dir], __ATOMIC_ACQUIRE);
    return v;
}

// The device's ring, created with its first batcher, and an id on it for batcher b.  The id's pass
// counters are the worker's to write; the batcher counts from their value now (every record of the
// id's previous owner was done before that batcher was destroyed; its pass's counter store follows
// within microseconds).
int ring_acquire(sym_batcher* b, int device) {
    if (device < 0 || device >= kMaxDevices) return fail(SYM_ERR_INVALID, "sym_batcher_create: device %d", device);
    std::lock_guard<std::mutex> lk(g_rings_mu);
    DevRings& d = g_rings[device];
    if (!d.ring) {
        const int rc = ring_create(device, &d.ring);
        if (rc != SYM_OK) return rc;
    }
    int id = 0;
    while (id < symhip::kMaxBatchers && d.id_used[id]) ++id;
    if (id == symhip::kMaxBatchers)
        return fail(SYM_ERR_INVALID, "sym_batcher_create: %d batchers on device %d already", symhip::kMaxBatchers, device);
    d.id_used[id] = true;
    ++d.refs;
    b->bid = id;
    for (int dir = 0; dir < 2; ++dir) {
        b->ring[dir] = d.ring;
        b->pass_base[dir] = ring_passes(*d.ring, id, dir);
    }
    return SYM_OK;
}

// The device's last batcher stops the worker and frees the ring.
void ring_release(int device, int bid) {
    std::lock_guard<std::mutex> lk(g_rings_mu);
    DevRings& d = g_rings[device];
    d.id_used[bid] = false;
    if (--d.refs > 0) return;
    if (d.ring) ring_destroy(d.ring);
    d.ring = nullptr;
}

// After a record is published: a worker that announced its exit (ctl->quit == its generation) is
// replaced once it has gone.  `waited`: the caller has waited long for its record -- a worker whose
// launch ended without serving it is replaced as well (a safety net: the announced exit serves every
// record it owes, record_worker.hip).
int ring_ensure_worker(Ring& r, bool waited) {
    const uint64_t gen = r.gen.load(std::memory_order_acquire);
    const uint64_t q = __atomic_load_n(&r.ctl->quit, __ATOMIC_SEQ_CST);
    bool gone = __atomic_load_n(&r.ctl->gone, __ATOMIC_ACQUIRE) == gen;
    if (q != gen && !gone && !waited) return SYM_OK;
    std::lock_guard<std::mutex> lk(r.mu);
    if (r.gen.load(std::memory_order_acquire) != gen) return SYM_OK;  // another caller relaunched it
    if (!gone && waited && q != gen) {  // a long wait: has the worker's launch ended anyway?
        DeviceGuard g(r.device);
        const hipError_t e = hipStreamQuery(r.stream);
        if (e == hipErrorNotReady) return SYM_OK;
        if (e != hipSuccess) return hip_fail(e, "sym_batcher: record worker");
        gone = true;
    }
    // announced: it serves what it owes, then leaves.  A launch that ended without storing `gone`
    // (a fault, an abort) must not hang every batcher of the device here: every few thousand spins the
    // stream is asked whether the launch is over (done: treat it as gone; an error: report it).
    for (uint64_t i = 0; !gone; ++i) {
        if (i < 256) {
            _mm_pause();
        } else {
            sched_yield();
            if ((i & 4095) == 0) {
                DeviceGuard g(r.device);
                const hipError_t e = hipStreamQuery(r.stream);
                if (e == hipSuccess) break;
                if (e != hipErrorNotReady) return hip_fail(e, "sym_batcher: record worker");
            }
        }
        gone = __atomic_load_n(&r.ctl->gone, __ATOMIC_ACQUIRE) == gen;
    }
    r.gen.store(gen + 1, std::memory_order_release);
    return ring_launch(r, gen + 1);
}

// Spin until *p == want (a pause first, then yielding the CPU: there may be more callers than cores);
// every ~10 ms make sure a worker runs.
int ring_wait(Ring& r, const uint64_t* p, uint64_t want) {
    for (uint64_t i = 0; __atomic_load_n(p, __ATOMIC_ACQUIRE) != want; ++i) {
        if (i < 256) {
            _mm_pause();
            continue;
        }
        sched_yield();
        if ((i & 4095) == 0) {
            const int rc = ring_ensure_worker(r, true);
            if (rc != SYM_OK) return rc;
        }
    }
    return SYM_OK;
}

// One record through the ring: take a ticket and its slot, `fill` the in area, publish, wait for the
// worker, `drain` the out area, free the slot.
template <typename Fill, typename Drain>
int ring_call(sym_batcher* b, int dir, uint64_t in_len, Fill&& fill, Drain&& drain) {
    Ring& r = *b->ring[dir];
    const uint64_t t = __atomic_fetch_add(&r.ctl->ticket, 1, __ATOMIC_SEQ_CST);
    uint8_t* slot = r.slots + (size_t)(t % symhip::kRingSlots) * symhip::kSlotBytes;
    symhip::SlotCtl* sc = (symhip::SlotCtl*)slot;
    int rc = ring_wait(r, &sc->turn, t);
    if (rc != SYM_OK) return rc;
    fill(slot + symhip::kSlotInAt);
    sc->in_len = in_len | symhip::slot_tag(t) | symhip::slot_kind(dir, b->lay, b->bid);
    __atomic_store_n(&sc->req, t + 1, __ATOMIC_RELEASE);
    __atomic_fetch_add(&r.ctl->posted[t % symhip::kGroups], 1, __ATOMIC_SEQ_CST);  // then look at quit (hand-shake)
    rc = ring_ensure_worker(r, false);
    if (rc == SYM_OK) rc = ring_wait(r, &sc->done, t + 1);
    if (rc != SYM_OK) return rc;  // (the slot stays taken: the device failed)
    drain(slot + symhip::kSlotOutAt);
    __atomic_store_n(&sc->turn, t + symhip::kRingSlots, __ATOMIC_RELEASE);
    b->ring_recs[dir].fetch_add(1, std::memory_order_relaxed);
    return SYM_OK;
}

void destroy_queue(Queue& q) {
    if (q.stream) (void)hipStreamDestroy(q.stream);
    for (BSlot& s : q.slot) {
        if (s.pin) (void)hipHostFree(s.pin);
        if (s.ev) (void)hipEventDestroy(s.ev);
    }
    if (q.ctx) (void)sym_ctx_destroy(q.ctx);
}

}  // namespace

extern "C" {

int sym_batcher_create(int device, int schema, uint32_t max_records, uint64_t max_bytes, uint32_t max_wait_us,
                       sym_batcher** out) {
    if (!out) return fail(SYM_ERR_INVALID, "sym_batcher_create: out is NULL");
    *out = nullptr;
    if (!schema_ok(schema)) return fail(SYM_ERR_INVALID, "sym_batcher_create: unknown schema %d", schema);
    if (max_records == 0 || max_bytes < 64 || max_bytes > (1ull << 30))
        return fail(SYM_ERR_INVALID, "sym_batcher_create: max_records >= 1 and max_bytes in [64, 2^30] required");
    sym_batcher* b = new (std::nothrow) sym_batcher;
    if (!b) return fail(SYM_ERR_NOMEM, "sym_batcher_create: out of host memory");
    b->device = device;
    b->schema = schema;
    b->lay = kLayouts[schema];
    b->ovh = sym_record_overhead(schema);
    b->R = max_records;
    b->B = max_bytes;
    b->wait_us = max_wait_us;
    int rc = SYM_OK;
    for (int dir = 0; dir < 2 && rc == SYM_OK; ++dir) {
        Queue& q = b->q[dir];
        rc = sym_ctx_create(device, &q.ctx);
        if (rc != SYM_OK) break;
        DeviceGuard g(device);
        hipError_t e = hipStreamCreateWithFlags(&q.stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            rc = hip_fail(e, "sym_batcher_create: stream");
            break;
        }
        if (dir == 1 && (rc = sym_ctx_reserve(q.ctx, b->R)) != SYM_OK) break;
        for (int k = 0; k < kBSlots && rc == SYM_OK; ++k) {
            rc = slot_alloc(b, dir, q.slot[k]);
            if (rc == SYM_OK && (e = hipEventCreateWithFlags(&q.slot[k].ev, hipEventDisableTiming)) != hipSuccess)
                rc = hip_fail(e, "sym_batcher_create: event");
        }
        if (rc != SYM_OK) break;
        for (BSlot& s : q.slot) slot_reset(s, b->lay.nvar);
    }
    if (rc == SYM_OK) rc = ring_acquire(b, device);
    if (rc != SYM_OK) {
        sym_batcher_destroy(b);
        return rc;
    }
    *out = b;
    return SYM_OK;
}

int sym_batcher_destroy(sym_batcher* b) {
    if (!b) return SYM_OK;
    if (b->bid >= 0) ring_release(b->device, b->bid);
    for (Queue& q : b->q) destroy_queue(q);
    delete b;
    return SYM_OK;
}

int sym_batcher_encode_one(sym_batcher* b, const int32_t* fixed, const uint8_t* const* fields, const uint64_t* lens,
                           uint32_t service_id, uint32_t method_id, uint8_t* out, uint64_t out_cap,
                           uint64_t* out_len) {
    if (!b || !out_len) return fail(SYM_ERR_INVALID, "sym_batcher_encode_one: NULL batcher or out_len");
    const Layout& L = b->lay;
    if ((L.nfixed && !fixed) || (L.nvar && (!fields || !lens)))
        return fail(SYM_ERR_INVALID, "sym_batcher_encode_one: NULL field argument");
    uint64_t var = 0;
    for (int f = 0; f < L.nvar; ++f) {
        if (lens[f] && !fields[f]) return fail(SYM_ERR_INVALID, "sym_batcher_encode_one: field %d is NULL", f);
        if (lens[f] > b->B) return fail(SYM_ERR_INVALID, "sym_batcher_encode_one: field %d exceeds max_bytes", f);
        var += lens[f];
    }
    const uint64_t size = b->ovh + var;
    *out_len = size;
    if (size > b->B) return fail(SYM_ERR_INVALID, "sym_batcher_encode_one: a %llu-byte record exceeds max_bytes",
                                 (unsigned long long)size);
    if (!out || out_cap < size) return fail(SYM_ERR_CAPACITY, "sym_batcher_encode_one: out needs %llu bytes",
                                            (unsigned long long)size);
    if (var <= symhip::kRingRecordMax) {  // the ring: the worker writes the record, IDs included
        return ring_call(
            b, 0, var,
            [&](uint8_t* in) {
                symhip::EncIn* h = (symhip::EncIn*)in;
                for (int f = 0; f < symhip::kMaxFixed; ++f) h->fixed[f] = f < L.nfixed ? fixed[f] : 0;
                h->service_id = service_id;
                h->method_id = method_id;
                uint8_t* p = in + sizeof(symhip::EncIn);
                for (int f = 0; f < symhip::kMaxVar; ++f) {
                    h->len[f] = f < L.nvar ? lens[f] : 0;
                    if (f < L.nvar && lens[f]) memcpy(p, fields[f], lens[f]);
                    p += f < L.nvar ? lens[f] : 0;
                }
            },
            [&](const uint8_t* o) { memcpy(out, o, size); });
    }
    Queue& q = b->q[0];
    std::unique_lock<std::mutex> lk(q.mu);
    BSlot& s = *reserve(b, q, lk, size);
    const uint64_t i = s.n++;
    for (int f = 0; f < L.nfixed; ++f) s.fixed[f][i] = fixed[f];
    for (int f = 0; f < L.nvar; ++f) {
        const uint64_t at = s.offs[f][i];
        if (lens[f]) memcpy(s.bytes[f] + at, fields[f], lens[f]);
        s.offs[f][i + 1] = at + lens[f];
    }
    s.used += size;
    await(b, 0, lk, s);
    const int rc = s.rc;
    char msg[256];
    memcpy(msg, s.msg, sizeof(msg));
    lk.unlock();
    if (rc == SYM_OK) {
        const uint8_t* src = s.rec + s.rec_off[i];
        memcpy(out, src, size);
        if (service_id || method_id) {  // the client's patch of bytes [5:13] (pkg/rpc/client.go:267-271)
            for (int k = 0; k < 4; ++k) {
                out[5 + k] = (uint8_t)(service_id >> (8 * k));
                out[9 + k] = (uint8_t)(method_id >> (8 * k));
            }
        }
    }
    release(q, lk, s);
    return rc == SYM_OK ? SYM_OK : fail(rc, "%s", msg);
}

int sym_batcher_decode_one(sym_batcher* b, const uint8_t* data, uint64_t len, int32_t* fixed, uint8_t* const* fields,
                           const uint64_t* caps, uint64_t* lens, uint8_t* status) {
    if (!b || !status) return fail(SYM_ERR_INVALID, "sym_batcher_decode_one: NULL batcher or status");
    const Layout& L = b->lay;
    if ((len && !data) || (L.nfixed && !fixed) || (L.nvar && (!fields || !caps || !lens)))
        return fail(SYM_ERR_INVALID, "sym_batcher_decode_one: NULL argument");
    if (len > b->B) return fail(SYM_ERR_INVALID, "sym_batcher_decode_one: a %llu-byte record exceeds max_bytes",
                                (unsigned long long)len);
    if (len <= symhip::kRingRecordMax) {
        bool short_cap = false;
        const int rc = ring_call(
            b, 1, len, [&](uint8_t* in) { if (len) memcpy(in, data, len); },
            [&](const uint8_t* o) {
                const symhip::DecOut* d = (const symhip::DecOut*)o;
                *status = (uint8_t)d->status;
                for (int f = 0; f < L.nfixed; ++f) fixed[f] = d->fixed[f];
                for (int f = 0; f < L.nvar; ++f) {
                    lens[f] = d->len[f];
                    const uint64_t c = lens[f] < caps[f] ? lens[f] : caps[f];
                    short_cap |= c < lens[f];
                    if (c) memcpy(fields[f], o + symhip::kDecData + (f ? d->at1 : 0), c);
                }
            });
        if (rc != SYM_OK) return rc;
        return short_cap ? fail(SYM_ERR_CAPACITY, "sym_batcher_decode_one: a field exceeds its cap") : SYM_OK;
    }
    Queue& q = b->q[1];
    std::unique_lock<std::mutex> lk(q.mu);
    BSlot& s = *reserve(b, q, lk, len);
    const uint64_t i = s.n++;
    const uint64_t at = s.rec_off[i];
    if (len) memcpy(s.rec + at, data, len);
    s.rec_off[i + 1] = at + len;
    s.used += len;
    await(b, 1, lk, s);
    const int rc = s.rc;
    char msg[256];
    memcpy(msg, s.msg, sizeof(msg));
    lk.unlock();
    bool short_cap = false;
    if (rc == SYM_OK) {
        *status = s.status[i];
        for (int f = 0; f < L.nfixed; ++f) fixed[f] = s.fixed[f][i];
        for (int f = 0; f < L.nvar; ++f) {
            const uint64_t a = s.offs[f][i], z = s.offs[f][i + 1];
            lens[f] = z - a;
            const uint64_t c = lens[f] < caps[f] ? lens[f] : caps[f];
            short_cap |= c < lens[f];
            if (c) memcpy(fields[f], s.bytes[f] + a, c);
        }
    }
    release(q, lk, s);
    if (rc != SYM_OK) return fail(rc, "%s", msg);
    return short_cap ? fail(SYM_ERR_CAPACITY, "sym_batcher_decode_one: a field exceeds its cap") : SYM_OK;
}

int sym_batcher_stats(sym_batcher* b, uint64_t* enc_batches, uint64_t* enc_records, uint64_t* dec_batches,
                      uint64_t* dec_records) {
    if (!b) return fail(SYM_ERR_INVALID, "sym_batcher_stats: NULL batcher");
    uint64_t v[4];
    for (int dir = 0; dir < 2; ++dir) {  // batches: the batched path's launches + the ring worker's passes
        std::lock_guard<std::mutex> lk(b->q[dir].mu);
        const Ring* r = b->ring[dir];
        const uint64_t passes = r ? ring_passes(*r, b->bid, dir) : 0;
        v[2 * dir] = b->q[dir].batches + (r ? passes - b->pass_base[dir] : 0);
        v[2 * dir + 1] = b->q[dir].records + b->ring_recs[dir].load(std::memory_order_relaxed);
    }
    if (enc_batches) *enc_batches = v[0];
    if (enc_records) *enc_records = v[1];
    if (dec_batches) *dec_batches = v[2];
    if (dec_records) *dec_records = v[3];
    return SYM_OK;
}

int sym_batcher_quiesce(sym_batcher* b) {
    if (!b || !b->ring[0]) return fail(SYM_ERR_INVALID, "sym_batcher_quiesce: NULL batcher");
    std::lock_guard<std::mutex> lk(b->ring[0]->mu);  // no relaunch meanwhile
    ring_stop(*b->ring[0]);
    return SYM_OK;
}

}  // extern "C"
