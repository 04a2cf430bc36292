// record_worker.hpp -- the ring of record slots shared by batcher.cpp (host) and record_worker.hip
// (the persistent per-record worker).  One ring and one worker per device, shared by every batcher
// on it and both directions: each slot says what it holds (slot_kind).  All of it lives in pinned host memory allocated coherent and
// mapped (hipHostMallocCoherent | hipHostMallocMapped): the callers write and read it with plain
// stores / loads and C11 atomics, the worker with system-scope 8-byte atomics.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "codec.hpp"

namespace symhip {

constexpr int kRingSlots = 256;            // tickets in flight per device ring (= the worker's window)
constexpr size_t kSlotBytes = 16384;       // one slot: control words, in area, out area
constexpr size_t kSlotInAt = 64;
constexpr size_t kSlotIn = 4096 - 64;      // in area bytes
constexpr size_t kSlotOutAt = 4096;
constexpr size_t kSlotOut = kSlotBytes - kSlotOutAt;
constexpr uint64_t kRingRecordMax = 4000;  // records (encode: field bytes; decode: record bytes) up to
                                           // this go through the ring; larger ones through batches
constexpr uint64_t kIdleTicks = 2000000;   // 20 ms without a record (s_memrealtime, 100 MHz): the worker exits
constexpr int kMaxBatchers = 256;         // batchers per device ring (their pass counters)
constexpr int kGroups = 4;                 // worker workgroups of one launch: group w serves tickets t % kGroups == w
constexpr uint64_t kLifeTicks = 200000;    // 2 ms: a busy worker hands over to a fresh launch, so work queued
                                           // behind it on a shared hardware queue waits at most this long

struct RingCtl {          // one per device, written as commented
    uint64_t posted[kGroups];  // callers: records published so far per ticket class t % kGroups (atomic add
                               // after the slot's req store)
    uint64_t stop;        // host: leave now (last sym_batcher_destroy of the device, sym_batcher_quiesce)
    uint64_t quit;        // worker: the generation that is about to exit (0: none)
    uint64_t gone;        // worker: the generation that has exited (its last group)
    uint64_t e[kGroups], nproc[kGroups];  // worker group, at exit: its window base and records served
    uint64_t served[kGroups];  // worker group: records served so far, every pass
    uint64_t passes[kGroups];  // worker group: passes that served records, every pass
    uint64_t ticket;      // callers: the next ticket (atomic fetch-add); the worker reads it when it
                          // announces its exit: every record it still owes has a smaller ticket
    uint64_t bpasses[kGroups][kMaxBatchers][2];  // worker group: passes that served records of batcher id b,
                                                 // direction d (stored after those records' done flags)
};

// A record's kind, in the high half of SlotCtl::in_len: direction (0 encode, 1 decode), layout and
// the batcher's id on the ring.
constexpr uint64_t slot_kind(int dir, Layout lay, int bid) {
    return ((uint64_t)dir | ((uint64_t)lay.nfixed << 8) | ((uint64_t)lay.nvar << 16) | ((uint64_t)bid << 24)) << 32;
}
// The low half of SlotCtl::in_len: the length (< 2^16, at most kRingRecordMax) in bits 0..15 and the
// ticket's low 16 bits in bits 16..31.  The worker reads req and in_len with one 16-byte load and
// takes the slot only when both name the same ticket, so a load that the fabric split into two
// 8-byte reads cannot pair a new req with the previous ticket's length and kind.
constexpr uint64_t kSlotLenMask = 0xffff;
constexpr uint64_t slot_tag(uint64_t ticket) { return (ticket & 0xffff) << 16; }

struct SlotCtl {          // the first 64 bytes of a slot
    uint64_t req;         // caller: ticket + 1 once the in area is written
    uint64_t in_len;      // caller: low half encode: field bytes after EncIn, decode: record bytes; high
                          // half slot_kind() (next to req: the worker reads both with one 16-byte load)
    uint64_t done;        // worker: ticket + 1 once the out area is written
    uint64_t turn;        // caller: the ticket that may use the slot next
    uint64_t pad[4];
};
static_assert(offsetof(SlotCtl, in_len) == 8, "req and in_len in one 16-byte load");
static_assert(kRingRecordMax <= kSlotLenMask, "the length fits below the ticket tag");

struct EncIn {            // encode in area: the record's scalars, then its var fields' bytes back to back
    int32_t fixed[kMaxFixed];
    uint32_t service_id, method_id;
    uint64_t len[kMaxVar];
};
static_assert(sizeof(EncIn) == 32, "EncIn layout");

struct DecOut {           // decode out area: the parse, then field 0's bytes at kDecData, field 1's at
    uint32_t status;      // kDecData + at1
    int32_t fixed[kMaxFixed];
    uint32_t pad;
    uint64_t len[kMaxVar];
    uint64_t at1;
};
constexpr size_t kDecData = 64;
static_assert(sizeof(DecOut) <= kDecData, "DecOut layout");
// decode out area bound: header + two fields of up to a record's bytes each (a malformed record may
// point both at the same bytes), 16-byte rounded
static_assert(kDecData + 2 * (kRingRecordMax + 16) <= kSlotOut, "decode out area");
static_assert(sizeof(EncIn) + kRingRecordMax <= kSlotIn, "encode in area");

// exits: a device word the worker's groups count their exits on (zero between launches)
hipError_t launch_record_worker(RingCtl* ctl, uint8_t* slots, unsigned* exits, uint64_t gen, hipStream_t stream);

}  // namespace symhip
