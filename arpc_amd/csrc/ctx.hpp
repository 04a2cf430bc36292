// ctx.hpp -- the sym_ctx object behind the C ABI and the helpers capi.cpp and host.cpp share.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/symphony_hip.h"
#include "codec.hpp"

namespace symhip {
namespace host {
constexpr int kSlots = 3;  // chunks in flight in the host-memory entry points
// One in-flight chunk of a *_host call: its events, device buffers and pinned staging.
struct Slot {
    hipEvent_t done = nullptr;    // the chunk's last D2H
    hipEvent_t kernel = nullptr;  // the chunk's kernels (on the H2D stream, in chunk order)
    void* dev = nullptr;
    size_t dev_bytes = 0;
    void* pin = nullptr;  // pinned staging for pageable caller memory (inputs, then outputs)
    size_t pin_bytes = 0;
};
}  // namespace host
}  // namespace symhip

struct sym_ctx {
    int device = 0;
    void* ws = nullptr;  // three-kernel decode workspace
    size_t ws_bytes = 0;
    void* flags = nullptr;  // default decode's aggregate / prefix words (epoch-tagged)
    size_t flag_bytes = 0;
    unsigned epoch = 0;     // tag of the last decode call's look-back words
    unsigned* err = nullptr;  // [0] device error word (kErr* bits); [1] unused; [2..3] the decode's
                              // speculation hold (decode_pipe.hip spec_held), [4..5] its tile-key
                              // hold (spec_tile_held), u64 call numbers; [6..7] the gate's re-decode
                              // count (sym_ctx_decode_redos)
    // scan workspace of the packetizer, the field getters, the flat decode and the mixed encode
    // (stream-ordered, so calls on one stream share it)
    void* frag = nullptr;
    size_t frag_bytes = 0;
    // segment cipher: device key schedule + GHASH tables of the last key pair, and that pair
    void* crypt_tables = nullptr;
    uint8_t crypt_keys[64] = {0};
    int num_cus = 0;
    int decode_impl = SYM_DECODE_PIPELINE;
    uint64_t decode_seq = 0;  // decode calls so far (DecodeParams::seq): the speculation hold counts them
    int encode_impl = 0;  // SYM_ENCODE_* (mixed batches' size scan)
    // reassembly: the stream its gated general path runs on beside the caller's, and the fork /
    // join events (created on first use)
    hipStream_t rx_aux = nullptr;
    hipEvent_t rx_ev[2] = {nullptr, nullptr};
    // host-memory entry points (created on first use): chunk slots; one stream per direction
    // ([0]: H2D and the kernels, [1]: D2H); the decode's per-slot column (base, total) pairs, written
    // by the device into coherent pinned memory; the device's running column bases (two sets,
    // alternating by chunk)
    symhip::host::Slot slots[symhip::host::kSlots];
    hipStream_t host_stream[2] = {nullptr, nullptr};
    uint64_t* host_meta = nullptr;
    uint64_t* host_base = nullptr;
    bool slots_ready = false;
};

namespace symhip {
namespace capi {
int fail(int code, const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);
extern const Layout kLayouts[SYM_SCHEMA_COUNT];
inline bool schema_ok(int schema) { return schema >= 0 && schema < SYM_SCHEMA_COUNT; }
inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Runs the body with ctx->device current, restoring the caller's device after.
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) err = hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// sym_encode with every out_off value written offset by out_base (capi.cpp)
int encode_call(sym_ctx* ctx, int schema, uint64_t n, const int32_t* const* d_fixed, const uint8_t* const* d_bytes,
                const uint64_t* const* d_offs, uint32_t service_id, uint32_t method_id, uint8_t* d_out,
                uint64_t* d_out_off, uint64_t out_base, void* stream);
// one decode of a flat layout; d_type non-null: a mixed kv batch (capi.cpp)
int decode_call(const char* what, sym_ctx* ctx, Layout lay, const uint8_t* d_type, uint64_t n, const uint8_t* d_in,
                const uint64_t* d_rec_off, int32_t* const* d_fixed, uint8_t* const* d_bytes, const uint64_t* caps,
                uint64_t* const* d_offs, uint8_t* d_status, void* stream);
void host_slots_destroy(sym_ctx* ctx);  // host.cpp
}  // namespace capi
}  // namespace symhip
