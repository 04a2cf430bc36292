// capi.cpp -- the extern "C" boundary declared in include/symphony_hip.h.
//
// Argument checking, schema dispatch, the per-ctx workspaces and device error reporting.  All
// compute goes to the HIP kernels (encode.hip, decode_pipe.hip, ...); the host-memory entry points
// are in host.cpp.  There is no CPU codec in this library.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>

#include "../../include/symphony_hip.h"
#include "codec.hpp"
#include "ctx.hpp"
#include "flat_schema.hpp"

using symhip::DecodeParams;
using symhip::EncodeParams;
using symhip::Layout;

namespace symhip {
namespace capi {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(SYM_ERR_HIP, "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
}

const Layout kLayouts[SYM_SCHEMA_COUNT] = {
    {0, 1},  // GetRequest{Key}
    {0, 2},  // SetRequest{Key, Value}
    {0, 1},  // GetResponse{Value}
    {0, 1},  // SetResponse{Value}
    {2, 2},  // EchoRequest{Id, Score, Username, Content}
    {2, 2},  // EchoResponse
};

}  // namespace capi
}  // namespace symhip

using namespace symhip::capi;

namespace {

int ensure_ws(sym_ctx* ctx, int nvar, uint64_t n) {
    const size_t need = symhip::decode_workspace_bytes(nvar, n);
    if (need <= ctx->ws_bytes) return SYM_OK;
    if (ctx->ws) (void)hipFree(ctx->ws);
    ctx->ws = nullptr;
    ctx->ws_bytes = 0;
    hipError_t e = hipMalloc(&ctx->ws, need);
    if (e != hipSuccess) return fail(SYM_ERR_NOMEM, "decode workspace of %zu bytes: %s", need, hipGetErrorString(e));
    ctx->ws_bytes = need;
    return SYM_OK;
}

// Look-back words for n records; zeroed when allocated, so every word starts with epoch 0,
// which no call uses.
int ensure_flags(sym_ctx* ctx, uint64_t n) {
    const size_t need = symhip::decode_pipe_flag_bytes(symhip::kMaxVar, n);
    if (need <= ctx->flag_bytes) return SYM_OK;
    if (ctx->flags) (void)hipFree(ctx->flags);
    ctx->flags = nullptr;
    ctx->flag_bytes = 0;
    hipError_t e = hipMalloc(&ctx->flags, need);
    if (e != hipSuccess) return fail(SYM_ERR_NOMEM, "decode look-back words of %zu bytes: %s", need, hipGetErrorString(e));
    if ((e = hipMemset(ctx->flags, 0, need)) != hipSuccess) return hip_fail(e, "zeroing look-back words");
    ctx->flag_bytes = need;
    ctx->epoch = 0;
    return SYM_OK;
}

// The next call's epochs [*epoch, *epoch + span); on wrap-around every word is zeroed again
// (stream-ordered) first.  A decode takes two: its gate's exact re-decode tags its words epoch + 1.
int next_epoch(sym_ctx* ctx, hipStream_t stream, unsigned* epoch, unsigned span = 1) {
    if (ctx->epoch + span >= symhip::kEpochLimit) {
        hipError_t e = hipMemsetAsync(ctx->flags, 0, ctx->flag_bytes, stream);
        if (e != hipSuccess) return hip_fail(e, "zeroing look-back words");
        ctx->epoch = 0;
    }
    *epoch = ctx->epoch + 1;
    ctx->epoch += span;
    return SYM_OK;
}

int ensure_scratch(sym_ctx* ctx, size_t need, const char* what) {
    if (need <= ctx->frag_bytes) return SYM_OK;
    if (ctx->frag) (void)hipFree(ctx->frag);
    ctx->frag = nullptr;
    ctx->frag_bytes = 0;
    hipError_t e = hipMalloc(&ctx->frag, need);
    if (e != hipSuccess) return fail(SYM_ERR_NOMEM, "%s workspace of %zu bytes: %s", what, need, hipGetErrorString(e));
    ctx->frag_bytes = need;
    return SYM_OK;
}

}  // namespace

#ifdef SYMHIP_TUNING
int symhip::tuning_variant(const char* env_name) {
    const char* v = getenv(env_name);
    return v ? atoi(v) : 0;
}
#endif

extern "C" {

int sym_abi_version(void) { return SYMPHONY_HIP_ABI_VERSION; }

const char* sym_last_error(void) { return g_err; }

int sym_ctx_create(int device, sym_ctx** out_ctx) {
    if (!out_ctx) return fail(SYM_ERR_INVALID, "sym_ctx_create: out_ctx is NULL");
    *out_ctx = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
    if (device < 0 || device >= ndev) return fail(SYM_ERR_INVALID, "device %d out of range (%d devices)", device, ndev);
    DeviceGuard g(device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    sym_ctx* c = new (std::nothrow) sym_ctx;
    if (!c) return fail(SYM_ERR_NOMEM, "sym_ctx_create: out of host memory");
    c->device = device;
    if ((e = hipMalloc(&c->err, 32)) != hipSuccess || (e = hipMemset(c->err, 0, 32)) != hipSuccess) {
        sym_ctx_destroy(c);
        return hip_fail(e, "sym_ctx_create");
    }
    *out_ctx = c;
    return SYM_OK;
}

int sym_ctx_destroy(sym_ctx* ctx) {
    if (!ctx) return SYM_OK;
    DeviceGuard g(ctx->device);
    host_slots_destroy(ctx);
    for (hipEvent_t ev : ctx->rx_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (ctx->rx_aux) (void)hipStreamDestroy(ctx->rx_aux);
    if (ctx->ws) (void)hipFree(ctx->ws);
    if (ctx->flags) (void)hipFree(ctx->flags);
    if (ctx->frag) (void)hipFree(ctx->frag);
    if (ctx->crypt_tables) (void)hipFree(ctx->crypt_tables);
    if (ctx->err) (void)hipFree(ctx->err);
    delete ctx;
    return SYM_OK;
}

int sym_ctx_reserve(sym_ctx* ctx, uint64_t max_records) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_ctx_reserve: ctx is NULL");
    DeviceGuard g(ctx->device);
    const int rc = ensure_ws(ctx, symhip::kMaxVar, max_records);
    return rc != SYM_OK ? rc : ensure_flags(ctx, max_records);
}

int sym_ctx_check(sym_ctx* ctx, void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_ctx_check: ctx is NULL");
    DeviceGuard g(ctx->device);
    hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    unsigned bits = 0;
    if ((e = hipMemcpy(&bits, ctx->err, sizeof(bits), hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_fail(e, "reading device error word");
    if (bits == 0) return SYM_OK;
    if ((e = hipMemset(ctx->err, 0, sizeof(bits))) != hipSuccess) return hip_fail(e, "clearing device error word");
    if (bits & symhip::kErrTimeout) return fail(SYM_ERR_DEVICE, "decode look-back timed out (device error bits 0x%x)", bits);
    if (bits & symhip::kErrTooLarge)
        return fail(SYM_ERR_INVALID, "64 consecutive records span >= 2 GiB; split the batch (device error bits 0x%x)", bits);
    if (bits & symhip::kErrBadNested)
        return fail(SYM_ERR_INVALID, "a nested (non-repeated) message field was given more than one item for a record "
                    "(device error bits 0x%x)", bits);
    if (bits & symhip::kErrBadLength)
        return fail(SYM_ERR_INVALID, "a repeated field's byte length is not a multiple of its element width "
                    "(device error bits 0x%x)", bits);
    return fail(SYM_ERR_CAPACITY, "output capacity exceeded (decode column, Raw getter values or firewall kept bytes; device error bits 0x%x)", bits);
}

int sym_ctx_decode_redos(sym_ctx* ctx, void* stream, uint64_t* out) {
    if (!ctx || !out) return fail(SYM_ERR_INVALID, "sym_ctx_decode_redos: ctx or out is NULL");
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    if (e == hipSuccess) e = hipMemcpy(out, ctx->err + 6, sizeof(uint64_t), hipMemcpyDeviceToHost);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "sym_ctx_decode_redos");
}

int sym_ctx_set_decode_impl(sym_ctx* ctx, int impl) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_ctx_set_decode_impl: ctx is NULL");
    if (impl != SYM_DECODE_PIPELINE && impl != SYM_DECODE_THREE_KERNEL && impl != SYM_DECODE_LOOKBACK)
        return fail(SYM_ERR_INVALID, "sym_ctx_set_decode_impl: unknown implementation %d", impl);
    ctx->decode_impl = impl;
    // A new choice starts without a speculation hold: every hold an earlier call set (or a call still
    // running sets) names a call number below the ones from now on, so it is stale (decode_pipe.hip
    // spec_held, spec_tile_held).  Host-side only: nothing to order against decodes still on the
    // caller's streams.
    ctx->decode_seq += (symhip::kSpecHoldCalls > symhip::kTileHoldCalls ? symhip::kSpecHoldCalls : symhip::kTileHoldCalls) + 1;
    return SYM_OK;
}

int sym_ctx_set_encode_impl(sym_ctx* ctx, int impl) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_ctx_set_encode_impl: ctx is NULL");
    if (impl != SYM_ENCODE_PIPELINE && impl != SYM_ENCODE_THREE_KERNEL && impl != SYM_ENCODE_LOOKBACK)
        return fail(SYM_ERR_INVALID, "sym_ctx_set_encode_impl: unknown implementation %d", impl);
    ctx->encode_impl = impl;
    return SYM_OK;
}

int sym_schema_info(int schema, int* nfixed, int* nvar) {
    if (!schema_ok(schema)) return fail(SYM_ERR_INVALID, "unknown schema %d", schema);
    if (nfixed) *nfixed = kLayouts[schema].nfixed;
    if (nvar) *nvar = kLayouts[schema].nvar;
    return SYM_OK;
}

uint64_t sym_record_overhead(int schema) {
    if (!schema_ok(schema)) return 0;
    const Layout& l = kLayouts[schema];
    return 14u + 4u * (uint64_t)(l.nfixed + l.nvar) + 4u * (uint64_t)l.nvar;
}

uint64_t sym_encoded_size(int schema, uint64_t n, uint64_t var_total) {
    return n * sym_record_overhead(schema) + var_total;
}

}  // extern "C"

int symhip::capi::encode_call(sym_ctx* ctx, int schema, uint64_t n, const int32_t* const* d_fixed,
                              const uint8_t* const* d_bytes, const uint64_t* const* d_offs, uint32_t service_id,
                              uint32_t method_id, uint8_t* d_out, uint64_t* d_out_off, uint64_t out_base,
                              void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_encode: ctx is NULL");
    if (!schema_ok(schema)) return fail(SYM_ERR_INVALID, "sym_encode: unknown schema %d", schema);
    const Layout lay = kLayouts[schema];
    if (!d_out_off) return fail(SYM_ERR_INVALID, "sym_encode: d_out_off is NULL");
    if (n > 0) {
        if (!d_out) return fail(SYM_ERR_INVALID, "sym_encode: d_out is NULL");
        if (lay.nfixed && !d_fixed) return fail(SYM_ERR_INVALID, "sym_encode: d_fixed is NULL");
        if (!d_bytes || !d_offs) return fail(SYM_ERR_INVALID, "sym_encode: d_bytes/d_offs is NULL");
        for (int f = 0; f < lay.nfixed; ++f)
            if (!d_fixed[f]) return fail(SYM_ERR_INVALID, "sym_encode: fixed column %d is NULL", f);
        for (int f = 0; f < lay.nvar; ++f)
            if (!d_offs[f] || !d_bytes[f]) return fail(SYM_ERR_INVALID, "sym_encode: var column %d is NULL", f);
    }
    EncodeParams p{};
    p.lay = lay;
    p.n = n;
    for (int f = 0; f < lay.nfixed; ++f) p.fixed[f] = d_fixed[f];
    for (int f = 0; f < lay.nvar && n; ++f) {
        p.bytes[f] = d_bytes[f];
        p.offs[f] = d_offs[f];
    }
    p.service_id = service_id;
    p.method_id = method_id;
    p.out = d_out;
    p.out_off = d_out_off;
    p.out_base = out_base;
    p.err = ctx->err;
#ifdef SYMHIP_TUNING
    p.variant = symhip::tuning_variant("SYMHIP_ENCODE_VARIANT");
    if (const char* d = getenv("SYMHIP_DEBUG_PTR")) p.dbg = (uint64_t*)(uintptr_t)strtoull(d, nullptr, 16);
    if ((p.variant == 6 || p.variant == 7 || p.variant == 10 || p.variant == 53) && !p.dbg) return fail(SYM_ERR_INVALID, "encode timeline needs SYMHIP_DEBUG_PTR");
#endif
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    if (n == 0 && out_base) return fail(SYM_ERR_INVALID, "sym_encode: empty batch with an output base");
    hipError_t e = symhip::launch_encode(p, (hipStream_t)stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "encode launch");
}

extern "C" {

int sym_encode(sym_ctx* ctx, int schema, uint64_t n, const int32_t* const* d_fixed, const uint8_t* const* d_bytes,
               const uint64_t* const* d_offs, uint32_t service_id, uint32_t method_id, uint8_t* d_out,
               uint64_t* d_out_off, void* stream) {
    return encode_call(ctx, schema, n, d_fixed, d_bytes, d_offs, service_id, method_id, d_out, d_out_off, 0, stream);
}

}  // extern "C"

// One decode call of a flat layout; `type` non-null: a mixed kv batch (layout {0, 2}).
int symhip::capi::decode_call(const char* what, sym_ctx* ctx, Layout lay, const uint8_t* d_type, uint64_t n,
                       const uint8_t* d_in, const uint64_t* d_rec_off, int32_t* const* d_fixed,
                       uint8_t* const* d_bytes, const uint64_t* caps, uint64_t* const* d_offs, uint8_t* d_status,
                       void* stream) {
    if (!d_offs) return fail(SYM_ERR_INVALID, "%s: d_offs is NULL", what);
    for (int f = 0; f < lay.nvar; ++f)
        if (!d_offs[f]) return fail(SYM_ERR_INVALID, "%s: offset column %d is NULL", what, f);
    if (n > 0) {
        if (!d_in || !d_rec_off || !d_status) return fail(SYM_ERR_INVALID, "%s: d_in/d_rec_off/d_status is NULL", what);
        if (lay.nfixed && !d_fixed) return fail(SYM_ERR_INVALID, "%s: d_fixed is NULL", what);
        for (int f = 0; f < lay.nfixed; ++f)
            if (!d_fixed[f]) return fail(SYM_ERR_INVALID, "%s: fixed column %d is NULL", what, f);
        if (!d_bytes || !caps) return fail(SYM_ERR_INVALID, "%s: d_bytes/caps is NULL", what);
        for (int f = 0; f < lay.nvar; ++f)
            if (!d_bytes[f] && caps[f]) return fail(SYM_ERR_INVALID, "%s: byte column %d is NULL", what, f);
    }
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    int rc = ensure_ws(ctx, lay.nvar, n);
    if (rc == SYM_OK) rc = ensure_flags(ctx, n);
    unsigned epoch = 0;
    if (rc == SYM_OK) rc = next_epoch(ctx, (hipStream_t)stream, &epoch, 2);
    if (rc != SYM_OK) return rc;
    DecodeParams p{};
    p.lay = lay;
    p.n = n;
    p.in = d_in;
    p.rec_off = d_rec_off;
    p.type = d_type;
    for (int f = 0; f < lay.nfixed; ++f) p.fixed[f] = d_fixed[f];
    for (int f = 0; f < lay.nvar; ++f) {
        p.bytes[f] = n ? d_bytes[f] : nullptr;
        p.cap[f] = n ? caps[f] : 0;
        p.offs[f] = d_offs[f];
    }
    p.status = d_status;
    p.ws = ctx->ws;
    p.flags = ctx->flags;
    p.epoch = epoch;
    p.seq = ++ctx->decode_seq;
    p.err = ctx->err;
    p.impl = ctx->decode_impl;
#ifdef SYMHIP_TUNING
    p.variant = symhip::tuning_variant("SYMHIP_DECODE_VARIANT");
    if (const char* d = getenv("SYMHIP_DEBUG_PTR")) p.dbg = (uint64_t*)(uintptr_t)strtoull(d, nullptr, 16);
#endif
    hipError_t e = symhip::launch_decode(p, (hipStream_t)stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "decode launch");
}

extern "C" {

int sym_decode(sym_ctx* ctx, int schema, uint64_t n, const uint8_t* d_in, const uint64_t* d_rec_off,
               int32_t* const* d_fixed, uint8_t* const* d_bytes, const uint64_t* caps, uint64_t* const* d_offs,
               uint8_t* d_status, void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_decode: ctx is NULL");
    if (!schema_ok(schema)) return fail(SYM_ERR_INVALID, "sym_decode: unknown schema %d", schema);
    return decode_call("sym_decode", ctx, kLayouts[schema], nullptr, n, d_in, d_rec_off, d_fixed, d_bytes, caps, d_offs,
                       d_status, stream);
}

// ---- typed entry points ----

int sym_encode_kv_set(sym_ctx* ctx, const uint8_t* d_key, const uint64_t* d_key_off, const uint8_t* d_val,
                      const uint64_t* d_val_off, uint64_t n, uint32_t service_id, uint32_t method_id,
                      uint8_t* d_out, uint64_t* d_out_off, void* stream) {
    const uint8_t* b[2] = {d_key, d_val};
    const uint64_t* o[2] = {d_key_off, d_val_off};
    return sym_encode(ctx, SYM_SCHEMA_KV_SET_REQUEST, n, nullptr, b, o, service_id, method_id, d_out, d_out_off, stream);
}

int sym_encode_kv_get(sym_ctx* ctx, const uint8_t* d_key, const uint64_t* d_key_off, uint64_t n,
                      uint32_t service_id, uint32_t method_id, uint8_t* d_out, uint64_t* d_out_off, void* stream) {
    const uint8_t* b[1] = {d_key};
    const uint64_t* o[1] = {d_key_off};
    return sym_encode(ctx, SYM_SCHEMA_KV_GET_REQUEST, n, nullptr, b, o, service_id, method_id, d_out, d_out_off, stream);
}

int sym_encode_kv_response(sym_ctx* ctx, int schema, const uint8_t* d_val, const uint64_t* d_val_off, uint64_t n,
                           uint32_t service_id, uint32_t method_id, uint8_t* d_out, uint64_t* d_out_off,
                           void* stream) {
    if (schema != SYM_SCHEMA_KV_GET_RESPONSE && schema != SYM_SCHEMA_KV_SET_RESPONSE)
        return fail(SYM_ERR_INVALID, "sym_encode_kv_response: schema %d is not a KV response", schema);
    const uint8_t* b[1] = {d_val};
    const uint64_t* o[1] = {d_val_off};
    return sym_encode(ctx, schema, n, nullptr, b, o, service_id, method_id, d_out, d_out_off, stream);
}

int sym_encode_echo(sym_ctx* ctx, const int32_t* d_id, const int32_t* d_score, const uint8_t* d_user,
                    const uint64_t* d_user_off, const uint8_t* d_content, const uint64_t* d_content_off, uint64_t n,
                    uint32_t service_id, uint32_t method_id, uint8_t* d_out, uint64_t* d_out_off, void* stream) {
    const int32_t* fx[2] = {d_id, d_score};
    const uint8_t* b[2] = {d_user, d_content};
    const uint64_t* o[2] = {d_user_off, d_content_off};
    return sym_encode(ctx, SYM_SCHEMA_ECHO_REQUEST, n, fx, b, o, service_id, method_id, d_out, d_out_off, stream);
}

int sym_decode_kv_set(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n, uint8_t* d_key,
                      uint64_t key_cap, uint64_t* d_key_off, uint8_t* d_val, uint64_t val_cap, uint64_t* d_val_off,
                      uint8_t* d_status, void* stream) {
    uint8_t* b[2] = {d_key, d_val};
    const uint64_t caps[2] = {key_cap, val_cap};
    uint64_t* o[2] = {d_key_off, d_val_off};
    return sym_decode(ctx, SYM_SCHEMA_KV_SET_REQUEST, n, d_in, d_rec_off, nullptr, b, caps, o, d_status, stream);
}

int sym_decode_kv_get(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n, uint8_t* d_key,
                      uint64_t key_cap, uint64_t* d_key_off, uint8_t* d_status, void* stream) {
    uint8_t* b[1] = {d_key};
    const uint64_t caps[1] = {key_cap};
    uint64_t* o[1] = {d_key_off};
    return sym_decode(ctx, SYM_SCHEMA_KV_GET_REQUEST, n, d_in, d_rec_off, nullptr, b, caps, o, d_status, stream);
}

int sym_decode_kv_response(sym_ctx* ctx, int schema, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n,
                           uint8_t* d_val, uint64_t val_cap, uint64_t* d_val_off, uint8_t* d_status, void* stream) {
    if (schema != SYM_SCHEMA_KV_GET_RESPONSE && schema != SYM_SCHEMA_KV_SET_RESPONSE)
        return fail(SYM_ERR_INVALID, "sym_decode_kv_response: schema %d is not a KV response", schema);
    uint8_t* b[1] = {d_val};
    const uint64_t caps[1] = {val_cap};
    uint64_t* o[1] = {d_val_off};
    return sym_decode(ctx, schema, n, d_in, d_rec_off, nullptr, b, caps, o, d_status, stream);
}

int sym_decode_echo(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n, int32_t* d_id,
                    int32_t* d_score, uint8_t* d_user, uint64_t user_cap, uint64_t* d_user_off, uint8_t* d_content,
                    uint64_t content_cap, uint64_t* d_content_off, uint8_t* d_status, void* stream) {
    int32_t* fx[2] = {d_id, d_score};
    uint8_t* b[2] = {d_user, d_content};
    const uint64_t caps[2] = {user_cap, content_cap};
    uint64_t* o[2] = {d_user_off, d_content_off};
    return sym_decode(ctx, SYM_SCHEMA_ECHO_REQUEST, n, d_in, d_rec_off, fx, b, caps, o, d_status, stream);
}

// ---- mixed GetRequest / SetRequest batches ----

uint64_t sym_encoded_size_kv_mixed(uint64_t n, uint64_t n_set, uint64_t key_total, uint64_t set_value_total) {
    return 22 * n + 8 * n_set + key_total + set_value_total;
}

int sym_encode_kv_mixed(sym_ctx* ctx, const uint8_t* d_type, const uint8_t* d_key, const uint64_t* d_key_off,
                        const uint8_t* d_val, const uint64_t* d_val_off, uint64_t n, uint32_t service_id,
                        uint32_t get_method_id, uint32_t set_method_id, uint8_t* d_out, uint64_t* d_out_off,
                        void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_encode_kv_mixed: ctx is NULL");
    if (!d_out_off || (n && (!d_type || !d_key || !d_key_off || !d_val || !d_val_off || !d_out)))
        return fail(SYM_ERR_INVALID, "sym_encode_kv_mixed: NULL argument");
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    EncodeParams p{};
    p.lay = kLayouts[SYM_SCHEMA_KV_SET_REQUEST];
    p.n = n;
    p.bytes[0] = d_key;
    p.offs[0] = d_key_off;
    p.bytes[1] = d_val;
    p.offs[1] = d_val_off;
    p.service_id = service_id;
    p.method_id = set_method_id;
    p.method_get = get_method_id;
    p.type = d_type;
    p.out = d_out;
    p.out_off = d_out_off;
    p.err = ctx->err;
    p.impl = ctx->encode_impl;
#ifdef SYMHIP_TUNING
    p.variant = symhip::tuning_variant("SYMHIP_ENCODE_VARIANT");
    if (p.variant == 37 || p.variant == 38 || p.variant == 52) {  // tools/mixed_timeline.py: 16 u64 per 64-record tile
        if (const char* d = getenv("SYMHIP_DEBUG_PTR")) p.dbg = (uint64_t*)(uintptr_t)strtoull(d, nullptr, 16);
        if (!p.dbg) return fail(SYM_ERR_INVALID, "mixed encode timeline needs SYMHIP_DEBUG_PTR");
    }
#endif
    if (n) {
        int rc = ensure_flags(ctx, n);
        unsigned epoch = 0;
        if (rc == SYM_OK) rc = next_epoch(ctx, (hipStream_t)stream, &epoch);
        if (rc == SYM_OK) rc = ensure_scratch(ctx, symhip::encode_mixed_ws_bytes(n), "mixed encode");
        if (rc != SYM_OK) return rc;
        p.flags = ctx->flags;
        p.epoch = epoch;
    }
    hipError_t e = symhip::launch_encode_mixed(p, ctx->frag, (hipStream_t)stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "mixed encode launch");
}

int sym_decode_kv_mixed(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, const uint8_t* d_type,
                        uint64_t n, uint8_t* d_key, uint64_t key_cap, uint64_t* d_key_off, uint8_t* d_val,
                        uint64_t val_cap, uint64_t* d_val_off, uint8_t* d_status, void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_decode_kv_mixed: ctx is NULL");
    if (n && !d_type) return fail(SYM_ERR_INVALID, "sym_decode_kv_mixed: d_type is NULL");
    uint8_t* b[2] = {d_key, d_val};
    const uint64_t caps[2] = {key_cap, val_cap};
    uint64_t* o[2] = {d_key_off, d_val_off};
    return decode_call("sym_decode_kv_mixed", ctx, kLayouts[SYM_SCHEMA_KV_SET_REQUEST], n ? d_type : nullptr, n, d_in,
                       d_rec_off, nullptr, b, caps, o, d_status, stream);
}

// ---- packetization ----

int sym_fragment_plan(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n,
                      uint32_t max_udp_payload, uint64_t* d_first, uint64_t* d_wire_off, uint8_t* d_status,
                      void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_fragment_plan: ctx is NULL");
    if (max_udp_payload <= SYM_DATA_PACKET_HEADER)  // FragmentPackets: "MTU must be positive"
        return fail(SYM_ERR_INVALID, "sym_fragment_plan: max_udp_payload %u leaves no payload", max_udp_payload);
    if (!d_rec_off || !d_first || !d_wire_off || (n && (!d_in || !d_status)))
        return fail(SYM_ERR_INVALID, "sym_fragment_plan: NULL argument");
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    const size_t cols = align256((n + 1) * sizeof(uint64_t));
    const size_t temp = symhip::frag_scan_temp_bytes(n);
    const int rc = ensure_scratch(ctx, 2 * cols + temp, "packetization");
    if (rc != SYM_OK) return rc;
    uint64_t* cnt = (uint64_t*)ctx->frag;
    uint64_t* bytes = (uint64_t*)((char*)ctx->frag + cols);
    void* tmp = (char*)ctx->frag + 2 * cols;
    hipError_t e = symhip::launch_frag_plan(d_in, d_rec_off, n, max_udp_payload - SYM_DATA_PACKET_HEADER, cnt, bytes,
                                            d_first, d_wire_off, d_status, tmp, temp, (hipStream_t)stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "fragment plan launch");
}

int sym_fragment_write(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n,
                       uint32_t max_udp_payload, uint8_t packet_type, const uint64_t* d_rpc_id,
                       const sym_endpoints* endpoints, const uint64_t* d_first, const uint64_t* d_wire_off,
                       const uint8_t* d_status, uint8_t* d_wire, uint64_t* d_dg_off, void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_fragment_write: ctx is NULL");
    if (max_udp_payload <= SYM_DATA_PACKET_HEADER)
        return fail(SYM_ERR_INVALID, "sym_fragment_write: max_udp_payload %u leaves no payload", max_udp_payload);
    if (!endpoints || !d_dg_off || (n && (!d_in || !d_rec_off || !d_rpc_id || !d_first || !d_wire_off || !d_status ||
                                          !d_wire)))
        return fail(SYM_ERR_INVALID, "sym_fragment_write: NULL argument");
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    if (n == 0) {
        hipError_t e = hipMemsetAsync(d_dg_off, 0, sizeof(uint64_t), (hipStream_t)stream);
        return e == hipSuccess ? SYM_OK : hip_fail(e, "hipMemsetAsync");
    }
    symhip::FragWriteArgs a{};
    a.in = d_in;
    a.rec_off = d_rec_off;
    a.n = n;
    a.M = max_udp_payload - SYM_DATA_PACKET_HEADER;
    a.type = packet_type;
    a.rpc_id = d_rpc_id;
    for (int i = 0; i < 4; ++i) {
        a.dst_ip[i] = endpoints->dst_ip[i];
        a.src_ip[i] = endpoints->src_ip[i];
    }
    a.dst_port = endpoints->dst_port;
    a.src_port = endpoints->src_port;
    a.first = d_first;
    a.out_off = d_wire_off;
    a.status = d_status;
    a.out = d_wire;
    a.dg_off = d_dg_off;
    a.err = ctx->err;
    hipError_t e = symhip::launch_frag_write(a, (hipStream_t)stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "fragment write launch");
}

int sym_raw_get_fixed(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n, int segment,
                      uint32_t table_off, uint32_t width, void* d_out, uint8_t* d_status, void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_raw_get_fixed: ctx is NULL");
    if (segment != SYM_SEGMENT_PUBLIC && segment != SYM_SEGMENT_PRIVATE)
        return fail(SYM_ERR_INVALID, "sym_raw_get_fixed: segment %d", segment);
    if (width != 1 && width != 4 && width != 8)
        return fail(SYM_ERR_INVALID, "sym_raw_get_fixed: width %u (fixed fields are 1, 4 or 8 bytes)", width);
    if (n && (!d_in || !d_rec_off || !d_out)) return fail(SYM_ERR_INVALID, "sym_raw_get_fixed: NULL argument");
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    hipError_t e = symhip::launch_raw_fixed(d_in, d_rec_off, n, segment, table_off, width, d_out, d_status,
                                            (hipStream_t)stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "raw fixed getter launch");
}

int sym_raw_get_bytes(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n, int segment,
                      uint32_t table_off, uint8_t* d_out, uint64_t out_cap, uint64_t* d_out_off, uint8_t* d_status,
                      void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_raw_get_bytes: ctx is NULL");
    if (segment != SYM_SEGMENT_PUBLIC && segment != SYM_SEGMENT_PRIVATE)
        return fail(SYM_ERR_INVALID, "sym_raw_get_bytes: segment %d", segment);
    if (!d_out_off || (n && (!d_in || !d_rec_off || (out_cap && !d_out))))
        return fail(SYM_ERR_INVALID, "sym_raw_get_bytes: NULL argument");
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    const int rc = ensure_scratch(ctx, symhip::raw_bytes_ws_bytes(n), "raw getter");
    if (rc != SYM_OK) return rc;
    hipError_t e = symhip::launch_raw_bytes(d_in, d_rec_off, n, segment, table_off, d_out, out_cap, d_out_off,
                                            d_status, ctx->frag, ctx->err, (hipStream_t)stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "raw bytes getter launch");
}

int sym_firewall_filter(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n,
                        uint32_t score_table_off, int32_t block_threshold, int32_t* d_score, uint8_t* d_verdict,
                        uint8_t* d_kept, uint64_t kept_cap, uint64_t* d_kept_off, uint64_t* d_kept_index,
                        uint64_t* d_nkept, void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_firewall_filter: ctx is NULL");
    if (!d_kept_off || !d_nkept || (n && (!d_in || !d_rec_off || !d_verdict || (kept_cap && !d_kept))))
        return fail(SYM_ERR_INVALID, "sym_firewall_filter: NULL argument");
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    if (n == 0) {
        hipError_t e = hipMemsetAsync(d_kept_off, 0, sizeof(uint64_t), (hipStream_t)stream);
        if (e == hipSuccess) e = hipMemsetAsync(d_nkept, 0, sizeof(uint64_t), (hipStream_t)stream);
        return e == hipSuccess ? SYM_OK : hip_fail(e, "hipMemsetAsync");
    }
    const int rc = ensure_scratch(ctx, symhip::firewall_ws_bytes(n), "firewall");
    if (rc != SYM_OK) return rc;
    hipError_t e = symhip::launch_firewall(d_in, d_rec_off, n, score_table_off, block_threshold, d_score, d_verdict,
                                           d_kept, kept_cap, d_kept_off, d_kept_index, d_nkept, ctx->frag, ctx->err,
                                           (hipStream_t)stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "firewall launch");
}

int sym_reassemble(sym_ctx* ctx, const uint8_t* d_wire, const uint64_t* d_dg_off, uint64_t n, uint8_t* d_msg,
                   uint64_t msg_cap, uint64_t* d_msg_off, uint64_t* d_msg_rpc, uint64_t* d_msg_dg, uint64_t* d_nmsg,
                   uint8_t* d_status, void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_reassemble: ctx is NULL");
    if (n >= ((uint64_t)1 << 31)) return fail(SYM_ERR_INVALID, "sym_reassemble: %llu datagrams (limit 2^31)",
                                              (unsigned long long)n);
    if (!d_msg_off || !d_nmsg ||
        (n && (!d_wire || !d_dg_off || !d_msg_rpc || !d_msg_dg || !d_status || (msg_cap && !d_msg))))
        return fail(SYM_ERR_INVALID, "sym_reassemble: NULL argument");
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    if (n == 0) {
        hipError_t e = hipMemsetAsync(d_msg_off, 0, sizeof(uint64_t), (hipStream_t)stream);
        if (e == hipSuccess) e = hipMemsetAsync(d_nmsg, 0, sizeof(uint64_t), (hipStream_t)stream);
        return e == hipSuccess ? SYM_OK : hip_fail(e, "hipMemsetAsync");
    }
    const int rc = ensure_scratch(ctx, symhip::reassemble_ws_bytes(n), "reassembly");
    if (rc != SYM_OK) return rc;
    if (!ctx->rx_aux) {
        // high priority: for a single-datagram batch its ~20 launches exit at once, and they should
        // not queue behind the copy running beside them
        int least = 0, greatest = 0;
        hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
        if (e == hipSuccess) e = hipStreamCreateWithPriority(&ctx->rx_aux, hipStreamNonBlocking, greatest);
        for (int i = 0; i < 2 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&ctx->rx_ev[i], hipEventDisableTiming);
        if (e != hipSuccess) return hip_fail(e, "reassembly stream / events");
    }
    hipError_t e = symhip::launch_reassemble(d_wire, d_dg_off, n, d_msg, msg_cap, d_msg_off, d_msg_rpc, d_msg_dg, d_nmsg,
                                             d_status, ctx->frag, ctx->err, (hipStream_t)stream, ctx->rx_aux,
                                             ctx->rx_ev[0], ctx->rx_ev[1]);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "reassembly launch");
}

// lists: accept the list-like widths (repeated string / bytes, nested and repeated messages)
static int flat_check(const char* what, const sym_field* fields, int nf, bool lists) {
    if (nf < 0 || nf > SYM_MAX_FLAT_FIELDS || (nf && !fields))
        return fail(SYM_ERR_INVALID, "%s: %d fields (0..%d)", what, nf, SYM_MAX_FLAT_FIELDS);
    for (int k = 0; k < nf; ++k) {
        if (fields[k].segment > 1) return fail(SYM_ERR_INVALID, "%s: field %d segment %u", what, k, fields[k].segment);
        const unsigned wd = fields[k].width;
        const unsigned w = wd & ~(SYM_FIELD_REPEATED | SYM_FIELD_MESSAGE | SYM_FIELD_FRAMED), rep = wd & SYM_FIELD_REPEATED;
        const bool list = symhip::flat::list_kind(fields[k]) != symhip::flat::kListNone;
        if ((w != 0 && w != 1 && w != 4 && w != 8) || ((wd & SYM_FIELD_MESSAGE) && w != 0) || (list && !lists) ||
            (rep && w == 0 && !lists) || ((wd & SYM_FIELD_FRAMED) && !(wd & SYM_FIELD_MESSAGE)))
            return fail(SYM_ERR_INVALID, "%s: field %d width 0x%x%s", what, k, wd,
                        list && !lists ? " (list-like fields need the _ex entry points)" : "");
    }
    return SYM_OK;
}

// scalar fixed-width field (a value column, no offsets); else string or repeated (bytes + offsets)
static bool flat_scalar(const sym_field& f) { return !symhip::flat::is_payload(f); }
static bool flat_list(const sym_field& f) { return symhip::flat::list_kind(f) != symhip::flat::kListNone; }

uint64_t sym_flat_encoded_size(const sym_field* fields, int nfields, uint64_t n, uint64_t var_total) {
    if (nfields == 0) return 14 * n;
    uint64_t per = 13 + 1;
    for (int k = 0; k < nfields; ++k)  // scalar inline, else table entry + length / count prefix
        per += flat_scalar(fields[k]) ? fields[k].width : 8;
    return per * n + var_total;
}

uint64_t sym_flat_encoded_size_ex(const sym_field* fields, int nfields, uint64_t n, const uint64_t* bytes,
                                  const uint64_t* items) {
    if (nfields == 0) return 14 * n;
    uint64_t t = 14 * n;
    for (int k = 0; k < nfields; ++k) {
        const sym_field& f = fields[k];
        const uint64_t b = bytes ? bytes[k] : 0, m = items ? items[k] : 0;
        if (flat_scalar(f)) t += (uint64_t)f.width * n;
        else if (!flat_list(f)) t += 8 * n + b;  // entry + prefix + payload
        else if (f.width & SYM_FIELD_REPEATED) t += 8 * n + ((f.width & SYM_FIELD_FRAMED) ? 0 : 4 * m) + b;  // entry + count + items
        else t += 4 * n + ((f.width & SYM_FIELD_FRAMED) ? 0 : 4 * m) + b;  // nested: entry, and [len] + message when present
        // (framed items: b holds their [len] prefixes already)
    }
    return t;
}

int sym_flat_encode_ex(sym_ctx* ctx, const sym_field* fields, int nfields, uint64_t n, const void* const* d_cols,
                       const uint64_t* const* d_offs, const uint64_t* const* d_items, const sym_flat_encode_opts* opts,
                       uint8_t* d_out, uint64_t* d_out_off, void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_flat_encode: ctx is NULL");
    int rc = flat_check("sym_flat_encode", fields, nfields, d_items != nullptr);
    if (rc != SYM_OK) return rc;
    const sym_flat_encode_opts o = opts ? *opts : sym_flat_encode_opts{};
    if (o.frame_prefix_len > SYM_FRAME_PREFIX_MAX || (o.frame_prefix_len && !o.framed))
        return fail(SYM_ERR_INVALID, "sym_flat_encode: frame_prefix_len %u (framed output only, <= %d)",
                    o.frame_prefix_len, SYM_FRAME_PREFIX_MAX);
    if (!d_out_off || (n && (!d_out || (nfields && (!d_cols || !d_offs)))))
        return fail(SYM_ERR_INVALID, "sym_flat_encode: NULL argument");
    for (int k = 0; k < nfields && n; ++k) {
        if (!d_cols[k] || (!flat_scalar(fields[k]) && !d_offs[k]) || (flat_list(fields[k]) && !d_items[k]))
            return fail(SYM_ERR_INVALID, "sym_flat_encode: field %d has no column", k);
        if (flat_scalar(fields[k]) && (uintptr_t)d_cols[k] % fields[k].width)
            return fail(SYM_ERR_INVALID, "sym_flat_encode: field %d column not %u-byte aligned", k, fields[k].width);
    }
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    if (n == 0) {
        if (o.d_gate_rec) return fail(SYM_ERR_INVALID, "sym_flat_encode: a gated launch needs records");
        hipError_t e = hipMemsetAsync(d_out_off, 0, sizeof(uint64_t), (hipStream_t)stream);
        return e == hipSuccess ? SYM_OK : hip_fail(e, "hipMemsetAsync");
    }
    hipError_t e = symhip::launch_flat_encode(fields, nfields, n, d_cols, d_offs, d_items, o, d_out, d_out_off, ctx->err,
                                              (hipStream_t)stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "flat encode launch");
}

int sym_flat_encode(sym_ctx* ctx, const sym_field* fields, int nfields, uint64_t n, const void* const* d_cols,
                    const uint64_t* const* d_offs, uint32_t service_id, uint32_t method_id, uint8_t* d_out,
                    uint64_t* d_out_off, void* stream) {
    sym_flat_encode_opts o{};
    o.service_id = service_id;
    o.method_id = method_id;
    return sym_flat_encode_ex(ctx, fields, nfields, n, d_cols, d_offs, nullptr, &o, d_out, d_out_off, stream);
}

int sym_flat_decode_ex(sym_ctx* ctx, const sym_field* fields, int nfields, uint64_t n, const uint64_t* d_n,
                       const uint8_t* d_in, const uint64_t* d_rec_src, const uint64_t* d_rec_len, const uint64_t* d_lo,
                       const uint64_t* d_hi, void* const* d_cols, const uint64_t* caps, uint64_t* const* d_offs,
                       uint64_t* const* d_items, uint64_t* const* d_item_len, const uint64_t* item_caps,
                       uint8_t* d_status, uint8_t* d_fail, void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_flat_decode: ctx is NULL");
    const bool lists = d_items != nullptr;
    int rc = flat_check("sym_flat_decode", fields, nfields, lists);
    if (rc != SYM_OK) return rc;
    if (n && (!d_in || !d_rec_src || !d_status || (nfields && (!d_cols || !caps || !d_offs))))
        return fail(SYM_ERR_INVALID, "sym_flat_decode: NULL argument");
    if ((d_lo == nullptr) != (d_hi == nullptr)) return fail(SYM_ERR_INVALID, "sym_flat_decode: give both d_lo and d_hi");
    if (n && d_rec_len && !d_lo) return fail(SYM_ERR_INVALID, "sym_flat_decode: records in place need d_lo / d_hi");
    for (int k = 0; k < nfields; ++k) {
        const bool inplace = d_item_len && d_item_len[k];
        if ((n && !d_cols[k] && (flat_scalar(fields[k]) || caps[k])) || (!flat_scalar(fields[k]) && !d_offs[k]))
            return fail(SYM_ERR_INVALID, "sym_flat_decode: field %d has no column", k);
        if (flat_list(fields[k]) && (!item_caps || !d_items[k]))
            return fail(SYM_ERR_INVALID, "sym_flat_decode: list-like field %d needs d_items and item_caps", k);
        if (inplace && !(fields[k].width & SYM_FIELD_MESSAGE))
            return fail(SYM_ERR_INVALID, "sym_flat_decode: field %d is not a message field (d_item_len)", k);
    }
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    if (n == 0) {
        for (int k = 0; k < nfields; ++k) {
            hipError_t e = hipSuccess;
            if (!flat_scalar(fields[k])) e = hipMemsetAsync(d_offs[k], 0, sizeof(uint64_t), (hipStream_t)stream);
            if (e == hipSuccess && flat_list(fields[k]))
                e = hipMemsetAsync(d_items[k], 0, sizeof(uint64_t), (hipStream_t)stream);
            if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync");
        }
        return SYM_OK;
    }
    if ((rc = ensure_scratch(ctx, symhip::flat_ws_bytes(fields, nfields, n, item_caps), "flat decode")) != SYM_OK)
        return rc;
    hipError_t e = symhip::launch_flat_decode(fields, nfields, n, d_n, d_in, d_rec_src, d_rec_len, d_lo, d_hi, d_cols,
                                              caps, d_offs, d_items, d_item_len, item_caps, d_status, d_fail, ctx->frag,
                                              ctx->err, (hipStream_t)stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "flat decode launch");
}

int sym_flat_decode(sym_ctx* ctx, const sym_field* fields, int nfields, uint64_t n, const uint8_t* d_in,
                    const uint64_t* d_rec_off, void* const* d_cols, const uint64_t* caps, uint64_t* const* d_offs,
                    uint8_t* d_status, void* stream) {
    return sym_flat_decode_ex(ctx, fields, nfields, n, nullptr, d_in, d_rec_off, nullptr, nullptr, nullptr, d_cols, caps,
                              d_offs, nullptr, nullptr, nullptr, d_status, nullptr, stream);
}

int sym_flat_nested_status(sym_ctx* ctx, const sym_field* fields, int nfields, int nk, const int* ks, uint64_t n,
                           const uint64_t* d_n, const uint64_t* const* d_rec_items,
                           const uint8_t* const* d_item_status, uint8_t* d_status, uint8_t* d_fail, void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_flat_nested_status: ctx is NULL");
    int rc = flat_check("sym_flat_nested_status", fields, nfields, true);
    if (rc != SYM_OK) return rc;
    if (nk < 0 || nk > nfields || (nk && (!ks || !d_rec_items || !d_item_status)))
        return fail(SYM_ERR_INVALID, "sym_flat_nested_status: %d fields", nk);
    uint32_t pos[SYM_MAX_FLAT_FIELDS];
    for (int q = 0; q < nk; ++q) {
        const int field = ks[q];
        if (field < 0 || field >= nfields || !(fields[field].width & SYM_FIELD_MESSAGE))
            return fail(SYM_ERR_INVALID, "sym_flat_nested_status: field %d is not a message field", field);
        if (n && (!d_rec_items[q] || !d_item_status[q] || !d_status || !d_fail))
            return fail(SYM_ERR_INVALID, "sym_flat_nested_status: NULL argument");
        pos[q] = 0;  // the field's position in unmarshal order: public fields, then private
        for (int k = 0; k < nfields; ++k)
            if (fields[k].segment < fields[field].segment || (fields[k].segment == fields[field].segment && k < field))
                ++pos[q];
    }
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    hipError_t e = symhip::launch_nested_status(n, d_n, nk, pos, d_rec_items, d_item_status, d_status, d_fail,
                                                (hipStream_t)stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "nested status launch");
}

int sym_flat_list_sizes(sym_ctx* ctx, int nl, uint64_t n, const uint64_t* d_n, const uint64_t* const* d_recs,
                        const uint64_t* const* d_items, const uint64_t* item_caps, uint64_t* d_out, void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_flat_list_sizes: ctx is NULL");
    if (nl < 0 || nl > SYM_MAX_FLAT_FIELDS) return fail(SYM_ERR_INVALID, "sym_flat_list_sizes: %d lists", nl);
    if (nl == 0) return SYM_OK;
    if (!d_recs || !d_items || !item_caps || !d_out) return fail(SYM_ERR_INVALID, "sym_flat_list_sizes: NULL argument");
    for (int i = 0; i < nl; ++i)
        if (!d_recs[i] || !d_items[i]) return fail(SYM_ERR_INVALID, "sym_flat_list_sizes: list %d is NULL", i);
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    hipError_t e = symhip::launch_list_sizes(nl, n, d_n, d_recs, d_items, item_caps, d_out, (hipStream_t)stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "list sizes launch");
}

int sym_raw_set(sym_ctx* ctx, const sym_field* fields, int nfields, int field, const uint8_t* d_in,
                const uint64_t* d_rec_off, uint64_t n, const void* d_val, const uint64_t* d_val_off, uint8_t* d_out,
                uint64_t out_cap, uint64_t* d_out_off, uint8_t* d_status, void* stream) {
    if (!ctx) return fail(SYM_ERR_INVALID, "sym_raw_set: ctx is NULL");
    int rc = flat_check("sym_raw_set", fields, nfields, false);
    if (rc != SYM_OK) return rc;
    if (field < 0 || field >= nfields) return fail(SYM_ERR_INVALID, "sym_raw_set: field %d of %d", field, nfields);
    const bool scalar = flat_scalar(fields[field]);
    if (!d_out_off || (n && (!d_in || !d_rec_off || !d_val || (!scalar && !d_val_off) || !d_out || !d_status)))
        return fail(SYM_ERR_INVALID, "sym_raw_set: NULL argument");
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    if (n && (rc = ensure_scratch(ctx, symhip::raw_set_ws_bytes(n), "raw setter")) != SYM_OK) return rc;
    hipError_t e = symhip::launch_raw_set(fields, nfields, field, n, d_in, d_rec_off, (const uint8_t*)d_val,
                                          scalar ? nullptr : d_val_off, d_out, out_cap, d_out_off, d_status, ctx->frag,
                                          ctx->err, (hipStream_t)stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, "raw setter launch");
}

static int crypt_call(bool enc, sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n,
                      const uint8_t* pub_key, const uint8_t* priv_key, const uint8_t* d_nonces, uint8_t* d_out,
                      uint64_t* d_out_off, uint8_t* d_status, void* stream) {
    const char* what = enc ? "sym_encrypt" : "sym_decrypt";
    if (!ctx) return fail(SYM_ERR_INVALID, "%s: ctx is NULL", what);
    if (!pub_key || !priv_key) return fail(SYM_ERR_INVALID, "%s: publicKey and privateKey are required", what);
    if (!d_out_off || (n && (!d_in || !d_rec_off || !d_out || !d_status || (enc && !d_nonces))))
        return fail(SYM_ERR_INVALID, "%s: NULL argument", what);
    DeviceGuard g(ctx->device);
    if (g.err != hipSuccess) return hip_fail(g.err, "hipSetDevice");
    if (n == 0) {
        hipError_t e = hipMemsetAsync(d_out_off, 0, sizeof(uint64_t), (hipStream_t)stream);
        return e == hipSuccess ? SYM_OK : hip_fail(e, "hipMemsetAsync");
    }
    hipError_t e;
    if (!ctx->num_cus && (e = hipDeviceGetAttribute(&ctx->num_cus, hipDeviceAttributeMultiprocessorCount,
                                                    ctx->device)) != hipSuccess)
        return hip_fail(e, "hipDeviceGetAttribute");
    const bool same = ctx->crypt_tables && !memcmp(ctx->crypt_keys, pub_key, 32) && !memcmp(ctx->crypt_keys + 32, priv_key, 32);
    if (!same) {  // key schedule + GHASH tables on the host, once per key pair
        const size_t tb = symhip::crypt_tables_bytes();
        if (!ctx->crypt_tables && (e = hipMalloc(&ctx->crypt_tables, tb)) != hipSuccess)
            return fail(SYM_ERR_NOMEM, "%s: key tables: %s", what, hipGetErrorString(e));
        void* h = malloc(tb);
        if (!h) return fail(SYM_ERR_NOMEM, "%s: out of host memory", what);
        symhip::crypt_build_tables(pub_key, priv_key, h);
        // stream-ordered behind earlier calls that may still read the old tables
        if ((e = hipStreamSynchronize((hipStream_t)stream)) == hipSuccess)
            e = hipMemcpy(ctx->crypt_tables, h, tb, hipMemcpyHostToDevice);
        free(h);
        if (e != hipSuccess) return hip_fail(e, "uploading key tables");
        memcpy(ctx->crypt_keys, pub_key, 32);
        memcpy(ctx->crypt_keys + 32, priv_key, 32);
    }
    const int rc = ensure_scratch(ctx, symhip::crypt_ws_bytes(n), "segment cipher");
    if (rc != SYM_OK) return rc;
    e = symhip::launch_crypt(enc, d_in, d_rec_off, n, d_nonces, ctx->crypt_tables, d_out, d_out_off, d_status,
                             ctx->frag, ctx->num_cus, (hipStream_t)stream);
    return e == hipSuccess ? SYM_OK : hip_fail(e, what);
}

int sym_encrypt(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n, const uint8_t* pub_key,
                const uint8_t* priv_key, const uint8_t* d_nonces, uint8_t* d_out, uint64_t* d_out_off,
                uint8_t* d_status, void* stream) {
    return crypt_call(true, ctx, d_in, d_rec_off, n, pub_key, priv_key, d_nonces, d_out, d_out_off, d_status, stream);
}

int sym_decrypt(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n, const uint8_t* pub_key,
                const uint8_t* priv_key, uint8_t* d_out, uint64_t* d_out_off, uint8_t* d_status, void* stream) {
    return crypt_call(false, ctx, d_in, d_rec_off, n, pub_key, priv_key, nullptr, d_out, d_out_off, d_status, stream);
}

}  // extern "C"
