// codec.hpp -- internal interface between the C ABI (capi.cpp) and the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

// Kernel-argument arrays indexed by a field / column number at run time must be 4-byte typed and
// sit at a 4-byte-aligned (pointers: 8-byte) offset of their struct.  With a 1-byte array the
// compiler once folded a field index into the base of a scalar load from the kernel arguments at a
// misaligned offset; the scalar load ignored the low address bits, read a wrong pointer and the
// kernel faulted on hardware (general schemas).  Every such array is checked here.
#define SYMHIP_KERNARG_ARRAY(S, m)                                                                      \
    static_assert(sizeof(((S*)nullptr)->m[0]) >= 4 && offsetof(S, m) % 4 == 0 &&                        \
                      offsetof(S, m) % alignof(decltype(((S*)nullptr)->m[0])) == 0,                      \
                  #S "::" #m ": an indexed kernel-argument array must be 4-byte typed and aligned")

namespace symhip {

typedef uint64_t u64_t;

constexpr int kMaxFixed = 2;
constexpr int kMaxVar = 2;

// Records per workgroup tile (one record per thread in the per-record phases).
constexpr int kTile = 256;

struct Layout {
    int nfixed;
    int nvar;
};

struct EncodeParams {
    Layout lay;
    uint64_t n;
    const int32_t* fixed[kMaxFixed];
    const uint8_t* bytes[kMaxVar];
    const uint64_t* offs[kMaxVar];
    uint32_t service_id;
    uint32_t method_id;
    uint8_t* out;
    uint64_t* out_off;
    unsigned* err;  // persistent device error word (kErr* bits), cleared by the host
    // mixed kv batch (sym_encode_kv_mixed): per-record type (0 GetRequest, else SetRequest); null
    // otherwise.  Record-size prefixes come from the launch's own sizers and scanner through the
    // ctx's epoch-tagged words (flags, epoch; pipe_words.hpp), or -- SYM_ENCODE_THREE_KERNEL -- from
    // a separate size pass (tile t starts at group_pre[t / 16] + tile_loc[t]).
    const uint8_t* type;
    const uint64_t* group_pre;
    const uint64_t* tile_loc;
    void* flags;             // decode_pipe_flag_bytes() bytes of look-back words (sym_ctx)
    unsigned epoch;          // their tag for this call, in [1, kEpochLimit)
    unsigned pipe_sizers;    // set by launch_encode_mixed: sizer workgroups of the launch
    int pipe_lookback;       // set by launch_encode_mixed: no sizers / scanner, every tile looks back
    int impl;                // mixed batches: SYM_ENCODE_* (sym_ctx_set_encode_impl)
    uint32_t method_get;  // method id written into [9:13] of GetRequest records (mixed batches)
    uint64_t out_base;    // added to every out_off value written (chunked host staging), 0 otherwise
    uint64_t* dbg;        // tuning builds only (tools/enc_timeline.py): per-tile timestamps, else null
    int variant;    // kernel tuning variant (tuning builds only, tuning_variant("SYMHIP_ENCODE_VARIANT"))
};

SYMHIP_KERNARG_ARRAY(EncodeParams, fixed);
SYMHIP_KERNARG_ARRAY(EncodeParams, bytes);
SYMHIP_KERNARG_ARRAY(EncodeParams, offs);

// Decode implementations selectable per ctx (sym_ctx_set_decode_impl).
constexpr int kImplPipeline = 0;      // one launch: parsers, streaming scanner, copiers (default)
constexpr int kImplThreeKernel = 1;   // parse -> scan -> copy, three stream-ordered launches
constexpr int kImplLookback = 2;      // the pipeline with parsers and scanner idle: every copier
                                      // resolves its prefix by look-back (the fallback path, forced)

struct DecodeParams {
    Layout lay;
    uint64_t n;
    const uint8_t* in;
    const uint64_t* rec_off;
    int32_t* fixed[kMaxFixed];
    uint8_t* bytes[kMaxVar];
    uint64_t cap[kMaxVar];
    uint64_t* offs[kMaxVar];
    uint8_t* status;
    const uint8_t* type;  // mixed kv batch: per-record type (0 GetRequest, else SetRequest); else null
    void* ws;       // decode_workspace_bytes() bytes (three-kernel decode)
    void* flags;    // decode_pipe_flag_bytes() bytes of aggregate / prefix words (default decode)
    unsigned epoch; // word tag of this call, in [1, kEpochLimit)
    uint64_t seq;   // this decode call's number in its ctx (1, 2, ...; never reset): the speculation
                    // hold counts decode calls with it (decode_pipe.hip spec_held)
    u64_t* dbg;     // tuning builds only (tools/fused_timeline.py): per-tile timestamps, else null
    unsigned pipe_parsers;  // set by launch_decode_pipe: parser workgroups of the launch
    unsigned* err;  // persistent device error word (kErr* bits), cleared by the host
    int impl;       // kImpl*
    int variant;    // kernel tuning variant (tuning builds only, tuning_variant("SYMHIP_DECODE_VARIANT"))
};

SYMHIP_KERNARG_ARRAY(DecodeParams, fixed);
SYMHIP_KERNARG_ARRAY(DecodeParams, bytes);
SYMHIP_KERNARG_ARRAY(DecodeParams, cap);
SYMHIP_KERNARG_ARRAY(DecodeParams, offs);

// Device workspace for the single-pass decode scan: [0,16) tile ticket, then per var
// field one u64 look-back word per tile.  Zeroed (as one block from its start) per call.
struct DecodeWsHeader {
    unsigned int ticket;
    unsigned int pad[3];
};
constexpr unsigned kErrCapacity = 1u;
constexpr unsigned kErrTimeout = 2u;   // a bounded device-side wait gave up (the reassembly sort's grid barrier)
constexpr unsigned kErrTooLarge = 4u;  // 64 consecutive records spanning >= 2 GiB
constexpr unsigned kErrBadNested = 16u;  // flat encode: a (non-repeated) nested field given more than one item
constexpr unsigned kErrBadLength = 8u;  // flat encode: a repeated field's byte length is not a multiple of its width

size_t decode_workspace_bytes(int nvar, uint64_t n);
// Aggregate / prefix words of the default decode (decode_pipe.hip): tagged with the call's epoch, so
// they need zeroing only when allocated and when the epoch wraps.
size_t decode_pipe_flag_bytes(int nvar, uint64_t n);
constexpr unsigned kEpochLimit = 1u << 20;
// Decode calls that parse exactly after a batch whose speculative lengths missed (decode_pipe.hip).
constexpr uint64_t kSpecHoldCalls = 64;
// Decode calls that read every SetRequest's own key length (instead of one per tile) after a batch
// whose tiles did not share one key length (decode_pipe.hip, tile-uniform speculation).
constexpr uint64_t kTileHoldCalls = 1024;
hipError_t launch_decode_pipe(const DecodeParams& p, void* flags, unsigned epoch, hipStream_t stream);

#ifdef SYMHIP_TUNING
// Kernel variant selected by an environment variable (0 = default); lets tools/kbench.py compare
// variants inside one process.  Only the tuning library (make tuning) has variants: the product
// library never reads the environment.
int tuning_variant(const char* env_name);
#endif

// ---- packetization (packetize.hip)
struct FragWriteArgs {
    const uint8_t* in;
    const uint64_t* rec_off;
    uint64_t n;
    uint64_t M;  // payload bytes per datagram: max UDP payload - 31
    uint8_t type;
    const uint64_t* rpc_id;
    uint8_t dst_ip[4], src_ip[4];
    uint16_t dst_port, src_port;
    const uint64_t* first;
    const uint64_t* out_off;
    const uint8_t* status;
    uint8_t* out;
    uint64_t* dg_off;
    unsigned* err;
};
size_t frag_scan_temp_bytes(uint64_t n);
hipError_t launch_frag_plan(const uint8_t* in, const uint64_t* rec_off, uint64_t n, uint64_t M, uint64_t* cnt,
                            uint64_t* bytes, uint64_t* first, uint64_t* out_off, uint8_t* status, void* temp,
                            size_t temp_bytes, hipStream_t stream);
hipError_t launch_frag_write(const FragWriteArgs& a, hipStream_t stream);

// ---- segment gather (raw_fields.hip): out = the segments in[src[i], src[i] + len[i]) back to back
namespace raw {
struct Pair {  // tile total / prefix: bytes, records (kept records for the firewall)
    uint64_t bytes, count;
};
struct GatherArgs {
    const uint8_t* in;
    const uint64_t* rec_off;  // FW: the records
    uint64_t n;               // segments, or an upper bound of them when n_ptr is set
    const uint64_t* n_ptr;    // nullable: the segment count, on the device
    const uint64_t* lo_ptr;   // readable input range [*lo_ptr, *hi_ptr) (for unconditional loads)
    const uint64_t* hi_ptr;
    const Pair* pre;          // tile prefixes of the lengths (tiles_of(n) + 1)
    // VAR: segment sources and lengths; FW: records, kept when verdict == PASS
    const uint64_t* seg_src;
    const uint64_t* seg_len;
    const uint8_t* verdict;
    uint8_t* out;
    uint64_t cap;
    uint64_t* out_off;     // VAR: segment offsets (n+1, nullable); FW: kept record offsets (nkept+1)
    uint64_t* kept_index;  // FW: input position of each kept record (nullable)
    uint64_t* nkept;       // FW
    unsigned* err;
    uint64_t seg_bytes_hint;  // VAR: the caller's estimate of the mean segment length (0: none)
    int nt;                   // nontemporal stores: 1 for wave spans of at most kNtSpan bytes, 2 at any span (st16)
};
}  // namespace raw
hipError_t launch_tile_scan(const raw::Pair* agg, raw::Pair* pre, uint64_t ntiles, hipStream_t stream);
// the same over the tiles of a device-side item count (*nlim) only
hipError_t launch_tile_scan_limited(const raw::Pair* agg, raw::Pair* pre, uint64_t ntiles, const uint64_t* nlim,
                                    hipStream_t stream);
// `rows` scans at once (one workgroup each): row r from agg + r * agg_stride into pre + r * pre_stride
hipError_t launch_tile_scan_rows(const raw::Pair* agg, uint64_t agg_stride, raw::Pair* pre, uint64_t pre_stride,
                                 uint64_t ntiles, int rows, const uint64_t* nlim, hipStream_t stream);
hipError_t launch_tile_scan_gated(const raw::Pair* agg, raw::Pair* pre, uint64_t ntiles, const unsigned* gate,
                                  hipStream_t stream);
hipError_t launch_segment_gather(const raw::GatherArgs& a, hipStream_t stream);

// ---- any flat schema (flat.hip); sym_field is defined in include/symphony_hip.h
}  // namespace symhip
struct sym_field;
struct sym_flat_encode_opts;
namespace symhip {
size_t flat_ws_bytes(const sym_field* f, int nf, uint64_t n, const uint64_t* item_caps);
hipError_t launch_flat_encode(const sym_field* f, int nf, uint64_t n, const void* const* cols,
                              const uint64_t* const* offs, const uint64_t* const* items, const sym_flat_encode_opts& o,
                              uint8_t* out, uint64_t* out_off, unsigned* err, hipStream_t stream);
// rec_len non-null: record i is in[rec_off[i], + rec_len[i]) (records in place); lo / hi: device
// values bounding in's readable extent (null: rec_off[0], rec_off[n]); item_len[k] non-null for a
// message field k: items[k] / item_len[k] receive each item's (offset into in, length), no bytes
// n_ptr (nullable): the record count on the device, n its capacity (flat.hip)
hipError_t launch_flat_decode(const sym_field* f, int nf, uint64_t n, const uint64_t* n_ptr, const uint8_t* in,
                              const uint64_t* rec_off, const uint64_t* rec_len, const uint64_t* lo, const uint64_t* hi,
                              void* const* cols, const uint64_t* caps, uint64_t* const* offs, uint64_t* const* items,
                              uint64_t* const* item_len, const uint64_t* item_caps, uint8_t* status, uint8_t* fail,
                              void* ws, unsigned* err, hipStream_t stream);
hipError_t launch_list_sizes(int nl, uint64_t n, const uint64_t* n_ptr, const uint64_t* const* recs,
                             const uint64_t* const* items, const uint64_t* caps, uint64_t* out, hipStream_t stream);
hipError_t launch_nested_status(uint64_t n, const uint64_t* n_ptr, int nk, const uint32_t* pos,
                                const uint64_t* const* rec_items, const uint8_t* const* item_status, uint8_t* status,
                                uint8_t* fail, hipStream_t stream);

// ---- batched Raw setters (setters.hip)
size_t raw_set_ws_bytes(uint64_t n);
hipError_t launch_raw_set(const sym_field* f, int nf, int k, uint64_t n, const uint8_t* in, const uint64_t* rec_off,
                          const uint8_t* val, const uint64_t* val_off, uint8_t* out, uint64_t cap, uint64_t* out_off,
                          uint8_t* status, void* ws, unsigned* err, hipStream_t stream);

// ---- per-segment AES-256-GCM (crypto.hip)
size_t crypt_tables_bytes();
void crypt_build_tables(const uint8_t pub_key[32], const uint8_t priv_key[32], void* host_tables);
size_t crypt_ws_bytes(uint64_t n);
hipError_t launch_crypt(bool enc, const uint8_t* in, const uint64_t* rec_off, uint64_t n, const uint8_t* nonces,
                        const void* d_tables, uint8_t* out, uint64_t* out_off, uint8_t* status, void* ws, int num_cus,
                        hipStream_t stream);

// ---- receive-side reassembly (reassemble.hip)
size_t reassemble_ws_bytes(uint64_t n);
// aux / fork / join: a second stream and two events of the ctx: the gated general path runs on
// aux, beside the single-datagram path on `stream` (nullptr aux: everything on `stream`)
hipError_t launch_reassemble(const uint8_t* wire, const uint64_t* dg_off, uint64_t n, uint8_t* msg, uint64_t msg_cap,
                             uint64_t* msg_off, uint64_t* msg_rpc, uint64_t* msg_dg, uint64_t* nmsg, uint8_t* status,
                             void* ws, unsigned* err, hipStream_t stream, hipStream_t aux = nullptr,
                             hipEvent_t fork = nullptr, hipEvent_t join = nullptr);

// ---- batched Raw getters and the firewall element (raw_fields.hip)
hipError_t launch_raw_fixed(const uint8_t* in, const uint64_t* rec_off, uint64_t n, int priv, uint32_t table_off,
                            uint32_t width, void* out, uint8_t* status, hipStream_t stream);
size_t raw_bytes_ws_bytes(uint64_t n);
hipError_t launch_raw_bytes(const uint8_t* in, const uint64_t* rec_off, uint64_t n, int priv, uint32_t table_off,
                            uint8_t* out, uint64_t cap, uint64_t* out_off, uint8_t* status, void* ws, unsigned* err,
                            hipStream_t stream);
size_t firewall_ws_bytes(uint64_t n);
hipError_t launch_firewall(const uint8_t* in, const uint64_t* rec_off, uint64_t n, uint32_t score_table_off,
                           int32_t threshold, int32_t* score, uint8_t* verdict, uint8_t* kept, uint64_t cap,
                           uint64_t* kept_off, uint64_t* kept_index, uint64_t* nkept, void* ws, unsigned* err,
                           hipStream_t stream);

hipError_t launch_encode(const EncodeParams& p, hipStream_t stream);
// Mixed Get/Set batch: one launch -- sizers, scanner and encode tiles over p.flags / p.epoch -- or
// (p.impl == SYM_ENCODE_THREE_KERNEL) size pass, group scan, encode over ws.
size_t encode_mixed_ws_bytes(uint64_t n);  // SYM_ENCODE_THREE_KERNEL's scratch
hipError_t launch_encode_mixed(EncodeParams p, void* ws, hipStream_t stream);
hipError_t launch_decode(const DecodeParams& p, hipStream_t stream);

}  // namespace symhip
