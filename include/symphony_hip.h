/*
 * symphony_hip.h -- C ABI of the MI355X (gfx950) batched Symphony codec.
 *
 * This is the drop-in boundary for aRPC's serializer hot path.  The reference
 * interface it replaces is the per-record Go plugin
 *
 *   type Serializer interface {                     pkg/serializer/serializer.go:3-6
 *       Marshal(msg any) ([]byte, error)
 *       Unmarshal(data []byte, out any) error
 *   }
 *   SymphonySerializer.Marshal   -> msg.(SymphonyMessage).MarshalSymphony()     pkg/serializer/symphony.go:10-12
 *   SymphonySerializer.Unmarshal -> out.(SymphonyMessage).UnmarshalSymphony()   pkg/serializer/symphony.go:14-16
 *
 * whose byte work lives in the generated per-schema methods, e.g.
 * (*SetRequest).MarshalSymphony / UnmarshalSymphony
 * (benchmark/kv-store-symphony/symphony/kv.syn.go:611-678 / :680-745).
 *
 * The reference has no batch API; this ABI is the batched, device-resident form of
 * those methods (one call = n records).  A cgo binding a maintainer would add is
 * shown in INTEGRATION.md.  Only C types cross the boundary: plain pointers, sizes
 * and a `void*` HIP stream (NULL = the legacy default stream).
 *
 * Column layout (struct-of-arrays, caller-owned device memory):
 *   string/bytes field f: a packed byte column `bytes` plus `offs[n+1]` (u64);
 *     record i's value is bytes[offs[i] .. offs[i+1]).  offs[0] need not be 0.
 *   int32 field: an int32 column of n values.
 *   encoded stream: `out` plus `out_off[n+1]`; record i is out[out_off[i] .. out_off[i+1]),
 *     out_off[0] = 0 on encode; rec_off[0] may be nonzero on decode.
 * Decode writes packed columns with offs[0] = 0.
 *
 * Byte parity: with service_id = method_id = 0 the encoded bytes equal the
 * reference MarshalSymphony output; nonzero IDs reproduce the client's on-wire
 * bytes after its in-place patch of [5:13] (pkg/rpc/client.go:267-271).
 * Decode follows UnmarshalSymphony into a fresh struct: skipped fields decode as
 * empty, and the per-record status says which error Go would have returned.
 *
 * Memory rules: every device pointer must be readable up to the 16-byte boundary
 * past its last byte (any hipMalloc / torch allocation is).  Kernels never write
 * outside the bytes the call defines.
 *
 * Threading: a sym_ctx owns a decode workspace; one ctx must not run two calls
 * concurrently.  Create one ctx per host thread / stream.  All entry points are
 * asynchronous on `stream` except the *_host variants and sym_ctx_check.
 */
#ifndef SYMPHONY_HIP_H
#define SYMPHONY_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SYMPHONY_HIP_ABI_VERSION 2

/* Return codes (0 = ok, negative = error); text via sym_last_error(). */
#define SYM_OK 0
#define SYM_ERR_INVALID (-1)  /* bad argument */
#define SYM_ERR_HIP (-2)      /* HIP runtime error */
#define SYM_ERR_NOMEM (-3)    /* device / pinned allocation failed */
#define SYM_ERR_CAPACITY (-4) /* a decode output column was too small (reported by sym_ctx_check) */
#define SYM_ERR_DEVICE (-5)   /* kernel-side fault report, e.g. look-back timeout (sym_ctx_check) */

/* Per-record decode status, the error UnmarshalSymphony would return
 * (benchmark/kv-store-symphony/symphony/kv.syn.go:681-698; examples/echo_symphony/symphony/echo.syn.go:223-231). */
#define SYM_STATUS_OK 0
#define SYM_STATUS_TOO_SHORT 1        /* "invalid data: too short"           */
#define SYM_STATUS_BAD_VERSION 2      /* "invalid data: wrong public version" */
#define SYM_STATUS_NO_PRIVATE 3       /* "missing private segment"           */
#define SYM_STATUS_FIELD_TOO_SHORT 4  /* "invalid data: too short for field" (int32 fields) */
#define SYM_STATUS_NESTED 5           /* "failed to unmarshal nested message" (sym_flat_nested_status) */

/* Flat schemas on the hot path: nfixed int32 fields followed by nvar string fields. */
#define SYM_SCHEMA_KV_GET_REQUEST 0  /* GetRequest{Key}        kv.syn.go:74-185   (0 fixed, 1 var) */
#define SYM_SCHEMA_KV_SET_REQUEST 1  /* SetRequest{Key,Value}  kv.syn.go:611-745  (0 fixed, 2 var) */
#define SYM_SCHEMA_KV_GET_RESPONSE 2 /* GetResponse{Value}     kv.syn.go:333-444  (0 fixed, 1 var) */
#define SYM_SCHEMA_KV_SET_RESPONSE 3 /* SetResponse{Value}     kv.syn.go:963-1074 (0 fixed, 1 var) */
#define SYM_SCHEMA_ECHO_REQUEST 4    /* EchoRequest{Id,Score,Username,Content} echo.syn.go:111-263 (2 fixed, 2 var) */
#define SYM_SCHEMA_ECHO_RESPONSE 5   /* EchoResponse, same fields as EchoRequest (examples/echo_symphony/symphony/echo.proto) */
#define SYM_SCHEMA_COUNT 6

typedef struct sym_ctx sym_ctx;

/* ---- context ---------------------------------------------------------------- */
int sym_abi_version(void);
const char* sym_last_error(void); /* thread-local text of the last error */
int sym_ctx_create(int device, sym_ctx** out_ctx);
int sym_ctx_destroy(sym_ctx* ctx);
/* Pre-size the decode workspace for up to max_records per call (so later calls never allocate). */
int sym_ctx_reserve(sym_ctx* ctx, uint64_t max_records);
/* Synchronize `stream` and report device-side errors of this ctx's calls since the last check
 * (SYM_ERR_CAPACITY, SYM_ERR_INVALID for a batch the kernels cannot place, SYM_ERR_DEVICE); clears them. */
int sym_ctx_check(sym_ctx* ctx, void* stream);
/* Decode implementation of this ctx's decode calls (all produce identical results):
 *   SYM_DECODE_PIPELINE     (default) one launch: parser, scanner and copier workgroups.  A copier
 *                           whose prefix has not arrived within 1 ms resolves it by a look-back that
 *                           never waits, so progress never depends on which workgroups are resident.
 *                           For kv schemas the parsers take each record's lengths from the generator's
 *                           layout and the copiers check them against the exact parse; a second small
 *                           launch on the same stream (no host sync) merges the error bits, or decodes
 *                           the batch again exactly when a record did not follow that layout; the
 *                           ctx then parses exactly for its next 64 decode calls.  Two-field records
 *                           (SetRequest) also take one key length per 64-record tile (the first
 *                           SetRequest's); a tile whose keys differ makes the batch decode again the
 *                           same way, and the ctx then reads every record's own key length for its
 *                           next 1024 decode calls.  Setting the impl clears both holds.
 *   SYM_DECODE_THREE_KERNEL parse -> scan -> copy as three stream-ordered launches (no
 *                           inter-workgroup waiting at all).
 *   SYM_DECODE_LOOKBACK     the pipeline with its parsers and scanner idle: every copier takes the
 *                           look-back path (what the fallback does; slower, for testing it). */
#define SYM_DECODE_PIPELINE 0
#define SYM_DECODE_THREE_KERNEL 1
#define SYM_DECODE_LOOKBACK 2
int sym_ctx_set_decode_impl(sym_ctx* ctx, int impl);
/* Re-decodes the speculative pipeline's gate has run on this ctx so far, after synchronizing `stream`
 * (a test and tuning aid; results are identical either way). */
int sym_ctx_decode_redos(sym_ctx* ctx, void* stream, uint64_t* out);
/* Size-scan implementation of this ctx's mixed Get/Set encodes (sym_encode_kv_mixed; identical results):
 *   SYM_ENCODE_PIPELINE     (default) one launch: sizer workgroups publish every 64-record tile's byte
 *                           total, a scanner workgroup chains them into prefixes, encode workgroups
 *                           wait for theirs (up to 1 ms, then resolve it by a look-back that never waits).
 *   SYM_ENCODE_THREE_KERNEL size pass -> group scan -> encode, three stream-ordered launches.
 *   SYM_ENCODE_LOOKBACK     the one launch without sizers or scanner: every tile looks back (testing). */
#define SYM_ENCODE_PIPELINE 0
#define SYM_ENCODE_THREE_KERNEL 1
#define SYM_ENCODE_LOOKBACK 2
int sym_ctx_set_encode_impl(sym_ctx* ctx, int impl);

/* ---- schema metadata (host-side, no GPU needed) -------------------------------- */
int sym_schema_info(int schema, int* nfixed, int* nvar);
/* Fixed bytes per record: 14 + 4*(nfixed+nvar) + 4*nvar.  A record's size is that plus its string lengths. */
uint64_t sym_record_overhead(int schema);
/* Encoded stream size for n records whose string fields total var_total bytes (all fields). */
uint64_t sym_encoded_size(int schema, uint64_t n, uint64_t var_total);

/* ---- generic columnar entry points (device memory, async on stream) ------------ */
/* d_fixed: nfixed int32 column pointers; d_bytes/d_offs: nvar column pointers (host arrays of device pointers).
 * Replaces n calls of MarshalSymphony (kv.syn.go:611-678) + the client ID patch (client.go:267-271). */
int sym_encode(sym_ctx* ctx, int schema, uint64_t n, const int32_t* const* d_fixed, const uint8_t* const* d_bytes,
               const uint64_t* const* d_offs, uint32_t service_id, uint32_t method_id, uint8_t* d_out,
               uint64_t* d_out_off, void* stream);
/* Replaces n calls of UnmarshalSymphony into fresh structs (kv.syn.go:680-745).  caps[f] = capacity in bytes of
 * d_bytes[f]; rec_off[n]-rec_off[0] always suffices.  d_status: n bytes (SYM_STATUS_*). */
int sym_decode(sym_ctx* ctx, int schema, uint64_t n, const uint8_t* d_in, const uint64_t* d_rec_off,
               int32_t* const* d_fixed, uint8_t* const* d_bytes, const uint64_t* caps, uint64_t* const* d_offs,
               uint8_t* d_status, void* stream);

/* ---- typed entry points (what a cgo binding calls) ------------------------------ */
/* (*SetRequest).MarshalSymphony x n -- kv.syn.go:611-678 */
int sym_encode_kv_set(sym_ctx* ctx, const uint8_t* d_key, const uint64_t* d_key_off, const uint8_t* d_val,
                      const uint64_t* d_val_off, uint64_t n, uint32_t service_id, uint32_t method_id,
                      uint8_t* d_out, uint64_t* d_out_off, void* stream);
/* (*GetRequest).MarshalSymphony x n -- kv.syn.go:74-132 */
int sym_encode_kv_get(sym_ctx* ctx, const uint8_t* d_key, const uint64_t* d_key_off, uint64_t n,
                      uint32_t service_id, uint32_t method_id, uint8_t* d_out, uint64_t* d_out_off, void* stream);
/* (*GetResponse|*SetResponse).MarshalSymphony x n -- kv.syn.go:333-391 / :963-1021 */
int sym_encode_kv_response(sym_ctx* ctx, int schema, const uint8_t* d_val, const uint64_t* d_val_off, uint64_t n,
                           uint32_t service_id, uint32_t method_id, uint8_t* d_out, uint64_t* d_out_off,
                           void* stream);
/* (*EchoRequest).MarshalSymphony x n -- echo.syn.go:111-184 */
int sym_encode_echo(sym_ctx* ctx, const int32_t* d_id, const int32_t* d_score, const uint8_t* d_user,
                    const uint64_t* d_user_off, const uint8_t* d_content, const uint64_t* d_content_off, uint64_t n,
                    uint32_t service_id, uint32_t method_id, uint8_t* d_out, uint64_t* d_out_off, void* stream);
/* (*SetRequest).UnmarshalSymphony x n -- kv.syn.go:680-745 */
int sym_decode_kv_set(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n, uint8_t* d_key,
                      uint64_t key_cap, uint64_t* d_key_off, uint8_t* d_val, uint64_t val_cap, uint64_t* d_val_off,
                      uint8_t* d_status, void* stream);
/* (*GetRequest).UnmarshalSymphony x n -- kv.syn.go:134-185 */
int sym_decode_kv_get(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n, uint8_t* d_key,
                      uint64_t key_cap, uint64_t* d_key_off, uint8_t* d_status, void* stream);
/* (*GetResponse|*SetResponse).UnmarshalSymphony x n -- kv.syn.go:393-444 / :1023-1074 */
int sym_decode_kv_response(sym_ctx* ctx, int schema, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n,
                           uint8_t* d_val, uint64_t val_cap, uint64_t* d_val_off, uint8_t* d_status, void* stream);
/* (*EchoRequest).UnmarshalSymphony x n -- echo.syn.go:186-263 */
int sym_decode_echo(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n, int32_t* d_id,
                    int32_t* d_score, uint8_t* d_user, uint64_t user_cap, uint64_t* d_user_off, uint8_t* d_content,
                    uint64_t content_cap, uint64_t* d_content_off, uint8_t* d_status, void* stream);

/* ---- mixed GetRequest / SetRequest batches (the kv-store's request stream) -------------
 * One batch of records of both types, in any order: d_type[i] == 0 is a GetRequest{Key}
 * (kv.syn.go:74-185, 22 + K bytes), any other value a SetRequest{Key, Value} (:611-745, 30 + K + V).
 * Columns as above; a GetRequest's value slice is not part of its record (it is normally empty, and
 * decode writes it empty).  Record sizes depend on the type, so the record offsets are a device-wide
 * scan (a size pass over the type column, a scan of its group totals, then the encode); d_out must hold
 * sym_encoded_size_kv_mixed(...) bytes.  The client's ID patch writes get_method_id into GetRequests
 * and set_method_id into SetRequests (KVService: service 1, Get 1, Set 2, kv_arpc.syn.go:11-28);
 * 0/0/0 reproduces MarshalSymphony.  Decode takes the type column the server's method dispatch
 * produced (pkg/rpc/server.go:104-153) and unmarshals each record as its type. */
uint64_t sym_encoded_size_kv_mixed(uint64_t n, uint64_t n_set, uint64_t key_total, uint64_t set_value_total);
int sym_encode_kv_mixed(sym_ctx* ctx, const uint8_t* d_type, const uint8_t* d_key, const uint64_t* d_key_off,
                        const uint8_t* d_val, const uint64_t* d_val_off, uint64_t n, uint32_t service_id,
                        uint32_t get_method_id, uint32_t set_method_id, uint8_t* d_out, uint64_t* d_out_off,
                        void* stream);
int sym_decode_kv_mixed(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, const uint8_t* d_type,
                        uint64_t n, uint8_t* d_key, uint64_t key_cap, uint64_t* d_key_off, uint8_t* d_val,
                        uint64_t val_cap, uint64_t* d_val_off, uint8_t* d_status, void* stream);

/* ---- host-memory entry points (synchronous) -------------------------------------
 * Same contracts with every pointer in host memory: what the per-record Go Serializer adapter and
 * the UDP buffers of pkg/transport hand over.  The batch moves through the GPU in record chunks of
 * about 32 MiB in three slots of the ctx over one stream per direction (H2D copies and kernels on one,
 * D2H copies on the other), so one chunk's H2D and kernel overlap another's D2H.  Host memory that is pinned (sym_host_alloc, hipHostMalloc, a hipHostRegister'ed
 * range) is transferred by DMA in place; pageable memory is staged through the ctx's pinned buffers
 * with a host copy.  sym_decode_host: caps[f] is the capacity of h_bytes[f]; a column that does not
 * fit returns SYM_ERR_CAPACITY with the bytes that fit written.  Device-side errors of the chunks
 * are returned (no sym_ctx_check needed). */
int sym_host_alloc(sym_ctx* ctx, uint64_t bytes, void** out); /* pinned host memory (hipHostMalloc) */
int sym_host_free(sym_ctx* ctx, void* p);
int sym_encode_host(sym_ctx* ctx, int schema, uint64_t n, const int32_t* const* h_fixed,
                    const uint8_t* const* h_bytes, const uint64_t* const* h_offs, uint32_t service_id,
                    uint32_t method_id, uint8_t* h_out, uint64_t* h_out_off);
int sym_decode_host(sym_ctx* ctx, int schema, uint64_t n, const uint8_t* h_in, const uint64_t* h_rec_off,
                    int32_t* const* h_fixed, uint8_t* const* h_bytes, const uint64_t* caps, uint64_t* const* h_offs,
                    uint8_t* h_status);

/* ---- coalescing batcher: the per-record Serializer path (SURVEY.md 8b "Threading") --------
 * The reference Serializer takes ONE record per call, concurrently from many goroutines:
 *   Marshal   client Call per request  pkg/rpc/client.go:233-310 (:252), server reply :173
 *   Unmarshal server receive loop      pkg/rpc/server.go:152, client response  client.go:205
 *   adapter                            pkg/serializer/symphony.go:10-16
 * A batcher serves those concurrent one-record calls without a launch per call.  Records of up to
 * 4000 bytes (encode: the fields' bytes; decode: the record) go through a ring of 256 slots in
 * coherent pinned host memory, one ring per DEVICE shared by all its batchers and both
 * directions: the caller writes its record into a slot and publishes it, a persistent kernel (one
 * launch of four workgroups; started with the device's first batcher, restarted by the next call after it leaves)
 * serves whatever is published in place and sets the slot's done flag, and the caller copies its
 * result out -- a few microseconds per call, many calls per pass under load.  Queue budget: that
 * kernel holds one hardware queue of the process (GPU_MAX_HW_QUEUES, 4 by default) while it runs,
 * and a launch of another stream that maps to the same queue waits behind it; so the worker hands
 * over to a fresh launch every 2 ms (busy or idle, and leaves for good after 20 ms without records),
 * and such a launch (the caller's own kernels, hipDeviceSynchronize / torch.cuda.synchronize, a
 * batch of large records) waits at most about that long.  sym_batcher_quiesce stops the worker at
 * once (it returns when the worker has left; the next call restarts it), e.g. before a device-wide
 * synchronisation.  Larger records join the open batch of their
 * direction and block; when no batch of that direction is on the GPU, one caller of the open batch
 * runs it (no extra thread): at once with max_wait_us = 0 -- under load a batch is whatever
 * arrived while the previous one ran -- else once it holds max_records records or max_bytes bytes
 * of records or its first record has waited max_wait_us; every caller then copies its own result
 * out.  All entry points are thread-safe.  The batcher owns two contexts on `device` (one per
 * direction), a reference to the device's ring, and pinned staging that the batch kernels read and
 * write in place (mapped host memory), so one batch is one kernel launch and one stream
 * synchronisation.  Results are bit-identical to sym_encode / sym_decode of the same records.
 * sym_batcher_stats counts the ring worker's passes that served this batcher's records as batches
 * (in completion order: an upper bound).
 *   sym_batcher_encode_one  MarshalSymphony of one record + the client's ID patch of bytes [5:13]
 *                           (service_id / method_id; 0 / 0 = MarshalSymphony's own bytes):
 *                           fixed[nfixed] int32 values, fields[nvar] pointers with lens[nvar]; out
 *                           receives sym_encoded_size(schema, 1, sum(lens)) bytes (*out_len; a
 *                           smaller out_cap returns SYM_ERR_CAPACITY with *out_len set).
 *   sym_batcher_decode_one  UnmarshalSymphony of data[0, len) into a fresh struct: fixed[nfixed],
 *                           field f's bytes into fields[f] (caps[f] bytes; len always suffices) and
 *                           lens[f]; *status = SYM_STATUS_* (a malformed record is SYM_OK with its
 *                           status, as Go returns an error value); a field longer than its cap
 *                           returns SYM_ERR_CAPACITY with the bytes that fit copied.
 * A record larger than max_bytes is SYM_ERR_INVALID.  The caller's memory is read and written only
 * during the call (cgo's pointer rules hold: nothing is kept after return).
 * At most 256 batchers exist per device and process at once (they share the device's record ring,
 * which counts each one's passes); sym_batcher_create beyond that returns SYM_ERR_INVALID (the
 * message says so) until one is destroyed. */
typedef struct sym_batcher sym_batcher;
int sym_batcher_create(int device, int schema, uint32_t max_records, uint64_t max_bytes, uint32_t max_wait_us,
                       sym_batcher** out);
int sym_batcher_destroy(sym_batcher* b); /* no call on b may be in progress; the device's last batcher stops
                                          * the ring worker */
int sym_batcher_quiesce(sym_batcher* b); /* stop the device's ring worker now; the next call restarts it */
int sym_batcher_encode_one(sym_batcher* b, const int32_t* fixed, const uint8_t* const* fields, const uint64_t* lens,
                           uint32_t service_id, uint32_t method_id, uint8_t* out, uint64_t out_cap,
                           uint64_t* out_len);
int sym_batcher_decode_one(sym_batcher* b, const uint8_t* data, uint64_t len, int32_t* fixed, uint8_t* const* fields,
                           const uint64_t* caps, uint64_t* lens, uint8_t* status);
/* batches run and records carried, per direction (any pointer may be NULL) */
int sym_batcher_stats(sym_batcher* b, uint64_t* enc_batches, uint64_t* enc_records, uint64_t* dec_batches,
                      uint64_t* dec_records);

/* ---- packetization: aRPC's send side over a batch of marshalled records ----------
 * What UDPTransport.Send does to one message (pkg/transport/transport.go:146-201), for n records:
 * FragmentPackets(data, max_udp_payload - 31) (pkg/transport/symphony_fragmentation.go:23-125), then
 * one serialized DataPacket per fragment (pkg/packet/builtin_packets.go:59-114): a 31-byte
 * little-endian header {type, rpc_id, TotalPackets = uint16(#fragments), SeqNumber = uint16(index),
 * MoreFragments = 0, FragmentIndex = 0, dst ip/port, src ip/port, payload length} and the fragment.
 * The wire output is every datagram back to back, record after record, datagram j at
 * wire[dg_off[j] .. dg_off[j+1]): the byte strings Send passes to WriteToUDP, in order.
 * Two calls, because the output size depends on the data:
 *   sym_fragment_plan   first[n+1]: datagrams before record i ([n] = total datagrams);
 *                       wire_off[n+1]: wire bytes before record i ([n] = total bytes);
 *                       status[n]: SYM_FRAG_* (a failed record emits nothing, as Send returns
 *                       the error before sending).
 *   sym_fragment_write  the datagrams, and dg_off[first[n] + 1]. */
#define SYM_MAX_UDP_PAYLOAD 1400 /* MaxUDPPayloadSize, pkg/packet/codec.go:10 */
#define SYM_DATA_PACKET_HEADER 31
#define SYM_PACKET_REQUEST 1  /* PacketTypeRequest, builtin_packets.go:15 */
#define SYM_PACKET_RESPONSE 2 /* PacketTypeResponse, builtin_packets.go:16 */
#define SYM_FRAG_OK 0
#define SYM_FRAG_TOO_SHORT 1  /* "data too short for offset header" (symphony_fragmentation.go:33-35) */
#define SYM_FRAG_BAD_OFFSET 2 /* "invalid offset" (symphony_fragmentation.go:37-39) */

typedef struct sym_endpoints {
    uint8_t dst_ip[4]; /* IPv4 bytes as in the packet (e.g. 127,0,0,1) */
    uint16_t dst_port;
    uint8_t src_ip[4];
    uint16_t src_port;
} sym_endpoints;

int sym_fragment_plan(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n,
                      uint32_t max_udp_payload, uint64_t* d_first, uint64_t* d_wire_off, uint8_t* d_status,
                      void* stream);
int sym_fragment_write(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n,
                       uint32_t max_udp_payload, uint8_t packet_type, const uint64_t* d_rpc_id,
                       const sym_endpoints* endpoints, const uint64_t* d_first, const uint64_t* d_wire_off,
                       const uint8_t* d_status, uint8_t* d_wire, uint64_t* d_dg_off, void* stream);

/* ---- Batched Raw getters and the proxy firewall element -----------------
 *
 * Replaces, for n buffers at once, the generated zero-copy getters
 *   func (m XxxRaw) GetField() T       cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:984-1036
 *     fixed-width                      main.go:1260-1294
 *     string / bytes                   main.go:1517-1565
 *   e.g. GetRequestRaw.GetScore / GetUsername
 *                                      benchmark/kv-store-symphony-element/symphony/kv.syn.go:285-310
 * and the proxy's firewall element
 *   func (f *FirewallElement) ProcessRequest(ctx, packet) (*BufferedPacket, PacketVerdict, ctx, error)
 *                                      cmd/proxy/element/firewall.go:39-52
 * Buffers are a batch as elsewhere: d_in + d_rec_off[n+1] (buffer i = d_in[rec_off[i], rec_off[i+1]);
 * offsets non-decreasing); a buffer may be a complete record or only its public segment.
 *
 * `segment` / `table_off` name the field as the generator does: SYM_SEGMENT_PUBLIC with the absolute
 * table offset (public fields start at 13), or SYM_SEGMENT_PRIVATE with the offset relative to the
 * private segment (private fields start at 1); each field advances the offset by its width (fixed) or
 * 4 (string / bytes) -- main.go:986-989, 1243-1257.
 *
 *   sym_raw_get_fixed   width 1 (bool), 4 (int32/uint32/float/enum) or 8 (int64/uint64/double);
 *                       d_out[n] of `width` bytes each, little-endian; a short buffer reads 0.
 *   sym_raw_get_bytes   the values back to back in d_out (at most out_cap bytes, else
 *                       SYM_ERR_CAPACITY from sym_ctx_check and nothing written) with
 *                       d_out_off[n+1]; an unset, truncated or out-of-range value reads empty.
 *   d_status[n] (nullable): SYM_RAW_OK, or for private fields the buffer assertion Go panics on
 *                       (main.go:1003-1013) -- the value then reads as zero / empty.
 *   sym_firewall_filter score = GetScore (public int32 at score_table_off, 13 for the element
 *                       schemas); verdict SYM_VERDICT_DROP when score >= block_threshold, else
 *                       SYM_VERDICT_PASS; the passing buffers, unchanged and in order, back to back
 *                       in d_kept (kept_cap >= rec_off[n] - rec_off[0] always suffices) with
 *                       d_kept_off[nkept+1] (room for n+1), d_kept_index[nkept] (nullable) and
 *                       *d_nkept, all on the device. */
#define SYM_SEGMENT_PUBLIC 0
#define SYM_SEGMENT_PRIVATE 1
#define SYM_PUBLIC_TABLE_START 13
#define SYM_PRIVATE_TABLE_START 1
#define SYM_RAW_OK 0
#define SYM_RAW_INVALID_BUFFER 1 /* "private getter called on invalid buffer" (len < 5) */
#define SYM_RAW_PUBLIC_ONLY 2    /* "private getter called on public-only buffer" */
#define SYM_VERDICT_PASS 1       /* util.PacketVerdictPass, cmd/proxy/util/packet.go:57-58 */
#define SYM_VERDICT_DROP 2       /* util.PacketVerdictDrop, cmd/proxy/util/packet.go:60-61 */

int sym_raw_get_fixed(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n, int segment,
                      uint32_t table_off, uint32_t width, void* d_out, uint8_t* d_status, void* stream);
int sym_raw_get_bytes(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n, int segment,
                      uint32_t table_off, uint8_t* d_out, uint64_t out_cap, uint64_t* d_out_off, uint8_t* d_status,
                      void* stream);
int sym_firewall_filter(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n,
                        uint32_t score_table_off, int32_t block_threshold, int32_t* d_score, uint8_t* d_verdict,
                        uint8_t* d_kept, uint64_t kept_cap, uint64_t* d_kept_off, uint64_t* d_kept_index,
                        uint64_t* d_nkept, void* stream);

/* ---- Receive-side reassembly of DataPackets -------------------------------
 *
 * Replaces, for n datagrams in arrival order, the per-datagram receive path
 *   func (t *UDPTransport) Receive(bufferSize, role) ([]byte, *net.UDPAddr, uint64, PacketType, error)
 *                                      pkg/transport/transport.go:253-317 (parse and route)
 *   func (c *DataPacketCodec) Deserialize(data []byte) (any, error)
 *                                      pkg/packet/builtin_packets.go:118-161
 *   func (r *DataReassembler) ProcessFragment(pkt, addr, buffer) ([]byte, *net.UDPAddr, uint64, bool)
 *                                      pkg/transport/fragmentation.go:49-183
 * with the reassembler starting empty.  Input: d_wire + d_dg_off[n+1] (datagram j =
 * wire[dg_off[j], dg_off[j+1])), e.g. the output of sym_fragment_write.  Output, in the order the
 * one-at-a-time loop returns them: the completed messages back to back in d_msg (msg_cap bytes;
 * the batch's payload bytes always suffice, else SYM_ERR_CAPACITY from sym_ctx_check),
 * d_msg_off[nmsg+1], d_msg_rpc[nmsg] (RPCID) and d_msg_dg[nmsg] (arrival index of the completing
 * datagram: its header carries the packet type and addresses Receive returns); *d_nmsg; all
 * arrays sized for n messages (n+1 offsets).  d_status[n]: SYM_RX_*.  n < 2^31.
 * When every DataPacket is a whole message (TotalPackets 1, one fragment) the messages are the
 * DataPackets in arrival order; when every datagram is a DataPacket, the RPCIDs never decrease and
 * each run of equal RPCIDs is one message as sym_fragment_write sends it (sequence numbers 0..k-1
 * in order, TotalPackets k, one fragment each), the messages are the runs in arrival order.  Both
 * are found on the device without grouping.  The general path -- grouping, sort, the
 * ProcessFragment state machine -- is queued too and its kernels exit at once for such a batch:
 * the call is asynchronous on `stream` like the others (no host read).  It runs on a stream of the
 * ctx forked from `stream` after the parse and joined back before the call's last operation
 * (events; stream capture follows both). */
#define SYM_RX_CONSUMED 0   /* part of a returned message */
#define SYM_RX_PENDING 1    /* still held by the reassembler after the batch */
#define SYM_RX_NOT_DATA 2   /* not a Request / Response DataPacket: not reassembled */
#define SYM_RX_TOO_SHORT 3  /* empty, or shorter than the 31-byte DataPacket header */
#define SYM_RX_BAD_LENGTH 4 /* "data too short for declared payload length" */

int sym_reassemble(sym_ctx* ctx, const uint8_t* d_wire, const uint64_t* d_dg_off, uint64_t n, uint8_t* d_msg,
                   uint64_t msg_cap, uint64_t* d_msg_off, uint64_t* d_msg_rpc, uint64_t* d_msg_dg, uint64_t* d_nmsg,
                   uint8_t* d_status, void* stream);

/* ---- Per-segment AES-256-GCM of Symphony records --------------------------
 *
 * Replaces, for n records at once,
 *   func EncryptSymphonyData(data, publicKey, privateKey []byte) []byte
 *   func DecryptSymphonyData(data, publicKey, privateKey []byte) []byte
 *                                      pkg/transport/encryption.go:82-256 (segments sealed by
 *                                      encryptSegmentWithNonce / opened by decryptSegment, :262-335)
 * The public segment data[13:offsetToPrivate] is sealed under pub_key, the private segment
 * data[offsetToPrivate:] (version byte included) under priv_key, each as nonce(12) || ciphertext ||
 * tag(16) (AES-256-GCM, no additional data); offsetToPrivate is rewritten.  Keys are 32 bytes (host
 * memory); their key schedule and GHASH tables are built on the host and cached in the ctx.
 *   sym_encrypt  d_nonces: 24 bytes per record (public nonce, then private), device memory -- the
 *                random nonces of encryption.go:115-121 made an input.  Output record i has
 *                len + 28 (+ 28 with a private segment) bytes.
 *   sym_decrypt  output record i has len - 28 (- 28) bytes; a record failing authentication or the
 *                private version check keeps that size and is zero-filled.
 * Both: d_out_off[n+1] (output offsets, computed on the device); d_out must hold d_out_off[n]
 * bytes (<= in bytes + 56 n for sym_encrypt, <= in bytes for sym_decrypt); d_status[n]: SYM_CRYPT_*
 * (where Go panics on the one message).  A record with a header error has no output. */
#define SYM_CRYPT_OK 0
#define SYM_CRYPT_TOO_SHORT 1    /* "too short for header" */
#define SYM_CRYPT_BAD_OFFSET 2   /* "invalid offsetToPrivate" / "invalid encrypted offsetToPrivate" */
#define SYM_CRYPT_AUTH_PUBLIC 3  /* public segment: "message authentication failed" */
#define SYM_CRYPT_AUTH_PRIVATE 4 /* private segment: shorter than nonce + tag, or authentication failed */
#define SYM_CRYPT_BAD_VERSION 5  /* "invalid decrypted private segment: missing or incorrect version byte" */
#define SYM_GCM_OVERHEAD 28      /* nonce (12) + tag (16) per segment */

int sym_encrypt(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n, const uint8_t* pub_key,
                const uint8_t* priv_key, const uint8_t* d_nonces, uint8_t* d_out, uint64_t* d_out_off,
                uint8_t* d_status, void* stream);
int sym_decrypt(sym_ctx* ctx, const uint8_t* d_in, const uint64_t* d_rec_off, uint64_t n, const uint8_t* pub_key,
                const uint8_t* priv_key, uint8_t* d_out, uint64_t* d_out_off, uint8_t* d_status, void* stream);

/* ---- Any flat schema (the flat part) ----------------------------------------
 *
 * The generated MarshalSymphony / UnmarshalSymphony of a message whose fields are fixed-width or
 * string / bytes, each public or private (generator cmd/symphony-gen-arpc/protoc-gen-symphony/
 * main.go:196-368, 439-620 marshal; :622-800 unmarshal), described at run time: fields[k] in
 * declaration order, `segment` SYM_SEGMENT_PUBLIC / SYM_SEGMENT_PRIVATE, `width` 1 (bool),
 * 4 (int32 / uint32 / float / enum), 8 (int64 / uint64 / double) or 0 (string / bytes), or
 * SYM_FIELD_REPEATED | 1 / 4 / 8 for a repeated fixed-width field (`repeated int32 xs`: a 4-byte
 * table entry, then a u32 element count and the elements, main.go:493-535 / :795-841).
 * Repeated string / bytes and nested messages: the _ex entry points below.  Columns are indexed by field: d_cols[k] is n
 * little-endian values of `width` bytes (fixed, `width`-aligned) or the packed bytes (string and
 * repeated fixed, with d_offs[k] its n+1 BYTE offsets; a repeated field's record lengths must be
 * multiples of its element width -- the count written is length / width; d_offs[k] is ignored
 * for scalar fields).  Bool values (scalar or repeated) are the wire byte, read as `!= 0`.  The
 * kv-store and echo schemas above are the all-private cases of this (and keep their specialised kernels).
 *   sym_flat_encode  output record i = MarshalSymphony + the client's ID patch; d_out holds
 *                    sym_flat_encoded_size(...) bytes; d_out_off[n+1] computed on the device.
 *                    A run of 64 records spanning 2 GiB or more is reported by sym_ctx_check as
 *                    SYM_ERR_INVALID ("64 consecutive records span >= 2 GiB").
 *   sym_flat_decode  UnmarshalSymphony into fresh structs: fixed columns (zero when not read),
 *                    string columns of caps[k] bytes (rec_off[n] - rec_off[0] always suffices)
 *                    with d_offs[k][n+1]; d_status[n] SYM_STATUS_*. */
#define SYM_MAX_FLAT_FIELDS 16
#define SYM_FIELD_REPEATED 0x80 /* or'ed into sym_field.width: repeated fixed-width field */
#define SYM_FIELD_MESSAGE 0x40  /* nested message; | SYM_FIELD_REPEATED: repeated message (sym_flat_*_ex) */
#define SYM_FIELD_FRAMED 0x20   /* | SYM_FIELD_MESSAGE, encode: the items already carry their [u32 len] (the
                                   inner level was encoded with framed output, sym_flat_encode_opts) */

typedef struct sym_field {
    uint8_t segment; /* SYM_SEGMENT_PUBLIC / SYM_SEGMENT_PRIVATE */
    uint8_t width;   /* 1, 4, 8, or 0 for string / bytes; SYM_FIELD_REPEATED | 1/4/8 for repeated */
} sym_field;

uint64_t sym_flat_encoded_size(const sym_field* fields, int nfields, uint64_t n, uint64_t var_total);

/* ---- Repeated string / bytes and nested messages (the rest) -----------------
 * List-like fields (generator main.go:537-620 marshal, :843-947 unmarshal):
 *   width SYM_FIELD_REPEATED            repeated string / bytes: [u32 count] then per item [u32 len][bytes]
 *   width SYM_FIELD_MESSAGE             nested message: [u32 len][inner MarshalSymphony] when set, and a
 *                                       0 table entry with no payload when nil
 *   width SYM_FIELD_REPEATED | SYM_FIELD_MESSAGE   repeated message: as repeated bytes, the items being
 *                                       inner MarshalSymphony outputs
 * A message field is one level: its items are the inner messages' bytes, produced (encode) or
 * consumed (decode) by calls on the inner schema -- the caller walks the message tree
 * (arpc_amd/flat.py does).  For a list-like field k, d_cols[k] holds the items' bytes,
 * d_items[k] their byte offsets (m_k + 1 entries, into d_cols[k]) and d_offs[k] each record's item
 * range (n + 1 item indices: record i has items [d_offs[k][i], d_offs[k][i+1])).  A nested
 * (non-repeated) field has at most one item per record: none = nil.  Other fields as above.
 *   sym_flat_encoded_size_ex  exact output size: bytes[k] = payload bytes of field k (strings and
 *                    repeated fixed: their column bytes; list-like: item bytes), items[k] = items of a
 *                    list-like field (nested: records where it is set).
 *   sym_flat_encode_ex  as sym_flat_encode; list bodies ([count], then [u32 len][item] per item)
 *                    are written by the same output-stationary kernel.  More than one item for a
 *                    nested field is SYM_ERR_INVALID from sym_ctx_check.  `opts` (nullable: IDs 0,
 *                    nothing else) -- see sym_flat_encode_opts.
 *   sym_flat_decode_ex  as sym_flat_decode; list-like field k: item bytes into d_cols[k] (caps[k]),
 *                    item offsets into d_items[k] (item_caps[k] + 1 entries) and record item ranges
 *                    into d_offs[k] (n + 1).  A list keeps the items that fit in the record, in order
 *                    (Go's loop stops making progress at the first that does not).  d_fail (n bytes,
 *                    nullable): the unmarshal position (public fields in order, then private) of
 *                    the field where decoding stopped, nfields when it did not.
 *                    Records in place: record i is d_in[d_rec_src[i], d_rec_src[i] + d_rec_len[i])
 *                    (d_rec_len NULL: contiguous, d_rec_src is d_rec_off), and d_in's readable extent
 *                    is [*d_lo, *d_hi) (device values; both NULL: d_rec_src[0], d_rec_src[n]; required
 *                    with d_rec_len).  For a message field k with d_item_len[k] non-NULL no item bytes
 *                    are written: d_items[k][j] receives item j's offset into d_in and d_item_len[k][j]
 *                    its length, and the inner level is decoded from there (d_rec_src = d_items[k],
 *                    d_rec_len = d_item_len[k], the same d_in), so a tree decodes without copying
 *                    inner messages out.  Record count on the device: d_n (nullable) holds it and n is
 *                    its capacity (an inner level of a tree walk, whose count is the outer level's
 *                    item count from sym_flat_list_sizes); columns are sized for the capacity and
 *                    every launch strides over the tiles of the count, so a tree decodes with no host
 *                    read until its end.
 *   sym_flat_nested_status  after decoding message fields ks[q] (q < nk; their items' statuses
 *                    d_item_status[q], item ranges d_rec_items[q]) with the inner schemas, marks the
 *                    records that reached the field and have a failed item SYM_STATUS_NESTED (Go
 *                    returns "failed to unmarshal nested message" there), all nk fields in one launch;
 *                    d_fail is updated, so fields can be folded in in any order.  Field values of a
 *                    record with a non-OK status are unspecified beyond the fields before the failing
 *                    one (Go callers discard the struct on error).  d_n as in sym_flat_decode_ex.
 *   sym_flat_list_sizes  after sym_flat_decode_ex, for `nl` list-like fields (record item ranges
 *                    d_recs[i], n + 1 entries; item offsets d_items[i], item_caps[i] + 1): item count
 *                    m_i = d_recs[i][n] - d_recs[i][0] (clamped to item_caps[i]) and item bytes
 *                    d_items[i][m_i] into d_out[2i], d_out[2i + 1] (device memory), in one launch,
 *                    so a host walking a message tree reads back one small array at the end.  d_n as
 *                    in sym_flat_decode_ex. */
#define SYM_FRAME_PREFIX_MAX 24
/* Options of sym_flat_encode_ex (all zero: MarshalSymphony with service / method IDs 0).
 *   framed         nonzero: each record is written as [frame_prefix][u32 size][record] (an inner level
 *                  of a tree walk: [u32 size][record] is what the outer level's body holds for one item,
 *                  so an outer message field takes the items with SYM_FIELD_FRAMED and its bodies become
 *                  one window each); d_out_off are the frames' offsets
 *   frame_prefix   framed only: frame_prefix_len (<= SYM_FRAME_PREFIX_MAX) constant bytes before each
 *                  frame.  A message whose one field is a private nested message (a wrapper such as
 *                  online-boutique's PlaceOrderResponse{Order}) is, when every record has its item,
 *                  exactly 18 constant bytes (header, marker, table entry 5) before the item's frame:
 *                  with them as the prefix the inner level's kernel writes the wrapper level itself
 *                  and the wrapper's own launch copies nothing (arpc_amd/flat.py)
 *   string_bytes   the caller's estimate of the string / bytes fields' payload bytes (0: unknown); a
 *                  level of short strings is then written with more payload windows per 16-byte chunk
 *   d_gate_rec     nullable, device memory: the launch does its work only when
 *                  (d_gate_rec[gate_n] - d_gate_rec[0] == gate_n) equals (gate_when_all != 0), and
 *                  otherwise leaves every output untouched -- a condition on device data (a nested
 *                  field's item ranges: is every record's item present?) that lets a tree walk queue
 *                  both alternatives without a host read */
typedef struct sym_flat_encode_opts {
    uint32_t service_id, method_id;
    uint32_t framed;
    uint32_t frame_prefix_len;
    uint8_t frame_prefix[SYM_FRAME_PREFIX_MAX];
    uint64_t string_bytes;
    const uint64_t* d_gate_rec;
    uint64_t gate_n;
    uint32_t gate_when_all;
    uint32_t reserved;
} sym_flat_encode_opts;

uint64_t sym_flat_encoded_size_ex(const sym_field* fields, int nfields, uint64_t n, const uint64_t* bytes,
                                  const uint64_t* items);
int sym_flat_encode_ex(sym_ctx* ctx, const sym_field* fields, int nfields, uint64_t n, const void* const* d_cols,
                       const uint64_t* const* d_offs, const uint64_t* const* d_items, const sym_flat_encode_opts* opts,
                       uint8_t* d_out, uint64_t* d_out_off, void* stream);
int sym_flat_decode_ex(sym_ctx* ctx, const sym_field* fields, int nfields, uint64_t n, const uint64_t* d_n,
                       const uint8_t* d_in, const uint64_t* d_rec_src, const uint64_t* d_rec_len, const uint64_t* d_lo,
                       const uint64_t* d_hi, void* const* d_cols, const uint64_t* caps, uint64_t* const* d_offs,
                       uint64_t* const* d_items, uint64_t* const* d_item_len, const uint64_t* item_caps,
                       uint8_t* d_status, uint8_t* d_fail, void* stream);
int sym_flat_nested_status(sym_ctx* ctx, const sym_field* fields, int nfields, int nk, const int* ks, uint64_t n,
                           const uint64_t* d_n, const uint64_t* const* d_rec_items,
                           const uint8_t* const* d_item_status, uint8_t* d_status, uint8_t* d_fail, void* stream);
int sym_flat_list_sizes(sym_ctx* ctx, int nl, uint64_t n, const uint64_t* d_n, const uint64_t* const* d_recs,
                        const uint64_t* const* d_items, const uint64_t* item_caps, uint64_t* d_out, void* stream);

/* ---- Batched Raw setters ----------------------------------------------------
 * XxxRaw.SetF(v_i) on buffer i of a flat schema (generator main.go:1038-1093 assertions,
 * :1296-1336 fixed, :1567-1620 string / bytes, :1685-1740 repeated fixed, :371-437 remarshal;
 * e.g. GetRequestRaw.SetScore / SetUsername / SetKey, kv-store-symphony-element kv.syn.go:340-412).
 * fields[field] is the field set.  Values: a fixed field takes n values of its width in d_val
 * (d_val_off ignored); a string / bytes field takes d_val[d_val_off[i], d_val_off[i+1]); a repeated
 * field takes its element bytes the same way.  Fixed fields and payloads that are not longer than the
 * old ones are written in place (the old tail stays as slack); otherwise the message is
 * remarshalled -- a public field through a fake private segment, keeping the public part and bytes
 * [5:13]; a private field into a complete message whose [5:13] are 0, as MarshalSymphony writes them.
 * Every buffer goes to d_out (sizes may change) with d_out_off[n+1]; a buffer whose setter would
 * panic or fail is copied unchanged and d_status[i] says why.  d_out must hold the result: a bound
 * is sum((nvar + 1) * len_i + G) + the new value bytes, G = 14 + tables + 4 * nvar (for well-formed
 * buffers sum(len_i + G) + new bytes); past out_cap buffers are not written and sym_ctx_check
 * reports SYM_ERR_CAPACITY. */
#define SYM_SET_OK 0
#define SYM_SET_COMPLETE_BUFFER 1 /* panic "public setter ... called on complete buffer" */
#define SYM_SET_INVALID_BUFFER 2  /* panic "private setter ... called on invalid buffer" (len < 5) */
#define SYM_SET_PUBLIC_ONLY 3     /* panic "private setter ... called on public-only buffer" */
#define SYM_SET_TOO_SHORT 4       /* error "buffer too short" / "buffer too short for table entry" */
#define SYM_SET_UNMARSHAL 5       /* error "failed to unmarshal: ..." (remarshal path) */
#define SYM_SET_BOUNDS 6          /* Go panics with an index out of range (in-place write, fake segment) */
#define SYM_SET_BAD_LENGTH 7      /* batch convention: a repeated field's value bytes are not a whole number of
                                     elements (Go's typed setters cannot express it; sym_flat_encode reports
                                     the same input as SYM_ERR_INVALID); the buffer is copied unchanged */
int sym_raw_set(sym_ctx* ctx, const sym_field* fields, int nfields, int field, const uint8_t* d_in,
                const uint64_t* d_rec_off, uint64_t n, const void* d_val, const uint64_t* d_val_off, uint8_t* d_out,
                uint64_t out_cap, uint64_t* d_out_off, uint8_t* d_status, void* stream);
int sym_flat_encode(sym_ctx* ctx, const sym_field* fields, int nfields, uint64_t n, const void* const* d_cols,
                    const uint64_t* const* d_offs, uint32_t service_id, uint32_t method_id, uint8_t* d_out,
                    uint64_t* d_out_off, void* stream);
int sym_flat_decode(sym_ctx* ctx, const sym_field* fields, int nfields, uint64_t n, const uint8_t* d_in,
                    const uint64_t* d_rec_off, void* const* d_cols, const uint64_t* caps, uint64_t* const* d_offs,
                    uint8_t* d_status, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SYMPHONY_HIP_H */
