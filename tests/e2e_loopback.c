/*
 * e2e_loopback.c -- C stand-in for the aRPC client/server pair of BASELINE.json config 5 (there is
 * no Go toolchain here or on the GPU box, so aRPC itself cannot run): kv-store Set RPCs over UDP
 * loopback with the HIP Symphony codec on both sides, every byte through the C ABI a cgo binding
 * would call.  This is a harness, not a re-implementation of aRPC's transport: no reliability
 * layer, no timers, one client and one server process.
 *
 * The reference pair it stands in for:
 *   client  frontend.go:109 (SymphonySerializer injected), rpc.Client.Call (pkg/rpc/client.go:233-310):
 *           Marshal the request, patch service / method IDs into bytes [5:13] (client.go:267-271),
 *           UDPTransport.Send (pkg/transport/transport.go:110-244): FragmentPackets + DataPacket
 *           headers, one WriteToUDP per datagram; then Receive + reassembly of the response and
 *           Unmarshal (client.go:205)
 *   server  rpc.Server.Start (pkg/rpc/server.go:81-189): Receive + DataReassembler, the IDs read from
 *           bytes [5:13], Unmarshal (server.go:152), the kv handler (kvstore.go:58-82: SetResponse
 *           {Value: value}), Marshal (server.go:173), Send as PacketTypeResponse
 * Here, per batch of RPCs, on the device:
 *   client  H2D request columns -> sym_encode_kv_set (service 1, Set 2) -> sym_fragment_plan/_write
 *           (PacketTypeRequest) -> D2H datagrams -> sendmmsg;  recvmmsg -> H2D -> sym_reassemble ->
 *           sym_decode_kv_response -> D2H values (checked against the request's value)
 *   server  recvmmsg -> H2D -> sym_reassemble -> sym_decode_kv_set -> D2H key / value columns ->
 *           handler on the host (the IDs checked, the fields checked against the generator, the
 *           response value = the request value) -> H2D -> sym_encode_kv_response (SetResponse) ->
 *           sym_fragment_plan/_write (PacketTypeResponse, the request's RPCIDs) -> D2H -> sendmmsg
 * Both processes bind 127.0.0.1 explicitly (the reference's own note on the loopback hazard,
 * transport.go:46-56).  The server is forked before either process makes a HIP call.  Datagrams of
 * a message that is still incomplete after a batch (PENDING) are carried into the next batch, as
 * the reference's reassembler keeps them.  Requests go out `window` RPCs at a time, up to `inflight`
 * windows ahead of the responses (the client's concurrent Calls), sized to the socket buffers so
 * that loopback drops nothing; a datagram lost anyway ends the run with an error, not a hang.
 *
 *   e2e_loopback RPCS WINDOW KEY VAL [INFLIGHT [DUMP_FILE]]
 *     prints one JSON line: RPC rate and the codec's algorithmic bytes per second, host clock
 *     around the whole exchange (H2D + kernels + D2H + sockets).  DUMP_FILE: the server's first
 *     batch of request messages as it reassembled them ([u64 RPCID][u32 len][bytes] each), for
 *     tests/test_e2e_loopback.py to compare with the oracle's MarshalSymphony.  E2E_NOVERIFY=1
 *     skips the host-side field checks (timing runs; statuses, lengths and RPCIDs stay checked).
 */
#define _GNU_SOURCE
#include <hip/hip_runtime_api.h>

#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <poll.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "../include/symphony_hip.h"

#define DIE(...)                                                               \
    do {                                                                       \
        fprintf(stderr, "e2e_loopback[%s]: ", g_role);                         \
        fprintf(stderr, __VA_ARGS__);                                          \
        fprintf(stderr, " (%s)\n", sym_last_error());                          \
        exit(1);                                                               \
    } while (0)
#define HIPOK(x)                                                               \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) DIE("%s: %s", #x, hipGetErrorString(e_));        \
    } while (0)
#define SYMOK(x)                                                               \
    do {                                                                       \
        if ((x) != SYM_OK) DIE("%s", #x);                                      \
    } while (0)

enum { kMTU = SYM_MAX_UDP_PAYLOAD, kSlot = 1408, kMmsg = 1024, kServiceId = 1, kSetMethodId = 2 };

static const char* g_role = "main";
static uint64_t g_key = 64, g_val = 256;

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

/* Request r's key and value bytes (the server regenerates them to check what it decoded). */
static uint8_t gen_byte(uint64_t r, uint64_t j, int field) {
    uint64_t x = (r + 1) * 0x9E3779B97F4A7C15ull ^ (j + 1) * 0xBF58476D1CE4E5B9ull ^ (uint64_t)field * 0x94D049BB133111EBull;
    x ^= x >> 31;
    x *= 0xD6E8FEB86645D07Bull;
    return (uint8_t)(x >> 56);
}

static void* pinned(size_t n) {
    void* p = NULL;
    HIPOK(hipHostMalloc(&p, n + 64, hipHostMallocDefault));
    return p;
}
static void* dmem(size_t n) {
    void* p = NULL;
    HIPOK(hipMalloc(&p, n + 64));
    return p;
}

static int udp_socket(uint16_t* port) {
    int s = socket(AF_INET, SOCK_DGRAM, 0);
    if (s < 0) DIE("socket: %s", strerror(errno));
    int big = 64 << 20;
    setsockopt(s, SOL_SOCKET, SO_RCVBUF, &big, sizeof(big));
    setsockopt(s, SOL_SOCKET, SO_SNDBUF, &big, sizeof(big));
    struct sockaddr_in a = {0};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK); /* 127.0.0.1, never the wildcard */
    if (bind(s, (struct sockaddr*)&a, sizeof(a)) < 0) DIE("bind: %s", strerror(errno));
    socklen_t l = sizeof(a);
    getsockname(s, (struct sockaddr*)&a, &l);
    *port = ntohs(a.sin_port);
    return s;
}

static int rcvbuf_bytes(int s) {
    int v = 0;
    socklen_t l = sizeof(v);
    getsockopt(s, SOL_SOCKET, SO_RCVBUF, &v, &l);
    return v;
}

/* Send datagrams wire[dg_off[j], dg_off[j+1]) for j < n to `to`, kMmsg per sendmmsg call. */
static void send_all(int s, const uint8_t* wire, const uint64_t* dg_off, uint64_t n, const struct sockaddr_in* to) {
    static struct mmsghdr mm[kMmsg];
    static struct iovec iov[kMmsg];
    for (uint64_t j = 0; j < n;) {
        const unsigned k = (unsigned)(n - j < kMmsg ? n - j : kMmsg);
        for (unsigned i = 0; i < k; ++i) {
            iov[i].iov_base = (void*)(wire + dg_off[j + i]);
            iov[i].iov_len = dg_off[j + i + 1] - dg_off[j + i];
            memset(&mm[i].msg_hdr, 0, sizeof(mm[i].msg_hdr));
            mm[i].msg_hdr.msg_iov = &iov[i];
            mm[i].msg_hdr.msg_iovlen = 1;
            mm[i].msg_hdr.msg_name = (void*)to;
            mm[i].msg_hdr.msg_namelen = sizeof(*to);
        }
        const int r = sendmmsg(s, mm, k, 0);
        if (r < 0) {
            if (errno == EAGAIN || errno == ENOBUFS || errno == EINTR) continue;
            DIE("sendmmsg: %s", strerror(errno));
        }
        j += (unsigned)r;
    }
}

/* Receive datagrams appended to wire / dg_off (starting at *n, at most cap in total): wait up to
 * `first_ms` for the first one, then keep reading while more arrive within `gap_us`.  Returns the
 * count received by this call; *from = the last sender. */
static uint64_t recv_batch(int s, uint8_t* stage, uint8_t* wire, uint64_t* dg_off, uint64_t* n, uint64_t cap,
                           int first_ms, int gap_us, struct sockaddr_in* from) {
    static struct mmsghdr mm[kMmsg];
    static struct iovec iov[kMmsg];
    static struct sockaddr_in src[kMmsg];
    uint64_t got = 0;
    int wait_ms = first_ms;
    while (*n < cap) {
        struct pollfd p = {s, POLLIN, 0};
        const int pr = poll(&p, 1, wait_ms);
        if (pr < 0 && errno == EINTR) continue;
        if (pr <= 0) break;
        const unsigned k = (unsigned)(cap - *n < kMmsg ? cap - *n : kMmsg);
        for (unsigned i = 0; i < k; ++i) {
            iov[i].iov_base = stage + (size_t)i * kSlot;
            iov[i].iov_len = kSlot;
            memset(&mm[i].msg_hdr, 0, sizeof(mm[i].msg_hdr));
            mm[i].msg_hdr.msg_iov = &iov[i];
            mm[i].msg_hdr.msg_iovlen = 1;
            mm[i].msg_hdr.msg_name = &src[i];
            mm[i].msg_hdr.msg_namelen = sizeof(src[i]);
        }
        const int r = recvmmsg(s, mm, k, MSG_DONTWAIT, NULL);
        if (r < 0) {
            if (errno == EAGAIN || errno == EINTR) continue;
            DIE("recvmmsg: %s", strerror(errno));
        }
        for (int i = 0; i < r; ++i) {  /* packed back to back, as sym_reassemble takes them */
            const uint64_t at = dg_off[*n];
            memcpy(wire + at, stage + (size_t)i * kSlot, mm[i].msg_len);
            dg_off[*n + 1] = at + mm[i].msg_len;
            ++*n;
        }
        if (r > 0) *from = src[r - 1];
        got += (uint64_t)r;
        wait_ms = 0;
        if (r < (int)k) {  /* drained: wait a little for the rest of a burst */
            struct pollfd q = {s, POLLIN, 0};
            const double t0 = now();
            int more = 0;
            while (!more && (now() - t0) * 1e6 < gap_us) more = poll(&q, 1, 0) > 0;
            if (!more) break;
        }
    }
    return got;
}

/* One side's receive path state: a batch of datagrams (pending ones carried over) through
 * sym_reassemble.  Device buffers sized for `maxdg` datagrams. */
typedef struct {
    uint64_t maxdg, maxbytes;
    uint8_t *h_stage, *h_wire, *h_status;
    uint64_t *h_dg_off, *h_nmsg, *h_msg_rpc, *h_msg_off;
    uint8_t *d_wire, *d_msg, *d_status;
    uint64_t *d_dg_off, *d_msg_off, *d_msg_rpc, *d_msg_dg, *d_nmsg;
    uint64_t ndg;  /* datagrams in h_wire (pending carried ones first) */
} Rx;

static void rx_init(Rx* x, uint64_t maxdg) {
    x->maxdg = maxdg;
    x->maxbytes = maxdg * kSlot;
    x->h_stage = pinned((size_t)kMmsg * kSlot);
    x->h_wire = pinned(x->maxbytes);
    x->h_dg_off = pinned(8 * (maxdg + 1));
    x->h_status = pinned(maxdg);
    x->h_nmsg = pinned(8);
    x->h_msg_rpc = pinned(8 * maxdg);
    x->h_msg_off = pinned(8 * (maxdg + 1));
    x->d_wire = dmem(x->maxbytes);
    x->d_msg = dmem(x->maxbytes);
    x->d_status = dmem(maxdg);
    x->d_dg_off = dmem(8 * (maxdg + 1));
    x->d_msg_off = dmem(8 * (maxdg + 1));
    x->d_msg_rpc = dmem(8 * maxdg);
    x->d_msg_dg = dmem(8 * maxdg);
    x->d_nmsg = dmem(8);
    x->h_dg_off[0] = 0;
    x->ndg = 0;
}

/* Reassemble the datagrams held: the completed messages are left in d_msg / d_msg_off / d_msg_rpc
 * (their count returned, RPCIDs and offsets copied to the host); PENDING datagrams move to the front
 * of the host batch for the next call. */
static uint64_t rx_reassemble(Rx* x, sym_ctx* ctx, hipStream_t st) {
    const uint64_t n = x->ndg;
    if (!n) return 0;
    HIPOK(hipMemcpyAsync(x->d_wire, x->h_wire, x->h_dg_off[n], hipMemcpyHostToDevice, st));
    HIPOK(hipMemcpyAsync(x->d_dg_off, x->h_dg_off, 8 * (n + 1), hipMemcpyHostToDevice, st));
    SYMOK(sym_reassemble(ctx, x->d_wire, x->d_dg_off, n, x->d_msg, x->maxbytes, x->d_msg_off, x->d_msg_rpc,
                         x->d_msg_dg, x->d_nmsg, x->d_status, st));
    HIPOK(hipMemcpyAsync(x->h_nmsg, x->d_nmsg, 8, hipMemcpyDeviceToHost, st));
    HIPOK(hipMemcpyAsync(x->h_status, x->d_status, n, hipMemcpyDeviceToHost, st));
    SYMOK(sym_ctx_check(ctx, st));
    const uint64_t m = x->h_nmsg[0];
    HIPOK(hipMemcpyAsync(x->h_msg_rpc, x->d_msg_rpc, 8 * m, hipMemcpyDeviceToHost, st));
    HIPOK(hipMemcpyAsync(x->h_msg_off, x->d_msg_off, 8 * (m + 1), hipMemcpyDeviceToHost, st));
    /* carry the pending datagrams over (host side, in arrival order) */
    uint64_t k = 0, at = 0;
    for (uint64_t j = 0; j < n; ++j) {
        if (x->h_status[j] == SYM_RX_PENDING) {
            const uint64_t a = x->h_dg_off[j], len = x->h_dg_off[j + 1] - a;
            memmove(x->h_wire + at, x->h_wire + a, len);
            x->h_dg_off[k] = at;
            at += len;
            ++k;
        } else if (x->h_status[j] != SYM_RX_CONSUMED) {
            DIE("datagram %llu: receive status %u", (unsigned long long)j, x->h_status[j]);
        }
    }
    x->h_dg_off[k] = at;
    x->ndg = k;
    HIPOK(hipStreamSynchronize(st));
    return m;
}

/* The send side: n records of a stream on the device -> datagrams on the host -> the socket. */
typedef struct {
    uint64_t maxrec, maxbytes;
    uint64_t *d_first, *d_woff, *d_dg_off, *h_tot, *h_dg_off;
    uint8_t *d_fst, *d_wire, *h_wire;
} Tx;

static void tx_init(Tx* t, uint64_t maxrec, uint64_t maxstream) {
    t->maxrec = maxrec;
    t->maxbytes = maxstream + (maxstream / (kMTU - SYM_DATA_PACKET_HEADER) + 2 * maxrec + 2) * SYM_DATA_PACKET_HEADER;
    t->d_first = dmem(8 * (maxrec + 1));
    t->d_woff = dmem(8 * (maxrec + 1));
    t->d_fst = dmem(maxrec);
    const uint64_t maxdg = t->maxbytes / SYM_DATA_PACKET_HEADER + 1;
    t->d_dg_off = dmem(8 * (maxdg + 1));
    t->h_dg_off = pinned(8 * (maxdg + 1));
    t->d_wire = dmem(t->maxbytes);
    t->h_wire = pinned(t->maxbytes);
    t->h_tot = pinned(16);
}

static void tx_send(Tx* t, sym_ctx* ctx, hipStream_t st, const uint8_t* d_stream, const uint64_t* d_off, uint64_t n,
                    uint8_t type, const uint64_t* d_rpc, const sym_endpoints* ep, int sock,
                    const struct sockaddr_in* to, uint64_t* wire_bytes, uint64_t* datagrams) {
    SYMOK(sym_fragment_plan(ctx, d_stream, d_off, n, kMTU, t->d_first, t->d_woff, t->d_fst, st));
    HIPOK(hipMemcpyAsync(t->h_tot, t->d_first + n, 8, hipMemcpyDeviceToHost, st));
    HIPOK(hipMemcpyAsync(t->h_tot + 1, t->d_woff + n, 8, hipMemcpyDeviceToHost, st));
    HIPOK(hipStreamSynchronize(st));
    const uint64_t ndg = t->h_tot[0], wb = t->h_tot[1];
    if (wb > t->maxbytes) DIE("wire of %llu bytes exceeds %llu", (unsigned long long)wb, (unsigned long long)t->maxbytes);
    SYMOK(sym_fragment_write(ctx, d_stream, d_off, n, kMTU, type, d_rpc, ep, t->d_first, t->d_woff, t->d_fst,
                             t->d_wire, t->d_dg_off, st));
    HIPOK(hipMemcpyAsync(t->h_wire, t->d_wire, wb, hipMemcpyDeviceToHost, st));
    HIPOK(hipMemcpyAsync(t->h_dg_off, t->d_dg_off, 8 * (ndg + 1), hipMemcpyDeviceToHost, st));
    SYMOK(sym_ctx_check(ctx, st));
    send_all(sock, t->h_wire, t->h_dg_off, ndg, to);
    *wire_bytes += wb;
    *datagrams += ndg;
}

static sym_endpoints endpoints(uint16_t dst_port, uint16_t src_port) {
    sym_endpoints e = {{127, 0, 0, 1}, dst_port, {127, 0, 0, 1}, src_port};
    return e;
}

/* ---------------------------------------------------------------- server ---- */
static int server(int sock, uint16_t my_port, uint64_t rpcs, uint64_t window, int verify, const char* dump) {
    g_role = "server";
    sym_ctx* ctx = NULL;
    SYMOK(sym_ctx_create(0, &ctx));
    hipStream_t st;
    HIPOK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const uint64_t rec = 30 + g_key + g_val;
    const uint64_t dg_per_rec = rec / (kMTU - SYM_DATA_PACKET_HEADER) + 2;
    const uint64_t maxmsg = 8 * window, maxdg = maxmsg * dg_per_rec;
    SYMOK(sym_ctx_reserve(ctx, maxmsg));
    Rx rx;
    rx_init(&rx, maxdg);
    Tx tx;
    tx_init(&tx, maxmsg, maxmsg * (22 + g_val));
    uint8_t *d_key = dmem(rx.maxbytes), *d_val = dmem(rx.maxbytes), *d_st = dmem(maxmsg);
    uint64_t *d_koff = dmem(8 * (maxmsg + 1)), *d_voff = dmem(8 * (maxmsg + 1));
    uint8_t *h_key = pinned(rx.maxbytes), *h_val = pinned(rx.maxbytes), *h_st = pinned(maxmsg);
    uint64_t *h_koff = pinned(8 * (maxmsg + 1)), *h_voff = pinned(8 * (maxmsg + 1));
    uint8_t *h_ids = pinned(8 * maxmsg), *d_ids = dmem(8 * maxmsg);
    uint8_t* d_resp = dmem(maxmsg * (22 + g_val));
    uint64_t* d_resp_off = dmem(8 * (maxmsg + 1));
    FILE* df = dump ? fopen(dump, "wb") : NULL;
    uint64_t served = 0, wire = 0, ndg = 0;
    struct sockaddr_in peer = {0};
    int dumped = 0;
    while (served < rpcs) {
        const uint64_t got = recv_batch(sock, rx.h_stage, rx.h_wire, rx.h_dg_off, &rx.ndg, rx.maxdg, 5000, 30, &peer);
        if (!got && !rx.ndg) DIE("no request for 5 s after %llu of %llu RPCs", (unsigned long long)served,
                                 (unsigned long long)rpcs);
        const uint64_t m = rx_reassemble(&rx, ctx, st);
        if (!m) continue;
        if (m > maxmsg) DIE("%llu messages in one batch", (unsigned long long)m);
        /* Unmarshal (server.go:152) */
        SYMOK(sym_decode_kv_set(ctx, rx.d_msg, rx.d_msg_off, m, d_key, rx.maxbytes, d_koff, d_val, rx.maxbytes, d_voff,
                                d_st, st));
        HIPOK(hipMemcpyAsync(h_koff, d_koff, 8 * (m + 1), hipMemcpyDeviceToHost, st));
        HIPOK(hipMemcpyAsync(h_voff, d_voff, 8 * (m + 1), hipMemcpyDeviceToHost, st));
        HIPOK(hipMemcpyAsync(h_st, d_st, m, hipMemcpyDeviceToHost, st));
        HIPOK(hipStreamSynchronize(st));
        HIPOK(hipMemcpyAsync(h_key, d_key, h_koff[m], hipMemcpyDeviceToHost, st));
        HIPOK(hipMemcpyAsync(h_val, d_val, h_voff[m], hipMemcpyDeviceToHost, st));
        /* the service / method IDs the server dispatches on (server.go:112-113): u32 at bytes 5 and 9 */
        SYMOK(sym_raw_get_fixed(ctx, rx.d_msg, rx.d_msg_off, m, SYM_SEGMENT_PUBLIC, 5, 4, d_ids, NULL, st));
        SYMOK(sym_raw_get_fixed(ctx, rx.d_msg, rx.d_msg_off, m, SYM_SEGMENT_PUBLIC, 9, 4, d_ids + 4 * maxmsg, NULL, st));
        HIPOK(hipMemcpyAsync(h_ids, d_ids, 4 * m, hipMemcpyDeviceToHost, st));
        HIPOK(hipMemcpyAsync(h_ids + 4 * maxmsg, d_ids + 4 * maxmsg, 4 * m, hipMemcpyDeviceToHost, st));
        SYMOK(sym_ctx_check(ctx, st));
        if (df && !dumped) {  /* the first batch's request messages as reassembled */
            uint8_t* h_msg = malloc(rx.h_msg_off[m] + 1);
            HIPOK(hipMemcpy(h_msg, rx.d_msg, rx.h_msg_off[m], hipMemcpyDeviceToHost));
            for (uint64_t i = 0; i < m; ++i) {
                const uint32_t len = (uint32_t)(rx.h_msg_off[i + 1] - rx.h_msg_off[i]);
                const uint64_t r = rx.h_msg_rpc[i];
                fwrite(&r, 8, 1, df);
                fwrite(&len, 4, 1, df);
                fwrite(h_msg + rx.h_msg_off[i], 1, len, df);
            }
            free(h_msg);
            fclose(df);
            df = NULL;
            dumped = 1;
        }
        /* the handler (kvstore.go:58-82): SetResponse{Value: req.Value} */
        for (uint64_t i = 0; i < m; ++i) {
            uint32_t sid, mid;
            memcpy(&sid, h_ids + 4 * i, 4);
            memcpy(&mid, h_ids + 4 * maxmsg + 4 * i, 4);
            if (h_st[i] != SYM_STATUS_OK || sid != kServiceId || mid != kSetMethodId)
                DIE("RPC %llu: status %u service %u method %u", (unsigned long long)rx.h_msg_rpc[i], h_st[i], sid, mid);
            if (verify) {
                const uint64_t r = rx.h_msg_rpc[i];
                if (h_koff[i + 1] - h_koff[i] != g_key || h_voff[i + 1] - h_voff[i] != g_val)
                    DIE("RPC %llu: field lengths", (unsigned long long)r);
                for (uint64_t j = 0; j < g_key; ++j)
                    if (h_key[h_koff[i] + j] != gen_byte(r, j, 0)) DIE("RPC %llu: key byte %llu", (unsigned long long)r, (unsigned long long)j);
                for (uint64_t j = 0; j < g_val; ++j)
                    if (h_val[h_voff[i] + j] != gen_byte(r, j, 1)) DIE("RPC %llu: value byte %llu", (unsigned long long)r, (unsigned long long)j);
            }
        }
        /* Marshal (server.go:173; IDs 0) and Send as PacketTypeResponse with the request's RPCIDs */
        HIPOK(hipMemcpyAsync(d_val, h_val, h_voff[m], hipMemcpyHostToDevice, st));
        HIPOK(hipMemcpyAsync(d_voff, h_voff, 8 * (m + 1), hipMemcpyHostToDevice, st));
        SYMOK(sym_encode_kv_response(ctx, SYM_SCHEMA_KV_SET_RESPONSE, d_val, d_voff, m, 0, 0, d_resp, d_resp_off, st));
        const sym_endpoints ep = endpoints(ntohs(peer.sin_port), my_port);
        tx_send(&tx, ctx, st, d_resp, d_resp_off, m, SYM_PACKET_RESPONSE, rx.d_msg_rpc, &ep, sock, &peer, &wire, &ndg);
        served += m;
    }
    if (df) fclose(df);
    sym_ctx_destroy(ctx);
    return 0;
}

/* ---------------------------------------------------------------- client ---- */
static int client(int sock, uint16_t my_port, uint16_t srv_port, uint64_t rpcs, uint64_t window, uint64_t inflight,
                  int verify) {
    g_role = "client";
    sym_ctx* ctx = NULL;
    SYMOK(sym_ctx_create(0, &ctx));
    hipStream_t st;
    HIPOK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const uint64_t K = g_key, V = g_val;
    /* the requests in flight fit the receiver's socket buffer (same size both sides): a loopback
     * datagram costs up to ~2.3 KB of it (skb truesize), a request ceil(size / 1369) + 1 datagrams */
    const uint64_t dg_per_req = (30 + K + V) / (kMTU - SYM_DATA_PACKET_HEADER) + 1;
    const uint64_t fit = (uint64_t)rcvbuf_bytes(sock) / 2304 / (inflight * dg_per_req);
    const uint64_t W = window < fit ? window : (fit ? fit : 1);
    SYMOK(sym_ctx_reserve(ctx, 8 * W));
    /* the application's request columns, generated before the clock starts */
    uint8_t* h_key = pinned(rpcs * K);
    uint8_t* h_val = pinned(rpcs * V);
    for (uint64_t r = 0; r < rpcs; ++r) {
        for (uint64_t j = 0; j < K; ++j) h_key[r * K + j] = gen_byte(r, j, 0);
        for (uint64_t j = 0; j < V; ++j) h_val[r * V + j] = gen_byte(r, j, 1);
    }
    uint64_t* h_koff = pinned(8 * (W + 1));
    uint64_t* h_voff = pinned(8 * (W + 1));
    for (uint64_t i = 0; i <= W; ++i) {
        h_koff[i] = i * K;
        h_voff[i] = i * V;
    }
    uint64_t* h_rpc = pinned(8 * rpcs);
    for (uint64_t r = 0; r < rpcs; ++r) h_rpc[r] = r;
    uint8_t *d_key = dmem(W * K), *d_val = dmem(W * V);
    uint64_t *d_koff = dmem(8 * (W + 1)), *d_voff = dmem(8 * (W + 1)), *d_rpc = dmem(8 * W);
    HIPOK(hipMemcpy(d_koff, h_koff, 8 * (W + 1), hipMemcpyHostToDevice));
    HIPOK(hipMemcpy(d_voff, h_voff, 8 * (W + 1), hipMemcpyHostToDevice));
    uint8_t* d_req = dmem(W * (30 + K + V));
    uint64_t* d_req_off = dmem(8 * (W + 1));
    Tx tx;
    tx_init(&tx, W, W * (30 + K + V));
    const uint64_t maxmsg = (inflight + 1) * W;
    Rx rx;
    rx_init(&rx, maxmsg * ((22 + V) / (kMTU - SYM_DATA_PACKET_HEADER) + 2));
    uint8_t *d_rv = dmem(rx.maxbytes), *d_rst = dmem(maxmsg), *h_rv = pinned(rx.maxbytes), *h_rst = pinned(maxmsg);
    uint64_t *d_rvoff = dmem(8 * (maxmsg + 1)), *h_rvoff = pinned(8 * (maxmsg + 1));
    uint8_t* answered = calloc(rpcs, 1);
    struct sockaddr_in to = {0};
    to.sin_family = AF_INET;
    to.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    to.sin_port = htons(srv_port);
    const sym_endpoints ep = endpoints(srv_port, my_port);
    uint64_t sent = 0, done = 0, wire_req = 0, dg_req = 0, resp_bytes = 0, batches = 0;
    struct sockaddr_in from;
    const double t0 = now();
    while (done < rpcs) {
        while (sent < rpcs && sent - done < inflight * W) {  /* Call: Marshal + patch IDs + Send */
            const uint64_t n = rpcs - sent < W ? rpcs - sent : W;
            HIPOK(hipMemcpyAsync(d_key, h_key + sent * K, n * K, hipMemcpyHostToDevice, st));
            HIPOK(hipMemcpyAsync(d_val, h_val + sent * V, n * V, hipMemcpyHostToDevice, st));
            HIPOK(hipMemcpyAsync(d_rpc, h_rpc + sent, 8 * n, hipMemcpyHostToDevice, st));
            SYMOK(sym_encode_kv_set(ctx, d_key, d_koff, d_val, d_voff, n, kServiceId, kSetMethodId, d_req, d_req_off, st));
            tx_send(&tx, ctx, st, d_req, d_req_off, n, SYM_PACKET_REQUEST, d_rpc, &ep, sock, &to, &wire_req, &dg_req);
            sent += n;
        }
        /* responses: Receive + reassembly, Unmarshal (client.go:205) */
        const uint64_t got = recv_batch(sock, rx.h_stage, rx.h_wire, rx.h_dg_off, &rx.ndg, rx.maxdg, 5000, 30, &from);
        if (!got && !rx.ndg) DIE("no response for 5 s: %llu of %llu answered", (unsigned long long)done, (unsigned long long)rpcs);
        const uint64_t m = rx_reassemble(&rx, ctx, st);
        if (!m) continue;
        ++batches;
        SYMOK(sym_decode_kv_response(ctx, SYM_SCHEMA_KV_SET_RESPONSE, rx.d_msg, rx.d_msg_off, m, d_rv, rx.maxbytes, d_rvoff,
                                     d_rst, st));
        HIPOK(hipMemcpyAsync(h_rvoff, d_rvoff, 8 * (m + 1), hipMemcpyDeviceToHost, st));
        HIPOK(hipMemcpyAsync(h_rst, d_rst, m, hipMemcpyDeviceToHost, st));
        HIPOK(hipStreamSynchronize(st));
        HIPOK(hipMemcpyAsync(h_rv, d_rv, h_rvoff[m], hipMemcpyDeviceToHost, st));
        SYMOK(sym_ctx_check(ctx, st));
        for (uint64_t i = 0; i < m; ++i) {
            const uint64_t r = rx.h_msg_rpc[i];
            if (r >= rpcs || answered[r]) DIE("response for RPC %llu unexpected", (unsigned long long)r);
            answered[r] = 1;
            if (h_rst[i] != SYM_STATUS_OK || h_rvoff[i + 1] - h_rvoff[i] != V) DIE("RPC %llu: bad response", (unsigned long long)r);
            if (verify && memcmp(h_rv + h_rvoff[i], h_val + r * V, V)) DIE("RPC %llu: response value differs", (unsigned long long)r);
        }
        resp_bytes += rx.h_msg_off[m];
        done += m;
    }
    const double el = now() - t0;
    /* the codec's algorithmic bytes: request encode + decode, response encode + decode */
    const double req_rec = 30.0 + K + V, resp_rec = 22.0 + V;
    const double enc_req = K + V + 16 + req_rec + 8, dec_req = req_rec + 8 + K + V + 16 + 1;
    const double enc_resp = V + 8 + resp_rec + 8, dec_resp = resp_rec + 8 + V + 8 + 1;
    const double alg = (enc_req + dec_req + enc_resp + dec_resp) * rpcs;
    printf("{\"rpcs\": %llu, \"window\": %llu, \"inflight\": %llu, \"key\": %llu, \"value\": %llu, \"seconds\": %.4f, "
           "\"rpc_per_s\": %.1f, \"gbps_algorithmic\": %.3f, \"request_wire_gbps\": %.3f, \"request_datagrams\": %llu, "
           "\"request_wire_bytes\": %llu, \"response_bytes\": %llu, \"response_batches\": %llu, \"rcvbuf\": %d, "
           "\"verified\": %s}\n",
           (unsigned long long)rpcs, (unsigned long long)W, (unsigned long long)inflight, (unsigned long long)K,
           (unsigned long long)V, el, rpcs / el, alg / el / 1e9, wire_req / el / 1e9, (unsigned long long)dg_req,
           (unsigned long long)wire_req, (unsigned long long)resp_bytes, (unsigned long long)batches,
           rcvbuf_bytes(sock), verify ? "true" : "false");
    fflush(stdout);
    free(answered);
    sym_ctx_destroy(ctx);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: e2e_loopback RPCS WINDOW KEY VAL [INFLIGHT [DUMP_FILE]]\n");
        return 2;
    }
    const uint64_t rpcs = strtoull(argv[1], NULL, 0), window = strtoull(argv[2], NULL, 0);
    g_key = strtoull(argv[3], NULL, 0);
    g_val = strtoull(argv[4], NULL, 0);
    const uint64_t inflight = argc > 5 ? strtoull(argv[5], NULL, 0) : 2;
    const char* dump = argc > 6 ? argv[6] : NULL;
    const int verify = getenv("E2E_NOVERIFY") == NULL;
    if (!rpcs || !window || !inflight || g_key > 1 << 16 || g_val > 1 << 20) DIE("bad arguments");
    uint16_t cport, sport;
    const int cs = udp_socket(&cport), ss = udp_socket(&sport);
    /* the server is a child forked before any HIP call in either process */
    const pid_t pid = fork();
    if (pid < 0) DIE("fork: %s", strerror(errno));
    if (pid == 0) {
        close(cs);
        _exit(server(ss, sport, rpcs, window, verify, dump));
    }
    close(ss);
    const int rc = client(cs, cport, sport, rpcs, window, inflight, verify);
    int status = 0;
    for (int i = 0; i < 400; ++i) {  /* the server has answered everything: it exits on its own */
        if (waitpid(pid, &status, WNOHANG) == pid) break;
        if (i == 399) {
            kill(pid, SIGKILL);
            waitpid(pid, &status, 0);
        }
        usleep(25000);
    }
    if (rc || !WIFEXITED(status) || WEXITSTATUS(status)) {
        fprintf(stderr, "e2e_loopback: client rc %d, server status %d\n", rc, status);
        return 1;
    }
    return 0;
}
