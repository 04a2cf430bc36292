"""Symphony encode+decode throughput on MI355X (BASELINE.json metric), one process per GPU.

One step = one device-resident Symphony encode of a record batch plus one decode of an
encoded batch (BASELINE.json configs[1]: 2^20 kv-store SetRequest records, 64 B keys,
256 B values, per GPU).  Inputs are resident in HBM before the timed region.  Four
buffer sets rotate so the 256 MiB Infinity Cache cannot serve a step from a previous
one: step s encodes set s%4 and decodes the stream encoded two steps earlier.

  python bench.py [--gpus N --steps K --warmup W] [--config 2|3|4] [--records R]
      (N > 1 without torchrun's env: bench.py starts the N rank processes itself, spawn_ranks)
  torchrun --nproc-per-node N bench.py --gpus N ...   (weak scaling, no data-path collective)

Prints ONE JSON line on rank 0.  `value` = algorithmic GB/s over all ranks (SURVEY.md
section 8d: 694 B encode + 695 B decode per 64/256 record), timed with a barrier +
device sync on both sides, max over ranks.  `roofline` reports the dominant single kernel
(encode_kernel, or decode_pipe_kernel) from HIP events on the stream the kernels run on (the
decode's events also cover its small gate launch, so `achieved` is conservative); `cpu_baseline` times the C restatement of the Go codec (oracle/) on a bounded sample on
this host, at 1 thread and at the host's core share, plus config 1's echo record.
--config 4 is SURVEY 8d config 4: 2^23 SetRequests per GPU (seed 0x5EED0003 + rank), the shards
of a 2^26-record batch on 8 GPUs.  Legs beside the headline (outside the timed region): the mixed
Get/Set batch at the trace ratio (BASELINE config 2 as written), config 3, the host-inclusive
rate through sym_encode_host / sym_decode_host, and the SURVEY 8f rows.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from arpc_amd import datagen, schemas  # noqa: E402
from arpc_amd.codec import Codec, DecodedBatch, to_device  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
NSETS = 4


def alg_bytes(n: int, nvar: int, var_total: int, stream_total: int) -> tuple[int, int]:
    """Algorithmic bytes of one encode and one decode call."""
    enc = var_total + 8 * nvar * n + stream_total + 8 * n
    dec = stream_total + 8 * n + var_total + 8 * nvar * n + n
    return enc, dec


def spawn_ranks(n: int, argv: list[str]) -> int:
    """`python bench.py --gpus N` with no torch.distributed env: start N rank processes of this same
    script (one per GPU, LOCAL_RANK = GPU index) with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR
    127.0.0.1 / MASTER_PORT set, and wait for them.  The parent makes no HIP call (it only imports
    torch, which does not initialise the GPU), so the children start on an untouched runtime; they are
    child processes, not an exec.  Rank 0 prints the JSON line to the inherited stdout.  When a rank
    fails the others are stopped (they would wait in the barrier forever) and its exit code returned."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *argv], env=env,
                                      start_new_session=True))
    rc = 0
    try:
        live = list(procs)
        while live:
            time.sleep(0.2)
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    for q in live:
                        os.killpg(q.pid, signal.SIGTERM)
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
    return rc


def dist_setup(launch_check: bool = False):
    """One process per GPU (torch.distributed.run env, or spawn_ranks).  RCCL ("nccl") carries only the
    barrier and the max-over-ranks of the elapsed time: the shards exchange no data.
    SYMHIP_BENCH_ONE_GPU=1 (rehearsal on a 1-GPU box) puts every rank on device 0 and uses gloo for
    that control traffic; so does --launch-check, which touches no GPU at all."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    one_gpu = os.environ.get("SYMHIP_BENCH_ONE_GPU") == "1"
    if one_gpu:
        local = 0
    if world > 1:
        import torch.distributed as dist
        if launch_check:
            dist.init_process_group(backend="gloo")
            return world, rank, local
        torch.cuda.set_device(local)
        if one_gpu:
            dist.init_process_group(backend="gloo")
        else:
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def launch_check(args) -> None:
    """--launch-check: the N-rank launch alone (no GPU, gloo): every rank joins the group, meets the
    barrier, contributes its elapsed time to the max, and rank 0 prints the world it saw."""
    world, rank, local = dist_setup(launch_check=True)
    barrier(world)
    t0 = time.perf_counter()
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world, None)
    ranks = [rank]
    if world > 1:
        import torch.distributed as dist
        got = [None] * world
        dist.all_gather_object(got, (rank, local, os.getpid()))
        ranks = got
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "gpus_requested": args.gpus, "config": args.config,
                          "ranks": ranks, "elapsed_max_s": el}), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, world: int, dev) -> float:
    if world == 1:
        return x
    import torch.distributed as dist
    on_gpu = dist.get_backend() == "nccl"
    t = torch.tensor([x], dtype=torch.float64, device=dev if on_gpu else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def workload(args, world, rank):
    if args.config == 4:  # shard `rank` of the 2^26-record batch
        base = datagen.config4_shard(rank)
    else:
        base = dict(datagen.CONFIG2 if args.config == 2 else datagen.CONFIG3)
        if world > 1:  # one seeded shard per GPU
            base["seed"] = 0x5EED0003 + rank if args.config == 2 else base["seed"] + 0x100 * rank
    if args.records:
        base["n"] = args.records
    return base


def cgroup_cpus() -> float | None:
    """CPUs this process may use by its cgroup's CPU quota (cgroup v2 cpu.max, or v1 cfs quota /
    period); None when unlimited or unreadable."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / p
    except (OSError, ValueError):
        return None


def host_cpu_info() -> dict:
    """nproc, the CPU model (lscpu's "Model name", from /proc/cpuinfo), this process's affinity and
    its cgroup CPU quota."""
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = cgroup_cpus()
    return {"nproc": os.cpu_count(), "affinity": share, "cgroup_cpu_quota": quota, "model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(kw: dict, seconds: float) -> dict:
    """The C restatement of the Go codec (oracle/symphony_oracle.c; no Go toolchain exists here or on
    the GPU box) on the headline's own batch: the same 2^20 records, encoded into a stream allocated
    once and decoded into columns allocated once (oracle.BatchBench), as the GPU is timed -- a working
    set of ~1 GB, far beyond the host's caches.  One thread pinned to one CPU: a warm-up round, then
    rounds for about seconds/2 (at least 5); `value` is the median round's GB/s, with the spread.  Then
    the batch record-sharded over the CPUs this process may use (its cgroup CPU quota, else its
    affinity, else OMP_NUM_THREADS), one pinned thread per shard (ctypes releases the GIL), rounds in
    lockstep for about seconds/2: the aggregate.  Plus config 1's echo record (ns per MarshalSymphony /
    UnmarshalSymphony, one record per call with Go's allocations)."""
    import statistics
    import threading

    from oracle import oracle
    info = host_cpu_info()
    b = datagen.make_batch(**kw)
    s = b.schema
    var_total = sum(int(o[-1] - o[0]) for _, o in b.var)
    enc_b, dec_b = alg_bytes(b.n, s.nvar, var_total, b.encoded_size())
    cpus = sorted(os.sched_getaffinity(0))
    mine = os.sched_getaffinity(0)

    bb = oracle.BatchBench(b.fixed, b.var)
    os.sched_setaffinity(0, {cpus[0]})  # this thread only (Linux: pid 0 = the calling thread)
    try:
        e, d = bb.run(1)
        reps = max(5, int(seconds / 2 / (e[0] + d[0])))
        e, d = bb.run(reps)
    finally:
        os.sched_setaffinity(0, mine)
    del bb
    rates = sorted((enc_b + dec_b) / (x + y) / 1e9 for x, y in zip(e, d))
    med = statistics.median(rates)

    omp = int(info["omp_num_threads"]) if (info["omp_num_threads"] or "").isdigit() else None
    share = info["cgroup_cpu_quota"] or omp or info["affinity"]
    threads = max(1, min(int(share), len(cpus)))
    from arpc_amd import shard
    benches = []
    for t in range(threads):
        lo, hi = shard.shard_range(b.n, threads, t)
        benches.append(oracle.BatchBench([c[lo:hi] for c in b.fixed], shard.shard_columns(b.var, lo, hi)))
    e1, d1 = benches[0].run(1)
    rounds = max(3, int(seconds / 2 / (e1[0] + d1[0]) / max(1, threads // 2)))
    go = threading.Barrier(threads + 1)

    def work(t):
        os.sched_setaffinity(0, {cpus[t % len(cpus)]})
        go.wait()
        benches[t].run(rounds)

    th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for x in th:
        x.start()
    go.wait()
    t0 = time.perf_counter()
    for x in th:
        x.join()
    el = time.perf_counter() - t0
    del benches
    agg = (enc_b + dec_b) * rounds / el / 1e9
    m_ns, u_ns = oracle.bench_echo(2_000_000)
    ws = (var_total + 16 * (b.n + 1)) * 2 + b.encoded_size() + 8 * (b.n + 1) + b.n
    return {"value": round(med, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "mrecords_per_s": round(med * 1e9 / ((enc_b + dec_b) / b.n) / 1e6, 3),
            "rounds": len(rates), "spread_gbps": [round(rates[0], 3), round(rates[-1], 3)],
            "encode_ms_median": round(1e3 * statistics.median(e), 2),
            "decode_ms_median": round(1e3 * statistics.median(d), 2),
            "working_set_bytes": ws,
            "all_cores": {"value": round(agg, 3), "cores": threads, "rounds": rounds,
                          "mrecords_per_s": round(b.n * rounds / el / 1e6, 3),
                          "share_from": "cgroup cpu quota" if info["cgroup_cpu_quota"] else
                                        ("OMP_NUM_THREADS" if omp else "affinity")},
            "host": info,
            "config1_echo": {"marshal_ns": round(m_ns, 2), "unmarshal_ns": round(u_ns, 2),
                             "records_per_s": round(1e9 / (m_ns + u_ns), 1),
                             "gbps": round(54 * 2 / (m_ns + u_ns), 4),
                             "note": "EchoRequest{42, 300, alice, hello world} (54 B), marshal then unmarshal, "
                                     "one record per call with Go's allocations (oracle/bench_oracle.c, "
                                     "testcases/simple/main.go:248-420 methodology), 1 thread"},
            "sample": f"the headline workload: {b.n} {s.go_type} records (seed {kw['seed']:#x}), encode into a "
                      f"preallocated stream + decode into preallocated columns, {len(rates)} rounds on 1 thread "
                      f"pinned to CPU {cpus[0]} (median, spread min..max), {rounds} rounds on {threads} pinned "
                      "threads over record shards (aggregate); oracle/symphony_oracle.c (-O2): the C "
                      "restatement of the Go codec, not Go (no Go toolchain)"}


def decode_kernel_name(s, mixed: bool = False) -> str:
    """rocprof's name of the default decode's main launch for schema s (mixed: the Get/Set batch):
    kv layouts (no int32 fields) run the speculative parsers with 256-tile scanner steps
    (decode_pipe.hip kSpecCfg), followed by the small gate launch; int32 layouts the exact parsers
    (kExactCfg); the mixed batch 8 waves per SIMD with a 16 KiB stage (kMixCfg).
    PipeCfg{mode, diag, sk, pr, stg, spec, specx, wpe, uk, fast, loc, canon, tilek} (trailing defaults
    are not printed); kSpecCfg's copiers locate chunks by ballots and check the generator's header image;
    both speculative configs read one key length per tile (tilek)."""
    if mixed:
        cfg = "0, 0, 1, 2, 16384, true, 0, 8, 2, false, false, false, true"
    else:
        cfg = "0, 0, 1, 2, 22528, true, 0, 6, 2, false, true, true, true" if s.nfixed == 0 else "0, 0, 2, 2, 22528, false, 0, 6, 2"
    return f"decode_pipe_kernel<{s.nfixed}, {s.nvar}, {'true' if mixed else 'false'}, symhip::pipe::PipeCfg{{{cfg}}}>"


ENCODE_KERNEL = "encode_kernel<0, 2, 1, false, 4, false, 64>"
ENCODE_MIXED_KERNEL = "encode_pipe_kernel<false, 1, 64>"


def load_traffic(kernel: str, workload: str):
    """Per-launch HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE) of `kernel` when it ran `workload`
    ("config2", "config3", "config4", "mixed"), from the committed PMC summary profiles/traffic.json
    (tools/make_traffic.py), else None: a kernel's bytes on one workload never stand in for another's."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        return d.get("workloads", {}).get(workload, {}).get("kernels", {}).get(kernel, {}).get("hbm_bytes_per_launch")
    except (ValueError, OSError):
        return None


def packetize_leg(codec: Codec, data: torch.Tensor, rec_off: torch.Tensor, dev, reps: int) -> dict:
    """SURVEY.md 8f N2 beside the headline: the send side of aRPC's transport (FragmentPackets +
    DataPacket framing) over the encoded batch, device-resident, timed with HIP events.
    Algorithmic bytes: stream + record offsets + rpc ids in; wire bytes + datagram offsets + per-record
    first datagram, wire offset and status out."""
    import ctypes
    from arpc_amd import _native
    n = rec_off.numel() - 1
    rpc = torch.arange(n, dtype=torch.int64, device=dev)
    first = torch.empty(n + 1, dtype=torch.int64, device=dev)
    wire_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    status = torch.empty(n, dtype=torch.uint8, device=dev)
    L, ctx = codec._lib, codec._ctx
    sh = torch.cuda.current_stream(dev).cuda_stream
    mtu = _native.SYM_MAX_UDP_PAYLOAD

    def plan():
        _native.check(L.sym_fragment_plan(ctx, data.data_ptr(), rec_off.data_ptr(), n, mtu, first.data_ptr(),
                                          wire_off.data_ptr(), status.data_ptr(), sh), "sym_fragment_plan")
    plan()
    torch.cuda.synchronize()
    ndg, total = int(first[n].item()), int(wire_off[n].item())
    wire = torch.empty(total, dtype=torch.uint8, device=dev)
    dg_off = torch.empty(ndg + 1, dtype=torch.int64, device=dev)
    ep = _native.Endpoints((ctypes.c_uint8 * 4)(127, 0, 0, 1), 9000, (ctypes.c_uint8 * 4)(127, 0, 0, 1), 9001)

    def write():
        _native.check(L.sym_fragment_write(ctx, data.data_ptr(), rec_off.data_ptr(), n, mtu, _native.SYM_PACKET_REQUEST,
                                           rpc.data_ptr(), ctypes.byref(ep), first.data_ptr(), wire_off.data_ptr(),
                                           status.data_ptr(), wire.data_ptr(), dg_off.data_ptr(), sh),
                      "sym_fragment_write")
    write()
    torch.cuda.synchronize()
    ev = []
    for _ in range(reps):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        plan()
        e1.record()
        write()
        e2.record()
        ev.append((e0, e1, e2))
    torch.cuda.synchronize()
    codec.check()
    plan_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in ev]))
    write_ms = float(np.mean([b.elapsed_time(c) for _, b, c in ev]))
    stream_b = int(rec_off[n].item() - rec_off[0].item())
    alg = stream_b + 16 * n + total + 8 * (ndg + 1) + 17 * n
    return {"records": n, "datagrams": ndg, "wire_bytes": total, "plan_ms": round(plan_ms, 4),
            "write_ms": round(write_ms, 4), "alg_bytes": alg,
            "gbps_algorithmic": round(alg / ((plan_ms + write_ms) * 1e-3) / 1e9, 1),
            "note": "FragmentPackets(MaxUDPPayloadSize-31) + 31-byte DataPacket headers (pkg/transport/"
                    "transport.go:146-201), device-resident, outside the timed region"}


def byte_gather(src: torch.Tensor, start: torch.Tensor, length: torch.Tensor) -> torch.Tensor:
    """src[start[i] : start[i] + length[i]] for every i, back to back (torch, for the bench's setup)."""
    total = int(length.sum().item())
    if total == 0:
        return src[:0].clone()
    dst0 = torch.cumsum(length, 0) - length
    idx = torch.repeat_interleave(start - dst0, length) + torch.arange(total, device=src.device)
    return src[idx]


def reassembly_leg(codec: Codec, data: torch.Tensor, rec_off: torch.Tensor, dev, reps: int, window: int = 0) -> dict:
    """SURVEY.md 8f N3 beside the headline: the receive side of aRPC's transport (Receive parse +
    DataReassembler.ProcessFragment) over the packetized batch, datagrams in send order (window 0) or
    shuffled inside consecutive windows of `window` datagrams (UDP's local reordering: packets of a
    message arrive out of order and RPCIDs interleave), device-resident, HIP events.  Algorithmic
    bytes: datagram offsets + every datagram read; message bytes, message offsets / RPCIDs /
    completing datagrams and a status byte per datagram written."""
    n = rec_off.numel() - 1
    rpc = torch.arange(n, dtype=torch.int64, device=dev)
    dg = codec.fragment(data, rec_off, rpc)
    torch.cuda.synchronize()
    codec.check()
    nd = dg.dg_off.numel() - 1
    wire, dg_off = dg.wire, dg.dg_off
    if window:
        g = torch.Generator(device=dev)
        g.manual_seed(7)
        key = torch.div(torch.arange(nd, device=dev), window, rounding_mode="floor").double() + \
            torch.rand(nd, device=dev, dtype=torch.float64, generator=g)
        perm = torch.argsort(key)
        lens = (dg_off[1:] - dg_off[:-1])[perm]
        wire = byte_gather(dg.wire, dg_off[:-1][perm], lens)
        dg_off = torch.zeros(nd + 1, dtype=torch.int64, device=dev)
        dg_off[1:] = torch.cumsum(lens, 0)
        del perm, lens, key
    r = codec.reassemble(wire, dg_off)
    torch.cuda.synchronize()
    codec.check()
    k = int(r.nmsg.item())
    mbytes = int(r.offsets[k].item())
    if window:  # every record, in completion order: message m is record rpc[m]
        m_rpc = r.rpc_id[:k]
        want = byte_gather(data, rec_off[:-1][m_rpc], (rec_off[1:] - rec_off[:-1])[m_rpc])
        ok = k == n and bool(torch.equal(r.data[:mbytes], want))
        del want
    else:
        ok = k == n and bool(torch.equal(r.data[:mbytes], data[:mbytes]))  # one message per record, in order
    ev = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        codec.reassemble(wire, dg_off)
        e1.record()
        ev.append((e0, e1))
    torch.cuda.synchronize()
    codec.check()
    ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
    wire_b = int(wire.numel())
    alg = 8 * (nd + 1) + wire_b + mbytes + 8 * (k + 1) + 16 * k + nd
    return {"datagrams": nd, "messages": k, "wire_bytes": wire_b, "message_bytes": mbytes, "round_trip_ok": ok,
            "reassemble_ms": round(ms, 4), "alg_bytes": alg, "gbps_algorithmic": round(alg / (ms * 1e-3) / 1e9, 1),
            "note": "UDPTransport.Receive + DataReassembler.ProcessFragment (pkg/transport/transport.go:253-317, "
                    "fragmentation.go:49-183) batched; datagrams from sym_fragment_write, "
                    + (f"shuffled within windows of {window}" if window else "send order")}


def crypto_leg(codec: Codec, data: torch.Tensor, rec_off: torch.Tensor, dev, reps: int) -> dict:
    """SURVEY.md 8f N4 beside the headline: EncryptSymphonyData / DecryptSymphonyData
    (pkg/transport/encryption.go:82-256) over the encoded batch with the reference's default keys,
    device-resident, HIP events.  Algorithmic bytes: records + offsets (+ 24-byte nonces) in, sealed
    (opened) records + offsets + status out."""
    n = rec_off.numel() - 1
    pk = bytes.fromhex("27e1fa17d72b1faf722362deb1974a7675058db98843705124a074c61172f796")
    vk = bytes.fromhex("9b5300678420678a3157a4bcacdc3e864693971f8a3fab05b06913fb43c7ebf9")
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    nonces = torch.randint(0, 256, (n, 24), dtype=torch.uint8, device=dev, generator=g)
    sealed = codec.encrypt(data, rec_off, nonces, pk, vk)
    opened = codec.decrypt(sealed.data, sealed.offsets, pk, vk)
    torch.cuda.synchronize()
    codec.check()
    in_b = int(rec_off[n].item() - rec_off[0].item())
    enc_b = int(sealed.offsets[n].item())
    ok = bool((opened.status == 0).all().item()) and bool(torch.equal(opened.data[:in_b], data[:in_b]))

    def timed(fn) -> float:
        ev = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            ev.append((e0, e1))
        torch.cuda.synchronize()
        codec.check()
        return float(np.median([a.elapsed_time(b) for a, b in ev]))

    enc_ms = timed(lambda: codec.encrypt(data, rec_off, nonces, pk, vk))
    dec_ms = timed(lambda: codec.decrypt(sealed.data, sealed.offsets, pk, vk))
    enc_alg = in_b + 8 * (n + 1) + 24 * n + enc_b + 8 * (n + 1) + n
    dec_alg = enc_b + 8 * (n + 1) + in_b + 8 * (n + 1) + n
    gbps = lambda a, ms: round(a / (ms * 1e-3) / 1e9, 1)
    return {"records": n, "plain_bytes": in_b, "sealed_bytes": enc_b, "round_trip_ok": ok,
            "encrypt_ms": round(enc_ms, 4), "encrypt_gbps": gbps(enc_alg, enc_ms),
            "decrypt_ms": round(dec_ms, 4), "decrypt_gbps": gbps(dec_alg, dec_ms),
            "note": "AES-256-GCM per Symphony segment, nonces supplied (encryption.go:115-121 draws them at random)"}


def proxy_leg(codec: Codec, dev, reps: int) -> dict:
    """SURVEY.md 8f N1 beside the headline: the proxy's firewall element (GetScore, shouldBlock, and
    the passing requests compacted into a forwardable batch) and the Raw getters GetScore /
    GetUsername, over 2^20 element-schema SetRequests (datagen.ELEMENT_FW: Username 16, Key 64,
    Value 256 -> 378-byte records), device-resident, HIP events.  Threshold 50 on scores uniform in
    [0, 100): half the requests pass.
    Algorithmic bytes -- firewall: offsets 8(n+1) + score 4n read, kept bytes read and written,
    score 4n + verdict n + kept offsets 8(k+1) + kept index 8k written; GetScore: offsets + 4n read,
    4n value + n status written; GetUsername: offsets + table entry, length and value read, value +
    offsets 8(n+1) + n status written."""
    from arpc_amd import datagen
    b = datagen.make_element_batch(**datagen.ELEMENT_FW)
    n = len(b.score)
    data = torch.from_numpy(b.data).to(dev)
    off = torch.from_numpy(b.rec_off.view(np.int64)).to(dev)
    fw = codec.firewall(data, off, 50)
    codec.raw_get_fixed(data, off, 13, 4)
    ub, uo, _ = codec.raw_get_bytes(data, off, 17)
    torch.cuda.synchronize()
    codec.check()
    k = int(fw.nkept.item())
    kept_b = int(fw.kept_off[k].item())
    user_b = int(uo[n].item())

    def timed(fn) -> float:
        ev = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            ev.append((e0, e1))
        torch.cuda.synchronize()
        codec.check()
        return float(np.median([a.elapsed_time(c) for a, c in ev]))

    fw_ms = timed(lambda: codec.firewall(data, off, 50))
    sc_ms = timed(lambda: codec.raw_get_fixed(data, off, 13, 4))
    un_ms = timed(lambda: codec.raw_get_bytes(data, off, 17))
    fw_alg = 8 * (n + 1) + 4 * n + 2 * kept_b + 4 * n + n + 8 * (k + 1) + 8 * k
    sc_alg = 8 * (n + 1) + 4 * n + 4 * n + n
    un_alg = 8 * (n + 1) + 8 * n + 2 * user_b + 8 * (n + 1) + n
    gbps = lambda a, ms: round(a / (ms * 1e-3) / 1e9, 1)
    return {"records": n, "record_bytes": int(b.rec_off[1]), "threshold": 50, "kept": k, "kept_bytes": kept_b,
            "firewall_ms": round(fw_ms, 4), "firewall_alg_bytes": fw_alg, "firewall_gbps": gbps(fw_alg, fw_ms),
            "firewall_mrps": round(n / (fw_ms * 1e-3) / 1e6, 1),
            "get_score_ms": round(sc_ms, 4), "get_score_gbps": gbps(sc_alg, sc_ms),
            "get_username_ms": round(un_ms, 4), "get_username_gbps": gbps(un_alg, un_ms),
            "note": "FirewallElement.ProcessRequest (cmd/proxy/element/firewall.go:39-52) and GetRequestRaw "
                    "getters (kv-store-symphony-element kv.syn.go:285-310) batched; outside the timed region"}


def flat_leg(codec: Codec, dev, reps: int) -> dict:
    """SURVEY.md 8f N5 (flat part) beside the headline: the run-time-described flat codec
    (arpc_amd/flat.py) on the element-schema SetRequest (public Score + Username, private Key +
    Value; kv-store-symphony-element kv.proto:18-41), 2^20 records of datagen.ELEMENT_FW, encode
    and decode device-resident, HIP events.  Algorithmic bytes -- encode: score 4n + string bytes +
    3 x 8(n+1) offsets read, records + 8(n+1) offsets written; decode: records + offsets read,
    score 4n + string bytes + 3 x 8(n+1) offsets + n status written."""
    from arpc_amd import datagen, flat
    b = datagen.make_element_batch(**datagen.ELEMENT_FW)
    n = len(b.score)
    cols = [torch.from_numpy(b.score).to(dev)] + [(torch.from_numpy(x).to(dev), torch.from_numpy(o.view(np.int64)).to(dev))
                                                  for x, o in b.strings]
    sch = flat.ELEMENT_SET_REQUEST
    data, off = flat.encode(codec, sch, cols)
    dcols, st = flat.decode(codec, sch, data, off)
    torch.cuda.synchronize()
    codec.check()
    rec_b = int(b.rec_off[-1])
    str_b = sum(int(o[-1]) for _, o in b.strings)
    ok = bool(np.array_equal(data.cpu().numpy(), b.data)) and bool((st == 0).all().item()) and \
        bool(torch.equal(dcols[0], cols[0])) and all(torch.equal(dcols[k][0][:int(b.strings[k - 1][1][-1])], cols[k][0])
                                                    for k in (1, 2, 3))

    def timed(fn) -> float:
        ev = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            ev.append((e0, e1))
        torch.cuda.synchronize()
        codec.check()
        return float(np.median([a.elapsed_time(c) for a, c in ev]))

    eout = (torch.empty_like(data), torch.empty_like(off))
    enc_ms = timed(lambda: flat.encode(codec, sch, cols, out=eout))
    dec_ms = timed(lambda: flat.decode(codec, sch, data, off, span=rec_b))
    cols_b = 4 * n + str_b + 3 * 8 * (n + 1)
    enc_alg = cols_b + rec_b + 8 * (n + 1)
    dec_alg = rec_b + 8 * (n + 1) + cols_b + n
    gbps = lambda a, ms: round(a / (ms * 1e-3) / 1e9, 1)
    return {"schema": sch.name, "records": n, "record_bytes": int(b.rec_off[1]), "matches_oracle_marshal": ok,
            "encode_ms": round(enc_ms, 4), "encode_gbps": gbps(enc_alg, enc_ms),
            "decode_ms": round(dec_ms, 4), "decode_gbps": gbps(dec_alg, dec_ms),
            "note": "generic flat-schema path; encode into a preallocated buffer, decode allocates its "
                    "columns (caching allocator)"}


def boutique_leg(codec: Codec, dev, reps: int, n: int = 1 << 18) -> dict:
    """SURVEY.md 8f N5 (nested / repeated): online-boutique PlaceOrderResponse messages
    (onlineboutique.proto: OrderResult{ids, Money, Address, 1..5 OrderItem{CartItem, Money}}),
    synthetic (datagen.ob_place_order), the whole message tree encoded and decoded by
    arpc_amd.flat (one launch set per message level, no host read until the end).  Host clock
    around each full call.  The reference README's numbers are Go, one message
    per call, on its 99,848-message trace (Xeon 6142): Symphony Write 2079 ns/op, Read 2939 ns/op."""
    import time

    from arpc_amd import datagen, flat
    sch = flat.OB_PLACE_ORDER_RESPONSE
    tree = datagen.ob_place_order(n)
    cols = flat.columns_from_tree(sch, tree[1], dev)
    data, off = flat.encode(codec, sch, cols)
    dcols, st = flat.decode(codec, sch, data, off)
    data2, off2 = flat.encode(codec, sch, dcols)
    torch.cuda.synchronize()
    codec.check()
    ok = bool(torch.equal(data, data2)) and bool(torch.equal(off, off2)) and bool((st == 0).all().item())
    inner = int(tree[1][0][1][4][2][-1])  # OrderItems

    def timed(fn) -> float:
        fn()  # the timed call's own shapes once untimed (the caching allocator's first blocks)
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        codec.check()
        return float(np.median(ts)) * 1e3, [round(t * 1e3, 3) for t in ts]

    enc_ms, enc_all = timed(lambda: flat.encode(codec, sch, cols))
    dec_ms, dec_all = timed(lambda: flat.decode(codec, sch, data, off, span=data.numel()))
    # the same two walks captured once as HIP graphs over the same buffers (flat.EncodeGraph /
    # DecodeGraph) and replayed; checked against the eager results first
    eg = flat.EncodeGraph(dev, sch, cols)
    dg = flat.DecodeGraph(dev, sch, data, off)
    gd, go = eg.replay()
    gcols, gst = dg.replay()
    gd2, go2 = flat.encode(codec, sch, gcols)
    torch.cuda.synchronize()
    eg.codec.check()
    dg.codec.check()
    g_ok = bool(torch.equal(gd, data)) and bool(torch.equal(go, off)) and bool(torch.equal(gd2, data)) \
        and bool((gst == 0).all().item())
    genc_ms, genc_all = timed(eg.replay)
    gdec_ms, gdec_all = timed(dg.replay)
    eg.codec.close()
    dg.codec.close()
    del eg, dg, gd, go, gcols, gst, gd2, go2
    sb = int(off[-1].item())
    msgs = 4 * n + 3 * inner  # PlaceOrderResponse, OrderResult, Money, Address; per item OrderItem, CartItem, Money
    return {"schema": sch.name, "records": n, "order_items": inner, "messages_per_batch": msgs, "stream_bytes": sb,
            "round_trip_ok": ok, "encode_ms": round(enc_ms, 3), "decode_ms": round(dec_ms, 3),
            "encode_ms_each": enc_all, "decode_ms_each": dec_all,
            "encode_records_per_s": round(n / (enc_ms * 1e-3)), "decode_records_per_s": round(n / (dec_ms * 1e-3)),
            "encode_ns_per_record": round(enc_ms * 1e6 / n, 2), "decode_ns_per_record": round(dec_ms * 1e6 / n, 2),
            "stream_gbps_encode": round(sb / (enc_ms * 1e-3) / 1e9, 1),
            "stream_gbps_decode": round(sb / (dec_ms * 1e-3) / 1e9, 1),
            "reference_readme_ns_per_op": {"write": 2079, "read": 2939},
            "graph": {"round_trip_ok": g_ok, "encode_ms": round(genc_ms, 3), "decode_ms": round(gdec_ms, 3),
                      "encode_ms_each": genc_all, "decode_ms_each": gdec_all,
                      "note": "flat.EncodeGraph / DecodeGraph: each walk captured once as a HIP graph (one stream) "
                              "over the same bound buffers and replayed; host clock around replay + its one read"},
            "note": "host clock around the whole tree call (one launch set per level, inner levels' counts on "
                    "the device, one read of all levels' sizes at the end; one untimed call first, median "
                    "of the rest); synthetic payloads, not the reference's trace"}


def boutique_payloads_leg(codec: Codec, dev, reps: int) -> dict:
    """SURVEY.md 8f N5 on the reference's own workload: the 93,275 online-boutique payloads of 30
    message types (benchmark/serialization/online-boutique/payloads/*.jsonl, kept as data in
    tests/golden/boutique_payloads.json.xz), each type one batch through arpc_amd.flat with
    arpc_amd.boutique's schemas (onlineboutique.proto), device-resident columns.  Host clock around
    all 30 encodes (then all 30 decodes), synchronised at the end.  The reference benchmark
    (bench_test.go:282-351) runs the same payloads one message per call on one CPU core:
    README.md:74-75 quotes Symphony Write 481,109 msg/s and Read 340,225 msg/s (Xeon Gold 6142,
    99,848 payloads of an earlier payload set) -- context, not a like-for-like target."""
    import lzma

    from arpc_amd import boutique, flat
    with lzma.open(os.path.join(ROOT, "tests", "golden", "boutique_payloads.json.xz"), "rt", encoding="utf-8") as fh:
        types = json.load(fh)["types"]
    batches = []
    for name, objs in sorted(types.items()):
        s = boutique.SCHEMAS[name]
        batches.append((s, len(objs), boutique.columns_from_json(s, objs, dev)))
    nmsg = sum(n for _, n, _ in batches)
    enc = [flat.encode(codec, s, cols, n=n) for s, n, cols in batches]
    dec = [flat.decode(codec, s, d, o, span=d.numel()) for (s, n, _), (d, o) in zip(batches, enc)]
    torch.cuda.synchronize()
    codec.check()
    ok = all(bool((st == 0).all().item()) for _, st in dec)
    stream_b = sum(int(d.numel()) for d, _ in enc)

    def timed(fn) -> float:
        fn()  # once untimed: the timed calls' own allocations
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        codec.check()
        return float(np.median(ts))

    te = timed(lambda: [flat.encode(codec, s, cols, n=n) for s, n, cols in batches])
    td = timed(lambda: [flat.decode(codec, s, d, o, span=d.numel()) for (s, n, _), (d, o) in zip(batches, enc)])
    # the same 30 walks each captured as a HIP graph (flat.EncodeGraph / DecodeGraph over the same
    # buffers), all 30 launched before any result is read; checked against the eager results first
    graphs = [(flat.EncodeGraph(dev, s, cols, n=n), flat.DecodeGraph(dev, s, d, o))
              for (s, n, cols), (d, o) in zip(batches, enc)]
    g_ok = True
    for (s, n, _), (d, o), (eg, dg) in zip(batches, enc, graphs):
        gd, go = eg.replay()
        gcols, gst = dg.replay()
        rd, ro = flat.encode(codec, s, gcols, n=n)
        g_ok &= bool(torch.equal(gd, d)) and bool(torch.equal(go, o)) and bool(torch.equal(rd, d)) \
            and bool((gst == 0).all().item())
    torch.cuda.synchronize()
    for eg, dg in graphs:
        eg.codec.check()
        dg.codec.check()

    def replay_all(k):
        for g in graphs:
            g[k].launch()
        for g in graphs:
            g[k].result()
    tge = timed(lambda: replay_all(0))
    tgd = timed(lambda: replay_all(1))
    for eg, dg in graphs:
        eg.codec.close()
        dg.codec.close()
    del graphs
    return {"types": len(batches), "messages": nmsg, "stream_bytes": stream_b, "all_ok": ok,
            "encode_ms": round(te * 1e3, 3), "decode_ms": round(td * 1e3, 3),
            "encode_msg_per_s": round(nmsg / te), "decode_msg_per_s": round(nmsg / td),
            "graph": {"all_ok": g_ok, "encode_ms": round(tge * 1e3, 3), "decode_ms": round(tgd * 1e3, 3),
                      "encode_msg_per_s": round(nmsg / tge), "decode_msg_per_s": round(nmsg / tgd),
                      "note": "each type's walk captured once as a HIP graph over the same buffers; all 30 "
                              "launched, then their sizes read (host clock around both)"},
            "reference_readme_msg_per_s": {"write": 481109, "read": 340225},
            "note": "all 30 payload files, one batch per type (30 encode and 30 decode tree walks), host clock; "
                    "the reference README's numbers are Go, one message per call, one core"}


def host_inclusive(codec: Codec, kw: dict, dev, steps: int, warm_s: float = 2.0) -> dict:
    """Host memory in, host memory out, through the C ABI's host entry points (what a cgo Serializer
    adapter calls): sym_encode_host then sym_decode_host on the same workload, each call chunked over
    one stream per direction with H2D / kernel / D2H overlapped (arpc_amd/csrc/host.cpp).  Timed with the host
    clock around the synchronous calls, after `warm_s` seconds of the same calls.  Two caller-memory
    kinds: pinned (DMA in place) and pageable (staged through the ctx's pinned buffers).  For
    comparison, the same work serially on one stream (pinned H2D, kernel, D2H, no chunking)."""
    import ctypes

    from arpc_amd import _native
    L, ctx = codec._lib, codec._ctx
    b = datagen.make_batch(**kw)
    s = b.schema
    n = b.n
    var_total = sum(int(o[-1] - o[0]) for _, o in b.var)
    total = b.encoded_size()
    enc_b, dec_b = alg_bytes(n, s.nvar, var_total, total)

    def cols(pinned: bool):
        mk = (lambda a: torch.from_numpy(a).pin_memory()) if pinned else (lambda a: torch.from_numpy(a.copy()))
        var = [(mk(by), mk(o.view(np.int64))) for by, o in b.var]
        out = torch.empty(total + 16, dtype=torch.uint8, pin_memory=pinned)
        off = torch.empty(n + 1, dtype=torch.int64, pin_memory=pinned)
        dec = [(torch.empty(int(o[-1] - o[0]) + 16, dtype=torch.uint8, pin_memory=pinned),
                torch.empty(n + 1, dtype=torch.int64, pin_memory=pinned)) for _, o in b.var]
        st = torch.empty(n, dtype=torch.uint8, pin_memory=pinned)
        return var, out, off, dec, st

    def run(pinned: bool) -> dict:
        var, out, off, dec, st = cols(pinned)
        bp = _native.ptr_array([x.data_ptr() for x, _ in var])
        op = _native.ptr_array([o.data_ptr() for _, o in var])
        dbp = _native.ptr_array([x.data_ptr() for x, _ in dec])
        dop = _native.ptr_array([o.data_ptr() for _, o in dec])
        caps = _native.u64_array([x.numel() for x, _ in dec])

        def enc():
            _native.check(L.sym_encode_host(ctx, s.schema_id, n, None, bp, op, 0, 0, out.data_ptr(), off.data_ptr()),
                          "sym_encode_host")

        def dcd():
            _native.check(L.sym_decode_host(ctx, s.schema_id, n, out.data_ptr(), off.data_ptr(), None, dbp, caps, dop,
                                            st.data_ptr()), "sym_decode_host")
        enc()
        dcd()  # warm (allocates the slots)
        # PCIe warm-up: a process's first ~1.5 s of copies run at 55 GB/s both ways, 90 after
        # (tools/pcie_pattern.hip, profiles/r04_pcie_pattern.txt: two identical sweeps)
        t_w = time.perf_counter()
        while time.perf_counter() - t_w < warm_s:
            enc()
            dcd()
        ok = bool((st == 0).all()) and all(torch.equal(d[0][:x.numel()], x) for d, (x, _) in zip(dec, var))
        te = td = 0.0
        for _ in range(steps):
            t0 = time.perf_counter()
            enc()
            t1 = time.perf_counter()
            dcd()
            te += t1 - t0
            td += time.perf_counter() - t1
        return {"encode_gbps": round(enc_b * steps / te / 1e9, 2), "decode_gbps": round(dec_b * steps / td / 1e9, 2),
                "gbps_algorithmic": round((enc_b + dec_b) * steps / (te + td) / 1e9, 2),
                "ms_per_step": round((te + td) / steps * 1e3, 3), "round_trip_ok": ok}

    def serial() -> dict:
        var, out, off, dec, st = cols(True)
        d_var = [(torch.empty_like(x, device=dev), torch.empty_like(o, device=dev)) for x, o in var]
        d_out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
        d_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        dd = DecodedBatch(fixed=[], var=[(torch.empty_like(x, device=dev), torch.empty_like(o, device=dev))
                                         for x, o in dec], status=torch.empty(n, dtype=torch.uint8, device=dev))

        def one():
            for (hx, ho), (dx, do) in zip(var, d_var):
                dx.copy_(hx, non_blocking=True)
                do.copy_(ho, non_blocking=True)
            codec.encode(s, [], d_var, out=d_out, out_off=d_off)
            out.copy_(d_out, non_blocking=True)
            off.copy_(d_off, non_blocking=True)
            d_out.copy_(out, non_blocking=True)
            d_off.copy_(off, non_blocking=True)
            codec.decode(s, d_out, d_off, outputs=dd)
            for (hx, ho), (dx, do) in zip(dec, dd.var):
                hx.copy_(dx, non_blocking=True)
                ho.copy_(do, non_blocking=True)
            st.copy_(dd.status, non_blocking=True)
        one()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            one()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        return {"gbps_algorithmic": round((enc_b + dec_b) * steps / el / 1e9, 2), "ms_per_step": round(el / steps * 1e3, 3)}

    def c_caller() -> dict:
        """tests/bin/host_bench: the same entry points from a plain-C process (no torch: /opt/rocm's HIP
        runtime, as a cgo adapter links it) on a config-2-shaped batch (64-byte keys, 256-byte values)."""
        import subprocess
        drv = os.path.join(ROOT, "tests", "bin", "host_bench")
        if not os.path.exists(drv):
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests")], check=True, capture_output=True)
        r = subprocess.run([drv, str(max(steps, 4)), str(warm_s)], capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            raise RuntimeError(r.stdout + r.stderr)
        return json.loads(r.stdout.strip().splitlines()[-1])

    return {"pinned": c_caller(), "pinned_in_torch_process": run(True), "pageable": run(False),
            "serial_one_stream": serial(), "e2e_loopback": e2e_leg(),
            "note": "sym_encode_host + sym_decode_host (chunked, one stream per direction, H2D/kernel/D2H "
                    "overlapped), host clock after a 2 s warm-up of the same calls; pinned: from a plain-C "
                    "process (tests/host_bench.c), the caller a cgo adapter is; pinned_in_torch_process: the same "
                    "calls on torch's bundled HIP runtime, which runs D2H copies as blit kernels "
                    "(profiles/r04_host_timeline.txt); "
                    "algorithmic bytes as the headline; serial_one_stream: the same work unchunked on one stream"}


def e2e_leg(rpcs: int = 1 << 18, window: int = 4096, inflight: int = 2) -> dict:
    """BASELINE config 5's stand-in: tests/e2e_loopback.c, a plain-C client and server process over UDP
    127.0.0.1 exchanging kv Set RPCs (K=64, V=256) with the HIP codec, packetizer and reassembler on
    both sides (C stand-in for the aRPC pair: no Go toolchain).  Host clock around the whole exchange:
    H2D + kernels + D2H + sendmmsg / recvmmsg.  One untimed short run first (process and HIP start-up,
    PCIe warm-up)."""
    import subprocess
    drv = os.path.join(ROOT, "tests", "bin", "e2e_loopback")
    if not os.path.exists(drv):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests")], check=True, capture_output=True)
    env = dict(os.environ, E2E_NOVERIFY="1")
    subprocess.run([drv, str(4 * window), str(window), "64", "256", str(inflight)], capture_output=True, text=True,
                   timeout=120, env=env)
    r = subprocess.run([drv, str(rpcs), str(window), "64", "256", str(inflight)], capture_output=True, text=True,
                       timeout=300, env=env)
    if r.returncode != 0:
        raise RuntimeError(r.stdout + r.stderr)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    out["note"] = ("C stand-in for the aRPC client/server pair (tests/e2e_loopback.c; no Go toolchain): Set RPCs "
                   "over UDP loopback, request and response each encoded, packetized, reassembled and decoded "
                   "on the GPU through the C ABI; gbps_algorithmic counts the four codec calls' bytes "
                   "(SURVEY 8d definition) per RPC; host clock around the whole exchange; every response's "
                   "status and length checked (verified: false = the value bytes are not compared here, "
                   "tests/test_e2e_loopback.py compares them)")
    return out


def per_record_leg(records: int, threads: int) -> dict:
    """The per-record Serializer path (SURVEY.md 8b "Threading"; pkg/rpc/client.go:233-310,
    pkg/serializer/symphony.go:10-16): one SetRequest per call, from a plain-C client
    (tests/batcher_driver.c, a child process) -- without coalescing (one sym_encode_host +
    sym_decode_host call per record: the latency of a record alone) and through the coalescing
    batcher (sym_batcher_encode_one + decode_one) at 1 thread (its per-record latency) and at
    `threads` threads (throughput).  Records: key 0-69 B, value 0-299 B (the driver's rec())."""
    import subprocess
    drv = os.path.join(ROOT, "tests", "bin", "batcher_driver")
    if not os.path.exists(drv):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests")], check=True, capture_output=True)

    def run(*args) -> float:
        r = subprocess.run([drv, *[str(a) for a in args]], capture_output=True, text=True, timeout=120)
        if r.returncode != 0:
            raise RuntimeError(r.stdout + r.stderr)
        return float(r.stdout.rsplit("elapsed_s=", 1)[1].split()[0])

    h1 = run(1, records, "-", "host1")
    b1 = run(1, records, "-", "bench")
    per = max(1, (4 * records) // threads)
    bt = run(threads, per, "-", "bench")
    us = lambda el, k: round(el / k * 1e6, 2)  # noqa: E731
    return {"unbatched_n1": {"records": records, "us_per_record_enc_plus_dec": us(h1, records),
                             "records_per_s": round(records / h1, 1)},
            "batcher_1_thread": {"records": records, "us_per_record_enc_plus_dec": us(b1, records),
                                 "records_per_s": round(records / b1, 1)},
            f"batcher_{threads}_threads": {"records": threads * per, "records_per_s": round(threads * per / bt, 1),
                                           "calls_per_s": round(2 * threads * per / bt, 1)},
            "note": "plain-C client (tests/batcher_driver.c): each record is one Marshal-like and one "
                    "Unmarshal-like call; records_per_s counts records through both; compare "
                    "cpu_baseline.config1_echo (the C restatement, one record per call on one core)"}


def pair_timing(reps: int, enc_fn, dec_fn) -> tuple[float, float, float]:
    """Times `reps` (encode i, decode i) pairs twice on the current stream: once with HIP events around
    each call (the per-kernel averages), once with events only around the whole block (ms per pair:
    a timing event's record adds a system-scope release, ~3 us, to the stream, so per-call events
    inflate the pair time; the headline's steps are timed the same way).  Returns (encode ms,
    decode ms, ms per pair)."""
    ev_e, ev_d = [], []
    for i in range(reps):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        enc_fn(i)
        e1.record()
        dec_fn(i)
        e2.record()
        ev_e.append((e0, e1))
        ev_d.append((e1, e2))
    b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    b0.record()
    for i in range(reps):
        enc_fn(i)
        dec_fn(i)
    b1.record()
    torch.cuda.synchronize()
    enc_ms = float(np.mean([a.elapsed_time(c) for a, c in ev_e]))
    dec_ms = float(np.mean([a.elapsed_time(c) for a, c in ev_d]))
    return enc_ms, dec_ms, b0.elapsed_time(b1) / reps


def mixed_leg(codec: Codec, dev, reps: int, cfg=None) -> dict:
    """BASELINE config 2 as written ("1 M kv-store-symphony Get/Set records"): 2^20 requests at the
    trace's 36.9 % SetRequest share (datagen.CONFIG2_MIXED), K=64, V=256, encoded with
    sym_encode_kv_mixed (size pass + encode) and decoded with sym_decode_kv_mixed, device-resident,
    HIP events, two rotating buffer sets.  Algorithmic bytes -- encode: type n + keys + key offsets
    8(n+1) + Set values + value offsets 8(n+1) read, stream + 8(n+1) offsets written; decode: stream +
    8(n+1) + type n read, keys + values + 2 x 8(n+1) offsets + n status written."""
    b = datagen.make_mixed_batch(**(cfg or datagen.CONFIG2_MIXED))
    n = b.n
    total = b.encoded_size()
    kb, vb = int(b.key[1][-1]), int(b.val[1][-1])
    sets = []
    for k in range(2):
        t = torch.from_numpy(b.type).to(dev)
        key = (torch.from_numpy(b.key[0]).to(dev) ^ (0x3B * k), torch.from_numpy(b.key[1].view(np.int64)).to(dev))
        val = (torch.from_numpy(b.val[0]).to(dev) ^ (0x3B * k), torch.from_numpy(b.val[1].view(np.int64)).to(dev))
        out = (torch.empty(total + 16, dtype=torch.uint8, device=dev), torch.empty(n + 1, dtype=torch.int64, device=dev))
        dec = DecodedBatch(fixed=[], var=[(torch.empty(kb + 16, dtype=torch.uint8, device=dev),
                                           torch.empty(n + 1, dtype=torch.int64, device=dev)),
                                          (torch.empty(vb + 16, dtype=torch.uint8, device=dev),
                                           torch.empty(n + 1, dtype=torch.int64, device=dev))],
                           status=torch.empty(n, dtype=torch.uint8, device=dev))
        sets.append((t, key, val, out, dec))
    for t, key, val, out, dec in sets:
        codec.encode_kv_mixed(t, key, val, 1, 1, 2, out=out[0], out_off=out[1])
        codec.decode_kv_mixed(out[0], out[1], t, outputs=dec)
    codec.check()
    ok = all(bool((dec.status == 0).all()) and torch.equal(dec.var[1][0][:vb], val[0]) and
             torch.equal(dec.var[0][0][:kb], key[0]) for t, key, val, out, dec in sets)
    def enc_fn(i):
        t, key, val, out, _ = sets[i % 2]
        codec.encode_kv_mixed(t, key, val, 1, 1, 2, out=out[0], out_off=out[1])

    def dec_fn(i):
        t, _, _, out, dec = sets[(i + 1) % 2]
        codec.decode_kv_mixed(out[0], out[1], t, outputs=dec)

    enc_ms, dec_ms, pair_ms = pair_timing(reps, enc_fn, dec_fn)
    codec.check()
    enc_alg = n + kb + 8 * (n + 1) + vb + 8 * (n + 1) + total + 8 * (n + 1)
    dec_alg = total + 8 * (n + 1) + n + kb + vb + 16 * (n + 1) + n
    nset = int(b.type.sum())
    # the leg's own roofline: its dominant kernel by time, traffic from the mixed workload's profile
    if enc_ms >= dec_ms:
        kname, dom_ms, dom_b = ENCODE_MIXED_KERNEL, enc_ms, enc_alg
    else:
        kname, dom_ms, dom_b = decode_kernel_name(schemas.BY_NAME["kv_set_request"], mixed=True), dec_ms, dec_alg
    ach = dom_b / (dom_ms * 1e-3) / 1e9
    roof = {"bound": "hbm", "kernel": kname, "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBPS, 4),
            "traffic": load_traffic(kname, "mixed") if cfg is None else None}
    return {"records": n, "set_records": nset, "set_fraction": round(nset / n, 4), "stream_bytes": total,
            "roofline": roof,
            "round_trip_ok": ok, "encode_ms": round(enc_ms, 4), "encode_gbps": round(enc_alg / enc_ms / 1e6, 1),
            "decode_ms": round(dec_ms, 4), "decode_gbps": round(dec_alg / dec_ms / 1e6, 1),
            "ms_per_pair": round(pair_ms, 4),
            "gbps_algorithmic": round((enc_alg + dec_alg) / pair_ms / 1e6, 1),
            "gbps_algorithmic_per_call_events": round((enc_alg + dec_alg) / (enc_ms + dec_ms) / 1e6, 1),
            "mrecords_per_s": round(n / pair_ms / 1e3, 1),
            "note": "Get/Set mix at the trace_large.req ratio (9,267 SET / 25,125); encode = one launch (sizer "
                    "groups, scanner, encode tiles); client IDs: service 1, Get 1, Set 2"}


def config3_leg(codec: Codec, dev, reps: int, cfg=None, workload: str | None = "config3") -> dict:
    """2^20 SetRequests, K=64, V log-uniform 16-4096 B (mean ~736 B, 774 MB stream:
    no set fits the Infinity Cache), encode + decode device-resident, HIP events, two buffer sets.
    `cfg` another SetRequest workload (the trace sizes, config 4's shard); `workload` names its traffic
    entry in profiles/traffic.json for the leg's roofline (None: no traffic figure)."""
    b = datagen.make_batch(**(cfg or datagen.CONFIG3))
    s = b.schema
    n = b.n
    var_total = sum(int(o[-1] - o[0]) for _, o in b.var)
    total = b.encoded_size()
    fixed0, var0 = to_device(b, dev)
    del b
    caps = [int(o[-1].item() - o[0].item()) for _, o in var0]
    sets = []
    for k in range(2):
        var = [((x ^ (0x3B * k)) if k else x, o.clone()) for x, o in var0]
        enc = (torch.empty(total + 16, dtype=torch.uint8, device=dev), torch.empty(n + 1, dtype=torch.int64, device=dev))
        dec = DecodedBatch(fixed=[], var=[(torch.empty(c + 16, dtype=torch.uint8, device=dev),
                                           torch.empty(n + 1, dtype=torch.int64, device=dev)) for c in caps],
                           status=torch.empty(n, dtype=torch.uint8, device=dev))
        codec.encode(s, [], var, out=enc[0], out_off=enc[1])
        sets.append((var, enc, dec))
    for _, enc, dec in sets:  # untimed decodes: first-touch of the output columns stays out of the timing
        codec.decode(s, enc[0], enc[1], outputs=dec)
    codec.check()
    def enc_fn(i):
        var, enc, _ = sets[i % 2]
        codec.encode(s, [], var, out=enc[0], out_off=enc[1])

    def dec_fn(i):
        _, enc, dec = sets[(i + 1) % 2]
        codec.decode(s, enc[0], enc[1], outputs=dec)

    enc_ms, dec_ms, pair_ms = pair_timing(reps, enc_fn, dec_fn)
    codec.check()
    ok = all(bool((dec.status == 0).all()) and torch.equal(dec.var[1][0][:caps[1]], var[1][0])
             for var, _, dec in sets)
    enc_b, dec_b = alg_bytes(n, s.nvar, var_total, total)
    dname = decode_kernel_name(s)
    kname, dom_ms, dom_b = (ENCODE_KERNEL, enc_ms, enc_b) if enc_ms >= dec_ms else (dname, dec_ms, dec_b)
    ach = dom_b / (dom_ms * 1e-3) / 1e9
    roof = {"bound": "hbm", "kernel": kname, "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": load_traffic(kname, workload) if workload else None}
    return {"records": n, "stream_bytes": total, "round_trip_ok": ok, "roofline": roof,
            "encode_ms": round(enc_ms, 4), "encode_gbps": round(enc_b / enc_ms / 1e6, 1),
            "decode_ms": round(dec_ms, 4), "decode_gbps": round(dec_b / dec_ms / 1e6, 1),
            "ms_per_pair": round(pair_ms, 4),
            "gbps_algorithmic": round((enc_b + dec_b) / pair_ms / 1e6, 1),
            "gbps_algorithmic_per_call_events": round((enc_b + dec_b) / (enc_ms + dec_ms) / 1e6, 1),
            "kernels": {"encode": ENCODE_KERNEL, "decode": dname},
            "note": "config 3 (seed 0x5EED0002), the headline's algorithmic byte definition"}


def summary_of(line: dict) -> dict:
    """A compact digest of the line's legs (GB/s, roofline fraction, ms), printed LAST so that a reader
    keeping only the tail of the line (the driver's record) still sees every BASELINE configuration."""
    r = lambda x, k=1: None if x is None else round(x, k)  # noqa: E731
    frac = lambda g: r(g / HBM_PEAK_GBPS, 4)  # noqa: E731
    out = {"headline": {"config": line["config"]["workload"].split(":")[0], "gbps": line["value"],
                        "frac": line["roofline"]["frac"], "kernel": line["roofline"]["kernel"].split("<")[0],
                        "enc_ms": line["kernels"]["encode"]["avg_ms"], "dec_ms": line["kernels"]["decode"]["avg_ms"],
                        "n_gpus": line["n_gpus"]}}
    for k in ("mixed", "config3", "config4_shard", "config3_trace", "mixed_trace"):
        if k in line:
            x = line[k]
            rf = x.get("roofline", {})
            out[k] = {"gbps": x["gbps_algorithmic"], "frac": rf.get("frac"),
                      "frac_of": "dec" if rf.get("kernel", "").startswith("decode") else "enc", "enc_ms": x["encode_ms"], "dec_ms": x["decode_ms"],
                      "ms_per_pair": x["ms_per_pair"]}
    for k in ("reassembly", "reassembly_config3", "reassembly_config3_reordered"):
        if k in line:
            out[k] = {"gbps": line[k]["gbps_algorithmic"], "frac": frac(line[k]["gbps_algorithmic"]),
                      "ms": line[k]["reassemble_ms"]}
    if "packetize" in line:
        out["packetize"] = {"gbps": line["packetize"]["gbps_algorithmic"], "frac": frac(line["packetize"]["gbps_algorithmic"])}
    if "crypto" in line:
        c = line["crypto"]
        out["crypto"] = {"enc_gbps": c["encrypt_gbps"], "dec_gbps": c["decrypt_gbps"], "enc_ms": c["encrypt_ms"],
                         "dec_ms": c["decrypt_ms"]}
    if "proxy" in line:
        out["firewall"] = {"gbps": line["proxy"]["firewall_gbps"], "ms": line["proxy"]["firewall_ms"]}
    if "flat" in line:
        out["flat"] = {"enc_gbps": line["flat"]["encode_gbps"], "dec_gbps": line["flat"]["decode_gbps"]}
    if "boutique" in line:
        b = line["boutique"]
        out["boutique"] = {"graph_enc_ms": b["graph"]["encode_ms"], "graph_dec_ms": b["graph"]["decode_ms"],
                           "eager_enc_ms": b["encode_ms"], "eager_dec_ms": b["decode_ms"]}
    if "boutique_payloads" in line:
        b = line["boutique_payloads"]
        out["boutique_payloads"] = {"graph_enc_msg_s": b["graph"]["encode_msg_per_s"],
                                    "graph_dec_msg_s": b["graph"]["decode_msg_per_s"]}
    if "host_inclusive" in line:
        h = line["host_inclusive"]
        out["host_inclusive"] = {"pinned_gbps": h["pinned"].get("gbps_algorithmic"),
                                 "e2e_rpc_s": h["e2e_loopback"].get("rpc_per_s")}
    if "per_record" in line:
        pr = line["per_record"]
        many = [v for k, v in pr.items() if k.startswith("batcher_") and k != "batcher_1_thread"]
        out["per_record"] = {"us_1_thread": pr["batcher_1_thread"]["us_per_record_enc_plus_dec"],
                             "records_s_many": many[0]["records_per_s"] if many else None}
    if "cpu_baseline" in line:
        c = line["cpu_baseline"]
        out["cpu_baseline"] = {"gbps_1_core": c["value"], "gbps_all": c["all_cores"]["value"],
                               "cores_all": c["all_cores"]["cores"], "kind": c["kind"]}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--prewarm-ms", type=float, default=200.0,
                    help="untimed steps for this much wall time before the warmup steps (GPU clock ramp)")
    ap.add_argument("--kernel-events", type=int, default=5,
                    help="per-kernel HIP events on every k-th timed step (and on the last one if none "
                         "before it); 1: every step; 0: none (the roofline is then unmeasured)")
    ap.add_argument("--overlap", type=int, default=0,
                    help="1: encode and decode of a step on two HIP streams (independent buffer sets), overlapped")
    ap.add_argument("--config", type=int, default=None, choices=(2, 3, 4),
                    help="workload (SURVEY 8d): default 2 at one GPU, 4 (a 2^23-record shard per GPU) at --gpus >= 2")
    ap.add_argument("--records", type=int, default=0, help="records per GPU (default: the config's 2^20)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--host-steps", type=int, default=5, help="host-inclusive steps (0 = skip)")
    ap.add_argument("--packetize-reps", type=int, default=5, help="packetization leg repetitions (0 = skip)")
    ap.add_argument("--proxy-reps", type=int, default=10, help="firewall / Raw getter leg repetitions (0 = skip)")
    ap.add_argument("--reassembly-reps", type=int, default=5, help="reassembly leg repetitions (0 = skip)")
    ap.add_argument("--crypto-reps", type=int, default=3, help="segment cipher leg repetitions (0 = skip)")
    ap.add_argument("--flat-reps", type=int, default=5, help="flat-schema codec leg repetitions (0 = skip)")
    ap.add_argument("--boutique-reps", type=int, default=5, help="online-boutique nested leg repetitions (0 = skip)")
    ap.add_argument("--payload-reps", type=int, default=3,
                    help="online-boutique reference payloads leg (all 30 types) repetitions (0 = skip)")
    ap.add_argument("--mixed-reps", type=int, default=10, help="mixed Get/Set leg repetitions (0 = skip)")
    ap.add_argument("--config3-reps", type=int, default=6, help="config 3 leg repetitions (0 = skip)")
    ap.add_argument("--config4-reps", type=int, default=8,
                    help="config 4 shard leg (2^23 records on this GPU) repetitions at N=1 (0 = skip)")
    ap.add_argument("--trace-reps", type=int, default=3,
                    help="trace-replay legs (config 3 trace sizes, Get/Set trace sequence) repetitions (0 = skip)")
    ap.add_argument("--per-record", type=int, default=2000,
                    help="per-record Serializer path: records per timing run of tests/batcher_driver (0 = skip)")
    ap.add_argument("--ref-reps", type=int, default=-1,
                    help="decode reference timings (three-kernel, look-back only); -1 = max(5, steps/2), 0 = skip")
    ap.add_argument("--launch-check", action="store_true",
                    help="exercise the N-rank launch only (gloo, no GPU) and print the world rank 0 saw")
    args = ap.parse_args()
    if args.config is None:  # BASELINE config 4 is the multi-GPU configuration; config 2 the 1-GPU one
        args.config = 4 if args.gpus > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1 else 2

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if args.launch_check:
        return launch_check(args)
    world, rank, local = dist_setup()
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}; measuring {world} rank(s)", file=sys.stderr)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    kw = workload(args, world, rank)
    s = schemas.BY_NAME[kw["schema"]]
    codec = Codec(dev)

    # ---- synthetic inputs, resident in HBM: NSETS distinct buffer sets ----
    b = datagen.make_batch(**kw)
    n = b.n
    var_total = sum(int(o[-1] - o[0]) for _, o in b.var)
    total = b.encoded_size()
    fixed0, var0 = to_device(b, dev)
    del b
    sets = []
    for k in range(NSETS):  # distinct bytes AND distinct offset tensors per set (nothing stays cache-hot)
        var_k = [((x ^ (0x3B * k)) if k else x, o.clone() if k else o) for x, o in var0]
        sets.append(([f ^ k for f in fixed0], var_k))
    enc = [(torch.empty(total, dtype=torch.uint8, device=dev), torch.empty(n + 1, dtype=torch.int64, device=dev))
           for _ in range(NSETS)]
    caps = [int(o[-1].item() - o[0].item()) for _, o in var0]
    dec = [DecodedBatch(fixed=[torch.empty(n, dtype=torch.int32, device=dev) for _ in range(s.nfixed)],
                        var=[(torch.empty(max(1, c), dtype=torch.uint8, device=dev),
                              torch.empty(n + 1, dtype=torch.int64, device=dev)) for c in caps],
                        status=torch.empty(n, dtype=torch.uint8, device=dev)) for _ in range(NSETS)]
    codec.reserve(n)

    ev = {"enc": [], "dec": []}

    s_enc = torch.cuda.current_stream(dev)
    s_dec = torch.cuda.Stream(dev) if args.overlap else s_enc
    enc_done: list = [None] * NSETS  # event: last encode into enc[k] finished
    dec_done: list = [None] * NSETS  # event: last decode reading enc[k] finished

    def step_overlap(i: int, timed: bool):
        """Encode set a on one stream while set d (encoded two steps earlier) decodes on another:
        the same work as step(), with the cross-stream hazards made explicit by events."""
        a, d = i % NSETS, (i + 2) % NSETS
        fx, vr = sets[a]
        if dec_done[a] is not None:
            s_enc.wait_event(dec_done[a])  # enc[a] is free once its previous decode is done
        if enc_done[d] is not None:
            s_dec.wait_event(enc_done[d])  # enc[d] is complete
        if timed:
            e0, e1, e2, e3 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
            e0.record(s_enc)
        codec.encode(s, fx, vr, out=enc[a][0], out_off=enc[a][1], stream=s_enc)
        ea = torch.cuda.Event()
        ea.record(s_enc)
        enc_done[a] = ea
        if timed:
            e1.record(s_enc)
            e2.record(s_dec)
        codec.decode(s, enc[d][0], enc[d][1], outputs=dec[d], stream=s_dec)
        ed = torch.cuda.Event()
        ed.record(s_dec)
        dec_done[d] = ed
        if timed:
            e3.record(s_dec)
            ev["enc"].append((e0, e1))
            ev["dec"].append((e2, e3))

    last_ev = [None, -2]  # the last instrumented step's closing event and its index (it opens the next one's encode)

    def step(i: int, timed: bool):
        # Every --kernel-events-th timed step carries the per-kernel events (encode, decode + gate): each
        # record is a marker with a system-scope release (~3 us with the L2 a decode leaves dirty; the
        # fence-free and device-release HIP event flags measured slower still), so instrumenting every
        # step would add ~6.5 us of markers to a ~290 us step.
        if args.overlap:
            return step_overlap(i, timed)
        timed = timed and args.kernel_events > 0 and (i % args.kernel_events == args.kernel_events - 1 or
                                                       (i == args.steps - 1 and not ev["dec"]))
        a, d = i % NSETS, (i + 2) % NSETS
        fx, vr = sets[a]
        if timed:
            e0 = last_ev[0] if last_ev[1] == i - 1 else None
            if e0 is None:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record()
            e1, e2 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        codec.encode(s, fx, vr, out=enc[a][0], out_off=enc[a][1])
        if timed:
            e1.record()
        codec.decode(s, enc[d][0], enc[d][1], outputs=dec[d])
        if timed:
            e2.record()
            last_ev[0], last_ev[1] = e2, i
            ev["enc"].append((e0, e1))
            ev["dec"].append((e1, e2))

    for k in range(NSETS):  # every set encoded once before any decode reads it
        fx, vr = sets[k]
        codec.encode(s, fx, vr, out=enc[k][0], out_off=enc[k][1])
    torch.cuda.synchronize()
    # Leave the idle power state first: untimed steps for --prewarm-ms of wall time (a GPU that has
    # just been idle runs the first milliseconds of work at lower clocks), then the W warmup steps.
    t_pw = time.perf_counter()
    k_pw = 0
    while (time.perf_counter() - t_pw) * 1e3 < args.prewarm_ms:
        step(k_pw, False)
        k_pw += 1
        if k_pw % 8 == 0:
            torch.cuda.synchronize()
    for i in range(args.warmup):
        step(k_pw + i, False)
    codec.check()

    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, True)
    torch.cuda.synchronize()
    barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world, dev)
    codec.check()
    # correctness spot check of the last decode (outside the timed region)
    d_last = (args.steps - 1 + 2) % NSETS
    assert int(dec[d_last].status.sum().item()) == 0, "decode reported errors"
    assert torch.equal(dec[d_last].var[-1][0][:caps[-1]], sets[d_last][1][-1][0]), "round trip mismatch"

    enc_ms = float(np.mean([a.elapsed_time(b_) for a, b_ in ev["enc"]]))
    dec_ms = float(np.mean([a.elapsed_time(b_) for a, b_ in ev["dec"]]))
    enc_b, dec_b = alg_bytes(n, s.nvar, var_total, total)
    value = world * (enc_b + dec_b) * args.steps / elapsed / 1e9
    # Reference points for the decode, outside the timed region on the same buffers and stream: the
    # three-kernel decode and the pipeline's forced look-back mode (its progress fallback), selected
    # with sym_ctx_set_decode_impl.  Same results; timings only.
    def time_impl(impl: int, reps: int) -> float:
        evs = []
        codec.set_decode_impl(impl)
        try:
            for i in range(reps):
                d = (i + 2) % NSETS
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                codec.decode(s, enc[d][0], enc[d][1], outputs=dec[d])
                e1.record()
                evs.append((e0, e1))
        finally:
            codec.set_decode_impl(0)
        torch.cuda.synchronize()
        return float(np.mean([a.elapsed_time(b_) for a, b_ in evs]))

    reps = max(5, args.steps // 2) if args.ref_reps < 0 else args.ref_reps
    refs = {}
    if reps:
        three_ms, lookback_ms = time_impl(1, reps), time_impl(2, reps)
        refs = {"three_kernel_ms": round(three_ms, 4), "three_kernel_gbps": round(dec_b / three_ms / 1e6, 1),
                "lookback_only_ms": round(lookback_ms, 4),
                "lookback_note": "SYM_DECODE_LOOKBACK: parsers and scanner idle, every copier resolves its prefix "
                                 "by look-back (the progress fallback)"}
    codec.check()
    glob = None
    if world > 1:  # the shards as one global stream: rebase by the exclusive scan of shard totals
        from arpc_amd import shard
        base, gtotal = shard.global_base(total)
        glob = {"rank0_base": base, "global_stream_bytes": gtotal, "global_records": n * world}
    # roofline: the dominant single kernel by time (the default decode is one launch)
    if enc_ms >= dec_ms:
        kname, dom_ms, dom_bytes = f"encode_kernel<{s.nfixed}, {s.nvar}, 1, false, 4, false, 64>", enc_ms, enc_b
    else:
        kname, dom_ms, dom_bytes = (decode_kernel_name(s),
                                     dec_ms, dec_b)
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    traffic = load_traffic(kname, f"config{args.config}")

    if rank != 0:
        return
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic: splitmix64 bytes, seed {kw['seed']:#x}"
                + (" + rank (config 4 shard seeds)" if world > 1 else "") + f"; {NSETS} rotating buffer sets",
        "config": {"workload": {2: "config2: kv-store SetRequest K=64 B, V=256 B",
                                 3: "config3: kv-store SetRequest K=64 B, V log-uniform 16-4096 B",
                                 4: "config4: kv-store SetRequest K=64 B, V=256 B, 2^23-record shard per GPU"}[args.config]
                   + ", device-resident encode+decode",
                   "records_per_gpu": n, "global_records": n * world, "parallelism": f"shard{world}", "streams": 2 if args.overlap else 1,
                   "bytes_per_record_algorithmic": round((enc_b + dec_b) / n, 3)},
        "mrecords_per_s": round(world * n * args.steps / elapsed / 1e6, 2),
        "mrecords_per_s_note": "records per second, each record encoded once and decoded once (record "
                               "operations per second = 2x)",
        "wire_gbps": round(world * 2 * total * args.steps / elapsed / 1e9, 2),
        "kernels": {"event_steps": len(ev["dec"]),
                    "event_note": f"HIP events on every {args.kernel_events}th timed step (encode; decode + gate)",
                    "encode": {"avg_ms": round(enc_ms, 4), "alg_bytes": enc_b,
                               "gbps": round(enc_b / enc_ms / 1e6, 1)},
                    "decode": {"avg_ms": round(dec_ms, 4), "alg_bytes": dec_b,
                               "gbps": round(dec_b / dec_ms / 1e6, 1),
                               "kernel": decode_kernel_name(s),
                               **refs}},
        "per_gpu_gbps": round((enc_b + dec_b) * args.steps / elapsed / 1e9, 2),
        "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic},
    }
    if glob:
        line["config"]["global"] = glob
    if world == 1 and args.mixed_reps > 0:
        line["mixed"] = mixed_leg(codec, dev, args.mixed_reps)
    if world == 1 and args.config3_reps > 0 and args.config == 2:
        line["config3"] = config3_leg(codec, dev, args.config3_reps)
    if world == 1 and args.config4_reps > 0 and args.config == 2:
        # the single-GPU anchor of the config-4 scaling curve: rank 0's 2^23-record shard on this GPU
        c4 = config3_leg(codec, dev, args.config4_reps, datagen.config4_shard(0), workload="config4")
        c4["note"] = ("SURVEY 8d config 4's shard 0 (2^23 SetRequests, K=64, V=256, seed 0x5EED0003): what each "
                      "rank of `bench.py --gpus N` (default config 4 at N >= 2) encodes and decodes per step")
        line["config4_shard"] = c4
    if world == 1 and args.reassembly_reps > 0:  # the general (multi-datagram) reassembly path
        b3 = datagen.make_batch(**datagen.CONFIG3)
        f3, v3 = to_device(b3, dev)
        e3 = codec.encode(b3.schema, f3, v3, var_total=b3.encoded_size() - b3.n * b3.schema.overhead)
        del b3, f3, v3
        rc3 = reassembly_leg(codec, e3.data, e3.offsets, dev, args.reassembly_reps)
        rc3["note"] = ("config 3 (V log-uniform 16-4096 B) packetized, send order: records over 1369 payload bytes "
                       "span several datagrams; the parse recognises the packetizer's runs, so no regrouping")
        line["reassembly_config3"] = rc3
        rr = reassembly_leg(codec, e3.data, e3.offsets, dev, args.reassembly_reps, window=64)
        rr["note"] = ("config 3 packetized, datagrams shuffled within windows of 64: the general path (hash "
                      "grouping, radix sort, group passes, the exclusive scan in arrival order)")
        line["reassembly_config3_reordered"] = rr
        del e3
    if world == 1 and args.trace_reps > 0:
        t3 = config3_leg(codec, dev, args.trace_reps, datagen.config3_trace())
        t3["note"] = ("SURVEY 8d config 3, secondary variant: 2^20 SetRequests with the SET key sizes and "
                      "the SET value sizes (clipped to [16, 4096]) of benchmark/meta-kv-trace/trace_large.req "
                      "in trace order (tests/golden/trace_large_sizes.json), seed 0x5EED0002")
        line["config3_trace"] = t3
        tm = mixed_leg(codec, dev, args.trace_reps, datagen.config2_trace_mixed())
        tm["note"] = ("the kv benchmark's request stream replayed: trace_large.req's GET/SET sequence, key sizes "
                      "and SET value sizes (clipped to [16, 4096]), cycled to 2^20 requests; one-launch "
                      "encode, pipeline decode")
        line["mixed_trace"] = tm
    if world == 1 and args.host_steps > 0:
        line["host_inclusive"] = host_inclusive(codec, kw, dev, args.host_steps)
    if world == 1 and args.packetize_reps > 0:
        line["packetize"] = packetize_leg(codec, enc[0][0], enc[0][1], dev, args.packetize_reps)
    if world == 1 and args.reassembly_reps > 0:
        line["reassembly"] = reassembly_leg(codec, enc[0][0], enc[0][1], dev, args.reassembly_reps)
    if world == 1 and args.crypto_reps > 0:
        line["crypto"] = crypto_leg(codec, enc[0][0], enc[0][1], dev, args.crypto_reps)
    if world == 1 and args.proxy_reps > 0:
        line["proxy"] = proxy_leg(codec, dev, args.proxy_reps)
    if world == 1 and args.flat_reps > 0:
        line["flat"] = flat_leg(codec, dev, args.flat_reps)
    if world == 1 and args.boutique_reps > 0:
        line["boutique"] = boutique_leg(codec, dev, args.boutique_reps)
    if world == 1 and args.payload_reps > 0:
        line["boutique_payloads"] = boutique_payloads_leg(codec, dev, args.payload_reps)
    if world == 1 and args.per_record > 0:
        line["per_record"] = per_record_leg(args.per_record, 64)
    if args.cpu_seconds > 0:  # rank 0 at any N, after the timed region: a bounded sample of <= 2^20 records
        line["cpu_baseline"] = cpu_baseline(dict(kw, n=min(kw["n"], 1 << 20)), args.cpu_seconds)
    line["summary"] = summary_of(line)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
