"""BASELINE.json config 5 stand-in: tests/e2e_loopback.c, a plain-C client and server (two processes,
UDP over 127.0.0.1) exchanging kv-store Set RPCs with the HIP codec, packetizer and reassembler on
both sides through the C ABI.  aRPC itself is Go and cannot run here (no Go toolchain); the harness
stands in for frontend.go:109 + pkg/rpc/client.go:233-310 and pkg/rpc/server.go:81-189.

The server checks every decoded request against the generator and the client every response; here
the server's first batch of reassembled request messages is compared byte for byte with the C
oracle's MarshalSymphony plus the client's ID patch (client.go:267-271).
"""
import json
import os
import struct
import subprocess

import numpy as np
import pytest

from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "bin", "e2e_loopback")


def gen_bytes(r: int, n: int, field: int) -> bytes:
    """tests/e2e_loopback.c gen_byte(r, j, field) for j < n."""
    m = (1 << 64) - 1
    j = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = np.uint64(((r + 1) * 0x9E3779B97F4A7C15) & m) ^ (j * np.uint64(0xBF58476D1CE4E5B9)) \
            ^ np.uint64((field * 0x94D049BB133111EB) & m)
        x ^= x >> np.uint64(31)
        x *= np.uint64(0xD6E8FEB86645D07B)
    return (x >> np.uint64(56)).astype(np.uint8).tobytes()


def test_harness_builds():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests"), "bin/e2e_loopback"], check=True)
    assert os.path.exists(BIN)


def test_gen_bytes_matches_c():
    # a value the C expression gives (computed by hand from gen_byte for r=0, j=0, field=0)
    x = (1 * 0x9E3779B97F4A7C15) ^ (1 * 0xBF58476D1CE4E5B9) ^ 0
    x ^= x >> 31
    x = (x * 0xD6E8FEB86645D07B) & ((1 << 64) - 1)
    assert gen_bytes(0, 1, 0)[0] == x >> 56


@pytest.mark.gpu
def test_e2e_loopback_round_trip(tmp_path):
    dump = tmp_path / "req.bin"
    rpcs, K, V = 1 << 16, 64, 256
    r = subprocess.run([BIN, str(rpcs), "4096", str(K), str(V), "2", str(dump)], capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["rpcs"] == rpcs and line["verified"] is True
    assert line["request_datagrams"] == rpcs  # a 350-byte request is one datagram
    blob = dump.read_bytes()
    pos, seen = 0, 0
    while pos < len(blob):
        rpc, n = struct.unpack_from("<QI", blob, pos)
        got = blob[pos + 12:pos + 12 + n]
        pos += 12 + n
        want = oracle.marshal([], [gen_bytes(rpc, K, 0), gen_bytes(rpc, V, 1)], 1, 2)
        assert got == want, rpc
        seen += 1
    assert seen > 0 and pos == len(blob)


@pytest.mark.gpu
def test_e2e_loopback_multi_datagram_requests():
    """4000-byte values: every request spans three datagrams, responses two; the fragments of a
    message may straddle two receive batches (carried over as PENDING)."""
    r = subprocess.run([BIN, "6000", "512", "64", "4000", "2"], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["verified"] is True and line["request_datagrams"] >= 3 * 6000
