"""Derive the request-size fixture tests/golden/trace_large_sizes.json from the reference's trace.

SURVEY.md section 8d, config 3 (secondary variant) and the config-2 Get/Set mix: the kv-store
benchmark replays benchmark/meta-kv-trace/trace_large.req, one request per line
`/?op={GET,SET}&key=<16 hex>&key_size=<n>&value_size=<n>` (the format kv-store/bench_test.go:208-237
parses).  Only the operation sequence and the two sizes are kept -- the sizes are what the codec
sees; the key text itself is workload content and is not needed (datagen draws the bytes).

  python tests/golden/make_trace_sizes.py [/root/reference/benchmark/meta-kv-trace/trace_large.req]
"""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/benchmark/meta-kv-trace/trace_large.req"
LINE = re.compile(r"op=(GET|SET)&key=[0-9a-f]+&key_size=(\d+)&value_size=(\d+)")


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else SRC
    ops, ks, vs = [], [], []
    with open(path) as f:
        for line in f:
            m = LINE.search(line)
            if not m:
                continue
            ops.append("S" if m.group(1) == "SET" else "G")
            ks.append(int(m.group(2)))
            vs.append(int(m.group(3)))
    out = {"source": "benchmark/meta-kv-trace/trace_large.req", "requests": len(ops),
           "sets": ops.count("S"), "ops": "".join(ops), "key_size": ks, "value_size": vs}
    with open(os.path.join(HERE, "trace_large_sizes.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(f"{len(ops)} requests, {ops.count('S')} SET, key sizes {min(ks)}..{max(ks)}, "
          f"SET value sizes {min(v for o, v in zip(ops, vs) if o == 'S')}..{max(vs)}")


if __name__ == "__main__":
    main()
