"""Fixture: the online-boutique benchmark's payloads as data (tests/golden/boutique_payloads.json.xz).

Reads every JSONL file under /root/reference/benchmark/serialization/online-boutique/payloads/ (the
messages the reference benchmark loads, loader.go:16-101: one JSON object per non-empty line, the
file name is the message type) and writes them, in file and line order, as one xz-compressed JSON
document {"source": ..., "types": {type: [object, ...]}}.  Data only: the objects are copied as
parsed (json.loads), nothing of the reference's code is kept.  Run in the build container (the
reference is not on the GPU box); the fixture travels with the repo.

  python tests/golden/make_boutique_payloads.py
"""
import glob
import json
import lzma
import os

SRC = "/root/reference/benchmark/serialization/online-boutique/payloads"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "boutique_payloads.json.xz")


def main():
    types = {}
    for path in sorted(glob.glob(os.path.join(SRC, "*.jsonl"))):
        name = os.path.basename(path)[:-len(".jsonl")]
        with open(path, encoding="utf-8") as fh:
            types[name] = [json.loads(line) for line in fh if line.strip()]
    doc = {"source": "benchmark/serialization/online-boutique/payloads/*.jsonl (appnet-org/arpc)",
           "messages": sum(len(v) for v in types.values()), "types": types}
    with lzma.open(OUT, "wt", encoding="utf-8", preset=9) as fh:
        json.dump(doc, fh, separators=(",", ":"), ensure_ascii=False)
    print(f"{OUT}: {len(types)} types, {doc['messages']} messages")


if __name__ == "__main__":
    main()
