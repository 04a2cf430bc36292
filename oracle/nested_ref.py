"""CPU restatement of the generated MarshalSymphony / UnmarshalSymphony for ANY schema, including
repeated string / bytes and nested (and repeated nested) messages.  TEST INFRASTRUCTURE: only
tests/ and __graft_entry__.smoke() use it, as the checker of the GPU path (arpc_amd/flat.py).

Follows the generator cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:
  marshal   :196-330 (struct: public segment, header, private segment), :334-368 (segment walk),
            :439-469 fixed, :471-491 string / bytes, :493-535 repeated fixed, :537-563 repeated
            string / bytes, :565-590 nested (nil -> 0 table entry, no payload), :592-620 repeated
            nested; the empty message :202-212.
  unmarshal :622-694 (header checks), :696-732 (segment walk), :734-763 fixed ("too short for
            field"), :765-793 string / bytes, :795-841 repeated fixed, :843-880 repeated string /
            bytes (items while they fit: the loop makes no progress after the first that does
            not), :882-909 nested, :911-947 repeated nested (an inner error returns "failed to
            unmarshal nested message").

A schema is any object with `.fields`, each field having name, kind ("bool", "int32", "uint32",
"float", "enum", "int64", "uint64", "double", "string", "bytes", "message"), public, repeated
and message (the inner schema) -- arpc_amd.flat.FlatSchema qualifies.  Values: scalars as their
little-endian bytes, strings / bytes as bytes, repeated scalars as the concatenated element
bytes, repeated strings / bytes as a list of bytes, messages as a dict (None = nil), repeated
messages as a list of dicts.  Pure Python: small batches only.
"""
import struct

WIDTH = {"bool": 1, "int32": 4, "uint32": 4, "float": 4, "enum": 4, "int64": 8, "uint64": 8, "double": 8,
         "string": 0, "bytes": 0, "message": 0}

OK, TOO_SHORT, BAD_VERSION, NO_PRIVATE, FIELD_TOO_SHORT, NESTED = 0, 1, 2, 3, 4, 5


def _fixed(f):
    return WIDTH[f.kind] and not f.repeated


def default(f):
    """The fresh struct's value of a field."""
    if _fixed(f):
        return b"\x00" * WIDTH[f.kind]
    if f.kind == "message":
        return [] if f.repeated else None
    if f.repeated and not WIDTH[f.kind]:
        return []
    return b""


def _payload(f, v):
    """A payload field's bytes after its table entry, or None for a nil message (entry 0)."""
    u32 = lambda x: struct.pack("<I", x)  # noqa: E731
    if f.kind == "message":
        if not f.repeated:
            if v is None:
                return None
            inner = marshal(f.message, v)
            return u32(len(inner)) + inner
        return u32(len(v)) + b"".join(u32(len(b)) + b for b in (marshal(f.message, x) for x in v))
    if f.repeated and not WIDTH[f.kind]:
        return u32(len(v)) + b"".join(u32(len(b)) + b for b in v)
    if f.repeated:
        return u32(len(v) // WIDTH[f.kind]) + v
    return u32(len(v)) + v


def marshal(schema, rec: dict) -> bytes:
    """MarshalSymphony (service / method ids 0)."""
    fields = schema.fields
    if not fields:
        return b"\x01" + struct.pack("<I", 13) + b"\x00" * 8 + b"\x01"

    def segment(fs, table_start, rel):
        table_size = sum(WIDTH[f.kind] if _fixed(f) else 4 for f in fs)
        tab, pay = b"", b""
        for f in fs:
            v = rec.get(f.name, default(f))
            if _fixed(f):
                tab += v
                continue
            p = _payload(f, v)
            if p is None:
                tab += struct.pack("<I", 0)
            else:
                tab += struct.pack("<I", table_start + table_size + len(pay) - rel)
                pay += p
        return tab + pay

    pub = segment([f for f in fields if f.public], 13, 0)
    off2p = 13 + len(pub)
    priv = segment([f for f in fields if not f.public], off2p + 1, off2p)
    return b"\x01" + struct.pack("<I", off2p) + b"\x00" * 8 + pub + b"\x01" + priv


def unmarshal(schema, data: bytes):
    """UnmarshalSymphony into a fresh struct -> (status, values dict, fail position): the position
    in unmarshal order (public fields, then private) of the field where it stopped, len(fields)
    when it did not."""
    fields = schema.fields
    rec = {f.name: default(f) for f in fields}
    L = len(data)
    u32 = lambda q: struct.unpack_from("<I", data, q)[0]  # noqa: E731
    if L < (13 if fields else 14):
        return TOO_SHORT, rec, 0
    if data[0] != 1:
        return BAD_VERSION, rec, 0
    off2p = u32(1)
    if off2p >= L or data[off2p] != 1:
        return NO_PRIVATE, rec, 0
    pos = 0
    for seg in (0, 1):
        ts = 13 if seg == 0 else off2p + 1
        t = 0
        for f in fields:
            if f.public != (seg == 0):
                continue
            if _fixed(f):
                w = WIDTH[f.kind]
                if L < ts + t + w:
                    return FIELD_TOO_SHORT, rec, pos
                rec[f.name] = data[ts + t:ts + t + w]
                t += w
                pos += 1
                continue
            if L >= ts + t + 4:
                po = u32(ts + t)
                if seg and po > 0:
                    po += off2p
                if po > 0 and L >= po + 4:
                    head = u32(po)
                    if f.kind == "message" and not f.repeated:
                        if L >= po + 4 + head:
                            st, inner, _ = unmarshal(f.message, data[po + 4:po + 4 + head])
                            rec[f.name] = inner
                            if st != OK:
                                return NESTED, rec, pos
                    elif f.repeated and not WIDTH[f.kind]:
                        cur, items = po + 4, []
                        for _ in range(head):
                            if L < cur + 4:
                                break
                            il = u32(cur)
                            if L < cur + 4 + il:
                                break
                            items.append(data[cur + 4:cur + 4 + il])
                            cur += 4 + il
                        if f.kind == "message":
                            out = []
                            for it in items:
                                st, inner, _ = unmarshal(f.message, it)
                                out.append(inner)
                                if st != OK:
                                    rec[f.name] = out
                                    return NESTED, rec, pos
                            rec[f.name] = out
                        else:
                            rec[f.name] = items
                    else:
                        nb = head * (WIDTH[f.kind] if f.repeated else 1)
                        if L >= po + 4 + nb:
                            rec[f.name] = data[po + 4:po + 4 + nb]
            t += 4
            pos += 1
    return OK, rec, len(fields)
