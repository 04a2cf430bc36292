// flat_schema.hpp -- the run-time field descriptor of a flat Symphony message (flat.hip, setters.hip).
#pragma once

#include "../../include/symphony_hip.h"
#include "codec.hpp"

namespace symhip {
namespace flat {

constexpr int kMax = SYM_MAX_FLAT_FIELDS;

// width: a scalar field's width, 0 for payload fields (string / bytes, and repeated fixed-width
// fields, whose payload is [u32 count][count * w bytes], main.go:493-535, :795-841); shift:
// log2 of a repeated field's element width (0 for strings), so count = bytes >> shift.
// list: the list-like payload fields, whose wire payload is a sequence of [u32 len][bytes] items
// (main.go:537-620, :843-947): kListCount = repeated string / bytes / message ([u32 count] then
// the items), kListOne = a nested message (one item, or nothing and a 0 table entry when nil).
// The encoder takes their payload ("body") with its prefixes already in place.
constexpr uint8_t kListNone = 0, kListCount = 1, kListOne = 2;
struct Schema {
    int nf;
    // 32-bit entries: the compiler may fold a byte-array index into the scalar base of a later
    // pointer-array load from the same kernel arguments (base kernarg + k), and a scalar load
    // ignores the low address bits of an unaligned base -- a wrong pointer, then a fault
    uint32_t seg[kMax], width[kMax], shift[kMax], list[kMax];
    uint32_t table[2];  // public / private table bytes
};
SYMHIP_KERNARG_ARRAY(Schema, seg);
SYMHIP_KERNARG_ARRAY(Schema, width);
SYMHIP_KERNARG_ARRAY(Schema, shift);
SYMHIP_KERNARG_ARRAY(Schema, list);
SYMHIP_KERNARG_ARRAY(Schema, table);
static_assert(alignof(Schema) >= 4 && sizeof(Schema) % 4 == 0, "Schema is embedded in kernel arguments");

inline bool is_payload(const sym_field& f) { return f.width == 0 || (f.width & (SYM_FIELD_REPEATED | SYM_FIELD_MESSAGE)); }
inline uint8_t list_kind(const sym_field& f) {
    if (f.width & SYM_FIELD_MESSAGE) return (f.width & SYM_FIELD_REPEATED) ? kListCount : kListOne;
    return f.width == SYM_FIELD_REPEATED ? kListCount : kListNone;  // repeated string / bytes
}

inline Schema make_schema(const sym_field* f, int nf) {
    Schema s{};
    s.nf = nf;
    for (int k = 0; k < nf; ++k) {
        const int ew = f[k].width & ~(SYM_FIELD_REPEATED | SYM_FIELD_MESSAGE | SYM_FIELD_FRAMED);
        s.seg[k] = f[k].segment;
        s.width[k] = is_payload(f[k]) ? 0 : f[k].width;
        s.list[k] = list_kind(f[k]);
        s.shift[k] = (f[k].width & SYM_FIELD_REPEATED) && !s.list[k] ? (ew == 8 ? 3 : ew == 4 ? 2 : 0) : 0;
        s.table[f[k].segment] += s.width[k] ? s.width[k] : 4;
    }
    return s;
}

}  // namespace flat
}  // namespace symhip
