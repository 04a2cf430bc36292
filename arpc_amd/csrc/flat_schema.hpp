// flat_schema.hpp -- the run-time field descriptor of a flat Symphony message (flat.hip, setters.hip).
#pragma once

#include "../../include/symphony_hip.h"
#include "codec.hpp"

namespace symhip {
namespace flat {

constexpr int kMax = SYM_MAX_FLAT_FIELDS;

// width: a scalar field's width, 0 for payload fields (string / bytes, and repeated fixed-width
// fields, whose payload is [u32 count][count * w bytes], main.go:493-535, :795-841); shift:
// log2 of a repeated field's element width (0 for strings), so count = bytes >> shift
struct Schema {
    int nf;
    uint8_t seg[kMax], width[kMax], shift[kMax];
    uint32_t table[2];  // public / private table bytes
};

inline bool is_payload(const sym_field& f) { return f.width == 0 || (f.width & SYM_FIELD_REPEATED); }

inline Schema make_schema(const sym_field* f, int nf) {
    Schema s{};
    s.nf = nf;
    for (int k = 0; k < nf; ++k) {
        const int ew = f[k].width & ~SYM_FIELD_REPEATED;
        s.seg[k] = f[k].segment;
        s.width[k] = is_payload(f[k]) ? 0 : f[k].width;
        s.shift[k] = (f[k].width & SYM_FIELD_REPEATED) ? (ew == 8 ? 3 : ew == 4 ? 2 : 0) : 0;
        s.table[f[k].segment] += s.width[k] ? s.width[k] : 4;
    }
    return s;
}

}  // namespace flat
}  // namespace symhip
