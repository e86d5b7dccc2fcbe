// sk_hllstr.h -- Redis HLL strings on the host: the codec of the `HYLL` string format (redis 3.2 hyperloglog.c)
// that GET / SET / adopted strings and the exact-strings mode use.  Host-only and free of HIP, so the same code is
// built into the engine (sk_store.cpp) and into the sanitizer fuzz harness (tests/fuzz/fuzz_host.cpp, ASan + UBSan).
#pragma once
#include <stdint.h>

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/redisson_sketch.h"

namespace sk_hll {

// one HLL key as a Redis string in exact mode (see "Redis HLL strings, exact")
struct HllStr {
    uint8_t hdr[16];
    std::vector<uint8_t> ops; // sparse opcodes; empty when dense (the registers are the arena slab)
    bool sparse = false;
};

// redis-server 3.2 keeps an HLL as a string (hyperloglog.c): a 16-B header ("HYLL", encoding, 3 unused bytes, an
// 8-B cached cardinality whose top bit marks it stale) and sparse opcodes -- ZERO 00xxxxxx, XZERO 01xxxxxx
// yyyyyyyy, VAL 1vvvvvxx -- until an update would take the string past hll_sparse_max_bytes (3000) or a register
// past 32, dense after.  Sparse bytes depend on the order registers rose (hllSparseSet splits the opcode that
// covers a register and merges neighbouring VAL opcodes within 5 opcodes of the previous one), so in exact mode
// the apply kernel logs the record of every register rise, and the host replays them in batch order into each
// sparse key's opcodes: the GPU decides every rise, the host keeps the string format (as it keeps the PFCOUNT
// estimator's scalar tail).  The cached-cardinality bytes follow PFADD (stale), single-key PFCOUNT (stored) and
// PFMERGE (dest made dense, stale).
namespace hs {
constexpr size_t kSparseMax = 3000; // server.hll_sparse_max_bytes default
inline bool zero(uint8_t b) { return (b & 0xc0) == 0; }
inline bool xzero(uint8_t b) { return (b & 0xc0) == 0x40; }
inline uint32_t zero_len(uint8_t b) { return (b & 0x3fu) + 1; }
inline uint32_t xzero_len(uint8_t b0, uint8_t b1) { return ((uint32_t(b0 & 0x3f) << 8) | b1) + 1; }
inline int val_value(uint8_t b) { return ((b >> 2) & 0x1f) + 1; }
inline int val_len(uint8_t b) { return (b & 3) + 1; }
inline uint8_t val(int v, int len) { return uint8_t(0x80 | ((v - 1) << 2) | (len - 1)); }
inline int put_zeros(uint8_t *q, uint32_t len) { // ZERO up to 64, XZERO beyond (HLL_SPARSE_ZERO_MAX_LEN)
    if (len > 64) {
        q[0] = uint8_t(0x40 | ((len - 1) >> 8));
        q[1] = uint8_t((len - 1) & 0xff);
        return 2;
    }
    q[0] = uint8_t(len - 1);
    return 1;
}
} // namespace hs

inline void hll_str_init(HllStr &h) { // createHLLObject: sparse XZERO(16384); PFADD / PFMERGE creating it mark the card stale
    std::memset(h.hdr, 0, 16);
    std::memcpy(h.hdr, "HYLL", 4);
    h.hdr[4] = 1;
    h.hdr[15] = 0x80;
    h.ops.assign({0x7f, 0xff});
    h.sparse = true;
}

inline void hll_str_densify(HllStr &h) { // hllSparseToDense: header kept, encoding dense
    h.sparse = false;
    h.hdr[4] = 0;
    std::vector<uint8_t>().swap(h.ops);
}

// hllSparseSet on a sparse string: 0 register not raised, 1 raised, 2 promote (the caller densifies; the arena
// already holds the raised register), -1 the opcodes do not cover the register
inline int hll_sparse_set(HllStr &h, uint32_t index, uint8_t count) {
    if (count > 32) return 2; // HLL_SPARSE_VAL_MAX_VALUE
    std::vector<uint8_t> &o = h.ops;
    size_t p = 0, prev = SIZE_MAX, oplen = 1;
    uint32_t first = 0, span = 0;
    while (p < o.size()) { // the opcode covering `index`
        oplen = 1;
        if (hs::zero(o[p])) span = hs::zero_len(o[p]);
        else if (o[p] & 0x80) span = uint32_t(hs::val_len(o[p]));
        else {
            if (p + 1 >= o.size()) return -1;
            span = hs::xzero_len(o[p], o[p + 1]), oplen = 2;
        }
        if (index <= first + span - 1) break;
        prev = p;
        p += oplen;
        first += span;
    }
    if (p >= o.size() || span == 0) return -1;
    const bool is_zero = hs::zero(o[p]), is_xzero = hs::xzero(o[p]), is_val = !is_zero && !is_xzero;
    bool done = false;
    if (is_val) {
        if (hs::val_value(o[p]) >= count) return 0;
        if (span == 1) o[p] = hs::val(count, 1), done = true;
    }
    if (!done && is_zero && span == 1) o[p] = hs::val(count, 1), done = true;
    if (!done) { // split the opcode: [run before] VAL(count, 1) [run after]
        uint8_t seq[5];
        int n = 0;
        const uint32_t last = first + span - 1;
        if (is_val) {
            const int cur = hs::val_value(o[p]);
            if (index != first) seq[n++] = hs::val(cur, int(index - first));
            seq[n++] = hs::val(count, 1);
            if (index != last) seq[n++] = hs::val(cur, int(last - index));
        } else {
            if (index != first) n += hs::put_zeros(seq + n, index - first);
            seq[n++] = hs::val(count, 1);
            if (index != last) n += hs::put_zeros(seq + n, last - index);
        }
        const long delta = long(n) - long(oplen);
        if (delta > 0 && 16 + o.size() + size_t(delta) > hs::kSparseMax) return 2;
        o.erase(o.begin() + long(p), o.begin() + long(p + oplen));
        o.insert(o.begin() + long(p), seq, seq + n);
    }
    // merge neighbouring VAL opcodes of one value (runs <= 4), scanning <= 5 opcodes from the previous one
    size_t q = prev == SIZE_MAX ? 0 : prev;
    int scan = 5;
    while (q < o.size() && scan--) {
        if (hs::xzero(o[q])) {
            q += 2;
            continue;
        }
        if (hs::zero(o[q])) {
            q++;
            continue;
        }
        if (q + 1 < o.size() && (o[q + 1] & 0x80) && hs::val_value(o[q]) == hs::val_value(o[q + 1])) {
            const int l = hs::val_len(o[q]) + hs::val_len(o[q + 1]);
            if (l <= 4) {
                o[q + 1] = hs::val(hs::val_value(o[q]), l);
                o.erase(o.begin() + long(q));
                continue;
            }
        }
        q++;
    }
    return 1;
}

// Redis HLL strings -> registers (redis 3.2 hyperloglog.c: the 16-B header
// "HYLL", encoding, 3 unused bytes, 8-B cached cardinality; dense = 16384
// 6-bit registers LSB first; sparse = opcodes ZERO 00xxxxxx (1..64 zeros),
// XZERO 01xxxxxx yyyyyyyy (1..16384 zeros), VAL 1vvvvvxx (1..4 registers of
// value 1..32)).  Returns SK_OK, SK_EWRONGTYPE (not an HLL string: what
// isHLLObjectOrReply rejects) or SK_ECORRUPT (sparse opcodes that do not cover
// exactly 16384 registers).
// the 12,288-B dense register body (HLL_DENSE_GET_REGISTER / _SET_REGISTER: 6 bits at bit 6*i, LSB first) <-> 16384
// u8 registers.  The engine's HBM arena holds exactly these bodies.
inline void hll_body_unpack(const uint8_t *body, uint8_t *regs) {
    for (int i = 0; i < 16384; i++) {
        unsigned bit = unsigned(i) * 6, byte = bit >> 3, fb = bit & 7;
        unsigned v = unsigned(body[byte]) >> fb;
        if (fb > 2) v |= unsigned(body[byte + 1]) << (8 - fb);
        regs[i] = uint8_t(v & 63);
    }
}
inline void hll_body_pack(const uint8_t *regs, uint8_t *body) {
    std::memset(body, 0, 12288);
    for (int i = 0; i < 16384; i++) {
        unsigned byte = unsigned(i * 6) / 8, fb = unsigned(i * 6) & 7, v = regs[i] & 63;
        body[byte] |= uint8_t(v << fb);
        if (fb > 2) body[byte + 1] |= uint8_t(v >> (8 - fb));
    }
}

inline int hll_decode(const uint8_t *s, uint64_t len, uint8_t *regs) {
    if (len < 16 || std::memcmp(s, "HYLL", 4) != 0 || s[4] > 1) return SK_EWRONGTYPE;
    if (s[4] == 0) { // dense
        if (len != SK_HLL_DENSE_SIZE) return SK_EWRONGTYPE;
        hll_body_unpack(s + 16, regs);
        return SK_OK;
    }
    uint64_t idx = 0;
    for (uint64_t p = 16; p < len;) {
        uint8_t op = s[p];
        uint64_t run;
        uint8_t val = 0;
        if ((op & 0xc0) == 0x00) run = (op & 0x3f) + 1, p += 1;                            // ZERO
        else if ((op & 0xc0) == 0x40) {                                                    // XZERO
            if (p + 1 >= len) return SK_ECORRUPT;
            run = ((uint64_t(op & 0x3f) << 8) | s[p + 1]) + 1, p += 2;
        } else run = (op & 3) + 1, val = uint8_t(((op >> 2) & 31) + 1), p += 1;            // VAL
        if (idx + run > 16384) return SK_ECORRUPT;
        std::memset(regs + idx, val, run);
        idx += run;
    }
    return idx == 16384 ? SK_OK : SK_ECORRUPT;
}

// registers -> the dense string (HLL_DENSE_SET_REGISTER: 6 bits at bit 6*i, LSB first) into out[SK_HLL_DENSE_SIZE];
// hdr: the 16 header bytes to keep (exact mode), else "HYLL", dense, cached cardinality marked stale
inline void hll_dense_encode(const uint8_t *regs, const uint8_t *hdr, uint8_t *out) {
    std::memset(out, 0, SK_HLL_DENSE_SIZE);
    std::memcpy(out, "HYLL", 4);
    out[15] = 0x80;
    if (hdr) std::memcpy(out, hdr, 16);
    hll_body_pack(regs, out + 16);
}

} // namespace sk_hll
