// Sanitizer fuzz harness for the engine's host-side parsers, built with ASan + UBSan on the CPU
// (tests/test_sanitize.py; SURVEY §5 "ASan/UBSan on the C++ CPU path"):
//   * the Redis HLL string codec (redisson_amd/csrc/sk_hllstr.h), which decodes caller-supplied strings on SET /
//     PFADD of an adopted string: hll_decode of valid, random and mutated dense / sparse strings; hllSparseSet replays
//     on decoded sparse strings, each step checked against a register model by decoding the opcodes again; dense
//     encode -> decode round trips;
//     every hllSparseSet step is also compared byte for byte with the oracle's (or_hllstr_set, oracle/);
//   * the RESP request parser of the front-end (redisson_amd/csrc/sk_resp_parse.h), which reads network input:
//     random byte streams, valid pipelines (binary-safe bulk arguments, inline commands) fed in random chunk sizes
//     and parsed back exactly, and mutated pipelines;
//   * the device hash code of redisson_amd/csrc/sk_device.h compiled for the CPU (hipstub/ stands in for the HIP
//     header): XXH64, farmhashuo, the shared-prefix path bloom_hashes_pre and BloomIdx against the oracle, for keys of
//     every length 0..200 at every byte alignment, so a wrong hash is caught before any GPU run;
//   * the Bloom add hash block's per-thread arrays and their index expressions (window bounds, probe indexes, packed
//     ranks, record layout) for one block at k = 2..PM, against the oracle's probes (fuzz_rc_block).
// Usage: fuzz_host ITERATIONS SEED.  Exits non-zero on a wrong result; the sanitizers abort on any report.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include <unistd.h>

#include "../../oracle/sketch_oracle.h"
#include "../../redisson_amd/csrc/sk_device.h"
#include "../../redisson_amd/csrc/sk_hllstr.h"
#include "../../redisson_amd/csrc/sk_rdb.h"
#include "../../redisson_amd/csrc/sk_resp_parse.h"

using namespace sk_hll;

namespace {

struct Rng {
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    }
    uint32_t below(uint32_t n) { return n ? uint32_t(next() % n) : 0; }
};

long g_fail = 0;
void check(bool ok, const char *what, long it) {
    if (!ok) {
        if (g_fail < 20) fprintf(stderr, "FAIL %s (iteration %ld)\n", what, it);
        g_fail++;
    }
}

// a register model: mostly zeros with runs, values 1..maxv
std::vector<uint8_t> random_regs(Rng &r, int maxv) {
    std::vector<uint8_t> m(16384, 0);
    const uint32_t touched = r.below(4) == 0 ? r.below(16385) : r.below(300);
    for (uint32_t t = 0; t < touched; t++) {
        uint32_t i = r.below(16384), run = 1 + r.below(r.below(3) == 0 ? 12 : 2);
        uint8_t v = uint8_t(1 + r.below(uint32_t(maxv)));
        for (uint32_t j = i; j < i + run && j < 16384; j++) m[j] = v;
    }
    return m;
}

// registers (values <= 32) -> sparse opcodes, the encoding redis-server's conversions produce (ZERO <= 64,
// XZERO beyond, VAL runs <= 4)
std::string sparse_encode(const std::vector<uint8_t> &m) {
    std::string o("HYLL\x01\0\0\0\0\0\0\0\0\0\0\x80", 16);
    uint32_t i = 0;
    while (i < 16384) {
        uint32_t j = i;
        while (j < 16384 && m[j] == m[i]) j++;
        uint32_t run = j - i;
        if (m[i] == 0) {
            while (run) {
                uint32_t l = run > 16384 ? 16384 : run;
                uint8_t q[2];
                int n = hs::put_zeros(q, l);
                o.append(reinterpret_cast<char *>(q), size_t(n));
                run -= l;
            }
        } else {
            while (run) {
                uint32_t l = run > 4 ? 4 : run;
                o.push_back(char(hs::val(m[i], int(l))));
                run -= l;
            }
        }
        i = j;
    }
    return o;
}

std::string dense_encode(const std::vector<uint8_t> &m) {
    std::string o(SK_HLL_DENSE_SIZE, '\0');
    hll_dense_encode(m.data(), nullptr, reinterpret_cast<uint8_t *>(&o[0]));
    return o;
}

void mutate(Rng &r, std::string &s) {
    const uint32_t n = 1 + r.below(6);
    for (uint32_t k = 0; k < n; k++) {
        switch (r.below(6)) {
        case 0: if (!s.empty()) s[r.below(uint32_t(s.size()))] ^= char(1u << r.below(8)); break;
        case 1: if (!s.empty()) s[r.below(uint32_t(s.size()))] = char(r.below(256)); break;
        case 2: s.resize(r.below(uint32_t(s.size()) + 1)); break;
        case 3: s.insert(s.begin() + r.below(uint32_t(s.size()) + 1), char(r.below(256))); break;
        case 4: if (!s.empty()) s.erase(s.begin() + r.below(uint32_t(s.size()))); break;
        default: s.append(r.below(8), char(r.below(256))); break;
        }
    }
}

// decode into an exactly sized heap buffer (ASan sees any write past the 16384 registers)
int decode(const std::string &s, std::vector<uint8_t> &regs) {
    regs.assign(16384, 0xee);
    std::vector<uint8_t> copy(s.begin(), s.end()); // exact length: reads past the string are reported too
    return hll_decode(copy.data(), copy.size(), regs.data());
}

void fuzz_hll(Rng &r, long it) {
    std::vector<uint8_t> regs;
    const uint32_t kind = r.below(5);
    if (kind == 0) { // valid dense: exact round trip, values 0..63
        std::vector<uint8_t> m = random_regs(r, 63);
        check(decode(dense_encode(m), regs) == SK_OK && regs == m, "dense round trip", it);
        return;
    }
    if (kind == 1) { // valid sparse, then hllSparseSet replays against the model
        std::vector<uint8_t> m = random_regs(r, 32);
        std::string s = sparse_encode(m);
        check(decode(s, regs) == SK_OK && regs == m, "sparse decode", it);
        HllStr h;
        std::memcpy(h.hdr, s.data(), 16);
        h.ops.assign(s.begin() + 16, s.end());
        h.sparse = true;
        std::vector<uint8_t> o(SK_HLL_DENSE_SIZE + 64, 0); // the oracle's string (room for the dense form)
        std::memcpy(o.data(), s.data(), s.size());
        uint64_t olen = s.size();
        const uint32_t steps = 1 + r.below(200);
        for (uint32_t t = 0; t < steps; t++) {
            const uint32_t idx = r.below(16384);
            const uint8_t cnt = uint8_t(1 + r.below(r.below(8) == 0 ? 40 : 32));
            const int rc = hll_sparse_set(h, idx, cnt);
            const int orc = or_hllstr_set(o.data(), &olen, long(idx), cnt);
            check(rc >= 0 && orc >= 0, "sparse set on a valid string", it);
            if (rc == 2) { // promote: the caller densifies (the register is raised in the arena)
                hll_str_densify(h);
                check(!h.sparse && h.hdr[4] == 0 && o[4] == 0, "densify (the oracle promoted too)", it);
                break;
            }
            check((rc == 1) == (cnt > m[idx]) && orc == rc, "sparse set reply", it);
            if (cnt > m[idx]) m[idx] = cnt;
            std::string cur(reinterpret_cast<const char *>(h.hdr), 16);
            cur.append(h.ops.begin(), h.ops.end());
            check(cur.size() == olen && std::memcmp(cur.data(), o.data(), olen) == 0, "sparse bytes equal the oracle's",
                  it);
            check(decode(cur, regs) == SK_OK && regs == m, "sparse opcodes after a set", it);
            if (g_fail) break;
        }
        return;
    }
    // random or mutated strings: any result code, no memory error, and SK_OK only with every register written
    std::string s;
    if (kind == 2) {
        s.assign("HYLL", 4);
        s.push_back(char(r.below(3)));
        for (uint32_t n = r.below(3000); n; n--) s.push_back(char(r.below(256)));
    } else {
        s = kind == 3 ? sparse_encode(random_regs(r, 32)) : dense_encode(random_regs(r, 63));
        mutate(r, s);
    }
    const int rc = decode(s, regs);
    check(rc == SK_OK || rc == SK_EWRONGTYPE || rc == SK_ECORRUPT, "decode result code", it);
    if (rc == SK_OK) {
        bool all = true;
        for (uint8_t v : regs) all = all && v <= 63;
        check(all, "decoded registers <= 63", it);
    }
}

std::string resp_cmd(const std::vector<std::string> &a) {
    std::string o = "*" + std::to_string(a.size()) + "\r\n";
    for (const std::string &x : a) o += "$" + std::to_string(x.size()) + "\r\n" + x + "\r\n";
    return o;
}

void fuzz_resp(Rng &r, long it) {
    std::vector<std::string> args;
    std::string err;
    if (r.below(3) == 0) { // random stream: parse until it needs bytes or errs; every parsed command advances
        std::string buf;
        const char alpha[] = "*$\r\n0123456789-+ \tabcXYZ";
        for (uint32_t n = r.below(400); n; n--)
            buf.push_back(r.below(2) ? alpha[r.below(sizeof(alpha) - 1)] : char(r.below(256)));
        size_t pos = 0;
        for (int guard = 0; guard < 10000; guard++) {
            const size_t before = pos;
            const int rc = sk_resp::parse_command(buf, pos, args, err);
            if (rc != 1) break;
            check(pos > before && pos <= buf.size(), "parser advances", it);
        }
        return;
    }
    // a valid pipeline: multibulk commands with binary arguments and inline commands
    std::vector<std::vector<std::string>> cmds;
    std::string stream;
    for (uint32_t c = 1 + r.below(12); c; c--) {
        std::vector<std::string> a;
        if (r.below(4) == 0) { // inline: words of printable characters
            for (uint32_t w = 1 + r.below(4); w; w--) {
                std::string word;
                for (uint32_t n = 1 + r.below(8); n; n--) word.push_back(char('a' + r.below(26)));
                a.push_back(word);
            }
            std::string line;
            for (size_t i = 0; i < a.size(); i++) line += (i ? " " : "") + a[i];
            stream += line + (r.below(2) ? "\r\n" : "\n");
        } else {
            for (uint32_t w = 1 + r.below(6); w; w--) {
                std::string x;
                for (uint32_t n = r.below(r.below(8) == 0 ? 3000 : 40); n; n--) x.push_back(char(r.below(256)));
                a.push_back(x);
            }
            stream += resp_cmd(a);
        }
        cmds.push_back(a);
    }
    const bool mutated = r.below(3) == 0;
    if (mutated) mutate(r, stream);
    // fed in random chunks, as a socket would deliver it
    std::string buf;
    size_t pos = 0, got = 0, fed = 0;
    bool dead = false;
    while (fed < stream.size() && !dead) {
        const size_t chunk = 1 + r.below(r.below(2) ? 16 : 1500);
        buf.append(stream, fed, chunk);
        fed += chunk;
        for (;;) {
            const size_t before = pos;
            const int rc = sk_resp::parse_command(buf, pos, args, err);
            if (rc == 0) break;
            if (rc < 0) {
                dead = true;
                check(mutated, "valid pipeline parsed without a protocol error", it);
                break;
            }
            check(pos > before, "parser advances", it);
            if (!mutated) {
                check(got < cmds.size() && args == cmds[got], "pipeline command parsed back exactly", it);
            }
            got++;
        }
    }
    if (!mutated) check(got == cmds.size() && pos == buf.size(), "whole pipeline parsed", it);
    long long v;
    check(!sk_resp::parse_ll("", v) && !sk_resp::parse_ll("12a", v) && sk_resp::parse_ll("-42", v) && v == -42,
          "parse_ll", it);
}

// --------------------------------------------------------------- device hash code on the host
struct KeyBuf { // a key at byte alignment `shift` inside zero-padded words, as the device reads it
    uint64_t w[40] = {};
    const uint8_t *put(const uint8_t *p, uint32_t len, uint32_t shift) {
        std::memset(w, 0, sizeof w);
        std::memcpy(reinterpret_cast<uint8_t *>(w) + shift, p, len);
        return reinterpret_cast<const uint8_t *>(w) + shift;
    }
};

void fuzz_hash(Rng &r, long it) {
    static const char jpre[] = "[\"java.lang.Long\",";
    std::string key;
    switch (r.below(4)) {
    case 0: key = jpre + std::to_string(int64_t(r.next())) + "]"; break;                 // a Jackson Long
    case 1: key = std::string(jpre).substr(0, 16); for (uint32_t n = r.below(90); n; n--) key.push_back(char('0' + r.below(10))); break;
    case 2: for (uint32_t n = r.below(200); n; n--) key.push_back(char(r.below(256))); break;
    default: key = jpre + std::to_string(r.below(1000)) + "]"; key[r.below(16)] ^= 1; break;   // one byte off
    }
    std::string pat = r.below(4) ? std::string(jpre).substr(0, 16) : key + std::string(16, 'x'); // the block's pattern
    pat.resize(16);
    const uint32_t len = uint32_t(key.size()), shift = r.below(8);
    KeyBuf kb;
    const uint8_t *p = kb.put(reinterpret_cast<const uint8_t *>(key.data()), len, shift);
    const uint64_t x = or_xxh64(reinterpret_cast<const uint8_t *>(key.data()), len, 0);
    const uint64_t f = or_farmhash_uo64(reinterpret_cast<const uint8_t *>(key.data()), len);
    check(sk::xxh64(p, len) == x, "device xxh64 == oracle", it);
    check(sk::farm_uo64(p, len) == f, "device farmUo == oracle", it);
    uint64_t pw[2];
    std::memcpy(pw, pat.data(), 16);
    const sk::BloomPre pre = sk::bloom_pre(pw[0], pw[1]);
    uint64_t h1, h2;
    sk::bloom_hashes_pre(sk::LdsReader{kb.w, shift}, len, pre, &h1, &h2);
    check(h1 == x && h2 == f, "shared-prefix path == oracle", it);
    // BloomIdx: k probe indexes by two reductions per element == Redisson's per-probe modulo (or_bloom_indexes)
    // Bloom sizes are <= 4,294,967,294 (Q4); BloomIdx is exact below 2^62, tried up to 2^61
    const uint64_t size = r.below(3) ? 4271038538ull : 1 + (r.next() >> (3 + r.below(61)));
    const int k = 1 + int(r.below(12));
    int64_t want[16];
    or_bloom_indexes(reinterpret_cast<const uint8_t *>(key.data()), len, k, int64_t(size), want);
    sk::BloomIdx bi(x, f, size, ~0ull / size);
    for (int q = 0; q < k; q++) {
        check(bi.r == uint64_t(want[q]), "BloomIdx == or_bloom_indexes", it);
        bi.next(q);
    }
    // BloomIdx32 (the region schedule's walk, sizes < 2^32), sizes drawn up to the largest Bloom size
    const uint64_t s32 = r.below(4) == 0 ? 4294967294ull - r.below(3) : r.below(2) ? 4271038538ull : 1 + r.below(~0u - 2);
    or_bloom_indexes(reinterpret_cast<const uint8_t *>(key.data()), len, k, int64_t(s32), want);
    sk::BloomIdx32 b32(x, f, s32, ~0ull / s32);
    for (int q = 0; q < k; q++) {
        check(uint64_t(b32.r) == uint64_t(want[q]), "BloomIdx32 == or_bloom_indexes", it);
        b32.next(q);
    }
}

// ------------------------------------------ the add hash block's per-thread indexing on the host
// k_bloom_rc_hash<true, AEPB> (sk_kernels.hip, "probe p of round e") keeps, per thread, wb[ROUNDS + 1] window bounds
// read at wb[e + 1] / wb[e + 2], and ix[ROUNDS][PM] / rk[ROUNDS][(PM + 1) / 2] (u16 ranks, two per word, rk[e][p >> 1])
// across the block's rounds; the round-4 build that faulted held these in a runtime loop.  The same arrays and index
// expressions run here for one block of AEPB elements (a partial block, ragged round counts, k = 2 a third of the
// time), under UBSan's array-bounds checks and ASan; the block's records (bit-in-region << 13 | element << 1 | last
// probe), laid out by the counting sort's segment starts, must be a permutation of the oracle's probes.
template <uint32_t AEPB, uint32_t PM>
void fuzz_rc_block(Rng &r, long it) {
    constexpr uint32_t TPB = 1024, RB = 19;
    constexpr int ROUNDS = int(AEPB / TPB);
    const uint32_t P = r.below(3) == 0 ? 2u : 2u + r.below(PM - 1);          // k = 2..PM
    const uint64_t size = r.below(3) ? 4271038538ull : 1u << 19 | r.below(~0u - (1u << 19));
    const uint32_t NR = uint32_t((size + (1u << RB) - 1) >> RB);
    const uint32_t n = r.below(4) == 0 ? AEPB : 1 + r.below(AEPB);          // elements of the block
    std::vector<std::string> keys(n);
    std::vector<uint64_t> off(n + 1, 0);
    for (uint32_t i = 0; i < n; i++) {
        keys[i] = "[\"java.lang.Long\"," + std::to_string(int64_t(r.next() >> r.below(64))) + "]";
        off[i + 1] = off[i] + keys[i].size();
    }
    const int nr = int(std::min<uint64_t>((n + TPB - 1) / TPB, ROUNDS));
    uint64_t wb[ROUNDS + 1];
    for (int e = 0; e <= ROUNDS; e++) {
        const uint64_t i0 = uint64_t(e) * TPB;
        wb[e] = off[i0 < n ? i0 : n];
    }
    struct Thread {
        uint32_t ix[ROUNDS][PM], rk[ROUNDS][(PM + 1) / 2];
    };
    std::vector<Thread> th(TPB);
    std::vector<uint32_t> hist(NR, 0);
    for (int e = 0; e < ROUNDS; e++) {
        for (uint32_t t = 0; t < TPB; t++) {
            Thread &T = th[t];
            for (int q = 0; q < int(PM); q++) T.ix[e][q] = 0;
            for (int q = 0; q < int(PM + 1) / 2; q++) T.rk[e][q] = 0;
            if (e >= nr) continue;
            if (e + 1 < nr) check(wb[e + 1] <= wb[e + 2], "window bounds ordered", it);
            const uint64_t i = uint64_t(e) * TPB + t;
            if (i >= n) continue;
            check(off[i] >= wb[e] && off[i + 1] <= wb[e + 1], "element inside its round's window", it);
            const uint32_t len = uint32_t(off[i + 1] - off[i]);
            KeyBuf kb; // the device reads whole words: the key inside zero-padded words, as in the byte arena
            const uint8_t *kp = kb.put(reinterpret_cast<const uint8_t *>(keys[i].data()), len, uint32_t(off[i] & 7u));
            sk::BloomIdx32 bi(sk::xxh64(kp, len), sk::farm_uo64(kp, len), size, ~0ull / size);
            for (int p = 0; p < int(PM); p++) {
                if (uint32_t(p) >= P) break;
                const uint32_t idx = uint32_t(bi.r);
                T.ix[e][p] = idx;
                const uint32_t rank = hist.at(idx >> RB)++;
                T.rk[e][p >> 1] |= rank << ((p & 1) * 16);
                bi.next(p);
            }
        }
    }
    std::vector<uint32_t> start(NR);
    uint32_t tot = 0;
    for (uint32_t q = 0; q < NR; q++) {
        start[q] = tot;
        tot += hist[q];
    }
    check(tot == n * P, "records == elements x probes", it);
    std::vector<uint32_t> lrec(AEPB * PM, 0xffffffffu);
    for (int e = 0; e < ROUNDS; e++)
        for (uint32_t t = 0; t < TPB; t++) {
            const uint64_t i = uint64_t(e) * TPB + t;
            if (e >= nr || i >= n) continue;
            for (int p = 0; p < int(PM); p++) {
                if (uint32_t(p) >= P) break;
                const uint32_t idx = th[t].ix[e][p], rank = (th[t].rk[e][p >> 1] >> ((p & 1) * 16)) & 0xffffu;
                const uint32_t el = uint32_t(e) * TPB + t;
                uint32_t &slot = lrec.at(start.at(idx >> RB) + rank);
                check(slot == 0xffffffffu, "each record slot written once", it);
                slot = (idx << 13) | (el << 1) | (uint32_t(p) + 1 == P ? 1u : 0u);
            }
        }
    // decode by segment: (global bit, element, last) against the oracle's probes
    std::vector<uint64_t> got, want;
    for (uint32_t q = 0; q < NR; q++)
        for (uint32_t s = start[q]; s < start[q] + hist[q]; s++) {
            const uint32_t x = lrec[s];
            got.push_back((uint64_t(q) << RB | (x >> 13)) << 14 | ((x >> 1) & 0xfffu) << 1 | (x & 1u));
        }
    int64_t w[16];
    for (uint32_t i = 0; i < n; i++) {
        or_bloom_indexes(reinterpret_cast<const uint8_t *>(keys[i].data()), uint32_t(keys[i].size()), int(P),
                         int64_t(size), w);
        for (uint32_t p = 0; p < P; p++)
            want.push_back(uint64_t(w[p]) << 14 | uint64_t(i) << 1 | (p + 1 == P ? 1u : 0u));
    }
    std::sort(got.begin(), got.end());
    std::sort(want.begin(), want.end());
    check(got == want, "block records == oracle probes", it);
}

} // namespace

// ---------------------------------------------------------------- redis persistence formats (sk_rdb.h)
// known answers once, then random values through DUMP payloads and RDB file images, and mutated images that must be
// refused or parsed without a memory error
std::string bytes_of(std::initializer_list<int> b) {
    std::string o;
    for (int x : b) o.push_back(char(x));
    return o;
}

void rdb_known(long it) {
    check(sk_rdb::crc64(0, reinterpret_cast<const uint8_t *>("123456789"), 9) == 0xe9c6d914c4b8d9caull,
          "crc64 check value", it);
    // the Redis documentation's DUMP example: SET mykey 10 -> "\x00\xc0\n\t\x00\xbem\x06\x89Z(\x00\n" (RDB 9,
    // the value integer-encoded)
    const std::string doc = bytes_of({0x00, 0xc0, 0x0a, 0x09, 0x00, 0xbe, 0x6d, 0x06, 0x89, 0x5a, 0x28, 0x00, 0x0a});
    sk_rdb::Value v;
    std::string why = sk_rdb::load_payload(reinterpret_cast<const uint8_t *>(doc.data()), doc.size(), v);
    check(why.empty() && v.type == sk_rdb::kTypeString && v.bytes == "10", "redis docs DUMP payload", it);
    std::string bad = doc;
    bad[2] = 0x0b;
    check(!sk_rdb::load_payload(reinterpret_cast<const uint8_t *>(bad.data()), bad.size(), v).empty(),
          "checksum mismatch refused", it);
    // LZF: literal 'a', then a back reference of 9 bytes at distance 1 (ctrl 0xE0, length byte 0, offset 0)
    const std::string lz = bytes_of({0x00, 'a', 0xe0, 0x00, 0x00});
    std::string out(10, '\0');
    check(sk_rdb::lzf_decompress(reinterpret_cast<const uint8_t *>(lz.data()), lz.size(),
                                 reinterpret_cast<uint8_t *>(&out[0]), 10) && out == std::string(10, 'a'),
          "lzf back reference", it);
    // an LZF string claiming a huge uncompressed length: refused before any allocation, valid CRC
    for (uint64_t ulen : {uint64_t(1) << 40, uint64_t(1) << 33, uint64_t(5) * 88 + 1}) {
        std::string pl(1, char(sk_rdb::kTypeString));
        pl.push_back(char(0xc3));
        sk_rdb::put_len(pl, 5);
        sk_rdb::put_len(pl, ulen);
        pl += bytes_of({0x00, 'a', 0xe0, 0xff, 0x00});
        sk_rdb::finish_payload(pl);
        check(!sk_rdb::load_payload(reinterpret_cast<const uint8_t *>(pl.data()), pl.size(), v).empty(),
              "huge LZF ulen refused", it);
    }
    // a ziplist hash as redis 3.2 stores a small HMSET: "size" -> 729 (int16), "hashIterations" -> 5 (immediate)
    std::string ents;
    std::vector<size_t> sizes;
    auto entry = [&](const std::string &e) {
        const size_t prev = sizes.empty() ? 0 : sizes.back();
        std::string x(1, char(prev));
        x += e;
        sizes.push_back(x.size());
        ents += x;
    };
    entry(bytes_of({0x04}) + "size");
    entry(bytes_of({0xc0, 0xd9, 0x02}));
    entry(bytes_of({0x0e}) + "hashIterations");
    entry(bytes_of({0xf6}));
    const uint32_t zlbytes = uint32_t(10 + ents.size() + 1), zltail = uint32_t(10 + ents.size() - sizes.back());
    std::string zl(10, '\0');
    std::memcpy(&zl[0], &zlbytes, 4);
    std::memcpy(&zl[4], &zltail, 4);
    zl[8] = 4;
    zl += ents;
    zl.push_back(char(0xff));
    std::vector<std::string> e;
    check(sk_rdb::ziplist_entries(zl, e) && e.size() == 4 && e[0] == "size" && e[1] == "729" &&
              e[2] == "hashIterations" && e[3] == "5",
          "ziplist hash", it);
    // Redisson's falseProbability strings: BigDecimal.valueOf(d).toPlainString()
    check(sk_rdb::java_plain_double(0.03) == "0.03", "plain 0.03", it);
    check(sk_rdb::java_plain_double(0.008) == "0.008", "plain 0.008", it);
    check(sk_rdb::java_plain_double(1e-6) == "0.0000010", "plain 1.0E-6", it);
    check(sk_rdb::java_plain_double(1.5e-6) == "0.0000015", "plain 1.5E-6", it);
    check(sk_rdb::java_plain_double(0.5) == "0.5", "plain 0.5", it);
    check(sk_rdb::java_plain_double(1.0) == "1.0", "plain 1.0", it);
    check(sk_rdb::java_plain_double(1e7) == "10000000", "plain 1.0E7", it);
}

std::string random_bytes(Rng &r, size_t n) {
    std::string s(n, '\0');
    for (auto &ch : s) ch = char(r.below(256));
    return s;
}

void fuzz_rdb(Rng &r, long it) {
    if (it == 0) rdb_known(it);
    // a random value through a DUMP payload
    sk_rdb::Value v, got;
    std::string p;
    if (r.below(3)) {
        const uint32_t pick = r.below(4);
        const size_t n = pick == 0 ? r.below(64) : pick == 1 ? 64 + r.below(16320) : pick == 2 ? r.below(20) : 16384 + r.below(70000);
        v.bytes = random_bytes(r, n);
        p = sk_rdb::dump_string(v.bytes.data(), v.bytes.size());
    } else {
        v.type = sk_rdb::kTypeHash;
        for (uint32_t i = 0, nf = r.below(9); i < nf; i++)
            v.fields.emplace_back(random_bytes(r, r.below(40)), random_bytes(r, r.below(r.below(8) ? 30 : 300)));
        p = sk_rdb::dump_hash(v.fields);
    }
    {
        std::vector<uint8_t> copy(p.begin(), p.end()); // exact length: reads past it are reported
        std::string why = sk_rdb::load_payload(copy.data(), copy.size(), got);
        check(why.empty() && got.type == v.type && got.bytes == v.bytes && got.fields == v.fields,
              "DUMP payload round trip", it);
    }
    std::string m = p;
    mutate(r, m);
    {
        std::vector<uint8_t> copy(m.begin(), m.end());
        sk_rdb::Value x;
        (void)sk_rdb::load_payload(copy.data(), copy.size(), x); // refused or decoded, never a memory error
        // the CRC is bypassed: the decoder itself over mutated bytes
        if (copy.size() > 1) {
            sk_rdb::Reader rd{copy.data() + 1, copy.data() + copy.size()};
            (void)sk_rdb::load_value(rd, copy[0], x);
        }
    }
    std::string lz = random_bytes(r, r.below(40));
    std::vector<uint8_t> lin(lz.begin(), lz.end()), lout(r.below(80));
    (void)sk_rdb::lzf_decompress(lin.data(), lin.size(), lout.data(), lout.size());
    std::vector<std::string> ze;
    (void)sk_rdb::ziplist_entries(random_bytes(r, r.below(60)), ze);
    // an RDB image of a few records, written through FileWriter and parsed back (every 64th iteration)
    if (it % 64 == 0) {
        char path[] = "/tmp/sk_fuzz_rdbXXXXXX";
        const int fd = mkstemp(path);
        if (fd < 0) return check(false, "mkstemp", it);
        close(fd);
        std::vector<std::pair<std::string, sk_rdb::Value>> recs;
        sk_rdb::FileWriter w;
        check(w.open(path), "rdb open", it);
        for (uint32_t i = 0, n = r.below(6); i < n; i++) {
            sk_rdb::Value x;
            const std::string key = random_bytes(r, 1 + r.below(20));
            if (r.below(2)) {
                x.bytes = random_bytes(r, r.below(3000));
                w.record_head(sk_rdb::kTypeString, key);
                std::string h;
                sk_rdb::put_string(h, x.bytes);
                w.put(h);
            } else {
                x.type = sk_rdb::kTypeHash;
                x.fields = sk_rdb::bloom_config_fields(r.below(1u << 30), int32_t(1 + r.below(9)), r.below(1u << 30),
                                                       1.0 / (2 + r.below(1000)));
                w.record_head(sk_rdb::kTypeHash, key);
                std::string h;
                sk_rdb::put_len(h, x.fields.size());
                for (auto &kv : x.fields) sk_rdb::put_string(h, kv.first), sk_rdb::put_string(h, kv.second);
                w.put(h);
            }
            recs.emplace_back(key, x);
        }
        check(w.close(), "rdb close", it);
        check(access(w.tmp_path.c_str(), F_OK) != 0, "rdb temporary renamed away", it);
        {   // an abandoned writer (an error before close) leaves neither its temporary nor a file at its path
            const std::string gone = std::string(path) + ".abandoned";
            std::string tmp;
            {
                sk_rdb::FileWriter a;
                check(a.open(gone.c_str()), "rdb open (abandoned)", it);
                a.put(reinterpret_cast<const uint8_t *>("x"), 1);
                tmp = a.tmp_path;
            }
            check(access(tmp.c_str(), F_OK) != 0 && access(gone.c_str(), F_OK) != 0, "abandoned rdb leaves nothing",
                  it);
        }
        FILE *f = fopen(path, "rb");
        std::string img;
        char buf[4096];
        size_t k;
        while (f && (k = fread(buf, 1, sizeof buf, f)) > 0) img.append(buf, k);
        if (f) fclose(f);
        unlink(path);
        size_t at = 0;
        auto parse = [&](const std::string &im) {
            std::vector<uint8_t> copy(im.begin(), im.end());
            at = 0;
            return sk_rdb::parse_rdb(copy.data(), copy.size(), [&](const std::string &key, uint8_t t, sk_rdb::Reader &rd) {
                sk_rdb::Value x;
                std::string why = sk_rdb::load_value(rd, t, x);
                if (!why.empty()) return why;
                if (at < recs.size() && (recs[at].first != key || recs[at].second.bytes != x.bytes ||
                                         recs[at].second.fields != x.fields))
                    return std::string("record differs");
                at++;
                return std::string();
            });
        };
        check(parse(img).empty() && at == recs.size(), "RDB file round trip", it);
        std::string bad = img;
        mutate(r, bad);
        (void)parse(bad); // refused or parsed, never a memory error
    }
}

int main(int argc, char **argv) {
    const long iters = argc > 1 ? atol(argv[1]) : 20000;
    Rng r{argc > 2 ? strtoull(argv[2], nullptr, 10) : 1};
    for (long it = 0; it < iters && g_fail == 0; it++) {
        fuzz_hll(r, it);
        fuzz_resp(r, it);
        for (int j = 0; j < 8; j++) fuzz_hash(r, it);
        fuzz_rdb(r, it);
        if (it % 40 == 0) fuzz_rc_block<4096, 7>(r, it);   // k <= RA_K4: 4096-element blocks
        if (it % 40 == 20) fuzz_rc_block<2048, 8>(r, it);  // k = 8
    }
    printf("fuzz_host: %ld iterations, %ld failures\n", iters, g_fail);
    return g_fail ? 1 : 0;
}
