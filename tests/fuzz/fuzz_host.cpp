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
//     every length 0..200 at every byte alignment, so a wrong hash is caught before any GPU run.
// Usage: fuzz_host ITERATIONS SEED.  Exits non-zero on a wrong result; the sanitizers abort on any report.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../oracle/sketch_oracle.h"
#include "../../redisson_amd/csrc/sk_device.h"
#include "../../redisson_amd/csrc/sk_hllstr.h"
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

} // namespace

int main(int argc, char **argv) {
    const long iters = argc > 1 ? atol(argv[1]) : 20000;
    Rng r{argc > 2 ? strtoull(argv[2], nullptr, 10) : 1};
    for (long it = 0; it < iters && g_fail == 0; it++) {
        fuzz_hll(r, it);
        fuzz_resp(r, it);
        for (int j = 0; j < 8; j++) fuzz_hash(r, it);
    }
    printf("fuzz_host: %ld iterations, %ld failures\n", iters, g_fail);
    return g_fail ? 1 : 0;
}
