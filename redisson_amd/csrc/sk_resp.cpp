// sk_resp.cpp -- RESP2 front-end over the sketch engine.
//
// A redis-protocol server for the commands Redisson's probabilistic objects
// send (M:RedissonHyperLogLog.java, M:RedissonBitSet.java,
// M:RedissonBloomFilter.java), so an unmodified Redisson (or redis-cli) can
// point at it instead of redis-server.  One process per GPU, one epoll loop.
//
// Pipelining is where the GPU pays: every read drains the socket, the parsed
// commands run in order, and a run of consecutive PFADD / GETBIT / SETBIT
// commands of one connection becomes ONE engine batch (sk_pfadd / sk_getbit /
// sk_setbit give exact sequential replies inside a batch), which is what an
// RBatch of 100k PFADDs turns into.  Per-command errors (bad offsets, wrong
// types) are answered for that command alone, as redis-server does.
//
// Keys: HLLs and bit strings live in the engine (HBM); small hashes (the Bloom
// filter's "{name}__config", HMSET/HGETALL) live in this process.  EVAL runs
// the three scripts Redisson sends on this path, recognised by the SHA1 of
// their body (tools/script_digests.py derives the digests), natively.
#include "../../include/redisson_sketch.h"
#include "sk_resp_parse.h"
#include "sk_rdb.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace {
using sk_resp::parse_command;
using sk_resp::parse_ll;

// ------------------------------------------------------------------ SHA1
std::string sha1_hex(const std::string &msg) {
    uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    std::string m = msg;
    uint64_t bits = uint64_t(msg.size()) * 8;
    m.push_back(char(0x80));
    while (m.size() % 64 != 56) m.push_back(0);
    for (int i = 7; i >= 0; i--) m.push_back(char((bits >> (8 * i)) & 0xff));
    auto rol = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
    for (size_t blk = 0; blk < m.size(); blk += 64) {
        uint32_t w[80];
        for (int i = 0; i < 16; i++)
            w[i] = uint32_t(uint8_t(m[blk + 4 * i])) << 24 | uint32_t(uint8_t(m[blk + 4 * i + 1])) << 16 |
                   uint32_t(uint8_t(m[blk + 4 * i + 2])) << 8 | uint32_t(uint8_t(m[blk + 4 * i + 3]));
        for (int i = 16; i < 80; i++) w[i] = rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
        for (int i = 0; i < 80; i++) {
            uint32_t f, k;
            if (i < 20) f = (b & c) | (~b & d), k = 0x5A827999u;
            else if (i < 40) f = b ^ c ^ d, k = 0x6ED9EBA1u;
            else if (i < 60) f = (b & c) | (b & d) | (c & d), k = 0x8F1BBCDCu;
            else f = b ^ c ^ d, k = 0xCA62C1D6u;
            uint32_t t = rol(a, 5) + f + e + k + w[i];
            e = d, d = c, c = rol(b, 30), b = a, a = t;
        }
        h[0] += a, h[1] += b, h[2] += c, h[3] += d, h[4] += e;
    }
    char out[41];
    for (int i = 0; i < 5; i++) snprintf(out + 8 * i, 9, "%08x", h[i]);
    return std::string(out, 40);
}

// digests of the scripts Redisson sends (tools/script_digests.py)
const char *kScriptBloomCheck = "e678c622b160a7f36fe9f26aecd0c1a5992e5b0c";  // add/contains config check (:180-186)
const char *kScriptBloomInit = "bae33949534234b07cb5de743c296685dbafadff";   // tryInit config check (:232-236)
const char *kScriptBitsetLength = "a80ae5bc82f0ec7382e36b49cdc6bc589a9a80b3"; // RBitSet.length (:181-191)


void r_simple(std::string &o, const char *s) { o += '+', o += s, o += "\r\n"; }
void r_error(std::string &o, const std::string &s) { o += '-', o += s, o += "\r\n"; }
void r_int(std::string &o, long long v) { o += ':', o += std::to_string(v), o += "\r\n"; }
void r_nil(std::string &o) { o += "$-1\r\n"; }
void r_bulk(std::string &o, const char *p, size_t n) {
    o += '$', o += std::to_string(n), o += "\r\n";
    o.append(p, n);
    o += "\r\n";
}
void r_bulk(std::string &o, const std::string &s) { r_bulk(o, s.data(), s.size()); }
void r_array(std::string &o, size_t n) { o += '*', o += std::to_string(n), o += "\r\n"; }

const char *kWrongType = "WRONGTYPE Operation against a key holding the wrong kind of value";
const char *kNotHll = "WRONGTYPE Key is not a valid HyperLogLog string value.";
const char *kBitOffset = "ERR bit offset is not an integer or out of range";
const char *kBitValue = "ERR bit is not an integer or out of range";
const char *kNotInt = "ERR value is not an integer or out of range";
const char *kSyntax = "ERR syntax error";


std::string lower(std::string s) {
    for (auto &ch : s) ch = char(tolower(uint8_t(ch)));
    return s;
}

// glob-style pattern (KEYS / SCAN MATCH, redis util.c stringmatchlen): * ? [set] [^set] [a-z] and \ escapes
bool glob_match(const char *p, const char *pe, const char *s, const char *se) {
    while (p < pe) {
        if (*p == '*') {
            while (p + 1 < pe && p[1] == '*') p++;
            if (p + 1 == pe) return true;
            for (const char *t = s; t <= se; t++)
                if (glob_match(p + 1, pe, t, se)) return true;
            return false;
        }
        if (s == se) return false;
        if (*p == '?') {
            s++, p++;
            continue;
        }
        if (*p == '[') {
            const char *q = p + 1;
            bool neg = q < pe && *q == '^', hit = false;
            if (neg) q++;
            for (; q < pe && *q != ']'; q++) {
                if (*q == '\\' && q + 1 < pe) {
                    q++;
                    hit |= *q == *s;
                } else if (q + 2 < pe && q[1] == '-' && q[2] != ']') {
                    char a = q[0], b = q[2];
                    if (a > b) std::swap(a, b);
                    hit |= *s >= a && *s <= b;
                    q += 2;
                } else {
                    hit |= *q == *s;
                }
            }
            if (hit == neg) return false;
            p = q < pe ? q + 1 : q;
            s++;
            continue;
        }
        if (*p == '\\' && p + 1 < pe) p++;
        if (*p != *s) return false;
        p++, s++;
    }
    return s == se;
}
bool glob_match(const std::string &pat, const std::string &s) {
    return glob_match(pat.data(), pat.data() + pat.size(), s.data(), s.data() + s.size());
}

// (off u64[n+1], bytes) packing of byte strings for the C ABI
struct Packed {
    std::vector<uint64_t> off{0};
    std::string bytes;
    void add(const std::string &s) {
        bytes += s;
        off.push_back(bytes.size());
    }
    const uint8_t *data() {
        if (bytes.capacity() < bytes.size() + 16) bytes.reserve(bytes.size() + 16);
        return reinterpret_cast<const uint8_t *>(bytes.data());
    }
};

enum KType { T_NONE = 0, T_HLL = 1, T_STR = 2, T_HASH = 10 };

struct Server {
    sk_ctx *ctx = nullptr;
    uint64_t max_bit_offset = 1ull << 32;
    std::string rdb_path = "dump.rdb"; // --dir / --dbfilename: SAVE writes it, startup loads it when present
    // small hashes, field order kept (Redis returns ziplist order for small hashes)
    std::unordered_map<std::string, std::vector<std::pair<std::string, std::string>>> hashes;

    std::string engine_error() { return sk_last_error(ctx); }

    int type_of(const std::string &k) {
        if (hashes.count(k)) return T_HASH;
        int t = 0;
        sk_type(ctx, reinterpret_cast<const uint8_t *>(k.data()), k.size(), &t);
        return (t == SK_TYPE_HLL || t == SK_TYPE_STRING) ? t : T_NONE;
    }
    const std::string *hget(const std::string &k, const std::string &f) {
        auto it = hashes.find(k);
        if (it == hashes.end()) return nullptr;
        for (auto &kv : it->second)
            if (kv.first == f) return &kv.second;
        return nullptr;
    }
    bool del_one(const std::string &k) {
        if (hashes.erase(k)) return true;
        Packed p;
        p.add(k);
        uint64_t n = 0;
        sk_del(ctx, 1, p.off.data(), p.data(), &n);
        return n > 0;
    }
    bool parse_offset(const std::string &s, uint64_t &off) {
        long long v;
        if (!parse_ll(s, v) || v < 0 || uint64_t(v) >= max_bit_offset) return false;
        off = uint64_t(v);
        return true;
    }

    // ---- persistence (sk_rdb.h formats) ---------------------------------
    // every key name: the engine's (a full SCAN) then this process's hashes
    std::vector<std::string> all_keys() {
        std::vector<std::string> out;
        uint64_t cur = 0, nk = 0;
        if (sk_dbsize(ctx, &nk) != SK_OK) return out;
        // one SCAN call for the whole keyspace (a second only if the names outgrow the buffer): O(N log N), not a
        // full pass per 1024 keys
        const uint32_t want = uint32_t(std::min<uint64_t>(nk + 64, 0xfffffff0u));
        std::vector<uint64_t> off(want + 1);
        std::vector<uint8_t> names(std::max<uint64_t>(1 << 20, nk * 48));
        std::vector<int32_t> types(want);
        do {
            uint32_t n = 0;
            if (sk_scan(ctx, cur, want, &cur, &n, off.data(), names.data(), names.size(), types.data()) != SK_OK) break;
            for (uint32_t i = 0; i < n; i++)
                out.emplace_back(reinterpret_cast<const char *>(names.data()) + off[i], off[i + 1] - off[i]);
        } while (cur);
        for (auto &kv : hashes) out.push_back(kv.first);
        return out;
    }
    int save() {
        Packed extra; // the hashes as (key, DUMP payload) pairs
        for (auto &kv : hashes) {
            extra.add(kv.first);
            extra.add(sk_rdb::dump_hash(kv.second));
        }
        uint64_t n = 0;
        return sk_save(ctx, rdb_path.c_str(), uint32_t(hashes.size()), extra.off.data(), extra.data(), &n);
    }
    // sk_load's `take`: every hash stays in this process (the EVAL scripts read the Bloom configs here)
    static int take_hash(void *user, const uint8_t *key, uint64_t klen, const uint8_t *payload, uint64_t plen) {
        sk_rdb::Value v;
        if (!sk_rdb::load_payload(payload, plen, v).empty()) return -1;
        static_cast<Server *>(user)->hashes[std::string(reinterpret_cast<const char *>(key), klen)] = v.fields;
        return 1;
    }
    int load() {
        uint64_t n = 0;
        return sk_load(ctx, rdb_path.c_str(), &Server::take_hash, this, &n);
    }

    // ---- batched runs -------------------------------------------------
    // PFADD key [element ...]: one sk_pfadd over the run
    void run_pfadd(std::vector<std::vector<std::string>> &cmds, size_t a, size_t b, std::vector<std::string> &rep) {
        Packed keys, elems;
        std::vector<uint32_t> counts;
        std::vector<size_t> which;
        for (size_t i = a; i < b; i++) {
            auto &c = cmds[i];
            if (!hashes.empty() && hashes.count(c[1])) {
                r_error(rep[i], kWrongType);
                continue;
            }
            keys.add(c[1]);
            counts.push_back(uint32_t(c.size() - 2));
            for (size_t e = 2; e < c.size(); e++) elems.add(c[e]);
            which.push_back(i);
        }
        if (which.empty()) return;
        std::vector<uint8_t> out(which.size());
        int st = sk_pfadd(ctx, uint32_t(which.size()), keys.off.data(), keys.data(), counts.data(), elems.off.data(),
                          elems.data(), out.data());
        // the engine applies every command on an HLL key (or a valid HLL string, adopted) and
        // skips the rest with a status: key types are looked up only then, to answer those alone
        for (size_t j = 0; j < which.size(); j++) {
            auto &c = cmds[which[j]];
            if (st == SK_OK) r_int(rep[which[j]], out[j]);
            else if (st != SK_EWRONGTYPE && st != SK_ECORRUPT) r_error(rep[which[j]], engine_error());
            else if (type_of(c[1]) == T_HLL) r_int(rep[which[j]], out[j]);
            else { // that command alone again, for its own error (a failed adoption changes nothing)
                Packed k1, e1;
                k1.add(c[1]);
                uint32_t cnt = uint32_t(c.size() - 2);
                for (size_t e = 2; e < c.size(); e++) e1.add(c[e]);
                uint8_t o1;
                sk_pfadd(ctx, 1, k1.off.data(), k1.data(), &cnt, e1.off.data(), e1.data(), &o1);
                r_error(rep[which[j]], engine_error());
            }
        }
    }
    // GETBIT key offset / SETBIT key offset value: one sk_getbit / sk_setbit over the run
    void run_bits(std::vector<std::vector<std::string>> &cmds, size_t a, size_t b, std::vector<std::string> &rep,
                  bool set) {
        Packed keys;
        std::vector<uint64_t> offs;
        std::vector<uint8_t> vals;
        std::vector<size_t> which;
        for (size_t i = a; i < b; i++) {
            auto &c = cmds[i];
            uint64_t off;
            long long v = 0;
            if (!parse_offset(c[2], off)) {
                r_error(rep[i], kBitOffset);
                continue;
            }
            if (set && (!parse_ll(c[3], v) || (v & ~1ll))) {
                r_error(rep[i], kBitValue);
                continue;
            }
            if (!hashes.empty() && hashes.count(c[1])) {
                r_error(rep[i], kWrongType);
                continue;
            }
            keys.add(c[1]);
            offs.push_back(off);
            vals.push_back(uint8_t(v));
            which.push_back(i);
        }
        if (which.empty()) return;
        std::vector<uint8_t> out(which.size());
        int st = set ? sk_setbit(ctx, uint32_t(which.size()), keys.off.data(), keys.data(), offs.data(), vals.data(),
                                 out.data())
                     : sk_getbit(ctx, uint32_t(which.size()), keys.off.data(), keys.data(), offs.data(), out.data());
        // commands on HLL keys are skipped by the engine with SK_EWRONGTYPE (offsets were checked above)
        for (size_t j = 0; j < which.size(); j++) {
            if (st == SK_OK) r_int(rep[which[j]], out[j]);
            else if (st != SK_EWRONGTYPE) r_error(rep[which[j]], engine_error());
            else if (type_of(cmds[which[j]][1]) == T_HLL) r_error(rep[which[j]], kWrongType);
            else r_int(rep[which[j]], out[j]);
        }
    }

    // ---- scripts --------------------------------------------------------
    void run_script(const std::string &sha, const std::vector<std::string> &c, size_t first, std::string &o) {
        long long nk;
        if (!parse_ll(c[first], nk)) return r_error(o, kNotInt);
        if (nk < 0) return r_error(o, "ERR Number of keys can't be negative");
        if (size_t(nk) > c.size() - first - 1) return r_error(o, "ERR Number of keys can't be greater than number of args");
        std::vector<std::string> keys(c.begin() + first + 1, c.begin() + first + 1 + nk);
        std::vector<std::string> argv(c.begin() + first + 1 + nk, c.end());
        std::string fail = "ERR Error running script (call to f_" + sha + "): @user_script:1: ";
        if (sha == kScriptBloomCheck || sha == kScriptBloomInit) {
            if (keys.empty()) return r_error(o, fail + "Script attempted to access a non local key");
            const std::string *size = hget(keys[0], "size"), *hi = hget(keys[0], "hashIterations");
            bool ok = sha == kScriptBloomInit
                          ? (!size && !hi)
                          : (size && hi && argv.size() >= 2 && *size == argv[0] && *hi == argv[1]);
            if (!ok) return r_error(o, fail + "Bloom filter config has been changed");
            return r_nil(o);
        }
        if (sha == kScriptBitsetLength) {
            if (keys.empty()) return r_error(o, fail + "Script attempted to access a non local key");
            if (type_of(keys[0]) == T_HASH) return r_error(o, fail + kWrongType);
            int64_t len = 0;
            int st = sk_bitset_length(ctx, reinterpret_cast<const uint8_t *>(keys[0].data()), keys[0].size(), &len);
            if (st != SK_OK) return r_error(o, engine_error());
            return r_int(o, len);
        }
        r_error(o, "NOSCRIPT No matching script. Please use EVAL.");
    }

    // ---- one command ----------------------------------------------------
    // returns false when the connection should close after the reply (QUIT)
    bool run_one(const std::vector<std::string> &c, std::string &o) {
        std::string name = lower(c[0]);
        auto arity = [&](size_t need, bool at_least) {
            bool ok = at_least ? c.size() >= need : c.size() == need;
            if (!ok) r_error(o, "ERR wrong number of arguments for '" + name + "' command");
            return ok;
        };
        const uint8_t *k1 = c.size() > 1 ? reinterpret_cast<const uint8_t *>(c[1].data()) : nullptr;
        if (name == "ping") {
            if (c.size() > 2) return arity(1, false), true;
            c.size() == 2 ? r_bulk(o, c[1]) : r_simple(o, "PONG");
        } else if (name == "echo") {
            if (arity(2, false)) r_bulk(o, c[1]);
        } else if (name == "quit") {
            r_simple(o, "OK");
            return false;
        } else if (name == "select") {
            if (arity(2, false)) c[1] == "0" ? r_simple(o, "OK") : r_error(o, "ERR invalid DB index");
        } else if (name == "command") {
            r_array(o, 0);
        } else if (name == "flushall" || name == "flushdb") {
            hashes.clear();
            sk_flushall(ctx) == SK_OK ? r_simple(o, "OK") : r_error(o, engine_error());
        } else if (name == "del") {
            if (!arity(2, true)) return true;
            long long n = 0;
            for (size_t i = 1; i < c.size(); i++) n += del_one(c[i]);
            r_int(o, n);
        } else if (name == "exists") {
            if (!arity(2, true)) return true;
            long long n = 0;
            for (size_t i = 1; i < c.size(); i++) n += type_of(c[i]) != T_NONE;
            r_int(o, n);
        } else if (name == "type") {
            if (!arity(2, false)) return true;
            int t = type_of(c[1]);
            r_simple(o, t == T_NONE ? "none" : t == T_HASH ? "hash" : "string");
        } else if (name == "pfcount") {
            if (!arity(2, true)) return true;
            Packed keys;
            for (size_t i = 1; i < c.size(); i++) {
                int t = type_of(c[i]);
                if (t == T_HASH) return r_error(o, kWrongType), true;
                if (t == T_STR) return r_error(o, kNotHll), true;
                keys.add(c[i]);
            }
            uint32_t nk = uint32_t(c.size() - 1);
            int64_t cnt = 0;
            int st = sk_pfcount(ctx, 1, &nk, keys.off.data(), keys.data(), &cnt);
            st == SK_OK ? r_int(o, cnt) : r_error(o, engine_error());
        } else if (name == "pfmerge") {
            if (!arity(2, true)) return true;
            Packed srcs;
            for (size_t i = 1; i < c.size(); i++) {
                int t = type_of(c[i]);
                if (t == T_HASH) return r_error(o, kWrongType), true;
                if (t == T_STR) return r_error(o, kNotHll), true;
                if (i > 1) srcs.add(c[i]);
            }
            int st = sk_pfmerge(ctx, k1, c[1].size(), uint32_t(c.size() - 2), srcs.off.data(), srcs.data());
            st == SK_OK ? r_simple(o, "OK") : r_error(o, engine_error());
        } else if (name == "bitcount") {
            if (!arity(2, true)) return true;
            if (c.size() != 2) return r_error(o, "ERR BITCOUNT with a byte range is not served by this engine"), true;
            if (type_of(c[1]) == T_HASH) return r_error(o, kWrongType), true;
            uint64_t n = 0;
            sk_bitcount(ctx, k1, c[1].size(), &n) == SK_OK ? r_int(o, (long long)n) : r_error(o, engine_error());
        } else if (name == "bitop") {
            if (!arity(4, true)) return true;
            std::string op = lower(c[1]);
            int code = op == "and" ? SK_BITOP_AND : op == "or" ? SK_BITOP_OR : op == "xor" ? SK_BITOP_XOR
                     : op == "not" ? SK_BITOP_NOT : -1;
            if (code < 0) return r_error(o, kSyntax), true;
            Packed srcs;
            for (size_t i = 3; i < c.size(); i++) {
                if (type_of(c[i]) == T_HASH) return r_error(o, kWrongType), true;
                srcs.add(c[i]);
            }
            if (type_of(c[2]) == T_HASH) hashes.erase(c[2]); // BITOP overwrites the destination
            uint64_t len = 0;
            int st = sk_bitop(ctx, code, reinterpret_cast<const uint8_t *>(c[2].data()), c[2].size(),
                              uint32_t(c.size() - 3), srcs.off.data(), srcs.data(), &len);
            st == SK_OK ? r_int(o, (long long)len) : r_error(o, engine_error());
        } else if (name == "strlen") {
            if (!arity(2, false)) return true;
            if (type_of(c[1]) == T_HASH) return r_error(o, kWrongType), true;
            uint64_t n = 0;
            sk_strlen(ctx, k1, c[1].size(), &n) == SK_OK ? r_int(o, (long long)n) : r_error(o, engine_error());
        } else if (name == "get") {
            if (!arity(2, false)) return true;
            if (type_of(c[1]) == T_HASH) return r_error(o, kWrongType), true;
            int64_t len = 0;
            if (sk_get(ctx, k1, c[1].size(), nullptr, 0, &len) != SK_OK) return r_error(o, engine_error()), true;
            if (len < 0) return r_nil(o), true;
            std::string v(size_t(len), '\0');
            if (sk_get(ctx, k1, c[1].size(), reinterpret_cast<uint8_t *>(&v[0]), v.size(), &len) != SK_OK)
                return r_error(o, engine_error()), true;
            r_bulk(o, v);
        } else if (name == "set") {
            if (c.size() < 3) return arity(3, false), true;
            if (c.size() > 3) return r_error(o, kSyntax), true; // EX/PX/NX/XX are not served
            del_one(c[1]); // SET replaces a key of any type
            int st = sk_set(ctx, k1, c[1].size(), reinterpret_cast<const uint8_t *>(c[2].data()), c[2].size());
            st == SK_OK ? r_simple(o, "OK") : r_error(o, engine_error());
        } else if (name == "hmset" || name == "hset") {
            if (!arity(4, true)) return true;
            if ((c.size() - 2) % 2) return r_error(o, "ERR wrong number of arguments for '" + name + "' command"), true;
            if (name == "hset" && c.size() != 4) return arity(4, false), true;
            int t = type_of(c[1]);
            if (t != T_NONE && t != T_HASH) return r_error(o, kWrongType), true;
            auto &h = hashes[c[1]];
            long long added = 0;
            for (size_t i = 2; i + 1 < c.size(); i += 2) {
                auto it = std::find_if(h.begin(), h.end(), [&](auto &kv) { return kv.first == c[i]; });
                if (it == h.end()) h.emplace_back(c[i], c[i + 1]), added++;
                else it->second = c[i + 1];
            }
            name == "hset" ? r_int(o, added) : r_simple(o, "OK");
        } else if (name == "hget") {
            if (!arity(3, false)) return true;
            int t = type_of(c[1]);
            if (t != T_NONE && t != T_HASH) return r_error(o, kWrongType), true;
            const std::string *v = hget(c[1], c[2]);
            v ? r_bulk(o, *v) : r_nil(o);
        } else if (name == "hgetall") {
            if (!arity(2, false)) return true;
            int t = type_of(c[1]);
            if (t != T_NONE && t != T_HASH) return r_error(o, kWrongType), true;
            auto it = hashes.find(c[1]);
            if (it == hashes.end()) return r_array(o, 0), true;
            r_array(o, it->second.size() * 2);
            for (auto &kv : it->second) r_bulk(o, kv.first), r_bulk(o, kv.second);
        } else if (name == "hdel") {
            if (!arity(3, true)) return true;
            int t = type_of(c[1]);
            if (t != T_NONE && t != T_HASH) return r_error(o, kWrongType), true;
            long long n = 0;
            auto it = hashes.find(c[1]);
            if (it != hashes.end()) {
                for (size_t i = 2; i < c.size(); i++) {
                    auto &h = it->second;
                    auto f = std::find_if(h.begin(), h.end(), [&](auto &kv) { return kv.first == c[i]; });
                    if (f != h.end()) h.erase(f), n++;
                }
                if (it->second.empty()) hashes.erase(it);
            }
            r_int(o, n);
        } else if (name == "hlen") {
            if (!arity(2, false)) return true;
            auto it = hashes.find(c[1]);
            r_int(o, it == hashes.end() ? 0 : (long long)it->second.size());
        } else if (name == "eval") {
            if (arity(3, true)) run_script(sha1_hex(c[1]), c, 2, o);
        } else if (name == "evalsha") {
            if (arity(3, true)) run_script(lower(c[1]), c, 2, o);
        } else if (name == "script") {
            if (c.size() == 3 && lower(c[1]) == "load") r_bulk(o, sha1_hex(c[2]));
            else r_error(o, "ERR SCRIPT supports only LOAD here");
        } else if (name == "keys") {
            if (!arity(2, false)) return true;
            std::vector<std::string> ks;
            for (auto &k : all_keys())
                if (glob_match(c[1], k)) ks.push_back(k);
            r_array(o, ks.size());
            for (auto &k : ks) r_bulk(o, k);
        } else if (name == "dbsize") {
            uint64_t nk = 0;
            if (arity(1, false)) {
                if (sk_dbsize(ctx, &nk) != SK_OK) return r_error(o, engine_error()), true;
                r_int(o, (long long)(nk + hashes.size()));
            }
        } else if (name == "scan") {
            // SCAN cursor [MATCH pattern] [COUNT n]: the engine's cursor, then one last step with this process's
            // hashes (cursor kHashStep)
            if (!arity(2, true)) return true;
            const uint64_t kHashStep = 1ull << 62;
            long long cur;
            if (!parse_ll(c[1], cur) || cur < 0) return r_error(o, "ERR invalid cursor"), true;
            std::string pat;
            long long count = 10;
            for (size_t i = 2; i < c.size(); i += 2) {
                std::string opt = lower(c[i]);
                if (i + 1 >= c.size()) return r_error(o, kSyntax), true;
                if (opt == "match") pat = c[i + 1];
                else if (opt == "count") {
                    if (!parse_ll(c[i + 1], count) || count < 1) return r_error(o, kNotInt), true;
                } else return r_error(o, kSyntax), true;
            }
            std::vector<std::string> ks;
            uint64_t next = 0;
            if (uint64_t(cur) != kHashStep) {
                uint32_t n = 0;
                const uint32_t want = uint32_t(std::min<long long>(count, 1 << 20));
                std::vector<uint64_t> off(want + 1);
                std::vector<uint8_t> names(1 << 20);
                std::vector<int32_t> types(want);
                if (sk_scan(ctx, uint64_t(cur), want, &next, &n, off.data(), names.data(), names.size(), types.data()) !=
                    SK_OK)
                    return r_error(o, engine_error()), true;
                for (uint32_t i = 0; i < n; i++)
                    ks.emplace_back(reinterpret_cast<const char *>(names.data()) + off[i], off[i + 1] - off[i]);
                if (!next && !hashes.empty()) next = kHashStep;
            } else {
                for (auto &kv : hashes) ks.push_back(kv.first);
            }
            r_array(o, 2);
            r_bulk(o, std::to_string(next));
            std::vector<std::string> hit;
            for (auto &k : ks)
                if (pat.empty() || glob_match(pat, k)) hit.push_back(k);
            r_array(o, hit.size());
            for (auto &k : hit) r_bulk(o, k);
        } else if (name == "dump") {
            if (!arity(2, false)) return true;
            auto h = hashes.find(c[1]);
            if (h != hashes.end()) return r_bulk(o, sk_rdb::dump_hash(h->second)), true;
            int64_t len = 0;
            if (sk_dump(ctx, k1, c[1].size(), nullptr, 0, &len) != SK_OK) return r_error(o, engine_error()), true;
            if (len < 0) return r_nil(o), true;
            std::string v(size_t(len), '\0');
            if (sk_dump(ctx, k1, c[1].size(), reinterpret_cast<uint8_t *>(&v[0]), v.size(), &len) != SK_OK)
                return r_error(o, engine_error()), true;
            r_bulk(o, v);
        } else if (name == "restore") {
            // RESTORE key ttl payload [REPLACE]; no TTL is served, so ttl must be 0
            if (!arity(4, true)) return true;
            bool replace = false;
            for (size_t i = 4; i < c.size(); i++) {
                if (lower(c[i]) == "replace") replace = true;
                else return r_error(o, kSyntax), true;
            }
            long long ttl;
            if (!parse_ll(c[2], ttl) || ttl < 0) return r_error(o, "ERR Invalid TTL value, must be >= 0"), true;
            if (ttl) return r_error(o, "ERR a TTL is not served by this engine (RESTORE with ttl 0)"), true;
            sk_rdb::Value v;
            std::string why = sk_rdb::load_payload(reinterpret_cast<const uint8_t *>(c[3].data()), c[3].size(), v);
            if (!why.empty()) return r_error(o, "ERR " + why), true;
            if (!replace && type_of(c[1]) != T_NONE) return r_error(o, "BUSYKEY Target key name already exists."), true;
            if (v.type == sk_rdb::kTypeHash) {
                del_one(c[1]);
                hashes[c[1]] = v.fields;
                return r_simple(o, "OK"), true;
            }
            hashes.erase(c[1]);
            int st = sk_restore(ctx, k1, c[1].size(), reinterpret_cast<const uint8_t *>(c[3].data()), c[3].size(), 1);
            st == SK_OK ? r_simple(o, "OK") : r_error(o, engine_error());
        } else if (name == "save" || name == "bgsave") {
            if (!arity(1, false)) return true;
            if (save() != SK_OK) return r_error(o, "ERR " + engine_error()), true;
            name == "save" ? r_simple(o, "OK") : r_simple(o, "Background saving started");
        } else if (name == "debug") {
            // DEBUG RELOAD: save, empty the store, load the file back (what redis' persistence tests run)
            if (c.size() == 2 && lower(c[1]) == "reload") {
                if (save() != SK_OK) return r_error(o, "ERR " + engine_error()), true;
                hashes.clear();
                if (sk_flushall(ctx) != SK_OK || load() != SK_OK) return r_error(o, "ERR " + engine_error()), true;
                r_simple(o, "OK");
            } else {
                r_error(o, "ERR DEBUG supports only RELOAD here");
            }
        } else if (name == "pfadd" || name == "getbit" || name == "setbit") { // batched kinds with a bad arity
            r_error(o, "ERR wrong number of arguments for '" + name + "' command");
        } else {
            r_error(o, "ERR unknown command '" + c[0] + "'");
        }
        return true;
    }

    // run a connection's parsed commands in order; same-kind PFADD / GETBIT /
    // SETBIT runs become one engine batch.  Returns false after QUIT.
    bool run(std::vector<std::vector<std::string>> &cmds, std::string &out) {
        std::vector<std::string> rep(cmds.size());
        bool keep = true;
        size_t i = 0;
        auto kind = [&](size_t j) -> int {
            auto &c = cmds[j];
            if (c.empty()) return 0;
            std::string n = lower(c[0]);
            if (n == "pfadd" && c.size() >= 2) return 1;
            if (n == "getbit" && c.size() == 3) return 2;
            if (n == "setbit" && c.size() == 4) return 3;
            return 0;
        };
        while (i < cmds.size() && keep) {
            int kd = kind(i);
            size_t j = i + 1;
            if (kd) {
                while (j < cmds.size() && kind(j) == kd) j++;
                if (kd == 1) run_pfadd(cmds, i, j, rep);
                else run_bits(cmds, i, j, rep, kd == 3);
            } else if (!cmds[i].empty()) {
                keep = run_one(cmds[i], rep[i]);
            }
            i = j;
        }
        for (size_t r = 0; r < i; r++) out += rep[r];
        return keep;
    }
};

// ------------------------------------------------------------- event loop
struct Conn {
    int fd;
    std::string in, out;
    size_t pos = 0;
    bool closing = false;
};

volatile sig_atomic_t g_stop = 0;
void on_signal(int) { g_stop = 1; }

void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }

bool flush(Conn &c) { // false: the peer is gone
    while (!c.out.empty()) {
        ssize_t w = send(c.fd, c.out.data(), c.out.size(), MSG_NOSIGNAL);
        if (w < 0) return errno == EAGAIN || errno == EWOULDBLOCK;
        c.out.erase(0, size_t(w));
    }
    return true;
}

int selftest() {
    int bad = 0;
    auto check = [&](bool ok, const char *what) {
        if (!ok) fprintf(stderr, "selftest FAILED: %s\n", what), bad++;
    };
    check(sha1_hex("abc") == "a9993e364706816aba3e25717850c26c9cd0d89d", "sha1 abc");
    check(sha1_hex("") == "da39a3ee5e6b4b0d3255bfef95601890afd80709", "sha1 empty");
    check(sha1_hex(std::string(1000, 'a')) == "291e9a6c66994949b57ba5e650361e98fc36b1ba", "sha1 1000 x a");
    std::string buf = "*3\r\n$5\r\nPFADD\r\n$3\r\nfoo\r\n$0\r\n\r\nPING\r\n*2\r\n$3\r\nGET\r\n$2\r\nab";
    size_t pos = 0;
    std::vector<std::string> a;
    std::string err;
    check(parse_command(buf, pos, a, err) == 1 && a.size() == 3 && a[0] == "PFADD" && a[2].empty(), "multibulk");
    check(parse_command(buf, pos, a, err) == 1 && a.size() == 1 && a[0] == "PING", "inline");
    size_t keep = pos;
    check(parse_command(buf, pos, a, err) == 0 && pos == keep, "partial bulk waits");
    buf += "\r\n";
    check(parse_command(buf, pos, a, err) == 1 && a.size() == 2 && a[1] == "ab", "completed bulk");
    std::string bin = std::string("*2\r\n$4\r\nECHO\r\n$4\r\n") + std::string("\r\n\0x", 4) + "\r\n";
    pos = 0;
    check(parse_command(bin, pos, a, err) == 1 && a[1] == std::string("\r\n\0x", 4), "binary-safe bulk");
    std::string badb = "*1\r\n#3\r\nfoo\r\n";
    pos = 0;
    check(parse_command(badb, pos, a, err) == -1 && err == "expected '$', got '#'", "protocol error");
    std::string o;
    r_int(o, -3), r_nil(o), r_bulk(o, "hi"), r_simple(o, "OK"), r_error(o, "ERR x");
    check(o == ":-3\r\n$-1\r\n$2\r\nhi\r\n+OK\r\n-ERR x\r\n", "reply encoding");
    check(glob_match("tenant:*:hll", "tenant:12:hll") && !glob_match("tenant:*:hll", "tenant:12:hl"), "glob *");
    check(glob_match("h?llo", "hello") && glob_match("h[ae]llo", "hallo") && !glob_match("h[^e]llo", "hello"),
          "glob ? and sets");
    check(glob_match("h[a-c]x", "hbx") && glob_match("a\\*b", "a*b") && !glob_match("a\\*b", "axb"), "glob ranges, escapes");
    printf(bad ? "selftest: %d failure(s)\n" : "selftest: OK\n", bad);
    return bad ? 1 : 0;
}

void usage() {
    fprintf(stderr,
            "usage: sk-resp-server [--bind ADDR] [--port P (0 = any)] [--device D] [--redis-major 3|5]\n"
            "                      [--max-bit-offset N] [--hll-capacity N] [--max-batch N] [--hll-exact-strings]\n"
            "                      [--dir D] [--dbfilename F (RDB: SAVE writes it, startup loads it if present)]\n"
            "                      | --selftest\n");
}

} // namespace

int main(int argc, char **argv) {
    std::string bind_addr = "127.0.0.1";
    int port = 6379;
    sk_config cfg = {0, 3, 0, 0, 0};
    bool exact = false;
    std::string dir = ".", dbfile = "dump.rdb";
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto next = [&]() -> const char * {
            if (i + 1 >= argc) usage(), exit(2);
            return argv[++i];
        };
        if (a == "--selftest") return selftest();
        else if (a == "--bind") bind_addr = next();
        else if (a == "--port") port = atoi(next());
        else if (a == "--device") cfg.device = atoi(next());
        else if (a == "--redis-major") cfg.redis_major = atoi(next());
        else if (a == "--max-bit-offset") cfg.max_bit_offset = strtoull(next(), nullptr, 10);
        else if (a == "--hll-capacity") cfg.hll_capacity = strtoull(next(), nullptr, 10);
        else if (a == "--max-batch") cfg.max_batch = strtoull(next(), nullptr, 10);
        else if (a == "--hll-exact-strings") exact = true; // GET of an HLL: redis-server's sparse / dense bytes
        else if (a == "--dir") dir = next();
        else if (a == "--dbfilename") dbfile = next();
        else return usage(), 2;
    }
    Server srv;
    if (cfg.max_bit_offset) srv.max_bit_offset = cfg.max_bit_offset;
    int st = sk_open(&cfg, &srv.ctx);
    if (st != SK_OK) {
        fprintf(stderr, "sk-resp-server: sk_open failed: %s\n", sk_strerror(st));
        return 1;
    }
    if (exact && (st = sk_hll_exact_strings(srv.ctx, 1)) != SK_OK) {
        fprintf(stderr, "sk-resp-server: %s\n", sk_strerror(st));
        return 1;
    }
    srv.rdb_path = dir + "/" + dbfile;
    struct stat sst;
    if (stat(srv.rdb_path.c_str(), &sst) == 0) { // redis-server loads its RDB file at startup
        if (srv.load() != SK_OK) {
            fprintf(stderr, "sk-resp-server: cannot load %s: %s\n", srv.rdb_path.c_str(), sk_last_error(srv.ctx));
            sk_close(srv.ctx);
            return 1;
        }
    }
    int lfd = socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons(uint16_t(port));
    if (inet_pton(AF_INET, bind_addr.c_str(), &sa.sin_addr) != 1 || bind(lfd, (sockaddr *)&sa, sizeof sa) != 0 ||
        listen(lfd, 511) != 0) {
        fprintf(stderr, "sk-resp-server: cannot listen on %s:%d: %s\n", bind_addr.c_str(), port, strerror(errno));
        sk_close(srv.ctx);
        return 1;
    }
    socklen_t sl = sizeof sa;
    getsockname(lfd, (sockaddr *)&sa, &sl);
    set_nonblock(lfd);
    signal(SIGINT, on_signal);
    signal(SIGTERM, on_signal);
    signal(SIGPIPE, SIG_IGN);
    int ep = epoll_create1(0);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.fd = lfd;
    epoll_ctl(ep, EPOLL_CTL_ADD, lfd, &ev);
    printf("ready %s:%d\n", bind_addr.c_str(), ntohs(sa.sin_port));
    fflush(stdout);

    std::unordered_map<int, Conn> conns;
    std::vector<epoll_event> evs(256);
    std::vector<char> rbuf(1 << 20);
    std::vector<std::vector<std::string>> cmds;
    while (!g_stop) {
        int n = epoll_wait(ep, evs.data(), int(evs.size()), 200);
        if (n < 0 && errno != EINTR) break;
        for (int e = 0; e < n; e++) {
            int fd = evs[e].data.fd;
            if (fd == lfd) {
                for (;;) {
                    int cfd = accept(lfd, nullptr, nullptr);
                    if (cfd < 0) break;
                    set_nonblock(cfd);
                    setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
                    epoll_event cev{};
                    cev.events = EPOLLIN | EPOLLRDHUP;
                    cev.data.fd = cfd;
                    epoll_ctl(ep, EPOLL_CTL_ADD, cfd, &cev);
                    conns[cfd] = Conn{cfd, {}, {}, 0, false};
                }
                continue;
            }
            auto it = conns.find(fd);
            if (it == conns.end()) continue;
            Conn &c = it->second;
            bool gone = false;
            if (evs[e].events & EPOLLIN) {
                for (;;) { // drain the socket: the bigger the pipeline slice, the bigger the engine batch
                    ssize_t r = recv(fd, rbuf.data(), rbuf.size(), 0);
                    if (r > 0) c.in.append(rbuf.data(), size_t(r));
                    else if (r == 0) {
                        gone = true;
                        break;
                    } else {
                        if (errno != EAGAIN && errno != EWOULDBLOCK) gone = true;
                        break;
                    }
                }
                cmds.clear();
                std::vector<std::string> args;
                std::string err;
                int pr;
                while ((pr = parse_command(c.in, c.pos, args, err)) == 1) cmds.push_back(std::move(args));
                if (c.pos > (1u << 20) || c.pos == c.in.size()) c.in.erase(0, c.pos), c.pos = 0;
                if (!cmds.empty() && !srv.run(cmds, c.out)) c.closing = true;
                if (pr < 0) {
                    r_error(c.out, "ERR Protocol error: " + err);
                    c.closing = true;
                }
            }
            if (!flush(c)) gone = true;
            if (!gone && c.closing && c.out.empty()) gone = true;
            epoll_event mev{};
            mev.data.fd = fd;
            mev.events = EPOLLIN | EPOLLRDHUP | (c.out.empty() ? 0u : uint32_t(EPOLLOUT));
            if (gone || (evs[e].events & (EPOLLHUP | EPOLLERR))) {
                epoll_ctl(ep, EPOLL_CTL_DEL, fd, nullptr);
                close(fd);
                conns.erase(it);
            } else {
                epoll_ctl(ep, EPOLL_CTL_MOD, fd, &mev);
            }
        }
    }
    for (auto &kv : conns) close(kv.first);
    close(lfd);
    close(ep);
    sk_close(srv.ctx);
    return 0;
}
