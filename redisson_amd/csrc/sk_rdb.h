// sk_rdb.h -- redis-server's persistence formats on the host (SURVEY 5 "Checkpoint / resume", 8(f) rank 1): the
// DUMP / RESTORE payload and the RDB file, as redis-server 3.2 writes them (rdb.c, RDB_VERSION 7; cluster.c
// createDumpPayload / verifyDumpPayload; crc64.c; ziplist.c; lzf_d.c).  The store writes and reads the two value
// types its keys have -- strings (HLLs are strings in Redis: the `HYLL` encoding) and hashes (a Bloom filter's
// "{name}__config", M:RedissonBloomFilter.java:231-256) -- and reads every encoding redis-server 3.2-5.0 produces for
// them: 6/14/32/64-bit lengths, integer- and LZF-encoded strings, plain and ziplist hashes.  Host-only and free of
// HIP: the same code is built into the engine (sk_store.cpp), the RESP front-end (sk_resp.cpp) and the sanitizer
// fuzz harness (tests/fuzz/fuzz_host.cpp).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include <unistd.h>

namespace sk_rdb {

constexpr uint8_t kTypeString = 0, kTypeHash = 4, kTypeHashZiplist = 13;
constexpr uint8_t kOpAux = 0xFA, kOpResizeDb = 0xFB, kOpExpireMs = 0xFC, kOpExpire = 0xFD, kOpSelectDb = 0xFE,
                  kOpEof = 0xFF;
constexpr int kVersionWritten = 7;  // redis 3.2's RDB_VERSION: DUMP payloads and files this store writes
constexpr int kVersionRead = 9;     // newest RDB version whose string / hash encodings are read (redis 5.0)

using Fields = std::vector<std::pair<std::string, std::string>>;

// ---------------------------------------------------------------- CRC64 (crc64.c: Jones polynomial, reflected,
// init 0, no final xor; check value crc64("123456789") = 0xe9c6d914c4b8d9ca), slicing by 8
struct Crc64Tables {
    uint64_t t[8][256];
    Crc64Tables() {
        const uint64_t poly = 0x95ac9329ac4bc9b5ull; // 0xad93d23594c935a9 bit-reversed
        for (int i = 0; i < 256; i++) {
            uint64_t c = uint64_t(i);
            for (int b = 0; b < 8; b++) c = (c >> 1) ^ ((c & 1) ? poly : 0);
            t[0][i] = c;
        }
        for (int i = 0; i < 256; i++)
            for (int s = 1; s < 8; s++) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
    }
};
inline const Crc64Tables &crc_tables() {
    static const Crc64Tables tb;
    return tb;
}
inline uint64_t crc64(uint64_t crc, const uint8_t *p, size_t n) {
    const Crc64Tables &T = crc_tables();
    while (n >= 8) {
        uint64_t w;
        std::memcpy(&w, p, 8); // little-endian host
        w ^= crc;
        crc = T.t[7][w & 0xff] ^ T.t[6][(w >> 8) & 0xff] ^ T.t[5][(w >> 16) & 0xff] ^ T.t[4][(w >> 24) & 0xff] ^
              T.t[3][(w >> 32) & 0xff] ^ T.t[2][(w >> 40) & 0xff] ^ T.t[1][(w >> 48) & 0xff] ^ T.t[0][w >> 56];
        p += 8;
        n -= 8;
    }
    while (n--) crc = T.t[0][(crc ^ *p++) & 0xff] ^ (crc >> 8);
    return crc;
}

// ---------------------------------------------------------------- encoders (rdbSaveLen / rdbSaveRawString)
inline void put_len(std::string &o, uint64_t len) {
    if (len < 64) {
        o.push_back(char(len));
    } else if (len < 16384) {
        o.push_back(char(0x40 | (len >> 8)));
        o.push_back(char(len & 0xff));
    } else if (len <= 0xffffffffull) {
        o.push_back(char(0x80));
        for (int s = 24; s >= 0; s -= 8) o.push_back(char((len >> s) & 0xff));
    } else { // RDB_64BITLEN (redis >= 4 reads it; 3.2 strings never reach 4 GiB)
        o.push_back(char(0x81));
        for (int s = 56; s >= 0; s -= 8) o.push_back(char((len >> s) & 0xff));
    }
}
inline void put_string(std::string &o, const void *p, uint64_t n) {
    put_len(o, n);
    o.append(static_cast<const char *>(p), n);
}
inline void put_string(std::string &o, const std::string &s) { put_string(o, s.data(), s.size()); }

// DUMP payload: type, value, 2-byte RDB version, CRC64 of everything before (createDumpPayload)
inline void finish_payload(std::string &o) {
    o.push_back(char(kVersionWritten & 0xff));
    o.push_back(char((kVersionWritten >> 8) & 0xff));
    const uint64_t crc = crc64(0, reinterpret_cast<const uint8_t *>(o.data()), o.size());
    for (int i = 0; i < 8; i++) o.push_back(char((crc >> (8 * i)) & 0xff));
}
inline std::string dump_string(const void *p, uint64_t n) {
    std::string o;
    o.reserve(n + 16);
    o.push_back(char(kTypeString));
    put_string(o, p, n);
    finish_payload(o);
    return o;
}
inline std::string dump_hash(const Fields &f) {
    std::string o(1, char(kTypeHash));
    put_len(o, f.size());
    for (auto &kv : f) put_string(o, kv.first), put_string(o, kv.second);
    finish_payload(o);
    return o;
}

// ---------------------------------------------------------------- decoder (rdbLoadLen / rdbGenericLoadStringObject)
struct Reader {
    const uint8_t *p, *end;
    bool ok = true;
    uint8_t u8() {
        if (p >= end) return ok = false, 0;
        return *p++;
    }
    bool take(uint64_t n, const uint8_t **out) {
        if (uint64_t(end - p) < n) return ok = false;
        *out = p;
        p += n;
        return true;
    }
    // length or special encoding (enc = true: the low 6 bits name it)
    uint64_t len(bool *enc) {
        *enc = false;
        const uint8_t b = u8();
        switch (b >> 6) {
        case 0: return b & 0x3f;
        case 1: return (uint64_t(b & 0x3f) << 8) | u8();
        case 3: *enc = true; return b & 0x3f;
        default:
            if (b == 0x80 || b == 0x81) {
                uint64_t v = 0;
                for (int i = 0; i < (b == 0x80 ? 4 : 8); i++) v = (v << 8) | u8();
                return v;
            }
            ok = false;
            return 0;
        }
    }
    uint64_t plain_len() {
        bool enc;
        uint64_t v = len(&enc);
        if (enc) ok = false;
        return v;
    }
};

// lzf_decompress (liblzf lzf_d.c): literal runs 000LLLLL + L+1 bytes; back references LLLooooo [LLL == 7: + a
// length byte] + an offset byte: copy len + 2 bytes from (out - offset - 1), overlapping allowed
inline bool lzf_decompress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_len) {
    const uint8_t *ip = in, *ie = in + n;
    uint8_t *op = out, *oe = out + out_len;
    while (ip < ie) {
        uint32_t ctrl = *ip++;
        if (ctrl < 32) {
            uint32_t l = ctrl + 1;
            if (uint64_t(oe - op) < l || uint64_t(ie - ip) < l) return false;
            std::memcpy(op, ip, l);
            op += l, ip += l;
        } else {
            uint32_t l = ctrl >> 5;
            uint64_t back = uint64_t(ctrl & 0x1f) << 8;
            if (l == 7) {
                if (ip >= ie) return false;
                l += *ip++;
            }
            if (ip >= ie) return false;
            back += *ip++;
            l += 2;
            if (back + 1 > uint64_t(op - out) || uint64_t(oe - op) < l) return false;
            const uint8_t *ref = op - back - 1;
            for (uint32_t i = 0; i < l; i++) *op++ = *ref++; // byte by byte: the reference may overlap the output
        }
    }
    return op == oe;
}

// a string object: raw, integer-encoded (INT8 / INT16 / INT32, written back as decimal) or LZF-compressed
inline bool load_string(Reader &r, std::string &out) {
    bool enc;
    const uint64_t l = r.len(&enc);
    if (!r.ok) return false;
    if (enc) {
        int64_t v;
        if (l == 0) v = int8_t(r.u8());
        else if (l == 1) {
            uint16_t x = uint16_t(r.u8());
            x |= uint16_t(r.u8()) << 8;
            v = int16_t(x);
        } else if (l == 2) {
            uint32_t x = 0;
            for (int i = 0; i < 4; i++) x |= uint32_t(r.u8()) << (8 * i);
            v = int32_t(x);
        } else if (l == 3) {
            const uint64_t clen = r.plain_len(), ulen = r.plain_len();
            const uint8_t *c;
            if (!r.ok || !r.take(clen, &c)) return false;
            // bound the allocation by what clen can decompress to: the longest LZF back-reference (3 bytes) yields
            // 264 bytes, literal runs never expand, so ulen <= 88 * clen; and no string past 4 GiB (the engine's
            // largest bit string is 2 GiB at max_bit_offset 2^34)
            if (ulen > clen * 88 || ulen > (uint64_t(1) << 32)) return r.ok = false;
            out.assign(ulen, '\0');
            return lzf_decompress(c, clen, reinterpret_cast<uint8_t *>(&out[0]), ulen) || (r.ok = false);
        } else {
            return r.ok = false;
        }
        out = std::to_string(v);
        return r.ok;
    }
    const uint8_t *b;
    if (!r.take(l, &b)) return false;
    out.assign(reinterpret_cast<const char *>(b), l);
    return true;
}

// ziplist (ziplist.c) of a small hash: zlbytes u32, zltail u32, zllen u16, entries [prevlen][encoding][data], 0xFF;
// entries alternate field, value; integer entries are returned as decimal strings
inline bool ziplist_entries(const std::string &zl, std::vector<std::string> &out) {
    const uint8_t *p = reinterpret_cast<const uint8_t *>(zl.data()), *e = p + zl.size();
    if (zl.size() < 11) return false;
    uint32_t zlbytes;
    std::memcpy(&zlbytes, p, 4);
    if (zlbytes != zl.size() || e[-1] != 0xFF) return false;
    p += 10;
    while (p < e && *p != 0xFF) {
        if (*p == 0xFE) p += 5; // prevlen: 0xFE + u32
        else p += 1;
        if (p >= e) return false;
        const uint8_t enc = *p;
        int64_t iv = 0;
        bool is_int = true;
        uint64_t slen = 0;
        switch (enc >> 6) {
        case 0: slen = enc & 0x3f, p += 1, is_int = false; break;
        case 1:
            if (e - p < 2) return false;
            slen = (uint64_t(enc & 0x3f) << 8) | p[1], p += 2, is_int = false;
            break;
        case 2:
            if (e - p < 5) return false;
            slen = (uint64_t(p[1]) << 24) | (uint64_t(p[2]) << 16) | (uint64_t(p[3]) << 8) | p[4], p += 5;
            is_int = false;
            break;
        default: {
            int nb;
            if (enc == 0xC0) nb = 2;
            else if (enc == 0xD0) nb = 4;
            else if (enc == 0xE0) nb = 8;
            else if (enc == 0xF0) nb = 3;
            else if (enc == 0xFE) nb = 1;
            else if (enc >= 0xF1 && enc <= 0xFD) nb = 0, iv = int64_t(enc & 0x0f) - 1; // immediate 0..12
            else return false;
            p += 1;
            if (e - p < nb) return false;
            if (nb) {
                uint64_t x = 0;
                for (int i = 0; i < nb; i++) x |= uint64_t(p[i]) << (8 * i);
                const int sh = 64 - 8 * nb; // sign-extend nb bytes
                iv = int64_t(x << sh) >> sh;
                p += nb;
            }
        }
        }
        if (is_int) {
            out.push_back(std::to_string(iv));
        } else {
            if (uint64_t(e - p) < slen) return false;
            out.emplace_back(reinterpret_cast<const char *>(p), slen);
            p += slen;
        }
    }
    return p < e && *p == 0xFF && p + 1 == e;
}

// one value of a type the store keeps: a string (bytes) or a hash (fields, in stored order)
struct Value {
    uint8_t type = kTypeString; // kTypeString or kTypeHash after load_value
    std::string bytes;
    Fields fields;
};
// returns "" on success, else the reason
inline std::string load_value(Reader &r, uint8_t type, Value &v) {
    if (type == kTypeString) {
        v.type = kTypeString;
        return load_string(r, v.bytes) ? "" : "bad string encoding";
    }
    if (type == kTypeHash) {
        v.type = kTypeHash;
        const uint64_t n = r.plain_len();
        if (!r.ok) return "bad hash length";
        for (uint64_t i = 0; i < n; i++) {
            std::string f, x;
            if (!load_string(r, f) || !load_string(r, x)) return "bad hash field";
            v.fields.emplace_back(std::move(f), std::move(x));
        }
        return "";
    }
    if (type == kTypeHashZiplist) {
        v.type = kTypeHash;
        std::string zl;
        std::vector<std::string> ent;
        if (!load_string(r, zl) || !ziplist_entries(zl, ent) || ent.size() % 2) return "bad ziplist hash";
        for (size_t i = 0; i < ent.size(); i += 2) v.fields.emplace_back(std::move(ent[i]), std::move(ent[i + 1]));
        return "";
    }
    return "unsupported RDB value type " + std::to_string(type) +
           " (the sketch store keeps strings -- HLLs, bit strings -- and Bloom filter config hashes)";
}

// verifyDumpPayload + the value: "" on success
inline std::string load_payload(const uint8_t *p, uint64_t n, Value &v) {
    if (n < 10) return "DUMP payload version or checksum are wrong";
    const int ver = p[n - 10] | (p[n - 9] << 8);
    uint64_t crc = 0;
    for (int i = 0; i < 8; i++) crc |= uint64_t(p[n - 8 + i]) << (8 * i);
    if (ver > kVersionRead || crc64(0, p, n - 8) != crc) return "DUMP payload version or checksum are wrong";
    Reader r{p + 1, p + n - 10};
    std::string why = load_value(r, p[0], v);
    if (why.empty() && (!r.ok || r.p != r.end)) why = "Bad data format";
    return why;
}

// ---------------------------------------------------------------- RDB file writer: streamed, CRC kept running
// Written to "<path>.tmp-<pid>", flushed to disk, then renamed over <path> (as redis-server's rdbSave does), so a
// failed or interrupted SAVE never leaves a torn file at <path>; the temporary is removed on failure.
struct FileWriter {
    FILE *f = nullptr;
    uint64_t crc = 0;
    bool ok = true;
    std::string buf, final_path, tmp_path;
    bool open(const char *path) {
        final_path = path;
        tmp_path = final_path + ".tmp-" + std::to_string(long(getpid()));
        f = std::fopen(tmp_path.c_str(), "wb");
        if (!f) return ok = false;
        buf.reserve(1 << 20);
        put(reinterpret_cast<const uint8_t *>("REDIS0007"), 9);
        const uint8_t sel[2] = {kOpSelectDb, 0};
        put(sel, 2);
        return true;
    }
    void flush_buf() {
        if (buf.empty()) return;
        crc = crc64(crc, reinterpret_cast<const uint8_t *>(buf.data()), buf.size());
        if (std::fwrite(buf.data(), 1, buf.size(), f) != buf.size()) ok = false;
        buf.clear();
    }
    void put(const uint8_t *p, uint64_t n) {
        if (n >= (1u << 20)) { // large values bypass the buffer
            flush_buf();
            crc = crc64(crc, p, n);
            if (std::fwrite(p, 1, n, f) != n) ok = false;
            return;
        }
        buf.append(reinterpret_cast<const char *>(p), n);
        if (buf.size() >= (1u << 20)) flush_buf();
    }
    void put(const std::string &s) { put(reinterpret_cast<const uint8_t *>(s.data()), s.size()); }
    // a record: value type, key, then the value (the caller writes it: `value_head` and the bytes that follow)
    void record_head(uint8_t type, const std::string &key) {
        std::string h(1, char(type));
        put_string(h, key);
        put(h);
    }
    bool close() { // EOF + CRC64 (little-endian) of everything before
        const uint8_t eof = kOpEof;
        put(&eof, 1);
        flush_buf();
        uint8_t c8[8];
        for (int i = 0; i < 8; i++) c8[i] = uint8_t(crc >> (8 * i));
        if (std::fwrite(c8, 1, 8, f) != 8) ok = false;
        if (std::fflush(f) != 0 || fsync(fileno(f)) != 0) ok = false;
        if (std::fclose(f) != 0) ok = false;
        f = nullptr;
        if (ok && std::rename(tmp_path.c_str(), final_path.c_str()) != 0) ok = false;
        if (!ok) std::remove(tmp_path.c_str());
        return ok;
    }
    ~FileWriter() { // abandoned (an error before close): no file at the path, no temporary left
        if (f) {
            std::fclose(f);
            std::remove(tmp_path.c_str());
        }
    }
};

// ---------------------------------------------------------------- RDB file reader (rdbLoad): the whole image in
// memory; calls on_record(key, type, Reader positioned at the value) for each key, skipping aux fields, RESIZEDB
// and expire times (the store serves no TTL).  "" on success.
template <class F> std::string parse_rdb(const uint8_t *img, uint64_t n, F &&on_record) {
    if (n < 9 || std::memcmp(img, "REDIS", 5) != 0) return "not an RDB file (bad signature)";
    int ver = 0;
    for (int i = 5; i < 9; i++) {
        if (img[i] < '0' || img[i] > '9') return "not an RDB file (bad version)";
        ver = ver * 10 + (img[i] - '0');
    }
    if (ver < 1 || ver > kVersionRead) return "unsupported RDB version " + std::to_string(ver);
    Reader r{img + 9, img + n};
    for (;;) {
        uint8_t t = r.u8();
        if (!r.ok) return "truncated RDB file";
        if (t == kOpEof) break;
        if (t == kOpSelectDb) {
            if (r.plain_len() != 0) return "only database 0 is served";
            continue;
        }
        if (t == kOpResizeDb) {
            r.plain_len(), r.plain_len();
            continue;
        }
        if (t == kOpAux) {
            std::string a, b;
            if (!load_string(r, a) || !load_string(r, b)) return "bad aux field";
            continue;
        }
        if (t == kOpExpireMs || t == kOpExpire) {
            const uint8_t *skip;
            if (!r.take(t == kOpExpireMs ? 8 : 4, &skip)) return "truncated RDB file";
            continue;
        }
        std::string key;
        if (!load_string(r, key)) return "bad key";
        std::string why = on_record(key, t, r);
        if (!why.empty()) return why;
        if (!r.ok) return "truncated RDB file";
    }
    if (ver >= 5) { // CRC64 of everything before it; 0 = written with rdbchecksum no
        const uint8_t *c8;
        if (!r.take(8, &c8)) return "truncated RDB file (checksum)";
        uint64_t crc = 0;
        for (int i = 0; i < 8; i++) crc |= uint64_t(c8[i]) << (8 * i);
        if (crc && crc != crc64(0, img, uint64_t(c8 - img))) return "RDB file checksum mismatch";
    }
    return "";
}

// ---------------------------------------------------------------- Redisson's Bloom config hash
// BigDecimal.valueOf(d).toPlainString() (M:RedissonBloomFilter.java:240): Double.toString's digits (the shortest
// decimal that reads back as d, at least one digit after the point; scientific below 1e-3 and from 1e7) written
// without an exponent.  So 0.03 -> "0.03", 1.0E-6 -> "0.0000010", 1.0E7 -> "10000000" (BigDecimal keeps the
// mantissa's digits: "1.0E-6" has unscaled value 10 at scale 7).  Shortest digits as JDK >= 19 prints them
// (older JDKs could print extra digits for a few values: parity unpinned there).
inline std::string java_plain_double(double d) {
    if (d == 0) return "0.0";
    char buf[40];
    int prec = 1;
    for (; prec <= 17; prec++) { // shortest round trip
        std::snprintf(buf, sizeof buf, "%.*e", prec - 1, d);
        if (std::strtod(buf, nullptr) == d) break;
    }
    // buf = [-]D.DDDe[+-]XX
    std::string s(buf);
    const bool neg = s[0] == '-';
    if (neg) s.erase(0, 1);
    const size_t epos = s.find('e');
    const int exp10 = std::atoi(s.c_str() + epos + 1);
    std::string digits;
    for (size_t i = 0; i < epos; i++)
        if (s[i] != '.') digits.push_back(s[i]);
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    std::string out;
    if (exp10 >= -3 && exp10 < 7) { // Double.toString's plain range: digits with the point placed, >= 1 decimal
        if (exp10 >= 0) {
            std::string ip = digits.substr(0, std::min<size_t>(digits.size(), size_t(exp10) + 1));
            while (ip.size() < size_t(exp10) + 1) ip.push_back('0');
            std::string fp = digits.size() > size_t(exp10) + 1 ? digits.substr(size_t(exp10) + 1) : "0";
            out = ip + "." + fp;
        } else {
            out = "0." + std::string(size_t(-exp10 - 1), '0') + digits;
        }
    } else { // "D.DDDE[-]X": BigDecimal keeps the mantissa's digits (at least two: "1.0")
        std::string m = digits.size() == 1 ? digits + "0" : digits; // unscaled value, one digit before the point
        const int scale = int(m.size()) - 1 - exp10;                  // BigDecimal scale
        if (scale <= 0) out = m + std::string(size_t(-scale), '0');    // an integer: no point (toPlainString)
        else if (size_t(scale) >= m.size()) out = "0." + std::string(size_t(scale) - m.size(), '0') + m;
        else out = m.substr(0, m.size() - size_t(scale)) + "." + m.substr(m.size() - size_t(scale));
    }
    return neg ? "-" + out : out;
}

// the HMSET of tryInit, in its field order (M:RedissonBloomFilter.java:238-240)
inline Fields bloom_config_fields(int64_t size, int32_t k, int64_t expected, double fpp) {
    return {{"size", std::to_string(size)},
            {"hashIterations", std::to_string(k)},
            {"expectedInsertions", std::to_string(expected)},
            {"falseProbability", java_plain_double(fpp)}};
}

} // namespace sk_rdb
