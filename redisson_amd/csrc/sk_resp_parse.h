// sk_resp_parse.h -- the RESP2 request parser of the front-end (sk_resp.cpp), host-only so the sanitizer fuzz
// harness (tests/fuzz/fuzz_host.cpp, ASan + UBSan) drives the same code with random and mutated byte streams.
#pragma once
#include <cerrno>
#include <cstdlib>
#include <string>
#include <vector>

namespace sk_resp {

// ------------------------------------------------------------------ RESP
// 1 = one command parsed into args, 0 = need more bytes, -1 = protocol error
inline int parse_command(const std::string &buf, size_t &pos, std::vector<std::string> &args, std::string &err) {
    args.clear();
    if (pos >= buf.size()) return 0;
    if (buf[pos] == '*') {
        size_t nl = buf.find("\r\n", pos);
        if (nl == std::string::npos) return buf.size() - pos > 65536 ? (err = "invalid multibulk length", -1) : 0;
        char *end;
        long long n = strtoll(buf.c_str() + pos + 1, &end, 10);
        if (end != buf.c_str() + nl || n > 1024 * 1024) return err = "invalid multibulk length", -1;
        size_t p = nl + 2;
        std::vector<std::string> out;
        out.reserve(n > 0 ? size_t(n) : 0);
        for (long long i = 0; i < n; i++) {
            if (p >= buf.size()) return 0;
            if (buf[p] != '$') return err = std::string("expected '$', got '") + buf[p] + "'", -1;
            size_t nl2 = buf.find("\r\n", p);
            if (nl2 == std::string::npos) return buf.size() - p > 65536 ? (err = "invalid bulk length", -1) : 0;
            long long len = strtoll(buf.c_str() + p + 1, &end, 10);
            if (end != buf.c_str() + nl2 || len < 0 || len > (512ll << 20)) return err = "invalid bulk length", -1;
            size_t d = nl2 + 2;
            if (d + size_t(len) + 2 > buf.size()) return 0;
            if (buf[d + len] != '\r' || buf[d + len + 1] != '\n') return err = "invalid bulk length", -1;
            out.emplace_back(buf, d, size_t(len));
            p = d + size_t(len) + 2;
        }
        pos = p;
        args.swap(out);
        return 1;
    }
    // inline command: one line, arguments split on blanks
    size_t nl = buf.find('\n', pos);
    if (nl == std::string::npos) return buf.size() - pos > 65536 ? (err = "too big inline request", -1) : 0;
    size_t e = nl;
    if (e > pos && buf[e - 1] == '\r') e--;
    size_t i = pos;
    while (i < e) {
        while (i < e && (buf[i] == ' ' || buf[i] == '\t')) i++;
        size_t s = i;
        while (i < e && buf[i] != ' ' && buf[i] != '\t') i++;
        if (i > s) args.emplace_back(buf, s, i - s);
    }
    pos = nl + 1;
    return 1;
}

inline bool parse_ll(const std::string &s, long long &v) {
    if (s.empty() || s.size() > 20) return false;
    char *end;
    errno = 0;
    v = strtoll(s.c_str(), &end, 10);
    return errno == 0 && end == s.c_str() + s.size();
}

} // namespace sk_resp
