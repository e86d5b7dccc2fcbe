// resp_load.cpp -- pipelined RESP load generator for sk-resp-server (the
// end-to-end path an unmodified Redisson RBatch takes): C connections, each
// sending N commands in pipelined windows of P and reading every reply.
//   PFADD tenant:<t>:hll <Jackson Long>   (C2 shape, tenant uniform)
//   GETBIT bits <offset>                  (C5 shape)
// Prints one JSON line: commands/s over all connections.
#include "../include/redisson_sketch.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

uint64_t splitmix(uint64_t &s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void bulk(std::string &o, const char *p, size_t n) {
    o += '$';
    o += std::to_string(n);
    o += "\r\n";
    o.append(p, n);
    o += "\r\n";
}

// one connection's command stream, cut into windows of P commands
std::vector<std::string> build(const std::string &op, uint64_t n, uint64_t P, uint64_t seed, uint32_t tenants) {
    std::vector<uint64_t> off(n + 1);
    sk_gen_jackson_longs(seed, n, off.data(), nullptr);
    std::vector<uint8_t> bytes(off[n] + 16);
    sk_gen_jackson_longs(seed, n, off.data(), bytes.data());
    std::vector<std::string> wins;
    std::string w;
    uint64_t rs = seed * 7 + 1;
    char key[64];
    for (uint64_t i = 0; i < n; i++) {
        if (op == "pfadd") {
            int kl = snprintf(key, sizeof key, "tenant:%u:hll", uint32_t(splitmix(rs) % tenants));
            w += "*3\r\n$5\r\nPFADD\r\n";
            bulk(w, key, size_t(kl));
            bulk(w, reinterpret_cast<const char *>(bytes.data() + off[i]), size_t(off[i + 1] - off[i]));
        } else {
            std::string o = std::to_string(splitmix(rs) % (1ull << 32));
            w += "*3\r\n$6\r\nGETBIT\r\n$4\r\nbits\r\n";
            bulk(w, o.data(), o.size());
        }
        if ((i + 1) % P == 0 || i + 1 == n) wins.push_back(std::move(w)), w.clear();
    }
    return wins;
}

// read `count` integer replies (":0\r\n" / ":1\r\n"); false on error replies or EOF
bool read_replies(int fd, uint64_t count, std::string &buf) {
    uint64_t got = 0;
    size_t pos = 0;
    char tmp[1 << 16];
    while (got < count) {
        size_t nl;
        while (got < count && (nl = buf.find("\r\n", pos)) != std::string::npos) {
            if (buf[pos] != ':') {
                fprintf(stderr, "unexpected reply: %s\n", buf.substr(pos, nl - pos).c_str());
                return false;
            }
            pos = nl + 2;
            got++;
        }
        if (got == count) break;
        buf.erase(0, pos);
        pos = 0;
        ssize_t r = recv(fd, tmp, sizeof tmp, 0);
        if (r <= 0) return false;
        buf.append(tmp, size_t(r));
    }
    buf.erase(0, pos);
    return true;
}

} // namespace

int main(int argc, char **argv) {
    int port = 6379, conns = 4;
    uint64_t n = 1 << 20, P = 1 << 16;
    uint32_t tenants = 100000;
    std::string op = "pfadd";
    for (int i = 1; i + 1 < argc; i += 2) {
        std::string a = argv[i];
        if (a == "--port") port = atoi(argv[i + 1]);
        else if (a == "--conns") conns = atoi(argv[i + 1]);
        else if (a == "--cmds") n = strtoull(argv[i + 1], nullptr, 10);
        else if (a == "--pipeline") P = strtoull(argv[i + 1], nullptr, 10);
        else if (a == "--tenants") tenants = uint32_t(atoi(argv[i + 1]));
        else if (a == "--op") op = argv[i + 1];
    }
    std::vector<std::vector<std::string>> streams(conns);
    for (int c = 0; c < conns; c++) streams[c] = build(op, n, P, 0x5EED0B00 + c, tenants);
    std::vector<int> fds(conns);
    for (int c = 0; c < conns; c++) {
        fds[c] = socket(AF_INET, SOCK_STREAM, 0);
        int one = 1;
        setsockopt(fds[c], IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        sockaddr_in sa{};
        sa.sin_family = AF_INET;
        sa.sin_port = htons(uint16_t(port));
        inet_pton(AF_INET, "127.0.0.1", &sa.sin_addr);
        if (connect(fds[c], (sockaddr *)&sa, sizeof sa) != 0) {
            perror("connect");
            return 1;
        }
    }
    std::atomic<int> fails{0};
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int c = 0; c < conns; c++)
        th.emplace_back([&, c] {
            std::string rb;
            auto &wins = streams[c];
            for (size_t w = 0; w < wins.size(); w++) {
                const std::string &s = wins[w];
                uint64_t cnt = (w + 1 < wins.size() || n % P == 0) ? P : n % P;
                // writer thread per window so a window larger than the socket buffers cannot deadlock
                std::thread wr([&] {
                    size_t o = 0;
                    while (o < s.size()) {
                        ssize_t k = send(fds[c], s.data() + o, s.size() - o, MSG_NOSIGNAL);
                        if (k <= 0) return;
                        o += size_t(k);
                    }
                });
                bool ok = read_replies(fds[c], cnt, rb);
                wr.join();
                if (!ok) {
                    fails++;
                    return;
                }
            }
        });
    for (auto &t : th) t.join();
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (int fd : fds) close(fd);
    printf("{\"metric\": \"RESP %s commands/sec end to end (pipelined, %d connections)\", \"value\": %.1f, "
           "\"unit\": \"commands/s\", \"commands\": %llu, \"pipeline\": %llu, \"seconds\": %.4f, \"ok\": %s}\n",
           op.c_str(), conns, double(n) * conns / s, (unsigned long long)(n * conns), (unsigned long long)P, s,
           fails ? "false" : "true");
    return fails ? 1 : 0;
}
