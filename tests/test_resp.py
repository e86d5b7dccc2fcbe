"""RESP front-end (redisson_amd/sk-resp-server): the wire commands Redisson's
HLL / BitSet / Bloom objects send, pipelined as RBatch sends them, answered as
redis-server answers them, with the sketch state checked against the oracle.

The scripts Redisson EVALs on this path are addressed by their SHA1
(tools/script_digests.py derives them from the reference's Java literals; the
server recognises EVAL bodies by the same digest)."""
import os
import socket
import subprocess
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SERVER = os.path.join(ROOT, "redisson_amd", "sk-resp-server")
SHA_BLOOM_CHECK = "e678c622b160a7f36fe9f26aecd0c1a5992e5b0c"
SHA_BLOOM_INIT = "bae33949534234b07cb5de743c296685dbafadff"
SHA_BITSET_LENGTH = "a80ae5bc82f0ec7382e36b49cdc6bc589a9a80b3"
CONFIG_CHANGED = "Bloom filter config has been changed"


class RespError(Exception):
    pass


class Client:
    """Minimal pipelining RESP2 client."""

    def __init__(self, port):
        self.s = socket.create_connection(("127.0.0.1", port), timeout=60)
        self.buf = b""

    def close(self):
        self.s.close()

    @staticmethod
    def encode(cmd):
        parts = [c if isinstance(c, bytes) else str(c).encode() for c in cmd]
        return b"*%d\r\n" % len(parts) + b"".join(b"$%d\r\n%s\r\n" % (len(p), p) for p in parts)

    def _line(self):
        while b"\r\n" not in self.buf:
            self._fill()
        i = self.buf.index(b"\r\n")
        line, self.buf = self.buf[:i], self.buf[i + 2:]
        return line

    def _fill(self):
        d = self.s.recv(1 << 20)
        if not d:
            raise ConnectionError("server closed the connection")
        self.buf += d

    def _reply(self):
        line = self._line()
        t, rest = line[:1], line[1:]
        if t == b"+":
            return rest.decode()
        if t == b"-":
            return RespError(rest.decode())
        if t == b":":
            return int(rest)
        if t == b"$":
            n = int(rest)
            if n < 0:
                return None
            while len(self.buf) < n + 2:
                self._fill()
            v, self.buf = self.buf[:n], self.buf[n + 2:]
            return v
        if t == b"*":
            return [self._reply() for _ in range(int(rest))]
        raise AssertionError("bad reply type %r" % line)

    def pipeline(self, cmds):
        self.s.sendall(b"".join(self.encode(c) for c in cmds))
        return [self._reply() for _ in cmds]

    def call(self, *cmd):
        r = self.pipeline([cmd])[0]
        if isinstance(r, RespError):
            raise r
        return r


def test_server_selftest():
    """Parser, reply encoding and SHA1 (script digests) without a device."""
    r = subprocess.run([SERVER, "--selftest"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "selftest: OK" in r.stdout


def test_server_fails_loudly_without_device():
    from redisson_amd import device_count

    if device_count() > 0:
        pytest.skip("a GPU is visible")
    r = subprocess.run([SERVER, "--port", "0"], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "sk_open failed" in r.stderr


def _start(*extra):
    p = subprocess.Popen([SERVER, "--port", "0", "--device", "0", *extra], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    if not line.startswith("ready"):
        p.kill()
        raise RuntimeError("server did not start: %s %s" % (line, p.stderr.read()))
    return p, int(line.split(":")[-1])


def _stop(p):
    p.terminate()
    try:
        p.wait(30)
    except subprocess.TimeoutExpired:
        p.kill()


@pytest.fixture(scope="module")
def server(tmp_path_factory):
    # its own --dir: a dump.rdb in the working directory is never loaded (redis-server loads it at startup)
    p, port = _start("--dir", str(tmp_path_factory.mktemp("resp")))
    yield port
    _stop(p)


@pytest.fixture()
def cli(server):
    c = Client(server)
    c.call("FLUSHALL")
    yield c
    c.close()


def _jlongs(seed, n):
    from redisson_amd import gen_jackson_longs

    off, buf = gen_jackson_longs(seed, n)
    return [buf[off[i]:off[i + 1]].tobytes() for i in range(n)]


@pytest.mark.gpu
def test_resp_hll(cli, O):
    # T:RedissonHyperLogLogTest.java:10-38 on the wire (Integer elements encode as "1", "2", ...)
    assert cli.pipeline([["PFADD", "hll", "1", "2", "3"], ["PFCOUNT", "hll"]]) == [1, 3]
    assert cli.pipeline([["PFADD", "h1", "foo1"], ["PFADD", "h1", "foo1"], ["PFADD", "h2", "bar"]]) == [1, 0, 1]
    # an RBatch of single-element PFADDs over many keys -> one engine batch, exact replies
    els = _jlongs(0x5EED0600, 20000)
    els += els[:3000]                                    # repeats reply 0
    rng = np.random.default_rng(6)
    keys = [b"r:%d" % rng.integers(0, 50) for _ in els]
    got = cli.pipeline([["PFADD", k, e] for k, e in zip(keys, els)])
    ref = O.HLLStore()
    assert got == [int(x) for x in ref.pfadd(keys, [[e] for e in els])]
    names = sorted(set(keys))
    assert cli.pipeline([["PFCOUNT", k] for k in names]) == [ref.count([k]) for k in names]
    assert cli.call("PFCOUNT", *names) == ref.count(names)
    assert cli.call("PFMERGE", "r:dest", *names) == "OK"
    ref.merge(b"r:dest", names)
    assert cli.call("PFCOUNT", "r:dest") == ref.count([b"r:dest"])
    # GET returns the Redis dense string (cache marked invalid)
    v = cli.call("GET", "r:dest")
    assert v[:4] == b"HYLL" and v[4] == 0 and v[15] & 0x80 and v[16:] == O.dense_pack(ref.regs[b"r:dest"])
    assert cli.call("STRLEN", "r:dest") == 16 + 12288
    assert cli.call("TYPE", "r:dest") == "string" and cli.call("EXISTS", "r:dest", "nope", "r:dest") == 2


@pytest.mark.gpu
def test_resp_bloom(cli, O):
    """RedissonBloomFilter's wire sequence (M:RedissonBloomFilter.java:80-199, 223-252):
    tryInit = check script + HMSET, add = check + k SETBITs, contains = check +
    k GETBITs, count = HGETALL + BITCOUNT; every pipeline as the reference sends it."""
    name, cfg = "bf", "{bf}__config"
    size = O.bloom_optimal_bits(100, 0.03)
    k = O.bloom_optimal_k(100, size)
    init = [["EVALSHA", SHA_BLOOM_INIT, 1, cfg, size, k],
            ["HMSET", cfg, "size", size, "hashIterations", k, "expectedInsertions", 100, "falseProbability", "0.03"]]
    assert cli.pipeline(init) == [None, "OK"]
    # a second tryInit: the assert fails, the HMSET still runs (Q6)
    r = cli.pipeline([["EVALSHA", SHA_BLOOM_INIT, 1, cfg, size, k],
                      ["HMSET", cfg, "size", size, "hashIterations", k, "expectedInsertions", 101,
                       "falseProbability", "0.03"]])
    assert isinstance(r[0], RespError) and CONFIG_CHANGED in str(r[0]) and r[1] == "OK"
    cfgmap = cli.call("HGETALL", cfg)
    assert dict(zip(cfgmap[::2], cfgmap[1::2]))[b"expectedInsertions"] == b"101"
    bits = O.BitString()
    for obj in [b'"123"', b'"hflgs;jl;ao1-32471320o31803-24"', b'"123"']:
        idx = O.bloom_indexes(obj, k, size)
        contains = cli.pipeline([["EVALSHA", SHA_BLOOM_CHECK, 1, cfg, size, k]] + [["GETBIT", name, i] for i in idx])
        assert contains[0] is None
        assert all(contains[1:-1]) == bits.bloom_contains(size, k, [obj])[0]
        added = cli.pipeline([["EVALSHA", SHA_BLOOM_CHECK, 1, cfg, size, k]] + [["SETBIT", name, i, 1] for i in idx])
        want_old = [bits.setbit(i, 1) for i in idx]
        assert added[1:] == want_old
    assert cli.call("GET", name) == bits.bytes()
    cnt = cli.pipeline([["HGETALL", cfg], ["BITCOUNT", name]])
    assert cnt[1] == bits.bitcount()
    # a changed config fails the check (the Java retry loop matches the message)
    r = cli.pipeline([["EVALSHA", SHA_BLOOM_CHECK, 1, cfg, size + 1, k], ["GETBIT", name, 0]])
    assert isinstance(r[0], RespError) and CONFIG_CHANGED in str(r[0]) and r[1] in (0, 1)
    assert cli.call("DEL", name, cfg) == 2 and cli.call("EXISTS", name, cfg) == 0


@pytest.mark.gpu
def test_resp_bitset(cli, O):
    ref = O.BitString()
    rng = np.random.default_rng(8)
    offs = [int(x) for x in rng.integers(0, 50000, 3000)]
    vals = [int(x) for x in rng.integers(0, 2, 3000)]
    got = cli.pipeline([["SETBIT", "bs", o, v] for o, v in zip(offs, vals)])
    assert got == [ref.setbit(o, v) for o, v in zip(offs, vals)]
    probe = [int(x) for x in rng.integers(0, 60000, 2000)]
    assert cli.pipeline([["GETBIT", "bs", o] for o in probe]) == [ref.getbit(o) for o in probe]
    assert cli.call("BITCOUNT", "bs") == ref.bitcount()
    assert cli.call("STRLEN", "bs") == len(ref.bytes())
    assert cli.call("GET", "bs") == ref.bytes()
    # RBitSet.length() (Lua: BITPOS key 1 -1 looks at the LAST byte only): the
    # highest set bit + 1 when the last byte has one, else GETBIT 0 / GETBIT -1
    data = ref.bytes()
    r = cli.pipeline([["EVALSHA", SHA_BITSET_LENGTH, 1, "bs"]])[0]
    if data[-1]:
        assert r == 8 * (len(data) - 1) + 8 - ((data[-1] & -data[-1]).bit_length() - 1)
    elif data[0] & 0x80:
        assert r == 1
    else:
        assert "bit offset" in str(r)
    cli.call("SETBIT", "bs", 8 * len(data) - 3, 1)
    ref.setbit(8 * len(data) - 3, 1)
    assert cli.call("EVALSHA", SHA_BITSET_LENGTH, 1, "bs") == 8 * len(data) - 2
    # BITOP AND/OR/XOR/NOT against the oracle
    assert cli.call("SET", "b2", b"\x0f\xf0\xaa") == "OK"
    for op in ["AND", "OR", "XOR"]:
        n = cli.call("BITOP", op, "dst", "bs", "b2")
        want = O.bitop(op, [ref.bytes(), b"\x0f\xf0\xaa"])
        assert n == len(want) and cli.call("GET", "dst") == want
    assert cli.call("BITOP", "NOT", "dst", "b2") == 3 and cli.call("GET", "dst") == b"\xf0\x0f\x55"
    # per-command errors inside one pipeline leave the other commands' replies intact
    r = cli.pipeline([["SETBIT", "bs", -1, 1], ["SETBIT", "bs", 5, 2], ["GETBIT", "bs", "x"], ["SETBIT", "bs", 7, 1],
                      ["PFADD", "bs", "a"], ["GETBIT", "nokey", 10], ["BITOP", "NOT", "d", "a", "b"],
                      ["FOO"], ["GETBIT", "bs"], ["HSET", "bs", "f", "v"]])
    assert "bit offset" in str(r[0]) and "bit is not an integer" in str(r[1]) and "bit offset" in str(r[2])
    assert r[3] == ref.setbit(7, 1)
    assert "HyperLogLog" in str(r[4]) and r[5] == 0 and "BITOP NOT" in str(r[6])
    assert "unknown command" in str(r[7]) and "wrong number of arguments" in str(r[8])
    assert str(r[9]).startswith("WRONGTYPE")
    assert cli.call("GET", "bs") == ref.bytes()


@pytest.mark.gpu
def test_resp_protocol(server, cli):
    # inline commands, byte-at-a-time delivery, binary-safe values, pipelined order
    raw = socket.create_connection(("127.0.0.1", server), timeout=30)
    raw.sendall(b"PING\r\n")
    assert raw.recv(100) == b"+PONG\r\n"
    msg = Client.encode(["ECHO", b"a\r\nb\x00c"])
    for i in range(len(msg)):
        raw.sendall(msg[i:i + 1])
        time.sleep(0.001)
    exp = b"$6\r\na\r\nb\x00c\r\n"
    got = b""
    while len(got) < len(exp):
        got += raw.recv(100)
    assert got == exp
    raw.sendall(b"*1\r\n#4\r\n")
    assert raw.recv(200).startswith(b"-ERR Protocol error")
    raw.close()
    r = cli.pipeline([["PFADD", "o", "a"], ["PFCOUNT", "o"], ["PFADD", "o", "b"], ["PFCOUNT", "o"],
                      ["SELECT", 0], ["SELECT", 1]])
    assert r[:5] == [1, 1, 1, 2, "OK"] and "invalid DB index" in str(r[5])
    assert cli.call("QUIT") == "OK"
    assert cli.s.recv(10) == b""


@pytest.mark.gpu
def test_resp_persistence(tmp_path, O):
    """SURVEY 8(f) rank 1 / VERDICT r4 item 6 on the wire: KEYS / SCAN (MATCH, COUNT) / DUMP / RESTORE / SAVE, a
    restart that loads the file (redis-server loads its dump.rdb at startup), and DEBUG RELOAD -- the HLLs, the
    Bloom filter's bit array and "{name}__config" hash, and a bitset come back identical."""
    from tests.test_gpu_persist import parse_payload

    p, port = _start("--dir", str(tmp_path), "--dbfilename", "snap.rdb")
    c = Client(port)
    try:
        elems = _jlongs(0x5EED7100, 4000)
        c.pipeline([["PFADD", "t:%d" % (i % 9), e] for i, e in enumerate(elems)])
        c.pipeline([["SETBIT", "bs", str(i * 131), "1"] for i in range(500)])
        assert c.call("EVALSHA", SHA_BLOOM_INIT, 1, "{bf}__config", "729", "5") is None
        c.call("HMSET", "{bf}__config", "size", "729", "hashIterations", "5", "expectedInsertions", "100",
               "falseProbability", "0.03")
        c.pipeline([["SETBIT", "bf", str(i * 7 % 729), "1"] for i in range(300)])
        keys = {b"t:%d" % i for i in range(9)} | {b"bs", b"bf", b"{bf}__config"}
        assert set(c.call("KEYS", "*")) == keys
        assert set(c.call("KEYS", "t:*")) == {b"t:%d" % i for i in range(9)}
        assert c.call("DBSIZE") == len(keys)
        seen, cur = [], b"0"
        while True:
            cur, part = c.call("SCAN", cur, "COUNT", "2")
            seen += part
            if cur == b"0":
                break
        assert sorted(seen) == sorted(keys)
        cur, part = c.call("SCAN", "0", "MATCH", "t:[0-3]", "COUNT", "1000")
        assert set(part) <= {b"t:0", b"t:1", b"t:2", b"t:3"}
        before = {k: c.call("DUMP", k) for k in keys}
        t, f = parse_payload(before[b"{bf}__config"])
        assert t == 4 and f[0] == (b"size", b"729")
        gets = {k: c.call("GET", k) for k in keys if not k.startswith(b"{")}
        counts = c.pipeline([["PFCOUNT", "t:%d" % i] for i in range(9)])
        assert c.call("RESTORE", "copy", "0", before[b"t:4"]) == "OK"
        assert c.call("GET", "copy") == gets[b"t:4"]
        assert "BUSYKEY" in str(c.pipeline([["RESTORE", "copy", "0", before[b"bs"]]])[0])
        assert c.call("RESTORE", "copy", "0", before[b"bs"], "REPLACE") == "OK"
        assert c.call("GET", "copy") == gets[b"bs"]
        assert c.call("RESTORE", "hcopy", "0", before[b"{bf}__config"]) == "OK"
        assert c.call("HGETALL", "hcopy") == c.call("HGETALL", "{bf}__config")
        c.call("DEL", "copy", "hcopy")
        assert c.call("SAVE") == "OK"
        c.close()
        _stop(p)
        p, port = _start("--dir", str(tmp_path), "--dbfilename", "snap.rdb")   # loads snap.rdb
        c = Client(port)
        assert set(c.call("KEYS", "*")) == keys
        assert {k: c.call("DUMP", k) for k in keys} == before
        assert {k: c.call("GET", k) for k in gets} == gets
        assert c.pipeline([["PFCOUNT", "t:%d" % i] for i in range(9)]) == counts
        assert c.call("EVALSHA", SHA_BLOOM_CHECK, 1, "{bf}__config", "729", "5") is None
        assert c.call("DEBUG", "RELOAD") == "OK"
        assert {k: c.call("DUMP", k) for k in keys} == before
    finally:
        c.close()
        _stop(p)
