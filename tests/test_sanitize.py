"""ASan + UBSan on the engine's host C++, CPU only.

tests/fuzz/fuzz_host.cpp is built with -fsanitize=address,undefined (no recovery: any report aborts the run) over
the host-side code that parses caller or network input -- the Redis HLL string codec (sk_hllstr.h: dense / sparse
decode of random and mutated strings, hllSparseSet replays compared byte for byte with the oracle's), the RESP
request parser (sk_resp_parse.h: random streams, valid pipelines in random chunks, mutated pipelines), the redis
persistence formats (sk_rdb.h: CRC64 and the Redis documentation's DUMP example as known answers, LZF, ziplist hashes,
DUMP payloads and RDB file images round-tripped and mutated) -- and the
device hash code of sk_device.h compiled for the host (XXH64, farmhashuo, the shared-prefix path, BloomIdx against the
oracle at every alignment)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fuzz_host_parsers_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "fuzz")], check=True)
    exe = os.path.join(ROOT, "build", "fuzz_host")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    for seed in (1, 2):
        r = subprocess.run([exe, "6000", str(seed)], capture_output=True, text=True, env=env, timeout=600)
        out = r.stdout + r.stderr
        assert r.returncode == 0, out[-4000:]
        assert "runtime error" not in out and "AddressSanitizer" not in out, out[-4000:]
        assert "0 failures" in out, out[-2000:]
