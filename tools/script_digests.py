"""Derive the SHA1 digests of the Lua scripts Redisson sends for the sketch
path (EVAL bodies in M:RedissonBloomFilter.java and M:RedissonBitSet.java).

The RESP front-end (redisson_amd/csrc/sk_resp.cpp) recognises a script by its
digest and runs the native equivalent; this generator reads the reference's
Java string literals (study only, run in the build container where
/root/reference exists) and prints the digests that sk_resp.cpp holds.
"""
import hashlib
import re
import sys

REF = "/root/reference/src/main/java/org/redisson/"


def literals_after(src, anchor, stop):
    """Concatenate the Java string literals between `anchor` and the first `stop` after it."""
    i = src.index(anchor)
    j = src.index(stop, i)
    return "".join(bytes(m, "utf-8").decode("unicode_escape") for m in re.findall(r'"((?:[^"\\]|\\.)*)"', src[i:j]))


def main():
    bloom = open(REF + "RedissonBloomFilter.java").read()
    bits = open(REF + "RedissonBitSet.java").read()
    out = {
        "bloom_config_check": literals_after(bloom, "private void addConfigCheck", "Arrays.<Object>asList"),
        "bloom_try_init_check": literals_after(bloom[bloom.index("public boolean tryInit"):], "RedisCommands.EVAL_VOID",
                                               "Arrays.<Object>asList"),
        "bitset_length": literals_after(bits, "public Future<Long> lengthAsync", "Collections.<Object>singletonList"),
    }
    for k, v in out.items():
        print(k, hashlib.sha1(v.encode()).hexdigest(), len(v), file=sys.stdout)


if __name__ == "__main__":
    main()
