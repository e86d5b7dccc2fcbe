"""The incremental probe-index recurrence the Bloom kernels use (sk_device.h BloomIdx): two 64-bit reductions per
element instead of one per probe.  Checked here against Redisson's direct formula (RedissonBloomFilter.java hash():
index_i = (h_i & Long.MAX_VALUE) % size, h_{i+1} = h_i + (i even ? h2 : h1) with 64-bit wrap) over random hashes,
sizes from 1 to 2^32 and every probe count the kernels take; the GPU parity tests check the kernels themselves."""
import random

M64, MAXL = (1 << 64) - 1, (1 << 63) - 1


def direct(h1, h2, k, size):
    h, out = h1, []
    for i in range(k):
        out.append((h & MAXL) % size)
        h = (h + (h2 if i % 2 == 0 else h1)) & M64
    return out


def recurrence(h1, h2, k, size):
    d1, d2 = h1 & MAXL, h2 & MAXL
    a1, a2 = d1 % size, d2 % size
    c = (MAXL % size + 1) % size
    m, r, out = d1, a1, []
    for p in range(k):
        out.append(r)
        d, a = (d1, a1) if p & 1 else (d2, a2)
        s = m + d
        w = s >= 1 << 63
        m = s - (1 << 63) if w else s
        t = r + a - (c if w else 0)
        if t < 0:
            t += size
        elif t >= size:
            t -= size
        r = t
    return out


def test_recurrence_matches_redisson_formula():
    rng = random.Random(7)
    sizes = [1, 2, 3, 7, 1000, 4_271_038_538, (1 << 32) - 2, (1 << 32), rng.randrange(1, 1 << 32)]
    for _ in range(3000):
        h1, h2 = rng.getrandbits(64), rng.getrandbits(64)
        size = rng.choice(sizes)
        k = rng.randrange(1, 12)
        assert recurrence(h1, h2, k, size) == direct(h1, h2, k, size)
    for h1, h2 in [(0, 0), (M64, M64), (MAXL, MAXL), (1 << 63, 1 << 63), (MAXL, 1)]:
        for size in sizes:
            assert recurrence(h1, h2, 9, size) == direct(h1, h2, 9, size)
