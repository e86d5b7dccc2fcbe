"""Multi-rank protocol on CPU (gloo, world size 2) and the RCCL wiring on one GPU.

CPU: the partitioner gives every key exactly one owner; the global
countWith protocol (local union -> MAX all-reduce -> estimator) equals the
single-process oracle count of the union; range-sharded BITCOUNT sums.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ret):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist

    from oracle import oracle as O
    from redisson_amd import _native, owner
    from redisson_amd.cluster import HostCollective, host_global_count_with, partition

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = _native.load()

    keys = [b"tenant:%d:hll" % i for i in range(64)] + [b"{grp}:a", b"{grp}:b"]
    parts = partition(keys, world)
    # every rank builds ONLY the keys it owns (what its GPU would hold)
    store = O.HLLStore()
    rng = np.random.default_rng(7)
    for k in keys:
        n = int(rng.integers(0, 3000))
        els = [b'["java.lang.Long",%d]' % int(x) for x in rng.integers(-(1 << 62), 1 << 62, n)]
        if owner(k, world) == rank:
            store.pfadd([k] * n, [[e] for e in els])
    coll = HostCollective(dist)
    got = host_global_count_with(store.regs, keys, rank, world, coll,
                                 lambda h: int(lib.sk_hll_estimate_hist(h.ctypes.data, 3)))
    # range-sharded bitcount: rank r owns bytes [r*L/world, (r+1)*L/world)
    data = np.random.default_rng(3).integers(0, 256, 10007, dtype=np.uint8)
    lo, hi = rank * len(data) // world, (rank + 1) * len(data) // world
    local_bits = int(np.unpackbits(data[lo:hi]).sum())
    total_bits = coll.sum_u64(local_bits)
    ret[rank] = (got, total_bits, sorted(len(v) for v in parts.values()), int(np.unpackbits(data).sum()))
    dist.destroy_process_group()


def test_global_countwith_and_bitcount_two_ranks(O):
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    ret = mgr.dict()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ret)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    # single-process reference: the same keys and elements, one store
    rng = np.random.default_rng(7)
    keys = [b"tenant:%d:hll" % i for i in range(64)] + [b"{grp}:a", b"{grp}:b"]
    store = O.HLLStore()
    for k in keys:
        n = int(rng.integers(0, 3000))
        els = [b'["java.lang.Long",%d]' % int(x) for x in rng.integers(-(1 << 62), 1 << 62, n)]
        store.pfadd([k] * n, [[e] for e in els])
    want = store.count(keys)
    assert ret[0][0] == ret[1][0] == want
    assert ret[0][1] == ret[1][1] == ret[0][3]
    assert sum(ret[0][2]) == len(keys)


def test_partition_colocates_hashtags():
    from redisson_amd import owner
    from redisson_amd.cluster import partition

    parts = partition([b"{bf}__config", b"bf", b"{x}1", b"{x}2"], 8)
    owners = {k: r for r, ks in parts.items() for k in ks}
    assert owners[b"{x}1"] == owners[b"{x}2"]
    # RBloomFilter's config hash "{name}__config" lives with "name" (same slot)
    assert owner(b"{bf}__config", 8) == owner(b"bf", 8)
    with pytest.raises(ValueError):
        partition([b"a}b{c"], 2)


@pytest.mark.gpu
def test_rccl_single_rank_exchange(engine, O):
    """The engine's RCCL communicator on one GPU: union + MAX all-reduce +
    merge + countWith, exact vs the oracle; u64 SUM all-reduce."""
    from redisson_amd.cluster import RcclCollective, global_count_with, global_merge

    coll = RcclCollective(engine, 0, 1)
    keys = [b"g4:%d" % i for i in range(50)]
    ref = O.HLLStore()
    rng = np.random.default_rng(9)
    for k in keys:
        n = int(rng.integers(1, 2000))
        els = [b"%d" % int(x) for x in rng.integers(0, 1 << 60, n)]
        engine.pfadd([k] * n, [[e] for e in els])
        ref.pfadd([k] * n, [[e] for e in els])
    assert global_count_with(engine, keys + [b"g4:absent"], 0, 1, coll) == ref.count(keys)
    global_merge(engine, b"g4:dest", keys, 0, 1, coll)
    ref.merge(b"g4:dest", keys)
    np.testing.assert_array_equal(engine.hll_registers(b"g4:dest"), ref.regs[b"g4:dest"])
    assert coll.sum_u64(12345) == 12345
