"""Multi-GPU orchestration: key partitioning and the exchange steps.

One process per GPU, one engine context each.  Keys are owned by
``calcSlot(key) % world`` (M:cluster/ClusterConnectionManager.java:543-558,
SURVEY 8e): every per-key command runs on its owner with no exchange.  The
only exchange steps are the global ones:

* countWith / PFMERGE over keys spread across GPUs (C4): every rank unions
  its own keys into 16,384 registers on its GPU, then a uint8 MAX all-reduce
  (RCCL over xGMI, ``sk_allreduce_max_u8``), then the estimator / merge.
* BITCOUNT of a range-sharded bitset (C5): local popcount, then a uint64 SUM
  all-reduce.

The collective is a small interface so the same protocol runs with the
engine's RCCL communicator on GPUs and with torch.distributed/gloo on host
arrays (the CPU tests).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence

import numpy as np

from .engine import owner

HLL_REGISTERS = 16384


def partition(keys: Iterable, world: int) -> Dict[int, List]:
    """rank -> keys it owns (calcSlot % world); keys whose calcSlot throws are rejected."""
    out: Dict[int, List] = {r: [] for r in range(world)}
    for k in keys:
        r = owner(k, world)
        if r < 0:
            raise ValueError(f"calcSlot throws for key {k!r} (a '}}' before the '{{')")
        out[r].append(k)
    return out


class HostCollective:
    """torch.distributed on host arrays (gloo); what the CPU tests run."""

    def __init__(self, dist):
        self.dist = dist

    def max_u8(self, regs: np.ndarray) -> np.ndarray:
        import torch

        t = torch.from_numpy(np.ascontiguousarray(regs, dtype=np.uint8).astype(np.int32))
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return t.numpy().astype(np.uint8)

    def sum_u64(self, v: int) -> int:
        import torch

        t = torch.tensor([int(v)], dtype=torch.int64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return int(t.item())


class RcclCollective:
    """RCCL over xGMI through the engine (device buffers, the context's stream)."""

    def __init__(self, engine, rank: int, world: int, dist=None):
        self.engine = engine
        uid = engine.comm_unique_id() if rank == 0 else b"\0" * 128
        if world > 1:
            box = [uid]
            dist.broadcast_object_list(box, src=0)  # gloo on the host: only the 128-byte id travels
            uid = box[0]
        engine.comm_init(world, rank, uid)
        self.buf = engine.alloc(HLL_REGISTERS)
        self.u64 = engine.alloc(8)

    def max_u8_dev(self, dbuf, n: int = HLL_REGISTERS):
        self.engine.allreduce_max_u8(dbuf, n)

    def sum_u64(self, v: int) -> int:
        self.u64.upload(np.array([v], dtype=np.uint64))
        self.engine.allreduce_sum_u64(self.u64, 1)
        return int(self.u64.download(np.uint64, 1)[0])


def global_union_registers(engine, keys: Sequence, rank: int, world: int, coll: RcclCollective):
    """Union (register max) of every key in `keys`, wherever it lives; result
    left in coll.buf on every rank.  Missing keys count as empty (PFCOUNT rule)."""
    mine = [k for k in keys if owner(k, world) == rank and engine.key_type(k) != 0]
    if mine:
        ids = engine.hll_resolve(mine)              # existing keys: ids only
        d_ids = engine.to_device(ids)
        engine.hll_union_dev(len(ids), d_ids, coll.buf)
        d_ids.free()
    else:
        coll.buf.zero()
    coll.max_u8_dev(coll.buf)
    return coll.buf


def global_count_with(engine, keys: Sequence, rank: int, world: int, coll: RcclCollective,
                      tmp_key: bytes = b"__sk_global_union__") -> int:
    """countWith over GPU-sharded keys: exact PFCOUNT of the union (raw order)."""
    d = global_union_registers(engine, keys, rank, world, coll)
    engine.hll_merge_registers_dev(tmp_key, d)
    try:
        return engine.pfcount([[tmp_key, b"__sk_missing__"]])[0]   # multi-key PFCOUNT = raw-register union
    finally:
        engine.delete([tmp_key])


def global_merge(engine, dest, keys: Sequence, rank: int, world: int, coll: RcclCollective) -> None:
    """PFMERGE dest keys... across GPUs: dest (on its owner) = max(dest, union)."""
    d = global_union_registers(engine, list(keys) + [dest], rank, world, coll)
    if owner(dest, world) == rank:
        engine.hll_merge_registers_dev(dest, d)


def host_global_count_with(local_regs: Dict, keys: Sequence, rank: int, world: int, coll: HostCollective,
                           estimate) -> int:
    """The same protocol over host register arrays (CPU tests): union of the
    keys this rank owns, MAX all-reduce, estimator from the 64-bin histogram."""
    u = np.zeros(HLL_REGISTERS, dtype=np.uint8)
    for k in keys:
        if owner(k, world) == rank and k in local_regs:
            np.maximum(u, local_regs[k], out=u)
    u = coll.max_u8(u)
    hist = np.bincount(u, minlength=64).astype(np.uint32)
    return estimate(hist)
