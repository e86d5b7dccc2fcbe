"""Multi-GPU orchestration: key partitioning and the exchange steps.

One process per GPU, one engine context each.  Keys are owned by
``calcSlot(key) % world`` (M:cluster/ClusterConnectionManager.java:543-558,
SURVEY 8e): every per-key command runs on its owner with no exchange.  The
only exchange steps are the global ones:

* countWith / PFMERGE over keys spread across GPUs (C4): every rank unions
  its own keys into 16,384 registers on its GPU, then a uint8 MAX all-reduce
  (RCCL over xGMI, ``sk_allreduce_max_u8``), then the estimator / merge.
* RBitSet range-sharded over the GPUs (C5, ``ShardedBitSet``): rank r holds
  bytes [r*S, (r+1)*S) of the Redis string.  SETBIT / GETBIT go to the owner of
  the byte; BITCOUNT = local popcount + uint64 SUM all-reduce; length = the
  last non-empty shard (u64 all-gather); BITOP AND / OR / XOR / NOT between
  bitsets of the same sharding is shard-local (RedissonBitSet.opAsync,
  M:RedissonBitSet.java:138-145) once every operand's shards are padded to
  its logical length.
* BITOP over whole keys that live on different GPUs (``keyed_bitop``; a Bloom
  filter union is BITOP OR of the filters): every rank contributes the
  operands it owns to ONE all-gather (RCCL, device buffers), and the owner of
  the destination runs the local BITOP over the gathered copies
  (north_star: "Bloom/BitSet union uses all-gather plus a local OR").
* One RBloomFilter over several GPUs: ``RangeShardedBloom`` splits its bit
  array by range (the RBitSet shards above): the probe indexes of a batch are
  computed on the submitting GPU and routed to each bit's owner, so capacity
  and add rate grow with the GPUs; ``ReplicatedBloom`` keeps a full copy on
  every GPU (adds on all, contains split and all-gathered, device path
  ``contains_dev``).

The collective is a small interface so the same protocol runs with the
engine's RCCL communicator on GPUs and with torch.distributed/gloo on host
arrays (the CPU tests).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence

import numpy as np

from .engine import owner, owners

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

    @property
    def world(self) -> int:
        return self.dist.get_world_size()

    def allgather_bytes(self, b: bytes) -> List[bytes]:
        out = [None] * self.world
        self.dist.all_gather_object(out, bytes(b))
        return out

    def allgather_u64(self, v: int) -> List[int]:
        out = [None] * self.world
        self.dist.all_gather_object(out, int(v))
        return out

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

    def alltoallv_bytes(self, parts: Sequence[bytes]) -> List[bytes]:
        """parts[p] goes to rank p; returns what every rank sent to this one (gloo: through all_gather_object)."""
        allp = [None] * self.world
        self.dist.all_gather_object(allp, [bytes(x) for x in parts])
        me = self.dist.get_rank()
        return [allp[r][me] for r in range(self.world)]


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

        self.world = world
        self.rank = rank

    def max_u8_dev(self, dbuf, n: int = HLL_REGISTERS):
        self.engine.allreduce_max_u8(dbuf, n)

    def sum_u64(self, v: int) -> int:
        self.u64.upload(np.array([v], dtype=np.uint64))
        self.engine.allreduce_sum_u64(self.u64, 1)
        return int(self.u64.download(np.uint64, 1)[0])

    def max_u8(self, a: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a, dtype=np.uint8)
        if not len(a):
            return a.copy()
        d = self.engine.to_device(a)
        self.engine.allreduce_max_u8(d, len(a))
        out = d.download(np.uint8, len(a))
        d.free()
        return out

    def alltoallv_dev(self, send, send_bytes, recv, recv_bytes):
        """RCCL all-to-all with per-peer byte counts, device buffers (sk_alltoallv)."""
        self.engine.alltoallv(send, send_bytes, recv, recv_bytes)

    def allgather_dev(self, send, recv, nbytes: int):
        """RCCL all-gather of nbytes per rank, device buffers (recv holds world * nbytes)."""
        self.engine.allgather(send, recv, nbytes)

    def allgather_u64(self, v: int) -> List[int]:
        send, recv = self.engine.alloc(8), self.engine.alloc(8 * self.world)
        send.upload(np.array([v], dtype=np.uint64))
        self.engine.allgather(send, recv, 8)
        out = [int(x) for x in recv.download(np.uint64, self.world)]
        send.free()
        recv.free()
        return out

    def allgather_bytes(self, b: bytes) -> List[bytes]:
        sizes = self.allgather_u64(len(b))
        P = max(max(sizes), 1)
        send, recv = self.engine.alloc(P), self.engine.alloc(P * self.world)
        if b:
            send.upload(np.frombuffer(bytes(b), dtype=np.uint8))
        self.engine.allgather(send, recv, P)
        flat = recv.download(np.uint8, P * self.world)
        send.free()
        recv.free()
        return [flat[r * P:r * P + sizes[r]].tobytes() for r in range(self.world)]


class GlobalKeySet:
    """The key set of a repeated global countWith / PFMERGE (C4), resolved once per rank: the slab ids of the
    existing HLLs among `keys` that this rank owns (calcSlot % world), kept on the device.  Each union then streams
    those slabs (sk_hll_union_dev) with no name resolution.  The set is resolved again when the engine's HLL
    keyspace epoch moved (a key created or removed since), so it always names exactly the keys' existing HLLs:
    missing keys count as empty and a key created later is included (PFCOUNT rule, M:RedissonHyperLogLog.java:
    84-89)."""

    def __init__(self, engine, keys, rank: int, world: int):
        from .engine import pack

        self.engine, self.rank, self.world = engine, rank, world
        self.packed = keys if isinstance(keys, tuple) else pack([bytes(k) for k in keys])
        self.n_keys = len(self.packed[0]) - 1
        self.d_ids = None
        self.epoch = None
        self.n = 0
        self.resolves = 0

    def ids(self):
        """(device slab ids, how many): the owned existing HLLs, re-resolved if the keyspace changed."""
        ep = self.engine.hll_epoch()
        if ep != self.epoch:
            own = owners(self.packed, self.world) == self.rank
            h = self.engine.hll_lookup(self.packed)
            mine = np.ascontiguousarray(h[own & (h != 0xFFFFFFFF)], dtype=np.uint32)
            if self.d_ids is not None:
                self.d_ids.free()
            self.d_ids = self.engine.to_device(mine) if len(mine) else None
            self.n, self.epoch = len(mine), ep
            self.resolves += 1
        return self.d_ids, self.n


def _union_buf(engine, coll):
    """The 16 KiB device array a rank's union lands in (the RCCL collective's own buffer, else one per engine)."""
    if hasattr(coll, "buf"):
        return coll.buf
    b = getattr(engine, "_sk_union_buf", None)
    if b is None:
        b = engine.alloc(HLL_REGISTERS)
        engine._sk_union_buf = b
    return b


def agree(coll, err: "Exception | None") -> None:
    """SPMD failure agreement before a protocol's next collective: every rank learns whether any rank failed and all
    of them raise (a failure on one rank alone would leave the others blocked in the collective).  The failing
    rank re-raises its own error; the others raise RedisException naming the first failing rank."""
    from .engine import RedisException

    msg = b"" if err is None else ("%s: %s" % (type(err).__name__, err)).encode()[:1024]
    msgs = coll.allgather_bytes(msg)
    bad = [(r, m) for r, m in enumerate(msgs) if m]
    if not bad:
        return
    if err is not None:
        raise err
    r, m = bad[0]
    raise RedisException("rank %d failed: %s" % (r, m.decode(errors="replace")))


def global_union_registers(engine, keys, rank: int, world: int, coll):
    """Union (register max) of every key in `keys` -- a sequence, an engine.pack() result, or a GlobalKeySet --
    wherever it lives; the result is left in a 16 KiB device array on every rank (returned).  Missing keys count
    as empty (PFCOUNT rule).  Local step: a GlobalKeySet streams its cached device slab ids (sk_hll_union_dev);
    names go through sk_hll_union_keys (owner filter + directory lookup on host threads, then k_hll_union).
    Exchange: RCCL u8 MAX all-reduce on the device, or (HostCollective, gloo) the 16 KiB array through the host."""
    out = _union_buf(engine, coll)
    if isinstance(keys, GlobalKeySet):
        d_ids, n = keys.ids()
        if n:
            engine.hll_union_dev(n, d_ids, out)
        else:
            out.zero()
    else:
        engine.hll_union_keys(keys, world, rank, out)
    if hasattr(coll, "max_u8_dev"):
        coll.max_u8_dev(out)
    else:
        out.upload(coll.max_u8(out.download(np.uint8, HLL_REGISTERS)))
    return out


def global_count_with(engine, keys, rank: int, world: int, coll) -> int:
    """countWith over GPU-sharded keys: exact PFCOUNT of the union (multi-key PFCOUNT: raw-register order), from
    the all-reduced registers on the device -- no key is created or modified."""
    return engine.hll_count_registers_dev(global_union_registers(engine, keys, rank, world, coll))


def global_merge(engine, dest, keys, rank: int, world: int, coll) -> None:
    """PFMERGE dest keys... across GPUs: dest (on its owner) = max(dest, union of keys)."""
    d = global_union_registers(engine, keys, rank, world, coll)
    if owner(dest, world) == rank:
        engine.hll_merge_registers_dev(dest, d)   # the max includes dest's own registers (pfmergeCommand)


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


# ---------------------------------------------------------------- RBitSet across GPUs
def shard_bytes(nbits: int, world: int) -> int:
    """Bytes of the Redis string each rank holds (a multiple of 16)."""
    total = (int(nbits) + 7) // 8
    per = (total + world - 1) // world
    return max(16, (per + 15) // 16 * 16)


class ShardedBitSet:
    """RBitSet of `nbits` bits range-sharded over the ranks (C5): rank r holds bytes [r*S, (r+1)*S) of the Redis
    string as its local key `name`.  Every method is SPMD: all ranks call it with the same arguments and get the
    same reply.  Bit i of the logical string is bit i - 8*r*S of shard r (MSB-first bytes, M:RedissonBitSet.java:
    152-173), so GET of the logical string is the shards concatenated, each zero-filled to min(S, L - r*S)."""

    def __init__(self, engine, name, nbits: int, rank: int, world: int, coll):
        self.engine, self.name, self.rank, self.world, self.coll = engine, name, rank, world, coll
        self.S = shard_bytes(nbits, world)
        self.lo = rank * self.S          # first byte of this rank's shard

    def _device(self) -> bool:
        return hasattr(self.coll, "alltoallv_dev") and hasattr(self.engine, "route_bits")

    def set(self, offsets, values) -> np.ndarray:
        """SETBIT batch submitted on THIS rank (RBitSet.set(i, v) in an RBatch; M:RedissonBitSet.java:79-81): the old
        bits in batch order.  SPMD: every rank calls it, each with its own batch (possibly empty).  Ops travel to
        their shard's owner, which applies them in (submitting rank, batch position) order -- the same result as
        the ranks' batches executed one after another on one redis-server -- and the replies come back; no rank
        sees another shard's ops."""
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        vals = np.ascontiguousarray(np.broadcast_to(np.asarray(values, dtype=np.uint8), offs.shape))
        return self._routed("set", offs, vals)

    def get(self, offsets) -> np.ndarray:
        """GETBIT batch submitted on this rank (RBitSet.get(i), M:RedissonBitSet.java:53-56), routed as set()."""
        return self._routed("get", np.ascontiguousarray(offsets, dtype=np.uint64), None)

    def _routed(self, op, offs, vals) -> np.ndarray:
        if self._device():
            e = self.engine
            n = len(offs)
            bufs = [e.to_device(offs) if n else None, e.to_device(vals) if (n and vals is not None) else None,
                    e.alloc(max(n, 1))]
            try:
                if op == "set":
                    self.set_dev(n, bufs[0], bufs[2], d_values=bufs[1])
                else:
                    self.get_dev(n, bufs[0], bufs[2])
                return bufs[2].download(np.uint8, n)
            finally:
                for b in bufs:
                    if b is not None:
                        b.free()
        return self._routed_host(op, offs, vals)

    def _routed_host(self, op, offs, vals) -> np.ndarray:
        """The router over host arrays and a HostCollective (gloo): the same protocol as set_dev / get_dev."""
        from .engine import RedisException

        W, sb = self.world, 8 * self.S
        sh = (offs // np.uint64(sb)).astype(np.int64) if len(offs) else np.zeros(0, np.int64)
        err = RedisException("ERR bit offset is not an integer or out of range") if (sh >= W).any() else None
        agree(self.coll, err)
        order = np.argsort(sh, kind="stable")
        cnt = np.bincount(sh, minlength=W)
        loc = offs[order] - sh[order].astype(np.uint64) * np.uint64(sb)
        cut = np.concatenate([[0], np.cumsum(cnt)])
        parts = [loc[cut[p]:cut[p + 1]].tobytes() + (vals[order][cut[p]:cut[p + 1]].tobytes() if vals is not None
                                                       else b"") for p in range(W)]
        got = self.coll.alltoallv_bytes(parts)
        # this rank's shard: every rank's ops in rank order, each in its batch order
        ro, rv = [], []
        for g in got:
            k = len(g) // (9 if vals is not None else 8)
            ro.append(np.frombuffer(g[:8 * k], dtype=np.uint64))
            if vals is not None:
                rv.append(np.frombuffer(g[8 * k:], dtype=np.uint8))
        mo = np.concatenate(ro) if ro else np.zeros(0, np.uint64)
        rep = np.zeros(len(mo), dtype=np.uint8)
        err = None
        try:
            if len(mo):
                if op == "set":
                    rep = np.asarray(self.engine.setbit([self.name] * len(mo), mo, np.concatenate(rv)), dtype=np.uint8)
                else:
                    rep = np.asarray(self.engine.getbit([self.name] * len(mo), mo), dtype=np.uint8)
        except Exception as e:  # noqa: BLE001 - agreed on below
            err = e
        agree(self.coll, err)
        rc = np.concatenate([[0], np.cumsum([len(x) for x in ro])])
        back = self.coll.alltoallv_bytes([rep[rc[r]:rc[r + 1]].tobytes() for r in range(W)])
        mine = np.frombuffer(b"".join(back), dtype=np.uint8)
        out = np.zeros(len(offs), dtype=np.uint8)
        out[order] = mine
        return out

    def set_dev(self, n: int, d_offsets, d_out, value: int = 1, d_values=None) -> None:
        """SETBIT of a device batch submitted on this rank (RCCL collective): sk_route_bits splits it by shard on the
        device, sk_alltoallv sends each owner its part (counts first, by an all-gather), the owner applies the ops
        it received in (rank, position) order, the old bits travel back the same way and sk_unroute_u8 puts them in
        batch order into d_out.  One value for every op, or one per op in d_values (u8, device).  d_out None:
        SETBIT_VOID (RBitSet.set(i) with no reply, M:RedissonBitSet.java:79-81): nothing travels back."""
        self._route_dev("set", n, d_offsets, d_out, value, d_values)

    def get_dev(self, n: int, d_offsets, d_out) -> None:
        """GETBIT of a device batch submitted on this rank, routed as set_dev."""
        self._route_dev("get", n, d_offsets, d_out, 0, None)

    _OPS = {"set": 1, "get": 2}

    def _route_dev(self, op, n, d_offsets, d_out, value, d_values) -> None:
        """The device router.  Every rank's call shape travels with its per-shard counts in ONE all-gather (ADVICE
        r3): op, value, whether it passed per-op values and whether it wants replies.  So the collective sequence
        below is decided from the same gathered words on every rank: per-op values travel whenever any rank passed
        them or the ranks' values differ (a rank with one value sends it per op), replies travel back whenever any
        rank wants them, and ranks that called different operations all raise instead of mismatching RCCL calls."""
        from .engine import RedisException

        e, W, me = self.engine, self.world, self.rank
        send, dst = e.alloc(max(8 * n, 8)), e.alloc(max(4 * n, 4))
        tmp = [send, dst]
        try:
            hdr = np.array([self._OPS[op], int(value) & 1, d_values is not None, d_out is not None], dtype=np.uint64)
            gathered = [np.frombuffer(b, dtype=np.uint64)
                        for b in self.coll.allgather_bytes(hdr.tobytes())]
            hdrs = np.stack(gathered)
            if len(set(hdrs[:, 0].tolist())) != 1:
                raise RedisException("ranks called different routed operations on %r: %s"
                                     % (self.name, sorted({k for k, v in self._OPS.items() if v in hdrs[:, 0]})))
            per_op = op == "set" and (bool(hdrs[:, 2].any()) or len(set(hdrs[:, 1].tolist())) != 1)
            want = bool(hdrs[:, 3].any())
            svals = None
            if per_op:
                svals = e.alloc(max(n, 1))
                tmp.append(svals)
                if d_values is None and n:        # this rank's one value, per op
                    d_values = e.to_device(np.full(n, int(value) & 1, dtype=np.uint8))
                    tmp.append(d_values)
            cnt, err = np.zeros(W, dtype=np.uint64), None
            try:
                cnt = e.route_bits(n, d_offsets, d_values if per_op else None, 8 * self.S, W, send, svals, dst)
            except Exception as x:  # noqa: BLE001 - agreed on below
                err = x
            agree(self.coll, err)
            allc = np.stack([np.frombuffer(b, dtype=np.uint64) for b in self.coll.allgather_bytes(cnt.tobytes())])
            rcv = allc[:, me].copy()          # ops this rank owns, from each submitting rank
            m = int(rcv.sum())
            recv, rep = e.alloc(max(8 * m, 8)), e.alloc(max(m, 1))
            tmp += [recv, rep]
            self.coll.alltoallv_dev(send, cnt * 8, recv, rcv * 8)
            rvals = None
            if per_op:
                rvals = e.alloc(max(m, 1))
                tmp.append(rvals)
                self.coll.alltoallv_dev(svals, cnt, rvals, rcv)
            err = None
            try:
                if m and op == "set" and per_op:
                    e.setbit_values_dev(self.name, m, recv, rvals, rep if want else None)
                elif m and op == "set":
                    e.setbit_dev(self.name, m, recv, int(hdrs[0, 1]), rep if want else None)
                elif m:
                    e.getbit_dev(self.name, m, recv, rep)
            except Exception as x:  # noqa: BLE001 - agreed on below
                err = x
            agree(self.coll, err)
            if not want:
                return
            back = e.alloc(max(n, 1))
            tmp.append(back)
            self.coll.alltoallv_dev(rep, rcv, back, cnt)
            if n and d_out is not None:
                e.unroute_u8(n, dst, back, d_out)
        finally:
            for b in tmp:
                b.free()

    def _local_len(self) -> int:
        return self.engine.strlen(self.name)

    def length_bytes(self) -> int:
        """STRLEN of the logical string: the end of the last non-empty shard."""
        lens = self.coll.allgather_u64(self._local_len())
        return max([r * self.S + ln for r, ln in enumerate(lens) if ln] or [0])

    def size(self) -> int:
        """RBitSet.size() = STRLEN * 8 (int overflow, Q3: M:client/protocol/convertor/BitsSizeReplayConvertor.java)."""
        v = (self.length_bytes() * 8) & 0xFFFFFFFF
        return v - (1 << 32) if v >= 1 << 31 else v

    def cardinality(self) -> int:
        """BITCOUNT: local popcount + u64 SUM all-reduce (RedissonBitSet.cardinalityAsync, :240-243)."""
        return self.coll.sum_u64(self.engine.bitcount(self.name))

    def _pad_to(self, L: int):
        """Grow this shard with zero bytes to its part of a logical length L (content unchanged)."""
        want = min(self.S, max(0, L - self.lo))
        if want > self._local_len():
            self.engine.setbit([self.name], [8 * want - 1], [0], want_old=False)

    def op(self, op: str, others: Sequence["ShardedBitSet"] = ()) -> None:
        """BITOP op name name others... (RedissonBitSet.and/or/xor/not -> opAsync, M:RedissonBitSet.java:138-145,
        216-219, 255-268): shard-local once every operand is padded to its logical length, since byte j of the
        result depends only on byte j of the operands and the result length is the longest operand."""
        ops = [self] + list(others)
        for o in ops:
            if o.S != self.S:
                raise ValueError("BITOP across bitsets of different shardings")
        lens = [o.length_bytes() for o in ops]
        for o, L in zip(ops, lens):
            o._pad_to(L)
        self.engine.bitop(op, self.name, [o.name for o in ops])

    def to_bytes(self) -> bytes:
        """GET of the logical string (RBitSet.toByteArray, :88-91): the shards, each zero-filled to its part."""
        L = self.length_bytes()
        mine = self.engine.get(self.name) or b""
        want = min(self.S, max(0, L - self.lo))
        parts = self.coll.allgather_bytes(mine[:want] + b"\0" * (want - len(mine[:want])))
        return b"".join(parts)[:L]


def _owned_lengths(engine, keys: Sequence, rank: int, world: int, coll) -> List[int]:
    """Byte length of every key (-1: missing), each reported by its owner.  SPMD: a failure on one rank raises on
    every rank (cluster.agree) before the all-gather."""
    mine = np.full(len(keys), -2, dtype=np.int64)
    err = None
    try:
        for i, k in enumerate(keys):
            if owner(k, world) == rank:
                t = engine.key_type(k)
                mine[i] = engine.strlen(k) if t else -1
    except Exception as e:  # noqa: BLE001 - agreed on below
        err = e
    agree(coll, err)
    parts = coll.allgather_bytes(mine.tobytes())
    allv = np.stack([np.frombuffer(p, dtype=np.int64) for p in parts])
    return [int(allv[owner(k, world), i]) for i, k in enumerate(keys)]


def _source_to_dev(engine, key, buf, at: int, n: int) -> None:
    """The first n bytes of a BITOP source into device buffer `buf` at byte `at`: a bit string device to device; any
    other string (an HLL reads as its Redis encoding, as BITOP on redis-server takes it) through the host."""
    from . import _native as N

    if engine.key_type(key) == N.SK_TYPE_STRING:
        engine.get_dev(key, buf.ptr + at, n)
    else:
        buf.upload(np.frombuffer((engine.get(key) or b"")[:n], dtype=np.uint8), at)


def keyed_bitop(engine, op: str, dest, srcs: Sequence, rank: int, world: int, coll,
                tmp_prefix: bytes = b"__sk_bitop_src__:") -> int:
    """BITOP op dest srcs... where every key lives whole on its owner (calcSlot % world): each rank contributes the
    sources it owns to one all-gather, and dest's owner runs the local BITOP over the gathered copies (missing
    sources are empty strings, as in Redis; an HLL source reads as its Redis string).  Returns the result length on
    every rank.  A Bloom filter union is keyed_bitop("OR", ...) over the filters' names (same size and k).  SPMD:
    a failure on any rank (reading a source, the destination's BITOP) raises on every rank (cluster.agree) instead
    of leaving the others in a collective."""
    if op.upper() == "NOT" and len(srcs) != 1:
        raise ValueError("BITOP NOT must be called with a single source key.")
    lens = _owned_lengths(engine, srcs, rank, world, coll)
    mine = [i for i, k in enumerate(srcs) if owner(k, world) == rank]
    base = {}
    pos = 0
    for i in mine:                            # this rank's blob: its sources back to back
        base[i] = pos
        pos += max(lens[i], 0)
    blobs = coll.allgather_u64(pos)
    P = max(max(blobs), 1)
    # where every source sits in the gathered buffer: rank owner(src) * P + offset inside that rank's blob
    where = {}
    for r in range(world):
        q = 0
        for i, k in enumerate(srcs):
            if owner(k, world) == r:
                where[i] = r * P + q
                q += max(lens[i], 0)
    d_owner = owner(dest, world)
    tmp = [tmp_prefix + b"%d" % i for i in range(len(srcs))]
    if hasattr(coll, "allgather_dev"):        # GPUs: bit-string operands never leave HBM
        send, recv = engine.alloc(P), engine.alloc(P * world)
        try:
            err = None
            try:
                for i in mine:
                    if lens[i] > 0:
                        _source_to_dev(engine, srcs[i], send, base[i], lens[i])
            except Exception as e:  # noqa: BLE001 - agreed on below
                err = e
            agree(coll, err)
            coll.allgather_dev(send, recv, P)
            if rank == d_owner:
                for i in range(len(srcs)):
                    if lens[i] >= 0:
                        engine.set_dev(tmp[i], recv.ptr + where[i], lens[i])
        finally:
            send.free()
            recv.free()
    else:
        blob, err = b"", None
        try:
            blob = b"".join((engine.get(srcs[i]) or b"") for i in mine)
        except Exception as e:  # noqa: BLE001 - agreed on below
            err = e
        agree(coll, err)
        parts = coll.allgather_bytes(blob)
        flat = b"".join(p + b"\0" * (P - len(p)) for p in parts)
        if rank == d_owner:
            for i in range(len(srcs)):
                if lens[i] >= 0:
                    engine.set(tmp[i], flat[where[i]:where[i] + lens[i]])
    n, err = 0, None
    if rank == d_owner:
        try:
            n = engine.bitop(op, dest, tmp)
        except Exception as e:  # noqa: BLE001 - agreed on below
            err = e
        finally:
            engine.delete(tmp)
    agree(coll, err)
    return max(coll.allgather_u64(n))


# ---------------------------------------------------------------- one Bloom filter served by N GPUs
class ReplicatedBloom:
    """One RBloomFilter served by every GPU of the node: each rank holds a full replica of the bit array.
    SPMD: ``add`` is called by every rank with the same elements and applied to every replica (the replicas stay
    identical, so every rank gets the same exact replies); ``contains`` splits the batch, rank r answers elements
    [r*n/N, (r+1)*n/N) on its replica, and the replies are all-gathered.  Read traffic (the C3 metric) scales
    with the GPUs; adds cost every GPU the whole batch, which is the price of serving one hot filter from N.
    (A filter that only one GPU should hold simply lives on its calcSlot owner, like any other key.)"""

    def __init__(self, engine, name, rank: int, world: int, coll):
        self.engine, self.name, self.rank, self.world, self.coll = engine, name, rank, world, coll

    def try_init(self, expected: int, fpp: float) -> bool:
        return self.engine.bloom_try_init(self.name, expected, fpp)

    def _cfg(self):
        size, k, _, _ = self.engine.bloom_config(self.name)
        return size, k

    def add(self, elems: Sequence[bytes]) -> List[bool]:
        size, k = self._cfg()
        return self.engine.bloom_add(self.name, size, k, list(elems))

    def contains(self, elems: Sequence[bytes]) -> List[bool]:
        size, k = self._cfg()
        n = len(elems)
        lo, hi = self.rank * n // self.world, (self.rank + 1) * n // self.world
        mine = self.engine.bloom_contains(self.name, size, k, list(elems[lo:hi])) if hi > lo else []
        parts = self.coll.allgather_bytes(bytes(int(x) for x in mine))
        return [bool(b) for p in parts for b in p]

    def add_dev(self, n: int, d_off, d_bytes, bytes_len: int, d_out) -> None:
        """add of a device batch (the same batch on every rank): applied to every replica, the same exact replies."""
        self.engine.bloom_add_dev(self.name, n, d_off, d_bytes, bytes_len, d_out)

    def contains_dev(self, n: int, d_off, d_bytes, bytes_len: int, d_out) -> None:
        """contains of a device batch held by every rank, with no host copy: rank r answers elements [r*P, (r+1)*P)
        (P = ceil(n / world)) on its replica, and one RCCL all-gather of the P-byte reply pieces lays the replies out
        in batch order on every rank (into d_out, n bytes)."""
        W, r = self.world, self.rank
        P = max((n + W - 1) // W, 1)
        lo, hi = min(r * P, n), min((r + 1) * P, n)
        e = self.engine
        part, recv = e.alloc(P), e.alloc(P * W)
        try:
            err = None
            try:
                if hi > lo:
                    e.bloom_contains_dev(self.name, hi - lo, d_off.view(8 * lo), d_bytes, bytes_len, part)
            except Exception as x:  # noqa: BLE001 - agreed on below
                err = x
            agree(self.coll, err)
            self.coll.allgather_dev(part, recv, P)
            if n:
                e.d2d(d_out, recv, n)
        finally:
            part.free()
            recv.free()


def java_int(x: float) -> int:
    """Java's (int) of a double: NaN -> 0, saturating, else truncation toward zero."""
    if x != x:
        return 0
    if x >= 2147483647.0:
        return 2147483647
    if x <= -2147483648.0:
        return -2147483648
    return int(x)


class RangeShardedBloom:
    """One RBloomFilter whose bit array is range-sharded over the GPUs: rank r holds bits [r*S, (r+1)*S) of the
    m-bit array as its local bit string `name` (the RBitSet shards of ShardedBitSet).  add / contains of a device
    batch submitted on any rank (M:RedissonBloomFilter.java:80-168):
      1. the probe bit indexes are computed on the submitting GPU (sk_bloom_indexes_dev: k for add, the k-1 that
         decide contains for contains -- Q2), element-major;
      2. they travel to the owner of each bit through the RBitSet router (sk_route_bits + RCCL all-to-all), which
         applies them in (submitting rank, element, probe) order -- SETBIT with old-bit replies for add, GETBIT for
         contains -- so every reply is the one redis-server gives when the ranks' batches run one after another;
      3. the per-probe replies come back in element order and sk_reduce_groups_u8 makes one reply per element:
         contains = AND of probes 0..k-2, add = one of probes 0..k-2 was 0.
    Each GPU holds 1/N of the array and applies 1/N of every batch's probes, so the filter's capacity and its add
    rate grow with N; ReplicatedBloom instead applies every add on every GPU.  Every method is SPMD: all ranks call
    it (an empty batch is fine) with the same filter configuration."""

    def __init__(self, engine, name, rank: int, world: int, coll):
        self.engine, self.name, self.rank, self.world, self.coll = engine, name, rank, world, coll
        self.size = self.k = 0
        self.bits = None

    def try_init(self, expected: int, fpp: float) -> bool:
        """RedissonBloomFilter.tryInit sizing (:69-78, :223-252): False when already initialized (config replaced,
        Q6); IllegalArgumentException above 4,294,967,294 bits (Q4)."""
        from .engine import IllegalArgumentException, bloom_optimal_bits, bloom_optimal_k

        m = bloom_optimal_bits(expected, fpp)
        if m > 2 * 2147483647:
            raise IllegalArgumentException("Bloom filter can't be greater than %d. But calculated size is %d"
                                           % (2 * 2147483647, m))
        fresh = self.bits is None
        self.size, self.k = int(m), int(bloom_optimal_k(expected, m))
        if fresh:
            self.bits = ShardedBitSet(self.engine, self.name, self.size, self.rank, self.world, self.coll)
        elif self.size > 8 * self.bits.S * self.world:
            # Q6 keeps the one global bit string and only replaces the config: bit i stays bit i.  The first layout
            # is kept while it covers the new size; a larger filter gets a wider layout, and the existing bits are
            # moved to their new owners (every rank holds the logical string after to_bytes, then keeps its part)
            whole = self.bits.to_bytes()
            self.bits = ShardedBitSet(self.engine, self.name, self.size, self.rank, self.world, self.coll)
            mine = whole[self.bits.lo:self.bits.lo + self.bits.S]
            if mine:
                self.engine.set(self.name, mine)
            else:
                self.engine.delete([self.name])
        return fresh

    def _check(self):
        from .engine import IllegalStateException

        if self.bits is None:
            raise IllegalStateException("Bloom filter is not initialized!")

    def add_dev(self, n: int, d_off, d_bytes, d_out=None) -> None:
        """add of n device elements submitted on this rank; d_out: one reply per element (None: no replies)."""
        self._check()
        e, k = self.engine, self.k
        idx, rep = e.alloc(max(8 * n * k, 8)), e.alloc(max(n * k, 1))
        try:
            e.bloom_indexes_dev(n, d_off, d_bytes, self.size, k, k, idx)
            self.bits.set_dev(n * k, idx, rep if d_out is not None else None, value=1)
            if d_out is not None and n:
                e.reduce_groups_u8(n, k, k - 1, True, rep, d_out)
        finally:
            idx.free()
            rep.free()

    def contains_dev(self, n: int, d_off, d_bytes, d_out) -> None:
        """contains of n device elements submitted on this rank (one reply per element in d_out)."""
        self._check()
        e, np_ = self.engine, self.k - 1
        idx, rep = e.alloc(max(8 * n * np_, 8)), e.alloc(max(n * np_, 1))
        try:
            e.bloom_indexes_dev(n, d_off, d_bytes, self.size, self.k, np_, idx)
            self.bits.get_dev(n * np_, idx, rep)
            if n:
                e.reduce_groups_u8(n, np_, np_, False, rep, d_out)
        finally:
            idx.free()
            rep.free()

    def _host(self, op, elems: Sequence[bytes]) -> List[bool]:
        from .engine import pack

        e, n = self.engine, len(elems)
        off, buf = pack([bytes(x) for x in elems])
        d_off, d_bytes, d_out = e.to_device(off), e.to_device(buf, pad=16), e.alloc(max(n, 1))
        try:
            (self.add_dev if op == "add" else self.contains_dev)(n, d_off, d_bytes, d_out)
            return [bool(x) for x in d_out.download(np.uint8, n)]
        finally:
            for b in (d_off, d_bytes, d_out):
                b.free()

    def add(self, elems: Sequence[bytes]) -> List[bool]:
        return self._host("add", elems)

    def contains(self, elems: Sequence[bytes]) -> List[bool]:
        return self._host("contains", elems)

    def count(self) -> int:
        """RedissonBloomFilter.count (:188-199): BITCOUNT over every shard, then -m/k * ln(1 - bits/m) as a Java int."""
        import math

        self._check()
        c = self.bits.cardinality()
        x = 1 - c / self.size
        v = (-self.size / self.k) * (math.log(x) if x > 0 else float("-inf"))
        return java_int(v)

    def to_bytes(self) -> bytes:
        """GET of the filter's bit array (the Redis string: every shard's bytes, up to the last non-empty one)."""
        self._check()
        return self.bits.to_bytes()
