#!/usr/bin/env python3
"""bench_configs.py -- the other BASELINE.json configs, one JSON line each.

bench.py measures the headline (C2 PFADD + C3 Bloom contains).  This script
measures the remaining configs on one MI355X with inputs resident in HBM:

  c1  RHyperLogLog: 1M random Longs into ONE key as 1M RBatch PFADDs (dense
      path: exact replies via radix sort), and the reference addAll (Q1: one
      element = the Jackson array, ~38 MB) + count().
  c2zipf  the C2 PFADD batches with Zipf(1.1) tenants (SURVEY 8d variant).
  c4  1M tenant HLLs x 1,000 elements (1B PFADD, sharded by calcSlot % 8 ->
      the slab set of one GPU of 8 is timed at full size here), then the
      global union / countWith over all of them: k_hll_union streams 16 KiB
      per source (roofline: HBM streaming).
  c5  RBitSet 2^34 bits (2 GiB): 1B random SETBIT (SETBIT_VOID), 1B GETBIT,
      BITCOUNT, AND/OR across 4 bitsets (BITOP streams (s+1)*N/8 bytes).
  host  the host-buffer C ABI the JNI shim calls (PCIe-inclusive): C2-shaped
      PFADD and C3-shaped Bloom add/contains batches from pageable host arrays.

N-rank modes (one process per GPU under torch.distributed.run, RCCL over xGMI
between the engine contexts; they also run at world size 1):
  c4mr  C4 as stated: 1M tenant HLLs x 1,000 elements sharded by calcSlot % N,
      then countWith / PFMERGE over ALL of them: local union + RCCL u8 MAX
      all-reduce (redisson_amd/cluster.py).  Total keys fixed: strong scaling.
  c5mr  C5 as stated: 2^34-bit RBitSets range-sharded over the N GPUs
      (ShardedBitSet): SETBIT/GETBIT on each rank's own range, BITCOUNT (local
      + u64 SUM all-reduce), AND/OR of sharded bitsets (shard-local), and a
      BITOP OR of two whole bitsets owned by different GPUs (one RCCL
      all-gather + a local OR).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
from redisson_amd import JsonJacksonCodec, JLong, SketchEngine, gen_jackson_longs, owner  # noqa: E402
from redisson_amd.engine import owners, pack  # noqa: E402

PEAK = 8000.0


def line(d):
    print(json.dumps(d), flush=True)


SLAB = 12288   # bytes a PFCOUNT / union kernel reads per key: the arena's packed 6-bit register body


def timed(eng, fn, reps=1):
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    eng.sync()
    return (time.perf_counter() - t0) / reps


def c1(eng, args):
    n = args.c1_n
    off, byt, tot = eng.gen_jackson_longs_dev(0x5EED0001, n)
    ids = eng.hll_resolve([b"hll:c1"])
    d_ids = eng.to_device(np.full(n, ids[0], dtype=np.uint32))
    d_out = eng.alloc(n)
    eng.pfadd_dev(n, d_ids, off, byt, tot, d_out)            # warm (and fills the registers)
    eng.delete([b"hll:c1"])
    ids = eng.hll_resolve([b"hll:c1"])
    d_ids.upload(np.full(n, ids[0], dtype=np.uint32))
    t = timed(eng, lambda: eng.pfadd_dev(n, d_ids, off, byt, tot, d_out))   # one 1M batch, host-timed
    cnt = eng.pfcount([[b"hll:c1"]])[0]
    # steady state: 10 more 1M batches of fresh Longs into the same key, back to back
    steps = 10
    off2, byt2, tot2 = eng.gen_jackson_longs_dev(0x5EED0011, n * steps)
    d_ids2 = eng.to_device(np.full(n * steps, ids[0], dtype=np.uint32))
    eng.pfadd_dev(n, d_ids2, off2, byt2, tot2, d_out)
    eng.set_async(True)   # batches are enqueued back to back; timed() syncs once at the end
    t_ss = timed(eng, lambda: [eng.pfadd_dev(n, d_ids2.ptr + s * n * 4, off2.ptr + s * n * 8, byt2, tot2, d_out)
                               for s in range(steps)])
    eng.set_async(False)
    # group commit: the same 10 RBatches as ONE device call (line schedule); replies checked equal-sized only
    d_out10 = eng.alloc(n * steps)
    eng.delete([b"hll:c1"])
    ids = eng.hll_resolve([b"hll:c1"])
    d_ids2.upload(np.full(n * steps, ids[0], dtype=np.uint32))
    eng.pfadd_dev(n, d_ids2, off2, byt2, tot2, d_out)            # the same first batch as above, then the group
    eng.pfadd_dev(n * steps, d_ids2, off2, byt2, tot2, d_out10)  # warm: the line schedule's scratch is allocated
    eng.delete([b"hll:c1"])                                      # the key again as it was before the warm call
    ids = eng.hll_resolve([b"hll:c1"])
    d_ids2.upload(np.full(n * steps, ids[0], dtype=np.uint32))
    eng.pfadd_dev(n, d_ids2, off2, byt2, tot2, d_out)
    eng.prof_reset(); eng.prof_enable(True)
    t_g = timed(eng, lambda: eng.pfadd_dev(n * steps, d_ids2, off2, byt2, tot2, d_out10))
    eng.prof_enable(False)
    g_ms = {p: eng.prof_read(p)[1] for p in ("pfl_hash", "pfl_part", "pfl_apply")}
    d_out10.free()
    off2.free(); byt2.free(); d_ids2.free()
    # Q1: addAll(1M Longs) = ONE PFADD element, the Jackson encoding of Object[]{name, e1..en}
    vals = np.random.default_rng(1).integers(-(1 << 63), (1 << 63) - 1, min(n, 1 << 20), dtype=np.int64)
    blob = JsonJacksonCodec().encode(["hll:c1q"] + [JLong(int(v)) for v in vals])
    eng.pfadd([b"hll:c1q"], [[blob]])                          # warm (staging buffers)
    eng.prof_reset(); eng.prof_enable(True)
    t_q1 = timed(eng, lambda: eng.pfadd([b"hll:c1q"], [[blob]]))
    eng.prof_enable(False)
    n_l, ms_long = eng.prof_read("pfadd_long")   # the element's bit-round hash (k_ms_planes + k_ms_rounds), device time
    line({"metric": "C1 PFADD inserts/sec (one key, RBatch of single-element PFADDs)", "value": n * steps / t_ss,
          "unit": "inserts/s", "config": {"workload": "c1", "elements": n, "count_after": cnt},
          "steady_state": "%d back-to-back batches of %d fresh Longs into the one key" % (steps, n),
          "single_batch_inserts_per_s_host_timed": n / t,
          "group_commit_inserts_per_s": n * steps / t_g,
          "group_commit": "the %d batches as one call (line schedule), host-timed after a warm call" % steps,
          "group_commit_kernel_ms": g_ms,
          "group_commit_device_inserts_per_s": n * steps / (sum(g_ms.values()) * 1e-3) if all(g_ms.values()) else None,
          "addAll_q1": {"element_bytes": len(blob), "seconds": t_q1, "hash_ms_device": ms_long / max(n_l, 1),
                        "count_after":
                        eng.pfcount([[b"hll:c1q"]])[0]}})


def c2u(eng, args):
    """C2 as one RBatch per call (RedissonBatch.execute -> one device call, M:RedissonBatch.java:226-228): 1M-command
    PFADD batches over 100k uniform tenants, each its own sk_pfadd_dev call (the partition path: k_pfp_hash +
    k_pfp_apply), device-timed (HIP events around each call's chain) and host-timed."""
    B, steps, nt = 1 << 20, 20, 100_000
    names = [b"tenant:%d:hll" % t for t in range(nt)]
    ids = eng.hll_resolve(names)
    rng = np.random.default_rng(23)
    nb = 2 + 4 * steps   # warm, then fresh batches for each timing pass (a re-applied batch raises no register)
    kid = rng.integers(0, nt, B * nb)
    d_ids = eng.to_device(ids[kid].astype(np.uint32))
    off, byt, tot = eng.gen_jackson_longs_dev(0x5EED0023, B * nb)
    d_out = eng.alloc(B)
    for s in range(2):   # warm
        eng.pfadd_dev(B, d_ids.ptr + s * B * 4, off.ptr + s * B * 8, byt, tot, d_out)
    def calls(first):
        for s in range(first, first + steps):
            eng.pfadd_dev(B, d_ids.ptr + s * B * 4, off.ptr + s * B * 8, byt, tot, d_out)
    # back to back, no host waits: host-timed, and device-timed by two HIP events around the whole run
    eng.set_async(True)
    eng.sync()
    t0 = time.perf_counter()
    eng.timer_record(0)
    calls(2)
    eng.timer_record(1)
    eng.sync()
    t = time.perf_counter() - t0
    eng.set_async(False)
    dev_ms = eng.timer_elapsed_ms(0, 1)
    t_sync = timed(eng, lambda: calls(2 + steps))       # each call waits for its replies
    sync_dev = 0.0                              # ... and its device time: two HIP events around each call
    for s_ in range(2 + 2 * steps, 2 + 3 * steps):
        eng.timer_record(2)
        eng.pfadd_dev(B, d_ids.ptr + s_ * B * 4, off.ptr + s_ * B * 8, byt, tot, d_out)
        eng.timer_record(3)
        sync_dev += eng.timer_elapsed_ms(2, 3)
    eng.prof_reset()                            # per-kernel times (events around each launch), a separate pass
    eng.prof_enable(True)
    eng.prof_only("pfp_hash,pfp_apply")
    calls(2 + 3 * steps)
    eng.sync()
    eng.prof_enable(False)
    eng.prof_only(None)
    k = {p: eng.prof_read(p) for p in ("pfp_hash", "pfp_apply")}
    n_c, ms_c = steps, dev_ms
    line({"metric": "C2 PFADD inserts/sec, one 1M-command RBatch per device call (100k uniform tenants)",
          "value": B * steps / t, "unit": "inserts/s",
          "config": {"workload": "c2u", "batch": B, "tenants": nt, "calls": steps},
          "device_inserts_per_s": B / (ms_c / n_c * 1e-3) if n_c else None,
          "device_ms_per_call": ms_c / n_c if n_c else None,
          "kernel_ms": {p: (v[1] / v[0] if v[0] else None) for p, v in k.items()},
          "synchronous_calls_inserts_per_s": B * steps / t_sync,
          "synchronous_calls_device_inserts_per_s": B * steps / (sync_dev * 1e-3),
          "note": "value: back-to-back async calls host-timed; device: two HIP events around the same run / calls; "
                  "kernel_ms: events around each launch in a separate pass"})


def c2zipf(eng, args):
    """SURVEY 8d C2 variant: 1M-command PFADD batches with Zipf(1.1) tenants (device-resident)."""
    B, steps, nt, G = 1 << 20, 10, 100_000, 64
    names = [b"tenant:%d:hll" % t for t in range(nt)]
    ids = eng.hll_resolve(names)
    rng = np.random.default_rng(22)
    nbat = steps + 1 + 2 * G    # batches: warm, steps, a warm group, the timed group
    kid = (np.minimum(rng.zipf(1.1, B * nbat), nt) - 1).astype(np.int64)
    d_ids = eng.to_device(ids[kid].astype(np.uint32))
    off, byt, tot = eng.gen_jackson_longs_dev(0x5EED0022, B * nbat)
    d_out = eng.alloc(B)
    eng.pfadd_dev(B, d_ids, off, byt, tot, d_out)            # warm
    eng.set_async(True)
    t = timed(eng, lambda: [eng.pfadd_dev(B, d_ids.ptr + s * B * 4, off.ptr + s * B * 8, byt, tot, d_out)
                            for s in range(1, steps + 1)])
    eng.set_async(False)
    t_sync = timed(eng, lambda: [eng.pfadd_dev(B, d_ids.ptr + s * B * 4, off.ptr + s * B * 8, byt, tot, d_out)
                                 for s in range(1, steps + 1)])
    d_out10 = eng.alloc(B * G)   # group commit: G fresh batches as one call (line schedule), as in bench.py's step
    g0 = steps + 1   # batches not applied yet: one group to warm the line schedule's scratch, then the timed one
    eng.pfadd_dev(B * G, d_ids.ptr + g0 * B * 4, off.ptr + g0 * B * 8, byt, tot, d_out10)
    g0 += G
    eng.prof_reset(); eng.prof_enable(True)
    t_g = timed(eng, lambda: eng.pfadd_dev(B * G, d_ids.ptr + g0 * B * 4, off.ptr + g0 * B * 8, byt, tot, d_out10))
    eng.prof_enable(False)
    g_ms = {p: eng.prof_read(p)[1] for p in ("pfl_hash", "pfl_part", "pfl_apply")}
    d_out10.free()
    top = float(np.bincount(kid[:B]).max()) / B
    # per-key PFCOUNT of every tenant (C2): the histogram kernel alone, and the whole RHyperLogLog.count path
    d_all = eng.to_device(ids)
    d_hist = eng.alloc(nt * 64 * 4)
    eng.prof_reset(); eng.prof_enable(True)
    t_h = timed(eng, lambda: eng.hll_histogram_dev(nt, d_all, d_hist), reps=3)
    eng.prof_enable(False)
    n_l, ms = eng.prof_read("hll_hist")
    k_ms = ms / max(n_l, 1)
    d_sum = eng.alloc(nt * 16)
    eng.prof_reset(); eng.prof_enable(True)
    timed(eng, lambda: eng.hll_sum_dev(nt, d_all, d_sum), reps=3)
    eng.prof_enable(False)
    n_s, ms_s = eng.prof_read("hll_sum")
    s_ms = ms_s / max(n_s, 1)
    t_c = timed(eng, lambda: eng.pfcount([[nm] for nm in names]))
    t_ci = timed(eng, lambda: eng.pfcount_ids(ids))                  # slab ids cached by the caller
    gbs = nt * SLAB / (k_ms * 1e-3) / 1e9
    line({"metric": "C2 Zipf(1.1) PFADD inserts/sec (1M-command batches, 100k tenants)", "value": B * steps / t,
          "unit": "inserts/s", "config": {"workload": "c2zipf", "batch": B, "tenants": nt, "zipf_s": 1.1,
                                          "hottest_tenant_share": top},
          "synchronous_calls_inserts_per_s": B * steps / t_sync,
          "group_commit_inserts_per_s": B * G / t_g, "group_commit_kernel_ms": g_ms,
          "group_commit_device_inserts_per_s": B * G / (sum(g_ms.values()) * 1e-3) if all(g_ms.values()) else None,
          "group_commit": "%d fresh 1M batches as one call (line schedule), host-timed after a warm group" % G,
          "pfcount_keys_per_s": nt / t_c, "pfcount_ids_keys_per_s": nt / t_ci, "hist_keys_per_s_host_timed": nt / t_h,
          "hll_hist": {"achieved_GBps": gbs, "frac": gbs / PEAK, "avg_launch_ms": k_ms,
                       "note": "64-bin histograms (sk_hll_histogram_dev; the redis >= 5 estimator's input)"},
          "roofline": {"kernel": "hll_sum (PFCOUNT, redis 3.x: exact register sums)", "bound": "hbm",
                       "achieved": nt * SLAB / (s_ms * 1e-3) / 1e9, "peak": PEAK, "unit": "GB/s",
                       "frac": nt * SLAB / (s_ms * 1e-3) / 1e9 / PEAK, "bytes_per_unit": SLAB,
                       "avg_launch_ms": s_ms}})


def c4(eng, args):
    nk, per = args.c4_keys, args.c4_per_key
    names = [b"t4:%d" % i for i in range(nk)]
    ids = eng.hll_resolve(names)
    chunk = 1 << 24
    total = nk * per
    d_out = eng.alloc(chunk)
    rng = np.random.default_rng(4)
    t_add = 0.0
    for s in range(0, total, chunk):
        m = min(chunk, total - s)
        off, byt, tot = eng.gen_jackson_longs_dev(0x5EED0004, m, first=s)
        d_ids = eng.to_device(ids[rng.integers(0, nk, m)].astype(np.uint32))
        t_add += timed(eng, lambda: eng.pfadd_dev(m, d_ids, off, byt, tot, d_out))
        off.free(); byt.free(); d_ids.free()
    d_all = eng.to_device(ids)
    d_u = eng.alloc(16384)
    eng.prof_reset(); eng.prof_enable(True)
    t_u = timed(eng, lambda: eng.hll_union_dev(nk, d_all, d_u), reps=3)
    eng.prof_enable(False)
    n_l, ms = eng.prof_read("hll_union")
    k_ms = ms / max(n_l, 1)
    eng.hll_merge_registers_dev(b"t4:union", d_u)
    est = eng.pfcount([[b"t4:union"]])[0]
    gbs = nk * SLAB / (k_ms * 1e-3) / 1e9
    line({"metric": "C4 global union (countWith/PFMERGE) sources/sec, one GPU's shard", "value": nk / t_u,
          "unit": "sources/s", "config": {"workload": "c4", "keys": nk, "elements_per_key": per},
          "pfadd_inserts_per_s": total / t_add, "union_estimate": est,
          "roofline": {"kernel": "hll_union", "bound": "hbm", "achieved": gbs, "peak": PEAK, "unit": "GB/s",
                       "frac": gbs / PEAK, "bytes_per_unit": SLAB, "avg_launch_ms": k_ms}})


def c5(eng, args):
    bits = 1 << args.c5_log2_bits
    n = args.c5_ops
    rng = np.random.default_rng(5)
    chunk = 1 << 26
    keys = [b"bs5:%d" % i for i in range(4)]
    t_set = t_get = 0.0
    set_dev_ms = 0.0
    d_out = eng.alloc(chunk)
    # the cold form as well -- a first 64 M-op call on a key that does not exist yet, timed with the
    # string's creation and growth to full length inside the call (rounds <= 3 timed C5 this way)
    m0 = min(chunk, n)
    d_off = eng.to_device(rng.integers(0, bits, m0, dtype=np.uint64))
    t_cold = timed(eng, lambda: eng.setbit_dev(b"bs5:cold", m0, d_off, 1))
    d_off.free()
    eng.delete([b"bs5:cold"])
    eng.setbit([keys[0]], [bits - 1], [1])   # the string created at full length untimed (a 2 GiB allocation)
    for key in keys:
        for s in range(0, n if key == keys[0] else n // 16, chunk):
            m = min(chunk, n - s)
            d_off = eng.to_device(rng.integers(0, bits, m, dtype=np.uint64))
            if key == keys[0]:
                eng.prof_reset()
                eng.prof_enable(True)
            dt = timed(eng, lambda: eng.setbit_dev(key, m, d_off, 1))
            if key == keys[0]:
                eng.prof_enable(False)
                k_, ms_ = eng.prof_read("setbit")
                set_dev_ms += ms_ if k_ else 0.0
                t_set += dt
                t_get += timed(eng, lambda: eng.getbit_dev(key, m, d_off, d_out))
            d_off.free()
    # the C ABI the Java executors call: one 64 M-op RBatch run by key name from host buffers --
    # SETBIT_VOID (no reply array), SETBIT with replies, GETBIT -- host-timed (key scan, pageable H2D, kernels, replies)
    m = min(chunk, n)
    h_off = rng.integers(0, bits, m, dtype=np.uint64)
    kb_ = keys[0]
    koff = np.arange(m + 1, dtype=np.uint64) * np.uint64(len(kb_))
    kbuf = np.frombuffer(kb_ * m + b"\0" * 16, dtype=np.uint8)
    ones = np.ones(m, dtype=np.uint8)
    h_rep = np.zeros(m, dtype=np.uint8)
    eng.setbit_packed(koff, kbuf, h_off[:1024], ones[:1024])                      # warm the paths
    eng.setbit_packed(koff, kbuf, h_off[:1024], ones[:1024], h_rep[:1024])
    eng.prof_reset()
    eng.prof_enable(True)
    t_hv = timed(eng, lambda: eng.setbit_packed(koff, kbuf, h_off, ones))
    eng.prof_enable(False)
    k_, ms_ = eng.prof_read("setbit")
    hv_dev = ms_ / k_ if k_ else None
    eng.prof_reset()
    eng.prof_enable(True)
    t_hr = timed(eng, lambda: eng.setbit_packed(koff, kbuf, h_off, ones, h_rep))
    eng.prof_enable(False)
    k_, ms_ = eng.prof_read("setbit")
    hr_dev = ms_ / k_ if k_ else None
    t_hg = timed(eng, lambda: eng.getbit_packed(koff, kbuf, h_off, h_rep))
    host_path = {"ops_per_call": m, "setbit_void_per_s": m / t_hv, "setbit_void_device_per_s": m / (hv_dev * 1e-3)
                 if hv_dev else None, "setbit_replies_per_s": m / t_hr,
                 "setbit_replies_device_per_s": m / (hr_dev * 1e-3) if hr_dev else None, "getbit_per_s": m / t_hg,
                 "note": "sk_setbit / sk_getbit by key name from pageable host buffers (what SketchNative.setbit / getbit "
                         "pass): one key scan, the offsets' H2D, the kernels (SETBIT_VOID: k_sbv_part/fine/runs; with "
                         "replies: k_sbv_part<u64>/k_sbv_fine<u64>/k_sbr_runs), the replies' D2H; no library sort"}
    for key in keys[1:]:     # make every bitset full length (2^34 bits)
        eng.setbit([key], [bits - 1], [1])
    # host-timed (the call, its launch and the reply copy) and device-timed (HIP events around the kernel)
    def dev_ms(phase, fn, reps):
        eng.prof_reset()
        eng.prof_enable(True)
        t = timed(eng, fn, reps=reps)
        eng.prof_enable(False)
        k_, ms_ = eng.prof_read(phase)
        return t, (ms_ / k_ * 1e-3 if k_ else None)
    t_bc, d_bc = dev_ms("bitcount", lambda: eng.bitcount(keys[0]), 3)
    t_and, d_and = dev_ms("bitop", lambda: eng.bitop("AND", b"bs5:and", keys), 2)
    t_or, d_or = dev_ms("bitop", lambda: eng.bitop("OR", b"bs5:or", keys[:2]), 2)
    nbytes = bits // 8
    gbps = lambda b_, t_: b_ / t_ / 1e9 if t_ else None
    line({"metric": "C5 RBitSet 2^%d bits: SETBIT+GETBIT ops/sec" % args.c5_log2_bits,
          "value": 2 * n / (t_set + t_get), "unit": "ops/s",
          "config": {"workload": "c5", "bits": bits, "ops": n},
          "setbit_per_s": n / t_set, "getbit_per_s": n / t_get, "host_path": host_path,
          "setbit_device_per_s": n / (set_dev_ms * 1e-3) if set_dev_ms else None,
          "setbit_cold_first_call_per_s": m0 / t_cold,
          "setbit_cold": "one %d-op call on a missing key: the 2 GiB string's creation and growth timed inside it" % m0,
          "setbit": "SETBIT_VOID (RBitSet.set(i)) in 64 M-op calls on the full-length string (created untimed); a dense "
                    "call (>= 2 ops per 128-B line) takes the region path (partition by 32 KiB region: k_sbv_part + k_sbv_fine + k_sbv_runs)",
          "bitcount_GBps": nbytes / t_bc / 1e9, "bitop_and4_GBps": 5 * nbytes / t_and / 1e9,
          "bitop_or2_GBps": 3 * nbytes / t_or / 1e9,
          "device_GBps": {"bitcount": gbps(nbytes, d_bc), "bitop_and4": gbps(5 * nbytes, d_and),
                          "bitop_or2": gbps(3 * nbytes, d_or)},
          "roofline": {"kernel": "bitcount", "bound": "hbm", "achieved": gbps(nbytes, d_bc or t_bc), "peak": PEAK,
                       "unit": "GB/s", "frac": gbps(nbytes, d_bc or t_bc) / PEAK,
                       "host_timed_GBps": nbytes / t_bc / 1e9,
                       "note": "achieved: HIP events around the kernel (host-timed incl. launch and reply copy beside)"}})


def _dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)   # rendezvous only; data moves over RCCL
    return world, rank, dist


def c4mr(eng, args):
    from redisson_amd.cluster import RcclCollective, global_count_with, global_merge
    world, rank, dist = _dist()
    coll = RcclCollective(eng, rank, world, dist)
    nk, per = args.c4mr_keys, args.c4_per_key
    names = [b"t4:%d" % i for i in range(nk)]
    own = owners(names, world) == rank
    mine = [k for k, o in zip(names, own) if o]
    ids = eng.hll_resolve(mine)
    chunk, total = 1 << 24, len(mine) * per
    d_out = eng.alloc(chunk)
    rng = np.random.default_rng(40 + rank)
    t_add = 0.0
    for s in range(0, total, chunk):
        m = min(chunk, total - s)
        off, byt, tot = eng.gen_jackson_longs_dev(0x5EED0004, m, first=(rank << 40) + s)
        d_ids = eng.to_device(ids[rng.integers(0, len(mine), m)].astype(np.uint32))
        t_add += timed(eng, lambda: eng.pfadd_dev(m, d_ids, off, byt, tot, d_out))
        off.free(); byt.free(); d_ids.free()
    from redisson_amd.cluster import GlobalKeySet
    packed = pack(names)     # the key names as a client hands them over (one byte buffer + offsets)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    est_names = global_count_with(eng, packed, rank, world, coll)      # by names: resolve on every call
    t_names = time.perf_counter() - t0
    ks = GlobalKeySet(eng, packed, rank, world)
    t0 = time.perf_counter()
    ks.ids()                                                            # one-time: owner filter + directory
    t_resolve = time.perf_counter() - t0
    reps = 10
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):                                               # cached device slab ids
        est = global_count_with(eng, ks, rank, world, coll)
    t_cw = (time.perf_counter() - t0) / reps
    assert est == est_names and ks.resolves == 1
    t0 = time.perf_counter()
    global_merge(eng, b"t4:dest", ks, rank, world, coll)
    t_mg = time.perf_counter() - t0
    walls = coll.allgather_u64(int(t_cw * 1e9))
    walls_n = coll.allgather_u64(int(t_names * 1e9))
    if rank == 0:
        line({"metric": "C4 global countWith over %d tenant HLLs on %d GPUs (sources/sec, whole job)" % (nk, world),
              "value": nk / (max(walls) * 1e-9), "unit": "sources/s", "n_gpus": world, "scaling": "strong",
              "config": {"workload": "c4mr", "keys": nk, "elements_per_key": per, "partitioner": "calcSlot %% %d" % world},
              "countwith_estimate": est, "countwith_s": max(walls) * 1e-9, "pfmerge_s": t_mg,
              "countwith_by_names_s": max(walls_n) * 1e-9, "key_set_resolve_s_rank0": t_resolve,
              "pfadd_inserts_per_s_rank0": total / t_add,
              "note": "host-timed, mean of %d countWith calls over a GlobalKeySet (each rank's owned slab ids cached "
                      "on its device, re-resolved only when the HLL keyspace epoch moves): local union "
                      "(k_hll_union) + RCCL u8 MAX all-reduce + estimator; countwith_by_names_s resolves the 1M "
                      "names on every call" % reps})


def c5mr(eng, args):
    from redisson_amd.cluster import RcclCollective, ShardedBitSet, keyed_bitop
    world, rank, dist = _dist()
    coll = RcclCollective(eng, rank, world, dist)
    bits = 1 << args.c5_log2_bits
    a = ShardedBitSet(eng, b"bs5:a", bits, rank, world, coll)
    b = ShardedBitSet(eng, b"bs5:b", bits, rank, world, coll)
    n = args.c5_ops // world                 # ops submitted on this rank, offsets uniform over the whole bitset
    rng = np.random.default_rng(50 + rank)
    chunk = 1 << 26
    t_set = t_get = 0.0
    d_out = eng.alloc(chunk)
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        d_off = eng.to_device(rng.integers(0, bits, m, dtype=np.uint64))
        if dist:
            dist.barrier()
        t_set += timed(eng, lambda: a.set_dev(m, d_off, None, 1))     # SETBIT_VOID, routed to the owners
        t_get += timed(eng, lambda: a.get_dev(m, d_off, d_out))       # GETBIT, replies routed back
        d_off.free()
    hi_local = a.S * 8
    eng.setbit([b"bs5:a"], [min(hi_local, bits - rank * hi_local) - 1], [1])   # every shard full length
    eng.setbit([b"bs5:b"], [min(hi_local, bits - rank * hi_local) - 1], [1])
    if dist:
        dist.barrier()
    t0 = time.perf_counter(); card = a.cardinality(); t_bc = time.perf_counter() - t0
    t0 = time.perf_counter(); a.op("OR", [b]); t_or = time.perf_counter() - t0
    # two whole bitsets (1/16 of C5 each) owned by different GPUs: one all-gather + a local OR
    kb = 1 << (args.c5_log2_bits - 4)
    keys = [b"k5:%d" % i for i in range(64)]
    ka = next(k for k in keys if owner(k, world) == 0)
    kb_ = next(k for k in keys if owner(k, world) == (1 % world) and k != ka)
    for k in (ka, kb_):
        if owner(k, world) == rank:
            eng.setbit([k] * 2, [0, kb - 1], [1, 1])
    t0 = time.perf_counter(); nres = keyed_bitop(eng, "OR", b"k5:or", [ka, kb_], rank, world, coll)
    t_kor = time.perf_counter() - t0
    walls = coll.allgather_u64(int((t_set + t_get) * 1e9))
    if rank == 0:
        line({"metric": "C5 RBitSet 2^%d bits range-sharded over %d GPUs: SETBIT+GETBIT ops/sec (whole job)"
              % (args.c5_log2_bits, world), "value": 2 * n * world / (max(walls) * 1e-9), "unit": "ops/s",
              "n_gpus": world, "scaling": "weak", "config": {"workload": "c5mr", "bits": bits, "ops": n * world,
                                                            "shard_bytes": a.S},
              "setbit_per_s_rank0": n / t_set, "getbit_per_s_rank0": n / t_get,
              "bitcount_s": t_bc, "cardinality": card, "sharded_or_s": t_or,
              "keyed_or_bytes": nres, "keyed_or_s": t_kor,
              "note": "each rank submits its own ops (uniform over all 2^%d bits); ShardedBitSet.set_dev / get_dev "
                      "route them on the device (sk_route_bits), exchange them over RCCL (sk_alltoallv), apply "
                      "them on the owners and route GETBIT replies back (sk_unroute_u8); host-timed per 64M chunk. "
                      "BITCOUNT / OR / keyed OR host-timed including the collectives" % args.c5_log2_bits})


def host(eng, args):
    """The host-buffer C ABI (what the JNI shim calls): sk_pfadd / sk_bloom_add / sk_bloom_contains with caller-owned
    host arrays, so each call stages its inputs H2D and copies replies D2H (PCIe-inclusive; DESIGN 'Measurement').
    C2 shape (1M single-element PFADDs over 100k tenants, names resolved per call) and C3 shape (m=4,271,038,538,
    k=7, 1M adds then 1M contains, 50% members)."""
    from redisson_amd.engine import pack
    eng.flushall()
    B, reps, nt = 1 << 20, 4, 100_000
    rng = np.random.default_rng(33)
    names = [b"tenant:%d:hll" % t for t in range(nt)]
    eng.hll_resolve(names)                     # tenants exist (the steady state of C2)
    koff, kbuf = pack([names[t] for t in rng.integers(0, nt, B)])
    counts = np.ones(B, dtype=np.uint32)
    batches = [gen_jackson_longs(0x5EED0033 + r, B) for r in range(reps + 1)]
    out = np.zeros(B, dtype=np.uint8)
    lib, ctx = eng.lib, eng.ctx

    def pf(r):
        eoff, ebuf = batches[r]
        eng._check(lib.sk_pfadd(ctx, B, koff.ctypes.data, kbuf.ctypes.data, counts.ctypes.data, eoff.ctypes.data,
                                ebuf.ctypes.data, out.ctypes.data))
    pf(0)
    t_pf = timed(eng, lambda: [pf(r) for r in range(1, reps + 1)]) / reps
    kids = np.ascontiguousarray(eng.hll_resolve(names)[rng.integers(0, nt, B)], dtype=np.uint32)

    def pfi(r):  # the same batches with slab ids cached on the caller's side (sk_pfadd_ids)
        eoff, ebuf = batches[r]
        eng._check(lib.sk_pfadd_ids(ctx, B, kids.ctypes.data, counts.ctypes.data, eoff.ctypes.data,
                                    ebuf.ctypes.data, out.ctypes.data))
    pfi(0)
    t_pfi = timed(eng, lambda: [pfi(r) for r in range(1, reps + 1)]) / reps
    h2d_pf = koff.nbytes + kbuf.nbytes + counts.nbytes + batches[1][0].nbytes + batches[1][1].nbytes
    nm = b"bf:host"
    assert eng.bloom_try_init(nm, 425_000_000, 0.008)
    size, k, _, _ = eng.bloom_config(nm)

    def bl(fn, r):
        eoff, ebuf = batches[r]
        eng._check(fn(ctx, nm, len(nm), size, k, B, eoff.ctypes.data, ebuf.ctypes.data, out.ctypes.data))
    bl(lib.sk_bloom_add, 0)
    t_add = timed(eng, lambda: [bl(lib.sk_bloom_add, r) for r in range(1, reps + 1)]) / reps
    # contains: half of each batch re-probes added elements (the first half of batch r is batch r-1's)
    probe = []
    for r in range(1, reps + 1):
        a = [batches[r - 1][1][batches[r - 1][0][i]:batches[r - 1][0][i + 1]].tobytes() for i in range(B // 2)]
        b = [batches[r][1][batches[r][0][i]:batches[r][0][i + 1]].tobytes() for i in range(B // 2, B)]
        probe.append(pack(a + b))
    eoffs = [p_[0] for p_ in probe]

    def ct(r):
        eoff, ebuf = probe[r]
        eng._check(lib.sk_bloom_contains(ctx, nm, len(nm), size, k, B, eoff.ctypes.data, ebuf.ctypes.data,
                                         out.ctypes.data))
    ct(0)
    t_ct = timed(eng, lambda: [ct(r) for r in range(reps)]) / reps
    h2d_bl = eoffs[0].nbytes + probe[0][1].nbytes
    # group commit through the host ABI (what GpuBatchCoalescer sends): G RBatches of 1M one-element PFADDs as ONE
    # sk_pfadd_ids call over cached slab ids; pageable inputs go through HIP's own pageable copy (the library's pinned
    # double buffer is opt-in, SK_STAGE=1)
    G = 32
    gof, gbuf = gen_jackson_longs(0x5EED0034, B * G)
    gids = np.ascontiguousarray(eng.hll_resolve(names)[rng.integers(0, nt, B * G)], dtype=np.uint32)
    gcounts = np.ones(B * G, dtype=np.uint32)
    gout = np.zeros(B * G, dtype=np.uint8)

    def grp():
        eng._check(lib.sk_pfadd_ids(ctx, B * G, gids.ctypes.data, gcounts.ctypes.data, gof.ctypes.data,
                                    gbuf.ctypes.data, gout.ctypes.data))
    grp()
    t_grp = timed(eng, grp, reps=2)
    # the same group from pinned host buffers (sk_host_alloc: what the JNI side's direct ByteBuffers would be)
    pin = eng.host_alloc(gids.nbytes + gcounts.nbytes + gof.nbytes + gbuf.nbytes + 64)
    views, at = [], 0
    for a in (gids, gcounts, gof, gbuf):
        v = pin[at:at + a.nbytes].view(a.dtype)
        v[:] = a
        views.append(v)
        at += (a.nbytes + 15) // 16 * 16
    pids, pcnt, poff, pbuf = views

    def grp_pinned():
        eng._check(lib.sk_pfadd_ids(ctx, B * G, pids.ctypes.data, pcnt.ctypes.data, poff.ctypes.data,
                                    pbuf.ctypes.data, gout.ctypes.data))
    t_grp_pin = timed(eng, grp_pinned, reps=2)
    del views, pids, pcnt, poff, pbuf
    eng.host_free(pin)
    # the same PFADD batch with inputs already on the device (diagnostic: device share of the host path)
    dk, do_, db, dout = (eng.to_device(kids), eng.to_device(batches[1][0]), eng.to_device(batches[1][1], pad=16),
                         eng.alloc(B))
    t_dev = timed(eng, lambda: eng.pfadd_dev(B, dk, do_, db, int(batches[1][0][-1]), dout), reps=3)
    for x in (dk, do_, db, dout):
        x.free()
    # the prefix form (what the Java coalescers send for a codec's shared type header): the same batches with the
    # 18-byte Jackson Long header sent once and only the suffixes + u32 offsets per element
    plen = 18

    def suffix_form(eoff, ebuf):
        n_ = len(eoff) - 1
        mask = np.zeros(len(ebuf), dtype=bool)
        mask[(eoff[:-1, None].astype(np.int64) + np.arange(plen)).ravel()] = True
        mask[int(eoff[-1]):] = True
        sbuf = np.concatenate([ebuf[~mask], np.zeros(16, np.uint8)])
        soff = (eoff.astype(np.int64) - np.arange(n_ + 1) * plen).astype(np.uint32)
        return soff, sbuf
    preb = np.frombuffer(batches[1][1][int(batches[1][0][0]):int(batches[1][0][0]) + plen].tobytes(), np.uint8).copy()
    sforms = [suffix_form(*b) for b in batches]

    def pfx(r):
        soff, sbuf = sforms[r]
        eng._check(lib.sk_pfadd_ids_prefix(ctx, B, kids.ctypes.data, preb.ctypes.data, plen, soff.ctypes.data,
                                           sbuf.ctypes.data, out.ctypes.data))
    pfx(0)
    t_pfx = timed(eng, lambda: [pfx(r) for r in range(1, reps + 1)]) / reps
    gsoff, gsbuf = suffix_form(gof, gbuf)

    def grp_pfx():
        eng._check(lib.sk_pfadd_ids_prefix(ctx, B * G, gids.ctypes.data, preb.ctypes.data, plen, gsoff.ctypes.data,
                                           gsbuf.ctypes.data, gout.ctypes.data))
    grp_pfx()
    t_grp_pfx = timed(eng, grp_pfx, reps=2)
    pin = eng.host_alloc(gids.nbytes + gsoff.nbytes + gsbuf.nbytes + 64)
    views, at = [], 0
    for a in (gids, gsoff, gsbuf):
        v = pin[at:at + a.nbytes].view(a.dtype)
        v[:] = a
        views.append(v)
        at += (a.nbytes + 15) // 16 * 16
    pids, psoff, psbuf = views

    def grp_pfx_pinned():
        eng._check(lib.sk_pfadd_ids_prefix(ctx, B * G, pids.ctypes.data, preb.ctypes.data, plen, psoff.ctypes.data,
                                           psbuf.ctypes.data, gout.ctypes.data))
    t_grp_pfx_pin = timed(eng, grp_pfx_pinned, reps=2)
    del views, pids, psoff, psbuf
    eng.host_free(pin)
    pforms = [suffix_form(*p_) for p_ in probe]

    def ctp(r):
        soff, sbuf = pforms[r]
        eng._check(lib.sk_bloom_contains_prefix(ctx, nm, len(nm), size, k, B, preb.ctypes.data, plen,
                                                soff.ctypes.data, sbuf.ctypes.data, out.ctypes.data))
    ctp(0)
    t_ctp = timed(eng, lambda: [ctp(r) for r in range(reps)]) / reps
    # raw pageable H2D rate of one PFADD batch's element bytes (diagnostic for the rates above)
    raw = batches[1][1]
    t_h2d = timed(eng, lambda: eng.to_device(raw).free(), reps=3)
    line({"metric": "Host-buffer C ABI (PCIe-inclusive) PFADD + Bloom contains ops/sec",
          "value": 2 * B / (t_pfi + t_ct), "unit": "ops/s",
          "config": {"workload": "host", "batch": B, "tenants": nt, "bloom_bits": size, "bloom_k": k},
          "pfadd_host_per_s": B / t_pf, "pfadd_ids_host_per_s": B / t_pfi,
          "group_commit_ids_host_per_s": B * G / t_grp, "group_commit_ids_pinned_per_s": B * G / t_grp_pin,
          "group_commit": "%d RBatches of 1M PFADDs as one sk_pfadd_ids call (host buffers, cached slab ids; the "
                          "pinned: the same inputs in sk_host_alloc memory)" % G,
          "pfadd_ids_ms_per_batch": t_pfi * 1e3,
          "prefix_form": "the same inputs with the 18-B Jackson Long header sent once (sk_pfadd_ids_prefix, "
                         "sk_bloom_contains_prefix): suffixes + u32 offsets cross the link",
          "pfadd_ids_prefix_host_per_s": B / t_pfx, "pfadd_ids_prefix_ms_per_batch": t_pfx * 1e3,
          "group_commit_prefix_host_per_s": B * G / t_grp_pfx, "group_commit_prefix_pinned_per_s": B * G / t_grp_pfx_pin,
          "bloom_contains_prefix_host_per_s": B / t_ctp, "bloom_add_host_per_s": B / t_add, "bloom_contains_host_per_s": B / t_ct,
          "pfadd_ms_per_batch": t_pf * 1e3, "bloom_contains_ms_per_batch": t_ct * 1e3,
          "pfadd_h2d_bytes": int(h2d_pf), "pageable_h2d_GBps": raw.nbytes / t_h2d / 1e9,
          "pfadd_dev_ms_per_batch": t_dev * 1e3, "contains_h2d_bytes": int(h2d_bl),
          "note": "synchronous calls, inputs in pageable host memory, replies copied back; value = sk_pfadd_ids (ids cached by the caller) + sk_bloom_contains; pfadd_host_per_s resolves names per call"})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c2u,c2zipf,c4,c5,host")
    ap.add_argument("--c1-n", type=int, default=1 << 20)
    ap.add_argument("--c4-keys", type=int, default=125_000)       # 1M keys / 8 GPUs
    ap.add_argument("--c4-per-key", type=int, default=1000)
    ap.add_argument("--c4mr-keys", type=int, default=1_000_000)   # C4 as stated, sharded over the ranks
    ap.add_argument("--c5-log2-bits", type=int, default=34)
    ap.add_argument("--c5-ops", type=int, default=1 << 28)
    args = ap.parse_args()
    cfgs = args.configs.split(",")
    cap = args.c4_keys + 64
    if "c4mr" in cfgs:
        cap = max(cap, args.c4mr_keys // int(os.environ.get("WORLD_SIZE", "1")) + 4096)
    eng = SketchEngine(device=int(os.environ.get("LOCAL_RANK", "0")), max_bit_offset=1 << 36,
                       hll_capacity=cap, max_batch=1 << 24)
    for c in cfgs:
        {"c1": c1, "c2u": c2u, "c2zipf": c2zipf, "c4": c4, "c5": c5, "host": host, "c4mr": c4mr, "c5mr": c5mr}[c](eng, args)
    eng.close()


if __name__ == "__main__":
    main()
