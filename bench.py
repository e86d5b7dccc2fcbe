#!/usr/bin/env python3
"""bench.py -- HLL inserts/s + Bloom contains/s (whole node) on the MI355X sketch engine.

One "step" = one RBatch-sized batch of PFADD (C2: 100k tenants, Jackson-encoded
random Longs, one element per command, 1M commands) + one batch of Bloom
contains (C3: tryInit(425,000,000, 0.008) -> m = 4,271,038,538 bits, k = 7,
50 % members / 50 % fresh, 1M elements), both with inputs already resident in
HBM.  value = (PFADD elements + contains elements) / wall time, all ranks.

Multi-GPU (torch.distributed.run, one process per GPU): keys are partitioned by
calcSlot(key) % world (the north-star partitioner), each rank owns its tenants
and its own Bloom filter, no data-path collective -> "scaling": "weak".
Rendezvous / barrier / max-over-ranks timing use torch.distributed's gloo (CPU)
backend: the engine owns the GPU through the system HIP runtime, so this
process never initialises torch's bundled HIP runtime.
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

from redisson_amd import SketchEngine, device_count, owner  # noqa: E402

PROF_STEPS = 5          # steps in each per-kernel breakdown pass (outside the timed region)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# in-library event-timed phases (sk_prof_*): one kernel each, except pfadd_sort
# (rocPRIM onesweep passes); only the path in use has launches
HLL_PHASES = ["pfp_hash", "pfp_apply", "pfp_reply",
              "pfadd_claim", "pfadd_commit", "pfadd_hash", "pfadd_sort", "pfadd_apply"]
PHASES = HLL_PHASES + ["bloom_contains"]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if world > 1:
        import torch.distributed as dist  # gloo only: CPU-side rendezvous / barrier / max

        dist.init_process_group("gloo", rank=rank, world_size=world)
        pg = dist
    return world, rank, local, pg


def barrier(pg):
    if pg is not None:
        pg.barrier()


def allmax(pg, x: float) -> float:
    if pg is None:
        return x
    import torch

    t = torch.tensor([x], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 20, help="commands per PFADD / contains batch")
    ap.add_argument("--tenants", type=int, default=100_000)
    ap.add_argument("--bloom-n", type=int, default=425_000_000)
    ap.add_argument("--bloom-p", type=float, default=0.008)
    ap.add_argument("--bloom-fill", type=int, default=-1, help="elements added before contains (default bloom-n)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=2_000_000)
    args = ap.parse_args()

    world, rank, local, pg = dist_setup()
    B, K, W = args.batch, args.steps, args.warmup
    fill = args.bloom_n if args.bloom_fill < 0 else args.bloom_fill

    # ------------------------------------------------------------ setup (untimed)
    names = ["tenant:%d:hll" % t for t in range(args.tenants)]
    mine = [nm for nm in names if owner(nm, world) == rank]
    ndev = max(device_count(), 1)   # one rank per GPU; rehearsals with more ranks than GPUs share devices
    eng = SketchEngine(device=local % ndev, hll_capacity=len(mine) + 16, max_batch=max(8 * B, 1 << 22),
                       max_bit_offset=1 << 34)
    ids = eng.hll_resolve(mine)
    rng = np.random.default_rng(0x5EED0002 + rank)

    nsteps = W + K + 2 * PROF_STEPS   # warmup, isolated breakdown, overlapped breakdown, timed: fresh inputs each
    seed_h = 0x5EED0002
    base_h = rank << 40                      # disjoint element streams per rank
    h_off, h_bytes, h_total = eng.gen_jackson_longs_dev(seed_h, nsteps * B, first=base_h)
    kid = rng.integers(0, len(mine), nsteps * B)
    d_ids = eng.to_device(ids[kid].astype(np.uint32))
    d_changed = eng.alloc(B)
    mean_len_h = h_total / (nsteps * B)

    bloom = "bloom:c3:%d" % rank
    eng.bloom_try_init(bloom, args.bloom_n, args.bloom_p)
    size, k, _, _ = eng.bloom_config(bloom)
    seed_b = 0x5EED0003
    chunk = 1 << 23
    d_add_out = eng.alloc(chunk)
    add_s = 0.0      # the add batches only (input generation excluded), host-timed around each call
    for s in range(0, fill, chunk):
        n = min(chunk, fill - s)
        a_off, a_bytes, a_tot = eng.gen_jackson_longs_dev(seed_b, n, first=(rank << 40) + s)
        eng.sync()
        t0 = time.perf_counter()
        eng.bloom_add_dev(bloom, n, a_off, a_bytes, a_tot, d_add_out)
        eng.sync()
        add_s += time.perf_counter() - t0
        a_off.free()
        a_bytes.free()
    # contains inputs: 50 % members, 50 % fresh
    member = rng.integers(0, max(fill, 1), nsteps * B, dtype=np.uint64) + np.uint64(rank << 40)
    fresh = rng.integers(1 << 39, 1 << 40, nsteps * B, dtype=np.uint64) + np.uint64(rank << 40)
    pick = rng.random(nsteps * B) < 0.5
    idx = np.where(pick, member, fresh)
    d_idx = eng.to_device(idx)
    c_off, c_bytes, c_total = eng.gen_jackson_longs_dev(seed_b, nsteps * B, d_idx=d_idx)
    d_idx.free()
    d_contains = eng.alloc(B)
    mean_len_b = c_total / (nsteps * B)
    log(f"[rank {rank}] setup: {len(mine)} tenants, bloom m={size} k={k} filled with {fill} in {add_s:.1f}s")

    def step(s):
        eng.pfadd_dev(B, d_ids.ptr + s * B * 4, h_off.ptr + s * B * 8, h_bytes, h_total, d_changed)
        eng.bloom_contains_dev(bloom, B, c_off.ptr + s * B * 8, c_bytes, c_total, d_contains)

    P = PROF_STEPS
    for s in range(W):
        step(s)
    eng.sync()

    def profiled(first, mode_async):
        """Per-phase device time over P fresh steps (every launch event-timed)."""
        eng.set_async(mode_async)
        eng.prof_only(None)
        eng.prof_reset()
        eng.prof_enable(True)
        for s in range(first, first + P):
            step(s)
        eng.sync()
        eng.prof_enable(False)
        eng.set_async(False)
        r = {p: eng.prof_read(p) for p in PHASES}
        return {p: r[p][1] / r[p][0] for p in PHASES if r[p][0]}

    # each kernel alone (sync mode: PFADD and contains do not overlap): the dominant
    # kernel is the one with the most device time of its own (overlapped launch times
    # mostly measure contention, and PFADD's apply and contains run neck and neck there)
    iso_ms = profiled(W, False)
    dom = max([p for p in iso_ms if p != "pfadd_sort"], key=lambda p: iso_ms[p])
    # breakdown as in the timed region (PFADD on the main stream, contains on the
    # read stream, no host sync)
    over_ms = profiled(W + P, True)

    # ------------------------------------------------------------ timed region
    # async: PFADD batches never wait on the host; only `dom` is event-timed
    T0 = W + 2 * P
    eng.set_async(True)
    eng.prof_only(dom)
    eng.prof_reset()
    eng.prof_enable(True)
    barrier(pg)
    eng.sync()
    t0 = time.perf_counter()
    eng.timer_record(0)
    for s in range(T0, T0 + K):
        step(s)
    eng.timer_record(1)
    eng.sync()
    t1 = time.perf_counter()
    barrier(pg)
    eng.prof_enable(False)
    eng.prof_only(None)
    eng.set_async(False)
    wall = allmax(pg, t1 - t0)
    dev_ms = eng.timer_elapsed_ms(0, 1)
    n_launch, tot_ms = eng.prof_read(dom)

    units = 2 * B * K * world
    value = units / wall
    # roofline of the dominant kernel: algorithmic bytes per unit x units / avg launch time
    per_unit = per_unit_of(dom, mean_len_h, mean_len_b, k)
    avg_ms = tot_ms / max(n_launch, 1)
    achieved = per_unit * B / (avg_ms * 1e-3) / 1e9

    hll_ms = sum(v for p, v in iso_ms.items() if p in HLL_PHASES)
    bl_ms = iso_ms["bloom_contains"]
    iso_dom_ms = iso_ms[dom]
    iso_achieved = per_unit_of(dom, mean_len_h, mean_len_b, k) * B / (iso_dom_ms * 1e-3) / 1e9
    traffic = pmc_traffic(dom)
    iso_traffic = traffic
    # every kernel of the step: algorithmic GB/s alone and in the overlapped schedule
    kernels = {}
    for p_, ms in iso_ms.items():
        if p_ == "pfadd_sort":
            continue
        pu = per_unit_of(p_, mean_len_h, mean_len_b, k)
        tr = pmc_traffic(p_)
        kernels[p_] = {"bytes_per_unit": pu, "ms_isolated": ms, "GBps_isolated": pu * B / (ms * 1e-3) / 1e9,
                       "ms_overlapped": over_ms.get(p_),
                       "GBps_overlapped": pu * B / (over_ms[p_] * 1e-3) / 1e9 if over_ms.get(p_) else None,
                       "pmc_traffic_bytes": tr,
                       "pmc_GBps_isolated": tr / (ms * 1e-3) / 1e9 if tr else None}
    # measured HBM-side bytes of every kernel of a step (PMC summary) over the step's wall time
    step_tr = [pmc_traffic(p) for p in over_ms]
    step_traffic = sum(step_tr) if step_tr and all(t is not None for t in step_tr) else None
    step_bytes = B * (per_unit_of("bloom_contains", mean_len_h, mean_len_b, k) + (mean_len_h + 12 + 2.5))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(eng, args, h_off, h_bytes, ids, kid, len(mine), c_off, c_bytes, bloom, size, k, nsteps * B)

    out = {
        "metric": "HLL inserts/sec + Bloom contains/sec (whole node)",
        "value": value,
        "unit": "ops/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": wall / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/u64",
        "data": "synthetic: SplitMix64 Longs as Jackson bytes [\"java.lang.Long\",v] (mean %.1f B)" % mean_len_h,
        "config": {
            "workload": "C2 PFADD 1 elem/cmd over %d tenants + C3 Bloom contains (m=%d, k=%d, filled with %d, "
                        "50%% members), %d commands per batch each" % (args.tenants, size, k, fill, B),
            "batch": B, "tenants": args.tenants, "bloom_bits": size, "bloom_k": k, "bloom_fill": fill,
            "partitioner": "calcSlot(key) %% %d" % world,
        },
        # device-time rates of each chain run alone (roofline_isolated's launches), whole job
        "hll_inserts_per_s": B * world / (hll_ms * 1e-3) if hll_ms else None,
        "bloom_contains_per_s": B * world / (bl_ms * 1e-3) if bl_ms else None,
        "bloom_add_per_s": fill / add_s if add_s else None,
        "device_ms_timed_region": dev_ms,
        "kernel_ms_per_launch": over_ms,   # overlapped breakdown pass (same schedule as the timed region)
        "roofline": {"kernel": dom, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     # measured HBM-side bytes (PMC, 128-B lines per random probe) over the same launch time
                     "traffic_GBps": traffic / (avg_ms * 1e-3) / 1e9 if traffic else None,
                     "traffic_frac": traffic / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if traffic else None,
                     "traffic_source": "profiles/*_pmc_summary.json: 2 x FETCH_SIZE (gfx950) + WRITE_SIZE per launch",
                     "bytes_per_unit": per_unit, "units_per_launch": B, "avg_launch_ms": avg_ms,
                     "note": "avg launch of the dominant kernel, HIP events on its stream inside the timed region "
                             "(PFADD and Bloom contains overlap on two streams)"},
        "kernels": kernels,
        "roofline_isolated": {"kernel": dom, "achieved": iso_achieved, "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": iso_achieved / HBM_PEAK_GBS, "avg_launch_ms": iso_dom_ms,
                              "traffic_GBps": iso_traffic / (iso_dom_ms * 1e-3) / 1e9 if iso_traffic else None,
                              "kernel_ms_per_launch": iso_ms},
        "step_algorithmic_GBps": step_bytes * K * world / wall / 1e9,
        "step_traffic_bytes": step_traffic,
        "step_traffic_GBps": step_traffic * K * world / wall / 1e9 if step_traffic else None,
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()


def per_unit_of(phase, mean_len_h, mean_len_b, k):
    """Algorithmic bytes per unit (SURVEY 8d / DESIGN.md kernel table)."""
    return {
        "pfp_hash": mean_len_h + 8 + 4 + 8,            # key bytes + offset + slab id in, record out
        "pfp_apply": 8 + 64 + 64 + 1,                  # record + register sector load (R0) + store + reply
        "pfp_reply": 1 + 2 + 1,                        # chunk-order reply + chunk slot in, reply out
        "pfadd_claim": mean_len_h + 8 + 4 + 1 + 8,     # key bytes + offset + slab id + register in, record out
        "pfadd_commit": 8 + 1 + 1,                     # record in, register + reply out
        "pfadd_hash": mean_len_h + 8 + 4 + 8,          # key bytes + offset + slab id in, sort key out
        "pfadd_sort": 2 * 8 * 5,                       # 5 radix passes over 8-byte keys (read + write)
        "pfadd_apply": 8 + 64 + 64 + 1,                # sorted key + register sector RMW + reply byte
        "bloom_contains": mean_len_b + 8 + 1 + (k - 1) * 64,   # len + 9 + (k-1)*64 B
    }[phase]


def pmc_traffic(phase):
    """HBM bytes per launch of the phase's kernel from the newest committed PMC summary (or None)."""
    import glob

    kern = {"bloom_contains": "sk::k_bloom_contains", "pfadd_claim": "sk::k_pfadd_claim",
            "pfadd_commit": "sk::k_pfadd_commit", "pfp_hash": "sk::k_pfp_hash", "pfp_apply": "sk::k_pfp_apply",
            "pfp_reply": "sk::k_pfp_reply"}.get(phase)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json")))
    if not kern or not files:
        return None
    try:
        d = json.load(open(files[-1]))["kernels"].get(kern)
        return d["traffic_bytes_per_launch"] if d else None
    except (OSError, ValueError, KeyError):
        return None


def cpu_baseline(eng, args, h_off, h_bytes, ids, kid, n_keys, c_off, c_bytes, bloom, size, k, n_avail):
    """The oracle (CPU restatement) on bounded samples of the same workload: one core, and the whole host's
    CPU share (threads owning keys id % T, like one redis-server per core with client-side routing)."""
    from oracle import oracle as O

    T = int(os.environ.get("OMP_NUM_THREADS") or 0) or min(16, os.cpu_count() or 1)
    S1 = min(args.cpu_sample, n_avail)
    ST = min(args.cpu_sample * max(T // 2, 1), n_avail, 1 << 24)
    S = max(S1, ST)
    off = h_off.download(np.uint64, S + 1)
    buf = h_bytes.download(np.uint8, int(off[S]) + 16)
    ko = kid[:S].astype(np.uint32)
    t0 = time.perf_counter()
    _, r1 = O.HLLStore().pfadd_bulk(ko[:S1], off[:S1 + 1], buf, n_keys)
    th1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    _, rT = O.HLLStore().pfadd_bulk_mt(ko[:ST], off[:ST + 1], buf, n_keys, T)
    thT = time.perf_counter() - t0
    assert np.array_equal(r1[:min(S1, ST)], rT[:min(S1, ST)]), "threaded oracle PFADD differs"

    bits = O.BitString(0)
    full = eng.get(bloom) or b""
    bits.buf = np.frombuffer(full + b"\0" * 16, dtype=np.uint8).copy()
    bits.len.value = len(full)
    coff = c_off.download(np.uint64, S + 1)
    cbuf = c_bytes.download(np.uint8, int(coff[S]) + 16)
    t0 = time.perf_counter()
    c1 = bits.bloom_contains_raw(size, k, coff[:S1 + 1], cbuf)
    tb1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    cT = bits.bloom_contains_raw_mt(size, k, coff[:ST + 1], cbuf, T)
    tbT = time.perf_counter() - t0
    assert np.array_equal(c1[:min(S1, ST)], cT[:min(S1, ST)]), "threaded oracle contains differs"
    return {"value": 2 * ST / (thT + tbT), "unit": "ops/s", "cores": T,
            "kind": "port",
            "sample": "%d PFADD (same tenants/elements) + %d Bloom contains on the same filled filter, "
                      "oracle/sketch_oracle.c on %d host threads (oracle_mt.c: a thread owns the keys id %% %d, "
                      "contains split in ranges)" % (ST, ST, T, T),
            "hll_inserts_per_s": ST / thT, "bloom_contains_per_s": ST / tbT,
            "single_core": {"value": 2 * S1 / (th1 + tb1), "cores": 1, "sample": "%d PFADD + %d contains" % (S1, S1),
                            "hll_inserts_per_s": S1 / th1, "bloom_contains_per_s": S1 / tb1}}


if __name__ == "__main__":
    main()
