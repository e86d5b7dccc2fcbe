#!/usr/bin/env python3
"""bench.py -- HLL inserts/s + Bloom contains/s (whole node) on the MI355X sketch engine.

One "step" = HB RBatch-sized PFADD batches (C2: 100k tenants, Jackson-encoded random Longs, one element per
command, B = 1M commands each), group-committed G at a time into one device call (default: all HB, which the
engine applies with the line schedule), + one Bloom contains batch of CB elements (C3: tryInit(425,000,000,
0.008) -> m = 4,271,038,538 bits, k = 7, filled with the config's 1B adds, 50 % members / 50 % fresh), inputs
already resident in HBM.  Defaults: HB = 64, CB = 64M, so a step is 64M PFADD + 64M contains; every step's PFADD
elements are fresh.
value = (PFADD elements + contains elements) / wall time, all ranks.

Multi-GPU (torch.distributed.run, one process per GPU): HLL keys are partitioned by calcSlot(key) % world (the
north-star partitioner), each rank owns its tenants; the C3 Bloom filter is ONE logical filter replicated on every
GPU (identical 1B adds), each rank serving its share of the contains traffic (redisson_amd/cluster.py
ReplicatedBloom).  No data-path collective -> "scaling": "weak".  Rendezvous / barrier / max-over-ranks timing use torch.distributed's gloo (CPU) backend: the
engine owns the GPU through the system HIP runtime, so this process never initialises torch's bundled HIP runtime.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from redisson_amd import SketchEngine, device_count, owner  # noqa: E402

PROF_STEPS = 1          # steps in each per-kernel breakdown pass (outside the timed region)
C_POOL = 4              # distinct contains batches, used in turn (contains is read-only: repeats change no work)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# in-library event-timed phases (sk_prof_*): one kernel each, except the chains "pfadd" (every kernel of one
# PFADD batch) and "bloom_contains" (every kernel of one contains call), and pfadd_sort (rocPRIM passes)
HLL_KERNELS = ["pfp_hash", "pfp_apply", "pfp_reply", "pfl_hash", "pfl_part", "pfl_fill", "pfl_apply", "pfadd_claim",
               "pfadd_commit", "pfadd_hash", "pfadd_apply"]
BLOOM_KERNELS = ["bloom_rc_hash", "bloom_rc_probe"]
# the kernels each timed phase launches (the roofline label names them all)
PHASE_KERNELS = {"bloom_rc_hash": "k_bloom_rc_hash + k_rc_stranspose", "bloom_rc_probe": "k_bloom_rc_probe + k_bloom_rc_zero",
                 "pfl_part": "k_pfl_tot + k_pfl_region", "pfl_apply": "k_pfl_plan + k_pfl_apply"}
CHAINS = ["pfadd", "bloom_contains"]
# rocprof names of the kernels each phase launches (PMC / SQ summaries)
PMC_KERNELS = {"bloom_contains": "sk::k_bloom_contains", "pfadd_claim": "sk::k_pfadd_claim",
               "pfadd_commit": "sk::k_pfadd_commit", "pfp_hash": "sk::k_pfp_hash", "pfp_apply": "sk::k_pfp_apply",
               "pfp_reply": "sk::k_pfp_reply", "bloom_rc_hash": "sk::k_bloom_rc_hash<false>+sk::k_rc_stranspose",
               "pfl_hash": "sk::k_pfl_hash",
               "pfl_fill": "sk::k_pfl_fill", "pfl_apply": "sk::k_pfl_plan+sk::k_pfl_apply", "pfl_part": "sk::k_pfl_tot+sk::k_pfl_region",
               "bloom_rc_probe": "sk::k_bloom_rc_probe_p|sk::k_bloom_rc_probe+sk::k_bloom_rc_zero"}
PHASES = HLL_KERNELS + ["pfadd_sort"] + BLOOM_KERNELS + CHAINS


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if world > 1:
        import torch.distributed as dist  # gloo only: CPU-side rendezvous / barrier / max

        # gloo prints its peer-connection notice on the C-level stdout: send it to stderr, so that rank 0's stdout
        # carries the one JSON line the driver parses
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1 << 20, help="commands per PFADD RBatch (C2: 1M)")
    ap.add_argument("--hll-batches", type=int, default=64, help="PFADD RBatches per step")
    ap.add_argument("--group", type=int, default=0,
                    help="RBatches group-committed per sk_pfadd_dev call (0 = all of a step's; 1 = one call each)")
    ap.add_argument("--contains-batch", type=int, default=64 << 20, help="Bloom contains elements per step")
    ap.add_argument("--tenants", type=int, default=100_000)
    ap.add_argument("--bloom-n", type=int, default=425_000_000)
    ap.add_argument("--bloom-p", type=float, default=0.008)
    ap.add_argument("--bloom-fill", type=int, default=1_000_000_000, help="elements added before contains (C3: 1B)")
    ap.add_argument("--add-chunk", type=int, default=1 << 25, help="elements per Bloom add call of the fill")
    ap.add_argument("--overlap", action="store_true",
                    help="contains on the engine's read stream beside the PFADD stream (default: one stream, chains "
                         "back to back -- overlapping them gains ~2 %% and makes each chain's launch time measure "
                         "the contention)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=2_000_000)
    args = ap.parse_args()

    world, rank, local, pg = dist_setup()
    if not args.overlap:
        os.environ["SK_READ_STREAM"] = "0"   # contains on the main stream: the chains run back to back
    B, HB, CB, K, W = args.batch, args.hll_batches, args.contains_batch, args.steps, args.warmup
    G = args.group if args.group > 0 else HB   # RBatches per device call (group commit)
    assert HB % G == 0, "--hll-batches must be a multiple of --group"
    fill = args.bloom_fill

    # ------------------------------------------------------------ setup (untimed)
    t_setup = time.perf_counter()
    names = ["tenant:%d:hll" % t for t in range(args.tenants)]
    mine = [nm for nm in names if owner(nm, world) == rank]
    ndev = max(device_count(), 1)   # one rank per GPU; rehearsals with more ranks than GPUs share devices
    eng = SketchEngine(device=local % ndev, hll_capacity=len(mine) + 16, max_batch=max(8 * B, 1 << 22),
                       max_bit_offset=1 << 34)
    ids = eng.hll_resolve(mine)
    rng = np.random.default_rng(0x5EED0002 + rank)

    nsteps = W + K + 2 * PROF_STEPS   # warmup, isolated breakdown, overlapped breakdown, timed: fresh inputs each
    NH = HB * B                       # PFADD elements per step
    seed_h = 0x5EED0002
    # PFADD inputs, one device buffer set per step: element stream of this rank (disjoint per rank)
    h_in = []
    h_total = 0
    kid_all = []
    for s in range(nsteps):
        off, byt, tot = eng.gen_jackson_longs_dev(seed_h, NH, first=(rank << 40) + s * NH)
        kid = rng.integers(0, len(mine), NH)
        kid_all.append(kid if s == 0 else None)
        d_ids = eng.to_device(ids[kid].astype(np.uint32))
        h_in.append((off, byt, tot, d_ids))
        h_total += tot
    d_changed = eng.alloc(G * B)
    mean_len_h = h_total / (nsteps * NH)

    # ONE logical C3 filter for the whole node: every rank holds an identical replica (the same 1B adds), and the
    # contains traffic is split over the replicas (cluster.ReplicatedBloom's layout); at N = 1 it is the filter
    bloom = "bloom:c3"
    eng.bloom_try_init(bloom, args.bloom_n, args.bloom_p)
    size, k, _, _ = eng.bloom_config(bloom)
    seed_b = 0x5EED0003
    chunk = args.add_chunk
    d_add_out = eng.alloc(chunk)
    add_s = 0.0      # the add batches only (input generation excluded), host-timed around each call
    for s in range(0, fill, chunk):
        n = min(chunk, fill - s)
        a_off, a_bytes, a_tot = eng.gen_jackson_longs_dev(seed_b, n, first=s)
        eng.sync()
        t0 = time.perf_counter()
        eng.bloom_add_dev(bloom, n, a_off, a_bytes, a_tot, d_add_out)
        eng.sync()
        add_s += time.perf_counter() - t0
        a_off.free()
        a_bytes.free()
    # contains inputs: 50 % members (drawn from the fill), 50 % fresh
    c_in = []
    c_total = 0
    for s in range(min(nsteps, C_POOL)):
        member = rng.integers(0, max(fill, 1), CB, dtype=np.uint64)
        fresh = rng.integers(1 << 39, 1 << 40, CB, dtype=np.uint64) + np.uint64(rank << 40)
        idx = np.where(rng.random(CB) < 0.5, member, fresh)
        d_idx = eng.to_device(idx)
        off, byt, tot = eng.gen_jackson_longs_dev(seed_b, CB, d_idx=d_idx)
        d_idx.free()
        c_in.append((off, byt, tot))
        c_total += tot
    d_contains = eng.alloc(CB)
    mean_len_b = c_total / (len(c_in) * CB)
    log(f"[rank {rank}] setup: {len(mine)} tenants, bloom m={size} k={k} filled with {fill} "
        f"(adds {add_s:.2f}s), {nsteps} steps of {HB}x{B} PFADD + {CB} contains, {time.perf_counter() - t_setup:.0f}s")

    def step(s):
        off, byt, tot, d_ids = h_in[s]
        for h in range(0, HB, G):
            eng.pfadd_dev(G * B, d_ids.ptr + h * B * 4, off.ptr + h * B * 8, byt, tot, d_changed)
        off, byt, tot = c_in[s % len(c_in)]
        eng.bloom_contains_dev(bloom, CB, off, byt, tot, d_contains)

    P = PROF_STEPS
    for s in range(W):
        step(s)
    eng.sync()

    def profiled(first, mode_async):
        """Per-phase device time over P fresh steps (every launch event-timed): {phase: (launches, ms)}."""
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
        return {p: (r[p][0] / P, r[p][1] / r[p][0]) for p in PHASES if r[p][0]}

    # each kernel alone (sync mode: PFADD and contains do not overlap).  The roofline unit is the chain (every
    # kernel of one PFADD batch / one contains call) with the most device time per step of its own: SURVEY 8(d)
    # prices whole operations (53 B per PFADD element, len + 9 + 64(k-1) per contains), not single kernels.
    # Overlapped launch times mostly measure contention.
    iso = profiled(W, False)
    kern = [p for p in iso if p not in CHAINS and p != "pfadd_sort"]
    if "bloom_rc_hash" not in iso:   # one-element-per-thread contains: the chain is one kernel
        kern.append("bloom_contains")
    dom_kernel = max(kern, key=lambda p: iso[p][0] * iso[p][1])
    dom = max([c for c in CHAINS if c in iso], key=lambda c: iso[c][0] * iso[c][1])
    chain_kernels = {"pfadd": [p for p in ("pfp_hash", "pfp_apply", "pfp_reply", "pfl_hash", "pfl_part", "pfl_fill",
                                         "pfl_apply")
                               if p in iso],
                     "bloom_contains": [p for p in BLOOM_KERNELS if p in iso] or ["bloom_contains"]}
    # breakdown as in the timed region (PFADD on the main stream, contains on the read stream, no host sync)
    over = profiled(W + P, True)

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
    t_enq = time.perf_counter() - t0   # host time to enqueue the K steps (the device may still be running)
    eng.sync()
    t1 = time.perf_counter()
    barrier(pg)
    eng.prof_enable(False)
    eng.prof_only(None)
    eng.set_async(False)
    wall = allmax(pg, t1 - t0)
    dev_ms = eng.timer_elapsed_ms(0, 1)
    n_launch, tot_ms = eng.prof_read(dom)   # chain events: the per-launch period

    units = (NH + CB) * K * world
    value = units / wall
    nr = (size + (1 << 20) - 1) >> 20
    bpu = per_unit_bytes(mean_len_h, mean_len_b, k, size, CB, nr, len(mine), G * B)
    upl = {"pfp_hash": B, "pfp_apply": B, "pfp_reply": B, "pfadd": G * B if G > 1 else B, "pfl_hash": G * B,
           "pfl_part": G * B, "pfl_fill": G * B, "pfl_apply": G * B, "bloom_contains": CB,
           "bloom_rc_hash": CB, "bloom_rc_probe": CB}
    # the chain's events span one launch of the chain in the steady state of the timed region (for PFADD: the
    # previous batch's apply end to this batch's apply end, i.e. the per-batch period; its hash overlaps the
    # previous apply on the other stream)
    avg_ms = tot_ms / max(n_launch, 1)
    # SURVEY 8(d) per-unit bytes of each chain (53 B per PFADD element at C2; len + 9 + 64(k-1) per contains)
    s8 = {"pfadd": mean_len_h + 12 + 2.5, "bloom_contains": mean_len_b + 8 + 1 + 64 * (k - 1)}
    # the schedule's own minimum HBM bytes per unit (a second roofline, DESIGN.md "Measurement"): what the chain
    # must move as built -- inputs, replies, its intermediate records written and read back, the register lines or
    # the bit array once per pass -- so that a chain which beats SURVEY 8(d)'s per-probe pricing still reads < 1
    lines = 128.0 * len(mine)
    touched = lines * (1.0 - math.exp(-(G * B) / lines))
    piece = min(CB, 32 << 20)                         # contains pieces of <= 32 M elements (sk_store.cpp)
    own = {"pfadd": mean_len_h + 8 + 4 + 1 + 4 * 8 + 2 * 96 * touched / (G * B),
           "bloom_contains": mean_len_b + 8 + 1 + 2 * 4 * (k - 1) + 2 * 4.0 * nr / 4096 + (size / 8.0) / piece}
    # PMC bytes per dispatch x dispatches of each kernel per launch of the chain (a 64 M contains call is two
    # 32 M pieces)
    tr_parts = [(pmc_traffic(p_), iso[p_][0] / iso[dom][0]) for p_ in chain_kernels[dom] if p_ in iso]
    traffic = sum(t * f for t, f in tr_parts) if tr_parts and all(t is not None for t, _ in tr_parts) else None
    # The headline roofline is the bytes the chain's kernels actually move (rocprofv3 FETCH/WRITE counters of this
    # build, per launch) over the chain's launch time measured here.  SURVEY 8(d) charges one random 64-B sector
    # per Bloom probe, which the region schedule never pays (probes are sorted into LDS-resident regions), so its
    # bytes over the same time are an "effective" bandwidth that can exceed the HBM peak; it is reported beside it.
    eff_gbs = s8[dom] * upl[dom] / (avg_ms * 1e-3) / 1e9
    if traffic:
        achieved, a_src = traffic / (avg_ms * 1e-3) / 1e9, "pmc"
    else:   # no counter summary for this build: the schedule's own minimum bytes
        achieved, a_src = own[dom] * upl[dom] / (avg_ms * 1e-3) / 1e9, "schedule_min"
    valu = sq_valu(dom_chain_kernel(dom, iso, chain_kernels))

    kernels = {}
    for p_, (lps, ms) in iso.items():
        if p_ == "pfadd_sort" or p_ in CHAINS:
            continue
        # units one launch processes: the step's units of the kernel's chain over its launches per step (a 64 M
        # contains call runs each region kernel on two 32 M pieces)
        u = (CB if p_.startswith("bloom") else NH) / lps
        tr = pmc_traffic(p_)
        kernels[p_] = {"line_bytes_per_unit": bpu.get(p_), "units_per_launch": u, "launches_per_step": lps,
                       "ms_isolated": ms, "GBps_isolated": bpu[p_] * u / (ms * 1e-3) / 1e9 if p_ in bpu else None,
                       "ms_overlapped": over.get(p_, (0, None))[1],
                       "pmc_traffic_bytes": tr,
                       "pmc_GBps_isolated": tr / (ms * 1e-3) / 1e9 if tr else None}
    # chains against SURVEY 8(d)'s per-unit figures
    chains = {}
    for ch in CHAINS:
        if ch not in iso:
            continue
        lps, ms = iso[ch]
        u = upl[ch]
        chains[ch] = {"s8d_bytes_per_unit": s8[ch], "units_per_launch": u, "ms_isolated": ms,
                      "units_per_s_isolated": u / (ms * 1e-3),
                      "s8d_GBps_isolated": s8[ch] * u / (ms * 1e-3) / 1e9,
                      "s8d_frac_isolated": s8[ch] * u / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                      "schedule_min_bytes_per_unit": own[ch],
                      "schedule_min_frac_isolated": own[ch] * u / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                      "ms_overlapped": over.get(ch, (0, None))[1]}
    hll_ms = iso["pfadd"][1] if "pfadd" in iso else None
    bl_ms = iso["bloom_contains"][1] if "bloom_contains" in iso else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        off, byt, _, _ = h_in[0]
        coff, cbyt, _ = c_in[0]
        cpu = cpu_baseline(eng, args, off, byt, ids, kid_all[0], len(mine), coff, cbyt, bloom, size, k,
                           min(NH, CB))

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
            "workload": "C2 PFADD 1 elem/cmd over %d tenants, %d RBatches of %d commands (group-committed %d per "
                        "device call) + C3 Bloom contains (m=%d, k=%d, filled with %d adds, 50%% members), %d elements, "
                        "per step and GPU; one C3 filter replicated on the %d GPU(s)"
                        % (args.tenants, HB, B, G, size, k, fill, CB, world),
            "pfadd_batch": B, "pfadd_batches_per_step": HB, "pfadd_batches_per_call": G, "contains_batch": CB,
            "tenants": args.tenants,
            "bloom_bits": size, "bloom_k": k, "bloom_fill": fill, "partitioner": "calcSlot(key) %% %d" % world,
        },
        # device-time rates of each chain run alone, whole job
        "hll_inserts_per_s": upl["pfadd"] * world / (hll_ms * 1e-3) if hll_ms else None,
        "bloom_contains_per_s": CB * world / (bl_ms * 1e-3) if bl_ms else None,
        "bloom_add_per_s": fill / add_s if add_s else None,
        "device_ms_timed_region": dev_ms,
        "host_enqueue_ms_per_step": t_enq / K * 1e3,
        "roofline": {"kernel": "%s chain (%s)" % (dom, " + ".join(PHASE_KERNELS.get(p_, "k_" + p_)
                                                                 for p_ in chain_kernels[dom])),
                     "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "achieved_source": a_src,
                     "traffic_source": "newest profiles/*_pmc_summary.json: 2 x FETCH_SIZE (gfx950) + WRITE_SIZE per "
                                       "dispatch, times dispatches per chain launch, summed over the chain's kernels",
                     "traffic_bytes_per_unit": traffic / upl[dom] if traffic else None,
                     "effective_GBps": eff_gbs, "effective_frac_s8d": eff_gbs / HBM_PEAK_GBS,
                     "effective_bytes_per_unit": s8[dom], "effective_bytes_source": "SURVEY 8(d) (one 64-B sector "
                     "per decisive probe; the region schedule does not pay it, so this can exceed the peak)",
                     "schedule_min_bytes_per_unit": own[dom],
                     "schedule_min_frac": own[dom] * upl[dom] / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "units_per_launch": upl[dom], "avg_launch_ms": avg_ms, "launches_timed": n_launch,
                     "kernel_ms_isolated": {p_: iso[p_][1] for p_ in chain_kernels[dom] if p_ in iso},
                     "kernel_ms_overlapped": {p_: over[p_][1] for p_ in chain_kernels[dom] if p_ in over},
                     "dominant_kernel": {"kernel": dom_kernel, "line_bytes_per_unit": bpu.get(dom_kernel),
                                         "ms_isolated": iso[dom_kernel][1],
                                         "launches_per_step": iso[dom_kernel][0]},
                     "valu_frac": valu,
                     "note": "frac = PMC bytes of the chain per launch / avg_launch_ms / 8 TB/s.  avg_launch_ms = HIP "
                             "events around each launch of the chain on its stream inside the timed region (PFADD: "
                             "the per-batch period); valu_frac = SQ_ACTIVE_INST_VALU x 4 cycles / (SIMDs x dispatch "
                             "cycles) of the chain's longest kernel from the newest profiles/*_sq_summary.json: an "
                             "upper bound on its VALU busy share, since gfx950 issues a wave64 integer add in 2 cycles "
                             "and a 32-bit multiply in ~3.5 (profiles/r05_mulrate.log); line-level bytes per kernel: "
                             "DESIGN.md kernel table"},
        "kernels": kernels,
        "chains": chains,
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()


def per_unit_bytes(mean_len_h, mean_len_b, k, size, CB, nr, tenants, group):
    """Algorithmic bytes per unit of each kernel (DESIGN.md kernel table).  Random probes / register lines are
    priced at one 64-B sector; streamed data at its bytes."""
    P = k - 1
    seg = 4.0 * nr / 4096            # segment table entry per hash block, per element
    lines = 128.0 * tenants          # 128-register lines (96 B packed) of the arena; a group of `group` elements touches
    touched = lines * (1.0 - math.exp(-group / lines))   # this many of them (uniform tenants)
    return {
        "pfl_hash": mean_len_h + 8 + 4 + 8,            # key bytes + offset + slab id in, record out
        "pfl_part": 8 + 8,                             # records read once and written once (tile-major region sort)
        "pfl_fill": 1,                                 # the default reply, streamed
        "pfl_apply": 6 + 2 * 96 * touched / group,     # 6-B record + each touched 96-B packed line in and out once
        "pfp_hash": mean_len_h + 8 + 4 + 8,            # key bytes + offset + slab id in, record out
        "pfp_apply": 8 + 64 + 64 + 1,                  # record + register sector load (R0) + store + reply
        "pfp_reply": 1 + 2 + 1,                        # chunk-order reply + chunk slot in, reply out
        "pfadd_claim": mean_len_h + 8 + 4 + 1 + 8,
        "pfadd_commit": 8 + 1 + 1,
        "pfadd_hash": mean_len_h + 8 + 4 + 8,
        "pfadd_apply": 8 + 64 + 64 + 1,
        "pfadd": mean_len_h + 12 + 2.5,                # SURVEY 8d PFADD element (53 B at C2)
        # contains, one element per thread: SURVEY 8d (len + 9 + 64 B per decisive probe)
        "bloom_contains": mean_len_b + 8 + 1 + 64 * P,
        # region schedule: key + offset in, reply out, probe records + segment entries out
        "bloom_rc_hash": mean_len_b + 8 + 1 + 4 * P + seg,
        # records + segment entries in, the bit array streamed once per batch
        "bloom_rc_probe": 4 * P + seg + (size / 8.0) / CB,
    }


def _summary_find(ks, k_):
    """a kernel's entry in a summary; template kernels may carry more arguments in newer builds; "a|b": the first of
    the alternatives the summary has (a kernel replaced by another form)"""
    if "|" in k_:
        for alt in k_.split("|"):
            d = _summary_find(ks, alt)
            if d:
                return d
        return None
    if k_ in ks:
        return ks[k_]
    stem = k_[:-1] + "," if k_.endswith(">") else k_ + "<"   # or a kernel that became a template
    hit = [v for n_, v in ks.items() if stem and n_.startswith(stem)]
    return hit[0] if len(hit) == 1 else None


def dom_chain_kernel(dom, iso, chain_kernels):
    """the phase of the chain with the most device time per chain launch"""
    ps = [p_ for p_ in chain_kernels[dom] if p_ in iso]
    return max(ps, key=lambda p_: iso[p_][0] * iso[p_][1]) if ps else None


def sq_valu(phase):
    """VALU busy fraction of the phase's first kernel from the newest committed SQ summary (or None)"""
    import glob

    if not phase or phase not in PMC_KERNELS:
        return None
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_sq_summary.json")))
    if not files:
        return None
    try:
        d = _summary_find(json.load(open(files[-1]))["kernels"], PMC_KERNELS[phase].split("+")[0])
        return {"kernel": PMC_KERNELS[phase].split("+")[0], "valu_frac": d["valu_util"],
                "lds_conflict_share": d.get("lds_conflict_share"),
                "valu_insts_per_dispatch": d["counters"]["SQ_INSTS_VALU"],
                "source": os.path.relpath(files[-1], ROOT)} if d else None
    except (OSError, ValueError, KeyError):
        return None


def pmc_traffic(phase):
    """HBM bytes per launch of the phase's kernel from the newest committed PMC summary (or None)."""
    import glob

    kern = PMC_KERNELS.get(phase)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json")))
    if not kern or not files:
        return None
    try:
        ks = json.load(open(files[-1]))["kernels"]

        parts = [_summary_find(ks, k_) for k_ in kern.split("+")]   # a phase of several launches: their sum
        return sum(d["traffic_bytes_per_launch"] for d in parts) if all(parts) else None
    except (OSError, ValueError, KeyError):
        return None


def host_cpu_info():
    """what the host offers the CPU baseline: nproc, the affinity mask, the cgroup CPU quota, the CPU model"""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity_cpus"] = None
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    info["cgroup_cpu_quota"] = quota
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    info["cpu_model"] = model
    return info


def cpu_baseline(eng, args, h_off, h_bytes, ids, kid, n_keys, c_off, c_bytes, bloom, size, k, n_avail):
    """The oracle (CPU restatement) on bounded samples of the same workload: one core, and the whole host -- one
    thread per CPU nproc reports (threads owning keys id % T, like one redis-server per core with client-side
    routing); the 16-thread figure (the box's CPU share per GPU) beside it."""
    from oracle import oracle as O

    host = host_cpu_info()
    T = int(os.environ.get("SK_CPU_THREADS") or 0) or (host["nproc"] or 1)
    S1 = min(args.cpu_sample, n_avail)
    ST = min(args.cpu_sample * 8, n_avail, 1 << 24)
    S = max(S1, ST)
    off = h_off.download(np.uint64, S + 1)
    buf = h_bytes.download(np.uint8, int(off[S]) + 16)
    ko = kid[:S].astype(np.uint32)
    bits = O.BitString(0)
    full = eng.get(bloom) or b""
    bits.buf = np.frombuffer(full + b"\0" * 16, dtype=np.uint8).copy()
    bits.len.value = len(full)
    coff = c_off.download(np.uint64, S + 1)
    cbuf = c_bytes.download(np.uint8, int(coff[S]) + 16)

    def timed(threads, n):
        t0 = time.perf_counter()
        _, r = O.HLLStore().pfadd_bulk_mt(ko[:n], off[:n + 1], buf, n_keys, threads)
        th = time.perf_counter() - t0
        t0 = time.perf_counter()
        c = bits.bloom_contains_raw_mt(size, k, coff[:n + 1], cbuf, threads)
        tb = time.perf_counter() - t0
        return th, tb, r, c

    t0 = time.perf_counter()
    _, r1 = O.HLLStore().pfadd_bulk(ko[:S1], off[:S1 + 1], buf, n_keys)
    th1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    c1 = bits.bloom_contains_raw(size, k, coff[:S1 + 1], cbuf)
    tb1 = time.perf_counter() - t0
    thT, tbT, rT, cT = timed(T, ST)
    assert np.array_equal(r1[:min(S1, ST)], rT[:min(S1, ST)]), "threaded oracle PFADD differs"
    assert np.array_equal(c1[:min(S1, ST)], cT[:min(S1, ST)]), "threaded oracle contains differs"
    # the process's CPU share: a cgroup quota below nproc (the GPU box gives a 1-GPU job 16 of its 256 CPUs) runs
    # nproc threads on quota CPUs' time, so the whole-host leg is also timed at the quota and the better of the two
    # is the baseline (both reported)
    legs = {T: (thT, tbT)}
    for t_ in {min(16, T), int(host["cgroup_cpu_quota"] or T)}:
        if t_ not in legs and 1 <= t_ <= T:
            legs[t_] = timed(t_, ST)[:2]
    best = min(legs, key=lambda t_: sum(legs[t_]))
    tb_h, tb_b = legs[best]
    return {"value": 2 * ST / (tb_h + tb_b), "unit": "ops/s", "cores": best,
            "kind": "port", "host": host,
            "sample": "%d PFADD (same tenants/elements) + %d Bloom contains on the same 1B-filled filter, "
                      "oracle/sketch_oracle.c on %d host threads (oracle_mt.c: commands routed once to the thread "
                      "owning key id %% threads, contains split in ranges); the best of %s threads (nproc %s, cgroup "
                      "quota %s CPUs)" % (ST, ST, best, sorted(legs), host["nproc"], host["cgroup_cpu_quota"]),
            "hll_inserts_per_s": ST / tb_h, "bloom_contains_per_s": ST / tb_b,
            "by_threads": {str(t_): {"value": 2 * ST / sum(v_), "hll_inserts_per_s": ST / v_[0],
                                     "bloom_contains_per_s": ST / v_[1]} for t_, v_ in sorted(legs.items())},
            "single_core": {"value": 2 * S1 / (th1 + tb1), "cores": 1, "sample": "%d PFADD + %d contains" % (S1, S1),
                            "hll_inserts_per_s": S1 / th1, "bloom_contains_per_s": S1 / tb1}}


if __name__ == "__main__":
    main()
