"""Summarize SQ / LDS / atomic counter passes (tools/r03_sq.sh, tools/r03_lds.sh) into one committed file.

Inputs: DIR/sq*/pmc_means.json and DIR/lds*/pmc_means.json (per-kernel mean counter value per dispatch, from
tools/pmc_reduce.py) and a rocprofv3 kernel-stats CSV for the dispatch durations.  Per kernel it derives:
  wave-cycle split   SQ_ACTIVE_INST_ANY / SQ_WAIT_INST_ANY / SQ_WAIT_ANY over SQ_WAVE_CYCLES (disjoint buckets,
                     MI355X_MICROARCH.md "rocprofv3 PMC slots")
  valu_util          SQ_ACTIVE_INST_VALU x 4 (quad-cycles -> cycles) / (1024 SIMDs x dispatch cycles)
  lds_util           SQ_LDS_IDX_ACTIVE / (256 CUs x dispatch cycles): the LDS array's busy fraction (rocprofv3's
                     LdsUtil); dispatch cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) when collected, else
                     duration x the nominal clock
  lds_conflict       SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE: the share of LDS-array cycles lost to bank conflicts
  lds_atomic_rate    SQ_INSTS_LDS_ATOMIC wave-instructions per second and x64 lane-ops per second, against the LDS
                     array's peak for 32-bit accesses (2 LDS cycles per wave-instruction, 256 CUs)
  global atomics     TCC_ATOMIC (L2 atomic requests) per second
usage: python profiles/sq_summary.py DIR[,DIR...] TAG STATS_CSV [--clock-ghz 2.1]
"""
import csv
import glob
import json
import os
import sys

CUS, SIMDS = 256, 1024


def main(d, tag, stats_csv, clock_ghz=2.1):
    means = {}
    # directories in the given order, later ones overriding a counter both collected (the newer build's pass last)
    for f in sum((sorted(glob.glob(os.path.join(x, "*", "pmc_means.json"))) for x in d.split(",")), []):
        for k, cs in json.load(open(f)).items():
            means.setdefault(k, {}).update({c: v for c, v in cs.items() if c != "dispatches"})
    dur = {}
    for r in csv.DictReader(open(stats_csv)):
        dur[r["Name"].split("(")[0].replace("void ", "")] = float(r["AverageNs"]) * 1e-9
    out = {}
    for k, c in sorted(means.items()):
        if not k.startswith("sk::") or k not in dur:
            continue
        t = dur[k]
        cyc = c["GRBM_GUI_ACTIVE"] / 8 if "GRBM_GUI_ACTIVE" in c else t * clock_ghz * 1e9
        e = {"ms": t * 1e3, "dispatch_cycles": cyc, "counters": {n: round(v) for n, v in c.items()}}
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            e["wave_cycles_active"] = c.get("SQ_ACTIVE_INST_ANY", 0) / wc
            e["wave_cycles_wait_inst"] = c.get("SQ_WAIT_INST_ANY", 0) / wc
            e["wave_cycles_parked"] = c.get("SQ_WAIT_ANY", 0) / wc
        if "SQ_ACTIVE_INST_VALU" in c:
            e["valu_util"] = c["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * cyc)
        if "SQ_LDS_IDX_ACTIVE" in c:
            e["lds_util"] = c["SQ_LDS_IDX_ACTIVE"] / (CUS * cyc)
            if "SQ_LDS_BANK_CONFLICT" in c:
                e["lds_conflict_share"] = c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1)
        if "SQ_INSTS_LDS_ATOMIC" in c:
            rate = c["SQ_INSTS_LDS_ATOMIC"] / t
            e["lds_atomic_wave_instr_per_s"] = rate
            e["lds_atomic_lane_ops_per_s"] = rate * 64
            e["lds_atomic_frac_of_peak"] = rate / (CUS * clock_ghz * 1e9 / 2)
        if "TCC_ATOMIC" in c:
            e["l2_atomics_per_s"] = c["TCC_ATOMIC"] / t
        out[k] = e
    res = {"source": d, "stats": stats_csv, "clock_ghz_nominal": clock_ghz,
           "peaks": {"lds_array": "256 CUs x 128 B/clk (ds_read_b32 / 32-bit atomics: 2 LDS cycles per "
                                  "wave-instruction)", "valu": "1024 SIMDs"},
           "kernels": out}
    json.dump(res, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), f"{tag}_sq_summary.json"), "w"),
              indent=1)
    for k, e in out.items():
        print("%-30s %7.3f ms  active %.2f wait_inst %.2f parked %.2f  valu %s  lds %s  confl %s  lds-atomic %s" % (
            k[4:34], e["ms"], e.get("wave_cycles_active", 0), e.get("wave_cycles_wait_inst", 0),
            e.get("wave_cycles_parked", 0), fmt(e.get("valu_util")), fmt(e.get("lds_util")),
            fmt(e.get("lds_conflict_share")), fmt(e.get("lds_atomic_frac_of_peak"))))


def fmt(x):
    return "-" if x is None else "%.3f" % x


if __name__ == "__main__":
    a = [x for x in sys.argv[1:] if not x.startswith("--")]
    ck = float(sys.argv[sys.argv.index("--clock-ghz") + 1]) if "--clock-ghz" in sys.argv else 2.1
    main(a[0], a[1], a[2], ck)
