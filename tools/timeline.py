"""Timeline of the bench's timed region from a rocprofv3 kernel trace (dev tool).

usage: python tools/timeline.py TRACE.csv FIRST_STEP N_STEPS
Step s is the s-th pfp_hash / bloom_contains launch of the run (bench order: W warmup, P isolated, P breakdown,
K timed).  Prints each stream's busy time, idle gaps, and when each stream finishes."""
import csv
import sys


def main(path, first, n):
    rows = list(csv.DictReader(open(path)))
    ks = {}
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("sk::", "")
        ks.setdefault(name, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for v in ks.values():
        v.sort()
    pf = []
    for nm in ("k_pfp_hash", "k_pfp_apply", "k_pfp_reply"):  # k_pfp_reply: multi-element commands only
        pf += ks.get(nm, [])[first:first + n]
    bc = ks.get("k_bloom_contains", [])[first:first + n]
    pf.sort()
    t0 = min(pf[0][0], bc[0][0])
    t1 = max(max(e for _, e in pf), max(e for _, e in bc))

    def busy(iv):
        tot, gaps, last = 0, 0, None
        for s, e in iv:
            tot += e - s
            if last is not None and s > last:
                gaps += s - last
            last = max(last or 0, e)
        return tot, gaps, last

    pb, pg, pe = busy(pf)
    bb, bg, be = busy(bc)
    span = t1 - t0
    print("window %.1f us for %d steps: %.1f us/step" % (span / 1e3, n, span / 1e3 / n))
    print("pfadd stream: busy %.1f us/step, gaps %.1f us/step, ends at %.1f us" % (pb / 1e3 / n, pg / 1e3 / n, (pe - t0) / 1e3))
    print("contains stream: busy %.1f us/step, gaps %.1f us/step, ends at %.1f us" % (bb / 1e3 / n, bg / 1e3 / n, (be - t0) / 1e3))
    # time with both / one / none running
    ev = [(s, 1, 0) for s, _ in pf] + [(e, -1, 0) for _, e in pf] + [(s, 1, 1) for s, _ in bc] + [(e, -1, 1) for _, e in bc]
    ev.sort()
    cnt, acc, last = [0, 0], {}, t0
    for t, d, w in ev:
        key = (cnt[0] > 0, cnt[1] > 0)
        acc[key] = acc.get(key, 0) + (t - last)
        last = t
        cnt[w] += d
    for key, v in sorted(acc.items()):
        lab = {(True, True): "both", (True, False): "pfadd only", (False, True): "contains only",
               (False, False): "idle"}[key]
        print("  %-14s %.1f us/step" % (lab, v / 1e3 / n))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]))
