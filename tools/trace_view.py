"""Print the per-kernel summary and the tail of a rocprofv3 kernel trace (dev tool)."""
import csv
import sys


def short(n):
    n = n.split("(")[0].replace("void ", "").replace("sk::", "")
    if "rocprim" in n:
        for t in ["onesweep_iteration", "global_offsets", "block_sort", "init_lookback", "scan_impl"]:
            if t in n:
                return "rocprim:" + t
        return "rocprim:other"
    return n


def main(path, first, last):
    rows = list(csv.DictReader(open(path)))
    agg = {}
    for r in rows:
        k = short(r["Kernel_Name"])
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        a = agg.setdefault(k, [0, 0])
        a[0] += 1
        a[1] += d
    for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print("%-34s %6d %10.2f us avg" % (k, n, t / n / 1e3))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tail = rows[first:last]
    t0 = int(tail[0]["Start_Timestamp"])
    for r in tail:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print("%-30s q%s s=%9.1f e=%9.1f d=%6.1f" % (short(r["Kernel_Name"])[:30], r["Queue_Id"], s / 1e3, e / 1e3,
                                                   (e - s) / 1e3))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else -60, int(sys.argv[3]) if len(sys.argv) > 3 else None)
