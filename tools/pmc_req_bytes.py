"""Bytes per dispatch from tools/pmc_req.sh's request counts (dev tool).
usage: python tools/pmc_req_bytes.py DIR VARIANT  -> DIR/VARIANT.req_bytes.json; prints one line per kernel.
read bytes = 32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B (RDREQ printed beside their sum as a check);
write bytes = 64 x WRREQ_64B + 32 x (WRREQ - WRREQ_64B)."""
import json
import sys


def main(o, v):
    rd = json.load(open(f"{o}/{v}.rd/pmc_means.json"))
    wr = json.load(open(f"{o}/{v}.wr/pmc_means.json"))
    out = {}
    for k in sorted(rd):
        if not k.startswith("sk::"):
            continue
        r, w = rd[k], wr.get(k, {})
        n32, n64, n128 = (r.get("TCC_EA0_RDREQ_%s_sum" % s, 0.0) for s in ("32B", "64B", "128B"))
        nw, nw64 = w.get("TCC_EA0_WRREQ_sum", 0.0), w.get("TCC_EA0_WRREQ_64B_sum", 0.0)
        out[k] = {"read_bytes": 32 * n32 + 64 * n64 + 128 * n128, "write_bytes": 64 * nw64 + 32 * (nw - nw64),
                  "rdreq": r.get("TCC_EA0_RDREQ_sum", 0.0), "rdreq_32b": n32, "rdreq_64b": n64, "rdreq_128b": n128,
                  "wrreq": nw, "wrreq_64b": nw64, "dispatches": r.get("dispatches", 0)}
        d = out[k]
        print("%-8s %-44s read %.3f write %.3f GB  (rdreq %.0f = %.0f + %.0f + %.0f)" % (
            v, k[4:48], d["read_bytes"] / 1e9, d["write_bytes"] / 1e9, d["rdreq"], n32, n64, n128))
    json.dump(out, open(f"{o}/{v}.req_bytes.json", "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
