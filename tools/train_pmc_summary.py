"""Per-kernel memory-side traffic of a profiled run (tools/train_pmc.sh): for each kernel name,
launches, mean duration (kernel trace), FETCH_SIZE x the gfx950 calibration factor
(profiles/pmc_traffic.json) + WRITE_SIZE per launch (their own --pmc passes; KiB counters) and
the resulting TB/s against 8 TB/s. Only the last third of each kernel's launches is used (the
timed steps, past plan building and warm-up).
python tools/train_pmc_summary.py PROFILE_DIR"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def tail(xs):
    return xs[len(xs) * 2 // 3:] if len(xs) >= 3 else xs


def main():
    d = sys.argv[1]
    factor = next(iter(json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json"))).values())).get(
        "fetch_correction_factor", 1.944)
    dur = collections.defaultdict(list)
    for r in sorted(rows(os.path.join(d, "trace"), "*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"])):
        dur[r["Kernel_Name"].split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    ctr = {}
    for name, sub, counter in (("fetch", "fetch", "FETCH_SIZE"), ("write", "write", "WRITE_SIZE")):
        per = collections.defaultdict(dict)
        for r in rows(os.path.join(d, sub), "*counter_collection.csv"):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0]
            per[k][int(r["Dispatch_Id"])] = per[k].get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
        ctr[name] = {k: [v[i] for i in sorted(v)] for k, v in per.items()}
    print(f"fetch calibration x{factor}; per launch over the last third of each kernel's launches")
    print(f"{'kernel':60s} {'n':>5s} {'us':>8s} {'fetch MB':>9s} {'write MB':>9s} {'TB/s':>6s} {'frac':>5s}")
    out = []
    for k, ds in dur.items():
        t = tail(ds)
        us = sum(t) / len(t)
        f = tail(ctr["fetch"].get(k, []))
        w = tail(ctr["write"].get(k, []))
        if not f or not w:
            continue
        mb = (sum(f) / len(f) * factor + sum(w) / len(w)) * 1024 / 1e6
        out.append((us * len(ds), k, len(ds), us, sum(f) / len(f) * factor * 1024 / 1e6, sum(w) / len(w) * 1024 / 1e6,
                    mb / us))
    for _, k, n, us, fm, wm, tbs in sorted(out, reverse=True)[:20]:
        print(f"{k[:60]:60s} {n:5d} {us:8.2f} {fm:9.2f} {wm:9.2f} {tbs:6.2f} {tbs / 8:5.2f}")


if __name__ == "__main__":
    main()
