"""Turn a round profile (tools/profile_round.sh output dir) into the roofline.traffic entry of
profiles/pmc_traffic.json: average memory-side bytes per k_spmm_vec launch =
FETCH_SIZE x calibration (tools/calib_fetch.py: a permutation gather that must read every byte
once) + WRITE_SIZE, each from its own --pmc pass.
python tools/pmc_to_traffic.py <profile dir> <workload key> [--kernel k_spmm_vec,k_spmm_ride]"""
import argparse
import csv
import glob
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, counter, kernel):
    vals = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if any(k in r["Kernel_Name"] for k in kernel.split(",")) and r["Counter_Name"] == counter:
                vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof")
    ap.add_argument("workload")
    # the item pass: plain slice launches and the ones carrying a riding combine (comma = any of)
    ap.add_argument("--kernel", default="k_spmm_vec,k_spmm_ride")
    args = ap.parse_args()
    # FETCH_SIZE / WRITE_SIZE are in KiB on gfx950 (rocprofv3 derived counters)
    fetch = per_launch(os.path.join(args.prof, "pmc_fetch"), "FETCH_SIZE", args.kernel)
    write = per_launch(os.path.join(args.prof, "pmc_write"), "WRITE_SIZE", args.kernel)
    cal_f = per_launch(os.path.join(args.prof, "calib_fetch"), "FETCH_SIZE", "k_spmm_vec")
    tj = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    data = json.load(open(tj))
    factor = data[next(iter(data))].get("fetch_correction_factor")
    log = os.path.join(args.prof, "calib_fetch.log")
    if cal_f and os.path.exists(log):
        for line in open(log):
            if line.startswith("expected_read_bytes"):
                factor = float(line.split()[1]) / (statistics.median(cal_f) * 1024)
    # the plan/kernel the counters were taken on: bench.py's roofline.signature of the profiled run
    sig = None
    for name in ("pmc_fetch.log", "pmc_write.log"):
        lp = os.path.join(args.prof, name)
        if os.path.exists(lp):
            for line in open(lp):
                if line.startswith("{"):
                    rec = json.loads(line)
                    s = rec.get("roofline", {}).get("signature")
                    if sig is not None and s != sig:
                        raise SystemExit(f"{name}: the two PMC passes ran different plans")
                    sig = s
    if sig is None or sig.get("workload") != args.workload:
        raise SystemExit("no bench.py signature for this workload in the PMC pass logs")
    f = statistics.mean(fetch) * 1024 * factor
    w = statistics.mean(write) * 1024
    data[args.workload] = {
        "hbm_bytes_per_launch": f + w, "fetch_bytes_corrected": f, "write_bytes": w,
        "fetch_correction_factor": factor, "kernel": args.kernel, "launches_measured": len(fetch),
        "signature": sig,
        "source": f"{os.path.relpath(args.prof, ROOT)} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)",
        "note": "average memory-side (L2-miss) bytes per launch; FETCH_SIZE also counts Infinity-Cache hits, so "
                "this bounds HBM traffic from above"}
    json.dump(data, open(tj, "w"), indent=1)
    print(json.dumps(data[args.workload], indent=1))


if __name__ == "__main__":
    main()
