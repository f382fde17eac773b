"""Summarise tools/pmc_limiter.sh passes: per-launch averages of every counter for one kernel,
plus the derived ratios that name the item pass's bound.
python tools/pmc_limiter.py <out dir> [--kernel k_spmm_vec] [--edges-per-launch E] [--json out.json]"""
import argparse
import csv
import glob
import json
import os
import statistics


def collect(out, kernel):
    per = {}
    for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"]:
                continue
            key = (os.path.relpath(f, out).split(os.sep)[0], r["Dispatch_Id"])
            per.setdefault(r["Counter_Name"], {}).setdefault(key, 0.0)
            per[r["Counter_Name"]][key] += float(r["Counter_Value"])
    return {c: statistics.mean(v.values()) for c, v in per.items()}, {c: len(v) for c, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--kernel", default="k_spmm_vec")
    ap.add_argument("--edges-per-launch", type=float, default=None)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    c, n = collect(a.out, a.kernel)
    d = {}

    def ratio(name, num, den):
        if num in c and den in c and c[den]:
            d[name] = c[num] / c[den]

    ratio("wait_any_frac", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES")
    ratio("wait_inst_any_frac", "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES")
    ratio("active_inst_any_frac", "SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES")
    ratio("valu_per_vmem_rd", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD")
    ratio("avg_waves_resident", "SQ_LEVEL_WAVES", "SQ_BUSY_CYCLES")
    ratio("ta_busy_frac", "TA_TA_BUSY_sum", "GRBM_GUI_ACTIVE")
    ratio("tcp_tcc_req_per_access", "TCP_TCC_READ_REQ_sum", "TCP_TOTAL_CACHE_ACCESSES_sum")
    ratio("tcc_read_latency_cycles", "TCP_TCC_READ_REQ_LATENCY_sum", "TCP_TCC_READ_REQ_sum")
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        d["tcc_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if a.edges_per_launch:
        for k in ("SQ_INSTS_VMEM_RD", "SQ_INSTS_VALU", "TCP_TCC_READ_REQ_sum", "TCP_TOTAL_CACHE_ACCESSES_sum"):
            if k in c:
                d[f"{k}_per_edge"] = c[k] / a.edges_per_launch
    res = {"kernel": a.kernel, "per_launch": c, "launches": n, "derived": d}
    print(json.dumps(res, indent=1))
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
