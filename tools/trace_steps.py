"""Per-launch timeline of a rocprofv3 --kernel-trace database (rocpd sqlite, tools/gpu.sh trace):
the last N launches of the run in dispatch order, with their duration, the gap before each and the
grid size — to read a probe's steady-state step launch by launch.
python tools/trace_steps.py <run_results.db> [--last 60] [--match spmm|combine|stack]"""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=60)
    ap.add_argument("--match", default="")
    args = ap.parse_args()
    c = sqlite3.connect(args.db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    suf = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch_"))[len("rocpd_kernel_dispatch_"):]
    rows = c.execute(f"select d.start, d.end, d.grid_size_x, d.workgroup_size_x, d.stream_id, k.kernel_name "
                     f"from rocpd_kernel_dispatch_{suf} d join rocpd_info_kernel_symbol_{suf} k on d.kernel_id = k.id "
                     f"order by d.start").fetchall()
    if args.match:
        rows = [r for r in rows if re.search(args.match, r[5])]
    rows = rows[-args.last:]
    prev = None
    for s, e, gx, wx, stream, name in rows:
        short = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))[:60]
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"{(e - s) / 1e3:8.2f} us  gap {gap:7.2f}  wgs {gx // max(wx, 1):7d}  s{stream}  {short}")
        prev = e


if __name__ == "__main__":
    main()
