"""Median duration of a kernel's launches in a rocprofv3 trace directory (rocpd sqlite output of
tools/gpu.sh trace), split by launch parity (e.g. a step's catch-up and update row Adam).
python tools/trace_kernel_medians.py DIR KERNEL [--last N]"""
import argparse
import glob
import sqlite3
import statistics as st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("kernel")
    ap.add_argument("--last", type=int, default=40)
    args = ap.parse_args()
    db = glob.glob(f"{args.dir}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, grid_x from kernels order by start").fetchall()
    ks = [((e - s) / 1e3, g) for n, s, e, g in rows if args.kernel in n][-args.last:]
    for par in (0, 1):
        sel = ks[par::2]
        print(f"{args.dir} {args.kernel} launches {par}::2: median {st.median([x for x, _ in sel]):.2f} us, "
              f"grid {st.median([g for _, g in sel]):.0f} threads ({len(sel)} launches)")


if __name__ == "__main__":
    main()
