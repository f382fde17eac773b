"""Per-step kernel time from a rocprofv3 kernel trace: the last STEPS occurrences of a marker kernel
(one per step) delimit the steps; prints span per step, busy kernel time per step and each
kernel's share. python tools/trace_per_step.py run_kernel_trace.csv STEPS MARKER"""
import csv, sys, collections
f, steps, marker = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# index of each marker kernel (one per step)
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(marker)]
sel = idx[-steps:]
lo, hi = sel[0], sel[-1]
seg = rows[lo:hi]
n = len(sel) - 1
span = (int(rows[hi]["Start_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) / n / 1e3
busy = collections.defaultdict(float); cnt = collections.Counter()
for r in seg:
    k = r["Kernel_Name"].split("(")[0][:60]
    busy[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / n / 1e3
    cnt[k] += 1
tot = sum(busy.values())
print(f"steps {n}: span {span:.1f} us/step, kernel busy {tot:.1f} us/step, launches/step {len(seg)/n:.1f}")
for k, v in sorted(busy.items(), key=lambda x: -x[1]):
    print(f"{v:8.2f} us  {cnt[k]/n:5.2f}x  {k}")
