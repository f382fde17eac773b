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
# per position within a step (when every step launches the same sequence): mean duration, grid
# (workgroups) and registers of each launch
starts = sel
per = [rows[a:b] for a, b in zip(starts[:-1], starts[1:])]
common = collections.Counter(len(p) for p in per).most_common(1)
per = [p for p in per if common and len(p) == common[0][0]]
if per:
    print(f"{len(per)} steps of {len(per[0])} launches; position: mean us, workgroups, arch/accum VGPRs, LDS")
    for j in range(len(per[0])):
        r0 = per[0][j]
        us = sum((int(p[j]["End_Timestamp"]) - int(p[j]["Start_Timestamp"])) for p in per) / len(per) / 1e3
        gap = sum(int(p[j]["Start_Timestamp"]) - int(p[j - 1]["End_Timestamp"]) for p in per) / len(per) / 1e3 if j else 0.0
        wg = int(r0.get("Grid_Size_X", r0.get("Grid_Size", 0)) or 0) // max(1, int(r0.get("Workgroup_Size_X", r0.get("Workgroup_Size", 1)) or 1))
        print(f"{j:3d} {us:8.2f} us (gap {gap:5.2f})  {wg:8d} wg  v{r0.get('Arch_VGPR_Count', '?')}/{r0.get('Accum_VGPR_Count', '?')}"
              f"  lds {r0.get('LDS_Block_Size', r0.get('Group_Segment_Size', '?'))}  {r0['Kernel_Name'].split('(')[0][:70]}")
