"""Every kernel of one step (rocprofv3 kernel trace csv) in start order: queue, duration, gap on its queue, grid.
    python scripts/step_list.py TRACE_CSV [STEP_FROM_END] [MIN_GAP_US]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
min_gap = float(sys.argv[3]) if len(sys.argv) > 3 else -1.0
idx = [i for i, r in enumerate(rows) if "stft_mel" in r["Kernel_Name"]]
step = rows[idx[-k - 1]:idx[-k]]
t0 = int(step[0]["Start_Timestamp"])
prev = {}
for r in step:
    q = r["Queue_Id"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev[q]) / 1e3 if q in prev else 0.0
    prev[q] = e
    n = r["Kernel_Name"].replace("hlmc::", "").replace("(anonymous namespace)::", "").replace("__hip_bfloat16", "bf")
    n = n.replace("void ", "").split("(")[0][:70]
    if gap >= min_gap:
        g = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        print(f"{(s - t0) / 1e3:8.1f} q{q} {(e - s) / 1e3:7.1f} gap {gap:6.1f} grid {g:5d}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']} {n}")
