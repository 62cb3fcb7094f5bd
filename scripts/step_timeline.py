"""One training step from a rocprofv3 kernel trace: per-launch start offset, duration, stream (queue) and name.
    python scripts/step_timeline.py TRACE_CSV [STEP_FROM_END]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
idx = [i for i, r in enumerate(rows) if "stft_mel" in r["Kernel_Name"]]
a, b = idx[-k - 1], idx[-k]
step = rows[a:b]
t0 = int(step[0]["Start_Timestamp"])
t1 = int(rows[b]["Start_Timestamp"])
print(f"step wall {(t1 - t0) / 1e3:.1f} us, {len(step)} kernels")


def short(n):
    n = n.replace("hlmc::", "").replace("(anonymous namespace)::", "").replace("__hip_bfloat16", "bf16")
    return n[:100]


for r in step:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    g = f"{int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
    print(f"{s / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{r['Queue_Id']:>2} {g:>12} {short(r['Kernel_Name'])}")
