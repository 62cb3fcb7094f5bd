"""Timeline of one step's main queue from a rocprofv3 kernel trace: every kernel with its duration and the idle
gap before it (the launch / dependency bubbles), plus the side-queue kernels running meanwhile.
    python scripts/step_gaps.py TRACE_CSV [STEP_FROM_END]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
idx = [i for i, r in enumerate(rows) if "stft_mel" in r["Kernel_Name"]]
a, b = idx[-k - 1], idx[-k]
step = rows[a:b]
mainq = step[0]["Queue_Id"]
t0 = int(step[0]["Start_Timestamp"])


def short(n):
    n = n.replace("hlmc::", "").replace("(anonymous namespace)::", "").replace("__hip_bfloat16", "bf16")
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    return n[:95]


last = None
for r in step:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    side = r["Queue_Id"] != mainq
    gap = "" if side or last is None else f"{(s - last) / 1e3:6.1f}"
    print(f"{(s - t0) / 1e3:8.1f} {'   side' if side else '   main'} {gap:>6} {(e - s) / 1e3:7.1f}  {short(r['Kernel_Name'])}")
    if not side:
        last = e
