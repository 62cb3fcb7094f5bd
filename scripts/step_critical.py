"""Critical-path view of one training step from a rocprofv3 kernel trace (csv): main queue (the STFT's) busy
time, its idle gaps, the weight-gradient queue's busy time, and the main-queue kernel families by time.
    python scripts/step_critical.py TRACE_CSV [STEP_FROM_END]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
idx = [i for i, r in enumerate(rows) if "stft_mel" in r["Kernel_Name"]]
a, b = idx[-k - 1], idx[-k]
step = rows[a:b]
t0, t1 = int(step[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
mainq = step[0]["Queue_Id"]


def fam(n):
    n = n.replace("hlmc::", "").replace("(anonymous namespace)::", "").replace("__hip_bfloat16", "bf16")
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    m = re.match(r"([A-Za-z0-9_:]+)(<[^,>]*)?", n)
    base = m.group(1) if m else n[:40]
    if base.startswith("gemm"):
        loaders = re.findall(r"(ConvS2Loader|SubpixelLoader|DenseLoader|KRowConvS2|KRowDense|WithStats|WithBnBwd|StorePartialZ)", n)
        base += "[" + ",".join(dict.fromkeys(loaders)) + "]"
    return base


busy = collections.Counter()
fam_t = collections.defaultdict(lambda: collections.Counter())
last_end = {}
gaps = collections.Counter()
for r in step:
    q = r["Queue_Id"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy[q] += e - s
    fam_t[q][fam(r["Kernel_Name"])] += e - s
    if q in last_end and s > last_end[q]:
        gaps[q] += s - last_end[q]
    last_end[q] = max(last_end.get(q, 0), e)
print(f"step wall {(t1 - t0) / 1e3:.1f} us, {len(step)} kernels, main queue {mainq}")
for q in busy:
    print(f"queue {q}: busy {busy[q] / 1e3:.1f} us, gaps {gaps[q] / 1e3:.1f} us, launches "
          f"{sum(1 for r in step if r['Queue_Id'] == q)}")
    for f, t in fam_t[q].most_common(14):
        n = sum(1 for r in step if r["Queue_Id"] == q and fam(r["Kernel_Name"]) == f)
        print(f"   {t / 1e3:8.1f} us  {n:3d}x  {f}")
