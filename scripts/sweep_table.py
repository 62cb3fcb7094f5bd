"""Tabulate gpurun_out/sweep.log (scripts/gpu_gemm_sweep.sh): us per layer per knob setting."""
import collections
import re
import sys

cur = None
d = collections.OrderedDict()
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sweep.log"):
    if line.startswith("=="):
        cur = line[3:].strip()
        continue
    m = re.match(r"(\S+ \S+ \S+ \S+)\s+([\d.]+) us", line)
    if m and cur:
        d.setdefault(m.group(1), {})[cur] = float(m.group(2))
    m = re.match(r"TOTAL\s+([\d.]+)", line)
    if m:
        d.setdefault("TOTAL", {})[cur] = float(m.group(1))
cfgs = list(next(iter(d.values())).keys())
print(f"{'layer':34s}" + "".join(f"{c[-15:]:>16s}" for c in cfgs))
for k, v in d.items():
    print(f"{k:34s}" + "".join(f"{v.get(c, 0):16.1f}" for c in cfgs))
