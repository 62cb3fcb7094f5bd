"""HBM traffic per launch of every probed kernel kind from rocprofv3 PMC passes over bench.py, and the
rocprofv3 kernel-trace average duration of the same kinds (the check on bench.py's live HIP-event timing).

    python scripts/pmc_traffic.py OUT_JSON FETCH_DIR WRITE_DIR TRACE_DIR [MFMA_DIR] [BENCH_LOG]

FETCH_DIR / WRITE_DIR: `rocprofv3 --kernel-trace --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` output directories;
TRACE_DIR: a `--kernel-trace --stats` run of the bench command.  HBM bytes per dispatch =
(2 x FETCH_SIZE + WRITE_SIZE) x 1024: rocprofv3 reports both in KiB, and on gfx950 FETCH_SIZE counts half the
bytes of 16-B-per-lane streaming reads (/opt/skills/guides/MI355X_MICROARCH.md, HBM section).
BENCH_LOG (optional): an unprofiled bench.py output; its roofline.per_kind_untimed bytes_per_launch (the probe
sites' algorithmic bytes, common.hpp probe::site) are copied per kind with traffic_ratio = HBM bytes / algorithmic.
MFMA_DIR (optional): a `--kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE` pass.
MFMA busy per dispatch = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): the MFMA-unit cycles
(MI355X_MICROARCH.md: "counts cycles") over the SIMD-cycles of the dispatch (GRBM_GUI_ACTIVE is summed over
the 8 XCDs; 256 CUs x 4 SIMDs), i.e. the fraction of the dense MFMA peak the kernel's MFMAs occupy.
"""
import csv
import glob
import json
import re
import sys

KINDS = {  # op kind of include/hlmc.h hlmc_probe_arm -> kernel-name pattern
    "conv_s2": r"(gemm_nt\w*<.*ConvS2Loader|conv_s2_halo_kernel)",
    "subpixel": r"(gemm_nt\w*<.*SubpixelLoader|subpixel_halo_kernel)",
    "wgrad_s2": r"(gemm_tn_kernel<.*KRowConvS2|wgrad_halo_kernel)",
    "linear": r"gemm_nt\w*<[^<>]*, hlmc::DenseLoader<",
    "linear_wgrad": r"gemm_tn_kernel<[^<>]*, hlmc::(\(anonymous namespace\)::)?KRowDenseV?<[^<>]*>, hlmc::(\(anonymous namespace\)::)?KRowDenseV?<",
    "stft_mel": r"stft_mel0?_kernel",
    "bn": r"(bn_act_kernel|bn_bwd_moments_kernel|bn_bwd_apply_kernel|col_moments_kernel|parts_fold_kernel|"
          r"bn_finalize_kernel|bn_bwd_finalize_kernel|colsum_finalize_kernel)",
}


def kind_of(name):
    for k, pat in KINDS.items():
        if re.search(pat, name):
            return k
    return None


def counters(d, counter):
    vals = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = kind_of(r["Kernel_Name"])
            if k:
                vals.setdefault(k, {}).setdefault(r["Dispatch_Id"], 0.0)
                vals[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def trace_avg(d):
    durs = {}
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = kind_of(r["Kernel_Name"])
            if k:
                durs.setdefault(k, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return {k: (sum(v) / len(v) / 1e3, len(v)) for k, v in durs.items()}


def main():
    out, fdir, wdir, tdir = sys.argv[1:5]
    mdir = sys.argv[5] if len(sys.argv) > 5 else None
    algo = {}
    if len(sys.argv) > 6:
        for line in open(sys.argv[6]):
            if line.startswith("{") and '"roofline"' in line:
                pk = json.loads(line)["roofline"].get("per_kind_untimed", {})
                algo = {k: v.get("bytes_per_launch") for k, v in pk.items() if v.get("bytes_per_launch")}
    fetch, nf = counters(fdir, "FETCH_SIZE")
    write, nw = counters(wdir, "WRITE_SIZE")
    tr = trace_avg(tdir)
    mf, gr, nm = {}, {}, {}
    if mdir:
        mf, nm = counters(mdir, "SQ_VALU_MFMA_BUSY_CYCLES")
        gr, _ = counters(mdir, "GRBM_GUI_ACTIVE")
    kinds = {}
    for k in KINDS:
        e = {}
        if k in fetch and k in write:
            e["fetch_kib_raw"] = round(fetch[k], 1)
            e["write_kib"] = round(write[k], 1)
            e["hbm_bytes_per_launch"] = (2.0 * fetch[k] + write[k]) * 1024.0
            e["pmc_dispatches"] = min(nf[k], nw[k])
            if algo.get(k):
                e["bytes_per_launch"] = algo[k]
                e["traffic_ratio"] = round(e["hbm_bytes_per_launch"] / algo[k], 3)
        if k in tr:
            e["trace_avg_us"] = round(tr[k][0], 2)
            e["trace_dispatches"] = tr[k][1]
        if k in mf and gr.get(k):
            e["mfma_busy_cycles"] = round(mf[k], 1)
            e["grbm_gui_active"] = round(gr[k], 1)
            e["mfma_busy"] = round(mf[k] / (gr[k] / 8.0 * 1024.0), 4)
            e["mfma_dispatches"] = nm[k]
        if e:
            kinds[k] = e
    res = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py ({fdir}, {wdir}); "
                     f"2*FETCH_SIZE+WRITE_SIZE KiB per dispatch (gfx950 correction)", "kinds": kinds}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
