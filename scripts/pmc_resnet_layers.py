"""Per-GEMM table of one eager ResNet-50 training step (scripts/pmc_resnet_layers.sh).

Joins, dispatch by dispatch, the last step's GEMM launches as the engine logged them (CDP_GEMM_LOG:
kind, M, N, K, tile, split-K; a bwd_pair launch is a data-gradient and a weight-gradient GEMM in one
dispatch) with rocprofv3's kernel trace (durations) and three counter passes: MFMA busy / wave waits,
FETCH_SIZE, WRITE_SIZE. Prints a markdown table (us, TF/s fp32-equivalent, TB/s read and written,
MFMA busy share of all SIMD cycles, wait share of wave cycles) and a per-class summary.
usage: python scripts/pmc_resnet_layers.py gpurun_out/<tag>
"""
import collections
import csv
import glob
import json
import os
import sys

SIMDS = 1024


def is_gemm(name):
    return any(k in name for k in ("conv_x3_kernel", "conv_igemm_kernel", "wgrad_kernel", "wgrad_x3_kernel",
                                   "bwd_pair_kernel", "stem_fwd_kernel", "stem_wgrad_kernel"))


def rows_of(pattern):
    f = glob.glob(pattern)
    return list(csv.DictReader(open(f[0]))) if f else []


def counters(d, sub):
    rows = rows_of(os.path.join(d, sub, "*counter_collection.csv"))
    byd = collections.defaultdict(dict)
    names = {}
    for r in rows:
        did = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        byd[did][r["Counter_Name"]] = byd[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[did] = r["Kernel_Name"]
    return [byd[did] for did in sorted(byd) if is_gemm(names[did])]


def main(d):
    log = json.load(open(os.path.join(d, "gemm_log.json")))
    disp = []  # one entry per GEMM dispatch
    i = 0
    while i < len(log):
        e = log[i]
        if e["kind"] == "pair_dgrad" and i + 1 < len(log) and log[i + 1]["kind"] == "pair_wgrad":
            disp.append(("pair", [e, log[i + 1]]))
            i += 2
        else:
            disp.append((e["kind"], [e]))
            i += 1
    kt = sorted(rows_of(os.path.join(d, "kt", "*kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
    g = [r for r in kt if is_gemm(r["Kernel_Name"])]
    n = len(disp)
    if len(g) < n:
        raise SystemExit(f"trace has {len(g)} GEMM dispatches, the log {n}")
    g = g[-n:]
    pm, fe, wr = counters(d, "pmc")[-n:], counters(d, "fetch")[-n:], counters(d, "write")[-n:]
    print("| # | GEMM | M x N x K (per GEMM) | tile / splits | us | TF/s | read TB/s | write TB/s | MFMA busy % | wait % |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    cls = collections.defaultdict(lambda: [0.0, 0.0, 0.0, 0.0, 0])
    tot_us = tot_fl = 0.0
    for k, ((kind, es), r) in enumerate(zip(disp, g)):
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        fl = sum(2.0 * e["M"] * e["N"] * e["K"] for e in es)
        shape = " + ".join(f"{e['M']}x{e['N']}x{e['K']}" for e in es)
        tile = " + ".join(f"{e['bm']}x{e['bn']}/{e['splits']}" for e in es)
        c = pm[k] if k < len(pm) else {}
        wall = c.get("GRBM_GUI_ACTIVE", 0) / 8.0
        mfma = 100.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (SIMDS * wall) if wall else float("nan")
        wc = c.get("SQ_WAVE_CYCLES", 0)
        wa = 100.0 * c.get("SQ_WAIT_ANY", 0) / wc if wc else float("nan")
        rb = (fe[k].get("FETCH_SIZE", 0) * 1024) if k < len(fe) else 0.0  # KB -> bytes
        wb = (wr[k].get("WRITE_SIZE", 0) * 1024) if k < len(wr) else 0.0
        tot_us += us
        tot_fl += fl
        key = kind
        cl = cls[key]
        cl[0] += us
        cl[1] += fl
        cl[2] += rb
        cl[3] += wb
        cl[4] += 1
        print(f"| {k} | {kind} | {shape} | {tile} | {us:.1f} | {fl / us / 1e6:.0f} | {rb / us / 1e6:.2f} | "
              f"{wb / us / 1e6:.2f} | {mfma:.1f} | {wa:.1f} |")
    print(f"\nGEMM total {tot_us:.1f} us over {n} dispatches, {tot_fl / 1e9:.1f} GFLOP, "
          f"{tot_fl / tot_us / 1e6:.0f} TF/s fp32-equivalent\n")
    print("| class | dispatches | us | TF/s | read TB/s | write TB/s |\n|---|---|---|---|---|---|")
    for key, (us, fl, rb, wb, c) in sorted(cls.items(), key=lambda t: -t[1][0]):
        print(f"| {key} | {c} | {us:.1f} | {fl / us / 1e6:.0f} | {rb / us / 1e6:.2f} | {wb / us / 1e6:.2f} |")


if __name__ == "__main__":
    main(sys.argv[1])
