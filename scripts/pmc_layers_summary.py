"""Label the last training step's GEMM dispatches of a VGG-11 bench run by layer and report, per
dispatch: time, achieved TFLOP/s (fp32-equivalent), MFMA busy share of all SIMD cycles, issue-stall
and wait shares of wave cycles, LDS bank conflicts (scripts/pmc_layers.sh)."""
import collections
import csv
import glob
import os
import sys

VGG = [(3, 64, 32), (64, 128, 16), (128, 256, 8), (256, 256, 8), (256, 512, 4), (512, 512, 4), (512, 512, 2),
       (512, 512, 2)]
SIMDS = 1024


def kind(name):
    if "stem_fwd" in name:
        return "fwd0"
    if "stem_wgrad" in name:
        return "wgrad0"
    if "bwd_pair" in name:
        return "pair"
    if "wgrad" in name and "slab" not in name:
        return "wgrad"
    if "conv_x3_kernel" in name or "conv_igemm" in name:
        inner = name.split("<", 1)[1] if "<" in name else ""
        parts = [p.strip() for p in inner.split(">")[0].split(",")]
        return "dgrad" if len(parts) > 3 and parts[3] == "true" else "fwd"
    return None


def rows_of(pattern):
    f = glob.glob(pattern)
    return list(csv.DictReader(open(f[0]))) if f else []


def main(d, B):
    B = int(B)
    kt = rows_of(os.path.join(d, "kt", "*kernel_trace.csv"))
    kt.sort(key=lambda r: int(r["Start_Timestamp"]))
    gemm = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in kt
            if kind(r["Kernel_Name"])]
    # one step = stem fwd + 7 fwd + (7 pairs or 7 dgrad + 7 wgrad) + stem wgrad; find the last stem_fwd
    last = max(i for i, (n, _) in enumerate(gemm) if kind(n) == "fwd0")
    step = gemm[last:]
    pmc = rows_of(os.path.join(d, "pmc", "*counter_collection.csv"))
    byd = collections.defaultdict(dict)
    names = {}
    for r in pmc:
        did = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        byd[did][r["Counter_Name"]] = byd[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[did] = r["Kernel_Name"]
    pd = [(did, names[did]) for did in sorted(byd) if kind(names[did])]
    plast = max(i for i, (_, n) in enumerate(pd) if kind(n) == "fwd0")
    pstep = pd[plast:]
    print(f"# VGG-11 B={B}: GEMM dispatches of one training step (eager, rocprofv3)\n")
    print("| # | layer | GEMM | us | TF/s | MFMA busy % | wait-inst % | wait % | LDS conflict / LDS cycles |")
    print("|---|---|---|---|---|---|---|---|---|")
    cnt = collections.Counter()
    tot_us = tot_fl = 0.0
    for i, (n, us) in enumerate(step):
        k = kind(n)
        cnt[k] += 1
        if k == "fwd0":
            layer, fl = 0, 2.0 * B * 32 * 32 * 64 * 27
        elif k == "wgrad0":
            layer, fl = 0, 2.0 * B * 32 * 32 * 64 * 27
        elif k == "fwd":
            layer = cnt[k]
            ci, co, hw = VGG[layer]
            fl = 2.0 * B * hw * hw * co * ci * 9
        else:
            layer = 8 - cnt[k]
            ci, co, hw = VGG[layer]
            fl = 2.0 * B * hw * hw * co * ci * 9 * (2 if k == "pair" else 1)
        c = byd[pstep[i][0]] if i < len(pstep) and kind(pstep[i][1]) == k else {}
        wall = c.get("GRBM_GUI_ACTIVE", 0) / 8.0
        mfma = 100.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (SIMDS * wall) if wall else float("nan")
        wc = c.get("SQ_WAVE_CYCLES", 0)
        wi = 100.0 * c.get("SQ_WAIT_INST_ANY", 0) / wc if wc else float("nan")
        wa = 100.0 * c.get("SQ_WAIT_ANY", 0) / wc if wc else float("nan")
        lds = c.get("SQ_LDS_IDX_ACTIVE", 0)
        bc = c.get("SQ_LDS_BANK_CONFLICT", 0) / lds if lds else float("nan")
        tot_us += us
        tot_fl += fl
        print(f"| {i} | {layer} | {k} | {us:.1f} | {fl / us / 1e6:.0f} | {mfma:.1f} | {wi:.1f} | {wa:.1f} | {bc:.3f} |")
    print(f"\nGEMM total {tot_us:.1f} us, {tot_fl / 1e9:.1f} GFLOP, {tot_fl / tot_us / 1e6:.0f} TF/s fp32-equivalent")
    mix = rows_of(os.path.join(d, "mix", "*counter_collection.csv"))
    if mix:
        byd2 = collections.defaultdict(dict)
        nm2 = {}
        for r in mix:
            did = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
            byd2[did][r["Counter_Name"]] = byd2[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            nm2[did] = r["Kernel_Name"]
        md = [(did, nm2[did]) for did in sorted(byd2) if kind(nm2[did])]
        ml = max(i for i, (_, n) in enumerate(md) if kind(n) == "fwd0")
        print("\n| # | GEMM | waves | VALU/wave | MFMA/wave | LDS/wave | VMEM/wave | SALU/wave | VALU-active % of wall x SIMDs | LDS issue-stall / wave |")
        print("|---|---|---|---|---|---|---|---|---|---|")
        for i, (did, n) in enumerate(md[ml:]):
            c = byd2[did]
            w = c.get("SQ_WAVES", 0) or 1
            wall = c.get("GRBM_GUI_ACTIVE", 0) / 8.0
            va = 100.0 * 4 * c.get("SQ_ACTIVE_INST_VALU", 0) / (SIMDS * wall) if wall else float("nan")
            print(f"| {i} | {kind(n)} | {w:.0f} | {c.get('SQ_INSTS_VALU', 0) / w:.0f} | {c.get('SQ_INSTS_MFMA', 0) / w:.0f} | "
                  f"{c.get('SQ_INSTS_LDS', 0) / w:.0f} | {c.get('SQ_INSTS_VMEM', 0) / w:.0f} | {c.get('SQ_INSTS_SALU', 0) / w:.0f} | "
                  f"{va:.1f} | {c.get('SQ_WAIT_INST_LDS', 0) / w:.0f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else 256)


def mem_table(d):
    mem = rows_of(os.path.join(d, "mem", "*counter_collection.csv"))
    if not mem:
        return
    byd = collections.defaultdict(dict)
    nm = {}
    for r in mem:
        did = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        byd[did][r["Counter_Name"]] = byd[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        nm[did] = r["Kernel_Name"]
    md = [(did, nm[did]) for did in sorted(byd) if kind(nm[did])]
    ml = max(i for i, (_, n) in enumerate(md) if kind(n) == "fwd0")
    print("\n| # | GEMM | L2 hit % | L2 requests (M) | memory-side read requests (M) | write requests (M) | wall us (GRBM/8 @ 2.1 GHz) |")
    print("|---|---|---|---|---|---|---|")
    for i, (did, n) in enumerate(md[ml:]):
        c = byd[did]
        h, m = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        print(f"| {i} | {kind(n)} | {100 * h / max(1, h + m):.1f} | {(h + m) / 1e6:.2f} | {c.get('TCC_EA0_RDREQ_sum', 0) / 1e6:.2f} | "
              f"{c.get('TCC_EA0_WRREQ_sum', 0) / 1e6:.2f} | {c.get('GRBM_GUI_ACTIVE', 0) / 8 / 2.1e3:.1f} |")


if __name__ == "__main__" and len(sys.argv) > 1:
    mem_table(sys.argv[1])
