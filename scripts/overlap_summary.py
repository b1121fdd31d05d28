"""Summarise the last step of scripts/overlap_timeline.py from rocprofv3 CSVs (markdown table).

usage: python scripts/overlap_summary.py run_kernel_trace.csv run_marker_api_trace.csv [out.md]
"""
import csv
import sys


def _ts(r, k):
    return int(r[k])


def main(kpath, mpath, out=None):
    ks = sorted(csv.DictReader(open(kpath)), key=lambda r: _ts(r, "Start_Timestamp"))
    ms = sorted(csv.DictReader(open(mpath)), key=lambda r: _ts(r, "Start_Timestamp"))
    name_col = next((c for c in ("Function", "Marker_Name", "Message", "Name") if ms and c in ms[0]), None)
    steps = [m for m in ms if name_col and m[name_col].startswith("step")]
    last = steps[-1]
    t0, t1 = _ts(last, "Start_Timestamp"), _ts(last, "End_Timestamp")
    stream_col = next((c for c in ("Stream_Id", "Queue_Id") if c in ks[0]), None)
    rows = [r for r in ks if t0 <= _ts(r, "Start_Timestamp") <= t1 + 20_000_000]
    phases = {m[name_col]: m for m in ms if t0 <= _ts(m, "Start_Timestamp") <= t1}
    lines = [f"Last step (host range {(t1 - t0) / 1e3:.1f} us). Host phases: "
             + ", ".join(f"{k} +{(_ts(v, 'Start_Timestamp') - t0) / 1e3:.0f}us" for k, v in phases.items()
                         if not k.startswith("step")),
             "", "| # | start us | dur us | stream | kernel |", "|---|---|---|---|---|"]
    k0 = _ts(rows[0], "Start_Timestamp") if rows else t0
    nb = 0
    for i, r in enumerate(rows):
        nm = r["Kernel_Name"].split("(")[0]
        nm = nm if len(nm) < 60 else nm[:57] + "..."
        tag = ""
        if "delay_scale_kernel" in nm:
            tag = f" **<- bucket {nb} collective done (comm stream)**"
            nb += 1
        lines.append(f"| {i} | {(_ts(r, 'Start_Timestamp') - k0) / 1e3:.1f} | "
                     f"{(_ts(r, 'End_Timestamp') - _ts(r, 'Start_Timestamp')) / 1e3:.1f} | "
                     f"{r.get(stream_col, '?') if stream_col else '?'} | `{nm}`{tag} |")
    launches = [m for m in ms if name_col and m[name_col].startswith("cdp.bucket_allreduce")
                and t0 <= _ts(m, "Start_Timestamp") <= t1]
    lines += ["", "Host-side bucket launches (roctx, us after step start): "
              + ", ".join(f"{m[name_col]} +{(_ts(m, 'Start_Timestamp') - t0) / 1e3:.0f}" for m in launches)]
    text = "\n".join(lines)
    if out:
        open(out, "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1], a[2] if len(a) > 2 else None)
