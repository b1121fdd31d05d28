"""Timeline of the last training step in a rocprofv3 kernel trace: the bucket collectives (RCCL kernel
+ modelled-xGMI delay on the comm queue), the optimizer launches (sgd_prep / sgd) and the step's end.

usage: python scripts/step_overlap_timeline.py <run_kernel_trace.csv> [label]
Prints a markdown table (us from the step's first dispatch) -- the evidence that, with
``--overlap-step``, the per-bucket SGD runs on its own queue under the later buckets' collectives.
"""
import csv
import sys


def main(path, label=""):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "augment_kernel" in r["Kernel_Name"]]
    step = rows[starts[-2]:starts[-1]]  # the last complete step (the last augment opens a trailing one)
    t0 = int(step[0]["Start_Timestamp"])
    end = max(int(r["End_Timestamp"]) for r in step)
    last_compute = max(int(r["End_Timestamp"]) for r in step
                       if not any(k in r["Kernel_Name"] for k in ("sgd", "delay", "Reduce", "nccl")))
    print(f"### {label or path}\n")
    print("| kernel | queue | start us | end us | dur us |\n|---|---|---|---|---|")
    for r in step:
        nm = r["Kernel_Name"]
        if not any(k in nm for k in ("sgd", "delay_scale", "oneRankReduce", "nccl", "Nccl")):
            continue
        short = nm.replace("void ", "").replace("cdp::", "").replace("(anonymous namespace)::", "")
        short = short.split("(")[0].split("<")[0][:40]
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print(f"| `{short}` | {r['Queue_Id']} | {s / 1e3:.1f} | {e / 1e3:.1f} | {(e - s) / 1e3:.1f} |")
    print(f"\nlast backward/forward compute kernel ends at {(last_compute - t0) / 1e3:.1f} us; "
          f"step ends at {(end - t0) / 1e3:.1f} us ({len(step)} dispatches)\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
