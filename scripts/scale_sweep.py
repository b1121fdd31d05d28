"""Per-strategy scaling sweep over the self-launching bench (BASELINE.md "sync cost" rows on MI355X).

For every strategy (gather_scatter = Part 2a, allreduce_blocking = Part 2b, bucketed_overlap =
hook-bucketed overlap, ddp = Part 3) and every N in --gpus, runs

    python bench.py --gpus N --strategy S [--model M --bucket-cap-mb C] --steps K --warmup W

(bench.py starts the N rank processes itself) and collects img/s for weak scaling (256 images per
GPU) and the reference's strong scaling (global 256 split int(256/N), /root/reference/src/Part
2a/main.py:22), plus the exposed gradient-sync time per iteration (ms/step with sync minus without)
that the bench reports for N > 1. Writes one JSON line per run and a markdown table.

    python scripts/scale_sweep.py --gpus 1,2,4,8 --out sweep.md          # 8-GPU node
    python scripts/scale_sweep.py --gpus 1 --model resnet50 --bucket-cap 8,25

Only run the N your node has; nothing here invents numbers for GPUs that were not measured.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STRATEGIES = ["gather_scatter", "allreduce_blocking", "bucketed_overlap", "ddp"]


def run_one(n, strategy, args, cap=None):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--strategy", strategy,
           "--steps", str(args.steps), "--warmup", str(args.warmup), "--model", args.model]
    if cap is not None:
        cmd += ["--bucket-cap-mb", str(cap)]
    if args.model.startswith("resnet"):
        cmd += ["--local-batch", str(args.resnet_batch)]
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=args.timeout, cwd=REPO)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"n_gpus": n, "strategy": strategy, "bucket_cap_mb": cap, "error": (r.stderr or "")[-800:]}
    rec = json.loads(lines[-1])
    rec["bucket_cap_mb"] = cap
    return rec


def table(recs):
    out = ["| model | strategy | N | bucket MiB | weak img/s | weak ms/step | strong img/s (global 256) | "
           "exposed sync ms/iter | ranks seen |",
           "|---|---|---|---|---|---|---|---|---|"]
    for r in recs:
        if "error" in r:
            out.append(f"| | {r['strategy']} | {r['n_gpus']} | {r.get('bucket_cap_mb') or 'default'} | "
                       f"failed | | | | |")
            continue
        strong = r.get("strong", {}).get("value", r["value"] if r["n_gpus"] == 1 else "")
        out.append(f"| {r['config']['model']} | {r['config']['strategy']} | {r['n_gpus']} | "
                   f"{r.get('bucket_cap_mb') or 'default'} | {r['value']} | {r['ms_per_step']} | {strong} | "
                   f"{r.get('exposed_comm_ms', 0.0 if r['n_gpus'] == 1 else '')} | {r.get('ranks_seen', '')} |")
    return "\n".join(out)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", default="1")
    p.add_argument("--strategies", default=",".join(STRATEGIES))
    p.add_argument("--model", default="vgg11")
    p.add_argument("--bucket-cap", default="", help="comma list of bucket caps (MiB); default: library default")
    p.add_argument("--resnet-batch", type=int, default=64)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--timeout", type=float, default=900)
    p.add_argument("--out", default=None)
    p.add_argument("--jsonl", default=None)
    args = p.parse_args()
    caps = [float(c) for c in args.bucket_cap.split(",") if c] or [None]
    recs = []
    for n in [int(x) for x in args.gpus.split(",")]:
        strategies = args.strategies.split(",") if n > 1 else ["ddp"]  # N = 1: no sync, one row
        for s in strategies:
            for cap in (caps if s in ("ddp", "bucketed_overlap") else [None]):
                rec = run_one(n, s, args, cap)
                recs.append(rec)
                print(json.dumps(rec), flush=True)
                if args.jsonl:
                    with open(args.jsonl, "a") as fh:
                        fh.write(json.dumps(rec) + "\n")
    text = table(recs)
    print(text)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    main()
