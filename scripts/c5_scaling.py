#!/usr/bin/env python3
"""Predicted strong-scaling efficiency of config 5 (BASELINE configs[4]: the mixed
corpus file-sharded over N GPUs, no collectives) from measured per-rank times.

For each N, every rank's share of the N-way split (shard.partition over
shard.KIND_COST, the split bench.py's ranks make) is decoded alone on this one GPU by
`bench.py --workload c5 --c5-share N:r` (same batches, copies in flight and timed
steps as an N-GPU run's rank r), one process per share.  With T_r the share's time
for K steps, the N-GPU job takes max_r T_r (the ranks share nothing), so

    predicted efficiency(N) = T_1 / (N * max_r T_r)

Usage: python scripts/c5_scaling.py [--files 100000] [--ns 1,2,4,8] [--steps 20]
       [--warmup 2] [--out gpurun_out/c5_scaling.jsonl] [-- extra bench.py args]
Each line of --out is one share's bench line (trimmed) plus, per N, a summary line.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_share(args, n, r, extra):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c5", "--c5-files", str(args.files),
           "--steps", str(args.steps), "--warmup", str(args.warmup), "--no-cpu", "--c5-share", f"{n}:{r}"] + extra
    t0 = time.perf_counter()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=args.timeout)
    if p.returncode != 0:
        sys.stderr.write(p.stderr[-3000:])
        raise SystemExit(f"share {n}:{r} failed (rc {p.returncode})")
    line = json.loads(p.stdout.strip().splitlines()[-1])
    cfg = line["config"]
    return {"n": n, "rank": r, "ms_per_step": line["ms_per_step"], "value": line["value"],
            "files": cfg["files_rank0"], "blocks": cfg["blocks_rank0"], "frames": cfg["frames_rank0"],
            "slices": cfg["slices_rank0"], "copies": line.get("c5_copies"), "kernel_ms": line["kernel_ms"],
            "redo_blocks": line["verified"]["redo_blocks"], "crc_errors": line["verified"]["crc_errors"],
            "wall_s": round(time.perf_counter() - t0, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=100000)
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--timeout", type=int, default=600)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "c5_scaling.jsonl"))
    args, extra = ap.parse_known_args()
    extra = [x for x in extra if x != "--"]
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    t1 = None
    with open(args.out, "a") as out:
        for n in [int(x) for x in args.ns.split(",")]:
            rows = []
            for r in range(n):
                row = run_share(args, n, r, extra)
                rows.append(row)
                out.write(json.dumps(row) + "\n")
                out.flush()
                print(json.dumps(row), flush=True)
            tmax = max(x["ms_per_step"] for x in rows)
            frames = sum(x["frames"] for x in rows)
            if n == 1:
                t1 = rows[0]["ms_per_step"]
            summ = {"n": n, "summary": True, "files": args.files, "steps": args.steps, "extra": extra,
                    "ms_per_step_max": tmax, "ms_per_step_min": min(x["ms_per_step"] for x in rows),
                    "ms_per_step_ranks": [x["ms_per_step"] for x in rows],
                    "predicted_Msamples_s": round(frames / (tmax * 1e-3) / 1e6, 1),
                    "predicted_efficiency": None if t1 is None else round(t1 / (n * tmax), 4)}
            out.write(json.dumps(summ) + "\n")
            out.flush()
            print(json.dumps(summ), flush=True)


if __name__ == "__main__":
    main()
