"""Same-box, in-graph A/B of kernel-lab libraries: the bench's captured training step
(tools/step_trace.py) under rocprofv3 --kernel-trace once per library and round, alternating,
and per launch position the mean in-graph duration (bench.step_breakdown's kernels_mean_us).

  python tools/lab/ab_step.py --reps 2 base wsd prec      (base = the product library;
                                                           <name> = leak-det-gnn_amd/lib/<name>/;
                                                           <name>:K=V,.. also sets environment)
"""
import argparse
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO), str(REPO / "leak-det-gnn_amd")]

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--B", type=int, default=256)
    args = ap.parse_args()
    res = {v: [] for v in args.variants}
    for r in range(args.reps):
        for v in args.variants:
            lib, _, envs = v.partition(":")  # <lib>[:K=V,K=V]: environment for the traced step too
            if lib == "base":
                os.environ.pop("LEAKGNN_LIB", None)
            else:
                os.environ["LEAKGNN_LIB"] = str(REPO / "leak-det-gnn_amd" / "lib" / lib / "libleakgnn.so")
            kv = dict(e.split("=", 1) for e in envs.split(",") if e)
            old = {k: os.environ.get(k) for k in kv}
            os.environ.update(kv)
            bd = bench.step_breakdown(args.B, 1.0)
            for k, o in old.items():
                if o is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = o
            if bd is None:
                print(f"{v} round {r}: no trace", flush=True)
                continue
            row = dict(bd["kernels_mean_us"], sum_us=bd["sum_us"], span_us=bd["replay_span_us"])
            res[v].append(row)
            print(v, r, json.dumps({k: row[k] for k in ("sum_us", "span_us", "k_gcn_fwd_pc#0", "k_gcn_fwd_pc#1")
                                    if k in row}), flush=True)
    os.environ.pop("LEAKGNN_LIB", None)
    keys = list(res[args.variants[0]][0]) if res[args.variants[0]] else []
    print("position " + " ".join(f"{v:>22s}" for v in args.variants))
    for k in keys:
        cells = []
        for v in args.variants:
            xs = sorted(row.get(k) for row in res[v] if k in row)
            cells.append(f"{'/'.join(f'{x:.1f}' for x in xs):>22s}")
        print(f"{k:28s} " + " ".join(cells))


if __name__ == "__main__":
    main()
