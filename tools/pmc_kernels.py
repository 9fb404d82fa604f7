"""Counter summary of the hot kernels (GPU box): rocprofv3 --pmc passes over tools/kbench.py.

Each pass is its own child process (never exec), kernel trace only, killed after 60 s;
counters are grouped to fit one pass (SQ <= 8, TCC <= 4, GRBM <= 2; MI355X_MICROARCH.md
"rocprofv3 PMC slots").  Per dispatch of the named kernel every counter is summed over
its dimensions, then averaged over dispatches.  Writes <out>/pmc_<tag>.json and a text
summary with the derived figures: where wave cycles go (WAIT_ANY = parked on
s_waitcnt/barrier, WAIT_INST_ANY = issue stall, ACTIVE_INST_ANY = issuing), instructions
per wave by class, MFMA busy share of SIMD cycles, LDS bank conflicts, and HBM bytes
(2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of that guide's HBM section).

usage: python tools/pmc_kernels.py --out gpurun_out/pmc --tag r02 [--targets gcn_fwd_nm_train:k_gcn_fwd_nm3,...]
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
PASSES = [
    ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
     "SQ_WAIT_INST_LDS", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE"],
    ["SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
     "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_LDS_BANK_CONFLICT"],
    ["SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_VALU_MFMA_MOPS_BF16",
     "SQ_INSTS_VALU_MFMA_MOPS_F32"],
    ["FETCH_SIZE"],
    ["WRITE_SIZE"],
    ["TCC_HIT_sum", "TCC_MISS_sum"],
]
DEFAULT_TARGETS = ("gcn_fwd_nm_train:k_gcn_fwd_pc,gcn_bwd_nm:k_gcn_bwd_nm3,edge_fwd:k_edge_fwd,"
                   "edge_bwd:k_edge_bwd,gru_fwd:k_gru_fwd,gru_bwd:k_gru_bwd")


def run_pass(which: str, kname: str, counters: list, B: int) -> dict:
    prof = "/opt/rocm/bin/rocprofv3"
    env = dict(os.environ, TMPDIR="/tmp")
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        cmd = ["timeout", "-s", "KILL", "60", prof, "--pmc", *counters, "--kernel-trace", "-d", d, "-o", "pmc",
               "--output-format", "csv", "--", sys.executable, str(REPO / "tools" / "kbench.py"), "--which", which,
               "--B", str(B), "--iters", "10", "--eager"]
        r = subprocess.run(cmd, env=env, cwd=str(REPO), stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
        if r.returncode != 0:
            print(f"  pass {counters} failed rc={r.returncode}: {r.stderr[-400:]}", flush=True)
            return {}
        per: dict = {}
        for f in Path(d).rglob("*counter_collection.csv"):
            for row in csv.DictReader(open(f)):
                if kname not in row["Kernel_Name"]:
                    continue
                key = (row["Dispatch_Id"], row["Counter_Name"])
                per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
        out: dict = {}
        for c in counters:
            vals = [v for (dsp, cn), v in per.items() if cn == c]
            if vals:
                out[c] = sum(vals) / len(vals)
        return out


def derive(c: dict) -> dict:
    g = c.get
    d = {}
    if g("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in c:
                d[f"{k}/WAVE_CYCLES"] = round(c[k] / c["SQ_WAVE_CYCLES"], 4)
    if g("SQ_WAVES"):
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                  "SQ_INSTS_SALU", "SQ_INSTS_SMEM"):
            if k in c:
                d[f"{k}/wave"] = round(c[k] / c["SQ_WAVES"], 1)
    if g("GRBM_GUI_ACTIVE"):
        # GRBM_GUI_ACTIVE comes back summed over the 8 XCDs' instances: per-XCD busy cycles
        # = the dispatch's duration in GPU cycles
        gui = c["GRBM_GUI_ACTIVE"] / 8.0
        simds = 1024  # 256 CUs x 4 SIMDs
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            d["MFMA_busy_of_SIMD_cycles"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui * simds), 4)
        d["duration_us_at_2.4GHz(GRBM_GUI_ACTIVE/8)"] = round(gui / 2400.0, 2)
    if "SQ_LDS_BANK_CONFLICT" in c and g("SQ_LDS_IDX_ACTIVE"):
        d["LDS_bank_conflict/LDS_active"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4)
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        d["HBM_bytes(2*FETCH+WRITE)"] = int((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
    if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None and (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]):
        d["L2_hit_rate"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/pmc")
    ap.add_argument("--tag", default="run")
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--targets", default=DEFAULT_TARGETS)
    args = ap.parse_args()
    out = Path(args.out)
    out.mkdir(parents=True, exist_ok=True)
    res = {}
    lines = [f"rocprofv3 --pmc passes over tools/kbench.py --B {args.B} --iters 10 --eager "
             f"(per-dispatch mean of each counter, summed over its dimensions)", ""]
    for t in args.targets.split(","):
        which, kname = t.split(":")
        print(f"{which} ({kname})", flush=True)
        c = {}
        for p in PASSES:
            c.update(run_pass(which, kname, p, args.B))
            print(f"  pass {p[0]}...: {len(c)} counters so far", flush=True)
        res[which] = {"kernel": kname, "counters": c, "derived": derive(c)}
        lines.append(f"== {which}  ({kname})")
        for k, v in sorted(c.items()):
            lines.append(f"   {k:32s} {v:,.1f}")
        for k, v in res[which]["derived"].items():
            lines.append(f"   > {k:32s} {v}")
        lines.append("")
        (out / f"pmc_{args.tag}.json").write_text(json.dumps(res, indent=1))
        (out / f"pmc_{args.tag}.txt").write_text("\n".join(lines))
    print("\n".join(lines))


if __name__ == "__main__":
    main()
