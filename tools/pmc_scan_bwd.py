"""Summarise the C2 scan-backward PMC passes of tools/gpu/evidence_r06.sh
(gpurun_out/ev6/sbwd: FETCH_SIZE, WRITE_SIZE, SQ counters, kernel trace of
tools/scan_bwd_once.py) into profiles/<tag>_scan_bwd_pmc_summary.json, per
kernel of the backward (main pass, carry pass, reduce): HBM bytes per launch
(FETCH_SIZE x2, the gfx950 correction of MI355X_MICROARCH.md's HBM section
for wide coalesced streaming reads; WRITE_SIZE exact), the rocprof average
duration, the achieved traffic rate, and the SQ issue fractions.

Algorithmic bytes of one backward at C2 (B 8, L 2048, d_inner 2048, N 16,
bf16 I/O): reads u, delta, z, dout (4 x 2 B) and the fp32 checkpoints
(16 states x 4 B every 16 steps = 4 B) per (b, d, l), writes du, d(delta),
dz (3 x 2 B): 18 B per (b, d, l) = 604 MB (B and C rows and the dB / dC
slabs are < 1 %).

python tools/pmc_scan_bwd.py r06 [gpurun_out/ev6/sbwd]"""
import csv
import json
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "r06"
src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/ev6/sbwd"
B, L, D = 8, 2048, 2048
ALG = 18 * B * L * D


def short(name):
    for k in ("scan_bwd_carry", "scan_bwd_reduce", "scan_bwd_kernel", "scan_fwd"):
        if k in name:
            return k
    return None


def per_kernel(path):
    vals = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if k:
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sorted(v)[len(v) // 2] for c, v in cs.items()} for k, cs in vals.items()}


fetch = per_kernel(f"{src}/fetch_counter_collection.csv")
write = per_kernel(f"{src}/write_counter_collection.csv")
sq = per_kernel(f"{src}/sq_counter_collection.csv")
stats = {short(r["Name"]): r for r in csv.DictReader(open(f"{src}/trace_kernel_stats.csv")) if short(r["Name"])}
out = {"shape": {"B": B, "L": L, "d_inner": D, "N": 16, "io": "bf16"},
       "algorithmic_bytes_per_backward": ALG,
       "note": ("FETCH_SIZE x2 (gfx950 reports half of wide coalesced streaming reads; MI355X_MICROARCH.md HBM); "
                "WRITE_SIZE exact; per-launch medians over the ITERS=5 launches of tools/scan_bwd_once.py; "
                "valu_active = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES (per wave)"),
       "kernels": {}}
total_bytes = total_us = 0.0
for k in ("scan_bwd_kernel", "scan_bwd_carry", "scan_bwd_reduce"):
    if k not in fetch:
        continue
    fb = 2 * fetch[k]["FETCH_SIZE"] * 1024
    wb = write[k]["WRITE_SIZE"] * 1024
    us = float(stats[k]["AverageNs"]) / 1e3 if k in stats else None
    rec = {"fetch_bytes_corrected": fb, "write_bytes": wb, "traffic_bytes": fb + wb, "rocprof_avg_us": us,
           "rocprof_calls": int(stats[k]["Calls"]) if k in stats else None,
           "traffic_TB_per_s": (fb + wb) / us / 1e6 if us else None}
    if k in sq:
        c = sq[k]
        rec["valu_active"] = c.get("SQ_ACTIVE_INST_VALU", 0) / max(c.get("SQ_WAVE_CYCLES", 1), 1)
        rec["wait_any"] = c.get("SQ_WAIT_ANY", 0) / max(c.get("SQ_WAVE_CYCLES", 1), 1)
        rec["valu_insts_per_wave"] = c.get("SQ_INSTS_VALU", 0) / max(c.get("SQ_WAVES", 1), 1)
    out["kernels"][k] = rec
    total_bytes += fb + wb
    total_us += us or 0.0
out["total"] = {"traffic_bytes": total_bytes, "traffic_over_algorithmic": total_bytes / ALG, "us": total_us,
                "algorithmic_TB_per_s": ALG / total_us / 1e6 if total_us else None,
                "frac_of_8TBps_algorithmic": ALG / (total_us * 1e-6) / 8e12 if total_us else None}
json.dump(out, open(f"profiles/{tag}_scan_bwd_pmc_summary.json", "w"), indent=1)
print(json.dumps(out["total"]), {k: round(v["rocprof_avg_us"] or 0, 1) for k, v in out["kernels"].items()})
