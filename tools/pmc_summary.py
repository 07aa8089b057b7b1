"""Summarise the rocprofv3 PMC passes of tools/gpu/scripts_pmc.sh into
profiles/<tag>_scan_*: per-dispatch FETCH_SIZE / WRITE_SIZE of the scan
forward and the kernel-trace average, with the gfx950 FETCH_SIZE correction
(x2 for wide coalesced streaming reads, MI355X_MICROARCH.md HBM section).

python tools/pmc_summary.py r01 [gpurun_out/pmc]"""
import csv
import json
import os
import shutil
import sys


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/pmc"
    out = {}
    for dt in ("bf16", "fp32"):
        rec = {}
        for kind in ("fetch", "write"):
            rows = [r for r in csv.DictReader(open(f"{src}/{kind}_{dt}_counter_collection.csv"))
                    if "scan_fwd" in r["Kernel_Name"]]
            with open(f"profiles/{tag}_scan_{dt}_{kind}_size.csv", "w", newline="") as f:
                fields = ["Dispatch_Id", "Kernel_Name", "Grid_Size", "Workgroup_Size", "VGPR_Count", "LDS_Block_Size",
                          "Counter_Name", "Counter_Value"]
                w = csv.DictWriter(f, fieldnames=fields)
                w.writeheader()
                for r in rows:
                    w.writerow({k: r.get(k, "") for k in fields})
            vals = sorted(float(r["Counter_Value"]) for r in rows)
            rec[kind + "_kb_median"] = vals[len(vals) // 2]
            rec["kernel"] = rows[0]["Kernel_Name"]
        rec["fetch_bytes_corrected"] = 2 * rec["fetch_kb_median"] * 1024
        rec["write_bytes"] = rec["write_kb_median"] * 1024
        rec["traffic_bytes"] = rec["fetch_bytes_corrected"] + rec["write_bytes"]
        st = [r for r in csv.DictReader(open(f"{src}/trace_{dt}_kernel_stats.csv")) if "scan_fwd" in r["Name"]][0]
        rec["rocprof_avg_us"] = float(st["AverageNs"]) / 1e3
        rec["rocprof_calls"] = int(st["Calls"])
        rec["note"] = ("FETCH_SIZE x2 (gfx950 reports half of wide coalesced streaming reads; MI355X_MICROARCH.md "
                       "HBM); WRITE_SIZE exact")
        out[dt] = rec
        shutil.copy(f"{src}/trace_{dt}_kernel_stats.csv", f"profiles/{tag}_scan_{dt}_kernel_stats.csv")
    json.dump(out, open(f"profiles/{tag}_scan_pmc_summary.json", "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
