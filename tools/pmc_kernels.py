"""Per-kernel sums of rocprofv3 --pmc counter_collection.csv files:
python tools/pmc_kernels.py p1.csv [p2.csv ...] [--match substr]"""
import csv
import sys
from collections import defaultdict

files = [a for a in sys.argv[1:] if a.endswith(".csv")]
match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else None
tot = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for f in files:
    for r in csv.DictReader(open(f)):
        if f.endswith(".csv") and r["Kernel_Name"] == match:
            pass
        k = r["Kernel_Name"][:90]
        if match and match not in r["Kernel_Name"]:
            continue
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k].add((f, r["Dispatch_Id"]))
rows = sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", kv[1].get("SQ_VALU_MFMA_BUSY_CYCLES", 0)))
for k, c in rows[:25]:
    n = len(calls[k])
    wc = c.get("SQ_WAVE_CYCLES", 0)
    line = f"{k[:70]:70s} disp {n:4d}"
    if wc:
        line += (f" | valu_active {c['SQ_ACTIVE_INST_VALU'] / wc:5.2f} any_active {c['SQ_ACTIVE_INST_ANY'] / wc:5.2f}"
                 f" wait {c['SQ_WAIT_ANY'] / wc:5.2f} wait_inst {c['SQ_WAIT_INST_ANY'] / wc:5.2f}"
                 f" valu_insts/wave {c['SQ_INSTS_VALU'] / max(c['SQ_WAVES'], 1):8.0f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        g = c.get("GRBM_GUI_ACTIVE", 0)
        line += (f" | mfma_busy/gui {c['SQ_VALU_MFMA_BUSY_CYCLES'] / max(g, 1):7.3f}"
                 f" mops_bf16 {c.get('SQ_INSTS_VALU_MFMA_MOPS_BF16', 0):.3g}"
                 f" mops_f32 {c.get('SQ_INSTS_VALU_MFMA_MOPS_F32', 0):.3g}"
                 f" lds {c.get('SQ_INSTS_LDS', 0):.3g} vmem {c.get('SQ_INSTS_VMEM', 0):.3g}")
    if wc and "SQ_WAIT_INST_LDS" in c:
        line += (f" | wait_inst_lds {c['SQ_WAIT_INST_LDS'] / wc:5.2f}"
                 f" lds_active {c.get('SQ_ACTIVE_INST_LDS', 0) / wc:5.2f}"
                 f" bank_conf/lds_active {c.get('SQ_LDS_BANK_CONFLICT', 0) / max(c.get('SQ_ACTIVE_INST_LDS', 1), 1):5.2f}"
                 f" busy/gui {c.get('SQ_BUSY_CYCLES', 0) / max(c.get('GRBM_GUI_ACTIVE', 1), 1):5.2f}")
    print(line)
