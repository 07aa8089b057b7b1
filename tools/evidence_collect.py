"""Copy the evidence pass outputs (tools/gpu/evidence_r03.sh -> gpurun_out/ev3)
into profiles/<tag>_*: the bench line, kernel stats of the bench command, of
C2 training steps and of the C5 train.py step, the C2 SQ / MFMA PMC summary
and the test / smoke summary.  python tools/evidence_collect.py r03"""
import csv
import os
import shutil
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "r03"
src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/ev3"
os.makedirs("profiles", exist_ok=True)
line = [ln for ln in open(f"{src}/bench.json") if ln.startswith("{")][-1]
open(f"profiles/{tag}_bench.json", "w").write(line)
for a, b in [("bprof/bench_kernel_stats.csv", "bench_kernel_stats.csv"),
             ("c2/kt_kernel_stats.csv", "c2_step_kernel_stats.csv"),
             ("c5/c5_kernel_stats.csv", "c5_step_kernel_stats.csv")]:
    if os.path.exists(f"{src}/{a}"):
        shutil.copy(f"{src}/{a}", f"profiles/{tag}_{b}")
tests = [ln.strip() for ln in open(f"{src}/tests.log") if " passed" in ln][-1:]
smoke = [ln.strip() for ln in open(f"{src}/smoke.log") if "smoke" in ln][-1:]
open(f"profiles/{tag}_gpu_tests.txt", "w").write("\n".join(tests + smoke) + "\n")

tot = defaultdict(lambda: defaultdict(float))
for p in ("p1", "p2"):
    f = f"{src}/c2/{p}_counter_collection.csv"
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        tot[r["Kernel_Name"][:100]][r["Counter_Name"]] += float(r["Counter_Value"])
rows = []
for k, c in tot.items():
    if "GRBM_GUI_ACTIVE" not in c or "SQ_WAVE_CYCLES" not in c:
        continue
    busy = c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(c["GRBM_GUI_ACTIVE"], 1) / 128
    va = c["SQ_ACTIVE_INST_VALU"] / max(c["SQ_WAVE_CYCLES"], 1)
    rows.append((c["GRBM_GUI_ACTIVE"], f"{k:100s} | mfma_busy {busy:6.3f} valu_active {va:6.3f} "
                                       f"mops_bf16 {c['SQ_INSTS_VALU_MFMA_MOPS_BF16']:.3e} lds {c['SQ_INSTS_LDS']:.3e}"))
rows.sort(key=lambda t: -t[0])
with open(f"profiles/{tag}_c2_step_pmc_mfma.txt", "w") as f:
    f.write("C2 training step (tools/gemm_step_ab.py hip 1: 2 warmup + 1 step, 12 layers), rocprofv3 --pmc passes p1 (SQ) "
            "and p2 (MFMA) of tools/gpu/evidence_r03.sh, sorted by GRBM_GUI_ACTIVE.\n"
            "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE / 128 (GUI_ACTIVE sums the 8 XCDs; 128 SIMDs per XCD); "
            "valu_active = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (per wave)\n")
    for _, ln in rows[:40]:
        f.write(ln + "\n")
print("wrote profiles/%s_*" % tag)
