"""Per-step kernel time of two rocprofv3 kernel_stats.csv files side by side:
python tools/kstat_diff.py before.csv after.csv [steps=7] [n=40]"""
import csv
import sys


def load(p, steps):
    return {r["Name"]: (float(r["TotalDurationNs"]) / steps / 1e3, int(r["Calls"]) / steps) for r in csv.DictReader(open(p))}


steps = float(sys.argv[3]) if len(sys.argv) > 3 else 7.0
n = int(sys.argv[4]) if len(sys.argv) > 4 else 40
a, b = load(sys.argv[1], steps), load(sys.argv[2], steps)
ks = sorted(set(a) | set(b), key=lambda k: -max(a.get(k, (0, 0))[0], b.get(k, (0, 0))[0]))
print(f"{'us/step A':>9} {'B':>8}  {'calls A':>7} {'B':>5}  kernel")
for k in ks[:n]:
    x, y = a.get(k, (0, 0)), b.get(k, (0, 0))
    print(f"{x[0]:9.0f} {y[0]:8.0f}  {x[1]:7.0f} {y[1]:5.0f}  {k[:90]}")
print(f"total kernel time per step: {sum(v[0] for v in a.values()) / 1e3:.2f} ms -> {sum(v[0] for v in b.values()) / 1e3:.2f} ms")
