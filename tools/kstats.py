"""Summarise / diff rocprofv3 kernel_stats.csv files: python tools/kstats.py A.csv [B.csv] [--per N]"""
import csv
import sys

per = 1.0
argv = list(sys.argv[1:])
if "--per" in argv:
    i = argv.index("--per")
    per = float(argv[i + 1])
    del argv[i:i + 2]
args = [a for a in argv if not a.startswith("--")]


def load(p):
    d = {}
    for r in csv.DictReader(open(p)):
        d[r["Name"][:100]] = (float(r["TotalDurationNs"]) / 1e3 / per, int(r["Calls"]) / per)
    return d


A = load(args[0])
B = load(args[1]) if len(args) > 1 else {}
keys = sorted(set(A) | set(B), key=lambda k: -max(A.get(k, (0, 0))[0], B.get(k, (0, 0))[0]))
print(f"{'A us':>10} {'calls':>6} {'B us':>10} {'calls':>6}  name")
for k in keys[:45]:
    a, b = A.get(k, (0, 0)), B.get(k, (0, 0))
    print(f"{a[0]:10.1f} {a[1]:6.1f} {b[0]:10.1f} {b[1]:6.1f}  {k}")
print(f"total A {sum(v[0] for v in A.values()):.1f} us  B {sum(v[0] for v in B.values()):.1f} us")
