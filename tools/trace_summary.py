"""Per-kernel time of one graph-replayed step from a rocprofv3 kernel trace:
python tools/trace_summary.py <kernel_trace.csv> <marker-substring> [steps]
Steps are delimited by kernels whose name contains the marker (e.g. ArgMax)."""
import collections
import csv
import re
import sys


def short(n):
    m = re.search(r"(\w+_kernel\w*)(<[^()]*>)?", n)
    return (m.group(1) + (m.group(2) or ""))[:70] if m else n[:70]


def main(path, marker, nsteps=20):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    am = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    seg = list(zip(am[-nsteps - 1:-1], am[-nsteps:]))
    tot, cnt = collections.Counter(), collections.Counter()
    wall = busy = 0
    for a, b in seg:
        wall += int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])
        for r in rows[a + 1:b + 1]:
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            k = short(r["Kernel_Name"])
            tot[k] += d
            cnt[k] += 1
            busy += d
    S = len(seg)
    print(f"steps {S}: wall {wall / S / 1e3:.1f} us, kernel busy {busy / S / 1e3:.1f} us, "
          f"{sum(cnt.values()) / S:.0f} kernels/step")
    for k, v in tot.most_common(40):
        print(f"{v / S / 1e3:8.1f} us {cnt[k] / S:5.1f}x {v / cnt[k] / 1e3:6.2f} us/call  {k}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 20)
