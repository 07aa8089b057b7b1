"""Instruction-mix summary of kernels in a hipcc -S (device) listing.

python tools/isa_stats.py file.s [substring]   -> per kernel: total and
per-basic-block counts of exp / fma / mul / add / dpp / permlane / cndmask /
LDS / global / SALU instructions (largest blocks first)."""
import collections
import re
import sys


def classify(i):
    if i.startswith("v_exp"):
        return "exp"
    if "_dpp" in i:
        return "dpp"
    if i.startswith("v_permlane"):
        return "permlane"
    if i.startswith("v_cndmask"):
        return "cndmask"
    if i.startswith(("v_fma", "v_fmac", "v_pk_fma")):
        return "fma"
    if i.startswith(("v_mul", "v_pk_mul")):
        return "mul"
    if i.startswith(("v_add", "v_pk_add", "v_sub")):
        return "add"
    if i.startswith("v_mfma"):
        return "mfma"
    if i.startswith("ds_"):
        return "lds"
    if i.startswith(("global_", "buffer_", "flat_")):
        return "gmem"
    if i.startswith("s_waitcnt"):
        return "wait"
    if i.startswith("s_"):
        return "salu"
    if i.startswith("v_"):
        return "v_other"
    return i


def main():
    s = open(sys.argv[1]).read()
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    for m in re.finditer(r"^(_Z\w+):.*?$(.*?)^\.Lfunc_end", s, re.S | re.M):
        name, body = m.group(1), m.group(2)
        if pat not in name:
            continue
        blocks, cur, label = [], collections.Counter(), "entry"
        tot = collections.Counter()
        for line in body.splitlines():
            l = line.split(";")[0].strip()
            if l.endswith(":") and not l.startswith(";"):
                blocks.append((label, cur))
                cur, label = collections.Counter(), l[:-1]
                continue
            if not l or l.startswith((";", ".", "//")):
                continue
            if False:
                blocks.append((label, cur))
                cur, label = collections.Counter(), l[:-1]
                continue
            k = classify(l.split()[0])
            cur[k] += 1
            tot[k] += 1
        blocks.append((label, cur))
        print(f"== {name}  total {sum(tot.values())}: {dict(tot.most_common())}")
        for lab, c in sorted(blocks, key=lambda x: -sum(x[1].values()))[:4]:
            print(f"   {lab:16s} {sum(c.values()):5d}: {dict(c.most_common())}")


if __name__ == "__main__":
    main()
