"""Summarise the loops of one kernel in a hipcc -S listing: per back-edge loop, instruction counts by
class (VALU / DPP / SALU / LDS / VMEM / waitcnt).  Diagnostics for kernel tuning.
    python tools/isa_loops.py <file.s> <kernel symbol substring>"""
import re
import sys
from collections import Counter


def main(path, name):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(name) + r"\S*:", l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, l in enumerate(body):
        m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\S+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))

    def classify(ins):
        op = ins.split()[0]
        if op.startswith("s_waitcnt"):
            return "waitcnt"
        if op.startswith("ds_"):
            return "lds"
        if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            return "vmem"
        if op.startswith("s_"):
            return "salu"
        if op.startswith("v_"):
            return "valu_dpp" if ("dpp" in ins or "row_" in ins or "quad_perm" in ins) else "valu"
        return "other"

    inner = [(a, b) for (a, b) in loops if not any(a <= a2 and b2 <= b and (a2, b2) != (a, b) for a2, b2 in loops)]
    for a, b in sorted(inner, key=lambda x: x[0]):
        c = Counter()
        ops = Counter()
        for l in body[a:b + 1]:
            s = l.strip()
            if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
                continue
            c[classify(s)] += 1
            ops[s.split()[0]] += 1
        print(f"loop lines {start + a + 1}-{start + b + 1}: {dict(c)}")
        print("   top ops:", ops.most_common(14))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
