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


F64_OPS = ("v_fma_f64", "v_fmac_f64", "v_mul_f64", "v_add_f64", "v_ldexp_f64", "v_max_f64", "v_min_f64",
           "v_rcp_f64", "v_div", "v_cmp_", "v_cndmask")


def steady_loops(path, name, steps_per_trip=32):
    """Per-step instruction counts of the steady (leanest) forward and backward loops of one small E-step kernel:
    backward = loops with ds_add_f64 (the histogram), forward = loops with row_shr DPP and ds_read_b128 but no
    ds_add_f64; of each, the one with the fewest instructions (the unmasked full-wave loop).  Classes: f64 (fp64
    VALU: 4 cycles per wave64 on a SIMD-32), v32 (other VALU incl. 32-bit DPP moves: 2), lds, vmem, salu,
    waitcnt, nop."""
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(name) + r"\S*:", l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    labels = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r"^(\.LBB\S+):", l)] if m}
    loops = []
    for i, l in enumerate(body):
        m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\S+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))
    inner = [(a, b) for (a, b) in loops if not any(a <= a2 and b2 <= b and (a2, b2) != (a, b) for a2, b2 in loops)]

    def classes(a, b):
        c = Counter()
        for l in body[a:b + 1]:
            s = l.strip()
            if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
                continue
            op = s.split()[0]
            if op.startswith("s_waitcnt"):
                c["waitcnt"] += 1
            elif op.startswith("s_nop"):
                c["nop"] += 1
            elif op.startswith("ds_"):
                c["lds"] += 1
                if op.startswith("ds_add_f64"):
                    c["lds_atomic"] += 1
            elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
                c["vmem"] += 1
            elif op.startswith("s_"):
                c["salu"] += 1
            elif op.startswith("v_"):
                is64 = ("_f64" in op) and not op.startswith(("v_cmp", "v_cndmask"))
                c["f64" if is64 else "v32"] += 1
                if "dpp" in s or "row_" in s or "quad_perm" in s:
                    c["dpp"] += 1
        return c

    fwd, bwd = [], []
    for a, b in inner:
        c = classes(a, b)
        txt = "\n".join(body[a:b + 1])
        if c["lds_atomic"] and "ds_read_b128" in txt:
            bwd.append((sum(v for k, v in c.items() if k not in ("lds_atomic", "dpp")), a, c))
        elif "row_shr" in txt and "ds_read_b128" in txt and not c["lds_atomic"]:
            fwd.append((sum(v for k, v in c.items() if k not in ("lds_atomic", "dpp")), a, c))
    out = {}
    for nm, cand in (("forward", fwd), ("backward", bwd)):
        if not cand:
            continue
        tot, a, c = min(cand, key=lambda x: x[0])
        out[nm] = {"loop_first_line": start + a + 1, "candidates": len(cand), "steps_per_trip": steps_per_trip,
                   "per_step": {k: v / steps_per_trip for k, v in sorted(c.items())}}
    return out


if __name__ == "__main__" and False:
    pass
