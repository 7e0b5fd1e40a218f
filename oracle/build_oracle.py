"""Build oracle/liboracle.so from oracle/bw_oracle.c (plain C, gcc).  TEST INFRASTRUCTURE ONLY.

There is no compiled reference to build into oracle/_ref: the reference
(DemianMArin/HMM_Training) is pure Python/NumPy, so the oracle is this C restatement, pinned by
the golden vectors in tests/golden/ that were produced by running the reference itself.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def build(verbose: bool = False) -> str:
    src = os.path.join(HERE, "bw_oracle.c")
    out = os.path.join(HERE, "liboracle.so")
    if os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(src):
        return out
    cmd = ["gcc", "-O2", "-fPIC", "-shared", "-std=c99", "-Wall", "-Wextra", "-fno-fast-math", src, "-o", out, "-lm"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    print(build(verbose=True))
