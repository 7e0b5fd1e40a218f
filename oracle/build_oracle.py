"""Build oracle/liboracle.so from oracle/bw_oracle.c (plain C, gcc, OpenMP).  TEST INFRASTRUCTURE ONLY.

There is no compiled reference to build into oracle/_ref: the reference
(DemianMArin/HMM_Training) is pure Python/NumPy, so the oracle is this C restatement, pinned by
the golden vectors in tests/golden/ that were produced by running the reference itself.

``build_asan()`` links the same source with oracle/asan_main.c (a driver over the oracle's entry
points, edge cases included) under AddressSanitizer + UBSan into oracle/_build/oracle_asan; the CPU
test suite runs it (tests/test_oracle_golden.py::test_oracle_under_asan).
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "bw_oracle.c")
CFLAGS = ["-O2", "-std=c99", "-Wall", "-Wextra", "-fno-fast-math", "-fopenmp"]


def build(verbose: bool = False) -> str:
    out = os.path.join(HERE, "liboracle.so")
    if os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(SRC) and \
            os.path.getmtime(out) >= os.path.getmtime(__file__):
        return out
    cmd = ["gcc", *CFLAGS, "-fPIC", "-shared", SRC, "-o", out + ".tmp", "-lm"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build_asan(verbose: bool = False) -> str:
    drv = os.path.join(HERE, "asan_main.c")
    os.makedirs(os.path.join(HERE, "_build"), exist_ok=True)
    out = os.path.join(HERE, "_build", "oracle_asan")
    srcs = [SRC, drv]
    if os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(p) for p in srcs):
        return out
    cmd = ["gcc", "-O1", "-g", "-std=c99", "-Wall", "-Wextra", "-fopenmp", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", *srcs, "-o", out, "-lm"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    print(build(verbose=True))
    print(build_asan(verbose=True))
