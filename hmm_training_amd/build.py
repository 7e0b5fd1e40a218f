"""Build libhmmbw.so in-tree for gfx950 with hipcc (the driver's build() check runs this on CPU)."""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(PKG, "csrc", "hmmbw.hip")
HDR = os.path.join(os.path.dirname(PKG), "include", "hmmbw.h")
OUT = os.path.join(PKG, "libhmmbw.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("HMMBW_ARCH", "gfx950")

FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
         "-Wall", "-Wno-unused-function"]


def build(force: bool = False, verbose: bool = False) -> str:
    stamp = max(os.path.getmtime(SRC), os.path.getmtime(HDR))
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= stamp:
        return OUT
    cmd = [HIPCC, *FLAGS, SRC, "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
