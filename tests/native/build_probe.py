"""Build the test-only probe library tests/native/libucprobe.so (gfx950, the engine's atomics flags)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "uc_probe.hip")
OUT = os.path.join(HERE, "libucprobe.so")


def build(verbose: bool = False) -> str:
    if os.path.exists(OUT) and os.path.getmtime(OUT) >= os.path.getmtime(SRC):
        return OUT
    cmd = [os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), "-O2", "-std=c++17", "-fPIC", "-shared",
           f"--offload-arch={os.environ.get('HMMBW_ARCH', 'gfx950')}", "-munsafe-fp-atomics", SRC, "-o", OUT]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    print(build(verbose=True))
