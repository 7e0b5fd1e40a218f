"""Build libhmmbw.so in-tree for gfx950 with hipcc (the driver's build() check runs this on CPU).

The engine is split into translation units that compile in parallel: the host/ABI unit
(csrc/hmmbw.hip), one small-N E-step instantiation unit per state count N = 1..16
(csrc/estep_small_inst.hip with -DHMMBW_INST_N=n) and the wide-N unit (csrc/estep_wide_inst.hip).
Objects go to hmm_training_amd/_obj/<tag>/ and are linked into one shared library.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
SRC = os.path.join(CSRC, "hmmbw.hip")
HDR = os.path.join(os.path.dirname(PKG), "include", "hmmbw.h")
OUT = os.path.join(PKG, "libhmmbw.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("HMMBW_ARCH", "gfx950")

FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
         "-Wall", "-Wno-unused-function"]
SMALL_N = range(1, 17)


def units():
    """(source, extra defines, object stem) of every translation unit."""
    # the wide (fp64 MFMA) kernels with LLVM's memory-clause scheduler: fewer spills in k_estep_mfma<4>
    # (31 VGPRs against 38) and the cfg5 shard's E-step 1,447 against 1,477 us (profiles/r5/ab_sched_strategy.txt)
    wide_flags = ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]
    u = [(SRC, [], "hmmbw"), (os.path.join(CSRC, "estep_wide_inst.hip"), wide_flags, "estep_wide"),
         (os.path.join(CSRC, "vq.hip"), [], "vq")]
    u += [(os.path.join(CSRC, "estep_small_inst.hip"), [f"-DHMMBW_INST_N={n}"], f"estep_small_n{n}")
          for n in SMALL_N]
    return u


def _jobs():
    env = os.environ.get("MAX_JOBS")
    if env and env.isdigit():
        return max(1, int(env))
    return max(1, min(16, os.cpu_count() or 1))


def build(force: bool = False, verbose: bool = False, defines=(), out: str = OUT, tag: str = "release",
          only=None) -> str:
    """Compile every unit (in parallel) and link `out`; skipped when `out` is newer than all sources.
    only: object stems to recompile (development: the other units' existing objects are relinked)."""
    sources = [HDR] + glob.glob(os.path.join(CSRC, "*"))
    stamp = max(os.path.getmtime(p) for p in sources)
    if not force and only is None and os.path.exists(out) and os.path.getmtime(out) >= stamp:
        return out
    objdir = os.path.join(PKG, "_obj", tag)
    os.makedirs(objdir, exist_ok=True)
    cmds = []
    for src, extra, stem in units():
        obj = os.path.join(objdir, stem + ".o")
        cmds.append((obj, [HIPCC, *FLAGS, *defines, *extra, "-c", src, "-o", obj]))
    links = [o for o, _ in cmds]
    if only is not None:
        cmds = [(o, c) for o, c in cmds if os.path.basename(o)[:-2] in set(only) or not os.path.exists(o)]

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if r.stderr.strip() and verbose:
            print(r.stderr, flush=True)

    # the heaviest units first so the pool drains evenly
    cmds.sort(key=lambda x: ("small_n" not in x[0], -int(x[0].rsplit("_n", 1)[-1][:-2]) if "small_n" in x[0] else 0))
    with cf.ThreadPoolExecutor(max_workers=_jobs()) as ex:
        list(ex.map(run, [c for _, c in cmds]))
    link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *links, "-o", out + ".tmp"]
    run(link)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    only = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--only=")]
    print(build(force="--force" in sys.argv, verbose=True, only=only[0].split(",") if only else None))
