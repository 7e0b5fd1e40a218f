"""Per-step instruction counts of the LR headline kernel's steady forward and backward loops (k_estep_join<8, 8>),
from a hipcc -S listing of the current sources (tools/isa_loops.steady_loops), written as JSON with the kernel
source hash (bench.py's phase model reads it):  python tools/isa_steps.py [out.json]"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import bench
    import isa_loops
    from hmm_training_amd import build as B
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r6", "isa_lr_steps.json")
    with tempfile.TemporaryDirectory() as td:
        s = os.path.join(td, "n8.s")
        cmd = [B.HIPCC, *[f for f in B.FLAGS if f not in ("-fPIC",)], "-DHMMBW_INST_N=8", "--cuda-device-only", "-S",
               os.path.join(B.CSRC, "estep_small_inst.hip"), "-o", s]
        subprocess.run(cmd, check=True, capture_output=True)
        loops = isa_loops.steady_loops(s, "k_estep_join")
    d = {"tool": "tools/isa_steps.py", "kernel": "k_estep_join<8,8>", "loops": loops,
         "kernel_src_sha16": bench.kernel_source_hash(), "collected_utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
         "note": "per step = per loop trip / 32 (4 chunks of 8 steps); f64 = fp64 VALU (4 cycles per wave64 on a SIMD-32), "
                 "v32 = other VALU incl. 32-bit DPP moves (2 cycles), lds includes the histogram ds_add_f64"}
    with open(out, "w") as fh:
        json.dump(d, fh, indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
