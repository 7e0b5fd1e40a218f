#!/usr/bin/env python3
"""Per-launch HBM traffic of a kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE CSVs (separate
passes), corrected with the calibration run of tools/pmc_calib.hip (MI355X_MICROARCH.md §HBM:
FETCH_SIZE under-reports wide coalesced reads; WRITE_SIZE exact for streaming stores; both in KiB).

  python tools/traffic_summary.py --fetch F.csv --write W.csv --calib-fetch CF.csv --calib-write CW.csv \
      --kernel k_estep_small --config-key R10000_T200_N8_K256_left_to_right --out profiles/r1/traffic.json
"""
import argparse
import csv
import json
import os
import time
from statistics import mean



def _stamp(d):
    """Provenance of a summary: UTC collection time and the kernel-source hash of the tree it was collected
    on (bench.kernel_source_hash), so bench.py can tell a bound from a stale profile."""
    import sys as _sys
    _sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    # the profiling run's own record (tools/profile_all.sh writes both on the box), else this tree's
    d["collected_utc"] = os.environ.get("HMMBW_PROFILE_UTC") or time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
    d["kernel_src_sha16"] = os.environ.get("HMMBW_PROFILE_SHA") or bench.kernel_source_hash()
    return d

def per_kernel(path, name_sub, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if name_sub in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit(f"no {counter} rows for {name_sub} in {path}")
    return vals


def per_launch(path, names, counter):
    """Mean per launch of the E-step, summed over its kernels (comma-separated substrings)."""
    return sum(mean(per_kernel(path, n, counter)) for n in names.split(","))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--calib-fetch", required=True)
    ap.add_argument("--calib-write", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--config-key", required=True)
    ap.add_argument("--calib-bytes", type=float, default=float(1 << 30))
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    kib = 1024.0
    # calibration: KiB reported per known byte count, 8-B-per-lane access (k_read8 / k_write8)
    cf = a.calib_bytes / (mean(per_kernel(a.calib_fetch, "k_read8", "FETCH_SIZE")) * kib)
    cw = a.calib_bytes / (mean(per_kernel(a.calib_write, "k_write8", "WRITE_SIZE")) * kib)
    f = per_launch(a.fetch, a.kernel, "FETCH_SIZE")
    w = per_launch(a.write, a.kernel, "WRITE_SIZE")
    rd = f * kib * cf
    wr = w * kib * cw
    out = {"kernel": a.kernel, "config_key": a.config_key,
           "launches": [len(per_kernel(a.fetch, a.kernel.split(",")[0], "FETCH_SIZE")),
                        len(per_kernel(a.write, a.kernel.split(",")[0], "WRITE_SIZE"))],
           "fetch_size_kib_mean": f, "write_size_kib_mean": w,
           "calibration": {"fetch_factor": cf, "write_factor": cw, "access": "8 B per lane, 1 GiB streams"},
           "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
           "hbm_bytes_per_launch": rd + wr,
           "note": "L2-miss (fabric) bytes: Infinity-Cache hits are counted, as on every gfx950 PMC read"}
    _stamp(out)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
