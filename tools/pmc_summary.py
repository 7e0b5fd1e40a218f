"""Average per-dispatch PMC values of the named kernels from a rocprofv3 counter_collection CSV (or a
tools/pmc_sq.sh output directory), as JSON, with the derived LDS bank-conflict rate
(SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE: extra cycles / all LDS-array cycles, MI355X_MICROARCH.md §LDS)
and VALU / LDS instructions per wave.

    python tools/pmc_summary.py <csv or dir> <kernel substring[,substring...]> [--config-key KEY]
        [--kernel-stats run_kernel_stats.csv]

With GRBM_GUI_ACTIVE in the pass and the kernel's mean duration from a kernel-trace stats CSV of the same
workload, also the loaded clock (GRBM_GUI_ACTIVE / 8 XCDs / duration, MI355X_MICROARCH.md DVFS note).
"""
import collections
import csv
import glob
import json
import time
import os
import sys



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

def mean_ns(stats_csv, kern):
    rows = [r for r in csv.DictReader(open(stats_csv)) if kern in r["Name"]]
    return sum(float(r["AverageNs"]) for r in rows) / len(rows) if rows else None


def main(src, kernels, config_key=None, kernel_stats=None):
    files = []
    for one in src.split(","):  # several CSVs (separate counter passes of the same workload) merge
        files += [one] if os.path.isfile(one) else glob.glob(f"{one}/p*/run_counter_collection.csv")
    out = {}
    for kern in kernels.split(","):
        vals = collections.defaultdict(list)
        for f in files:
            for r in csv.DictReader(open(f)):
                if kern in r["Kernel_Name"]:
                    vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        d = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
        if d.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_bank_conflict_fraction"] = d.get("SQ_LDS_BANK_CONFLICT", 0.0) / d["SQ_LDS_IDX_ACTIVE"]
        if d.get("SQ_WAVES"):
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS"):
                if c in d:
                    d[c.lower() + "_per_wave"] = d[c] / d["SQ_WAVES"]
        f64 = sum(d.get(c, 0.0) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                          "SQ_INSTS_VALU_TRANS_F64"))
        if "SQ_INSTS_VALU_FMA_F64" in d:
            d["valu_fp64_insts"] = f64  # 4-cycle issue on a SIMD-32 (half the fp32 rate); the rest 2 cycles
        d["dispatches"] = max((len(v) for v in vals.values()), default=0)
        if config_key:
            d["config_key"] = config_key
        if kernel_stats and d.get("GRBM_GUI_ACTIVE"):
            ns = mean_ns(kernel_stats, kern)
            if ns:
                d["kernel_ns_trace"] = ns
                d["clock_ghz"] = d["GRBM_GUI_ACTIVE"] / 8.0 / ns
        out[kern] = _stamp(d)
    print(json.dumps(out, indent=2))


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("kernels")
    ap.add_argument("--config-key")
    ap.add_argument("--kernel-stats")
    a = ap.parse_args()
    main(a.src, a.kernels, a.config_key, a.kernel_stats)
