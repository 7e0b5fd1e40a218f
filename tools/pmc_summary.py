"""Average per-dispatch PMC values of one kernel from tools/pmc_sq.sh output directories."""
import csv, glob, sys, collections
root, kern = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(list)
for f in glob.glob(f"{root}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
