"""Average PMC counters per kernel instantiation from scripts/pmc_bench.sh output."""
import csv, glob, sys, collections, re
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcb"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        k = re.sub(r"\(rdn_.*", "", k)
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
only = sys.argv[2] if len(sys.argv) > 2 else ""
for k, d in sorted(acc.items()):
    if only and not re.search(only, k):
        continue
    print(k[:90])
    print("   " + "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(d.items())))
