"""Mean counter value per dispatch of each kernel in the counter_collection CSVs under a
directory (tools/bn_pmc.sh output): python tools/bn_pmc_sum.py gpurun_out/bnpmc"""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: [0, 0.0])
for path in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    with open(path) as f:
        for r in csv.DictReader(f):
            k = (r["Kernel_Name"][:60], r["Counter_Name"])
            acc[k][0] += 1
            acc[k][1] += float(r["Counter_Value"])
for (kern, ctr), (n, s) in sorted(acc.items()):
    print(f"{kern:60s} {ctr:14s} n={n:4d} mean={s / n:14.1f}")
