"""Per-kernel mean PMC values of a tools/profile_mix.sh run (all passes): python tools/mix_summary.py <dir> [kernels]"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from parse_prof import short  # noqa: E402


def summary(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            per[(r["Dispatch_Id"], short(r["Kernel_Name"]), r["Counter_Name"])] += float(r["Counter_Value"])
        for (did, k, c), v in per.items():
            acc[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


if __name__ == "__main__":
    s = summary(sys.argv[1])
    want = sys.argv[2:] or sorted(s)
    for k in want:
        if k in s:
            print(k)
            for c, v in sorted(s[k].items()):
                print(f"   {c:28s} {v:.4g}")
