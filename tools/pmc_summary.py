"""Summarise rocprofv3 --pmc counter_collection CSVs per kernel (sum over dispatches)."""
import collections
import csv
import glob
import sys

for path in sys.argv[1:]:
    for f in sorted(glob.glob(path)):
        rows = list(csv.DictReader(open(f)))
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        dur = collections.defaultdict(float)
        seen = set()
        for r in rows:
            k = r["Kernel_Name"].split("(")[0][-60:]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if (r["Dispatch_Id"], k) not in seen:
                seen.add((r["Dispatch_Id"], k))
                dur[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        print("==", f)
        for k, v in sorted(agg.items(), key=lambda kv: -dur[kv[0]]):
            if dur[k] < 1e6:
                continue
            print(f"  {k}  dur {dur[k] / 1e6:.2f} ms  " + "  ".join(f"{c}={x:.3e}" for c, x in sorted(v.items())))
