"""Per-kernel totals of a rocprofv3 --pmc counter_collection CSV: counters summed over
dispatches, plus derived ratios (SQ cycle buckets, MFMA busy share, effective clock)."""
import collections
import csv
import sys

for f in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(float)
    n = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("eosv::", "")[:64]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Dispatch_Id"] not in n[k]:
            n[k].add(r["Dispatch_Id"])
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    print("==", f)
    for k in sorted(agg, key=lambda k: -dur[k]):
        if dur[k] < 1e-3:
            continue
        v = agg[k]
        s = f"{k:64s} n={len(n[k]):4d} {dur[k] * 1e3:8.2f} ms"
        wc = v.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in v:
                    s += f" {c[3:]}={v[c] / wc:.2f}"
        if "GRBM_GUI_ACTIVE" in v:
            s += f" clk={v['GRBM_GUI_ACTIVE'] / 8 / dur[k] / 1e9:.2f}GHz"
            if "SQ_VALU_MFMA_BUSY_CYCLES" in v:
                # MFMA busy cycles are summed over SIMDs: 256 CUs x 4 SIMDs
                s += f" mfma_busy={v['SQ_VALU_MFMA_BUSY_CYCLES'] / (v['GRBM_GUI_ACTIVE'] / 8) / 1024:.2f}"
        if "TCC_HIT_sum" in v and "TCC_MISS_sum" in v:
            s += f" L2hit={v['TCC_HIT_sum'] / max(1.0, v['TCC_HIT_sum'] + v['TCC_MISS_sum']):.3f}"
        for c in sorted(v):
            if c not in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                         "GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"):
                s += f" {c}={v[c]:.3e}"
        print(s)
