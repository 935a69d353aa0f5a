"""Summarise a tools/gpu_round.sh run into profiles/<tag>_summary.md.

Inputs (gpurun_out/): prof/trace/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats of
the default bench command), prof/pmc_{FETCH,WRITE}_SIZE/<tag>_counter_collection.csv
(separate PMC passes), bench.log (the JSON line).

HBM traffic per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 B: rocprofv3 reports KiB, and
on gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads
(MI355X_MICROARCH.md, HBM section).
"""
import collections
import csv
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
dst = sys.argv[3] if len(sys.argv) > 3 else "profiles"
os.makedirs(dst, exist_ok=True)


def short(name):
    return name.split("(")[0].replace("void ", "").replace("eosv::", "")[:70]


stats = list(csv.DictReader(open(f"{src}/prof/trace/{tag}_kernel_stats.csv")))
pmc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    p = f"{src}/prof/pmc_{c}/{tag}_counter_collection.csv"
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        k = short(r["Kernel_Name"])
        pmc[k][c] += float(r["Counter_Value"])
        cnt[k][c] += 1

bench = None
for line in open(f"{src}/bench.log"):
    if line.startswith("{"):
        bench = json.loads(line)

out = [f"# {tag} profile summary", "",
       "Command: `python bench.py --no-cpu-baseline` under `rocprofv3 --kernel-trace --stats` "
       "(f32 primary + bf16 and f32x3 secondary legs); PMC passes `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` "
       "on `--steps 2` of the same command.", ""]
if bench:
    rl = bench["roofline"]
    out += ["## bench line (same box, un-profiled run)", "",
            f"- value **{bench['value']} clips/s** ({bench['dtype']}), {bench['frames_per_s']} frames/s, "
            f"ms/step {bench['ms_per_step']}, episode acc {bench['episode_acc']}",
            f"- roofline: achieved {rl['achieved']} TF/s of {rl['peak']} ({rl['frac'] * 100:.1f} %), "
            f"end-to-end {rl.get('end_to_end_tflops')} TF/s",
            ]
    for key in [k for k in bench if k.startswith("secondary")]:
        s = bench[key]
        out.append(f"- secondary {s['dtype']}: {s['value']} clips/s, roofline {s['roofline']['achieved']} TF/s "
                   f"({s['roofline']['frac'] * 100:.1f} % of {s['roofline']['peak']}), prediction agreement "
                   f"{s['prediction_agreement_vs_primary']}, embeddings max rel vs primary "
                   f"{s.get('embedding_max_rel_vs_primary')}")
    if bench.get("cpu_baseline"):
        cb = bench["cpu_baseline"]
        out.append(f"- cpu_baseline: {cb['value']} clips/s on {cb['cores']} cores ({cb['kind']})")
    out.append("")
out += ["## kernel stats (rocprofv3 --stats)", "",
        "| kernel | calls | avg us | total ms | % | HBM MB/launch (2xFETCH+WRITE) |", "|---|---|---|---|---|---|"]
for r in stats:
    k = short(r["Name"])
    tot = float(r["TotalDurationNs"]) / 1e6
    if tot < 0.05:
        continue
    traffic = ""
    if k in pmc and cnt[k].get("FETCH_SIZE"):
        mb = (2 * pmc[k]["FETCH_SIZE"] / cnt[k]["FETCH_SIZE"] + pmc[k]["WRITE_SIZE"] / max(1, cnt[k]["WRITE_SIZE"])) / 1024
        traffic = f"{mb:.1f}"
    out.append(f"| `{k}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {tot:.2f} | {float(r['Percentage']):.2f} | {traffic} |")
open(f"{dst}/{tag}_summary.md", "w").write("\n".join(out) + "\n")
shutil.copy(f"{src}/prof/trace/{tag}_kernel_stats.csv", f"{dst}/{tag}_kernel_stats.csv")
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    p = f"{src}/prof/pmc_{c}/{tag}_counter_collection.csv"
    if os.path.exists(p):
        shutil.copy(p, f"{dst}/{tag}_pmc_{c}.csv")
if bench:
    open(f"{dst}/{tag}_bench.json", "w").write(json.dumps(bench) + "\n")

# HBM traffic (roofline.traffic) is written by tools/traffic_json.py from PMC passes over the
# library's profiling window (tools/gpu_traffic.sh), not here: whole-run counters mix warmup and
# setup dispatches into the figure
print("\n".join(out))
