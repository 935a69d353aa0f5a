#!/usr/bin/env python3
"""Training-step profile summary: rocprofv3 --kernel-trace --stats CSV of tools/bench_train.py
(tools/gpu_train_prof.sh) -> a markdown table with the time split by kernel class.

  python tools/train_profile_md.py gpurun_out/prof/train/r05t_kernel_stats.csv gpurun_out/train_bench.log \
      profiles/r05t_train_profile.md r05t
"""
import csv
import json
import sys

stats_path, bench_log, out, tag = sys.argv[1:5]
rows = list(csv.DictReader(open(stats_path)))
line = [json.loads(l) for l in open(bench_log) if l.startswith("{")][-1]


def cls(name):
    n = name.lower()
    if "bn_" in n:
        return "BN passes"
    if "gemm_f32" in n or "gemm_slice_sum" in n:
        return "in-tree GEMMs (gemm_f32.hip: stem, strided dgrad, 1x1 / stem wgrad, fc)"
    if "cijk" in n or "rocblas" in n:
        return "rocBLAS"
    if "wgrad" in n:
        return "weight gradient (wgrad_f32.hip)"
    if "conv_" in n or "ksplit" in n:
        return "conv forward / dgrad (conv_f32*.hip)"
    if "im2col" in n or "col2im" in n:
        return "im2col / col2im"
    return "other (pool, SGD, sums, flips, copies)"


tot = sum(float(r["TotalDurationNs"]) for r in rows)
split = {}
for r in rows:
    split[cls(r["Name"])] = split.get(cls(r["Name"]), 0.0) + float(r["TotalDurationNs"])
with open(out, "w") as f:
    f.write(f"# {tag} training-step profile (R50, 6 clips x 16 frames, 224x224, f32)\n\n")
    f.write("Command: `rocprofv3 --kernel-trace --stats -- python tools/bench_train.py` (tools/gpu_train_prof.sh; "
            "1 warmup + 5 timed steps, all 6 in the trace).\n\n")
    f.write(f"Bench line of the un-profiled run: {line['clips_per_s']} clips/s, {line['ms_per_step']} ms/step "
            f"(torch-CPU baseline {line.get('cpu_baseline', {}).get('clips_per_s')} clips/s).\n\n")
    f.write(f"Kernel time over the 6 steps: {tot / 1e6:.1f} ms ({tot / 6e6:.1f} ms per step).\n\n")
    f.write("Split: " + ", ".join(f"{k} {100 * v / tot:.1f} %" for k, v in sorted(split.items(), key=lambda t: -t[1]))
            + ".\n\n")
    f.write("| kernel | calls | avg us | total ms | % |\n|---|---|---|---|---|\n")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
        name = r["Name"].replace("|", "/")[:90]
        f.write(f"| `{name}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                f"{float(r['TotalDurationNs']) / 1e6:.2f} | {100 * float(r['TotalDurationNs']) / tot:.1f} |\n")
print(open(out).read()[:1500])
