"""Conv-family HBM traffic per launch from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
of one command, written as a profiles/<tag>_traffic.json that bench.py / bench_configs.py attach
as roofline.traffic only to the same workload (key) on the same kernel sources (src_sha16).

  python tools/traffic_json.py <fetch counter_collection.csv> <write counter_collection.csv> \
      <out.json> <key> <dtype> [source note]

HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: rocprofv3 reports KiB and on gfx950
FETCH_SIZE counts half of the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM section)."""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "embodied-one-shot-video-recognition_amd"))
from eosv._lib import source_digest  # noqa: E402

FAMILIES = {"f32": ("conv_f32", "conv_rows_f32", "stem_pool_f32"),
            "bf16": ("conv_bf16", "conv_rows_bf16", "stem_pool_bf16", "pair1x1_bf16", "pairw_bf16"),
            "f32x3": ("conv_bf16", "conv_rows_x3", "stem_pool_x3")}


def per_kernel(path):
    tot, n = collections.defaultdict(float), collections.defaultdict(int)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("eosv::", "")
        tot[k] += float(r["Counter_Value"])
        n[k] += 1
    return tot, n


def main():
    fetch, write, out, key, dtype = sys.argv[1:6]
    note = sys.argv[6] if len(sys.argv) > 6 else ""
    ft, fn = per_kernel(fetch)
    wt, wn = per_kernel(write)
    keys = [k for k in ft if any(f in k for f in FAMILIES[dtype])]
    launches = sum(fn[k] for k in keys)
    fetch_kib = sum(ft[k] for k in keys)
    write_kib = sum(wt.get(k, 0.0) for k in keys)
    wl = sum(wn.get(k, 0) for k in keys) or 1
    d = {"source": note or f"{fetch} + {write}",
         "formula": "(2 x FETCH_SIZE + WRITE_SIZE) x 1024 B per launch, averaged over the conv family",
         "key": key, "src_sha16": source_digest(),
         dtype: {"launches": launches,
                 "hbm_bytes_per_launch": round((2 * fetch_kib / max(1, launches) + write_kib / wl) * 1024)},
         "kernels": {k: {"launches": fn[k], "fetch_kib_per_launch": round(ft[k] / fn[k], 1),
                         "write_kib_per_launch": round(wt.get(k, 0.0) / max(1, wn.get(k, 0)), 1)} for k in keys}}
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d[dtype]))


if __name__ == "__main__":
    main()
