"""Conv-family HBM traffic per launch from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes,
one pair per dtype (tools/gpu_traffic.sh), written as profiles/<tag>_traffic.json.  bench.py and
tools/bench_configs.py attach it as roofline.traffic only to the same workload (key) on the same
kernel sources (src_sha16).

  python tools/traffic_json.py <out.json> <dir> <dtype> [<dtype> ...]

<dir>/<dtype>_FETCH_SIZE/ and <dir>/<dtype>_WRITE_SIZE/ hold the counter CSVs of two runs of the
same command at that dtype (its secondary legs off), <dir>/<dtype>_FETCH_SIZE.log that run's JSON
line.  Like for like: from that line come the workload key, the number of conv-family launches of
the timed region (roofline.conv_launches) and their algorithmic bytes per launch
(roofline.traffic_algorithmic); the measured figure sums the counters over exactly those launches,
the LAST conv_launches conv-family dispatches of the run (Dispatch_Id order: warmup and setup
launches come first).  The family is every kernel the library's conv profile records cover: the
stems, the implicit GEMMs, the row / strip kernels and the fused pairs.

HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: rocprofv3 reports KiB and on gfx950
FETCH_SIZE counts half of the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM section)."""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "embodied-one-shot-video-recognition_amd"))
from eosv._lib import source_digest  # noqa: E402

FAMILIES = {"f32": ("conv_f32", "conv_rows_f32", "stem_pool_f32"),
            "bf16": ("conv_bf16", "conv_rows_bf16", "conv_strip_bf16", "stem_pool_bf16", "pair1x1_bf16", "pairw_bf16"),
            "f32x3": ("conv_bf16", "conv_rows_x3", "stem_pool_x3")}


def short(name):
    return name.split("(")[0].replace("void ", "").replace("eosv::", "")


def dispatches(d):
    """[(dispatch id, kernel, KiB)] of one PMC pass, in dispatch order."""
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            rows.append((int(r["Dispatch_Id"]), short(r["Kernel_Name"]), float(r["Counter_Value"])))
    return sorted(rows)


def bench_line(path):
    for line in open(path):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


def one_dtype(d, dtype):
    line = bench_line(os.path.join(d, f"{dtype}_FETCH_SIZE.log"))
    rl = line["roofline"]
    n = int(rl["conv_launches"])
    out, kernels = {}, {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        fam = [r for r in dispatches(os.path.join(d, f"{dtype}_{c}")) if r[1].startswith(FAMILIES[dtype])]
        if len(fam) < n:
            raise SystemExit(f"{dtype} {c}: {len(fam)} conv-family dispatches, the timed region has {n}")
        last = fam[-n:]
        out[c] = sum(v for _, _, v in last)
        for _, k, v in last:
            e = kernels.setdefault(k, {"launches": 0, "FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0})
            e[c] += v
            if c == "FETCH_SIZE":
                e["launches"] += 1
    hbm = (2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024 / n
    alg = rl.get("traffic_algorithmic")
    res = {"launches": n, "hbm_bytes_per_launch": round(hbm),
           "algorithmic_bytes_per_launch": alg, "ratio": round(hbm / alg, 3) if alg else None,
           "profiled_line": {"value": line.get("value"), "unit": line.get("unit"), "dtype": line.get("dtype"),
                             "steps": line.get("steps"), "warmup": line.get("warmup")}}
    kb = {k: {"launches": e["launches"],
              "hbm_mb_per_launch": round((2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024 / e["launches"] / 1e6, 2),
              "fetch_kib_per_launch": round(e["FETCH_SIZE"] / e["launches"], 1),
              "write_kib_per_launch": round(e["WRITE_SIZE"] / e["launches"], 1)} for k, e in sorted(kernels.items())}
    return rl["traffic_key"], res, kb


def main():
    out, d, dtypes = sys.argv[1], sys.argv[2], sys.argv[3:]
    doc = {"source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes per dtype ({d})",
           "formula": "(2 x FETCH_SIZE + WRITE_SIZE) x 1024 B per launch over the timed region's conv-family "
                      "launches (the last roofline.conv_launches family dispatches of the profiled run)",
           "src_sha16": source_digest(), "kernels": {}}
    for dt in dtypes:
        key, res, kb = one_dtype(d, dt)
        if doc.get("key", key) != key:
            raise SystemExit(f"dtype {dt}: workload {key} differs from {doc['key']}")
        doc["key"] = key
        doc[dt] = res
        doc["kernels"][dt] = kb
        print(dt, json.dumps(res))
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    json.dump(doc, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
