"""Conv-family HBM traffic per launch from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes,
one pair per dtype (tools/gpu_traffic.sh), written as profiles/<tag>_traffic.json.  bench.py and
tools/bench_configs.py attach it as roofline.traffic only to the same workload (key) on the same
kernel sources (src_sha16), the build configuration (lib_kind) and, for information, the library's
bytes (lib_sha16).

  python tools/traffic_json.py <out.json> <dir> <dtype> [<dtype> ...]

<dir>/<dtype>_FETCH_SIZE/ and <dir>/<dtype>_WRITE_SIZE/ hold the counter CSVs of two runs of the
same command at that dtype (its secondary legs off), <dir>/<dtype>_FETCH_SIZE.log that run's JSON
line.  Like for like (r05): the timed region is the profiling window the library brackets with
two marker dispatches (eosv_profile_enable: profile_window_begin_kernel ... profile_window_end_kernel,
the last such window of the run); the measured figure sums the counters over the conv-family
dispatches inside it, and their number must equal the line's roofline.conv_launches (the launches
its traffic_algorithmic covers) -- nothing is back-filled from warmup or setup dispatches.  The
family is every kernel the library's conv profile records cover (the stems, the implicit GEMMs,
the row / strip kernels and the fused pairs: names starting conv_, stem_pool_, pair1x1 (both
pair1x1_bf16 and the r04 pair1x1r_bf16), pairw_, bneck_, bblock_ or bblock2_ (the r06 whole-block stage-1
kernels));
the other kernels of the window (clip
embedding, matching) are listed under "other_in_window".

HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: rocprofv3 reports KiB and on gfx950
FETCH_SIZE counts half of the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM section)."""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "embodied-one-shot-video-recognition_amd"))
from eosv._lib import library_digest, library_kind, source_digest  # noqa: E402

FAMILY = ("conv_", "stem_pool_", "pair1x1", "pairw_", "bneck_", "bblock_", "bblock2_")
BEGIN, END = "profile_window_begin_kernel", "profile_window_end_kernel"


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


def window(rows):
    """The dispatches strictly inside the run's last profiling window (marker kernels)."""
    begins = [i for i, r in enumerate(rows) if r[1] == BEGIN]
    if not begins:
        raise SystemExit("no profile_window_begin_kernel dispatch: library without window markers")
    b = begins[-1]
    ends = [i for i in range(b + 1, len(rows)) if rows[i][1] == END]
    if not ends:
        raise SystemExit("profiling window never closed (no profile_window_end_kernel after the last begin)")
    return rows[b + 1:ends[0]]


def one_dtype(d, dtype):
    line = bench_line(os.path.join(d, f"{dtype}_FETCH_SIZE.log"))
    rl = line["roofline"]
    n = int(rl["conv_launches"])
    out, kernels, other = {}, {}, {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        win = window(dispatches(os.path.join(d, f"{dtype}_{c}")))
        fam = [r for r in win if r[1].startswith(FAMILY)]
        if len(fam) != n:
            raise SystemExit(f"{dtype} {c}: {len(fam)} conv-family dispatches in the profiling window, "
                             f"the timed region records {n} conv launches")
        out[c] = sum(v for _, _, v in fam)
        for _, k, v in fam:
            e = kernels.setdefault(k, {"launches": 0, "FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0})
            e[c] += v
            if c == "FETCH_SIZE":
                e["launches"] += 1
        if c == "FETCH_SIZE":
            for _, k, _ in win:
                if not k.startswith(FAMILY):
                    other[k] = other.get(k, 0) + 1
    launches = {k: e["launches"] for k, e in kernels.items()}
    wl = {}
    for _, k, _ in [r for r in window(dispatches(os.path.join(d, f"{dtype}_WRITE_SIZE"))) if r[1].startswith(FAMILY)]:
        wl[k] = wl.get(k, 0) + 1
    if wl != launches:
        raise SystemExit(f"{dtype}: the FETCH_SIZE and WRITE_SIZE passes launched different conv kernels")
    hbm = (2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024 / n
    alg = rl.get("traffic_algorithmic")
    res = {"launches": n, "hbm_bytes_per_launch": round(hbm), "other_in_window": other,
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
           "formula": "(2 x FETCH_SIZE + WRITE_SIZE) x 1024 B per launch over the conv-family dispatches inside "
                      "the profiled run's timed window (between the library's window marker kernels); their count "
                      "equals roofline.conv_launches",
           "src_sha16": source_digest(), "lib_kind": library_kind(), "lib_sha16": library_digest(), "kernels": {}}
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
