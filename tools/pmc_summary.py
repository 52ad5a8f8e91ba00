"""Summarise rocprofv3 --pmc passes (tools/pmc.sh output) for the classify kernel.

Averages every counter over the classify_kernel dispatches of each pass and
prints one JSON object.  With --traffic, also writes profiles/pmc_traffic.json
(HBM bytes per launch for bench.py's roofline.traffic): FETCH_SIZE is reported
in KiB and, on gfx950, at half the bytes of 16-B-per-lane reads
(MI355X_MICROARCH.md, HBM section), so bytes = FETCH_SIZE * 1024 * 2."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def collect(tag_dir, kernel="classify"):
    out = {}
    for path in sorted(glob.glob(os.path.join(tag_dir, "p*", "*counter_collection.csv"))):
        per = defaultdict(lambda: defaultdict(float))
        meta = {}
        with open(path) as fh:
            for row in csv.DictReader(fh):
                if kernel not in row["Kernel_Name"]:
                    continue
                d = int(row["Dispatch_Id"])
                per[d][row["Counter_Name"]] += float(row["Counter_Value"])
                meta = {k: row[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count",
                                            "SGPR_Count", "Scratch_Size")}
        if not per:
            continue
        names = sorted({c for v in per.values() for c in v})
        for c in names:
            vals = [v[c] for v in per.values() if c in v]
            out[c] = sum(vals) / len(vals)
        out["dispatches_" + os.path.basename(os.path.dirname(path))] = len(per)
        out.setdefault("meta", meta)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag_dir")
    ap.add_argument("--traffic", action="store_true")
    ap.add_argument("--frames", type=int, default=1 << 24)
    ap.add_argument("--out", default="")
    ap.add_argument("--key", default="config3", help="pmc_traffic.json entry: config2 / config3 / config5 / config5_tc")
    ap.add_argument("--profile", default="", help="where the passes' summaries are committed (profiles/...)")
    ap.add_argument("--kernel", default="classify", help="summarise the dispatches whose name contains this")
    a = ap.parse_args()
    if a.tag_dir.endswith(".json"):   # a summary this script wrote on the GPU box (--out)
        with open(a.tag_dir) as fh:
            s = json.load(fh)
    else:
        s = collect(a.tag_dir, a.kernel)
    if "FETCH_SIZE" in s:
        s["hbm_read_bytes_per_launch"] = s["FETCH_SIZE"] * 1024 * 2
        s["hbm_read_bytes_per_pkt"] = s["hbm_read_bytes_per_launch"] / a.frames
    if "WRITE_SIZE" in s:
        s["hbm_write_bytes_per_launch"] = s["WRITE_SIZE"] * 1024
    print(json.dumps(s, indent=1))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(s, fh, indent=1)
    if a.traffic and "FETCH_SIZE" in s:
        # bench.py reports this entry as roofline.traffic only while the kernel sources
        # hash the same (bench.kernel_src_hash) and the batch has the same size
        import sys
        sys.path.insert(0, ROOT)
        from bench import kernel_src_hash
        t = {"frames": a.frames, "hbm_bytes_per_launch": round(s["hbm_read_bytes_per_launch"]
                                                               + s.get("hbm_write_bytes_per_launch", 0)),
             "read_bytes": round(s["hbm_read_bytes_per_launch"]),
             "write_bytes": round(s.get("hbm_write_bytes_per_launch", 0)),
             "read_bytes_per_frame": round(s["hbm_read_bytes_per_launch"] / a.frames, 3),
             "src_hash": kernel_src_hash(), "profile": a.profile,
             "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over the classify kernel the product "
                       "runs, FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count correction), WRITE_SIZE KiB x 1024"}
        path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        doc = {}
        if os.path.exists(path):
            with open(path) as fh:
                doc = json.load(fh)
        doc.setdefault("configs", {})[a.key] = t
        with open(path, "w") as fh:
            json.dump({"configs": doc["configs"]}, fh, indent=1)

if __name__ == "__main__":
    main()
