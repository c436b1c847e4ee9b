"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into per-launch HBM
bytes for the bench's kernel classes -> profiles/pmc_traffic.json (read by bench.py).

Corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts 64 B per 128-B request of wide
coalesced streaming reads on gfx950 -> doubled; WRITE_SIZE is exact for 16-B/lane stores.
Both are reported in KiB by rocprofv3.  Infinity-Cache hits are counted, not excluded."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CLASSES = {"rows_gemm_kernel": "gemm", "wsg_kernel": "gemm", "sg_kernel": "gemm", "mlp_kernel": "gemm", "ffn_kernel": "ffn",
           "tailw_kernel": "ffn", "tail_kernel": "ffn", "attn32_bf16": "attention", "attn32_dma": "attention", "scan2_kernel": "knn_scan", "knn_emb_dot_kernel": "knn_emb"}


def load(d, counter):
    files = glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"]
            for key, cls in CLASSES.items():
                if key in name:
                    short = name.split("(")[0].replace("void ", "").replace("snvrag::", "")
                    vals[(cls, r.get("Grid_Size", ""), short)].append(float(r["Counter_Value"]))
                    break
    return vals, files


def main(d):
    out = {}
    fetch, ff = load(d, "FETCH_SIZE")
    write, wf = load(d, "WRITE_SIZE")
    for (cls, grid, short), v in fetch.items():
        w = write.get((cls, grid, short), [])
        e = out.setdefault(cls, [])
        e.append({"kernel": short, "grid": grid, "launches": len(v), "fetch_bytes": 2 * 1024 * sum(v) / len(v),
                  "write_bytes": 1024 * sum(w) / len(w) if w else None})
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) of bench.py --steps 2",
           "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), KiB -> bytes", "kernels": out,
           "files": [os.path.relpath(f) for f in ff + wf]}
    os.makedirs("profiles", exist_ok=True)
    json.dump(res, open("profiles/pmc_traffic.json", "w"), indent=1)
    print(json.dumps(res, indent=1)[:3000])


if __name__ == "__main__":
    main(sys.argv[1])
