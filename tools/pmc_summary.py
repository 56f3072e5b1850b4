"""Summarise rocprofv3 --pmc CSV output per kernel (mean value per dispatch).

usage: python tools/pmc_summary.py gpurun_out/pmc1 [gpurun_out/pmc2 ...] [--json out.json]

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of a wide
coalesced streaming read, so hbm_read_bytes = 2 * FETCH_SIZE(KiB) * 1024 for our 16-B/lane streams;
WRITE_SIZE is exact for 16-B/lane stores.  Both count Infinity-Cache hits as well.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    m = re.search(r"admm::(\w+?)(<[^>]*>)?\(", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name[:40]


def load(dirs):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            per = collections.defaultdict(float)
            names = {}
            for row in csv.DictReader(open(f)):
                key = (row["Dispatch_Id"], row["Counter_Name"])
                per[key] += float(row["Counter_Value"])
                names[row["Dispatch_Id"]] = short(row["Kernel_Name"])
            for (disp, cname), v in per.items():
                acc[names[disp]][cname].append(v)
    return acc


def main():
    args = sys.argv[1:]
    out = None
    if "--json" in args:
        i = args.index("--json")
        out = args[i + 1]
        args = args[:i] + args[i + 2:]
    acc = load(args)
    res = {}
    for k, cs in sorted(acc.items()):
        res[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        line = ", ".join(f"{c}={res[k][c]:.4g}" for c in sorted(res[k]))
        print(f"{k}: {line}")
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
