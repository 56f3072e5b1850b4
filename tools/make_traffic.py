"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes per kernel class.

usage: python tools/make_traffic.py CONFIG PLANES OUT.json gpurun_out/prof_TAG/pmc_fetch gpurun_out/prof_TAG/pmc_write [pmc_sq]

PLANES = the plane count of the profiled launches (bench.py reports the figures only for launches of that size).

hbm_bytes_per_launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024   (FETCH_SIZE reads half the bytes of
a wide coalesced stream on gfx950 -- MI355X_MICROARCH.md, HBM section; WRITE_SIZE is exact for 16-B
stores).  Infinity-Cache hits are counted too (same section).  Values merge into OUT.json[CONFIG].
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402

CLASS = {"line_kernel": "line", "column_kernel<256, false>": "column", "iso_a_kernel": "iso_a",
         "iso_b_kernel": "iso_b", "plane_kernel": "plane"}


def klass(name):
    if "plane256_isoadj_kernel" in name:
        return "adjoint"
    if "plane256_iso_kernel" in name:
        return "plane"
    if "iso_norm_kernel" in name:
        return "norm"
    if "iso_radj_kernel" in name:
        return "radj"
    if "plane256_kernel" in name:
        return "plane"
    if "plane256_adj_kernel" in name:
        return "adjoint"
    for k, v in CLASS.items():
        if name.startswith(k):
            return v
    if name.startswith("column_kernel") and "false" in name:
        return "column"
    return None


def main():
    cfg, planes, out, fdir, wdir = sys.argv[1:6]
    sq = load([sys.argv[6]]) if len(sys.argv) > 6 else {}
    f = load([fdir])
    w = load([wdir])
    res = json.load(open(out)) if os.path.exists(out) else {}
    ent = res.setdefault(cfg, {})
    for name in f:
        c = klass(name)
        if c is None or name not in w:
            continue
        fs = sum(f[name]["FETCH_SIZE"]) / len(f[name]["FETCH_SIZE"])
        ws = sum(w[name]["WRITE_SIZE"]) / len(w[name]["WRITE_SIZE"])
        ent[c] = {"kernel": name, "fetch_size_kib": fs, "write_size_kib": ws,
                  "hbm_bytes_per_launch": int(2 * fs * 1024 + ws * 1024),
                  "note": "2*FETCH_SIZE + WRITE_SIZE (gfx950 correction); includes Infinity-Cache hits",
                  "planes": int(planes)}
        if name in sq and "SQ_INSTS_VALU" in sq[name]:
            avg = lambda k: sum(sq[name][k]) / len(sq[name][k])
            # wave-level instruction counts per launch (SQ counters sum over the whole chip)
            ent[c]["valu_insts_per_launch"] = avg("SQ_INSTS_VALU")
            ent[c]["lds_insts_per_launch"] = avg("SQ_INSTS_LDS")
            ent[c]["salu_insts_per_launch"] = avg("SQ_INSTS_SALU")
            ent[c]["waves_per_launch"] = avg("SQ_WAVES")
            ent[c]["wait_any_frac"] = avg("SQ_WAIT_ANY") / max(avg("SQ_WAVE_CYCLES"), 1.0)
        print(cfg, c, ent[c]["hbm_bytes_per_launch"], ent[c].get("valu_insts_per_launch"))
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
