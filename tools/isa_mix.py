"""Static instruction mix of one kernel in a gfx950 device-assembly file (hipcc --cuda-device-only -S).

usage: python tools/isa_mix.py FILE.s KERNEL_SUBSTRING [--blocks]
Counts VALU by class (FMA, add/sub, mul, cndmask, DPP moves, other), LDS, VMEM and scalar instructions over the
kernel body; --blocks prints the same per basic block (the fused kernels' iteration loop is one large block
range between its back-edge labels, so the per-iteration mix can be read off there).
"""
import collections
import re
import sys


def classify(line):
    op = line.split()[0]
    if op.startswith("v_"):
        if "dpp" in line or "row_" in line or "quad_perm" in line or "wave_sh" in line:
            return "v_dpp"
        if op.startswith("v_cndmask"):
            return "v_cndmask"
        if op.startswith(("v_fma", "v_fmac", "v_pk_fma")):
            return "v_fma"
        if op.startswith(("v_add", "v_sub", "v_pk_add")):
            return "v_add_sub"
        if op.startswith(("v_mul", "v_pk_mul")):
            return "v_mul"
        if op.startswith(("v_mov", "v_accvgpr")):
            return "v_mov"
        return "v_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith("s_barrier"):
        return "s_barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    s = open(path).read()
    m = re.search(r"\n(\S*" + re.escape(name) + r"\S*):", s)
    if not m:
        sys.exit(f"no kernel matching {name}")
    start = m.end()
    end = s.index(".Lfunc_end", start)
    body = s[start:end].split("\n")
    blocks = [("entry", collections.Counter())]
    for raw in body:
        line = raw.split(";")[0].strip()
        if line.endswith(":"):
            blocks.append((line[:-1], collections.Counter()))
            continue
        if not line or line.startswith((".", "//")):
            continue
        blocks[-1][1][classify(line)] += 1
    tot = collections.Counter()
    for _, c in blocks:
        tot.update(c)
    valu = sum(v for k, v in tot.items() if k.startswith("v_"))
    print(f"{m.group(1)[:100]}\n  VALU {valu}: " + ", ".join(f"{k} {v}" for k, v in sorted(tot.items()) if k.startswith("v_")))
    print("  " + ", ".join(f"{k} {v}" for k, v in sorted(tot.items()) if not k.startswith("v_")))
    if "--blocks" in sys.argv:
        for lab, c in blocks:
            n = sum(c.values())
            if n > 200:
                v = sum(x for k, x in c.items() if k.startswith("v_"))
                print(f"  {lab:12s} {n:6d} instr, VALU {v:6d}: " + ", ".join(f"{k} {x}" for k, x in sorted(c.items())))


if __name__ == "__main__":
    main()
