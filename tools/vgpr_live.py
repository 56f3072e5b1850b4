"""Approximate VGPR liveness of one kernel in a gfx9 device-assembly file (hipcc --cuda-device-only -S).

usage: python tools/vgpr_live.py FILE.s KERNEL_SUBSTRING [top]
Prints the instructions with the most live VGPRs (backward dataflow over the basic blocks; an exec-masked
def is taken as a kill, so divergent code is undercounted) with the nearest preceding label, to find where
a kernel's register peak sits.  Measurement tool only."""
import re
import sys

REG = re.compile(r'\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b')


def regs(s):
    # AGPRs (a0..a255) count as registers 256.. (values the allocator parked there are live too)
    out = set()
    for m in REG.finditer(s):
        if m.group(5) is not None:
            out.add(int(m.group(5)) + (256 if m.group(4) == 'a' else 0))
        else:
            b = 256 if m.group(1) == 'a' else 0
            out.update(range(b + int(m.group(2)), b + int(m.group(3)) + 1))
    return out


NODEF = ("store", "ds_write", "v_cmp", "s_", "v_readfirstlane", "v_readlane", "buffer_atomic", "ds_add")
# v_accvgpr_write a, v: def a; v_accvgpr_read v, a: def v (generic first-operand rule)


def defs_uses(mn, ops):
    parts = [p.strip() for p in re.split(r',(?![^\[]*\])', ops)] if ops else []
    if not parts:
        return set(), set()
    if any(mn.startswith(p) or p in mn for p in NODEF) and not mn.startswith("v_cmpx"):
        if mn.startswith(("v_readfirstlane", "v_readlane")) or mn.startswith("v_cmp"):
            return set(), regs(",".join(parts[1:]))
        return set(), regs(",".join(parts))
    d = regs(parts[0])
    u = regs(",".join(parts[1:]))
    if mn.startswith(("v_fmac", "v_mac", "v_writelane", "v_dot2c")) or "_dpp" in mn:
        u |= d
    return d, u


def main():
    path, name = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r'^_Z\S*' + re.escape(name) + r'\S*:', l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
    body = lines[start + 1:end]
    # blocks
    blocks, cur, label_of = [], None, {}
    for i, l in enumerate(body):
        m = re.match(r'^(\.LBB\S+):', l)
        if m or cur is None:
            cur = {"label": m.group(1) if m else "entry", "ins": []}
            blocks.append(cur)
            label_of[cur["label"]] = len(blocks) - 1
            if m:
                continue
        t = l.split(';')[0].strip()
        if not t or t.startswith('.'):
            continue
        mn, _, ops = t.partition(' ')
        cur["ins"].append((i, mn, ops.strip()))
    succ = []
    for bi, b in enumerate(blocks):
        s = []
        last = b["ins"][-1] if b["ins"] else None
        if last and last[1].startswith("s_branch"):
            s.append(label_of[last[2]])
        else:
            if last and last[1].startswith("s_cbranch"):
                s.append(label_of[last[2]])
            if bi + 1 < len(blocks) and not (last and last[1] == "s_endpgm"):
                s.append(bi + 1)
        succ.append(s)
    du = [[defs_uses(mn, ops) for (_, mn, ops) in b["ins"]] for b in blocks]
    live_in = [set() for _ in blocks]
    changed = True
    while changed:
        changed = False
        for bi in reversed(range(len(blocks))):
            out = set().union(*[live_in[s] for s in succ[bi]]) if succ[bi] else set()
            for d, u in reversed(du[bi]):
                out = (out - d) | u
            if out != live_in[bi]:
                live_in[bi] = out
                changed = True
    res = []
    for bi, b in enumerate(blocks):
        out = set().union(*[live_in[s] for s in succ[bi]]) if succ[bi] else set()
        for (i, mn, ops), (d, u) in reversed(list(zip(b["ins"], du[bi]))):
            res.append((len(out | d), i, b["label"], mn))
            out = (out - d) | u
    res.sort(reverse=True)
    print(f"{len(blocks)} blocks; peak {res[0][0]}")
    seen = set()
    for n, i, lab, mn in res:
        if (lab, n) in seen:
            continue
        seen.add((lab, n))
        print(f"{n:4d} line {i + start + 2:6d} {lab:12s} {mn}")
        if len(seen) >= top:
            break


if __name__ == "__main__":
    main()


def explain(path, name, line_no):
    """The registers live at (1-based) line line_no and, for each, the text of the closest def above it."""
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r'^_Z\S*' + re.escape(name) + r'\S*:', l))
    return lines, start
