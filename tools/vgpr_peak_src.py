"""Where the live registers at a kernel's register-pressure peak come from, by source line.

usage: python tools/vgpr_peak_src.py FILE.s KERNEL_SUBSTRING [rank]
FILE.s: device assembly compiled with -g (the .loc directives map instructions to source lines).  For the
rank-th highest-pressure instruction (tools/vgpr_live.py's count, AGPRs included), each live register is
attributed to the source line of its nearest def above it in program order (or, for a value carried around
a loop, the last def below it).  Measurement tool only."""
import collections
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
import vgpr_live as V  # noqa: E402


def main():
    path, name = sys.argv[1], sys.argv[2]
    rank = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    lines = open(path).read().splitlines()
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', l)
        if m:
            files[m.group(1)] = m.group(2)
    start = next(i for i, l in enumerate(lines) if re.match(r'^_Z\S*' + re.escape(name) + r'\S*:', l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
    body = lines[start + 1:end]
    loc, locs = "?", []
    blocks, cur, label_of, flat = [], None, {}, []
    for i, l in enumerate(body):
        m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', l)
        if m:
            loc = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
            continue
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
        d, u = V.defs_uses(mn, ops.strip())
        cur["ins"].append((len(flat), mn, ops.strip()))
        flat.append((mn, d, u, loc))
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
    live_in = [set() for _ in blocks]
    changed = True
    while changed:
        changed = False
        for bi in reversed(range(len(blocks))):
            out = set().union(*[live_in[s] for s in succ[bi]]) if succ[bi] else set()
            for k, _, _ in reversed(blocks[bi]["ins"]):
                out = (out - flat[k][1]) | flat[k][2]
            if out != live_in[bi]:
                live_in[bi] = out
                changed = True
    pts = []
    for bi, b in enumerate(blocks):
        out = set().union(*[live_in[s] for s in succ[bi]]) if succ[bi] else set()
        for k, _, _ in reversed(b["ins"]):
            pts.append((len(out | flat[k][1]), k, frozenset(out | flat[k][1])))
            out = (out - flat[k][1]) | flat[k][2]
    pts.sort(key=lambda p: -p[0])
    n, k0, live = pts[rank]
    print(f"peak #{rank}: {n} registers live at instruction {k0} ({flat[k0][0]}, {flat[k0][3]})")
    by = collections.Counter()
    for r in live:
        src = None
        for k in range(k0, -1, -1):
            if r in flat[k][1]:
                src = flat[k][3] + "  " + flat[k][0]
                break
        if src is None:
            for k in range(len(flat) - 1, k0, -1):
                if r in flat[k][1]:
                    src = "(loop-carried) " + flat[k][3] + "  " + flat[k][0]
                    break
        by[src or "?"] += 1
    for src, c in by.most_common():
        print(f"{c:4d}  {src}")


if __name__ == "__main__":
    main()
