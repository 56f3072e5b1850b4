"""Build a library variant whose fused-kernel TU (plane_launch.hip) gets extra compile flags, for A/B timing on one box
(tools/ab_variants.sh).  The other translation units are the in-tree objects (build them first).

usage: python tools/build_plane_variant.py NAME [--tu SOURCE.hip] [-DFLAG=V ...]   -> tools/ab/lib_NAME.so
(--tu: the translation unit that gets the flags, default plane_launch.hip)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as g  # noqa: E402


def main():
    name, extra = sys.argv[1], sys.argv[2:]
    tu = "plane_launch.hip"
    if "--tu" in extra:
        i = extra.index("--tu")
        tu = extra[i + 1]
        extra = extra[:i] + extra[i + 2:]
    out = os.path.join(REPO, "tools", "ab")
    os.makedirs(out, exist_ok=True)
    objs = []
    for src, obj, flags in g.LIB_TUS:
        if src == tu:
            o = os.path.join(out, f"tu_{name}.o")
            g._hip_tu(os.path.join(g.CSRC, src), o, [*flags, *extra], False)
            objs.append(o)
        else:
            objs.append(os.path.join(g.CSRC, obj))
    g._run(["hipcc", "--offload-arch=gfx950", "-fPIC", "-shared", "-o", os.path.join(out, f"lib_{name}.so"), *objs], False)
    print(os.path.join(out, f"lib_{name}.so"))


if __name__ == "__main__":
    main()
