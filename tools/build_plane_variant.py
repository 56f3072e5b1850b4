"""Build a library variant whose fused-kernel TU (plane_launch.hip) gets extra compile flags, for A/B timing on one box
(tools/ab_variants.sh).  The other translation units are the in-tree objects (build them first).

usage: python tools/build_plane_variant.py NAME [--tu SOURCE.hip] [--patch tools/variants/X.patch] [-DFLAG=V ...]
       -> tools/ab/lib_NAME.so
(--tu: the translation unit that gets the flags, default plane_launch.hip; --patch: a measured-and-retired experiment
kept out of the product sources (tools/variants/README.md): the sources are copied to tools/ab/src_NAME, the patch is
applied there and EVERY translation unit is rebuilt from the copy)
"""
import os
import shutil
import subprocess
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
    patch = None
    if "--patch" in extra:
        i = extra.index("--patch")
        patch = os.path.abspath(extra[i + 1])
        extra = extra[:i] + extra[i + 2:]
    out = os.path.join(REPO, "tools", "ab")
    os.makedirs(out, exist_ok=True)
    objs = []
    if patch:
        root = os.path.join(out, f"src_{name}")
        shutil.rmtree(root, ignore_errors=True)
        shutil.copytree(os.path.join(REPO, "include"), os.path.join(root, "include"))
        csrc = os.path.join(root, "admm-deconv_amd", "csrc")
        shutil.copytree(g.CSRC, csrc, ignore=shutil.ignore_patterns("*.o"))
        subprocess.run(["patch", "-p1", "-d", root, "-i", patch], check=True)
        for src, obj, flags in g.LIB_TUS:
            o = os.path.join(out, f"tu_{name}_{obj}")
            g._hip_tu(os.path.join(csrc, src), o, [*flags, *(extra if src == tu else [])], False)
            objs.append(o)
    for src, obj, flags in ([] if patch else g.LIB_TUS):
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
