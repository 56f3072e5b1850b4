"""Hazard bisection for the fused kernel: rebuild plane_launch.hip from its device
assembly with `s_nop` inserted at chosen instruction classes, and link libadmm_deconv_<TAG>.so.

The failing build (packed FP32, the compiler's default) is fixed by `-mllvm -amdgpu-snop-padding=1`
(an s_nop before EVERY instruction) but not by waiting for every load (`-amdgpu-waitcnt-load-forcezero`):
a pipeline hazard the compiler does not pad, not a memory-ordering one.  This tool pads selectively to
find the instruction pair.

usage (in this container, after __graft_entry__.build()):
  [ASMX_WORK=dir] python tools/asm_variant.py prepare [--nopk] [-DMACRO=..]   # hipcc -save-temps steps 1-3
  python tools/asm_variant.py build TAG RULE [NOPS]    # pad per RULE, assemble, link the variant .so
RULE: all | pk_after | pk_before | dpp_before | raw1 | raw1_pk | raw1_dpp | vmem_before | war_vmem | ...
"""
import os
import re
import shlex
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "admm-deconv_amd", "csrc")
WORK = os.environ.get("ASMX_WORK", "/tmp/asmx")   # one work dir per base build
DEV_S = "plane_launch-hip-amdgcn-amd-amdhsa-gfx950.s"

INSN = re.compile(r"^\t([sv]_\w+|buffer_\w+|global_\w+|ds_\w+|flat_\w+|scratch_\w+)(\s+(.*))?$")
VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def vregs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def split_ops(ops):
    # operands separated by ", " before any modifiers (dpp/offset words follow after a space)
    parts = [p.strip() for p in ops.split(",")]
    return parts


def parse(line):
    m = INSN.match(line)
    if not m:
        return None
    mn = m.group(1)
    ops = (m.group(3) or "").split(";")[0]
    parts = split_ops(ops)
    dst, src = set(), set()
    is_store = mn.startswith(("buffer_store", "global_store", "ds_write", "scratch_store", "flat_store"))
    if mn.startswith("v_") or mn.startswith(("buffer_load", "global_load", "ds_read", "scratch_load", "flat_load",
                                             "ds_bpermute", "ds_permute", "ds_swizzle")):
        if parts and parts[0]:
            dst = vregs(parts[0])
            src = vregs(",".join(parts[1:]))
    else:
        src = vregs(ops)
    if is_store:
        src, dst = vregs(ops), set()
    return mn, dst, src


def is_valu(mn):
    return mn.startswith("v_")


def is_vmem_load(mn):
    return mn.startswith(("buffer_load", "global_load", "scratch_load", "flat_load"))


def rule_fn(rule):
    """(prev instructions [(mn,dst,src)], this (mn,dst,src)) -> bool: insert the nop before `this`."""
    def raw(prev, cur, pred_prev=lambda mn: True, pred_cur=lambda mn: True, dist=1):
        if not is_valu(cur[0]) or not pred_cur(cur[0]):
            return False
        for p in prev[-dist:]:
            if p and is_valu(p[0]) and pred_prev(p[0]) and (p[1] & cur[2]):
                return True
        return False
    pk = lambda mn: mn.startswith("v_pk_")  # noqa: E731

    def vmv(prev, cur):
        if len(prev) < 2 or prev[-2] is None or prev[-1] is None or not is_valu(cur[0]):
            return False
        pp, mm = prev[-2], prev[-1]
        return is_valu(pp[0]) and MIDS["mem"](mm[0]) and bool(pp[1] & cur[2])

    def d2(prev, cur, pp=lambda mn: True, pc=lambda mn: True, pm=lambda mn: True):
        if not is_valu(cur[0]) or not pc(cur[0]) or len(prev) < 2 or prev[-2] is None:
            return False
        p = prev[-2]
        mid = prev[-1][0] if prev[-1] is not None else None
        return is_valu(p[0]) and pp(p[0]) and pm(mid) and bool(p[1] & cur[2])

    def war(prev, cur, dist, pred_prev=lambda mn: True):
        if not cur[1]:
            return False
        for p in prev[-dist:]:
            if p and is_valu(p[0]) and pred_prev(p[0]) and (p[2] & cur[1]):
                return True
        return False
    dpp = lambda mn: "_dpp" in mn  # noqa: E731
    rules = {
        "none": lambda prev, cur: False,
        "all": lambda prev, cur: True,
        "valu": lambda prev, cur: is_valu(cur[0]),
        "pk_before": lambda prev, cur: pk(cur[0]),
        "pk_after": lambda prev, cur: bool(prev) and prev[-1] is not None and pk(prev[-1][0]),
        "dpp_before": lambda prev, cur: dpp(cur[0]),
        "dpp_after": lambda prev, cur: bool(prev) and prev[-1] is not None and dpp(prev[-1][0]),
        "raw1": lambda prev, cur: raw(prev, cur),
        "raw2": lambda prev, cur: raw(prev, cur, dist=2),
        # producer exactly 2 instructions back (one instruction in between)
        "d2": lambda prev, cur: d2(prev, cur),
        "d2_pkprod": lambda prev, cur: d2(prev, cur, pp=pk),
        "d2_pkcons": lambda prev, cur: d2(prev, cur, pc=pk),
        "d2_pkboth": lambda prev, cur: d2(prev, cur, pp=pk, pc=pk),
        "d2_nopk": lambda prev, cur: d2(prev, cur, pp=lambda m: not pk(m), pc=lambda m: not pk(m)),
        "d2_midvalu": lambda prev, cur: d2(prev, cur, pm=lambda m: m is not None and is_valu(m)),
        "d2_midnonvalu": lambda prev, cur: d2(prev, cur, pm=lambda m: m is None or not is_valu(m)),
        "d2_dppcons": lambda prev, cur: d2(prev, cur, pc=dpp),
        "raw1_pkprod": lambda prev, cur: raw(prev, cur, pred_prev=pk),
        "raw1_pkcons": lambda prev, cur: raw(prev, cur, pred_cur=pk),
        "raw1_dppcons": lambda prev, cur: raw(prev, cur, pred_cur=dpp),
        "raw1_dppprod": lambda prev, cur: raw(prev, cur, pred_prev=dpp),
        "vmem_before": lambda prev, cur: is_vmem_load(cur[0]),
        # a VMEM load overwriting a VGPR read by one of the 4 previous VALU instructions
        "war_vmem": lambda prev, cur: is_vmem_load(cur[0]) and any(
            p and is_valu(p[0]) and (p[2] & cur[1]) for p in prev[-4:]),
        # write-after-read: this instruction writes a VGPR that one of the previous `dist` VALU ops read
        "war1": lambda prev, cur: war(prev, cur, 1),
        "war1_pk": lambda prev, cur: war(prev, cur, 1, pk),
        "war2_pk": lambda prev, cur: war(prev, cur, 2, pk),
        "war3_pk": lambda prev, cur: war(prev, cur, 3, pk),
        "war1_pk_valu": lambda prev, cur: is_valu(cur[0]) and war(prev, cur, 1, pk),
        "war1_pk_nonvalu": lambda prev, cur: not is_valu(cur[0]) and war(prev, cur, 1, pk),
        "lane_before": lambda prev, cur: cur[0].startswith(("v_readlane", "v_writelane")),
        "ds_before": lambda prev, cur: cur[0].startswith("ds_"),
        # VALU -> memory instruction -> VALU consumer of the first VALU's result, split by whether the memory
        # instruction overwrites (load destination) a source VGPR of the first VALU
        "vmv_warload": lambda prev, cur: vmv(prev, cur) and bool(prev[-1][1] & prev[-2][2]),
        "vmv_other": lambda prev, cur: vmv(prev, cur) and not (prev[-1][1] & prev[-2][2]),
        "salu_before": lambda prev, cur: cur[0].startswith("s_") and not cur[0].startswith(("s_nop", "s_waitcnt")),
    }
    return rules[rule]


PRODS = {"any": lambda mn: True, "pk": lambda mn: mn.startswith("v_pk_"),
         "nonpk": lambda mn: not mn.startswith("v_pk_"), "cnd": lambda mn: mn.startswith("v_cndmask"),
         "nondpp": lambda mn: "_dpp" not in mn}
CONS = {"any": lambda mn: True, "dpp": lambda mn: "_dpp" in mn, "nondpp": lambda mn: "_dpp" not in mn,
        "pk": lambda mn: mn.startswith("v_pk_"), "nonpk": lambda mn: not mn.startswith("v_pk_")}


def pad_ws(src, prod, cons, need, kernels=None):
    """Ensure at least `need` wait states between a VALU (class prod) writing a VGPR and a later VALU (class
    cons) reading it, counting each intervening instruction as 1 and `s_nop N` as N + 1."""
    P, C = PRODS[prod], CONS[cons]
    out, hist, n_ins, cur_fn = [], [], 0, None   # hist: list of (dst set or None, mnemonic, wait states)
    for line in src.split("\n"):
        if re.match(r"^_Z\S*:", line):
            cur_fn, hist = line.split(":")[0], []
        p = parse(line)
        if p is not None:
            if is_valu(p[0]) and C(p[0]) and (kernels is None or any(k in (cur_fn or "") for k in kernels)):
                ws = 0
                short = 0
                for dst, mn, w in reversed(hist):
                    if ws >= need:
                        break
                    if dst and is_valu(mn) and P(mn) and (dst & p[2]):
                        short = max(short, need - ws)
                    ws += w
                if short > 0:
                    out.append(f"\ts_nop {short - 1}")
                    hist.append((None, "s_nop", short))
                    n_ins += 1
            w = int(line.split()[1]) + 1 if p[0] == "s_nop" else 1
            hist.append((p[1], p[0], w))
            hist = hist[-16:]
        elif re.match(r"^\.LBB", line):
            hist = []   # unknown predecessor: conservatively nothing known (rare inside the unrolled loop)
        out.append(line)
    return "\n".join(out), n_ins


MIDS = {"any": lambda mn: True, "salu": lambda mn: mn.startswith("s_") and not mn.startswith(("s_nop", "s_waitcnt")),
        "wait": lambda mn: mn.startswith("s_waitcnt"), "nop": lambda mn: mn.startswith("s_nop"),
        "mem": lambda mn: mn.startswith(("ds_", "buffer_", "global_", "scratch_", "flat_")),
        "nonvalu": lambda mn: not is_valu(mn)}


# a >64-bit MUBUF store whose soffset operand is a register (any SGPR name: s12, vcc_lo, m0, ...), not an
# inline constant
SSTORE = re.compile(r"^\s+buffer_store_dword(x3|x4)\s+(v\[\d+:\d+\]),\s*[^,]+,\s*s\[\d+:\d+\],\s*([a-z][a-z_0-9]*)\b")


def pad_sstore(src, need, kernels=None):
    """A VALU writing a data VGPR of a preceding >64-bit MUBUF store whose soffset is an SGPR, fewer than
    `need` wait states after it.  (LLVM exempts MUBUF stores with a register soffset from its >8-byte
    store-data hazard.)"""
    out, hist, n_ins = [], [], 0
    for line in src.split("\n"):
        if re.match(r"^[\w.$]+:", line.strip()):
            hist = []
        p = parse(line)
        if p is not None:
            mn, dst, srcs = p
            if is_valu(mn) and dst:
                ws, short = 0, 0
                for data, w in reversed(hist):
                    if ws >= need:
                        break
                    if data & dst:
                        short = max(short, need - ws)
                    ws += w
                if short:
                    out.append(f"\ts_nop {short - 1}")
                    hist.append((set(), short))
                    n_ins += 1
            m = SSTORE.match(line)
            w = int(line.split()[1]) + 1 if mn == "s_nop" else 1
            hist.append((vregs(m.group(2)) if m else set(), w))
            hist = hist[-16:]
        out.append(line)
    return "\n".join(out), n_ins


def pad_mem(src, kind, need, kernels=None):
    """warst: a VALU writing a VGPR that a memory instruction (store data / address) read fewer than `need`
    wait states earlier; rawmem: a memory instruction reading a VGPR a VALU wrote fewer than `need` wait
    states earlier.  Pads with s_nop before the later instruction."""
    out, hist, n_ins = [], [], 0
    for line in src.split("\n"):
        if re.match(r"^[\w.$]+:", line.strip()):
            hist = []
        p = parse(line)
        if p is not None:
            mn, dst, srcs = p
            allregs = vregs((line.split(";")[0].split(None, 1) + [""])[1])
            short = 0
            ws = 0
            for hmn, hdst, hsrc, w in reversed(hist):
                if ws >= need:
                    break
                if kind == "warst" and is_valu(mn) and not is_valu(hmn) and hmn.startswith(
                        ("ds_", "buffer_", "global_", "scratch_")) and (hsrc & dst):
                    short = max(short, need - ws)
                if kind == "rawmem" and mn.startswith(("ds_", "buffer_", "global_", "scratch_")) and is_valu(hmn) \
                        and (hdst & allregs):
                    short = max(short, need - ws)
                ws += w
            if short:
                out.append(f"\ts_nop {short - 1}")
                hist.append(("s_nop", set(), set(), short))
                n_ins += 1
            w = int(line.split()[1]) + 1 if mn == "s_nop" else 1
            msrc = allregs if mn.startswith(("ds_", "buffer_", "global_", "scratch_")) and not mn.startswith(
                ("buffer_load", "global_load", "scratch_load", "ds_read")) else srcs
            if mn.startswith(("buffer_load", "global_load", "scratch_load", "ds_read")):
                msrc = vregs(",".join((line.split(";")[0].split(None, 1) + [""])[1].split(",")[1:]))
            hist.append((mn, dst, msrc, w))
            hist = hist[-16:]
        out.append(line)
    return "\n".join(out), n_ins


def pad(src, rule, nops, kernels=None):
    if rule.startswith("t:"):               # t:<prod>:<mid>:<cons>: producer, ONE non-VALU of class mid, consumer
        _, prod, mid, cons = rule.split(":")
        P, Mi, C = PRODS[prod], MIDS[mid], CONS[cons]

        def fn(prev, cur):
            if len(prev) < 2 or prev[-2] is None or prev[-1] is None or not is_valu(cur[0]) or not C(cur[0]):
                return False
            pp, mm = prev[-2], prev[-1]
            return is_valu(pp[0]) and P(pp[0]) and not is_valu(mm[0]) and Mi(mm[0]) and bool(pp[1] & cur[2])
        return _pad_fn(src, fn, nops, kernels)
    if rule.startswith("sstore:"):
        return pad_sstore(src, int(rule.split(":")[1]), kernels)
    if rule.startswith("warst:") or rule.startswith("rawmem:"):
        return pad_mem(src, rule.split(":")[0], int(rule.split(":")[1]), kernels)
    if rule.startswith("ws:"):              # ws:<prod>:<cons>:<wait states>
        _, prod, cons, need = rule.split(":")
        return pad_ws(src, prod, cons, int(need), kernels)
    return _pad_fn(src, rule_fn(rule), nops, kernels)


def _pad_fn(src, fn, nops, kernels):
    out, prev, n_ins, cur_fn = [], [], 0, None
    for line in src.split("\n"):
        if re.match(r"^_Z\S*:", line):
            cur_fn = line.split(":")[0]
            prev = []
        elif line.startswith(".L") or line.startswith("\ts_cbranch") or line.startswith("\ts_branch"):
            pass
        p = parse(line)
        if p is not None and (kernels is None or (cur_fn and any(k in cur_fn for k in kernels))):
            if fn(prev, p):
                out.append(f"\ts_nop {nops}")
                n_ins += 1
        if p is not None:
            prev.append(p)
            prev = prev[-8:]
        elif re.match(r"^\.LBB", line):
            prev.append(None)     # a branch target: the predecessor is unknown
        out.append(line)
    return "\n".join(out), n_ins


def run(cmd_line, cwd):
    r = subprocess.run(cmd_line, shell=True, cwd=cwd, capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(f"step failed: {cmd_line[:200]}\n{r.stderr[-2000:]}")


def prepare(nopk, extra=""):
    os.makedirs(WORK, exist_ok=True)
    flags = ("-Xclang -target-feature -Xclang -packed-fp32-ops " if nopk else "") + extra
    cmd = (f"hipcc -### --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c {flags} -mllvm -pragma-unroll-threshold=100000 "
           f"-save-temps -o plane_launch.o {CSRC}/plane_launch.hip")
    r = subprocess.run(cmd, shell=True, cwd=WORK, capture_output=True, text=True)
    lines = [l for l in r.stderr.split("\n") if l.startswith(' "')]
    open(os.path.join(WORK, "cmds.txt"), "w").write("\n".join(lines) + "\n")
    for l in lines[:3]:
        run(l, WORK)
    print("prepared", os.path.join(WORK, DEV_S))


def build(tag, rule, nops, kernels=None):
    lines = open(os.path.join(WORK, "cmds.txt")).read().strip().split("\n")
    d = os.path.join(WORK, tag)
    os.makedirs(d, exist_ok=True)
    src = open(os.path.join(WORK, DEV_S)).read()
    if os.environ.get("ASMX_PREPAD") == "1":     # the product's hazard pass first (csrc/hazard_pad.py)
        sys.path.insert(0, CSRC)
        import hazard_pad
        src, n0 = hazard_pad.pad_asm(src)
        print(f"prepad: {n0} s_nop")
    mod, n = pad(src, rule, nops, kernels)
    open(os.path.join(d, DEV_S), "w").write(mod)
    for f in os.listdir(WORK):
        if f.endswith((".hipi", ".bc")) and not os.path.exists(os.path.join(d, f)):
            os.symlink(os.path.join(WORK, f), os.path.join(d, f))
    for l in lines[3:]:
        run(l, d)
    so = os.path.join(REPO, "admm-deconv_amd", f"libadmm_deconv_{tag}.so")
    run(f"hipcc --offload-arch=gfx950 -fPIC -shared -o {so} {CSRC}/admm_capi.o {d}/plane_launch.o "
        f"{CSRC}/metrics_capi.o", d)
    print(f"built {tag}: rule {rule}, {n} s_nop {nops} inserted -> {so}")


if __name__ == "__main__":
    if sys.argv[1] == "prepare":
        prepare("--nopk" in sys.argv, " ".join(a for a in sys.argv[2:] if a.startswith("-D")))
    else:
        kern = sys.argv[5].split(",") if len(sys.argv) > 5 else None
        build(sys.argv[2], sys.argv[3], int(sys.argv[4]) if len(sys.argv) > 4 else 1, kern)
