"""Build step: pad a gfx950 store-data hazard that ROCm 7.2's hazard recognizer skips, in every HIP
translation unit of the library (used by __graft_entry__.build()).

The hazard (root-caused by bisection on the fused per-plane kernel; tools/asm_variant.py):

    buffer_store_dwordx4 v[46:49], v189, s[24:27], s34 offen    ; 128-bit store, soffset = an SGPR
    v_med3_f32           v48, v46, -s28, s28                    ; next instruction overwrites v48

A VALU write of a data VGPR of a store with more than 64 bits of data, issued right after the store,
corrupts the stored value (nondeterministically, in some lanes).  LLVM knows this hazard (">8-byte
store data", 1-2 wait states) but exempts MUBUF stores whose soffset is a register; on gfx950 the
exemption is wrong.  The fused kernel's lane-native stores (`buffer_store_dwordx4 ... sN offen`, the
per-register offset in soffset) hit it whenever the scheduler placed the prox arithmetic of the next
chunk right behind the store.  Measured (2 x 3 x 2,048 plane-solve census per build): packed FP32,
prefetch depth 2, the v_med3/FMA prox, and packed FP32 + that prox -- the four builds that failed in
round 1 -- all pass with only these sites padded (2 to 252 s_nop 0), and fail without.

The pass: compile the translation unit with hipcc's own pipeline (hipcc -### -save-temps) and, in the
device assembly, put at least 2 wait states between any VMEM store with more than 64 bits of data
(buffer/global/scratch/flat, dwordx3/x4 or b96/b128, any soffset) and a later VALU instruction that
writes one of its data VGPRs (an `s_nop` before that VALU).  The window is tracked along the
straight-line fallthrough; a branch inside the window is padded to the full wait count first, so no
jump target can start inside it.  Then assemble, link and bundle exactly as hipcc would.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess

INSN = re.compile(r"^\s+([a-z][a-z0-9_]*)(\s+(.*))?$")
VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
WIDE_STORE = re.compile(r"^(buffer|global|scratch|flat)_store_(dwordx3|dwordx4|b96|b128)$")
# control transfers: the window cannot follow the jump into its target block, so it is closed (padded)
# before the branch instead -- every path into a block then arrives with the wait states already spent
BRANCH = re.compile(r"^s_(branch|cbranch_\w+|setpc_b64|swappc_b64|callpc_b64|call_b64)$")
NEED = int(os.environ.get("ADMM_HAZARD_NEED", "2"))   # wait states after the store (experiments: env)


def _vregs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def _store_data(mn, ops):
    """Data VGPRs of a wide VMEM store (buffer: operand 0; global / flat / scratch: operand 1)."""
    parts = ops.split(",")
    if mn.startswith("buffer_"):
        return _vregs(parts[0])
    return _vregs(parts[1]) if len(parts) > 1 else set()


def _valu_dst(mn, ops):
    """VGPRs a VALU instruction writes: operand 0, and operand 1 as well for the swap forms
    (v_swap_b32, gfx950's v_permlane16_swap_b32 / v_permlane32_swap_b32 exchange both operands)."""
    parts = ops.split(",")
    dst = _vregs(parts[0])
    if "swap" in mn and len(parts) > 1:
        dst |= _vregs(parts[1])
    return dst


def _short(recent, dst=None):
    """Wait states still missing after a wide store whose data VGPRs meet `dst` (None: any wide store)."""
    ws, short = 0, 0
    for data, w in reversed(recent):
        if ws >= NEED:
            break
        if data and (dst is None or data & dst):
            short = max(short, NEED - ws)
        ws += w
    return short


def pad_asm(text):
    """Returns (padded assembly, number of s_nop inserted)."""
    out = []
    recent = []         # (data VGPRs of a wide store or empty, wait states of the instruction)
    inserted = 0
    for line in text.split("\n"):
        st = line.split(";")[0].strip()
        if re.match(r"^[\w.$]+:", st):        # a label: the predecessor may be a branch -- keep the window
            out.append(line)
            continue
        m = INSN.match(line.split(";")[0])
        if not m or st.startswith("."):
            out.append(line)
            continue
        mn, ops = m.group(1), m.group(3) or ""
        short = 0
        if mn.startswith("v_"):
            short = _short(recent, _valu_dst(mn, ops))
        elif BRANCH.match(mn):
            short = _short(recent)
        if short:
            out.append(f"\ts_nop {short - 1}")
            recent.append((set(), short))
            inserted += 1
        w = 1
        if mn == "s_nop":
            try:
                w = int(ops.split()[0]) + 1
            except (IndexError, ValueError):
                w = 1
        recent.append((_store_data(mn, ops) if WIDE_STORE.match(mn) else set(), w))
        if len(recent) > 8:
            recent = recent[-8:]
        out.append(line)
    return "\n".join(out), inserted


KERNEL = re.compile(r"^\s*\.amdhsa_kernel\s+(\S+)")
SCRATCH = re.compile(r"^\s*\.amdhsa_private_segment_fixed_size\s+(\d+)")


def scratch_sizes(text):
    """{kernel symbol: private (scratch) segment bytes per lane} from the kernel descriptors of device assembly."""
    out, cur = {}, None
    for line in text.split("\n"):
        m = KERNEL.match(line)
        if m:
            cur = m.group(1)
            continue
        m = SCRATCH.match(line)
        if m and cur is not None:
            out[cur] = int(m.group(1))
    return out


def compile_tu(src, obj, flags, verbose=False, scratch_out=None):
    """hipcc -c `src` -> `obj` with `flags`, the device assembly padded by pad_asm.  Returns the s_nop count;
    `scratch_out` (a dict), when given, receives every kernel's scratch bytes per lane (scratch_sizes)."""
    work = obj + ".hz"
    shutil.rmtree(work, ignore_errors=True)
    os.makedirs(work)
    cmd = ["hipcc", "-###", *flags, "-save-temps", "-c", "-o", os.path.abspath(obj), os.path.abspath(src)]
    r = subprocess.run(cmd, cwd=work, capture_output=True, text=True)
    steps = [l for l in r.stderr.split("\n") if l.startswith(' "')]
    if r.returncode != 0 or not steps:
        raise RuntimeError(f"hipcc -### failed for {src}:\n{r.stderr[-2000:]}")
    try:
        return _run_steps(steps, work, src, verbose, scratch_out)
    finally:
        shutil.rmtree(work, ignore_errors=True)   # also after a failed step (no .hipi left in the tree)


def _run_steps(steps, work, src, verbose, scratch_out):
    total = 0
    for i, step in enumerate(steps):
        is_dev_as = "-cc1as" in step and "amdgcn-amd-amdhsa" in step
        if is_dev_as:
            m = re.search(r'"([^"]*amdgcn[^"]*\.s)"\s*$', step.strip())
            if not m:
                raise RuntimeError(f"cannot find the device assembly in: {step[:200]}")
            path = os.path.join(work, m.group(1))
            text, n = pad_asm(open(path).read())
            if scratch_out is not None:
                scratch_out.update(scratch_sizes(text))
            open(path, "w").write(text)
            total += n
        rr = subprocess.run(step, shell=True, cwd=work, capture_output=True, text=True)
        noise = "is not a recognized feature for this target"
        err = "\n".join(l for l in rr.stderr.split("\n") if noise not in l and l.strip())
        if rr.returncode != 0:
            raise RuntimeError(f"build step {i} failed for {src}:\n{err[-3000:]}")
        if verbose and err:
            print(err)
    return total
