"""Parse the `ccall`s of julia/ADMMDeconvHIP.jl (the Julia binding a maintainer would add; Julia itself is
absent here) and the C prototypes of include/admm_deconv.h, so tests can check that every type tuple
matches its prototype (CPU) and replay every call's argument list through ctypes (GPU)."""
from __future__ import annotations

import ctypes
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JL = os.path.join(REPO, "julia", "ADMMDeconvHIP.jl")
HDR = os.path.join(REPO, "include", "admm_deconv.h")

# Julia ccall argument type -> (kind, ctypes type)
JTYPES = {
    "Ptr{Float32}": ("ptr", ctypes.c_void_p), "Ptr{Cvoid}": ("ptr", ctypes.c_void_p),
    "Ref{Csize_t}": ("ptr", ctypes.POINTER(ctypes.c_size_t)), "Cint": ("int", ctypes.c_int),
    "Cfloat": ("float", ctypes.c_float), "Csize_t": ("size", ctypes.c_size_t), "Cstring": ("ptr", ctypes.c_char_p),
}


def _split_top(s):
    """Split on commas not nested in (), {} or []."""
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "({[":
            depth += 1
        elif ch in ")}]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def julia_ccalls():
    """{symbol: [julia type, ...]} for every ccall((:symbol, LIB), Cint, types, ...) in the shim."""
    src = open(JL).read()
    consts = {}
    for m in re.finditer(r"const (_\w+Sig) = \((.*?)\)\n", src, re.S):
        consts[m.group(1)] = [t.strip() for t in _split_top(m.group(2).replace("\n", " "))]
    calls = {}
    for m in re.finditer(r"ccall\(\(:(\w+), LIB\),\s*(\w+),\s*(\(.*?\)|_\w+Sig)", src, re.S):
        name, sig = m.group(1), m.group(3)
        if sig.startswith("("):
            types = [t.strip() for t in _split_top(sig[1:-1].replace("\n", " ")) if t.strip()]
        else:
            types = consts[sig]
        calls[name] = types
    return calls


def c_prototypes():
    """{symbol: [kind, ...]} of every function declared in include/admm_deconv.h."""
    src = re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)
    protos = {}
    for m in re.finditer(r"\b(?:int|const char\*)\s+(admm_\w+)\s*\(([^)]*)\)\s*;", src, re.S):
        params = [p.strip() for p in m.group(2).replace("\n", " ").split(",") if p.strip() and p.strip() != "void"]
        kinds = []
        for p in params:
            if "*" in p:
                kinds.append("ptr")
            elif p.startswith("size_t"):
                kinds.append("size")
            elif p.startswith("float"):
                kinds.append("float")
            else:
                kinds.append("int")
        protos[m.group(1)] = kinds
    return protos


def ctypes_function(lib, name, jtypes):
    """A ctypes function of `lib` typed exactly by the Julia ccall tuple (returns Cint)."""
    f = getattr(lib, name)
    f.restype = ctypes.c_int
    f.argtypes = [JTYPES[t][1] for t in jtypes]
    return f
