"""Boundary drift (CPU): every prototype of include/cess_ec.h against the ctypes table
(cess_amd/_lib.SIGNATURES) and the Rust crate's extern declarations (utils/ec-hip/src/lib.rs),
argument by argument: arity, and per argument its ABI class (pointer, 32-bit int, 32-bit unsigned,
64-bit integer / size_t, function pointer). A drift in either binding corrupts arguments at run
time without a compiler to notice, so the CPU suite catches it here."""
import ctypes
import os
import re

import pytest

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "cess_ec.h")
RUST = os.path.join(ROOT, "utils", "ec-hip", "src", "lib.rs")

# ---- C header -------------------------------------------------------------------------------


def _strip_c_comments(txt):
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    return re.sub(r"//[^\n]*", " ", txt)


def c_class(decl: str, fn_types) -> str:
    """ABI class of one C parameter / return declaration (names dropped)."""
    d = decl.strip()
    if "*" in d or "[" in d:
        return "ptr"
    toks = [t for t in re.split(r"\s+", d) if t and t != "const"]
    if any(t in fn_types for t in toks):
        return "fn"
    base = " ".join(toks[:-1]) if len(toks) > 1 and toks[-1] not in (
        "int", "void", "size_t", "uint32_t", "uint64_t", "int32_t", "uint8_t") else " ".join(toks)
    return {"void": "void", "int": "i32", "int32_t": "i32", "uint32_t": "u32",
            "uint64_t": "u64", "size_t": "u64", "uint8_t": "u8", "long long": "i64",
            "double": "f64"}[base]


def header_prototypes():
    """{name: (ret_class, [arg_class])} of every cec_* function the header declares."""
    with open(HEADER) as f:
        txt = _strip_c_comments(f.read())
    fn_types = set(re.findall(r"\(\s*\*\s*(cec_\w+_fn)\s*\)", txt))
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w \t\*]*?)\b(cec_\w+)\s*\(([^;{}]*?)\)\s*;", txt, re.S):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        if "typedef" in ret or name.endswith("_fn"):
            continue
        ret = ret.split("\n")[-1]
        args = " ".join(args.split())
        plist = [] if args in ("", "void") else [a for a in args.split(",")]
        out[name] = (c_class(ret, fn_types), [c_class(a, fn_types) for a in plist])
    return out


# ---- ctypes ---------------------------------------------------------------------------------


def ctypes_class(t) -> str:
    if t is None:
        return "void"
    if isinstance(t, type) and issubclass(t, ctypes._CFuncPtr):
        return "fn"
    if t is ctypes.c_double:
        return "f64"
    if t in (ctypes.c_void_p, ctypes.c_char_p) or (
            isinstance(t, type) and issubclass(t, ctypes._Pointer)):
        return "ptr"
    size = ctypes.sizeof(t)
    signed = t(-1).value == -1
    if size == 4:
        return "i32" if signed else "u32"
    if size == 8:
        return "i64" if signed else "u64"
    if size == 1:
        return "u8"
    raise AssertionError(f"unclassified ctypes type {t}")


def ctypes_prototypes(sigs):
    return {n: (ctypes_class(r), [ctypes_class(a) for a in args]) for n, (r, args) in sigs.items()}


# ---- Rust -----------------------------------------------------------------------------------


def rust_class(t: str) -> str:
    t = t.strip()
    if t.startswith("*"):
        return "ptr"
    if re.fullmatch(r"(Option<\s*)?cec_\w+_fn(\s*>)?", t):
        return "fn"
    return {"c_int": "i32", "i32": "i32", "u32": "u32", "u64": "u64", "usize": "u64",
            "c_longlong": "i64", "i64": "i64", "u8": "u8", "f64": "f64"}[t]


def rust_prototypes():
    with open(RUST) as f:
        src = re.sub(r"//[^\n]*", " ", f.read())
    out = {}
    for m in re.finditer(r"pub fn (cec_\w+)\s*\(([^)]*)\)\s*(->\s*([^;]+))?;", src, re.S):
        name, args, ret = m.group(1), " ".join(m.group(2).split()), m.group(4)
        plist = [a for a in args.split(",") if a.strip()]
        out[name] = ("void" if ret is None else rust_class(ret),
                     [rust_class(a.split(":", 1)[1]) for a in plist])
    return out


def diff(want, got, who):
    bad = []
    for name, (ret, args) in want.items():
        if name not in got:
            bad.append(f"{who}: {name} missing")
            continue
        gret, gargs = got[name]
        if len(gargs) != len(args):
            bad.append(f"{who}: {name} takes {len(gargs)} arguments, header {len(args)}")
        elif gargs != args:
            bad.append(f"{who}: {name} argument classes {gargs} != header {args}")
        if gret != ret:
            bad.append(f"{who}: {name} returns {gret}, header {ret}")
    bad += [f"{who}: {n} not in the header" for n in got if n not in want]
    return bad


def test_header_parse_sanity():
    p = header_prototypes()
    assert len(p) >= 45
    assert p["cec_create"] == ("i32", ["i32", "i32", "i32", "ptr"])
    assert p["cec_destroy"] == ("void", ["ptr"])
    assert p["cec_version"] == ("ptr", [])
    assert p["cec_pipeline_run"] == ("i32", ["ptr", "fn", "fn", "fn", "ptr", "ptr"])
    assert p["cec_hashq_tick"] == ("i32", ["ptr", "u32"])


def test_ctypes_table_matches_header_per_argument():
    from cess_amd import _lib
    bad = diff(header_prototypes(), ctypes_prototypes(_lib.SIGNATURES), "ctypes")
    assert not bad, "\n".join(bad)


def test_rust_externs_match_header_per_argument():
    bad = diff(header_prototypes(), rust_prototypes(), "rust")
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("mutation", ["drop_arg", "swap_class", "extra_arg", "ret"])
def test_checker_catches_drift(mutation):
    """A deliberate change to the ctypes table fails the comparison above."""
    from cess_amd import _lib
    sigs = dict(_lib.SIGNATURES)
    res, args = sigs["cec_reconstruct_batch"]
    args = list(args)
    if mutation == "drop_arg":
        args.pop()
    elif mutation == "swap_class":
        args[4] = ctypes.c_int  # shard_len: size_t -> int
    elif mutation == "extra_arg":
        args.append(ctypes.c_void_p)
    else:
        res = None
    sigs["cec_reconstruct_batch"] = (res, args)
    assert diff(header_prototypes(), ctypes_prototypes(sigs), "ctypes")
