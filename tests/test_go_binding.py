"""Mechanical check of the cgo binding against include/hundcrc.h (CPU suite).

No Go toolchain exists here or on the GPU box, so nothing compiles the cgo
files under integration/go.  This test does the part of cgo's type check that
catches a drifting header: for every `C.hc_*(...)` call it

  * counts the top-level arguments against the prototype in hundcrc.h;
  * infers each argument's C type from the Go expression -- `C.uint64_t(x)`,
    `(*C.uint32_t)(unsafe.Pointer(...))`, `&v` / `&v[0]` of a variable declared
    `var v C.int64_t` or `v := make([]C.int, ...)`, a helper returning
    `*C.uint8_t`, `rc := C.hc_f(...)` (the return type of hc_f), `nil`, an
    untyped integer constant -- and requires it to be the parameter's type
    (`const` ignored, `T x[16]` is `T *`, `void *` takes unsafe.Pointer or nil);
  * for arguments that name a variable (`&v`, `&v[0]`, `C.T(v)`), requires the
    variable's name to match the parameter's (one is a subsequence of the
    other, case and underscores ignored: `posBlock` ~ `pos_block`, `ln` ~
    `rec_len`), which catches two same-typed arguments swapped.

test_checker_catches_mutations drops, swaps and retypes arguments of the
17-argument hc_wal_replay_v call in crc_util.go and of every other call, and
requires the checker to report each mutation.
"""
import os
import re


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO_DIR = os.path.join(ROOT, "integration", "go")

SCALARS = {"int", "size_t", "uint8_t", "uint32_t", "uint64_t", "int64_t", "int32_t", "uint16_t", "char"}


def _norm_ctype(t):
    t = re.sub(r"\bconst\b", "", t)
    t = re.sub(r"\s+", "", t)
    return t


def header_prototypes():
    """{name: (return type, [(param type, param name)])} from include/hundcrc.h."""
    src = open(os.path.join(ROOT, "include", "hundcrc.h")).read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    src = re.sub(r"^\s*#.*$", " ", src, flags=re.M)
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(hc_[a-z0-9_]+)\s*\(([^;{}]*?)\)\s*;", src):
        ret, name, params = m.group(1), m.group(2), m.group(3).strip()
        ret = _norm_ctype(ret.split("}")[-1])
        plist = []
        if params and params != "void":
            for p in params.split(","):
                p = p.strip()
                arr = re.match(r"(.*?)(\w+)\s*\[\s*\d*\s*\]$", p)
                if arr:
                    ptype, pname = _norm_ctype(arr.group(1)) + "*", arr.group(2)
                else:
                    pm = re.match(r"(.*?)(\w+)$", p)
                    ptype, pname = _norm_ctype(pm.group(1)), pm.group(2)
                plist.append((ptype, pname))
        protos[name] = (ret, plist)
    return protos


def _split_top(s):
    """Split at top-level commas (outside (), [], {} and string literals)."""
    out, depth, cur, q = [], 0, [], None
    for ch in s:
        if q:
            cur.append(ch)
            if ch == q:
                q = None
            continue
        if ch in "\"'`":
            q = ch
        elif ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append("".join(cur).strip())
            cur = []
        else:
            cur.append(ch)
    if "".join(cur).strip():
        out.append("".join(cur).strip())
    return out


def _close_paren(src, i):
    """Index of the ')' matching the '(' at src[i]."""
    depth = 0
    for j in range(i, len(src)):
        if src[j] == "(":
            depth += 1
        elif src[j] == ")":
            depth -= 1
            if depth == 0:
                return j
    raise ValueError("unbalanced parentheses")


def _strip_go_comments(src):
    src = re.sub(r"/\*.*?\*/", lambda m: "\n" * m.group(0).count("\n"), src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def _scopes(src):
    """Top-level Go declarations (func bodies) with their text, plus the file."""
    starts = [m.start() for m in re.finditer(r"^func\b", src, flags=re.M)] + [len(src)]
    return [src[starts[k]:starts[k + 1]] for k in range(len(starts) - 1)]


def _declared(scope, protos, helpers):
    """Variable name -> C type ('T', 'T*', or 'T[]' for slices) in one func."""
    env = {}
    sig = re.match(r"func\s+(?:\([^)]*\)\s*)?\w+\(([^)]*)\)", scope)
    if sig:  # parameters declared C.T in the func's own signature
        for m in re.finditer(r"(\w+)\s+(\*?)C\.(\w+)", sig.group(1)):
            env[m.group(1)] = m.group(3) + ("*" if m.group(2) else "")
    for m in re.finditer(r"\bvar\s+([\w\s,]+?)\s+(\*?)C\.(\w+)", scope):
        for v in m.group(1).split(","):
            env[v.strip()] = m.group(3) + ("*" if m.group(2) else "")
    for m in re.finditer(r"\b(\w+)\s*:?=\s*make\(\[\]C\.(\w+)", scope):
        env[m.group(1)] = m.group(2) + "[]"
    for m in re.finditer(r"\b(\w+)\s*:?=\s*C\.(hc_\w+)\(", scope):
        if m.group(2) in protos:
            env[m.group(1)] = protos[m.group(2)][0]
    for m in re.finditer(r"\b(\w+)\s*:?=\s*(\w+)\(", scope):
        if m.group(2) in helpers:
            env[m.group(1)] = helpers[m.group(2)]
    return env


def _subseq(a, b):
    it = iter(b)
    return all(ch in it for ch in a)


# Go variable -> parameters it may fill although the names differ: a batch of
# equal blocks passes its block size as both stride and ulen (hundcrc.h
# "off==NULL -> off[i] = i*stride; len==NULL -> len[i] = ulen").
NAME_ALIASES = {"blocksize": {"stride", "ulen", "blocksize"}}


def _names_match(go_name, c_name):
    a, b = go_name.lower().replace("_", ""), c_name.lower().replace("_", "")
    return _subseq(a, b) or _subseq(b, a) or b in NAME_ALIASES.get(a, ())


def infer(expr, env, helpers):
    """(C type or marker, variable name or None) for a Go argument expression."""
    e = expr.strip()
    if e == "nil":
        return "nil", None
    if re.fullmatch(r"-?\d+|C\.HC_\w+|\^?C\.\w+\(0\)", e) and not re.fullmatch(r"C\.\w+\(\w+\)", e):
        return "const", None
    m = re.fullmatch(r"C\.(\w+)\((.*)\)", e, flags=re.S)
    if m and m.group(1) in SCALARS:
        inner = m.group(2).strip()
        return m.group(1), inner if re.fullmatch(r"\w+", inner) else None
    m = re.fullmatch(r"\(\*C\.(\w+)\)\(unsafe\.Pointer\((.*)\)\)", e, flags=re.S)
    if m:
        inner = re.fullmatch(r"&(\w+)(\[[^\]]*\])*", m.group(2).strip())
        return m.group(1) + "*", inner.group(1) if inner else None
    if re.fullmatch(r"unsafe\.Pointer\(.*\)", e, flags=re.S):
        return "void*", None
    m = re.fullmatch(r"&(\w+)(\[[^\]]*\])?", e)
    if m:
        t = env.get(m.group(1))
        if t is None:
            return None, m.group(1)
        if m.group(2):
            return (t[:-2] + "*" if t.endswith("[]") else None), m.group(1)
        return t + "*", m.group(1)
    m = re.fullmatch(r"(\w+)\((.*)\)", e, flags=re.S)
    if m and m.group(1) in helpers:
        return helpers[m.group(1)], None
    if re.fullmatch(r"\w+", e):
        return env.get(e), None
    return None, None


def check_source(src, protos, fname="<src>"):
    """Every mismatch between the cgo calls in one Go file and hundcrc.h."""
    src = _strip_go_comments(src)
    helpers = {m.group(1): m.group(2) + "*"
               for m in re.finditer(r"^func\s+(\w+)\([^)]*\)\s*\*C\.(\w+)\s*\{", src, flags=re.M)}
    errors, calls = [], 0
    for scope in _scopes(src) or [src]:
        env = _declared(scope, protos, helpers)
        for m in re.finditer(r"\bC\.(hc_[a-z0-9_]+)\(", scope):
            name = m.group(1)
            calls += 1
            where = f"{fname}: C.{name}"
            if name not in protos:
                errors.append(f"{where}: not declared in hundcrc.h")
                continue
            open_i = m.end() - 1
            args = _split_top(scope[open_i + 1:_close_paren(scope, open_i)])
            params = protos[name][1]
            if len(args) != len(params):
                errors.append(f"{where}: {len(args)} arguments, hundcrc.h declares {len(params)}")
                continue
            for k, (arg, (ptype, pname)) in enumerate(zip(args, params)):
                got, var = infer(arg, env, helpers)
                is_ptr = ptype.endswith("*")
                if got is None:
                    errors.append(f"{where} arg {k + 1} `{arg}`: C type not inferable (cast it explicitly)")
                    continue
                if got == "nil":
                    ok = is_ptr
                elif got == "const":
                    ok = not is_ptr
                elif ptype == "void*":
                    ok = got == "void*"
                else:
                    ok = got == ptype
                if not ok:
                    errors.append(f"{where} arg {k + 1} `{arg}`: Go passes {got}, hundcrc.h wants {ptype} {pname}")
                elif var is not None and not _names_match(var, pname):
                    errors.append(f"{where} arg {k + 1} `{arg}`: variable {var!r} passed as parameter {pname!r}")
    return errors, calls


def go_files():
    out = []
    for dirpath, _dirs, files in os.walk(GO_DIR):
        out += [os.path.join(dirpath, f) for f in files if f.endswith(".go")]
    return sorted(out)


def test_header_parses():
    protos = header_prototypes()
    assert len(protos) >= 40
    assert protos["hc_wal_replay_v"][1][10] == ("uint64_t*", "rec_end_block")
    assert len(protos["hc_wal_replay_v"][1]) == 17
    assert protos["hc_md5"][1][2] == ("uint8_t*", "out")
    assert protos["hc_version"] == ("char*", [])


def test_every_cgo_call_matches_the_header():
    protos = header_prototypes()
    total, errors = 0, []
    for path in go_files():
        e, n = check_source(open(path).read(), protos, os.path.relpath(path, ROOT))
        errors += e
        total += n
    assert total >= 25, total
    assert not errors, "\n".join(errors)


def _call_span(src, name):
    i = src.index(f"C.{name}(")
    open_i = i + len(f"C.{name}")
    return open_i + 1, _close_paren(src, open_i)


def test_checker_catches_mutations():
    """Dropping any argument, swapping any two adjacent arguments that differ,
    or changing a scalar cast is reported, for every call in every file."""
    protos = header_prototypes()
    crc = open(os.path.join(GO_DIR, "utils", "crc", "crc_util.go")).read()
    # the verdict's case: hc_wal_replay_v (crc_util.go WalReplay), 17 arguments
    a, b = _call_span(crc, "hc_wal_replay_v")
    n = len(_split_top(crc[a:b]))
    assert n == 17
    missed, tried = [], 0
    for path in go_files():
        src = open(path).read()
        base_err, _ = check_source(src, protos)
        assert not base_err
        clean = _strip_go_comments(src)
        for m in re.finditer(r"\bC\.(hc_[a-z0-9_]+)\(", clean):
            name = m.group(1)
            open_i = m.end() - 1
            args = _split_top(clean[open_i + 1:_close_paren(clean, open_i)])

            def mutated(new_args):
                return clean[:open_i + 1] + ", ".join(new_args) + clean[_close_paren(clean, open_i):]

            variants = []
            for k in range(len(args)):
                variants.append((f"drop {k + 1}", args[:k] + args[k + 1:]))
            for k in range(len(args) - 1):
                if args[k] != args[k + 1]:
                    s = list(args)
                    s[k], s[k + 1] = s[k + 1], s[k]
                    variants.append((f"swap {k + 1}/{k + 2}", s))
            for k, arg in enumerate(args):
                c = re.fullmatch(r"C\.(uint64_t|uint32_t|size_t|int)\((.*)\)", arg, flags=re.S)
                if c:
                    other = "int64_t" if c.group(1) != "int64_t" else "uint64_t"
                    s = list(args)
                    s[k] = f"C.{other}({c.group(2)})"
                    variants.append((f"retype {k + 1}", s))
            for what, new_args in variants:
                tried += 1
                errs, _ = check_source(mutated(new_args), protos)
                if not errs:
                    missed.append(f"{os.path.relpath(path, ROOT)} C.{name}: {what} ({new_args})")
    assert tried >= 150, tried
    assert not missed, "\n".join(missed)
