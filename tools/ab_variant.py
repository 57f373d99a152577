"""Build a timing or A/B variant of libhundcrc from the product sources:
copies hunddb_amd/csrc + Makefile to tools/ab/<name>/, applies exact string
replacements to one source file and builds tools/ab/<name>/libhundcrc.so
(tools/ab/ is git-ignored; bench.py loads a variant with HUNDCRC_LIB=...).

  python tools/ab_variant.py <name> <file in csrc> <spec.py> [source file]

spec.py defines SUBS = [(old, new), ...]; every `old` must occur exactly once.
An optional source file replaces csrc/<file> before the substitutions (a
variant stacked on an uncommitted one, e.g. a patch applied elsewhere)."""
import os
import runpy
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    name, fname, spec = sys.argv[1:4]
    alt = sys.argv[4] if len(sys.argv) > 4 else None
    dst = os.path.join(ROOT, "tools", "ab", name)
    shutil.rmtree(dst, ignore_errors=True)
    shutil.copytree(os.path.join(ROOT, "hunddb_amd", "csrc"), os.path.join(dst, "csrc"))
    shutil.copy(os.path.join(ROOT, "hunddb_amd", "Makefile"), dst)
    inc = os.path.join(ROOT, "tools", "ab", "include")
    os.makedirs(inc, exist_ok=True)
    shutil.copy(os.path.join(ROOT, "include", "hundcrc.h"), inc)
    path = os.path.join(dst, "csrc", fname)
    if alt:
        shutil.copy(alt, path)
    src = open(path).read()
    for old, new in runpy.run_path(spec)["SUBS"]:
        k = src.count(old)
        if k != 1:
            raise SystemExit(f"{name}: pattern occurs {k} times: {old[:80]!r}")
        src = src.replace(old, new)
    open(path, "w").write(src)
    subprocess.run(["make", "-s", "-j8", "-C", dst, "libhundcrc.so"], check=True)
    print(os.path.join(dst, "libhundcrc.so"))


if __name__ == "__main__":
    main()
