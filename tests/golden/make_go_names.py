"""Generate tests/golden/go_ref_names.json: the top-level names (funcs, methods per receiver
type, types with their struct fields, vars, consts) of the reference's Go packages that the
drop-in files under go/ are added to or import — shared/state, shared/colour, shared/geom,
worker/shared/tracer.  tests/test_go_boundary.py checks go/ against this list (no Go
toolchain exists in this image, so this is the compile check we can make: no redeclared
name, no reference to a name the reference does not export or declare).

Run here, where /root/reference exists (the GPU box has no reference tree):
    python tests/golden/make_go_names.py
The output is data (names only), not reference source.
"""
from __future__ import annotations

import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
PACKAGES = ("shared/state", "shared/colour", "shared/geom", "worker/shared/tracer")

_FUNC = re.compile(r"^func\s+(\w+)\s*[\[(]")
_METHOD = re.compile(r"^func\s+\(\s*\w*\s*\*?\s*(\w+)\s*\)\s*(\w+)\s*\(")
_TYPE = re.compile(r"^type\s+(\w+)\s+(.*)$")
_VAR = re.compile(r"^(var|const)\s+(\w+)")
_BLOCK = re.compile(r"^(var|const)\s*\($")


def strip_comments(src: str) -> str:
    src = re.sub(r"/\*.*?\*/", lambda m: "\n" * m.group(0).count("\n"), src, flags=re.S)
    out = []
    for ln in src.splitlines():
        # drop // comments outside string literals (the files below have none inside strings
        # that matter for declarations; backquoted struct tags never contain //)
        q = None
        for k, ch in enumerate(ln):
            if q:
                if ch == q and ln[k - 1] != "\\":
                    q = None
            elif ch in "\"`'":
                q = ch
            elif ch == "/" and ln[k:k + 2] == "//":
                ln = ln[:k]
                break
        out.append(ln.rstrip())
    return "\n".join(out)


def parse_go(src: str) -> dict:
    """Top-level declarations of one Go file (gofmt'ed or not: declarations start a line)."""
    src = strip_comments(src)
    pkg = re.search(r"^package\s+(\w+)", src, re.M)
    d = {"package": pkg.group(1) if pkg else None, "funcs": [], "methods": {}, "types": {}, "vars": [], "consts": []}
    lines = src.splitlines()
    i = 0
    while i < len(lines):
        ln = lines[i]
        m = _METHOD.match(ln)
        if m:
            d["methods"].setdefault(m.group(1), []).append(m.group(2))
            i += 1
            continue
        m = _FUNC.match(ln)
        if m:
            d["funcs"].append(m.group(1))
            i += 1
            continue
        m = _TYPE.match(ln)
        if m:
            name, rest = m.group(1), m.group(2)
            t = {"kind": "struct" if rest.startswith("struct") else "other", "fields": []}
            if rest.startswith("struct") and rest.rstrip().endswith("{") and not rest.rstrip().endswith("{}"):
                i += 1
                while i < len(lines) and not lines[i].startswith("}"):
                    f = lines[i].strip()
                    fm = re.match(r"^([A-Za-z_]\w*(?:\s*,\s*[A-Za-z_]\w*)*)\s+\S", f)
                    if fm:
                        t["fields"].extend(x.strip() for x in fm.group(1).split(","))
                    elif re.match(r"^\*?[\w.]+$", f):  # embedded type: its name is the field
                        t["fields"].append(f.lstrip("*").split(".")[-1])
                    i += 1
            d["types"][name] = t
            i += 1
            continue
        m = _BLOCK.match(ln)
        if m:
            kind = "vars" if m.group(1) == "var" else "consts"
            i += 1
            while i < len(lines) and not lines[i].startswith(")"):
                bm = re.match(r"^\s+(\w+)", lines[i])
                if bm:
                    d[kind].append(bm.group(1))
                i += 1
            i += 1
            continue
        m = _VAR.match(ln)
        if m:
            d["vars" if m.group(1) == "var" else "consts"].append(m.group(2))
        i += 1
    return d


def merge(into: dict, d: dict) -> None:
    into["package"] = into.get("package") or d["package"]
    into.setdefault("funcs", []).extend(d["funcs"])
    into.setdefault("methods", {})
    for t, ms in d["methods"].items():
        into.setdefault("methods", {}).setdefault(t, []).extend(ms)
    into.setdefault("types", {}).update(d["types"])
    into.setdefault("vars", []).extend(d["vars"])
    into.setdefault("consts", []).extend(d["consts"])


def main() -> None:
    if not os.path.isdir(REF):
        sys.exit(f"{REF} is not here (run this in the build container)")
    out = {"generator": "tests/golden/make_go_names.py", "reference": "MWindels/distributed-raytracer",
           "packages": {}}
    for p in PACKAGES:
        acc: dict = {}
        files = sorted(f for f in os.listdir(os.path.join(REF, p)) if f.endswith(".go"))
        for f in files:
            merge(acc, parse_go(open(os.path.join(REF, p, f)).read()))
        for k in ("funcs", "vars", "consts"):
            acc[k] = sorted(set(acc[k]))
        acc["methods"] = {t: sorted(set(v)) for t, v in sorted(acc["methods"].items())}
        acc["files"] = files
        out["packages"][p] = acc
    path = os.path.join(HERE, "go_ref_names.json")
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)
    print(f"wrote {path}")


if __name__ == "__main__":
    main()
