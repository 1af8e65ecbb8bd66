"""The Go drop-in files under go/ against the reference's declared names and include/mirt.h
(reference worker/distributed/main.go:46-185).

No Go toolchain exists in this image or on the GPU box, so this is the compile check that
can be made here, CPU only:
  * go/shared/state and go/shared/colour are NEW files added to the reference's packages:
    they must redeclare no top-level name of that package (tests/golden/go_ref_names.json,
    extracted from the reference by tests/golden/make_go_names.py) and add no method whose
    name is already a method or field of its receiver type;
  * every `state.X` / `colour.X` / `geom.X` the files use is exported and declared by the
    reference or by the accessors these files add;
  * every selector on a value is a field or method the reference, these files, mirt.h's
    structs or the Go / gRPC APIs used declare (a typo'd or removed field fails here);
  * every `C.name` the cgo binding uses is declared by include/mirt.h (or is a cgo / libc
    builtin), every C struct field it touches exists, and every `C.mirt_*` call passes as many
    arguments as the prototype takes;
  * the cgo directives hold no fixed path: where libmirt lives comes from CGO_CFLAGS /
    CGO_LDFLAGS.
"""
from __future__ import annotations

import json
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "go")
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from make_go_names import parse_go, strip_comments  # noqa: E402

REF = json.load(open(os.path.join(ROOT, "tests", "golden", "go_ref_names.json")))["packages"]
IMPORT_PATH = "github.com/mwindels/distributed-raytracer/"
# which reference package each added file joins
ADDED = {"shared/state/export_mirt.go": "shared/state", "shared/colour/export_mirt.go": "shared/colour"}
# selectors of the Go standard library, gRPC / protobuf generated code and rtreego the files call
EXTERNAL_SELECTORS = {
    "Err", "Done", "Decode", "Close", "Serve", "GracefulStop", "Register", "SearchCondition",
    "GetX", "GetY", "GetWidth", "GetHeight", "GetDiff", "GetState", "GetScreenWidth", "GetScreenHeight",
    "Results", "R", "G", "B", "Port",
}
CGO_BUILTINS = {"double", "int", "char", "size_t", "uint8_t", "uint32_t", "uint64_t", "calloc", "malloc", "free",
                "GoString", "GoBytes", "CString"}


def go_files():
    out = []
    for d, _, fs in os.walk(GO):
        out += [os.path.relpath(os.path.join(d, f), GO) for f in fs if f.endswith(".go")]
    return sorted(out)


def code(rel):
    return strip_comments(open(os.path.join(GO, rel)).read())


def imports(src):
    """alias -> import path (an unaliased import is known by its last element)."""
    out = {}
    blk = re.search(r"^import\s*\((.*?)^\)", src, re.S | re.M)
    specs = blk.group(1).splitlines() if blk else re.findall(r"^import\s+(.*)$", src, re.M)
    for s in specs:
        m = re.match(r'\s*(\w+)?\s*"([^"]+)"', s)
        if m:
            out[m.group(1) or m.group(2).rsplit("/", 1)[-1]] = m.group(2)
    return out


def strip_strings(src):
    return re.sub(r'"(?:\\.|[^"\\])*"|`[^`]*`', '""', src)


def our_decls():
    """Everything the go/ files declare: (package dir -> parse), merged per package name."""
    per = {}
    for rel in go_files():
        per[rel] = parse_go(open(os.path.join(GO, rel)).read())
    return per


def header_decls():
    """include/mirt.h: prototypes (name -> parameter count), struct fields, macros, types."""
    src = open(os.path.join(ROOT, "include", "mirt.h")).read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    src = re.sub(r"//[^\n]*", " ", src)
    macros = set(re.findall(r"^\s*#define\s+(\w+)", src, re.M))
    flat = re.sub(r"^\s*#.*$", " ", src, flags=re.M)
    protos = {}
    for name, params in re.findall(r"\b(mirt_\w+)\s*\(([^;{)]*)\)\s*;", flat):
        p = params.strip()
        protos[name] = 0 if p in ("", "void") else p.count(",") + 1
    fields, types = set(), set(re.findall(r"typedef\s+struct\s+\w*\s*(?:\{[^}]*\})?\s*(\w+)\s*;", flat))
    for body in re.findall(r"typedef\s+struct\s*\w*\s*\{([^}]*)\}", flat):
        for decl in body.split(";"):
            decl = re.sub(r"\[[^\]]*\]", "", decl).strip()
            if not decl:
                continue
            parts = decl.split(",")
            first = parts[0].split()
            names = [first[-1]] + [p.strip() for p in parts[1:]]
            fields |= {n.lstrip("*") for n in names}
    return protos, fields, macros, types


def call_arity(src, start):
    """Top-level argument count of the call whose '(' is at src[start]."""
    depth, n, saw = 0, 0, False
    for ch in src[start:]:
        if ch in "([{":
            depth += 1
            if depth == 1:
                continue
        elif ch in ")]}":
            depth -= 1
            if depth == 0:
                return n + 1 if saw else 0
        elif ch == "," and depth == 1:
            n += 1
        if depth >= 1 and not ch.isspace():
            saw = True
    raise AssertionError("unbalanced call")


@pytest.mark.parametrize("rel,pkg", sorted(ADDED.items()))
def test_added_files_redeclare_nothing(rel, pkg):
    ref = REF[pkg]
    d = parse_go(open(os.path.join(GO, rel)).read())
    assert d["package"] == ref["package"], f"{rel}: package {d['package']} is not {ref['package']}"
    top = set(ref["funcs"]) | set(ref["types"]) | set(ref["vars"]) | set(ref["consts"])
    mine = (set(d["funcs"]) - {"init"}) | set(d["types"]) | set(d["vars"]) | set(d["consts"])
    assert not (mine & top), f"{rel} redeclares {sorted(mine & top)} of package {pkg}"
    for t, ms in d["methods"].items():
        taken = set(ref["methods"].get(t, [])) | set(ref["types"].get(t, {}).get("fields", []))
        assert not (set(ms) & taken), f"{rel}: {t} already has {sorted(set(ms) & taken)}"
        assert t in ref["types"] or t in d["types"], f"{rel}: methods on unknown type {t}"


def test_package_qualified_names_exist():
    decl = our_decls()
    added = {pkg: decl[rel] for rel, pkg in ADDED.items()}
    for rel in go_files():
        src = strip_strings(code(rel))
        for alias, path in imports(code(rel)).items():
            if not path.startswith(IMPORT_PATH):
                continue
            pkg = path[len(IMPORT_PATH):]
            if pkg not in REF:
                continue  # comms (generated), worker/shared/gpu (ours)
            ref = REF[pkg]
            known = set(ref["funcs"]) | set(ref["types"]) | set(ref["vars"]) | set(ref["consts"])
            if pkg in added:
                a = added[pkg]
                known |= set(a["funcs"]) | set(a["types"]) | set(a["vars"]) | set(a["consts"])
            for name in re.findall(rf"\b{alias}\.(\w+)", src):
                assert name[0].isupper(), f"{rel}: {alias}.{name} is unexported"
                assert name in known, f"{rel}: {alias}.{name} is not declared by {pkg}"


def test_value_selectors_exist():
    """Every `.name` on a value is a field / method the reference, go/, mirt.h or the external
    APIs declare."""
    decl = our_decls()
    known = set(EXTERNAL_SELECTORS)
    for ref in REF.values():
        for t, v in ref["types"].items():
            known |= set(v["fields"])
        for ms in ref["methods"].values():
            known |= set(ms)
    for d in decl.values():
        for t, v in d["types"].items():
            known |= set(v["fields"])
        for ms in d["methods"].values():
            known |= set(ms)
    _, cfields, _, _ = header_decls()
    for rel in go_files():
        src = strip_strings(code(rel))
        aliases = set(imports(code(rel))) | {"C"}
        for lhs, name in re.findall(r"(?<![\w.])([A-Za-z_]\w*|\)|\])\s*\.\s*([A-Za-z_]\w*)", src):
            if lhs in aliases or name == "":
                continue
            if rel.endswith("gpu/mirt.go") and name in cfields:
                continue
            assert name in known, f"{rel}: selector .{name} (on {lhs}) is declared nowhere"


def test_cgo_binding_matches_header():
    protos, fields, macros, types = header_decls()
    rel = "worker/shared/gpu/mirt.go"
    raw = open(os.path.join(GO, rel)).read()
    directives = re.findall(r"^#cgo\s+(.*)$", raw, re.M)
    assert directives, "no #cgo directive"
    for d in directives:
        assert "${SRCDIR}" not in d and not re.search(r"-[IL]\s*\S", d), \
            f"fixed path in '#cgo {d}': use CGO_CFLAGS / CGO_LDFLAGS (INTEGRATION.md)"
    assert any("-lmirt" in d for d in directives)
    assert '#include "mirt.h"' in raw
    src = strip_strings(code(rel))
    for name in set(re.findall(r"\bC\.(\w+)", src)):
        ok = name in CGO_BUILTINS or name in protos or name in macros or name in types or name in (
            "mirt_ctx", "mirt_group")
        assert ok, f"{rel}: C.{name} is not declared by include/mirt.h"
    for m in re.finditer(r"\bC\.(mirt_\w+)\s*\(", src):
        name = m.group(1)
        if name in types:
            continue  # a conversion, not a call
        n = call_arity(src, m.end() - 1)
        assert n == protos[name], f"{rel}: C.{name} called with {n} arguments, mirt.h takes {protos[name]}"
    assert protos["mirt_trace_tile"] >= 10 and "rgb8" in fields and "proj_half_width" in fields
    # the box-level worker (one process, the box's GPUs): created, fed meshes and orders through the box
    for n in ("mirt_box_create", "mirt_box_mesh_upload", "mirt_box_trace_tile", "mirt_box_destroy", "mirt_device_count"):
        assert f"C.{n}(" in src, f"{rel} does not call {n}"


def test_header_parser_sees_the_boundary():
    """The checker itself: it finds the entries and fields INTEGRATION.md names."""
    protos, fields, macros, types = header_decls()
    for n in ("mirt_create", "mirt_mesh_upload", "mirt_trace_tile", "mirt_trace_frame", "mirt_group_create"):
        assert n in protos
    assert {"mirt_frame", "mirt_outputs", "mirt_material", "mirt_camera"} <= types
    assert {"MIRT_OK", "MIRT_MAX_OBJECTS", "MIRT_MAX_LIGHTS"} <= macros
    assert {"ka", "ns", "mesh_id", "n_objects", "n_lights", "max_bounces"} <= fields
