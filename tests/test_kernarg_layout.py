"""The kernel-argument layout the device code assumes vs the code object's own metadata.

k_trace reads its frame records at offset 0 of the kernarg segment and its WorkArgs / FusedCopy
arguments at hand-computed offsets (kernels.hip kTraceWaOffset / kTraceFcOffset, through
__builtin_amdgcn_kernarg_segment_ptr).  This test reads the gfx950 code object out of the built
libmirt.so (the .hip_fatbin offload bundle), decodes its AMDGPU metadata note (msgpack) and
checks every instantiation of every trace kernel: explicit arguments at the offsets and sizes
the library reports (mirt_debug_kernarg_layout), hidden arguments after them, the segment
large enough.  CPU only: nothing is launched.
"""
from __future__ import annotations

import struct

import msgpack
import pytest

from distributed_raytracer_amd import _lib

NT_AMDGPU_METADATA = 32
SHT_NOTE = 7


def _sections(elf: bytes):
    assert elf[:4] == b"\x7fELF" and elf[4] == 2, "not an ELF64 file"
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = []
    for i in range(shnum):
        name, typ, _flags, _addr, off, size = struct.unpack_from("<IIQQQQ", elf, shoff + i * shentsize)
        hdrs.append((name, typ, off, size))
    stro = hdrs[shstrndx][2]
    out = []
    for name, typ, off, size in hdrs:
        end = elf.index(b"\0", stro + name)
        out.append((elf[stro + name:end].decode(), typ, off, size))
    return out


def _code_object(path: str) -> bytes:
    so = open(path, "rb").read()
    fat = [s for s in _sections(so) if s[0] == ".hip_fatbin"]
    assert fat, "libmirt.so has no .hip_fatbin section"
    _, _, off, size = fat[0]
    b = so[off:off + size]
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    assert b.startswith(magic), "offload bundle magic missing (compressed bundle?)"
    n, = struct.unpack_from("<Q", b, len(magic))
    p = len(magic) + 8
    for _ in range(n):
        boff, bsize, tsize = struct.unpack_from("<QQQ", b, p)
        triple = b[p + 24:p + 24 + tsize].decode()
        p += 24 + tsize
        if "gfx950" in triple:
            return b[boff:boff + bsize]
    raise AssertionError("no gfx950 code object in the bundle")


def _kernels(co: bytes):
    for name, typ, off, size in _sections(co):
        if typ != SHT_NOTE:
            continue
        p, end = off, off + size
        while p < end:
            namesz, descsz, ntype = struct.unpack_from("<III", co, p)
            p += 12
            nm = co[p:p + namesz].rstrip(b"\0")
            p += (namesz + 3) & ~3
            desc = co[p:p + descsz]
            p += (descsz + 3) & ~3
            if nm == b"AMDGPU" and ntype == NT_AMDGPU_METADATA:
                return msgpack.unpackb(desc, raw=False, strict_map_key=False)["amdhsa.kernels"]
    raise AssertionError("no AMDGPU metadata note")


def _align(x: int, a: int) -> int:
    return (x + a - 1) & ~(a - 1)


@pytest.fixture(scope="module")
def layout():
    L = _lib.lib()
    out = (_lib.C.c_uint64 * 8)()
    assert L.mirt_debug_kernarg_layout(out, 8) == 8
    names = ("recs", "wa_off", "wa", "fc_off", "fc", "fa", "out", "ba")
    return dict(zip(names, list(out)))


@pytest.fixture(scope="module")
def kernels():
    return _kernels(_code_object(_lib.LIB_PATH))


def _explicit(k):
    return [a for a in k[".args"] if not a[".value_kind"].startswith("hidden_")]


def _check_hidden_after(k, end):
    for a in k[".args"]:
        if a[".value_kind"].startswith("hidden_"):
            assert a[".offset"] >= end, f"{k['.name']}: {a['.value_kind']} at {a['.offset']} overlaps the arguments"
    assert k[".kernarg_segment_size"] >= end


def test_k_trace_offsets_match_metadata(layout, kernels):
    """Every k_trace instantiation: FrameRecs at 0, WorkArgs at kTraceWaOffset, FusedCopy at
    kTraceFcOffset (the offsets the kernel reads through the kernarg segment pointer)."""
    ks = [k for k in kernels if "7k_trace" in k[".name"]]
    assert len(ks) >= 8, [k[".name"] for k in kernels]
    for k in ks:
        args = _explicit(k)
        got = [(a[".offset"], a[".size"]) for a in args]
        want = [(0, layout["recs"]), (layout["wa_off"], layout["wa"]), (layout["fc_off"], layout["fc"])]
        assert got == want, f"{k['.name']}: metadata {got} vs hand-computed {want}"
        _check_hidden_after(k, layout["fc_off"] + layout["fc"])


@pytest.mark.parametrize("kname,third", [("9k_primary", "out"), ("8k_shadow", "out"), ("9k_reflect", "out"),
                                         ("8k_bounce", "ba")])
def test_split_kernels_args_by_value(layout, kernels, kname, third):
    """The split kernels take (FrameArgs, WorkArgs, third) by value: the compiler's placement is
    the natural one and the hidden arguments follow, whatever the segment's size."""
    ks = [k for k in kernels if kname in k[".name"]]
    assert ks, kname
    for k in ks:
        args = _explicit(k)
        o1 = _align(layout["fa"], 8)
        o2 = _align(o1 + layout["wa"], 8)
        want = [(0, layout["fa"]), (o1, layout["wa"]), (o2, layout[third])]
        assert [(a[".offset"], a[".size"]) for a in args] == want, k[".name"]
        _check_hidden_after(k, o2 + layout[third])


def test_every_kernel_segment_within_limit(kernels):
    """No kernel's kernarg segment exceeds the 32 KB k_trace was measured at."""
    assert max(k[".kernarg_segment_size"] for k in kernels) <= 32 * 1024
