"""Build identity of libflinkgpu.so for measurement provenance.

A PMC pass (profiles/**/pmc_traffic.json) counts the HBM bytes of the engine's KERNELS, so it is
keyed by the sha256 of the library's device code -- the `.hip_fatbin` section holding the gfx950
code objects of every translation unit -- not of the whole file: a host-only change (fg_engine.cpp's
C++ side) leaves the kernels, and so their traffic, unchanged, and keeps the summary valid.
"""
from __future__ import annotations

import hashlib
import os
import struct

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "flink_amd", "libflinkgpu.so")


def file_sha256(path: str = LIB) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def elf_section(path: str, name: str) -> bytes:
    """Bytes of section `name` of a little-endian ELF64 file (section headers + .shstrtab)."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"\x7fELF" or data[4] != 2 or data[5] != 1:
        raise ValueError(f"{path}: not a little-endian ELF64 file")
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)

    def sh(i):
        # sh_name, sh_type, sh_flags, sh_addr, sh_offset, sh_size
        return struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize)
    strtab = sh(shstrndx)
    names = data[strtab[4]:strtab[4] + strtab[5]]
    for i in range(shnum):
        s = sh(i)
        nm = names[s[0]:names.index(b"\0", s[0])].decode()
        if nm == name:
            return data[s[4]:s[4] + s[5]]
    raise KeyError(f"{path}: no section {name}")


def kernels_sha256(path: str = LIB) -> str:
    """sha256 of the device code objects (.hip_fatbin) of the library."""
    return hashlib.sha256(elf_section(path, ".hip_fatbin")).hexdigest()
