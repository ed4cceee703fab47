"""Per-kernel resource metadata of the gfx950 code objects inside libpsgla_hip.so (no ROCm tools needed).

The shared library's .hip_fatbin holds one clang offload bundle per translation unit; each bundle's gfx950 entry is an
AMDGPU ELF whose NT_AMDGPU_METADATA note (msgpack) lists every kernel with its .vgpr_count, .vgpr_spill_count,
.sgpr_spill_count and .private_segment_fixed_size.  Used by tests/test_native_abi.py (no shipped kernel may spill a
VGPR: DESIGN.md 3.9) and from the command line:

    python3 tools/code_object_meta.py [path/to/libpsgla_hip.so]
"""
from __future__ import annotations

import os
import struct
import sys

import msgpack

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
NT_AMDGPU_METADATA = 32


def _bundles(data: bytes):
    """(triple, bytes) of every entry of every offload bundle in `data`."""
    i = data.find(MAGIC)
    while i >= 0:
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode()
            p += tl
            if size:
                yield triple, data[i + off:i + off + size]
        i = data.find(MAGIC, i + 1)


def _notes(elf: bytes):
    """Payloads of the ELF64 notes (SHT_NOTE sections) named AMDGPU of type NT_AMDGPU_METADATA."""
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    for k in range(shnum):
        sh = shoff + k * shentsize
        sh_type, = struct.unpack_from("<I", elf, sh + 4)
        if sh_type != 7:                                    # SHT_NOTE
            continue
        off, size = struct.unpack_from("<QQ", elf, sh + 0x18)
        p, end = off, off + size
        while p + 12 <= end:
            namesz, descsz, ntype = struct.unpack_from("<III", elf, p)
            name = elf[p + 12:p + 12 + namesz].rstrip(b"\0")
            q = p + 12 + ((namesz + 3) & ~3)
            if name == b"AMDGPU" and ntype == NT_AMDGPU_METADATA:
                yield elf[q:q + descsz]
            p = q + ((descsz + 3) & ~3)


def kernels(lib_path: str, arch: str = "gfx950") -> list[dict]:
    """One dict per kernel of the library's `arch` code objects (the metadata map of each kernel)."""
    data = open(lib_path, "rb").read()
    out = []
    for triple, blob in _bundles(data):
        if not triple.endswith(arch):
            continue
        for note in _notes(blob):
            meta = msgpack.unpackb(note, raw=False, strict_map_key=False)
            out.extend(meta.get("amdhsa.kernels", []))
    return out


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "psgla_for_posterior_sampling_amd", "libpsgla_hip.so")
    ks = kernels(path)
    for k in sorted(ks, key=lambda k: k[".name"]):
        print(f"{k['.name'][:100]:100s} vgpr {k.get('.vgpr_count', '?'):>4} agpr {k.get('.agpr_count', '?'):>4} "
              f"vspill {k.get('.vgpr_spill_count', '?'):>3} sspill {k.get('.sgpr_spill_count', '?'):>4} "
              f"private {k.get('.private_segment_fixed_size', '?'):>5}")
    print(f"{len(ks)} kernels")


if __name__ == "__main__":
    main()
