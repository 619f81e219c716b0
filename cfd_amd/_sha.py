"""Source identity of the native libraries, shared by the build and the loader.

`library_source_sha()` hashes every file libcfd_hip.so is built from
(csrc/hip/*.hip|*.hpp, csrc/host/*.c|*.h, csrc/Makefile, include/cfd_hip/*.h);
the Makefile embeds it in the library as hip_proj_build_id() and
cfd_amd._native refuses a library whose id differs from the sources beside it.
`kernel_source_sha()` hashes the HIP sources only, and `device_code_sha(lib)`
the device code inside a built library: PMC profiles are keyed on both
(their byte counts depend on the kernels, not on host code; the HIP sources
also hold host code, so a host-only edit changes the first key, not the
second).

Standard library only: the Makefile runs this file as a script
(`python3 _sha.py` prints the library sha).
"""
from __future__ import annotations

import hashlib
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC_DIR = PKG_DIR / "csrc"
INC_DIR = PKG_DIR.parent / "include" / "cfd_hip"


def _digest(files) -> str:
    h = hashlib.sha256()
    for f in files:
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()[:16]


def kernel_source_sha() -> str:
    hip = CSRC_DIR / "hip"
    return _digest(sorted(hip.glob("*.hip")) + sorted(hip.glob("*.hpp")))


def _elf_sections(data: bytes) -> dict:
    """name -> [(offset, size)] of an ELF64 little-endian image."""
    import struct

    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)

    def sec(i):
        return struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize)

    str_off = sec(shstrndx)[4]
    out: dict = {}
    for i in range(shnum):
        name_off, _typ, _flags, _addr, off, size = sec(i)
        end = data.index(b"\0", str_off + name_off)
        out.setdefault(data[str_off + name_off:end].decode(), []).append((off, size))
    return out


def _offload_bundles(fb: bytes):
    """(triple, image) of every clang offload bundle in a .hip_fatbin blob."""
    import struct

    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos = fb.find(magic)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fb, pos + 24)
        q = pos + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", fb, q)
            q += 24
            triple = fb[q:q + tl].decode()
            q += tl
            yield triple, fb[pos + off:pos + off + size]
        pos = fb.find(magic, pos + 1)


def device_code_sha(lib) -> str | None:
    """sha256[:16] of the gfx950 device code inside a built library: the
    .text and .rodata (instructions and kernel descriptors) of every code
    object in its .hip_fatbin. Host-only source edits and the build
    directory (which enters the per-file compilation id, hence the code
    objects' symbols) leave it unchanged; any kernel change alters it. None
    for a file without gfx950 code."""
    data = Path(lib).read_bytes()
    if data[:4] != b"\x7fELF" or data[4] != 2 or data[5] != 1:
        return None
    h = hashlib.sha256()
    n = 0
    for off, size in _elf_sections(data).get(".hip_fatbin", []):
        for triple, co in _offload_bundles(data[off:off + size]):
            if "gfx950" not in triple:
                continue
            n += 1
            secs = _elf_sections(co)
            for name in (".text", ".rodata"):
                for o, z in secs.get(name, []):
                    h.update(co[o:o + z])
    return h.hexdigest()[:16] if n else None


def library_source_sha() -> str:
    hip, host = CSRC_DIR / "hip", CSRC_DIR / "host"
    files = (sorted(hip.glob("*.hip")) + sorted(hip.glob("*.hpp")) + sorted(host.glob("*.c"))
             + sorted(host.glob("*.h")) + [CSRC_DIR / "Makefile"] + sorted(INC_DIR.glob("*.h")))
    return _digest(files)


if __name__ == "__main__":
    print(library_source_sha())
