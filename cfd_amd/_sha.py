"""Source identity of the native libraries, shared by the build and the loader.

`library_source_sha()` hashes every file libcfd_hip.so is built from
(csrc/hip/*.hip|*.hpp, csrc/host/*.c|*.h, csrc/Makefile, include/cfd_hip/*.h);
the Makefile embeds it in the library as hip_proj_build_id() and
cfd_amd._native refuses a library whose id differs from the sources beside it.
`kernel_source_sha()` hashes the HIP sources only: PMC profiles are keyed on it
(their byte counts depend on the kernels, not on host code).

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


def library_source_sha() -> str:
    hip, host = CSRC_DIR / "hip", CSRC_DIR / "host"
    files = (sorted(hip.glob("*.hip")) + sorted(hip.glob("*.hpp")) + sorted(host.glob("*.c"))
             + sorted(host.glob("*.h")) + [CSRC_DIR / "Makefile"] + sorted(INC_DIR.glob("*.h")))
    return _digest(files)


if __name__ == "__main__":
    print(library_source_sha())
