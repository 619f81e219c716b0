"""Runs tests/native/libfirst_launch_race.so in this process (torch's HIP
runtime loaded first, as in the GPU suite): one single-threaded launch loads
the code object, then groups of never-launched kernels are each launched by
3, 8 and 16 host threads at the same moment. argv[1] == "prewarm" resolves
every kernel on the main thread first; without it, concurrent pageable
host-to-device copies and concurrent allocations are probed too. Prints one
JSON line per group; a
host crash ends the process (the caller reads its exit status)."""
import ctypes
import json
import sys
from pathlib import Path

import torch  # noqa: F401  (the suite's process layout: torch's HIP runtime)

lib = ctypes.CDLL(str(Path(__file__).resolve().parent / "libfirst_launch_race.so"))
prewarm = 1 if len(sys.argv) > 1 and sys.argv[1] == "prewarm" else 0
print(json.dumps({"group": "load", "fails": lib.probe_run(1, 0, 1, 0, 1)}), flush=True)
for nt, first, count, ext in [(3, 1, 127, 1), (8, 128, 128, 0), (16, 256, 128, 1)]:
    r = lib.probe_run(nt, first, count, prewarm, ext)
    print(json.dumps({"threads": nt, "kernels": count, "prewarm": prewarm, "ext": ext,
                      "fails": r}), flush=True)
if not prewarm:  # the other shared-state suspects of the slab steps
    for nt in (3, 8):
        print(json.dumps({"probe": "memcpy_pageable_h2d", "threads": nt,
                          "fails": lib.probe_memcpy(nt, 200, 600)}), flush=True)
        print(json.dumps({"probe": "malloc_memset_launch", "threads": nt,
                          "fails": lib.probe_malloc(nt, 100)}), flush=True)
print("done", flush=True)
