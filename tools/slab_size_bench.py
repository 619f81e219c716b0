#!/usr/bin/env python3
"""Per-iteration CG time on slab-sized domains on ONE GPU: what each rank of
an N-way Z-slab split of n^3 computes, without the communication. Run on the
GPU box: python tools/slab_size_bench.py [--n 512] [--ranks 1 2 4 8]"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from cfd_amd import api  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--ranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--kchunk", type=int, nargs="+", default=[0])
    a = ap.parse_args()
    n = a.n
    for R in a.ranks:
        _, nzl = api.slab_layout(n, 0, R)
        for kc in a.kchunk:
            ctx = api.HipProjection(n, n, nzl, kchunk=kc)
            rhs = np.zeros((nzl, n, n))
            rhs[1:-1, 1:-1, 1:-1] = np.cos(np.linspace(0, 3, n - 2))[None, None, :]
            d = 1.0 / (n - 1)
            ctx.cg_fixed_iters(rhs, d, d, d, 20)  # warm
            ms = ctx.cg_fixed_iters(rhs, d, d, d, a.iters)
            kt = None
            ctx.close()
            cells = (n - 2) ** 2 * (nzl - 2)
            it_us = ms / a.iters * 1e3
            print(json.dumps({"ranks": R, "nz_local": nzl, "kchunk": kc,
                              "cg_iter_us": round(it_us, 2),
                              "GBps_64B": round(64.0 * cells / (it_us * 1e-6) / 1e9, 1)}))


if __name__ == "__main__":
    main()
