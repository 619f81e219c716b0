#!/usr/bin/env python3
"""Interleaved one-box A/B of several environment settings at once (ab.sh
varies one switch; this takes whole settings). Each setting is a string of
NAME=VALUE words ("-" = no change); the measuring command runs once per
setting per round, and every JSON line it prints is tagged with
{"setting": ..., "round": r}.

usage: SETTINGS="CFD_HIP_CCF_KC=24;CFD_HIP_CCF_KC=32 CFD_HIP_CCF_TAIL=2" ROUNDS=3 \
       CMD="python3 tools/cg_variant_bench.py" python3 tools/env_ab.py > ab.jsonl
(k_ccf run layout, r06: SHAPES=512 VARIANTS=1 ITERS=200 CFD_HIP_CCF_KC_FIXED=1)
"""
import json
import os
import shlex
import subprocess
import sys


def main():
    settings = [s.strip() for s in os.environ["SETTINGS"].split(";") if s.strip()]
    rounds = int(os.environ.get("ROUNDS", "2"))
    cmd = shlex.split(os.environ["CMD"])
    tmo = int(os.environ.get("CMD_TIMEOUT", "300"))
    for r in range(1, rounds + 1):
        for st in settings:
            env = dict(os.environ)
            if st != "-":
                for w in st.split():
                    k, v = w.split("=", 1)
                    env[k] = v
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=tmo)
            if p.returncode != 0:
                sys.stderr.write(p.stderr[-2000:])
                raise SystemExit(f"setting {st!r}: exit {p.returncode}")
            for line in p.stdout.splitlines():
                if line.startswith("{"):
                    d = json.loads(line)
                    print(json.dumps({"setting": st, "round": r, **d}), flush=True)


if __name__ == "__main__":
    main()
