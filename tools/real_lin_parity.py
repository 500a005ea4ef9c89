"""Batch-scale parity on real linearisations: for each
system, B device-linearised problems at the reference's rho_reg = 1e-12, the
product select paths against the reference association and the oracle
(tests/real_lin.py).  Writes one JSON line per system.

    python tools/real_lin_parity.py [B] [out.jsonl]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import torch  # noqa: E402

import real_lin  # noqa: E402

Bn = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
out = sys.argv[2] if len(sys.argv) > 2 else None
dev = torch.device("cuda", 0)
lines = []
for seed, name in enumerate(real_lin.SYSTEMS):
    t0 = time.time()
    st = real_lin.stats(name, Bn, 1000 + seed, dev)
    st["wall_s"] = round(time.time() - t0, 1)
    print(json.dumps(st), flush=True)
    lines.append(st)
if out:
    with open(out, "w") as f:
        for st in lines:
            f.write(json.dumps(st) + "\n")
