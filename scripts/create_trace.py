"""Context creation, part by part (kano_create with KANO_CREATE_TRACE=1 prints
each part's time to stderr): three contexts one after another.

    KANO_CREATE_TRACE=1 python3 scripts/create_trace.py
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "kubernetes-verification_amd"))

from kano._engine import DeviceBuild  # noqa: E402

for k in range(4):
    lean = k % 2 == 1                  # kano_create, kano_create_lean alternately
    t = time.perf_counter()
    e = DeviceBuild(None, lean=lean)
    print(f"total{' (lean)' if lean else ''} {(time.perf_counter() - t) * 1e3:.3f} ms",
          file=sys.stderr, flush=True)
    e.close()
