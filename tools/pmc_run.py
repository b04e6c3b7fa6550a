#!/usr/bin/env python
"""Short cfg-3 run for PMC collection under rocprofv3 (one process, no CPU leg)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from kbench import engine_for  # noqa: E402

pooling = sys.argv[1] if len(sys.argv) > 1 else "partial"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
eng, fam = engine_for("linreg", 256, 64, 1000, pooling, 0)
eng.set_schedule(2 * iters, 2 * iters, 1)
eng.run(0, iters)
eng.synchronize()
eng.close()
print("done")
