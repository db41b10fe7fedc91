"""kNN filter diagnostic: GPU kNN vs the oracle on C1 and a few synthetic
shapes; for mismatching rows prints the true neighbours the GPU missed."""
import os
import sys

import numpy as np

sys.path.insert(0, "tsne-flink_amd")
sys.path.insert(0, "tests")
import configs as CF  # noqa: E402
import oracle_ctypes as O  # noqa: E402
import tsne_amd as T  # noqa: E402

rng = np.random.default_rng(0)
cases = {"c1": CF.c1(), "g3000x128": rng.normal(size=(3000, 128)), "g1500x64": rng.normal(size=(1500, 64)),
         "g1500x32": rng.normal(size=(1500, 32))}
with T.Context(0) as ctx:
    for name, X in cases.items():
        gi, gd = ctx.kNearestNeighbors(X, 90)
        oi, od = O.knn(X, 90)
        bad = np.where((gi != oi).any(1) | (gd != od).any(1))[0]
        print(name, "rows differing:", len(bad), flush=True)
        for r in bad[:3]:
            miss = sorted(set(oi[r].tolist()) - set(gi[r].tolist()))
            extra = sorted(set(gi[r].tolist()) - set(oi[r].tolist()))
            print("  row", r, "missed", miss[:12], "extra", extra[:12])
