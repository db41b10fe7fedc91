"""Summarise BH wave timelines written by `scripts/bh_snap.py --stats
--wavelog PREFIX` (option wave_log): per kind (0 the 64-query traversal, 1 the
narrow waves, 2 tile_apply) the first / last start, last end, mean / max
duration and the sum over 8192 wave slots; the traversal + narrow waves' mean
concurrency in each tenth of their span, and their start counts per tenth.

usage: python scripts/wave_timeline.py PREFIX_Y_t250.npz [...]
"""
import sys

import numpy as np


def summary(path):
    d = np.load(path)
    s = d["start"].astype(np.int64)
    e = d["end"].astype(np.int64)
    k = d["kind"]
    t0 = s.min()
    s, e = s - t0, e - t0
    lines = [f"== {path}: waves {len(s)} by kind " + str({kk: int((k == kk).sum()) for kk in (0, 1, 2)})]
    for kk, name in ((0, "traversal"), (1, "narrow"), (2, "tile_apply")):
        m = k == kk
        if not m.any():
            continue
        dur = (e[m] - s[m]) / 100.0
        lines.append(f"  {name}: first start {s[m].min() / 100:.0f} us, last start {s[m].max() / 100:.0f}, "
                     f"last end {e[m].max() / 100:.0f} us; duration mean {dur.mean():.0f} max {dur.max():.0f} us; "
                     f"sum / 8192 slots {dur.sum() / 8192:.0f} us")
    m = k < 2
    T = e[m].max()
    bins = np.linspace(0, T, 11)
    conc = [int(np.clip(np.minimum(e[m], b) - np.maximum(s[m], a), 0, None).sum() / (b - a))
            for a, b in zip(bins[:-1], bins[1:])]
    lines.append("  traversal + narrow: mean concurrent waves per tenth of the span " + str(conc))
    lines.append("  traversal + narrow: wave starts per tenth " + str(np.histogram(s[m], bins=bins)[0].tolist()))
    return "\n".join(lines)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(summary(p))
