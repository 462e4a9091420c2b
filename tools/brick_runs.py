"""How contiguous are a brick's tetra records in the background's own order?
(a brick-resident volume stage over the existing
numbering, no per-call renumbering.)  Bricks are b^3 cells of the volume
seed grid (g = cbrt(ne / 8) cells per axis); a tetra belongs to the brick of
its centroid.  For every brick: its records sorted by index, split into
maximal runs of consecutive indices; reports the share of records in runs of
at least 4 (one 128-byte line of tet8 records) and the mean run length.
    python tools/brick_runs.py [cfg4] [b ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parmmg_amd import configs, synth  # noqa: E402

w = configs.SHORT[sys.argv[1] if len(sys.argv) > 1 else "cfg4"]
bs = [int(x) for x in sys.argv[2:]] or [4, 8]
bg = synth.lattice(w.kind, w.n_old, jitter=0.0)
ne = bg.ne
g = max(1, int(round((ne / 8) ** (1 / 3))))
lo, hi = bg.xyz.min(0), bg.xyz.max(0)
cent = np.zeros((ne, 3))
for j in range(4):
    cent += bg.xyz[bg.tetv[:, j] - 1]
cent /= 4
cell = np.minimum(((cent - lo) / (hi - lo) * g).astype(np.int64), g - 1)
del cent
print(f"{w.name}: {ne} tetra, seed grid {g}^3")
for b in bs:
    nb = (g + b - 1) // b
    brick = ((cell[:, 2] // b) * nb + cell[:, 1] // b) * nb + cell[:, 0] // b
    order = np.argsort(brick, kind="stable")  # tetra by brick, ascending index inside a brick
    sb = brick[order]
    # a run breaks where the brick changes or the index is not previous + 1
    brk = np.ones(ne, bool)
    brk[1:] = (sb[1:] != sb[:-1]) | (order[1:] != order[:-1] + 1)
    starts = np.nonzero(brk)[0]
    lens = np.diff(np.append(starts, ne))
    used = np.unique(sb).shape[0]
    print(f"  bricks of {b}^3 cells: {used} non-empty, {ne / used:.0f} tetra each; runs: mean {lens.mean():.2f} "
          f"records, {100 * lens[lens >= 4].sum() / ne:.1f} % of the records in runs >= 4, "
          f"{100 * lens[lens >= 32].sum() / ne:.1f} % in runs >= 32")
