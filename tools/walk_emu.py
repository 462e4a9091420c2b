"""CPU emulation of the module's exact fp64 walk (pmmg_vol.hpp walk_exact:
the most-negative eligible face, a 4-entry visited history, the stochastic
rule past kDetSteps), vectorised over queries with numpy — a diagnostic for
walks that never reach an accepting tetra (2655 interior walks of
the carried cfg4 iteration hit the step cap).

  python tools/walk_emu.py --n-old 134 --n-new 142 [--maxstep 1024] [--seed-mode centroid|far]

Builds the second iteration's geometry (background: the jittered shell
lattice of the first iteration's new mesh; queries: the unjittered background
points, volume class only), seeds each walk at the tetra whose centroid is
nearest, walks every query in lockstep and reports how many reach the cap,
with the first steps of a few of them.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from parmmg_amd import synth  # noqa: E402

EPS = 1e-6
K_DET = 24
HIST = 4


def rsel(ip: np.ndarray, steps: int) -> np.ndarray:
    """walk_rsel (pmmg_vol.hpp): 0 up to kDetSteps, else a nonzero hash"""
    if steps <= K_DET:
        return np.zeros_like(ip, dtype=np.uint32)
    h = (ip.astype(np.uint32) * np.uint32(0x9E3779B1)) ^ np.uint32((steps * 0x85EBCA77) & 0xFFFFFFFF)
    h ^= h >> np.uint32(15)
    h = h * np.uint32(0x2C1B3C6D)
    h ^= h >> np.uint32(12)
    return h | np.uint32(0x80000000)


def tet_dots(x, p):
    """s[f] and vol as tet_dots (pmmg_device.hpp), vectorised: p (n, 4, 3)"""
    p0, p1, p2, p3 = p[:, 0], p[:, 1], p[:, 2], p[:, 3]
    vol = np.einsum("ij,ij->i", p1 - p0, np.cross(p2 - p0, p3 - p0))
    s = np.empty((x.shape[0], 4))
    for f, (a, b, c) in enumerate(((1, 2, 3), (0, 3, 2), (0, 1, 3), (0, 2, 1))):
        pa, pb, pc = p[:, a], p[:, b], p[:, c]
        n = np.cross(pb - pa, pc - pa)
        s[:, f] = np.einsum("ij,ij->i", x - pa, n)
    return s, vol


def walk(xyz, tetv, adja, x, ip, k0, maxstep, trace_n=0):
    n = x.shape[0]
    k = k0.copy()
    hist = np.zeros((n, HIST), np.int64)
    status = np.zeros(n, np.int8)  # 0 walking, 1 found, 2 stuck, 3 limit
    steps = np.zeros(n, np.int64)
    traces = [[] for _ in range(trace_n)]
    act = np.arange(n)
    for it in range(maxstep):
        if act.size == 0:
            break
        kk = k[act]
        tv = tetv[kk - 1]
        p = xyz[tv - 1]
        s, vol = tet_dots(x[act], p)
        steps[act] += 1
        with np.errstate(divide="ignore", invalid="ignore"):
            b = -s / vol[:, None]
        found = (vol != 0) & (b.min(1) > -EPS)
        key = np.where(vol[:, None] > 0, s, -s)
        key = np.where(vol[:, None] == 0, s, key)
        ad = adja[kk - 1] >> 2
        vis = (ad[:, :, None] == hist[act][:, None, :]).any(2)
        elig = (ad != 0) & ~vis
        # most negative eligible face (ties: lowest face)
        kk_ = np.where(elig, key, -np.inf)
        fdet = np.argmax(kk_, 1)
        fdet = np.where(elig.any(1), fdet, -1)
        f = fdet
        r = rsel(ip[act], it + 1)
        if it + 1 > K_DET:
            f0 = (r & 3).astype(np.int64)
            fst = np.full(act.size, -1)
            for j in range(3, -1, -1):  # first in cyclic order: scan backwards, keep the earliest
                ff = (f0 + j) & 3
                ok = elig[np.arange(act.size), ff] & (key[np.arange(act.size), ff] > 0)
                fst = np.where(ok, ff, fst)
            f = np.where(fst >= 0, fst, fdet)
        for t in range(min(trace_n, n)):
            w = np.nonzero(act == t)[0]
            if w.size:
                w = w[0]
                traces[t].append((int(kk[w]), float(b[w].min()), int(f[w]) if not found[w] else -9))
        status[act[found]] = 1
        stuck = ~found & (f < 0)
        status[act[stuck]] = 2
        mv = ~found & ~stuck
        am = act[mv]
        hist[am, 1:] = hist[am, :-1]
        hist[am, 0] = k[am]
        k[am] = adja[k[am] - 1, f[mv]] >> 2
        act = am
    status[act] = 3
    return status, steps, k, traces


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-old", type=int, default=134)
    ap.add_argument("--n-new", type=int, default=142)
    ap.add_argument("--jitter", type=float, default=0.2)
    ap.add_argument("--maxstep", type=int, default=1024)
    ap.add_argument("--trace", type=int, default=4)
    ap.add_argument("--out", default=None)
    ap.add_argument("--valid", action="store_true", help="jitter capped so that no tetra inverts (synth_vertices_valid)")
    a = ap.parse_args()
    t0 = time.time()
    bg = synth.lattice(synth.SHELL, a.n_new, jitter=a.jitter, seed=synth.SEED, with_trias=False, valid=a.valid)
    q = synth.lattice(synth.SHELL, a.n_old, jitter=0.0, with_tetra=False)
    pc = synth.classes(q)
    vol_ids = np.nonzero(pc == 1)[0]  # PMMG_PT_VOL
    x = q.xyz[vol_ids]
    print(f"bg {bg.ne} tets, {vol_ids.size} volume queries ({time.time() - t0:.1f}s)", flush=True)
    tv = bg.tetv.astype(np.int64)
    cen = bg.xyz[tv - 1].mean(1)
    vols = np.einsum("ij,ij->i", bg.xyz[tv[:, 1] - 1] - bg.xyz[tv[:, 0] - 1],
                     np.cross(bg.xyz[tv[:, 2] - 1] - bg.xyz[tv[:, 0] - 1], bg.xyz[tv[:, 3] - 1] - bg.xyz[tv[:, 0] - 1]))
    print(f"tetra volumes: min {vols.min():.3e} max {vols.max():.3e} nonpositive {(vols <= 0).sum()}", flush=True)
    from scipy.spatial import cKDTree

    tree = cKDTree(cen)
    _, near = tree.query(x, k=1, workers=8)
    k0 = near.astype(np.int64) + 1
    print(f"seeds ({time.time() - t0:.1f}s)", flush=True)
    status, steps, k, tr = walk(bg.xyz, tv, bg.adja.astype(np.int64), x, (vol_ids + 1).astype(np.int64), k0, a.maxstep)
    lim = np.nonzero(status == 3)[0]
    print(f"found {np.sum(status == 1)} stuck {np.sum(status == 2)} limit {lim.size}; steps mean "
          f"{steps.mean():.2f} max {steps.max()} ({time.time() - t0:.1f}s)", flush=True)
    if lim.size:
        r = np.linalg.norm(x[lim], axis=1)
        rinf = np.abs(x[lim]).max(1)
        print("limit walks: |x| quantiles", np.quantile(r, [0, .5, 1]), "ninf", np.quantile(rinf, [0, .5, 1]))
        sub = lim[: a.trace]
        st2, _, _, tr = walk(bg.xyz, tv, bg.adja.astype(np.int64), x[sub], (vol_ids[sub] + 1).astype(np.int64),
                             k0[sub], 64, trace_n=len(sub))
        for j, t in enumerate(tr):
            print(f"query {vol_ids[sub[j]] + 1} x={x[sub[j]]} seed {k0[sub[j]]}:")
            print("   ", " ".join(f"{kk}:{mb:.2e}/{f}" for kk, mb, f in t[:40]))
    if a.out:
        np.savez(a.out, vol_ids=vol_ids, status=status, steps=steps, k0=k0)


if __name__ == "__main__":
    main()
