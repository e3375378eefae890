"""Seeded synthetic frames of the BASELINE.json configs.

There is no network for video data, so bench.py, the tests and the scripts
all build their frames here: S-smooth RGB (sinusoids plus noise, natural-like
after the DCT), the C4 sequence (shifted copies of four S-smooth 1080p frames)
and the C5 sequence (a panning window of one larger picture).  Pure numpy; no
device work.
"""
from __future__ import annotations

import numpy as np


def synth_frame(H: int, W: int, seed: int) -> np.ndarray:
    """S-smooth of SURVEY.md §8(d): natural-like synthetic RGB (seeded)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    y = np.arange(H, dtype=np.float32)[:, None]
    x = np.arange(W, dtype=np.float32)[None, :]
    chans = []
    for c in range(3):
        v = 128 + 60 * np.sin(x / 97 + c + seed) + 50 * np.cos(y / 61 - c - seed)
        v = v + rng.normal(0, 4, (H, W)).astype(np.float32)
        chans.append(v)
    return np.clip(np.rint(np.stack(chans, -1)), 0, 255).astype(np.uint8)


def c4_frame(bases, i: int) -> np.ndarray:
    """Frame i of the C4 sequence: one of four S-smooth 1080p frames, shifted
    by a frame-dependent constant (u8 wrap), so every frame's code-stream
    differs and any rank can regenerate any frame cheaply."""
    return bases[i % len(bases)] + np.uint8((i // len(bases)) * 7 % 256)


def c5_frame(base, i: int, H: int, W: int) -> np.ndarray:
    """Frame i of the C5 sequence: a window of a larger S-smooth picture panning
    by (2i mod 41, 3i mod 53) pixels, so the motion search finds real vectors."""
    dy, dx = (2 * i) % 41, (3 * i) % 53
    return np.ascontiguousarray(base[dy:dy + H, dx:dx + W])
