"""Deterministic synthetic video content for tests and bench.py (no datasets
are available offline).  SURVEY.md section 8(d): a smooth moving gradient plus
texture plus N(0, 2% of max) noise, seed 1234; the "prediction" for the
residual is the same content displaced by a known motion vector."""
import numpy as np


def frame(width, height, bit_depth=8, seed=1234, t=0):
    """One luma plane (uint8 for 8-bit, uint16 otherwise)."""
    rng = np.random.RandomState(seed + 7919 * t)
    maxv = (1 << bit_depth) - 1
    y, x = np.mgrid[0:height, 0:width].astype(np.float32)
    base = 0.45 + 0.25 * np.sin((x + 3.0 * t) / 97.0) * np.cos((y - 2.0 * t) / 71.0)
    tex = 0.12 * np.sin((x * 0.9 + y * 0.4) / 5.3) * np.sin((y * 1.1 - x * 0.3) / 7.9)
    img = (base + tex) * maxv + rng.normal(0.0, 0.02 * maxv, size=(height, width))
    img = np.clip(np.rint(img), 0, maxv)
    return img.astype(np.uint8 if bit_depth == 8 else np.uint16)


def shifted(img, dx, dy):
    """img displaced by (dx, dy) with edge replication."""
    h, w = img.shape
    ys = np.clip(np.arange(h) - dy, 0, h - 1)
    xs = np.clip(np.arange(w) - dx, 0, w - 1)
    return np.ascontiguousarray(img[ys][:, xs])


def residual_plane(width, height, bit_depth=8, seed=1234, mv=(3, -2)):
    """int16 residual = src - pred, pred = src displaced by mv (C2 input)."""
    src = frame(width, height, bit_depth, seed)
    pred = shifted(frame(width, height, bit_depth, seed), *mv)
    return src.astype(np.int16) - pred.astype(np.int16)


def pad_plane(img, border):
    """aom_extend_frame_borders-style edge replication by `border` pixels."""
    return np.pad(img, border, mode="edge")


def motion_planes(width, height, nrefs, border=160, seed=1234):
    """C3 input: the current frame and `nrefs` references,
    ref_k = the current content displaced by (3k, -2k) with fresh noise, all
    padded by `border` pixels.  Returns (src[Hp, Wp], refs[nrefs, Hp, Wp])."""
    src = pad_plane(frame(width, height, 8, seed), border)
    refs = np.stack([pad_plane(shifted(frame(width, height, 8, seed + 101 * k), 3 * k, -2 * k),
                               border) for k in range(1, nrefs + 1)])
    return np.ascontiguousarray(src), np.ascontiguousarray(refs)


def tpl_motion_planes(width, height, nrefs, border, seed):
    """TPL motion-search input: the current frame and nrefs references whose
    content moves by a different large displacement (up to +-28 pixels) in
    each quadrant, with fresh +-3 noise -- beyond a zero-start FAST_BIGDIA's
    reach, so the neighbour-seeded start mvs (tpl_model.c:640-735) decide
    the result.  Returns (src[Hp, Wp], refs[nrefs, Hp, Wp]), padded."""
    rng = np.random.default_rng(seed)
    src = frame(width, height, 8, seed)
    refs = []
    for _ in range(nrefs):
        ref = np.empty_like(src)
        for qy in range(2):
            for qx in range(2):
                dx, dy = (int(v) for v in rng.integers(-28, 29, size=2))
                sh = shifted(src, dx, dy).astype(np.int16)
                sh = np.clip(sh + rng.integers(-3, 4, size=sh.shape), 0, 255).astype(np.uint8)
                ys = slice(qy * height // 2, (qy + 1) * height // 2)
                xs = slice(qx * width // 2, (qx + 1) * width // 2)
                ref[ys, xs] = sh[ys, xs]
        refs.append(pad_plane(ref, border))
    return np.ascontiguousarray(pad_plane(src, border)), np.ascontiguousarray(np.stack(refs))
