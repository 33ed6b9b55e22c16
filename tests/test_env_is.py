"""Env importance sampling (the build's opt-in re-derivation,
TPT_FLAG_ENV_IS): the oracle's sampler is an unbiased estimator of the
cosine-weighted env integral -- E[Le*cos/(pi*pdf)] equals the brute-force sum
over texels -- and it concentrates samples where the env is bright."""
import numpy as np

import tinypathtracer_amd as T
from oracle import oracle as O


def _brute_force(rgba_bu, nf):
    """Integral of Le(w) cos+(n, w) / pi over the sphere, texel by texel
    (centre direction, solid angle 2 pi^2 sin(theta) / (W H))."""
    h, w = rgba_bu.shape[:2]
    iy, ix = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    v = (iy + 0.5) / h
    u = (ix + 0.5) / w
    theta = np.pi * (1.0 - v)
    phi = 2.0 * np.pi * u
    d = np.stack([np.sin(theta) * np.cos(phi), np.cos(theta), np.sin(theta) * np.sin(phi)], -1)
    c = np.clip(d @ np.asarray(nf, np.float64), 0.0, None)
    dw = 2.0 * np.pi ** 2 * np.sin(theta) / (w * h)
    le = rgba_bu[..., :3].astype(np.float64) / 255.0
    return (le * (c * dw / np.pi)[..., None]).sum(axis=(0, 1))


def test_env_is_unbiased_on_sky():
    sky = T.procedural_sky(256, 128)[::-1]            # stored bottom-up like the env texture
    for nf in ([0.0, 1.0, 0.0], [0.6, 0.0, 0.8], [0.0, -1.0, 0.0]):
        _, k = O.env_is_samples(sky, nf, 200000, seed=3)
        est = k.astype(np.float64).mean(0)
        ref = _brute_force(sky, nf)
        assert np.allclose(est, ref, rtol=0.03, atol=2e-3), (nf, est, ref)


def test_env_is_follows_brightness():
    h, w = 64, 128
    env = np.full((h, w, 4), 10, np.uint8)
    env[40:44, 90:96, :3] = 250                      # a bright patch (bottom-up rows 40-43)
    env[..., 3] = 255
    d, k = O.env_is_samples(env, [0.0, 1.0, 0.0], 20000, seed=5)
    u = (np.arctan2(d[:, 2], d[:, 0]) / (2 * np.pi)) % 1.0
    v = 1.0 - np.arccos(np.clip(d[:, 1], -1, 1)) / np.pi
    inpatch = ((v * h >= 40) & (v * h < 44) & (u * w >= 90) & (u * w < 96)).mean()
    # expected share: the patch's weight (luma * sin(theta at the row centre)) over the total
    luma = (0.2126 * env[..., 0] + 0.7152 * env[..., 1] + 0.0722 * env[..., 2]).astype(np.float64)
    sinr = np.sin(np.pi * (1.0 - (np.arange(h) + 0.5) / h))[:, None]
    wt = luma * sinr
    share = wt[40:44, 90:96].sum() / wt.sum()
    assert abs(inpatch - share) < 0.01, (inpatch, share)
    assert share > 20 * (24 / (h * w))               # far above the patch's share of texels
    est = k.astype(np.float64).mean(0)
    assert np.allclose(est, _brute_force(env, [0.0, 1.0, 0.0]), rtol=0.05, atol=2e-3)


def _block(w, h):
    """The IS block side (api.cpp env_is_block, oracle env_is_block)."""
    b = 1
    while ((w + b - 1) // b) * ((h + b - 1) // b) > (1 << 17):
        b *= 2
    return b


def test_env_is_block_tables_unbiased_and_follow_brightness():
    """Maps above 2^17 texels sample blocks of B x B texels (here 1024 x 512 ->
    B = 2, a patch straddling block edges): still unbiased, and the share of
    samples inside a bright patch is the blocks' probabilities times the
    patch's share of each block's area (uniform inside a block)."""
    h, w = 512, 1024
    b = _block(w, h)
    assert b == 2
    sky = T.procedural_sky(w, h)[::-1].copy()
    for nf in ([0.0, 1.0, 0.0], [0.6, 0.0, 0.8]):
        _, k = O.env_is_samples(sky, nf, 200000, seed=11)
        est = k.astype(np.float64).mean(0)
        assert np.allclose(est, _brute_force(sky, nf), rtol=0.03, atol=2e-3), (nf, est)
    env = np.full((h, w, 4), 10, np.uint8)
    y0, y1, x0, x1 = 301, 310, 601, 618            # odd edges: partial blocks on every side
    env[y0:y1, x0:x1, :3] = 250
    env[..., 3] = 255
    d, _ = O.env_is_samples(env, [0.0, 1.0, 0.0], 40000, seed=5)
    u = (np.arctan2(d[:, 2], d[:, 0]) / (2 * np.pi)) % 1.0
    v = 1.0 - np.arccos(np.clip(d[:, 1], -1, 1)) / np.pi
    inpatch = ((v * h >= y0) & (v * h < y1) & (u * w >= x0) & (u * w < x1)).mean()
    luma = (0.2126 * env[..., 0] + 0.7152 * env[..., 1] + 0.0722 * env[..., 2]).astype(np.float64)
    wt = luma * np.sin(np.pi * (1.0 - (np.arange(h) + 0.5) / h))[:, None]
    bw_ = wt.reshape(h // b, b, w // b, b).sum(axis=(1, 3))
    inside = np.zeros((h, w))
    inside[y0:y1, x0:x1] = 1.0
    frac = inside.reshape(h // b, b, w // b, b).mean(axis=(1, 3))
    expect = (bw_ * frac).sum() / bw_.sum()
    assert abs(inpatch - expect) < 0.01, (inpatch, expect)
