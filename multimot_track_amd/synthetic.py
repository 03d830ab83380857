"""Seeded synthetic RGB-D inputs for tests and bench (band-limited value noise
with 8-bit contrast >= 40 so FAST fires in every cell).  Host-side data generation only."""
import numpy as np


def value_noise(h, w, seed, octaves=(8, 16, 32, 64), contrast=200):
    rng = np.random.default_rng(seed)
    acc = np.zeros((h, w), np.float64)
    amp = 1.0
    for cell in octaves:
        gh, gw = h // cell + 2, w // cell + 2
        grid = rng.random((gh, gw))
        ys = np.arange(h) / cell
        xs = np.arange(w) / cell
        y0 = ys.astype(int)
        x0 = xs.astype(int)
        fy = (ys - y0)[:, None]
        fx = (xs - x0)[None, :]
        fy = fy * fy * (3 - 2 * fy)
        fx = fx * fx * (3 - 2 * fx)
        g00 = grid[y0][:, x0]
        g01 = grid[y0][:, x0 + 1]
        g10 = grid[y0 + 1][:, x0]
        g11 = grid[y0 + 1][:, x0 + 1]
        acc += amp * ((g00 * (1 - fx) + g01 * fx) * (1 - fy) + (g10 * (1 - fx) + g11 * fx) * fy)
        amp *= 0.6
    acc -= acc.min()
    acc /= max(acc.max(), 1e-9)
    img = 28 + contrast * acc + rng.normal(0, 6, (h, w))
    return np.clip(img, 0, 255).astype(np.uint8)


def gray_frame(h, w, seed):
    return value_noise(h, w, seed)


def bgr_frame(h, w, seed):
    g = value_noise(h, w, seed).astype(np.int32)
    rng = np.random.default_rng(seed + 7)
    tint = rng.integers(-12, 12, 3)
    return np.clip(g[:, :, None] + tint[None, None, :], 0, 255).astype(np.uint8)
