"""Synthetic images for the front-end tests: a random texture rendered from a
continuous function (cubic interpolation of a coarse random grid), so that a
sub-pixel motion of the scene is known exactly (no resampling of a discrete
image)."""
import numpy as np
from scipy.ndimage import map_coordinates


def texture_fn(seed=0, W=752, H=480, cell=5.0, contrast=110.0):
    rng = np.random.default_rng(seed)
    gh, gw = int(H / cell) + 8, int(W / cell) + 8
    G = 128.0 + contrast * (rng.random((gh, gw)) - 0.5) * 2

    def f(x, y):
        return map_coordinates(G, [np.asarray(y) / cell + 4, np.asarray(x) / cell + 4], order=3, mode="reflect")
    return f


def render(f, W, H, dx=0.0, dy=0.0):
    """Image of the scene moved by (dx, dy) pixels: I(x, y) = f(x - dx, y - dy)."""
    yy, xx = np.mgrid[0:H, 0:W].astype(float)
    return np.clip(np.rint(f(xx - dx, yy - dy)), 0, 255).astype(np.uint8)


def squares(W=160, H=120, lo=40, hi=210):
    """Dark background with bright axis-aligned squares."""
    img = np.full((H, W), lo, np.uint8)
    boxes = [(20, 20, 40, 40), (80, 30, 110, 55), (30, 70, 60, 100)]
    for x0, y0, x1, y1 in boxes:
        img[y0:y1, x0:x1] = hi
    return img, boxes
