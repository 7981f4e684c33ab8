"""Synthetic test-image generators (utils/test_images.py:6-178 of the reference).

Vectorised restatements producing byte-identical images (pinned against the
reference's own outputs in tests/test_host_utils_cpu.py).
"""

from typing import Optional

import numpy as np


def generate_colored_checkerboard(size: int = 512) -> np.ndarray:
    """High-contrast 32-px checkerboard, values 30 / 220 (test_images.py:6-19)."""
    cell = np.arange(size) // 32
    dark = ((cell[:, None] + cell[None, :]) % 2) == 0
    img = np.where(dark, np.uint8(30), np.uint8(220)).astype(np.uint8)
    return np.repeat(img[:, :, None], 3, axis=2)


def generate_thin_stripes(size: int = 512, stripe_width: int = 4) -> np.ndarray:
    """Vertical stripes alternating two colours (test_images.py:22-32)."""
    even = ((np.arange(size) // stripe_width) % 2) == 0
    row = np.where(even[:, None], np.array([200, 60, 60], np.uint8), np.array([60, 180, 200], np.uint8))
    return np.ascontiguousarray(np.broadcast_to(row[None], (size, size, 3))).astype(np.uint8)


def generate_gradient(size: int = 512) -> np.ndarray:
    """Diagonal gradient (test_images.py:35-48): float32 image, clip, truncate."""
    idx = np.arange(size)
    t = (idx[:, None] + idx[None, :]) / (2 * size - 2)
    img = np.stack([40 + t * 180, 60 + t * 140, 120 + t * 100], axis=-1).astype(np.float32)
    return np.clip(img, 0, 255).astype(np.uint8)


def generate_text_edges(size: int = 512) -> np.ndarray:
    """Bars and a diagonal on a light background (test_images.py:51-77)."""
    img = np.ones((size, size, 3), dtype=np.uint8) * 245
    margin = size // 10
    bar_height = size // 16
    y = margin
    for thickness in [bar_height, bar_height // 2, bar_height // 4, 2]:
        img[y:y + thickness, margin:size - margin] = [25, 25, 25]
        y += thickness + margin // 2
    x = margin
    for thickness in [bar_height, bar_height // 2, bar_height // 4, 2]:
        img[size // 2 + margin:size - margin, x:x + thickness] = [25, 25, 25]
        x += thickness + margin // 2
    for i in range(size // 4):
        y_pos = size // 2 + margin + i
        x_pos = size // 2 + i
        if y_pos < size - margin and x_pos < size - margin:
            img[y_pos:y_pos + 3, x_pos:x_pos + 3] = [25, 25, 25]
    return img


def generate_chroma_stripes(size: int = 512) -> np.ndarray:
    """Eight saturated vertical colour bars (test_images.py:80-102)."""
    colors = [[180, 40, 40], [40, 160, 40], [40, 80, 180], [180, 180, 40],
              [180, 40, 180], [40, 180, 180], [200, 120, 40], [120, 40, 180]]
    img = np.zeros((size, size, 3), dtype=np.uint8)
    w = size // len(colors)
    for i, c in enumerate(colors):
        img[:, i * w:((i + 1) * w if i < len(colors) - 1 else size)] = c
    return img


def generate_photo(size: int = 512) -> np.ndarray:
    """Sky / mountains / textured ground / sun (test_images.py:105-162).

    Uses the legacy global NumPy RNG seeded with 123 exactly like the
    reference (draw order preserved: 4 phases, then one draw per ground pixel
    in raster order)."""
    img = np.zeros((size, size, 3), dtype=np.float32)
    horizon = int(size * 0.45)
    mountain_base = int(size * 0.55)
    t = np.arange(horizon) / horizon
    img[:horizon, :] = np.stack([180 - t * 60, 210 - t * 80, 240 - t * 40], -1)[:, None, :]
    np.random.seed(123)
    heights = np.zeros(size)
    for freq in [8, 16, 32, 64]:
        phase = np.random.rand() * 2 * np.pi
        amplitude = (size * 0.15) / (freq / 8)
        heights += amplitude * np.sin(np.linspace(0, freq * np.pi, size) + phase)
    heights = heights - heights.min()
    heights = heights / heights.max() * (mountain_base - horizon - 20)
    for j in range(size):
        peak = int(horizon + 20 + heights[j])
        rows = np.arange(horizon, mountain_base)
        above = rows < peak
        depth = (rows[above] - horizon) / (peak - horizon)
        img[rows[above], j] = np.stack([70 + depth * 30, 80 + depth * 20, 100 + depth * 10], -1)
        img[rows[~above], j] = [90, 95, 85]
    n_ground = size - mountain_base
    noise = (np.random.rand(n_ground * size) * 15 - 7.5).reshape(n_ground, size)
    tg = ((np.arange(mountain_base, size) - mountain_base) / (size - mountain_base))[:, None]
    img[mountain_base:, :] = np.stack([60 + tg * 40 + noise, 100 + tg * 30 + noise, 50 + tg * 20 + noise], -1)
    sun_x, sun_y = size // 4, size // 6
    r = size // 10
    for i in range(max(0, sun_y - r * 2), min(horizon, sun_y + r * 2)):
        for j in range(max(0, sun_x - r * 2), min(size, sun_x + r * 2)):
            dist = np.sqrt((i - sun_y) ** 2 + (j - sun_x) ** 2)
            if dist < r * 1.5:
                glow = max(0, 1 - (dist / (r * 1.5)) ** 2)
                img[i, j] = img[i, j] * (1 - glow * 0.7) + np.array([255, 240, 200]) * glow * 0.7
    return np.clip(img, 0, 255).astype(np.uint8)


def generate_demo_image(key: str) -> Optional[np.ndarray]:
    """Demo image by key (test_images.py:165-178)."""
    generators = {
        "photo": lambda: generate_photo(512),
        "text_edges": lambda: generate_text_edges(512),
        "gradient": lambda: generate_gradient(512),
        "checkerboard": lambda: generate_colored_checkerboard(512),
        "chroma_stripes": lambda: generate_chroma_stripes(512),
    }
    if key in generators:
        return generators[key]()
    return None
