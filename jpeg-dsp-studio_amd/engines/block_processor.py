"""Block processing: padding, splitting, merging (engines/block_processor.py:1-48).

Pure data movement (no arithmetic), kept on the host like the reference; the
fused GPU path does this addressing inside its kernels."""

from typing import List, Tuple

import numpy as np


def pad_to_multiple(channel: np.ndarray, block_size: int) -> Tuple[np.ndarray, Tuple[int, int]]:
    """Pad channel to multiple of block_size using reflect mode (bottom/right)."""
    h, w = channel.shape
    pad_h = (block_size - h % block_size) % block_size
    pad_w = (block_size - w % block_size) % block_size
    if pad_h > 0 or pad_w > 0:
        return np.pad(channel, ((0, pad_h), (0, pad_w)), mode='reflect'), (h, w)
    return channel.copy(), (h, w)


def split_into_blocks(channel: np.ndarray, block_size: int) -> List[Tuple[int, int, np.ndarray]]:
    """Split a 2D channel into BxB blocks, raster order; partial blocks zero-filled."""
    h, w = channel.shape
    blocks = []
    for i in range(0, h, block_size):
        for j in range(0, w, block_size):
            block = channel[i:i + block_size, j:j + block_size]
            if block.shape != (block_size, block_size):
                full = np.zeros((block_size, block_size), dtype=channel.dtype)
                full[:block.shape[0], :block.shape[1]] = block
                block = full
            blocks.append((i, j, block.copy()))
    return blocks


def merge_blocks(blocks: List[Tuple[int, int, np.ndarray]], shape: Tuple[int, int], block_size: int) -> np.ndarray:
    """Merge blocks back into a float64 2D channel of the given shape."""
    h, w = shape
    result = np.zeros((h, w), dtype=np.float64)
    for (i, j, block) in blocks:
        bh = min(i + block_size, h) - i
        bw = min(j + block_size, w) - j
        result[i:i + bh, j:j + bw] = block[:bh, :bw]
    return result
