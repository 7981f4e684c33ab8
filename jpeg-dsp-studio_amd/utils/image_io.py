"""Image file I/O (utils/image_io.py:7-17 of the reference) — caller-side, out of the
hot path.  Needs opencv-python, which this image does not ship; imported lazily."""

import numpy as np


def load_image(path: str) -> np.ndarray:
    import cv2
    img = cv2.imread(path, cv2.IMREAD_COLOR)
    if img is None:
        raise ValueError(f"Could not load image: {path}")
    return cv2.cvtColor(img, cv2.COLOR_BGR2RGB)


def save_image(image: np.ndarray, path: str) -> None:
    import cv2
    cv2.imwrite(path, cv2.cvtColor(image, cv2.COLOR_RGB2BGR))
