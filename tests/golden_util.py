"""Loader for the committed golden fixtures (tests/golden/, made by make_golden.py)."""
import functools
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


@functools.lru_cache(None)
def golden():
    return json.load(open(os.path.join(GOLDEN, 'golden.json')))['cases']


@functools.lru_cache(None)
def arrays():
    with np.load(os.path.join(GOLDEN, 'arrays.npz'), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def case_input(name):
    """Regenerate (or load) the input image of a golden case and check its digest."""
    from oracle import cpu_ref
    g = golden()[name]
    h, w, _ = g['shape']
    key = f'{name}/input'
    a = arrays()
    if key in a:
        img = a[key]
    elif name.startswith('cfg1_checker'):
        img = cpu_ref.generate_colored_checkerboard(h)
    else:
        seed = int(name.split('_s')[1].split('_')[0])
        img = cpu_ref.random_image(h, w, seed)
    assert sha(img) == g['sha_input'], name
    return img


def case_params(name):
    g = golden()[name]
    return dict(quality=g['quality'], mode=g['mode'], prefilter=g['prefilter'],
                selected_block_idx=tuple(g['selected_block_idx']))
