"""Nested-structure helpers used by the learner (cf. handyrl/util.py:7-29)."""


def map_r(x, fn):
    """Apply ``fn`` to every leaf of nested lists / tuples / dicts."""
    if isinstance(x, (list, tuple)):
        return type(x)(map_r(v, fn) for v in x)
    if isinstance(x, dict):
        return type(x)((k, map_r(v, fn)) for k, v in x.items())
    return fn(x)


def bimap_r(x, y, fn):
    """Apply ``fn(leaf_x, leaf_y)`` over two structures shaped like ``x``."""
    if isinstance(x, (list, tuple)):
        return type(x)(bimap_r(v, y[i], fn) for i, v in enumerate(x))
    if isinstance(x, dict):
        return type(x)((k, bimap_r(v, y[k], fn)) for k, v in x.items())
    return fn(x, y)


def trimap_r(x, y, z, fn):
    if isinstance(x, (list, tuple)):
        return type(x)(trimap_r(v, y[i], z[i], fn) for i, v in enumerate(x))
    if isinstance(x, dict):
        return type(x)((k, trimap_r(v, y[k], z[k], fn)) for k, v in x.items())
    return fn(x, y, z)
