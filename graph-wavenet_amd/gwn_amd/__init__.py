"""gwn_amd — MI355X-native Graph WaveNet hot path (gwnet forward/backward + trainer step).

Public surface mirrors the reference (sklin93/Graph-WaveNet): ``gwn_amd.model.gwnet``,
``gwn_amd.engine.trainer``, ``gwn_amd.util``.  Compute runs in libgwn.so (HIP, gfx950).
"""
from . import synthetic  # noqa: F401  (numpy only)

__version__ = "0.1.0"


def lib():
    from . import _lib
    return _lib.load()
