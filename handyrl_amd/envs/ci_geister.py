"""CIGeister: Geister with complete information (handyrl/envs/ci_geister.py).

The reference module is geister.py with one change in the observation
(ci_geister.py:520-568): the opponent's blue/red planes are shown in every
view, not only in ``observation(None)``.  Same rules, actions and net.
"""

from .geister import GeisterBatch, GeisterNet, Environment as _Geister  # noqa: F401


class CIGeisterBatch(GeisterBatch):
    COMPLETE_INFO = True


class Environment(_Geister):
    BATCH = CIGeisterBatch
