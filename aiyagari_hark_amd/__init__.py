"""aiyagari_hark_amd -- MI355X-native (gfx950) Aiyagari household block.

Drop-in for the hot path of Dostenlinus/Aiyagari-HARK (EGM backward step ->
panel / histogram cross-section -> GE loop).  Compute runs in hand-written HIP
kernels (``csrc/``, built into ``lib/libaiyagari.so`` and called through the C ABI
``include/aiyagari.h``); PyTorch-ROCm only owns device buffers and streams.

The reference's call surface lives in :mod:`aiyagari_hark_amd.model`
(``AiyagariType``, ``AiyagariEconomy``); the batched stationary extensions (GE
bisection on r, Young-lottery histogram, Rouwenhorst) in
:mod:`aiyagari_hark_amd.stationary`.
"""
from __future__ import annotations

__version__ = "0.1.0"


def __getattr__(name):
    # Lazy: importing the package must not require a GPU (the C ABI loads on first use).
    if name in ("AiyagariType", "AiyagariEconomy", "AggregateSavingRule", "AggShocksDynamicRule",
                "init_Aiyagari_agents", "init_Aiyagari_economy"):
        from . import model
        return getattr(model, name)
    raise AttributeError(name)
