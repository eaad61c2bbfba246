"""nemo -- MI355X-native order-score engine for Nested Effects Model order MCMC.

Drop-in for the hot path of MrGreyPanda/NEM-MCMC-optimization: the reference's
``NEM`` model, ``utils`` helpers and ``NEMOrderMCMC`` sampler keep their
Python API here, while the per-step order-score evaluation and the per-pair
local optimisation run as hand-written HIP kernels for gfx950 behind the C-ABI
of ``include/nemo.h`` (``libnemo.so``, loaded with ctypes).
"""
from . import generator, utils
from .nem import NEM

__all__ = ["NEM", "generator", "utils", "Engine", "NEMOrderMCMC", "ExactArithmeticWarning"]


def __getattr__(name):
    # the GPU-facing pieces load libnemo lazily
    if name == "Engine":
        from .engine import Engine
        return Engine
    if name == "ExactArithmeticWarning":
        from .engine import ExactArithmeticWarning
        return ExactArithmeticWarning
    if name == "NEMOrderMCMC":
        from .nem_order_mcmc import NEMOrderMCMC
        return NEMOrderMCMC
    raise AttributeError(name)
