"""ddr_amd -- MI355X-native differentiable Muskingum-Cunge routing (the hot path of taddyb/ddr).

Public surface mirrors the reference's routing API (``ddr.dmc``, ``ddr.routing.*``) on top of the HIP
library ``ddr_amd/lib/libddr_mc.so`` (C ABI: ``include/ddr_mc.h``).
"""

__version__ = "0.1.0"


def __getattr__(name):
    # lazy: importing the package must not require the HIP library (CPU-only tooling, tests)
    if name == "dmc":
        from .routing.torch_mc import dmc

        return dmc
    if name == "MuskingumCunge":
        from .routing.mmc import MuskingumCunge

        return MuskingumCunge
    raise AttributeError(name)
