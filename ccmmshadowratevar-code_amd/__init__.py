"""MI355X-native Gibbs sweep of the CCMM shadow-rate BVAR-SV.

Import name: ``ccmm_amd`` (the directory name contains a hyphen; use
``__graft_entry__.load_package()`` or ``tests/conftest.py``'s loader, which
register this directory as the package ``ccmm_amd``).

Layers:
  csrc/            HIP kernels (gfx950) + C ABI -> libccmm.so  (include/ccmm.h)
  _abi.py          ctypes binding of the C ABI
  model.py         host setup of one vintage (mcmcVAR.m:28-206,
                   mcmcVARshadowrateBlockHybrid.m:30-295)
  samplers.py      reference-interface mirror (mcmcVAR, mcmcVARshadowrateBlockHybrid,
                   CTA, CTAsys, drawTruncNormal)
  distributed.py   vintage/chain sharding over GPUs, end-of-run reductions
"""
from . import _abi, distributed, model, samplers, synthetic  # noqa: F401
from ._abi import (MODEL_BLOCKHYBRID, MODEL_HYBRID, MODEL_LINEAR, MODEL_SHADOWRATE, Chains,  # noqa: F401
                   Context, load_library)
from .samplers import (CTA, CTAsys, drawTruncNormal, mcmcVAR,  # noqa: F401
                       mcmcVARshadowrateBlockHybrid)
