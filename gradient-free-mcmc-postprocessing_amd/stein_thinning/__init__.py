"""MI355X-native Stein thinning (drop-in for the reference's ``stein_thinning`` dependency).

Public surface used by aglebov/gradient-free-mcmc-postprocessing:
``stein_thinning.thinning.{thin, thin_gf, _greedy_search, _validate_and_standardize,
_make_stein_integrand, _make_stein_gf_integrand}``, ``stein_thinning.stein.{ksd, kmat}``,
``stein_thinning.kernel.{vfk0_imq, make_imq, make_precon}``.  Multi-GPU (one process per GPU,
RCCL): ``stein_thinning.distributed``.  Importing this package touches no GPU.
"""
from ._native import set_arithmetic  # noqa: F401
from .thinning import set_dedup, set_rank_sharding, thin, thin_chains, thin_gf, thin_gf_chains  # noqa: F401

__version__ = '0.1.0'
