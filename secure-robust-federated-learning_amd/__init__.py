"""MI355X-native Byzantine-robust gradient-reduction engine.

Drop-in for the aggregation path of wanglun1996/secure-robust-federated-learning
(src/robust_estimator.py behind src/simulate.py's ``--agg`` dispatch):

* ``robust_estimator`` — the reference's module API (same names, signatures
  and return types), backed by hand-written gfx950 HIP kernels;
* ``engine``           — device-resident N x d fp32 API used by the above and by
  the bench;
* ``_lib``             — ctypes binding of libsra.so (include/sra.h).

Import as ``srfl_amd`` via ``srfl_loader.load()`` (the directory name is not a
Python identifier).
"""
__version__ = "0.1.0"

from . import _lib  # noqa: F401
