"""admmtor -- MI355X (gfx950) build of the ADMM-TV deconvolution hot path of
georgegrosu1/torch-admm-deconv.

Public surface (same import paths as the reference):
  admmtor.eops.deconv.fft_admm_tv           (reference: src/admmtor/eops/deconv.py:35)
  admmtor.elayers.admmdeconv.ADMMDeconv     (reference: src/admmtor/elayers/admmdeconv.py:6)
The solver runs as hand-written HIP kernels through the C ABI in include/admm_tv.h.
"""
__version__ = "0.1.0"

# Overlay: when the reference tree is also on sys.path (after this package), its modules that
# this build does not provide (training loop, metrics, data loading, other models) stay
# importable under the same package name; modules present here take precedence.
__path__ = __import__("pkgutil").extend_path(__path__, __name__)
