"""admmtor -- MI355X (gfx950) build of the ADMM-TV deconvolution hot path of
georgegrosu1/torch-admm-deconv.

Public surface (same import paths as the reference):
  admmtor.eops.deconv.fft_admm_tv           (reference: src/admmtor/eops/deconv.py:35)
  admmtor.elayers.admmdeconv.ADMMDeconv     (reference: src/admmtor/elayers/admmdeconv.py:6)
The solver runs as hand-written HIP kernels through the C ABI in include/admm_tv.h.
"""
__version__ = "0.1.0"
