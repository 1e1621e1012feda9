"""Autograd for fft_admm_tv (unrolled-iteration adjoint).  Not implemented yet."""
from __future__ import annotations


def fft_admm_tv_autograd(xin, lmbd, rho, kern, iso, maxit):
    raise NotImplementedError("admmtor (MI355X build): backward of fft_admm_tv is not implemented yet")
