"""Kernel-combination consumers of the Gram matrices, on the device.

The reference combines its Grams on the host with numpy temporaries of p x n x n float64:
  NLCK.svm_step / NLCK.get_K   (NLCKernels.py:52, 97)  K = (sum_m u_m K_m) ** degree
  NLCK.grad                    (NLCKernels.py:61-66)   -degree * [alpha^T (K_t o K_m) alpha]_m
  ALIGNF.get_a / ALIGNF.get_M  (ALIGNF.py:43-58)       alignment of the centred kernels
These functions compute the same quantities with one fused HIP kernel each
(csrc/kmg_combine.hip), so a maintainer can replace those three numpy expressions by one
call each.  No CPU fallback: they raise without the library or a GPU.
"""
import numpy as np

from .engine import default_engine


def _ctx():
    return default_engine().ctx


def nlck_combine(kernels, u, degree):
    """np.sum(kernels * u[:, None, None], axis=0) ** degree (NLCKernels.py:52, 97).
    Bit-exact for degree 1 and 2 (same fp64 operation order); pow() for higher degrees."""
    return _ctx().combine(kernels, np.asarray(u, dtype=np.float64), int(degree))


def nlck_grad(kernels_fit, u, degree, alpha):
    """NLCK.grad (NLCKernels.py:61-66): -degree * [alpha^T (K_t * K_m) alpha for each m],
    K_t = (sum_m u_m K_m) ** (degree - 1).  fp64; the reduction order differs from BLAS."""
    return _ctx().nlck_grad(kernels_fit, np.asarray(u, dtype=np.float64), int(degree),
                            np.asarray(alpha, dtype=np.float64))


def alignf_stats(kernels_fit, y):
    """(a, M) of ALIGNF (ALIGNF.py:43-58): a_m = sum(center_K(K_m) * outer(y, y)),
    M_lm = sum(center_K(K_l) * center_K(K_m)); centring as in center_K (kernels.py:387-395)
    done in O(n^2) per matrix instead of the reference's O(n^3) multi_dot."""
    return _ctx().alignf(kernels_fit, np.asarray(y, dtype=np.float64))
