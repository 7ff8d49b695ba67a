"""Drop-in replacement of afiliot/Kernel-Methods-For-Genomics ``SVM.py``: ``from SVM import
C_SVM`` (run.py:3, utils.py:9) gets the same class, with the QP of ``fit`` (SVM.py:78-89,
cvxopt in the reference) solved on the MI355X by libkmgram (kmgram/learners.py)."""
from kmgram.learners import C_SVM

__all__ = ["C_SVM"]
