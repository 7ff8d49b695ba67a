"""Drop-in replacement of afiliot/Kernel-Methods-For-Genomics ``KRR.py``: ``from KRR import
KRR`` (utils.py:11) gets the same class, with the n x n solve of ``fit`` (KRR.py:33) done on
the MI355X by libkmgram (kmgram/learners.py)."""
from kmgram.learners import KRR

__all__ = ["KRR"]
