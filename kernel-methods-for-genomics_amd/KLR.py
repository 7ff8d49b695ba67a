"""Drop-in replacement of afiliot/Kernel-Methods-For-Genomics ``KLR.py``: ``from KLR import
KLR`` (utils.py:10) gets the same class, with the IRLS loop of ``fit`` (KLR.py:57-75) run on
the MI355X by libkmgram (kmgram/learners.py)."""
from kmgram.learners import KLR

__all__ = ["KLR"]
