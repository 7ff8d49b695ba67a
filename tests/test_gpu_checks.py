"""KMG_CHECK (include/kmgram.h KMG_EINTERNAL): the neighbourhood lists' metadata, which the
mismatch Gram kernel reads without a bound, is validated after every fill; an inconsistent
list stops the build with KMG_EINTERNAL before any Gram launch (the round-5 r05ah fault,
DESIGN §7).  The GPU suite runs with KMG_CHECK=1 (conftest.py).  Reference:
get_mismatch_K, kernels.py:196-217."""
import numpy as np
import pytest

import cref
from kmgram import _lib as L
from kmgram import encode as E
from kmgram import params as P

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fill", ["0", "1", "4"])
def test_check_stops_a_build_with_stale_list_counts(ctx, tune, fill):
    """KMG_CHECK=2 overwrites every list's piece counts after the fill (a fill that skipped
    its last phase): the call fails with KMG_EINTERNAL naming a list, nothing reads past the
    table, and the next build on the same context (KMG_CHECK=1) is exact."""
    codes, lens = E.synthetic(1500, 101, seed=71)
    p = P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=0)
    tune(KMG_CHECK="2", KMG_NB_FILL=fill, KMG_MM_FORM="4")
    with pytest.raises(L.KmgError) as ei:
        ctx.gram(p, codes, lens, L.KMG_I32)
    assert ei.value.status == L.KMG_EINTERNAL
    assert "KMG_CHECK: neighbourhood list" in str(ei.value)
    tune(KMG_CHECK="1", KMG_NB_FILL=fill, KMG_MM_FORM="4")
    K = ctx.gram(p, codes, lens, L.KMG_I32)
    assert ctx.last_plan()["formulation"] == "neighbourhood"
    assert np.array_equal(K[:40].astype(np.int64), cref.mismatch_raw(codes, lens, 9, 1, rows=(0, 40)))


def test_check_is_on_in_the_gpu_suite():
    import os
    assert os.environ.get("KMG_CHECK") == "1"
