"""The reference's module-level feature maps get_phi_u / get_phi_km / gappy_k and the
substring auxiliary B_k (kernels.py:12-25, 161-175, 308-342, 420-433), CPU side:

* the oracle restatements (oracle/cpu_ref.py phi_u, phi_km, gappy1_phi, ss_b) are pinned
  bit-for-bit to every fixture the unmodified reference produced (tests/golden, round 4);
* the drop-in kernels.py raises exactly the reference's errors for the fixtures where the
  reference raises (short mismatch rows, every gappy (k, g) but (1, 0)) -- decided on the
  host before any device call, so these run without a GPU."""
import numpy as np
import pytest

import cpu_ref
import feature_cases as F
import kernels as km


def _oracle(golden, name):
    e = golden.entry(name)
    kw = e["kwargs"]
    x = golden.seqs(name)
    b = F.betas(e)
    if e["fn"] == "get_phi_u":
        return cpu_ref.phi_u(x[0], kw["k"], b)
    if e["fn"] == "get_phi_km":
        return cpu_ref.phi_km(F.fmt(x[0]), kw["k"], kw["m"], b)
    if e["fn"] == "gappy_k":
        return cpu_ref.gappy1_phi(F.fmt(x[0]), b)
    return np.array([cpu_ref.ss_b(x[0], x[1], kw["lbda"], kw["k"])], dtype=np.float64)


def test_fixture_count(golden):
    assert len(F.names(golden)) >= 80


@pytest.mark.parametrize("prefix", F.PREFIXES)
def test_oracle_matches_reference_fixtures(golden, prefix):
    done = 0
    for name in F.names(golden):
        if not name.startswith(prefix) or golden.entry(name)["error"]:
            continue
        if name.startswith("GAPK_") and golden.entry(name)["kwargs"]["k"] != 1:
            continue  # gap_set empty: all zeros, checked below
        ref = golden.K(name)
        got = _oracle(golden, name)
        assert got.dtype == np.float64 and got.shape == ref.shape, name
        assert np.array_equal(got, ref), name
        done += 1
    assert done > 0


def test_gappy_empty_gap_set(golden):
    """gappy_k with no window pair to compare returns zeros without raising."""
    assert not golden.entry("GAPK_xe_k3_g1")["error"]
    assert not golden.K("GAPK_xe_k3_g1").any()
    assert np.array_equal(km.gappy_k(F.fmt(""), 3, 1, F.betas(golden.entry("GAPK_xe_k3_g1"))),
                          golden.K("GAPK_xe_k3_g1"))


def test_reference_errors_on_host(golden):
    """Every fixture where the reference raises: the drop-in raises the same type and
    message, before touching the device."""
    n = 0
    for name in F.names(golden):
        e = golden.entry(name)
        if not e["error"]:
            continue
        with pytest.raises(ValueError) as ei:
            F.call(km, golden, name)
        assert e["error"] == "ValueError", name
        assert str(ei.value) == e["error_msg"], (name, str(ei.value), e["error_msg"])
        n += 1
    assert n >= 10


@pytest.mark.parametrize("k,g", [(3, 1), (3, 0), (2, 3), (3, 2), (3, 3), (1, 1), (1, 0), (5, 4)])
def test_gappy_gram_errors_follow_the_feature_map(k, g):
    """get_gappy_K raises what its first gappy_k call raises (kernels.py:449)."""
    from kmgram import engine
    x = "ACGTACGTAC" * 11
    try:
        engine.gappy_reference_errors(len(x), k, g)
        ok = True
    except ValueError:
        ok = False
    assert ok == (k == 1 and g == 0)


def test_rec_memoises_on_printed_arguments():
    calls = []

    @km.rec
    def f(a, b):
        calls.append((a, b))
        return a * 10 + b

    assert f(1, 2) == 12 and f(1, 2) == 12 and len(calls) == 1
    assert f("1", "2") == 12 and len(calls) == 1  # '[1]-[2]' either way
    assert f(2, 1) == 21 and len(calls) == 2
    # tuple arguments format as in kernels.py:315 ('[%s]' % arg): a 1-tuple prints bare, so
    # it shares the key of its element; a longer tuple raises TypeError
    assert f((1,), 2) == 12 and len(calls) == 2
    with pytest.raises(TypeError):
        f((1, 2), 3)


def test_b_k_base_cases_without_device():
    assert km.B_k(0.5, 0, "ACG", "T") == 1
    assert km.B_k(0.5, 4, "ACG", "TTTTT") == 0
