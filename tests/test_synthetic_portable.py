"""higgs_like_portable is bit-identical on every host (precision-pin data,
profiles/r4/precision_pin_r4.md): NumPy PCG64 + IEEE-exact operations only."""
import hashlib


def test_portable_higgs_hash_is_pinned():
    from h2omx.frame.synthetic import higgs_like_portable

    X, y = higgs_like_portable(100_000, 1)
    assert X.shape == (28, 100_000) and y.shape == (100_000,)
    assert hashlib.sha1(X.numpy().tobytes()).hexdigest()[:16] == "150904d174e984d5"
    assert hashlib.sha1(y.numpy().tobytes()).hexdigest()[:16] == "1825a6f8c1713d4e"
    assert 0.3 < float(y.mean()) < 0.6
