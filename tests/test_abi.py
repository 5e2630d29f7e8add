"""libcdr.so loads and exports every symbol include/cdr.h declares (CPU)."""
import os
import re

import pytest

from conftest import PKG, REPO


def _declared():
    with open(os.path.join(REPO, "include", "cdr.h")) as fh:
        text = fh.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(cdr_[a-z0-9_]+)\s*\(", text)))


def test_library_built():
    assert os.path.exists(os.path.join(PKG, "libcdr.so")), "run __graft_entry__.build()"


def test_every_declared_symbol_is_exported_and_bound():
    import _cdr

    lib = _cdr.load_library()
    names = _declared()
    assert len(names) >= 25
    for name in names:
        assert hasattr(lib, name), name
        assert name in _cdr.SIGNATURES, f"{name} has no ctypes signature"
    assert lib.cdr_version() == 1


def test_host_seq_sum_is_left_to_right():
    import numpy as np
    import _cdr

    v = np.array([1e16, 1.0, -1e16, 1.0])
    assert _cdr.host_seq_sum(v) == (((0.0 + 1e16) + 1.0) + -1e16) + 1.0


def test_no_cpu_fallback_without_gpu():
    import _cdr

    if _cdr.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises((RuntimeError, ValueError)):
        _cdr.Context(0)


def test_product_modules_do_not_import_oracle():
    for name in ("kmeans_plusplus.py", "scoring.py", "compute_features.py", "_cdr.py",
                 "cdr_dist.py"):
        path = os.path.join(PKG, name)
        if os.path.exists(path):
            with open(path) as fh:
                src = fh.read()
            assert not re.search(r"^\s*(from|import)\s+oracle", src, flags=re.M), name
