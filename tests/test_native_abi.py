"""CPU: the C-ABI library loads and exports every entry point include/vtf.h declares
(no compute calls: there is no GPU here)."""
import ctypes
import os
import re

from conftest import ROOT


def _header_symbols():
    src = open(os.path.join(ROOT, 'include', 'vtf.h')).read()
    return sorted(set(re.findall(r'^(?:int|const char\*)\s+(vtf_\w+)\(', src, re.M)))


def test_header_declares_entry_points():
    syms = _header_symbols()
    assert 'vtf_mtcnn_detect' in syms and 'vtf_batched_nms' in syms and len(syms) >= 20


def test_library_exports_every_header_symbol():
    from videotofaces import _native
    L = ctypes.CDLL(_native.LIB_PATH)
    missing = [s for s in _header_symbols() if not hasattr(L, s)]
    assert not missing, missing
    assert L.vtf_version() >= 1


def test_python_binding_covers_header():
    from videotofaces import _native
    assert set(_header_symbols()) <= set(_native.SIGNATURES)


def test_product_has_no_cpu_fallback():
    # the product package must never import the oracle
    pkg = os.path.join(ROOT, 'video-to-faces_amd', 'videotofaces')
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith('.py'):
                assert 'oracle' not in open(os.path.join(dp, f)).read().replace('# no oracle', ''), f
