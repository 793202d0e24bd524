"""The C-ABI library loads and exports every symbol include/edet.h declares (no GPU calls)."""
import ctypes
import os
import re

from tf2mv_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "edet.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(edet_[a-z0-9_]+)\s*\(", src)))


def test_every_header_symbol_is_exported_and_bound():
    fns = header_functions()
    assert len(fns) >= 30
    dll = ctypes.CDLL(_lib.LIB_PATH)
    for f in fns:
        assert hasattr(dll, f), f"libedet.so does not export {f}"
    assert set(fns) == set(_lib.SIGNATURES), set(fns) ^ set(_lib.SIGNATURES)


def test_struct_layouts_match_header():
    # sizes follow from the C layout rules for the declared field order
    assert ctypes.sizeof(_lib.Pyramid) == 4 * (2 + 3 * 5)
    assert ctypes.sizeof(_lib.BN) == 8 * 20 + 8
    assert ctypes.sizeof(_lib.Lazy) == 8 + 8 + ctypes.sizeof(_lib.BN) + 8
    assert ctypes.sizeof(_lib.FuseInput) == ctypes.sizeof(_lib.Lazy) + 8 + 16 + 8  # + pool_arg
    assert ctypes.sizeof(_lib.Sched) == 40


def test_error_path_without_gpu():
    lib = _lib.lib()
    assert lib.fns["edet_abi_version"]() == _lib.ABI_VERSION == 10
    # argument validation happens before any HIP call
    rc = lib.fns["edet_conv1x1_fwd"](0, None, None, 8, None, 8, None, None, 8, 0, None, None)
    assert rc == -1 and "null" in lib.last_error()
    try:
        lib.call("edet_dwconv_fwd", 0, None, None, 8, 3, 1, None, None, None, None, None)
    except _lib.EdetError as e:
        assert "dwconv_fwd" in str(e)
    else:
        raise AssertionError("expected EdetError")


def test_conv1x1_fwd_rejects_accumulate_with_lazy_a():
    """the lazy K-loop instances overwrite C, so an accumulating forward with a BN /
    swish / gated A is refused before any launch (EDET_EINVAL) instead of silently overwriting;
    a plain A with accumulate passes the check (and fails later, at the null output)."""
    lib = _lib.lib()
    lz = _lib.Lazy()
    lz.x, lz.ld, lz.act = 16, 8, _lib.ACT_SWISH
    pyr = _lib.Pyramid()
    pyr.nseg, pyr.batch, pyr.H[0], pyr.W[0] = 1, 1, 4, 4
    dummy = ctypes.c_void_p(16)
    rc = lib.fns["edet_conv1x1_fwd"](0, ctypes.byref(lz), ctypes.byref(pyr), 8, dummy, 8, None, dummy, 8, 1,
                                     None, None)
    assert rc == -1 and "plain A" in lib.last_error()


def test_stat_layout_helpers():
    """include/edet.h "Statistics vectors" (ABI 9): channel c of replica r at
    (c / 16) * 64 + r * 16 + c % 16; the value is (r0 + r1) + (r2 + r3)."""
    import torch
    assert _lib.stat_len(1) == 64 and _lib.stat_len(16) == 64 and _lib.stat_len(17) == 128
    assert _lib.stat_idx(0, 0) == 0 and _lib.stat_idx(5, 2) == 37 and _lib.stat_idx(17, 3) == 64 + 48 + 1
    v = torch.arange(1, 21, dtype=torch.float64)
    t = _lib.stat_unfold(v)
    assert t.shape == (128,) and float(t.sum()) == float(v.sum())
    t[_lib.stat_idx(3, 1)] += 0.5
    t[_lib.stat_idx(3, 0)] -= 0.5
    assert torch.equal(_lib.stat_fold(t, 20), v)
    two = _lib.stat_unfold(torch.stack([v, 2 * v]))
    assert two.shape == (2, 128) and torch.equal(_lib.stat_fold(two, 20)[1], 2 * v)
