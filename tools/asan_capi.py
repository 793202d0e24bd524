"""Host-side AddressSanitizer run of the C-ABI's argument validation (VERDICT r02
item 9), CPU only: no kernel is launched.

    make -C tensorflow2-machine-vision_amd asan
    ASAN_OPTIONS=detect_leaks=0 LD_PRELOAD=$(hipcc -print-file-name=libclang_rt.asan-x86_64.so) \\
        EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_asan.so python tools/asan_capi.py

1. every entry point of include/edet.h (the _lib SIGNATURES table) called with null pointers
   and zero sizes must return a non-zero status (or EDET_OK where the call is a documented
   no-op) with a message, never touch memory it was not given;
2. targeted invalid descriptors (bad channel alignment, mismatched pyramids, unsupported
   kernel sizes, the fused backward's fold preconditions, too many segments) must be
   rejected by the validation layer before any device work;
3. edet_launched_kernels into a 1-byte buffer must stay inside it.
ASan aborts the process on any out-of-bounds or use-after-free in the library's host code.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tf2mv_amd import _lib as L  # noqa: E402

NOOP_OK = {"edet_abi_version", "edet_memset_async", "edet_memcpy_async", "edet_set_workspace",
           "edet_launched_kernels", "edet_cast_f32", "edet_count_positives", "edet_onehot_to_index",
           "edet_opt_norm", "edet_opt_apply", "edet_bn_inference_stats", "edet_bn_update_moving",
           "edet_dropmask", "edet_transpose_cast", "edet_anchor_boxes", "edet_se_bn_combine"}


def zero_args(argtypes):
    out = []
    for t in argtypes:
        if t in (ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t, ctypes.c_uint64):
            out.append(0)
        elif t is ctypes.c_float:
            out.append(0.0)
        else:
            out.append(None)  # every pointer / descriptor null
    return out


def main():
    lib = L.lib()
    f = lib.fns
    assert f["edet_abi_version"]() == L.ABI_VERSION
    rejected, noop = [], []
    for name, argtypes in L.SIGNATURES.items():
        if name in ("edet_last_error", "edet_abi_version", "edet_launched_kernels", "edet_dev_set",
                    "edet_wall_clock_khz", "edet_probe"):
            continue
        rc = f[name](*zero_args(argtypes))
        if rc != 0:
            rejected.append(name)
            assert lib.last_error(), name
        else:
            assert name in NOOP_OK, f"{name} accepted null arguments"
            noop.append(name)
    print(f"null/zero arguments: {len(rejected)} entry points rejected, {len(noop)} documented no-ops")

    # targeted descriptors
    pyr = L.Pyramid()
    pyr.nseg, pyr.batch = 1, 2
    pyr.H[0], pyr.W[0] = 8, 8
    lz = L.Lazy()
    buf = (ctypes.c_uint16 * (2 * 8 * 8 * 64))()
    lz.x = ctypes.cast(buf, ctypes.c_void_p)
    lz.ld = 60  # not a multiple of 8
    out = (ctypes.c_uint16 * (2 * 8 * 8 * 64))()
    w = (ctypes.c_uint16 * (25 * 64))()
    dw = (ctypes.c_float * (25 * 64))()
    P = ctypes.c_void_p
    cases = {
        "conv1x1_fwd lda%8": lambda: f["edet_conv1x1_fwd"](1, ctypes.byref(lz), ctypes.byref(pyr), 64, P(ctypes.addressof(w)),
                                                          64, None, P(ctypes.addressof(out)), 64, 0, None, None),
        "dwconv_fwd C%8": lambda: f["edet_dwconv_fwd"](1, ctypes.byref(lz), ctypes.byref(pyr), 60, 3, 1, P(ctypes.addressof(w)),
                                                      P(ctypes.addressof(out)), ctypes.byref(pyr), None, None),
    }
    for name, fn in cases.items():  # while lz.ld = 60
        rc = fn()
        assert rc == -1, f"{name}: rc {rc}"
        print(f"  {name:30s} rc={rc:3d}  {lib.last_error()}")
    cases = {}
    lz.ld = 64
    pout = L.Pyramid()
    pout.nseg, pout.batch = 1, 2
    pout.H[0], pout.W[0] = 8, 8  # stride 2 needs 4 x 4
    cases.update({
        "dwconv_fwd pyramid mismatch": lambda: f["edet_dwconv_fwd"](1, ctypes.byref(lz), ctypes.byref(pyr), 64, 3, 2,
                                                                   P(ctypes.addressof(w)), P(ctypes.addressof(out)),
                                                                   ctypes.byref(pout), None, None),
        "dwconv_fwd k=7": lambda: f["edet_dwconv_fwd"](1, ctypes.byref(lz), ctypes.byref(pyr), 64, 7, 1, P(ctypes.addressof(w)),
                                                      P(ctypes.addressof(out)), ctypes.byref(pyr), None, None),
        "dwconv_bwd stride 2": lambda: f["edet_dwconv_bwd"](1, ctypes.byref(lz), ctypes.byref(pyr), 64, 3, 2,
                                                           P(ctypes.addressof(out)), ctypes.byref(pout), P(ctypes.addressof(w)),
                                                           P(ctypes.addressof(out)), 0, P(ctypes.addressof(dw)), None, None),
        "dwconv_bwd fold+accumulate": lambda: f["edet_dwconv_bwd"](1, ctypes.byref(lz), ctypes.byref(pyr), 64, 3, 1,
                                                                  P(ctypes.addressof(out)), ctypes.byref(pyr), P(ctypes.addressof(w)),
                                                                  P(ctypes.addressof(out)), 1, P(ctypes.addressof(dw)),
                                                                  ctypes.byref(L.BnGrad64()), None),
        "dtype 7": lambda: f["edet_lazy_materialize"](7, ctypes.byref(lz), ctypes.byref(pyr), 64, P(ctypes.addressof(out)), None),
    })
    bad = L.Pyramid()
    bad.nseg, bad.batch = 9, 2  # more segments than EDET_MAX_SEG
    cases["conv1x1_fwd nseg 9"] = lambda: f["edet_conv1x1_fwd"](1, ctypes.byref(lz), ctypes.byref(bad), 64,
                                                               P(ctypes.addressof(w)), 64, None, P(ctypes.addressof(out)),
                                                               64, 0, None, None)
    for name, fn in cases.items():
        rc = fn()
        assert rc != 0, f"{name}: accepted"
        print(f"  {name:30s} rc={rc:3d}  {lib.last_error()}")

    # string outputs stay inside their buffers
    one = ctypes.create_string_buffer(1)
    f["edet_launched_kernels"](one, 1)
    assert one.raw == b"\x00"
    assert f["edet_launched_kernels"](None, 0) != 0
    assert f["edet_dev_set"](3, 1) != 0  # production library: no development slots
    print("asan_capi: OK")


if __name__ == "__main__":
    main()
