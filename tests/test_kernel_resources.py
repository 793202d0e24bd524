"""Register / LDS budget of the built gfx950 code objects (host-only: the AMDGPU metadata of the
offload bundle in libedet.so, read with llvm-readelf through scripts/kernel_resources.py).

The tuned kernels' speed rests on their occupancy: the tiled depthwise backward lost 5-10 % when
its registers crossed a waves-per-SIMD step (`k_dwt`), and a packed-FMA rewrite that
went from 247 to 300 VGPRs at k5 was rejected on exactly that.  These checks turn such a
regression into a CPU test failure instead of a GPU measurement: no kernel spills VGPRs to scratch,
and the measured hot kernels keep the waves per SIMD they were tuned at.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tensorflow2-machine-vision_amd", "lib", "libedet.so")
sys.path.insert(0, os.path.join(ROOT, "scripts"))

kr = pytest.importorskip("kernel_resources")


@pytest.fixture(scope="module")
def table():
    if not os.path.exists(LIB):
        pytest.skip("libedet.so not built")
    if not os.path.exists(kr.READELF):
        pytest.skip("llvm-readelf not available")
    rows = []
    for co in kr.code_objects(LIB):
        rows += kr.kernels(co)
    for r, n in zip(rows, kr.demangle([r["name"] for r in rows])):
        r["pretty"] = n
    return rows


def test_code_objects_present(table):
    assert len(table) > 100
    assert any("k_dwt" in r["pretty"] for r in table)


def test_no_kernel_spills(table):
    # (SGPR spills go to VGPR lanes, not to memory: several GEMM instances have a few)
    bad = [r["pretty"] for r in table if r.get("private_segment_fixed_size", 0) or r.get("vgpr_spill_count", 0)]
    assert not bad, f"kernels spilling VGPRs to scratch memory: {bad[:5]}"


# (kernel name prefix, waves per SIMD the instance was measured at) -- bf16 storage instances
FLOORS = [
    ("void edet::k_dwt<unsigned short, 3, true, false>", 3),
    ("void edet::k_dwt<unsigned short, 3, false, false>", 3),
    ("void edet::k_dwt<unsigned short, 5, true, false>", 2),
    ("void edet::k_dwt<unsigned short, 5, false, false>", 2),
    # the lazy-dy forms (edet_dwconv_bwd_lazy) at the same occupancy
    ("void edet::k_dwt<unsigned short, 3, true, true>", 3),
    ("void edet::k_dwt<unsigned short, 5, true, true>", 2),
    ("void edet::k_fuse_bwd_m<", 3),
    ("void edet::k_fuse_fwd_m<", 3),
]


@pytest.mark.parametrize("prefix,floor", FLOORS)
def test_hot_kernel_occupancy(table, prefix, floor):
    rows = [r for r in table if r["pretty"].startswith(prefix)]
    assert rows, prefix
    for r in rows:
        w, _, _ = kr.waves_per_simd(r)
        assert w >= floor, f"{r['pretty']}: {w} waves/SIMD (VGPR {r.get('vgpr_count')}, AGPR {r.get('agpr_count')}) < {floor}"


@pytest.mark.parametrize("inst", ["false, 64, 2, 0", "true, 64, 2, 0", "true, 64, 2, 1"])
def test_wgrad_pipeline_waits_are_partial(inst):
    """The bf16 weight gradient's stage loop (round 4, DESIGN.md "Loads the compiler can count";
    the lazy instances since the round-5 gate fetch) waits for one stage's loads at a time: no
    s_waitcnt vmcnt(0) in the loop, which would drain the stage fetched ahead as well
    (scripts/wait_scan.py).  Plain A, lazy BN-only A and lazy BN + swish A."""
    if not os.path.exists(LIB) or not os.path.exists(kr.READELF):
        pytest.skip("libedet.so or llvm tools not available")
    ws = pytest.importorskip("wait_scan")
    if not os.path.exists(ws.OBJDUMP):
        pytest.skip("llvm-objdump not available")
    found = ws.scan(LIB, f"void edet::k_wgrad_tr<{inst}>")
    assert found, f"k_wgrad_tr<{inst}> not in the library"
    (_, loops), = found
    main = loops[0]
    assert main["loads"] >= 8 and main["vmcnt"], main
    assert 0 not in main["vmcnt"], f"vmcnt(0) in the stage loop: {main['vmcnt']}"
