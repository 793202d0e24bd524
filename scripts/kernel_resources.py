"""Per-kernel resource table of the built library's gfx950 code object: VGPRs, AGPRs, SGPRs,
LDS bytes, scratch bytes and the waves per SIMD the registers and LDS allow (CDNA4: 512 VGPRs
per SIMD lane in a unified VGPR/AGPR file allocated in granules of 8, 160 KB of LDS per CU,
at most 8 waves per SIMD).  Host-only: reads the offload bundle out of the .so, hands the ELF to
llvm-readelf --notes and parses the AMDGPU metadata.

    python scripts/kernel_resources.py [lib.so] [--filter k_dwt] [--out profiles/r04_kernel_resources.txt]
"""
import argparse
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
FILT = "c++filt"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(so):
    """gfx950 code objects of every offload bundle embedded in the shared library."""
    blob = open(so, "rb").read()
    out, pos = [], 0
    while True:
        pos = blob.find(MAGIC, pos)
        if pos < 0:
            return out
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "gfx950" in triple and size:
                out.append(blob[pos + off:pos + off + size])
        pos += 32


def kernels(elf):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(elf)
        f.flush()
        notes = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True).stdout
    rows, cur = [], None
    for line in notes.splitlines():
        s = line.strip()
        m = re.match(r"-?\s*\.(\w+):\s*(.*)$", s)
        if not m:
            continue
        key, val = m.group(1), m.group(2).strip()
        if s.startswith("- .") and key in ("agpr_count", "args"):
            cur = {}
            rows.append(cur)
        if cur is None:
            continue
        if key in ("agpr_count", "vgpr_count", "sgpr_count", "group_segment_fixed_size",
                   "private_segment_fixed_size", "max_flat_workgroup_size", "vgpr_spill_count",
                   "sgpr_spill_count"):
            cur[key] = int(val)
        elif key == "name":
            cur["name"] = val.strip("'\"")
    return [r for r in rows if "name" in r and not r["name"].endswith(".kd")]


def demangle(names):
    r = subprocess.run([FILT], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else names


def waves_per_simd(r):
    v = (r.get("vgpr_count", 0) + 7) // 8 * 8 + (r.get("agpr_count", 0) + 7) // 8 * 8
    by_v = 8 if v == 0 else min(8, 512 // v)
    wg = max(1, r.get("max_flat_workgroup_size", 256))
    wpg = (wg + 63) // 64  # waves of one workgroup, spread over the CU's 4 SIMDs
    lds = r.get("group_segment_fixed_size", 0)
    by_l = 8 if lds == 0 else min(8, (160 * 1024 // lds) * wpg // 4)
    return min(by_v, by_l), by_v, by_l


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(ROOT, "tensorflow2-machine-vision_amd/lib/libedet.so"))
    ap.add_argument("--filter", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = []
    for co in code_objects(a.lib):
        rows += kernels(co)
    names = demangle([r["name"] for r in rows])
    for r, n in zip(rows, names):
        r["pretty"] = n
    rows = [r for r in rows if a.filter in r["pretty"]]
    rows.sort(key=lambda r: r["pretty"])
    lines = [f"# {os.path.basename(a.lib)}: {len(rows)} kernels (gfx950); waves/SIMD = min(by registers, by LDS)",
             f"{'vgpr':>5} {'agpr':>5} {'sgpr':>5} {'lds':>7} {'scr':>5} {'waves':>5} {'(reg':>5} {'lds)':>5}  kernel"]
    for r in rows:
        w, bv, bl = waves_per_simd(r)
        lines.append(f"{r.get('vgpr_count', 0):5d} {r.get('agpr_count', 0):5d} {r.get('sgpr_count', 0):5d} "
                     f"{r.get('group_segment_fixed_size', 0):7d} {r.get('private_segment_fixed_size', 0):5d} "
                     f"{w:5d} {bv:5d} {bl:5d}  {r['pretty']}")
    text = "\n".join(lines) + "\n"
    if a.out:
        open(a.out, "w").write(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
