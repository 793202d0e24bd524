"""Memory-wait scan of the built library's gfx950 kernels: for every loop (a backward branch) of
each kernel, the vector-memory loads and stores it issues and the `s_waitcnt vmcnt(N)` it
executes.  `vmcnt` is an in-order counter: `vmcnt(0)` inside a software-pipelined loop means the
chunk fetched ahead is waited for together with the one needed (DESIGN.md, round 4 "Loads the
compiler can count").  Host-only: llvm-objdump over the offload bundle's code objects.

    python scripts/wait_scan.py [lib.so] [--filter k_wgrad_tr] [--all-loops]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kernel_resources as kr  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
_SYM = re.compile(r"^[0-9a-f]+ <(\S+)>:$")
_INS = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):")
_TGT = re.compile(r"<(\S+?)\+0x([0-9a-f]+)>")
_MEM = re.compile(r"^(global|buffer|flat)_(load|store|atomic)")


def disassemble(co):
    """{mangled kernel: [(address, opcode, operands, branch target address or None)]}"""
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        text = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", f.name], capture_output=True, text=True).stdout
    funcs, cur, base = {}, None, 0
    for line in text.splitlines():
        m = _SYM.match(line.strip())
        if m:
            cur = funcs.setdefault(m.group(1), [])
            base = int(line.split()[0], 16)
            continue
        m = _INS.match(line)
        if cur is None or not m:
            continue
        op, args, addr = m.group(1), m.group(2), int(m.group(3), 16)
        t = _TGT.search(line)
        tgt = base + int(t.group(2), 16) if (t and op.startswith("s_cbranch") or t and op == "s_branch") else None
        cur.append((addr, op, args, tgt))
    return funcs


def loops(ins):
    """Loops of one kernel as (start index, end index) from its backward branches, outermost
    first; each with its loads, stores and vmcnt waits."""
    idx = {a: i for i, (a, *_r) in enumerate(ins)}
    out = []
    for i, (a, op, args, tgt) in enumerate(ins):
        if tgt is not None and tgt <= a and tgt in idx:
            j = idx[tgt]
            body = ins[j:i + 1]
            waits = [int(w) for (_, o, ar, _) in body if o == "s_waitcnt" for w in re.findall(r"vmcnt\((\d+)\)", ar)]
            loads = sum(1 for (_, o, *_r) in body if _MEM.match(o) and "_load" in o)
            stores = sum(1 for (_, o, *_r) in body if _MEM.match(o) and ("_store" in o or "_atomic" in o))
            out.append({"start": j, "end": i, "n": i - j + 1, "loads": loads, "stores": stores, "vmcnt": waits})
    out.sort(key=lambda l: -l["n"])
    return out


def scan(lib, flt=""):
    """[(demangled name, loops)] of every kernel whose demangled name contains flt."""
    funcs = {}
    for co in kr.code_objects(lib):
        funcs.update(disassemble(co))
    names = list(funcs)
    pretty = kr.demangle(names)
    return [(p, loops(funcs[n])) for n, p in sorted(zip(names, pretty), key=lambda t: t[1]) if flt in p]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(kr.ROOT, "tensorflow2-machine-vision_amd/lib/libedet.so"))
    ap.add_argument("--filter", default="")
    ap.add_argument("--all-loops", action="store_true", help="every loop, not only the largest")
    a = ap.parse_args()
    for name, ls in scan(a.lib, a.filter):
        if not ls:
            continue
        print(name)
        for l in (ls if a.all_loops else ls[:1]):
            w = " ".join(str(x) for x in l["vmcnt"]) or "-"
            print(f"   loop {l['n']:5d} instr  loads {l['loads']:3d}  stores {l['stores']:3d}  vmcnt waits: {w}"
                  + ("   <-- vmcnt(0)" if 0 in l["vmcnt"] else ""))


if __name__ == "__main__":
    main()
