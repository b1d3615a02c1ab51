"""Checks a built gfx950 code object for scalar loads whose destination SGPRs
are touched before the load has landed.

The scalar memory pipe returns loads out of order, so a scalar load's result
is defined only after an `s_waitcnt lgkmcnt(0)`. The compiler places those
waits for the loads it emits itself; a load issued from inline asm is invisible
to it, and the register allocator may copy or reuse its destination in between
(round 4 hit exactly that: nondeterministic wide-path results). For every
s_load / s_buffer_load in every kernel this walks the control-flow graph from
the load (fall-through and branch targets) until each path meets
lgkmcnt(0), and reports any instruction on the way that reads or writes one
of the load's destination SGPRs.

    python tools/smem_check.py timetabling-ga-mpi-openmp_amd/libttga.so
"""
from __future__ import annotations

import pathlib
import re
import struct
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

_SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")
_LINE = re.compile(r"^\s+(\S+)(.*?)\s*//\s*([0-9A-Fa-f]+):")
_FUNC = re.compile(r"^[0-9a-f]+ <(.+)>:$")


def code_objects(lib: str, arch: str = "gfx950") -> list[bytes]:
    """Every `arch` code object in the library's .hip_fatbin section (one
    offload bundle per translation unit, back to back)."""
    with tempfile.TemporaryDirectory() as d:
        fb = pathlib.Path(d) / "fatbin"
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, str(fb)], check=True)
        b = fb.read_bytes()
    out, i = [], 0
    while (i := b.find(MAGIC, i)) >= 0:
        (n,) = struct.unpack_from("<Q", b, i + 24)
        o = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", b, o)
            triple = b[o + 24:o + 24 + tl].decode()
            o += 24 + tl
            if triple.endswith(arch):
                out.append(b[i + off:i + off + size])
        i += len(MAGIC)
    return out


def sregs(text: str) -> set[int]:
    regs: set[int] = set()
    for a, b, c in _SREG.findall(text):
        if c:
            regs.add(int(c))
        else:
            regs.update(range(int(a), int(b) + 1))
    return regs


def functions(disasm: str):
    """{name: [(addr, mnemonic, operands)]} in address order."""
    funcs: dict[str, list] = {}
    cur = None
    for ln in disasm.splitlines():
        m = _FUNC.match(ln)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        m = _LINE.match(ln)
        if m and cur is not None:
            cur.append((int(m.group(3), 16), m.group(1), m.group(2).strip()))
    return funcs


def _successors(ins, k, index):
    addr, op, opnds = ins[k]
    if op in ("s_endpgm", "s_setpc_b64", "s_trap") or op.startswith("s_endpgm"):
        return []
    succ = []
    if op.startswith("s_branch") or op.startswith("s_cbranch"):
        imm = int(opnds.split()[0], 0) & 0xFFFF
        imm = imm - 0x10000 if imm & 0x8000 else imm
        tgt = index.get(addr + 4 + 4 * imm)
        if tgt is not None:
            succ.append(tgt)
        if op.startswith("s_branch"):
            return succ
    if k + 1 < len(ins):
        succ.append(k + 1)
    return succ


def check_function(ins) -> list[str]:
    index = {a: k for k, (a, _, _) in enumerate(ins)}
    bad = []
    for k, (addr, op, opnds) in enumerate(ins):
        if not (op.startswith("s_load") or op.startswith("s_buffer_load")):
            continue
        dst = sregs(opnds.split(",")[0])
        seen, stack = set(), _successors(ins, k, index)
        while stack:
            j = stack.pop()
            if j in seen:
                continue
            seen.add(j)
            a2, op2, o2 = ins[j]
            if op2.startswith("s_waitcnt"):
                m = re.search(r"lgkmcnt\((\d+)\)", o2)
                if m and int(m.group(1)) == 0:
                    continue
            if (op2.startswith("s_load") or op2.startswith("s_buffer_load")) and not (sregs(o2.split(",")[0]) & dst):
                # another load in flight; its base operand must not be a pending destination
                if sregs(o2.split(",", 1)[1] if "," in o2 else "") & dst:
                    bad.append(f"{addr:#x} {op} {opnds}  ->  {a2:#x} {op2} {o2}")
                    continue
            elif sregs(o2) & dst:
                bad.append(f"{addr:#x} {op} {opnds}  ->  {a2:#x} {op2} {o2}")
                continue
            stack.extend(_successors(ins, j, index))
    return bad


def check_library(lib: str, arch: str = "gfx950"):
    """(scalar loads checked, violations)."""
    loads, bad = 0, []
    with tempfile.TemporaryDirectory() as d:
        for n, co in enumerate(code_objects(lib, arch)):
            f = pathlib.Path(d) / f"co{n}.elf"
            f.write_bytes(co)
            dis = subprocess.run([OBJDUMP, "-d", f"--mcpu={arch}", str(f)], check=True, capture_output=True,
                                 text=True).stdout
            for name, ins in functions(dis).items():
                loads += sum(op.startswith(("s_load", "s_buffer_load")) for _, op, _ in ins)
                bad += [f"{name}: {b}" for b in check_function(ins)]
    return loads, bad


if __name__ == "__main__":
    n, bad = check_library(sys.argv[1] if len(sys.argv) > 1 else "timetabling-ga-mpi-openmp_amd/libttga.so")
    print(f"{n} scalar loads checked, {len(bad)} touched before lgkmcnt(0)")
    for b in bad[:50]:
        print(" ", b)
    sys.exit(1 if bad else 0)
