"""ISA lint of the gfx950 code objects: no vector-memory load's destination VGPR may be
read or written while the load can still be in flight.

Why: kq_rows / kq_gemv issue their activation loads from inline asm (gload16_asm,
gload4_asm in csrc/kq_rows_device.h) so the compiler's waitcnt pass does not drain the
weight ring on them. The compiler therefore does not know the destination registers are
pending: if it reads one (a copy) or reuses it (its value looked dead) before the
covering `s_waitcnt vmcnt`, the kernel computes with garbage or the load lands in a
register that now holds something else (round 2: an HSA memory aperture violation,
profiles/r02_attn_epilogue_rejected.md). The source pins registers with empty
`asm volatile("" : "+v"(...))` statements; this lint checks the result in the ISA.

Model (MI355X_MICROARCH.md, last section): every vector-memory instruction (loads,
stores, LDS-DMA, atomics) enters ONE in-order counter; `s_waitcnt vmcnt(N)` retires all
but the N youngest. Per kernel, a dataflow over the basic blocks carries the list of
outstanding operations (merged at joins as a union, so the check is conservative);
an instruction that names a VGPR of a pending load's destination, as a source or as
its result, is a hazard. Two loads to the same register (the L2-prefetch sink) are
not: returns are in order.

    python tools/vmem_lint.py ggml-neon-opt_amd/lib/libggml_mi355x.so   # exit 1 on hazards
"""
from __future__ import annotations

import os
import re
import shutil
import struct
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

VMEM_PREFIX = ("global_", "buffer_", "flat_", "scratch_")
REG_RE = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
LINE_RE = re.compile(r"^\s+([a-z_0-9]+)(.*?)\s*//\s*([0-9A-Fa-f]+):")
FUNC_RE = re.compile(r"^([0-9a-f]+) <([^>]+)>:")
TARGET_RE = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>")
VMCNT_RE = re.compile(r"vmcnt\((\d+)\)")


def code_objects(path, arch="gfx950"):
    """ELF code objects for `arch` of every clang offload bundle in a shared library."""
    data = open(path, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    objs, i = [], data.find(magic)
    while i >= 0:
        n = struct.unpack_from("<Q", data, i + 24)[0]
        off = i + 32
        for _ in range(n):
            eo, es, tl = struct.unpack_from("<QQQ", data, off)
            off += 24
            triple = data[off:off + tl].decode(errors="replace")
            off += tl
            if arch in triple and es:
                objs.append(data[i + eo:i + eo + es])
        i = data.find(magic, i + 1)
    return objs


def disassemble(obj: bytes, mcpu="gfx950"):
    """{kernel: [(addr, mnemonic, operand text, branch target addr or None)]}."""
    tool = OBJDUMP if os.path.exists(OBJDUMP) else shutil.which("llvm-objdump")
    with tempfile.NamedTemporaryFile(suffix=".o") as f:
        f.write(obj)
        f.flush()
        txt = subprocess.run([tool, "-d", f"--mcpu={mcpu}", f.name], capture_output=True, text=True,
                             check=True).stdout
    funcs, cur, base = {}, None, 0
    for line in txt.splitlines():
        m = FUNC_RE.match(line)
        if m:
            base = int(m.group(1), 16)
            cur = funcs.setdefault(m.group(2), [])
            continue
        m = LINE_RE.match(line)
        if not m or cur is None:
            continue
        mn, ops, addr = m.group(1), m.group(2).strip(), int(m.group(3), 16)
        tgt = None
        t = TARGET_RE.search(line)
        if t and (mn.startswith("s_cbranch") or mn == "s_branch"):
            tgt = base + int(t.group(2), 16)
        cur.append((addr, mn, ops, tgt))
    return funcs


def vregs(text):
    out = set()
    for m in REG_RE.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def split_ops(ops):
    """Operands of an instruction (commas outside brackets); modifiers stay on the last."""
    parts, depth, cur = [], 0, ""
    for ch in ops:
        if ch in "[(":
            depth += 1
        elif ch in "])":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur.strip())
    return parts


def classify(mn, ops):
    """(is_vmem, vmem load dest VGPRs, VGPRs read, VGPRs written)."""
    parts = split_ops(ops)
    is_vmem = mn.startswith(VMEM_PREFIX)
    if is_vmem:
        returns = ("_load" in mn and "_lds" not in mn and "load_lds" not in mn) or \
                  ("_atomic" in mn and " glc" in " " + ops)
        if returns and parts:
            return True, vregs(parts[0]), set().union(*[vregs(p) for p in parts[1:]]) if len(parts) > 1 else set(), set()
        return True, set(), vregs(ops), set()
    if mn.startswith("s_"):
        return False, set(), set(), set()
    stores = mn.startswith("ds_write") or mn.startswith("ds_store") or mn in ("ds_swizzle_b32",) and False
    if stores or not parts:
        return False, set(), vregs(ops), set()
    dst = vregs(parts[0])
    src = set().union(*[vregs(p) for p in parts[1:]]) if len(parts) > 1 else set()
    if mn.startswith("v_writelane") or mn.startswith("v_mfma") or "_mac_" in mn or mn.startswith("v_fmac") \
            or mn.startswith("v_dot2c") or mn.startswith("v_pk_fmac"):
        src |= dst  # read-modify-write
    return False, set(), src, dst


def blocks_of(insts):
    """Basic blocks: leaders at the entry, at branch targets and after branches."""
    addrs = [a for a, *_ in insts]
    leaders = {addrs[0]} if addrs else set()
    for k, (a, mn, ops, tgt) in enumerate(insts):
        if tgt is not None:
            leaders.add(tgt)
        if (mn.startswith("s_cbranch") or mn in ("s_branch", "s_endpgm", "s_setpc_b64")) and k + 1 < len(insts):
            leaders.add(insts[k + 1][0])
    blocks, cur = [], []
    for ins in insts:
        if ins[0] in leaders and cur:
            blocks.append(cur)
            cur = []
        cur.append(ins)
    if cur:
        blocks.append(cur)
    return blocks


def merge(a, b):
    seen = {e[0] for e in a}
    return tuple(list(a) + [e for e in b if e[0] not in seen])


def lint_kernel(name, insts, max_iter=64):
    """Hazards of one kernel: [(addr, instruction, load addr, VGPRs)]."""
    if not insts:
        return []
    blocks = blocks_of(insts)
    index = {blk[0][0]: k for k, blk in enumerate(blocks)}
    succ = []
    for k, blk in enumerate(blocks):
        a, mn, ops, tgt = blk[-1]
        s = []
        if tgt is not None and tgt in index:
            s.append(index[tgt])
        if mn not in ("s_branch", "s_endpgm", "s_setpc_b64") and k + 1 < len(blocks):
            s.append(k + 1)
        succ.append(s)
    state_in = {0: ()}
    hazards = {}
    for _ in range(max_iter):
        changed = False
        for k, blk in enumerate(blocks):
            if k not in state_in:
                continue
            st = list(state_in[k])
            for a, mn, ops, tgt in blk:
                if mn == "s_waitcnt":
                    m = VMCNT_RE.search(ops)
                    if m:
                        n = int(m.group(1))
                        while len(st) > n:
                            st.pop(0)
                    continue
                is_vmem, dest, rd, wr = classify(mn, ops)
                pend = set()
                for e in st:
                    pend |= e[1]
                bad = (rd | wr) & pend
                if bad:
                    for e in st:
                        if e[1] & bad:
                            hazards[(a, e[0])] = (a, f"{mn} {ops}", e[0], sorted(e[1] & bad))
                if is_vmem:
                    st = [e for e in st if e[0] != a]  # the same instruction again (a loop): once
                    st.append((a, frozenset(dest)))
            out = tuple(st)
            for s in succ[k]:
                new = out if s not in state_in else merge(state_in[s], out)
                if state_in.get(s) != new:
                    state_in[s] = new
                    changed = True
        if not changed:
            break
    return sorted(hazards.values())


def lint_library(path, kernel_filter=None):
    """{kernel: hazards} over every gfx950 kernel of a shared library."""
    out = {}
    for obj in code_objects(path):
        for name, insts in disassemble(obj).items():
            if kernel_filter and not re.search(kernel_filter, name):
                continue
            h = lint_kernel(name, insts)
            out[name] = h
    return out


def main(argv):
    path = argv[1] if len(argv) > 1 else os.path.join(os.path.dirname(__file__), "..",
                                                      "ggml-neon-opt_amd/lib/libggml_mi355x.so")
    res = lint_library(path, argv[2] if len(argv) > 2 else None)
    bad = {k: v for k, v in res.items() if v}
    print(f"{len(res)} kernels, {len(bad)} with hazards")
    for k, hs in bad.items():
        print(k)
        for a, ins, la, regs in hs[:8]:
            print(f"   {a:#x}: {ins}   <- pending load at {la:#x}, v{regs}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
